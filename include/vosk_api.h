/* vosk_api.h -- C ABI of the MI355X-native Vosk hot path (libvosk.so).
 *
 * Drop-in boundary: every declaration below has exactly the name, argument
 * types, return type and calling convention of the reference's public header
 * (/root/reference/src/vosk_api.h); the line cited next to each entry is the
 * reference declaration it replaces.  Opaque handles, NULL / -1 error
 * conventions and ownership are unchanged, so the reference's
 * language bindings (Python cffi, JNA, P/Invoke, cgo, ffi-napi) bind this
 * library without modification.  The header stays plain C that `cpp` +
 * pycparser can parse (python/vosk_builder.py:7-11 generates its cdef from it).
 *
 * Behavioural notes for this implementation are in INTEGRATION.md.
 */
#ifndef VOSK_API_H
#define VOSK_API_H

#ifdef __cplusplus
extern "C" {
#endif

/* Opaque handles (reference vosk_api.h:20-51). */
typedef struct VoskModel VoskModel;
typedef struct VoskSpkModel VoskSpkModel;
typedef struct VoskRecognizer VoskRecognizer;
typedef struct VoskBatchModel VoskBatchModel;
typedef struct VoskBatchRecognizer VoskBatchRecognizer;

/* Loads a model directory (V2: am/ conf/ graph/, or V1 flat layout).
 * Returns NULL on failure.  Replaces vosk_api.h:58. */
VoskModel *vosk_model_new(const char *model_path);

/* Releases the caller's reference; the model lives while recognizers use it.
 * Replaces vosk_api.h:66. */
void vosk_model_free(VoskModel *model);

/* Word id in the model's symbol table, -1 if absent.  Replaces vosk_api.h:74. */
int vosk_model_find_word(VoskModel *model, const char *word);

/* Speaker model (x-vector path: not implemented in this build, returns NULL).
 * Replaces vosk_api.h:81 and :89. */
VoskSpkModel *vosk_spk_model_new(const char *model_path);
void vosk_spk_model_free(VoskSpkModel *model);

/* Streaming recognizer.  Replaces vosk_api.h:100 / :115 / :137. */
VoskRecognizer *vosk_recognizer_new(VoskModel *model, float sample_rate);
VoskRecognizer *vosk_recognizer_new_spk(VoskModel *model, float sample_rate, VoskSpkModel *spk_model);
VoskRecognizer *vosk_recognizer_new_grm(VoskModel *model, float sample_rate, const char *grammar);

/* Result options.  Replace vosk_api.h:146, :166, :175, :191, :209. */
void vosk_recognizer_set_spk_model(VoskRecognizer *recognizer, VoskSpkModel *spk_model);
void vosk_recognizer_set_max_alternatives(VoskRecognizer *recognizer, int max_alternatives);
void vosk_recognizer_set_words(VoskRecognizer *recognizer, int words);
void vosk_recognizer_set_partial_words(VoskRecognizer *recognizer, int partial_words);
void vosk_recognizer_set_nlsml(VoskRecognizer *recognizer, int nlsml);

/* Audio input: returns 1 when an endpoint was detected (call
 * vosk_recognizer_result), 0 otherwise, -1 on error.  `length` is bytes of
 * s16le for the char* form and samples for the short / float forms (float
 * samples in the int16 range).  Replace vosk_api.h:221, :226, :231. */
int vosk_recognizer_accept_waveform(VoskRecognizer *recognizer, const char *data, int length);
int vosk_recognizer_accept_waveform_s(VoskRecognizer *recognizer, const short *data, int length);
int vosk_recognizer_accept_waveform_f(VoskRecognizer *recognizer, const float *data, int length);

/* JSON results; the returned string is owned by the recognizer and valid
 * until the next result call.  Replace vosk_api.h:250, :264, :273. */
const char *vosk_recognizer_result(VoskRecognizer *recognizer);
const char *vosk_recognizer_partial_result(VoskRecognizer *recognizer);
const char *vosk_recognizer_final_result(VoskRecognizer *recognizer);

/* Replace vosk_api.h:279, :285. */
void vosk_recognizer_reset(VoskRecognizer *recognizer);
void vosk_recognizer_free(VoskRecognizer *recognizer);

/* Replace vosk_api.h:294, :301, :308. */
void vosk_set_log_level(int log_level);
void vosk_gpu_init();
void vosk_gpu_thread_init();

/* Batch (GPU) API: reads ./model like the reference.  Replace
 * vosk_api.h:313-346. */
VoskBatchModel *vosk_batch_model_new();
void vosk_batch_model_free(VoskBatchModel *model);
void vosk_batch_model_wait(VoskBatchModel *model);
VoskBatchRecognizer *vosk_batch_recognizer_new(VoskBatchModel *model, float sample_rate);
void vosk_batch_recognizer_free(VoskBatchRecognizer *recognizer);
void vosk_batch_recognizer_accept_waveform(VoskBatchRecognizer *recognizer, const char *data, int length);
void vosk_batch_recognizer_set_nlsml(VoskBatchRecognizer *recognizer, int nlsml);
void vosk_batch_recognizer_finish_stream(VoskBatchRecognizer *recognizer);
const char *vosk_batch_recognizer_front_result(VoskBatchRecognizer *recognizer);
void vosk_batch_recognizer_pop(VoskBatchRecognizer *recognizer);
int vosk_batch_recognizer_get_pending_chunks(VoskBatchRecognizer *recognizer);

#ifdef __cplusplus
}
#endif

#endif /* VOSK_API_H */
