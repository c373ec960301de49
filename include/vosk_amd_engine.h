/* vosk_amd_engine.h -- diagnostic C ABI of libvosk.so's GPU engine.
 *
 * Not part of the reference interface.  These entry points expose the
 * engine's stages (MFCC, looped nnet3, token passing, traceback) with plain
 * pointers so that kernel-level parity tests and the benchmark can drive the
 * same code path the vosk_* API uses (Model -> Engine, src/recognizer.cc:
 * 297-323 equivalent) and compare it with the CPU oracle.  All functions
 * return < 0 (or NULL) on error; vamd_last_error() returns the message.
 */
#ifndef VOSK_AMD_ENGINE_H
#define VOSK_AMD_ENGINE_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct VamdEngine VamdEngine;

/* host-only (no GPU needed): nnet plan of a model directory */
const char *vamd_plan_describe(const char *model_dir, int frames_per_chunk);
/* [fpc, fss, left_ctx, right_ctx, priming, out_dim, ops, stored nodes] */
int vamd_plan_info(const char *model_dir, int frames_per_chunk, int *out8, double *flops_per_chunk);

/* JSON bytes of a word list exactly as the recognizer writes results
 * (json.h dump format): {list_key: [{conf,end,start,word}...], text_key: ...} */
const char *vamd_json_words(const char *list_key, const char *text_key, int n,
                            const char *const *words, const double *start, const double *end,
                            const double *conf);

/* host-only: the recognizer's silence weighting (silence.h) over a sequence
 * of calls; call c passes the best-path traceback (per decoded frame: tid and
 * source token) in [trace_off[c], trace_off[c+1]) and receives its (feature
 * frame, delta weight) list in [out_off[c], out_off[c+1]).  Returns the total. */
int vamd_silence_weighting_run(int ncalls, const int *num_frames_ready, const int *first_decoder_frame,
                               const int *trace_off, const int *tids, const int *toks,
                               const unsigned char *tid_is_silence, int num_tids, float silence_weight,
                               int fss, int *out_off, int *out_frame, float *out_w, int cap);

/* host-only: the decode graph of a model directory as the engine uploads it
 * (graph/HCLG.fst as stored, or graph/HCLr.fst o graph/Gr.fst expanded by
 * graph_compose.h), or with grammar != NULL the grammar recognizer's runtime
 * graph (HCLr o the phrase-list bigram).  NULL on error.  vamd_graph_dims
 * returns the state count (start state and arc count through the pointers);
 * vamd_graph_copy fills final costs [S], arc offsets [S+1] (emitting arcs
 * first per state) and the arcs [A]. */
void *vamd_graph_new(const char *model_dir, const char *grammar);
int vamd_graph_dims(void *graph, int *start, long long *num_arcs);
int vamd_graph_copy(void *graph, float *final_cost, long long *arc_begin, int *ilabel, int *olabel,
                    float *weight, int *nextstate);
/* OpenFST's lazy ComposeFst numbering of a composed (lookahead) graph: per
 * state its arc destinations in the composition's own arc order, as ids
 * [0, ids) (the graph's states, then states the trim dropped).  Returns ids
 * (0: not a composed graph); fills row [S+1] and next [row[S]] when non-NULL. */
int vamd_graph_lazy(void *graph, long long *row, int *next);
void vamd_graph_free(void *graph);

/* speaker x-vector of a sample sequence (the GPU path GetSpkVector uses,
 * xvector.h): samples at the speaker MFCC rate since the speaker front end
 * started (at `rate`, resampled to the speaker model's rate on the GPU), the
 * segment's frames from first_frame, frame i used iff
 * keep[(i - first_frame) / 3].  Returns the vector length (0: fewer than 50
 * frames selected; -1: error); *num_frames = the selected frame count. */
int vamd_spk_extract(VoskSpkModel *spk, const float *samples, long long n, int rate, int first_frame,
                     const signed char *keep, int nkeep, float *out, int cap, int *num_frames);
/* count such requests extracted as one batch (one launch sequence per up to
 * 256 utterances; each vector equals vamd_spk_extract's bit for bit): vector
 * i goes to out + i * cap, status[i] = its length (0: fewer than 50 frames).
 * Returns count (-1: error).  Concurrent vamd_spk_extract / recognizer
 * callers are batched the same way (group commit); vamd_spk_stats reports the
 * launch sequences run, the utterances they extracted, and the frame-level
 * layers' GEMM flops and HIP-event milliseconds (either pointer may be NULL). */
int vamd_spk_extract_batch(VoskSpkModel *spk, int count, const float *const *samples, const long long *n,
                           const int *rate, const int *first_frame, const signed char *const *keep,
                           const int *nkeep, float *out, int cap, int *num_frames, int *status);
int vamd_spk_stats(VoskSpkModel *spk, long long *batches, long long *utterances, double *layer_flops,
                   double *layer_ms);

/* host-only: LM rescoring (rescore.h) applied by vamd_lattice_words_json
 * after determinization (both paths NULL: off); vamd_carpa_logprob is a
 * ConstArpa n-gram lookup (natural log, history oldest word first). */
int vamd_lattice_set_rescore(const char *g_fst, const char *g_carpa);
float vamd_carpa_logprob(const char *g_carpa, int word, const int *hist, int nhist);

/* host-only: with ntids > 0, vamd_lattice_words_json determinizes as the
 * reference's GetLattice (DeterminizeLatticePhonePrunedWrapper: a phone +
 * word pass, then words; per transition-id its phone and whether it is a
 * phone's first transition-id); ntids == 0: word level only (the default). */
int vamd_lattice_set_phones(const int *tid2phone, const signed char *tid_first, int ntids);

/* host-only: the pruned determinization's memory limit in bytes
 * (DeterminizeLatticePhonePrunedOptions::max_mem, default 50000000; a smaller
 * one exercises the narrower-beam retry). */
int vamd_lattice_set_det_max_mem(long long bytes);

/* host-only: the result pipeline over a state-level lattice (the arrays of
 * vamd_stream_lattice; arc_ilabel / arc_olabel index the graph's arcs):
 * lattice-beam pruning, word determinization, graph scaling, word alignment
 * (when ntids > 0: per transition-id phone boundary type, IsFinal, IsSelfLoop),
 * MBR and n-best.
 * Returns JSON {pruned_tokens, pruned_links, det_ok, det_states, det_arcs,
 * mbr: {words, conf, times}, nbest: [{words, spans, graph, acoustic}]}. */
const char *vamd_lattice_words_json(int num_frames, const int *frame_begin, const int *tok_state,
                                    const float *tok_cost, const int *link_src, const int *link_dst,
                                    const int *link_arc, const float *link_graph, const float *link_ac,
                                    int nlink, const float *final_cost, int nfinal, const int *arc_ilabel,
                                    const int *arc_olabel, int narcs, float lattice_beam, float graph_scale,
                                    int nbest, const signed char *tid_type, const signed char *tid_final,
                                    const signed char *tid_loop, int ntids);

/* host-only: the KaldiRecognizer's incremental lattice (incremental.h:
 * LatticeIncrementalDecoder's PruneActiveTokens schedule and
 * LatticeIncrementalDeterminizer) over per-frame decoder records: tokens of
 * frame k = [frame_begin[k], frame_begin[k+1]) in list order, links of frame k
 * (emitting links into it, epsilon links inside it) with frame-local source /
 * destination indices and the raw acoustic cost; the phone tables of
 * vamd_lattice_set_phones.  Events: type 0 = decode up to ev_arg frames then
 * UpdateLatticeDeterminization, 1 = GetLattice(NumFramesInLattice(), false),
 * 2 = FinalizeDecoding + GetLattice(NumFramesDecoded(), true).  Returns a JSON
 * list, per query {nfl, ok, chunks, arcs: per state [[word, next, graph,
 * acoustic, [tids]]], finals: per state [graph, acoustic, [tids]] | null}. */
const char *vamd_incremental_json(int nframes, const int *frame_begin, const int *tok_state,
                                  const float *tok_cost, const float *cost_offset, int nlink,
                                  const int *link_frame, const int *link_src, const int *link_dst,
                                  const int *link_arc, const float *link_ac, int narcs,
                                  const int *arc_ilabel, const int *arc_olabel,
                                  const float *arc_weight, int nstates, const float *final_cost,
                                  int start_state, float lattice_beam, int prune_interval,
                                  float prune_scale, int max_delay, int min_chunk, int nev,
                                  const int *ev_type, const int *ev_arg);

const char *vamd_last_error(void);
int vamd_device_count(void);

/* frames_per_chunk <= 0 uses the model's decodable option (default 20->21);
 * flags: 1 = collect per-frame decoder stats, 2 = keep decoded LLH rows,
 *        4 = HIP-event timing of each stage on the engine's stream,
 *        8 = two-stream pipeline (decoder of step i-1 beside the nnet of step
 *            i; decoder results lag one step, vamd_engine_flush drains),
 *       16 = lattice generation (vamd_stream_lattice),
 *       32 = order-independent token passing (the BatchModel lanes' form)
 *            instead of Kaldi's sequential order (VOSK_AMD_DEC_ORDER overrides). */
VamdEngine *vamd_engine_new(const char *model_dir, int frames_per_chunk, int max_streams,
                            int flags);
void vamd_engine_free(VamdEngine *e);
/* pipeline mode: run the pending decoder step (no-op otherwise) */
int vamd_engine_flush(VamdEngine *e);
/* human-readable nnet plan / engine description (owned by the engine) */
const char *vamd_engine_describe(VamdEngine *e);
/* plan facts: [fpc, fss, left_ctx, right_ctx, priming, out_dim, ops, ring] */
int vamd_engine_info(VamdEngine *e, int *out8, double *flops_per_chunk);

int vamd_stream_new(VamdEngine *e);
int vamd_stream_free(VamdEngine *e, int stream);
/* input sample rate of a stream (default: the model's); others are resampled
 * on the GPU (windowed sinc, Kaldi LinearResample; replaces the resampling of
 * the reference's feature pipeline, src/model.cc:221, and batch path,
 * src/batch_recognizer.cc:27-29).  Set before the stream's first samples. */
int vamd_stream_set_rate(VamdEngine *e, int stream, int rate);
int vamd_stream_reset(VamdEngine *e, int stream, int pipeline);
/* queue samples (int16-range floats); finished=1 marks end of input */
int vamd_stream_accept(VamdEngine *e, int stream, const float *samples, int n, int finished);
/* run batched engine steps over the listed streams until no work remains */
int vamd_engine_advance(VamdEngine *e, const int *streams, int n);
int vamd_stream_frames_decoded(VamdEngine *e, int stream);
int vamd_stream_error(VamdEngine *e, int stream);
/* device decoder state: {tokens, arena tokens used, frames, lattice links
   used, err, lattice overflow, prune_from, last pruned frame} */
int vamd_stream_decoder_state(VamdEngine *e, int stream, long long *out8);
/* feature rows [first, first+n) from the device ring, n*dim floats */
int vamd_stream_features(VamdEngine *e, int stream, int first, int n, float *out);
/* decoded log-likelihood rows (flag 2): copies up to cap floats, returns count */
long long vamd_stream_llh(VamdEngine *e, int stream, float *out, long long cap);
/* i-vector of every chunk computed so far (flag 2), [chunks][ivector dim]:
 * copies up to cap floats, returns the count; ivector dim 0 = no i-vector input */
long long vamd_stream_ivectors(VamdEngine *e, int stream, float *out, long long cap);
int vamd_engine_ivector_dim(VamdEngine *e);
/* state-level lattice of a stream's decoder segment (engine flag 16): call
 * with frame_begin == NULL to build it and get sizes4 = [frames, tokens,
 * links, final costs | overflow << 30], then again with arrays of those sizes
 * ([frames + 2], [tokens] x2, [links] x5, [final costs]) to copy it out.
 * Link acoustic costs have the frame's cost offset removed (Kaldi GetRawLattice). */
int vamd_stream_lattice(VamdEngine *e, int stream, int use_final, int *sizes4, int *frame_begin,
                        int *tok_state, float *tok_cost, int *link_src, int *link_dst, int *link_arc,
                        float *link_graph, float *link_ac, float *final_cost);
/* silence weighting of the i-vector statistics (the reference Recognizer's
 * UpdateSilenceWeights, src/recognizer.cc:226-237): call after accepting
 * samples and before advancing; first_decoder_frame = feature frame of the
 * decoder segment's frame 0.  Returns 1 if active for the model, 0 if not. */
int vamd_stream_update_silence_weights(VamdEngine *e, int stream, int first_decoder_frame);
/* per-frame stats of the last advance (flag 1): 8 floats per frame
 * {ntok_in, ntok_out, arcs_emit, arcs_eps, best, cutoff, next_cutoff, adaptive_beam} */
int vamd_stream_stats(VamdEngine *e, int stream, float *out, int cap_frames);
/* decode externally supplied log-likelihoods [nframes][out_dim] */
int vamd_stream_decode_llh(VamdEngine *e, int stream, const float *llh, int nframes, int reset);
/* best path: arc indices into the graph (emitting-first CSR order) */
int vamd_stream_best_path(VamdEngine *e, int stream, int use_final, int *arcs, int cap,
                          double *cost, float *final_relative_cost);
/* The same path from the segment's lattice records copied to the host
 * (final costs used when any token is final): the batch path's fallback
 * words when a segment's lattice is unusable.  Returns the arc count. */
int vamd_stream_segment_best_path(VamdEngine *e, int stream, int *arcs, int cap);
/* upload a stream's whole audio into HBM (read by later steps, no per-step
 * host->device copy); finished=1 marks end of input after it */
int vamd_stream_preload(VamdEngine *e, int stream, const float *samples, long long n, int finished);
/* exactly one batched step over the listed streams: 1 = ran, 0 = idle */
int vamd_engine_step(VamdEngine *e, const int *streams, int n);
/* samples each stream consumes per step (default: chunk + margin) */
int vamd_engine_set_step_samples(VamdEngine *e, int n);
/* HIP-event stage times (flag 4): ms and launch counts for
 * [samples+MFCC, nnet ops, decoder, whole step]; reset=1 clears them */
int vamd_engine_stage_times(VamdEngine *e, double *ms4, long long *launches4, int reset);
/* decoder work since the last stage-time reset (flag 1): [frames, tokens in,
 * tokens out, emitting arcs examined, epsilon arcs examined, lattice links
 * written] */
int vamd_engine_decoder_totals(VamdEngine *e, long long *out6);
/* decoder phase clocks (env VOSK_AMD_DEC_PROFILE=1), summed over streams:
 * the first eight of the decoder's counters [cutoff, seed, exp_tokens,
 * exp_items, exp_winners, eps, commit_toks, commit_links] (s_memtime clocks;
 * the full list is vosk/engine.py Engine.PHASES) */
int vamd_engine_decoder_phases(VamdEngine *e, long long *out8);
/* all decoder phase counters: writes min(cap, N) values, returns N (43) */
int vamd_engine_decoder_phases_n(VamdEngine *e, long long *out, int cap);
/* the N counters per stream slot: out[max_streams][N] */
int vamd_engine_decoder_phases_per_stream(VamdEngine *e, long long *out);
/* engine counters: [steps, launches, mfcc frames, chunk jobs, frames decoded] */
int vamd_engine_counters(VamdEngine *e, long long *out5);

/* ---- batch path diagnostics (the VoskBatchModel of vosk_api.h) ---- */
struct VoskBatchModel;
/* GPU lanes of a batch model (one engine + batcher thread per GPU) */
int vamd_batch_lanes(struct VoskBatchModel *m);
/* one lane: load3 = {device, streams, pending chunks}; with env
 * VOSK_AMD_BATCH_TIMING=1 / VOSK_AMD_BATCH_STATS=1 at model creation also the
 * lane engine's stage times (as vamd_engine_stage_times) and decoder totals
 * (as vamd_engine_decoder_totals); reset=1 clears them.  Call while the lane
 * is quiescent (after vosk_batch_model_wait). */
int vamd_batch_lane_stats(struct VoskBatchModel *m, int lane, int *load3, double *ms4,
                          long long *launches4, long long *dec6, int reset);
/* one lane's device memory: {bytes allocated, token arena per stream, link
 * arena per stream, the highest token / link arena fill of any stream after
 * a decoder launch (the in-kernel pruning compacts them)} */
int vamd_batch_lane_memory(struct VoskBatchModel *m, int lane, long long *out5);
/* the lane's token-passing order: 1 Kaldi's sequential order (the CPU
 * reference's LatticeFasterDecoder), 0 the order-independent form */
int vamd_batch_lane_kaldi_order(struct VoskBatchModel *m, int lane);
/* result production totals: {segments, lattice links copied, ms copying
 * (lane threads), ms building raw lattices, ms prune + determinize + align,
 * ms MBR, ms formatting} */
int vamd_batch_result_profile(struct VoskBatchModel *m, double *out13);
/* dynamic batching: {lane steps, bounded waits that expired (a feeding
 * round split in two steps), waits ended by a vosk_batch_model_wait caller
 * before the round was complete, decoder jobs of one stream completed with
 * no endpoint probe between them (must stay 0)} */
int vamd_batch_batching_counters(struct VoskBatchModel *m, long long *out4);
/* the lane's dynamic batching rule (host only, no GPU): 1 if a step would
 * still wait for streams of the feeding round, given each stream's chunks
 * pushed, chunks handed to the engine and input-ended flag */
int vamd_feeding_round_incomplete(int n, const long long *pushed, const long long *taken, const int *ended);
/* stream -> lane index it was admitted to */
int vamd_batch_recognizer_lane(struct VoskBatchRecognizer *r);
/* admission policy (host only, no GPU): replays `n` admissions against lanes
 * whose pending-chunk loads drain at the given per-admission rates; writes
 * the lane of each admission to out[n] */
int vamd_admission_replay(int lanes, const int *drain_per_step, int n, const int *chunks, int *out);

#ifdef __cplusplus
}
#endif
#endif
