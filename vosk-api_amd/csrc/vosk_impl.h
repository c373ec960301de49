// Vosk object layer on top of the GPU engine: Model, Recognizer, BatchModel,
// BatchRecognizer.  Mirrors the reference's objects (src/model.h:41-104,
// src/recognizer.h:43-111, src/batch_model.h:43-66,
// src/batch_recognizer.h:28-53) and their state machines.
#pragma once

#include <array>
#include <atomic>
#include <functional>
#include <condition_variable>
#include <deque>
#include <map>
#include <exception>
#include <memory>
#include <mutex>
#include <queue>
#include <string>
#include <thread>
#include <vector>

#include "engine.h"
#include "incremental.h"
#include "xvector.h"
#include "json_out.h"

namespace vamd {

// One decoded word of the best path (frames are decoder frames).
struct WordSeg {
  int word;
  int start, end;
};
std::vector<WordSeg> PathWords(const ModelData& m, const std::vector<int>& arcs);
int TrailingSilenceFrames(const ModelData& m, const std::vector<int>& arcs);
// Best path (arc indices) of a segment from its copied lattice records, by the
// traceback kernel's rule (the batch path's fallback words).
std::vector<int> SegmentBestPath(const Graph& g, const SegmentLattice& sl);
// OnlineEndpointConfig rules (Kaldi online2/online-endpoint.cc [K]).
bool EndpointRulesFire(const EndpointConfig& c, int frames_decoded, int trailing_sil,
                       float frame_shift_s, float final_relative_cost);

class Recognizer;

// The streaming recognizers on one engine.  Applications run one recognizer
// per connection thread (vosk-server); their AcceptWaveform / FinalResult
// calls arriving together are served by one batched pass (group commit):
// per 0.2-s piece one UpdateSilenceWeights traceback launch and one Advance
// over all their streams, then one endpoint traceback launch, where each
// call alone would run its own.  Per-stream results are unchanged.
struct RecognizerGroup {
  explicit RecognizerGroup(Engine* e);
  std::unique_ptr<Engine> engine;
  SlotGroupCommit gc;
  std::vector<Recognizer*> by_slot;
  // the leader's batched pass; a request with pieces left after the pass's
  // decoder round is not complete (carried into the next pass)
  void Serve(const std::vector<int>& slots, std::vector<char>* complete);
};

class Model {
 public:
  explicit Model(const std::string& path);
  void Ref() { ref_.fetch_add(1); }
  void Unref() {
    if (ref_.fetch_sub(1) == 1) delete this;
  }
  int FindWord(const std::string& w) const;
  const std::shared_ptr<ModelData>& data() const { return md_; }
  // A free stream slot on one of the model's stream engines (created
  // lazily; a new engine of VOSK_AMD_MAX_STREAMS slots when all are full).
  // At most VOSK_AMD_MAX_STREAM_ENGINES (default 16) engines; an engine
  // other than the first is released when its last recognizer is freed.
  RecognizerGroup* AllocStreamSlot(int* slot);
  void FreeStreamSlot(RecognizerGroup* g, int slot);
  // Engine of the grammar recognizers with this phrase list (JSON array of
  // strings, src/recognizer.cc:49-108): the runtime graph HCLr o G(grammar),
  // one engine per distinct grammar, created on first use.  Models without
  // HCLr.fst warn and return null (the caller takes a static-graph stream
  // slot, as the reference falls back to its static graph).
  RecognizerGroup* GrammarEngine(const std::string& grammar);

 private:
  ~Model() = default;
  std::shared_ptr<ModelData> md_;
  std::vector<std::unique_ptr<RecognizerGroup>> engines_;  // stream engines
  std::map<std::string, std::unique_ptr<RecognizerGroup>> grammar_engines_;
  std::mutex mu_;
  std::atomic<int> ref_{1};
};

// Speaker model (src/spk_model.cc): refcounted like Model; the GPU x-vector
// extractor is created on first use on the recognizers' device.
class SpkModel {
 public:
  explicit SpkModel(const std::string& dir);
  void Ref() { ref_.fetch_add(1); }
  void Unref() {
    if (ref_.fetch_sub(1) == 1) delete this;
  }
  const SpkModelData& data() const { return *md_; }
  SpkExtractor* Extractor();

 private:
  ~SpkModel() = default;
  std::shared_ptr<SpkModelData> md_;
  std::unique_ptr<SpkExtractor> ex_;
  std::mutex mu_;
  std::atomic<int> ref_{1};
};

enum RecognizerState { RECOGNIZER_INITIALIZED, RECOGNIZER_RUNNING, RECOGNIZER_ENDPOINT,
                       RECOGNIZER_FINALIZED };

class Recognizer {
 public:
  Recognizer(Model* model, float sample_frequency);
  Recognizer(Model* model, float sample_frequency, const char* grammar);
  Recognizer(Model* model, float sample_frequency, SpkModel* spk);
  // src/recognizer.cc:259-268 (refused while an utterance is running)
  void SetSpkModel(SpkModel* spk);
  ~Recognizer();
  void SetMaxAlternatives(int n) { max_alternatives_ = n; }
  void SetWords(bool w) { words_ = w; }
  void SetPartialWords(bool w) { partial_words_ = w; }
  void SetNLSML(bool n) { nlsml_ = n; }
  bool AcceptWaveform(const char* data, int len);
  bool AcceptWaveform(const short* data, int len);
  bool AcceptWaveform(const float* data, int len);
  const char* Result();
  const char* PartialResult();
  const char* FinalResult();
  void Reset();

 private:
  bool AcceptWaveform(std::vector<float>& wave);
  void CleanUp();
  const char* GetResult();
  const char* StoreEmptyReturn();
  const char* StoreReturn(const std::string& s);
  std::string WordsText(const std::vector<WordSeg>& w) const;
  // GetSpkVector (src/recognizer.cc:356-419): the segment's non-silence
  // frames on the best path -> x-vector on the GPU
  bool GetSpkVector(std::vector<float>* xvec, int* num_frames);

  friend struct RecognizerGroup;
  // AcceptWaveform / FinalResult through the group's batched pass
  bool Submit(const std::vector<float>* wave, bool final);
  // The decoder segment's incremental lattice (incremental.h): the group's
  // passes record every AdvanceDecoding end (the segment's decoded frames
  // after it); SyncLattice copies the frames decoded since the last call and
  // replays those ends on them.  False if the records are unusable (lattice
  // overflow): the results fall back to the best path.
  bool SyncLattice();
  void ResetLattice();
  // The replay also runs in the background between calls (a lattice worker
  // after each AcceptWaveform), so a result finds most of it done; every
  // foreground use waits for a running task first.
  void KickLattice();
  void WaitLattice();
  bool SyncLatticeWork(bool background);
  // the MBR of an incremental lattice (graph scale, rescoring, alignment as
  // the reference's GetResult / PartialResult); false: empty lattice
  bool LatticeMbr(WordLattice&& wl, float graph_scale, bool rescore, MbrResult* r) const;

  Model* model_;
  RecognizerGroup* group_ = nullptr;
  bool grammar_group_ = false;  // a grammar engine's slot (else a model stream engine's)
  Engine* engine_;
  int slot_;
  // the request the group's batched pass serves (Submit)
  const std::vector<float>* req_wave_ = nullptr;
  bool req_final_ = false, req_endpoint_ = false;
  size_t req_piece_ = 0;  // the request's next 0.2-s piece (carried across passes)
  std::exception_ptr req_error_;  // this stream's own failure in a group pass
  float sample_frequency_;
  int max_alternatives_ = 0;
  bool words_ = false, partial_words_ = false, nlsml_ = false;
  int frame_offset_ = 0;
  long long samples_processed_ = 0, samples_round_start_ = 0;
  RecognizerState state_ = RECOGNIZER_INITIALIZED;
  IncrementalLattice inc_;
  std::mutex inc_mu_;  // adv_ends_ (appended by the group's passes), inc_busy_
  std::condition_variable inc_cv_;
  bool inc_busy_ = false;  // a background replay is running
  bool inc_init_ = false, inc_bad_ = false;
  std::vector<int> adv_ends_;  // AdvanceDecoding ends of the segment (decoded frames)
  size_t adv_done_ = 0;        // ends replayed
  int inc_next_frame_ = 0;     // the next frame record to ingest
  LatFrame inc_last_{};        // the last ingested frame's record (a compaction check)
  int inc_last_prune_ = 0;     // DecSlot::last_prune at the last copy (another compaction check)
  std::string last_result_;
  std::vector<float> resample_buf_;
  SpkModel* spk_ = nullptr;
  std::vector<float> spk_samples_;  // the speaker front end's input since its last reset
};

class BatchRecognizer;

// Admission policy of the batch path: the lane with the
// fewest pending chunks, then the fewest streams, then the lowest index.
// loads[i] = {pending chunks, streams}.
int PickLane(const std::vector<std::array<int, 2>>& loads);

// Dynamic batching rule of a lane: per stream {chunks
// pushed, chunks handed to the engine, input ended}.  The feeding round's
// chunk number n is the furthest queued chunk (a stream with a queued chunk
// offers chunk handed+1); the round is incomplete while a running stream that
// pushed chunk n-1 has not pushed chunk n.
bool FeedingRoundIncomplete(const std::vector<std::array<long long, 3>>& streams);

// Host threads for the batch path's result production: segment lattice ->
// word lattice -> MBR -> JSON, off the GPU lanes' critical path (the
// reference runs lattice post-processing on num_worker_threads=-1 worker
// threads, src/batch_model.cc:69, callback src/batch_recognizer.cc:138-149).
class WorkerPool {
 public:
  explicit WorkerPool(int threads, int nice = 0);
  ~WorkerPool();
  void Submit(std::function<void()> task);
  void WaitIdle();
  // runs one queued task on the calling thread (an idle lane or a caller
  // waiting in Wait() helps with the final segments); false: none queued
  bool RunOne();
  int size() const { return (int)threads_.size(); }

 private:
  void Run();
  struct TaskScope;
  std::mutex mu_;
  std::condition_variable cv_, idle_cv_;
  std::deque<std::function<void()>> tasks_;
  int busy_ = 0;
  bool stop_ = false;
  std::vector<std::thread> threads_;
};

// The batch path (src/batch_model.cc:23-121): one model, one GPU engine and
// one batcher thread ("lane") per visible MI355X.  A BatchRecognizer is
// admitted once, to the lane with the fewest pending chunks (then the fewest
// streams), and stays there (independent streams, no data-path
// collective).  Each lane thread steps its engine's three-stage pipeline over
// every stream with queued chunks (one chunk per stream per step), checks
// endpoints on the decoder state between steps without draining the
// pipeline (reset_on_endpoint, src/batch_model.cc:72: the segment ends after
// the frames decoded so far, exactly as an in-order reset), and hands each
// finished segment's lattice to the result workers.
class BatchModel {
 public:
  explicit BatchModel(const std::string& dir = "model");
  // Refcounted like Model: vosk_batch_model_free drops the caller's
  // reference, every BatchRecognizer holds one, so recognizers freed after
  // their model (any binding's garbage-collection order) stay valid.
  void Ref() { ref_.fetch_add(1); }
  void Unref() {
    if (ref_.fetch_sub(1) == 1) delete this;
  }
  void WaitForCompletion();  // src/batch_model.cc:118-121
  const ModelData& data() const { return *md_; }
  int samples_per_chunk() const { return samples_per_chunk_; }
  int num_lanes() const { return (int)lanes_.size(); }
  // Admission: picks the lane, allocates the stream slot on its engine.
  void Admit(BatchRecognizer* r, int rate);
  // Waits until the stream has no queued work and no result in production.
  void Release(BatchRecognizer* r);
  void Push(BatchRecognizer* r, std::vector<float>&& chunk, bool last);
  int PendingChunks(const BatchRecognizer* r);
  // per lane: {device, streams, pending chunks}
  std::vector<std::array<int, 3>> LaneLoads();
  Engine* lane_engine(int i) { return LaneEngine(i); }
  // result production totals: {segments, lattice links copied, ms copying
  // (lane thread), ms building raw lattices, ms prune + determinize + align,
  // ms MBR, ms formatting}
  void ResultProfile(double* out7) const;
  int LaneOf(const BatchRecognizer* r) const;
  void BatchingCounters(long long* out4) const;

 private:
  struct Lane;
  Engine* LaneEngine(int i);
  void LaneLoop(Lane* L);
  static bool RoundIncomplete(const std::vector<BatchRecognizer*>& recs);
  // Segments of streams rs end (endpoint or end of stream): their lattice
  // records copied from HBM now (batched), MBR and JSON on the result workers.
  void EmitSegments(Lane* L, const std::vector<BatchRecognizer*>& rs, bool final_segment);
  void EmitSegment(Lane* L, BatchRecognizer* r, bool final_segment, std::shared_ptr<SegmentCopy> copy,
                   int frames);
  std::shared_ptr<ModelData> md_;
  int samples_per_chunk_ = 0;
  std::vector<std::unique_ptr<Lane>> lanes_;
  std::unique_ptr<WorkerPool> pool_;
  std::mutex admit_mu_;
  std::atomic<int> ref_{1};
  // segment lattice buffers recycled between segments (their vectors keep
  // their capacity: no fresh allocation and page faults per copy)
  std::shared_ptr<SegmentLattice> TakeSegmentBuffer();
  void ReturnSegmentBuffer(std::shared_ptr<SegmentLattice> sl);
  std::mutex sl_mu_;
  std::vector<std::shared_ptr<SegmentLattice>> sl_pool_;
  // ResultProfile (ns except counts): segments, links, copy, build, det, MBR,
  // format; lane loop: dynamic batching wait, step, endpoints, finals, steps;
  // endpoint probe launches (within endpoints)
  std::atomic<long long> prof_[13] = {};
  // dynamic batching: {steps, bounded waits that expired (split rounds),
  // waits ended by a Wait() caller}
  // development (VOSK_AMD_FINISH_TRACE): the FinishStream tail's timeline on stderr
  bool fin_trace_ = false;
  std::atomic<long long> fin_t0_{0}, fin_last_{0};
  std::atomic<long long> batching_[4] = {};  // steps, split rounds, released by Wait, merged probes
  ~BatchModel();
};

class BatchRecognizer {
 public:
  BatchRecognizer(BatchModel* model, float sample_frequency);
  ~BatchRecognizer();
  void AcceptWaveform(const char* data, int len);
  void FinishStream();
  void SetNLSML(bool n) { nlsml_ = n; }
  const char* FrontResult();
  void Pop();
  int GetNumPendingChunks() { return model_->PendingChunks(this); }
  int lane() const { return lane_; }

 private:
  friend class BatchModel;
  struct Chunk {
    std::vector<float> data;
    bool last;
  };
  // results are produced out of order by the worker pool and published in
  // segment order
  void PublishResult(uint64_t seq, std::string&& json);
  std::string FormatResult(const MbrResult& r, double offset_s) const;  // PushLattice

  BatchModel* model_;
  bool nlsml_ = false;
  std::vector<float> buffer_;  // model-rate samples not yet pushed as a chunk
  int call_rate_ = 0;          // input rate resampled per call (0: the model's rate)
  int call_table_ = -1;        // its table on the lane's engine (and a host copy)
  ResampleTable call_tab_;
  // lane state (guarded by the lane's mutex)
  int lane_ = -1, slot_ = -1;
  std::deque<Chunk> queue_;
  int handed_ = 0;          // chunks given to the engine whose work is not finished
  long long pushed_ = 0;    // chunks pushed since admission (the stream's chunk sequence)
  long long taken_ = 0;     // chunks handed to the engine since admission
  bool busy_ = false;       // has work in the engine
  bool finishing_ = false;  // last chunk handed: final result when the stream is idle
  int tasks_ = 0;           // results in production on the worker pool
  bool ended_ = false;      // FinishStream pushed: Wait() also covers its results in production
  double segment_offset_ = 0;  // seconds at the start of the current segment
  long long utt_samples_ = 0;  // model-rate samples handed to the engine since the utterance began
  uint64_t next_seq_ = 0;
  // results
  std::mutex rmu_;
  uint64_t publish_seq_ = 0;
  std::map<uint64_t, std::string> reorder_;
  std::deque<std::string> results_;
  std::string front_;
  int front_state_ = -1;  // last FrontResult: 1 a result, 0 none (Pop then pops nothing), -1 not read
};

}  // namespace vamd
