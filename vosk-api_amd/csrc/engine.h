// GPU engine: owns the device copy of one model and the device-resident state
// of up to `max_slots` concurrent streams, and advances any set of streams
// through MFCC -> looped nnet3 -> token passing in batched launches.
//
// It is the MI355X replacement of what the reference obtains from Kaldi's
// online2 / nnet3 / decoder libraries (CPU path, src/recognizer.cc:297-323)
// and from BatchedThreadedNnet3CudaOnlinePipeline + CudaDecoder (batch path,
// src/batch_model.cc:69-98).  Streams are independent: one engine step batches
// every stream that has work, so the single-stream Recognizer and the
// BatchRecognizer share the same kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <exception>
#include <atomic>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "engine_dev.h"
#include "model_io.h"
#include "nnet_plan.h"
#include "resample.h"
#include "lattice.h"
#include "rescore.h"
#include "silence.h"

namespace vamd {

// Host copy of everything read from a model directory.
struct ModelData {
  std::string dir;
  MfccOptions mfcc;
  DecoderOptions dec;
  DecodableOptions dcb;
  EndpointConfig endpoint;
  TransitionModel tm;
  Nnet nnet;
  Graph graph;
  // Lookahead models (graph/HCLr.fst + graph/Gr.fst, src/model.cc:282-285):
  // the HCLr FST and disambiguation transition-ids, kept for the grammar
  // recognizers' runtime graphs (graph_compose.h); null for HCLG models.
  std::shared_ptr<const HostFst> lookahead_hcl;
  std::vector<int> disambig;
  // rescore/G.fst + rescore/G.carpa (src/model.cc:308-314): LM rescoring of
  // final results (rescore.h); null without them
  std::shared_ptr<const RescoreLm> rescore;
  SymbolTable words;
  std::vector<char> phone_is_silence;  // indexed by phone id
  bool has_word_boundary = false;
  // word_boundary.int (WordBoundaryInfo): per phone 1 nonword, 2 begin,
  // 3 end, 4 internal, 5 singleton (0 = unlisted)
  std::vector<char> phone_boundary;
  std::vector<char> tid_boundary;  // the same per transition-id (word alignment)
  bool use_ivector = false;            // ivector/final.ie present (src/model.cc:247)
  IvectorModel ivec;
  // global_cmvn.stats present (src/model.cc:265-269): online CMVN (window 600,
  // 200 global frames, mean only) on the nnet input features
  bool use_cmvn = false;
  std::vector<double> global_cmvn;     // [2][feat_dim + 1]
  // Loads a V2 (am/, conf/, graph/) or V1 (flat) layout (src/model.cc:106-128).
  void Load(const std::string& dir);
  void LoadBatchLayout(const std::string& dir);  // src/batch_model.cc:23-54
};

// host tables of the MFCC / fbank front end (mfcc_kernel); pointers in dev unset
struct MfccTables {
  MfccDev dev{};
  std::vector<float> win, melw, dct, lift, twr, twi;
  std::vector<int> first, last;
};
MfccTables BuildMfccTables(const MfccOptions& o);

struct EngineConfig {
  int frames_per_chunk = 21;
  int max_slots = 64;
  int max_step_samples = 8192;  // samples consumed per stream per step
  int max_tokens = 1 << 16;     // token list capacity per stream per frame
  long long arena_tokens = 1 << 21;  // backpointer arena per stream
  int device = 0;
  bool collect_stats = false;
  bool collect_llh = false;  // tests: keep a host copy of every decoded LLH row
  bool time_kernels = false; // HIP-event timing of each stage on the engine stream
  // Three-stage pipeline over three HIP streams: one engine step runs the
  // front end (samples, MFCC, i-vectors) of step s, the nnet of step s-1 and
  // the decoder of step s-2 concurrently (staging triple-buffered, LLH and
  // per-job i-vectors double-buffered).  Results lag two steps; every call
  // that reads or resets decoder state drains the pipeline first.
  bool pipeline = false;
  // Lattice generation: the decoder keeps Kaldi's forward links in HBM per
  // stream (engine_dev.h LatFrame); GetRawLattice reads the segment's.
  bool lattice = false;
  long long lattice_links = 1 << 22;  // link arena per stream (16 B each)
  int lattice_frames = 1 << 14;       // frames per decoder segment with a lattice
  // The KaldiRecognizer's incremental lattice is kept on the host
  // (incremental.h), which reads a segment's records as they come: the
  // in-kernel pruning passes (which compact the arenas) then run only when a
  // stream's arena is half full, never by segment length.
  bool host_lattice = false;
  // the in-kernel pruning also starts once a stream's token or link arena is
  // this full (percent; VOSK_AMD_DEC_PRUNE_FILL overrides)
  int prune_fill_pct = 50;
  bool track_decoded = false;  // record completed decoder jobs for TakeDecoded
  // token passing in Kaldi's sequential order (LatticeFasterDecoder's HashList
  // order, running emitting cutoff, LIFO epsilon queue: the reference's
  // KaldiRecognizer decoder), else the order-independent form (the
  // deterministic form of the reference's batch CudaDecoder, BatchModel's
  // default); env VOSK_AMD_DEC_ORDER=kaldi|parallel overrides
  bool kaldi_order = true;
};

// HIP-event times accumulated on the engine stream (time_kernels).
struct StageTimes {
  double ms[4] = {0, 0, 0, 0};     // 0 samples+MFCC, 1 nnet ops, 2 decoder, 3 whole step
  long long launches[4] = {0, 0, 0, 0};
  // decoder work totals (collect_stats): frames, tokens in, tokens out,
  // emitting arcs examined, epsilon arcs examined
  long long dec[6] = {0, 0, 0, 0, 0, 0};  // [5] lattice links written
};

struct PathResult {
  std::vector<int> arcs;  // best path arc indices (forward order)
  float end_cost = 0;     // tot_cost (+ final) of the end token
  double cost = 0;        // offset-corrected path cost
  float final_relative_cost = 0;
  int end_state = -1;
};

// A decoder segment's lattice records copied from HBM (GetRawLattice input;
// BuildRawLattice turns them into the canonical state-level lattice).
struct SegmentLattice {
  std::vector<LatFrame> frames;
  std::vector<int4> arena, links;
  bool overflow = false;  // link arena / frame table overflow or decoder error
  // CopySegmentTail: frames from first_frame, arena from arena_base, links
  // from link_base (0 for a whole segment)
  int first_frame = 0, arena_base = 0;
  long long link_base = 0;
  int last_prune = 0;  // DecSlot::last_prune (a pruning pass compacts the records: it changes)
};

// Pinned host blocks for asynchronous segment copies, shared by an engine
// and the copies in flight (thread-safe; blocks are reused by size).
class PinnedPool {
 public:
  ~PinnedPool();
  char* Take(size_t bytes, size_t* cap);
  void Give(char* p, size_t cap);

 private:
  std::mutex mu_;
  std::vector<std::pair<size_t, char*>> free_;
};

// One StartSegmentCopies call's pinned block and completion event, shared by
// the call's segments: the block goes back to the pool and the event is
// destroyed when the last segment has been finished (one host allocation and
// one event per call, not per segment).
struct CopyBatch {
  std::shared_ptr<PinnedPool> pool;
  char* block = nullptr;
  size_t cap = 0;
  hipEvent_t done = nullptr;
  int device = 0;
  ~CopyBatch();
};

// A segment's records being copied to the host (StartSegmentCopies): the
// consumer calls Finish, which waits for the copy and fills the lattice.
struct SegmentCopy {
  std::shared_ptr<CopyBatch> batch;
  size_t f = 0, a = 0, l = 0;
  int nf = 0, na = 0;
  long long nl = 0;
  bool overflow = false;
  void Finish(SegmentLattice* out);  // once, from any thread
};

struct EndpointProbe {
  int frames = 0, trailing_sil = 0;
  float final_relative_cost = 0;
};

struct EngineCounters {
  long long steps = 0, launches = 0, frames_mfcc = 0, chunk_jobs = 0, frames_decoded = 0;
};

constexpr int kMaxResampleTables = 32;  // distinct input sample rates per engine

// Group commit of per-stream requests: callers on different threads (one
// stream each) are served together by one batched call made by whichever
// caller leads; each Run returns once a batch that started after its call
// has served its stream (the batch's exception, if any, is rethrown in every
// caller it served).
//
// Coalescing window: the callers a batch served come back with their next
// request right after it (vosk-server's shape: one thread per stream calling
// in a loop), while the next batch would start at once with only the
// requests that arrived during the last one -- the streams would settle into
// groups served by alternating batches, each decoder launch with a fraction
// of them.  So a batch waits, bounded by window_us after the previous batch
// ended, until the streams the previous batch served have posted again (a
// stream whose caller stops is waited for at most that long, once).  The
// serving order of each stream's requests is unchanged (results too: streams
// are independent in every kernel).
//
// Carried requests: the batched call may leave a request unfinished (it marks
// the finished ones in `complete`); an unfinished request leads the next batch
// (its caller keeps waiting), so a request's later work shares a batch with
// the requests posted meanwhile instead of running alone.
class SlotGroupCommit {
 public:
  void Resize(int slots) {
    req_.assign(slots, 0);
    done_.assign(slots, 0);
    err_.assign(slots, nullptr);
    owner_.assign(slots, std::thread::id());
    served_.assign(slots, std::chrono::steady_clock::time_point{});
    gap_us_.assign(slots, -1.0);
  }
  void SetWindowUs(int us) { window_us_ = us; }
  void SetAdaptive(bool on) { adaptive_ = on; }
  template <class BatchFn>
  void Run(int slot, BatchFn&& fn) {
    std::unique_lock<std::mutex> lk(mu_);
    const long long ticket = ++req_.at(slot);
    pending_.push_back(slot);
    owner_[slot] = std::this_thread::get_id();
    timed_out_.erase(slot);
    // the caller's gap between being served and posting again (a running
    // mean): a caller that does host work between its calls (e.g. a
    // PartialResult after every AcceptWaveform) longer than the window is not
    // waited for -- each batch would otherwise wait the whole window for it
    if (done_[slot] > 0) {
      const double g = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - served_[slot]).count();
      gap_us_[slot] = gap_us_[slot] < 0 ? g : 0.5 * gap_us_[slot] + 0.5 * g;
    }
    if (leader_ && waiting_) cv_lead_.notify_one();
    while (done_[slot] < ticket) {
      if (leader_) {
        cv_.wait(lk);
        continue;
      }
      leader_ = true;  // lead batches until this caller's stream is served
      while (done_[slot] < ticket && (!pending_.empty() || !carry_.empty())) {
        if (window_us_ > 0 && !last_.empty()) {
          const auto deadline = last_end_ + std::chrono::microseconds(window_us_);
          // (a stream whose caller is this thread cannot post meanwhile)
          const std::thread::id me = std::this_thread::get_id();
          auto all_back = [&] {
            for (int s : last_)
              if (req_[s] <= done_[s] && owner_[s] != me) return false;
            return true;
          };
          waiting_ = true;
          while (!all_back() && std::chrono::steady_clock::now() < deadline) cv_lead_.wait_until(lk, deadline);
          waiting_ = false;
          for (int s : last_)
            if (req_[s] <= done_[s] && owner_[s] != me) timed_out_.insert(s);
          last_.clear();
        }
        std::vector<int> batch;
        batch.swap(carry_);
        batch.insert(batch.end(), pending_.begin(), pending_.end());
        pending_.clear();
        std::vector<long long> tick;
        for (int s : batch) tick.push_back(req_[s]);
        lk.unlock();
        std::exception_ptr e;
        std::vector<char> complete(batch.size(), 1);
        try {
          fn(batch, &complete);
        } catch (...) {
          e = std::current_exception();
          complete.assign(batch.size(), 1);
        }
        lk.lock();
        // the streams to wait for next time: those served, except one that
        // never came back within the last window (its caller stopped) or
        // whose caller usually comes back later than the window
        last_end_ = std::chrono::steady_clock::now();
        last_.clear();
        for (size_t i = 0; i < batch.size(); i++) {
          const int s = batch[i];
          if (!complete[i]) {
            carry_.push_back(s);
            continue;
          }
          done_[s] = std::max(done_[s], tick[i]);
          err_[s] = e;
          served_[s] = last_end_;
          if (!timed_out_.count(s) && (!adaptive_ || gap_us_[s] < (double)window_us_)) last_.push_back(s);
        }
        cv_.notify_all();
      }
      leader_ = false;
      cv_.notify_all();  // a waiting caller with a pending stream leads next
    }
    if (err_[slot]) {
      std::exception_ptr e = err_[slot];
      err_[slot] = nullptr;
      std::rethrow_exception(e);
    }
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<long long> req_, done_;  // per stream: request / served tickets
  std::vector<std::thread::id> owner_;  // per stream: the thread of its last request
  std::vector<std::exception_ptr> err_;
  std::vector<int> pending_;
  std::vector<int> carry_;  // unfinished requests of the last batch (they lead the next)
  bool leader_ = false;
  // coalescing window (see above)
  int window_us_ = 0;
  bool adaptive_ = true;  // skip streams whose callers come back later than the window
  bool waiting_ = false;
  std::condition_variable cv_lead_;
  std::vector<int> last_;
  std::set<int> timed_out_;
  std::chrono::steady_clock::time_point last_end_{};
  std::vector<std::chrono::steady_clock::time_point> served_;  // per stream: end of its last batch
  std::vector<double> gap_us_;  // per stream: running mean of served -> next post (-1: none yet)
};

class Engine {
 public:
  Engine(std::shared_ptr<const ModelData> md, const EngineConfig& cfg);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  const NnetPlan& plan() const { return plan_; }
  const ModelData& model() const { return *md_; }
  const EngineConfig& config() const { return cfg_; }
  std::mutex& mutex() { return mu_; }

  int AllocSlot();
  int TryAllocSlot();  // -1 when every slot is in use
  void FreeSlot(int slot);
  int SlotsInUse();
  // New utterance: features restart at sample 0, decoder restarts.
  void ResetPipeline(int slot);
  // InitDecoding: the decoder restarts, the feature/nnet pipeline continues.
  void ResetDecoder(int slot);
  // Input sample rate of a stream (default: the model's); other rates are
  // resampled on the GPU (resample.h).  Set before the stream's first samples.
  void SetSampleRate(int slot, int rate);
  // One AcceptWaveform call of the batch path resampled on its own, flushed
  // at its end (the reference's BatchRecognizer: LinearResample::Resample(
  // input, flush = true) per call, src/batch_recognizer.cc:27-29,157-158):
  // the call's samples to the device, resample_kernel over the whole call,
  // the model-rate samples back.  Thread-safe; its own HIP stream.
  // ResampleTableFor: the table of an input rate (created on first use) and
  // a copy of it (its NumOutputSamples); ResampleCall then takes only the
  // calls' own lock, never the engine's (a lane step holds that one).
  int ResampleTableFor(int rate, ResampleTable* copy);
  std::vector<float> ResampleCall(int table, const ResampleTable& T, const float* x, int n);
  void AcceptSamples(int slot, const float* x, int n);
  // The same, taking the buffer (no copy when the stream's pending samples
  // are all consumed, the batch lane's usual case)
  void AcceptSamples(int slot, std::vector<float>&& x);
  // Uploads a stream's whole audio into HBM; later steps read it from there
  // (no host->device copy inside the steps).  finished: end of input after it.
  void PreloadSamples(int slot, const float* x, long long n, bool finished);
  // Exactly one batched step over the given streams; returns false if idle.
  // allow_pipeline=false (pipeline mode): this step's three stages run in
  // order after any pending pipeline stages (a batch with nothing behind it).
  bool Step(const std::vector<int>& slots, bool allow_pipeline = true);
  void SetStepSamples(int n) { cfg_.max_step_samples = n; }
  const StageTimes& stage_times() const { return times_; }
  bool kaldi_order() const { return dec_.kaldi != 0; }  // the decoder's token-passing order
  void ResetStageTimes() { times_ = StageTimes(); }
  void InputFinished(int slot);
  // Runs batched steps until the given streams have no runnable work
  // (drains the pipeline).
  void Advance(const std::vector<int>& slots);
  // Pipeline mode: runs the pending decoder step, if any.
  void Flush();
  int NumFramesDecoded(int slot) const;
  // host_lattice: the last frame of the stream's decoder segment whose
  // records the host has read (-1: none).  The in-kernel pruning pass, which
  // compacts the records, waits until it covers every decoded frame.
  void SetHostRead(int slot, int frame) { host_read_[slot].store(frame, std::memory_order_release); }
  // ... and true once that pass is due and waits for the host (as of the
  // stream's last launch): the host should read the records before the next
  // one, or the arenas fill up
  bool PruneWaiting(int slot) const { return prune_wait_[slot].load(std::memory_order_acquire) != 0; }
  int NumFramesReady(int slot) const;  // output frames available to the decoder
  bool InputIsFinished(int slot) const;
  int PendingSamples(int slot) const;
  int DecoderError(int slot) const;
  // device decoder state of a stream: {tokens, arena tokens used, frames,
  // lattice links used, err, lattice overflow, prune_from, last prune frame}
  void DecoderState(int slot, long long* out8);
  // Best path of the current utterance (batched over slots).  drain=false
  // (pipeline mode, between steps): the state as of the last completed
  // decoder job, without running the jobs still in the pipeline.
  void BestPaths(const std::vector<int>& slots, bool use_final, std::vector<PathResult>* out,
                 bool drain = true);
  // Optional per-frame decoder statistics of the last Advance (collect_stats).
  const std::vector<FrameStat>& LastStats(int slot) const;
  const EngineCounters& counters() const { return counters_; }
  // {device bytes, token arena per stream, link arena per stream, highest
  // token arena fill of any stream after a launch, highest link arena fill}
  void MemoryStats(long long* out5) const {
    out5[0] = (long long)dev_bytes_;
    out5[1] = cfg_.arena_tokens;
    out5[2] = cfg_.lattice ? cfg_.lattice_links : 0;
    out5[3] = arena_hwm_;
    out5[4] = links_hwm_;
  }
  // Tests: feature rows from the device ring; LLH rows decoded so far
  // (collect_llh); decoding of externally supplied log-likelihoods.
  void DebugFeatures(int slot, int first_frame, int n, std::vector<float>* out);
  const std::vector<float>& DecodedLlh(int slot) const { return slots_.at(slot).llh; }
  // Tests (collect_llh): the i-vector of every chunk computed so far [chunks][dim]
  const std::vector<float>& ChunkIvectors(int slot) const { return slots_.at(slot).ivecs; }
  int IvectorDim() const { return use_iv_ ? plan_.ivector_dim : 0; }
  void DecodeExternal(int slot, const float* llh, int nframes, bool reset);
  // Canonical state-level lattice of the stream's decoder segment (empty
  // without EngineConfig::lattice); use_final: final costs if any token is final.
  void GetRawLattice(int slot, bool use_final, RawLattice* out);
  // The segment's lattice records (drain as BestPaths); empty without a lattice.
  void CopySegmentLattice(int slot, SegmentLattice* out, bool drain = true);
  // Frames [from, decoded] of the segment with their tokens and links (the
  // recognizer's incremental lattice takes them as they come; drains).
  // upto: the last frame wanted (-1: every decoded frame).  concurrent: for
  // a stream engine without pipelining, from a thread other than the
  // stream's while passes over other streams run: no engine lock, plain
  // copies on the null stream, only frames <= upto read (their records are
  // final); out->overflow is also set when a pruning pass compacted the
  // stream's records meanwhile.
  void CopySegmentTail(int slot, int from, SegmentLattice* out, int upto = -1, bool concurrent = false);
  // The same for several streams with the copies batched.
  void CopySegmentLattices(const std::vector<int>& slots, const std::vector<SegmentLattice*>& outs,
                           bool drain = true);
  // The same, asynchronously (pipeline state as of the last completed decoder
  // job): the copies run on the copy stream, the next decoder launch waits for
  // them on the device, and each SegmentCopy is finished by its consumer.
  void StartSegmentCopies(const std::vector<int>& slots, std::vector<std::shared_ptr<SegmentCopy>>* out);

  // ---- asynchronous driving (BatchModel lanes: one thread steps the engine,
  // results are produced between steps without draining the pipeline)
  // Decoder jobs completed since the last call, in completion order;
  // input_ended: the job was built after the stream's input had ended (its
  // last frames; no endpoint check applies to it).
  struct DecodedJob {
    int slot;
    bool input_ended;
  };
  void TakeDecoded(std::vector<DecodedJob>* out);
  // Frames of the current decoder segment already decoded on the device.
  int DeviceFramesDecoded(int slot) const { return slots_.at(slot).dev_frames; }
  // Nothing of the stream is in the pipeline and nothing is runnable.
  bool StreamIdle(int slot) const;
  // Whether `extra` more host-fed samples would make a chunk of the stream
  // ready for the nnet and decoder (a prediction for batching decoder
  // launches; true when it cannot tell cheaply, e.g. a resampled stream)
  bool ChunkReadyAfter(int slot, long long extra) const;
  std::string DescribeSlot(int slot) const;  // development tracing
  bool PipelineBusy() const { return pendn_active_ || pend_active_; }
  // Ends the decoder segment after the frames decoded on the device so far:
  // the stream's next decoder job not yet launched restarts the decoder (a
  // job already staged in the pipeline gets its reset flag patched in HBM),
  // so the segment boundary is the same as with an in-order ResetDecoder.
  void ResetDecoderAtNextJob(int slot);
  // Endpoint inputs of the streams as of their last completed decoder job
  // (no drain): a traceback that stops at the first non-silence frame.
  // Requires silence phones (model endpoint configuration).
  void ProbeEndpoints(const std::vector<int>& slots, std::vector<EndpointProbe>* out);
  // Silence weighting of the i-vector statistics (Recognizer::UpdateSilenceWeights,
  // src/recognizer.cc:226-237): traceback of the stream's best path, weight
  // changes for the feature frames ready once the accepted samples are
  // consumed, queued for the stream's next i-vector requests.  No-op without
  // an i-vector extractor or silence phones.  first_decoder_frame = feature
  // frame of the decoder segment's frame 0 (frame_offset * 3).
  void UpdateSilenceWeights(int slot, int first_decoder_frame);
  // The same for several streams with one batched traceback.
  void UpdateSilenceWeights(const std::vector<int>& slots, const std::vector<int>& first_decoder_frame);
  bool SilenceWeightingActive() const { return use_iv_ && !md_->endpoint.silence_phones.empty(); }
  // i-vector feature frames ready once the accepted samples are consumed
  // (OnlineNnet2FeaturePipeline::NumFramesReady: the splice's right context
  // waits for more frames until input is finished)
  int IvectorFramesReady(int slot) const;
  // VOSK_AMD_DEC_PROFILE=1: summed s_memtime clocks per decoder phase and
  // event counts, kDecProf values (decoder.hip Prof); per_slot (optional):
  // the same per slot [max_slots][kDecProf]
  void DecoderPhaseClocks(long long* out, long long* per_slot = nullptr);

 private:
  struct SlotHost {
    bool used = false;
    std::vector<float> pending;
    size_t pending_pos = 0;
    long long samples = 0;   // samples pushed to the device since pipeline reset
    int frames = 0;          // MFCC frames computed
    int next_chunk = 0;      // next chunk index (negative while priming)
    int out_ready = 0;       // output frames computed
    int decoded = 0;         // frames decoded since the decoder reset (incl. a pending batch)
    int decoded_at_build = 0;
    int dev_frames = 0;      // frames of the decoder segment decoded on the device
    bool finished = false;
    bool need_reset = true;
    bool fresh_decoder = true;  // the pending reset starts a new decoder (Kaldi order: HashList size 1000)
    bool fresh_stream = true;   // ... of a new stream (reset 3: OpenFST's lazy numbering starts over)
    int err = 0;
    std::vector<FrameStat> stats;
    std::vector<float> llh;
    float* resident = nullptr;  // HBM-resident audio (PreloadSamples)
    long long resident_n = 0, resident_pos = 0;
    bool resident_finish = false;
    int rate = 0;              // input rate when resampled (0: model rate)
    int table = -1;            // resample table
    long long raw_pushed = 0;  // raw (input-rate) samples pushed to the raw ring
    bool res_flushed = false;  // resampler flushed at end of input
    bool iv_reset = true;      // i-vector state restarts at the next request
    bool cmvn_reset = true;    // nnet-input CMVN restarts at the next frames
    int iv_norm_done = 0, iv_norm_to = 0;  // frames CMVN-normalized (after this step)
    int iv_stats_done = 0;     // frames accumulated into the i-vector statistics
    std::vector<float> ivecs;  // collect_llh: per-chunk i-vectors
    long long links_seen = 0;  // lattice links counted so far (stage totals)
    // silence weighting: the decoder segment's weighting state and the
    // stream's queue of (feature frame, delta weight) not yet applied
    bool iv_weighted = false;
    std::vector<std::pair<int, float>> iv_pending;
    SilenceWeighting sw;
  };
  bool HasRunnableWork(const SlotHost& h) const;
  bool SlotInFlight(int slot) const;
  struct DecBatch {  // one decoder launch's jobs, staged in one staging buffer
    std::vector<DecJob> jobs;
    std::vector<int> expect;  // decoded-frame count each job's slot must reach
    size_t o_ej = 0;
    int buf = 0;  // staging buffer of the jobs
    int llh = 0;  // LLH buffer the nnet wrote
  };
  struct NnetBatch {  // one nnet pass: chunk jobs staged in one staging buffer
    int njobs = 0;
    size_t o_dj = 0;
    int buf = 0;
    int par = 0;  // LLH / i-vector buffer
    DecBatch dec;
  };
  bool BuildStep(const std::vector<int>& slots);
  void RunStep(bool allow_pipeline = true);
  void LaunchNnet(const NnetBatch& b, hipStream_t s);
  void LaunchDecodeBatch(const DecBatch& b, hipStream_t s);
  void FinishDecodeBatch(const DecBatch& b);
  void DrainOnce();  // pipeline tail: the pending nnet and decoder passes
  void FlushLocked();
  int NumFramesFor(long long samples) const;

  std::shared_ptr<const ModelData> md_;
  EngineConfig cfg_;
  NnetPlan plan_;
  std::mutex mu_;
  hipStream_t stream_ = nullptr;
  hipStream_t dstream_ = nullptr;  // decoder stream (pipeline mode)
  hipStream_t fstream_ = nullptr;  // front-end stream (pipeline mode)
  int ring_ = 0, sample_ring_ = 0, jobs_per_slot_ = 0;
  std::vector<SlotHost> slots_;
  std::unique_ptr<std::atomic<int>[]> host_read_;    // SetHostRead, per slot
  std::unique_ptr<std::atomic<char>[]> prune_wait_;  // PruneWaiting, per slot
  EngineCounters counters_;
  StageTimes times_;
  hipEvent_t ev_[7] = {};
  long long seq_ = 0;       // steps run: staging buffer seq % 3, LLH / i-vector buffer seq % 2
  bool pendn_active_ = false, pend_active_ = false;
  NnetBatch pendn_;         // pipeline mode: front end done, nnet waiting
  DecBatch pend_;           // pipeline mode: nnet done, decoder waiting
  std::vector<DecodedJob> decoded_;  // completed decoder jobs (TakeDecoded)

  // device: model
  MfccDev mfcc_{};
  std::vector<void*> dev_allocs_;
  size_t dev_bytes_ = 0;  // DevAlloc total (logged at construction)
  long long arena_hwm_ = 0, links_hwm_ = 0;  // MemoryStats
  std::vector<NnetOpArgs> op_args_;
  std::vector<int> op_bk_;
  float** d_ring_ptrs_ = nullptr;
  int* d_ring_dims_ = nullptr;
  RingSet rings_{};
  int4* d_sinfo_ = nullptr;
  int4* d_arcs_ = nullptr;
  unsigned char* d_arc_sil_ = nullptr;  // per arc: 0 epsilon, 1 silence phone, 2 other
  int* d_probe_ = nullptr;              // ProbeEndpoints buffers
  int* h_probe_ = nullptr;
  hipStream_t copy_stream_ = nullptr;  // segment lattice copies
  std::mutex tail_mu_;                  // host_lattice: CopySegmentTail's concurrent copies on copy_stream_
  double step_prof_[4] = {0, 0, 0, 0};  // Step host profile: build, sync wait, after sync, total (ms)
  long long step_prof_n_ = 0;
  double copy_prof_[4] = {0, 0, 0, 0};  // StartSegmentCopies: prune + state read, pinned take, rest (ms), MB copied
  long long copy_prof_n_ = 0;
  int ResampleTableLocked(int rate);    // the table of an input rate (created on first use)
  std::mutex call_mu_;                 // ResampleCall's stream and buffers
  hipStream_t call_stream_ = nullptr;
  // BestPaths' request / path block (device) and its read-back (pinned),
  // grown on demand: a per-call hipMalloc / hipFree would synchronize the
  // device on every partial result
  char* d_bp_ = nullptr;
  char* h_bp_ = nullptr;
  size_t bp_cap_ = 0;
  float* d_call_raw_ = nullptr;
  float* d_call_out_ = nullptr;
  ResampleJob* d_call_jobs_ = nullptr;
  size_t call_cap_raw_ = 0, call_cap_out_ = 0, call_cap_jobs_ = 0;
  char* h_lat_stage_ = nullptr;        // pinned staging of segment lattice copies
  size_t lat_stage_bytes_ = 0;
  long long copy_us_[4] = {0, 0, 0, 0}, copy_calls_ = 0;  // development (VOSK_AMD_COPY_DEBUG)
  std::shared_ptr<PinnedPool> pinned_ = std::make_shared<PinnedPool>();
  DecSlot* h_copy_slots_ = nullptr;  // decoder-state snapshot of the segment copies
  char* h_copy_stage_ = nullptr;     // pinned staging of the segment copies' slot list and gather items
  int* d_prune_slots_ = nullptr;
  unsigned* d_pack_ = nullptr;     // segment copies: records gathered on the device
  CopyItem* d_pack_items_ = nullptr;
  size_t pack_cap_ = 0, pack_items_cap_ = 0;     // stream list of the segments' final prune
  hipEvent_t copy_ev_ = nullptr;  // last asynchronous segment copy (decoder launches wait for it)
  bool copy_pending_ = false;
  // device: per-stream state
  float* d_samples_ = nullptr;
  float* d_raw_ = nullptr;  // [slots][raw_ring_] input-rate samples of resampled streams
  int raw_ring_ = 0, max_raw_step_ = 0;
  std::vector<ResampleTable> res_tables_;
  ResampleDev* d_res_tables_ = nullptr;  // [kMaxResampleTables]
  float* d_llh_ = nullptr;  // = d_llh_buf_[0]
  float* d_llh_buf_[2] = {nullptr, nullptr};
  DecArgs dec_{};
  DecSlot* d_slots_ = nullptr;
  FrameStat* d_stats_ = nullptr;
  // step staging (pinned host + device mirror)
  char* h_stage_ = nullptr;
  char* d_stage_ = nullptr;
  size_t stage_bytes_ = 0;
  DecSlot* h_slots_ = nullptr;
  FrameStat* h_stats_ = nullptr;
  // current step
  std::vector<SampleJob> st_samples_;
  std::vector<SampleJob> st_raw_;      // raw (input-rate) samples of resampled streams
  std::vector<int> st_raw_src_;
  std::vector<ResampleJob> st_res_;
  std::vector<int> st_sample_src_;  // offset into st_sample_data_, -1 = resident
  // host-fed samples of the step being built, written straight into the
  // step's pinned staging buffer (its first region)
  float* st_sample_data_ = nullptr;
  size_t st_sample_n_ = 0, stage_sample_cap_ = 0;
  void StageSamples(const float* x, size_t n);
  std::vector<MfccJob> st_mfcc_;
  int st_mfcc_total_ = 0;
  std::vector<DevJob> st_jobs_;
  std::vector<DecJob> st_dec_;
  std::vector<IvStreamJob> st_iv_jobs_;
  std::vector<IvReq> st_iv_reqs_;
  std::vector<IvFrameBlock> st_iv_blocks_;
  std::vector<DevJob> st_iv_devjobs_;  // GEMM rows of the blocks
  std::vector<CmvnJob> st_ncmvn_, st_ivcmvn_;  // nnet-input / i-vector CMVN
  CmvnDev ncmvn_{}, ivcmvn_{};
  int st_iv_frames_ = 0, max_iv_frames_ = 0;
  // i-vector extraction (nnet with a per-chunk i-vector input)
  bool use_iv_ = false;
  IvArgs iv_{};
  float* d_ivec_buf_[2] = {nullptr, nullptr};  // [max jobs][ivector dim] per chunk job of a step
  float* d_iv_ll_ = nullptr; // [GEMM rows][num_gauss] UBM log-likelihoods
  std::vector<NnetOpArgs> iv_ops_;  // LDA (normalized -> [x | x*x]), LDA (raw), UBM
  std::vector<int> iv_op_bk_;
  int max_iv_rows_ = 0, max_iv_ents_ = 0;
  std::vector<IvEntry> st_iv_ents_;  // silence-weighted entries of this step
  std::vector<IvBatch> st_iv_batches_;  // statistics batches of this step's requests
  int max_jobs_ = 0, max_dec_frames_ = 0;

  void* DevAlloc(size_t bytes);
  template <class T> T* Upload(const std::vector<T>& v);
};

}  // namespace vamd
