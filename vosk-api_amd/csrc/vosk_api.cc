// C ABI (include/vosk_api.h, include/vosk_amd_engine.h).
//
// Error conventions of the reference (src/vosk_api.cc:30-282): constructors
// return NULL on any exception, accept_waveform returns -1, *_free(NULL) is a
// no-op.  Unlike the reference, the batch entry points are always compiled
// (the GPU path is the only path).
#include <hip/hip_runtime.h>

#include <cmath>
#include <chrono>
#include <cstring>
#include <memory>
#include <sstream>
#include <string>

#include "common.h"
#include "graph_compose.h"
#include "incremental.h"
#include "vosk_impl.h"
#include "../../include/vosk_api.h"
#include "../../include/vosk_amd_engine.h"

using namespace vamd;

namespace {
thread_local std::string g_last_error;
}

#define API_TRY try {
#define API_CATCH(ret)                                   \
  }                                                      \
  catch (const std::exception& e) {                      \
    g_last_error = e.what();                             \
    return ret;                                          \
  }                                                      \
  catch (...) {                                          \
    g_last_error = "unknown exception";                  \
    return ret;                                          \
  }
#define API_CATCH_VOID                                   \
  }                                                      \
  catch (const std::exception& e) {                      \
    g_last_error = e.what();                             \
    VAMD_WARN(e.what());                                 \
  }                                                      \
  catch (...) {                                          \
    g_last_error = "unknown exception";                  \
  }

extern "C" {

VoskModel* vosk_model_new(const char* model_path) {
  API_TRY
  return (VoskModel*)new Model(model_path);
  API_CATCH(nullptr)
}

void vosk_model_free(VoskModel* model) {
  if (!model) return;
  ((Model*)model)->Unref();
}

int vosk_model_find_word(VoskModel* model, const char* word) {
  API_TRY
  return ((Model*)model)->FindWord(word);
  API_CATCH(-1)
}

VoskSpkModel* vosk_spk_model_new(const char* model_path) {  // src/vosk_api.cc:52-59
  API_TRY
  return (VoskSpkModel*)new SpkModel(model_path ? model_path : "");
  API_CATCH(nullptr)
}

void vosk_spk_model_free(VoskSpkModel* model) {
  if (model == nullptr) return;
  ((SpkModel*)model)->Unref();
}

VoskRecognizer* vosk_recognizer_new(VoskModel* model, float sample_rate) {
  API_TRY
  return (VoskRecognizer*)new Recognizer((Model*)model, sample_rate);
  API_CATCH(nullptr)
}

VoskRecognizer* vosk_recognizer_new_spk(VoskModel* model, float sample_rate, VoskSpkModel* spk) {
  API_TRY
  return (VoskRecognizer*)new Recognizer((Model*)model, sample_rate, (SpkModel*)spk);
  API_CATCH(nullptr)
}

VoskRecognizer* vosk_recognizer_new_grm(VoskModel* model, float sample_rate, const char* grammar) {
  API_TRY
  return (VoskRecognizer*)new Recognizer((Model*)model, sample_rate, grammar ? grammar : "");
  API_CATCH(nullptr)
}

void vosk_recognizer_set_spk_model(VoskRecognizer* recognizer, VoskSpkModel* spk_model) {
  if (recognizer == nullptr || spk_model == nullptr) return;
  API_TRY
  ((Recognizer*)recognizer)->SetSpkModel((SpkModel*)spk_model);
  API_CATCH_VOID
}

int vamd_spk_extract(VoskSpkModel* spk, const float* samples, long long n, int rate, int first_frame,
                     const signed char* keep, int nkeep, float* out, int cap, int* num_frames) {
  API_TRY
  std::vector<char> k(keep, keep + nkeep);
  std::vector<float> xv;
  SpkExtractor* ex = ((SpkModel*)spk)->Extractor();
  if (!ex->Extract(samples, n, rate, first_frame, k, &xv, num_frames)) return 0;
  if ((int)xv.size() > cap) VAMD_ERR("output capacity");
  std::copy(xv.begin(), xv.end(), out);
  return (int)xv.size();
  API_CATCH(-1)
}

int vamd_spk_extract_batch(VoskSpkModel* spk, int count, const float* const* samples, const long long* n,
                           const int* rate, const int* first_frame, const signed char* const* keep,
                           const int* nkeep, float* out, int cap, int* num_frames, int* status) {
  API_TRY
  if (count < 0) VAMD_ERR("bad request count " << count);
  SpkExtractor* ex = ((SpkModel*)spk)->Extractor();
  if (ex->OutputDim() > cap) VAMD_ERR("output capacity");
  std::vector<std::vector<char>> ks(count);
  std::vector<std::vector<float>> xv(count);
  std::vector<XvecRequest> rq(count);
  std::vector<XvecRequest*> ptr(count);
  for (int i = 0; i < count; i++) {
    ks[i].assign(keep[i], keep[i] + nkeep[i]);
    rq[i].samples = samples[i];
    rq[i].n = n[i];
    rq[i].rate = rate[i];
    rq[i].first_frame = first_frame[i];
    rq[i].keep = &ks[i];
    rq[i].xvec = &xv[i];
    ptr[i] = &rq[i];
  }
  ex->ExtractBatch(ptr);
  for (int i = 0; i < count; i++) {
    num_frames[i] = rq[i].num_frames;
    status[i] = rq[i].ok ? (int)xv[i].size() : 0;
    if (rq[i].ok) std::copy(xv[i].begin(), xv[i].end(), out + (size_t)i * cap);
  }
  return count;
  API_CATCH(-1)
}

int vamd_spk_stats(VoskSpkModel* spk, long long* batches, long long* utterances, double* layer_flops,
                   double* layer_ms) {
  API_TRY
  SpkExtractor* ex = ((SpkModel*)spk)->Extractor();
  *batches = ex->Batches();
  *utterances = ex->Utterances();
  if (layer_flops) *layer_flops = ex->LayerFlops();
  if (layer_ms) *layer_ms = ex->LayerMs();
  return 0;
  API_CATCH(-1)
}

void vosk_recognizer_set_max_alternatives(VoskRecognizer* r, int n) {
  if (r) ((Recognizer*)r)->SetMaxAlternatives(n);
}
void vosk_recognizer_set_words(VoskRecognizer* r, int words) {
  if (r) ((Recognizer*)r)->SetWords(words != 0);
}
void vosk_recognizer_set_partial_words(VoskRecognizer* r, int pw) {
  if (r) ((Recognizer*)r)->SetPartialWords(pw != 0);
}
void vosk_recognizer_set_nlsml(VoskRecognizer* r, int nlsml) {
  if (r) ((Recognizer*)r)->SetNLSML(nlsml != 0);
}

int vosk_recognizer_accept_waveform(VoskRecognizer* r, const char* data, int length) {
  API_TRY
  return ((Recognizer*)r)->AcceptWaveform(data, length) ? 1 : 0;
  API_CATCH(-1)
}

int vosk_recognizer_accept_waveform_s(VoskRecognizer* r, const short* data, int length) {
  API_TRY
  return ((Recognizer*)r)->AcceptWaveform(data, length) ? 1 : 0;
  API_CATCH(-1)
}

int vosk_recognizer_accept_waveform_f(VoskRecognizer* r, const float* data, int length) {
  API_TRY
  return ((Recognizer*)r)->AcceptWaveform(data, length) ? 1 : 0;
  API_CATCH(-1)
}

const char* vosk_recognizer_result(VoskRecognizer* r) { return ((Recognizer*)r)->Result(); }
const char* vosk_recognizer_partial_result(VoskRecognizer* r) {
  return ((Recognizer*)r)->PartialResult();
}
const char* vosk_recognizer_final_result(VoskRecognizer* r) { return ((Recognizer*)r)->FinalResult(); }
void vosk_recognizer_reset(VoskRecognizer* r) { ((Recognizer*)r)->Reset(); }
void vosk_recognizer_free(VoskRecognizer* r) { delete (Recognizer*)r; }

void vosk_set_log_level(int log_level) { SetLogLevel(log_level); }

void vosk_gpu_init() {
  API_TRY
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) VAMD_ERR("no HIP device");
  const char* lr = getenv("LOCAL_RANK");
  (void)hipSetDevice(lr ? atoi(lr) % n : 0);
  API_CATCH_VOID
}

void vosk_gpu_thread_init() {
  const char* lr = getenv("LOCAL_RANK");
  int n = 0;
  if (hipGetDeviceCount(&n) == hipSuccess && n > 0) (void)hipSetDevice(lr ? atoi(lr) % n : 0);
}

VoskBatchModel* vosk_batch_model_new() {
  API_TRY
  const char* dir = getenv("VOSK_BATCH_MODEL_DIR");
  return (VoskBatchModel*)new BatchModel(dir && *dir ? dir : "model");
  API_CATCH(nullptr)
}

void vosk_batch_model_free(VoskBatchModel* model) {
  if (model) ((BatchModel*)model)->Unref();
}

void vosk_batch_model_wait(VoskBatchModel* model) {
  API_TRY
  ((BatchModel*)model)->WaitForCompletion();
  API_CATCH_VOID
}

VoskBatchRecognizer* vosk_batch_recognizer_new(VoskBatchModel* model, float sample_rate) {
  API_TRY
  return (VoskBatchRecognizer*)new BatchRecognizer((BatchModel*)model, sample_rate);
  API_CATCH(nullptr)
}

void vosk_batch_recognizer_free(VoskBatchRecognizer* r) { delete (BatchRecognizer*)r; }

void vosk_batch_recognizer_accept_waveform(VoskBatchRecognizer* r, const char* data, int length) {
  API_TRY
  ((BatchRecognizer*)r)->AcceptWaveform(data, length);
  API_CATCH_VOID
}

void vosk_batch_recognizer_set_nlsml(VoskBatchRecognizer* r, int nlsml) {
  if (r) ((BatchRecognizer*)r)->SetNLSML(nlsml != 0);
}

void vosk_batch_recognizer_finish_stream(VoskBatchRecognizer* r) {
  API_TRY
  ((BatchRecognizer*)r)->FinishStream();
  API_CATCH_VOID
}

const char* vosk_batch_recognizer_front_result(VoskBatchRecognizer* r) {
  return ((BatchRecognizer*)r)->FrontResult();
}

void vosk_batch_recognizer_pop(VoskBatchRecognizer* r) { ((BatchRecognizer*)r)->Pop(); }

int vosk_batch_recognizer_get_pending_chunks(VoskBatchRecognizer* r) {
  return ((BatchRecognizer*)r)->GetNumPendingChunks();
}

// ---------------------------------------------------------------------------
// diagnostic engine ABI
// ---------------------------------------------------------------------------
struct VamdEngine {
  std::shared_ptr<ModelData> md;
  std::unique_ptr<Engine> eng;
  std::string desc;
  RawLattice lat;  // last lattice read by vamd_stream_lattice
};

const char* vamd_last_error(void) { return g_last_error.c_str(); }

int vamd_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

VamdEngine* vamd_engine_new(const char* model_dir, int fpc, int max_streams, int flags) {
  API_TRY
  auto e = std::make_unique<VamdEngine>();
  e->md = std::make_shared<ModelData>();
  e->md->Load(model_dir);
  EngineConfig cfg;
  cfg.frames_per_chunk = fpc > 0 ? fpc : e->md->dcb.frames_per_chunk;
  cfg.max_slots = max_streams > 0 ? max_streams : 8;
  cfg.collect_stats = (flags & 1) != 0;
  cfg.collect_llh = (flags & 2) != 0;
  cfg.time_kernels = (flags & 4) != 0;
  cfg.pipeline = (flags & 8) != 0;
  cfg.lattice = (flags & 16) != 0;
  cfg.kaldi_order = (flags & 32) == 0;
  const char* d = getenv("VOSK_AMD_DEVICE");
  cfg.device = d ? atoi(d) : 0;
  const char* at = getenv("VOSK_AMD_ARENA_TOKENS");
  if (at) cfg.arena_tokens = atoll(at);
  e->eng.reset(new Engine(e->md, cfg));
  e->desc = e->eng->plan().Describe();
  return e.release();
  API_CATCH(nullptr)
}

int vamd_engine_flush(VamdEngine* e) {
  API_TRY
  e->eng->Flush();
  return 0;
  API_CATCH(-1)
}

void vamd_engine_free(VamdEngine* e) { delete e; }

const char* vamd_engine_describe(VamdEngine* e) { return e->desc.c_str(); }

const char* vamd_plan_describe(const char* model_dir, int fpc) {
  static thread_local std::string out;
  API_TRY
  ModelData md;
  md.Load(model_dir);
  NnetPlan p = BuildNnetPlan(md.nnet, fpc > 0 ? fpc : md.dcb.frames_per_chunk,
                             md.dcb.frame_subsampling_factor, md.dcb.acoustic_scale);
  std::ostringstream os;
  os << p.Describe() << "graph states=" << md.graph.NumStates() << " arcs=" << md.graph.NumArcs()
     << " words=" << md.words.id2sym.size() << "\n";
  out = os.str();
  return out.c_str();
  API_CATCH(nullptr)
}

void* vamd_graph_new(const char* model_dir, const char* grammar) {
  API_TRY
  auto md = std::make_unique<ModelData>();
  md->Load(model_dir);
  if (grammar) {
    if (!md->lookahead_hcl) VAMD_ERR("Runtime graphs are not supported by this model");
    HostFst g, composed;
    EstimateGrammarLm(ParseGrammarJson(grammar, md->words), 2, 0.5f, &g);
    ComposeLookahead(*md->lookahead_hcl, g, md->disambig, &composed);
    md->graph = Graph();
    ToGraph(composed, &md->graph, "grammar graph");
  }
  return (void*)new Graph(std::move(md->graph));
  API_CATCH(nullptr)
}

int vamd_graph_dims(void* graph, int* start, long long* num_arcs) {
  const Graph* g = (const Graph*)graph;
  *start = g->start;
  *num_arcs = (long long)g->NumArcs();
  return g->NumStates();
}

int vamd_graph_copy(void* graph, float* final_cost, long long* arc_begin, int* ilabel, int* olabel,
                    float* weight, int* nextstate) {
  const Graph* g = (const Graph*)graph;
  std::copy(g->final_cost.begin(), g->final_cost.end(), final_cost);
  std::copy(g->arc_begin.begin(), g->arc_begin.end(), arc_begin);
  std::copy(g->ilabel.begin(), g->ilabel.end(), ilabel);
  std::copy(g->olabel.begin(), g->olabel.end(), olabel);
  std::copy(g->weight.begin(), g->weight.end(), weight);
  std::copy(g->nextstate.begin(), g->nextstate.end(), nextstate);
  return g->NumStates();
}

// OpenFST lazy numbering CSR of a composed graph: returns lazy_ids (0: none);
// row [S+1] and next [row[S]] filled when non-NULL
int vamd_graph_lazy(void* graph, long long* row, int* next) {
  const Graph* g = (const Graph*)graph;
  if (g->lazy_ids == 0) return 0;
  if (row) std::copy(g->lazy_row.begin(), g->lazy_row.end(), row);
  if (next) std::copy(g->lazy_next.begin(), g->lazy_next.end(), next);
  return g->lazy_ids;
}

void vamd_graph_free(void* graph) { delete (Graph*)graph; }

int vamd_silence_weighting_run(int ncalls, const int* num_frames_ready, const int* first_decoder_frame,
                               const int* trace_off, const int* tids, const int* toks,
                               const unsigned char* tid_is_silence, int num_tids, float silence_weight,
                               int fss, int* out_off, int* out_frame, float* out_w, int cap) {
  API_TRY
  SilenceWeighting sw(silence_weight, fss);
  auto is_sil = [&](int t) { return t >= 0 && t < num_tids && tid_is_silence[t] != 0; };
  int n = 0;
  out_off[0] = 0;
  std::vector<std::pair<int, float>> d;
  for (int c = 0; c < ncalls; c++) {
    std::vector<int> ti(tids + trace_off[c], tids + trace_off[c + 1]);
    std::vector<int> to(toks + trace_off[c], toks + trace_off[c + 1]);
    sw.ComputeCurrentTraceback(ti, to);
    sw.GetDeltaWeights(num_frames_ready[c], first_decoder_frame[c], is_sil, &d);
    for (auto& x : d) {
      if (n >= cap) VAMD_ERR("output capacity");
      out_frame[n] = x.first;
      out_w[n] = x.second;
      n++;
    }
    out_off[c + 1] = n;
  }
  return n;
  API_CATCH(-1)
}

static std::shared_ptr<RescoreLm> g_host_rescore;  // vamd_lattice_set_rescore (tests)

int vamd_lattice_set_rescore(const char* g_fst, const char* g_carpa) {
  API_TRY
  if (!g_fst || !g_carpa) {
    g_host_rescore.reset();
    return 0;
  }
  auto r = std::make_shared<RescoreLm>();
  r->Load(g_fst, g_carpa);
  g_host_rescore = r;
  return 0;
  API_CATCH(-1)
}

static std::vector<int> g_host_tid2phone;  // vamd_lattice_set_phones (tests)
static std::vector<char> g_host_tid_first;
static long long g_host_det_max_mem = LatticeOptions().det_max_mem;  // vamd_lattice_set_det_max_mem

int vamd_lattice_set_det_max_mem(long long bytes) {
  API_TRY
  g_host_det_max_mem = bytes;
  return 0;
  API_CATCH(-1)
}

int vamd_lattice_set_phones(const int* tid2phone, const signed char* tid_first, int ntids) {
  API_TRY
  if (ntids > 0 && (!tid2phone || !tid_first)) VAMD_ERR("null transition-id tables");
  g_host_tid2phone.assign(tid2phone, tid2phone + std::max(ntids, 0));
  g_host_tid_first.assign(tid_first, tid_first + std::max(ntids, 0));
  return 0;
  API_CATCH(-1)
}

// host-only: the KaldiRecognizer's incremental lattice (incremental.h) over
// per-frame decoder records, driven by a script of events

const char* vamd_incremental_json(int nframes, const int* frame_begin, const int* tok_state, const float* tok_cost,
                                  const float* cost_offset, int nlink, const int* link_frame, const int* link_src,
                                  const int* link_dst, const int* link_arc, const float* link_ac, int narcs,
                                  const int* arc_ilabel, const int* arc_olabel, const float* arc_weight,
                                  int nstates, const float* final_cost, int start_state, float lattice_beam,
                                  int prune_interval, float prune_scale, int max_delay, int min_chunk, int nev,
                                  const int* ev_type, const int* ev_arg) {
  static thread_local std::string out;
  API_TRY
  for (double& x : vamd::vamd_inc_prof) x = 0;
  Graph g;
  g.ilabel.assign(arc_ilabel, arc_ilabel + narcs);
  g.olabel.assign(arc_olabel, arc_olabel + narcs);
  g.weight.assign(arc_weight, arc_weight + narcs);
  g.final_cost.assign(final_cost, final_cost + nstates);
  g.start = start_state;
  IncrementalOptions o;
  o.lattice_beam = lattice_beam;
  o.prune_interval = prune_interval;
  o.prune_scale = prune_scale;
  o.determinize_max_delay = max_delay;
  o.determinize_min_chunk_size = min_chunk;
  o.det_max_mem = g_host_det_max_mem;
  IncrementalLattice inc;
  inc.Init(&g, &g_host_tid2phone, &g_host_tid_first, o);
  // links per frame (link_frame ascending)
  std::vector<std::vector<IncFrameIn::Link>> fl(std::max(nframes, 0));
  for (int i = 0; i < nlink; i++) {
    if (link_frame[i] < 0 || link_frame[i] >= nframes) VAMD_ERR("link frame out of range");
    fl[link_frame[i]].push_back(IncFrameIn::Link{link_src[i], link_dst[i], link_arc[i], link_ac[i],
                                                 arc_ilabel[link_arc[i]] != 0});
  }
  auto add = [&](int k) {
    IncFrameIn f;
    f.state = tok_state + frame_begin[k];
    f.cost = tok_cost + frame_begin[k];
    f.ntok = frame_begin[k + 1] - frame_begin[k];
    f.cost_offset = cost_offset[k];
    f.links = fl[k].data();
    f.nlinks = (int)fl[k].size();
    inc.AddFrame(f);
  };
  std::ostringstream os;
  os.precision(9);
  os << "[";
  bool firstq = true;
  const auto t_start = std::chrono::steady_clock::now();
  for (int e = 0; e < nev; e++) {
    if (ev_type[e] == 0) {  // frames up to ev_arg decoded, then the AdvanceDecoding end
      if (ev_arg[e] >= nframes) VAMD_ERR("event past the records");
      while (inc.NumFramesDecoded() < ev_arg[e]) add(inc.NumFramesDecoded() + 1);
      inc.AdvanceEnd();
      continue;
    }
    WordLattice wl;
    bool ok;
    if (ev_type[e] == 1) {
      ok = inc.GetLattice(inc.NumFramesInLattice(), false, &wl);
    } else {
      inc.FinalizeDecoding();
      ok = inc.GetLattice(inc.NumFramesDecoded(), true, &wl);
    }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    os << (firstq ? "" : ", ") << "{\"ms\": " << ms << ", \"prof\": [" << vamd::vamd_inc_prof[0] << ", " << vamd::vamd_inc_prof[1]
       << ", " << vamd::vamd_inc_prof[2] << ", " << vamd::vamd_inc_prof[3] << ", " << vamd::vamd_inc_prof[4] << "], \"nfl\": " << inc.NumFramesInLattice() << ", \"ok\": " << (ok ? 1 : 0)
       << ", \"chunks\": " << inc.chunks() << ", \"arcs\": [";
    firstq = false;
    for (int s = 0; s < wl.NumStates(); s++) {
      os << (s ? ", " : "") << "[";
      for (size_t i = 0; i < wl.arcs[s].size(); i++) {
        const auto& a = wl.arcs[s][i];
        os << (i ? ", " : "") << "[" << a.word << ", " << a.next << ", " << a.graph << ", " << a.acoustic << ", [";
        for (size_t j = 0; j < a.tids.size(); j++) os << (j ? ", " : "") << a.tids[j];
        os << "]]";
      }
      os << "]";
    }
    os << "], \"finals\": [";
    for (int s = 0; s < wl.NumStates(); s++) {
      os << (s ? ", " : "");
      if (wl.final_graph[s] == INFINITY) {
        os << "null";
        continue;
      }
      os << "[" << wl.final_graph[s] << ", " << wl.final_acoustic[s] << ", [";
      for (size_t j = 0; j < wl.final_tids[s].size(); j++) os << (j ? ", " : "") << wl.final_tids[s][j];
      os << "]]";
    }
    os << "]}";
  }
  os << "]";
  out = os.str();
  return out.c_str();
  API_CATCH(nullptr)
}

float vamd_carpa_logprob(const char* g_carpa, int word, const int* hist, int nhist) {
  static std::string loaded;
  static ConstArpaLm lm;
  API_TRY
  if (loaded != g_carpa) {
    lm.Read(g_carpa);
    loaded = g_carpa;
  }
  return lm.NgramLogprob(word, std::vector<int>(hist, hist + nhist));
  API_CATCH(NAN)
}

const char* vamd_lattice_words_json(int num_frames, const int* frame_begin, const int* tok_state,
                                    const float* tok_cost, const int* link_src, const int* link_dst,
                                    const int* link_arc, const float* link_graph, const float* link_ac,
                                    int nlink, const float* final_cost, int nfinal, const int* arc_ilabel,
                                    const int* arc_olabel, int narcs, float lattice_beam, float graph_scale,
                                    int nbest, const signed char* tid_type, const signed char* tid_final,
                                    const signed char* tid_loop, int ntids) {
  static thread_local std::string out;
  API_TRY
  RawLattice L;
  L.num_frames = num_frames;
  L.frame_begin.assign(frame_begin, frame_begin + num_frames + 2);
  const int ntok = L.frame_begin.back();
  L.tok_state.assign(tok_state, tok_state + ntok);
  L.tok_cost.assign(tok_cost, tok_cost + ntok);
  for (int i = 0; i < nlink; i++)
    L.links.push_back(RawLattice::Link{link_src[i], link_dst[i], link_arc[i], link_graph[i], link_ac[i]});
  L.final_cost.assign(final_cost, final_cost + nfinal);
  Graph g;
  g.ilabel.assign(arc_ilabel, arc_ilabel + narcs);
  g.olabel.assign(arc_olabel, arc_olabel + narcs);
  using clk = std::chrono::steady_clock;
  auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  const auto t0 = clk::now();
  PruneRawLattice(&L, lattice_beam);
  const auto t1 = clk::now();
  std::ostringstream os;
  os.precision(9);
  os << "{\"pruned_tokens\": " << L.tok_state.size() << ", \"pruned_links\": " << L.links.size();
  WordLattice wl;
  LatticeOptions opt;
  opt.lattice_beam = lattice_beam;
  opt.det_max_mem = g_host_det_max_mem;
  const bool ok = g_host_tid2phone.empty()
                      ? DeterminizeToWords(L, g, opt, &wl)
                      : DeterminizePhonePruned(L, g, g_host_tid2phone, g_host_tid_first, opt, &wl);
  const auto t2 = clk::now();
  os << ", \"det_ok\": " << (ok ? 1 : 0) << ", \"det_states\": " << wl.NumStates();
  int det_arcs = 0;
  for (auto& v : wl.arcs) det_arcs += (int)v.size();
  os << ", \"det_arcs\": " << det_arcs;
  if (g_host_rescore) {
    WordLattice r;
    const bool rok = RescoreLattice(wl, *g_host_rescore, opt, &r);
    if (rok) wl = std::move(r);
    int rarcs = 0;
    for (auto& v : wl.arcs) rarcs += (int)v.size();
    os << ", \"rescored\": " << (rok ? 1 : 0) << ", \"rescored_states\": " << wl.NumStates()
       << ", \"rescored_arcs\": " << rarcs;
  }
  if (graph_scale != 1.0f) ScaleGraph(&wl, graph_scale);
  if (ntids > 0) {
    std::vector<char> ty(tid_type, tid_type + ntids), fi(tid_final, tid_final + ntids),
        lo(tid_loop, tid_loop + ntids);
    WordLattice al;
    const bool aok = WordAlignLattice(wl, ty, fi, lo, 1000000, &al);
    int aarcs = 0;
    for (auto& v : al.arcs) aarcs += (int)v.size();
    os << ", \"align_ok\": " << (aok ? 1 : 0) << ", \"align_states\": " << al.NumStates()
       << ", \"align_arcs\": " << aarcs;
    wl = std::move(al);
  }
  const auto t3 = clk::now();
  MbrResult r;
  MinimumBayesRisk(wl, &r);
  const auto t4 = clk::now();
  os << ", \"ms\": {\"prune\": " << ms(t0, t1) << ", \"determinize\": " << ms(t1, t2)
     << ", \"scale_align\": " << ms(t2, t3) << ", \"mbr\": " << ms(t3, t4) << "}";
  os << ", \"mbr\": {\"words\": [";
  for (size_t i = 0; i < r.words.size(); i++) os << (i ? ", " : "") << r.words[i];
  os << "], \"conf\": [";
  for (size_t i = 0; i < r.conf.size(); i++) os << (i ? ", " : "") << r.conf[i];
  os << "], \"times\": [";
  for (size_t i = 0; i < r.times.size(); i++)
    os << (i ? ", " : "") << "[" << r.times[i].first << ", " << r.times[i].second << "]";
  os << "]}, \"nbest\": [";
  std::vector<NbestPath> nb;
  NbestPaths(wl, nbest, &nb);
  for (size_t k = 0; k < nb.size(); k++) {
    os << (k ? ", " : "") << "{\"words\": [";
    for (size_t i = 0; i < nb[k].words.size(); i++) os << (i ? ", " : "") << nb[k].words[i];
    os << "], \"spans\": [";
    for (size_t i = 0; i < nb[k].spans.size(); i++)
      os << (i ? ", " : "") << "[" << nb[k].spans[i].first << ", " << nb[k].spans[i].second << "]";
    os << "], \"graph\": " << nb[k].graph << ", \"acoustic\": " << nb[k].acoustic << "}";
  }
  os << "]}";
  out = os.str();
  return out.c_str();
  API_CATCH(nullptr)
}

int vamd_plan_info(const char* model_dir, int fpc, int* o, double* flops) {
  API_TRY
  ModelData md;
  md.Load(model_dir);
  NnetPlan p = BuildNnetPlan(md.nnet, fpc > 0 ? fpc : md.dcb.frames_per_chunk,
                             md.dcb.frame_subsampling_factor, md.dcb.acoustic_scale);
  o[0] = p.fpc; o[1] = p.fss; o[2] = p.left_context; o[3] = p.right_context;
  o[4] = p.priming_chunks; o[5] = p.out_dim; o[6] = (int)p.ops.size(); o[7] = (int)p.nodes.size();
  if (flops) *flops = p.flops_per_chunk;
  return 0;
  API_CATCH(-1)
}

const char* vamd_json_words(const char* list_key, const char* text_key, int n,
                            const char* const* words, const double* start, const double* end,
                            const double* conf) {
  static thread_local std::string out;
  API_TRY
  Json obj;
  std::string text;
  for (int i = 0; i < n; i++) {
    Json w;
    w["word"] = Json::Str(words[i]);
    w["start"] = Json::Float(start[i]);
    w["end"] = Json::Float(end[i]);
    if (conf) w["conf"] = Json::Float(conf[i]);
    obj[list_key].Append(w);
    if (i) text += " ";
    text += words[i];
  }
  obj[text_key] = Json::Str(text);
  out = obj.Dump();
  return out.c_str();
  API_CATCH(nullptr)
}

int vamd_engine_info(VamdEngine* e, int* o, double* flops) {
  API_TRY
  const NnetPlan& p = e->eng->plan();
  o[0] = p.fpc; o[1] = p.fss; o[2] = p.left_context; o[3] = p.right_context;
  o[4] = p.priming_chunks; o[5] = p.out_dim; o[6] = (int)p.ops.size(); o[7] = 0;
  if (flops) *flops = p.flops_per_chunk;
  return 0;
  API_CATCH(-1)
}

int vamd_stream_new(VamdEngine* e) {
  API_TRY
  int s = e->eng->AllocSlot();
  e->eng->ResetPipeline(s);
  return s;
  API_CATCH(-1)
}

int vamd_stream_set_rate(VamdEngine* e, int s, int rate) {
  API_TRY
  e->eng->SetSampleRate(s, rate);
  return 0;
  API_CATCH(-1)
}

int vamd_stream_free(VamdEngine* e, int s) {
  API_TRY
  e->eng->FreeSlot(s);
  return 0;
  API_CATCH(-1)
}

int vamd_stream_reset(VamdEngine* e, int s, int pipeline) {
  API_TRY
  if (pipeline) e->eng->ResetPipeline(s);
  else e->eng->ResetDecoder(s);
  return 0;
  API_CATCH(-1)
}

int vamd_stream_accept(VamdEngine* e, int s, const float* x, int n, int finished) {
  API_TRY
  if (n > 0) e->eng->AcceptSamples(s, x, n);
  if (finished) e->eng->InputFinished(s);
  return 0;
  API_CATCH(-1)
}

int vamd_engine_advance(VamdEngine* e, const int* streams, int n) {
  API_TRY
  e->eng->Advance(std::vector<int>(streams, streams + n));
  return 0;
  API_CATCH(-1)
}

int vamd_stream_frames_decoded(VamdEngine* e, int s) {
  API_TRY
  return e->eng->NumFramesDecoded(s);
  API_CATCH(-1)
}

int vamd_stream_error(VamdEngine* e, int s) {
  API_TRY
  return e->eng->DecoderError(s);
  API_CATCH(-1)
}

int vamd_stream_decoder_state(VamdEngine* e, int s, long long* out8) {
  API_TRY
  e->eng->DecoderState(s, out8);
  return 0;
  API_CATCH(-1)
}

int vamd_stream_features(VamdEngine* e, int s, int first, int n, float* out) {
  API_TRY
  std::vector<float> v;
  e->eng->DebugFeatures(s, first, n, &v);
  memcpy(out, v.data(), sizeof(float) * v.size());
  return n;
  API_CATCH(-1)
}

long long vamd_stream_llh(VamdEngine* e, int s, float* out, long long cap) {
  API_TRY
  const std::vector<float>& v = e->eng->DecodedLlh(s);
  long long n = std::min<long long>(cap, (long long)v.size());
  if (out && n > 0) memcpy(out, v.data(), sizeof(float) * n);
  return (long long)v.size();
  API_CATCH(-1)
}

long long vamd_stream_ivectors(VamdEngine* e, int s, float* out, long long cap) {
  API_TRY
  const std::vector<float>& v = e->eng->ChunkIvectors(s);
  long long n = std::min<long long>(cap, (long long)v.size());
  if (out && n > 0) memcpy(out, v.data(), sizeof(float) * n);
  return (long long)v.size();
  API_CATCH(-1)
}

int vamd_stream_update_silence_weights(VamdEngine* e, int s, int first_decoder_frame) {
  API_TRY
  e->eng->UpdateSilenceWeights(s, first_decoder_frame);
  return e->eng->SilenceWeightingActive() ? 1 : 0;
  API_CATCH(-1)
}

int vamd_stream_lattice(VamdEngine* e, int s, int use_final, int* sizes4, int* frame_begin,
                        int* tok_state, float* tok_cost, int* link_src, int* link_dst, int* link_arc,
                        float* link_graph, float* link_ac, float* final_cost) {
  API_TRY
  RawLattice& L = e->lat;
  if (!frame_begin) e->eng->GetRawLattice(s, use_final != 0, &L);
  sizes4[0] = L.num_frames;
  sizes4[1] = (int)L.tok_state.size();
  sizes4[2] = (int)L.links.size();
  sizes4[3] = (int)L.final_cost.size() | (L.overflow ? (1 << 30) : 0);
  if (frame_begin) {
    std::copy(L.frame_begin.begin(), L.frame_begin.end(), frame_begin);
    std::copy(L.tok_state.begin(), L.tok_state.end(), tok_state);
    std::copy(L.tok_cost.begin(), L.tok_cost.end(), tok_cost);
    for (size_t i = 0; i < L.links.size(); i++) {
      link_src[i] = L.links[i].src;
      link_dst[i] = L.links[i].dst;
      link_arc[i] = L.links[i].arc;
      link_graph[i] = L.links[i].graph_cost;
      link_ac[i] = L.links[i].acoustic_cost;
    }
    std::copy(L.final_cost.begin(), L.final_cost.end(), final_cost);
  }
  return 0;
  API_CATCH(-1)
}

int vamd_engine_ivector_dim(VamdEngine* e) {
  API_TRY
  return e->eng->IvectorDim();
  API_CATCH(-1)
}

int vamd_stream_stats(VamdEngine* e, int s, float* out, int cap) {
  API_TRY
  const std::vector<FrameStat>& st = e->eng->LastStats(s);
  int n = std::min<int>(cap, (int)st.size());
  for (int i = 0; i < n; i++) {
    const FrameStat& f = st[i];
    float* o = out + 8 * i;
    o[0] = (float)f.ntok_in; o[1] = (float)f.ntok_out; o[2] = (float)f.arcs_emit;
    o[3] = (float)f.arcs_eps; o[4] = f.best; o[5] = f.cutoff; o[6] = f.next_cutoff;
    o[7] = f.adaptive_beam;
  }
  return (int)st.size();
  API_CATCH(-1)
}

int vamd_stream_decode_llh(VamdEngine* e, int s, const float* llh, int nframes, int reset) {
  API_TRY
  e->eng->DecodeExternal(s, llh, nframes, reset != 0);
  return 0;
  API_CATCH(-1)
}

int vamd_stream_best_path(VamdEngine* e, int s, int use_final, int* arcs, int cap, double* cost,
                          float* frel) {
  API_TRY
  std::vector<PathResult> pr;
  e->eng->BestPaths({s}, use_final != 0, &pr);
  const PathResult& p = pr[0];
  for (int i = 0; i < (int)p.arcs.size() && i < cap; i++) arcs[i] = p.arcs[i];
  if (cost) *cost = p.cost;
  if (frel) *frel = p.final_relative_cost;
  return (int)p.arcs.size();
  API_CATCH(-1)
}

int vamd_stream_segment_best_path(VamdEngine* e, int s, int* arcs, int cap) {
  API_TRY
  SegmentLattice sl;
  e->eng->CopySegmentLattice(s, &sl, true);
  const std::vector<int> p = SegmentBestPath(e->eng->model().graph, sl);
  for (int i = 0; i < (int)p.size() && i < cap; i++) arcs[i] = p[i];
  return (int)p.size();
  API_CATCH(-1)
}

int vamd_stream_preload(VamdEngine* e, int s, const float* x, long long n, int finished) {
  API_TRY
  e->eng->PreloadSamples(s, x, n, finished != 0);
  return 0;
  API_CATCH(-1)
}

int vamd_engine_step(VamdEngine* e, const int* streams, int n) {
  API_TRY
  return e->eng->Step(std::vector<int>(streams, streams + n)) ? 1 : 0;
  API_CATCH(-1)
}

int vamd_engine_set_step_samples(VamdEngine* e, int n) {
  API_TRY
  if (n <= 0) VAMD_ERR("step samples must be positive");
  e->eng->SetStepSamples(n);
  return 0;
  API_CATCH(-1)
}

int vamd_engine_stage_times(VamdEngine* e, double* ms4, long long* launches4, int reset) {
  API_TRY
  const StageTimes& t = e->eng->stage_times();
  for (int i = 0; i < 4; i++) {
    if (ms4) ms4[i] = t.ms[i];
    if (launches4) launches4[i] = t.launches[i];
  }
  if (reset) e->eng->ResetStageTimes();
  return 0;
  API_CATCH(-1)
}

int vamd_engine_decoder_totals(VamdEngine* e, long long* o6) {
  API_TRY
  const StageTimes& t = e->eng->stage_times();
  for (int i = 0; i < 6; i++) o6[i] = t.dec[i];
  return 0;
  API_CATCH(-1)
}

int vamd_engine_decoder_phases(VamdEngine* e, long long* o8) {
  API_TRY
  long long all[kDecProf];
  e->eng->DecoderPhaseClocks(all);
  for (int i = 0; i < 8; i++) o8[i] = all[i];  // the base ABI's eight slots
  return 0;
  API_CATCH(-1)
}

int vamd_engine_decoder_phases_n(VamdEngine* e, long long* out, int cap) {
  API_TRY
  long long all[kDecProf];
  e->eng->DecoderPhaseClocks(all);
  const int n = std::min(cap, (int)kDecProf);
  for (int i = 0; i < n; i++) out[i] = all[i];
  return kDecProf;
  API_CATCH(-1)
}

int vamd_engine_decoder_phases_per_stream(VamdEngine* e, long long* o) {
  API_TRY
  long long tot[kDecProf];
  e->eng->DecoderPhaseClocks(tot, o);
  return 0;
  API_CATCH(-1)
}

int vamd_batch_lanes(VoskBatchModel* m) {
  API_TRY
  return ((BatchModel*)m)->num_lanes();
  API_CATCH(-1)
}

int vamd_batch_lane_stats(VoskBatchModel* m, int lane, int* load3, double* ms4, long long* launches4,
                          long long* dec6, int reset) {
  API_TRY
  BatchModel* bm = (BatchModel*)m;
  const auto loads = bm->LaneLoads();
  if (lane < 0 || lane >= (int)loads.size()) VAMD_ERR("bad lane " << lane);
  if (load3)
    for (int i = 0; i < 3; i++) load3[i] = loads[lane][i];
  Engine* e = bm->lane_engine(lane);
  const StageTimes& t = e->stage_times();
  for (int i = 0; i < 4; i++) {
    if (ms4) ms4[i] = t.ms[i];
    if (launches4) launches4[i] = t.launches[i];
  }
  if (dec6)
    for (int i = 0; i < 6; i++) dec6[i] = t.dec[i];
  if (reset) e->ResetStageTimes();
  return 0;
  API_CATCH(-1)
}

int vamd_batch_lane_memory(VoskBatchModel* m, int lane, long long* out5) {
  API_TRY
  BatchModel* bm = (BatchModel*)m;
  if (lane < 0 || lane >= bm->num_lanes()) VAMD_ERR("bad lane " << lane);
  bm->lane_engine(lane)->MemoryStats(out5);
  return 0;
  API_CATCH(-1)
}

int vamd_batch_lane_kaldi_order(VoskBatchModel* m, int lane) {
  API_TRY
  BatchModel* bm = (BatchModel*)m;
  if (lane < 0 || lane >= bm->num_lanes()) VAMD_ERR("bad lane " << lane);
  return bm->lane_engine(lane)->kaldi_order() ? 1 : 0;
  API_CATCH(-1)
}

int vamd_batch_result_profile(VoskBatchModel* m, double* out13) {
  API_TRY
  ((BatchModel*)m)->ResultProfile(out13);
  return 0;
  API_CATCH(-1)
}

int vamd_batch_batching_counters(VoskBatchModel* m, long long* out4) {
  API_TRY
  ((BatchModel*)m)->BatchingCounters(out4);
  return 0;
  API_CATCH(-1)
}

int vamd_feeding_round_incomplete(int n, const long long* pushed, const long long* taken, const int* ended) {
  API_TRY
  if (n < 0) VAMD_ERR("bad stream count");
  std::vector<std::array<long long, 3>> s(n);
  for (int i = 0; i < n; i++) s[i] = {pushed[i], taken[i], ended[i] ? 1LL : 0LL};
  return FeedingRoundIncomplete(s) ? 1 : 0;
  API_CATCH(-1)
}

int vamd_batch_recognizer_lane(VoskBatchRecognizer* r) {
  API_TRY
  return ((BatchRecognizer*)r)->lane();
  API_CATCH(-1)
}

int vamd_admission_replay(int lanes, const int* drain, int n, const int* chunks, int* out) {
  API_TRY
  if (lanes <= 0 || n < 0) VAMD_ERR("bad admission replay arguments");
  // each admission adds the stream's chunks to its lane; between admissions
  // every lane processes drain[lane] pending chunks
  std::vector<std::array<int, 2>> loads(lanes, {0, 0});
  for (int k = 0; k < n; k++) {
    const int l = PickLane(loads);
    out[k] = l;
    loads[l][0] += chunks[k];
    loads[l][1] += 1;
    for (int i = 0; i < lanes; i++) loads[i][0] = std::max(0, loads[i][0] - drain[i]);
  }
  return 0;
  API_CATCH(-1)
}

int vamd_engine_counters(VamdEngine* e, long long* o) {
  API_TRY
  const EngineCounters& c = e->eng->counters();
  o[0] = c.steps; o[1] = c.launches; o[2] = c.frames_mfcc; o[3] = c.chunk_jobs;
  o[4] = c.frames_decoded;
  return 0;
  API_CATCH(-1)
}

}  // extern "C"
