// Vosk object layer (see vosk_impl.h).
#include "vosk_impl.h"

#include <sys/resource.h>
#include <sys/syscall.h>
#include <unistd.h>
#include "graph_compose.h"

#include <sched.h>

#include <algorithm>
#include <limits>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sstream>

#include "common.h"

namespace vamd {

static int EnvInt(const char* name, int def) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : def;
}

static int DeviceFromEnv() {
  // one process per GPU: LOCAL_RANK (torchrun) or VOSK_AMD_DEVICE
  int d = EnvInt("VOSK_AMD_DEVICE", -1);
  if (d >= 0) return d;
  return EnvInt("LOCAL_RANK", 0);
}

// ---------------------------------------------------------------------------
// best-path post-processing
// ---------------------------------------------------------------------------
std::vector<WordSeg> PathWords(const ModelData& m, const std::vector<int>& arcs) {
  // Word spans from the best path: a word ends at the frame its output label
  // is emitted; it starts at its first non-silence frame after the previous
  // word.  (Approximation of WordAlignLattice + MBR times, src/recognizer.cc:
  // 430-482; exact word alignment is the next row, see DESIGN.md.)
  std::vector<WordSeg> out;
  int t = 0, seg_start = -1;
  for (int a : arcs) {
    const int il = m.graph.ilabel[a];
    if (il != 0) {
      const int ph = m.tm.tid2phone[il];
      if (seg_start < 0 && !(ph < (int)m.phone_is_silence.size() && m.phone_is_silence[ph]))
        seg_start = t;
      t++;
    }
    const int ol = m.graph.olabel[a];
    if (ol != 0) {
      int st = seg_start >= 0 ? seg_start : (out.empty() ? 0 : out.back().end);
      out.push_back(WordSeg{ol, st, std::max(st, t)});
      seg_start = -1;
    }
  }
  return out;
}

int TrailingSilenceFrames(const ModelData& m, const std::vector<int>& arcs) {
  // online2/online-endpoint.cc TrailingSilenceLength [K]
  int n = 0;
  for (auto it = arcs.rbegin(); it != arcs.rend(); ++it) {
    const int il = m.graph.ilabel[*it];
    if (il == 0) continue;
    const int ph = m.tm.tid2phone[il];
    if (ph < (int)m.phone_is_silence.size() && m.phone_is_silence[ph]) n++;
    else break;
  }
  return n;
}

bool EndpointRulesFire(const EndpointConfig& c, int frames_decoded, int trailing_sil,
                       float frame_shift_s, float final_relative_cost) {
  const float utt = frames_decoded * frame_shift_s, sil = trailing_sil * frame_shift_s;
  for (int r = 0; r < 5; r++) {
    const EndpointRule& rule = c.rule[r];
    const bool contains_nonsilence = utt > sil;
    if ((contains_nonsilence || !rule.must_contain_nonsilence) &&
        sil >= rule.min_trailing_silence && final_relative_cost <= rule.max_relative_cost &&
        utt >= rule.min_utterance_length) {
      VAMD_LOG_VERBOSE("Endpointing rule " << r + 1 << " activated");
      return true;
    }
  }
  return false;
}

// ---------------------------------------------------------------------------
// Model (src/model.cc:106-128, refcount :343-354)
// ---------------------------------------------------------------------------
Model::Model(const std::string& path) : md_(std::make_shared<ModelData>()) { md_->Load(path); }

int Model::FindWord(const std::string& w) const { return md_->words.Find(w); }

RecognizerGroup::RecognizerGroup(Engine* e) : engine(e), by_slot(e->config().max_slots, nullptr) {
  gc.Resize(e->config().max_slots);
  // coalescing window of the group commit (engine.h SlotGroupCommit)
  gc.SetWindowUs(EnvInt("VOSK_AMD_GROUP_WINDOW_US", 1000));
  gc.SetAdaptive(EnvInt("VOSK_AMD_GROUP_ADAPTIVE", 1) != 0);
}

// Recognizers are spread over VOSK_AMD_STREAM_ENGINES engines of
// VOSK_AMD_MAX_STREAMS (32) slots, the least-loaded first; each engine's
// group commit batches the recognizers that call together, and the engines'
// passes run beside each other on the GPU.  Each engine holds a HIP stream
// and a copy stream, and the runtime hands its GPU_MAX_HW_QUEUES hardware
// queues (4 unless the process sets a number; the Python package asks for 8
// when unset) to streams in turn, so the default spread is queues / 2 (at
// most 4): more engines than that make one engine's pass wait behind
// another's.  Measured (profiles/r06_stream_engines.log,
// r06_conc_queues.log, 20-s streams, 32 threads): 4 queues: one engine 551 x
// RT, two 669, four 463; 8 queues: two 716-720, four 744-810.  More engines
// are created when all are full (VOSK_AMD_MAX_STREAM_ENGINES).
static int StreamEngineSpread() {
  const int queues = std::max(1, EnvInt("GPU_MAX_HW_QUEUES", 4));
  return std::max(1, EnvInt("VOSK_AMD_STREAM_ENGINES", std::max(1, std::min(4, queues / 2))));
}

RecognizerGroup* Model::AllocStreamSlot(int* slot) {
  std::lock_guard<std::mutex> lk(mu_);
  const int spread = StreamEngineSpread();
  RecognizerGroup* best = nullptr;
  int best_use = 0;
  for (auto& g : engines_) {
    const int use = g->engine->SlotsInUse();
    if (use < g->engine->config().max_slots && (!best || use < best_use)) {
      best = g.get();
      best_use = use;
    }
  }
  if (best && (best_use == 0 || (int)engines_.size() >= spread)) {
    *slot = best->engine->TryAllocSlot();
    if (*slot >= 0) return best;
  }
  // each engine holds the decoder state of all its slots (~140 MB per slot
  // with lattices): the number of engines is capped
  const int cap = EnvInt("VOSK_AMD_MAX_STREAM_ENGINES", 32);
  if ((int)engines_.size() >= cap) {
    for (auto& g : engines_) {  // (a full spread: any free slot)
      *slot = g->engine->TryAllocSlot();
      if (*slot >= 0) return g.get();
    }
    VAMD_ERR("all " << engines_.size() << " stream engines of the model are full "
                    "(VOSK_AMD_MAX_STREAM_ENGINES x VOSK_AMD_MAX_STREAMS recognizers)");
  }
  EngineConfig cfg;
  cfg.frames_per_chunk = md_->dcb.frames_per_chunk;
  cfg.max_slots = EnvInt("VOSK_AMD_MAX_STREAMS", 32);
  cfg.device = DeviceFromEnv();
  cfg.max_step_samples = 4096;
  cfg.lattice = true;  // results come from the segment's lattice (MBR)
  cfg.host_lattice = true;  // the incremental lattice reads the records as they come
  // the records stay on the device until the in-kernel pruning compacts
  // them at half full, once the host has read them all (Engine::SetHostRead):
  // 4 M tokens / 8 M links per stream hold ~15 s at the bench model's density
  // (~2 200 tokens, ~3 100 links per frame) before the first compaction, and
  // leave room for the host's replay to lag behind the decoder
  cfg.arena_tokens = EnvInt("VOSK_AMD_REC_ARENA_TOKENS", 1 << 22);
  cfg.lattice_links = EnvInt("VOSK_AMD_REC_LINKS", 1 << 23);
  engines_.emplace_back(new RecognizerGroup(new Engine(md_, cfg)));
  *slot = engines_.back()->engine->AllocSlot();
  return engines_.back().get();
}

void Model::FreeStreamSlot(RecognizerGroup* g, int slot) {
  std::lock_guard<std::mutex> lk(mu_);
  g->by_slot.at(slot) = nullptr;
  g->engine->FreeSlot(slot);
  // an emptied engine past the spread gives its device memory back
  const size_t keep = (size_t)StreamEngineSpread();
  for (size_t i = keep; i < engines_.size(); i++)
    if (engines_[i].get() == g && g->engine->SlotsInUse() == 0) {
      engines_.erase(engines_.begin() + (long)i);
      break;
    }
}

RecognizerGroup* Model::GrammarEngine(const std::string& grammar) {
  std::lock_guard<std::mutex> lk(mu_);
  if (!md_->lookahead_hcl) {
    VAMD_WARN("Runtime graphs are not supported by this model");
    return nullptr;
  }
  auto it = grammar_engines_.find(grammar);
  if (it != grammar_engines_.end()) return it->second.get();
  HostFst g, composed;
  EstimateGrammarLm(ParseGrammarJson(grammar, md_->words), 2, 0.5f, &g);
  ComposeLookahead(*md_->lookahead_hcl, g, md_->disambig, &composed);
  auto md = std::make_shared<ModelData>(*md_);
  md->graph = Graph();
  ToGraph(composed, &md->graph, "grammar graph");
  EngineConfig cfg;
  cfg.frames_per_chunk = md->dcb.frames_per_chunk;
  cfg.max_slots = EnvInt("VOSK_AMD_GRAMMAR_STREAMS", 8);
  cfg.device = DeviceFromEnv();
  cfg.max_step_samples = 4096;
  cfg.lattice = true;
  cfg.host_lattice = true;
  cfg.arena_tokens = EnvInt("VOSK_AMD_REC_ARENA_TOKENS", 1 << 22);
  cfg.lattice_links = EnvInt("VOSK_AMD_REC_LINKS", 1 << 23);
  RecognizerGroup* grp = new RecognizerGroup(new Engine(md, cfg));
  grammar_engines_[grammar].reset(grp);
  return grp;
}

void RecognizerGroup::Serve(const std::vector<int>& slots, std::vector<char>* complete) {
  std::vector<Recognizer*> rs;
  for (int s : slots) rs.push_back(by_slot.at(s));
  // pieces of 0.2 s as the reference's AcceptWaveform loop (src/recognizer.cc:305-311):
  // per stream, in order, UpdateSilenceWeights then AdvanceDecoding of each
  // piece.  Streams are independent, so pieces of different streams need not
  // share a round: a round takes, for every stream, its next piece -- first
  // only the streams whose next piece readies no chunk (no decoder work),
  // then all the others together, so the decoder launch is shared by every
  // stream that decodes.  A pass runs one such decoder round: a request whose
  // later piece readies another chunk (a 0.25 s call is a 0.2 s and a 0.05 s
  // piece, and either may complete a chunk) is carried into the next pass,
  // whose decoder round it shares with the requests posted meanwhile, instead
  // of a round of its own.
  std::vector<int> step(rs.size());
  std::vector<size_t> npiece(rs.size()), cur(rs.size(), 0);
  for (size_t i = 0; i < rs.size(); i++) {
    step[i] = (int)(rs[i]->sample_frequency_ * 0.2f);
    const size_t n = rs[i]->req_wave_ ? rs[i]->req_wave_->size() : 0;
    npiece[i] = (n + step[i] - 1) / step[i];
    if (rs[i]->req_final_ && npiece[i] == 0) npiece[i] = 1;  // a FinalResult request: one piece, no samples
    cur[i] = rs[i]->req_piece_;
  }
  // a stream whose own input fails (AcceptSamples) is dropped from the
  // pass with its error kept for its caller; failures of the batched
  // launches themselves reach every caller of the pass
  std::vector<size_t> quiet, busy;
  // development: each pass's rounds on stderr (streams, which ran, ms)
  static const bool trace = EnvInt("VOSK_AMD_GROUP_TRACE", 0) != 0;
  std::ostringstream tr;
  const auto ts0 = std::chrono::steady_clock::now();
  if (trace) tr << "[group] pass " << rs.size() << ":";
  bool decoded = false;
  while (true) {
    quiet.clear();
    busy.clear();
    for (size_t i = 0; i < rs.size(); i++) {
      Recognizer* r = rs[i];
      if (r->req_error_ || cur[i] >= npiece[i]) continue;
      const size_t n = r->req_wave_ ? r->req_wave_->size() : 0;
      const size_t o = cur[i] * step[i];
      const long long add = o < n ? (long long)std::min<size_t>(step[i], n - o) : 0;
      const bool decodes = r->req_final_ || engine->ChunkReadyAfter(r->slot_, add);
      (decodes ? busy : quiet).push_back(i);
    }
    if (quiet.empty() && decoded) break;  // the next pieces decode: the next pass
    const std::vector<size_t>& run = !quiet.empty() ? quiet : busy;
    if (run.empty()) break;
    if (quiet.empty()) decoded = true;
    std::vector<int> sl, first;
    std::vector<Recognizer*> sr;
    for (size_t i : run) {
      Recognizer* r = rs[i];
      const size_t n = r->req_wave_ ? r->req_wave_->size() : 0;
      const size_t o = cur[i] * step[i];
      cur[i]++;
      if (o < n) {
        try {
          engine->AcceptSamples(r->slot_, r->req_wave_->data() + o, (int)std::min<size_t>(step[i], n - o));
        } catch (...) {
          r->req_error_ = std::current_exception();
          continue;
        }
      }
      sl.push_back(r->slot_);
      sr.push_back(r);
      first.push_back(r->frame_offset_ * 3);  // src/recognizer.cc:309, :825
    }
    if (sl.empty()) continue;
    engine->UpdateSilenceWeights(sl, first);
    const auto ta = std::chrono::steady_clock::now();
    engine->Advance(sl);
    if (trace)
      tr << " " << (!quiet.empty() ? "q" : "b") << sl.size() << "/"
         << std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ta).count();
    // each stream's AdvanceDecoding ended here: its incremental lattice runs
    // UpdateLatticeDeterminization at this frame count (replayed lazily)
    for (Recognizer* r : sr) {
      std::lock_guard<std::mutex> lk(r->inc_mu_);
      r->adv_ends_.push_back(engine->NumFramesDecoded(r->slot_));
    }
  }
  // the requests with every piece done are complete; the others are carried
  std::vector<Recognizer*> done;
  complete->assign(rs.size(), 1);
  for (size_t i = 0; i < rs.size(); i++) {
    rs[i]->req_piece_ = cur[i];
    if (!rs[i]->req_error_ && cur[i] < npiece[i]) (*complete)[i] = 0;
    else done.push_back(rs[i]);
  }
  if (trace) {
    tr << " done " << done.size() << " total "
       << std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ts0).count();
    fprintf(stderr, "%s\n", tr.str().c_str());
  }
  rs.swap(done);
  // EndpointDetected (src/recognizer.cc:318) of the AcceptWaveform requests
  std::vector<int> ep;
  std::vector<Recognizer*> er;
  for (Recognizer* r : rs) {
    r->req_endpoint_ = false;
    if (!r->req_error_ && !r->req_final_ && engine->NumFramesDecoded(r->slot_) > 0) {
      ep.push_back(r->slot_);
      er.push_back(r);
    }
  }
  if (ep.empty()) return;
  const ModelData& m = engine->model();
  const float shift = 0.01f * m.dcb.frame_subsampling_factor;
  if (!m.phone_is_silence.empty()) {  // (the engine's per-arc silence classes exist)
    // the endpoint probe: trailing silence and final relative cost from the
    // traceback kernel, without copying the paths (same walk as
    // TrailingSilenceFrames over the best path)
    std::vector<EndpointProbe> pr;
    engine->ProbeEndpoints(ep, &pr);
    for (size_t i = 0; i < ep.size(); i++)
      er[i]->req_endpoint_ = EndpointRulesFire(m.endpoint, engine->NumFramesDecoded(ep[i]), pr[i].trailing_sil,
                                               shift, pr[i].final_relative_cost);
    return;
  }
  std::vector<PathResult> pr;
  engine->BestPaths(ep, false, &pr);
  for (size_t i = 0; i < ep.size(); i++)
    er[i]->req_endpoint_ = EndpointRulesFire(m.endpoint, engine->NumFramesDecoded(ep[i]),
                                             TrailingSilenceFrames(m, pr[i].arcs), shift,
                                             pr[i].final_relative_cost);
}

// ---------------------------------------------------------------------------
// Recognizer (src/recognizer.cc)
// ---------------------------------------------------------------------------
// Input at another rate than the model's is resampled on the GPU (windowed
// sinc, Kaldi LinearResample; the reference's feature pipeline resamples with
// allow_downsample/upsample, src/model.cc:221).
static int InputRate(float sr) {
  const int r = (int)std::lround(sr);
  if (r <= 0 || std::fabs(sr - r) > 1e-3f) VAMD_ERR("unsupported sample rate " << sr);
  return r;
}

Recognizer::Recognizer(Model* model, float sr) : Recognizer(model, sr, (const char*)nullptr) {}

Recognizer::Recognizer(Model* model, float sr, const char* grammar)
    : model_(model), sample_frequency_(sr) {
  const int rate = InputRate(sr);
  group_ = grammar ? model->GrammarEngine(grammar) : nullptr;
  grammar_group_ = group_ != nullptr;
  if (group_) slot_ = group_->engine->AllocSlot();
  else group_ = model->AllocStreamSlot(&slot_);
  engine_ = group_->engine.get();
  group_->by_slot.at(slot_) = this;
  try {
    engine_->SetSampleRate(slot_, rate);
  } catch (...) {
    if (grammar_group_) {
      group_->by_slot.at(slot_) = nullptr;
      engine_->FreeSlot(slot_);
    } else {
      model_->FreeStreamSlot(group_, slot_);
    }
    throw;
  }
  model_->Ref();
}

Recognizer::Recognizer(Model* model, float sr, SpkModel* spk) : Recognizer(model, sr, (const char*)nullptr) {
  if (spk) {
    spk_ = spk;
    spk_->Ref();
  }
}

void Recognizer::SetSpkModel(SpkModel* spk) {
  if (state_ == RECOGNIZER_RUNNING) {
    VAMD_WARN("Can't add speaker model to already running recognizer");
    return;
  }
  spk->Ref();
  if (spk_) spk_->Unref();
  spk_ = spk;
  spk_samples_.clear();
}

Recognizer::~Recognizer() {
  WaitLattice();
  if (grammar_group_) {
    group_->by_slot.at(slot_) = nullptr;
    engine_->FreeSlot(slot_);
  } else {
    model_->FreeStreamSlot(group_, slot_);
  }
  if (spk_) spk_->Unref();
  model_->Unref();
}

SpkModel::SpkModel(const std::string& dir) : md_(std::make_shared<SpkModelData>()) {
  md_->Load(dir);
}

SpkExtractor* SpkModel::Extractor() {
  std::lock_guard<std::mutex> lk(mu_);
  if (!ex_) ex_.reset(new SpkExtractor(md_, DeviceFromEnv()));
  return ex_.get();
}

bool Recognizer::GetSpkVector(std::vector<float>* xvec, int* num_frames) {
  const ModelData& m = engine_->model();
  *num_frames = 0;
  // OnlineSilenceWeighting::Active() with the reference's configuration
  // (silence weight 1e-3, the endpoint silence phones; src/model.cc:230-231)
  std::vector<char> keep;
  if (!m.endpoint.silence_phones.empty() && engine_->NumFramesDecoded(slot_) > 0) {
    std::vector<PathResult> pr;
    engine_->BestPaths({slot_}, true, &pr);
    for (int a : pr[0].arcs) {
      const int il = m.graph.ilabel[a];
      if (il == 0) continue;
      const int ph = m.tm.tid2phone[il];
      keep.push_back(ph < (int)m.phone_is_silence.size() && m.phone_is_silence[ph] ? 0 : 1);
    }
  }
  return spk_->Extractor()->Extract(spk_samples_.data(), (long long)spk_samples_.size(),
                                    (int)std::lround(sample_frequency_), frame_offset_ * 3, keep,
                                    xvec, num_frames);
}

void Recognizer::CleanUp() {  // src/recognizer.cc:188-224
  frame_offset_ += engine_->NumFramesDecoded(slot_);
  ResetLattice();  // a new decoder (InitDecoding)
  if (state_ == RECOGNIZER_FINALIZED || frame_offset_ > 20000) {
    samples_round_start_ += samples_processed_;
    samples_processed_ = 0;
    frame_offset_ = 0;
    engine_->ResetPipeline(slot_);
    spk_samples_.clear();  // a new speaker front end (src/recognizer.cc:217-220)
  } else {
    engine_->ResetDecoder(slot_);
  }
}

bool Recognizer::AcceptWaveform(const char* data, int len) {
  std::vector<float> w(len / 2);
  const short* s = reinterpret_cast<const short*>(data);
  for (int i = 0; i < len / 2; i++) w[i] = s[i];
  return AcceptWaveform(w);
}

bool Recognizer::AcceptWaveform(const short* data, int len) {
  std::vector<float> w(data, data + len);
  return AcceptWaveform(w);
}

bool Recognizer::AcceptWaveform(const float* data, int len) {
  std::vector<float> w(data, data + len);
  return AcceptWaveform(w);
}

bool Recognizer::AcceptWaveform(std::vector<float>& w) {  // src/recognizer.cc:297-323
  if (!(state_ == RECOGNIZER_RUNNING || state_ == RECOGNIZER_INITIALIZED)) CleanUp();
  state_ = RECOGNIZER_RUNNING;
  // the engine's pruning pass waits for the host to read the records
  // (Engine::SetHostRead): read them now, or the arenas fill up
  if (engine_->PruneWaiting(slot_)) SyncLattice();
  const bool endpoint = Submit(&w, false);  // pieces, silence weights, decoding, endpoint
  KickLattice();  // the lattice replay of the new frames, in the background
  samples_processed_ += w.size();
  if (spk_) spk_samples_.insert(spk_samples_.end(), w.begin(), w.end());  // src/recognizer.cc:314-316
  return endpoint;
}

bool Recognizer::Submit(const std::vector<float>* wave, bool final) {
  req_wave_ = wave;
  req_final_ = final;
  req_error_ = nullptr;
  req_piece_ = 0;
  group_->gc.Run(slot_, [this](const std::vector<int>& slots, std::vector<char>* complete) {
    group_->Serve(slots, complete);
  });
  req_wave_ = nullptr;
  if (req_error_) {  // a failure of this stream alone (the others were served)
    std::exception_ptr e = req_error_;
    req_error_ = nullptr;
    std::rethrow_exception(e);
  }
  return req_endpoint_;
}

// ---------------------------------------------------------------------------
// lattice -> words (src/recognizer.cc:422-482 MbrResult, :669-729 GetResult)
// ---------------------------------------------------------------------------
// A decoder segment's raw lattice pruned at the lattice beam and determinized
// as GetLattice does (phone + word pass, then words); false if unusable (overflow, determinization guard).  Then the
// graph scale, and word alignment when the model has word_boundary.int
// (WordAlignLattice, src/recognizer.cc:433-434; CopyLatticeForMbr otherwise).
static void FinishWordLattice(WordLattice* wl, const ModelData& m, float graph_scale, bool rescore);

static bool WordLatticeFromRaw(RawLattice& raw, const ModelData& m, float graph_scale, WordLattice* wl,
                               bool rescore) {
  if (raw.overflow || raw.tok_state.empty()) return false;
  PruneRawLattice(&raw, m.dec.lattice_beam);
  LatticeOptions opt;
  opt.lattice_beam = m.dec.lattice_beam;
  if (!DeterminizePhonePruned(raw, m.graph, m.tm.tid2phone, m.tm.tid2first, opt, wl) || wl->NumStates() == 0)
    return false;
  FinishWordLattice(wl, m, graph_scale, rescore);
  return true;
}

// After determinization: LM rescoring (final results), the graph scale, word
// alignment when the model has word_boundary.int (WordAlignLattice /
// WordAlignLatticePartial: the same aligner, a word cut at the lattice's end
// forced out with its label; CopyLatticeForMbr otherwise)
static void FinishWordLattice(WordLattice* wl, const ModelData& m, float graph_scale, bool rescore) {
  LatticeOptions opt;
  opt.lattice_beam = m.dec.lattice_beam;
  if (rescore && m.rescore) {  // src/recognizer.cc:680-711
    WordLattice r;
    if (RescoreLattice(*wl, *m.rescore, opt, &r)) *wl = std::move(r);
  }
  if (graph_scale != 1.0f) ScaleGraph(wl, graph_scale);
  if (m.has_word_boundary) {
    WordLattice al;
    if (!WordAlignLattice(*wl, m.tid_boundary, m.tm.tid2final, m.tm.tid2selfloop, opt.max_states, &al) ||
        al.NumStates() == 0) {
      VAMD_WARN("word alignment failed; using the unaligned lattice");
      return;
    }
    *wl = std::move(al);
  }
}

// The decoder segment's lattice (kept on the GPU) as a word lattice.
static bool SegmentWordLattice(Engine* e, int slot, const ModelData& m, bool use_final, float graph_scale,
                               WordLattice* wl, bool rescore = false) {
  RawLattice raw;
  e->GetRawLattice(slot, use_final, &raw);
  return WordLatticeFromRaw(raw, m, graph_scale, wl, rescore);
}

// Without a usable lattice: the best path's words, confidence 1.
static MbrResult PathMbr(const ModelData& m, const std::vector<int>& arcs) {
  MbrResult r;
  for (const WordSeg& w : PathWords(m, arcs)) {
    r.words.push_back(w.word);
    r.conf.push_back(1.0f);
    r.times.push_back({(float)w.start, (float)w.end});
  }
  return r;
}

// Best path of a segment from its copied records, for a segment whose
// lattice is unusable: the traceback kernel's rule (decoder.hip
// traceback_kernel) on the host — the last frame's live token with the
// smallest (cost, plus the final cost if any token is final; state), then its
// backpointers.
static float BitsToFloat(int b) {
  float f;
  std::memcpy(&f, &b, 4);
  return f;
}
static uint32_t OrderedBits(float f) {  // dev_util.h ford
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

std::vector<int> SegmentBestPath(const Graph& g, const SegmentLattice& sl) {
  std::vector<int> arcs;
  if (sl.frames.empty()) return arcs;
  const LatFrame& F = sl.frames.back();
  const long long n = (long long)sl.arena.size();
  if (F.tok_base < 0 || (long long)F.tok_base + F.ntok > n) return arcs;
  const float inf = std::numeric_limits<float>::infinity();
  float bf = inf;
  for (int i = F.tok_base; i < F.tok_base + F.ntok; i++) {
    const int4& e = sl.arena[i];
    if (e.x == -2 || e.w < 0 || e.w >= g.NumStates()) continue;  // dead entry
    if (std::isfinite(g.final_cost[e.w])) bf = std::min(bf, BitsToFloat(e.z) + g.final_cost[e.w]);
  }
  const bool use_f = bf != inf;
  unsigned long long bk = ~0ull;
  long long end = -1;
  for (int i = F.tok_base; i < F.tok_base + F.ntok; i++) {
    const int4& e = sl.arena[i];
    if (e.x == -2 || e.w < 0 || e.w >= g.NumStates()) continue;
    const float c = use_f ? BitsToFloat(e.z) + g.final_cost[e.w] : BitsToFloat(e.z);
    const unsigned long long k = ((unsigned long long)OrderedBits(c) << 32) | (unsigned)e.w;
    if (k < bk) { bk = k; end = i; }
  }
  for (long long k = end; k >= 0 && k < n && (long long)arcs.size() <= n;) {
    const int4& e = sl.arena[k];
    if (e.y < 0) break;
    arcs.push_back(e.y);
    k = e.x;
  }
  std::reverse(arcs.begin(), arcs.end());
  return arcs;
}

// MBR words, confidences and frame times of the segment; graph_scale as the
// reference applies to final results (GraphLatticeScale(0.9), :718), 1 for
// partial results.
static MbrResult SegmentMbr(Engine* e, int slot, const ModelData& m, bool use_final, float graph_scale,
                            bool rescore = false) {
  MbrResult r;
  WordLattice wl;
  if (SegmentWordLattice(e, slot, m, use_final, graph_scale, &wl, rescore)) {
    MinimumBayesRisk(wl, &r);
    return r;
  }
  std::vector<PathResult> pr;
  e->BestPaths({slot}, use_final, &pr);
  return PathMbr(m, pr[0].arcs);
}

std::string Recognizer::WordsText(const std::vector<WordSeg>& w) const {
  std::ostringstream text;
  for (size_t i = 0; i < w.size(); i++) {
    if (i) text << " ";
    text << model_->data()->words.Find(w[i].word);
  }
  return text.str();
}

// ---------------------------------------------------------------------------
// The decoder segment's incremental lattice (incremental.h)
// ---------------------------------------------------------------------------
void Recognizer::ResetLattice() {
  WaitLattice();
  if (inc_init_) inc_.Reset();
  if (engine_ && slot_ >= 0) engine_->SetHostRead(slot_, -1);
  std::lock_guard<std::mutex> lk(inc_mu_);
  adv_ends_.clear();
  adv_done_ = 0;
  inc_next_frame_ = 0;
  inc_last_ = LatFrame{};
  inc_last_prune_ = 0;
  inc_bad_ = false;
}

// the recognizers' lattice replays between calls (VOSK_AMD_LATTICE_THREADS,
// default a quarter of the host threads, 2 to 16)
static WorkerPool& LatticeWorkers() {
  static WorkerPool pool([] {
    const int hw = (int)std::thread::hardware_concurrency();
    return EnvInt("VOSK_AMD_LATTICE_THREADS", std::max(2, std::min(16, hw / 4)));
  }());
  return pool;
}

void Recognizer::WaitLattice() {
  std::unique_lock<std::mutex> lk(inc_mu_);
  inc_cv_.wait(lk, [&] { return !inc_busy_; });
}

void Recognizer::KickLattice() {
  static const bool on = EnvInt("VOSK_AMD_LATTICE_BACKGROUND", 1) != 0;
  if (!on) return;
  {
    std::lock_guard<std::mutex> lk(inc_mu_);
    if (inc_busy_ || inc_bad_ || adv_done_ >= adv_ends_.size()) return;
    inc_busy_ = true;
  }
  LatticeWorkers().Submit([this] {
    try {
      SyncLatticeWork(true);
    } catch (const std::exception& e) {
      VAMD_WARN("recognizer lattice replay failed: " << e.what());
      inc_bad_ = true;
      engine_->SetHostRead(slot_, std::numeric_limits<int>::max());  // nothing reads the records now
    }
    std::lock_guard<std::mutex> lk(inc_mu_);
    inc_busy_ = false;
    inc_cv_.notify_all();
  });
}

bool Recognizer::SyncLattice() {
  WaitLattice();
  return SyncLatticeWork(false);
}

bool Recognizer::SyncLatticeWork(bool background) {
  const ModelData& m = engine_->model();
  if (!inc_init_) {
    IncrementalOptions o;  // LatticeIncrementalDecoderConfig with the model's options
    o.lattice_beam = m.dec.lattice_beam;
    o.prune_interval = m.dec.prune_interval;
    o.determinize_max_delay = m.dec.determinize_max_delay;
    o.determinize_min_chunk_size = m.dec.determinize_min_chunk_size;
    inc_.Init(&m.graph, &m.tm.tid2phone, &m.tm.tid2first, o);
    inc_init_ = true;
  }
  if (inc_bad_) return false;
  // the AdvanceDecoding ends recorded since the last replay (the passes
  // append to adv_ends_ under inc_mu_)
  std::vector<int> ends;
  {
    std::lock_guard<std::mutex> lk(inc_mu_);
    ends.assign(adv_ends_.begin() + (long)adv_done_, adv_ends_.end());
  }
  if (ends.empty() || ends.back() <= 0 || ends.back() < inc_next_frame_) {  // no new frames: nothing to read
    for (size_t i = 0; i < ends.size(); i++, adv_done_++)
      if (ends[i] > 0) inc_.AdvanceEnd();
    return !inc_.failed();
  }
  // the frames decoded since the last replay, with one frame of overlap: the
  // last frame read before, whose tokens the new frame's links point into.
  // The engine's pruning pass compacts the records only once this replay's
  // frames have all been read (Engine::SetHostRead), so between two reads it
  // runs at most once, at the last frame read, moving that frame's tokens as
  // one block in order: its record then has a new base and the same tokens.
  // Anything else (an overflow) falls back.
  const int from = std::max(0, inc_next_frame_ - 1);
  SegmentLattice sl;
  // (no engine lock: a recognizer engine does not pipeline, and passes over
  // other streams -- or this one's next call, when the replay runs in the
  // background -- only append to the records read here)
  (void)background;
  engine_->CopySegmentTail(slot_, from, &sl, ends.back(), true);
  const char* bad = nullptr;
  if (sl.overflow) {
    bad = "lattice arena overflow";
  } else if (sl.frames.empty() || (int)sl.frames.size() + from - 1 < ends.back()) {
    bad = "frames missing";
  } else if (inc_next_frame_ > 0) {
    const LatFrame& f0 = sl.frames[0];
    if (sl.last_prune != inc_last_prune_) {
      if (sl.last_prune != from || f0.ntok != inc_last_.ntok) bad = "records compacted past the last frame read";
    } else if (f0.tok_base != inc_last_.tok_base || f0.ntok != inc_last_.ntok ||
               f0.link_begin != inc_last_.link_begin || f0.link_end != inc_last_.link_end) {
      bad = "records moved";
    }
  }
  if (bad) {
    VAMD_WARN("recognizer lattice records unusable (" << bad << "): results from the best path");
    inc_bad_ = true;
    // the segment's results come from the best path: the engine's pruning
    // need not wait for reads any more (it would let the arenas fill up)
    engine_->SetHostRead(slot_, std::numeric_limits<int>::max());
    return false;
  }
  inc_last_prune_ = sl.last_prune;
  std::vector<int> st;
  std::vector<float> co;
  std::vector<IncFrameIn::Link> ln;
  auto add = [&](int k) {
    const LatFrame& fr = sl.frames[k - from];
    const int a = fr.tok_base - sl.arena_base;
    if (a < 0 || a + fr.ntok > (int)sl.arena.size()) VAMD_ERR("recognizer lattice: arena range");
    st.resize(fr.ntok);
    co.resize(fr.ntok);
    for (int i = 0; i < fr.ntok; i++) {
      const int4 e = sl.arena[a + i];
      if (e.x == -2) VAMD_ERR("recognizer lattice: a dead token in Kaldi order");
      st[i] = e.w;
      co[i] = BitsToFloat(e.z);
    }
    ln.clear();
    const long long lb = fr.link_begin - sl.link_base, le = fr.link_end - sl.link_base;
    if (lb < 0 || le > (long long)sl.links.size()) VAMD_ERR("recognizer lattice: link range");
    const int prev_base = k > 0 ? sl.frames[k - 1 - from].tok_base : 0;
    for (long long i = lb; i < le; i++) {
      const int4 r = sl.links[i];
      const bool emit = r.x < fr.tok_base;  // a source in the previous frame: an emitting arc
      ln.push_back(IncFrameIn::Link{r.x - (emit ? prev_base : fr.tok_base), r.y - fr.tok_base, r.z,
                                    BitsToFloat(r.w), emit});
    }
    IncFrameIn f;
    f.state = st.data();
    f.cost = co.data();
    f.ntok = fr.ntok;
    f.cost_offset = fr.cost_offset;
    f.links = ln.data();
    f.nlinks = (int)ln.size();
    inc_.AddFrame(f);
    inc_last_ = fr;
    inc_next_frame_ = k + 1;
  };
  for (int c : ends) {
    while (inc_.NumFramesDecoded() < c) add(inc_.NumFramesDecoded() + 1);
    inc_.AdvanceEnd();
    adv_done_++;
  }
  engine_->SetHostRead(slot_, inc_next_frame_ - 1);
  return !inc_.failed();
}

// The incremental lattice after determinization -> MBR: rescoring, graph
// scale, alignment, then Kaldi's MBR
bool Recognizer::LatticeMbr(WordLattice&& wl, float graph_scale, bool rescore, MbrResult* r) const {
  *r = MbrResult();
  if (wl.NumStates() == 0) return false;
  FinishWordLattice(&wl, engine_->model(), graph_scale, rescore);
  MinimumBayesRisk(wl, r);
  return true;
}

const char* Recognizer::GetResult() {  // src/recognizer.cc:669-729
  if (engine_->NumFramesDecoded(slot_) == 0) return StoreEmptyReturn();
  const ModelData& m = engine_->model();
  const double t0 = samples_round_start_ / sample_frequency_;
  const double shift = 0.01 * m.dcb.frame_subsampling_factor;
  auto wtext = [&](const std::vector<int>& words) {
    std::ostringstream text;
    for (size_t i = 0; i < words.size(); i++) text << (i ? " " : "") << m.words.Find(words[i]);
    return text.str();
  };
  // FinalizeDecoding, then GetLattice(NumFramesDecoded(), true) over the
  // incremental determinizer (:678); an unusable record set falls back to the
  // one-shot lattice / best path of the segment
  WordLattice clat;
  // development (VOSK_AMD_RESULT_TRACE=1): the result's parts on stderr
  static const bool trace = EnvInt("VOSK_AMD_RESULT_TRACE", 0) != 0;
  using clk = std::chrono::steady_clock;
  const auto tr0 = clk::now();
  const bool synced = SyncLattice();
  const auto tr1 = clk::now();
  const bool inc = synced && (inc_.FinalizeDecoding(), inc_.GetLattice(inc_.NumFramesDecoded(), true, &clat));
  const auto tr2 = clk::now();
  if (inc && clat.NumStates() == 0) return StoreEmptyReturn();  // (rlat.Start() != 0, :714-716)
  if (max_alternatives_ == 0) {  // MbrResult, :429-482
    MbrResult r;
    if (!inc || !LatticeMbr(std::move(clat), 0.9f, true, &r)) r = SegmentMbr(engine_, slot_, m, true, 0.9f, true);
    if (trace) {
      auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
      fprintf(stderr, "[result] frames %d sync %.2f final %.2f mbr %.2f ms\n", inc_.NumFramesDecoded(), ms(tr0, tr1),
              ms(tr1, tr2), ms(tr2, clk::now()));
    }
    Json obj;
    for (size_t i = 0; i < r.words.size(); i++) {
      if (!words_) continue;
      Json word;
      word["word"] = Json::Str(m.words.Find(r.words[i]));
      word["start"] = Json::Float(t0 + (frame_offset_ + r.times[i].first) * shift);
      word["end"] = Json::Float(t0 + (frame_offset_ + r.times[i].second) * shift);
      word["conf"] = Json::Float(r.conf[i]);
      obj["result"].Append(word);
    }
    obj["text"] = Json::Str(wtext(r.words));
    if (spk_) {  // :470-479
      std::vector<float> xv;
      int nspk = 0;
      if (GetSpkVector(&xv, &nspk)) {
        for (float v : xv) obj["spk"].Append(Json::Float(v));
        obj["spk_frames"] = Json::Int(nspk);
      }
    }
    return StoreReturn(obj.Dump());
  }
  // n-best (NbestResult :526-607 / NlsmlResult :609-667): the shortest
  // paths of the graph-scaled word lattice, likelihood = -(graph + acoustic)
  std::vector<NbestPath> nb;
  WordLattice wl;
  bool have = false;
  if (inc) {
    wl = std::move(clat);
    FinishWordLattice(&wl, m, 0.9f, true);
    have = true;
  } else {
    have = SegmentWordLattice(engine_, slot_, m, true, 0.9f, &wl, true);
  }
  if (have) {
    NbestPaths(wl, max_alternatives_, &nb);
  } else {
    std::vector<PathResult> pr;
    engine_->BestPaths({slot_}, true, &pr);
    NbestPath p;
    for (const WordSeg& w : PathWords(m, pr[0].arcs)) {
      p.words.push_back(w.word);
      p.spans.push_back({w.start, w.end});
    }
    p.graph = (float)pr[0].cost;
    nb.push_back(p);
  }
  if (nlsml_) {
    std::stringstream ss;
    ss << "<?xml version=\"1.0\"?>\n<result grammar=\"default\">\n";
    for (const NbestPath& p : nb) {
      const std::string text = wtext(p.words);
      ss << "<interpretation grammar=\"default\" confidence=\"" << -(p.graph + p.acoustic) << "\">\n";
      ss << "<input mode=\"speech\">" << text << "</input>\n";
      ss << "<instance>" << text << "</instance>\n";
      ss << "</interpretation>\n";
    }
    ss << "</result>\n";
    return StoreReturn(ss.str());
  }
  Json obj;
  for (const NbestPath& p : nb) {
    Json entry;
    for (size_t i = 0; i < p.words.size(); i++) {
      if (!words_) continue;
      Json word;
      word["word"] = Json::Str(m.words.Find(p.words[i]));
      word["start"] = Json::Float(t0 + (frame_offset_ + p.spans[i].first) * shift);
      word["end"] = Json::Float(t0 + (frame_offset_ + p.spans[i].second) * shift);
      entry["result"].Append(word);
    }
    entry["text"] = Json::Str(wtext(p.words));
    entry["confidence"] = Json::Float(-(p.graph + p.acoustic));
    obj["alternatives"].Append(entry);
  }
  return StoreReturn(obj.Dump());
}

const char* Recognizer::PartialResult() {  // src/recognizer.cc:732-806
  if (state_ != RECOGNIZER_RUNNING) return StoreEmptyReturn();
  Json res;
  if (engine_->NumFramesDecoded(slot_) == 0) {
    res["partial"] = Json::Str("");
    return StoreReturn(res.Dump());
  }
  const ModelData& m = engine_->model();
  if (partial_words_) {
    // the frames the incremental determinizer has covered: "" until its
    // first chunk, then MBR over GetLattice(NumFramesInLattice(), false)
    // word-aligned (WordAlignLatticePartial), no graph scale (:740-780)
    MbrResult r;
    if (SyncLattice()) {
      if (inc_.NumFramesInLattice() == 0) {
        res["partial"] = Json::Str("");
        return StoreReturn(res.Dump());
      }
      WordLattice clat;
      if (inc_.GetLattice(inc_.NumFramesInLattice(), false, &clat)) {
        LatticeMbr(std::move(clat), 1.0f, false, &r);
      } else {
        r = SegmentMbr(engine_, slot_, m, false, 1.0f);
      }
    } else {
      r = SegmentMbr(engine_, slot_, m, false, 1.0f);
    }
    const double shift = 0.01 * m.dcb.frame_subsampling_factor;
    std::ostringstream text;
    for (size_t i = 0; i < r.words.size(); i++) {
      Json word;
      word["word"] = Json::Str(m.words.Find(r.words[i]));
      word["start"] = Json::Float(samples_round_start_ / sample_frequency_ + (frame_offset_ + r.times[i].first) * shift);
      word["end"] = Json::Float(samples_round_start_ / sample_frequency_ + (frame_offset_ + r.times[i].second) * shift);
      word["conf"] = Json::Float(r.conf[i]);
      res["partial_result"].Append(word);
      text << (i ? " " : "") << m.words.Find(r.words[i]);
    }
    res["partial"] = Json::Str(text.str());
    return StoreReturn(res.Dump());
  }
  std::vector<PathResult> pr;
  engine_->BestPaths({slot_}, false, &pr);
  std::vector<WordSeg> w = PathWords(m, pr[0].arcs);
  res["partial"] = Json::Str(WordsText(w));
  return StoreReturn(res.Dump());
}

const char* Recognizer::Result() {  // src/recognizer.cc:808-816
  if (state_ != RECOGNIZER_RUNNING) return StoreEmptyReturn();
  state_ = RECOGNIZER_ENDPOINT;
  return GetResult();
}

const char* Recognizer::FinalResult() {  // src/recognizer.cc:818-844
  if (state_ != RECOGNIZER_RUNNING) return StoreEmptyReturn();
  engine_->InputFinished(slot_);
  Submit(nullptr, true);  // UpdateSilenceWeights + AdvanceDecoding (src/recognizer.cc:825-826)
  state_ = RECOGNIZER_FINALIZED;
  GetResult();
  return last_result_.c_str();
}

void Recognizer::Reset() {  // src/recognizer.cc:846-853
  StoreEmptyReturn();
  state_ = RECOGNIZER_ENDPOINT;
}

const char* Recognizer::StoreEmptyReturn() {  // src/recognizer.cc:855-871
  if (!max_alternatives_) return StoreReturn("{\"text\": \"\"}");
  if (nlsml_)
    return StoreReturn("<?xml version=\"1.0\"?>\n<result grammar=\"default\">\n"
                       "<interpretation confidence=\"1.0\">\n<instance/>\n"
                       "<input><noinput/></input>\n</interpretation>\n</result>\n");
  return StoreReturn("{\"alternatives\" : [{\"text\": \"\", \"confidence\" : 1.0}] }");
}

const char* Recognizer::StoreReturn(const std::string& s) {
  last_result_ = s;
  return last_result_.c_str();
}

// ---------------------------------------------------------------------------
// WorkerPool
// ---------------------------------------------------------------------------
WorkerPool::WorkerPool(int n, int nice) {
  for (int i = 0; i < std::max(1, n); i++)
    threads_.emplace_back([this, nice] {
      // result work yields to the lanes and the callers' threads when the
      // cores are contended (a thread may always lower its own priority)
      if (nice > 0) (void)setpriority(PRIO_PROCESS, (id_t)syscall(SYS_gettid), nice);
      Run();
    });
}

WorkerPool::~WorkerPool() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : threads_) t.join();
}

void WorkerPool::Submit(std::function<void()> task) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    tasks_.push_back(std::move(task));
  }
  cv_.notify_one();
}

void WorkerPool::WaitIdle() {
  std::unique_lock<std::mutex> lk(mu_);
  idle_cv_.wait(lk, [&] { return tasks_.empty() && busy_ == 0; });
}

// A task's end, also when it throws: busy_ back down (WaitIdle would block
// for ever otherwise) and the caller's current HIP device restored (a task
// may switch devices: SegmentCopy::Finish of a lane on another GPU).
struct WorkerPool::TaskScope {
  WorkerPool* p;
  int dev = -1;
  explicit TaskScope(WorkerPool* pool) : p(pool) {
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  }
  ~TaskScope() {
    if (dev >= 0) (void)hipSetDevice(dev);
    {
      std::lock_guard<std::mutex> lk(p->mu_);
      p->busy_--;
    }
    p->idle_cv_.notify_all();
  }
};

bool WorkerPool::RunOne() {
  std::function<void()> t;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (tasks_.empty()) return false;
    t = std::move(tasks_.front());
    tasks_.pop_front();
    busy_++;
  }
  TaskScope scope(this);
  t();
  return true;
}

void WorkerPool::Run() {
  while (true) {
    std::function<void()> t;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || !tasks_.empty(); });
      if (tasks_.empty()) return;  // stop_
      t = std::move(tasks_.front());
      tasks_.pop_front();
      busy_++;
    }
    TaskScope scope(this);
    try {
      t();
    } catch (const std::exception& e) {  // (tasks publish their own failures)
      VAMD_WARN("result worker task failed: " << e.what());
    }
  }
}

// ---------------------------------------------------------------------------
// BatchModel / BatchRecognizer (src/batch_model.cc, src/batch_recognizer.cc)
// ---------------------------------------------------------------------------
struct BatchModel::Lane {
  int index = 0, device = 0;
  std::unique_ptr<Engine> engine;
  std::mutex mu;
  std::condition_variable cv, done_cv;
  std::vector<BatchRecognizer*> recs;     // admitted streams
  std::vector<BatchRecognizer*> by_slot;  // engine slot -> stream
  int queued = 0;   // chunks queued, not yet handed to the engine
  int streams_queued = 0;  // streams with a queued chunk
  int waiters = 0;         // threads in WaitForCompletion: their feeding round is complete
  int handed = 0;  // chunks handed to the engine, work not finished
  int busy = 0;     // streams with work in the engine
  int tasks = 0;    // results in production
  bool round_wait = false;  // the lane waits for the rest of a feeding round
  bool stop = false;
  std::thread thread;
};

// GPUs of the batch path: VOSK_AMD_BATCH_DEVICES lists the lanes' devices
// explicitly (repeats allowed: "0,0" runs two lanes on device 0);
// VOSK_AMD_DEVICE / LOCAL_RANK pin one (one process per GPU deployments);
// otherwise every visible device (VOSK_AMD_BATCH_GPUS caps).
static std::vector<int> BatchDevices() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
    VAMD_ERR("no HIP device available: the MI355X batch path requires a GPU");
  if (const char* list = getenv("VOSK_AMD_BATCH_DEVICES")) {
    std::vector<int> d;
    std::stringstream ss(list);
    std::string item;
    while (std::getline(ss, item, ',')) {
      if (item.empty()) continue;
      const int dev = atoi(item.c_str());
      if (dev < 0 || dev >= n) VAMD_ERR("VOSK_AMD_BATCH_DEVICES: device " << dev << " of " << n);
      d.push_back(dev);
    }
    if (d.empty()) VAMD_ERR("VOSK_AMD_BATCH_DEVICES lists no device");
    return d;
  }
  if (getenv("VOSK_AMD_DEVICE") || getenv("LOCAL_RANK")) return {DeviceFromEnv()};
  const int cap = EnvInt("VOSK_AMD_BATCH_GPUS", n);
  std::vector<int> d;
  for (int i = 0; i < std::min(n, std::max(cap, 1)); i++) d.push_back(i);
  return d;
}

BatchModel::BatchModel(const std::string& dir) : md_(std::make_shared<ModelData>()) {
  md_->LoadBatchLayout(dir);
  EngineConfig cfg;
  // frames_per_chunk = max(51, right context rounded up to 3) (batch_model.cc:84-88)
  Nnet& nn = md_->nnet;
  NnetPlan probe = BuildNnetPlan(nn, 51, md_->dcb.frame_subsampling_factor, md_->dcb.acoustic_scale);
  int rc = probe.right_context;
  cfg.frames_per_chunk = std::max(51, rc + 3 - rc % 3);
  // channels per GPU: the reference's num_channels = 600 (batch_model.cc:71)
  cfg.max_slots = EnvInt("VOSK_AMD_BATCH_SLOTS", 600);
  cfg.max_step_samples = cfg.frames_per_chunk * md_->mfcc.WindowShift() + 512;
  // per stream: a 1.5 M-token backpointer arena and 2 M lattice links; the
  // in-kernel pruning starts at 300 frames or once one is 3/4 full (~1.1 M
  // tokens / ~1.5 M links: ~370 frames of the bench model, ~2 700 tokens and
  // ~4 000 links per frame), and a quarter is left for the 25 frames between
  // passes (measured high-water marks of the pruned records: 0.86 M tokens /
  // 1.25 M links on the driver's bench, 1.2 M / 1.8 M on 60-s streams with
  // 4 M arenas)
  cfg.arena_tokens = EnvInt("VOSK_AMD_ARENA_TOKENS", 3 << 19);
  cfg.lattice_links = EnvInt("VOSK_AMD_BATCH_LINKS", 1 << 21);
  cfg.prune_fill_pct = 75;
  cfg.lattice = true;  // PushLattice: MBR over each segment's lattice (batch_recognizer.cc:43-107)
  // Kaldi's sequential token-passing order (LatticeFasterDecoder, the CPU
  // reference's 1-best, as north_star asks).  The reference's
  // own batch path decodes with Kaldi's CudaDecoder, whose token set depends
  // on thread timing; its deterministic limit, the order-independent form,
  // stays available (VOSK_AMD_DEC_ORDER=parallel).
  cfg.kaldi_order = true;
  cfg.pipeline = EnvInt("VOSK_AMD_BATCH_PIPELINE", 1) != 0;
  cfg.track_decoded = true;
  cfg.time_kernels = EnvInt("VOSK_AMD_BATCH_TIMING", 0) != 0;
  cfg.collect_stats = EnvInt("VOSK_AMD_BATCH_STATS", 0) != 0;
  samples_per_chunk_ = cfg.frames_per_chunk * md_->mfcc.WindowShift();
  const std::vector<int> devs = BatchDevices();
  for (size_t i = 0; i < devs.size(); i++) {
    auto L = std::make_unique<Lane>();
    L->index = (int)i;
    L->device = devs[i];
    EngineConfig c = cfg;
    c.device = devs[i];
    L->engine.reset(new Engine(md_, c));
    L->by_slot.assign(c.max_slots, nullptr);
    lanes_.push_back(std::move(L));
  }
  // result workers: VOSK_AMD_RESULT_THREADS, default half the host cores
  // this process may use (affinity, capped by OMP_NUM_THREADS when set; at
  // most 16 per GPU) (reference: num_worker_threads = -1, all cores)
  int hc = (int)std::thread::hardware_concurrency();
  {
    cpu_set_t cs;
    if (sched_getaffinity(0, sizeof(cs), &cs) == 0) hc = CPU_COUNT(&cs);
    const int omp = EnvInt("OMP_NUM_THREADS", 0);
    if (omp > 0) hc = std::min(hc, omp);
  }
  // all but the lane threads' (the feeding thread sleeps in Wait() while
  // the tail runs): a stream's final segments all arrive together at
  // FinishStream, when the GPU side is idle, and their lattice work is the
  // tail of the batch; during chunk rounds the workers only see endpoint
  // segments, at a lower priority (nice 5) than the lanes and the callers
  const int cores = std::min(hc > 0 ? hc : 8, 16 * (int)lanes_.size());
  int nt = EnvInt("VOSK_AMD_RESULT_THREADS", std::max(2, cores - (int)lanes_.size()));
  pool_.reset(new WorkerPool(nt, 5));
  fin_trace_ = EnvInt("VOSK_AMD_FINISH_TRACE", 0) != 0;
  for (auto& L : lanes_) {
    Lane* l = L.get();
    l->thread = std::thread([this, l] { LaneLoop(l); });
  }
  VAMD_LOG("batch model: " << lanes_.size() << " GPU lane(s), " << cfg.max_slots << " channels each, "
                           << pool_->size() << " result workers");
}

BatchModel::~BatchModel() {
  for (auto& L : lanes_) {
    {
      std::lock_guard<std::mutex> lk(L->mu);
      L->stop = true;
    }
    L->cv.notify_all();
  }
  for (auto& L : lanes_)
    if (L->thread.joinable()) L->thread.join();
  pool_.reset();
}

int PickLane(const std::vector<std::array<int, 2>>& loads) {
  int best = -1;
  for (int i = 0; i < (int)loads.size(); i++)
    if (best < 0 || loads[i] < loads[best]) best = i;
  return best;
}

Engine* BatchModel::LaneEngine(int i) { return lanes_.at(i)->engine.get(); }

void BatchModel::ResultProfile(double* out) const {
  out[0] = (double)prof_[0];
  out[1] = (double)prof_[1];
  for (int i = 2; i < 11; i++) out[i] = prof_[i] * 1e-6;
  out[11] = (double)prof_[11];
  out[12] = prof_[12] * 1e-6;
}

int BatchModel::LaneOf(const BatchRecognizer* r) const { return r->lane_; }

void BatchModel::BatchingCounters(long long* out) const {
  for (int i = 0; i < 4; i++) out[i] = batching_[i];
}

bool FeedingRoundIncomplete(const std::vector<std::array<long long, 3>>& s) {
  long long n = 0;
  for (const auto& x : s)
    if (x[0] > x[1]) n = std::max(n, x[1] + 1);
  if (n == 0) return false;
  for (const auto& x : s)
    if (!x[2] && x[0] == x[1] && x[0] == n - 1) return true;
  return false;
}

// FeedingRoundIncomplete over a lane's streams (under the lane's mutex)
bool BatchModel::RoundIncomplete(const std::vector<BatchRecognizer*>& recs) {
  std::vector<std::array<long long, 3>> s;
  s.reserve(recs.size());
  for (const BatchRecognizer* r : recs) s.push_back({r->pushed_, r->taken_, r->ended_ ? 1LL : 0LL});
  return FeedingRoundIncomplete(s);
}

void BatchModel::Admit(BatchRecognizer* r, int rate) {
  std::lock_guard<std::mutex> g(admit_mu_);
  std::vector<std::array<int, 2>> loads;
  for (auto& L : lanes_) {
    std::lock_guard<std::mutex> lk(L->mu);
    loads.push_back({L->queued + L->handed, (int)L->recs.size()});
  }
  // PickLane's order; a lane whose channels are all in use is skipped
  std::vector<int> tried(lanes_.size(), 0);
  for (size_t k = 0; k < lanes_.size(); k++) {
    std::vector<std::array<int, 2>> avail;
    std::vector<int> idx;
    for (size_t i = 0; i < lanes_.size(); i++)
      if (!tried[i]) { avail.push_back(loads[i]); idx.push_back((int)i); }
    const int li = idx[PickLane(avail)];
    tried[li] = 1;
    Lane* L = lanes_[li].get();
    int slot;
    try {
      slot = L->engine->AllocSlot();
    } catch (const std::exception&) {
      continue;  // this GPU's channels are all in use
    }
    try {
      L->engine->ResetPipeline(slot);
      L->engine->SetSampleRate(slot, rate);
    } catch (...) {
      L->engine->FreeSlot(slot);
      throw;
    }
    std::lock_guard<std::mutex> lk(L->mu);
    r->lane_ = L->index;
    r->slot_ = slot;
    L->recs.push_back(r);
    L->by_slot[slot] = r;
    return;
  }
  VAMD_ERR("all batch channels of the " << lanes_.size() << " GPU lane(s) are in use");
}

void BatchModel::Release(BatchRecognizer* r) {
  Lane* L = lanes_.at(r->lane_).get();
  {
    std::unique_lock<std::mutex> lk(L->mu);
    L->done_cv.wait(lk, [&] { return r->queue_.empty() && !r->busy_ && r->tasks_ == 0; });
    L->recs.erase(std::remove(L->recs.begin(), L->recs.end(), r), L->recs.end());
    L->by_slot[r->slot_] = nullptr;
  }
  L->engine->FreeSlot(r->slot_);
}

void BatchModel::Push(BatchRecognizer* r, std::vector<float>&& chunk, bool last) {
  Lane* L = lanes_.at(r->lane_).get();
  bool wake;
  {
    std::lock_guard<std::mutex> lk(L->mu);
    if (r->queue_.empty()) L->streams_queued++;
    r->queue_.push_back(BatchRecognizer::Chunk{std::move(chunk), last});
    r->pushed_++;
    L->queued++;
    r->ended_ = last;  // a chunk after FinishStream starts a new utterance
    // a lane waiting for the rest of a feeding round polls every millisecond
    // and is released by Wait(): a push wakes it only when the round it waits
    // for is complete (the lane's own predicate; an idle, ended or slower
    // stream does not hold it back) -- a wake per push made the lane and the
    // feeding thread take turns on the lock
    wake = !L->round_wait || !RoundIncomplete(L->recs);
  }
  if (wake) L->cv.notify_one();
}

int BatchModel::PendingChunks(const BatchRecognizer* r) {
  Lane* L = lanes_.at(r->lane_).get();
  std::lock_guard<std::mutex> lk(L->mu);
  return (int)r->queue_.size() + r->handed_;
}

std::vector<std::array<int, 3>> BatchModel::LaneLoads() {
  std::vector<std::array<int, 3>> out;
  for (auto& L : lanes_) {
    std::lock_guard<std::mutex> lk(L->mu);
    out.push_back({L->device, (int)L->recs.size(), L->queued + L->handed});
  }
  return out;
}

// src/batch_model.cc:118-121.  Every pushed chunk has been decoded; the
// results of finished streams (FinishStream) are published.  An endpoint
// segment of a stream still running may still be in production on the
// worker pool and arrives with a later Result(), as the reference's
// lattice callbacks run asynchronously on its worker threads
// (batch_model.cc:69, batch_recognizer.cc:138-149).
void BatchModel::WaitForCompletion() {
  // the caller's feeding round is complete: every lane's dynamic batching
  // stops waiting for more of it
  for (auto& L : lanes_) {
    {
      std::lock_guard<std::mutex> lk(L->mu);
      L->waiters++;
    }
    L->cv.notify_all();
  }
  struct Leave {
    std::vector<std::unique_ptr<Lane>>& lanes;
    ~Leave() {
      for (auto& L : lanes) {
        std::lock_guard<std::mutex> lk(L->mu);
        L->waiters--;
      }
    }
  } leave{lanes_};
  for (auto& L : lanes_) {
    auto done = [&] {
      if (L->queued != 0 || L->busy != 0) return false;
      for (const BatchRecognizer* r : L->recs)
        if (r->ended_ && r->tasks_ > 0) return false;
      return true;
    };
    while (true) {
      {
        std::lock_guard<std::mutex> lk(L->mu);
        if (done()) break;
      }
      // the caller's thread is idle here: it takes queued result work
      // (final segments arrive together at FinishStream) before sleeping
      if (pool_->RunOne()) continue;
      std::unique_lock<std::mutex> lk(L->mu);
      L->done_cv.wait_for(lk, std::chrono::milliseconds(1), done);
    }
  }
}

std::shared_ptr<SegmentLattice> BatchModel::TakeSegmentBuffer() {
  std::lock_guard<std::mutex> lk(sl_mu_);
  if (sl_pool_.empty()) return std::make_shared<SegmentLattice>();
  auto sl = std::move(sl_pool_.back());
  sl_pool_.pop_back();
  return sl;
}

void BatchModel::ReturnSegmentBuffer(std::shared_ptr<SegmentLattice> sl) {
  std::lock_guard<std::mutex> lk(sl_mu_);
  if (sl_pool_.size() < 64) sl_pool_.push_back(std::move(sl));
}

void BatchModel::EmitSegments(Lane* L, const std::vector<BatchRecognizer*>& rs, bool final_segment) {
  Engine* e = L->engine.get();
  using clk = std::chrono::steady_clock;
  auto ns = [](clk::time_point a, clk::time_point b) {
    return (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count();
  };
  // the segments' lattice records: copies started together (asynchronous,
  // finished by the result workers; the stream's next decoder launch waits
  // for them on the device)
  std::vector<int> frames(rs.size()), cslots;
  std::vector<size_t> ci;
  for (size_t i = 0; i < rs.size(); i++) {
    frames[i] = e->DeviceFramesDecoded(rs[i]->slot_);
    if (frames[i] > 0) {
      cslots.push_back(rs[i]->slot_);
      ci.push_back(i);
    }
  }
  std::vector<std::shared_ptr<SegmentCopy>> started, copies(rs.size());
  const auto tc = clk::now();
  if (!cslots.empty()) e->StartSegmentCopies(cslots, &started);
  for (size_t k = 0; k < ci.size(); k++) copies[ci[k]] = started[k];
  prof_[2] += ns(tc, clk::now());
  if (fin_trace_ && fin_t0_ && final_segment)
    fprintf(stderr, "[finish] +%.2f ms segment copies started (%.2f ms)\n",
            (clk::now().time_since_epoch().count() - fin_t0_) * 1e-6, ns(tc, clk::now()) * 1e-6);
  // the largest lattices first (longest-processing-time order over the
  // result workers: the batch's tail is not one big segment started last);
  // each stream has one segment here, so its results stay in order
  std::vector<size_t> order(rs.size());
  for (size_t i = 0; i < rs.size(); i++) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) {
    const long long nx = copies[x] ? copies[x]->nl : 0, ny = copies[y] ? copies[y]->nl : 0;
    return nx > ny;
  });
  for (size_t i : order) {
    prof_[0]++;
    if (copies[i]) prof_[1] += copies[i]->nl;
    EmitSegment(L, rs[i], final_segment, copies[i], frames[i]);
  }
}

void BatchModel::EmitSegment(Lane* L, BatchRecognizer* r, bool final_segment,
                             std::shared_ptr<SegmentCopy> copy, int frames) {
  const float shift = 0.01f * md_->dcb.frame_subsampling_factor;
  using clk = std::chrono::steady_clock;
  auto ns = [](clk::time_point a, clk::time_point b) {
    return (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count();
  };
  const double offset = r->segment_offset_;
  r->segment_offset_ = final_segment ? 0.0 : r->segment_offset_ + frames * shift;
  if (final_segment) r->utt_samples_ = 0;
  const uint64_t seq = r->next_seq_++;
  {
    std::lock_guard<std::mutex> lk(L->mu);
    r->tasks_++;
    L->tasks++;
  }
  pool_->Submit([this, L, r, copy, seq, offset, frames, ns]() {
    const ModelData& m = *md_;
    MbrResult res;
    std::shared_ptr<SegmentLattice> sl = TakeSegmentBuffer();
    try {
      const auto tw = clk::now();
      if (copy) copy->Finish(sl.get());
      else *sl = SegmentLattice();
      prof_[2] += ns(tw, clk::now());
      if (frames > 0) {
        RawLattice raw;
        const auto t0 = clk::now();
        if (!sl->frames.empty())
          BuildRawLattice(m.graph, m.graph.start, sl->frames, sl->arena, sl->links, true, &raw);
        raw.overflow = raw.overflow || sl->overflow;
        const auto t1 = clk::now();
        WordLattice wl;
        const bool ok = WordLatticeFromRaw(raw, m, 0.9f, &wl, false);
        const auto t2 = clk::now();
        if (ok) MinimumBayesRisk(wl, &res);
        else res = PathMbr(m, SegmentBestPath(m.graph, *sl));  // lattice unusable: 1-best words
        prof_[3] += ns(t0, t1);
        prof_[4] += ns(t1, t2);
        prof_[5] += ns(t2, clk::now());
      }
    } catch (const std::exception& ex) {
      VAMD_WARN("batch result failed: " << ex.what());
      res = MbrResult();
    }
    ReturnSegmentBuffer(sl);
    const auto tf = clk::now();
    std::string js = r->FormatResult(res, offset);
    prof_[6] += ns(tf, clk::now());
    r->PublishResult(seq, std::move(js));
    int left;
    {
      std::lock_guard<std::mutex> lk(L->mu);
      r->tasks_--;
      left = --L->tasks;
    }
    if (fin_trace_ && fin_t0_ && left == 0)
      fprintf(stderr, "[finish] +%.2f ms last result task done\n",
              (clk::now().time_since_epoch().count() - fin_t0_) * 1e-6);
    L->done_cv.notify_all();
  });
}

void BatchModel::LaneLoop(Lane* L) {
  Engine* e = L->engine.get();
  (void)hipSetDevice(L->device);
  const ModelData& m = *md_;
  const float shift = 0.01f * m.dcb.frame_subsampling_factor;
  // no endpoint rule fires before its minimum utterance length
  float min_len = 1e30f;
  for (const EndpointRule& rule : m.endpoint.rule) min_len = std::min(min_len, rule.min_utterance_length);
  std::vector<BatchRecognizer*> active;  // streams with work in the engine
  std::vector<Engine::DecodedJob> decoded;
  std::vector<int> slots, probe;
  std::vector<BatchRecognizer*> probe_r, ends, retire, finals;
  std::vector<EndpointProbe> pr;
  bool pipelined = false;
  const bool trace = EnvInt("VOSK_AMD_BATCH_TRACE", 0) != 0;  // development: one line per lane step
  // test hook (VOSK_AMD_BATCH_SCHEDULE=<seed>): a seeded random lane schedule.
  // Each queued stream's chunk is taken or left for a later step at random,
  // the bounded wait for the feeding round is skipped, and a step with an
  // idle pipeline runs in order or pipelined at random.  Segment boundaries
  // and results must not depend on any of it (tests/test_batching.py).
  uint64_t rng = (uint64_t)(unsigned)EnvInt("VOSK_AMD_BATCH_SCHEDULE", 0) * 0x9E3779B97F4A7C15ull;
  const bool sched = rng != 0;
  auto rnd = [&rng]() {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return rng >> 11;
  };
  std::vector<int> seen_slot(L->by_slot.size(), 0);
  long long iter = 0;
  using clk = std::chrono::steady_clock;
  auto ns = [](clk::time_point a, clk::time_point b) {
    return (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count();
  };
  while (true) {
    std::vector<std::pair<BatchRecognizer*, BatchRecognizer::Chunk>> batch;
    clk::time_point tw;
    {
      std::unique_lock<std::mutex> lk(L->mu);
      // idle with every stream finished (FinishStream): the lane's thread
      // helps with the final segments' result work (no chunk can be waiting
      // for it; a push ends the help after the task at hand)
      while (!L->stop && L->queued == 0 && active.empty() && !L->recs.empty() &&
             std::all_of(L->recs.begin(), L->recs.end(), [](const BatchRecognizer* r) { return r->ended_; })) {
        lk.unlock();
        const bool ran = pool_->RunOne();
        lk.lock();
        if (!ran) break;
      }
      L->cv.wait(lk, [&] { return L->stop || L->queued > 0 || !active.empty(); });
      if (L->stop) return;
      tw = clk::now();
      // dynamic batching (CudaOnlinePipelineDynamicBatcher, batch_model.cc:94-96):
      // with the GPU idle, wait for the rest of this feeding round, i.e. by
      // chunk sequence: the round's chunk number n is the furthest queued
      // chunk, and every running stream that has pushed chunk n-1 is waited
      // for until it has pushed chunk n.  The wait ends early when a thread
      // calls Wait() (its feeding round is complete) and is bounded (12 ms,
      // or no push for 4 ms).  A round split by a feeding pause costs a
      // second step as long as its slowest stream; the next round is whole
      // again, since the rule looks at sequence numbers, not at the last
      // batch's size.
      if (!sched && L->queued > 0 && !e->PipelineBusy()) {
        const auto t0 = clk::now();
        auto last_push = t0;
        L->round_wait = true;
        while (!L->stop && L->waiters == 0 && RoundIncomplete(L->recs)) {
          const int before = L->queued;
          L->cv.wait_for(lk, std::chrono::microseconds(1000));
          const auto now = clk::now();
          if (L->queued != before) last_push = now;
          if (now - t0 > std::chrono::milliseconds(12) || now - last_push > std::chrono::milliseconds(4)) {
            batching_[1]++;  // bounded wait expired: the round is split
            break;
          }
        }
        L->round_wait = false;
        if (L->waiters > 0 && RoundIncomplete(L->recs)) batching_[2]++;
      }
      auto take = [&](BatchRecognizer* r) {
        batch.emplace_back(r, std::move(r->queue_.front()));
        r->queue_.pop_front();
        L->queued--;
        if (r->queue_.empty()) L->streams_queued--;
        r->handed_++;
        r->taken_++;
        r->utt_samples_ += (long long)batch.back().second.data.size();
        L->handed++;
        if (!r->busy_) {
          r->busy_ = true;
          L->busy++;
          active.push_back(r);
        }
      };
      BatchRecognizer* first_queued = nullptr;
      for (BatchRecognizer* r : L->recs) {  // one chunk per stream per step
        if (r->queue_.empty()) continue;
        if (!first_queued) first_queued = r;
        if (sched && (rnd() & 1)) continue;  // left for a later step
        take(r);
      }
      // (the random schedule always takes a chunk when nothing else would run)
      if (sched && batch.empty() && active.empty() && first_queued) take(first_queued);
      // pipeline the stages while a backlog keeps them fed; a batch with
      // nothing queued behind it runs its stages in order (one sync, not three)
      pipelined = L->queued > 0 || e->PipelineBusy();
      // (an in-order step drains the pipeline first: only with it idle)
      if (sched && !e->PipelineBusy()) pipelined = (rnd() & 1) != 0;
    }
    const auto ts = clk::now();
    prof_[7] += ns(tw, ts);
    prof_[11]++;
    batching_[0]++;
    bool failed = false;
    const bool tr = trace && (++iter < 300 || iter % 20000 == 0);
    if (tr)
      fprintf(stderr, "[lane %d] batch=%zu active=%zu queued=%d busy=%d tasks=%d pipelined=%d pipe_busy=%d\n",
              L->index, batch.size(), active.size(), L->queued, L->busy, L->tasks, (int)pipelined,
              (int)e->PipelineBusy());
    auto fin_ms = [&]() { return (clk::now().time_since_epoch().count() - fin_t0_) * 1e-6; };
    bool fin_step = false;
    try {
      for (auto& [r, c] : batch) {
        if (!c.data.empty()) e->AcceptSamples(r->slot_, std::move(c.data));
        if (c.last) {
          e->InputFinished(r->slot_);
          r->finishing_ = true;
          if (fin_trace_ && !fin_t0_) fin_t0_ = (long long)ts.time_since_epoch().count();
        }
      }
      slots.clear();
      for (BatchRecognizer* r : active) {
        slots.push_back(r->slot_);
        fin_step = fin_step || r->finishing_;
      }
      fin_step = fin_step && fin_trace_ && fin_t0_;
      if (fin_step)
        fprintf(stderr, "[finish] +%.2f ms step: batch %zu active %zu pipelined %d\n", fin_ms(), batch.size(),
                active.size(), (int)pipelined);
      e->Step(slots, pipelined);
      if (fin_step) fprintf(stderr, "[finish] +%.2f ms step returned\n", fin_ms());
      prof_[8] += ns(ts, clk::now());
      const auto tp = clk::now();
      // reset_on_endpoint (batch_model.cc:72): streams whose decoder job just
      // completed, checked on the device state without draining the pipeline
      e->TakeDecoded(&decoded);
      probe.clear();
      probe_r.clear();
      // every decoder job of a stream is followed by its own probe: a step
      // completes at most one job per stream (one decoder batch per step, one
      // job per stream in a batch), so the rules always see the state after
      // each chunk -- counted if that ever fails to hold
      for (const Engine::DecodedJob& dj : decoded)
        if (seen_slot[dj.slot]++) batching_[3]++;
      for (const Engine::DecodedJob& dj : decoded) seen_slot[dj.slot] = 0;
      for (const Engine::DecodedJob& dj : decoded) {
        const int s = dj.slot;
        BatchRecognizer* r = L->by_slot[s];
        // the last frames of a stream: its final segment ends when it is idle
        if (!r || dj.input_ended) continue;
        const int frames = e->DeviceFramesDecoded(s);
        if (frames <= 0 || frames * shift < min_len) continue;
        probe.push_back(s);
        probe_r.push_back(r);
      }
      if (!probe.empty()) {
        const auto tq = clk::now();
        e->ProbeEndpoints(probe, &pr);
        prof_[12] += ns(tq, clk::now());
        ends.clear();
        std::vector<int> end_slots;
        for (size_t i = 0; i < probe.size(); i++)
          if (EndpointRulesFire(m.endpoint, pr[i].frames, pr[i].trailing_sil, shift, pr[i].final_relative_cost)) {
            ends.push_back(probe_r[i]);
            end_slots.push_back(probe[i]);
          }
        if (!ends.empty()) {
          EmitSegments(L, ends, false);
          for (BatchRecognizer* r : ends) e->ResetDecoderAtNextJob(r->slot_);
        }
      }
      prof_[9] += ns(tp, clk::now());
    } catch (const std::exception& ex) {
      VAMD_WARN("batch step failed on GPU " << L->device << ": " << ex.what());
      failed = true;
    }
    const auto tr0 = clk::now();
    // streams with nothing left in the engine: their chunks are done; a
    // finishing stream's final segment ends here (FinishStream)
    retire.clear();
    finals.clear();
    for (BatchRecognizer* r : active) {
      bool idle = failed;
      if (!idle) {
        try {
          idle = e->StreamIdle(r->slot_);
        } catch (const std::exception&) {
          idle = true;
        }
      }
      if (!idle) continue;
      retire.push_back(r);
      if (r->finishing_) {
        finals.push_back(r);
      } else if (failed) {
        // the step failed: the stream's decoder segment is lost.  Its engine
        // slot is restarted (staged jobs and pending samples dropped, so the
        // engine's state matches the retirement) and the segment ends with an
        // empty result, so Result() reports the gap instead of staying silent
        try {
          e->ResetPipeline(r->slot_);
        } catch (const std::exception& ex) {
          VAMD_WARN("batch stream reset after a failed step: " << ex.what());
        }
        // later segments keep the stream's time base: they start after every
        // sample handed to the engine so far (the dropped chunk included)
        const double gap_start = r->segment_offset_;
        r->segment_offset_ = (double)r->utt_samples_ / md_->mfcc.samp_freq;
        r->PublishResult(r->next_seq_++, r->FormatResult(MbrResult(), gap_start));
      }
    }
    if (!finals.empty()) {
      try {
        slots.clear();
        for (BatchRecognizer* r : finals) slots.push_back(r->slot_);
        if (fin_step) fprintf(stderr, "[finish] +%.2f ms %zu finals, segment copies\n", fin_ms(), finals.size());
        EmitSegments(L, finals, true);
        if (fin_step) fprintf(stderr, "[finish] +%.2f ms segment tasks submitted\n", fin_ms());
        for (BatchRecognizer* r : finals) e->ResetPipeline(r->slot_);  // a later AcceptWaveform: new utterance
      } catch (const std::exception& ex) {
        // every finished stream still gets a (empty) final result
        VAMD_WARN("batch final results failed on GPU " << L->device << ": " << ex.what());
        for (BatchRecognizer* r : finals) r->PublishResult(r->next_seq_++, r->FormatResult(MbrResult(), 0.0));
      }
    }
    if (tr) {
      fprintf(stderr, "[lane %d] decoded=%zu probed=%zu retire=%zu finals=%zu failed=%d\n", L->index,
              decoded.size(), probe.size(), retire.size(), finals.size(), (int)failed);
      for (BatchRecognizer* r : active)
        if (std::find(retire.begin(), retire.end(), r) == retire.end()) {
          fprintf(stderr, "  busy: %s finishing=%d\n", e->DescribeSlot(r->slot_).c_str(), (int)r->finishing_);
          break;
        }
    }
    prof_[10] += ns(tr0, clk::now());
    if (!retire.empty()) {
      {
        std::lock_guard<std::mutex> lk(L->mu);
        for (BatchRecognizer* r : retire) {
          r->busy_ = false;
          r->finishing_ = false;
          L->busy--;
          L->handed -= r->handed_;
          r->handed_ = 0;
          active.erase(std::find(active.begin(), active.end(), r));
        }
      }
      L->done_cv.notify_all();
    }
  }
}

BatchRecognizer::BatchRecognizer(BatchModel* model, float sr) : model_(model) {
  // the reference resamples each call on its own, flushed at the call's end
  // (src/batch_recognizer.cc:27-29,157-158), and chunks the model-rate
  // samples: the stream's engine slot runs at the model rate and each call
  // at another rate goes through Engine::ResampleCall (GPU) first
  const int rate = InputRate(sr);
  const int model_rate = (int)std::lround(model_->data().mfcc.samp_freq);
  call_rate_ = rate == model_rate ? 0 : rate;
  model_->Admit(this, model_rate);
  if (call_rate_) {
    // a failed table lookup (too many distinct rates, an upload error) must
    // not leave this half-built recognizer admitted on the lane
    try {
      call_table_ = model_->lane_engine(lane_)->ResampleTableFor(call_rate_, &call_tab_);
    } catch (...) {
      model_->Release(this);
      throw;
    }
  }
  model_->Ref();
}

BatchRecognizer::~BatchRecognizer() {
  model_->Release(this);
  model_->Unref();
}

void BatchRecognizer::AcceptWaveform(const char* data, int len) {  // batch_recognizer.cc:115-181
  const short* s = reinterpret_cast<const short*>(data);
  if (call_rate_) {
    std::vector<float> x(s, s + len / 2);
    std::vector<float> y = model_->lane_engine(lane_)->ResampleCall(call_table_, call_tab_, x.data(), (int)x.size());
    buffer_.insert(buffer_.end(), y.begin(), y.end());
  } else {
    buffer_.insert(buffer_.end(), s, s + len / 2);
  }
  const int spc = model_->samples_per_chunk();
  size_t i = 0;
  while (i + spc <= buffer_.size()) {
    model_->Push(this, std::vector<float>(buffer_.begin() + i, buffer_.begin() + i + spc), false);
    i += spc;
  }
  if (i) buffer_.erase(buffer_.begin(), buffer_.begin() + i);
}

void BatchRecognizer::FinishStream() {  // batch_recognizer.cc:37-41
  model_->Push(this, std::move(buffer_), true);
  buffer_.clear();
}

std::string BatchRecognizer::FormatResult(const MbrResult& r, double offset) const {
  // batch_recognizer.cc:43-107 (PushLattice: MBR words, confidences, rounded frame times)
  const ModelData& m = model_->data();
  std::stringstream text;
  for (size_t i = 0; i < r.words.size(); i++) {
    if (i) text << " ";
    text << m.words.Find(r.words[i]);
  }
  if (nlsml_) {
    float confidence = 0.0f;
    for (float c : r.conf) confidence += c;
    confidence /= (float)r.words.size();  // NaN for an empty result, as the reference
    std::stringstream ss;
    ss << "<?xml version=\"1.0\"?>\n<result grammar=\"default\">\n";
    ss << "<interpretation grammar=\"default\" confidence=\"" << confidence
       << "\">\n<input mode=\"speech\">" << text.str() << "</input>\n<instance>" << text.str()
       << "</instance>\n</interpretation>\n</result>\n";
    return ss.str();
  }
  Json obj;
  for (size_t i = 0; i < r.words.size(); i++) {
    Json word;
    word["word"] = Json::Str(m.words.Find(r.words[i]));
    word["start"] = Json::Float(std::round((double)r.times[i].first) * 0.03 + offset);
    word["end"] = Json::Float(std::round((double)r.times[i].second) * 0.03 + offset);
    word["conf"] = Json::Float(r.conf[i]);
    obj["result"].Append(word);
  }
  obj["text"] = Json::Str(text.str());
  return obj.Dump();
}

void BatchRecognizer::PublishResult(uint64_t seq, std::string&& json) {
  std::lock_guard<std::mutex> lk(rmu_);
  reorder_[seq] = std::move(json);
  for (auto it = reorder_.find(publish_seq_); it != reorder_.end(); it = reorder_.find(publish_seq_)) {
    results_.push_back(std::move(it->second));
    reorder_.erase(it);
    publish_seq_++;
  }
}

// The bindings read a result as FrontResult() then Pop() (python/vosk
// BatchRecognizer.Result).  A Pop() right after a FrontResult() that found
// nothing pops nothing: a result published by a worker in between stays for
// the next read instead of being dropped unseen.
const char* BatchRecognizer::FrontResult() {
  std::lock_guard<std::mutex> lk(rmu_);
  if (results_.empty()) {
    front_state_ = 0;
    return "";
  }
  front_ = results_.front();
  front_state_ = 1;
  return front_.c_str();
}

void BatchRecognizer::Pop() {
  std::lock_guard<std::mutex> lk(rmu_);
  if (front_state_ != 0 && !results_.empty()) results_.pop_front();
  front_state_ = -1;
}

}  // namespace vamd
