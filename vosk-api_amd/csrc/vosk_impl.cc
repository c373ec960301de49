// Vosk object layer (see vosk_impl.h).
#include "vosk_impl.h"
#include "graph_compose.h"

#include <cmath>
#include <cstdlib>
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

Engine* Model::StreamEngine() {
  std::lock_guard<std::mutex> lk(mu_);
  return StreamEngineLocked();
}

Engine* Model::GrammarEngine(const std::string& grammar) {
  std::lock_guard<std::mutex> lk(mu_);
  if (!md_->lookahead_hcl) {
    VAMD_WARN("Runtime graphs are not supported by this model");
    return StreamEngineLocked();
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
  Engine* e = new Engine(md, cfg);
  grammar_engines_[grammar].reset(e);
  return e;
}

Engine* Model::StreamEngineLocked() {
  if (!engine_) {
    EngineConfig cfg;
    cfg.frames_per_chunk = md_->dcb.frames_per_chunk;
    cfg.max_slots = EnvInt("VOSK_AMD_MAX_STREAMS", 64);
    cfg.device = DeviceFromEnv();
    cfg.max_step_samples = 4096;
    cfg.lattice = true;  // results come from the segment's lattice (MBR)
    engine_.reset(new Engine(md_, cfg));
  }
  return engine_.get();
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
  engine_ = grammar ? model->GrammarEngine(grammar) : model->StreamEngine();
  slot_ = engine_->AllocSlot();
  try {
    engine_->SetSampleRate(slot_, rate);
  } catch (...) {
    engine_->FreeSlot(slot_);
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
  engine_->FreeSlot(slot_);
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
  const int step = (int)(sample_frequency_ * 0.2f);
  for (size_t i = 0; i < w.size(); i += step) {
    const int n = (int)std::min<size_t>(step, w.size() - i);
    engine_->AcceptSamples(slot_, w.data() + i, n);
    engine_->UpdateSilenceWeights(slot_, frame_offset_ * 3);  // src/recognizer.cc:309
    engine_->Advance({slot_});
  }
  samples_processed_ += w.size();
  if (spk_) spk_samples_.insert(spk_samples_.end(), w.begin(), w.end());  // src/recognizer.cc:314-316
  return EndpointDetected();
}

bool Recognizer::EndpointDetected() {
  const int frames = engine_->NumFramesDecoded(slot_);
  if (frames == 0) return false;
  std::vector<PathResult> pr;
  engine_->BestPaths({slot_}, false, &pr);
  const ModelData& m = engine_->model();
  const float shift = 0.01f * m.dcb.frame_subsampling_factor;
  return EndpointRulesFire(m.endpoint, frames, TrailingSilenceFrames(m, pr[0].arcs), shift,
                           pr[0].final_relative_cost);
}

// ---------------------------------------------------------------------------
// lattice -> words (src/recognizer.cc:422-482 MbrResult, :669-729 GetResult)
// ---------------------------------------------------------------------------
// The decoder segment's lattice (kept on the GPU), pruned at the lattice beam
// and determinized on words; false if unavailable (no lattice engine,
// overflow, determinization guard).
// Then the graph scale, and word alignment when the model has
// word_boundary.int (WordAlignLattice, :433-434; CopyLatticeForMbr otherwise).
static bool SegmentWordLattice(Engine* e, int slot, const ModelData& m, bool use_final, float graph_scale,
                               WordLattice* wl, bool rescore = false) {
  RawLattice raw;
  e->GetRawLattice(slot, use_final, &raw);
  if (raw.overflow || raw.tok_state.empty()) return false;
  PruneRawLattice(&raw, m.dec.lattice_beam);
  LatticeOptions opt;
  opt.lattice_beam = m.dec.lattice_beam;
  if (!DeterminizeToWords(raw, m.graph, opt, wl) || wl->NumStates() == 0) return false;
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
      return true;
    }
    *wl = std::move(al);
  }
  return true;
}

// MBR words, confidences and frame times of the segment; graph_scale as the
// reference applies to final results (GraphLatticeScale(0.9), :718), 1 for
// partial results.  Without a lattice: the best path, confidence 1.
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
  for (const WordSeg& w : PathWords(m, pr[0].arcs)) {
    r.words.push_back(w.word);
    r.conf.push_back(1.0f);
    r.times.push_back({(float)w.start, (float)w.end});
  }
  return r;
}

std::string Recognizer::WordsText(const std::vector<WordSeg>& w) const {
  std::ostringstream text;
  for (size_t i = 0; i < w.size(); i++) {
    if (i) text << " ";
    text << model_->data()->words.Find(w[i].word);
  }
  return text.str();
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
  if (max_alternatives_ == 0) {  // MbrResult, :429-482
    const MbrResult r = SegmentMbr(engine_, slot_, m, true, 0.9f, true);
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
  if (SegmentWordLattice(engine_, slot_, m, true, 0.9f, &wl, true)) {
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
  if (partial_words_) {  // MBR over the partial lattice, no final costs, no graph scale (:740-780)
    const MbrResult r = SegmentMbr(engine_, slot_, m, false, 1.0f);
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
  engine_->UpdateSilenceWeights(slot_, frame_offset_ * 3);  // src/recognizer.cc:825
  engine_->Advance({slot_});
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
// BatchModel / BatchRecognizer (src/batch_model.cc, src/batch_recognizer.cc)
// ---------------------------------------------------------------------------
BatchModel::BatchModel(const std::string& dir) : md_(std::make_shared<ModelData>()) {
  md_->LoadBatchLayout(dir);
  EngineConfig cfg;
  // frames_per_chunk = max(51, right context rounded up to 3) (batch_model.cc:84-88)
  Nnet& nn = md_->nnet;
  NnetPlan probe = BuildNnetPlan(nn, 51, md_->dcb.frame_subsampling_factor, md_->dcb.acoustic_scale);
  int rc = probe.right_context;
  cfg.frames_per_chunk = std::max(51, rc + 3 - rc % 3);
  cfg.max_slots = EnvInt("VOSK_AMD_BATCH_SLOTS", 256);
  cfg.device = DeviceFromEnv();
  cfg.max_step_samples = cfg.frames_per_chunk * md_->mfcc.WindowShift() + 512;
  cfg.arena_tokens = EnvInt("VOSK_AMD_ARENA_TOKENS", 1 << 22);
  cfg.lattice = true;  // PushLattice: MBR over each segment's lattice (batch_recognizer.cc:43-107)
  engine_.reset(new Engine(md_, cfg));
  samples_per_chunk_ = cfg.frames_per_chunk * md_->mfcc.WindowShift();
  worker_ = std::thread([this] { Worker(); });
}

BatchModel::~BatchModel() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (worker_.joinable()) worker_.join();
}

void BatchModel::Register(BatchRecognizer* r) {
  std::lock_guard<std::mutex> lk(mu_);
  queues_[r];
}

void BatchModel::Unregister(BatchRecognizer* r) {
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [&] { return queues_[r].empty() && in_flight_ == 0; });
  queues_.erase(r);
}

void BatchModel::Push(BatchRecognizer* r, std::vector<float>&& chunk, bool last) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    queues_[r].push_back(Chunk{std::move(chunk), last});
  }
  cv_.notify_all();
}

int BatchModel::PendingChunks(const BatchRecognizer* r) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = queues_.find(const_cast<BatchRecognizer*>(r));
  return it == queues_.end() ? 0 : (int)it->second.size();
}

void BatchModel::WaitForCompletion() {  // src/batch_model.cc:118-121
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [&] {
    if (in_flight_) return false;
    for (auto& q : queues_)
      if (!q.second.empty()) return false;
    return true;
  });
}

void BatchModel::Worker() {
  const ModelData& m = *md_;
  const float shift = 0.01f * m.dcb.frame_subsampling_factor;
  while (true) {
    std::vector<std::pair<BatchRecognizer*, Chunk>> batch;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] {
        if (stop_) return true;
        for (auto& q : queues_)
          if (!q.second.empty()) return true;
        return false;
      });
      if (stop_) return;
      for (auto& q : queues_)
        if (!q.second.empty()) {
          batch.emplace_back(q.first, std::move(q.second.front()));
          q.second.pop_front();
        }
      in_flight_ = 1;
    }
    try {
      std::vector<int> slots;
      for (auto& [r, c] : batch) {
        if (!c.data.empty()) engine_->AcceptSamples(r->slot(), c.data.data(), (int)c.data.size());
        if (c.last) engine_->InputFinished(r->slot());
        slots.push_back(r->slot());
      }
      engine_->Advance(slots);
      // endpoint (reset_on_endpoint, batch_model.cc:72) and end-of-stream results
      std::vector<int> tb;
      for (auto& [r, c] : batch)
        if (engine_->NumFramesDecoded(r->slot()) > 0) tb.push_back(r->slot());
      std::vector<PathResult> nofinal, withfinal;
      engine_->BestPaths(tb, false, &nofinal);
      size_t k = 0;
      for (auto& [r, c] : batch) {
        const int s = r->slot();
        const int frames = engine_->NumFramesDecoded(s);
        if (c.last) {
          r->PushResult(frames > 0 ? SegmentMbr(engine_.get(), s, m, true, 0.9f) : MbrResult(),
                        r->segment_offset_);
          if (frames > 0) k++;
          continue;
        }
        if (frames == 0) continue;
        const PathResult& p = nofinal[k++];
        if (EndpointRulesFire(m.endpoint, frames, TrailingSilenceFrames(m, p.arcs), shift,
                              p.final_relative_cost)) {
          r->PushResult(SegmentMbr(engine_.get(), s, m, true, 0.9f), r->segment_offset_);
          r->segment_offset_ += frames * shift;
          engine_->ResetDecoder(s);
        }
      }
    } catch (const std::exception& e) {
      VAMD_WARN("batch step failed: " << e.what());
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      in_flight_ = 0;
    }
    done_cv_.notify_all();
  }
}

BatchRecognizer::BatchRecognizer(BatchModel* model, float sr) : model_(model), sample_frequency_(sr) {
  // the reference resamples each call independently (flush per call,
  // src/batch_recognizer.cc:27-29,157-158); here the stream is resampled
  // continuously (no discontinuity at call boundaries)
  const int rate = InputRate(sr);
  slot_ = model_->engine()->AllocSlot();
  model_->engine()->ResetPipeline(slot_);
  try {
    model_->engine()->SetSampleRate(slot_, rate);
  } catch (...) {
    model_->engine()->FreeSlot(slot_);
    throw;
  }
  model_->Register(this);
}

BatchRecognizer::~BatchRecognizer() {
  model_->Unregister(this);
  model_->engine()->FreeSlot(slot_);
}

void BatchRecognizer::AcceptWaveform(const char* data, int len) {  // batch_recognizer.cc:115-181
  const short* s = reinterpret_cast<const short*>(data);
  buffer_.insert(buffer_.end(), s, s + len / 2);
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

void BatchRecognizer::PushResult(const MbrResult& r, double offset) {
  // batch_recognizer.cc:43-107 (PushLattice: MBR words, confidences, rounded frame times)
  const ModelData& m = model_->data();
  std::string out;
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
    out = ss.str();
  } else {
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
    out = obj.Dump();
  }
  std::lock_guard<std::mutex> lk(rmu_);
  results_.push_back(out);
}

const char* BatchRecognizer::FrontResult() {
  std::lock_guard<std::mutex> lk(rmu_);
  if (results_.empty()) return "";
  front_ = results_.front();
  return front_.c_str();
}

void BatchRecognizer::Pop() {
  std::lock_guard<std::mutex> lk(rmu_);
  if (!results_.empty()) results_.pop_front();
}

}  // namespace vamd
