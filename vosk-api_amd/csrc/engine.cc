// GPU engine (see engine.h).
#include "engine.h"

#include <sstream>
#include "graph_compose.h"

#include <algorithm>
#include <fstream>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>

#include "common.h"
#include "kernels.h"

#define HIPCHECK(x)                                                                  \
  do {                                                                               \
    hipError_t _e = (x);                                                             \
    if (_e != hipSuccess) VAMD_ERR("HIP error " << hipGetErrorString(_e) << " at " \
                                                << __FILE__ << ":" << __LINE__);     \
  } while (0)
// HIP's current device is per host thread: every entry point that touches the
// device selects the engine's (BatchModel lanes drive one engine per GPU)
#define DEVICE_GUARD() HIPCHECK(hipSetDevice(cfg_.device))

namespace vamd {

namespace {
int Pow2AtLeast(long long n) {
  int p = 1;
  while (p < n) p <<= 1;
  return p;
}
size_t Align256(size_t x) { return (x + 255) & ~(size_t)255; }
float MelScale(float f) { return 1127.0f * logf(1.0f + f / 700.0f); }
}  // namespace

// ---------------------------------------------------------------------------
// model directory loading (src/model.cc:106-341, src/batch_model.cc:23-54)
// ---------------------------------------------------------------------------
void ModelData::Load(const std::string& path) {
  dir = path;
  std::string mdl, hclg, hcl, gr, disambig_int, words_txt, wb, mfcc_conf, fbank_conf, cmvn_stats, pitch_conf, conf_file;
  if (FileExists(path + "/am/final.mdl") && FileExists(path + "/conf/model.conf")) {
    // V2 layout (src/model.cc:180-207)
    ApplyModelOptions(ReadConfigFile(path + "/conf/model.conf"), &dec, &dcb, &endpoint);
    mdl = path + "/am/final.mdl";
    hclg = path + "/graph/HCLG.fst";
    hcl = path + "/graph/HCLr.fst";
    gr = path + "/graph/Gr.fst";
    disambig_int = path + "/graph/disambig_tid.int";
    words_txt = path + "/graph/words.txt";
    wb = path + "/graph/phones/word_boundary.int";
    mfcc_conf = path + "/conf/mfcc.conf";
    fbank_conf = path + "/conf/fbank.conf";
    cmvn_stats = path + "/am/global_cmvn.stats";
    pitch_conf = path + "/conf/pitch.conf";
  } else if (FileExists(path + "/final.mdl") && FileExists(path + "/mfcc.conf")) {
    // V1 layout: hard-coded options (src/model.cc:132-158)
    std::map<std::string, std::string> kv = {
        {"max-active", "7000"}, {"beam", "13.0"}, {"lattice-beam", "6.0"},
        {"acoustic-scale", "1.0"}, {"frame-subsampling-factor", "3"},
        {"endpoint.silence-phones", "1:2:3:4:5:6:7:8:9:10"},
        {"endpoint.rule2.min-trailing-silence", "0.5"},
        {"endpoint.rule3.min-trailing-silence", "1.0"},
        {"endpoint.rule4.min-trailing-silence", "2.0"}};
    ApplyModelOptions(kv, &dec, &dcb, &endpoint);
    mdl = path + "/final.mdl";
    hclg = path + "/HCLG.fst";
    hcl = path + "/HCLr.fst";
    gr = path + "/Gr.fst";
    disambig_int = path + "/disambig_tid.int";
    words_txt = path + "/words.txt";
    wb = path + "/word_boundary.int";
    mfcc_conf = path + "/mfcc.conf";
    fbank_conf = path + "/fbank.conf";
    cmvn_stats = path + "/global_cmvn.stats";
    pitch_conf = path + "/pitch.conf";
  } else {
    VAMD_ERR("Folder '" << path << "' does not contain model files. Make sure you specified "
                           "the model path properly in Model constructor.");
  }
  VAMD_LOG("Decoding params beam=" << dec.beam << " max-active=" << dec.max_active
                                   << " lattice-beam=" << dec.lattice_beam);
  // front end (src/model.cc:218-228): mfcc.conf, else fbank.conf
  if (FileExists(mfcc_conf)) {
    mfcc.Apply(ReadConfigFile(mfcc_conf));
  } else if (FileExists(fbank_conf)) {
    mfcc.SetFbankDefaults();
    mfcc.Apply(ReadConfigFile(fbank_conf));
  } else {
    VAMD_ERR("Failed to find feature config file");
  }
  mfcc.allow_downsample = true;
  ReadFinalMdl(mdl, &tm, &nnet);
  if (FileExists(path + "/ivector/final.ie")) {
    VAMD_LOG("Loading i-vector extractor from " << path << "/ivector/final.ie");
    ReadIvectorModel(path + "/ivector", &ivec);
    use_ivector = true;
    if (ivec.feat_dim != mfcc.FeatDim())
      VAMD_ERR("i-vector extractor expects " << ivec.feat_dim << "-dim features, the front end gives "
                                             << mfcc.FeatDim());
  }
  if (FileExists(cmvn_stats)) {
    VAMD_LOG("Reading CMVN stats from " << cmvn_stats);
    int rows = 0, cols = 0;
    global_cmvn = ReadKaldiMatrixFile(cmvn_stats, &rows, &cols);
    if (rows != 2 || cols != mfcc.FeatDim() + 1)
      VAMD_ERR("global_cmvn.stats must be 2 x " << mfcc.FeatDim() + 1);
    if (!(global_cmvn[cols - 1] > 0.0)) VAMD_ERR("global_cmvn.stats has no frames");
    use_cmvn = true;
  }
  if (FileExists(pitch_conf))
    VAMD_ERR("pitch front-ends (" << pitch_conf << ") are not supported yet");
  if (FileExists(hclg)) {
    VAMD_LOG("Loading HCLG from " << hclg);
    ReadFstGraph(hclg, &graph);
  } else if (FileExists(hcl) && FileExists(gr)) {
    // src/model.cc:281-285 + src/recognizer.cc:31-37: HCLr o Gr, expanded
    // once into a static graph (graph_compose.h)
    VAMD_LOG("Loading HCL and G from " << hcl << " " << gr);
    auto h = std::make_shared<HostFst>();
    ReadFst(hcl, h.get());
    HostFst g, composed;
    ReadFst(gr, &g);
    {
      std::ifstream in(disambig_int);
      if (!in) VAMD_ERR("cannot open " << disambig_int);
      int d;
      while (in >> d) disambig.push_back(d);
    }
    ComposeLookahead(*h, g, disambig, &composed);
    ToGraph(composed, &graph, hcl + " o " + gr);
    lookahead_hcl = h;
  } else {
    VAMD_ERR("Can't create decoding graph: neither " << hclg << " nor " << hcl << " + " << gr);
  }
  if (!graph.osyms.empty()) {
    for (auto& [id, sym] : graph.osyms) { words.id2sym[id] = sym; words.sym2id[sym] = id; }
  } else {
    VAMD_LOG("Loading words from " << words_txt);
    ReadSymbolTable(words_txt, &words);
  }
  if (FileExists(path + "/rescore/G.carpa")) {
    VAMD_LOG("Loading subtract G.fst model from " << path << "/rescore/G.fst");
    VAMD_LOG("Loading CARPA model from " << path << "/rescore/G.carpa");
    auto r = std::make_shared<RescoreLm>();
    r->Load(path + "/rescore/G.fst", path + "/rescore/G.carpa");
    rescore = r;
  }
  if (FileExists(path + "/rnnlm/final.raw"))
    VAMD_WARN("RNNLM rescoring (rnnlm/) is not supported; final results use the ConstArpa rescoring only");
  has_word_boundary = FileExists(wb);
  int max_phone = 0;
  for (int p : tm.tid2phone) max_phone = std::max(max_phone, p);
  if (has_word_boundary) {
    phone_boundary.assign(max_phone + 1, 0);
    std::ifstream in(wb);
    int ph;
    std::string type;
    static const char* kTypes[] = {"", "nonword", "begin", "end", "internal", "singleton"};
    while (in >> ph >> type) {
      int t = 0;
      for (int i = 1; i <= 5; i++)
        if (type == kTypes[i]) t = i;
      if (t == 0) VAMD_ERR("bad phone type '" << type << "' in " << wb);
      if (ph >= 0 && ph <= max_phone) phone_boundary[ph] = (char)t;
    }
    tid_boundary.assign(tm.tid2phone.size(), 0);
    for (size_t t = 1; t < tm.tid2phone.size(); t++) tid_boundary[t] = phone_boundary[tm.tid2phone[t]];
  }
  phone_is_silence.assign(max_phone + 1, 0);
  for (int p : endpoint.silence_phones)
    if (p >= 0 && p <= max_phone) phone_is_silence[p] = 1;
}

void ModelData::LoadBatchLayout(const std::string& path) {
  // src/batch_model.cc:26-54 reads model/conf/model.conf, model/am/final.mdl,
  // model/graph/HCLG.fst, model/graph/words.txt with batch overrides (:69-88).
  Load(path);
  dec.max_active = 7000;
  dec.beam = 13.0f;
  dec.lattice_beam = 6.0f;
  dcb.acoustic_scale = 1.0f;
  dcb.frame_subsampling_factor = 3;
}

// ---------------------------------------------------------------------------
void* Engine::DevAlloc(size_t bytes) {
  void* p = nullptr;
  const hipError_t err = hipMalloc(&p, std::max<size_t>(bytes, 16));
  if (err != hipSuccess) {
    size_t fr = 0, tot = 0;
    (void)hipMemGetInfo(&fr, &tot);
    VAMD_ERR("device allocation of " << (bytes >> 20) << " MB failed (" << hipGetErrorString(err) << "): this engine holds "
                                     << (dev_bytes_ >> 20) << " MB, " << (fr >> 20) << " MB of " << (tot >> 20)
                                     << " MB free; fewer channels (VOSK_AMD_BATCH_SLOTS) or tokens "
                                        "(max-active) need less");
  }
  dev_allocs_.push_back(p);
  dev_bytes_ += bytes;
  static const bool trace = getenv("VOSK_AMD_MEM_TRACE") != nullptr;  // development: allocations in order
  if (trace && bytes >= (1u << 20))
    fprintf(stderr, "[mem] #%zu %.1f MB (total %.1f MB)\n", dev_allocs_.size() - 1, bytes / 1048576.0,
            dev_bytes_ / 1048576.0);
  return p;
}

template <class T>
T* Engine::Upload(const std::vector<T>& v) {
  T* d = (T*)DevAlloc(sizeof(T) * v.size());
  if (!v.empty()) HIPCHECK(hipMemcpy(d, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice));
  return d;
}

int Engine::NumFramesFor(long long samples) const {
  const int L = md_->mfcc.WindowSize(), S = md_->mfcc.WindowShift();
  if (samples < L) return 0;
  return (int)(1 + (samples - L) / S);
}

// MFCC / fbank tables (float arithmetic as Kaldi MelBanks /
// FeatureWindowFunction / ComputeDctMatrix) for mfcc_kernel.  snip_edges
// false (the speaker front end) starts frame t at t*shift + shift/2 -
// length/2 and reflects samples before the start (Kaldi ExtractWindow).
MfccTables BuildMfccTables(const MfccOptions& o) {
  MfccTables t;
  if (o.htk_compat) VAMD_ERR("htk-compat is not supported");
  const int L = o.WindowSize(), N = o.PaddedWindowSize();
  if (N > 512 || (N & (N - 1))) VAMD_ERR("FFT size " << N << " unsupported (power of two <= 512)");
  if (o.num_bins > 64 || o.num_ceps > 64) VAMD_ERR("num-mel-bins / num-ceps must be <= 64");
  std::vector<float> win(L);
  double a = 2.0 * M_PI / (L - 1);
  for (int i = 0; i < L; i++) {
    double c = cos(a * i), w;
    if (o.window_type == "povey") w = pow(0.5 - 0.5 * c, 0.85);
    else if (o.window_type == "hamming") w = 0.54 - 0.46 * c;
    else if (o.window_type == "hanning") w = 0.5 - 0.5 * c;
    else if (o.window_type == "rectangular") w = 1.0;
    else if (o.window_type == "blackman")
      w = o.blackman_coeff - 0.5 * c + (0.5 - o.blackman_coeff) * cos(2 * a * i);
    else VAMD_ERR("unsupported window type " << o.window_type);
    win[i] = (float)w;
  }
  const int nfft = N / 2, nb = o.num_bins, nc = o.num_ceps;
  std::vector<float> melw((size_t)nb * nfft, 0.0f);
  std::vector<int> first(nb, -1), last(nb, -1);
  float nyq = 0.5f * o.samp_freq;
  float hi = o.high_freq > 0.0f ? o.high_freq : nyq + o.high_freq;
  float width = o.samp_freq / (float)N;
  float ml = MelScale(o.low_freq), mh = MelScale(hi);
  float delta = (mh - ml) / (float)(nb + 1);
  for (int b = 0; b < nb; b++) {
    float left = ml + (float)b * delta, center = ml + (float)(b + 1) * delta,
          right = ml + (float)(b + 2) * delta;
    for (int i = 0; i < nfft; i++) {
      float mel = MelScale(width * (float)i);
      if (mel > left && mel < right) {
        float w = mel <= center ? (mel - left) / (center - left) : (right - mel) / (right - center);
        melw[(size_t)b * nfft + i] = w;
        if (first[b] < 0) first[b] = i;
        last[b] = i;
      }
    }
  }
  std::vector<float> dct((size_t)nc * nb);
  float norm0 = (float)sqrt(1.0 / (double)nb), norm = (float)sqrt(2.0 / (double)nb);
  for (int j = 0; j < nb; j++) dct[j] = norm0;
  for (int k = 1; k < nc; k++)
    for (int j = 0; j < nb; j++) dct[(size_t)k * nb + j] = (float)((double)norm * cos(M_PI / nb * (j + 0.5) * k));
  std::vector<float> lift(nc);
  for (int i = 0; i < nc; i++) {
    double q = o.cepstral_lifter;
    lift[i] = q != 0.0 ? (float)(1.0 + 0.5 * q * sin(M_PI * i / q)) : 1.0f;
  }
  std::vector<float> twr(N / 2), twi(N / 2);
  for (int k = 0; k < N / 2; k++) {
    twr[k] = (float)cos(2.0 * M_PI * k / N);
    twi[k] = (float)(-sin(2.0 * M_PI * k / N));
  }
  int log2n = 0;
  while ((1 << log2n) < N) log2n++;
  t.dev.frame_length = L;
  t.dev.frame_shift = o.WindowShift();
  t.dev.first_offset = o.snip_edges ? 0 : o.WindowShift() / 2 - L / 2;
  t.dev.padded = N;
  t.dev.log2n = log2n;
  t.dev.num_bins = nb;
  t.dev.num_ceps = nc;
  t.dev.nfft = nfft;
  t.dev.use_energy = o.use_energy ? 1 : 0;
  t.dev.remove_dc = o.remove_dc_offset ? 1 : 0;
  t.dev.preemph = o.preemph_coeff;
  t.dev.fbank = o.fbank ? 1 : 0;
  t.dev.use_log_fbank = o.use_log_fbank ? 1 : 0;
  t.dev.use_power = o.use_power ? 1 : 0;
  t.dev.feat_dim = o.FeatDim();
  t.win = std::move(win); t.melw = std::move(melw); t.first = std::move(first); t.last = std::move(last);
  t.dct = std::move(dct); t.lift = std::move(lift); t.twr = std::move(twr); t.twi = std::move(twi);
  return t;
}

Engine::Engine(std::shared_ptr<const ModelData> md, const EngineConfig& cfg) : md_(md), cfg_(cfg) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    VAMD_ERR("no HIP device available: the MI355X engine requires a GPU (there is no CPU fallback)");
  HIPCHECK(hipSetDevice(cfg_.device));
  HIPCHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  // an engine that does not pipeline runs its stages in order on one stream:
  // the HIP runtime hands streams hardware queues in turn (GPU_MAX_HW_QUEUES,
  // 4 by default), so every stream an engine creates but does not need makes
  // another engine's work share a queue with it (and wait behind it)
  if (cfg_.pipeline) {
    HIPCHECK(hipStreamCreateWithFlags(&dstream_, hipStreamNonBlocking));
    HIPCHECK(hipStreamCreateWithFlags(&fstream_, hipStreamNonBlocking));
  } else {
    dstream_ = fstream_ = stream_;
  }
  // a recognizer engine's record reads (CopySegmentTail from the lattice
  // workers) get a queue of their own, next to the engine's: two engines
  // take the 4 hardware queues without sharing (per-thread streams would be
  // handed queues the engines' passes hold)
  if (cfg_.host_lattice) HIPCHECK(hipStreamCreateWithFlags(&copy_stream_, hipStreamNonBlocking));
  const ModelData& m = *md_;
  const int fss = m.dcb.frame_subsampling_factor;
  int fpc = cfg_.frames_per_chunk;
  if (fpc % fss) fpc += fss - fpc % fss;  // GetChunkSize rounding [K]
  cfg_.frames_per_chunk = fpc;
  plan_ = BuildNnetPlan(m.nnet, fpc, fss, m.dcb.acoustic_scale);
  if (LogLevel() > 0) VAMD_LOG(plan_.Describe());
  for (int pdf : m.tm.tid2pdf)
    if (pdf >= plan_.out_dim) VAMD_ERR("transition model pdf " << pdf << " >= nnet output dim");

  // ---- MFCC tables (float arithmetic as Kaldi MelBanks / FeatureWindowFunction)
  const MfccOptions& o = m.mfcc;
  if (o.dither != 0.0f)
    VAMD_WARN("dither=" << o.dither << " ignored: the pipeline is deterministic (dither 0)");
  if (o.htk_compat || !o.snip_edges) VAMD_ERR("htk-compat / snip-edges=false are not supported");
  const int L = o.WindowSize();
  if (plan_.input_dim != o.FeatDim())
    VAMD_ERR("nnet input dim " << plan_.input_dim << " != feature dim " << o.FeatDim());
  {
    MfccTables t = BuildMfccTables(o);
    mfcc_ = t.dev;
    mfcc_.window = Upload(t.win);
    mfcc_.melw = Upload(t.melw);
    mfcc_.mel_first = Upload(t.first);
    mfcc_.mel_last = Upload(t.last);
    mfcc_.dct = Upload(t.dct);
    mfcc_.lifter = Upload(t.lift);
    mfcc_.twr = Upload(t.twr);
    mfcc_.twi = Upload(t.twi);
  }

  // ---- rings
  jobs_per_slot_ = plan_.priming_chunks + 2;
  const int step_frames = cfg_.max_step_samples / o.WindowShift() + 2;
  ring_ = std::max(512, plan_.RingFrames(jobs_per_slot_));
  // the pipelined front end runs one step ahead of the nnet
  ring_ = std::max(ring_, Pow2AtLeast((long long)jobs_per_slot_ * fpc + plan_.left_context +
                                      plan_.right_context + 2 * step_frames + fpc + 16));
  sample_ring_ = Pow2AtLeast((long long)cfg_.max_step_samples + 2 * L + o.WindowShift() + 64);
  const int S = cfg_.max_slots;
  std::vector<float*> ring_ptrs(plan_.nodes.size());
  std::vector<int> ring_dims(plan_.nodes.size());
  for (size_t i = 0; i < plan_.nodes.size(); i++) {
    size_t bytes = sizeof(float) * (size_t)S * ring_ * plan_.nodes[i].dim;
    ring_ptrs[i] = (float*)DevAlloc(bytes);
    HIPCHECK(hipMemset(ring_ptrs[i], 0, bytes));
    ring_dims[i] = plan_.nodes[i].dim;
  }
  d_ring_ptrs_ = Upload(ring_ptrs);
  d_ring_dims_ = Upload(ring_dims);
  rings_.base = d_ring_ptrs_;
  rings_.dim = d_ring_dims_;
  rings_.mask = ring_ - 1;
  rings_.ring = ring_;
  rings_.slots = S;
  rings_.input_node = plan_.input_node;
  // features: MFCC/fbank straight into the nnet input ring, or (global CMVN)
  // into a raw ring that the CMVN kernel normalizes into the input ring
  const int FD = o.FeatDim();
  float* feat_src = ring_ptrs[plan_.input_node];
  if (m.use_cmvn) {
    feat_src = (float*)DevAlloc(sizeof(float) * (size_t)S * ring_ * FD);
    HIPCHECK(hipMemset(feat_src, 0, sizeof(float) * (size_t)S * ring_ * FD));
    if (FD > kCmvnMaxD) VAMD_ERR("CMVN feature dim must be <= " << kCmvnMaxD);
    ncmvn_ = CmvnDev{FD, 600, 200, 0, Upload(m.global_cmvn),
                     (double*)DevAlloc(sizeof(double) * (size_t)S * FD),
                     (float*)DevAlloc(sizeof(float) * (size_t)S * kCmvnHist * FD),
                     feat_src, ring_ptrs[plan_.input_node], ring_ - 1, S};
  }
  mfcc_.out = feat_src;
  d_samples_ = (float*)DevAlloc(sizeof(float) * (size_t)S * sample_ring_);
  // raw input ring for resampled streams: up to 6x the model rate per step
  raw_ring_ = Pow2AtLeast((long long)cfg_.max_step_samples * 6 + 8192);
  max_raw_step_ = raw_ring_ - 8192;
  d_raw_ = (float*)DevAlloc(sizeof(float) * (size_t)S * raw_ring_);
  d_res_tables_ = (ResampleDev*)DevAlloc(sizeof(ResampleDev) * kMaxResampleTables);

  // ---- i-vector extractor (src/model.cc:247-263; OnlineIvectorFeature)
  use_iv_ = plan_.ivector_node >= 0;
  if (use_iv_) {
    if (!m.use_ivector) VAMD_ERR("the nnet has an i-vector input but the model has no ivector/ extractor");
    const IvectorModel& iv = m.ivec;
    const int Si = iv.ivec_dim, QS = Si * (Si + 1) / 2;
    if (Si != plan_.ivector_dim)
      VAMD_ERR("i-vector dim " << Si << " != nnet i-vector input dim " << plan_.ivector_dim);
    if (iv.feat_dim != plan_.input_dim) VAMD_ERR("i-vector feature dim != nnet input dim");
    if (Si > kIvMaxS || QS > kIvMaxQ || iv.feat_dim > kIvMaxD || iv.lda_dim > kIvMaxD ||
        (iv.left + iv.right + 1) * iv.feat_dim > kIvMaxK || iv.num_gauss > kIvMaxG ||
        iv.num_gselect > 5 || iv.num_gselect < 1 || iv.cmn_window >= kCmvnHist || iv.cmn_window < 16 ||
        iv.left < 0 || iv.right < 0)
      VAMD_ERR("i-vector extractor dimensions exceed the kernel limits");
    IvectorDev& d = iv_.m;
    d.feat_dim = iv.feat_dim; d.left = iv.left; d.right = iv.right;
    d.lda_dim = iv.lda_dim; d.lda_cols = iv.lda.cols; d.num_gauss = iv.num_gauss;
    d.ivec_dim = Si; d.cmn_window = iv.cmn_window; d.global_frames = iv.global_frames;
    d.num_gselect = iv.num_gselect; d.num_cg_iters = iv.num_cg_iters;
    d.min_post = iv.min_post; d.posterior_scale = iv.posterior_scale;
    d.log_min_post = iv.log_min_post;
    d.prior_offset = iv.prior_offset; d.max_count = iv.max_count;
    d.cmvn = Upload(iv.cmvn);
    d.sigma_inv_m = Upload(iv.sigma_inv_m);
    d.U = Upload(iv.U);
    const int D = iv.feat_dim, DL = iv.lda_dim, G = iv.num_gauss;
    const int ctx = iv.left + iv.right + 1, K = ctx * D;
    iv_.state = (IvState*)DevAlloc(sizeof(IvState) * S);
    HIPCHECK(hipMemset(iv_.state, 0, sizeof(IvState) * S));
    iv_.quad = (double*)DevAlloc(sizeof(double) * (size_t)S * QS);
    iv_.qfull = (double*)DevAlloc(sizeof(double) * (size_t)S * Si * Si);
    if (D > kCmvnMaxD) VAMD_ERR("i-vector feature dim must be <= " << kCmvnMaxD);
    // CMVN-normalized features and the UBM input [x | x*x] live in rings laid
    // out like the activation rings, so the nnet GEMM kernels read them with
    // the splice as input segments (clamped like the feature input)
    iv_.norm = (float*)DevAlloc(sizeof(float) * (size_t)S * ring_ * D);
    float* ivx = (float*)DevAlloc(sizeof(float) * (size_t)S * ring_ * 2 * DL);
    iv_.in_base = feat_src;  // the raw front-end features (before any global CMVN)
    ivcmvn_ = CmvnDev{D, iv.cmn_window, iv.global_frames, 0, Upload(iv.cmvn),
                      (double*)DevAlloc(sizeof(double) * (size_t)S * D),
                      (float*)DevAlloc(sizeof(float) * (size_t)S * kCmvnHist * D),
                      feat_src, iv_.norm, ring_ - 1, S};
    iv_.in_mask = ring_ - 1;
    iv_.slots = S;
    // frame records of one step: per stream at most the chunks' new frames
    max_iv_frames_ = S * (jobs_per_slot_ * fpc + plan_.right_context + 8);
    max_iv_rows_ = (max_iv_frames_ / kIvFrameBlock + 2 * S) * kIvFrameBlock;
    // silence-weighted entries (single-stream recognizers) get rows after the
    // GEMM rows; their frames' records come from the per-stream history ring
    max_iv_ents_ = std::max(16384, 4 * max_iv_frames_);
    const size_t all_rows = (size_t)max_iv_rows_ + max_iv_ents_;
    iv_.frames = (IvFrame*)DevAlloc(sizeof(IvFrame) * all_rows);
    float* xraw = (float*)DevAlloc(sizeof(float) * all_rows * DL);
    d_iv_ll_ = (float*)DevAlloc(sizeof(float) * (size_t)max_iv_rows_ * G);
    iv_.xraw = xraw;
    iv_.snap = (double*)DevAlloc(sizeof(double) * (size_t)S * jobs_per_slot_ * (QS + Si));
    iv_.snap_nfr = (double*)DevAlloc(sizeof(double) * (size_t)S * jobs_per_slot_);
    iv_.ring = (IvFrame*)DevAlloc(sizeof(IvFrame) * (size_t)S * kIvRing);
    iv_.ring_x = (float*)DevAlloc(sizeof(float) * (size_t)S * kIvRing * DL);
    iv_.ent_row0 = max_iv_rows_;
    for (int i = 0; i < 2; i++) {
      d_ivec_buf_[i] = (float*)DevAlloc(sizeof(float) * (size_t)S * jobs_per_slot_ * Si);
      HIPCHECK(hipMemset(d_ivec_buf_[i], 0, sizeof(float) * (size_t)S * jobs_per_slot_ * Si));
    }
    iv_.ivec = d_ivec_buf_[0];
    // GEMM ops over blocks of kIvFrameBlock frames (DevJob: slot, first frame,
    // splice clamp), canonical order as oracle.c canon_dot
    std::vector<int> pat(kIvFrameBlock);
    for (int i = 0; i < kIvFrameBlock; i++) pat[i] = i;
    const int* d_pat = Upload(pat);
    std::vector<float> wl((size_t)DL * K), bl(DL, 0.0f);
    for (int r = 0; r < DL; r++) {
      for (int j = 0; j < K; j++) wl[(size_t)r * K + j] = iv.lda.row(r)[j];
      if (iv.lda.cols == K + 1) bl[r] = iv.lda.row(r)[K];
    }
    auto base_op = [&](int N, int Kk, const std::vector<float>& W) {
      NnetOpArgs o;
      memset(&o, 0, sizeof(o));
      o.N = N;
      o.K = Kk;
      o.P = kIvFrameBlock;
      o.pattern = d_pat;
      o.W = Upload(W);
      o.rings = rings_;
      o.kslices = GemmKSlices(Kk);
      o.out_node = -1;
      return o;
    };
    auto splice = [&](NnetOpArgs& o, const float* ring) {
      o.nsegs = ctx;
      for (int c = 0; c < ctx; c++) o.segs[c] = DevSeg{ring, D, 1, c - iv.left, c * D, D, 0};
    };
    // (0) normalized frames -> [x | x*x] ring: LDA rows twice, squared right half
    {
      std::vector<float> w2(wl);
      w2.insert(w2.end(), wl.begin(), wl.end());
      std::vector<float> b2(bl);
      b2.insert(b2.end(), bl.begin(), bl.end());
      NnetOpArgs o = base_op(2 * DL, K, w2);
      splice(o, iv_.norm);
      o.nstages = 2;
      o.stages[0] = DevStage{nullptr, Upload(b2), nullptr, 0, 0, 0, 0, 0, 0, 1.0f};
      o.stages[1] = DevStage{nullptr, nullptr, nullptr, 5, 0, 0, 0, DL, 0, 1.0f};
      o.out_node = 0;
      o.out_base = ivx;
      o.out_ldim = 2 * DL;
      iv_ops_.push_back(o);
    }
    // (1) raw frames -> x_raw rows
    {
      NnetOpArgs o = base_op(DL, K, wl);
      splice(o, iv_.in_base);
      o.nstages = 1;
      o.stages[0] = DevStage{nullptr, Upload(bl), nullptr, 0, 0, 0, 0, 0, 0, 1.0f};
      o.llh = xraw;
      iv_ops_.push_back(o);
    }
    // (2) UBM log-likelihoods: [means_invvars | -0.5 inv_vars] . [x | x*x] + gconst
    {
      std::vector<float> wu((size_t)G * 2 * DL);
      for (int g = 0; g < G; g++)
        for (int e = 0; e < DL; e++) {
          wu[(size_t)g * 2 * DL + e] = iv.means_invvars[(size_t)g * DL + e];
          wu[(size_t)g * 2 * DL + DL + e] = -0.5f * iv.inv_vars[(size_t)g * DL + e];
        }
      NnetOpArgs o = base_op(G, 2 * DL, wu);
      o.nsegs = 1;
      o.segs[0] = DevSeg{ivx, 2 * DL, 0, 0, 0, 2 * DL, 0};
      o.nstages = 1;
      o.stages[0] = DevStage{nullptr, Upload(iv.gconsts), nullptr, 0, 0, 0, 0, 0, 0, 1.0f};
      o.llh = d_iv_ll_;
      iv_ops_.push_back(o);
    }
    for (auto& o : iv_ops_) {
      int bk = 64;
      for (int i = 0; i < o.nsegs; i++)
        while (bk > 8 && (o.segs[i].col0 % bk || o.segs[i].dim % bk)) bk >>= 1;
      for (int i = 0; i < o.nsegs; i++)
        if (o.segs[i].col0 % 8 || o.segs[i].dim % 8)
          VAMD_ERR("i-vector feature dims must be multiples of 8 for the GEMM kernels");
      if (o.kslices != 1 && !GemmStreamable(o)) VAMD_ERR("i-vector GEMM shape unsupported");
      iv_op_bk_.push_back(bk);
    }
  } else if (m.use_ivector) {
    VAMD_WARN("ivector/ extractor present but the nnet has no i-vector input: not used");
  }

  // ---- nnet ops
  std::vector<float*> vec_ptrs;
  for (auto& v : plan_.vecs) vec_ptrs.push_back(Upload(v));
  const float* const* d_vecs = Upload(vec_ptrs);
  auto is_in = [&](int node) { return node == plan_.input_node ? 1 : 0; };
  for (auto& op : plan_.ops) {
    NnetOpArgs a;
    memset(&a, 0, sizeof(a));
    a.N = op.N;
    a.K = op.K;
    a.P = (int)op.pattern.size();
    a.pattern = Upload(op.pattern);
    a.rings = rings_;
    a.vecs = d_vecs;
    a.out_node = op.out_node;
    a.out_base = op.out_node >= 0 ? ring_ptrs[op.out_node] : nullptr;
    a.out_ldim = op.out_node >= 0 ? ring_dims[op.out_node] : 0;
    int bk = 64;
    if (op.kind == Op::GEMM) {
      a.W = Upload(plan_.mats[op.weight].data);
      if ((int)op.segs.size() > kMaxSegs) VAMD_ERR("too many input segments in op " << op.name);
      a.nsegs = (int)op.segs.size();
      for (size_t i = 0; i < op.segs.size(); i++) {
        const ASegment& s = op.segs[i];
        a.segs[i] = DevSeg{ring_ptrs[s.node], ring_dims[s.node], is_in(s.node), s.offset, s.col0,
                           s.dim, s.src_col};
        if (s.dim % 4 || s.src_col % 4 || plan_.nodes[s.node].dim % 4)
          VAMD_ERR("op " << op.name << ": segment dims must be multiples of 4");
        while (bk > 8 && (s.col0 % bk || s.dim % bk)) bk >>= 1;
        if (s.col0 % bk || s.dim % bk) VAMD_ERR("op " << op.name << ": K segments must be multiples of 8");
      }
      if (op.K % 4) VAMD_ERR("op " << op.name << ": K must be a multiple of 4");
      a.kslices = GemmKSlices(op.K);
      if (op.K % 8) VAMD_ERR("op " << op.name << ": K must be a multiple of 8");
      if (a.kslices > 1 && !GemmStreamable(a))
        VAMD_ERR("op " << op.name << ": split-K op must fit the streaming GEMM kernel");
    } else {
      a.nparts = (int)op.parts.size();
      if (a.nparts > kMaxParts) VAMD_ERR("too many descriptor parts in op " << op.name);
      int ni = 0;
      for (size_t i = 0; i < op.parts.size(); i++) {
        const GPart& gp = op.parts[i];
        a.parts[i] = DevPart{gp.col0, gp.dim, ni, (int)gp.prog.size()};
        for (auto& g : gp.prog) {
          if (ni >= kMaxInstr) VAMD_ERR("descriptor program too long in op " << op.name);
          if (g.op == GInstr::PUSH_JOB)  // the step's per-job i-vector rows (buffer set per step)
            a.instr[ni++] = DevInstr{d_ivec_buf_[0], g.op, plan_.ivector_dim, 0, 0, g.src_col, g.c};
          else
            a.instr[ni++] = DevInstr{g.op == GInstr::PUSH ? ring_ptrs[g.node] : nullptr, g.op,
                                     g.op == GInstr::PUSH ? ring_dims[g.node] : 0,
                                     g.op == GInstr::PUSH ? is_in(g.node) : 0, g.offset,
                                     g.src_col, g.c};
        }
      }
    }
    if ((int)op.epi.size() > kMaxStages) VAMD_ERR("too many fused stages in op " << op.name);
    a.nstages = (int)op.epi.size();
    for (size_t i = 0; i < op.epi.size(); i++) {
      const EpiStage& e = op.epi[i];
      DevStage d;
      d.base = e.kind == EpiStage::ADD_NODE ? ring_ptrs[e.node] : nullptr;
      d.v0 = e.vec0 >= 0 ? vec_ptrs[e.vec0] : nullptr;
      d.v1 = e.vec1 >= 0 ? vec_ptrs[e.vec1] : nullptr;
      d.kind = e.kind;
      d.ldim = e.kind == EpiStage::ADD_NODE ? ring_dims[e.node] : 0;
      d.is_input = e.kind == EpiStage::ADD_NODE ? is_in(e.node) : 0;
      d.offset = e.offset;
      d.src_col = e.src_col;
      d.scaled = e.scaled ? 1 : 0;
      d.c = e.c;
      a.stages[i] = d;
    }
    op_args_.push_back(a);
    op_bk_.push_back(bk);
  }

  // ---- graph: per state {arc_begin, eps_begin, arc_end, final bits}; per arc
  // {nextstate, weight bits, pdf (-1 for epsilon), ilabel}
  const Graph& g = m.graph;
  if (g.NumArcs() >= INT_MAX) VAMD_ERR("graph too large for 32-bit arc indices");
  {
    std::vector<int4> sinfo(g.NumStates());
    for (int s = 0; s < g.NumStates(); s++) {
      float fc = g.final_cost[s];
      int fb;
      memcpy(&fb, &fc, 4);
      sinfo[s] = make_int4((int)g.arc_begin[s], (int)g.eps_begin[s], (int)g.arc_begin[s + 1], fb);
    }
    std::vector<int4> arcs(g.NumArcs());
    for (int s = 0; s < g.NumStates(); s++)
      for (int64_t a = g.arc_begin[s]; a < g.arc_begin[s + 1]; a++) {
        int wb;
        memcpy(&wb, &g.weight[a], 4);
        int il = g.ilabel[a];
        int pdf = -1;
        if (il != 0) {
          if (il <= 0 || il >= (int)m.tm.tid2pdf.size()) VAMD_ERR("graph ilabel " << il << " is not a transition id");
          pdf = m.tm.tid2pdf[il];
        }
        const int d = g.nextstate[a];
        const bool dest_eps = g.eps_begin[d] < g.arc_begin[d + 1];
        arcs[a] = make_int4(d, wb, pdf, (int)((unsigned)s | (dest_eps ? 0x80000000u : 0u)));
      }
    d_sinfo_ = Upload(sinfo);
    d_arcs_ = Upload(arcs);
    // endpoint probes: per arc epsilon / silence-phone / other (ProbeEndpoints)
    if (!m.phone_is_silence.empty()) {
      std::vector<unsigned char> cls(g.NumArcs());
      for (int64_t a = 0; a < g.NumArcs(); a++) {
        const int il = g.ilabel[a];
        if (il == 0) { cls[a] = 0; continue; }
        const int ph = m.tm.tid2phone[il];
        cls[a] = ph < (int)m.phone_is_silence.size() && m.phone_is_silence[ph] ? 1 : 2;
      }
      d_arc_sil_ = Upload(cls);
    }
  }

  // ---- decoder state
  const long long NS = g.NumStates();
  max_jobs_ = S * jobs_per_slot_;
  max_dec_frames_ = max_jobs_ * plan_.opc;
  for (int i = 0; i < 2; i++)
    d_llh_buf_[i] = (float*)DevAlloc(sizeof(float) * (size_t)max_jobs_ * plan_.opc * plan_.out_dim);
  d_llh_ = d_llh_buf_[0];
  dec_.sinfo = d_sinfo_;
  dec_.arcs = d_arcs_;
  dec_.num_states = (int)NS;
  dec_.start_state = g.start;
  dec_.beam = m.dec.beam;
  dec_.beam_delta = m.dec.beam_delta;
  dec_.max_active = m.dec.max_active;
  dec_.min_active = m.dec.min_active;
  dec_.P = plan_.out_dim;
  dec_.llh = d_llh_;
  // bounded per-stream decoder state (decoder.hip): one HBM frame table of
  // H >= 2 * max_tokens slots for the states a frame's LDS table cannot hold
  if (const char* mt = getenv("VOSK_AMD_DEC_MAX_TOKENS")) cfg_.max_tokens = std::max(64, atoi(mt));  // tests
  const long long MT = cfg_.max_tokens;
  int hbits = 10;
  while ((1ll << hbits) < 2 * MT) hbits++;
  const long long H = 1ll << hbits;
  dec_.hbits = hbits;
  dec_.hprobe = 256;
  dec_.ht_state = (int*)DevAlloc(sizeof(int) * S * H);
  dec_.ht_key = (unsigned long long*)DevAlloc(sizeof(unsigned long long) * S * H);
  dec_.ht_pos = (int*)DevAlloc(sizeof(int) * S * H);
  dec_.ht_stamp = (int*)DevAlloc(sizeof(int) * S * H);
  dec_.ht_bp = (int*)DevAlloc(sizeof(int) * S * H);
  // backpointers and positions are written before they are read in a frame;
  // zeroed so that a slot never holds another engine's data
  HIPCHECK(hipMemset(dec_.ht_pos, 0, sizeof(int) * S * H));
  HIPCHECK(hipMemset(dec_.ht_bp, 0, sizeof(int) * S * H));
  dec_.ht_list = (int*)DevAlloc(sizeof(int) * S * MT);
  dec_.front_g = (int*)DevAlloc(sizeof(int) * 2 * S * MT);
  dec_.cur_state = (int*)DevAlloc(sizeof(int) * S * MT);
  dec_.cur_cost = (float*)DevAlloc(sizeof(float) * S * MT);
  dec_.cur_pos = (int*)DevAlloc(sizeof(int) * S * MT);
  dec_.arena = (int4*)DevAlloc(sizeof(int4) * S * cfg_.arena_tokens);
  // PruneActiveTokens state: extra cost per arena token + compaction scratch
  dec_.extra = (float*)DevAlloc(sizeof(float) * S * cfg_.arena_tokens);
  dec_.remap = (int*)DevAlloc(sizeof(int) * S * cfg_.arena_tokens);
  dec_.max_tok = (int)MT;
  // LDS probe limit of the frame table (decoder.hip); tests force the HBM
  // tables with VOSK_AMD_DEC_LDS_PROBE (0 = every state in HBM)
  dec_.lds_probe = DecoderLdsProbe();
  if (const char* lp = getenv("VOSK_AMD_DEC_LDS_PROBE")) dec_.lds_probe = atoi(lp);
  dec_.lattice_beam = m.dec.lattice_beam;
  // Kaldi prunes every prune_interval (25) frames; VOSK_AMD_DEC_PRUNE=0 turns
  // pruning off (tests that compare the raw per-frame lattice with the oracle)
  dec_.prune_interval = m.dec.prune_interval;
  // By default the passes start once the segment is 300 frames (9 s) long,
  // or earlier if the stream's token or link arena is half full: a pass only
  // bounds memory (the lattice a result is built from is the same with or
  // without it), so a shorter segment runs none (its lattice
  // is pruned once, by the segment's final prune; +3-5 % on the bench's API
  // line) and a longer one pays one walk over its first 300 frames, then
  // Kaldi's interval.  VOSK_AMD_DEC_PRUNE=1 prunes at every interval from the
  // start (Kaldi's schedule); VOSK_AMD_DEC_PRUNE_START / _FILL set the
  // thresholds.
  dec_.prune_fill_pct = cfg_.prune_fill_pct;
  dec_.prune_start = cfg_.host_lattice ? (1 << 30) : 300;
  if (const char* pe = getenv("VOSK_AMD_DEC_PRUNE")) {
    dec_.prune_interval = atoi(pe) ? m.dec.prune_interval : 0;
    dec_.prune_fill_pct = 0;
    dec_.prune_start = 0;
  }
  if (const char* pf = getenv("VOSK_AMD_DEC_PRUNE_FILL")) dec_.prune_fill_pct = std::max(0, atoi(pf));
  if (const char* ps = getenv("VOSK_AMD_DEC_PRUNE_START")) dec_.prune_start = std::max(0, atoi(ps));
  // a longer interval prunes less often (the lattice-beam prune of a result
  // is exact either way; only the arenas grow between prunes)
  if (const char* pi = getenv("VOSK_AMD_DEC_PRUNE_INTERVAL")) dec_.prune_interval = std::max(0, atoi(pi));
  // re-walk depth below the last pruned frame (Kaldi walks until the extra
  // costs settle; a shallower re-walk only prunes less, the final lattice-beam
  // prune is exact either way)
  dec_.host_gate = cfg_.host_lattice ? 1 : 0;
  dec_.prune_revisit = getenv("VOSK_AMD_DEC_PRUNE_REVISIT") ? atoi(getenv("VOSK_AMD_DEC_PRUNE_REVISIT")) : 5;
  dec_.debug = getenv("VOSK_AMD_DEC_DEBUG") ? atoi(getenv("VOSK_AMD_DEC_DEBUG")) : 0;
  dec_.arena_cap = cfg_.arena_tokens;
  dec_.links = nullptr;
  dec_.link_dst = nullptr;
  dec_.link_cap = cfg_.lattice_links;
  dec_.lat_frame_cap = cfg_.lattice_frames;
  // frame records are kept with or without a lattice (pruning walks them)
  dec_.lat_frames = (LatFrame*)DevAlloc(sizeof(LatFrame) * (size_t)S * cfg_.lattice_frames);
  if (cfg_.lattice) {
    dec_.links = (int4*)DevAlloc(sizeof(int4) * (size_t)S * cfg_.lattice_links);
    dec_.link_dst = (int*)DevAlloc(sizeof(int) * (size_t)S * cfg_.lattice_links);
  }
  d_slots_ = (DecSlot*)DevAlloc(sizeof(DecSlot) * S);
  HIPCHECK(hipMemset(d_slots_, 0, sizeof(DecSlot) * S));
  dec_.slots = d_slots_;
  d_stats_ = (FrameStat*)DevAlloc(sizeof(FrameStat) * max_dec_frames_);
  dec_.stats = cfg_.collect_stats ? d_stats_ : nullptr;
  dec_.prof = nullptr;
  if (getenv("VOSK_AMD_DEC_PROFILE")) {
    dec_.prof = (long long*)DevAlloc(sizeof(long long) * kDecProf * S);
    HIPCHECK(hipMemset(dec_.prof, 0, sizeof(long long) * kDecProf * S));
  }
  LaunchInitTables(dec_.ht_state, dec_.ht_key, dec_.ht_stamp, S * H, stream_);
  // token-passing order: Kaldi's (default) or the
  // order-independent form (VOSK_AMD_DEC_ORDER=parallel)
  dec_.kaldi = cfg_.kaldi_order ? 1 : 0;
  if (const char* o = getenv("VOSK_AMD_DEC_ORDER")) {
    const std::string v(o);
    if (v == "parallel" || v == "0" || v == "order-independent") dec_.kaldi = 0;
    else if (v == "kaldi" || v == "1") dec_.kaldi = 1;
  }
  dec_.kb_cap = (int)(2 * MT + 1024);
  dec_.kord_cap = (int)((MT + 4096 + 3) & ~3LL);  // (a multiple of 4: 16-byte loads of four entries)
  size_t kaldi_bytes = dev_bytes_;
  if (dec_.kaldi) {
    const size_t KB = (size_t)S * dec_.kb_cap, KO = (size_t)S * dec_.kord_cap;
    dec_.kb_first = (int*)DevAlloc(sizeof(int) * KB);
    dec_.kb_cnt = (int*)DevAlloc(sizeof(int) * KB);
    dec_.kb_start = (int*)DevAlloc(sizeof(int) * KB);
    dec_.kb_memb = (int*)DevAlloc(sizeof(int) * kKbMemb * KB);
    dec_.kord = (int*)DevAlloc(sizeof(int) * KO);
    dec_.kbkt = (int*)DevAlloc(sizeof(int) * KO);
    dec_.kstk = (int*)DevAlloc(sizeof(int) * KO);
    dec_.kcost0 = (float*)DevAlloc(sizeof(float) * KO);
    dec_.kmem = (int*)DevAlloc(sizeof(int) * 8 * KO);
    dec_.kadj_cap = 4 * dec_.kord_cap;
    dec_.kadj = (int2*)DevAlloc(sizeof(int2) * (size_t)S * dec_.kadj_cap);
    // OpenFST's lazy numbering of a composed graph:
    // VOSK_AMD_LAZY_IDS=0 buckets by the static graph's ids instead
    const char* le = getenv("VOSK_AMD_LAZY_IDS");
    if (g.lazy_ids > 0 && !(le && atoi(le) == 0)) {
      if ((int64_t)g.lazy_row.size() != (int64_t)NS + 1 || g.lazy_row.back() >= (1LL << 31) ||
          g.lazy_ids >= kLazyExpanded)
        VAMD_ERR("lazy numbering table does not match the graph");
      dec_.lazy_ids = g.lazy_ids;
      dec_.lazy_row = Upload(std::vector<long long>(g.lazy_row.begin(), g.lazy_row.end()));
      dec_.lazy_next = Upload(g.lazy_next);
      dec_.lazy_id = (int*)DevAlloc(sizeof(int) * (size_t)S * g.lazy_ids);
      dec_.lazy_cand = (int*)DevAlloc(sizeof(int) * (size_t)S * g.lazy_ids);
      dec_.lazy_new = (int*)DevAlloc(sizeof(int) * (size_t)S * 3 * kLazyNewCap);
    }
    HIPCHECK(hipMemset(dec_.kb_first, 0x7f, sizeof(int) * KB));  // 0x7f7f7f7f: empty (above any creation index)
    HIPCHECK(hipMemset(dec_.kb_cnt, 0, sizeof(int) * KB));
    // creation order / buckets: valid indices from the start (slot 0, bucket 0)
    HIPCHECK(hipMemset(dec_.kord, 0, sizeof(int) * KO));
    HIPCHECK(hipMemset(dec_.kbkt, 0, sizeof(int) * KO));
    kaldi_bytes = dev_bytes_ - kaldi_bytes;
  } else {
    kaldi_bytes = 0;
    dec_.kb_first = dec_.kb_cnt = dec_.kb_start = dec_.kb_memb = nullptr;
    dec_.kord = dec_.kbkt = dec_.kstk = dec_.kmem = nullptr;
    dec_.kcost0 = nullptr;
    dec_.kadj = nullptr;
    dec_.kadj_cap = 0;
  }
  if (!dec_.lazy_id) {
    dec_.lazy_row = nullptr;
    dec_.lazy_next = nullptr;
    dec_.lazy_cand = dec_.lazy_new = nullptr;
    dec_.lazy_ids = 0;
  }

  // ---- staging
  stage_sample_cap_ = (size_t)S * cfg_.max_step_samples;
  stage_bytes_ = Align256(sizeof(float) * (size_t)S * cfg_.max_step_samples) +
                 2 * Align256(sizeof(SampleJob) * S) + Align256(sizeof(ResampleJob) * S) +
                 Align256(sizeof(MfccJob) * S) +
                 Align256(sizeof(DevJob) * max_jobs_) + Align256(sizeof(DecJob) * S) +
                 Align256(sizeof(IvStreamJob) * S) + Align256(sizeof(IvReq) * max_jobs_) +
                 2 * Align256(sizeof(CmvnJob) * S) +
                 2 * Align256(sizeof(IvFrameBlock) * ((size_t)max_iv_frames_ / kIvFrameBlock + 2 * S)) +
                 Align256(sizeof(IvEntry) * (size_t)max_iv_ents_) +
                 Align256(sizeof(IvBatch) * ((size_t)max_jobs_ + max_iv_ents_)) + 1024;
  // three buffers: the pipelined nnet and decoder passes keep their jobs
  // while the next step stages
  HIPCHECK(hipHostMalloc((void**)&h_stage_, 3 * stage_bytes_, hipHostMallocDefault));
  d_stage_ = (char*)DevAlloc(3 * stage_bytes_);
  HIPCHECK(hipHostMalloc((void**)&h_slots_, sizeof(DecSlot) * S, hipHostMallocDefault));
  HIPCHECK(hipHostMalloc((void**)&h_stats_, sizeof(FrameStat) * max_dec_frames_, hipHostMallocDefault));
  for (auto& ev : ev_) HIPCHECK(hipEventCreate(&ev));
  // the segment copies' pinned pool starts with one block (128 KB per
  // channel, at most 128 MB): pinning host memory when the first segments end
  // costs ~5 ms per 20 MB on the lane thread
  if (cfg_.lattice) {
    const size_t want = std::min<size_t>((size_t)S << 17, (size_t)128 << 20);
    char* blk = nullptr;
    HIPCHECK(hipHostMalloc((void**)&blk, want, hipHostMallocDefault));
    pinned_->Give(blk, want);
    // and the rest of StartSegmentCopies' buffers: allocated on the lane
    // thread, they were ~10 ms of the first segments' tail (a recognizer
    // engine created its copy stream beside its main stream, above)
    if (!copy_stream_) HIPCHECK(hipStreamCreateWithFlags(&copy_stream_, hipStreamNonBlocking));
    HIPCHECK(hipEventCreateWithFlags(&copy_ev_, hipEventDisableTiming));
    HIPCHECK(hipHostMalloc((void**)&h_copy_slots_, sizeof(DecSlot) * S, hipHostMallocDefault));
    d_prune_slots_ = (int*)DevAlloc(sizeof(int) * S);
    HIPCHECK(hipHostMalloc((void**)&h_copy_stage_, Align256(sizeof(int) * S) + sizeof(CopyItem) * 3 * S,
                           hipHostMallocDefault));
    pack_cap_ = want;
    HIPCHECK(hipMalloc((void**)&d_pack_, pack_cap_));
    pack_items_cap_ = 3 * (size_t)S + 16;
    HIPCHECK(hipMalloc((void**)&d_pack_items_, sizeof(CopyItem) * pack_items_cap_));
  }
  // the tables above were cleared with null-stream memsets, which the
  // engine's non-blocking streams are not ordered after
  HIPCHECK(hipDeviceSynchronize());
  if (cfg_.lattice && !cfg_.host_lattice) {
    // the segment copies' path run once on an idle slot (frames 0: the
    // prune returns at once): the copy stream's first commands and first
    // launches cost ~9 ms each on the host, paid here instead of in the first
    // segments' tail
    memset(h_copy_stage_, 0, sizeof(int));
    HIPCHECK(hipMemcpyAsync(d_prune_slots_, h_copy_stage_, sizeof(int), hipMemcpyHostToDevice, copy_stream_));
    LaunchPruneFinal(dec_, d_prune_slots_, 1, true, copy_stream_);
    HIPCHECK(hipMemcpyAsync(h_copy_slots_, d_slots_, sizeof(DecSlot) * S, hipMemcpyDeviceToHost, copy_stream_));
    CopyItem* it = (CopyItem*)(h_copy_stage_ + Align256(sizeof(int) * S));
    *it = CopyItem{(const unsigned*)d_slots_, 0, 1};
    HIPCHECK(hipMemcpyAsync(d_pack_items_, it, sizeof(CopyItem), hipMemcpyHostToDevice, copy_stream_));
    LaunchGatherCopy(d_pack_items_, 1, d_pack_, copy_stream_);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipMemcpyAsync(h_copy_slots_, d_pack_, sizeof(unsigned), hipMemcpyDeviceToHost, copy_stream_));
    HIPCHECK(hipStreamSynchronize(copy_stream_));
  }
  slots_.resize(S);
  host_read_.reset(new std::atomic<int>[S]);
  prune_wait_.reset(new std::atomic<char>[S]);
  for (int i = 0; i < S; i++) {
    host_read_[i].store(-1);
    prune_wait_[i].store(0);
  }
  VAMD_LOG("engine: device memory " << (dev_bytes_ >> 20) << " MB (Kaldi-order scratch "
                                    << (kaldi_bytes >> 20) << " MB), slots=" << S << " fpc=" << fpc << " priming=" << plan_.priming_chunks
                            << " ring=" << ring_ << " ops=" << plan_.ops.size()
                            << " graph states=" << NS << " arcs=" << g.NumArcs());
}

Engine::~Engine() {
  if (step_prof_n_ && getenv("VOSK_AMD_STEP_PROFILE"))
    fprintf(stderr, "[engine] steps %lld: build %.3f ms, sync wait %.3f ms, after sync %.3f ms, total %.3f ms per step\n",
            step_prof_n_, step_prof_[0] / step_prof_n_, step_prof_[1] / step_prof_n_, step_prof_[2] / step_prof_n_,
            step_prof_[3] / step_prof_n_);
  if (copy_prof_n_ && getenv("VOSK_AMD_STEP_PROFILE"))
    fprintf(stderr, "[engine] segment copy calls %lld: prune + state read %.3f ms, pinned take %.3f ms, after %.3f ms, %.1f MB (totals over calls)\n",
            copy_prof_n_, copy_prof_[0], copy_prof_[1], copy_prof_[2], copy_prof_[3]);
  (void)hipSetDevice(cfg_.device);
  if (stream_) (void)hipStreamSynchronize(stream_);
  if (dstream_) (void)hipStreamSynchronize(dstream_);
  if (fstream_) (void)hipStreamSynchronize(fstream_);
  for (auto& ev : ev_)
    if (ev) (void)hipEventDestroy(ev);
  for (auto& h : slots_)
    if (h.resident) (void)hipFree(h.resident);
  for (void* p : dev_allocs_) (void)hipFree(p);
  if (h_stage_) (void)hipHostFree(h_stage_);
  if (h_slots_) (void)hipHostFree(h_slots_);
  if (h_stats_) (void)hipHostFree(h_stats_);
  if (h_probe_) (void)hipHostFree(h_probe_);
  if (copy_stream_) (void)hipStreamSynchronize(copy_stream_);
  if (h_lat_stage_) (void)hipHostFree(h_lat_stage_);
  if (h_copy_slots_) (void)hipHostFree(h_copy_slots_);
  if (h_copy_stage_) (void)hipHostFree(h_copy_stage_);
  if (copy_ev_) (void)hipEventDestroy(copy_ev_);
  if (copy_stream_) (void)hipStreamDestroy(copy_stream_);
  if (dstream_ && dstream_ != stream_) (void)hipStreamDestroy(dstream_);
  if (fstream_ && fstream_ != stream_) (void)hipStreamDestroy(fstream_);
  if (stream_) (void)hipStreamDestroy(stream_);
  if (call_stream_) (void)hipStreamSynchronize(call_stream_);
  if (d_bp_) (void)hipFree(d_bp_);
  if (h_bp_) (void)hipHostFree(h_bp_);
  if (d_pack_) (void)hipFree(d_pack_);
  if (d_pack_items_) (void)hipFree(d_pack_items_);
  if (d_call_raw_) (void)hipFree(d_call_raw_);
  if (d_call_out_) (void)hipFree(d_call_out_);
  if (d_call_jobs_) (void)hipFree(d_call_jobs_);
  if (call_stream_) (void)hipStreamDestroy(call_stream_);
}

int Engine::TryAllocSlot() {
  std::lock_guard<std::mutex> lk(mu_);
  for (size_t i = 0; i < slots_.size(); i++)
    if (!slots_[i].used) {
      slots_[i] = SlotHost();
      slots_[i].used = true;
      slots_[i].next_chunk = -plan_.priming_chunks;
      return (int)i;
    }
  return -1;
}

int Engine::AllocSlot() {
  const int s = TryAllocSlot();
  if (s < 0) VAMD_ERR("all " << slots_.size() << " stream slots of the engine are in use");
  return s;
}

void Engine::FreeSlot(int slot) {
  std::lock_guard<std::mutex> lk(mu_);
  DEVICE_GUARD();
  if (SlotInFlight(slot)) FlushLocked();
  slots_.at(slot).used = false;
}

int Engine::SlotsInUse() {
  std::lock_guard<std::mutex> lk(mu_);
  int n = 0;
  for (const SlotHost& h : slots_) n += h.used ? 1 : 0;
  return n;
}

void Engine::ResetPipeline(int slot) {
  std::lock_guard<std::mutex> lk(mu_);
  DEVICE_GUARD();
  if (SlotInFlight(slot)) FlushLocked();
  SlotHost& h = slots_.at(slot);
  h.pending.clear();
  h.pending_pos = 0;
  h.samples = 0;
  h.frames = 0;
  h.next_chunk = -plan_.priming_chunks;
  h.out_ready = 0;
  h.decoded = 0;
  h.finished = false;
  h.need_reset = true;
  h.fresh_decoder = true;
  h.err = 0;
  if (h.resident) (void)hipFree(h.resident);
  h.resident = nullptr;
  h.resident_n = h.resident_pos = 0;
  h.resident_finish = false;
  h.raw_pushed = 0;
  h.res_flushed = false;
  h.iv_reset = true;
  h.cmvn_reset = true;
  h.iv_norm_done = h.iv_norm_to = h.iv_stats_done = 0;
  h.iv_weighted = false;
  h.iv_pending.clear();
  h.sw.Reset();
}

void Engine::ResetDecoder(int slot) {
  std::lock_guard<std::mutex> lk(mu_);
  DEVICE_GUARD();
  if (SlotInFlight(slot)) FlushLocked();
  SlotHost& h = slots_.at(slot);
  h.decoded = 0;
  h.need_reset = true;
  h.sw.Reset();  // a new OnlineSilenceWeighting per decoder segment (src/recognizer.cc:190-191)
}

void Engine::AcceptSamples(int slot, const float* x, int n) {
  std::lock_guard<std::mutex> lk(mu_);
  SlotHost& h = slots_.at(slot);
  if (h.finished) VAMD_ERR("AcceptSamples after InputFinished");
  if (h.pending_pos > 0 && h.pending_pos == h.pending.size()) {
    h.pending.clear();
    h.pending_pos = 0;
  }
  h.pending.insert(h.pending.end(), x, x + n);
}

void Engine::AcceptSamples(int slot, std::vector<float>&& x) {
  std::lock_guard<std::mutex> lk(mu_);
  SlotHost& h = slots_.at(slot);
  if (h.finished) VAMD_ERR("AcceptSamples after InputFinished");
  if (h.pending_pos == h.pending.size()) {
    h.pending.swap(x);
    h.pending_pos = 0;
  } else {
    h.pending.insert(h.pending.end(), x.begin(), x.end());
  }
}

void Engine::StageSamples(const float* x, size_t n) {
  if (st_sample_n_ + n > stage_sample_cap_) VAMD_ERR("step staging overflow (samples)");
  memcpy(st_sample_data_ + st_sample_n_, x, sizeof(float) * n);
  st_sample_n_ += n;
}

void Engine::SetSampleRate(int slot, int rate) {
  std::lock_guard<std::mutex> lk(mu_);
  DEVICE_GUARD();
  SlotHost& h = slots_.at(slot);
  if (h.samples > 0 || h.raw_pushed > 0) VAMD_ERR("SetSampleRate after samples were accepted");
  const int model_rate = (int)std::lround(md_->mfcc.samp_freq);
  if (rate <= 0) VAMD_ERR("bad sample rate " << rate);
  if (rate == model_rate) {
    h.rate = 0;
    h.table = -1;
    return;
  }
  h.rate = rate;
  h.table = ResampleTableLocked(rate);
}

int Engine::ResampleTableLocked(int rate) {
  const int model_rate = (int)std::lround(md_->mfcc.samp_freq);
  int t = -1;
  for (size_t i = 0; i < res_tables_.size(); i++)
    if (res_tables_[i].rate_in == rate) t = (int)i;
  if (t < 0) {
    if ((int)res_tables_.size() >= kMaxResampleTables) VAMD_ERR("too many distinct input sample rates");
    ResampleTable tb = BuildResampleTable(rate, model_rate);
    ResampleDev d;
    d.first = Upload(tb.first);
    d.ntaps = Upload(tb.ntaps);
    d.w = Upload(tb.w);
    d.in_unit = tb.in_unit;
    d.out_unit = tb.out_unit;
    d.taps = tb.taps;
    d.pad = 0;
    t = (int)res_tables_.size();
    HIPCHECK(hipMemcpy(d_res_tables_ + t, &d, sizeof(d), hipMemcpyHostToDevice));
    res_tables_.push_back(std::move(tb));
    VAMD_LOG_VERBOSE("resampling " << rate << " -> " << model_rate << " Hz, " << res_tables_[t].taps
                                   << " taps");
  }
  return t;
}

int Engine::ResampleTableFor(int rate, ResampleTable* copy) {
  std::lock_guard<std::mutex> lk(mu_);
  DEVICE_GUARD();
  const int t = ResampleTableLocked(rate);
  *copy = res_tables_[t];
  return t;
}

std::vector<float> Engine::ResampleCall(int t, const ResampleTable& T, const float* x, int n) {
  const long long n_out = T.NumOutputSamples(n, true);
  std::vector<float> out((size_t)n_out);
  if (n_out == 0) return out;
  std::lock_guard<std::mutex> lk(call_mu_);
  DEVICE_GUARD();
  if (!call_stream_) HIPCHECK(hipStreamCreateWithFlags(&call_stream_, hipStreamNonBlocking));
  // the kernel indexes its input and output as rings (power-of-two lengths)
  auto pow2 = [](long long v) {
    size_t p = 1024;
    while ((long long)p < v) p <<= 1;
    return p;
  };
  const size_t raw_len = pow2(n), out_len = pow2(n_out);
  constexpr int kPer = 2048;  // outputs per workgroup
  const size_t njobs = (size_t)((n_out + kPer - 1) / kPer);
  auto grow = [&](auto** p, size_t* cap, size_t want, size_t elem) {
    if (*cap >= want) return;
    if (*p) HIPCHECK(hipFree(*p));
    HIPCHECK(hipMalloc((void**)p, want * elem));
    *cap = want;
  };
  grow(&d_call_raw_, &call_cap_raw_, raw_len, sizeof(float));
  grow(&d_call_out_, &call_cap_out_, out_len, sizeof(float));
  grow(&d_call_jobs_, &call_cap_jobs_, njobs, sizeof(ResampleJob));
  std::vector<ResampleJob> jobs(njobs);
  for (size_t k = 0; k < njobs; k++) {
    const long long o = (long long)k * kPer;
    jobs[k] = ResampleJob{0, (int)o, (int)std::min<long long>(kPer, n_out - o), t, o, (long long)n};
  }
  HIPCHECK(hipMemcpyAsync(d_call_raw_, x, sizeof(float) * n, hipMemcpyHostToDevice, call_stream_));
  HIPCHECK(hipMemcpyAsync(d_call_jobs_, jobs.data(), sizeof(ResampleJob) * njobs, hipMemcpyHostToDevice,
                          call_stream_));
  LaunchResample(d_call_jobs_, (int)njobs, d_res_tables_, d_call_raw_, (int)raw_len, d_call_out_, (int)out_len,
                 call_stream_);
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipMemcpyAsync(out.data(), d_call_out_, sizeof(float) * n_out, hipMemcpyDeviceToHost, call_stream_));
  HIPCHECK(hipStreamSynchronize(call_stream_));
  return out;
}


void Engine::PreloadSamples(int slot, const float* x, long long n, bool finished) {
  std::lock_guard<std::mutex> lk(mu_);
  DEVICE_GUARD();
  SlotHost& h = slots_.at(slot);
  if (h.resident && h.resident_pos < h.resident_n) VAMD_ERR("previous preloaded audio not consumed");
  if (h.resident) (void)hipFree(h.resident);
  h.resident = nullptr;
  HIPCHECK(hipMalloc((void**)&h.resident, sizeof(float) * std::max<long long>(n, 1)));
  if (n) HIPCHECK(hipMemcpy(h.resident, x, sizeof(float) * n, hipMemcpyHostToDevice));
  h.resident_n = n;
  h.resident_pos = 0;
  h.resident_finish = finished;
}

void Engine::InputFinished(int slot) {
  std::lock_guard<std::mutex> lk(mu_);
  slots_.at(slot).finished = true;
}

int Engine::NumFramesDecoded(int slot) const { return slots_.at(slot).decoded; }
int Engine::NumFramesReady(int slot) const { return slots_.at(slot).out_ready; }
bool Engine::InputIsFinished(int slot) const { return slots_.at(slot).finished; }
int Engine::PendingSamples(int slot) const {
  const SlotHost& h = slots_.at(slot);
  return (int)(h.pending.size() - h.pending_pos);
}
int Engine::DecoderError(int slot) const { return slots_.at(slot).err; }

void Engine::DecoderState(int slot, long long* o8) {
  std::lock_guard<std::mutex> lk(mu_);
  DEVICE_GUARD();
  FlushLocked();
  slots_.at(slot);
  DecSlot st;
  HIPCHECK(hipMemcpy(&st, d_slots_ + slot, sizeof(DecSlot), hipMemcpyDeviceToHost));
  o8[0] = st.ntok;
  o8[1] = st.arena_used;
  o8[2] = st.frames;
  o8[3] = st.links_used;
  o8[4] = st.err;
  o8[5] = st.lat_ovf;
  o8[6] = st.prune_from;
  o8[7] = st.last_prune;
}
const std::vector<FrameStat>& Engine::LastStats(int slot) const { return slots_.at(slot).stats; }

bool Engine::BuildStep(const std::vector<int>& slots) {
  st_samples_.clear();
  st_sample_src_.clear();
  st_sample_data_ = (float*)(h_stage_ + (size_t)(seq_ % 3) * stage_bytes_);  // RunStep's buffer
  st_sample_n_ = 0;
  st_raw_.clear();
  st_raw_src_.clear();
  st_res_.clear();
  st_mfcc_.clear();
  st_mfcc_total_ = 0;
  st_jobs_.clear();
  st_dec_.clear();
  st_iv_jobs_.clear();
  st_iv_reqs_.clear();
  st_iv_blocks_.clear();
  st_iv_devjobs_.clear();
  st_ncmvn_.clear();
  st_ivcmvn_.clear();
  st_iv_frames_ = 0;
  st_iv_ents_.clear();
  st_iv_batches_.clear();
  const int fpc = plan_.fpc, opc = plan_.opc, fss = plan_.fss, R = plan_.right_context;
  int stats_rows = 0;
  bool any = false;
  for (int s : slots) {
    SlotHost& h = slots_.at(s);
    if (!h.used) continue;
    // 1. samples: HBM-resident audio first, then host-fed samples
    if (h.rate != 0) {
      // resampled stream: raw samples -> raw ring, then the outputs their
      // windows complete (all remaining ones at end of input) -> sample ring
      const ResampleTable& T = res_tables_[h.table];
      const bool from_res = h.resident && h.resident_pos < h.resident_n;
      const long long avail = from_res ? h.resident_n - h.resident_pos
                                       : (long long)(h.pending.size() - h.pending_pos);
      long long n = std::min<long long>(avail, max_raw_step_);
      if (!from_res)  // host-fed samples share the step's staging buffer
        n = std::min<long long>(n, (long long)stage_sample_cap_ - (long long)st_sample_n_);
      if (n < 0) n = 0;
      auto ends_after = [&](long long nn) {
        return nn == avail && (from_res ? h.resident_finish : h.finished);
      };
      bool flush = !h.res_flushed && ends_after(n);
      long long tot = T.NumOutputSamples(h.raw_pushed + n, flush);
      while (tot - h.samples > cfg_.max_step_samples && n > 0) {
        n -= std::max<long long>(1, (tot - h.samples - cfg_.max_step_samples) * T.in_unit / T.out_unit + 1);
        if (n < 0) n = 0;
        flush = false;
        tot = T.NumOutputSamples(h.raw_pushed + n, false);
      }
      if (n > 0) {
        const int pos = (int)(h.raw_pushed & (raw_ring_ - 1));
        if (from_res) {
          st_raw_.push_back(SampleJob{s, pos, (int)n, 0, h.resident + h.resident_pos});
          st_raw_src_.push_back(-1);
          h.resident_pos += n;
          if (h.resident_pos == h.resident_n && h.resident_finish) h.finished = true;
        } else {
          st_raw_.push_back(SampleJob{s, pos, (int)n, 0, nullptr});
          st_raw_src_.push_back((int)st_sample_n_);
          StageSamples(h.pending.data() + h.pending_pos, (size_t)n);
          h.pending_pos += n;
        }
        h.raw_pushed += n;
        any = true;
      }
      if (tot > h.samples) {
        st_res_.push_back(ResampleJob{s, (int)(h.samples & (sample_ring_ - 1)), (int)(tot - h.samples),
                                      h.table, h.samples, h.raw_pushed});
        h.samples = tot;
        any = true;
      }
      if (flush) h.res_flushed = true;
    } else if (h.resident && h.resident_pos < h.resident_n) {
      int n = (int)std::min<long long>(h.resident_n - h.resident_pos, cfg_.max_step_samples);
      SampleJob j{s, (int)(h.samples & (sample_ring_ - 1)), n, 0, h.resident + h.resident_pos};
      st_samples_.push_back(j);
      st_sample_src_.push_back(-1);
      h.resident_pos += n;
      h.samples += n;
      if (h.resident_pos == h.resident_n && h.resident_finish) h.finished = true;
      any = true;
    } else {
      int avail = (int)(h.pending.size() - h.pending_pos);
      int n = std::min(avail, cfg_.max_step_samples);
      if (n > 0) {
        st_samples_.push_back(SampleJob{s, (int)(h.samples & (sample_ring_ - 1)), n, 0, nullptr});
        st_sample_src_.push_back((int)st_sample_n_);
        StageSamples(h.pending.data() + h.pending_pos, (size_t)n);
        h.pending_pos += n;
        h.samples += n;
        any = true;
      }
    }
    // 2. MFCC frames
    int nf_total = NumFramesFor(h.samples);
    if (nf_total > h.frames) {
      st_mfcc_.push_back(MfccJob{s, h.frames, nf_total - h.frames, st_mfcc_total_});
      if (md_->use_cmvn) {
        st_ncmvn_.push_back(CmvnJob{s, h.frames, nf_total, h.cmvn_reset ? 1 : 0});
        h.cmvn_reset = false;
      }
      st_mfcc_total_ += nf_total - h.frames;
      h.frames = nf_total;
      any = true;
    }
    // 3. chunk jobs (DecodableNnetLoopedOnline::NumFramesReady semantics)
    const bool fin = h.finished && h.pending_pos == h.pending.size() &&
                     (!h.resident || h.resident_pos == h.resident_n) &&
                     (h.rate == 0 || h.res_flushed);
    const int T = h.frames;
    const int need_out = fin ? (T + fss - 1) / fss : 0;
    int first_real = -1, dec_frames = 0, njobs = 0;
    const int jobs0 = (int)st_jobs_.size(), req0 = (int)st_iv_reqs_.size();
    // with an i-vector input a chunk also waits for the i-vector splice's right
    // context of its last input frame (OnlineIvectorFeature::NumFramesReady)
    const int iv_wait = use_iv_ ? iv_.m.right : 0;
    while (njobs < jobs_per_slot_) {
      const int c = h.next_chunk;
      bool ready;
      if (fin) ready = T > 0 && (c < 0 || c * opc < need_out);
      else ready = T >= (std::max(c, 0) + 1) * fpc + R + iv_wait;
      if (!ready) break;
      if (use_iv_ && c >= 0) {
        // the chunk's i-vector: at its last input frame incl. right context,
        // clamped to the utterance (DecodableNnetLoopedOnline); priming
        // jobs (same step, just before) share chunk 0's
        const int job = (int)st_jobs_.size(), f = std::min((c + 1) * fpc + R, T) - 1;
        IvReq r{f, c == 0 ? jobs0 : job, job + 1, st_iv_frames_, st_iv_frames_, 0, 0, 0};
        if (f >= h.iv_stats_done) {  // new frames: records, then CG (else reuse)
          r.upd = 1;
          const int ivjob = (int)st_iv_jobs_.size();
          const int ring = h.iv_weighted ? s * kIvRing : -1;
          for (int t0 = h.iv_stats_done; t0 <= f; t0 += kIvFrameBlock) {
            const int nf = std::min(kIvFrameBlock, f + 1 - t0);
            // frame records are indexed by GEMM row: kIvFrameBlock per block,
            // rows past the block's frames are empty records (no posteriors)
            st_iv_blocks_.push_back(IvFrameBlock{ivjob, t0, nf, st_iv_frames_, ring, 0, 0, 0});
            st_iv_devjobs_.push_back(DevJob{s, t0, T - 1, 0});
            st_iv_frames_ += kIvFrameBlock;
          }
          r.row_to = st_iv_frames_;
          r.batch0 = (int)st_iv_batches_.size();
          if (!h.iv_weighted) {
            // UpdateStatsUntilFrame: the new frames form one batch
            st_iv_batches_.push_back(IvBatch{r.row_from, r.row_to});
          } else {
            // OnlineIvectorFeature::UpdateStatsUntilFrameWeighted: the queued
            // delta weights of frames <= f, popped in (frame, weight) order;
            // one UpdateStatsForFrames batch at the first new frame (every
            // entry of a frame <= it), then one per later frame
            auto& q = h.iv_pending;
            std::stable_sort(q.begin(), q.end());
            size_t n = 0;
            while (n < q.size() && q[n].first <= f) n++;
            const int done = h.iv_stats_done;
            r.row_from = max_iv_rows_ + (int)st_iv_ents_.size();
            int key = -1;
            for (size_t i = 0; i < n; i++) {
              const int t = q[i].first;
              if (t <= f - kIvRing) VAMD_ERR("silence weight for frame " << t << " left the history ring");
              const int row = max_iv_rows_ + (int)st_iv_ents_.size();
              const int k = std::max(t, done);
              if (k != key) {
                st_iv_batches_.push_back(IvBatch{row, row});
                key = k;
              }
              st_iv_batches_.back().row_to = row + 1;
              st_iv_ents_.push_back(IvEntry{s * kIvRing + t % kIvRing, q[i].second});
            }
            q.erase(q.begin(), q.begin() + n);
            r.row_to = max_iv_rows_ + (int)st_iv_ents_.size();
            if ((int)st_iv_ents_.size() > max_iv_ents_) VAMD_ERR("silence-weighted i-vector entries overflow");
          }
          r.nbatch = (int)st_iv_batches_.size() - r.batch0;
          for (int b = r.batch0; b < (int)st_iv_batches_.size(); b++)
            if (st_iv_batches_[b].row_to - st_iv_batches_[b].row_from > kIvBatchRows)
              VAMD_ERR("i-vector statistics batch of " << st_iv_batches_[b].row_to - st_iv_batches_[b].row_from
                                                        << " frames exceeds " << kIvBatchRows);
          h.iv_stats_done = f + 1;
          h.iv_norm_to = std::max(h.iv_norm_to, std::min(f + iv_.m.right, T - 1) + 1);
        }
        st_iv_reqs_.push_back(r);
      }
      if (c >= 0) {
        if (first_real < 0) first_real = (int)st_jobs_.size();
        int valid = fin ? std::min(opc, need_out - c * opc) : opc;
        dec_frames += valid;
      }
      st_jobs_.push_back(DevJob{s, c * fpc, fin ? T - 1 : INT_MAX, 0});
      h.next_chunk++;
      njobs++;
      any = true;
    }
    if ((int)st_iv_reqs_.size() > req0) {
      st_iv_jobs_.push_back(IvStreamJob{s, req0, (int)st_iv_reqs_.size() - req0, h.iv_reset ? 1 : 0, T,
                                        0, 0, 0});
      st_ivcmvn_.push_back(CmvnJob{s, h.iv_norm_done, h.iv_norm_to, h.iv_reset ? 1 : 0});
      h.iv_norm_done = h.iv_norm_to;
      h.iv_reset = false;
    }
    h.out_ready += dec_frames;
    if (dec_frames > 0 || h.need_reset) {
      if (dec_frames > 0 || h.samples > 0 || fin) {
        // reset 2: a new decoder; 1: InitDecoding of the same decoder (a
        // Recognizer's next segment keeps its HashList size, Kaldi order)
        if (h.need_reset) {  // a new segment: nothing read yet
          host_read_[s].store(-1);
          prune_wait_[s].store(0);
        }
        st_dec_.push_back(DecJob{s, first_real < 0 ? 0 : first_real * opc, dec_frames,
                                 h.need_reset ? (h.fresh_stream ? 3 : h.fresh_decoder ? 2 : 1) : 0, stats_rows,
                                 fin ? 1 : 0, host_read_[s].load(std::memory_order_acquire), 0});
        if (h.need_reset) h.fresh_decoder = h.fresh_stream = false;
        stats_rows += dec_frames;
        if (h.need_reset) h.decoded = 0;
        h.need_reset = false;
        h.decoded += dec_frames;
        h.decoded_at_build = h.decoded;
        any = true;
      }
    }
  }
  return any;
}

void Engine::LaunchDecodeBatch(const DecBatch& b, hipStream_t s) {
  if (b.jobs.empty()) return;
  DecArgs d = dec_;
  d.jobs = (const DecJob*)(d_stage_ + (size_t)b.buf * stage_bytes_ + b.o_ej);
  d.llh = d_llh_buf_[b.llh];
  if (copy_pending_) {  // segment records still being copied (StartSegmentCopies)
    HIPCHECK(hipStreamWaitEvent(s, copy_ev_, 0));
    copy_pending_ = false;
  }
  LaunchDecode(d, (int)b.jobs.size(), s);
  HIPCHECK(hipMemcpyAsync(h_slots_, d_slots_, sizeof(DecSlot) * slots_.size(),
                          hipMemcpyDeviceToHost, s));
  int rows = 0;
  for (auto& j : b.jobs) rows += j.nframes;
  if (cfg_.collect_stats && rows)
    HIPCHECK(hipMemcpyAsync(h_stats_, d_stats_, sizeof(FrameStat) * rows, hipMemcpyDeviceToHost, s));
  counters_.launches++;
}

// Host side of a finished decoder launch (its stream has been synchronized).
void Engine::FinishDecodeBatch(const DecBatch& b) {
  for (size_t i = 0; i < b.jobs.size(); i++) {
    const DecJob& j = b.jobs[i];
    SlotHost& h = slots_[j.slot];
    const DecSlot& ds = h_slots_[j.slot];
    if (ds.frames != b.expect[i])
      VAMD_WARN("decoder frame count mismatch on slot " << j.slot << ": " << ds.frames << " vs "
                                                         << b.expect[i]);
    h.err = ds.err;
    h.dev_frames = ds.frames;
    arena_hwm_ = std::max(arena_hwm_, (long long)ds.arena_used);
    links_hwm_ = std::max(links_hwm_, ds.links_used);
    if (dec_.host_gate) {  // decode_kernel's prune_due: a pass waiting for the host's read
      const bool full = dec_.prune_fill_pct <= 0 || ds.frames >= dec_.prune_start ||
                        (long long)ds.arena_used * 100 >= (long long)dec_.arena_cap * dec_.prune_fill_pct ||
                        (dec_.links && ds.links_used * 100 >= dec_.link_cap * dec_.prune_fill_pct);
      prune_wait_[j.slot].store(dec_.prune_interval > 0 && !ds.err && ds.frames - ds.last_prune >= dec_.prune_interval &&
                                full);
    }
    if (cfg_.track_decoded) decoded_.push_back(DecodedJob{j.slot, j.pad0 != 0});
    if (ds.err) VAMD_WARN("decoder error flags " << ds.err << " on stream slot " << j.slot);
    counters_.frames_decoded += j.nframes;
    if (cfg_.collect_llh && j.nframes) {
      size_t n = (size_t)j.nframes * plan_.out_dim, o = h.llh.size();
      h.llh.resize(o + n);
      HIPCHECK(hipMemcpy(h.llh.data() + o, d_llh_buf_[b.llh] + (size_t)j.llh_row0 * plan_.out_dim,
                         sizeof(float) * n, hipMemcpyDeviceToHost));
    }
    if (cfg_.collect_stats) {
      // the decoder segment's frames (a reset starts a new segment)
      if (j.reset) h.stats.clear();
      h.stats.insert(h.stats.end(), h_stats_ + j.stats_row0, h_stats_ + j.stats_row0 + j.nframes);
      for (int f = 0; f < j.nframes; f++) {
        const FrameStat& fs = h_stats_[j.stats_row0 + f];
        times_.dec[0]++;
        times_.dec[1] += fs.ntok_in;
        times_.dec[2] += fs.ntok_out;
        times_.dec[3] += fs.arcs_emit;
        times_.dec[4] += fs.arcs_eps;
      }
      // links written by this launch (the counter restarts with the decoder)
      const long long lu = ds.links_used;
      times_.dec[5] += lu >= h.links_seen ? lu - h.links_seen : lu;
      h.links_seen = lu;
    }
  }
}

void Engine::LaunchNnet(const NnetBatch& b, hipStream_t s) {
  if (b.njobs == 0) return;
  const DevJob* dj = (const DevJob*)(d_stage_ + (size_t)b.buf * stage_bytes_ + b.o_dj);
  for (size_t i = 0; i < plan_.ops.size(); i++) {
    NnetOpArgs a = op_args_[i];
    a.M = b.njobs * a.P;
    a.jobs = dj;
    a.llh = d_llh_buf_[b.par];
    if (plan_.ops[i].kind == Op::GEMM) {
      LaunchNnetGemm(a, op_bk_[i], s);
    } else {
      for (int k = 0; k < a.nparts; k++)
        for (int j = a.parts[k].instr0; j < a.parts[k].instr0 + a.parts[k].ninstr; j++)
          if (a.instr[j].op == GInstr::PUSH_JOB) a.instr[j].base = d_ivec_buf_[b.par];
      LaunchNnetGather(a, s);
    }
  }
  counters_.launches += (long long)plan_.ops.size();
}

// One engine step.  Front end (staging copy, samples, MFCC, i-vectors) of the
// step just built, the nnet of the previous step and the decoder of the one
// before run concurrently on three streams (pipeline), or all three stages of
// this step in order on the main stream.
void Engine::RunStep(bool allow_pipeline) {
  const bool pipe = cfg_.pipeline && allow_pipeline;
  if (!pipe) FlushLocked();
  const int buf = (int)(seq_ % 3), par = (int)(seq_ % 2);
  char* hs = h_stage_ + (size_t)buf * stage_bytes_;
  char* dsg = d_stage_ + (size_t)buf * stage_bytes_;
  size_t off = 0;
  auto put = [&](const void* src, size_t bytes) {
    size_t o = off;
    if (bytes) memcpy(hs + o, src, bytes);
    off += Align256(bytes);
    return o;
  };
  // the samples are already in place (BuildStep wrote them into this buffer)
  if (st_sample_n_ > 0 && (char*)st_sample_data_ != hs) VAMD_ERR("staging buffer mismatch");
  const size_t o_data = 0;
  off = Align256(sizeof(float) * st_sample_n_);
  for (size_t i = 0; i < st_samples_.size(); i++)
    if (st_sample_src_[i] >= 0)
      st_samples_[i].src = (const float*)(dsg + o_data) + st_sample_src_[i];
  for (size_t i = 0; i < st_raw_.size(); i++)
    if (st_raw_src_[i] >= 0) st_raw_[i].src = (const float*)(dsg + o_data) + st_raw_src_[i];
  size_t o_sj = put(st_samples_.data(), sizeof(SampleJob) * st_samples_.size());
  size_t o_rj = put(st_raw_.data(), sizeof(SampleJob) * st_raw_.size());
  size_t o_resj = put(st_res_.data(), sizeof(ResampleJob) * st_res_.size());
  size_t o_mj = put(st_mfcc_.data(), sizeof(MfccJob) * st_mfcc_.size());
  NnetBatch cur;
  cur.njobs = (int)st_jobs_.size();
  cur.o_dj = put(st_jobs_.data(), sizeof(DevJob) * st_jobs_.size());
  cur.buf = buf;
  cur.par = par;
  size_t o_ivj = put(st_iv_jobs_.data(), sizeof(IvStreamJob) * st_iv_jobs_.size());
  size_t o_ivr = put(st_iv_reqs_.data(), sizeof(IvReq) * st_iv_reqs_.size());
  size_t o_ivb = put(st_iv_blocks_.data(), sizeof(IvFrameBlock) * st_iv_blocks_.size());
  size_t o_ivd = put(st_iv_devjobs_.data(), sizeof(DevJob) * st_iv_devjobs_.size());
  size_t o_ncm = put(st_ncmvn_.data(), sizeof(CmvnJob) * st_ncmvn_.size());
  size_t o_icm = put(st_ivcmvn_.data(), sizeof(CmvnJob) * st_ivcmvn_.size());
  size_t o_ive = put(st_iv_ents_.data(), sizeof(IvEntry) * st_iv_ents_.size());
  size_t o_ivbt = put(st_iv_batches_.data(), sizeof(IvBatch) * st_iv_batches_.size());
  cur.dec.jobs = st_dec_;
  cur.dec.o_ej = put(st_dec_.data(), sizeof(DecJob) * st_dec_.size());
  cur.dec.buf = buf;
  cur.dec.llh = par;
  for (auto& j : st_dec_) cur.dec.expect.push_back(slots_[j.slot].decoded_at_build);
  if (off > stage_bytes_) VAMD_ERR("step staging overflow");

  const bool tk = cfg_.time_kernels;
  hipStream_t fs = pipe ? fstream_ : stream_, ns = stream_, ds = pipe ? dstream_ : stream_;
  if (tk) HIPCHECK(hipEventRecord(ev_[0], fs));
  HIPCHECK(hipMemcpyAsync(dsg, hs, off, hipMemcpyHostToDevice, fs));
  // ---- front end of this step
  int lf = 0;
  if (tk) HIPCHECK(hipEventRecord(ev_[1], fs));
  LaunchAppendSamples((const SampleJob*)(dsg + o_rj), (int)st_raw_.size(), d_raw_, raw_ring_, fs);
  LaunchResample((const ResampleJob*)(dsg + o_resj), (int)st_res_.size(), d_res_tables_, d_raw_,
                 raw_ring_, d_samples_, sample_ring_, fs);
  lf += !st_raw_.empty() + !st_res_.empty();
  LaunchAppendSamples((const SampleJob*)(dsg + o_sj), (int)st_samples_.size(), d_samples_,
                      sample_ring_, fs);
  lf += !st_samples_.empty();
  LaunchMfcc(mfcc_, (const MfccJob*)(dsg + o_mj), (int)st_mfcc_.size(), st_mfcc_total_, d_samples_,
             sample_ring_, rings_, fs);
  lf += st_mfcc_total_ > 0;
  if (!st_ncmvn_.empty()) {
    LaunchCmvn(ncmvn_, (const CmvnJob*)(dsg + o_ncm), (int)st_ncmvn_.size(), fs);
    lf++;
  }
  if (!st_iv_jobs_.empty()) {
    IvArgs ia = iv_;
    ia.jobs = (const IvStreamJob*)(dsg + o_ivj);
    ia.reqs = (const IvReq*)(dsg + o_ivr);
    ia.blocks = (const IvFrameBlock*)(dsg + o_ivb);
    ia.ivec = d_ivec_buf_[par];
    ia.ents = (const IvEntry*)(dsg + o_ive);
    ia.nents = (int)st_iv_ents_.size();
    ia.batches = (const IvBatch*)(dsg + o_ivbt);
    const int rows = (int)st_iv_blocks_.size() * kIvFrameBlock;
    if (rows > max_iv_rows_) VAMD_ERR("i-vector frame records overflow");
    LaunchCmvn(ivcmvn_, (const CmvnJob*)(dsg + o_icm), (int)st_ivcmvn_.size(), fs);
    for (size_t i = 0; i < iv_ops_.size() && rows > 0; i++) {
      NnetOpArgs o = iv_ops_[i];
      o.M = rows;
      o.jobs = (const DevJob*)(dsg + o_ivd);
      LaunchNnetGemm(o, iv_op_bk_[i], fs);
    }
    LaunchIvectorStats(ia, d_iv_ll_, rows, (int)st_iv_jobs_.size(), fs);
    lf += 4 + (rows > 0 ? 4 : 0);
  }
  if (tk) HIPCHECK(hipEventRecord(ev_[2], fs));
  // ---- nnet: this step's (in order) or the previous step's (pipeline)
  const NnetBatch* nb = pipe ? (pendn_active_ ? &pendn_ : nullptr) : &cur;
  if (tk) {
    if (pipe) HIPCHECK(hipStreamWaitEvent(ns, ev_[0], 0));
    HIPCHECK(hipEventRecord(ev_[3], ns));
  }
  if (nb) LaunchNnet(*nb, ns);
  if (tk) HIPCHECK(hipEventRecord(ev_[4], ns));
  // ---- decoder: this step's (in order) or the one before the previous (pipeline)
  const DecBatch* db = pipe ? (pend_active_ ? &pend_ : nullptr) : &cur.dec;
  if (tk) {
    if (pipe) HIPCHECK(hipStreamWaitEvent(ds, ev_[0], 0));
    HIPCHECK(hipEventRecord(ev_[5], ds));
  }
  if (db) LaunchDecodeBatch(*db, ds);
  if (tk) HIPCHECK(hipEventRecord(ev_[6], ds));
  HIPCHECK(hipGetLastError());
  const auto tq0 = std::chrono::steady_clock::now();
  HIPCHECK(hipStreamSynchronize(ns));
  if (pipe) {
    HIPCHECK(hipStreamSynchronize(fs));
    HIPCHECK(hipStreamSynchronize(ds));
  }
  const auto tq1 = std::chrono::steady_clock::now();
  step_prof_[1] += std::chrono::duration<double, std::milli>(tq1 - tq0).count();
  if (tk) {
    float a = 0, b = 0, c = 0, t1 = 0, t2 = 0, t3 = 0;
    HIPCHECK(hipEventElapsedTime(&a, ev_[1], ev_[2]));
    HIPCHECK(hipEventElapsedTime(&b, ev_[3], ev_[4]));
    HIPCHECK(hipEventElapsedTime(&c, ev_[5], ev_[6]));
    HIPCHECK(hipEventElapsedTime(&t1, ev_[0], ev_[2]));
    HIPCHECK(hipEventElapsedTime(&t2, ev_[0], ev_[4]));
    HIPCHECK(hipEventElapsedTime(&t3, ev_[0], ev_[6]));
    times_.ms[0] += a; times_.ms[1] += b; times_.ms[2] += c;
    times_.ms[3] += std::max(t1, std::max(t2, t3));
    times_.launches[0] += lf;
    times_.launches[1] += nb && nb->njobs ? (long long)plan_.ops.size() : 0;
    times_.launches[2] += db && !db->jobs.empty() ? 1 : 0;
    times_.launches[3] += 1;
  }
  counters_.steps++;
  counters_.launches += lf;
  counters_.frames_mfcc += st_mfcc_total_;
  counters_.chunk_jobs += st_jobs_.size();
  if (db) FinishDecodeBatch(*db);
  step_prof_[2] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tq1).count();
  if (cfg_.collect_llh && !st_iv_reqs_.empty()) {
    const int Si = plan_.ivector_dim;
    std::vector<float> rows((size_t)st_jobs_.size() * Si);
    HIPCHECK(hipMemcpy(rows.data(), d_ivec_buf_[par], sizeof(float) * rows.size(), hipMemcpyDeviceToHost));
    for (const IvStreamJob& j : st_iv_jobs_)
      for (int q = 0; q < j.nreq; q++) {
        const IvReq& r = st_iv_reqs_[j.req0 + q];
        const float* v = rows.data() + (size_t)(r.job_hi - 1) * Si;
        slots_[j.slot].ivecs.insert(slots_[j.slot].ivecs.end(), v, v + Si);
      }
  }
  seq_++;
  if (pipe) {
    pend_active_ = pendn_active_ && !pendn_.dec.jobs.empty();
    if (pend_active_) pend_ = std::move(pendn_.dec);
    pendn_active_ = cur.njobs > 0 || !cur.dec.jobs.empty();
    if (pendn_active_) pendn_ = std::move(cur);
  }
}

void Engine::Advance(const std::vector<int>& slots) {
  std::lock_guard<std::mutex> lk(mu_);
  DEVICE_GUARD();
  while (BuildStep(slots)) RunStep();
  FlushLocked();
}

void Engine::Flush() {
  std::lock_guard<std::mutex> lk(mu_);
  DEVICE_GUARD();
  FlushLocked();
}

// One pipeline-tail pass: the pending nnet beside the pending decoder, or the
// last decoder alone.
void Engine::DrainOnce() {
  if (pendn_active_) {
    LaunchNnet(pendn_, stream_);
    if (pend_active_) LaunchDecodeBatch(pend_, dstream_);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(stream_));
    HIPCHECK(hipStreamSynchronize(dstream_));
    if (pend_active_) FinishDecodeBatch(pend_);
    pendn_active_ = false;
    pend_active_ = !pendn_.dec.jobs.empty();
    if (pend_active_) pend_ = std::move(pendn_.dec);
  } else if (pend_active_) {
    pend_active_ = false;
    LaunchDecodeBatch(pend_, dstream_);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(dstream_));
    FinishDecodeBatch(pend_);
  }
}

void Engine::FlushLocked() {
  while (pendn_active_ || pend_active_) DrainOnce();
}

bool Engine::Step(const std::vector<int>& slots, bool allow_pipeline) {
  std::lock_guard<std::mutex> lk(mu_);
  DEVICE_GUARD();
  const auto t0 = std::chrono::steady_clock::now();
  if (!BuildStep(slots)) {
    if (!pendn_active_ && !pend_active_) return false;
    DrainOnce();  // pipeline tail: only pending nnet / decoder passes are left
    return true;
  }
  const auto t1 = std::chrono::steady_clock::now();
  RunStep(allow_pipeline);
  // host-side step profile (VOSK_AMD_STEP_PROFILE): build, total
  step_prof_[0] += std::chrono::duration<double, std::milli>(t1 - t0).count();
  step_prof_[3] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  step_prof_n_++;
  static const bool print_prof = getenv("VOSK_AMD_STEP_PROFILE") != nullptr;
  if (print_prof && step_prof_n_ % 10 == 0)
    fprintf(stderr, "[engine] steps %lld: build %.3f ms, sync wait %.3f ms, after sync %.3f ms, total %.3f ms per step\n",
            step_prof_n_, step_prof_[0] / step_prof_n_, step_prof_[1] / step_prof_n_, step_prof_[2] / step_prof_n_,
            step_prof_[3] / step_prof_n_);
  return true;
}

void Engine::BestPaths(const std::vector<int>& slots, bool use_final,
                       std::vector<PathResult>* out, bool drain) {
  std::lock_guard<std::mutex> lk(mu_);
  DEVICE_GUARD();
  if (drain) FlushLocked();
  out->assign(slots.size(), PathResult());
  if (slots.empty()) return;
  // frames decoded on the device (equal to the host count once drained)
  auto frames_of = [&](int s) { return drain ? slots_.at(s).decoded : slots_.at(s).dev_frames; };
  int maxf = 0;
  for (int s : slots) maxf = std::max(maxf, frames_of(s));
  int cap = 4 * maxf + 64;
  const int n = (int)slots.size();
  for (int attempt = 0; attempt < 3; attempt++) {
    size_t bytes = Align256(sizeof(int) * n) + Align256(sizeof(int) * (size_t)n * cap) +
                   4 * Align256(sizeof(int) * n);
    if (bytes > bp_cap_) {
      if (d_bp_) HIPCHECK(hipFree(d_bp_));
      if (h_bp_) HIPCHECK(hipHostFree(h_bp_));
      d_bp_ = nullptr;
      h_bp_ = nullptr;
      bp_cap_ = 0;
      const size_t want = std::max<size_t>(bytes + bytes / 2, (size_t)1 << 20);
      HIPCHECK(hipMalloc((void**)&d_bp_, want));
      HIPCHECK(hipHostMalloc((void**)&h_bp_, want, hipHostMallocDefault));
      bp_cap_ = want;
    }
    char* d = d_bp_;
    char* h = h_bp_;
    size_t o_req = 0, o_path = Align256(sizeof(int) * n);
    size_t o_len = o_path + Align256(sizeof(int) * (size_t)n * cap);
    size_t o_cost = o_len + Align256(sizeof(int) * n);
    size_t o_rel = o_cost + Align256(sizeof(int) * n);
    size_t o_st = o_rel + Align256(sizeof(int) * n);
    HIPCHECK(hipMemcpyAsync(d + o_req, slots.data(), sizeof(int) * n, hipMemcpyHostToDevice, stream_));
    TraceArgs t;
    t.arc_sil = nullptr;
    t.sinfo = d_sinfo_;
    t.arena = dec_.arena;
    t.cur_state = dec_.cur_state;
    t.cur_cost = dec_.cur_cost;
    t.cur_pos = dec_.cur_pos;
    t.slots = d_slots_;
    t.req_slot = (const int*)(d + o_req);
    t.use_final = use_final ? 1 : 0;
    t.max_tok = dec_.max_tok;
    t.arena_cap = dec_.arena_cap;
    t.tie_pos = dec_.kaldi;
    t.path_cap = cap;
    t.path = (int*)(d + o_path);
    t.path_len = (int*)(d + o_len);
    t.end_cost = (float*)(d + o_cost);
    t.final_rel = (float*)(d + o_rel);
    t.end_state = (int*)(d + o_st);
    LaunchTraceback(t, n, stream_);
    HIPCHECK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, stream_));
    HIPCHECK(hipMemcpyAsync(h_slots_, d_slots_, sizeof(DecSlot) * slots_.size(),
                            hipMemcpyDeviceToHost, stream_));
    HIPCHECK(hipStreamSynchronize(stream_));
    bool retry = false;
    for (int i = 0; i < n; i++) {
      int len = ((int*)(h + o_len))[i];
      if (len > cap) { retry = true; cap = len + 64; }
    }
    if (retry) continue;
    for (int i = 0; i < n; i++) {
      PathResult& r = (*out)[i];
      int len = ((int*)(h + o_len))[i];
      const int* p = (const int*)(h + o_path) + (size_t)i * cap;
      r.arcs.assign(p, p + len);
      std::reverse(r.arcs.begin(), r.arcs.end());
      r.end_cost = ((float*)(h + o_cost))[i];
      r.final_relative_cost = ((float*)(h + o_rel))[i];
      r.end_state = ((int*)(h + o_st))[i];
      r.cost = (double)r.end_cost - h_slots_[slots[i]].offset_sum;
      if (frames_of(slots[i]) == 0) r.arcs.clear();
    }
    return;
  }
  VAMD_ERR("traceback path buffer could not be sized");
}

void Engine::GetRawLattice(int slot, bool use_final, RawLattice* out) {
  SegmentLattice sl;
  CopySegmentLattice(slot, &sl, true);
  *out = RawLattice();
  if (sl.frames.empty()) return;
  BuildRawLattice(md_->graph, md_->graph.start, sl.frames, sl.arena, sl.links, use_final, out);
  if (sl.overflow) out->overflow = true;
}

void Engine::CopySegmentLattice(int slot, SegmentLattice* out, bool drain) {
  CopySegmentLattices({slot}, {out}, drain);
}

// The segments' records go through one pinned staging buffer on a copy
// stream of their own (not queued behind the pipeline's kernels): one read
// of the decoder states, then all frames / arena / link copies in flight
// together, one synchronization.
void Engine::CopySegmentLattices(const std::vector<int>& slots, const std::vector<SegmentLattice*>& outs,
                                 bool drain) {
  std::lock_guard<std::mutex> lk(mu_);
  DEVICE_GUARD();
  if (drain) FlushLocked();
  for (SegmentLattice* o : outs) {  // (recycled buffers keep their capacity)
    o->frames.clear();
    o->arena.clear();
    o->links.clear();
    o->overflow = false;
  }
  if (!dec_.links || slots.empty()) return;
  if (!copy_stream_) HIPCHECK(hipStreamCreateWithFlags(&copy_stream_, hipStreamNonBlocking));
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  if (!h_copy_slots_)  // own snapshot: h_slots_ may be the target of a decoder batch's read-back
    HIPCHECK(hipHostMalloc((void**)&h_copy_slots_, sizeof(DecSlot) * slots_.size(), hipHostMallocDefault));
  HIPCHECK(hipMemcpyAsync(h_copy_slots_, d_slots_, sizeof(DecSlot) * slots_.size(), hipMemcpyDeviceToHost,
                          copy_stream_));
  HIPCHECK(hipStreamSynchronize(copy_stream_));
  const auto t1 = clk::now();
  struct Part { size_t f, a, l; int nf = 0; int na = 0; long long nl = 0; };
  std::vector<Part> parts(slots.size());
  size_t bytes = 0;
  auto take = [&](size_t n) { const size_t o = bytes; bytes += Align256(n); return o; };
  for (size_t i = 0; i < slots.size(); i++) {
    const DecSlot& st = h_copy_slots_[slots[i]];
    const int host_frames = drain ? slots_.at(slots[i]).decoded : slots_.at(slots[i]).dev_frames;
    if (host_frames == 0 && st.frames == 0 && st.arena_used == 0) continue;
    Part& q = parts[i];
    q.nf = std::min(st.frames + 1, dec_.lat_frame_cap);
    q.na = st.arena_used;
    q.nl = std::min(st.links_used, dec_.link_cap);
    q.f = take(sizeof(LatFrame) * q.nf);
    q.a = take(sizeof(int4) * q.na);
    q.l = take(sizeof(int4) * q.nl);
    outs[i]->overflow = st.lat_ovf || st.frames + 1 > dec_.lat_frame_cap || st.err;
  }
  if (bytes > lat_stage_bytes_) {
    if (h_lat_stage_) HIPCHECK(hipHostFree(h_lat_stage_));
    h_lat_stage_ = nullptr;
    lat_stage_bytes_ = std::max(bytes, lat_stage_bytes_ * 2);
    HIPCHECK(hipHostMalloc((void**)&h_lat_stage_, lat_stage_bytes_, hipHostMallocDefault));
  }
  for (size_t i = 0; i < slots.size(); i++) {
    const Part& q = parts[i];
    const size_t s = (size_t)slots[i];
    if (q.nf > 0)
      HIPCHECK(hipMemcpyAsync(h_lat_stage_ + q.f, dec_.lat_frames + s * dec_.lat_frame_cap,
                              sizeof(LatFrame) * q.nf, hipMemcpyDeviceToHost, copy_stream_));
    if (q.na > 0)
      HIPCHECK(hipMemcpyAsync(h_lat_stage_ + q.a, dec_.arena + s * dec_.arena_cap, sizeof(int4) * q.na,
                              hipMemcpyDeviceToHost, copy_stream_));
    if (q.nl > 0)
      HIPCHECK(hipMemcpyAsync(h_lat_stage_ + q.l, dec_.links + s * dec_.link_cap, sizeof(int4) * q.nl,
                              hipMemcpyDeviceToHost, copy_stream_));
  }
  HIPCHECK(hipStreamSynchronize(copy_stream_));
  const auto t2 = clk::now();
  for (size_t i = 0; i < slots.size(); i++) {
    const Part& q = parts[i];
    SegmentLattice* o = outs[i];
    const LatFrame* F = (const LatFrame*)(h_lat_stage_ + q.f);
    const int4* A = (const int4*)(h_lat_stage_ + q.a);
    const int4* L = (const int4*)(h_lat_stage_ + q.l);
    o->frames.assign(F, F + q.nf);
    o->arena.assign(A, A + q.na);
    o->links.assign(L, L + q.nl);
  }
  auto us = [](clk::time_point a, clk::time_point b) {
    return (long long)std::chrono::duration_cast<std::chrono::microseconds>(b - a).count();
  };
  copy_us_[0] += us(t0, t1);
  copy_us_[1] += us(t1, t2);
  copy_us_[2] += us(t2, clk::now());
  copy_us_[3] += (long long)bytes;
  if (getenv("VOSK_AMD_COPY_DEBUG") && ++copy_calls_ % 20 == 0)
    fprintf(stderr, "segment copies: %lld calls, states %lld us, records %lld us, host %lld us, %lld MB\n",
            copy_calls_, copy_us_[0], copy_us_[1], copy_us_[2], copy_us_[3] >> 20);
}

void Engine::CopySegmentTail(int slot, int from, SegmentLattice* out, int upto, bool concurrent) {
  std::unique_lock<std::mutex> lk(mu_, std::defer_lock);
  if (!concurrent) lk.lock();
  int prev_dev = -1;
  if (hipGetDevice(&prev_dev) != hipSuccess) prev_dev = -1;
  HIPCHECK(hipSetDevice(cfg_.device));
  struct Restore {
    int d;
    ~Restore() {
      if (d >= 0) (void)hipSetDevice(d);
    }
  } restore{concurrent ? prev_dev : -1};
  if (concurrent && cfg_.pipeline) VAMD_ERR("concurrent segment copies need an engine without pipelining");
  if (!concurrent) FlushLocked();
  out->frames.clear();
  out->arena.clear();
  out->links.clear();
  out->overflow = false;
  out->first_frame = from;
  out->arena_base = 0;
  out->link_base = 0;
  if (!dec_.links) return;
  // concurrent: the engine's copy stream, one read at a time
  std::unique_lock<std::mutex> tl(tail_mu_, std::defer_lock);
  if (concurrent) {
    tl.lock();
    if (!copy_stream_) HIPCHECK(hipStreamCreateWithFlags(&copy_stream_, hipStreamNonBlocking));
  }
  auto copy = [&](void* dst, const void* src, size_t bytes) {
    if (concurrent) {  // through a pinned block (direct DMA)
      size_t cap = 0;
      char* pin = pinned_->Take(bytes, &cap);
      struct Back {
        PinnedPool* pool;
        char* p;
        size_t cap;
        ~Back() { pool->Give(p, cap); }
      } back{pinned_.get(), pin, cap};
      HIPCHECK(hipMemcpyAsync(pin, src, bytes, hipMemcpyDeviceToHost, copy_stream_));
      HIPCHECK(hipStreamSynchronize(copy_stream_));
      memcpy(dst, pin, bytes);
    } else {
      HIPCHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, copy_stream_));
    }
  };
  auto sync = [&] {
    if (!concurrent) HIPCHECK(hipStreamSynchronize(copy_stream_));
  };
  if (!concurrent && !copy_stream_) HIPCHECK(hipStreamCreateWithFlags(&copy_stream_, hipStreamNonBlocking));
  DecSlot st, st2;
  copy(&st, d_slots_ + slot, sizeof(DecSlot));
  sync();
  out->overflow = st.lat_ovf || st.frames + 1 > dec_.lat_frame_cap || st.err;
  out->last_prune = st.last_prune;
  int nf = std::min(st.frames + 1, dec_.lat_frame_cap);
  if (upto >= 0) nf = std::min(nf, upto + 1);
  if (from >= nf || from < 0) return;
  out->frames.resize(nf - from);
  copy(out->frames.data(), dec_.lat_frames + (size_t)slot * dec_.lat_frame_cap + from, sizeof(LatFrame) * (nf - from));
  sync();
  const LatFrame& f0 = out->frames[0];
  const LatFrame& fl = out->frames.back();
  const int a0 = std::max(0, f0.tok_base);
  const long long l0 = std::max(0ll, f0.link_begin);
  // the wanted frames' records only (later frames may be in the making)
  const int na = std::max(0, fl.tok_base + fl.ntok - a0);
  const long long nl = std::max(0ll, std::min(fl.link_end, dec_.link_cap) - l0);
  out->arena_base = a0;
  out->link_base = l0;
  out->arena.resize(na);
  out->links.resize(nl);
  if (na > 0) copy(out->arena.data(), dec_.arena + (size_t)slot * dec_.arena_cap + a0, sizeof(int4) * na);
  if (nl > 0) copy(out->links.data(), dec_.links + (size_t)slot * dec_.link_cap + l0, sizeof(int4) * nl);
  sync();
  if (concurrent) {  // a pruning pass may have compacted the records meanwhile
    copy(&st2, d_slots_ + slot, sizeof(DecSlot));
    if (st2.last_prune != st.last_prune || st2.frames < st.frames || st2.lat_ovf || st2.err) out->overflow = true;
  }
}

PinnedPool::~PinnedPool() {
  for (auto& b : free_) (void)hipHostFree(b.second);
}

char* PinnedPool::Take(size_t bytes, size_t* cap) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    size_t best = free_.size();
    for (size_t i = 0; i < free_.size(); i++)
      if (free_[i].first >= bytes && (best == free_.size() || free_[i].first < free_[best].first)) best = i;
    if (best < free_.size()) {
      char* p = free_[best].second;
      *cap = free_[best].first;
      free_.erase(free_.begin() + best);
      return p;
    }
  }
  *cap = std::max<size_t>(Align256(bytes), 1 << 20);
  char* p = nullptr;
  HIPCHECK(hipHostMalloc((void**)&p, *cap, hipHostMallocDefault));
  return p;
}

void PinnedPool::Give(char* p, size_t cap) {
  std::lock_guard<std::mutex> lk(mu_);
  free_.push_back({cap, p});
}

CopyBatch::~CopyBatch() {
  if (done) {
    (void)hipSetDevice(device);
    (void)hipEventSynchronize(done);  // never recycle a block a copy still writes
    (void)hipEventDestroy(done);
  }
  if (block) pool->Give(block, cap);
}

void SegmentCopy::Finish(SegmentLattice* out) {
  out->frames.clear();
  out->arena.clear();
  out->links.clear();
  out->overflow = overflow;
  if (!batch) return;
  int prev = -1;  // the caller's current device is restored (a waiting caller may run this)
  if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  (void)hipSetDevice(batch->device);
  const hipError_t se = hipEventSynchronize(batch->done);
  if (prev >= 0) (void)hipSetDevice(prev);
  HIPCHECK(se);
  const char* block = batch->block;
  const LatFrame* F = (const LatFrame*)(block + f);
  const int4* A = (const int4*)(block + a);
  const int4* L = (const int4*)(block + l);
  out->frames.assign(F, F + nf);
  out->arena.assign(A, A + na);
  out->links.assign(L, L + nl);
  batch.reset();  // the last segment of the call returns the block
}

void Engine::StartSegmentCopies(const std::vector<int>& slots, std::vector<std::shared_ptr<SegmentCopy>>* out) {
  std::lock_guard<std::mutex> lk(mu_);
  DEVICE_GUARD();
  out->clear();
  for (size_t i = 0; i < slots.size(); i++) out->push_back(std::make_shared<SegmentCopy>());
  if (!dec_.links || slots.empty()) return;
  if (!copy_stream_) HIPCHECK(hipStreamCreateWithFlags(&copy_stream_, hipStreamNonBlocking));
  if (!copy_ev_) HIPCHECK(hipEventCreateWithFlags(&copy_ev_, hipEventDisableTiming));
  if (!h_copy_slots_)  // own snapshot: h_slots_ may be the target of a decoder batch's read-back
    HIPCHECK(hipHostMalloc((void**)&h_copy_slots_, sizeof(DecSlot) * slots_.size(), hipHostMallocDefault));
  // the segments end (each stream's decoder restarts after its copy): their
  // last lattice prune (final costs, every frame) on the copy stream, so the
  // copies below take the pruned records
  const bool final_prune = !getenv("VOSK_AMD_FINAL_PRUNE") || atoi(getenv("VOSK_AMD_FINAL_PRUNE")) != 0;
  if (final_prune) {
    if (!d_prune_slots_) d_prune_slots_ = (int*)DevAlloc(sizeof(int) * slots_.size());
    // from pinned staging (a pageable source makes the copy synchronous):
    // [slots][items]; the slot part's last reader is the previous call's
    // copy, finished at that call's synchronization below
    if (!h_copy_stage_)
      HIPCHECK(hipHostMalloc((void**)&h_copy_stage_,
                             Align256(sizeof(int) * slots_.size()) + sizeof(CopyItem) * 3 * slots_.size(),
                             hipHostMallocDefault));
    memcpy(h_copy_stage_, slots.data(), sizeof(int) * slots.size());
    HIPCHECK(hipMemcpyAsync(d_prune_slots_, h_copy_stage_, sizeof(int) * slots.size(), hipMemcpyHostToDevice,
                            copy_stream_));
    LaunchPruneFinal(dec_, d_prune_slots_, (int)slots.size(), true, copy_stream_);
  }
  const auto tc0 = std::chrono::steady_clock::now();
  HIPCHECK(hipMemcpyAsync(h_copy_slots_, d_slots_, sizeof(DecSlot) * slots_.size(), hipMemcpyDeviceToHost,
                          copy_stream_));
  HIPCHECK(hipStreamSynchronize(copy_stream_));
  const auto tc1 = std::chrono::steady_clock::now();
  copy_prof_[0] += std::chrono::duration<double, std::milli>(tc1 - tc0).count();
  // one pinned block and one completion event for all of the call's segments
  size_t bytes = 0;
  std::vector<int> copied;
  for (size_t i = 0; i < slots.size(); i++) {
    const DecSlot& st = h_copy_slots_[slots[i]];
    SegmentCopy& c = *(*out)[i];
    if (slots_.at(slots[i]).dev_frames == 0 && st.frames == 0 && st.arena_used == 0) continue;
    c.nf = std::min(st.frames + 1, dec_.lat_frame_cap);
    c.na = st.arena_used;
    c.nl = std::min(st.links_used, dec_.link_cap);
    c.overflow = st.lat_ovf || st.frames + 1 > dec_.lat_frame_cap || st.err;
    c.f = bytes;
    bytes += Align256(sizeof(LatFrame) * c.nf);
    c.a = bytes;
    bytes += Align256(sizeof(int4) * c.na);
    c.l = bytes;
    bytes += Align256(sizeof(int4) * c.nl);
    copied.push_back((int)i);
  }
  if (!copied.empty()) {
    auto cb = std::make_shared<CopyBatch>();
    cb->pool = pinned_;
    cb->device = cfg_.device;
    const auto tt0 = std::chrono::steady_clock::now();
    cb->block = pinned_->Take(bytes, &cb->cap);
    copy_prof_[3] += bytes / 1048576.0;
    copy_prof_[1] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tt0).count();
    // the records gathered into one device block in the host layout (a
    // workgroup per record range), then one copy to the pinned block
    std::vector<CopyItem> items;
    items.reserve(copied.size() * 3);
    auto add = [&](const void* src, size_t off, size_t nbytes) {
      if (nbytes == 0) return;
      if ((nbytes | off) & 3) VAMD_ERR("segment copy: unaligned record range");
      items.push_back(CopyItem{(const unsigned*)src, (long long)(off / 4), (long long)(nbytes / 4)});
    };
    for (int i : copied) {
      SegmentCopy& c = *(*out)[i];
      c.batch = cb;
      const size_t s = (size_t)slots[i];
      add(dec_.lat_frames + s * dec_.lat_frame_cap, c.f, sizeof(LatFrame) * c.nf);
      add(dec_.arena + s * dec_.arena_cap, c.a, sizeof(int4) * c.na);
      add(dec_.links + s * dec_.link_cap, c.l, sizeof(int4) * c.nl);
    }
    if (bytes > pack_cap_) {
      if (d_pack_) HIPCHECK(hipFree(d_pack_));
      pack_cap_ = bytes + bytes / 4;
      HIPCHECK(hipMalloc((void**)&d_pack_, pack_cap_));
    }
    if (items.size() > pack_items_cap_) {
      if (d_pack_items_) HIPCHECK(hipFree(d_pack_items_));
      pack_items_cap_ = items.size() + items.size() / 4 + 16;
      HIPCHECK(hipMalloc((void**)&d_pack_items_, sizeof(CopyItem) * pack_items_cap_));
    }
    if (!items.empty()) {
      const CopyItem* src = items.data();
      if (h_copy_stage_ && items.size() <= 3 * slots_.size()) {  // (every earlier copy is finished here)
        CopyItem* st = (CopyItem*)(h_copy_stage_ + Align256(sizeof(int) * slots_.size()));
        memcpy(st, items.data(), sizeof(CopyItem) * items.size());
        src = st;
      }
      HIPCHECK(hipMemcpyAsync(d_pack_items_, src, sizeof(CopyItem) * items.size(), hipMemcpyHostToDevice,
                              copy_stream_));
      LaunchGatherCopy(d_pack_items_, (int)items.size(), d_pack_, copy_stream_);
      HIPCHECK(hipGetLastError());
      HIPCHECK(hipMemcpyAsync(cb->block, d_pack_, bytes, hipMemcpyDeviceToHost, copy_stream_));
    }
    // a waiting worker sleeps, not spins
    HIPCHECK(hipEventCreateWithFlags(&cb->done, hipEventDisableTiming | hipEventBlockingSync));
    HIPCHECK(hipEventRecord(cb->done, copy_stream_));
  }
  // the stream's next decoder launch (which may reset and overwrite these
  // records) waits for the copies on the device
  HIPCHECK(hipEventRecord(copy_ev_, copy_stream_));
  copy_pending_ = true;
  copy_prof_[2] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tc1).count();
  copy_prof_n_++;
}

void Engine::TakeDecoded(std::vector<DecodedJob>* out) {
  std::lock_guard<std::mutex> lk(mu_);
  out->swap(decoded_);
  decoded_.clear();
}

void Engine::ProbeEndpoints(const std::vector<int>& slots, std::vector<EndpointProbe>* out) {
  std::lock_guard<std::mutex> lk(mu_);
  DEVICE_GUARD();
  const int n = (int)slots.size();
  out->assign(n, EndpointProbe());
  if (n == 0) return;
  if (!d_arc_sil_) VAMD_ERR("endpoint probe without silence phones");
  const int S = (int)slots_.size();
  if (!d_probe_) {  // [req][len][final_rel][end_cost][end_state], S entries each
    d_probe_ = (int*)DevAlloc(sizeof(int) * 5 * S);
    HIPCHECK(hipHostMalloc((void**)&h_probe_, sizeof(int) * 5 * S, hipHostMallocDefault));
  }
  if (n > S) VAMD_ERR("endpoint probe over more streams than slots");
  memcpy(h_probe_, slots.data(), sizeof(int) * n);
  HIPCHECK(hipMemcpyAsync(d_probe_, h_probe_, sizeof(int) * n, hipMemcpyHostToDevice, stream_));
  TraceArgs t;
  memset(&t, 0, sizeof(t));
  t.tie_pos = dec_.kaldi;
  t.arc_sil = d_arc_sil_;
  t.sinfo = d_sinfo_;
  t.arena = dec_.arena;
  t.cur_state = dec_.cur_state;
  t.cur_cost = dec_.cur_cost;
  t.cur_pos = dec_.cur_pos;
  t.slots = d_slots_;
  t.req_slot = d_probe_;
  t.use_final = 0;
  t.max_tok = dec_.max_tok;
  t.arena_cap = dec_.arena_cap;
  t.path_len = d_probe_ + S;
  t.final_rel = (float*)(d_probe_ + 2 * S);
  t.end_cost = (float*)(d_probe_ + 3 * S);
  t.end_state = d_probe_ + 4 * S;
  LaunchTraceback(t, n, stream_);
  HIPCHECK(hipMemcpyAsync(h_probe_ + S, d_probe_ + S, sizeof(int) * 2 * S, hipMemcpyDeviceToHost, stream_));
  HIPCHECK(hipStreamSynchronize(stream_));
  for (int i = 0; i < n; i++) {
    EndpointProbe& p = (*out)[i];
    p.frames = slots_.at(slots[i]).dev_frames;
    p.trailing_sil = h_probe_[S + i];
    memcpy(&p.final_relative_cost, h_probe_ + 2 * S + i, 4);
  }
}

bool Engine::SlotInFlight(int slot) const {
  auto has = [slot](const DecBatch& b) {
    for (const DecJob& j : b.jobs)
      if (j.slot == slot) return true;
    return false;
  };
  return (pend_active_ && has(pend_)) || (pendn_active_ && has(pendn_.dec));
}

// Whether BuildStep would stage any work for the stream (its predicates).
bool Engine::HasRunnableWork(const SlotHost& h) const {
  if (!h.used) return false;
  if (h.pending_pos < h.pending.size()) return true;
  if (h.resident && h.resident_pos < h.resident_n) return true;
  if (h.rate != 0) {
    const ResampleTable& T = res_tables_[h.table];
    if (T.NumOutputSamples(h.raw_pushed, h.finished && !h.res_flushed) > h.samples) return true;
    if (h.finished && !h.res_flushed) return true;
  }
  if (NumFramesFor(h.samples) > h.frames) return true;
  const bool fin = h.finished && h.pending_pos == h.pending.size() &&
                   (!h.resident || h.resident_pos == h.resident_n) && (h.rate == 0 || h.res_flushed);
  const int T = h.frames, c = h.next_chunk;
  bool ready;
  if (fin) ready = T > 0 && (c < 0 || c * plan_.opc < (T + plan_.fss - 1) / plan_.fss);
  else ready = T >= (std::max(c, 0) + 1) * plan_.fpc + plan_.right_context + (use_iv_ ? iv_.m.right : 0);
  if (ready) return true;
  // a pending decoder reset alone waits for the stream's next frames (it is
  // folded into that job) unless the input has ended
  return h.need_reset && fin && h.samples > 0;
}

std::string Engine::DescribeSlot(int slot) const {
  const SlotHost& h = slots_.at(slot);
  std::ostringstream o;
  o << "slot " << slot << " used=" << h.used << " pending=" << h.pending.size() - h.pending_pos
    << " samples=" << h.samples << " frames=" << h.frames << " next_chunk=" << h.next_chunk
    << " out_ready=" << h.out_ready << " decoded=" << h.decoded << " dev=" << h.dev_frames
    << " finished=" << h.finished << " need_reset=" << h.need_reset << " rate=" << h.rate
    << " inflight=" << SlotInFlight(slot) << " runnable=" << HasRunnableWork(h)
    << " nf(samples)=" << NumFramesFor(h.samples);
  return o.str();
}

bool Engine::ChunkReadyAfter(int slot, long long extra) const {
  std::lock_guard<std::mutex> lk(const_cast<std::mutex&>(mu_));
  const SlotHost& h = slots_.at(slot);
  if (!h.used || h.rate != 0 || h.resident || h.finished) return true;
  const long long samples = h.samples + (long long)(h.pending.size() - h.pending_pos) + extra;
  const int T = NumFramesFor(samples);
  const int iv_wait = use_iv_ ? iv_.m.right : 0;
  return T >= (std::max(h.next_chunk, 0) + 1) * plan_.fpc + plan_.right_context + iv_wait;
}

bool Engine::StreamIdle(int slot) const {
  std::lock_guard<std::mutex> lk(const_cast<std::mutex&>(mu_));
  return !SlotInFlight(slot) && !HasRunnableWork(slots_.at(slot));
}

void Engine::ResetDecoderAtNextJob(int slot) {
  std::lock_guard<std::mutex> lk(mu_);
  DEVICE_GUARD();
  SlotHost& h = slots_.at(slot);
  h.sw.Reset();
  h.dev_frames = 0;
  // the earliest staged decoder job of the stream: pend_ launches next
  DecBatch* order[2] = {pend_active_ ? &pend_ : nullptr, pendn_active_ ? &pendn_.dec : nullptr};
  for (int b = 0; b < 2; b++) {
    if (!order[b]) continue;
    DecBatch& db = *order[b];
    for (size_t i = 0; i < db.jobs.size(); i++) {
      if (db.jobs[i].slot != slot) continue;
      db.jobs[i].reset = std::max(db.jobs[i].reset, 2);  // a batch segment starts a new decoder
      // the patch goes through the batch's pinned staging copy, ordered on
      // the decoder stream: every staged decoder batch launches on dstream_
      // (the next pipelined step, or a drain), so the launch reads the
      // patched job whatever else is in flight (a synchronous copy from
      // pageable memory on the null stream is not ordered with the engine's
      // non-blocking streams)
      const size_t o = (size_t)db.buf * stage_bytes_ + db.o_ej + sizeof(DecJob) * i;
      memcpy(h_stage_ + o, &db.jobs[i], sizeof(DecJob));
      HIPCHECK(hipMemcpyAsync(d_stage_ + o, h_stage_ + o, sizeof(DecJob), hipMemcpyHostToDevice, dstream_));
      // frame counts of the new segment: this job's, then the later staged one's
      int n = db.jobs[i].nframes;
      db.expect[i] = n;
      if (b == 0 && order[1])
        for (size_t k = 0; k < order[1]->jobs.size(); k++)
          if (order[1]->jobs[k].slot == slot) {
            n += order[1]->jobs[k].nframes;
            order[1]->expect[k] = n;
          }
      h.decoded = n;
      h.decoded_at_build = n;
      return;
    }
  }
  h.decoded = 0;
  h.need_reset = true;
  h.fresh_decoder = true;
}

int Engine::IvectorFramesReady(int slot) const {
  const SlotHost& h = slots_.at(slot);
  long long remaining = (long long)(h.pending.size() - h.pending_pos);
  if (h.resident) remaining += h.resident_n - h.resident_pos;
  const bool fin = h.finished || (h.resident && h.resident_finish);
  long long samples;
  if (h.rate != 0) {
    const ResampleTable& T = res_tables_[h.table];
    samples = T.NumOutputSamples(h.raw_pushed + remaining, fin);
  } else {
    samples = h.samples + remaining;
  }
  const int frames = NumFramesFor(samples);
  if (fin) return frames;
  return std::max(0, frames - (use_iv_ ? iv_.m.right : 0));
}

void Engine::UpdateSilenceWeights(int slot, int first_decoder_frame) {
  UpdateSilenceWeights(std::vector<int>{slot}, std::vector<int>{first_decoder_frame});
}

void Engine::UpdateSilenceWeights(const std::vector<int>& slots, const std::vector<int>& first_decoder_frame) {
  if (!SilenceWeightingActive()) return;
  const size_t n = slots.size();
  std::vector<int> ready(n, 0), with_path;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (size_t i = 0; i < n; i++) {
      const SlotHost& h = slots_.at(slots[i]);
      // statistics already accumulated without weights stay unweighted
      if (!h.iv_weighted && h.iv_stats_done > 0) continue;
      ready[i] = IvectorFramesReady(slots[i]);
      if (ready[i] > 0 && h.decoded > 0) with_path.push_back(slots[i]);
    }
  }
  if (with_path.empty() && std::all_of(ready.begin(), ready.end(), [](int r) { return r <= 0; })) return;
  std::vector<PathResult> pr;
  if (!with_path.empty()) BestPaths(with_path, false, &pr);  // one traceback launch for all
  const Graph& g = md_->graph;
  const ModelData& m = *md_;
  auto is_sil = [&m](int t) {
    const int ph = m.tm.tid2phone[t];
    return ph < (int)m.phone_is_silence.size() && m.phone_is_silence[ph] != 0;
  };
  std::lock_guard<std::mutex> lk(mu_);
  size_t k = 0;
  for (size_t i = 0; i < n; i++) {
    if (ready[i] <= 0) continue;
    std::vector<int> tid, tok;
    if (k < with_path.size() && with_path[k] == slots[i]) {
      for (int a : pr[k].arcs) {
        if (g.ilabel[a] == 0) continue;
        // source state of the arc: the token it leaves (unique per frame and state)
        const int src = (int)(std::upper_bound(g.arc_begin.begin(), g.arc_begin.end(), (int64_t)a) -
                              g.arc_begin.begin()) - 1;
        tid.push_back(g.ilabel[a]);
        tok.push_back(src);
      }
      k++;
    }
    SlotHost& h = slots_.at(slots[i]);
    std::vector<std::pair<int, float>> d;
    h.sw.ComputeCurrentTraceback(tid, tok);
    h.sw.GetDeltaWeights(ready[i], first_decoder_frame[i], is_sil, &d);
    h.iv_pending.insert(h.iv_pending.end(), d.begin(), d.end());
    h.iv_weighted = true;
  }
}

void Engine::DecodeExternal(int slot, const float* llh, int nframes, bool reset) {
  std::lock_guard<std::mutex> lk(mu_);
  DEVICE_GUARD();
  FlushLocked();
  SlotHost& h = slots_.at(slot);
  const int P = plan_.out_dim;
  int done = 0;
  bool first = true;
  while (first || done < nframes) {
    const int n = std::min(nframes - done, max_dec_frames_);
    if (n > 0)
      HIPCHECK(hipMemcpyAsync(d_llh_buf_[seq_ % 2], llh + (size_t)done * P, sizeof(float) * n * P,
                              hipMemcpyHostToDevice, stream_));
    st_samples_.clear();
    st_sample_src_.clear();
    st_sample_n_ = 0;
    st_raw_.clear();
    st_raw_src_.clear();
    st_res_.clear();
    st_mfcc_.clear();
    st_mfcc_total_ = 0;
    st_jobs_.clear();
    st_dec_.clear();
    st_iv_jobs_.clear();
    st_iv_reqs_.clear();
    st_iv_blocks_.clear();
    st_iv_devjobs_.clear();
    st_iv_batches_.clear();
    st_iv_ents_.clear();
    st_ncmvn_.clear();
    st_ivcmvn_.clear();
    st_iv_frames_ = 0;
    h.stats.clear();
    const bool rs = first && (reset || h.need_reset);
    // (a decode from scratch is a new stream: lazy numbering starts over)
    st_dec_.push_back(DecJob{slot, 0, n, rs ? (reset || h.fresh_stream ? 3 : h.fresh_decoder ? 2 : 1) : 0, 0, 0, -1,
                             0});
    if (rs) h.fresh_decoder = h.fresh_stream = false;
    if (rs) h.decoded = 0;
    h.need_reset = false;
    h.decoded += n;
    h.decoded_at_build = h.decoded;
    RunStep(false);
    done += n;
    first = false;
  }
}

void Engine::DecoderPhaseClocks(long long* out, long long* per_slot) {
  std::lock_guard<std::mutex> lk(mu_);
  DEVICE_GUARD();
  FlushLocked();
  for (int i = 0; i < kDecProf; i++) out[i] = 0;
  std::vector<long long> h((size_t)kDecProf * slots_.size(), 0);
  if (dec_.prof)
    HIPCHECK(hipMemcpy(h.data(), dec_.prof, sizeof(long long) * h.size(), hipMemcpyDeviceToHost));
  for (size_t s = 0; s < slots_.size(); s++)
    for (int i = 0; i < kDecProf; i++) out[i] += h[s * kDecProf + i];
  if (per_slot) std::copy(h.begin(), h.end(), per_slot);
}

void Engine::DebugFeatures(int slot, int first, int n, std::vector<float>* out) {
  std::lock_guard<std::mutex> lk(mu_);
  DEVICE_GUARD();
  const int dim = plan_.input_dim;
  std::vector<float> ring((size_t)ring_ * dim);
  float* base = nullptr;
  HIPCHECK(hipMemcpy(&base, d_ring_ptrs_ + plan_.input_node, sizeof(float*), hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy2D(ring.data(), sizeof(float) * dim, base + (size_t)slot * dim,
                       sizeof(float) * dim * cfg_.max_slots, sizeof(float) * dim, ring_,
                       hipMemcpyDeviceToHost));
  out->resize((size_t)n * dim);
  for (int i = 0; i < n; i++)
    memcpy(out->data() + (size_t)i * dim, ring.data() + (size_t)((first + i) & (ring_ - 1)) * dim,
           sizeof(float) * dim);
}

}  // namespace vamd
