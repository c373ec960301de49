// Speaker x-vectors on the GPU (xvector.h).
#include "xvector.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>

#include "common.h"
#include "engine.h"
#include "kernels.h"

namespace vamd {

#define XV_HIPCHECK(x)                                                               \
  do {                                                                               \
    hipError_t _e = (x);                                                             \
    if (_e != hipSuccess) VAMD_ERR("HIP error " << hipGetErrorString(_e) << " at "   \
                                                << __FILE__ << ":" << __LINE__);     \
  } while (0)

namespace {
bool IsAffineType(const std::string& t) {
  return t == "AffineComponent" || t == "NaturalGradientAffineComponent" ||
         t == "FixedAffineComponent" || t == "LinearComponent";
}

// Input columns padded to a multiple of 8 (the GEMM kernels' K granularity):
// every block of the affine input that reads "input" gets zero columns.
void PadInput(Nnet* nn, int D, int Dp) {
  if (Dp == D) return;
  auto& in = nn->nodes[nn->node_index.at("input")];
  in.dim = Dp;
  for (auto& nd : nn->nodes) {
    if (nd.kind != NnetNode::COMPONENT) continue;
    // blocks of the descriptor, in column order: (dim, reads input)
    std::vector<std::pair<int, bool>> blocks;
    bool reads = false;
    std::function<void(const Desc&)> walk = [&](const Desc& d) {
      if (d.kind == Desc::APPEND) {
        for (auto& a : d.args) walk(a);
        return;
      }
      const Desc* b = &d;
      while (b->kind == Desc::OFFSET || b->kind == Desc::ROUND) b = &b->args[0];
      const bool is_in = b->kind == Desc::NODE && b->node == "input";
      reads = reads || is_in;
      blocks.push_back({is_in ? D : nn->DescDim(d), is_in});
    };
    walk(nd.input);
    if (!reads) continue;
    Component& c = nn->components.at(nd.component);
    if (!IsAffineType(c.type) && c.type != "TdnnComponent")
      VAMD_ERR("x-vector nnet: component " << nd.component << " (" << c.type
                                           << ") reads the input directly (unsupported)");
    if (c.type == "TdnnComponent") {
      if (blocks.size() != 1) VAMD_ERR("x-vector nnet: TdnnComponent input must be the plain input");
      blocks.assign(std::max<size_t>(1, c.time_offsets.size()), {D, true});
    }
    Matrix& W = c.m.count("LinearParams") ? c.m["LinearParams"] : c.m.at("Params");
    int K = 0;
    for (auto& b : blocks) K += b.first;
    if (K != W.cols) VAMD_ERR("x-vector nnet: input blocks of " << nd.component << " do not match its weights");
    int Kp = 0;
    for (auto& b : blocks) Kp += b.second ? Dp : b.first;
    Matrix P;
    P.rows = W.rows;
    P.cols = Kp;
    P.data.assign((size_t)P.rows * Kp, 0.0f);
    for (int r = 0; r < W.rows; r++) {
      int src = 0, dst = 0;
      for (auto& b : blocks) {
        memcpy(&P.data[(size_t)r * Kp + dst], &W.data[(size_t)r * W.cols + src], sizeof(float) * b.first);
        src += b.first;
        dst += b.second ? Dp : b.first;
      }
    }
    W = std::move(P);
  }
}
}  // namespace

void SpkModelData::Load(const std::string& d) {
  dir = d;
  mfcc.Apply(ReadConfigFile(d + "/mfcc.conf"));
  mfcc.allow_downsample = true;  // src/spk_model.cc:21
  ReadNnetRaw(d + "/final.ext.raw", &nnet);
  mean = ReadKaldiVectorFloat(d + "/mean.vec");
  transform = ReadKaldiMatrixFloat(d + "/transform.mat");
  feat_dim = mfcc.FeatDim();
  input_dim = (feat_dim + 7) / 8 * 8;
  if (!nnet.HasNode("input") || nnet.Node("input").dim != feat_dim)
    VAMD_ERR("speaker nnet input dim != MFCC dim " << feat_dim);
  if (transform.cols != (int)mean.size())
    VAMD_ERR("transform.mat has " << transform.cols << " columns, mean.vec " << mean.size());
  if (mfcc.dither != 0.0f)
    VAMD_WARN("speaker model dither=" << mfcc.dither << " ignored (deterministic front end)");
  PadInput(&nnet, feat_dim, input_dim);
}

int SpkNumFrames(const MfccOptions& o, long long n) {
  const long long L = o.WindowSize(), S = o.WindowShift();
  if (o.snip_edges) return n < L ? 0 : (int)(1 + (n - L) / S);
  // FeatureWindow NumFrames(flush=false) with snip_edges=false
  long long nf = (n + S / 2) / S;
  long long end = (nf - 1) * S + S / 2 - L / 2 + L;
  while (nf > 0 && end > n) {
    nf--;
    end -= S;
  }
  return (int)nf;
}

XvectorNet BuildXvectorNet(const SpkModelData& m, int fpc) {
  const Nnet& nn = m.nnet;
  XvectorNet x;
  std::string ext, pool;
  for (auto& nd : nn.nodes) {
    if (nd.kind != NnetNode::COMPONENT) continue;
    const std::string& t = nn.components.at(nd.component).type;
    if (t == "StatisticsExtractionComponent") ext = nd.name;
    if (t == "StatisticsPoolingComponent") pool = nd.name;
  }
  if (ext.empty() || pool.empty()) VAMD_ERR("speaker nnet has no statistics extraction / pooling layer");
  const NnetNode& en = nn.Node(ext);
  const NnetNode& pn = nn.Node(pool);
  if (en.input.kind != Desc::NODE) VAMD_ERR("statistics extraction input must be a plain node");
  if (pn.input.kind != Desc::NODE || pn.input.node != ext)
    VAMD_ERR("statistics pooling must read the extraction directly");
  const Component& ec = nn.components.at(en.component);
  const Component& pc = nn.components.at(pn.component);
  auto geti = [](const Component& c, const char* k, int dflt) {
    return c.i.count(k) ? c.i.at(k) : dflt;
  };
  if (geti(ec, "InputPeriod", 1) != 1 || geti(ec, "OutputPeriod", 1) != 1 || geti(pc, "InputPeriod", 1) != 1)
    VAMD_ERR("statistics periods other than 1 are not supported");
  const bool var = ec.b.count("IncludeVarinance") && ec.b.at("IncludeVarinance");
  x.stddevs = pc.b.count("OutputStddevs") && pc.b.at("OutputStddevs");
  if (x.stddevs && !var) VAMD_ERR("stddev pooling needs variance statistics");
  x.num_log_count = geti(pc, "NumLogCountFeatures", 0);
  x.variance_floor = pc.f.count("VarianceFloor") ? pc.f.at("VarianceFloor") : 1e-10f;
  x.pool_left = geti(pc, "LeftContext", 0);
  x.pool_right = geti(pc, "RightContext", 0);
  // frame-level part: the same network with "output" moved to the
  // statistics input
  Nnet fn = nn;
  if (!fn.HasNode("output")) VAMD_ERR("speaker nnet has no 'output' node");
  fn.nodes[fn.node_index.at("output")].input = en.input;
  x.frames = BuildNnetPlan(fn, fpc, 1, 1.0f);
  x.stats_in = nn.OutputDimOf(en.input.node);
  if (x.frames.input_dim != m.input_dim) VAMD_ERR("speaker nnet plan input dim mismatch");
  // head: the chain from the pooling node to "output"
  std::string cur = pool;
  int dim = x.num_log_count + x.stats_in * (x.stddevs ? 2 : 1);
  const NnetNode& out = nn.Node("output");
  while (true) {
    if (out.input.kind == Desc::NODE && out.input.node == cur) break;
    const NnetNode* next = nullptr;
    for (auto& nd : nn.nodes) {
      if (nd.kind != NnetNode::COMPONENT) continue;
      const Desc* d = &nd.input;
      if (d->kind == Desc::ROUND) d = &d->args[0];
      if (d->kind == Desc::NODE && d->node == cur) {
        if (next) VAMD_ERR("speaker nnet head must be a chain (" << cur << " has two consumers)");
        next = &nd;
      }
    }
    if (!next) VAMD_ERR("speaker nnet: no path from the pooling layer to 'output'");
    const Component& c = nn.components.at(next->component);
    XvectorNet::HeadOp op;
    op.in = dim;
    if (IsAffineType(c.type)) {
      const Matrix& W = c.m.count("LinearParams") ? c.m.at("LinearParams") : c.m.at("Params");
      if (W.cols != dim) VAMD_ERR("speaker nnet head: " << next->component << " expects " << W.cols);
      op.kind = XvectorNet::HeadOp::AFFINE;
      op.out = W.rows;
      op.w = W.data;
      if (c.v.count("BiasParams")) op.b = c.v.at("BiasParams");
      x.head.push_back(op);
      dim = W.rows;
    } else if (c.type == "RectifiedLinearComponent") {
      op.kind = XvectorNet::HeadOp::RELU;
      op.out = dim;
      x.head.push_back(op);
    } else if (c.type == "BatchNormComponent") {
      op.kind = XvectorNet::HeadOp::MUL_ADD;
      op.out = dim;
      BatchNormScaleOffset(c, &op.w, &op.b);
      x.head.push_back(op);
    } else if (c.type != "NoOpComponent" && c.type != "DropoutComponent" &&
               c.type != "GeneralDropoutComponent") {
      VAMD_ERR("unsupported component " << c.type << " in the speaker nnet head");
    }
    cur = next->name;
  }
  x.embed_dim = dim;
  if (dim != (int)m.mean.size()) VAMD_ERR("x-vector dim " << dim << " != mean.vec dim " << m.mean.size());
  if (dim > 1024) VAMD_ERR("x-vector dim above 1024 is not supported");
  return x;
}

void* SpkExtractor::DevAlloc(size_t bytes) {
  void* p = nullptr;
  XV_HIPCHECK(hipMalloc(&p, std::max<size_t>(bytes, 16)));
  allocs_.push_back(p);
  return p;
}

void SpkExtractor::DevFree(void* p) {
  if (!p) return;
  auto it = std::find(allocs_.begin(), allocs_.end(), p);
  if (it != allocs_.end()) allocs_.erase(it);
  (void)hipFree(p);
}

template <class T>
T* SpkExtractor::Upload(const std::vector<T>& v) {
  T* d = (T*)DevAlloc(sizeof(T) * v.size());
  if (!v.empty()) XV_HIPCHECK(hipMemcpy(d, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice));
  return d;
}

SpkExtractor::SpkExtractor(std::shared_ptr<const SpkModelData> m, int device)
    : md_(std::move(m)), device_(device) {
  XV_HIPCHECK(hipSetDevice(device_));
  XV_HIPCHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  for (hipEvent_t& e : ev_) XV_HIPCHECK(hipEventCreate(&e));
  net_ = BuildXvectorNet(*md_, 64);
  MfccTables t = BuildMfccTables(md_->mfcc);
  mfcc_ = t.dev;
  mfcc_.window = Upload(t.win);
  mfcc_.melw = Upload(t.melw);
  mfcc_.mel_first = Upload(t.first);
  mfcc_.mel_last = Upload(t.last);
  mfcc_.dct = Upload(t.dct);
  mfcc_.lifter = Upload(t.lift);
  mfcc_.twr = Upload(t.twr);
  mfcc_.twi = Upload(t.twi);
  for (auto& v : net_.frames.vecs) vec_ptrs_.push_back(Upload(v));
  d_vecs_ = Upload(vec_ptrs_);
  for (auto& op : net_.frames.ops) {
    if (op.kind == Op::GEMM) weights_.push_back(Upload(net_.frames.mats[op.weight].data));
    else weights_.push_back(nullptr);
    patterns_.push_back(Upload(op.pattern));
  }
  head_max_ = net_.num_log_count + net_.stats_in * 2;
  for (auto& h : net_.head) {
    head_w_.push_back(h.w.empty() ? nullptr : Upload(h.w));
    head_b_.push_back(h.b.empty() ? nullptr : Upload(h.b));
    head_max_ = std::max(head_max_, h.out);
  }
  d_mean_ = Upload(md_->mean);
  d_transform_ = Upload(md_->transform.data);
}

SpkExtractor::~SpkExtractor() {
  (void)hipSetDevice(device_);
  if (stream_) (void)hipStreamSynchronize(stream_);
  for (void* p : allocs_) (void)hipFree(p);
  if (h_xvec_) (void)hipHostFree(h_xvec_);
  for (hipEvent_t e : ev_)
    if (e) (void)hipEventDestroy(e);
  if (stream_) (void)hipStreamDestroy(stream_);
}

namespace {
long long Pow2Min(long long v, long long lo) {
  long long c = lo;
  while (c < v) c <<= 1;
  return c;
}
// caps of one launch sequence: utterance slots, and the frame-level rings'
// bytes (every node's ring holds an utterance's whole selection; the
// operator may lower it through VOSK_AMD_XVEC_RING_MB)
constexpr int kXvecMaxSlots = 256;
long long RingBudgetBytes() {
  const char* v = getenv("VOSK_AMD_XVEC_RING_MB");
  const long long mb = v ? atoll(v) : 8192;
  return std::max(1LL, mb) << 20;
}
}  // namespace

long long SpkExtractor::RingBytesPerSlot(int jobs_per_slot) const {
  long long dims = 0;
  for (auto& nd : net_.frames.nodes) dims += nd.dim;
  return (long long)net_.frames.RingFrames(jobs_per_slot) * dims * (long long)sizeof(float);
}

int SpkExtractor::TableIndex(int rate) {
  for (size_t i = 0; i < table_rates_.size(); i++)
    if (table_rates_[i] == rate) return (int)i;
  const int spk_rate = (int)std::lround(md_->mfcc.samp_freq);
  tables_.push_back(BuildResampleTable(rate, spk_rate));
  table_rates_.push_back(rate);
  std::vector<ResampleDev> devs;
  for (const ResampleTable& t : tables_) {
    ResampleDev td{};
    td.first = Upload(t.first);
    td.ntaps = Upload(t.ntaps);
    td.w = Upload(t.w);
    td.in_unit = t.in_unit;
    td.out_unit = t.out_unit;
    td.taps = t.taps;
    devs.push_back(td);
  }
  // the earlier tables' arrays are re-uploaded with the list (a handful of
  // rates per process); the old ones stay allocated until the destructor
  d_tables_ = Upload(devs);
  return (int)tables_.size() - 1;
}

void SpkExtractor::Reserve(int slots, long long samples, long long raw, int frames, int sel,
                           int jobs_per_slot, int jobs) {
  const NnetPlan& plan = net_.frames;
  const int R = std::max(1, md_->transform.rows);
  const bool grow = slots > slot_cap_;
  if (grow) {
    slot_cap_ = (int)Pow2Min(slots, 1);
    for (void* p : {(void*)d_utts_, (void*)d_mjobs_, (void*)d_stats_, (void*)d_head_, (void*)d_xvec_})
      DevFree(p);
    d_utts_ = (XvecUtt*)DevAlloc(sizeof(XvecUtt) * slot_cap_);
    d_mjobs_ = (MfccJob*)DevAlloc(sizeof(MfccJob) * slot_cap_);
    d_stats_ = (float*)DevAlloc(sizeof(float) * (size_t)slot_cap_ * head_max_);
    d_head_ = (float*)DevAlloc(sizeof(float) * 2 * (size_t)slot_cap_ * head_max_);
    d_xvec_ = (float*)DevAlloc(sizeof(float) * (size_t)slot_cap_ * R);
    if (h_xvec_) (void)hipHostFree(h_xvec_);
    h_xvec_ = nullptr;
    XV_HIPCHECK(hipHostMalloc((void**)&h_xvec_, sizeof(float) * (size_t)slot_cap_ * R, hipHostMallocDefault));
  }
  if (grow || samples + 1 > wave_len_) {
    wave_len_ = std::max(wave_len_, Pow2Min(samples + 1, 1024));
    DevFree(d_wave_);
    d_wave_ = (float*)DevAlloc(sizeof(float) * (size_t)slot_cap_ * wave_len_);
  }
  if (raw > 0 && (grow || raw + 1 > raw_len_)) {
    raw_len_ = std::max(raw_len_, Pow2Min(raw + 1, 1024));
    DevFree(d_raw_);
    d_raw_ = (float*)DevAlloc(sizeof(float) * (size_t)slot_cap_ * raw_len_);
  }
  if (grow || frames > feat_ring_) {
    feat_ring_ = std::max(feat_ring_, (int)Pow2Min(frames, 256));
    DevFree(d_feats_);
    d_feats_ = (float*)DevAlloc(sizeof(float) * (size_t)feat_ring_ * slot_cap_ * md_->feat_dim);
  }
  if (sel > sel_cap_) {
    sel_cap_ = (int)Pow2Min(sel, 256);
    DevFree(d_rows_);
    d_rows_ = (int*)DevAlloc(sizeof(int) * sel_cap_);
  }
  if (jobs > jobs_cap_) {
    jobs_cap_ = (int)Pow2Min(jobs, 16);
    DevFree(d_jobs_);
    DevFree(d_out_);
    d_jobs_ = (DevJob*)DevAlloc(sizeof(DevJob) * jobs_cap_);
    d_out_ = (float*)DevAlloc(sizeof(float) * (size_t)jobs_cap_ * plan.fpc * net_.stats_in);
  }
  if (!grow && jobs_per_slot <= slot_jobs_cap_) return;
  // node rings [ring][slot][dim] and the op arguments that point into them
  slot_jobs_cap_ = std::max(slot_jobs_cap_, jobs_per_slot);
  const int ring = plan.RingFrames(slot_jobs_cap_);
  for (float* p : ring_ptrs_) DevFree(p);
  ring_ptrs_.clear();
  std::vector<int> dims;
  for (auto& nd : plan.nodes) {
    const size_t bytes = sizeof(float) * (size_t)ring * slot_cap_ * nd.dim;
    ring_ptrs_.push_back((float*)DevAlloc(bytes));
    XV_HIPCHECK(hipMemset(ring_ptrs_.back(), 0, bytes));
    dims.push_back(nd.dim);
  }
  DevFree(d_ring_ptrs_);
  DevFree(d_ring_dims_);
  d_ring_ptrs_ = Upload(ring_ptrs_);
  d_ring_dims_ = Upload(dims);
  ring_ = ring;
  RingSet rs{};
  rs.base = d_ring_ptrs_;
  rs.dim = d_ring_dims_;
  rs.mask = ring - 1;
  rs.ring = ring;
  rs.slots = slot_cap_;
  rs.input_node = plan.input_node;
  auto is_in = [&](int node) { return node == plan.input_node ? 1 : 0; };
  op_args_.clear();
  op_bk_.clear();
  for (size_t oi = 0; oi < plan.ops.size(); oi++) {
    const Op& op = plan.ops[oi];
    NnetOpArgs a;
    memset(&a, 0, sizeof(a));
    a.N = op.N;
    a.K = op.K;
    a.P = (int)op.pattern.size();
    a.pattern = patterns_[oi];
    a.rings = rs;
    a.vecs = d_vecs_;
    a.out_node = op.out_node;
    a.out_base = op.out_node >= 0 ? ring_ptrs_[op.out_node] : nullptr;
    a.out_ldim = op.out_node >= 0 ? dims[op.out_node] : 0;
    int bk = 64;
    if (op.kind == Op::GEMM) {
      a.W = weights_[oi];
      if ((int)op.segs.size() > kMaxSegs) VAMD_ERR("too many input segments in op " << op.name);
      a.nsegs = (int)op.segs.size();
      for (size_t i = 0; i < op.segs.size(); i++) {
        const ASegment& s = op.segs[i];
        a.segs[i] = DevSeg{ring_ptrs_[s.node], dims[s.node], is_in(s.node), s.offset, s.col0, s.dim,
                           s.src_col};
        if (s.dim % 4 || s.src_col % 4 || dims[s.node] % 4)
          VAMD_ERR("speaker op " << op.name << ": segment dims must be multiples of 4");
        while (bk > 8 && (s.col0 % bk || s.dim % bk)) bk >>= 1;
        if (s.col0 % bk || s.dim % bk) VAMD_ERR("speaker op " << op.name << ": K segments must be multiples of 8");
      }
      if (op.K % 8) VAMD_ERR("speaker op " << op.name << ": K must be a multiple of 8");
      a.kslices = GemmKSlices(op.K);
      if (a.kslices > 1 && !GemmStreamable(a))
        VAMD_ERR("speaker op " << op.name << ": split-K op must fit the streaming GEMM kernel");
    } else {
      a.nparts = (int)op.parts.size();
      if (a.nparts > kMaxParts) VAMD_ERR("too many descriptor parts in op " << op.name);
      int ni = 0;
      for (size_t i = 0; i < op.parts.size(); i++) {
        const GPart& gp = op.parts[i];
        a.parts[i] = DevPart{gp.col0, gp.dim, ni, (int)gp.prog.size()};
        for (auto& g : gp.prog) {
          if (ni >= kMaxInstr) VAMD_ERR("descriptor program too long in op " << op.name);
          if (g.op == GInstr::PUSH_JOB) VAMD_ERR("speaker nnet with a per-chunk input is not supported");
          a.instr[ni++] = DevInstr{g.op == GInstr::PUSH ? ring_ptrs_[g.node] : nullptr, g.op,
                                   g.op == GInstr::PUSH ? dims[g.node] : 0,
                                   g.op == GInstr::PUSH ? is_in(g.node) : 0, g.offset, g.src_col, g.c};
        }
      }
    }
    if ((int)op.epi.size() > kMaxStages) VAMD_ERR("too many fused stages in op " << op.name);
    a.nstages = (int)op.epi.size();
    for (size_t i = 0; i < op.epi.size(); i++) {
      const EpiStage& e = op.epi[i];
      DevStage d;
      d.base = e.kind == EpiStage::ADD_NODE ? ring_ptrs_[e.node] : nullptr;
      d.v0 = e.vec0 >= 0 ? vec_ptrs_[e.vec0] : nullptr;
      d.v1 = e.vec1 >= 0 ? vec_ptrs_[e.vec1] : nullptr;
      d.kind = e.kind;
      d.ldim = e.kind == EpiStage::ADD_NODE ? dims[e.node] : 0;
      d.is_input = e.kind == EpiStage::ADD_NODE ? is_in(e.node) : 0;
      d.offset = e.offset;
      d.src_col = e.src_col;
      d.scaled = e.scaled ? 1 : 0;
      d.c = e.c;
      a.stages[i] = d;
    }
    if (op.out_node < 0 && a.P != plan.fpc) VAMD_ERR("speaker nnet output op pattern");
    op_args_.push_back(a);
    op_bk_.push_back(bk);
  }
}

bool SpkExtractor::Extract(const float* samples, long long n, int rate, int first_frame,
                           const std::vector<char>& keep, std::vector<float>* xvec, int* num_frames) {
  if (rate <= 0) VAMD_ERR("bad sample rate " << rate);
  if (n < 0) VAMD_ERR("bad sample count " << n);
  XvecRequest r;
  r.samples = samples;
  r.n = n;
  r.rate = rate;
  r.first_frame = first_frame;
  r.keep = &keep;
  r.xvec = xvec;
  Pending p{&r};
  // group commit: the first caller to find no batch running takes the whole
  // queue (its own request included) and runs it; the others wait
  std::unique_lock<std::mutex> lk(qmu_);
  queue_.push_back(&p);
  while (!p.done) {
    if (leader_) {
      qcv_.wait(lk);
      continue;
    }
    leader_ = true;
    std::vector<Pending*> batch(queue_.begin(), queue_.end());
    queue_.clear();
    lk.unlock();
    std::vector<XvecRequest*> reqs;
    for (Pending* q : batch) reqs.push_back(q->r);
    std::exception_ptr err;
    try {
      std::lock_guard<std::mutex> dev(mu_);
      RunBatch(reqs);
    } catch (...) {
      err = std::current_exception();
    }
    lk.lock();
    for (Pending* q : batch) {
      q->done = true;
      q->err = err;
    }
    leader_ = false;
    qcv_.notify_all();
  }
  lk.unlock();
  if (p.err) std::rethrow_exception(p.err);
  *num_frames = r.num_frames;
  return r.ok;
}

void SpkExtractor::ExtractBatch(const std::vector<XvecRequest*>& reqs) {
  for (XvecRequest* r : reqs) {
    if (r->rate <= 0) VAMD_ERR("bad sample rate " << r->rate);
    if (r->n < 0) VAMD_ERR("bad sample count " << r->n);
  }
  std::lock_guard<std::mutex> dev(mu_);
  RunBatch(reqs);
}

void SpkExtractor::RunBatch(const std::vector<XvecRequest*>& reqs) {
  XV_HIPCHECK(hipSetDevice(device_));
  const NnetPlan& plan = net_.frames;
  const int spk_rate = (int)std::lround(md_->mfcc.samp_freq);
  const int P = plan.priming_chunks, fpc = plan.fpc;
  // the usable frame-level rows of an utterance: computable from its frames
  // [0, sel) and inside the pooling window of output time 0
  const int r_lo = std::max(plan.left_context, -net_.pool_left);
  struct Utt {
    XvecRequest* r;
    long long n;  // samples at the speaker rate
    int nfr, sel, rows0, njobs, table, r_hi;
  };
  std::vector<Utt> us;
  std::vector<int> rows;
  for (XvecRequest* r : reqs) {
    r->ok = false;
    r->num_frames = 0;
    long long n = r->n;
    int table = -1;
    if (r->rate != spk_rate) {
      table = TableIndex(r->rate);
      n = tables_[table].NumOutputSamples(r->n, false);
    }
    const int nfr = SpkNumFrames(md_->mfcc, n);
    const int rows0 = (int)rows.size();
    const std::vector<char>& keep = *r->keep;
    for (int i = std::max(0, r->first_frame); i < nfr; i++) {
      const size_t k = (size_t)((i - r->first_frame) / 3);
      if (k < keep.size() && keep[k]) rows.push_back(i);
    }
    const int sel = (int)rows.size() - rows0;
    r->num_frames = sel;
    const int r_hi = std::min(sel - 1 - plan.right_context, net_.pool_right);
    if (sel < 50 || r_lo > r_hi) {  // MIN_SPK_FEATS, src/recognizer.cc:354
      rows.resize(rows0);
      continue;
    }
    us.push_back(Utt{r, n, nfr, sel, rows0, P + (sel + fpc - 1) / fpc, table, r_hi});
  }
  const int R = md_->transform.rows;
  const long long budget = RingBudgetBytes();
  for (size_t a = 0; a < us.size();) {
    // this launch sequence's utterances: up to the slot cap and ring budget
    size_t b = a;
    int max_jobs = 0;
    while (b < us.size() && (int)(b - a) < kXvecMaxSlots) {
      const int mj = std::max(max_jobs, us[b].njobs);
      if (b > a && RingBytesPerSlot(mj) * (long long)Pow2Min((long long)(b - a + 1), 1) > budget) break;
      max_jobs = mj;
      b++;
    }
    const int B = (int)(b - a);
    long long max_n = 0, max_raw = 0;
    int max_nfr = 0, total_jobs = 0;
    for (size_t k = a; k < b; k++) {
      max_n = std::max(max_n, us[k].n);
      if (us[k].table >= 0) max_raw = std::max(max_raw, us[k].r->n);
      max_nfr = std::max(max_nfr, us[k].nfr);
      total_jobs += us[k].njobs;
    }
    const int sel0 = us[a].rows0;
    const int nsel = us[b - 1].rows0 + us[b - 1].sel - sel0;
    Reserve(B, max_n, max_raw, max_nfr, nsel, max_jobs, total_jobs);
    // samples (resampled per utterance where the rate differs)
    const int per = 4096;
    std::vector<ResampleJob> rj;
    for (int k = 0; k < B; k++) {
      const Utt& u = us[a + k];
      if (u.table < 0) {
        XV_HIPCHECK(hipMemcpyAsync(d_wave_ + (size_t)k * wave_len_, u.r->samples, sizeof(float) * u.n,
                                   hipMemcpyHostToDevice, stream_));
      } else {
        XV_HIPCHECK(hipMemcpyAsync(d_raw_ + (size_t)k * raw_len_, u.r->samples, sizeof(float) * u.r->n,
                                   hipMemcpyHostToDevice, stream_));
        for (long long p0 = 0; p0 < u.n; p0 += per)
          rj.push_back(ResampleJob{k, (int)p0, (int)std::min<long long>(per, u.n - p0), u.table, p0, u.r->n});
      }
    }
    if (!rj.empty()) {
      if ((int)rj.size() > rjobs_cap_) {
        DevFree(d_rjobs_);
        rjobs_cap_ = (int)Pow2Min((long long)rj.size(), 16);
        d_rjobs_ = (ResampleJob*)DevAlloc(sizeof(ResampleJob) * rjobs_cap_);
      }
      XV_HIPCHECK(hipMemcpyAsync(d_rjobs_, rj.data(), sizeof(ResampleJob) * rj.size(), hipMemcpyHostToDevice,
                                 stream_));
      LaunchResample(d_rjobs_, (int)rj.size(), d_tables_, d_raw_, (int)raw_len_, d_wave_, (int)wave_len_,
                     stream_);
    }
    // speaker MFCC of every frame of every utterance, slot k of the feature ring
    std::vector<MfccJob> mj(B);
    std::vector<XvecUtt> ut(B);
    std::vector<DevJob> jobs;
    int mrows = 0;
    for (int k = 0; k < B; k++) {
      const Utt& u = us[a + k];
      mj[k] = MfccJob{k, 0, u.nfr, mrows};
      mrows += u.nfr;
      const int job0 = (int)jobs.size();
      for (int j = 0; j < u.njobs; j++) jobs.push_back(DevJob{k, (j - P) * fpc, u.sel - 1, 0});
      // frame-level output row of the utterance's time t: (job0 + P) * fpc + t
      ut[k] = XvecUtt{u.rows0 - sel0, u.sel, (job0 + P) * fpc + r_lo, u.r_hi - r_lo + 1};
    }
    XV_HIPCHECK(hipMemcpyAsync(d_mjobs_, mj.data(), sizeof(MfccJob) * B, hipMemcpyHostToDevice, stream_));
    XV_HIPCHECK(hipMemcpyAsync(d_utts_, ut.data(), sizeof(XvecUtt) * B, hipMemcpyHostToDevice, stream_));
    XV_HIPCHECK(hipMemcpyAsync(d_rows_, rows.data() + sel0, sizeof(int) * nsel, hipMemcpyHostToDevice, stream_));
    XV_HIPCHECK(hipMemcpyAsync(d_jobs_, jobs.data(), sizeof(DevJob) * jobs.size(), hipMemcpyHostToDevice,
                               stream_));
    MfccDev m = mfcc_;
    m.out = d_feats_;
    RingSet fr{};
    fr.mask = feat_ring_ - 1;
    fr.ring = feat_ring_;
    fr.slots = slot_cap_;
    LaunchMfcc(m, d_mjobs_, B, mrows, d_wave_, (int)wave_len_, fr, stream_);
    LaunchXvecCmn(d_feats_, feat_ring_ - 1, slot_cap_, md_->feat_dim, d_rows_, d_utts_, B, 300,
                  ring_ptrs_[plan.input_node], ring_ - 1, slot_cap_, md_->input_dim, stream_);
    // the frame-level layers: every op over all utterances' jobs at once
    // (HIP events on the extractor's stream bracket them: the GEMM roofline)
    XV_HIPCHECK(hipEventRecord(ev_[0], stream_));
    for (size_t i = 0; i < plan.ops.size(); i++) {
      NnetOpArgs op = op_args_[i];
      op.M = total_jobs * op.P;
      op.jobs = d_jobs_;
      op.llh = d_out_;
      if (plan.ops[i].kind == Op::GEMM) {
        LaunchNnetGemm(op, op_bk_[i], stream_);
        gemm_flops_ += 2.0 * op.M * (double)op.N * (double)op.K;
      } else {
        LaunchNnetGather(op, stream_);
      }
    }
    XV_HIPCHECK(hipEventRecord(ev_[1], stream_));
    LaunchXvecPool(d_out_, net_.stats_in, d_utts_, B, net_.stats_in, net_.num_log_count, net_.stddevs ? 1 : 0,
                   net_.variance_floor, d_stats_, head_max_, stream_);
    const float* x = d_stats_;
    for (size_t k = 0; k < net_.head.size(); k++) {
      const auto& h = net_.head[k];
      float* y = d_head_ + (k % 2) * (size_t)slot_cap_ * head_max_;
      LaunchXvecAffine(head_w_[k], head_b_[k], x, h.in, h.out, h.kind, y, head_max_, B, stream_);
      x = y;
    }
    LaunchXvecFinish(x, head_max_, d_mean_, net_.embed_dim, d_transform_, R, d_xvec_, B, stream_);
    XV_HIPCHECK(hipMemcpyAsync(h_xvec_, d_xvec_, sizeof(float) * (size_t)B * R, hipMemcpyDeviceToHost, stream_));
    XV_HIPCHECK(hipStreamSynchronize(stream_));
    float ms = 0.0f;
    XV_HIPCHECK(hipEventElapsedTime(&ms, ev_[0], ev_[1]));
    layers_ms_ += ms;
    for (int k = 0; k < B; k++) {
      XvecRequest* r = us[a + k].r;
      r->xvec->assign(h_xvec_ + (size_t)k * R, h_xvec_ + (size_t)(k + 1) * R);
      r->ok = true;
    }
    batches_++;
    utterances_ += B;
    a = b;
  }
}

}  // namespace vamd
