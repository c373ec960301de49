// Kaldi's LatticeIncrementalDecoder token bookkeeping and
// LatticeIncrementalDeterminizer on the host (see incremental.h).
// Restated by tests/oracle_incremental.py, function for function.
#include "incremental.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <limits>
#include <memory>

#include "common.h"
#include "model_io.h"

namespace vamd {

// per-thread phase times (the host-only test ABI reports them)
thread_local double vamd_inc_prof[6];  // (development) ms: add frame, prune, chunk build, determinize, accept, set finals
struct IncProf {
  int k;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  explicit IncProf(int i) : k(i) {}
  ~IncProf() { vamd_inc_prof[k] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); }
};

namespace {
constexpr float kInf = std::numeric_limits<float>::infinity();

inline LW Times(const LW& x, const LW& y) { return LW{x.g + y.g, x.a + y.a}; }
// ConvertToCost(LatticeWeight) is a double; Kaldi stores forward costs as float
inline float FwdPlus(float fwd, const LW& w) { return (float)((double)fwd + ((double)w.g + (double)w.a)); }

// kaldi-math ApproxEqual
inline bool ApproxEqual(float a, float b, float tol) {
  if (a == b) return true;
  const float diff = std::fabs(a - b);
  if (diff == kInf || diff != diff) return false;
  return diff <= tol * (std::fabs(a) + std::fabs(b));
}

// CompactLatticeWeight Compare: LatticeWeight (total cost, then graph cost),
// then the shorter string, then the lexicographically larger one
int CompareCW(const LW& w1, const std::vector<int>& s1, const LW& w2, const std::vector<int>& s2) {
  const float f1 = w1.g + w1.a, f2 = w2.g + w2.a;
  if (f1 < f2) return 1;
  if (f1 > f2) return -1;
  if (w1.g < w2.g) return 1;
  if (w1.g > w2.g) return -1;
  if (s1.size() > s2.size()) return -1;
  if (s1.size() < s2.size()) return 1;
  for (size_t i = 0; i < s1.size(); i++) {
    if (s1[i] < s2[i]) return -1;
    if (s1[i] > s2[i]) return 1;
  }
  return 0;
}

// AddCompactLatticeArcToLattice: a chain of one-transition-id links, label
// and weight on the first (intermediate states in the source's bucket)
void AddChain(DetGraph* D, int src, int dst, int label, const LW& w, const std::vector<int>& tids) {
  const size_t n = tids.size();
  if (n == 0) {
    D->links.push_back(DetGraph::Link{src, dst, 0, label, w.g, w.a});
    return;
  }
  int cur = src;
  for (size_t i = 0; i < n; i++) {
    const int nx = i + 1 == n ? dst : D->AddState(D->frame[src]);
    D->links.push_back(DetGraph::Link{cur, nx, tids[i], i == 0 ? label : 0, i == 0 ? w.g : 0.0f, i == 0 ? w.a : 0.0f});
    cur = nx;
  }
}
}  // namespace

void IncrementalLattice::Init(const Graph* g, const std::vector<int>* tid2phone, const std::vector<char>* tid_first,
                              const IncrementalOptions& opt) {
  g_ = g;
  tid2phone_ = tid2phone;
  tid_first_ = tid_first;
  opt_ = opt;
  // address space for ~20 s of tokens at the bench model's density up front
  // (32 MB): the pages are touched only as tokens come, and the array is
  // never moved while it grows (a 20-s segment has ~1.4 M tokens)
  if (toks_.capacity() < (1u << 21)) toks_.reserve(1u << 21);
  Reset();
}

void IncrementalLattice::Reset() {
  toks_.clear();
  frames_.clear();
  finalized_ = failed_ = false;
  final_costs_.clear();
  final_best_cost_ = 0;
  num_in_lattice_ = 0;
  token2label_.clear();
  next_label_ = kTokenLabelOffset;
  chunks_ = prune_passes_ = 0;
  deferred_.clear();
  DetInit();
}

// ---------------------------------------------------------------------------
// token bookkeeping (LatticeIncrementalDecoderTpl)
// ---------------------------------------------------------------------------
template <class F>
void IncrementalLattice::ForLinks(int t, F&& f) {
  const HTok& tk = toks_[t];
  HFrame& fr = frames_[tk.frame];
  const int local = t - fr.first;
  if (!fr.emit_rng.empty())
    for (int i = fr.emit_rng[local].b; i < fr.emit_rng[local].e; i++)
      if (fr.emit[i].arc >= 0) f(fr.emit[i]);
  for (int i = fr.eps_rng[local].b; i < fr.eps_rng[local].e; i++)
    if (fr.eps[i].arc >= 0) f(fr.eps[i]);
}

void IncrementalLattice::AddFrame(const IncFrameIn& in) {
  const int k = (int)frames_.size();
  if (k > 0) {
    // AdvanceDecoding: "if (NumFramesDecoded() % config_.prune_interval == 0)
    // PruneActiveTokens(lattice_beam * prune_scale)" before each frame
    if (opt_.prune_interval > 0 && (k - 1) % opt_.prune_interval == 0) PruneActiveTokens(Delta());
    frames_[k - 1].cost_offset = in.cost_offset;
  }
  IncProf prof(0);
  frames_.emplace_back();
  HFrame& fr = frames_.back();
  const int base = (int)toks_.size();
  fr.first = base;
  fr.toks.reserve(in.ntok);
  for (int i = 0; i < in.ntok; i++) {
    toks_.push_back(HTok{in.state[i], in.cost[i], 0.0f, k, true});
    fr.toks.push_back(base + i);
  }
  // split the links: emitting ones belong to the previous frame's tokens
  // (the graph's weights are the only scattered reads; labels are read for
  // the links a chunk keeps)
  const int prev_n = k > 0 ? base - frames_[k - 1].first : 0;
  std::vector<int>& ce = scratch_ce_;
  std::vector<int>& cp = scratch_cp_;
  ce.assign(prev_n + 1, 0);
  cp.assign(in.ntok + 1, 0);
  for (int i = 0; i < in.nlinks; i++) {
    const IncFrameIn::Link& l = in.links[i];
    if (l.emit && k == 0) VAMD_ERR("incremental lattice: an emitting link into frame 0");
    if (l.dst < 0 || l.dst >= in.ntok || l.src < 0 || l.src >= (l.emit ? prev_n : in.ntok))
      VAMD_ERR("incremental lattice: link to a missing token");
    (l.emit ? ce : cp)[l.src + 1]++;
  }
  for (int i = 0; i < prev_n; i++) ce[i + 1] += ce[i];
  for (int i = 0; i < in.ntok; i++) cp[i + 1] += cp[i];
  std::vector<HLink> em(ce[prev_n]), ep(cp[in.ntok]);
  const float* wt = g_->weight.data();
  for (int i = 0; i < in.nlinks; i++) {
    const IncFrameIn::Link& l = in.links[i];
    if (i + 16 < in.nlinks) __builtin_prefetch(wt + in.links[i + 16].arc);  // scattered graph reads
    const HLink h{base + l.dst, l.arc, wt[l.arc], l.emit ? l.ac : 0.0f};
    if (l.emit) em[ce[l.src]++] = h;
    else ep[cp[l.src]++] = h;
  }
  // ce[i] / cp[i] now end source i's links (and begin i + 1's)
  std::vector<Rng>& rp = fr.eps_rng;
  rp.resize(in.ntok);
  for (int i = 0; i < in.ntok; i++) rp[i] = Rng{i ? cp[i - 1] : 0, cp[i]};
  std::vector<Rng> re_none;
  std::vector<Rng>& re = k > 0 ? frames_[k - 1].emit_rng : re_none;
  re.resize(prev_n);
  for (int i = 0; i < prev_n; i++) re[i] = Rng{i ? ce[i - 1] : 0, ce[i]};
  auto sort_range = [](HLink* a, int n) {  // by graph arc; ranges are short (insertion sort)
    for (int i = 1; i < n; i++) {
      const HLink x = a[i];
      int j = i - 1;
      for (; j >= 0 && a[j].arc > x.arc; j--) a[j + 1] = a[j];
      a[j + 1] = x;
    }
  };
  for (int i = 0; i < prev_n; i++) sort_range(em.data() + re[i].b, re[i].e - re[i].b);
  for (int i = 0; i < in.ntok; i++) sort_range(ep.data() + rp[i].b, rp[i].e - rp[i].b);
  fr.eps.swap(ep);
  if (k > 0) frames_[k - 1].emit.swap(em);
}

// PruneForwardLinks: the extra costs of frame f's tokens from their links'
// destinations, links beyond lattice_beam removed, iterated until no extra
// cost moves by more than delta (the links are not in topological order)
void IncrementalLattice::PruneForwardLinks(int f, bool* extra_costs_changed, bool* links_pruned, float delta) {
  *extra_costs_changed = false;
  *links_pruned = false;
  HFrame& fr = frames_[f];
  const bool has_emit = !fr.emit_rng.empty();
  HTok* const T = toks_.data();
  const float beam = opt_.lattice_beam;
  bool pruned = false;
  // a token's links of one kind: an excised one leaves its range (the rest
  // move down in order), so later passes do not visit it again
  auto links = [&](HLink* a, Rng& r, float tot, float* tok_extra) {
    int w = r.b;
    for (int i = r.b; i < r.e; i++) {
      const HLink l = a[i];
      if (l.arc < 0) continue;  // (excised by PruneForwardLinksFinal)
      const HTok& nt = T[l.dst];
      float link_extra = nt.extra + ((tot + l.ac + l.graph) - nt.tot);
      if (!nt.alive || link_extra > beam) {  // excise
        pruned = true;
        continue;
      }
      if (link_extra < 0.0f) link_extra = 0.0f;
      if (link_extra < *tok_extra) *tok_extra = link_extra;
      a[w++] = l;
    }
    r.e = w;
  };
  // one sweep over the frame's tokens in list order (Gauss-Seidel: an epsilon
  // link sees the destination's value of this sweep when it came earlier)
  auto sweep = [&](int t) {
    HTok& tk = T[t];
    float tok_extra = kInf;
    const int local = t - fr.first;
    if (has_emit) links(fr.emit.data(), fr.emit_rng[local], tk.tot, &tok_extra);
    Rng& rp = fr.eps_rng[local];
    links(fr.eps.data(), rp, tk.tot, &tok_extra);
    const bool ch = std::fabs(tok_extra - tk.extra) > delta;
    tk.extra = tok_extra;
    return std::make_pair(ch, rp.e > rp.b);
  };
  // the first sweep visits every token; a later one (Kaldi's loop "until no
  // extra cost moved by more than delta") only the tokens with epsilon links
  // left: a token with emitting links only gets the same value again (the
  // next frame's extra costs do not move here), so skipping it changes
  // nothing
  bool changed = false;
  std::vector<int> eps_toks;
  for (int t : fr.toks) {
    const auto r = sweep(t);
    changed |= r.first;
    if (r.second) eps_toks.push_back(t);
  }
  while (changed) {
    *extra_costs_changed = true;
    changed = false;
    for (int t : eps_toks) changed |= sweep(t).first;
  }
  *links_pruned = pruned;
}

void IncrementalLattice::PruneTokensForFrame(int f) {
  HFrame& fr = frames_[f];
  size_t m = 0;
  for (size_t i = 0; i < fr.toks.size(); i++) {
    HTok& tk = toks_[fr.toks[i]];
    if (tk.extra == kInf) {
      tk.alive = false;
      continue;
    }
    fr.toks[m++] = fr.toks[i];
  }
  fr.toks.resize(m);
  fr.num_toks = (int)m;
}

// PruneActiveTokens.  The next chunk holds frames N = NumFramesInLattice()
// on; the walk's steps below N (forward links of frames B = N - 1 and down,
// tokens of frames N - 1 and down) are read again only when a GetLattice
// starts over from frame 0 (a final start state; FinalizeDecoding then too).
// So that part of each pass is deferred: the pass records where it would
// continue (B, delta, whether frame B's flag was raised, and frame N's extra
// costs and liveness as the step read them), prunes frame N's tokens (the
// step's other half, which the chunk reads), and ReplayDeferred runs the
// recorded parts in order before a start-over, which then finds every frame
// as the eager walk leaves it (the deferred part reads nothing above frame
// N, and nothing else writes frames below it).
void IncrementalLattice::PruneActiveTokens(float delta) {
  IncProf prof(1);
  const int cur = NumFramesDecoded();
  prune_passes_++;
  // the current frame's tokens are not pruned, so they are counted here
  // (UpdateLatticeDeterminization reads every frame's count)
  if (frames_[cur].num_toks == -1) frames_[cur].num_toks = (int)frames_[cur].toks.size();
  const int B = num_in_lattice_ - 1;
  for (int f = cur - 1; f >= 0; f--) {
    if (f == B && B + 1 < cur) {
      DeferredPass d;
      d.B = B;
      d.delta = delta;
      d.fl = frames_[B].must_prune_fl;
      frames_[B].must_prune_fl = false;  // (raised again from d.fl when the part runs)
      const int t0 = frames_[B + 1].first, t1 = frames_[B + 2].first;
      d.extra.resize(t1 - t0);
      d.alive.resize(t1 - t0);
      for (int t = t0; t < t1; t++) {
        d.extra[t - t0] = toks_[t].extra;
        d.alive[t - t0] = toks_[t].alive;
      }
      deferred_.push_back(std::move(d));
      if (frames_[B + 1].must_prune_tok) {  // the step's eager half: frame B + 1's tokens
        PruneTokensForFrame(B + 1);
        frames_[B + 1].must_prune_tok = false;
      }
      break;
    }
    if (frames_[f].must_prune_fl) {
      bool ec = false, lp = false;
      PruneForwardLinks(f, &ec, &lp, delta);
      if (ec && f > 0) frames_[f - 1].must_prune_fl = true;
      if (lp) frames_[f].must_prune_tok = true;
      frames_[f].must_prune_fl = false;
    }
    if (f + 1 < cur && frames_[f + 1].must_prune_tok) {
      PruneTokensForFrame(f + 1);
      frames_[f + 1].must_prune_tok = false;
    }
  }
}

void IncrementalLattice::ReplayDeferred() {
  for (DeferredPass& d : deferred_) {
    const int B = d.B, t0 = frames_[B + 1].first;
    std::vector<float> x(d.extra.size());
    std::vector<char> al(d.alive.size());
    for (size_t i = 0; i < x.size(); i++) {  // frame B + 1 as the pass saw it
      HTok& tk = toks_[t0 + i];
      x[i] = tk.extra;
      al[i] = tk.alive;
      tk.extra = d.extra[i];
      tk.alive = d.alive[i];
    }
    if (d.fl) frames_[B].must_prune_fl = true;
    for (int f = B; f >= 0; f--) {
      if (frames_[f].must_prune_fl) {
        bool ec = false, lp = false;
        PruneForwardLinks(f, &ec, &lp, d.delta);
        if (ec && f > 0) frames_[f - 1].must_prune_fl = true;
        if (lp) frames_[f].must_prune_tok = true;
        frames_[f].must_prune_fl = false;
      }
      if (f < B && frames_[f + 1].must_prune_tok) {
        PruneTokensForFrame(f + 1);
        frames_[f + 1].must_prune_tok = false;
      }
    }
    for (size_t i = 0; i < x.size(); i++) {
      toks_[t0 + i].extra = x[i];
      toks_[t0 + i].alive = al[i];
    }
  }
  deferred_.clear();
}

// ComputeFinalCosts over the last frame's tokens (list order)
void IncrementalLattice::ComputeFinalCosts(std::unordered_map<int, float>* fc, float* final_best_cost) const {
  fc->clear();
  float best = kInf, best_with_final = kInf;
  for (int t : frames_.back().toks) {
    const HTok& tk = toks_[t];
    const float f = g_->final_cost[tk.state];
    const float cost = tk.tot, cwf = cost + f;
    best = std::min(best, cost);
    best_with_final = std::min(best_with_final, cwf);
    if (f != kInf) (*fc)[t] = f;
  }
  *final_best_cost = best_with_final != kInf ? best_with_final : best;
}

void IncrementalLattice::PruneForwardLinksFinal() {
  ComputeFinalCosts(&final_costs_, &final_best_cost_);
  finalized_ = true;
  const int F = NumFramesDecoded();
  const float delta = 1.0e-05f;
  bool changed = true;
  while (changed) {
    changed = false;
    for (int t : frames_[F].toks) {
      HTok& tk = toks_[t];
      float final_cost;
      if (final_costs_.empty()) {
        final_cost = 0.0f;
      } else {
        auto it = final_costs_.find(t);
        final_cost = it != final_costs_.end() ? it->second : kInf;
      }
      float tok_extra = (tk.tot + final_cost) - final_best_cost_;
      ForLinks(t, [&](HLink& l) {
        const HTok& nt = toks_[l.dst];
        float link_extra = nt.extra + ((tk.tot + l.ac + l.graph) - nt.tot);
        if (!nt.alive || link_extra > opt_.lattice_beam) {
          l.arc = -1;
          return;
        }
        if (link_extra < 0.0f) link_extra = 0.0f;
        if (link_extra < tok_extra) tok_extra = link_extra;
      });
      if (tok_extra > opt_.lattice_beam) tok_extra = kInf;
      if (!ApproxEqual(tk.extra, tok_extra, delta)) changed = true;
      tk.extra = tok_extra;
    }
  }
}

void IncrementalLattice::FinalizeDecoding() {
  if (frames_.empty() || finalized_) return;
  const int F = NumFramesDecoded();
  PruneForwardLinksFinal();
  // Kaldi walks every frame.  What the walk does below frame N - 1 (N =
  // NumFramesInLattice(), already determinized) reaches no later output: the
  // final chunk holds frames N.., whose tokens' extra costs come from the
  // frames after them, and the walk's step at N - 1 prunes frame N's tokens.
  // So the walk stops there -- unless the next GetLattice starts over from
  // frame 0 (no chunk yet, or a final start state).
  const bool restart = num_in_lattice_ == 0 || carcs_.empty() || cfin_[0].is;
  const int lo = restart ? 0 : num_in_lattice_ - 1;
  if (restart) ReplayDeferred();
  for (int f = F - 1; f >= lo; f--) {
    bool b1, b2;
    PruneForwardLinks(f, &b1, &b2, 0.0f);
    PruneTokensForFrame(f + 1);
  }
  if (lo == 0) PruneTokensForFrame(0);
}

// UpdateLatticeDeterminization
void IncrementalLattice::AdvanceEnd() {
  if (frames_.empty() || finalized_ || failed_) return;
  if (NumFramesDecoded() - num_in_lattice_ < opt_.determinize_max_delay) return;
  PruneActiveTokens(Delta());
  const int first = num_in_lattice_ + opt_.determinize_min_chunk_size, last = NumFramesDecoded();
  int fewest = std::numeric_limits<int>::max(), best = -1;
  for (int t = last; t >= first; t--) {
    if (frames_[t].num_toks == -1) VAMD_ERR("incremental lattice: token count not computed");
    if (frames_[t].num_toks < fewest) {
      fewest = frames_[t].num_toks;
      best = t;
    }
  }
  if (best < 0) return;
  GetLattice(best, false, nullptr);
}

bool IncrementalLattice::GetLattice(int M, bool use_final, WordLattice* out) {
  if (out) *out = WordLattice();
  if (failed_) return false;
  if (M < num_in_lattice_ || M > NumFramesDecoded()) VAMD_ERR("incremental lattice: frame range");
  if (num_in_lattice_ > 0 && carcs_.empty()) {  // failed earlier: stays empty
    num_in_lattice_ = M;
    return true;
  }
  if (M > num_in_lattice_) {
    PruneActiveTokens(Delta());
    // a start state that is final (the previous chunk's start reached its
    // last frame without a word) cannot be re-determinized: start over
    if (carcs_.empty() || cfin_[0].is) {
      ReplayDeferred();
      num_in_lattice_ = 0;
      DetInit();
    }
    BuildChunk(M);
    num_in_lattice_ = M;
    if (failed_) return false;
  }
  if (carcs_.empty()) return true;
  std::unordered_map<int, float> lfc;
  if (use_final) {
    std::unordered_map<int, float> t2f;
    float fb;
    ComputeFinalCosts(&t2f, &fb);
    for (auto& p : t2f) {
      auto it = token2label_.find(p.first);
      if (it != token2label_.end()) lfc[it->second] = p.second;
    }
  }
  SetFinalCosts(lfc.empty() ? nullptr : &lfc);
  if (out) ExportClat(out);
  return true;
}

// GetLattice's raw chunk (frames N = NumFramesInLattice() .. M), with
// InitializeRawLatticeChunk's part for a later chunk, then
// AcceptRawLatticeChunk.  Buckets (DetGraph::frame): the start 0, a
// re-determinized state 1 + its depth in the re-determinized part, then one
// per frame from N, then the token-final states.
void IncrementalLattice::BuildChunk(int M) {
  std::unique_ptr<IncProf> prof(new IncProf(2));
  const int N = num_in_lattice_;
  DetGraph D;
  std::unordered_map<int, int> label2state;  // token_label2state
  int T0 = 0;
  if (N != 0) {
    D.start = D.AddState(0);
    const std::vector<int> R(redet_.begin(), redet_.end());
    // depth of each re-determinized state (longest path inside the part)
    std::unordered_map<int, int> depth, indeg;
    for (int r : R) depth[r] = 0, indeg[r] = 0;
    for (int r : R)
      for (const CArc& a : carcs_[r]) indeg[a.next]++;
    std::vector<int> st;
    for (auto it = R.rbegin(); it != R.rend(); ++it)
      if (indeg[*it] == 0) st.push_back(*it);
    int maxd = 0;
    while (!st.empty()) {
      const int u = st.back();
      st.pop_back();
      maxd = std::max(maxd, depth[u]);
      for (const CArc& a : carcs_[u]) {
        depth[a.next] = std::max(depth[a.next], depth[u] + 1);
        if (--indeg[a.next] == 0) st.push_back(a.next);
      }
    }
    std::unordered_map<int, int> r2d;
    for (int r : R) r2d[r] = D.AddState(1 + depth[r]);
    for (int r : R)
      for (const CArc& a : carcs_[r]) AddChain(&D, r2d[r], r2d.at(a.next), a.label, a.w, a.tids);
    T0 = maxd + 2;
    for (const CArc& fa : final_arcs_) {
      auto it = label2state.find(fa.label);
      if (it == label2state.end()) it = label2state.emplace(fa.label, D.AddState(T0)).first;
      auto sit = r2d.find(fa.next);  // (an inaccessible source: Kaldi's redet_state_map[] gives state 0)
      AddChain(&D, sit != r2d.end() ? sit->second : D.start, it->second, 0, fa.w, fa.tids);
    }
    for (int r : R) D.links.push_back(DetGraph::Link{D.start, r2d[r], 0, kStateLabelOffset + r, fwd_[r], 0.0f});
    for (int r : R) {  // their arcs are re-created from the chunk
      carcs_[r].clear();
      cfin_[r] = CFin{};
    }
  }
  // token -> chunk state (the chunk's tokens are the toks_ range of its frames)
  const int tbase = frames_[N].first;
  const int tend = M + 1 < (int)frames_.size() ? frames_[M + 1].first : (int)toks_.size();
  std::vector<int> t2s_v(tend - tbase, -1);
  auto t2s_of = [&](int t) { return t >= tbase && t < tend ? t2s_v[t - tbase] : -1; };
  for (int f = N; f <= M; f++) {
    const int bucket = T0 + (f - N);
    for (int t : frames_[f].toks) {
      int s = -1;
      if (f == N && N != 0) {
        auto lit = token2label_.find(t);
        if (lit != token2label_.end()) {
          auto it = label2state.find(lit->second);
          if (it != label2state.end()) s = it->second;
        }
      }
      if (s < 0) s = D.AddState(bucket);
      t2s_v[t - tbase] = s;
    }
  }
  for (int f = N; f <= M; f++) {
    const float off = frames_[f].cost_offset;
    for (int t : frames_[f].toks) {
      const int s = t2s_v[t - tbase];
      ForLinks(t, [&](HLink& l) {
        const int d = t2s_of(l.dst);
        if (d < 0) return;  // emitting links out of the last frame
        const int il = g_->ilabel[l.arc];
        D.links.push_back(DetGraph::Link{s, d, il, g_->olabel[l.arc], l.graph, il != 0 ? l.ac - off : l.ac});
      });
    }
  }
  // the last frame: token labels, final states with the final costs (after
  // FinalizeDecoding) or extra_cost - tot_cost (the pruning's backward costs)
  std::unordered_map<int, int> next_t2l;
  const int fbucket = T0 + (M - N) + 1;
  for (int t : frames_[M].toks) {
    const HTok& tk = toks_[t];
    float fc;
    if (finalized_) {
      if (final_costs_.empty()) {
        fc = 0.0f;
      } else {
        auto it = final_costs_.find(t);
        fc = it != final_costs_.end() ? it->second : kInf;
      }
    } else {
      fc = tk.extra - tk.tot;
    }
    if (!(fc < kInf)) continue;
    const int lab = next_label_++;
    next_t2l[t] = lab;
    const int fs = D.AddState(fbucket);
    D.links.push_back(DetGraph::Link{t2s_v[t - tbase], fs, 0, lab, 0.0f, 0.0f});
    D.fin[fs] = LW{fc, 0.0f};
  }
  if (N == 0) {
    for (int t : frames_[0].toks)
      if (toks_[t].state == g_->start) {
        D.start = t2s_v[t - tbase];
        break;
      }
    if (D.start < 0) {  // no start token: an empty lattice
      token2label_.swap(next_t2l);
      DetInit();
      return;
    }
  }
  token2label_.swap(next_t2l);
  prof.reset();
  AcceptRawLatticeChunk(std::move(D));
}

// ---------------------------------------------------------------------------
// LatticeIncrementalDeterminizer
// ---------------------------------------------------------------------------
void IncrementalLattice::DetInit() {
  carcs_.clear();
  cfin_.clear();
  fwd_.clear();
  arcs_in_.clear();
  final_arcs_.clear();
  redet_.clear();
}

int IncrementalLattice::AddStateToClat() {
  carcs_.emplace_back();
  cfin_.emplace_back();
  fwd_.push_back(kInf);
  arcs_in_.emplace_back();
  return (int)carcs_.size() - 1;
}

void IncrementalLattice::AddArcToClat(int state, const CArc& arc) {
  const float fc = FwdPlus(fwd_[state], arc.w);
  if (fc == kInf) return;
  const int idx = (int)carcs_[state].size();
  carcs_[state].push_back(arc);
  arcs_in_[arc.next].push_back({state, idx});
  if (fc < fwd_[arc.next]) fwd_[arc.next] = fc;
}

bool IncrementalLattice::AcceptRawLatticeChunk(DetGraph&& raw) {
  // GetRawLatticeFinalCosts: the (temporary) final costs of the token-final states
  std::unordered_map<int, float> old_final;
  for (const DetGraph::Link& l : raw.links)
    if (l.lout >= kTokenLabelOffset && l.lout < kMaxTokenLabel) {
      const LW& fw = raw.fin[l.dst];
      if (fw.g == kInf || fw.a != 0.0f) VAMD_ERR("incremental lattice: token label without a final state");
      old_final[l.lout] = fw.g;
    }
  LatticeOptions lo;
  lo.lattice_beam = opt_.lattice_beam;
  lo.det_max_mem = opt_.det_max_mem;
  lo.max_states = opt_.max_states;
  WordLattice chunk;
  std::unique_ptr<IncProf> prof(new IncProf(3));
  const bool det_ok = DeterminizePhonePrunedGraph(std::move(raw), *tid2phone_, *tid_first_, lo, &chunk);  // (raw is not read after)
  prof.reset(new IncProf(4));
  if (!det_ok) {
    failed_ = true;
    DetInit();
    return false;
  }
  chunks_++;
  const int S = chunk.NumStates();
  if (S == 0) {  // (Kaldi warns "Empty lattice"; the lattice stays empty)
    DetInit();
    return false;
  }
  // IdentifyTokenFinalStates
  std::unordered_map<int, int> c2tok;
  for (int s = 0; s < S; s++)
    for (const auto& a : chunk.arcs[s])
      if (a.word >= kTokenLabelOffset && a.word < kMaxTokenLabel) c2tok[a.next] = a.word;
  // ProcessArcsFromChunkStartState
  std::unordered_map<int, int> smap;
  bool first_chunk = false;
  const int nclat = (int)carcs_.size();
  for (const auto& a : chunk.arcs[0]) {
    if (!(a.word >= kStateLabelOffset && a.word - kStateLabelOffset < nclat)) {
      if (!smap.empty()) VAMD_ERR("incremental lattice: mixed start arcs");
      first_chunk = true;
      break;
    }
    const int cs = a.word - kStateLabelOffset;
    const int dest = smap.emplace(a.next, cs).first->second;
    if (!carcs_[cs].empty()) VAMD_ERR("incremental lattice: re-determinized state kept its arcs");
    // arcs entering it get the start arc's weight and string, its forward
    // cost (put on that arc for the pruning) cancelled
    const LW ew = Times(LW{a.graph, a.acoustic}, LW{-fwd_[cs], 0.0f});
    fwd_[cs] = cs == dest ? fwd_[cs] : kInf;
    std::vector<std::pair<int, int>> in;
    in.swap(arcs_in_[cs]);
    for (const auto& p : in) {
      const int src = p.first, pos = p.second;
      if (pos >= (int)carcs_[src].size()) continue;
      CArc& ia = carcs_[src][pos];
      if (ia.next != cs) continue;  // an out-of-date record
      ia.next = dest;
      ia.w = Times(ia.w, ew);
      ia.tids.insert(ia.tids.end(), a.tids.begin(), a.tids.end());
      const float nf = FwdPlus(fwd_[src], ia.w);
      if (nf < fwd_[dest]) fwd_[dest] = nf;
      arcs_in_[dest].push_back(p);
    }
  }
  // states for the rest (token-final states get none)
  for (int s = first_chunk ? 0 : 1; s < S; s++) {
    if (c2tok.count(s)) continue;
    const int ns = (int)carcs_.size();
    if (smap.emplace(s, ns).second) AddStateToClat();
  }
  if (first_chunk) {
    if (smap.at(0) != 0) VAMD_ERR("incremental lattice: start state");
    fwd_[0] = 0.0f;
  }
  final_arcs_.clear();
  // TransferArcsToClat
  for (int s = first_chunk ? 0 : 1; s < S; s++) {
    auto it = smap.find(s);
    if (it == smap.end()) continue;  // token-final
    const int cs = it->second;
    CFin& cf = cfin_[cs];
    cf.is = chunk.final_graph[s] != kInf;
    cf.w = cf.is ? LW{chunk.final_graph[s], chunk.final_acoustic[s]} : LW{};
    cf.tids = cf.is ? chunk.final_tids[s] : std::vector<int>();
    for (const auto& a : chunk.arcs[s]) {
      auto nit = smap.find(a.next);
      if (nit != smap.end()) {
        if (a.word >= kTokenLabelOffset && a.word < kMaxTokenLabel) VAMD_ERR("incremental lattice: token label");
        AddArcToClat(cs, CArc{a.word, nit->second, LW{a.graph, a.acoustic}, a.tids});
        continue;
      }
      auto ot = old_final.find(a.word);
      if (chunk.final_graph[a.next] == kInf || ot == old_final.end() || !c2tok.count(a.next))
        VAMD_ERR("incremental lattice: arc to a token-final state");
      CArc fa{a.word, cs, Times(LW{a.graph, a.acoustic}, LW{chunk.final_graph[a.next], chunk.final_acoustic[a.next]}),
              a.tids};
      const std::vector<int>& ft = chunk.final_tids[a.next];
      fa.tids.insert(fa.tids.end(), ft.begin(), ft.end());
      fa.w = Times(fa.w, LW{-ot->second, 0.0f});
      final_arcs_.push_back(std::move(fa));
    }
  }
  GetNonFinalRedetStates();
  return true;
}

void IncrementalLattice::GetNonFinalRedetStates() {
  redet_.clear();
  std::vector<int> q;
  for (const CArc& fa : final_arcs_)
    if (fwd_[fa.next] != kInf && redet_.insert(fa.next).second) q.push_back(fa.next);
  while (!q.empty()) {
    const int s = q.back();
    q.pop_back();
    for (const CArc& a : carcs_[s])
      if (redet_.insert(a.next).second) q.push_back(a.next);
  }
}

// SetFinalCosts: a state with final arcs becomes final with the best (Plus)
// of its final arcs times the tokens' final costs (all 0 without them)
void IncrementalLattice::SetFinalCosts(const std::unordered_map<int, float>* lfc) {
  std::set<int> prefinal;
  for (const CArc& fa : final_arcs_) prefinal.insert(fa.next);
  for (int s : prefinal) cfin_[s] = CFin{};
  for (const CArc& fa : final_arcs_) {
    float gfc = 0.0f;
    if (lfc) {
      auto it = lfc->find(fa.label);
      if (it == lfc->end()) continue;
      gfc = it->second;
    }
    const LW w = Times(fa.w, LW{gfc, 0.0f});
    CFin& cf = cfin_[fa.next];
    if (!cf.is || CompareCW(cf.w, cf.tids, w, fa.tids) < 0) {
      cf.is = true;
      cf.w = w;
      cf.tids = fa.tids;
    }
  }
}

// clat_ as a WordLattice: states on a path from the start to a final state,
// topologically renumbered (start first; the determinizer's Output order)
void IncrementalLattice::ExportClat(WordLattice* out) const {
  WordLattice& W = *out;
  W = WordLattice();
  const int S = (int)carcs_.size();
  if (S == 0) return;
  std::vector<char> acc(S, 0), coacc(S, 0);
  std::vector<int> st{0};
  acc[0] = 1;
  while (!st.empty()) {
    const int s = st.back();
    st.pop_back();
    for (const CArc& a : carcs_[s])
      if (!acc[a.next]) {
        acc[a.next] = 1;
        st.push_back(a.next);
      }
  }
  std::vector<std::vector<int>> rev(S);
  for (int s = 0; s < S; s++)
    for (const CArc& a : carcs_[s]) rev[a.next].push_back(s);
  for (int s = 0; s < S; s++)
    if (cfin_[s].is) {
      coacc[s] = 1;
      st.push_back(s);
    }
  while (!st.empty()) {
    const int s = st.back();
    st.pop_back();
    for (int p : rev[s])
      if (!coacc[p]) {
        coacc[p] = 1;
        st.push_back(p);
      }
  }
  if (!coacc[0]) return;
  std::vector<int> keep(S, -1), orig;
  for (int s = 0; s < S; s++)
    if (acc[s] && coacc[s]) {
      keep[s] = (int)orig.size();
      orig.push_back(s);
    }
  const int K = (int)orig.size();
  std::vector<int> indeg(K, 0), order;
  for (int k = 0; k < K; k++)
    for (const CArc& a : carcs_[orig[k]])
      if (keep[a.next] >= 0) indeg[keep[a.next]]++;
  st.assign(1, 0);
  while (!st.empty()) {
    const int k = st.back();
    st.pop_back();
    order.push_back(k);
    const auto& arcs = carcs_[orig[k]];
    for (auto it = arcs.rbegin(); it != arcs.rend(); ++it)
      if (keep[it->next] >= 0 && --indeg[keep[it->next]] == 0) st.push_back(keep[it->next]);
  }
  if ((int)order.size() != K) VAMD_ERR("incremental lattice: cycle in the compact lattice");
  std::vector<int> pos(K);
  for (int i = 0; i < K; i++) pos[order[i]] = i;
  W.arcs.resize(K);
  W.final_graph.assign(K, kInf);
  W.final_acoustic.assign(K, 0.0f);
  W.final_tids.resize(K);
  for (int k = 0; k < K; k++) {
    const int s = orig[k], p = pos[k];
    for (const CArc& a : carcs_[s]) {
      if (keep[a.next] < 0) continue;
      if (a.label >= kStateLabelOffset) VAMD_ERR("incremental lattice: a state or token label in the lattice");
      W.arcs[p].push_back(WordLattice::Arc{a.label, pos[keep[a.next]], a.w.g, a.w.a, a.tids});
    }
    if (cfin_[s].is) {
      W.final_graph[p] = cfin_[s].w.g;
      W.final_acoustic[p] = cfin_[s].w.a;
      W.final_tids[p] = cfin_[s].tids;
    }
  }
}

}  // namespace vamd
