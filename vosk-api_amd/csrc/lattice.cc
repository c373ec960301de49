#include "lattice.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <limits>
#include <map>
#include <queue>
#include <unordered_map>

#include "common.h"
#include "model_io.h"

namespace vamd {

namespace {
constexpr float kInf = std::numeric_limits<float>::infinity();

int ArcSource(const Graph& g, int arc) {
  return (int)(std::upper_bound(g.arc_begin.begin(), g.arc_begin.end(), (int64_t)arc) -
               g.arc_begin.begin()) - 1;
}
}  // namespace

void BuildRawLattice(const Graph& g, int start_state, const std::vector<LatFrame>& frames,
                     const std::vector<int4>& arena, const std::vector<int4>& links,
                     bool use_final, RawLattice* out) {
  RawLattice& L = *out;
  L = RawLattice();
  const int F = (int)frames.size() - 1;
  if (F < 0) return;
  L.num_frames = F;
  L.frame_begin.assign(F + 2, 0);
  std::vector<int> arena2tok(arena.size(), -1);
  for (int k = 0; k <= F; k++) {
    const LatFrame& fr = frames[k];
    L.frame_begin[k] = (int)L.tok_state.size();
    for (int a = fr.tok_base; a < fr.tok_base + fr.ntok; a++) {
      if (a < 0 || a >= (int)arena.size()) VAMD_ERR("lattice: arena index out of range");
      const int4 e = arena[a];
      if (e.x == -2) continue;  // dead list entry
      arena2tok[a] = (int)L.tok_state.size();
      L.tok_state.push_back(e.w);
      L.tok_cost.push_back(__builtin_bit_cast(float, e.z));
    }
    L.frame_begin[k + 1] = (int)L.tok_state.size();
  }
  (void)start_state;
  auto tok = [&](int a) {
    if (a < 0 || a >= (int)arena.size() || arena2tok[a] < 0) VAMD_ERR("lattice: link to a missing token");
    return arena2tok[a];
  };
  for (int k = 0; k <= F; k++) {
    const LatFrame& fr = frames[k];
    const long long lb = std::max<long long>(0, fr.link_begin),
                    le = std::min<long long>((long long)links.size(), fr.link_end);
    if (fr.link_end > (long long)links.size()) L.overflow = true;
    std::vector<RawLattice::Link> fl;
    fl.reserve(le > lb ? le - lb : 0);
    for (long long i = lb; i < le; i++) {
      const int4 r = links[i];
      const int arc = r.z;
      const bool eps = g.ilabel[arc] == 0;
      const float ac = eps ? 0.0f : __builtin_bit_cast(float, r.w) - fr.cost_offset;
      fl.push_back(RawLattice::Link{tok(r.x), tok(r.y), arc, g.weight[arc], ac});
    }
    std::sort(fl.begin(), fl.end(), [](const RawLattice::Link& a, const RawLattice::Link& b) {
      return a.src != b.src ? a.src < b.src : a.arc < b.arc;
    });
    L.links.insert(L.links.end(), fl.begin(), fl.end());
  }
  if (use_final) {
    std::vector<float> fc;
    bool any = false;
    for (int t = L.frame_begin[F]; t < L.frame_begin[F + 1]; t++) {
      const float c = g.final_cost[L.tok_state[t]];
      fc.push_back(c);
      any |= c != kInf;
    }
    if (any) L.final_cost = fc;
  }
}

}  // namespace vamd

// ===========================================================================
// word level
// ===========================================================================
namespace vamd {

namespace {

// Kaldi LatticeWeight order: smaller total cost is better; ties by graph cost
// (LW: lattice.h)
inline int CompareLW(const LW& x, const LW& y) {  // 1: x better, -1: y better
  const float fx = x.g + x.a, fy = y.g + y.a;
  if (fx < fy) return 1;
  if (fx > fy) return -1;
  if (x.g < y.g) return 1;
  if (x.g > y.g) return -1;
  if (x.a < y.a) return 1;
  if (x.a > y.a) return -1;
  return 0;
}
inline LW Times(const LW& x, const LW& y) { return LW{x.g + y.g, x.a + y.a}; }
inline LW Divide(const LW& x, const LW& y) { return LW{x.g - y.g, x.a - y.a}; }

// Transition-id strings of the determinizer as nodes of one trie (Kaldi's
// LatticeDeterminizer keeps a StringRepository for the same reason): a string
// is a node (the path from the root), appending a label is one hash lookup.
// The elements of a subset share a base node (the prefixes already moved to
// arcs); an element's residual string is the path base -> node, compared by
// length and a polynomial hash mod 2^61 - 1, so removing a common prefix is
// a change of base (a lowest common ancestor by jump pointers), not a copy.
struct StrRepo {
  static constexpr uint64_t kMod = (1ull << 61) - 1, kBase = 1000003ull;
  // jump[]: skew-binary jump pointers (one per node, O(log depth) ancestor
  // and common-prefix queries)
  std::vector<int> parent{-1}, label{0}, len{0}, jump{0};
  std::vector<uint64_t> hash{0}, pw{1};
  // each node's first successor (label, node; label -1: none yet) beside it:
  // most nodes get one (a transition-id string mostly extends one way), and
  // the table below then holds only the later ones
  struct Child {
    int lab, val;
  };
  std::vector<Child> first{Child{-1, -1}};
  // (node, label) -> successor node beyond the first: open addressing,
  // linear probing (key and value side by side: one cache line per probe)
  struct Slot {
    uint64_t key;
    int val;
  };
  std::vector<Slot> slot = std::vector<Slot>(1024, Slot{~0ull, -1});
  size_t sused = 0;
  static size_t Mix(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    return (size_t)k;
  }
  void Grow() {
    std::vector<Slot> old(slot.size() * 2, Slot{~0ull, -1});
    old.swap(slot);
    const size_t m = slot.size() - 1;
    for (const Slot& o : old)
      if (o.key != ~0ull) {
        size_t h = Mix(o.key) & m;
        while (slot[h].key != ~0ull) h = (h + 1) & m;
        slot[h] = o;
      }
  }
  static uint64_t MulMod(uint64_t x, uint64_t y) {
    const unsigned __int128 p = (unsigned __int128)x * y;
    uint64_t r = (uint64_t)(p & kMod) + (uint64_t)(p >> 61);
    return r >= kMod ? r - kMod : r;
  }
  int Succ(int id, int lab) {
    Child& fc = first[id];
    if (fc.lab == lab) return fc.val;
    const int n = (int)parent.size();
    if (fc.lab < 0) {
      fc = Child{lab, n};
    } else {
      const uint64_t k = ((uint64_t)(uint32_t)id << 32) | (uint32_t)lab;
      size_t m = slot.size() - 1, q = Mix(k) & m;
      while (slot[q].key != ~0ull) {
        if (slot[q].key == k) return slot[q].val;
        q = (q + 1) & m;
      }
      slot[q] = Slot{k, n};
      if (2 * ++sused > slot.size()) Grow();
    }
    first.push_back(Child{-1, -1});
    parent.push_back(id);
    label.push_back(lab);
    len.push_back(len[id] + 1);
    uint64_t h = MulMod(hash[id], kBase) + (uint64_t)(uint32_t)lab + 1;
    hash.push_back(h >= kMod ? h - kMod : h);
    if ((int)pw.size() <= len[n]) pw.push_back(MulMod(pw.back(), kBase));
    const int j1 = jump[id], j2 = jump[j1];
    jump.push_back(id != 0 && len[id] - len[j1] == len[j1] - len[j2] ? j2 : id);
    return n;
  }
  int Ancestor(int id, int depth) const {  // the prefix of id with `depth` labels
    while (len[id] > depth) id = len[jump[id]] >= depth ? jump[id] : parent[id];
    return id;
  }
  int Lca(int a, int b) const {  // longest common prefix of two strings
    if (len[a] > len[b]) a = Ancestor(a, len[b]);
    else if (len[b] > len[a]) b = Ancestor(b, len[a]);
    while (a != b) {  // equal depths: the jump structure is the same on both sides
      if (jump[a] != jump[b]) {
        a = jump[a];
        b = jump[b];
      } else {
        a = parent[a];
        b = parent[b];
      }
    }
    return a;
  }
  // residual string base -> id (base a prefix of id): length and hash
  int ResLen(int id, int base) const { return len[id] - len[base]; }
  uint64_t ResHash(int id, int base) const {
    const uint64_t sub = MulMod(hash[base], pw[len[id] - len[base]]);
    return hash[id] >= sub ? hash[id] - sub : hash[id] + kMod - sub;
  }
  // residuals (ba -> a) and (bb -> b) of equal length: equal strings?
  bool ResEqual(int a, int ba, int b, int bb) const {
    int n = len[a] - len[ba];
    if (n != len[b] - len[bb]) return false;
    for (; n > 0 && a != b; n--, a = parent[a], b = parent[b])
      if (label[a] != label[b]) return false;
    return true;
  }
  void Get(int id, int base, std::vector<int>* out) const {
    out->resize(len[id] - len[base]);
    for (int i = (int)out->size() - 1; i >= 0; i--, id = parent[id]) (*out)[i] = label[id];
  }
  bool Less(int a, int b, int base) const {  // residuals: shorter first, then lexicographic
    if (len[a] != len[b]) return len[a] < len[b];
    if (a == b) return false;
    std::vector<int> x, y;
    Get(a, base, &x);
    Get(b, base, &y);
    return x < y;
  }
};

struct Elem {
  int tok;
  LW w;
  int str;  // StrRepo node; the residual string is base -> str
};
// (weight, string) order of Kaldi's determinizer when one state is reached twice
inline bool ElemBetter(const StrRepo& R, int base, const Elem& x, const Elem& y) {
  const int c = CompareLW(x.w, y.w);
  if (c != 0) return c > 0;
  return R.Less(x.str, y.str, base);
}

}  // namespace

void PruneRawLattice(RawLattice* lat, float beam) {
  RawLattice& L = *lat;
  const int N = (int)L.tok_state.size(), F = L.num_frames;
  if (N == 0) return;
  std::vector<int> frame(N);
  for (int k = 0; k <= F; k++)
    for (int t = L.frame_begin[k]; t < L.frame_begin[k + 1]; t++) frame[t] = k;
  // links grouped by destination frame (BuildRawLattice order)
  std::vector<int> lb(F + 2, 0);
  for (auto& l : L.links) lb[frame[l.dst] + 1]++;
  for (int k = 0; k <= F; k++) lb[k + 1] += lb[k];
  auto cost = [](const RawLattice::Link& l) { return l.graph_cost + l.acoustic_cost; };
  std::vector<double> alpha(N, INFINITY), beta(N, INFINITY);
  for (int t = L.frame_begin[0]; t < L.frame_begin[1]; t++)
    if (L.tok_cost[t] == 0.0f && L.tok_state[t] >= 0) { alpha[t] = 0.0; break; }
  for (int k = 0; k <= F; k++) {
    // emitting links (from frame k-1) first, then epsilon links to a fixpoint
    for (int i = lb[k]; i < lb[k + 1]; i++) {
      const auto& l = L.links[i];
      if (frame[l.src] != k) alpha[l.dst] = std::min(alpha[l.dst], alpha[l.src] + cost(l));
    }
    for (bool ch = true; ch;) {
      ch = false;
      for (int i = lb[k]; i < lb[k + 1]; i++) {
        const auto& l = L.links[i];
        if (frame[l.src] == k && alpha[l.src] + cost(l) < alpha[l.dst]) {
          alpha[l.dst] = alpha[l.src] + cost(l);
          ch = true;
        }
      }
    }
  }
  double best = INFINITY;
  for (int t = L.frame_begin[F]; t < L.frame_begin[F + 1]; t++) {
    const double fc = L.final_cost.empty() ? 0.0 : (double)L.final_cost[t - L.frame_begin[F]];
    beta[t] = fc;
    best = std::min(best, alpha[t] + fc);
  }
  for (int k = F; k >= 0; k--) {
    for (bool ch = true; ch;) {
      ch = false;
      for (int i = lb[k]; i < lb[k + 1]; i++) {
        const auto& l = L.links[i];
        if (frame[l.src] == k && cost(l) + beta[l.dst] < beta[l.src]) {
          beta[l.src] = cost(l) + beta[l.dst];
          ch = true;
        }
      }
    }
    for (int i = lb[k]; i < lb[k + 1]; i++) {
      const auto& l = L.links[i];
      if (frame[l.src] != k) beta[l.src] = std::min(beta[l.src], cost(l) + beta[l.dst]);
    }
  }
  // keep what lies on a path within the beam of the best one
  std::vector<int> remap(N, -1);
  RawLattice out;
  out.num_frames = F;
  out.frame_begin.assign(F + 2, 0);
  out.overflow = L.overflow;
  for (int k = 0; k <= F; k++) {
    out.frame_begin[k] = (int)out.tok_state.size();
    for (int t = L.frame_begin[k]; t < L.frame_begin[k + 1]; t++) {
      if (!(alpha[t] + beta[t] - best <= beam)) continue;
      remap[t] = (int)out.tok_state.size();
      out.tok_state.push_back(L.tok_state[t]);
      out.tok_cost.push_back(L.tok_cost[t]);
    }
    out.frame_begin[k + 1] = (int)out.tok_state.size();
  }
  for (auto& l : L.links) {
    if (remap[l.src] < 0 || remap[l.dst] < 0) continue;
    if (!(alpha[l.src] + cost(l) + beta[l.dst] - best <= beam)) continue;
    RawLattice::Link m = l;
    m.src = remap[l.src];
    m.dst = remap[l.dst];
    out.links.push_back(m);
  }
  if (!L.final_cost.empty())
    for (int t = L.frame_begin[F]; t < L.frame_begin[F + 1]; t++)
      if (remap[t] >= 0) out.final_cost.push_back(L.final_cost[t - L.frame_begin[F]]);
  L = std::move(out);
}

namespace {

DetGraph FromRaw(const RawLattice& L, const Graph& g) {
  DetGraph D;
  const int N = (int)L.tok_state.size(), F = L.num_frames;
  D.n = N;
  D.frame.resize(N);
  for (int k = 0; k <= F; k++)
    for (int t = L.frame_begin[k]; t < L.frame_begin[k + 1]; t++) D.frame[t] = k;
  D.fin.assign(N, LW{kInf, 0.0f});
  for (int t = L.frame_begin[F]; t < L.frame_begin[F + 1]; t++)
    D.fin[t].g = L.final_cost.empty() ? 0.0f : L.final_cost[t - L.frame_begin[F]];
  for (int t = L.frame_begin[0]; t < L.frame_begin[1]; t++)
    if (L.tok_cost[t] == 0.0f) { D.start = t; break; }
  // the labels of every link, gathered once (the graph's label arrays are
  // large: random reads of them in every closure miss the caches)
  D.links.resize(L.links.size());
  for (size_t i = 0; i < L.links.size(); i++) {
    const auto& l = L.links[i];
    D.links[i] = DetGraph::Link{l.src, l.dst, g.ilabel[l.arc], g.olabel[l.arc], l.graph_cost, l.acoustic_cost};
  }
  return D;
}

bool Determinize(const DetGraph& D, const LatticeOptions& opt, WordLattice* out) {
  WordLattice& W = *out;
  W = WordLattice();
  const int N = D.n;
  if (N == 0 || D.start < 0) return true;
  int F = 0;
  for (int f : D.frame) F = f > F ? f : F;
  const std::vector<DetGraph::Link>& links = D.links;
  // out-links per token (CSR): the word-epsilon ones (closures) first, then
  // the word links (transitions)
  const int NL = (int)links.size();
  std::vector<int> ob(N + 1, 0), oe(N, 0), ol(NL);
  for (int i = 0; i < NL; i++) ob[links[i].src + 1]++;
  for (int t = 0; t < N; t++) ob[t + 1] += ob[t];
  {
    std::vector<int> fill(ob.begin(), ob.end() - 1);
    for (int i = 0; i < NL; i++)
      if (links[i].lout == 0) ol[fill[links[i].src]++] = i;
    for (int t = 0; t < N; t++) oe[t] = fill[t];
    for (int i = 0; i < NL; i++)
      if (links[i].lout != 0) ol[fill[links[i].src]++] = i;
  }
  // the links in that order, packed (the closures walk them sequentially)
  std::vector<DetGraph::Link> cl(NL);
  for (int k = 0; k < NL; k++) cl[k] = links[ol[k]];
  const std::vector<LW>& fin = D.fin;
  const int start = D.start;
  const bool dbg = getenv("VOSK_AMD_DET_DEBUG") != nullptr;
  StrRepo R;
  long long dbg_ext = 0;
  double dt_clo = 0, dt_norm = 0, dt_bw = 0, dt_find = 0;
  using dclk = std::chrono::steady_clock;
  auto dms = [](dclk::time_point a) { return std::chrono::duration<double, std::milli>(dclk::now() - a).count(); };
  // closure over word-epsilon links (emitting arcs without a word label too):
  // for each token the best (weight, string) reaching it
  // frame of every token: the closure visits tokens frame by frame (links go
  // from frame k to k + 1, or within frame k), so a token is expanded once its
  // frame's predecessors are final -- not once per improvement along every
  // path (the same fixpoint: the best (weight, string) per token)
  const std::vector<int>& tframe = D.frame;
  std::vector<int> at_pos(N, -1);  // closure scratch: token -> element (reset after each closure)
  std::vector<char> pending;      // closure scratch: element queued
  // per link: the last (string, extended string) of R.Succ through it -- a
  // token reached by the same path from any subset has the same trie node,
  // so most extensions repeat (the trie's hash table is large and cold)
  // (indexed by packed link position)
  std::vector<int> memo_in(NL, -1), memo_out(NL, -1);
  auto extend = [&](int str, int k) {
    if (cl[k].lin == 0) return str;
    if (memo_in[k] == str) return memo_out[k];
    const int n = R.Succ(str, cl[k].lin);
    memo_in[k] = str;
    memo_out[k] = n;
    return n;
  };
  // closure work queue: elements bucketed by token frame (links go forward
  // in time or stay in the frame), earliest frame first, FIFO within a frame
  std::vector<std::vector<int>> fbucket(F + 1);
  auto closure = [&](std::vector<Elem>* sub, int base) {
    struct AtMap {
      std::vector<int>& pos;
      std::vector<int> touched;
      struct It {
        int second;
      };
      int find_idx(int t) const { return pos[t]; }
      void set(int t, int i) {
        if (pos[t] < 0) touched.push_back(t);
        pos[t] = i;
      }
      ~AtMap() {
        for (int t : touched) pos[t] = -1;
      }
    } at{at_pos, {}};
    pending.assign(sub->size(), 1);
    int fmin = F + 1, fmax = -1;
    auto push = [&](int i) {
      const int f = tframe[(*sub)[i].tok];
      fbucket[f].push_back(i);
      fmin = f < fmin ? f : fmin;
      fmax = f > fmax ? f : fmax;
    };
    for (int i = 0; i < (int)sub->size(); i++) {
      at.set((*sub)[i].tok, i);
      push(i);
    }
    for (int f = fmin; f <= fmax; f++) {
      std::vector<int>& bq = fbucket[f];
      for (size_t qi = 0; qi < bq.size(); qi++) {  // (grows while walked: same-frame links)
        const int i = bq[qi];
        pending[i] = 0;  // an element improved while queued is expanded once, at its best
        const Elem e = (*sub)[i];
        dbg_ext++;
        for (int k = ob[e.tok]; k < oe[e.tok]; k++) {
          const auto& l = cl[k];
          const LW w = Times(e.w, LW{l.g, l.a});
          const int ei = at.find_idx(l.dst);
          if (ei < 0) {
            at.set(l.dst, (int)sub->size());
            sub->push_back(Elem{l.dst, w, extend(e.str, k)});
            pending.push_back(1);
            push((int)sub->size() - 1);
            continue;
          }
          // the string only when the weight does not decide (ElemBetter's
          // order): a losing candidate adds no trie node
          const int c = CompareLW(w, (*sub)[ei].w);
          if (c < 0) continue;
          const Elem n{l.dst, w, extend(e.str, k)};
          if (c > 0 || R.Less(n.str, (*sub)[ei].str, base)) {
            (*sub)[ei] = n;
            if (!pending[ei]) {
              pending[ei] = 1;
              push(ei);
            }
          }
        }
      }
      bq.clear();
    }
    // Kaldi's ConvertToMinimal: only tokens with word links or a final cost
    // matter past the closure (transitions and finals); the subset's weight,
    // common prefix and identity are those of the rest
    size_t m = 0;
    for (size_t i = 0; i < sub->size(); i++) {
      const int t = (*sub)[i].tok;
      if (oe[t] < ob[t + 1] || fin[t].g != kInf) (*sub)[m++] = (*sub)[i];
    }
    sub->resize(m);
    std::sort(sub->begin(), sub->end(), [](const Elem& x, const Elem& y) { return x.tok < y.tok; });
  };
  // normalization: the best weight and the common string prefix move to the
  // arc (the prefix = base -> lowest common ancestor, the subset's new base)
  auto normalize = [&](std::vector<Elem>* sub, int base, LW* tot, std::vector<int>* prefix) {
    *tot = (*sub)[0].w;
    int common = (*sub)[0].str;
    for (auto& e : *sub) {
      if (CompareLW(e.w, *tot) > 0) *tot = e.w;
      common = R.Lca(common, e.str);
    }
    R.Get(common, base, prefix);
    for (auto& e : *sub) e.w = Divide(e.w, *tot);
    return common;
  };
  // subsets are equal with the same tokens and strings and weights within
  // delta (Kaldi's determinizer, delta = kDelta = 1/1024)
  const float delta = 1.0f / 1024.0f;
  std::unordered_map<uint64_t, std::vector<int>> index;
  std::vector<std::vector<Elem>> subsets;
  std::vector<int> bases;  // per subset: the base node of its residual strings
  // key: a hash of the (token, residual length, residual hash) sequence; a
  // hit is confirmed element by element (tokens, weights within delta,
  // residual strings exactly)
  auto key_of = [&](const std::vector<Elem>& sub, int base) {
    uint64_t k = 0x9e3779b97f4a7c15ull ^ sub.size();
    for (auto& e : sub) {
      const uint64_t h = R.ResHash(e.str, base);
      k = (k ^ (uint64_t)(uint32_t)e.tok) * 0xff51afd7ed558ccdull;
      k = (k ^ (uint64_t)(uint32_t)R.ResLen(e.str, base)) * 0xc4ceb9fe1a85ec53ull;
      k = (k ^ h) * 0xff51afd7ed558ccdull;
      k ^= k >> 29;
    }
    return k;
  };
  auto find_or_add = [&](std::vector<Elem>&& sub, int base, bool* added) {
    const uint64_t k = key_of(sub, base);
    auto& cand = index[k];
    for (int id : cand) {
      const auto& o = subsets[id];
      bool eq = o.size() == sub.size();
      for (size_t i = 0; i < o.size() && eq; i++) eq = o[i].tok == sub[i].tok;
      for (size_t i = 0; i < o.size() && eq; i++)
        eq = std::fabs(o[i].w.g - sub[i].w.g) <= delta && std::fabs(o[i].w.a - sub[i].w.a) <= delta;
      // the key holds residual lengths and hashes: the strings themselves
      // are compared too (Kaldi compares them exactly), walking both up the
      // trie together until they meet (equal-length residuals ending in the
      // same node are equal)
      for (size_t i = 0; i < o.size() && eq; i++) eq = R.ResEqual(o[i].str, bases[id], sub[i].str, base);
      if (eq) {
        *added = false;
        return id;
      }
    }
    const int id = (int)subsets.size();
    subsets.push_back(std::move(sub));
    bases.push_back(base);
    cand.push_back(id);
    *added = true;
    return id;
  };
  // start state: the closure of the start token, not normalized (its weight
  // and string stay on the first arcs / final weight)
  std::vector<Elem> s0{Elem{start, LW{}, 0}};
  closure(&s0, 0);
  bool added;
  find_or_add(std::move(s0), 0, &added);
  std::vector<std::vector<WordLattice::Arc>> arcs(1);
  std::vector<int> queue{0};
  std::vector<std::pair<int, Elem>> tr_scratch;
  for (size_t qi = 0; qi < queue.size(); qi++) {
    const int sid = queue[qi];
    const int sbase = bases[sid];
    // transitions per word label, in label order: (word, element) pairs,
    // sorted by (word, token), one element per (word, token) -- the better
    std::vector<std::pair<int, Elem>>& tr = tr_scratch;
    tr.clear();
    for (const Elem& e : subsets[sid])
      for (int k = oe[e.tok]; k < ob[e.tok + 1]; k++) {
        const auto& l = cl[k];
        tr.push_back({l.lout, Elem{l.dst, Times(e.w, LW{l.g, l.a}), extend(e.str, k)}});
      }
    std::sort(tr.begin(), tr.end(), [&](const std::pair<int, Elem>& x, const std::pair<int, Elem>& y) {
      if (x.first != y.first) return x.first < y.first;
      if (x.second.tok != y.second.tok) return x.second.tok < y.second.tok;
      return ElemBetter(R, sbase, x.second, y.second);
    });
    for (size_t g0 = 0; g0 < tr.size();) {
      const int word = tr[g0].first;
      size_t g1 = g0;
      std::vector<Elem> sub;
      for (; g1 < tr.size() && tr[g1].first == word; g1++)
        if (sub.empty() || sub.back().tok != tr[g1].second.tok) sub.push_back(tr[g1].second);
      g0 = g1;
      dclk::time_point t0;
      if (dbg) t0 = dclk::now();
      closure(&sub, sbase);
      if (dbg) dt_clo += dms(t0);
      if (sub.empty()) continue;  // a dead end (cannot occur on a pruned lattice)
      LW tot;
      std::vector<int> prefix;
      if (dbg) t0 = dclk::now();
      const int nbase = normalize(&sub, sbase, &tot, &prefix);
      if (dbg) dt_norm += dms(t0);
      if (dbg) t0 = dclk::now();
      const int dst = find_or_add(std::move(sub), nbase, &added);
      if (dbg) dt_find += dms(t0);
      if (added) {
        if ((int)subsets.size() > opt.max_states) return false;
        queue.push_back(dst);
        arcs.emplace_back();
      }
      arcs[sid].push_back(WordLattice::Arc{word, dst, tot.g, tot.a, std::move(prefix)});
    }
  }
  const int S = (int)subsets.size();
  if (dbg) {
    long long el = 0;
    for (auto& x : subsets) el += (long long)x.size();
    fprintf(stderr, "det: tokens %d links %zu subsets %d elems %lld expansions %lld strings %zu clo %.2f norm %.2f find %.2f\n",
            N, links.size(), S, el, dbg_ext, R.parent.size(), dt_clo, dt_norm, dt_find);
  }
  std::vector<LW> fw(S);
  std::vector<std::vector<int>> fs(S);
  std::vector<char> isf(S, 0);
  for (int s = 0; s < S; s++) {
    bool have = false;
    Elem best{0, LW{}, 0};
    for (const Elem& e : subsets[s]) {
      if (fin[e.tok].g == kInf) continue;
      Elem c{e.tok, Times(e.w, fin[e.tok]), e.str};
      if (!have || ElemBetter(R, bases[s], c, best)) {
        best = c;
        have = true;
      }
    }
    if (have) {
      isf[s] = 1;
      fw[s] = best.w;
      R.Get(best.str, bases[s], &fs[s]);
    }
  }
  // topological order (the lattice is acyclic), start state first
  std::vector<int> indeg(S, 0), order;
  for (int s = 0; s < S; s++)
    for (auto& a : arcs[s]) indeg[a.next]++;
  std::vector<int> st{0};
  while (!st.empty()) {
    const int s = st.back();
    st.pop_back();
    order.push_back(s);
    for (auto it = arcs[s].rbegin(); it != arcs[s].rend(); ++it)
      if (--indeg[it->next] == 0) st.push_back(it->next);
  }
  if ((int)order.size() != S) VAMD_ERR("lattice determinization produced a cycle");
  std::vector<int> pos(S);
  for (int i = 0; i < S; i++) pos[order[i]] = i;
  W.arcs.resize(S);
  W.final_graph.assign(S, INFINITY);
  W.final_acoustic.assign(S, 0.0f);
  W.final_tids.resize(S);
  for (int s = 0; s < S; s++) {
    const int p = pos[s];
    for (auto& a : arcs[s]) {
      WordLattice::Arc b = a;
      b.next = pos[a.next];
      W.arcs[p].push_back(std::move(b));
    }
    if (isf[s]) {
      W.final_graph[p] = fw[s].g;
      W.final_acoustic[p] = fw[s].a;
      W.final_tids[p] = fs[s];
    }
  }
  return true;
}


// ---------------------------------------------------------------------------
// Kaldi's pruned lattice determinization (lat/determinize-lattice-pruned.{h,cc}
// [K]: LatticeDeterminizerPruned + DeterminizeLatticePruned), the
// determinization of the reference's GetLattice (src/recognizer.cc:678) and
// of its batch lattice callback (src/batch_recognizer.cc:138-149 ->
// DeterminizeLatticePhonePrunedWrapper).  Unlike the exact subset
// construction above it
//  - keeps each input state's backward cost (best cost to a final state) and
//    each output state's forward cost (set when the state is created);
//  - turns every (output state, label) transition into a task whose
//    priority is forward cost + min over the elements of (weight + backward
//    cost), drops tasks beyond cutoff = best path cost + beam, and runs the
//    rest best first (priority queue; equal priorities in push order);
//  - normalizes a transition's subset before its closure (weight and common
//    prefix onto the arc), again after it, and caches the closure of each
//    normalized initial subset (Kaldi's initial_hash_);
//  - stores a final weight only when it is within the cutoff;
//  - stops when its memory estimate passes max_mem (checked every tenth
//    state, after a repository rebuild), reporting the effective beam; the
//    caller then prunes the input at a narrower beam and retries
//    (DeterminizeLatticePruned, retry_cutoff 0.7, at most 10 tries);
//  - writes states in creation order and trims what is not on a path from
//    the start to a final state (fst::Connect in the wrapper).
// Element order ties: (weight, string) with Kaldi's Compare -- lower total
// cost, then lower graph cost, then the shorter string, then the
// lexicographically larger one.
// ---------------------------------------------------------------------------
struct PrunedDetOptions {
  double beam = 6.0;
  float delta = 1.0f / 1024.0f;   // kDelta
  long long max_mem = 50000000;   // DeterminizeLatticePhonePrunedOptions default
  int max_states = 100000;        // this build's guard (Kaldi: -1)
};

// LatticeWeight ApproxEqual: identical, or total costs within delta
inline bool ApproxEqualLW(const LW& x, const LW& y, float delta) {
  if (x.g == y.g && x.a == y.a) return true;
  return std::fabs((x.g + x.a) - (y.g + y.a)) <= delta;
}
// fst::Compare(LatticeWeight): total cost, then graph cost (no third key)
inline int CompareLWK(const LW& x, const LW& y) {
  const float fx = x.g + x.a, fy = y.g + y.a;
  if (fx < fy) return 1;
  if (fx > fy) return -1;
  if (x.g < y.g) return 1;
  if (x.g > y.g) return -1;
  return 0;
}
inline double CostOf(const LW& w) { return (double)w.g + (double)w.a; }

class PrunedDeterminizer {
 public:
  PrunedDeterminizer(const DetGraph& D, const std::vector<int>& topo, const PrunedDetOptions& o)
      : D_(D), topo_(topo), opt_(o) {}

  // Determinize(): false when it stopped early (memory / state guard)
  bool Run(double* effective_beam);
  void Output(WordLattice* out);  // creation order, Connect-trimmed, then topologically renumbered
  bool guard_tripped() const { return guard_; }

 private:
  struct OArc {
    int label, next;  // next -1: the final weight
    LW w;
    int str, base;    // arc string = residual base -> str
  };
  struct OState {
    std::vector<Elem> sub;  // minimal normalized subset, sorted by token
    int base;               // residuals relative to this node
    double fwd;             // forward cost at creation
    std::vector<OArc> arcs;
  };
  struct Task {
    double prio;
    long long seq;
    int state, label;
    std::vector<Elem> sub;  // unnormalized, unique per token, sorted; strings relative to the state's base
  };
  // Kaldi's TaskCompare orders by priority_cost only and std::priority_queue
  // leaves ties unordered; ties here go in push order (deterministic).  Which
  // tasks run before a max_mem / max_states stop can therefore differ from
  // Kaldi on exactly tied priorities (parity with LatticeDeterminizerPruned is
  // unpinned: no Kaldi build or fixture here).
  struct TaskLess {
    bool operator()(const Task* a, const Task* b) const {
      if (a->prio != b->prio) return a->prio > b->prio;
      return a->seq > b->seq;
    }
  };
  struct Cached {  // initial_hash_ entry: the normalized initial subset -> state, remaining weight and string
    std::vector<Elem> sub;
    int base;
    int state;
    LW rem;
    int rem_str, rem_base;
  };

  int Compare(const Elem& x, int bx, const Elem& y, int by) const;  // 1: x better (Kaldi Compare)
  void Closure(std::vector<Elem>* sub, int base);
  void ConvertToMinimal(std::vector<Elem>* sub) const;
  LW Normalize(std::vector<Elem>* sub, int* base);  // returns the total weight; *base -> the new base
  int MinimalToState(std::vector<Elem>&& sub, int base, double fwd);
  int InitialToState(const std::vector<Elem>& sub, int base, double fwd, LW* rem, int* rem_str, int* rem_base);
  void ProcessFinal(int s);
  void ProcessTransitions(int s);
  void ProcessTransition(Task* t);
  bool CheckMemory(double* eff);
  uint64_t SubKey(const std::vector<Elem>& sub, int base) const;
  bool SubEqual(const std::vector<Elem>& x, int bx, const std::vector<Elem>& y, int by) const;
  int AppendString(int node, int from_base, int to_node) ;  // node ++ (from_base -> to_node)

  const DetGraph& D_;
  const std::vector<int>& topo_;
  PrunedDetOptions opt_;
  StrRepo R_;
  std::vector<int> ob_, oe_;
  std::vector<DetGraph::Link> cl_;
  std::vector<double> bwd_;
  double cutoff_ = 0;
  std::vector<OState> states_;
  std::unordered_map<uint64_t, std::vector<int>> minimal_;
  std::unordered_map<uint64_t, std::vector<int>> initial_;
  std::vector<Cached> cached_;
  std::priority_queue<Task*, std::vector<Task*>, TaskLess> queue_;
  long long seq_ = 0, num_elems_ = 0, num_arcs_ = 0;
  double eff_beam_ = 0;
  bool guard_ = false;
  // the repository as Kaldi's RebuildRepository leaves it: the strings live
  // at the last rebuild, plus every string added since -- new nodes, and
  // nodes the rebuild would have deleted that are referenced again (Kaldi
  // re-adds those; here they still exist: Revive counts them) (-1: never
  // rebuilt)
  long long rebuilt_live_ = -1, revived_ = 0;
  size_t rebuilt_at_ = 0;
  std::vector<char> rebuilt_mark_;  // nodes below rebuilt_at_ live at the rebuild (or revived)
  int Revive(int n) {
    if (rebuilt_live_ >= 0 && n > 0 && (size_t)n < rebuilt_at_ && !rebuilt_mark_[n]) {
      rebuilt_mark_[n] = 1;
      revived_++;
    }
    return n;
  }
  std::vector<int> at_pos_;
  std::vector<char> pending_;
  std::vector<std::vector<int>> fbucket_;
  std::vector<int> memo_in_, memo_out_;
};

int PrunedDeterminizer::Compare(const Elem& x, int bx, const Elem& y, int by) const {
  const int c = CompareLWK(x.w, y.w);
  if (c != 0) return c;
  const int lx = R_.ResLen(x.str, bx), ly = R_.ResLen(y.str, by);
  if (lx > ly) return -1;  // the shorter string wins
  if (lx < ly) return 1;
  if (lx == 0) return 0;
  std::vector<int> a, b;
  R_.Get(x.str, bx, &a);
  R_.Get(y.str, by, &b);
  for (int i = 0; i < lx; i++) {
    if (a[i] < b[i]) return -1;  // then the lexicographically larger one
    if (a[i] > b[i]) return 1;
  }
  return 0;
}

// EpsilonClosure: the best (weight, string) per input state reachable through
// label-epsilon links (the fixpoint; states visited in topological buckets)
void PrunedDeterminizer::Closure(std::vector<Elem>* sub, int base) {
  const std::vector<int>& tframe = D_.frame;
  std::vector<int> touched;
  pending_.assign(sub->size(), 1);
  int fmin = (int)fbucket_.size(), fmax = -1;
  auto push = [&](int i) {
    const int f = tframe[(*sub)[i].tok];
    fbucket_[f].push_back(i);
    fmin = f < fmin ? f : fmin;
    fmax = f > fmax ? f : fmax;
  };
  for (int i = 0; i < (int)sub->size(); i++) {
    at_pos_[(*sub)[i].tok] = i;
    touched.push_back((*sub)[i].tok);
    push(i);
  }
  auto extend = [&](int str, int k) {
    if (cl_[k].lin == 0) return str;
    if (memo_in_[k] == str) return Revive(memo_out_[k]);
    const int n = Revive(R_.Succ(str, cl_[k].lin));
    memo_in_[k] = str;
    memo_out_[k] = n;
    return n;
  };
  for (int f = fmin; f <= fmax; f++) {
    std::vector<int>& bq = fbucket_[f];
    for (size_t qi = 0; qi < bq.size(); qi++) {
      const int i = bq[qi];
      pending_[i] = 0;
      const Elem e = (*sub)[i];
      for (int k = ob_[e.tok]; k < oe_[e.tok]; k++) {
        const auto& l = cl_[k];
        const LW w = Times(e.w, LW{l.g, l.a});
        const int ei = at_pos_[l.dst];
        if (ei < 0) {
          at_pos_[l.dst] = (int)sub->size();
          touched.push_back(l.dst);
          sub->push_back(Elem{l.dst, w, extend(e.str, k)});
          pending_.push_back(1);
          push((int)sub->size() - 1);
          continue;
        }
        const int c = CompareLWK(w, (*sub)[ei].w);
        if (c < 0) continue;
        const Elem n{l.dst, w, extend(e.str, k)};
        if (c > 0 || Compare(n, base, (*sub)[ei], base) > 0) {
          (*sub)[ei] = n;
          if (!pending_[ei]) {
            pending_[ei] = 1;
            push(ei);
          }
        }
      }
    }
    bq.clear();
  }
  for (int t : touched) at_pos_[t] = -1;
}

// ConvertToMinimal: only states with label links or a final weight remain
void PrunedDeterminizer::ConvertToMinimal(std::vector<Elem>* sub) const {
  size_t m = 0;
  for (size_t i = 0; i < sub->size(); i++) {
    const int t = (*sub)[i].tok;
    if (oe_[t] < ob_[t + 1] || D_.fin[t].g != kInf) (*sub)[m++] = (*sub)[i];
  }
  sub->resize(m);
  std::sort(sub->begin(), sub->end(), [](const Elem& x, const Elem& y) { return x.tok < y.tok; });
}

// NormalizeSubset: the best weight (Plus) and the common prefix move out;
// *base becomes the prefix's node
LW PrunedDeterminizer::Normalize(std::vector<Elem>* sub, int* base) {
  LW tot = (*sub)[0].w;
  int common = (*sub)[0].str;
  for (size_t i = 1; i < sub->size(); i++) {
    if (CompareLWK(tot, (*sub)[i].w) < 0) tot = (*sub)[i].w;
    common = R_.Lca(common, (*sub)[i].str);
  }
  for (auto& e : *sub) e.w = Divide(e.w, tot);
  *base = common;
  return tot;
}

uint64_t PrunedDeterminizer::SubKey(const std::vector<Elem>& sub, int base) const {
  uint64_t k = 0x9e3779b97f4a7c15ull ^ sub.size();
  for (auto& e : sub) {
    k = (k ^ (uint64_t)(uint32_t)e.tok) * 0xff51afd7ed558ccdull;
    k = (k ^ (uint64_t)(uint32_t)R_.ResLen(e.str, base)) * 0xc4ceb9fe1a85ec53ull;
    k = (k ^ R_.ResHash(e.str, base)) * 0xff51afd7ed558ccdull;
    k ^= k >> 29;
  }
  return k;
}

// SubsetEqual: same states and strings, weights ApproxEqual within delta
bool PrunedDeterminizer::SubEqual(const std::vector<Elem>& x, int bx, const std::vector<Elem>& y, int by) const {
  if (x.size() != y.size()) return false;
  for (size_t i = 0; i < x.size(); i++)
    if (x[i].tok != y[i].tok || !ApproxEqualLW(x[i].w, y[i].w, opt_.delta)) return false;
  for (size_t i = 0; i < x.size(); i++)
    if (!R_.ResEqual(x[i].str, bx, y[i].str, by)) return false;
  return true;
}

int PrunedDeterminizer::AppendString(int node, int from_base, int to_node) {
  if (from_base == to_node) return node;
  std::vector<int> labels;
  R_.Get(to_node, from_base, &labels);
  for (int l : labels) node = Revive(R_.Succ(node, l));
  return node;
}

void PrunedDeterminizer::ProcessFinal(int s) {
  OState& st = states_[s];
  bool is_final = false;
  Elem best{0, LW{}, 0};
  for (const Elem& e : st.sub) {
    if (D_.fin[e.tok].g == kInf) continue;
    const Elem c{e.tok, Times(e.w, D_.fin[e.tok]), e.str};
    if (!is_final || Compare(c, st.base, best, st.base) > 0) {
      best = c;
      is_final = true;
    }
  }
  if (is_final && CostOf(best.w) + st.fwd <= cutoff_) {
    st.arcs.push_back(OArc{0, -1, best.w, best.str, st.base});
    num_arcs_++;
  }
}

void PrunedDeterminizer::ProcessTransitions(int s) {
  // (label, element) pairs of every label link out of the subset, sorted by
  // (label, state); one element per (label, state): the better one
  std::vector<std::pair<int, Elem>> all;
  {
    const OState& st = states_[s];
    for (const Elem& e : st.sub)
      for (int k = oe_[e.tok]; k < ob_[e.tok + 1]; k++) {
        const auto& l = cl_[k];
        int str = e.str;
        if (l.lin != 0) {
          if (memo_in_[k] == str) str = Revive(memo_out_[k]);
          else {
            const int n = Revive(R_.Succ(str, l.lin));
            memo_in_[k] = str;
            memo_out_[k] = n;
            str = n;
          }
        }
        all.push_back({l.lout, Elem{l.dst, Times(e.w, LW{l.g, l.a}), str}});
      }
  }
  const int base = states_[s].base;
  std::sort(all.begin(), all.end(), [&](const std::pair<int, Elem>& x, const std::pair<int, Elem>& y) {
    if (x.first != y.first) return x.first < y.first;
    if (x.second.tok != y.second.tok) return x.second.tok < y.second.tok;
    return Compare(x.second, base, y.second, base) > 0;
  });
  const double fwd = states_[s].fwd;
  for (size_t g0 = 0; g0 < all.size();) {
    const int label = all[g0].first;
    double prio = std::numeric_limits<double>::infinity();
    size_t g1 = g0;
    std::vector<Elem> sub;
    for (; g1 < all.size() && all[g1].first == label; g1++) {
      const Elem& e = all[g1].second;
      prio = std::min(prio, CostOf(e.w) + bwd_[e.tok]);
      if (sub.empty() || sub.back().tok != e.tok) sub.push_back(e);  // MakeSubsetUnique (sorted best first)
    }
    g0 = g1;
    prio += fwd;
    if (prio > cutoff_) continue;  // past the pruning cutoff: never done
    num_elems_ += (long long)sub.size();
    queue_.push(new Task{prio, seq_++, s, label, std::move(sub)});
  }
}

int PrunedDeterminizer::MinimalToState(std::vector<Elem>&& sub, int base, double fwd) {
  const uint64_t k = SubKey(sub, base);
  auto& cand = minimal_[k];
  for (int id : cand)
    if (SubEqual(states_[id].sub, states_[id].base, sub, base)) return id;
  const int id = (int)states_.size();
  num_elems_ += (long long)sub.size();
  states_.push_back(OState{std::move(sub), base, fwd, {}});
  cand.push_back(id);
  ProcessFinal(id);
  ProcessTransitions(id);
  return id;
}

int PrunedDeterminizer::InitialToState(const std::vector<Elem>& sub, int base, double fwd, LW* rem, int* rem_str,
                                       int* rem_base) {
  const uint64_t k = SubKey(sub, base);
  auto& cand = initial_[k];
  for (int ci : cand) {
    const Cached& c = cached_[ci];
    if (SubEqual(c.sub, c.base, sub, base)) {
      *rem = c.rem;
      *rem_str = c.rem_str;
      *rem_base = c.rem_base;
      return c.state;
    }
  }
  std::vector<Elem> cur(sub);
  Closure(&cur, base);
  ConvertToMinimal(&cur);
  if (cur.empty()) return -1;  // (cannot happen on a trimmed lattice)
  int nbase = base;
  const LW w2 = Normalize(&cur, &nbase);
  const int id = MinimalToState(std::move(cur), nbase, fwd + CostOf(w2));
  *rem = w2;
  *rem_str = nbase;
  *rem_base = base;
  num_elems_ += (long long)sub.size();
  initial_[k].push_back((int)cached_.size());
  cached_.push_back(Cached{sub, base, id, w2, nbase, base});
  return id;
}

void PrunedDeterminizer::ProcessTransition(Task* t) {
  const int s = t->state;
  double fwd = states_[s].fwd;
  int b1 = states_[s].base;
  const LW w1 = Normalize(&t->sub, &b1);  // prefix 1: state base -> b1
  fwd += CostOf(w1);
  LW w2;
  int s2 = 0, b2 = 0;
  const int next = InitialToState(t->sub, b1, fwd, &w2, &s2, &b2);
  if (next < 0) return;
  // the arc string: prefix 1 followed by the remaining prefix (b2 -> s2)
  const int str = AppendString(b1, b2, s2);
  states_[s].arcs.push_back(OArc{t->label, next, Times(w1, w2), str, states_[s].base});
  num_arcs_++;
}

// memory estimate (Kaldi CheckMemoryUsage: string repository + 32-byte temp
// arcs + 24-byte elements; the repository counted as 32 bytes per string,
// and after a rebuild as the strings then in use plus those added since, as
// RebuildRepository leaves Kaldi's repository -- so a check after a rebuild
// is cheap until the repository has grown past max_mem again)
bool PrunedDeterminizer::CheckMemory(double* eff) {
  const long long arcs = num_arcs_ * 32, elems = num_elems_ * 24;
  const long long nstr = rebuilt_live_ < 0 ? (long long)R_.parent.size()
                                           : rebuilt_live_ + revived_ + (long long)(R_.parent.size() - rebuilt_at_);
  long long repo = nstr * 32;
  if (opt_.max_mem <= 0 || repo + arcs + elems <= opt_.max_mem) return true;
  // rebuild: only strings referenced by states, arcs, tasks and the cache
  std::vector<char> used(R_.parent.size(), 0);
  auto mark = [&](int n) {
    while (n > 0 && !used[n]) {
      used[n] = 1;
      n = R_.parent[n];
    }
  };
  for (const OState& st : states_) {
    for (const Elem& e : st.sub) mark(e.str);
    mark(st.base);
    for (const OArc& a : st.arcs) mark(a.str);
  }
  for (const Cached& c : cached_) {
    for (const Elem& e : c.sub) mark(e.str);
    mark(c.rem_str);
  }
  std::vector<Task*> tmp;
  while (!queue_.empty()) {
    tmp.push_back(queue_.top());
    queue_.pop();
  }
  for (Task* t : tmp) {
    for (const Elem& e : t->sub) mark(e.str);
    queue_.push(t);
  }
  long long live = 0;
  for (char u : used) live += u;
  rebuilt_live_ = live;
  revived_ = 0;
  rebuilt_at_ = R_.parent.size();
  rebuilt_mark_.swap(used);
  repo = live * 32;
  if (repo + arcs + elems > (long long)(opt_.max_mem * 0.8)) {
    if (!queue_.empty()) *eff = queue_.top()->prio - bwd_[D_.start];
    return false;
  }
  return true;
}

bool PrunedDeterminizer::Run(double* effective_beam) {
  const int N = D_.n;
  eff_beam_ = opt_.beam;
  // out-links per state (CSR): label-epsilon links first, then label links
  const int NL = (int)D_.links.size();
  ob_.assign(N + 1, 0);
  oe_.assign(N, 0);
  std::vector<int> ol(NL);
  for (int i = 0; i < NL; i++) ob_[D_.links[i].src + 1]++;
  for (int t = 0; t < N; t++) ob_[t + 1] += ob_[t];
  {
    std::vector<int> fill(ob_.begin(), ob_.end() - 1);
    for (int i = 0; i < NL; i++)
      if (D_.links[i].lout == 0) ol[fill[D_.links[i].src]++] = i;
    for (int t = 0; t < N; t++) oe_[t] = fill[t];
    for (int i = 0; i < NL; i++)
      if (D_.links[i].lout != 0) ol[fill[D_.links[i].src]++] = i;
  }
  cl_.resize(NL);
  for (int k = 0; k < NL; k++) cl_[k] = D_.links[ol[k]];
  memo_in_.assign(NL, -1);
  memo_out_.assign(NL, -1);
  at_pos_.assign(N, -1);
  int F = 0;
  for (int f : D_.frame) F = f > F ? f : F;
  fbucket_.assign(F + 1, {});
  // ComputeBackwardWeight (reverse topological order) and the cutoff
  bwd_.assign(N, std::numeric_limits<double>::infinity());
  for (int i = (int)topo_.size() - 1; i >= 0; i--) {
    const int s = topo_[i];
    double c = D_.fin[s].g == kInf ? std::numeric_limits<double>::infinity() : CostOf(D_.fin[s]);
    for (int k = ob_[s]; k < ob_[s + 1]; k++) c = std::min(c, CostOf(LW{cl_[k].g, cl_[k].a}) + bwd_[cl_[k].dst]);
    bwd_[s] = c;
  }
  cutoff_ = bwd_[D_.start] + opt_.beam;
  // the start state: closure of the start, minimal, not normalized, forward cost 0
  {
    std::vector<Elem> s0{Elem{D_.start, LW{}, 0}};
    Closure(&s0, 0);
    ConvertToMinimal(&s0);
    num_elems_ += (long long)s0.size();
    states_.push_back(OState{std::move(s0), 0, 0.0, {}});
    minimal_[SubKey(states_[0].sub, 0)].push_back(0);
    ProcessFinal(0);
    ProcessTransitions(0);
  }
  bool done = true;
  while (!queue_.empty()) {
    const size_t ns = states_.size();
    if ((opt_.max_states > 0 && (int)ns > opt_.max_states)) {
      guard_ = true;
      done = false;
      break;
    }
    if (ns % 10 == 0 && !CheckMemory(&eff_beam_)) {
      done = false;
      break;
    }
    Task* t = queue_.top();
    queue_.pop();
    ProcessTransition(t);
    delete t;
  }
  while (!queue_.empty()) {
    delete queue_.top();
    queue_.pop();
  }
  *effective_beam = eff_beam_;
  return done;
}

void PrunedDeterminizer::Output(WordLattice* out) {
  WordLattice& W = *out;
  W = WordLattice();
  const int S = (int)states_.size();
  if (S == 0) return;
  // fst::Connect: states on a path from the start to a final weight
  std::vector<char> acc(S, 0), coacc(S, 0);
  {
    std::vector<int> st{0};
    acc[0] = 1;
    while (!st.empty()) {
      const int s = st.back();
      st.pop_back();
      for (const OArc& a : states_[s].arcs)
        if (a.next >= 0 && !acc[a.next]) {
          acc[a.next] = 1;
          st.push_back(a.next);
        }
    }
    std::vector<std::vector<int>> rev(S);
    for (int s = 0; s < S; s++)
      for (const OArc& a : states_[s].arcs) {
        if (a.next >= 0) rev[a.next].push_back(s);
        else coacc[s] = 1;
      }
    for (int s = 0; s < S; s++)
      if (coacc[s]) st.push_back(s);
    while (!st.empty()) {
      const int s = st.back();
      st.pop_back();
      for (int p : rev[s])
        if (!coacc[p]) {
          coacc[p] = 1;
          st.push_back(p);
        }
    }
  }
  if (!acc[0] || !coacc[0]) return;  // nothing within the beam reaches a final state
  std::vector<int> keep(S, -1);
  int K = 0;
  for (int s = 0; s < S; s++)
    if (acc[s] && coacc[s]) keep[s] = K++;
  // topological order (the lattice is acyclic), start state first: the
  // same DFS renumbering as the exact determinizer's output
  std::vector<int> indeg(K, 0), order;
  for (int s = 0; s < S; s++) {
    if (keep[s] < 0) continue;
    for (const OArc& a : states_[s].arcs)
      if (a.next >= 0 && keep[a.next] >= 0) indeg[keep[a.next]]++;
  }
  std::vector<int> orig(K);
  for (int s = 0; s < S; s++)
    if (keep[s] >= 0) orig[keep[s]] = s;
  std::vector<int> stk{0};
  while (!stk.empty()) {
    const int k = stk.back();
    stk.pop_back();
    order.push_back(k);
    const auto& arcs = states_[orig[k]].arcs;
    for (auto it = arcs.rbegin(); it != arcs.rend(); ++it)
      if (it->next >= 0 && keep[it->next] >= 0 && --indeg[keep[it->next]] == 0) stk.push_back(keep[it->next]);
  }
  if ((int)order.size() != K) VAMD_ERR("lattice determinization produced a cycle");
  std::vector<int> pos(K);
  for (int i = 0; i < K; i++) pos[order[i]] = i;
  W.arcs.resize(K);
  W.final_graph.assign(K, INFINITY);
  W.final_acoustic.assign(K, 0.0f);
  W.final_tids.resize(K);
  for (int k = 0; k < K; k++) {
    const OState& st = states_[orig[k]];
    const int p = pos[k];
    for (const OArc& a : st.arcs) {
      if (a.next < 0) {
        W.final_graph[p] = a.w.g;
        W.final_acoustic[p] = a.w.a;
        R_.Get(a.str, a.base, &W.final_tids[p]);
        continue;
      }
      if (keep[a.next] < 0) continue;
      WordLattice::Arc b;
      b.word = a.label;
      b.next = pos[keep[a.next]];
      b.graph = a.w.g;
      b.acoustic = a.w.a;
      R_.Get(a.str, a.base, &b.tids);
      W.arcs[p].push_back(std::move(b));
    }
  }
}

// topological order of a determinizer input (Kahn; links go forward in time
// or within a frame without cycles)
bool TopoOrder(const DetGraph& D, std::vector<int>* order) {
  std::vector<int> indeg(D.n, 0), ob(D.n + 1, 0), adj(D.links.size());
  for (const auto& l : D.links) {
    indeg[l.dst]++;
    ob[l.src + 1]++;
  }
  for (int s = 0; s < D.n; s++) ob[s + 1] += ob[s];
  {
    std::vector<int> fill(ob.begin(), ob.end() - 1);
    for (const auto& l : D.links) adj[fill[l.src]++] = l.dst;
  }
  order->clear();
  std::vector<int> st;
  for (int s = D.n - 1; s >= 0; s--)
    if (indeg[s] == 0) st.push_back(s);
  while (!st.empty()) {
    const int s = st.back();
    st.pop_back();
    order->push_back(s);
    for (int k = ob[s + 1] - 1; k >= ob[s]; k--)
      if (--indeg[adj[k]] == 0) st.push_back(adj[k]);
  }
  return (int)order->size() == D.n;
}

// kaldi::PruneLattice on a determinizer input: links (and final weights)
// whose best path through them is beyond best + beam are dropped, then the
// states off every start -> final path
DetGraph PruneDetGraph(const DetGraph& D, const std::vector<int>& topo, double beam) {
  const int N = D.n;
  const double inf = std::numeric_limits<double>::infinity();
  std::vector<double> fw(N, inf), bw(N, inf);
  std::vector<std::vector<int>> out(N);
  for (int i = 0; i < (int)D.links.size(); i++) out[D.links[i].src].push_back(i);
  fw[D.start] = 0.0;
  double best = inf;
  for (int s : topo) {
    for (int i : out[s]) {
      const auto& l = D.links[i];
      fw[l.dst] = std::min(fw[l.dst], fw[s] + CostOf(LW{l.g, l.a}));
    }
    if (D.fin[s].g != kInf) best = std::min(best, fw[s] + CostOf(D.fin[s]));
  }
  const double cut = best + beam;
  std::vector<char> keep_link(D.links.size(), 1);
  DetGraph P = D;
  for (int k = N - 1; k >= 0; k--) {
    const int s = topo[k];
    double b = D.fin[s].g == kInf ? inf : CostOf(D.fin[s]);
    if (b != inf && b + fw[s] > cut) P.fin[s] = LW{kInf, 0.0f};
    for (int i : out[s]) {
      const auto& l = D.links[i];
      const double ab = CostOf(LW{l.g, l.a}) + bw[l.dst];
      if (ab < b) b = ab;
      if (fw[s] + ab > cut) keep_link[i] = 0;
    }
    bw[s] = b;
  }
  P.links.clear();
  for (size_t i = 0; i < D.links.size(); i++)
    if (keep_link[i]) P.links.push_back(D.links[i]);
  return P;  // (unreachable states stay, isolated: the determinizer never visits them)
}

// DeterminizeLatticePruned: retry at a narrower beam when memory stopped the
// determinization short of beam * retry_cutoff
bool DeterminizePrunedRetry(const DetGraph& D, double beam, const LatticeOptions& opt, WordLattice* out) {
  WordLattice& W = *out;
  W = WordLattice();
  if (D.n == 0 || D.start < 0) return true;
  std::vector<int> topo;
  if (!TopoOrder(D, &topo)) VAMD_ERR("lattice determinization: input has a cycle");
  const int kMaxIters = 10;
  const double retry_cutoff = 0.7;
  DetGraph tmp;
  for (int iter = 0; iter < kMaxIters; iter++) {
    PrunedDetOptions po;
    po.beam = beam;
    po.max_states = opt.max_states;
    po.max_mem = opt.det_max_mem;
    PrunedDeterminizer det(iter == 0 ? D : tmp, topo, po);
    double eff = beam;
    const bool ok = det.Run(&eff);
    if (det.guard_tripped()) return false;
    if (eff >= beam * retry_cutoff || std::isinf(beam) || iter + 1 == kMaxIters) {
      det.Output(out);
      (void)ok;  // stopped at a narrower beam: still the lattice Kaldi returns (and uses)
      return true;
    }
    double nb = beam * std::sqrt(std::max(eff, 0.0) / beam);  // (rounding can put eff just below 0: Kaldi would take NaN)
    if (nb < 0.25 * beam) nb = 0.25 * beam;
    beam = nb;
    tmp = PruneDetGraph(iter == 0 ? D : tmp, topo, beam);
  }
  return false;
}

}  // namespace

bool DeterminizeToWords(const RawLattice& L, const Graph& g, const LatticeOptions& opt, WordLattice* out) {
  return Determinize(FromRaw(L, g), opt, out);
}

bool DeterminizePhonePruned(const RawLattice& L, const Graph& g, const std::vector<int>& tid2phone,
                            const std::vector<char>& tid_first, const LatticeOptions& opt, WordLattice* out) {
  return DeterminizePhonePrunedGraph(FromRaw(L, g), tid2phone, tid_first, opt, out);
}

bool DeterminizePhonePrunedGraph(DetGraph D, const std::vector<int>& tid2phone, const std::vector<char>& tid_first,
                                 const LatticeOptions& opt, WordLattice* out) {
  // DeterminizeLatticeInsertPhones: a phone label (first_phone_label + phone,
  // first_phone_label = the highest word label + 1) at the first
  // transition-id of every phone (HMM state 0, not a self-loop); on the link
  // itself when it has no word, else on a new link after it (through a new
  // state), weight One
  int first = 1;
  for (const auto& l : D.links) first = std::max(first, l.lout + 1);
  const size_t nl = D.links.size();
  for (size_t i = 0; i < nl; i++) {
    const int t = D.links[i].lin;
    if (D.links[i].src == D.start) continue;  // the start state's arcs get no phone (Kaldi skips them)
    if (t <= 0 || t >= (int)tid_first.size() || !tid_first[t]) continue;
    const int ph = first + tid2phone[t];
    if (D.links[i].lout == 0) {
      D.links[i].lout = ph;
    } else {
      const int dst = D.links[i].dst;
      const int x = D.AddState(D.frame[dst]);
      D.links[i].dst = x;
      D.links.push_back(DetGraph::Link{x, dst, 0, ph, 0.0f, 0.0f});
    }
  }
  // first pass: pruned determinization on phones + words
  WordLattice P;
  if (!DeterminizePrunedRetry(D, opt.lattice_beam, opt, &P)) return false;
  if (P.NumStates() == 0) {
    *out = WordLattice();
    return true;
  }
  // LatticeDeterminizerPruned::Output to a Lattice: each arc's string as a
  // chain of one-transition-id links, label and weight on the first; a final
  // string as a chain to a new final state (weight on its first link);
  // DeterminizeLatticeDeletePhones: phone labels -> 0
  const int S = P.NumStates();
  DetGraph E;
  E.n = S;
  E.start = 0;
  E.frame.assign(S, 0);
  E.fin.assign(S, LW{kInf, 0.0f});
  for (int s = 0; s < S; s++)  // topologically sorted: frames forward
    for (const auto& a : P.arcs[s]) E.frame[a.next] = std::max(E.frame[a.next], E.frame[s] + (int)a.tids.size());
  auto label = [&](int w) { return w >= first ? 0 : w; };
  for (int s = 0; s < S; s++) {
    for (const auto& a : P.arcs[s]) {
      const int n = (int)a.tids.size();
      if (n == 0) {
        E.links.push_back(DetGraph::Link{s, a.next, 0, label(a.word), a.graph, a.acoustic});
        continue;
      }
      int cur = s;
      for (int i = 0; i < n; i++) {
        const int nx = i + 1 == n ? a.next : E.AddState(E.frame[s] + i + 1);
        E.links.push_back(DetGraph::Link{cur, nx, a.tids[i], i == 0 ? label(a.word) : 0, i == 0 ? a.graph : 0.0f,
                                         i == 0 ? a.acoustic : 0.0f});
        cur = nx;
      }
    }
    if (P.final_graph[s] == kInf) continue;
    const std::vector<int>& ft = P.final_tids[s];
    if (ft.empty()) {
      E.fin[s] = LW{P.final_graph[s], P.final_acoustic[s]};
      continue;
    }
    int cur = s;
    for (size_t i = 0; i < ft.size(); i++) {
      const int nx = E.AddState(E.frame[s] + (int)i + 1);
      E.links.push_back(DetGraph::Link{cur, nx, ft[i], 0, i == 0 ? P.final_graph[s] : 0.0f,
                                       i == 0 ? P.final_acoustic[s] : 0.0f});
      cur = nx;
    }
    E.fin[cur] = LW{0.0f, 0.0f};
  }
  // second pass: word level (DeterminizeLatticePruned)
  return DeterminizePrunedRetry(E, opt.lattice_beam, opt, out);
}

void ScaleGraph(WordLattice* lat, float scale) {
  for (auto& v : lat->arcs)
    for (auto& a : v) a.graph *= scale;
  for (auto& f : lat->final_graph)
    if (f != INFINITY) f *= scale;
}

namespace {

// Kaldi LogAdd (base/kaldi-math.h)
inline double LogAdd(double x, double y) {
  double diff;
  if (x < y) {
    diff = x - y;
    x = y;
  } else {
    diff = y - x;
  }
  static const double kMinLogDiff = std::log(std::numeric_limits<double>::epsilon());
  if (diff >= kMinLogDiff) return x + std::log1p(std::exp(diff));
  return x;
}

struct MbrArc {
  int word, start, end;
  double loglike;
};

class Mbr {
 public:
  explicit Mbr(const WordLattice& W) {
    // CreateSuperFinal: final weights become epsilon arcs into one new final
    // state (numbered last: the lattice stays topologically sorted)
    const int S = W.NumStates();
    N_ = S + 1;
    pre_.assign(N_ + 1, {});
    times_st_.assign(N_ + 1, 0);
    std::vector<int> t(S + 1, -1);
    t[0] = 0;
    for (int s = 0; s < S; s++) {
      for (const auto& a : W.arcs[s]) {
        add(s + 1, a.next + 1, a.word, -(double)(a.graph + a.acoustic));
        t[a.next] = t[s] + (int)a.tids.size();
      }
      if (W.final_graph[s] != INFINITY) {
        add(s + 1, N_, 0, -(double)(W.final_graph[s] + W.final_acoustic[s]));
        t[S] = t[s] + (int)W.final_tids[s].size();
      }
    }
    for (int s = 0; s <= S; s++) times_st_[s + 1] = std::max(0, t[s]);
    // initial hypothesis: the best path's words
    std::vector<double> best(N_ + 1, -INFINITY);
    std::vector<int> from(N_ + 1, -1);
    best[1] = 0.0;
    for (int n = 2; n <= N_; n++)
      for (int ai : pre_[n]) {
        const MbrArc& a = arcs_[ai];
        const double v = best[a.start] + a.loglike;
        if (v > best[n]) {
          best[n] = v;
          from[n] = ai;
        }
      }
    for (int n = N_; n > 1 && from[n] >= 0; n = arcs_[from[n]].start)
      if (arcs_[from[n]].word != 0) R_.push_back(arcs_[from[n]].word);
    std::reverse(R_.begin(), R_.end());
    Decode();
  }
  MbrResult result;

 private:
  void add(int s, int e, int w, double ll) {
    pre_[e].push_back((int)arcs_.size());
    arcs_.push_back(MbrArc{w, s, e, ll});
  }
  static double l(int a, int b, bool penalize = false) {
    return a == b ? 0.0 : (penalize ? 1.0 + 1.0e-05 : 1.0);
  }
  int r(int q) const { return R_[q - 1]; }
  void NormalizeEps() {
    std::vector<int> x{0};
    for (int w : R_)
      if (w != 0) {
        x.push_back(w);
        x.push_back(0);
      }
    R_ = x;
  }
  double EditDistance(int N, int Q, std::vector<double>& alpha, std::vector<std::vector<double>>& ad,
                      std::vector<double>& ada) {
    alpha[1] = 0.0;
    ad[1][0] = 0.0;
    for (int q = 1; q <= Q; q++) ad[1][q] = ad[1][q - 1] + l(0, r(q));
    for (int n = 2; n <= N; n++) {
      double an = -INFINITY;
      for (int ai : pre_[n]) an = LogAdd(an, alpha[arcs_[ai].start] + arcs_[ai].loglike);
      alpha[n] = an;
      for (int ai : pre_[n]) {
        const MbrArc& a = arcs_[ai];
        for (int q = 0; q <= Q; q++) {
          if (q == 0) {
            ada[q] = ad[a.start][q] + l(a.word, 0, true);
          } else {
            // substitution, insertion of the arc's word, deletion of r_q
            const int rq = r(q);
            const double a1 = ad[a.start][q - 1] + l(a.word, rq), a2 = ad[a.start][q] + l(a.word, 0, true),
                         a3 = ada[q - 1] + l(0, rq);
            ada[q] = std::min(a1, std::min(a2, a3));
          }
          ad[n][q] += std::exp(alpha[a.start] + a.loglike - alpha[n]) * ada[q];
        }
      }
    }
    return ad[N][Q];
  }
  void AccStats() {
    const int N = N_, Q = (int)R_.size();
    std::vector<double> alpha(N + 1, 0.0), ada(Q + 1, 0.0), bda(Q + 1, 0.0);
    std::vector<std::vector<double>> ad(N + 1, std::vector<double>(Q + 1, 0.0)),
        bd(N + 1, std::vector<double>(Q + 1, 0.0));
    std::vector<char> b_arc(Q + 1, 0);
    std::vector<std::map<int, double>> gamma(Q + 1);
    std::vector<double> tau_b(Q + 1, 0.0), tau_e(Q + 1, 0.0);
    EditDistance(N, Q, alpha, ad, ada);
    bd[N][Q] = 1.0;
    for (int n = N; n >= 2; n--) {
      for (int ai : pre_[n]) {
        const MbrArc& a = arcs_[ai];
        const int sa = a.start, wa = a.word;
        ada[0] = ad[sa][0] + l(wa, 0, true);
        for (int q = 1; q <= Q; q++) {
          const int rq = r(q);
          const double a1 = ad[sa][q - 1] + l(wa, rq), a2 = ad[sa][q] + l(wa, 0, true),
                       a3 = ada[q - 1] + l(0, rq);
          if (a1 <= a2) {
            if (a1 <= a3) { b_arc[q] = 1; ada[q] = a1; }
            else { b_arc[q] = 3; ada[q] = a3; }
          } else {
            if (a2 <= a3) { b_arc[q] = 2; ada[q] = a2; }
            else { b_arc[q] = 3; ada[q] = a3; }
          }
        }
        std::fill(bda.begin(), bda.end(), 0.0);
        const double post = std::exp(alpha[sa] + a.loglike - alpha[n]);
        for (int q = Q; q >= 1; q--) {
          bda[q] += post * bd[n][q];
          switch (b_arc[q]) {
            case 1:  // the arc's word in bin q
              bd[sa][q - 1] += bda[q];
              gamma[q][wa] += bda[q];
              tau_b[q] += times_st_[sa] * bda[q];
              tau_e[q] += times_st_[n] * bda[q];
              break;
            case 2:
              bd[sa][q] += bda[q];
              break;
            default:  // epsilon in bin q, within the arc
              bda[q - 1] += bda[q];
              gamma[q][0] += bda[q];
              tau_b[q] += times_st_[sa] * bda[q];
              tau_e[q] += times_st_[n] * bda[q];
              break;
          }
        }
        bda[0] += post * bd[n][0];
        bd[sa][0] += bda[0];
      }
    }
    std::fill(bda.begin(), bda.end(), 0.0);
    for (int q = Q; q >= 1; q--) {
      bda[q] += bd[1][q];
      bda[q - 1] += bda[q];
      gamma[q][0] += bda[q];
      tau_b[q] += times_st_[1] * bda[q];
      tau_e[q] += times_st_[1] * bda[q];
    }
    gamma_.assign(Q, {});
    times_.assign(Q, {});
    for (int q = 1; q <= Q; q++) {
      for (auto& kv : gamma[q]) gamma_[q - 1].push_back({kv.first, (float)kv.second});
      std::stable_sort(gamma_[q - 1].begin(), gamma_[q - 1].end(),
                       [](const std::pair<int, float>& x, const std::pair<int, float>& y) {
                         return x.second > y.second;
                       });
      times_[q - 1] = {(float)tau_b[q], (float)tau_e[q]};
    }
  }
  void Decode() {
    for (int iter = 0;; iter++) {
      NormalizeEps();
      AccStats();
      double dq = 0.0;
      result = MbrResult();
      for (size_t q = 0; q < R_.size(); q++) {
        const auto& g = gamma_[q];
        double old_g = 0.0;
        const double new_g = g.empty() ? 0.0 : g[0].second;
        for (auto& x : g)
          if (x.first == R_[q]) old_g = x.second;
        dq += old_g - new_g;
        if (!g.empty()) R_[q] = g[0].first;
        if (R_[q] != 0) {
          float conf = 0.0f;
          for (auto& x : g)
            if (x.first == R_[q]) conf = x.second;
          result.words.push_back(R_[q]);
          result.conf.push_back(conf);
          result.times.push_back(times_[q]);
        }
      }
      if (dq == 0.0 || iter > 100) break;
    }
  }
  int N_ = 0;
  std::vector<MbrArc> arcs_;
  std::vector<std::vector<int>> pre_;
  std::vector<int> times_st_;
  std::vector<int> R_;
  std::vector<std::vector<std::pair<int, float>>> gamma_;
  std::vector<std::pair<float, float>> times_;
};

}  // namespace

void MinimumBayesRisk(const WordLattice& lat, MbrResult* out) {
  *out = MbrResult();
  if (lat.NumStates() == 0) return;
  Mbr m(lat);
  *out = m.result;
}

void NbestPaths(const WordLattice& W, int n, std::vector<NbestPath>* out) {
  out->clear();
  const int S = W.NumStates();
  if (S == 0 || n <= 0) return;
  // k best completions per state (the lattice is determinized: distinct
  // paths are distinct word sequences), backwards in topological order
  struct Cand {
    float g, a;
    int arc;   // index into W.arcs[s], -1 = final
    int rank;  // rank of the continuation at the arc's next state
  };
  auto better = [](const Cand& x, const Cand& y) {
    return CompareLW(LW{x.g, x.a}, LW{y.g, y.a}) > 0;
  };
  std::vector<std::vector<Cand>> best(S);
  for (int s = S - 1; s >= 0; s--) {
    std::vector<Cand> c;
    if (W.final_graph[s] != INFINITY) c.push_back(Cand{W.final_graph[s], W.final_acoustic[s], -1, 0});
    for (int i = 0; i < (int)W.arcs[s].size(); i++) {
      const auto& a = W.arcs[s][i];
      for (int k = 0; k < (int)best[a.next].size(); k++)
        c.push_back(Cand{a.graph + best[a.next][k].g, a.acoustic + best[a.next][k].a, i, k});
    }
    std::stable_sort(c.begin(), c.end(), better);
    if ((int)c.size() > n) c.resize(n);
    best[s] = std::move(c);
  }
  for (int k = 0; k < (int)best[0].size(); k++) {
    NbestPath p;
    p.graph = best[0][k].g;
    p.acoustic = best[0][k].a;
    int s = 0, rank = k, t = 0;
    while (true) {
      const Cand& c = best[s][rank];
      if (c.arc < 0) break;
      const auto& a = W.arcs[s][c.arc];
      const int len = (int)a.tids.size();
      if (a.word != 0) {
        p.words.push_back(a.word);
        p.spans.push_back({t, t + len});
      }
      t += len;
      s = a.next;
      rank = c.rank;
    }
    out->push_back(std::move(p));
  }
}

}  // namespace vamd

// ===========================================================================
// word alignment
// ===========================================================================
namespace vamd {

namespace {

struct AlignCtx {
  const std::vector<char>& type;  // per tid: boundary type of its phone
  const std::vector<char>& fin;   // per tid: IsFinal
  const std::vector<char>& loop;  // per tid: IsSelfLoop
  int Type(int tid) const { return tid < (int)type.size() ? type[tid] : 0; }
};

// index just past the phone that starts at i (its final transition-id and,
// with reorder, the self-loops after it); -1 if the phone is not known to be
// complete within t
int PhoneEnd(const AlignCtx& c, const std::vector<int>& t, size_t i) {
  const size_t len = t.size();
  for (; i < len; i++)
    if (c.fin[t[i]]) break;
  if (i == len) return -1;
  i++;
  while (i < len && c.loop[t[i]]) i++;
  if (i == len) return -1;
  return (int)i;
}

// LatticeWordAligner::ComputationState::OutputArc: silence phone, one-phone
// word, normal word; returns the number of transition-ids consumed and the
// label (0 for silence), or -1 if nothing can be output yet
int TryOutput(const AlignCtx& c, const std::vector<int>& t, const std::vector<int>& words, int* label) {
  if (t.empty()) return -1;
  const int ty = c.Type(t[0]);
  if (ty == 1) {  // nonword
    *label = 0;
    return PhoneEnd(c, t, 0);
  }
  if (words.empty()) return -1;
  if (ty == 5) {  // begin-and-end
    *label = words[0];
    return PhoneEnd(c, t, 0);
  }
  if (ty == 2) {  // begin: up to the end phone's end
    size_t i = 0;
    while (i < t.size() && c.Type(t[i]) != 3) i++;
    if (i == t.size()) return -1;
    *label = words[0];
    return PhoneEnd(c, t, i);
  }
  return -1;
}

struct ANode {
  int in;                  // input (word lattice) state, -1 = past a final flush
  std::vector<int> t, w;   // pending transition-ids and word labels
};

}  // namespace

bool WordAlignLattice(const WordLattice& W, const std::vector<char>& type, const std::vector<char>& fin,
                      const std::vector<char>& loop, int max_states, WordLattice* out) {
  *out = WordLattice();
  const int S = W.NumStates();
  if (S == 0) return true;
  const AlignCtx c{type, fin, loop};
  std::vector<ANode> nodes;
  std::unordered_map<std::string, int> index;
  // node edges: epsilon advances (weight) and output arcs (label, tids)
  struct Eps { int to; LW w; };
  struct Out { int to, label; std::vector<int> tids; };
  std::vector<std::vector<Eps>> eps;
  std::vector<std::vector<Out>> outs;
  std::vector<char> is_final;
  auto key_of = [](const ANode& n) {
    std::string k((const char*)&n.in, sizeof(int));
    const int a = (int)n.t.size(), b = (int)n.w.size();
    k.append((const char*)&a, sizeof(int));
    k.append((const char*)n.t.data(), sizeof(int) * a);
    k.append((const char*)&b, sizeof(int));
    k.append((const char*)n.w.data(), sizeof(int) * b);
    return k;
  };
  std::vector<int> queue;
  auto get = [&](ANode&& n) {
    const std::string k = key_of(n);
    auto it = index.find(k);
    if (it != index.end()) return it->second;
    const int id = (int)nodes.size();
    index[k] = id;
    nodes.push_back(std::move(n));
    eps.emplace_back();
    outs.emplace_back();
    is_final.push_back(0);
    queue.push_back(id);
    return id;
  };
  get(ANode{0, {}, {}});
  for (size_t qi = 0; qi < queue.size(); qi++) {
    if ((int)nodes.size() > max_states) return false;
    const int id = queue[qi];
    const ANode n = nodes[id];
    int label = 0;
    const int k = TryOutput(c, n.t, n.w, &label);
    if (k >= 0) {  // something pending goes out first (no advancing)
      ANode m{n.in, std::vector<int>(n.t.begin() + k, n.t.end()), n.w};
      if (label != 0) m.w.erase(m.w.begin());
      std::vector<int> tids(n.t.begin(), n.t.begin() + k);
      const int to = get(std::move(m));
      outs[id].push_back(Out{to, label, std::move(tids)});
      continue;
    }
    if (n.in < 0) {  // past the input's final weight: flush (OutputArcForce)
      if (n.t.empty() && n.w.empty()) {
        is_final[id] = 1;
        continue;
      }
      // a leading non-word phone: everything pending goes out as silence
      // (word labels follow with empty strings); else a partial word with
      // the first pending label (partial_word_label 0 if none)
      ANode m{-1, {}, n.w};
      int lab = 0;
      if (!(!n.t.empty() && c.Type(n.t[0]) == 1) && !m.w.empty()) {
        lab = m.w[0];
        m.w.erase(m.w.begin());
      }
      const int to = get(std::move(m));
      outs[id].push_back(Out{to, lab, n.t});
      continue;
    }
    // the input state's final weight (CreateSuperFinal: an epsilon arc with
    // the final string into a super-final input state)
    if (W.final_graph[n.in] != INFINITY) {
      ANode m{-1, n.t, n.w};
      m.t.insert(m.t.end(), W.final_tids[n.in].begin(), W.final_tids[n.in].end());
      const int to = get(std::move(m));
      eps[id].push_back(Eps{to, LW{W.final_graph[n.in], W.final_acoustic[n.in]}});
    }
    for (const auto& a : W.arcs[n.in]) {
      ANode m{a.next, n.t, n.w};
      m.t.insert(m.t.end(), a.tids.begin(), a.tids.end());
      if (a.word != 0) m.w.push_back(a.word);
      const int to = get(std::move(m));
      eps[id].push_back(Eps{to, LW{a.graph, a.acoustic}});
    }
  }
  // RmEpsilon: each node's output arcs and finality through its epsilon
  // closure (best weight per reached node, Kaldi LatticeWeight order)
  const int N = (int)nodes.size();
  std::vector<std::vector<WordLattice::Arc>> arcs(N);
  std::vector<LW> fw(N);
  std::vector<char> isf(N, 0);
  for (int x = 0; x < N; x++) {
    std::unordered_map<int, LW> clo;
    std::vector<int> order, st{x};
    clo[x] = LW{};
    // the epsilon graph is acyclic: relax in DFS discovery order, then
    // settle in topological order
    std::vector<int> topo;
    {
      std::unordered_map<int, int> mark;  // 1 = visiting, 2 = done
      std::vector<std::pair<int, size_t>> stk{{x, 0}};
      mark[x] = 1;
      while (!stk.empty()) {
        auto& [u, i] = stk.back();
        if (i < eps[u].size()) {
          const int v = eps[u][i++].to;
          if (!mark.count(v)) {
            mark[v] = 1;
            stk.push_back({v, 0});
          }
        } else {
          mark[u] = 2;
          topo.push_back(u);
          stk.pop_back();
        }
      }
      std::reverse(topo.begin(), topo.end());
    }
    for (int u : topo)
      for (const Eps& e : eps[u]) {
        const LW cand = Times(clo[u], e.w);
        auto it = clo.find(e.to);
        if (it == clo.end() || CompareLW(cand, it->second) > 0) clo[e.to] = cand;
      }
    for (int u : topo) {
      const LW cw = clo[u];
      for (const Out& o : outs[u]) arcs[x].push_back(WordLattice::Arc{o.label, o.to, cw.g, cw.a, o.tids});
      if (is_final[u] && (!isf[x] || CompareLW(cw, fw[x]) > 0)) {
        isf[x] = 1;
        fw[x] = cw;
      }
    }
  }
  // connect: states reachable by output arcs from the start and co-reachable
  std::vector<char> reach(N, 0), coreach(N, 0);
  std::vector<int> st{0};
  reach[0] = 1;
  while (!st.empty()) {
    const int u = st.back();
    st.pop_back();
    for (auto& a : arcs[u])
      if (!reach[a.next]) {
        reach[a.next] = 1;
        st.push_back(a.next);
      }
  }
  std::vector<std::vector<int>> rev(N);
  for (int u = 0; u < N; u++)
    for (auto& a : arcs[u]) rev[a.next].push_back(u);
  for (int u = 0; u < N; u++)
    if (isf[u] && reach[u]) {
      coreach[u] = 1;
      st.push_back(u);
    }
  while (!st.empty()) {
    const int u = st.back();
    st.pop_back();
    for (int p : rev[u])
      if (!coreach[p] && reach[p]) {
        coreach[p] = 1;
        st.push_back(p);
      }
  }
  if (!coreach[0]) return true;  // nothing complete: empty lattice
  // topological renumbering (output arcs only; acyclic), start first
  std::vector<int> indeg(N, 0), order;
  for (int u = 0; u < N; u++)
    if (coreach[u])
      for (auto& a : arcs[u])
        if (coreach[a.next]) indeg[a.next]++;
  st.assign(1, 0);
  while (!st.empty()) {
    const int u = st.back();
    st.pop_back();
    order.push_back(u);
    for (auto it = arcs[u].rbegin(); it != arcs[u].rend(); ++it)
      if (coreach[it->next] && --indeg[it->next] == 0) st.push_back(it->next);
  }
  std::vector<int> pos(N, -1);
  for (size_t i = 0; i < order.size(); i++) pos[order[i]] = (int)i;
  const int M = (int)order.size();
  out->arcs.resize(M);
  out->final_graph.assign(M, INFINITY);
  out->final_acoustic.assign(M, 0.0f);
  out->final_tids.resize(M);
  for (int i = 0; i < M; i++) {
    const int u = order[i];
    for (auto& a : arcs[u])
      if (coreach[a.next]) {
        WordLattice::Arc b = a;
        b.next = pos[a.next];
        out->arcs[i].push_back(std::move(b));
      }
    if (isf[u]) {
      out->final_graph[i] = fw[u].g;
      out->final_acoustic[i] = fw[u].a;
    }
  }
  return true;
}

}  // namespace vamd
