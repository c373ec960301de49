// Static composition of lookahead graph pairs and runtime grammars
// (graph_compose.h).
#include "graph_compose.h"

#include <algorithm>
#include <chrono>
#include <cctype>
#include <cmath>
#include <functional>
#include <sstream>
#include <limits>
#include <cstring>
#include <map>
#include <unordered_map>
#include <memory>
#include <utility>

#include "common.h"

namespace vamd {
namespace {

using Intervals = std::vector<std::pair<int, int>>;  // sorted, disjoint, non-adjacent [lo, hi]

void Coalesce(Intervals* v) {
  if (v->empty()) return;
  std::sort(v->begin(), v->end());
  size_t o = 0;
  for (size_t i = 1; i < v->size(); i++) {
    auto& b = (*v)[o];
    const auto& c = (*v)[i];
    if ((long long)c.first <= (long long)b.second + 1) {
      b.second = std::max(b.second, c.second);
    } else {
      (*v)[++o] = c;
    }
  }
  v->resize(o + 1);
}

// Output labels reachable from each state of `a` through output-epsilon arcs
// (the label of the first non-epsilon output arc on such a path), and whether
// a final state is reachable that way: per strongly connected component of
// the output-epsilon subgraph (Tarjan, iterative; components complete sinks
// first, so successors are done before their predecessors).
struct Reach {
  std::vector<int> comp;               // per state
  std::vector<Intervals> labels;       // per component
  std::vector<char> final;             // per component
  std::vector<int> cls;                // per component: id of its (labels, final) set
};

void ComputeReach(const HostFst& a, Reach* r) {
  const int S = a.NumStates();
  std::vector<int> idx(S, -1), low(S, 0);
  std::vector<char> onst(S, 0);
  std::vector<int> st;
  struct Frame { int v; int64_t arc; };
  std::vector<Frame> cs;
  r->comp.assign(S, -1);
  int counter = 0, ncomp = 0;
  for (int root = 0; root < S; root++) {
    if (idx[root] >= 0) continue;
    idx[root] = low[root] = counter++;
    st.push_back(root);
    onst[root] = 1;
    cs.push_back({root, a.row[root]});
    while (!cs.empty()) {
      Frame& fr = cs.back();
      const int v = fr.v;
      if (fr.arc < a.row[v + 1]) {
        const int64_t e = fr.arc++;
        if (a.olabel[e] != 0) continue;
        const int w = a.nextstate[e];
        if (idx[w] < 0) {
          idx[w] = low[w] = counter++;
          st.push_back(w);
          onst[w] = 1;
          cs.push_back({w, a.row[w]});
        } else if (onst[w]) {
          low[v] = std::min(low[v], idx[w]);
        }
      } else {
        if (low[v] == idx[v]) {
          while (true) {
            const int x = st.back();
            st.pop_back();
            onst[x] = 0;
            r->comp[x] = ncomp;
            if (x == v) break;
          }
          ncomp++;
        }
        cs.pop_back();
        if (!cs.empty()) low[cs.back().v] = std::min(low[cs.back().v], low[v]);
      }
    }
  }
  // members of each component
  std::vector<int> cbeg(ncomp + 1, 0), members(S);
  for (int s = 0; s < S; s++) cbeg[r->comp[s] + 1]++;
  for (int c = 0; c < ncomp; c++) cbeg[c + 1] += cbeg[c];
  {
    std::vector<int> fill(cbeg.begin(), cbeg.end() - 1);
    for (int s = 0; s < S; s++) members[fill[r->comp[s]]++] = s;
  }
  r->labels.assign(ncomp, Intervals());
  r->final.assign(ncomp, 0);
  // components reaching the same set of successor components (word-boundary
  // states: every word's first phone) share the merged successor lists
  std::map<std::vector<int>, std::pair<Intervals, char>> merged;
  std::vector<int> succ;
  for (int c = 0; c < ncomp; c++) {
    Intervals acc;
    char fin = 0;
    succ.clear();
    for (int m = cbeg[c]; m < cbeg[c + 1]; m++) {
      const int v = members[m];
      if (std::isfinite(a.final_cost[v])) fin = 1;
      for (int64_t e = a.row[v]; e < a.row[v + 1]; e++) {
        if (a.olabel[e] != 0) {
          acc.push_back({a.olabel[e], a.olabel[e]});
        } else {
          const int d = r->comp[a.nextstate[e]];
          if (d != c) succ.push_back(d);
        }
      }
    }
    std::sort(succ.begin(), succ.end());
    succ.erase(std::unique(succ.begin(), succ.end()), succ.end());
    if (succ.size() >= 16) {
      auto it = merged.find(succ);
      if (it == merged.end()) {
        Intervals u;
        char f = 0;
        for (int d : succ) {
          f |= r->final[d];
          u.insert(u.end(), r->labels[d].begin(), r->labels[d].end());
        }
        Coalesce(&u);
        it = merged.emplace(succ, std::make_pair(std::move(u), f)).first;
      }
      fin |= it->second.second;
      acc.insert(acc.end(), it->second.first.begin(), it->second.first.end());
    } else {
      for (int d : succ) {
        fin |= r->final[d];
        acc.insert(acc.end(), r->labels[d].begin(), r->labels[d].end());
      }
    }
    Coalesce(&acc);
    r->labels[c] = std::move(acc);
    r->final[c] = fin;
  }
  // components with equal reachable sets (e.g. the word-end states, which
  // all continue with every word) share a class: lookahead results and arc
  // indexes depend only on the set
  std::map<std::pair<Intervals, char>, int> classes;
  r->cls.assign(ncomp, 0);
  for (int c = 0; c < ncomp; c++)
    r->cls[c] = classes.emplace(std::make_pair(r->labels[c], r->final[c]), (int)classes.size()).first->second;
}

// composed state -> id (open addressing; key = q1 << 33 | q2 << 1 | filter)
struct StateTable {
  std::vector<uint64_t> keys;
  std::vector<int> vals;
  size_t count = 0;
  static uint64_t Mix(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
  }
  StateTable() { keys.assign(1 << 16, ~0ull); vals.assign(1 << 16, -1); }
  void Grow() {
    std::vector<uint64_t> ok;
    std::vector<int> ov;
    ok.swap(keys);
    ov.swap(vals);
    keys.assign(ok.size() * 2, ~0ull);
    vals.assign(ok.size() * 2, -1);
    const uint64_t mask = keys.size() - 1;
    for (size_t i = 0; i < ok.size(); i++) {
      if (ok[i] == ~0ull) continue;
      uint64_t h = Mix(ok[i]) & mask;
      while (keys[h] != ~0ull) h = (h + 1) & mask;
      keys[h] = ok[i];
      vals[h] = ov[i];
    }
  }
  // returns the id; *added when new (id = next_id)
  int FindOrAdd(uint64_t key, int next_id, bool* added) {
    if ((count + 1) * 2 > keys.size()) Grow();
    const uint64_t mask = keys.size() - 1;
    uint64_t h = Mix(key) & mask;
    while (keys[h] != ~0ull) {
      if (keys[h] == key) { *added = false; return vals[h]; }
      h = (h + 1) & mask;
    }
    keys[h] = key;
    vals[h] = next_id;
    count++;
    *added = true;
    return next_id;
  }
};

// Trim to the states that reach a final state and renumber breadth-first from
// the start over each state's emitting arcs, then its epsilon-input arcs.
void ConnectCanonical(const HostFst& in, HostFst* out) {
  const int S = in.NumStates();
  const int64_t A = in.NumArcs();
  std::vector<int64_t> rbeg(S + 1, 0);
  for (int64_t e = 0; e < A; e++) rbeg[in.nextstate[e] + 1]++;
  for (int s = 0; s < S; s++) rbeg[s + 1] += rbeg[s];
  std::vector<int> rsrc(A);
  {
    std::vector<int64_t> fill(rbeg.begin(), rbeg.end() - 1);
    for (int s = 0; s < S; s++)
      for (int64_t e = in.row[s]; e < in.row[s + 1]; e++) rsrc[fill[in.nextstate[e]]++] = s;
  }
  std::vector<char> coacc(S, 0);
  std::vector<int> q;
  for (int s = 0; s < S; s++)
    if (std::isfinite(in.final_cost[s])) { coacc[s] = 1; q.push_back(s); }
  for (size_t i = 0; i < q.size(); i++)
    for (int64_t k = rbeg[q[i]]; k < rbeg[q[i] + 1]; k++)
      if (!coacc[rsrc[k]]) { coacc[rsrc[k]] = 1; q.push_back(rsrc[k]); }
  if (in.start < 0 || !coacc[in.start]) VAMD_ERR("the composed decoding graph is empty (no path reaches a final state)");
  std::vector<int> nid(S, -1);
  std::vector<int> order;
  order.push_back(in.start);
  nid[in.start] = 0;
  *out = HostFst();
  out->osyms = in.osyms;
  out->start = 0;
  out->row.push_back(0);
  for (size_t i = 0; i < order.size(); i++) {
    const int s = order[i];
    out->final_cost.push_back(in.final_cost[s]);
    for (int pass = 0; pass < 2; pass++) {
      for (int64_t e = in.row[s]; e < in.row[s + 1]; e++) {
        if ((in.ilabel[e] == 0) != (pass == 1)) continue;
        const int d = in.nextstate[e];
        if (!coacc[d]) continue;
        if (nid[d] < 0) { nid[d] = (int)order.size(); order.push_back(d); }
        out->ilabel.push_back(in.ilabel[e]);
        out->olabel.push_back(in.olabel[e]);
        out->weight.push_back(in.weight[e]);
        out->nextstate.push_back(nid[d]);
      }
    }
    out->row.push_back((int64_t)out->ilabel.size());
  }
  // OpenFST's lazy numbering needs each state's destinations in the
  // composition's own arc order (emitting and epsilon arcs interleaved) and
  // the states the trim dropped: those take ids past the graph's (a source's
  // expansion numbers them too; the decoder never reaches them)
  const int NS = (int)order.size();
  std::vector<int> dead(S, -1);
  int ndead = 0;
  out->lazy_row.assign(1, 0);
  for (int i = 0; i < NS; i++) {
    const int s = order[i];
    for (int64_t e = in.row[s]; e < in.row[s + 1]; e++) {
      const int d = in.nextstate[e];
      int id = nid[d];
      if (id < 0) {
        if (dead[d] < 0) dead[d] = NS + ndead++;
        id = dead[d];
      }
      out->lazy_next.push_back(id);
    }
    out->lazy_row.push_back((int64_t)out->lazy_next.size());
  }
  out->lazy_ids = NS + ndead;
}

}  // namespace

namespace {
// OpenFST's FastLogAccumulator<StdArc> (arc_limit 20, arc_period 10), the
// accumulator of the LabelReachable behind the olabel_lookahead matcher
// [O: fst/accumulator.h]: log-semiring sums in double, rounded to float per
// step; states with at least 20 arcs keep a cumulative sum every 10 arcs.
constexpr double kDInf = std::numeric_limits<double>::infinity();
constexpr float kFInf = std::numeric_limits<float>::infinity();
constexpr int kAccLimit = 20, kAccPeriod = 10;
double LogPosExp(double x) { return x == kDInf ? 0.0 : std::log(1.0F + std::exp(-x)); }
double LogMinusExp(double x) { return x == kDInf ? 0.0 : std::log(1.0F - std::exp(-x)); }
float LogPlusW(float w, float v) {  // Weight LogPlus(Weight, Weight)
  if (w == kFInf && v == kFInf) return kFInf;
  const double f1 = w, f2 = v;
  return f1 > f2 ? (float)(f2 - LogPosExp(f1 - f2)) : (float)(f1 - LogPosExp(f2 - f1));
}
double LogPlusD(double f1, float v) {  // double LogPlus(double, Weight) (Init)
  const double f2 = v;
  if (f1 == kDInf) return f2;
  return f1 > f2 ? f2 - LogPosExp(f1 - f2) : f1 - LogPosExp(f2 - f1);
}
float LogMinusW(double f1, double f2) {  // f1 < f2
  if (f2 == kDInf) return (float)f1;
  return (float)(f1 - LogMinusExp(f2 - f1));
}
// FastLogAccumulator::Sum(w, aiter, begin, end) over arc weights wt[] of a
// state whose stored cumulative sums are sw (nullptr: fewer than 20 arcs)
float AccSum(float sum, const float* wt, const double* sw, int64_t begin, int64_t end) {
  int64_t ib = -1, ie = -1, sb = end, se = end;
  if (sw) {
    ib = begin > 0 ? (begin - 1) / kAccPeriod + 1 : 0;
    ie = end / kAccPeriod;
    sb = ib * kAccPeriod;
    se = ie * kAccPeriod;
  }
  if (begin < sb)
    for (int64_t p = begin, pe = std::min(sb, end); p < pe; p++) sum = LogPlusW(sum, wt[p]);
  if (sb < se) {
    const double f1 = sw[ie], f2 = sw[ib];
    if (f1 < f2) sum = LogPlusW(sum, LogMinusW(f1, f2));
  }
  if (se < end)
    for (int64_t p = std::max(sb, se); p < end; p++) sum = LogPlusW(sum, wt[p]);
  return sum;
}
// TropicalWeight::Quantize(kDelta): the lookahead weight a filter state keeps
float Quantize(float v) {
  if (!std::isfinite(v)) return v;
  const float delta = 1.0F / 1024.0F;
  return std::floor(v / delta + 0.5F) * delta;
}
bool Member(const Intervals& iv, int l) {
  auto it = std::upper_bound(iv.begin(), iv.end(), std::make_pair(l, std::numeric_limits<int>::max()));
  return it != iv.begin() && std::prev(it)->second >= l;
}
}  // namespace

// The composition the reference builds, ComposeFst(HCLr, G) with HCLr an
// olabel_lookahead FST, uses OpenFST's default lookahead filter chain for
// MATCH_OUTPUT [O: fst/lookahead-filter.h, compose.h CreateBase]:
//   PushLabelsComposeFilter<PushWeightsComposeFilter<LookAheadComposeFilter<
//     AltSequenceComposeFilter>>>
// with the olabel_lookahead flags (output lookahead, weight, prefix,
// epsilons, non-epsilon prefix).  A composed state is (HCLr state, G state,
// alternative-sequence bit, quantized lookahead weight, pushed label):
//  * G epsilon arcs (bit 0 only): weight g - fw, the lookahead weight reset;
//  * HCLr output-epsilon arcs into p at G state q: LabelLookAheadMatcher::
//    LookAheadFst over q's arcs whose labels p reaches (and q's final weight
//    when p reaches a final state): none -> no arc; exactly one arc and no
//    final -> that G arc is taken now (label pushing: its word is output on
//    this arc, the G state advances, its weight is added, the state keeps
//    the label HCLr still has to output); otherwise the arc weight becomes
//    a + (lw - fw) with lw the log-sum of those arcs' weights (min'd with the
//    final weight), and the state keeps Quantize(lw) (weight pushing);
//  * HCLr word arcs matched with G arcs: a + (g - fw), lookahead weight reset;
//  * with a pushed label L: only HCLr output-epsilon arcs whose destination
//    reaches L (the state kept), or HCLr arcs outputting L, which become
//    output-epsilon arcs back to the start filter state; never final;
//  * final weight (f_HCLr - fw) + f_G.
// Float operations follow the filters' Times / Divide order.
void ComposeLookahead(const HostFst& a, const HostFst& b, const std::vector<int>& disambig,
                      HostFst* out) {
  if (a.NumStates() == 0 || b.NumStates() == 0) VAMD_ERR("cannot compose an empty FST");
  if ((uint64_t)a.NumStates() >= (1ull << 31) || (uint64_t)b.NumStates() >= (1ull << 31))
    VAMD_ERR("graph too large to compose");
  int max_il = 0;
  for (int l : a.ilabel) max_il = std::max(max_il, l);
  std::vector<char> is_disambig(max_il + 1, 0);
  for (int d : disambig)
    if (d > 0 && d <= max_il) is_disambig[d] = 1;
  auto t0 = std::chrono::steady_clock::now();
  Reach reach;
  ComputeReach(a, &reach);
  auto t1 = std::chrono::steady_clock::now();
  // grammar side: per state the epsilon arcs in order and the non-epsilon
  // arcs sorted by input label (stable) -- the ilabel-sorted arc order the
  // matcher and the accumulator see
  const int SB = b.NumStates();
  std::vector<int64_t> bsorted(b.NumArcs());
  std::vector<int64_t> beps_end(SB);  // arcs [row[s], beps_end[s]) of bsorted are epsilon
  std::vector<int> bword(b.NumArcs());
  std::vector<float> bw(b.NumArcs());
  std::vector<char> b_has_eps(SB), b_alleps(SB);
  std::vector<int64_t> acc_pos(SB, -1);
  std::vector<double> acc_w;
  for (int s = 0; s < SB; s++) {
    int64_t o = b.row[s];
    for (int64_t e = b.row[s]; e < b.row[s + 1]; e++)
      if (b.ilabel[e] == 0) bsorted[o++] = e;
    beps_end[s] = o;
    for (int64_t e = b.row[s]; e < b.row[s + 1]; e++)
      if (b.ilabel[e] != 0) bsorted[o++] = e;
    std::stable_sort(bsorted.begin() + beps_end[s], bsorted.begin() + b.row[s + 1],
                     [&](int64_t x, int64_t y) { return b.ilabel[x] < b.ilabel[y]; });
    for (int64_t k = b.row[s]; k < b.row[s + 1]; k++) {
      bword[k] = b.ilabel[bsorted[k]];
      bw[k] = b.weight[bsorted[k]];
    }
    b_has_eps[s] = beps_end[s] > b.row[s];
    b_alleps[s] = beps_end[s] == b.row[s + 1] && !std::isfinite(b.final_cost[s]);
    if (b.row[s + 1] - b.row[s] >= kAccLimit) {  // FastLogAccumulator::Init
      acc_pos[s] = (int64_t)acc_w.size();
      double sum = kDInf;
      acc_w.push_back(sum);
      int64_t n = 0;
      for (int64_t k = b.row[s]; k < b.row[s + 1]; k++) {
        sum = LogPlusD(sum, bw[k]);
        if (++n % kAccPeriod == 0) acc_w.push_back(sum);
      }
    }
  }
  // LabelLookAheadMatcher::LookAheadFst for HCLr state p (component c) at G
  // state q: ok (some label or the final reachable), the prefix arc (index
  // into bsorted, -1 none) and the lookahead weight
  struct LookAhead {
    bool ok;
    int64_t prefix;
    float lw;
  };
  // LookAheadFst depends only on (reachability component, G state): memoized
  struct LaHash {
    size_t operator()(uint64_t k) const { return (size_t)StateTable::Mix(k); }
  };
  std::unordered_map<uint64_t, LookAhead, LaHash> la_memo;
  auto lookahead_uncached = [&](int c, int q) {
    const Intervals& iv = reach.labels[c];
    const bool rfin = reach.final[c] && std::isfinite(b.final_cost[q]);
    const int64_t r0 = b.row[q], n = b.row[q + 1] - r0;
    const int* lab = bword.data() + r0;
    const float* wt = bw.data() + r0;
    // LabelReachable::Reach: per arc when the arcs are fewer than half the
    // intervals (the final label counts as one), else per interval
    const int64_t nint = (int64_t)iv.size() + (reach.final[c] ? 1 : 0);
    int64_t rb = -1, re = -1;
    float w = kFInf;
    if (2 * n < nint) {
      int last = -1;
      for (int64_t k = 0; k < n; k++) {
        if (lab[k] == last || Member(iv, lab[k])) {
          last = lab[k];
          if (rb < 0) rb = k;
          re = k + 1;
          w = LogPlusW(w, wt[k]);
        }
      }
    } else {
      const double* sw = acc_pos[q] >= 0 ? acc_w.data() + acc_pos[q] : nullptr;
      int64_t lo = 0;
      for (const auto& r : iv) {
        const int64_t bl = std::lower_bound(lab + lo, lab + n, r.first) - lab;
        const long long hi1 = (long long)r.second + 1;
        const int64_t el = std::lower_bound(lab + bl, lab + n, hi1, [](int x, long long v) { return x < v; }) - lab;
        lo = el;
        if (el > bl) {
          if (rb < 0) rb = bl;
          re = el;
          w = AccSum(w, wt, sw, bl, el);
        }
      }
    }
    LookAhead la{false, -1, 0.0f};
    const bool rarc = rb >= 0;
    bool cw = true;
    if (rarc) {
      if (re - rb == 1 && !rfin) {
        la.prefix = r0 + rb;
        cw = false;
      } else {
        la.lw = w;
      }
    }
    if (rfin && cw) la.lw = rarc ? std::min(la.lw, b.final_cost[q]) : b.final_cost[q];
    la.ok = rarc || rfin;
    return la;
  };
  auto lookahead = [&](int c, int q) {
    const uint64_t k = ((uint64_t)(uint32_t)reach.cls[c] << 32) | (uint32_t)q;
    auto it = la_memo.find(k);
    if (it != la_memo.end()) return it->second;
    const LookAhead la = lookahead_uncached(c, q);
    la_memo.emplace(k, la);
    return la;
  };

  // Wide HCL states (the word-start states: one output-epsilon arc per first
  // phone) are checked per grammar word instead of per arc: the label line is
  // cut into segments, each listing the arcs whose reachable labels cover it,
  // and each word of the grammar state marks the arcs of its segment (the
  // arcs LookAheadFst can accept; only those are looked ahead).
  struct ArcIndex {
    std::vector<int> seg_lo;      // segment starts (ascending); segment k = [seg_lo[k], seg_lo[k+1])
    std::vector<int> seg_begin;   // [nseg + 1] into arcs
    std::vector<int> arcs;        // local arc indices covering each segment
    std::vector<int> final_arcs;  // arcs that reach a final state
    std::vector<std::pair<int, int>> labelled;  // (output label, arc) of the word arcs, sorted
    // per G state: the arcs that can produce composed arcs there (the
    // output-epsilon arcs LookAheadFst can accept, the word arcs the G state
    // matches), in arc order
    std::unordered_map<int, std::vector<int>> cand;
  };
  constexpr int kWide = 16;
  std::vector<ArcIndex*> arc_index(a.NumStates(), nullptr);
  // states whose output-epsilon arcs reach the same components in the same
  // order (the word-boundary states) share one index
  std::map<std::vector<int>, std::unique_ptr<ArcIndex>> index_by_sig;
  auto index_of = [&](int q1) -> const ArcIndex* {
    const int64_t b0 = a.row[q1], n = a.row[q1 + 1] - b0;
    if (n < kWide) return nullptr;
    if (arc_index[q1]) return arc_index[q1];
    std::vector<int> sig(n);
    for (int64_t e = b0; e < b0 + n; e++)
      sig[e - b0] = a.olabel[e] != 0 ? -1 - a.olabel[e] : reach.cls[reach.comp[a.nextstate[e]]];
    auto found = index_by_sig.find(sig);
    if (found != index_by_sig.end()) return arc_index[q1] = found->second.get();
    auto ix = std::make_unique<ArcIndex>();
    std::vector<std::pair<long long, int>> ev;  // (position, +arc+1 / -(arc+1))
    for (int64_t e = b0; e < b0 + n; e++) {
      if (a.olabel[e] != 0) {
        ix->labelled.push_back({a.olabel[e], (int)(e - b0)});
        continue;
      }
      const int c = reach.comp[a.nextstate[e]];
      if (reach.final[c]) ix->final_arcs.push_back((int)(e - b0));
      for (const auto& r : reach.labels[c]) {
        ev.push_back({r.first, (int)(e - b0) + 1});
        ev.push_back({(long long)r.second + 1, -((int)(e - b0) + 1)});
      }
    }
    std::sort(ev.begin(), ev.end());
    std::vector<int> active;
    size_t i = 0;
    while (i < ev.size()) {
      const long long x = ev[i].first;
      for (; i < ev.size() && ev[i].first == x; i++) {
        const int v = ev[i].second;
        if (v > 0) active.push_back(v - 1);
        else active.erase(std::find(active.begin(), active.end(), -v - 1));
      }
      ix->seg_lo.push_back((int)std::min<long long>(x, std::numeric_limits<int>::max()));
      ix->seg_begin.push_back((int)ix->arcs.size());
      std::vector<int> sorted_active(active);
      std::sort(sorted_active.begin(), sorted_active.end());
      ix->arcs.insert(ix->arcs.end(), sorted_active.begin(), sorted_active.end());
    }
    ix->seg_begin.push_back((int)ix->arcs.size());
    std::sort(ix->labelled.begin(), ix->labelled.end());
    arc_index[q1] = ix.get();
    index_by_sig.emplace(std::move(sig), std::move(ix));
    return arc_index[q1];
  };
  std::vector<char> mark;

  // composed states: key = (q1 << 32 | q2 | bit << 31, fw bits << 32 | pushed label)
  struct Key {
    uint64_t k0, k1;
  };
  std::vector<Key> keys;
  struct KeyHash {
    size_t operator()(const std::pair<uint64_t, uint64_t>& k) const {
      return (size_t)StateTable::Mix(k.first ^ StateTable::Mix(k.second));
    }
  };
  std::unordered_map<std::pair<uint64_t, uint64_t>, int, KeyHash> table;
  table.reserve(1 << 20);
  constexpr int kNoLabel = -1;
  auto id_of = [&](int q1, int q2, int sb, float fw, int fl) {
    uint32_t fwb;
    std::memcpy(&fwb, &fw, 4);
    const Key k{((uint64_t)q1 << 32) | (uint32_t)q2 | ((uint64_t)sb << 31), ((uint64_t)fwb << 32) | (uint32_t)fl};
    auto it = table.emplace(std::make_pair(k.k0, k.k1), (int)keys.size());
    if (it.second) {
      if (keys.size() >= (size_t)std::numeric_limits<int>::max() - 1) VAMD_ERR("composed graph too large");
      keys.push_back(k);
    }
    return it.first->second;
  };
  HostFst c;
  c.osyms = b.osyms;
  c.start = id_of(a.start, b.start, 0, 0.0f, kNoLabel);
  c.row.push_back(0);
  for (size_t s = 0; s < keys.size(); s++) {
    const int q1 = (int)(keys[s].k0 >> 32), q2 = (int)(keys[s].k0 & 0x7fffffffu);
    const int sb = (int)((keys[s].k0 >> 31) & 1);
    const uint32_t fwb = (uint32_t)(keys[s].k1 >> 32);
    const int fl = (int)(uint32_t)(keys[s].k1 & 0xffffffffu);
    float fw;
    std::memcpy(&fw, &fwb, 4);
    const float fa = a.final_cost[q1], fb = b.final_cost[q2];
    c.final_cost.push_back(fl == kNoLabel && std::isfinite(fa) && std::isfinite(fb) ? (fa - fw) + fb : kFInf);
    auto push = [&](int il, int ol, float w, int dst) {
      c.ilabel.push_back(il); c.olabel.push_back(ol); c.weight.push_back(w); c.nextstate.push_back(dst);
    };
    auto in_label = [&](int64_t e) {
      return (a.ilabel[e] > 0 && a.ilabel[e] <= max_il && is_disambig[a.ilabel[e]]) ? 0 : a.ilabel[e];
    };
    if (fl != kNoLabel) {  // PushedLabelFilterArc: HCLr must still output fl
      for (int64_t e = a.row[q1]; e < a.row[q1 + 1]; e++) {
        const int p = a.nextstate[e];
        if (a.olabel[e] == fl) {
          push(in_label(e), 0, a.weight[e] + 0.0f, id_of(p, q2, 0, 0.0f, kNoLabel));
        } else if (a.olabel[e] == 0 && Member(reach.labels[reach.comp[p]], fl)) {
          push(in_label(e), 0, a.weight[e] + 0.0f, id_of(p, q2, sb, fw, fl));
        }
      }
      c.row.push_back((int64_t)c.ilabel.size());
      continue;
    }
    const float nfw = 0.0f - fw;  // Divide(One, fw)
    if (sb == 0)  // the grammar moves alone on its epsilon (backoff) arcs
      for (int64_t k = b.row[q2]; k < beps_end[q2]; k++) {
        const int64_t e = bsorted[k];
        push(0, b.olabel[e], 0.0f + (bw[k] + nfw), id_of(q1, b.nextstate[e], 0, 0.0f, kNoLabel));
      }
    ArcIndex* ix = b_alleps[q2] ? nullptr : const_cast<ArcIndex*>(index_of(q1));
    const std::vector<int>* cand = nullptr;
    if (ix) {
      auto ci = ix->cand.find(q2);
      if (ci == ix->cand.end()) {
        // mark the output-epsilon arcs the lookahead can accept, and the
        // word arcs G matches (intersecting the smaller list into the larger)
        const int n = (int)(a.row[q1 + 1] - a.row[q1]);
        mark.assign(n, 0);
        if (std::isfinite(b.final_cost[q2]))
          for (int k : ix->final_arcs) mark[k] = 1;
        for (int64_t k = beps_end[q2]; k < b.row[q2 + 1]; k++) {
          const int w = bword[k];
          auto it = std::upper_bound(ix->seg_lo.begin(), ix->seg_lo.end(), w);
          if (it == ix->seg_lo.begin()) continue;
          const size_t sg = (size_t)(it - ix->seg_lo.begin()) - 1;
          for (int j = ix->seg_begin[sg]; j < ix->seg_begin[sg + 1]; j++) mark[ix->arcs[j]] = 1;
        }
        const int* wb = bword.data() + beps_end[q2];
        const int* we = bword.data() + b.row[q2 + 1];
        if ((size_t)(we - wb) < ix->labelled.size()) {
          for (const int* w = wb; w < we; w++) {
            auto it = std::lower_bound(ix->labelled.begin(), ix->labelled.end(), std::make_pair(*w, -1));
            for (; it != ix->labelled.end() && it->first == *w; ++it) mark[it->second] = 1;
          }
        } else {
          for (const auto& lw : ix->labelled)
            if (std::binary_search(wb, we, lw.first)) mark[lw.second] = 1;
        }
        std::vector<int> v;
        for (int k = 0; k < n; k++)
          if (mark[k]) v.push_back(k);
        ci = ix->cand.emplace(q2, std::move(v)).first;
      }
      cand = &ci->second;
    }
    const int nsb = b_has_eps[q2] ? 1 : 0;
    const int64_t ncand = cand ? (int64_t)cand->size() : a.row[q1 + 1] - a.row[q1];
    for (int64_t ki = 0; ki < ncand; ki++) {
      const int64_t e = cand ? a.row[q1] + (*cand)[ki] : a.row[q1] + ki;
      const int il = in_label(e);
      const int p = a.nextstate[e];
      if (a.olabel[e] == 0) {  // HCL moves alone, looking ahead into G
        if (b_alleps[q2]) continue;
        const LookAhead la = lookahead(reach.comp[p], q2);
        if (!la.ok) continue;
        if (la.prefix >= 0) {  // label pushing: the single reachable G arc now
          const int64_t g = bsorted[la.prefix];
          push(il, b.olabel[g], a.weight[e] + ((0.0f + nfw) + bw[la.prefix]),
               id_of(p, b.nextstate[g], nsb, 0.0f, bword[la.prefix]));
        } else {  // weight pushing
          push(il, 0, a.weight[e] + (0.0f + (la.lw - fw)), id_of(p, q2, nsb, Quantize(la.lw), kNoLabel));
        }
      } else {  // matched word
        const int* wb = bword.data() + beps_end[q2];
        const int* we = bword.data() + b.row[q2 + 1];
        const int* lo = std::lower_bound(wb, we, a.olabel[e]);
        for (const int* it = lo; it != we && *it == a.olabel[e]; it++) {
          const int64_t k = it - bword.data();
          const int64_t g = bsorted[k];
          push(il, b.olabel[g], a.weight[e] + (bw[k] + nfw), id_of(p, b.nextstate[g], 0, 0.0f, kNoLabel));
        }
      }
    }
    c.row.push_back((int64_t)c.ilabel.size());
  }
  VAMD_LOG("Composed lookahead graph: " << c.NumStates() << " states, " << c.NumArcs() << " arcs expanded");
  auto t2 = std::chrono::steady_clock::now();
  if (getenv("VOSK_AMD_GRAPH_RAW")) {
    // measurement hook (tools/numbering_discovery.py): the composition as
    // OpenFST's ComposeFst holds it -- untrimmed, its own arc order, states
    // numbered in expansion order -- instead of the decoding graph
    *out = std::move(c);
    return;
  }
  ConnectCanonical(c, out);
  auto t3 = std::chrono::steady_clock::now();
  VAMD_LOG_VERBOSE("compose timing: reach " << std::chrono::duration<double>(t1 - t0).count() << " s, expand " << std::chrono::duration<double>(t2 - t1).count() << " s, connect " << std::chrono::duration<double>(t3 - t2).count() << " s");
  VAMD_LOG("Static decoding graph: " << out->NumStates() << " states, " << out->NumArcs() << " arcs");
}

void EstimateGrammarLm(const std::vector<std::vector<int>>& sentences, int order, float discount,
                       HostFst* out) {
  if (order < 2) VAMD_ERR("--ngram-order must be >= 2");
  struct LmState {
    std::vector<int> history;
    std::map<int, int> counts;
    int tot = 0, backoff = -1, fst_state = -1;
  };
  std::vector<LmState> st;
  std::map<std::vector<int>, int> index;
  int num_active = 0;
  std::function<int(const std::vector<int>&)> find_or_create = [&](const std::vector<int>& h) {
    auto it = index.find(h);
    if (it != index.end()) return it->second;
    const int ans = (int)st.size();
    st.emplace_back();
    st.back().history = h;
    index[h] = ans;
    if (!h.empty()) {
      const int b = find_or_create(std::vector<int>(h.begin() + 1, h.end()));
      st[ans].backoff = b;
    }
    return ans;
  };
  auto add_count = [](LmState& s, int w, int n) {
    s.counts[w] += n;
    s.tot += n;
  };
  auto increment = [&](const std::vector<int>& h, int w) {
    const int l = find_or_create(h);
    if (st[l].tot == 0) num_active++;
    add_count(st[l], w, 1);
  };
  for (const auto& sent : sentences) {  // AddCounts
    std::vector<int> h;
    for (int w : sent) {
      if (w == 0) VAMD_ERR("word id 0 in a grammar sentence");
      increment(h, w);
      h.push_back(w);
      if ((int)h.size() >= order) h.erase(h.begin());
    }
    increment(h, 0);
  }
  if (st.empty()) VAMD_ERR("empty grammar");
  const int nst = (int)st.size();
  for (int l = 0; l < nst; l++)  // SetParentCounts
    for (int p = st[l].backoff; p != -1; p = st[p].backoff) {
      const std::map<int, int> counts = st[l].counts;
      for (const auto& [w, n] : counts) add_count(st[p], w, n);
    }
  int nfst = 0;  // AssignFstStates
  for (int l = 0; l < nst; l++)
    if (st[l].tot != 0) st[l].fst_state = nfst++;
  if (nfst != num_active) VAMD_ERR("grammar LM estimation: inconsistent state counts");
  auto find_nonzero = [&](std::vector<int> h) {
    while (true) {
      auto it = index.find(h);
      if (it == index.end() || st[it->second].tot == 0) {
        if (h.empty()) VAMD_ERR("grammar LM: no state for a history");
        h.erase(h.begin());
      } else {
        return it->second;
      }
    }
  };
  std::vector<std::vector<std::pair<int, std::pair<float, int>>>> arcs(nfst);  // (label, (cost, dst))
  *out = HostFst();
  out->final_cost.assign(nfst, std::numeric_limits<float>::infinity());
  out->start = st[find_nonzero({})].fst_state;
  for (int l = 0; l < nst; l++) {
    const LmState& s = st[l];
    if (s.fst_state < 0) continue;
    for (const auto& [w, n] : s.counts) {
      const float p = (float)n * discount / (float)s.tot;
      const float logprob = std::log(p);
      if (w == 0) {
        out->final_cost[s.fst_state] = -logprob;
      } else {
        std::vector<int> next = s.history;
        next.push_back(w);
        const int d = st[find_nonzero(next)].fst_state;
        arcs[s.fst_state].push_back({w, {-logprob, d}});
      }
    }
    if (s.backoff >= 0)
      arcs[s.fst_state].push_back({0, {-std::log(1.0f - discount), st[s.backoff].fst_state}});
  }
  out->row.push_back(0);
  for (int s = 0; s < nfst; s++) {
    std::sort(arcs[s].begin(), arcs[s].end(),
              [](const auto& x, const auto& y) { return x.first < y.first; });
    for (const auto& a : arcs[s]) {
      out->ilabel.push_back(a.first);
      out->olabel.push_back(a.first);
      out->weight.push_back(a.second.first);
      out->nextstate.push_back(a.second.second);
    }
    out->row.push_back((int64_t)out->ilabel.size());
  }
}

namespace {
// json.h parse_string / json_escape (src/json.h:34-48,519-555): a grammar
// phrase is the parsed string re-escaped, as JSON::ToString returns it.
std::string JsonEscape(const std::string& s) {
  std::string o;
  for (char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\b': o += "\\b"; break;
      case '\f': o += "\\f"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      default: o += c;
    }
  }
  return o;
}
}  // namespace

std::vector<std::vector<int>> ParseGrammarJson(const std::string& js, const SymbolTable& words) {
  size_t p = 0;
  auto ws = [&]() { while (p < js.size() && (js[p] == ' ' || js[p] == '\t' || js[p] == '\n' || js[p] == '\r')) p++; };
  ws();
  if (p >= js.size() || js[p] != '[') VAMD_ERR("Expecting array of strings, got: '" << js << "'");
  p++;
  std::vector<std::string> phrases;
  ws();
  if (p < js.size() && js[p] == ']') {
    p++;
  } else {
    while (true) {
      ws();
      if (p >= js.size() || js[p] != '"') VAMD_ERR("Expecting array of strings, got: '" << js << "'");
      std::string val;
      for (p++; p < js.size() && js[p] != '"'; p++) {
        if (js[p] != '\\') { val += js[p]; continue; }
        if (++p >= js.size()) break;
        switch (js[p]) {
          case '"': val += '"'; break;
          case '\\': val += '\\'; break;
          case '/': val += '/'; break;
          case 'b': val += '\b'; break;
          case 'f': val += '\f'; break;
          case 'n': val += '\n'; break;
          case 'r': val += '\r'; break;
          case 't': val += '\t'; break;
          case 'u':
            val += "\\u";
            for (int i = 1; i <= 4; i++) {
              const char c = p + i < js.size() ? js[p + i] : 0;
              if (!isxdigit((unsigned char)c)) VAMD_ERR("bad unicode escape in grammar");
              val += c;
            }
            p += 4;
            break;
          default: val += '\\';
        }
      }
      if (p >= js.size()) VAMD_ERR("unterminated string in grammar");
      p++;
      phrases.push_back(JsonEscape(val));
      ws();
      if (p < js.size() && js[p] == ',') { p++; continue; }
      if (p < js.size() && js[p] == ']') { p++; break; }
      VAMD_ERR("Expecting array of strings, got: '" << js << "'");
    }
  }
  if (phrases.empty()) VAMD_ERR("Expecting array of strings, got: '" << js << "'");
  std::vector<std::vector<int>> out;
  for (const auto& line : phrases) {
    std::vector<int> sent;
    std::string tok;
    std::istringstream ss(line);
    while (std::getline(ss, tok, ' ')) {
      const int id = words.Find(tok);
      if (id < 0) {
        VAMD_WARN("Ignoring word missing in vocabulary: '" << tok << "'");
      } else {
        sent.push_back(id);
      }
    }
    out.push_back(std::move(sent));
  }
  return out;
}

}  // namespace vamd
