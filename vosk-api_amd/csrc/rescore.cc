// LM rescoring of a segment's word lattice (rescore.h).
#include "rescore.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <iterator>
#include <limits>
#include <map>
#include <unordered_map>

#include "common.h"

namespace vamd {
namespace {
constexpr float kInf = std::numeric_limits<float>::infinity();

struct BinReader {
  std::string d, what;
  size_t p = 0;
  void Need(size_t n) const {
    if (p + n > d.size()) VAMD_ERR("unexpected end of " << what);
  }
  std::string Token() {
    while (p < d.size() && d[p] == ' ') p++;
    size_t b = p;
    while (p < d.size() && d[p] != ' ') p++;
    std::string t = d.substr(b, p - b);
    if (p < d.size()) p++;
    return t;
  }
  void Expect(const char* t) {
    std::string g = Token();
    if (g != t) VAMD_ERR("expected " << t << " in " << what << ", got " << g);
  }
  int64_t Int() {
    Need(1);
    const int n = (unsigned char)d[p++];
    Need(n);
    int64_t v = 0;
    if (n == 4) {
      int32_t x;
      memcpy(&x, d.data() + p, 4);
      v = x;
    } else if (n == 8) {
      memcpy(&v, d.data() + p, 8);
    } else {
      VAMD_ERR("bad integer size " << n << " in " << what);
    }
    p += n;
    return v;
  }
};

inline float AsFloat(int32_t i) {
  float f;
  memcpy(&f, &i, 4);
  return f;
}
}  // namespace

void ConstArpaLm::Read(const std::string& path) {
  BinReader r;
  r.what = path;
  {
    std::ifstream in(path, std::ios::binary);
    if (!in) VAMD_ERR("cannot open " << path);
    r.d.assign((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  }
  if (r.d.size() < 2 || r.d[0] != '\0' || r.d[1] != 'B') VAMD_ERR(path << ": only binary ConstArpaLm is supported");
  r.p = 2;
  r.Expect("<ConstArpaLm>");
  r.Expect("<LmInfo>");
  bos = (int)r.Int();
  eos = (int)r.Int();
  unk = (int)r.Int();
  order = (int)r.Int();
  r.Expect("</LmInfo>");
  r.Expect("<LmStates>");
  const int64_t n = r.Int();
  if (n < 0 || n > (int64_t)1 << 36) VAMD_ERR("bad LmStates size in " << path);
  r.Need((size_t)n * 4);
  states_.resize(n);
  memcpy(states_.data(), r.d.data() + r.p, (size_t)n * 4);
  r.p += (size_t)n * 4;
  r.Expect("</LmStates>");
  r.Expect("<LmUnigram>");
  const int64_t nw = r.Int();
  if (nw < 0 || nw > (int64_t)1 << 31) VAMD_ERR("bad LmUnigram size in " << path);
  unigram_.resize(nw);
  // Kaldi's ConstArpaLm::Write stores -1 for a word without a unigram state
  // (<eps>, disambiguation symbols); offset 0 is an ordinary state
  for (auto& u : unigram_) {
    u = r.Int();
    if (u == -1) continue;
    if (u < 0 || u + 3 > n) VAMD_ERR("bad unigram offset in " << path);
  }
  r.Expect("</LmUnigram>");
  r.Expect("<LmOverflow>");
  const int64_t no = r.Int();
  if (no < 0 || no > n) VAMD_ERR("bad LmOverflow size in " << path);
  overflow_.resize(no);
  for (auto& o : overflow_) {
    o = r.Int();
    if (o == -1) continue;
    if (o < 0 || o + 3 > n) VAMD_ERR("bad overflow offset in " << path);
  }
  r.Expect("</LmOverflow>");
  r.Expect("</ConstArpaLm>");
  if (order < 1 || bos < 0 || eos < 0) VAMD_ERR("bad ConstArpaLm header in " << path);
}

const int32_t* ConstArpaLm::UnigramState(int w) const {
  if (w < 0 || w >= (int)unigram_.size() || unigram_[w] < 0) return nullptr;
  return states_.data() + unigram_[w];
}

bool ConstArpaLm::ChildInfo(int word, const int32_t* parent, int32_t* info) const {
  const int32_t n = parent[2];
  int lo = 1, hi = n;
  while (lo <= hi) {
    const int mid = (lo + hi) / 2;
    const int32_t w = parent[1 + 2 * mid];
    if (w == word) {
      *info = parent[2 + 2 * mid];
      return true;
    }
    if (w < word) lo = mid + 1;
    else hi = mid - 1;
  }
  return false;
}

void ConstArpaLm::Decode(int32_t info, const int32_t* parent, const int32_t** child,
                         float* logprob) const {
  if (info % 2 == 0) {  // a leaf: the n-gram's logprob
    *child = nullptr;
    *logprob = AsFloat(info);
    return;
  }
  const int32_t off = info / 2;
  if (off > 0) {
    *child = parent + off;
  } else {
    if (-off >= (int32_t)overflow_.size() || overflow_[-off] < 0)
      VAMD_ERR("ConstArpaLm overflow index out of range");
    *child = states_.data() + overflow_[-off];
  }
  *logprob = AsFloat(**child);
}

const int32_t* ConstArpaLm::State(const std::vector<int>& seq) const {
  if (seq.empty()) return nullptr;
  const int32_t* s = UnigramState(seq[0]);
  for (size_t i = 1; s && i < seq.size(); i++) {
    int32_t info;
    if (!ChildInfo(seq[i], s, &info)) return nullptr;
    const int32_t* c = nullptr;
    float lp;
    Decode(info, s, &c, &lp);
    s = c;
  }
  return s;
}

bool ConstArpaLm::HistoryStateExists(const std::vector<int>& hist) const {
  return !hist.empty() && State(hist) != nullptr;
}

float ConstArpaLm::Recurse(int word, const std::vector<int>& hist) const {
  if (hist.empty()) {
    const int32_t* s = UnigramState(word);
    return s ? AsFloat(s[0]) : -kInf;
  }
  float backoff = 0.0f;
  if (const int32_t* s = State(hist)) {
    int32_t info;
    if (ChildInfo(word, s, &info)) {
      const int32_t* c = nullptr;
      float lp;
      Decode(info, s, &c, &lp);
      return lp;
    }
    backoff = AsFloat(s[1]);
  }
  return backoff + Recurse(word, std::vector<int>(hist.begin() + 1, hist.end()));
}

float ConstArpaLm::NgramLogprob(int word, std::vector<int> hist) const {
  while ((int)hist.size() >= order) hist.erase(hist.begin());
  if (unk != -1) {
    if (!UnigramState(word)) word = unk;
    for (int& h : hist)
      if (!UnigramState(h)) h = unk;
  }
  return Recurse(word, hist);
}

void RescoreLm::Load(const std::string& g_fst, const std::string& g_carpa) {
  ReadFst(g_fst, &g);
  // ReadAndPrepareLmFst: project on the output labels (the backoff arcs'
  // #0 becomes epsilon), sort each state's arcs by label
  for (size_t a = 0; a < g.ilabel.size(); a++) g.ilabel[a] = g.olabel[a];
  for (int s = 0; s < g.NumStates(); s++) {
    const int64_t b = g.row[s], e = g.row[s + 1];
    std::vector<int64_t> idx(e - b);
    for (int64_t i = 0; i < e - b; i++) idx[i] = b + i;
    std::stable_sort(idx.begin(), idx.end(), [&](int64_t x, int64_t y) { return g.ilabel[x] < g.ilabel[y]; });
    std::vector<int> il(e - b), ol(e - b), nx(e - b);
    std::vector<float> w(e - b);
    for (int64_t i = 0; i < e - b; i++) {
      il[i] = g.ilabel[idx[i]]; ol[i] = g.olabel[idx[i]]; nx[i] = g.nextstate[idx[i]]; w[i] = g.weight[idx[i]];
    }
    for (int64_t i = 0; i < e - b; i++) {
      g.ilabel[b + i] = il[i]; g.olabel[b + i] = ol[i]; g.nextstate[b + i] = nx[i]; g.weight[b + i] = w[i];
    }
  }
  carpa.Read(g_carpa);
}

namespace {
// topological order of an acyclic word lattice (Kahn, smallest id first)
bool TopoOrder(const WordLattice& w, std::vector<int>* order) {
  const int S = w.NumStates();
  std::vector<int> indeg(S, 0);
  for (int s = 0; s < S; s++)
    for (auto& a : w.arcs[s]) indeg[a.next]++;
  std::vector<int> st;
  for (int s = S - 1; s >= 0; s--)
    if (indeg[s] == 0) st.push_back(s);
  order->clear();
  while (!st.empty()) {
    const int s = st.back();
    st.pop_back();
    order->push_back(s);
    for (auto& a : w.arcs[s])
      if (--indeg[a.next] == 0) st.push_back(a.next);
  }
  return (int)order->size() == S;
}

// Keep the states on a path from 0 to a final state, renumbered in a
// topological order (the composed lattices here are built in one).
void TrimWordLattice(WordLattice* w) {
  const int S = w->NumStates();
  std::vector<std::vector<int>> rev(S);
  for (int s = 0; s < S; s++)
    for (auto& a : w->arcs[s]) rev[a.next].push_back(s);
  std::vector<char> co(S, 0);
  std::vector<int> q;
  for (int s = 0; s < S; s++)
    if (w->final_graph[s] != kInf) { co[s] = 1; q.push_back(s); }
  for (size_t i = 0; i < q.size(); i++)
    for (int p : rev[q[i]])
      if (!co[p]) { co[p] = 1; q.push_back(p); }
  std::vector<int> nid(S, -1);
  int n = 0;
  for (int s = 0; s < S; s++)
    if (co[s]) nid[s] = n++;
  WordLattice o;
  o.arcs.resize(n);
  o.final_graph.resize(n);
  o.final_acoustic.resize(n);
  o.final_tids.resize(n);
  for (int s = 0; s < S; s++) {
    if (!co[s]) continue;
    const int t = nid[s];
    for (auto& a : w->arcs[s])
      if (co[a.next]) {
        auto b = a;
        b.next = nid[a.next];
        o.arcs[t].push_back(std::move(b));
      }
    o.final_graph[t] = w->final_graph[s];
    o.final_acoustic[t] = w->final_acoustic[s];
    o.final_tids[t] = w->final_tids[s];
  }
  *w = std::move(o);
}
}  // namespace

bool RescoreLattice(const WordLattice& in, const RescoreLm& lm, const LatticeOptions& opt,
                    WordLattice* out) {
  const HostFst& G = lm.g;
  if (in.NumStates() == 0 || G.NumStates() == 0) return false;
  // ---- 1. old LM subtraction: (-graph) o G with the sequence filter
  struct CArc { int word, next; float graph, acoustic; const std::vector<int>* tids; };
  std::vector<std::vector<CArc>> carcs;
  std::vector<float> cfg, cfa;
  std::vector<const std::vector<int>*> cft;
  std::map<std::tuple<int, int, int>, int> ids;
  std::vector<std::tuple<int, int, int>> keys;
  static const std::vector<int> kNoTids;
  auto id_of = [&](int q, int gq, int fs) {
    auto k = std::make_tuple(q, gq, fs);
    auto it = ids.find(k);
    if (it != ids.end()) return it->second;
    const int id = (int)keys.size();
    ids[k] = id;
    keys.push_back(k);
    if ((int)keys.size() > opt.max_states) VAMD_ERR("rescoring composition guard");
    return id;
  };
  id_of(0, G.start, 0);
  for (size_t s = 0; s < keys.size(); s++) {
    const auto [q, gq, fs] = keys[s];
    std::vector<CArc> arcs;
    bool has_eps = false, all_eps = true;
    for (auto& a : in.arcs[q]) {
      if (a.word == 0) has_eps = true;
      else all_eps = false;
    }
    const bool lat_final = in.final_graph[q] != kInf;
    if (!(all_eps && !lat_final))  // G moves alone on its epsilon arcs
      for (int64_t e = G.row[gq]; e < G.row[gq + 1]; e++)
        if (G.ilabel[e] == 0)
          arcs.push_back({0, id_of(q, G.nextstate[e], has_eps ? 1 : 0), G.weight[e], 0.0f, &kNoTids});
    for (auto& a : in.arcs[q]) {
      if (a.word == 0) {  // the lattice moves alone
        if (fs != 0) continue;
        arcs.push_back({0, id_of(a.next, gq, 0), -a.graph, a.acoustic, &a.tids});
        continue;
      }
      for (int64_t e = G.row[gq]; e < G.row[gq + 1]; e++) {
        if (G.ilabel[e] < a.word) continue;
        if (G.ilabel[e] > a.word) break;
        arcs.push_back({a.word, id_of(a.next, G.nextstate[e], 0), -a.graph + G.weight[e], a.acoustic, &a.tids});
      }
    }
    if (carcs.size() <= s) carcs.resize(s + 1);
    carcs[s] = std::move(arcs);
    const float gf = G.final_cost[gq];
    if (lat_final && gf != kInf) {
      cfg.push_back(-in.final_graph[q] + gf);
      cfa.push_back(in.final_acoustic[q]);
      cft.push_back(&in.final_tids[q]);
    } else {
      cfg.push_back(kInf);
      cfa.push_back(0.0f);
      cft.push_back(&kNoTids);
    }
  }
  const int C = (int)keys.size();
  carcs.resize(C);
  // times of the composed states (acyclic: G's backoff arcs go to lower orders)
  std::vector<int> time(C, -1), indeg(C, 0);
  for (int s = 0; s < C; s++)
    for (auto& a : carcs[s]) indeg[a.next]++;
  std::vector<int> order, st{0};
  time[0] = 0;
  while (!st.empty()) {
    const int s = st.back();
    st.pop_back();
    order.push_back(s);
    for (auto& a : carcs[s]) {
      const int t = time[s] + (int)a.tids->size();
      if (time[a.next] >= 0 && time[a.next] != t) {
        VAMD_WARN("rescoring: lattice states without consistent times; not rescored");
        return false;
      }
      time[a.next] = t;
      if (--indeg[a.next] == 0) st.push_back(a.next);
    }
  }
  if ((int)order.size() != C) {
    VAMD_WARN("rescoring: cyclic composition; not rescored");
    return false;
  }
  int F = -1;
  for (int s = 0; s < C; s++)
    if (cfg[s] != kInf) {
      const int t = time[s] + (int)cft[s]->size();
      if (F >= 0 && t != F) {
        VAMD_WARN("rescoring: final states at different times; not rescored");
        return false;
      }
      F = t;
    }
  if (F < 0) return false;
  // ---- state-level form for the word determinizer: one token per composed
  // state, chains for multi-transition-id strings, one super-final token
  struct PLink { int src, dst, il, ol; float g, a; };
  std::vector<int> tok_time(C);
  for (int s = 0; s < C; s++) tok_time[s] = time[s];
  std::vector<PLink> pl;
  auto chain = [&](int src, int dst, int word, float g, float a, const std::vector<int>& tids) {
    if (tids.size() <= 1) {
      pl.push_back({src, dst, tids.empty() ? 0 : tids[0], word, g, a});
      return;
    }
    int cur = src;
    for (size_t i = 0; i < tids.size(); i++) {
      int nxt = dst;
      if (i + 1 < tids.size()) {
        nxt = (int)tok_time.size();
        tok_time.push_back(tok_time[src] + (int)i + 1);
      }
      pl.push_back({cur, nxt, tids[i], i == 0 ? word : 0, i == 0 ? g : 0.0f, i == 0 ? a : 0.0f});
      cur = nxt;
    }
  };
  const int superfinal = C;
  tok_time.push_back(F);
  for (int s = 0; s < C; s++) {
    for (auto& a : carcs[s]) chain(s, a.next, a.word, a.graph, a.acoustic, *a.tids);
    if (cfg[s] != kInf) chain(s, superfinal, 0, cfg[s], cfa[s], *cft[s]);
  }
  const int T = (int)tok_time.size();
  std::vector<int> perm(T);
  for (int i = 0; i < T; i++) perm[i] = i;
  std::stable_sort(perm.begin(), perm.end(), [&](int x, int y) { return tok_time[x] < tok_time[y]; });
  std::vector<int> pos(T);
  for (int i = 0; i < T; i++) pos[perm[i]] = i;
  RawLattice raw;
  raw.num_frames = F;
  raw.frame_begin.assign(F + 2, 0);
  for (int i = 0; i < T; i++) raw.frame_begin[tok_time[i] + 1]++;
  for (int f = 0; f <= F; f++) raw.frame_begin[f + 1] += raw.frame_begin[f];
  raw.tok_state.assign(T, 0);
  raw.tok_cost.assign(T, 1.0f);
  raw.tok_cost[pos[0]] = 0.0f;
  Graph fake;
  fake.ilabel.resize(pl.size());
  fake.olabel.resize(pl.size());
  fake.weight.resize(pl.size());
  for (size_t i = 0; i < pl.size(); i++) {
    fake.ilabel[i] = pl[i].il;
    fake.olabel[i] = pl[i].ol;
    fake.weight[i] = pl[i].g;
    raw.links.push_back({pos[pl[i].src], pos[pl[i].dst], (int)i, pl[i].g, pl[i].a});
  }
  raw.final_cost.assign(raw.frame_begin[F + 1] - raw.frame_begin[F], kInf);
  raw.final_cost[pos[superfinal] - raw.frame_begin[F]] = 0.0f;
  WordLattice det;
  if (!DeterminizeToWords(raw, fake, opt, &det) || det.NumStates() == 0) {
    VAMD_WARN("rescoring: determinization failed; not rescored");
    return false;
  }
  ScaleGraph(&det, -1.0f);
  // ---- 2. ConstArpa LM: deterministic composition (ConstArpaLmDeterministicFst)
  const ConstArpaLm& lmc = lm.carpa;
  std::vector<int> topo;
  if (!TopoOrder(det, &topo)) return false;
  std::vector<int> topo_idx(det.NumStates());
  for (size_t i = 0; i < topo.size(); i++) topo_idx[topo[i]] = (int)i;
  std::map<std::vector<int>, int> hist_id;
  std::vector<std::vector<int>> hists;
  auto hid = [&](const std::vector<int>& h) {
    auto it = hist_id.find(h);
    if (it != hist_id.end()) return it->second;
    const int id = (int)hists.size();
    hist_id[h] = id;
    hists.push_back(h);
    return id;
  };
  std::map<std::pair<int, int>, int> rid;
  std::vector<std::pair<int, int>> rkeys;
  auto rid_of = [&](int q, int h) {
    auto k = std::make_pair(q, h);
    auto it = rid.find(k);
    if (it != rid.end()) return it->second;
    const int id = (int)rkeys.size();
    rid[k] = id;
    rkeys.push_back(k);
    if ((int)rkeys.size() > opt.max_states) VAMD_ERR("rescoring composition guard");
    return id;
  };
  rid_of(0, hid({lmc.bos}));
  WordLattice r;
  for (size_t s = 0; s < rkeys.size(); s++) {
    const auto [q, h] = rkeys[s];
    std::vector<WordLattice::Arc> arcs;
    for (auto& a : det.arcs[q]) {
      if (a.word == 0) {
        arcs.push_back({0, rid_of(a.next, h), a.graph, a.acoustic, a.tids});
        continue;
      }
      const float lp = lmc.NgramLogprob(a.word, hists[h]);
      if (lp == -kInf) continue;
      std::vector<int> nh = hists[h];
      nh.push_back(a.word);
      if ((int)nh.size() >= lmc.order) nh.erase(nh.begin());
      while (!lmc.HistoryStateExists(nh)) {
        if (nh.empty()) VAMD_ERR("ConstArpaLm: no history state for a word");
        nh.erase(nh.begin());
      }
      arcs.push_back({a.word, rid_of(a.next, hid(nh)), a.graph + (-lp), a.acoustic, a.tids});
    }
    r.arcs.push_back(std::move(arcs));
    float fg = kInf, fa = 0.0f;
    if (det.final_graph[q] != kInf) {
      const float lp = lmc.NgramLogprob(lmc.eos, hists[h]);
      if (lp != -kInf) {
        fg = det.final_graph[q] + (-lp);
        fa = det.final_acoustic[q];
      }
    }
    r.final_graph.push_back(fg);
    r.final_acoustic.push_back(fa);
    r.final_tids.push_back(det.final_tids[q]);
  }
  // topological renumbering (by the determinized state's order, then creation)
  const int R = (int)rkeys.size();
  std::vector<int> rorder(R);
  for (int i = 0; i < R; i++) rorder[i] = i;
  std::stable_sort(rorder.begin(), rorder.end(),
                   [&](int x, int y) { return topo_idx[rkeys[x].first] < topo_idx[rkeys[y].first]; });
  std::vector<int> rnew(R);
  for (int i = 0; i < R; i++) rnew[rorder[i]] = i;
  WordLattice o;
  o.arcs.resize(R);
  o.final_graph.resize(R);
  o.final_acoustic.resize(R);
  o.final_tids.resize(R);
  for (int s = 0; s < R; s++) {
    const int t = rnew[s];
    o.arcs[t] = std::move(r.arcs[s]);
    for (auto& a : o.arcs[t]) a.next = rnew[a.next];
    o.final_graph[t] = r.final_graph[s];
    o.final_acoustic[t] = r.final_acoustic[s];
    o.final_tids[t] = std::move(r.final_tids[s]);
  }
  TrimWordLattice(&o);
  if (o.NumStates() == 0) {
    VAMD_WARN("rescoring: empty lattice; not rescored");
    return false;
  }
  *out = std::move(o);
  return true;
}

}  // namespace vamd
