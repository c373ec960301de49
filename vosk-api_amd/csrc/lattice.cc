#include "lattice.h"

#include <algorithm>
#include <cmath>
#include <limits>
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
                     const std::vector<int2>& arena, const std::vector<int4>& links,
                     bool use_final, RawLattice* out) {
  RawLattice& L = *out;
  L = RawLattice();
  const int F = (int)frames.size() - 1;
  if (F < 0) return;
  L.num_frames = F;
  L.frame_begin.assign(F + 2, 0);
  std::vector<int> arena2tok(arena.size(), -1);
  std::vector<std::unordered_map<int, int>> state2tok(F + 1);
  for (int k = 0; k <= F; k++) {
    const LatFrame& fr = frames[k];
    L.frame_begin[k] = (int)L.tok_state.size();
    for (int a = fr.tok_base; a < fr.tok_base + fr.ntok; a++) {
      if (a < 0 || a >= (int)arena.size()) VAMD_ERR("lattice: arena index out of range");
      const int2 e = arena[a];
      if (e.x == -2) continue;  // dead list entry
      const int s = e.y >= 0 ? g.nextstate[e.y] : start_state;
      const int id = (int)L.tok_state.size();
      arena2tok[a] = id;
      state2tok[k][s] = id;
      L.tok_state.push_back(s);
      L.tok_cost.push_back(kInf);
    }
    L.frame_begin[k + 1] = (int)L.tok_state.size();
  }
  auto tok_of = [&](int k, int s) {
    auto it = state2tok[k].find(s);
    if (it == state2tok[k].end()) VAMD_ERR("lattice: link to a missing token (frame " << k << ", state " << s << ")");
    return it->second;
  };
  if (L.frame_begin[1] > L.frame_begin[0]) L.tok_cost[tok_of(0, start_state)] = 0.0f;
  for (int k = 0; k <= F; k++) {
    const LatFrame& fr = frames[k];
    const float cutoff = fr.cutoff;
    const long long lb = std::max<long long>(0, fr.link_begin),
                    le = std::min<long long>((long long)links.size(), fr.link_end);
    if (fr.link_end > (long long)links.size()) L.overflow = true;
    // emitting links into frame k: exact tot from the kernel
    std::vector<RawLattice::Link> emit;
    std::vector<int> eps_arcs;
    for (long long i = lb; i < le; i++) {
      const int4 r = links[i];
      const int arc = r.y;
      if (r.x >= 0) {
        const float tot = __builtin_bit_cast(float, r.w);
        if (!(tot < cutoff)) continue;
        if (r.x >= (int)arena.size() || arena2tok[r.x] < 0) VAMD_ERR("lattice: link from a missing token");
        const int src = arena2tok[r.x], dst = tok_of(k, g.nextstate[arc]);
        const float ac = __builtin_bit_cast(float, r.z);
        emit.push_back(RawLattice::Link{src, dst, arc, g.weight[arc], ac - fr.cost_offset});
        if (tot < L.tok_cost[dst]) L.tok_cost[dst] = tot;
      } else {
        eps_arcs.push_back(arc);
      }
    }
    // epsilon links: one per arc, costs relaxed to the fixpoint (the
    // decoder's final token costs), kept when below the cutoff
    std::sort(eps_arcs.begin(), eps_arcs.end());
    eps_arcs.erase(std::unique(eps_arcs.begin(), eps_arcs.end()), eps_arcs.end());
    std::vector<std::pair<int, int>> ends(eps_arcs.size());
    for (size_t i = 0; i < eps_arcs.size(); i++)
      ends[i] = {tok_of(k, ArcSource(g, eps_arcs[i])), tok_of(k, g.nextstate[eps_arcs[i]])};
    for (bool changed = true; changed;) {
      changed = false;
      for (size_t i = 0; i < eps_arcs.size(); i++) {
        const float tot = L.tok_cost[ends[i].first] + g.weight[eps_arcs[i]];
        if (tot < L.tok_cost[ends[i].second]) {
          L.tok_cost[ends[i].second] = tot;
          changed = true;
        }
      }
    }
    for (size_t i = 0; i < eps_arcs.size(); i++) {
      const float tot = L.tok_cost[ends[i].first] + g.weight[eps_arcs[i]];
      if (tot < cutoff)
        emit.push_back(RawLattice::Link{ends[i].first, ends[i].second, eps_arcs[i],
                                        g.weight[eps_arcs[i]], 0.0f});
    }
    std::sort(emit.begin(), emit.end(), [](const RawLattice::Link& a, const RawLattice::Link& b) {
      return a.src != b.src ? a.src < b.src : a.arc < b.arc;
    });
    L.links.insert(L.links.end(), emit.begin(), emit.end());
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
