"""Canonical forms of state-level lattices for parity tests (engine vs
oracle): per frame, the set of (state, cost) tokens and the set of
(source state, arc, graph cost, acoustic cost) links."""
import numpy as np


def canon_engine(L):
    fb = L["frame_begin"]
    F = L["num_frames"]
    frame_of = np.zeros(len(L["tok_state"]), np.int64)
    for k in range(F + 1):
        frame_of[fb[k]:fb[k + 1]] = k
    toks = [sorted(zip(L["tok_state"][fb[k]:fb[k + 1]].tolist(),
                       L["tok_cost"][fb[k]:fb[k + 1]].view(np.int32).tolist())) for k in range(F + 1)]
    links = [[] for _ in range(F + 1)]
    for s, d, a, gcost, ac in zip(L["link_src"], L["link_dst"], L["link_arc"], L["link_graph"],
                                  L["link_ac"]):
        links[frame_of[d]].append((int(L["tok_state"][s]), int(a), float(gcost),
                                   int(np.float32(ac).view(np.int32))))
    return toks, [sorted(x) for x in links]


def canon_oracle(r, graph):
    L = r["lattice"]
    fb = L["frame_begin"]
    F = len(fb) - 2
    toks = [sorted(zip(L["tok_state"][fb[k]:fb[k + 1]].tolist(),
                       L["tok_cost"][fb[k]:fb[k + 1]].view(np.int32).tolist())) for k in range(F + 1)]
    links = [[] for _ in range(F + 1)]
    for k, s, a, ac in zip(L["link_frame"], L["link_src"], L["link_arc"], L["link_ac"]):
        acx = np.float32(ac) - np.float32(L["cost_offset"][k]) if graph.ilabel[a] != 0 else np.float32(0)
        links[k].append((int(s), int(a), float(graph.weight[a]), int(np.float32(acx).view(np.int32))))
    return toks, [sorted(x) for x in links]
