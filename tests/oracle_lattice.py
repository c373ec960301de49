"""Oracle restatement of the result pipeline over a state-level lattice
(test infrastructure).

The reference builds every result from the decoder's lattice
(src/recognizer.cc:669-729 GetResult: GraphLatticeScale(0.9) then MbrResult
:429-482 / NbestResult :526-607 / NlsmlResult :609-667; the batch path
src/batch_recognizer.cc:43-107).  The algorithms are Kaldi's [K], absent from
the reference tree: lattice-beam pruning (LatticeFasterDecoder
PruneForwardLinks / PruneForwardLinksFinal), word-level lattice
determinization (DeterminizeLatticePruned: one path per word sequence, its
best alignment, residual strings, subsets equal within kDelta = 1/1024),
MinimumBayesRisk (lat/sausages.cc, Xu et al. 2011: edit-distance forward
pass, backward gamma accumulation, iterated hypothesis) and n-best shortest
paths.  Parity with Kaldi is unpinned (no Kaldi here, no reference vectors
for confidences); this restatement pins libvosk.so's C++ (csrc/lattice.cc)
to the same algorithm.  Word alignment (WordAlignLattice) is not restated:
both sides use the unaligned lattice (the reference's CopyLatticeForMbr path).
"""
import math

import numpy as np

F32 = np.float32
INF = float("inf")


def raw_from_oracle(r, graph, use_final=True):
    """Oracle decode(lattice=True) -> the arrays of vamd_stream_lattice
    (numpy form of raw_from_oracle_loop, which states it link by link; the
    same arrays, tests/test_lattice.py)."""
    L = r["lattice"]
    fb = np.asarray(L["frame_begin"], np.int64)
    F = len(fb) - 2
    ts = np.asarray(L["tok_state"], np.int64)
    NS = int(max(int(ts.max()) if len(ts) else 0, int(np.max(graph.nextstate)) if len(graph.nextstate) else 0)) + 1
    tf = np.repeat(np.arange(F + 1, dtype=np.int64), np.diff(fb[:F + 2]))
    key = tf * NS + ts
    order = np.argsort(key, kind="stable")
    skey = key[order]
    lk = np.asarray(L["link_frame"], np.int64)
    la = np.asarray(L["link_arc"], np.int64)
    ls = np.asarray(L["link_src"], np.int64)
    lx = np.asarray(L["link_ac"], np.float32)
    il = np.asarray(graph.ilabel)[la]
    emit = il != 0
    sk = (lk - emit.astype(np.int64)) * NS + ls
    dk = lk * NS + np.asarray(graph.nextstate, np.int64)[la]
    sid = order[np.searchsorted(skey, sk)]
    did = order[np.searchsorted(skey, dk)]
    assert np.array_equal(skey[np.searchsorted(skey, sk)], sk) and np.array_equal(skey[np.searchsorted(skey, dk)], dk)
    co = np.asarray(L["cost_offset"], np.float32)[lk]
    acx = np.where(emit, (lx - co).astype(np.float32), np.float32(0)).astype(np.float32)
    srt = np.lexsort((la, sid, lk))  # per frame, by (source, arc); stable
    last = ts[fb[F]:fb[F + 1]]
    fin = graph.final[last].astype(np.float32)
    final = fin if (use_final and np.isfinite(fin).any()) else np.zeros(0, np.float32)
    return dict(num_frames=F, frame_begin=np.asarray(fb, np.int32),
                tok_state=np.asarray(L["tok_state"], np.int32), tok_cost=np.asarray(L["tok_cost"], np.float32),
                link_src=sid[srt].astype(np.int32), link_dst=did[srt].astype(np.int32),
                link_arc=la[srt].astype(np.int32),
                link_graph=np.asarray(graph.weight, np.float32)[la][srt], link_ac=acx[srt], final_cost=final)


# ---------------------------------------------------------------- pruning
def prune(L, beam):
    """Lattice-beam pruning (numpy form of prune_loop: per frame, the
    cross-frame links' relaxations, then the within-frame (epsilon) links
    relaxed to their fixpoint -- min-plus shortest paths, whose float values
    do not depend on the relaxation order -- backwards the same; the same
    arrays, tests/test_lattice.py)."""
    F = L["num_frames"]
    fb = np.asarray(L["frame_begin"], np.int64)
    N = len(L["tok_state"])
    frame = np.repeat(np.arange(F + 1, dtype=np.int64), np.diff(fb[:F + 2]))
    src = np.asarray(L["link_src"], np.int64)
    dst = np.asarray(L["link_dst"], np.int64)
    g32 = np.asarray(L["link_graph"], np.float32)
    x32 = np.asarray(L["link_ac"], np.float32)
    cost = (g32 + x32).astype(np.float32).astype(np.float64)
    lf = frame[dst] if len(dst) else np.zeros(0, np.int64)
    within = frame[src] == lf if len(dst) else np.zeros(0, bool)
    byf = np.argsort(lf, kind="stable")
    lb = np.searchsorted(lf[byf], np.arange(F + 2))
    alpha = np.full(N, INF)
    beta = np.full(N, INF)
    tc = np.asarray(L["tok_cost"], np.float32)
    z = np.nonzero(tc[fb[0]:fb[1]] == 0.0)[0]
    if len(z):
        alpha[fb[0] + z[0]] = 0.0
    for k in range(F + 1):
        idx = byf[lb[k]:lb[k + 1]]
        cr, wi = idx[~within[idx]], idx[within[idx]]
        if len(cr):
            np.minimum.at(alpha, dst[cr], alpha[src[cr]] + cost[cr])
        while len(wi):
            cand = alpha[src[wi]] + cost[wi]
            if not (cand < alpha[dst[wi]]).any():
                break
            np.minimum.at(alpha, dst[wi], cand)
    fin = L["final_cost"]
    fc = np.zeros(fb[F + 1] - fb[F]) if len(fin) == 0 else np.asarray(fin, np.float32).astype(np.float64)
    beta[fb[F]:fb[F + 1]] = fc
    best = float(np.min(alpha[fb[F]:fb[F + 1]] + fc)) if fb[F + 1] > fb[F] else INF
    for k in range(F, -1, -1):
        idx = byf[lb[k]:lb[k + 1]]
        cr, wi = idx[~within[idx]], idx[within[idx]]
        while len(wi):
            cand = cost[wi] + beta[dst[wi]]
            if not (cand < beta[src[wi]]).any():
                break
            np.minimum.at(beta, src[wi], cand)
        if len(cr):
            np.minimum.at(beta, src[cr], cost[cr] + beta[dst[cr]])
    keep = alpha + beta - best <= beam
    remap = np.full(N, -1, np.int64)
    remap[keep] = np.arange(int(keep.sum()))
    nfb = np.zeros(F + 2, np.int64)
    ck = np.concatenate([[0], np.cumsum(keep)])
    nfb[:F + 2] = ck[fb[:F + 2]]
    lk = (remap[src] >= 0) & (remap[dst] >= 0) & (alpha[src] + cost + beta[dst] - best <= beam)
    nfin = np.asarray(fin, np.float32)[keep[fb[F]:fb[F + 1]]] if len(fin) else np.zeros(0, np.float32)
    return dict(num_frames=F, frame_begin=nfb.astype(np.int32),
                tok_state=np.asarray(L["tok_state"], np.int32)[keep], tok_cost=tc[keep],
                link_src=remap[src[lk]].astype(np.int32), link_dst=remap[dst[lk]].astype(np.int32),
                link_arc=np.asarray(L["link_arc"], np.int32)[lk], link_graph=g32[lk], link_ac=x32[lk],
                final_cost=nfin.astype(np.float32))


def raw_from_oracle_loop(r, graph, use_final=True):
    """Oracle decode(lattice=True) -> the arrays of vamd_stream_lattice."""
    L = r["lattice"]
    fb = L["frame_begin"]
    F = len(fb) - 2
    ids = {}
    for k in range(F + 1):
        for t in range(fb[k], fb[k + 1]):
            ids[(k, int(L["tok_state"][t]))] = t
    src, dst, arc, gc, ac = [], [], [], [], []
    per_frame = [[] for _ in range(F + 1)]
    for k, s, a, x in zip(L["link_frame"], L["link_src"], L["link_arc"], L["link_ac"]):
        emit = graph.ilabel[a] != 0
        sid = ids[(int(k) - 1 if emit else int(k), int(s))]
        did = ids[(int(k), int(graph.nextstate[a]))]
        acx = F32(F32(x) - F32(L["cost_offset"][k])) if emit else F32(0)
        per_frame[int(k)].append((sid, int(a), did, F32(graph.weight[a]), acx))
    for k in range(F + 1):
        for sid, a, did, g, x in sorted(per_frame[k], key=lambda z: (z[0], z[1])):
            src.append(sid)
            dst.append(did)
            arc.append(a)
            gc.append(g)
            ac.append(x)
    last = L["tok_state"][fb[F]:fb[F + 1]]
    fin = graph.final[last].astype(np.float32)
    final = fin if (use_final and np.isfinite(fin).any()) else np.zeros(0, np.float32)
    return dict(num_frames=F, frame_begin=np.asarray(fb, np.int32),
                tok_state=np.asarray(L["tok_state"], np.int32), tok_cost=np.asarray(L["tok_cost"], np.float32),
                link_src=np.asarray(src, np.int32), link_dst=np.asarray(dst, np.int32),
                link_arc=np.asarray(arc, np.int32), link_graph=np.asarray(gc, np.float32),
                link_ac=np.asarray(ac, np.float32), final_cost=final)


# ---------------------------------------------------------------- pruning
def prune_loop(L, beam):
    F = L["num_frames"]
    fb = L["frame_begin"]
    N = len(L["tok_state"])
    frame = np.zeros(N, np.int64)
    for k in range(F + 1):
        frame[fb[k]:fb[k + 1]] = k
    links = list(zip(L["link_src"].tolist(), L["link_dst"].tolist(), L["link_arc"].tolist(),
                     L["link_graph"], L["link_ac"]))
    by_frame = [[] for _ in range(F + 1)]
    for i, l in enumerate(links):
        by_frame[frame[l[1]]].append(i)
    cost = [float(F32(l[3]) + F32(l[4])) for l in links]
    alpha = [INF] * N
    beta = [INF] * N
    for t in range(fb[0], fb[1]):
        if L["tok_cost"][t] == 0.0:
            alpha[t] = 0.0
            break
    for k in range(F + 1):
        for i in by_frame[k]:
            s, d = links[i][0], links[i][1]
            if frame[s] != k:
                alpha[d] = min(alpha[d], alpha[s] + cost[i])
        ch = True
        while ch:
            ch = False
            for i in by_frame[k]:
                s, d = links[i][0], links[i][1]
                if frame[s] == k and alpha[s] + cost[i] < alpha[d]:
                    alpha[d] = alpha[s] + cost[i]
                    ch = True
    best = INF
    fin = L["final_cost"]
    for t in range(fb[F], fb[F + 1]):
        fc = 0.0 if len(fin) == 0 else float(fin[t - fb[F]])
        beta[t] = fc
        best = min(best, alpha[t] + fc)
    for k in range(F, -1, -1):
        ch = True
        while ch:
            ch = False
            for i in by_frame[k]:
                s, d = links[i][0], links[i][1]
                if frame[s] == k and cost[i] + beta[d] < beta[s]:
                    beta[s] = cost[i] + beta[d]
                    ch = True
        for i in by_frame[k]:
            s, d = links[i][0], links[i][1]
            if frame[s] != k:
                beta[s] = min(beta[s], cost[i] + beta[d])
    remap = [-1] * N
    out_state, out_cost, nfb = [], [], [0] * (F + 2)
    for k in range(F + 1):
        nfb[k] = len(out_state)
        for t in range(fb[k], fb[k + 1]):
            if not (alpha[t] + beta[t] - best <= beam):
                continue
            remap[t] = len(out_state)
            out_state.append(int(L["tok_state"][t]))
            out_cost.append(L["tok_cost"][t])
        nfb[k + 1] = len(out_state)
    ls, ld, la, lg, lx = [], [], [], [], []
    for i, (s, d, a, g, x) in enumerate(links):
        if remap[s] < 0 or remap[d] < 0:
            continue
        if not (alpha[s] + cost[i] + beta[d] - best <= beam):
            continue
        ls.append(remap[s]); ld.append(remap[d]); la.append(a); lg.append(g); lx.append(x)
    nfin = [fin[t - fb[F]] for t in range(fb[F], fb[F + 1]) if remap[t] >= 0] if len(fin) else []
    return dict(num_frames=F, frame_begin=np.asarray(nfb, np.int32), tok_state=np.asarray(out_state, np.int32),
                tok_cost=np.asarray(out_cost, np.float32), link_src=np.asarray(ls, np.int32),
                link_dst=np.asarray(ld, np.int32), link_arc=np.asarray(la, np.int32),
                link_graph=np.asarray(lg, np.float32), link_ac=np.asarray(lx, np.float32),
                final_cost=np.asarray(nfin, np.float32))


# ---------------------------------------------------------- determinization
def _cmp(x, y):  # Kaldi LatticeWeight Compare: 1 if x is better
    fx, fy = F32(x[0] + x[1]), F32(y[0] + y[1])
    if fx < fy:
        return 1
    if fx > fy:
        return -1
    if x[0] < y[0]:
        return 1
    if x[0] > y[0]:
        return -1
    if x[1] < y[1]:
        return 1
    if x[1] > y[1]:
        return -1
    return 0


def _better(e, f):  # (weight, string) order
    c = _cmp(e[1], f[1])
    if c != 0:
        return c > 0
    if len(e[2]) != len(f[2]):
        return len(e[2]) < len(f[2])
    return e[2] < f[2]


def _graph_from_raw(L, ilabel, olabel):
    """The determinizer's input from a raw lattice: (n, links [(src, dst, tid,
    label, g, a)], finals [(g, a) | None], start)."""
    N = len(L["tok_state"])
    F = L["num_frames"]
    fb = L["frame_begin"]
    links = [(s, d, int(ilabel[a]), int(olabel[a]), g, x) for s, d, a, g, x in
             zip(L["link_src"].tolist(), L["link_dst"].tolist(), L["link_arc"].tolist(),
                 L["link_graph"], L["link_ac"])]
    fin = [None] * N
    for t in range(fb[F], fb[F + 1]):
        c = F32(0) if len(L["final_cost"]) == 0 else L["final_cost"][t - fb[F]]
        fin[t] = None if c == INF else (c, F32(0))
    start = next((t for t in range(fb[0], fb[1]) if L["tok_cost"][t] == 0.0), -1) if N else -1
    return N, links, fin, start


def determinize(L, ilabel, olabel):
    """-> (arcs per state [(word, next, g, a, tids)], finals [(g, a, tids) | None]),
    states topologically sorted as the C++ does (word level only)."""
    return _determinize(*_graph_from_raw(L, ilabel, olabel))


def determinize_phone(L, ilabel, olabel, tid2phone, tid_first, beam=6.0, max_mem=50000000):
    """Kaldi DeterminizeLatticePhonePrunedWrapper (the reference's GetLattice,
    src/recognizer.cc:678): DeterminizeLatticeInsertPhones (phone label
    first_phone_label + phone at a phone's first transition-id -- HMM state 0,
    not a self-loop -- on the link when it has no word, else on a new link
    after it), determinization on phones + words, the result written out as a
    lattice (LatticeDeterminizerPruned::Output: a chain per arc string, label
    and weight on the first link; a final string as a chain to a new final
    state), DeterminizeLatticeDeletePhones, then word-level determinization."""
    n, links, fin, start = _graph_from_raw(L, ilabel, olabel)
    return determinize_phone_graph(n, links, fin, start, tid2phone, tid_first, beam, max_mem)


def determinize_phone_graph(n, links, fin, start, tid2phone, tid_first, beam=6.0, max_mem=50000000):
    """determinize_phone on a determinizer input (n, links [(src, dst, tid,
    label, g, a)], finals, start) built by the caller (csrc/lattice.cc
    DeterminizePhonePrunedGraph; labels above the words -- the incremental
    determinizer's state and token labels -- are words to it)."""
    links, fin = list(links), list(fin)
    first = max([1] + [l[3] + 1 for l in links])
    out = []
    for (s, d, t, w, g, a) in links:
        if s == start or t <= 0 or t >= len(tid_first) or not tid_first[t]:  # (no phone on the start's arcs)
            out.append((s, d, t, w, g, a))
            continue
        ph = first + int(tid2phone[t])
        if w == 0:
            out.append((s, d, t, ph, g, a))
        else:
            x = n
            n += 1
            fin.append(None)
            out.append((s, x, t, w, g, a))
            out.append((x, d, 0, ph, F32(0), F32(0)))
    r = determinize_pruned(n, out, fin, start, beam, max_mem)
    if r is None:
        return None
    W, Fi = r
    if not W:
        return W, Fi
    S = len(W)
    lab = lambda w: 0 if w >= first else w
    n2, links2, fin2 = S, [], [None] * S
    for s in range(S):
        for (w, d, g, a, tids) in W[s]:
            if not tids:
                links2.append((s, d, 0, lab(w), g, a))
                continue
            cur = s
            for i, t in enumerate(tids):
                if i + 1 == len(tids):
                    nx = d
                else:
                    nx = n2
                    n2 += 1
                    fin2.append(None)
                links2.append((cur, nx, int(t), lab(w) if i == 0 else 0, g if i == 0 else F32(0),
                               a if i == 0 else F32(0)))
                cur = nx
        f = Fi[s]
        if f is None:
            continue
        if not f[2]:
            fin2[s] = (f[0], f[1])
            continue
        cur = s
        for i, t in enumerate(f[2]):
            nx = n2
            n2 += 1
            fin2.append(None)
            links2.append((cur, nx, int(t), 0, f[0] if i == 0 else F32(0), f[1] if i == 0 else F32(0)))
            cur = nx
        fin2[cur] = (F32(0), F32(0))
    return determinize_pruned(n2, links2, fin2, 0, beam, max_mem)


# ------------------------------------------------- pruned determinization
# Kaldi lat/determinize-lattice-pruned.{h,cc} [K]: LatticeDeterminizerPruned
# (the determinization of the reference's GetLattice, src/recognizer.cc:678,
# through DeterminizeLatticePhonePrunedWrapper, and of the batch pipeline's
# lattice callback, src/batch_recognizer.cc:138-149) and the retry loop of
# DeterminizeLatticePruned.  Restated as csrc/lattice.cc PrunedDeterminizer:
# element strings are absolute transition-id tuples, a subset's base the
# common prefix its residuals hang off; the string repository's size is the
# number of distinct strings ever created (csrc StrRepo nodes).

def _cmp_k(x, y):  # fst::Compare(LatticeWeight): total cost, then graph cost
    fx, fy = F32(x[0] + x[1]), F32(y[0] + y[1])
    if fx < fy:
        return 1
    if fx > fy:
        return -1
    if x[0] < y[0]:
        return 1
    if x[0] > y[0]:
        return -1
    return 0


def _cmp_det(e, eb, f, fb):
    """The determinizer's Compare on (weight, residual string): 1 if e is
    better; weight, then the shorter string, then the lexicographically larger."""
    c = _cmp_k(e[1], f[1])
    if c:
        return c
    x, y = e[2][len(eb):], f[2][len(fb):]
    if len(x) != len(y):
        return 1 if len(x) < len(y) else -1
    if x == y:
        return 0
    return 1 if x > y else -1


def _approx_eq(x, y, delta):  # LatticeWeight ApproxEqual
    if x[0] == y[0] and x[1] == y[1]:
        return True
    return abs(F32(F32(x[0] + x[1]) - F32(y[0] + y[1]))) <= F32(delta)


def _cost(w):  # ConvertToCost: in double
    return float(w[0]) + float(w[1])


def _topo(N, links):
    indeg = [0] * N
    out = [[] for _ in range(N)]
    for (s, d, *_r) in links:
        indeg[d] += 1
        out[s].append(d)
    order, st = [], [s for s in range(N - 1, -1, -1) if indeg[s] == 0]
    while st:
        s = st.pop()
        order.append(s)
        for d in reversed(out[s]):
            indeg[d] -= 1
            if indeg[d] == 0:
                st.append(d)
    assert len(order) == N, "lattice has a cycle"
    return order


def _prune_det_input(N, links, fin, start, topo, beam):
    """kaldi::PruneLattice on the determinizer's input."""
    out = [[] for _ in range(N)]
    for i, l in enumerate(links):
        out[l[0]].append(i)
    fw = [INF] * N
    fw[start] = 0.0
    best = INF
    for s in topo:
        for i in out[s]:
            d, g, a = links[i][1], links[i][4], links[i][5]
            fw[d] = min(fw[d], fw[s] + _cost((g, a)))
        if fin[s] is not None:
            best = min(best, fw[s] + _cost(fin[s]))
    cut = best + beam
    keep = [True] * len(links)
    fin2 = list(fin)
    bw = [INF] * N
    for s in reversed(topo):
        b = INF if fin[s] is None else _cost(fin[s])
        if b != INF and b + fw[s] > cut:
            fin2[s] = None
        for i in out[s]:
            d, g, a = links[i][1], links[i][4], links[i][5]
            ab = _cost((g, a)) + bw[d]
            if ab < b:
                b = ab
            if fw[s] + ab > cut:
                keep[i] = False
        bw[s] = b
    return [l for l, k in zip(links, keep) if k], fin2


class _PrunedDet:
    def __init__(self, N, links, fin, start, topo, beam, max_mem, max_states=100000, delta=1.0 / 1024.0):
        self.N, self.links, self.fin, self.start = N, links, fin, start
        self.beam, self.max_mem, self.max_states, self.delta = beam, max_mem, max_states, delta
        self.outl = [[] for _ in range(N)]
        for i, l in enumerate(links):
            self.outl[l[0]].append(i)
        # per state: label-epsilon links first, then label links (graph order within each)
        self.outl = [[i for i in v if links[i][3] == 0] + [i for i in v if links[i][3] != 0] for v in self.outl]
        self.has_label = [any(links[i][3] != 0 for i in v) for v in self.outl]
        self.bwd = [INF] * N
        for s in reversed(topo):
            c = INF if fin[s] is None else _cost(fin[s])
            for i in self.outl[s]:
                l = links[i]
                c = min(c, _cost((l[4], l[5])) + self.bwd[l[1]])
            self.bwd[s] = c
        self.cutoff = self.bwd[start] + beam
        self.states = []     # dict(sub, base, fwd, arcs)
        self.minimal = {}
        self.initial = {}
        self.queue = []
        self.seq = 0
        self.num_elems = 0
        self.num_arcs = 0
        self.nodes = set()   # distinct non-empty strings created (the repository)
        self.eff = beam
        self.guard = False

    def _ext(self, s, t):
        if t == 0:
            return s
        n = s + (t,)
        self.nodes.add(n)
        self._revive(n)
        return n

    def _revive(self, n):
        # after a rebuild, a string Kaldi's RebuildRepository deleted and that
        # is referenced again is re-added: counted as added since the rebuild
        rb = getattr(self, "rb_nodes", None)
        if rb is not None and n in rb and n not in self.rb_live:
            self.rb_live.add(n)
            self.revived += 1

    @staticmethod
    def _times(w, g, a):
        return (F32(w[0] + F32(g)), F32(w[1] + F32(a)))

    def closure(self, sub, base):
        at = {e[0]: i for i, e in enumerate(sub)}
        work = list(range(len(sub)))
        while work:
            i = work.pop()
            e = sub[i]
            for li in self.outl[e[0]]:
                s, d, t, w, g, x = self.links[li]
                if w != 0:
                    break
                n = (d, self._times(e[1], g, x), self._ext(e[2], t))
                if d not in at:
                    at[d] = len(sub)
                    work.append(len(sub))
                    sub.append(n)
                elif _cmp_det(n, base, sub[at[d]], base) > 0:
                    sub[at[d]] = n
                    work.append(at[d])
        return sub

    def minimal_form(self, sub):
        sub = [e for e in sub if self.fin[e[0]] is not None or self.has_label[e[0]]]
        sub.sort(key=lambda e: e[0])
        return sub

    def normalize(self, sub, base):
        tot = sub[0][1]
        n = len(sub[0][2])
        for e in sub[1:]:
            if _cmp_k(tot, e[1]) < 0:
                tot = e[1]
        for e in sub:
            j = 0
            while j < n and j < len(e[2]) and e[2][j] == sub[0][2][j]:
                j += 1
            n = j
        nbase = sub[0][2][:n]
        out = [(e[0], (F32(e[1][0] - tot[0]), F32(e[1][1] - tot[1])), e[2]) for e in sub]
        return out, nbase, tot

    def _key(self, sub, base):
        return tuple((e[0], e[2][len(base):]) for e in sub)

    def _eq(self, x, bx, y, by):
        return len(x) == len(y) and all(
            a[0] == b[0] and _approx_eq(a[1], b[1], self.delta) and a[2][len(bx):] == b[2][len(by):]
            for a, b in zip(x, y))

    def process_final(self, sid):
        st = self.states[sid]
        best = None
        for e in st["sub"]:
            if self.fin[e[0]] is None:
                continue
            c = (e[0], self._times(e[1], *self.fin[e[0]]), e[2])
            if best is None or _cmp_det(c, st["base"], best, st["base"]) > 0:
                best = c
        if best is not None and _cost(best[1]) + st["fwd"] <= self.cutoff:
            st["arcs"].append((0, -1, best[1], best[2]))
            self.num_arcs += 1

    def process_transitions(self, sid):
        import heapq
        import functools
        st = self.states[sid]
        base = st["base"]
        allp = []
        for e in st["sub"]:
            for li in self.outl[e[0]]:
                s, d, t, w, g, x = self.links[li]
                if w == 0:
                    continue
                allp.append((w, (d, self._times(e[1], g, x), self._ext(e[2], t))))

        def order(p, q):
            if p[0] != q[0]:
                return -1 if p[0] < q[0] else 1
            if p[1][0] != q[1][0]:
                return -1 if p[1][0] < q[1][0] else 1
            return -_cmp_det(p[1], base, q[1], base)
        allp.sort(key=functools.cmp_to_key(order))
        i = 0
        while i < len(allp):
            label = allp[i][0]
            prio = INF
            sub = []
            while i < len(allp) and allp[i][0] == label:
                e = allp[i][1]
                prio = min(prio, _cost(e[1]) + self.bwd[e[0]])
                if not sub or sub[-1][0] != e[0]:
                    sub.append(e)
                i += 1
            prio += st["fwd"]
            if prio > self.cutoff:
                continue
            self.num_elems += len(sub)
            heapq.heappush(self.queue, (prio, self.seq, sid, label, sub, base))
            self.seq += 1

    def minimal_to_state(self, sub, base, fwd):
        key = self._key(sub, base)
        for sid in self.minimal.get(key, []):
            o = self.states[sid]
            if self._eq(o["sub"], o["base"], sub, base):
                return sid
        sid = len(self.states)
        self.num_elems += len(sub)
        self.states.append(dict(sub=sub, base=base, fwd=fwd, arcs=[]))
        self.minimal.setdefault(key, []).append(sid)
        self.process_final(sid)
        self.process_transitions(sid)
        return sid

    def initial_to_state(self, sub, base, fwd):
        key = self._key(sub, base)
        for (csub, cbase, sid, rem, rstr, rbase) in self.initial.get(key, []):
            if self._eq(csub, cbase, sub, base):
                return sid, rem, rstr[len(rbase):]
        cur = self.minimal_form(self.closure(list(sub), base))
        if not cur:
            return -1, None, None
        cur, nbase, w2 = self.normalize(cur, base)
        sid = self.minimal_to_state(cur, nbase, fwd + _cost(w2))
        self.num_elems += len(sub)
        self.initial.setdefault(key, []).append((sub, base, sid, w2, nbase, base))
        return sid, w2, nbase[len(base):]

    def check_memory(self):
        # (the repository as Kaldi's RebuildRepository leaves it: the strings
        # live at the last rebuild plus those added since)
        arcs, elems = self.num_arcs * 32, self.num_elems * 24
        n = len(self.nodes) + 1
        rebuilt = getattr(self, "rebuilt", None)
        repo = (n if rebuilt is None else rebuilt[0] + self.revived + n - rebuilt[1]) * 32
        if self.max_mem <= 0 or repo + arcs + elems <= self.max_mem:
            return True
        live = set()

        def mark(s):
            for k in range(1, len(s) + 1):
                live.add(s[:k])
        for st in self.states:
            for e in st["sub"]:
                mark(e[2])
            mark(st["base"])
            for a in st["arcs"]:
                mark(a[3])
        for v in self.initial.values():
            for (csub, cbase, sid, rem, rstr, rbase) in v:
                for e in csub:
                    mark(e[2])
                mark(rstr)
        for t in self.queue:
            for e in t[4]:
                mark(e[2])
        self.rebuilt = (len(live), n)
        self.rb_nodes, self.rb_live, self.revived = set(self.nodes), live, 0
        repo = len(live) * 32
        if repo + arcs + elems > int(self.max_mem * 0.8):
            if self.queue:
                self.eff = min(self.queue)[0] - self.bwd[self.start]
            return False
        return True

    def run(self):
        import heapq
        s0 = self.minimal_form(self.closure([(self.start, (F32(0), F32(0)), ())], ()))
        self.num_elems += len(s0)
        self.states.append(dict(sub=s0, base=(), fwd=0.0, arcs=[]))
        self.minimal.setdefault(self._key(s0, ()), []).append(0)
        self.process_final(0)
        self.process_transitions(0)
        done = True
        while self.queue:
            ns = len(self.states)
            if self.max_states > 0 and ns > self.max_states:
                self.guard = True
                return False
            if ns % 10 == 0 and not self.check_memory():
                done = False
                break
            prio, _, sid, label, sub, sbase = heapq.heappop(self.queue)
            fwd = self.states[sid]["fwd"]
            sub, b1, w1 = self.normalize(sub, sbase)
            fwd += _cost(w1)
            nxt, w2, rest = self.initial_to_state(sub, b1, fwd)
            if nxt < 0:
                continue
            full = b1 + tuple(rest)
            for k in range(len(b1) + 1, len(full) + 1):
                self.nodes.add(full[:k])
                self._revive(full[:k])
            self.states[sid]["arcs"].append((label, nxt, (F32(w1[0] + w2[0]), F32(w1[1] + w2[1])), full))
            self.num_arcs += 1
        return done

    def output(self):
        """Creation order, trimmed to start -> final paths (fst::Connect), then
        the topological renumbering of csrc/lattice.cc."""
        S = len(self.states)
        acc, coacc = [False] * S, [False] * S
        acc[0] = True
        st = [0]
        while st:
            s = st.pop()
            for a in self.states[s]["arcs"]:
                if a[1] >= 0 and not acc[a[1]]:
                    acc[a[1]] = True
                    st.append(a[1])
        rev = [[] for _ in range(S)]
        for s in range(S):
            for a in self.states[s]["arcs"]:
                if a[1] >= 0:
                    rev[a[1]].append(s)
                else:
                    coacc[s] = True
        st = [s for s in range(S) if coacc[s]]
        while st:
            s = st.pop()
            for q in rev[s]:
                if not coacc[q]:
                    coacc[q] = True
                    st.append(q)
        if not (acc[0] and coacc[0]):
            return [], []
        keep = [-1] * S
        K = 0
        for s in range(S):
            if acc[s] and coacc[s]:
                keep[s] = K
                K += 1
        orig = [0] * K
        for s in range(S):
            if keep[s] >= 0:
                orig[keep[s]] = s
        indeg = [0] * K
        for s in range(S):
            if keep[s] < 0:
                continue
            for a in self.states[s]["arcs"]:
                if a[1] >= 0 and keep[a[1]] >= 0:
                    indeg[keep[a[1]]] += 1
        order, stk = [], [0]
        while stk:
            k = stk.pop()
            order.append(k)
            for a in reversed(self.states[orig[k]]["arcs"]):
                if a[1] >= 0 and keep[a[1]] >= 0:
                    indeg[keep[a[1]]] -= 1
                    if indeg[keep[a[1]]] == 0:
                        stk.append(keep[a[1]])
        assert len(order) == K
        pos = [0] * K
        for i, k in enumerate(order):
            pos[k] = i
        W, Fi = [[] for _ in range(K)], [None] * K
        for k in range(K):
            stt = self.states[orig[k]]
            p = pos[k]
            for (label, nxt, w, full) in stt["arcs"]:
                res = list(full[len(stt["base"]):])
                if nxt < 0:
                    Fi[p] = (w[0], w[1], res)
                elif keep[nxt] >= 0:
                    W[p].append((label, pos[keep[nxt]], w[0], w[1], res))
        return W, Fi


def determinize_pruned(N, links, fin, start, beam=6.0, max_mem=50000000):
    """DeterminizeLatticePruned: LatticeDeterminizerPruned at `beam`; when its
    memory estimate stops it short of 0.7 x beam, the input is pruned at a
    narrower beam (beam x sqrt(effective / beam), at least beam / 4) and the
    determinization retried (at most 10 times).  -> (W, Fi) as _determinize."""
    if N == 0 or start < 0:
        return [], []
    topo = _topo(N, links)
    cur_links, cur_fin = links, fin
    for it in range(10):
        d = _PrunedDet(N, cur_links, cur_fin, start, topo, beam, max_mem)
        d.run()
        if d.guard:
            return None
        if d.eff >= beam * 0.7 or beam == INF or it + 1 == 10:
            return d.output()
        nb = beam * math.sqrt(max(d.eff, 0.0) / beam)  # (rounding can put eff just below 0: Kaldi would take NaN)
        beam = max(nb, 0.25 * beam)
        cur_links, cur_fin = _prune_det_input(N, cur_links, cur_fin, start, topo, beam)
    return None


def tid_first(tm):
    """Per transition-id: a phone's first one (out of HMM state 0, not a
    self-loop; Kaldi TransitionIdToHmmState == 0 && !IsSelfLoop)."""
    return (np.asarray(tm.tid2hmmstate) == 0) & (np.asarray(tm.tid_is_selfloop) == 0)


def _determinize(N, links, fin, start):
    if N == 0 or start < 0:
        return [], []
    outl = [[] for _ in range(N)]
    for i, l in enumerate(links):
        outl[l[0]].append(i)

    def times(w, g, a):
        return (F32(w[0] + F32(g)), F32(w[1] + F32(a)))

    def closure(sub):
        at = {e[0]: i for i, e in enumerate(sub)}
        work = list(range(len(sub)))
        while work:
            i = work.pop()
            e = sub[i]
            for li in outl[e[0]]:
                s, d, t, w, g, x = links[li]
                if w != 0:
                    continue
                n = (d, times(e[1], g, x), e[2] + ((t,) if t != 0 else ()))
                if d not in at:
                    at[d] = len(sub)
                    work.append(len(sub))
                    sub.append(n)
                elif _better(n, sub[at[d]]):
                    sub[at[d]] = n
                    work.append(at[d])
        # Kaldi's ConvertToMinimal: tokens with word links or a final cost
        sub = [e for e in sub if fin[e[0]] is not None or any(links[li][3] != 0 for li in outl[e[0]])]
        sub.sort(key=lambda e: e[0])
        return sub

    def normalize(sub):
        tot = sub[0][1]
        for e in sub:
            if _cmp(e[1], tot) > 0:
                tot = e[1]
        n = len(sub[0][2])
        for e in sub:
            j = 0
            while j < n and j < len(e[2]) and e[2][j] == sub[0][2][j]:
                j += 1
            n = j
        prefix = list(sub[0][2][:n])
        out = [(e[0], (F32(e[1][0] - tot[0]), F32(e[1][1] - tot[1])), e[2][n:]) for e in sub]
        return out, tot, prefix

    delta = 1.0 / 1024.0
    index, subsets = {}, []

    def find_or_add(sub):
        key = tuple((e[0], e[2]) for e in sub)
        for sid in index.get(key, []):
            o = subsets[sid]
            if all(abs(float(o[i][1][0]) - float(sub[i][1][0])) <= delta and
                   abs(float(o[i][1][1]) - float(sub[i][1][1])) <= delta for i in range(len(o))):
                return sid, False
        sid = len(subsets)
        subsets.append(sub)
        index.setdefault(key, []).append(sid)
        return sid, True

    s0 = closure([(start, (F32(0), F32(0)), ())])
    find_or_add(s0)
    arcs = [[]]
    queue = [0]
    qi = 0
    while qi < len(queue):
        sid = queue[qi]
        qi += 1
        by_word = {}
        for e in subsets[sid]:
            for li in outl[e[0]]:
                s, d, t, w, g, x = links[li]
                if w == 0:
                    continue
                n = (d, times(e[1], g, x), e[2] + ((t,) if t != 0 else ()))
                v = by_word.setdefault(w, [])
                for j, y in enumerate(v):
                    if y[0] == d:
                        if _better(n, y):
                            v[j] = n
                        break
                else:
                    v.append(n)
        for w in sorted(by_word):
            sub = closure(by_word[w])
            if not sub:
                continue
            sub, tot, prefix = normalize(sub)
            dst, added = find_or_add(sub)
            if added:
                queue.append(dst)
                arcs.append([])
            arcs[sid].append((w, dst, tot[0], tot[1], prefix))
    S = len(subsets)
    finals = [None] * S
    for s in range(S):
        best = None
        for e in subsets[s]:
            if fin[e[0]] is None:
                continue
            c = (e[0], (F32(e[1][0] + F32(fin[e[0]][0])), F32(e[1][1] + F32(fin[e[0]][1]))), e[2])
            if best is None or _better(c, best):
                best = c
        if best is not None:
            finals[s] = (best[1][0], best[1][1], list(best[2]))
    # topological order: DFS stack as the C++ (arcs pushed in reverse)
    indeg = [0] * S
    for s in range(S):
        for a in arcs[s]:
            indeg[a[1]] += 1
    order, st = [], [0]
    while st:
        s = st.pop()
        order.append(s)
        for a in reversed(arcs[s]):
            indeg[a[1]] -= 1
            if indeg[a[1]] == 0:
                st.append(a[1])
    pos = {s: i for i, s in enumerate(order)}
    W = [[] for _ in range(S)]
    Fi = [None] * S
    for s in range(S):
        W[pos[s]] = [(w, pos[d], g, a, p) for (w, d, g, a, p) in arcs[s]]
        Fi[pos[s]] = finals[s]
    return W, Fi


def scale_graph(W, Fi, scale):
    W = [[(w, d, F32(F32(g) * F32(scale)), a, p) for (w, d, g, a, p) in v] for v in W]
    Fi = [None if f is None else (F32(F32(f[0]) * F32(scale)), f[1], f[2]) for f in Fi]
    return W, Fi


# -------------------------------------------------------------------- MBR
def _logadd(x, y):
    if x < y:
        diff = x - y
        x = y
    else:
        diff = y - x
    if diff >= math.log(np.finfo(np.float64).eps):
        return x + math.log1p(math.exp(diff))
    return x


def mbr(W, Fi):
    S = len(W)
    if S == 0:
        return dict(words=[], conf=[], times=[])
    N = S + 1
    arcs, pre = [], [[] for _ in range(N + 1)]

    def add(s, e, w, ll):
        pre[e].append(len(arcs))
        arcs.append((w, s, e, ll))
    t = [-1] * (S + 1)
    t[0] = 0
    for s in range(S):
        for (w, d, g, a, p) in W[s]:
            add(s + 1, d + 1, w, -float(F32(F32(g) + F32(a))))
            t[d] = t[s] + len(p)
        if Fi[s] is not None:
            add(s + 1, N, 0, -float(F32(F32(Fi[s][0]) + F32(Fi[s][1]))))
            t[S] = t[s] + len(Fi[s][2])
    st = [0] * (N + 1)
    for s in range(S + 1):
        st[s + 1] = max(0, t[s])
    best = [-INF] * (N + 1)
    frm = [-1] * (N + 1)
    best[1] = 0.0
    for n in range(2, N + 1):
        for ai in pre[n]:
            w, s, e, ll = arcs[ai]
            v = best[s] + ll
            if v > best[n]:
                best[n] = v
                frm[n] = ai
    R = []
    n = N
    while n > 1 and frm[n] >= 0:
        if arcs[frm[n]][0] != 0:
            R.append(arcs[frm[n]][0])
        n = arcs[frm[n]][1]
    R.reverse()

    def l(a, b, pen=False):
        return 0.0 if a == b else (1.0 + 1.0e-05 if pen else 1.0)

    result = None
    for it in range(1000):
        R = [0] + [x for w in R if w != 0 for x in (w, 0)]
        Q = len(R)
        alpha = [0.0] * (N + 1)
        ad = [[0.0] * (Q + 1) for _ in range(N + 1)]
        bd = [[0.0] * (Q + 1) for _ in range(N + 1)]
        ada = [0.0] * (Q + 1)
        alpha[1] = 0.0
        ad[1][0] = 0.0
        for q in range(1, Q + 1):
            ad[1][q] = ad[1][q - 1] + l(0, R[q - 1])
        for n in range(2, N + 1):
            an = -INF
            for ai in pre[n]:
                an = _logadd(an, alpha[arcs[ai][1]] + arcs[ai][3])
            alpha[n] = an
            for ai in pre[n]:
                w, s, e, ll = arcs[ai]
                for q in range(Q + 1):
                    if q == 0:
                        ada[q] = ad[s][q] + l(w, 0, True)
                    else:
                        rq = R[q - 1]  # substitution, insertion, deletion (within the arc)
                        ada[q] = min(ad[s][q - 1] + l(w, rq), ad[s][q] + l(w, 0, True), ada[q - 1] + l(0, rq))
                    ad[n][q] += math.exp(alpha[s] + ll - alpha[n]) * ada[q]
        gamma = [dict() for _ in range(Q + 1)]
        tau_b, tau_e = [0.0] * (Q + 1), [0.0] * (Q + 1)
        b_arc = [0] * (Q + 1)
        bd[N][Q] = 1.0
        for n in range(N, 1, -1):
            for ai in pre[n]:
                w, s, e, ll = arcs[ai]
                ada[0] = ad[s][0] + l(w, 0, True)
                for q in range(1, Q + 1):
                    rq = R[q - 1]
                    a1, a2, a3 = ad[s][q - 1] + l(w, rq), ad[s][q] + l(w, 0, True), ada[q - 1] + l(0, rq)
                    if a1 <= a2:
                        b_arc[q], ada[q] = (1, a1) if a1 <= a3 else (3, a3)
                    else:
                        b_arc[q], ada[q] = (2, a2) if a2 <= a3 else (3, a3)
                bda = [0.0] * (Q + 1)
                post = math.exp(alpha[s] + ll - alpha[n])
                for q in range(Q, 0, -1):
                    bda[q] += post * bd[n][q]
                    if b_arc[q] == 1:
                        bd[s][q - 1] += bda[q]
                        gamma[q][w] = gamma[q].get(w, 0.0) + bda[q]
                        tau_b[q] += st[s] * bda[q]
                        tau_e[q] += st[n] * bda[q]
                    elif b_arc[q] == 2:
                        bd[s][q] += bda[q]
                    else:
                        bda[q - 1] += bda[q]
                        gamma[q][0] = gamma[q].get(0, 0.0) + bda[q]
                        tau_b[q] += st[s] * bda[q]
                        tau_e[q] += st[n] * bda[q]
                bda[0] += post * bd[n][0]
                bd[s][0] += bda[0]
        bda = [0.0] * (Q + 1)
        for q in range(Q, 0, -1):
            bda[q] += bd[1][q]
            bda[q - 1] += bda[q]
            gamma[q][0] = gamma[q].get(0, 0.0) + bda[q]
            tau_b[q] += st[1] * bda[q]
            tau_e[q] += st[1] * bda[q]
        g_ = []
        for q in range(1, Q + 1):
            v = sorted(((k, float(F32(x))) for k, x in gamma[q].items()), key=lambda z: z[0])
            v = sorted(v, key=lambda z: -z[1])  # stable: ties keep word order
            g_.append(v)
        times = [(float(F32(tau_b[q])), float(F32(tau_e[q]))) for q in range(1, Q + 1)]
        dq = 0.0
        result = dict(words=[], conf=[], times=[])
        for q in range(Q):
            g = g_[q]
            old = 0.0
            new = g[0][1] if g else 0.0
            for k, x in g:
                if k == R[q]:
                    old = x
            dq += old - new
            if g:
                R[q] = g[0][0]
            if R[q] != 0:
                conf = 0.0
                for k, x in g:
                    if k == R[q]:
                        conf = x
                result["words"].append(R[q])
                result["conf"].append(conf)
                result["times"].append(times[q])
        if dq == 0.0 or it > 100:
            break
    return result


def nbest(W, Fi, n):
    S = len(W)
    if S == 0 or n <= 0:
        return []
    best = [None] * S
    for s in range(S - 1, -1, -1):
        c = []
        if Fi[s] is not None:
            c.append((F32(Fi[s][0]), F32(Fi[s][1]), -1, 0))
        for i, (w, d, g, a, p) in enumerate(W[s]):
            for k, (bg, ba, _, _) in enumerate(best[d]):
                c.append((F32(F32(g) + bg), F32(F32(a) + ba), i, k))
        import functools
        c.sort(key=functools.cmp_to_key(lambda x, y: -_cmp((x[0], x[1]), (y[0], y[1]))))
        best[s] = c[:n]
    out = []
    for k in range(len(best[0])):
        g, a = best[0][k][0], best[0][k][1]
        words, spans = [], []
        s, rank, t = 0, k, 0
        while True:
            _, _, ai, r = best[s][rank]
            if ai < 0:
                break
            w, d, _, _, p = W[s][ai]
            if w != 0:
                words.append(w)
                spans.append((t, t + len(p)))
            t += len(p)
            s, rank = d, r
        out.append(dict(words=words, spans=spans, graph=float(g), acoustic=float(a)))
    return out


# ---------------------------------------------------------------- alignment
def align_tables(tm, boundary_file):
    """Per transition-id (phone boundary type, IsFinal, IsSelfLoop) from the
    transition model and word_boundary.int (1 nonword .. 5 singleton)."""
    names = {"nonword": 1, "begin": 2, "end": 3, "internal": 4, "singleton": 5}
    ptype = {}
    with open(boundary_file) as f:
        for line in f:
            p, t = line.split()
            ptype[int(p)] = names[t]
    ty = np.array([ptype.get(int(p), 0) for p in tm.tid2phone], np.int8)
    ty[0] = 0
    return ty, np.asarray(tm.tid_is_final, np.int8), np.asarray(tm.tid_is_selfloop, np.int8)


def _phone_end(fin, loop, t, i):
    n = len(t)
    while i < n and not fin[t[i]]:
        i += 1
    if i == n:
        return -1
    i += 1
    while i < n and loop[t[i]]:
        i += 1
    return -1 if i == n else i


def _try_output(ty, fin, loop, t, w):
    if not t:
        return -1, 0
    k = ty[t[0]]
    if k == 1:
        return _phone_end(fin, loop, t, 0), 0
    if not w:
        return -1, 0
    if k == 5:
        return _phone_end(fin, loop, t, 0), w[0]
    if k == 2:
        i = 0
        while i < len(t) and ty[t[i]] != 3:
            i += 1
        if i == len(t):
            return -1, 0
        return _phone_end(fin, loop, t, i), w[0]
    return -1, 0


def word_align(W, Fi, tables):
    """LatticeWordAligner restated as the C++ (csrc/lattice.cc) does it."""
    ty, fin, loop = tables
    S = len(W)
    if S == 0:
        return [], []
    nodes, index, eps, outs, isfin, queue = [], {}, [], [], [], []

    def get(n):
        k = (n[0], tuple(n[1]), tuple(n[2]))
        if k in index:
            return index[k]
        index[k] = len(nodes)
        nodes.append(n)
        eps.append([])
        outs.append([])
        isfin.append(False)
        queue.append(len(nodes) - 1)
        return len(nodes) - 1

    get((0, [], []))
    qi = 0
    while qi < len(queue):
        i = queue[qi]
        qi += 1
        s, t, w = nodes[i]
        k, lab = _try_output(ty, fin, loop, t, w)
        if k >= 0:
            to = get((s, t[k:], w[1:] if lab != 0 else w))
            outs[i].append((to, lab, list(t[:k])))
            continue
        if s < 0:
            if not t and not w:
                isfin[i] = True
                continue
            lab, nw = 0, w
            if not (t and ty[t[0]] == 1) and w:
                lab, nw = w[0], w[1:]
            to = get((-1, [], nw))
            outs[i].append((to, lab, list(t)))
            continue
        if Fi[s] is not None:
            to = get((-1, t + list(Fi[s][2]), w))
            eps[i].append((to, (F32(Fi[s][0]), F32(Fi[s][1]))))
        for (word, d, g, a, p) in W[s]:
            to = get((d, t + list(p), w + ([word] if word != 0 else [])))
            eps[i].append((to, (F32(g), F32(a))))
    N = len(nodes)
    arcs = [[] for _ in range(N)]
    fw, isf = [None] * N, [False] * N
    for x in range(N):
        # DFS postorder of the epsilon graph from x, reversed = topological
        mark, topo, stk = {x: 1}, [], [[x, 0]]
        while stk:
            u, j = stk[-1]
            if j < len(eps[u]):
                stk[-1][1] += 1
                v = eps[u][j][0]
                if v not in mark:
                    mark[v] = 1
                    stk.append([v, 0])
            else:
                topo.append(u)
                stk.pop()
        topo.reverse()
        clo = {x: (F32(0), F32(0))}
        for u in topo:
            for v, wt in eps[u]:
                cand = (F32(clo[u][0] + wt[0]), F32(clo[u][1] + wt[1]))
                if v not in clo or _cmp(cand, clo[v]) > 0:
                    clo[v] = cand
        for u in topo:
            cw = clo[u]
            for (to, lab, tids) in outs[u]:
                arcs[x].append((lab, to, cw[0], cw[1], tids))
            if isfin[u] and (not isf[x] or _cmp(cw, fw[x]) > 0):
                isf[x] = True
                fw[x] = cw
    reach = [False] * N
    reach[0] = True
    st = [0]
    while st:
        u = st.pop()
        for a in arcs[u]:
            if not reach[a[1]]:
                reach[a[1]] = True
                st.append(a[1])
    rev = [[] for _ in range(N)]
    for u in range(N):
        for a in arcs[u]:
            rev[a[1]].append(u)
    co = [False] * N
    st = [u for u in range(N) if isf[u] and reach[u]]
    for u in st:
        co[u] = True
    while st:
        u = st.pop()
        for p in rev[u]:
            if not co[p] and reach[p]:
                co[p] = True
                st.append(p)
    if not co[0]:
        return [], []
    indeg = [0] * N
    for u in range(N):
        if co[u]:
            for a in arcs[u]:
                if co[a[1]]:
                    indeg[a[1]] += 1
    order, st = [], [0]
    while st:
        u = st.pop()
        order.append(u)
        for a in reversed(arcs[u]):
            if co[a[1]]:
                indeg[a[1]] -= 1
                if indeg[a[1]] == 0:
                    st.append(a[1])
    pos = {u: i for i, u in enumerate(order)}
    A = [[(lab, pos[to], g, a, tids) for (lab, to, g, a, tids) in arcs[u] if co[to]] for u in order]
    F = [None if not isf[u] else (fw[u][0], fw[u][1], []) for u in order]
    return A, F


def results(oracle, llh, use_final=True, graph_scale=0.9, nbest_n=0, rescore=None, hash_size=0, kaldi=None,
            lazy_state=None):
    """The reference's result chain over the oracle decoder's lattice of
    `llh`: prune, determinize, graph scale, word alignment (when the model has
    word_boundary.int), then MBR (and n-best).  hash_size: the decoder's
    HashList size at the segment start (Kaldi order; 0 = a new decoder).
    kaldi: the decoder order (None: oracle_py.decoder_order()).  lazy_state:
    the stream's OpenFST lazy numbering at the segment start
    (oracle_py.LazyState, updated in place; None: a fresh one)."""
    import os
    r = oracle.graph.decode(llh, oracle.beam, oracle.max_active, oracle.min_active, oracle.beam_delta,
                            use_final, lattice=True, hash_size=hash_size, kaldi=kaldi, lazy_state=lazy_state)
    W, Fi = determinize_phone(prune(raw_from_oracle(r, oracle.graph, use_final), 6.0),
                              oracle.graph.ilabel, oracle.graph.olabel, oracle.tm.tid2phone,
                              tid_first(oracle.tm))
    if rescore is not None:  # (W, Fi) -> rescored (W, Fi) or None (unchanged)
        rr = rescore(W, Fi)
        if rr is not None:
            W, Fi = rr
    if graph_scale != 1.0:
        W, Fi = scale_graph(W, Fi, graph_scale)
    wb = os.path.join(oracle.dir, "graph", "phones", "word_boundary.int")
    if os.path.exists(wb):
        W, Fi = word_align(W, Fi, align_tables(oracle.tm, wb))
    out = dict(mbr=mbr(W, Fi))
    if nbest_n:
        out["nbest"] = nbest(W, Fi, nbest_n)
    return out
