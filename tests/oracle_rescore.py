"""CPU restatement of the final-result LM rescoring (TEST INFRASTRUCTURE ONLY).

Follows the reference's GetResult (src/recognizer.cc:675-711) with the
objects src/model.cc:308-314 loads: the determinized lattice with negated
graph costs composed with rescore/G.fst (ReadAndPrepareLmFst: projected on
its output labels, ilabel-sorted; sequence composition filter), determinized
on words (oracle_lattice.determinize over the same state-level form the C++
builds), negated back, then composed with the ConstArpa LM
(ConstArpaLmDeterministicFst: histories of at most order-1 words reduced to
existing LM states, -logprob on the graph part, -logprob(</s>) on finals).
Mirrors vosk-api_amd/csrc/rescore.cc operation for operation.  Parity
unpinned against Kaldi: the ConstArpa file layout is the restatement in
kaldi_formats.write_const_arpa / rescore.h, no real G.carpa exists here.
"""
from __future__ import annotations

import struct

import numpy as np

import oracle_lattice as OL

F32 = np.float32
INF = F32(np.inf)


class ConstArpa:
    def __init__(self, path):
        d = open(path, "rb").read()
        assert d[:2] == b"\0B"
        p = [2]

        def tok():
            while d[p[0]:p[0] + 1] == b" ":
                p[0] += 1
            e = d.index(b" ", p[0])
            t = d[p[0]:e].decode()
            p[0] = e + 1
            return t

        def integer():
            n = d[p[0]]
            v = struct.unpack_from("<i" if n == 4 else "<q", d, p[0] + 1)[0]
            p[0] += 1 + n
            return v

        assert tok() == "<ConstArpaLm>" and tok() == "<LmInfo>"
        self.bos, self.eos, self.unk, self.order = integer(), integer(), integer(), integer()
        assert tok() == "</LmInfo>" and tok() == "<LmStates>"
        n = integer()
        self.st = np.frombuffer(d, np.int32, n, p[0]).copy()
        p[0] += 4 * n
        assert tok() == "</LmStates>" and tok() == "<LmUnigram>"
        self.uni = [integer() for _ in range(integer())]
        assert tok() == "</LmUnigram>" and tok() == "<LmOverflow>"
        self.ovf = [integer() for _ in range(integer())]

    @staticmethod
    def _f(i):
        return F32(np.array([i], np.int32).view(np.float32)[0])

    def _ustate(self, w):
        if w < 0 or w >= len(self.uni) or self.uni[w] < 0:  # -1 = no state (Kaldi)
            return None
        return self.uni[w]

    def _child(self, word, parent):
        n = int(self.st[parent + 2])
        lo, hi = 1, n
        while lo <= hi:
            mid = (lo + hi) // 2
            w = int(self.st[parent + 1 + 2 * mid])
            if w == word:
                return int(self.st[parent + 2 + 2 * mid])
            if w < word:
                lo = mid + 1
            else:
                hi = mid - 1
        return None

    def _decode(self, info, parent):
        if info % 2 == 0:
            return None, self._f(info)
        off = int(info / 2)  # C++ truncation toward zero
        c = parent + off if off > 0 else self.ovf[-off]
        return c, self._f(self.st[c])

    def _state(self, seq):
        if not seq:
            return None
        s = self._ustate(seq[0])
        for w in seq[1:]:
            if s is None:
                return None
            info = self._child(w, s)
            if info is None:
                return None
            s, _ = self._decode(info, s)
        return s

    def history_exists(self, hist):
        return len(hist) > 0 and self._state(hist) is not None

    def _recurse(self, word, hist):
        if not hist:
            s = self._ustate(word)
            return self._f(self.st[s]) if s is not None else F32(-np.inf)
        backoff = F32(0)
        s = self._state(hist)
        if s is not None:
            info = self._child(word, s)
            if info is not None:
                return self._decode(info, s)[1]
            backoff = self._f(self.st[s + 1])
        return F32(backoff + self._recurse(word, hist[1:]))

    def logprob(self, word, hist):
        hist = list(hist)
        while len(hist) >= self.order:
            hist.pop(0)
        if self.unk != -1:
            if self._ustate(word) is None:
                word = self.unk
            hist = [h if self._ustate(h) is not None else self.unk for h in hist]
        return self._recurse(word, hist)


def prepare_g(fst):
    """ReadAndPrepareLmFst: project on the output labels, stable-sort each
    state's arcs by label."""
    il = fst.olabel.copy()
    ol, wt, nx = fst.olabel.copy(), fst.weight.copy(), fst.nextstate.copy()
    for s in range(fst.num_states):
        b, e = int(fst.row[s]), int(fst.row[s + 1])
        idx = sorted(range(b, e), key=lambda a: int(il[a]))
        il[b:e], ol[b:e], wt[b:e], nx[b:e] = il[idx], ol[idx], wt[idx], nx[idx]
    return dict(start=int(fst.start), final=fst.final, row=fst.row, ilabel=il, olabel=ol,
                weight=wt, nextstate=nx)


def _topo(W):
    S = len(W)
    indeg = [0] * S
    for s in range(S):
        for a in W[s]:
            indeg[a[1]] += 1
    st = [s for s in range(S - 1, -1, -1) if indeg[s] == 0]
    order = []
    while st:
        s = st.pop()
        order.append(s)
        for a in W[s]:
            indeg[a[1]] -= 1
            if indeg[a[1]] == 0:
                st.append(a[1])
    return order


def _trim(W, Fi):
    S = len(W)
    rev = [[] for _ in range(S)]
    for s in range(S):
        for a in W[s]:
            rev[a[1]].append(s)
    co = [Fi[s] is not None for s in range(S)]
    q = [s for s in range(S) if co[s]]
    i = 0
    while i < len(q):
        for p in rev[q[i]]:
            if not co[p]:
                co[p] = True
                q.append(p)
        i += 1
    nid, n = {}, 0
    for s in range(S):
        if co[s]:
            nid[s] = n
            n += 1
    W2 = [[(a[0], nid[a[1]], a[2], a[3], a[4]) for a in W[s] if co[a[1]]] for s in range(S) if co[s]]
    F2 = [Fi[s] for s in range(S) if co[s]]
    return W2, F2


def rescore(W, Fi, G, lm: ConstArpa):
    """(W, Fi): oracle_lattice.determinize output (graph unscaled) ->
    rescored lattice, or None when rescoring fails (as the C++ falls back)."""
    ids, keys = {}, []

    def id_of(q, gq, fs):
        k = (q, gq, fs)
        if k not in ids:
            ids[k] = len(keys)
            keys.append(k)
        return ids[k]

    id_of(0, G["start"], 0)
    carcs, cfin = [], []
    s = 0
    while s < len(keys):
        q, gq, fs = keys[s]
        arcs = []
        has_eps = any(a[0] == 0 for a in W[q])
        all_eps = all(a[0] == 0 for a in W[q])
        lat_final = Fi[q] is not None
        b, e = int(G["row"][gq]), int(G["row"][gq + 1])
        if not (all_eps and not lat_final):
            for x in range(b, e):
                if G["ilabel"][x] == 0:
                    arcs.append((0, id_of(q, int(G["nextstate"][x]), 1 if has_eps else 0),
                                 F32(G["weight"][x]), F32(0), []))
        for (w, nx, g, a, tids) in W[q]:
            if w == 0:
                if fs != 0:
                    continue
                arcs.append((0, id_of(nx, gq, 0), F32(-F32(g)), F32(a), tids))
                continue
            for x in range(b, e):
                if G["ilabel"][x] < w:
                    continue
                if G["ilabel"][x] > w:
                    break
                arcs.append((w, id_of(nx, int(G["nextstate"][x]), 0), F32(F32(-F32(g)) + F32(G["weight"][x])),
                             F32(a), tids))
        carcs.append(arcs)
        gf = F32(G["final"][gq])
        if lat_final and gf != INF:
            cfin.append((F32(F32(-F32(Fi[q][0])) + gf), F32(Fi[q][1]), Fi[q][2]))
        else:
            cfin.append(None)
        s += 1
    C = len(keys)
    time = [-1] * C
    indeg = [0] * C
    for s in range(C):
        for a in carcs[s]:
            indeg[a[1]] += 1
    st, order = [0], []
    time[0] = 0
    while st:
        s = st.pop()
        order.append(s)
        for a in carcs[s]:
            t = time[s] + len(a[4])
            if time[a[1]] >= 0 and time[a[1]] != t:
                return None
            time[a[1]] = t
            indeg[a[1]] -= 1
            if indeg[a[1]] == 0:
                st.append(a[1])
    if len(order) != C:
        return None
    F = -1
    for s in range(C):
        if cfin[s] is not None:
            t = time[s] + len(cfin[s][2])
            if F >= 0 and t != F:
                return None
            F = t
    if F < 0:
        return None
    tok_time = list(time)
    pl = []

    def chain(src, dst, word, g, a, tids):
        if len(tids) <= 1:
            pl.append((src, dst, tids[0] if tids else 0, word, g, a))
            return
        cur = src
        for i, t in enumerate(tids):
            nxt = dst
            if i + 1 < len(tids):
                nxt = len(tok_time)
                tok_time.append(tok_time[src] + i + 1)
            pl.append((cur, nxt, t, word if i == 0 else 0, g if i == 0 else F32(0), a if i == 0 else F32(0)))
            cur = nxt

    superfinal = C
    tok_time.append(F)
    for s in range(C):
        for a in carcs[s]:
            chain(s, a[1], a[0], a[2], a[3], a[4])
        if cfin[s] is not None:
            chain(s, superfinal, 0, cfin[s][0], cfin[s][1], cfin[s][2])
    T = len(tok_time)
    perm = sorted(range(T), key=lambda i: tok_time[i])
    pos = [0] * T
    for i, t in enumerate(perm):
        pos[t] = i
    fb = np.zeros(F + 2, np.int64)
    for t in tok_time:
        fb[t + 1] += 1
    fb = np.cumsum(fb)
    tc = np.ones(T, np.float32)
    tc[pos[0]] = 0.0
    fc = np.full(int(fb[F + 1] - fb[F]), np.inf, np.float32)
    fc[pos[superfinal] - fb[F]] = 0.0
    L = dict(num_frames=F, frame_begin=fb, tok_state=np.zeros(T, np.int32), tok_cost=tc,
             link_src=np.array([pos[x[0]] for x in pl], np.int32),
             link_dst=np.array([pos[x[1]] for x in pl], np.int32),
             link_arc=np.arange(len(pl), dtype=np.int32),
             link_graph=np.array([x[4] for x in pl], np.float32),
             link_ac=np.array([x[5] for x in pl], np.float32), final_cost=fc)
    il = np.array([x[2] for x in pl], np.int32)
    ol = np.array([x[3] for x in pl], np.int32)
    D, DF = OL.determinize(L, il, ol)
    if not D:
        return None
    D, DF = OL.scale_graph(D, DF, -1.0)
    # ConstArpa deterministic composition
    topo = _topo(D)
    tix = {q: i for i, q in enumerate(topo)}
    hid, hists = {}, []

    def h_of(h):
        h = tuple(h)
        if h not in hid:
            hid[h] = len(hists)
            hists.append(h)
        return hid[h]

    rid, rkeys = {}, []

    def r_of(q, h):
        if (q, h) not in rid:
            rid[(q, h)] = len(rkeys)
            rkeys.append((q, h))
        return rid[(q, h)]

    r_of(0, h_of([lm.bos]))
    RA, RF = [], []
    s = 0
    while s < len(rkeys):
        q, h = rkeys[s]
        arcs = []
        for (w, nx, g, a, tids) in D[q]:
            if w == 0:
                arcs.append((0, r_of(nx, h), g, a, tids))
                continue
            lp = lm.logprob(w, hists[h])
            if lp == -np.inf:
                continue
            nh = list(hists[h]) + [w]
            if len(nh) >= lm.order:
                nh.pop(0)
            while not lm.history_exists(nh):
                nh.pop(0)
            arcs.append((w, r_of(nx, h_of(nh)), F32(F32(g) + F32(-lp)), a, tids))
        RA.append(arcs)
        fin = None
        if DF[q] is not None:
            lp = lm.logprob(lm.eos, hists[h])
            if lp != -np.inf:
                fin = (F32(F32(DF[q][0]) + F32(-lp)), DF[q][1], DF[q][2])
        RF.append(fin)
        s += 1
    R = len(rkeys)
    rorder = sorted(range(R), key=lambda x: tix[rkeys[x][0]])
    rnew = [0] * R
    for i, x in enumerate(rorder):
        rnew[x] = i
    W2 = [None] * R
    F2 = [None] * R
    for x in range(R):
        W2[rnew[x]] = [(a[0], rnew[a[1]], a[2], a[3], a[4]) for a in RA[x]]
        F2[rnew[x]] = RF[x]
    W2, F2 = _trim(W2, F2)
    if not W2:
        return None
    return W2, F2
