"""CPU restatement of the static lookahead / grammar graph construction.

TEST INFRASTRUCTURE ONLY (the checker for ``vosk-api_amd/csrc/graph_compose.cc``;
nothing in the product imports it).  Follows:

* OpenFST composition of HCLr.fst with Gr.fst as the reference requests it,
  ``LookaheadComposeFst(*hcl_fst_, *g_fst_, disambig_)``
  (``src/recognizer.cc:31-37``): ComposeFst with an olabel_lookahead first
  FST selects OpenFST's lookahead filter chain [O: compose.h CreateBase,
  lookahead-filter.h DefaultLookAhead<StdArc, MATCH_OUTPUT>]: the
  alternative sequence filter (grammar epsilons before HCL output epsilons),
  label lookahead with weight pushing (FastLogAccumulator log-sums of the
  reachable grammar arcs, quantized to 1/1024 in the filter state) and
  label pushing (a single reachable grammar arc is taken early), then
  disambiguation transition-ids mapped to epsilon.  The label reachability
  is a plain per-state search here (the C++ uses strongly connected
  components and a per-word index for wide states), and every HCL arc is
  looked ahead (no index), so agreement checks those shortcuts too.
* ``LanguageModelEstimator`` (``src/language_model.cc:27-211``) with the
  grammar recognizer's order 2 / discount 0.5 (``src/recognizer.cc:68-71``);
  float arithmetic as the C++ (``count * discount / total`` in float, logf).
* the grammar phrase list parse (``src/recognizer.cc:60-92``, ``src/json.h``
  ``parse_string`` + ``json_escape``).

Parity unpinned against Kaldi/OpenFST themselves: no lookahead model exists
in this container; the synthetic lookahead models are written by
``vosk-api_amd/tools/make_synth_model.py --graph lookahead``.
"""
from __future__ import annotations

import ctypes
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "vosk-api_amd", "tools"))
import kaldi_formats as kf  # noqa: E402

_libm = ctypes.CDLL("libm.so.6")
_libm.logf.restype = ctypes.c_float
_libm.logf.argtypes = [ctypes.c_float]


def logf(x):
    return np.float32(_libm.logf(ctypes.c_float(float(x))))


F32 = np.float32
_DINF = float("inf")
_ACC_LIMIT, _ACC_PERIOD = 20, 10


def _log_pos_exp(x):
    return 0.0 if x == _DINF else math.log(1.0 + math.exp(-x))


def _log_minus_exp(x):
    return 0.0 if x == _DINF else math.log(1.0 - math.exp(-x))


def _logplus_w(w, v):
    """FastLogAccumulator::LogPlus(Weight, Weight): double, rounded to float."""
    f1, f2 = float(w), float(v)
    if f1 == _DINF and f2 == _DINF:
        return F32(np.inf)
    return F32(f2 - _log_pos_exp(f1 - f2)) if f1 > f2 else F32(f1 - _log_pos_exp(f2 - f1))


def _logplus_d(f1, v):
    f2 = float(v)
    if f1 == _DINF:
        return f2
    return f2 - _log_pos_exp(f1 - f2) if f1 > f2 else f1 - _log_pos_exp(f2 - f1)


def _logminus_w(f1, f2):
    return F32(f1) if f2 == _DINF else F32(f1 - _log_minus_exp(f2 - f1))


def _acc_sum(s, wt, sw, begin, end):
    """FastLogAccumulator::Sum(w, aiter, begin, end)."""
    sb = se = end
    if sw is not None:
        ib = (begin - 1) // _ACC_PERIOD + 1 if begin > 0 else 0
        ie = end // _ACC_PERIOD
        sb, se = ib * _ACC_PERIOD, ie * _ACC_PERIOD
    for p in range(begin, min(sb, end)):
        s = _logplus_w(s, wt[p])
    if sb < se:
        f1, f2 = sw[ie], sw[ib]
        if f1 < f2:
            s = _logplus_w(s, _logminus_w(f1, f2))
    for p in range(max(sb, se), end):
        s = _logplus_w(s, wt[p])
    return s


def _quantize(v):
    if not np.isfinite(v):
        return F32(v)
    d = F32(1.0) / F32(1024.0)
    return F32(np.floor(F32(F32(v) / d) + F32(0.5)) * d)


def _intervals(labels):
    out = []
    for l in sorted(labels):
        if out and l <= out[-1][1] + 1:
            out[-1][1] = max(out[-1][1], l)
        else:
            out.append([l, l])
    return out


def reach_sets(hcl: kf.Fst):
    """Per HCLr state: the output labels reachable through output-epsilon
    arcs (first non-epsilon output label of such a path) and whether a final
    state is reachable that way -- a plain search from every state (the C++
    computes it per strongly connected component)."""
    S = hcl.num_states
    labs, fins = [], []
    for s0 in range(S):
        seen, st, L, fin = {s0}, [s0], set(), False
        while st:
            u = st.pop()
            fin = fin or bool(np.isfinite(hcl.final[u]))
            for a in range(int(hcl.row[u]), int(hcl.row[u + 1])):
                o = int(hcl.olabel[a])
                if o != 0:
                    L.add(o)
                elif int(hcl.nextstate[a]) not in seen:
                    seen.add(int(hcl.nextstate[a]))
                    st.append(int(hcl.nextstate[a]))
        labs.append(_intervals(L))
        fins.append(fin)
    return labs, fins


def _member(iv, l):
    return any(lo <= l <= hi for lo, hi in iv)


def compose(hcl: kf.Fst, g: kf.Fst, disambig) -> kf.Fst:
    """ComposeFst(HCLr, G) with OpenFST's default MATCH_OUTPUT lookahead
    filter chain (PushLabels(PushWeights(LookAhead(AltSequence)))), states
    (q1, q2, alt-sequence bit, quantized lookahead weight, pushed label);
    see graph_compose.cc for the arc rules this restates."""
    dis = set(int(d) for d in disambig)
    labs, fins = reach_sets(hcl)
    # grammar: epsilon arcs in order, non-epsilon arcs stably sorted by label
    SB = g.num_states
    gsort, gneps = [], []
    acc = []
    for s in range(SB):
        b, e = int(g.row[s]), int(g.row[s + 1])
        eps = [a for a in range(b, e) if g.ilabel[a] == 0]
        ws = sorted((a for a in range(b, e) if g.ilabel[a] != 0), key=lambda a: int(g.ilabel[a]))
        gsort.append(eps + ws)
        gneps.append(len(eps))
        if e - b >= _ACC_LIMIT:
            sw, tot = [_DINF], _DINF
            for n, a in enumerate(eps + ws, 1):
                tot = _logplus_d(tot, g.weight[a])
                if n % _ACC_PERIOD == 0:
                    sw.append(tot)
            acc.append(sw)
        else:
            acc.append(None)
    gfinal = np.isfinite(g.final)
    has_eps = [n > 0 for n in gneps]
    alleps = [gneps[s] == len(gsort[s]) and not gfinal[s] for s in range(SB)]

    def lookahead(p, q):
        iv, cf = labs[p], fins[p]
        arcs = gsort[q]
        lab = [int(g.ilabel[a]) for a in arcs]
        wt = [F32(g.weight[a]) for a in arcs]
        rfin = cf and bool(gfinal[q])
        n, nint = len(arcs), len(iv) + (1 if cf else 0)
        rb = re = -1
        w = F32(np.inf)
        if 2 * n < nint:
            for k in range(n):
                if _member(iv, lab[k]):
                    rb = k if rb < 0 else rb
                    re = k + 1
                    w = _logplus_w(w, wt[k])
        else:
            lo = 0
            for ilo, ihi in iv:
                bl = lo + int(np.searchsorted(lab[lo:], ilo, "left"))
                el = bl + int(np.searchsorted(lab[bl:], ihi + 1, "left"))
                lo = el
                if el > bl:
                    rb = bl if rb < 0 else rb
                    re = el
                    w = _acc_sum(w, wt, acc[q], bl, el)
        rarc = rb >= 0
        prefix, lw = None, F32(0.0)
        if rarc:
            if re - rb == 1 and not rfin:
                prefix = arcs[rb]
            else:
                lw = w
        if rfin and prefix is None:
            lw = min(lw, F32(g.final[q])) if rarc else F32(g.final[q])
        return rarc or rfin, prefix, lw

    ids = {}
    keys = []

    def sid(q1, q2, sb, fw, fl):
        k = (q1, q2, sb, F32(fw).tobytes(), fl)
        i = ids.get(k)
        if i is None:
            i = ids[k] = len(keys)
            keys.append((q1, q2, sb, F32(fw), fl))
        return i

    start = sid(int(hcl.start), int(g.start), 0, 0.0, -1)
    finals, rows, il, ol, wt, nx = [], [0], [], [], [], []

    def arc(i, o, w, d):
        il.append(i); ol.append(o); wt.append(F32(w)); nx.append(d)

    s = 0
    Z = F32(0.0)
    while s < len(keys):
        q1, q2, sb, fw, fl = keys[s]
        fa, fb = hcl.final[q1], g.final[q2]
        finals.append(F32(F32(F32(fa) - fw) + F32(fb)) if fl == -1 and np.isfinite(fa) and np.isfinite(fb)
                      else F32(np.inf))
        hrange = range(int(hcl.row[q1]), int(hcl.row[q1 + 1]))

        def lab_in(a):
            x = int(hcl.ilabel[a])
            return 0 if x in dis else x

        if fl != -1:
            for a in hrange:
                p, o, aw = int(hcl.nextstate[a]), int(hcl.olabel[a]), F32(hcl.weight[a])
                if o == fl:
                    arc(lab_in(a), 0, aw + Z, sid(p, q2, 0, 0.0, -1))
                elif o == 0 and _member(labs[p], fl):
                    arc(lab_in(a), 0, aw + Z, sid(p, q2, sb, fw, fl))
            rows.append(len(il))
            s += 1
            continue
        nfw = Z - fw
        if sb == 0:
            for a in gsort[q2][:gneps[q2]]:
                arc(0, int(g.olabel[a]), Z + F32(F32(g.weight[a]) + nfw), sid(q1, int(g.nextstate[a]), 0, 0.0, -1))
        nsb = 1 if has_eps[q2] else 0
        for a in hrange:
            p, o, aw = int(hcl.nextstate[a]), int(hcl.olabel[a]), F32(hcl.weight[a])
            if o == 0:
                if alleps[q2]:
                    continue
                ok, pre, lw = lookahead(p, q2)
                if not ok:
                    continue
                if pre is not None:
                    arc(lab_in(a), int(g.olabel[pre]), aw + F32(F32(Z + nfw) + F32(g.weight[pre])),
                        sid(p, int(g.nextstate[pre]), nsb, 0.0, int(g.ilabel[pre])))
                else:
                    arc(lab_in(a), 0, aw + F32(Z + F32(lw - fw)), sid(p, q2, nsb, _quantize(lw), -1))
            else:
                for b in gsort[q2][gneps[q2]:]:
                    if int(g.ilabel[b]) != o:
                        continue
                    arc(lab_in(a), int(g.olabel[b]), aw + F32(F32(g.weight[b]) + nfw),
                        sid(p, int(g.nextstate[b]), 0, 0.0, -1))
        rows.append(len(il))
        s += 1
    c = kf.Fst(start, np.array(finals, np.float32), np.array(rows, np.int64), np.array(il, np.int32),
               np.array(ol, np.int32), np.array(wt, np.float32), np.array(nx, np.int32))
    return connect_canonical(c)


def connect_canonical(f: kf.Fst) -> kf.Fst:
    """Trim to co-accessible states, renumber breadth-first from the start
    over each state's emitting arcs then epsilon-input arcs."""
    S = f.num_states
    radj = [[] for _ in range(S)]
    for s in range(S):
        for a in range(int(f.row[s]), int(f.row[s + 1])):
            radj[int(f.nextstate[a])].append(s)
    co = np.isfinite(f.final).copy()
    q = [int(x) for x in np.nonzero(co)[0]]
    i = 0
    while i < len(q):
        for p in radj[q[i]]:
            if not co[p]:
                co[p] = True
                q.append(p)
        i += 1
    if not co[f.start]:
        raise ValueError("empty composed graph")
    nid = {f.start: 0}
    order = [f.start]
    finals, rows, il, ol, wt, nx = [], [0], [], [], [], []
    i = 0
    while i < len(order):
        s = order[i]
        finals.append(f.final[s])
        arcs = list(range(int(f.row[s]), int(f.row[s + 1])))
        for a in [a for a in arcs if f.ilabel[a] != 0] + [a for a in arcs if f.ilabel[a] == 0]:
            d = int(f.nextstate[a])
            if not co[d]:
                continue
            if d not in nid:
                nid[d] = len(order)
                order.append(d)
            il.append(int(f.ilabel[a])); ol.append(int(f.olabel[a])); wt.append(f.weight[a]); nx.append(nid[d])
        rows.append(len(il))
        i += 1
    out = kf.Fst(0, np.array(finals, np.float32), np.array(rows, np.int64), np.array(il, np.int32),
                 np.array(ol, np.int32), np.array(wt, np.float32), np.array(nx, np.int32))
    # OpenFST's lazy numbering (graph_compose.cc ConnectCanonical): per state
    # its destinations in the composition's own arc order, states the trim
    # dropped numbered past the graph's
    NS = len(order)
    dead, lrow, lnext = {}, [0], []
    for s in order:
        for a in range(int(f.row[s]), int(f.row[s + 1])):
            d = int(f.nextstate[a])
            if d in nid:
                lnext.append(nid[d])
            else:
                if d not in dead:
                    dead[d] = NS + len(dead)
                lnext.append(dead[d])
        lrow.append(len(lnext))
    out.lazy = (np.array(lrow, np.int64), np.array(lnext, np.int32), NS + len(dead))
    return out


def write_lazy(out_dir, lazy):
    """graph/lazy_ids.npz next to an expanded graph/HCLG.fst: the oracle then
    buckets Kaldi's HashList by OpenFST's lazy ids (oracle_py.OracleGraph)."""
    row, nxt, ids = lazy
    if ids:
        np.savez(os.path.join(out_dir, "graph", "lazy_ids.npz"), row=row, next=nxt, ids=np.int64(ids))


def estimate_grammar_lm(sentences, order=2, discount=0.5) -> kf.Fst:
    """LanguageModelEstimator (src/language_model.cc)."""
    assert order >= 2
    states = []   # [history, counts dict, tot, backoff, fst_state]
    index = {}
    active = [0]

    def find_or_create(h):
        h = tuple(h)
        if h in index:
            return index[h]
        ans = len(states)
        states.append([h, {}, 0, -1, -1])
        index[h] = ans
        if h:
            states[ans][3] = find_or_create(h[1:])
        return ans

    def add(st, w, n):
        st[1][w] = st[1].get(w, 0) + n
        st[2] += n

    def inc(h, w):
        l = find_or_create(h)
        if states[l][2] == 0:
            active[0] += 1
        add(states[l], w, 1)

    for sent in sentences:
        h = []
        for w in sent:
            assert w != 0
            inc(h, w)
            h.append(w)
            if len(h) >= order:
                h.pop(0)
        inc(h, 0)
    n = len(states)
    for l in range(n):
        p = states[l][3]
        while p != -1:
            for w, c in sorted(states[l][1].items()):
                add(states[p], w, c)
            p = states[p][3]
    nf = 0
    for st in states:
        if st[2]:
            st[4] = nf
            nf += 1
    assert nf == active[0]

    def nonzero(h):
        h = tuple(h)
        while True:
            l = index.get(h)
            if l is None or states[l][2] == 0:
                assert h, "no state"
                h = h[1:]
            else:
                return l

    arcs = [[] for _ in range(nf)]
    final = np.full(nf, np.inf, np.float32)
    disc = np.float32(discount)
    for st in states:
        if st[4] < 0:
            continue
        for w in sorted(st[1]):
            c = st[1][w]
            pr = np.float32(np.float32(c) * disc) / np.float32(st[2])
            lp = logf(pr)
            if w == 0:
                final[st[4]] = -lp
            else:
                d = states[nonzero(st[0] + (w,))][4]
                arcs[st[4]].append((w, -lp, d))
        if st[3] >= 0:
            arcs[st[4]].append((0, -logf(np.float32(1.0) - disc), states[st[3]][4]))
    rows, il, wt, nx = [0], [], [], []
    for s in range(nf):
        for w, c, d in sorted(arcs[s], key=lambda x: x[0]):
            il.append(w); wt.append(c); nx.append(d)
        rows.append(len(il))
    return kf.Fst(states[nonzero(())][4], final, np.array(rows, np.int64), np.array(il, np.int32),
                  np.array(il, np.int32), np.array(wt, np.float32), np.array(nx, np.int32))


def _json_escape(s):
    m = {'"': '\\"', '\\': '\\\\', '\b': '\\b', '\f': '\\f', '\n': '\\n', '\r': '\\r', '\t': '\\t'}
    return "".join(m.get(c, c) for c in s)


def parse_grammar(js: str, sym2id: dict):
    """Phrase list -> word-id sentences (src/recognizer.cc:60-92)."""
    p = 0
    ws = " \t\n\r"

    def skip():
        nonlocal p
        while p < len(js) and js[p] in ws:
            p += 1

    skip()
    if p >= len(js) or js[p] != "[":
        raise ValueError("Expecting array of strings")
    p += 1
    phrases = []
    skip()
    if p < len(js) and js[p] == "]":
        p += 1
    else:
        while True:
            skip()
            if p >= len(js) or js[p] != '"':
                raise ValueError("Expecting array of strings")
            val = ""
            p += 1
            while p < len(js) and js[p] != '"':
                if js[p] != "\\":
                    val += js[p]
                    p += 1
                    continue
                p += 1
                c = js[p]
                if c == "u":
                    val += "\\u" + js[p + 1:p + 5]
                    p += 4
                else:
                    val += {'"': '"', "\\": "\\", "/": "/", "b": "\b", "f": "\f", "n": "\n",
                            "r": "\r", "t": "\t"}.get(c, "\\")
                p += 1
            p += 1
            phrases.append(_json_escape(val))
            skip()
            if p < len(js) and js[p] == ",":
                p += 1
                continue
            if p < len(js) and js[p] == "]":
                p += 1
                break
            raise ValueError("Expecting array of strings")
    if not phrases:
        raise ValueError("Expecting array of strings")
    out = []
    for line in phrases:
        out.append([sym2id[t] for t in line.split(" ") if t in sym2id])
    return out


def model_graph(model_dir, grammar=None) -> kf.Fst:
    """The static graph of a lookahead model dir (or its grammar graph)."""
    gd = os.path.join(model_dir, "graph")
    hcl = kf.read_fst(os.path.join(gd, "HCLr.fst"))
    dis = [int(x) for x in open(os.path.join(gd, "disambig_tid.int")).read().split()]
    if grammar is None:
        g = kf.read_fst(os.path.join(gd, "Gr.fst"))
    else:
        words = {v: k for k, v in kf.read_symbol_table(os.path.join(gd, "words.txt")).items()}
        g = estimate_grammar_lm(parse_grammar(grammar, words))
    return compose(hcl, g, dis)


def write_hclg_model(src_dir, out_dir, grammar=None):
    """A copy of a lookahead model dir whose graph is the composed static
    graph as graph/HCLG.fst (what the C oracle decodes)."""
    import shutil
    if os.path.exists(out_dir):
        shutil.rmtree(out_dir)
    shutil.copytree(src_dir, out_dir, ignore=shutil.ignore_patterns("HCLr.fst", "Gr.fst", "disambig_tid.int"))
    g = model_graph(src_dir, grammar)
    kf.write_const_fst(os.path.join(out_dir, "graph", "HCLG.fst"), g)
    write_lazy(out_dir, g.lazy)
    return out_dir


def lazy_csr(model_dir):
    """libvosk's OpenFST lazy-numbering CSR of a lookahead model's composed
    graph (vamd_graph_lazy): (row [S+1] int64, next int32, ids) -- per state
    of the decoding graph, its arc destinations in the composition's own arc
    order."""
    import ctypes as C
    lib = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "vosk-api_amd", "vosk",
                              "libvosk.so"))
    lib.vamd_graph_new.restype = C.c_void_p
    lib.vamd_graph_new.argtypes = [C.c_char_p, C.c_char_p]
    lib.vamd_graph_dims.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_longlong)]
    lib.vamd_graph_lazy.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.vamd_graph_free.argtypes = [C.c_void_p]
    h = lib.vamd_graph_new(model_dir.encode(), None)
    assert h
    st, na = C.c_int(), C.c_longlong()
    S = lib.vamd_graph_dims(h, C.byref(st), C.byref(na))
    row = np.zeros(S + 1, np.int64)
    ids = lib.vamd_graph_lazy(h, row.ctypes.data, None)
    nxt = np.zeros(int(row[-1]), np.int32)
    lib.vamd_graph_lazy(h, row.ctypes.data, nxt.ctypes.data)
    lib.vamd_graph_free(h)
    return row, nxt, ids


def expanded_hclg_model(model_dir, out_dir):
    """A copy of a lookahead model whose graph/HCLG.fst is libvosk's own
    static expansion of HCLr o Gr (vamd_graph_*; the expansion itself is
    checked against the Python restatement in test_lookahead_graph.py): the
    oracle decodes the graph the engine decodes.  Returns (dir, states)."""
    import ctypes as C
    import shutil
    lib = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "vosk-api_amd", "vosk",
                              "libvosk.so"))
    lib.vamd_graph_new.restype = C.c_void_p
    lib.vamd_graph_new.argtypes = [C.c_char_p, C.c_char_p]
    lib.vamd_graph_dims.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_longlong)]
    lib.vamd_graph_copy.argtypes = [C.c_void_p] + [C.c_void_p] * 6
    lib.vamd_graph_free.argtypes = [C.c_void_p]
    h = lib.vamd_graph_new(model_dir.encode(), None)
    assert h
    st, na = C.c_int(), C.c_longlong()
    S = lib.vamd_graph_dims(h, C.byref(st), C.byref(na))
    A = na.value
    g = kf.Fst(st.value, np.zeros(S, np.float32), np.zeros(S + 1, np.int64), np.zeros(A, np.int32),
               np.zeros(A, np.int32), np.zeros(A, np.float32), np.zeros(A, np.int32))
    lib.vamd_graph_copy(h, g.final.ctypes.data, g.row.ctypes.data, g.ilabel.ctypes.data,
                        g.olabel.ctypes.data, g.weight.ctypes.data, g.nextstate.ctypes.data)
    lib.vamd_graph_lazy.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lrow = np.zeros(S + 1, np.int64)
    ids = lib.vamd_graph_lazy(h, lrow.ctypes.data, None)
    lnext = np.zeros(int(lrow[-1]) if ids else 0, np.int32)
    if ids:
        lib.vamd_graph_lazy(h, lrow.ctypes.data, lnext.ctypes.data)
    lib.vamd_graph_free(h)
    if os.path.exists(out_dir):
        shutil.rmtree(out_dir)
    shutil.copytree(model_dir, out_dir, ignore=shutil.ignore_patterns("HCLr.fst", "Gr.fst", "disambig_tid.int"))
    kf.write_const_fst(os.path.join(out_dir, "graph", "HCLG.fst"), g)
    write_lazy(out_dir, (lrow, lnext, ids))
    return out_dir, S
