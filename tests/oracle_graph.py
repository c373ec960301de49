"""CPU restatement of the static lookahead / grammar graph construction.

TEST INFRASTRUCTURE ONLY (the checker for ``vosk-api_amd/csrc/graph_compose.cc``;
nothing in the product imports it).  Follows:

* OpenFST composition of HCLr.fst with Gr.fst as the reference requests it,
  ``LookaheadComposeFst(*hcl_fst_, *g_fst_, disambig_)``
  (``src/recognizer.cc:31-37``): the alternative sequence composition filter
  (grammar epsilons before HCL output epsilons), disambiguation
  transition-ids mapped to epsilon.  Unlike the C++ expansion this one does
  NOT prune with label reachability: it expands every composed state and
  then trims, so agreement with the product also checks that the lookahead
  pruning removes only dead states.
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


def compose(hcl: kf.Fst, g: kf.Fst, disambig) -> kf.Fst:
    dis = set(int(d) for d in disambig)
    # grammar: epsilon arcs in order, non-epsilon arcs stably sorted by label
    SB = g.num_states
    geps, gwords = [], []
    for s in range(SB):
        b, e = int(g.row[s]), int(g.row[s + 1])
        geps.append([a for a in range(b, e) if g.ilabel[a] == 0])
        ws = sorted((a for a in range(b, e) if g.ilabel[a] != 0), key=lambda a: int(g.ilabel[a]))
        by = {}
        for a in ws:
            by.setdefault(int(g.ilabel[a]), []).append(a)
        gwords.append(by)
    gfinal = np.isfinite(g.final)
    has_eps = [len(x) > 0 for x in geps]
    alleps = [len(gwords[s]) == 0 and not gfinal[s] for s in range(SB)]

    ids = {}
    keys = []

    def sid(q1, q2, fs):
        k = (q1, q2, fs)
        i = ids.get(k)
        if i is None:
            i = ids[k] = len(keys)
            keys.append(k)
        return i

    start = sid(int(hcl.start), int(g.start), 0)
    finals, rows, il, ol, wt, nx = [], [0], [], [], [], []
    s = 0
    while s < len(keys):
        q1, q2, fs = keys[s]
        fa, fb = hcl.final[q1], g.final[q2]
        finals.append(np.float32(fa + fb) if np.isfinite(fa) and np.isfinite(fb) else np.float32(np.inf))
        if fs == 0:
            for a in geps[q2]:
                il.append(0); ol.append(int(g.olabel[a])); wt.append(np.float32(g.weight[a]))
                nx.append(sid(q1, int(g.nextstate[a]), 0))
        for a in range(int(hcl.row[q1]), int(hcl.row[q1 + 1])):
            lab = int(hcl.ilabel[a])
            lab = 0 if lab in dis else lab
            p = int(hcl.nextstate[a])
            o = int(hcl.olabel[a])
            if o == 0:
                if alleps[q2]:
                    continue
                il.append(lab); ol.append(0); wt.append(np.float32(hcl.weight[a]))
                nx.append(sid(p, q2, 1 if has_eps[q2] else 0))
            else:
                for b in gwords[q2].get(o, []):
                    il.append(lab); ol.append(int(g.olabel[b]))
                    wt.append(np.float32(np.float32(hcl.weight[a]) + np.float32(g.weight[b])))
                    nx.append(sid(p, int(g.nextstate[b]), 0))
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
    return kf.Fst(0, np.array(finals, np.float32), np.array(rows, np.int64), np.array(il, np.int32),
                  np.array(ol, np.int32), np.array(wt, np.float32), np.array(nx, np.int32))


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
    kf.write_const_fst(os.path.join(out_dir, "graph", "HCLG.fst"), model_graph(src_dir, grammar))
    return out_dir


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
    lib.vamd_graph_free(h)
    if os.path.exists(out_dir):
        shutil.rmtree(out_dir)
    shutil.copytree(model_dir, out_dir, ignore=shutil.ignore_patterns("HCLr.fst", "Gr.fst", "disambig_tid.int"))
    kf.write_const_fst(os.path.join(out_dir, "graph", "HCLG.fst"), g)
    return out_dir, S
