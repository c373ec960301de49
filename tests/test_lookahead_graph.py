"""Lookahead graphs and runtime grammars on the host (CPU).

* the ngram (LOUDS) reader against hand-built n-gram models (the explicit
  destinations are the longest existing history, the backoff arc goes to
  the history without its oldest word);
* the static expansion of HCLr o Gr in libvosk.so (graph_compose.cc, through
  the host-only ``vamd_graph_*`` ABI) against the unpruned restatement in
  tests/oracle_graph.py, array for array, for the model graph and for
  grammar graphs;
* LanguageModelEstimator known answers (src/language_model.cc) and the
  grammar JSON handling (src/recognizer.cc:60-92).
"""
import ctypes as C
import os

import numpy as np
import pytest

import kaldi_formats as kf
import oracle_graph as OG

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "vosk-api_amd", "vosk", "libvosk.so")


@pytest.fixture(scope="module")
def lib():
    lib = C.CDLL(LIB)
    lib.vamd_graph_new.restype = C.c_void_p
    lib.vamd_graph_new.argtypes = [C.c_char_p, C.c_char_p]
    lib.vamd_graph_dims.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_longlong)]
    lib.vamd_graph_copy.argtypes = [C.c_void_p] + [C.c_void_p] * 6
    lib.vamd_graph_free.argtypes = [C.c_void_p]
    lib.vosk_set_log_level(-2)
    return lib


def _cgraph(lib, model, grammar=None):
    h = lib.vamd_graph_new(model.encode(), grammar.encode() if grammar is not None else None)
    if not h:
        return None
    st, na = C.c_int(), C.c_longlong()
    S = lib.vamd_graph_dims(h, C.byref(st), C.byref(na))
    A = na.value
    out = kf.Fst(st.value, np.zeros(S, np.float32), np.zeros(S + 1, np.int64), np.zeros(A, np.int32),
                 np.zeros(A, np.int32), np.zeros(A, np.float32), np.zeros(A, np.int32))
    lib.vamd_graph_copy(h, out.final.ctypes.data, out.row.ctypes.data, out.ilabel.ctypes.data,
                        out.olabel.ctypes.data, out.weight.ctypes.data, out.nextstate.ctypes.data)
    # OpenFST's lazy numbering table (vamd_graph_lazy)
    lib.vamd_graph_lazy.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lrow = np.zeros(S + 1, np.int64)
    ids = lib.vamd_graph_lazy(h, lrow.ctypes.data, None)
    lnext = np.zeros(int(lrow[-1]), np.int32)
    lib.vamd_graph_lazy(h, lrow.ctypes.data, lnext.ctypes.data)
    out.lazy = (lrow, lnext, ids)
    lib.vamd_graph_free(h)
    return out


def _assert_same_fst(a, b):
    assert a.start == b.start
    if hasattr(a, "lazy") and hasattr(b, "lazy"):  # the lazy numbering tables
        np.testing.assert_array_equal(a.lazy[0], b.lazy[0])
        np.testing.assert_array_equal(a.lazy[1], b.lazy[1])
        assert a.lazy[2] == b.lazy[2] and a.lazy[2] >= a.num_states
    np.testing.assert_array_equal(a.row, b.row)
    np.testing.assert_array_equal(a.ilabel, b.ilabel)
    np.testing.assert_array_equal(a.olabel, b.olabel)
    np.testing.assert_array_equal(a.nextstate, b.nextstate)
    np.testing.assert_array_equal(a.weight.view(np.int32), b.weight.view(np.int32))
    np.testing.assert_array_equal(a.final.view(np.int32), b.final.view(np.int32))


def _toy_lm():
    # histories most recent word first; () root, (0,) sentence start
    return {
        (): {"fut": {1: 2.0, 2: 2.5, 3: 3.0, 4: 3.5}, "final": 1.5},
        (0,): {"fut": {1: 0.5, 3: 1.25}, "backoff": 0.75, "final": None},
        (1,): {"fut": {2: 0.25, 4: 1.0}, "backoff": 0.5, "final": 2.0},
        (2,): {"fut": {3: 0.125}, "backoff": 0.625, "final": None},
        (1, 0): {"fut": {2: 0.0625}, "backoff": 0.375, "final": None},
        (2, 1): {"fut": {1: 0.3, 4: 0.2}, "backoff": 0.1, "final": 0.9},
    }


def test_ngram_fst_semantics(tmp_path):
    lm = _toy_lm()
    path = str(tmp_path / "Gr.fst")
    kf.write_ngram_fst(path, lm)
    f = kf.read_fst(path)
    # level order of the reversed-history trie: (), then children by label
    order = [(), (0,), (1,), (2,), (1, 0), (2, 1)]
    assert f.num_states == len(order) and f.start == 1
    for s, h in enumerate(order):
        arcs = [(int(f.ilabel[a]), int(f.olabel[a]), float(f.weight[a]), order[int(f.nextstate[a])])
                for a in range(int(f.row[s]), int(f.row[s + 1]))]
        want = []
        if h:
            want.append((0, 0, float(np.float32(lm[h]["backoff"])), h[:-1]))
        for w, c in sorted(lm[h]["fut"].items()):
            nh = (w,) + h
            while nh not in lm:  # longest existing history
                nh = nh[:-1]
            want.append((w, w, float(np.float32(c)), nh))
        assert arcs == want, h
        fc = lm[h]["final"]
        assert (f.final[s] == np.float32(fc)) if fc is not None else np.isinf(f.final[s])


def test_lookahead_file_roundtrip(tmp_path):
    f = kf.Fst(0, np.array([0.0, np.inf], np.float32), np.array([0, 2, 3], np.int64),
               np.array([5, 0, 7], np.int32), np.array([0, 3, 4], np.int32),
               np.array([0.5, 1.0, 0.25], np.float32), np.array([1, 0, 0], np.int32))
    path = str(tmp_path / "HCLr.fst")
    kf.write_lookahead_fst(path, f)
    g = kf.read_fst(path)
    _assert_same_fst(f, g)


def test_lookahead_graph_matches_restatement(lib, synth_lookahead):
    c = _cgraph(lib, synth_lookahead)
    assert c is not None
    p = OG.model_graph(synth_lookahead)
    _assert_same_fst(c, p)
    # every disambiguation id became epsilon; ilabels are transition-ids
    dis = [int(x) for x in open(os.path.join(synth_lookahead, "graph", "disambig_tid.int")).read().split()]
    assert not np.isin(c.ilabel, dis).any()
    hcl = kf.read_fst(os.path.join(synth_lookahead, "graph", "HCLr.fst"))
    assert np.isin(hcl.ilabel, dis).any()
    # every state is useful (trimmed), emitting arcs first per state
    for s in range(c.num_states):
        il = c.ilabel[c.row[s]:c.row[s + 1]]
        assert not np.any((il[:-1] == 0) & (il[1:] != 0))


@pytest.mark.parametrize("grammar", [
    '["w00001 w00002", "w00003 w00005 w00007", "w00002"]',
    '["w00010", "w00010 w00011 w00010", "nonexistent w00012", "[unk]"]',
    ' [ "w00004\\tw00005" , "w00006  w00007"] ',
])
def test_grammar_graph_matches_restatement(lib, synth_lookahead, grammar):
    c = _cgraph(lib, synth_lookahead, grammar)
    assert c is not None
    _assert_same_fst(c, OG.model_graph(synth_lookahead, grammar))
    # the grammar's words (and only those) appear on output labels
    words = {v: k for k, v in kf.read_symbol_table(os.path.join(synth_lookahead, "graph", "words.txt")).items()}
    sents = OG.parse_grammar(grammar, words)
    assert set(int(x) for x in c.olabel if x) == set(w for s in sents for w in s)


@pytest.mark.parametrize("grammar", ['{"a": 1}', "[1, 2]", "[]", "not json", '["unterminated'])
def test_bad_grammar_is_an_error(lib, synth_lookahead, grammar):
    assert _cgraph(lib, synth_lookahead, grammar) is None
    with pytest.raises(ValueError):
        OG.parse_grammar(grammar, {})


def test_grammar_on_hclg_model_is_an_error_here(lib, synth_model):
    # the recognizer falls back to the static graph with a warning; the
    # diagnostic graph builder reports it
    assert _cgraph(lib, synth_model, '["w00001"]') is None


def test_grammar_lm_known_answer():
    g = OG.estimate_grammar_lm([[1, 2], [1]], order=2, discount=0.5)
    L = lambda x: float(-OG.logf(np.float32(x)))  # noqa: E731
    assert g.start == 0 and g.num_states == 3
    arcs = [[(int(g.ilabel[a]), float(g.weight[a]), int(g.nextstate[a]))
             for a in range(int(g.row[s]), int(g.row[s + 1]))] for s in range(3)]
    # root: counts {</s>: 2, 1: 2, 2: 1} of 5 (own + children's)
    assert arcs[0] == [(1, L(0.2), 1), (2, L(0.1), 2)]
    assert g.final[0] == np.float32(L(0.2))
    # history (1): {</s>: 1, 2: 1}; backoff -log(0.5)
    assert arcs[1] == [(0, L(0.5), 0), (2, L(0.25), 2)]
    assert g.final[1] == np.float32(L(0.25))
    assert arcs[2] == [(0, L(0.5), 0)]
    assert g.final[2] == np.float32(L(0.5))


def test_grammar_parse_escapes():
    words = {"a": 1, "b/c": 2, 'q"x': 3, "\\u00e9": 4}
    # JSON::ToString re-escapes the parsed string (src/json.h:295-298): "\/"
    # becomes "/", but a parsed quote is looked up as \" and is not found
    assert OG.parse_grammar('["a b\\/c", "q\\"x", "a"]', words) == [[1, 2], [], [1]]
    # json.h keeps \\u escapes as text, and ToString re-escapes the backslash
    assert OG.parse_grammar('["\\u00e9 a"]', words) == [[1]]


def test_truncated_graph_files_fail_cleanly(lib, synth_lookahead, tmp_path):
    import shutil
    d = str(tmp_path / "m")
    shutil.copytree(synth_lookahead, d)
    gr = os.path.join(d, "graph", "Gr.fst")
    data = open(gr, "rb").read()
    open(gr, "wb").write(data[:len(data) // 2])
    assert _cgraph(lib, d) is None
    os.remove(gr)
    assert _cgraph(lib, d) is None  # neither HCLG nor HCLr + Gr


def _tiny_pair(model_src, out):
    """A hand-built HCLr / G pair on a copy of a lookahead model: words 1 =
    'a', 2 = 'a b', 3 = 'c' in a prefix tree (word labels on the word-end arcs
    back to state 0, as the synthetic HCLr), G = unigram state 0 (final 1.0;
    w1 1.0, w2 2.0, w3 3.0 -> history w3) and history w3 (backoff 0.5, w1
    0.25)."""
    import shutil
    shutil.copytree(model_src, out)
    gd = os.path.join(out, "graph")
    # (src, tid, olabel, weight, dst), per state olabel-sorted
    arcs = [(0, 1, 0, 0.0, 1), (0, 5, 0, 0.0, 3), (1, 3, 0, 0.0, 2), (1, 2, 1, 0.0, 0),
            (2, 4, 2, 0.0, 0), (3, 6, 3, 0.0, 0)]
    hcl = kf.Fst(0, np.array([0.0, np.inf, np.inf, np.inf], np.float32), np.array([0, 2, 4, 5, 6], np.int64),
                 np.array([a[1] for a in arcs], np.int32), np.array([a[2] for a in arcs], np.int32),
                 np.array([a[3] for a in arcs], np.float32), np.array([a[4] for a in arcs], np.int32))
    kf.write_lookahead_fst(os.path.join(gd, "HCLr.fst"), hcl)
    g = kf.Fst(0, np.array([1.0, np.inf], np.float32), np.array([0, 3, 5], np.int64),
               np.array([1, 2, 3, 0, 1], np.int32), np.array([1, 2, 3, 0, 1], np.int32),
               np.array([1.0, 2.0, 3.0, 0.5, 0.25], np.float32), np.array([0, 0, 1, 0, 0], np.int32))
    kf.write_const_fst(os.path.join(gd, "Gr.fst"), g)
    return out, hcl, g


def test_lookahead_pushing_known_answer(lib, synth_lookahead, tmp_path):
    """Per-arc pushed weights and pushed labels of OpenFST's lookahead
    composition (PushWeights / PushLabels filters), worked by hand:
    * 0 -a-> 1 reaches w1, w2 at G state 0: weight log-sum(1, 2) = 0.686738,
      the state keeps Quantize(0.686738) = 703/1024;
    * 0 -c-> 3 reaches w3 only: w3 (3.0) is output on this arc, G advances;
    * 1 -(w1)-> 0 matched at G 0: 1.0 - 703/1024; 1 -b-> 2 reaches w2 only:
      pushed, 2.0 - 703/1024; the word-end arcs of pushed words output nothing;
    * at history w3: the backoff 0.5; 0 -a-> 1 reaches w1 only there: w1
      (0.25) pushed; 'c' is not reachable at history w3."""
    d, hcl, g = _tiny_pair(synth_lookahead, str(tmp_path / "m"))
    lw = np.float32(1.0 - np.log(1.0 + np.exp(-1.0)))
    q = np.float32(703.0 / 1024.0)
    assert np.float32(np.floor(lw * np.float32(1024) + np.float32(0.5)) / np.float32(1024)) == q
    want = sorted([(1, 0, lw), (5, 3, np.float32(3.0)), (2, 1, np.float32(1.0) - q), (3, 2, np.float32(2.0) - q),
                   (4, 0, np.float32(0.0)), (6, 0, np.float32(0.0)), (0, 0, np.float32(0.5)),
                   (1, 1, np.float32(0.25)), (2, 0, np.float32(0.0))])
    for c in (OG.compose(hcl, g, []), _cgraph(lib, d)):
        assert c is not None and c.num_states == 6
        got = sorted(zip(c.ilabel.tolist(), c.olabel.tolist(), c.weight.tolist()))
        assert [(a, b) for a, b, _ in got] == [(a, b) for a, b, _ in want]
        np.testing.assert_array_equal(np.array([w for _, _, w in got], np.float32),
                                      np.array([w for _, _, w in want], np.float32))
        fin = c.final[np.isfinite(c.final)]
        assert fin.tolist() == [1.0]
    # the unpruned composition's path weights, up to the quantization residue
    # of each pushed weight (lw - q), as OpenFST's filter leaves them


def test_lookahead_pushing_is_exercised(synth_lookahead):
    """On the synthetic lookahead model both pushes happen (labels output
    before the word-end arc, fractional pushed weights on epsilon-output
    arcs)."""
    hcl = kf.read_fst(os.path.join(synth_lookahead, "graph", "HCLr.fst"))
    g = kf.read_fst(os.path.join(synth_lookahead, "graph", "Gr.fst"))
    dis = [int(x) for x in open(os.path.join(synth_lookahead, "graph", "disambig_tid.int")).read().split()]
    c = OG.compose(hcl, g, dis)
    # word-end transition-ids of HCLr (the arcs carrying word labels there)
    wend = set(int(x) for x in hcl.ilabel[hcl.olabel != 0]) - set(dis) - {0}
    pushed = (c.olabel != 0) & ~np.isin(c.ilabel, list(wend)) & (c.ilabel != 0)
    assert pushed.sum() > 0
    frac = (c.olabel == 0) & (c.ilabel != 0) & (c.weight != 0) & (np.abs(c.weight) < 50)
    assert frac.sum() > 0


def test_lazy_numbering_hand_built(lib, synth_lookahead, tmp_path):
    """OpenFST's lazy ComposeFst numbering order on the hand-built pair of
    test_lookahead_pushing_known_answer, worked by hand from the model
    graph_compose.cc implements: ComposeFstImpl::Expand -> OrderedExpand
    over HCLr's arcs (MATCH_BOTH resolved to matching G's input, as
    ComposeFstImpl::MatchInput does when HCLr's state has no more arcs than
    G's): first the "loop" -- G's epsilon (backoff) arcs against HCLr's
    implicit self-loop --, then each HCLr arc in arc order against G (an
    output-epsilon arc against G's implicit loop, with the lookahead /
    pushing filters; with a pushed label pending only the arcs towards it).
    States (by their arcs): A = (h0, G0) start, B = (h1, G0) after 'a' with
    the pushed weight, C = (h3, G1) with w3 pending, D = (h2, G0) with w2
    pending, E = (h0, G1), F = (h1, G0) with w1 pending.  Destinations in
    composition order: A: B C; B: D A; C: E; D: A; E: A F (G1's backoff
    first, then 'a' with w1 pushed); F: A.  This pins the lazy table
    (vamd_graph_lazy) independently of the oracle, which decodes with the
    same table; that OpenFST resolves MATCH_BOTH to this side on every
    state is this restatement's reading, unpinned."""
    d, hcl, g = _tiny_pair(synth_lookahead, str(tmp_path / "m"))
    c = _cgraph(lib, d)
    assert c is not None and c.num_states == 6
    sig = {}
    for s in range(c.num_states):
        sig[s] = tuple(sorted(zip(c.ilabel[c.row[s]:c.row[s + 1]].tolist(),
                                  c.olabel[c.row[s]:c.row[s + 1]].tolist())))
    names = {((1, 0), (5, 3)): "A", ((2, 1), (3, 2)): "B", ((6, 0),): "C", ((4, 0),): "D",
             ((0, 0), (1, 1)): "E", ((2, 0),): "F"}
    name = {s: names[sig[s]] for s in range(c.num_states)}
    assert name[c.start] == "A"
    lrow, lnext, nids = c.lazy
    assert nids == c.num_states  # no dead state in this composition
    got = {name[s]: "".join(name[int(t)] for t in lnext[lrow[s]:lrow[s + 1]]) for s in range(c.num_states)}
    assert got == {"A": "BC", "B": "DA", "C": "E", "D": "A", "E": "AF", "F": "A"}
