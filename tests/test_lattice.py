"""Result pipeline over lattices (host code of libvosk.so, csrc/lattice.cc)
against its oracle restatement (tests/oracle_lattice.py): lattice-beam
pruning, word-level determinization, graph scaling, word alignment, Kaldi MBR
(words, confidences, times) and n-best, on the oracle decoder's lattices of
the synthetic models.  CPU only (host-only ABI, no GPU)."""
import os
import numpy as np
import pytest

import oracle_lattice as OL
import oracle_py


def _lattice(model, wave, use_final=True):
    o = oracle_py.OracleModel(model)
    llh = o.loglikes(wave)
    r = o.graph.decode(llh, o.beam, o.max_active, o.min_active, o.beam_delta, use_final, lattice=True)
    return o, r, OL.raw_from_oracle(r, o.graph, use_final)


def _python(o, L, beam=6.0, scale=0.9, n=5):
    P = OL.prune(L, beam)
    W, Fi = OL.determinize(P, o.graph.ilabel, o.graph.olabel)
    if scale != 1.0:
        W, Fi = OL.scale_graph(W, Fi, scale)
    return P, W, OL.mbr(W, Fi), OL.nbest(W, Fi, n)


@pytest.mark.parametrize("secs,use_final", [(1.5, True), (4, True), (8.3, True), (5, False)])
def test_cpp_pipeline_matches_restatement(synth_model, test_wave, secs, use_final):
    from vosk import engine
    o, r, L = _lattice(synth_model, test_wave[:int(16000 * secs)], use_final)
    scale = 0.9 if use_final else 1.0
    got = engine.lattice_words(L, o.graph.ilabel, o.graph.olabel, 6.0, scale, 5)
    P, W, mb, nb = _python(o, L, 6.0, scale, 5)
    assert got["pruned_tokens"] == len(P["tok_state"])
    assert got["pruned_links"] == len(P["link_src"])
    assert got["det_ok"] == 1
    assert got["det_states"] == len(W)
    assert got["det_arcs"] == sum(len(v) for v in W)
    assert got["mbr"]["words"] == mb["words"]
    np.testing.assert_allclose(got["mbr"]["conf"], mb["conf"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(np.reshape(got["mbr"]["times"], (-1, 2)),
                               np.reshape(mb["times"], (-1, 2)), rtol=0, atol=1e-4)
    assert [x["words"] for x in got["nbest"]] == [x["words"] for x in nb]
    assert [x["spans"] for x in got["nbest"]] == [[list(s) for s in x["spans"]] for x in nb]
    np.testing.assert_allclose([x["graph"] + x["acoustic"] for x in got["nbest"]],
                               [x["graph"] + x["acoustic"] for x in nb], rtol=0, atol=1e-3)
    # sanity of the semantics: confidences are posteriors, n-best is sorted
    # and distinct, the best path is the first alternative
    assert all(0.0 <= c <= 1.0 + 1e-6 for c in got["mbr"]["conf"])
    costs = [x["graph"] + x["acoustic"] for x in got["nbest"]]
    assert costs == sorted(costs)
    assert len({tuple(x["words"]) for x in got["nbest"]}) == len(got["nbest"])
    # without the graph scale the first alternative is the decoder's best path
    unscaled = engine.lattice_words(L, o.graph.ilabel, o.graph.olabel, 6.0, 1.0, 1)
    assert unscaled["nbest"][0]["words"] == r["words"]


@pytest.mark.parametrize("secs,use_final", [(4, True), (6, False)])
def test_numpy_raw_lattice_and_prune_equal_the_loop_restatement(synth_model, test_wave, secs, use_final):
    """raw_from_oracle / prune (numpy) give exactly the arrays of their
    link-by-link statements (raw_from_oracle_loop / prune_loop)."""
    o, r, L = _lattice(synth_model, test_wave[:int(16000 * secs)], use_final)
    L0 = OL.raw_from_oracle_loop(r, o.graph, use_final)
    for k in L0:
        np.testing.assert_array_equal(np.asarray(L[k]), np.asarray(L0[k]), err_msg=k)
    for beam in (6.0, 2.0):
        P, P0 = OL.prune(L, beam), OL.prune_loop(L, beam)
        for k in P0:
            np.testing.assert_array_equal(np.asarray(P[k]), np.asarray(P0[k]), err_msg=f"{k} beam {beam}")


def test_pruning_keeps_best_path_and_shrinks(synth_model, test_wave):
    o, r, L = _lattice(synth_model, test_wave[:16000 * 3])
    P = OL.prune(L, 6.0)
    assert 0 < len(P["tok_state"]) < len(L["tok_state"])
    # every best-path arc survives the beam
    arcs = set(P["link_arc"].tolist())
    assert all(a in arcs for a in r["path"])
    # a zero beam keeps only best-path ties
    P0 = OL.prune(L, 0.0)
    assert len(P0["link_src"]) <= len(r["path"]) + 4


def test_mbr_confidences_on_a_two_word_choice():
    """Hand-made lattice: one frame, two competing words with costs 0 and
    ln(3): posteriors 0.75 / 0.25, MBR picks the likelier word."""
    import math
    L = dict(num_frames=1, frame_begin=np.array([0, 1, 3], np.int32), tok_state=np.array([0, 1, 2], np.int32),
             tok_cost=np.array([0, 0, 1], np.float32), link_src=np.array([0, 0], np.int32),
             link_dst=np.array([1, 2], np.int32), link_arc=np.array([0, 1], np.int32),
             link_graph=np.array([0.0, math.log(3.0)], np.float32), link_ac=np.zeros(2, np.float32),
             final_cost=np.zeros(0, np.float32))
    ilabel, olabel = np.array([5, 6], np.int32), np.array([11, 12], np.int32)
    from vosk import engine
    got = engine.lattice_words(L, ilabel, olabel, 6.0, 1.0, 3)
    assert got["mbr"]["words"] == [11]
    assert got["mbr"]["conf"][0] == pytest.approx(0.75, abs=1e-6)
    assert got["mbr"]["times"] == [[0, 1]]
    assert [x["words"] for x in got["nbest"]] == [[11], [12]]


def _tables(o):
    return OL.align_tables(o.tm, os.path.join(o.dir, "graph", "phones", "word_boundary.int"))


@pytest.mark.parametrize("secs", [2, 4, 8.3])
def test_word_alignment_matches_restatement(synth_model, test_wave, secs):
    from vosk import engine
    o, r, L = _lattice(synth_model, test_wave[:int(16000 * secs)])
    tables = _tables(o)
    got = engine.lattice_words(L, o.graph.ilabel, o.graph.olabel, 6.0, 0.9, 4, align=tables)
    W, Fi = OL.scale_graph(*OL.determinize(OL.prune(L, 6.0), o.graph.ilabel, o.graph.olabel), 0.9)
    A, AF = OL.word_align(W, Fi, tables)
    assert got["align_ok"] == 1
    assert got["align_states"] == len(A) and got["align_arcs"] == sum(len(v) for v in A)
    mb, nb = OL.mbr(A, AF), OL.nbest(A, AF, 4)
    assert got["mbr"]["words"] == mb["words"]
    np.testing.assert_allclose(got["mbr"]["conf"], mb["conf"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(np.reshape(got["mbr"]["times"], (-1, 2)),
                               np.reshape(mb["times"], (-1, 2)), rtol=0, atol=1e-4)
    assert [x["words"] for x in got["nbest"]] == [x["words"] for x in nb]
    assert [x["spans"] for x in got["nbest"]] == [[list(s) for s in x["spans"]] for x in nb]
    # alignment keeps every path and its cost
    nb0 = OL.nbest(W, Fi, 4)
    assert [x["words"] for x in nb0] == [x["words"] for x in nb]
    np.testing.assert_allclose([x["graph"] + x["acoustic"] for x in nb0],
                               [x["graph"] + x["acoustic"] for x in nb], rtol=0, atol=1e-2)
    # every aligned word arc spans whole phones from a begin (or singleton)
    # phone to an end (or singleton) phone; silence arcs hold non-word phones
    ty, fin, loop = tables
    for arcs in A:
        for (w, d, g, a, tids) in arcs:
            if not tids:
                continue
            if w == 0:
                assert all(ty[t] == 1 for t in tids) or d == len(A) - 1
            else:
                assert ty[tids[0]] in (2, 5)
                ends = [t for t in tids if ty[t] in (3, 5) and fin[t]]
                assert ends or d == len(A) - 1


@pytest.mark.parametrize("secs,use_final", [(1.5, True), (4, True), (8.3, True), (5, False)])
def test_phone_pass_determinization_matches_restatement(synth_model, test_wave, secs, use_final):
    """The reference's GetLattice determinization (DeterminizeLatticePhonePrunedWrapper:
    phone + word pass, phones deleted, word pass; src/recognizer.cc:678) in the
    C++ vs its restatement: same determinized lattice size, MBR and n-best.
    And what determinization preserves: the word-level n-best (word sequences,
    best costs) equals the word-only determinization's."""
    from vosk import engine
    o, r, L = _lattice(synth_model, test_wave[:int(16000 * secs)], use_final)
    scale = 0.9 if use_final else 1.0
    first = OL.tid_first(o.tm)
    assert first.sum() > 0
    word_only = engine.lattice_words(L, o.graph.ilabel, o.graph.olabel, 6.0, scale, 8)
    engine.set_phones(o.tm.tid2phone, first)
    try:
        got = engine.lattice_words(L, o.graph.ilabel, o.graph.olabel, 6.0, scale, 8)
    finally:
        engine.set_phones(None)
    W, Fi = OL.determinize_phone(OL.prune(L, 6.0), o.graph.ilabel, o.graph.olabel, o.tm.tid2phone, first)
    assert got["det_ok"] == 1
    assert got["det_states"] == len(W)
    assert got["det_arcs"] == sum(len(v) for v in W)
    if scale != 1.0:
        W, Fi = OL.scale_graph(W, Fi, scale)
    mb, nb = OL.mbr(W, Fi), OL.nbest(W, Fi, 8)
    assert got["mbr"]["words"] == mb["words"]
    np.testing.assert_allclose(got["mbr"]["conf"], mb["conf"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(np.reshape(got["mbr"]["times"], (-1, 2)),
                               np.reshape(mb["times"], (-1, 2)), rtol=0, atol=1e-4)
    assert [x["words"] for x in got["nbest"]] == [x["words"] for x in nb]
    assert [x["spans"] for x in got["nbest"]] == [[list(s) for s in x["spans"]] for x in nb]
    assert [x["words"] for x in got["nbest"]] == [x["words"] for x in word_only["nbest"]]
    np.testing.assert_allclose([x["graph"] + x["acoustic"] for x in got["nbest"]],
                               [x["graph"] + x["acoustic"] for x in word_only["nbest"]], rtol=1e-6, atol=1e-3)


def _pruning_lattice():
    """Hand-made lattice where the exact determinization keeps a word
    sequence the pruned one drops.  Frame 1: token 1 after X (cost 0) or B
    (5), token 2 after B (5.5); frame 2 (final): C from token 1 (0), D from
    token 2 (0), E from token 1 (5.5).  Every link lies on a path within the
    beam (6): XC 0, BC 5, BD 5.5, XE 5.5; but B followed by E costs 10.5.
    Exact determinization: the prefixes X ({1}) and B ({1, 2}) are different
    states and B's keeps E (BE = 10.5); Kaldi's pruned one drops that
    transition (forward 5 + 5.5 > best + beam)."""
    L = dict(num_frames=2, frame_begin=np.array([0, 1, 3, 6], np.int32),
             tok_state=np.array([0, 1, 2, 3, 4, 5], np.int32), tok_cost=np.array([0, 0, 5.5, 0, 5.5, 5.5], np.float32),
             link_src=np.array([0, 0, 0, 1, 2, 1], np.int32), link_dst=np.array([1, 1, 2, 3, 4, 5], np.int32),
             link_arc=np.arange(6, dtype=np.int32),
             link_graph=np.array([0, 5, 5.5, 0, 0, 5.5], np.float32), link_ac=np.zeros(6, np.float32),
             final_cost=np.zeros(3, np.float32))
    ilabel = np.array([5, 6, 7, 8, 9, 10], np.int32)
    olabel = np.array([11, 12, 12, 13, 14, 15], np.int32)
    return L, ilabel, olabel


def test_pruned_determinization_known_answer():
    from vosk import engine
    L, il, ol = _pruning_lattice()
    exact = engine.lattice_words(L, il, ol, 6.0, 1.0, 10)
    assert sorted(tuple(x["words"]) for x in exact["nbest"]) == [(11, 13), (11, 15), (12, 13), (12, 14), (12, 15)]
    zeros = np.zeros(11, np.int32)
    engine.set_phones(zeros, zeros.astype(np.int8))  # no phone starts: both passes on words, pruned
    try:
        got = engine.lattice_words(L, il, ol, 6.0, 1.0, 10)
    finally:
        engine.set_phones(None)
    assert got["det_ok"] == 1
    assert sorted(tuple(x["words"]) for x in got["nbest"]) == [(11, 13), (11, 15), (12, 13), (12, 14)]
    costs = {tuple(x["words"]): x["graph"] + x["acoustic"] for x in got["nbest"]}
    assert costs[(11, 13)] == 0.0 and costs[(12, 13)] == 5.0 and costs[(12, 14)] == 5.5 and costs[(11, 15)] == 5.5
    W, Fi = OL.determinize_phone(OL.prune(L, 6.0), il, ol, zeros, zeros.astype(bool))
    assert got["det_states"] == len(W) and got["det_arcs"] == sum(len(v) for v in W)
    assert sorted(tuple(x["words"]) for x in OL.nbest(W, Fi, 10)) == sorted(costs)


@pytest.mark.parametrize("secs,max_mem", [(6, 20000), (8.3, 20000), (8.3, 30000)])
def test_pruned_determinization_memory_retry(synth_model, test_wave, secs, max_mem):
    """A memory limit the determinization passes: it stops, reports the beam it
    reached, and DeterminizeLatticePruned retries on the input pruned at a
    narrower beam -- the C++ and the restatement agree step for step, and the
    best path survives."""
    from vosk import engine
    o, r, L = _lattice(synth_model, test_wave[:int(16000 * secs)])
    first = OL.tid_first(o.tm)
    engine.set_phones(o.tm.tid2phone, first)
    engine.set_det_max_mem(max_mem)
    try:
        got = engine.lattice_words(L, o.graph.ilabel, o.graph.olabel, 6.0, 1.0, 6)
        full = None
        engine.set_det_max_mem()
        full = engine.lattice_words(L, o.graph.ilabel, o.graph.olabel, 6.0, 1.0, 6)
    finally:
        engine.set_phones(None)
        engine.set_det_max_mem()
    W, Fi = OL.determinize_phone(OL.prune(L, 6.0), o.graph.ilabel, o.graph.olabel, o.tm.tid2phone, first,
                                 max_mem=max_mem)
    assert got["det_ok"] == 1
    assert got["det_states"] == len(W) and got["det_arcs"] == sum(len(v) for v in W)
    assert got["det_states"] < full["det_states"] or got["det_arcs"] < full["det_arcs"]  # the limit bit
    nb = OL.nbest(W, Fi, 6)
    assert [x["words"] for x in got["nbest"]] == [x["words"] for x in nb]
    assert got["nbest"][0]["words"] == full["nbest"][0]["words"] == r["words"]
