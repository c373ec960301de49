"""OpenFST's lazy ComposeFst numbering of a lookahead model's states (the
reference composes HCLr o Gr lazily per recognizer, src/recognizer.cc:31-37;
Kaldi's HashList buckets tokens by state id, so the Kaldi-order search
depends on it).  CPU only.

libvosk decodes a static expansion (trimmed, renumbered breadth-first, arcs
partitioned emitting-first) and carries, per state, its destinations in the
composition's own arc order (vamd_graph_lazy), from which the decoder numbers
states as OpenFST would.  The Kaldi-order oracle decoding the untrimmed
composition in its own arc order with lazy numbering (the reference's
semantics) and decoding libvosk's graph with libvosk's lazy CSR give the same
search, frame by frame."""
import os

import numpy as np
import pytest

import kaldi_formats as kf
import oracle_graph as OG
import oracle_py
from conftest import perturbed_stream


@pytest.fixture(scope="module")
def graphs(synth_lookahead, tmp_path_factory):
    d = tmp_path_factory.mktemp("lazy")
    canon, _ = OG.expanded_hclg_model(synth_lookahead, str(d / "canon"))
    os.environ["VOSK_AMD_GRAPH_RAW"] = "1"
    try:
        raw, _ = OG.expanded_hclg_model(synth_lookahead, str(d / "raw"))
    finally:
        del os.environ["VOSK_AMD_GRAPH_RAW"]
    return canon, raw, OG.lazy_csr(synth_lookahead)


def test_lazy_csr_shape(graphs):
    canon, raw, (row, nxt, ids) = graphs
    gc = kf.read_fst(os.path.join(canon, "graph", "HCLG.fst"))
    gr = kf.read_fst(os.path.join(raw, "graph", "HCLG.fst"))
    S = len(gc.final)
    assert len(row) == S + 1 and ids >= S
    # every state keeps all of its composed arcs (destinations the trim
    # dropped included), so the CSR has the composition's arc count minus the
    # arcs of dropped states
    assert row[-1] <= len(gr.ilabel) and row[-1] >= len(gc.ilabel)
    assert ids - S == len(gr.final) - S  # dropped states get ids past the graph's
    # the arc multiset per state is the graph's (destinations inside the graph)
    for s in range(0, S, max(1, S // 200)):
        a = sorted(int(x) for x in nxt[row[s]:row[s + 1]] if x < S)
        b = sorted(int(x) for x in gc.nextstate[gc.row[s]:gc.row[s + 1]])
        assert a == b, s


def test_lazy_numbering_search_equals_the_composition_s(graphs, test_wave):
    canon, raw, (row, nxt, ids) = graphs
    oc = oracle_py.OracleModel(canon)
    orw = oracle_py.OracleModel(raw)
    grw = kf.read_fst(os.path.join(raw, "graph", "HCLG.fst"))
    lazy_raw = (np.asarray(grw.row, np.int64), np.asarray(grw.nextstate, np.int32))
    for i in range(3):
        x = perturbed_stream(test_wave, 800 + i, seconds=4.0)
        llh = oc.loglikes(x)
        a = oc.graph.decode(llh, oc.beam, oc.max_active, oc.min_active, oc.beam_delta, True, kaldi=True,
                            lazy=(row, nxt))
        b = orw.graph.decode(llh, orw.beam, orw.max_active, orw.min_active, orw.beam_delta, True, kaldi=True,
                             lazy=lazy_raw)
        for k in ("ntok", "best", "cutoff", "next_cutoff"):
            np.testing.assert_array_equal(a[k], b[k], err_msg=f"stream {i} {k}")
        assert a["words"] == b["words"]
        assert a["best_cost"] == pytest.approx(b["best_cost"], abs=1e-5)
