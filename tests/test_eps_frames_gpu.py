"""Frames whose surviving tokens have no epsilon arcs, right after frames that
emitted epsilon links (the round-2 race: the commit read the frame's
epsilon-link count without a barrier after thread 0 reset it, so with no
epsilon token the threads could advance different link offsets; fixed in
1a43c6d).  A hand-built graph alternates such frames deterministically; under
the decoder's device invariant checks (VOSK_AMD_DEC_DEBUG) every stream's
lattice (tokens, costs, links per frame) equals the oracle's, with no
overflow and no error, over many streams and both frame tables."""
import os
import shutil

import numpy as np
import pytest

import kaldi_formats as kf
import oracle_py
from lattice_util import canon_engine, canon_oracle

pytestmark = pytest.mark.gpu


def _tiny_graph(tids):
    t = tids
    # state: [(ilabel, olabel, weight, nextstate)], emitting arcs first
    arcs = {
        0: [(t[0], 0, 0.5, 1), (t[1], 0, 0.7, 1), (t[0], 0, 1.0, 0)],
        1: [(t[2], 0, 0.3, 1), (0, 3, 0.2, 2), (0, 4, 0.4, 3), (0, 0, 0.1, 4)],
        2: [(t[3], 0, 0.2, 5)],
        3: [(t[4], 0, 0.3, 5), (t[3], 0, 0.1, 6)],
        4: [(t[5], 0, 0.2, 6)],
        5: [(t[6], 0, 0.1, 5), (t[7], 0, 0.4, 7)],
        6: [(t[6], 0, 0.2, 7)],
        7: [(t[7], 0, 0.3, 7), (0, 5, 0.5, 0)],
    }
    S = len(arcs)
    row = [0]
    il, ol, w, ns = [], [], [], []
    for s in range(S):
        for a in arcs[s]:
            il.append(a[0]); ol.append(a[1]); w.append(a[2]); ns.append(a[3])
        row.append(len(il))
    final = np.full(S, np.inf, np.float32)
    final[7] = 0.0
    return kf.Fst(start=0, final=final, row=np.array(row, np.int64), ilabel=np.array(il, np.int32),
                  olabel=np.array(ol, np.int32), weight=np.array(w, np.float32),
                  nextstate=np.array(ns, np.int32))


@pytest.fixture(scope="module")
def eps_model(synth_model, tmp_path_factory):
    d = str(tmp_path_factory.mktemp("eps_model") / "m")
    shutil.copytree(synth_model, d, symlinks=True)
    o = oracle_py.OracleModel(synth_model)
    t2p = o.graph.tid2pdf
    tids, pdfs = [], set()
    for tid in range(1, len(t2p)):
        if int(t2p[tid]) not in pdfs:
            tids.append(tid)
            pdfs.add(int(t2p[tid]))
        if len(tids) == 8:
            break
    kf.write_const_fst(os.path.join(d, "graph", "HCLG.fst"), _tiny_graph(tids))
    # min_active 200 would keep every token of a graph this small
    with open(os.path.join(d, "conf", "model.conf"), "a") as f:
        f.write("--min-active=1\n")
    return d, tids, t2p


def _llh(t2p, tids, frames, rng):
    P = int(t2p.max()) + 1
    llh = np.full((frames, P), -30.0, np.float32)
    for f in range(frames):
        ph = f % 4
        # phases: 0 enter 0/1 (epsilon links out of 1), 1 kill 0/1 (no epsilon
        # token survives), 2 stay in 5/6, 3 reach 7 (epsilon back to 0)
        good = {0: (0, 1, 2), 1: (3, 4, 5), 2: (6,), 3: (7, 0)}[ph]
        for k in good:
            llh[f, t2p[tids[k]]] = -1.0 + 0.3 * rng.standard_normal()
    return llh


@pytest.mark.parametrize("probe", ["default", "0"])
def test_frames_without_epsilon_tokens(eps_model, monkeypatch, probe):
    from vosk import engine
    d, tids, t2p = eps_model
    monkeypatch.setenv("VOSK_AMD_DEC_DEBUG", "1")
    monkeypatch.setenv("VOSK_AMD_DEC_PRUNE", "0")
    if probe == "default":
        monkeypatch.delenv("VOSK_AMD_DEC_LDS_PROBE", raising=False)
    else:
        monkeypatch.setenv("VOSK_AMD_DEC_LDS_PROBE", probe)
    o = oracle_py.OracleModel(d)
    e = engine.Engine(d, max_streams=4, lattice=True)
    s = e.new_stream()
    rng = np.random.default_rng(5)
    no_eps_frames = 0
    for rep in range(48):
        llh = _llh(t2p, tids, 40 + rep % 7, rng)
        r = o.graph.decode(llh, o.beam, o.max_active, o.min_active, o.beam_delta, True, lattice=True)
        e.decode_llh(s, llh, reset=True)
        assert e.error(s) == 0
        L = e.lattice(s, True)
        assert not L["overflow"]
        gt, gl = canon_engine(L)
        rt, rl = canon_oracle(r, o.graph)
        assert len(gt) == len(rt)
        for k in range(len(rt)):
            assert gt[k] == rt[k], (rep, k)
            assert gl[k] == rl[k], (rep, k)
        # frames that emit no epsilon link (no token below the cutoff has an
        # epsilon arc), right after a frame that emitted epsilon links
        neps = [sum(1 for (_, arc, _, _) in gl[k] if o.graph.ilabel[arc] == 0) for k in range(len(gl))]
        no_eps_frames += sum(1 for k in range(1, len(neps)) if neps[k] == 0 and neps[k - 1] > 0)
    assert no_eps_frames >= 48
    e.close()
