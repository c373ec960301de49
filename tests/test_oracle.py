"""The C oracle against an independent float64 numpy restatement and against
the algorithmic invariants of Kaldi's token passing."""
import math

import numpy as np
import pytest

import np_kaldi as nk
import oracle_py


@pytest.fixture(scope="module")
def oracle(synth_model):
    return oracle_py.OracleModel(synth_model)


def test_logf_accuracy():
    lib = oracle_py.lib()
    xs = np.concatenate([np.geomspace(1.1920929e-07, 1e12, 2000), [0.5, 1.0, 2.0, math.e]])
    for x in xs.astype(np.float32):
        got = lib.orc_logf(float(x))
        ref = math.log(float(x))
        assert abs(got - ref) <= 2.5e-7 * max(1.0, abs(ref)), (x, got, ref)


def test_mfcc_vs_numpy(oracle, test_wave):
    f = oracle.features(test_wave)
    ref = nk.mfcc(test_wave.astype(np.float64), nk.MfccOpts(oracle.mfcc_conf))
    assert f.shape == ref.shape == (829, 40)
    assert np.abs(f - ref).max() <= 1e-5 * np.abs(ref).max()


def test_mfcc_frame_count_edges(oracle, test_wave):
    for n, expect in ((0, 0), (399, 0), (400, 1), (559, 1), (560, 2), (16000, 98)):
        assert oracle.features(test_wave[:n]).shape[0] == expect


def test_mfcc_is_chunking_invariant(oracle, test_wave):
    """Frames only depend on their own 25 ms window (snip-edges)."""
    full = oracle.features(test_wave[:48000])
    part = oracle.features(test_wave[16000:48000])
    np.testing.assert_array_equal(part, full[100:100 + part.shape[0]])


def _fixed_ivector(oracle):
    """One i-vector for every row (net-level tests: no extraction involved)."""
    dim = oracle.ivector.m.ivec_dim
    v = np.random.default_rng(5).normal(0, 1, (1, dim)).astype(np.float32)
    return dict(ivecs=v, ivec_of_time=np.zeros(1, np.int32), ivec_t0=0)


def test_nnet_vs_numpy(oracle, test_wave):
    feats = oracle.features(test_wave[:32000])
    iv = _fixed_ivector(oracle)
    llh = oracle.net.forward(feats, **iv)
    ref = nk.NnetGraph(oracle.nn).forward({"input": feats.astype(np.float64),
                                           "ivector_at": lambda t: iv["ivecs"][0].astype(np.float64)})
    assert llh.shape == ref.shape
    assert np.abs(llh - ref).max() <= 2e-5 * np.abs(ref).max()


def test_nnet_edge_replication(oracle, test_wave):
    """Output frame t only sees inputs t-L..t+R, replicated at the edges."""
    feats = oracle.features(test_wave[:32000])
    iv = _fixed_ivector(oracle)
    llh = oracle.net.forward(feats, **iv)
    # the middle of the utterance is unaffected by truncating far-away frames
    llh2 = oracle.net.forward(feats[60:], **iv)
    np.testing.assert_array_equal(llh2[20:50], llh[40:70])


def _path_cost(g, llh, path):
    """Recompute the best path's cost from arc weights and log-likelihoods."""
    cost, t = 0.0, 0
    for a in path:
        cost += float(g.weight[a])
        if g.ilabel[a] != 0:
            cost -= float(llh[t, g.tid2pdf[g.ilabel[a]]])
            t += 1
    return cost, t


def test_decoder_invariants(oracle, test_wave):
    llh = oracle.loglikes(test_wave)
    r = oracle.decode_llh(llh, use_final=False)
    g = oracle.graph
    cost, frames = _path_cost(g, llh, r["path"])
    assert frames == llh.shape[0]
    assert cost == pytest.approx(r["best_cost"], rel=1e-5, abs=1e-3)
    # the path is connected from the start state
    s = g.start
    for a in r["path"]:
        assert g.arc_begin[s] <= a < g.arc_begin[s + 1]
        s = g.nextstate[a]
    assert s == r["end_state"]
    assert (r["ntok"] > 0).all()
    assert (r["cutoff"] >= r["best"][:-1]).all()


def test_decoder_max_active_enforced(oracle, test_wave):
    llh = oracle.loglikes(test_wave[:48000])
    wide = oracle.graph.decode(llh, beam=40.0, max_active=100000, min_active=0)
    narrow = oracle.graph.decode(llh, beam=40.0, max_active=50, min_active=0)
    assert wide["ntok"].max() > 200
    # cutoff keeps (at most) ~max_active tokens expandable per frame
    assert narrow["ntok"].mean() < wide["ntok"].mean()
    assert narrow["best_cost"] >= wide["best_cost"] - 1e-3


def test_decoder_beam_monotone(oracle, test_wave):
    llh = oracle.loglikes(test_wave[:48000])
    costs = [oracle.graph.decode(llh, beam=b, max_active=7000)["best_cost"] for b in (4, 8, 13, 20)]
    # a wider beam never finds a worse best path
    assert all(costs[i + 1] <= costs[i] + 1e-3 for i in range(3))


def test_recognize_deterministic(oracle, test_wave):
    a = oracle.recognize(test_wave)
    b = oracle.recognize(test_wave)
    assert a["text"] == b["text"] and np.array_equal(a["path"], b["path"])
    assert len(a["words"]) > 0


@pytest.mark.parametrize("kaldi", [False, True], ids=["parallel", "kaldi"])
def test_batch_segments_fast_equals_per_chunk_decodes(synth_model_ep, test_wave, kaldi):
    """The one-pass segmentation (endpoint probes inside one decode per
    segment) equals the per-chunk re-decodes it replaces (CPU)."""
    import oracle_endpoint as OE
    from conftest import perturbed_stream
    from vosk import engine
    info = engine.plan_info(synth_model_ep, 51)
    o = oracle_py.OracleModel(synth_model_ep, fpc=51)
    nseg = 0
    for i in range(2):
        w = perturbed_stream(test_wave, 900 + i, seconds=9.0 + 0.7 * i)
        llh = o.loglikes(w)
        a = OE.batch_segments(o, w, llh, info["right_context"], info["priming"], kaldi=kaldi)
        b = OE.batch_segments_fast(o, w, llh, info["right_context"], info["priming"], kaldi=kaldi)
        assert a == b
        nseg += len(a)
    assert nseg >= 4  # the rules fire


@pytest.mark.parametrize("kaldi", [False, True], ids=["parallel", "kaldi"])
def test_decoder_probes_equal_prefix_decodes(oracle, test_wave, kaldi):
    llh = oracle.loglikes(test_wave[:16000 * 3])
    g = oracle.graph
    probes = [0, 1, 17, 50, len(llh)]
    r = g.decode(llh, use_final=False, kaldi=kaldi, probes=probes)
    for n, (path, frc) in zip(probes, r["probes"]):
        ref = g.decode(llh[:n], use_final=False, kaldi=kaldi)
        np.testing.assert_array_equal(path, ref["path"])
        assert frc == ref["final_relative_cost"] or (math.isinf(frc) and math.isinf(ref["final_relative_cost"]))
