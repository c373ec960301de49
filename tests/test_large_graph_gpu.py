"""Large decoding graphs at batch scale (BASELINE configs 3 and 4; SURVEY.md
A10/A11): 64 streams decoded together through the pipelined engine with
lattices (and PruneActiveTokens) on

* a 2.4 M-state static HCLG (config 4's per-GPU share of a large model), and
* the ~275 k-state static expansion (label pushing merges histories) of a
  vosk-model-small-en-us-scale
  lookahead model (config 3's model),

both with flat enough scores that max-active 7000 engages (the oracle sees
frames with far more than 7000 tokens).  Every stream's best path equals the
C oracle's on the same graph.  A 60 s stream without an endpoint keeps a
bounded arena and never sets an error.
"""
import multiprocessing as mp
import os

import numpy as np
import pytest

import oracle_py
from conftest import perturbed_stream

pytestmark = pytest.mark.gpu

NSTREAMS = 64
SECS = 5.0
_ORC = {}


def _orc_job(i):
    r = _ORC["o"].recognize(_ORC["waves"][i])
    return r["path"], int(r["ntok"].max())


def _oracle_paths(oracle_dir, waves):
    o = oracle_py.OracleModel(oracle_dir, fpc=51)  # the engine's chunking (i-vector per chunk)
    _ORC.update(o=o, waves=waves)
    workers = max(1, min(16, len(os.sched_getaffinity(0))))
    with mp.get_context("fork").Pool(workers) as pool:
        res = pool.map(_orc_job, range(len(waves)))
    _ORC.clear()
    return res, o.max_active


def _expanded_model(model_dir, out_dir):
    import oracle_graph as OG
    return OG.expanded_hclg_model(model_dir, out_dir)


def _batch_decode(model_dir, test_wave):
    from vosk import engine
    waves = [perturbed_stream(test_wave, 100 + i, seconds=SECS + 0.05 * i) for i in range(NSTREAMS)]
    # pruning passes at Kaldi's interval (the default schedule would not run
    # them on these short streams; the best paths must not depend on them)
    old = os.environ.get("VOSK_AMD_DEC_PRUNE")
    os.environ["VOSK_AMD_DEC_PRUNE"] = "1"
    try:
        e = engine.Engine(model_dir, frames_per_chunk=51, max_streams=NSTREAMS, pipeline=True, lattice=True)
    finally:
        if old is None:
            os.environ.pop("VOSK_AMD_DEC_PRUNE")
        else:
            os.environ["VOSK_AMD_DEC_PRUNE"] = old
    e.set_step_samples(51 * 160)
    ss = [e.new_stream() for _ in range(NSTREAMS)]
    for s, w in zip(ss, waves):
        e.preload(s, w, finished=True)
    steps = 0
    while e.step(ss):
        steps += 1
        assert steps < 2000
    out = []
    for s in ss:
        st = e.decoder_state(s)
        assert st["err"] == 0 and st["lat_ovf"] == 0, st
        assert st["last_prune"] > 0
        out.append(e.best_path(s, use_final=True)[0])
    e.close()
    return waves, out


def test_static_hclg_2m_states_64_streams(synth_bigram_2m, test_wave):
    waves, paths = _batch_decode(synth_bigram_2m, test_wave)
    ref, max_active = _oracle_paths(synth_bigram_2m, waves)
    for k in range(NSTREAMS):
        np.testing.assert_array_equal(paths[k], ref[k][0], err_msg=f"stream {k}")
    assert max(r[1] for r in ref) > max_active  # max-active engaged


def test_lookahead_expansion_64_streams(synth_la_small_en_us, test_wave, tmp_path):
    odir, S = _expanded_model(synth_la_small_en_us, str(tmp_path / "la_hclg"))
    assert S > 200_000
    waves, paths = _batch_decode(synth_la_small_en_us, test_wave)
    ref, max_active = _oracle_paths(odir, waves)
    for k in range(NSTREAMS):
        np.testing.assert_array_equal(paths[k], ref[k][0], err_msg=f"stream {k}")
    assert max(r[1] for r in ref) > max_active


def test_60s_stream_without_endpoint_stays_bounded(synth_bigram_2m, test_wave):
    """One decoder segment of 60 s (2000 frames, thousands of tokens per
    frame): pruning keeps the arena and link arena bounded and nothing
    overflows; the best path equals the oracle's.  (The default schedule
    starts the passes at 300 frames, engine.cc.)"""
    from vosk import engine
    w = perturbed_stream(test_wave, 4242, seconds=60.0)
    e = engine.Engine(synth_bigram_2m, frames_per_chunk=51, max_streams=2, lattice=True)
    s = e.new_stream()
    e.preload(s, w, finished=True)
    while e.step([s]):
        pass
    st = e.decoder_state(s)
    assert st["err"] == 0 and st["lat_ovf"] == 0, st
    assert st["frames"] >= 1990
    # ~2000 frames of several thousand tokens each without pruning
    assert st["last_prune"] > 0, st
    assert st["arena_used"] < 1_000_000 and st["links_used"] < 2_000_000, st
    o = oracle_py.OracleModel(synth_bigram_2m, fpc=51)
    r = o.recognize(w)
    np.testing.assert_array_equal(e.best_path(s, use_final=True)[0], r["path"])
