"""The decoder in the product's configuration (Kaldi order with lattices on:
the emitting pass's running cutoff by decoupled look-back, deferred winners
and creation ranks) is a function of each stream's
log-likelihoods only, whatever else runs on the GPU.

Many copies of a few streams are decoded in one engine, in order and
pipelined: every copy of a stream must give the same per-frame token counts,
best costs, cutoffs, 1-best and lattice records, and each distinct stream
must equal the Kaldi-order oracle (orc_decode_kaldi,
LatticeFasterDecoderTpl restated; src/recognizer.cc:39-43,
src/batch_model.cc:78-80) frame by frame.  test_kaldi_order_gpu.py checks
the same equality with lattices off (the barrier form of the running
cutoff); a race between the waves of one workgroup in the look-back form
would show here as copies that disagree."""
import multiprocessing as mp
import os

import numpy as np
import pytest

import oracle_py
from conftest import perturbed_stream

pytestmark = pytest.mark.gpu

_ORC = {}
LAT_KEYS = ("frame_begin", "tok_state", "tok_cost", "link_src", "link_dst", "link_arc", "link_graph",
            "link_ac", "final_cost")


def _orc_job(i):
    o = _ORC["o"]
    r = o.graph.decode(_ORC["llh"][i], o.beam, o.max_active, o.min_active, o.beam_delta, True, kaldi=True)
    return dict(ntok=r["ntok"], best=r["best"], cutoff=r["cutoff"], next_cutoff=r["next_cutoff"],
                path=r["path"])


def _oracle(model_dir, llhs):
    o = oracle_py.OracleModel(model_dir, fpc=51)
    _ORC.update(o=o, llh=llhs)
    workers = max(1, min(16, len(os.sched_getaffinity(0))))
    with mp.get_context("fork").Pool(workers) as pool:
        res = pool.map(_orc_job, range(len(llhs)), chunksize=1)
    _ORC.clear()
    return res


def _decode(model_dir, waves, pipeline):
    from vosk import engine
    e = engine.Engine(model_dir, frames_per_chunk=51, max_streams=len(waves), stats=True, keep_llh=True,
                      lattice=True, pipeline=pipeline)
    ss = [e.new_stream() for _ in waves]
    for s, w in zip(ss, waves):
        e.accept(s, w, finished=True)
    e.advance(ss)
    out = []
    for s in ss:
        st = e.decoder_state(s)
        assert st["err"] == 0, st
        L = e.lattice(s, True)
        assert not L["overflow"]
        out.append(dict(stats=e.stats(s), llh=e.llh(s), path=e.best_path(s, use_final=True)[0],
                        lat={k: L[k] for k in LAT_KEYS}))
    e.close()
    return out


def _same(a, b, what):
    np.testing.assert_array_equal(a["llh"], b["llh"], err_msg=f"{what}: log-likelihoods")
    np.testing.assert_array_equal(a["stats"][:, [1, 4, 5, 6]], b["stats"][:, [1, 4, 5, 6]],
                                  err_msg=f"{what}: per-frame tokens / best / cutoffs")
    np.testing.assert_array_equal(a["path"], b["path"], err_msg=f"{what}: 1-best")
    for k in LAT_KEYS:
        np.testing.assert_array_equal(a["lat"][k], b["lat"][k], err_msg=f"{what}: lattice {k}")


@pytest.mark.parametrize("pipeline", [False, True], ids=["in_order", "pipelined"])
def test_copies_agree_and_equal_oracle(synth_la_small_en_us, test_wave, monkeypatch, pipeline):
    """256 streams = 16 distinct streams x 16 copies on the small-en-us-scale
    lookahead model (thousands of tokens per frame, max-active engaged)."""
    import oracle_graph as OG
    monkeypatch.delenv("VOSK_AMD_DEC_ORDER", raising=False)
    distinct = [perturbed_stream(test_wave, 7100 + i, seconds=3.0 + 0.1 * i) for i in range(16)]
    waves = [distinct[k % 16] for k in range(256)]
    gpu = _decode(synth_la_small_en_us, waves, pipeline)
    for k in range(16, 256):
        _same(gpu[k], gpu[k % 16], f"stream {k} vs its copy {k % 16}")
    out = synth_la_small_en_us.rstrip("/") + "_oracle_hclg"
    if not os.path.exists(os.path.join(out, "graph", "lazy_ids.npz")):
        OG.expanded_hclg_model(synth_la_small_en_us, out + ".tmp")
        __import__("shutil").rmtree(out, ignore_errors=True)
        os.rename(out + ".tmp", out)
    ref = _oracle(out, [g["llh"] for g in gpu[:16]])
    for k, (g, r) in enumerate(zip(gpu[:16], ref)):
        st = g["stats"]
        np.testing.assert_array_equal(st[:, 1].astype(np.int64), r["ntok"][1:], err_msg=f"stream {k} tokens")
        np.testing.assert_array_equal(st[:, 4], r["best"][1:], err_msg=f"stream {k} best costs")
        np.testing.assert_array_equal(st[:, 5], r["cutoff"], err_msg=f"stream {k} cutoffs")
        np.testing.assert_array_equal(st[:, 6], r["next_cutoff"], err_msg=f"stream {k} next cutoffs")
        np.testing.assert_array_equal(g["path"], r["path"], err_msg=f"stream {k} 1-best")
