"""GPU parity: HIP kernels (through libvosk.so's engine ABI) vs the CPU oracle.

Bit-exact contract (see oracle/oracle.h): MFCC features, nnet3
log-likelihoods, per-frame decoder statistics and the best path are compared
with exact equality; path costs are compared exactly as well.
"""
import numpy as np
import pytest

from conftest import perturbed_stream
import oracle_py

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def oracle(synth_model):
    return oracle_py.OracleModel(synth_model)


_ORACLES = {}


def _oracle_fpc(model, fpc):
    """Oracle with the engine's chunk size (one i-vector per chunk)."""
    if (model, fpc) not in _ORACLES:
        _ORACLES[(model, fpc)] = oracle_py.OracleModel(model, fpc=fpc)
    return _ORACLES[(model, fpc)]


def _engine(model, fpc=0, streams=8, stats=True, llh=True):
    from vosk import engine
    return engine.Engine(model, frames_per_chunk=fpc, max_streams=streams, stats=stats,
                         keep_llh=llh)


def _feed(e, s, wave, chunk=3200, finish=True):
    for i in range(0, len(wave), chunk):
        e.accept(s, wave[i:i + chunk])
        e.advance([s])
    if finish:
        e.accept(s, np.zeros(0, np.float32), finished=True)
        e.advance([s])


def test_mfcc_bit_exact(synth_model, oracle, test_wave):
    e = _engine(synth_model)
    s = e.new_stream()
    e.accept(s, test_wave[:16000 * 2])
    e.advance([s])
    ref = oracle.features(test_wave[:16000 * 2])
    n = ref.shape[0]
    got = e.features(s, 0, min(n, 64), ref.shape[1])
    np.testing.assert_array_equal(got, ref[:got.shape[0]])
    got2 = e.features(s, n - 64, 64, ref.shape[1])
    np.testing.assert_array_equal(got2, ref[n - 64:])


@pytest.mark.parametrize("fpc", [51, 21])
def test_llh_bit_exact(synth_model, oracle, test_wave, fpc):
    e = _engine(synth_model, fpc=fpc)
    s = e.new_stream()
    _feed(e, s, test_wave)
    llh = e.llh(s)
    ref = _oracle_fpc(synth_model, fpc).loglikes(test_wave)
    assert llh.shape == ref.shape, (llh.shape, ref.shape)
    np.testing.assert_array_equal(llh, ref)


@pytest.mark.parametrize("fpc,chunk", [(51, 3200), (21, 3200), (51, 480), (21, 100000)])
def test_ivectors_bit_exact(synth_model, test_wave, fpc, chunk):
    """Online i-vectors (CMVN -> LDA -> UBM posteriors -> stats -> CG), one
    per chunk, identical to the oracle whatever the feeding granularity."""
    o = _oracle_fpc(synth_model, fpc)
    e = _engine(synth_model, fpc=fpc)
    s = e.new_stream()
    _feed(e, s, test_wave, chunk=chunk)
    got = e.ivectors(s)
    ref = o.ivectors(o.features(test_wave))
    assert got.shape == ref.shape, (got.shape, ref.shape)
    np.testing.assert_array_equal(got, ref)


# decoder frame construction: LDS table with HBM overflow (default), every
# state in the HBM tables, and one LDS bucket per state (states split between
# LDS and HBM in every frame)
FRAME_PATHS = {"default": None, "hbm": "0", "mixed": "1"}


@pytest.fixture(params=sorted(FRAME_PATHS))
def frame_path(request, monkeypatch):
    v = FRAME_PATHS[request.param]
    if v is None:
        monkeypatch.delenv("VOSK_AMD_DEC_LDS_PROBE", raising=False)
    else:
        monkeypatch.setenv("VOSK_AMD_DEC_LDS_PROBE", v)
    return request.param


def test_decoder_from_oracle_llh(synth_model, oracle, test_wave, frame_path):
    ref_llh = oracle.loglikes(test_wave)
    r = oracle.decode_llh(ref_llh)
    e = _engine(synth_model)
    s = e.new_stream()
    e.decode_llh(s, ref_llh, reset=True)
    st = e.stats(s)
    assert st.shape[0] == ref_llh.shape[0]
    np.testing.assert_array_equal(st[:, 1].astype(int), r["ntok"][1:])
    np.testing.assert_array_equal(st[:, 4], r["best"][1:])
    np.testing.assert_array_equal(st[:, 5], r["cutoff"])
    np.testing.assert_array_equal(st[:, 6], r["next_cutoff"])
    arcs, cost, frel = e.best_path(s, use_final=True)
    np.testing.assert_array_equal(arcs, r["path"])
    assert cost == pytest.approx(r["best_cost"], abs=1e-6)


def test_decoder_wide_beam_all_paths(synth_model_wide, test_wave, frame_path):
    """Thousands of tokens per frame (more than the LDS table holds): the HBM
    overflow tables give the oracle's best path and statistics."""
    import oracle_py
    ow = oracle_py.OracleModel(synth_model_wide)
    llh = ow.loglikes(test_wave[:64000])
    r = ow.decode_llh(llh)
    assert r["ntok"].max() > 3000  # the table capacity is exceeded somewhere
    e = _engine(synth_model_wide)
    s = e.new_stream()
    e.decode_llh(s, llh, reset=True)
    st = e.stats(s)
    np.testing.assert_array_equal(st[:, 1].astype(np.int64), r["ntok"][1:])
    arcs, _, _ = e.best_path(s, use_final=True)
    np.testing.assert_array_equal(arcs, r["path"])


def test_end_to_end_single_stream(synth_model, oracle, test_wave):
    e = _engine(synth_model)
    s = e.new_stream()
    _feed(e, s, test_wave)
    r = oracle.recognize(test_wave)
    arcs, cost, _ = e.best_path(s, use_final=True)
    np.testing.assert_array_equal(arcs, r["path"])
    assert e.frames_decoded(s) == len(r["ntok"]) - 1
    assert e.error(s) == 0


def test_batched_streams_match_oracle(synth_model, test_wave, frame_path):
    """Eight different streams advanced together in the same batched steps."""
    oracle = _oracle_fpc(synth_model, 51)
    n = 8
    e = _engine(synth_model, fpc=51, streams=n, stats=False, llh=True)
    waves = [perturbed_stream(test_wave, i, seconds=3.0 + 0.37 * i) for i in range(n)]
    ss = [e.new_stream() for _ in range(n)]
    chunk = 8000
    pos = [0] * n
    while any(p < len(w) for p, w in zip(pos, waves)):
        for k in range(n):
            if pos[k] < len(waves[k]):
                e.accept(ss[k], waves[k][pos[k]:pos[k] + chunk])
                pos[k] += chunk
        e.advance(ss)
    for k in range(n):
        e.accept(ss[k], np.zeros(0, np.float32), finished=True)
    e.advance(ss)
    for k in range(n):
        feats = oracle.features(waves[k])
        np.testing.assert_array_equal(e.ivectors(ss[k]), oracle.ivectors(feats),
                                      err_msg=f"ivectors {k}")
        np.testing.assert_array_equal(e.llh(ss[k]), oracle.loglikes_feats(feats), err_msg=f"llh {k}")
        r = oracle.recognize(waves[k])
        arcs, _, _ = e.best_path(ss[k], use_final=True)
        np.testing.assert_array_equal(arcs, r["path"], err_msg=f"stream {k}")


def test_pipelined_steps_match_oracle(synth_model, test_wave):
    """Two-stream pipeline (bench.py's mode): HBM-preloaded audio, one chunk
    per stream per step, the decoder of step i-1 beside the nnet of step i;
    transcripts and every decoded LLH row identical to the oracle."""
    from vosk import engine
    oracle = _oracle_fpc(synth_model, 51)
    n = 6
    e = engine.Engine(synth_model, frames_per_chunk=51, max_streams=n, keep_llh=True,
                      pipeline=True)
    e.set_step_samples(51 * 160)
    waves = [perturbed_stream(test_wave, i, seconds=2.5 + 0.41 * i) for i in range(n)]
    ss = [e.new_stream() for _ in range(n)]
    for s, w in zip(ss, waves):
        e.preload(s, w, finished=True)
    steps = 0
    while e.step(ss):
        steps += 1
        assert steps < 1000
    for k in range(n):
        r = oracle.recognize(waves[k])
        np.testing.assert_array_equal(e.llh(ss[k]), oracle.loglikes(waves[k]), err_msg=f"llh {k}")
        arcs, _, _ = e.best_path(ss[k], use_final=True)
        np.testing.assert_array_equal(arcs, r["path"], err_msg=f"stream {k}")


@pytest.mark.parametrize("nsamples", [0, 100, 399, 400, 1000, 16000])
def test_short_inputs(synth_model, oracle, test_wave, nsamples):
    e = _engine(synth_model)
    s = e.new_stream()
    w = test_wave[:nsamples]
    _feed(e, s, w)
    nf = oracle.features(w).shape[0] if nsamples else 0
    expect_frames = (nf + 2) // 3
    assert e.frames_decoded(s) == expect_frames
    if expect_frames:
        r = oracle.recognize(w)
        arcs, _, _ = e.best_path(s, use_final=True)
        np.testing.assert_array_equal(arcs, r["path"])


def test_decoder_reset_continues_frames(synth_model, oracle, test_wave):
    """InitDecoding mid-stream: the nnet continues, the decoder restarts."""
    e = _engine(synth_model)
    s = e.new_stream()
    half = len(test_wave) // 2
    _feed(e, s, test_wave[:half], finish=False)
    f1 = e.frames_decoded(s)
    e.reset(s, pipeline=False)
    _feed(e, s, test_wave[half:])
    llh = e.llh(s)
    ref = oracle.loglikes(test_wave)
    np.testing.assert_array_equal(llh, ref)
    r = oracle.decode_llh(ref[f1:])
    arcs, _, _ = e.best_path(s, use_final=True)
    np.testing.assert_array_equal(arcs, r["path"])


def test_pipeline_reset_restarts(synth_model, oracle, test_wave):
    e = _engine(synth_model)
    s = e.new_stream()
    _feed(e, s, test_wave[:20000])
    e.reset(s, pipeline=True)
    w = test_wave[30000:70000]
    _feed(e, s, w)
    r = oracle.recognize(w)
    arcs, _, _ = e.best_path(s, use_final=True)
    np.testing.assert_array_equal(arcs, r["path"])
