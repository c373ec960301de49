"""GPU lattice generation: the decoder's forward links (kept in HBM per
stream) rebuilt into the state-level lattice must equal the oracle's
(LatticeFasterDecoder tokens and links, order-independent formulation) for
every frame: the same tokens with the same costs, the same links with the
same graph and acoustic costs.  Exercises the LDS frame table, the HBM
overflow tables and a mix of both in every frame, and a wide-beam model."""
import numpy as np
import pytest

import oracle_py
from lattice_util import canon_engine, canon_oracle

pytestmark = pytest.mark.gpu

FRAME_PATHS = {"default": None, "hbm": "0", "mixed": "1"}


@pytest.fixture(autouse=True)
def no_pruning(monkeypatch):
    """Frame-by-frame raw lattices are compared: PruneActiveTokens off (its
    effect, nothing after the lattice-beam prune, is tested in
    test_decoder_prune_gpu.py)."""
    monkeypatch.setenv("VOSK_AMD_DEC_PRUNE", "0")


@pytest.fixture(params=sorted(FRAME_PATHS))
def frame_path(request, monkeypatch):
    v = FRAME_PATHS[request.param]
    if v is None:
        monkeypatch.delenv("VOSK_AMD_DEC_LDS_PROBE", raising=False)
    else:
        monkeypatch.setenv("VOSK_AMD_DEC_LDS_PROBE", v)
    return request.param


def _check(model, llh, use_final=True):
    from vosk import engine
    o = oracle_py.OracleModel(model)
    r = o.graph.decode(llh, o.beam, o.max_active, o.min_active, o.beam_delta, use_final, lattice=True)
    e = engine.Engine(model, max_streams=2, lattice=True)
    s = e.new_stream()
    e.decode_llh(s, llh, reset=True)
    L = e.lattice(s, use_final)
    assert not L["overflow"]
    assert L["num_frames"] == llh.shape[0]
    gt, gl = canon_engine(L)
    rt, rl = canon_oracle(r, o.graph)
    assert len(gt) == len(rt)
    for k in range(len(rt)):
        assert gt[k] == rt[k], f"tokens differ at frame {k}"
        assert gl[k] == rl[k], f"links differ at frame {k}"
    # final costs of the last frame's tokens (graph finals when any is final)
    last = L["tok_state"][L["frame_begin"][-2]:L["frame_begin"][-1]]
    fin = o.graph.final[last]
    if use_final and np.isfinite(fin).any():
        np.testing.assert_array_equal(L["final_cost"], fin)
    else:
        assert len(L["final_cost"]) == 0
    return L


def test_lattice_matches_oracle(synth_model, test_wave, frame_path):
    o = oracle_py.OracleModel(synth_model)
    llh = o.loglikes(test_wave)
    L = _check(synth_model, llh)
    assert len(L["link_arc"]) > len(L["tok_state"]) // 2


def test_lattice_wide_beam(synth_model_wide, test_wave, frame_path):
    o = oracle_py.OracleModel(synth_model_wide)
    llh = o.loglikes(test_wave[:16000 * 3])
    _check(synth_model_wide, llh)


def test_lattice_streaming_matches_oracle(synth_model, test_wave):
    """Through the streaming engine (MFCC -> nnet -> decoder in steps)."""
    from vosk import engine
    o = oracle_py.OracleModel(synth_model, fpc=51)
    llh = o.loglikes(test_wave)
    r = o.graph.decode(llh, o.beam, o.max_active, o.min_active, o.beam_delta, False, lattice=True)
    e = engine.Engine(synth_model, frames_per_chunk=51, max_streams=2, lattice=True)
    s = e.new_stream()
    for i in range(0, len(test_wave), 8160):
        e.accept(s, test_wave[i:i + 8160])
        e.advance([s])
    e.accept(s, np.zeros(0, np.float32), finished=True)
    e.advance([s])
    L = e.lattice(s, use_final=False)
    gt, gl = canon_engine(L)
    rt, rl = canon_oracle(r, o.graph)
    assert gt == rt and gl == rl
