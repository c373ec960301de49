"""PruneActiveTokens on the GPU (decoder.hip prune_segment; Kaldi
LatticeFasterDecoder prunes every prune_interval frames).

Pruning only drops links and tokens whose extra cost already exceeds the
lattice beam, and extra costs only grow as the frontier advances, so the
lattice a result is built from -- the raw lattice after the exact
lattice-beam prune -- must be identical with and without it, and so must the
best path; what changes is the arena, which stays bounded.  Without a
lattice the same compaction keeps the frontier's backpointer chains only.
"""
import numpy as np
import pytest

import oracle_lattice as OL
import oracle_py
from conftest import perturbed_stream
from lattice_util import canon_engine

pytestmark = pytest.mark.gpu


def _decode(model, llh, prune, lattice, monkeypatch):
    from vosk import engine
    monkeypatch.setenv("VOSK_AMD_DEC_PRUNE", "1" if prune else "0")
    e = engine.Engine(model, max_streams=2, lattice=lattice)
    s = e.new_stream()
    e.decode_llh(s, llh, reset=True)
    return e, s


def _words(L, o):
    from vosk import engine
    return engine.lattice_words(L, o.graph.ilabel, o.graph.olabel, 6.0, 0.9, 5)


@pytest.mark.parametrize("model_fx", ["synth_model", "synth_model_wide"])
def test_pruned_lattice_gives_the_same_results(model_fx, request, test_wave, monkeypatch):
    model = request.getfixturevalue(model_fx)
    o = oracle_py.OracleModel(model)
    wave = perturbed_stream(test_wave, 5, seconds=12.0 if model_fx == "synth_model" else 4.0)
    llh = o.loglikes(wave)
    e0, s0 = _decode(model, llh, False, True, monkeypatch)
    e1, s1 = _decode(model, llh, True, True, monkeypatch)
    st0, st1 = e0.decoder_state(s0), e1.decoder_state(s1)
    assert st1["err"] == 0 and st1["lat_ovf"] == 0
    assert st1["last_prune"] >= st1["frames"] - 25 - 17 and st1["last_prune"] > 0
    # the arena and link arena shrink ...
    assert st1["arena_used"] < st0["arena_used"] // 2, (st0, st1)
    assert st1["links_used"] < st0["links_used"] // 2, (st0, st1)
    # ... the best path, and everything derived from the pruned lattice, do not
    for uf in (True, False):
        a0, c0, f0 = e0.best_path(s0, use_final=uf)
        a1, c1, f1 = e1.best_path(s1, use_final=uf)
        np.testing.assert_array_equal(a0, a1)
        assert c0 == c1 and (f0 == f1 or (np.isnan(f0) and np.isnan(f1)))
        L0, L1 = e0.lattice(s0, uf), e1.lattice(s1, uf)
        assert not L1["overflow"]
        assert _words(L0, o) == _words(L1, o)
        # the pruned raw lattice is a subset of the unpruned one, frame by frame
        t0, l0 = canon_engine(L0)
        t1, l1 = canon_engine(L1)
        assert len(t0) == len(t1)
        for k in range(len(t0)):
            assert set(t1[k]) <= set(t0[k]), f"frame {k} tokens"
            assert set(l1[k]) <= set(l0[k]), f"frame {k} links"


def test_pruning_without_lattice_keeps_the_backpointers(synth_model_wide, test_wave, monkeypatch):
    o = oracle_py.OracleModel(synth_model_wide)
    llh = o.loglikes(perturbed_stream(test_wave, 2, seconds=5.0))
    e0, s0 = _decode(synth_model_wide, llh, False, False, monkeypatch)
    e1, s1 = _decode(synth_model_wide, llh, True, False, monkeypatch)
    st0, st1 = e0.decoder_state(s0), e1.decoder_state(s1)
    assert st1["err"] == 0
    assert st1["arena_used"] < st0["arena_used"] // 3, (st0, st1)
    r = o.decode_llh(llh)
    for uf in (True, False):
        a1, c1, _ = e1.best_path(s1, use_final=uf)
        a0, c0, _ = e0.best_path(s0, use_final=uf)
        np.testing.assert_array_equal(a0, a1)
        assert c0 == c1
    np.testing.assert_array_equal(e1.best_path(s1, use_final=True)[0], r["path"])


def test_raw_lattice_across_launches_with_pruning_matches_oracle_after_beam_prune(
        synth_model, test_wave, monkeypatch):
    """Streaming engine (17-frame launches, pruning between them) vs the
    oracle's unpruned lattice: identical results after the lattice-beam prune."""
    from vosk import engine
    monkeypatch.setenv("VOSK_AMD_DEC_PRUNE", "1")  # (Kaldi's schedule: a pass every interval)
    o = oracle_py.OracleModel(synth_model, fpc=51)
    wave = perturbed_stream(test_wave, 9, seconds=15.0)
    llh = o.loglikes(wave)
    r = o.graph.decode(llh, o.beam, o.max_active, o.min_active, o.beam_delta, False, lattice=True)
    e = engine.Engine(synth_model, frames_per_chunk=51, max_streams=2, lattice=True)
    s = e.new_stream()
    for i in range(0, len(wave), 8160):
        e.accept(s, wave[i:i + 8160])
        e.advance([s])
    e.accept(s, np.zeros(0, np.float32), finished=True)
    e.advance([s])
    st = e.decoder_state(s)
    assert st["err"] == 0 and st["last_prune"] > 0
    L = e.lattice(s, use_final=False)
    # the oracle's unpruned lattice through the same host pipeline (exact
    # lattice-beam prune, determinization, MBR, n-best)
    assert _words(L, o) == _words(OL.raw_from_oracle(r, o.graph, False), o)


def test_default_policy_prunes_only_when_an_arena_fills(synth_model, test_wave, monkeypatch):
    """The default schedule (engine.cc: a pass at the interval once the
    segment is VOSK_AMD_DEC_PRUNE_START frames long, 300, or the token or link
    arena VOSK_AMD_DEC_PRUNE_FILL percent full, 50): a 4-s stream on the
    default arenas (2 M tokens) runs none, a 1 % fill threshold runs them at
    the interval; the best path and the lattice's results equal the unpruned
    decode's either way."""
    o = oracle_py.OracleModel(synth_model)
    llh = o.loglikes(perturbed_stream(test_wave, 5, seconds=4.0))
    e0, s0 = _decode(synth_model, llh, False, True, monkeypatch)
    ref = (_words(e0.lattice(s0, True), o), e0.best_path(s0, use_final=True)[0])
    for fill, pruned in (("50", False), ("1", True)):
        monkeypatch.delenv("VOSK_AMD_DEC_PRUNE", raising=False)
        monkeypatch.setenv("VOSK_AMD_DEC_PRUNE_FILL", fill)
        from vosk import engine
        e = engine.Engine(synth_model, max_streams=2, lattice=True)
        s = e.new_stream()
        e.decode_llh(s, llh, reset=True)
        st = e.decoder_state(s)
        assert st["err"] == 0 and st["lat_ovf"] == 0
        assert (st["last_prune"] > 0) == pruned, (fill, st)
        assert _words(e.lattice(s, True), o) == ref[0]
        np.testing.assert_array_equal(e.best_path(s, use_final=True)[0], ref[1])
