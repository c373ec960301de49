"""The KaldiRecognizer's incremental lattice (csrc/incremental.{h,cc}: Kaldi's
LatticeIncrementalDecoder PruneActiveTokens schedule, UpdateLatticeDeterminization
and LatticeIncrementalDeterminizer; src/recognizer.cc:39-43, 678, 740-752)
against its restatement (tests/oracle_incremental.py) on the oracle decoder's
records of the synthetic models: the same chunk sequence, the same partial
lattice after every AdvanceDecoding of a 0.25-s-call stream, the same final
lattice, arc for arc and bit for bit.  CPU only (host-only ABI)."""
import numpy as np
import pytest

import oracle_incremental as OI
import oracle_lattice as OL
import oracle_py
from conftest import perturbed_stream

F32 = np.float32


def _records(model, wave, max_active=None):
    o = oracle_py.OracleModel(model)
    llh = o.loglikes(wave)
    ma = o.max_active if max_active is None else max_active
    r = o.graph.decode(llh, o.beam, ma, o.min_active, o.beam_delta, True, lattice=True, kaldi=True)
    return o, OI.frames_from_oracle(r, o.graph)


def _events(nframes, step=7, repeat_every=5):
    """AdvanceDecoding ends of a 0.2-s-piece recognizer (7 frames per chunk,
    some advances without a new chunk), a partial query after each, the
    final lattice at the end."""
    ev, d, i = [], 0, 0
    while d < nframes - 1:
        d = min(d + step, nframes - 1)
        ev.append((0, d))
        if i % repeat_every == 0:
            ev.append((0, d))  # an advance that decoded nothing (a 0.05 s piece)
        ev.append((1, None))
        i += 1
    ev.append((2, None))
    return ev


def _python(o, frames, events):
    inc = OI.IncrementalLattice(o.graph, o.tm.tid2phone, OL.tid_first(o.tm))
    out = []
    for t, a in events:
        if t == 0:
            while inc.num_decoded() < a:
                k = inc.num_decoded() + 1
                inc.add_frame(*frames[k][:2], frames[k][2], frames[k][3])
            inc.advance_end()
            continue
        if t == 1:
            r = inc.get_lattice(inc.nil, False)
        else:
            inc.finalize()
            r = inc.get_lattice(inc.num_decoded(), True)
        out.append(dict(nfl=inc.nil, ok=r is not None, chunks=inc.chunks, lat=r))
    return out


def _compare(got, exp):
    assert len(got) == len(exp)
    for i, (g, e) in enumerate(zip(got, exp)):
        assert g["nfl"] == e["nfl"], i
        assert bool(g["ok"]) == e["ok"], i
        assert g["chunks"] == e["chunks"], i
        if not e["ok"]:
            continue
        W, Fi = e["lat"]
        assert len(g["arcs"]) == len(W), i
        for s, (ga, ea) in enumerate(zip(g["arcs"], W)):
            assert [(a[0], a[1], a[4]) for a in ga] == [(a[0], a[1], list(a[4])) for a in ea], (i, s)
            assert [F32(a[2]) for a in ga] == [F32(a[2]) for a in ea], (i, s)
            assert [F32(a[3]) for a in ga] == [F32(a[3]) for a in ea], (i, s)
        for s, (gf, ef) in enumerate(zip(g["finals"], Fi)):
            assert (gf is None) == (ef is None), (i, s)
            if ef is not None:
                assert (F32(gf[0]), F32(gf[1]), gf[2]) == (F32(ef[0]), F32(ef[1]), list(ef[2])), (i, s)


@pytest.mark.parametrize("secs,seed", [(8.3, None), (12.0, 5)])
def test_incremental_lattice_matches_restatement(synth_model, test_wave, secs, seed):
    from vosk import engine
    wave = test_wave[:int(16000 * secs)] if seed is None else perturbed_stream(test_wave, seed, seconds=secs)
    o, frames = _records(synth_model, wave)
    events = _events(len(frames))
    exp = _python(o, frames, events)
    engine.set_phones(o.tm.tid2phone, OL.tid_first(o.tm))
    try:
        got = engine.incremental_lattice(frames, o.graph, events)
    finally:
        engine.set_phones(None)
    _compare(got, exp)
    # the schedule did what the reference's does: several chunks, partial
    # lattices only once the first chunk exists, all frames in the final one
    nfl = [e["nfl"] for e in exp]
    assert exp[-1]["chunks"] >= 3 and nfl[-1] == len(frames) - 1
    assert nfl[0] == 0 and max(nfl[:-1]) > 0
    assert nfl == sorted(nfl)  # (the start over from frame 0 of a silent start keeps this too)


def test_incremental_final_equals_one_shot_words(synth_model, test_wave):
    """What incremental determinization preserves: after FinalizeDecoding the
    appended chunks hold the lattice's best path -- its MBR words equal the
    one-shot pipeline's (src/batch_recognizer.cc's GetLattice) on a clean
    utterance."""
    o, frames = _records(synth_model, test_wave)
    exp = _python(o, frames, _events(len(frames)))
    W, Fi = exp[-1]["lat"]
    one = OL.results(o, o.loglikes(test_wave), graph_scale=1.0, kaldi=True)["mbr"]
    assert OL.mbr(W, Fi)["words"] == one["words"]


def test_chunk_choice_fewest_tokens(synth_model, test_wave):
    """UpdateLatticeDeterminization: the first chunk ends at the frame with the
    fewest tokens (after pruning) among [min_chunk, decoded], later on ties."""
    o, frames = _records(synth_model, test_wave)
    inc = OI.IncrementalLattice(o.graph, o.tm.tid2phone, OL.tid_first(o.tm))
    for k in range(0, 61):
        inc.add_frame(*frames[k][:2], frames[k][2], frames[k][3])
    inc.prune_active(inc.delta)
    counts = [inc.frames[t][4] for t in range(20, 61)]
    want = 20 + max(i for i, c in enumerate(counts) if c == min(counts))
    inc2 = OI.IncrementalLattice(o.graph, o.tm.tid2phone, OL.tid_first(o.tm))
    for k in range(0, 61):
        inc2.add_frame(*frames[k][:2], frames[k][2], frames[k][3])
    inc2.advance_end()
    assert inc2.nil == want
