"""Expected BatchRecognizer results from the oracle (TEST INFRASTRUCTURE
ONLY): per stream, the decoder segments of the batch path's endpointing
(oracle_endpoint.batch_segments_fast: the engine's chunk schedule, the rules
after every chunk; reset_on_endpoint, src/batch_model.cc:72) and each
segment's MBR words and times (oracle_lattice.results; PushLattice,
src/batch_recognizer.cc:43-107)."""
import json

import numpy as np
import pytest

import oracle_endpoint as OE
import oracle_lattice as OL
import oracle_py


def expected(model_dir, waves):
    from vosk import engine
    info = engine.plan_info(model_dir, 51)
    o = oracle_py.OracleModel(model_dir, fpc=51)
    kaldi = oracle_py.decoder_order(batch=True) == "kaldi"
    out = []
    for w in waves:
        llh = o.loglikes(w)
        states = []  # the stream's lazy numbering at each segment's start
        segs = OE.batch_segments_fast(o, w, llh, info["right_context"], info["priming"], kaldi=kaldi,
                                      lazy_states=states)
        res = []
        for (s0, s1), ls in zip(segs, states):
            mb = OL.results(o, llh[s0:s1], kaldi=kaldi, lazy_state=ls)["mbr"]
            res.append(dict(text=" ".join(o.words[x] for x in mb["words"]), start=s0 * 0.03,
                            times=[(np.floor(a + 0.5) * 0.03, np.floor(b + 0.5) * 0.03) for a, b in mb["times"]]))
        out.append(res)
    return out


def check(results, exp, what=""):
    """results: one stream's result messages (JSON strings or dicts) in order."""
    results = [json.loads(r) if isinstance(r, str) else r for r in results]
    assert len(results) == len(exp), (what, [r["text"] for r in results], [e["text"] for e in exp])
    for k, (r, e) in enumerate(zip(results, exp)):
        assert r["text"] == e["text"], (what, k, r["text"], e["text"])
        for w, (tb, te) in zip(r.get("result", []), e["times"]):
            assert w["start"] == pytest.approx(e["start"] + tb, abs=1e-4), (what, k)
            assert w["end"] == pytest.approx(e["start"] + te, abs=1e-4), (what, k)
