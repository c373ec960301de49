"""The opt-in order-independent token passing (oracle.c orc_decode, the GPU's
VOSK_AMD_DEC_ORDER=parallel) against the Kaldi-sequential restatement (orc_decode_kaldi:
LatticeFasterDecoderTpl with its HashList order, running emitting cutoff and
LIFO epsilon queue).  Kaldi creates a superset of tokens (those between the
frame's final emitting cutoff and the running one); they are never expanded
while the beam decides the cutoff, so without an active-token limit the two
forms give the same 1-best.  With min_active / max_active the extra tokens
enter Kaldi's nth_element and the searches diverge: the opt-in form's
tolerance is asserted here on the synthetic model (flat
random-nnet scores, the hard case).  The GPU's default is the Kaldi order
itself (tests/test_kaldi_order_gpu.py)."""
import numpy as np
import pytest

from conftest import perturbed_stream
import oracle_py

N, SECS = 16, 10.0


def _ed(a, b):
    d = list(range(len(b) + 1))
    for i in range(1, len(a) + 1):
        prev, d[0] = d[0], i
        for j in range(1, len(b) + 1):
            cur = d[j]
            d[j] = min(d[j] + 1, d[j - 1] + 1, prev + (a[i - 1] != b[j - 1]))
            prev = cur
    return d[len(b)]


@pytest.fixture(scope="module")
def llhs(synth_model, test_wave):
    o = oracle_py.OracleModel(synth_model, fpc=51)
    return o, [o.loglikes(perturbed_stream(test_wave, 7000 + i, seconds=SECS)) for i in range(N)]


def test_same_one_best_without_active_limits(llhs):
    o, ls = llhs
    for llh in ls:
        a = o.graph.decode(llh, o.beam, 2 ** 31 - 1, 0, o.beam_delta, True, kaldi=False)
        b = o.graph.decode(llh, o.beam, 2 ** 31 - 1, 0, o.beam_delta, True, kaldi=True)
        assert a["words"] == b["words"]
        assert a["best_cost"] == pytest.approx(b["best_cost"], rel=1e-6)
        assert (b["ntok"] >= a["ntok"]).all()  # Kaldi's superset


def test_stated_tolerance_with_active_limits(llhs):
    o, ls = llhs
    same = errs = words = 0
    rel = []
    for llh in ls:
        a = o.graph.decode(llh, o.beam, o.max_active, o.min_active, o.beam_delta, True, kaldi=False)
        b = o.graph.decode(llh, o.beam, o.max_active, o.min_active, o.beam_delta, True, kaldi=True)
        same += a["words"] == b["words"]
        errs += _ed(b["words"], a["words"])
        words += len(b["words"])
        rel.append(abs(a["best_cost"] - b["best_cost"]) / abs(b["best_cost"]))
    # >= 65 % identical 1-best, <= 10 % WER between the
    # forms, best-path costs within 5 % (synthetic flat-score model)
    assert same / N >= 0.65, same
    assert errs / words <= 0.10, (errs, words)
    assert max(rel) <= 0.05, max(rel)
