"""Recovery after a decoder overflow (a relaxation that finds
no room must not leave stale per-state data behind for the slot's next
utterance).  With every state in the HBM frame table (VOSK_AMD_DEC_LDS_PROBE
0) and a token capacity (VOSK_AMD_DEC_MAX_TOKENS) between the two
utterances' token counts, utterance A overflows the table's list (entries
created but never listed for clearing); the stream is then reset and decodes
utterance B, whose frames fit: its statistics and best path equal the
oracle's, and equal those of a fresh stream."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def oracle(synth_model):
    import oracle_py
    return oracle_py.OracleModel(synth_model)


def test_reset_after_token_overflow(synth_model, oracle, test_wave, monkeypatch):
    from vosk import engine as ve
    llh_b = np.ascontiguousarray(oracle.loglikes(test_wave[:32000]), np.float32)
    llh_a = np.zeros((40, llh_b.shape[1]), np.float32)  # flat scores: thousands of tokens
    ra = oracle.decode_llh(llh_a)
    rb = oracle.decode_llh(llh_b)
    amax, bmax = int(ra["ntok"].max()), int(rb["ntok"].max())
    cap = (amax + bmax) // 2
    assert amax > cap + 100 and bmax < cap - 100
    monkeypatch.setenv("VOSK_AMD_DEC_MAX_TOKENS", str(cap))
    monkeypatch.setenv("VOSK_AMD_DEC_LDS_PROBE", "0")
    e = ve.Engine(synth_model, max_streams=2, stats=True, keep_llh=True)
    s = e.new_stream()
    e.decode_llh(s, llh_a, reset=True)
    assert e.error(s) & 1  # token list / table overflow
    e.decode_llh(s, llh_b, reset=True)  # the same slot, a new utterance
    assert e.error(s) == 0
    st = e.stats(s)
    np.testing.assert_array_equal(st[:, 1].astype(np.int64), rb["ntok"][1:])
    np.testing.assert_array_equal(st[:, 4], rb["best"][1:])
    arcs, cost, _ = e.best_path(s, use_final=True)
    np.testing.assert_array_equal(arcs, rb["path"])
    fresh = e.new_stream()
    e.decode_llh(fresh, llh_b, reset=True)
    np.testing.assert_array_equal(e.best_path(fresh, use_final=True)[0], arcs)
    e.close()
