"""Final results with LM rescoring through the public API on the GPU
(src/recognizer.cc:675-729 with rescore/G.fst + rescore/G.carpa): MBR words,
confidences and times of the rescored lattice against the oracle chain
(tests/oracle_rescore.py over the oracle's online decode)."""
import json
import os

import numpy as np
import pytest

import kaldi_formats as kf
import oracle_incremental as OI
import oracle_lattice as OL  # noqa: F401
import oracle_py
import oracle_rescore as ORS

pytestmark = pytest.mark.gpu


def test_recognizer_rescored_result_matches_oracle(synth_model_rescore, test_wave):
    import vosk
    vosk.SetLogLevel(-1)
    rd = os.path.join(synth_model_rescore, "rescore")
    G = ORS.prepare_g(kf.read_fst(os.path.join(rd, "G.fst")))
    lm = ORS.ConstArpa(os.path.join(rd, "G.carpa"))
    oracle = oracle_py.OracleModel(synth_model_rescore)
    m = vosk.Model(synth_model_rescore)
    for wave in (test_wave, test_wave[:40000]):
        rec = vosk.KaldiRecognizer(m, 16000)
        rec.SetWords(True)
        data = np.asarray(wave, np.float32).astype("<i2").tobytes()
        for i in range(0, len(data), 8000):
            assert rec.AcceptWaveform(data[i:i + 8000]) == 0
        final = json.loads(rec.FinalResult())
        on = oracle.online(wave, chunk=4000)
        resc = lambda W, Fi: ORS.rescore(W, Fi, G, lm)  # noqa: E731
        mb = OI.final_result(oracle, wave, 4000, rescore=resc, on=on)["mbr"]
        assert final["text"] == " ".join(oracle.words[w] for w in mb["words"])
        for w, c, (tb, te) in zip(final.get("result", []), mb["conf"], mb["times"]):
            assert w["conf"] == pytest.approx(c, abs=1e-5)
            assert w["start"] == pytest.approx(tb * 0.03, abs=1e-5)
            assert w["end"] == pytest.approx(te * 0.03, abs=1e-5)
        # n-best alternatives come from the rescored lattice too
        rec = vosk.KaldiRecognizer(m, 16000)
        rec.SetMaxAlternatives(3)
        for i in range(0, len(data), 8000):
            rec.AcceptWaveform(data[i:i + 8000])
        alts = json.loads(rec.FinalResult())["alternatives"]
        nb = OI.final_result(oracle, wave, 4000, rescore=resc, nbest_n=3, on=on)["nbest"]
        assert [a["text"] for a in alts] == [" ".join(oracle.words[w] for w in x["words"]) for x in nb]
