"""Golden fixtures recorded by the reference (python/example/colab/vosk.ipynb):
test.wav identity, the JSON byte format of results, and -- when a real
vosk-model-small-en-us-0.15 directory is supplied -- the recorded transcripts.
"""
import ctypes as C
import hashlib
import json
import os

import pytest

from conftest import REPO

GOLD = os.path.join(REPO, "tests", "golden", "notebook_small_en_us.json")


@pytest.fixture(scope="module")
def gold():
    return json.load(open(GOLD))


def test_test_wav_identity(gold):
    data = open(os.path.join(REPO, "tests", "golden", "test.wav"), "rb").read()
    sha = hashlib.sha256(data).hexdigest()
    assert sha == gold["test_wav_sha256"]
    assert sha.startswith("dcfea571") and sha.endswith("15bb")


def test_recorded_transcripts_present(gold):
    finals = [o["text"] for o in gold["runs"][0]["outputs"] if "text" in o]
    assert finals == ["one zero zero zero one", "nah no to i know", "zero one eight zero three"]


def _json_words(list_key, text_key, words):
    import vosk  # noqa: F401
    lib = vosk._c
    f = lib.vamd_json_words
    f.restype = C.c_char_p
    n = len(words)
    arr = (C.c_char_p * n)(*[w["word"].encode() for w in words])
    st = (C.c_double * n)(*[w["start"] for w in words])
    en = (C.c_double * n)(*[w["end"] for w in words])
    cf = (C.c_double * n)(*[w["conf"] for w in words])
    return f(list_key.encode(), text_key.encode(), n, arr, st, en, cf).decode()


def test_result_json_bytes_match_reference(gold):
    """The library's JSON writer reproduces json.h's dump() byte format
    (src/json.h:343-380) for every recorded result / partial_result object."""
    checked = 0
    run = gold["runs"][0]
    for obj, raw in zip(run["outputs"], run["raw_objects"]):
        if "result" in obj:
            assert _json_words("result", "text", obj["result"]) == raw
            checked += 1
        elif "partial_result" in obj:
            assert _json_words("partial_result", "partial", obj["partial_result"]) == raw
            checked += 1
    assert checked >= 5


@pytest.mark.gpu
@pytest.mark.skipif(not os.environ.get("VOSK_TEST_MODEL"),
                    reason="set VOSK_TEST_MODEL to a vosk-model-small-en-us-0.15 directory")
def test_real_model_transcripts(gold, test_wave):
    """End-to-end pin against the recorded outputs (needs the real model)."""
    import vosk
    m = vosk.Model(os.environ["VOSK_TEST_MODEL"])
    rec = vosk.KaldiRecognizer(m, 16000)
    rec.SetWords(True)
    rec.SetPartialWords(True)
    texts, words = [], []
    # test_wave holds the samples after the RIFF header (wave.readframes), so
    # 4000-frame reads are 8000-byte slices from byte 0 (vosk.ipynb's loop)
    data = test_wave.astype("<i2").tobytes()
    for i in range(0, len(data), 8000):
        if rec.AcceptWaveform(data[i:i + 8000]):
            r = json.loads(rec.Result())
            texts.append(r["text"])
            words += r.get("result", [])
    r = json.loads(rec.FinalResult())
    texts.append(r["text"])
    words += r.get("result", [])
    assert " ".join(t for t in texts if t) == "one zero zero zero one nah no to i know zero one eight zero three"
    # MBR confidences and aligned word times of the notebook (dither differs:
    # the notebook ran with Kaldi's default dither, so tolerances, not bytes)
    ref = [w for o in gold["runs"][0]["outputs"] if "result" in o for w in o["result"]]
    assert [w["word"] for w in words] == [w["word"] for w in ref]
    for w, g in zip(words, ref):
        assert abs(w["conf"] - g["conf"]) < 0.1
        assert abs(w["start"] - g["start"]) < 0.061 and abs(w["end"] - g["end"]) < 0.061
