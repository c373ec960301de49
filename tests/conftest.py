import os
import shutil
import sys
import wave

import numpy as np
import pytest

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
PKG = os.path.join(REPO, "vosk-api_amd")
for p in (PKG, os.path.join(PKG, "tools"), os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

MODEL_CACHE = os.environ.get("VAMD_MODEL_CACHE", os.path.join(
    os.environ.get("TMPDIR", "/tmp"), "vamd_models"))
SYNTH_VERSION = "v4"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


def _make(name, post=None, **kw):
    import make_synth_model as msm
    path = os.path.join(MODEL_CACHE, f"{name}_{SYNTH_VERSION}")
    if not os.path.exists(os.path.join(path, "README")):
        tmp = path + f".tmp{os.getpid()}"
        shutil.rmtree(tmp, ignore_errors=True)
        msm.make_model(tmp, **kw)
        if post is not None:
            post(tmp)
        shutil.rmtree(path, ignore_errors=True)
        os.rename(tmp, path)
    return path


@pytest.fixture(scope="session")
def synth_model():
    """Seeded synthetic model in the real Kaldi/OpenFST on-disk formats."""
    return _make("synth", seed=7, vocab=3000, num_pdfs=2000)


@pytest.fixture(scope="session")
def synth_model_noep(synth_model):
    """Same model with endpointing disabled (single segment per stream)."""
    path = os.path.join(MODEL_CACHE, f"synth_noep_{SYNTH_VERSION}")
    if not os.path.exists(os.path.join(path, "README")):
        tmp = path + f".tmp{os.getpid()}"
        shutil.rmtree(tmp, ignore_errors=True)
        shutil.copytree(synth_model, tmp)
        with open(os.path.join(tmp, "conf", "model.conf"), "a") as f:
            for r in range(1, 6):
                f.write(f"--endpoint.rule{r}.min-utterance-length=1e9\n")
        shutil.rmtree(path, ignore_errors=True)
        os.rename(tmp, path)
    return path


# endpoint rules that fire on the synthetic model (its best paths carry
# almost no silence-phone frames): rule 1 on the final relative cost alone
# (data-dependent positions), rule 5 after 4 s
EP_RULES = ("--endpoint.rule1.min-trailing-silence=0\n--endpoint.rule1.max-relative-cost=12\n"
            "--endpoint.rule5.min-utterance-length=4\n")


@pytest.fixture(scope="session")
def synth_model_ep(synth_model):
    """synth_model with endpoint rules that fire every few seconds."""
    path = os.path.join(MODEL_CACHE, f"synth_ep_{SYNTH_VERSION}")
    if not os.path.exists(os.path.join(path, "README")):
        tmp = path + f".tmp{os.getpid()}"
        shutil.rmtree(tmp, ignore_errors=True)
        shutil.copytree(synth_model, tmp)
        with open(os.path.join(tmp, "conf", "model.conf"), "a") as f:
            f.write(EP_RULES)
        shutil.rmtree(path, ignore_errors=True)
        os.rename(tmp, path)
    return path


@pytest.fixture(scope="session")
def synth_model_wide(synth_model):
    """Same model with a wide beam (30) and max-active 20000: frames with
    thousands of tokens (decoder capacity and fallback paths)."""
    path = os.path.join(MODEL_CACHE, f"synth_wide_{SYNTH_VERSION}")
    if not os.path.exists(os.path.join(path, "README")):
        tmp = path + f".tmp{os.getpid()}"
        shutil.rmtree(tmp, ignore_errors=True)
        shutil.copytree(synth_model, tmp)
        with open(os.path.join(tmp, "conf", "model.conf"), "a") as f:
            f.write("--beam=30.0\n--max-active=20000\n")
        shutil.rmtree(path, ignore_errors=True)
        os.rename(tmp, path)
    return path


@pytest.fixture(scope="session")
def synth_lookahead():
    """Lookahead model (graph/HCLr.fst + graph/Gr.fst + disambig_tid.int, no
    HCLG), endpointing disabled (one segment per stream)."""
    def noep(d):
        with open(os.path.join(d, "conf", "model.conf"), "a") as f:
            for r in range(1, 6):
                f.write(f"--endpoint.rule{r}.min-utterance-length=1e9\n")
    return _make("synth_la", post=noep, seed=11, vocab=300, num_pdfs=2000, graph="lookahead")


@pytest.fixture(scope="session")
def synth_model_rescore(synth_model_noep):
    """synth_model_noep + rescore/G.fst and rescore/G.carpa."""
    import make_synth_model as msm
    path = os.path.join(MODEL_CACHE, f"synth_rescore_{SYNTH_VERSION}")
    if not os.path.exists(os.path.join(path, "README")):
        tmp = path + f".tmp{os.getpid()}"
        shutil.rmtree(tmp, ignore_errors=True)
        shutil.copytree(synth_model_noep, tmp)
        msm.add_rescore(tmp)
        shutil.rmtree(path, ignore_errors=True)
        os.rename(tmp, path)
    return path


@pytest.fixture(scope="session")
def synth_spk():
    """Synthetic x-vector speaker model (mfcc.conf, final.ext.raw, mean.vec,
    transform.mat)."""
    import make_synth_model as msm
    path = os.path.join(MODEL_CACHE, f"synth_spk_{SYNTH_VERSION}")
    if not os.path.exists(os.path.join(path, "README")):
        tmp = path + f".tmp{os.getpid()}"
        shutil.rmtree(tmp, ignore_errors=True)
        msm.make_spk_model(tmp)
        shutil.rmtree(path, ignore_errors=True)
        os.rename(tmp, path)
    return path


def _make_preset(name):
    import make_synth_model as msm
    return _make(name, **msm.PRESETS[name])


@pytest.fixture(scope="session")
def synth_bigram_2m():
    """BASELINE config 4's per-GPU share: a 2.4 M-state static HCLG (bigram
    LM over 20 k words), flat scores (max-active 7000 engaged)."""
    return _make_preset("bigram_2m")


@pytest.fixture(scope="session")
def synth_bigram_8m():
    """A static HCLG several times the 2.4 M-state one (~7.7 M states),
    standing in for vosk-model-en-us-0.22's graph (BASELINE config 4)."""
    return _make_preset("bigram_8m")


@pytest.fixture(scope="session")
def synth_la_small_en_us():
    """vosk-model-small-en-us scale lookahead model (20 k-word HCLr + a
    29 k-history trigram Gr; ~275 k states once expanded at load with
    OpenFST's weight and label pushing)."""
    return _make_preset("la_small_en_us")


@pytest.fixture(scope="session")
def test_wave():
    w = wave.open(os.path.join(REPO, "tests", "golden", "test.wav"), "rb")
    return np.frombuffer(w.readframes(w.getnframes()), "<i2").astype(np.float32)


def perturbed_stream(base, i, seconds=None, sr=16000):
    """Synthetic stream i (BASELINE.md workload): test.wav tiled, circularly
    shifted by (i*7919) mod len, gain U[0.5,1.5], N(0,10 LSB) noise."""
    rng = np.random.default_rng(1234 + i)
    n = len(base) if seconds is None else int(seconds * sr)
    reps = int(np.ceil(n / len(base))) + 1
    x = np.tile(base, reps)
    sh = (i * 7919) % len(base)
    x = x[sh:sh + n].astype(np.float64)
    x = x * rng.uniform(0.5, 1.5) + rng.normal(0.0, 10.0, n)
    return np.clip(np.round(x), -32768, 32767).astype(np.float32)


def has_gpu():
    try:
        from vosk import engine
        return engine.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session", params=[("fbank", True), ("mfcc", True)],
                ids=["fbank_cmvn", "mfcc_cmvn"])
def synth_model_frontend(request):
    """Small models with the other front ends of src/model.cc:218-269: a log
    fbank front end and/or global CMVN on the nnet input (am/global_cmvn.stats)."""
    fe, cmvn = request.param
    return _make(f"synth_{fe}{'_cmvn' if cmvn else ''}", seed=5, vocab=500, num_pdfs=300,
                 frontend=fe, global_cmvn=cmvn)
