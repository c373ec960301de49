"""The reference's own Python binding, unchanged, against this libvosk.so
(north_star: "keeping ... the Python cffi binding unchanged").

Build-container only (CPU, no GPU calls): the reference's
python/vosk_builder.py:7-11 generates the ABI-mode cffi module from
include/vosk_api.h (its `cpp $VOSK_SOURCE/src/vosk_api.h` step pointed at this
repository's header), and the unchanged python/vosk/__init__.py is imported
from a temporary directory beside this libvosk.so (its open_dll,
python/vosk/__init__.py:17-32).  The checks cover what needs no device:
Model(path), vosk_model_find_word, SpkModel, the NULL -> exception paths of
the constructors (python/vosk/__init__.py:134-183) and SetLogLevel.

Skips when /root/reference (never present on the GPU box) or the cffi
interpreter (/opt/conda/bin/python3.9, cffi 1.14.6; the system Python has no
cffi) is absent.  Nothing from the reference is written into the repository:
the package is copied into a pytest tmp directory for the run only."""
import os
import shutil
import subprocess
import textwrap

import pytest

from conftest import REPO

REF = "/root/reference"
PY39 = "/opt/conda/bin/python3.9"
LIB = os.path.join(REPO, "vosk-api_amd", "vosk", "libvosk.so")

pytestmark = pytest.mark.skipif(
    not (os.path.isdir(os.path.join(REF, "python", "vosk")) and os.path.exists(PY39) and os.path.exists(LIB)),
    reason="needs /root/reference, /opt/conda/bin/python3.9 (cffi) and a built libvosk.so")


@pytest.fixture(scope="module")
def ref_pkg(tmp_path_factory):
    root = tmp_path_factory.mktemp("refbind")
    # VOSK_SOURCE/src/vosk_api.h -> this repository's header
    os.makedirs(root / "src")
    os.symlink(os.path.join(REPO, "include", "vosk_api.h"), root / "src" / "vosk_api.h")
    pkg = root / "pkg"
    shutil.copytree(os.path.join(REF, "python", "vosk"), pkg / "vosk")
    os.symlink(LIB, pkg / "vosk" / "libvosk.so")
    env = dict(os.environ, VOSK_SOURCE=str(root))
    r = subprocess.run([PY39, os.path.join(REF, "python", "vosk_builder.py")], cwd=pkg, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert (pkg / "vosk" / "vosk_cffi.py").exists()
    return pkg


def _run(pkg, code, timeout=300):
    env = dict(os.environ, PYTHONPATH=str(pkg))
    r = subprocess.run([PY39, "-c", textwrap.dedent(code)], cwd=pkg, env=env, capture_output=True, text=True,
                       timeout=timeout)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    return r.stdout


def test_cdef_declares_every_export(ref_pkg):
    out = _run(ref_pkg, """
        import vosk
        from vosk.vosk_cffi import ffi
        names = sorted(n for n in dir(vosk._c) if n.startswith("vosk_"))
        print(len(names))
        print(" ".join(names))
    """)
    n, names = out.split("\n")[:2]
    assert int(n) == 35, names


def test_model_and_find_word(ref_pkg, synth_model):
    import vosk as ours
    words = open(os.path.join(synth_model, "graph", "words.txt")).read().split()
    w, wid = words[10], int(words[11])
    out = _run(ref_pkg, f"""
        import vosk
        vosk.SetLogLevel(-1)
        m = vosk.Model({synth_model!r})
        print(m.vosk_model_find_word({w!r}))
        print(m.vosk_model_find_word("no-such-word-xyz"))
        del m
    """)
    a, b = out.split("\n")[:2]
    assert int(a) == wid
    assert int(b) == -1
    assert ours is not None


def test_speaker_model(ref_pkg, synth_spk):
    out = _run(ref_pkg, f"""
        import vosk
        vosk.SetLogLevel(-1)
        s = vosk.SpkModel({synth_spk!r})
        print("ok")
        del s
    """)
    assert out.startswith("ok")


def test_constructor_failures_raise(ref_pkg):
    # vosk_model_new / vosk_spk_model_new return NULL on any exception
    # (src/vosk_api.cc:30-94) and the binding raises (python/vosk/__init__.py:50-51,126-127)
    out = _run(ref_pkg, """
        import vosk
        vosk.SetLogLevel(-1)
        for ctor, msg in ((vosk.Model, "Failed to create a model"), (vosk.SpkModel, "Failed to create a speaker model")):
            try:
                ctor("/nonexistent/model/dir")
                print("no exception")
            except Exception as e:
                print(str(e) == msg)
    """)
    assert out.split("\n")[:2] == ["True", "True"]


def test_recognizer_without_a_gpu_fails_loudly(ref_pkg, synth_model):
    """No CPU fallback: without a HIP device vosk_recognizer_new returns NULL
    and the unchanged binding raises (python/vosk/__init__.py:146-147)."""
    from conftest import has_gpu
    if has_gpu():
        pytest.skip("a GPU is visible")
    out = _run(ref_pkg, f"""
        import vosk
        vosk.SetLogLevel(-1)
        m = vosk.Model({synth_model!r})
        try:
            vosk.KaldiRecognizer(m, 16000.0)
            print("no exception")
        except Exception as e:
            print(str(e))
    """)
    assert out.split("\n")[0] == "Failed to create a recognizer"
