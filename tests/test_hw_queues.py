"""The Python package's hardware-queue request (vosk/__init__.py
_hardware_queues): 8 queues when the process set no number and has not
started the HIP runtime; a number the process set is kept.  The recognizer
engines' spread follows it (csrc/vosk_impl.cc StreamEngineSpread,
profiles/r06_conc_queues.log).  CPU-only: importing the package loads
libvosk.so without touching a device."""
import os
import subprocess
import sys

from conftest import REPO

PKG = os.path.join(REPO, "vosk-api_amd")


def _queues_after_import(env_value, pre=""):
    env = {k: v for k, v in os.environ.items() if k != "GPU_MAX_HW_QUEUES"}
    if env_value is not None:
        env["GPU_MAX_HW_QUEUES"] = env_value
    code = (f"import sys, os; sys.path.insert(0, {PKG!r}); {pre}"
            "import vosk; print(os.environ.get('GPU_MAX_HW_QUEUES'))")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    return out.stdout.strip().splitlines()[-1]


def test_unset_queue_count_becomes_8():
    assert _queues_after_import(None) == "8"


def test_queue_count_set_by_the_process_is_kept():
    assert _queues_after_import("4") == "4"
    assert _queues_after_import("16") == "16"


def test_imported_torch_without_a_started_runtime_still_gets_8():
    # torch loaded but torch.cuda not initialized: the runtime has not read
    # the variable yet
    assert _queues_after_import(None, pre="import torch; ") == "8"
