"""C-ABI boundary: libvosk.so loads, exports every symbol include/*.h declares,
and include/vosk_api.h is ABI-identical to the reference header."""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import REPO

LIB = os.path.join(REPO, "vosk-api_amd", "vosk", "libvosk.so")
HDRS = [os.path.join(REPO, "include", h) for h in ("vosk_api.h", "vosk_amd_engine.h")]
REF_HDR = "/root/reference/src/vosk_api.h"


def _decls(path):
    """(name, normalized signature) of every function declaration."""
    src = subprocess.run(["cpp", "-P", path], capture_output=True, text=True, check=True).stdout
    src = re.sub(r"\s+", " ", src)
    out = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(v\w+)\s*\(([^;{]*?)\)\s*;", src):
        ret, name, args = m.group(1).strip(), m.group(2), m.group(3).strip()
        args = ",".join(re.sub(r"\s*\*\s*", "*", a.strip()) for a in args.split(","))
        # drop parameter names: keep types only
        types = []
        for a in args.split(","):
            a = a.strip()
            if a in ("", "void"):
                continue
            t = re.sub(r"\b\w+$", "", a).strip() if re.search(r"[\w\*]\s*\w+$", a) and not a.endswith("*") else a
            types.append(t.replace(" ", ""))
        out[name] = (re.sub(r"\s*\*\s*", "*", ret).replace(" ", ""), tuple(types))
    return out


def test_library_loads_and_exports_all_declared_symbols():
    assert os.path.exists(LIB), "build libvosk.so first (make -C vosk-api_amd)"
    lib = C.CDLL(LIB)
    names = set()
    for h in HDRS:
        names |= set(_decls(h))
    assert len(names) >= 35 + 20
    missing = [n for n in sorted(names) if not hasattr(lib, n)]
    assert not missing, missing


def test_vosk_api_has_the_35_reference_functions():
    d = _decls(HDRS[0])
    assert len(d) == 35
    for n in ("vosk_recognizer_accept_waveform", "vosk_batch_recognizer_get_pending_chunks",
              "vosk_gpu_thread_init", "vosk_model_find_word"):
        assert n in d


@pytest.mark.skipif(not os.path.exists(REF_HDR), reason="reference not mounted")
def test_header_is_abi_identical_to_reference():
    ours, ref = _decls(HDRS[0]), _decls(REF_HDR)
    assert set(ours) == set(ref)
    for n in ref:
        assert ours[n] == ref[n], (n, ours[n], ref[n])


def test_header_is_plain_c_for_cffi_cdef():
    """python/vosk_builder.py feeds `cpp vosk_api.h` to cffi: only plain C."""
    out = subprocess.run(["cpp", "-P", HDRS[0]], capture_output=True, text=True, check=True).stdout
    assert "extern" not in out and "#" not in out
    subprocess.run(["gcc", "-fsyntax-only", "-x", "c", HDRS[0]], check=True)
