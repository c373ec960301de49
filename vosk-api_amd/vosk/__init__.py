"""Python binding of the MI355X-native libvosk.so.

Same public surface as the reference package (python/vosk/__init__.py:45-235):
Model, SpkModel, KaldiRecognizer, BatchModel, BatchRecognizer, SetLogLevel,
GpuInit, GpuThreadInit.  The reference binds libvosk.so through cffi in ABI
mode; the cffi module is not installed in this image's python3.10, so the
same C functions are bound with ctypes here (identical argument meaning,
return values and error behaviour: constructors raise on NULL,
AcceptWaveform raises on a negative return).  Model download by name or
language needs network access and is not available offline: local model
directories (explicit path or MODEL_DIRS) are used instead.
"""
from __future__ import annotations

import ctypes as C
import os
import sys
from pathlib import Path
from re import match

MODEL_DIRS = [os.getenv("VOSK_MODEL_PATH"), Path("/usr/share/vosk"),
              Path.home() / "AppData/Local/vosk", Path.home() / ".cache/vosk"]


def _hardware_queues():
    """HIP gives a process GPU_MAX_HW_QUEUES hardware queues (4 by default)
    and hands them to its streams in turn; streams beyond that share a queue,
    one's launches waiting behind another's.  KaldiRecognizers are spread over
    up to 4 engines of two streams each (csrc/vosk_impl.cc StreamEngineSpread,
    from this variable), so ask for 8 -- unless the process chose a number or
    has started the HIP runtime already (it reads the variable when it
    starts: the first HIP call)."""
    if "GPU_MAX_HW_QUEUES" in os.environ:
        return
    torch = sys.modules.get("torch")
    try:
        if torch is not None and torch.cuda.is_initialized():
            return
    except Exception:
        return
    os.environ["GPU_MAX_HW_QUEUES"] = "8"


def open_dll():
    dlldir = os.path.abspath(os.path.dirname(__file__))
    if sys.platform != "linux":
        raise TypeError("Unsupported platform")
    _hardware_queues()
    # (VOSK_AMD_LIB: another build of the library, for A/B measurements)
    path = os.getenv("VOSK_AMD_LIB") or os.path.join(dlldir, "libvosk.so")
    if not os.path.exists(path):
        raise OSError(f"cannot load library {path}: build it with `make -C vosk-api_amd`")
    return C.CDLL(path)


_c = open_dll()

_vp = C.c_void_p
_SIGS = {
    "vosk_model_new": (_vp, [C.c_char_p]),
    "vosk_model_free": (None, [_vp]),
    "vosk_model_find_word": (C.c_int, [_vp, C.c_char_p]),
    "vosk_spk_model_new": (_vp, [C.c_char_p]),
    "vosk_spk_model_free": (None, [_vp]),
    "vosk_recognizer_new": (_vp, [_vp, C.c_float]),
    "vosk_recognizer_new_spk": (_vp, [_vp, C.c_float, _vp]),
    "vosk_recognizer_new_grm": (_vp, [_vp, C.c_float, C.c_char_p]),
    "vosk_recognizer_set_spk_model": (None, [_vp, _vp]),
    "vosk_recognizer_set_max_alternatives": (None, [_vp, C.c_int]),
    "vosk_recognizer_set_words": (None, [_vp, C.c_int]),
    "vosk_recognizer_set_partial_words": (None, [_vp, C.c_int]),
    "vosk_recognizer_set_nlsml": (None, [_vp, C.c_int]),
    "vosk_recognizer_accept_waveform": (C.c_int, [_vp, C.c_char_p, C.c_int]),
    "vosk_recognizer_accept_waveform_s": (C.c_int, [_vp, _vp, C.c_int]),
    "vosk_recognizer_accept_waveform_f": (C.c_int, [_vp, _vp, C.c_int]),
    "vosk_recognizer_result": (C.c_char_p, [_vp]),
    "vosk_recognizer_partial_result": (C.c_char_p, [_vp]),
    "vosk_recognizer_final_result": (C.c_char_p, [_vp]),
    "vosk_recognizer_reset": (None, [_vp]),
    "vosk_recognizer_free": (None, [_vp]),
    "vosk_set_log_level": (None, [C.c_int]),
    "vosk_gpu_init": (None, []),
    "vosk_gpu_thread_init": (None, []),
    "vosk_batch_model_new": (_vp, []),
    "vosk_batch_model_free": (None, [_vp]),
    "vosk_batch_model_wait": (None, [_vp]),
    "vosk_batch_recognizer_new": (_vp, [_vp, C.c_float]),
    "vosk_batch_recognizer_free": (None, [_vp]),
    "vosk_batch_recognizer_accept_waveform": (None, [_vp, C.c_char_p, C.c_int]),
    "vosk_batch_recognizer_set_nlsml": (None, [_vp, C.c_int]),
    "vosk_batch_recognizer_finish_stream": (None, [_vp]),
    "vosk_batch_recognizer_front_result": (C.c_char_p, [_vp]),
    "vosk_batch_recognizer_pop": (None, [_vp]),
    "vosk_batch_recognizer_get_pending_chunks": (C.c_int, [_vp]),
}
for _name, (_res, _args) in _SIGS.items():
    _f = getattr(_c, _name)
    _f.restype = _res
    _f.argtypes = _args


def _s(b):
    return (b or b"").decode("utf-8")


class Model(object):
    def __init__(self, model_path=None, model_name=None, lang=None):
        if model_path is None:
            model_path = self.get_model_path(model_name, lang)
        self._handle = _c.vosk_model_new(str(model_path).encode("utf-8"))
        if not self._handle:
            raise Exception("Failed to create a model")

    def __del__(self):
        if getattr(self, "_handle", None):
            _c.vosk_model_free(self._handle)

    def vosk_model_find_word(self, word):
        return _c.vosk_model_find_word(self._handle, word.encode("utf-8"))

    def get_model_path(self, model_name, lang):
        for directory in MODEL_DIRS:
            if directory is None or not Path(directory).exists():
                continue
            for m in os.listdir(directory):
                if (model_name is not None and m == model_name) or (
                        model_name is None and lang is not None and
                        match(r"vosk-model(-small)?-{}".format(lang), m)):
                    return str(Path(directory, m))
        raise Exception("model %s not found locally (downloads need network access)"
                        % (model_name or lang))


class SpkModel(object):
    def __init__(self, model_path):
        self._handle = _c.vosk_spk_model_new(model_path.encode("utf-8"))
        if not self._handle:
            raise Exception("Failed to create a speaker model")

    def __del__(self):
        if getattr(self, "_handle", None):
            _c.vosk_spk_model_free(self._handle)


class KaldiRecognizer(object):
    def __init__(self, *args):
        if len(args) == 2:
            self._handle = _c.vosk_recognizer_new(args[0]._handle, args[1])
        elif len(args) == 3 and type(args[2]) is SpkModel:
            self._handle = _c.vosk_recognizer_new_spk(args[0]._handle, args[1], args[2]._handle)
        elif len(args) == 3 and type(args[2]) is str:
            self._handle = _c.vosk_recognizer_new_grm(args[0]._handle, args[1],
                                                      args[2].encode("utf-8"))
        else:
            raise TypeError("Unknown arguments")
        if not self._handle:
            raise Exception("Failed to create a recognizer")

    def __del__(self):
        if getattr(self, "_handle", None):
            _c.vosk_recognizer_free(self._handle)

    def SetMaxAlternatives(self, max_alternatives):
        _c.vosk_recognizer_set_max_alternatives(self._handle, max_alternatives)

    def SetWords(self, enable_words):
        _c.vosk_recognizer_set_words(self._handle, 1 if enable_words else 0)

    def SetPartialWords(self, enable_partial_words):
        _c.vosk_recognizer_set_partial_words(self._handle, 1 if enable_partial_words else 0)

    def SetNLSML(self, enable_nlsml):
        _c.vosk_recognizer_set_nlsml(self._handle, 1 if enable_nlsml else 0)

    def SetSpkModel(self, spk_model):
        _c.vosk_recognizer_set_spk_model(self._handle, spk_model._handle)

    def AcceptWaveform(self, data):
        res = _c.vosk_recognizer_accept_waveform(self._handle, bytes(data), len(data))
        if res < 0:
            raise Exception("Failed to process waveform")
        return res

    def Result(self):
        return _s(_c.vosk_recognizer_result(self._handle))

    def PartialResult(self):
        return _s(_c.vosk_recognizer_partial_result(self._handle))

    def FinalResult(self):
        return _s(_c.vosk_recognizer_final_result(self._handle))

    def Reset(self):
        return _c.vosk_recognizer_reset(self._handle)


def SetLogLevel(level):
    return _c.vosk_set_log_level(level)


def GpuInit():
    _c.vosk_gpu_init()


def GpuThreadInit():
    _c.vosk_gpu_thread_init()


class BatchModel(object):
    def __init__(self, *args):
        self._handle = _c.vosk_batch_model_new()
        if not self._handle:
            raise Exception("Failed to create a model")

    def __del__(self):
        if getattr(self, "_handle", None):
            _c.vosk_batch_model_free(self._handle)

    def Wait(self):
        _c.vosk_batch_model_wait(self._handle)


class BatchRecognizer(object):
    def __init__(self, *args):
        self._handle = _c.vosk_batch_recognizer_new(args[0]._handle, args[1])
        if not self._handle:
            raise Exception("Failed to create a recognizer")

    def __del__(self):
        if getattr(self, "_handle", None):
            _c.vosk_batch_recognizer_free(self._handle)

    def AcceptWaveform(self, data):
        _c.vosk_batch_recognizer_accept_waveform(self._handle, bytes(data), len(data))

    def Result(self):
        res = _s(_c.vosk_batch_recognizer_front_result(self._handle))
        _c.vosk_batch_recognizer_pop(self._handle)
        return res

    def FinishStream(self):
        _c.vosk_batch_recognizer_finish_stream(self._handle)

    def GetPendingChunks(self):
        return _c.vosk_batch_recognizer_get_pending_chunks(self._handle)
