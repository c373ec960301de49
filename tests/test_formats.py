"""Model-format layer: Python writer/reader round trips and the product's C++
readers (libvosk.so, no GPU needed) against the independent Python reader."""
import os

import numpy as np
import pytest

import kaldi_formats as kf


def test_kaldi_basic_roundtrip():
    w = kf.KaldiWriter()
    w.token("<Foo>")
    w.i32(-7)
    w.f32(1.5)
    w.boolean(True)
    w.int_vector([3, 1, 4])
    w.fvector(np.arange(5, dtype=np.float32))
    w.fmatrix(np.arange(6, dtype=np.float32).reshape(2, 3))
    r = kf.KaldiReader(w.bytes())
    assert r.token() == "<Foo>"
    assert r.i32() == -7
    assert r.f32() == 1.5
    assert r.boolean() is True
    assert r.int_vector().tolist() == [3, 1, 4]
    assert r.vector().tolist() == [0, 1, 2, 3, 4]
    assert r.matrix().tolist() == [[0, 1, 2], [3, 4, 5]]


def test_fst_roundtrip_const_and_vector(tmp_path):
    f = kf.Fst(0, np.array([np.inf, 0.5], np.float32), np.array([0, 2, 3], np.int64),
               np.array([3, 0, 5], np.int32), np.array([1, 0, 2], np.int32),
               np.array([0.25, 1.0, 2.0], np.float32), np.array([1, 1, 0], np.int32))
    for writer, name in ((kf.write_const_fst, "c.fst"), (kf.write_vector_fst, "v.fst")):
        p = str(tmp_path / name)
        writer(p, f)
        g = kf.read_fst(p)
        assert g.start == 0 and g.num_states == 2 and g.num_arcs == 3
        np.testing.assert_array_equal(g.ilabel, f.ilabel)
        np.testing.assert_array_equal(g.nextstate, f.nextstate)
        np.testing.assert_array_equal(g.weight, f.weight)
        np.testing.assert_array_equal(g.final, f.final)


def test_synth_model_reads_back(synth_model):
    tm, nn = kf.read_final_mdl(os.path.join(synth_model, "am", "final.mdl"))
    assert tm.num_tids > 0 and tm.tid2pdf.max() < 2000
    # chain topology: self-loop and forward transitions map to different pdf classes
    assert len(tm.tuples) == len(set(tm.tuples))
    assert "output.affine" in nn.components
    fst = kf.read_fst(os.path.join(synth_model, "graph", "HCLG.fst"))
    assert fst.num_states > 1000
    emitting = fst.ilabel[fst.ilabel != 0]
    assert emitting.min() >= 1 and emitting.max() <= tm.num_tids


def test_cpp_reader_agrees_with_python(synth_model):
    """libvosk.so's C++ readers (model load is host-only) vs the Python reader."""
    import vosk
    from vosk import engine as ve
    vosk.SetLogLevel(-1)
    m = vosk.Model(synth_model)
    words = kf.read_symbol_table(os.path.join(synth_model, "graph", "words.txt"))
    for wid in (1, 17, 2999):
        assert m.vosk_model_find_word(words[wid]) == wid
    assert m.vosk_model_find_word("no-such-word") == -1
    info = ve.plan_info(synth_model, 51)
    assert info["out_dim"] == 2000
    assert (info["left_context"], info["right_context"]) == (26, 26)
    assert info["fpc"] == 51 and info["fss"] == 3


def test_model_missing_files(tmp_path):
    import vosk
    vosk.SetLogLevel(-1)
    with pytest.raises(Exception):
        vosk.Model(str(tmp_path))


def test_recognizer_fails_loudly_without_gpu(synth_model):
    """No CPU fallback: without a HIP device the recognizer cannot be created."""
    import vosk
    from vosk import engine as ve
    if ve.device_count() > 0:
        pytest.skip("a GPU is present")
    vosk.SetLogLevel(-1)
    m = vosk.Model(synth_model)
    with pytest.raises(Exception):
        vosk.KaldiRecognizer(m, 16000)
