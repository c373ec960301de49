"""Kaldi binary object + OpenFST binary FST writer/reader (numpy).

This is the Python half of the model-format layer.  The product reads the
same files with the C++ readers in ``csrc/kaldi_io.cc`` / ``csrc/fst_io.cc``;
this module exists so that (a) the synthetic-model generator can emit models
in the exact on-disk formats a real Vosk model directory uses, and (b) tests
can parse a model independently of the C++ reader and cross-check it.

Formats restated (third-party, not vendored in /root/reference -- Kaldi
``base/io-funcs``, ``matrix/kaldi-vector``, ``hmm/transition-model``,
``hmm/hmm-topology``, ``nnet3/nnet-nnet``, ``nnet3/am-nnet-simple``; OpenFST
``fst/fst.h`` FstHeader, ``fst/const-fst.h``, ``fst/vector-fst.h``):

* binary Kaldi stream starts with ``\\0B``; a token is its text followed by a
  single space; an int32/float basic type is one size byte (4) + 4 LE bytes;
  ``bool`` is the single char ``T``/``F``; an integer vector is one size byte,
  an int32 count and the raw elements; ``FV``/``FM`` (``DV``/``DM``) vectors and
  matrices are the token, int32 dims as basic types, then raw row-major data.
* OpenFST: FstHeader = int32 magic 2125659606, string fst type, string arc
  type, int32 version, int32 flags, uint64 properties, int64 start, int64
  #states, int64 #arcs (strings are int32 length + bytes).  ``const`` body
  (version 2): 20-byte states {float final, u32 pos, u32 narcs, u32
  niepsilons, u32 noepsilons} then 16-byte arcs {i32 ilabel, i32 olabel,
  float weight, i32 nextstate}, each section 16-byte aligned when flags has
  kIsAligned (4).  ``vector`` body (version 2): per state float final, int64
  narcs, narcs arcs.

Reference call sites that read these files: ``src/model.cc:233-243`` (final.mdl),
``src/model.cc:278-285`` (HCLG.fst / HCLr.fst + Gr.fst),
``src/model.cc:288-300`` (words.txt), ``src/batch_model.cc:39-54``.
"""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass, field

import numpy as np

FST_MAGIC = 2125659606
SYMTAB_MAGIC = 2125658996
K_IS_ALIGNED = 4
K_HAS_ISYMBOLS = 1
K_HAS_OSYMBOLS = 2


# ----------------------------------------------------------------------------
# Kaldi binary writer
# ----------------------------------------------------------------------------
class KaldiWriter:
    def __init__(self):
        self.buf = bytearray(b"\0B")

    def token(self, t: str):
        self.buf += t.encode() + b" "

    def raw(self, b: bytes):
        self.buf += b

    def i32(self, v: int):
        self.buf += b"\x04" + struct.pack("<i", int(v))

    def f32(self, v: float):
        self.buf += b"\x04" + struct.pack("<f", float(v))

    def boolean(self, v: bool):
        self.buf += b"T" if v else b"F"

    def int_vector(self, v):
        a = np.asarray(v, dtype="<i4")
        self.buf += b"\x04" + struct.pack("<i", a.size) + a.tobytes()

    def fvector(self, v):
        a = np.asarray(v, dtype="<f4").ravel()
        self.token("FV")
        self.i32(a.size)
        self.buf += a.tobytes()

    def fmatrix(self, m):
        a = np.ascontiguousarray(np.asarray(m, dtype="<f4"))
        assert a.ndim == 2
        self.token("FM")
        self.i32(a.shape[0])
        self.i32(a.shape[1])
        self.buf += a.tobytes()

    def f64(self, v: float):
        self.buf += b"\x08" + struct.pack("<d", float(v))

    def dvector(self, v):
        a = np.asarray(v, dtype="<f8").ravel()
        self.token("DV")
        self.i32(a.size)
        self.buf += a.tobytes()

    def dmatrix(self, m):
        a = np.ascontiguousarray(np.asarray(m, dtype="<f8"))
        assert a.ndim == 2
        self.token("DM")
        self.i32(a.shape[0])
        self.i32(a.shape[1])
        self.buf += a.tobytes()

    def dspmatrix(self, m):
        """SpMatrix<double>: lower triangle, row-major packed."""
        a = np.asarray(m, dtype=np.float64)
        n = a.shape[0]
        self.token("DP")
        self.i32(n)
        self.buf += np.concatenate([a[i, :i + 1] for i in range(n)]).astype("<f8").tobytes()

    def bytes(self) -> bytes:
        return bytes(self.buf)


# ----------------------------------------------------------------------------
# Kaldi binary reader
# ----------------------------------------------------------------------------
class KaldiReader:
    def __init__(self, data: bytes, pos: int = 0):
        self.d = data
        self.p = pos
        if pos == 0:
            if self.d[:2] != b"\0B":
                raise ValueError("not a binary Kaldi stream")
            self.p = 2

    def peek_char(self) -> str:
        return chr(self.d[self.p])

    def skip_ws(self):
        while self.p < len(self.d) and self.d[self.p] in b" \t\n\r":
            self.p += 1

    def token(self) -> str:
        self.skip_ws()
        e = self.p
        while e < len(self.d) and self.d[e] not in b" \t\n\r":
            e += 1
        t = self.d[self.p:e].decode()
        self.p = e
        if self.p < len(self.d) and self.d[self.p] == 0x20:
            self.p += 1
        return t

    def expect(self, t: str):
        got = self.token()
        if got != t:
            raise ValueError(f"expected token {t!r}, got {got!r} at {self.p}")

    def peek_token(self) -> str:
        save = self.p
        t = self.token()
        self.p = save
        return t

    def i32(self) -> int:
        sz = self.d[self.p]
        if sz != 4:
            raise ValueError(f"bad int size byte {sz}")
        v = struct.unpack_from("<i", self.d, self.p + 1)[0]
        self.p += 5
        return v

    def f32(self) -> float:
        sz = self.d[self.p]
        if sz == 4:
            v = struct.unpack_from("<f", self.d, self.p + 1)[0]
            self.p += 5
        elif sz == 8:
            v = struct.unpack_from("<d", self.d, self.p + 1)[0]
            self.p += 9
        else:
            raise ValueError(f"bad float size byte {sz}")
        return v

    def boolean(self) -> bool:
        self.skip_ws()
        c = chr(self.d[self.p])
        self.p += 1
        if c not in "TF":
            raise ValueError("bad bool")
        return c == "T"

    def int_vector(self) -> np.ndarray:
        sz = self.d[self.p]
        n = struct.unpack_from("<i", self.d, self.p + 1)[0]
        self.p += 5
        dt = {4: "<i4", 8: "<i8", 2: "<i2", 1: "<i1"}[sz]
        a = np.frombuffer(self.d, dtype=dt, count=n, offset=self.p).astype(np.int32)
        self.p += n * sz
        return a

    def vector(self) -> np.ndarray:
        t = self.token()
        n = self.i32()
        if t == "FV":
            a = np.frombuffer(self.d, "<f4", n, self.p).copy()
            self.p += 4 * n
        elif t == "DV":
            a = np.frombuffer(self.d, "<f8", n, self.p).astype(np.float32)
            self.p += 8 * n
        else:
            raise ValueError(f"unsupported vector type {t}")
        return a

    def matrix(self) -> np.ndarray:
        t = self.token()
        r = self.i32()
        c = self.i32()
        if t == "FM":
            a = np.frombuffer(self.d, "<f4", r * c, self.p).reshape(r, c).copy()
            self.p += 4 * r * c
        elif t == "DM":
            a = np.frombuffer(self.d, "<f8", r * c, self.p).reshape(r, c).astype(np.float32)
            self.p += 8 * r * c
        else:
            raise ValueError(f"unsupported matrix type {t}")
        return a

    def f64(self) -> float:
        return self.f32()

    def dvector64(self) -> np.ndarray:
        t = self.token()
        n = self.i32()
        dt = {"FV": "<f4", "DV": "<f8"}[t]
        a = np.frombuffer(self.d, dt, n, self.p).astype(np.float64)
        self.p += np.dtype(dt).itemsize * n
        return a

    def matrix64(self) -> np.ndarray:
        t = self.token()
        r = self.i32()
        c = self.i32()
        dt = {"FM": "<f4", "DM": "<f8"}[t]
        a = np.frombuffer(self.d, dt, r * c, self.p).reshape(r, c).astype(np.float64)
        self.p += np.dtype(dt).itemsize * r * c
        return a

    def spmatrix64(self) -> np.ndarray:
        t = self.token()
        n = self.i32()
        dt = {"FP": "<f4", "DP": "<f8"}[t]
        cnt = n * (n + 1) // 2
        v = np.frombuffer(self.d, dt, cnt, self.p).astype(np.float64)
        self.p += np.dtype(dt).itemsize * cnt
        m = np.zeros((n, n))
        k = 0
        for i in range(n):
            m[i, :i + 1] = v[k:k + i + 1]
            k += i + 1
        return m + np.tril(m, -1).T

    def line(self) -> str:
        e = self.d.index(b"\n", self.p)
        s = self.d[self.p:e].decode()
        self.p = e + 1
        return s


# ----------------------------------------------------------------------------
# HMM topology / transition model (chain-style topologies included)
# ----------------------------------------------------------------------------
@dataclass
class HmmState:
    forward_pdf_class: int
    self_loop_pdf_class: int
    transitions: list  # [(dest_state, prob)]


@dataclass
class Topology:
    phones: list
    phone2idx: list
    entries: list  # list[list[HmmState]]

    def is_hmm(self) -> bool:
        return all(s.forward_pdf_class == s.self_loop_pdf_class for e in self.entries for s in e)


@dataclass
class TransitionModel:
    topo: Topology
    tuples: list  # (phone, hmm_state, forward_pdf, self_loop_pdf)
    log_probs: np.ndarray
    # derived
    tid2pdf: np.ndarray = field(default=None)
    tid2phone: np.ndarray = field(default=None)
    tid_is_selfloop: np.ndarray = field(default=None)
    tid_is_final: np.ndarray = field(default=None)  # into the HMM's final state (IsFinal)
    tuple_first_tid: np.ndarray = field(default=None)
    tid2hmmstate: np.ndarray = field(default=None)  # the transition's source HMM state

    def derive(self):
        """Transition-id numbering (1-based): tuple i owns one id per
        transition of its HMM state; a transition back to the same HMM state
        is a self-loop and maps to the self-loop pdf, any other transition to
        the forward pdf (Kaldi ``TransitionModel::ComputeDerived`` semantics)."""
        pdf = [0]
        phone = [0]
        sl = [0]
        fin = [0]
        hmm = [0]
        first = []
        for (ph, hs, fpdf, spdf) in self.tuples:
            first.append(len(pdf))
            entry = self.topo.entries[self.topo.phone2idx[ph]]
            st = entry[hs]
            for (dst, _p) in st.transitions:
                is_sl = dst == hs
                pdf.append(spdf if is_sl else fpdf)
                phone.append(ph)
                sl.append(1 if is_sl else 0)
                fin.append(1 if dst == len(entry) - 1 else 0)
                hmm.append(hs)
        self.tid2pdf = np.array(pdf, np.int32)
        self.tid2phone = np.array(phone, np.int32)
        self.tid_is_selfloop = np.array(sl, np.int32)
        self.tid_is_final = np.array(fin, np.int32)
        self.tuple_first_tid = np.array(first, np.int32)
        self.tid2hmmstate = np.array(hmm, np.int32)
        return self

    @property
    def num_tids(self):
        return len(self.tid2pdf) - 1


def write_topology(w: KaldiWriter, t: Topology):
    w.token("<Topology>")
    w.int_vector(t.phones)
    w.int_vector(t.phone2idx)
    is_hmm = t.is_hmm()
    if not is_hmm:
        w.i32(-1)
    w.i32(len(t.entries))
    for e in t.entries:
        w.i32(len(e))
        for s in e:
            w.i32(s.forward_pdf_class)
            if not is_hmm:
                w.i32(s.self_loop_pdf_class)
            w.i32(len(s.transitions))
            for (d, p) in s.transitions:
                w.i32(d)
                w.f32(p)
    w.token("</Topology>")


def read_topology(r: KaldiReader) -> Topology:
    r.expect("<Topology>")
    phones = r.int_vector().tolist()
    phone2idx = r.int_vector().tolist()
    n = r.i32()
    is_hmm = True
    if n == -1:
        is_hmm = False
        n = r.i32()
    entries = []
    for _ in range(n):
        ns = r.i32()
        e = []
        for _ in range(ns):
            fpc = r.i32()
            spc = fpc if is_hmm else r.i32()
            nt = r.i32()
            tr = [(r.i32(), r.f32()) for _ in range(nt)]
            e.append(HmmState(fpc, spc, tr))
        entries.append(e)
    r.expect("</Topology>")
    return Topology(phones, phone2idx, entries)


def write_transition_model(w: KaldiWriter, tm: TransitionModel):
    is_hmm = tm.topo.is_hmm()
    w.token("<TransitionModel>")
    write_topology(w, tm.topo)
    w.token("<Triples>" if is_hmm else "<Tuples>")
    w.i32(len(tm.tuples))
    for (ph, hs, fp, sp) in tm.tuples:
        w.i32(ph)
        w.i32(hs)
        w.i32(fp)
        if not is_hmm:
            w.i32(sp)
    w.token("</Triples>" if is_hmm else "</Tuples>")
    w.token("<LogProbs>")
    w.fvector(tm.log_probs)
    w.token("</LogProbs>")
    w.token("</TransitionModel>")


def read_transition_model(r: KaldiReader) -> TransitionModel:
    r.expect("<TransitionModel>")
    topo = read_topology(r)
    t = r.token()
    is_hmm = t == "<Triples>"
    n = r.i32()
    tuples = []
    for _ in range(n):
        ph, hs, fp = r.i32(), r.i32(), r.i32()
        sp = fp if is_hmm else r.i32()
        tuples.append((ph, hs, fp, sp))
    r.expect("</Triples>" if is_hmm else "</Tuples>")
    r.expect("<LogProbs>")
    lp = r.vector()
    r.expect("</LogProbs>")
    r.expect("</TransitionModel>")
    return TransitionModel(topo, tuples, lp).derive()


# ----------------------------------------------------------------------------
# nnet3 components (the subset a TDNN-F chain model uses)
# ----------------------------------------------------------------------------
# value kind of every field tag we know how to read/write
FIELD_KIND = {
    # floats
    "<LearningRateFactor>": "f", "<MaxChange>": "f", "<L2Regularize>": "f",
    "<LearningRate>": "f", "<OrthonormalConstraint>": "f", "<NumSamplesHistory>": "f",
    "<Alpha>": "f", "<Epsilon>": "f", "<TargetRms>": "f", "<Count>": "f",
    "<DropoutProportion>": "f", "<BackpropScale>": "f", "<OderivCount>": "f",
    "<SelfRepairLowerThreshold>": "f", "<SelfRepairUpperThreshold>": "f",
    "<SelfRepairScale>": "f", "<ZeroedProportion>": "f", "<Scale>": "f",
    "<BiasStddev>": "f", "<ParamStddev>": "f",
    "<NumDimsSelfRepaired>": "f", "<NumDimsProcessed>": "f", "<SelfRepairTarget>": "f",
    "<Rank>": "i",
    # ints
    "<Dim>": "i", "<BlockDim>": "i", "<InputDim>": "i", "<OutputDim>": "i",
    "<RankIn>": "i", "<RankOut>": "i", "<UpdatePeriod>": "i", "<TimePeriod>": "i",
    "<TimeMaskMaxFrames>": "i",
    # statistics extraction / pooling (x-vector nnets; Kaldi spells "Varinance")
    "<InputPeriod>": "i", "<OutputPeriod>": "i", "<IncludeVarinance>": "b",
    "<LeftContext>": "i", "<RightContext>": "i", "<NumLogCountFeatures>": "i",
    "<OutputStddevs>": "b", "<VarianceFloor>": "f",
    # bools
    "<IsGradient>": "b", "<TestMode>": "b", "<UseNaturalGradient>": "b",
    "<Continuous>": "b",
    # vectors / matrices
    "<BiasParams>": "v", "<StatsMean>": "v", "<StatsVar>": "v", "<ValueAvg>": "v",
    "<DerivAvg>": "v", "<OderivRms>": "v", "<Scales>": "v", "<Offsets>": "v",
    "<LinearParams>": "m", "<Params>": "m",
    # misc
    "<TimeOffsets>": "iv", "<AlphaInOut>": "ff", "<RankInOut>": "ii",
}


def write_component(w: KaldiWriter, ctype: str, fields: list):
    """fields: ordered list of (tag, value)."""
    w.token(f"<{ctype}>")
    for tag, val in fields:
        kind = FIELD_KIND[tag]
        w.token(tag)
        if kind == "f":
            w.f32(val)
        elif kind == "i":
            w.i32(val)
        elif kind == "b":
            w.boolean(val)
        elif kind == "v":
            w.fvector(val)
        elif kind == "m":
            w.fmatrix(val)
        elif kind == "iv":
            w.int_vector(val)
        elif kind == "ff":
            w.f32(val[0]); w.f32(val[1])
        elif kind == "ii":
            w.i32(val[0]); w.i32(val[1])
    w.token(f"</{ctype}>")


def read_component(r: KaldiReader):
    open_tag = r.token()
    assert open_tag.startswith("<") and open_tag.endswith(">"), open_tag
    ctype = open_tag[1:-1]
    close = f"</{ctype}>"
    fields = {}
    while True:
        tag = r.token()
        if tag == close:
            break
        kind = FIELD_KIND.get(tag)
        if kind is None:
            raise ValueError(f"unknown field {tag} in component {ctype}")
        if kind == "f":
            fields[tag] = r.f32()
        elif kind == "i":
            fields[tag] = r.i32()
        elif kind == "b":
            fields[tag] = r.boolean()
        elif kind == "v":
            fields[tag] = r.vector()
        elif kind == "m":
            fields[tag] = r.matrix()
        elif kind == "iv":
            fields[tag] = r.int_vector()
        elif kind == "ff":
            fields[tag] = (r.f32(), r.f32())
        elif kind == "ii":
            fields[tag] = (r.i32(), r.i32())
    return ctype, fields


@dataclass
class Nnet3:
    config_lines: list
    components: dict  # name -> (type, fields)
    component_order: list
    left_context: int = 0
    right_context: int = 0
    priors: np.ndarray = None


def write_nnet3_am(w: KaldiWriter, nn: Nnet3):
    w.token("<Nnet3>")
    w.raw(b"\n")
    for ln in nn.config_lines:
        w.raw(ln.encode() + b"\n")
    w.raw(b"\n")
    w.token("<NumComponents>")
    w.i32(len(nn.component_order))
    for name in nn.component_order:
        ctype, fields = nn.components[name]
        w.token("<ComponentName>")
        w.token(name)
        write_component(w, ctype, fields)
    w.token("</Nnet3>")
    w.token("<LeftContext>")
    w.i32(nn.left_context)
    w.token("<RightContext>")
    w.i32(nn.right_context)
    w.token("<Priors>")
    w.fvector(nn.priors if nn.priors is not None else np.zeros(0, np.float32))


def read_nnet3_am(r: KaldiReader) -> Nnet3:
    r.expect("<Nnet3>")
    r.line()  # rest of the token line
    lines = []
    while True:
        ln = r.line()
        if ln.strip() == "":
            break
        lines.append(ln)
    r.expect("<NumComponents>")
    n = r.i32()
    comps, order = {}, []
    for _ in range(n):
        r.expect("<ComponentName>")
        name = r.token()
        comps[name] = read_component(r)
        order.append(name)
    r.expect("</Nnet3>")
    lc = rc = 0
    pri = None
    if r.p < len(r.d) and r.peek_token() == "<LeftContext>":
        r.expect("<LeftContext>"); lc = r.i32()
        r.expect("<RightContext>"); rc = r.i32()
        if r.p < len(r.d) and r.peek_token() == "<Priors>":
            r.expect("<Priors>"); pri = r.vector()
    return Nnet3(lines, comps, order, lc, rc, pri)


def write_nnet3_raw(path: str, nn: Nnet3):
    """Nnet::Write (binary): config lines, components, </Nnet3> -- a raw
    nnet such as a speaker model's final.ext.raw."""
    w = KaldiWriter()
    w.token("<Nnet3>")
    w.raw(b"\n")
    for ln in nn.config_lines:
        w.raw(ln.encode() + b"\n")
    w.raw(b"\n")
    w.token("<NumComponents>")
    w.i32(len(nn.component_order))
    for name in nn.component_order:
        ctype, fields = nn.components[name]
        w.token("<ComponentName>")
        w.token(name)
        write_component(w, ctype, fields)
    w.token("</Nnet3>")
    with open(path, "wb") as f:
        f.write(w.bytes())


def read_nnet3_raw(path: str) -> Nnet3:
    return read_nnet3_am(KaldiReader(open(path, "rb").read()))


def write_vector_file(path: str, v):
    w = KaldiWriter()
    w.fvector(v)
    open(path, "wb").write(w.bytes())


def read_vector_file(path: str) -> np.ndarray:
    return np.asarray(KaldiReader(open(path, "rb").read()).vector(), np.float32)


def write_final_mdl(path: str, tm: TransitionModel, nn: Nnet3):
    w = KaldiWriter()
    write_transition_model(w, tm)
    write_nnet3_am(w, nn)
    with open(path, "wb") as f:
        f.write(w.bytes())


def read_final_mdl(path: str):
    data = open(path, "rb").read()
    r = KaldiReader(data)
    tm = read_transition_model(r)
    nn = read_nnet3_am(r)
    return tm, nn


# ----------------------------------------------------------------------------
# OpenFST (StdArc: tropical float weights)
# ----------------------------------------------------------------------------
@dataclass
class Fst:
    """CSR form: arcs of state s are [row[s], row[s+1])."""
    start: int
    final: np.ndarray      # float32 [S], +inf = not final
    row: np.ndarray        # int64 [S+1]
    ilabel: np.ndarray     # int32 [A]
    olabel: np.ndarray     # int32 [A]
    weight: np.ndarray     # float32 [A]
    nextstate: np.ndarray  # int32 [A]
    isyms: dict = None
    osyms: dict = None

    @property
    def num_states(self):
        return len(self.final)

    @property
    def num_arcs(self):
        return len(self.ilabel)


def _wstr(s: str) -> bytes:
    b = s.encode()
    return struct.pack("<i", len(b)) + b


def _pad16(buf: bytearray):
    while len(buf) % 16:
        buf += b"\0"


def write_const_fst(path: str, f: Fst, aligned: bool = True):
    S, A = f.num_states, f.num_arcs
    buf = bytearray()
    buf += struct.pack("<i", FST_MAGIC)
    buf += _wstr("const") + _wstr("standard")
    buf += struct.pack("<i", 2)                         # version
    buf += struct.pack("<i", K_IS_ALIGNED if aligned else 0)
    buf += struct.pack("<Q", 0)                         # properties (unknown)
    buf += struct.pack("<q", f.start)
    buf += struct.pack("<q", S)
    buf += struct.pack("<q", A)
    if aligned:
        _pad16(buf)
    st = np.zeros(S, dtype=[("w", "<f4"), ("pos", "<u4"), ("narcs", "<u4"),
                            ("nie", "<u4"), ("noe", "<u4")])
    st["w"] = f.final
    st["pos"] = f.row[:-1]
    st["narcs"] = np.diff(f.row)
    ie = (f.ilabel == 0).astype(np.int64)
    oe = (f.olabel == 0).astype(np.int64)
    cie = np.concatenate([[0], np.cumsum(ie)])
    coe = np.concatenate([[0], np.cumsum(oe)])
    st["nie"] = cie[f.row[1:]] - cie[f.row[:-1]]
    st["noe"] = coe[f.row[1:]] - coe[f.row[:-1]]
    buf += st.tobytes()
    if aligned:
        _pad16(buf)
    arcs = np.zeros(A, dtype=[("i", "<i4"), ("o", "<i4"), ("w", "<f4"), ("n", "<i4")])
    arcs["i"], arcs["o"], arcs["w"], arcs["n"] = f.ilabel, f.olabel, f.weight, f.nextstate
    buf += arcs.tobytes()
    with open(path, "wb") as fh:
        fh.write(bytes(buf))


def write_vector_fst(path: str, f: Fst):
    buf = bytearray()
    buf += struct.pack("<i", FST_MAGIC)
    buf += _wstr("vector") + _wstr("standard")
    buf += struct.pack("<i", 2) + struct.pack("<i", 0) + struct.pack("<Q", 0)
    buf += struct.pack("<q", f.start) + struct.pack("<q", f.num_states) + struct.pack("<q", f.num_arcs)
    for s in range(f.num_states):
        b, e = int(f.row[s]), int(f.row[s + 1])
        buf += struct.pack("<f", float(f.final[s])) + struct.pack("<q", e - b)
        a = np.zeros(e - b, dtype=[("i", "<i4"), ("o", "<i4"), ("w", "<f4"), ("n", "<i4")])
        a["i"], a["o"], a["w"], a["n"] = f.ilabel[b:e], f.olabel[b:e], f.weight[b:e], f.nextstate[b:e]
        buf += a.tobytes()
    with open(path, "wb") as fh:
        fh.write(bytes(buf))


ADDON_MAGIC = 446681434


def _fst_header(ftype, start, ns, na, version=2, flags=0):
    return (struct.pack("<i", FST_MAGIC) + _wstr(ftype) + _wstr("standard")
            + struct.pack("<i", version) + struct.pack("<i", flags) + struct.pack("<Q", 0)
            + struct.pack("<q", start) + struct.pack("<q", ns) + struct.pack("<q", na))


def write_lookahead_fst(path: str, f: Fst):
    """OpenFST "olabel_lookahead" add-on FST: outer header, add-on magic, the
    contained const FST (aligned, its own header), then the add-on flag.  The
    synthetic files carry no label-reachability data (flag 0); readers here
    compute reachability themselves."""
    inner_path = path + ".inner.tmp"
    write_const_fst(inner_path, f, aligned=False)
    inner = open(inner_path, "rb").read()
    os.remove(inner_path)
    buf = bytearray(_fst_header("olabel_lookahead", -1, 0, 0, version=1))
    buf += struct.pack("<i", ADDON_MAGIC)
    buf += inner
    buf += b"\0"  # have_addon = false
    with open(path, "wb") as fh:
        fh.write(bytes(buf))


def write_ngram_fst(path: str, lm: dict):
    """OpenFST "ngram" (LOUDS) backoff n-gram acceptor.  lm maps a history,
    most recent word first (a tuple; () = the unigram root, (0,) = sentence
    start), to {"fut": {word: cost}, "backoff": cost (not for the root),
    "final": cost or None}.  Every history's parent (oldest word dropped)
    must exist, and (0,) must exist (it becomes the start state 1)."""
    kids = {}
    for h in lm:
        if h:
            if h[:-1] not in lm:
                raise ValueError(f"history {h} has no parent")
            kids.setdefault(h[:-1], []).append(h)
    if (0,) not in lm:
        raise ValueError("no sentence-start history (0,)")
    order = [()]
    i = 0
    while i < len(order):
        order.extend(sorted(kids.get(order[i], []), key=lambda x: x[-1]))
        i += 1
    n = len(order)
    ctx = [1, 0]
    for h in order:
        ctx += [1] * len(kids.get(h, [])) + [0]
    fut = [0]
    fwords, fprobs, finals, finbits = [], [], [], []
    for h in order:
        f = sorted(lm[h]["fut"].items())
        fut += [1] * len(f) + [0]
        fwords += [w for w, _ in f]
        fprobs += [c for _, c in f]
        fc = lm[h].get("final")
        finbits.append(1 if fc is not None else 0)
        if fc is not None:
            finals.append(fc)

    def pack(bits):
        words = np.zeros((len(bits) + 63) // 64, np.uint64)
        for j, b in enumerate(bits):
            if b:
                words[j >> 6] |= np.uint64(1) << np.uint64(j & 63)
        return words.tobytes()

    cwords = [0] + [h[-1] for h in order[1:]] + [0]
    backoff = [0.0] + [lm[h].get("backoff", 0.0) for h in order[1:]] + [0.0]
    data = struct.pack("<QQQ", n, len(fwords), len(finals))
    data += pack(ctx) + pack(fut) + pack(finbits)
    data += np.array(cwords, "<i4").tobytes() + np.array(fwords, "<i4").tobytes()
    while len(data) % 4:
        data += b"\0"
    data += np.array(backoff, "<f4").tobytes() + np.array(finals, "<f4").tobytes()
    data += np.array(fprobs + [0.0], "<f4").tobytes()
    with open(path, "wb") as fh:
        fh.write(_fst_header("ngram", 1, n, -1, version=4) + data)


def _read_ngram_body(d, p):
    """Mirror of the C++ reader (model_io.cc ParseNgramBody): explicit arcs,
    backoff arc first for every state but the root, then the futures with
    NGramFstImpl::Transition destinations."""
    n, nfut, nfin = struct.unpack_from("<QQQ", d, p)
    p += 24

    def bits(nbits):
        nonlocal p
        nw = (nbits + 63) // 64
        w = np.frombuffer(d, "<u8", nw, p)
        p += 8 * nw
        return np.unpackbits(w.view(np.uint8), bitorder="little")[:nbits]

    ctx, fut, fin = bits(2 * n + 1), bits(nfut + n + 1), bits(n)
    cwords = np.frombuffer(d, "<i4", n + 1, p); p += 4 * (n + 1)
    fwords = np.frombuffer(d, "<i4", nfut, p); p += 4 * nfut
    # (OpenFST pads the weights to 4 bytes relative to the data block, whose
    # preceding fields are all multiples of 4 bytes: no padding)
    backoff = np.frombuffer(d, "<f4", n + 1, p); p += 4 * (n + 1)
    finals = np.frombuffer(d, "<f4", nfin, p); p += 4 * nfin
    fprob = np.frombuffer(d, "<f4", nfut + 1, p); p += 4 * (nfut + 1)
    assert ctx[0] == 1 and ctx[1] == 0
    parent = [-1] * n
    first, nch = [0] * n, [0] * n
    pos, nxt = 2, 1
    for k in range(n):
        first[k] = nxt
        while ctx[pos]:
            parent[nxt] = k
            nxt += 1
            nch[k] += 1
            pos += 1
        pos += 1
    assert nxt == n
    fbeg = [0] * (n + 1)
    pos, ones = 1, 0
    for s in range(n):
        fbeg[s] = ones
        while fut[pos]:
            ones += 1
            pos += 1
        pos += 1
    fbeg[n] = ones

    def child(k, w):
        lo, hi = first[k], first[k] + nch[k]
        j = lo + int(np.searchsorted(cwords[lo:hi], w))
        return j if j < hi and cwords[j] == w else -1

    final = np.full(n, np.inf, np.float32)
    rows, il, ol, wt, nx = [0], [], [], [], []
    nf = 0
    for s in range(n):
        if fin[s]:
            final[s] = finals[nf]
            nf += 1
        if s != 0:
            il.append(0); ol.append(0); wt.append(backoff[s]); nx.append(parent[s])
        ctxw = []
        k = s
        while k != 0:
            ctxw.append(int(cwords[k]))
            k = parent[k]
        for i in range(fbeg[s], fbeg[s + 1]):
            w = int(fwords[i])
            node = child(0, w)
            if node < 0:
                node = 0
            else:
                for j in range(len(ctxw) - 1, -1, -1):
                    if nch[node] == 0:
                        break
                    c = child(node, ctxw[j])
                    if c < 0:
                        break
                    node = c
            il.append(w); ol.append(w); wt.append(fprob[i]); nx.append(node)
        rows.append(len(il))
    return Fst(1, final, np.array(rows, np.int64), np.array(il, np.int32), np.array(ol, np.int32),
               np.array(wt, np.float32), np.array(nx, np.int32)), p


def _rstr(d, p):
    n = struct.unpack_from("<i", d, p)[0]
    return d[p + 4:p + 4 + n].decode(), p + 4 + n


def _read_symtab(d, p):
    magic = struct.unpack_from("<i", d, p)[0]
    if magic != SYMTAB_MAGIC:
        raise ValueError("bad symbol table magic")
    p += 4
    _name, p = _rstr(d, p)
    _avail, size = struct.unpack_from("<qq", d, p)
    p += 16
    tab = {}
    for _ in range(size):
        sym, p = _rstr(d, p)
        key = struct.unpack_from("<q", d, p)[0]
        p += 8
        tab[sym] = key
    return tab, p


def read_fst(path: str) -> Fst:
    d = open(path, "rb").read()
    return _parse_fst(d, 0, 0)


def _parse_fst(d, p, depth):
    magic = struct.unpack_from("<i", d, p)[0]
    if magic != FST_MAGIC:
        raise ValueError("not an OpenFST binary file")
    p += 4
    ftype, p = _rstr(d, p)
    atype, p = _rstr(d, p)
    if atype != "standard":
        raise ValueError(f"unsupported arc type {atype}")
    version, flags = struct.unpack_from("<ii", d, p)
    p += 8
    _props, start, ns, na = struct.unpack_from("<Qqqq", d, p)
    p += 32
    isyms = osyms = None
    if flags & K_HAS_ISYMBOLS:
        isyms, p = _read_symtab(d, p)
    if flags & K_HAS_OSYMBOLS:
        osyms, p = _read_symtab(d, p)
    if ftype == "const":
        if flags & K_IS_ALIGNED:
            p = (p + 15) // 16 * 16
        st = np.frombuffer(d, dtype=[("w", "<f4"), ("pos", "<u4"), ("narcs", "<u4"),
                                     ("nie", "<u4"), ("noe", "<u4")], count=ns, offset=p)
        p += 20 * ns
        if flags & K_IS_ALIGNED:
            p = (p + 15) // 16 * 16
        arcs = np.frombuffer(d, dtype=[("i", "<i4"), ("o", "<i4"), ("w", "<f4"), ("n", "<i4")],
                             count=na, offset=p)
        row = np.zeros(ns + 1, np.int64)
        row[:-1] = st["pos"]
        row[-1] = na
        # const fst stores states' arcs contiguously in state order
        return Fst(int(start), st["w"].astype(np.float32).copy(), row,
                   arcs["i"].copy(), arcs["o"].copy(), arcs["w"].copy(), arcs["n"].copy(), isyms, osyms)
    if ftype == "vector":
        finals, rows, arcl = [], [0], []
        s = 0
        while (ns < 0 and p < len(d)) or s < ns:
            fw = struct.unpack_from("<f", d, p)[0]
            n = struct.unpack_from("<q", d, p + 4)[0]
            p += 12
            a = np.frombuffer(d, dtype=[("i", "<i4"), ("o", "<i4"), ("w", "<f4"), ("n", "<i4")],
                              count=n, offset=p)
            p += 16 * n
            finals.append(fw)
            arcl.append(a)
            rows.append(rows[-1] + n)
            s += 1
        a = np.concatenate(arcl) if arcl else np.zeros(0, dtype=[("i", "<i4"), ("o", "<i4"), ("w", "<f4"), ("n", "<i4")])
        return Fst(int(start), np.array(finals, np.float32), np.array(rows, np.int64),
                   a["i"].copy(), a["o"].copy(), a["w"].copy(), a["n"].copy(), isyms, osyms)
    if ftype == "ngram":
        f, p = _read_ngram_body(d, p)
        f.isyms, f.osyms = isyms, osyms
        return f
    if ftype == "olabel_lookahead" and depth == 0:
        if struct.unpack_from("<i", d, p)[0] != ADDON_MAGIC:
            raise ValueError("bad add-on header")
        f = _parse_fst(d, p + 4, 1)
        if f.osyms is None:
            f.osyms = osyms
        return f
    raise ValueError(f"unsupported fst type {ftype}")


def read_symbol_table(path: str) -> dict:
    """words.txt: '<symbol> <id>' per line -> {id: symbol}."""
    out = {}
    for ln in open(path, encoding="utf-8"):
        parts = ln.split()
        if len(parts) >= 2:
            out[int(parts[1])] = parts[0]
    return out


def parse_conf(path: str) -> dict:
    """Kaldi ParseOptions config file: '--key=value' per line, '#' comments."""
    out = {}
    for ln in open(path):
        ln = ln.split("#", 1)[0].strip()
        if not ln.startswith("--"):
            continue
        if "=" in ln:
            k, v = ln[2:].split("=", 1)
        else:
            k, v = ln[2:], "true"
        out[k.strip()] = v.strip()
    return out


# ----------------------------------------------------------------------------
# i-vector extractor files (Kaldi gmm/diag-gmm.cc, ivector/ivector-extractor.cc)
# ----------------------------------------------------------------------------
@dataclass
class DiagGmm:
    gconsts: np.ndarray        # [G]
    weights: np.ndarray        # [G]
    means_invvars: np.ndarray  # [G, D]
    inv_vars: np.ndarray       # [G, D]


def diag_gmm_from_params(weights, means, variances) -> DiagGmm:
    inv = 1.0 / variances
    D = means.shape[1]
    gc = (np.log(weights) - 0.5 * (D * np.log(2 * np.pi) + np.log(variances).sum(1) +
                                   (means * means * inv).sum(1)))
    return DiagGmm(gc.astype(np.float32), weights.astype(np.float32),
                   (means * inv).astype(np.float32), inv.astype(np.float32))


def write_diag_gmm(path: str, g: DiagGmm):
    w = KaldiWriter()
    w.token("<DiagGMM>")
    w.token("<GCONSTS>"); w.fvector(g.gconsts)
    w.token("<WEIGHTS>"); w.fvector(g.weights)
    w.token("<MEANS_INVVARS>"); w.fmatrix(g.means_invvars)
    w.token("<INV_VARS>"); w.fmatrix(g.inv_vars)
    w.token("</DiagGMM>")
    open(path, "wb").write(w.bytes())


def read_diag_gmm(path: str) -> DiagGmm:
    r = KaldiReader(open(path, "rb").read())
    r.expect("<DiagGMM>")
    r.expect("<GCONSTS>"); gc = r.vector()
    r.expect("<WEIGHTS>"); wt = r.vector()
    r.expect("<MEANS_INVVARS>"); mi = r.matrix()
    r.expect("<INV_VARS>"); iv = r.matrix()
    r.expect("</DiagGMM>")
    return DiagGmm(gc, wt, mi, iv)


@dataclass
class IvectorExtractor:
    w: np.ndarray          # [G, S] weight projection (unused online)
    w_vec: np.ndarray      # [G]
    M: list                # G x [D, S]
    sigma_inv: list        # G x [D, D] (full, symmetric)
    prior_offset: float


def write_ivector_extractor(path: str, x: IvectorExtractor):
    w = KaldiWriter()
    w.token("<IvectorExtractor>")
    w.token("<w>"); w.dmatrix(x.w)
    w.token("<w_vec>"); w.dvector(x.w_vec)
    w.token("<M>"); w.i32(len(x.M))
    for m in x.M:
        w.dmatrix(m)
    w.token("<SigmaInv>")
    for s in x.sigma_inv:
        w.dspmatrix(s)
    w.token("<IvectorOffset>"); w.f64(x.prior_offset)
    w.token("</IvectorExtractor>")
    open(path, "wb").write(w.bytes())


def read_ivector_extractor(path: str) -> IvectorExtractor:
    r = KaldiReader(open(path, "rb").read())
    r.expect("<IvectorExtractor>")
    r.expect("<w>"); wm = r.matrix64()
    r.expect("<w_vec>"); wv = r.dvector64()
    r.expect("<M>")
    n = r.i32()
    M = [r.matrix64() for _ in range(n)]
    r.expect("<SigmaInv>")
    S = [r.spmatrix64() for _ in range(n)]
    r.expect("<IvectorOffset>")
    off = r.f64()
    r.expect("</IvectorExtractor>")
    return IvectorExtractor(wm, wv, M, S, off)


def write_matrix_file(path: str, m, double=False):
    w = KaldiWriter()
    (w.dmatrix if double else w.fmatrix)(m)
    open(path, "wb").write(w.bytes())


def read_matrix_file(path: str) -> np.ndarray:
    return KaldiReader(open(path, "rb").read()).matrix64()


# ----------------------------------------------------------------------------
# Kaldi ConstArpaLm (lm/const-arpa-lm.{h,cc}) binary object, as read by
# vosk-api_amd/csrc/rescore.cc
# ----------------------------------------------------------------------------
def write_const_arpa(path: str, ngrams: dict, bos: int, eos: int, unk: int, order: int):
    """ngrams: {(w1, ..., wn): (logprob, backoff_logprob)} natural log, every
    prefix of an n-gram present.  States: one per n-gram that is a unigram or
    a history of a longer n-gram: [logprob][backoff][num children]
    [(word, child info)...] with children sorted by word; child info = 2 *
    (child offset - parent offset) + 1 for children with a state, else the
    child's logprob bits with the lowest bit cleared.  Words without a
    unigram state get offset -1 (Kaldi's ConstArpaLm::Write); the first
    state sits at offset 0."""
    kids = {}
    for ng in ngrams:
        if len(ng) > 1:
            kids.setdefault(ng[:-1], []).append(ng)
    has_state = {ng for ng in ngrams if len(ng) == 1 or ng in kids}
    order_states = sorted((ng for ng in has_state if len(ng) == 1))
    frontier = list(order_states)
    while frontier:
        nxt = []
        for h in frontier:
            for c in sorted(kids.get(h, []), key=lambda x: x[-1]):
                if c in has_state:
                    nxt.append(c)
        order_states += nxt
        frontier = nxt
    pos, p = {}, 0
    for st in order_states:
        pos[st] = p
        p += 3 + 2 * len(kids.get(st, []))
    arr = np.zeros(p, np.int32)

    def fbits(x):
        return int(np.array([x], np.float32).view(np.int32)[0])

    for st in order_states:
        q = pos[st]
        lp, bo = ngrams[st]
        ch = sorted(kids.get(st, []), key=lambda x: x[-1])
        arr[q], arr[q + 1], arr[q + 2] = fbits(lp), fbits(bo), len(ch)
        for i, c in enumerate(ch):
            arr[q + 3 + 2 * i] = c[-1]
            if c in has_state:
                arr[q + 4 + 2 * i] = 2 * (pos[c] - q) + 1
            else:
                arr[q + 4 + 2 * i] = fbits(ngrams[c][0]) & ~1
    num_words = max(w for ng in ngrams for w in ng) + 1
    uni = [pos.get((w,), -1) for w in range(num_words)]
    b = bytearray(b"\0B")

    def tok(t):
        b.extend(t.encode() + b" ")

    def i32(v):
        b.extend(b"\x04" + struct.pack("<i", v))

    def i64(v):
        b.extend(b"\x08" + struct.pack("<q", v))

    tok("<ConstArpaLm>"); tok("<LmInfo>")
    i32(bos); i32(eos); i32(unk); i32(order)
    tok("</LmInfo>"); tok("<LmStates>")
    i64(len(arr))
    b.extend(arr.tobytes())
    tok("</LmStates>"); tok("<LmUnigram>")
    i32(num_words)
    for u in uni:
        i64(u)
    tok("</LmUnigram>"); tok("<LmOverflow>")
    i32(0)
    tok("</LmOverflow>"); tok("</ConstArpaLm>")
    with open(path, "wb") as f:
        f.write(bytes(b))
