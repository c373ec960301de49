"""ctypes driver for the C oracle (oracle/liboracle.so) -- test infrastructure.

Parses a model directory with the independent Python readers in
``vosk-api_amd/tools`` (not the product's C++ readers), builds the oracle's
node program and graph arrays, and runs MFCC / nnet3 forward / token passing
on the CPU.  Used only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.
"""
from __future__ import annotations

import ctypes as C
import math
import os
import subprocess
import sys

import numpy as np

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(REPO, "vosk-api_amd", "tools"))
import kaldi_formats as kf  # noqa: E402
import np_kaldi as nk  # noqa: E402

LIB_PATH = os.path.join(REPO, "oracle", "build", "liboracle.so")


def load_lib():
    if not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle")])
    lib = C.CDLL(LIB_PATH)
    lib.orc_mfcc.restype = C.c_int
    lib.orc_mfcc_num_frames.restype = C.c_int
    lib.orc_feat_dim.restype = C.c_int
    lib.orc_online_cmvn.restype = None
    lib.orc_online_cmvn.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                    C.c_void_p]
    lib.orc_logf.restype = C.c_float
    lib.orc_logf.argtypes = [C.c_float]
    lib.orc_nnet_forward.restype = C.c_int
    lib.orc_decode.restype = C.c_int
    lib.orc_resample_num_outputs.restype = C.c_long
    lib.orc_resample_num_outputs.argtypes = [C.c_int, C.c_int, C.c_long]
    lib.orc_resample.restype = C.c_long
    lib.orc_resample.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_long, C.c_void_p, C.c_long]
    lib.orc_ivector_extract.restype = C.c_int
    lib.orc_ivector_extract.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                        C.c_int, C.c_void_p]
    lib.orc_ivector_extract_w.restype = C.c_int
    lib.orc_ivector_extract_w.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                          C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.orc_expf.restype = C.c_float
    lib.orc_expf.argtypes = [C.c_float]
    return lib


_lib = None


def resample(x, rate_in, rate_out):
    """Whole-signal windowed-sinc resampling with end flush (oracle.c)."""
    x = np.ascontiguousarray(x, np.float32)
    n = lib().orc_resample_num_outputs(rate_in, rate_out, len(x))
    out = np.zeros(max(n, 1), np.float32)
    got = lib().orc_resample(rate_in, rate_out, x.ctypes.data, len(x), out.ctypes.data, len(out))
    assert got == n, (got, n)
    return out[:n]


def lib():
    global _lib
    if _lib is None:
        _lib = load_lib()
    return _lib


class OrcMfccOpts(C.Structure):
    _fields_ = [("samp_freq", C.c_float), ("frame_shift_ms", C.c_float),
                ("frame_length_ms", C.c_float), ("preemph_coeff", C.c_float),
                ("low_freq", C.c_float), ("high_freq", C.c_float),
                ("cepstral_lifter", C.c_float), ("blackman_coeff", C.c_float),
                ("num_bins", C.c_int), ("num_ceps", C.c_int), ("use_energy", C.c_int),
                ("remove_dc_offset", C.c_int), ("window_type", C.c_int),
                ("round_to_power_of_two", C.c_int), ("fbank", C.c_int),
                ("use_log_fbank", C.c_int), ("use_power", C.c_int), ("snip_edges", C.c_int)]


def mfcc_opts(conf: dict, fbank: bool = False) -> OrcMfccOpts:
    o = nk.MfccOpts(conf, fbank)
    wt = {"povey": 0, "hamming": 1, "hanning": 2, "rectangular": 3, "blackman": 4}[o.window_type]
    return OrcMfccOpts(o.samp_freq, o.frame_shift_ms, o.frame_length_ms, o.preemph,
                       o.low_freq, o.high_freq, o.cepstral_lifter, o.blackman_coeff,
                       o.num_bins, o.num_ceps, int(o.use_energy), int(o.remove_dc), wt,
                       int(o.round_pow2), int(fbank), int(o.use_log_fbank), int(o.use_power),
                       int(o.snip_edges))


def online_cmvn(feats, gstats, window=600, global_frames=200) -> np.ndarray:
    """C oracle's Kaldi OnlineCmvn (global stats, mean normalization)."""
    f = np.ascontiguousarray(feats, np.float32)
    g = np.ascontiguousarray(gstats, np.float64)
    out = np.zeros_like(f)
    if f.shape[0]:
        lib().orc_online_cmvn(g.ctypes.data, f.shape[1], window, global_frames, f.ctypes.data,
                              f.shape[0], out.ctypes.data)
    return out


def recognizer_pieces(n, chunk, rate):
    """Sample counts the reference Recognizer processes per decoding advance
    when fed `chunk` samples per AcceptWaveform call: 0.2 s steps inside each
    call (src/recognizer.cc:305-311)."""
    step = int(rate * 0.2)
    out = []
    for i in range(0, n, chunk):
        m = min(chunk, n - i)
        out += [min(step, m - j) for j in range(0, m, step)]
    return out


def resample_num_outputs(rate_in, rate_out, n, flush):
    """Kaldi LinearResample::GetNumOutputSamples (feat/resample.cc [K]):
    without flush, outputs whose filter window reaches past the input wait."""
    tick = rate_in * rate_out // math.gcd(rate_in, rate_out)
    interval = n * (tick // rate_in)
    if not flush:
        cutoff = 0.5 * min(rate_in, rate_out)
        interval -= int(math.floor(6 / (2.0 * cutoff) * tick))
    if interval <= 0:
        return 0
    tpo = tick // rate_out
    last = interval // tpo
    if last * tpo == interval:
        last -= 1
    return last + 1


def mfcc_num_frames(num_samples, conf: dict, fbank: bool = False) -> int:
    o = mfcc_opts(conf, fbank)
    return int(lib().orc_mfcc_num_frames(C.byref(o), C.c_long(num_samples)))


def mfcc(wave, conf: dict, fbank: bool = False) -> np.ndarray:
    """The model's front end: MFCC, or log fbank with fbank=True."""
    o = mfcc_opts(conf, fbank)
    w = np.ascontiguousarray(wave, np.float32)
    n = lib().orc_mfcc_num_frames(C.byref(o), C.c_long(len(w)))
    out = np.zeros((max(n, 0), lib().orc_feat_dim(C.byref(o))), np.float32)
    if n > 0:
        lib().orc_mfcc(C.byref(o), w.ctypes.data_as(C.c_void_p), C.c_long(len(w)),
                       out.ctypes.data_as(C.c_void_p))
    return out


# ----------------------------------------------------------------------------
# nnet3 program
# ----------------------------------------------------------------------------
class OrcIvectorModel(C.Structure):
    _fields_ = [("feat_dim", C.c_int), ("left", C.c_int), ("right", C.c_int),
                ("lda_rows", C.c_int), ("lda_cols", C.c_int), ("lda", C.c_void_p),
                ("cmvn", C.c_void_p), ("cmn_window", C.c_int), ("global_frames", C.c_int),
                ("num_gauss", C.c_int), ("gconsts", C.c_void_p), ("means_invvars", C.c_void_p),
                ("inv_vars", C.c_void_p), ("ivec_dim", C.c_int), ("M", C.c_void_p),
                ("sigma_inv", C.c_void_p), ("prior_offset", C.c_double),
                ("max_count", C.c_double), ("num_gselect", C.c_int), ("num_cg_iters", C.c_int),
                ("min_post", C.c_float), ("posterior_scale", C.c_float)]


class OracleIvector:
    """ivector/ directory -> the C oracle's online i-vector extractor
    (configuration of the reference, src/model.cc:247-263)."""

    def __init__(self, ivector_dir):
        lda = kf.read_matrix_file(os.path.join(ivector_dir, "final.mat"))
        cmvn = kf.read_matrix_file(os.path.join(ivector_dir, "global_cmvn.stats"))
        ubm = kf.read_diag_gmm(os.path.join(ivector_dir, "final.dubm"))
        ie = kf.read_ivector_extractor(os.path.join(ivector_dir, "final.ie"))
        sp = kf.parse_conf(os.path.join(ivector_dir, "splice.conf"))
        self.keep = dict(
            lda=np.ascontiguousarray(lda, np.float32), cmvn=np.ascontiguousarray(cmvn, np.float64),
            gc=np.ascontiguousarray(ubm.gconsts, np.float32),
            mi=np.ascontiguousarray(ubm.means_invvars, np.float32),
            iv=np.ascontiguousarray(ubm.inv_vars, np.float32),
            M=np.ascontiguousarray(np.stack(ie.M), np.float64),
            SI=np.ascontiguousarray(np.stack(ie.sigma_inv), np.float64))
        k = self.keep
        left, right = int(sp.get("left-context", 4)), int(sp.get("right-context", 4))
        D = cmvn.shape[1] - 1
        self.dim = ie.M[0].shape[1]
        self.m = OrcIvectorModel(D, left, right, lda.shape[0], lda.shape[1], k["lda"].ctypes.data,
                                 k["cmvn"].ctypes.data, 600, 200, ubm.gconsts.size,
                                 k["gc"].ctypes.data, k["mi"].ctypes.data, k["iv"].ctypes.data,
                                 self.dim, k["M"].ctypes.data, k["SI"].ctypes.data,
                                 ie.prior_offset, 100.0, 5, 15, 0.025, 0.1)

    def extract(self, feats, requests):
        feats = np.ascontiguousarray(feats, np.float32)
        T = feats.shape[0]
        req = np.ascontiguousarray(requests, np.int32)
        tr = np.full(len(req), T, np.int32)
        out = np.zeros((len(req), self.dim), np.float32)
        lib().orc_ivector_extract(C.byref(self.m), feats.ctypes.data, T, req.ctypes.data,
                                  tr.ctypes.data, len(req), out.ctypes.data)
        return out


    def extract_weighted(self, feats, requests, entries):
        """Silence-weighted extraction: entries[q] = the (frame, delta weight)
        list request q applies, in order (empty for requests that reuse the
        current i-vector)."""
        feats = np.ascontiguousarray(feats, np.float32)
        T = feats.shape[0]
        req = np.ascontiguousarray(requests, np.int32)
        tr = np.full(len(req), T, np.int32)
        off = np.zeros(len(req) + 1, np.int32)
        off[1:] = np.cumsum([len(e) for e in entries])
        fr = np.ascontiguousarray([f for e in entries for f, _ in e] or [0], np.int32)
        w = np.ascontiguousarray([x for e in entries for _, x in e] or [0], np.float32)
        out = np.zeros((len(req), self.dim), np.float32)
        rc = lib().orc_ivector_extract_w(C.byref(self.m), feats.ctypes.data, T, req.ctypes.data,
                                         tr.ctypes.data, len(req), off.ctypes.data, fr.ctypes.data,
                                         w.ctypes.data, out.ctypes.data)
        assert rc == 0, rc
        return out


class SilenceWeighting:
    """Restatement of Kaldi's OnlineSilenceWeighting (online2/online-ivector-
    feature.cc [K]; not vendored in the reference) as the reference's
    Recognizer drives it: silence weight 1e-3 and the endpoint silence phones
    (src/model.cc:230-231), ComputeCurrentTraceback + GetDeltaWeights before
    every decoding advance (src/recognizer.cc:226-237), a new object per
    decoder segment (src/recognizer.cc:188-191).  max_state_duration is
    unset in the reference (no duration rule)."""

    def __init__(self, is_silence_tid, silence_weight=1e-3, fss=3):
        self.is_sil = is_silence_tid
        self.sw = np.float32(silence_weight)
        self.fss = fss
        self.info = []  # [token, tid, current_weight]

    def compute_current_traceback(self, tids, toks):
        n, prev = len(tids), len(self.info)
        if prev < n:
            self.info += [[-1, -1, np.float32(0)] for _ in range(n - prev)]
        if prev > n and self.info[n][1] != -1:
            raise RuntimeError("number of frames decoded decreased")
        for fr in range(n - 1, -1, -1):
            if self.info[fr][0] == toks[fr]:
                break  # unchanged from here back
            self.info[fr][0] = toks[fr]
            self.info[fr][1] = tids[fr]

    def get_delta_weights(self, num_frames_ready, first_decoder_frame):
        fs = self.fss
        ndec = (num_frames_ready - first_decoder_frame + fs - 1) // fs
        prev = len(self.info)
        if len(self.info) < ndec:
            self.info += [[-1, -1, np.float32(0)] for _ in range(ndec - len(self.info))]
        begin = max(0, prev - 100)
        nout = len(self.info) - begin
        out = []
        if nout <= 0:
            return out
        fw = [np.float32(1.0)] * nout
        if self.info[begin][1] == -1:
            w = self.sw if begin == 0 else self.info[begin - 1][2]
            fw = [w] * nout
        else:
            for o in range(nout):
                tid = self.info[begin + o][1]
                if tid == -1:
                    fw[o] = fw[o - 1]
                elif self.is_sil(tid):
                    fw[o] = self.sw
        for o in range(nout):
            fi = self.info[begin + o]
            diff = np.float32(fw[o] - fi[2])
            fi[2] = fw[o]
            if diff != 0 or o + 1 == nout:
                out += [(first_decoder_frame + (begin + o) * fs + i, diff) for i in range(fs)]
        return out


class OrcNet(C.Structure):
    _fields_ = [("num_nodes", C.c_int), ("kind", C.c_void_p), ("dim", C.c_void_p),
                ("in_dim", C.c_void_p), ("w_off", C.c_void_p), ("b_off", C.c_void_p),
                ("s_off", C.c_void_p), ("o_off", C.c_void_p), ("params", C.c_void_p),
                ("toff_begin", C.c_void_p), ("toff_count", C.c_void_p), ("toffs", C.c_void_p),
                ("prog_begin", C.c_void_p), ("prog", C.c_void_p), ("progf", C.c_void_p),
                ("output_node", C.c_int), ("fss", C.c_int), ("acoustic_scale", C.c_float),
                ("ivec", C.c_void_p), ("ivec_of_time", C.c_void_p), ("ivec_t0", C.c_int),
                ("ivec_ntimes", C.c_int), ("ivec_dim", C.c_int)]


def bn_scale_offset_f32(fields):
    """Double-precision derivation rounded once (matches the product)."""
    mean = np.asarray(fields["<StatsMean>"], np.float64)
    var = np.asarray(fields["<StatsVar>"], np.float64)
    eps = float(np.float32(fields.get("<Epsilon>", 1e-3)))
    tr = float(np.float32(fields.get("<TargetRms>", 1.0)))
    s = tr / np.sqrt(np.maximum(var, 0.0) + eps)
    return s.astype(np.float32), (-mean * s).astype(np.float32)


class OracleNet:
    """Whole-utterance nnet3 forward on the CPU oracle."""

    AFFINE = {"FixedAffineComponent", "AffineComponent", "NaturalGradientAffineComponent",
              "LinearComponent", "TdnnComponent"}
    IDENT = {"NoOpComponent", "GeneralDropoutComponent", "DropoutComponent",
             "SpecAugmentTimeMaskComponent"}

    def __init__(self, nn: kf.Nnet3, acoustic_scale=1.0, fss=3):
        g = nk.NnetGraph(nn)
        self.graph = g
        comps = {k: (t, dict(f) if isinstance(f, list) else f) for k, (t, f) in nn.components.items()}
        # topological order from the output
        order, seen = [], set()

        def deps(d, out):
            if d[0] == "node":
                out.append(d[1])
            elif d[0] in ("append", "sum"):
                for e in d[1]:
                    deps(e, out)
            elif d[0] in ("offset", "replace_index", "round", "ifdefined"):
                deps(d[1], out)
            elif d[0] == "scale":
                deps(d[2], out)

        def topo(n):
            if n in seen:
                return
            seen.add(n)
            nd = g.nodes[n]
            ds = []
            if nd["kind"] in ("component", "output"):
                deps(nd["input"], ds)
            if nd["kind"] == "dimrange":
                ds.append(nd["src"])
            for x in ds:
                topo(x)
            order.append(n)

        topo("output")
        out_desc = g.nodes["output"]["input"]
        assert out_desc[0] == "node"
        # nodes of the program: input first, then component nodes (dim-range
        # nodes are resolved into column offsets)
        prog_nodes = ["input"] + [n for n in order if g.nodes[n]["kind"] == "component"]
        idx = {n: i for i, n in enumerate(prog_nodes)}
        params = []
        poff = [0]

        def addp(a):
            a = np.ascontiguousarray(a, np.float32).ravel()
            off = poff[0]
            params.append(a)
            poff[0] += a.size
            return off

        kind, dim, in_dim, w_off, b_off, s_off, o_off = [], [], [], [], [], [], []
        toff_begin, toff_count, toffs = [], [], []
        prog_begin, prog, progf = [], [], []

        def node_dim(n):
            nd = g.nodes[n]
            if nd["kind"] == "input":
                return nd["dim"]
            if nd["kind"] == "dimrange":
                return nd["dim"]
            t, f = comps[nd["component"]]
            if "<LinearParams>" in f:
                return f["<LinearParams>"].shape[0]
            if "<Params>" in f:
                return f["<Params>"].shape[0]
            return f["<Dim>"]

        def desc_dim(d):
            if d[0] == "node":
                return node_dim(d[1])
            if d[0] == "append":
                return sum(desc_dim(e) for e in d[1])
            if d[0] == "const":
                return d[2]
            if d[0] == "scale":
                return desc_dim(d[2])
            return desc_dim(d[1])

        def resolve(n):
            nd = g.nodes[n]
            if nd["kind"] == "dimrange":
                src, col = resolve(nd["src"])
                return src, col + nd["offset"]
            return idx[n], 0

        def compile_desc(d, toff, code):
            k = d[0]
            if k == "node":
                ni, col = resolve(d[1])
                code.append((0, ni, toff, col))
            elif k == "offset":
                compile_desc(d[1], toff + d[2], code)
            elif k == "ifdefined":
                compile_desc(d[1], toff, code)
            elif k == "scale":
                compile_desc(d[2], toff, code)
                progf.append(d[1])
                code.append((1, 0, 0, len(progf) - 1))
            elif k == "sum":
                compile_desc(d[1][0], toff, code)
                for e in d[1][1:]:
                    compile_desc(e, toff, code)
                    code.append((2, 0, 0, 0))
            elif k == "const":
                progf.append(d[1])
                code.append((3, 0, 0, len(progf) - 1))
            elif k == "replace_index" and d[1] == ("node", "ivector"):
                code.append((4, 0, 0, 0))  # the row's chunk i-vector
                self.ivector_consumers.add(cur_node[0])
            else:
                raise ValueError(f"descriptor {k} unsupported by the oracle")

        self.ivector_consumers = set()
        cur_node = [None]
        for n in prog_nodes:
            cur_node[0] = n
            if n == "input":
                kind.append(0); dim.append(g.nodes[n]["dim"]); in_dim.append(0)
                w_off.append(-1); b_off.append(-1); s_off.append(-1); o_off.append(-1)
                toff_begin.append(0); toff_count.append(0)
                prog_begin.append(len(prog)); prog.append(0)
                continue
            nd = g.nodes[n]
            t, f = comps[nd["component"]]
            d = nd["input"]
            parts = d[1] if d[0] == "append" else [d]
            prog_begin.append(len(prog))
            prog.append(len(parts))
            for p in parts:
                code = []
                compile_desc(p, 0, code)
                prog.append(desc_dim(p))
                prog.append(len(code))
                for c in code:
                    prog.extend(c)
            in_dim.append(desc_dim(d))
            dim.append(node_dim(n))
            wo = bo = so = oo = -1
            if t == "TdnnComponent":
                toff_begin.append(len(toffs)); toff_count.append(len(f["<TimeOffsets>"]))
                toffs.extend(int(x) for x in f["<TimeOffsets>"])
            else:
                toff_begin.append(0); toff_count.append(0)
            if t in self.AFFINE:
                kind.append(1)
                W = f["<LinearParams>"] if "<LinearParams>" in f else f["<Params>"]
                wo = addp(W)
                b = f.get("<BiasParams>")
                if b is not None and len(b):
                    bo = addp(b)
            elif t == "RectifiedLinearComponent":
                kind.append(2)
            elif t == "BatchNormComponent":
                kind.append(3)
                s, o = bn_scale_offset_f32(f)
                reps = dim[-1] // len(s)
                so, oo = addp(np.tile(s, reps)), addp(np.tile(o, reps))
            elif t == "ScaleAndOffsetComponent":
                kind.append(3)
                reps = dim[-1] // len(f["<Scales>"])
                so, oo = addp(np.tile(f["<Scales>"], reps)), addp(np.tile(f["<Offsets>"], reps))
            elif t in self.IDENT:
                kind.append(4)
            else:
                raise ValueError(f"component {t} unsupported by the oracle")
            w_off.append(wo); b_off.append(bo); s_off.append(so); o_off.append(oo)

        self.arrays = dict(
            kind=np.array(kind, np.int32), dim=np.array(dim, np.int32),
            in_dim=np.array(in_dim, np.int32), w_off=np.array(w_off, np.int64),
            b_off=np.array(b_off, np.int64), s_off=np.array(s_off, np.int64),
            o_off=np.array(o_off, np.int64),
            params=np.concatenate(params) if params else np.zeros(1, np.float32),
            toff_begin=np.array(toff_begin, np.int32), toff_count=np.array(toff_count, np.int32),
            toffs=np.array(toffs if toffs else [0], np.int32),
            prog_begin=np.array(prog_begin, np.int32), prog=np.array(prog, np.int32),
            progf=np.array(progf if progf else [0.0], np.float32))
        a = self.arrays
        self.out_dim = int(dim[idx[out_desc[1]]])
        self.fss = fss
        self.net = OrcNet(len(prog_nodes), *(a[k].ctypes.data for k in
                                              ("kind", "dim", "in_dim", "w_off", "b_off",
                                               "s_off", "o_off", "params", "toff_begin",
                                               "toff_count", "toffs", "prog_begin", "prog",
                                               "progf")),
                          idx[out_desc[1]], fss, acoustic_scale)

    def forward(self, feats: np.ndarray, ivecs=None, ivec_of_time=None, ivec_t0=0) -> np.ndarray:
        """ivecs: [chunks][dim] i-vectors; ivec_of_time[t - ivec_t0]: the chunk
        whose i-vector the rows at time t use."""
        feats = np.ascontiguousarray(feats, np.float32)
        T = feats.shape[0]
        rows = (T + self.fss - 1) // self.fss
        out = np.zeros((rows, self.out_dim), np.float32)
        if ivecs is not None:
            iv = np.ascontiguousarray(ivecs, np.float32)
            it = np.ascontiguousarray(ivec_of_time, np.int32)
            self._keep = (iv, it)
            self.net.ivec, self.net.ivec_of_time = iv.ctypes.data, it.ctypes.data
            self.net.ivec_t0, self.net.ivec_ntimes, self.net.ivec_dim = ivec_t0, len(it), iv.shape[1]
        else:
            if self.ivector_consumers:
                raise ValueError("this nnet has an i-vector input: pass ivecs / ivec_of_time")
            self.net.ivec = self.net.ivec_of_time = None
            self.net.ivec_ntimes = 0
        r = lib().orc_nnet_forward(C.byref(self.net), feats.ctypes.data_as(C.c_void_p),
                                   C.c_int(T), out.ctypes.data_as(C.c_void_p))
        assert r == rows, r
        return out


# ----------------------------------------------------------------------------
# decoder
# ----------------------------------------------------------------------------
class OrcGraph(C.Structure):
    _fields_ = [("num_states", C.c_int), ("start", C.c_int), ("arc_begin", C.c_void_p),
                ("eps_begin", C.c_void_p), ("ilabel", C.c_void_p), ("olabel", C.c_void_p),
                ("nextstate", C.c_void_p), ("weight", C.c_void_p), ("final_cost", C.c_void_p),
                ("tid2pdf", C.c_void_p)]


def decoder_order(batch=False):
    """The token-passing semantics the GPU decoder runs (VOSK_AMD_DEC_ORDER,
    as the engine reads it): "kaldi" (LatticeFasterDecoder's sequential
    order: the default of engines, KaldiRecognizers and BatchModel lanes) or
    "parallel" (the order-independent form, opt-in).  `batch` is kept for
    the call sites: both paths default to Kaldi's order."""
    v = os.environ.get("VOSK_AMD_DEC_ORDER", "kaldi").strip().lower()
    return "parallel" if v in ("parallel", "0", "order-independent") else "kaldi"


class OrcDecOpts(C.Structure):
    _fields_ = [("beam", C.c_float), ("beam_delta", C.c_float), ("max_active", C.c_int),
                ("min_active", C.c_int), ("hash_size", C.c_int), ("lazy_row", C.c_void_p),
                ("lazy_next", C.c_void_p), ("lazy_disc", C.c_void_p), ("lazy_expanded", C.c_void_p),
                ("lazy_count", C.c_void_p)]


class LazyState:
    """OpenFST's lazy numbering carried across decodes of one stream (a
    recognizer's ComposeFst outlives its decoder's InitDecoding; the GPU keeps
    it per stream slot): ids, expanded flags, next id (0: not started)."""

    def __init__(self, graph):
        row = graph.lazy[0]
        self.disc = np.full(graph.num_states + int(row[-1]), -1, np.int32)
        self.exp = np.zeros(graph.num_states, np.int8)
        self.count = np.zeros(1, np.int32)

    def copy(self):
        c = LazyState.__new__(LazyState)
        c.disc, c.exp, c.count = self.disc.copy(), self.exp.copy(), self.count.copy()
        return c


class OrcDecResult(C.Structure):
    _fields_ = [("ntok", C.c_void_p), ("best", C.c_void_p), ("cutoff", C.c_void_p),
                ("next_cutoff", C.c_void_p), ("arcs_emit", C.c_void_p), ("path", C.c_void_p),
                ("path_cap", C.c_int), ("path_len", C.c_int), ("best_cost", C.c_double),
                ("best_tot", C.c_float), ("end_state", C.c_int),
                ("final_relative_cost", C.c_float),
                ("lat_frame_begin", C.c_void_p), ("lat_tok_state", C.c_void_p),
                ("lat_tok_cost", C.c_void_p), ("lat_tok_cap", C.c_int), ("lat_ntok", C.c_int),
                ("lat_link_frame", C.c_void_p), ("lat_link_src", C.c_void_p),
                ("lat_link_arc", C.c_void_p), ("lat_link_ac", C.c_void_p),
                ("lat_link_cap", C.c_int), ("lat_nlink", C.c_int), ("lat_cost_offset", C.c_void_p),
                ("hash_size", C.c_int),
                ("probe_frames", C.c_void_p), ("nprobe", C.c_int), ("probe_path", C.c_void_p),
                ("probe_path_cap", C.c_longlong), ("probe_off", C.c_void_p), ("probe_frc", C.c_void_p)]


class OracleGraph:
    """CSR graph with per-state emitting arcs first (stable), as the product."""

    def __init__(self, fst: kf.Fst, tid2pdf: np.ndarray):
        S = fst.num_states
        src = np.repeat(np.arange(S), np.diff(fst.row))
        eps = (fst.ilabel == 0).astype(np.int64)
        order = np.lexsort((np.arange(fst.num_arcs), eps, src))
        self.ilabel = np.ascontiguousarray(fst.ilabel[order], np.int32)
        self.olabel = np.ascontiguousarray(fst.olabel[order], np.int32)
        self.weight = np.ascontiguousarray(fst.weight[order], np.float32)
        self.nextstate = np.ascontiguousarray(fst.nextstate[order], np.int32)
        self.arc_begin = np.ascontiguousarray(fst.row, np.int64)
        n_emit = np.bincount(src, weights=1 - eps, minlength=S).astype(np.int64)
        self.eps_begin = np.ascontiguousarray(self.arc_begin[:-1] + n_emit, np.int64)
        self.final = np.ascontiguousarray(fst.final, np.float32)
        self.tid2pdf = np.ascontiguousarray(tid2pdf, np.int32)
        self.start = fst.start
        self.num_states = S
        self.lazy = None  # OpenFST lazy numbering table (OracleModel loads graph/lazy_ids.npz)
        self.g = OrcGraph(S, fst.start, self.arc_begin.ctypes.data, self.eps_begin.ctypes.data,
                          self.ilabel.ctypes.data, self.olabel.ctypes.data,
                          self.nextstate.ctypes.data, self.weight.ctypes.data,
                          self.final.ctypes.data, self.tid2pdf.ctypes.data)

    def decode(self, llh: np.ndarray, beam=13.0, max_active=7000, min_active=200,
               beam_delta=0.5, use_final=True, lattice=False, kaldi=None, hash_size=0, probes=None,
               lattice_caps=None, lazy="auto", lazy_state=None):
        """kaldi=True: the Kaldi-sequential restatement (orc_decode_kaldi:
        HashList order, running emitting cutoff, LIFO epsilon queue), the
        GPU decoder's default; False: the order-independent form (the GPU's
        VOSK_AMD_DEC_ORDER=parallel mode); None: as the environment selects
        (decoder_order()).  hash_size: the Kaldi HashList size the decoder
        starts with (0: a new decoder); out["hash_size"] is its size at the end.
        probes: ascending frame counts; out["probes"] is a
        list of (path without final costs, final relative cost) after each,
        from the same single pass (the endpoint checks of a segment).
        lazy: (row, nextstate) of the graph in its own arc order -- Kaldi
        order buckets by OpenFST's lazy ComposeFst numbering (orc_dec_opts
        lazy_row / lazy_next) instead of the graph's state ids; "auto": the
        graph's own lazy table (graph/lazy_ids.npz of an expanded lookahead
        model, as the GPU decoder uses by default; VOSK_AMD_LAZY_IDS=0
        turns both off), None: off."""
        if isinstance(lazy, str):
            off = os.environ.get("VOSK_AMD_LAZY_IDS", "1").strip() == "0"
            lazy = None if off else self.lazy
        # lazy_state: a LazyState updated in place (the numbering carried
        # from the stream's earlier decodes), None: a fresh numbering
        if kaldi is None:
            kaldi = decoder_order() == "kaldi"
        llh = np.ascontiguousarray(llh, np.float32)
        F = llh.shape[0]
        ntok = np.zeros(F + 1, np.int32)
        best = np.zeros(F + 1, np.float32)
        cut = np.zeros(max(F, 1), np.float32)
        ncut = np.zeros(max(F, 1), np.float32)
        ex = np.zeros(max(F, 1), np.int64)
        cap = 4 * F + 64
        path = np.zeros(cap, np.int32)
        res = OrcDecResult(ntok.ctypes.data, best.ctypes.data, cut.ctypes.data, ncut.ctypes.data,
                           ex.ctypes.data, path.ctypes.data, cap, 0, 0.0, 0.0, -1, 0.0)
        if lattice:
            tcap, lcap = lattice_caps if lattice_caps else (4000 * (F + 1) + 4096, 16000 * (F + 1) + 16384)
            lat = dict(frame_begin=np.zeros(F + 2, np.int32), tok_state=np.zeros(tcap, np.int32),
                       tok_cost=np.zeros(tcap, np.float32), link_frame=np.zeros(lcap, np.int32),
                       link_src=np.zeros(lcap, np.int32), link_arc=np.zeros(lcap, np.int32),
                       link_ac=np.zeros(lcap, np.float32), cost_offset=np.zeros(F + 1, np.float32))
            res.lat_frame_begin = lat["frame_begin"].ctypes.data
            res.lat_tok_state, res.lat_tok_cost = lat["tok_state"].ctypes.data, lat["tok_cost"].ctypes.data
            res.lat_tok_cap = tcap
            res.lat_link_frame, res.lat_link_src = lat["link_frame"].ctypes.data, lat["link_src"].ctypes.data
            res.lat_link_arc, res.lat_link_ac = lat["link_arc"].ctypes.data, lat["link_ac"].ctypes.data
            res.lat_link_cap = lcap
            res.lat_cost_offset = lat["cost_offset"].ctypes.data
        if probes is not None:
            pf = np.ascontiguousarray(probes, np.int32)
            assert np.all(np.diff(pf) >= 0)
            pcap = int(4 * pf.astype(np.int64).clip(0).sum() + 64)
            ppath = np.zeros(pcap, np.int32)
            poff = np.zeros(len(pf) + 1, np.int64)
            pfrc = np.zeros(max(len(pf), 1), np.float32)
            res.probe_frames, res.nprobe = pf.ctypes.data, len(pf)
            res.probe_path, res.probe_path_cap = ppath.ctypes.data, pcap
            res.probe_off, res.probe_frc = poff.ctypes.data, pfrc.ctypes.data
        o = OrcDecOpts(beam, beam_delta, max_active, min_active, int(hash_size))
        if lazy is not None:
            lrow = np.ascontiguousarray(lazy[0], np.int64)
            lnext = np.ascontiguousarray(lazy[1], np.int32)
            o.lazy_row, o.lazy_next = lrow.ctypes.data, lnext.ctypes.data
            if lazy_state is not None and kaldi:
                o.lazy_disc = lazy_state.disc.ctypes.data
                o.lazy_expanded = lazy_state.exp.ctypes.data
                o.lazy_count = lazy_state.count.ctypes.data
        ls0 = lazy_state.copy() if (lazy_state is not None and lattice) else None
        fn = lib().orc_decode_kaldi if kaldi else lib().orc_decode
        rc = fn(C.byref(self.g), llh.ctypes.data_as(C.c_void_p), C.c_int(F),
                              C.c_int(llh.shape[1]), C.byref(o), C.c_int(int(use_final)),
                              C.byref(res))
        p = path[:res.path_len].copy()
        words = [int(self.olabel[a]) for a in p if self.olabel[a] != 0]
        out = dict(rc=rc, ntok=ntok, best=best, cutoff=cut[:F], next_cutoff=ncut[:F],
                   arcs_emit=ex[:F], path=p, words=words, best_cost=res.best_cost,
                   best_tot=res.best_tot, end_state=res.end_state,
                   final_relative_cost=res.final_relative_cost, hash_size=res.hash_size)
        if probes is not None:
            assert poff[-1] <= pcap
            out["probes"] = [(ppath[poff[i]:poff[i + 1]].copy(), float(pfrc[i])) for i in range(len(pf))]
        if lattice and (res.lat_ntok > res.lat_tok_cap or res.lat_nlink > res.lat_link_cap):
            # the counts past the capacities are exact: decode again with room
            if ls0 is not None:  # the numbering as it was before this attempt
                lazy_state.disc[:], lazy_state.exp[:], lazy_state.count[:] = ls0.disc, ls0.exp, ls0.count
            return self.decode(llh, beam, max_active, min_active, beam_delta, use_final, lattice, kaldi,
                               hash_size, probes, lattice_caps=(res.lat_ntok + 1, res.lat_nlink + 1),
                               lazy=lazy, lazy_state=lazy_state)
        if lattice:
            nt, nl = res.lat_ntok, res.lat_nlink
            out["lattice"] = dict(
                frame_begin=lat["frame_begin"], tok_state=lat["tok_state"][:nt],
                tok_cost=lat["tok_cost"][:nt], link_frame=lat["link_frame"][:nl],
                link_src=lat["link_src"][:nl], link_arc=lat["link_arc"][:nl],
                link_ac=lat["link_ac"][:nl], cost_offset=lat["cost_offset"])
        return out


class OracleModel:
    """All oracle pieces for a model directory (V2 layout).  fpc: looped
    chunk size in input frames (defaults to the model's decodable option,
    20 rounded up to the subsampling factor, as the single-stream
    Recognizer); it matters only with i-vectors (one i-vector per chunk)."""

    def __init__(self, model_dir: str, fpc=None):
        self.dir = model_dir
        # front end (src/model.cc:218-228): mfcc.conf, else fbank.conf;
        # am/global_cmvn.stats adds online CMVN on the nnet input (:265-269)
        mconf = os.path.join(model_dir, "conf", "mfcc.conf")
        self.fbank = not os.path.exists(mconf)
        self.mfcc_conf = kf.parse_conf(mconf if not self.fbank else
                                       os.path.join(model_dir, "conf", "fbank.conf"))
        cpath = os.path.join(model_dir, "am", "global_cmvn.stats")
        self.global_cmvn = kf.read_matrix_file(cpath) if os.path.exists(cpath) else None
        self.model_conf = kf.parse_conf(os.path.join(model_dir, "conf", "model.conf"))
        self.tm, self.nn = kf.read_final_mdl(os.path.join(model_dir, "am", "final.mdl"))
        self.fst = kf.read_fst(os.path.join(model_dir, "graph", "HCLG.fst"))
        self.words = kf.read_symbol_table(os.path.join(model_dir, "graph", "words.txt"))
        mc = self.model_conf
        self.acoustic_scale = float(mc.get("acoustic-scale", 0.1))
        self.fss = int(mc.get("frame-subsampling-factor", 1))
        self.beam = float(mc.get("beam", 16.0))
        self.max_active = int(mc.get("max-active", 2 ** 31 - 1))
        self.min_active = int(mc.get("min-active", 200))
        self.beam_delta = float(mc.get("beam-delta", 0.5))
        self.net = OracleNet(self.nn, self.acoustic_scale, self.fss)
        self.graph = OracleGraph(self.fst, self.tm.tid2pdf)
        lz = os.path.join(model_dir, "graph", "lazy_ids.npz")
        if os.path.exists(lz):  # an expanded lookahead model (oracle_graph.write_lazy)
            with np.load(lz) as z:
                self.graph.lazy = (np.ascontiguousarray(z["row"], np.int64), np.ascontiguousarray(z["next"], np.int32))
        fpc = int(fpc or mc.get("frames-per-chunk", 20))
        self.fpc = fpc + (-fpc) % self.fss
        idir = os.path.join(model_dir, "ivector")
        self.ivector = OracleIvector(idir) if os.path.exists(os.path.join(idir, "final.ie")) else None
        if self.ivector is not None:
            self._ivector_schedule()

    def _ivector_schedule(self):
        """Looped-chunk bookkeeping: right context, and for the rows of the
        i-vector's consumer node the chunk that first computes them (chunk 0,
        then a periodic window of fpc times per chunk)."""
        g, fss, fpc = self.net.graph, self.fss, self.fpc
        opc = fpc // fss
        self.right_context = max(nk.needed_times(g, [0], "input"))
        assert len(self.net.ivector_consumers) == 1
        node = next(iter(self.net.ivector_consumers))
        sets = [nk.needed_times(g, [c * fpc + fss * i for i in range(opc)], node) for c in range(3)]
        new1 = sorted(sets[1] - sets[0])
        new2 = sorted(sets[2] - sets[1] - sets[0])
        assert new2 == [t + fpc for t in new1] and new1 == list(range(new1[0], new1[0] + fpc)), \
            "i-vector consumer is not periodic"
        self._iv_first0 = min(sets[0])
        self._iv_new1 = new1[0]

    def ivector_requests(self, T):
        """Frame whose i-vector each chunk uses: the last input frame of the
        chunk incl. right context (DecodableNnetLoopedOnline), clamped to the
        utterance (the engine waits for the splice's 3 right-context frames)."""
        opc = self.fpc // self.fss
        nch = -(-(-(-T // self.fss)) // opc) if T > 0 else 0
        return [min((c + 1) * self.fpc + self.right_context, T) - 1 for c in range(nch)]

    def ivectors(self, feats):
        return self.ivector.extract(feats, self.ivector_requests(feats.shape[0]))

    def _ivec_of_time(self, T, nch):
        t0 = self._iv_first0
        t1 = nch * self.fpc + self._iv_new1 + self.fpc
        times = np.arange(t0, t1)
        c = np.where(times < self._iv_new1, 0, 1 + (times - self._iv_new1) // self.fpc)
        return np.minimum(c, max(nch - 1, 0)).astype(np.int32), t0

    def features(self, wave):
        """Raw front-end features (the i-vector extractor's input)."""
        return mfcc(wave, self.mfcc_conf, self.fbank)

    def nnet_features(self, feats):
        """The nnet's input: the features, CMVN-normalized with global stats."""
        return feats if self.global_cmvn is None else online_cmvn(feats, self.global_cmvn)

    def loglikes(self, wave):
        return self.loglikes_feats(self.features(wave))

    def loglikes_feats(self, raw):
        feats = self.nnet_features(raw)
        if self.ivector is None or feats.shape[0] == 0:
            return self.net.forward(feats)
        iv = self.ivectors(raw)
        ivt, t0 = self._ivec_of_time(feats.shape[0], len(iv))
        return self.net.forward(feats, iv, ivt, t0)

    def decode_llh(self, llh, use_final=True, hash_size=0, kaldi=None):
        return self.graph.decode(llh, self.beam, self.max_active, self.min_active,
                                 self.beam_delta, use_final, hash_size=hash_size, kaldi=kaldi)

    def online(self, wave, chunk=None, rate=16000, silence_weighting=True, endpoints=False):
        """The single-stream Recognizer's online flow (src/recognizer.cc:297-
        323, FinalResult :818-830) with the engine's chunk schedule: per
        piece, features of all samples so far, UpdateSilenceWeights from the
        best path of the frames decoded so far, then every chunk that became
        ready (its i-vector request applies the queued delta weights of
        frames <= the request).  Returns per-chunk i-vectors, the LLH rows,
        and the final decode.

        endpoints=True: after every AcceptWaveform call of `chunk` samples the
        endpoint rules run on the decoder segment (EndpointDetected,
        :318; tests/oracle_endpoint.py); when they fire the caller takes
        Result() and the next call starts with CleanUp (:188-224): the
        decoder restarts at the frames decoded so far and the silence
        weighting restarts with first decoder frame = frame offset * 3
        (features and i-vector statistics continue).  Adds "segments":
        [(first frame, end frame)] with the last one ended by FinalResult."""
        assert self.ivector is not None
        wave = np.asarray(wave, np.float32)
        model_rate = int(float(self.mfcc_conf.get("sample-frequency", 16000)))
        feats_all = self.features(wave if rate == model_rate else resample(wave, rate, model_rate))
        fss, fpc, R = self.fss, self.fpc, self.right_context
        right = self.ivector.m.right
        opc = fpc // fss
        tm, g = self.tm, self.graph
        sil = set(int(p) for p in str(self.model_conf.get("endpoint.silence-phones", "")).replace(",", ":").split(":") if p)
        sw = SilenceWeighting(lambda tid: int(tm.tid2phone[tid]) in sil, 1e-3, fss)
        active = silence_weighting and bool(sil)
        pending, weighted = [], False
        reqs, ents = [], []
        c, done, dec = 0, 0, 0
        seg0, segs, reset_next = 0, [], False
        # Kaldi order: InitDecoding keeps the decoder's HashList size, so a
        # segment starts with the size the previous one grew to
        hs_seg, hs_last, seg_hash = 0, 0, []
        if endpoints:
            import oracle_endpoint as OE
            rules, _ = OE.endpoint_config(self.model_conf)
            shift = np.float32(np.float32(0.01) * np.float32(fss))
        ivecs = np.zeros((0, self.ivector.dim), np.float32)
        llh = np.zeros((0, self.net.out_dim), np.float32)
        calls, n = [], 0
        step = int(rate * 0.2)
        ch = chunk or len(wave)
        for i in range(0, len(wave), ch):
            m = min(ch, len(wave) - i)
            calls.append([n + j + min(step, m - j) for j in range(0, m, step)])
            n += m
        calls.append(None)  # FinalResult
        call_log = []
        for call in calls:
            if call is not None and reset_next:  # CleanUp: InitDecoding, new OnlineSilenceWeighting
                seg0, reset_next = dec, False
                hs_seg = hs_last
                sw = SilenceWeighting(lambda tid: int(tm.tid2phone[tid]) in sil, 1e-3, fss)
            log = dict(segment=len(segs), seg0=seg0, pieces=[], endpoint=False, final=call is None)
            call_log.append(log)
            for n, fin in ([(x, False) for x in call] if call is not None else [(len(wave), True)]):
                n_out = n if rate == model_rate else resample_num_outputs(rate, model_rate, n, fin)
                T = mfcc_num_frames(n_out, self.mfcc_conf, self.fbank)
                ready = T if fin else max(0, T - right)
                if active and ready > 0 and (weighted or done == 0):
                    tids, toks = [], []
                    if dec > seg0:
                        r = self.decode_llh(llh[seg0:dec], use_final=False, hash_size=hs_seg)
                        for a in r["path"]:
                            if g.ilabel[a] != 0:
                                tids.append(int(g.ilabel[a]))
                                toks.append(int(np.searchsorted(g.arc_begin, a, side="right") - 1))
                    sw.compute_current_traceback(tids, toks)
                    pending += sw.get_delta_weights(ready, seg0 * fss)
                    weighted = True
                need_out = -(-T // fss) if fin else 0
                new = False
                while True:
                    ok = (T > 0 and c * opc < need_out) if fin else T >= (c + 1) * fpc + R + right
                    if not ok:
                        break
                    f = min((c + 1) * fpc + R, T) - 1
                    e = []
                    if f >= done and weighted:
                        pending.sort()
                        e = [x for x in pending if x[0] <= f]
                        pending = [x for x in pending if x[0] > f]
                    reqs.append(f)
                    ents.append(e)
                    done = max(done, f + 1)
                    dec += min(opc, need_out - c * opc) if fin else opc
                    c += 1
                    new = True
                if new:
                    feats = feats_all[:T]
                    if weighted:
                        ivecs = self.ivector.extract_weighted(feats, reqs, ents)
                    else:
                        ivecs = self.ivector.extract(feats, reqs)
                    nf = self.nnet_features(feats)
                    ivt, t0 = self._ivec_of_time(T, len(ivecs))
                    llh = self.net.forward(nf, ivecs, ivt, t0)[:dec]
                log["pieces"].append(dec)  # an AdvanceDecoding ends here
            if endpoints and call is not None and dec > seg0:
                r = self.decode_llh(llh[seg0:dec], use_final=False, hash_size=hs_seg)
                hs_last = r["hash_size"]
                ts = OE.trailing_silence(r["path"], g.ilabel, tm.tid2phone, sil)
                if OE.rules_fire(rules, dec - seg0, ts, shift, r["final_relative_cost"]):
                    segs.append((seg0, dec))
                    seg_hash.append(hs_seg)
                    reset_next = True
                    log["endpoint"] = True
        if endpoints:
            segs.append((seg0, dec))
            seg_hash.append(hs_seg)
        r = self.decode_llh(llh[seg0:], hash_size=hs_seg) if endpoints else self.decode_llh(llh)
        return dict(ivectors=ivecs, llh=llh, decode=r, requests=reqs, entries=ents, segments=segs,
                    segment_hash_sizes=seg_hash, calls=call_log)

    def recognize(self, wave):
        r = self.decode_llh(self.loglikes(wave))
        r["text"] = " ".join(self.words[w] for w in r["words"])
        return r
