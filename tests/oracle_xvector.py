"""CPU restatement of the speaker x-vector path (TEST INFRASTRUCTURE ONLY).

Follows the reference's GetSpkVector (src/recognizer.cc:356-419) and speaker
model (src/spk_model.cc:17-32): the speaker MFCC (the C oracle's orc_mfcc with
the speaker options, snip-edges=false framing), the non-silence frame
selection (frame i kept iff decoder frame i / 3 is non-silence on the best
path), sliding-window CMN (orc_sliding_cmn), the frame-level x-vector layers
(orc_nnet_forward up to the statistics input, input columns zero-padded to a
multiple of 8 exactly as the product pads them), statistics pooling over the
computable frames, the head, mean subtraction, transform.mat and the length
normalisation (orc_xvector_tail).  Parity unpinned against Kaldi: no speaker
model exists here; tools/make_synth_model.py writes a synthetic one.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "vosk-api_amd", "tools"))
import kaldi_formats as kf  # noqa: E402
import np_kaldi as nk  # noqa: E402
import oracle_py  # noqa: E402


class OrcXvec(C.Structure):
    _fields_ = [("stats_dim", C.c_int), ("nlog", C.c_int), ("stddevs", C.c_int),
                ("var_floor", C.c_float), ("nops", C.c_int), ("kind", C.c_void_p),
                ("in_dim", C.c_void_p), ("out_dim", C.c_void_p), ("w_off", C.c_void_p),
                ("b_off", C.c_void_p), ("params", C.c_void_p), ("embed_dim", C.c_int),
                ("out_dim_final", C.c_int), ("mean", C.c_void_p), ("transform", C.c_void_p)]


AFFINE = {"AffineComponent", "NaturalGradientAffineComponent", "FixedAffineComponent",
          "LinearComponent"}


def _pad_input(nn: kf.Nnet3, D: int, Dp: int) -> kf.Nnet3:
    """Zero columns after every block of an affine input that reads 'input'
    (xvector.cc PadInput)."""
    if Dp == D:
        return nn
    lines = []
    comps = dict(nn.components)
    for ln in nn.config_lines:
        kind, kv = nk.split_config_line(ln)
        if kind == "input-node" and kv["name"] == "input":
            ln = ln.replace(f"dim={D}", f"dim={Dp}")
        lines.append(ln)
        if kind != "component-node":
            continue
        d = nk.parse_descriptor(kv["input"])
        terms = d[1] if d[0] == "append" else [d]
        blocks = []
        for t in terms:
            b = t
            while b[0] in ("offset", "round"):
                b = b[1]
            is_in = b[0] == "node" and b[1] == "input"
            blocks.append((D if is_in else None, is_in, t))
        if not any(b[1] for b in blocks):
            continue
        ctype, fields = comps[kv["component"]]
        fl = dict(fields)
        key = "<LinearParams>" if "<LinearParams>" in fl else "<Params>"
        W = fl[key]
        if ctype == "TdnnComponent":
            nb = len(fl["<TimeOffsets>"])
            widths = [(D, True)] * nb
        else:
            n_in = sum(1 for b in blocks if b[1])
            if len(blocks) - n_in > 1:
                raise NotImplementedError("more than one non-input block next to the input")
            rest = W.shape[1] - D * n_in
            widths = [(D, True) if is_in else (rest, False) for _w, is_in, _t in blocks]
        cols, src = [], 0
        for w, is_in in widths:
            cols.append(W[:, src:src + w])
            if is_in:
                cols.append(np.zeros((W.shape[0], Dp - D), np.float32))
            src += w
        assert src == W.shape[1]
        Wp = np.ascontiguousarray(np.concatenate(cols, axis=1), np.float32)
        fl[key] = Wp
        comps[kv["component"]] = (ctype, fl)
    return kf.Nnet3(lines, comps, nn.component_order, nn.left_context, nn.right_context, nn.priors)


class OracleSpk:
    def __init__(self, spk_dir):
        self.conf = kf.parse_conf(os.path.join(spk_dir, "mfcc.conf"))
        self.mo = nk.MfccOpts(self.conf)
        self.opts = oracle_py.mfcc_opts(self.conf)
        nn = kf.read_nnet3_raw(os.path.join(spk_dir, "final.ext.raw"))
        self.mean = kf.read_vector_file(os.path.join(spk_dir, "mean.vec"))
        self.transform = np.ascontiguousarray(kf.read_matrix_file(os.path.join(spk_dir, "transform.mat")),
                                              np.float32)
        self.D = self.mo.num_ceps
        self.Dp = (self.D + 7) // 8 * 8
        nn = _pad_input(nn, self.D, self.Dp)
        g = nk.NnetGraph(nn)
        ext = pool = None
        for n, nd in g.nodes.items():
            if nd["kind"] == "component":
                t = nn.components[nd["component"]][0]
                if t == "StatisticsExtractionComponent":
                    ext = n
                if t == "StatisticsPoolingComponent":
                    pool = n
        src = g.nodes[ext]["input"]
        assert src[0] == "node"
        pf = dict(nn.components[g.nodes[pool]["component"]][1])
        self.pool_left, self.pool_right = pf.get("<LeftContext>", 0), pf.get("<RightContext>", 0)
        self.nlog = pf.get("<NumLogCountFeatures>", 0)
        self.stddevs = bool(pf.get("<OutputStddevs>", False))
        self.var_floor = float(np.float32(pf.get("<VarianceFloor>", 1e-10)))
        lines = [ln for ln in nn.config_lines if not ln.startswith("output-node")]
        lines.append(f"output-node name=output input={src[1]}")
        fnn = kf.Nnet3(lines, nn.components, nn.component_order)
        self.nn_components = nn.components
        self.frames = oracle_py.OracleNet(fnn, acoustic_scale=1.0, fss=1)
        self.stats_in = self.frames.out_dim
        # the head chain pool -> output
        kinds, ind, outd, woff, boff, params = [], [], [], [], [], []
        off = [0]

        def addp(a):
            a = np.ascontiguousarray(a, np.float32).ravel()
            o = off[0]
            params.append(a)
            off[0] += a.size
            return o

        dim = self.nlog + self.stats_in * (2 if self.stddevs else 1)
        out_src = g.nodes["output"]["input"]
        cur = pool
        while not (out_src[0] == "node" and out_src[1] == cur):
            nxt = None
            for n, nd in g.nodes.items():
                if nd["kind"] != "component":
                    continue
                d = nd["input"]
                if d[0] == "round":
                    d = d[1]
                if d[0] == "node" and d[1] == cur:
                    nxt = n
            ctype, f = nn.components[g.nodes[nxt]["component"]]
            f = dict(f)
            if ctype in AFFINE:
                W = f.get("<LinearParams>", f.get("<Params>"))
                kinds.append(1); ind.append(dim); outd.append(W.shape[0])
                woff.append(addp(W))
                boff.append(addp(f["<BiasParams>"]) if "<BiasParams>" in f else -1)
                dim = W.shape[0]
            elif ctype == "RectifiedLinearComponent":
                kinds.append(2); ind.append(dim); outd.append(dim); woff.append(0); boff.append(-1)
            elif ctype == "BatchNormComponent":
                s, o = oracle_py.bn_scale_offset_f32(f)
                kinds.append(3); ind.append(dim); outd.append(dim)
                woff.append(addp(s)); boff.append(addp(o))
            cur = nxt
        self.embed_dim = dim
        self.k = dict(kind=np.array(kinds, np.int32), ind=np.array(ind, np.int32),
                      outd=np.array(outd, np.int32), woff=np.array(woff, np.int64),
                      boff=np.array(boff, np.int64),
                      params=np.concatenate(params) if params else np.zeros(1, np.float32),
                      mean=np.ascontiguousarray(self.mean, np.float32), tr=self.transform)
        k = self.k
        self.x = OrcXvec(self.stats_in, self.nlog, int(self.stddevs), self.var_floor, len(kinds),
                         k["kind"].ctypes.data, k["ind"].ctypes.data, k["outd"].ctypes.data,
                         k["woff"].ctypes.data, k["boff"].ctypes.data, k["params"].ctypes.data,
                         dim, self.transform.shape[0], k["mean"].ctypes.data, k["tr"].ctypes.data)

    def features(self, wave):
        return oracle_py.mfcc(wave, self.conf)

    def select(self, nframes, first_frame, keep):
        return [i for i in range(max(0, first_frame), nframes)
                if (i - first_frame) // 3 < len(keep) and keep[(i - first_frame) // 3]]

    def cmn(self, feats):
        f = np.ascontiguousarray(feats, np.float32)
        out = np.zeros_like(f)
        oracle_py.lib().orc_sliding_cmn(C.c_void_p(f.ctypes.data), C.c_int(f.shape[0]), C.c_int(f.shape[1]),
                                        C.c_int(300), C.c_void_p(out.ctypes.data))
        return out

    def xvector(self, wave, first_frame, keep):
        """-> (x-vector or None, number of selected frames)"""
        feats = self.features(wave)
        rows = self.select(feats.shape[0], first_frame, keep)
        if len(rows) < 50:
            return None, len(rows)
        x = self.cmn(feats[rows])
        xp = np.zeros((x.shape[0], self.Dp), np.float32)
        xp[:, :self.D] = x
        fr = self.frames.forward(xp)
        # computable frames of the frame-level part inside the pooling window
        lc, rc = self.frames_context()
        r0 = max(lc, -self.pool_left)
        r1 = min(len(rows) - 1 - rc, self.pool_right)
        out = np.zeros(self.transform.shape[0], np.float32)
        fr = np.ascontiguousarray(fr, np.float32)
        rc_ = oracle_py.lib().orc_xvector_tail(C.byref(self.x), C.c_void_p(fr.ctypes.data),
                                               C.c_int(fr.shape[1]), C.c_int(r0), C.c_int(r1),
                                               C.c_void_p(out.ctypes.data))
        assert rc_ == 0
        return out, len(rows)

    def frames_context(self):
        """Left / right context of the frame-level part (Kaldi
        ComputeSimpleNnetContext at t = 0), from the descriptor offsets."""
        g = self.frames.graph
        comps = self.nn_components
        memo = {}

        def ctx(n):
            if n in memo:
                return memo[n]
            nd = g.nodes[n]
            if nd["kind"] == "input":
                r = (0, 0)
            elif nd["kind"] == "dimrange":
                r = ctx(nd["src"])
            else:
                r = dctx(nd["input"])
                if nd["kind"] == "component":
                    ctype, f = comps[nd["component"]]
                    if ctype == "TdnnComponent":
                        offs = [int(o) for o in dict(f)["<TimeOffsets>"]]
                        r = (max(r[0] - o for o in offs), max(r[1] + o for o in offs))
            memo[n] = r
            return r

        def dctx(d):
            k = d[0]
            if k == "node":
                return ctx(d[1])
            if k == "offset":
                lo, hi = dctx(d[1])
                return (lo - d[2], hi + d[2])
            if k in ("append", "sum"):
                rs = [dctx(e) for e in d[1]]
                return (max(x[0] for x in rs), max(x[1] for x in rs))
            if k == "scale":
                return dctx(d[2])
            if k in ("round", "ifdefined", "replace_index"):
                return dctx(d[1])
            return (-(10 ** 9), -(10 ** 9))

        lo, hi = ctx("output")
        return max(0, lo), max(0, hi)
