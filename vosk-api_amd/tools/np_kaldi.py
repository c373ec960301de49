"""Independent float64 numpy restatement of the Kaldi front-end and nnet3
forward, used (1) by the synthetic-model generator to calibrate BatchNorm
statistics and (2) by tests as a tolerance-level cross-check of the bit-exact
C oracle in ``oracle/`` (which is the parity checker proper).

Algorithms follow Kaldi (third-party, not vendored in /root/reference):
``feat/feature-window.cc`` (framing, DC removal, pre-emphasis, Povey window),
``feat/mel-computations.cc`` (mel banks), ``feat/feature-mfcc.cc`` (log, DCT,
lifter) and ``nnet3/nnet-descriptor.cc`` (Append/Sum/Scale/Offset/
ReplaceIndex).  Reference call sites: ``src/model.cc:218-221`` (mfcc.conf),
``src/model.cc:233-246`` (nnet + looped decodable).
"""
from __future__ import annotations

import math
import os
import re

import numpy as np


# ----------------------------------------------------------------------------
# MFCC
# ----------------------------------------------------------------------------
class MfccOpts:
    """MfccOptions, or FbankOptions with fbank=True (feat/feature-fbank.h:
    use-energy defaults to false, log mel energies, power spectrum)."""

    def __init__(self, conf: dict | None = None, fbank: bool = False):
        c = conf or {}
        self.fbank = fbank
        self.use_log_fbank = c.get("use-log-fbank", "true") == "true"
        self.use_power = c.get("use-power", "true") == "true"
        self.samp_freq = float(c.get("sample-frequency", 16000))
        self.frame_shift_ms = float(c.get("frame-shift", 10))
        self.frame_length_ms = float(c.get("frame-length", 25))
        self.dither = float(c.get("dither", 1.0))
        self.preemph = float(c.get("preemphasis-coefficient", 0.97))
        self.remove_dc = c.get("remove-dc-offset", "true") == "true"
        self.window_type = c.get("window-type", "povey")
        self.round_pow2 = c.get("round-to-power-of-two", "true") == "true"
        self.blackman_coeff = float(c.get("blackman-coeff", 0.42))
        self.snip_edges = c.get("snip-edges", "true") == "true"
        self.num_bins = int(c.get("num-mel-bins", 23))
        self.num_ceps = int(c.get("num-ceps", 13))
        self.use_energy = c.get("use-energy", "false" if fbank else "true") == "true"
        self.low_freq = float(c.get("low-freq", 20))
        self.high_freq = float(c.get("high-freq", 0))
        self.cepstral_lifter = float(c.get("cepstral-lifter", 22))

    @property
    def feat_dim(self):
        return self.num_bins + int(self.use_energy) if self.fbank else self.num_ceps

    @property
    def shift(self):
        return int(self.samp_freq * 0.001 * self.frame_shift_ms)

    @property
    def length(self):
        return int(self.samp_freq * 0.001 * self.frame_length_ms)

    @property
    def padded(self):
        n = self.length
        return 1 << (n - 1).bit_length() if self.round_pow2 else n


def num_frames(n_samples, o: MfccOpts):
    if n_samples < o.length:
        return 0
    return 1 + (n_samples - o.length) // o.shift


def window_fn(o: MfccOpts):
    n = o.length
    a = 2 * math.pi / (n - 1)
    i = np.arange(n, dtype=np.float64)
    if o.window_type == "povey":
        return (0.5 - 0.5 * np.cos(a * i)) ** 0.85
    if o.window_type == "hamming":
        return 0.54 - 0.46 * np.cos(a * i)
    if o.window_type == "hanning":
        return 0.5 - 0.5 * np.cos(a * i)
    if o.window_type == "rectangular":
        return np.ones(n)
    if o.window_type == "blackman":
        return o.blackman_coeff - 0.5 * np.cos(a * i) + (0.5 - o.blackman_coeff) * np.cos(2 * a * i)
    raise ValueError(o.window_type)


def mel_scale(f):
    return 1127.0 * np.log(1.0 + np.asarray(f, np.float64) / 700.0)


def mel_banks(o: MfccOpts):
    """Dense [num_bins, padded/2] float64 weight matrix (FFT bins 0..N/2-1)."""
    nfft = o.padded // 2
    nyq = 0.5 * o.samp_freq
    hi = o.high_freq if o.high_freq > 0 else nyq + o.high_freq
    width = o.samp_freq / o.padded
    ml, mh = mel_scale(o.low_freq), mel_scale(hi)
    delta = (mh - ml) / (o.num_bins + 1)
    W = np.zeros((o.num_bins, nfft))
    for b in range(o.num_bins):
        left, center, right = ml + b * delta, ml + (b + 1) * delta, ml + (b + 2) * delta
        for i in range(nfft):
            m = mel_scale(width * i)
            if left < m < right:
                W[b, i] = (m - left) / (center - left) if m <= center else (right - m) / (right - center)
    return W


def dct_matrix(o: MfccOpts):
    n = o.num_bins
    M = np.zeros((o.num_ceps, n))
    M[0, :] = math.sqrt(1.0 / n)
    for k in range(1, o.num_ceps):
        for j in range(n):
            M[k, j] = math.sqrt(2.0 / n) * math.cos(math.pi / n * (j + 0.5) * k)
    return M


def lifter(o: MfccOpts):
    q = o.cepstral_lifter
    i = np.arange(o.num_ceps, dtype=np.float64)
    return 1.0 + 0.5 * q * np.sin(math.pi * i / q) if q != 0 else np.ones(o.num_ceps)


def online_cmvn(feats, gstats, window=600, global_frames=200):
    """Kaldi OnlineCmvn (mean only) with global stats [2][D+1]: sliding
    window sums smoothed with up to global_frames of the global mean."""
    feats = np.asarray(feats, np.float64)
    T, D = feats.shape
    g = np.asarray(gstats, np.float64)
    out = np.zeros_like(feats)
    for t in range(T):
        lo = max(0, t + 1 - window)
        st = feats[lo:t + 1].sum(0)
        cnt = float(t + 1 - lo)
        if cnt < window:
            sc = min(window - cnt, global_frames) / g[0, D]
            st = st + sc * g[0, :D]
            cnt = cnt + sc * g[0, D]
        out[t] = feats[t] - st / cnt
    return out


def features(wave, o: MfccOpts):
    """The front end the options describe: MFCC or (log) fbank."""
    return fbank(wave, o) if o.fbank else mfcc(wave, o)


def fbank(wave, o: MfccOpts):
    """FbankComputer::Compute: [log raw energy,] log mel energies."""
    wave = np.asarray(wave, np.float64)
    nf = num_frames(len(wave), o)
    win = window_fn(o)
    W = mel_banks(o)
    off = int(o.use_energy)
    out = np.zeros((nf, o.num_bins + off))
    for f in range(nf):
        x = wave[f * o.shift: f * o.shift + o.length].copy()
        if o.remove_dc:
            x -= x.mean()
        energy = max(float(np.dot(x, x)), np.finfo(np.float32).eps)
        if o.preemph != 0:
            x[1:] = x[1:] - o.preemph * x[:-1]
            x[0] -= o.preemph * x[0]
        x *= win
        X = np.fft.rfft(x, o.padded)
        p = (X.real ** 2 + X.imag ** 2)[: o.padded // 2]
        if not o.use_power:
            p = np.sqrt(p)
        e = W @ p
        if o.use_log_fbank:
            e = np.log(np.maximum(e, np.finfo(np.float32).eps))
        out[f, off:] = e
        if o.use_energy:
            out[f, 0] = math.log(energy)
    return out


def mfcc(wave, o: MfccOpts):
    """wave: float array (int16-range values).  Dither is NOT applied here."""
    wave = np.asarray(wave, np.float64)
    nf = num_frames(len(wave), o)
    win = window_fn(o)
    W = mel_banks(o)
    D = dct_matrix(o)
    L = lifter(o)
    out = np.zeros((nf, o.num_ceps))
    for f in range(nf):
        x = wave[f * o.shift: f * o.shift + o.length].copy()
        if o.remove_dc:
            x -= x.mean()
        energy = max(float(np.dot(x, x)), np.finfo(np.float32).eps)
        if o.preemph != 0:
            x[1:] = x[1:] - o.preemph * x[:-1]
            x[0] -= o.preemph * x[0]
        x *= win
        X = np.fft.rfft(x, o.padded)
        p = (X.real ** 2 + X.imag ** 2)[: o.padded // 2]
        e = W @ p
        e = np.log(np.maximum(e, np.finfo(np.float32).eps))
        c = (D @ e) * L
        if o.use_energy:
            c[0] = math.log(energy)
        out[f] = c
    return out


# ----------------------------------------------------------------------------
# nnet3 descriptors and forward
# ----------------------------------------------------------------------------
def split_config_line(line: str):
    """'component-node name=x component=y input=Append(a, b)' ->
    ('component-node', {'name':'x', ...})."""
    line = line.strip()
    kind, _, rest = line.partition(" ")
    out = {}
    i = 0
    n = len(rest)
    while i < n:
        while i < n and rest[i] == " ":
            i += 1
        if i >= n:
            break
        eq = rest.index("=", i)
        key = rest[i:eq].strip()
        j = eq + 1
        depth = 0
        while j < n and (depth > 0 or rest[j] != " "):
            if rest[j] == "(":
                depth += 1
            elif rest[j] == ")":
                depth -= 1
            j += 1
        out[key] = rest[eq + 1:j]
        i = j
    return kind, out


_tok_re = re.compile(r"\s*([A-Za-z_][A-Za-z0-9_.\-]*|-?[0-9.]+(?:e-?[0-9]+)?|[(),])")


def parse_descriptor(s: str):
    """Parse into nested tuples:
    ('node', name) | ('offset', d, t) | ('scale', a, d) | ('sum', [d...]) |
    ('append', [d...]) | ('replace_index', d, var, val) | ('round', d, m) |
    ('const', value, dim) | ('ifdefined', d)."""
    toks = []
    pos = 0
    while pos < len(s):
        m = _tok_re.match(s, pos)
        if not m:
            raise ValueError(f"bad descriptor {s!r} at {pos}")
        toks.append(m.group(1))
        pos = m.end()
        while pos < len(s) and s[pos] == " ":
            pos += 1
    it = iter(toks)
    cur = [next(it)]

    def nxt():
        v = cur[0]
        try:
            cur[0] = next(it)
        except StopIteration:
            cur[0] = None
        return v

    def expect(t):
        v = nxt()
        if v != t:
            raise ValueError(f"expected {t} got {v} in {s}")

    def parse():
        name = nxt()
        if cur[0] != "(":
            return ("node", name)
        expect("(")
        if name == "Append" or name == "Sum":
            args = [parse()]
            while cur[0] == ",":
                nxt()
                args.append(parse())
            expect(")")
            return ("append" if name == "Append" else "sum", args)
        if name == "Offset":
            d = parse(); expect(",")
            t = int(nxt())
            if cur[0] == ",":
                nxt(); nxt()  # x offset (unsupported, must be 0)
            expect(")")
            return ("offset", d, t)
        if name == "Scale":
            a = float(nxt()); expect(",")
            d = parse(); expect(")")
            return ("scale", a, d)
        if name == "ReplaceIndex":
            d = parse(); expect(",")
            var = nxt(); expect(",")
            val = int(nxt()); expect(")")
            return ("replace_index", d, var, val)
        if name == "Round":
            d = parse(); expect(",")
            m = int(nxt()); expect(")")
            return ("round", d, m)
        if name == "Const":
            v = float(nxt()); expect(",")
            dim = int(nxt()); expect(")")
            return ("const", v, dim)
        if name == "IfDefined":
            d = parse(); expect(")")
            return ("ifdefined", d)
        raise ValueError(f"unsupported descriptor {name}")

    return parse()


class NnetGraph:
    """Parsed nnet3 (from kaldi_formats.Nnet3) evaluated over a whole
    utterance with edge-replicated input (float64)."""

    AFFINE = {"FixedAffineComponent", "AffineComponent", "NaturalGradientAffineComponent"}

    def __init__(self, nn):
        self.nn = nn
        self.nodes = {}  # name -> dict
        self.order = []
        for ln in nn.config_lines:
            kind, kv = split_config_line(ln)
            name = kv["name"]
            if kind == "input-node":
                self.nodes[name] = {"kind": "input", "dim": int(kv["dim"])}
            elif kind == "component-node":
                self.nodes[name] = {"kind": "component", "component": kv["component"],
                                    "input": parse_descriptor(kv["input"])}
            elif kind == "output-node":
                self.nodes[name] = {"kind": "output", "input": parse_descriptor(kv["input"])}
            elif kind == "dim-range-node":
                self.nodes[name] = {"kind": "dimrange", "src": kv["input-node"],
                                    "offset": int(kv["dim-offset"]), "dim": int(kv["dim"])}
            else:
                raise ValueError(kind)
            self.order.append(name)

    def forward(self, inputs: dict, out_name="output", t_out=None):
        """inputs: name -> [T, dim] array; returns [len(t_out), dim]."""
        T = inputs["input"].shape[0]
        cache = {}
        comps = self.nn.components

        def node_val(name, t):
            key = (name, t)
            if key in cache:
                return cache[key]
            nd = self.nodes[name]
            if nd["kind"] == "input":
                a = inputs[name]
                v = a[min(max(t, 0), a.shape[0] - 1)] if name == "input" else a[t]
            elif nd["kind"] == "dimrange":
                v = node_val(nd["src"], t)[nd["offset"]: nd["offset"] + nd["dim"]]
            elif nd["kind"] == "output":
                v = desc_val(nd["input"], t)
            else:
                ctype, f = comps[nd["component"]]
                if isinstance(f, list):
                    f = dict(f)
                if ctype == "TdnnComponent":
                    x = np.concatenate([desc_val(nd["input"], t + o) for o in f["<TimeOffsets>"]])
                else:
                    x = desc_val(nd["input"], t)
                v = apply_component(ctype, f, x)
            cache[key] = v
            return v

        def desc_val(d, t):
            k = d[0]
            if k == "node":
                return node_val(d[1], t)
            if k == "offset":
                return desc_val(d[1], t + d[2])
            if k == "scale":
                return d[1] * desc_val(d[2], t)
            if k == "sum":
                acc = desc_val(d[1][0], t)
                for e in d[1][1:]:
                    acc = acc + desc_val(e, t)
                return acc
            if k == "append":
                return np.concatenate([desc_val(e, t) for e in d[1]])
            if k == "replace_index":
                if d[1] == ("node", "ivector") and "ivector_at" in inputs:
                    return inputs["ivector_at"](t)  # the i-vector of the chunk computing row t
                return desc_val(d[1], d[3] if d[2] == "t" else t)
            if k == "round":
                return desc_val(d[1], (t // d[2]) * d[2])
            if k == "const":
                return np.full(d[2], d[1])
            if k == "ifdefined":
                return desc_val(d[1], t)
            raise ValueError(k)

        if t_out is None:
            t_out = range(0, T, 3)
        return np.stack([node_val(out_name, t) for t in t_out])


def bn_scale_offset(f):
    mean = np.asarray(f["<StatsMean>"], np.float64)
    var = np.asarray(f["<StatsVar>"], np.float64)
    eps = f.get("<Epsilon>", 1e-3)
    tr = f.get("<TargetRms>", 1.0)
    scale = tr / np.sqrt(np.maximum(var, 0.0) + eps)
    return scale, -mean * scale


def apply_component(ctype, f, x):
    if ctype in NnetGraph.AFFINE:
        return f["<LinearParams>"].astype(np.float64) @ x + f["<BiasParams>"]
    if ctype == "TdnnComponent":
        y = f["<LinearParams>"].astype(np.float64) @ x
        b = f.get("<BiasParams>")
        return y + b if b is not None and len(b) else y
    if ctype == "LinearComponent":
        return f["<Params>"].astype(np.float64) @ x
    if ctype == "RectifiedLinearComponent":
        return np.maximum(x, 0.0)
    if ctype == "BatchNormComponent":
        s, o = bn_scale_offset(f)
        reps = len(x) // len(s)
        return x * np.tile(s, reps) + np.tile(o, reps)
    if ctype in ("NoOpComponent", "GeneralDropoutComponent", "DropoutComponent",
                 "SpecAugmentTimeMaskComponent"):
        return x
    if ctype == "ScaleAndOffsetComponent":
        s, o = f["<Scales>"], f["<Offsets>"]
        reps = len(x) // len(s)
        return x * np.tile(s, reps) + np.tile(o, reps)
    raise ValueError(f"unsupported component {ctype}")


# ----------------------------------------------------------------------------
# Online i-vector extraction (Kaldi online2/online-ivector-feature.cc,
# ivector/ivector-extractor.cc OnlineIvectorEstimationStats, matrix/
# optimization.cc LinearCgd) -- float64 restatement used to calibrate the
# synthetic model and to cross-check the C oracle.  Configuration as the
# reference sets it (src/model.cc:247-263): splice +-3, LDA, online CMVN with
# global stats (window 600, global frames 200), 5-best UBM posteriors
# (min-post 0.025, scale 0.1), max-count 100, 15 CG iterations.
# ----------------------------------------------------------------------------
class IvectorModel:
    def __init__(self, ivector_dir):
        import kaldi_formats as kf
        self.lda = kf.read_matrix_file(os.path.join(ivector_dir, "final.mat"))
        self.cmvn = kf.read_matrix_file(os.path.join(ivector_dir, "global_cmvn.stats"))
        self.ubm = kf.read_diag_gmm(os.path.join(ivector_dir, "final.dubm"))
        self.ie = kf.read_ivector_extractor(os.path.join(ivector_dir, "final.ie"))
        self.left = self.right = 3
        self.num_gselect, self.min_post, self.post_scale = 5, 0.025, 0.1
        self.max_count, self.num_cg_iters = 100.0, 15
        self.cmn_window, self.global_frames = 600, 200
        self.S = self.ie.M[0].shape[1]
        self.SigmaInvM = [si @ m for si, m in zip(self.ie.sigma_inv, self.ie.M)]
        self.U = [m.T @ sm for m, sm in zip(self.ie.M, self.SigmaInvM)]

    def cmvn_feats(self, feats):
        T, D = feats.shape
        out = np.zeros_like(feats, dtype=np.float64)
        s = np.zeros(D)
        n = 0.0
        g = self.cmvn
        for t in range(T):
            s += feats[t]
            n += 1
            if t - self.cmn_window >= 0:
                s -= feats[t - self.cmn_window]
                n -= 1
            st, cnt = s.copy(), n
            if cnt < self.cmn_window:
                cg = min(self.cmn_window - cnt, self.global_frames)
                st = st + cg / g[0, D] * g[0, :D]
                cnt = cnt + cg / g[0, D] * g[0, D]
            out[t] = feats[t] - st / cnt
        return out

    def lda_frame(self, src, t, T_ready):
        idx = [min(max(t + o, 0), T_ready - 1) for o in range(-self.left, self.right + 1)]
        x = np.concatenate([src[i] for i in idx])
        D = x.size
        if self.lda.shape[1] == D + 1:
            return self.lda[:, :D] @ x + self.lda[:, D]
        return self.lda @ x

    def extract(self, feats, requests, finished=True):
        """i-vectors (prior offset removed) at each requested frame, in
        order, processing frames as Kaldi's OnlineIvectorFeature::GetFrame."""
        feats = np.asarray(feats, np.float64)
        T = feats.shape[0]
        norm = self.cmvn_feats(feats)
        S = self.S
        lin = np.zeros(S)
        lin[0] = self.ie.prior_offset
        quad = np.eye(S)
        nfr = 0.0
        cur = np.zeros(S)
        cur[0] = self.ie.prior_offset
        done = 0
        ubm = self.ubm
        out = []
        for f in requests:
            if f >= done:
                for t in range(done, f + 1):
                    xn = self.lda_frame(norm, t, T)
                    ll = ubm.gconsts + ubm.means_invvars @ xn - 0.5 * (ubm.inv_vars @ (xn * xn))
                    order = sorted(range(len(ll)), key=lambda g: (-ll[g], g))[:self.num_gselect]
                    while len(order) > 1 and ll[order[-1]] < ll[order[0]] + np.log(self.min_post):
                        order.pop()
                    e = np.exp(ll[order] - ll[order[0]])
                    post = e / e.sum() * self.post_scale
                    xr = self.lda_frame(feats, t, T)
                    for g, w in zip(order, post):
                        lin += w * (self.SigmaInvM[g].T @ xr)
                        quad += w * self.U[g]
                    tw = post.sum()
                    old = max(nfr, self.max_count) / self.max_count
                    new = max(nfr + tw, self.max_count) / self.max_count
                    if new != old:
                        lin[0] += self.ie.prior_offset * (new - old)
                        quad += np.eye(S) * (new - old)
                    nfr += tw
                done = f + 1
                if nfr > 0:
                    cur = linear_cgd(quad, lin, cur, self.num_cg_iters)
            v = cur.copy()
            v[0] -= self.ie.prior_offset
            out.append(v)
        return np.array(out)


def linear_cgd(A, b, x, max_iters):
    x = x.copy()
    p = b - A @ x
    r = -p
    rcur = r @ r
    rrec = rcur
    for k in range(min(max_iters, len(b) + 5)):
        Ap = A @ p
        alpha = -(p @ r) / (p @ Ap)
        x += alpha * p
        r += alpha * Ap
        rnext = r @ r
        if rnext < 1e-4 * rrec or rnext > 1e4 * rrec:
            r = A @ x - b
            rnext = r @ r
            rrec = rnext
        if rnext <= np.finfo(np.float64).tiny:
            break
        p = (rnext / rcur) * p - r
        rcur = rnext
    return x


def needed_times(graph, out_times, node):
    """Times at which `node` is evaluated to compute the output at out_times
    (dependency cone through the descriptors and TDNN time offsets)."""
    need = {}

    def visit_desc(d, t, acc):
        k = d[0]
        if k == "node":
            acc.add((d[1], t))
        elif k == "offset":
            visit_desc(d[1], t + d[2], acc)
        elif k == "scale":
            visit_desc(d[2], t, acc)
        elif k in ("sum", "append"):
            for e in d[1]:
                visit_desc(e, t, acc)
        elif k == "replace_index":
            visit_desc(d[1], d[3] if d[2] == "t" else t, acc)
        elif k == "ifdefined":
            visit_desc(d[1], t, acc)
        elif k == "round":
            visit_desc(d[1], (t // d[2]) * d[2], acc)

    todo = [("output", t) for t in out_times]
    seen = set(todo)
    while todo:
        name, t = todo.pop()
        need.setdefault(name, set()).add(t)
        nd = graph.nodes[name]
        acc = set()
        if nd["kind"] == "dimrange":
            acc.add((nd["src"], t))
        elif nd["kind"] in ("component", "output"):
            offs = [0]
            if nd["kind"] == "component":
                ctype, f = graph.nn.components[nd["component"]]
                f = dict(f) if isinstance(f, list) else f
                if ctype == "TdnnComponent":
                    offs = list(f["<TimeOffsets>"])
            for o in offs:
                visit_desc(nd["input"], t + o, acc)
        for a in acc:
            if a not in seen:
                seen.add(a)
                todo.append(a)
    return need.get(node, set())
