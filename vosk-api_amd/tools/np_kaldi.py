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
import re

import numpy as np


# ----------------------------------------------------------------------------
# MFCC
# ----------------------------------------------------------------------------
class MfccOpts:
    def __init__(self, conf: dict | None = None):
        c = conf or {}
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
        self.use_energy = c.get("use-energy", "true") == "true"
        self.low_freq = float(c.get("low-freq", 20))
        self.high_freq = float(c.get("high-freq", 0))
        self.cepstral_lifter = float(c.get("cepstral-lifter", 22))

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
        T = next(iter(inputs.values())).shape[0] if "input" not in inputs else inputs["input"].shape[0]
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
