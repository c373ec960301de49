"""ctypes wrapper of the diagnostic engine ABI (include/vosk_amd_engine.h).

Drives the same GPU engine the vosk_* API uses, stage by stage, for the
parity tests and the benchmark.  Every call raises if the native library
reports an error; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _c

_vp = C.c_void_p
_SIGS = {
    "vamd_last_error": (C.c_char_p, []),
    "vamd_device_count": (C.c_int, []),
    "vamd_plan_describe": (C.c_char_p, [C.c_char_p, C.c_int]),
    "vamd_plan_info": (C.c_int, [C.c_char_p, C.c_int, _vp, _vp]),
    "vamd_engine_new": (_vp, [C.c_char_p, C.c_int, C.c_int, C.c_int]),
    "vamd_engine_free": (None, [_vp]),
    "vamd_engine_describe": (C.c_char_p, [_vp]),
    "vamd_engine_info": (C.c_int, [_vp, _vp, _vp]),
    "vamd_stream_new": (C.c_int, [_vp]),
    "vamd_stream_free": (C.c_int, [_vp, C.c_int]),
    "vamd_stream_set_rate": (C.c_int, [_vp, C.c_int, C.c_int]),
    "vamd_stream_reset": (C.c_int, [_vp, C.c_int, C.c_int]),
    "vamd_stream_accept": (C.c_int, [_vp, C.c_int, _vp, C.c_int, C.c_int]),
    "vamd_engine_advance": (C.c_int, [_vp, _vp, C.c_int]),
    "vamd_stream_frames_decoded": (C.c_int, [_vp, C.c_int]),
    "vamd_stream_error": (C.c_int, [_vp, C.c_int]),
    "vamd_stream_decoder_state": (C.c_int, [_vp, C.c_int, _vp]),
    "vamd_stream_features": (C.c_int, [_vp, C.c_int, C.c_int, C.c_int, _vp]),
    "vamd_stream_llh": (C.c_longlong, [_vp, C.c_int, _vp, C.c_longlong]),
    "vamd_stream_ivectors": (C.c_longlong, [_vp, C.c_int, _vp, C.c_longlong]),
    "vamd_engine_ivector_dim": (C.c_int, [_vp]),
    "vamd_stream_update_silence_weights": (C.c_int, [_vp, C.c_int, C.c_int]),
    "vamd_stream_lattice": (C.c_int, [_vp, C.c_int, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                      _vp, _vp, _vp]),
    "vamd_lattice_words_json": (C.c_char_p, [C.c_int] + [_vp] * 8 + [C.c_int, _vp, C.c_int, _vp, _vp,
                                                                   C.c_int, C.c_float, C.c_float,
                                                                   C.c_int, _vp, _vp, _vp, C.c_int]),
    "vamd_silence_weighting_run": (C.c_int, [C.c_int, _vp, _vp, _vp, _vp, _vp, _vp, C.c_int,
                                             C.c_float, C.c_int, _vp, _vp, _vp, C.c_int]),
    "vamd_stream_stats": (C.c_int, [_vp, C.c_int, _vp, C.c_int]),
    "vamd_stream_decode_llh": (C.c_int, [_vp, C.c_int, _vp, C.c_int, C.c_int]),
    "vamd_stream_best_path": (C.c_int, [_vp, C.c_int, C.c_int, _vp, C.c_int, _vp, _vp]),
    "vamd_engine_counters": (C.c_int, [_vp, _vp]),
    "vamd_stream_preload": (C.c_int, [_vp, C.c_int, _vp, C.c_longlong, C.c_int]),
    "vamd_stream_segment_best_path": (C.c_int, [_vp, C.c_int, _vp, C.c_int]),
    "vamd_engine_step": (C.c_int, [_vp, _vp, C.c_int]),
    "vamd_engine_flush": (C.c_int, [_vp]),
    "vamd_engine_decoder_totals": (C.c_int, [_vp, _vp]),
    "vamd_engine_decoder_phases": (C.c_int, [_vp, _vp]),
    "vamd_engine_decoder_phases_n": (C.c_int, [_vp, _vp, C.c_int]),
    "vamd_batch_batching_counters": (C.c_int, [_vp, _vp]),
    "vamd_feeding_round_incomplete": (C.c_int, [C.c_int, _vp, _vp, _vp]),
    "vamd_engine_decoder_phases_per_stream": (C.c_int, [_vp, _vp]),
    "vamd_engine_set_step_samples": (C.c_int, [_vp, C.c_int]),
    "vamd_engine_stage_times": (C.c_int, [_vp, _vp, _vp, C.c_int]),
    "vamd_lattice_set_rescore": (C.c_int, [C.c_char_p, C.c_char_p]),
    "vamd_lattice_set_phones": (C.c_int, [_vp, _vp, C.c_int]),
    "vamd_lattice_set_det_max_mem": (C.c_int, [C.c_longlong]),
    "vamd_carpa_logprob": (C.c_float, [C.c_char_p, C.c_int, _vp, C.c_int]),
    "vamd_batch_lanes": (C.c_int, [_vp]),
    "vamd_batch_lane_kaldi_order": (C.c_int, [_vp, C.c_int]),
    "vamd_batch_lane_stats": (C.c_int, [_vp, C.c_int, _vp, _vp, _vp, _vp, C.c_int]),
    "vamd_batch_lane_memory": (C.c_int, [_vp, C.c_int, _vp]),
    "vamd_batch_recognizer_lane": (C.c_int, [_vp]),
    "vamd_batch_result_profile": (C.c_int, [_vp, _vp]),
    "vamd_admission_replay": (C.c_int, [C.c_int, _vp, C.c_int, _vp, _vp]),
    "vamd_incremental_json": (C.c_char_p, [C.c_int] + [_vp] * 4 + [C.c_int] + [_vp] * 5 + [C.c_int] + [_vp] * 3 +
                              [C.c_int, _vp, C.c_int, C.c_float, C.c_int, C.c_float, C.c_int, C.c_int, C.c_int,
                               _vp, _vp]),
}
for _name, (_res, _args) in _SIGS.items():
    _f = getattr(_c, _name)
    _f.restype = _res
    _f.argtypes = _args

STATS_FIELDS = ("ntok_in", "ntok_out", "arcs_emit", "arcs_eps", "best", "cutoff",
                "next_cutoff", "adaptive_beam")


def _err():
    return (_c.vamd_last_error() or b"").decode()


def _chk(r):
    if r is None or (isinstance(r, int) and r < 0):
        raise RuntimeError("libvosk engine error: " + _err())
    return r


def admission_replay(drain_per_step, chunks):
    """Host-only: the batch path's admission policy (BatchModel::Admit,
    PickLane) replayed over len(chunks) admissions against lanes draining
    drain_per_step[i] pending chunks between admissions; returns the lane of
    each admission."""
    d = np.ascontiguousarray(drain_per_step, np.int32)
    c = np.ascontiguousarray(chunks, np.int32)
    out = np.zeros(len(c), np.int32)
    _chk(_c.vamd_admission_replay(len(d), d.ctypes.data, len(c), c.ctypes.data, out.ctypes.data))
    return out


def feeding_round_incomplete(pushed, taken, ended):
    """Host-only: the lane's dynamic batching rule (FeedingRoundIncomplete):
    True while a step would still wait for streams of the feeding round."""
    p = np.ascontiguousarray(pushed, np.int64)
    t = np.ascontiguousarray(taken, np.int64)
    e = np.ascontiguousarray(ended, np.int32)
    return bool(_chk(_c.vamd_feeding_round_incomplete(len(p), p.ctypes.data, t.ctypes.data, e.ctypes.data)))


def batch_batching_counters(model):
    """{steps, split_rounds, released_by_wait, merged_probes} of a
    vosk.BatchModel's lanes (merged_probes: decoder jobs of one stream that
    completed without an endpoint probe between them; must stay 0)."""
    o = np.zeros(4, np.int64)
    _chk(_c.vamd_batch_batching_counters(model._handle, o.ctypes.data))
    return dict(zip(("steps", "split_rounds", "released_by_wait", "merged_probes"), (int(x) for x in o)))


def batch_lanes(model):
    """Number of GPU lanes of a vosk.BatchModel."""
    return _chk(_c.vamd_batch_lanes(model._handle))


def batch_lane_order(model, lane=0):
    """"kaldi" or "parallel": the token-passing order of a batch lane."""
    return "kaldi" if _chk(_c.vamd_batch_lane_kaldi_order(model._handle, lane)) else "parallel"


def batch_lane_stats(model, lane, reset=False):
    """{device, streams, pending, stage ms / launches, decoder totals} of one lane."""
    ld = np.zeros(3, np.int32)
    ms = np.zeros(4, np.float64)
    ln = np.zeros(4, np.int64)
    dec = np.zeros(6, np.int64)
    _chk(_c.vamd_batch_lane_stats(model._handle, lane, ld.ctypes.data, ms.ctypes.data, ln.ctypes.data,
                                  dec.ctypes.data, 1 if reset else 0))
    names = ("front", "nnet", "decode", "step")
    return {"device": int(ld[0]), "streams": int(ld[1]), "pending": int(ld[2]),
            "stages": {k: (float(ms[i]), int(ln[i])) for i, k in enumerate(names)},
            "decoder": dict(zip(("frames", "tok_in", "tok_out", "arcs_emit", "arcs_eps", "links"),
                                (int(x) for x in dec)))}


def batch_lane_memory(model, lane=0):
    """{device bytes, token / link arena per stream, their highest fill} of a lane."""
    o = np.zeros(5, np.int64)
    _chk(_c.vamd_batch_lane_memory(model._handle, lane, o.ctypes.data))
    return dict(zip(("device_bytes", "arena_tokens", "arena_links", "arena_tokens_high", "arena_links_high"),
                    (int(x) for x in o)))


def batch_result_profile(model):
    """Result production totals of a vosk.BatchModel (segments, links copied,
    ms copy / build / prune+determinize+align / MBR / format) and the lane
    loops' host time (ms in the dynamic batching wait, the engine step,
    endpoint checks + segment hand-off, finals + retiring; lane iterations;
    the endpoint probe launches within the endpoint checks)."""
    o = np.zeros(13, np.float64)
    _chk(_c.vamd_batch_result_profile(model._handle, o.ctypes.data))
    return dict(zip(("segments", "links_copied", "copy_ms", "build_ms", "det_ms", "mbr_ms", "format_ms",
                     "lane_batch_wait_ms", "lane_step_ms", "lane_endpoint_ms", "lane_finals_ms",
                     "lane_iterations", "lane_probe_ms"), (float(x) for x in o)))


def batch_recognizer_lane(rec):
    return _chk(_c.vamd_batch_recognizer_lane(rec._handle))


def lattice_words(L, arc_ilabel, arc_olabel, lattice_beam=6.0, graph_scale=0.9, nbest=5, align=None,
                  timings=False):
    """Host-only: the result pipeline (prune, determinize, scale, MBR,
    n-best) over a lattice in the vamd_stream_lattice array form; align =
    (tid phone-boundary type, tid IsFinal, tid IsSelfLoop) arrays to word-align
    before MBR / n-best."""
    import json
    il = np.ascontiguousarray(arc_ilabel, np.int32)
    ol = np.ascontiguousarray(arc_olabel, np.int32)
    a = {k: np.ascontiguousarray(L[k]) for k in ("frame_begin", "tok_state", "tok_cost", "link_src",
                                                 "link_dst", "link_arc", "link_graph", "link_ac",
                                                 "final_cost")}
    fc = a["final_cost"] if len(a["final_cost"]) else np.zeros(1, np.float32)
    al = [np.ascontiguousarray(x, np.int8) for x in align] if align is not None else None
    r = _c.vamd_lattice_words_json(int(L["num_frames"]), a["frame_begin"].ctypes.data,
                                   a["tok_state"].ctypes.data, a["tok_cost"].ctypes.data,
                                   a["link_src"].ctypes.data, a["link_dst"].ctypes.data,
                                   a["link_arc"].ctypes.data, a["link_graph"].ctypes.data,
                                   a["link_ac"].ctypes.data, len(a["link_src"]), fc.ctypes.data,
                                   len(L["final_cost"]), il.ctypes.data, ol.ctypes.data, len(il),
                                   lattice_beam, graph_scale, nbest,
                                   *(([x.ctypes.data for x in al] + [len(al[0])]) if al is not None
                                     else [None, None, None, 0]))
    if r is None:
        raise RuntimeError("vamd_lattice_words_json failed: " + _err())
    d = json.loads(r.decode())
    if not timings:
        d.pop("ms", None)  # host stage times (vary run to run)
    return d


def incremental_lattice(frames, graph, events, lattice_beam=6.0, prune_interval=25, prune_scale=0.01,
                        max_delay=60, min_chunk=20):
    """Host-only: the KaldiRecognizer's incremental lattice (csrc/incremental.h)
    over per-frame records [(states, costs, links [(src, dst, arc, ac)],
    cost_offset)] (tests/oracle_incremental.frames_from_oracle), driven by
    events [(0, frames) | (1, None) | (2, None)]; returns one dict per query
    (1: the partial lattice, 2: the final one): {nfl, ok, chunks, arcs,
    finals}.  Phones from vamd_lattice_set_phones."""
    import json
    fb = np.zeros(len(frames) + 1, np.int32)
    fb[1:] = np.cumsum([len(f[0]) for f in frames])
    ts = np.ascontiguousarray(np.concatenate([f[0] for f in frames]) if frames else np.zeros(0), np.int32)
    tc = np.ascontiguousarray(np.concatenate([f[1] for f in frames]) if frames else np.zeros(0), np.float32)
    co = np.ascontiguousarray([f[3] for f in frames], np.float32)
    lk = [(k, *l) for k, f in enumerate(frames) for l in f[2]]
    lf = np.ascontiguousarray([l[0] for l in lk] or [0], np.int32)
    ls = np.ascontiguousarray([l[1] for l in lk] or [0], np.int32)
    ld = np.ascontiguousarray([l[2] for l in lk] or [0], np.int32)
    la = np.ascontiguousarray([l[3] for l in lk] or [0], np.int32)
    lx = np.ascontiguousarray([l[4] for l in lk] or [0], np.float32)
    il = np.ascontiguousarray(graph.ilabel, np.int32)
    ol = np.ascontiguousarray(graph.olabel, np.int32)
    w = np.ascontiguousarray(graph.weight, np.float32)
    fin = np.ascontiguousarray(graph.final, np.float32)
    et = np.ascontiguousarray([e[0] for e in events] or [0], np.int32)
    ea = np.ascontiguousarray([e[1] if e[1] is not None else 0 for e in events] or [0], np.int32)
    r = _c.vamd_incremental_json(len(frames), fb.ctypes.data, ts.ctypes.data, tc.ctypes.data, co.ctypes.data,
                                 len(lk), lf.ctypes.data, ls.ctypes.data, ld.ctypes.data, la.ctypes.data,
                                 lx.ctypes.data, len(il), il.ctypes.data, ol.ctypes.data, w.ctypes.data,
                                 len(fin), fin.ctypes.data, int(graph.start), lattice_beam, prune_interval,
                                 prune_scale, max_delay, min_chunk, len(events), et.ctypes.data, ea.ctypes.data)
    if r is None:
        raise RuntimeError("vamd_incremental_json failed: " + _err())
    return json.loads(r.decode())


def silence_weighting_run(calls, tid_is_silence, silence_weight=1e-3, fss=3):
    """Host-only: the recognizer's silence weighting over a call sequence.
    calls: [(num_frames_ready, first_decoder_frame, tids, toks)]; returns the
    (frame, delta weight) list of each call."""
    n = len(calls)
    ready = np.array([c[0] for c in calls] or [0], np.int32)
    first = np.array([c[1] for c in calls] or [0], np.int32)
    off = np.zeros(n + 1, np.int32)
    off[1:] = np.cumsum([len(c[2]) for c in calls])
    tids = np.array([t for c in calls for t in c[2]] or [0], np.int32)
    toks = np.array([t for c in calls for t in c[3]] or [0], np.int32)
    sil = np.ascontiguousarray(tid_is_silence, np.uint8)
    cap = 1 << 20
    oo = np.zeros(n + 1, np.int32)
    of = np.zeros(cap, np.int32)
    ow = np.zeros(cap, np.float32)
    _chk(_c.vamd_silence_weighting_run(n, ready.ctypes.data, first.ctypes.data, off.ctypes.data,
                                       tids.ctypes.data, toks.ctypes.data, sil.ctypes.data, len(sil),
                                       silence_weight, fss, oo.ctypes.data, of.ctypes.data,
                                       ow.ctypes.data, cap))
    return [list(zip(of[oo[i]:oo[i + 1]].tolist(), ow[oo[i]:oo[i + 1]].tolist())) for i in range(n)]


def plan_describe(model_dir, frames_per_chunk=0):
    r = _c.vamd_plan_describe(str(model_dir).encode(), frames_per_chunk)
    if r is None:
        raise RuntimeError("vamd_plan_describe failed: " + _err())
    return r.decode()


def plan_info(model_dir, frames_per_chunk=0):
    info = np.zeros(8, np.int32)
    fl = C.c_double(0)
    _chk(_c.vamd_plan_info(str(model_dir).encode(), frames_per_chunk, info.ctypes.data,
                           C.addressof(fl)))
    keys = ("fpc", "fss", "left_context", "right_context", "priming", "out_dim", "ops", "nodes")
    d = dict(zip(keys, (int(x) for x in info)))
    d["flops_per_chunk"] = fl.value
    return d


def device_count():
    return _c.vamd_device_count()


class Engine:
    def __init__(self, model_dir, frames_per_chunk=0, max_streams=8, stats=False, keep_llh=False,
                 time_kernels=False, pipeline=False, lattice=False, order="kaldi"):
        """order: "kaldi" (LatticeFasterDecoder's sequential token passing,
        the KaldiRecognizer path) or "parallel" (the order-independent form
        the BatchModel lanes run); VOSK_AMD_DEC_ORDER overrides either."""
        if order not in ("kaldi", "parallel"):
            raise ValueError("order: 'kaldi' or 'parallel'")
        flags = ((1 if stats else 0) | (2 if keep_llh else 0) | (4 if time_kernels else 0)
                 | (8 if pipeline else 0) | (16 if lattice else 0) | (32 if order == "parallel" else 0))
        h = _c.vamd_engine_new(str(model_dir).encode(), frames_per_chunk, max_streams, flags)
        if not h:
            raise RuntimeError("vamd_engine_new failed: " + _err())
        self.h = h
        self.max_streams = max_streams
        info = np.zeros(8, np.int32)
        fl = C.c_double(0)
        _chk(_c.vamd_engine_info(h, info.ctypes.data, C.addressof(fl)))
        (self.fpc, self.fss, self.left_context, self.right_context, self.priming,
         self.out_dim, self.num_ops, _) = [int(x) for x in info]
        self.flops_per_chunk = fl.value

    def close(self):
        if self.h:
            _c.vamd_engine_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def describe(self):
        return _c.vamd_engine_describe(self.h).decode()

    def new_stream(self):
        return _chk(_c.vamd_stream_new(self.h))

    def set_rate(self, s, rate):
        _chk(_c.vamd_stream_set_rate(self.h, s, int(rate)))

    def free_stream(self, s):
        _chk(_c.vamd_stream_free(self.h, s))

    def reset(self, s, pipeline=True):
        _chk(_c.vamd_stream_reset(self.h, s, 1 if pipeline else 0))

    def accept(self, s, samples, finished=False):
        x = np.ascontiguousarray(samples, np.float32)
        _chk(_c.vamd_stream_accept(self.h, s, x.ctypes.data, len(x), 1 if finished else 0))

    def advance(self, streams):
        a = np.ascontiguousarray(streams, np.int32)
        _chk(_c.vamd_engine_advance(self.h, a.ctypes.data, len(a)))

    def frames_decoded(self, s):
        return _chk(_c.vamd_stream_frames_decoded(self.h, s))

    def error(self, s):
        return _chk(_c.vamd_stream_error(self.h, s))

    def decoder_state(self, s):
        out = np.zeros(8, np.int64)
        _chk(_c.vamd_stream_decoder_state(self.h, s, out.ctypes.data))
        return dict(zip(("ntok", "arena_used", "frames", "links_used", "err", "lat_ovf",
                         "prune_from", "last_prune"), out.tolist()))

    def features(self, s, first, n, dim):
        out = np.zeros((n, dim), np.float32)
        _chk(_c.vamd_stream_features(self.h, s, first, n, out.ctypes.data))
        return out

    def llh(self, s):
        n = _c.vamd_stream_llh(self.h, s, None, 0)
        _chk(n)
        out = np.zeros(n, np.float32)
        _c.vamd_stream_llh(self.h, s, out.ctypes.data, n)
        return out.reshape(-1, self.out_dim)

    def ivectors(self, s):
        """Per-chunk i-vectors computed so far (flag collect_llh) [chunks][dim]."""
        dim = _chk(_c.vamd_engine_ivector_dim(self.h))
        n = _c.vamd_stream_ivectors(self.h, s, None, 0)
        _chk(n)
        out = np.zeros(n, np.float32)
        _c.vamd_stream_ivectors(self.h, s, out.ctypes.data, n)
        return out.reshape(-1, dim) if dim else out.reshape(0, 0)

    def lattice(self, s, use_final=True):
        """State-level lattice of the stream's decoder segment (engine built
        with lattice=True): dict of numpy arrays."""
        sz = np.zeros(4, np.int32)
        _chk(_c.vamd_stream_lattice(self.h, s, 1 if use_final else 0, sz.ctypes.data, *([None] * 9)))
        F, nt, nl = int(sz[0]), int(sz[1]), int(sz[2])
        nfc, ovf = int(sz[3]) & ((1 << 30) - 1), bool(int(sz[3]) >> 30)
        out = dict(frame_begin=np.zeros(F + 2, np.int32), tok_state=np.zeros(nt, np.int32),
                   tok_cost=np.zeros(nt, np.float32), link_src=np.zeros(nl, np.int32),
                   link_dst=np.zeros(nl, np.int32), link_arc=np.zeros(nl, np.int32),
                   link_graph=np.zeros(nl, np.float32), link_ac=np.zeros(nl, np.float32),
                   final_cost=np.zeros(nfc, np.float32))
        keys = ("frame_begin", "tok_state", "tok_cost", "link_src", "link_dst", "link_arc",
                "link_graph", "link_ac", "final_cost")
        _chk(_c.vamd_stream_lattice(self.h, s, 1 if use_final else 0, sz.ctypes.data,
                                    *[out[k].ctypes.data for k in keys]))
        out["num_frames"] = F
        out["overflow"] = ovf
        return out

    def update_silence_weights(self, s, first_decoder_frame=0):
        """Silence-weight the stream's i-vector statistics from its current
        best path (Recognizer::UpdateSilenceWeights); True if active."""
        return bool(_chk(_c.vamd_stream_update_silence_weights(self.h, s, first_decoder_frame)))

    def stats(self, s, cap=100000):
        out = np.zeros((cap, 8), np.float32)
        n = _chk(_c.vamd_stream_stats(self.h, s, out.ctypes.data, cap))
        return out[:min(n, cap)]

    def decode_llh(self, s, llh, reset=True):
        x = np.ascontiguousarray(llh, np.float32)
        _chk(_c.vamd_stream_decode_llh(self.h, s, x.ctypes.data, x.shape[0], 1 if reset else 0))

    def best_path(self, s, use_final=True, cap=1 << 20):
        arcs = np.zeros(cap, np.int32)
        cost = C.c_double(0)
        frel = C.c_float(0)
        n = _chk(_c.vamd_stream_best_path(self.h, s, 1 if use_final else 0, arcs.ctypes.data,
                                           cap, C.addressof(cost), C.addressof(frel)))
        return arcs[:n].copy(), cost.value, frel.value

    def segment_best_path(self, s, cap=1 << 20):
        """Best path from the segment's lattice records on the host (final
        costs if any token is final): the batch path's fallback words."""
        arcs = np.zeros(cap, np.int32)
        n = _chk(_c.vamd_stream_segment_best_path(self.h, s, arcs.ctypes.data, cap))
        return arcs[:n].copy()

    def preload(self, s, samples, finished=True):
        x = np.ascontiguousarray(samples, np.float32)
        _chk(_c.vamd_stream_preload(self.h, s, x.ctypes.data, len(x), 1 if finished else 0))

    def flush(self):
        _chk(_c.vamd_engine_flush(self.h))

    def step(self, streams):
        a = np.ascontiguousarray(streams, np.int32)
        return _chk(_c.vamd_engine_step(self.h, a.ctypes.data, len(a))) == 1

    def set_step_samples(self, n):
        _chk(_c.vamd_engine_set_step_samples(self.h, n))

    def stage_times(self, reset=False):
        ms = np.zeros(4, np.float64)
        ln = np.zeros(4, np.int64)
        _chk(_c.vamd_engine_stage_times(self.h, ms.ctypes.data, ln.ctypes.data, 1 if reset else 0))
        names = ("front", "nnet", "decode", "step")
        return {n: (float(m), int(l)) for n, m, l in zip(names, ms, ln)}

    def decoder_totals(self):
        out = np.zeros(6, np.int64)
        _chk(_c.vamd_engine_decoder_totals(self.h, out.ctypes.data))
        return dict(zip(("frames", "tok_in", "tok_out", "arcs_emit", "arcs_eps", "links"), out.tolist()))

    def decoder_phases(self):
        out = np.zeros(len(self.PHASES), np.int64)
        n = _c.vamd_engine_decoder_phases_n(self.h, out.ctypes.data, len(out))
        if n != len(out):
            raise RuntimeError(f"decoder phase counters: library has {n}, binding expects {len(out)}")
        return dict(zip(self.PHASES, out.tolist()))

    # decoder.hip Prof: s_memtime clocks per phase (slots 0-10), then counts
    PHASES = ("cutoff", "seed", "exp_tokens", "exp_items", "exp_winners", "eps", "commit_toks",
              "commit_links", "commit_eps_links", "commit_clear", "prune", "n_hbm_created",
              "n_created", "n_eps_rounds", "n_chunks", "frames", "prune_walk", "prune_remap",
              "prune_links", "prune_move", "n_prune_frames", "n_prunes", "exp_relax", "exp_links",
              "kq_members", "kq_rank", "kq_replay", "kq_final", "n_kq_frames", "n_kq_fast",
              "n_kq_replayed", "n_kq_members", "n_kq_pops", "n_kq_pops_crit", "kq_label", "kq_lanes",
              "n_kq_label_iters", "n_kq_init", "n_kq_big_init", "n_kq_stack_ovf", "n_kq_unsettled",
              "kq_seg_sort", "kq_seg_lanes", "kpos", "n_kpos_crowded", "n_kq_components",
              "n_kq_comp_max_pops", "keps_pre", "n_big_nonemit_clk", "n_big_frames", "n_big_lanes_clk", "n_members_gt1536",
              "n_members_gt2048", "n_adj_gt_lds", "n_kq_wave_arcs", "n_kq_wave_arcs_crit", "n_kq_wave_hbm_pops",
              "n_kq_hot_members", "n_kq_renumbered", "n_kq_lane_phase_clk", "n_kq_segments", "n_kq_comp_max_clk",
              "exp_lookback", "lazy_ids", "n_lazy_new", "n_lazy_general", "lazy_keys", "lazy_rank",
              "lazy_arcs", "lazy_scan", "lazy_general", "n_frame_clk_all", "n_frame_clk_big")
    PHASE_CLOCK_IDX = list(range(11)) + [16, 17, 18, 19, 22, 23, 24, 25, 26, 27, 34, 35, 41, 42, 43, 47, 62,
                                          63, 66, 67, 68, 69, 70]  # clock slots
    PHASE_CLOCKS = tuple(map(PHASES.__getitem__, PHASE_CLOCK_IDX))

    def decoder_phases_per_stream(self):
        """[max_streams, len(PHASES)] int64: decoder_phases() per stream slot."""
        out = np.zeros((self.max_streams, len(self.PHASES)), np.int64)
        _chk(_c.vamd_engine_decoder_phases_per_stream(self.h, out.ctypes.data))
        return out

    def counters(self):
        out = np.zeros(5, np.int64)
        _chk(_c.vamd_engine_counters(self.h, out.ctypes.data))
        return dict(zip(("steps", "launches", "mfcc_frames", "chunk_jobs", "frames_decoded"),
                        out.tolist()))


def set_rescore(g_fst=None, g_carpa=None):
    """Host-only: LM rescoring (rescore.h) inside lattice_words (None: off)."""
    r = _c.vamd_lattice_set_rescore(g_fst.encode() if g_fst else None,
                                    g_carpa.encode() if g_carpa else None)
    if r != 0:
        raise RuntimeError("vamd_lattice_set_rescore failed: " + _err())


def set_phones(tid2phone=None, tid_first=None):
    """Host-only: phone + word determinization (as GetLattice) inside
    lattice_words; None: word level only."""
    if tid2phone is None:
        r = _c.vamd_lattice_set_phones(None, None, 0)
    else:
        p = np.ascontiguousarray(tid2phone, np.int32)
        f = np.ascontiguousarray(tid_first, np.int8)
        r = _c.vamd_lattice_set_phones(p.ctypes.data, f.ctypes.data, len(p))
    if r != 0:
        raise RuntimeError("vamd_lattice_set_phones failed: " + _err())


def set_det_max_mem(nbytes=50000000):
    """Host-only: the pruned determinization's memory limit (max_mem)."""
    if _c.vamd_lattice_set_det_max_mem(int(nbytes)) != 0:
        raise RuntimeError("vamd_lattice_set_det_max_mem failed: " + _err())


def carpa_logprob(g_carpa, word, hist):
    """Host-only: ConstArpa n-gram log probability (natural log)."""
    h = np.ascontiguousarray(list(hist) or [0], np.int32)
    return float(_c.vamd_carpa_logprob(g_carpa.encode(), int(word), h.ctypes.data, len(hist)))
