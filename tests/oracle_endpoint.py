"""CPU restatement of endpointing and of the batch path's segmentation
(TEST INFRASTRUCTURE ONLY).

Endpoint rules: Kaldi OnlineEndpointConfig / EndpointDetected
(online2/online-endpoint.{h,cc} [K], not vendored in the reference) as the
reference calls it, src/recognizer.cc:318 (rules from model.conf, V1
defaults src/model.cc:142-145); float32 arithmetic like the C++ restatement
(vosk-api_amd/csrc/vosk_impl.cc EndpointRulesFire).

Batch segmentation: BatchRecognizer (src/batch_recognizer.cc:115-181) pushes
8160-sample chunks, the GPU pipeline decodes each chunk's ready frames and,
with reset_on_endpoint (src/batch_model.cc:72), ends the decoder segment when
the rules fire after a chunk; the final chunk (FinishStream) ends the last
segment.  The chunk schedule mirrors the engine's (DecodableNnetLoopedOnline
readiness: a chunk waits for the nnet's right context and the i-vector
splice's).
"""
from __future__ import annotations

import numpy as np

F32 = np.float32
INF = F32(np.inf)

# (must_contain_nonsilence, min_trailing_silence, max_relative_cost, min_utterance_length)
DEFAULT_RULES = [(False, 5.0, np.inf, 0.0), (True, 0.5, 2.0, 0.0), (True, 1.0, 8.0, 0.0),
                 (True, 2.0, np.inf, 0.0), (False, 0.0, np.inf, 20.0)]
_FIELDS = ("must-contain-nonsilence", "min-trailing-silence", "max-relative-cost",
           "min-utterance-length")


def endpoint_config(model_conf: dict):
    """(rules as float32 tuples, silence phone set) from conf/model.conf."""
    rules = [list(r) for r in DEFAULT_RULES]
    for k, v in model_conf.items():
        if not k.startswith("endpoint.rule"):
            continue
        r = int(k[len("endpoint.rule")]) - 1
        f = _FIELDS.index(k[len("endpoint.ruleN."):])
        rules[r][f] = str(v).lower() in ("true", "1") if f == 0 else float(v)
    sil = set(int(p) for p in str(model_conf.get("endpoint.silence-phones", "")).replace(",", ":").split(":") if p)
    return [(bool(a), F32(b), F32(c), F32(d)) for a, b, c, d in rules], sil


def trailing_silence(path, ilabel, tid2phone, sil):
    """TrailingSilenceLength over the best path's emitting arcs."""
    n = 0
    for a in reversed(list(path)):
        il = int(ilabel[a])
        if il == 0:
            continue
        if int(tid2phone[il]) in sil:
            n += 1
        else:
            break
    return n


def rules_fire(rules, frames, trailing_sil, shift, final_relative_cost):
    utt = F32(frames) * F32(shift)
    s = F32(trailing_sil) * F32(shift)
    for must, min_sil, max_rel, min_len in rules:
        if ((utt > s) or not must) and s >= min_sil and F32(final_relative_cost) <= max_rel and utt >= min_len:
            return True
    return False


def batch_segments(oracle, wave, llh, right_context, priming, spc=8160, kaldi=False):
    """Decoder segments [(first frame, end frame)] of one BatchRecognizer
    stream fed `wave` and finished; llh = the stream's log-likelihood rows
    (whole-stream, the batch chunking); kaldi: the decoder order (the batch
    lanes' default is the order-independent form)."""
    from oracle_py import mfcc_num_frames
    rules, sil = endpoint_config(oracle.model_conf)
    shift = F32(F32(0.01) * F32(oracle.fss))
    min_len = min(r[3] for r in rules)
    fpc, fss = oracle.fpc, oracle.fss
    opc = fpc // fss
    ivr = oracle.ivector.m.right if oracle.ivector is not None else 0
    N = len(wave)
    g = oracle.graph
    c, out_ready, seg0, segs = -priming, 0, 0, []
    for k in range(N // spc):
        T = mfcc_num_frames((k + 1) * spc, oracle.mfcc_conf, oracle.fbank)
        njobs = 0
        while njobs < priming + 2 and T >= (max(c, 0) + 1) * fpc + right_context + ivr:
            if c >= 0:
                out_ready += opc
            c += 1
            njobs += 1
        frames = out_ready - seg0
        if frames <= 0 or F32(frames) * shift < min_len:
            continue
        r = oracle.decode_llh(llh[seg0:out_ready], use_final=False, kaldi=kaldi)
        ts = trailing_silence(r["path"], g.ilabel, oracle.tm.tid2phone, sil)
        if rules_fire(rules, frames, ts, shift, r["final_relative_cost"]):
            segs.append((seg0, out_ready))
            seg0 = out_ready
    T = mfcc_num_frames(N, oracle.mfcc_conf, oracle.fbank)
    segs.append((seg0, -(-T // fss)))
    return segs


def _chunk_checks(oracle, N, right_context, priming, spc):
    """The frame count ready after each chunk where the lane checks the
    rules (batch_segments' schedule); the last entry is the stream's end."""
    from oracle_py import mfcc_num_frames
    fpc, fss = oracle.fpc, oracle.fss
    opc = fpc // fss
    ivr = oracle.ivector.m.right if oracle.ivector is not None else 0
    c, out_ready, checks = -priming, 0, []
    for k in range(N // spc):
        T = mfcc_num_frames((k + 1) * spc, oracle.mfcc_conf, oracle.fbank)
        njobs = 0
        while njobs < priming + 2 and T >= (max(c, 0) + 1) * fpc + right_context + ivr:
            if c >= 0:
                out_ready += opc
            c += 1
            njobs += 1
        checks.append(out_ready)
    T = mfcc_num_frames(N, oracle.mfcc_conf, oracle.fbank)
    return checks, -(-T // fss)


def batch_segments_fast(oracle, wave, llh, right_context, priming, spc=8160, kaldi=False, lazy_states=None):
    """batch_segments with one decoding pass per segment: the segment's
    decoder is probed at every later chunk check (orc_decode_kaldi endpoint
    probes: the state after n frames does not depend on the frames after
    them), and ends at the first probe whose rules fire.  Same result as
    batch_segments (tests/test_oracle.py), linear instead of quadratic in the
    stream length.  On a graph with OpenFST's lazy numbering (Kaldi order)
    the stream's numbering carries from segment to segment (the stream's
    ComposeFst outlives its decoder resets; the GPU keeps it per slot):
    lazy_states, a list, receives the numbering at each segment's start."""
    rules, sil = endpoint_config(oracle.model_conf)
    shift = F32(F32(0.01) * F32(oracle.fss))
    min_len = min(r[3] for r in rules)
    g = oracle.graph
    import oracle_py
    lazy_on = kaldi and g.lazy is not None and __import__("os").environ.get("VOSK_AMD_LAZY_IDS", "1") != "0"
    ls = oracle_py.LazyState(g) if lazy_on else None
    checks, end = _chunk_checks(oracle, len(wave), right_context, priming, spc)
    seg0, segs, k = 0, [], 0
    while True:
        if lazy_states is not None:
            lazy_states.append(ls.copy() if ls is not None else None)
        cand = [(i, x) for i, x in enumerate(checks) if i >= k and x - seg0 > 0 and F32(x - seg0) * shift >= min_len]
        if not cand:
            break
        last = max(x for _, x in cand)
        r = g.decode(llh[seg0:last], oracle.beam, oracle.max_active, oracle.min_active, oracle.beam_delta,
                     use_final=False, kaldi=kaldi, probes=[x - seg0 for _, x in cand],
                     lazy_state=ls.copy() if ls is not None else None)
        fired = None
        for (i, x), (path, frc) in zip(cand, r["probes"]):
            ts = trailing_silence(path, g.ilabel, oracle.tm.tid2phone, sil)
            if rules_fire(rules, x - seg0, ts, shift, frc):
                fired = (i, x)
                break
        if fired is None:
            break
        segs.append((seg0, fired[1]))
        if ls is not None:  # the numbering after the segment's frames
            g.decode(llh[seg0:fired[1]], oracle.beam, oracle.max_active, oracle.min_active, oracle.beam_delta,
                     use_final=False, kaldi=kaldi, lazy_state=ls)
        seg0, k = fired[1], fired[0] + 1
    segs.append((seg0, end))
    if lazy_states is not None:
        del lazy_states[len(segs):]
    return segs
