#!/usr/bin/env python3
"""Deterministic synthetic Vosk model directory (V2 layout, real on-disk formats).

No real Vosk model exists in this container or on the GPU box (SURVEY.md
§8c), so the framework is exercised on a seeded synthetic model written in
exactly the formats ``vosk_model_new`` reads (``src/model.cc:180-207``,
``:209-300``):

* ``am/final.mdl``      Kaldi binary TransitionModel (chain topology) +
                        nnet3 AmNnetSimple with the TDNN-F topology of the
                        reference training recipe
                        (``training/local/chain/run_tdnn.sh:98-129``; the
                        i-vector branch is omitted),
                        BatchNorm statistics calibrated on test.wav so that
                        activations are well scaled.
* ``graph/HCLG.fst``    OpenFST ``const`` StdArc graph: a lexicon prefix tree
                        over chain-topology biphone HMMs looped through a
                        unigram LM state, with 2-level epsilon backoff chains
                        and optional silence (exercises emitting and
                        non-emitting token passing).
* ``graph/words.txt``, ``conf/model.conf``, ``conf/mfcc.conf``,
  ``graph/phones/word_boundary.int``.

Usage: python make_synth_model.py OUT_DIR [--seed N] [--vocab N] [--pdfs N]
"""
from __future__ import annotations

import argparse
import math
import os
import sys
import wave

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import kaldi_formats as kf  # noqa: E402
import np_kaldi as nk  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
TEST_WAV = os.path.join(REPO, "tests", "golden", "test.wav")

MFCC_CONF = """--use-energy=false
--sample-frequency=16000
--num-mel-bins=40
--num-ceps=40
--low-freq=20
--high-freq=-400
--dither=0
--allow-upsample=true
--allow-downsample=true
"""

# log-fbank front end (src/model.cc:222-225), for models without mfcc.conf
FBANK_CONF = """--sample-frequency=16000
--num-mel-bins=40
--low-freq=20
--high-freq=-400
--dither=0
"""

MODEL_CONF = """--min-active=200
--max-active=7000
--beam=13.0
--lattice-beam=6.0
--acoustic-scale=1.0
--frame-subsampling-factor=3
--endpoint.silence-phones=1
--endpoint.rule2.min-trailing-silence=0.5
--endpoint.rule3.min-trailing-silence=1.0
--endpoint.rule4.min-trailing-silence=2.0
"""


def load_test_wav():
    w = wave.open(TEST_WAV, "rb")
    return np.frombuffer(w.readframes(w.getnframes()), "<i2").astype(np.float64)


# ----------------------------------------------------------------------------
# transition model + graph
# ----------------------------------------------------------------------------
def build_transition_model(rng, num_phones, num_pdfs):
    """Chain topology for every phone: HMM state 0 has forward pdf-class 0 and
    self-loop pdf-class 1 and transitions {0 (self-loop), 1 (exit)}; state 1
    is the non-emitting final state.  Biphone tree: (left, centre) -> a
    (forward pdf, self-loop pdf) pair."""
    phones = list(range(1, num_phones + 1))
    phone2idx = [-1] + [0] * num_phones
    entry = [kf.HmmState(0, 1, [(0, 0.5), (1, 0.5)]), kf.HmmState(-1, -1, [])]
    topo = kf.Topology(phones, phone2idx, [entry])
    tree = {}
    tuples = {}
    for c in phones:
        for l in [0] + phones:
            fp = int(rng.integers(num_pdfs))
            sp = int(rng.integers(num_pdfs))
            tree[(l, c)] = (fp, sp)
            tuples[(c, 0, fp, sp)] = True
    # guarantee every pdf is used at least once
    tl = sorted(tuples)
    tm = kf.TransitionModel(topo, tl, np.zeros(0, np.float32))
    tm.derive()
    tm.log_probs = np.full(tm.num_tids + 1, math.log(0.5), np.float32)
    tuple_index = {t: i for i, t in enumerate(tl)}

    def tids(l, c):
        fp, sp = tree[(l, c)]
        i = tuple_index[(c, 0, fp, sp)]
        first = int(tm.tuple_first_tid[i])
        # transition 0 is the self-loop (dest 0 == hmm state), 1 the exit
        return first + 1, first  # (forward tid, self-loop tid)

    return tm, tids


def position_phone(base, pos, n, num_base):
    """Word-position-dependent phone (Kaldi _B/_E/_I/_S): base phones
    2..num_base map to 2 + 4*(base-2) + {0 begin, 1 end, 2 internal, 3 singleton}."""
    k = 3 if n == 1 else (0 if pos == 0 else (1 if pos == n - 1 else 2))
    return 2 + 4 * (base - 2) + k


def build_graph(rng, tids, num_base, vocab):
    """Lexicon prefix tree over word-position-dependent phones + unigram
    loop.  Returns kf.Fst and words list (prons in base phones)."""
    words = []
    seen = set()
    while len(words) < vocab:
        n = int(rng.integers(1, 8))
        pron = tuple(int(p) for p in rng.integers(2, num_base + 1, size=n))
        if pron in seen:
            continue
        seen.add(pron)
        words.append(pron)
    # Zipf unigram costs
    ranks = rng.permutation(vocab) + 1
    p = 1.0 / ranks
    p /= p.sum()
    costs = -np.log(p)

    arcs = []  # (src, ilabel, olabel, weight, dst)
    LOOP = 0
    n_states = [1]

    def new_state():
        n_states[0] += 1
        return n_states[0] - 1

    num_hist = 16
    hist = [new_state() for _ in range(num_hist)]
    for h in hist:
        arcs.append((h, 0, 0, float(rng.uniform(0.5, 2.0)), LOOP))  # backoff
    # optional silence
    sil_f, sil_s = tids(0, 1)
    s_sil = new_state()
    arcs.append((LOOP, sil_f, 0, 0.7, s_sil))
    arcs.append((s_sil, sil_s, 0, 0.0, s_sil))
    arcs.append((s_sil, 0, 0, 0.0, LOOP))

    children = {}  # (node, phone) -> child node
    node_ctx = {LOOP: 0}
    for wi, pron in enumerate(words):
        node = LOOP
        prev = 0
        for j, bph in enumerate(pron):
            ph = position_phone(bph, j, len(pron), num_base)
            key = (node, ph)
            if key not in children:
                child = new_state()
                children[key] = child
                f, s = tids(prev, ph)
                arcs.append((node, f, 0, 0.0, child))
                arcs.append((child, s, 0, 0.0, child))
            node = children[key]
            prev = ph
        w = wi + 1
        h = hist[int(rng.integers(num_hist))]
        arcs.append((node, 0, w, float(costs[wi]), h))

    S = n_states[0]
    arcs.sort(key=lambda a: (a[0], a[1] == 0))  # per state: emitting first
    src = np.array([a[0] for a in arcs], np.int64)
    row = np.zeros(S + 1, np.int64)
    np.add.at(row, src + 1, 1)
    row = np.cumsum(row)
    final = np.full(S, np.inf, np.float32)
    final[LOOP] = 0.0
    f = kf.Fst(LOOP, final, row,
               np.array([a[1] for a in arcs], np.int32), np.array([a[2] for a in arcs], np.int32),
               np.array([a[3] for a in arcs], np.float32), np.array([a[4] for a in arcs], np.int32))
    return f, words


def build_bigram_graph(rng, tids, num_base, vocab, num_hist=1000, fut=400):
    """Bigram HCLG at the scale of a large model's static graph (BASELINE
    config 4: vosk-model-en-us-0.22's HCLG, src/batch_model.cc:51-54): the
    unigram state owns a lexicon prefix tree over the whole vocabulary, and
    each of `num_hist` bigram histories owns its own prefix tree over `fut`
    successor words (as a determinized/minimized HCLG keeps one word-prefix
    copy per LM state), a backoff epsilon arc to the unigram state and a final
    cost.  A word end goes to the word's bigram history when it has one, else
    to the unigram state.  Built vectorized (numpy) so multi-million-state
    graphs take seconds.  Returns (kf.Fst, words)."""
    words, seen = [], set()
    while len(words) < vocab:
        n = int(rng.integers(1, 8))
        pron = tuple(int(p) for p in rng.integers(2, num_base + 1, size=n))
        if pron in seen:
            continue
        seen.add(pron)
        words.append(pron)
    V = len(words)
    ranks = rng.permutation(V) + 1
    p = 1.0 / ranks
    p /= p.sum()
    uni = -np.log(p)
    # full prefix trie over position-dependent phones; node 0 = root
    parent, phone, prevph = [0], [0], [0]
    children = {}
    paths, ends = [], np.zeros(V, np.int64)
    for wi, pron in enumerate(words):
        node, prev, path = 0, 0, []
        for j, bph in enumerate(pron):
            ph = position_phone(bph, j, len(pron), num_base)
            key = (node, ph)
            if key not in children:
                children[key] = len(parent)
                parent.append(node)
                phone.append(ph)
                prevph.append(prev)
            node = children[key]
            prev = ph
            path.append(node)
        paths.append(path)
        ends[wi] = node
    parent, phone, prevph = (np.array(x, np.int64) for x in (parent, phone, prevph))
    num_pp = int(phone.max()) + 1
    tidf = np.zeros((num_pp, num_pp), np.int64)
    tids_ = np.zeros((num_pp, num_pp), np.int64)
    for l in range(num_pp):
        for c in range(1, num_pp):
            try:
                tidf[l, c], tids_[l, c] = tids(l, c)
            except KeyError:
                pass
    wn_ptr = np.zeros(V + 1, np.int64)
    wn_ptr[1:] = np.cumsum([len(x) for x in paths])
    wn_idx = np.array([n for x in paths for n in x], np.int64)
    hist_words = rng.choice(V, size=min(num_hist, V), replace=False)
    dest = np.zeros(V, np.int64)  # unigram state 0 unless the word is a history

    src_l, il_l, ol_l, w_l, dst_l = [], [], [], [], []

    def add(s, i, o, w, d):
        s, i, o, w, d = np.broadcast_arrays(np.atleast_1d(np.asarray(s, np.int64)),
                                            np.asarray(i, np.int64), np.asarray(o, np.int64),
                                            np.asarray(w, np.float64), np.asarray(d, np.int64))
        for l, x in zip((src_l, il_l, ol_l, w_l, dst_l), (s, i, o, w, d)):
            l.append(x.ravel())

    def tree(root, wsel, costs, next_state):
        """prefix tree of the words wsel hanging off `root`; states from next_state"""
        st = wn_ptr[wsel]
        ln = wn_ptr[wsel + 1] - st
        rep = np.repeat(st - np.concatenate([[0], np.cumsum(ln)[:-1]]), ln) + np.arange(ln.sum())
        nodes = np.unique(wn_idx[rep])
        sid = next_state + np.arange(len(nodes))
        par = parent[nodes]
        psid = np.where(par == 0, root, next_state + np.searchsorted(nodes, par))
        add(psid, tidf[prevph[nodes], phone[nodes]], 0, 0.0, sid)       # enter the phone
        add(sid, tids_[prevph[nodes], phone[nodes]], 0, 0.0, sid)       # self-loop
        end_sid = next_state + np.searchsorted(nodes, ends[wsel])
        return nodes, end_sid, next_state + len(nodes)

    n = 1
    s_sil = n
    n += 1
    sil_f, sil_s = tids(0, 1)
    add([0, s_sil, s_sil], [sil_f, sil_s, 0], 0, [0.7, 0.0, 0.0], [s_sil, s_sil, 0])
    hist_state = n + np.arange(len(hist_words))
    n += len(hist_words)
    dest[hist_words] = hist_state
    allw = np.arange(V)
    _, end_u, n = tree(0, allw, uni, n)
    add(end_u, 0, allw + 1, uni, dest[allw])
    final_h = np.full(len(hist_words), np.inf)
    for k, h in enumerate(hist_words):
        wsel = np.sort(rng.choice(V, size=min(fut, V), replace=False))
        cost = uni[wsel] * rng.uniform(0.3, 0.9, size=len(wsel))
        _, end_h, n = tree(hist_state[k], wsel, cost, n)
        add(end_h, 0, wsel + 1, cost, dest[wsel])
        add(hist_state[k], 0, 0, float(rng.uniform(0.3, 1.5)), 0)        # backoff
        if rng.random() < 0.4:
            final_h[k] = float(rng.uniform(1.0, 4.0))
    src, il, ol, wt, dst = (np.concatenate(l) for l in (src_l, il_l, ol_l, w_l, dst_l))
    order = np.lexsort((il == 0, src))  # per state: emitting first (stable)
    src, il, ol, wt, dst = src[order], il[order], ol[order], wt[order], dst[order]
    row = np.zeros(n + 1, np.int64)
    np.add.at(row, src + 1, 1)
    row = np.cumsum(row)
    final = np.full(n, np.inf, np.float32)
    final[0] = 0.0
    final[hist_state] = final_h
    f = kf.Fst(0, final, row, il.astype(np.int32), ol.astype(np.int32), wt.astype(np.float32),
               dst.astype(np.int32))
    return f, words


def build_lookahead_graph(rng, tids, num_base, vocab, num_tids, n_big=40, fut_big=12, n_tri=12):
    """Lookahead graph pair (src/model.cc:281-285): an HCLr
    transducer shaped as a determinized H o C o L is (Kaldi's lexicon puts a
    word's label on its first phone arc; determinizing the transducer delays
    it to where the pronunciation prefix becomes unique, utils/mkgraph_
    lookahead.sh), and a backoff trigram LM in the ngram trie form
    (write_ngram_fst).  HCLr: a prefix tree over the chain HMMs (entry
    transition-id on the arc into a phone state, self-loop on the state);
    each word's output label on the first arc into a state no other word
    passes through; words end in a state shared by every word ending with the
    same (previous phone, last phone) pair, which -- like the start state --
    is final and continues with the first phones of every word or optional
    silence (so word ends are emitting transitions, as in a real HCL).
    Homophones (one word in 25 repeats an earlier pronunciation) share their
    whole path and output their labels on epsilon arcs to the start state,
    told apart by disambiguation transition-ids (Kaldi's #1, #2 ...).
    Returns (hclr Fst, lm dict, words, disambig ids)."""
    words = []
    seen = {}
    while len(words) < vocab:
        if len(words) >= 25 and len(words) % 25 == 0:
            pron = words[int(rng.integers(len(words)))]
            if seen[pron] >= 3:
                continue
        else:
            n = int(rng.integers(1, 6))
            pron = tuple(int(p) for p in rng.integers(2, num_base + 1, size=n))
            if pron in seen:
                continue
        seen[pron] = seen.get(pron, -1) + 1
        words.append(pron)
    disambig = [num_tids + 1, num_tids + 2, num_tids + 3]
    arcs = []
    LOOP = 0
    n_states = [1]

    def new_state():
        n_states[0] += 1
        return n_states[0] - 1

    sil_f, sil_s = tids(0, 1)
    s_sil = new_state()
    # phone sequences (position-dependent) and how many words share each prefix
    seqs = [[position_phone(b, j, len(pr), num_base) for j, b in enumerate(pr)] for pr in words]
    nwords = {}
    for sq in seqs:
        for j in range(1, len(sq) + 1):
            nwords[tuple(sq[:j])] = nwords.get(tuple(sq[:j]), 0) + 1
    homo = {}  # pronunciation -> its words
    for wi, pr in enumerate(words):
        homo.setdefault(pr, []).append(wi)
    children = {}  # (node, phone) -> tree state
    ends = {}      # (previous phone, last phone) -> shared word-end state
    tree_arcs = {}  # (node, phone) -> arc index (the label goes on it)
    labels = {}
    homo_end = {}
    for wi, sq in enumerate(seqs):
        pr = words[wi]
        shared_pron = len(homo[pr]) > 1
        node, prev = LOOP, 0
        labelled = shared_pron
        for j, ph in enumerate(sq):
            last = j == len(sq) - 1
            key = (node, ph)
            if last and not shared_pron:
                e = ends.get((prev, ph))
                if e is None:
                    e = ends[(prev, ph)] = new_state()
                    arcs.append((e, tids(prev, ph)[1], 0, 0.0, e))
                if key not in tree_arcs:
                    tree_arcs[key] = len(arcs)
                    arcs.append((node, tids(prev, ph)[0], 0, 0.0, e))
                child = e
            else:
                if key not in children:
                    child = children[key] = new_state()
                    tree_arcs[key] = len(arcs)
                    f, sl = tids(prev, ph)
                    arcs.append((node, f, 0, 0.0, child))
                    arcs.append((child, sl, 0, 0.0, child))
                child = children[key]
            if not labelled and (last or nwords[tuple(sq[:j + 1])] == 1):
                labels[tree_arcs[key]] = wi + 1  # the first arc only this word takes
                labelled = True
            node, prev = child, ph
        if shared_pron:
            homo_end[wi] = node
    for pr, ws in homo.items():
        if len(ws) > 1:
            for k, wi in enumerate(ws):
                arcs.append((homo_end[wi], disambig[k - 1] if k else 0, wi + 1, 0.0, LOOP))
    arcs = [(a[0], a[1], labels.get(i, a[2]), a[3], a[4]) for i, a in enumerate(arcs)]
    # word boundaries (the start state, the shared word-end states, silence)
    # continue with every word's first phone, or optional silence
    boundary = list(ends.values()) + [s_sil]
    loop_out = [a for a in arcs if a[0] == LOOP]
    arcs.append((LOOP, sil_f, 0, 0.7, s_sil))
    arcs.append((s_sil, sil_s, 0, 0.0, s_sil))
    for b in boundary:
        for a in loop_out:
            arcs.append((b, a[1], a[2], a[3], a[4]))
        if b != s_sil:
            arcs.append((b, sil_f, 0, 0.7, s_sil))
    S = n_states[0]
    arcs.sort(key=lambda a: a[0])
    row = np.zeros(S + 1, np.int64)
    np.add.at(row, np.array([a[0] for a in arcs], np.int64) + 1, 1)
    row = np.cumsum(row)
    final = np.full(S, np.inf, np.float32)
    final[LOOP] = 0.0
    for b in boundary:
        final[b] = 0.0
    hclr = kf.Fst(LOOP, final, row,
                  np.array([a[1] for a in arcs], np.int32), np.array([a[2] for a in arcs], np.int32),
                  np.array([a[3] for a in arcs], np.float32), np.array([a[4] for a in arcs], np.int32))
    # backoff trigram: unigram root over the vocabulary, sentence start,
    # bigram histories, trigram histories under some of them
    V = len(words)
    ranks = rng.permutation(V) + 1
    p = 1.0 / ranks
    p /= p.sum()
    uni = -np.log(p)

    def fut(nw):
        ws = rng.choice(V, size=min(nw, V), replace=False) + 1
        return {int(w): float(uni[w - 1] * rng.uniform(0.3, 0.9)) for w in ws}

    lm = {(): {"fut": {w + 1: float(uni[w]) for w in range(V)}, "final": 4.0},
          (0,): {"fut": fut(30), "backoff": 0.6, "final": None}}
    big = [int(w) for w in rng.choice(V, size=min(n_big, V), replace=False) + 1]
    for h in big:
        lm[(h,)] = {"fut": fut(fut_big), "backoff": float(rng.uniform(0.3, 1.5)),
                    "final": float(rng.uniform(1.0, 4.0)) if rng.random() < 0.4 else None}
    for h in big[:n_tri]:
        for u in [0] + [int(x) for x in rng.choice(big, size=2, replace=False)]:
            lm[(h, u)] = {"fut": fut(6), "backoff": float(rng.uniform(0.2, 1.0)), "final": None}
    return hclr, lm, words, disambig


# ----------------------------------------------------------------------------
# nnet3
# ----------------------------------------------------------------------------
def nat_affine(rng, din, dout, gain=math.sqrt(2.0), bias=0.05):
    W = (rng.standard_normal((dout, din)) * gain / math.sqrt(din)).astype(np.float32)
    b = (rng.standard_normal(dout) * bias).astype(np.float32)
    return ("NaturalGradientAffineComponent", [
        ("<MaxChange>", 0.75), ("<L2Regularize>", 0.008), ("<LearningRate>", 0.001),
        ("<LinearParams>", W), ("<BiasParams>", b),
        ("<RankIn>", 20), ("<RankOut>", 80), ("<UpdatePeriod>", 4),
        ("<NumSamplesHistory>", 2000.0), ("<Alpha>", 4.0)])


def tdnn_comp(rng, din, dout, offsets, use_bias):
    k = din * len(offsets)
    W = (rng.standard_normal((dout, k)) * math.sqrt(2.0 / k)).astype(np.float32)
    b = (rng.standard_normal(dout) * 0.05).astype(np.float32) if use_bias else np.zeros(0, np.float32)
    return ("TdnnComponent", [
        ("<MaxChange>", 0.75), ("<L2Regularize>", 0.008), ("<LearningRate>", 0.001),
        ("<TimeOffsets>", np.array(offsets, np.int32)),
        ("<LinearParams>", W), ("<BiasParams>", b),
        ("<OrthonormalConstraint>", -1.0 if not use_bias else 0.0),
        ("<UseNaturalGradient>", True), ("<NumSamplesHistory>", 2000.0),
        ("<AlphaInOut>", (4.0, 4.0)), ("<RankInOut>", (20, 80))])


def linear_comp(rng, din, dout):
    W = (rng.standard_normal((dout, din)) * math.sqrt(1.0 / din)).astype(np.float32)
    return ("LinearComponent", [
        ("<MaxChange>", 0.75), ("<L2Regularize>", 0.008), ("<LearningRate>", 0.001),
        ("<Params>", W), ("<OrthonormalConstraint>", -1.0), ("<UseNaturalGradient>", True),
        ("<RankInOut>", (20, 80)), ("<Alpha>", 4.0), ("<NumSamplesHistory>", 2000.0),
        ("<UpdatePeriod>", 4)])


def relu(dim):
    return ("RectifiedLinearComponent", [
        ("<Dim>", dim), ("<ValueAvg>", np.zeros(dim, np.float32)),
        ("<DerivAvg>", np.zeros(dim, np.float32)), ("<Count>", 0.0),
        ("<OderivRms>", np.zeros(dim, np.float32)), ("<OderivCount>", 0.0)])


def batchnorm(dim):
    return ("BatchNormComponent", [
        ("<Dim>", dim), ("<BlockDim>", dim), ("<Epsilon>", 0.001), ("<TargetRms>", 1.0),
        ("<TestMode>", False), ("<Count>", 1.0),
        ("<StatsMean>", np.zeros(dim, np.float32)), ("<StatsVar>", np.ones(dim, np.float32))])


def dropout(dim):
    return ("GeneralDropoutComponent", [
        ("<Dim>", dim), ("<BlockDim>", dim), ("<TimePeriod>", 0),
        ("<DropoutProportion>", 0.0), ("<Continuous>", True)])


def build_nnet(rng, num_pdfs, mfcc_opts, ivector_dim=0):
    comps = {}
    order = []
    lines = ([f"input-node name=ivector dim={ivector_dim}"] if ivector_dim else []) + \
        ["input-node name=input dim=40"]

    def add(name, comp, inp):
        comps[name] = comp
        order.append(name)
        lines.append(f"component-node name={name} component={name} input={inp}")

    # idct: inverse of (lifter * DCT), as the recipe's idct.mat (a fixed 40x40
    # map in front of an fbank front end too)
    if mfcc_opts.fbank:
        mfcc_opts = nk.MfccOpts({"num-mel-bins": "40", "num-ceps": "40"})
    D = nk.dct_matrix(mfcc_opts) * nk.lifter(mfcc_opts)[:, None]
    idct = np.linalg.inv(D).astype(np.float32)
    add("idct", ("FixedAffineComponent", [("<LinearParams>", idct),
                                          ("<BiasParams>", np.zeros(40, np.float32))]), "input")
    add("batchnorm0", batchnorm(40), "idct")
    add("spec-augment", ("SpecAugmentTimeMaskComponent", [
        ("<Dim>", 40), ("<ZeroedProportion>", 0.2), ("<TimeMaskMaxFrames>", 20)]), "batchnorm0")
    sa = "spec-augment"
    add("delta", ("NoOpComponent", [("<Dim>", 120), ("<BackpropScale>", 1.0)]),
        f"Append(Offset({sa}, 0), Sum(Offset(Scale(-1.0, {sa}), -1), Offset({sa}, 1)), "
        f"Sum(Sum(Offset({sa}, -2), Offset({sa}, 2)), Offset(Scale(-2.0, {sa}), 0)))")
    tin = "delta"
    if ivector_dim:  # run_tdnn.sh:106 no-op input2 = Append(delta, ReplaceIndex(ivector, t, 0))
        add("input2", ("NoOpComponent", [("<Dim>", 120 + ivector_dim), ("<BackpropScale>", 1.0)]),
            "Append(delta, ReplaceIndex(ivector, t, 0))")
        tin = "input2"
    add("tdnn1.affine", nat_affine(rng, 120 + ivector_dim, 512), tin)
    add("tdnn1.relu", relu(512), "tdnn1.affine")
    add("tdnn1.batchnorm", batchnorm(512), "tdnn1.relu")
    add("tdnn1.dropout", dropout(512), "tdnn1.batchnorm")
    prev = "tdnn1.dropout"
    for i, stride in zip(range(2, 13), [1, 1, 1, 0, 3, 3, 3, 3, 3, 3, 3]):
        n = f"tdnnf{i}"
        lo = [-stride, 0] if stride else [0]
        ao = [0, stride] if stride else [0]
        add(f"{n}.linear", tdnn_comp(rng, 512, 96, lo, False), prev)
        add(f"{n}.affine", tdnn_comp(rng, 96, 512, ao, True), f"{n}.linear")
        add(f"{n}.relu", relu(512), f"{n}.affine")
        add(f"{n}.batchnorm", batchnorm(512), f"{n}.relu")
        add(f"{n}.dropout", dropout(512), f"{n}.batchnorm")
        add(f"{n}.noop", ("NoOpComponent", [("<Dim>", 512), ("<BackpropScale>", 1.0)]),
            f"Sum(Scale(0.75, {prev}), {n}.dropout)")
        prev = f"{n}.noop"
    add("prefinal-l", linear_comp(rng, 512, 192), prev)
    add("prefinal-chain.affine", nat_affine(rng, 192, 512), "prefinal-l")
    add("prefinal-chain.relu", relu(512), "prefinal-chain.affine")
    add("prefinal-chain.batchnorm1", batchnorm(512), "prefinal-chain.relu")
    add("prefinal-chain.linear", linear_comp(rng, 512, 192), "prefinal-chain.batchnorm1")
    add("prefinal-chain.batchnorm2", batchnorm(192), "prefinal-chain.linear")
    add("output.affine", nat_affine(rng, 192, num_pdfs, gain=1.0, bias=0.5), "prefinal-chain.batchnorm2")
    lines.append("output-node name=output input=output.affine objective=linear")
    # xent branch: present in real chain models, never evaluated at decode time
    add("prefinal-xent.affine", nat_affine(rng, 192, 512), "prefinal-l")
    add("prefinal-xent.relu", relu(512), "prefinal-xent.affine")
    add("prefinal-xent.batchnorm1", batchnorm(512), "prefinal-xent.relu")
    add("prefinal-xent.linear", linear_comp(rng, 512, 192), "prefinal-xent.batchnorm1")
    add("prefinal-xent.batchnorm2", batchnorm(192), "prefinal-xent.linear")
    add("output-xent.affine", nat_affine(rng, 192, num_pdfs, gain=1.0), "prefinal-xent.batchnorm2")
    add("output-xent.log-softmax", ("LogSoftmaxComponent", [
        ("<Dim>", num_pdfs), ("<ValueAvg>", np.zeros(num_pdfs, np.float32)),
        ("<DerivAvg>", np.zeros(num_pdfs, np.float32)), ("<Count>", 0.0),
        ("<OderivRms>", np.zeros(num_pdfs, np.float32)), ("<OderivCount>", 0.0)]),
        "output-xent.affine")
    lines.append("output-node name=output-xent input=output-xent.log-softmax objective=linear")
    return kf.Nnet3(lines, comps, order, 0, 0, np.zeros(0, np.float32))


def _inputs(feats, ivec):
    d = {"input": feats}
    if ivec is not None:
        d["ivector_at"] = lambda t: ivec
    return d


def build_ivector_extractor(rng, out_dir, feats, ivector_dim=40, num_gauss=512,
                            prior_offset=100.0):
    """ivector/ in the recipe's layout (run_ivector_common.sh: PCA over
    +-3 spliced features, 512-Gaussian diagonal UBM, 40-dim extractor), with
    seeded random parameters fitted loosely to test.wav."""
    d = os.path.join(out_dir, "ivector")
    os.makedirs(d, exist_ok=True)
    T, D = feats.shape
    gstats = np.zeros((2, D + 1))
    gstats[0, :D] = feats.sum(0)
    gstats[0, D] = T
    gstats[1, :D] = (feats * feats).sum(0)
    kf.write_matrix_file(os.path.join(d, "global_cmvn.stats"), gstats, double=True)
    norm = feats - feats.mean(0)
    spl = np.concatenate([norm[np.clip(np.arange(T) + o, 0, T - 1)] for o in range(-3, 4)], 1)
    mu = spl.mean(0)
    u, sv, vt = np.linalg.svd(spl - mu, full_matrices=False)
    W = vt[:D] / (sv[:D, None] / math.sqrt(T))  # unit-variance projections
    lda = np.concatenate([W, -(W @ mu)[:, None]], 1)
    kf.write_matrix_file(os.path.join(d, "final.mat"), lda.astype(np.float32))
    x = spl @ W.T - W @ mu
    means = x[rng.choice(T, num_gauss)] + 0.3 * rng.standard_normal((num_gauss, D))
    var = np.full((num_gauss, D), 0.6)
    kf.write_diag_gmm(os.path.join(d, "final.dubm"),
                      kf.diag_gmm_from_params(np.full(num_gauss, 1.0 / num_gauss), means, var))
    M = []
    for g in range(num_gauss):
        m = 0.15 * rng.standard_normal((D, ivector_dim))
        m[:, 0] = means[g] / prior_offset
        M.append(m)
    ie = kf.IvectorExtractor(np.zeros((num_gauss, ivector_dim)), np.zeros(num_gauss), M,
                             [np.diag(1.0 / var[g]) for g in range(num_gauss)], prior_offset)
    kf.write_ivector_extractor(os.path.join(d, "final.ie"), ie)
    with open(os.path.join(d, "splice.conf"), "w") as f:
        f.write("--left-context=3\n--right-context=3\n")
    open(os.path.join(d, "online_cmvn.conf"), "w").close()
    return d


def calibrate(nn, feats, llh_std, ivec=None):
    """Set every BatchNorm's statistics (in config order) from the activations
    of its input on test.wav, then scale the output layer so the
    log-likelihoods have roughly the requested spread."""
    T = feats.shape[0]
    for name in nn.component_order:
        ctype, fields = nn.components[name]
        if ctype != "BatchNormComponent" or name.startswith("prefinal-xent"):
            continue
        g = nk.NnetGraph(nn)
        src = g.nodes[name]["input"]
        assert src[0] == "node"
        vals = g.forward(_inputs(feats, ivec), out_name=src[1], t_out=range(0, T))
        fd = dict(fields)
        fd["<StatsMean>"] = vals.mean(0).astype(np.float32)
        fd["<StatsVar>"] = vals.var(0).astype(np.float32)
        fd["<TestMode>"] = True
        nn.components[name] = (ctype, [(k, fd[k]) for k, _ in fields])
    g = nk.NnetGraph(nn)
    out = g.forward(_inputs(feats, ivec))
    ctype, fields = nn.components["output.affine"]
    fd = dict(fields)
    s = llh_std / max(out.std(), 1e-6)
    fd["<LinearParams>"] = (fd["<LinearParams>"] * s).astype(np.float32)
    fd["<BiasParams>"] = (fd["<BiasParams>"] * s).astype(np.float32)
    nn.components["output.affine"] = (ctype, [(k, fd[k]) for k, _ in fields])


def make_model(out_dir, seed=7, vocab=3000, num_pdfs=2000, num_phones=40, llh_std=3.0,
               ivector_dim=40, frontend="mfcc", global_cmvn=False, graph="hclg", graph_opts=None,
               model_conf=None):
    """frontend: "mfcc" (conf/mfcc.conf) or "fbank" (conf/fbank.conf);
    global_cmvn: write am/global_cmvn.stats (online CMVN on the nnet input);
    graph: "hclg" (graph/HCLG.fst, unigram lexicon tree), "bigram"
    (graph/HCLG.fst, build_bigram_graph: the multi-million-state static graph
    of a large model) or "lookahead" (graph/HCLr.fst + graph/Gr.fst +
    graph/disambig_tid.int, no HCLG); graph_opts: keyword arguments of the
    graph builder; model_conf: conf/model.conf text (default MODEL_CONF)."""
    graph_opts = graph_opts or {}
    rng = np.random.default_rng(seed)
    os.makedirs(os.path.join(out_dir, "am"), exist_ok=True)
    os.makedirs(os.path.join(out_dir, "conf"), exist_ok=True)
    os.makedirs(os.path.join(out_dir, "graph", "phones"), exist_ok=True)
    fb = frontend == "fbank"
    conf_path = os.path.join(out_dir, "conf", "fbank.conf" if fb else "mfcc.conf")
    with open(conf_path, "w") as f:
        f.write(FBANK_CONF if fb else MFCC_CONF)
    with open(os.path.join(out_dir, "conf", "model.conf"), "w") as f:
        f.write(model_conf or MODEL_CONF)
    mo = nk.MfccOpts(kf.parse_conf(conf_path), fbank=fb)

    # silence + 4 word-position variants of each of the other base phones
    num_pos_phones = 1 + 4 * (num_phones - 1)
    tm, tids = build_transition_model(rng, num_pos_phones, num_pdfs)
    if graph == "lookahead":
        fst, lm, words, disambig = build_lookahead_graph(rng, tids, num_phones, vocab, tm.num_tids,
                                                         **graph_opts)
    elif graph == "bigram":
        fst, words = build_bigram_graph(rng, tids, num_phones, vocab, **graph_opts)
    else:
        fst, words = build_graph(rng, tids, num_phones, vocab)
    nn = build_nnet(rng, num_pdfs, mo, ivector_dim)
    feats = nk.features(load_test_wav(), mo)
    nnet_feats = feats
    if global_cmvn:
        st = np.zeros((2, feats.shape[1] + 1))
        st[0, :-1] = feats.sum(0)
        st[0, -1] = feats.shape[0]
        st[1, :-1] = (feats * feats).sum(0)
        kf.write_matrix_file(os.path.join(out_dir, "am", "global_cmvn.stats"), st, double=True)
        nnet_feats = nk.online_cmvn(feats, st)
    ivec = None
    if ivector_dim:
        idir = build_ivector_extractor(rng, out_dir, feats, ivector_dim)
        im = nk.IvectorModel(idir)
        ivec = im.extract(feats, [feats.shape[0] - 1])[-1]
    calibrate(nn, nnet_feats, llh_std, ivec)
    kf.write_final_mdl(os.path.join(out_dir, "am", "final.mdl"), tm, nn)
    if graph == "lookahead":
        kf.write_lookahead_fst(os.path.join(out_dir, "graph", "HCLr.fst"), fst)
        kf.write_ngram_fst(os.path.join(out_dir, "graph", "Gr.fst"), lm)
        with open(os.path.join(out_dir, "graph", "disambig_tid.int"), "w") as f:
            f.write("".join(f"{d}\n" for d in disambig))
    else:
        kf.write_const_fst(os.path.join(out_dir, "graph", "HCLG.fst"), fst)
    with open(os.path.join(out_dir, "graph", "words.txt"), "w") as f:
        f.write("<eps> 0\n")
        for i, _ in enumerate(words):
            f.write(f"w{i + 1:05d} {i + 1}\n")
        f.write(f"#0 {len(words) + 1}\n<s> {len(words) + 2}\n</s> {len(words) + 3}\n")
    with open(os.path.join(out_dir, "graph", "phones", "word_boundary.int"), "w") as f:
        f.write("1 nonword\n")
        for p in range(2, num_pos_phones + 1):
            f.write(f"{p} {('begin', 'end', 'internal', 'singleton')[(p - 2) % 4]}\n")
    with open(os.path.join(out_dir, "README"), "w") as f:
        f.write(f"synthetic vosk-api_amd model seed={seed} vocab={vocab} pdfs={num_pdfs} "
                f"phones={num_pos_phones} ivector_dim={ivector_dim} frontend={frontend} "
                f"global_cmvn={int(global_cmvn)} graph={graph} states={fst.num_states} "
                f"arcs={fst.num_arcs}\n")
    return out_dir


SPK_MFCC_CONF = """--sample-frequency=16000
--frame-length=25 # the default is 25
--low-freq=20 # the default.
--high-freq=7600 # the default is zero meaning use the Nyquist (8k in this case).
--num-mel-bins=30
--num-ceps=30
--snip-edges=false
--dither=0
"""


def make_spk_model(out_dir, seed=5, hidden=128, stats_dim=192, embed=128, out=64):
    """Synthetic speaker model (the reference reads
    mfcc.conf, final.ext.raw, mean.vec and transform.mat,
    src/spk_model.cc:17-32): a Kaldi x-vector topology (TDNN layers with
    splicing, statistics extraction + mean/stddev pooling over the whole
    input, the embedding affine) with seeded random weights."""
    rng = np.random.default_rng(seed)
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "mfcc.conf"), "w") as f:
        f.write(SPK_MFCC_CONF)
    D = 30
    lines = [f"input-node name=input dim={D}"]
    comps, order = {}, []

    def add(name, comp, inp):
        lines.append(f"component-node name={name} component={name} input={inp}")
        comps[name] = comp
        order.append(name)

    def layer(i, din, dout, splice, src):
        terms = [src if o == 0 else f"Offset({src}, {o})" for o in splice]
        inp = terms[0] if len(terms) == 1 else "Append(" + ", ".join(terms) + ")"
        add(f"tdnn{i}.affine", nat_affine(rng, din * len(splice), dout), inp)
        add(f"tdnn{i}.relu", relu(dout), f"tdnn{i}.affine")
        add(f"tdnn{i}.batchnorm", batchnorm(dout), f"tdnn{i}.relu")
        return f"tdnn{i}.batchnorm"

    x = layer(1, D, hidden, [-2, -1, 0, 1, 2], "input")
    x = layer(2, hidden, hidden, [-2, 0, 2], x)
    x = layer(3, hidden, hidden, [-3, 0, 3], x)
    x = layer(4, hidden, hidden, [0], x)
    x = layer(5, hidden, stats_dim, [0], x)
    add("stats-extraction-0-10000", ("StatisticsExtractionComponent", [
        ("<InputDim>", stats_dim), ("<InputPeriod>", 1), ("<OutputPeriod>", 1),
        ("<IncludeVarinance>", True)]), x)
    add("stats-pooling-0-10000", ("StatisticsPoolingComponent", [
        ("<InputDim>", 1 + 2 * stats_dim), ("<InputPeriod>", 1), ("<LeftContext>", 0),
        ("<RightContext>", 10000), ("<NumLogCountFeatures>", 0), ("<OutputStddevs>", True),
        ("<VarianceFloor>", 1e-10)]), "stats-extraction-0-10000")
    add("tdnn6.affine", nat_affine(rng, 2 * stats_dim, embed, gain=1.0), "Round(stats-pooling-0-10000, 1)")
    lines.append("output-node name=output input=tdnn6.affine objective=linear")
    kf.write_nnet3_raw(os.path.join(out_dir, "final.ext.raw"), kf.Nnet3(lines, comps, order))
    kf.write_vector_file(os.path.join(out_dir, "mean.vec"),
                         (rng.standard_normal(embed) * 0.1).astype(np.float32))
    kf.write_matrix_file(os.path.join(out_dir, "transform.mat"),
                         (rng.standard_normal((out, embed)) / math.sqrt(embed)).astype(np.float32))
    with open(os.path.join(out_dir, "README"), "w") as f:
        f.write(f"synthetic vosk-api_amd speaker model seed={seed} stats={stats_dim} "
                f"embed={embed} out={out}\n")
    return out_dir


def add_rescore(model_dir, seed=3):
    """rescore/G.fst (the LM to subtract: a backoff bigram acceptor whose
    backoff arcs carry #0 on the input, as Kaldi's G.fst) and rescore/G.carpa
    (a ConstArpa trigram over the model's words with <s> / </s>),
    src/model.cc:308-314."""
    rng = np.random.default_rng(seed)
    words = kf.read_symbol_table(os.path.join(model_dir, "graph", "words.txt"))
    sym = {v: k for k, v in words.items()}
    vocab = sorted(i for i, w in words.items() if w.startswith("w"))
    disamb, bos, eos = sym["#0"], sym["<s>"], sym["</s>"]
    os.makedirs(os.path.join(model_dir, "rescore"), exist_ok=True)
    # G.fst: state 0 = unigram; bigram states for some words
    big = [int(w) for w in rng.choice(vocab, size=min(60, len(vocab)), replace=False)]
    bstate = {w: i + 1 for i, w in enumerate(big)}
    arcs = []
    uni = {w: float(rng.uniform(4.0, 10.0)) for w in vocab}
    for w in vocab:
        arcs.append((0, w, w, uni[w], bstate.get(w, 0)))
    for w, s in bstate.items():
        for v in rng.choice(vocab, size=12, replace=False):
            v = int(v)
            arcs.append((s, v, v, float(uni[v] * rng.uniform(0.3, 0.9)), bstate.get(v, 0)))
        arcs.append((s, disamb, 0, float(rng.uniform(0.3, 1.5)), 0))
    S = 1 + len(big)
    arcs.sort(key=lambda a: (a[0], a[1]))
    row = np.zeros(S + 1, np.int64)
    np.add.at(row, np.array([a[0] for a in arcs]) + 1, 1)
    final = np.full(S, np.inf, np.float32)
    final[0] = 3.0
    for s in range(1, S):
        if rng.random() < 0.3:
            final[s] = float(rng.uniform(1.0, 4.0))
    g = kf.Fst(0, final, np.cumsum(row), np.array([a[1] for a in arcs], np.int32),
               np.array([a[2] for a in arcs], np.int32), np.array([a[3] for a in arcs], np.float32),
               np.array([a[4] for a in arcs], np.int32))
    kf.write_vector_fst(os.path.join(model_dir, "rescore", "G.fst"), g)
    # ConstArpa trigram (natural-log probabilities, backoffs)
    ng = {(bos,): (-99.0, float(-rng.uniform(0.1, 1.0))), (eos,): (-3.0, 0.0)}
    for w in vocab:
        ng[(w,)] = (-uni[w], float(-rng.uniform(0.1, 1.0)))
    hist1 = [bos] + [int(w) for w in rng.choice(vocab, size=min(80, len(vocab)), replace=False)]
    for h in hist1:
        for v in list(rng.choice(vocab, size=10, replace=False)) + [eos]:
            ng[(h, int(v))] = (float(-rng.uniform(0.5, 6.0)), float(-rng.uniform(0.05, 0.8)))
    pairs = [k for k in ng if len(k) == 2 and k[1] != eos]
    for k in pairs[: len(pairs) // 3]:
        for v in rng.choice(vocab, size=4, replace=False):
            ng[k + (int(v),)] = (float(-rng.uniform(0.2, 3.0)), 0.0)
    # an n-gram that extends to no longer n-gram backs off with weight 1 (log 0)
    ctx = {k[:-1] for k in ng if len(k) > 1}
    ng = {k: (v[0], v[1] if (k in ctx or len(k) == 1) else 0.0) for k, v in ng.items()}
    kf.write_const_arpa(os.path.join(model_dir, "rescore", "G.carpa"), ng, bos, eos, -1, 3)
    return ng


# Named models for the large-graph tests and the benchmark.  llh_std 1.5
# gives the realistic active-token regime (hundreds to ~20 k tokens per frame
# at beam 13, max-active 7000 engaged in some frames) that the reference's
# batch decoder settings target (src/batch_model.cc:78-80).
PRESETS = {
    # BASELINE config 4's per-GPU share: a multi-million-state static HCLG
    "bigram_2m": dict(seed=21, vocab=20000, num_pdfs=2000, llh_std=1.5, graph="bigram",
                      graph_opts=dict(num_hist=2000, fut=300)),
    # BASELINE config 4 stand-in several times the 2.4 M-state graph (the
    # static HCLG of vosk-model-en-us-0.22 is larger than any graph the
    # tests can build in seconds; what matters is that per-stream decoder
    # state does not grow with the graph)
    "bigram_8m": dict(seed=23, vocab=20000, num_pdfs=2000, llh_std=1.5, graph="bigram",
                      graph_opts=dict(num_hist=6400, fut=300)),
    # vosk-model-small-en-us scale (BASELINE config 3): 20 k-word HCLr + a
    # ~29 k-history trigram Gr, expanded at load to ~275 k states (with pushing)
    "la_small_en_us": dict(seed=11, vocab=20000, num_pdfs=2000, llh_std=1.5, graph="lookahead",
                           graph_opts=dict(n_big=20000, fut_big=24, n_tri=3000)),
}


def make_preset(name, out_dir):
    return make_model(out_dir, **PRESETS[name])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--vocab", type=int, default=3000)
    ap.add_argument("--pdfs", type=int, default=2000)
    ap.add_argument("--graph", choices=("hclg", "bigram", "lookahead"), default="hclg")
    ap.add_argument("--num-hist", type=int, default=None, help="bigram: LM histories")
    ap.add_argument("--fut", type=int, default=None, help="bigram: successor words per history")
    ap.add_argument("--llh-std", type=float, default=3.0,
                    help="output log-likelihood spread the nnet is calibrated to (smaller: "
                         "flatter scores, more active tokens)")
    ap.add_argument("--preset", choices=sorted(PRESETS), default=None,
                    help="a named model of models_for_bench(); overrides the other options")
    a = ap.parse_args()
    if a.preset:
        make_preset(a.preset, a.out)
    else:
        go = {k: v for k, v in (("num_hist", a.num_hist), ("fut", a.fut)) if v is not None}
        make_model(a.out, a.seed, a.vocab, a.pdfs, llh_std=a.llh_std, graph=a.graph, graph_opts=go)
    print(open(os.path.join(a.out, "README")).read().strip())


if __name__ == "__main__":
    main()
