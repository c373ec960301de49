/*
 * oracle.h -- CPU restatement of the Vosk/Kaldi hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * (or the timed CPU baseline).  The product (libvosk.so) never links it.
 *
 * PARITY STATUS: "parity unpinned" against real Kaldi.  The reference's
 * arithmetic lives in Kaldi/OpenFST, which are not vendored in
 * /root/reference, cannot be built here and ship no
 * golden vectors for MFCC / nnet3 / decoder values.  The only recorded
 * outputs (python/example/colab/vosk.ipynb) need vosk-model-small-en-us-0.15,
 * which is absent.  This oracle restates the published Kaldi algorithms
 * (citations per function in oracle.c) with a fully specified fp32
 * operation order; the HIP kernels reproduce that order, so GPU-vs-oracle
 * parity is checked bit-exactly.
 */
#ifndef VAMD_ORACLE_H
#define VAMD_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- MFCC (Kaldi feat/feature-mfcc.cc et al.) ---------------- */
typedef struct {
  float samp_freq, frame_shift_ms, frame_length_ms, preemph_coeff;
  float low_freq, high_freq, cepstral_lifter, blackman_coeff;
  int num_bins, num_ceps, use_energy, remove_dc_offset;
  int window_type; /* 0 povey, 1 hamming, 2 hanning, 3 rectangular, 4 blackman */
  int round_to_power_of_two;
  /* fbank front end (Kaldi feat/feature-fbank.cc, src/model.cc:222-225):
     log mel energies, log energy first when use_energy */
  int fbank, use_log_fbank, use_power;
  /* snip_edges = 0 (the speaker front end, Kaldi FeatureWindow): frame t
     starts at t*shift + shift/2 - length/2, samples before 0 are reflected,
     and the online (not flushed) frame count applies */
  int snip_edges;
} orc_mfcc_opts;

/* feature dimension of the front end: num_ceps (MFCC) or num_bins (+1) (fbank) */
int orc_feat_dim(const orc_mfcc_opts* o);
/* Kaldi OnlineCmvn with global stats only (mean normalization; the running
   window sums in double, SmoothOnlineCmvnStats, ApplyCmvn), as the
   reference's feature pipeline applies it with am/global_cmvn.stats
   (src/model.cc:265-269) and as the i-vector extractor's CMVN does.
   gstats: [2][D+1] (row 0 sums and count).  out may equal nothing of feats. */
void orc_online_cmvn(const double* gstats, int D, int window, int global_frames,
                     const float* feats, int T, float* out);

/* Windowed-sinc resampling (Kaldi feat/resample.cc LinearResample, as the
   reference uses it: src/batch_recognizer.cc:27-29, filter cutoff
   min(rate_in, rate_out)/2, 6 zeros), whole signal with end-of-input flush.
   Output sample k = sequential fmaf chain over the taps of its phase (in tap
   order, from 0), input samples outside [0, n) contribute nothing.
   Returns the number of output samples (<= cap) or -1. */
long orc_resample_num_outputs(int rate_in, int rate_out, long n);
long orc_resample(int rate_in, int rate_out, const float* x, long n, float* out, long cap);

int orc_mfcc_num_frames(const orc_mfcc_opts* o, long num_samples);
/* wave: float samples (int16 range).  out: [frames][orc_feat_dim]. returns frames */
int orc_mfcc(const orc_mfcc_opts* o, const float* wave, long num_samples, float* out);
int orc_kslices(int K);
float orc_logf(float x);

/* ---------------- nnet3 forward (whole utterance, edge-replicated input) ---- */
typedef struct {
  int num_nodes;      /* topological order; node 0 is the feature input */
  const int* kind;    /* 0 input, 1 affine, 2 relu, 3 mul_add, 4 identity */
  const int* dim;     /* output dim per node */
  const int* in_dim;  /* descriptor dim per node (before TDNN splicing) */
  const int64_t* w_off; const int64_t* b_off; const int64_t* s_off; const int64_t* o_off;
  const float* params;
  const int* toff_begin; const int* toff_count; const int* toffs;
  const int* prog_begin; const int* prog; const float* progf;
  int output_node, fss;
  float acoustic_scale;
  /* i-vector input (ReplaceIndex(ivector, t, 0), descriptor op 4): the row
     computed at time t uses ivec[ivec_of_time[clamp(t - ivec_t0)]] -- the
     i-vector of the looped chunk that first computes row t */
  const float* ivec; const int* ivec_of_time;
  int ivec_t0, ivec_ntimes, ivec_dim;
} orc_net;

/* out: [ceil(T/fss)][dim(output)] */
int orc_nnet_forward(const orc_net* net, const float* feats, int T, float* out);

/* ---------------- speaker x-vectors (src/recognizer.cc:356-419) -------------
   Sliding-window CMN (Kaldi SlidingWindowCmn, centered, means only, in
   double: out = x + (-1 / frames) * window sum), then -- after the
   frame-level nnet (orc_nnet_forward up to the statistics input) --
   orc_xvector_tail: statistics pooling over rows [r0, r1] (double sums in row
   order; [log count x nlog], mean, stddev = sqrt(max(floor, E[x^2] -
   mean^2))), the head ops (1 affine W [out][in] + b in the canonical order,
   2 ReLU, 3 x * scale + offset), x - mean, transform rows (canonical order),
   and the scale to norm sqrt(R) (sequential float sum of squares; ratio and
   1/ratio through double).  Shared bit-for-bit with kernels.hip xvec_*. */
void orc_sliding_cmn(const float* feats, int T, int D, int window, float* out);
typedef struct {
  int stats_dim, nlog, stddevs;
  float var_floor;
  int nops;
  const int* kind; const int* in_dim; const int* out_dim;
  const int64_t* w_off; const int64_t* b_off;  /* into params; b_off -1: no bias */
  const float* params;
  int embed_dim, out_dim_final;
  const float* mean;       /* [embed_dim] */
  const float* transform;  /* [out_dim_final][embed_dim] */
} orc_xvec;
int orc_xvector_tail(const orc_xvec* x, const float* rows, int ld, int r0, int r1, float* out);

/* ---------------- online i-vector extraction ----------------------------------
   Kaldi online2/online-ivector-feature.cc (OnlineIvectorFeature with
   use_most_recent_ivector), ivector/ivector-extractor.cc
   (OnlineIvectorEstimationStats, max_count via prior scaling),
   matrix/optimization.cc (LinearCgd), as configured by the reference
   (src/model.cc:247-263).  Operation order is fixed (shared with the GPU):
   CMVN running double sums, ApplyCmvn float offsets, LDA / UBM dot products
   as sequential fmaf chains, posteriors with orc_expf, double statistics,
   CG with sequential dot products and row-wise mat-vecs. */
float orc_expf(float x);
typedef struct {
  int feat_dim;             /* D_in (40) */
  int left, right;          /* splice context (3, 3) */
  int lda_rows, lda_cols;   /* lda: [lda_rows][lda_cols], cols = (l+r+1)*D_in (+1 offset) */
  const float* lda;
  const double* cmvn;       /* global stats [2][D_in + 1] */
  int cmn_window, global_frames;
  int num_gauss;
  const float* gconsts;     /* [G] */
  const float* means_invvars; /* [G][lda_rows] */
  const float* inv_vars;    /* [G][lda_rows] */
  int ivec_dim;             /* S */
  const double* M;          /* [G][lda_rows][S] */
  const double* sigma_inv;  /* [G][lda_rows][lda_rows] (full) */
  double prior_offset, max_count;
  int num_gselect, num_cg_iters;
  float min_post, posterior_scale;
} orc_ivector_model;
/* requests[i]: frame whose i-vector is wanted (ascending); t_ready[i]: MFCC
   frames available at the request (splice clamps at t_ready - 1); out: [nreq][S]
   with the prior offset removed from dimension 0.  Returns 0. */
int orc_ivector_extract(const orc_ivector_model* m, const float* feats, int T, const int* requests,
                        const int* t_ready, int nreq, float* out);
/* the same with silence weighting: request q applies the (frame, delta
   weight) entries [ent_off[q], ent_off[q+1]) instead of its new frames */
int orc_ivector_extract_w(const orc_ivector_model* m, const float* feats, int T, const int* requests,
                          const int* t_ready, int nreq, const int* ent_off, const int* ent_frame,
                          const float* ent_w, float* out);

/* ---------------- token-passing decoder (Kaldi decoder/lattice-faster-decoder.cc) */
typedef struct {
  float beam, beam_delta;
  int max_active, min_active;
  int hash_size;  /* orc_decode_kaldi: the HashList size at the start (0: a new decoder's 1000) */
  /* orc_decode_kaldi, optional (NULL: state ids as numbered in the graph):
     OpenFST's lazy ComposeFst numbering.  The graph's states are renumbered
     for HashList bucketing as the decoder first expands them: the start is
     0, and a state's arc destinations without an id take the next ids in
     the order of the state's arcs, lazy_next[lazy_row[s] .. lazy_row[s+1])
     (the composed FST's own arc order, emitting and epsilon arcs
     interleaved).  Kaldi's decoder expands a state when it first iterates
     its arcs or asks NumInputEpsilons (ProcessNonemitting's queue fill over
     every new token in list order, then each token the queue creates or
     improves). */
  const int64_t* lazy_row;
  const int* lazy_next;
  /* optional with lazy_next: the numbering state carried across decodes (a
     recognizer's ComposeFst outlives its decoder's InitDecoding): ids
     [lazy_ids], expanded flags [states], the next id (0: start fresh);
     updated in place.  NULL: a fresh numbering for this decode. */
  int* lazy_disc;
  char* lazy_expanded;
  int* lazy_count;
} orc_dec_opts;

typedef struct {
  int num_states, start;
  const int64_t* arc_begin; /* [S+1] */
  const int64_t* eps_begin; /* [S]   */
  const int* ilabel; const int* olabel; const int* nextstate;
  const float* weight; const float* final_cost;
  const int* tid2pdf;
} orc_graph;

typedef struct {
  int* ntok;          /* [F+1] tokens per frame (frame 0 = after init) */
  float* best;        /* [F+1] min tot_cost per frame                  */
  float* cutoff;      /* [F]   GetCutoff result per frame               */
  float* next_cutoff; /* [F]   emitting cutoff per frame                */
  int64_t* arcs_emit; /* [F]   emitting arcs examined (roofline counter) */
  int* path;          /* traceback arc indices (forward order)          */
  int path_cap, path_len;
  double best_cost;   /* offset-corrected cost of the best path (+final) */
  float best_tot;     /* raw tot_cost of the chosen end token            */
  int end_state;
  float final_relative_cost;
  /* optional raw lattice (LatticeFasterDecoder tokens and forward links, in
     the order-independent formulation): frame index k = 0 for the initial
     closure, f + 1 after frame f.  Tokens of frame k are
     [lat_frame_begin[k], lat_frame_begin[k+1]) with (state, cost); links
     (frame k of their destination, source state, arc, acoustic cost incl.
     the frame's cost offset; 0 for epsilon links). NULL = not wanted. */
  int* lat_frame_begin;  /* [F + 2] */
  int* lat_tok_state; float* lat_tok_cost; int lat_tok_cap, lat_ntok;
  int* lat_link_frame; int* lat_link_src; int* lat_link_arc; float* lat_link_ac;
  int lat_link_cap, lat_nlink;
  float* lat_cost_offset; /* [F + 1] cost offset of the links into frame k */
  int hash_size;          /* orc_decode_kaldi: the HashList size at the end */
  /* optional endpoint probes (orc_decode_kaldi; nprobe 0 = none): after
     probe_frames[i] decoded frames (ascending), the best path WITHOUT final
     costs (what an endpoint check traces back) as arc indices in
     probe_path[probe_off[i] .. probe_off[i+1]), and the final relative cost
     in probe_frc[i].  One decoding pass answers every probe of a segment. */
  const int* probe_frames; int nprobe;
  int* probe_path; long long probe_path_cap; long long* probe_off; float* probe_frc;
} orc_dec_result;

int orc_decode(const orc_graph* g, const float* llh, int num_frames, int llh_stride,
               const orc_dec_opts* o, int use_final, orc_dec_result* r);
/* Kaldi-sequential token passing (LatticeFasterDecoderTpl with its HashList
   iteration order, running emitting cutoff and LIFO epsilon queue), the GPU
   decoder's default semantics.  Fills everything orc_decode does (lattice
   included) and the HashList size at the end. */
int orc_decode_kaldi(const orc_graph* g, const float* llh, int num_frames, int llh_stride,
                     const orc_dec_opts* o, int use_final, orc_dec_result* r);

#ifdef __cplusplus
}
#endif
#endif
