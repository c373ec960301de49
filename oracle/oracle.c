/*
 * oracle.c -- CPU restatement of the Vosk/Kaldi hot path (TEST INFRASTRUCTURE
 * ONLY; see oracle.h for the parity status: unpinned vs Kaldi, bit-exact
 * contract vs the HIP kernels).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off).  Contraction must stay
 * off: every fused multiply-add below is an explicit fmaf(), every other
 * product/sum is rounded separately, exactly as in the HIP kernels.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ===================================================================== */
/* MFCC                                                                  */
/* Kaldi feat/feature-window.cc (ExtractWindow/ProcessWindow),            */
/* feat/mel-computations.cc (MelBanks), feat/feature-mfcc.cc (Compute),   */
/* matrix/matrix-functions.cc (ComputeDctMatrix).  Reference call site:   */
/* src/model.cc:218-221 (mfcc.conf -> OnlineNnet2FeaturePipeline).        */
/* Deviation (documented): radix-2 complex FFT instead of Kaldi's         */
/* split-radix real FFT; sums as sequential fp32 chains; custom log.      */
/* ===================================================================== */

static int frame_length(const orc_mfcc_opts* o) { return (int)(o->samp_freq * 0.001f * o->frame_length_ms); }
static int frame_shift(const orc_mfcc_opts* o) { return (int)(o->samp_freq * 0.001f * o->frame_shift_ms); }
static int padded_length(const orc_mfcc_opts* o) {
  int n = frame_length(o), p = 1;
  if (!o->round_to_power_of_two) return n;
  while (p < n) p <<= 1;
  return p;
}

int orc_mfcc_num_frames(const orc_mfcc_opts* o, long n) {
  int L = frame_length(o), S = frame_shift(o);
  if (!o->snip_edges) { /* FeatureWindow NumFrames(flush=false), snip_edges=false */
    long nf = (n + S / 2) / S, end = (nf - 1) * S + S / 2 - L / 2 + L;
    while (nf > 0 && end > n) { nf--; end -= S; }
    return (int)nf;
  }
  if (n < L) return 0;
  return (int)(1 + (n - L) / S);
}

/* natural log, x > 0 normal: log(m*2^e) = e*ln2 + log1p(m-1),
   m in [sqrt(.5), sqrt(2)); log1p via a degree-10 polynomial (Horner fmaf) */
/* Canonical affine summation order shared with the GPU engine
   (vosk-api_amd/csrc/nnet_plan.h GemmKSlices / kernels.hip): K is cut into
   orc_kslices(K) equal slices, slice sums added left to right.  Inside a
   slice the fmaf chain starts from 0 and walks each aligned group of eight k
   as 0,4,1,5,2,6,3,7 (the pair order in which a 32x32x2 MFMA fed with one
   float4 per lane accumulates).  Kaldi's own order is whatever its BLAS does
   (matrix/kaldi-matrix.cc AddMatMat -> cblas_sgemm), so any fixed order is a
   faithful restatement of the arithmetic. */
/* ---- exp for posteriors: 2^k * e^r, |r| <= ln2/2, degree-7 Taylor (Horner,
   fmaf).  Shared bit-for-bit with kernels.hip dev_expf. */
float orc_expf(float x) {
  if (x < -87.0f) return 0.0f;
  const float k = rintf(x * 1.44269504f);
  float r = fmaf(-k, 0.693145752f, x);
  r = fmaf(-k, 1.42860677e-6f, r);
  float p = 1.98412698e-4f;
  p = fmaf(p, r, 1.38888889e-3f);
  p = fmaf(p, r, 8.33333333e-3f);
  p = fmaf(p, r, 4.16666667e-2f);
  p = fmaf(p, r, 1.66666667e-1f);
  p = fmaf(p, r, 0.5f);
  p = fmaf(p, r, 1.0f);
  p = fmaf(p, r, 1.0f);
  return ldexpf(p, (int)k);
}

/* ---- online CMVN (Kaldi feat/online-feature.cc OnlineCmvn::GetFrame with
   global stats only: ComputeStatsForFrame's running window sums, then
   SmoothOnlineCmvnStats and ApplyCmvn without variance normalization) ---- */
void orc_online_cmvn(const double* gstats, int D, int window, int global_frames,
                     const float* feats, int T, float* out) {
  double sum[256] = {0}, n = 0.0;
  const double gcount = gstats[D];
  for (int t = 0; t < T; t++) {
    for (int d = 0; d < D; d++) sum[d] = sum[d] + (double)feats[(size_t)t * D + d];
    n = n + 1.0;
    if (t - window >= 0) {
      for (int d = 0; d < D; d++) sum[d] = sum[d] - (double)feats[(size_t)(t - window) * D + d];
      n = n - 1.0;
    }
    double st[256], cnt = n;
    for (int d = 0; d < D; d++) st[d] = sum[d];
    if (cnt < window) {
      double cg = window - cnt;
      if (cg > global_frames) cg = global_frames;
      const double sc = cg / gcount;
      for (int d = 0; d < D; d++) st[d] = st[d] + sc * gstats[d];
      cnt = cnt + sc * gcount;
    }
    const float alpha = (float)(-1.0 / cnt);
    for (int d = 0; d < D; d++) {
      const float off = (float)((double)alpha * st[d]);
      out[(size_t)t * D + d] = feats[(size_t)t * D + d] + off;
    }
  }
}

/* ---- online i-vector extraction ----------------------------------------- */
/* one row of an affine map in the canonical order (see the nnet affine
   case in orc_nnet_forward): fmaf chains from 0 over orc_kslices(K) slices,
   each aligned group of eight walked 0,4,1,5,2,6,3,7, slices summed left to
   right.  Kaldi leaves these products to BLAS (the LDA's AddMatVec,
   DiagGmm::LogLikelihoods' AddMatVec pair), so any fixed order restates it;
   this one is the GPU GEMM's. */
static float canon_dot(const float* w, const float* x, int K) {
  const int ns = orc_kslices(K), kw = K / ns;
  float a = 0.0f;
  for (int z = 0; z < ns; z++) {
    float p = 0.0f;
    const int ke = (z + 1) * kw;
    for (int kg = z * kw; kg < ke; kg += 8)
      for (int i = 0; i < 8 && kg + i < ke; i++) {
        const int k = kg + 8 <= ke ? kg + ((i & 1) << 2) + (i >> 1) : kg + i;
        p = fmaf(x[k], w[k], p);
      }
    a = z == 0 ? p : a + p;
  }
  return a;
}

static void iv_lda(const orc_ivector_model* m, const float* src, int t, int t_ready, float* y) {
  const int D = m->feat_dim, ctx = m->left + m->right + 1, K = ctx * D;
  float x[64 * 16];
  for (int c = 0; c < ctx; c++) {
    int u = t - m->left + c;
    if (u < 0) u = 0;
    if (u > t_ready - 1) u = t_ready - 1;
    memcpy(x + c * D, src + (size_t)u * D, sizeof(float) * D);
  }
  for (int i = 0; i < m->lda_rows; i++) {
    const float* w = m->lda + (size_t)i * m->lda_cols;
    float a = canon_dot(w, x, K);
    if (m->lda_cols == K + 1) a = a + w[K];
    y[i] = a;
  }
}

static void iv_matvec(const double* Q, int S, const double* x, double* y) {
  /* Q packed lower triangle (row i: i+1 entries) */
  for (int i = 0; i < S; i++) {
    double a = 0.0;
    for (int j = 0; j < S; j++) {
      const int r = i > j ? i : j, c = i > j ? j : i;
      a = a + Q[(size_t)r * (r + 1) / 2 + c] * x[j];
    }
    y[i] = a;
  }
}

static double iv_dot(const double* a, const double* b, int n) {
  double s = 0.0;
  for (int i = 0; i < n; i++) s = s + a[i] * b[i];
  return s;
}

static void iv_cgd(const double* Q, const double* b, int S, int max_iters, double* x) {
  double p[128], r[128], Ap[128];
  iv_matvec(Q, S, x, Ap);
  for (int i = 0; i < S; i++) p[i] = b[i] - Ap[i];
  for (int i = 0; i < S; i++) r[i] = -p[i];
  double rcur = iv_dot(r, r, S), rrec = rcur;
  for (int k = 0; k < S + 5 && k != max_iters; k++) {
    iv_matvec(Q, S, p, Ap);
    const double alpha = -iv_dot(p, r, S) / iv_dot(p, Ap, S);
    for (int i = 0; i < S; i++) x[i] = x[i] + alpha * p[i];
    for (int i = 0; i < S; i++) r[i] = r[i] + alpha * Ap[i];
    double rnext = iv_dot(r, r, S);
    if (rnext < 1e-4 * rrec || rnext > 1e4 * rrec) {
      iv_matvec(Q, S, x, Ap);
      for (int i = 0; i < S; i++) r[i] = Ap[i] - b[i];
      rnext = iv_dot(r, r, S);
      rrec = rnext;
    }
    if (rnext <= 2.2250738585072014e-308) break;
    const double beta = rnext / rcur;
    for (int i = 0; i < S; i++) p[i] = beta * p[i] - r[i];
    rcur = rnext;
  }
}

/* one frame's record (OnlineIvectorFeature::UpdateStatsForFrames): LDA of
   the CMVN-normalized splice, diagonal-UBM log-likelihoods, num_gselect best
   Gaussians (descending, ties by lower index) pruned by min_post, their
   posteriors before any frame weight, and the LDA of the raw splice */
typedef struct {
  int ns, sel[16];
  float post[16];
  float xr[256];
} iv_rec;

static void iv_record(const orc_ivector_model* m, const float* norm, const float* feats, int t,
                      int t_ready, const float* wubm, float* ll, iv_rec* R) {
  const int DL = m->lda_rows, G = m->num_gauss;
  const float log_min_post = (float)log((double)m->min_post);
  float xn[256], xq[512];
  iv_lda(m, norm, t, t_ready, xn);
  for (int d = 0; d < DL; d++) {
    xq[d] = xn[d];
    xq[DL + d] = xn[d] * xn[d];
  }
  for (int g = 0; g < G; g++) ll[g] = canon_dot(wubm + (size_t)g * 2 * DL, xq, 2 * DL) + m->gconsts[g];
  int ns = 0;
  for (int k = 0; k < m->num_gselect && k < G; k++) {
    int b = -1;
    for (int g = 0; g < G; g++) {
      int used = 0;
      for (int j = 0; j < ns; j++) used |= R->sel[j] == g;
      if (used) continue;
      if (b < 0 || ll[g] > ll[b]) b = g;
    }
    R->sel[ns++] = b;
  }
  while (ns > 1 && ll[R->sel[ns - 1]] < ll[R->sel[0]] + log_min_post) ns--;
  float e[16], tot = 0.0f;
  for (int k = 0; k < ns; k++) {
    e[k] = orc_expf(ll[R->sel[k]] - ll[R->sel[0]]);
    tot = tot + e[k];
  }
  for (int k = 0; k < ns; k++) R->post[k] = e[k] / tot;
  R->ns = ns;
  iv_lda(m, feats, t, t_ready, R->xr);
}

/* One statistics batch (OnlineIvectorFeature::UpdateStatsForFrames ->
   OnlineIvectorEstimationStats::AccStats over a matrix of frames [K]): the
   frame weight folded into the posteriors as Kaldi does (post *
   (posterior_scale * w), in float; zero-weight frames dropped; negative
   weights undo earlier contributions), zeroth and first order statistics
   aggregated per Gaussian (gamma_g, X_g = sum post * x, in frame order),
   then per Gaussian in ascending index: linear += SigmaInvM_g^T X_g,
   quadratic += gamma_g U_g; the batch weight (sum of gamma_g, ascending g)
   updates the frame count and Kaldi's max-count prior rescaling once. */
typedef struct {
  double lin[128], cur[128];
  double* quad;
  double nfr;
  double* gamma;   /* [G] scratch */
  double* X;       /* [G][DL] scratch */
  char* used;      /* [G] */
} iv_stats;

static void iv_accumulate_batch(const orc_ivector_model* m, const double* SIM, const double* U,
                                const iv_rec* const* recs, const float* ws, int n, iv_stats* st) {
  const int DL = m->lda_rows, S = m->ivec_dim, QS = S * (S + 1) / 2, G = m->num_gauss;
  memset(st->used, 0, G);
  for (int i = 0; i < n; i++) {
    const iv_rec* R = recs[i];
    const float w = ws[i];
    if (w == 0.0f) continue;
    for (int k = 0; k < R->ns; k++) {
      const double p = (double)(R->post[k] * (m->posterior_scale * w));
      if (p == 0.0) continue;
      const int g = R->sel[k];
      if (!st->used[g]) {
        st->used[g] = 1;
        st->gamma[g] = 0.0;
        for (int d = 0; d < DL; d++) st->X[(size_t)g * DL + d] = 0.0;
      }
      st->gamma[g] = st->gamma[g] + p;
      for (int d = 0; d < DL; d++)
        st->X[(size_t)g * DL + d] = st->X[(size_t)g * DL + d] + p * (double)R->xr[d];
    }
  }
  double tw = 0.0;
  for (int g = 0; g < G; g++) {
    if (!st->used[g]) continue;
    const double* sm = SIM + (size_t)g * DL * S;
    const double* x = st->X + (size_t)g * DL;
    for (int s2 = 0; s2 < S; s2++) {
      double a = 0.0;
      for (int d = 0; d < DL; d++) a = fma(sm[(size_t)d * S + s2], x[d], a);
      st->lin[s2] = st->lin[s2] + a;
    }
    const double* u = U + (size_t)g * QS;
    for (int i = 0; i < QS; i++) st->quad[i] = st->quad[i] + st->gamma[g] * u[i];
    tw = tw + st->gamma[g];
  }
  if (m->max_count > 0.0) {
    const double mc = m->max_count, nfr = st->nfr;
    const double oldp = (nfr > mc ? nfr : mc) / mc, newn = nfr + tw;
    const double newp = (newn > mc ? newn : mc) / mc, ch = newp - oldp;
    if (ch != 0.0) {
      st->lin[0] = st->lin[0] + m->prior_offset * ch;
      for (int i = 0; i < S; i++) st->quad[(size_t)i * (i + 1) / 2 + i] += ch;
    }
  }
  st->nfr = st->nfr + tw;
}

/* Requests in order; request q = the i-vector at frame requests[q] with
   t_ready[q] feature frames available.  A request past the frames already
   accumulated first computes the records of the new frames, then applies
   either every new frame with weight 1 (ent_off == NULL: no silence
   weighting, OnlineIvectorFeature::UpdateStatsUntilFrame) or the entries
   [ent_off[q], ent_off[q+1]) (frame, delta weight) in the given order
   (UpdateStatsUntilFrameWeighted: the queued delta weights of frames <= the
   request, popped in (frame, weight) order), then the warm-started CG
   (IvectorEstimationStats::GetIvector; no net frames -> the prior). */
int orc_ivector_extract_w(const orc_ivector_model* m, const float* feats, int T, const int* requests,
                          const int* t_ready, int nreq, const int* ent_off, const int* ent_frame,
                          const float* ent_w, float* out) {
  const int D = m->feat_dim, DL = m->lda_rows, S = m->ivec_dim, G = m->num_gauss;
  const int QS = S * (S + 1) / 2;
  if (DL > 256 || S > 128 || m->num_gselect > 16) return -1;
  /* derived extractor terms (IvectorExtractor::ComputeDerivedVars) */
  double* SIM = (double*)malloc(sizeof(double) * (size_t)G * DL * S);
  double* U = (double*)malloc(sizeof(double) * (size_t)G * QS);
  for (int g = 0; g < G; g++) {
    const double* M = m->M + (size_t)g * DL * S;
    const double* SI = m->sigma_inv + (size_t)g * DL * DL;
    double* sm = SIM + (size_t)g * DL * S;
    for (int d = 0; d < DL; d++)
      for (int s2 = 0; s2 < S; s2++) {
        double a = 0.0;
        for (int e = 0; e < DL; e++) a = a + SI[(size_t)d * DL + e] * M[(size_t)e * S + s2];
        sm[(size_t)d * S + s2] = a;
      }
    double* u = U + (size_t)g * QS;
    for (int i = 0; i < S; i++)
      for (int j = 0; j <= i; j++) {
        double a = 0.0;
        for (int d = 0; d < DL; d++) a = a + M[(size_t)d * S + i] * sm[(size_t)d * S + j];
        u[(size_t)i * (i + 1) / 2 + j] = a;
      }
  }
  /* online CMVN (window cmn_window, smoothed with global_frames of global stats) */
  float* norm = (float*)malloc(sizeof(float) * (size_t)(T > 0 ? T : 1) * D);
  orc_online_cmvn(m->cmvn, D, m->cmn_window, m->global_frames, feats, T, norm);
  iv_stats st;
  memset(&st, 0, sizeof(st));
  st.quad = (double*)calloc(QS, sizeof(double));
  st.gamma = (double*)calloc(G, sizeof(double));
  st.X = (double*)calloc((size_t)G * DL, sizeof(double));
  st.used = (char*)calloc(G, 1);
  const int bcap = (T > 0 ? T : 1) + (ent_off ? ent_off[nreq] : 0) + 8;
  const iv_rec** brec = (const iv_rec**)malloc(sizeof(iv_rec*) * (size_t)bcap);
  float* bw = (float*)malloc(sizeof(float) * (size_t)bcap);
  st.lin[0] = m->prior_offset;
  for (int i = 0; i < S; i++) st.quad[(size_t)i * (i + 1) / 2 + i] = 1.0;
  st.cur[0] = m->prior_offset;
  int done = 0;
  float* ll = (float*)malloc(sizeof(float) * G);
  iv_rec* recs = (iv_rec*)malloc(sizeof(iv_rec) * (size_t)(T > 0 ? T : 1));
  /* UBM log-likelihoods as one affine row per Gaussian over [x | x*x]:
     [means_invvars | -0.5 inv_vars] (the -0.5 scaling is exact), gconst last */
  float* wubm = (float*)malloc(sizeof(float) * (size_t)G * 2 * DL);
  for (int g = 0; g < G; g++)
    for (int d = 0; d < DL; d++) {
      wubm[(size_t)g * 2 * DL + d] = m->means_invvars[(size_t)g * DL + d];
      wubm[(size_t)g * 2 * DL + DL + d] = -0.5f * m->inv_vars[(size_t)g * DL + d];
    }
  int rc = 0;
  for (int q = 0; q < nreq; q++) {
    const int f = requests[q];
    if (f >= done) {
      if (f >= T) { rc = -2; break; }
      for (int t = done; t <= f; t++) iv_record(m, norm, feats, t, t_ready[q], wubm, ll, &recs[t]);
      if (!ent_off) {  /* one batch: the new frames with weight 1 */
        for (int t = done; t <= f; t++) {
          brec[t - done] = &recs[t];
          bw[t - done] = 1.0f;
        }
        iv_accumulate_batch(m, SIM, U, brec, bw, f + 1 - done, &st);
      } else {  /* batches as popped: entries with frame <= done, then one per frame */
        int i = ent_off[q];
        while (i < ent_off[q + 1]) {
          const int key = ent_frame[i] > done ? ent_frame[i] : done;
          int nb = 0;
          while (i < ent_off[q + 1] && (ent_frame[i] > done ? ent_frame[i] : done) == key) {
            if (ent_frame[i] < 0 || ent_frame[i] > f || nb >= bcap) { rc = -3; break; }
            brec[nb] = &recs[ent_frame[i]];
            bw[nb++] = ent_w[i];
            i++;
          }
          if (rc) break;
          iv_accumulate_batch(m, SIM, U, brec, bw, nb, &st);
        }
        if (rc) break;
      }
      done = f + 1;
      if (st.nfr > 0.0) {
        iv_cgd(st.quad, st.lin, S, m->num_cg_iters, st.cur);
      } else {
        for (int i = 0; i < S; i++) st.cur[i] = 0.0;
        st.cur[0] = m->prior_offset;
      }
    }
    for (int i = 0; i < S; i++) out[(size_t)q * S + i] = (float)st.cur[i];
    out[(size_t)q * S] = out[(size_t)q * S] - (float)m->prior_offset;
  }
  free(SIM); free(U); free(norm); free(st.quad); free(ll); free(wubm); free(recs);
  free(st.gamma); free(st.X); free(st.used); free(brec); free(bw);
  return rc;
}

int orc_ivector_extract(const orc_ivector_model* m, const float* feats, int T, const int* requests,
                        const int* t_ready, int nreq, float* out) {
  return orc_ivector_extract_w(m, feats, T, requests, t_ready, nreq, NULL, NULL, NULL, out);
}

/* ---- resampling (Kaldi LinearResample, feat/resample.cc) ---------------- */
static long gcd_l(long a, long b) { while (b) { long t = a % b; a = b; b = t; } return a; }

static float resample_filter(double cutoff, int num_zeros, float t) {
  float window, filter;
  if (fabs(t) < num_zeros / (2.0 * cutoff))
    window = (float)(0.5 * (1 + cos(2.0 * M_PI * cutoff / num_zeros * t)));
  else
    window = 0.0f;
  if (t != 0.0f)
    filter = (float)(sin(2.0 * M_PI * cutoff * t) / (M_PI * t));
  else
    filter = (float)(2.0 * cutoff);
  return filter * window;
}

long orc_resample_num_outputs(int rate_in, int rate_out, long n) {
  /* GetNumOutputSamples with flush */
  const long g = gcd_l(rate_in, rate_out);
  const long tick = (long)rate_in / g * rate_out;
  long interval = n * (tick / rate_in);
  if (interval <= 0) return 0;
  const long tpo = tick / rate_out;
  long last = interval / tpo;
  if (last * tpo == interval) last--;
  return last + 1;
}

long orc_resample(int rate_in, int rate_out, const float* x, long n, float* out, long cap) {
  const int num_zeros = 6;
  const double cutoff = 0.5 * (rate_in < rate_out ? rate_in : rate_out);
  const long g = gcd_l(rate_in, rate_out);
  const int in_unit = (int)(rate_in / g), out_unit = (int)(rate_out / g);
  const double ww = num_zeros / (2.0 * cutoff);
  const long nout = orc_resample_num_outputs(rate_in, rate_out, n);
  if (nout > cap) return -1;
  for (long k = 0; k < nout; k++) {
    const long unit = k / out_unit;
    const int ph = (int)(k - unit * out_unit);
    const double output_t = ph / (double)rate_out;
    const int lo = (int)ceil((output_t - ww) * rate_in), hi = (int)floor((output_t + ww) * rate_in);
    const long first = lo + unit * in_unit;
    float acc = 0.0f;
    for (int j = 0; j <= hi - lo; j++) {
      const long idx = first + j;
      if (idx < 0 || idx >= n) continue;
      const double delta_t = (lo + j) / (double)rate_in - output_t;
      const float w = resample_filter(cutoff, num_zeros, (float)delta_t) / (float)rate_in;
      acc = fmaf(w, x[idx], acc);
    }
    out[k] = acc;
  }
  return nout;
}

int orc_kslices(int K) {  /* nnet_plan.h GemmKSlices: K / 256 down to a power of two, at most 8 */
  if (K < 512 || K % 256) return 1;
  int n = 1;
  while (n < 8 && 2 * n <= K / 256) n *= 2;
  return n;
}

float orc_logf(float x) {
  static const float C[11] = {1.000000000e+00f, -5.000000000e-01f, 3.333330154e-01f,
                              -2.500002384e-01f, 2.000257671e-01f, -1.666804254e-01f,
                              1.421260685e-01f,  -1.239922047e-01f, 1.192392558e-01f,
                              -1.172722951e-01f, 6.740232557e-02f};
  union { float f; uint32_t u; } v;
  v.f = x;
  int e = (int)((v.u >> 23) & 0xff) - 127;
  v.u = (v.u & 0x7fffffu) | 0x3f800000u;
  float m = v.f;
  if (m > 1.41421356f) { m = m * 0.5f; e += 1; }
  float f = m - 1.0f;
  float p = C[10];
  for (int i = 9; i >= 0; i--) p = fmaf(p, f, C[i]);
  return fmaf((float)e, 0.693147182f, f * p);
}

static float mel_scale(float f) { return 1127.0f * logf(1.0f + f / 700.0f); }

int orc_feat_dim(const orc_mfcc_opts* o) {
  return o->fbank ? o->num_bins + (o->use_energy ? 1 : 0) : o->num_ceps;
}

int orc_mfcc(const orc_mfcc_opts* o, const float* wave, long n, float* out) {
  const int L = frame_length(o), S = frame_shift(o), N = padded_length(o);
  const int nf = orc_mfcc_num_frames(o, n);
  const int nb = o->num_bins, nc = o->num_ceps;
  if (N & (N - 1)) return -1; /* only power-of-two FFT sizes */
  float* win = (float*)malloc(sizeof(float) * L);
  double a = 2.0 * M_PI / (L - 1);
  for (int i = 0; i < L; i++) {
    double c = cos(a * i), w;
    switch (o->window_type) {
      case 0: w = pow(0.5 - 0.5 * c, 0.85); break;
      case 1: w = 0.54 - 0.46 * c; break;
      case 2: w = 0.5 - 0.5 * c; break;
      case 3: w = 1.0; break;
      default: w = o->blackman_coeff - 0.5 * c + (0.5 - o->blackman_coeff) * cos(2 * a * i); break;
    }
    win[i] = (float)w;
  }
  /* mel banks: float arithmetic as MelBanks::MelBanks */
  const int nfft = N / 2;
  float* melw = (float*)calloc((size_t)nb * nfft, sizeof(float));
  int* first = (int*)malloc(sizeof(int) * nb);
  int* last = (int*)malloc(sizeof(int) * nb);
  {
    float nyq = 0.5f * o->samp_freq;
    float hi = o->high_freq > 0.0f ? o->high_freq : nyq + o->high_freq;
    float width = o->samp_freq / (float)N;
    float ml = mel_scale(o->low_freq), mh = mel_scale(hi);
    float delta = (mh - ml) / (float)(nb + 1);
    for (int b = 0; b < nb; b++) {
      float left = ml + (float)b * delta, center = ml + (float)(b + 1) * delta,
            right = ml + (float)(b + 2) * delta;
      first[b] = -1;
      last[b] = -1;
      for (int i = 0; i < nfft; i++) {
        float mel = mel_scale(width * (float)i);
        if (mel > left && mel < right) {
          float w = mel <= center ? (mel - left) / (center - left) : (right - mel) / (right - center);
          melw[(size_t)b * nfft + i] = w;
          if (first[b] < 0) first[b] = i;
          last[b] = i;
        }
      }
    }
  }
  float* dct = (float*)malloc(sizeof(float) * nc * nb);
  {
    float norm0 = (float)sqrt(1.0 / (double)nb);
    float norm = (float)sqrt(2.0 / (double)nb);
    for (int j = 0; j < nb; j++) dct[j] = norm0;
    for (int k = 1; k < nc; k++)
      for (int j = 0; j < nb; j++)
        dct[k * nb + j] = (float)((double)norm * cos(M_PI / nb * (j + 0.5) * k));
  }
  float* lift = (float*)malloc(sizeof(float) * nc);
  for (int i = 0; i < nc; i++) {
    double q = o->cepstral_lifter;
    lift[i] = q != 0.0 ? (float)(1.0 + 0.5 * q * sin(M_PI * i / q)) : 1.0f;
  }
  float* twr = (float*)malloc(sizeof(float) * (N / 2));
  float* twi = (float*)malloc(sizeof(float) * (N / 2));
  for (int k = 0; k < N / 2; k++) {
    twr[k] = (float)cos(2.0 * M_PI * k / N);
    twi[k] = (float)(-sin(2.0 * M_PI * k / N));
  }
  int logn = 0;
  while ((1 << logn) < N) logn++;
  float* re = (float*)malloc(sizeof(float) * N);
  float* im = (float*)malloc(sizeof(float) * N);
  float* x = (float*)malloc(sizeof(float) * L);
  float* mel = (float*)malloc(sizeof(float) * nb);

  for (int f = 0; f < nf; f++) {
    const long s0 = (long)f * S + (o->snip_edges ? 0 : S / 2 - L / 2);
    for (int i = 0; i < L; i++) {
      long k = s0 + i;
      if (k < 0) k = -k - 1; /* ExtractWindow reflection */
      if (k >= n) k = 2 * n - 1 - k;
      x[i] = wave[k];
    }
    if (o->remove_dc_offset) {
      float sum = 0.0f;
      for (int i = 0; i < L; i++) sum = sum + x[i];
      float c = -sum / (float)L;
      for (int i = 0; i < L; i++) x[i] = x[i] + c;
    }
    float log_energy = 0.0f;
    if (o->use_energy) {
      float e = 0.0f;
      for (int i = 0; i < L; i++) e = fmaf(x[i], x[i], e);
      log_energy = orc_logf(e > 1.1920929e-07f ? e : 1.1920929e-07f);
    }
    if (o->preemph_coeff != 0.0f) {
      for (int i = L - 1; i > 0; i--) x[i] = x[i] - o->preemph_coeff * x[i - 1];
      x[0] = x[0] - o->preemph_coeff * x[0];
    }
    for (int i = 0; i < L; i++) x[i] = x[i] * win[i];
    /* radix-2 DIT complex FFT of the zero-padded frame */
    for (int i = 0; i < N; i++) {
      int r = 0;
      for (int b = 0; b < logn; b++) r |= ((i >> b) & 1) << (logn - 1 - b);
      re[r] = i < L ? x[i] : 0.0f;
      im[r] = 0.0f;
    }
    for (int len = 2; len <= N; len <<= 1) {
      int half = len >> 1, step = N / len;
      for (int i = 0; i < N; i += len)
        for (int j = 0; j < half; j++) {
          float wr = twr[j * step], wi = twi[j * step];
          float br = re[i + j + half], bi = im[i + j + half];
          float tr = br * wr - bi * wi;
          float ti = br * wi + bi * wr;
          float ur = re[i + j], ui = im[i + j];
          re[i + j] = ur + tr;
          im[i + j] = ui + ti;
          re[i + j + half] = ur - tr;
          im[i + j + half] = ui - ti;
        }
    }
    /* power spectrum bins 0..N/2-1, mel energies, floor, log */
    for (int b = 0; b < nb; b++) {
      float e = 0.0f;
      if (first[b] >= 0)
        for (int i = first[b]; i <= last[b]; i++) {
          float p = re[i] * re[i] + im[i] * im[i];
          if (o->fbank && !o->use_power) p = sqrtf(p);
          e = fmaf(melw[(size_t)b * nfft + i], p, e);
        }
      if (o->fbank && !o->use_log_fbank) {
        mel[b] = e;
        continue;
      }
      if (e < 1.1920929e-07f) e = 1.1920929e-07f;
      mel[b] = orc_logf(e);
    }
    if (o->fbank) {  /* FbankComputer::Compute: [log energy,] log mel energies */
      const int off = o->use_energy ? 1 : 0;
      float* o_row = out + (size_t)f * (nb + off);
      for (int b = 0; b < nb; b++) o_row[off + b] = mel[b];
      if (o->use_energy) o_row[0] = log_energy;
      continue;
    }
    float* o_row = out + (size_t)f * nc;
    for (int k = 0; k < nc; k++) {
      float c = 0.0f;
      for (int j = 0; j < nb; j++) c = fmaf(dct[k * nb + j], mel[j], c);
      o_row[k] = c * lift[k];
    }
    if (o->use_energy) o_row[0] = log_energy;
  }
  free(win); free(melw); free(first); free(last); free(dct); free(lift);
  free(twr); free(twi); free(re); free(im); free(x); free(mel);
  return nf;
}

/* ===================================================================== */
/* nnet3 forward (Kaldi nnet3/nnet-simple-component.cc, nnet-descriptor) */
/* Whole-utterance evaluation with the input replicated at both edges    */
/* (DecodableNnetSimpleLooped pads with the first/last frame [K]).        */
/* Reference call site: src/model.cc:233-246, src/recognizer.cc:39-43.    */
/* ===================================================================== */
#define ORC_MARGIN 256

typedef struct { int lo, hi; float* v; } node_vals;

static float node_at(const orc_net* net, node_vals* nv, int node, int t, int col) {
  node_vals* n = &nv[node];
  if (node == 0) { /* input: replicate the first / last frame */
    if (t < 0) t = 0;
    if (t > n->hi) t = n->hi;
    return n->v[(size_t)t * net->dim[node] + col];
  }
  return n->v[(size_t)(t - n->lo) * net->dim[node] + col];
}

/* evaluate node `i`'s descriptor at time t into x[in_dim] */
static void eval_desc(const orc_net* net, node_vals* nv, int i, int t, float* x) {
  const int* p = net->prog + net->prog_begin[i];
  int nparts = *p++;
  int col = 0;
  for (int q = 0; q < nparts; q++) {
    int pdim = *p++;
    int ninstr = *p++;
    const int* code = p;
    p += 4 * ninstr;
    for (int d = 0; d < pdim; d++) {
      float stack[16];
      int sp = 0;
      for (int k = 0; k < ninstr; k++) {
        int op = code[4 * k], node = code[4 * k + 1], off = code[4 * k + 2], fi = code[4 * k + 3];
        if (op == 0) stack[sp++] = node_at(net, nv, node, t + off, fi + d);
        else if (op == 4) {
          int k = t - net->ivec_t0;
          if (k < 0) k = 0;
          if (k >= net->ivec_ntimes) k = net->ivec_ntimes - 1;
          stack[sp++] = net->ivec[(size_t)net->ivec_of_time[k] * net->ivec_dim + fi + d];
        }
        else if (op == 1) stack[sp - 1] = net->progf[fi] * stack[sp - 1];
        else if (op == 2) { stack[sp - 2] = stack[sp - 2] + stack[sp - 1]; sp--; }
        else stack[sp++] = net->progf[fi];
      }
      x[col + d] = stack[0];
    }
    col += pdim;
  }
}

/* time range over which node i is computable given its inputs' ranges */
static void node_range(const orc_net* net, node_vals* nv, int i, int* lo, int* hi) {
  const int* p = net->prog + net->prog_begin[i];
  int nparts = *p++;
  int L = -1000000000, H = 1000000000;
  int tb = net->toff_begin[i], tc = net->toff_count[i];
  for (int q = 0; q < nparts; q++) {
    p++;
    int ninstr = *p++;
    for (int k = 0; k < ninstr; k++) {
      if (p[4 * k] == 0) {
        int node = p[4 * k + 1], off = p[4 * k + 2];
        if (node == 0) continue; /* the input is edge-replicated: unbounded */
        for (int z = 0; z < (tc ? tc : 1); z++) {
          int to = tc ? net->toffs[tb + z] : 0;
          if (nv[node].lo - off - to > L) L = nv[node].lo - off - to;
          if (nv[node].hi - off - to < H) H = nv[node].hi - off - to;
        }
      }
    }
    p += 4 * ninstr;
  }
  *lo = L;
  *hi = H;
}

/* mark the times each node must be computed at (backward from the outputs) */
static void mark_needed(const orc_net* net, node_vals* nv, unsigned char** need, int i) {
  const int* p = net->prog + net->prog_begin[i];
  int nparts = *p++;
  int tb = net->toff_begin[i], tc = net->toff_count[i];
  for (int q = 0; q < nparts; q++) {
    p++;
    int ninstr = *p++;
    for (int k = 0; k < ninstr; k++) {
      if (p[4 * k] != 0) continue;
      int node = p[4 * k + 1], off = p[4 * k + 2];
      if (node == 0) continue;
      for (int t = nv[i].lo; t <= nv[i].hi; t++) {
        if (!need[i][t - nv[i].lo]) continue;
        for (int z = 0; z < (tc ? tc : 1); z++) {
          int tt = t + off + (tc ? net->toffs[tb + z] : 0);
          need[node][tt - nv[node].lo] = 1;
        }
      }
    }
    p += 4 * ninstr;
  }
}

#define ORC_TB 16
int orc_nnet_forward(const orc_net* net, const float* feats, int T, float* out) {
  const int NN = net->num_nodes;
  node_vals* nv = (node_vals*)calloc(NN, sizeof(node_vals));
  unsigned char** need = (unsigned char**)calloc(NN, sizeof(unsigned char*));
  nv[0].lo = 0;
  nv[0].hi = T - 1; /* clamp bounds for the replicated input */
  nv[0].v = (float*)feats;
  int maxk = 0, maxd = 0;
  for (int i = 1; i < NN; i++) {
    int lo, hi;
    node_range(net, nv, i, &lo, &hi);
    if (lo < -ORC_MARGIN) lo = -ORC_MARGIN;
    if (hi > T - 1 + ORC_MARGIN) hi = T - 1 + ORC_MARGIN;
    if (hi < lo) return -1;
    nv[i].lo = lo;
    nv[i].hi = hi;
    need[i] = (unsigned char*)calloc(hi - lo + 1, 1);
    int k = net->in_dim[i] * (net->toff_count[i] ? net->toff_count[i] : 1);
    if (k > maxk) maxk = k;
    if (net->dim[i] > maxd) maxd = net->dim[i];
  }
  const int on = net->output_node, OD = net->dim[on];
  const int rows = (T + net->fss - 1) / net->fss;
  for (int j = 0; j < rows; j++) {
    int t = j * net->fss;
    if (t < nv[on].lo || t > nv[on].hi) return -2;
    need[on][t - nv[on].lo] = 1;
  }
  for (int i = NN - 1; i >= 1; i--) mark_needed(net, nv, need, i);

  float* xb = (float*)malloc(sizeof(float) * (size_t)ORC_TB * (maxk + 1));
  float* acc = (float*)malloc(sizeof(float) * (size_t)ORC_TB * (maxd + 1));
  float* part = (float*)malloc(sizeof(float) * (size_t)ORC_TB * (maxd + 1));
  int tlist[ORC_TB];
  for (int i = 1; i < NN; i++) {
    const int D = net->dim[i], ID = net->in_dim[i];
    const int tc = net->toff_count[i], tb = net->toff_begin[i];
    const int K = ID * (tc ? tc : 1);
    nv[i].v = (float*)malloc(sizeof(float) * (size_t)(nv[i].hi - nv[i].lo + 1) * D);
    float* WT = NULL; /* transposed weights [K][D] so the n-loop vectorises */
    if (net->kind[i] == 1) {
      const float* W = net->params + net->w_off[i];
      WT = (float*)malloc(sizeof(float) * (size_t)K * D);
      for (int n = 0; n < D; n++)
        for (int k = 0; k < K; k++) WT[(size_t)k * D + n] = W[(size_t)n * K + k];
    }
    int t = nv[i].lo;
    while (t <= nv[i].hi) {
      int nb = 0;
      while (t <= nv[i].hi && nb < ORC_TB) {
        if (need[i][t - nv[i].lo]) tlist[nb++] = t;
        t++;
      }
      for (int b = 0; b < nb; b++) {
        float* x = xb + (size_t)b * K;
        if (tc) for (int z = 0; z < tc; z++) eval_desc(net, nv, i, tlist[b] + net->toffs[tb + z], x + z * ID);
        else eval_desc(net, nv, i, tlist[b], x);
      }
      for (int b = 0; b < nb; b++) {
        const float* x = xb + (size_t)b * K;
        float* y = nv[i].v + (size_t)(tlist[b] - nv[i].lo) * D;
        switch (net->kind[i]) {
          case 1: { /* affine: y = (sum over k-slices of fmaf chains from 0) + b */
            float* a = acc + (size_t)b * D;
            float* p = part + (size_t)b * D;
            const int ns = orc_kslices(K), kw = K / ns;
            for (int z = 0; z < ns; z++) {
              for (int n = 0; n < D; n++) p[n] = 0.0f;
              const int ke = (z + 1) * kw;
              for (int kg = z * kw; kg < ke; kg += 8) {
                for (int i = 0; i < 8 && kg + i < ke; i++) {
                  /* 0,4,1,5,2,6,3,7 in a full group; a (GPU-unsupported)
                     partial tail group is walked in order */
                  const int k = kg + 8 <= ke ? kg + ((i & 1) << 2) + (i >> 1) : kg + i;
                  const float xk = x[k];
                  const float* w = WT + (size_t)k * D;
                  for (int n = 0; n < D; n++) p[n] = fmaf(xk, w[n], p[n]);
                }
              }
              if (z == 0) memcpy(a, p, sizeof(float) * D);
              else for (int n = 0; n < D; n++) a[n] = a[n] + p[n];
            }
            const float* B = net->b_off[i] >= 0 ? net->params + net->b_off[i] : NULL;
            if (B) for (int n = 0; n < D; n++) y[n] = a[n] + B[n];
            else memcpy(y, a, sizeof(float) * D);
            break;
          }
          case 2: /* RectifiedLinear: ApplyFloor(0) */
            for (int n = 0; n < D; n++) y[n] = x[n] < 0.0f ? 0.0f : x[n];
            break;
          case 3: { /* BatchNorm test mode / ScaleAndOffset: x*s + o */
            const float* s = net->params + net->s_off[i];
            const float* o = net->params + net->o_off[i];
            for (int n = 0; n < D; n++) y[n] = x[n] * s[n] + o[n];
            break;
          }
          default:
            memcpy(y, x, sizeof(float) * D);
        }
      }
    }
    free(WT);
  }
  for (int j = 0; j < rows; j++) {
    int t = j * net->fss;
    const float* v = nv[on].v + (size_t)(t - nv[on].lo) * OD;
    for (int n = 0; n < OD; n++) out[(size_t)j * OD + n] = v[n] * net->acoustic_scale;
  }
  for (int i = 1; i < NN; i++) { free(nv[i].v); free(need[i]); }
  free(nv); free(need); free(xb); free(acc); free(part);
  return rows;
}

/* ===================================================================== */
/* Token passing (Kaldi decoder/lattice-faster-decoder.cc:               */
/* InitDecoding, GetCutoff, ProcessEmitting, ProcessNonemitting,         */
/* FinalizeDecoding/GetBestPath).  Reference call sites:                 */
/* src/recognizer.cc:39-43 (decoder), :318 (endpoint), :790 (best path); */
/* options src/model.cc:135-137.                                         */
/* Order-independent formulation (documented in DESIGN.md): a token is    */
/* created iff its cost beats the frame's FINAL emitting cutoff, and a    */
/* token's backpointer is the min of (cost, arc index).                   */
/* ===================================================================== */
static inline uint32_t ford(float f) {
  union { float f; uint32_t u; } v;
  v.f = f;
  return (v.u & 0x80000000u) ? ~v.u : (v.u | 0x80000000u);
}
static inline float funord(uint32_t k) {
  union { float f; uint32_t u; } v;
  v.u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return v.f;
}
#define EMPTY_KEY 0xffffffffffffffffull

typedef struct { int prev, arc; } orc_link;

typedef struct {
  uint64_t* key;     /* per state: packed (ord(cost) << 32 | arc) for the frame being built */
  int* prevtok;      /* per state: arena index of the winner's source token */
  int* pos;          /* per state: position in the new token list */
  int* inq;          /* per state: queued flag for the epsilon closure */
  int* toks; int ntoks, cap;        /* new-frame states */
  orc_link* arena; int narena, acap;
} dstate;

static void push_tok(dstate* d, int s) {
  if (d->ntoks == d->cap) { d->cap *= 2; d->toks = (int*)realloc(d->toks, sizeof(int) * d->cap); }
  d->pos[s] = d->ntoks;
  d->toks[d->ntoks++] = s;
}

/* relax dest with (tot, arc) from source token index `src_idx`; returns 1 if improved */
static int relax(dstate* d, int dest, float tot, int arc, int src_idx) {
  uint64_t k = ((uint64_t)ford(tot) << 32) | (uint32_t)arc;
  uint64_t old = d->key[dest];
  if (old == EMPTY_KEY) push_tok(d, dest);
  if (k < old) {
    d->key[dest] = k;
    d->prevtok[dest] = src_idx;
    return 1;
  }
  return 0;
}

static int cmp_float(const void* a, const void* b) {
  float x = *(const float*)a, y = *(const float*)b;
  return x < y ? -1 : x > y ? 1 : 0;
}

static float kth_smallest(const float* c, int n, int k, float* tmp) {
  memcpy(tmp, c, sizeof(float) * n);
  qsort(tmp, n, sizeof(float), cmp_float);
  return tmp[k];
}

/* epsilon closure over the tokens in d->toks (frame under construction) */
static void eps_closure(const orc_graph* g, dstate* d, int base, float cutoff) {
  int* queue = (int*)malloc(sizeof(int) * (g->num_states + 1));
  int qh = 0, qt = 0;
  for (int i = 0; i < d->ntoks; i++) { queue[qt++] = d->toks[i]; d->inq[d->toks[i]] = 1; }
  while (qh != qt) {
    int s = queue[qh];
    qh = (qh + 1) % (g->num_states + 1);
    d->inq[s] = 0;
    float c = funord((uint32_t)(d->key[s] >> 32));
    if (c > cutoff) continue;
    int src_idx = base + d->pos[s];
    for (int64_t a = g->eps_begin[s]; a < g->arc_begin[s + 1]; a++) {
      float tot = c + g->weight[a];
      if (tot < cutoff) {
        int dest = g->nextstate[a];
        if (relax(d, dest, tot, (int)a, src_idx) && !d->inq[dest]) {
          d->inq[dest] = 1;
          queue[qt] = dest;
          qt = (qt + 1) % (g->num_states + 1);
        }
      }
    }
  }
  free(queue);
}

/* move the frame under construction into the arena; returns its base index */
static void commit_frame(dstate* d, int base, int* cur_state, float* cur_cost, int* cur_idx) {
  for (int i = 0; i < d->ntoks; i++) {
    int s = d->toks[i];
    if (d->narena == d->acap) { d->acap *= 2; d->arena = (orc_link*)realloc(d->arena, sizeof(orc_link) * d->acap); }
    d->arena[base + i].prev = d->prevtok[s];
    d->arena[base + i].arc = (int)(uint32_t)(d->key[s] & 0xffffffffu);
    d->narena++;
    cur_state[i] = s;
    cur_cost[i] = funord((uint32_t)(d->key[s] >> 32));
    cur_idx[i] = base + i;
  }
  for (int i = 0; i < d->ntoks; i++) d->key[d->toks[i]] = EMPTY_KEY;
}

static void lat_link(orc_dec_result* r, int k, int src, int arc, float ac) {
  if (!r->lat_frame_begin) return;
  if (r->lat_nlink < r->lat_link_cap) {
    r->lat_link_frame[r->lat_nlink] = k;
    r->lat_link_src[r->lat_nlink] = src;
    r->lat_link_arc[r->lat_nlink] = arc;
    r->lat_link_ac[r->lat_nlink] = ac;
  }
  r->lat_nlink++;
}

/* the committed frame k: its tokens, then its epsilon links (Kaldi keeps,
   per token, the epsilon links of its final cost: tokens are re-expanded
   when improved, ProcessNonemitting) */
static void lat_frame(const orc_graph* g, orc_dec_result* r, int k, const int* st, const float* co,
                      int n, float cutoff, float cost_offset) {
  if (!r->lat_frame_begin) return;
  r->lat_frame_begin[k] = r->lat_ntok;
  r->lat_cost_offset[k] = cost_offset;
  for (int i = 0; i < n; i++) {
    if (r->lat_ntok < r->lat_tok_cap) {
      r->lat_tok_state[r->lat_ntok] = st[i];
      r->lat_tok_cost[r->lat_ntok] = co[i];
    }
    r->lat_ntok++;
  }
  r->lat_frame_begin[k + 1] = r->lat_ntok;
  for (int i = 0; i < n; i++)
    for (int64_t a = g->eps_begin[st[i]]; a < g->arc_begin[st[i] + 1]; a++)
      if (co[i] + g->weight[a] < cutoff) lat_link(r, k, st[i], (int)a, 0.0f);
}

/* best path of the current frame (order-independent form): the lowest cost
   (with final costs if any token is final and use_final), ties to the lowest
   state; arcs in forward order into path[0 .. min(*len, cap)) */
static int od_best_path(const orc_graph* g, const int* cur_state, const float* cur_cost, const int* cur_idx,
                        int ncur, const orc_link* arena, int use_final, int* path, long long cap, int* len,
                        float* frc, float* end_tot, int* end_state) {
  int end = -1;
  float end_cost = INFINITY, best_nofinal = INFINITY, best_final = INFINITY;
  for (int i = 0; i < ncur; i++) {
    float c = cur_cost[i];
    if (c < best_nofinal) best_nofinal = c;
    float fc = g->final_cost[cur_state[i]];
    if (fc != INFINITY) {
      float cf = c + fc;
      if (cf < best_final) best_final = cf;
    }
  }
  int any_final = best_final != INFINITY;
  for (int i = 0; i < ncur; i++) {
    float c = (use_final && any_final) ? cur_cost[i] + g->final_cost[cur_state[i]] : cur_cost[i];
    if (c < end_cost || (c == end_cost && end >= 0 && cur_state[i] < cur_state[end])) {
      end_cost = c;
      end = i;
    }
  }
  *frc = any_final ? best_final - best_nofinal : INFINITY;
  *len = 0;
  if (end >= 0) {
    *end_state = cur_state[end];
    *end_tot = end_cost;
    int n = 0;
    for (int k = cur_idx[end]; k >= 0 && arena[k].arc >= 0; k = arena[k].prev) n++;
    *len = n;
    int k = cur_idx[end];
    for (int j = n - 1; j >= 0; j--) {
      if (j < cap) path[j] = arena[k].arc;
      k = arena[k].prev;
    }
  }
  return end;
}

static void od_probe(const orc_graph* g, const int* cs, const float* cc, const int* ci, int ncur,
                     const orc_link* arena, orc_dec_result* r, int i) {
  const long long off = r->probe_off[i];
  int len = 0, es = 0;
  float tot = 0.0f;
  const long long room = r->probe_path_cap - off > 0 ? r->probe_path_cap - off : 0;
  od_best_path(g, cs, cc, ci, ncur, arena, 0, r->probe_path + off, room, &len, &r->probe_frc[i], &tot, &es);
  r->probe_off[i + 1] = off + len;
}

int orc_decode(const orc_graph* g, const float* llh, int F, int stride, const orc_dec_opts* o,
               int use_final, orc_dec_result* r) {
  const int S = g->num_states;
  dstate d;
  d.key = (uint64_t*)malloc(sizeof(uint64_t) * S);
  for (int s = 0; s < S; s++) d.key[s] = EMPTY_KEY;
  d.prevtok = (int*)malloc(sizeof(int) * S);
  d.pos = (int*)malloc(sizeof(int) * S);
  d.inq = (int*)calloc(S, sizeof(int));
  d.cap = 1024;
  d.toks = (int*)malloc(sizeof(int) * d.cap);
  d.acap = 1 << 16;
  d.arena = (orc_link*)malloc(sizeof(orc_link) * d.acap);
  d.narena = 0;
  int* cur_state = (int*)malloc(sizeof(int) * S);
  float* cur_cost = (float*)malloc(sizeof(float) * S);
  int* cur_idx = (int*)malloc(sizeof(int) * S);
  float* tmp = (float*)malloc(sizeof(float) * S);
  double offsets_sum = 0.0;

  /* InitDecoding: start token (cost 0, no predecessor), closure with cutoff = beam */
  d.ntoks = 0;
  relax(&d, g->start, 0.0f, -1, -1);
  d.key[g->start] = ((uint64_t)ford(0.0f) << 32) | 0xffffffffu;
  eps_closure(g, &d, 0, o->beam);
  int ncur = d.ntoks;
  commit_frame(&d, 0, cur_state, cur_cost, cur_idx);
  if (r->lat_frame_begin) { r->lat_ntok = 0; r->lat_nlink = 0; }
  lat_frame(g, r, 0, cur_state, cur_cost, ncur, o->beam, 0.0f);
  if (r->ntok) r->ntok[0] = ncur;
  if (r->best) {
    float b = INFINITY;
    for (int i = 0; i < ncur; i++) if (cur_cost[i] < b) b = cur_cost[i];
    r->best[0] = b;
  }
  int pi = 0;
  if (r->nprobe > 0) r->probe_off[0] = 0;
  for (; pi < r->nprobe && r->probe_frames[pi] <= 0; pi++) od_probe(g, cur_state, cur_cost, cur_idx, ncur, d.arena, r, pi);

  for (int f = 0; f < F; f++) {
    const float* L = llh + (size_t)f * stride;
    /* ---- GetCutoff */
    float best = INFINITY;
    int best_i = -1;
    for (int i = 0; i < ncur; i++)
      if (cur_cost[i] < best || (cur_cost[i] == best && cur_state[i] < cur_state[best_i])) {
        best = cur_cost[i];
        best_i = i;
      }
    if (best_i < 0) break; /* no surviving tokens */
    float beam_cutoff = best + o->beam, adaptive, cutoff;
    float max_cut = INFINITY, min_cut = INFINITY;
    if (ncur > o->max_active) max_cut = kth_smallest(cur_cost, ncur, o->max_active, tmp);
    if (max_cut < beam_cutoff) {
      adaptive = max_cut - best + o->beam_delta;
      cutoff = max_cut;
    } else {
      if (ncur > o->min_active) {
        if (o->min_active == 0) min_cut = best;
        else min_cut = kth_smallest(cur_cost, ncur, o->min_active, tmp);
      }
      if (min_cut > beam_cutoff) {
        adaptive = min_cut - best + o->beam_delta;
        cutoff = min_cut;
      } else {
        adaptive = o->beam;
        cutoff = beam_cutoff;
      }
    }
    /* ---- ProcessEmitting */
    float cost_offset = -best;
    float next_cutoff = INFINITY;
    {
      int s = cur_state[best_i];
      for (int64_t a = g->arc_begin[s]; a < g->eps_begin[s]; a++) {
        float nw = ((g->weight[a] + cost_offset) - L[g->tid2pdf[g->ilabel[a]]]) + best;
        if (nw + adaptive < next_cutoff) next_cutoff = nw + adaptive;
      }
    }
    float m = INFINITY;
    int64_t examined = 0;
    for (int i = 0; i < ncur; i++) {
      if (!(cur_cost[i] <= cutoff)) continue;
      int s = cur_state[i];
      for (int64_t a = g->arc_begin[s]; a < g->eps_begin[s]; a++) {
        float ac = cost_offset - L[g->tid2pdf[g->ilabel[a]]];
        float tot = (cur_cost[i] + ac) + g->weight[a];
        if (tot < m) m = tot;
        examined++;
      }
    }
    if (m + adaptive < next_cutoff) next_cutoff = m + adaptive;
    d.ntoks = 0;
    for (int i = 0; i < ncur; i++) {
      if (!(cur_cost[i] <= cutoff)) continue;
      int s = cur_state[i];
      for (int64_t a = g->arc_begin[s]; a < g->eps_begin[s]; a++) {
        float ac = cost_offset - L[g->tid2pdf[g->ilabel[a]]];
        float tot = (cur_cost[i] + ac) + g->weight[a];
        if (tot < next_cutoff) {
          relax(&d, g->nextstate[a], tot, (int)a, cur_idx[i]);
          lat_link(r, f + 1, s, (int)a, ac);
        }
      }
    }
    int base = d.narena;
    /* ---- ProcessNonemitting */
    eps_closure(g, &d, base, next_cutoff);
    ncur = d.ntoks;
    commit_frame(&d, base, cur_state, cur_cost, cur_idx);
    lat_frame(g, r, f + 1, cur_state, cur_cost, ncur, next_cutoff, cost_offset);
    offsets_sum += cost_offset;
    if (r->ntok) r->ntok[f + 1] = ncur;
    if (r->cutoff) r->cutoff[f] = cutoff;
    if (r->next_cutoff) r->next_cutoff[f] = next_cutoff;
    if (r->arcs_emit) r->arcs_emit[f] = examined;
    if (r->best) {
      float b = INFINITY;
      for (int i = 0; i < ncur; i++) if (cur_cost[i] < b) b = cur_cost[i];
      r->best[f + 1] = b;
    }
    for (; pi < r->nprobe && r->probe_frames[pi] <= f + 1; pi++)
      od_probe(g, cur_state, cur_cost, cur_idx, ncur, d.arena, r, pi);
    if (ncur == 0) break;
  }

  for (; pi < r->nprobe; pi++) {  /* probes past the decoded frames: nothing */
    r->probe_off[pi + 1] = r->probe_off[pi];
    r->probe_frc[pi] = INFINITY;
  }
  /* ---- best path end: with final costs if any token is final */
  const int end = od_best_path(g, cur_state, cur_cost, cur_idx, ncur, d.arena, use_final, r->path, r->path_cap,
                               &r->path_len, &r->final_relative_cost, &r->best_tot, &r->end_state);
  if (end >= 0) r->best_cost = (double)r->best_tot - offsets_sum;
  free(d.key); free(d.prevtok); free(d.pos); free(d.inq); free(d.toks); free(d.arena);
  free(cur_state); free(cur_cost); free(cur_idx); free(tmp);
  return end >= 0 ? 0 : -1;
}

/* ===================================================================== */
/* Kaldi-sequential token passing: the decoder as Kaldi runs it           */
/* (decoder/lattice-faster-decoder.cc [K], LatticeFasterDecoderTpl, whose  */
/* search the LatticeIncrementalDecoder of the reference shares,          */
/* src/recognizer.cc:39-43), which the GPU decoder reproduces by default  */
/* (DESIGN.md §4).  TEST INFRASTRUCTURE.  Operation for operation:         */
/*  - toks_ is a HashList<StateId, Token*> (util/hash-list-inl.h): list    */
/*    order by bucket (state % hash_size) in order of the bucket's first   */
/*    occupancy, then insertion order within a bucket; hash_size is 1000   */
/*    for a new decoder (kept across InitDecoding: opts.hash_size in,      */
/*    result.hash_size out) and grows to tok_cnt * hash_ratio (2) at each  */
/*    ProcessEmitting (PossiblyResizeHash)                                 */
/*  - GetCutoff: the first minimum in list order is best_elem; nth_element */
/*    for max_active / min_active                                          */
/*  - ProcessEmitting: seed next_cutoff from best_elem's arcs, then every  */
/*    token in list order with cost <= cutoff, its emitting arcs in graph  */
/*    order: skip tot >= next_cutoff, tighten next_cutoff to tot +         */
/*    adaptive_beam; every accepted relaxation is a forward link and       */
/*    FindOrAddToken keeps the minimum cost                                */
/*  - ProcessNonemitting: queue = list order of tokens with epsilon arcs,  */
/*    LIFO (pop_back), cost >= cutoff skipped, a token's forward links     */
/*    replaced at each expansion, created / cheaper tokens re-queued       */
/* Backpointer of a token (this restatement's 1-best; Kaldi reads the     */
/* best path from the lattice): the (source, arc) of its minimum          */
/* (cost, arc) relaxation, the GPU key minimum's tie rule.                */
/* ===================================================================== */
typedef struct {
  int* where;       /* per state: element index in the frame being built, -1 */
  int* st; float* cost; int* bp; int* arc; int* bucket; int n, cap;
  int* bucket_rank; /* per bucket: first-occupancy rank in this frame, -1 */
  int nranks;
  size_t hash_size, bucket_cap;
  const int* ids;   /* bucketing id per state (lazy numbering), NULL: the state */
} khash;

static void kh_reserve(khash* h, int n) {
  if (n <= h->cap) return;
  while (h->cap < n) h->cap *= 2;
  h->st = (int*)realloc(h->st, sizeof(int) * h->cap);
  h->cost = (float*)realloc(h->cost, sizeof(float) * h->cap);
  h->bp = (int*)realloc(h->bp, sizeof(int) * h->cap);
  h->arc = (int*)realloc(h->arc, sizeof(int) * h->cap);
  h->bucket = (int*)realloc(h->bucket, sizeof(int) * h->cap);
}

static void kh_set_size(khash* h, size_t size) {  /* HashList::SetSize (list empty) */
  h->hash_size = size;
  if (size > h->bucket_cap) {
    h->bucket_rank = (int*)realloc(h->bucket_rank, sizeof(int) * size);
    for (size_t b = h->bucket_cap; b < size; b++) h->bucket_rank[b] = -1;
    h->bucket_cap = size;
  }
}

static void kh_clear(khash* h) {
  for (int i = 0; i < h->n; i++) { h->where[h->st[i]] = -1; h->bucket_rank[h->bucket[i]] = -1; }
  h->n = 0;
  h->nranks = 0;
}

/* FindOrAddToken: *changed = created or a strictly lower cost (Kaldi's
   test); the backpointer follows the minimum (cost, arc) */
static int kh_find_or_add(khash* h, int s, float tot, int bp, int arc, int* changed) {
  int e = h->where[s];
  if (e < 0) {
    kh_reserve(h, h->n + 1);
    e = h->n++;
    h->where[s] = e;
    h->st[e] = s; h->cost[e] = tot; h->bp[e] = bp; h->arc[e] = arc;
    int b = (int)((size_t)(h->ids ? h->ids[s] : s) % h->hash_size);
    h->bucket[e] = b;
    if (h->bucket_rank[b] < 0) h->bucket_rank[b] = h->nranks++;
    *changed = 1;
    return e;
  }
  *changed = 0;
  if (tot < h->cost[e]) {
    h->cost[e] = tot; h->bp[e] = bp; h->arc[e] = arc; *changed = 1;
  } else if (tot == h->cost[e] && (unsigned)arc < (unsigned)h->arc[e]) {
    h->bp[e] = bp; h->arc[e] = arc;
  }
  return e;
}

/* list order: elements by their bucket's first-occupancy rank, then insertion */
static void kh_order(const khash* h, int* order, int* cnt) {
  for (int r = 0; r <= h->nranks; r++) cnt[r] = 0;
  for (int i = 0; i < h->n; i++) cnt[h->bucket_rank[h->bucket[i]] + 1]++;
  for (int r = 0; r < h->nranks; r++) cnt[r + 1] += cnt[r];
  for (int i = 0; i < h->n; i++) order[cnt[h->bucket_rank[h->bucket[i]]]++] = i;
}

/* work counters of orc_decode_kaldi (diagnostics: how much of a frame is
   the sequential epsilon queue): frames, emitting items examined, emitting
   relaxations accepted, tokens created by the emitting pass, epsilon-queue
   pops, pops skipped (cost >= cutoff), epsilon relaxations below the cutoff,
   tokens created by the epsilon pass, re-queued improvements */
static long long g_kstats[9];
void orc_kaldi_stats(long long* out, int reset) {
  for (int i = 0; i < 9; i++) { out[i] = g_kstats[i]; if (reset) g_kstats[i] = 0; }
}

typedef struct {
  khash h;
  /* OpenFST lazy numbering (orc_dec_opts.lazy_next): id per state, -1 none */
  int* disc; char* expanded; int next_id;
  const int64_t* lazy_row; const int* lazy_next;
  int* order; int* cnt; int ocap, ccap;
  int* queue; int qcap;
  int* elem_pos;     /* element -> list position (frame being committed) */
  int* a_prev; int* a_arc; int narena, acap;  /* committed tokens: backpointer, arc */
  int* cur_state; float* cur_cost; int* cur_idx; int ncur, cur_cap;
} kdec;

static void kd_list_order(kdec* d) {
  khash* h = &d->h;
  if (h->n + 1 > d->ocap) { d->ocap = 2 * (h->n + 1); d->order = (int*)realloc(d->order, sizeof(int) * d->ocap); }
  if (h->nranks + 2 > d->ccap) { d->ccap = 2 * (h->nranks + 2); d->cnt = (int*)realloc(d->cnt, sizeof(int) * d->ccap); }
  kh_order(h, d->order, d->cnt);
}

/* the composed FST expands state s (its arcs computed): destinations
   without an id are numbered in arc order (OpenFST's lazy numbering) */
static void kd_expand(kdec* d, int s) {
  if (!d->disc || d->expanded[s]) return;
  d->expanded[s] = 1;
  for (int64_t a = d->lazy_row[s]; a < d->lazy_row[s + 1]; a++) {
    const int t = d->lazy_next[a];
    if (d->disc[t] < 0) d->disc[t] = d->next_id++;
  }
}

/* ProcessNonemitting over the frame being built */
static void kd_nonemitting(const orc_graph* g, kdec* d, float cutoff) {
  khash* h = &d->h;
  kd_list_order(d);
  int qn = 0;
  for (int q = 0; q < h->n; q++) {
    const int s = h->st[d->order[q]];
    kd_expand(d, s);  /* fst_->NumInputEpsilons(state) */
    if (g->eps_begin[s] < g->arc_begin[s + 1]) {
      if (qn + 1 > d->qcap) { d->qcap = 2 * (qn + 1); d->queue = (int*)realloc(d->queue, sizeof(int) * d->qcap); }
      d->queue[qn++] = s;
    }
  }
  while (qn > 0) {
    const int s = d->queue[--qn];
    const int e = h->where[s];
    const float cc = h->cost[e];
    g_kstats[4]++;
    if (cc >= cutoff) { g_kstats[5]++; continue; }
    const int src = -2 - e;  /* element e of this frame (resolved at commit) */
    for (int64_t a = g->eps_begin[s]; a < g->arc_begin[s + 1]; a++) {
      const float tot = cc + g->weight[a];
      if (tot < cutoff) {
        int ch;
        const int dst = g->nextstate[a];
        const int nb = h->n;
        kh_find_or_add(h, dst, tot, src, (int)a, &ch);
        g_kstats[6]++;
        if (h->n > nb) g_kstats[7]++;
        else if (ch) g_kstats[8]++;
        if (ch) kd_expand(d, dst);  /* (changed && fst_->NumInputEpsilons(nextstate)) */
        if (ch && g->eps_begin[dst] < g->arc_begin[dst + 1]) {
          if (qn + 1 > d->qcap) { d->qcap = 2 * (qn + 1); d->queue = (int*)realloc(d->queue, sizeof(int) * d->qcap); }
          d->queue[qn++] = dst;
        }
      }
    }
  }
}

/* commit the frame being built (list order becomes the current token order);
   its tokens and epsilon links go to the lattice output as frame k */
static void kd_commit(const orc_graph* g, kdec* d, orc_dec_result* r, int k, float cutoff, float cost_offset) {
  khash* h = &d->h;
  const int n = h->n;
  kd_list_order(d);
  d->elem_pos = (int*)realloc(d->elem_pos, sizeof(int) * (n + 1));
  for (int q = 0; q < n; q++) d->elem_pos[d->order[q]] = q;
  if (n > d->cur_cap) {
    d->cur_cap = 2 * n;
    d->cur_state = (int*)realloc(d->cur_state, sizeof(int) * d->cur_cap);
    d->cur_cost = (float*)realloc(d->cur_cost, sizeof(float) * d->cur_cap);
    d->cur_idx = (int*)realloc(d->cur_idx, sizeof(int) * d->cur_cap);
  }
  const int base = d->narena;
  if (d->narena + n > d->acap) {
    while (d->narena + n > d->acap) d->acap *= 2;
    d->a_prev = (int*)realloc(d->a_prev, sizeof(int) * d->acap);
    d->a_arc = (int*)realloc(d->a_arc, sizeof(int) * d->acap);
  }
  for (int q = 0; q < n; q++) {
    const int e = d->order[q];
    int bp = h->bp[e];
    if (bp <= -2) bp = base + d->elem_pos[-2 - bp];  /* epsilon source in this frame */
    d->a_prev[base + q] = bp;
    d->a_arc[base + q] = h->arc[e];
    d->cur_state[q] = h->st[e];
    d->cur_cost[q] = h->cost[e];
    d->cur_idx[q] = base + q;
  }
  d->narena += n;
  d->ncur = n;
  kh_clear(h);
  if (!r->lat_frame_begin) return;
  r->lat_frame_begin[k] = r->lat_ntok;
  r->lat_cost_offset[k] = cost_offset;
  for (int i = 0; i < n; i++) {
    if (r->lat_ntok < r->lat_tok_cap) {
      r->lat_tok_state[r->lat_ntok] = d->cur_state[i];
      r->lat_tok_cost[r->lat_ntok] = d->cur_cost[i];
    }
    r->lat_ntok++;
  }
  r->lat_frame_begin[k + 1] = r->lat_ntok;
  /* a token's epsilon links are those of its last expansion: its final cost,
     when below the cutoff (ProcessNonemitting never expands the others) */
  for (int i = 0; i < n; i++) {
    const float c = d->cur_cost[i];
    if (c >= cutoff) continue;
    const int s = d->cur_state[i];
    for (int64_t a = g->eps_begin[s]; a < g->arc_begin[s + 1]; a++)
      if (c + g->weight[a] < cutoff) lat_link(r, k, s, (int)a, 0.0f);
  }
}

/* best path of the current frame: its end with final costs if any token is
   final (and use_final), else the lowest cost (the first minimum in list
   order); the arcs in forward order into path[0 .. min(*len, cap)).  Returns
   the end token's index in the current list, -1 if there is none. */
static int kd_best_path(const orc_graph* g, const kdec* d, int use_final, int* path, long long cap, int* len,
                        float* frc, float* end_tot, int* end_state) {
  const int ncur = d->ncur;
  int end = -1;
  float end_cost = INFINITY, best_nofinal = INFINITY, best_final = INFINITY;
  for (int i = 0; i < ncur; i++) {
    const float c = d->cur_cost[i];
    if (c < best_nofinal) best_nofinal = c;
    const float fc = g->final_cost[d->cur_state[i]];
    if (fc != INFINITY && c + fc < best_final) best_final = c + fc;
  }
  const int any_final = best_final != INFINITY;
  for (int i = 0; i < ncur; i++) {
    const float c = (use_final && any_final) ? d->cur_cost[i] + g->final_cost[d->cur_state[i]] : d->cur_cost[i];
    if (c < end_cost) { end_cost = c; end = i; }
  }
  *frc = any_final ? best_final - best_nofinal : INFINITY;
  *len = 0;
  if (end >= 0) {
    *end_state = d->cur_state[end];
    *end_tot = end_cost;
    int n = 0;
    for (int k = d->cur_idx[end]; k >= 0 && d->a_arc[k] >= 0; k = d->a_prev[k]) n++;
    *len = n;
    int k = d->cur_idx[end];
    for (int j = n - 1; j >= 0; j--) {
      if (j < cap) path[j] = d->a_arc[k];
      k = d->a_prev[k];
    }
  }
  return end;
}

/* endpoint probe i after the current frame: the no-final best path appended */
static void kd_probe(const orc_graph* g, const kdec* d, orc_dec_result* r, int i) {
  const long long off = r->probe_off[i];
  int len = 0, es = 0;
  float tot = 0.0f;
  const long long room = r->probe_path_cap - off > 0 ? r->probe_path_cap - off : 0;
  kd_best_path(g, d, 0, r->probe_path + off, room, &len, &r->probe_frc[i], &tot, &es);
  r->probe_off[i + 1] = off + len;
}

int orc_decode_kaldi(const orc_graph* g, const float* llh, int F, int stride, const orc_dec_opts* o,
                     int use_final, orc_dec_result* r) {
  const int S = g->num_states;
  kdec d;
  memset(&d, 0, sizeof(d));
  khash* h = &d.h;
  h->where = (int*)malloc(sizeof(int) * S);
  for (int s = 0; s < S; s++) h->where[s] = -1;
  h->cap = 1024;
  h->st = (int*)malloc(sizeof(int) * h->cap); h->cost = (float*)malloc(sizeof(float) * h->cap);
  h->bp = (int*)malloc(sizeof(int) * h->cap); h->arc = (int*)malloc(sizeof(int) * h->cap);
  h->bucket = (int*)malloc(sizeof(int) * h->cap);
  const int own_lazy = o->lazy_next && !o->lazy_disc;
  if (o->lazy_next) {
    const int64_t nids_max = S + (o->lazy_row[S] > 0 ? o->lazy_row[S] : 0);  /* (dead ids < S + arcs) */
    if (own_lazy) {
      d.disc = (int*)malloc(sizeof(int) * nids_max);
      d.expanded = (char*)malloc(S);
    } else {
      d.disc = o->lazy_disc;
      d.expanded = o->lazy_expanded;
    }
    d.lazy_row = o->lazy_row;
    d.lazy_next = o->lazy_next;
    if (own_lazy || *o->lazy_count <= 0) {
      for (int64_t s = 0; s < nids_max; s++) d.disc[s] = -1;
      memset(d.expanded, 0, S);
      d.disc[g->start] = 0;  /* ComposeFst::Start() */
      d.next_id = 1;
    } else {
      d.next_id = *o->lazy_count;
    }
    h->ids = d.disc;
  }
  /* a new decoder's toks_.SetSize(1000), or the size the decoder had (InitDecoding keeps it) */
  kh_set_size(h, o->hash_size > 0 ? (size_t)o->hash_size : 1000);
  d.acap = 1 << 16;
  d.a_prev = (int*)malloc(sizeof(int) * d.acap);
  d.a_arc = (int*)malloc(sizeof(int) * d.acap);
  float* tmp = NULL;
  int tcap = 0;
  double offsets_sum = 0.0;
  const float hash_ratio = 2.0f;
  if (r->lat_frame_begin) { r->lat_ntok = 0; r->lat_nlink = 0; }
  int pi = 0;
  if (r->nprobe > 0) r->probe_off[0] = 0;

  /* InitDecoding: start token, ProcessNonemitting(beam) */
  {
    int ch;
    kh_find_or_add(h, g->start, 0.0f, -1, -1, &ch);
    kd_nonemitting(g, &d, o->beam);
    kd_commit(g, &d, r, 0, o->beam, 0.0f);
  }
  for (; pi < r->nprobe && r->probe_frames[pi] <= 0; pi++) kd_probe(g, &d, r, pi);
  if (r->ntok) r->ntok[0] = d.ncur;
  if (r->best) { float b = INFINITY; for (int i = 0; i < d.ncur; i++) if (d.cur_cost[i] < b) b = d.cur_cost[i]; r->best[0] = b; }

  for (int f = 0; f < F; f++) {
    const float* L = llh + (size_t)f * stride;
    const int ncur = d.ncur;
    if (ncur == 0) break;
    const float* cur_cost = d.cur_cost;
    const int* cur_state = d.cur_state;
    /* ---- GetCutoff: best_elem = first minimum in list order */
    float best = INFINITY;
    int best_i = -1;
    for (int i = 0; i < ncur; i++) if (cur_cost[i] < best) { best = cur_cost[i]; best_i = i; }
    float beam_cutoff = best + o->beam, adaptive, cutoff;
    float max_cut = INFINITY, min_cut = INFINITY;
    if (ncur + 1 > tcap) { tcap = 2 * (ncur + 1); tmp = (float*)realloc(tmp, sizeof(float) * tcap); }
    memcpy(tmp, cur_cost, sizeof(float) * ncur);
    int sorted = 0;
    if (ncur > o->max_active) { qsort(tmp, ncur, sizeof(float), cmp_float); sorted = 1; max_cut = tmp[o->max_active]; }
    if (max_cut < beam_cutoff) {
      adaptive = max_cut - best + o->beam_delta;
      cutoff = max_cut;
    } else {
      if (ncur > o->min_active) {
        if (o->min_active == 0) min_cut = best;
        else {
          if (!sorted) qsort(tmp, ncur, sizeof(float), cmp_float);
          min_cut = tmp[o->min_active];
        }
      }
      if (min_cut > beam_cutoff) { adaptive = min_cut - best + o->beam_delta; cutoff = min_cut; }
      else { adaptive = o->beam; cutoff = beam_cutoff; }
    }
    /* PossiblyResizeHash(tok_cnt) on the emptied hash */
    {
      size_t nsz = (size_t)((float)ncur * hash_ratio);
      if (nsz > h->hash_size) kh_set_size(h, nsz);
    }
    /* ---- ProcessEmitting */
    float next_cutoff = INFINITY;
    const float cost_offset = -best;
    {
      const int s = cur_state[best_i];
      kd_expand(&d, s);  /* ArcIterator (expanded when created: a no-op) */
      for (int64_t a = g->arc_begin[s]; a < g->eps_begin[s]; a++) {
        const float nw = ((g->weight[a] + cost_offset) - L[g->tid2pdf[g->ilabel[a]]]) + best;
        if (nw + adaptive < next_cutoff) next_cutoff = nw + adaptive;
      }
    }
    int64_t examined = 0;
    for (int i = 0; i < ncur; i++) {
      if (!(cur_cost[i] <= cutoff)) continue;
      const int s = cur_state[i];
      for (int64_t a = g->arc_begin[s]; a < g->eps_begin[s]; a++) {
        const float ac = cost_offset - L[g->tid2pdf[g->ilabel[a]]];
        const float tot = (cur_cost[i] + ac) + g->weight[a];
        examined++;
        if (tot >= next_cutoff) continue;
        if (tot + adaptive < next_cutoff) next_cutoff = tot + adaptive;
        int ch;
        const int nb = h->n;
        kh_find_or_add(h, g->nextstate[a], tot, d.cur_idx[i], (int)a, &ch);
        g_kstats[2]++;
        if (h->n > nb) g_kstats[3]++;
        lat_link(r, f + 1, s, (int)a, ac);
      }
    }
    /* ---- ProcessNonemitting(next_cutoff) */
    kd_nonemitting(g, &d, next_cutoff);
    kd_commit(g, &d, r, f + 1, next_cutoff, cost_offset);
    offsets_sum += cost_offset;
    g_kstats[0]++;
    g_kstats[1] += examined;
    if (r->ntok) r->ntok[f + 1] = d.ncur;
    if (r->cutoff) r->cutoff[f] = cutoff;
    if (r->next_cutoff) r->next_cutoff[f] = next_cutoff;
    if (r->arcs_emit) r->arcs_emit[f] = examined;
    if (r->best) { float b = INFINITY; for (int i = 0; i < d.ncur; i++) if (d.cur_cost[i] < b) b = d.cur_cost[i]; r->best[f + 1] = b; }
    for (; pi < r->nprobe && r->probe_frames[pi] <= f + 1; pi++) kd_probe(g, &d, r, pi);
  }
  for (; pi < r->nprobe; pi++) {  /* probes past the decoded frames: nothing */
    r->probe_off[pi + 1] = r->probe_off[pi];
    r->probe_frc[pi] = INFINITY;
  }
  r->hash_size = (int)h->hash_size;
  const int end = kd_best_path(g, &d, use_final, r->path, r->path_cap, &r->path_len, &r->final_relative_cost,
                               &r->best_tot, &r->end_state);
  if (end >= 0) r->best_cost = (double)r->best_tot - offsets_sum;
  free(h->where); free(h->st); free(h->cost); free(h->bp); free(h->arc); free(h->bucket); free(h->bucket_rank);
  free(d.a_prev); free(d.a_arc); free(d.cur_state); free(d.cur_cost); free(d.cur_idx); free(d.order);
  free(d.cnt); free(d.queue); free(d.elem_pos); free(tmp);
  if (own_lazy) { free(d.disc); free(d.expanded); }
  else if (o->lazy_next) *o->lazy_count = d.next_id;
  return end >= 0 ? 0 : -1;
}

/* ===================================================================== */
/* Speaker x-vectors (src/recognizer.cc:356-419, Kaldi                    */
/* feat/feature-functions.cc SlidingWindowCmnInternal,                    */
/* nnet3/nnet-general-component.cc Statistics{Extraction,Pooling}).       */
/* ===================================================================== */
void orc_sliding_cmn(const float* feats, int T, int D, int window, float* out) {
  for (int d = 0; d < D; d++) {
    double sum = 0.0;
    int last_start = -1, last_end = -1;
    for (int t = 0; t < T; t++) {
      int ws = t - window / 2, we = ws + window;
      if (ws < 0) { we -= ws; ws = 0; }
      if (we > T) { ws -= we - T; we = T; if (ws < 0) ws = 0; }
      if (last_start < 0) {
        for (int u = ws; u < we; u++) sum = sum + (double)feats[(size_t)u * D + d];
      } else {
        if (ws > last_start) sum = sum - (double)feats[(size_t)last_start * D + d];
        if (we > last_end) sum = sum + (double)feats[(size_t)last_end * D + d];
      }
      last_start = ws;
      last_end = we;
      const double alpha = -1.0 / (double)(we - ws);
      out[(size_t)t * D + d] = (float)((double)feats[(size_t)t * D + d] + alpha * sum);
    }
  }
}

int orc_xvector_tail(const orc_xvec* x, const float* rows, int ld, int r0, int r1, float* out) {
  const int D = x->stats_dim, n = r1 - r0 + 1;
  if (n <= 0) return -1;
  int maxd = x->nlog + 2 * D;
  for (int i = 0; i < x->nops; i++) if (x->out_dim[i] > maxd) maxd = x->out_dim[i];
  float* a = (float*)calloc((size_t)maxd, sizeof(float));
  float* b = (float*)calloc((size_t)maxd, sizeof(float));
  for (int k = 0; k < x->nlog; k++) a[k] = (float)log((double)n);
  for (int d = 0; d < D; d++) {
    double s = 0.0, s2 = 0.0;
    for (int t = 0; t < n; t++) {
      const double v = (double)rows[(size_t)(r0 + t) * ld + d];
      s = s + v;
      s2 = s2 + v * v;
    }
    const double mean = s / (double)n;
    a[x->nlog + d] = (float)mean;
    if (x->stddevs) {
      double var = s2 / (double)n - mean * mean;
      if (var < (double)x->var_floor) var = (double)x->var_floor;
      a[x->nlog + D + d] = (float)sqrt(var);
    }
  }
  for (int i = 0; i < x->nops; i++) {
    const int K = x->in_dim[i], N = x->out_dim[i];
    const float* W = x->params + x->w_off[i];
    const float* B = x->b_off[i] >= 0 ? x->params + x->b_off[i] : NULL;
    for (int o = 0; o < N; o++) {
      if (x->kind[i] == 1) {
        const float v = canon_dot(W + (size_t)o * K, a, K);
        b[o] = B ? v + B[o] : v;
      } else if (x->kind[i] == 2) {
        b[o] = a[o] < 0.0f ? 0.0f : a[o];
      } else {
        b[o] = a[o] * W[o] + B[o];
      }
    }
    float* t = a; a = b; b = t;
  }
  const int E = x->embed_dim, R = x->out_dim_final;
  float* xc = (float*)malloc(sizeof(float) * E);
  for (int e = 0; e < E; e++) xc[e] = a[e] - x->mean[e];
  for (int r = 0; r < R; r++) out[r] = canon_dot(x->transform + (size_t)r * E, xc, E);
  float ss = 0.0f;
  for (int r = 0; r < R; r++) ss = ss + out[r] * out[r];
  const float norm = sqrtf(ss);
  const float ratio = (float)((double)norm / sqrt((double)R));
  const float scale = (float)(1.0 / (double)ratio);
  for (int r = 0; r < R; r++) out[r] = out[r] * scale;
  free(a); free(b); free(xc);
  return 0;
}
