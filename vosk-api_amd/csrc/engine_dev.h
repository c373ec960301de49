// Plain-old-data structures shared by the host engine and the HIP kernels.
#pragma once

#include <cstdint>

namespace vamd {

constexpr int kMaxSegs = 16;
constexpr int kMaxStages = 8;
constexpr int kMaxParts = 8;
constexpr int kMaxInstr = 48;

// One chunk job of one stream slot: the op rows of this job are at times
// base_t + pattern[k]; reads of the feature input are clamped to
// [0, clamp_max] (Kaldi replicates the first / last frame).
struct DevJob {
  int slot, base_t, clamp_max, pad;
};

// Ring references carry the resolved ring base pointer and row length so the
// kernels never chase a pointer table before a data load.
struct DevSeg { const float* base; int ldim, is_input, offset, col0, dim, src_col; };
struct DevStage { const float* base; const float* v0; const float* v1; int kind, ldim, is_input,
                  offset, src_col, scaled; float c; };
struct DevInstr { const float* base; int op, ldim, is_input, offset, src_col; float c; };
struct DevPart { int col0, dim, instr0, ninstr; };

struct RingSet {
  float* const* base;  // per stored node: [ring][slots][dim] (time-major: the rows
                       // of one frame for all streams are adjacent in HBM)
  const int* dim;      // per stored node
  int mask;            // ring - 1 (power of two)
  int ring;
  int slots;
  int input_node;
};

struct NnetOpArgs {
  int M, N, K, P;          // rows, cols, reduction, pattern length (rows per job)
  const int* pattern;      // [P]
  const float* W;          // [N][K] (GEMM only)
  const DevJob* jobs;
  RingSet rings;
  const float* const* vecs;
  int out_node;            // -1: write log-likelihood rows
  float* out_base;         // ring of out_node
  int out_ldim;
  float* llh;              // [M][N] when out_node < 0
  int nsegs, nstages, nparts;
  int kslices;             // K split into equal slices reduced in fixed order (GemmKSlices)
  DevSeg segs[kMaxSegs];
  DevStage stages[kMaxStages];
  DevPart parts[kMaxParts];
  DevInstr instr[kMaxInstr];
};

// ---- MFCC
struct MfccDev {
  int frame_length, frame_shift, padded, log2n, num_bins, num_ceps, nfft;
  int use_energy, remove_dc;
  float preemph;
  const float* window;   // [frame_length]
  const float* melw;     // [num_bins][nfft] dense
  const int* mel_first;  // [num_bins]
  const int* mel_last;   // [num_bins]
  const float* dct;      // [num_ceps][num_bins]
  const float* lifter;   // [num_ceps]
  const float* twr;      // [padded/2]
  const float* twi;      // [padded/2]
  int fbank, use_log_fbank, use_power, feat_dim;
  int first_offset;      // frame t starts at t*frame_shift + first_offset (snip-edges=false:
                         // shift/2 - length/2; samples before 0 are reflected)
  float* out;            // feature ring [ring][slots][feat_dim]
};

// online CMVN (Kaldi OnlineCmvn, global stats, mean only): running window
// sums per stream, sequential in time; in/out rings [ring][slots][D]
struct CmvnDev {
  int D, window, global_frames, pad;
  const double* gstats;  // [2][D + 1]
  double* sums;          // [slots][D] window sums (persistent)
  float* hist;           // [slots][kCmvnHist][D] raw frames (the window's tail)
  const float* in_base;
  float* out_base;
  int mask, slots;
};
struct CmvnJob {  // normalize frames [from, to) of a stream
  int slot, from, to, reset;
};
constexpr int kCmvnHist = 1024, kCmvnMaxD = 128;

struct MfccJob {  // frames [first, first+count) of one slot; rows [row0, row0+count)
  int slot, first, count, row0;
};

// one utterance of an x-vector batch (xvector.h): its selected frame indices
// rows[rows0, rows0 + nsel), its pooled frame-level output rows
// [pool_row0, pool_row0 + npool)
struct XvecUtt {
  int rows0, nsel, pool_row0, npool;
};

// windowed-sinc resampling (resample.h): output sample k of a stream is the
// tap-ordered fma chain over raw[first[k % out_unit] + (k / out_unit) * in_unit + j]
struct ResampleDev {
  const int* first;   // [out_unit]
  const int* ntaps;   // [out_unit]
  const float* w;     // [out_unit][taps]
  int in_unit, out_unit, taps, pad;
};
struct ResampleJob {  // outputs [out_first, out_first + count) into the sample ring
  int slot, pos, count, table;
  long long out_first, raw_total;  // raw samples available (later ones read as 0)
};

struct CopyItem {  // gather copy: nwords 32-bit words from src to dst + dst_off
  const unsigned* src;
  long long dst_off, nwords;
};

struct SampleJob {  // append count samples from src[] to ring position pos
  int slot, pos, count, pad;
  const float* src;  // staging buffer (host-fed) or the stream's HBM-resident audio
};

// ---- decoder
struct DecSlot {
  int ntok;         // tokens of the current frame
  int cur_base;     // arena index of the current frame's first token
  int arena_used;
  int frames;       // frames decoded since the last reset
  int stamp;        // epsilon-closure round stamp (monotonic; HBM table stamps)
  int err;          // bit 0: token list / table overflow, bit 1: arena overflow, bit 2: no tokens,
                    // bit 3: unplaceable backpointer source, bit 4: pruning lost a backpointer,
                    // bit 5: a link record with a backpointer candidate did not fit (deferred winners)
  int lat_ovf;      // lattice overflow (results fall back to 1-best): bit 0 link arena, bit 1 an
                    // epsilon link's destination missing, bit 2 frame-record table
  int prune_from;   // first LatFrame whose extra costs were never computed (PruneActiveTokens)
  double offset_sum;
  unsigned long long best_key;  // min over current tokens of (ordered cost << 32 | state)
  long long links_used;         // lattice links in the stream's link arena
  int last_prune;   // frames decoded at the last pruning pass
  float commit_cutoff;  // cutoff of the last commit: every current token's cost is below it
  int khash;        // Kaldi order: the decoder's HashList size (0 = a new decoder's 1000)
  int lazy_count;   // Kaldi order on a composed graph: state ids OpenFST has given so far
};

// ---- lattice (LatticeFasterDecoder forward links, kept in HBM per stream).
// A link {src arena index, dst arena index, arc, acoustic cost bits}: an
// emitting link goes from a token of frame k-1 to one of frame k, an epsilon
// link (arcs[arc] has no pdf) joins two tokens of frame k.  The frame's
// links are exactly Kaldi's: emitting links below the frame's final cutoff,
// epsilon links once per arc at the final source cost (decoder.hip
// commit_links).  Their total cost is recomputed from the source token's
// cost: (cost + ac) + weight (emitting), cost + weight (epsilon).
struct LatFrame {   // per decoded frame (index 0 = InitDecoding's closure)
  int tok_base, ntok;      // arena slots [tok_base, tok_base + ntok) (dead slots: prev == -2)
  long long link_begin, link_end;
  float cutoff;            // tokens and links of this frame are below it
  float cost_offset;       // cost offset of the emitting links INTO this frame
  int new_base, new_ntok;  // pruning scratch (compacted token range)
};

// ---- online i-vector extraction (kernels.hip ivector_kernel)
constexpr int kIvMaxS = 100, kIvMaxD = 64, kIvMaxK = 320, kIvMaxG = 512, kIvMaxQ = 20 * 256;
constexpr int kIvFrameBlock = 8;  // frames per ivector_frame_kernel workgroup
struct IvectorDev {
  int feat_dim, left, right, lda_dim, lda_cols, num_gauss, ivec_dim, cmn_window;
  int global_frames, num_gselect, num_cg_iters, pad;
  float min_post, posterior_scale, log_min_post, pad2;
  double prior_offset, max_count;
  const double* cmvn;          // [2][feat_dim + 1]
  const double* sigma_inv_m;   // [G][lda_dim][S]
  const double* U;             // [G][S(S+1)/2]
};
struct IvState {  // per stream, persistent across steps (reset with the pipeline)
  double nfr;           // posterior-weighted frame count
  double lin[kIvMaxS];  // linear term (incl. prior)
  double cur[kIvMaxS];  // current i-vector (CG warm start)
};
struct IvStreamJob {  // one stream's i-vector work in this step
  int slot, req0, nreq, reset;
  int t_ready;             // MFCC frames available (splice clamp)
  int pad0, pad1, pad2;
};
struct IvReq {  // i-vector at `frame` -> rows [job_lo, job_hi) of the per-job buffer,
                // after accumulating frame records [row_from, row_to) in the
                // statistics batches [batch0, batch0 + nbatch); upd = the
                // statistics advance to `frame` here (else the current i-vector
                // is reused, OnlineIvectorFeature::GetFrame with no new frames)
  int frame, job_lo, job_hi, row_from, row_to, upd, batch0, nbatch;
};
// one UpdateStatsForFrames call: frame records [row_from, row_to) aggregated
// per Gaussian (OnlineIvectorEstimationStats::AccStats over a matrix)
struct IvBatch {
  int row_from, row_to;
};
constexpr int kIvBatchRows = 512;  // frame records per statistics batch (host-checked)
struct IvFrameBlock {  // ivector_top_kernel rows: frames t0.. (nf) of a job's stream;
                       // ring >= 0: also keep the records in the stream's history
                       // ring (silence-weighted streams re-weight past frames)
  int job, t0, nf, row, ring, pad0, pad1, pad2;
};
// silence weighting (src/recognizer.cc:226-237): one (frame, delta weight)
// entry of the stream's Kaldi delta-weight queue, applied in (frame, weight)
// order; rec = the frame's record in the history ring [slot * kIvRing + t % kIvRing]
struct IvEntry {
  int rec;
  float w;
};
constexpr int kIvRing = 1024;  // history ring frames per stream (>= 3 x 100 re-weighted + chunk)
struct IvFrame {  // per-frame result: selected Gaussians and posteriors
  int nsel;
  int sel[5];
  float post[5];
  int xrow;  // row of the frame in the step's LDA / UBM GEMM outputs
};
struct IvArgs {
  IvectorDev m;
  IvState* state;     // [slots]
  double* quad;       // [slots][S(S+1)/2]
  double* qfull;      // [slots][S][S] the same, unpacked for the CG mat-vec (S > 48)
  float* norm;        // [ring][slots][feat_dim] CMVN-normalized features (MFCC ring layout)
  const float* in_base;  // MFCC input ring [ring][slots][feat_dim]
  int in_mask, slots;
  IvFrame* frames;    // [max frames per step]
  float* xraw;        // [GEMM rows + entry rows][lda_dim] LDA projection of the raw features
  double* snap;       // [max requests per step][S(S+1)/2 + S] terms at each request
  double* snap_nfr;   // [max requests per step] frame count at each request

  float* ivec;        // [jobs][S] per chunk job, prior offset removed
  const IvStreamJob* jobs;
  const IvReq* reqs;
  const IvFrameBlock* blocks;
  IvFrame* ring;        // [slots][kIvRing] records, posteriors unscaled (e/tot)
  float* ring_x;        // [slots][kIvRing][lda_dim]
  const IvEntry* ents;  // this step's weighted entries -> rows ent_row0 + i
  int ent_row0, nents;
  const IvBatch* batches;
};

struct DecJob {
  int slot, llh_row0, nframes, reset, stats_row0;  // reset: 1 InitDecoding, 2 a new decoder, 3 a new stream
  int pad0;  // host bookkeeping: 1 = built after the stream's input ended (not read by the kernel)
  int host_read;  // DecArgs::host_gate: the last frame whose records the host has read (-1: none)
  int pad2;
};

struct FrameStat {
  int ntok_in, ntok_out, arcs_emit, arcs_eps;
  float best, cutoff, next_cutoff, adaptive_beam;
};

constexpr int kDecProf = 73;               // decoder phase-clock slots per stream (decoder.hip Prof)
constexpr int kLazyExpanded = 1 << 30;  // lazy_id flag: the state's arcs are numbered
constexpr int kLazyNewCap = 1024;       // lazy_new entries per list (>= decoder threads)
constexpr int kKbMemb = 8;    // Kaldi order: members kept per hash bucket (more: counted by a scan; a multiple of 4)
struct DecArgs {
  long long* prof;       // optional per-slot phase clocks [slots][kDecProf] (diagnostics)
  const int4* sinfo;     // per state {arc_begin, eps_begin, arc_end, final cost bits}
  const int4* arcs;      // per arc {nextstate, weight bits, pdf (-1 eps),
                         //          source state | (nextstate has eps arcs) << 31}
  int num_states, start_state;
  float beam, beam_delta;
  int max_active, min_active;
  int P;
  const float* llh;
  const DecJob* jobs;
  // per stream, one HBM frame table of H = 1 << hbits slots (decoder.hip):
  // states that do not fit the LDS table of the frame under construction
  int* ht_state;            // [slots][H]
  unsigned long long* ht_key;  // [slots][H]
  int* ht_pos;              // [slots][H] creation index | has-epsilon-arcs << 30
  int* ht_stamp;            // [slots][H]
  int* ht_bp;               // [slots][H] backpointer (decoder.hip kBpEps encoding)
  int* ht_list;             // [slots][max_tok]
  int hbits, hprobe;
  int* front_g;             // [slots][2][max_tok] epsilon frontier spill
  int* cur_state;           // [slots][max_tok]
  float* cur_cost;          // [slots][max_tok]
  int* cur_pos;             // [slots][max_tok] list position (arena offset from cur_base)
  int4* arena;              // [slots][arena_cap] {prev, arc, cost bits, state}
  DecSlot* slots;
  FrameStat* stats;
  int max_tok;
  int lds_probe;          // LDS probe limit (states past it live in HBM); tests: 0 = all HBM
  long long arena_cap;
  int4* links;            // [slots][link_cap] lattice links (nullptr: no lattice)
  int* link_dst;          // [slots][link_cap] destination frame-table slot of a raw link
  LatFrame* lat_frames;   // [slots][lat_frame_cap] (always kept: pruning walks the frames)
  long long link_cap;
  int lat_frame_cap;
  float lattice_beam;     // pruning (PruneActiveTokens)
  int prune_interval;     // frames between pruning passes (0 = never)
  int prune_fill_pct;     // and only once the token or link arena is this full (percent; 0: always) ...
  int prune_start;        // ... or the segment is this many frames long
  int prune_revisit;      // frames below the last pruned frame a pass may re-walk
  int host_gate;          // 1: the host reads the records as they come (EngineConfig::host_lattice):
                          // a pass runs at the start of a launch, only when DecJob::host_read
                          // covers every decoded frame (a compaction never moves unread records)
  int debug;              // VOSK_AMD_DEC_DEBUG bits (development): 1 invariant checks with printf,
                          // 2 no Kaldi-order GetCutoff shortcut, 4 Kaldi epsilon queue through HBM records
  float* extra;           // [slots][arena_cap] Kaldi extra_cost per token (pruning)
  int* remap;             // [slots][arena_cap] pruning scratch (old -> new arena index)
  // Kaldi order (decoder.hip): the frame's token list in
  // LatticeFasterDecoder's HashList order (bucket state % khash in order of
  // first occupancy, then creation), the emitting pass's running cutoff as a
  // prefix minimum, the epsilon queue run as Kaldi's LIFO
  int kaldi;              // 1: Kaldi order, 0: the order-independent form
  int* kb_first;          // [slots][kb_cap] per bucket: first creation index (INT_MAX: empty)
  int* kb_cnt;            // [slots][kb_cap] per bucket: tokens
  int* kb_start;          // [slots][kb_cap] per bucket: list position of its first token
  int* kb_memb;           // [slots][kb_cap][4] per bucket: creation indices of its first four tokens
  int kb_cap;             // >= the largest HashList size (2 * max_tok + 1024)
  int* kord;              // [slots][kord_cap] frame under construction: slot code by creation index
  int* kbkt;              // [slots][kord_cap] bucket by creation index
  int* kstk;              // [slots][kord_cap] epsilon queue entries past the LDS part
  float* kcost0;          // [slots][kord_cap] emitting pass cost by creation index
  int* kmem;              // [slots][kord_cap][8] epsilon queue tokens past the LDS part
  int2* kadj;             // [slots][kadj_cap] their epsilon arcs past the LDS part
  int kord_cap;           // >= tokens a frame may create (max_tok + LDS table slots)
  int kadj_cap;
  // OpenFST's lazy ComposeFst numbering (Graph::lazy_*; nullptr: the graph's
  // ids): HashList buckets are lazy_id % khash.  Per stream, kept for the
  // stream's life (a recognizer's ComposeFst, src/recognizer.cc:31-37): a new
  // stream's first job (reset 3) clears it
  const long long* lazy_row;  // [states + 1] arcs of a state in the composition's order
  const int* lazy_next;       // their destinations as ids [0, lazy_ids)
  int* lazy_id;               // [slots][lazy_ids] OpenFST's id (-1: none yet) | kLazyExpanded
  int* lazy_cand;             // [slots][lazy_ids] numbering scratch (INT_MAX between frames)
  int* lazy_new;              // [slots][3][kLazyNewCap] a frame's emitting tokens not yet expanded
  int lazy_ids;
};

struct TraceArgs {
  const int4* sinfo;
  const int4* arena;
  const int* cur_state;
  const float* cur_cost;
  const int* cur_pos;
  const DecSlot* slots;
  const int* req_slot;   // [n] slots to trace
  int use_final;
  int max_tok;
  long long arena_cap;
  int path_cap;
  int* path;             // [n][path_cap] reversed arc indices
  int* path_len;         // [n]
  float* end_cost;       // [n] (with final cost if used)
  float* final_rel;      // [n] final relative cost
  int* end_state;        // [n]
  // endpoint probe (optional): per arc 0 = epsilon, 1 = silence-phone
  // emitting, 2 = other emitting; the walk stops at the first 2 and path_len
  // counts the trailing silence frames (no path is written)
  const unsigned char* arc_sil;
  int tie_pos;           // end-token ties: 1 the first in list order (Kaldi order), 0 the lowest state
};

}  // namespace vamd
