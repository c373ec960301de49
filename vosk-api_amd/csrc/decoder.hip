// Token passing on MI355X (gfx950): Kaldi LatticeFasterDecoder's per-frame
// GetCutoff / ProcessEmitting / ProcessNonemitting over a CSR graph in HBM,
// with Kaldi's forward links kept per stream for lattices, the best-path
// traceback, and the periodic pruning that keeps every stream's arenas
// bounded (PruneActiveTokens).  Reference call sites: src/recognizer.cc:39-43
// (decoder), :318 (endpoint), :790 (best path); src/batch_model.cc:78-80
// (batch options).
//
// Per-stream state is bounded by the token counts, never by the graph size:
// the frame under construction lives in an LDS table (4096 slots, two-choice
// buckets of four); a state whose two buckets are taken by other states
// lives in the stream's HBM hash table instead.  Placement is deterministic
// within a frame -- slots are only ever claimed, never released, while a
// frame is built -- so a relaxation's slot stays valid until the commit, and
// the table a state lands in has no effect on any cost, key or backpointer:
// results are those of the order-independent formulation restated in
// oracle/oracle.c.
//
// Backpointers are resolved while relaxing: a relaxation whose (cost, arc)
// key is still its slot's minimum after the pass's next barrier writes its
// source (the arena index of an emitting source, the frame-table slot of an
// epsilon source) into the slot.  A later pass can only lower the key, and a
// later winner writes after that barrier, so the last write is the final
// winner's.  The commit therefore never reloads an arc or looks a source up.
#include <hip/hip_runtime.h>
#include <type_traits>

#include <cstdint>

#include "dev_util.h"
#include "engine_dev.h"
#include "kernels.h"

namespace vamd {

// Per-stream scratch in global memory (frame tables, token lists, Kaldi-order
// bookkeeping) is private to the stream's workgroup during a launch: its
// plain loads and stores need only workgroup scope (the CU's vector L1 is
// shared by the workgroup's waves and write-through), not the agent scope of
// dev_util.h, which sends every load to L2.  Launch boundaries order it
// across kernels.
#undef AG_LD
#undef AG_ST
#define AG_LD(p) __hip_atomic_load((p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
#define AG_ST(p, v) __hip_atomic_store((p), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
__device__ __forceinline__ int4 wg_ld4(const int4* p) {
  unsigned long long* q = reinterpret_cast<unsigned long long*>(const_cast<int4*>(p));
  const unsigned long long lo = AG_LD(q), hi = AG_LD(q + 1);
  return make_int4((int)(unsigned)lo, (int)(unsigned)(lo >> 32), (int)(unsigned)hi, (int)(unsigned)(hi >> 32));
}
__device__ __forceinline__ void wg_st4(int4* p, int4 v) {
  unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
  AG_ST(q, (unsigned long long)(unsigned)v.x | ((unsigned long long)(unsigned)v.y << 32));
  AG_ST(q + 1, (unsigned long long)(unsigned)v.z | ((unsigned long long)(unsigned)v.w << 32));
}

#ifndef VAMD_DEC_THREADS
#define VAMD_DEC_THREADS 1024
#endif
constexpr int DT = VAMD_DEC_THREADS;  // threads per decoder workgroup
constexpr int DW = DT / 64;           // waves
constexpr int kLlhLds = 4096;         // log-likelihood row staged in LDS up to this size
constexpr int kTokLds = 1024;         // current-frame tokens cached in LDS up to this count
constexpr int kHashCap = 4096;        // LDS frame table slots (power of two)
constexpr int kHashBits = 12;
constexpr int kMaxProbe = 2;          // LDS buckets a state may use (DecArgs::lds_probe: 0 all HBM, 1 one bucket)
constexpr int kFrontLds = 2048;       // epsilon frontier entries in LDS (more spill to HBM)
// emitting-pass backpointers resolved at commit from the frame's link
// records (no per-sub-round winner barrier) while the link arena has at
// least this much room left; otherwise the sub-round winner checks run
constexpr long long kDeferHeadroom = 1 << 20;
#ifndef VAMD_DEC_UNROLL
#define VAMD_DEC_UNROLL (1024 / VAMD_DEC_THREADS)
#endif
constexpr int kUnroll = VAMD_DEC_UNROLL;            // (token, arc) items in flight per thread in the emitting pass
constexpr unsigned long long kEmpty = 0xffffffffffffffffull;
constexpr int kNoSlot = 0x7fffffff;   // no frame-table slot
constexpr unsigned kDestEps = 0x80000000u;  // arcs[].w: nextstate has epsilon arcs
// backpointer of a frame-table slot: an emitting source's arena index (>= 0),
// or kBpEps | the epsilon source's slot (kBpHbm: an HBM-table slot)
constexpr int kBpEps = (int)0x80000000u;
constexpr int kBpHbm = 0x40000000;
constexpr unsigned short kPosEps = 0x8000;  // LDS list position flag: the state has epsilon arcs
constexpr int kHPosEps = 0x40000000;        // the same flag in an HBM table position
// pruning: links / tokens are dropped only beyond lattice_beam + this margin,
// so float rounding never drops what the host's exact (double) lattice-beam
// prune keeps (the pruned lattice is unchanged)
constexpr float kPruneMargin = 0.5f;

struct DecShared {
  int scan[DT + 1];   // exclusive prefix sums of the chunk's degrees
  int abeg[DT];       // first arc per chunk token
  float tcost[DT];    // cost per chunk token
  int tsrc[DT];       // source per chunk token (arena index / epsilon slot code)
  unsigned hist[256];
  unsigned long long red_u[DW];
  float red_f[DW];
  int red_i[DW];
  int n_new_l, n_new_g, n_next, n_front, n_fnext, total, sel_k, n_links, lat_ovf, n_eps;
  unsigned sel_prefix, sel_mask;
  float seed;
  unsigned run_bound;  // emitting pass: running next_cutoff bound (ordered float bits)
  int bad, flag, kk;
  int fl[8];                  // FixRound flags (two sets of three) + change flags
  unsigned char kbits[DT];    // pruning: per-thread keep bits of the chunk
  LatFrame fr;        // pruning: the frame record being processed (broadcast)
  LatFrame fr1;
  // Kaldi order: emitting pass running cutoff (prefix minimum, two sets for
  // alternating sub-rounds), creator-rank scan, epsilon queue bookkeeping
  float kmin_w[2][DW];
  float kcar[2];
  // emitting pass running cutoff by decoupled look-back (kaldi_lookback_min):
  // per (sub-round, wave) index q, {q << 1 | inclusive, ordered min} in a ring
  unsigned long long kls[4 * DW];
  int ksum_w[2][DW];
  int kn0, kne;
  int klazy_ne;  // lazy numbering: the frame's tokens created by the emitting pass
  int klazy_k;   // lazy numbering: the frame's states not yet expanded
  int klazy_def; // lazy numbering: queue tokens whose state has no id yet
  int kpop_sum, kpop_max;  // component replay: pops over all lanes / on the longest lane
  int kcomp_n, kcomp_max;  // component replay: components / pops of the largest (profile)
  int karc_sum, karc_max, khbm_pops;  // wave replay: arcs iterated (all waves / the busiest), pops of HBM members
  int kheads;                         // wave replay: multi-token component heads listed in hist[]
  int kcomp_clk;                      // (profile) clocks of the longest component replay
  int kbig;                           // (profile) this frame's queue members overflow the LDS records
};

// optional phase clocks (VOSK_AMD_DEC_PROFILE): thread 0 stamps s_memtime
// at phase ends; slots as vosk/engine.py Engine.PHASES
// The accumulators live in LDS (a register array of kDecProf 64-bit values
// per thread would spill the whole kernel to scratch and time a different
// program); only thread 0 touches them.
struct Prof {
  bool on;
  long long t;
  long long* acc;  // [kDecProf] in LDS
  __device__ __forceinline__ void init(bool o, long long* lds_acc) {
    on = o;
    acc = lds_acc;
    if (on)
      for (int i = 0; i < kDecProf; i++) acc[i] = 0;
    t = on ? (long long)__builtin_amdgcn_s_memtime() : 0;
  }
  __device__ __forceinline__ void mark(int i) {
    if (on) {
      const long long n = (long long)__builtin_amdgcn_s_memtime();
      acc[i] += n - t;
      t = n;
    }
  }
  __device__ __forceinline__ void count(int i, long long v) {
    if (on) acc[i] += v;
  }
};

// s_waitcnt vmcnt(0): every vector memory operation of this wave, no-return
// atomics included, has completed (gfx9 encoding: expcnt 7, lgkmcnt 15)
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// Wave-wide inclusive scans by DPP: row shifts by 1, 2, 4, 8 within each
// 16-lane row, then CDNA's row broadcasts (lane 15 into the next row, lane 31
// into the upper half).  VALU moves only -- a __shfl is an LDS round trip
// (ds_bpermute) per step.  Lanes without a source keep the identity (`old`).
template <int CTRL, int ROWM>
__device__ __forceinline__ int dpp_mov(int old, int x) {
  return __builtin_amdgcn_update_dpp(old, x, CTRL, ROWM, 0xf, false);
}
__device__ __forceinline__ float wave_incl_min(float v) {
  constexpr int kI = 0x7f800000;  // +inf
  v = fminf(v, __int_as_float(dpp_mov<0x111, 0xf>(kI, __float_as_int(v))));
  v = fminf(v, __int_as_float(dpp_mov<0x112, 0xf>(kI, __float_as_int(v))));
  v = fminf(v, __int_as_float(dpp_mov<0x114, 0xf>(kI, __float_as_int(v))));
  v = fminf(v, __int_as_float(dpp_mov<0x118, 0xf>(kI, __float_as_int(v))));
  v = fminf(v, __int_as_float(dpp_mov<0x142, 0xa>(kI, __float_as_int(v))));
  v = fminf(v, __int_as_float(dpp_mov<0x143, 0xc>(kI, __float_as_int(v))));
  return v;
}
__device__ __forceinline__ int wave_incl_sum(int v) {
  v += dpp_mov<0x111, 0xf>(0, v);
  v += dpp_mov<0x112, 0xf>(0, v);
  v += dpp_mov<0x114, 0xf>(0, v);
  v += dpp_mov<0x118, 0xf>(0, v);
  v += dpp_mov<0x142, 0xa>(0, v);
  v += dpp_mov<0x143, 0xc>(0, v);
  return v;
}
// the value of the lane below (lane 0: fill)
__device__ __forceinline__ float wave_shr1(float v, float fill) {
  return __int_as_float(dpp_mov<0x138, 0xf>(__float_as_int(fill), __float_as_int(v)));
}
__device__ __forceinline__ float wave_min_f(float v) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wave_incl_min(v)), 63));
}
__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long w = __shfl_xor(v, o, 64);
    v = w < v ? w : v;
  }
  return v;
}

__device__ __forceinline__ float block_min_f(DecShared& sh, float v) {
  v = wave_min_f(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh.red_f[w] = v;
  __syncthreads();
  float r = sh.red_f[0];
  for (int i = 1; i < DW; i++) r = fminf(r, sh.red_f[i]);
  return r;
}

__device__ __forceinline__ unsigned long long block_min_u64(DecShared& sh, unsigned long long v) {
  v = wave_min_u64(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh.red_u[w] = v;
  __syncthreads();
  unsigned long long r = sh.red_u[0];
  for (int i = 1; i < DW; i++) r = sh.red_u[i] < r ? sh.red_u[i] : r;
  return r;
}

__device__ __forceinline__ unsigned long long block_sum_u64(DecShared& sh, unsigned long long v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh.red_u[w] = v;
  __syncthreads();
  unsigned long long r = 0;
  for (int i = 0; i < DW; i++) r += sh.red_u[i];
  return r;
}

// exclusive scan of deg over the block; writes sh.scan[0..DT], sh.total
__device__ __forceinline__ void block_scan(DecShared& sh, int deg) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int v = wave_incl_sum(deg);
  __syncthreads();
  if (lane == 63) sh.red_i[w] = v;
  __syncthreads();
  int off = 0;
  for (int i = 0; i < w; i++) off += sh.red_i[i];
  sh.scan[threadIdx.x] = off + v - deg;
  if (threadIdx.x == DT - 1) {
    sh.scan[DT] = off + v;
    sh.total = off + v;
  }
  __syncthreads();
}

// token index j within the chunk that owns item `it` (largest j: scan[j] <= it)
__device__ __forceinline__ int owner(const DecShared& sh, int it) {
  int lo = 0, hi = DT - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (sh.scan[mid] <= it) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// Block-start owners of a chunk's items (sh.hist, free during the emitting
// passes): BO[b] = the token owning item 64 b, written by that token's thread
// after the scan.  An item's owner then lies between its block's and the next
// block's starts -- a search over the few tokens starting inside one block
// instead of over the whole chunk (10 dependent LDS reads).
constexpr int kOwnBlk = 256;
__device__ __forceinline__ void owner_blocks(DecShared& sh) {
  const int s = sh.scan[threadIdx.x], e = sh.scan[threadIdx.x + 1];
  int* BO = reinterpret_cast<int*>(sh.hist);
  for (int b = (s + 63) >> 6; (b << 6) < e && b < kOwnBlk; b++) BO[b] = (int)threadIdx.x;
}
// nbo = the chunk's block count when it is at most kOwnBlk, else 0 (plain search)
__device__ __forceinline__ int owner_bo(const DecShared& sh, int nbo, int it) {
  const int b = it >> 6;
  if (b >= nbo) return owner(sh, it);
  const int* BO = reinterpret_cast<const int*>(sh.hist);
  int lo = BO[b], hi = b + 1 < nbo ? BO[b + 1] : DT - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (sh.scan[mid] <= it) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// current-frame tokens: LDS cache when they fit, else global (agent loads)
struct TokView {
  int* gs;
  float* gc;
  const int* ls;
  const float* lc;
  bool lds;
  __device__ __forceinline__ int s(int i) const { return lds ? ls[i] : AG_LD(&gs[i]); }
  __device__ __forceinline__ float c(int i) const { return lds ? lc[i] : AG_LD(&gc[i]); }
};

// token costs held in registers for GetCutoff when the frame has at most
// DT * kCutRegs tokens (element r of a thread: token threadIdx.x + r * DT);
// loaded once, with all loads in flight together, for the count and every
// radix pass
constexpr int kCutRegs = 4096 / DT;
struct CostRegs {
  float c[kCutRegs];
  __device__ __forceinline__ void load(const TokView& tv, int n, int base = 0) {
#pragma unroll
    for (int r = 0; r < kCutRegs; r++) {
      const int i = base + (int)threadIdx.x + r * DT;
      c[r] = i < n ? tv.c(i) : 0.0f;
    }
  }
};

// exact k-th smallest (0-based) of the token costs by 4-pass 8-bit radix
// select; the costs come from registers (cr) or from the token view
template <bool REGS>
__device__ __forceinline__ float kth_smallest(DecShared& sh, const TokView& tv, const CostRegs& cr, int n,
                                              int k) {
  if (threadIdx.x == 0) {
    sh.sel_prefix = 0;
    sh.sel_mask = 0;
    sh.sel_k = k;
  }
  for (int shift = 24; shift >= 0; shift -= 8) {
    __syncthreads();
    for (int i = threadIdx.x; i < 256; i += DT) sh.hist[i] = 0;
    __syncthreads();
    const unsigned prefix = sh.sel_prefix, mask = sh.sel_mask;
    if (REGS) {
#pragma unroll
      for (int r = 0; r < kCutRegs; r++) {
        const unsigned u = ford(cr.c[r]);
        if ((int)threadIdx.x + r * DT < n && (u & mask) == prefix) atomicAdd(&sh.hist[(u >> shift) & 255u], 1u);
      }
    } else {  // blocks of DT * kCutRegs costs, each block's loads in flight together
      for (int b0 = 0; b0 < n; b0 += DT * kCutRegs) {
        CostRegs blk;
        blk.load(tv, n, b0);
#pragma unroll
        for (int r = 0; r < kCutRegs; r++) {
          const unsigned u = ford(blk.c[r]);
          if (b0 + (int)threadIdx.x + r * DT < n && (u & mask) == prefix)
            atomicAdd(&sh.hist[(u >> shift) & 255u], 1u);
        }
      }
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // wave 0: prefix over the 256 buckets (4 per lane)
      const int l = threadIdx.x;
      const int h0 = sh.hist[4 * l], h1 = sh.hist[4 * l + 1], h2 = sh.hist[4 * l + 2],
                h3 = sh.hist[4 * l + 3];
      const int tot = h0 + h1 + h2 + h3;
      const int incl = wave_incl_sum(tot);
      const int excl = incl - tot;
      const int kk = sh.sel_k;
      if (kk >= excl && kk < incl) {  // exactly one lane holds the bucket
        int r = kk - excl, b = 4 * l;
        if (r >= h0) { r -= h0; b++;
          if (r >= h1) { r -= h1; b++;
            if (r >= h2) { r -= h2; b++; } } }
        sh.sel_k = r;
        sh.sel_prefix = prefix | ((unsigned)b << shift);
        sh.sel_mask = mask | (255u << shift);
      }
    }
  }
  __syncthreads();
  return funord(sh.sel_prefix);
}

// ---------------------------------------------------------------------------
// frame table: LDS slots first, the stream's HBM table for the rest
// ---------------------------------------------------------------------------
struct FrameLds {
  int* hs;                  // [kHashCap] state, -1 = empty
  unsigned long long* hk;   // [kHashCap] (ordered cost << 32 | arc), kEmpty
  int* hb;                  // [kHashCap] backpointer (kBpEps encoding)
  unsigned short* hp;       // [kHashCap] list position | kPosEps
  int* hst;                 // [kHashCap] epsilon round stamp
  unsigned short* nl;       // [kHashCap] list -> slot
  int* fr0;                 // [kFrontLds] epsilon frontiers (slot codes)
  int* fr1;
};

struct HbmTab {
  int* state;               // [H] -1 = empty
  unsigned long long* key;  // [H]
  int* pos;                 // [H] creation index | kHPosEps
  int* stamp;               // [H]
  int* bp;                  // [H]
  int* list;                // [max_tok] slots in creation order
};

// LDS frame table: kHashCap / 4 buckets of four slots; a state lives in the
// first empty slot of its first bucket, else of its second bucket, else in
// the HBM table (two-choice bucketed hashing: at most eight slots looked at)
constexpr int kBucketBits = kHashBits - 2;
__device__ __forceinline__ unsigned bucket1(int s) {
  return ((unsigned)s * 2654435761u) >> (32 - kBucketBits);
}
__device__ __forceinline__ unsigned bucket2(int s, unsigned b1) {
  unsigned x = (unsigned)s * 0x85ebca6bu;
  x ^= x >> 15;
  x *= 0x27d4eb2du;
  x ^= x >> 13;
  const unsigned b = x >> (32 - kBucketBits);
  return b == b1 ? b ^ 1u : b;
}
// independent of lds_hash, so states crowded in LDS spread out in HBM
__device__ __forceinline__ unsigned hbm_hash(int s, int bits) {
  unsigned x = (unsigned)s * 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x >> (32 - bits);
}

struct DecPtrs {
  int* cs;     // current tokens: state
  float* cc;   //                 cost
  int* cp;     //                 list position (arena index = cur_base + cp)
  int4* arena; // {prev, arc, cost bits, state} per token of the segment
  int* fg0;    // HBM frontier spill [max_tok]
  int* fg1;
  int slot;
};

__device__ __forceinline__ HbmTab hbm_tab(const DecArgs& a, int slot) {
  const long long o = (long long)slot << a.hbits;
  HbmTab r;
  r.state = a.ht_state + o;
  r.key = a.ht_key + o;
  r.pos = a.ht_pos + o;
  r.stamp = a.ht_stamp + o;
  r.bp = a.ht_bp + o;
  r.list = a.ht_list + (long long)slot * a.max_tok;
  return r;
}

// result of a relaxation: slot >= 0 LDS slot, < 0 ~(HBM slot);
// flags 2 created, 1 improved, 0 not improved, -1 no room (sh.bad set)
struct Relax {
  int slot, flags;
};

// a new HBM-table entry at slot g: listed, key by atomic min (a concurrent
// relaxation of the same state may already have lowered it)
__device__ __forceinline__ void hbm_created(const DecArgs& a, DecShared& sh, const HbmTab& T, unsigned g,
                                            unsigned long long k, bool eps) {
  const int pos = atomicAdd(&sh.n_new_g, 1);
  if (pos < a.max_tok) {
    AG_ST(&T.list[pos], (int)g);
    AG_ST(&T.pos[g], pos | (eps ? kHPosEps : 0));
  } else {
    sh.bad |= 1;
  }
  __hip_atomic_fetch_min(&T.key[g], k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// LDS part of a relaxation (key k); slot kNoSlot: both buckets are full.
// Without NEED_OLD the key is lowered without waiting for the old value and
// an existing state reports flags 1.
template <bool NEED_OLD>
__device__ __forceinline__ Relax relax_lds(const DecArgs& a, DecShared& sh, const FrameLds& t, int dest,
                                           unsigned long long k, bool eps) {
  const int nbk = a.lds_probe < 2 ? a.lds_probe : 2;
  const unsigned b1 = bucket1(dest);
  for (int nb = 0; nb < nbk; nb++) {
    const int h0 = 4 * (int)(nb ? bucket2(dest, b1) : b1);
    while (true) {  // buckets fill left to right: claim the first empty slot
      int e = -1, f = -1;
#pragma unroll
      for (int i = 3; i >= 0; i--) {
        const int c = __hip_atomic_load(&t.hs[h0 + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (c == dest) f = i;
        if (c == -1) e = i;
      }
      int h = h0 + f;
      if (f < 0) {
        if (e < 0) break;  // full: the second bucket, then HBM
        h = h0 + e;
        const int cur = atomicCAS(&t.hs[h], -1, dest);
        if (cur == -1) {
          const int pos = atomicAdd(&sh.n_new_l, 1);  // < kHashCap: one per claimed slot
          t.nl[pos] = (unsigned short)h;
          t.hp[h] = (unsigned short)(pos | (eps ? kPosEps : 0));
          __hip_atomic_fetch_min(&t.hk[h], k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          return Relax{h, 2};
        }
        if (cur != dest) continue;  // another state took it: look again
      }
      if (NEED_OLD) {
        const unsigned long long old = atomicMin(&t.hk[h], k);
        return Relax{h, k < old ? 1 : 0};
      }
      __hip_atomic_fetch_min(&t.hk[h], k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return Relax{h, 1};
    }
  }
  return Relax{kNoSlot, 0};
}

__device__ __forceinline__ Relax relax(const DecArgs& a, DecShared& sh, const FrameLds& t,
                                       const HbmTab& T, int dest, float tot, int arc, bool eps) {
  const unsigned long long k = ((unsigned long long)ford(tot) << 32) | (unsigned)arc;
  const Relax rl = relax_lds<true>(a, sh, t, dest, k, eps);
  if (rl.slot != kNoSlot) return rl;
  const unsigned hm = (1u << a.hbits) - 1u;
  unsigned g = hbm_hash(dest, a.hbits);
  for (int probe = 0; probe < a.hprobe; probe++) {
    const int cur = atomicCAS(&T.state[g], -1, dest);  // one round trip per probe
    if (cur == -1) {
      hbm_created(a, sh, T, g, k, eps);
      return Relax{~(int)g, 2};
    }
    if (cur == dest) {
      const unsigned long long old = atomicMin(&T.key[g], k);
      return Relax{~(int)g, k < old ? 1 : 0};
    }
    g = (g + 1) & hm;
  }
  sh.bad |= 1;
  return Relax{0, -1};
}

// The emitting pass's relaxations, kUnroll per thread: the LDS buckets
// first, then the HBM probes of all items that need them in flight together
// (one CAS per probe); keys by atomic min without waiting for the result
// (the winners are found after the sub-round's barrier).  Output per item:
// slot (kNoSlot: no relaxation) and created.
template <int NU = kUnroll>
__device__ __forceinline__ void relax_batch(const DecArgs& a, DecShared& sh, const FrameLds& t, const HbmTab& T,
                                            const int* dest, const unsigned long long* key, const bool* eps,
                                            const bool* want, int* slot_out, bool* created) {
  bool pend[NU];
  unsigned g[NU];
  bool any = false;
#pragma unroll
  for (int u = 0; u < NU; u++) {
    slot_out[u] = kNoSlot;
    created[u] = false;
    pend[u] = false;
    if (!want[u]) continue;
    const Relax r = relax_lds<false>(a, sh, t, dest[u], key[u], eps[u]);
    if (r.slot != kNoSlot) {
      slot_out[u] = r.slot;
      created[u] = r.flags == 2;
    } else {
      pend[u] = true;
      g[u] = hbm_hash(dest[u], a.hbits);
      any = true;
    }
  }
  const unsigned hm = (1u << a.hbits) - 1u;
  for (int probe = 0; any && probe < a.hprobe; probe++) {
    int cur[NU];
#pragma unroll
    for (int u = 0; u < NU; u++)
      if (pend[u]) cur[u] = atomicCAS(&T.state[g[u]], -1, dest[u]);
    any = false;
#pragma unroll
    for (int u = 0; u < NU; u++) {
      if (!pend[u]) continue;
      if (cur[u] == -1) {
        hbm_created(a, sh, T, g[u], key[u], eps[u]);
        slot_out[u] = ~(int)g[u];
        created[u] = true;
        pend[u] = false;
      } else if (cur[u] == dest[u]) {
        __hip_atomic_fetch_min(&T.key[g[u]], key[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        slot_out[u] = ~(int)g[u];
        pend[u] = false;
      } else {
        g[u] = (g[u] + 1) & hm;
        any = true;
      }
    }
  }
#pragma unroll
  for (int u = 0; u < NU; u++)
    if (pend[u]) sh.bad |= 1;
}

__device__ __forceinline__ unsigned long long slot_key(const FrameLds& t, const HbmTab& T, int v) {
  return v >= 0 ? t.hk[v] : AG_LD(&T.key[~v]);
}
__device__ __forceinline__ int slot_state(const FrameLds& t, const HbmTab& T, int v) {
  return v >= 0 ? t.hs[v] : AG_LD(&T.state[~v]);
}
__device__ __forceinline__ void set_bp(const FrameLds& t, const HbmTab& T, int v, int bp) {
  if (v >= 0) t.hb[v] = bp;
  else AG_ST(&T.bp[~v], bp);
}
// position of a slot of the frame under construction in the committed frame
// (arena offset): its creation index (nl_n = the LDS count), or in Kaldi
// order its list position (kaldi_positions, kept in the slot's hst / stamp)
__device__ __forceinline__ int slot_pos(const DecArgs& a, const FrameLds& t, const HbmTab& T, int nl_n, int v) {
  if (a.kaldi) return v >= 0 ? t.hst[v] : AG_LD(&T.stamp[~v]);
  return v >= 0 ? (int)(t.hp[v] & 0x7fff) : nl_n + (AG_LD(&T.pos[~v]) & (kHPosEps - 1));
}
// the epsilon-source slot code of a relaxation from slot v
__device__ __forceinline__ int eps_bp(int v) { return kBpEps | (v >= 0 ? v : (kBpHbm | ~v)); }
__device__ __forceinline__ int bp_slot(int bp) {
  const int c = bp & ~kBpEps;
  return (c & kBpHbm) ? ~(c & (kBpHbm - 1)) : c;
}

// slot of state s in the frame under construction (eps links at commit);
// kNoSlot if absent
__device__ __forceinline__ int frame_slot(const DecArgs& a, const FrameLds& t, const HbmTab& T, int s) {
  const int nbk = a.lds_probe < 2 ? a.lds_probe : 2;
  const unsigned b1 = bucket1(s);
  for (int nb = 0; nb < nbk; nb++) {
    const int h0 = 4 * (int)(nb ? bucket2(s, b1) : b1);
    for (int i = 0; i < 4; i++) {
      const int c = t.hs[h0 + i];
      if (c == s) return h0 + i;
      if (c == -1) return kNoSlot;  // the state would be here
    }
  }
  const unsigned hm = (1u << a.hbits) - 1u;
  unsigned g = hbm_hash(s, a.hbits);
  for (int probe = 0; probe < a.hprobe; probe++) {
    const int c = AG_LD(&T.state[g]);
    if (c == s) return ~(int)g;
    if (c == -1) break;
    g = (g + 1) & hm;
  }
  return kNoSlot;
}

__device__ __forceinline__ void push_front(const DecArgs& a, DecShared& sh, const FrameLds& t,
                                           const DecPtrs& p, int b, int* count, int v) {
  const int q = atomicAdd(count, 1);
  if (q < kFrontLds) (b ? t.fr1 : t.fr0)[q] = v;
  else if (q - kFrontLds < a.max_tok) AG_ST(&(b ? p.fg1 : p.fg0)[q - kFrontLds], v);
  else sh.bad |= 1;
}
__device__ __forceinline__ int get_front(const FrameLds& t, const DecPtrs& p, int b, int i) {
  return i < kFrontLds ? (b ? t.fr1 : t.fr0)[i] : AG_LD(&(b ? p.fg1 : p.fg0)[i - kFrontLds]);
}

// ---------------------------------------------------------------------------
// lattice links.  During the emitting pass every relaxation below the bound
// appends {src arena index, tot bits, arc, acoustic cost bits} to the
// stream's link arena and its destination slot to link_dst; the commit keeps
// those below the frame's final cutoff with tot replaced by the destination's
// arena index, then appends the frame's epsilon links from the final token
// costs (one per arc, Kaldi re-expands a token whenever it improves:
// ProcessNonemitting).  A committed link is {src arena index, dst arena
// index, arc, acoustic cost bits}.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void emit_link(const DecArgs& a, DecShared& sh, long long used, int slot,
                                          int4 rec, int dslot, bool defer) {
  const unsigned long long m = __ballot(1);
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((long long)m) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(&sh.n_links, __popcll(m));
  base = __builtin_amdgcn_readlane(base, leader);
  const int off = __popcll(m & ((1ull << lane) - 1ull));
  const long long pos = used + base + off;
  if (pos < a.link_cap) {
    a.links[(long long)slot * a.link_cap + pos] = rec;
    a.link_dst[(long long)slot * a.link_cap + pos] = dslot;
  } else {
    sh.lat_ovf = 1;
    if (defer) sh.bad |= 32;  // the record held a backpointer candidate (deferred winners)
  }
}

// one emitting expansion pass over the current tokens (ProcessEmitting):
// mode 0 = minimum only, 1 = relax below `bound` (+ minimum).  Items are
// processed kUnroll per thread at a time (arc loads in flight together),
// each sub-round closed by a barrier after which the sub-round's winners
// write their backpointers.
__device__ __forceinline__ float expand_emitting(const DecArgs& a, DecShared& sh, const FrameLds& t,
                                 const HbmTab& T, const DecPtrs& p, const TokView& tv, int ntok,
                                 float cutoff, float cost_offset, const float* Lp, int mode,
                                 float bound, float adaptive, int* examined, const DecSlot& st, int slot,
                                 bool defer, Prof& pr) {
  float m = __int_as_float(0x7f800000);
  // Running bound (Kaldi's running next_cutoff): min(bound, tot + adaptive)
  // over the relaxations seen so far.  It never falls below the pass's final
  // next_cutoff (min over all of tot + adaptive), so a relaxation at or
  // above it could only create an entry the commit drops as dead.
  if (threadIdx.x == 0) sh.run_bound = ford(bound);
  // defer: every relaxation leaves a link record and the winners are
  // resolved from the records at commit (commit_emit_links)
  const bool lat = a.links != nullptr && mode == 1;
  defer = defer && lat;
  // the next chunk's token (cost, state, list position) is loaded while
  // this chunk's arcs are processed
  float cn = 0.0f;
  int sn = 0, pn = 0;
  if ((int)threadIdx.x < ntok) {
    cn = tv.c(threadIdx.x);
    sn = tv.s(threadIdx.x);
    if (mode == 1) pn = AG_LD(&p.cp[threadIdx.x]);
  }
  for (int c0 = 0; c0 < ntok; c0 += DT) {
    const int i = c0 + threadIdx.x;
    int deg = 0, ab = 0, src = 0;
    float c = 0.0f;
    if (i < ntok) {
      c = cn;
      if (c <= cutoff) {
        const int4 si = a.sinfo[sn];
        ab = si.x;
        deg = si.y - si.x;
        if (mode == 1) src = st.cur_base + pn;
      }
    }
    block_scan(sh, deg);
    owner_blocks(sh);
    sh.abeg[threadIdx.x] = ab;
    sh.tcost[threadIdx.x] = c;
    sh.tsrc[threadIdx.x] = src;
    __syncthreads();
    if (i + DT < ntok) {
      cn = tv.c(i + DT);
      sn = tv.s(i + DT);
      if (mode == 1) pn = AG_LD(&p.cp[i + DT]);
    }
    pr.mark(2);
    pr.count(14, 1);
    const int total = sh.total;
    const int nbo = (total + 63) >> 6 <= kOwnBlk ? (total + 63) >> 6 : 0;
    *examined += total;
    for (int sb = 0; sb < total; sb += DT * kUnroll) {
      int4 A[kUnroll];
      int jv[kUnroll], arcv[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; u++) {
        const int it = sb + u * DT + (int)threadIdx.x;
        jv[u] = -1;
        if (it < total) {
          const int j = owner_bo(sh, nbo, it);
          jv[u] = j;
          arcv[u] = sh.abeg[j] + (it - sh.scan[j]);
          A[u] = a.arcs[arcv[u]];
        }
      }
      int sv[kUnroll], dst[kUnroll];
      unsigned long long kv[kUnroll];
      float acv[kUnroll], totv[kUnroll];
      bool want[kUnroll], de[kUnroll], cr[kUnroll];
      const float rb = mode == 1 ? funord(__hip_atomic_load(&sh.run_bound, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_WORKGROUP))
                                 : bound;
      float wm = __int_as_float(0x7f800000);
#pragma unroll
      for (int u = 0; u < kUnroll; u++) {
        want[u] = false;
        if (jv[u] < 0) continue;
        const int j = jv[u];
        acv[u] = cost_offset - Lp[A[u].z];
        totv[u] = (sh.tcost[j] + acv[u]) + __int_as_float(A[u].y);
        m = fminf(m, totv[u]);
        wm = fminf(wm, totv[u]);
        want[u] = mode == 1 && totv[u] < rb;
        dst[u] = A[u].x;
        de[u] = ((unsigned)A[u].w & kDestEps) != 0;
        kv[u] = ((unsigned long long)ford(totv[u]) << 32) | (unsigned)arcv[u];
      }
      pr.mark(3);
      if (mode == 1) {
        wm = wave_min_f(wm);
        if ((threadIdx.x & 63) == 0 && wm + adaptive < rb) atomicMin(&sh.run_bound, ford(wm + adaptive));
        relax_batch(a, sh, t, T, dst, kv, de, want, sv, cr);
        pr.mark(22);
#pragma unroll
        for (int u = 0; u < kUnroll; u++) {
          if (!want[u]) continue;
          if (lat)
            emit_link(a, sh, st.links_used, slot,
                      make_int4(sh.tsrc[jv[u]], __float_as_int(totv[u]), arcv[u], __float_as_int(acv[u])),
                      sv[u], defer);
          if (cr[u] && de[u]) push_front(a, sh, t, p, 0, &sh.n_front, sv[u]);
        }
      }
      pr.mark(23);
      if (mode == 1 && !defer) {
        // the relaxations' key minima are issued without waiting for them
        // (no-return atomics): wait for their completion (vmcnt, no cache
        // maintenance) before the barrier, so every winner check below reads
        // keys that include its own relaxation
        vm_drain();
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kUnroll; u++)
          if (want[u] && sv[u] != kNoSlot && slot_key(t, T, sv[u]) == kv[u])
            set_bp(t, T, sv[u], sh.tsrc[jv[u]]);
        pr.mark(4);
      }
    }
    // deferred: the keys' no-return minima complete before the chunk's
    // barrier (the epsilon closure and the commit read them)
    if (defer) vm_drain();
    __syncthreads();
    pr.mark(2);
  }
  return block_min_f(sh, m);
}

// ProcessNonemitting: epsilon closure in rounds over frontiers that only
// hold states with epsilon arcs (round 0: created by the emitting pass);
// a state improved in a round is expanded again in the next one.
__device__ __forceinline__ void eps_closure(const DecArgs& a, DecShared& sh, const FrameLds& t, const HbmTab& T,
                            const DecPtrs& p, DecSlot& st, float cutoff, int nfront, int* arcs_eps,
                            Prof& pr) {
  int b = 0;
  int examined = 0;
  const int cap = kFrontLds + a.max_tok;
  nfront = nfront < cap ? nfront : cap;
  while (nfront > 0) {
    pr.count(13, 1);
    st.stamp++;
    const int stamp = st.stamp;
    __syncthreads();
    if (threadIdx.x == 0) sh.n_fnext = 0;
    for (int c0 = 0; c0 < nfront; c0 += DT) {
      const int i = c0 + threadIdx.x;
      int deg = 0, ab = 0, v = 0;
      float c = 0.0f;
      if (i < nfront) {
        v = get_front(t, p, b, i);
        c = funord((uint32_t)(slot_key(t, T, v) >> 32));
        if (c < cutoff) {  // created tokens are < cutoff; dead ones are not
          const int4 si = a.sinfo[slot_state(t, T, v)];
          ab = si.y;
          deg = si.z - si.y;
        }
      }
      block_scan(sh, deg);
      sh.abeg[threadIdx.x] = ab;
      sh.tcost[threadIdx.x] = c;
      sh.tsrc[threadIdx.x] = eps_bp(v);
      __syncthreads();
      const int total = sh.total;
      examined += total;
      for (int sb = 0; sb < total; sb += DT) {
        const int it = sb + threadIdx.x;
        int sv = 0x7fffffff, j = 0;
        unsigned long long kk = 0;
        if (it < total) {
          j = owner(sh, it);
          const int arc = sh.abeg[j] + (it - sh.scan[j]);
          const int4 A = a.arcs[arc];
          const float tot = sh.tcost[j] + __int_as_float(A.y);
          if (tot < cutoff) {
            const bool de = ((unsigned)A.w & kDestEps) != 0;
            const Relax r = relax(a, sh, t, T, A.x, tot, arc, de);
            if (r.flags > 0) {
              sv = r.slot;
              kk = ((unsigned long long)ford(tot) << 32) | (unsigned)arc;
              if (de) {
                const int old = r.slot >= 0 ? atomicExch(&t.hst[r.slot], stamp)
                                            : atomicExch(&T.stamp[~r.slot], stamp);
                if (old != stamp) push_front(a, sh, t, p, b ^ 1, &sh.n_fnext, r.slot);
              }
            }
          }
        }
        vm_drain();  // a created HBM entry's key minimum is a no-return atomic (hbm_created)
        __syncthreads();
        if (sv != 0x7fffffff && slot_key(t, T, sv) == kk) set_bp(t, T, sv, sh.tsrc[j]);
      }
      __syncthreads();
    }
    nfront = sh.n_fnext < cap ? sh.n_fnext : cap;
    b ^= 1;
  }
  *arcs_eps += examined;
}

// hst / stamp: the epsilon round stamp of the order-independent closure, or
// in Kaldi order the creation index, then the list position; kNoStamp when
// the entry is free
constexpr int kNoStamp = 0x7fffffff;

__device__ __forceinline__ void lds_clear_build(const FrameLds& t) {
  for (int h = threadIdx.x; h < kHashCap; h += DT) {
    t.hs[h] = -1;
    t.hk[h] = kEmpty;
    t.hst[h] = kNoStamp;
  }
}

// clears the listed entries of the HBM table
__device__ __forceinline__ void hbm_clear_listed(const DecArgs& a, const HbmTab& T, int n) {
  for (int j = threadIdx.x; j < n; j += DT) {
    const int g = AG_LD(&T.list[j]);
    AG_ST(&T.state[g], -1);
    AG_ST(&T.key[g], kEmpty);
    if (a.kaldi) AG_ST(&T.stamp[g], kNoStamp);
  }
}
__device__ __forceinline__ void hbm_clear_all(const DecArgs& a, const HbmTab& T) {
  const int H = 1 << a.hbits;
  for (int g = threadIdx.x; g < H; g += DT) {
    AG_ST(&T.state[g], -1);
    AG_ST(&T.key[g], kEmpty);
    AG_ST(&T.stamp[g], kNoStamp);
  }
}

// ---------------------------------------------------------------------------
// Kaldi order (DecArgs::kaldi, the default).  Kaldi's
// ProcessEmitting walks the frame's tokens in HashList order and tightens
// next_cutoff as it goes, so which relaxations create tokens depends on that
// order.  Here:
//  - the current-token arrays are kept in HashList order (kaldi_positions:
//    buckets state % khash in order of first occupancy, then creation);
//  - the emitting pass enumerates the (token, arc) items in that order and
//    accepts item i iff tot_i < min(seed, min_{j<i} tot_j + adaptive_beam),
//    a block prefix minimum carried across sub-rounds (a rejected item never
//    lowers it: tot_j >= the running cutoff and adaptive_beam > 0);
//  - a token's creation index is the rank of its first accepted relaxation
//    (ranked densely per sub-round), then its order of creation in the
//    epsilon queue;
//  - ProcessNonemitting runs as Kaldi's LIFO queue on one thread, seeded in
//    list order with the tokens that can relax an epsilon arc below the
//    cutoff (another token does nothing when Kaldi pops it; if its cost later
//    falls it is pushed again, as in Kaldi);
//  - a token's cost is the minimum over its accepted relaxations and its
//    backpointer the minimum (cost, arc) one; every token Kaldi creates is
//    kept, every accepted emitting relaxation is a lattice link.
// ---------------------------------------------------------------------------

// exclusive running minimum over the block in thread order, seeded with
// sh.kcar[par]; leaves the running minimum after the block in sh.kcar[par ^ 1]
__device__ __forceinline__ float kaldi_excl_min(DecShared& sh, float v, int par) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float incl = wave_incl_min(v);
  const float excl = wave_shr1(incl, __int_as_float(0x7f800000));
  if (lane == 63) sh.kmin_w[par][w] = incl;
  __syncthreads();
  float pre = sh.kcar[par];
  for (int i = 0; i < w; i++) pre = fminf(pre, sh.kmin_w[par][i]);
  if (threadIdx.x == DT - 1) sh.kcar[par ^ 1] = fminf(pre, incl);
  return fminf(pre, excl);
}

// The same running minimum without a block barrier (decoupled look-back,
// Merrill & Garland's single-pass scan): wave w of sub-round s is item block
// q = s * DW + w; it publishes its block minimum, then walks back over the
// published blocks (spinning on one not yet published) until one carries
// its inclusive prefix (or q = 0, whose carry-in is `seed`), and publishes
// its own inclusive prefix.  A wave never waits for another wave's
// relaxations, only for its block minimum.  Returns the exclusive running
// minimum before this lane's item; *incl_out (wave-uniform) the inclusive
// prefix through this block.  The ring holds four sub-rounds: a wave can be
// at most one sub-round ahead of the slowest (it needs that wave's block
// minimum to finish its own look-back).
constexpr unsigned kLbIncl = 1u;
__device__ __forceinline__ unsigned long long kaldi_lb_pack(int q, unsigned fl, float x) {
  return ((unsigned long long)(((unsigned)q << 1) | fl) << 32) | (unsigned long long)ford(x);
}
// a block's aggregate published before its look-back (lane 0)
__device__ __forceinline__ void kaldi_lb_publish(DecShared& sh, int q, float agg) {
  if ((threadIdx.x & 63) == 0)
    __hip_atomic_store(&sh.kls[q % (4 * DW)], kaldi_lb_pack(q, 0u, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ float kaldi_lookback_min(DecShared& sh, float v, int q, float seed, float* incl_out) {
  const int lane = threadIdx.x & 63;
  const float incl = wave_incl_min(v);
  const float excl = wave_shr1(incl, __int_as_float(0x7f800000));
  const float agg = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(incl), 63));
  constexpr int R = 4 * DW;
  kaldi_lb_publish(sh, q, agg);
  float carry = __int_as_float(0x7f800000);
  if (q == 0) {
    carry = seed;
  } else {
    // the look-back reads a window of kLbWin blocks at once, one per lane
    // (blocks k - lane), and folds the window up to its nearest inclusive
    // prefix when every block before it is published.  A wave is never more
    // than DW blocks ahead of the slowest, so the ring's R >= 2 kLbWin
    // entries in the window are the blocks named, or not yet published.
    constexpr int kLbWin = 32;
    static_assert(R >= 2 * kLbWin && kLbWin >= DW, "look-back window");
    int k = q - 1;
    while (true) {
      const int kb = k - lane;
      const bool in = lane < kLbWin && kb >= 0;
      unsigned long long st = 0;
      if (in) st = __hip_atomic_load(&sh.kls[kb % R], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const unsigned hi = (unsigned)(st >> 32);
      const bool have = in && (int)(hi >> 1) == kb;
      const bool stop = have && ((hi & kLbIncl) || kb == 0);
      const unsigned long long hv = __ballot(have), hs = __ballot(stop);
      const int nin = k + 1 < kLbWin ? k + 1 : kLbWin;
      const unsigned long long need = hs ? ((hs & (0ull - hs)) << 1) - 1ull : (1ull << nin) - 1ull;
      if ((hv & need) != need) {
        // a block before the nearest prefix is not published yet: one lane
        // waits for the nearest such block (spinning lanes would take LDS
        // bandwidth from the relaxations), then the window is read again
        const int km = k - (__ffsll((long long)(need & ~hv)) - 1);
        if (lane == 0)
          while ((int)((unsigned)(__hip_atomic_load(&sh.kls[km % R], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >>
                                  32) >> 1) != km)
            __builtin_amdgcn_s_sleep(1);
        continue;
      }
      // fold the needed lanes (usually one or two) with scalar lane reads
      const int lo = (int)(unsigned)st;
      for (unsigned long long mm = need; mm; mm &= mm - 1ull)
        carry = fminf(carry, funord((uint32_t)__builtin_amdgcn_readlane(lo, __ffsll((long long)mm) - 1)));
      if (hs) {
        const int lf = __ffsll((long long)hs) - 1;
        if (k == lf && !((unsigned)__builtin_amdgcn_readlane((int)hi, lf) & kLbIncl))
          carry = fminf(carry, seed);  // block 0's aggregate: add the seed
        break;
      }
      k -= kLbWin;
    }
  }
  const float inc = fminf(carry, agg);
  if (lane == 0)
    __hip_atomic_store(&sh.kls[q % R], kaldi_lb_pack(q, kLbIncl, inc), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  *incl_out = inc;
  return fminf(carry, excl);
}

// exclusive prefix sum over the block in thread order; *total = the block's sum
__device__ __forceinline__ int kaldi_excl_sum(DecShared& sh, int v, int par, int* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int incl = wave_incl_sum(v);
  if (lane == 63) sh.ksum_w[par][w] = incl;
  __syncthreads();
  int off = 0, tot = 0;
  for (int i = 0; i < DW; i++) {
    const int x = sh.ksum_w[par][i];
    off += i < w ? x : 0;
    tot += x;
  }
  *total = tot;
  return off + incl - v;
}

// the epsilon queue's HBM member records (kaldi_nonemitting), ints per record
constexpr int kKMRec = 8;

// a state's HashList bucket: its id % khash -- OpenFST's lazy id on a
// composed graph (DecArgs::lazy_id), else the graph's
// (the expanded flag masked off)
static_assert(DT <= kLazyNewCap, "lazy_new holds a frame's new emitting tokens up to DT");
__device__ __forceinline__ int kid(const DecArgs& a, int slot, int state) {
  return a.lazy_id ? AG_LD(&a.lazy_id[(long long)slot * a.lazy_ids + state]) : state;
}
__device__ __forceinline__ int kbucket_of(int id, int khash) {
  return (int)((unsigned)(id & (kLazyExpanded - 1)) % (unsigned)khash);
}
__device__ __forceinline__ int kbucket(const DecArgs& a, int slot, int state, int khash) {
  return kbucket_of(kid(a, slot, state), khash);
}
// HashList bookkeeping loops: creation indices per thread in flight together
constexpr int kHlU = 4;

// Creation ranks of the emitting pass's new tokens (deferred form): each
// created slot holds the index of its first accepted relaxation (hst /
// stamp); its creation index is that item's rank among all such items -- a
// bitmap over the pass's items and the popcount prefix sums of its words
// (bits / pre: nw = ceil(nitems / 32) words each, LDS or HBM).  Returns the
// number of created tokens.
template <typename BitsT, typename PreT>
__device__ __forceinline__ int kaldi_rank_creators(const DecArgs& a, DecShared& sh, const FrameLds& t,
                                                   const HbmTab& T, int slot, int nitems, BitsT* bits, PreT* pre) {
  int* KO = a.kord + (long long)slot * a.kord_cap;
  const int nw = (nitems + 31) >> 5;
  for (int w = threadIdx.x; w < nw; w += DT) bits[w] = 0u;
  vm_drain();
  __syncthreads();
  const int nl = sh.n_new_l, ng = sh.n_new_g < a.max_tok ? sh.n_new_g : a.max_tok;
  for (int j = threadIdx.x; j < nl + ng; j += DT) {
    const int v = j < nl ? (int)t.nl[j] : ~AG_LD(&T.list[j - nl]);
    const int it = v >= 0 ? t.hst[v] : AG_LD(&T.stamp[~v]);
    if (it >= 0 && it < nitems) atomicOr(&bits[it >> 5], 1u << (it & 31));
  }
  vm_drain();
  __syncthreads();
  int run = 0, par = 0;
  for (int w0 = 0; w0 < nw; w0 += DT) {
    const int w = w0 + threadIdx.x;
    const int c = w < nw ? __popc(bits[w]) : 0;
    int tot;
    const int ex = run + kaldi_excl_sum(sh, c, par, &tot);
    if (w < nw) pre[w] = ex;
    run += tot;
    par ^= 1;
  }
  vm_drain();
  __syncthreads();
  for (int j = threadIdx.x; j < nl + ng; j += DT) {
    const int v = j < nl ? (int)t.nl[j] : ~AG_LD(&T.list[j - nl]);
    const int it = v >= 0 ? t.hst[v] : AG_LD(&T.stamp[~v]);
    if (it < 0 || it >= nitems) {
      sh.bad |= 1;
      continue;
    }
    const int rk = pre[it >> 5] + __popc(bits[it >> 5] & ((1u << (it & 31)) - 1u));
    if (rk < a.kord_cap) {
      if (v >= 0) t.hst[v] = rk;
      else AG_ST(&T.stamp[~v], rk);
      AG_ST(&KO[rk], v);
    } else {
      sh.bad |= 1;
    }
  }
  vm_drain();
  __syncthreads();
  return run;
}

// consecutive items per thread per sub-round of the deferred emitting pass
#ifndef VAMD_EMIT_ITEMS
#define VAMD_EMIT_ITEMS 2
#endif
constexpr int kEmitU = VAMD_EMIT_ITEMS;

// ProcessEmitting in list order (see above); returns next_cutoff.  The
// created tokens get creation indices [0, *ncreated) (kord: index -> slot).
// defer: backpointers are resolved at commit from the link records and the
// creation ranks after the pass (one barrier per sub-round, the running
// cutoff's); otherwise both are settled per sub-round.
__device__ __forceinline__ float expand_emitting_kaldi(const DecArgs& a, DecShared& sh, const FrameLds& t,
                                                       const HbmTab& T, const DecPtrs& p, const TokView& tv,
                                                       int ntok, float cutoff, float cost_offset, const float* Lp,
                                                       float seed, float adaptive, int* examined, const DecSlot& st,
                                                       int slot, int* ncreated, bool defer, float* Lbuf, Prof& pr) {
  const bool lat = a.links != nullptr;
  int* KO = a.kord + (long long)slot * a.kord_cap;
  if (threadIdx.x == 0) sh.kcar[0] = seed;  // read after the next barrier
  for (int i = threadIdx.x; i < 4 * DW; i += DT) sh.kls[i] = ~0ull;  // no block published (cleared before the first chunk's barrier)
  int par = 0, ibase = 0, nc = 0, qsub = 0;
  float incl_last = seed;
  float cn = 0.0f;
  int sn = 0, pn = 0;
  if ((int)threadIdx.x < ntok) {
    cn = tv.c(threadIdx.x);
    sn = tv.s(threadIdx.x);
    pn = AG_LD(&p.cp[threadIdx.x]);
  }
  for (int c0 = 0; c0 < ntok; c0 += DT) {
    const int i = c0 + threadIdx.x;
    int deg = 0, ab = 0, src = 0;
    float c = 0.0f;
    if (i < ntok) {
      c = cn;
      if (c <= cutoff) {
        const int4 si = a.sinfo[sn];
        ab = si.x;
        deg = si.y - si.x;
        src = st.cur_base + pn;
      }
    }
    block_scan(sh, deg);
    owner_blocks(sh);
    sh.abeg[threadIdx.x] = ab;
    sh.tcost[threadIdx.x] = c;
    sh.tsrc[threadIdx.x] = src;
    __syncthreads();
    if (i + DT < ntok) {
      cn = tv.c(i + DT);
      sn = tv.s(i + DT);
      pn = AG_LD(&p.cp[i + DT]);
    }
    pr.mark(2);
    pr.count(14, 1);
    const int total = sh.total;
    const int nbo = (total + 63) >> 6 <= kOwnBlk ? (total + 63) >> 6 : 0;
    *examined += total;
    if (defer && kEmitU > 1) {
      // deferred winners: kEmitU consecutive items per thread per sub-round
      // -- fewer sub-rounds, so fewer look-back blocks in the running
      // cutoff's chain (the lane's minimum over its items feeds the
      // look-back; each item's running cutoff adds its predecessors')
      constexpr int U = kEmitU;
      const float kInfE = __int_as_float(0x7f800000);
      int jn[U], an[U];
      int4 An[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int i = U * (int)threadIdx.x + u;
        jn[u] = 0;
        an[u] = 0;
        An[u] = make_int4(0, 0, 0, 0);
        if (i < total) {
          jn[u] = owner_bo(sh, nbo, i);
          an[u] = sh.abeg[jn[u]] + (i - sh.scan[jn[u]]);
          An[u] = a.arcs[an[u]];
        }
      }
      for (int sb = 0; sb < total; sb += U * DT) {
        const int it0 = sb + U * (int)threadIdx.x;
        int jj[U], aa[U];
        int4 AA[U];
        float ac[U], tot[U], x[U];
        float lane_min = kInfE;
#pragma unroll
        for (int u = 0; u < U; u++) {
          jj[u] = jn[u];
          aa[u] = an[u];
          AA[u] = An[u];
          ac[u] = 0.0f;
          tot[u] = kInfE;
          x[u] = kInfE;
          if (it0 + u < total) {
            ac[u] = cost_offset - Lp[AA[u].z];
            tot[u] = (sh.tcost[jj[u]] + ac[u]) + __int_as_float(AA[u].y);
            x[u] = tot[u] + adaptive;
          }
          lane_min = fminf(lane_min, x[u]);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
          const int i = it0 + U * DT + u;
          if (i < total) {
            jn[u] = owner_bo(sh, nbo, i);
            an[u] = sh.abeg[jn[u]] + (i - sh.scan[jn[u]]);
            An[u] = a.arcs[an[u]];
          }
        }
        pr.mark(3);
        float run = kaldi_lookback_min(sh, lane_min, qsub * DW + (int)(threadIdx.x >> 6), seed, &incl_last);
        qsub++;
        pr.mark(62);
#pragma unroll
        for (int u = 0; u < U; u++) {
          const bool want = it0 + u < total && tot[u] < run;
          run = fminf(run, x[u]);
          if (!want) continue;
          const int item = ibase + it0 + u;
          const int dsts[1] = {AA[u].x};
          const unsigned long long keys[1] = {((unsigned long long)ford(tot[u]) << 32) | (unsigned)aa[u]};
          const bool des[1] = {((unsigned)AA[u].w & kDestEps) != 0}, wants[1] = {true};
          int svs[1];
          bool crs[1];
          relax_batch<1>(a, sh, t, T, dsts, keys, des, wants, svs, crs);
          int sv = kNoSlot;
          if (svs[0] != kNoSlot) {
            sv = svs[0];
            if (sv >= 0) atomicMin(&t.hst[sv], item);
            else __hip_atomic_fetch_min(&T.stamp[~sv], item, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          if (lat)
            emit_link(a, sh, st.links_used, slot,
                      make_int4(sh.tsrc[jj[u]], __float_as_int(tot[u]), aa[u], __float_as_int(ac[u])), sv, false);
        }
        pr.mark(22);
        par ^= 1;
      }
      ibase += total;
      __syncthreads();
      pr.mark(2);
      continue;
    }
    // software pipeline: a sub-round's item (owner search, arc load) is
    // fetched before the previous sub-round's scan barrier, so the arc
    // latency overlaps the barrier and the relaxations
    int jn = 0, arcn = 0;
    int4 An = make_int4(0, 0, 0, 0);
    if ((int)threadIdx.x < total) {
      jn = owner_bo(sh, nbo, threadIdx.x);
      arcn = sh.abeg[jn] + ((int)threadIdx.x - sh.scan[jn]);
      An = a.arcs[arcn];
    }
    for (int sb = 0; sb < total; sb += DT) {
      const int it = sb + (int)threadIdx.x;
      const bool valid = it < total;
      const int j = jn, arc = arcn;
      const int4 A = An;
      float ac = 0.0f, tot = __int_as_float(0x7f800000);
      if (valid) {
        ac = cost_offset - Lp[A.z];
        tot = (sh.tcost[j] + ac) + __int_as_float(A.y);
      }
      if (it + DT < total) {
        jn = owner_bo(sh, nbo, it + DT);
        arcn = sh.abeg[jn] + (it + DT - sh.scan[jn]);
        An = a.arcs[arcn];
      }
      pr.mark(3);
      // defer: the running cutoff by look-back (no barrier per sub-round)
      const float run = defer ? kaldi_lookback_min(sh, valid ? tot + adaptive : __int_as_float(0x7f800000),
                                                   qsub * DW + (int)(threadIdx.x >> 6), seed, &incl_last)
                              : kaldi_excl_min(sh, valid ? tot + adaptive : __int_as_float(0x7f800000), par);
      qsub++;
      pr.mark(62);
      const bool want = valid && tot < run;
      const int item = ibase + it;
      const unsigned long long kv = ((unsigned long long)ford(tot) << 32) | (unsigned)arc;
      int sv = kNoSlot;
      if (want) {
        // key minima without waiting for the old values (no-return atomics;
        // only the slot matters here)
        const bool de = ((unsigned)A.w & kDestEps) != 0;
        const int dsts[1] = {A.x};
        const unsigned long long keys[1] = {((unsigned long long)ford(tot) << 32) | (unsigned)arc};
        const bool des[1] = {de}, wants[1] = {true};
        int svs[1];
        bool crs[1];
        relax_batch<1>(a, sh, t, T, dsts, keys, des, wants, svs, crs);
        if (svs[0] != kNoSlot) {
          sv = svs[0];
          if (sv >= 0) atomicMin(&t.hst[sv], item);
          else __hip_atomic_fetch_min(&T.stamp[~sv], item, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lat)
          emit_link(a, sh, st.links_used, slot, make_int4(sh.tsrc[j], __float_as_int(tot), arc, __float_as_int(ac)),
                    sv, false);
      }
      pr.mark(22);
      par ^= 1;
      if (defer) continue;
      vm_drain();  // the relaxations' atomics (keys, creation indices) are complete at the barrier
      __syncthreads();
      // each slot's winner writes its backpointer; its creator (the slot's
      // first accepted relaxation) takes the next creation index
      int cf = 0;
      if (sv != kNoSlot) {
        if (slot_key(t, T, sv) == kv) set_bp(t, T, sv, sh.tsrc[j]);
        cf = (sv >= 0 ? t.hst[sv] : AG_LD(&T.stamp[~sv])) == item;
      }
      int ncr;
      const int rk = nc + kaldi_excl_sum(sh, cf, par, &ncr);
      if (cf) {
        if (rk < a.kord_cap) {
          if (sv >= 0) t.hst[sv] = rk;
          else AG_ST(&T.stamp[~sv], rk);
          AG_ST(&KO[rk], sv);
        } else {
          sh.bad |= 1;
        }
      }
      vm_drain();
      nc += ncr;
      pr.mark(4);
    }
    ibase += total;
    __syncthreads();
    pr.mark(2);
  }
  // the running cutoff after every item: the last block's inclusive prefix
  // (defer; the last wave of the last sub-round), else the barrier scan's carry
  if (defer && qsub > 0 && (threadIdx.x >> 6) == DW - 1 && (threadIdx.x & 63) == 0) sh.kcar[par] = incl_last;
  __syncthreads();
  const float next_cutoff = sh.kcar[par];
  if (defer) {
    vm_drain();
    __syncthreads();
    // the item bitmap and its prefix sums in the staged log-likelihood row
    // (no longer read in this frame) when they fit, else in the stream's
    // epsilon-queue scratch (unused until the queue runs)
    if (ibase <= 32 * (kLlhLds / 2)) {
      unsigned* bits = reinterpret_cast<unsigned*>(Lbuf);
      nc = kaldi_rank_creators(a, sh, t, T, slot, ibase, bits, reinterpret_cast<int*>(Lbuf) + kLlhLds / 2);
    } else {
      int* KM = a.kmem + (long long)slot * a.kord_cap * kKMRec;
      const long long room = (long long)a.kord_cap * kKMRec;
      const int nw = (ibase + 31) >> 5;
      if (2LL * nw <= room) {
        nc = kaldi_rank_creators(a, sh, t, T, slot, ibase, reinterpret_cast<unsigned*>(KM), KM + nw);
      } else {
        if (threadIdx.x == 0) sh.bad |= 1;
        __syncthreads();
        nc = 0;
      }
    }
    pr.mark(4);
  }
  __syncthreads();
  if (nc > a.kord_cap && threadIdx.x == 0) sh.bad |= 1;
  *ncreated = nc < a.kord_cap ? nc : a.kord_cap;
  return next_cutoff;
}

// LDS views for Kaldi's epsilon queue (kaldi_nonemitting): regions no other
// phase uses between the emitting pass and the commit (the log-likelihood
// row, the token cache, the block-scan arrays, the frontier arrays); entries
// past the LDS capacities live in the stream's HBM scratch.
constexpr int kKM = 1024;  // queue tokens held in LDS
constexpr int kKE = 2048;  // their epsilon arcs held in LDS
struct KaldiLds {
  // [kKM] per member one 16-byte record {slot code, cost during the queue (float
  // bits), productive epsilon arcs: offset, count} -- the layout of the first
  // four fields of an HBM member record, so a pop reads a member in one load
  int4* rec;
  int* mcr;    // [kKM] creation index of a token of the emitting pass, -1 for one the queue creates
  int* mord;   // [kKM] order in which the queue creates it (-1: not yet)
  int* v0hi;   // [kKM] initial queue keys: bucket's first creation index
  int* v0lo;   //                            creation index
  int* stk;    // [kKM] the LIFO queue
  int2* adj;   // [kKE] (destination token, arc weight bits)
};
// member record in HBM past kKM: {slot, cost bits, offset, count, creation index, order,
// component label, root rank} (the last two: the component replay)
enum { kMSlot = 0, kMCost = 1, kMOff = 2, kMCnt = 3, kMC = 4, kMOrd = 5, kMComp = 6, kMRoot = 7 };
__device__ __forceinline__ int* km_lds(const KaldiLds& K, int i, int f) {
  switch (f) {
    case kMSlot: return &K.rec[i].x;
    case kMCost: return &K.rec[i].y;
    case kMOff: return &K.rec[i].z;
    case kMCnt: return &K.rec[i].w;
    case kMC: return &K.mcr[i];
    default: return &K.mord[i];
  }
}
__device__ __forceinline__ int km_get(const KaldiLds& K, int* KM, int i, int f) {
  return i < kKM ? *km_lds(K, i, f) : AG_LD(&KM[(long long)(i - kKM) * kKMRec + f]);
}
// a member's {slot, cost, offset, count} in one 16-byte load (LDS or HBM record)
__device__ __forceinline__ int4 km_rec4(const KaldiLds& K, int* KM, int i) {
  return i < kKM ? K.rec[i] : wg_ld4(reinterpret_cast<const int4*>(&KM[(long long)(i - kKM) * kKMRec]));
}
__device__ __forceinline__ void km_set(const KaldiLds& K, int* KM, int i, int f, int v) {
  if (i < kKM) *km_lds(K, i, f) = v;
  else AG_ST(&KM[(long long)(i - kKM) * kKMRec + f], v);
}

// block-wide bitonic sort in LDS (ascending; n <= DT, padded to a power of
// two with the maximum key) of 64-bit keys as (hi, lo) int pairs
__device__ __forceinline__ void bitonic_sort64(int* hi, int* lo, int n) {
  int np = 1;
  while (np < n) np <<= 1;
  for (int i = n + threadIdx.x; i < np; i += DT) {
    hi[i] = 0x7fffffff;
    lo[i] = 0x7fffffff;
  }
  __syncthreads();
  for (int k = 2; k <= np; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      const int i = threadIdx.x, l = i ^ j;
      if (i < np && l > i) {
        const unsigned long long x = ((unsigned long long)(unsigned)hi[i] << 32) | (unsigned)lo[i];
        const unsigned long long y = ((unsigned long long)(unsigned)hi[l] << 32) | (unsigned)lo[l];
        if (((i & k) == 0) ? (x > y) : (x < y)) {
          hi[i] = (int)(y >> 32); lo[i] = (int)(unsigned)y;
          hi[l] = (int)(x >> 32); lo[l] = (int)(unsigned)x;
        }
      }
      __syncthreads();
    }
}

// ProcessNonemitting in Kaldi order.  The frame under construction holds the
// emitting pass's tokens, creation indices [0, ne) (bucket state % khash).
// The epsilon closure itself (final token set, costs, backpointers and the
// links of the final costs) is order-independent, so it runs in parallel
// (eps_closure); the order in which Kaldi's LIFO queue CREATES tokens is
// not, and decides their list positions.  The queue is replayed on one
// thread over LDS-staged data: only tokens that can relax an epsilon arc
// below the cutoff at their final cost matter (at any higher cost they relax
// nothing), with those arcs, plus the tokens the closure created.  Their
// queue costs start at the emitting pass's costs (+inf: not yet created).
// Returns the frame's token count; the created tokens get creation indices
// [ne, count) in the queue's order.
struct KaldiLds;
__device__ __forceinline__ void kaldi_lazy_frame(const DecArgs& a, DecShared& sh, const FrameLds& t, const HbmTab& T,
                                                 const KaldiLds& K, DecSlot& st, int slot, int ne, int n_eps, int khash,
                                                 Prof& pr);
__device__ __forceinline__ int kaldi_nonemitting(const DecArgs& a, DecShared& sh, FrameLds& t, const HbmTab& T,
                                                 const DecPtrs& p, DecSlot& st, const KaldiLds& K, int slot,
                                                 int khash, float cutoff, int ne, int* arcs_eps, Prof& pr) {
  int* KO = a.kord + (long long)slot * a.kord_cap;
  int* KB = a.kbkt + (long long)slot * a.kord_cap;
  int* KS = a.kstk + (long long)slot * a.kord_cap;
  float* KC = a.kcost0 + (long long)slot * a.kord_cap;
  int* KM = a.kmem + (long long)slot * a.kord_cap * kKMRec;
  int2* KA = a.kadj + (long long)slot * a.kadj_cap;
  int* BF = a.kb_first + (long long)slot * a.kb_cap;
  int* BC = a.kb_cnt + (long long)slot * a.kb_cap;
  int* BM = a.kb_memb + (long long)slot * a.kb_cap * kKbMemb;
  const float kInf = __int_as_float(0x7f800000);
  const long long t_nonemit0 = pr.on ? (long long)__builtin_amdgcn_s_memtime() : 0;
  // the emitting pass's tokens: buckets, queue costs, stamps cleared for the
  // closure's rounds, and the closure's first frontier (tokens with epsilon arcs)
  if (threadIdx.x == 0) {
    sh.n_front = 0;
    sh.kn0 = 0;
    sh.kne = 0;
    sh.klazy_ne = ne;
    sh.klazy_k = 0;
    sh.klazy_def = 0;
  }
  __syncthreads();
  // kHlU creation indices per thread at a time, each step's loads (slot,
  // then state / key / flags, then the bucket count) in flight together
  for (int c0 = 0; c0 < ne; c0 += kHlU * DT) {
    int v[kHlU], b[kHlU], m[kHlU];
    unsigned long long key[kHlU];
    bool eps[kHlU];
#pragma unroll
    for (int u = 0; u < kHlU; u++) {
      const int c = c0 + u * DT + (int)threadIdx.x;
      v[u] = c < ne ? AG_LD(&KO[c]) : 0;
    }
#pragma unroll
    for (int u = 0; u < kHlU; u++) {
      const int c = c0 + u * DT + (int)threadIdx.x;
      if (c >= ne) continue;
      const int s = slot_state(t, T, v[u]);
      const int id = kid(a, slot, s);
      b[u] = kbucket_of(id, khash);
      if (a.lazy_id && !(id & kLazyExpanded)) {  // (lazy numbering: a state to expand this frame)
        const int at = atomicAdd(&sh.klazy_k, 1);
        if (at < DT) {
          int* LN = a.lazy_new + (long long)slot * 3 * kLazyNewCap;
          AG_ST(&LN[at], c);
          AG_ST(&LN[kLazyNewCap + at], b[u]);
          AG_ST(&LN[2 * kLazyNewCap + at], s);
        }
      }
      key[u] = slot_key(t, T, v[u]);
      eps[u] = v[u] >= 0 ? (t.hp[v[u]] & kPosEps) != 0 : (AG_LD(&T.pos[~v[u]]) & kHPosEps) != 0;
    }
#pragma unroll
    for (int u = 0; u < kHlU; u++) {
      const int c = c0 + u * DT + (int)threadIdx.x;
      if (c >= ne) continue;
      AG_ST(&KB[c], b[u]);
      __hip_atomic_fetch_min(&BF[b[u]], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      m[u] = __hip_atomic_fetch_add(&BC[b[u]], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      AG_ST(&KC[c], funord((uint32_t)(key[u] >> 32)));
      if (v[u] >= 0) t.hst[v[u]] = kNoStamp;
      else AG_ST(&T.stamp[~v[u]], kNoStamp);
      if (eps[u]) push_front(a, sh, t, p, 0, &sh.n_front, v[u]);
    }
#pragma unroll
    for (int u = 0; u < kHlU; u++) {
      const int c = c0 + u * DT + (int)threadIdx.x;
      if (c < ne && m[u] < kKbMemb) AG_ST(&BM[kKbMemb * b[u] + m[u]], c);
    }
  }
  vm_drain();
  __syncthreads();
  const int nl_e = sh.n_new_l, ng_e = sh.n_new_g;
  pr.mark(47);
  eps_closure(a, sh, t, T, p, st, cutoff, sh.n_front, arcs_eps, pr);
  __syncthreads();
  pr.mark(5);
  const int nl_n = sh.n_new_l, ng = sh.n_new_g < a.max_tok ? sh.n_new_g : a.max_tok;
  const int n_eps = (nl_n - nl_e) + (ng - ng_e);
  // an overflow (unlisted HBM entries, creation indices past kord_cap): no
  // replay, the commit stores nothing (sh.bad is uniform after the barrier)
  if (sh.bad || ng_e > a.max_tok || n_eps < 0 || ne + n_eps > a.kord_cap) {
    __syncthreads();
    if (threadIdx.x == 0) sh.bad |= 1;
    __syncthreads();
    return ne;
  }
  if (n_eps <= 1) {  // the creation order is the closure's (none or one)
    if (n_eps == 1 && threadIdx.x == 0) {
      const int v = nl_n > nl_e ? (int)t.nl[nl_e] : ~AG_LD(&T.list[ng_e]);
      AG_ST(&KO[ne], v);
      if (!a.lazy_id) {
        const int b = kbucket(a, slot, slot_state(t, T, v), khash);
        AG_ST(&KB[ne], b);
        if (AG_LD(&BF[b]) > ne) AG_ST(&BF[b], ne);
        const int m = AG_LD(&BC[b]);
        AG_ST(&BC[b], m + 1);
        if (m < kKbMemb) AG_ST(&BM[kKbMemb * b + m], ne);
      }
    }
    vm_drain();
    __syncthreads();
    if (a.lazy_id) kaldi_lazy_frame(a, sh, t, T, K, st, slot, ne, n_eps, khash, pr);
    return ne + n_eps;
  }
  // every entry's stamp cleared, then the queue's tokens numbered: tokens of
  // the emitting pass that can relax an epsilon arc below the cutoff at
  // their final cost, and every token the closure created
  for (int j = threadIdx.x; j < nl_n + ng; j += DT) {
    const int v = j < nl_n ? (int)t.nl[j] : ~AG_LD(&T.list[j - nl_n]);
    if (v >= 0) t.hst[v] = kNoStamp;
    else AG_ST(&T.stamp[~v], kNoStamp);
  }
  vm_drain();
  __syncthreads();
  const int cap_m = kKM + a.kord_cap;
  for (int j = threadIdx.x; j < ne + n_eps; j += DT) {
    int v, c;
    if (j < ne) {
      c = j;
      v = AG_LD(&KO[c]);
      const bool eps = v >= 0 ? (t.hp[v] & kPosEps) != 0 : (AG_LD(&T.pos[~v]) & kHPosEps) != 0;
      if (!eps) continue;
    } else {
      const int q = j - ne;  // the closure's q-th created entry
      c = -1;
      v = q < nl_n - nl_e ? (int)t.nl[nl_e + q] : ~AG_LD(&T.list[ng_e + q - (nl_n - nl_e)]);
    }
    const float fc = funord((uint32_t)(slot_key(t, T, v) >> 32));
    const int4 si = a.sinfo[slot_state(t, T, v)];
    const float c0 = c >= 0 ? AG_LD(&KC[c]) : kInf;
    // one walk over the epsilon arcs: the productive ones at the final cost,
    // and whether one is productive at the emitting cost (c0 >= fc)
    int cnt = 0;
    bool prod = false;
    if (fc < cutoff)
      for (int arc = si.y; arc < si.z; arc++) {
        const float w = __int_as_float(a.arcs[arc].y);
        cnt += fc + w < cutoff;
        prod = prod || c0 + w < cutoff;
      }
    if (c >= 0 && cnt == 0) continue;  // relaxes nothing at any cost: not a queue token
    const int i = atomicAdd(&sh.kne, 1);
    if (i >= cap_m) {
      sh.bad |= 1;
      continue;
    }
    if (v >= 0) t.hst[v] = i;
    else AG_ST(&T.stamp[~v], i);
    km_set(K, KM, i, kMSlot, v);
    km_set(K, KM, i, kMCost, __float_as_int(c0));
    km_set(K, KM, i, kMCnt, cnt);
    km_set(K, KM, i, kMC, c);
    km_set(K, KM, i, kMOrd, -1);
    // Kaldi's initial queue: a token of the emitting pass that relaxes an
    // arc below the cutoff at its emitting cost, keyed by its list order
    if (c >= 0 && c0 < cutoff) {
      if (prod) {
        const int q = atomicAdd(&sh.kn0, 1);
        if (q < kKM) {
          K.v0hi[q] = AG_LD(&BF[AG_LD(&KB[c])]);
          K.v0lo[q] = c;
        } else {
          reinterpret_cast<unsigned long long*>(p.fg0)[q - kKM] =
              ((unsigned long long)(unsigned)AG_LD(&BF[AG_LD(&KB[c])]) << 32) | (unsigned)c;
        }
      }
    }
  }
  vm_drain();
  __syncthreads();
  const int nm = sh.kne < cap_m ? sh.kne : cap_m;
  long long t_lanes = 0;  // (profile) replay clocks of this frame
  const int n0 = sh.kn0 < nm ? sh.kn0 : nm;
  // adjacency offsets (a scan over the members), then each member's
  // productive arcs in graph order: (destination member or -1, weight)
  {
    int run = 0, par = 0;
    for (int i0 = 0; i0 < nm; i0 += DT) {
      const int i = i0 + threadIdx.x;
      const int cnt = i < nm ? km_get(K, KM, i, kMCnt) : 0;
      int tot;
      const int off = run + kaldi_excl_sum(sh, cnt, par, &tot);
      if (i < nm) km_set(K, KM, i, kMOff, off);
      run += tot;
      par ^= 1;
    }
    if (run > kKE + a.kadj_cap && threadIdx.x == 0) sh.bad |= 1;
  }
  vm_drain();
  __syncthreads();
  for (int i = threadIdx.x; i < nm; i += DT) {
    const int cnt = km_get(K, KM, i, kMCnt);
    if (cnt == 0) continue;
    const int off = km_get(K, KM, i, kMOff);
    const int v = km_get(K, KM, i, kMSlot);
    const float fc = funord((uint32_t)(slot_key(t, T, v) >> 32));
    const int4 si = a.sinfo[slot_state(t, T, v)];
    int k = 0;
    for (int arc = si.y; arc < si.z; arc++) {
      const int4 A = a.arcs[arc];
      if (!(fc + __int_as_float(A.y) < cutoff)) continue;
      const int dv = frame_slot(a, t, T, A.x);
      int d = -1;
      if (dv != kNoSlot) {
        const int h = dv >= 0 ? t.hst[dv] : AG_LD(&T.stamp[~dv]);
        d = h == kNoStamp ? -1 : h;
      }
      const int e = off + k++;
      const int2 rec = make_int2(d, A.y);
      if (e < kKE) K.adj[e] = rec;
      else if (e - kKE < a.kadj_cap) {
        AG_ST(&reinterpret_cast<long long*>(KA)[e - kKE],
              (long long)(((unsigned long long)(unsigned)rec.y << 32) | (unsigned)rec.x));
      }
    }
  }
  pr.mark(24);
  // the initial queue in list order: sorted in LDS when it fits; else
  // chunks of kKM sorted in LDS into the frontier scratch (after the keys
  // past kKM already there), each key ranked by its chunk index plus a binary
  // search in every other chunk (keys are unique: creation index); ranked by
  // counting when the scratch is too small
  long long* const SK = reinterpret_cast<long long*>(p.fg0);  // [max_tok] 8-byte entries over fg0, fg1
  if (n0 <= kKM) {
    bitonic_sort64(K.v0hi, K.v0lo, n0);
    for (int r = threadIdx.x; r < n0; r += DT) {
      const int v = AG_LD(&KO[K.v0lo[r]]);
      K.stk[r] = v >= 0 ? t.hst[v] : AG_LD(&T.stamp[~v]);
    }
  } else if (2 * n0 - kKM <= a.max_tok) {
    long long* const S = SK + (n0 - kKM);  // sorted chunks
    const int nch = (n0 + kKM - 1) / kKM;
    for (int ch = 0; ch < nch; ch++) {
      const int c0 = ch * kKM, len = n0 - c0 < kKM ? n0 - c0 : kKM;
      if (ch > 0) {
        for (int r = threadIdx.x; r < len; r += DT) {
          const unsigned long long k = (unsigned long long)AG_LD(&SK[c0 + r - kKM]);
          K.v0hi[r] = (int)(unsigned)(k >> 32);
          K.v0lo[r] = (int)(unsigned)k;
        }
        vm_drain();
        __syncthreads();
      }
      bitonic_sort64(K.v0hi, K.v0lo, len);
      for (int r = threadIdx.x; r < len; r += DT)
        AG_ST(&S[c0 + r], (long long)(((unsigned long long)(unsigned)K.v0hi[r] << 32) | (unsigned)K.v0lo[r]));
      vm_drain();
      __syncthreads();
    }
    for (int x = threadIdx.x; x < n0; x += DT) {
      const unsigned long long kx = (unsigned long long)AG_LD(&S[x]);
      const int own = x / kKM;
      int r = x - own * kKM;
      for (int ch = 0; ch < nch; ch++) {
        if (ch == own) continue;
        int lo = ch * kKM, hi = lo + (n0 - lo < kKM ? n0 - lo : kKM);
        const int first = lo;
        while (lo < hi) {  // first entry of the chunk not below kx
          const int mid = (lo + hi) >> 1;
          if ((unsigned long long)AG_LD(&S[mid]) < kx) lo = mid + 1;
          else hi = mid;
        }
        r += lo - first;
      }
      const int c = (int)(unsigned)(kx & 0xffffffffu);
      const int v = AG_LD(&KO[c]);
      const int i = v >= 0 ? t.hst[v] : AG_LD(&T.stamp[~v]);
      if (r < kKM) K.stk[r] = i;
      else AG_ST(&KS[r - kKM], i);
    }
  } else
  for (int q = threadIdx.x; q < n0; q += DT) {
    auto key = [&](int r) -> unsigned long long {
      if (r < kKM) return ((unsigned long long)(unsigned)K.v0hi[r] << 32) | (unsigned)K.v0lo[r];
      return reinterpret_cast<unsigned long long*>(p.fg0)[r - kKM];
    };
    const unsigned long long kq = key(q);
    int r = 0;
    for (int j = 0; j < n0; j++) r += key(j) < kq;
    // the member of creation index c: its stamp
    const int c = (int)(unsigned)(kq & 0xffffffffu);
    const int v = AG_LD(&KO[c]);
    const int i = v >= 0 ? t.hst[v] : AG_LD(&T.stamp[~v]);
    if (r < kKM) K.stk[r] = i;
    else AG_ST(&KS[r - kKM], i);
  }
  vm_drain();
  __syncthreads();
  pr.mark(25);
  // the LIFO queue (pop_back), one thread, over the staged tokens: LDS only
  // when everything fits (the common case), else through the HBM records
  int adj_n = 0;
  if (nm > 0) adj_n = km_get(K, KM, nm - 1, kMOff) + km_get(K, KM, nm - 1, kMCnt);
  const bool fast = nm <= kKM && adj_n <= kKE && n0 <= kKM && !(a.debug & 4);
  // Component-parallel replay.  The LIFO queue processes the initial tokens
  // from the top (the last in list order first), each one's pushes before the
  // next initial token; a token's expansion only touches tokens connected
  // to it through productive epsilon arcs.  So the queue restricted to one
  // connected component of those arcs is the queue of that component's own
  // initial tokens, in the same order, and the components replay
  // independently, one lane each: the creation order is by initial token
  // (processing rank), then by creation within its expansion.  A component
  // whose stack outgrows the lane's eight registers, or labels that do not
  // settle, send the frame to the sequential replay below.
  bool replayed = false;
  if (n0 <= a.max_tok && nm < (1 << 22) && !(a.debug & (8 | 16))) {
    // members past kKM keep their component label and root in the HBM
    // record (fields kMComp, kMRoot), their arcs past kKE in the HBM adjacency
    int* comp = K.v0lo;    // members < kKM (the sort keys are consumed)
    unsigned* key = reinterpret_cast<unsigned*>(K.v0hi);
    int* mroot = sh.tsrc;  // members < kKM
    const float kInfL = __int_as_float(0x7f800000);
    auto rec_at = [&](int i, int f) -> int* { return &KM[(long long)(i - kKM) * kKMRec + f]; };
    auto cget = [&](int i) -> int { return i < kKM ? comp[i] : AG_LD(rec_at(i, kMComp)); };
    auto rget = [&](int i) -> int { return i < kKM ? mroot[i] : AG_LD(rec_at(i, kMRoot)); };
    auto rset = [&](int i, int v) {
      if (i < kKM) mroot[i] = v;
      else AG_ST(rec_at(i, kMRoot), v);
    };
    auto adj_at = [&](int e) -> int2 {
      if (e < kKE) return K.adj[e];
      const unsigned long long w = (unsigned long long)AG_LD(&reinterpret_cast<long long*>(KA)[e - kKE]);
      return make_int2((int)(unsigned)w, (int)(unsigned)(w >> 32));
    };
    for (int i = threadIdx.x; i < nm; i += DT) {
      if (i < kKM) comp[i] = i;
      else AG_ST(rec_at(i, kMComp), i);
    }
    if (threadIdx.x == 0) {
      sh.flag = 0;
      sh.kpop_sum = 0;
      sh.kpop_max = 0;
      sh.kcomp_n = 0;
      sh.kcomp_max = 0;
      sh.kcomp_clk = 0;
      sh.karc_sum = 0;
      sh.karc_max = 0;
      sh.khbm_pops = 0;
    }
    vm_drain();
    __syncthreads();
    // connected components: minimum member index, propagated along the arcs
    bool settled = false;
    for (int it = 0; it < 64 && !settled; it++) {
      if (threadIdx.x == 0) sh.kk = 0;
      __syncthreads();
      for (int u = threadIdx.x; u < nm; u += DT) {
        const int e0 = km_get(K, KM, u, kMOff), e1 = e0 + km_get(K, KM, u, kMCnt);
        for (int e = e0; e < e1; e++) {
          const int d = adj_at(e).x;
          if (d < 0) continue;
          const int cu = cget(u), cd = cget(d), m = cu < cd ? cu : cd;
          if (cu > m) {
            if (u < kKM) atomicMin(&comp[u], m);
            else __hip_atomic_fetch_min(rec_at(u, kMComp), m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sh.kk = 1;
          }
          if (cd > m) {
            if (d < kKM) atomicMin(&comp[d], m);
            else __hip_atomic_fetch_min(rec_at(d, kMComp), m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sh.kk = 1;
          }
        }
      }
      vm_drain();
      __syncthreads();
      settled = sh.kk == 0;
      __syncthreads();
      pr.count(36, 1);
    }
    pr.mark(34);
    pr.count(40, settled ? 0 : 1);
    if (settled) {
      // the component of the initial token of each processing rank q (the
      // initial token of rank q is the queue entry n0 - 1 - q: the top of
      // the LIFO first), in the frontier scratch (free after the closure)
      int* CQ = p.fg1;
      auto stk_at = [&](int r) -> int { return r < kKM ? K.stk[r] : AG_LD(&KS[r - kKM]); };
      // Hot-first renumbering when the members overflow the LDS records:
      // members of components with two or more initial tokens -- the ones
      // the waves replay pop by pop -- move to the low (LDS) indices;
      // single-token components replay one per lane, their HBM records'
      // latency overlapped across lanes.  Records, adjacency destinations,
      // the initial queue and the slots' member stamps are rewritten; the
      // component labels stay (they are only ids from here on).
      if (nm > kKM && nm <= a.max_tok && 2LL * nm - kKM <= (long long)a.kord_cap) {
        int* CC = p.fg0;       // [nm] initial tokens per component label (fg0..fg1: 2 * max_tok ints)
        int* NI = p.fg0 + nm;  // [nm] new index of each member
        int* TM = KM + (long long)(nm - kKM) * kKMRec;  // [nm] record copies, past the records in use
        auto cset = [&](int i, int v) {
          if (i < kKM) comp[i] = v;
          else AG_ST(rec_at(i, kMComp), v);
        };
        for (int i = threadIdx.x; i < nm; i += DT) AG_ST(&CC[i], 0);
        vm_drain();
        __syncthreads();
        for (int q = threadIdx.x; q < n0; q += DT)
          __hip_atomic_fetch_add(&CC[cget(stk_at(q))], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        vm_drain();
        __syncthreads();
        int hot_n = 0;
        for (int pass = 0; pass < 2; pass++) {  // hot members, then the rest, each in member order
          int run = pass == 0 ? 0 : hot_n, par = 0;
          for (int i0 = 0; i0 < nm; i0 += DT) {
            const int i = i0 + threadIdx.x;
            const bool hot = i < nm && AG_LD(&CC[cget(i)]) >= 2;
            const bool take = i < nm && (pass == 0 ? hot : !hot);
            int tot;
            const int ex = run + kaldi_excl_sum(sh, take ? 1 : 0, par, &tot);
            if (take) AG_ST(&NI[i], ex);
            run += tot;
            par ^= 1;
          }
          if (pass == 0) hot_n = run;
        }
        vm_drain();
        __syncthreads();
        if (hot_n > 0) {
          for (int i = threadIdx.x; i < nm; i += DT) {
            for (int f = kMSlot; f <= kMOrd; f++) AG_ST(&TM[(long long)i * kKMRec + f], km_get(K, KM, i, f));
            AG_ST(&TM[(long long)i * kKMRec + kMComp], cget(i));
          }
          vm_drain();
          __syncthreads();
          for (int i = threadIdx.x; i < nm; i += DT) {
            const int j = AG_LD(&NI[i]);
            for (int f = kMSlot; f <= kMOrd; f++) km_set(K, KM, j, f, AG_LD(&TM[(long long)i * kKMRec + f]));
            cset(j, AG_LD(&TM[(long long)i * kKMRec + kMComp]));
          }
          for (int e = threadIdx.x; e < adj_n; e += DT) {
            int2 rec = adj_at(e);
            if (rec.x < 0) continue;
            rec.x = AG_LD(&NI[rec.x]);
            if (e < kKE) K.adj[e] = rec;
            else
              AG_ST(&reinterpret_cast<long long*>(KA)[e - kKE],
                    (long long)(((unsigned long long)(unsigned)rec.y << 32) | (unsigned)rec.x));
          }
          for (int r = threadIdx.x; r < n0; r += DT) {
            const int j = AG_LD(&NI[stk_at(r)]);
            if (r < kKM) K.stk[r] = j;
            else AG_ST(&KS[r - kKM], j);
          }
          vm_drain();
          __syncthreads();
          for (int j = threadIdx.x; j < nm; j += DT) {  // slot -> member stamps (the sequential fallback reads them)
            const int v = km_get(K, KM, j, kMSlot);
            if (v >= 0) t.hst[v] = j;
            else AG_ST(&T.stamp[~v], j);
          }
          vm_drain();
          __syncthreads();
        }
        pr.count(57, hot_n);
        pr.count(58, 1);
      }
      for (int q = threadIdx.x; q < n0; q += DT) AG_ST(&CQ[q], cget(stk_at(n0 - 1 - q)));
      vm_drain();
      __syncthreads();
      for (int i = threadIdx.x; i < nm; i += DT) rset(i, -1);
      vm_drain();
      __syncthreads();
      // segments of kKM processing ranks in order: the queue restricted to a
      // segment starts from the costs the earlier segments left
      // the segments' replay, specialised for frames whose members and arcs
      // all fit the LDS records (no HBM address branches in the pop loops)
      auto replay_segments = [&](auto lds_only) -> int {
        constexpr bool L = decltype(lds_only)::value;
        auto rec4 = [&](int i) -> int4 {
          return (L || i < kKM) ? K.rec[i] : wg_ld4(reinterpret_cast<const int4*>(rec_at(i, 0)));
        };
        auto setf = [&](int i, int f, int v) {
          if (L || i < kKM) *km_lds(K, i, f) = v;
          else AG_ST(rec_at(i, f), v);
        };
        auto getf = [&](int i, int f) -> int { return (L || i < kKM) ? *km_lds(K, i, f) : AG_LD(rec_at(i, f)); };
        auto adj = [&](int e) -> int2 { return (L || e < kKE) ? K.adj[e] : adj_at(e); };
        auto rootg = [&](int i) -> int { return (L || i < kKM) ? mroot[i] : AG_LD(rec_at(i, kMRoot)); };
        auto roots = [&](int i, int v) {
          if (L || i < kKM) mroot[i] = v;
          else AG_ST(rec_at(i, kMRoot), v);
        };
        auto stk2 = [&](int r) -> int { return (L || r < kKM) ? K.stk[r] : AG_LD(&KS[r - kKM]); };
        int created_total = 0;
        for (int base = 0; base < n0 && sh.flag == 0; base += kKM) {
          const int ns = n0 - base < kKM ? n0 - base : kKM;
          // the segment's component labels by processing rank (one rank per
          // thread: ns <= kKM = DT); the ranks of each component are counted
          // in its label member's root field (-1 + count; the field is -1
          // between replays), and a component's second rank lists it for the
          // waves (past 256 heads: in the frontier scratch, free here)
          static_assert(kKM <= DT, "one processing rank per thread");
          int* HL = p.fg0;
          if (threadIdx.x == 0) sh.kheads = 0;
          int myc = -1, before = 0;
          if ((int)threadIdx.x < ns) {
            myc = AG_LD(&CQ[base + threadIdx.x]);
            key[threadIdx.x] = (unsigned)myc;
          }
          __syncthreads();
          if (myc >= 0) {
            before = (L || myc < kKM) ? atomicAdd(&mroot[myc], 1)
                               : __hip_atomic_fetch_add(rec_at(myc, kMRoot), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (before == 0) {
              const int q = atomicAdd(&sh.kheads, 1);
              if (q < 256) sh.hist[q] = (unsigned)myc;
              else AG_ST(&HL[q - 256], myc);
            }
          }
          vm_drain();
          __syncthreads();
          const bool single = myc >= 0 && rootg(myc) == 0;
          vm_drain();
          __syncthreads();
          if (before == -1) roots(myc, -1);  // the component's first rank restores the field
          vm_drain();
          __syncthreads();
          pr.mark(41);
          const long long t_l0 = pr.on ? (long long)__builtin_amdgcn_s_memtime() : 0;
          // Components with a single initial token in this segment (most of
          // them) replay one per lane, all at once: the same pops and arc
          // order as the wave form below, the lane's LIFO in a four-deep shift
          // register (a deeper queue sends the frame to the sequential replay).
          // Components are disjoint, so the lanes never touch the same member.
          {
            if (single) {
              const int prank = (int)threadIdx.x;
              int s0 = stk2(n0 - 1 - (base + prank)), s1 = 0, s2 = 0, s3 = 0;
              int sp = 1, j = 0, np = 0;
              bool lovf = false;
              while (sp > 0) {
                const int u = s0;  // pop
                s0 = s1;
                s1 = s2;
                s2 = s3;
                sp--;
                np++;
                const int4 ur = rec4(u);  // (one read: no branch before its fields' uses)
                const float cu = __int_as_float(ur.y);
                const int off = ur.z, cnt = ur.w & -(int)(cu < cutoff);
                // arcs four at a time: their records, then their destinations'
                // records, in flight together; applied in arc order (a later
                // arc of the group to the same token sees the new cost)
                for (int k0 = 0; k0 < cnt && !lovf; k0 += 4) {
                  int2 r4[4];
                  int4 d4[4];
  #pragma unroll
                  for (int m = 0; m < 4; m++) r4[m] = k0 + m < cnt ? adj(off + k0 + m) : make_int2(-1, 0);
  #pragma unroll
                  for (int m = 0; m < 4; m++)
                    d4[m] = r4[m].x >= 0 ? rec4(r4[m].x) : make_int4(0, 0, 0, 0);
  #pragma unroll
                  for (int m = 0; m < 4; m++) {
                    const int d = r4[m].x;
                    if (d < 0 || lovf) continue;
                    const float tot = cu + __int_as_float(r4[m].y);
                    if (!(tot < cutoff)) continue;
                    const float old = __int_as_float(d4[m].y);
                    if (!(tot < old)) continue;
  #pragma unroll
                    for (int m2 = m + 1; m2 < 4; m2++)
                      if (r4[m2].x == d) d4[m2].y = __float_as_int(tot);
                    if (old == kInfL) {  // FindOrAddToken creates it
                      setf(d, kMOrd, j++);
                      roots(d, prank);
                    }
                    setf(d, kMCost, __float_as_int(tot));
                    if (d4[m].w > 0) {  // changed: re-queued
                      if (sp == 4) {
                        lovf = true;
                        continue;
                      }
                      s3 = s2;  // push
                      s2 = s1;
                      s1 = s0;
                      s0 = d;
                      sp++;
                    }
                  }
                }
                if (lovf) break;
              }
              K.v0lo[prank] = j;
              if (lovf) sh.flag = 1;
              atomicAdd(&sh.kpop_sum, np);
            }
          }
          // one wave per multi-token component, claimed from the list.  A popped
          // token's arcs are read by the wave's lanes together (records, then
          // the destinations' costs and arc counts), then applied in arc order
          // (v_readlane; a later arc to the same token sees the new cost); the
          // LIFO stack lives one entry per lane (depth 64).  A rank's creation
          // count goes to K.v0lo[rank - base] (the labels were consumed into CQ).
          const int lane = threadIdx.x & 63;
          if (threadIdx.x == 0) sh.kk = 0;
          __syncthreads();
          if (pr.on) {  // the lane phase (all lanes done at the barrier)
            pr.count(59, (long long)__builtin_amdgcn_s_memtime() - t_l0);
            pr.count(60, 1);
          }
          int npop = 0, narc = 0, nhbm = 0;
          bool ovf = false;
          // the multi-token components, one claim each from the list; a
          // component's ranks in processing order by a ballot over the labels
          const int nheads = sh.kheads;
          while (!ovf) {
            int c0 = 0;
            if (lane == 0) c0 = atomicAdd(&sh.kk, 1);
            c0 = __builtin_amdgcn_readfirstlane(c0);
            if (c0 >= nheads) break;
            // (LDS values the whole wave reads are made scalar: branching on
            // them would otherwise make the replay loop divergent, every
            // v_readlane a waterfall loop)
            const int cmp = __builtin_amdgcn_readfirstlane(c0 < 256 ? (int)sh.hist[c0] : AG_LD(&HL[c0 - 256]));
            const int npop0 = npop;
            const long long tc0 = (long long)__builtin_amdgcn_s_memtime();
            for (int ch = 0; ch < ns && !ovf; ch += 64) {
              unsigned long long rm = __ballot(ch + lane < ns && (int)key[ch + lane] == cmp);
              while (rm && !ovf) {
                const int prank = ch + __ffsll((long long)rm) - 1;
                rm &= rm - 1;
                int stk = lane == 0 ? stk2(n0 - 1 - (base + prank)) : 0;
                int sp = 1, j = 0;
                while (sp > 0 && !ovf) {
                  --sp;
                  npop++;
                  const int u = __builtin_amdgcn_readlane(stk, sp);
                  // cost, offset and count in one load: no branch between
                  // them (a token at or above the cutoff relaxes no arc), so
                  // the compiler does not split the record into two reads
                  const int4 ur = rec4(u);
                  const float cu = __int_as_float(__builtin_amdgcn_readfirstlane(ur.y));
                  const int off = __builtin_amdgcn_readfirstlane(ur.z);
                  const int cnt = __builtin_amdgcn_readfirstlane(ur.w) & -(int)(cu < cutoff);
                  narc += cnt;
                  if (!L && u >= kKM && cnt > 0) nhbm++;
                  if (cnt == 1) {
                    // one productive arc (most pops): the same steps with
                    // wave-uniform values only -- no per-lane arc and
                    // destination reads, no v_readlane extraction
                    const int2 r1 = adj(off);
                    const int d = __builtin_amdgcn_readfirstlane(r1.x);
                    if (d < 0) continue;
                    const float tot = cu + __int_as_float(__builtin_amdgcn_readfirstlane(r1.y));
                    if (!(tot < cutoff)) continue;
                    const int4 dr = rec4(d);
                    const float old = __int_as_float(__builtin_amdgcn_readfirstlane(dr.y));
                    if (!(tot < old)) continue;
                    if (lane == 0) {
                      if (old == kInfL) {  // FindOrAddToken creates it
                        setf(d, kMOrd, j);
                        roots(d, prank);
                      }
                      setf(d, kMCost, __float_as_int(tot));
                    }
                    if (old == kInfL) j++;
                    if (__builtin_amdgcn_readfirstlane(dr.w) > 0) {  // changed: re-queued
                      if (sp == 64) {
                        ovf = true;
                        continue;
                      }
                      if (lane == sp) stk = d;
                      sp++;
                    }
                    continue;
                  }
                  for (int k0 = 0; k0 < cnt && !ovf; k0 += 64) {
                    const int kn = cnt - k0 < 64 ? cnt - k0 : 64;
                    const int2 rec = lane < kn ? adj(off + k0 + lane) : make_int2(-1, 0);
                    int oldl = __float_as_int(kInfL), cntl = 0;
                    if (rec.x >= 0) {
                      const int4 dr = rec4(rec.x);
                      oldl = dr.y;
                      cntl = dr.w;
                    }
                    for (int k = 0; k < kn; k++) {
                      const int d = __builtin_amdgcn_readlane(rec.x, k);
                      if (d < 0) continue;
                      const float tot = cu + __int_as_float(__builtin_amdgcn_readlane(rec.y, k));
                      if (!(tot < cutoff)) continue;
                      const float old = __int_as_float(__builtin_amdgcn_readlane(oldl, k));
                      if (!(tot < old)) continue;
                      if (rec.x == d) oldl = __float_as_int(tot);
                      if (lane == k) {
                        if (old == kInfL) {  // FindOrAddToken creates it
                          setf(d, kMOrd, j);
                          roots(d, prank);
                        }
                        setf(d, kMCost, __float_as_int(tot));
                      }
                      if (old == kInfL) j++;
                      if (__builtin_amdgcn_readlane(cntl, k) > 0) {  // changed: re-queued
                        if (sp == 64) {
                          ovf = true;
                          break;
                        }
                        if (lane == sp) stk = d;
                        sp++;
                      }
                    }
                  }
                }
                if (lane == 0) K.v0lo[prank] = j;
              }
            }
            if (lane == 0) {
              atomicAdd(&sh.kcomp_n, 1);
              atomicMax(&sh.kcomp_max, npop - npop0);
              atomicMax(&sh.kcomp_clk, (int)((long long)__builtin_amdgcn_s_memtime() - tc0));
            }
          }
          if (lane == 0 && npop > 0) {
            atomicAdd(&sh.karc_sum, narc);
            atomicMax(&sh.karc_max, narc);
            atomicAdd(&sh.khbm_pops, nhbm);
          }
          if (lane == 0) {
            if (ovf) sh.flag = 1;
            if (npop > 0) {
              atomicAdd(&sh.kpop_sum, npop);
              atomicMax(&sh.kpop_max, npop);
            }
          }
          vm_drain();
          __syncthreads();
          pr.mark(42);
          if (pr.on) t_lanes += (long long)__builtin_amdgcn_s_memtime() - t_l0;
          if (sh.flag == 0) {
            // creations per initial token in processing order, then the global
            // creation order = (earlier segments) + (rank offset) + creation
            // within the rank's expansion
            int tot;
            const int c = threadIdx.x < ns ? K.v0lo[threadIdx.x] : 0;
            const int ex = kaldi_excl_sum(sh, c, 0, &tot);
            __syncthreads();
            if (threadIdx.x < ns) K.v0lo[threadIdx.x] = ex;
            __syncthreads();
            for (int m = threadIdx.x; m < nm; m += DT) {
              const int r = rootg(m);
              if (r < 0) continue;
              setf(m, kMOrd, getf(m, kMOrd) + created_total + K.v0lo[r]);
              roots(m, -1);
            }
            created_total += tot;
            vm_drain();
            __syncthreads();
          }
        }
        return created_total;
      };
      const int created_total = (nm <= kKM && adj_n <= kKE) ? replay_segments(std::true_type{})
                                                            : replay_segments(std::false_type{});
      if (sh.flag == 0) {
        if (threadIdx.x == 0) sh.kn0 = created_total;
        __syncthreads();
        replayed = true;
      }
    }
    if (!replayed) {  // back to the sequential replay: the members' queue state reset
      for (int m = threadIdx.x; m < nm; m += DT) {
        const int c = km_get(K, KM, m, kMC);
        km_set(K, KM, m, kMCost, __float_as_int(c >= 0 ? AG_LD(&KC[c]) : kInfL));
        km_set(K, KM, m, kMOrd, -1);
      }
      // the initial queue's sort keys again (consumed; K.stk / KS are intact)
      vm_drain();
      __syncthreads();
      if (threadIdx.x == 0) sh.kn0 = 0;
      __syncthreads();
      for (int m = threadIdx.x; m < nm && n0 <= kKM; m += DT) {
        const int c = km_get(K, KM, m, kMC);
        if (c < 0) continue;
        const float c0 = AG_LD(&KC[c]);
        if (!(c0 < cutoff)) continue;
        const int v = km_get(K, KM, m, kMSlot);
        const int4 si = a.sinfo[slot_state(t, T, v)];
        bool prod = false;
        for (int arc = si.y; arc < si.z && !prod; arc++) prod = c0 + __int_as_float(a.arcs[arc].y) < cutoff;
        if (!prod) continue;
        const int q = atomicAdd(&sh.kn0, 1);
        K.v0hi[q] = AG_LD(&BF[AG_LD(&KB[c])]);
        K.v0lo[q] = c;
      }
      vm_drain();
      __syncthreads();
      if (n0 <= kKM) bitonic_sort64(K.v0hi, K.v0lo, n0);
      if (threadIdx.x == 0) sh.kn0 = n0;
      __syncthreads();
    }
  }
  pr.mark(35);
  pr.count(37, n0);
  pr.count(38, n0 > kKM ? 1 : 0);
  pr.count(39, (n0 <= kKM && !replayed && sh.flag) ? 1 : 0);
  if (replayed) {
  } else if (a.debug & 8) {  // development timing only: no replay (creation order = member order; wrong lists)
    for (int i = threadIdx.x; i < nm; i += DT) K.mord[i] = -1;
    if (threadIdx.x == 0) {
      int created = 0;
      for (int i = 0; i < nm; i++)
        if (K.mcr[i] < 0) K.mord[i] = created++;
      sh.kn0 = created;
    }
  } else if (fast && nm <= 256 && threadIdx.x < 64) {
    // up to 256 tokens: wave 0 keeps their queue costs and counts in
    // registers (token i: lane i & 63, register i >> 6) and the queue in two
    // registers (depth 128); token and arc indices are wave-uniform, so every
    // read is a v_readlane and every write a lane select (a ds_bpermute
    // shuffle costs an LDS round trip); the arcs of a popped token are read by its lanes
    // together.  Plain register variables: an indexed register array would
    // live in scratch memory.
    const int lane = threadIdx.x;
    int c0 = __float_as_int(kInf), c1 = c0, c2 = c0, c3 = c0;
    int n0r = 0, n1r = 0, n2r = 0, n3r = 0, o0 = 0, o1 = 0, o2 = 0, o3 = 0, d0 = -1, d1 = -1, d2 = -1, d3 = -1;
    if (lane < nm) { c0 = __float_as_int((*reinterpret_cast<float*>(&K.rec[lane].y))); n0r = K.rec[lane].w; o0 = K.rec[lane].z; }
    if (lane + 64 < nm) { c1 = __float_as_int((*reinterpret_cast<float*>(&K.rec[lane + 64].y))); n1r = K.rec[lane + 64].w; o1 = K.rec[lane + 64].z; }
    if (lane + 128 < nm) { c2 = __float_as_int((*reinterpret_cast<float*>(&K.rec[lane + 128].y))); n2r = K.rec[lane + 128].w; o2 = K.rec[lane + 128].z; }
    if (lane + 192 < nm) { c3 = __float_as_int((*reinterpret_cast<float*>(&K.rec[lane + 192].y))); n3r = K.rec[lane + 192].w; o3 = K.rec[lane + 192].z; }
    int q0 = lane < n0 ? K.stk[lane] : 0, q1 = lane + 64 < n0 ? K.stk[lane + 64] : 0;
#define KSEL(r, a0, a1, a2, a3) ((r) == 0 ? (a0) : (r) == 1 ? (a1) : (r) == 2 ? (a2) : (a3))
#define KRD(r, i, a0, a1, a2, a3) __builtin_amdgcn_readlane(KSEL(r, a0, a1, a2, a3), (i))
    int sp = n0 < 128 ? n0 : 128, created = 0;
    bool ovf = n0 > 128;
    while (sp > 0 && !ovf) {
      --sp;
      const int u = sp < 64 ? __builtin_amdgcn_readlane(q0, sp) : __builtin_amdgcn_readlane(q1, sp - 64);
      const int ur = u >> 6, ul = u & 63;
      const float cu = __int_as_float(KRD(ur, ul, c0, c1, c2, c3));
      if (!(cu < cutoff)) continue;
      const int cnt = KRD(ur, ul, n0r, n1r, n2r, n3r), off = KRD(ur, ul, o0, o1, o2, o3);
      for (int k0 = 0; k0 < cnt && !ovf; k0 += 64) {
        const int2 rec = lane < cnt - k0 ? K.adj[off + k0 + lane] : make_int2(-1, 0);
        const int kn = cnt - k0 < 64 ? cnt - k0 : 64;
        for (int k = 0; k < kn; k++) {
          const int d = __builtin_amdgcn_readlane(rec.x, k);
          const float tot = cu + __int_as_float(__builtin_amdgcn_readlane(rec.y, k));
          if (d < 0 || !(tot < cutoff)) continue;  // (d < 0: a token of the emitting pass that relaxes nothing)
          const int dr = d >> 6, dl = d & 63;
          const float old = __int_as_float(KRD(dr, dl, c0, c1, c2, c3));
          if (!(tot < old)) continue;
          const int tb = __float_as_int(tot);
          if (dr == 0) c0 = (lane == (dl) ? (tb) : c0);
          else if (dr == 1) c1 = (lane == (dl) ? (tb) : c1);
          else if (dr == 2) c2 = (lane == (dl) ? (tb) : c2);
          else c3 = (lane == (dl) ? (tb) : c3);
          if (old == kInf) {  // FindOrAddToken creates it
            if (dr == 0) d0 = (lane == (dl) ? (created) : d0);
            else if (dr == 1) d1 = (lane == (dl) ? (created) : d1);
            else if (dr == 2) d2 = (lane == (dl) ? (created) : d2);
            else d3 = (lane == (dl) ? (created) : d3);
            created++;
          }
          if (KRD(dr, dl, n0r, n1r, n2r, n3r) > 0) {  // changed: re-queued (tokens that relax arcs)
            if (sp == 128) {
              ovf = true;
              break;
            }
            if (sp < 64) q0 = (lane == (sp) ? (d) : q0);
            else q1 = (lane == (sp - 64) ? (d) : q1);
            sp++;
          }
        }
      }
    }
#undef KRD
#undef KSEL
    if (lane < nm) { (*reinterpret_cast<float*>(&K.rec[lane].y)) = __int_as_float(c0); K.mord[lane] = d0; }
    if (lane + 64 < nm) { (*reinterpret_cast<float*>(&K.rec[lane + 64].y)) = __int_as_float(c1); K.mord[lane + 64] = d1; }
    if (lane + 128 < nm) { (*reinterpret_cast<float*>(&K.rec[lane + 128].y)) = __int_as_float(c2); K.mord[lane + 128] = d2; }
    if (lane + 192 < nm) { (*reinterpret_cast<float*>(&K.rec[lane + 192].y)) = __int_as_float(c3); K.mord[lane + 192] = d3; }
    if (lane == 0) sh.kn0 = ovf ? -1 : created;
  } else if (threadIdx.x == 0 && fast) {
    int sp = n0, created = 0;
    bool ovf = false;
    while (sp > 0 && !ovf) {
      const int u = K.stk[--sp];
      const float cu = (*reinterpret_cast<float*>(&K.rec[u].y));
      if (!(cu < cutoff)) continue;
      const int e1 = K.rec[u].z + K.rec[u].w;
      for (int e = K.rec[u].z; e < e1; e++) {
        const int2 rec = K.adj[e];
        const float tot = cu + __int_as_float(rec.y);
        if (rec.x < 0 || !(tot < cutoff)) continue;
        const float old = (*reinterpret_cast<float*>(&K.rec[rec.x].y));
        if (tot < old) {
          if (old == kInf) K.mord[rec.x] = created++;  // FindOrAddToken creates it
          (*reinterpret_cast<float*>(&K.rec[rec.x].y)) = tot;
          if (K.rec[rec.x].w > 0) {  // changed: re-queued (only tokens that relax arcs matter)
            if (sp == kKM) {
              ovf = true;
              break;
            }
            K.stk[sp++] = rec.x;
          }
        }
      }
    }
    sh.kn0 = ovf ? -1 : created;
  }
  __syncthreads();
  const bool slow = !replayed && !(a.debug & 8) && (!fast || sh.kn0 < 0);
  if (slow && fast) {  // the LDS queue overflowed: start over through the HBM records
    for (int i = threadIdx.x; i < nm; i += DT) {
      const int c = K.mcr[i];
      (*reinterpret_cast<float*>(&K.rec[i].y)) = c >= 0 ? AG_LD(&KC[c]) : kInf;
      K.mord[i] = -1;
    }
    __syncthreads();
    for (int q = threadIdx.x; q < n0; q += DT) {  // the initial queue again (the LDS stack was consumed)
      const unsigned long long kq = ((unsigned long long)(unsigned)K.v0hi[q] << 32) | (unsigned)K.v0lo[q];
      int r = 0;
      for (int j = 0; j < n0; j++) r += (((unsigned long long)(unsigned)K.v0hi[j] << 32) | (unsigned)K.v0lo[j]) < kq;
      const int v = AG_LD(&KO[(int)(unsigned)(kq & 0xffffffffu)]);
      const int i = v >= 0 ? t.hst[v] : AG_LD(&T.stamp[~v]);
      if (r < kKM) K.stk[r] = i;
      else AG_ST(&KS[r - kKM], i);
    }
    vm_drain();
    __syncthreads();
  }
  if (threadIdx.x == 0 && slow) {
    int sp = n0, created = 0;
    const int scap = kKM + a.kord_cap;
    while (sp > 0) {
      --sp;
      const int u = sp < kKM ? K.stk[sp] : AG_LD(&KS[sp - kKM]);
      const float cu = __int_as_float(km_get(K, KM, u, kMCost));
      if (!(cu < cutoff)) continue;
      const int cnt = km_get(K, KM, u, kMCnt), off = km_get(K, KM, u, kMOff);
      for (int k = 0; k < cnt; k++) {
        const int e = off + k;
        int2 rec;
        if (e < kKE) {
          rec = K.adj[e];
        } else {
          const unsigned long long w = (unsigned long long)AG_LD(&reinterpret_cast<long long*>(KA)[e - kKE]);
          rec = make_int2((int)(unsigned)w, (int)(unsigned)(w >> 32));
        }
        if (rec.x < 0) continue;  // a token of the emitting pass that relaxes nothing: no effect
        const float tot = cu + __int_as_float(rec.y);
        if (!(tot < cutoff)) continue;
        const float old = __int_as_float(km_get(K, KM, rec.x, kMCost));
        if (old == kInf) km_set(K, KM, rec.x, kMOrd, created++);  // FindOrAddToken creates it
        if (tot < old) {
          km_set(K, KM, rec.x, kMCost, __float_as_int(tot));
          if (km_get(K, KM, rec.x, kMCnt) > 0) {  // changed: re-queued (only tokens that relax arcs matter)
            if (sp < kKM) K.stk[sp] = rec.x;
            else if (sp - kKM < a.kord_cap) AG_ST(&KS[sp - kKM], rec.x);
            else sh.bad |= 1;
            sp++;
            if (sp >= scap) break;
          }
        }
      }
      if (sp >= scap) break;
    }
    sh.kn0 = created;
  }
  __syncthreads();
  if (threadIdx.x == 0 && sh.kn0 != n_eps) sh.bad |= 1;  // the queue must create exactly the closure's tokens
  vm_drain();
  __syncthreads();
  pr.mark(26);
  pr.count(28, 1);
  pr.count(29, fast ? 1 : 0);
  pr.count(30, replayed ? 1 : 0);
  pr.count(31, nm);
  if (replayed) {
    pr.count(32, sh.kpop_sum);
    pr.count(33, sh.kpop_max);
    pr.count(45, sh.kcomp_n);
    pr.count(46, sh.kcomp_max);
    pr.count(61, sh.kcomp_clk);
    pr.count(54, sh.karc_sum);
    pr.count(55, sh.karc_max);
    pr.count(56, sh.khbm_pops);
  }
  // the created tokens' creation indices [ne, ne + n_eps) in the queue's order, and their buckets
  for (int i = threadIdx.x; i < nm; i += DT) {
    if (km_get(K, KM, i, kMC) >= 0) continue;
    const int o = km_get(K, KM, i, kMOrd);
    if (o < 0 || o >= n_eps) continue;
    const int c = ne + o;
    const int v = km_get(K, KM, i, kMSlot);
    AG_ST(&KO[c], v);
    if (a.lazy_id) continue;  // (buckets after the frame's lazy numbering)
    const int b = kbucket(a, slot, slot_state(t, T, v), khash);
    AG_ST(&KB[c], b);
    __hip_atomic_fetch_min(&BF[b], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int m = __hip_atomic_fetch_add(&BC[b], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (m < kKbMemb) AG_ST(&BM[kKbMemb * b + m], c);
  }
  vm_drain();
  __syncthreads();
  pr.mark(27);
  if (a.lazy_id && sh.bad == 0) kaldi_lazy_frame(a, sh, t, T, K, st, slot, ne, n_eps, khash, pr);
  if (pr.on) {
    pr.count(51, nm > 1536 ? 1 : 0);
    pr.count(52, nm > 2048 ? 1 : 0);
    pr.count(53, adj_n > kKE ? 1 : 0);
  }
  if (pr.on && threadIdx.x == 0) sh.kbig = nm > kKM;
  if (pr.on && nm > kKM) {  // frames whose queue members overflow the LDS records
    pr.count(48, (long long)__builtin_amdgcn_s_memtime() - t_nonemit0);
    pr.count(49, 1);
    pr.count(50, t_lanes);
  }
  return ne + n_eps;
}

// List positions of the frame's n tokens (HashList order: buckets by their
// first creation index, then creation index), written to each slot's hst /
// stamp (slot_pos).  Bucket starts: a scan over the creation order in which
// each bucket's first token contributes the bucket's size.
__device__ __forceinline__ void kaldi_positions(const DecArgs& a, DecShared& sh, const FrameLds& t, const HbmTab& T,
                                                int slot, int n, Prof& pr) {
  int crowded = 0;
  if (threadIdx.x == 0) sh.kk = 0;  // crowded buckets (profile count; visible after the scans' barriers)
  const int* KO = a.kord + (long long)slot * a.kord_cap;
  const int* KB = a.kbkt + (long long)slot * a.kord_cap;
  int* BF = a.kb_first + (long long)slot * a.kb_cap;
  int* BC = a.kb_cnt + (long long)slot * a.kb_cap;
  int* BS = a.kb_start + (long long)slot * a.kb_cap;
  int* BM = a.kb_memb + (long long)slot * a.kb_cap * kKbMemb;
  // kHlU creation indices per thread at a time, each step's loads in flight
  // together (bucket, then its first index and size; the scans in order)
  int run = 0, par = 0;
  for (int c0 = 0; c0 < n; c0 += kHlU * DT) {
    int b[kHlU], bf[kHlU], bc[kHlU];
#pragma unroll
    for (int u = 0; u < kHlU; u++) {
      const int c = c0 + u * DT + (int)threadIdx.x;
      b[u] = c < n ? AG_LD(&KB[c]) : 0;
    }
#pragma unroll
    for (int u = 0; u < kHlU; u++) {
      const int c = c0 + u * DT + (int)threadIdx.x;
      bf[u] = -1;
      bc[u] = 0;
      if (c < n) {
        bf[u] = AG_LD(&BF[b[u]]);
        bc[u] = AG_LD(&BC[b[u]]);
      }
    }
#pragma unroll
    for (int u = 0; u < kHlU; u++) {
      if (c0 + u * DT >= n) break;
      const int c = c0 + u * DT + (int)threadIdx.x;
      const bool lead = c < n && bf[u] == c;
      int tot;
      const int ex = run + kaldi_excl_sum(sh, lead ? bc[u] : 0, par, &tot);
      if (lead) AG_ST(&BS[b[u]], ex);
      run += tot;
      par ^= 1;
    }
  }
  vm_drain();
  __syncthreads();
  for (int c0 = 0; c0 < n; c0 += kHlU * DT) {
    int b[kHlU], v[kHlU], cnt[kHlU], bs[kHlU];
#pragma unroll
    for (int u = 0; u < kHlU; u++) {
      const int c = c0 + u * DT + (int)threadIdx.x;
      if (c >= n) continue;
      b[u] = AG_LD(&KB[c]);
      v[u] = AG_LD(&KO[c]);
    }
#pragma unroll
    for (int u = 0; u < kHlU; u++) {
      const int c = c0 + u * DT + (int)threadIdx.x;
      if (c >= n) continue;
      cnt[u] = AG_LD(&BC[b[u]]);
      bs[u] = AG_LD(&BS[b[u]]);
    }
#pragma unroll
    for (int u = 0; u < kHlU; u++) {
      const int c = c0 + u * DT + (int)threadIdx.x;
      if (c >= n) continue;
      int rk = 0;
      if (cnt[u] > 1 && cnt[u] <= kKbMemb) {  // the bucket's members created before c
        for (int m = 0; m < cnt[u]; m += 4) {
          const int4 q = wg_ld4(reinterpret_cast<const int4*>(&BM[kKbMemb * b[u] + m]));
          rk += (q.x < c) + (m + 1 < cnt[u] && q.y < c) + (m + 2 < cnt[u] && q.z < c) + (m + 3 < cnt[u] && q.w < c);
        }
      } else if (cnt[u] > kKbMemb) {  // a crowded bucket: count its tokens created before
        // (from the bucket's first creation index: none of its tokens is older)
        crowded++;
        for (int c2 = AG_LD(&BF[b[u]]); c2 < c; c2++) rk += AG_LD(&KB[c2]) == b[u];
      }
      const int pos = bs[u] + rk;
      if (v[u] >= 0) t.hst[v[u]] = pos;
      else AG_ST(&T.stamp[~v[u]], pos);
    }
  }
  if (crowded) atomicAdd(&sh.kk, crowded);
  vm_drain();
  __syncthreads();
  pr.count(44, sh.kk);
  pr.mark(43);
}

// OpenFST's lazy ComposeFst numbering, in two parts.
// Kaldi's decoder expands a composed state (its arcs computed, their
// destinations numbered) when it first iterates its arcs or asks for its
// input epsilons: per frame, ProcessNonemitting's queue fill asks every token
// of the emitting pass in list order, then every token the queue creates, in
// creation order (a token's state is expanded when the token appears; the
// emitting pass of the next frame and GetCutoff only revisit them).  A
// token the queue creates may take an id its source's expansion gives in the
// same frame, so the queue's tokens join their HashList buckets only after
// (kaldi_lazy_frame, at the end of kaldi_nonemitting): the emitting pass's
// tokens' list positions among themselves (kaldi_positions over them), then
// kaldi_lazy_order: the frame's states in expansion order into kstk; then
// kaldi_lazy_number: the states not yet expanded number their destinations
// without an id, in order (state, arc): the first arc to reach a destination
// -- an atomic minimum of its dense arc number -- gives it the next id, the
// ids ranked by a bitmap over the arc numbers and its prefix popcounts; then
// the queue's tokens' buckets.
__device__ __forceinline__ void kaldi_lazy_order(const DecArgs& a, DecShared& sh, const FrameLds& t, const HbmTab& T,
                                                 int slot, int n) {
  const int* KO = a.kord + (long long)slot * a.kord_cap;
  int* SQ = a.kstk + (long long)slot * a.kord_cap;
  int* FL = reinterpret_cast<int*>(a.kcost0 + (long long)slot * a.kord_cap);
  const int ne = sh.klazy_ne;
  // (the positions leave gaps: the buckets' counts include the queue's
  // numbered tokens, which joined them already; the order is the list's)
  for (int p = threadIdx.x; p < n; p += DT) AG_ST(&FL[p], 0);
  vm_drain();
  __syncthreads();
  for (int c = threadIdx.x; c < n; c += DT) {
    const int v = AG_LD(&KO[c]);
    const int s = slot_state(t, T, v);
    if (c >= ne) {  // the queue's tokens in creation order
      AG_ST(&SQ[c], s);
      continue;
    }
    const int pos = v >= 0 ? t.hst[v] : AG_LD(&T.stamp[~v]);
    if (pos < 0 || pos >= n) {
      sh.bad |= 1;
      continue;
    }
    AG_ST(&FL[pos], s + 1);
  }
  vm_drain();
  __syncthreads();
  int run = 0, par = 0;
  for (int p0 = 0; p0 < n; p0 += DT) {  // the emitting pass's tokens in list order
    const int p = p0 + threadIdx.x;
    const int x = p < n ? AG_LD(&FL[p]) : 0;
    int tot;
    const int ex = run + kaldi_excl_sum(sh, x > 0 ? 1 : 0, par, &tot);
    if (x > 0) AG_ST(&SQ[ex], x - 1);
    run += tot;
    par ^= 1;
  }
  vm_drain();
  __syncthreads();
}

// the arcs (destination, dense arc number) of the frame's states not yet
// expanded, one item per arc over chunks of DT states (owner search as the
// emitting pass), fn(d, q)
template <class Fn>
__device__ __forceinline__ void lazy_arcs(const DecArgs& a, DecShared& sh, const int* SQ, const int* Q0, int n,
                                          Fn&& fn) {
  for (int c0 = 0; c0 < n; c0 += DT) {
    const int i = c0 + threadIdx.x;
    int deg = 0, q0 = -1, b = 0;
    if (i < n) {
      q0 = AG_LD(&Q0[i]);
      if (q0 >= 0) {
        const int s = AG_LD(&SQ[i]);
        b = (int)a.lazy_row[s];
        deg = (int)(a.lazy_row[s + 1] - a.lazy_row[s]);
      }
    }
    block_scan(sh, deg);
    owner_blocks(sh);
    sh.abeg[threadIdx.x] = b;
    sh.tsrc[threadIdx.x] = q0;
    __syncthreads();
    const int total = sh.total;
    const int nbo = (total + 63) >> 6 <= kOwnBlk ? (total + 63) >> 6 : 0;
    for (int it = threadIdx.x; it < total; it += DT) {
      const int j = owner_bo(sh, nbo, it);
      const int k = it - sh.scan[j];
      fn(a.lazy_next[sh.abeg[j] + k], sh.tsrc[j] + k);
    }
    vm_drain();
    __syncthreads();
  }
}

__device__ __forceinline__ void kaldi_lazy_number(const DecArgs& a, DecShared& sh, DecSlot& st, int slot, int n) {
  const int* SQ = a.kstk + (long long)slot * a.kord_cap;
  int* Q0 = reinterpret_cast<int*>(a.kcost0 + (long long)slot * a.kord_cap);
  int* ID = a.lazy_id + (long long)slot * a.lazy_ids;
  int* CA = a.lazy_cand + (long long)slot * a.lazy_ids;
  // the states to expand and their first dense arc numbers
  int run = 0, par = 0;
  for (int i0 = 0; i0 < n; i0 += DT) {
    const int i = i0 + threadIdx.x;
    int deg = 0;
    bool nw = false;
    if (i < n) {
      const int s = AG_LD(&SQ[i]);
      const int id = AG_LD(&ID[s]);  // (-1: a queue token's state numbered this frame)
      nw = id < 0 || !(id & kLazyExpanded);
      if (nw) deg = (int)(a.lazy_row[s + 1] - a.lazy_row[s]);
    }
    int tot;
    const int ex = run + kaldi_excl_sum(sh, deg, par, &tot);
    if (i < n) AG_ST(&Q0[i], nw ? ex : -1);
    run += tot;
    par ^= 1;
  }
  const int nq = run;
  // kmem (free after the queue): the bitmap over the arc numbers, its prefix
  // popcounts, and when there is room each arc's destination by arc number
  // (the later passes then skip the owner search)
  const int nw = (nq + 31) >> 5;
  const long long words = (long long)a.kord_cap * kKMRec;
  if (2LL * nw > words) {  // (capacity: arcs of one frame's new states)
    if (threadIdx.x == 0) sh.bad |= 1;
    __syncthreads();
    return;
  }
  unsigned* BITS = reinterpret_cast<unsigned*>(a.kmem + (long long)slot * words);
  int* PRE = reinterpret_cast<int*>(BITS + nw);
  int* DST = PRE + nw;
  const bool flat = 2LL * nw + nq <= words;
  for (int w = threadIdx.x; w < nw; w += DT) AG_ST(&BITS[w], 0u);
  vm_drain();
  __syncthreads();
  // each destination without an id: its first arc number
  lazy_arcs(a, sh, SQ, Q0, n, [&](int d, int q) {
    if (flat) AG_ST(&DST[q], d);
    if (AG_LD(&ID[d]) < 0) __hip_atomic_fetch_min(&CA[d], q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  });
  auto arcs = [&](auto&& fn) {
    if (flat) {
      for (int q = threadIdx.x; q < nq; q += DT) fn(AG_LD(&DST[q]), q);
      vm_drain();
      __syncthreads();
    } else {
      lazy_arcs(a, sh, SQ, Q0, n, fn);
    }
  };
  arcs([&](int d, int q) {
    if (AG_LD(&ID[d]) < 0 && AG_LD(&CA[d]) == q)
      __hip_atomic_fetch_or(&BITS[q >> 5], 1u << (q & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  });
  run = 0;
  par = 0;
  for (int w0 = 0; w0 < nw; w0 += DT) {
    const int w = w0 + threadIdx.x;
    const int c = w < nw ? __popc(AG_LD(&BITS[w])) : 0;
    int tot;
    const int ex = run + kaldi_excl_sum(sh, c, par, &tot);
    if (w < nw) AG_ST(&PRE[w], ex);
    run += tot;
    par ^= 1;
  }
  const int numbered = run;
  vm_drain();
  __syncthreads();
  const int base = st.lazy_count;
  arcs([&](int d, int q) {
    if (AG_LD(&ID[d]) < 0 && AG_LD(&CA[d]) == q) {
      const unsigned bw = AG_LD(&BITS[q >> 5]);
      AG_ST(&ID[d], base + AG_LD(&PRE[q >> 5]) + __popc(bw & ((1u << (q & 31)) - 1u)));
      AG_ST(&CA[d], 0x7fffffff);
    }
  });
  vm_drain();
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += DT)
    if (AG_LD(&Q0[i]) >= 0)
      __hip_atomic_fetch_or(&ID[AG_LD(&SQ[i])], kLazyExpanded, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  vm_drain();
  __syncthreads();
  st.lazy_count = base + numbered;
}

// the lazy numbering of a frame (see above).  Most frames expand few states
// (~170 of ~2500 tokens on the bench model): the emitting pass's are listed
// as its tokens take their buckets (lazy_new: creation index, bucket, state);
// the queue's tokens join their buckets here when their state has an id
// already (else after the numbering) and add theirs.  Their expansion order is
// the order of (key, creation index): an emitting token's key is its bucket's
// first creation index -- HashList's list is the buckets in first-insertion
// order -- a queue token's is ne (after every emitting one).  Up to DT of them
// are ranked in LDS and numbered in one chunk: their arcs by dense number q
// (owner search over the ranked degrees), each destination without an id its
// first arc by atomic minimum, then the winners' ids by a scan over q.  More
// (a stream's first frames) take the list positions and the chunked passes.
__device__ __forceinline__ void kaldi_lazy_frame(const DecArgs& a, DecShared& sh, const FrameLds& t, const HbmTab& T,
                                                 const KaldiLds& K, DecSlot& st, int slot, int ne, int n_eps, int khash,
                                                 Prof& pr) {
  const int n = ne + n_eps;
  const int* KO = a.kord + (long long)slot * a.kord_cap;
  int* KB = a.kbkt + (long long)slot * a.kord_cap;
  int* BF = a.kb_first + (long long)slot * a.kb_cap;
  int* BC = a.kb_cnt + (long long)slot * a.kb_cap;
  int* BM = a.kb_memb + (long long)slot * a.kb_cap * kKbMemb;
  int* ID = a.lazy_id + (long long)slot * a.lazy_ids;
  int* CA = a.lazy_cand + (long long)slot * a.lazy_ids;
  const int* LN = a.lazy_new + (long long)slot * 3 * kLazyNewCap;
  int* SQ = a.kstk + (long long)slot * a.kord_cap;
  int* KI = reinterpret_cast<int*>(sh.tcost);  // (LDS, free here) states of the listed tokens
  const long long words = (long long)a.kord_cap * kKMRec;
  int* DST = a.kmem + (long long)slot * words;  // (free after the queue) destination by arc number
  // (the queue's LDS, free after it: each listed state's first arc and degree)
  int* KR = K.stk;
  int* KD = K.v0hi;
  const int ke = sh.klazy_k;                    // the emitting pass's (listed when at most DT)
  __syncthreads();
  if (ke <= DT && (int)threadIdx.x < ke) {
    const int c = AG_LD(&LN[threadIdx.x]);
    const int b = AG_LD(&LN[kLazyNewCap + threadIdx.x]);
    const int s = AG_LD(&LN[2 * kLazyNewCap + threadIdx.x]);
    const long long r0 = a.lazy_row[s], r1 = a.lazy_row[s + 1];
    KI[threadIdx.x] = s;
    sh.abeg[threadIdx.x] = AG_LD(&BF[b]);
    sh.tsrc[threadIdx.x] = c;
    KR[threadIdx.x] = (int)r0;
    KD[threadIdx.x] = (int)(r1 - r0);
  }
  for (int c = ne + (int)threadIdx.x; c < n; c += DT) {  // the queue's tokens
    const int s = slot_state(t, T, AG_LD(&KO[c]));
    const int id = AG_LD(&ID[s]);
    const long long r0 = a.lazy_row[s], r1 = a.lazy_row[s + 1];  // (in flight with the id)
    if (id >= 0) {
      const int b = kbucket_of(id, khash);
      AG_ST(&KB[c], b);
      __hip_atomic_fetch_min(&BF[b], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int m = __hip_atomic_fetch_add(&BC[b], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (m < kKbMemb) AG_ST(&BM[kKbMemb * b + m], c);
    } else {
      AG_ST(&KB[c], -1);
      atomicAdd(&sh.klazy_def, 1);
    }
    if (id < 0 || !(id & kLazyExpanded)) {
      const int at = atomicAdd(&sh.klazy_k, 1);
      if (at < DT) {
        KI[at] = s;
        sh.abeg[at] = ne;
        sh.tsrc[at] = c;
        KR[at] = (int)r0;
        KD[at] = (int)(r1 - r0);
      }
    }
  }
  vm_drain();
  __syncthreads();
  const int k = sh.klazy_k;
  pr.count(64, k);
  pr.count(65, k > DT ? 1 : 0);
  pr.mark(66);
  if (k > DT) {
    kaldi_positions(a, sh, t, T, slot, ne, pr);
    kaldi_lazy_order(a, sh, t, T, slot, n);
    kaldi_lazy_number(a, sh, st, slot, n);
    pr.mark(70);
  } else if (k > 0) {
    int rk = 0, s = -1, b = 0, deg = 0;
    if ((int)threadIdx.x < k) {
      const int kh = sh.abeg[threadIdx.x], kl = sh.tsrc[threadIdx.x];
      s = KI[threadIdx.x];
      b = KR[threadIdx.x];
      deg = KD[threadIdx.x];
#pragma unroll 8
      for (int j = 0; j < k; j++) {
        const int h = sh.abeg[j];
        rk += h < kh || (h == kh && sh.tsrc[j] < kl);
      }
    }
    __syncthreads();
    if ((int)threadIdx.x < k) {
      sh.abeg[rk] = b;
      sh.tsrc[rk] = deg;
    }
    __syncthreads();
    pr.mark(67);
    const int dj = (int)threadIdx.x < k ? sh.tsrc[threadIdx.x] : 0;
    block_scan(sh, dj);
    const int nq = sh.total;
    if (nq > words) {  // (the general passes re-expand instead of keeping destinations)
      if (s >= 0) AG_ST(&SQ[rk], s);
      vm_drain();
      __syncthreads();
      kaldi_lazy_number(a, sh, st, slot, k);
    } else {
      owner_blocks(sh);
      __syncthreads();
      const int nbo = (nq + 63) >> 6 <= kOwnBlk ? (nq + 63) >> 6 : 0;
      for (int q = threadIdx.x; q < nq; q += DT) {
        const int j = owner_bo(sh, nbo, q);
        const int d = a.lazy_next[sh.abeg[j] + q - sh.scan[j]];
        const bool open = AG_LD(&ID[d]) < 0;
        AG_ST(&DST[q], open ? d : -1);
        if (open) __hip_atomic_fetch_min(&CA[d], q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      vm_drain();
      __syncthreads();
      pr.mark(68);
      const int base = st.lazy_count;
      int run = 0, par = 0;
      for (int q0 = 0; q0 < nq; q0 += DT) {
        const int q = q0 + threadIdx.x;
        const int d = q < nq ? AG_LD(&DST[q]) : -1;
        const bool win = d >= 0 && AG_LD(&CA[d]) == q;
        int tot;
        const int ex = run + kaldi_excl_sum(sh, win ? 1 : 0, par, &tot);
        if (win) {
          AG_ST(&ID[d], base + ex);
          AG_ST(&CA[d], 0x7fffffff);
        }
        run += tot;
        par ^= 1;
      }
      vm_drain();
      __syncthreads();
      if (s >= 0) __hip_atomic_fetch_or(&ID[s], kLazyExpanded, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      st.lazy_count = base + run;
      pr.mark(69);
    }
  }
  if (sh.klazy_def) {  // the queue's tokens whose state this frame numbered
    for (int c = ne + (int)threadIdx.x; c < n; c += DT) {
      if (AG_LD(&KB[c]) >= 0) continue;
      const int b = kbucket(a, slot, slot_state(t, T, AG_LD(&KO[c])), khash);
      AG_ST(&KB[c], b);
      __hip_atomic_fetch_min(&BF[b], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int m = __hip_atomic_fetch_add(&BC[b], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (m < kKbMemb) AG_ST(&BM[kKbMemb * b + m], c);
    }
  }
  vm_drain();
  __syncthreads();
  pr.mark(63);
}

// the buckets the frame used, emptied for the next one
__device__ __forceinline__ void kaldi_clear_buckets(const DecArgs& a, int slot, int n) {
  const int* KB = a.kbkt + (long long)slot * a.kord_cap;
  int* BF = a.kb_first + (long long)slot * a.kb_cap;
  int* BC = a.kb_cnt + (long long)slot * a.kb_cap;
  for (int c = threadIdx.x; c < n; c += DT) {
    const int b = AG_LD(&KB[c]);
    AG_ST(&BF[b], kNoStamp);
    AG_ST(&BC[b], 0);
  }
}

// Lattice side of a commit (all threads; the frame tables are still intact).
// commit_emit_links: keep this frame's emitting records below the cutoff,
// resolved to arena indices through their destination slots (chunked
// in-place compaction: writes never pass the chunk being read); with
// deferred winners a kept record whose (cost, arc) key is its destination's
// final key writes its source as the destination's backpointer (exactly one
// relaxation per surviving slot holds the final key: emitting arcs are
// relaxed once per frame, and a slot an epsilon arc improved holds an
// epsilon key).  commit_eps_links: the epsilon links of the committed tokens
// that have epsilon arcs (listed by the commit in the frontier arrays, neps
// of them).  Every kept link's cost above its destination's, tot - cost(dst)
// >= 0 (the link's extra cost over the destination for PruneActiveTokens),
// replaces its destination slot in link_dst.
__device__ __forceinline__ int commit_emit_links(const DecArgs& a, DecShared& sh, const FrameLds& t,
                                                 const HbmTab& T, const DecSlot& st, int slot, int base,
                                                 int nl_n, float cutoff, bool defer) {
  int4* L = a.links + (long long)slot * a.link_cap;
  int* LD = a.link_dst + (long long)slot * a.link_cap;
  const long long lb = st.links_used;
  long long nrec = sh.n_links;
  if (lb + nrec > a.link_cap) nrec = a.link_cap - lb > 0 ? a.link_cap - lb : 0;
  int out = 0;
  // records of the next chunk are loaded while this one is compacted
  int4 rn = make_int4(0, 0, 0, 0);
  int vn = kNoSlot;
  if (threadIdx.x < nrec) {
    rn = L[lb + threadIdx.x];
    vn = LD[lb + threadIdx.x];
  }
  for (long long c0 = 0; c0 < nrec; c0 += DT) {
    const long long i = c0 + threadIdx.x;
    int keep = 0;
    int4 r = rn;
    const int v = vn;
    if (i + DT < nrec) {
      rn = L[lb + i + DT];
      vn = LD[lb + i + DT];
    }
    float d = 0.0f;
    if (i < nrec) {
      const float tot = __int_as_float(r.y);
      if (tot < cutoff && v != kNoSlot) {  // (kNoSlot: a failed relaxation, the frame is in error)
        const unsigned long long key = slot_key(t, T, v);
        if (defer && key == (((unsigned long long)ford(tot) << 32) | (unsigned)r.z)) set_bp(t, T, v, r.x);
        r.y = base + slot_pos(a, t, T, nl_n, v);
        d = tot - funord((uint32_t)(key >> 32));
        keep = 1;
      }
    }
    block_scan(sh, keep);
    if (keep) {
      L[lb + out + sh.scan[threadIdx.x]] = r;
      LD[lb + out + sh.scan[threadIdx.x]] = __float_as_int(d);
    }
    out += sh.total;
    __syncthreads();
  }
  if (defer) vm_drain();  // HBM backpointers visible to the token commit after its barrier
  return out;
}

__device__ __forceinline__ int commit_eps_links(const DecArgs& a, DecShared& sh, const FrameLds& t,
                                                const HbmTab& T, const DecPtrs& p, const DecSlot& st,
                                                int slot, int base, int nl_n, int neps, int out,
                                                float cutoff) {
  int4* L = a.links + (long long)slot * a.link_cap;
  int* LD = a.link_dst + (long long)slot * a.link_cap;
  const long long lb = st.links_used;
  // epsilon links of the committed tokens, at their final costs
  if (threadIdx.x == 0) sh.n_eps = 0;
  __syncthreads();  // every thread reads n_eps below, also when neps == 0
  for (int c0 = 0; c0 < neps; c0 += DT) {
    const int q = c0 + threadIdx.x;
    int deg = 0, ab = 0, src = 0;
    float c = 0.0f;
    if (q < neps) {
      const int v = get_front(t, p, 0, q);
      const int s = slot_state(t, T, v);
      c = funord((uint32_t)(slot_key(t, T, v) >> 32));
      const int4 si = a.sinfo[s];
      ab = si.y;
      deg = si.z - si.y;
      src = base + slot_pos(a, t, T, nl_n, v);
    }
    block_scan(sh, deg);
    sh.abeg[threadIdx.x] = ab;
    sh.tcost[threadIdx.x] = c;
    sh.tsrc[threadIdx.x] = src;
    __syncthreads();
    const int total = sh.total;
    for (int it = threadIdx.x; it < total; it += DT) {
      const int j = owner(sh, it);
      const int arc = sh.abeg[j] + (it - sh.scan[j]);
      const int4 A = a.arcs[arc];
      const float tot = sh.tcost[j] + __int_as_float(A.y);
      if (tot < cutoff) {
        const int v = frame_slot(a, t, T, A.x);
        const unsigned long long m = __ballot(1);
        const int lane = threadIdx.x & 63;
        const int leader = __ffsll((long long)m) - 1;
        int w0 = 0;
        if (lane == leader) w0 = atomicAdd(&sh.n_eps, __popcll(m));
        w0 = __builtin_amdgcn_readlane(w0, leader);
        const long long pos = lb + out + w0 + __popcll(m & ((1ull << lane) - 1ull));
        if (pos < a.link_cap && v != kNoSlot) {
          L[pos] = make_int4(sh.tsrc[j], base + slot_pos(a, t, T, nl_n, v), arc, 0);
          LD[pos] = __float_as_int(tot - funord((uint32_t)(slot_key(t, T, v) >> 32)));
        } else {
          atomicOr(&sh.lat_ovf, v == kNoSlot ? 2 : 1);  // 2: an epsilon link's destination is not in the frame
        }
      }
    }
    __syncthreads();
  }
  const long long nrec = sh.n_links;
  const int n = out + sh.n_eps;
  if (lb + nrec > a.link_cap || lb + n > a.link_cap) sh.lat_ovf = 1;
  return lb + n > a.link_cap ? (int)(a.link_cap - lb) : n;
}

// Move the frame under construction into the arena + current token arrays
// (global, and the LDS cache when it fits).  List entries whose cost is not
// below `cutoff` (dead: created by the single emitting pass above the final
// next_cutoff) keep an arena slot marked dead.  Then both tables are cleared.
__device__ __forceinline__ void commit(const DecArgs& a, DecShared& sh, FrameLds& t, DecPtrs& p, DecSlot& st,
                       int* TS, float* TC, bool* lds, float cutoff, float* best_out, int slot,
                       int* nlinks, bool defer, Prof& pr, float* max_out = nullptr) {
  __syncthreads();
  const HbmTab T = hbm_tab(a, slot);
  const int nl_n = sh.n_new_l;
  const int ng = sh.n_new_g < a.max_tok ? sh.n_new_g : a.max_tok;
  const int n = nl_n + ng;
  const int base = st.arena_used;
  // Kaldi order after an overflow (sh.bad: tokens created but not listed,
  // creation indices past kord_cap): list positions are not defined, so
  // nothing is committed (the stream stops with its error bits; the next
  // reset clears every table)
  const bool ok = (long long)base + n <= a.arena_cap && !(a.kaldi && sh.bad);
  const bool lat = a.links != nullptr;
  // Kaldi order: the tokens' list positions (slot_pos) first
  if (a.kaldi && ok) kaldi_positions(a, sh, t, T, slot, n, pr);
  // the emitting records first: with deferred winners they set the
  // backpointers the token commit below reads (Kaldi order: every record is
  // an accepted relaxation, kept)
  const int n_emit = (lat && ok) ? commit_emit_links(a, sh, t, T, st, slot, base, nl_n,
                                                     a.kaldi ? __int_as_float(0x7f800000) : cutoff, defer)
                                 : 0;
  pr.mark(7);
  if (threadIdx.x == 0) {
    sh.n_next = 0;
    sh.n_front = 0;
  }
  __syncthreads();
  unsigned long long bk = kEmpty;
  float mx = -__int_as_float(0x7f800000);  // the largest token cost (Kaldi order: GetCutoff's shortcut)
  for (int j0 = threadIdx.x; j0 < n; j0 += 2 * DT) {
   // two entries per thread: the HBM entries' dependent loads in flight together
   int sq[2], bpq[2], vq[2];
   unsigned long long kq[2];
   bool eq[2];
#pragma unroll
   for (int q = 0; q < 2; q++) {
    const int j = j0 + q * DT;
    vq[q] = j < nl_n ? (int)t.nl[j] : j < n ? ~AG_LD(&T.list[j - nl_n]) : 0;
   }
#pragma unroll
   for (int q = 0; q < 2; q++) {
    const int j = j0 + q * DT;
    if (j >= n) continue;
    const int v = vq[q];
    if (j < nl_n) {
      sq[q] = t.hs[v];
      kq[q] = t.hk[v];
      bpq[q] = t.hb[v];
      eq[q] = (t.hp[v] & kPosEps) != 0;
    } else {
      const int g = ~v;
      sq[q] = AG_LD(&T.state[g]);
      kq[q] = AG_LD(&T.key[g]);
      bpq[q] = AG_LD(&T.bp[g]);
      eq[q] = (AG_LD(&T.pos[g]) & kHPosEps) != 0;
    }
   }
#pragma unroll
   for (int q = 0; q < 2; q++) {
    const int j = j0 + q * DT;
    if (j >= n) continue;
    const int s = sq[q], bp = bpq[q], v = vq[q];
    const unsigned long long k = kq[q];
    const bool has_eps = eq[q];
    const int arc = (int)(unsigned)(k & 0xffffffffu);
    const float cost = funord((uint32_t)(k >> 32));
    if (ok && (a.kaldi || cost < cutoff)) {  // Kaldi order: every created token is a token
      int prev = -1;
      if (arc >= 0) {
        if (bp & kBpEps) {
          const int sv = bp_slot(bp);
          // a source slot outside both tables can only be a backpointer that
          // was never written: flagged, never dereferenced
          if (sv >= kHashCap || (sv < 0 && ~sv >= (1 << a.hbits))) {
            sh.bad |= 8;
          } else {
            prev = base + slot_pos(a, t, T, nl_n, sv);
          }
        } else {
          prev = bp;
        }
      }
      // arena offset: the creation index, or the list position (Kaldi order,
      // whose current-token arrays are in list order)
      const int ao = a.kaldi ? slot_pos(a, t, T, nl_n, v) : j;
      wg_st4(&p.arena[base + ao], make_int4(prev, arc, __float_as_int(cost), s));
      const int qa = atomicAdd(&sh.n_next, 1);
      const int q = a.kaldi ? ao : qa;
      if (q < a.max_tok) {  // the current-token arrays hold max_tok entries
        AG_ST(&p.cs[q], s);
        AG_ST(&p.cc[q], cost);
        AG_ST(&p.cp[q], ao);
      } else {
        sh.bad |= 1;
      }
      if (q < kTokLds) {
        TS[q] = s;
        TC[q] = cost;
      }
      // epsilon links: tokens Kaldi expands (cost below the cutoff)
      if (lat && has_eps && cost < cutoff) push_front(a, sh, t, p, 0, &sh.n_front, v);
      // GetCutoff's best token: the first minimum in list order (Kaldi), else the lowest state
      const unsigned long long tk = ((unsigned long long)ford(cost) << 32) | (unsigned)(a.kaldi ? q : s);
      bk = tk < bk ? tk : bk;
      mx = fmaxf(mx, cost);
    } else if (ok) {
      wg_st4(&p.arena[base + j], make_int4(-2, -1, __float_as_int(cost), s));  // dead list entry
    }
   }
  }
  bk = block_min_u64(sh, bk);  // ends with a barrier
  if (max_out) *max_out = -block_min_f(sh, -mx);
  pr.mark(6);
  pr.count(12, n);
  if (!ok) sh.bad |= 2;
  const int live = sh.n_next < a.max_tok ? sh.n_next : a.max_tok;
  const int neps = sh.n_front < kFrontLds + a.max_tok ? sh.n_front : kFrontLds + a.max_tok;
  *nlinks = (lat && ok) ? commit_eps_links(a, sh, t, T, p, st, slot, base, nl_n, neps, n_emit, cutoff) : 0;
  pr.mark(8);
  __syncthreads();
  if (a.kaldi && ok) kaldi_clear_buckets(a, slot, n);
  hbm_clear_listed(a, T, ng);
  lds_clear_build(t);
  __syncthreads();
  pr.mark(9);
  if (ok) {
    st.cur_base = base;
    st.arena_used = base + n;
    st.ntok = live;
  } else {
    st.ntok = 0;
  }
  *lds = live <= kTokLds;
  st.best_key = bk;  // GetCutoff's best token of the next frame
  *best_out = funord((uint32_t)(bk >> 32));
}

// after a commit (all threads, past its barriers): the frame's record; every
// thread advances its copy of links_used identically
__device__ __forceinline__ void frame_done(const DecArgs& a, DecShared& sh, DecSlot& st, int slot, int index,
                                           float cutoff, float cost_offset, int nl) {
  if (threadIdx.x == 0 && index < a.lat_frame_cap) {
    LatFrame F;
    F.tok_base = st.cur_base;
    F.ntok = st.arena_used - st.cur_base;
    F.link_begin = st.links_used;
    F.link_end = st.links_used + nl;
    F.cutoff = cutoff;
    F.cost_offset = cost_offset;
    F.new_base = F.new_ntok = 0;
    a.lat_frames[(long long)slot * a.lat_frame_cap + index] = F;
  }
  // bits: 1 link arena full, 2 epsilon-link destination missing, 4 frame table full
  st.lat_ovf |= sh.lat_ovf | (index >= a.lat_frame_cap ? 4 : 0);
  st.links_used += nl;
}

// ---------------------------------------------------------------------------
// PruneActiveTokens (Kaldi LatticeFasterDecoder, every prune_interval
// frames): extra costs backwards from the frontier (whose tokens have extra
// cost 0), links whose extra cost exceeds the beam dropped, tokens with no
// surviving link dropped, and the stream's arena and link arena compacted
// in place.  Extra costs only grow as the frontier advances, so a link
// dropped here is one the final lattice-beam prune drops too: the pruned
// lattice is unchanged.  Frames below prune_from keep their
// last extra costs; the backward walk stops at the first such frame whose
// costs did not change.  Without a lattice (no links) the same compaction
// keeps the tokens on the backpointer chains of the frontier's tokens.
//
// A link's extra cost is X[dst] + d with d = tot - cost(dst) >= 0 stored at
// commit (link_dst), so the backward pass reads only the destination's
// extra cost.  The compaction passes run over the whole window at once,
// four items per thread.
// ---------------------------------------------------------------------------
constexpr int kDropped = (int)0x80000000u;  // remap entry flag: token dropped (low bits: kept before it)
constexpr int kPI = 4;                      // items per thread in the compaction passes

__device__ __forceinline__ void atomic_min_pos(float* p, float v) {  // v >= 0
  atomicMin(reinterpret_cast<int*>(p), __float_as_int(v));
}

__device__ __forceinline__ void load_frame(DecShared& sh, const LatFrame* LF, int k, int k1) {
  __syncthreads();
  if (threadIdx.x == 0) {
    sh.fr = LF[k];
    if (k1 >= 0) sh.fr1 = LF[k1];
  }
  __syncthreads();
}

// block-wide "did any thread set its flag" loop helper: three rotating LDS
// flags, one barrier per round
struct FixRound {
  int it = 0;
  int base = 0;  // flag set (alternate sets in consecutive loops need no barrier between them)
  __device__ __forceinline__ void begin(DecShared& sh) {
    if (threadIdx.x == 0) sh.fl[base + (it + 1) % 3] = 0;
  }
  __device__ __forceinline__ void mark(DecShared& sh) { sh.fl[base + it % 3] = 1; }
  __device__ __forceinline__ bool end(DecShared& sh) {  // true: another round
    __syncthreads();
    const bool again = sh.fl[base + it % 3] != 0;
    it++;
    return again;
  }
};

// development: structural invariants of frames kmin..F (links of frame k:
// destination in frame k, source in frame k-1 or k); tag = call site
__device__ void prune_check(const DecArgs& a, const LatFrame* LF, const int4* LK, int kmin, int F, int slot,
                            int tag, bool use_new) {
  for (int k = kmin; k <= F; k++) {
    const int tb = use_new ? LF[k].new_base : LF[k].tok_base;
    const int te = tb + (use_new ? LF[k].new_ntok : LF[k].ntok);
    const int tp = k > 0 ? (use_new && k > kmin ? LF[k - 1].new_base : LF[k - 1].tok_base) : tb;
    for (long long i = LF[k].link_begin + threadIdx.x; i < LF[k].link_end; i += DT) {
      const int4 r = LK[i];
      if (r.y < tb || r.y >= te || r.x < tp || r.x >= te)
        printf("prune_check tag %d slot %d frame %d kmin %d F %d link %lld src %d dst %d frame [%d,%d) prev %d\n",
               tag, slot, k, kmin, F, i, r.x, r.y, tb, te, tp);
    }
  }
  __syncthreads();
}

// fin: the segment's last prune (Kaldi FinalizeDecoding: PruneForwardLinksFinal
// then every frame with delta 0): the frontier's extra costs are its tokens'
// cost (plus the final cost when any token is final) above the best such
// total, and the walk goes back to frame 0.  Links into frontier tokens past
// the beam are dropped; the frontier tokens themselves stay (the current-token
// arrays keep their positions).
template <bool fin>
__device__ __forceinline__ void prune_segment(const DecArgs& a, DecShared& sh, DecSlot& st, const DecPtrs& p, int slot,
                                              Prof& pr, bool use_final = false) {
  const int F = st.frames;
  if (F <= 0 || F >= a.lat_frame_cap || st.err) return;
  if constexpr (fin)
    if (a.links == nullptr || st.lat_ovf) return;
  LatFrame* LF = a.lat_frames + (long long)slot * a.lat_frame_cap;
  float* X = a.extra + (long long)slot * a.arena_cap;
  int* R = a.remap + (long long)slot * a.arena_cap;
  int4* AR = p.arena;
  const bool lat = a.links != nullptr && !st.lat_ovf;
  int4* LK = a.links ? a.links + (long long)slot * a.link_cap : nullptr;
  int* LDd = a.links ? a.link_dst + (long long)slot * a.link_cap : nullptr;  // d bits of committed links
  const float beamp = a.lattice_beam + kPruneMargin;
  const float kInf = __int_as_float(0x7f800000);
  const int pf = st.prune_from;
  load_frame(sh, LF, F, -1);
  const int tbF = sh.fr.tok_base, endF = sh.fr.tok_base + sh.fr.ntok;
  if constexpr (!fin) {
    for (int t = tbF + threadIdx.x; t < endF; t += DT) AG_ST(&X[t], 0.0f);
  } else {
    float bn = kInf, bf = kInf;
    for (int t = tbF + threadIdx.x; t < endF; t += DT) {
      const int4 r = wg_ld4(&AR[t]);
      if (r.x == -2) continue;  // a dead list entry
      const float c = __int_as_float(r.z);
      bn = fminf(bn, c);
      bf = fminf(bf, c + __int_as_float(a.sinfo[r.w].w));
    }
    bn = block_min_f(sh, bn);
    bf = block_min_f(sh, bf);
    const bool use_f = use_final && bf != kInf;
    const float best = use_f ? bf : bn;
    for (int t = tbF + threadIdx.x; t < endF; t += DT) {
      const int4 r = wg_ld4(&AR[t]);
      float x = kInf;
      if (r.x != -2) {
        const float c = __int_as_float(r.z), fc = use_f ? __int_as_float(a.sinfo[r.w].w) : 0.0f;
        if (fc != kInf) x = fmaxf(0.0f, (c + fc) - best);
      }
      AG_ST(&X[t], x);
    }
    __syncthreads();
    // through the frontier's epsilon links (a non-final token that reaches a
    // final one within the frame has that token's extra cost plus the link's)
    FixRound fx;
    fx.base = 3 * (F & 1);
    if (threadIdx.x == 0) sh.fl[fx.base] = 0;
    __syncthreads();
    do {
      fx.begin(sh);
      for (long long i = sh.fr.link_begin + threadIdx.x; i < sh.fr.link_end; i += DT) {
        const int src = LK[i].x;
        if (src < tbF) continue;
        const float le = AG_LD(&X[LK[i].y]) + __int_as_float(LDd[i]);
        if (le <= beamp && le < AG_LD(&X[src])) {
          atomic_min_pos(&X[src], le);
          fx.mark(sh);
        }
      }
    } while (fx.end(sh));
  }
  int kmin = F;
  // Frames below prune_from are revisited at most prune_revisit deep: a
  // frame past that keeps the extra costs of its last walk, which are never
  // above the current ones (safe, it is only pruned less).  The final prune
  // walks every frame.
  const int kstop = fin ? 0 : (pf - a.prune_revisit > 0 ? pf - a.prune_revisit : 0);
  for (int k = F - 1; k >= kstop; k--) {
    // frame records read by every thread (nothing writes them during this walk)
    const LatFrame fk = LF[k], fk1 = LF[k + 1];
    const int tb = fk.tok_base, te = fk.tok_base + fk.ntok;
    for (int t = tb + threadIdx.x; t < te; t += DT) {
      if (k < pf) AG_ST(&R[t], __float_as_int(AG_LD(&X[t])));  // old extra cost
      AG_ST(&X[t], kInf);
    }
    // flags of this frame: the other set than frame k + 1's (whose last
    // readers may still be reading), reset before this barrier
    FixRound fx;
    fx.base = 3 * (k & 1);
    const int cf = 6 + (k & 1);
    if (threadIdx.x == 0) {
      sh.fl[fx.base] = 0;
      sh.fl[cf] = 0;
    }
    __syncthreads();
    if (lat) {
      // emitting out-links of frame k (stored with frame k + 1: sources below its tokens)
      // (kPI links per thread at a time: the records, then the destinations'
      // extra costs, in flight together -- a frame's links are one chain of
      // dependent loads, not one per DT links)
      const int tb1 = fk1.tok_base;
      for (long long c0 = fk1.link_begin; c0 < fk1.link_end; c0 += kPI * DT) {
        int2 r[kPI];
        float le[kPI];
#pragma unroll
        for (int u = 0; u < kPI; u++) {
          const long long i = c0 + u * DT + threadIdx.x;
          r[u] = make_int2(-1, 0);
          if (i < fk1.link_end) {
            const int4 l = LK[i];
            r[u] = make_int2(l.x < tb1 ? l.x : -1, l.y);
          }
        }
#pragma unroll
        for (int u = 0; u < kPI; u++) {
          const long long i = c0 + u * DT + threadIdx.x;
          le[u] = r[u].x >= 0 ? AG_LD(&X[r[u].y]) + __int_as_float(LDd[i]) : kInf;
        }
#pragma unroll
        for (int u = 0; u < kPI; u++)
          if (r[u].x >= 0 && le[u] <= beamp) atomic_min_pos(&X[r[u].x], le[u]);
      }
      __syncthreads();
      // epsilon links within frame k, to a fixpoint
      do {
        fx.begin(sh);
        for (long long c0 = fk.link_begin; c0 < fk.link_end; c0 += kPI * DT) {
          int2 r[kPI];
          float le[kPI], xs[kPI];
#pragma unroll
          for (int u = 0; u < kPI; u++) {
            const long long i = c0 + u * DT + threadIdx.x;
            r[u] = make_int2(-1, 0);
            if (i < fk.link_end) {
              const int4 l = LK[i];
              r[u] = make_int2(l.x >= tb ? l.x : -1, l.y);
            }
          }
#pragma unroll
          for (int u = 0; u < kPI; u++) {
            const long long i = c0 + u * DT + threadIdx.x;
            le[u] = kInf;
            xs[u] = 0.0f;
            if (r[u].x >= 0) {
              le[u] = AG_LD(&X[r[u].y]) + __int_as_float(LDd[i]);
              xs[u] = AG_LD(&X[r[u].x]);
            }
          }
#pragma unroll
          for (int u = 0; u < kPI; u++)
            if (r[u].x >= 0 && le[u] <= beamp && le[u] < xs[u]) {
              atomic_min_pos(&X[r[u].x], le[u]);
              fx.mark(sh);
            }
        }
      } while (fx.end(sh));
    } else {
      // backpointer chains: frame k + 1's kept tokens keep their frame-k sources
      for (int t = fk1.tok_base + threadIdx.x; t < fk1.tok_base + fk1.ntok; t += DT) {
        if (AG_LD(&X[t]) != 0.0f) continue;
        const int pv = AG_LD(&AR[t].x);
        if (pv >= tb && pv < te) AG_ST(&X[pv], 0.0f);
      }
      __syncthreads();
      do {  // epsilon backpointers inside frame k
        fx.begin(sh);
        for (int t = tb + threadIdx.x; t < te; t += DT) {
          if (AG_LD(&X[t]) != 0.0f) continue;
          const int pv = AG_LD(&AR[t].x);
          if (pv >= tb && pv < te && AG_LD(&X[pv]) != 0.0f) {
            AG_ST(&X[pv], 0.0f);
            fx.mark(sh);
          }
        }
      } while (fx.end(sh));
    }
    kmin = k;
    if (k < pf) {
      // Kaldi's delta (lattice_beam * prune_scale 0.1): when no extra cost of
      // this frame moved by more than it, the frames below keep theirs.  A
      // kept extra cost is never above the current one (they only grow), so
      // it prunes less, never more.  Backpointer marks compare exactly.
      const float delta = (lat && !fin) ? a.lattice_beam * 0.1f : 0.0f;
      for (int t = tb + threadIdx.x; t < te; t += DT)
        if (fabsf(AG_LD(&X[t]) - __int_as_float(AG_LD(&R[t]))) > delta) sh.fl[cf] = 1;
      __syncthreads();
      if (!sh.fl[cf]) break;
    }
  }
  pr.mark(16);
  pr.count(20, F - kmin);
  pr.count(21, 1);
  if ((a.debug & 1) && a.links) prune_check(a, LF, LK, kmin, F, slot, 1, false);
  // ---- token remap over the window [wb, arena_used): R[t - wb] = number of
  // kept tokens before t (kDropped: t itself is dropped)
  load_frame(sh, LF, kmin, -1);
  const int wb = sh.fr.tok_base;
  const long long lw = sh.fr.link_begin;
  const int end = st.arena_used;
  int out = wb;
  for (int c0 = wb; c0 < end; c0 += kPI * DT) {
    const int t0 = c0 + kPI * (int)threadIdx.x;
    int kb = 0, cnt = 0;
#pragma unroll
    for (int u = 0; u < kPI; u++) {
      const int t = t0 + u;
      const int k = t < end && (t >= tbF || AG_LD(&X[t]) <= beamp);
      kb |= k << u;
      cnt += k;
    }
    block_scan(sh, cnt);
    int pre = out + sh.scan[threadIdx.x];
#pragma unroll
    for (int u = 0; u < kPI; u++) {
      const int t = t0 + u;
      if (t < end) AG_ST(&R[t - wb], ((kb >> u) & 1) ? pre : (pre | kDropped));
      pre += (kb >> u) & 1;
    }
    out += sh.total;
    __syncthreads();
  }
  const int new_end = out;
  for (int k = kmin + threadIdx.x; k <= F; k += DT) {
    const int tbk = LF[k].tok_base;
    LF[k].new_base = tbk < end ? (AG_LD(&R[tbk - wb]) & ~kDropped) : new_end;
  }
  __syncthreads();
  for (int k = kmin + threadIdx.x; k <= F; k += DT)
    LF[k].new_ntok = (k < F ? LF[k + 1].new_base : new_end) - LF[k].new_base;
  pr.mark(17);
  // ---- links (before the tokens move: extra costs by old index), whole
  // window; wave 0 moves the frame boundaries that fall in each chunk
  long long lout = lw;
  if (a.links) {
    const long long lend = st.links_used;
    if (threadIdx.x == 0) sh.kk = kmin;
    __syncthreads();
    for (long long c0 = lw; c0 < lend; c0 += kPI * DT) {
      const long long i0 = c0 + kPI * (long long)threadIdx.x;
      int4 r[kPI];
      int dv[kPI];
      int kb = 0, cnt = 0;
#pragma unroll
      for (int u = 0; u < kPI; u++) {
        const long long i = i0 + u;
        int k = 0;
        if (i < lend) {
          r[u] = LK[i];
          dv[u] = LDd[i];
          const int rs = r[u].x >= wb ? AG_LD(&R[r[u].x - wb]) : r[u].x;
          const int rd = r[u].y >= wb ? AG_LD(&R[r[u].y - wb]) : r[u].y;
          if (((rs | rd) & kDropped) == 0) {
            k = !lat || AG_LD(&X[r[u].y]) + __int_as_float(dv[u]) <= beamp;
            r[u].x = rs;
            r[u].y = rd;
          }
        }
        kb |= k << u;
        cnt += k;
      }
      sh.kbits[threadIdx.x] = (unsigned char)kb;
      block_scan(sh, cnt);  // every thread has read its links: writes may follow
      int pre = sh.scan[threadIdx.x];
#pragma unroll
      for (int u = 0; u < kPI; u++) {
        if ((kb >> u) & 1) {
          LK[lout + pre] = r[u];
          LDd[lout + pre] = dv[u];
        }
        pre += (kb >> u) & 1;
      }
      if (threadIdx.x < 64) {  // frame boundaries inside this chunk
        const long long cend = c0 + kPI * DT;
        int kk = sh.kk;  // wave-uniform; sh.kk is only written back for the next chunk
        while (true) {
          const int k = kk + (int)threadIdx.x;
          long long olb = 0;
          bool in = false;
          if (k <= F) {
            olb = LF[k].link_begin;
            in = olb < cend;
          }
          const unsigned long long m = __ballot(in);
          if (in) {
            const int q = (int)(olb - c0), th = q / kPI, w = q % kPI;
            const int before = __popc((unsigned)sh.kbits[th] & ((1u << w) - 1u));
            LF[k].link_begin = lout + sh.scan[th] + before;
          }
          const int nin = __popcll(m);
          kk += nin;
          if (nin < 64) break;
        }
        if (threadIdx.x == 0) sh.kk = kk;
      }
      lout += sh.total;
      __syncthreads();
    }
    // boundaries at or past the end of the links
    for (int k = sh.kk + threadIdx.x; k <= F; k += DT) LF[k].link_begin = lout;
    __syncthreads();
    for (int k = kmin + threadIdx.x; k <= F; k += DT) LF[k].link_end = k < F ? LF[k + 1].link_begin : lout;
  }
  pr.mark(18);
  // ---- move the kept tokens (and their extra costs) down, in order
  for (int c0 = wb; c0 < end; c0 += kPI * DT) {
    const int t0 = c0 + kPI * (int)threadIdx.x;
    int nt[kPI];
    int4 rec[kPI];
    float x[kPI];
#pragma unroll
    for (int u = 0; u < kPI; u++) {
      const int t = t0 + u;
      nt[u] = -1;
      if (t < end) {
        const int rv = AG_LD(&R[t - wb]);
        if ((rv & kDropped) == 0) {
          nt[u] = rv;
          rec[u] = wg_ld4(&AR[t]);
          x[u] = AG_LD(&X[t]);
          if (rec[u].x >= wb) {
            const int np = AG_LD(&R[rec[u].x - wb]);
            if (!(np & kDropped)) {
              rec[u].x = np;
            } else if (fin && t >= tbF) {
              // the final prune keeps every frontier token, also those past
              // the beam whose predecessors it dropped: no backpointer
              rec[u].x = -1;
            } else {
              sh.bad |= 16;
              rec[u].x = np & ~kDropped;
            }
          }
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kPI; u++)
      if (nt[u] >= 0) {
        wg_st4(&AR[nt[u]], rec[u]);
        AG_ST(&X[nt[u]], x[u]);
      }
    __syncthreads();
  }
  for (int k = kmin + threadIdx.x; k <= F; k += DT) {
    LF[k].tok_base = LF[k].new_base;
    LF[k].ntok = LF[k].new_ntok;
  }
  __syncthreads();
  pr.mark(19);
  if ((a.debug & 1) && a.links) prune_check(a, LF, LK, kmin, F, slot, 2, false);
  if ((a.debug & 1) && threadIdx.x == 0)
    printf("prune slot %d F %d pf %d kmin %d wb %d end %d new_end %d links %lld -> %lld\n", slot, F, pf, kmin,
           wb, end, new_end, lw, lout);
  st.cur_base = new_end - (endF - tbF);
  st.arena_used = new_end;
  if (a.links) st.links_used = lout;
  st.prune_from = F;
  st.last_prune = F;
}

template <bool PROF>
__global__ __launch_bounds__(DT) void decode_kernel(DecArgs a) {
  __shared__ DecShared sh;
  __shared__ __attribute__((aligned(16))) float L[kLlhLds];
  __shared__ int TS[kTokLds];
  __shared__ float TC[kTokLds];
  __shared__ int t_hs[kHashCap];
  __shared__ unsigned long long t_hk[kHashCap];
  __shared__ int t_hb[kHashCap];
  __shared__ unsigned short t_hp[kHashCap];
  __shared__ int t_hst[kHashCap];
  __shared__ unsigned short t_nl[kHashCap];
  __shared__ __attribute__((aligned(16))) int t_fr[2][kFrontLds];  // (Kaldi order: 8-byte queue keys)
  FrameLds t;
  t.hs = t_hs;
  t.hk = t_hk;
  t.hb = t_hb;
  t.hp = t_hp;
  t.hst = t_hst;
  t.nl = t_nl;
  t.fr0 = t_fr[0];
  t.fr1 = t_fr[1];
  lds_clear_build(t);
  // Kaldi order: the epsilon queue's LDS views (kaldi_nonemitting)
  static_assert(kLlhLds >= 4 * kKM && kTokLds >= kKM && DT + 1 >= kKM && 2 * kFrontLds >= 2 * kKE, "LDS views");
  KaldiLds K;
  K.rec = reinterpret_cast<int4*>(L);
  K.mcr = sh.scan;
  K.mord = sh.abeg;
  K.v0lo = reinterpret_cast<int*>(sh.tcost);
  K.v0hi = reinterpret_cast<int*>(TC);
  K.stk = TS;
  K.adj = reinterpret_cast<int2*>(&t_fr[0][0]);
  const DecJob job = a.jobs[blockIdx.x];
  const int slot = job.slot;
  DecSlot st = a.slots[slot];
  DecPtrs p;
  p.cs = a.cur_state + (long long)slot * a.max_tok;
  p.cc = a.cur_cost + (long long)slot * a.max_tok;
  p.cp = a.cur_pos + (long long)slot * a.max_tok;
  p.arena = a.arena + (long long)slot * a.arena_cap;
  p.fg0 = a.front_g + ((long long)slot * 2) * a.max_tok;
  p.fg1 = p.fg0 + a.max_tok;
  p.slot = slot;
  const HbmTab T = hbm_tab(a, slot);
  if (threadIdx.x == 0) {
    sh.bad = 0;
    sh.n_links = 0;
    sh.lat_ovf = 0;
  }
  int arcs_eps = 0;
  bool lds = false;
  Prof pr;
  __shared__ long long prof_acc[PROF ? kDecProf : 1];
  __shared__ long long prof_snap[PROF ? kDecProf : 1];  // (VOSK_AMD_DEC_DEBUG 32: the frame's start values)
  pr.init(PROF && threadIdx.x == 0, prof_acc);

  // PruneActiveTokens every prune_interval frames, once the segment is
  // prune_start frames long or an arena prune_fill_pct full
  auto prune_due = [&](const DecSlot& s) {
    const bool full = a.prune_fill_pct <= 0 || s.frames >= a.prune_start ||
                      (long long)s.arena_used * 100 >= (long long)a.arena_cap * a.prune_fill_pct ||
                      (a.links && (long long)s.links_used * 100 >= (long long)a.link_cap * a.prune_fill_pct);
    return a.prune_interval > 0 && !s.err && s.frames - s.last_prune >= a.prune_interval && full;
  };
  // records the host reads as they come (host_gate): the pass runs before
  // this launch's frames, once the host has read every frame decoded so far
  // -- the compaction then moves only records it holds, and the frontier's
  // tokens (which the next frame's links point into) as one block, in order
  if (a.host_gate && !job.reset && job.host_read >= st.frames && prune_due(st)) {
    prune_segment<false>(a, sh, st, p, slot, pr);
    __syncthreads();
    if (sh.bad) st.err |= sh.bad;
    __syncthreads();
  }

  if (job.reset) {  // InitDecoding: start token, closure with cutoff = beam
    __syncthreads();
    if (st.err) {  // an overflow may have left unlisted entries
      hbm_clear_all(a, T);
      if (a.kaldi)
        for (int b = threadIdx.x; b < a.kb_cap; b += DT) {
          AG_ST(&a.kb_first[(long long)slot * a.kb_cap + b], kNoStamp);
          AG_ST(&a.kb_cnt[(long long)slot * a.kb_cap + b], 0);
        }
    }
    st.ntok = 0;
    st.cur_base = 0;
    st.arena_used = 0;
    st.frames = 0;
    st.offset_sum = 0.0;
    st.err = 0;
    st.links_used = 0;
    st.lat_ovf = 0;
    st.prune_from = 0;
    st.last_prune = 0;
    // Kaldi order: a new decoder's HashList holds 1000 buckets; InitDecoding
    // (reset 1, a Recognizer's next segment) keeps the size it grew to
    if (job.reset >= 2 || st.khash <= 0) st.khash = 1000;
    if (job.reset == 3 && a.lazy_id) {  // a new stream: OpenFST numbers from its start state
      int* ID = a.lazy_id + (long long)slot * a.lazy_ids;
      int* CA = a.lazy_cand + (long long)slot * a.lazy_ids;
      for (int i = threadIdx.x; i < a.lazy_ids; i += DT) {
        AG_ST(&ID[i], i == a.start_state ? 0 : -1);
        AG_ST(&CA[i], 0x7fffffff);
      }
      st.lazy_count = 1;
      vm_drain();
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      sh.n_new_l = 0;
      sh.n_new_g = 0;
      sh.n_front = 0;
      sh.n_links = 0;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const Relax r = relax(a, sh, t, T, a.start_state, 0.0f, -1,
                            ((unsigned)a.sinfo[a.start_state].z - (unsigned)a.sinfo[a.start_state].y) != 0);
      t.fr0[0] = r.slot;
      sh.n_front = 1;
      if (a.kaldi) {  // creation index 0
        if (r.slot >= 0) t.hst[r.slot] = 0;
        else AG_ST(&T.stamp[~r.slot], 0);
        AG_ST(&a.kord[(long long)slot * a.kord_cap], r.slot);
      }
    }
    if (a.kaldi) {
      vm_drain();
      __syncthreads();
      kaldi_nonemitting(a, sh, t, T, p, st, K, slot, st.khash, a.beam, 1, &arcs_eps, pr);
    } else {
      eps_closure(a, sh, t, T, p, st, a.beam, 1, &arcs_eps, pr);
    }
    float b;
    int nl = 0;
    float mxc;
    commit(a, sh, t, p, st, TS, TC, &lds, a.beam, &b, slot, &nl, false, pr, &mxc);
    // every current token's cost is below the commit's cutoff (GetCutoff's
    // shortcut); Kaldi order keeps tokens above it: their largest cost
    st.commit_cutoff = a.kaldi ? mxc : a.beam;
    frame_done(a, sh, st, slot, 0, a.beam, 0.0f, nl);
  } else if (st.ntok > 0 && st.ntok <= kTokLds) {
    for (int i = threadIdx.x; i < st.ntok; i += DT) {
      TS[i] = AG_LD(&p.cs[i]);
      TC[i] = AG_LD(&p.cc[i]);
    }
    lds = true;
  }

  // log-likelihood rows staged in LDS: row f+1 is loaded into registers
  // while frame f is processed and written to L once frame f's emitting
  // expansion no longer reads it (just before its commit)
  constexpr int kLlhRegs = kLlhLds / DT;
  const bool stage_llh = a.P <= kLlhLds;
  float nxt[kLlhRegs];
  if (stage_llh && job.nframes > 0) {
    const float* llh0 = a.llh + (size_t)job.llh_row0 * a.P;
    for (int i = threadIdx.x; i < a.P; i += DT) L[i] = llh0[i];
  }
  for (int f = 0; f < job.nframes; f++) {
    if (st.ntok == 0 || st.err) break;
    const long long t_frame0 = pr.on ? (long long)__builtin_amdgcn_s_memtime() : 0;
    if (pr.on && threadIdx.x == 0) sh.kbig = 0;
    if (PROF && pr.on && (a.debug & 32))
      for (int i = 0; i < kDecProf; i++) prof_snap[i] = pr.acc[i];
    const float* llh = a.llh + (size_t)(job.llh_row0 + f) * a.P;
    const float* Lp = stage_llh ? L : llh;
    const bool pf = stage_llh && f + 1 < job.nframes;
    if (pf) {
      const float* nrow = llh + a.P;
#pragma unroll
      for (int r = 0; r < kLlhRegs; r++) {
        const int i = threadIdx.x + r * DT;
        nxt[r] = i < a.P ? nrow[i] : 0.0f;
      }
    }
    const int ntok = st.ntok;
    const TokView tv{p.cs, p.cc, TS, TC, lds};
    // ---- GetCutoff (best token: min (cost, state), kept by the previous commit)
    const unsigned long long bk = st.best_key;
    const float best = funord((uint32_t)(bk >> 32));
    // the best token: its state (order-independent form), or its list
    // position (Kaldi order: the first minimum in list order, best_elem)
    const int bk_lo = (int)(unsigned)(bk & 0xffffffffu);
    const int best_state = !a.kaldi ? bk_lo : lds ? TS[bk_lo] : AG_LD(&p.cs[bk_lo]);
    if (a.kaldi) {  // PossiblyResizeHash(tok_cnt): the size the next frame's tokens hash with
      const int nsz = (int)((float)ntok * 2.0f);
      if (nsz > st.khash) st.khash = nsz;
      if (st.khash > a.kb_cap) {  // (cannot happen: tokens <= max_tok, kb_cap > 2 * max_tok)
        st.khash = a.kb_cap;
        if (threadIdx.x == 0) sh.bad |= 1;
      }
    }
    const float beam_cutoff = best + a.beam;
    float max_cut = __int_as_float(0x7f800000), min_cut = __int_as_float(0x7f800000);
    float adaptive, cutoff;
    // The k-th smallest cost is only needed when it can change the outcome:
    // max_cut < beam_cutoff  <=>  more than max_active costs are < beam_cutoff,
    // min_cut > beam_cutoff  <=>  at most min_active costs are <= beam_cutoff.
    bool need_max = ntok > a.max_active, need_min = ntok > a.min_active && a.min_active > 0;
    const bool regs = ntok <= DT * kCutRegs;
    CostRegs cr;
    // every token's cost is below the last commit's cutoff: when that is at
    // most beam_cutoff, all ntok are < (and <=) beam_cutoff without counting
    // (Kaldi order: commit_cutoff is the largest token cost instead)
    const bool all_in = a.kaldi ? st.commit_cutoff < beam_cutoff && !(a.debug & 2) : st.commit_cutoff <= beam_cutoff;
    // the costs in registers for the radix passes (also when the count below is skipped)
    if ((need_max || need_min) && regs) cr.load(tv, ntok);
    if ((need_max || need_min) && !all_in) {
      unsigned long long cnt = 0;  // (# cost < beam_cutoff) << 32 | # cost <= beam_cutoff
      if (regs) {
#pragma unroll
        for (int r = 0; r < kCutRegs; r++) {
          const float c = cr.c[r];
          if ((int)threadIdx.x + r * DT < ntok)
            cnt += ((unsigned long long)(c < beam_cutoff) << 32) | (unsigned)(c <= beam_cutoff);
        }
      } else {
        for (int b0 = 0; b0 < ntok; b0 += DT * kCutRegs) {
          CostRegs blk;
          blk.load(tv, ntok, b0);
#pragma unroll
          for (int r = 0; r < kCutRegs; r++) {
            const float c = blk.c[r];
            if (b0 + (int)threadIdx.x + r * DT < ntok)
              cnt += ((unsigned long long)(c < beam_cutoff) << 32) | (unsigned)(c <= beam_cutoff);
          }
        }
      }
      cnt = block_sum_u64(sh, cnt);
      const int n_lt = (int)(cnt >> 32), n_le = (int)(unsigned)(cnt & 0xffffffffu);
      need_max = need_max && n_lt > a.max_active;
      need_min = need_min && n_le <= a.min_active;
    } else {
      __syncthreads();  // the LLH row staged above is read by wave 0 below
    }
    if (all_in) need_min = false;  // n_le = ntok > min_active (need_max stays ntok > max_active)
    auto kth = [&](int k) {
      return regs ? kth_smallest<true>(sh, tv, cr, ntok, k) : kth_smallest<false>(sh, tv, cr, ntok, k);
    };
    if (need_max) max_cut = kth(a.max_active);
    if (max_cut < beam_cutoff) {
      adaptive = max_cut - best + a.beam_delta;
      cutoff = max_cut;
    } else {
      if (ntok > a.min_active)
        min_cut = a.min_active == 0 ? best
                  : need_min ? kth(a.min_active)
                             : beam_cutoff;  // proven <= beam_cutoff: the exact value is unused
      if (min_cut > beam_cutoff) {
        adaptive = min_cut - best + a.beam_delta;
        cutoff = min_cut;
      } else {
        adaptive = a.beam;
        cutoff = beam_cutoff;
      }
    }
    const float cost_offset = -best;
    pr.mark(0);
    // ---- ProcessEmitting: Kaldi's seed from the best token's arcs (wave 0)
    if (threadIdx.x < 64) {
      float sd = __int_as_float(0x7f800000);
      const int4 si = a.sinfo[best_state];
      for (int arc = si.x + (int)threadIdx.x; arc < si.y; arc += 64) {
        const int4 A = a.arcs[arc];
        const float nw = ((__int_as_float(A.y) + cost_offset) - Lp[A.z]) + best;
        sd = fminf(sd, nw + adaptive);
      }
      sd = wave_min_f(sd);
      if (threadIdx.x == 0) {
        sh.seed = sd;
        sh.n_new_l = 0;
        sh.n_new_g = 0;
        sh.n_front = 0;
        sh.n_links = 0;
      }
    }
    __syncthreads();
    pr.mark(1);
    const float seed = sh.seed;
    int examined = 0;
    const bool defer = a.links != nullptr && a.link_cap - st.links_used >= kDeferHeadroom;
    float next_cutoff, new_best;
    // one emitting pass relaxing below the seed bound (a superset), then the
    // epsilon closure; tokens whose best cost is not below the final
    // next_cutoff stay as dead list entries (never expanded: cost >= cutoff)
    // and are dropped at commit -- exactly the tokens a relax-below-
    // next_cutoff pass creates, with the same keys.  Without a finite seed
    // the exact two-pass form runs.
    if (a.kaldi) {
      int nc = 0;
      next_cutoff = expand_emitting_kaldi(a, sh, t, T, p, tv, ntok, cutoff, cost_offset, Lp, seed, adaptive,
                                          &examined, st, slot, &nc, defer, L, pr);
      pr.count(11, sh.n_new_g);
      kaldi_nonemitting(a, sh, t, T, p, st, K, slot, st.khash, next_cutoff, nc, &arcs_eps, pr);
    } else if (seed != __int_as_float(0x7f800000)) {
      const float m = expand_emitting(a, sh, t, T, p, tv, ntok, cutoff, cost_offset, Lp, 1, seed, adaptive,
                                      &examined, st, slot, defer, pr);
      next_cutoff = seed;
      if (m + adaptive < next_cutoff) next_cutoff = m + adaptive;
    } else {
      const float m = expand_emitting(a, sh, t, T, p, tv, ntok, cutoff, cost_offset, Lp, 0, 0.0f, adaptive,
                                      &examined, st, slot, false, pr);
      next_cutoff = seed;
      if (m + adaptive < next_cutoff) next_cutoff = m + adaptive;
      int dummy = 0;
      expand_emitting(a, sh, t, T, p, tv, ntok, cutoff, cost_offset, Lp, 1, next_cutoff, adaptive, &dummy, st,
                      slot, defer, pr);
    }
    if (!a.kaldi) {
      __syncthreads();
      pr.mark(2);
      pr.count(11, sh.n_new_g);  // tokens the emitting pass created in the HBM table
      eps_closure(a, sh, t, T, p, st, next_cutoff, sh.n_front, &arcs_eps, pr);
    }
    __syncthreads();
    pr.mark(5);
    if (pf) {  // L is not read again in this frame
#pragma unroll
      for (int r = 0; r < kLlhRegs; r++) {
        const int i = threadIdx.x + r * DT;
        if (i < a.P) L[i] = nxt[r];
      }
    }
    int nl = 0;
    float mxc;
    commit(a, sh, t, p, st, TS, TC, &lds, next_cutoff, &new_best, slot, &nl, defer, pr, &mxc);
    st.commit_cutoff = a.kaldi ? mxc : next_cutoff;
    pr.count(15, 1);
    frame_done(a, sh, st, slot, st.frames + 1, next_cutoff, cost_offset, nl);
    st.offset_sum += (double)cost_offset;
    st.frames++;
    if (threadIdx.x == 0 && a.stats) {
      FrameStat fs;
      fs.ntok_in = ntok;
      fs.ntok_out = st.ntok;
      fs.arcs_emit = examined;
      fs.arcs_eps = arcs_eps;
      fs.best = new_best;
      fs.cutoff = cutoff;
      fs.next_cutoff = next_cutoff;
      fs.adaptive_beam = adaptive;
      a.stats[job.stats_row0 + f] = fs;
    }
    arcs_eps = 0;
    __syncthreads();
    if (sh.bad) st.err |= sh.bad;
    if (pr.on) {  // whole-frame clocks, all frames and the big-queue ones
      const long long dt = (long long)__builtin_amdgcn_s_memtime() - t_frame0;
      pr.count(71, dt);
      if (sh.kbig) pr.count(72, dt);
      // development (VOSK_AMD_DEC_DEBUG 32): the phases of the big-queue frames only
      if (PROF && (a.debug & 32) && !sh.kbig)
        for (int i = 0; i < 71; i++) pr.acc[i] = prof_snap[i];
    }
  }
  __syncthreads();
  if (sh.bad) st.err |= sh.bad;
  if (st.ntok == 0 && !st.err) st.err |= 4;
  // PruneActiveTokens at the end of a launch (host_gate: at the start of one)
  if (!a.host_gate && prune_due(st)) {
    pr.mark(10);
    prune_segment<false>(a, sh, st, p, slot, pr);
    __syncthreads();
    if (sh.bad) st.err |= sh.bad;
  }
  pr.mark(10);
  if (threadIdx.x == 0) a.slots[slot] = st;
  if (pr.on)
    for (int i = 0; i < kDecProf; i++) a.prof[slot * kDecProf + i] += pr.acc[i];
}

// the final prune of segments that end (before their lattice copy), one
// workgroup per listed stream
__global__ __launch_bounds__(DT) void prune_final_kernel(DecArgs a, const int* slots, int use_final) {
  __shared__ DecShared sh;
  const int slot = slots[blockIdx.x];
  DecSlot st = a.slots[slot];
  DecPtrs p;
  p.cs = a.cur_state + (long long)slot * a.max_tok;
  p.cc = a.cur_cost + (long long)slot * a.max_tok;
  p.cp = a.cur_pos + (long long)slot * a.max_tok;
  p.arena = a.arena + (long long)slot * a.arena_cap;
  p.fg0 = a.front_g + ((long long)slot * 2) * a.max_tok;
  p.fg1 = p.fg0 + a.max_tok;
  Prof pr;
  pr.init(false, nullptr);
  if (threadIdx.x == 0) sh.bad = 0;
  __syncthreads();
  prune_segment<true>(a, sh, st, p, slot, pr, use_final != 0);
  __syncthreads();
  if (sh.bad) st.err |= sh.bad;
  if (threadIdx.x == 0) a.slots[slot] = st;
}

void LaunchPruneFinal(const DecArgs& a, const int* slots, int n, bool use_final, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(prune_final_kernel, dim3(n), dim3(DT), 0, s, a, slots, use_final ? 1 : 0);
}

int DecoderLdsProbe() { return kMaxProbe; }

void LaunchDecode(const DecArgs& a, int njobs, hipStream_t s) {
  if (njobs <= 0) return;
  if (a.prof) hipLaunchKernelGGL(decode_kernel<true>, dim3(njobs), dim3(DT), 0, s, a);
  else hipLaunchKernelGGL(decode_kernel<false>, dim3(njobs), dim3(DT), 0, s, a);
}

// ---------------------------------------------------------------------------
// traceback: best end token (with final costs if any is final), then walk
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void traceback_kernel(TraceArgs a) {
  __shared__ unsigned long long red[4];
  __shared__ float redf[4][2];
  __shared__ int endpos;
  const int slot = a.req_slot[blockIdx.x];
  const DecSlot st = a.slots[slot];
  const int* cs = a.cur_state + (long long)slot * a.max_tok;
  const float* cc = a.cur_cost + (long long)slot * a.max_tok;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float bn = __int_as_float(0x7f800000), bf = __int_as_float(0x7f800000);
  for (int i = threadIdx.x; i < st.ntok; i += 256) {
    const float c = cc[i];
    bn = fminf(bn, c);
    const float fc = __int_as_float(a.sinfo[cs[i]].w);
    if (fc != __int_as_float(0x7f800000)) bf = fminf(bf, c + fc);
  }
  for (int o = 32; o > 0; o >>= 1) {
    bn = fminf(bn, __shfl_xor(bn, o, 64));
    bf = fminf(bf, __shfl_xor(bf, o, 64));
  }
  if (lane == 0) { redf[w][0] = bn; redf[w][1] = bf; }
  __syncthreads();
  bn = fminf(fminf(redf[0][0], redf[1][0]), fminf(redf[2][0], redf[3][0]));
  bf = fminf(fminf(redf[0][1], redf[1][1]), fminf(redf[2][1], redf[3][1]));
  const bool any_final = bf != __int_as_float(0x7f800000);
  const bool use_f = a.use_final && any_final;
  unsigned long long bk = kEmpty;
  for (int i = threadIdx.x; i < st.ntok; i += 256) {
    float c = cc[i];
    if (use_f) c = c + __int_as_float(a.sinfo[cs[i]].w);
    const unsigned long long k = ((unsigned long long)ford(c) << 32) | (unsigned)(a.tie_pos ? i : cs[i]);
    bk = k < bk ? k : bk;
  }
  bk = wave_min_u64(bk);
  if (lane == 0) red[w] = bk;
  if (threadIdx.x == 0) endpos = -1;
  __syncthreads();
  bk = red[0];
  for (int i = 1; i < 4; i++) bk = red[i] < bk ? red[i] : bk;
  if (a.tie_pos) {
    if (threadIdx.x == 0 && bk != kEmpty) endpos = (int)(unsigned)(bk & 0xffffffffu);
  } else {
    for (int i = threadIdx.x; i < st.ntok; i += 256)
      if (cs[i] == (int)(unsigned)(bk & 0xffffffffu)) endpos = i;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int n = 0;
    int* out = a.path + (long long)blockIdx.x * a.path_cap;
    if (endpos >= 0 && a.arc_sil) {
      // OnlineEndpoint TrailingSilenceLength: silence frames back from the best token
      const int4* arena = a.arena + (long long)slot * a.arena_cap;
      int k = st.cur_base + a.cur_pos[(long long)slot * a.max_tok + endpos];
      while (k >= 0) {
        const int4 e = arena[k];
        if (e.y < 0) break;
        const int c = a.arc_sil[e.y];
        if (c == 2) break;
        n += c;
        k = e.x;
      }
    } else if (endpos >= 0) {
      const int4* arena = a.arena + (long long)slot * a.arena_cap;
      int k = st.cur_base + a.cur_pos[(long long)slot * a.max_tok + endpos];
      while (k >= 0) {
        const int4 e = arena[k];
        if (e.y < 0) break;
        if (n < a.path_cap) out[n] = e.y;
        n++;
        k = e.x;
      }
    }
    a.path_len[blockIdx.x] = n;
    a.end_cost[blockIdx.x] = endpos >= 0 ? funord((uint32_t)(bk >> 32)) : __int_as_float(0x7f800000);
    a.final_rel[blockIdx.x] = any_final ? bf - bn : __int_as_float(0x7f800000);
    a.end_state[blockIdx.x] = endpos >= 0 ? cs[endpos] : -1;
  }
}

void LaunchTraceback(const TraceArgs& a, int n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(traceback_kernel, dim3(n), dim3(256), 0, s, a);
}

// HBM frame tables at engine construction: all slots empty
__global__ void init_tables_kernel(int* state, unsigned long long* key, int* stamp, long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    state[i] = -1;
    key[i] = kEmpty;
    stamp[i] = kNoStamp;
  }
}

void LaunchInitTables(int* state, unsigned long long* key, int* stamp, long long n, hipStream_t s) {
  if (n <= 0) return;
  long long blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(init_tables_kernel, dim3((unsigned)blocks), dim3(256), 0, s, state, key, stamp, n);
}

}  // namespace vamd
