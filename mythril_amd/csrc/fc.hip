// fc.hip — flat conjunctions on gfx950: tapes and Bool columns that are an AND of Bool model
// variables (negated or not) and comparisons of one model variable with a constant, evaluated
// without an interpreter.  After batch-level hoisting (lower.py lower_batch) this is the shape of
// most of a path's conjunction: the shared sub-terms are columns and what is left per path is the
// AND of their Bool columns plus a few word compares (C4's tapes: ~11 packed masks and 2-3
// compares).  On the G interpreter each (tape, 64-model tile) paid the tape frame (descriptor,
// early-exit test, program window) and ~6 threaded dispatches.
//
// One workgroup = one 64-model tile; its 4 waves take one tape group (FcRun.tpg tapes) each:
// grid.x = tiles, grid.y = quads of groups.  The prologue stages in LDS, once per workgroup, the
// variable rows the launch's compares read (256 B a limb row) and the tile's packed lane masks of
// the Bool variables the launch reads (8 B each).
//
// The scalar unit (one per CU, shared by its four SIMDs) bound the first versions of this
// kernel at ~190 scalar instructions a tape; the work is therefore laid out for the vector unit:
//  * Bool variables: lane k of a wave reads the k-th mask of the tape (k < 16; the host pads a
//    tape's list to 16 with its last entry, and lanes 16-63 repeat lanes 0-15) from LDS, negated
//    where the list says so (bit 0 of its LDS offset), and a four-step DPP AND across the row of
//    16 lanes leaves the AND of all 16 in lane 15: one vector load, one LDS read, ~12 VALU;
//  * a compare reads its variable's limbs from LDS as 64-bit pairs and compares them with the
//    constant's (two VALU compares a pair: x < c and x == c lane masks); the predicate is three
//    accept masks over (x < c, x == c, x > c) (host-encoded, signed compares with the sign bit
//    pre-flipped), so no scalar branching on it.  Variables of one or two limbs (most hoisted
//    words are narrow) take one pair, wider ones four.
// A descriptor with bit 31 of n_mask set is the negation of its conjunction: an OR of atoms.
// Modes: 0 first hit (best[] atomicMin, early exit on best[]), 1 verdict bytes, 3 Bool columns
// (packed lane mask stored, and the 0/1 row when a HIP C++ kernel reads rows or the column has no
// mask index).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qs_launch.h"

namespace mq {

__device__ __forceinline__ uint32_t uniform(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// 64-model tiles per workgroup (each wave runs its tape group over all of them)
constexpr int FC_TILES = 4;

// lane 15 of each row of 16 = the AND of the row's 16 values of lo and of hi: v_and_b32 with a DPP
// row_shr source (1, 2, 4, 8), lanes whose source lies before the row are not written (they keep
// their own value); one wait state pads each VALU write -> DPP read of the same register
__device__ __forceinline__ void and_row16(uint32_t& lo, uint32_t& hi) {
  asm volatile(
      "s_nop 1\n"
      "v_and_b32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n"
      "v_and_b32_dpp %1, %1, %1 row_shr:1 row_mask:0xf bank_mask:0xf\n"
      "s_nop 0\n"
      "v_and_b32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n"
      "v_and_b32_dpp %1, %1, %1 row_shr:2 row_mask:0xf bank_mask:0xf\n"
      "s_nop 0\n"
      "v_and_b32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n"
      "v_and_b32_dpp %1, %1, %1 row_shr:4 row_mask:0xf bank_mask:0xf\n"
      "s_nop 0\n"
      "v_and_b32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf\n"
      "v_and_b32_dpp %1, %1, %1 row_shr:8 row_mask:0xf bank_mask:0xf\n"
      "s_nop 1"
      : "+v"(lo), "+v"(hi));
}

// The lane mask of (x ACCEPT c) over a staged variable for tile j of the workgroup (limb l of
// tile j at LDS row (q.slot + l) * FC_TILES + j, the sign bit of a signed compare flipped by q.f,
// c pre-flipped): 64-bit compares of limb pairs, each higher pair refining the (lt, eq) of the
// ones below; per lane, the accept bit of the case (x < c, x == c, x > c) it falls in, so the
// predicate costs no scalar work
__device__ __forceinline__ uint64_t fc_cmp(const uint32_t* lds_lane, const FcCmpHead& h, const FcCmp* __restrict__ qp,
                                           int j) {
  const uint32_t* p = lds_lane + (h.slot * FC_TILES + (uint32_t)j) * 64u;
  constexpr int R = FC_TILES * 64;   // one limb further
  const uint64_t x0 = ((uint64_t)(p[R] ^ (uint32_t)(h.f01 >> 32)) << 32) | (p[0] ^ (uint32_t)h.f01);
  bool lt = x0 < h.c01, eq = x0 == h.c01;
  if (h.nl > 2) {   // (eight staged limbs: the other pairs)
    const FcCmpTail t = qp->t;
#pragma unroll
    for (int k = 0; k < 3; k++) {   // limbs 2-3, 4-5, 6-7: each pair above the ones before
      const uint64_t x = ((uint64_t)(p[(2 * k + 3) * R] ^ t.f[2 * k + 1]) << 32) | (p[(2 * k + 2) * R] ^ t.f[2 * k]);
      const uint64_t c = ((uint64_t)t.c[2 * k + 1] << 32) | t.c[2 * k];
      lt = x < c || (x == c && lt);
      eq = x == c && eq;
    }
  }
  const uint32_t bit = lt ? 1u : (eq ? 2u : 4u);
  return __ballot((h.accept & bit) != 0);
}

// One workgroup = FC_TILES consecutive 64-model tiles; each of its 4 waves runs one tape group
// over all of them (lane l holds model l of every tile): a tape's descriptor, early-exit test,
// mask list and compare constants are scalar work paid once for FC_TILES tiles, and the mask AND
// of all FC_TILES tiles is one DPP reduction (lanes 16 j .. 16 j + 15 reduce tile j's masks).
__global__ __launch_bounds__(256) void fc_kernel(const FcTape* __restrict__ tapes, const uint32_t* __restrict__ mask_lds,
                                                 const FcCmp* __restrict__ cmps, const uint32_t* __restrict__ vars,
                                                 const uint64_t* __restrict__ masks_in,
                                                 const int32_t* __restrict__ best_ro,
                                                 const uint32_t* __restrict__ stage_rows,
                                                 const uint32_t* __restrict__ stage_masks, FcRun r) {
  extern __shared__ uint32_t lds[];
  const uint32_t wave = uniform(threadIdx.x >> 6);
  const int64_t tile0 = (int64_t)blockIdx.x * FC_TILES;
  const int64_t m0 = tile0 * 64;
  const int lane = threadIdx.x & 63;
  // stage the compared rows (LDS row s * FC_TILES + j = slot s of tile j, 256 B) and the tiles'
  // masks (after the rows: tile j's mask k at 8 (j * n_smask + k)); wave w stages tile w's rows
  {
    const int j = (int)wave;
    const int64_t mj = min(m0 + 64 * j + lane, r.M - 1);
    for (int s0 = 0; s0 < r.n_stage; s0 += 8) {
      uint32_t v[8];
#pragma unroll
      for (int k = 0; k < 8; k++) v[k] = __builtin_nontemporal_load(vars + (int64_t)stage_rows[min(s0 + k, r.n_stage - 1)] * r.M + mj);
#pragma unroll
      for (int k = 0; k < 8; k++)
        if (s0 + k < r.n_stage) lds[((s0 + k) * FC_TILES + j) * 64 + lane] = v[k];
    }
  }
  uint64_t* lmask = reinterpret_cast<uint64_t*>(lds + r.n_stage * FC_TILES * 64);
  const int64_t tiles = (r.M + 63) / 64;
  for (int i = (int)threadIdx.x; i < FC_TILES * r.n_smask; i += 256) {
    const int j = i / r.n_smask, k = i - j * r.n_smask;
    const int64_t tj = min(tile0 + j, tiles - 1);
    lmask[i] = masks_in[tj * (int64_t)r.n_bool_masks + stage_masks[k]];
  }
  __syncthreads();
  uint64_t valid[FC_TILES];
  int32_t first[FC_TILES];
#pragma unroll
  for (int j = 0; j < FC_TILES; j++) {
    valid[j] = __ballot(m0 + 64 * j + lane < r.M);
    first[j] = (int32_t)(r.index_base + m0 + 64 * j);
  }
  const int t0 = ((int)blockIdx.y * 4 + (int)wave) * r.tpg;
  const int t1 = min(r.n, t0 + r.tpg);
  if (t0 >= t1) return;
  const uint32_t* lds_lane = lds + lane;
  // lane l reads tile (l / 16)'s copy of the masks
  const char* lmask_b = reinterpret_cast<const char*>(lmask + (lane >> 4) * r.n_smask);
  unsigned long long skipped_nodes = 0, skipped_ops = 0;
  int skipped = 0;
  FcTape d = tapes[t0];
  for (int t = t0; t < t1; t++) {
    // the next tape's descriptor is requested with this one's first loads
    const FcTape dn = tapes[min(t + 1, t1 - 1)];
    // best[] only decreases within a launch: a stale (scalar-cache) value only skips less
    if (r.mode == 0 && r.early_exit && first[0] >= best_ro[d.out]) {
      skipped++;
      skipped_nodes += d.n_nodes;
      skipped_ops += d.alg_ops;
      d = dn;
      continue;
    }
    uint64_t acc[FC_TILES];
#pragma unroll
    for (int j = 0; j < FC_TILES; j++) acc[j] = valid[j];
    // Bool variables, 16 at a time: lane l takes entry l % 16 of the list (LDS offset, bit 0:
    // negated) for tile l / 16
    const uint32_t n_mask = d.n_mask & 0x7FFFFFFFu;
    for (uint32_t e0 = 0; e0 < n_mask; e0 += 16) {
      const uint32_t e = mask_lds[d.mask_off + e0 + (lane & 15)];
      uint64_t w = *reinterpret_cast<const uint64_t*>(lmask_b + (e & ~7u));
      if (e & 1u) w = ~w;
      uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
      and_row16(lo, hi);
#pragma unroll
      for (int j = 0; j < FC_TILES; j++)
        acc[j] &= ((uint64_t)__builtin_amdgcn_readlane(hi, 16 * j + 15) << 32) |
                  (uint32_t)__builtin_amdgcn_readlane(lo, 16 * j + 15);
    }
    for (uint32_t k = 0; k < d.n_cmp; k++) {
      const FcCmp* qp = cmps + d.cmp_off + k;
      const FcCmpHead h = qp->h;
#pragma unroll
      for (int j = 0; j < FC_TILES; j++) acc[j] &= fc_cmp(lds_lane, h, qp, j);
    }
    if (d.n_mask >> 31) {   // a negated conjunction (an OR of atoms, De Morgan)
#pragma unroll
      for (int j = 0; j < FC_TILES; j++) acc[j] = ~acc[j] & valid[j];
    }
#pragma unroll
    for (int j = 0; j < FC_TILES; j++) {
      const int64_t mj = m0 + 64 * j + lane;
      if (r.mode == 0) {
        if (acc[j]) {   // the lowest tile with a hit has the lowest model
          if (lane == 0) atomicMin(r.best + d.out, first[j] + (int32_t)__builtin_ctzll(acc[j]));
          break;
        }
      } else if (r.mode == 1) {
        if (mj < r.M) r.verdicts[(int64_t)d.out * r.M + mj] = (uint8_t)((acc[j] >> lane) & 1u);
      } else if (mj - lane < r.M) {
        if (d.mask_out >= 0 && lane == 0) r.masks_out[(tile0 + j) * (int64_t)r.n_bool_masks + d.mask_out] = acc[j];
        if ((r.bool_rows || d.mask_out < 0) && mj < r.M) r.vars_out[(int64_t)d.out * r.M + mj] = (uint32_t)((acc[j] >> lane) & 1u);
      }
    }
    d = dn;
  }
  // counters: the group's totals (FcRun prefix sums over the tapes) less the skipped tapes', times
  // the workgroup's valid models
  if (lane == 0 && r.counters) {
    unsigned long long nv = 0;
#pragma unroll
    for (int j = 0; j < FC_TILES; j++) nv += (unsigned long long)__popcll(valid[j]);
    const unsigned long long runs = (unsigned long long)(t1 - t0 - skipped);
    const unsigned long long nodes = r.prefix[2 * t1] - r.prefix[2 * t0] - skipped_nodes;
    const unsigned long long ops = r.prefix[2 * t1 + 1] - r.prefix[2 * t0 + 1] - skipped_ops;
    unsigned long long* cnt = r.counters + ((blockIdx.x * 4 + wave + blockIdx.y) % kCounterSlots) * kCounterStride;
    if (r.mode != 3) atomicAdd(&cnt[0], runs * nv);   // (tape evaluations; a column is not one)
    atomicAdd(&cnt[1], nodes * nv);
    atomicAdd(&cnt[2], ops * nv);
  }
}

// ---- unary atoms: the transform of an 8-limb value (w uniform, bits above w zero) --------------
__device__ __forceinline__ void fx_mask(uint32_t y[8], uint32_t w) {
#pragma unroll
  for (int l = 0; l < 8; l++) {
    const uint32_t lo = 32u * l;
    if (w <= lo) y[l] = 0u;
    else if (w < lo + 32u) y[l] &= (1u << (w - lo)) - 1u;
  }
}
// bits [w_in, w_out) set (sign-fill) where s
__device__ __forceinline__ void fx_fill(uint32_t y[8], uint32_t w_in, uint32_t w_out, bool s) {
#pragma unroll
  for (int l = 0; l < 8; l++) {
    const uint32_t lo = 32u * l;
    const uint32_t a = max(w_in, lo), b = min(w_out, lo + 32u);
    if (a < b) {
      const uint32_t m = (b - a == 32u ? 0xFFFFFFFFu : ((1u << (b - a)) - 1u)) << (a - lo);
      if (s) y[l] |= m;
    }
  }
}
__device__ __forceinline__ bool fx_sign(const uint32_t y[8], uint32_t w) {
  const uint32_t li = (w - 1u) >> 5, bi = (w - 1u) & 31u;
  uint32_t t = 0;
#pragma unroll
  for (int l = 0; l < 8; l++)
    if ((uint32_t)l == li) t = y[l];
  return (t >> bi) & 1u;
}
// y >> k over 256 bits, `top` shifted in from above (0 or all ones)
__device__ __forceinline__ void fx_shr(uint32_t y[8], uint32_t k, uint32_t top) {
  if (k >= 256u) {
#pragma unroll
    for (int l = 0; l < 8; l++) y[l] = top;
    return;
  }
  const uint32_t q = k >> 5, r = k & 31u;
  if (q & 4u) {
#pragma unroll
    for (int l = 0; l < 8; l++) y[l] = l + 4 < 8 ? y[l + 4] : top;
  }
  if (q & 2u) {
#pragma unroll
    for (int l = 0; l < 8; l++) y[l] = l + 2 < 8 ? y[l + 2] : top;
  }
  if (q & 1u) {
#pragma unroll
    for (int l = 0; l < 8; l++) y[l] = l + 1 < 8 ? y[l + 1] : top;
  }
  if (r) {
#pragma unroll
    for (int l = 0; l < 8; l++) {
      const uint32_t hi = l + 1 < 8 ? y[l + 1] : top;
      y[l] = (uint32_t)((((uint64_t)hi << 32) | y[l]) >> r);
    }
  }
}
__device__ __forceinline__ void fx_shl(uint32_t y[8], uint32_t k) {
  if (k >= 256u) {
#pragma unroll
    for (int l = 0; l < 8; l++) y[l] = 0u;
    return;
  }
  const uint32_t q = k >> 5, r = k & 31u;
  if (q & 4u) {
#pragma unroll
    for (int l = 7; l >= 0; l--) y[l] = l >= 4 ? y[l - 4] : 0u;
  }
  if (q & 2u) {
#pragma unroll
    for (int l = 7; l >= 0; l--) y[l] = l >= 2 ? y[l - 2] : 0u;
  }
  if (q & 1u) {
#pragma unroll
    for (int l = 7; l >= 0; l--) y[l] = l >= 1 ? y[l - 1] : 0u;
  }
  if (r) {
#pragma unroll
    for (int l = 7; l >= 0; l--) {
      const uint32_t lo = l >= 1 ? y[l - 1] : 0u;
      y[l] = (uint32_t)((((uint64_t)y[l] << 32) | lo) >> (32u - r));
    }
  }
}
// two's complement negation at width w
__device__ __forceinline__ void fx_neg(uint32_t y[8], uint32_t w) {
  uint64_t cy = 1;
#pragma unroll
  for (int l = 0; l < 8; l++) {
    const uint64_t t = (uint64_t)(~y[l]) + cy;
    y[l] = (uint32_t)t;
    cy = t >> 32;
  }
  fx_mask(y, w);
}
// y = y / d (quotient limbs), returns y mod d; 0 < d < 2^21: each step's dividend r * 2^32 + limb
// is below 2^53, so the fp64 estimate of its quotient is exact up to one unit either way
__device__ __forceinline__ uint32_t fx_divmod(uint32_t y[8], uint32_t d) {
  const double inv = 1.0 / (double)d;
  uint32_t r = 0;
#pragma unroll
  for (int l = 7; l >= 0; l--) {
    const uint64_t v = ((uint64_t)r << 32) | y[l];
    uint32_t q = (uint32_t)((double)v * inv);
    int64_t rem = (int64_t)(v - (uint64_t)q * d);
    if (rem < 0) {
      q--;
      rem += d;
    } else if (rem >= (int64_t)d) {
      q++;
      rem -= d;
    }
    y[l] = q;
    r = (uint32_t)rem;
  }
  return r;
}
__device__ __forceinline__ void fx_apply(uint32_t y[8], const FcXf& X) {
  for (uint32_t k = 0; k < X.n; k++) {
    const FcXop o = X.op[k];
    const uint32_t code = o.code & 0xFFu, w = o.code >> 8;
    if (code == FX_SEXT) {
      fx_fill(y, w, o.p0, fx_sign(y, w));
    } else if (code == FX_EXTRACT) {
      fx_shr(y, o.p0, 0u);
      fx_mask(y, o.p1);
    } else if (code == FX_LSHR) {
      fx_shr(y, o.p0 >= w ? 256u : o.p0, 0u);
    } else if (code == FX_SHL) {
      fx_shl(y, o.p0 >= w ? 256u : o.p0);
      fx_mask(y, w);
    } else if (code == FX_ASHR) {
      const bool s = fx_sign(y, w);
      fx_fill(y, w, 256u, s);
      fx_shr(y, min(o.p0, w - 1u), s ? 0xFFFFFFFFu : 0u);
      fx_mask(y, w);
    } else if (code == FX_UREM || code == FX_UDIV) {
      const uint32_t r = fx_divmod(y, o.p0);
      if (code == FX_UREM) {
#pragma unroll
        for (int l = 0; l < 8; l++) y[l] = l == 0 ? r : 0u;
      }
    } else {   // FX_SMOD / FX_SREM / FX_SDIV: on |y| and |d|, then the signs (SMT-LIB)
      const bool neg = fx_sign(y, w), dneg = o.p1 != 0u;
      if (neg) fx_neg(y, w);
      const uint32_t r = fx_divmod(y, o.p0);
      if (code == FX_SDIV) {
        if (neg != dneg) fx_neg(y, w);
      } else {
#pragma unroll
        for (int l = 0; l < 8; l++) y[l] = l == 0 ? r : 0u;
        if (code == FX_SREM) {
          if (neg) fx_neg(y, w);
        } else if (r != 0u) {
          // x >= 0, d > 0: r; x < 0, d > 0: |d| - r; x >= 0, d < 0: r - |d|; x < 0, d < 0: -r
          if (neg != dneg) {
            y[0] = o.p0 - r;
            if (dneg) fx_neg(y, w);
          } else if (neg) {
            fx_neg(y, w);
          }
        }
      }
    }
  }
}
// the accept bit of y (8 limbs, signed compares pre-flipped by f) against the atom's constant
__device__ __forceinline__ uint32_t fx_case(const uint32_t y[8], const FcCmpHead& h, const FcCmpTail& t) {
  const uint64_t x0 = (((uint64_t)y[1] << 32) | y[0]) ^ h.f01;
  bool lt = x0 < h.c01, eq = x0 == h.c01;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const uint64_t xv = ((uint64_t)(y[2 * k + 3] ^ t.f[2 * k + 1]) << 32) | (y[2 * k + 2] ^ t.f[2 * k]);
    const uint64_t c = ((uint64_t)t.c[2 * k + 1] << 32) | t.c[2 * k];
    lt = xv < c || (xv == c && lt);
    eq = xv == c && eq;
  }
  return lt ? 1u : (eq ? 2u : 4u);
}

// Two-phase form for tapes (FcaArgs).  fc_kernel pays a tape's scalar frame, mask reduction and
// compares once per (tape, tile): ~110 instructions, and it can only compare variables staged in
// LDS.  Here a workgroup of FC_TILES tiles first evaluates the launch's DISTINCT compares (C4: 647
// compares in 200 tapes, 390 distinct; C3: 8 835 in 1 000, 6 626) into LDS lane masks: the atoms
// are grouped by variable, a wave loads a group's variable limbs for its FC_TILES tiles into
// registers once (any variable: nothing is staged) and compares them with each atom's constant.
// Then each wave takes chunks of 64 tapes, one tape per lane, and ANDs the tape's list of LDS masks
// (entries k-major per chunk: one coalesced load per entry) for the FC_TILES tiles.

// (MODE: the launch's r.mode as a template parameter, so the first-hit kernel carries none of the
// verdict / column store code and its loop-invariant addresses; XF: the launch has unary atoms --
// the transforms' registers made the kernel spill SGPRs and use scratch, so launches without one,
// every launch by default, run the instantiation without them)
template <int MODE, bool XF>
__global__ __launch_bounds__(256) void fca_kernel(const FcaGroup* __restrict__ groups, const FcCmp* __restrict__ atoms,
                                                  const FcXf* __restrict__ xfs,
                                                  const uint32_t* __restrict__ lists,
                                                  const uint32_t* __restrict__ chunk_off,
                                                  const uint32_t* __restrict__ tape_out,
                                                  const uint32_t* __restrict__ tape_metric,
                                                  const uint32_t* __restrict__ vars,
                                                  const uint64_t* __restrict__ masks_in,
                                                  const uint32_t* __restrict__ stage_masks, FcaArgs r) {
  static_assert(FC_TILES == 4, "the table entries are read and written as two 16-byte pairs");
  // the mask table: entry e of tile j at tab[e * FC_TILES + j] (an entry's four tiles in 32
  // bytes); entries: 0 all ones, 1 .. n_smask the Bool masks, then the atoms
  extern __shared__ __align__(16) uint64_t tab[];
  const uint32_t wave = uniform(threadIdx.x >> 6);
  const int64_t tile0 = (int64_t)blockIdx.x * FC_TILES;
  const int64_t m0 = tile0 * 64;
  const int lane = threadIdx.x & 63;
  const int64_t tiles = (r.M + 63) / 64;
  for (int i = (int)threadIdx.x; i < FC_TILES * (1 + r.n_smask); i += 256) {
    const int k = i / FC_TILES, j = i - k * FC_TILES;
    const int64_t tj = min(tile0 + j, tiles - 1);
    tab[i] = k == 0 ? ~0ull : masks_in[tj * (int64_t)r.n_bool_masks + stage_masks[k - 1]];
  }
  // phase 1: the atoms, a variable group at a time (wave w: groups w, w + 4, ...).  A compare's
  // lane masks are two VALU compares of 64-bit limb pairs into SGPR masks a tile; the accept
  // (canonical: 1 x < c, 2 x == c, 3 x <= c) selects them on the scalar unit; lane 0 stores the
  // atom's four tiles as two 16-byte LDS writes
  int64_t mj[FC_TILES];
#pragma unroll
  for (int j = 0; j < FC_TILES; j++) mj[j] = min(m0 + 64 * j + lane, r.M - 1);
  const int abase = 1 + r.n_smask;
  for (int g = (int)wave; g < r.n_groups; g += 4) {
    const FcaGroup G = groups[g];
    if (G.nl <= 2) {
      uint64_t x[FC_TILES];
#pragma unroll
      for (int j = 0; j < FC_TILES; j++)
        x[j] = ((uint64_t)vars[(int64_t)G.rows[1] * r.M + mj[j]] << 32) | vars[(int64_t)G.rows[0] * r.M + mj[j]];
      for (uint32_t a = G.first; a < G.first + G.count; a++) {
        const FcCmpHead h = atoms[a].h;
        uint64_t m[FC_TILES];
#pragma unroll
        for (int j = 0; j < FC_TILES; j++) {
          const uint64_t xv = x[j] ^ h.f01;
          const uint64_t lt = __ballot(xv < h.c01), eq = __ballot(xv == h.c01);
          m[j] = ((h.accept & 1u) ? lt : 0ull) | ((h.accept & 2u) ? eq : 0ull);
        }
        if (lane == 0) {
          ulonglong2* p = reinterpret_cast<ulonglong2*>(tab + (abase + (int)a) * FC_TILES);
          p[0] = make_ulonglong2(m[0], m[1]);
          p[1] = make_ulonglong2(m[2], m[3]);
        }
      }
    } else {
      uint32_t x[FC_TILES][8];
#pragma unroll
      for (int j = 0; j < FC_TILES; j++)
#pragma unroll
        for (int l = 0; l < 8; l++) x[j][l] = vars[(int64_t)G.rows[l] * r.M + mj[j]];
      for (uint32_t a = G.first; a < G.first + G.count; a++) {
        const FcCmpHead h = atoms[a].h;
        const FcCmpTail t = atoms[a].t;
        uint64_t m[FC_TILES];
        const uint32_t nx = XF ? xfs[a].n : 0u;
        if (XF && nx) {   // a unary atom: the transform of the variable, then the compare
          const FcXf X = xfs[a];
#pragma unroll
          for (int j = 0; j < FC_TILES; j++) {
            uint32_t y[8];
#pragma unroll
            for (int l = 0; l < 8; l++) y[l] = x[j][l];
            fx_apply(y, X);
            const uint64_t b = __ballot((h.accept & fx_case(y, h, t)) != 0u);
            m[j] = b;
          }
          if (lane == 0) {
            ulonglong2* p = reinterpret_cast<ulonglong2*>(tab + (abase + (int)a) * FC_TILES);
            p[0] = make_ulonglong2(m[0], m[1]);
            p[1] = make_ulonglong2(m[2], m[3]);
          }
          continue;
        }
#pragma unroll
        for (int j = 0; j < FC_TILES; j++) {
          const uint64_t x0 = (((uint64_t)x[j][1] << 32) | x[j][0]) ^ h.f01;
          bool lt = x0 < h.c01, eq = x0 == h.c01;
#pragma unroll
          for (int k = 0; k < 3; k++) {   // limbs 2-3, 4-5, 6-7: each pair above the ones before
            const uint64_t xv = ((uint64_t)(x[j][2 * k + 3] ^ t.f[2 * k + 1]) << 32) | (x[j][2 * k + 2] ^ t.f[2 * k]);
            const uint64_t c = ((uint64_t)t.c[2 * k + 1] << 32) | t.c[2 * k];
            lt = xv < c || (xv == c && lt);
            eq = xv == c && eq;
          }
          const uint64_t lm = __ballot(lt), em = __ballot(eq);
          m[j] = ((h.accept & 1u) ? lm : 0ull) | ((h.accept & 2u) ? em : 0ull);
        }
        if (lane == 0) {
          ulonglong2* p = reinterpret_cast<ulonglong2*>(tab + (abase + (int)a) * FC_TILES);
          p[0] = make_ulonglong2(m[0], m[1]);
          p[1] = make_ulonglong2(m[2], m[3]);
        }
      }
    }
  }
  __syncthreads();
  // phase 2: the tapes, one per lane
  uint64_t valid[FC_TILES];
#pragma unroll
  for (int j = 0; j < FC_TILES; j++) {
    const int64_t mt = m0 + 64 * j;
    valid[j] = mt >= r.M ? 0ull : (r.M - mt >= 64 ? ~0ull : ((1ull << (r.M - mt)) - 1ull));
  }
  const int32_t first0 = (int32_t)(r.index_base + m0);
  const int n_chunks = (r.n + 63) / 64;
  unsigned long long run_nodes = 0, run_ops = 0, runs = 0;
  for (int c = (int)wave; c < n_chunks; c += 4) {
    const int t = c * 64 + lane;
    const bool live = t < r.n;
    const uint32_t out = live ? tape_out[t] : 0u;
    const uint32_t row = out & 0x7FFFFFFFu;
    bool run = live;
    if (run && MODE == 0 && r.early_exit) run = first0 < r.best[row];   // (best[] only decreases)
    const uint32_t o0 = chunk_off[c], kmax = (chunk_off[c + 1] - o0) / 64u;
    uint64_t acc[FC_TILES];
#pragma unroll
    for (int j = 0; j < FC_TILES; j++) acc[j] = valid[j];
    const uint32_t* lp = lists + o0 + lane;
    for (uint32_t k = 0; k < kmax; k++) {
      const uint32_t e = lp[64u * k];
      const uint32_t idx = e & 0x7FFFFFFFu;
      const uint64_t neg = (e >> 31) ? ~0ull : 0ull;
      const ulonglong2* p = reinterpret_cast<const ulonglong2*>(tab + idx * FC_TILES);
      const ulonglong2 q0 = p[0], q1 = p[1];
      acc[0] &= q0.x ^ neg;
      acc[1] &= q0.y ^ neg;
      acc[2] &= q1.x ^ neg;
      acc[3] &= q1.y ^ neg;
    }
    if (out >> 31) {   // a negated conjunction (an OR of atoms)
#pragma unroll
      for (int j = 0; j < FC_TILES; j++) acc[j] = ~acc[j] & valid[j];
    }
    if (run) {
      runs++;
      run_nodes += tape_metric[2 * t];
      run_ops += tape_metric[2 * t + 1];
      if (MODE == 3) {
        // a Bool column: its tiles' lane masks (its 0/1 row, where one is needed, below)
        const int32_t mo = r.col_mask[t];
        if (mo >= 0) {
#pragma unroll
          for (int j = 0; j < FC_TILES; j++) {
            if (m0 + 64 * j >= r.M) break;
            r.bool_masks_out[(tile0 + j) * (int64_t)r.n_bool_masks + mo] = acc[j];
          }
        }
      } else if (MODE == 0) {
#pragma unroll
        for (int j = 0; j < FC_TILES; j++)
          if (acc[j]) {   // the lowest tile with a hit has the lowest model
            atomicMin(r.best + row, first0 + 64 * j + (int32_t)__builtin_ctzll(acc[j]));
            break;
          }
      } else {
        // verdict bytes: four models a dword where the row's whole tile lies below M, else bytes
#pragma unroll
        for (int j = 0; j < FC_TILES; j++) {
          const int64_t mt = m0 + 64 * j;
          if (mt >= r.M) break;
          uint8_t* vrow = r.verdicts + (int64_t)row * r.M + mt;
          if (r.M - mt >= 64 && ((((uintptr_t)vrow) & 3u) == 0)) {
            for (int q = 0; q < 16; q++) {
              const uint32_t b = (uint32_t)(acc[j] >> (4 * q)) & 0xFu;
              reinterpret_cast<uint32_t*>(vrow)[q] = (b & 1u) | ((b & 2u) << 7) | ((b & 4u) << 14) | ((b & 8u) << 21);
            }
          } else {
            const int lim = (int)min<int64_t>(64, r.M - mt);
            for (int q = 0; q < lim; q++) vrow[q] = (uint8_t)((acc[j] >> q) & 1u);
          }
        }
      }
    }
    if (MODE == 3) {
      // 0/1 rows of the chunk's Bool columns that need one (a HIP C++ kernel reads rows, or the
      // column has no mask index): the wave writes them one column at a time, lane l storing model
      // mt + l of the column's lane mask (broadcast from its lane), so every store is a coalesced
      // 256-byte row segment instead of 64 serial stores by the column's own lane
      uint64_t pend = __ballot(run && (r.bool_rows || r.col_mask[live ? t : 0] < 0));
      while (pend) {
        const int q = __builtin_ctzll(pend);
        pend &= pend - 1;
        const int64_t rq = (int64_t)__shfl((int)row, q);
#pragma unroll
        for (int j = 0; j < FC_TILES; j++) {
          const int64_t mt = m0 + 64 * j;
          if (mt >= r.M) break;
          const uint64_t aq = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(acc[j] >> 32), q) << 32) |
                              (uint32_t)__shfl((int)(uint32_t)acc[j], q);
          if (mt + lane < r.M) r.vars_out[rq * r.M + mt + lane] = (uint32_t)((aq >> lane) & 1u);
        }
      }
    }
  }
  // counters: this wave's evaluated tapes x the workgroup's valid models (lane sums, then lane 0)
  if (r.counters) {
    unsigned long long nv = 0;
#pragma unroll
    for (int j = 0; j < FC_TILES; j++) nv += (unsigned long long)__popcll(valid[j]);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      runs += __shfl_xor(runs, d);
      run_nodes += __shfl_xor(run_nodes, d);
      run_ops += __shfl_xor(run_ops, d);
    }
    if (lane == 0 && runs) {
      unsigned long long* cnt = r.counters + ((blockIdx.x * 4 + wave) % kCounterSlots) * kCounterStride;
      if (MODE != 3) atomicAdd(&cnt[0], runs * nv);   // (tape evaluations; a column is not one)
      atomicAdd(&cnt[1], run_nodes * nv);
      atomicAdd(&cnt[2], run_ops * nv);
    }
  }
}

template <int MODE>
static void launch_fca_mode(const FcaArgs& a, int64_t groups, size_t lds, hipStream_t st) {
  if (a.xfs)
    hipLaunchKernelGGL((fca_kernel<MODE, true>), dim3((unsigned)groups), dim3(256), lds, st, a.groups, a.atoms, a.xfs,
                       a.lists, a.chunk_off, a.tape_out, a.tape_metric, a.vars, a.bool_masks, a.stage_masks, a);
  else
    hipLaunchKernelGGL((fca_kernel<MODE, false>), dim3((unsigned)groups), dim3(256), lds, st, a.groups, a.atoms, a.xfs,
                       a.lists, a.chunk_off, a.tape_out, a.tape_metric, a.vars, a.bool_masks, a.stage_masks, a);
}

hipError_t launch_fca(const FcaArgs& a, hipStream_t st) {
  if (a.n <= 0 || a.M <= 0) return hipSuccess;
  const int64_t groups = (a.M + 64 * FC_TILES - 1) / (64 * FC_TILES);
  if (groups > 0x7FFFFFFF) return hipErrorInvalidValue;
  const size_t lds = (size_t)(1 + a.n_smask + a.n_atoms) * 8u * FC_TILES;
  if (a.mode == 0)
    launch_fca_mode<0>(a, groups, lds, st);
  else if (a.mode == 1)
    launch_fca_mode<1>(a, groups, lds, st);
  else if (a.mode == 3)
    launch_fca_mode<3>(a, groups, lds, st);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_fc(const FcArgs& a, hipStream_t st) {
  if (a.n <= 0 || a.M <= 0) return hipSuccess;
  const int64_t groups = (a.M + 64 * FC_TILES - 1) / (64 * FC_TILES);
  const int64_t quads = ((a.n + a.tpg - 1) / a.tpg + 3) / 4;
  if (quads > 65535 || groups > 0x7FFFFFFF) return hipErrorInvalidValue;
  FcRun r{};
  r.n = a.n;
  r.tpg = a.tpg;
  r.n_bool_masks = a.n_bool_masks;
  r.mode = a.mode;
  r.early_exit = a.early_exit;
  r.bool_rows = a.bool_rows;
  r.M = a.M;
  r.index_base = a.index_base;
  r.best = a.best;
  r.verdicts = a.verdicts;
  r.masks_out = a.bool_masks_out;
  r.vars_out = a.vars_out;
  r.counters = a.counters;
  r.n_stage = a.n_stage;
  r.n_smask = a.n_smask;
  r.prefix = a.prefix;
  const size_t lds = ((size_t)a.n_stage * 256u + (size_t)a.n_smask * 8u) * FC_TILES;
  hipLaunchKernelGGL(fc_kernel, dim3((unsigned)groups, (unsigned)quads), dim3(256), lds, st, a.tapes, a.mask_lds, a.cmps,
                     a.vars, a.bool_masks, (const int32_t*)a.best, a.stage_rows, a.stage_masks, r);
  return hipGetLastError();
}

}  // namespace mq
