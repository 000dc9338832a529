// fc.hip — flat conjunctions on gfx950: tapes and Bool columns that are an AND of Bool model
// variables (negated or not) and comparisons of one model variable with a constant, evaluated
// without an interpreter.  After batch-level hoisting (lower.py lower_batch) this is the shape of
// most of a path's conjunction: the shared sub-terms are columns and what is left per path is the
// AND of their Bool columns plus a few word compares (C4's tapes: ~11 packed masks and 2-3
// compares).  On the G interpreter each (tape, 64-model tile) paid the tape frame (descriptor,
// early-exit test, program window) and ~6 threaded dispatches; here the masks are scalar loads
// AND-ed on the scalar unit and a compare is its variable's limb rows (coalesced, all in flight
// together) against constants held in SGPRs, one ballot each.
//
// One workgroup = one 64-model tile; its 4 waves take one tape group (FcRun.tpg tapes) each:
// grid.x = tiles, grid.y = quads of groups.  The variable rows the launch's compares read most are
// staged in LDS once per workgroup (FcCmp.row bit 31: an LDS slot), as the G interpreter stages
// them: every tape of the tile then reads them there instead of from L2 (C4: 200 tapes a tile).
// Modes: 0 first hit (best[] atomicMin, early exit on best[]), 1 verdict bytes, 3 Bool columns
// (packed lane mask stored, and the 0/1 row when a HIP C++ kernel reads rows or the column has no
// mask index).
//
// The read-only tables are separate __restrict__ kernel arguments so that their uniform reads
// are scalar loads (s_load) rather than vector loads and v_readfirstlane; within one launch no
// output is read back (a column level never reads its own columns).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qs_launch.h"

namespace mq {

__device__ __forceinline__ uint32_t uniform(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

struct alignas(64) U16 {
  uint32_t v[16];
};

// x OP c over the NL little-endian limbs of the compare's variable, in VALU: the borrow of x - c
// (lt) and the OR of x ^ c (ne) per lane; the op turns the two lane masks into the compare's (on
// the scalar unit).  Unsigned; a signed compare arrives with the sign bit of the top limb flipped
// on both sides (flip is XOR-ed into the variable, the constant is pre-flipped).  A staged
// variable's limbs are LDS reads at fixed offsets from its slot, all issued before the first use.
template <int NL>
__device__ __forceinline__ uint64_t fc_compare_nl(const FcCmp& q, const uint32_t* __restrict__ vars, int64_t M,
                                                  int64_t m, const uint32_t* lds, int lane) {
  const uint32_t row = q.row, flip = q.flip, op = q.op;
  uint32_t x[NL];
  if (row & 0x80000000u) {   // staged: slot (row & 0x7fffffff) + limb
    const uint32_t* sl = lds + (row & 0x7FFFFFFFu) * 64u + lane;
#pragma unroll
    for (int l = 0; l < NL; l++) x[l] = sl[l * 64];
  } else {
    const uint32_t* g = vars + (int64_t)row * M + m;
#pragma unroll
    for (int l = 0; l < NL; l++) x[l] = __builtin_nontemporal_load(g + (int64_t)l * M);
  }
  x[NL - 1] ^= flip;
  uint64_t borrow = 0;
  uint32_t ne = 0;
#pragma unroll
  for (int l = 0; l < NL; l++) {
    const uint32_t c = q.c[l];
    borrow = ((uint64_t)x[l] - (uint64_t)c - borrow) >> 63;
    ne |= x[l] ^ c;
  }
  const uint64_t lt = __ballot(borrow != 0), eq = __ballot(ne == 0);
  switch (op) {
    case FC_EQ: return eq;
    case FC_NE: return ~eq;
    case FC_LT: return lt;
    case FC_LE: return lt | eq;
    case FC_GT: return ~(lt | eq);
    default: return ~lt;   // FC_GE
  }
}

// (the whole 48-byte compare descriptor is loaded at once: one scalar round trip)
__device__ __forceinline__ uint64_t fc_compare(const FcCmp* __restrict__ qp, const uint32_t* __restrict__ vars,
                                               int64_t M, int64_t m, const uint32_t* lds, int lane) {
  const FcCmp q = *qp;
  switch (q.nl) {
    case 1: return fc_compare_nl<1>(q, vars, M, m, lds, lane);
    case 2: return fc_compare_nl<2>(q, vars, M, m, lds, lane);
    case 3: return fc_compare_nl<3>(q, vars, M, m, lds, lane);
    case 4: return fc_compare_nl<4>(q, vars, M, m, lds, lane);
    case 5: return fc_compare_nl<5>(q, vars, M, m, lds, lane);
    case 6: return fc_compare_nl<6>(q, vars, M, m, lds, lane);
    case 7: return fc_compare_nl<7>(q, vars, M, m, lds, lane);
    default: return fc_compare_nl<8>(q, vars, M, m, lds, lane);
  }
}

__global__ __launch_bounds__(256) void fc_kernel(const FcTape* __restrict__ tapes, const uint32_t* __restrict__ mask_idx,
                                                 const FcCmp* __restrict__ cmps, const uint32_t* __restrict__ vars,
                                                 const uint64_t* __restrict__ masks_in,
                                                 const int32_t* __restrict__ best_ro,
                                                 const uint32_t* __restrict__ stage_rows, FcRun r) {
  extern __shared__ uint32_t lds[];
  const uint32_t wave = uniform(threadIdx.x >> 6);
  const int64_t tile = blockIdx.x;
  const int64_t m0 = tile * 64;
  const int lane = threadIdx.x & 63;
  const int64_t m_raw = m0 + lane;
  const bool valid = m_raw < r.M;
  const int64_t m = valid ? m_raw : r.M - 1;   // (invalid lanes read a valid row; their bits are dropped)
  // stage the launch's most read rows: wave w loads rows w, w + 4, ..., eight loads in flight
  for (int s0 = (int)wave; s0 < r.n_stage; s0 += 32) {
    uint32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int s = min(s0 + 4 * k, r.n_stage - 1);
      v[k] = __builtin_nontemporal_load(vars + (int64_t)stage_rows[s] * r.M + m);
    }
#pragma unroll
    for (int k = 0; k < 8; k++)
      if (s0 + 4 * k < r.n_stage) lds[(s0 + 4 * k) * 64 + lane] = v[k];
  }
  if (r.n_stage) __syncthreads();
  const uint64_t valid_mask = __ballot(valid);
  const int32_t first = (int32_t)(r.index_base + m0);
  const uint64_t* __restrict__ tmask = masks_in + tile * (int64_t)r.n_bool_masks;
  const int t0 = ((int)blockIdx.y * 4 + (int)wave) * r.tpg;
  const int t1 = min(r.n, t0 + r.tpg);
  unsigned long long runs = 0, nodes = 0, ops = 0;
  if (t0 >= t1) return;
  FcTape d = tapes[t0];
  for (int t = t0; t < t1; t++) {
    // the next tape's descriptor is requested with this one's first loads (one round trip less)
    const FcTape dn = tapes[min(t + 1, t1 - 1)];
    // best[] only decreases within a launch: a stale (scalar-cache) value only skips less
    if (r.mode == 0 && r.early_exit && first >= best_ro[d.out]) {
      d = dn;
      continue;
    }
    uint64_t acc = valid_mask;
    // Bool variables: byte offsets into the tile's packed masks, the plain ones then the negated
    // ones (FcTape.n_mask = plain | negated << 16), each group padded to a multiple of 16 with its
    // last offset (AND-ing a mask twice changes nothing): sixteen offsets are one scalar load and
    // sixteen mask loads are in flight together
    const U16* mi = reinterpret_cast<const U16*>(mask_idx + d.mask_off);
    const char* tm = reinterpret_cast<const char*>(tmask);
    const uint32_t n_pos = ((d.n_mask & 0xFFFFu) + 15u) >> 4, n_neg = ((d.n_mask >> 16) + 15u) >> 4;
    for (uint32_t j = 0; j < n_pos; j++) {
      const U16 o = mi[j];
      uint64_t w = ~0ull;
#pragma unroll
      for (int k = 0; k < 16; k++) w &= *reinterpret_cast<const uint64_t*>(tm + o.v[k]);
      acc &= w;
    }
    for (uint32_t j = 0; j < n_neg; j++) {
      const U16 o = mi[n_pos + j];
      uint64_t w = 0;
#pragma unroll
      for (int k = 0; k < 16; k++) w |= *reinterpret_cast<const uint64_t*>(tm + o.v[k]);
      acc &= ~w;
    }
    for (uint32_t k = 0; k < d.n_cmp; k++) acc &= fc_compare(cmps + d.cmp_off + k, vars, r.M, m, lds, lane);
    runs++;
    nodes += d.n_nodes;
    ops += d.alg_ops;
    if (r.mode == 0) {
      if (acc && lane == 0) atomicMin(r.best + d.out, first + (int32_t)__builtin_ctzll(acc));
    } else if (r.mode == 1) {
      if (valid) r.verdicts[(int64_t)d.out * r.M + m_raw] = (uint8_t)((acc >> lane) & 1u);
    } else {
      if (d.mask_out >= 0 && lane == 0) r.masks_out[tile * (int64_t)r.n_bool_masks + d.mask_out] = acc;
      if ((r.bool_rows || d.mask_out < 0) && valid) r.vars_out[(int64_t)d.out * r.M + m_raw] = (uint32_t)((acc >> lane) & 1u);
    }
    d = dn;
  }
  if (lane == 0 && r.counters && runs) {
    const unsigned long long nv = (unsigned long long)__popcll(valid_mask);
    unsigned long long* cnt = r.counters + ((blockIdx.x * 4 + wave + blockIdx.y) % kCounterSlots) * kCounterStride;
    atomicAdd(&cnt[0], runs * nv);
    atomicAdd(&cnt[1], nodes * nv);
    atomicAdd(&cnt[2], ops * nv);
  }
}

hipError_t launch_fc(const FcArgs& a, hipStream_t st) {
  if (a.n <= 0 || a.M <= 0) return hipSuccess;
  const int64_t tiles = (a.M + 63) / 64;
  const int64_t quads = ((a.n + a.tpg - 1) / a.tpg + 3) / 4;
  if (quads > 65535 || tiles > 0x7FFFFFFF) return hipErrorInvalidValue;
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
  hipLaunchKernelGGL(fc_kernel, dim3((unsigned)tiles, (unsigned)quads), dim3(256), (size_t)a.n_stage * 256u, st,
                     a.tapes, a.mask_idx, a.cmps, a.vars, a.bool_masks, (const int32_t*)a.best,
                     a.stage_rows, r);
  return hipGetLastError();
}

}  // namespace mq
