// fc.hip — flat conjunctions on gfx950: tapes and Bool columns that are an AND of Bool model
// variables (negated or not) and comparisons of one model variable with a constant, evaluated
// without an interpreter.  After batch-level hoisting (lower.py lower_batch) this is the shape of
// most of a path's conjunction: the shared sub-terms are columns and what is left per path is the
// AND of their Bool columns plus a few word compares (C4's tapes: ~11 packed masks and 2-3
// compares).  On the G interpreter each (tape, 64-model tile) paid the tape frame (descriptor,
// early-exit test, program window) and ~6 threaded dispatches; here the masks are scalar loads
// AND-ed on the scalar unit and a compare is its variable's limb rows (coalesced) against
// constants held in SGPRs, one ballot each.
//
// One wave = one 64-model tile; grid.x = tiles / 4 (4 waves per workgroup), grid.y = tape groups
// of FcArgs.tpg.  Modes: 0 first hit (best[] atomicMin, early exit on best[]), 1 verdict bytes,
// 3 Bool columns (packed lane mask stored, and the 0/1 row when a HIP C++ kernel reads rows or the
// column has no mask index).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qs_launch.h"

namespace mq {

__device__ __forceinline__ uint32_t uniform(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// x OP c over the nl little-endian limbs of the compare's variable (unsigned; a signed compare
// arrives with the sign bit of the top limb flipped on both sides: flip is XOR-ed into the
// variable, the constant is pre-flipped).  Unrolled over 8 limbs with uniform guards, so the
// constant's limbs are scalar loads at fixed offsets.
__device__ __forceinline__ bool fc_compare(const FcCmp* __restrict__ qp, const uint32_t* __restrict__ vars, int64_t M,
                                           int64_t m) {
  const uint32_t row = qp->row, nl = qp->nl, flip = qp->flip, op = qp->op;
  bool lt = false, eq = true;
#pragma unroll
  for (int l = 7; l >= 0; l--) {
    if ((uint32_t)l < nl) {
      uint32_t x = vars[(int64_t)(row + (uint32_t)l) * M + m];
      if ((uint32_t)l == nl - 1) x ^= flip;
      const uint32_t c = qp->c[l];
      lt = lt || (eq && x < c);
      eq = eq && x == c;
    }
  }
  switch (op) {
    case FC_EQ: return eq;
    case FC_NE: return !eq;
    case FC_LT: return lt;
    case FC_LE: return lt || eq;
    case FC_GT: return !lt && !eq;
    default: return !lt;   // FC_GE
  }
}

__global__ __launch_bounds__(256) void fc_kernel(FcArgs a) {
  const uint32_t wave = uniform(threadIdx.x >> 6);
  const int64_t tile = (int64_t)blockIdx.x * 4 + wave;
  const int64_t m0 = tile * 64;
  if (m0 >= a.M) return;
  const int lane = threadIdx.x & 63;
  const int64_t m_raw = m0 + lane;
  const bool valid = m_raw < a.M;
  const int64_t m = valid ? m_raw : a.M - 1;   // (invalid lanes read a valid row; their bits are dropped)
  const uint64_t valid_mask = __ballot(valid);
  const int32_t first = (int32_t)(a.index_base + m0);
  const uint64_t* __restrict__ tmask = a.bool_masks + tile * (int64_t)a.n_bool_masks;
  const int t0 = (int)blockIdx.y * a.tpg;
  const int t1 = min(a.n, t0 + a.tpg);
  unsigned long long runs = 0, nodes = 0, ops = 0;
  for (int t = t0; t < t1; t++) {
    const FcTape d = a.tapes[t];
    if (a.mode == 0 && a.early_exit) {
      // best[] only decreases within a launch: a stale (cached) value only skips less
      const int32_t b = a.best[d.out];
      if (first >= b) continue;
    }
    uint64_t acc = valid_mask;
    for (uint32_t j = 0; j < d.n_mask; j++) {
      const uint32_t e = a.mask_idx[d.mask_off + j];
      const uint64_t w = tmask[e & 0x7FFFFFFFu];
      acc &= (e >> 31) ? ~w : w;
    }
    for (uint32_t j = 0; j < d.n_cmp; j++) {
      acc &= __ballot(fc_compare(a.cmps + d.cmp_off + j, a.vars, a.M, m));
    }
    runs++;
    nodes += d.n_nodes;
    ops += d.alg_ops;
    if (a.mode == 0) {
      if (acc && lane == 0) atomicMin(a.best + d.out, first + (int32_t)__builtin_ctzll(acc));
    } else if (a.mode == 1) {
      if (valid) a.verdicts[(int64_t)d.out * a.M + m_raw] = (uint8_t)((acc >> lane) & 1u);
    } else {
      if (d.mask_out >= 0 && lane == 0) a.bool_masks_out[tile * (int64_t)a.n_bool_masks + d.mask_out] = acc;
      if ((a.bool_rows || d.mask_out < 0) && valid) a.vars_out[(int64_t)d.out * a.M + m_raw] = (uint32_t)((acc >> lane) & 1u);
    }
  }
  if (lane == 0 && a.counters && runs) {
    const unsigned long long nv = (unsigned long long)__popcll(valid_mask);
    unsigned long long* cnt = a.counters + ((blockIdx.x + blockIdx.y) % kCounterSlots) * kCounterStride;
    atomicAdd(&cnt[0], runs * nv);
    atomicAdd(&cnt[1], nodes * nv);
    atomicAdd(&cnt[2], ops * nv);
  }
}

hipError_t launch_fc(const FcArgs& a, hipStream_t st) {
  if (a.n <= 0 || a.M <= 0) return hipSuccess;
  const int64_t tiles = (a.M + 63) / 64;
  const int64_t groups = (a.n + a.tpg - 1) / a.tpg;
  if (groups > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fc_kernel, dim3((unsigned)((tiles + 3) / 4), (unsigned)groups), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace mq
