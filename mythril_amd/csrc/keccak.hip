// keccak.hip — keccak256 (Ethereum padding 0x01..0x80, rate 136 B) on gfx950, one message
// per lane, the 25-lane keccak-f[1600] state in 50 VGPRs (64-bit lanes as u32 pairs are
// handled by the compiler's 64-bit shifts -> v_alignbit pairs).
// Replaces eth_hash's keccak in mythril/support/support_utils.py:92-100 and
// keccak_function_manager.py:56-69 (find_concrete_keccak) for batched concrete hashing.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qs_launch.h"

namespace mq {

__constant__ uint64_t kRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
    0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
    0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

__device__ __forceinline__ uint64_t rol(uint64_t v, int n) { return n ? (v << n) | (v >> (64 - n)) : v; }

// gfx950 v_bitop3_b32: any function of three 32-bit operands, the truth table as an 8-bit
// immediate indexed by (a << 2) | (b << 1) | c.  A three-way XOR (0x96) halves theta's column
// parities, and chi's a ^ (~b & c) (0xD2) is one instruction instead of two.
template <int LUT>
__device__ __forceinline__ uint32_t bitop3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:%4" : "=v"(r) : "v"(a), "v"(b), "v"(c), "i"(LUT));
  return r;
}
template <int LUT>
__device__ __forceinline__ uint64_t bitop3_64(uint64_t a, uint64_t b, uint64_t c) {
  return (uint64_t)bitop3<LUT>((uint32_t)a, (uint32_t)b, (uint32_t)c) |
         ((uint64_t)bitop3<LUT>((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32)) << 32);
}

__device__ __forceinline__ void keccak_f(uint64_t (&A)[25]) {
  constexpr int R[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
  for (int r = 0; r < 24; r++) {
    uint64_t C[5], Dd[5], B[25];
#pragma unroll
    for (int x = 0; x < 5; x++)
      C[x] = bitop3_64<0x96>(bitop3_64<0x96>(A[x], A[x + 5], A[x + 10]), A[x + 15], A[x + 20]);
#pragma unroll
    for (int x = 0; x < 5; x++) Dd[x] = C[(x + 4) % 5] ^ rol(C[(x + 1) % 5], 1);
#pragma unroll
    for (int i = 0; i < 25; i++) A[i] ^= Dd[i % 5];
#pragma unroll
    for (int x = 0; x < 5; x++)
#pragma unroll
      for (int y = 0; y < 5; y++) B[y + 5 * ((2 * x + 3 * y) % 5)] = rol(A[x + 5 * y], R[x + 5 * y]);
#pragma unroll
    for (int y = 0; y < 5; y++)
#pragma unroll
      for (int x = 0; x < 5; x++)
        A[x + 5 * y] = bitop3_64<0xD2>(B[x + 5 * y], B[(x + 1) % 5 + 5 * y], B[(x + 2) % 5 + 5 * y]);
    A[0] ^= kRC[r];
  }
}

__global__ __launch_bounds__(64) void keccak256_kernel(const uint8_t* __restrict__ data, const int64_t* __restrict__ off,
                                                       int n, uint8_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t beg = off[i], len = off[i + 1] - off[i];
  const uint8_t* msg = data + beg;
  // 8-byte message words straight from memory when the message is 8-byte aligned (fixed-length
  // batches of 32 / 64-byte words: 17 loads per block instead of 136 byte loads); bytes, with the
  // 0x01 pad byte, for the tail and for unaligned messages
  const bool al8 = ((uintptr_t)msg & 7u) == 0;
  uint64_t A[25];
#pragma unroll
  for (int k = 0; k < 25; k++) A[k] = 0;
  for (int64_t pos = 0;; pos += 136) {
#pragma unroll
    for (int w = 0; w < 17; w++) {
      const int64_t p0 = pos + 8 * w;
      uint64_t lane = 0;
      if (al8 && p0 + 8 <= len) {
        lane = *reinterpret_cast<const uint64_t*>(msg + p0);
      } else if (p0 <= len) {
        for (int b = 0; b < 8; b++) {
          const int64_t p = p0 + b;
          const uint64_t byte = p < len ? msg[p] : (p == len ? 0x01u : 0u);
          lane |= byte << (8 * b);
        }
      }
      A[w] ^= lane;
    }
    const bool last = pos + 136 > len;
    if (last) A[16] ^= 0x8000000000000000ull;
    keccak_f(A);
    if (last) break;
  }
  uint64_t* o = reinterpret_cast<uint64_t*>(out + (int64_t)i * 32);
#pragma unroll
  for (int w = 0; w < 4; w++) o[w] = A[w];
}

// Keccak columns: grid.y = column, grid.x = 256-model blocks; the column's message layout is
// uniform (scalar loads), the variable words are coalesced SoA rows.  The digest read big-endian
// is the 256-bit value (mq.h MQ_OP_KECCAK), stored into the column's 8 variable rows.
// h OP c over 8 little-endian limbs (unsigned)
__device__ __forceinline__ bool kc_pred(const KcPred& p, const uint32_t (&h)[8]) {
  if (p.kind == KP_LOWZ) {
    bool z = true;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint32_t b = p.bits > 32u * i ? min(32u, p.bits - 32u * i) : 0u;
      const uint32_t m = b >= 32 ? 0xFFFFFFFFu : ((1u << b) - 1u);
      z = z && (h[i] & m) == 0u;
    }
    return z;
  }
  // lexicographic compare from the top limb: lt = h < c, eq = h == c
  bool lt = false, eq = true;
#pragma unroll
  for (int i = 7; i >= 0; i--) {
    lt = lt || (eq && h[i] < p.c[i]);
    eq = eq && h[i] == p.c[i];
  }
  switch (p.kind) {
    case KP_LT: return lt;
    case KP_GT: return !lt && !eq;
    case KP_GE: return !lt;
    case KP_LE: return lt || eq;
    default: return eq;
  }
}

__global__ __launch_bounds__(256) void keccak_column_kernel(const KcCol* __restrict__ cols,
                                                            const KcMapEntry* __restrict__ map,
                                                            const KcPred* __restrict__ preds,
                                                            uint32_t* __restrict__ vars, int64_t M,
                                                            unsigned long long* __restrict__ counters,
                                                            uint64_t* __restrict__ bool_masks, int n_bool_masks,
                                                            int bool_rows) {
  const KcCol col = cols[blockIdx.y];
  const int64_t m0 = (int64_t)blockIdx.x * 256;
  const int64_t m = m0 + threadIdx.x;
  if (threadIdx.x == 0 && counters) {
    const unsigned long long nvalid = (unsigned long long)min<int64_t>(256, M - m0);
    unsigned long long* cnt = counters + ((blockIdx.x + blockIdx.y) % kCounterSlots) * kCounterStride;
    atomicAdd(&cnt[1], nvalid * col.n_nodes);
    atomicAdd(&cnt[2], nvalid * col.alg_ops);
  }
  if (m >= M) return;
  const KcMapEntry* e = map + col.map_off;
  const uint32_t nw = col.nwords;
  const uint32_t nblocks = (4u * nw) / 136u + 1u;
  uint64_t A[25];
#pragma unroll
  for (int k = 0; k < 25; k++) A[k] = 0;
#pragma unroll
  for (int b = 0; b < 2; b++) {
    if ((uint32_t)b >= nblocks) break;
#pragma unroll
    for (int p = 0; p < 34; p++) {
      const uint32_t gi = 34u * b + p;
      uint32_t w = 0;
      if (gi < nw) {
        const KcMapEntry x = e[gi];
        w = __builtin_bswap32(x.row == ~0u ? x.value : vars[(int64_t)x.row * M + m]);
      } else if (gi == nw) {
        w = 0x01u;   // pad byte at message position 4 nw
      }
      A[p >> 1] ^= (uint64_t)w << (32 * (p & 1));
    }
    if ((uint32_t)b == nblocks - 1u) A[16] ^= 0x8000000000000000ull;
    keccak_f(A);
  }
  uint32_t h[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t q = A[(7 - i) >> 1];
    h[i] = __builtin_bswap32((uint32_t)(((7 - i) & 1) ? (q >> 32) : q));
    vars[(int64_t)(col.target_row + i) * M + m] = h[i];
  }
  // the column's predicate columns from the digest in registers: the tile's lane mask (lane 0 of
  // the wave = one 64-model tile stores it; lanes past M are inactive, so their bits are 0) and
  // the 0/1 row when a HIP C++ kernel of the launch reads rows or the column has no mask index
  // (past the mask cap: readers then read the row, as G's column store does)
  for (uint32_t j = 0; j < col.n_pred; j++) {
    const KcPred p = preds[col.pred_off + j];
    const bool bit = kc_pred(p, h);
    if (bool_rows || p.mask < 0) vars[(int64_t)p.row * M + m] = bit ? 1u : 0u;
    if (p.mask >= 0) {
      const unsigned long long b = __ballot(bit);
      if ((threadIdx.x & 63) == 0) bool_masks[(m >> 6) * (int64_t)n_bool_masks + p.mask] = b;
    }
  }
}

hipError_t launch_keccak_columns(const KcCol* cols, int n_cols, const KcMapEntry* map, const KcPred* preds,
                                 uint32_t* vars, int64_t M, unsigned long long* counters, uint64_t* bool_masks,
                                 int n_bool_masks, int bool_rows, hipStream_t st) {
  if (n_cols <= 0 || M <= 0) return hipSuccess;
  hipLaunchKernelGGL(keccak_column_kernel, dim3((unsigned)((M + 255) / 256), (unsigned)n_cols), dim3(256), 0, st, cols,
                     map, preds, vars, M, counters, bool_masks, n_bool_masks, bool_rows);
  return hipGetLastError();
}

hipError_t launch_keccak(const uint8_t* data, const int64_t* offsets, int n, uint8_t* out, hipStream_t st) {
  hipLaunchKernelGGL(keccak256_kernel, dim3((n + 63) / 64), dim3(64), 0, st, data, offsets, n, out);
  return hipGetLastError();
}

}  // namespace mq
