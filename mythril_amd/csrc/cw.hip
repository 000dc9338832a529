// cw.hip — bit-gather columns on gfx950: hoisted columns whose value is a fixed arrangement of
// model-variable bits and constants, each run of bits optionally gated by `i <s size`.  These
// are the calldata words of the reference's symbolic calldata
// (mythril/laser/ethereum/state/calldata.py:48-55 get_word_at = Concat of 32 bytes, each
// calldata.py:234-247 _load = If(i < calldatasize, calldata[i], 0)), their extracts (the
// 4-byte selector) and constant masks (address arguments), as lower.py hoists them.
//
// The interpreters spend ~160 nodes (32 x SLT/ITE/CONCAT on 256-bit stacks) per word; here the
// host (mq_api.cpp cw_compile) folds the program into slots, and one lane per model ORs
// ((row >> sb) & mask) << db over the slots of each output limb: one 4-byte load per byte that
// reaches the output (an extract of the top 4 bytes reads 4 rows, not 32), no stack.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qs_launch.h"

namespace mq {

__global__ __launch_bounds__(256) void cw_column_kernel(const CwCol* __restrict__ cols,
                                                        const CwChunk* __restrict__ chunks,
                                                        uint32_t* __restrict__ vars, int64_t M,
                                                        unsigned long long* __restrict__ counters) {
  const CwCol col = cols[blockIdx.y];
  const int64_t m0 = (int64_t)blockIdx.x * 256;
  const int64_t m = m0 + threadIdx.x;
  if (threadIdx.x == 0 && counters) {
    const unsigned long long nvalid = (unsigned long long)min<int64_t>(256, M - m0);
    unsigned long long* cnt = counters + ((blockIdx.x + blockIdx.y) % kCounterSlots) * kCounterStride;
    atomicAdd(&cnt[1], nvalid * col.n_nodes);
    atomicAdd(&cnt[2], nvalid * col.alg_ops);
  }
  if (m >= M) return;
  // the gate bound: i <s size for 0 <= i < 2^31 is szv > i with szv = 0 for a negative size,
  // all-ones for a size >= 2^32, else its low limb
  uint32_t szv = 0;
  if (col.size_row != ~0u) {
    uint32_t s[8];
#pragma unroll
    for (int l = 0; l < 8; l++) s[l] = vars[(int64_t)(col.size_row + l) * M + m];
    const uint32_t hi = s[1] | s[2] | s[3] | s[4] | s[5] | s[6] | s[7];
    szv = (s[7] >> 31) ? 0u : (hi ? ~0u : s[0]);
  }
  uint32_t acc = 0;
  for (uint32_t c = col.chunk_off; c < col.chunk_off + col.n_chunks; c++) {
    const CwChunk ch = chunks[c];
    uint32_t x[4];
#pragma unroll
    for (int j = 0; j < 4; j++) x[j] = vars[(int64_t)ch.s[j].row * M + m];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const CwSlot& sl = ch.s[j];
      uint32_t v = ((x[j] >> (sl.shifts & 31u)) & sl.mask) << ((sl.shifts >> 8) & 31u);
      if (sl.gate != ~0u && !(szv > sl.gate)) v = 0;
      acc |= v;
    }
    acc |= ch.const_or;
    if (ch.store) {
      vars[(int64_t)(col.target_row + ch.limb) * M + m] = acc;
      acc = 0;
    }
  }
}

hipError_t launch_cw_columns(const CwCol* cols, int n_cols, const CwChunk* chunks, uint32_t* vars, int64_t M,
                             unsigned long long* counters, hipStream_t st) {
  if (n_cols <= 0 || M <= 0) return hipSuccess;
  hipLaunchKernelGGL(cw_column_kernel, dim3((unsigned)((M + 255) / 256), (unsigned)n_cols), dim3(256), 0, st, cols,
                     chunks, vars, M, counters);
  return hipGetLastError();
}

}  // namespace mq
