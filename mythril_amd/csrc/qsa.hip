// qsa.hip — the gfx950 threaded-code tape interpreter (generated assembly, gen_qsa.py) wrapped
// in a HIP kernel so it ships in libmq.so's fat binary and launches like any HIP kernel.
// One workgroup = 4 waves = 256 candidate models; grid.y = tape groups.  See gen_qsa.py for
// the register map and the program encoding.
#include <hip/hip_runtime.h>

#include "qs_launch.h"
#include "qsa_gen.inc"

namespace mq {

__global__ __launch_bounds__(256) void qsa_kernel(const QArgs* __restrict__ args) {
  asm volatile(QSA_ASM_TEXT
               :
               : "s"(args), "s"(blockIdx.x), "s"(blockIdx.y), "v"(threadIdx.x)
               : QSA_CLOBBERS);
}

hipError_t launch_qsa(const QArgs* d_args, unsigned gx, unsigned gy, size_t lds, hipStream_t st) {
  hipLaunchKernelGGL(qsa_kernel, dim3(gx, gy), dim3(256), lds, st, d_args);
  return hipGetLastError();
}

}  // namespace mq
