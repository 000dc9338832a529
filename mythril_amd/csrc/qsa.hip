// qsa.hip — the gfx950 threaded-code tape interpreters (generated assembly, gen_qsa.py) wrapped
// in HIP kernels so they ship in libmq.so's fat binary and launch like any HIP kernel.
// P: one workgroup = 4 waves = 256 candidate models, grid.y = tape groups.
// G: one workgroup = 4 waves on the same 64 models, each wave its own tape group.  See gen_qsa.py for
// the register maps and the program encoding.
//   qsa_kernel (P): the first 8 model variables preloaded in VGPRs (C2-shaped batches)
//   qsg_kernel (G): no preloaded variables (a 4-slot stack, 80 VGPRs, 6 waves per SIMD): rows
//                   pushed from HBM or from the workgroup's LDS-staged rows, model-function
//                   lookups (EVM-shaped batches)
#include <hip/hip_runtime.h>

#include "qs_launch.h"
#include "qsa_gen.inc"

namespace mq {

__global__ __launch_bounds__(256) void qsa_kernel(const QArgs* __restrict__ args) {
  asm volatile(QSA_ASM_TEXT_P
               :
               : "s"(args), "s"(blockIdx.x), "s"(blockIdx.y), "v"(threadIdx.x)
               : QSA_CLOBBERS_P);
}

// G grid: blockIdx.x = xcd + 8 * g, blockIdx.y = t, gridDim.x a multiple of 8.  Workgroups are
// dispatched round-robin over the 8 XCDs in linear order, so workgroup (t, g) runs on XCD
// (linear id mod 8) = xcd next to the other groups g of the same 64-model tile 8t + xcd: the
// tile's model rows are read from HBM once per XCD and then served by that XCD's L2.
__global__ __launch_bounds__(256) void qsg_kernel(const QArgs* __restrict__ args) {
  const unsigned tile = blockIdx.y * 8u + (blockIdx.x & 7u);
  const unsigned grp = blockIdx.x >> 3;
  asm volatile(QSA_ASM_TEXT_G
               :
               : "s"(args), "s"(tile), "s"(grp), "v"(threadIdx.x)
               : QSA_CLOBBERS_G);
}

hipError_t launch_qsa(int variant, const QArgs* d_args, unsigned gx, unsigned gy, size_t lds, hipStream_t st) {
  if (lds > 65536) {   // temps + staged model rows beyond 64 KB (gfx950: 160 KB of LDS per CU)
    const void* f = variant == 0 ? reinterpret_cast<const void*>(qsa_kernel) : reinterpret_cast<const void*>(qsg_kernel);
    const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  if (variant == 0) hipLaunchKernelGGL(qsa_kernel, dim3(gx, gy), dim3(256), lds, st, d_args);
  else hipLaunchKernelGGL(qsg_kernel, dim3(gx, gy), dim3(256), lds, st, d_args);
  return hipGetLastError();
}

}  // namespace mq
