// valu_peak.hip — VALU throughput microbenchmark on gfx950 (the roofline's peak), one harness for
// the integer instructions the interpreters issue AND the fp32 controls:
//   v_add_u32, v_add_co/v_addc (the 256-bit adders), v_mad_u64_u32 (the multiplier's partial
//   product), v_fma_f32 and v_pk_fma_f32 (2 fp32 lanes per instruction lane),
// each as lane-ops/s (instructions x 64 lanes; packed fp32 counted twice), next to the derived
// 256 CU x 4 SIMD x 32 lanes x f_clk (MI355X_MICROARCH.md: a wave64 VALU instruction issues over
// 2 cycles on a SIMD-32) and 256 CU x 4 SIMD x 16 lanes x f_clk (4 cycles per wave64).
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int KIND>
__global__ __launch_bounds__(256) void bench(unsigned* out, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 ^ 1, a2 = a0 ^ 2, a3 = a0 ^ 3, a4 = a0 ^ 4, a5 = a0 ^ 5, a6 = a0 ^ 6, a7 = a0 ^ 7;
  const unsigned k = blockIdx.x | 1;
  for (int i = 0; i < iters; i++) {
    if (KIND == 0) {
#pragma unroll
      for (int r = 0; r < 16; r++) {
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "s"(k));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a1) : "s"(k));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a2) : "s"(k));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a3) : "s"(k));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a4) : "s"(k));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a5) : "s"(k));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a6) : "s"(k));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a7) : "s"(k));
      }
    } else if (KIND == 1) {
#pragma unroll
      for (int r = 0; r < 16; r++) {
        asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %3, vcc" : "+v"(a0), "+v"(a1) : "v"(a2), "v"(a3) : "vcc");
        asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %3, vcc" : "+v"(a4), "+v"(a5) : "v"(a6), "v"(a7) : "vcc");
        asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %3, vcc" : "+v"(a2), "+v"(a3) : "v"(a0), "v"(a1) : "vcc");
        asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %3, vcc" : "+v"(a6), "+v"(a7) : "v"(a4), "v"(a5) : "vcc");
      }
    } else if (KIND == 3 || KIND == 4) {
      float f0 = (float)a0, f1 = (float)a1, f2 = (float)a2, f3 = (float)a3;
      float f4 = (float)a4, f5 = (float)a5, f6 = (float)a6, f7 = (float)a7;
      const float m = 0.999f;
#pragma unroll
      for (int r = 0; r < 16; r++) {
        if (KIND == 3) {
          asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f0) : "v"(m));
          asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f1) : "v"(m));
          asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f2) : "v"(m));
          asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f3) : "v"(m));
          asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f4) : "v"(m));
          asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f5) : "v"(m));
          asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f6) : "v"(m));
          asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f7) : "v"(m));
        } else {
          typedef float f2v __attribute__((ext_vector_type(2)));
          f2v p0 = {f0, f1}, p1 = {f2, f3}, p2 = {f4, f5}, p3 = {f6, f7}, pm = {m, m};
          asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p0) : "v"(pm));
          asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p1) : "v"(pm));
          asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p2) : "v"(pm));
          asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p3) : "v"(pm));
          asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p0) : "v"(pm));
          asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p1) : "v"(pm));
          asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p2) : "v"(pm));
          asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p3) : "v"(pm));
          f0 = p0.x; f1 = p0.y; f2 = p1.x; f3 = p1.y; f4 = p2.x; f5 = p2.y; f6 = p3.x; f7 = p3.y;
        }
      }
      a0 = __float_as_uint(f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7);
    } else {
      unsigned long long c0 = a0, c1 = a1, c2 = a2, c3 = a3;
#pragma unroll
      for (int r = 0; r < 16; r++) {
        asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(c0) : "v"(a4), "v"(a5) : "s0", "s1");
        asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(c1) : "v"(a5), "v"(a6) : "s0", "s1");
        asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(c2) : "v"(a6), "v"(a7) : "s0", "s1");
        asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(c3) : "v"(a7), "v"(a4) : "s0", "s1");
      }
      a0 = (unsigned)c0; a1 = (unsigned)c1; a2 = (unsigned)c2; a3 = (unsigned)c3;
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

int main() {
  int dev = 0;
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, dev));
  const int blocks = p.multiProcessorCount * 8;  // 8 x 256 threads per CU = 8 waves/SIMD
  unsigned* out;
  CHK(hipMalloc(&out, sizeof(unsigned) * blocks * 256));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const int iters = 4096;
  double rates[5];
  // lane-ops per thread per iteration (v_pk_fma_f32: 8 instructions x 2 fp32 lanes each)
  const double per_iter[5] = {16.0 * 8, 16.0 * 8, 16.0 * 4, 16.0 * 8, 16.0 * 8 * 2};
  for (int kind = 0; kind < 5; kind++) {
    for (int rep = 0; rep < 2; rep++) {
      CHK(hipEventRecord(e0));
      if (kind == 0) hipLaunchKernelGGL(bench<0>, dim3(blocks), dim3(256), 0, 0, out, iters);
      if (kind == 1) hipLaunchKernelGGL(bench<1>, dim3(blocks), dim3(256), 0, 0, out, iters);
      if (kind == 2) hipLaunchKernelGGL(bench<2>, dim3(blocks), dim3(256), 0, 0, out, iters);
      if (kind == 3) hipLaunchKernelGGL(bench<3>, dim3(blocks), dim3(256), 0, 0, out, iters);
      if (kind == 4) hipLaunchKernelGGL(bench<4>, dim3(blocks), dim3(256), 0, 0, out, iters);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      rates[kind] = (double)blocks * 256 * iters * per_iter[kind] / (ms * 1e-3);
    }
  }
  const double derived32 = (double)p.multiProcessorCount * 4 * 32 * 2.4e9;
  const double derived16 = (double)p.multiProcessorCount * 4 * 16 * 2.4e9;
  printf("{\"cus\": %d, \"clock_mhz\": %d, \"derived_simd32_ops\": %.4e, \"derived_simd16_ops\": %.4e, "
         "\"v_add_u32_ops\": %.4e, \"v_add_co_addc_ops\": %.4e, \"v_mad_u64_u32_ops\": %.4e, "
         "\"v_fma_f32_ops\": %.4e, \"v_pk_fma_f32_lane_ops\": %.4e}\n",
         p.multiProcessorCount, p.clockRate / 1000, derived32, derived16, rates[0], rates[1], rates[2], rates[3],
         rates[4]);
  return 0;
}
