// Issue cost of the integer ops a per-element dropout hash can use (v_mul_lo_u32, v_mul_u32_u24, v_mul_hi_u32_u24,
// xor / shift), 8 independent chains per lane, one wave per SIMD and 2 waves per SIMD.
//   hipcc -O3 --offload-arch=gfx950 tools/experiments/valu_cost.hip -o tools/bin/valu_cost
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int OP>
__global__ void k(uint32_t* out, uint32_t seed, int iters) {
  uint32_t x[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = seed + threadIdx.x * 8 + i;
  const uint32_t c = 0x7FEB352Du ^ seed;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (OP == 0) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[i]) : "v"(c));
        else if constexpr (OP == 1) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x[i]) : "v"(c));
        else if constexpr (OP == 2) asm volatile("v_lshrrev_b32 %0, 15, %0" : "+v"(x[i]));
        else if constexpr (OP == 3) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[i]) : "v"(c));
        else if constexpr (OP == 4) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(x[i]) : "v"(c));
      }
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s ^= x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  uint32_t* out;
  hipMalloc(&out, 1024 * 256 * 4 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 4096;
  const char* names[] = {"mul_lo_u32", "mul_u32_u24", "lshrrev_b32", "add_u32", "mul_hi_u32_u24"};
  for (int wps = 1; wps <= 2; ++wps) {
    for (int op = 0; op < 5; ++op) {
      auto launch = [&] {
        dim3 g(256 * wps), blk(256);
        if (op == 0) hipLaunchKernelGGL(k<0>, g, blk, 0, 0, out, 1u, iters);
        if (op == 1) hipLaunchKernelGGL(k<1>, g, blk, 0, 0, out, 1u, iters);
        if (op == 2) hipLaunchKernelGGL(k<2>, g, blk, 0, 0, out, 1u, iters);
        if (op == 3) hipLaunchKernelGGL(k<3>, g, blk, 0, 0, out, 1u, iters);
        if (op == 4) hipLaunchKernelGGL(k<4>, g, blk, 0, 0, out, 1u, iters);
      };
      launch();
      hipEventRecord(a);
      launch();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      // per SIMD: wps waves x iters x 64 ops; cycles at an assumed 2.1 GHz
      const double ops_per_simd = (double)wps * iters * 64;
      printf("{\"waves_per_simd\": %d, \"op\": \"%s\", \"ns_per_op_per_simd\": %.3f, \"cyc_at_2.1GHz\": %.2f}\n", wps,
             names[op], ms * 1e6 / ops_per_simd, ms * 1e6 / ops_per_simd * 2.1);
    }
  }
  return 0;
}
