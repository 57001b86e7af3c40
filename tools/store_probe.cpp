// Epilogue store-rate probe (one-off measurement tool, not product code).
//
// Question: the persistent NT GEMM's heavy epilogues (FFN1 forward: 256 KiB of bf16 stores per 256 x 256 tile) take
// ~20k + 10k cycles per tile. Is that bound per CU (each CU cannot push its stores faster) or chip-wide (all 256 CUs
// store at once, HBM write bandwidth)? If chip-wide, spreading the epilogues in time (other CUs in their MFMA main
// loop meanwhile) would hide them.
//
// Kernel: G workgroups of 512 threads (one per CU), each storing `tiles` x 256 KiB in the GEMM epilogue's pattern
// (one 16-B nt buffer store per lane, 8 rows x 128 B per wave instruction, row stride `ld` bytes) into its own
// region; optional busy phase (MFMA chain of `busy` instructions per wave) before every tile's stores, and an
// optional start offset (half of the workgroups begin with a busy phase of `stag` MFMAs) to desynchronise the CUs.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/store_probe tools/store_probe.cpp
//   tools/bin/store_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) short bf16x8;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* ptr) {
  const uint64_t a = (uint64_t)ptr;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, 0x7FFFFFFF, 0x00020000);
}

__device__ __forceinline__ f32x4 busy_mfma(int n, f32x4 acc) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (short)(threadIdx.x + i); b[i] = (short)(i * 3); }
  for (int i = 0; i < n; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  return acc;
}

// per tile: each wave stores 32 instructions x 1 KiB = 32 KiB (8 waves: 256 KiB), rows of 128 B (one 64-column wave
// tile slice), 8 rows per instruction, like epilogue_bf16 (WN = 64, CPR = 8)
__global__ __launch_bounds__(512, 1) void store_kernel(char* out, char* out2, int64_t ld, int tiles, int busy, int stag,
                                                       int nt, float* sink) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (stag > 0 && (blockIdx.x & 1)) acc = busy_mfma(stag, acc);
  const int wm = wave >> 2, wn = wave & 3;
  for (int t = 0; t < tiles; ++t) {
    if (busy > 0) acc = busy_mfma(busy, acc);
    // tile (blockIdx, t): 256 rows x 512 B (256 bf16 columns) at row stride ld
    char* tb = out + ((int64_t)(blockIdx.x * tiles + t) * 256) * ld;
    char* wb = tb + (int64_t)(wm * 128) * ld + wn * 128;
    const __amdgpu_buffer_rsrc_t r = rsrc(wb);
    const __amdgpu_buffer_rsrc_t r2 = rsrc(wb - out + out2);
    const u32x4 v = {(uint32_t)t, (uint32_t)lane, (uint32_t)acc[0], 7u};
#pragma unroll
    for (int it = 0; it < 16; ++it) {  // 128 rows / 8 per instruction
      const int row = it * 8 + (lane >> 3);
      const uint32_t off = (uint32_t)(row * ld + (lane & 7) * 16);
      // two outputs (GELU, GELU'): the same shape into a second buffer
      if (nt) {
        __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 2);
        __builtin_amdgcn_raw_buffer_store_b128(v, r2, off, 0, 2);
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(v, r2, off, 0, 0);
      }
    }
  }
  if (acc[0] == 123.f) sink[blockIdx.x] = acc[1];
}

int main(int argc, char** argv) {
  const int64_t ld = 6144;  // FFN1 output row: 3072 bf16
  const int max_grid = 256, tiles = 24;
  const size_t bytes = (size_t)max_grid * tiles * 256 * ld;
  char *out, *out2;
  float* sink;
  CK(hipMalloc(&out, bytes));
  CK(hipMalloc(&out2, bytes));
  CK(hipMalloc(&sink, 4096));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct Cfg { int grid, busy, stag, nt; };
  std::vector<Cfg> cfgs = {
      {256, 0, 0, 1}, {128, 0, 0, 1}, {64, 0, 0, 1}, {32, 0, 0, 1}, {8, 0, 0, 1}, {1, 0, 0, 1},
      {256, 0, 0, 0}, {32, 0, 0, 0},
      // MFMA "main loop" of ~33k cycles per wave pair: 2 waves/SIMD x N MFMAs of 16 cycles -> N = 1024 per wave
      {256, 1024, 0, 1}, {256, 1024, 512, 1}, {256, 2048, 0, 1}, {256, 2048, 1024, 1},
  };
  for (auto c : cfgs) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(store_kernel, dim3(c.grid), dim3(512), 0, 0, out, out2, ld, tiles, c.busy, c.stag, c.nt, sink);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    // 16 iterations x 2 stores x 1 KiB x 8 waves = 256 KiB per tile
    const double per_wg = (double)tiles * 256 * 1024;
    const double tot = per_wg * c.grid;
    printf("{\"grid\": %d, \"busy_mfma\": %d, \"stagger\": %d, \"nt\": %d, \"ms\": %.4f, \"us_per_tile\": %.2f, "
           "\"GBps_per_cu\": %.1f, \"TBps_chip\": %.3f}\n",
           c.grid, c.busy, c.stag, c.nt, best, best * 1e3 / tiles, per_wg / (best * 1e-3) / 1e9,
           tot / (best * 1e-3) / 1e12);
  }
  CK(hipFree(out));
  CK(hipFree(out2));
  return 0;
}
