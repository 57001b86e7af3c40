// Standalone A/B probe: gemm2 (8 waves, 4 MFMA phases per K-tile) vs gemm4 (4 waves, one per SIMD) on the
// BERT-base B=1024 GEMM shapes and 8192^3, random [-1, 1) bf16 operands, interleaved rounds in ONE process
// (cdna_hip_programming.md §5.4 rule 24), every variant checked against an fp32 reference on sampled rows.
//
//   hipcc -O3 --offload-arch=gfx950 -Icsrc/kernels tools/gemm4_probe.cpp csrc/kernels/gemm2.hip \
//         csrc/kernels/gemm3.hip tools/experiments/gemm4.hip -o tools/bin/gemm4_probe
//   build/gemm4_probe [epi] [shape,...]  -> one JSON line per shape
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "gemm_common.h"

namespace hsd {
void launch_gemm2(int la, int lb, int epi, const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb, int M, int N,
                  int K, void* C, int64_t ldc, const bf16_t* bias, const bf16_t* aux, int64_t ldaux, bf16_t* C2,
                  double p_drop, uint64_t seed, int splits, float* ws, float* dbias, hipStream_t st);
void launch_gemm4(int epi, const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb, int M, int N, int K, bf16_t* C,
                  int64_t ldc, const bf16_t* bias, const bf16_t* aux, int64_t ldaux, bf16_t* C2, double p_drop,
                  uint64_t seed, hipStream_t st);

}  // namespace hsd

using hsd::bf16_t;

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

__global__ void fill_kernel(bf16_t* x, int64_t n, uint32_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t h = hsd::mix32((uint32_t)i * 2654435761u ^ seed ^ (uint32_t)(i >> 32));
    const float v = (float)(h >> 8) * (2.0f / 16777216.0f) - 1.0f;
    x[i] = hsd::f2bf(v);
  }
}

// C_ref[r][n] for sampled rows rows[r]: fp32 dot products
__global__ void ref_kernel(const bf16_t* A, const bf16_t* B, const int* rows, int nr, int N, int K, float* out) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int r = blockIdx.y;
  if (n >= N || r >= nr) return;
  const bf16_t* a = A + (int64_t)rows[r] * K;
  const bf16_t* b = B + (int64_t)n * K;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += hsd::bf2f(a[k]) * hsd::bf2f(b[k]);
  out[(int64_t)r * N + n] = s;
}

struct Shape {
  const char* name;
  int M, N, K;
};

int main(int argc, char** argv) {
  const int epi = argc > 1 ? atoi(argv[1]) : 0;
  std::string only = argc > 2 ? argv[2] : "";
  const int T = 131072;
  std::vector<Shape> shapes = {{"sq7680", 7680, 7680, 7680}, {"qkv_fwd", T, 2304, 768}, {"out_fwd", T, 768, 768},
                               {"ffn1_fwd", T, 3072, 768},    {"ffn2_fwd", T, 768, 3072}, {"qkv_dgrad", T, 768, 2304},
                               {"ffn2_dgrad", T, 3072, 768}};
  const char* variants[] = {"g2", "g4s0", "g4s1", "g4s3"};
  const int NV = 4;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  for (const Shape& s : shapes) {
    if (!only.empty() && only.find(s.name) == std::string::npos) continue;
    const int M = s.M, N = s.N, K = s.K;
    bf16_t *A, *B, *C, *bias, *aux, *C2;
    CK(hipMalloc(&A, (size_t)M * K * 2));
    CK(hipMalloc(&B, (size_t)N * K * 2));
    CK(hipMalloc(&C, (size_t)M * N * 2));
    CK(hipMalloc(&C2, (size_t)M * N * 2));
    CK(hipMalloc(&aux, (size_t)M * N * 2));
    CK(hipMalloc(&bias, (size_t)N * 2));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, st, A, (int64_t)M * K, 1u);
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, st, B, (int64_t)N * K, 2u);
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, st, aux, (int64_t)M * N, 3u);
    hipLaunchKernelGGL(fill_kernel, dim3(64), dim3(256), 0, st, bias, (int64_t)N, 4u);
    // sampled rows: first 64, last 64, 128 spread
    std::vector<int> rows;
    for (int i = 0; i < 64; ++i) rows.push_back(i);
    for (int i = 0; i < 64; ++i) rows.push_back(M - 64 + i);
    for (int i = 0; i < 128; ++i) rows.push_back((int)(((int64_t)i * 7919 * 257) % M));
    const int nr = (int)rows.size();
    int* drows;
    float* ref;
    CK(hipMalloc(&drows, nr * sizeof(int)));
    CK(hipMalloc(&ref, (size_t)nr * N * 4));
    CK(hipMemcpy(drows, rows.data(), nr * sizeof(int), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(ref_kernel, dim3((N + 255) / 256, nr), dim3(256), 0, st, A, B, drows, nr, N, K, ref);
    CK(hipStreamSynchronize(st));
    std::vector<float> href((size_t)nr * N);
    CK(hipMemcpy(href.data(), ref, href.size() * 4, hipMemcpyDeviceToHost));
    std::vector<bf16_t> hc((size_t)N);

    auto run = [&](int v) {
      if (v == 0) {
        hsd::launch_gemm2(0, 0, epi, A, K, B, K, M, N, K, C, N, bias, aux, N, C2, 0.0, 0, 1, nullptr, nullptr, st);
      } else {
        setenv("HSD_G4_SCHED", v == 1 ? "0" : v == 2 ? "1" : "3", 1);
        hsd::launch_gemm4(epi, A, K, B, K, M, N, K, C, N, bias, aux, N, C2, 0.0, 0, st);
      }
    };
    double err[NV];
    for (int v = 0; v < NV; ++v) {
      CK(hipMemsetAsync(C, 0, (size_t)M * N * 2, st));
      run(v);
      CK(hipStreamSynchronize(st));
      double mx = 0.0, mref = 0.0;
      if (epi == 0) {
        for (int r = 0; r < nr; ++r) {
          CK(hipMemcpy(hc.data(), C + (int64_t)rows[r] * N, N * 2, hipMemcpyDeviceToHost));
          for (int n = 0; n < N; ++n) {
            const uint32_t u = (uint32_t)hc[n] << 16;
            float f;
            memcpy(&f, &u, 4);
            mx = std::max(mx, (double)fabsf(f - href[(size_t)r * N + n]));
            mref = std::max(mref, (double)fabsf(href[(size_t)r * N + n]));
          }
        }
        err[v] = mx / (mref > 0 ? mref : 1.0);
      } else {
        err[v] = -1.0;
      }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<double> tf[NV];
    const double fl = 2.0 * M * N * K;
    for (int rnd = 0; rnd < 5; ++rnd) {
      for (int v = 0; v < NV; ++v) {
        run(v);
        CK(hipEventRecord(e0, st));
        const int it = 10;
        for (int i = 0; i < it; ++i) run(v);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        tf[v].push_back(fl / (ms / it * 1e-3) / 1e12);
      }
    }
    printf("{\"shape\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"epi\": %d", s.name, M, N, K, epi);
    for (int v = 0; v < NV; ++v) {
      std::sort(tf[v].begin(), tf[v].end());
      printf(", \"%s_TF\": %.1f, \"%s_err\": %.2e", variants[v], tf[v][tf[v].size() / 2], variants[v], err[v]);
    }
    printf("}\n");
    fflush(stdout);
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C)); CK(hipFree(C2)); CK(hipFree(aux)); CK(hipFree(bias));
    CK(hipFree(drows)); CK(hipFree(ref));
  }
  return 0;
}
