// ds_read_b64_tr_b8 lane mapping probe (gemm2.hip frag8t assumes: in each 16-lane group lane i addresses row i>>1,
// bytes 8(i&1)..+7 of a 16-byte-wide block, and receives column i's 8 rows). LDS holds byte (row*16 + col) for an
// 8 x 16 block per group; prints what each of the first 16 lanes receives. hipcc --offload-arch=gfx950 -O2.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(2))) int i32x2;
__global__ void probe(unsigned char* out) {
  __shared__ unsigned char lds[4 * 128];
  const int lane = threadIdx.x;
  for (int i = lane; i < 512; i += 64) lds[i] = (unsigned char)(i & 127);
  __syncthreads();
  const int g = lane >> 4, i = lane & 15;
  const unsigned char* a = lds + g * 128 + (i >> 1) * 16 + 8 * (i & 1);
  const i32x2 t = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) i32x2*)a);
  const unsigned char* b = reinterpret_cast<const unsigned char*>(&t);
  for (int j = 0; j < 8; ++j) out[lane * 8 + j] = b[j];
}
int main() {
  unsigned char* d;
  unsigned char h[512];
  if (hipMalloc(&d, 512) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, 512, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  int ok = 1;
  for (int l = 0; l < 64; ++l) {
    if (l < 16) printf("lane %2d:", l);
    for (int j = 0; j < 8; ++j) {
      if (l < 16) printf(" %3d", h[l * 8 + j]);
      ok &= h[l * 8 + j] == (unsigned char)(j * 16 + (l & 15));
    }
    if (l < 16) printf("\n");
  }
  printf("expected mapping (lane i <- column i, rows 0..7 in order): %s\n", ok ? "yes" : "NO");
  hipFree(d);
  return 0;
}
