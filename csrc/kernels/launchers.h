// Host-side launch functions of the gfx950 kernels (implemented in csrc/kernels/*.hip).
// Every launcher is stream-ordered and allocation-free, so callers may capture it into a hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hsd {
typedef uint16_t bf16_t;
struct DropoutParams;

// adam.hip
void launch_adam(float* p, float* m, float* v, const void* g, bool grad_bf16, bf16_t* out_bf16,
                 const uint8_t* decay, int64_t n, float step, float eps, float b1, float b2, float gscale,
                 float lr_wd, hipStream_t stream);

}  // namespace hsd
