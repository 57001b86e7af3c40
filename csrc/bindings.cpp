// Python bindings for the gfx950 kernels: argument validation + current-HIP-stream launch.
// Compiled into huggingface_sagemaker_tensorflow_distributed_amd/_C.so by _build.py (hipcc).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "kernels/launchers.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_CUDA(x) TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor")
#define CHECK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")
#define CHECK_DTYPE(x, d) TORCH_CHECK((x).scalar_type() == (d), #x " has wrong dtype")
#define BF(x) reinterpret_cast<hsd::bf16_t*>((x).data_ptr())
#define CBF(x) reinterpret_cast<const hsd::bf16_t*>((x).data_ptr())

void adam_step(torch::Tensor p, torch::Tensor m, torch::Tensor v, torch::Tensor g, c10::optional<torch::Tensor> out,
               c10::optional<torch::Tensor> decay, double step, double eps, double b1, double b2, double gscale,
               double lr_wd) {
  CHECK_CUDA(p); CHECK_CONTIG(p); CHECK_DTYPE(p, torch::kFloat32);
  CHECK_DTYPE(m, torch::kFloat32); CHECK_DTYPE(v, torch::kFloat32);
  TORCH_CHECK(p.numel() == m.numel() && p.numel() == v.numel() && p.numel() == g.numel(), "size mismatch");
  TORCH_CHECK(p.numel() % 1024 == 0, "flat buffer must be a multiple of 1024 elements");
  bool gbf = g.scalar_type() == torch::kBFloat16;
  TORCH_CHECK(gbf || g.scalar_type() == torch::kFloat32, "grad must be fp32 or bf16");
  hsd::bf16_t* o = nullptr;
  if (out.has_value()) {
    CHECK_DTYPE(*out, torch::kBFloat16);
    TORCH_CHECK(out->numel() == p.numel(), "out size");
    o = BF(*out);
  }
  const uint8_t* dm = nullptr;
  if (decay.has_value()) {
    TORCH_CHECK(decay->numel() * 64 >= p.numel(), "decay mask too small");
    dm = decay->data_ptr<uint8_t>();
  }
  hsd::launch_adam(p.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), g.data_ptr(), gbf, o, dm,
                   p.numel(), (float)step, (float)eps, (float)b1, (float)b2, (float)gscale, (float)lr_wd,
                   cur_stream());
}

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "gfx950 HIP kernels for huggingface_sagemaker_tensorflow_distributed_amd";
  m.def("adam_step", &adam_step);
}
