// GEMM dispatch by element type; kernels and tiling live in gemm_impl.h.
#include "kernels.h"

namespace wcb {
void gemm_bf16(const GemmArgs& g, hipStream_t s);
void gemm_f16(const GemmArgs& g, hipStream_t s);
void gemm_f32(const GemmArgs& g, hipStream_t s);

void gemm(DType t, const GemmArgs& g, hipStream_t s) {
  switch (t) {
    case kBF16: gemm_bf16(g, s); break;
    case kF16: gemm_f16(g, s); break;
    case kF32: gemm_f32(g, s); break;
  }
}
}  // namespace wcb
