// GEMM dispatch by element type; kernels and tiling live in gemm_impl.h.
#include <algorithm>

#include "kernels.h"

namespace wcb {
void gemm_bf16(const GemmArgs& g, hipStream_t s);
void gemm_f16(const GemmArgs& g, hipStream_t s);
void gemm_f32(const GemmArgs& g, hipStream_t s);

bool gemm_dec_supported(DType t, int K) {
  (void)t;
  return K == 64 || K == 128 || K == 256 || K == 384 || K == 512 || K == 768 || K == 1024 || K == 1280;
}

int lm_head_partials(DType t, int K, int vocab, int walkers) {
  return gemm_dec_supported(t, K) ? std::min((vocab + 15) / 16, walkers) : (vocab + 63) / 64;
}

void gemm(DType t, const GemmArgs& g, hipStream_t s) {
  switch (t) {
    case kBF16: gemm_bf16(g, s); break;
    case kF16: gemm_f16(g, s); break;
    case kF32: gemm_f32(g, s); break;
  }
}
}  // namespace wcb
