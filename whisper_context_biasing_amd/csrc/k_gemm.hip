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

// the lean decode projection's (waves, k-steps) table (gemm_impl.h launch_lean: the 16-bit rows of
// launch_dec_mf, so the lean and general kernels split K alike)
bool lean_cfg(int K, int& nw, int& kpw) {
  switch (K) {
    case 64: nw = 2; kpw = 1; return true;
    case 512: nw = 4; kpw = 4; return true;
    case 768: nw = 4; kpw = 6; return true;
    case 1024: nw = 4; kpw = 8; return true;
    case 1280: nw = 8; kpw = 5; return true;
    case 2048: nw = 8; kpw = 8; return true;
    case 3072: nw = 8; kpw = 12; return true;
    case 4096: nw = 16; kpw = 8; return true;
    case 5120: nw = 16; kpw = 10; return true;
    default: return false;
  }
}

int lm_head_partials(DType t, int K, int vocab) {
  return gemm_dec_supported(t, K) ? std::min((vocab + 15) / 16, kDecWalkers) : (vocab + 63) / 64;
}

void gemm(DType t, const GemmArgs& g, hipStream_t s) {
  switch (t) {
    case kBF16: gemm_bf16(g, s); break;
    case kF16: gemm_f16(g, s); break;
    case kF32: gemm_f32(g, s); break;
  }
}
}  // namespace wcb
