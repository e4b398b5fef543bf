// f16 instantiation of the GEMM kernels (split per dtype so the translation units build in parallel).
#include "gemm_impl.h"

namespace wcb {
void gemm_f16(const GemmArgs& g, hipStream_t s) { gemm_t<f16_t>(g, s); }
}  // namespace wcb
