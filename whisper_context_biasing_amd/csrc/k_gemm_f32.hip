// f32 instantiation of the GEMM kernels (split per dtype so the translation units build in parallel).
#include "gemm_impl.h"

namespace wcb {
void gemm_f32(const GemmArgs& g, hipStream_t s) { gemm_t<float>(g, s); }
}  // namespace wcb
