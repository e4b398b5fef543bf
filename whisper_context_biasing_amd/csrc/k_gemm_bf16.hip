// bf16 instantiation of the GEMM kernels (split per dtype so the translation units build in parallel).
#include "gemm_impl.h"

namespace wcb {
void gemm_bf16(const GemmArgs& g, hipStream_t s) { gemm_t<bf16_t>(g, s); }
}  // namespace wcb
