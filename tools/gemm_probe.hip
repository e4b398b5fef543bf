// Phase timing of the ping-pong encoder GEMM (gemm_impl.h gemm_pp_kernel, built here with
// WCB_GEMM_PROBE: wave 0 of every workgroup stamps s_memtime at kernel start (0), after the prologue
// LDS-DMA is issued (1), after the first wait (2), after K tile 0 (3), after K tile nk/2 (4), after the
// K loop (5), after its epilogue stores are issued (6) and after the second tile's K loop (7)). The four C2 encoder shapes (M = 48000), random
// bf16 operands, each a graph of 10 launches; prints the per-launch time, the per-workgroup phase
// offsets (cycles, median and p90) and how the workgroups spread over the launch (start rounds).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I whisper_context_biasing_amd/csrc tools/gemm_probe.hip -o tools/gemm_probe
#define WCB_GEMM_PROBE 1
#include "gemm_impl.h"

#include <algorithm>
#include <cstdio>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

using namespace wcb;
typedef unsigned short bf;

__global__ void fill_bf16(bf* p, long n, unsigned seed, float scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    const float v = ((h & 0xffffff) / 16777216.f * 2.f - 1.f) * scale;
    p[i] = (bf)(__float_as_uint(v) >> 16);
  }
}

int main(int argc, char** argv) {
  struct Shape { const char* name; int N, K, act; bool resid; };
  const bool medium = argc > 3 && atoi(argv[3]) == 1;   // C3's whisper-medium encoder (64 clips)
  const int M = medium ? 96000 : 48000;
  const Shape small_shapes[] = {{"qkv", 2304, 768, 0, false}, {"out", 768, 768, 0, true}, {"fc1", 3072, 768, 1, false},
                                {"fc2", 768, 3072, 0, true}};
  const Shape medium_shapes[] = {{"qkv", 3072, 1024, 0, false}, {"out", 1024, 1024, 0, true},
                                 {"fc1", 4096, 1024, 1, false}, {"fc2", 1024, 4096, 0, true}};
  const Shape* shapes = medium ? medium_shapes : small_shapes;
  const int raster = argc > 1 ? atoi(argv[1]) : 8;
  const int pp = argc > 2 ? atoi(argv[2]) : 2;   // 2: persistent grid, 3: one tile per workgroup
  bf *A, *W;
  float *bias, *out;
  CHK(hipMalloc(&A, (long)M * 4096 * 2));
  CHK(hipMalloc(&W, 4096L * 4096 * 2));
  CHK(hipMalloc(&bias, 4096 * 4));
  CHK(hipMalloc(&out, (long)M * 4096 * 4));
  CHK(hipMemset(bias, 0, 4096 * 4));
  CHK(hipMemset(out, 0, (long)M * 4096 * 4));
  fill_bf16<<<2048, 256>>>(A, (long)M * 4096, 1u, 1.f);
  fill_bf16<<<2048, 256>>>(W, 4096L * 4096, 2u, 0.03f);
  unsigned long long* probe;
  const int maxwg = 4096;
  CHK(hipMalloc(&probe, maxwg * 8 * 8));
  CHK(hipMemcpyToSymbol(HIP_SYMBOL(wcb_gemm_probe), &probe, sizeof(probe)));
  hipStream_t s;
  CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int si = 0; si < 4; ++si) {
    const Shape& sh = shapes[si];
    GemmArgs g;
    g.A = A; g.lda = sh.K; g.W = W; g.ldw = sh.K; g.M = M; g.N = sh.N; g.K = sh.K;
    g.bias = bias; g.act = sh.act; g.out = out; g.ldc = sh.N; g.out_f32 = sh.resid ? 1 : 0;
    g.resid = sh.resid ? out : nullptr; g.raster = raster; g.pp = pp;
    hipGraph_t gr;
    hipGraphExec_t ge;
    CHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < 10; ++i) gemm_t<bf16_t>(g, s);
    CHK(hipStreamEndCapture(s, &gr));
    CHK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
    CHK(hipGraphLaunch(ge, s));
    CHK(hipStreamSynchronize(s));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CHK(hipEventRecord(e0, s));
      CHK(hipGraphLaunch(ge, s));
      CHK(hipEventRecord(e1, s));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms);
    }
    const int nwg = pp == 3 ? ((M + 255) / 256) * (sh.N / 256) : 256;
    if (nwg * 8 > maxwg * 8) { printf("too many workgroups for the probe buffer\n"); continue; }
    std::vector<unsigned long long> h((size_t)nwg * 8);
    CHK(hipMemcpy(h.data(), probe, h.size() * 8, hipMemcpyDeviceToHost));
    const double us = best * 1e3 / 10;
    printf("%s N=%d K=%d raster %d pp %d: %.2f us per launch, %.1f TFLOP/s, %d workgroups\n", sh.name, sh.N, sh.K, raster, pp, us,
           2.0 * M * sh.N * sh.K / us / 1e6, nwg);
    unsigned long long t0 = ~0ull, t1 = 0;
    for (int k = 1; k <= 7; ++k) {
      std::vector<long> d;
      for (int w = 0; w < nwg; ++w) d.push_back((long)(h[w * 8 + k] - h[w * 8 + k - 1]));
      std::sort(d.begin(), d.end());
      printf("  phase %d-%d: median %7ld p10 %7ld p90 %7ld cycles\n", k - 1, k, d[d.size() / 2], d[d.size() / 10],
             d[d.size() * 9 / 10]);
    }
    std::vector<long> life;
    for (int w = 0; w < nwg; ++w) life.push_back((long)(h[w * 8 + 7] - h[w * 8 + 6]));
    std::sort(life.begin(), life.end());
    printf("  second tile (first epilogue issued -> its K loop done): median %ld p90 %ld cycles\n", life[life.size() / 2],
           life[life.size() * 9 / 10]);
    CHK(hipGraphExecDestroy(ge));
    CHK(hipGraphDestroy(gr));
  }
  return 0;
}
