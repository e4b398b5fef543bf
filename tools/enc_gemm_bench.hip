// Encoder GEMM variants of the LDS-ring kernel (gemm_impl.h gemm_ring_kernel) at the C2 encoder shapes
// (whisper-small, 32 clips: M = 48000) with the encoder's own epilogues, random bf16 operands, each
// variant replayed as a hipGraph of 10 launches, variants interleaved over rounds in one process
// (median µs per launch); every variant's output is compared bit for bit with variant 0's.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I whisper_context_biasing_amd/csrc tools/enc_gemm_bench.hip -o tools/enc_gemm_bench
#include "gemm_impl.h"

#include <algorithm>
#include <cstring>
#include <functional>
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
__global__ void fill_f32(float* p, long n, unsigned seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2246822519u ^ seed;
    h ^= h >> 15; h *= 2654435761u; h ^= h >> 13;
    p[i] = (h & 0xffffff) / 16777216.f * 2.f - 1.f;
  }
}

typedef void (*Launch)(const GemmArgs&, hipStream_t);
struct Variant { const char* name; Launch fn; };

double time_graph(const std::function<void(hipStream_t)>& launch, hipStream_t s, int reps) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < reps; ++i) launch(s);
  CHK(hipStreamEndCapture(s, &g));
  CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CHK(hipGraphLaunch(ge, s));
  CHK(hipStreamSynchronize(s));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  CHK(hipEventRecord(a, s));
  CHK(hipGraphLaunch(ge, s));
  CHK(hipEventRecord(b, s));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  CHK(hipEventDestroy(a));
  CHK(hipEventDestroy(b));
  CHK(hipGraphExecDestroy(ge));
  CHK(hipGraphDestroy(g));
  return ms * 1e3 / reps;
}

int main(int argc, char** argv) {
  const int M = 48000;
  struct Shape { const char* name; int N, K, act; bool resid; };
  std::vector<Shape> shapes = {{"qkv", 2304, 768, 0, false}, {"out", 768, 768, 0, true},
                               {"fc1", 3072, 768, 1, false}, {"fc2", 768, 3072, 0, true}};
  if (argc > 2) {   // "N:K:act:resid,..." custom shapes (M = 48000)
    shapes.clear();
    for (char* tok = strtok(argv[2], ","); tok; tok = strtok(nullptr, ",")) {
      int n, k, a, r;
      if (sscanf(tok, "%d:%d:%d:%d", &n, &k, &a, &r) == 4) shapes.push_back({"shape", n, k, a, r != 0});
    }
  }
  const Variant vars[] = {
      {"256x256", launch_ring<bf, 256, 256, 2, 4, 2>},
      {"256x256 raster 4", [](const GemmArgs& g, hipStream_t s) { GemmArgs h = g; h.raster = 4; launch_ring<bf, 256, 256, 2, 4, 2>(h, s); }},
      {"256x256 raster 8", [](const GemmArgs& g, hipStream_t s) { GemmArgs h = g; h.raster = 8; launch_ring<bf, 256, 256, 2, 4, 2>(h, s); }},
      {"256x192", launch_ring<bf, 256, 192, 2, 4, 2>},
      {"256x192 raster 8", [](const GemmArgs& g, hipStream_t s) { GemmArgs h = g; h.raster = 8; launch_ring<bf, 256, 192, 2, 4, 2>(h, s); }},
  };
  const int nv = sizeof(vars) / sizeof(vars[0]);
  const int rounds = argc > 1 ? atoi(argv[1]) : 5;
  hipStream_t s;
  CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (const Shape& sh : shapes) {
    const int N = sh.N, K = sh.K;
    bf *A, *W;
    float *bias, *R = nullptr;
    void* out;
    const size_t osz = (size_t)M * N * (sh.resid ? 4 : 2);
    CHK(hipMalloc(&A, (size_t)M * K * 2));
    CHK(hipMalloc(&W, (size_t)N * K * 2));
    CHK(hipMalloc(&bias, (size_t)N * 4));
    CHK(hipMalloc(&out, osz));
    fill_bf16<<<2048, 256, 0, s>>>(A, (long)M * K, 1u, 1.f);
    fill_bf16<<<2048, 256, 0, s>>>(W, (long)N * K, 2u, 1.f / sqrtf((float)K));
    fill_f32<<<64, 256, 0, s>>>(bias, N, 3u);
    if (sh.resid) {
      CHK(hipMalloc(&R, (size_t)M * N * 4));
      fill_f32<<<2048, 256, 0, s>>>(R, (long)M * N, 4u);
    }
    GemmArgs g;
    g.A = A; g.lda = K; g.W = W; g.ldw = K; g.M = M; g.N = N; g.K = K;
    g.bias = bias; g.act = sh.act; g.resid = R; g.out = out; g.out_f32 = sh.resid ? 1 : 0; g.ldc = N;
    std::vector<char> ref(osz), got(osz);
    std::vector<std::vector<double>> t(nv);
    for (int v = 0; v < nv; ++v) {   // correctness: bit-identical to variant 0
      CHK(hipMemsetAsync(out, 0, osz, s));
      vars[v].fn(g, s);
      CHK(hipStreamSynchronize(s));
      CHK(hipMemcpy(v == 0 ? ref.data() : got.data(), out, osz, hipMemcpyDeviceToHost));
      if (v > 0 && memcmp(ref.data(), got.data(), osz) != 0) printf("  %s %s: OUTPUT DIFFERS\n", sh.name, vars[v].name);
    }
    for (int r = 0; r < rounds; ++r)
      for (int v = 0; v < nv; ++v) t[v].push_back(time_graph([&](hipStream_t st) { vars[v].fn(g, st); }, s, 10));
    const double fl = 2.0 * M * N * K;
    for (int v = 0; v < nv; ++v) {
      std::sort(t[v].begin(), t[v].end());
      const double med = t[v][t[v].size() / 2];
      printf("%s M=%d N=%d K=%d %-18s median %8.1f us  min %8.1f  %7.1f TFLOP/s\n", sh.name, M, N, K, vars[v].name, med,
             t[v][0], fl / med / 1e6);
    }
    fflush(stdout);
    CHK(hipFree(A)); CHK(hipFree(W)); CHK(hipFree(bias)); CHK(hipFree(out));
    if (R) CHK(hipFree(R));
  }
  return 0;
}
