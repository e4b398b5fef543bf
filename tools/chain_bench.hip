// Kernel-chain latency microbenchmark (decode-step floor on MI355X): a hipGraph of N dependent
// launches replayed; prints µs per launch for
//   empty        : trivial kernel
//   weights      : every workgroup streams W_KB of weights (fresh region per launch), writes 64 B
//   act          : every workgroup also reads the previous launch's output (ACT_KB, L2/MALL) first
//   act+weights  : both, weight loads issued before the activation loads
// Build: hipcc -O3 --offload-arch=gfx950 tools/chain_bench.hip -o tools/chain_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <chrono>
static double g_host_us = 0;

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <int NT>
__global__ __launch_bounds__(NT) void k_empty(float* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && out[0] == 12345.f) out[1] = 1.f;
}

// WPL: 16-B weight loads per lane (all issued up front); APL: 16-B activation loads per lane
template <int NT, int WPL, int APL, bool NTL = true>
__global__ __launch_bounds__(NT) void k_stream(const f4* __restrict__ w, long w_stride_wg, const f4* __restrict__ act_in,
                                               long act_elems, f4* __restrict__ act_out) {
  const int tid = threadIdx.x;
  const f4* wp = w + blockIdx.x * w_stride_wg + tid;
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
  f4 wv[WPL > 0 ? WPL : 1];
#pragma unroll
  for (int i = 0; i < WPL; ++i) wv[i] = NTL ? __builtin_nontemporal_load(wp + i * NT) : wp[i * NT];
  f4 av[APL > 0 ? APL : 1];
#pragma unroll
  for (int i = 0; i < APL; ++i) av[i] = act_in[(tid + i * NT) % act_elems];
#pragma unroll
  for (int i = 0; i < WPL; ++i) acc += wv[i];
#pragma unroll
  for (int i = 0; i < APL; ++i) acc += av[i];
  // wave shuffles, then one LDS slot per wave
  float v = acc[0] + acc[1] + acc[2] + acc[3];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __shared__ float red[NT / 64];
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  if (tid < 4) {
    float s = 0.f;
    for (int j = 0; j < NT / 64; ++j) s += red[j];
    act_out[(blockIdx.x * 4 + tid) % act_elems] = f4{s, s, s, s};
  }
}

template <typename F>
double time_chain(int n, F launch) {
  hipStream_t s;
  CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipGraph_t g;
  hipGraphExec_t ge;
  CHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < n; ++i) launch(i, s);
  CHK(hipStreamEndCapture(s, &g));
  CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int w = 0; w < 3; ++w) CHK(hipGraphLaunch(ge, s));
  CHK(hipStreamSynchronize(s));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  const int reps = 10;
  CHK(hipEventRecord(a, s));
  for (int r = 0; r < reps; ++r) CHK(hipGraphLaunch(ge, s));
  CHK(hipEventRecord(b, s));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  CHK(hipGraphExecDestroy(ge));
  CHK(hipGraphDestroy(g));
  CHK(hipStreamDestroy(s));
  return ms * 1e3 / (reps * n);
}

template <int NT, int WPL, int APL, bool NTL = true>
void run_case(const char* name, int grid, f4* wbuf, size_t wbytes, f4* act, long act_elems, size_t wrap = 0) {
  if (wrap) wbytes = wrap;
  const int n = 100;
  const long per_wg = (long)NT * (WPL > 0 ? WPL : 1);
  const long per_launch = per_wg * grid;
  const long nreg = (long)(wbytes / 16) / per_launch;   // distinct weight regions
  double us = time_chain(n, [&](int i, hipStream_t s) {
    const f4* w = wbuf + (i % nreg) * per_launch;
    f4* in = act + (i & 1) * act_elems;
    f4* out = act + ((i + 1) & 1) * act_elems;
    hipLaunchKernelGGL((k_stream<NT, WPL, APL, NTL>), dim3(grid), dim3(NT), 0, s, w, per_wg, in, act_elems, out);
  });
  printf("%-12s%-6s NT=%4d grid=%4d W/wg=%6.1f KB A/wg=%6.1f KB footprint=%5zu MB: %7.2f us/launch\n", name,
         NTL ? "nt" : "plain", NT, grid, WPL * NT * 16 / 1024.0, APL * NT * 16 / 1024.0, (size_t)(wbytes >> 20), us);
}

// NS streams each replaying its own graph of n launches of k_stream<256,4,4> concurrently
double time_multi(int NS, f4* wbuf, size_t wbytes, f4* act, long act_elems, bool empty, float* o) {
  const int n = 100, grid = 256;
  std::vector<hipStream_t> st(NS);
  std::vector<hipGraphExec_t> ge(NS);
  for (int k = 0; k < NS; ++k) {
    CHK(hipStreamCreateWithFlags(&st[k], hipStreamNonBlocking));
    hipGraph_t g;
    CHK(hipStreamBeginCapture(st[k], hipStreamCaptureModeThreadLocal));
    const long per_wg = 256 * 4, per_launch = per_wg * grid, nreg = (long)(wbytes / 16) / per_launch;
    for (int i = 0; i < n; ++i) {
      if (empty) {
        hipLaunchKernelGGL((k_empty<256>), dim3(grid), dim3(256), 0, st[k], o);
      } else {
        const f4* w = wbuf + ((i + 37 * k) % nreg) * per_launch;
        f4* in = act + (2 * k + (i & 1)) * act_elems;
        f4* out = act + (2 * k + ((i + 1) & 1)) * act_elems;
        hipLaunchKernelGGL((k_stream<256, 4, 4>), dim3(grid), dim3(256), 0, st[k], w, per_wg, in, act_elems, out);
      }
    }
    CHK(hipStreamEndCapture(st[k], &g));
    CHK(hipGraphInstantiate(&ge[k], g, nullptr, nullptr, 0));
    CHK(hipGraphDestroy(g));
  }
  for (int r = 0; r < 2; ++r)
    for (int k = 0; k < NS; ++k) CHK(hipGraphLaunch(ge[k], st[k]));
  CHK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  const int reps = 10;
  CHK(hipEventRecord(a, nullptr));
  for (int k = 0; k < NS; ++k) CHK(hipStreamWaitEvent(st[k], a, 0));
  auto h0 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; ++r)
    for (int k = 0; k < NS; ++k) CHK(hipGraphLaunch(ge[k], st[k]));
  auto h1 = std::chrono::steady_clock::now();
  g_host_us = std::chrono::duration<double, std::micro>(h1 - h0).count() / (reps * n * NS);
  for (int k = 0; k < NS; ++k) {
    hipEvent_t ev;
    CHK(hipEventCreate(&ev));
    CHK(hipEventRecord(ev, st[k]));
    CHK(hipStreamWaitEvent(nullptr, ev, 0));
  }
  CHK(hipEventRecord(b, nullptr));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  for (int k = 0; k < NS; ++k) { CHK(hipGraphExecDestroy(ge[k])); CHK(hipStreamDestroy(st[k])); }
  return ms * 1e3 / (reps * n);   // µs per launch-slot (each stream did reps*n launches)
}

// weights in N separate hipMalloc buffers of `bytes` each vs sub-ranges of one big allocation
void frag_case(bool separate, size_t bytes, int nbuf, f4* big, f4* act, long act_elems) {
  std::vector<f4*> bufs(nbuf);
  for (int i = 0; i < nbuf; ++i) {
    if (separate) { CHK(hipMalloc(&bufs[i], bytes)); CHK(hipMemset(bufs[i], 0, bytes)); }
    else bufs[i] = big + (size_t)i * (bytes / 16);
  }
  const int grid = (int)(bytes / (256 * 4 * 16));   // 16 KB per workgroup
  double us = time_chain(100, [&](int i, hipStream_t s) {
    f4* in = act + (i & 1) * act_elems;
    f4* out = act + ((i + 1) & 1) * act_elems;
    hipLaunchKernelGGL((k_stream<256, 4, 4>), dim3(grid), dim3(256), 0, s, bufs[i % nbuf], 256L * 4, in, act_elems, out);
  });
  printf("weights in %s (%d x %.2f MB, grid %d, 16 KB W + 16 KB A per WG): %7.2f us/launch\n",
         separate ? "separate hipMallocs" : "one allocation     ", nbuf, bytes / 1048576.0, grid, us);
  if (separate)
    for (int i = 0; i < nbuf; ++i) CHK(hipFree(bufs[i]));
}

int main() {
  CHK(hipSetDevice(0));
  size_t wbytes = (size_t)1 << 30;   // 1 GiB of "weights": beyond the 256 MiB MALL
  f4* wbuf;
  CHK(hipMalloc(&wbuf, wbytes));
  CHK(hipMemset(wbuf, 0, wbytes));
  const long act_elems = 98304 / 16;   // 96 KiB activations (32 rows x 768 f32)
  f4* act;
  CHK(hipMalloc(&act, 2 * act_elems * 16));
  CHK(hipMemset(act, 0, 2 * act_elems * 16));
  float* o;
  CHK(hipMalloc(&o, 64));
  CHK(hipMemset(o, 0, 64));
  for (int grid : {96, 256, 1024}) {
    double us = time_chain(100, [&](int, hipStream_t s) { hipLaunchKernelGGL((k_empty<256>), dim3(grid), dim3(256), 0, s, o); });
    printf("empty          NT= 256 grid=%4d: %7.2f us/launch\n", grid, us);
  }
  double us = time_chain(100, [&](int, hipStream_t s) { hipLaunchKernelGGL((k_empty<1024>), dim3(256), dim3(1024), 0, s, o); });
  printf("empty          NT=1024 grid= 256: %7.2f us/launch\n", us);
  // weights only (16 KB / WG at NT=256 with 4 loads per lane)
  run_case<256, 1, 0>("weights", 256, wbuf, wbytes, act, act_elems);
  run_case<256, 1, 0>("weights", 256, wbuf, wbytes, act, act_elems, (size_t)8 << 20);
  run_case<256, 4, 0>("weights", 256, wbuf, wbytes, act, act_elems, (size_t)16 << 20);
  run_case<256, 4, 0>("weights", 256, wbuf, wbytes, act, act_elems, (size_t)128 << 20);
  run_case<256, 4, 0, false>("weights", 256, wbuf, wbytes, act, act_elems);
  run_case<256, 4, 0, false>("weights", 256, wbuf, wbytes, act, act_elems, (size_t)128 << 20);
  run_case<256, 4, 0>("weights", 96, wbuf, wbytes, act, act_elems);
  run_case<256, 4, 0>("weights", 256, wbuf, wbytes, act, act_elems);
  run_case<256, 8, 0>("weights", 256, wbuf, wbytes, act, act_elems);
  run_case<512, 4, 0>("weights", 256, wbuf, wbytes, act, act_elems);
  run_case<256, 16, 0>("weights", 256, wbuf, wbytes, act, act_elems);
  // activations (previous launch's output) only / both
  run_case<256, 0, 4>("act", 256, wbuf, wbytes, act, act_elems);
  run_case<256, 0, 24>("act", 256, wbuf, wbytes, act, act_elems);
  run_case<256, 4, 4>("act+weights", 256, wbuf, wbytes, act, act_elems);
  run_case<256, 8, 24>("act+weights", 256, wbuf, wbytes, act, act_elems);
  run_case<512, 4, 12>("act+weights", 288, wbuf, wbytes, act, act_elems);
  run_case<1024, 4, 6>("act+weights", 96, wbuf, wbytes, act, act_elems);
  frag_case(true, (size_t)1179648, 400, wbuf, act, act_elems);
  frag_case(false, (size_t)1179648, 400, wbuf, act, act_elems);
  frag_case(true, (size_t)3538944, 200, wbuf, act, act_elems);
  frag_case(false, (size_t)3538944, 200, wbuf, act, act_elems);
  f4* act8;
  CHK(hipMalloc(&act8, 16 * act_elems * 16));
  CHK(hipMemset(act8, 0, 16 * act_elems * 16));
  for (int ns : {1, 2, 3, 4}) {
    double t = time_multi(ns, wbuf, wbytes, act8, act_elems, true, o);
    printf("concurrent chains: %d streams, empty        : %7.2f us per launch per stream (host submit %.2f us per launch)\n", ns, t, g_host_us);
    t = time_multi(ns, wbuf, wbytes, act8, act_elems, false, o);
    printf("concurrent chains: %d streams, act+weights16: %7.2f us per launch per stream (host submit %.2f us per launch)\n", ns, t, g_host_us);
  }
  return 0;
}
