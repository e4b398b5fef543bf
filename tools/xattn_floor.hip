// Floor of the greedy decode's encoder-space cross-attention stream (k_xenc.hip attn_xenc_reg_kernel):
// the same grid (rows x key ranges) streaming the same bytes (every row's encoder output [1500][d]
// bf16, one contiguous key range per workgroup) with no arithmetic, in a hipGraph of dependent
// launches; prints µs per launch and GB/s. Variants: threads per workgroup, 16-B loads in flight per
// lane, ranges per row, one buffer re-read by every launch (the 12 layers of a token read the same
// encoder output: Infinity-Cache resident) or two buffers alternated (two decode contexts).
// Build: hipcc -O3 --offload-arch=gfx950 tools/xattn_floor.hip -o tools/xattn_floor
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef float f4 __attribute__((ext_vector_type(4)));

// workgroup (split, row) streams bytes [row * row_bytes + split * per, +per) in rounds of NT x U x 16 B
template <int NT, int U>
__global__ __launch_bounds__(NT) void k_range(const f4* __restrict__ e, long row_f4, int nsplit, f4* __restrict__ out) {
  const int split = blockIdx.x, row = blockIdx.y, tid = threadIdx.x;
  const long per = (row_f4 + nsplit - 1) / nsplit;
  const long lo = (long)row * row_f4 + split * per;
  const long hi = min(lo + per, (long)(row + 1) * row_f4);
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
  for (long base = lo; base < hi; base += (long)NT * U) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = min(base + u * NT + tid, hi - 1);
      v[u] = __builtin_nontemporal_load(e + i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  if (acc[0] == 1234.5f) out[blockIdx.y * gridDim.x + blockIdx.x] = acc;
}

// The attention kernel's own access pattern (k_xenc.hip attn_xenc_reg_kernel load_chunk): 4 waves, wave w
// owns columns [192w, 192w + 192); per 32-key chunk each lane loads keys k0 + (lane & 15) (+16), 16 B at
// column 192w + 8·(lane >> 4) + 32·ks, ks < 6 — every wave-instruction touches 16 rows x 64 B; NR chunks
// in flight per wave (the register ring)
template <int NR>
__global__ __launch_bounds__(256) void k_pattern(const unsigned short* __restrict__ e, int S, int nsplit, f4* __restrict__ out) {
  const int split = blockIdx.x, row = blockIdx.y, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int per = ((S + nsplit - 1) / nsplit + 31) / 32 * 32;
  const int k_lo = split * per, k_hi = min(S, k_lo + per);
  const int nch = (k_hi - k_lo + 31) / 32;
  const unsigned short* E = e + (long)row * S * 768 + wave * 192 + 8 * (lane >> 4);
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
  for (int c0 = 0; c0 < nch; c0 += NR) {
    f4 v[NR][2][6];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int key = k_lo + (c0 + r) * 32 + (lane & 15);
      const unsigned short* r0 = E + (long)min(key, k_hi - 1) * 768;
      const unsigned short* r1 = E + (long)min(key + 16, k_hi - 1) * 768;
#pragma unroll
      for (int ks = 0; ks < 6; ++ks) {
        v[r][0][ks] = *reinterpret_cast<const f4*>(r0 + ks * 32);
        v[r][1][ks] = *reinterpret_cast<const f4*>(r1 + ks * 32);
      }
    }
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int ks = 0; ks < 6; ++ks) acc += v[r][0][ks] + v[r][1][ks];
  }
  if (acc[0] == 1234.5f) out[blockIdx.y * gridDim.x + blockIdx.x] = acc;
}

template <int NR>
double run_pattern(const f4* e0, int S, int rows, int nsplit, f4* out, int nlaunch) {
  hipStream_t s;
  CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipGraph_t g;
  hipGraphExec_t ge;
  CHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < nlaunch; ++i)
    hipLaunchKernelGGL((k_pattern<NR>), dim3(nsplit, rows), dim3(256), 0, s, (const unsigned short*)e0, S, nsplit, out);
  CHK(hipStreamEndCapture(s, &g));
  CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  CHK(hipGraphLaunch(ge, s));
  CHK(hipStreamSynchronize(s));
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHK(hipEventRecord(a, s));
    CHK(hipGraphLaunch(ge, s));
    CHK(hipEventRecord(b, s));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  CHK(hipGraphExecDestroy(ge));
  CHK(hipGraphDestroy(g));
  CHK(hipStreamDestroy(s));
  return best * 1e3 / nlaunch;
}

template <int NT, int U>
double run(const f4* e0, const f4* e1, long row_f4, int rows, int nsplit, f4* out, int nlaunch) {
  hipStream_t s;
  CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipGraph_t g;
  hipGraphExec_t ge;
  CHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < nlaunch; ++i)
    hipLaunchKernelGGL((k_range<NT, U>), dim3(nsplit, rows), dim3(NT), 0, s, (i & 1) ? e1 : e0, row_f4, nsplit, out);
  CHK(hipStreamEndCapture(s, &g));
  CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  CHK(hipGraphLaunch(ge, s));
  CHK(hipStreamSynchronize(s));
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHK(hipEventRecord(a, s));
    CHK(hipGraphLaunch(ge, s));
    CHK(hipEventRecord(b, s));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  CHK(hipGraphExecDestroy(ge));
  CHK(hipGraphDestroy(g));
  CHK(hipStreamDestroy(s));
  return best * 1e3 / nlaunch;
}

int main() {
  const int rows = 32, S = 1500, d = 768;
  const long row_f4 = (long)S * d * 2 / 16;
  const size_t bytes = (size_t)rows * row_f4 * 16;
  f4 *e0, *e1, *out;
  CHK(hipMalloc(&e0, bytes));
  CHK(hipMalloc(&e1, bytes));
  CHK(hipMalloc(&out, 1 << 20));
  CHK(hipMemset(e0, 0, bytes));
  CHK(hipMemset(e1, 0, bytes));
  const double mb = bytes / 1e6;
  auto rep = [&](const char* nm, int nsplit, bool two, double us) {
    printf("%-22s nsplit %2d %s: %7.2f us/launch  %7.1f GB/s\n", nm, nsplit, two ? "2 buffers" : "1 buffer ", us, mb * 1e3 / us);
  };
  for (int ns : {8, 16}) {
    rep("attn pattern, 1 chunk", ns, false, run_pattern<1>(e0, S, rows, ns, out, 48));
    rep("attn pattern, 2 chunks", ns, false, run_pattern<2>(e0, S, rows, ns, out, 48));
    rep("attn pattern, 3 chunks", ns, false, run_pattern<3>(e0, S, rows, ns, out, 48));
  }
  for (int two = 0; two < 2; ++two) {
    const f4* b1 = two ? e1 : e0;
    for (int ns : {8, 16}) {
      rep("256 thr, 4 in flight", ns, two, run<256, 4>(e0, b1, row_f4, rows, ns, out, 48));
      rep("256 thr, 8 in flight", ns, two, run<256, 8>(e0, b1, row_f4, rows, ns, out, 48));
      rep("256 thr, 16 in flight", ns, two, run<256, 16>(e0, b1, row_f4, rows, ns, out, 48));
      rep("512 thr, 8 in flight", ns, two, run<512, 8>(e0, b1, row_f4, rows, ns, out, 48));
    }
  }
  return 0;
}
