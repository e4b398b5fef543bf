// Task-ordered in-launch stage chain vs one launch per stage (decode-layer feasibility on MI355X).
//
// One launch = S stages x T tasks; workgroup b runs task b % T of stage b / T (stages dispatched in
// blockIdx order, so a waiting task only ever waits on tasks already dispatched: no co-residency
// requirement). Each task issues its W bytes of weights (nontemporal) FIRST, then (stage > 0) lane 0
// polls the previous stage's arrival counter (relaxed agent-scope loads, bounded spin), then the
// workgroup reads A bytes of the previous stage's output, writes its 1 KiB of this stage's output and
// arrives (every storing wave drains, workgroup barrier, one relaxed agent-scope add).
//   MODE 0: payload stored and loaded sc1 (write-through, no fences)
//   MODE 1: plain stores + release fence / acquire fence + plain loads
// Baseline: the same tasks as S dependent launches of T workgroups (hipGraph replay).
// Prints µs per stage. Build: hipcc -O3 --offload-arch=gfx950 tools/task_chain_bench.hip -o tools/task_chain_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <functional>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned gu32;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

template <int NT, int WPL, int APL, int MODE, bool CHAINED>
__global__ __launch_bounds__(NT) void k_task(const f4* __restrict__ w, long w_stage, f4* act, unsigned act_bytes, unsigned* ctr,
                                             int T, int stage0, int* err) {
  const int tid = threadIdx.x;
  const int s = CHAINED ? (int)blockIdx.x / T : stage0, t = CHAINED ? (int)blockIdx.x % T : (int)blockIdx.x;
  // weights of this task: issued before anything waits
  f4 wv[WPL > 0 ? WPL : 1];
  const f4* wp = w + (long)(s % 8) * w_stage + (long)t * (WPL * NT) + tid;
#pragma unroll
  for (int i = 0; i < WPL; ++i) wv[i] = __builtin_nontemporal_load(wp + i * NT);
  const f4* ain = act + (long)((s + 1) & 1) * (act_bytes / 32);
  f4* aout = act + (long)(s & 1) * (act_bytes / 32);
  if (CHAINED && s > 0) {
    if (tid == 0) {
      unsigned spins = 0;
      while (__hip_atomic_load((gu32*)(ctr + s - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)T) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 22)) { atomicExch(err, 1); break; }
      }
      if (MODE == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  }
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
  const __amdgpu_buffer_rsrc_t rin = rsrc_of(ain, act_bytes / 2);
#pragma unroll
  for (int i = 0; i < APL; ++i) {
    const unsigned off = (unsigned)(((tid + i * NT) * 16) % (act_bytes / 2));
    if (MODE == 0) acc += __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rin, off, 0, 16));
    else acc += ain[off / 16];
  }
#pragma unroll
  for (int i = 0; i < WPL; ++i) acc += wv[i];
  // this task's 1 KiB of the stage output
  if (tid < 64) {
    const unsigned off = (unsigned)((t * 64 + tid) * 16) % (act_bytes / 2);
    if (MODE == 0) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, acc), rsrc_of(aout, act_bytes / 2), off, 0, 16);
    else aout[off / 16] = acc;
  }
  if (CHAINED) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      if (MODE == 1) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __hip_atomic_fetch_add((gu32*)(ctr + s), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

double time_graph(int n, const std::function<void(int, hipStream_t)>& launch) {
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
  return ms * 1e3 / reps;
}

f4 *g_w, *g_act;
unsigned* g_ctr;
int* g_err;
const unsigned kActBytes = 2u << 20;

template <int NT, int WPL, int APL, int MODE>
void run(int S, int T) {
  const int layers = 12;
  const long w_stage = (long)T * WPL * NT;
  double chained = time_graph(layers, [&](int l, hipStream_t st) {
    CHK(hipMemsetAsync(g_ctr + l * 64, 0, 64 * 4, st));
    hipLaunchKernelGGL((k_task<NT, WPL, APL, MODE, true>), dim3(S * T), dim3(NT), 0, st, g_w + (l % 3) * 8 * w_stage, w_stage,
                       g_act, kActBytes, g_ctr + l * 64, T, 0, g_err);
  });
  double launches = time_graph(layers * S, [&](int i, hipStream_t st) {
    const int l = i / S, s = i % S;
    hipLaunchKernelGGL((k_task<NT, WPL, APL, MODE, false>), dim3(T), dim3(NT), 0, st, g_w + (l % 3) * 8 * w_stage, w_stage,
                       g_act, kActBytes, g_ctr, T, s, g_err);
  });
  int e = 0;
  CHK(hipMemcpy(&e, g_err, 4, hipMemcpyDeviceToHost));
  printf("mode %d NT=%4d T=%4d S=%2d W/task=%5.1f KB A/task=%5.1f KB: chained %6.2f us/stage (launch incl. memset), "
         "launches %6.2f us/stage%s\n", MODE, NT, T, S, WPL * NT * 16 / 1024.0, APL * NT * 16 / 1024.0,
         chained / (layers * S), launches / (layers * S), e ? "  [SPIN TIMEOUT]" : "");
  fflush(stdout);
  if (e) exit(2);
}

int main() {
  CHK(hipSetDevice(0));
  const size_t wbytes = (size_t)1 << 30;
  CHK(hipMalloc(&g_w, wbytes));
  CHK(hipMemset(g_w, 0, wbytes));
  CHK(hipMalloc(&g_act, kActBytes));
  CHK(hipMemset(g_act, 0, kActBytes));
  CHK(hipMalloc(&g_ctr, 64 * 64 * 4));
  CHK(hipMemset(g_ctr, 0, 64 * 64 * 4));
  CHK(hipMalloc(&g_err, 4));
  CHK(hipMemset(g_err, 0, 4));
  // decode-projection-like tasks: 24 KB of weights, 48 KB of activations per task
  run<256, 6, 12, 0>(5, 96);
  run<256, 6, 12, 1>(5, 96);
  run<256, 6, 12, 0>(5, 144);
  run<256, 6, 12, 0>(10, 96);
  run<256, 6, 3, 0>(5, 96);
  run<256, 6, 0, 0>(5, 96);
  run<256, 0, 0, 0>(5, 96);
  run<256, 0, 0, 0>(5, 256);
  run<512, 6, 6, 0>(5, 96);
  run<256, 24, 12, 0>(5, 48);
  return 0;
}
