// Persistent-kernel phase latency on MI355X (feasibility of a one-launch decode step): NB workgroups
// (<= one per CU, all co-resident) run P phases separated by a grid barrier; per phase every
// workgroup (optionally) prefetches W_KB of fresh weights BEFORE the barrier, then after it reads
// ACT_KB of the activations all workgroups wrote in the previous phase, and writes its own 64 B.
// Prints µs per phase. The barrier spin is bounded (error flag instead of a hang).
// Build: hipcc -O3 --offload-arch=gfx950 tools/barrier_bench.hip -o tools/barrier_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bool grid_barrier(unsigned* count, unsigned* gen, unsigned nblocks, int* err) {
  __syncthreads();
  bool ok = true;
  if (threadIdx.x == 0) {
    const unsigned g = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __threadfence();
    if (atomicAdd(count, 1u) == nblocks - 1) {
      __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      long spins = 0;
      while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
        if (++spins > (1L << 24)) { atomicExch(err, 1); ok = false; break; }
      }
    }
    __threadfence();
  }
  __syncthreads();
  return ok;
}

// Flag-array barrier run by wave 0 only: every workgroup publishes its phase number in its own
// slot (no contended atomic), wave 0 polls all slots (64 lanes x nb/64 words) until every slot has
// reached the phase. The other waves do not wait on memory (their weight prefetches stay in flight
// across the barrier): they meet wave 0 at a bare s_barrier.
__device__ __forceinline__ bool flag_barrier(unsigned* flags, unsigned phase, unsigned nblocks, int* err) {
  bool ok = true;
  if (threadIdx.x < 64) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    if (threadIdx.x == 0) __hip_atomic_store(flags + blockIdx.x, phase, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    long spins = 0;
    for (;;) {
      bool done = true;
      for (unsigned i = threadIdx.x; i < nblocks; i += 64)
        done &= __hip_atomic_load(flags + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= phase;
      if (__all(done)) break;
      if (++spins > (1L << 22)) { atomicExch(err, 1); ok = false; break; }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __builtin_amdgcn_s_barrier();
  return ok;
}

template <int NT, int WPL, int APL>
__global__ __launch_bounds__(NT) void k_flags(const f4* __restrict__ w, long w_per_phase, f4* act, long act_elems,
                                              int phases, unsigned* flags, int* err) {
  const int tid = threadIdx.x;
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
  for (int p = 0; p < phases; ++p) {
    f4 wv[WPL > 0 ? WPL : 1];
    if (tid >= 64) {   // compute waves: prefetch this phase's weights, then wait at the barrier
      const f4* wp = w + (p % 8) * w_per_phase + (long)blockIdx.x * (WPL * NT) + tid;
#pragma unroll
      for (int i = 0; i < WPL; ++i) wv[i] = __builtin_nontemporal_load(wp + i * NT);
    }
    if (!flag_barrier(flags, (unsigned)(p + 1) + flags[1023], gridDim.x, err)) return;
    const f4* ain = act + (long)(p & 1) * act_elems;
    f4* aout = act + (long)((p + 1) & 1) * act_elems;
    f4 av[APL > 0 ? APL : 1];
#pragma unroll
    for (int i = 0; i < APL; ++i) av[i] = ain[(tid + i * NT) % act_elems];
    if (tid >= 64) {
#pragma unroll
      for (int i = 0; i < WPL; ++i) acc += wv[i];
    }
#pragma unroll
    for (int i = 0; i < APL; ++i) acc += av[i];
    if (tid < 4) aout[(blockIdx.x * 4 + tid) % act_elems] = acc;
    __builtin_amdgcn_s_waitcnt(0);   // this phase's stores complete before the next arrive
  }
}

template <int NT, int WPL, int APL>
__global__ __launch_bounds__(NT) void k_phases(const f4* __restrict__ w, long w_per_phase, f4* act, long act_elems,
                                               int phases, unsigned* bar, int* err) {
  const int tid = threadIdx.x;
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
  for (int p = 0; p < phases; ++p) {
    f4 wv[WPL > 0 ? WPL : 1];
    const f4* wp = w + (p % 8) * w_per_phase + (long)blockIdx.x * (WPL * NT) + tid;
#pragma unroll
    for (int i = 0; i < WPL; ++i) wv[i] = __builtin_nontemporal_load(wp + i * NT);
    if (!grid_barrier(bar, bar + 32, gridDim.x, err)) return;
    const f4* ain = act + (long)(p & 1) * act_elems;
    f4* aout = act + (long)((p + 1) & 1) * act_elems;
    f4 av[APL > 0 ? APL : 1];
#pragma unroll
    for (int i = 0; i < APL; ++i) av[i] = ain[(tid + i * NT) % act_elems];
#pragma unroll
    for (int i = 0; i < WPL; ++i) acc += wv[i];
#pragma unroll
    for (int i = 0; i < APL; ++i) acc += av[i];
    if (tid < 4) aout[(blockIdx.x * 4 + tid) % act_elems] = acc;
  }
}

template <int NT, int WPL, int APL>
void run(const char* name, int nb, int phases, f4* w, long w_per_phase, f4* act, long act_elems, unsigned* bar, int* err) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL((k_phases<NT, WPL, APL>), dim3(nb), dim3(NT), 0, 0, w, w_per_phase, act, act_elems, 10, bar, err);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(a, 0));
  hipLaunchKernelGGL((k_phases<NT, WPL, APL>), dim3(nb), dim3(NT), 0, 0, w, w_per_phase, act, act_elems, phases, bar, err);
  CHK(hipEventRecord(b, 0));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  int e = 0;
  CHK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
  printf("%-34s nb=%3d nt=%4d W=%3d KB/wg act=%3d KB/wg: %7.2f us/phase%s\n", name, nb, NT,
         WPL * NT * 16 / 1024, APL * NT * 16 / 1024, ms * 1e3 / phases, e ? "  [BARRIER TIMEOUT]" : "");
  fflush(stdout);
  if (e) exit(2);
}

template <int NT, int WPL, int APL>
void run_flags(const char* name, int nb, int phases, f4* w, long w_per_phase, f4* act, long act_elems, unsigned* flags, int* err) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  CHK(hipMemset(flags, 0, 4096));
  hipLaunchKernelGGL((k_flags<NT, WPL, APL>), dim3(nb), dim3(NT), 0, 0, w, w_per_phase, act, act_elems, 10, flags, err);
  CHK(hipDeviceSynchronize());
  CHK(hipMemset(flags, 0, 4096));
  CHK(hipEventRecord(a, 0));
  hipLaunchKernelGGL((k_flags<NT, WPL, APL>), dim3(nb), dim3(NT), 0, 0, w, w_per_phase, act, act_elems, phases, flags, err);
  CHK(hipEventRecord(b, 0));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  int e = 0;
  CHK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
  printf("flags: %-27s nb=%3d nt=%4d W=%3d KB/wg act=%3d KB/wg: %7.2f us/phase%s\n", name, nb, NT,
         WPL * (NT - 64) * 16 / 1024, APL * NT * 16 / 1024, ms * 1e3 / phases, e ? "  [BARRIER TIMEOUT]" : "");
  fflush(stdout);
  if (e) exit(2);
}

int main() {
  const int phases = 2000;
  const long w_per_phase = 256L * 1024 * 96 / 16;   // 96 KB per wg x 256 wgs, f4 units
  f4 *w, *act;
  unsigned* bar;
  int* err;
  CHK(hipMalloc(&w, w_per_phase * 8 * sizeof(f4)));
  CHK(hipMemset(w, 0, w_per_phase * 8 * sizeof(f4)));
  const long act_elems = 64 * 1024 / 16;
  CHK(hipMalloc(&act, 2 * act_elems * sizeof(f4)));
  CHK(hipMemset(act, 0, 2 * act_elems * sizeof(f4)));
  CHK(hipMalloc(&bar, 256));
  CHK(hipMemset(bar, 0, 256));
  CHK(hipMalloc(&err, 4));
  CHK(hipMemset(err, 0, 4));
  unsigned* flags;
  CHK(hipMalloc(&flags, 4096));
  run_flags<256, 0, 0>("barrier only", 256, phases, w, w_per_phase, act, act_elems, flags, err);
  run_flags<512, 0, 0>("barrier only", 256, phases, w, w_per_phase, act, act_elems, flags, err);
  run_flags<512, 0, 6>("barrier + act 48KB", 256, phases, w, w_per_phase, act, act_elems, flags, err);
  run_flags<512, 3, 6>("barrier + act 48KB + W 21KB", 256, phases, w, w_per_phase, act, act_elems, flags, err);
  run_flags<512, 6, 6>("barrier + act 48KB + W 42KB", 256, phases, w, w_per_phase, act, act_elems, flags, err);
  run_flags<512, 12, 6>("barrier + act 48KB + W 84KB", 256, phases, w, w_per_phase, act, act_elems, flags, err);
  run_flags<1024, 6, 3>("barrier + act 48KB + W 90KB", 256, phases, w, w_per_phase, act, act_elems, flags, err);
  run<256, 0, 0>("barrier only", 256, phases, w, w_per_phase, act, act_elems, bar, err);
  run<256, 0, 0>("barrier only", 128, phases, w, w_per_phase, act, act_elems, bar, err);
  run<512, 0, 0>("barrier only", 256, phases, w, w_per_phase, act, act_elems, bar, err);
  run<256, 0, 12>("barrier + act 48KB", 256, phases, w, w_per_phase, act, act_elems, bar, err);
  run<512, 0, 6>("barrier + act 48KB", 256, phases, w, w_per_phase, act, act_elems, bar, err);
  run<512, 0, 12>("barrier + act 96KB", 256, phases, w, w_per_phase, act, act_elems, bar, err);
  run<256, 6, 12>("barrier + act 48KB + W 24KB", 256, phases, w, w_per_phase, act, act_elems, bar, err);
  run<512, 3, 6>("barrier + act 48KB + W 24KB", 256, phases, w, w_per_phase, act, act_elems, bar, err);
  run<512, 6, 6>("barrier + act 48KB + W 48KB", 256, phases, w, w_per_phase, act, act_elems, bar, err);
  run<512, 12, 6>("barrier + act 48KB + W 96KB", 256, phases, w, w_per_phase, act, act_elems, bar, err);
  return 0;
}
