// CU-mask probe (measurement tool, not product): which XCD / shader engine / CU a stream's CU-mask bit
// selects on this GPU. A stream created with hipExtStreamCreateWithCUMask(mask) runs a kernel of many
// small workgroups; every workgroup records HW_REG_XCC_ID and HW_REG_HW_ID (se_id [15:13], sh_id [12],
// cu_id [11:8]); the host tallies the distinct CUs per XCD and per (XCD, SE).
// Masks probed: all bits; bits [8k, 8k + 8) for k = 0..31 (one bit per XCD if the driver stripes mask bits
// over the XCDs, so every XCD keeps a CU); and the decode / encoder split masks the runtime builds.
// A launch that has not finished within 2 s ends the process (the queue is torn down with it).
// Build: hipcc --offload-arch=gfx950 -O2 tools/cumask_probe.hip -o tools/cumask_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <set>
#include <thread>
#include <unistd.h>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void where_kernel(unsigned* out) {
  if (threadIdx.x == 0) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    // spin ~2 us so the workgroups spread over the CUs the mask allows
    const long long t0 = clock64();
    while (clock64() - t0 < 4000) {}
    out[blockIdx.x] = ((xcc & 0xf) << 16) | ((hw >> 8) & 0xff);   // xcc | se(3) sh(1) cu(4)
  }
}

static const int kWG = 8192;

static std::map<unsigned, int> run(const std::vector<uint32_t>& mask, unsigned* d_out) {
  hipStream_t s;
  if (mask.empty()) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  else CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
  CK(hipMemsetAsync(d_out, 0xff, kWG * 4, s));
  hipLaunchKernelGGL(where_kernel, dim3(kWG), dim3(64), 0, s, d_out);
  CK(hipGetLastError());
  const auto t0 = std::chrono::steady_clock::now();
  while (hipStreamQuery(s) == hipErrorNotReady) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
      fprintf(stderr, "launch did not finish within 2 s: exiting\n");
      fflush(stdout);
      _exit(3);
    }
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  std::vector<unsigned> h(kWG);
  CK(hipMemcpy(h.data(), d_out, kWG * 4, hipMemcpyDeviceToHost));
  CK(hipStreamDestroy(s));
  std::map<unsigned, int> cnt;
  for (unsigned v : h) cnt[v]++;
  return cnt;
}

static void report(const char* name, const std::map<unsigned, int>& cnt) {
  std::map<int, std::set<unsigned>> per_xcc;
  std::map<std::pair<int, int>, int> per_se;
  for (auto& kv : cnt) {
    const int xcc = kv.first >> 16, se = (kv.first >> 5) & 7;
    per_xcc[xcc].insert(kv.first);
    per_se[{xcc, se}]++;
  }
  printf("%-28s CUs %3zu |", name, cnt.size());
  for (auto& kv : per_xcc) printf(" x%d:%zu", kv.first, kv.second.size());
  printf(" | SE:");
  for (auto& kv : per_se) printf(" %d.%d=%d", kv.first.first, kv.first.second, kv.second);
  printf("\n");
}

static std::vector<uint32_t> mask_of(int ncu, bool (*pick)(int, int), int arg) {
  std::vector<uint32_t> m((ncu + 31) / 32, 0u);
  for (int i = 0; i < ncu; ++i)
    if (pick(i, arg)) m[i / 32] |= 1u << (i % 32);
  return m;
}

int main() {
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  printf("multiprocessors %d\n", ncu);
  unsigned* d_out;
  CK(hipMalloc(&d_out, kWG * 4));
  report("no mask", run({}, d_out));
  report("all bits", run(mask_of(ncu, [](int, int) { return true; }, 0), d_out));
  // bits [8k, 8k+8): which (SE, CU) sub-bit k selects in each XCD
  for (int k = 0; k < ncu / 8; ++k) {
    auto cnt = run(mask_of(ncu, [](int i, int a) { return i / 8 == a; }, k), d_out);
    char nm[64];
    snprintf(nm, sizeof nm, "bits [%d,%d)", 8 * k, 8 * k + 8);
    std::map<int, std::vector<unsigned>> xs;
    for (auto& kv : cnt) xs[kv.first >> 16].push_back(kv.first & 0xff);
    printf("%-28s CUs %3zu |", nm, cnt.size());
    for (auto& kv : xs) {
      printf(" x%d:", kv.first);
      for (unsigned v : kv.second) printf("se%u/sh%u/cu%u ", (v >> 5) & 7, (v >> 4) & 1, v & 15);
    }
    printf("\n");
  }
  // decode / encoder splits: decode on sub-bits j < n (bits < 8n), encoder on the rest
  for (int n : {4, 8, 12, 16}) {
    char nm[64];
    snprintf(nm, sizeof nm, "decode bits < %d", 8 * n);
    report(nm, run(mask_of(ncu, [](int i, int a) { return i < a; }, 8 * n), d_out));
    snprintf(nm, sizeof nm, "encoder bits >= %d", 8 * n);
    report(nm, run(mask_of(ncu, [](int i, int a) { return i >= a; }, 8 * n), d_out));
  }
  CK(hipFree(d_out));
  printf("done\n");
  return 0;
}
