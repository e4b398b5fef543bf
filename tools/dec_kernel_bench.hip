// Decode-projection launch cost on MI355X: the library's own gemm_dec_kernel instances (gemm_impl.h)
// at the C2 shapes (whisper-small, 32 rows), each replayed as a hipGraph chain of 100 dependent
// launches with the weights rotating over 1 GiB (cold, as in the decode step), against a bare
// stream kernel moving the same bytes. Prints µs per launch (gap included).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I whisper_context_biasing_amd/csrc tools/dec_kernel_bench.hip -o tools/dec_kernel_bench
#include "gemm_impl.h"

#include <algorithm>
#include <functional>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

using namespace wcb;

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
  return ms * 1e3 / (reps * n);
}

typedef float f4 __attribute__((ext_vector_type(4)));
template <int NT, int WPL, int APL>
__global__ __launch_bounds__(NT) void k_stream(const f4* __restrict__ w, long w_stride_wg, const f4* __restrict__ act_in,
                                               long act_elems, f4* __restrict__ act_out, unsigned long long* st) {
  const int tid = threadIdx.x;
  const unsigned long long t0 = st ? stamp_now() : 0ull;
  const f4* wp = w + blockIdx.x * w_stride_wg + tid;
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
  f4 wv[WPL > 0 ? WPL : 1];
#pragma unroll
  for (int i = 0; i < WPL; ++i) wv[i] = __builtin_nontemporal_load(wp + i * NT);
  f4 av[APL > 0 ? APL : 1];
#pragma unroll
  for (int i = 0; i < APL; ++i) av[i] = act_in[(blockIdx.x * 64 + tid + i * NT) % act_elems];
  unsigned long long t1 = 0;
  if (st) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); t1 = stamp_now(); }
#pragma unroll
  for (int i = 0; i < WPL; ++i) acc += wv[i];
#pragma unroll
  for (int i = 0; i < APL; ++i) acc += av[i];
  if (tid < 64) act_out[(blockIdx.x * 64 + tid) % act_elems] = acc;
  if (st && tid == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned long long* p = st + blockIdx.x * 4;
    p[0] = t0; p[1] = t1; p[2] = t1; p[3] = stamp_now();
  }
}

char* g_w;
const size_t kW = (size_t)1 << 30;
float *g_x, *g_bias, *g_lnw, *g_lnb;
bf16_t *g_x16, *g_a, *g_out, *g_kv;
int* g_pos;

GemmArgs base(int N, int K, long wsz) {
  GemmArgs g;
  g.M = 32; g.N = N; g.K = K; g.ldw = K; g.lda = K; g.ldc = N;
  (void)wsz;
  return g;
}

template <int MF, int NW, int KPW, int AM>
void run(const char* name, GemmArgs g0, int gx) {
  const long wbytes = (long)g0.N * g0.K * 2;
  const long nreg = (long)(kW / wbytes);
  const int gy = (g0.M + MF * 16 - 1) / (MF * 16);
  double us = time_graph(100, [&](int i, hipStream_t s) {
    GemmArgs g = g0;
    g.W = g_w + (i % nreg) * wbytes;
    hipLaunchKernelGGL((gemm_dec_kernel<bf16_t, MF, NW, KPW, AM, false>), dim3(gx, gy), dim3(NW * 64), 0, s, g);
  });
  printf("%-40s MF=%d NW=%2d KPW=%2d AM=%d grid=%4dx%d: %6.2f us/launch\n", name, MF, NW, KPW, AM, gx, gy, us);
  fflush(stdout);
}

void run_lean(const char* name, GemmArgs g0) {
  const long wbytes = (long)g0.N * g0.K * 2;
  const long nreg = (long)(kW / wbytes);
  bool ok = true;
  double us = time_graph(100, [&](int i, hipStream_t s) {
    GemmArgs g = g0;
    g.W = g_w + (i % nreg) * wbytes;
    ok &= launch_lean<bf16_t>(g, s);
  });
  printf("%-40s lean%s: %6.2f us/launch\n", name, ok ? "" : " (NOT TAKEN)", us);
  fflush(stdout);
}

// per-workgroup phase stamps of every launch of a 100-launch chain (s_memrealtime, 10 ns ticks):
// median over launches 10..99 of: dispatch gap (first start - previous launch's last end), start spread,
// loads landed, LN + MFMA + LDS exchange, epilogue + store drain, launch span
void stamp_report(const char* name, const unsigned long long* dev, int n, int nwg) {
  std::vector<unsigned long long> h((size_t)n * nwg * 4);
  CHK(hipMemcpy(h.data(), dev, h.size() * 8, hipMemcpyDeviceToHost));
  auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
  std::vector<double> gap, spread, ld, mid, ep, span, wgdur;
  for (int i = 10; i < n; ++i) {
    const unsigned long long* a = &h[(size_t)i * nwg * 4];
    const unsigned long long* b = &h[(size_t)(i - 1) * nwg * 4];
    unsigned long long s0 = ~0ull, s1 = 0, e1 = 0, pe = 0;
    std::vector<double> l, m, e, d;
    for (int w = 0; w < nwg; ++w) {
      s0 = std::min(s0, a[w * 4]); s1 = std::max(s1, a[w * 4]); e1 = std::max(e1, a[w * 4 + 3]);
      pe = std::max(pe, b[w * 4 + 3]);
      l.push_back((a[w * 4 + 1] - a[w * 4]) * 0.01); m.push_back((a[w * 4 + 2] - a[w * 4 + 1]) * 0.01);
      e.push_back((a[w * 4 + 3] - a[w * 4 + 2]) * 0.01); d.push_back((a[w * 4 + 3] - a[w * 4]) * 0.01);
    }
    gap.push_back(((double)s0 - (double)pe) * 0.01); spread.push_back((s1 - s0) * 0.01);
    ld.push_back(med(l)); mid.push_back(med(m)); ep.push_back(med(e)); wgdur.push_back(med(d)); span.push_back((e1 - s0) * 0.01);
  }
  printf("%-22s stamps (us, medians): gap %5.2f  start-spread %5.2f  loads %5.2f  ln+mfma+lds %5.2f  epilogue %5.2f  wg %5.2f  span %5.2f\n",
         name, med(gap), med(spread), med(ld), med(mid), med(ep), med(wgdur), med(span));
  fflush(stdout);
}

void run_lean_stamped(const char* name, GemmArgs g0) {
  const long wbytes = (long)g0.N * g0.K * 2;
  const long nreg = (long)(kW / wbytes);
  const int nwg = ((g0.N + 15) / 16) * ((g0.M + 15) / 16);
  const int n = 100;
  unsigned long long* st;
  CHK(hipMalloc(&st, (size_t)n * nwg * 32));
  CHK(hipMemset(st, 0, (size_t)n * nwg * 32));
  time_graph(n, [&](int i, hipStream_t s) {
    GemmArgs g = g0;
    g.W = g_w + (i % nreg) * wbytes;
    g_lean_stamp = st + (long)i * nwg * 4;
    launch_lean<bf16_t>(g, s);
    g_lean_stamp = nullptr;
  });
  stamp_report(name, st, n, nwg);
  CHK(hipFree(st));
}

// the lean out-projection with fragment-major weights (layout only: the bench's weights are zeros)
template <int NW, int KPW, bool LN, int EPI, int MF = 1, bool AFM = false>
void run_wfm(const char* name, GemmArgs g0, bool stamped) {
  const long wbytes = (long)g0.N * g0.K * 2;
  const long nreg = (long)(kW / wbytes);
  const int nwg = ((g0.N + 15) / 16) * ((g0.M + 15) / 16);
  unsigned long long* st = nullptr;
  if (stamped) { CHK(hipMalloc(&st, (size_t)100 * nwg * 32)); CHK(hipMemset(st, 0, (size_t)100 * nwg * 32)); }
  double us = time_graph(100, [&](int i, hipStream_t s) {
    DecLean<bf16_t> p;
    p.W = reinterpret_cast<const bf16_t*>(g_w + (i % nreg) * wbytes);
    p.A = reinterpret_cast<const bf16_t*>(LN ? g0.ln_a16 : g0.A); p.bias = g0.bias; p.gam = g0.ln_w; p.bet = g0.ln_b;
    p.x = EPI == 1 ? reinterpret_cast<float*>(g0.out) : nullptr;
    p.out = reinterpret_cast<bf16_t*>(EPI == 1 ? g0.out16 : g0.out);
    p.kv = reinterpret_cast<bf16_t*>(g0.kv_out); p.pos = g0.pos;
    p.M = g0.M; p.N = g0.N; p.lda = (int)g0.lda; p.ldo = (int)g0.ldc;
    p.n_split = g0.n_split; p.kvB = g0.hs_B; p.kvH = g0.hs_H; p.kvT = g0.kv_T; p.grp_n = 0; p.grp_off = 0;
    p.stamp = st ? st + (long)i * nwg * 4 : nullptr;
    hipLaunchKernelGGL((dec_lean_kernel<bf16_t, MF, NW, KPW, LN, EPI, false, false, true, AFM>),
                       dim3((g0.N + 15) / 16, (g0.M + 16 * MF - 1) / (16 * MF)), dim3(NW * 64), 0, s, p);
  });
  printf("%-40s lean, fragment-major W%s, %d-row wgs: %6.2f us/launch\n", name, AFM ? " and A" : "", 16 * MF, us);
  if (st) { stamp_report(name, st, 100, nwg); CHK(hipFree(st)); }
  fflush(stdout);
}

// weights cold in HBM vs Infinity-Cache resident, activations written by the previous launch vs
// constant: the lean d x d projection (EPI 0, fragment-major W), `nl` launches per graph (100: 118 MB
// of weights, replays hit the 256 MB Infinity Cache; 850: 1 GB, every replay from HBM)
void run_cold(int nl, bool fresh) {
  const long wbytes = 768L * 768 * 2;
  const long nreg = (long)(kW / wbytes);
  double us = time_graph(nl, [&](int i, hipStream_t s) {
    DecLean<bf16_t> p;
    p.W = reinterpret_cast<const bf16_t*>(g_w + (i % nreg) * wbytes);
    bf16_t* a0 = g_a;
    bf16_t* a1 = g_a + 32 * 768;
    p.A = fresh ? ((i & 1) ? a1 : a0) : a0;
    p.out = fresh ? ((i & 1) ? a0 : a1) : g_out;
    p.bias = g_bias; p.gam = p.bet = nullptr; p.x = nullptr; p.kv = nullptr; p.pos = g_pos;
    p.M = 32; p.N = 768; p.lda = 768; p.ldo = 768; p.n_split = 0; p.kvB = p.kvH = p.kvT = 0; p.grp_n = p.grp_off = 0;
    hipLaunchKernelGGL((dec_lean_kernel<bf16_t, 1, 4, 6, false, 0, false, false, true>), dim3(48, 2), dim3(256), 0, s, p);
  });
  printf("lean d x d, fragment-major W: %4d launches/graph (%s weights), %s activations: %6.2f us/launch\n", nl,
         nl * wbytes > (300L << 20) ? "HBM-cold" : "cache-resident", fresh ? "fresh (previous launch's output)" : "constant", us);
  fflush(stdout);
}

// instruction-cache pressure: the same d x d projection chain, one kernel object vs a cycle through
// 8 distinct instances of the lean kernel (different code, same work: EPI 0 with/without GELU, LN
// on/off, 4 / 8 waves)
template <int NW, int KPW, bool LN, bool GELU>
void launch_var(int i, hipStream_t s) {
  const long wbytes = 768L * 768 * 2;
  const long nreg = (long)(kW / wbytes);
  DecLean<bf16_t> p;
  p.W = reinterpret_cast<const bf16_t*>(g_w + (i % nreg) * wbytes);
  bf16_t* a0 = g_a;
  bf16_t* a1 = g_a + 32 * 768;
  p.A = (i & 1) ? a1 : a0;
  p.out = (i & 1) ? a0 : a1;
  p.bias = g_bias; p.gam = g_lnw; p.bet = g_lnb; p.x = nullptr; p.kv = nullptr; p.pos = g_pos;
  p.M = 32; p.N = 768; p.lda = 768; p.ldo = 768; p.n_split = 0; p.kvB = p.kvH = p.kvT = 0; p.grp_n = p.grp_off = 0;
  hipLaunchKernelGGL((dec_lean_kernel<bf16_t, 1, NW, KPW, LN, 0, GELU, false, true>), dim3(48, 2), dim3(NW * 64), 0, s, p);
}
void run_icache() {
  double one = time_graph(400, [&](int i, hipStream_t s) { launch_var<4, 6, false, false>(i, s); });
  double cyc = time_graph(400, [&](int i, hipStream_t s) {
    switch (i % 8) {
      case 0: launch_var<4, 6, false, false>(i, s); break;
      case 1: launch_var<4, 6, false, true>(i, s); break;
      case 2: launch_var<4, 6, true, false>(i, s); break;
      case 3: launch_var<4, 6, true, true>(i, s); break;
      case 4: launch_var<8, 3, false, false>(i, s); break;
      case 5: launch_var<8, 3, false, true>(i, s); break;
      case 6: launch_var<8, 3, true, false>(i, s); break;
      default: launch_var<8, 3, true, true>(i, s); break;
    }
  });
  double cyc_ln = time_graph(400, [&](int i, hipStream_t s) {   // the LN half alone, 2 objects
    if (i & 1) launch_var<4, 6, true, false>(i, s); else launch_var<4, 6, true, true>(i, s);
  });
  printf("icache: one kernel object %6.2f us/launch, 8 objects cycled %6.2f us/launch, 2 LN objects %6.2f\n", one, cyc, cyc_ln);
  fflush(stdout);
}

// the LM head: persistent column walk (gemm_dec_kernel P), LN-fused, argmax partials, with and
// without the bias boost (root bits read per tile)
template <int AM = 2, bool WFM = false>
void run_lm_head(bool boost) {
  const int V = 51865, K = 768, M = 32;
  static uint32_t* bits = nullptr;
  static float *pv = nullptr;
  static int *pi = nullptr, *rb = nullptr, *step = nullptr;
  if (!bits) {
    CHK(hipMalloc(&bits, (V / 32 + 1) * 4)); CHK(hipMemset(bits, 0x55, (V / 32 + 1) * 4));
    CHK(hipMalloc(&pv, M * kDecWalkers * 4)); CHK(hipMalloc(&pi, M * kDecWalkers * 4));
    CHK(hipMalloc(&rb, M * 4)); CHK(hipMemset(rb, 0, M * 4));
    CHK(hipMalloc(&step, 4)); CHK(hipMemset(step, 0, 4));
  }
  const long wbytes = (long)V * K * 2;
  double us = time_graph(20, [&](int i, hipStream_t s) {
    GemmArgs g = base(V, K, 0);
    g.M = M; g.ldc = V;
    g.W = g_w + (i % 8) * wbytes;
    g.A = AM == 0 ? (const void*)g_x16 : (const void*)g_x; g.lda = K; g.out_f32 = 1; g.out = nullptr;
    if (AM == 2) { g.ln_w = g_lnw; g.ln_b = g_lnb; g.ln_a16 = g_x16; }
    g.W_fm = g.W;
    g.sel_val = pv; g.sel_idx = pi; g.sel_root_bits = bits; g.sel_lam = boost ? 2.f : 0.f; g.sel_rowbase = rb;
    g.sel_eos = 50257; g.sel_step = step; g.sel_min_new = 0;
    const int gx = std::min((V + 15) / 16, kDecWalkers);
    hipLaunchKernelGGL((gemm_dec_kernel<bf16_t, 2, 4, 6, AM, true, WFM>), dim3(gx, 1), dim3(256), 0, s, g);
  });
  printf("lm head (V=%d, 32 rows, %d walkers, AM %d, WFM %d)%s: %6.2f us/launch\n", V, kDecWalkers, AM, (int)WFM,
         boost ? " + boost" : "", us);
  fflush(stdout);
}

template <int NT, int WPL, int APL>
void run_stream(const char* name, int grid, bool stamped = false) {
  const long per_wg = (long)NT * WPL, per_launch = per_wg * grid;
  const long nreg = (long)(kW / 16) / per_launch;
  const long act_elems = 98304 / 16;
  unsigned long long* st = nullptr;
  if (stamped) { CHK(hipMalloc(&st, (size_t)100 * grid * 32)); CHK(hipMemset(st, 0, (size_t)100 * grid * 32)); }
  double us = time_graph(100, [&](int i, hipStream_t s) {
    const f4* w = reinterpret_cast<const f4*>(g_w) + (i % nreg) * per_launch;
    f4* in = reinterpret_cast<f4*>(g_x) + (i & 1) * act_elems;
    f4* out = reinterpret_cast<f4*>(g_x) + ((i + 1) & 1) * act_elems;
    hipLaunchKernelGGL((k_stream<NT, WPL, APL>), dim3(grid), dim3(NT), 0, s, w, per_wg, in, act_elems, out,
                       st ? st + (long)i * grid * 4 : nullptr);
  });
  printf("%-40s NT=%d W/wg=%5.1f KB A/wg=%5.1f KB grid=%4d: %6.2f us/launch\n", name, NT, WPL * NT * 16 / 1024.0,
         APL * NT * 16 / 1024.0, grid, us);
  fflush(stdout);
  if (st) { stamp_report(name, st, 100, grid); CHK(hipFree(st)); }
}

int main() {
  CHK(hipSetDevice(0));
  CHK(hipMalloc(&g_w, kW));
  CHK(hipMemset(g_w, 0, kW));
  CHK(hipMalloc(&g_x, 4 << 20));
  CHK(hipMemset(g_x, 0, 4 << 20));
  CHK(hipMalloc(&g_x16, 4 << 20));
  CHK(hipMemset(g_x16, 0, 4 << 20));
  CHK(hipMalloc(&g_a, 4 << 20));
  CHK(hipMemset(g_a, 0, 4 << 20));
  CHK(hipMalloc(&g_out, 4 << 20));
  CHK(hipMalloc(&g_kv, 64 << 20));
  CHK(hipMalloc(&g_bias, 1 << 16));
  CHK(hipMemset(g_bias, 0, 1 << 16));
  CHK(hipMalloc(&g_lnw, 1 << 16));
  CHK(hipMemset(g_lnw, 0, 1 << 16));
  CHK(hipMalloc(&g_lnb, 1 << 16));
  CHK(hipMemset(g_lnb, 0, 1 << 16));
  CHK(hipMalloc(&g_pos, 64));
  CHK(hipMemset(g_pos, 0, 64));

  if (getenv("OUT_ONLY")) {   // the out projection's load phase against the byte-matched stream kernel
    GemmArgs o = base(768, 768, 0);
    o.A = g_a; o.bias = g_bias; o.resid = g_x; o.out = g_x; o.out_f32 = 1; o.out16 = g_x16;
    run_stream<256, 0, 0>("stream: nothing", 96, true);
    run_stream<256, 6, 6>("stream: out-proj bytes", 96, true);
    run_stream<256, 6, 0>("stream: out-proj W only", 96, true);
    run_wfm<4, 6, false, 1>("out", o, true);
    run_wfm<4, 6, false, 1, 1, true>("out", o, true);
    GemmArgs x = base(768, 768, 0);
    x.ln_w = g_lnw; x.ln_b = g_lnb; x.ln_a16 = g_x16; x.A = g_x; x.bias = g_bias; x.out = g_out;
    run_wfm<4, 6, true, 0>("xq (LN)", x, true);
    run_wfm<4, 6, true, 0, 1, true>("xq (LN)", x, true);
    return 0;
  }
  // reference points: empty-ish and byte-matched stream kernels
  run_stream<256, 0, 0>("stream: nothing", 96);
  run_stream<256, 6, 6>("stream: out-proj bytes", 96);
  run_stream<256, 6, 6>("stream: out-proj bytes, 192 wgs", 192);

  run_lm_head(false);
  run_lm_head(true);
  run_lm_head<2, true>(true);
  run_lm_head<0, true>(true);
  run_lm_head<0, true>(false);
  run_stream<256, 39, 0>("stream: LM-head bytes (80 MB), 512 wgs", 512);
  run_stream<256, 20, 0>("stream: LM-head bytes (80 MB), 1024 wgs", 1024);
  if (getenv("LM_ONLY")) return 0;
  run_icache();
  run_cold(100, false);
  run_cold(850, false);
  run_cold(100, true);
  run_cold(850, true);
  // out / xo projection: A = T rows, bias, residual f32 in place, 16-bit copy
  GemmArgs o = base(768, 768, 0);
  o.A = g_a; o.bias = g_bias; o.resid = g_x; o.out = g_x; o.out_f32 = 1; o.out16 = g_x16;
  run<1, 4, 6, 0>("out: bias+resid+f32+x16 (library)", o, 48);
  run_lean("out", o);
  run_lean_stamped("out", o);
  run_wfm<4, 6, false, 1>("out", o, false);
  run_wfm<4, 6, false, 1, 2>("out", o, false);
  run<2, 4, 6, 0>("out: MF=2", o, 48);
  run<1, 8, 3, 0>("out: NW=8", o, 48);
  run<2, 8, 3, 0>("out: MF=2 NW=8", o, 48);
  GemmArgs o2 = o; o2.out16 = nullptr;
  run<1, 4, 6, 0>("out: no x16", o2, 48);
  GemmArgs o3 = o; o3.resid = nullptr; o3.out16 = nullptr; o3.out_f32 = 0; o3.out = g_out; o3.bias = nullptr;
  run<1, 4, 6, 0>("out: plain T out", o3, 48);
  // LN-fused projections (A = LN of the 16-bit residual copy)
  GemmArgs q = base(2304, 768, 0);
  q.ln_w = g_lnw; q.ln_b = g_lnb; q.ln_a16 = g_x16; q.A = g_x; q.lda = 768; q.bias = g_bias;
  q.out = g_out; q.mode = 2; q.n_split = 768; q.kv_out = g_kv; q.hs_B = 32; q.hs_H = 12; q.kv_T = 80; q.pos = g_pos;
  run<1, 4, 6, 2>("qkv: LN16 + kv append (library)", q, 144);
  run_lean("qkv", q);
  run_lean_stamped("qkv", q);
  run_wfm<4, 6, true, 2>("qkv", q, false);
  run<2, 4, 6, 2>("qkv: MF=2", q, 144);
  GemmArgs xq = base(768, 768, 0);
  xq.ln_w = g_lnw; xq.ln_b = g_lnb; xq.ln_a16 = g_x16; xq.A = g_x; xq.bias = g_bias; xq.out = g_out;
  run<1, 4, 6, 2>("xq: LN16 (library)", xq, 48);
  run_lean("xq", xq);
  run_lean_stamped("xq", xq);
  run_wfm<4, 6, true, 0>("xq", xq, false);
  run_wfm<4, 6, true, 0, 2>("xq", xq, false);
  run<2, 4, 6, 2>("xq: MF=2", xq, 48);
  GemmArgs xq0 = xq; xq0.ln_w = xq0.ln_b = nullptr; xq0.ln_a16 = nullptr; xq0.A = g_a;
  run<1, 4, 6, 0>("xq without LN", xq0, 48);
  GemmArgs f1 = base(3072, 768, 0);
  f1.ln_w = g_lnw; f1.ln_b = g_lnb; f1.ln_a16 = g_x16; f1.A = g_x; f1.bias = g_bias; f1.out = g_out; f1.act = 1;
  run<1, 4, 6, 2>("fc1: LN16 + gelu (library)", f1, 192);
  run_lean("fc1", f1);
  run<2, 4, 6, 2>("fc1: MF=2", f1, 192);
  GemmArgs f2 = base(768, 3072, 0);
  f2.A = g_a; f2.bias = g_bias; f2.resid = g_x; f2.out = g_x; f2.out_f32 = 1; f2.out16 = g_x16;
  run<1, 8, 12, 0>("fc2: K=3072 (library)", f2, 48);
  run_lean("fc2", f2);
  run_lean_stamped("fc2", f2);
  run_wfm<8, 12, false, 1>("fc2", f2, false);
  run_wfm<8, 12, false, 1, 2>("fc2", f2, false);
  run_wfm<16, 6, false, 1>("fc2 NW=16", f2, false);
  run<2, 8, 12, 0>("fc2: MF=2", f2, 48);
  run<1, 16, 6, 0>("fc2: NW=16", f2, 48);
  // grouped q' = W_k,h^T q_h (K = 64)
  GemmArgs kq = base(9216, 64, 0);
  kq.A = g_a; kq.lda = 768; kq.out = g_out; kq.ldc = 9216; kq.a_grp_n = 768; kq.a_grp_off = 64;
  run<1, 2, 1, 3>("kq: grouped K=64 (library)", kq, 576);
  run_lean("kq", kq);
  run<2, 2, 1, 3>("kq: MF=2", kq, 576);
  return 0;
}
