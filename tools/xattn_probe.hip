// Phase timing of the greedy decode's encoder-space cross-attention kernel (k_xenc.hip
// attn_xenc_reg_kernel, built here with WCB_XENC_PROBE: wave 0 of every workgroup stamps s_memtime at
// kernel start (0), after its first chunk loads are issued (1), after each chunk (2..7), before the
// range-partial stores (10) and after they drained (11)). C2 shape: 32 rows, 1500 keys, d 768,
// 12 heads, 8 key ranges; row layout and fragment-major layout. Prints the per-launch time of a graph of
// 48 launches and the phase offsets (cycles, median over workgroups) of the last launch.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/xattn_probe.hip -o tools/xattn_probe
#define WCB_XENC_PROBE 1
#include "../whisper_context_biasing_amd/csrc/k_xenc.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void fill_rand(unsigned short* p, long n, unsigned seed, float scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)(i * 2654435761u) ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    const float f = ((x & 0xffff) / 65535.f - 0.5f) * scale;
    p[i] = (unsigned short)(__float_as_uint(f) >> 16);
  }
}

int main() {
  using namespace wcb;
  const int rows = 32, S = 1500, D = 768, H = 12, nsplit = 8;
  unsigned short *enc, *encfm, *qp;
  float *part, *ml;
  unsigned long long* probe;
  const long n_enc = (long)rows * S * D, n_fm = xenc_fm_elems(rows, S, D);
  CHK(hipMalloc(&enc, n_enc * 2));
  CHK(hipMalloc(&encfm, n_fm * 2));
  CHK(hipMalloc(&qp, (long)rows * H * D * 2));
  CHK(hipMalloc(&part, (long)rows * nsplit * H * D * 4));
  CHK(hipMalloc(&ml, (long)rows * nsplit * H * 2 * 4));
  CHK(hipMalloc(&probe, 256 * 16 * 8));
  fill_rand<<<1024, 256>>>(enc, n_enc, 1u, 2.f);
  fill_rand<<<1024, 256>>>(qp, (long)rows * H * D, 7u, 0.2f);
  hipStream_t s;
  CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  xenc_to_fm(kBF16, enc, encfm, rows, S, D, s);
  CHK(hipStreamSynchronize(s));
  for (int fm = 0; fm < 2; ++fm) {
    XencArgs a;
    a.enc = fm ? (const void*)encfm : (const void*)enc;
    a.enc_sb = fm ? xenc_fm_elems(1, S, D) : (long)S * D;
    a.qp = qp; a.rows = rows; a.H = H; a.D = D; a.S = S; a.nsplit = nsplit; a.part = part; a.ml = ml;
    a.variant = 1; a.fm = fm;
    a.stamp.base = probe;
    hipGraph_t g;
    hipGraphExec_t ge;
    CHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < 48; ++i) xenc_attention(kBF16, a, s);
    CHK(hipStreamEndCapture(s, &g));
    CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
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
    std::vector<unsigned long long> h(256 * 16);
    CHK(hipMemcpy(h.data(), probe, h.size() * 8, hipMemcpyDeviceToHost));
    printf("%s layout: %.2f us per launch (48 in a graph)\n", fm ? "fragment-major" : "row", best * 1e3 / 48);
    const int ks[] = {1, 2, 3, 4, 5, 6, 7, 10, 11};
    for (int k : ks) {
      std::vector<long> d;
      for (int w = 0; w < 256; ++w)
        if (h[w * 16 + k] && h[w * 16]) d.push_back((long)(h[w * 16 + k] - h[w * 16]));
      if (d.empty()) continue;
      std::sort(d.begin(), d.end());
      printf("  phase %2d: median %7ld  p90 %7ld cycles after start (%zu workgroups)\n", k, d[d.size() / 2],
             d[d.size() * 9 / 10], d.size());
    }
    // spread of workgroup start / end over the launch
    unsigned long long mn = ~0ull, mx = 0, mn_end = ~0ull, mx_end = 0;
    for (int w = 0; w < 256; ++w) {
      mn = std::min(mn, h[w * 16]); mx = std::max(mx, h[w * 16]);
      mn_end = std::min(mn_end, h[w * 16 + 11]); mx_end = std::max(mx_end, h[w * 16 + 11]);
    }
    printf("  workgroup starts spread %llu cycles; first start -> last end %llu cycles\n", mx - mn, mx_end - mn);
    CHK(hipGraphExecDestroy(ge));
    CHK(hipGraphDestroy(g));
    if (fm) {   // the range merge + W_v behind the fragment-major xattn (the runtime's pair)
      unsigned short* wv;
      float* bv;
      unsigned short* o;
      unsigned long long* mp;
      CHK(hipMalloc(&wv, (long)D * D * 2));
      CHK(hipMalloc(&bv, D * 4));
      CHK(hipMalloc(&o, (long)rows * D * 2));
      CHK(hipMalloc(&mp, 4096 * 8 * 8));
      CHK(hipMemset(bv, 0, D * 4));
      fill_rand<<<1024, 256>>>(wv, (long)D * D, 11u, 0.05f);
      CHK(hipMemcpyToSymbol(HIP_SYMBOL(wcb_merge_probe), &mp, sizeof(mp)));
      hipGraph_t g2;
      hipGraphExec_t ge2;
      CHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (int i = 0; i < 48; ++i) { xenc_attention(kBF16, a, s); xenc_merge_v(kBF16, a, wv, bv, o, D, s); }
      CHK(hipStreamEndCapture(s, &g2));
      CHK(hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0));
      CHK(hipGraphLaunch(ge2, s));
      CHK(hipStreamSynchronize(s));
      float best2 = 1e30f;
      for (int r = 0; r < 5; ++r) {
        CHK(hipEventRecord(e0, s));
        CHK(hipGraphLaunch(ge2, s));
        CHK(hipEventRecord(e1, s));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        best2 = std::min(best2, ms);
      }
      const int nm = H * rows / 2;
      std::vector<unsigned long long> hm((size_t)nm * 8);
      CHK(hipMemcpy(hm.data(), mp, hm.size() * 8, hipMemcpyDeviceToHost));
      printf("xattn + merge_v: %.2f us per pair (48 in a graph)\n", best2 * 1e3 / 48);
      for (int k = 1; k <= 4; ++k) {
        std::vector<long> d;
        for (int w = 0; w < nm; ++w) d.push_back((long)(hm[w * 8 + k] - hm[w * 8 + k - 1]));
        std::sort(d.begin(), d.end());
        printf("  merge phase %d-%d: median %6ld p90 %6ld cycles\n", k - 1, k, d[d.size() / 2], d[d.size() * 9 / 10]);
      }
      unsigned long long mn = ~0ull, mx = 0;
      for (int w = 0; w < nm; ++w) { mn = std::min(mn, hm[w * 8]); mx = std::max(mx, hm[w * 8 + 4]); }
      printf("  merge: first start -> last end %llu cycles over %d workgroups\n", mx - mn, nm);
    }
  }
  return 0;
}
