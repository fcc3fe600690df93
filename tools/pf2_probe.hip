// Diagnostic probe for gemm_pf2_k (csrc/gemm_pf2.hip, built with per-block s_memtime stamps): times one prefill
// linear shape per tile configuration and reports, per configuration, the median block's cycles in the main loop and
// the epilogue, the blocks resident at once, and the clock (s_memtime ticks vs s_memrealtime).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I qwen3-tts_amd/csrc -I include tools/pf2_probe.hip -o tools/pf2_probe
// run:   tools/pf2_probe M N K epi(0 store f32 / 1 add f32 / 2 swiglu bf16) rms(0/1)
#define QT_PF2_STAMPS
#define QT_PF2_PROBE
#include "../qwen3-tts_amd/csrc/gemm_pf2.hip"
#include <algorithm>
#include <cstdio>
#include <vector>
#include <string>
#include <cstring>
#include <cmath>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void fill_bf16(bf16_t* p, long long n, unsigned seed) {
  long long i = blockIdx.x * 256LL + threadIdx.x;
  for (; i < n; i += gridDim.x * 256LL) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    p[i] = f2bf(((h & 0xFFFF) / 32768.f - 1.f) * 0.5f);
  }
}
__global__ void clock_k(unsigned long long* o) {
  if (threadIdx.x == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long t = t0;
    while (t - t0 < 2000000) t = __builtin_amdgcn_s_memtime();
    o[0] = t - t0; o[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

static std::vector<unsigned char> g_ref;
static double g_relerr = 0;
static unsigned* g_cnt = nullptr;
static float* g_part = nullptr;
constexpr long long PART_BYTES = 64ll << 20;
template <typename OT, int BM, int NTB, int NS, int WM, int WN, int EPI, int ABL = 0, int PP = 0, int KS = 1>
void run(const char* name, GemmP p, int reps) {
  if (!g_cnt) {
    CK(hipMalloc(&g_cnt, 4096 * 4)); CK(hipMemset(g_cnt, 0, 4096 * 4));
    CK(hipMalloc(&g_part, PART_BYTES));
  }
  p.cnt = g_cnt; p.part = g_part; p.part_bytes = PART_BYTES;
  {  // the split records must fit the partial buffer (and the counters their array)
    constexpr long long REC = 8ll * (BM / WM / 16) * (NTB / WN) * 256 + WN * BM;
    const long long tiles = (long long)((p.M + BM - 1) / BM) * (((p.N + 15) / 16 + NTB - 1) / NTB);
    if (KS > 1 && (tiles * KS * REC * 4 > PART_BYTES || tiles > 4096)) { printf("%-28s skipped (records)\n", name); return; }
  }
  const int ntl = (p.N + 15) / 16;
  const int nwg = ((p.M + BM - 1) / BM) * ((ntl + NTB - 1) / NTB);
  auto go = [&] { hipLaunchKernelGGL((gemm_pf2_k<OT, BM, NTB, NS, WM, WN, true, EPI, ABL, (KS > 1), PP>), dim3(nwg, KS), dim3(WM * WN * 64), 0, 0, p); };
  // one launch on a zeroed output, compared bit for bit with the first configuration's (same per-element k order)
  const size_t obytes = (size_t)p.M * p.ldo * sizeof(OT);
  CK(hipMemset(p.out, 0, obytes));
  go();
  CK(hipDeviceSynchronize());
  std::vector<unsigned char> mine(obytes);
  CK(hipMemcpy(mine.data(), p.out, obytes, hipMemcpyDeviceToHost));
  size_t diff = 0;
  if (g_ref.size() != obytes) g_ref = mine;
  else for (size_t i = 0; i < obytes; i += sizeof(OT)) diff += memcmp(&mine[i], &g_ref[i], sizeof(OT)) != 0;
  double maxd = 0, maxr = 0;
  for (size_t i = 0; i < obytes; i += sizeof(OT)) {
    float a, b;
    if constexpr (sizeof(OT) == 4) { memcpy(&a, &mine[i], 4); memcpy(&b, &g_ref[i], 4); }
    else { unsigned ua = (unsigned)(*(unsigned short*)&mine[i]) << 16, ub = (unsigned)(*(unsigned short*)&g_ref[i]) << 16;
           memcpy(&a, &ua, 4); memcpy(&b, &ub, 4); }
    maxd = std::max(maxd, (double)fabsf(a - b)); maxr = std::max(maxr, (double)fabsf(b));
  }
  g_relerr = maxd / std::max(maxr, 1e-30);
  for (int i = 0; i < 20; ++i) go();
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) go();
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> st((size_t)nwg * KS * 4);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(pf2_stamps), st.size() * 8));
  std::vector<double> loop, epi, life;
  unsigned long long t_min = ~0ull, t_max = 0;
  for (int b = 0; b < nwg * KS; ++b) {
    loop.push_back((double)(st[b * 4 + 1] - st[b * 4 + 0]));
    const unsigned long long t2 = (ABL & 8) ? st[b * 4 + 1] : st[b * 4 + 2];
    epi.push_back((double)(t2 - st[b * 4 + 1]));
    life.push_back((double)(t2 - st[b * 4 + 0]));
    t_min = std::min(t_min, st[b * 4]); t_max = std::max(t_max, st[b * 4 + 2]);
  }
  auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
  const double span = (double)(t_max - t_min);
  const double us = 1e3 * ms / reps;
  const double fl = 2.0 * p.M * p.N * (double)p.Klog;
  (void)span;
  printf("%-28s %5d blocks x%d  %8.1f us  %7.1f TF/s | block median: loop %7.0f cyc  epilogue %6.0f cyc | %zu differ, max rel %.2e\n",
         name, nwg, KS, us, fl / us / 1e6, med(loop), med(epi), diff, g_relerr);
}

struct Shape { int M, N, K, epi, rms; };

template <typename OT, int E>
void sweep(GemmP p, int reps) {
  run<OT, 128, 4, 3, 2, 2, E>("cfg3 128x64 4w", p, reps);
  run<OT, 256, 8, 3, 4, 2, E>("cfg4 256x128 8w", p, reps);
  run<OT, 128, 8, 3, 2, 4, E>("cfg5 128x128 8w", p, reps);
  run<OT, 128, 8, 4, 2, 2, E>("cfg13 128x128 4w", p, reps);
  run<OT, 64, 6, 4, 2, 2, E>("cfg11 64x96 4w", p, reps);
  run<OT, 256, 10, 3, 2, 2, E>("cfg9 256x160 4w", p, reps);
  run<OT, 64, 8, 4, 4, 2, E>("8w 64x128 ns4", p, reps);
  run<OT, 64, 4, 4, 4, 2, E>("8w 64x64 ns4", p, reps);
  run<OT, 64, 4, 6, 4, 2, E>("8w 64x64 ns6", p, reps);
  run<OT, 128, 4, 4, 4, 2, E>("8w 128x64 ns4", p, reps);
  run<OT, 64, 8, 4, 2, 4, E>("8w 64x128 2x4 ns4", p, reps);
}

int main(int argc, char** argv) {
  // shapes: M N K epi rms, repeated; or "abl M N K epi rms" for the cfg 3 ablation set
  bool abl = argc > 1 && std::string(argv[1]) == "abl";
  std::vector<Shape> shapes;
  for (int i = abl ? 2 : 1; i + 4 < argc; i += 5)
    shapes.push_back({atoi(argv[i]), atoi(argv[i + 1]), atoi(argv[i + 2]), atoi(argv[i + 3]), atoi(argv[i + 4])});
  if (shapes.empty()) shapes.push_back({680, 12288, 2048, 2, 1});
  int Mx = 0; long long Ax = 0, Wx = 0;
  for (auto& s : shapes) { Mx = std::max(Mx, s.M); Ax = std::max(Ax, (long long)s.M * s.K); Wx = std::max(Wx, (long long)s.N * s.K); }
  bf16_t *A, *W; void* out;
  long long Ox = 0;
  for (auto& s : shapes) Ox = std::max(Ox, (long long)s.M * s.N);
  CK(hipMalloc(&A, Ax * 2)); CK(hipMalloc(&W, Wx * 2)); CK(hipMalloc(&out, Ox * 4));
  hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, 0, A, Ax, 1u);
  hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, 0, W, Wx, 2u);
  CK(hipMemset(out, 0, Ox * 4));
  unsigned long long* clk; CK(hipMalloc(&clk, 16));
  hipLaunchKernelGGL(clock_k, dim3(1), dim3(64), 0, 0, clk);
  unsigned long long c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  printf("s_memtime %.3f GHz (vs 100 MHz s_memrealtime, idle)\n", (double)c[0] / c[1] * 0.1);
  const int reps = 50;
  for (auto& sh : shapes) {
    GemmP p{};
    p.M = sh.M; p.N = sh.N; p.Kp = sh.K; p.Klog = sh.K; p.A = A; p.lda = sh.K; p.W = W; p.eps = 1e-6f; p.rms = sh.rms;
    p.act = QT_ACT_NONE; p.epi = sh.epi; p.out = out; p.ldo = sh.epi == QT_EPI_SWIGLU ? sh.N / 2 : sh.N; p.ks = 1;
    printf("M=%d N=%d K=%d epi=%d rms=%d\n", sh.M, sh.N, sh.K, sh.epi, sh.rms);
    g_ref.clear();
    if (abl) {
      if (sh.epi == QT_EPI_SWIGLU) {
        constexpr int E = PF2_SWIGLU;
        run<bf16_t, 128, 4, 3, 2, 2, E>("cfg3 128x64 4w", p, reps);
        run<bf16_t, 128, 4, 3, 2, 2, PF2_GENERIC>("cfg3 generic epilogue", p, reps);
        run<bf16_t, 128, 4, 3, 2, 2, E, 8>("cfg3 no epilogue", p, reps);
        run<bf16_t, 128, 4, 3, 2, 2, E, 10>("cfg3 no loads no epilogue", p, reps);
        run<bf16_t, 128, 4, 3, 2, 2, E, 15>("cfg3 skeleton", p, reps);
      } else {
        constexpr int E = PF2_ADD;
        run<float, 128, 4, 3, 2, 2, E>("cfg3 128x64 4w", p, reps);
        run<float, 128, 4, 3, 2, 2, E, 8>("cfg3 no epilogue", p, reps);
        run<float, 128, 4, 3, 2, 2, E, 10>("cfg3 no loads no epilogue", p, reps);
        run<float, 128, 4, 3, 2, 2, E, 15>("cfg3 skeleton", p, reps);
      }
    } else if (sh.epi == QT_EPI_SWIGLU) sweep<bf16_t, PF2_SWIGLU>(p, reps);
    else if (sh.epi == QT_EPI_ADD) sweep<float, PF2_ADD>(p, reps);
    else sweep<float, PF2_STORE>(p, reps);
  }
  return 0;
}
