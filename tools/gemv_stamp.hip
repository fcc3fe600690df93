// Where does a small decode GEMV's time go?  In-kernel s_memrealtime stamps (100 MHz, comparable across CUs) of a
// code-predictor-shaped GEMV (shipped gemv_wt structure: one 16-column tile per block, K split over the block's
// waves, fold 2, bf16 A, LDS reduction, wave-0 epilogue), launched right after a 1-block marker kernel that stamps
// its own end.  Per launch: marker end -> first block start (boundary), block start spread (dispatch), start ->
// loads landed, -> MFMA done, -> LDS reduction done, -> stored, last block end.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gemv_stamp.hip -o tools/gemv_stamp
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
#define DEV __device__ __forceinline__
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

DEV unsigned long long now() { return __builtin_amdgcn_s_memrealtime(); }
template <int S>
DEV u32x4_t ror4(u32x4_t x) {
  u32x4_t r;
#pragma unroll
  for (int e = 0; e < 4; ++e) r[e] = (unsigned)__builtin_amdgcn_update_dpp(0, (int)x[e], 0x120 + S, 0xF, 0xF, false);
  return r;
}

__global__ void marker(unsigned long long* st) {
  __builtin_amdgcn_s_waitcnt(0);
  if (threadIdx.x == 0) st[0] = now();
}

// stamps per block: [0] start, [1] loads landed (wave 0), [2] MFMA done (wave 0), [3] after LDS barrier, [4] end
template <int WPB, int U>
__global__ __launch_bounds__(WPB * 64) void gv(const bf16_t* __restrict__ W, const bf16_t* __restrict__ A,
                                               float* __restrict__ out, int N, int K, unsigned long long* st) {
  __shared__ float red[WPB][64][4];
  const unsigned long long t0 = now();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lm = lane & 15, lk = lane >> 4;
  const int nt = blockIdx.x, ktiles = K / 32, per = ktiles / WPB, kt0 = w * per;
  const int hsel = lm >> 3, row = lm & 7;
  const bf16_t* arow = A + (size_t)row * K + lk * 8;
  const bf16_t* wp = W + (size_t)nt * ktiles * 512 + lane * 8;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  unsigned long long t1 = 0, t2 = 0;
  for (int c = kt0; c < kt0 + per; c += U) {
    u32x4_t wv[U], av[U / 2];
#pragma unroll
    for (int u = 0; u < U; ++u) wv[u] = *(const u32x4_t*)(wp + (size_t)(c + u) * 512);
#pragma unroll
    for (int q = 0; q < U / 2; ++q) av[q] = *(const u32x4_t*)(arow + (c + 2 * q + hsel) * 32);
    __builtin_amdgcn_s_waitcnt(0);
    if (c == kt0) t1 = now();
#pragma unroll
    for (int q = 0; q < U / 2; ++q) {
      const u32x4_t zero = {0u, 0u, 0u, 0u};
      u32x4_t a0 = hsel ? zero : av[q], a1 = ror4<8>(av[q]);
      a1 = hsel ? zero : a1;
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a0), __builtin_bit_cast(bf16x8_t, wv[2 * q]), acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a1), __builtin_bit_cast(bf16x8_t, wv[2 * q + 1]), acc, 0, 0, 0);
    }
  }
  red[w][lane][0] = acc[0]; red[w][lane][1] = acc[1]; red[w][lane][2] = acc[2]; red[w][lane][3] = acc[3];
  t2 = now();
  __syncthreads();
  const unsigned long long t3 = now();
  if (threadIdx.x >= 64) return;
  float v[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ww = 0; ww < WPB; ++ww) {
    v[0] += red[ww][lane][0]; v[1] += red[ww][lane][1]; v[2] += red[ww][lane][2]; v[3] += red[ww][lane][3];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = lk * 4 + i;
    if (m < 8) out[(size_t)m * N + nt * 16 + lm] = v[i];
  }
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t4 = now();
  if (lane == 0) {
    unsigned long long* s = st + 8 + (size_t)blockIdx.x * 8;
    s[0] = t0; s[1] = t1; s[2] = t2; s[3] = t3; s[4] = t4;
  }
}

__global__ void fill(bf16_t* p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (bf16_t)(0x3c00 + (i * 2654435761u >> 24) % 64);
}

template <int WPB, int U>
void run(const char* name, int N, int K, int nmat) {
  std::vector<bf16_t*> Ws(nmat);
  for (auto& w : Ws) { CK(hipMalloc(&w, (size_t)N * K * 2)); hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, w, (size_t)N * K); }
  bf16_t* A; float* out; unsigned long long* st;
  CK(hipMalloc(&A, 8 * K * 2)); CK(hipMalloc(&out, 8 * N * 4));
  const int nb = N / 16;
  CK(hipMalloc(&st, (8 + (size_t)nb * 8) * 8));
  hipLaunchKernelGGL(fill, dim3(64), dim3(256), 0, 0, A, (size_t)8 * K);
  CK(hipDeviceSynchronize());
  const int reps = 50;
  std::vector<double> gap, spread, load, mfma, barrier, epi, tot;
  std::vector<unsigned long long> h(8 + (size_t)nb * 8);
  for (int r = 0; r < reps; ++r) {
    hipLaunchKernelGGL(marker, dim3(1), dim3(64), 0, 0, st);
    hipLaunchKernelGGL((gv<WPB, U>), dim3(nb), dim3(WPB * 64), 0, 0, Ws[r % nmat], A, out, N, K, st);
    CK(hipDeviceSynchronize());
    if (r < 5) continue;
    CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
    unsigned long long m0 = h[0], s_min = ~0ull, s_max = 0, e_max = 0;
    double l = 0, mf = 0, b = 0, e = 0;
    for (int i = 0; i < nb; ++i) {
      const unsigned long long* s = &h[8 + i * 8];
      s_min = std::min(s_min, s[0]); s_max = std::max(s_max, s[0]); e_max = std::max(e_max, s[4]);
      l += (double)(s[1] - s[0]); mf += (double)(s[2] - s[1]); b += (double)(s[3] - s[2]); e += (double)(s[4] - s[3]);
    }
    gap.push_back((double)(s_min - m0) * 10e-3); spread.push_back((double)(s_max - s_min) * 10e-3);
    load.push_back(l / nb * 10e-3); mfma.push_back(mf / nb * 10e-3); barrier.push_back(b / nb * 10e-3);
    epi.push_back(e / nb * 10e-3); tot.push_back((double)(e_max - m0) * 10e-3);
  }
  auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
  printf("%-26s N=%5d K=%5d blocks=%4d WPB=%2d U=%d %s: boundary %.2f | dispatch spread %.2f | load %.2f | mfma %.2f | "
         "barrier %.2f | epilogue+store %.2f | marker end -> last block end %.2f us\n",
         name, N, K, nb, WPB, U, nmat > 1 ? "cold" : "hot", med(gap), med(spread), med(load), med(mfma), med(barrier),
         med(epi), med(tot));
  fflush(stdout);
  for (auto w : Ws) CK(hipFree(w));
  CK(hipFree(A)); CK(hipFree(out)); CK(hipFree(st));
}

int main() {
  for (int cold = 0; cold < 2; ++cold) {
    const int nmat = cold ? 40 : 1;
    run<8, 4>("cp qkv", 4096, 1024, nmat);
    run<8, 4>("cp gate-up", 6144, 1024, nmat);
    run<4, 4>("cp gate-up", 6144, 1024, nmat);
    run<8, 4>("cp lm_head", 2048, 1024, nmat);
    run<16, 4>("talker qkv", 4096, 2048, nmat);
    run<4, 4>("talker gate-up", 12288, 2048, nmat);
  }
  printf("done\n");
  return 0;
}
