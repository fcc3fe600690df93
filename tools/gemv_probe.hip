// Decode-GEMV probe (talker MLP gate-up shape: N = 12288, K = 2048, M = 8 rows, bf16 tiled weights): how the
// weight stream is issued decides the bandwidth.  Variants (all compute the same RMS-scaled products):
//   reg<U, AT>  : the shipped gemv_wt structure (4 waves / block, one 16-column tile per block, fold 2, U weight
//                 fragments per chunk in VGPRs), A fp32 or bf16
//   glds<WPB, KPW, AT>: every wave issues ALL of its KPW weight fragments at once as LDS-DMA
//                 (global_load_lds_dwordx4, no VGPR destination), then consumes them in order behind counted
//                 vmcnt waits; A in registers, loaded before the weight stream
// Weights cycle through 28 distinct matrices (1.4 GB > the 256 MiB Infinity Cache): every launch streams HBM.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gemv_probe.hip -o tools/gemv_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#include <utility>
#include <cstring>

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
#define DEV __device__ __forceinline__

DEV bf16_t f2bf(float f) {
  unsigned u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (bf16_t)(u >> 16);
}
DEV unsigned pack2bf(float a, float b) { return (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16); }
DEV void load8f(const float* p, float* o) {
  f32x4_t a = *(const f32x4_t*)p, b = *(const f32x4_t*)(p + 4);
  o[0] = a[0]; o[1] = a[1]; o[2] = a[2]; o[3] = a[3]; o[4] = b[0]; o[5] = b[1]; o[6] = b[2]; o[7] = b[3];
}
DEV void load8f(const bf16_t* p, float* o) {
  u32x4_t v = *(const u32x4_t*)p;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = __uint_as_float(v[i] << 16);
    o[2 * i + 1] = __uint_as_float(v[i] & 0xFFFF0000u);
  }
}
template <int S>
DEV u32x4_t ror4(u32x4_t x) {
  u32x4_t r;
#pragma unroll
  for (int e = 0; e < 4; ++e) r[e] = (unsigned)__builtin_amdgcn_update_dpp(0, (int)x[e], 0x120 + S, 0xF, 0xF, false);
  return r;
}
DEV float dpp128(float x) { return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x128, 0xF, 0xF, false)); }

constexpr int M = 8;  // rows
constexpr float EPS = 1e-6f;

// epilogue shared by the variants: block-wide sum of the waves' 16x16 partial tiles + the RMS row sums
template <int WPB>
DEV void finish(float (*red)[64][4], float (*red_ss)[16], f32x4_t acc, float ss, float* out, int N, int K, int nt) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lm = lane & 15, lk = lane >> 4;
  red[w][lane][0] = acc[0]; red[w][lane][1] = acc[1]; red[w][lane][2] = acc[2]; red[w][lane][3] = acc[3];
  ss += dpp128(ss);
  ss += __shfl_xor(ss, 16, 64);
  ss += __shfl_xor(ss, 32, 64);
  if (lk == 0) red_ss[w][lm] = lm >= 8 ? 0.f : ss;
  __syncthreads();
  if (threadIdx.x >= 64) return;
  float v[4] = {0.f, 0.f, 0.f, 0.f}, s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ww = 0; ww < WPB; ++ww) {
    v[0] += red[ww][lane][0]; v[1] += red[ww][lane][1]; v[2] += red[ww][lane][2]; v[3] += red[ww][lane][3];
#pragma unroll
    for (int i = 0; i < 4; ++i) s[i] += red_ss[ww][lk * 4 + i];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = lk * 4 + i;
    if (m < M) out[(size_t)m * N + nt * 16 + lm] = v[i] * rsqrtf(s[i] / (float)K + EPS);
  }
}

// folded MFMA pair: lanes lm < 8 hold k tile 2q, lanes lm >= 8 hold k tile 2q+1 of the same 8 rows
DEV f32x4_t mfma_pair(const float* a, u32x4_t w0, u32x4_t w1, f32x4_t acc, int hsel) {
  const u32x4_t own = {pack2bf(a[0], a[1]), pack2bf(a[2], a[3]), pack2bf(a[4], a[5]), pack2bf(a[6], a[7])};
  const u32x4_t zero = {0u, 0u, 0u, 0u};
  u32x4_t a0 = hsel ? zero : own;
  u32x4_t a1 = ror4<8>(own);
  a1 = hsel ? zero : a1;
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a0), __builtin_bit_cast(bf16x8_t, w0), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a1), __builtin_bit_cast(bf16x8_t, w1), acc, 0, 0, 0);
  return acc;
}

// ---------------------------------------------------------------- reg: the shipped structure
template <int WPB, int U, typename AT, bool NTL>
__global__ __launch_bounds__(WPB * 64) void gv_reg(const bf16_t* __restrict__ W, const AT* __restrict__ A,
                                                   float* __restrict__ out, int N, int K) {
  __shared__ float red[WPB][64][4];
  __shared__ float red_ss[WPB][16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lm = lane & 15, lk = lane >> 4;
  const int nt = blockIdx.x, ktiles = K / 32, per = ktiles / WPB, kt0 = w * per, kt1 = kt0 + per;
  const int hsel = lm >> 3, row = lm & 7;
  const AT* arow = A + (size_t)row * K + lk * 8;
  const bf16_t* wp = W + (size_t)nt * ktiles * 512 + lane * 8;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  float ssv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int c = kt0; c < kt1; c += U) {
    u32x4_t wv[U];
    float a[U / 2][8];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (NTL) wv[u] = __builtin_nontemporal_load((const u32x4_t*)(wp + (size_t)(c + u) * 512));
      else wv[u] = *(const u32x4_t*)(wp + (size_t)(c + u) * 512);
    }
#pragma unroll
    for (int q = 0; q < U / 2; ++q) load8f(arow + (c + 2 * q + hsel) * 32, a[q]);
#pragma unroll
    for (int q = 0; q < U / 2; ++q) {
#pragma unroll
      for (int i = 0; i < 8; ++i) ssv[i] += a[q][i] * a[q][i];
      acc = mfma_pair(a[q], wv[2 * q], wv[2 * q + 1], acc, hsel);
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) ss += ssv[i];
  finish<WPB>(red, red_ss, acc, ss, out, N, K, nt);
}

// ---------------------------------------------------------------- glds: all weight fragments of a wave in flight
// LDS-DMA by inline asm (hipcc cannot then drain it with its own vmcnt(0) waits); M0 saved / restored in the statement
template <int NT_>
DEV void glds16(const void* g, unsigned lds) {
  unsigned keep;
  if constexpr (NT_)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}
template <int N_> DEV void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory"); }
DEV unsigned lds_addr(const void* p) {
  return __builtin_amdgcn_readfirstlane((unsigned)(size_t)(const __attribute__((address_space(3))) void*)p);
}

// folded pair from packed bf16 A (lanes lm >= 8 hold the odd k tile)
DEV f32x4_t mfma_pair_p(u32x4_t own, u32x4_t w0, u32x4_t w1, f32x4_t acc, int hsel) {
  const u32x4_t zero = {0u, 0u, 0u, 0u};
  u32x4_t a0 = hsel ? zero : own;
  u32x4_t a1 = ror4<8>(own);
  a1 = hsel ? zero : a1;
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a0), __builtin_bit_cast(bf16x8_t, w0), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a1), __builtin_bit_cast(bf16x8_t, w1), acc, 0, 0, 0);
  return acc;
}

template <int KPW, int I = 0>
DEV void glds_consume(const u32x4_t* wl, const u32x4_t* ap, f32x4_t& acc, int hsel, int lane) {
  if constexpr (I < KPW) {
    vm_wait<KPW - 2 - I>();  // weight fragments I, I + 1 landed
    const u32x4_t w0 = wl[I * 64 + lane], w1 = wl[(I + 1) * 64 + lane];
    acc = mfma_pair_p(ap[I / 2], w0, w1, acc, hsel);
    glds_consume<KPW, I + 2>(wl, ap, acc, hsel, lane);
  }
}

// AMODE 0: A (bf16) loaded to registers and converted before the weight stream is issued; 1: no A (constant)
template <int WPB, int KPW, int NT_, int AMODE>
__global__ __launch_bounds__(WPB * 64) void gv_glds(const bf16_t* __restrict__ W, const bf16_t* __restrict__ A,
                                                    float* __restrict__ out, int N, int K) {
  __shared__ u32x4_t wl[WPB][KPW * 64];
  __shared__ float red[WPB][64][4];
  __shared__ float red_ss[WPB][16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lm = lane & 15, lk = lane >> 4;
  const int nt = blockIdx.x, ktiles = K / 32, kt0 = w * KPW;
  const int hsel = lm >> 3, row = lm & 7;
  u32x4_t ap[KPW / 2];
  float ss = 0.f;
  if constexpr (AMODE == 0) {
    const bf16_t* arow = A + (size_t)row * K + lk * 8;
#pragma unroll
    for (int q = 0; q < KPW / 2; ++q) ap[q] = *(const u32x4_t*)(arow + (kt0 + 2 * q + hsel) * 32);
#pragma unroll
    for (int q = 0; q < KPW / 2; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float lo = __uint_as_float(ap[q][e] << 16), hi = __uint_as_float(ap[q][e] & 0xFFFF0000u);
        ss += lo * lo + hi * hi;
      }
#pragma unroll
    for (int q = 0; q < KPW / 2; ++q) asm volatile("" ::"v"(ap[q]));  // A resident before the weight stream issues
  } else {
#pragma unroll
    for (int q = 0; q < KPW / 2; ++q) ap[q] = u32x4_t{0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u};
    ss = 1.f;
  }
  const bf16_t* wp = W + ((size_t)nt * ktiles + kt0) * 512 + lane * 8;
  const unsigned lb = lds_addr(&wl[w][0]);
#pragma unroll
  for (int i = 0; i < KPW; ++i) glds16<NT_>(wp + (size_t)i * 512, lb + i * 1024);
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  glds_consume<KPW>(wl[w], ap, acc, hsel, lane);
  finish<WPB>(red, red_ss, acc, ss, out, N, K, nt);
}

// register-streamed ceiling: no A traffic (constant A)
template <int WPB, int U>
__global__ __launch_bounds__(WPB * 64) void gv_reg_noa(const bf16_t* __restrict__ W, const bf16_t* __restrict__ A,
                                                       float* __restrict__ out, int N, int K) {
  __shared__ float red[WPB][64][4];
  __shared__ float red_ss[WPB][16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lm = lane & 15;
  const int nt = blockIdx.x, ktiles = K / 32, per = ktiles / WPB, kt0 = w * per, kt1 = kt0 + per;
  const int hsel = lm >> 3;
  const bf16_t* wp = W + (size_t)nt * ktiles * 512 + lane * 8;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  const u32x4_t own = {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u};
  for (int c = kt0; c < kt1; c += U) {
    u32x4_t wv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) wv[u] = __builtin_nontemporal_load((const u32x4_t*)(wp + (size_t)(c + u) * 512));
#pragma unroll
    for (int q = 0; q < U / 2; ++q) acc = mfma_pair_p(own, wv[2 * q], wv[2 * q + 1], acc, hsel);
  }
  finish<WPB>(red, red_ss, acc, 1.f, out, N, K, nt);
}

// rewrites A like the residual-add epilogue of the preceding decode GEMV does (16 columns per block, every row):
// the next GEMV then reads freshly written activations, as in the frame graph
template <typename AT>
__global__ void rewrite_a(const AT* __restrict__ src, AT* __restrict__ A, int K) {
  const int lane = threadIdx.x & 63, col = blockIdx.x * 16 + (lane & 15);
  for (int m = lane >> 4; m < M; m += 4) A[(size_t)m * K + col] = src[(size_t)m * K + col];
}

// ---------------------------------------------------------------- host
__global__ void fill_bf16(bf16_t* p, size_t n, unsigned seed) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    float v = ((float)(h & 0xFFFF) / 65536.f - 0.5f) * 0.04f;
    p[i] = f2bf(v);
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main() {
  const int N = 12288, K = 2048, NMAT = 28;
  const size_t welems = (size_t)N * K;
  std::vector<bf16_t*> Ws(NMAT);
  for (int i = 0; i < NMAT; ++i) {
    CK(hipMalloc(&Ws[i], welems * 2));
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, Ws[i], welems, 1234u + i);
  }
  float *Af, *out, *ref;
  bf16_t* Ab;
  CK(hipMalloc(&Af, M * K * 4)); CK(hipMalloc(&Ab, M * K * 2));
  CK(hipMalloc(&out, (size_t)M * N * 4)); CK(hipMalloc(&ref, (size_t)M * N * 4));
  std::vector<float> ha(M * K);
  std::vector<bf16_t> hb(M * K);
  for (int i = 0; i < M * K; ++i) {
    float v = sinf(0.37f * i) * 1.5f;
    unsigned u; std::memcpy(&u, &v, 4); u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000u; std::memcpy(&v, &u, 4);  // bf16-exact
    ha[i] = v; hb[i] = (bf16_t)(u >> 16);
  }
  CK(hipMemcpy(Af, ha.data(), M * K * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(Ab, hb.data(), M * K * 2, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  std::vector<float> h_ref((size_t)M * N), h_out((size_t)M * N);

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto bench = [&](const char* name, auto launch, bool is_ref) {
    launch(Ws[0], out);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h_out.data(), out, (size_t)M * N * 4, hipMemcpyDeviceToHost));
    if (is_ref) h_ref = h_out;
    double maxd = 0, maxr = 0;
    for (size_t i = 0; i < h_out.size(); ++i) { maxd = fmax(maxd, fabs(h_out[i] - h_ref[i])); maxr = fmax(maxr, fabs(h_ref[i])); }
    for (int i = 0; i < NMAT; ++i) launch(Ws[i], out);
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r)
      for (int i = 0; i < NMAT; ++i) launch(Ws[i], out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / (reps * NMAT);
    // hot: the same matrix every launch (resident in the Infinity Cache)
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps * NMAT; ++r) launch(Ws[0], out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double hus = ms * 1e3 / (reps * NMAT);
    const double bytes = (double)welems * 2 + M * K * 4 + M * N * 4;
    printf("%-34s cold %7.2f us  %6.0f GB/s  frac %.3f | hot %7.2f us | maxdiff %.2e (max |ref| %.2e)\n", name, us,
           bytes / us / 1e3, bytes / us / 1e3 / 8000.0, hus, maxd, maxr);
    fflush(stdout);
  };
  const int nt = N / 16;
#define REG(WPB, U, AT, NTL, A_) \
  bench("reg<" #WPB "," #U "," #AT "," #NTL ">", [&](const bf16_t* w, float* o) { hipLaunchKernelGGL((gv_reg<WPB, U, AT, NTL>), dim3(nt), dim3(WPB * 64), 0, 0, w, A_, o, N, K); }, false)
#define GLDS(WPB, KPW, NT_, AM) \
  bench("glds<" #WPB "," #KPW ",nt" #NT_ ",amode" #AM ">", [&](const bf16_t* w, float* o) { hipLaunchKernelGGL((gv_glds<WPB, KPW, NT_, AM>), dim3(nt), dim3(WPB * 64), 0, 0, w, Ab, o, N, K); }, false)
#define NOA(WPB, U) \
  bench("reg_noa<" #WPB "," #U ">", [&](const bf16_t* w, float* o) { hipLaunchKernelGGL((gv_reg_noa<WPB, U>), dim3(nt), dim3(WPB * 64), 0, 0, w, Ab, o, N, K); }, false)
  bench("reg<4,4,float,1> (shipped)", [&](const bf16_t* w, float* o) { hipLaunchKernelGGL((gv_reg<4, 4, float, true>), dim3(nt), dim3(256), 0, 0, w, Af, o, N, K); }, true);
  REG(4, 4, float, false, Af);
  REG(4, 4, bf16_t, true, Ab);
  REG(4, 8, bf16_t, true, Ab);
  REG(4, 16, bf16_t, true, Ab);
  REG(8, 8, bf16_t, true, Ab);
  REG(2, 16, bf16_t, true, Ab);
  NOA(4, 4);
  NOA(4, 8);
  NOA(4, 16);
  NOA(8, 8);
  GLDS(4, 16, 1, 0);
  GLDS(4, 16, 0, 0);
  GLDS(8, 8, 1, 0);
  GLDS(2, 32, 1, 0);
  GLDS(4, 16, 1, 1);
  GLDS(8, 8, 1, 1);
  GLDS(2, 32, 1, 1);
  // freshly written A (rewrite kernel before every GEMV): time(rewrite + GEMV) - time(rewrite alone)
  float *Af2; bf16_t* Ab2;
  CK(hipMalloc(&Af2, M * K * 4)); CK(hipMalloc(&Ab2, M * K * 2));
  CK(hipMemcpy(Af2, Af, M * K * 4, hipMemcpyDeviceToDevice)); CK(hipMemcpy(Ab2, Ab, M * K * 2, hipMemcpyDeviceToDevice));
  auto pair = [&](const char* name, auto rw, auto gv) {
    const int reps = 20;
    for (int i = 0; i < NMAT; ++i) { rw(); gv(Ws[i]); }
    CK(hipDeviceSynchronize());
    float ms1, ms2;
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) for (int i = 0; i < NMAT; ++i) rw();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms1, e0, e1));
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) for (int i = 0; i < NMAT; ++i) { rw(); gv(Ws[i]); }
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms2, e0, e1));
    printf("%-34s fresh-A: rewrite %6.2f us, rewrite+gemv %6.2f us -> gemv %6.2f us\n", name, ms1 * 1e3 / (reps * NMAT),
           ms2 * 1e3 / (reps * NMAT), (ms2 - ms1) * 1e3 / (reps * NMAT));
    fflush(stdout);
  };
  pair("reg<4,4,float,1>", [&] { hipLaunchKernelGGL(rewrite_a<float>, dim3(K / 16), dim3(64), 0, 0, Af2, Af, K); },
       [&](const bf16_t* w) { hipLaunchKernelGGL((gv_reg<4, 4, float, true>), dim3(nt), dim3(256), 0, 0, w, Af, out, N, K); });
  pair("reg<4,4,bf16,1>", [&] { hipLaunchKernelGGL(rewrite_a<bf16_t>, dim3(K / 16), dim3(64), 0, 0, Ab2, Ab, K); },
       [&](const bf16_t* w) { hipLaunchKernelGGL((gv_reg<4, 4, bf16_t, true>), dim3(nt), dim3(256), 0, 0, w, Ab, out, N, K); });
  pair("reg_noa<4,4> (A untouched)", [&] { hipLaunchKernelGGL(rewrite_a<bf16_t>, dim3(K / 16), dim3(64), 0, 0, Ab2, Ab, K); },
       [&](const bf16_t* w) { hipLaunchKernelGGL((gv_reg_noa<4, 4>), dim3(nt), dim3(256), 0, 0, w, Ab, out, N, K); });
  pair("glds<4,16,nt1,amode0> bf16", [&] { hipLaunchKernelGGL(rewrite_a<bf16_t>, dim3(K / 16), dim3(64), 0, 0, Ab2, Ab, K); },
       [&](const bf16_t* w) { hipLaunchKernelGGL((gv_glds<4, 16, 1, 0>), dim3(nt), dim3(256), 0, 0, w, Ab, out, N, K); });
  printf("done\n");
  return 0;
}
