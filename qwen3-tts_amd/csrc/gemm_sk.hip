// gemm_sk_k: skinny GEMM for 17..64 rows of a wide output (talker / code-predictor q/k/v prefill of streaming-text
// prompts, single-request refills; qt_gemm's routing rule), bf16 A (row-major) x bf16 pre-tiled W, K % 32 == 0.
// Own translation unit (routed by qt_gemm, gemm.hip).
//
// Block = one 16-column n-tile x ALL rows (MI row fragments of 16); its WPB waves split K.  Every weight fragment
// (1 KiB) is fetched once per launch and multiplied against all MI row fragments, where the decode GEMV's row
// groups (gridDim.z) each re-read it: at M = 80 the row-group GEMV moved 5x the weight bytes through L2 and the
// talker prefill layer took ~130 us.  A (M x K bf16, <= 1 MiB) is re-read from L2 by every block.
//
// Per-row results do not depend on M: a row's sum runs over the same k tiles in the same order (the K partition
// depends on K only), so a request prefilled alone or inside a batch gets the same bits.
#include "gemm_p.h"
#include <cstdlib>

namespace {

using qt_gemm_impl::GemmP;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;

constexpr int SK_WPB = 8;  // waves per block (K split); fixed so the per-row summation order is M-independent

template <typename OT, int MI, int U>
__global__ __launch_bounds__(SK_WPB * 64) void gemm_sk_k(GemmP p) {
  __shared__ f32x4_t red[SK_WPB * MI * 64];  // [WPB][MI][64] partial accumulators
  __shared__ float red_ss[SK_WPB * MI * 16];  // [WPB][MI * 16] partial row sums of squares
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lm = lane & 15, lk = lane >> 4;
  const int nt = blockIdx.x;
  const int ktiles = p.Kp / 32;
  const int per = (ktiles + SK_WPB - 1) / SK_WPB;
  const int kt0 = min(ktiles, w * per), kt1 = min(ktiles, kt0 + per);
  const bool norm = p.rms != 0;
  const bf16_t* A = (const bf16_t*)p.A;
  // this lane's A rows (row lm of each fragment, clamped: rows >= M compute values that are never stored)
  const bf16_t* arow[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) arow[i] = A + (long long)min(i * 16 + lm, p.M - 1) * p.lda + lk * 8;
  const bf16_t* wp = (const bf16_t*)p.W + (size_t)nt * ktiles * 512 + lane * 8;
  f32x4_t acc[MI];
  float ss[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) { acc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f}; ss[i] = 0.f; }
  for (int c = kt0; c < kt1; c += U) {
    u32x4_t wv[U], av[U][MI];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // clamped k tiles (no branch around a load); the extra ones are zeroed below
      const int kc = min(c + u, kt1 - 1);
      wv[u] = __builtin_nontemporal_load((const u32x4_t*)(wp + (size_t)kc * 512));
#pragma unroll
      for (int i = 0; i < MI; ++i) av[u][i] = *(const u32x4_t*)(arow[i] + kc * 32);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = c + u < kt1;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const u32x4_t a = ok ? av[u][i] : u32x4_t{0u, 0u, 0u, 0u};
        if (norm) {  // (a v_dot2 on bit-cast vector elements compiled to the same source dword 4x: fp32 FMAs)
          const float x0 = __uint_as_float(a[0] << 16), x1 = __uint_as_float(a[0] & 0xFFFF0000u);
          const float x2 = __uint_as_float(a[1] << 16), x3 = __uint_as_float(a[1] & 0xFFFF0000u);
          const float x4 = __uint_as_float(a[2] << 16), x5 = __uint_as_float(a[2] & 0xFFFF0000u);
          const float x6 = __uint_as_float(a[3] << 16), x7 = __uint_as_float(a[3] & 0xFFFF0000u);
          ss[i] += ((x0 * x0 + x1 * x1) + (x2 * x2 + x3 * x3)) + ((x4 * x4 + x5 * x5) + (x6 * x6 + x7 * x7));
        }
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                         __builtin_bit_cast(bf16x8_t, wv[u]), acc[i], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < MI; ++i) red[(w * MI + i) * 64 + lane] = acc[i];
  if (norm) {
#pragma unroll
    for (int i = 0; i < MI; ++i) {  // lanes lm, lm+16, lm+32, lm+48 hold the four k chunks of row lm
      float v = ss[i] + xor_lane<16>(ss[i]);
      v += xor_lane<32>(v);
      if (lk == 0) red_ss[w * MI * 16 + i * 16 + lm] = v;
    }
  }
  __syncthreads();
  // epilogue: wave w finishes row fragments i = w, w + WPB, ... (sums in wave order)
  const int n = nt * 16 + lm;
  const bool nval = n < p.N;
  const int nc = min(n, p.N - 1);
  const float bias = (p.bias && nval) ? p.bias[nc] : 0.f;
  const float cs = (p.colscale && nval) ? p.colscale[nc] : 1.f;
  OT* out = (OT*)p.out;
  for (int i = w; i < MI; i += SK_WPB) {
    if (i * 16 >= p.M) break;
    f32x4_t v = red[i * 64 + lane];
#pragma unroll
    for (int ww = 1; ww < SK_WPB; ++ww) v += red[(ww * MI + i) * 64 + lane];
    float x[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float y = v[e];
      if (norm) {
        float s = 0.f;
#pragma unroll
        for (int ww = 0; ww < SK_WPB; ++ww) s += red_ss[ww * MI * 16 + i * 16 + lk * 4 + e];
        y *= rsqrtf(s / (float)p.Klog + p.eps);
      }
      y += bias;
      y = act_f(y, p.act);
      x[e] = y * cs;
    }
    if (p.epi == QT_EPI_SWIGLU) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float up = __shfl_xor(x[e], 8, 64);
        const int m = i * 16 + lk * 4 + e;
        if (lm < 8 && m < p.M && nt * 8 + lm < (p.N >> 1))
          out[(long long)m * p.ldo + nt * 8 + lm] = from_f<OT>(silu_f(x[e]) * up);
      }
      continue;
    }
    float res[4] = {0.f, 0.f, 0.f, 0.f};
    if (p.epi == QT_EPI_ADD) {
#pragma unroll
      for (int e = 0; e < 4; ++e) res[e] = to_f(out[(long long)min(i * 16 + lk * 4 + e, p.M - 1) * p.ldo + nc]);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = i * 16 + lk * 4 + e;
      if (m >= p.M || !nval) continue;
      const float r = res[e] + x[e];
      out[(long long)m * p.ldo + n] = from_f<OT>(r);
      if (p.out2) p.out2[(long long)m * p.ldo2 + n] = f2bf(r);
    }
  }
}

template <typename OT, int MI>
void launch_mi(const GemmP& p, hipStream_t s) {
  constexpr int U = MI <= 8 ? 2 : 1;
  hipLaunchKernelGGL((gemm_sk_k<OT, MI, U>), dim3((p.N + 15) / 16), dim3(SK_WPB * 64), 0, s, p);
}

template <typename OT>
void launch_sk(const GemmP& p, hipStream_t s) {
  switch ((p.M + 15) / 16) {  // qt_gemm routes 17..64 rows here
    case 2: launch_mi<OT, 2>(p, s); break;
    case 3: launch_mi<OT, 3>(p, s); break;
    default: launch_mi<OT, 4>(p, s); break;
  }
}


// gemm_sk2_k: 49..128 rows of a K % 512 == 0, <= 4096-deep weight (the talker prefill's q/k/v and o_proj at
// streaming-text prompt sizes).  gemm_sk_k's one-column-tile blocks each re-read all of A (M x K bf16: 384 KiB at
// 96 rows) -- the per-block intake, not the weights, set its time.  Here a block = 4 column tiles (64 columns, one per
// wave) x one 512-deep K slice (gridDim.y = K / 512 splits): the slice's A rows (<= 128 KiB) go to LDS once by LDS-DMA
// in MFMA fragment order (conflict-free ds_read_b128), the waves stream their weight tiles straight to registers, and
// the splits' partials (with the RMS row sums) meet in the caller's workspace: the last block of a column group to
// arrive sums them in split order (deterministic) and runs the epilogue.  Per-row results do not depend on M.
QT_DEV void sk2_glds16(const void* g, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}

constexpr int SK2_KS = 512;  // K per split
template <typename OT, int MI>
__global__ __launch_bounds__(256) void gemm_sk2_k(GemmP p) {
  constexpr int KTS = SK2_KS / 32;  // k tiles per split
  __shared__ __attribute__((aligned(16))) bf16_t a_img[MI * KTS * 512];  // [MI][KTS] 1 KiB fragments
  __shared__ float ss_sh[MI * 16];
  __shared__ unsigned last_sh;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lm = lane & 15, lk = lane >> 4;
  const int cb = blockIdx.x, z = blockIdx.y, S = gridDim.y;
  const int nt = cb * 4 + w;  // this wave's column tile
  const int ktiles = p.Kp / 32;
  const int k0 = z * SK2_KS;
  const bool norm = p.rms != 0;
  // 1. A slice -> LDS (fragment f = (i, kt): lane j copies row i*16 + (j & 15), k chunk (j >> 4) of k tile kt)
  const unsigned lbase = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(const __attribute__((address_space(3))) void*)a_img);
  const bf16_t* A = (const bf16_t*)p.A;
  for (int f = w; f < MI * KTS; f += 4) {
    const int i = f / KTS, kt = f % KTS;
    const int row = min(i * 16 + lm, p.M - 1);
    sk2_glds16(A + (long long)row * p.lda + k0 + kt * 32 + lk * 8,
               __builtin_amdgcn_readfirstlane(lbase + (unsigned)f * 1024u));  // M0 takes a wave-uniform SGPR
  }
  // 2. this wave's weight tiles of the slice (registers), issued after the DMAs
  const bf16_t* wp = (const bf16_t*)p.W + ((size_t)min(nt, (p.N + 15) / 16 - 1) * ktiles + z * KTS) * 512 + lane * 8;
  u32x4_t wv[KTS];
#pragma unroll
  for (int kt = 0; kt < KTS; ++kt) wv[kt] = __builtin_nontemporal_load((const u32x4_t*)(wp + (size_t)kt * 512));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMAs (and the weight loads) have landed
  __syncthreads();
  // 3. MFMA over the slice; wave 0 also sums the squares of the A rows it reads (RMS)
  f32x4_t acc[MI];
  float ss[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) { acc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f}; ss[i] = 0.f; }
#pragma unroll
  for (int kt = 0; kt < KTS; ++kt) {
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const u32x4_t a = *(const u32x4_t*)(a_img + (i * KTS + kt) * 512 + lane * 8);
      if (norm && w == 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const unsigned u = a[e];
          ss[i] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, u), __builtin_bit_cast(bf16x2_t, u), ss[i],
                                                  false);
        }
      }
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, wv[kt]),
                                                       acc[i], 0, 0, 0);
    }
  }
  if (norm && w == 0) {
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      float v = ss[i] + xor_lane<16>(ss[i]);
      v += xor_lane<32>(v);
      if (lk == 0) ss_sh[i * 16 + lm] = v;
    }
  }
  // 4. split-K: every split stores its record write-through; one arrival per block after the drain; the last block
  // of column group cb sums the records in split order
  constexpr int REC = 4 * MI * 256 + MI * 16;  // floats: [wave][i][lane][4] + row sums
  if (S > 1) {
    __syncthreads();  // ss_sh complete
    float* rec = p.part + ((size_t)cb * S + z) * REC;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        __hip_atomic_store(rec + ((w * MI + i) * 64 + lane) * 4 + e, acc[i][e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (norm && w == 0)
      for (int t = lane; t < MI * 16; t += 64)
        __hip_atomic_store(rec + 4 * MI * 256 + t, ss_sh[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0)
      last_sh = __hip_atomic_fetch_add(p.cnt + cb, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)S - 1;
    __syncthreads();
    if (!last_sh) return;
    if (threadIdx.x == 0) __hip_atomic_store(p.cnt + cb, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    const float* base = p.part + (size_t)cb * S * REC;
#pragma unroll
    for (int i = 0; i < MI; ++i) acc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int zz = 0; zz < S; ++zz) {  // split order
      const float* r = base + (size_t)zz * REC;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc[i][e] += __hip_atomic_load(r + ((w * MI + i) * 64 + lane) * 4 + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (norm) {
      __syncthreads();
      for (int t = threadIdx.x; t < MI * 16; t += 256) {
        float v = 0.f;
        for (int zz = 0; zz < S; ++zz)
          v += __hip_atomic_load(base + (size_t)zz * REC + 4 * MI * 256 + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ss_sh[t] = v;
      }
    }
  }
  __syncthreads();
  // 5. epilogue (as gemm_sk_k's): wave w owns column tile nt, rows i*16 + lk*4 + e
  const int n = nt * 16 + lm;
  const bool nval = n < p.N;
  const int nc = min(n, p.N - 1);
  const float bias = (p.bias && nval) ? p.bias[nc] : 0.f;
  const float cs = (p.colscale && nval) ? p.colscale[nc] : 1.f;
  OT* out = (OT*)p.out;
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    if (i * 16 >= p.M) break;
    float x[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float y = acc[i][e];
      if (norm) y *= rsqrtf(ss_sh[i * 16 + lk * 4 + e] / (float)p.Klog + p.eps);
      y += bias;
      y = act_f(y, p.act);
      x[e] = y * cs;
    }
    if (p.epi == QT_EPI_SWIGLU) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float up = __shfl_xor(x[e], 8, 64);
        const int m = i * 16 + lk * 4 + e;
        if (lm < 8 && m < p.M && nt * 8 + lm < (p.N >> 1))
          out[(long long)m * p.ldo + nt * 8 + lm] = from_f<OT>(silu_f(x[e]) * up);
      }
      continue;
    }
    float res[4] = {0.f, 0.f, 0.f, 0.f};
    if (p.epi == QT_EPI_ADD) {
#pragma unroll
      for (int e = 0; e < 4; ++e) res[e] = to_f(out[(long long)min(i * 16 + lk * 4 + e, p.M - 1) * p.ldo + nc]);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = i * 16 + lk * 4 + e;
      if (m >= p.M || !nval) continue;
      const float r = res[e] + x[e];
      out[(long long)m * p.ldo + n] = from_f<OT>(r);
      if (p.out2) p.out2[(long long)m * p.ldo2 + n] = f2bf(r);
    }
  }
}

template <typename OT>
void launch_sk2(const GemmP& p, hipStream_t s) {
  const dim3 g((p.N + 63) / 64, p.Kp / SK2_KS), b(256);
  switch ((p.M + 15) / 16) {  // qt_gemm routes 49..128 rows here
    case 4: hipLaunchKernelGGL((gemm_sk2_k<OT, 4>), g, b, 0, s, p); break;
    case 5: hipLaunchKernelGGL((gemm_sk2_k<OT, 5>), g, b, 0, s, p); break;
    case 6: hipLaunchKernelGGL((gemm_sk2_k<OT, 6>), g, b, 0, s, p); break;
    case 7: hipLaunchKernelGGL((gemm_sk2_k<OT, 7>), g, b, 0, s, p); break;
    default: hipLaunchKernelGGL((gemm_sk2_k<OT, 8>), g, b, 0, s, p); break;
  }
}

}  // namespace

namespace qt_gemm_impl {
void launch_sk_f32(const GemmP& p, hipStream_t s) { launch_sk<float>(p, s); }
void launch_sk_bf16(const GemmP& p, hipStream_t s) { launch_sk<bf16_t>(p, s); }
void launch_sk2_f32(const GemmP& p, hipStream_t s) { launch_sk2<float>(p, s); }
void launch_sk2_bf16(const GemmP& p, hipStream_t s) { launch_sk2<bf16_t>(p, s); }
long long sk2_part_bytes(int M, int N, int K) {
  const int MI = (M + 15) / 16;
  return (long long)((N + 63) / 64) * (K / SK2_KS) * (4 * MI * 256 + MI * 16) * 4;
}
}  // namespace qt_gemm_impl
