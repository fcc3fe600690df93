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

}  // namespace

namespace qt_gemm_impl {
void launch_sk_f32(const GemmP& p, hipStream_t s) { launch_sk<float>(p, s); }
void launch_sk_bf16(const GemmP& p, hipStream_t s) { launch_sk<bf16_t>(p, s); }
}  // namespace qt_gemm_impl
