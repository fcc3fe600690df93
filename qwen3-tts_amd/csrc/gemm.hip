// Weight-tiled MFMA GEMM for gfx950: every Linear / Conv1d of the hot path.
//
//   out[m][n] (op)= epi( rs[m] * sum_k W[n][k] * (gamma[k] * A[m][k]) + bias[n] ) * colscale[n]
//
// * Weights are pre-tiled once at load time (qt_tile_weight) into MFMA B-fragment order:
//   tile (nt, kt) = 16 output rows x KT k-columns = 1 KiB, lane l holds W[nt*16 + (l&15)][kt*KT + (l>>4)*E .. +E)
//   (E = 8 bf16 / 4 fp32, KT = 4E).  A wave streaming one n-tile along K reads 1 KiB contiguous per
//   instruction: fully coalesced HBM traffic, no cross-lane reduction (MFMA does the k-sum).
// * A (activations, fp32 or bf16) is read straight from global/L2 in the matching A-fragment order.
//   Optional prologues: RMSNorm (gamma + per-row rsqrt from the same loads), row gather (embedding
//   lookup), implicit im2col for causal / transposed Conv1d on channels-last [batch][time][cin].
// * K is split across the block's waves; partial 16x16 tiles are reduced through LDS, then the fused
//   epilogue (bias, SiLU/GELU, LayerScale, residual add, SwiGLU pairing) writes the output.
// Decode (M <= 16) is HBM-bound on W: roofline = W bytes / 8 TB/s.
#include "gemm_p.h"
#include <algorithm>
#include <type_traits>
#include <cstdlib>

namespace {

using qt_gemm_impl::GemmP;

// SnakeBeta exactly as qt_snake computes it (fp32 math on the stored activation)
QT_DEV float snake1(float v, float al, float ib) {
  const float s = sinf(v * al);
  return v + ib * (s * s);
}

template <typename T> QT_DEV void load_vec(const T* p, float* o, int E);

// Load the E-element A fragment of row m at padded k index kk (fp32 out), zero outside.
template <typename AT, int E>
QT_DEV void load_a(const GemmP& p, int m, int kk, float* v) {
#pragma unroll
  for (int i = 0; i < E; ++i) v[i] = 0.f;
  if (m >= p.M) return;
  const AT* A = (const AT*)p.A;
  const AT* src;
  if (p.taps > 0) {  // implicit im2col, channels-last input [batch][t_in][cin]
    int j = kk / p.cin_pad, c = kk - j * p.cin_pad;
    if (c >= p.cin) return;
    int b = m / p.t_out, t = m - b * p.t_out;
    int ti = t + p.t_off + j * p.dil;
    if (ti < 0 || ti >= p.t_in) return;
    src = A + ((long long)b * p.t_in + ti) * p.lda + c;
  } else {
    if (kk >= p.Klog) return;
    long long row = p.a_index ? (long long)p.a_index[m] : (long long)m;
    src = A + row * p.lda + kk;
  }
  if constexpr (E == 8) load8f(src, v); else load4f(src, v);
  if (p.a_elu) {
#pragma unroll
    for (int i = 0; i < E; ++i) v[i] = elu_f(v[i]);
  }
  if (p.sn_a) {
    const int c0 = p.taps > 0 ? (kk % p.cin_pad) : kk;
#pragma unroll
    for (int i = 0; i < E; ++i) v[i] = snake1(v[i], p.sn_a[c0 + i], p.sn_ib[c0 + i]);
  }
}

template <typename WT, typename AT, typename OT, int MT, int WPB>
__global__ __launch_bounds__(WPB * 64) void gemm_wt(GemmP p) {
  constexpr bool BF = sizeof(WT) == 2;
  constexpr int E = BF ? 8 : 4;
  constexpr int KT = 4 * E;
  __shared__ float red[WPB][MT][64][4];
  __shared__ float red_ss[WPB][MT][16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lm = lane & 15, lk = lane >> 4;
  const int nt = blockIdx.x;
  const int m0 = blockIdx.y * 16 * MT;
  const int ktiles = p.Kp / KT;
  const int per = (ktiles + WPB - 1) / WPB;
  const int kt0 = w * per, kt1 = min(ktiles, kt0 + per);
  const bool norm = p.rms != 0;
  const bool hasg = p.gamma != nullptr;

  f32x4_t acc[MT];
  float ss[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) { acc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f}; ss[i] = 0.f; }

  const WT* wp = (const WT*)p.W + ((size_t)nt * ktiles) * 64 * E + lane * E;
  for (int kt = kt0; kt < kt1; ++kt) {
    u32x4_t wv = *(const u32x4_t*)(wp + (size_t)kt * 64 * E);
    const int kk = kt * KT + lk * E;
    float g[E];
    if (hasg) {
#pragma unroll
      for (int i = 0; i < E; ++i) g[i] = (kk + i < p.Klog) ? p.gamma[kk + i] : 0.f;
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      float a[E];
      load_a<AT, E>(p, m0 + mt * 16 + lm, kk, a);
      if (norm) {
#pragma unroll
        for (int i = 0; i < E; ++i) ss[mt] += a[i] * a[i];
      }
      if (hasg) {
#pragma unroll
        for (int i = 0; i < E; ++i) a[i] *= g[i];
      }
      if constexpr (BF) {
        u32x4_t av = {pack2bf(a[0], a[1]), pack2bf(a[2], a[3]), pack2bf(a[4], a[5]), pack2bf(a[6], a[7])};
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, av),
                                                          __builtin_bit_cast(bf16x8_t, wv), acc[mt], 0, 0, 0);
      } else {
        f32x4_t wf = __builtin_bit_cast(f32x4_t, wv);
#pragma unroll
        for (int s = 0; s < 4; ++s)
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], wf[s], acc[mt], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    red[w][mt][lane][0] = acc[mt][0]; red[w][mt][lane][1] = acc[mt][1];
    red[w][mt][lane][2] = acc[mt][2]; red[w][mt][lane][3] = acc[mt][3];
    if (norm) {
      float s = ss[mt];
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      if (lk == 0) red_ss[w][mt][lm] = s;
    }
  }
  __syncthreads();
  if (threadIdx.x >= MT * 64) return;
  const int mt = threadIdx.x >> 6;  // == w: the epilogue thread block keeps wave boundaries
  float v[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ww = 0; ww < WPB; ++ww) {
    v[0] += red[ww][mt][lane][0]; v[1] += red[ww][mt][lane][1];
    v[2] += red[ww][mt][lane][2]; v[3] += red[ww][mt][lane][3];
  }
  const int n = nt * 16 + lm;
  const bool nval = n < p.N;
  const float bias = (p.bias && nval) ? p.bias[n] : 0.f;
  const float cs = (p.colscale && nval) ? p.colscale[n] : 1.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rloc = lk * 4 + i;
    float x = v[i];
    if (norm) {
      float s = 0.f;
#pragma unroll
      for (int ww = 0; ww < WPB; ++ww) s += red_ss[ww][mt][rloc];
      x *= rsqrtf(s / (float)p.Klog + p.eps);
    }
    x += bias;
    x = act_f(x, p.act);
    x *= cs;
    v[i] = x;
  }
  OT* out = (OT*)p.out;
  if (p.epi == QT_EPI_SWIGLU) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float up = __shfl_xor(v[i], 8, 64);
      const int m = m0 + mt * 16 + lk * 4 + i;
      if (lm < 8 && m < p.M && nt * 8 + lm < (p.N >> 1))
        out[(long long)m * p.ldo + nt * 8 + lm] = from_f<OT>(silu_f(v[i]) * up);
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + mt * 16 + lk * 4 + i;
    if (m >= p.M || !nval) continue;
    OT* o = out + (long long)m * p.ldo + n;
    const float r = p.epi == QT_EPI_ADD ? to_f(*o) + v[i] : v[i];
    *o = from_f<OT>(r);
    if (p.out2) p.out2[(long long)m * p.ldo2 + n] = f2bf(r);
  }
}

// Decode GEMV (M <= 16, plain or gathered rows, K % KT == 0): one wave owns a 16-row n-tile over a K
// slice.  Branch-free inner loop: the lane's A row pointer is hoisted, tail tiles are clamped and zeroed
// by select, so every chunk issues its U weight fragments (1 KiB contiguous per wave-instruction), A
// fragments and gamma before a single wait -- the block keeps all of its weight bytes in flight.
// Split-K partials reduce through LDS; the epilogue is shared with gemm_wt.
// Fold F (bf16 weights, rows per block <= 16 / F): the MFMA rows past the block's rows are zero, so the lanes
// feeding them fetch the block's rows of the next F - 1 k tiles instead of re-fetching a clamped row, and DPP row
// rotations (row_ror 16/F * t) hand those fragments to the live lanes for the t-th MFMA: 1/F of the activation
// requests, the same MFMA operands.  Row groups (gridDim.z): block z owns rows [z * p.mr, z * p.mr + p.mr) -- a
// few-column-tile GEMV gets more blocks without a cross-block split-K reduction (its weight tiles are re-read
// from L2 by the z blocks; blockIdx.x-major launch keeps a tile's row blocks ntiles apart, same XCD when
// ntiles % 8 == 0).
// Loads hipcc does not track (see gemv_wt's epilogue prefetch): the destination is only read after an
// asm_wait that names it "+v", so the compiler never reads it before the data has landed.
QT_DEV unsigned asm_load_b32(const void* ptr) {
  unsigned v;
  asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(ptr) : "memory");
  return v;
}
QT_DEV unsigned asm_load_raw(const float* ptr) { return asm_load_b32(ptr); }
QT_DEV unsigned asm_load_raw(const bf16_t* ptr) {
  unsigned v;
  asm volatile("global_load_ushort %0, %1, off" : "=v"(v) : "v"(ptr) : "memory");
  return v;
}
template <typename T> QT_DEV float raw_to_f(unsigned u);
template <> QT_DEV float raw_to_f<float>(unsigned u) { return __uint_as_float(u); }
template <> QT_DEV float raw_to_f<bf16_t>(unsigned u) { return __uint_as_float(u << 16); }

// DPP row_ror:S on each dword of a 16-byte fragment (rotate right: lane l of a 16-lane row receives lane
// (l - S) mod 16)
template <int S>
QT_DEV u32x4_t ror4(u32x4_t x) {
  u32x4_t r;
#pragma unroll
  for (int e = 0; e < 4; ++e) r[e] = (unsigned)__builtin_amdgcn_update_dpp(0, (int)x[e], 0x120 + S, 0xF, 0xF, false);
  return r;
}

template <typename WT, typename AT, typename OT, int WPB, int U, bool NORM, bool NTL, int F>
__global__ __launch_bounds__(WPB * 64) void gemv_wt(GemmP p) {
  constexpr bool BF = sizeof(WT) == 2;
  constexpr int E = BF ? 8 : 4;
  constexpr int KT = 4 * E;
  constexpr int RPF = 16 / F;  // MFMA rows fed by real rows
  static_assert(F == 1 || (BF && U % F == 0), "fold: bf16 weights, U multiple of F");
  __shared__ float red[WPB][64][4];
  __shared__ float red_ss[WPB][16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lm = lane & 15, lk = lane >> 4;
  const int nt = blockIdx.x, sp = blockIdx.y;
  const int m0 = blockIdx.z * p.mr;           // first row of this row group
  const int mr = min(p.mr, p.M - m0);         // rows of this block
  const int ktiles = p.Kp / KT;
  const int kps = (ktiles + p.ks - 1) / p.ks;  // k tiles of this split
  const int ks0 = sp * kps, ks1 = min(ktiles, ks0 + kps);
  const int per = (kps + WPB - 1) / WPB;
  const int kt0 = ks0 + w * per, kt1 = min(ks1, kt0 + per);
  const int arow_i = lm % RPF;  // the block row this lane fetches
  const int hsel = lm / RPF;    // which k tile of the fold group it fetches
  const bool rowok = arow_i < mr;
  const int mrow = m0 + (rowok ? arow_i : mr - 1);
  // gathered row (a_index): an untracked load waited for here, so no compiler-visible load is pending at the chunk
  // loop's preheader (hipcc flushes those with a vmcnt(0) that would also wait for the epilogue prefetch)
  unsigned grow = (unsigned)mrow;
  if (p.a_index) {
    grow = asm_load_b32(p.a_index + mrow);
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(grow)::"memory");
  }
  const AT* arow = (const AT*)p.A + (long long)(int)grow * p.lda + lk * E;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  float ssv[E];
#pragma unroll
  for (int i = 0; i < E; ++i) ssv[i] = 0.f;
  // epilogue operands of wave 0 issued before the weight stream (hides one dependent round trip).  Inline-asm loads
  // (waited for by asm_wait_epi below): hipcc would otherwise flush them with a vmcnt(0) at the chunk loop's
  // preheader, i.e. wait a full round trip before issuing the first weight fragment.
  const int n = nt * 16 + lm;
  const bool nval = n < p.N;
  const int nc = min(n, p.N - 1);  // clamped column: every lane loads, no per-load branch
  unsigned pre_bias = 0u, pre_cs = 0u, pre_out[4] = {0u, 0u, 0u, 0u};
  const bool pre = w == 0;
  if (pre) {
    if (p.bias) pre_bias = asm_load_b32(p.bias + nc);
    if (p.colscale) pre_cs = asm_load_b32(p.colscale + nc);
    if (p.epi == QT_EPI_ADD) {
      const OT* ob = (const OT*)p.out + nc;
#pragma unroll
      for (int i = 0; i < 4; ++i) pre_out[i] = asm_load_raw(ob + (long long)(m0 + min(lk * 4 + i, mr - 1)) * p.ldo);
    }
  }
  const WT* wp = (const WT*)p.W + ((size_t)nt * ktiles) * 64 * E + lane * E;
  constexpr int NA = U / F;  // A fragments per chunk
  for (int c = kt0; c < kt1; c += U) {
    u32x4_t wv[U];
    float a[NA][E];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kc = min(c + u, kt1 - 1);
      if constexpr (NTL)  // streamed-once weights: non-temporal, so they do not evict re-read data from L2 / MALL
        wv[u] = __builtin_nontemporal_load((const u32x4_t*)(wp + (size_t)kc * 64 * E));
      else
        wv[u] = *(const u32x4_t*)(wp + (size_t)kc * 64 * E);
    }
#pragma unroll
    for (int q = 0; q < NA; ++q) {
      // every lane loads (with F == 1, rows >= M re-fetch row M-1 from L2: predicating the load on the row was
      // measured slower, profiles/r01_gemv_variants_ab.jsonl)
      // (no runtime branch around these loads: hipcc then waits vmcnt(0) after each one, serialising the chunk's
      // round trips -- tools/gemv_probe.hip)
      const int kc = min(c + F * q + hsel, kt1 - 1);
      if constexpr (E == 8) load8f(arow + kc * KT, a[q]); else load4f(arow + kc * KT, a[q]);
    }
#pragma unroll
    for (int q = 0; q < NA; ++q) {
      const bool ok = rowok && (c + F * q + hsel < kt1);
#pragma unroll
      for (int i = 0; i < E; ++i) {
        float x = ok ? a[q][i] : 0.f;
        if constexpr (NORM) ssv[i] += x * x;  // E independent chains (not one 4*U*E-long chain)
        a[q][i] = x;
      }
      if constexpr (F > 1) {
        const u32x4_t own = {pack2bf(a[q][0], a[q][1]), pack2bf(a[q][2], a[q][3]), pack2bf(a[q][4], a[q][5]),
                             pack2bf(a[q][6], a[q][7])};
        const u32x4_t zero = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int t = 0; t < F; ++t) {
          // row_ror:(16 - RPF*t) -- lane r receives lane r + RPF*t: the fold group's t-th k tile
          u32x4_t av = own;
          if constexpr (F >= 2) if (t == 1) av = ror4<16 - RPF>(own);
          if constexpr (F >= 4) if (t == 2) av = ror4<16 - 2 * RPF>(own);
          if constexpr (F >= 4) if (t == 3) av = ror4<16 - 3 * RPF>(own);
          av = hsel ? zero : av;
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, av),
                                                        __builtin_bit_cast(bf16x8_t, wv[F * q + t]), acc, 0, 0, 0);
        }
      } else if constexpr (BF) {
        u32x4_t av = {pack2bf(a[q][0], a[q][1]), pack2bf(a[q][2], a[q][3]), pack2bf(a[q][4], a[q][5]),
                      pack2bf(a[q][6], a[q][7])};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, av),
                                                      __builtin_bit_cast(bf16x8_t, wv[q]), acc, 0, 0, 0);
      } else {
        f32x4_t wf = __builtin_bit_cast(f32x4_t, wv[q]);
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q][s], wf[s], acc, 0, 0, 0);
      }
    }
  }
  red[w][lane][0] = acc[0]; red[w][lane][1] = acc[1]; red[w][lane][2] = acc[2]; red[w][lane][3] = acc[3];
  if (NORM) {
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < E; ++i) ss += ssv[i];
    // + the lanes holding the same row's other k tiles of the fold group
    if constexpr (F == 4) ss += dpp_f<0x124>(ss);
    if constexpr (F >= 2) ss += dpp_f<0x128>(ss);
    ss += __shfl_xor(ss, 16, 64);
    ss += __shfl_xor(ss, 32, 64);
    if (lk == 0) red_ss[w][lm] = lm >= RPF ? 0.f : ss;
  }
  __syncthreads();
  if (threadIdx.x >= 64) return;
  // the epilogue prefetch has landed (it was issued before every weight load the loop waited for)
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(pre_bias), "+v"(pre_cs), "+v"(pre_out[0]), "+v"(pre_out[1]), "+v"(pre_out[2]),
               "+v"(pre_out[3])::"memory");
  float v[4] = {0.f, 0.f, 0.f, 0.f}, ssr[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ww = 0; ww < WPB; ++ww) {
    v[0] += red[ww][lane][0]; v[1] += red[ww][lane][1]; v[2] += red[ww][lane][2]; v[3] += red[ww][lane][3];
  }
  if (NORM) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ww = 0; ww < WPB; ++ww) ssr[i] += red_ss[ww][lk * 4 + i];
  }
  if (p.ks > 1) {
    // deterministic split-K: every split stores its partial, the last to arrive sums them in split order.
    // Agent-scope relaxed atomics (sc1: coherent across the 8 XCD L2s) + an explicit vmcnt drain instead of
    // __threadfence(), whose release half is an XCD-wide L2 writeback (buffer_wbl2) costing ~0.4 us per block.
    constexpr int PS = 64 * 4 + 16;
    float* mine = p.part + ((size_t)nt * p.ks + sp) * PS;
#pragma unroll
    for (int i = 0; i < 4; ++i) __hip_atomic_store(mine + lane * 4 + i, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (NORM && lm == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __hip_atomic_store(mine + 256 + lk * 4 + i, ssr[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __builtin_amdgcn_s_waitcnt(0);  // partial stores acknowledged before the arrival is counted
    unsigned old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(p.cnt + nt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __shfl(old, 0, 64);
    if (old != (unsigned)p.ks - 1) return;
    if (lane == 0) __hip_atomic_store(p.cnt + nt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    const float* base = p.part + (size_t)nt * p.ks * PS;
#pragma unroll
    for (int i = 0; i < 4; ++i) { v[i] = 0.f; ssr[i] = 0.f; }
    // four splits' partials in flight before their adds (a dependent add per split would serialise the round trips)
    for (int s0 = 0; s0 < p.ks; s0 += 4) {
      float pv[4][4], ps[4][4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int sc = min(s0 + s, p.ks - 1);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          pv[s][i] = __hip_atomic_load(base + sc * PS + lane * 4 + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ps[s][i] = NORM ? __hip_atomic_load(base + sc * PS + 256 + lk * 4 + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.f;
        }
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if (s0 + s < p.ks) {
#pragma unroll
          for (int i = 0; i < 4; ++i) { v[i] += pv[s][i]; ssr[i] += ps[s][i]; }
        }
      }
    }
  }
  const float bias = (p.bias && nval) ? __uint_as_float(pre_bias) : 0.f;
  const float cs = (p.colscale && nval) ? __uint_as_float(pre_cs) : 1.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float x = v[i];
    if (NORM) x *= rsqrtf(ssr[i] / (float)p.Klog + p.eps);
    x += bias;
    x = act_f(x, p.act);
    v[i] = x * cs;
  }
  OT* out = (OT*)p.out;
  if (p.epi == QT_EPI_SWIGLU) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float up = __shfl_xor(v[i], 8, 64);
      const int m = lk * 4 + i;
      if (lm < 8 && m < mr && nt * 8 + lm < (p.N >> 1))
        out[(long long)(m0 + m) * p.ldo + nt * 8 + lm] = from_f<OT>(silu_f(v[i]) * up);
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = lk * 4 + i;
    if (m >= mr || !nval) continue;
    OT* o = out + (long long)(m0 + m) * p.ldo + n;
    const float r = p.epi == QT_EPI_ADD ? raw_to_f<OT>(pre_out[i]) + v[i] : v[i];
    *o = from_f<OT>(r);
    if (p.out2) p.out2[(long long)(m0 + m) * p.ldo2 + n] = f2bf(r);
  }
}

// LDS-tiled implicit GEMM for large M with bf16 weights (codec convs / transposed convs as taps, prefill
// linears as taps = 1).  Block = 128 output rows x NT*16 columns (NT = 6 or 8), 4 waves; wave w owns rows
// [32w, 32w+32) x all the block's columns = 2 x NT MFMA 16x16x32 tiles.  A tile's rows are one batch item's consecutive time steps, so the
// input window [t0 + t_off, t0 + t_off + 127 + (taps-1)*dil] x 32 channels is staged into LDS once per channel
// chunk (optional SnakeBeta applied while staging, rounded to bf16 like the MFMA operand) and every tap reads
// its shifted rows from it: the im2col expansion (taps x) never leaves the CU.  The next chunk is loaded into
// registers while the current one is multiplied (double-buffered window, one barrier per chunk).  Weights
// are the pre-tiled MFMA B fragments (1 KiB per 16 x 32 tile), read through L1/L2 one tap ahead.
// Row sums of squares (RMSNorm, taps == 1 only) accumulate from the fp32 A values during staging.
// out-of-line activation for the implicit-GEMM epilogue: inlined, the erf / exp bodies make the epilogue too large
// to unroll and the accumulators then go through scratch memory
__attribute__((noinline)) QT_DEV float act_f_call(float x, int act) { return act_f(x, act); }

constexpr int IG_BM = 128, IG_BN = 64, IG_KC = 32, IG_LDSW = 40;  // LDS row stride 40 bf16 (80 B)
constexpr int IG_GPT = 3;  // staged 8-channel groups per thread (window rows <= 192)
#ifndef IG_PD
#define IG_PD 1  // B-fragment prefetch distance in k tiles (2-4 measured slower: codec 41.0 / 34.1 / 38.2 vs 31.0 ms)
#endif

// G2 = 2 x 2 wave grid: wave (w >> 1, w & 1) owns BM/2 rows x NT/2 column tiles, so each B fragment is fetched by
// 2 waves instead of 4 (the 4 x 1 layout is L1/TA-bound on the shared B fragments: 4 x NT KiB per k tile per block).
template <typename AT, typename OT, int NT, int MI, bool G2>
__global__ __launch_bounds__(256) void igemm_k(GemmP p) {
  constexpr int BM = 64 * MI;  // output rows per block
  constexpr int RT = G2 ? BM / 32 : MI;  // 16-row MFMA tiles per wave
  constexpr int CT = G2 ? NT / 2 : NT;   // 16-column tiles per wave
  static_assert(!G2 || NT % 2 == 0, "2 x 2 wave grid needs an even column tile count");
  extern __shared__ unsigned char ig_smem[];
  bf16_t* win = (bf16_t*)ig_smem;  // [2][WR][IG_LDSW]
  __shared__ float ss_row[BM];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lm = lane & 15, lk = lane >> 4;
  const bool lin = p.taps == 0;
  const int taps = lin ? 1 : p.taps, dil = lin ? 1 : p.dil;
  const int cin = lin ? p.Klog : p.cin, cin_pad = lin ? p.Kp : p.cin_pad;
  const int t_in = lin ? p.M : p.t_in, t_out = lin ? p.M : p.t_out, t_off = lin ? 0 : p.t_off;
  const int WR = BM + (taps - 1) * dil;
  const int tiles_t = (t_out + BM - 1) / BM;
  const int bi = blockIdx.x / tiles_t, t0 = (blockIdx.x - bi * tiles_t) * BM;
  const int ntl = (p.N + 15) / 16, nt0 = blockIdx.y * NT + (G2 ? (w & 1) * CT : 0);
  const int wrow = G2 ? (w >> 1) * (BM / 2) : w * (16 * MI);  // first output row of this wave in the tile
  const int nch = cin_pad / IG_KC, ktiles = p.Kp / IG_KC;
  const AT* A = (const AT*)p.A + (long long)bi * t_in * p.lda;
  const bool norm = p.rms != 0;

  // staging: group q = tid + i*256 -> window row q/4, channels (q%4)*8 .. +8 of the chunk
  float sst[IG_GPT];
  float stg[IG_GPT][8];
#pragma unroll
  for (int i = 0; i < IG_GPT; ++i) sst[i] = 0.f;
  auto load_chunk = [&](int c) {
#pragma unroll
    for (int i = 0; i < IG_GPT; ++i) {
      const int q = tid + i * 256, r = q >> 2, ch = c * IG_KC + (q & 3) * 8;
      const int ti = t0 + t_off + r;
#pragma unroll
      for (int e = 0; e < 8; ++e) stg[i][e] = 0.f;
      if (r < WR && ti >= 0 && ti < t_in && ch < cin) load8f(A + (long long)ti * p.lda + ch, stg[i]);
    }
  };
  auto store_chunk = [&](int buf, int c) {
    bf16_t* wb = win + (size_t)buf * WR * IG_LDSW;
#pragma unroll
    for (int i = 0; i < IG_GPT; ++i) {
      const int q = tid + i * 256, r = q >> 2, ch = c * IG_KC + (q & 3) * 8;
      if (r >= WR) continue;
      float* v = stg[i];
      if (p.a_elu) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = elu_f(v[e]);
      }
      if (p.sn_a && ch < cin) {  // bf16 operand: the hardware sine's error is far below the bf16 rounding
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float sn = __sinf(v[e] * p.sn_a[ch + e]);
          v[e] = v[e] + p.sn_ib[ch + e] * (sn * sn);
        }
      }
      if (norm) {
#pragma unroll
        for (int e = 0; e < 8; ++e) sst[i] += v[e] * v[e];
      }
      *(u32x4_t*)(wb + r * IG_LDSW + (q & 3) * 8) =
          u32x4_t{pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7])};
    }
  };

  f32x4_t acc[RT][CT];
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int j = 0; j < CT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const bf16_t* Wb = (const bf16_t*)p.W + lane * 8;
  auto load_b = [&](u32x4_t* bf, int kt) {
#pragma unroll
    for (int j = 0; j < CT; ++j) {
      const int nt = min(nt0 + j, ntl - 1);
      bf[j] = *(const u32x4_t*)(Wb + ((size_t)nt * ktiles + kt) * 512);
    }
  };

  load_chunk(0);
  store_chunk(0, 0);
  __syncthreads();
  // B fragments PD k tiles ahead (a ring of PD register sets, the step loop unrolled by PD so every set index is a
  // compile-time constant): one tap of MFMA work was too little to cover an L2 round trip.  Steps run over
  // (chunk c, tap j) in chunk-major order; k tile = j * nch + c.
  constexpr int PD = IG_PD;
  const int S = nch * taps;
  u32x4_t bb[PD][CT];
  int pc = 0, pj = 0;  // (chunk, tap) of the next k tile to prefetch
#pragma unroll
  for (int u = 0; u < PD; ++u) {
    if (u < S) load_b(bb[u], pj * nch + pc);
    if (++pj == taps) { pj = 0; ++pc; }
  }
  int c = 0, j = 0;
  for (int s0 = 0; s0 < S; s0 += PD) {
#pragma unroll
    for (int u = 0; u < PD; ++u) {
      if (s0 + u < S) {
        if (j == 0 && c + 1 < nch) load_chunk(c + 1);
        const bf16_t* wb = win + (size_t)(c & 1) * WR * IG_LDSW;
        u32x4_t af[RT];
#pragma unroll
        for (int i = 0; i < RT; ++i) af[i] = *(const u32x4_t*)(wb + (wrow + i * 16 + lm + j * dil) * IG_LDSW + lk * 8);
#pragma unroll
        for (int i = 0; i < RT; ++i)
#pragma unroll
          for (int q = 0; q < CT; ++q)
            acc[i][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[i]),
                                                                __builtin_bit_cast(bf16x8_t, bb[u][q]), acc[i][q], 0, 0, 0);
        if (pc < nch) load_b(bb[u], pj * nch + pc);
        if (++pj == taps) { pj = 0; ++pc; }
        if (j == taps - 1) {
          if (c + 1 < nch) store_chunk((c & 1) ^ 1, c + 1);
          __syncthreads();
        }
        if (++j == taps) { j = 0; ++c; }
      }
    }
  }
  if (norm) {  // rows 0..127 staged by 4 consecutive lanes each (window == tile when taps == 1)
#pragma unroll
    for (int i = 0; i < IG_GPT; ++i) {
      float s = sst[i];
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      const int q = tid + i * 256, r = q >> 2;
      if ((q & 3) == 0 && r < BM) ss_row[r] = s;
    }
    __syncthreads();
  }
  OT* out = (OT*)p.out;
#pragma unroll
  for (int i = 0; i < RT; ++i) {
#pragma unroll
    for (int q = 0; q < CT; ++q) {
      const int nt = nt0 + q;
      if (nt >= ntl) continue;
      const int n = nt * 16 + lm;
      const bool nval = n < p.N;
      const float bias = (p.bias && nval) ? p.bias[n] : 0.f;
      const float cs = (p.colscale && nval) ? p.colscale[n] : 1.f;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rl = wrow + i * 16 + lk * 4 + e;
        float x = acc[i][q][e];
        if (norm) x *= rsqrtf(ss_row[rl] / (float)p.Klog + p.eps);
        x += bias;
        if (p.act != QT_ACT_NONE) x = act_f_call(x, p.act);
        v[e] = x * cs;
      }
      if (p.epi == QT_EPI_SWIGLU) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float up = __shfl_xor(v[e], 8, 64);
          const int t = t0 + wrow + i * 16 + lk * 4 + e;
          if (lm < 8 && t < t_out && nt * 8 + lm < (p.N >> 1))
            out[((long long)bi * t_out + t) * p.ldo + nt * 8 + lm] = from_f<OT>(silu_f(v[e]) * up);
        }
        continue;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int t = t0 + wrow + i * 16 + lk * 4 + e;
        if (t >= t_out || !nval) continue;
        OT* o = out + ((long long)bi * t_out + t) * p.ldo + n;
        if (p.epi == QT_EPI_ADD) *o = from_f<OT>(to_f(*o) + v[e]);
        else *o = from_f<OT>(v[e]);
      }
    }
  }
}

// Prefill linear GEMM (taps == 0, bf16 pre-tiled weights, M >= 128 rows): block tile 128 rows x NTB*16 columns,
// 4 waves in a 2 x 2 grid (wave = 64 rows x NTB/2 column tiles of 16x16x32 MFMAs), K in 64-wide stages.  Both
// operands are staged through LDS and double-buffered: the next stage's global loads (A rows fp32/bf16 -> bf16 with
// the RMS sums of squares taken on the way, B as the pre-tiled 1 KiB fragments, copied verbatim) are in flight
// while the current stage is multiplied, one barrier per stage.  igemm_k streamed B straight from L2 one k tile
// ahead, which left every MFMA group waiting on an L2 round trip (tools/prefill_gemm_bench.py: M=680 gate-up
// 106.8 us = 320 TFLOP/s).  Same operand rounding and per-element k order as igemm_k.
constexpr int PF_BM = 128, PF_BK = 64, PF_AST = PF_BK + 8;  // A LDS row stride (bf16): 144 B

template <typename AT, typename OT, int NTB>
__global__ __launch_bounds__(256) void gemm_pf_k(GemmP p) {
  constexpr int CT = NTB / 2;                 // column tiles per wave
  constexpr int BT = NTB * 2;                 // B fragments (1 KiB) per stage
  constexpr int BPT = BT * 64 / 256;          // 16-byte B loads per thread per stage
  constexpr int AE = sizeof(AT) == 4 ? 8 : 4; // 16-byte A loads per thread per stage (32 elements)
  __shared__ __attribute__((aligned(16))) bf16_t As[2][PF_BM * PF_AST];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[2][BT * 512];
  __shared__ float ss_row[PF_BM];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lm = lane & 15, lk = lane >> 4;
  const int m0 = blockIdx.x * PF_BM, nt0 = blockIdx.y * NTB;
  const int ntl = (p.N + 15) / 16, ktiles = p.Kp / 32, S = (ktiles + 1) / 2;
  const int wr = (w >> 1) * 64, wc = (w & 1) * CT;
  const bool norm = p.rms != 0;
  // A staging: thread -> row ar (0..127), k half ah (32 elements)
  const int ar = tid >> 1, ah = tid & 1;
  const bool arow = m0 + ar < p.M;
  const AT* Ar = (const AT*)p.A + (long long)(arow ? m0 + ar : 0) * p.lda;
  float sst = 0.f;
  u32x4_t ra[AE], rb[BPT];
  auto load_stage = [&](int st, u32x4_t* ra, u32x4_t* rb) {
    const int k0 = st * PF_BK + ah * 32;
#pragma unroll
    for (int i = 0; i < AE; ++i) {
      const int k = k0 + i * (32 / AE);
      ra[i] = (arow && k < p.Klog) ? *(const u32x4_t*)(Ar + k) : u32x4_t{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int q = tid + i * 256, ti = q >> 6;      // fragment ti of the stage: column tile ti >> 1, k tile ti & 1
      const int nt = min(nt0 + (ti >> 1), ntl - 1), kt = st * 2 + (ti & 1);
      const bf16_t* src = (const bf16_t*)p.W + ((size_t)nt * ktiles + min(kt, ktiles - 1)) * 512 + (q & 63) * 8;
      rb[i] = kt < ktiles ? *(const u32x4_t*)src : u32x4_t{0u, 0u, 0u, 0u};
    }
  };
  auto store_stage = [&](int buf, const u32x4_t* ra, const u32x4_t* rb) {
    bf16_t* ad = As[buf] + ar * PF_AST + ah * 32;
    if constexpr (sizeof(AT) == 4) {
#pragma unroll
      for (int i = 0; i < AE; i += 2) {  // two 16-byte fp32 loads -> one 16-byte bf16 store
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) { v[e] = __uint_as_float(ra[i][e]); v[4 + e] = __uint_as_float(ra[i + 1][e]); }
        if (norm) {
#pragma unroll
          for (int e = 0; e < 8; ++e) sst += v[e] * v[e];
        }
        *(u32x4_t*)(ad + i * 4) =
            u32x4_t{pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7])};
      }
    } else {
#pragma unroll
      for (int i = 0; i < AE; ++i) {
        if (norm) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float lo = __uint_as_float(ra[i][e] << 16), hi = __uint_as_float(ra[i][e] & 0xFFFF0000u);
            sst += lo * lo + hi * hi;
          }
        }
        *(u32x4_t*)(ad + i * 8) = ra[i];
      }
    }
    bf16_t* bd = Bs[buf];
#pragma unroll
    for (int i = 0; i < BPT; ++i) *(u32x4_t*)(bd + (size_t)(tid + i * 256) * 8) = rb[i];
  };
  f32x4_t acc[4][CT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < CT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int buf) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      u32x4_t af[4], bf[CT];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *(const u32x4_t*)(As[buf] + (wr + i * 16 + lm) * PF_AST + kk * 32 + lk * 8);
#pragma unroll
      for (int j = 0; j < CT; ++j) bf[j] = *(const u32x4_t*)(Bs[buf] + ((wc + j) * 2 + kk) * 512 + lane * 8);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < CT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[i]),
                                                              __builtin_bit_cast(bf16x8_t, bf[j]), acc[i][j], 0, 0, 0);
    }
  };
  load_stage(0, ra, rb);
  store_stage(0, ra, rb);
  __syncthreads();
  for (int st = 0; st < S; ++st) {
    const int buf = st & 1;
    if (st + 1 < S) load_stage(st + 1, ra, rb);
    compute(buf);
    if (st + 1 < S) store_stage(buf ^ 1, ra, rb);
    __syncthreads();
  }
  if (norm) {
    const float s2 = sst + __shfl_xor(sst, 1, 64);
    if (ah == 0) ss_row[ar] = s2;
    __syncthreads();
  }
  OT* out = (OT*)p.out;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int q = 0; q < CT; ++q) {
      const int nt = nt0 + wc + q;
      if (nt >= ntl) continue;
      const int n = nt * 16 + lm;
      const bool nval = n < p.N;
      const float bias = (p.bias && nval) ? p.bias[n] : 0.f;
      const float cs = (p.colscale && nval) ? p.colscale[n] : 1.f;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rl = wr + i * 16 + lk * 4 + e;
        float x = acc[i][q][e];
        if (norm) x *= rsqrtf(ss_row[rl] / (float)p.Klog + p.eps);
        x += bias;
        if (p.act != QT_ACT_NONE) x = act_f_call(x, p.act);
        v[e] = x * cs;
      }
      if (p.epi == QT_EPI_SWIGLU) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float up = __shfl_xor(v[e], 8, 64);
          const int m = m0 + wr + i * 16 + lk * 4 + e;
          if (lm < 8 && m < p.M && nt * 8 + lm < (p.N >> 1))
            out[(long long)m * p.ldo + nt * 8 + lm] = from_f<OT>(silu_f(v[e]) * up);
        }
        continue;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wr + i * 16 + lk * 4 + e;
        if (m >= p.M || !nval) continue;
        OT* o = out + (long long)m * p.ldo + n;
        const float r = p.epi == QT_EPI_ADD ? to_f(*o) + v[e] : v[e];
        *o = from_f<OT>(r);
        if (p.out2) p.out2[(long long)m * p.ldo2 + n] = f2bf(r);
      }
    }
  }
}


// Single-output-channel causal conv (codec conv_last, Cout = 1): memory-bound, so no MFMA.  A block owns
// 256 consecutive outputs of one batch item; the input window (256 + (taps-1)*dil rows) x 32 channels is staged
// in LDS per channel chunk (SnakeBeta applied on staging) and each thread accumulates its output's taps x cin
// products in fp32.  Weights are read from the row-major [taps][cin_pad] tile row 0 (N = 1 -> tile 0, lane
// group layout: element (k) of tile kt sits at lane (k % 32) / 8 * 16, offset k % 8).
template <typename AT, typename WT, typename OT>
__global__ __launch_bounds__(256) void conv_n1_k(GemmP p) {
  constexpr int KC = 32, WS = KC + 1;
  extern __shared__ float c1_win[];  // [WR][WS]
  const int tid = threadIdx.x;
  const int taps = p.taps, dil = p.dil;
  const int WR = 256 + (taps - 1) * dil;
  const int tiles_t = (p.t_out + 255) / 256;
  const int bi = blockIdx.x / tiles_t, t0 = (blockIdx.x - bi * tiles_t) * 256;
  const AT* A = (const AT*)p.A + (long long)bi * p.t_in * p.lda;
  const WT* W = (const WT*)p.W;
  constexpr int E = sizeof(WT) == 2 ? 8 : 4, KT = 4 * E;
  __shared__ float wsh[2048];  // taps * cin_pad weights of output channel 0 (host checks the size)
  for (int k = tid; k < taps * p.cin_pad; k += 256) {
    const int kt = k / KT, kin = k % KT;
    wsh[k] = to_f(W[(size_t)kt * 64 * E + (kin / E) * 16 * E + (kin % E)]);
  }
  float acc = 0.f;
  // vector staging (8 channels = one 16-byte load per group, every load of a chunk issued before the first use;
  // clamped addresses, no branch around the loads) when the channel layout allows it
  const bool vec = sizeof(AT) == 2 && p.cin % 8 == 0 && p.lda % 8 == 0 && WR * (KC / 8) <= 256 * 8;
  for (int c0 = 0; c0 < p.cin; c0 += KC) {
    __syncthreads();
    if (vec) {
      float v[8][8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int g = tid + i * 256, r = min(g >> 2, WR - 1), ch = min(c0 + (g & 3) * 8, p.cin - 8);
        const int ti = min(max(t0 + p.t_off + r, 0), p.t_in - 1);
        load8f(A + (long long)ti * p.lda + ch, v[i]);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int g = tid + i * 256, r = g >> 2, cl = (g & 3) * 8, c = c0 + cl;
        const int ti = t0 + p.t_off + r;
        if (r >= WR) continue;
        const bool ok = ti >= 0 && ti < p.t_in && c < p.cin;
        float sa[8], sb[8];  // SnakeBeta parameters of the group's 8 channels: two vector loads
        if (p.sn_a) {
          load8f(p.sn_a + min(c, p.cin - 8), sa);
          load8f(p.sn_ib + min(c, p.cin - 8), sb);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float x = 0.f;
          if (ok) {
            x = v[i][e];
            if (p.a_elu) x = elu_f(x);
            if (p.sn_a) x = snake1(x, sa[e], sb[e]);
            if (sizeof(WT) == 2) x = __uint_as_float((unsigned)f2bf(x) << 16);  // bf16 operand, as the MFMA paths
          }
          c1_win[r * WS + cl + e] = x;
        }
      }
    } else {
    for (int q = tid; q < WR * KC; q += 256) {
      const int r = q / KC, c = c0 + q % KC;
      const int ti = t0 + p.t_off + r;
      float v = 0.f;
      if (ti >= 0 && ti < p.t_in && c < p.cin) {
        v = to_f(A[(long long)ti * p.lda + c]);
        if (p.a_elu) v = elu_f(v);
        if (p.sn_a) v = snake1(v, p.sn_a[c], p.sn_ib[c]);
        if (sizeof(WT) == 2) v = __uint_as_float((unsigned)f2bf(v) << 16);  // bf16 operand, as the MFMA paths
      }
      c1_win[r * WS + q % KC] = v;
    }
    }
    __syncthreads();
    for (int j = 0; j < taps; ++j) {
      const float* row = c1_win + (tid + j * dil) * WS;
      const float* wr = wsh + j * p.cin_pad + c0;  // K index of the [1][taps*cin_pad] weight row
      const int nc = min(KC, p.cin - c0);
#pragma unroll 8
      for (int cc = 0; cc < nc; ++cc) acc += wr[cc] * row[cc];
    }
  }
  const int t = t0 + tid;
  if (t < p.t_out) {
    float x = acc + (p.bias ? p.bias[0] : 0.f);
    OT* o = (OT*)p.out + ((long long)bi * p.t_out + t) * p.ldo;
    *o = from_f<OT>(p.epi == QT_EPI_ADD ? to_f(*o) + x : x);
  }
}

template <typename WT, typename AT, typename OT, int WPB, int U, int F>
void launch_gemv_f(const GemmP& p, int nt, hipStream_t s) {
  const dim3 grid(nt, p.ks, (p.M + p.mr - 1) / p.mr), block(WPB * 64);
  if (p.ntl) {
    if (p.rms) hipLaunchKernelGGL((gemv_wt<WT, AT, OT, WPB, U, true, true, F>), grid, block, 0, s, p);
    else hipLaunchKernelGGL((gemv_wt<WT, AT, OT, WPB, U, false, true, F>), grid, block, 0, s, p);
  } else {
    if (p.rms) hipLaunchKernelGGL((gemv_wt<WT, AT, OT, WPB, U, true, false, F>), grid, block, 0, s, p);
    else hipLaunchKernelGGL((gemv_wt<WT, AT, OT, WPB, U, false, false, F>), grid, block, 0, s, p);
  }
}

// fold factor from the rows per block (bf16 weights): 4 for <= 4 rows, 2 for <= 8 (QT_GEMV_FOLD=1 disables)
template <typename WT, typename AT, typename OT, int WPB, int U>
void launch_gemv_u(const GemmP& p, int nt, hipStream_t s) {
  static const int fold_env = qt_knob("QT_GEMV_FOLD", 4);
  if constexpr (sizeof(WT) == 2) {
    if (fold_env >= 4 && p.mr <= 4) return launch_gemv_f<WT, AT, OT, WPB, U, 4>(p, nt, s);
    if (fold_env >= 2 && p.mr <= 8) return launch_gemv_f<WT, AT, OT, WPB, U, 2>(p, nt, s);
  }
  launch_gemv_f<WT, AT, OT, WPB, U, 1>(p, nt, s);
}

// U = k tiles in flight per wave: 8 when a wave owns 5..8 (one round trip instead of two).  Forcing U = 8 on
// every shape, or 16, was measured slower (register pressure; profiles/r01_gemv_variants_ab.jsonl).
// QT_GEMV_U (4 / 8) overrides for A/B measurement.
template <typename WT, typename AT, typename OT, int WPB>
void launch_gemv(const GemmP& p, int nt, int per, hipStream_t s) {
  static const int u_env = qt_knob("QT_GEMV_U", 0);
  const int u = u_env ? u_env : ((per > 4 && per <= 8) ? 8 : 4);
  if (u >= 8) launch_gemv_u<WT, AT, OT, WPB, 8>(p, nt, s);
  else launch_gemv_u<WT, AT, OT, WPB, 4>(p, nt, s);
}

// largest row count run as the decode GEMV over row groups of gemv_mr() rows (QT_GEMV_MAX_M / QT_GEMV_MR override,
// measurement; 16 = decode only)
inline int gemv_max_m() {
  static const int v = qt_knob("QT_GEMV_MAX_M", 256);
  return v;
}
inline int gemv_mr() {
  static const int v = qt_knob("QT_GEMV_MR", 16);
  return std::max(1, std::min(16, v));
}

// largest row count served by the skinny GEMM gemm_sk_k (QT_SK=0 disables it: measurement)
inline int sk_max_m() {
  static const int v = [] {
    if (qt_knob("QT_SK", 1) == 0) return 0;
    return std::min(qt_knob("QT_SK_MAX_M", 48), 64);  // (48 vs 64: bench --workload vd64 451 vs 442 audio-s/s)
  }();
  return v;
}

// largest row count of a conv routed to im2col + the linear GEMMs (QT_IM2COL_MAX_M, measurement)
inline int im2col_max_m() {
  // (first streamed window at B = 8: 256 rows 1.70 ms, 512 1.39, 1024 1.39, 2048 1.40; profiles/r03_codec_first_window_im2col.txt)
  static const int v = qt_knob("QT_IM2COL_MAX_M", 1024);
  return v;
}

// smallest row count routed to the LDS-tiled implicit GEMM (QT_IGEMM_MIN_M overrides, measurement)
inline int igemm_min_m() {
  static const int v = qt_knob("QT_IGEMM_MIN_M", 128);
  return v;
}

// the LDS-staged prefill GEMM (gemm_pf_k) for taps == 0 linears; QT_PF=0 keeps them on igemm_k (measurement)
inline bool pf_on() {
  static const bool v = (qt_knob("QT_PF", 1) != 0);
  return v;
}
// fewest rows served by gemm_pf_k (QT_PF_MIN_M, measurement; default the igemm_k threshold)
inline int pf_min_m() {
  static const int v = qt_knob("QT_PF_MIN_M", 0);
  return v;
}
// widest output served by gemm_pf_k (QT_PF_NMAX, measurement; 0 = any)
inline int pf_nmax() {
  static const int v = qt_knob("QT_PF_NMAX", 0);
  return v;
}

// gemm_pf_k serves bf16-A linears (the bf16 residual shadow, attention / SwiGLU outputs); with fp32 A its 32 KiB
// per-stage A fetch from beyond L2 is not hidden by one stage of prefetch (M=680 gate-up 184 vs 107 us on igemm_k)
template <typename WT, typename AT>
bool pf_route(const GemmP& p) {
  return sizeof(WT) == 2 && sizeof(AT) == 2 && p.taps == 0 && pf_on() && p.a_index == nullptr && p.gamma == nullptr &&
         p.N >= 32 && (pf_nmax() == 0 || p.N <= pf_nmax()) && (p.pf_small || p.M >= std::max(igemm_min_m(), pf_min_m())) && p.mr > 16 && p.Klog % 8 == 0 && p.lda % 8 == 0 && !p.a_elu &&
         p.sn_a == nullptr && !p.no_igemm;
}

// gemm_pf2_k (deep-pipelined LDS-DMA prefill GEMM, gemm_pf2.hip): QT_PF2=0 keeps gemm_pf_k (A/B)
inline int pf2_mode() {
  static const int v = qt_knob("QT_PF2", 1);
  return v;
}


template <typename WT, typename AT, typename OT>
int launch(const GemmP& p, hipStream_t s) {
  const int nt = (p.N + 15) / 16;
  constexpr int KT = sizeof(WT) == 2 ? 32 : 16;
  if constexpr (sizeof(WT) == 2 && sizeof(AT) == 2) {
    if (p.sk) {
      if constexpr (std::is_same<OT, float>::value) qt_gemm_impl::launch_sk_f32(p, s);
      else qt_gemm_impl::launch_sk_bf16(p, s);
      return hipGetLastError() == hipSuccess ? 0 : QT_ERR_LAUNCH;
    }
  }
  if (p.mr <= 16 && p.taps == 0 && p.Klog % KT == 0 && p.gamma == nullptr && !p.a_elu) {
    const int kts = (p.Kp / KT + p.ks - 1) / p.ks;  // k tiles per split
    if (kts >= 48 && p.wpb_max >= 16) launch_gemv<WT, AT, OT, 16>(p, nt, (kts + 15) / 16, s);
    else if (kts >= 16 && p.wpb_max >= 8) launch_gemv<WT, AT, OT, 8>(p, nt, (kts + 7) / 8, s);
    else launch_gemv<WT, AT, OT, 4>(p, nt, (kts + 3) / 4, s);
  } else if (p.N == 1 && p.taps > 0 && p.taps * p.cin_pad <= 2048 && p.act == QT_ACT_NONE &&
             p.epi != QT_EPI_SWIGLU && !p.rms &&
             p.colscale == nullptr && p.a_index == nullptr && p.gamma == nullptr &&
             (size_t)(256 + (p.taps - 1) * p.dil) * 33 * sizeof(float) <= 64 * 1024) {
    const size_t smem = (size_t)(256 + (p.taps - 1) * p.dil) * 33 * sizeof(float);
    const int batches = p.M / p.t_out;
    hipLaunchKernelGGL((conv_n1_k<AT, WT, OT>), dim3(batches * ((p.t_out + 255) / 256)), dim3(256), smem, s, p);
  } else if (p.M <= 16) {
    hipLaunchKernelGGL((gemm_wt<WT, AT, OT, 1, 8>), dim3(nt, 1), dim3(512), 0, s, p);
  } else if (pf_route<WT, AT>(p) && pf2_mode() && p.Klog % 64 == 0 && p.Kp == p.Klog &&
             ((size_t)p.A & 15) == 0) {
    if constexpr (std::is_same<OT, float>::value) qt_gemm_impl::launch_pf2_auto_f32(p, s);
    else qt_gemm_impl::launch_pf2_auto_bf16(p, s);
  } else if (pf_route<WT, AT>(p)) {
    // prefill linears: LDS-staged A and B, 128 x 128 tiles (128 x 64 when that leaves < 256 blocks)
    const int mt = (p.M + PF_BM - 1) / PF_BM;
    const bool narrow = (long long)mt * ((nt + 7) / 8) < 256;
    if (narrow) hipLaunchKernelGGL((gemm_pf_k<AT, OT, 4>), dim3(mt, (nt + 3) / 4), dim3(256), 0, s, p);
    else hipLaunchKernelGGL((gemm_pf_k<AT, OT, 8>), dim3(mt, (nt + 7) / 8), dim3(256), 0, s, p);
  } else if (sizeof(WT) == 2 && p.a_index == nullptr && p.gamma == nullptr && p.N >= 32 &&
             p.M >= (p.taps > 0 ? 16 : igemm_min_m()) &&
             (p.taps == 0 ? p.Klog % 8 == 0 : IG_BM + (p.taps - 1) * p.dil <= 256 * IG_GPT / 4) && !p.no_igemm) {
    const int taps = p.taps == 0 ? 1 : p.taps, dil = p.taps == 0 ? 1 : p.dil;
    const int t_out = p.taps == 0 ? p.M : p.t_out, batches = p.taps == 0 ? 1 : p.M / p.t_out;
    // column tile per block: 6 x 16 for 96 / 192-channel layers (no idle tiles, the snake-staged window is
    // shared by all of a row tile's columns), else 8 x 16; QT_IGEMM_CFG = "NT,MI" overrides (measurement)
    static const int cfg = [] { const char* e = qt_knob_str("QT_IGEMM_CFG"); return e ? atoi(e) * 10 + atoi(e + 2) : 0; }();
    // QT_IGEMM_G2 = 0 selects the 4 x 1 wave layout (measurement); default 2 x 2
    static const int g2 = qt_knob("QT_IGEMM_G2", 1);
    int ntb = (nt % 6 == 0 && nt <= 12) ? 6 : 8, mi = 2;
    // short windows (a streamed codec window, 1-3 frames x batch rows per conv): 64-row tiles and 4 (6) column
    // tiles per block when the default tiling leaves fewer than 256 blocks -- the first streamed window's feed
    // 2.53 -> 2.08 ms at B=8 (tools/codec_feed_prof.py)
    if (!cfg) {
      const int tout = p.taps == 0 ? p.M : p.t_out, nb = p.taps == 0 ? 1 : p.M / p.t_out;
      const long long blocks = (long long)nb * ((tout + 127) / 128) * ((nt + ntb - 1) / ntb);
      if (blocks < 256) { mi = 1; ntb = ntb == 6 ? 6 : 4; }
    }
    if (cfg) { ntb = cfg / 10; mi = cfg % 10; }
    const int bm = 64 * mi;
    const int WR = bm + (taps - 1) * dil;
    const size_t smem = (size_t)2 * WR * IG_LDSW * sizeof(bf16_t);
    dim3 grid(batches * ((t_out + bm - 1) / bm), (nt + ntb - 1) / ntb);
#define IG_GO(N_, M_)                                                                            \
  do {                                                                                           \
    if (g2) hipLaunchKernelGGL((igemm_k<AT, OT, N_, M_, true>), grid, dim3(256), smem, s, p);    \
    else hipLaunchKernelGGL((igemm_k<AT, OT, N_, M_, false>), grid, dim3(256), smem, s, p);      \
  } while (0)
    if (ntb == 6 && mi == 2) IG_GO(6, 2);
    else if (ntb == 6 && mi == 1) IG_GO(6, 1);
    else if (ntb == 4 && mi == 2) IG_GO(4, 2);
    else if (ntb == 4 && mi == 1) IG_GO(4, 1);
    else if (ntb == 8 && mi == 1) IG_GO(8, 1);
    else IG_GO(8, 2);
#undef IG_GO
  } else if (p.M <= 32) {
    hipLaunchKernelGGL((gemm_wt<WT, AT, OT, 2, 8>), dim3(nt, (p.M + 31) / 32), dim3(512), 0, s, p);
  } else {
    hipLaunchKernelGGL((gemm_wt<WT, AT, OT, 4, 4>), dim3(nt, (p.M + 63) / 64), dim3(256), 0, s, p);
  }
  return hipGetLastError() == hipSuccess ? 0 : QT_ERR_LAUNCH;
}

// row-major [N][Kp] -> tiled fragments
template <typename T, int E>
__global__ void tile_weight_k(const T* __restrict__ src, T* __restrict__ dst, int N, int Kp) {
  const long long tile = blockIdx.x;  // nt * ktiles + kt
  const int ktiles = Kp / (4 * E);
  const int nt = tile / ktiles, kt = tile % ktiles;
  const int lane = threadIdx.x;
  const int n = nt * 16 + (lane & 15);
  const int k = kt * 4 * E + (lane >> 4) * E;
  T* d = dst + tile * 64 * E + lane * E;
#pragma unroll
  for (int i = 0; i < E; ++i) d[i] = (n < N) ? src[(long long)n * Kp + k + i] : T(0);
}

}  // namespace

namespace {
// im2col for short conv windows (qt_gemm's small-M conv route below): row m = (item b, output step t), column
// j * cin_pad + c = input channel c at time t + t_off + j * dil of item b (zero outside [0, t_in) and past cin), with
// the ELU / SnakeBeta prologue applied and the value rounded to bf16 exactly as igemm_k stages it.  One thread per
// (row, tap, 8-channel group), 16-byte loads and stores.
template <typename AT>
__global__ __launch_bounds__(256) void im2col_k(GemmP p, bf16_t* __restrict__ out) {
  const int g = p.cin_pad / 8, tg = p.taps * g;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)p.M * tg) return;
  const int m = (int)(idx / tg), r = (int)(idx % tg), j = r / g, ch = (r % g) * 8;
  const int b = m / p.t_out, t = m % p.t_out, ti = t + p.t_off + j * p.dil;
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = 0.f;
  if (ti >= 0 && ti < p.t_in && ch < p.cin) load8f((const AT*)p.A + ((long long)b * p.t_in + ti) * p.lda + ch, v);
  if (p.a_elu) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = elu_f(v[e]);
  }
  if (p.sn_a && ch < p.cin) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float sn = __sinf(v[e] * p.sn_a[ch + e]);
      v[e] = v[e] + p.sn_ib[ch + e] * (sn * sn);
    }
  }
  *(u32x4_t*)(out + (long long)m * p.Kp + j * p.cin_pad + ch) =
      u32x4_t{pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7])};
}

// short conv windows (<= 1024 rows: a streamed codec window's stages; tens of rows, K = taps x cin_pad up to ~7k): igemm_k's
// 128-row tiles leave a few dozen blocks each walking hundreds of k chunks (~110-130 us per conv at B = 8 x 1 frame);
// as im2col + the linear routes (decode GEMV / skinny GEMMs / split-K prefill GEMM) the weights stream over the chip.
// The im2col image lives in the upper half of the caller's workspace.  QT_IM2COL=0 disables (measurement).
constexpr long long IM2COL_WS = 16ll << 20, IM2COL_OFF = 8ll << 20;
inline bool im2col_route(const qt_gemm_args* a) {
  static const int env = qt_knob("QT_IM2COL", 1);
  if (!env || a->taps <= 0 || a->w_dtype != QT_BF16 || a->M <= 0 || a->M > im2col_max_m() || a->rmsnorm ||
      a->gamma != nullptr || a->a_index != nullptr || !a->ws || a->ws_bytes < IM2COL_WS || a->t_out <= 0 ||
      a->cin_pad % 32 || a->cin % 8 || a->splitk == 1)
    return false;
  const long long kp = (long long)a->taps * a->cin_pad;
  return (long long)a->M * kp * 2 <= IM2COL_WS - IM2COL_OFF && a->M % a->t_out == 0;
}
}  // namespace

extern "C" int qt_gemm(const qt_gemm_args* a, void* stream) {
  if (!a || !a->A || !a->W || !a->out) return QT_ERR_ARG;
  if (im2col_route(a)) {
    GemmP q;
    q.M = a->M; q.A = a->A; q.lda = a->lda; q.taps = a->taps; q.dil = a->dil > 0 ? a->dil : 1; q.cin = a->cin;
    q.cin_pad = a->cin_pad; q.t_in = a->t_in; q.t_out = a->t_out; q.t_off = a->t_off; q.Kp = a->taps * a->cin_pad;
    q.a_elu = a->a_act == QT_AACT_ELU; q.sn_a = a->snake_alpha; q.sn_ib = a->snake_inv_beta;
    bf16_t* img = (bf16_t*)((char*)a->ws + IM2COL_OFF);
    const long long n = (long long)a->M * a->taps * (a->cin_pad / 8);
    hipStream_t s = (hipStream_t)stream;
    if (a->a_dtype == QT_BF16) hipLaunchKernelGGL(im2col_k<bf16_t>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, q, img);
    else if (a->a_dtype == QT_F32) hipLaunchKernelGGL(im2col_k<float>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, q, img);
    else return QT_ERR_DTYPE;
    if (hipGetLastError() != hipSuccess) return QT_ERR_LAUNCH;
    qt_gemm_args b = *a;
    b.taps = 0; b.A = img; b.a_dtype = QT_BF16; b.lda = q.Kp; b.K = (int)q.Kp; b.a_act = QT_AACT_NONE;
    b.snake_alpha = nullptr; b.snake_inv_beta = nullptr; b.ws_bytes = IM2COL_OFF;  // split records below the image
    return qt_gemm(&b, stream);
  }
  const int E = a->w_dtype == QT_BF16 ? 8 : 4;
  const int KT = 4 * E;
  GemmP p;
  p.M = a->M; p.N = a->N;
  p.taps = a->taps; p.dil = a->dil > 0 ? a->dil : 1; p.cin = a->cin; p.cin_pad = a->cin_pad;
  p.t_in = a->t_in; p.t_out = a->t_out; p.t_off = a->t_off;
  if (a->taps > 0) {
    if (a->cin_pad % KT || a->cin % E || a->t_out <= 0) return QT_ERR_SHAPE;
    p.Kp = a->taps * a->cin_pad;
  } else {
    p.Kp = (a->K + KT - 1) / KT * KT;
    if (a->K % E) return QT_ERR_SHAPE;
  }
  p.Klog = a->K;
  if (a->M <= 0 || a->N <= 0 || (a->epi == QT_EPI_SWIGLU && a->N % 16)) return QT_ERR_SHAPE;
  if (a->epi == QT_EPI_SWIGLU && (a->bias || a->colscale)) return QT_ERR_ARG;
  p.A = a->A; p.lda = a->lda; p.a_index = a->a_index; p.W = a->W;
  p.gamma = a->gamma; p.eps = a->eps; p.rms = a->rmsnorm || a->gamma != nullptr; p.bias = a->bias; p.colscale = a->colscale;
  p.act = a->act; p.epi = a->epi; p.out = a->out; p.ldo = a->ldo;
  p.out2 = (bf16_t*)a->out2; p.ldo2 = a->ldo2;
  if (p.out2 && (a->taps > 0 || a->epi == QT_EPI_SWIGLU || a->o_dtype != QT_F32)) return QT_ERR_ARG;
  p.sn_a = a->snake_alpha; p.sn_ib = a->snake_inv_beta;
  if ((p.sn_a == nullptr) != (p.sn_ib == nullptr)) return QT_ERR_ARG;
  if (a->a_act != QT_AACT_NONE && a->a_act != QT_AACT_ELU) return QT_ERR_ARG;
  if (a->act < QT_ACT_NONE || a->act > QT_ACT_RELU_TANH) return QT_ERR_ARG;
  p.a_elu = a->a_act == QT_AACT_ELU;
  static const int no_ig = qt_knob("QT_NO_IGEMM", 0);
  p.no_igemm = no_ig;
  // weights streamed once per frame (talker-size matrices) bypass cache retention so the re-read code-predictor
  // weights stay in L2 / Infinity Cache; QT_GEMV_NT=0/1 forces it off/on for every decode GEMV (measurement)
  static const int nt_env = qt_knob("QT_GEMV_NT", -1);
  const long long wbytes = (long long)((a->N + 15) / 16) * 16 * p.Kp * (a->w_dtype == QT_BF16 ? 2 : 4);
  p.ntl = nt_env >= 0 ? nt_env : (wbytes >= (16ll << 20));
  // split-K for the decode GEMV when it has too few column tiles to fill 256 CUs twice
  p.ks = 1; p.cnt = nullptr; p.part = nullptr; p.part_bytes = 0;
  if (a->M > 16 && a->ws && a->ws_bytes >= QT_GEMM_WS_MIN && a->splitk != 1) {
    // gemm_pf2_k split-K records (narrow outputs with few tiles, gemm_pf2.hip pf2_splits)
    p.cnt = (unsigned*)a->ws;
    p.part = (float*)((char*)a->ws + 4096 * sizeof(unsigned));
    p.part_bytes = a->ws_bytes - 4096 * (long long)sizeof(unsigned);
  }
  // wide grids use smaller blocks so several fit per CU (fewer block rounds; measured: N=12288 K=2048
  // 14.7 us at 16 waves/block -> 12.0 at 4); QT_GEMV_WPB overrides the cap for A/B measurement
  static const int wpb_env = qt_knob("QT_GEMV_WPB", 0);
  const int ntc = (a->N + 15) / 16;
  p.wpb_max = wpb_env > 0 ? wpb_env : (ntc > 512 ? 4 : (ntc > 256 ? 8 : 16));
  const int ntl = (a->N + 15) / 16, ktl = p.Kp / KT;
  if (a->M <= 16 && a->taps == 0 && a->K % KT == 0 && a->gamma == nullptr && a->ws && a->ws_bytes >= QT_GEMM_WS_MIN &&
      a->splitk != 1 && ntl <= 4096) {
    // auto: split only deep-K shapes on < 256 column tiles (the arrival / partial round trips pay only when they
    // remove weight round trips).  Measured cold, paired-A GEMV, partial loads of four splits in flight:
    // 2048x6144 11.4 (no split) / 10.9 (2) / 10.3 us (4), 1024x3072 8.5 / 7.6 / 7.1 us; other shapes lose.
    // In the frame graph split 2 wins (bench 158.6 vs 157.2 audio-s/s, same box): QT_GEMV_SPLIT_AUTO overrides
    const int wpb1 = ktl >= 48 ? 16 : (ktl >= 16 ? 8 : 4), per1 = (ktl + wpb1 - 1) / wpb1;
    static const int ks_auto = qt_knob("QT_GEMV_SPLIT_AUTO", 2);
    int ks = a->splitk > 1 ? a->splitk : ((per1 > 4 && ntl < 256) ? ks_auto : 1);
    ks = std::max(1, std::min({ks, 16, ktl / 2}));
    const size_t need = 4096 * sizeof(unsigned) + (size_t)ntl * ks * (64 * 4 + 16) * sizeof(float);
    if (ks > 1 && need <= (size_t)a->ws_bytes) {
      p.ks = ks;
      p.cnt = (unsigned*)a->ws;
      p.part = (float*)((char*)a->ws + 4096 * sizeof(unsigned));
    }
  }
  // decode GEMV row groups (bf16 weights): rows split over gridDim.z blocks instead of K over gridDim.y for
  // shapes with <= 128 column tiles (measured cold, M = 8, two groups of 4 rows with fold 4: talker o 6.0 -> 5.3,
  // talker down 10.9 (split-K 2) -> 9.4, CP down 7.6 -> 6.5, CP lm_head 4.9 -> 4.5 us; wider shapes lose:
  // talker qkv 6.7 -> 9.6).  QT_GEMV_RG = n forces n groups, 1 = off, 0 = auto.
  p.mr = std::max(1, a->M);
  // 17..256 rows of bf16 A x bf16 weights (prefills of streaming-text / voice-clone prompts, single-request refills):
  // three kernels, picked by the per-launch times of tools/prefill_gemm_bench.py at 1.7B / 0.6B dims
  // (profiles/r03_skinny_routes.txt).  The row-group GEMV grows linearly in M (each group re-reads the weights), the
  // tiled gemm_pf2_k is flat in M but has few blocks on narrow outputs, gemm_sk_k (every row in one block per column
  // tile) reads the weights once but every block re-reads A:
  //   outputs >= 4096 columns: gemm_sk_k at <= 48 rows of a <= 8 Mi-element weight (1.7B qkv 24 rows 11.5 -> 7.6 us,
  //     48 rows 16.5 -> 10.7), else gemm_pf2_k (gate-up 80 rows 51.4 -> 16.2, 112 rows 87.6 -> 16.9; qkv 112 rows
  //     35.1 -> 16.0);
  //   narrower outputs: the row-group GEMV while M x N x K <= 400 Mi (1.7B o up to 100 rows: 80 rows 12.2 vs 13.0 us
  //     on gemm_pf2_k; 1.7B down up to 33 rows: 24 rows 11.5 vs 16.9), else gemm_pf2_k with its narrow-output
  //     split-K (1.7B down 80 rows 29.0 -> 16.9, 112 rows 37.7 -> 17.7; o 112 rows 15.5 -> 13.8, 200 rows 24.3 -> 13.5;
  //     profiles/r03_skinny_routes.txt).
  // QT_SKINNY=0 restores the round-2 rule (row-group GEMV up to 96 rows / 256 rows of <= 2048 columns).
  p.sk = 0;
  p.pf_small = 0;
  static const int skinny_env = qt_knob("QT_SKINNY", 1);
  const bool skinny = skinny_env != 0 && a->M > 16 && a->M <= 256 && a->taps == 0 && a->w_dtype == QT_BF16 &&
                      a->a_dtype == QT_BF16 && a->K % 64 == 0 && a->a_index == nullptr && a->gamma == nullptr &&
                      a->a_act == QT_AACT_NONE && a->snake_alpha == nullptr && a->lda % 8 == 0 &&
                      ((size_t)a->A & 15) == 0 && a->N >= 32;
  bool skinny_gemv = false;
  if (skinny) {
    if (a->N >= 4096) {
      if (a->M <= sk_max_m() && (long long)a->N * a->K <= (8ll << 20)) p.sk = 1;
      else p.pf_small = 1;
    } else if ((long long)a->M * a->N * a->K <= (400ll << 20)) {
      skinny_gemv = true;
    } else {
      p.pf_small = 1;
    }
  }
  static const int rg_env = qt_knob("QT_GEMV_RG", 0);
  if (a->M <= 16 && a->taps == 0 && a->w_dtype == QT_BF16 && a->K % KT == 0 && a->gamma == nullptr) {
    // four groups of 2 rows for <= 64 tiles (CP down 6.5 -> 5.8 us; 128-tile shapes lose with four)
    const int rg = rg_env > 0 ? rg_env : (a->M > 4 ? (ntl <= 64 ? 4 : (ntl <= 128 ? 2 : 1)) : 1);
    if (rg > 1) {
      p.mr = (a->M + rg - 1) / rg;
      p.ks = 1;
      // deep-K row-group shapes (the down projections) prefer 8 waves per block: talker down 9.4 -> 8.6,
      // CP down 5.8 -> 5.6 us (o_proj / lm_head keep 16)
      if (wpb_env <= 0 && ktl >= 96) p.wpb_max = 8;
    }
  } else if (skinny ? skinny_gemv
                     : (a->M <= gemv_max_m() && (a->M <= 96 || a->N <= 2048) && a->taps == 0 && a->w_dtype == QT_BF16 &&
                        a->K % KT == 0 && a->gamma == nullptr && a->a_act == QT_AACT_NONE &&
                        a->snake_alpha == nullptr)) {
    // skinny GEMM (17..96 rows, or up to gemv_max_m rows of a <= 2048-column output: the talker prefill of
    // streaming-text prompts, short codec windows): the decode GEMV over row groups of 16 -- one block per (column
    // tile, row group), the weight tile streamed from HBM once and re-read from L2 by the other row groups of its
    // XCD.  Its time grows with the row groups; the tiled GEMMs' is flat in M but their grids are small for narrow
    // outputs (tools/prefill_gemm_bench.py: M=80 o 29.6 -> 12.2 us, down 93.7 -> 29.0, qkv 36.0 -> 30.0, gate-up
    // 79.0 -> 65.4; at M=160 gate-up 86 (igemm) vs 130, down 233 vs 48)
    p.mr = gemv_mr();
    p.ks = 1;
    if (wpb_env <= 0 && ktl >= 96) p.wpb_max = 8;
  }
  const int w = a->w_dtype, o = a->o_dtype;
  // out2 is written by the decode GEMV's epilogue (M <= 16, or the skinny row-group path above) and by gemm_pf_k
  // (bf16-A prefill linears)
  const bool pf = w == QT_BF16 && a->a_dtype == QT_BF16 && pf_route<bf16_t, bf16_t>(p);
  if (p.out2 && !pf && !p.sk && (p.mr > 16 || a->K % KT != 0 || a->gamma != nullptr || a->a_act != QT_AACT_NONE))
    return QT_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int ad = a->a_dtype;
  if (w == QT_BF16 && ad == QT_F32 && o == QT_F32) return launch<bf16_t, float, float>(p, s);
  if (w == QT_BF16 && ad == QT_BF16 && o == QT_BF16) return launch<bf16_t, bf16_t, bf16_t>(p, s);
  if (w == QT_BF16 && ad == QT_BF16 && o == QT_F32) return launch<bf16_t, bf16_t, float>(p, s);
  if (w == QT_BF16 && ad == QT_F32 && o == QT_BF16) return launch<bf16_t, float, bf16_t>(p, s);
  if (w == QT_F32 && ad == QT_F32 && o == QT_F32) return launch<float, float, float>(p, s);
  return QT_ERR_DTYPE;
}

extern "C" int qt_tile_weight(const void* src, int dtype, int N, int Kp, void* dst, void* stream) {
  const int E = dtype == QT_BF16 ? 8 : 4;
  if (N <= 0 || Kp % (4 * E)) return QT_ERR_SHAPE;
  const int ntiles = (N + 15) / 16, ktiles = Kp / (4 * E);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == QT_BF16)
    hipLaunchKernelGGL((tile_weight_k<bf16_t, 8>), dim3(ntiles * ktiles), dim3(64), 0, s, (const bf16_t*)src,
                       (bf16_t*)dst, N, Kp);
  else if (dtype == QT_F32)
    hipLaunchKernelGGL((tile_weight_k<float, 4>), dim3(ntiles * ktiles), dim3(64), 0, s, (const float*)src,
                       (float*)dst, N, Kp);
  else
    return QT_ERR_DTYPE;
  return hipGetLastError() == hipSuccess ? 0 : QT_ERR_LAUNCH;
}
