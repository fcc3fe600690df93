// Persistent code-predictor MLP step: gate/up GEMV (+ RMSNorm, SwiGLU) -> down GEMV (+ residual) -> the next
// RMS-normalised GEMV (the next layer's q/k/v projection, or the step's lm_head) in ONE launch of 256 workgroups x
// 512 threads (one per CU), the two all-to-all hand-offs kept inside the launch.
//
// Why: every launch of the code predictor's chain pays a dependent-launch floor (~1.7 us in a graph,
// tools/launch_floor.hip) on top of its ~3 us body; an in-launch hand-off through data-tagged granules costs ~0.8 us
// less per edge than a kernel boundary carrying the same data (tools/bar_probe3.hip: 4.1 vs 4.95 us per phase).
//
// Hand-offs: the SwiGLU output h [M][I] and the new residual shadow x16 [M][H] are published as 8-byte granules
// {2 bf16 values, 32-bit tag} with agent-scope (sc1) stores; a consumer polls each granule it needs until the tag
// equals this launch's edge tag (2 * epoch, 2 * epoch + 1; epoch = *epoch_ctr * epoch_mul + epoch_add, distinct for
// every launch between two clears of the tag buffer), so there is no separate flag and no fence: a granule's value
// and tag land together.  Every poll is bounded: on time-out *err is set and the kernel finishes (never hangs).
// All 256 workgroups must be co-resident (host-checked: >= 256 CUs, one 512-thread workgroup fits per CU).
//
// Work split (M <= 16 rows, bf16 weights in MFMA B-fragment tiles, gate/up interleaved 8 + 8 per tile):
//   phase 1 gate/up: 2I/16 tiles over 256 blocks x 2 four-wave groups, K = H split over a group's 4 waves;
//   phase 2 down:    H/16 tiles x (256 / (H/16)) row groups, K = I split over 8 waves;
//   phase 3 third:   N3/16 tiles x (256 / (N3/16)) row groups, K = H split over 8 waves.
// The MFMA rows are the batch rows (rows >= the block's rows are zero); RMSNorm row sums come from the bf16
// values the MFMA consumes, as in the decode GEMV (csrc/gemm.hip).  Replaces, for the code predictor's decode steps,
// M:1000-1011 (post_attention_layernorm + Qwen3TTSTalkerTextMLP + residual) followed by the next layer's
// input_layernorm + q/k/v projections (M:940-945) or the final norm + lm_head[g] (M:1299).
#include "common.h"
#include <cstdlib>

namespace {

constexpr int NBLK = 256, NTH = 512, NWV = 8;
constexpr unsigned SPIN_MAX = 1u << 18;

QT_DEV unsigned long long ld_tag(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
QT_DEV void st_tag(unsigned long long* p, unsigned v, unsigned tag) {
  __hip_atomic_store(p, ((unsigned long long)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
QT_DEV f32x4_t mfma_bf16(u32x4_t a, u32x4_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}

struct LdsT {
  unsigned a[16 * (1024 + 8) / 2];  // A rows [nr][K + 8] bf16 (16-byte row pad: conflict-free 16-byte row reads);
                                    // 16 rows of K = 1024 or 4 rows of K = 3072
  float red[NWV][64][4];            // per-wave MFMA partials
  float rsp[NWV][16];               // per-wave row sums of squares
  float rss[16];                    // per-row 1 / rms (0 for rows without data)
};

// Stage rows [r0, r0 + nr) of a [*][K] bf16 matrix into lds.a ([nr][K + 8]), from plain memory (row stride ld) or
// from tagged granules ([*][K/2], waited for), and -- K == 2 * NTH -- each row's RMSNorm scale into lds.rss.
// Granule j = tid + NTH * q of the block's nr x K/2: every load of a round is issued before any is checked (a poll
// loop around each load would serialise the round trips); rounds repeat until every tag matches (bounded).
template <int K, int NRMAX, bool TAGGED, bool RMS>
QT_DEV void stage_rows(LdsT& s, const bf16_t* src, long long ld, const unsigned long long* gsrc, int r0, int nr,
                       unsigned tag, float eps, int* err) {
  constexpr int KH = K / 2, KS = (K + 8) / 2, QMAX = NRMAX * KH / NTH;
  static_assert(!RMS || (KH == NTH && NRMAX == 16), "row sums: one granule per thread per row");
  static_assert(NRMAX * KS <= 16 * (1024 + 8) / 2, "staged rows fit lds.a");
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int G = nr * KH;
  unsigned v[QMAX];
  if constexpr (TAGGED) {
    const unsigned long long* base = gsrc + (long long)r0 * KH;
    unsigned spins = 0;
    while (true) {
      unsigned long long g[QMAX];
#pragma unroll
      for (int q = 0; q < QMAX; ++q) g[q] = ld_tag(base + min(tid + NTH * q, max(G - 1, 0)));
      bool ok = true;
#pragma unroll
      for (int q = 0; q < QMAX; ++q) {
        v[q] = (unsigned)g[q];
        ok = ok && (tid + NTH * q >= G || (unsigned)(g[q] >> 32) == tag);
      }
      if (ok) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spins > SPIN_MAX) { atomicOr(err, 1); break; }
    }
  } else {
#pragma unroll
    for (int q = 0; q < QMAX; ++q) {
      const int j = min(tid + NTH * q, max(G - 1, 0));
      v[q] = *(const unsigned*)(src + (long long)(r0 + j / KH) * ld + 2 * (j % KH));
    }
  }
#pragma unroll
  for (int q = 0; q < QMAX; ++q) {
    const int j = tid + NTH * q;
    if (j < G) s.a[(j / KH) * KS + j % KH] = v[q];
  }
  if constexpr (RMS) {  // KH == NTH: granule q of this thread lies in row q
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float lo = __uint_as_float(v[q] << 16), hi = __uint_as_float(v[q] & 0xFFFF0000u);
      const float ss = wave_sum_dpp(lo * lo + hi * hi);
      if (lane == 0) s.rsp[w][q] = ss;
    }
    __syncthreads();
    if (tid < 16) {
      float ss = 0.f;
#pragma unroll
      for (int ww = 0; ww < NWV; ++ww) ss += s.rsp[ww][tid];
      s.rss[tid] = tid < nr ? rsqrtf(ss / (float)K + eps) : 0.f;
    }
  }
}

// One 16-column tile: KPW k tiles per wave from wave index wi.  load_w issues the wave's weight fragments (before the
// hand-off wait, so their latency overlaps it); tile_dot then feeds MFMA row lm from lds.a row lm (rows >= nr are
// zero), lane (lm, lk) holding output column lm, rows lk*4 .. lk*4+3 of the partial product.
template <int K, int KPW>
QT_DEV void load_w(const bf16_t* wt, int wi, u32x4_t (&wv)[KPW]) {
  constexpr int KT = K / 32;
  const int lane = threadIdx.x & 63, kt0 = wi * KPW;
#pragma unroll
  for (int u = 0; u < KPW; ++u) wv[u] = *(const u32x4_t*)(wt + ((long long)min(kt0 + u, KT - 1) * 64 + lane) * 8);
}
template <int K, int KPW>
QT_DEV f32x4_t tile_dot(const LdsT& s, const u32x4_t (&wv)[KPW], int nr, int wi) {
  constexpr int KT = K / 32, KS = (K + 8) / 2;
  const int lane = threadIdx.x & 63, lm = lane & 15, lk = lane >> 4;
  const int kt0 = wi * KPW;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  const u32x4_t zero = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int u = 0; u < KPW; ++u) {
    const int kt = kt0 + u;
    const u32x4_t av = (lm < nr && kt < KT) ? *(const u32x4_t*)(s.a + lm * KS + kt * 16 + lk * 4) : zero;
    acc = mfma_bf16(av, wv[u], acc);
  }
  return acc;
}

__global__ __launch_bounds__(NTH) void cp_mlp_k(qt_cp_mlp_args p, int stop) {
  __shared__ LdsT s;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lm = lane & 15, lk = lane >> 4;
  const int M = p.M, H = p.H, I = p.I;
  const unsigned ep = (unsigned)(*(const volatile int*)p.epoch_ctr) * (unsigned)p.epoch_mul + (unsigned)p.epoch_add;
  const unsigned tag1 = 2u * ep, tag2 = 2u * ep + 1u;
  unsigned long long* htag = (unsigned long long*)p.tags;             // [16][I/2]
  unsigned long long* xtag = htag + (long long)16 * (I / 2);           // [16][H/2]
  const bf16_t* wgu = (const bf16_t*)p.w_gu;
  const bf16_t* wdn = (const bf16_t*)p.w_down;
  const bf16_t* w3 = (const bf16_t*)p.w3;

  // ---- phase 1: h = SwiGLU(rms(x16) * (x16 . W_gu)): tile b (waves 0-3) and tile b + 256 (waves 4-7)
  const int nt1 = 2 * I / 16;
  const int tile1 = b + (w >> 2) * NBLK;
  u32x4_t w1[8];
  load_w<1024, 8>(wgu + (long long)min(tile1, nt1 - 1) * (H / 32) * 512, w & 3, w1);  // 32 k tiles over 4 waves
  stage_rows<1024, 16, false, true>(s, (const bf16_t*)p.x16, p.ldx16, nullptr, 0, M, 0u, p.eps, p.err);
  __syncthreads();
  {
    const int gi = w >> 2, wi = w & 3;
    const int tile = tile1;
    const bool live = tile < nt1;
    f32x4_t acc = tile_dot<1024, 8>(s, w1, M, wi);
#pragma unroll
    for (int i = 0; i < 4; ++i) s.red[w][lane][i] = acc[i];
    __syncthreads();
    if (wi == 0 && live) {
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        v[i] = (s.red[w][lane][i] + s.red[w + 1][lane][i] + s.red[w + 2][lane][i] + s.red[w + 3][lane][i]) *
               s.rss[lk * 4 + i];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float up = __shfl_xor(v[i], 8, 64);
        const float h = silu_f(v[i]) * up;           // lanes lm < 8: output column tile * 8 + lm
        const float h2 = __shfl_xor(h, 1, 64);
        const int m = lk * 4 + i;
        if (lm < 8 && !(lm & 1) && m < M)
          st_tag(htag + (long long)m * (I / 2) + (tile * 8 + lm) / 2, pack2bf(h, h2), tag1);
      }
    }
  }

  if (stop == 1) return;  // measurement hook (QT_CPMLP_STOP): phases 1 .. stop only
  // ---- phase 2: x += h . W_down; x16 = bf16(x), published to phase 3
  {
    const int nt2 = H / 16, rg = NBLK / nt2, mr = (M + rg - 1) / rg;
    const int tile = b % nt2, r0 = (b / nt2) * mr;
    const int nr = max(0, min(mr, M - r0));
    const int kt2 = I / 32;
    // weights and residual operands of this block's outputs, in flight across the hand-off
    u32x4_t w2[12];
    load_w<3072, 12>(wdn + (long long)tile * kt2 * 512, w, w2);  // I = 3072: 96 k tiles over 8 waves
    float xold[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      xold[i] = p.x[(long long)min(r0 + min(lk * 4 + i, max(nr - 1, 0)), M - 1) * p.ldx + tile * 16 + lm];
    __syncthreads();  // lds.a reuse: phase 1's reads are done
    stage_rows<3072, 4, true, false>(s, nullptr, 0, htag, r0, nr, tag1, 0.f, p.err);
    __syncthreads();
    f32x4_t acc = tile_dot<3072, 12>(s, w2, nr, w);
#pragma unroll
    for (int i = 0; i < 4; ++i) s.red[w][lane][i] = acc[i];
    __syncthreads();
    if (w == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = 0.f;
#pragma unroll
        for (int ww = 0; ww < NWV; ++ww) v += s.red[ww][lane][i];
        const int m = lk * 4 + i;
        const float r = xold[i] + v;
        const float r2 = __shfl_xor(r, 1, 64);
        if (m < nr) {
          const int col = tile * 16 + lm;
          p.x[(long long)(r0 + m) * p.ldx + col] = r;
          ((bf16_t*)p.x16)[(long long)(r0 + m) * p.ldx16 + col] = f2bf(r);
          if (!(lm & 1)) st_tag(xtag + (long long)(r0 + m) * (H / 2) + col / 2, pack2bf(r, r2), tag2);
        }
      }
    }
  }

  if (stop == 2) return;
  // ---- phase 3: out3 = rms(x16) * (x16 . W3)
  {
    const int nt3 = p.N3 / 16, rg = NBLK / nt3, mr = (M + rg - 1) / rg;
    const int tile = b % nt3, r0 = (b / nt3) * mr;
    const int nr = max(0, min(mr, M - r0));
    const int kt3 = H / 32;
    u32x4_t w3v[4];
    load_w<1024, 4>(w3 + (long long)tile * kt3 * 512, w, w3v);  // H = 1024: 32 k tiles over 8 waves
    __syncthreads();
    stage_rows<1024, 16, true, true>(s, nullptr, 0, xtag, r0, nr, tag2, p.eps, p.err);
    __syncthreads();
    f32x4_t acc = tile_dot<1024, 4>(s, w3v, nr, w);
#pragma unroll
    for (int i = 0; i < 4; ++i) s.red[w][lane][i] = acc[i];
    __syncthreads();
    if (w == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = 0.f;
#pragma unroll
        for (int ww = 0; ww < NWV; ++ww) v += s.red[ww][lane][i];
        const int m = lk * 4 + i;
        if (m < nr) p.out3[(long long)(r0 + m) * p.ldo3 + tile * 16 + lm] = v * s.rss[m];
      }
    }
  }
}

}  // namespace

extern "C" long long qt_cp_mlp_tags_bytes(int H, int I) { return (long long)16 * (I / 2 + H / 2) * 8; }

extern "C" int qt_cp_mlp_supported(int M, int H, int I, int N3) {
  // the work split above: phase 1 tiles over 2 x 256 four-wave groups with 8 k tiles each (H = 1024), phase 2's
  // 96 k tiles over 8 waves (I = 3072), row groups that cover 256 blocks exactly, <= 16 rows
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    return n;
  }();
  return cus >= NBLK && M >= 1 && M <= 16 && H == 1024 && I == 3072 && 2 * I / 16 <= 2 * NBLK &&
         (N3 == 4096 || N3 == 2048 || N3 == 1024) && (M + NBLK / (N3 / 16) - 1) / (NBLK / (N3 / 16)) <= 16;
}

extern "C" int qt_cp_mlp(const qt_cp_mlp_args* a, void* stream) {
  if (!a || !a->x16 || !a->x || !a->w_gu || !a->w_down || !a->w3 || !a->out3 || !a->tags || !a->epoch_ctr || !a->err)
    return QT_ERR_ARG;
  if (!qt_cp_mlp_supported(a->M, a->H, a->I, a->N3)) return QT_ERR_SHAPE;
  if (a->tags_bytes < qt_cp_mlp_tags_bytes(a->H, a->I)) return QT_ERR_ARG;
  static const int stop = [] { const char* e = getenv("QT_CPMLP_STOP"); return e ? atoi(e) : 0; }();
  hipLaunchKernelGGL(cp_mlp_k, dim3(NBLK), dim3(NTH), 0, (hipStream_t)stream, *a, stop);
  return hipGetLastError() == hipSuccess ? 0 : QT_ERR_LAUNCH;
}
