// Fused decode MLP with residual (Qwen3 MLP, M:655-668; talker T7-T8, code predictor P2):
//   x[m] += W_down . ( silu(W_gate . n(x[m])) * (W_up . n(x[m])) ),   n = RMSNorm (gamma folded into W_gate/up)
// for M <= 16 decode rows in ONE launch instead of two dependent GEMVs.
//
// Block b owns intermediate columns [32b, 32b+32) = gate/up tiles 4b..4b+3 (8 gate + 8 up rows each) = down
// k-tile b.  16 waves: wave w = (gate/up tile w&3, k quarter w>>2); the 4 quarters reduce through LDS, the
// RMS scale and SwiGLU are applied, the 16 x 32 bf16 slice of h goes to LDS and is multiplied by the
// block's down k-tile for all H outputs -> a partial [M][H] written with agent-scope stores (coherent across
// the 8 XCD L2s).  Each block then takes an arrival ticket; the last H/16 arrivals each own one 16-column
// output tile: they wait (bounded spin) until every block has arrived, sum the partials of all blocks in
// block order (fixed order -> bit-reproducible), add the residual and store.  The final reducer re-arms the
// counters.  Only late blocks ever wait, and every block of the grid is resident (grid <= 256 blocks of one
// per CU), so the wait cannot deadlock; a timeout still exits and raises *err.
#include "common.h"

namespace {

constexpr int MLP_WS_HEAD = 256;  // bytes: arrive counter @0, done counter @64

template <int H, int U>
__global__ __launch_bounds__(1024) void mlp_decode_k(qt_mlp_args p) {
  constexpr int KT = H / 32;     // gate/up k tiles
  constexpr int KTW = KT / 4;    // per wave (k quarter)
  constexpr int NTD = H / 16;    // down n tiles = reducer blocks
  constexpr int NTW = NTD / 16;  // down n tiles per wave
  static_assert(KTW % U == 0, "k quarter must be a multiple of U");
  __shared__ float red[16][64][4];
  __shared__ float red_ss[4][16];
  __shared__ bf16_t hbuf[16][40];
  __shared__ float rsum[8][16][16];
  __shared__ unsigned ticket_sh;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lm = lane & 15, lk = lane >> 4;
  const int b = blockIdx.x, nblk = gridDim.x;
  const int M = p.M;
  const int ti = w & 3, kq = w >> 2;
  unsigned* arrive = (unsigned*)p.ws;
  unsigned* done = (unsigned*)((char*)p.ws + 64);
  float* part = (float*)((char*)p.ws + MLP_WS_HEAD);

  // down-proj B fragments of this block's k tile: independent of everything, issued first when they fit
  // in registers beside the gate/up stream (H = 1024), else right after the gate/up MFMAs (H = 2048)
  constexpr bool EARLY_BD = NTW <= 4;
  const int KTD = p.I / 32;
  const bf16_t* Wd = (const bf16_t*)p.w_down + lane * 8;
  u32x4_t bd[NTW];
  auto load_bd = [&] {
#pragma unroll
    for (int j = 0; j < NTW; ++j) bd[j] = *(const u32x4_t*)(Wd + ((size_t)(w * NTW + j) * KTD + b) * 512);
  };
  if constexpr (EARLY_BD) load_bd();

  // gate/up: this wave's k quarter of tile 4b + ti
  const bf16_t* Wg = (const bf16_t*)p.w_gu + lane * 8 + (size_t)(4 * b + ti) * KT * 512;
  const bool rowok = lm < M;
  const float* arow = p.x + (long long)(rowok ? lm : M - 1) * p.ldx + lk * 8;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  float ssv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) ssv[i] = 0.f;
#pragma unroll 1
  for (int c = 0; c < KTW; c += U) {
    u32x4_t wv[U];
    float a[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kt = kq * KTW + c + u;
      wv[u] = *(const u32x4_t*)(Wg + (size_t)kt * 512);
      load8f(arow + kt * 32, a[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float v = rowok ? a[u][i] : 0.f;
        ssv[i] += v * v;
        a[u][i] = v;
      }
      const u32x4_t av = {pack2bf(a[u][0], a[u][1]), pack2bf(a[u][2], a[u][3]), pack2bf(a[u][4], a[u][5]),
                          pack2bf(a[u][6], a[u][7])};
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, av),
                                                    __builtin_bit_cast(bf16x8_t, wv[u]), acc, 0, 0, 0);
    }
  }
  if constexpr (!EARLY_BD) load_bd();
  *(f32x4_t*)red[w][lane] = acc;
  if (ti == 0) {
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) ss += ssv[i];
    ss += __shfl_xor(ss, 16, 64);
    ss += __shfl_xor(ss, 32, 64);
    if (lk == 0) red_ss[kq][lm] = ss;
  }
  __syncthreads();
  if (w < 4) {  // wave w finishes gate/up tile w: k quarters in order, RMS scale, SwiGLU -> hbuf (bf16)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = lk * 4 + e;
      float v = red[w][lane][e] + red[w + 4][lane][e] + red[w + 8][lane][e] + red[w + 12][lane][e];
      const float ss = red_ss[0][row] + red_ss[1][row] + red_ss[2][row] + red_ss[3][row];
      v *= rsqrtf(ss / (float)H + p.eps);
      const float up = __shfl_xor(v, 8, 64);
      if (lm < 8) hbuf[row][w * 8 + lm] = f2bf(silu_f(v) * up);
    }
  }
  __syncthreads();
  // down partial for all H outputs: A = hbuf [16 rows][32 k], B = this block's k tile
  const u32x4_t af = *(const u32x4_t*)&hbuf[lm][lk * 8];
  float* mine = part + (size_t)b * M * H;
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const f32x4_t d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af),
                                                              __builtin_bit_cast(bf16x8_t, bd[j]),
                                                              f32x4_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    const int n = (w * NTW + j) * 16 + lm;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = lk * 4 + e;
      if (m < M) __hip_atomic_store(mine + (size_t)m * H + n, d[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __builtin_amdgcn_s_waitcnt(0);  // partial stores acknowledged before the arrival is counted
  __syncthreads();
  if (tid == 0) ticket_sh = __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const unsigned first_red = (unsigned)(nblk - NTD);
  if (ticket_sh < first_red) return;
  const int tile = (int)(ticket_sh - first_red);
  if (tid == 0) {
    unsigned spins = 0;
    while (__hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)nblk) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 22)) {  // ~0.1-1 s: report instead of hanging the GPU
        if (p.err) *p.err = 1;
        break;
      }
    }
  }
  __syncthreads();
  // tile reduction: S slices of the block range per (row, column) pair (S = 8 for M <= 8, else 4); each
  // thread issues all of its slice's partial loads before summing them in block order, slices combined in order
  const int PR = M <= 8 ? 128 : 256, S = 1024 / PR;
  const int slice = tid / PR, rc = tid % PR, m = rc >> 4, col = tile * 16 + (rc & 15);
  const int per = (nblk + S - 1) / S, b0 = slice * per, b1 = min(nblk, b0 + per);
  constexpr int RB = 32;  // loads in flight per thread (per <= 64 for grid <= 256)
  if (m < M) {
    float s = 0.f;
    for (int c0 = b0; c0 < b1; c0 += RB) {
      float v[RB];
#pragma unroll
      for (int i = 0; i < RB; ++i)
        v[i] = c0 + i < b1 ? __hip_atomic_load(part + ((size_t)(c0 + i) * M + m) * H + col, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)
                           : 0.f;
#pragma unroll
      for (int i = 0; i < RB; ++i) s += v[i];
    }
    rsum[slice][m][rc & 15] = s;
  }
  __syncthreads();
  if (tid < M * 16) {
    const int mm = tid >> 4, cc = tid & 15;
    float s = 0.f;
    for (int sl = 0; sl < S; ++sl) s += rsum[sl][mm][cc];
    float* xo = p.x + (long long)mm * p.ldx + tile * 16 + cc;
    *xo = *xo + s;
  }
  if (tid == 0) {
    const unsigned d = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d == (unsigned)NTD - 1) {  // every reducer is past its wait: re-arm for the next launch
      __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace

extern "C" long long qt_mlp_ws_bytes(int M, int H, int I) {
  return MLP_WS_HEAD + (long long)(I / 32) * M * H * (long long)sizeof(float);
}

extern "C" int qt_mlp_decode(const qt_mlp_args* a, void* stream) {
  if (!a || !a->x || !a->w_gu || !a->w_down || !a->ws) return QT_ERR_ARG;
  if (a->M <= 0 || a->M > 16 || a->I % 32 || a->I / 32 > 256 || a->I / 32 < a->H / 16) return QT_ERR_SHAPE;
  if (a->ws_bytes < qt_mlp_ws_bytes(a->M, a->H, a->I)) return QT_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(a->I / 32), block(1024);
  switch (a->H) {
    case 1024: hipLaunchKernelGGL((mlp_decode_k<1024, 8>), grid, block, 0, s, *a); break;
    case 2048: hipLaunchKernelGGL((mlp_decode_k<2048, 8>), grid, block, 0, s, *a); break;
    default: return QT_ERR_SHAPE;
  }
  return hipGetLastError() == hipSuccess ? 0 : QT_ERR_LAUNCH;
}
