// Voice-clone front end kernels: the non-GEMM pieces of the 12 Hz tokenizer ENCODER
// (Mimi: padding, LayerNorm, residual-VQ nearest-codeword search) and of the mel + ECAPA-TDNN speaker encoder
// (reflect padding, log-mel, time statistics / attentive pooling, squeeze-excitation).  Every conv / linear of
// both networks runs on the weight-tiled MFMA GEMM (gemm.hip); these kernels are the glue between them.
// All of it is bandwidth- or latency-bound one-shot work per reference clip (a 3 s clip is 38 frames).
//
// T = transformers models/mimi/modeling_mimi.py, M = qwen_tts/core/models/modeling_qwen3_tts.py.
#include "common.h"

namespace {

// ---------------------------------------------------------------------------------------------------------
// time-axis pad / copy (channels-last); one thread per output element, channels fastest (coalesced)
template <typename T>
__global__ void pad_time_k(const T* __restrict__ x, long long ldx, const T* __restrict__ x2, long long ldx2, int B,
                           int Tn, int C, int left, int right, int mode, int t_total, T* __restrict__ out, long long ldo) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long tot = (long long)B * t_total * C;
  if (idx >= tot) return;
  const int c = (int)(idx % C);
  const long long bt = idx / C;
  const int t = (int)(bt % t_total), b = (int)(bt / t_total);
  int s = t - left;
  float v = 0.f;
  bool ok = t < Tn + left + right;
  if (ok && (s < 0 || s >= Tn)) {
    if (mode == QT_PAD_REFLECT) s = s < 0 ? -s : 2 * (Tn - 1) - s;
    else if (mode == QT_PAD_REPLICATE) s = s < 0 ? 0 : Tn - 1;
    else ok = false;
  }
  if (ok) {
    v = to_f(x[((long long)b * Tn + s) * ldx + c]);
    if (x2) v += to_f(x2[((long long)b * Tn + s) * ldx2 + c]);
  }
  out[((long long)b * t_total + t) * ldo + c] = from_f<T>(v);
}

template <typename T>
__global__ void zero_tail_k(T* __restrict__ x, int B, int Tp, int v, int C, long long ldx) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int rows = Tp - v;
  if (idx >= (long long)B * rows * C) return;
  const int c = (int)(idx % C);
  const long long br = idx / C;
  const int t = v + (int)(br % rows), b = (int)(br / rows);
  x[((long long)b * Tp + t) * ldx + c] = from_f<T>(0.f);
}

// ---------------------------------------------------------------------------------------------------------
// LayerNorm: one 256-thread block per row, two passes over the row (mean, then centred variance) like torch
template <typename OT>
__global__ __launch_bounds__(256) void layernorm_k(const float* __restrict__ x, long long ldx, const float* __restrict__ w,
                                                   const float* __restrict__ b, float eps, OT* __restrict__ out,
                                                   long long ldo, int N) {
  __shared__ float red[4];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float* xr = x + (long long)row * ldx;
  auto block_sum = [&](float s) {
    s = wave_sum(s);
    __syncthreads();
    if (lane == 0) red[wv] = s;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
  };
  float s = 0.f;
  for (int i = tid; i < N; i += 256) s += xr[i];
  const float mean = block_sum(s) / (float)N;
  float q = 0.f;
  for (int i = tid; i < N; i += 256) { const float d = xr[i] - mean; q += d * d; }
  const float rs = rsqrtf(block_sum(q) / (float)N + eps);
  OT* o = out + (long long)row * ldo;
  for (int i = tid; i < N; i += 256) o[i] = from_f<OT>((xr[i] - mean) * rs * w[i] + b[i]);
}

// ---------------------------------------------------------------------------------------------------------
// Residual VQ encode, one launch per codebook stage q.  Grid = (cb / 64 codeword slices) x (row tiles of 32
// frames): each block stages its slice of the transposed table [D][64] and its 32 residual rows in LDS and
// scores all 32 x 64 (row, codeword) pairs as exact fp32 sums of (res - e)^2 (no |x|^2 + |e|^2 - 2 x.e
// cancellation); wave w owns rows 8w..8w+7, lane j codeword j of the slice.  Per row the slice minimum
// (lowest index on ties) goes to a partial record; the last block of the row tile to arrive (agent-scope
// relaxed atomics + explicit vmcnt drain: coherent across the 8 XCD L2s without an L2 writeback) reduces the
// partials in slice order, writes the code and advances the residual res = res - E_q[code] for stage q+1.
// The stage-to-stage dependency is carried by the launch boundary.
constexpr int RVQ_W = 64, RVQ_RB = 32, RVQ_MAXD = 256;

struct RvqWs {
  unsigned* cnt; float* pd; int* pi; float* res;
};

__host__ __device__ inline RvqWs rvq_ws(void* ws, int R, int D, int S) {
  const int tiles = (R + RVQ_RB - 1) / RVQ_RB;
  char* p = (char*)ws;
  RvqWs w;
  w.cnt = (unsigned*)p; p += ((size_t)tiles * sizeof(unsigned) + 255) / 256 * 256;
  w.pd = (float*)p; p += ((size_t)R * S * sizeof(float) + 255) / 256 * 256;
  w.pi = (int*)p; p += ((size_t)R * S * sizeof(int) + 255) / 256 * 256;
  w.res = (float*)p;
  return w;
}

__global__ __launch_bounds__(256) void rvq_stage_k(const float* __restrict__ x, long long ldx,
                                                   const float* __restrict__ tab, const float* __restrict__ tabT, int q,
                                                   int cb, int D, int R, int* __restrict__ codes, long long codes_ld,
                                                   RvqWs ws) {
  __shared__ float eT[RVQ_MAXD][RVQ_W + 1];
  __shared__ __attribute__((aligned(16))) float rs[RVQ_RB][RVQ_MAXD];
  __shared__ int last;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int s = blockIdx.x, S = gridDim.x, r0 = blockIdx.y * RVQ_RB;
  const int nr = min(RVQ_RB, R - r0);
  // staging: every load of the slice and of the rows is issued before the first LDS store (16-byte codeword loads;
  // one scalar load per row element), so the block waits for one round trip instead of one per loop iteration
  const float* tq = tabT + (size_t)q * D * cb + (size_t)s * RVQ_W;
  constexpr int EL = RVQ_MAXD * RVQ_W / 4 / 256, RL = RVQ_RB * RVQ_MAXD / 256;
  f32x4_t ev[EL];
#pragma unroll
  for (int j = 0; j < EL; ++j) {
    const int i = tid + 256 * j, d = min(i / (RVQ_W / 4), D - 1), c4 = (i % (RVQ_W / 4)) * 4;
    ev[j] = *(const f32x4_t*)(tq + (size_t)d * cb + c4);
  }
  const float* src = q == 0 ? x : ws.res;
  const long long lds = q == 0 ? ldx : D;
  float rv[RL];
#pragma unroll
  for (int j = 0; j < RL; ++j) {
    const int i = tid + 256 * j, r = i / RVQ_MAXD, d = i % RVQ_MAXD;
    rv[j] = src[(long long)(r0 + min(r, nr - 1)) * lds + min(d, D - 1)];
  }
#pragma unroll
  for (int j = 0; j < EL; ++j) {
    const int i = tid + 256 * j, d = i / (RVQ_W / 4), c4 = (i % (RVQ_W / 4)) * 4;
    if (d < D) { eT[d][c4] = ev[j][0]; eT[d][c4 + 1] = ev[j][1]; eT[d][c4 + 2] = ev[j][2]; eT[d][c4 + 3] = ev[j][3]; }
  }
#pragma unroll
  for (int j = 0; j < RL; ++j) {
    const int i = tid + 256 * j, r = i / RVQ_MAXD, d = i % RVQ_MAXD;
    rs[r][d] = (r < nr && d < D) ? rv[j] : 0.f;
  }
  __syncthreads();
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  // d in order (the same fp32 sums as one d at a time); the 8 rows' values 4 d at a time (16-byte LDS reads)
  for (int d = 0; d < D; d += 4) {
    const float e0 = eT[d][lane], e1 = eT[d + 1][lane], e2 = eT[d + 2][lane], e3 = eT[d + 3][lane];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const f32x4_t r4 = *(const f32x4_t*)&rs[wv * 8 + k][d];
      float t = r4[0] - e0;
      acc[k] = fmaf(t, t, acc[k]);
      t = r4[1] - e1;
      acc[k] = fmaf(t, t, acc[k]);
      t = r4[2] - e2;
      acc[k] = fmaf(t, t, acc[k]);
      t = r4[3] - e3;
      acc[k] = fmaf(t, t, acc[k]);
    }
  }
  const int cidx = s * RVQ_W + lane;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float bd = acc[k];
    int bi = cidx;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float od = __shfl_xor(bd, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (od < bd || (od == bd && oi < bi)) { bd = od; bi = oi; }
    }
    const int r = wv * 8 + k;
    if (lane == 0 && r < nr) {
      __hip_atomic_store(ws.pd + (size_t)(r0 + r) * S + s, bd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ws.pi + (size_t)(r0 + r) * S + s, bi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __builtin_amdgcn_s_waitcnt(0);  // partials acknowledged before this block's arrival is counted
  __syncthreads();
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add(ws.cnt + blockIdx.y, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == (unsigned)S - 1;
    if (last) __hip_atomic_store(ws.cnt + blockIdx.y, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
  }
  __syncthreads();
  if (!last) return;
  // last arriver: per row (one wave per row, rows strided by 4 waves) reduce the S slice minima in order
  for (int r = wv; r < nr; r += 4) {
    float bd = INFINITY;
    int bi = 0x7fffffff;
    for (int j = lane; j < S; j += 64) {
      const float d = __hip_atomic_load(ws.pd + (size_t)(r0 + r) * S + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int i = __hip_atomic_load(ws.pi + (size_t)(r0 + r) * S + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (d < bd || (d == bd && i < bi)) { bd = d; bi = i; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float od = __shfl_xor(bd, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (od < bd || (od == bd && oi < bi)) { bd = od; bi = oi; }
    }
    if (lane == 0) codes[(long long)(r0 + r) * codes_ld + q] = bi;
    const float* e = tab + ((size_t)q * cb + bi) * D;
    for (int d = lane; d < D; d += 64) ws.res[(long long)(r0 + r) * D + d] = rs[r][d] - e[d];
  }
}

// ---------------------------------------------------------------------------------------------------------
// log-mel: one block per frame; magnitudes of the nbin DFT bins into LDS, then each thread one mel band
constexpr int MEL_MAXBIN = 1040;

__global__ __launch_bounds__(256) void mel_logmag_k(const float* __restrict__ spec, long long ld_spec, int nbin,
                                                    const float* __restrict__ basis, int nmel, float* __restrict__ out,
                                                    long long ldo) {
  __shared__ float mag[MEL_MAXBIN];
  const int f = blockIdx.x, tid = threadIdx.x;
  const float* s = spec + (long long)f * ld_spec;
  for (int k = tid; k < nbin; k += 256) {
    const float re = s[2 * k], im = s[2 * k + 1];
    mag[k] = sqrtf(re * re + im * im + 1e-9f);
  }
  __syncthreads();
  for (int m = tid; m < nmel; m += 256) {
    const float* br = basis + (long long)m * nbin;
    float acc = 0.f;
    for (int k = 0; k < nbin; ++k) acc = fmaf(br[k], mag[k], acc);
    out[(long long)f * ldo + m] = logf(fmaxf(acc, 1e-5f));
  }
}

// ---------------------------------------------------------------------------------------------------------
// time statistics (attentive statistics pooling): one block per (item, 64 channels), its TS_W waves split time; per
// wave an online softmax (max, sum of exp) of the logits, then the weighted mean and variance sums, each merged over
// the waves through LDS in wave order.  (One thread per channel looping over all T frames ran 116 us per call on 4 x
// 300 frames x 1536 channels.)
constexpr int TS_W = 8;
template <typename T>
__global__ __launch_bounds__(TS_W * 64) void time_stats_k(const T* __restrict__ x, long long ldx,
                                                          const float* __restrict__ lg, long long ldl, int B, int Tn,
                                                          int C, float eps, float* __restrict__ mean_out,
                                                          float* __restrict__ std_out, long long ld_out) {
  __shared__ float pm[TS_W][64], ps[TS_W][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane, b = blockIdx.y;
  const int cc = min(c, C - 1);  // clamped: every lane runs the block's barriers
  const int per = (Tn + TS_W - 1) / TS_W, t0 = min(Tn, w * per), t1 = min(Tn, t0 + per);
  const T* xc = x + (long long)b * Tn * ldx + cc;
  const float* lc = lg ? lg + (long long)b * Tn * ldl + cc : nullptr;
  float mx = 0.f, inv = 1.0f / (float)Tn;
  if (lc) {
    float m = -INFINITY, s = 0.f;
    for (int t = t0; t < t1; ++t) {
      const float v = lc[(long long)t * ldl];
      if (v > m) { s = s * expf(m - v) + 1.f; m = v; }
      else s += expf(v - m);
    }
    pm[w][lane] = m; ps[w][lane] = s;
    __syncthreads();
    mx = pm[0][lane];
#pragma unroll
    for (int j = 1; j < TS_W; ++j) mx = fmaxf(mx, pm[j][lane]);
    float se = 0.f;
#pragma unroll
    for (int j = 0; j < TS_W; ++j) se += pm[j][lane] == -INFINITY ? 0.f : ps[j][lane] * expf(pm[j][lane] - mx);
    inv = 1.0f / se;
    __syncthreads();
  }
  float mean = 0.f;
  for (int t = t0; t < t1; ++t) {
    const float wt = lc ? expf(lc[(long long)t * ldl] - mx) * inv : inv;
    mean = fmaf(wt, to_f(xc[(long long)t * ldx]), mean);
  }
  pm[w][lane] = mean;
  __syncthreads();
  mean = 0.f;
#pragma unroll
  for (int j = 0; j < TS_W; ++j) mean += pm[j][lane];
  if (w == 0 && c < C) mean_out[(long long)b * ld_out + c] = mean;
  if (!std_out) return;
  float var = 0.f;
  for (int t = t0; t < t1; ++t) {
    const float wt = lc ? expf(lc[(long long)t * ldl] - mx) * inv : inv;
    const float d = to_f(xc[(long long)t * ldx]) - mean;
    var = fmaf(wt, d * d, var);
  }
  ps[w][lane] = var;
  __syncthreads();
  var = 0.f;
#pragma unroll
  for (int j = 0; j < TS_W; ++j) var += ps[j][lane];
  if (w == 0 && c < C) std_out[(long long)b * ld_out + c] = sqrtf(fmaxf(var, eps));
}

template <typename T>
__global__ void scale_add_k(const T* __restrict__ x, long long ldx, const float* __restrict__ s, long long lds,
                            const T* __restrict__ res, long long ldr, int Tn, int C, long long total,
                            T* __restrict__ out, long long ldo) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int c = (int)(idx % C);
  const long long bt = idx / C;
  const int b = (int)(bt / Tn);
  const float v = to_f(x[bt * ldx + c]) * s[(long long)b * lds + c] + to_f(res[bt * ldr + c]);
  out[bt * ldo + c] = from_f<T>(v);
}

template <typename T>
__global__ void bcast_rows_k(const float* __restrict__ v, long long ldv, int Tn, int W, long long total,
                             T* __restrict__ out, long long ldo) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int w = (int)(idx % W);
  const long long bt = idx / W;
  const int b = (int)(bt / Tn);
  out[bt * ldo + w] = from_f<T>(v[(long long)b * ldv + w]);
}

inline unsigned nblk(long long n, int t = 256) { return (unsigned)((n + t - 1) / t); }

}  // namespace

extern "C" int qt_pad_time(const void* x, long long ldx, const void* x2, long long ldx2, int dtype, int B, int T, int C,
                           int left, int right, int mode, int t_total, void* out, long long ldo, void* stream) {
  if (!x || !out || B <= 0 || T <= 0 || C <= 0 || left < 0 || right < 0) return QT_ERR_ARG;
  if (t_total < T + left + right || mode < QT_PAD_ZERO || mode > QT_PAD_REPLICATE) return QT_ERR_SHAPE;
  if (mode == QT_PAD_REFLECT && (left >= T || right >= T)) return QT_ERR_SHAPE;  // torch reflect pad limit
  const long long tot = (long long)B * t_total * C;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == QT_F32)
    hipLaunchKernelGGL(pad_time_k<float>, dim3(nblk(tot)), dim3(256), 0, s, (const float*)x, ldx, (const float*)x2, ldx2,
                       B, T, C, left, right, mode, t_total, (float*)out, ldo);
  else if (dtype == QT_BF16)
    hipLaunchKernelGGL(pad_time_k<bf16_t>, dim3(nblk(tot)), dim3(256), 0, s, (const bf16_t*)x, ldx, (const bf16_t*)x2,
                       ldx2, B, T, C, left, right, mode, t_total, (bf16_t*)out, ldo);
  else return QT_ERR_DTYPE;
  return hipGetLastError() == hipSuccess ? QT_OK : QT_ERR_LAUNCH;
}

extern "C" int qt_zero_tail(void* x, int dtype, int B, int Tp, int v, int C, long long ldx, void* stream) {
  if (!x || B <= 0 || C <= 0 || v < 0 || v > Tp) return QT_ERR_ARG;
  if (v == Tp) return QT_OK;
  const long long tot = (long long)B * (Tp - v) * C;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == QT_F32) hipLaunchKernelGGL(zero_tail_k<float>, dim3(nblk(tot)), dim3(256), 0, s, (float*)x, B, Tp, v, C, ldx);
  else if (dtype == QT_BF16)
    hipLaunchKernelGGL(zero_tail_k<bf16_t>, dim3(nblk(tot)), dim3(256), 0, s, (bf16_t*)x, B, Tp, v, C, ldx);
  else return QT_ERR_DTYPE;
  return hipGetLastError() == hipSuccess ? QT_OK : QT_ERR_LAUNCH;
}

extern "C" int qt_layernorm(const float* x, long long ldx, const float* w, const float* b, float eps, void* out,
                            int o_dtype, long long ldo, int M, int N, void* stream) {
  if (!x || !w || !b || !out || M <= 0 || N <= 0) return QT_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (o_dtype == QT_F32) hipLaunchKernelGGL(layernorm_k<float>, dim3(M), dim3(256), 0, s, x, ldx, w, b, eps, (float*)out, ldo, N);
  else if (o_dtype == QT_BF16)
    hipLaunchKernelGGL(layernorm_k<bf16_t>, dim3(M), dim3(256), 0, s, x, ldx, w, b, eps, (bf16_t*)out, ldo, N);
  else return QT_ERR_DTYPE;
  return hipGetLastError() == hipSuccess ? QT_OK : QT_ERR_LAUNCH;
}

extern "C" long long qt_rvq_encode_ws_bytes(int R, int D, int cb) {
  if (R <= 0 || D <= 0 || cb <= 0) return 0;
  const int S = (cb + RVQ_W - 1) / RVQ_W, tiles = (R + RVQ_RB - 1) / RVQ_RB;
  auto up = [](size_t n) { return (n + 255) / 256 * 256; };
  return (long long)(up((size_t)tiles * 4) + up((size_t)R * S * 4) + up((size_t)R * S * 4) + (size_t)R * D * 4);
}

extern "C" int qt_rvq_encode(const float* x, long long ldx, const float* tab, const float* tabT, int Q, int cb, int D,
                             int R, int* codes, long long codes_ld, void* ws, long long ws_bytes, void* stream) {
  if (!x || !tab || !tabT || !codes || !ws || Q < 0 || R < 0) return QT_ERR_ARG;
  if (cb <= 0 || cb % RVQ_W || D <= 0 || D > RVQ_MAXD || D % 4) return QT_ERR_SHAPE;
  if (((size_t)tabT & 15) != 0) return QT_ERR_ARG;  // 16-byte codeword loads
  if (Q == 0 || R == 0) return QT_OK;
  if (ws_bytes < qt_rvq_encode_ws_bytes(R, D, cb)) return QT_ERR_ARG;
  const int S = cb / RVQ_W;
  const RvqWs w = rvq_ws(ws, R, D, S);
  const dim3 grid(S, (R + RVQ_RB - 1) / RVQ_RB);
  for (int q = 0; q < Q; ++q) {
    hipLaunchKernelGGL(rvq_stage_k, grid, dim3(256), 0, (hipStream_t)stream, x, ldx, tab, tabT, q, cb, D, R, codes,
                       codes_ld, w);
  }
  return hipGetLastError() == hipSuccess ? QT_OK : QT_ERR_LAUNCH;
}

extern "C" int qt_mel_logmag(const float* spec, long long ld_spec, int F, int nbin, const float* basis, int nmel,
                             float* out, long long ldo, void* stream) {
  if (!spec || !basis || !out || F < 0 || nmel <= 0) return QT_ERR_ARG;
  if (nbin <= 0 || nbin > MEL_MAXBIN || ld_spec < 2LL * nbin) return QT_ERR_SHAPE;
  if (F == 0) return QT_OK;
  hipLaunchKernelGGL(mel_logmag_k, dim3(F), dim3(256), 0, (hipStream_t)stream, spec, ld_spec, nbin, basis, nmel, out, ldo);
  return hipGetLastError() == hipSuccess ? QT_OK : QT_ERR_LAUNCH;
}

extern "C" int qt_time_stats(const void* x, int dtype, long long ldx, const float* logits, long long ldl, int B, int T,
                             int C, float eps, float* mean_out, float* std_out, long long ld_out, void* stream) {
  if (!x || !mean_out || B <= 0 || T <= 0 || C <= 0) return QT_ERR_ARG;
  const dim3 grid(nblk(C, 64), B);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == QT_F32)
    hipLaunchKernelGGL(time_stats_k<float>, grid, dim3(TS_W * 64), 0, s, (const float*)x, ldx, logits, ldl, B, T, C, eps,
                       mean_out, std_out, ld_out);
  else if (dtype == QT_BF16)
    hipLaunchKernelGGL(time_stats_k<bf16_t>, grid, dim3(TS_W * 64), 0, s, (const bf16_t*)x, ldx, logits, ldl, B, T, C, eps,
                       mean_out, std_out, ld_out);
  else return QT_ERR_DTYPE;
  return hipGetLastError() == hipSuccess ? QT_OK : QT_ERR_LAUNCH;
}

extern "C" int qt_scale_add(const void* x, long long ldx, const float* sc, long long lds, const void* res, long long ldr,
                            int dtype, int B, int T, int C, void* out, long long ldo, void* stream) {
  if (!x || !sc || !res || !out || B <= 0 || T <= 0 || C <= 0) return QT_ERR_ARG;
  const long long tot = (long long)B * T * C;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == QT_F32)
    hipLaunchKernelGGL(scale_add_k<float>, dim3(nblk(tot)), dim3(256), 0, s, (const float*)x, ldx, sc, lds,
                       (const float*)res, ldr, T, C, tot, (float*)out, ldo);
  else if (dtype == QT_BF16)
    hipLaunchKernelGGL(scale_add_k<bf16_t>, dim3(nblk(tot)), dim3(256), 0, s, (const bf16_t*)x, ldx, sc, lds,
                       (const bf16_t*)res, ldr, T, C, tot, (bf16_t*)out, ldo);
  else return QT_ERR_DTYPE;
  return hipGetLastError() == hipSuccess ? QT_OK : QT_ERR_LAUNCH;
}

extern "C" int qt_bcast_rows(const float* v, long long ldv, int B, int T, int W, void* out, int o_dtype, long long ldo,
                             void* stream) {
  if (!v || !out || B <= 0 || T <= 0 || W <= 0) return QT_ERR_ARG;
  const long long tot = (long long)B * T * W;
  hipStream_t s = (hipStream_t)stream;
  if (o_dtype == QT_F32)
    hipLaunchKernelGGL(bcast_rows_k<float>, dim3(nblk(tot)), dim3(256), 0, s, v, ldv, T, W, tot, (float*)out, ldo);
  else if (o_dtype == QT_BF16)
    hipLaunchKernelGGL(bcast_rows_k<bf16_t>, dim3(nblk(tot)), dim3(256), 0, s, v, ldv, T, W, tot, (bf16_t*)out, ldo);
  else return QT_ERR_DTYPE;
  return hipGetLastError() == hipSuccess ? QT_OK : QT_ERR_LAUNCH;
}
