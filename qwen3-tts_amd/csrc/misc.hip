// Small memory-bound kernels: RMSNorm, embedding gathers, frame embedding sum, counters, codec
// elementwise (RVQ gather-sum, SnakeBeta, ConvNeXt depthwise conv + LayerNorm, clamp).
// All vectorised 16 B/lane where the row layout allows (channels-last, C % 8 == 0).
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void rmsnorm_k(const float* __restrict__ x, const float* __restrict__ g, float eps,
                                                 float* __restrict__ out, int N, float* __restrict__ rec = nullptr,
                                                 long long rec_ld = 0, const int* __restrict__ step = nullptr,
                                                 int step_off = 0, int step_stride = 0) {
  __shared__ float red[4];
  const int m = blockIdx.x, tid = threadIdx.x;
  const float* xr = x + (long long)m * N;
  float s = 0.f;
  for (int i = tid; i < N; i += 256) s += xr[i] * xr[i];
  s = wave_sum(s);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  const float rs = rsqrtf((red[0] + red[1] + red[2] + red[3]) / (float)N + eps);
  float* rr = rec ? rec + (long long)m * rec_ld + (long long)(step[m * step_stride] + step_off) * N : nullptr;
  for (int i = tid; i < N; i += 256) {
    const float v = g[i] * (xr[i] * rs);
    out[(long long)m * N + i] = v;
    if (rr) rr[i] = v;
  }
}

template <typename T>
__global__ void gather_rows_k(const T* __restrict__ tab, const int* __restrict__ idx, int H, float* __restrict__ out,
                              long long ldo) {
  const int m = blockIdx.x;
  const T* src = tab + (long long)idx[m] * H;
  for (int i = threadIdx.x; i < H; i += blockDim.x) out[(long long)m * ldo + i] = to_f(src[i]);
}

template <typename ET>
__global__ __launch_bounds__(64) void frame_embed_k(const ET* __restrict__ e0, const ET* __restrict__ ecp, int V0,
                                                     int Vcp, int G, int H, const int* __restrict__ codes,
                                                     long long codes_ld, const int* __restrict__ step,
                                                     int step_stride, const float* __restrict__ trailing, int T,
                                                     const float* __restrict__ pad, float* __restrict__ x,
                                                     bf16_t* __restrict__ x16) {
  // ET: table dtype.  Block (b, y) sums dims [y * 8 * blockDim, ...) of row b (several blocks per row: the 16
  // table-row slices are spread over CUs instead of one CU taking in the whole 16-row gather).  Codes to LDS once,
  // then every thread issues its 16 row-slice loads before summing.
  __shared__ int cs[32];
  const int b = blockIdx.x;
  const int t = step[b * step_stride];  // per-row frame index (step_stride 1) or one shared counter (0)
  if (threadIdx.x < G) cs[threadIdx.x] = codes[(long long)b * codes_ld + (long long)t * G + threadIdx.x];
  __syncthreads();
  const float* tr = t < T ? trailing + ((long long)b * T + t) * H : pad;
  for (int i = (blockIdx.y * blockDim.x + threadIdx.x) * 8; i < H; i += gridDim.y * blockDim.x * 8) {
    float acc[8], v[8];
    load8f(e0 + (long long)cs[0] * H + i, acc);
    for (int g = 1; g < G; ++g) {  // sum order: cat([...16 codebooks]).sum(1) then + text (M:1681-1692)
      load8f(ecp + ((long long)(g - 1) * Vcp + cs[g]) * H + i, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
    load8f(tr + i, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += v[j];
    store4(x + (long long)b * H + i, acc);
    store4(x + (long long)b * H + i + 4, acc + 4);
    if (x16)
      *(u32x4_t*)(x16 + (long long)b * H + i) =
          u32x4_t{pack2bf(acc[0], acc[1]), pack2bf(acc[2], acc[3]), pack2bf(acc[4], acc[5]), pack2bf(acc[6], acc[7])};
  }
}

__global__ void advance_k(int* c, int n) {
  int i = threadIdx.x;
  if (i < n) c[i] += 1;
}

// per-row counters, field-major [nf][B] with field 0 = the row's frame index: a row advances all its fields
// together until its frame index reaches cap, then stays (a finished slot waiting to be refilled keeps re-running
// frame `cap` in place instead of writing past its buffers)
__global__ void advance_rows_k(int* c, int B, int nf, int cap) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B || c[b] >= cap) return;
  for (int f = 0; f < nf; ++f) c[f * B + b] += 1;
}

__global__ void rvq_gather_k(const float* __restrict__ tabs, int Q, int n_first, int cb, int dim,
                             const int* __restrict__ codes, float* __restrict__ o1, float* __restrict__ o2) {
  const long long bt = blockIdx.x;  // b*T + t
  const int* c = codes + bt * Q;
  for (int i = threadIdx.x; i < dim; i += blockDim.x) {
    float s1 = 0.f, s2 = 0.f;
    for (int q = 0; q < Q; ++q) {
      const int code = min(max(c[q], 0), cb - 1);  // callers validate; never read outside the table
      float v = tabs[((long long)q * cb + code) * dim + i];
      if (q < n_first) s1 += v; else s2 += v;
    }
    o1[bt * dim + i] = s1;
    o2[bt * dim + i] = s2;
  }
}

template <typename T>
__global__ void snake_k(const T* __restrict__ x, T* __restrict__ y, long long n8, int C, const float* __restrict__ al,
                        const float* __restrict__ ib) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    float v[8];
    load8f(x + i * 8, v);
    const int c0 = (int)((i * 8) % C);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float s = sinf(v[j] * al[c0 + j]);
      v[j] = v[j] + ib[c0 + j] * (s * s);
    }
    store4(y + i * 8, v);
    store4(y + i * 8 + 4, v + 4);
  }
}

// one block per (b, t) row: depthwise causal conv k=7 over time, then LayerNorm over C (fp32 math)
template <typename T>
__global__ __launch_bounds__(256) void dwconv_ln_k(const T* __restrict__ x, int Tn, int C, const float* __restrict__ w,
                                                   const float* __restrict__ bias, const float* __restrict__ lw,
                                                   const float* __restrict__ lb, float eps, T* __restrict__ out) {
  extern __shared__ float buf[];
  __shared__ float red[2][4];
  const long long row = blockIdx.x;
  const int b = row / Tn, t = row % Tn;
  const int tid = threadIdx.x;
  float s1 = 0.f;
  for (int c = tid; c < C; c += 256) {
    float a = bias[c];
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      const int ti = t - 6 + j;
      if (ti >= 0) a += w[c * 7 + j] * to_f(x[((long long)b * Tn + ti) * C + c]);
    }
    buf[c] = a;
    s1 += a;
  }
  s1 = wave_sum(s1);
  if ((tid & 63) == 0) red[0][tid >> 6] = s1;
  __syncthreads();
  const float mean = (red[0][0] + red[0][1] + red[0][2] + red[0][3]) / (float)C;
  float s2 = 0.f;
  for (int c = tid; c < C; c += 256) { float d = buf[c] - mean; s2 += d * d; }
  s2 = wave_sum(s2);
  if ((tid & 63) == 0) red[1][tid >> 6] = s2;
  __syncthreads();
  const float rstd = rsqrtf((red[1][0] + red[1][1] + red[1][2] + red[1][3]) / (float)C + eps);
  for (int c = tid; c < C; c += 256) out[row * C + c] = from_f<T>((buf[c] - mean) * rstd * lw[c] + lb[c]);
}

template <typename T>
__global__ void clamp_k(const T* __restrict__ x, long long n, float* __restrict__ o) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    o[i] = fminf(fmaxf(to_f(x[i]), -1.f), 1.f);
}

inline int ok() { return hipGetLastError() == hipSuccess ? 0 : QT_ERR_LAUNCH; }
inline unsigned grid_for(long long n, int bs) {
  long long g = (n + bs - 1) / bs;
  return (unsigned)(g > 65536 ? 65536 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" int qt_rmsnorm(const float* x, const float* g, float eps, float* out, int M, int N, void* s) {
  if (M <= 0 || N <= 0) return QT_ERR_SHAPE;
  hipLaunchKernelGGL(rmsnorm_k, dim3(M), dim3(256), 0, (hipStream_t)s, x, g, eps, out, N);
  return ok();
}

extern "C" int qt_rmsnorm_rec(const float* x, const float* g, float eps, float* out, int M, int N, float* rec,
                              long long rec_ld, const int* step, int step_off, int step_stride, void* s) {
  if (M <= 0 || N <= 0 || !rec || !step || step_stride < 0) return QT_ERR_SHAPE;
  hipLaunchKernelGGL(rmsnorm_k, dim3(M), dim3(256), 0, (hipStream_t)s, x, g, eps, out, N, rec, rec_ld, step, step_off,
                     step_stride);
  return ok();
}

extern "C" int qt_gather_rows(const void* tab, int dtype, const int* idx, int M, int H, float* out, long long ldo,
                              void* s) {
  if (M <= 0 || H <= 0) return QT_ERR_SHAPE;
  if (dtype == QT_BF16)
    hipLaunchKernelGGL(gather_rows_k<bf16_t>, dim3(M), dim3(256), 0, (hipStream_t)s, (const bf16_t*)tab, idx, H, out, ldo);
  else if (dtype == QT_F32)
    hipLaunchKernelGGL(gather_rows_k<float>, dim3(M), dim3(256), 0, (hipStream_t)s, (const float*)tab, idx, H, out, ldo);
  else
    return QT_ERR_DTYPE;
  return ok();
}

extern "C" int qt_frame_embed(const void* e0, const void* ecp, int dtype, int V0, int Vcp, int G, int H,
                              const int* codes, long long codes_ld, const int* step, int step_stride,
                              const float* trailing, int T, const float* pad, float* x, void* x16, int B, void* s) {
  if (B <= 0 || H <= 0 || G < 1 || G > 32 || H % 8 || step_stride < 0) return QT_ERR_SHAPE;
  const dim3 grid(B, (H + 511) / 512);  // one wave per 512 dims
  if (dtype == QT_BF16)
    hipLaunchKernelGGL(frame_embed_k<bf16_t>, grid, dim3(64), 0, (hipStream_t)s, (const bf16_t*)e0,
                       (const bf16_t*)ecp, V0, Vcp, G, H, codes, codes_ld, step, step_stride, trailing, T, pad, x, (bf16_t*)x16);
  else if (dtype == QT_F32)
    hipLaunchKernelGGL(frame_embed_k<float>, grid, dim3(64), 0, (hipStream_t)s, (const float*)e0,
                       (const float*)ecp, V0, Vcp, G, H, codes, codes_ld, step, step_stride, trailing, T, pad, x, (bf16_t*)x16);
  else
    return QT_ERR_DTYPE;
  return ok();
}

extern "C" int qt_advance(int* c, int n, void* s) {
  if (n <= 0 || n > 1024) return QT_ERR_SHAPE;
  hipLaunchKernelGGL(advance_k, dim3(1), dim3(1024), 0, (hipStream_t)s, c, n);
  return ok();
}

extern "C" int qt_advance_rows(int* c, int B, int nfields, int cap, void* s) {
  if (B <= 0 || nfields <= 0) return QT_ERR_SHAPE;
  hipLaunchKernelGGL(advance_rows_k, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)s, c, B, nfields, cap);
  return ok();
}

extern "C" int qt_rvq_gather(const float* tabs, int Q, int n_first, int cb, int dim, const int* codes, int B, int T,
                             float* o1, float* o2, void* s) {
  if (B * T <= 0 || dim <= 0) return QT_ERR_SHAPE;
  hipLaunchKernelGGL(rvq_gather_k, dim3(B * T), dim3(256), 0, (hipStream_t)s, tabs, Q, n_first, cb, dim, codes, o1, o2);
  return ok();
}

extern "C" int qt_snake(const void* x, void* y, int dtype, long long rows, int C, const float* al, const float* ib,
                        void* s) {
  if (C % 8 || rows <= 0) return QT_ERR_SHAPE;
  const long long n8 = rows * C / 8;
  if (dtype == QT_BF16)
    hipLaunchKernelGGL(snake_k<bf16_t>, dim3(grid_for(n8, 256)), dim3(256), 0, (hipStream_t)s, (const bf16_t*)x,
                       (bf16_t*)y, n8, C, al, ib);
  else if (dtype == QT_F32)
    hipLaunchKernelGGL(snake_k<float>, dim3(grid_for(n8, 256)), dim3(256), 0, (hipStream_t)s, (const float*)x,
                       (float*)y, n8, C, al, ib);
  else
    return QT_ERR_DTYPE;
  return ok();
}

extern "C" int qt_dwconv_ln(const void* x, int dtype, int B, int T, int C, const float* w, const float* b,
                            const float* lw, const float* lb, float eps, void* out, void* s) {
  if (B * T <= 0 || C <= 0 || C > 8192) return QT_ERR_SHAPE;
  const size_t sh = C * sizeof(float);
  if (dtype == QT_BF16)
    hipLaunchKernelGGL(dwconv_ln_k<bf16_t>, dim3(B * T), dim3(256), sh, (hipStream_t)s, (const bf16_t*)x, T, C, w, b,
                       lw, lb, eps, (bf16_t*)out);
  else if (dtype == QT_F32)
    hipLaunchKernelGGL(dwconv_ln_k<float>, dim3(B * T), dim3(256), sh, (hipStream_t)s, (const float*)x, T, C, w, b,
                       lw, lb, eps, (float*)out);
  else
    return QT_ERR_DTYPE;
  return ok();
}

extern "C" int qt_clamp_pcm(const void* x, int dtype, long long n, float* o, void* s) {
  if (n <= 0) return QT_ERR_SHAPE;
  if (dtype == QT_BF16)
    hipLaunchKernelGGL(clamp_k<bf16_t>, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)s, (const bf16_t*)x, n, o);
  else if (dtype == QT_F32)
    hipLaunchKernelGGL(clamp_k<float>, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)s, (const float*)x, n, o);
  else
    return QT_ERR_DTYPE;
  return ok();
}
