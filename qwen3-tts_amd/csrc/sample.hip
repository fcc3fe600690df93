// Logits processing + token selection (transformers 4.57 semantics), one 256-thread block per row.
// Greedy: argmax with lowest-index tie break (torch.argmax).  Sampling: Temperature -> TopK -> TopP
// -> softmax -> inverse-CDF draw from a Philox-4x32-10 stream keyed by (seed, step, substep, row);
// distribution-level parity with torch.multinomial (RNG streams differ by device).
#include "common.h"

namespace {

constexpr int MAXV = 4096;

QT_DEV unsigned mulhilo(unsigned a, unsigned b, unsigned* hi) {
  unsigned long long p = (unsigned long long)a * b;
  *hi = (unsigned)(p >> 32);
  return (unsigned)p;
}

QT_DEV float philox_uniform(unsigned long long seed, unsigned c0, unsigned c1, unsigned c2) {
  unsigned k0 = (unsigned)seed, k1 = (unsigned)(seed >> 32);
  unsigned x0 = c0, x1 = c1, x2 = c2, x3 = 0x9E3779B9u;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    unsigned h0, h1;
    unsigned l0 = mulhilo(0xD2511F53u, x0, &h0);
    unsigned l1 = mulhilo(0xCD9E8D57u, x2, &h1);
    unsigned n0 = h1 ^ x1 ^ k0, n2 = h0 ^ x3 ^ k1;
    x0 = n0; x1 = l1; x2 = n2; x3 = l0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return ((x0 >> 8) + 0.5f) * (1.0f / 16777216.0f);  // (0, 1)
}

__global__ __launch_bounds__(256) void sample_k(qt_sample_args p) {
  __shared__ float sc[MAXV];
  __shared__ float srt[MAXV];
  __shared__ float rv[4];
  __shared__ int ri[4];
  const int r = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int V = p.V;
  const float* lg = p.logits + (long long)r * p.ld;
  const bool fin = p.finished && p.finished[r];
  const int ngen = p.n_generated ? *p.n_generated : 1 << 30;
  for (int v = tid; v < V; v += 256) {
    float s = lg[v];
    if (p.seen && p.rep_penalty != 1.0f && p.seen[(long long)r * V + v]) s = s < 0.f ? s * p.rep_penalty : s / p.rep_penalty;
    if (p.eos_id >= 0 && v == p.eos_id && (ngen < p.min_new_tokens || p.ignore_eos)) s = -INFINITY;
    if (v >= p.suppress_lo && v < p.suppress_hi && v != p.suppress_keep) s = -INFINITY;
    sc[v] = s;
  }
  __syncthreads();
  int tok;
  if (!p.do_sample) {
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int v = tid; v < V; v += 256) {
      float s = sc[v];
      if (s > best || (s == best && v < bi)) { best = s; bi = v; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      float ob = __shfl_xor(best, o, 64);
      int oi = __shfl_xor(bi, o, 64);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    if (lane == 0) { rv[w] = best; ri[w] = bi; }
    __syncthreads();
    best = rv[0]; bi = ri[0];
    for (int i = 1; i < 4; ++i)
      if (rv[i] > best || (rv[i] == best && ri[i] < bi)) { best = rv[i]; bi = ri[i]; }
    tok = bi;
  } else {
    const float invT = (p.temperature > 0.f && p.temperature != 1.0f) ? 1.0f / p.temperature : 1.0f;
    int P2 = 1;
    while (P2 < V) P2 <<= 1;
    for (int v = tid; v < P2; v += 256) {
      float s = v < V ? sc[v] * invT : -INFINITY;
      if (v < V) sc[v] = s;
      srt[v] = s;
    }
    __syncthreads();
    // bitonic sort, descending
    for (int k = 2; k <= P2; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = tid; i < P2; i += 256) {
          int ixj = i ^ j;
          if (ixj > i) {
            float a = srt[i], b = srt[ixj];
            bool desc = (i & k) == 0;
            if (desc ? (a < b) : (a > b)) { srt[i] = b; srt[ixj] = a; }
          }
        }
        __syncthreads();
      }
    float thr = -INFINITY;
    if (p.top_k > 0 && p.top_k < V) thr = srt[p.top_k - 1];
    const float mx = srt[0];
    // top-p on the sorted (descending) list: keep rank j while sum_{<j} p < top_p
    if (p.top_p < 1.0f) {
      if (tid == 0) {
        float tot = 0.f;
        for (int j = 0; j < V; ++j) { float s = srt[j]; if (s < thr || s == -INFINITY) break; tot += expf(s - mx); }
        float cum = 0.f, cut = thr;
        for (int j = 0; j < V; ++j) {
          float s = srt[j];
          if (s < thr || s == -INFINITY) break;
          if (cum >= p.top_p * tot) break;
          cum += expf(s - mx);
          cut = s;
        }
        rv[0] = cut;
      }
      __syncthreads();
      thr = fmaxf(thr, rv[0]);
      __syncthreads();
    }
    // inverse CDF over the kept set, in index order
    float part = 0.f;
    const int chunk = (V + 255) / 256;
    const int v0 = tid * chunk, v1 = min(V, v0 + chunk);
    for (int v = v0; v < v1; ++v) { float s = sc[v]; part += (s >= thr && s > -INFINITY) ? expf(s - mx) : 0.f; }
    srt[tid] = part;
    __syncthreads();
    if (tid == 0) {
      float tot = 0.f;
      for (int i = 0; i < 256; ++i) tot += srt[i];
      const float u = philox_uniform(p.seed, (unsigned)(p.step ? *p.step : 0), (unsigned)p.substep, (unsigned)r) * tot;
      float cum = 0.f;
      int pick = -1;
      for (int i = 0; i < 256 && pick < 0; ++i) {
        if (cum + srt[i] >= u && srt[i] > 0.f) {
          const int a0 = i * chunk, a1 = min(V, a0 + chunk);
          for (int v = a0; v < a1; ++v) {
            float s = sc[v];
            float e = (s >= thr && s > -INFINITY) ? expf(s - mx) : 0.f;
            cum += e;
            if (e > 0.f) pick = v;
            if (cum >= u && e > 0.f) break;
          }
        } else {
          cum += srt[i];
        }
      }
      ri[0] = pick < 0 ? 0 : pick;
    }
    __syncthreads();
    tok = ri[0];
  }
  if (tid != 0) return;
  if (fin) tok = p.eos_id;
  p.tok_out[r] = tok;
  if (p.codes) {
    const int st = (p.step ? *p.step : 0) + p.codes_step_off;
    p.codes[(long long)r * p.codes_ld + (long long)st * p.codes_w + p.codes_col] = tok;
  }
  if (p.seen) p.seen[(long long)r * V + tok] = 1;
  if (p.finished && p.eos_id >= 0 && tok == p.eos_id) p.finished[r] = 1;
}

}  // namespace

extern "C" int qt_sample(const qt_sample_args* a, void* stream) {
  if (!a || a->R <= 0 || a->V <= 0 || a->V > MAXV || !a->tok_out) return QT_ERR_SHAPE;
  if (a->do_sample && a->top_k > a->V) return QT_ERR_ARG;
  hipLaunchKernelGGL(sample_k, dim3(a->R), dim3(256), 0, (hipStream_t)stream, *a);
  return hipGetLastError() == hipSuccess ? 0 : QT_ERR_LAUNCH;
}
