// Logits processing + token selection (transformers 4.57 semantics), one 256-thread block per row.
// Each thread keeps its V/256 (<= 16) scores in registers (strided, coalesced loads).
// Greedy: argmax with lowest-index tie break (torch.argmax).
// Sampling: Temperature -> TopK -> TopP -> softmax -> draw from a Philox-4x32-10 stream keyed by
// (seed, step, substep, row).  Top-k threshold = exact k-th largest score, found by building its
// order-preserving 32-bit key MSB-first (<= 16 block-wide 2-bit steps, no sort); ties at the threshold are kept
// like TopKLogitsWarper.  The draw is an inverse CDF over a fixed category order (parallel prefix of
// per-thread masses), so it is an exact sample of the warped distribution; RNG streams differ from
// torch.multinomial, hence parity is distribution-level (tests/test_gpu_parity.py).
#include "common.h"
#include <cstdlib>

namespace {

constexpr int NT = 256;  // threads per row; PER = scores per thread (8 / 12 / 16 for V <= 2048 / 3072 / 4096)

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

QT_DEV unsigned okey(float f) {  // order-preserving float -> uint
  unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

QT_DEV float block_sum(float v, float* sh) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  return sh[0] + sh[1] + sh[2] + sh[3];
}
QT_DEV float block_max(float v, float* sh) {
  v = wave_max(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  return fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
}

struct SK {
  qt_sample_args a;
  int stop;  // measurement hook (QT_SAMPLE_STOP): end after phase 1..5; 0 = the full kernel
};

template <int PER>
__global__ __launch_bounds__(NT) void sample_k(SK pk) {
  const qt_sample_args& p = pk.a;
  __shared__ float sh[8];
  __shared__ int shi[4];
  __shared__ int cnt3[2][2][4];
  __shared__ unsigned cand[256];
  __shared__ int ncand;
  __shared__ unsigned shtk;
  __shared__ float srt[4096];
  const int r = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int V = p.V;
  const float* lg = p.logits + (long long)r * p.ld;
  const bool fin = p.finished && p.finished[r];
  const int ngen = p.n_generated ? *p.n_generated : 1 << 30;
  float s[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int v = tid + j * NT;
    float x = -INFINITY;
    if (v < V) {
      x = lg[v];
      if (p.seen && p.rep_penalty != 1.0f && p.seen[(long long)r * V + v]) x = x < 0.f ? x * p.rep_penalty : x / p.rep_penalty;
      if (p.eos_id >= 0 && v == p.eos_id && (ngen < p.min_new_tokens || p.ignore_eos)) x = -INFINITY;
      if (v >= p.suppress_lo && v < p.suppress_hi && v != p.suppress_keep) x = -INFINITY;
    }
    s[j] = x;
  }
  if (pk.stop == 1) {
    if (s[0] + s[PER - 1] == 1234.5f) p.tok_out[r] = 0;
    return;
  }
  int tok;
  if (!p.do_sample) {
    float best = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int v = tid + j * NT;
      if (v < V && (s[j] > best || (s[j] == best && v < bi))) { best = s[j]; bi = v; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      float ob = __shfl_xor(best, o, 64);
      int oi = __shfl_xor(bi, o, 64);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    if (lane == 0) { sh[w] = best; shi[w] = bi; }
    __syncthreads();
    best = sh[0]; bi = shi[0];
    for (int i = 1; i < 4; ++i)
      if (sh[i] > best || (sh[i] == best && shi[i] < bi)) { best = sh[i]; bi = shi[i]; }
    tok = bi;
  } else {
    const float invT = (p.temperature > 0.f && p.temperature != 1.0f) ? 1.0f / p.temperature : 1.0f;
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < PER; ++j) { s[j] *= invT; mx = fmaxf(mx, s[j]); }
    mx = block_max(mx, sh);
    if (pk.stop == 2) {
      if (mx == 1234.5f) p.tok_out[r] = 0;
      return;
    }
    unsigned tk = 0;  // keep keys >= tk
    if (p.top_k > 0 && p.top_k < V) {
      unsigned key[PER];
#pragma unroll
      for (int j = 0; j < PER; ++j) key[j] = (tid + j * NT < V) ? okey(s[j]) : 0u;
      // MSB-first construction of the k-th largest key, 2 bits per step.  Counts are per-thread VALU
      // compares summed by packed wave reductions (n1 | n2 << 16, n3) and one barrier per step; the search
      // stops as soon as exactly k keys are >= the prefix (that set is the top-k set).
      int cur = V, bit = 30;
      for (; bit >= 0 && cur != p.top_k && cur > 256; bit -= 2) {
        const unsigned c1 = tk | (1u << bit), c2 = tk | (2u << bit), c3 = tk | (3u << bit);
        int n12 = 0, n3 = 0;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
          n12 += (key[j] >= c1 ? 1 : 0) + (key[j] >= c2 ? 0x10000 : 0);
          n3 += key[j] >= c3 ? 1 : 0;
        }
        n12 = wave_sum_i(n12);
        n3 = wave_sum_i(n3);
        const int buf = (bit >> 1) & 1;
        if (lane == 0) { cnt3[buf][0][w] = n12; cnt3[buf][1][w] = n3; }
        __syncthreads();
        const int s12 = cnt3[buf][0][0] + cnt3[buf][0][1] + cnt3[buf][0][2] + cnt3[buf][0][3];
        const int t3 = cnt3[buf][1][0] + cnt3[buf][1][1] + cnt3[buf][1][2] + cnt3[buf][1][3];
        const int t1 = s12 & 0xFFFF, t2 = s12 >> 16;
        if (t3 >= p.top_k) { tk = c3; cur = t3; }
        else if (t2 >= p.top_k) { tk = c2; cur = t2; }
        else if (t1 >= p.top_k) { tk = c1; cur = t1; }
      }
      if (bit >= 0 && cur != p.top_k) {
        // <= 256 keys remain >= tk: compact them into LDS and finish the search in wave 0, barrier-free
        if (tid == 0) ncand = 0;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PER; ++j)
          if (tid + j * NT < V && key[j] >= tk) cand[atomicAdd(&ncand, 1)] = key[j];
        __syncthreads();
        if (w == 0) {
          unsigned ck[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) ck[i] = lane + 64 * i < cur ? cand[lane + 64 * i] : 0u;
          for (; bit >= 0 && cur != p.top_k; bit -= 2) {
            const unsigned c1 = tk | (1u << bit), c2 = tk | (2u << bit), c3 = tk | (3u << bit);
            int n12 = 0, n3 = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              n12 += (ck[i] >= c1 ? 1 : 0) + (ck[i] >= c2 ? 0x10000 : 0);
              n3 += ck[i] >= c3 ? 1 : 0;
            }
            const int s12 = wave_sum_i(n12), t3 = wave_sum_i(n3);
            const int t1 = s12 & 0xFFFF, t2 = s12 >> 16;
            if (t3 >= p.top_k) { tk = c3; cur = t3; }
            else if (t2 >= p.top_k) { tk = c2; cur = t2; }
            else if (t1 >= p.top_k) { tk = c1; cur = t1; }
          }
          if (lane == 0) shtk = tk;
        }
        __syncthreads();
        tk = shtk;
      }
    }
    if (pk.stop == 3) {
      if (tk == 12345u) p.tok_out[r] = 0;
      return;
    }
    if (p.top_p < 1.0f) {  // rare path: sorted list (descending) for the nucleus cut
      for (int j = 0; j < PER; ++j) {
        const int v = tid + j * NT;
        if (v < 4096) srt[v] = (v < V && okey(s[j]) >= tk) ? s[j] : -INFINITY;
      }
      int P2 = 1;
      while (P2 < V) P2 <<= 1;
      for (int v = PER * NT + tid; v < P2; v += NT) srt[v] = -INFINITY;  // slots beyond this PER's reach
      __syncthreads();
      for (int k = 2; k <= P2; k <<= 1)
        for (int jj = k >> 1; jj > 0; jj >>= 1) {
          for (int i = tid; i < P2; i += NT) {
            int ixj = i ^ jj;
            if (ixj > i) {
              float a = srt[i], b = srt[ixj];
              bool desc = (i & k) == 0;
              if (desc ? (a < b) : (a > b)) { srt[i] = b; srt[ixj] = a; }
            }
          }
          __syncthreads();
        }
      if (tid == 0) {
        float tot = 0.f;
        for (int j = 0; j < V && srt[j] > -INFINITY; ++j) tot += expf(srt[j] - mx);
        float cum = 0.f, cut = srt[0];
        for (int j = 0; j < V && srt[j] > -INFINITY; ++j) {
          if (cum >= p.top_p * tot) break;
          cum += expf(srt[j] - mx);
          cut = srt[j];
        }
        sh[4] = cut;
      }
      __syncthreads();
      tk = max(tk, okey(sh[4]));
    }
    float e[PER], mass = 0.f;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      e[j] = (tid + j * NT < V && okey(s[j]) >= tk && s[j] > -INFINITY) ? __expf(s[j] - mx) : 0.f;
      mass += e[j];
    }
    // inclusive prefix of per-thread masses (wave scan + wave offsets)
    float inc = mass;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      float y = __shfl_up(inc, o, 64);
      if (lane >= o) inc += y;
    }
    __syncthreads();
    if (lane == 63) sh[w] = inc;
    __syncthreads();
    float off = 0.f;
    for (int i = 0; i < w; ++i) off += sh[i];
    const float total = sh[0] + sh[1] + sh[2] + sh[3];
    inc += off;
    if (pk.stop == 4) {
      if (inc == 1234.5f) p.tok_out[r] = 0;
      return;
    }
    const float u = philox_uniform(p.seed, (unsigned)(p.step ? *p.step : 0), (unsigned)p.substep, (unsigned)(p.row_base + r)) * total;
    const float excl = inc - mass;
    if (tid == 0) shi[0] = -1;
    __syncthreads();
    if (mass > 0.f && u >= excl && (u < inc || tid == NT - 1 || inc >= total)) {
      float cum = excl;
      int pick = -1;
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        if (e[j] > 0.f) {
          pick = tid + j * NT;
          cum += e[j];
          if (cum > u) break;
        }
      }
      atomicCAS(&shi[0], -1, pick);
    }
    __syncthreads();
    tok = shi[0];
    if (tok < 0) {  // numerical edge: fall back to the argmax of the kept set
      tok = 0;
    }
  }
  if (fin) tok = p.eos_id;
  if (pk.stop == 5) {
    if (tid == 0) p.tok_out[r] = tok;
    return;
  }
  if (p.emb_table) {  // next-step input row: the chosen token's (projected) embedding
    const float* src = p.emb_table + (long long)tok * p.emb_dim;
    float* dst = p.emb_out + (long long)r * p.emb_ld;
    for (int i = tid * 4; i < p.emb_dim; i += NT * 4) *(f32x4_t*)(dst + i) = *(const f32x4_t*)(src + i);
  }
  if (tid != 0) return;
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
  if (!a || a->R <= 0 || a->V <= 0 || a->V > NT * 16 || !a->tok_out) return QT_ERR_SHAPE;
  if (a->do_sample && a->top_k > a->V) return QT_ERR_ARG;
  if (a->emb_table && (!a->emb_out || a->emb_dim % 4 || a->emb_ld % 4)) return QT_ERR_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  static const int stop = [] { const char* e = getenv("QT_SAMPLE_STOP"); return e ? atoi(e) : 0; }();
  const SK k{*a, stop};
  if (a->V <= NT * 8) hipLaunchKernelGGL(sample_k<8>, dim3(a->R), dim3(NT), 0, st, k);
  else if (a->V <= NT * 12) hipLaunchKernelGGL(sample_k<12>, dim3(a->R), dim3(NT), 0, st, k);
  else hipLaunchKernelGGL(sample_k<16>, dim3(a->R), dim3(NT), 0, st, k);
  return hipGetLastError() == hipSuccess ? 0 : QT_ERR_LAUNCH;
}
