// qkv post-processing (q/k RMSNorm + RoPE + KV-cache write) and row-wise GQA attention for gfx950.
//
// Attention is HBM-bound at decode: each (row, kv-head) block reads its K and V ranges once.
// Pass 1: 8-element (16 B bf16 / 32 B fp32) K fragments per lane, D/8 lanes per key, scores to LDS.
// Pass 2: softmax in fp32 over LDS; P.V with the same key-per-lane-group split, reduced across waves.
// Decode roofline: bytes = 2 * L * D * sizeof(kv) per (row, kv-head) / 8 TB/s.
#include "common.h"
#include "attn_dev.h"
#include <cstdlib>
#include <type_traits>

namespace {


template <typename KV>
__global__ __launch_bounds__(64) void qkv_post_k(qt_qkv_args p) {
  const int r = blockIdx.x, hh = blockIdx.y, lane = threadIdx.x;
  const int D = p.D, half = D >> 1;
  const int nq = p.Hq, nk = p.Hkv;
  const float* src = p.qkv + (long long)r * (nq + 2 * nk) * D + (long long)hh * D;
  const bool act = lane < half;
  float x0 = act ? src[lane] : 0.f, x1 = act ? src[lane + half] : 0.f;
  const bool isq = hh < nq, isk = !isq && hh < nq + nk;
  if (isq || isk) {
    const float* nw = isq ? p.q_norm : p.k_norm;
    if (nw) {  // Qwen3TTSRMSNorm over head_dim: x * rsqrt(mean(x^2) + eps), then weight *
      float ss = wave_sum(x0 * x0 + x1 * x1);
      float rs = rsqrtf(ss / (float)D + p.eps);
      if (act) { x0 = nw[lane] * (x0 * rs); x1 = nw[lane + half] * (x1 * rs); }
    }
    const int pos = p.rope_pos[r];
    if (act) {
      const float c = p.cos_tab[(long long)pos * half + lane], s = p.sin_tab[(long long)pos * half + lane];
      const float y0 = x0 * c - x1 * s, y1 = x1 * c + x0 * s;  // q*cos + rotate_half(q)*sin
      x0 = y0; x1 = y1;
    }
  }
  if (!act) return;
  if (isq) {
    float* q = p.q_out + (long long)r * nq * D + (long long)hh * D;
    q[lane] = x0; q[lane + half] = x1;
    return;
  }
  const int h = isk ? hh - nq : hh - nq - nk;
  KV* cache = (KV*)(isk ? p.k_cache : p.v_cache);
  KV* dst = cache + (((long long)p.row_batch[r] * nk + h) * p.Lmax + p.kv_pos[r]) * D;
  dst[lane] = from_f<KV>(x0);
  dst[lane + half] = from_f<KV>(x1);
}

// One block = one (query row, kv head); 4 waves split the key range.
template <typename KV, typename OT, int D, int NREP>
__global__ __launch_bounds__(256) void attn_rows_k(qt_attn_args p) {
  constexpr int LPK = D / 8;      // lanes per key
  constexpr int KPW = 64 / LPK;   // keys per wave-iteration
  extern __shared__ float smem[];  // [NREP][max_keys] scores, then [4][NREP][D] partial outputs
  __shared__ float red[2][4][NREP];
  const int r = blockIdx.x, h = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int grp = lane / LPK, sub = lane % LPK;
  const int b = p.row_batch[r];
  const int len = p.row_len[r];
  int start = p.row_start[r];
  if (p.window > 0) start = max(start, len - p.window);
  const int n = len - start;
  float* sc = smem;
  const float scale = rsqrtf((float)D);
  const long long base = ((long long)b * p.Hkv + h) * p.Lmax * D;
  const KV* Kc = (const KV*)p.k_cache + base;
  const KV* Vc = (const KV*)p.v_cache + base;

  float q[NREP][8];
#pragma unroll
  for (int j = 0; j < NREP; ++j)
    load8f(p.q + ((long long)r * p.Hq + h * NREP + j) * D + sub * 8, q[j]);

  // pass 1: scores
  for (int k0 = w * KPW; k0 < n; k0 += 4 * KPW) {
    const int kk = k0 + grp;
    float kv[8];
    if (kk < n) load8f(Kc + (long long)(start + kk) * D + sub * 8, kv);
    else {
#pragma unroll
      for (int i = 0; i < 8; ++i) kv[i] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < NREP; ++j) {
      float d = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) d += q[j][i] * kv[i];
#pragma unroll
      for (int o = LPK / 2; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
      if (sub == 0 && kk < n) sc[j * p.max_keys + kk] = d * scale;
    }
  }
  __syncthreads();
  // softmax (fp32) per rep head
  float mx[NREP], inv[NREP];
#pragma unroll
  for (int j = 0; j < NREP; ++j) {
    float m = -INFINITY;
    for (int k = threadIdx.x; k < n; k += 256) m = fmaxf(m, sc[j * p.max_keys + k]);
    m = wave_max(m);
    if (lane == 0) red[0][w][j] = m;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NREP; ++j) {
    mx[j] = fmaxf(fmaxf(red[0][0][j], red[0][1][j]), fmaxf(red[0][2][j], red[0][3][j]));
    float s = 0.f;
    for (int k = threadIdx.x; k < n; k += 256) {
      float e = expf(sc[j * p.max_keys + k] - mx[j]);
      sc[j * p.max_keys + k] = e;
      s += e;
    }
    s = wave_sum(s);
    if (lane == 0) red[1][w][j] = s;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NREP; ++j) inv[j] = 1.f / (red[1][0][j] + red[1][1][j] + red[1][2][j] + red[1][3][j]);

  // pass 2: P.V
  float acc[NREP][8];
#pragma unroll
  for (int j = 0; j < NREP; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = 0.f;
  for (int k0 = w * KPW; k0 < n; k0 += 4 * KPW) {
    const int kk = k0 + grp;
    if (kk < n) {
      float vv[8];
      load8f(Vc + (long long)(start + kk) * D + sub * 8, vv);
#pragma unroll
      for (int j = 0; j < NREP; ++j) {
        const float pj = sc[j * p.max_keys + kk] * inv[j];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[j][i] += pj * vv[i];
      }
    }
  }
  // reduce across key groups inside the wave (lanes with equal `sub`)
#pragma unroll
  for (int j = 0; j < NREP; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float v = acc[j][i];
#pragma unroll
      for (int o = LPK; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
      acc[j][i] = v;
    }
  float* part = smem + NREP * p.max_keys;  // [4][NREP][D]
  if (grp == 0) {
#pragma unroll
    for (int j = 0; j < NREP; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) part[(w * NREP + j) * D + sub * 8 + i] = acc[j][i];
  }
  __syncthreads();
  OT* out = (OT*)p.out;
  for (int e = threadIdx.x; e < NREP * D; e += 256) {
    const int j = e / D, d = e % D;
    float v = part[(0 * NREP + j) * D + d] + part[(1 * NREP + j) * D + d] + part[(2 * NREP + j) * D + d] +
              part[(3 * NREP + j) * D + d];
    out[((long long)r * p.Hq + h * NREP + j) * D + d] = from_f<OT>(v);
  }
}

template <typename KV, typename OT, int D>
int attn_dispatch_rep(const qt_attn_args& p, hipStream_t s) {
  const int nrep = p.Hq / p.Hkv;
  const size_t sh = (size_t)(nrep * p.max_keys + 4 * nrep * D) * sizeof(float);
  dim3 g(p.R, p.Hkv);
  switch (nrep) {
    case 1: hipLaunchKernelGGL((attn_rows_k<KV, OT, D, 1>), g, dim3(256), sh, s, p); break;
    case 2: hipLaunchKernelGGL((attn_rows_k<KV, OT, D, 2>), g, dim3(256), sh, s, p); break;
    case 4: hipLaunchKernelGGL((attn_rows_k<KV, OT, D, 4>), g, dim3(256), sh, s, p); break;
    default: return QT_ERR_SHAPE;
  }
  return hipGetLastError() == hipSuccess ? 0 : QT_ERR_LAUNCH;
}

template <typename KV, typename OT>
int attn_dispatch(const qt_attn_args& p, hipStream_t s) {
  switch (p.D) {
    case 16: return attn_dispatch_rep<KV, OT, 16>(p, s);
    case 64: return attn_dispatch_rep<KV, OT, 64>(p, s);
    case 128: return attn_dispatch_rep<KV, OT, 128>(p, s);
    default: return QT_ERR_SHAPE;
  }
}


// ---------------------------------------------------------------------------------------------------
// Fused decode attention: one 512-thread block per (query row, kv head).  Waves 0..NREP+1 first apply
// q/k RMSNorm + RoPE to this block's NREP query heads and its kv head's new key, append k/v to the cache
// at kv_pos (the new key itself is served from LDS, so no intra-launch global read-after-write), then all
// 8 waves stream the cached keys: lane group g (D/8 lanes, 16 B bf16 per lane) owns keys g, g+G, ...;
// K and V fragments of IC keys are loaded before any use (IC x 2 KiB in flight per group) and folded
// into an online softmax; partial (m, l, o) merge across groups by shuffles and across waves via LDS.
// Bytes per (row, head) = 2 * L * D * sizeof(kv): the decode-attention HBM roofline of SURVEY.md §8(d).
template <typename KV, int D, int NREP, int NW>
__global__ __launch_bounds__(NW * 64) void attn_decode_k(qt_decode_attn_args p) {
  // NW waves: 8 for long caches (8 x 64 lanes keeps kf/vf/o/q (~150 VGPRs) out of scratch), 4 for short ones
  // (code predictor, <= 17 keys: fewer idle waves in the merges)
  constexpr int LPK = D / 8, GPW = 64 / LPK, G = NW * GPW, IC = sizeof(KV) == 2 ? 4 : 2;
  __shared__ float qs[NREP][D];
  __shared__ float knew[D], vnew[D];
  __shared__ float mrg_ml[NW][NREP][2];
  __shared__ float mrg_o[NW][NREP][D];
  const int r = blockIdx.x, h = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int half = D / 2;
  const int nq = p.Hq, nk = p.Hkv;
  const bool cpos = p.const_pos >= 0;
  const int b = cpos ? r : p.row_batch[r];
  const int kvpos = cpos ? p.const_pos : p.kv_pos[r];
  const long long base = ((long long)b * nk + h) * p.Lmax * D;
  const int grp = lane / LPK, sub = lane % LPK;
  const int gid = w * GPW + grp;
  int start = cpos ? 0 : p.row_start[r];
  const int len = kvpos + 1;
  if (p.window > 0) start = max(start, len - p.window);
  const int n = len - start;  // keys [start, len); the last one (kvpos) comes from LDS
  const KV* Kc = (const KV*)p.k_cache + base;
  const KV* Vc = (const KV*)p.v_cache + base;
  // raw fragments stay packed (bf16: 4 VGPRs per 8 elements) until used: IC keys in flight per group
  constexpr int RW = sizeof(KV) * 8 / 4;  // 32-bit words per 8-element fragment
  unsigned kr[IC][RW], vr[IC][RW];   // chunk being consumed
  unsigned kn[IC][RW], vn[IC][RW];   // next chunk, in flight while the current one is consumed
  auto load_into = [&](int j0, unsigned (*kd)[RW], unsigned (*vd)[RW]) {  // cached keys only
#pragma unroll
    for (int c = 0; c < IC; ++c) {
      const int jj = min(j0 + c * G, max(n - 2, 0));
      const unsigned* ks = (const unsigned*)(Kc + (long long)(start + jj) * D + sub * 8);
      const unsigned* vs = (const unsigned*)(Vc + (long long)(start + jj) * D + sub * 8);
#pragma unroll
      for (int q4 = 0; q4 < RW; q4 += 4) {
        u32x4_t a = *(const u32x4_t*)(ks + q4), b = *(const u32x4_t*)(vs + q4);
        kd[c][q4] = a[0]; kd[c][q4 + 1] = a[1]; kd[c][q4 + 2] = a[2]; kd[c][q4 + 3] = a[3];
        vd[c][q4] = b[0]; vd[c][q4 + 1] = b[1]; vd[c][q4 + 2] = b[2]; vd[c][q4 + 3] = b[3];
      }
    }
  };
  auto load_chunk = [&](int j0) { load_into(j0, kr, vr); };
  auto unpack = [&](const unsigned* r, float* o8) {
    if constexpr (sizeof(KV) == 2) {
#pragma unroll
      for (int i = 0; i < 4; ++i) { o8[2 * i] = __uint_as_float(r[i] << 16); o8[2 * i + 1] = __uint_as_float(r[i] & 0xFFFF0000u); }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) o8[i] = __uint_as_float(r[i]);
    }
  };
  // split-KV: block z of gridDim.z owns keys [j_lo, j_hi) of [0, n) (the new key n-1 is in the last split)
  const int nsplit = gridDim.z, z = blockIdx.z;
  const int per_split = (n + nsplit - 1) / nsplit;
  const int j_lo = min(n, z * per_split), j_hi = min(n, j_lo + per_split);
  load_chunk(j_lo + gid);  // in flight while phase 0 runs (clamped addresses: no branch around the loads)
  // ---- phase 0: norm + rope of q heads / new k, v passthrough; append to cache
  if (w < NREP + 2) {
    const int hh = w < NREP ? h * NREP + w : (w == NREP ? nq + h : nq + nk + h);
    const float* src = p.qkv + (long long)r * (nq + 2 * nk) * D + (long long)hh * D;
    const bool act = lane < half;
    float x0 = act ? src[lane] : 0.f, x1 = act ? src[lane + half] : 0.f;
    if (w <= NREP) {
      const float* nw = w < NREP ? p.q_norm : p.k_norm;
      if (nw) {
        const float rs = rsqrtf(wave_sum(x0 * x0 + x1 * x1) / (float)D + p.eps);
        if (act) { x0 = nw[lane] * (x0 * rs); x1 = nw[lane + half] * (x1 * rs); }
      }
      const int pos = cpos ? p.const_pos : p.rope_pos[r];
      if (act) {
        const float c = p.cos_tab[(long long)pos * half + lane], sn = p.sin_tab[(long long)pos * half + lane];
        const float y0 = x0 * c - x1 * sn, y1 = x1 * c + x0 * sn;
        x0 = y0; x1 = y1;
      }
    }
    if (act) {
      float* dst = w < NREP ? qs[w] : (w == NREP ? knew : vnew);
      if (w >= NREP) {  // the new key/value as the cache will hold them (kv dtype rounding)
        x0 = to_f(from_f<KV>(x0));
        x1 = to_f(from_f<KV>(x1));
      }
      dst[lane] = x0; dst[lane + half] = x1;
      if (w >= NREP && z == nsplit - 1) {
        KV* cache = (KV*)(w == NREP ? p.k_cache : p.v_cache) + base + (long long)kvpos * D;
        cache[lane] = from_f<KV>(x0);
        cache[lane + half] = from_f<KV>(x1);
      }
    }
  }
  __syncthreads();
  // scores in log2 units: q pre-scaled by log2(e)/sqrt(D), every softmax exponential is one exp2
  const float scale = rsqrtf((float)D) * 1.4426950408889634f;
  float q[NREP][8];
#pragma unroll
  for (int j = 0; j < NREP; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) q[j][i] = qs[j][sub * 8 + i] * scale;
  float m[NREP], l[NREP], o[NREP][8];
#pragma unroll
  for (int j = 0; j < NREP; ++j) {
    m[j] = -INFINITY; l[j] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[j][i] = 0.f;
  }
  // ping-pong between the two register sets: chunk i is consumed from one while chunk i+1 streams into the
  // other (no register copies, so no wait on the prefetch before the next chunk's math)
  // one chunk = IC keys per lane group: all scores first, then one running-max update and one rescale
  auto consume = [&](auto& kd, auto& vd, const int jb) {
    float vf[IC][8], dd[NREP][IC];
#pragma unroll
    for (int c = 0; c < IC; ++c) {
      const bool valid = jb + c * G < j_hi;
      float kf[8];
      unpack(kd[c], kf);
      unpack(vd[c], vf[c]);
      if (jb + c * G >= n - 1) {
#pragma unroll
        for (int i = 0; i < 8; ++i) { kf[i] = knew[sub * 8 + i]; vf[c][i] = vnew[sub * 8 + i]; }
      }
#pragma unroll
      for (int j = 0; j < NREP; ++j) {
        float d = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) d += q[j][i] * kf[i];
        d = group_sum_dpp<LPK>(d);  // the key's LPK lanes are one DPP row (or part of one)
        dd[j][c] = valid ? d : -INFINITY;
      }
    }
#pragma unroll
    for (int j = 0; j < NREP; ++j) {
      float mn = m[j];
#pragma unroll
      for (int c = 0; c < IC; ++c) mn = fmaxf(mn, dd[j][c]);
      if (mn == -INFINITY) continue;  // no valid key yet in this lane group
      const float f = exp2_hw(m[j] - mn);
      float e[IC], es = 0.f;
#pragma unroll
      for (int c = 0; c < IC; ++c) { e[c] = exp2_hw(dd[j][c] - mn); es += e[c]; }
      l[j] = l[j] * f + es;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float acc = o[j][i] * f;
#pragma unroll
        for (int c = 0; c < IC; ++c) acc += e[c] * vf[c][i];
        o[j][i] = acc;
      }
      m[j] = mn;
    }
  };
  constexpr int GIC = G * IC;
  // The prefetches are unconditional (clamped addresses): a branch around them made hipcc's merged wait counts
  // drain the prefetch before the current chunk was consumed, serialising the two round trips.
  for (int j0 = j_lo + gid; j0 < j_hi; j0 += 2 * GIC) {
    load_into(j0 + GIC, kn, vn);
    consume(kr, vr, j0);
    if (j0 + GIC >= j_hi) break;
    load_into(j0 + 2 * GIC, kr, vr);
    consume(kn, vn, j0 + GIC);
  }
  // merge lane groups inside the wave (ds_bpermute butterflies: the permlane transpose-reduce GroupMerge was
  // measured 3 us slower in this kernel, 11.3 vs 8.2 us at 210 keys, tools/talker_attn_bench.py)
#pragma unroll
  for (int off = LPK; off < 64; off <<= 1) {
#pragma unroll
    for (int j = 0; j < NREP; ++j) {
      const float m2 = __shfl_xor(m[j], off, 64), l2 = __shfl_xor(l[j], off, 64);
      const float mn = fmaxf(m[j], m2);
      const float f1 = m[j] == -INFINITY ? 0.f : exp2_hw(m[j] - mn);
      const float f2 = m2 == -INFINITY ? 0.f : exp2_hw(m2 - mn);
      l[j] = l[j] * f1 + l2 * f2;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float o2 = __shfl_xor(o[j][i], off, 64);
        o[j][i] = o[j][i] * f1 + o2 * f2;
      }
      m[j] = mn;
    }
  }
  if (grp == 0) {
#pragma unroll
    for (int j = 0; j < NREP; ++j) {
      if (sub == 0) { mrg_ml[w][j][0] = m[j]; mrg_ml[w][j][1] = l[j]; }
#pragma unroll
      for (int i = 0; i < 8; ++i) mrg_o[w][j][sub * 8 + i] = o[j][i];
    }
  }
  __syncthreads();
  // split-KV partial record per (row, kv head, split, q head): [m, l, o[0..D)] (unnormalised)
  constexpr int REC = D + 2;
  float* part = nsplit > 1 ? (float*)((char*)p.ws + 4096) + (((size_t)r * nk + h) * nsplit) * NREP * REC : nullptr;
  for (int e = tid; e < NREP * D; e += NW * 64) {
    const int j = e / D, d = e % D;
    float mm = -INFINITY;
    for (int ww = 0; ww < NW; ++ww) mm = fmaxf(mm, mrg_ml[ww][j][0]);
    float ll = 0.f, oo = 0.f;
    for (int ww = 0; ww < NW; ++ww) {
      const float mw = mrg_ml[ww][j][0];
      const float f = mw == -INFINITY ? 0.f : exp2_hw(mw - mm);
      ll += mrg_ml[ww][j][1] * f;
      oo += mrg_o[ww][j][d] * f;
    }
    if (nsplit > 1) {
      float* rec = part + ((size_t)z * NREP + j) * REC;
      __hip_atomic_store(rec + 2 + d, oo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (d == 0) {
        __hip_atomic_store(rec, mm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(rec + 1, ll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      continue;
    }
    const long long oi = ((long long)r * nq + h * NREP + j) * D + d;
    if (p.o_dtype == QT_BF16) ((bf16_t*)p.out)[oi] = f2bf(oo / ll);
    else ((float*)p.out)[oi] = oo / ll;
  }
  if (nsplit == 1) return;
  // the last split to arrive merges all splits in split order (deterministic) and writes the output
  __shared__ unsigned last_sh;
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  unsigned* cnt = (unsigned*)p.ws + (size_t)r * nk + h;
  if (tid == 0)
    last_sh = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)nsplit - 1;
  __syncthreads();
  if (!last_sh) return;
  if (tid == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
  for (int e = tid; e < NREP * D; e += NW * 64) {
    const int j = e / D, d = e % D;
    float ms[8], ls[8], os[8];  // nsplit <= 8
    float mm = -INFINITY;
    for (int zz = 0; zz < nsplit; ++zz) {
      const float* rec = part + ((size_t)zz * NREP + j) * REC;
      ms[zz] = __hip_atomic_load(rec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ls[zz] = __hip_atomic_load(rec + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      os[zz] = __hip_atomic_load(rec + 2 + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    for (int zz = 0; zz < nsplit; ++zz) mm = fmaxf(mm, ms[zz]);
    float ll = 0.f, oo = 0.f;
    for (int zz = 0; zz < nsplit; ++zz) {
      const float f = ms[zz] == -INFINITY ? 0.f : exp2_hw(ms[zz] - mm);
      ll += ls[zz] * f;
      oo += os[zz] * f;
    }
    const long long oi = ((long long)r * nq + h * NREP + j) * D + d;
    if (p.o_dtype == QT_BF16) ((bf16_t*)p.out)[oi] = f2bf(oo / ll);
    else ((float*)p.out)[oi] = oo / ll;
  }
}

}  // namespace
extern "C" long long qt_decode_attn_ws_bytes(int R, int Hq, int Hkv, int D, int nsplit);
namespace {

// Short prefill where every key is new (code-predictor per-frame 2-token prefill, positions 0..T-1 of each
// batch item): one block per (batch item, kv head), one wave per (token, q head | k | v) for the q/k-norm +
// RoPE + cache append (as qkv_post_k), then one wave per (token, q head) for the causal softmax over the
// block's own T keys held in LDS.  Replaces qt_qkv_post + qt_attention (two launches) for this case.
template <typename KV, int D, int NREP, int T>
__global__ __launch_bounds__(64 * T * (NREP + 2)) void attn_small_prefill_k(qt_decode_attn_args p) {
  constexpr int half = D / 2;
  __shared__ float qs[T][NREP][D], ks[T][D], vs[T][D];
  const int b = blockIdx.x, h = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nq = p.Hq, nk = p.Hkv;
  {
    const int t = w / (NREP + 2), role = w % (NREP + 2);
    const int r = b * T + t;
    const int hh = role < NREP ? h * NREP + role : (role == NREP ? nq + h : nq + nk + h);
    const float* src = p.qkv + (long long)r * (nq + 2 * nk) * D + (long long)hh * D;
    const bool act = lane < half;
    float x0 = act ? src[lane] : 0.f, x1 = act ? src[lane + half] : 0.f;
    if (role <= NREP) {
      const float* nw = role < NREP ? p.q_norm : p.k_norm;
      if (nw) {
        const float rs = rsqrtf(wave_sum(x0 * x0 + x1 * x1) / (float)D + p.eps);
        if (act) { x0 = nw[lane] * (x0 * rs); x1 = nw[lane + half] * (x1 * rs); }
      }
      if (act) {
        const float c = p.cos_tab[(long long)t * half + lane], sn = p.sin_tab[(long long)t * half + lane];
        const float y0 = x0 * c - x1 * sn, y1 = x1 * c + x0 * sn;
        x0 = y0; x1 = y1;
      }
    }
    if (act) {
      if (role < NREP) {
        qs[t][role][lane] = x0; qs[t][role][lane + half] = x1;
      } else {  // as the cache holds them (kv dtype rounding), appended at position t
        const KV k0 = from_f<KV>(x0), k1 = from_f<KV>(x1);
        float* dst = role == NREP ? ks[t] : vs[t];
        dst[lane] = to_f(k0); dst[lane + half] = to_f(k1);
        KV* cache = (KV*)(role == NREP ? p.k_cache : p.v_cache) + (((long long)b * nk + h) * p.Lmax + t) * D;
        cache[lane] = k0; cache[lane + half] = k1;
      }
    }
  }
  __syncthreads();
  if (w >= T * NREP) return;
  const int t = w / NREP, j = w % NREP, r = b * T + t;
  const float scale = rsqrtf((float)D);
  const bool act = lane < half;
  const float q0 = act ? qs[t][j][lane] : 0.f, q1 = act ? qs[t][j][lane + half] : 0.f;
  float sc[T], mx = -INFINITY;
#pragma unroll
  for (int u = 0; u < T; ++u) {
    float d = act ? q0 * ks[u][lane] + q1 * ks[u][lane + half] : 0.f;
    d = wave_sum(d) * scale;
    sc[u] = u <= t ? d : -INFINITY;
    mx = fmaxf(mx, sc[u]);
  }
  float den = 0.f;
#pragma unroll
  for (int u = 0; u < T; ++u) { sc[u] = u <= t ? expf(sc[u] - mx) : 0.f; den += sc[u]; }
  if (!act) return;
  float o0 = 0.f, o1 = 0.f;
#pragma unroll
  for (int u = 0; u < T; ++u) { o0 += sc[u] * vs[u][lane]; o1 += sc[u] * vs[u][lane + half]; }
  const long long oi = ((long long)r * nq + h * NREP + j) * D;
  if (p.o_dtype == QT_BF16) {
    ((bf16_t*)p.out)[oi + lane] = f2bf(o0 / den);
    ((bf16_t*)p.out)[oi + lane + half] = f2bf(o1 / den);
  } else {
    ((float*)p.out)[oi + lane] = o0 / den;
    ((float*)p.out)[oi + lane + half] = o1 / den;
  }
}

// ---------------------------------------------------------------------------------------------------
// Decode attention fused into the output projection (code-predictor decode steps, <= 64 cached keys):
//   x[r] += W_o . attn(r)        (M:930-958 attention + o_proj + M:1004 residual, one launch instead of two)
// Block = (column group cg of NT o-proj column tiles, row r); wave w = kv head w (Hkv <= 8).  The block recomputes
// row r's attention for every kv head (q/k RMSNorm + RoPE of the raw projections, cached keys + the new key from
// LDS, online softmax with attn_decode_k's exp2 arithmetic), each wave multiplies its head's output (one K slice of
// o_proj) by its weight fragments -- in flight from the first instruction -- and the 8 head partials are summed in
// LDS in head order: no cross-block reduction (a split-K arrival across XCDs costs ~3 coherent memory round trips,
// ~5.6 us measured).  Blocks of one column group are XCD-aligned (linear id = r * CG + cg, CG % 8 == 0 at the
// model dims) so the weight slice is fetched into one L2 and re-read by the R row blocks.  Block cg == 0 appends
// the new k/v to the cache.  Re-reading a row's keys per column group costs R x CG x keys x 2 x D x sizeof(kv) of
// L2 / MALL reads: cheap for the code predictor's <= 17 keys, too much for the talker's long caches.
struct AOK {
  qt_attn_oproj_args a;
  int stop;  // measurement hook (QT_AO_STOP): end after phase 1..4; 0 = the full kernel
};

template <typename WT, typename KV, int D, int NREP, int NT, bool CPOS>
__global__ __launch_bounds__(512) void attn_oproj_k(AOK pk) {
  const qt_attn_oproj_args& p = pk.a;
  constexpr int NW = 8;
  constexpr bool BF = sizeof(WT) == 2;
  constexpr int E = BF ? 8 : 4, KT = 4 * E;
  constexpr int KS = NREP * D, KTS = KS / KT;  // o-proj K slice of one kv head, in k tiles
  // IC = cached keys per lane group per batch; 2 at NREP 4 (4 spilled asm-loaded registers to scratch before their
  // data landed -- tools/asm_audit.py)
  constexpr int LPK = D / 8, GPW = 64 / LPK, IC = NREP >= 4 ? 2 : 4, RW = sizeof(KV) * 8 / 4;
  constexpr int ALD = KS + 4 * (BF ? 2 : 1);  // 16 B pad per row
  typedef typename std::conditional<BF, bf16_t, float>::type AT;
  __shared__ float qs[NW * NREP][D];
  __shared__ float kn[NW][D], vn[NW][D];
  __shared__ __attribute__((aligned(16))) AT att[NW][ALD];
  __shared__ float red[NW][NT][16];
  const int R = p.R, nq = p.Hq, nk = p.Hkv, half = D / 2;
  const int CG = gridDim.x / R;
  const int cg = blockIdx.x % CG, r = blockIdx.x / CG;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lm = lane & 15, lk = lane >> 4;
  const int grp = lane / LPK, sub = lane % LPK;
  const int ntiles = (p.N + 15) / 16, ktiles = nq * D / KT;
  const bool head = w < nk;  // this wave owns kv head w

  // 1. every load of the prologue, issued in the order the phases need them -- this lane's q/k/v vector and its
  // norm / RoPE parameters (phase 2), the first batch of cached keys (phase 3), the o_proj weight fragments (phase 4),
  // the residual -- as inline-asm loads with counted waits: hipcc's own waits flush every outstanding load at each
  // loop preheader, which made the q/k norm wait for the o_proj weights (the largest and last-needed bytes).
  // Every wave issues the same loads (clamped head / row / column indices) so the counts hold in every wave.
  const int hw = head ? w : 0;
  const int kvpos = CPOS ? p.const_pos : p.kv_pos[r];
  const int start = CPOS ? 0 : p.row_start[r];
  const int pos = CPOS ? p.const_pos : p.rope_pos[r];
  const int nc = kvpos - start;  // cached keys [start, kvpos); the new key (kvpos) comes from LDS
  const int nvec = nq + 2 * nk;  // host-checked: nvec <= NW * GPW (one vector per lane group)
  const int e0 = sub * 8, ec = e0 % half;
  const int hh = w * GPW + grp;
  const float* xsrc = p.qkv + (long long)r * nvec * D + (long long)min(hh, nvec - 1) * D + e0;
  u32x4_t xq[2], qwr[2], kwr[2], cvr[2], svr[2];
  {
    const float* qn = p.q_norm ? p.q_norm + e0 : xsrc;
    const float* kn_ = p.k_norm ? p.k_norm + e0 : xsrc;
    const float* cs = p.cos_tab + (long long)pos * half + ec;
    const float* sn = p.sin_tab + (long long)pos * half + ec;
    asm_ld16(xq[0], xsrc); asm_ld16(xq[1], xsrc + 4);
    asm_ld16(qwr[0], qn); asm_ld16(qwr[1], qn + 4);
    asm_ld16(kwr[0], kn_); asm_ld16(kwr[1], kn_ + 4);
    asm_ld16(cvr[0], cs); asm_ld16(cvr[1], cs + 4);
    asm_ld16(svr[0], sn); asm_ld16(svr[1], sn + 4);
  }
  constexpr int RQ = RW / 4;  // 16-byte loads per key row slice
  const long long kvbase = ((long long)r * nk + hw) * p.Lmax * D;
  u32x4_t kq[IC][RQ], vq[IC][RQ];
  auto kv_addr = [&](int j0, int c, bool isv) {
    const int jj = min(j0 + c * GPW + grp, max(nc - 1, 0));  // clamped (masked in the math)
    return (const KV*)(isv ? p.v_cache : p.k_cache) + kvbase + (long long)(start + jj) * D + sub * 8;
  };
#pragma unroll
  for (int c = 0; c < IC; ++c)
#pragma unroll
    for (int q4 = 0; q4 < RQ; ++q4) {
      asm_ld16(kq[c][q4], (const unsigned*)kv_addr(0, c, false) + 4 * q4);
      asm_ld16(vq[c][q4], (const unsigned*)kv_addr(0, c, true) + 4 * q4);
    }
  u32x4_t wv[NT][KTS];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const WT* wp = (const WT*)p.w_o + ((size_t)min(cg * NT + t, ntiles - 1) * ktiles + (size_t)hw * KTS) * 64 * E + lane * E;
#pragma unroll
    for (int kt = 0; kt < KTS; ++kt) asm_ld16(wv[t][kt], wp + (size_t)kt * 64 * E);
  }
  const int col = cg * NT * 16 + lane;
  unsigned xres_u;
  asm_ld4(xres_u, p.x + (long long)r * p.ldx + min(cg * NT * 16 + (lane % (NT * 16)), p.N - 1));
  constexpr int N_W = NT * KTS + 1;  // loads younger than the cached keys (weights + residual)
  constexpr int N_KV = 2 * IC * RQ;
  if (kProbe && pk.stop == 1) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    reg_fence(xres_u); reg_fence(kq[0][0]); reg_fence(wv[0][0]);
    if ((kq[0][0][0] ^ wv[0][0][0]) == 0x9E3779B9u && xres_u == 7u) p.x[0] = 0.f;
    return;
  }

  // 2. q/k RMSNorm + RoPE, v passthrough for the Hq + 2 Hkv vectors of row r: one vector per lane group (LPK lanes
  // x 8 elements), DPP row reductions, rotate-half partner by a DPP row rotation
  {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_KV + N_W) : "memory");
    reg_fence(xq[0]); reg_fence(xq[1]); reg_fence(qwr[0]); reg_fence(qwr[1]); reg_fence(kwr[0]); reg_fence(kwr[1]);
    reg_fence(cvr[0]); reg_fence(cvr[1]); reg_fence(svr[0]); reg_fence(svr[1]);
    const bool lo = e0 < half;
    float qw[8], kw[8], cv[8], sv[8], xv[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      qw[i] = __uint_as_float(qwr[0][i]); qw[i + 4] = __uint_as_float(qwr[1][i]);
      kw[i] = __uint_as_float(kwr[0][i]); kw[i + 4] = __uint_as_float(kwr[1][i]);
      cv[i] = __uint_as_float(cvr[0][i]); cv[i + 4] = __uint_as_float(cvr[1][i]);
      sv[i] = __uint_as_float(svr[0][i]); sv[i + 4] = __uint_as_float(svr[1][i]);
      xv[i] = __uint_as_float(xq[0][i]); xv[i + 4] = __uint_as_float(xq[1][i]);
    }
    const bool ok = hh < nvec;
    if (hh < nq + nk) {
      const bool isq = hh < nq;
      float ss = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) ss += xv[i] * xv[i];
      ss = group_sum_dpp<LPK>(ss);
      const float rs = rsqrtf(ss / (float)D + p.eps);
      if (isq ? p.q_norm != nullptr : p.k_norm != nullptr) {
#pragma unroll
        for (int i = 0; i < 8; ++i) xv[i] = (isq ? qw[i] : kw[i]) * (xv[i] * rs);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {  // q*cos + rotate_half(q)*sin
        const float pt = half_partner<LPK>(xv[i]);
        xv[i] = lo ? xv[i] * cv[i] - pt * sv[i] : xv[i] * cv[i] + pt * sv[i];
      }
    }
    if (ok) {
      if (hh < nq) {
#pragma unroll
        for (int i = 0; i < 8; ++i) qs[hh][e0 + i] = xv[i];
      } else {  // as the cache holds them (kv dtype rounding)
        const bool isk = hh < nq + nk;
        const int h = isk ? hh - nq : hh - nq - nk;
        KV kv8[8];
        float* dst = isk ? kn[h] : vn[h];
#pragma unroll
        for (int i = 0; i < 8; ++i) { kv8[i] = from_f<KV>(xv[i]); dst[e0 + i] = to_f(kv8[i]); }
        if (cg == 0) {
          KV* cache = (KV*)(isk ? p.k_cache : p.v_cache) + (((long long)r * nk + h) * p.Lmax + kvpos) * D + e0;
#pragma unroll
          for (int i = 0; i < 8; ++i) cache[i] = kv8[i];
        }
      }
    }
  }
  __syncthreads();
  if (kProbe && pk.stop == 2) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    reg_fence(kq[0][0]); reg_fence(wv[0][0]);
    if (qs[0][lane] == 1234.5f && kq[0][0][0] == 7u && wv[0][0][0] == 7u) p.x[0] = 0.f;
    return;
  }
  // the first batch of cached keys has landed (the cache stores of phase 2, if any, are younger: they only make
  // this count wait for a few weight fragments too)
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_W) : "memory");
#pragma unroll
  for (int c = 0; c < IC; ++c)
#pragma unroll
    for (int q4 = 0; q4 < RQ; ++q4) { reg_fence(kq[c][q4]); reg_fence(vq[c][q4]); }
  auto load_batch = [&](int j0) {  // later batches (> GPW * IC cached keys): compiler-tracked loads
#pragma unroll
    for (int c = 0; c < IC; ++c)
#pragma unroll
      for (int q4 = 0; q4 < RQ; ++q4) {
        kq[c][q4] = *((const u32x4_t*)kv_addr(j0, c, false) + q4);
        vq[c][q4] = *((const u32x4_t*)kv_addr(j0, c, true) + q4);
      }
  };

  // 3. attention of head w: lane group grp owns cached keys grp, grp + GPW, ...; the new key is folded into lane
  // group 0's state; groups merge through a common max + plain sums (VALU permlane butterflies)
  if (head) {
    const float scale = rsqrtf((float)D) * 1.4426950408889634f;  // scores in log2 units (exp2 softmax)
    float q[NREP][8], m[NREP], l[NREP], o[NREP][8];
#pragma unroll
    for (int j = 0; j < NREP; ++j) {
      m[j] = -INFINITY; l[j] = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) { q[j][i] = qs[w * NREP + j][sub * 8 + i] * scale; o[j][i] = 0.f; }
    }
    for (int j0 = 0; j0 < nc; j0 += GPW * IC) {
      if (j0 > 0) load_batch(j0);
      float vf[IC][8], dd[NREP][IC];
#pragma unroll
      for (int c = 0; c < IC; ++c) {
        const int jj = j0 + c * GPW + grp;
        float kf[8];
        if constexpr (sizeof(KV) == 2) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            kf[2 * i] = __uint_as_float(kq[c][0][i] << 16); kf[2 * i + 1] = __uint_as_float(kq[c][0][i] & 0xFFFF0000u);
            vf[c][2 * i] = __uint_as_float(vq[c][0][i] << 16); vf[c][2 * i + 1] = __uint_as_float(vq[c][0][i] & 0xFFFF0000u);
          }
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i) { kf[i] = __uint_as_float(kq[c][i >> 2][i & 3]); vf[c][i] = __uint_as_float(vq[c][i >> 2][i & 3]); }
        }
        if (jj >= nc) {  // masked key: weight exactly 0, keep 0 * v finite
#pragma unroll
          for (int i = 0; i < 8; ++i) vf[c][i] = 0.f;
        }
#pragma unroll
        for (int j = 0; j < NREP; ++j) {
          float d = 0.f;
#pragma unroll
          for (int i = 0; i < 8; ++i) d += q[j][i] * kf[i];
          d = group_sum_dpp<LPK>(d);
          dd[j][c] = jj < nc ? d : -INFINITY;
        }
      }
#pragma unroll
      for (int j = 0; j < NREP; ++j) {
        float mn = m[j];
#pragma unroll
        for (int c = 0; c < IC; ++c) mn = fmaxf(mn, dd[j][c]);
        if (mn == -INFINITY) continue;
        const float f = exp2_hw(m[j] - mn);
        float e[IC], es = 0.f;
#pragma unroll
        for (int c = 0; c < IC; ++c) { e[c] = exp2_hw(dd[j][c] - mn); es += e[c]; }
        l[j] = l[j] * f + es;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float acc = o[j][i] * f;
#pragma unroll
          for (int c = 0; c < IC; ++c) acc += e[c] * vf[c][i];
          o[j][i] = acc;
        }
        m[j] = mn;
      }
    }
    {  // the new key (LDS), lane group 0
      float kf[8], vv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) { kf[i] = kn[w][sub * 8 + i]; vv[i] = vn[w][sub * 8 + i]; }
#pragma unroll
      for (int j = 0; j < NREP; ++j) {
        float d = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) d += q[j][i] * kf[i];
        d = group_sum_dpp<LPK>(d);
        if (grp == 0) {
          const float mn = fmaxf(m[j], d);
          const float f = exp2_hw(m[j] - mn), e = exp2_hw(d - mn);
          l[j] = l[j] * f + e;
#pragma unroll
          for (int i = 0; i < 8; ++i) o[j][i] = o[j][i] * f + e * vv[i];
          m[j] = mn;
        }
      }
    }
    GroupMerge<LPK, NREP> gm;
    gm.run(m, l, o);
    gm.each(lane, [&](int j, int d, float ov, float lv, float) { att[w][j * D + d] = from_f<AT>(ov / lv); });
  }
  __syncthreads();
  if (kProbe && pk.stop == 3) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (to_f(att[w][lane]) == 1234.5f) p.x[0] = 0.f;
    return;
  }

  // 4. this head's partial o-proj product (row r = MFMA row 0; rows 1..15 are zero)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int kt = 0; kt < KTS; ++kt) reg_fence(wv[t][kt]);
  reg_fence(xres_u);
  const float xres = __uint_as_float(xres_u);
  if (head) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < KTS; ++kt) {
        if constexpr (BF) {
          u32x4_t av = {0u, 0u, 0u, 0u};
          if (lm == 0) av = *(const u32x4_t*)&att[w][kt * KT + lk * E];
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, av),
                                                        __builtin_bit_cast(bf16x8_t, wv[t][kt]), acc, 0, 0, 0);
        } else {
          const f32x4_t wf = __builtin_bit_cast(f32x4_t, wv[t][kt]);
#pragma unroll
          for (int s2 = 0; s2 < 4; ++s2)
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(lm == 0 ? att[w][kt * KT + lk * E + s2] : 0.f, wf[s2], acc, 0, 0, 0);
        }
      }
      if (lane < 16) red[w][t][lane] = acc[0];  // row 0, column lane
    }
  }
  __syncthreads();
  if (kProbe && pk.stop == 4) {
    if (red[0][0][lane & 15] == 1234.5f) p.x[0] = 0.f;
    return;
  }
  // 5. sum the head partials in head order, add the residual
  if (w == 0 && lane < NT * 16 && col < p.N) {
    float v = 0.f;
    for (int h = 0; h < nk; ++h) v += red[h][lane >> 4][lane & 15];
    p.x[(long long)r * p.ldx + col] = xres + v;
    if (p.x16) ((bf16_t*)p.x16)[(long long)r * p.ldx16 + col] = f2bf(xres + v);
  }
}

// Head-split form of the fused code-predictor attention + o_proj (header: qt_attn_oproj_args.ws).  Block = (column
// group cg of NC = 32 o_proj columns, kv head h), linear id h * CG + cg: with CG % 8 == 0 the 8 head blocks of one
// column group are dealt to one XCD under round-robin placement (speed only, never correctness).  Wave w = row w:
// q/k RMSNorm + RoPE of head h's NREP + 2 vectors (one per lane group), attention over the row's cached keys + the
// new key, the NREP x D output into row w of the block's LDS A tile.  Then head h's K-slice of o_proj for the 32
// columns and every row (NT x KTS MFMA fragments spread over the 8 waves, reduced in LDS in a fixed order).  Row r's
// partial goes to the block of head r as 32 {value, sequence tag} granules (8-byte agent-scope stores: write-through);
// that block polls the other heads' granules of its row, sums the nk partials in head order, adds the residual and
// stores the row (fp32 + the bf16 shadow).  Per-block intake: 16 KiB of weights + head h's K/V of every row + 4
// vectors per row, against the (column group, row) form's 128 KiB of weights + every head's K/V of one row (that form
// is bound by the CU's load intake).
// Sequence tags: granule (cg, p, r, c) carries the number of its producer's publications (the producer reads its own
// previous tag at kernel start); the consumer keeps its own count C[cg][r] and waits for C + 1.  Nothing is reset, so
// a write that arrives after a consumer gave up (bounded spin; sticky error flag ws[0]) is never taken for the next
// launch's.  Cache appends of the new k/v are issued last, after every counted load wait.
struct AOHS {
  qt_attn_oproj_args a;
  int spin_limit;
  int stop;  // measurement hook (QT_AO_STOP, as attn_oproj_k): end after phase 1..4 (before any hand-off); 0 = full
  int cg_log2;  // log2(column groups) when a power of two (block -> (head, group) by shifts), else -1
};

typedef __attribute__((ext_vector_type(2))) unsigned int u32x2_t;


QT_DEV u32x4_t ld_u32x4(const void* p) { return *(const u32x4_t*)p; }
QT_DEV unsigned ld_u32(const void* p) { return *(const unsigned*)p; }

QT_DEV size_t aohs_gran_off(int CG, int nk) { return 256 + ((size_t)CG * nk * 4 + 255) / 256 * 256; }

template <int D, int NREP>
__global__ __launch_bounds__(512) void attn_oproj_hs_k(AOHS pk) {
  const qt_attn_oproj_args& p = pk.a;
  constexpr int NW = 8, NT = 2, E = 8, KT = 32, NC = NT * 16;
  constexpr int KS = NREP * D, KTS = KS / KT, FPW = NT * KTS / NW, WPT = KTS / FPW;  // waves per column tile
  constexpr int LPK = D / 8, GPW = 64 / LPK, IC = 4;
  static_assert(FPW >= 1 && KTS % FPW == 0 && GPW >= NREP + 2, "head-split attn_oproj shape");
  constexpr int ALD = KS + 8;  // bf16 A-tile row stride (16 B pad)
  // q and the new key as bf16 pairs (the cache's format: v_dot2 scores), the new value as fp32
  __shared__ __attribute__((aligned(16))) unsigned qs2[NW][NREP][D / 2];
  __shared__ __attribute__((aligned(16))) unsigned kn2[NW][D / 2];
  __shared__ float vn[NW][D];
  __shared__ __attribute__((aligned(16))) bf16_t att[NW][ALD];
  __shared__ float red[NW][64][4];
  __shared__ float part[NW][NC];
  __shared__ float gath[8][NC];
  __shared__ int fail_sh;
  const int R = p.R, nq = p.Hq, nk = p.Hkv;
  const int lg = pk.cg_log2;  // (the runtime divisions cost ~60 scalar instructions ahead of the first load)
  const int CG = lg >= 0 ? 1 << lg : (int)gridDim.x / nk;
  const int h = lg >= 0 ? (int)blockIdx.x >> lg : (int)blockIdx.x / CG;
  const int cg = lg >= 0 ? (int)blockIdx.x & (CG - 1) : (int)blockIdx.x % CG;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lm = lane & 15, lk = lane >> 4;
  const int grp = lane / LPK, sub = lane % LPK;
  const int r = min(w, R - 1);  // this wave's row (waves past R repeat row R - 1 and publish nothing)
  const int kvpos = p.const_pos, nc = kvpos;  // cached keys [0, kvpos); the new key (kvpos) comes from LDS
  const int nvec = nq + 2 * nk, half = D / 2;
  const int e0 = sub * 8, ec = e0 % half;
  const int vsel = min(grp, NREP + 1);  // lane group -> q head h*NREP + grp, k head h, v head h
  const int hh = vsel < NREP ? h * NREP + vsel : (vsel == NREP ? nq + h : nq + nk + h);
  const float* xsrc = p.qkv + (long long)r * nvec * D + (long long)hh * D + e0;
  unsigned* cnt = (unsigned*)((char*)p.ws + 256);
  unsigned long long* gran = (unsigned long long*)((char*)p.ws + aohs_gran_off(CG, nk));
  const int ktiles = nq * D / KT;

  // 1. every load, in the order the phases need them.  Plain loads: hipcc's own counted waits retire them (inline-asm
  // loads + explicit waits let the register allocator copy a destination before its wait -- stale data,
  // nondeterministic results; tools/asm_load_hazards.py)
  u32x4_t xq[2], nwr[2], cvr[2], svr[2];
  {
    const float* nwp = vsel < NREP ? (p.q_norm ? p.q_norm + e0 : xsrc) : (p.k_norm ? p.k_norm + e0 : xsrc);
    const float* cs = p.cos_tab + (long long)kvpos * half + ec;
    const float* sn = p.sin_tab + (long long)kvpos * half + ec;
    xq[0] = ld_u32x4(xsrc); xq[1] = ld_u32x4(xsrc + 4);
    nwr[0] = ld_u32x4(nwp); nwr[1] = ld_u32x4(nwp + 4);
    cvr[0] = ld_u32x4(cs); cvr[1] = ld_u32x4(cs + 4);
    svr[0] = ld_u32x4(sn); svr[1] = ld_u32x4(sn + 4);
  }
  const long long kvbase = ((long long)r * nk + h) * p.Lmax * D;
  u32x4_t kq[IC], vq[IC];
  auto kv_addr = [&](int j0, int c, bool isv) {
    const int jj = min(j0 + c * GPW + grp, max(nc - 1, 0));  // clamped (masked in the math)
    return (const bf16_t*)(isv ? p.v_cache : p.k_cache) + kvbase + (long long)jj * D + sub * 8;
  };
#pragma unroll
  for (int c = 0; c < IC; ++c) { kq[c] = ld_u32x4(kv_addr(0, c, false)); vq[c] = ld_u32x4(kv_addr(0, c, true)); }
  const int f0 = w * FPW, tw = f0 / KTS, kt0 = f0 % KTS;
  u32x4_t wv[FPW];
  {
    const bf16_t* wp = (const bf16_t*)p.w_o + ((size_t)(cg * NT + tw) * ktiles + (size_t)h * KTS + kt0) * 64 * E +
                       lane * E;
#pragma unroll
    for (int i = 0; i < FPW; ++i) wv[i] = ld_u32x4(wp + (size_t)i * 64 * E);
  }
  // the granule this lane publishes (row w, column lane & 31): its previous tag
  const size_t my_g = ((size_t)(cg * nk + h) * 8 + w) * NC + (lane & (NC - 1));
  u32x2_t gprev;
  gprev = *(const u32x2_t*)(gran + my_g);
  // residual of the row this block finalises (row h) at this lane's column; this block's consumed count
  unsigned xres_u, cprev;
  xres_u = ld_u32(p.x + (long long)min(h, R - 1) * p.ldx + cg * NC + (lane & (NC - 1)));
  cprev = ld_u32(cnt + cg * nk + h);
  __builtin_amdgcn_sched_barrier(0);  // every load above is issued before any of the phases' math
  if (kProbe && pk.stop == 1) {
    if ((xq[0][0] ^ kq[0][0] ^ wv[0][0] ^ gprev[0] ^ xres_u ^ cprev) == 0x9E3779B9u) p.x[0] = 0.f;
    return;
  }

  // 2. q/k RMSNorm + RoPE of head h's vectors of row r (v passes through), into LDS
  {
    const bool lo = e0 < half;
    float nwv[8], cv[8], sv[8], xv[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      nwv[i] = __uint_as_float(nwr[0][i]); nwv[i + 4] = __uint_as_float(nwr[1][i]);
      cv[i] = __uint_as_float(cvr[0][i]); cv[i + 4] = __uint_as_float(cvr[1][i]);
      sv[i] = __uint_as_float(svr[0][i]); sv[i + 4] = __uint_as_float(svr[1][i]);
      xv[i] = __uint_as_float(xq[0][i]); xv[i + 4] = __uint_as_float(xq[1][i]);
    }
    {  // branch-free over the lane groups (the v group's result is discarded): a lane-divergent branch here made
       // hipcc sink the norm-weight / cos / sin loads into it, behind a wait for the first loads (two round trips)
      const bool isq = vsel < NREP, normed = vsel <= NREP;
      const bool has_w = isq ? p.q_norm != nullptr : p.k_norm != nullptr;
      float ss = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) ss += xv[i] * xv[i];
      ss = group_sum_dpp<LPK>(ss);
      const float rs = rsqrtf(ss / (float)D + p.eps);
      float y[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) y[i] = has_w ? nwv[i] * (xv[i] * rs) : xv[i];
#pragma unroll
      for (int i = 0; i < 8; ++i) {  // q*cos + rotate_half(q)*sin
        const float pt = half_partner<LPK>(y[i]);
        const float ro = lo ? y[i] * cv[i] - pt * sv[i] : y[i] * cv[i] + pt * sv[i];
        xv[i] = normed ? ro : xv[i];
      }
    }
    if (grp <= NREP) {  // q heads, the new key: bf16 pairs (dims 2i, 2i + 1 = low, high half)
      u32x4_t pk2;
#pragma unroll
      for (int i = 0; i < 4; ++i) pk2[i] = pack2bf_rne(xv[2 * i], xv[2 * i + 1]);
      *(u32x4_t*)(grp < NREP ? &qs2[w][grp][e0 / 2] : &kn2[w][e0 / 2]) = pk2;
    } else if (grp == NREP + 1) {  // the new value as the cache holds it (bf16 rounding)
#pragma unroll
      for (int i = 0; i < 8; ++i) vn[w][e0 + i] = bf2f(f2bf(xv[i]));
    }
  }
  __syncthreads();
  if (kProbe && pk.stop == 2) {
    if (qs2[w][0][lane] == 12345u && kq[0][0] == 7u && wv[0][0] == 7u) p.x[0] = 0.f;
    return;
  }
  // 3. attention of (row r, head h): lane group grp owns cached keys grp, grp + GPW, ...; the new key is folded into
  // lane group 0's state; groups merge through a common max + plain sums
  {
    // One batch of <= GPW * IC cached keys + the new key, no running state: scores by v_dot2 on bf16 pairs (q rounded
    // to bf16 as the reference's bf16 attention holds it), fp32 softmax per lane group, the weights rounded to bf16
    // pairs of keys (c, c + 1) and P.V as v_dot2 over key pairs of V (v_perm regroups the cache's dim pairs);
    // l sums the rounded weights.  The attention phase was VALU-bound (2 waves / SIMD, ~535 VALU per wave).
    const float scale = rsqrtf((float)D) * 1.4426950408889634f;  // scores in log2 units (exp2 softmax)
    u32x4_t q2[NREP];
#pragma unroll
    for (int j = 0; j < NREP; ++j) q2[j] = *(const u32x4_t*)&qs2[w][j][sub * 4];
    const u32x4_t k2n = *(const u32x4_t*)&kn2[w][sub * 4];
    auto dot8 = [](const u32x4_t& a, const u32x4_t& b) {
      float d = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        // (elements copied out first: a __builtin_bit_cast of a vector-element lvalue read element 0 every time)
        const unsigned ai = a[i], bi = b[i];
        d = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, ai), __builtin_bit_cast(bf16x2_t, bi), d, false);
      }
      return d;
    };
    float dd[NREP][IC], dn[NREP];
#pragma unroll
    for (int j = 0; j < NREP; ++j) {
      dn[j] = group_sum_dpp<LPK>(dot8(q2[j], k2n)) * scale;  // the new key (every lane group computes it)
#pragma unroll
      for (int c = 0; c < IC; ++c) {
        const float d = group_sum_dpp<LPK>(dot8(q2[j], kq[c])) * scale;
        dd[j][c] = c * GPW + grp < nc ? d : -INFINITY;  // masked keys read a clamped, finite cached key: weight 0
      }
    }
    // V regrouped to key pairs: vp[pr][i] = (v[2pr][2i], v[2pr + 1][2i]), vp[pr][4 + i] = (v[2pr][2i+1], v[2pr+1][2i+1])
    unsigned vp[IC / 2][8];
#pragma unroll
    for (int pr = 0; pr < IC / 2; ++pr)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        vp[pr][i] = __builtin_amdgcn_perm(vq[2 * pr + 1][i], vq[2 * pr][i], 0x05040100u);
        vp[pr][4 + i] = __builtin_amdgcn_perm(vq[2 * pr + 1][i], vq[2 * pr][i], 0x07060302u);
      }
    float vnf[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) vnf[i] = vn[w][sub * 8 + i];
    float m[NREP], l[NREP], o[NREP][8];
#pragma unroll
    for (int j = 0; j < NREP; ++j) {
      float mn = dn[j];
#pragma unroll
      for (int c = 0; c < IC; ++c) mn = fmaxf(mn, dd[j][c]);
      const float en = grp == 0 ? exp2_hw(dn[j] - mn) : 0.f;  // the new key counts once (lane group 0)
      unsigned ep[IC / 2];
#pragma unroll
      for (int pr = 0; pr < IC / 2; ++pr) {
        const float ea = exp2_hw(dd[j][2 * pr] - mn), eb = exp2_hw(dd[j][2 * pr + 1] - mn);
        ep[pr] = pack2bf_rne(ea, eb);
      }
      float ls = en;
#pragma unroll
      for (int pr = 0; pr < IC / 2; ++pr)
        ls = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, ep[pr]),
                                             __builtin_bit_cast(bf16x2_t, 0x3F803F80u), ls, false);
#pragma unroll
      for (int d = 0; d < 8; ++d) {
        float acc = en * vnf[d];
        const int vi = (d & 1) * 4 + (d >> 1);
#pragma unroll
        for (int pr = 0; pr < IC / 2; ++pr)
          acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, ep[pr]),
                                                __builtin_bit_cast(bf16x2_t, vp[pr][vi]), acc, false);
        o[j][d] = acc;
      }
      m[j] = mn; l[j] = ls;
    }
    GroupMerge<LPK, NREP> gm;
    gm.run(m, l, o);
    gm.each(lane, [&](int j, int d, float ov, float lv, float) { att[w][j * D + d] = f2bf(ov * __builtin_amdgcn_rcpf(lv)); });
  }
  __syncthreads();
  if (kProbe && pk.stop == 3) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (bf2f(att[w][lane]) == 1234.5f) p.x[0] = 0.f;
    return;
  }
  // 4. head h's K-slice of o_proj for the block's 32 columns: wave w multiplies fragments f0 .. f0 + FPW - 1 (column
  // tile tw); MFMA rows = batch rows (rows >= NW zero)
  {
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < FPW; ++i) {
      u32x4_t av = {0u, 0u, 0u, 0u};
      if (lm < NW) av = *(const u32x4_t*)&att[lm][(kt0 + i) * KT + lk * E];
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, av), __builtin_bit_cast(bf16x8_t, wv[i]),
                                                    acc, 0, 0, 0);
    }
    red[w][lane][0] = acc[0]; red[w][lane][1] = acc[1]; red[w][lane][2] = acc[2]; red[w][lane][3] = acc[3];
  }
  if (tid == 0) fail_sh = 0;
  __syncthreads();
  // 5. row w's partial (thread (w, c < NC)): the column tile's waves summed in wave order; publish it to the block of
  // head w (rows < R other than h), keep row h
  if (lane < NC) {
    const int c = lane, t = c >> 4, cc = c & 15;
    float v = 0.f;
#pragma unroll
    for (int q2 = 0; q2 < WPT; ++q2) v += red[t * WPT + q2][(w >> 2) * 16 + cc][w & 3];
    part[w][c] = v;
    if (kProbe && pk.stop == 4) {
      if (v == 1234.5f) p.x[0] = 0.f;
    } else if (w < R && w != h)
      __hip_atomic_store(gran + my_g, ((unsigned long long)(gprev[1] + 1u) << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  if (kProbe && pk.stop == 4) return;
  // 6. block of head h < R: the other heads' partials of row h, then the row
  if (h < R) {
    const unsigned want = cprev + 1u;
    if (tid < (nk - 1) * NC) {
      const int pi = tid / NC, c = tid % NC, pp = pi < h ? pi : pi + 1;
      const unsigned long long* src = gran + ((size_t)(cg * nk + pp) * 8 + h) * NC + c;
      unsigned long long g = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int spins = 0;
      while ((unsigned)(g >> 32) != want) {
        if (++spins > pk.spin_limit) { fail_sh = 1; break; }
        __builtin_amdgcn_s_sleep(1);
        g = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      gath[pp][c] = __uint_as_float((unsigned)g);
    }
    __syncthreads();
    if (tid < NC) {
      float v = 0.f;
      for (int pp = 0; pp < nk; ++pp) v += pp == h ? part[h][tid] : gath[pp][tid];
      const float y = __uint_as_float(xres_u) + v;
      const int col = cg * NC + tid;
      p.x[(long long)h * p.ldx + col] = y;
      if (p.x16) ((bf16_t*)p.x16)[(long long)h * p.ldx16 + col] = f2bf(y);
    }
    if (tid == 0) {
      cnt[cg * nk + h] = want;
      if (fail_sh) atomicOr((int*)p.ws, 1);
    }
  }
  // 7. the new k / v of (row w, head h) into the caches (one column group appends)
  if (cg == 0 && w < R && lane < D) {
    const long long o = (((long long)w * nk + h) * p.Lmax + kvpos) * D + lane;
    if (lane < D / 2) ((unsigned*)p.k_cache)[(o - lane) / 2 + lane] = kn2[w][lane];  // the bf16 pairs (row start even)
    ((bf16_t*)p.v_cache)[o] = f2bf(vn[w][lane]);
    if (lane + 64 < D) ((bf16_t*)p.v_cache)[o + 64] = f2bf(vn[w][lane + 64]);
  }
}

template <typename WT, int D, int NREP, bool CPOS>
int attn_oproj_go(const qt_attn_oproj_args& a, hipStream_t s) {
  constexpr int KT = sizeof(WT) == 2 ? 32 : 16;
  constexpr int NT = sizeof(WT) == 2 ? 2 : 1;  // column tiles per block (fp32: register budget)
  if constexpr ((NREP * D) % KT != 0 || (NREP * D) / KT > 16) {
    return QT_ERR_SHAPE;
  } else {
    static const int stop = qt_knob("QT_AO_STOP", 0);
    if (a.Hq + 2 * a.Hkv > 8 * (64 / (D / 8))) return QT_ERR_SHAPE;  // one q/k/v vector per lane group
    const int cgs = ((a.N + 15) / 16 + NT - 1) / NT;
    hipLaunchKernelGGL((attn_oproj_k<WT, WT, D, NREP, NT, CPOS>), dim3(cgs * a.R), dim3(512), 0, s, AOK{a, stop});
    return hipGetLastError() == hipSuccess ? 0 : QT_ERR_LAUNCH;
  }
}

template <typename WT, int D>
int attn_oproj_rep(const qt_attn_oproj_args& a, hipStream_t s) {
  const bool c = a.const_pos >= 0;
  switch (a.Hq / a.Hkv) {
    case 1: return c ? attn_oproj_go<WT, D, 1, true>(a, s) : attn_oproj_go<WT, D, 1, false>(a, s);
    case 2: return c ? attn_oproj_go<WT, D, 2, true>(a, s) : attn_oproj_go<WT, D, 2, false>(a, s);
    case 4: return c ? attn_oproj_go<WT, D, 4, true>(a, s) : attn_oproj_go<WT, D, 4, false>(a, s);
    default: return QT_ERR_SHAPE;
  }
}

template <typename KV, int D>
int small_prefill_dispatch(const qt_decode_attn_args& a, int T, hipStream_t s) {
  if (T != 2 || a.R % T) return QT_ERR_SHAPE;
  dim3 g(a.R / T, a.Hkv);
  switch (a.Hq / a.Hkv) {
    case 1: hipLaunchKernelGGL((attn_small_prefill_k<KV, D, 1, 2>), g, dim3(64 * 2 * 3), 0, s, a); break;
    case 2: hipLaunchKernelGGL((attn_small_prefill_k<KV, D, 2, 2>), g, dim3(64 * 2 * 4), 0, s, a); break;
    case 4: hipLaunchKernelGGL((attn_small_prefill_k<KV, D, 4, 2>), g, dim3(64 * 2 * 6), 0, s, a); break;
    default: return QT_ERR_SHAPE;
  }
  return hipGetLastError() == hipSuccess ? 0 : QT_ERR_LAUNCH;
}

template <typename KV, int D>
int decode_dispatch(const qt_decode_attn_args& a, hipStream_t s) {
  const int ns = a.nsplit > 1 ? a.nsplit : 1;
  if (ns > 8) return QT_ERR_ARG;
  if (ns > 1 && (!a.ws || a.ws_bytes < qt_decode_attn_ws_bytes(a.R, a.Hq, a.Hkv, a.D, ns))) return QT_ERR_ARG;
  if (ns > 1 && a.R * a.Hkv > 1024) return QT_ERR_SHAPE;  // arrival counters live in the 4 KiB header
  dim3 g(a.R, a.Hkv, ns);
  static const int nw_env = qt_knob("QT_ATTN_SHORT", -1);
  const bool short_cache = nw_env >= 0 ? nw_env != 0 : a.Lmax <= 64;  // 4 waves cover <= 64 keys in one pass
  switch (a.Hq / a.Hkv) {
    case 1:
      if (short_cache) hipLaunchKernelGGL((attn_decode_k<KV, D, 1, 4>), g, dim3(256), 0, s, a);
      else hipLaunchKernelGGL((attn_decode_k<KV, D, 1, 8>), g, dim3(512), 0, s, a);
      break;
    case 2:
      if (short_cache) hipLaunchKernelGGL((attn_decode_k<KV, D, 2, 4>), g, dim3(256), 0, s, a);
      else hipLaunchKernelGGL((attn_decode_k<KV, D, 2, 8>), g, dim3(512), 0, s, a);
      break;
    case 4: hipLaunchKernelGGL((attn_decode_k<KV, D, 4, 8>), g, dim3(512), 0, s, a); break;
    default: return QT_ERR_SHAPE;
  }
  return hipGetLastError() == hipSuccess ? 0 : QT_ERR_LAUNCH;
}

}  // namespace

extern "C" int qt_qkv_post(const qt_qkv_args* a, void* stream) {
  if (!a || a->D > 128 || (a->D & 1) || a->R <= 0) return QT_ERR_SHAPE;
  dim3 g(a->R, a->Hq + 2 * a->Hkv);
  hipStream_t s = (hipStream_t)stream;
  if (a->kv_dtype == QT_BF16) hipLaunchKernelGGL(qkv_post_k<bf16_t>, g, dim3(64), 0, s, *a);
  else if (a->kv_dtype == QT_F32) hipLaunchKernelGGL(qkv_post_k<float>, g, dim3(64), 0, s, *a);
  else return QT_ERR_DTYPE;
  return hipGetLastError() == hipSuccess ? 0 : QT_ERR_LAUNCH;
}

extern "C" int qt_attention(const qt_attn_args* a, void* stream) {
  if (!a || a->R <= 0 || a->Hkv <= 0 || a->Hq % a->Hkv || a->max_keys <= 0) return QT_ERR_SHAPE;
  const size_t sh = (size_t)((a->Hq / a->Hkv) * (a->max_keys + 4 * a->D)) * sizeof(float);
  if (sh > 160 * 1024 - 256) return QT_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  if (a->kv_dtype == QT_BF16 && a->o_dtype == QT_F32) return attn_dispatch<bf16_t, float>(*a, s);
  if (a->kv_dtype == QT_BF16 && a->o_dtype == QT_BF16) return attn_dispatch<bf16_t, bf16_t>(*a, s);
  if (a->kv_dtype == QT_F32 && a->o_dtype == QT_F32) return attn_dispatch<float, float>(*a, s);
  return QT_ERR_DTYPE;
}

extern "C" long long qt_decode_attn_ws_bytes(int R, int Hq, int Hkv, int D, int nsplit) {
  return 4096 + (long long)R * Hq * nsplit * (D + 2) * (long long)sizeof(float);
}

extern "C" int qt_decode_attention(const qt_decode_attn_args* a, void* stream) {
  if (!a || a->R <= 0 || a->Hkv <= 0 || a->Hq % a->Hkv) return QT_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  const bool bf = a->kv_dtype == QT_BF16;
  if (!bf && a->kv_dtype != QT_F32) return QT_ERR_DTYPE;
  if (a->o_dtype != QT_F32 && a->o_dtype != QT_BF16) return QT_ERR_DTYPE;
  switch (a->D) {
    case 16: return bf ? decode_dispatch<bf16_t, 16>(*a, s) : decode_dispatch<float, 16>(*a, s);
    case 64: return bf ? decode_dispatch<bf16_t, 64>(*a, s) : decode_dispatch<float, 64>(*a, s);
    case 128: return bf ? decode_dispatch<bf16_t, 128>(*a, s) : decode_dispatch<float, 128>(*a, s);
    default: return QT_ERR_SHAPE;
  }
}

// The head-split form's consumers spin on granules that other blocks of the SAME launch publish, so every block of the
// grid must be resident at once (HIP does not schedule a waiting block out).  Checked against the occupancy of this
// kernel on the current device (cached per device): a smaller GPU / compute partition takes the (column group, row)
// form instead, which has no in-launch hand-off.
static bool aohs_all_resident(int blocks) {
  static int cap[64];  // resident blocks per device, 0 = not queried yet
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
  if (cap[dev] == 0) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)attn_oproj_hs_k<128, 2>, 512, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return false;
    cap[dev] = std::max(1, per_cu * cus);
  }
  return blocks <= cap[dev];
}

extern "C" int qt_attn_oproj_resident_blocks() {
  int dev = 0, per_cu = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)attn_oproj_hs_k<128, 2>, 512, 0) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return -1;
  return per_cu * cus;
}

extern "C" long long qt_attn_oproj_ws_bytes(int N, int Hkv) {
  const long long cg = (N + 31) / 32;
  return 256 + (cg * Hkv * 4 + 255) / 256 * 256 + cg * Hkv * 8 * 32 * 8;
}

extern "C" int qt_decode_attn_oproj(const qt_attn_oproj_args* a, void* stream) {
  if (!a || a->R <= 0 || a->Hkv <= 0 || a->Hkv > 8 || a->Hq % a->Hkv || a->N <= 0 || a->Lmax <= 0) return QT_ERR_SHAPE;
  if (!a->qkv || !a->w_o || !a->x || !a->k_cache || !a->v_cache || !a->cos_tab || !a->sin_tab) return QT_ERR_ARG;
  if (a->const_pos < 0 && (!a->rope_pos || !a->kv_pos || !a->row_start)) return QT_ERR_ARG;
  if (a->w_dtype != a->kv_dtype || (a->w_dtype != QT_BF16 && a->w_dtype != QT_F32)) return QT_ERR_DTYPE;
  hipStream_t s = (hipStream_t)stream;
  const bool bf = a->w_dtype == QT_BF16;
  // head-split form: a workspace was given and the shape is the code predictor's (the caller decides by passing ws);
  // QT_AO_SPIN (probe builds) bounds each hand-off poll (iterations of ~1 us), never below 1000
  static const int spin = std::max(1000, qt_knob("QT_AO_SPIN", 200000));
  if (a->ws && bf && a->const_pos >= 0 && a->const_pos <= 16 && a->D == 128 && a->Hq == 2 * a->Hkv &&
      a->R <= 8 && a->R <= a->Hkv && a->N % 256 == 0 && a->const_pos < a->Lmax &&  // row r's sum: head r's block
      a->ws_bytes >= qt_attn_oproj_ws_bytes(a->N, a->Hkv) && aohs_all_resident((a->N / 32) * a->Hkv)) {
    static const int stop = qt_knob("QT_AO_STOP", 0);
    const int cgs = a->N / 32;
    const int lg = (cgs & (cgs - 1)) == 0 ? __builtin_ctz((unsigned)cgs) : -1;
    hipLaunchKernelGGL((attn_oproj_hs_k<128, 2>), dim3(cgs * a->Hkv), dim3(512), 0, s, AOHS{*a, spin, stop, lg});
    return hipGetLastError() == hipSuccess ? 0 : QT_ERR_LAUNCH;
  }
  switch (a->D) {
    case 16: return bf ? attn_oproj_rep<bf16_t, 16>(*a, s) : attn_oproj_rep<float, 16>(*a, s);
    case 64: return bf ? attn_oproj_rep<bf16_t, 64>(*a, s) : attn_oproj_rep<float, 64>(*a, s);
    case 128: return bf ? attn_oproj_rep<bf16_t, 128>(*a, s) : attn_oproj_rep<float, 128>(*a, s);
    default: return QT_ERR_SHAPE;
  }
}

extern "C" int qt_small_prefill_attention(const qt_decode_attn_args* a, int T, void* stream) {
  if (!a || a->R <= 0 || a->Hkv <= 0 || a->Hq % a->Hkv || a->Lmax < T) return QT_ERR_SHAPE;
  if (a->o_dtype != QT_F32 && a->o_dtype != QT_BF16) return QT_ERR_DTYPE;
  hipStream_t s = (hipStream_t)stream;
  const bool bf = a->kv_dtype == QT_BF16;
  if (!bf && a->kv_dtype != QT_F32) return QT_ERR_DTYPE;
  switch (a->D) {
    case 16: return bf ? small_prefill_dispatch<bf16_t, 16>(*a, T, s) : small_prefill_dispatch<float, 16>(*a, T, s);
    case 64: return bf ? small_prefill_dispatch<bf16_t, 64>(*a, T, s) : small_prefill_dispatch<float, 64>(*a, T, s);
    case 128: return bf ? small_prefill_dispatch<bf16_t, 128>(*a, T, s) : small_prefill_dispatch<float, 128>(*a, T, s);
    default: return QT_ERR_SHAPE;
  }
}
