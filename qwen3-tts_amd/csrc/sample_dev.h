// Logits processing + token selection (transformers 4.57 semantics) for one row on 256 threads (4 waves): the body of
// qt_sample's kernel (sample.hip), also run inside the code-predictor step engine (cp_engine.hip) by waves 0-3 of a
// workgroup whose other waves do not take part -- hence the barrier is a parameter: __syncthreads in the kernel; in the
// engine a block-wide __syncthreads too, which the non-sampling waves 4-7 pass in a loop until the sampler marks its
// last barrier in the double-buffered LDS word sb_st (cp_engine.hip, the fused sampler block).  Method notes:
// sample.hip's header.
#pragma once
#include "common.h"

namespace qt_sample_dev {

typedef __attribute__((ext_vector_type(4))) int i32x4_t;
constexpr int NT = 256;  // threads per row; PER = scores per thread (8 / 12 / 16 for V <= 2048 / 3072 / 4096)

QT_DEV unsigned mulhilo(unsigned a, unsigned b, unsigned* hi) {
  unsigned long long p = (unsigned long long)a * b;
  *hi = (unsigned)(p >> 32);
  return (unsigned)p;
}

QT_DEV float philox_uniform4(unsigned long long seed, unsigned c0, unsigned c1, unsigned c2, unsigned c3) {
  unsigned k0 = (unsigned)seed, k1 = (unsigned)(seed >> 32);
  unsigned x0 = c0, x1 = c1, x2 = c2, x3 = c3;
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
QT_DEV float philox_uniform(unsigned long long seed, unsigned c0, unsigned c1, unsigned c2) {
  return philox_uniform4(seed, c0, c1, c2, 0x9E3779B9u);
}

QT_DEV unsigned okey(float f) {  // order-preserving float -> uint
  unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
QT_DEV float okey_inv(unsigned k) { return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k); }

// One MSB-first 2-bit step of the k-th-largest-key search over N keys per lane, counts summed over the wave:
// extends the prefix t (count(keys >= t) = cur >= k) by the largest 2-bit digit that keeps >= k keys.
template <int N>
QT_DEV void kth_step(const unsigned* key, int k, int bit, unsigned& t, int& cur) {
  const unsigned c1 = t | (1u << bit), c2 = t | (2u << bit), c3 = t | (3u << bit);
  int n12 = 0, n3 = 0;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    n12 += (key[j] >= c1 ? 1 : 0) + (key[j] >= c2 ? 0x10000 : 0);
    n3 += key[j] >= c3 ? 1 : 0;
  }
  const int s12 = wave_sum_i(n12), t3 = wave_sum_i(n3);
  const int t1 = s12 & 0xFFFF, t2 = s12 >> 16;
  if (t3 >= k) { t = c3; cur = t3; }
  else if (t2 >= k) { t = c2; cur = t2; }
  else if (t1 >= k) { t = c1; cur = t1; }
}

// (best, index) max with lowest-index tie break against the DPP partner CTRL (row-local all-reduce steps)
template <int CTRL>
QT_DEV void argmax_dpp(float& best, int& bi) {
  const float ob = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(best), CTRL, 0xF, 0xF, false));
  const int oi = __builtin_amdgcn_update_dpp(0, bi, CTRL, 0xF, 0xF, false);
  if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
}

template <class BAR>
QT_DEV float block_max(float v, float* sh, int tid, BAR& bar) {
  v = wave_max(v);
  bar();
  if ((tid & 63) == 0) sh[tid >> 6] = v;
  bar();
  return fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
}

// the row's LDS working set
struct SampSh {
  float sh[8];
  int shi[4];
  int cnt3[2][2][4];
  unsigned cand[256];
  int ncand;
  unsigned shtk;
  float srt[4096];
  __attribute__((aligned(16))) unsigned ck_s[4][64];
  int ci_s[4][64], nc_s[4];
  __attribute__((aligned(16))) int gi_s[16];
  __attribute__((aligned(16))) float gb_s[16];
  unsigned tk_s;
  int hist_s[NT];  // value histogram of the histogram fast path (one bin per thread)
  float hl_s[2][64];
  int hli_s[2][64], hln_s[2], hb_s[2], htok_s;
  float wmx_s[4];
};

// Row r on threads tid = 0 .. 255: returns the chosen token (every thread; -1 after a probe stop) and writes tok_out /
// codes / seen / finished / the embedding rows as qt_sample does.
template <int PER, class BAR>
QT_DEV int sample_row(const qt_sample_args& p, int stop, int r, int tid, SampSh& S, BAR bar) {
  float* sh = S.sh;
  int* shi = S.shi;
  auto& cnt3 = S.cnt3;
  unsigned* cand = S.cand;
  int& ncand = S.ncand;
  unsigned& shtk = S.shtk;
  float* srt = S.srt;
  auto& ck_s = S.ck_s;
  auto& ci_s = S.ci_s;
  int* nc_s = S.nc_s;
  int* gi_s = S.gi_s;
  float* gb_s = S.gb_s;
  unsigned& tk_s = S.tk_s;
  int* hist_s = S.hist_s;
  auto& hl_s = S.hl_s;
  auto& hli_s = S.hli_s;
  int* hln_s = S.hln_s;
  int* hb_s = S.hb_s;
  int& htok_s = S.htok_s;
  float* wmx_s = S.wmx_s;
  const int lane = tid & 63, w = tid >> 6;
  const int V = p.V;
  const float* lg = p.logits + (long long)r * p.ld;
  // Every global load of the kernel's prologue is issued back to back before the first wait: scores at clamped
  // indices, the seen flags and the device counters through always-valid pointers (the logits row stands in
  // when an optional pointer is null), selected afterwards -- a per-element or per-pointer branch made the
  // compiler wait for each load in turn (one L2 round trip each).
  const bool pen = p.seen && p.rep_penalty != 1.0f;
  const unsigned char* sr = pen ? p.seen + (long long)r * V : (const unsigned char*)lg;
  const int* ngp = p.n_generated ? p.n_generated + r * p.ctr_stride : (const int*)lg;
  const int* stpp = p.step ? p.step + r * p.ctr_stride : (const int*)lg;
  const int* prp = p.philox_row ? p.philox_row + r : (const int*)lg;
  const unsigned char* fnp = p.finished ? p.finished + r : (const unsigned char*)lg;
  const unsigned long long* sdp = p.seed_ptr ? p.seed_ptr : (const unsigned long long*)lg;
  float s[PER];
  unsigned char sn[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) s[j] = lg[min(tid + j * NT, V - 1)];
#pragma unroll
  for (int j = 0; j < PER; ++j) sn[j] = sr[min(tid + j * NT, V - 1)];
  const int ngr = __hip_atomic_load(ngp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int str = __hip_atomic_load(stpp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int fnr = *fnp;
  const unsigned long long sdv = __hip_atomic_load(sdp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int prr = __hip_atomic_load(prp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int ngen = p.n_generated ? ngr : 1 << 30;
  const unsigned stp = p.step ? (unsigned)str : 0u;
  const int finv = p.finished ? fnr : 0;
  const unsigned long long seed = p.seed_ptr ? sdv : p.seed;
  const unsigned prow = p.philox_row ? (unsigned)prr : (unsigned)(p.row_base + r);  // Philox stream id
  const bool eos_mask = p.eos_id >= 0 && (ngen < p.min_new_tokens || p.ignore_eos);
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int v = tid + j * NT;
    float x = s[j];
    if (pen && sn[j]) x = x < 0.f ? x * p.rep_penalty : x / p.rep_penalty;
    if ((eos_mask && v == p.eos_id) || (v >= p.suppress_lo && v < p.suppress_hi && v != p.suppress_keep) || v >= V)
      x = -INFINITY;
    s[j] = x;
  }
  if (kProbe && stop == 1) {
    if (s[0] + s[PER - 1] == 1234.5f) p.tok_out[r] = 0;
    return -1;
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
    bar();
    best = sh[0]; bi = shi[0];
    for (int i = 1; i < 4; ++i)
      if (sh[i] > best || (sh[i] == best && shi[i] < bi)) { best = sh[i]; bi = shi[i]; }
    tok = bi;
  } else {
    const float invT = (p.temperature > 0.f && p.temperature != 1.0f) ? 1.0f / p.temperature : 1.0f;
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < PER; ++j) { s[j] *= invT; mx = fmaxf(mx, s[j]); }
    unsigned key[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) key[j] = (tid + j * NT < V) ? okey(s[j]) : 0u;  // 0 = no token
    // Fast top-k (k <= 64, no top-p): the global top-k set lies inside the union of the four waves' own top-k sets.
    // (1) each wave narrows its keys to <= 64 candidates >= a prefix of its k-th largest key (wave sums only, no
    // barrier) and compacts them into LDS; (2) wave 0 finds the exact k-th largest key among the <= 256 candidates
    // (ties kept, TopKLogitsWarper) while every thread draws the Gumbel key of one candidate; (3) the draw is a
    // Gumbel-max over the kept ones: token = argmax (s_i + G_i), G_i = -log(-log(u_i)), u_i from Philox(seed,
    // step, substep, row, token) -- an exact sample of softmax(s / T) restricted to the top-k set.  A wave left
    // with > 64 tied keys falls back to the block search.
    bool fast = false;
    const bool fast_ok = p.top_k > 0 && p.top_k < V && p.top_k <= 64 && p.top_p >= 1.0f;
    // Histogram fast path (k <= 64, no top-p; p.algo 0 or 2): the k-th largest score located by a 256-bin value
    // histogram below the row maximum (bin = floor((max - s) * HB), HB bins per unit of s / T), then resolved exactly
    // among the boundary bin's scores; kept = {s >= k-th largest} (ties kept, TopKLogitsWarper).  Wave 0 then draws
    // the Gumbel-max over the kept set with the per-wave path's Philox stream (same token for the same kept set).
    // Falls through to the per-wave path when the top k span more than 256 / HB below the max or the boundary bin
    // holds more than 64 scores.  5 block barriers in all.
    if (fast_ok && p.algo != 1) {
      constexpr float HB = 16.f;
      hist_s[tid] = 0;
      const float wm = wave_max(mx);
      if (lane == 0) wmx_s[w] = wm;
      if (tid < 2) hln_s[tid] = 0;
      bar();
      const float M = fmaxf(fmaxf(wmx_s[0], wmx_s[1]), fmaxf(wmx_s[2], wmx_s[3]));
      int bin[PER];
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const float d = (M - s[j]) * HB;  // >= 0; -inf scores give +inf
        bin[j] = (tid + j * NT < V && d < (float)NT) ? (int)d : NT;
        if (bin[j] < NT) atomicAdd(&hist_s[bin[j]], 1);
      }
      bar();
      if (w == 0) {  // first bin (from the top) where the running count reaches k: scan of 4 bins per lane
        int h[4], loc = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) { h[i] = hist_s[lane * 4 + i]; loc += h[i]; }
        int scan = loc;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int y = __shfl_up(scan, o, 64);
          if (lane >= o) scan += y;
        }
        const int excl = scan - loc;
        const bool cross = excl < p.top_k && scan >= p.top_k;
        if (cross) {
          int c = excl, b = -1;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (b < 0) {
              if (c + h[i] >= p.top_k) b = lane * 4 + i;
              else c += h[i];
            }
          }
          hb_s[0] = b; hb_s[1] = c;  // boundary bin, scores strictly above it
        }
        if (lane == 63 && scan < p.top_k) hb_s[0] = -1;  // the top k reach below the histogram: fall through
      }
      bar();
      const int bs = hb_s[0];
      if (bs >= 0) {
#pragma unroll
        for (int j = 0; j < PER; ++j) {  // list 0: scores above the boundary bin (all kept); list 1: the bin's scores
          if (bin[j] <= bs) {
            const int l = bin[j] < bs ? 0 : 1;
            const int pos = atomicAdd(&hln_s[l], 1);
            if (pos < 64) { hl_s[l][pos] = s[j]; hli_s[l][pos] = tid + j * NT; }
          }
        }
      }
      bar();
      if (bs >= 0 && hln_s[1] <= 64) {
        fast = true;
        if (w == 0) {
          const int n0 = hln_s[0], n1 = hln_s[1], need = p.top_k - hb_s[1];  // 1 <= need <= n1
          const float mine = lane < n1 ? hl_s[1][lane] : -INFINITY;
          int gt = 0, ge = 0;
          for (int i = 0; i < n1; ++i) {
            const float o = hl_s[1][i];
            gt += o > mine ? 1 : 0;
            ge += o >= mine ? 1 : 0;
          }
          // v_k: the need-th largest boundary score (every lane whose rank window covers `need` holds that value)
          const unsigned long long kb = __ballot(lane < n1 && gt < need && need <= ge);
          const float vk = __shfl(mine, kb ? __ffsll((long long)kb) - 1 : 0, 64);
          float best = -INFINITY;
          int bi = 0x7fffffff;
          auto draw = [&](float sc, int ti) {
            const float u = philox_uniform4(seed, stp, (unsigned)p.substep, prow, (unsigned)ti);
            const float g = okey_inv(okey(sc)) - __logf(-__logf(u));
            if (g > best || (g == best && ti < bi)) { best = g; bi = ti; }
          };
          if (lane < n0) draw(hl_s[0][lane], hli_s[0][lane]);
          if (lane < n1 && mine >= vk) draw(mine, hli_s[1][lane]);
          argmax_dpp<0xB1>(best, bi);
          argmax_dpp<0x4E>(best, bi);
          argmax_dpp<0x141>(best, bi);
          argmax_dpp<0x140>(best, bi);
#pragma unroll
          for (int rr = 16; rr < 64; rr += 16) {
            const float ob = __shfl(best, rr, 64);
            const int oi = __shfl(bi, rr, 64);
            if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
          }
          if (lane == 0) htok_s = bi == 0x7fffffff ? 0 : bi;
        }
        bar();
        tok = htok_s;
      }
    }
    if (fast_ok && !fast) {
      int nv = 0;
#pragma unroll
      for (int j = 0; j < PER; ++j) nv += key[j] != 0u;
      int cw = wave_sum_i(nv);
      unsigned tw = 0u;
      for (int bit = 30; bit >= 0 && cw > 64; bit -= 2) kth_step<PER>(key, p.top_k, bit, tw, cw);
      int base = 0;
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const bool c = key[j] != 0u && key[j] >= tw;
        const unsigned long long m = __ballot(c);
        const int pos = base + __popcll(m & ((1ull << lane) - 1ull));
        if (c && pos < 64) { ck_s[w][pos] = key[j]; ci_s[w][pos] = tid + j * NT; }
        base += __popcll(m);
      }
      if (lane == 0) nc_s[w] = base;
      if (kProbe && stop == 6) {
        if (lane == 0 && base == 12345) p.tok_out[r] = 0;
        return -1;
      }
      bar();
      fast = nc_s[0] <= 64 && nc_s[1] <= 64 && nc_s[2] <= 64 && nc_s[3] <= 64;
      if (fast) {
        // wave 0: exact k-th largest key among the <= 256 candidates (4 per lane, 2-bit MSB-first steps with
        // wave sums, stop at exactly k); meanwhile every thread draws the Gumbel key of candidate (w, lane)
        if (w == 0) {
          unsigned ck[4];
          int tot = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int ni = nc_s[i];
            ck[i] = lane < ni ? ck_s[i][lane] : 0u;
            tot += ni;
          }
          unsigned t = 0u;
          int cur = tot;
          for (int bit = 30; bit >= 0 && cur > p.top_k; bit -= 2) kth_step<4>(ck, p.top_k, bit, t, cur);
          if (lane == 0) tk_s = t;
        }
        const bool has = lane < nc_s[w];
        const unsigned mk = has ? ck_s[w][lane] : 0u;
        const int mi = has ? ci_s[w][lane] : 0x7fffffff;
        float g = -INFINITY;
        if (has && mk > okey(-INFINITY)) {  // masked (-inf) scores are never drawn
          const float u = philox_uniform4(seed, stp, (unsigned)p.substep, prow, (unsigned)mi);
          g = okey_inv(mk) - __logf(-__logf(u));
        }
        bar();
        if (kProbe && stop == 7) {
          if (g == 1.5f && tk_s == 12345u) p.tok_out[r] = 0;
          return -1;
        }
        // Gumbel-max over the kept set (key >= k-th largest: ties kept): DPP argmax in rows, then across rows/waves
        float best = (has && mk >= tk_s) ? g : -INFINITY;
        int bi = best > -INFINITY ? mi : 0x7fffffff;
        argmax_dpp<0xB1>(best, bi);
        argmax_dpp<0x4E>(best, bi);
        argmax_dpp<0x141>(best, bi);
        argmax_dpp<0x140>(best, bi);
        if ((lane & 15) == 0) { gb_s[w * 4 + (lane >> 4)] = best; gi_s[w * 4 + (lane >> 4)] = bi; }
        bar();
        f32x4_t gb[4];  // all 16 row results in flight at once (8 x 16-byte LDS reads, one wait)
        i32x4_t gi[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) { gb[i] = ((const f32x4_t*)gb_s)[i]; gi[i] = ((const i32x4_t*)gi_s)[i]; }
        best = gb[0][0];
        bi = gi[0][0];
#pragma unroll
        for (int i = 1; i < 16; ++i)
          if (gb[i >> 2][i & 3] > best || (gb[i >> 2][i & 3] == best && gi[i >> 2][i & 3] < bi)) {
            best = gb[i >> 2][i & 3];
            bi = gi[i >> 2][i & 3];
          }
        tok = bi == 0x7fffffff ? 0 : bi;
      }
    }
    unsigned tk = 0;  // keep keys >= tk
    if (!fast) mx = block_max(mx, sh, tid, bar);
    if (kProbe && stop == 2) {
      if (mx == 1234.5f) p.tok_out[r] = 0;
      return -1;
    }
    if (!fast && p.top_k > 0 && p.top_k < V) {
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
        bar();
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
        bar();
#pragma unroll
        for (int j = 0; j < PER; ++j)
          if (tid + j * NT < V && key[j] >= tk) cand[atomicAdd(&ncand, 1)] = key[j];
        bar();
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
        bar();
        tk = shtk;
      }
    }
    if (kProbe && stop == 3) {
      if (tk == 12345u) p.tok_out[r] = 0;
      return -1;
    }
    if (!fast) {
    if (p.top_p < 1.0f) {  // rare path: sorted list (descending) for the nucleus cut
      for (int j = 0; j < PER; ++j) {
        const int v = tid + j * NT;
        if (v < 4096) srt[v] = (v < V && okey(s[j]) >= tk) ? s[j] : -INFINITY;
      }
      int P2 = 1;
      while (P2 < V) P2 <<= 1;
      for (int v = PER * NT + tid; v < P2; v += NT) srt[v] = -INFINITY;  // slots beyond this PER's reach
      bar();
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
          bar();
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
      bar();
      tk = max(tk, okey(sh[4]));
    }
    float e[PER], mass = 0.f;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      e[j] = (tid + j * NT < V && okey(s[j]) >= tk && s[j] > -INFINITY) ? __expf(s[j] - mx) : 0.f;
      mass += e[j];
    }
    // inclusive prefix of per-thread masses (wave scan + wave offsets).  Every bound is formed as off + scan, so
    // thread t's exclusive bound is bit-identical to thread t-1's inclusive one (float + is commutative: across a
    // wave edge both are sh[0] + ... + sh[w-1] in the same order) and the last thread's inclusive bound is
    // `total`: the intervals [excl, inc) tile [0, total) with no gaps.
    float scan = mass;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      float y = __shfl_up(scan, o, 64);
      if (lane >= o) scan += y;
    }
    float prev = __shfl_up(scan, 1, 64);
    bar();
    if (lane == 63) sh[w] = scan;
    bar();
    float off = 0.f;
    for (int i = 0; i < w; ++i) off += sh[i];
    const float total = ((sh[0] + sh[1]) + sh[2]) + sh[3];
    const float inc = scan + off;
    const float excl = lane == 0 ? off : prev + off;
    if (kProbe && stop == 4) {
      if (inc == 1234.5f) p.tok_out[r] = 0;
      return -1;
    }
    const float uu = p.debug_u >= 0.f ? p.debug_u : philox_uniform(seed, stp, (unsigned)p.substep, prow);
    const float u = uu * total;  // may round up to `total` itself
    if (tid == 0) shi[0] = -1;
    bar();
    // the interval holding u claims the draw; u >= total (rounding) goes to the last thread with mass, whose
    // inclusive bound equals total (the threads after it add exact zeros)
    if (mass > 0.f && u >= excl && (u < inc || inc >= total)) {
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
    bar();
    tok = shi[0];
    if (tok < 0) {  // no positive mass survived (cannot happen with finite scores): argmax of the kept set
      float best = -INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const int v = tid + j * NT;
        if (v < V && okey(s[j]) >= tk && (s[j] > best || (s[j] == best && v < bi))) { best = s[j]; bi = v; }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        float ob = __shfl_xor(best, o, 64);
        int oi = __shfl_xor(bi, o, 64);
        if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
      }
      bar();
      if (lane == 0) { sh[w] = best; shi[w] = bi; }
      bar();
      best = sh[0]; bi = shi[0];
      for (int i = 1; i < 4; ++i)
        if (sh[i] > best || (sh[i] == best && shi[i] < bi)) { best = sh[i]; bi = shi[i]; }
      tok = bi == 0x7fffffff ? 0 : bi;
    }
    }  // !fast
  }
  if (finv) tok = p.eos_id;
  if (p.force) {  // teacher forcing: record this path's choice, continue with the forced token
    const long long off = (long long)r * p.codes_ld + (long long)((int)stp + p.codes_step_off) * p.codes_w + p.codes_col;
    if (tid == 0) p.pick[off] = tok;
    tok = p.force[off];
  }
  if (kProbe && stop == 5) {
    if (tid == 0) p.tok_out[r] = tok;
    return -1;
  }
  if (p.emb_table) {  // next-step input row: the chosen token's (projected) embedding (+ its layer-0 q/k/v row)
    const float* src = p.emb_table + (long long)tok * p.emb_dim;
    float* dst = p.emb_out + (long long)r * p.emb_ld;
    bf16_t* d16 = p.emb_out16 ? (bf16_t*)p.emb_out16 + (long long)r * p.emb_ld16 : nullptr;
    // every load of a pass is issued before its stores, at clamped addresses (a branch around a load makes hipcc
    // wait for it right away); without a second table its loads re-read the first table's row
    const bool two = p.emb2_table != nullptr;
    const float* src2 = two ? p.emb2_table + (long long)tok * p.emb2_dim : src;
    const int lim2 = (two ? p.emb2_dim : p.emb_dim) - 4;
    float* dst2 = two ? p.emb2_out + (long long)r * p.emb2_ld : nullptr;
    constexpr int G2 = 4;  // second-table float4s per thread per pass
    for (int i = tid * 4, i2 = tid * 4; i < p.emb_dim || (two && i2 < p.emb2_dim); i += NT * 4, i2 += NT * 4 * G2) {
      f32x4_t v2[G2];
      const f32x4_t v = *(const f32x4_t*)(src + min(i, p.emb_dim - 4));
#pragma unroll
      for (int j = 0; j < G2; ++j) v2[j] = *(const f32x4_t*)(src2 + min(i2 + j * NT * 4, lim2));
      if (i < p.emb_dim) {
        *(f32x4_t*)(dst + i) = v;
        if (d16) *(uint2*)(d16 + i) = uint2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
      }
      if (two) {
#pragma unroll
        for (int j = 0; j < G2; ++j)
          if (i2 + j * NT * 4 < p.emb2_dim) *(f32x4_t*)(dst2 + i2 + j * NT * 4) = v2[j];
      }
    }
  }
  if (tid != 0) return tok;
  p.tok_out[r] = tok;
  if (p.codes) {
    const int st = (int)stp + p.codes_step_off;
    p.codes[(long long)r * p.codes_ld + (long long)st * p.codes_w + p.codes_col] = tok;
  }
  if (p.seen) p.seen[(long long)r * V + tok] = 1;
  if (p.finished && p.eos_id >= 0 && tok == p.eos_id) p.finished[r] = 1;
  return tok;
}

}  // namespace qt_sample_dev
