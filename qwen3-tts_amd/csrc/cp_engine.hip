// Code-predictor decode-step engine for gfx950: ONE persistent launch runs a whole code-predictor decode step -- the
// 5 decoder layers (q/k/v projection -> q/k RMSNorm + RoPE + attention + o_proj + residual -> gate/up + SwiGLU ->
// down + residual) and the final norm + lm_head[g] -- for up to 8 batch rows, where the launch chain issued ~21
// dependent kernels per step.  Replaces M:1250-1312 (Qwen3TTSTalkerCodePredictorModel.forward for one
// generated token, decoder layers M:961-1012, attention M:740-804 with q/k norm M:764-765) and M:1299 (lm_head[g]) for
// every decode step of the code predictor (M:1671-1680); the token choice stays qt_sample.
//
// Structure (256 workgroups x 8 waves, one per CU, all resident -- the host checks the occupancy):
//  * The residual stream is distributed: block (h, cg) OWNS x[rows 2q, 2q+1][cols 16t .. 16t+16) with t = 2cg + h/4,
//    q = h % 4, in LDS, for the whole launch.  Only bf16 copies of x (the next GEMV's A operand) cross blocks.
//  * Hand-offs are 8-byte {value, tag} granules written by one agent-scope (write-through) store each; the consumer
//    re-reads a granule until its tag is this launch's edge tag (no flags, no fences, no resets: tag = epoch * 32 +
//    edge + 1, the epoch a launch counter in the workspace, advanced by block 0 at the end of every launch once every
//    block has read it).  Every all-to-all edge orders the buffer reuse of the next layer.
//  * Every weight fragment a block multiplies in phase k + 1 is loaded into registers right after its phase-k MFMAs,
//    before phase k's outputs are published and the edge into phase k + 1 is polled: the weight latency (Infinity
//    Cache) overlaps the hand-off.
// Per layer: P1 q/k/v tile (h, cg) -> [QKV edge: the 32 blocks of head h] -> P2 head h's attention (every row) and its
// K-slice of o_proj for 32 columns -> [partial edge: the 8 head blocks of a column group] -> residual add by the
// owner -> [x16 edge, all-to-all] -> P3 gate/up tiles + SwiGLU -> [h edge: each owner's 2 rows] -> P4 down tile t
// for the owner's 2 rows + residual -> [x16 edge] -> next layer (or the lm_head).  Numerics follow the launch chain:
// bf16 weights and MFMA operands, fp32 accumulation, RMSNorm from the bf16 shadow's values, fp32 q/k/v, the attention
// of attn_oproj_hs_k (q and keys as bf16 pairs, fp32 softmax), SwiGLU / attention outputs rounded to bf16.
#include "common.h"
#include "attn_dev.h"
#include <algorithm>

namespace {

typedef unsigned long long u64;

constexpr int H = 1024, I = 3072, D = 128, NQ = 16, NKV = 8, NREP = 2, QKVW = (NQ + 2 * NKV) * D;
constexpr int NB = 256, NT = 512, NW = 8, MAXR = 8;
constexpr int KTH = H / 32, KTI = I / 32, KTO = NQ * D / 32;  // k tiles: 32 / 96 / 64
constexpr int LPK = D / 8, GPW = 64 / LPK, IC = 4;              // attention lane groups (attn_oproj_hs_k)
constexpr int XLD = H + 8, HLD = I + 8, ALD = NREP * D + 8;       // LDS row strides (bf16)
constexpr int NEDGE = 32;                                         // tag slots per launch (5 per layer)

// workspace layout (bytes)
constexpr size_t OFF_ERR = 0, OFF_EPOCH = 4;
constexpr size_t OFF_QKV = 256;                                       // [NKV][MAXR][512] granules
constexpr size_t OFF_PART = OFF_QKV + (size_t)NKV * MAXR * 512 * 8;   // [64 t][4 q][NKV][32]
constexpr size_t OFF_X16 = OFF_PART + (size_t)64 * 4 * NKV * 32 * 8;  // [2][MAXR][H/2]
constexpr size_t OFF_H = OFF_X16 + (size_t)2 * MAXR * (H / 2) * 8;    // [MAXR][I/2]
constexpr size_t WS_BYTES = OFF_H + (size_t)MAXR * (I / 2) * 8;
// optional intermediates of layer 0 (a workspace this much larger records them; parity diagnostics): [4][MAXR][4096]
// fp32 = x after the attention residual, the SwiGLU output, x after the MLP residual, the attention output
constexpr size_t DBG_BYTES = (size_t)4 * MAXR * 4096 * 4;

struct CEP {
  qt_cp_step_args a;
  int spin;
};

QT_DEV u64 ld_g(const u64* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
QT_DEV void st_g(u64* p, unsigned v, unsigned tag) {
  __hip_atomic_store(p, ((u64)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
QT_DEV f32x4_t mfma(u32x4_t a, u32x4_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c, 0,
                                                 0, 0);
}
QT_DEV u32x4_t ldw(const void* p) { return *(const u32x4_t*)p; }
// weight fragment (n tile, k tile) of a pre-tiled bf16 matrix with `kt` k tiles: 1 KiB, lane l's 16 bytes
QT_DEV const bf16_t* frag(const void* w, int nt, int ktile, int kt, int lane) {
  return (const bf16_t*)w + ((size_t)nt * kt + ktile) * 512 + lane * 8;
}
// keep a loaded register alive and unmoved: the loads above are issued here, not sunk to their first use
#define CE_ISSUED() asm volatile("" ::: "memory")

// Re-read N consecutive granules until each carries `tag` (bounded; a give-up sets the sticky error flag and keeps
// whatever was read).  Values are returned in v.
template <int N>
QT_DEV void poll_run(const u64* g, unsigned tag, unsigned (&v)[N], int spin, int* err) {
  u64 x[N];
#pragma unroll
  for (int k = 0; k < N; ++k) x[k] = ld_g(g + k);
  int spins = 0;
  while (true) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < N; ++k) ok = ok && (unsigned)(x[k] >> 32) == tag;
    if (ok) break;
    if (++spins > spin) { atomicOr(err, 1); break; }
    __builtin_amdgcn_s_sleep(1);
#pragma unroll
    for (int k = 0; k < N; ++k)
      if ((unsigned)(x[k] >> 32) != tag) x[k] = ld_g(g + k);
  }
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] = (unsigned)x[k];
}

struct Lds {
  union {
    bf16_t xa[MAXR][XLD];  // x16 rows (all), the A operand of q/k/v, gate/up, lm_head
    bf16_t ha[2][HLD];     // the owner's two SwiGLU rows, the A operand of down
  } a;
  float red[NW][64][4];                                   // per-wave MFMA partials
  float rs[MAXR];                                         // 1 / rms per row
  float rsp[NW];
  float xown[2][16];                                      // the owned residual slice
  float gath[NKV][32];                                    // the 8 head partials of the owned slice
  unsigned hsw[2][MAXR][8];                               // SwiGLU outputs of the block's tiles (bf16 pairs)
  __attribute__((aligned(16))) unsigned qs2[NW][NREP][D / 2];  // attention: q as bf16 pairs
  __attribute__((aligned(16))) unsigned kn2[NW][D / 2];        // the new key as bf16 pairs
  float vn[NW][D];                                             // the new value (bf16-rounded)
  __attribute__((aligned(16))) bf16_t att[NW][ALD];            // head h's attention output per row
};

// Stage the x16 edge (all rows, tag) into lds.a.xa and each row's 1 / rms (from the bf16 values, as the decode GEMV
// computes it from the bf16 shadow).  Thread -> row tid / 64, pairs (tid % 64) * 8 .. + 8.
QT_DEV void stage_x16(Lds& s, const u64* gx, unsigned tag, int R, float eps, int spin, int* err) {
  const int tid = threadIdx.x, row = tid >> 6, p0 = (tid & 63) * 8;
  unsigned v[8];
  if (row < R) {
    poll_run<8>(gx + (size_t)row * (H / 2) + p0, tag, v, spin, err);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = 0u;
  }
  *(u32x4_t*)&s.a.xa[row][2 * p0] = u32x4_t{v[0], v[1], v[2], v[3]};
  *(u32x4_t*)&s.a.xa[row][2 * p0 + 8] = u32x4_t{v[4], v[5], v[6], v[7]};
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float lo = __uint_as_float(v[k] << 16), hi = __uint_as_float(v[k] & 0xFFFF0000u);
    ss += lo * lo + hi * hi;
  }
  ss = wave_sum_dpp(ss);  // wave == row
  if ((tid & 63) == 0) s.rs[row] = rsqrtf(ss / (float)H + eps);
  __syncthreads();
}

// A fragment of MFMA row lm (batch row; rows >= R zero) at k tile kt from the staged x16 rows
QT_DEV u32x4_t afrag_x(const Lds& s, int lm, int lk, int kt, int R) {
  return lm < R ? *(const u32x4_t*)&s.a.xa[lm][kt * 32 + lk * 8] : u32x4_t{0u, 0u, 0u, 0u};
}

// Sum the per-wave partials of waves [w0, w0 + nw) for lane `lane` (fixed wave order)
QT_DEV f32x4_t red_sum(const Lds& s, int w0, int nw, int lane) {
  f32x4_t v = {0.f, 0.f, 0.f, 0.f};
  for (int ww = w0; ww < w0 + nw; ++ww) {
    v[0] += s.red[ww][lane][0]; v[1] += s.red[ww][lane][1]; v[2] += s.red[ww][lane][2]; v[3] += s.red[ww][lane][3];
  }
  return v;
}

__global__ __launch_bounds__(NT) void cp_step_k(CEP pk) {
  const qt_cp_step_args& p = pk.a;
  __shared__ Lds s;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lm = lane & 15, lk = lane >> 4;
  const int b = blockIdx.x, h = b >> 5, cg = b & 31;
  const int to = 2 * cg + (h >> 2), qo = h & 3;  // the owned residual slice: rows 2qo, 2qo + 1, cols 16to ..
  const int R = p.R;
  char* ws = (char*)p.ws;
  int* err = (int*)(ws + OFF_ERR);
  u64* gqkv = (u64*)(ws + OFF_QKV);
  u64* gpart = (u64*)(ws + OFF_PART);
  u64* gx16 = (u64*)(ws + OFF_X16);
  u64* gh = (u64*)(ws + OFF_H);
  const unsigned ep = (unsigned)(ld_g((const u64*)(ws + OFF_ERR)) >> 32);  // (low word: the error flag)
  float* dbg = p.ws_bytes >= (long long)(WS_BYTES + DBG_BYTES) ? (float*)(ws + WS_BYTES) : nullptr;
  auto tagof = [&](int e) { return ep * NEDGE + (unsigned)e + 1u; };
  const int kvpos = p.const_pos, nc = kvpos;
  const int grp = lane / LPK, sub = lane % LPK;
  const int r = min(w, R - 1);  // attention: wave w = row w
  const int vsel = min(grp, NREP + 1);
  const int e0 = sub * 8, half = D / 2, ec = e0 % half;
  const int slot = vsel * D + e0;  // this lane's 8 q/k/v values within head h's 512 (q0, q1, k, v)
  const int hh = vsel < NREP ? h * NREP + vsel : (vsel == NREP ? NQ + h : NQ + NKV + h);

  // the owned residual slice
  if (tid < 32) {
    const int rr = 2 * qo + (tid >> 4);
    s.xown[tid >> 4][tid & 15] = rr < R ? p.x[(long long)rr * p.ldx + 16 * to + (tid & 15)] : 0.f;
  }

  // register-resident weights of the next phase (see the header)
  u32x4_t w1[4];    // P1: q/k/v tile, k tiles 4w .. 4w + 3
  u32x4_t w2[2];    // P2: o_proj, 2 fragments per wave
  u32x4_t w3[8];    // P3: gate/up, 4 (one tile) or 8 (two tiles) fragments per wave
  u32x4_t w4[12];   // P4: down tile `to`, k tiles 12w .. 12w + 11
  u32x4_t kq[IC], vq[IC];  // P2: cached keys / values of (row r, head h)
  const int ntile3 = b < 3 * NB / 2 - NB ? 2 : 1;  // gate/up tiles: b and b + 256 for b < 128 (384 tiles)
  const int t3 = ntile3 == 2 ? b + (w >> 2) * NB : b;
  const int k3 = ntile3 == 2 ? (w & 3) * 8 : w * 4, n3 = ntile3 == 2 ? 8 : 4;
  // P1 tile of block (h, cg): head h's 32 q/k/v tiles (q: 16, k: 8, v: 8)
  const int t1 = cg < 16 ? h * 16 + cg : (cg < 24 ? NQ * D / 16 + h * 8 + (cg - 16) : (NQ + NKV) * D / 16 + h * 8 + (cg - 24));
  // P2: wave w multiplies o_proj fragments f0, f0 + 1 of tile (2cg + tw), head h's k tiles
  const int f0 = w * 2, tw = f0 / 8, kt0 = f0 % 8;

  auto load_p2 = [&](int l) {
#pragma unroll
    for (int i = 0; i < 2; ++i) w2[i] = ldw(frag(p.w_o[l], 2 * cg + tw, h * 8 + kt0 + i, KTO, lane));
    const long long kvb = ((long long)r * NKV + h) * p.Lmax * D;
#pragma unroll
    for (int c = 0; c < IC; ++c) {
      const int jj = min(c * GPW + grp, max(nc - 1, 0));
      kq[c] = ldw((const bf16_t*)p.k_cache[l] + kvb + (long long)jj * D + sub * 8);
      vq[c] = ldw((const bf16_t*)p.v_cache[l] + kvb + (long long)jj * D + sub * 8);
    }
    CE_ISSUED();
  };
  auto load_p3 = [&](int l) {
#pragma unroll
    for (int i = 0; i < 8; ++i) w3[i] = ldw(frag(p.w_gu[l], t3, k3 + min(i, n3 - 1), KTH, lane));
    CE_ISSUED();
  };
  auto load_p4 = [&](int l) {
#pragma unroll
    for (int i = 0; i < 12; ++i) w4[i] = ldw(frag(p.w_down[l], to, w * 12 + i, KTI, lane));
    CE_ISSUED();
  };
  auto load_p1 = [&](const void* wt, int tile) {
#pragma unroll
    for (int i = 0; i < 4; ++i) w1[i] = ldw(frag(wt, tile, w * 4 + i, KTH, lane));
    CE_ISSUED();
  };

  // publish the owned slice's bf16 copy (16 granules: 2 rows x 8 column pairs) to x16 buffer `buf`
  auto publish_x16 = [&](int buf, unsigned tag) {
    if (tid < 16) {
      const int rr = tid >> 3, pp = tid & 7;
      if (2 * qo + rr < R)
        st_g(gx16 + ((size_t)buf * MAXR + 2 * qo + rr) * (H / 2) + 8 * to + pp,
             pack2bf(s.xown[rr][2 * pp], s.xown[rr][2 * pp + 1]), tag);
    }
  };

  const int L = p.n_layers;
  load_p2(0);
  for (int l = 0; l < L; ++l) {
    // ------------------------------------------------------------------ P1: q/k/v projection (layers >= 1)
    if (l > 0) {
      stage_x16(s, gx16 + (size_t)1 * MAXR * (H / 2), tagof(5 * (l - 1) + 4), R, p.eps, pk.spin, err);
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) acc = mfma(afrag_x(s, lm, lk, w * 4 + i, R), w1[i], acc);
      load_p2(l);
      s.red[w][lane][0] = acc[0]; s.red[w][lane][1] = acc[1]; s.red[w][lane][2] = acc[2]; s.red[w][lane][3] = acc[3];
      __syncthreads();
      if (w == 0) {
        const f32x4_t v = red_sum(s, 0, NW, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rr = lk * 4 + i;
          if (rr < R) st_g(gqkv + ((size_t)h * MAXR + rr) * 512 + cg * 16 + lm, __float_as_uint(v[i] * s.rs[rr]),
                           tagof(5 * l));
        }
      }
    }
    // ------------------------------------------------------------------ P2: attention of head h + o_proj K-slice
    {
      float xv[8];
      if (l == 0) {
        load8f(p.qkv0 + (long long)r * p.ldq + (long long)hh * D + e0, xv);
      } else {
        unsigned v[8];
        poll_run<8>(gqkv + ((size_t)h * MAXR + r) * 512 + slot, tagof(5 * l), v, pk.spin, err);
#pragma unroll
        for (int k = 0; k < 8; ++k) xv[k] = __uint_as_float(v[k]);
      }
      float nwv[8], cv[8], sv[8];
      const float* nwp = vsel < NREP ? p.q_norm[l] : p.k_norm[l];
      load8f(nwp + e0, nwv);
      load8f(p.cos_tab + (long long)kvpos * half + ec, cv);
      load8f(p.sin_tab + (long long)kvpos * half + ec, sv);
      {  // q/k RMSNorm + RoPE (branch-free over the lane groups; the v group's result is discarded)
        const bool lo = e0 < half, normed = vsel <= NREP;
        float ss = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) ss += xv[i] * xv[i];
        ss = group_sum_dpp<LPK>(ss);
        const float rsn = rsqrtf(ss / (float)D + p.eps);
        float y[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) y[i] = nwv[i] * (xv[i] * rsn);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float pt = half_partner<LPK>(y[i]);
          const float ro = lo ? y[i] * cv[i] - pt * sv[i] : y[i] * cv[i] + pt * sv[i];
          xv[i] = normed ? ro : xv[i];
        }
      }
      if (grp <= NREP) {
        u32x4_t pk2;
#pragma unroll
        for (int i = 0; i < 4; ++i) pk2[i] = pack2bf_rne(xv[2 * i], xv[2 * i + 1]);
        *(u32x4_t*)(grp < NREP ? &s.qs2[w][grp][e0 / 2] : &s.kn2[w][e0 / 2]) = pk2;
      } else if (grp == NREP + 1) {
#pragma unroll
        for (int i = 0; i < 8; ++i) s.vn[w][e0 + i] = bf2f(f2bf(xv[i]));
      }
      __syncthreads();
      // attention of (row r, head h) over the cached keys [0, kvpos) + the new key (attn_oproj_hs_k, phase 3)
      {
        const float scale = rsqrtf((float)D) * 1.4426950408889634f;
        u32x4_t q2[NREP];
#pragma unroll
        for (int j = 0; j < NREP; ++j) q2[j] = *(const u32x4_t*)&s.qs2[w][j][sub * 4];
        const u32x4_t k2n = *(const u32x4_t*)&s.kn2[w][sub * 4];
        auto dot8 = [](const u32x4_t& a, const u32x4_t& bb) {
          float d = 0.f;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const unsigned ai = a[i], bi = bb[i];
            d = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, ai), __builtin_bit_cast(bf16x2_t, bi), d,
                                                false);
          }
          return d;
        };
        float dd[NREP][IC], dn[NREP];
#pragma unroll
        for (int j = 0; j < NREP; ++j) {
          dn[j] = group_sum_dpp<LPK>(dot8(q2[j], k2n)) * scale;
#pragma unroll
          for (int c = 0; c < IC; ++c) {
            const float d = group_sum_dpp<LPK>(dot8(q2[j], kq[c])) * scale;
            dd[j][c] = c * GPW + grp < nc ? d : -INFINITY;
          }
        }
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
        for (int i = 0; i < 8; ++i) vnf[i] = s.vn[w][sub * 8 + i];
        float m[NREP], lsum[NREP], o[NREP][8];
#pragma unroll
        for (int j = 0; j < NREP; ++j) {
          float mn = dn[j];
#pragma unroll
          for (int c = 0; c < IC; ++c) mn = fmaxf(mn, dd[j][c]);
          const float en = grp == 0 ? exp2_hw(dn[j] - mn) : 0.f;
          unsigned epk[IC / 2];
#pragma unroll
          for (int pr = 0; pr < IC / 2; ++pr) epk[pr] = pack2bf_rne(exp2_hw(dd[j][2 * pr] - mn), exp2_hw(dd[j][2 * pr + 1] - mn));
          float ls = en;
#pragma unroll
          for (int pr = 0; pr < IC / 2; ++pr)
            ls = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, epk[pr]),
                                                 __builtin_bit_cast(bf16x2_t, 0x3F803F80u), ls, false);
#pragma unroll
          for (int d = 0; d < 8; ++d) {
            float acc = en * vnf[d];
            const int vi = (d & 1) * 4 + (d >> 1);
#pragma unroll
            for (int pr = 0; pr < IC / 2; ++pr)
              acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, epk[pr]),
                                                    __builtin_bit_cast(bf16x2_t, vp[pr][vi]), acc, false);
            o[j][d] = acc;
          }
          m[j] = mn; lsum[j] = ls;
        }
        GroupMerge<LPK, NREP> gm;
        gm.run(m, lsum, o);
        gm.each(lane, [&](int j, int d, float ov, float lv, float) { s.att[w][j * D + d] = f2bf(ov * __builtin_amdgcn_rcpf(lv)); });
      }
      __syncthreads();
      if (dbg && l == 0 && cg == 0 && w < R)
        for (int j = lane; j < NREP * D; j += 64) dbg[((size_t)3 * MAXR + w) * 4096 + h * NREP * D + j] = bf2f(s.att[w][j]);
      // head h's K-slice of o_proj for columns 32cg .. 32cg + 32: wave w, fragments f0, f0 + 1 of tile 2cg + tw
      {
        f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const u32x4_t av = lm < NW ? *(const u32x4_t*)&s.att[lm][(kt0 + i) * 32 + lk * 8] : u32x4_t{0u, 0u, 0u, 0u};
          acc = mfma(av, w2[i], acc);
        }
        load_p3(l);
        s.red[w][lane][0] = acc[0]; s.red[w][lane][1] = acc[1]; s.red[w][lane][2] = acc[2]; s.red[w][lane][3] = acc[3];
      }
      // the new k / v of (row w, head h) into the caches (one column group appends)
      if (cg == 0 && w < R && lane < D / 2) {
        const long long o = (((long long)w * NKV + h) * p.Lmax + kvpos) * D;
        ((unsigned*)p.k_cache[l])[o / 2 + lane] = s.kn2[w][lane];
        ((bf16_t*)p.v_cache[l])[o + lane] = f2bf(s.vn[w][lane]);
        ((bf16_t*)p.v_cache[l])[o + lane + 64] = f2bf(s.vn[w][lane + 64]);
      }
      __syncthreads();
      // row rr's partial for column c (thread (rr, c < 32)): the tile's 4 waves summed in wave order -> the owner of
      // (tile 2cg + c / 16, row pair rr / 2)
      if (tid < MAXR * 32) {
        const int rr = tid >> 5, c = tid & 31, tt = c >> 4, cc = c & 15;
        float v = 0.f;
#pragma unroll
        for (int q2 = 0; q2 < 4; ++q2) v += s.red[tt * 4 + q2][(rr >> 2) * 16 + cc][rr & 3];
        if (rr < R)
          st_g(gpart + ((((size_t)(2 * cg + tt) * 4 + (rr >> 1)) * NKV + h) * 32 + (rr & 1) * 16 + cc),
               __float_as_uint(v), tagof(5 * l + 1));
      }
    }
    // ------------------------------------------------------------------ residual add by the owner, x16 edge
    {
      if (tid < NKV * 32) {
        const int hp = tid >> 5, sl = tid & 31;
        unsigned v[1] = {0u};
        if (2 * qo + (sl >> 4) < R)
          poll_run<1>(gpart + ((((size_t)to * 4 + qo) * NKV + hp) * 32 + sl), tagof(5 * l + 1), v, pk.spin, err);
        s.gath[hp][sl] = __uint_as_float(v[0]);
      }
      __syncthreads();
      if (tid < 32) {
        float v = 0.f;
#pragma unroll
        for (int hp = 0; hp < NKV; ++hp) v += s.gath[hp][tid];
        s.xown[tid >> 4][tid & 15] += v;
        if (dbg && l == 0 && 2 * qo + (tid >> 4) < R)
          dbg[((size_t)0 * MAXR + 2 * qo + (tid >> 4)) * 4096 + 16 * to + (tid & 15)] = s.xown[tid >> 4][tid & 15];
      }
      __syncthreads();
      publish_x16(0, tagof(5 * l + 2));
    }
    // ------------------------------------------------------------------ P3: gate/up + SwiGLU
    {
      stage_x16(s, gx16, tagof(5 * l + 2), R, p.eps, pk.spin, err);
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (i < n3) acc = mfma(afrag_x(s, lm, lk, k3 + i, R), w3[i], acc);
      load_p4(l);
      s.red[w][lane][0] = acc[0]; s.red[w][lane][1] = acc[1]; s.red[w][lane][2] = acc[2]; s.red[w][lane][3] = acc[3];
      __syncthreads();
      if (w < ntile3) {  // wave j finishes tile j: column lm (gate lm < 8, up lm + 8), rows lk*4 .. + 3
        const int nw = ntile3 == 2 ? 4 : 8;
        const f32x4_t v = red_sum(s, w * nw, nw, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rr = lk * 4 + i;  // MFMA rows 8..15 carry no batch row (zero A)
          const float g = rr < MAXR ? v[i] * s.rs[rr] : 0.f;
          const float up = __shfl_xor(g, 8, 64);
          const float hv = silu_f(g) * up;
          const float hv2 = __shfl_xor(hv, 1, 64);  // column lm + 1's value (pairs 2p, 2p + 1)
          if (lm < 8 && (lm & 1) == 0 && rr < MAXR) s.hsw[w][rr][lm >> 1] = pack2bf(hv, hv2);
        }
      }
      __syncthreads();
      if (tid < ntile3 * MAXR * 4) {
        const int j = tid >> 5, rr = (tid >> 2) & 7, pp = tid & 3;
        const int tile = j == 0 ? b : b + NB;
        if (rr < R) st_g(gh + (size_t)rr * (I / 2) + tile * 4 + pp, s.hsw[j][rr][pp], tagof(5 * l + 3));
        if (dbg && l == 0 && rr < R) {
          dbg[((size_t)1 * MAXR + rr) * 4096 + tile * 8 + 2 * pp] = __uint_as_float(s.hsw[j][rr][pp] << 16);
          dbg[((size_t)1 * MAXR + rr) * 4096 + tile * 8 + 2 * pp + 1] = __uint_as_float(s.hsw[j][rr][pp] & 0xFFFF0000u);
        }
      }
    }
    // ------------------------------------------------------------------ P4: down tile `to` for rows 2qo, 2qo + 1
    {
      {  // the owner's two SwiGLU rows: thread -> row tid / 256, pairs (tid % 256) * 6 .. + 5
        const int rr = tid >> 8, p0 = (tid & 255) * 6;
        unsigned v[6];
        if (2 * qo + rr < R) {
          poll_run<6>(gh + (size_t)(2 * qo + rr) * (I / 2) + p0, tagof(5 * l + 3), v, pk.spin, err);
        } else {
#pragma unroll
          for (int k = 0; k < 6; ++k) v[k] = 0u;
        }
        unsigned* hrow = (unsigned*)&s.a.ha[rr][0];
#pragma unroll
        for (int k = 0; k < 6; ++k) hrow[p0 + k] = v[k];
      }
      __syncthreads();
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 12; ++i) {
        const int kt = w * 12 + i;
        const u32x4_t av = lm < 2 ? *(const u32x4_t*)&s.a.ha[lm][kt * 32 + lk * 8] : u32x4_t{0u, 0u, 0u, 0u};
        acc = mfma(av, w4[i], acc);
      }
      if (l + 1 < L) load_p1(p.w_qkv[l + 1], t1);
      else if (b < p.V / 16) load_p1(p.w_lm, b);
      s.red[w][lane][0] = acc[0]; s.red[w][lane][1] = acc[1]; s.red[w][lane][2] = acc[2]; s.red[w][lane][3] = acc[3];
      __syncthreads();
      if (tid < 32) {  // (row tid / 16, column tid % 16) = MFMA row tid / 16 of lane tid % 16
        float v = 0.f;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) v += s.red[ww][tid & 15][tid >> 4];
        s.xown[tid >> 4][tid & 15] += v;
        if (dbg && l == 0 && 2 * qo + (tid >> 4) < R)
          dbg[((size_t)2 * MAXR + 2 * qo + (tid >> 4)) * 4096 + 16 * to + (tid & 15)] = s.xown[tid >> 4][tid & 15];
      }
      __syncthreads();
      publish_x16(1, tagof(5 * l + 4));
    }
  }
  // -------------------------------------------------------------------- final norm + lm_head[g] (tiles 0 .. V/16)
  stage_x16(s, gx16 + (size_t)1 * MAXR * (H / 2), tagof(5 * (L - 1) + 4), R, p.eps, pk.spin, err);
  if (b < p.V / 16) {
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) acc = mfma(afrag_x(s, lm, lk, w * 4 + i, R), w1[i], acc);
    s.red[w][lane][0] = acc[0]; s.red[w][lane][1] = acc[1]; s.red[w][lane][2] = acc[2]; s.red[w][lane][3] = acc[3];
    __syncthreads();
    if (w == 0) {
      const f32x4_t v = red_sum(s, 0, NW, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rr = lk * 4 + i;
        if (rr < R) p.logits[(long long)rr * p.ldl + b * 16 + lm] = v[i] * s.rs[rr];
      }
    }
  }
  // the launch counter: every block read it before its first publication, and block 0 has consumed an edge from every
  // block by now
  if (b == 0 && tid == 0)
    __hip_atomic_store((unsigned*)(ws + OFF_EPOCH), ep + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

bool cp_step_resident() {
  static int cap[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
  if (cap[dev] == 0) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)cp_step_k, NT, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return false;
    cap[dev] = std::max(1, per_cu * cus);
  }
  return cap[dev] >= NB;
}

}  // namespace

extern "C" long long qt_cp_step_ws_bytes(void) { return (long long)WS_BYTES; }
extern "C" long long qt_cp_step_dbg_bytes(void) { return (long long)DBG_BYTES; }

extern "C" int qt_cp_step_supported(int H_, int I_, int Hq, int Hkv, int D_, int n_layers, int V) {
  return H_ == H && I_ == I && Hq == NQ && Hkv == NKV && D_ == D && n_layers >= 1 && n_layers <= 6 && V % 16 == 0 &&
         V / 16 <= NB && cp_step_resident();
}

extern "C" int qt_cp_step(const qt_cp_step_args* a, void* stream) {
  if (!a || a->R < 1 || a->R > MAXR || a->n_layers < 1 || a->n_layers > 6) return QT_ERR_SHAPE;
  if (a->const_pos < 1 || a->const_pos > IC * GPW || a->const_pos >= a->Lmax) return QT_ERR_SHAPE;
  if (a->V % 16 || a->V / 16 > NB || a->V <= 0) return QT_ERR_SHAPE;
  if (!a->ws || a->ws_bytes < (long long)WS_BYTES || !a->x || !a->qkv0 || !a->logits || !a->w_lm || !a->cos_tab ||
      !a->sin_tab)
    return QT_ERR_ARG;
  for (int l = 0; l < a->n_layers; ++l)
    if (!a->w_qkv[l] || !a->w_o[l] || !a->w_gu[l] || !a->w_down[l] || !a->q_norm[l] || !a->k_norm[l] ||
        !a->k_cache[l] || !a->v_cache[l])
      return QT_ERR_ARG;
  if (!cp_step_resident()) return QT_ERR_SHAPE;
  static const int spin = std::max(1000, qt_knob("QT_CE_SPIN", 200000));
  hipLaunchKernelGGL(cp_step_k, dim3(NB), dim3(NT), 0, (hipStream_t)stream, CEP{*a, spin});
  return hipGetLastError() == hipSuccess ? 0 : QT_ERR_LAUNCH;
}
