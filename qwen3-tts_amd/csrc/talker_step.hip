// Talker decode-step engine for gfx950: ONE persistent launch runs every decoder layer of a talker decode step for up
// to 8 batch rows -- input RMSNorm + q/k/v, q/k RMSNorm + RoPE + KV append + attention, o_proj + residual,
// post-attention RMSNorm + gate/up + SwiGLU + down + residual -- where the launch chain issued 5 kernels per layer
// (DESIGN §11).  Replaces Qwen3TTSTalkerModel.forward's decoder-layer loop for one generated frame (M:1430-1480,
// layers M:961-1012, attention M:740-804 with q/k norm M:764-765, MLP M:842-855); the final norm + codec_head stay on
// the chain.
//
// The weight-ring machinery of qt_talker_tail (talker_tail.hip), stretched over the whole step: two loader waves per
// workgroup stream the block's weight fragments of all layers, in consumption order, into a 5-slot LDS ring by
// LDS-DMA (non-temporal), never waiting for a hand-off -- only for ring space -- so the next phase's and the next
// LAYER's weights arrive while the consumers wait for hand-offs or run the attention; before each hand-off wait the
// consumer waves move their fragments of the next slots into registers (NPRE slots), so the ring keeps draining.
//
// Per layer l (block b of 256): Q tile b of the q/k/v projection (16 of 4096 columns) -> [Q edge: the 32 tiles of a
// kv head] -> blocks b < 8R: attention of (row b / 8, kv head b % 8), the head-pair's output rows -> [A edge: the 32
// attention blocks of a K half, replicated per XCD] -> o_proj tile b / 2, K half b % 2 (split-K pair, the even block
// owns the residual slice) -> [pair granules] -> [X1: x16 rows, all-to-all] -> gate/up tiles b, b + 256, b + 512 +
// SwiGLU -> [H: SwiGLU rows, all-to-all] -> down tile b / 2, K half b % 2 -> [pair] -> [X2: x16 rows] -> layer l + 1.
// The residual stream stays in the owners' LDS for the whole launch (fp32); x is read at the start and the last
// layer's output written at the end.  Tags: epoch * 256 + 8 l + edge + 1 (a launch counter in the workspace).
#include "common.h"
#include "attn_dev.h"
#include "engine_dev.h"
#include <algorithm>

namespace {

using namespace qt_engine;

constexpr int H = 2048, I = 6144, NQKV = 4096, KO = 2048, NQ = 16, NKV = 8, NREP = 2, D = 128;
constexpr int NB = 256, NWC = 8, NWL = 2, NT = (NWC + NWL) * 64, MAXR = 8, MAXL = 32;
constexpr int KTH = H / 32, KTI = I / 32, KTO = KO / 32;
constexpr int NSLOT = 5, SLOT = 16;
constexpr int XLD = H + 8, ALD = KO / 2 + 8, HLD = I / 2 + 8;
constexpr int NPRE = 10;
constexpr int NSPL = 4;                 // key splits per (row, kv head): all 256 blocks share the K/V stream
constexpr int AREC = NREP * (D + 2);    // a split's partial: per q head m, l, o[D] (unnormalised)
constexpr int E_Q = 0, E_A = 1, E_PO = 2, E_X1 = 3, E_H = 4, E_PD = 5, E_X2 = 6, E_AP = 7;
// ring slots per layer, in consumption order: q/k/v 64 k tiles, o_proj 32, gate/up 3 x 64, down 96
constexpr int S_Q = KTH / SLOT, S_O = KTO / 2 / SLOT, S_GU = 3 * KTH / SLOT, S_D = KTI / 2 / SLOT;
constexpr int S_L = S_Q + S_O + S_GU + S_D;
static_assert(S_Q == 4 && S_O == 2 && S_GU == 12 && S_D == 6, "slot plan");
static_assert(S_O + 6 <= NPRE, "o_proj + the first gate/up slots pre-taken across the attention hand-off");

// workspace (bytes)
constexpr size_t OFF_ERR = 0, OFF_EPOCH = 4;
constexpr int NREPL = 8;
constexpr int FL_X1 = 0, FL_H = 1, FL_X2 = 2, FL_A = 3;
constexpr size_t OFF_QFL = 256;                                       // [NB] q/k/v tile flags
constexpr size_t OFF_FLAGS = OFF_QFL + NB * 4, REPL_FLAGS = (size_t)4 * NB * 4;
constexpr size_t OFF_QKV = OFF_FLAGS + NREPL * REPL_FLAGS;           // [MAXR][4096] fp32 q/k/v rows
constexpr size_t OFF_PART = OFF_QKV + (size_t)MAXR * NQKV * 4;       // [2][128][MAXR][16] granules
constexpr size_t OFF_X16 = OFF_PART + (size_t)2 * 128 * MAXR * 16 * 8;
constexpr size_t REPL_X16 = (size_t)2 * MAXR * (H / 2) * 4;
constexpr size_t OFF_H = OFF_X16 + NREPL * REPL_X16;
constexpr size_t REPL_H = (size_t)MAXR * (I / 2) * 4;
constexpr size_t OFF_ATT = OFF_H + NREPL * REPL_H;                   // replicas of [MAXR][KO/2] bf16 pairs
constexpr size_t REPL_ATT = (size_t)MAXR * (KO / 2) * 4;
constexpr size_t OFF_APART = OFF_ATT + NREPL * REPL_ATT;             // [64 pairs][NSPL - 1][AREC] granules
constexpr size_t WS_BYTES = OFF_APART + (size_t)NKV * MAXR * (NSPL - 1) * AREC * 8;
constexpr size_t STAMP_BYTES = (size_t)NB * 16 * MAXL * 8;          // optional: [NB][MAXL][16] phase stamps

enum { PT_QKV, PT_O, PT_GU, PT_DOWN, PT_QN, PT_KN, PT_KC, PT_VC };

struct SP {
  qt_talker_step_args a;
  int spin;
  int nwl;    // loader waves streaming (1 or NWL)
  int depth;  // slots a loader wave keeps in flight (1 or 2)
};

struct AttLds {                          // the attention phase (one (row, kv head) per attention block)
  float qs[NREP][D];
  float knew[D], vnew[D];
  float mrg_ml[NWC][NREP][2];
  float mrg_o[NWC][NREP][D];
  unsigned out[NREP * D / 2];            // the head pair's output row, bf16 pairs
  float part[AREC];                      // this split's partial (m, l, o) per q head
};

struct SLds {
  __attribute__((aligned(16))) unsigned char ring[NSLOT][SLOT * 1024];
  union {
    bf16_t xa[MAXR][XLD];
    bf16_t aa[MAXR][ALD];
    bf16_t ha[MAXR][HLD];
    AttLds at;
  } a;
  float red[2][NWC][64][4];
  float rs[MAXR];
  float xo[MAXR][16];
  unsigned hb[3][MAXR][4];
  __attribute__((aligned(16))) bf16_t zero[32];
  const void* ptab[8][MAXL];
  int rmeta[4][MAXR];  // per row: rope_pos, kv_pos, row_start, row_batch (constant for the launch)
  unsigned full[NSLOT];
  unsigned done[NWC];
};

__global__ __launch_bounds__(NT) void talker_step_k(SP pk) {
  const qt_talker_step_args& p = pk.a;
  __shared__ SLds s;
  __shared__ unsigned cb_cnt, cb_gen;
  const int b = blockIdx.x;
  const int ot = b >> 1, kh = b & 1;
  const bool owner = kh == 0;
  // layers [l0, l0 + L) of a LT-layer stack; qkv_in: layer l0's q/k/v rows are given (its Q phase is skipped);
  // qkv_out: the launch ends with layer l0 + L's q/k/v rows (written to global)
  const int R = p.R, L = p.n_layers, l0 = p.first_layer, LT = p.total_layers;
  const bool qin = p.qkv_in != nullptr, qout = p.qkv_out != nullptr;
  const bool ain = p.att_in != nullptr, aout = p.att_out != nullptr;  // attention rows in (skip Q, A) / out (+ Q, A)
  char* ws = (char*)p.ws;
  int* err = (int*)(ws + OFF_ERR);
  const int myrep = b % NREPL;
  auto fl_off = [&](int rp, int kind) { return (unsigned)(OFF_FLAGS + rp * REPL_FLAGS + kind * NB * 4); };
  u64* gpart = (u64*)(ws + OFF_PART);
  const rsrc_t wsr = mkr(ws, (unsigned)WS_BYTES);
  const unsigned ep = (unsigned)(ld_g((const u64*)(ws + OFF_ERR)) >> 32);
  auto tagof = [&](int l, int e) { return ep * 256u + (unsigned)(8 * l + e) + 1u; };
  u64* stamps = p.ws_bytes >= (long long)(WS_BYTES + STAMP_BYTES) ? (u64*)(ws + WS_BYTES) + b * 16 * MAXL : nullptr;
#define TS_STAMP(l, k) \
  if (kProbe && stamps && threadIdx.x == 0) stamps[(l) * 16 + (k)] = __builtin_amdgcn_s_memrealtime();
  const int nseq = S_L * L - (qin || ain ? S_Q : 0) + (qout || aout ? S_Q : 0);
  // per-lane coordinates, re-derived from an opaque thread id at every layer (refresh()): otherwise hipcc hoists the
  // per-lane addresses of every phase out of the layer loop and keeps them all alive (250 VGPRs, spills)
  int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  auto refresh = [&]() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    tid = t;
    w = __builtin_amdgcn_readfirstlane(t >> 6);
    lane = t & 63;
  };
  // attention: NSPL blocks per (row, kv head) pair, each over a quarter of the keys; split 0 merges
  const bool attb = b < NSPL * NKV * R;
  const int apair = b / NSPL, az = b % NSPL, ar = apair >> 3, ahk = apair & 7;

  if (tid < NSLOT) s.full[tid] = 0u;
  else if (tid >= 64 && tid < 64 + NWC) s.done[tid - 64] = 0u;
  else if (tid >= 128 && tid < 144) ((unsigned*)s.zero)[tid - 128] = 0u;
  if (tid >= 256 && tid < 256 + 8 * MAXL) {  // the per-layer pointer table
    const int k = (tid - 256) / MAXL, l = (tid - 256) % MAXL;
    s.ptab[k][l] = l < LT ? p.wtab[k * LT + l] : nullptr;
  }
  if (tid >= 160 && tid < 160 + 4 * MAXR) {
    const int k = (tid - 160) / MAXR, rr = (tid - 160) % MAXR;
    const int* src = k == 0 ? p.rope_pos : (k == 1 ? p.kv_pos : (k == 2 ? p.row_start : p.row_batch));
    s.rmeta[k][rr] = rr < R ? src[rr] : 0;
  }
  if (tid == 0) { cb_cnt = 0u; cb_gen = 0u; }
  __syncthreads();  // (the last block-wide barrier: the loader waves run free from here)
  auto lp = [&](int k, int l) -> const void* {
    const u64 v = (u64)s.ptab[k][l];
    return (const void*)(((u64)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(v >> 32)) << 32) |
                         (u64)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)v));
  };

  if (w >= NWC) {
    // ------------------------------------------------------------------ loader waves
    const int lw = w - NWC, nwl = pk.nwl;
    if (lw >= nwl) return;
    for (int sq = lw; sq < nseq; sq += nwl) {
      const int vq = sq + (qin || ain ? S_Q : 0), l = l0 + vq / S_L, j = vq % S_L;
      int pk_, tile, kt0, KT;
      if (j < S_Q) { pk_ = PT_QKV; tile = b; kt0 = SLOT * j; KT = KTH; }
      else if (j < S_Q + S_O) { pk_ = PT_O; tile = ot; kt0 = kh * (KTO / 2) + SLOT * (j - S_Q); KT = KTO; }
      else if (j < S_Q + S_O + S_GU) { const int g = j - S_Q - S_O; pk_ = PT_GU; tile = b + NB * (g / 4); kt0 = SLOT * (g % 4); KT = KTH; }
      else { pk_ = PT_DOWN; tile = ot; kt0 = kh * (KTI / 2) + SLOT * (j - S_Q - S_O - S_GU); KT = KTI; }
      const int slot = sq % NSLOT;
      if (sq >= NSLOT) {
        for (int spins = 0;; ++spins) {
          unsigned m = 0xFFFFFFFFu;
#pragma unroll
          for (int c = 0; c < NWC; ++c) m = min(m, lds_ld(&s.done[c]));
          if ((int)__builtin_amdgcn_readfirstlane(m) >= sq - NSLOT + 1) break;
          if (spins > 16 * pk.spin) { if (lane == 0) atomicOr(err, 2); break; }
          __builtin_amdgcn_s_sleep(0);
        }
      }
      const char* src = (const char*)lp(pk_, l) + ((size_t)(tile * KT + kt0) << 10) + lane * 16;
      const unsigned dst = lds_u32(&s.ring[slot][0]);
#pragma unroll
      for (int f = 0; f < SLOT; ++f) glds16_nt(src + f * 1024, dst + f * 1024);
      if (pk.depth == 1) {  // this slot landed before the next is issued
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) lds_st(&s.full[slot], (unsigned)(sq + 1));
      } else if (sq - nwl >= 0) {  // the previous slot of this wave has landed once only this one is outstanding
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        if (lane == 0) lds_st(&s.full[(sq - nwl) % NSLOT], (unsigned)(sq - nwl + 1));
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int last = lw + nwl * ((nseq - 1 - lw) / nwl);
    if (lane == 0 && last < nseq) lds_st(&s.full[last % NSLOT], (unsigned)(last + 1));
    return;
  }

  // ------------------------------------------------------------------ consumer waves (tid < 512)
  CBar cb{&cb_cnt, &cb_gen};
  unsigned cg = 0;
  int lm = lane & 15, lk = lane >> 4;
  int sq = 0;
  auto take = [&](u32x4_t& f0, u32x4_t& f1) {
    const int slot = sq % NSLOT;
    for (int spins = 0; (int)__builtin_amdgcn_readfirstlane(lds_ld(&s.full[slot])) < sq + 1; ++spins) {
      if (spins > 16 * pk.spin) { if (lane == 0) atomicOr(err, 4); break; }
      __builtin_amdgcn_s_sleep(0);
    }
    f0 = *(const u32x4_t*)&s.ring[slot][(2 * w) * 1024 + lane * 16];
    f1 = *(const u32x4_t*)&s.ring[slot][(2 * w + 1) * 1024 + lane * 16];
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f0), "+v"(f1)::"memory");
    ++sq;
    if (lane == 0) lds_st(&s.done[w], (unsigned)sq);
  };
  u32x4_t pf[2 * NPRE];
  auto pretake = [&](int n) {  // the next n (<= NPRE) slots into registers
#pragma unroll
    for (int k = 0; k < NPRE; ++k)
      if (k < n) take(pf[2 * k], pf[2 * k + 1]);
  };
  auto frags = [&](int k, u32x4_t& f0, u32x4_t& f1) {  // pre-taken slot k or the ring
    if (k < NPRE) { f0 = pf[2 * k]; f1 = pf[2 * k + 1]; } else take(f0, f1);
  };
  auto sync = [&]() { cons_sync<NWC>(cb, cg, pk.spin, err); };
  auto poll = [&](unsigned off, int n, unsigned tag) {  // (wave 0) n flag words at `off` carry tag
    if (w == 0) {
      for (int spins = 0;; ++spins) {
        bool ok = true;
        if (lane * 4 < n) {
          const u32x4_t v = bld_c(wsr, off + lane * 16);
          ok = v[0] == tag && v[1] == tag && v[2] == tag && v[3] == tag;
        }
        if (__all(ok)) break;
        if (spins > pk.spin) { if (lane == 0) atomicOr(err, 1); break; }
        __builtin_amdgcn_s_sleep(1);
      }
    }
  };
  auto red_put = [&](int buf, f32x4_t acc) {
    s.red[buf][w][lane][0] = acc[0]; s.red[buf][w][lane][1] = acc[1];
    s.red[buf][w][lane][2] = acc[2]; s.red[buf][w][lane][3] = acc[3];
  };
  auto red_sum = [&](int buf) {
    f32x4_t v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ww = 0; ww < NWC; ++ww) {
      v[0] += s.red[buf][ww][lane][0]; v[1] += s.red[buf][ww][lane][1];
      v[2] += s.red[buf][ww][lane][2]; v[3] += s.red[buf][ww][lane][3];
    }
    return v;
  };
  auto rms_rows = [&](const u32x4_t* v, int nv, int row) {  // (row = wave) 1 / rms from the row's bf16 values
    float ss = 0.f;
    for (int k = 0; k < nv; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float lo = __uint_as_float(v[k][e] << 16), hi = __uint_as_float(v[k][e] & 0xFFFF0000u);
        ss += lo * lo + hi * hi;
      }
    ss = wave_sum_dpp(ss);
    if (lane == 0) s.rs[row] = rsqrtf(ss / (float)H + p.eps);
  };
  auto stage_x16 = [&](int buf) {  // the x16 edge (replica myrep) -> xa, rs; thread -> row tid / 64
    const int row = tid >> 6;
    const unsigned base = (unsigned)(OFF_X16 + myrep * REPL_X16 + (size_t)buf * MAXR * (H / 2) * 4);
    u32x4_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      v[k] = row < R ? bld_c(wsr, base + (unsigned)(row * (H / 2)) * 4 + (lane + 64 * k) * 16) : u32x4_t{0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 4; ++k) *(u32x4_t*)&s.a.xa[row][(lane + 64 * k) * 8] = v[k];
    rms_rows(v, 4, row);
    sync();
  };
  auto pair_in = [&](f32x4_t v, int kind, unsigned tag) {  // the 4 granules of the lane in flight at once
    const u64* g = gpart + (((size_t)kind * 128 + ot) * MAXR + lk * 4) * 16 + lm;
    u64 x[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = lk * 4 + i < R ? ld_g(g + i * 16) : ((u64)tag << 32);
    for (int spins = 0;; ++spins) {
      bool ok = true;
#pragma unroll
      for (int i = 0; i < 4; ++i) ok = ok && (unsigned)(x[i] >> 32) == tag;
      if (ok) break;
      if (spins > pk.spin) { atomicOr(err, 1); break; }
      __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if ((unsigned)(x[i] >> 32) != tag) x[i] = ld_g(g + i * 16);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rr = lk * 4 + i;
      if (rr < R) s.xo[rr][lm] += v[i] + __uint_as_float((unsigned)x[i]);
    }
  };
  auto pair_out = [&](f32x4_t v, int kind, unsigned tag) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rr = lk * 4 + i;
      if (rr < R) st_g(gpart + (((size_t)kind * 128 + ot) * MAXR + rr) * 16 + lm, __float_as_uint(v[i]), tag);
    }
  };
  auto publish_x16 = [&](int buf, unsigned tag) {
    const int rr = lane >> 3, pp = lane & 7;
    if (rr < R) {
      const unsigned v = pack2bf(s.xo[rr][2 * pp], s.xo[rr][2 * pp + 1]);
      const unsigned o = (unsigned)OFF_X16 + (unsigned)(((buf * MAXR + rr) * (H / 2)) + 8 * ot + pp) * 4;
#pragma unroll
      for (int rp = 0; rp < NREPL; ++rp) bst_c(v, wsr, o + rp * (unsigned)REPL_X16);
    }
    drain_stores();
    if (lane < NREPL) st_flag((unsigned*)(ws + fl_off(lane, buf == 0 ? FL_X1 : FL_X2)) + ot, tag);
  };
  auto afrag = [&](const bf16_t* row0, int ld, int kt) {
    return *(const u32x4_t*)(lm < R ? row0 + (size_t)lm * ld + kt * 32 + lk * 8 : &s.zero[lk * 8]);
  };

  // the owner's residual slice: the step's input rows
  if (owner && tid < MAXR * 16) {
    const int rr = tid >> 4, c = tid & 15;
    s.xo[rr][c] = rr < R ? p.x[(long long)rr * p.ldx + 16 * ot + c] : 0.f;
  }
  {  // layer 0's A operand: the input rows rounded to bf16 (as the chain's x16 shadow), thread -> row tid / 64
    const int row = tid >> 6;
    u32x4_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      u32x4_t u = {0u, 0u, 0u, 0u};
      if (row < R) {
        const float* src = p.x + (long long)row * p.ldx + (lane + 64 * k) * 8;
        const f32x4_t a0 = *(const f32x4_t*)src, a1 = *(const f32x4_t*)(src + 4);
        u = u32x4_t{pack2bf(a0[0], a0[1]), pack2bf(a0[2], a0[3]), pack2bf(a1[0], a1[1]), pack2bf(a1[2], a1[3])};
      }
      v[k] = u;
      *(u32x4_t*)&s.a.xa[row][(lane + 64 * k) * 8] = u;
    }
    rms_rows(v, 4, row);
  }
  sync();

  // Q: q/k/v tile b of layer l (input RMSNorm folded) from the x16 rows of the previous layer (or the staged input
  // rows); out: the in-launch payload + flag, or the global rows of the next launch
  auto q_phase = [&](int l, bool first, float* qkv_glob) {
    if (!first) {
      pretake(S_Q);
      poll(fl_off(myrep, FL_X2), 128, tagof(l - 1, E_X2));
      sync();
      stage_x16(1);
    } else {
      pretake(S_Q);
    }
    TS_STAMP(l, 1);
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < S_Q; ++j) {
      u32x4_t f0, f1;
      frags(j, f0, f1);
      const int kt = SLOT * j + 2 * w;
      acc = mfma(afrag(&s.a.xa[0][0], XLD, kt), f0, acc);
      acc = mfma(afrag(&s.a.xa[0][0], XLD, kt + 1), f1, acc);
    }
    red_put(0, acc);
    sync();
    if (w == 0) {
      const f32x4_t v = red_sum(0);
      if (qkv_glob) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rr = lk * 4 + i;
          if (rr < R) qkv_glob[(long long)rr * p.ldq_out + 16 * b + lm] = v[i] * s.rs[rr];
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rr = lk * 4 + i;
          if (rr < R) bst_c(__float_as_uint(v[i] * s.rs[rr]), wsr, (unsigned)OFF_QKV + (unsigned)(rr * NQKV + 16 * b + lm) * 4);
        }
        drain_stores();
        if (lane == 0) st_flag((unsigned*)(ws + OFF_QFL) + b, tagof(l, E_Q));
      }
    }
  };

  // A: attention of layer l for (row ar, kv head ahk), key split az; the head pair's rows go to every replica + flag
  // (the o_proj of this launch), or to att_glob (bf16 [R][2048] of the next launch).  given: the q/k/v rows are the
  // caller's (qkv_in), else the in-launch Q payload after its flags
  auto a_phase = [&](int l, bool given, unsigned* att_glob) {
    if (attb) {
      AttLds& at = s.a.at;
      constexpr int LPK = D / 8, GPW = 64 / LPK, G = NWC * GPW, IC = 4;
      const int r = ar, h = ahk;
      const int half = D / 2;
      const int bb = s.rmeta[3][r];
      const int kvpos = s.rmeta[1][r];
      const unsigned char* Kc = (const unsigned char*)lp(PT_KC, l) + (((size_t)bb * NKV + h) * p.Lmax) * D * 2;
      const unsigned char* Vc = (const unsigned char*)lp(PT_VC, l) + (((size_t)bb * NKV + h) * p.Lmax) * D * 2;
      const int grp = lane / LPK, sub = lane % LPK;
      const int gid = w * GPW + grp;
      const int start = s.rmeta[2][r];
      const int n = kvpos + 1 - start;  // keys [start, kvpos]; the last one (the new key) from LDS
      const int per_split = (n + NSPL - 1) / NSPL;
      const int j_lo = min(n, az * per_split), j_hi = min(n, j_lo + per_split);
      unsigned kr[IC][4], vr[IC][4], kn[IC][4], vn[IC][4];
      auto load_into = [&](int j0, unsigned (*kd)[4], unsigned (*vd)[4]) {
#pragma unroll
        for (int c = 0; c < IC; ++c) {
          const int jj = min(j0 + c * G, max(n - 2, 0));
          const u32x4_t a = *(const u32x4_t*)(Kc + ((size_t)(start + jj) * D + sub * 8) * 2);
          const u32x4_t bv = *(const u32x4_t*)(Vc + ((size_t)(start + jj) * D + sub * 8) * 2);
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4) { kd[c][q4] = a[q4]; vd[c][q4] = bv[q4]; }
        }
      };
      load_into(j_lo + gid, kr, vr);  // the cached keys do not depend on the q/k/v edge: in flight during its wait
      // the norm weights and rotary rows neither
      const bool act = lane < half;
      float nw0 = 0.f, nw1 = 0.f, c0 = 0.f, s0 = 0.f;
      if (w <= NREP && act) {
        const float* nw = (const float*)lp(w < NREP ? PT_QN : PT_KN, l);
        const int pos = s.rmeta[0][r];
        nw0 = nw[lane]; nw1 = nw[lane + half];
        c0 = p.cos_tab[(long long)pos * half + lane]; s0 = p.sin_tab[(long long)pos * half + lane];
      }
      // q heads 2 ahk, 2 ahk + 1 = tiles 16 ahk .. +16, k head: 128 + 8 ahk .. +8, v head: 192 + 8 ahk .. +8
      if (w == 0 && !given) {
        const unsigned tag = tagof(l, E_Q);
        for (int spins = 0;; ++spins) {
          const int t = lane < 16 ? 16 * ahk + lane : (lane < 24 ? 128 + 8 * ahk + lane - 16 : 192 + 8 * ahk + lane - 24);
          const bool ok = lane >= 32 || ld_flag((const unsigned*)(ws + OFF_QFL) + t) == tag;
          if (__all(ok)) break;
          if (spins > pk.spin) { if (lane == 0) atomicOr(err, 1); break; }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      sync();
      if (w < NREP + 2) {  // q heads / new k / new v: norm + rope, the cache append
        const int hh = w < NREP ? h * NREP + w : (w == NREP ? NQ + h : NQ + NKV + h);
        float x0 = 0.f, x1 = 0.f;
        if (given) {  // the caller's rows (written before this launch)
          const float* src = p.qkv_in + (long long)r * p.ldq_in + hh * D;
          if (act) { x0 = src[lane]; x1 = src[lane + half]; }
        } else {
          const unsigned o = (unsigned)OFF_QKV + (unsigned)(r * NQKV + hh * D) * 4;
          x0 = act ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(wsr, (int)(o + lane * 4), 0, SC1)) : 0.f;
          x1 = act ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(wsr, (int)(o + (lane + half) * 4), 0, SC1)) : 0.f;
        }
        if (w <= NREP) {
          const float rs = rsqrtf(wave_sum(x0 * x0 + x1 * x1) / (float)D + p.eps);
          if (act) { x0 = nw0 * (x0 * rs); x1 = nw1 * (x1 * rs); }
          if (act) {
            const float y0 = x0 * c0 - x1 * s0, y1 = x1 * c0 + x0 * s0;
            x0 = y0; x1 = y1;
          }
        }
        if (act) {
          float* dst = w < NREP ? at.qs[w] : (w == NREP ? at.knew : at.vnew);
          if (w >= NREP) { x0 = bf2f(f2bf(x0)); x1 = bf2f(f2bf(x1)); }
          dst[lane] = x0; dst[lane + half] = x1;
          if (w >= NREP && az == NSPL - 1) {  // the split that holds the new key appends it
            bf16_t* cache = (bf16_t*)lp(w == NREP ? PT_KC : PT_VC, l) + (((size_t)bb * NKV + h) * p.Lmax + kvpos) * D;
            cache[lane] = f2bf(x0);
            cache[lane + half] = f2bf(x1);
          }
        }
      }
      sync();
      const float scale = rsqrtf((float)D) * 1.4426950408889634f;
      float q[NREP][8];
#pragma unroll
      for (int j = 0; j < NREP; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) q[j][i] = at.qs[j][sub * 8 + i] * scale;
      float m[NREP], lsum[NREP], o[NREP][8];
#pragma unroll
      for (int j = 0; j < NREP; ++j) {
        m[j] = -INFINITY; lsum[j] = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[j][i] = 0.f;
      }
      auto consume = [&](auto& kd, auto& vd, const int jb) {
        float vf[IC][8], dd[NREP][IC];
#pragma unroll
        for (int c = 0; c < IC; ++c) {
          const bool valid = jb + c * G < j_hi;
          float kf[8];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            kf[2 * i] = __uint_as_float(kd[c][i] << 16); kf[2 * i + 1] = __uint_as_float(kd[c][i] & 0xFFFF0000u);
            vf[c][2 * i] = __uint_as_float(vd[c][i] << 16); vf[c][2 * i + 1] = __uint_as_float(vd[c][i] & 0xFFFF0000u);
          }
          if (jb + c * G >= n - 1) {
#pragma unroll
            for (int i = 0; i < 8; ++i) { kf[i] = at.knew[sub * 8 + i]; vf[c][i] = at.vnew[sub * 8 + i]; }
          }
#pragma unroll
          for (int j = 0; j < NREP; ++j) {
            float d = 0.f;
#pragma unroll
            for (int i = 0; i < 8; ++i) d += q[j][i] * kf[i];
            d = group_sum_dpp<LPK>(d);
            dd[j][c] = valid ? d : -INFINITY;
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
          lsum[j] = lsum[j] * f + es;
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
      for (int j0 = j_lo + gid; j0 < j_hi; j0 += 2 * GIC) {
        load_into(j0 + GIC, kn, vn);
        consume(kr, vr, j0);
        if (j0 + GIC >= j_hi) break;
        load_into(j0 + 2 * GIC, kr, vr);
        consume(kn, vn, j0 + GIC);
      }
#pragma unroll
      for (int off = LPK; off < 64; off <<= 1) {
#pragma unroll
        for (int j = 0; j < NREP; ++j) {
          const float m2 = __shfl_xor(m[j], off, 64), l2 = __shfl_xor(lsum[j], off, 64);
          const float mn = fmaxf(m[j], m2);
          const float f1 = m[j] == -INFINITY ? 0.f : exp2_hw(m[j] - mn);
          const float f2 = m2 == -INFINITY ? 0.f : exp2_hw(m2 - mn);
          lsum[j] = lsum[j] * f1 + l2 * f2;
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
          if (sub == 0) { at.mrg_ml[w][j][0] = m[j]; at.mrg_ml[w][j][1] = lsum[j]; }
#pragma unroll
          for (int i = 0; i < 8; ++i) at.mrg_o[w][j][sub * 8 + i] = o[j][i];
        }
      }
      sync();
      // this split's partial (m, l, o[D]) per q head, merged over the 8 waves: to LDS (split 0) or as granules to
      // split 0 of the pair
      u64* apart = (u64*)(ws + OFF_APART) + (size_t)apair * (NSPL - 1) * AREC;
      for (int e = tid; e < NREP * (D + 2); e += NWC * 64) {
        const int j = e / (D + 2), d = e % (D + 2);
        float mm = -INFINITY;
        for (int ww = 0; ww < NWC; ++ww) mm = fmaxf(mm, at.mrg_ml[ww][j][0]);
        float ll = 0.f, oo = 0.f;
        for (int ww = 0; ww < NWC; ++ww) {
          const float mw = at.mrg_ml[ww][j][0];
          const float f = mw == -INFINITY ? 0.f : exp2_hw(mw - mm);
          ll += at.mrg_ml[ww][j][1] * f;
          if (d >= 2) oo += at.mrg_o[ww][j][d - 2] * f;
        }
        const float v = d == 0 ? mm : (d == 1 ? ll : oo);
        if (az == 0) at.part[e] = v;
        else st_g(apart + (size_t)(az - 1) * AREC + e, __float_as_uint(v), tagof(l, E_AP));
      }
      if (az == 0) {  // (block-uniform)
      sync();
      if (tid < NREP * D / 2) {  // split 0: merge the NSPL partials in split order -> the head pair's output, bf16 pairs
        float res[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int e = 2 * tid + u, j = e / D, d = e % D;
          float ms[NSPL], ls[NSPL], os[NSPL];
          ms[0] = at.part[j * (D + 2)]; ls[0] = at.part[j * (D + 2) + 1]; os[0] = at.part[j * (D + 2) + 2 + d];
          // the other splits' (m, l, o[d]): all 3 x (NSPL - 1) granules in flight at once, re-polled until tagged
          const unsigned want = tagof(l, E_AP);
          u64 gx[NSPL - 1][3];
          auto gaddr = [&](int z, int q3) { return apart + (size_t)(z - 1) * AREC + j * (D + 2) + (q3 < 2 ? q3 : 2 + d); };
#pragma unroll
          for (int z = 1; z < NSPL; ++z)
#pragma unroll
            for (int q3 = 0; q3 < 3; ++q3) gx[z - 1][q3] = ld_g(gaddr(z, q3));
          for (int spins = 0;; ++spins) {
            bool ok = true;
#pragma unroll
            for (int z = 1; z < NSPL; ++z)
#pragma unroll
              for (int q3 = 0; q3 < 3; ++q3) ok = ok && (unsigned)(gx[z - 1][q3] >> 32) == want;
            if (ok) break;
            if (spins > pk.spin) { atomicOr(err, 1); break; }
            __builtin_amdgcn_s_sleep(1);
#pragma unroll
            for (int z = 1; z < NSPL; ++z)
#pragma unroll
              for (int q3 = 0; q3 < 3; ++q3)
                if ((unsigned)(gx[z - 1][q3] >> 32) != want) gx[z - 1][q3] = ld_g(gaddr(z, q3));
          }
#pragma unroll
          for (int z = 1; z < NSPL; ++z) {
            ms[z] = __uint_as_float((unsigned)gx[z - 1][0]);
            ls[z] = __uint_as_float((unsigned)gx[z - 1][1]);
            os[z] = __uint_as_float((unsigned)gx[z - 1][2]);
          }
          float mm = -INFINITY;
#pragma unroll
          for (int z = 0; z < NSPL; ++z) mm = fmaxf(mm, ms[z]);
          float ll = 0.f, oo = 0.f;
#pragma unroll
          for (int z = 0; z < NSPL; ++z) {
            const float f = ms[z] == -INFINITY ? 0.f : exp2_hw(ms[z] - mm);
            ll += ls[z] * f;
            oo += os[z] * f;
          }
          res[u] = oo / ll;
        }
        at.out[tid] = pack2bf(res[0], res[1]);
      }
      sync();
      if (att_glob) {  // the next launch's attention rows: row r, pairs 128 h .. + 128
        if (w == 0) {
#pragma unroll
          for (int k = 0; k < 2; ++k) att_glob[(long long)r * (p.lda_out / 2) + 128 * h + lane + 64 * k] = at.out[lane + 64 * k];
        }
      } else if (w == 0) {  // to every replica: [K half h / 4][row r][pairs 128 (h % 4) .. + 128] (replica = [2][MAXR][512])
        const unsigned o = (unsigned)OFF_ATT + (unsigned)(((h >> 2) * MAXR + r) * (KO / 4) + (h & 3) * (NREP * D / 2)) * 4;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const unsigned v = at.out[lane + 64 * k];
#pragma unroll
          for (int rp = 0; rp < NREPL; ++rp) bst_c(v, wsr, o + rp * (unsigned)REPL_ATT + (lane + 64 * k) * 4);
        }
        drain_stores();
        if (lane < NREPL) st_flag((unsigned*)(ws + fl_off(lane, FL_A)) + apair, tagof(l, E_A));
      }
      }
    }
  };

  for (int li = 0; li < L; ++li) {
    const int l = l0 + li;
    refresh();
    lm = lane & 15;
    lk = lane >> 4;
    TS_STAMP(l, 0);
    const bool given_att = li == 0 && ain;  // this layer's attention rows come from the caller (no Q, no A)
    const bool given = li == 0 && (qin || ain);  // this layer's q/k/v rows come from the caller
    // ------------------------------------------------------------------ Q
    if (!given) q_phase(l, li == 0, nullptr);
    TS_STAMP(l, 2);
    // ------------------------------------------------------------------ A
    if (!given_att) a_phase(l, given, nullptr);
    TS_STAMP(l, 3);
    // ------------------------------------------------------------------ O: o_proj (K half) + residual
    pretake(S_O + 6);  // o_proj + the first 6 gate/up slots, across the attention hand-off
    {
      // producers of K half kh: the attention blocks (r, hk) with hk / 4 == kh, r < R -> flags 8 r + 4 kh .. + 4
      if (w == 0 && !given_att) {
        const unsigned tag = tagof(l, E_A);
        for (int spins = 0;; ++spins) {
          const int rr = lane >> 2, q = lane & 3;
          const bool ok = rr >= R || ld_flag((const unsigned*)(ws + fl_off(myrep, FL_A)) + 8 * rr + 4 * kh + q) == tag;
          if (__all(ok)) break;
          if (spins > pk.spin) { if (lane == 0) atomicOr(err, 1); break; }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      sync();
      {  // the attention rows' K half: thread -> row tid / 64, 2 x 16 B (the caller's rows, or the replica)
        const int row = tid >> 6;
        const unsigned base = (unsigned)(OFF_ATT + myrep * REPL_ATT) + (unsigned)kh * (unsigned)(MAXR * (KO / 4) * 4) +
                              (unsigned)(row * (KO / 4)) * 4;
        u32x4_t v[2];
        if (given_att) {
          const u32x4_t* src = (const u32x4_t*)((const unsigned*)p.att_in + (long long)row * (p.lda_in / 2) + kh * (KO / 4));
#pragma unroll
          for (int k = 0; k < 2; ++k) v[k] = row < R ? src[lane + 64 * k] : u32x4_t{0u, 0u, 0u, 0u};
        } else {
#pragma unroll
          for (int k = 0; k < 2; ++k) v[k] = row < R ? bld_c(wsr, base + (lane + 64 * k) * 16) : u32x4_t{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) *(u32x4_t*)&s.a.aa[row][(lane + 64 * k) * 8] = v[k];
      }
      sync();
      TS_STAMP(l, 4);
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < S_O; ++j) {
        u32x4_t f0, f1;
        frags(j, f0, f1);
        const int kt = SLOT * j + 2 * w;
        acc = mfma(afrag(&s.a.aa[0][0], ALD, kt), f0, acc);
        acc = mfma(afrag(&s.a.aa[0][0], ALD, kt + 1), f1, acc);
      }
      red_put(0, acc);
      sync();
      if (w == 0) {
        const f32x4_t v = red_sum(0);
        if (owner) {
          pair_in(v, 0, tagof(l, E_PO));
          publish_x16(0, tagof(l, E_X1));
        } else {
          pair_out(v, 0, tagof(l, E_PO));
        }
      }
    }
    TS_STAMP(l, 5);
    // ------------------------------------------------------------------ GU: gate/up (3 tiles) + SwiGLU
    {
      poll(fl_off(myrep, FL_X1), 128, tagof(l, E_X1));
      sync();
      stage_x16(0);
      TS_STAMP(l, 6);
#pragma unroll
      for (int t3 = 0; t3 < 3; ++t3) {
        f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int k = 4 * t3 + j;  // gate/up slot k = pre-taken slot S_O + k while k < 6
          u32x4_t f0, f1;
          frags(S_O + k < S_O + 6 ? S_O + k : NPRE, f0, f1);
          const int kt = SLOT * j + 2 * w;
          acc = mfma(afrag(&s.a.xa[0][0], XLD, kt), f0, acc);
          acc = mfma(afrag(&s.a.xa[0][0], XLD, kt + 1), f1, acc);
        }
        red_put(t3 & 1, acc);
        sync();
        if (w == 0 && lane < MAXR * 4) {
          const int rr = lane >> 2, pp = lane & 3;
          const int ml = (rr >> 2) * 16 + 2 * pp, e = rr & 3;
          float g0 = 0.f, g1 = 0.f, u0 = 0.f, u1 = 0.f;
#pragma unroll
          for (int ww = 0; ww < NWC; ++ww) {
            g0 += s.red[t3 & 1][ww][ml][e]; g1 += s.red[t3 & 1][ww][ml + 1][e];
            u0 += s.red[t3 & 1][ww][ml + 8][e]; u1 += s.red[t3 & 1][ww][ml + 9][e];
          }
          const float rsv = s.rs[rr];
          s.hb[t3][rr][pp] = pack2bf(silu_f(g0 * rsv) * (u0 * rsv), silu_f(g1 * rsv) * (u1 * rsv));
        }
      }
      if (w == 0) {
        for (int q = lane; q < 3 * MAXR * 4; q += 64) {
          const int t3 = q / (MAXR * 4), rr = (q >> 2) % MAXR, pp = q & 3;
          if (rr < R) {
            const unsigned o = (unsigned)OFF_H + (unsigned)(rr * (I / 2) + (b + NB * t3) * 4 + pp) * 4;
#pragma unroll
            for (int rp = 0; rp < NREPL; ++rp) bst_c(s.hb[t3][rr][pp], wsr, o + rp * (unsigned)REPL_H);
          }
        }
        drain_stores();
        if (lane < NREPL) st_flag((unsigned*)(ws + fl_off(lane, FL_H)) + b, tagof(l, E_H));
      }
    }
    TS_STAMP(l, 7);
    // ------------------------------------------------------------------ D: down (K half) + residual
    {
      pretake(S_D);
      poll(fl_off(myrep, FL_H), NB, tagof(l, E_H));
      sync();
      {
        const int row = tid >> 6;
        const unsigned base = (unsigned)(OFF_H + myrep * REPL_H) + (unsigned)(row * (I / 2) + kh * (I / 4)) * 4;
        u32x4_t v[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) v[k] = row < R ? bld_c(wsr, base + (lane + 64 * k) * 16) : u32x4_t{0u, 0u, 0u, 0u};
#pragma unroll
        for (int k = 0; k < 6; ++k) *(u32x4_t*)&s.a.ha[row][(lane + 64 * k) * 8] = v[k];
      }
      sync();
      TS_STAMP(l, 8);
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < S_D; ++j) {
        u32x4_t f0, f1;
        frags(j, f0, f1);
        const int kt = SLOT * j + 2 * w;
        acc = mfma(afrag(&s.a.ha[0][0], HLD, kt), f0, acc);
        acc = mfma(afrag(&s.a.ha[0][0], HLD, kt + 1), f1, acc);
      }
      red_put(0, acc);
      sync();
      if (w == 0) {
        const f32x4_t v = red_sum(0);
        if (owner) {
          pair_in(v, 1, tagof(l, E_PD));
          if (li + 1 == L) {  // the launch's output rows
            for (int q = lane; q < MAXR * 16; q += 64) {
              const int rr = q >> 4, c = q & 15;
              if (rr < R) p.x[(long long)rr * p.ldx + 16 * ot + c] = s.xo[rr][c];
            }
          }
          if (li + 1 < L || qout || aout) publish_x16(1, tagof(l, E_X2));
        } else {
          pair_out(v, 1, tagof(l, E_PD));
        }
      }
    }
    TS_STAMP(l, 9);
  }
  if (qout || aout) {  // the next launch's q/k/v rows (layer l0 + L), or its attention rows
    refresh();
    lm = lane & 15;
    lk = lane >> 4;
    q_phase(l0 + L, false, aout ? nullptr : p.qkv_out);
    if (aout) a_phase(l0 + L, false, (unsigned*)p.att_out);
  }
  if (b == 0 && tid == 0)
    __hip_atomic_store((unsigned*)(ws + OFF_EPOCH), ep + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

bool step_resident() {
  static int cap[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
  if (cap[dev] == 0) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)talker_step_k, NT, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return false;
    cap[dev] = std::max(1, per_cu * cus);
  }
  return cap[dev] >= NB;
}

}  // namespace

extern "C" long long qt_talker_step_ws_bytes(void) { return (long long)WS_BYTES; }
extern "C" long long qt_talker_step_stamp_bytes(void) { return (long long)STAMP_BYTES; }

extern "C" int qt_talker_step_supported(int H_, int I_, int Hq, int Hkv, int D_, int n_layers) {
  return H_ == H && I_ == I && Hq == NQ && Hkv == NKV && D_ == D && n_layers >= 1 && n_layers <= MAXL &&
         step_resident();
}

extern "C" int qt_talker_step(const qt_talker_step_args* a, void* stream) {
  if (!a || a->R < 1 || a->R > MAXR || a->n_layers < 1 || a->total_layers > MAXL || a->first_layer < 0 ||
      a->first_layer + a->n_layers > a->total_layers || (a->qkv_out && a->first_layer + a->n_layers >= a->total_layers))
    return QT_ERR_SHAPE;
  if ((a->qkv_in && a->ldq_in < NQKV) || (a->qkv_out && a->ldq_out < NQKV)) return QT_ERR_SHAPE;
  if ((a->att_in && (a->qkv_in || a->lda_in < KO || ((reinterpret_cast<uintptr_t>(a->att_in) | (a->lda_in * 2)) & 15))) ||
      (a->att_out && (a->qkv_out || a->lda_out < KO || (a->lda_out & 1) ||
                      a->first_layer + a->n_layers >= a->total_layers)))
    return QT_ERR_SHAPE;
  if (!a->ws || a->ws_bytes < (long long)WS_BYTES || !a->wtab || !a->x || !a->cos_tab || !a->sin_tab ||
      !a->rope_pos || !a->kv_pos || !a->row_start || !a->row_batch)
    return QT_ERR_ARG;
  if (a->ldx < H || (a->ldx & 3) || (reinterpret_cast<uintptr_t>(a->x) & 15) || a->Lmax < 2) return QT_ERR_SHAPE;
  if (!step_resident()) return QT_ERR_SHAPE;
  static const int spin = std::max(1000, qt_knob("QT_TS_SPIN", 200000));
  static const int nwl = std::min(NWL, std::max(1, qt_knob("QT_TS_NWL", NWL)));
  static const int depth = std::min(2, std::max(1, qt_knob("QT_TS_DEPTH", 2)));
  hipLaunchKernelGGL(talker_step_k, dim3(NB), dim3(NT), 0, (hipStream_t)stream, SP{*a, spin, nwl, depth});
  return hipGetLastError() == hipSuccess ? QT_OK : QT_ERR_LAUNCH;
}
