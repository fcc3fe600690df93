// Talker decode-layer tail engine for gfx950: ONE persistent launch runs the part of a talker decoder layer after its
// attention -- o_proj + residual -> post-attention RMSNorm + gate/up + SwiGLU -> down + residual -> the NEXT layer's
// input RMSNorm + q/k/v projection -- for up to 8 batch rows, where the launch chain issued four weight-streaming
// GEMV kernels.  Replaces M:961-1012 after the attention call (o_proj M:804, residual M:991, MLP
// M:995-1004 with Qwen3TTSTalkerTextMLP / the talker's SwiGLU) and the next layer's input_layernorm + q/k/v
// projections (M:985, M:752-754) of Qwen3TTSTalkerModel.forward's decode step (M:1430-1480).
//
// Why one launch: the four GEMVs stream 101 MB of bf16 weights per layer (1.7B talker); as separate launches each pays
// a launch ramp and tail (3.3 TB/s over the four, `profiles/r05_bench_line.json` kernel table).  Here the weights
// stream continuously: two LOADER waves per workgroup move the block's weight fragments, in the order the block
// consumes them, into an LDS ring by LDS-DMA (global_load_lds, non-temporal: read once per frame), running ahead of
// the eight CONSUMER waves by up to the ring's depth -- so the weights of the next phase arrive while the consumers
// wait for a hand-off -- and the consumers, whose own loads are only the hand-off polls and payloads, never wait
// behind a weight round trip (vmcnt retires in order per wave).
//
// Geometry, for a talker of hidden size H and intermediate size I = 3 H (the config's; the 1.7B talker H 2048, the 0.6B
// H 1024): NB = H / 8 workgroups (one per CU, all resident -- the host checks the occupancy) x (8 consumer + 2 loader)
// waves.  Block b:  o_proj and down: output tile t = b / 2 (16 of H columns), K half b % 2 (split-K pair; the even
// block OWNS x[rows][16t .. 16t + 16) and receives the odd block's partial as 8-byte {value, tag} granules);
// gate/up: tiles b, b + NB, b + 2 NB (I / 8 tiles of 8 gate + 8 up columns); next q/k/v: tiles b, b + NB, ... (256
// tiles of the 4096-wide q/k/v).
// Hand-offs: x16 after each residual (all-to-all) and the SwiGLU rows (all-to-all) in the R1 form with one replica
// per XCD (as qt_cp_step), the split-K pairs as granules.  Tags: epoch * 8 + edge + 1, the epoch a launch counter in
// the workspace advanced by block 0 at the end.
#include "common.h"
#include "engine_dev.h"
#include <algorithm>

namespace {

using namespace qt_engine;

constexpr int NQKV = 4096, KO = 2048;                    // q/k/v width, o_proj K (16 q heads x 128): both talkers
constexpr int NBMAX = 256, NWC = 8, NWL = 2, NT = (NWC + NWL) * 64, MAXR = 8;
constexpr int NSLOT = 5, SLOT = 16;                       // ring: 5 slots x 16 fragments (16 KiB)
constexpr int KTO = KO / 32, ALD = KO / 2 + 8;
constexpr int NEDGE = 8;
constexpr int NPRE = 8;  // ring slots a consumer wave holds in registers across a hand-off wait
constexpr int E_PO = 0, E_X1 = 1, E_H = 2, E_PD = 3, E_X2 = 4;
constexpr int HMAX = 2048, IMAX = 6144;

// per-config constants: H hidden, I intermediate
template <int H_, int I_>
struct TC {
  static constexpr int H = H_, I = I_;
  static constexpr int NB = H / 8;                        // workgroups: split-K pairs over the H / 16 output tiles
  static constexpr int NGU = I / H;                       // gate/up tiles per block (I / 8 tiles over NB blocks)
  static constexpr int NQT = (NQKV / 16) / NB;            // next-layer q/k/v tiles per block
  static constexpr int KTH = H / 32, KTI = I / 32;        // k tiles
  static constexpr int SPT = KTH / SLOT;                  // ring slots per H-deep tile (gate/up, q/k/v)
  static constexpr int XLD = H + 8, HLD = I / 2 + 8;
  // slots per phase: o_proj 32 k tiles, gate/up NGU tiles x KTH, down KTI / 2 k tiles, q/k/v NQT tiles x KTH
  static constexpr int S_O = KTO / 2 / SLOT, S_GU = NGU * SPT, S_D = KTI / 2 / SLOT, S_Q = NQT * SPT;
  static_assert(I % H == 0 && (NQKV / 16) % NB == 0 && KTH % SLOT == 0 && (KTI / 2) % SLOT == 0, "geometry");
  static_assert(S_O == 2 && S_D <= NPRE && NB <= NBMAX, "slot plan");
  static constexpr int NXK = H / 512, NHK = I / 1024;     // 16-byte loads per lane: an x16 row, a SwiGLU K half
};

// workspace (bytes; one layout, sized for the largest config)
constexpr size_t OFF_ERR = 0, OFF_EPOCH = 4;
constexpr int NREPL = 8;
constexpr int FL_X1 = 0, FL_H = 1, FL_X2 = 2;
constexpr size_t OFF_FLAGS = 256, REPL_FLAGS = (size_t)3 * NBMAX * 4;
constexpr size_t OFF_PART = OFF_FLAGS + NREPL * REPL_FLAGS;             // [2][128 tiles][MAXR][16] granules
constexpr size_t OFF_X16 = OFF_PART + (size_t)2 * 128 * MAXR * 16 * 8;
constexpr size_t REPL_X16 = (size_t)2 * MAXR * (HMAX / 2) * 4;         // [2 bufs][MAXR][H/2] bf16 pairs
constexpr size_t OFF_H = OFF_X16 + NREPL * REPL_X16;
constexpr size_t REPL_H = (size_t)MAXR * (IMAX / 2) * 4;               // [MAXR][I/2] bf16 pairs
constexpr size_t WS_BYTES = OFF_H + NREPL * REPL_H;
constexpr size_t STAMP_BYTES = (size_t)NBMAX * 32 * 8;                 // optional per-block phase stamps
// optional stage records after the stamps (a workspace STAMP_BYTES + DBG_BYTES larger; the stage-by-stage parity
// tests): fp32 [4][MAXR][IMAX] -- x after the o_proj residual, the SwiGLU output, x after the MLP residual, the next
// layer's q/k/v rows
constexpr size_t DBG_BYTES = (size_t)4 * MAXR * IMAX * 4;

struct TP {
  qt_talker_tail_args a;
  int spin;
};

template <class C>
struct TLds {
  __attribute__((aligned(16))) unsigned char ring[NSLOT][SLOT * 1024];
  union {
    bf16_t xa[MAXR][C::XLD];  // x16 rows: the A operand of gate/up and q/k/v
    bf16_t aa[MAXR][ALD];     // the attention rows' K half: the A operand of o_proj
    bf16_t ha[MAXR][C::HLD];  // the SwiGLU rows' K half: the A operand of down
  } a;
  float red[2][NWC][64][4];                     // per-wave MFMA partials (double-buffered: gate/up tiles)
  float rs[MAXR];                               // 1 / rms per row
  float xo[MAXR][16];                           // owner: the residual slice (fp32)
  unsigned hb[C::NGU][MAXR][4];                 // this block's SwiGLU output pairs
  __attribute__((aligned(16))) bf16_t zero[32];
  unsigned full[NSLOT];                         // ring slot s % NSLOT holds sequence number s (+1)
  unsigned done[NWC];                           // consumer wave w has finished with sequences < done[w]
};

template <class C>
__global__ __launch_bounds__(NT) void talker_tail_k(TP pk) {
  constexpr int H = C::H, I = C::I, NB = C::NB, KTH = C::KTH, KTI = C::KTI, SPT = C::SPT, NGU = C::NGU;
  constexpr int S_O = C::S_O, S_GU = C::S_GU, S_D = C::S_D, S_Q = C::S_Q, XLD = C::XLD, HLD = C::HLD;
  const qt_talker_tail_args& p = pk.a;
  __shared__ TLds<C> s;
  __shared__ unsigned cb_cnt, cb_gen;
  const int b = blockIdx.x;
  const int ot = b >> 1, kh = b & 1;  // o_proj / down: tile, K half
  const bool owner = kh == 0;
  const int R = p.R;
  const bool has_next = p.w_qkv_next != nullptr;
  char* ws = (char*)p.ws;
  int* err = (int*)(ws + OFF_ERR);
  const int myrep = b % NREPL;
  auto fl_off = [&](int rp, int kind) { return (unsigned)(OFF_FLAGS + rp * REPL_FLAGS + kind * NB * 4); };
  u64* gpart = (u64*)(ws + OFF_PART);
  const rsrc_t wsr = mkr(ws, (unsigned)WS_BYTES);
  const unsigned ep = (unsigned)(ld_g((const u64*)(ws + OFF_ERR)) >> 32);
  auto tagof = [&](int e) { return ep * NEDGE + (unsigned)e + 1u; };
  u64* stamps = p.ws_bytes >= (long long)(WS_BYTES + STAMP_BYTES) ? (u64*)(ws + WS_BYTES) + b * 32 : nullptr;
  float* dbg = p.ws_bytes >= (long long)(WS_BYTES + STAMP_BYTES + DBG_BYTES) ? (float*)(ws + WS_BYTES + STAMP_BYTES)
                                                                              : nullptr;
#define TT_STAMP(k) \
  if (kProbe && stamps && threadIdx.x == 0) stamps[(k)] = __builtin_amdgcn_s_memrealtime();
  TT_STAMP(0);
  const int nseq = S_O + S_GU + S_D + (has_next ? S_Q : 0);
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;

  if (tid < NSLOT) s.full[tid] = 0u;
  else if (tid >= 64 && tid < 64 + NWC) s.done[tid - 64] = 0u;
  else if (tid >= 128 && tid < 144) ((unsigned*)s.zero)[tid - 128] = 0u;
  if (tid == 0) { cb_cnt = 0u; cb_gen = 0u; }
  __syncthreads();  // (the last block-wide barrier: the loader waves run free from here)

  if (w >= NWC) {
    // ------------------------------------------------------------------ loader waves
    const int lw = w - NWC;
    for (int sq = lw; sq < nseq; sq += NWL) {
      const void* W;
      int tile, kt0, KT;
      if (sq < S_O) { W = p.w_o; tile = ot; kt0 = kh * (KTO / 2) + SLOT * sq; KT = KTO; }
      else if (sq < S_O + S_GU) { const int j = sq - S_O; W = p.w_gu; tile = b + NB * (j / SPT); kt0 = SLOT * (j % SPT); KT = KTH; }
      else if (sq < S_O + S_GU + S_D) { const int j = sq - S_O - S_GU; W = p.w_down; tile = ot; kt0 = kh * (KTI / 2) + SLOT * j; KT = KTI; }
      else { const int j = sq - S_O - S_GU - S_D; W = p.w_qkv_next; tile = b + NB * (j / SPT); kt0 = SLOT * (j % SPT); KT = KTH; }
      const int slot = sq % NSLOT;
      if (sq >= NSLOT) {  // the slot's previous sequence consumed by every consumer wave
        for (int spins = 0;; ++spins) {
          unsigned m = 0xFFFFFFFFu;
#pragma unroll
          for (int c = 0; c < NWC; ++c) m = min(m, lds_ld(&s.done[c]));
          if ((int)__builtin_amdgcn_readfirstlane(m) >= sq - NSLOT + 1) break;
          // a full ring waits for the consumers, which may themselves sit in a hand-off poll of up to pk.spin x
          // (global sc1 load + s_sleep 1): bounded like cons_sync (64 x spin LDS polls), not by pk.spin, so the loader
          // never gives up (and overwrites a slot in use) before the consumers' own poll would
          if (spins > 64 * pk.spin) { if (lane == 0) atomicOr(err, 2); break; }
          __builtin_amdgcn_s_sleep(0);
        }
      }
      const char* src = (const char*)W + ((size_t)(tile * KT + kt0) << 10) + lane * 16;
      const unsigned dst = lds_u32(&s.ring[slot][0]);
#pragma unroll
      for (int f = 0; f < SLOT; ++f) glds16_nt(src + f * 1024, dst + f * 1024);
      // this wave's previous slot has landed once only this slot's 16 transfers are outstanding
      if (sq - NWL >= 0) {
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        if (lane == 0) lds_st(&s.full[(sq - NWL) % NSLOT], (unsigned)(sq - NWL + 1));
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int last = lw + NWL * ((nseq - 1 - lw) / NWL);  // this wave's last sequence
    if (lane == 0 && last < nseq) lds_st(&s.full[last % NSLOT], (unsigned)(last + 1));
    return;
  }

  // ------------------------------------------------------------------ consumer waves (tid < 512)
  CBar cb{&cb_cnt, &cb_gen};
  unsigned cg = 0;  // consumer barrier generation
  const int lm = lane & 15, lk = lane >> 4;
  int sq = 0;  // next ring sequence
  // one ring slot: wait until it is full, read this wave's two fragments, release it
  auto take = [&](u32x4_t& f0, u32x4_t& f1) {
    const int slot = sq % NSLOT;
    for (int spins = 0; (int)__builtin_amdgcn_readfirstlane(lds_ld(&s.full[slot])) < sq + 1; ++spins) {
      if (spins > pk.spin) { if (lane == 0) atomicOr(err, 4); break; }
      __builtin_amdgcn_s_sleep(0);
    }
    f0 = *(const u32x4_t*)&s.ring[slot][(2 * w) * 1024 + lane * 16];
    f1 = *(const u32x4_t*)&s.ring[slot][(2 * w + 1) * 1024 + lane * 16];
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f0), "+v"(f1)::"memory");
    ++sq;
    if (lane == 0) lds_st(&s.done[w], (unsigned)sq);
  };
  // Before each hand-off wait every consumer wave copies its fragments of the next phase's first n ring slots into
  // registers and releases the slots: the ring (5 LDS slots, ~3 us of stream) would otherwise fill during the wait
  // and stall the loaders; registers extend it by NPRE slots.
  u32x4_t pf[2 * NPRE];
  auto pretake = [&](int n) {  // (n <= NPRE)
#pragma unroll
    for (int k = 0; k < NPRE; ++k)
      if (k < n) take(pf[2 * k], pf[2 * k + 1]);
  };
  auto frags = [&](int k, int npre, u32x4_t& f0, u32x4_t& f1) {  // slot k of the phase: pre-taken or from the ring
    if (k < npre) { f0 = pf[2 * k]; f1 = pf[2 * k + 1]; } else take(f0, f1);
  };
  auto wait_flags = [&](unsigned off, int n, unsigned tag) {
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
    cons_sync<NWC>(cb, cg, pk.spin, err);
  };
  auto red_put = [&](int buf, f32x4_t acc) {
    s.red[buf][w][lane][0] = acc[0]; s.red[buf][w][lane][1] = acc[1];
    s.red[buf][w][lane][2] = acc[2]; s.red[buf][w][lane][3] = acc[3];
  };
  auto red_sum = [&](int buf) {  // (wave 0) the 8 waves' partials of MFMA lane `lane`, in wave order
    f32x4_t v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ww = 0; ww < NWC; ++ww) {
      v[0] += s.red[buf][ww][lane][0]; v[1] += s.red[buf][ww][lane][1];
      v[2] += s.red[buf][ww][lane][2]; v[3] += s.red[buf][ww][lane][3];
    }
    return v;
  };
  // x16 rows from replica myrep of buffer `buf` -> s.a.xa, 1 / rms per row: thread -> row tid / 64
  auto stage_x16 = [&](int buf) {
    const int row = tid >> 6;
    const unsigned base = (unsigned)(OFF_X16 + myrep * REPL_X16 + (size_t)buf * MAXR * (H / 2) * 4);
    u32x4_t v[C::NXK];
#pragma unroll
    for (int k = 0; k < C::NXK; ++k)
      v[k] = row < R ? bld_c(wsr, base + (unsigned)(row * (H / 2)) * 4 + (lane + 64 * k) * 16) : u32x4_t{0u, 0u, 0u, 0u};
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < C::NXK; ++k) {
      *(u32x4_t*)&s.a.xa[row][(lane + 64 * k) * 8] = v[k];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float lo = __uint_as_float(v[k][e] << 16), hi = __uint_as_float(v[k][e] & 0xFFFF0000u);
        ss += lo * lo + hi * hi;
      }
    }
    ss = wave_sum_dpp(ss);
    if (lane == 0) s.rs[row] = rsqrtf(ss / (float)H + p.eps);
    cons_sync<NWC>(cb, cg, pk.spin, err);
  };
  // (wave 0, owner) the split-K pair's partial of (row 4 lk + i, column lm) in, summed with this block's, + the
  // residual slice; returns through s.xo
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
  auto pair_out = [&](f32x4_t v, int kind, unsigned tag) {  // (wave 0, odd block) this block's partial to the owner
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rr = lk * 4 + i;
      if (rr < R) st_g(gpart + (((size_t)kind * 128 + ot) * MAXR + rr) * 16 + lm, __float_as_uint(v[i]), tag);
    }
  };
  // (wave 0, owner) the owned slice's bf16 copy to x16 buffer `buf` of every replica, drain, flags
  auto publish_x16 = [&](int buf, unsigned tag) {
    const int rr = lane >> 3, pp = lane & 7;  // 8 rows x 8 column pairs
    if (rr < R) {
      const unsigned v = pack2bf(s.xo[rr][2 * pp], s.xo[rr][2 * pp + 1]);
      const unsigned o = (unsigned)OFF_X16 + (unsigned)(((buf * MAXR + rr) * (H / 2)) + 8 * ot + pp) * 4;
#pragma unroll
      for (int rp = 0; rp < NREPL; ++rp) bst_c(v, wsr, o + rp * (unsigned)REPL_X16);
    }
    drain_stores();
    if (lane < NREPL) st_flag((unsigned*)(ws + fl_off(lane, buf == 0 ? FL_X1 : FL_X2)) + ot, tag);
  };
  auto afrag = [&](const bf16_t* row0, int ld, int nrows, int kt) {  // A fragment of k tile kt from staged rows
    return *(const u32x4_t*)(lm < nrows ? row0 + (size_t)lm * ld + kt * 32 + lk * 8 : &s.zero[lk * 8]);
  };

  // the owner's residual slice (fp32, 8 rows x 16) and this block's attention rows (K half), staged up front
  if (owner && tid < MAXR * 16) {
    const int rr = tid >> 4, c = tid & 15;
    s.xo[rr][c] = rr < R ? p.x[(long long)rr * p.ldx + 16 * ot + c] : 0.f;
  }
  {
    const int row = tid >> 6;  // 2 x 16 B per thread: 1024 bf16 per row
    u32x4_t v[2];
#pragma unroll
    for (int k = 0; k < 2; ++k)
      v[k] = row < R ? *(const u32x4_t*)((const bf16_t*)p.att + (long long)row * p.lda + kh * (KO / 2) + (lane + 64 * k) * 8)
                     : u32x4_t{0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 2; ++k) *(u32x4_t*)&s.a.aa[row][(lane + 64 * k) * 8] = v[k];
  }
  cons_sync<NWC>(cb, cg, pk.spin, err);
  TT_STAMP(1);
  // ------------------------------------------------------------------ o_proj (K half) + residual
  {
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < S_O; ++j) {
      u32x4_t f0, f1;
      take(f0, f1);
      const int kt = SLOT * j + 2 * w;
      acc = mfma(afrag(&s.a.aa[0][0], ALD, R, kt), f0, acc);
      acc = mfma(afrag(&s.a.aa[0][0], ALD, R, kt + 1), f1, acc);
    }
    red_put(0, acc);
    cons_sync<NWC>(cb, cg, pk.spin, err);
    if (w == 0) {
      const f32x4_t v = red_sum(0);
      if (owner) {
        pair_in(v, 0, tagof(E_PO));
        publish_x16(0, tagof(E_X1));
        if (dbg)
          for (int q = lane; q < MAXR * 16; q += 64)
            if ((q >> 4) < R) dbg[((size_t)0 * MAXR + (q >> 4)) * IMAX + 16 * ot + (q & 15)] = s.xo[q >> 4][q & 15];
      } else {
        pair_out(v, 0, tagof(E_PO));
      }
    }
    TT_STAMP(2);
  }
  // ------------------------------------------------------------------ gate/up (3 tiles) + SwiGLU
  {
    constexpr int npre = S_GU < NPRE ? S_GU : NPRE;
    pretake(npre);
    wait_flags(fl_off(myrep, FL_X1), H / 16, tagof(E_X1));
    TT_STAMP(3);
    stage_x16(0);
    TT_STAMP(4);
#pragma unroll
    for (int t3 = 0; t3 < NGU; ++t3) {
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < SPT; ++j) {
        u32x4_t f0, f1;
        frags(SPT * t3 + j, npre, f0, f1);
        const int kt = SLOT * j + 2 * w;
        acc = mfma(afrag(&s.a.xa[0][0], XLD, R, kt), f0, acc);
        acc = mfma(afrag(&s.a.xa[0][0], XLD, R, kt + 1), f1, acc);
      }
      red_put(t3 & 1, acc);
      cons_sync<NWC>(cb, cg, pk.spin, err);
      if (w == 0 && lane < MAXR * 4) {  // SwiGLU of (row rr, column pair pp) of tile b + 256 t3
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
    if (w == 0) {  // this block's 3 tiles x 8 rows x 4 pairs to every replica, drain, flags
      for (int q = lane; q < NGU * MAXR * 4; q += 64) {
        const int t3 = q / (MAXR * 4), rr = (q >> 2) % MAXR, pp = q & 3;
        if (rr < R) {
          const unsigned o = (unsigned)OFF_H + (unsigned)(rr * (I / 2) + (b + NB * t3) * 4 + pp) * 4;
#pragma unroll
          for (int rp = 0; rp < NREPL; ++rp) bst_c(s.hb[t3][rr][pp], wsr, o + rp * (unsigned)REPL_H);
          if (dbg) {
            const size_t e = ((size_t)1 * MAXR + rr) * IMAX + (b + NB * t3) * 8 + 2 * pp;
            dbg[e] = __uint_as_float(s.hb[t3][rr][pp] << 16);
            dbg[e + 1] = __uint_as_float(s.hb[t3][rr][pp] & 0xFFFF0000u);
          }
        }
      }
      drain_stores();
      if (lane < NREPL) st_flag((unsigned*)(ws + fl_off(lane, FL_H)) + b, tagof(E_H));
    }
    TT_STAMP(5);
  }
  // ------------------------------------------------------------------ down (K half) + residual
  {
    pretake(S_D);
    wait_flags(fl_off(myrep, FL_H), NB, tagof(E_H));
    TT_STAMP(6);
    {  // the SwiGLU rows' K half: thread -> row tid / 64, 6 x 16 B
      const int row = tid >> 6;
      const unsigned base = (unsigned)(OFF_H + myrep * REPL_H) + (unsigned)(row * (I / 2) + kh * (I / 4)) * 4;
      u32x4_t v[C::NHK];
#pragma unroll
      for (int k = 0; k < C::NHK; ++k) v[k] = row < R ? bld_c(wsr, base + (lane + 64 * k) * 16) : u32x4_t{0u, 0u, 0u, 0u};
#pragma unroll
      for (int k = 0; k < C::NHK; ++k) *(u32x4_t*)&s.a.ha[row][(lane + 64 * k) * 8] = v[k];
    }
    cons_sync<NWC>(cb, cg, pk.spin, err);
    TT_STAMP(7);
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < S_D; ++j) {
      u32x4_t f0, f1;
      frags(j, S_D, f0, f1);
      const int kt = SLOT * j + 2 * w;
      acc = mfma(afrag(&s.a.ha[0][0], HLD, R, kt), f0, acc);
      acc = mfma(afrag(&s.a.ha[0][0], HLD, R, kt + 1), f1, acc);
    }
    red_put(0, acc);
    cons_sync<NWC>(cb, cg, pk.spin, err);
    if (w == 0) {
      const f32x4_t v = red_sum(0);
      if (owner) {
        pair_in(v, 1, tagof(E_PD));
        // the layer's output rows (fp32) for the next attention's residual / the final norm
        for (int q = lane; q < MAXR * 16; q += 64) {
          const int rr = q >> 4, c = q & 15;
          if (rr < R) p.x[(long long)rr * p.ldx + 16 * ot + c] = s.xo[rr][c];
          if (dbg && rr < R) dbg[((size_t)2 * MAXR + rr) * IMAX + 16 * ot + c] = s.xo[rr][c];
        }
        if (has_next) publish_x16(1, tagof(E_X2));
      } else {
        pair_out(v, 1, tagof(E_PD));
      }
    }
    TT_STAMP(8);
  }
  // ------------------------------------------------------------------ next layer's q/k/v (input RMSNorm folded)
  if (has_next) {
    constexpr int npre = S_Q < NPRE ? S_Q : NPRE;
    pretake(npre);
    wait_flags(fl_off(myrep, FL_X2), H / 16, tagof(E_X2));
    stage_x16(1);
    TT_STAMP(9);
#pragma unroll
    for (int tq = 0; tq < C::NQT; ++tq) {  // q/k/v tiles b + NB tq
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < SPT; ++j) {
        u32x4_t f0, f1;
        frags(SPT * tq + j, npre, f0, f1);
        const int kt = SLOT * j + 2 * w;
        acc = mfma(afrag(&s.a.xa[0][0], XLD, R, kt), f0, acc);
        acc = mfma(afrag(&s.a.xa[0][0], XLD, R, kt + 1), f1, acc);
      }
      red_put(tq & 1, acc);
      cons_sync<NWC>(cb, cg, pk.spin, err);
      if (w == 0) {
        const f32x4_t v = red_sum(tq & 1);
        const int col = 16 * (b + NB * tq) + lm;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rr = lk * 4 + i;
          if (rr < R) p.qkv[(long long)rr * p.ldq + col] = v[i] * s.rs[rr];
          if (dbg && rr < R) dbg[((size_t)3 * MAXR + rr) * IMAX + col] = v[i] * s.rs[rr];
        }
      }
    }
  }
  // the launch counter: every block read it before publishing, and block 0 has consumed an edge (the SwiGLU rows)
  // from every block by now
  if (b == 0 && tid == 0)
    __hip_atomic_store((unsigned*)(ws + OFF_EPOCH), ep + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  TT_STAMP(10);
}

template <class C>
bool tail_resident() {
  static int cap[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
  if (cap[dev] == 0) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)talker_tail_k<C>, NT, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return false;
    cap[dev] = std::max(1, per_cu * cus);
  }
  return cap[dev] >= C::NB;
}

using C17 = TC<2048, 6144>;  // the 1.7B talker
using C06 = TC<1024, 3072>;  // the 0.6B talker

}  // namespace

extern "C" long long qt_talker_tail_ws_bytes(void) { return (long long)WS_BYTES; }
extern "C" long long qt_talker_tail_stamp_bytes(void) { return (long long)STAMP_BYTES; }
extern "C" long long qt_talker_tail_dbg_bytes(void) { return (long long)(STAMP_BYTES + DBG_BYTES); }

extern "C" int qt_talker_tail_supported(int H_, int I_, int Hq, int D_, int qkv_w) {
  if (Hq * D_ != KO || qkv_w != NQKV) return 0;
  if (H_ == C17::H && I_ == C17::I) return tail_resident<C17>();
  if (H_ == C06::H && I_ == C06::I) return tail_resident<C06>();
  return 0;
}

extern "C" int qt_talker_tail(const qt_talker_tail_args* a, void* stream) {
  if (!a || a->R < 1 || a->R > MAXR) return QT_ERR_SHAPE;
  if (!a->ws || a->ws_bytes < (long long)WS_BYTES || !a->att || !a->x || !a->w_o || !a->w_gu || !a->w_down)
    return QT_ERR_ARG;
  if (a->w_qkv_next && !a->qkv) return QT_ERR_ARG;
  const bool big = a->H == C17::H && a->I == C17::I, small = a->H == C06::H && a->I == C06::I;
  if (!big && !small) return QT_ERR_SHAPE;
  if (a->lda < KO || a->ldx < a->H || (a->w_qkv_next && a->ldq < NQKV)) return QT_ERR_SHAPE;
  if ((reinterpret_cast<uintptr_t>(a->att) | (a->lda * 2)) & 15) return QT_ERR_ARG;  // 16-byte row loads
  if (big ? !tail_resident<C17>() : !tail_resident<C06>()) return QT_ERR_SHAPE;
  static const int spin = std::max(1000, qt_knob("QT_TT_SPIN", 200000));
  if (big) hipLaunchKernelGGL(talker_tail_k<C17>, dim3(C17::NB), dim3(NT), 0, (hipStream_t)stream, TP{*a, spin});
  else hipLaunchKernelGGL(talker_tail_k<C06>, dim3(C06::NB), dim3(NT), 0, (hipStream_t)stream, TP{*a, spin});
  return hipGetLastError() == hipSuccess ? QT_OK : QT_ERR_LAUNCH;
}
