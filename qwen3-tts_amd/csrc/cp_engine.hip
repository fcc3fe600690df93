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
//  * Bulk hand-offs (the q/k/v rows of a head, the x16 rows, the SwiGLU rows) follow the guide's R1 form: payload words
//    stored write-through (agent scope, sc1), the storing wave drains them (s_waitcnt vmcnt(0)), then ONE flag word per
//    producer block = the edge tag; a consumer's wave 0 polls the producers' flags, the block passes a barrier and reads
//    the payload once with sc1 loads (no stale L1 / L2 line, no acquire fence).  The o_proj partials (2 KB per owner)
//    are 8-byte {value, tag} granules (data = flag).  Tags: epoch * 32 + edge + 1, the epoch a launch counter in the
//    workspace advanced by block 0 at the end of every launch (every block has read it by then) -- nothing is reset
//    between launches.  Every all-to-all edge orders the buffer reuse of the next layer.
//  * Every weight fragment a block multiplies in phase k + 1 is loaded into registers right after its phase-k MFMAs,
//    before phase k's outputs are published and the edge into phase k + 1 is polled: the weight latency (Infinity
//    Cache) overlaps the hand-off.  Addressing is buffer-resource based (SGPR base + 32-bit lane offsets), and the
//    per-lane coordinates are re-derived from an opaque thread id every layer, so hipcc does not keep a 64-bit address
//    per load site alive across the layer loop (that spilled ~30 registers).
// Per layer: P1 q/k/v tile (h, cg) -> [QKV edge: the 32 blocks of head h] -> P2 head h's attention (every row) and its
// K-slice of o_proj for 32 columns -> [partial edge: the 8 head blocks of a column group] -> residual add by the
// owner -> [x16 edge, all-to-all] -> P3 gate/up tiles + SwiGLU -> [h edge: all-to-all] -> P4 down tile t for the
// owner's 2 rows + residual -> [x16 edge] -> next layer (or the lm_head).  Numerics follow the launch chain: bf16
// weights and MFMA operands, fp32 accumulation, RMSNorm from the bf16 shadow's values, fp32 q/k/v, the attention of
// attn_oproj_hs_k (q and keys as bf16 pairs, fp32 softmax), SwiGLU / attention outputs rounded to bf16.
#include "common.h"
#include "attn_dev.h"
#include "engine_dev.h"
#include "sample_dev.h"
#include <algorithm>

namespace {

using namespace qt_engine;

constexpr int H = 1024, I = 3072, D = 128, NQ = 16, NKV = 8, NREP = 2;
constexpr int NB = 256, NW = 8, NT = NW * 64, MAXR = 8;
constexpr int KTH = H / 32, KTI = I / 32, KTO = NQ * D / 32;  // k tiles: 32 / 96 / 64
constexpr int LPK = D / 8, GPW = 64 / LPK, IC = 4;              // attention lane groups (attn_oproj_hs_k)
constexpr int XLD = H + 8, HLD = I + 8, ALD = NREP * D + 8;       // LDS row strides (bf16)
constexpr int NEDGE = 32;                                         // tag slots per launch (5 per layer)

// workspace layout (bytes)
constexpr size_t OFF_ERR = 0, OFF_EPOCH = 4;
// The all-to-all edges (x16, SwiGLU rows) are written in NREPL replicas, one per XCD: a consumer polls and reads the
// replica of its own XCD (blockIdx % 8 under round-robin placement -- any replica is correct, the choice only
// spreads the traffic), so 32 blocks instead of 256 hammer one region's cache lines / memory channels (one shared
// copy measured ~4-5 us per edge, contention-bound).
constexpr int NREPL = 8;
constexpr size_t OFF_FLAGS = 256;                                     // [FL_QKV: NB] + [NREPL][3][NB] producer flags
constexpr int FL_X0 = 0, FL_X1 = 1, FL_H = 2;
constexpr size_t REPL_FLAGS = (size_t)3 * NB * 4;                     // one replica's flag block (3 KB)
// Payload regions for up to MR token rows (8: a decode step; 16: the 2-token prefill of 8 batch rows).  One workspace
// serves both forms (sized for 16): every launch is ordered after the previous one on its stream.
template <int MR>
struct Lay {
  static constexpr size_t OFF_QKV = OFF_FLAGS + (size_t)NB * 4 + NREPL * REPL_FLAGS;  // [NKV][MR][512] fp32 payload
  static constexpr size_t OFF_PART = OFF_QKV + (size_t)NKV * MR * 512 * 4;   // [64 t][MR / 2 q][NKV][32] granules
  static constexpr size_t REPL_X16 = (size_t)2 * MR * (H / 2) * 4;           // [2][MR][H/2] bf16 pairs per replica
  static constexpr size_t OFF_X16 = OFF_PART + (size_t)64 * (MR / 2) * NKV * 32 * 8;  // NREPL replicas
  static constexpr size_t REPL_H = (size_t)MR * (I / 2) * 4;                 // [MR][I/2] bf16 pairs per replica
  static constexpr size_t OFF_H = OFF_X16 + NREPL * REPL_X16;                // NREPL replicas
  static constexpr size_t WS = OFF_H + NREPL * REPL_H;
};
// the fused sampler's hand-off (qt_cp_step_sampled): per row one {token, tag} granule; the consumers read the chosen
// token's rows of the (read-only) tables themselves
constexpr size_t OFF_SG = Lay<16>::WS;                      // [8] u64 granules (256 B reserved)
constexpr int E_SAMP = 30;                                  // its tag slot
constexpr size_t WS_BYTES = OFF_SG + 256;
// optional per-stage intermediates of every layer (a workspace this much larger records them; the stage-by-stage parity
// tests): fp32 [6 layers][DBG_KINDS][16 token rows][4096] -- kind 0 x after the attention residual, 1 the SwiGLU output,
// 2 x after the MLP residual, 3 the attention output, 4 the layer's q/k/v rows (projected, before the q/k norm)
constexpr int DBG_KINDS = 5, DBG_ROWS = 16;
constexpr size_t DBG_BYTES = (size_t)6 * DBG_KINDS * DBG_ROWS * 4096 * 4;
// ... and a workspace larger still records per-block phase timestamps (s_memrealtime, 100 MHz) after that:
// [NB][64] u64 -- stamp 0 kernel start, 1 end, 2 + 12 l + k the layer-l events (tools/ce_debug.py names them)
constexpr size_t STAMP_BYTES = (size_t)NB * 128 * 8;  // + [64, 128): sub-phase stamps of layer 2

struct CEP {
  qt_cp_step_args a;
  int spin;
  // qt_cp_step_sampled: the previous step's token choice at the start of this launch (sa: qt_sample's arguments with
  // no embedding outputs; the engine gathers the rows of gx / gq itself and hands them to its blocks)
  int fuse;
  qt_sample_args sa;
  const float* gx;
  const float* gq;
};

// Wave 0 (the publishing wave) waits until the n (multiple of 4, <= 256) flag words at byte offset `off` all carry
// `tag` -- one 16-byte sc1 load per lane per pass -- (bounded: a give-up sets the sticky error flag), then a block
// barrier.
QT_DEV void wait_flags(rsrc_t r, unsigned off, int n, unsigned tag, int spin, int* err) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    for (int spins = 0;; ++spins) {
      bool ok = true;
      if (lane * 4 < n) {
        const u32x4_t v = bld_c(r, off + lane * 16);
        ok = v[0] == tag && v[1] == tag && v[2] == tag && v[3] == tag;
      }
      if (__all(ok)) break;
      if (spins > spin) {
        if (lane == 0) atomicOr(err, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

// the eight per-layer pointer arrays of qt_cp_step_args, in their declaration order (contiguous: read as one table)
enum { PT_QKV, PT_O, PT_GU, PT_DOWN, PT_QN, PT_KN, PT_KC, PT_VC };
static_assert(offsetof(qt_cp_step_args, w_o) == offsetof(qt_cp_step_args, w_qkv) + 8 * 8 * PT_O, "pointer table");
static_assert(offsetof(qt_cp_step_args, w_gu) == offsetof(qt_cp_step_args, w_qkv) + 8 * 8 * PT_GU, "pointer table");
static_assert(offsetof(qt_cp_step_args, w_down) == offsetof(qt_cp_step_args, w_qkv) + 8 * 8 * PT_DOWN, "pointer table");
static_assert(offsetof(qt_cp_step_args, q_norm) == offsetof(qt_cp_step_args, w_qkv) + 8 * 8 * PT_QN, "pointer table");
static_assert(offsetof(qt_cp_step_args, k_norm) == offsetof(qt_cp_step_args, w_qkv) + 8 * 8 * PT_KN, "pointer table");
static_assert(offsetof(qt_cp_step_args, k_cache) == offsetof(qt_cp_step_args, w_qkv) + 8 * 8 * PT_KC, "pointer table");
static_assert(offsetof(qt_cp_step_args, v_cache) == offsetof(qt_cp_step_args, w_qkv) + 8 * 8 * PT_VC, "pointer table");

// MR token rows: 8 (decode: one row per batch row) or 16 (prefill: rows 2b, 2b + 1 = positions 0, 1 of batch row b).
// A block owns MR / 8 residual slices (row pairs qo and qo + 4 in the prefill), MR / 4 rows in all.
template <int MR>
struct Lds {
  static constexpr bool PF = MR == 16;
  union {
    bf16_t xa[MR][XLD];     // x16 rows (all), the A operand of q/k/v, gate/up, lm_head
    bf16_t ha[MR / 4][HLD]; // the owner's SwiGLU rows, the A operand of down
    qt_sample_dev::SampSh samp;  // the fused sampler (layer 0, before any x16 staging)
  } a;
  unsigned sb_st[2];  // the fused sampler's barrier k: sb_st[k % 2] = 1 if it is the last (written before it)
  float red[NW][64][4];                                        // per-wave MFMA partials
  float rs[MR];                                                // 1 / rms per row
  float xown[MR / 4][16];                                      // the owned residual slices
  __attribute__((aligned(16))) bf16_t zero[32];                // the A rows past the batch (MFMA rows >= R)
  const void* ptab[8][8];  // per-layer pointers [PT_*][layer]: one LDS read instead of a scalar kernarg miss per use
  float gath[MR / 8][NKV][32];                                 // the 8 head partials of the owned slices
  __attribute__((aligned(16))) float qf[NW][NREP][D];          // decode attention: q (fp32)
  __attribute__((aligned(16))) unsigned kn2[NW][D / 2];        // the new key as bf16 pairs
  float vn[NW][D];                                             // the new value (bf16-rounded)
  // prefill attention (wave w = batch row w): q (fp32), k / v (bf16-rounded) at positions 0, 1
  float pq[PF ? NW : 1][2][NREP][D], pkk[PF ? NW : 1][2][D], pv[PF ? NW : 1][2][D];
  __attribute__((aligned(16))) bf16_t att[MR][ALD];            // head h's attention output per row
};

// Stage the x16 edge (all rows) into lds.a.xa and each row's 1 / rms (from the bf16 values, as the decode GEMV computes
// it from the bf16 shadow).  Thread -> rows tid / 64 (+ 8), pairs (tid % 64) * 8 .. + 8: the payload read is spread
// over all eight waves' memory queues.
template <int MR>
QT_DEV void stage_x16(Lds<MR>& s, rsrc_t gx, unsigned base, unsigned flag_off, unsigned tag, int R, float eps, int spin,
                      int* err, int tid) {
  constexpr int NRW = MR / 8;
  const int p0 = (tid & 63) * 8;
  wait_flags(gx, flag_off, NB, tag, spin, err);
  u32x4_t v0[NRW], v1[NRW];
#pragma unroll
  for (int k = 0; k < NRW; ++k) {
    const int row = (tid >> 6) + 8 * k;
    v0[k] = u32x4_t{0u, 0u, 0u, 0u};
    v1[k] = u32x4_t{0u, 0u, 0u, 0u};
    if (row < R) {
      const unsigned o = base + (unsigned)(row * (H / 2) + p0) * 4;
      v0[k] = bld_c(gx, o);
      v1[k] = bld_c(gx, o + 16);
    }
  }
#pragma unroll
  for (int k = 0; k < NRW; ++k) {
    const int row = (tid >> 6) + 8 * k;
    *(u32x4_t*)&s.a.xa[row][2 * p0] = v0[k];
    *(u32x4_t*)&s.a.xa[row][2 * p0 + 8] = v1[k];
    float ss = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const unsigned u = q < 4 ? v0[k][q] : v1[k][q - 4];
      const float lo = __uint_as_float(u << 16), hi = __uint_as_float(u & 0xFFFF0000u);
      ss += lo * lo + hi * hi;
    }
    ss = wave_sum_dpp(ss);  // wave == row
    if ((tid & 63) == 0) s.rs[row] = rsqrtf(ss / (float)H + eps);
  }
  __syncthreads();
}

// The prefill's layer-0 input: fp32 rows of x rounded to bf16 (as the launch chain's bf16 shadow holds them), staged
// like stage_x16 (no edge: x was written before the launch)
QT_DEV void stage_x32(Lds<16>& s, const float* x, long long ldx, int R, float eps, int tid) {
  const int p0 = (tid & 63) * 8;
  f32x4_t v[2][4];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int row = (tid >> 6) + 8 * k;
    const float* src = x + (long long)min(row, R - 1) * ldx + 2 * p0;
#pragma unroll
    for (int q = 0; q < 4; ++q) v[k][q] = *(const f32x4_t*)(src + 4 * q);
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int row = (tid >> 6) + 8 * k;
    u32x4_t a0, a1;
    float ss = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float e0 = v[k][q >> 1][(q & 1) * 2], e1 = v[k][q >> 1][(q & 1) * 2 + 1];
      const unsigned u = row < R ? pack2bf(e0, e1) : 0u;
      if (q < 4) a0[q] = u;
      else a1[q - 4] = u;
      const float lo = __uint_as_float(u << 16), hi = __uint_as_float(u & 0xFFFF0000u);
      ss += lo * lo + hi * hi;
    }
    *(u32x4_t*)&s.a.xa[row][2 * p0] = a0;
    *(u32x4_t*)&s.a.xa[row][2 * p0 + 8] = a1;
    ss = wave_sum_dpp(ss);
    if ((tid & 63) == 0) s.rs[row] = rsqrtf(ss / (float)H + eps);
  }
  __syncthreads();
}

// A fragment of MFMA row lm (batch row; rows >= R zero) at k tile kt from the staged x16 rows
template <int MR>
QT_DEV u32x4_t afrag_x(const Lds<MR>& s, int lm, int lk, int kt, int R) {
  return *(const u32x4_t*)(lm < R ? &s.a.xa[lm][kt * 32 + lk * 8] : &s.zero[lk * 8]);
}

// Sum the per-wave partials of waves [w0, w0 + nw) for lane `lane` (fixed wave order)
template <int MR>
QT_DEV f32x4_t red_sum(const Lds<MR>& s, int w0, int nw, int lane) {
  f32x4_t v = {0.f, 0.f, 0.f, 0.f};
  for (int ww = w0; ww < w0 + nw; ++ww) {
    v[0] += s.red[ww][lane][0]; v[1] += s.red[ww][lane][1]; v[2] += s.red[ww][lane][2]; v[3] += s.red[ww][lane][3];
  }
  return v;
}
template <int MR>
QT_DEV void red_put(Lds<MR>& s, int w, int lane, f32x4_t acc) {
  s.red[w][lane][0] = acc[0]; s.red[w][lane][1] = acc[1]; s.red[w][lane][2] = acc[2]; s.red[w][lane][3] = acc[3];
}

// When the next phase's weight fragments are issued (LM):
//  0 (early): by waves 1-7 right after their MFMAs, by the publishing wave after its flag -- the other waves' ~100 KiB
//    of loads then sit in the CU's memory pipeline ahead of the publisher's stores, drain and flag (critical path);
//  1 (late): by every wave after the phase's publication (one more block barrier) -- but a wave's edge poll / payload
//    loads then return behind its own weight loads (vmcnt is in order), so every edge also waits one weight round trip;
//  2 (ahead): one phase ahead, right after the edge that starts the previous phase (before its MFMAs): the memory
//    pipeline has drained them by the time that phase publishes, and they have landed before the next edge's polls.
// PF = 0: a decode step (rows = batch rows at cache position const_pos); PF = 1: the 2-token prefill (token rows 2b,
// 2b + 1 at positions 0, 1 of batch row b; every key is new, layer 0's q/k/v computed here from x).
template <int LM, int PF>
__global__ __launch_bounds__(NT) void cp_step_k(CEP pk) {
  constexpr bool LATE = LM == 1, AHEAD = LM == 2, EARLY = LM == 0;
  constexpr int MR = PF ? 16 : 8, NSL = MR / 8, NQO = MR / 2;
  using LY = Lay<MR>;
  const qt_cp_step_args& p = pk.a;
  __shared__ Lds<MR> s;
  const int b = blockIdx.x, h = b >> 5, cg = b & 31;
  // the owned residual slices: rows 2qo, 2qo + 1 (and 2qo + 8, 2qo + 9 in the prefill), cols 16to ..
  const int to = 2 * cg + (h >> 2), qo = h & 3;
  auto orow = [&](int i) { return 2 * (qo + 4 * (i >> 1)) + (i & 1); };  // token row of owned row i
  const int R = p.R;                    // batch rows
  const bool fuse = !PF && pk.fuse;     // the previous step's sampler runs here first (qt_cp_step_sampled)
  const int RT = PF ? 2 * R : R;        // token rows
  char* ws = (char*)p.ws;
  int* err = (int*)(ws + OFF_ERR);
  unsigned* flags = (unsigned*)(ws + OFF_FLAGS);  // [0, NB): the q/k/v edge's flags
  const int myrep = b % NREPL;                     // the replica this block reads (its XCD under round-robin placement)
  auto fl_off = [&](int rp, int kind) { return (unsigned)(OFF_FLAGS + NB * 4 + rp * REPL_FLAGS + kind * NB * 4); };
  u64* gpart = (u64*)(ws + LY::OFF_PART);
  const rsrc_t wsr = mkr(ws, (unsigned)WS_BYTES);  // payload regions, addressed by byte offset
  const unsigned ep = (unsigned)(ld_g((const u64*)(ws + OFF_ERR)) >> 32);  // (low word: the error flag)
  float* dbg = p.ws_bytes >= (long long)(WS_BYTES + DBG_BYTES) ? (float*)(ws + WS_BYTES) : nullptr;
  // element (layer, kind, token row, column) of the stage record
  auto dbgi = [](int l, int kind, int row, int col) { return (((size_t)l * DBG_KINDS + kind) * DBG_ROWS + row) * 4096 + col; };
  u64* stamps = p.ws_bytes >= (long long)(WS_BYTES + DBG_BYTES + STAMP_BYTES)
                    ? (u64*)(ws + WS_BYTES + DBG_BYTES) + b * 128 : nullptr;
#define CE_STAMP(k) \
  if (stamps && threadIdx.x == 0) stamps[(k)] = __builtin_amdgcn_s_memrealtime();
  CE_STAMP(0);
#define CE_SUB(k) \
  if (stamps && l == 2 && threadIdx.x == 0) stamps[64 + (k)] = __builtin_amdgcn_s_memrealtime();
  auto tagof = [&](int e) { return ep * NEDGE + (unsigned)e + 1u; };
  const int kvpos = p.const_pos, nc = kvpos;
  const int ntile3 = b < 128 ? 2 : 1;  // gate/up tiles: b and b + 256 for b < 128 (384 tiles)
  // P1 tile of block (h, cg): head h's 32 q/k/v tiles (q: 16, k: 8, v: 8)
  const int t1 = cg < 16 ? h * 16 + cg : (cg < 24 ? NQ * D / 16 + h * 8 + (cg - 16) : (NQ + NKV) * D / 16 + h * 8 + (cg - 24));
  const unsigned kvstride = (unsigned)p.Lmax * D * 2;  // bytes per (row, kv head) cache slab
  const unsigned kvbytes = (unsigned)R * NKV * kvstride;

  {  // the owned residual slice (wave 0), the zero A row, the per-layer pointer table (wave 1)
    const int tid = threadIdx.x;
    if (tid < 32 * NSL) {  // (fused sampler: the rows are the chosen tokens' -- read at the first residual add)
      const int rr = orow(tid >> 4);
      s.xown[tid >> 4][tid & 15] = rr < RT && !fuse ? p.x[(long long)rr * p.ldx + 16 * to + (tid & 15)] : 0.f;
    } else if (tid == 144) {
      s.sb_st[0] = 0u;
      s.sb_st[1] = 0u;
    } else if (tid >= 128 && tid < 144) {
      ((unsigned*)s.zero)[tid - 128] = 0u;
    } else if (tid >= 64 && tid < 128) {
      (&s.ptab[0][0])[tid - 64] = (&p.w_qkv[0])[tid - 64];
    }
    __syncthreads();
  }
  // a per-layer pointer, wave-uniform (SGPRs)
  auto lp = [&](int k, int l) -> const void* {
    const u64 v = (u64)s.ptab[k][l];
    // (readfirstlane returns int: widen through unsigned, or the low word's sign bit would smear into the high word)
    return (const void*)(((u64)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(v >> 32)) << 32) |
                         (u64)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)v));
  };

  // register-resident weights of the next phase (see the header)
  u32x4_t w1[4];    // P1: q/k/v tile, k tiles 4w .. 4w + 3 (or the lm_head tile)
  u32x4_t w2[2];    // P2: o_proj, 2 fragments per wave
  u32x4_t w3[8];    // P3: gate/up, 4 (one tile) or 8 (two tiles) fragments per wave
  u32x4_t w4[12];   // P4: down tile `to`, k tiles 12w .. 12w + 11
  u32x4_t kq[IC], vq[IC];  // P2: cached keys / values of (row r, head h)

  // P2's loads: o_proj fragments f0, f0 + 1 of tile 2cg + f0 / 8 (head h's k tiles), cached keys / values of (row
  // min(w, R - 1), head h) -- lane group grp owns keys grp, grp + 4, ... (clamped, masked in the math)
  auto load_p2 = [&](int l, int tid) {
    const int lane = tid & 63, w = tid >> 6, f0 = w * 2;
    const rsrc_t wo = mkr(lp(PT_O, l), (unsigned)H * NQ * D * 2);
#pragma unroll
    for (int i = 0; i < 2; ++i) w2[i] = bld(wo, fragoff(2 * cg + f0 / 8, h * 8 + f0 % 8 + i, KTO, lane));
    if constexpr (!PF) {
      const int r = min(w, R - 1), grp = lane / LPK, sub = lane % LPK;
      const rsrc_t kr = mkr(lp(PT_KC, l), kvbytes), vr = mkr(lp(PT_VC, l), kvbytes);
      const unsigned kvb = (unsigned)(r * NKV + h) * kvstride + sub * 16;
#pragma unroll
      for (int c = 0; c < IC; ++c) {
        const unsigned o = kvb + (unsigned)min(c * GPW + grp, max(nc - 1, 0)) * D * 2;
        kq[c] = bld(kr, o);
        vq[c] = bld(vr, o);
      }
    }
    CE_ISSUED();
  };
  auto load_p3 = [&](int l, int tid) {
    const int lane = tid & 63, w = tid >> 6;
    const int t3 = ntile3 == 2 ? b + (w >> 2) * NB : b, k3 = ntile3 == 2 ? (w & 3) * 8 : w * 4;
    const int n3 = ntile3 == 2 ? 8 : 4;
    const rsrc_t wg = mkr(lp(PT_GU, l), (unsigned)2 * I * H * 2);
#pragma unroll
    for (int i = 0; i < 8; ++i) w3[i] = bld(wg, fragoff(t3, k3 + min(i, n3 - 1), KTH, lane));
    CE_ISSUED();
  };
  auto load_p4 = [&](int l, int tid) {
    const int lane = tid & 63, w = tid >> 6;
    const rsrc_t wd = mkr(lp(PT_DOWN, l), (unsigned)H * I * 2);
#pragma unroll
    for (int i = 0; i < 12; ++i) w4[i] = bld(wd, fragoff(to, w * 12 + i, KTI, lane));
    CE_ISSUED();
  };
  auto load_p1 = [&](const void* wt, unsigned bytes, int tile, int tid) {
    const int lane = tid & 63, w = tid >> 6;
    const rsrc_t wr = mkr(wt, bytes);
#pragma unroll
    for (int i = 0; i < 4; ++i) w1[i] = bld(wr, fragoff(tile, w * 4 + i, KTH, lane));
    CE_ISSUED();
  };
  // (wave 0, lane `lane`) publish the owned slice's bf16 copy (2 rows x 8 column pairs) to x16 buffer `buf` of every
  // replica, drain, then the replicas' flags
  auto publish_x16 = [&](int buf, unsigned tag, int lane) {
    if constexpr (!PF) {
      const int rr = (lane >> 3) & 1, pp = lane & 7, r0 = lane >> 4;
      if (2 * qo + rr < R) {
        const unsigned v = pack2bf(s.xown[rr][2 * pp], s.xown[rr][2 * pp + 1]);
        const unsigned o = (unsigned)LY::OFF_X16 + (unsigned)(((buf * MR + 2 * qo + rr) * (H / 2)) + 8 * to + pp) * 4;
        bst_c(v, wsr, o + r0 * (unsigned)LY::REPL_X16);
        bst_c(v, wsr, o + (r0 + 4) * (unsigned)LY::REPL_X16);
      }
    } else {  // 2 slices x 2 rows x 8 pairs, each value by two lanes (4 replicas each)
      const int i = (lane >> 3) & 3, pp = lane & 7, rg = lane >> 5, tr = orow(i);
      if (tr < RT) {
        const unsigned v = pack2bf(s.xown[i][2 * pp], s.xown[i][2 * pp + 1]);
        const unsigned o = (unsigned)LY::OFF_X16 + (unsigned)(((buf * MR + tr) * (H / 2)) + 8 * to + pp) * 4;
#pragma unroll
        for (int k = 0; k < 4; ++k) bst_c(v, wsr, o + (rg * 4 + k) * (unsigned)LY::REPL_X16);
      }
    }
    drain_stores();
    if (lane < NREPL) st_flag((unsigned*)(ws + fl_off(lane, FL_X0 + buf)) + b, tag);
  };

  const int L = p.n_layers;
  // the fused sampler of row r = b / 33 (one workgroup per XCD) runs on its waves 0-3: qt_sample's body on the
  // previous launch's logits (visible: kernel boundary); the chosen token goes out as the row's {token, tag} granule.
  // Its barriers are block barriers: waves 4-7 pass barriers in a loop until the last one, which the sampler marks
  // in a double-buffered LDS word before it (slot k % 2 is not rewritten before every wave has passed barrier k + 1).
  // The sampler waves issue their own P2 loads only at the body's first barrier, after its logits loads (vmcnt
  // retires in order).
  u64* sgr = (u64*)(ws + OFF_SG);
  const bool samp_blk = fuse && b % 33 == 0 && b / 33 < R;
  if constexpr (PF) load_p1(lp(PT_QKV, 0), (unsigned)(NQ + 2 * NKV) * D * H * 2, t1, threadIdx.x);
  else if (!(samp_blk && threadIdx.x < 256)) load_p2(0, threadIdx.x);
  if (samp_blk) {
    if (threadIdx.x < 256) {
      const int r = b / 33, tid = threadIdx.x;
      bool issued = false;
      int kb = 0;
      const int tok = qt_sample_dev::sample_row<8>(pk.sa, 0, r, tid, s.a.samp, [&]() {
        if (!issued) { issued = true; load_p2(0, tid); }
        if (tid == 0) s.sb_st[kb & 1] = 0u;
        ++kb;
        __syncthreads();
      });
      if (!issued) load_p2(0, tid);
      if (tid == 0) {
        st_g(sgr + r, (unsigned)tok, tagof(E_SAMP));
        s.sb_st[kb & 1] = 1u;
      }
      __syncthreads();
    } else {
      for (int k = 0;; ++k) {
        __syncthreads();
        if (s.sb_st[k & 1]) break;
      }
    }
  }
  for (int l = 0; l < L; ++l) {
    // per-lane coordinates from an opaque thread id: derived values are recomputed per layer, not kept alive
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, w = tid >> 6, lm = lane & 15, lk = lane >> 4;
    // wave 0 publishes every edge: its weight loads are issued AFTER each publication, since its drain
    // (s_waitcnt vmcnt(0)) would otherwise wait for them; the other waves issue theirs right after their MFMAs
    const bool pubw = w == 0;
    // ------------------------------------------------------------------ P1: q/k/v projection (layers >= 1)
    const int sb = 2 + 12 * l;
    if (l > 0 || PF) {
      CE_STAMP(sb + 0);
      if (PF && l == 0) stage_x32(*(Lds<16>*)&s, p.x, p.ldx, RT, p.eps, tid);
      else
        stage_x16(s, wsr, (unsigned)(LY::OFF_X16 + myrep * LY::REPL_X16) + MR * (H / 2) * 4, fl_off(myrep, FL_X1),
                  tagof(5 * (l - 1) + 4), RT, p.eps, pk.spin, err, tid);
      CE_STAMP(sb + 1);
      if (AHEAD) load_p2(l, tid);
      u32x4_t af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = afrag_x(s, lm, lk, w * 4 + i, RT);
      pin4(af);
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) acc = mfma(af[i], w1[i], acc);
      CE_AFTER(acc);
      CE_SUB(0);
      red_put(s, w, lane, acc);
      if (EARLY && !pubw) load_p2(l, tid);
      __syncthreads();
      CE_SUB(2);
      if (pubw) {
        const f32x4_t v = red_sum(s, 0, NW, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rr = lk * 4 + i;
          if (rr < RT)
            bst_c(__float_as_uint(v[i] * s.rs[rr]), wsr,
                  (unsigned)LY::OFF_QKV + (unsigned)((h * MR + rr) * 512 + cg * 16 + lm) * 4);
        }
        CE_SUB(3);
        drain_stores();
        CE_SUB(4);
        if (lane == 0) st_flag(flags + b, tagof(5 * l));
        if (EARLY) load_p2(l, tid);
      }
      if (LATE) {
        __syncthreads();
        load_p2(l, tid);
      }
      CE_STAMP(sb + 2);
    }
    // ------------------------------------------------------------------ P2: attention of head h + o_proj K-slice
    {
      if constexpr (!PF) {
      const int r = min(w, R - 1);  // wave w = row w
      const int grp = lane / LPK, sub = lane % LPK;
      const int vsel = min(grp, NREP + 1);
      const int e0 = sub * 8, half = D / 2, ec = e0 % half;
      // the norm weights and rotary rows do not depend on the edge: issued before its wait
      float nwv[8], cv[8], sv[8];
      const float* qn = (const float*)lp(PT_QN, l);
      const float* kn = (const float*)lp(PT_KN, l);
      load8f((vsel < NREP ? qn : kn) + e0, nwv);
      load8f(p.cos_tab + (long long)kvpos * half + ec, cv);
      load8f(p.sin_tab + (long long)kvpos * half + ec, sv);
      float xv[8];
      if (l == 0) {
        const int hh = vsel < NREP ? h * NREP + vsel : (vsel == NREP ? NQ + h : NQ + NKV + h);
        if (fuse) {  // row r's q/k/v: the chosen token's row of the q/k/v table
          const unsigned want = tagof(E_SAMP);
          u64 gv = ld_g(sgr + r);
          for (int spins = 0; (unsigned)(__builtin_amdgcn_readfirstlane((unsigned)(gv >> 32))) != want; ++spins) {
            if (spins > pk.spin) { if (lane == 0) atomicOr(err, 1); break; }
            __builtin_amdgcn_s_sleep(1);
            gv = ld_g(sgr + r);
          }
          const int tok = min((int)(unsigned)gv, pk.sa.V - 1);
          load8f(pk.gq + (long long)tok * (NQ + 2 * NKV) * D + (long long)hh * D + e0, xv);
        } else {
          load8f(p.qkv0 + (long long)r * p.ldq + (long long)hh * D + e0, xv);
        }
      } else {
        wait_flags(wsr, (unsigned)OFF_FLAGS + h * 32 * 4, 32, tagof(5 * l), pk.spin, err);  // head h's 32 q/k/v tiles
        const unsigned o = (unsigned)LY::OFF_QKV + (unsigned)((h * MR + r) * 512 + vsel * D + e0) * 4;
        const u32x4_t a0 = bld_c(wsr, o), a1 = bld_c(wsr, o + 16);
#pragma unroll
        for (int k = 0; k < 4; ++k) { xv[k] = __uint_as_float(a0[k]); xv[4 + k] = __uint_as_float(a1[k]); }
      }
      if (dbg && cg == 0 && w < R) {  // (lane group vsel: q head 2h + vsel, k head h, v head h)
        const int hh = vsel < NREP ? h * NREP + vsel : (vsel == NREP ? NQ + h : NQ + NKV + h);
#pragma unroll
        for (int i = 0; i < 8; ++i) dbg[dbgi(l, 4, w, hh * D + e0 + i)] = xv[i];
      }
      CE_STAMP(sb + 3);
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
      if (grp < NREP) {
        *(f32x4_t*)&s.qf[w][grp][e0] = f32x4_t{xv[0], xv[1], xv[2], xv[3]};
        *(f32x4_t*)&s.qf[w][grp][e0 + 4] = f32x4_t{xv[4], xv[5], xv[6], xv[7]};
      } else if (grp == NREP) {
        u32x4_t pk2;
#pragma unroll
        for (int i = 0; i < 4; ++i) pk2[i] = pack2bf_rne(xv[2 * i], xv[2 * i + 1]);
        *(u32x4_t*)&s.kn2[w][e0 / 2] = pk2;
      } else if (grp == NREP + 1) {
#pragma unroll
        for (int i = 0; i < 8; ++i) s.vn[w][e0 + i] = bf2f(f2bf(xv[i]));
      }
      __syncthreads();
      // attention of (row r, head h) over the cached keys [0, kvpos) + the new key, fp32 arithmetic on the bf16 keys /
      // values as stored (q and the softmax weights stay fp32: only the output is rounded, as qt_decode_attention; the
      // bf16 q / weight pairs of attn_oproj_hs_k's form cost ~1.4x its rounding error, tests/test_gpu_engine_stages.py)
      {
        const float scale = rsqrtf((float)D) * 1.4426950408889634f;
        float qv[NREP][8];
#pragma unroll
        for (int j = 0; j < NREP; ++j) {
          const f32x4_t a = *(const f32x4_t*)&s.qf[w][j][sub * 8], b2 = *(const f32x4_t*)&s.qf[w][j][sub * 8 + 4];
#pragma unroll
          for (int i = 0; i < 4; ++i) { qv[j][i] = a[i]; qv[j][4 + i] = b2[i]; }
        }
        const u32x4_t k2n = *(const u32x4_t*)&s.kn2[w][sub * 4];
        typedef float f2v __attribute__((ext_vector_type(2)));
        // bf16 pair (dims 2i, 2i + 1) -> fp32 pair; each key / value fragment unpacked once for both q heads, the dot
        // products and the weighted value sums as packed fp32 FMAs (v_pk_fma_f32: two per instruction)
        auto unp = [](unsigned u) { return f2v{__uint_as_float(u << 16), __uint_as_float(u & 0xFFFF0000u)}; };
        f2v qp[NREP][4];
#pragma unroll
        for (int j = 0; j < NREP; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) qp[j][i] = f2v{qv[j][2 * i], qv[j][2 * i + 1]};
        auto dot_pk = [&](int j, const f2v (&kf)[4]) {
          f2v acc = qp[j][0] * kf[0];
#pragma unroll
          for (int i = 1; i < 4; ++i) acc = qp[j][i] * kf[i] + acc;
          return acc.x + acc.y;
        };
        float dd[NREP][IC], dn[NREP];
        {
          f2v kf[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) kf[i] = unp(k2n[i]);
#pragma unroll
          for (int j = 0; j < NREP; ++j) dn[j] = group_sum_dpp<LPK>(dot_pk(j, kf)) * scale;
        }
#pragma unroll
        for (int c = 0; c < IC; ++c) {
          f2v kf[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) kf[i] = unp(kq[c][i]);
#pragma unroll
          for (int j = 0; j < NREP; ++j) {
            const float d = group_sum_dpp<LPK>(dot_pk(j, kf)) * scale;
            dd[j][c] = c * GPW + grp < nc ? d : -INFINITY;
          }
        }
        f2v vn2[4], vf[IC][4];
#pragma unroll
        for (int i = 0; i < 4; ++i) vn2[i] = f2v{s.vn[w][sub * 8 + 2 * i], s.vn[w][sub * 8 + 2 * i + 1]};
#pragma unroll
        for (int c = 0; c < IC; ++c)
#pragma unroll
          for (int i = 0; i < 4; ++i) vf[c][i] = unp(vq[c][i]);
        float m[NREP], lsum[NREP], o[NREP][8];
#pragma unroll
        for (int j = 0; j < NREP; ++j) {
          float mn = dn[j];
#pragma unroll
          for (int c = 0; c < IC; ++c) mn = fmaxf(mn, dd[j][c]);
          const float en = grp == 0 ? exp2_hw(dn[j] - mn) : 0.f;
          float ev[IC];
          float ls = en;
#pragma unroll
          for (int c = 0; c < IC; ++c) {
            ev[c] = exp2_hw(dd[j][c] - mn);
            ls += ev[c];
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) {  // output dims 2i, 2i + 1
            f2v acc = f2v{en, en} * vn2[i];
#pragma unroll
            for (int c = 0; c < IC; ++c) acc = f2v{ev[c], ev[c]} * vf[c][i] + acc;
            o[j][2 * i] = acc.x;
            o[j][2 * i + 1] = acc.y;
          }
          m[j] = mn; lsum[j] = ls;
        }
        GroupMerge<LPK, NREP> gm;
        gm.run(m, lsum, o);
        gm.each(lane, [&](int j, int d, float ov, float lv, float) { s.att[w][j * D + d] = f2bf(ov * __builtin_amdgcn_rcpf(lv)); });
      }
      } else {
        // prefill: wave w = batch row w, token rows 2w (position 0) and 2w + 1 (position 1); lane group grp = q head 0,
        // q head 1, k, v (the chain's attn_small_prefill_k: fp32 q, bf16-rounded k / v, causal softmax over <= 2 keys)
        const int r = min(w, R - 1);
        const int grp = lane / LPK, sub = lane % LPK;
        const int e0 = sub * 8, half = D / 2, ec = e0 % half;
        float nwv[8], cv[2][8], sv[2][8];
        const float* qn = (const float*)lp(PT_QN, l);
        const float* kn = (const float*)lp(PT_KN, l);
        load8f((grp < NREP ? qn : kn) + e0, nwv);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          load8f(p.cos_tab + (long long)t * half + ec, cv[t]);
          load8f(p.sin_tab + (long long)t * half + ec, sv[t]);
        }
        wait_flags(wsr, (unsigned)OFF_FLAGS + h * 32 * 4, 32, tagof(5 * l), pk.spin, err);  // head h's 32 q/k/v tiles
        float xv[2][8];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const unsigned o = (unsigned)LY::OFF_QKV + (unsigned)((h * MR + 2 * r + t) * 512 + grp * D + e0) * 4;
          const u32x4_t a0 = bld_c(wsr, o), a1 = bld_c(wsr, o + 16);
#pragma unroll
          for (int k = 0; k < 4; ++k) { xv[t][k] = __uint_as_float(a0[k]); xv[t][4 + k] = __uint_as_float(a1[k]); }
        }
        if (dbg && cg == 0 && w < R) {  // (lane group grp: q head 2h + grp, k head h, v head h)
          const int hh = grp < NREP ? h * NREP + grp : (grp == NREP ? NQ + h : NQ + NKV + h);
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int i = 0; i < 8; ++i) dbg[dbgi(l, 4, 2 * w + t, hh * D + e0 + i)] = xv[t][i];
        }
        CE_STAMP(sb + 3);
        const bool lo = e0 < half, normed = grp <= NREP;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          float ss = 0.f;
#pragma unroll
          for (int i = 0; i < 8; ++i) ss += xv[t][i] * xv[t][i];
          ss = group_sum_dpp<LPK>(ss);
          const float rsn = rsqrtf(ss / (float)D + p.eps);
          float y[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) y[i] = nwv[i] * (xv[t][i] * rsn);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float pt = half_partner<LPK>(y[i]);
            const float ro = lo ? y[i] * cv[t][i] - pt * sv[t][i] : y[i] * cv[t][i] + pt * sv[t][i];
            const float xo = normed ? ro : xv[t][i];
            if (grp < NREP) s.pq[w][t][grp][e0 + i] = xo;
            else if (grp == NREP) s.pkk[w][t][e0 + i] = bf2f(f2bf(xo));
            else s.pv[w][t][e0 + i] = bf2f(f2bf(xo));
          }
        }
        __syncthreads();
        {  // lane group grp: token position t = grp / 2, q head j = grp % 2
          const int t = grp >> 1, j = grp & 1;
          const float scale = rsqrtf((float)D) * 1.4426950408889634f;
          float d0 = 0.f, d1 = 0.f;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float q = s.pq[w][t][j][e0 + i];
            d0 += q * s.pkk[w][0][e0 + i];
            d1 += q * s.pkk[w][1][e0 + i];
          }
          d0 = group_sum_dpp<LPK>(d0) * scale;
          d1 = group_sum_dpp<LPK>(d1) * scale;
          const float mx = t ? fmaxf(d0, d1) : d0;
          const float p0 = exp2_hw(d0 - mx), p1 = t ? exp2_hw(d1 - mx) : 0.f, den = p0 + p1;
#pragma unroll
          for (int i = 0; i < 8; ++i)
            s.att[2 * w + t][j * D + e0 + i] = f2bf((p0 * s.pv[w][0][e0 + i] + p1 * s.pv[w][1][e0 + i]) / den);
        }
      }
      __syncthreads();
      CE_STAMP(sb + 4);
      if (AHEAD) load_p3(l, tid);
      if (dbg && cg == 0 && w < R)
        for (int t = 0; t < (PF ? 2 : 1); ++t)
          for (int j = lane; j < NREP * D; j += 64)
            dbg[dbgi(l, 3, PF ? 2 * w + t : w, h * NREP * D + j)] = bf2f(s.att[PF ? 2 * w + t : w][j]);
      // head h's K-slice of o_proj for columns 32cg .. 32cg + 32: wave w, fragments 2w, 2w + 1 of tile 2cg + w / 4
      {
        const int kt0 = (2 * w) % 8;
        u32x4_t af[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = *(const u32x4_t*)(lm < MR ? &s.att[lm][(kt0 + i) * 32 + lk * 8] : &s.zero[lk * 8]);
        asm volatile("" : "+v"(af[0]), "+v"(af[1]));
        f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 2; ++i) acc = mfma(af[i], w2[i], acc);
        CE_AFTER(acc);
        red_put(s, w, lane, acc);
        if (EARLY && !pubw) load_p3(l, tid);
        // the new k / v of (row w, head h) into the caches (one column group appends)
        if constexpr (!PF) {
          if (cg == 0 && w < R && lane < D / 2) {
            const long long o = (((long long)w * NKV + h) * p.Lmax + kvpos) * D;
            ((unsigned*)lp(PT_KC, l))[o / 2 + lane] = s.kn2[w][lane];
            ((bf16_t*)lp(PT_VC, l))[o + lane] = f2bf(s.vn[w][lane]);
            ((bf16_t*)lp(PT_VC, l))[o + lane + 64] = f2bf(s.vn[w][lane + 64]);
          }
        } else if (cg == 0 && w < R) {  // positions 0 and 1 of batch row w
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const long long o = (((long long)w * NKV + h) * p.Lmax + t) * D;
            ((bf16_t*)lp(PT_KC, l))[o + lane] = f2bf(s.pkk[w][t][lane]);
            ((bf16_t*)lp(PT_KC, l))[o + lane + 64] = f2bf(s.pkk[w][t][lane + 64]);
            ((bf16_t*)lp(PT_VC, l))[o + lane] = f2bf(s.pv[w][t][lane]);
            ((bf16_t*)lp(PT_VC, l))[o + lane + 64] = f2bf(s.pv[w][t][lane + 64]);
          }
        }
      }
      __syncthreads();
      // row rr's partial for column c (thread (rr, c < 32), waves 0-3): the tile's 4 waves summed in wave order -> the
      // owner of (tile 2cg + c / 16, row pair rr / 2), as granules (data = flag: no drain)
      if (tid < MR * 32) {
        const int rr = tid >> 5, c = tid & 31, tt = c >> 4, cc = c & 15;
        float v = 0.f;
#pragma unroll
        for (int q2 = 0; q2 < 4; ++q2) v += s.red[tt * 4 + q2][(rr >> 2) * 16 + cc][rr & 3];
        if (rr < RT)
          st_g(gpart + ((((size_t)(2 * cg + tt) * NQO + (rr >> 1)) * NKV + h) * 32 + (rr & 1) * 16 + cc),
               __float_as_uint(v), tagof(5 * l + 1));
      }
      CE_STAMP(sb + 5);
    }
    // ------------------------------------------------------------------ residual add by the owner, x16 edge
    {
      if (tid < NKV * 32 * NSL) {  // the 8 head partials of the owned slices (granules, polled; waves 0-3 / 0-7)
        const int si = tid >> 8, hp = (tid >> 5) & 7, sl = tid & 31, qq = qo + 4 * si;
        unsigned v = 0u;
        if (2 * qq + (sl >> 4) < RT) {
          const u64* g = gpart + ((((size_t)to * NQO + qq) * NKV + hp) * 32 + sl);
          const unsigned want = tagof(5 * l + 1);
          u64 x = ld_g(g);
          for (int spins = 0; (unsigned)(x >> 32) != want; ++spins) {
            if (spins > pk.spin) { atomicOr(err, 1); break; }
            __builtin_amdgcn_s_sleep(1);
            x = ld_g(g);
          }
          v = (unsigned)x;
        }
        s.gath[si][hp][sl] = __uint_as_float(v);
      }
      __syncthreads();
      CE_STAMP(sb + 6);
      if (pubw) {
        if (lane < 32 * NSL) {
          float v = 0.f;
#pragma unroll
          for (int hp = 0; hp < NKV; ++hp) v += s.gath[lane >> 5][hp][lane & 31];  // head order
          if (fuse && l == 0) {  // the residual rows: the chosen tokens' x rows (every row's granule was seen in P2)
            const int rr = orow(lane >> 4);
            if (rr < RT) {
              const int tok = min((int)(unsigned)ld_g(sgr + rr), pk.sa.V - 1);
              s.xown[lane >> 4][lane & 15] = pk.gx[(long long)tok * H + 16 * to + (lane & 15)];
            }
          }
          s.xown[lane >> 4][lane & 15] += v;
          if (dbg && orow(lane >> 4) < RT)
            dbg[dbgi(l, 0, orow(lane >> 4), 16 * to + (lane & 15))] = s.xown[lane >> 4][lane & 15];
        }
        publish_x16(0, tagof(5 * l + 2), lane);  // (the wave's own LDS writes above are complete: one wave, in order)
        if (EARLY) load_p3(l, tid);
      }
      if (LATE) {
        __syncthreads();
        load_p3(l, tid);
      }
      CE_STAMP(sb + 7);
    }
    // ------------------------------------------------------------------ P3: gate/up + SwiGLU
    {
      stage_x16(s, wsr, (unsigned)(LY::OFF_X16 + myrep * LY::REPL_X16), fl_off(myrep, FL_X0), tagof(5 * l + 2), RT, p.eps,
                pk.spin, err, tid);
      CE_STAMP(sb + 8);
      if (AHEAD) load_p4(l, tid);
      const int k3 = ntile3 == 2 ? (w & 3) * 8 : w * 4, n3 = ntile3 == 2 ? 8 : 4;
      u32x4_t af[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) af[i] = afrag_x(s, lm, lk, k3 + min(i, n3 - 1), RT);
      pin4(af);
      pin4(af + 4);
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (i < n3) acc = mfma(af[i], w3[i], acc);
      CE_AFTER(acc);
      CE_SUB(12);
      red_put(s, w, lane, acc);
      if (EARLY && !pubw) load_p4(l, tid);
      __syncthreads();
      CE_SUB(14);
      if (pubw) {  // SwiGLU of (tile j, row rr, column pair pp) from the partials, every replica, drain, flags
#pragma unroll
       for (int it = 0; it < NSL; ++it) {
        const int idx = lane + 64 * it;
        const int j = idx / (MR * 4), rr = (idx >> 2) % MR, pp = idx & 3;
        const int tile = j == 0 ? b : b + NB, nw = ntile3 == 2 ? 4 : 8;
        const bool mine = idx < ntile3 * MR * 4 && rr < RT;
        if (mine) {
          const int ml = (rr >> 2) * 16 + 2 * pp, e = rr & 3;  // MFMA lane of (row rr, gate column 2pp)
          float g0 = 0.f, g1 = 0.f, u0 = 0.f, u1 = 0.f;
          for (int ww = j * nw; ww < j * nw + nw; ++ww) {
            g0 += s.red[ww][ml][e]; g1 += s.red[ww][ml + 1][e];
            u0 += s.red[ww][ml + 8][e]; u1 += s.red[ww][ml + 9][e];
          }
          const float rsv = s.rs[rr];
          const float h0 = silu_f(g0 * rsv) * (u0 * rsv), h1 = silu_f(g1 * rsv) * (u1 * rsv);
          const unsigned hv = pack2bf(h0, h1);
          const unsigned o = (unsigned)LY::OFF_H + (unsigned)(rr * (I / 2) + tile * 4 + pp) * 4;
#pragma unroll
          for (int rp = 0; rp < NREPL; ++rp) bst_c(hv, wsr, o + rp * (unsigned)LY::REPL_H);
          if (dbg) {
            dbg[dbgi(l, 1, rr, tile * 8 + 2 * pp)] = __uint_as_float(hv << 16);
            dbg[dbgi(l, 1, rr, tile * 8 + 2 * pp + 1)] = __uint_as_float(hv & 0xFFFF0000u);
          }
        }
       }
        CE_SUB(17);
        drain_stores();
        CE_SUB(18);
        if (lane < NREPL) st_flag((unsigned*)(ws + fl_off(lane, FL_H)) + b, tagof(5 * l + 3));
        if (EARLY) load_p4(l, tid);
      }
      if (LATE) {
        __syncthreads();
        load_p4(l, tid);
      }
      CE_STAMP(sb + 9);
    }
    // ------------------------------------------------------------------ P4: down tile `to` for rows 2qo, 2qo + 1
    {
      CE_SUB(20);
      wait_flags(wsr, fl_off(myrep, FL_H), NB, tagof(5 * l + 3), pk.spin, err);
      CE_STAMP(sb + 10);
      {  // the owner's SwiGLU rows: thread -> owned row tid / 256 (+ 2), pairs (tid % 256) * 6 .. + 5
        const int p0 = (tid & 255) * 6;
        uint2 v[NSL][3];
#pragma unroll
        for (int si = 0; si < NSL; ++si) {
          const int i = (tid >> 8) + 2 * si, tr = orow(i);
#pragma unroll
          for (int k = 0; k < 3; ++k) v[si][k] = uint2{0u, 0u};
          if (tr < RT) {
            const unsigned o = (unsigned)(LY::OFF_H + myrep * LY::REPL_H) + (unsigned)(tr * (I / 2) + p0) * 4;
#pragma unroll
            for (int k = 0; k < 3; ++k) v[si][k] = bld2_c(wsr, o + 8 * k);
          }
        }
#pragma unroll
        for (int si = 0; si < NSL; ++si) {
          uint2* hrow = (uint2*)&s.a.ha[(tid >> 8) + 2 * si][2 * p0];
#pragma unroll
          for (int k = 0; k < 3; ++k) hrow[k] = v[si][k];
        }
      }
      CE_SUB(21);
      __syncthreads();
      CE_SUB(22);
      auto next_w1 = [&]() {
        if (l + 1 < L) load_p1(lp(PT_QKV, l + 1), (unsigned)(NQ + 2 * NKV) * D * H * 2, t1, tid);
        else if (b < p.V / 16) load_p1(p.w_lm, (unsigned)p.V * H * 2, b, tid);
      };
      if (AHEAD) next_w1();
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i0 = 0; i0 < 12; i0 += 6) {
        u32x4_t af[6];
#pragma unroll
        for (int i = 0; i < 6; ++i)
          af[i] = *(const u32x4_t*)(lm < 2 * NSL ? &s.a.ha[lm][(w * 12 + i0 + i) * 32 + lk * 8] : &s.zero[lk * 8]);
        pin4(af);
        asm volatile("" : "+v"(af[4]), "+v"(af[5]));
#pragma unroll
        for (int i = 0; i < 6; ++i) acc = mfma(af[i], w4[i0 + i], acc);
      }
      CE_AFTER(acc);
      red_put(s, w, lane, acc);
      if (EARLY && !pubw) next_w1();
      __syncthreads();
      CE_SUB(25);
      if (pubw) {
        if (lane < 32 * NSL) {  // (row lane / 16, column lane % 16) = MFMA row lane / 16 of MFMA lane lane % 16
          float v = 0.f;
#pragma unroll
          for (int ww = 0; ww < NW; ++ww) v += s.red[ww][lane & 15][lane >> 4];
          s.xown[lane >> 4][lane & 15] += v;
          if (dbg && orow(lane >> 4) < RT)
            dbg[dbgi(l, 2, orow(lane >> 4), 16 * to + (lane & 15))] = s.xown[lane >> 4][lane & 15];
        }
        publish_x16(1, tagof(5 * l + 4), lane);
        if (EARLY) next_w1();
      }
      if (LATE) {
        __syncthreads();
        next_w1();
      }
      CE_STAMP(sb + 11);
    }
  }
  // -------------------------------------------------------------------- final norm + lm_head[g] (tiles 0 .. V/16)
  {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, lm = lane & 15, lk = lane >> 4;
    stage_x16(s, wsr, (unsigned)(LY::OFF_X16 + myrep * LY::REPL_X16) + MR * (H / 2) * 4, fl_off(myrep, FL_X1),
              tagof(5 * (L - 1) + 4), RT, p.eps, pk.spin, err, tid);
    if (b < p.V / 16) {
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) acc = mfma(afrag_x(s, lm, lk, w * 4 + i, RT), w1[i], acc);
      red_put(s, w, lane, acc);
      __syncthreads();
      if (w == 0) {
        const f32x4_t v = red_sum(s, 0, NW, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rr = lk * 4 + i;
          // (prefill: the logits of position 1, token rows 2b + 1)
          if (rr < RT && (!PF || (rr & 1))) p.logits[(long long)(PF ? rr >> 1 : rr) * p.ldl + b * 16 + lm] = v[i] * s.rs[rr];
        }
      }
    }
    // the launch counter: every block read it before its first publication, and block 0 has consumed an edge from
    // every block by now
    if (b == 0 && tid == 0)
      __hip_atomic_store((unsigned*)(ws + OFF_EPOCH), ep + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    CE_STAMP(1);
  }
}

bool cp_step_resident() {
  static int cap[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
  if (cap[dev] == 0) {
    int per_cu = 1 << 20, cus = 0;  // every load-timing variant
    for (const void* k : {(const void*)cp_step_k<0, 0>, (const void*)cp_step_k<1, 0>, (const void*)cp_step_k<2, 0>,
                          (const void*)cp_step_k<1, 1>}) {
      int n = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, NT, 0) != hipSuccess) return false;
      per_cu = std::min(per_cu, n);
    }
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return false;
    cap[dev] = std::max(1, per_cu * cus);
  }
  return cap[dev] >= NB;
}

static int cp_step_go(const CEP& pk, int lm, void* stream) {
  if (lm == 0) hipLaunchKernelGGL((cp_step_k<0, 0>), dim3(NB), dim3(NT), 0, (hipStream_t)stream, pk);
  else if (lm == 1) hipLaunchKernelGGL((cp_step_k<1, 0>), dim3(NB), dim3(NT), 0, (hipStream_t)stream, pk);
  else hipLaunchKernelGGL((cp_step_k<2, 0>), dim3(NB), dim3(NT), 0, (hipStream_t)stream, pk);
  return hipGetLastError() == hipSuccess ? 0 : QT_ERR_LAUNCH;
}

}  // namespace

extern "C" long long qt_cp_step_ws_bytes(void) { return (long long)WS_BYTES; }
extern "C" long long qt_cp_step_dbg_bytes(void) { return (long long)(DBG_BYTES + STAMP_BYTES); }

extern "C" int qt_cp_step_supported(int H_, int I_, int Hq, int Hkv, int D_, int n_layers, int V) {
  return H_ == H && I_ == I && Hq == NQ && Hkv == NKV && D_ == D && n_layers >= 1 && n_layers <= 6 && V % 16 == 0 &&
         V / 16 <= NB && cp_step_resident();
}

static int qt_cp_step_check(const qt_cp_step_args* a) {
  if (!a || a->R < 1 || a->R > MAXR || a->n_layers < 1 || a->n_layers > 6) return QT_ERR_SHAPE;
  if (a->const_pos < 1 || a->const_pos > IC * GPW || a->const_pos >= a->Lmax) return QT_ERR_SHAPE;
  if (a->V % 16 || a->V / 16 > NB || a->V <= 0) return QT_ERR_SHAPE;
  if ((long long)a->R * NKV * a->Lmax * D * 2 >= (1ll << 31)) return QT_ERR_SHAPE;  // 32-bit buffer offsets
  if (!a->ws || a->ws_bytes < (long long)WS_BYTES || !a->x || !a->qkv0 || !a->logits || !a->w_lm || !a->cos_tab ||
      !a->sin_tab)
    return QT_ERR_ARG;
  for (int l = 0; l < a->n_layers; ++l)
    if (!a->w_qkv[l] || !a->w_o[l] || !a->w_gu[l] || !a->w_down[l] || !a->q_norm[l] || !a->k_norm[l] ||
        !a->k_cache[l] || !a->v_cache[l])
      return QT_ERR_ARG;
  if (!cp_step_resident()) return QT_ERR_SHAPE;
  return 0;
}

extern "C" int qt_cp_step(const qt_cp_step_args* a, void* stream) {
  const int rc = qt_cp_step_check(a);
  if (rc) return rc;
  static const int spin = std::max(1000, qt_knob("QT_CE_SPIN", 200000));
  static const int lm = qt_knob("QT_CE_LM", 1);  // load timing (probe builds only: the product reads no env)
  const CEP pk{*a, spin};
  return cp_step_go(pk, lm, stream);
}

// qt_cp_step with the previous step's token choice at its start (qt_cp_step_sampled, include/qwen3tts_amd.h)
extern "C" int qt_cp_step_sampled(const qt_cp_step_args* a, const qt_sample_args* sa, void* stream) {
  if (!a || !sa || sa->R != a->R || sa->V <= 0 || sa->V > 2048 || !sa->tok_out || !sa->logits) return QT_ERR_SHAPE;
  if (sa->do_sample && sa->top_k > sa->V) return QT_ERR_ARG;
  if (sa->ctr_stride < 0 || (sa->force && (!sa->pick || !sa->codes))) return QT_ERR_ARG;
  if (!sa->emb_table || sa->emb_dim != H || !sa->emb2_table || sa->emb2_dim != (NQ + 2 * NKV) * D) return QT_ERR_SHAPE;
  qt_cp_step_args b = *a;  // qkv0 / x come from the sampler's rows: any non-null pointer passes the checks
  if (!b.qkv0) b.qkv0 = sa->emb2_table;
  if (!b.x) b.x = (float*)sa->emb_table;
  const int rc = qt_cp_step_check(&b);
  if (rc) return rc;
  static const int spin = std::max(1000, qt_knob("QT_CE_SPIN", 200000));
  static const int lm = qt_knob("QT_CE_LM", 1);
  CEP pk{b, spin};
  pk.fuse = 1;
  pk.sa = *sa;
  pk.sa.emb_table = nullptr;  // the engine gathers the rows itself
  pk.sa.emb2_table = nullptr;
  pk.sa.emb_out16 = nullptr;
  pk.gx = sa->emb_table;
  pk.gq = sa->emb2_table;
  return cp_step_go(pk, lm, stream);
}


// The 2-token prefill of the same code predictor (M:1671-1675: positions 0 and 1 of every batch row -- the talker's
// hidden state and its first code's embedding -- through all layers, their keys / values appended at cache positions 0
// and 1, the logits of position 1 through lm_head[0]) in one launch of the same engine with 2 token rows per batch
// row.  x: fp32 [2R][ldx] (rows 2b, 2b + 1); qkv0 / const_pos unused; logits [R][ldl].
extern "C" int qt_cp_prefill(const qt_cp_step_args* a, void* stream) {
  if (!a || a->R < 1 || a->R > MAXR || a->n_layers < 1 || a->n_layers > 6) return QT_ERR_SHAPE;
  if (a->Lmax < 2 || a->V % 16 || a->V / 16 > NB || a->V <= 0) return QT_ERR_SHAPE;
  if ((long long)a->R * NKV * a->Lmax * D * 2 >= (1ll << 31)) return QT_ERR_SHAPE;
  if (!a->ws || a->ws_bytes < (long long)WS_BYTES || !a->x || !a->logits || !a->w_lm || !a->cos_tab || !a->sin_tab)
    return QT_ERR_ARG;
  for (int l = 0; l < a->n_layers; ++l)
    if (!a->w_qkv[l] || !a->w_o[l] || !a->w_gu[l] || !a->w_down[l] || !a->q_norm[l] || !a->k_norm[l] ||
        !a->k_cache[l] || !a->v_cache[l])
      return QT_ERR_ARG;
  if (a->ldx % 4) return QT_ERR_SHAPE;  // 16-byte row loads
  if (!cp_step_resident()) return QT_ERR_SHAPE;
  static const int spin = std::max(1000, qt_knob("QT_CE_SPIN", 200000));
  const CEP pk{*a, spin};
  hipLaunchKernelGGL((cp_step_k<1, 1>), dim3(NB), dim3(NT), 0, (hipStream_t)stream, pk);
  return hipGetLastError() == hipSuccess ? 0 : QT_ERR_LAUNCH;
}
