// gemm_pf2_k: the prefill linears' GEMM (talker / code-predictor prefill q/k/v, o_proj, gate/up + SwiGLU, down;
// codec pre-transformer linears on bf16 activations), routed here by qt_gemm (gemm.hip) for bf16 A + bf16 pre-tiled
// weights with K % 64 == 0.  Own translation unit so the tile configurations build in parallel with gemm.hip.
#include "gemm_p.h"
#include "engine_dev.h"
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#ifdef QT_PF2_STAMPS  // diagnostic build only (tools/pf2_probe.hip): per-block cycle stamps of wave 0
__device__ unsigned long long pf2_stamps[1 << 14][4];
#define PF2_STAMP(k)                                                                            \
  do {                                                                                          \
    if (threadIdx.x == 0 && blockIdx.x + blockIdx.y * gridDim.x < (1 << 14))                   \
      pf2_stamps[blockIdx.x + blockIdx.y * gridDim.x][k] = __builtin_amdgcn_s_memtime();           \
  } while (0)
#else
#define PF2_STAMP(k) do { } while (0)
#endif

namespace {

using qt_gemm_impl::GemmP;

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
constexpr int PF2_KS_MAX = 4;  // split-K factor bound (narrow outputs)

// SiLU from the hardware exp2 / reciprocal (v_exp_f32, v_rcp_f32: ~1 ulp each, 4 instructions): the IEEE
// division + range-reduced expf of silu_f cost ~40 VALU per element, which made the SwiGLU epilogue of a
// 256 x 160 tile 30k cycles (the output is rounded to bf16 anyway).
QT_DEV float silu_fast(float g) {
  return g * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-1.44269504088896341f * g));
}

// Prefill linear GEMM, deep pipeline (taps == 0, bf16 A and bf16 pre-tiled W, K % 64 == 0): block tile BM rows x
// NTB*16 columns, 4 waves in a 2 x 2 grid (wave = BM/2 rows x NTB/2 column tiles of 16x16x32 MFMAs), K in 64-deep
// stages, NS LDS stages.  Both operands go global -> LDS by LDS-DMA (global_load_lds_dwordx4, inline asm, no VGPR
// staging) and NS - 1 stages are in flight while one is multiplied: a counted `s_waitcnt vmcnt` retires exactly the
// stage about to be read and a raw `s_barrier` (no vmcnt(0) drain) publishes it (cdna_hip_programming.md §5
// "Pipelining across barriers").  gemm_pf_k (one stage of register-staged prefetch) left each 512-cycle MFMA stage
// waiting on the next stage's L2/HBM round trip: M=680 talker layer 293 us = 234 TFLOP/s, hipBLASLt 130 us
// (tools/pf_gemm_probe.py).
// LDS images are lane-linear 1 KiB fragments, exactly the MFMA operand order: B fragments are the pre-tiled weight
// tiles copied verbatim (1 KiB contiguous per DMA instruction); an A fragment (16 rows x 32 k) is gathered by one DMA
// instruction whose lane j reads row j & 15, k chunk j >> 4 (16 rows x 64 B), so every ds_read_b128 of an operand is
// conflict-free.  The RMSNorm sums of squares come from the A fragments the MFMA reads (column-half-0 waves).
// Blocks are remapped so the row tiles of one column tile are dealt to one XCD (its weight slice is fetched into one
// L2 once, speed only).  Same operand rounding and per-element k order as gemm_pf_k / igemm_k.
QT_DEV void glds16(const void* g, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}
QT_DEV unsigned lds_u32(const void* p) {
  return __builtin_amdgcn_readfirstlane((unsigned)(size_t)(const __attribute__((address_space(3))) void*)p);
}
template <int N> QT_DEV void vm_wait_n() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// wait until at most min(after, MAXA) stages of G DMA instructions each remain in flight (vmcnt <= 63)
template <int G, int MAXA>
QT_DEV void vm_wait_stages(int after) {
  if constexpr (MAXA <= 0) {
    vm_wait_n<0>();
  } else {
    static_assert(MAXA * G <= 63, "vmcnt range");
    if (after >= MAXA) vm_wait_n<MAXA * G>();
    else vm_wait_stages<G, MAXA - 1>(after);
  }
}
QT_DEV void raw_barrier() { asm volatile("s_barrier" ::: "memory"); }
template <int I, int N, typename F>
QT_DEV void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// EPI: the epilogue, compile-time for the prefill linears' plain forms (no act / bias / colscale): PF2_STORE,
// PF2_ADD (residual add), PF2_ADD_OUT2 (+ bf16 shadow), PF2_SWIGLU; PF2_GENERIC reads all of it from GemmP.
// ABL (measurement only, tools/pf2_probe.hip), bit mask: 1 no MFMA (fragment reads kept live), 2 no loads after the
// prologue (the rest runs on stale stages), 4 no fragment reads (and no MFMA), 8 no epilogue (accumulators kept live),
// 16 (PP) every block reads column tile 0's weights, 32 (PP) every block reads row tile 0's activations
enum { PF2_GENERIC = -1, PF2_STORE = 0, PF2_ADD = 1, PF2_SWIGLU = 2, PF2_ADD_OUT2 = 3 };
// PP: the ping-pong schedule (8 waves = two groups of 4, WM = 4 x WN = 2: waves 0-3 own rows [0, BM/2), waves 4-7
// rows [BM/2, BM)).  Group 1 runs one barrier behind group 0, so on every SIMD one wave multiplies while the other
// group's wave reads its next stage's fragments from LDS and issues DMAs: the MFMA pipe no longer idles through the
// fragment reads and the barrier of a stage (cdna_hip_programming.md §5 "The 256^2 8-phase template": the staggered
// wave groups; two phases per 64-deep stage here).  Per stage s (PP = 3, the product form):
//   group 0:  R(s): issue stage s+NS-1, read stage s's fragments | k=2s   | C(s): MFMAs, wait stage s+1 | k=2s+1
//   group 1:  (stagger barrier k=0 first)  R(s): read, wait stage s+1 | k=2s+1 | C(s): MFMAs, issue stage s+NS | k=2s+2
// Stage s is waited for by every wave before barrier 2s-1 (the one before group 0 first reads it); its LDS slot is
// refilled (stage s+NS) only after barrier 2s+1, which ends group 1's read of it (lgkmcnt(0) before that barrier).
// PP = 1 issues group 1's stage before its MFMAs instead (measured slower: an LDS-DMA issue costs the issuing wave
// ~100 cycles, MI355X_MICROARCH.md cycle constants; profiles/r06_pf2_pingpong_probe.txt).
// The DMA pieces (A_FR + B_FR of 1 KiB) are dealt round-robin over the 8 waves (the first TOT % 8 waves take one
// more), so tile widths whose fragment count is not a multiple of 8 (BN = 160) work; each wave counts its own.
template <typename OT, int BM, int NTB, int NS, int WM, int WN, bool AFL, int EPI, int ABL = 0, bool SPLIT = false,
          int PP = 0>
__global__ __launch_bounds__(WM * WN * 64) void gemm_pf2_k(GemmP p) {
  constexpr int NW = WM * WN;
  constexpr int MI = BM / WM / 16;            // row fragments per wave
  constexpr int CT = NTB / WN;                // column tiles per wave
  constexpr int A_FR = BM / 8, B_FR = NTB * 2;  // 1 KiB fragments per stage
  constexpr int STAGE = (A_FR + B_FR) * 512;  // bf16 elements per stage
  constexpr int GA = A_FR / NW, GB = B_FR / NW, G = GA + GB;  // DMA instructions per wave per stage
  static_assert(PP || (A_FR % NW == 0 && B_FR % NW == 0), "fragments split over the waves");
  static_assert(MI >= 1 && CT >= 1 && NTB % WN == 0 && BM % (WM * 16) == 0, "wave tiles");
  static_assert(!PP || (WM == 4 && WN == 2 && AFL && NS >= 2 && (PP == 1 || PP == 3)), "ping-pong: two groups of 2 x 2 waves");
  // NS stages, then the row sums of squares: WN partial sums per row (one per wave of a row block)
  // (one __shared__ object: the split-K arrival flag lives at its end, after the row sums)
  __shared__ __attribute__((aligned(16))) bf16_t smem_pf2[NS * STAGE + 2 * WN * BM + 8];
  float* ss_row = (float*)(smem_pf2 + NS * STAGE);
  PF2_STAMP(0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lm = lane & 15, lk = lane >> 4;
  const int ntl = (p.N + 15) / 16, ktiles = p.Kp / 32, S_all = p.Klog / 64;
  // split-K (narrow outputs with few tiles): block z of gridDim.y runs stages [s_lo, s_lo + S)
  // (a separate instantiation: the merge's code after the loop made hipcc keep the accumulators in AGPRs and copy
  // them through VGPRs every k step of the unsplit kernel, +15-20 %)
  const int KS = SPLIT ? (int)gridDim.y : 1, z = SPLIT ? (int)blockIdx.y : 0;
  const int s_lo = S_all * z / KS, S = S_all * (z + 1) / KS - s_lo;
  // XCD-aware tile order: blocks that share an XCD (linear id % 8) take consecutive tiles, row tiles fastest
  const int mtiles = (p.M + BM - 1) / BM, ctiles = (ntl + NTB - 1) / NTB;
  const int nwg = mtiles * ctiles, orig = blockIdx.x, xcd = orig % 8, q = nwg / 8, rr = nwg % 8;
  const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int m0 = (wg % mtiles) * BM, nt0 = (wg / mtiles) * NTB;
  const int wr = (w / WN) * (BM / WM), wc = (w % WN) * CT;
  const bool norm = p.rms != 0;
  const bf16_t* Ab = (const bf16_t*)p.A;
  const bf16_t* Wb = (const bf16_t*)p.W;
  // this lane's DMA sources: A fragment f = w * GA + i covers rows (f >> 1) * 16.., k tile f & 1
  const int arow = min(m0 + lm, p.M - 1);
  const unsigned lbase = lds_u32(smem_pf2);
  // this lane's DMA sources at the split's first stage, computed once (row clamp, swizzle, 64-bit address math);
  // a stage advances an A piece by 64 k (128 B) and a B piece by two fragments (2 KiB)
  const bf16_t* asrc[GA > 0 ? GA : 1];
  const bf16_t* bsrc[GB > 0 ? GB : 1];
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int f = w * GA + i;
    if constexpr (AFL) {  // full 128-B lines: piece f = rows 8f..8f+7 x 64 k, 16-B chunk c of row r at c ^ ((r >> 1) & 7)
      const int rr = f * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((rr >> 1) & 7);
      const int row = min(m0 + rr, p.M - 1);
      asrc[i] = Ab + (long long)row * p.lda + s_lo * 64 + c * 8;
    } else {  // MFMA fragment order: 16 rows x 64 B per piece
      const int mt = f >> 1, kt = f & 1;
      const int row = min(arow + mt * 16, p.M - 1);
      asrc[i] = Ab + (long long)row * p.lda + s_lo * 64 + kt * 32 + lk * 8;
    }
  }
#pragma unroll
  for (int i = 0; i < GB; ++i) {
    const int f = w * GB + i, ct = f >> 1, kt = f & 1;
    const int nt = min(nt0 + ct, ntl - 1);
    bsrc[i] = Wb + ((size_t)nt * ktiles + s_lo * 2 + kt) * 512 + lane * 8;
  }
  auto issue = [&](int ls) {  // local stage ls of this split: LDS buffer ls % NS, k offset of global stage s_lo + ls
    const unsigned sb = lbase + (unsigned)((ls % NS) * STAGE * 2);
#pragma unroll
    for (int i = 0; i < GA; ++i) glds16(asrc[i] + ls * 64, sb + (w * GA + i) * 1024);
#pragma unroll
    for (int i = 0; i < GB; ++i) glds16(bsrc[i] + ls * 1024, sb + (A_FR + w * GB + i) * 1024);
  };
  f32x4_t acc[MI][CT];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < CT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // RMSNorm sums of squares from the A fragments the MFMAs read: the WN waves of a row block hold the same
  // fragments, wave j of them takes the fragment dwords e with e % WN == j (v_dot2 on the bf16 pairs, fp32 sums)
  float ss[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) ss[i] = 0.f;
  const int wj = w % WN;
  if constexpr (PP) {
    constexpr int TOT = A_FR + B_FR, GQ = TOT / NW, GR = TOT % NW, GMAX = GQ + (GR ? 1 : 0);
    const bool extra = w < GR;  // wave-uniform: this wave issues GQ + 1 pieces per stage
    const int g = w >> 2;
    // this lane's source of each of its pieces at the split's first stage (row clamp, swizzle and 64-bit address math
    // once, not per stage) and the piece's advance per stage: 64 k of an A row (128 B) or two B fragments (2 KiB)
    const bf16_t* gsrc[GMAX];
    bool isa[GMAX];
#pragma unroll
    for (int i = 0; i < GMAX; ++i) {
      const int f = min(w + NW * i, A_FR + B_FR - 1);
      isa[i] = f < A_FR;
      if (isa[i]) {  // full 128-B lines: rows 8f..8f+7 x 64 k, 16-B chunk c of row r at c ^ ((r >> 1) & 7)
        const int rr = f * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((rr >> 1) & 7);
        const int row = (ABL & 32) ? rr : min(m0 + rr, p.M - 1);
        gsrc[i] = Ab + (long long)row * p.lda + s_lo * 64 + c * 8;
      } else {
        const int fb = f - A_FR, ct = fb >> 1, kt = fb & 1;
        const int nt = (ABL & 16) ? ct : min(nt0 + ct, ntl - 1);
        gsrc[i] = Wb + ((size_t)nt * ktiles + s_lo * 2 + kt) * 512 + lane * 8;
      }
    }
    auto issue_pp = [&](int ls) {
      const unsigned sb = lbase + (unsigned)((ls % NS) * STAGE * 2);
#pragma unroll
      for (int i = 0; i < GMAX; ++i)
        if (i < GQ || extra) glds16(gsrc[i] + (isa[i] ? ls * 64 : ls * 1024), sb + (w + NW * i) * 1024);
    };
    // wait until at most `after` stages issued after the awaited one remain in flight (this wave's own DMAs)
    auto wait_pp = [&](int after) {
      if (GR && extra) vm_wait_stages<GQ + 1, NS - 1>(after);
      else vm_wait_stages<GQ, NS - 1>(after);
    };
    u32x4_t af[2][MI], bfr[2][CT];
    auto read_frags = [&](int s, auto&& between) {
      if constexpr ((ABL & 4) != 0) { between(); return; }
      const bf16_t* sa = smem_pf2 + (s % NS) * STAGE;
      const bf16_t* sbf = sa + A_FR * 512;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int j = 0; j < CT; ++j) bfr[kk][j] = *(const u32x4_t*)(sbf + ((wc + j) * 2 + kk) * 512 + lane * 8);
#pragma unroll
        for (int i = 0; i < MI; ++i)
          af[kk][i] = *(const u32x4_t*)(sa + (wr + i * 16 + lm) * 64 + (((kk * 4 + lk) ^ (lm >> 1)) * 8));
      }
      __builtin_amdgcn_sched_barrier(0);
      between();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    };
    auto compute = [&]() {
      if constexpr ((ABL & 4) != 0) return;
      if constexpr ((ABL & 1) != 0) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
          for (int i = 0; i < MI; ++i) asm volatile("" ::"v"(af[kk][i]));
#pragma unroll
          for (int j = 0; j < CT; ++j) asm volatile("" ::"v"(bfr[kk][j]));
        }
        return;
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < CT; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[kk][i]),
                                                                __builtin_bit_cast(bf16x8_t, bfr[kk][j]), acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      if (norm) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int e2 = 0; e2 < 4 / WN; ++e2) {
              unsigned d = af[kk][i][e2 * WN];
#pragma unroll
              for (int t = 1; t < WN; ++t) d = wj == t ? af[kk][i][e2 * WN + t] : d;
              const bf16x2_t h = __builtin_bit_cast(bf16x2_t, d);
              ss[i] = __builtin_amdgcn_fdot2_f32_bf16(h, h, ss[i], false);
            }
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    auto bar = [&]() {
      __builtin_amdgcn_sched_barrier(0);
      raw_barrier();
      __builtin_amdgcn_sched_barrier(0);
    };
    auto nop = [] {};
    {
      // prologue: group 0 stages 0..NS-2 (it issues NS-1 in R(0)), group 1 stages 0..NS-1; stage 0 landed for all
#pragma unroll
      for (int s = 0; s < NS - 1; ++s)
        if (s < S) issue_pp(s);
      if (g == 1 && NS - 1 < S) issue_pp(NS - 1);
      wait_pp(min(S - 1, g == 0 ? NS - 2 : NS - 1));
      bar();
      if (g == 0) {
        for (int s = 0; s < S; ++s) {
          if (!(ABL & 2) && s + NS - 1 < S) issue_pp(s + NS - 1);
          read_frags(s, nop);
          bar();  // k = 2s
          compute();
          if (s + 1 < S) wait_pp(min(S - 1, s + NS - 1) - (s + 1));
          bar();  // k = 2s + 1
        }
        bar();  // group 1's last barrier
      } else {
        bar();  // k = 0: the stagger
        for (int s = 0; s < S; ++s) {
          read_frags(s, nop);
          if (s + 1 < S) wait_pp(min(S - 1, s + NS - 1) - (s + 1));
          bar();  // k = 2s + 1
          if (PP == 1 && !(ABL & 2) && s + NS < S) issue_pp(s + NS);
          compute();
          if (PP == 3 && !(ABL & 2) && s + NS < S) issue_pp(s + NS);
          bar();  // k = 2s + 2
        }
      }
    }
  } else {
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < S) issue(s);
  for (int s = 0; s < S; ++s) {
    // retire stage s (this wave's DMAs): the stages issued after it may stay in flight
    const int after = min(S - 1, s + NS - 2) - s;
    vm_wait_stages<G, NS - 2>(after);
    raw_barrier();  // every wave's stage-s DMAs landed; every wave is done reading stage s - 1's buffer
    if (!(ABL & 2) && s + NS - 1 < S) issue(s + NS - 1);
    if constexpr ((ABL & 4) != 0) continue;
    const bf16_t* sa = smem_pf2 + (s % NS) * STAGE;
    const bf16_t* sbf = sa + A_FR * 512;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      u32x4_t af[MI], bfr[CT];
#pragma unroll
      for (int j = 0; j < CT; ++j) bfr[j] = *(const u32x4_t*)(sbf + ((wc + j) * 2 + kk) * 512 + lane * 8);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        if constexpr (AFL) af[i] = *(const u32x4_t*)(sa + (wr + i * 16 + lm) * 64 + (((kk * 4 + lk) ^ (lm >> 1)) * 8));
        else af[i] = *(const u32x4_t*)(sa + ((wr / 16 + i) * 2 + kk) * 512 + lane * 8);
      }
      if constexpr ((ABL & 1) != 0) {
#pragma unroll
        for (int i = 0; i < MI; ++i) asm volatile("" ::"v"(af[i]));
#pragma unroll
        for (int j = 0; j < CT; ++j) asm volatile("" ::"v"(bfr[j]));
      } else {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < CT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[i]),
                                                              __builtin_bit_cast(bf16x8_t, bfr[j]), acc[i][j], 0, 0, 0);
      }
      if (norm) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int e2 = 0; e2 < 4 / WN; ++e2) {
            unsigned d = af[i][e2 * WN];
#pragma unroll
            for (int t = 1; t < WN; ++t) d = wj == t ? af[i][e2 * WN + t] : d;  // wave-uniform select, no branch
            const bf16x2_t h = __builtin_bit_cast(bf16x2_t, d);
            ss[i] = __builtin_amdgcn_fdot2_f32_bf16(h, h, ss[i], false);
          }
      }
    }
  }
  }  // !PP
  PF2_STAMP(1);
  if (norm) {  // row sums: lanes l, l^16, l^32, l^48 hold the four k chunks of row l & 15
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      float v = ss[i] + xor_lane<16>(ss[i]);
      v += xor_lane<32>(v);
      if (lane < 16) ss_row[wj * BM + wr + i * 16 + lane] = v;
    }
    __syncthreads();  // (no DMA in flight any more)
  }
  if constexpr (SPLIT) {
    // deterministic split-K: every split stores its accumulators (and row sums of squares) write-through (16-byte sc1
    // buffer stores), one lane counts the arrival after every storing wave's drain + a barrier, and the last split to
    // arrive sums all splits' records in split order (its own from registers, the others by 16-byte sc1 loads), then
    // runs the epilogue (MI355X_MICROARCH.md visibility table, first row; cdna_hip_programming.md §5 "Projection GEMM
    // at M = 256" item 2, the sc1 form)
    constexpr int FR = MI * CT, REC = NW * FR * 256 + WN * BM;  // floats per split record
    int& pf2_last = *(int*)(smem_pf2 + NS * STAGE + 2 * WN * BM);
    const qt_engine::rsrc_t rr_all = qt_engine::mkr(p.part + (size_t)wg * KS * REC, (unsigned)(KS * REC * 4));
    const unsigned own = (unsigned)z * REC * 4;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < CT; ++j)
        qt_engine::bst4_c(__builtin_bit_cast(u32x4_t, acc[i][j]), rr_all,
                          own + (unsigned)(((w * FR + i * CT + j) * 256 + lane * 4) * 4));
    const unsigned sso = (unsigned)(NW * FR * 256) * 4;
    if (norm)
      for (int e = tid; e < WN * BM; e += NW * 64)
        qt_engine::bst_c(__float_as_uint(ss_row[e]), rr_all, own + sso + e * 4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains before the arrival is counted
    __syncthreads();
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(p.cnt + wg, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      pf2_last = old == (unsigned)KS - 1;
      if (pf2_last) __hip_atomic_store(p.cnt + wg, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    }
    __syncthreads();
    if (!pf2_last) return;
    auto merge = [&](auto KSC) {
      constexpr int KSN = decltype(KSC)::value;
      // the other KSN - 1 records (k -> split k + (k >= z)) in flight before the adds; no branch around a load
      f32x4_t v[KSN - 1][MI][CT];
#pragma unroll
      for (int k = 0; k < KSN - 1; ++k)
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < CT; ++j)
            v[k][i][j] = __builtin_bit_cast(f32x4_t, qt_engine::bld_c(rr_all, (unsigned)((k + (k >= z)) * REC * 4) +
                                                                       (unsigned)(((w * FR + i * CT + j) * 256 + lane * 4) * 4)));
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < CT; ++j) {
          f32x4_t t = z == 0 ? acc[i][j] : v[0][i][j];
#pragma unroll
          for (int zz = 1; zz < KSN; ++zz)  // split order: split zz is the own partial, v[zz] or v[zz - 1]
            t += zz == z ? acc[i][j] : (zz < z ? v[zz < KSN - 1 ? zz : KSN - 2][i][j] : v[zz - 1][i][j]);
          acc[i][j] = t;
        }
    };
    if (KS == 2) merge(std::integral_constant<int, 2>{});
    else if (KS == 3) merge(std::integral_constant<int, 3>{});
    else merge(std::integral_constant<int, PF2_KS_MAX>{});
    if (norm) {
      for (int e = tid; e < WN * BM; e += NW * 64) {
        float t = 0.f;
        for (int zz = 0; zz < KS; ++zz)
          t += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rr_all, (int)(zz * REC * 4 + sso + e * 4), 0, qt_engine::SC1));
        ss_row[e] = t;
      }
      __syncthreads();
    }
  }
  if constexpr ((ABL & 8) != 0) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < CT; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  OT* out = (OT*)p.out;
  // Epilogue.  Everything a store depends on is loaded before the first store: vmcnt counts loads and stores in
  // issue order, so a load issued after a store makes its consumer wait for that store's round trip (one per tile
  // when bias / residual loads were interleaved with the stores).  Interior blocks store without bounds checks, and
  // the plain forms have no per-element branches (each one had cost an exec-mask branch per element).
  const float inv_k = 1.f / (float)p.Klog;
  float rsc[MI][4];  // per-row RMS scale of this lane's rows wr + i*16 + lk*4 + e
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) rsc[i][e] = 1.f;
  if (norm) {
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      f32x4_t t = *(const f32x4_t*)(ss_row + wr + i * 16 + lk * 4);
#pragma unroll
      for (int j = 1; j < WN; ++j) t += *(const f32x4_t*)(ss_row + j * BM + wr + i * 16 + lk * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) rsc[i][e] = rsqrtf(t[e] * inv_k + p.eps);
    }
  }
  float cb[CT], cc[CT];  // bias / colscale of this lane's columns (clamped addresses: no branch around a load)
#pragma unroll
  for (int q = 0; q < CT; ++q) { cb[q] = 0.f; cc[q] = 1.f; }
  if constexpr (EPI == PF2_GENERIC) {
    if (p.bias) {
#pragma unroll
      for (int q = 0; q < CT; ++q) cb[q] = p.bias[min((nt0 + wc + q) * 16 + lm, p.N - 1)];
    }
    if (p.colscale) {
#pragma unroll
      for (int q = 0; q < CT; ++q) cc[q] = p.colscale[min((nt0 + wc + q) * 16 + lm, p.N - 1)];
    }
  }
  const bool add = EPI == PF2_GENERIC ? p.epi == QT_EPI_ADD : (EPI == PF2_ADD || EPI == PF2_ADD_OUT2);
  const bool swiglu = EPI == PF2_GENERIC ? p.epi == QT_EPI_SWIGLU : EPI == PF2_SWIGLU;
  // residual rows are loaded RCH row fragments at a time (all of them up to 64 registers)
  // (32 registers in the ping-pong kernels: two waves per SIMD, 256 registers each)
  constexpr int RB = PP ? 32 : 64;
  constexpr int RCH = (MI * CT * 4 <= RB) ? MI : (RB / (CT * 4) > 0 ? RB / (CT * 4) : 1);
  auto run = [&](auto FULLC) {
    constexpr bool FULL = decltype(FULLC)::value;
    static_for<0, (MI + RCH - 1) / RCH>([&](auto C) {
      constexpr int i0 = decltype(C)::value * RCH;
      constexpr int i1 = i0 + RCH < MI ? i0 + RCH : MI;
      float res[RCH][CT][4];
      if (add) {
#pragma unroll
        for (int i = i0; i < i1; ++i)
#pragma unroll
          for (int q = 0; q < CT; ++q) {
            const int n = FULL ? (nt0 + wc + q) * 16 + lm : min((nt0 + wc + q) * 16 + lm, p.N - 1);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int m = FULL ? m0 + wr + i * 16 + lk * 4 + e : min(m0 + wr + i * 16 + lk * 4 + e, p.M - 1);
              res[i - i0][q][e] = to_f(out[(long long)m * p.ldo + n]);
            }
          }
      }
      static_for<i0 * CT, i1 * CT>([&](auto I) {
        constexpr int i = decltype(I)::value / CT, qd = decltype(I)::value % CT;
        const f32x4_t a = acc[i][qd];
        const int nt = nt0 + wc + qd;
        const int mb = m0 + wr + i * 16 + lk * 4;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if constexpr (EPI == PF2_GENERIC) {
            float x = a[e] * rsc[i][e] + cb[qd];
            if (p.act != QT_ACT_NONE) x = act_f(x, p.act);
            v[e] = x * cc[qd];
          } else {
            v[e] = a[e] * rsc[i][e];
          }
        }
        if (swiglu) {
          // lanes lm < 8 hold the gate columns, lm >= 8 the matching up columns: every lane forms the products
          // of column lm & 7 and stores two of the four rows (no idle half)
          float r[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float pv = half_partner<16>(v[e]);
            const float g = lm < 8 ? v[e] : pv, u = lm < 8 ? pv : v[e];
            r[e] = silu_fast(g) * u;
          }
          const int c = nt * 8 + (lm & 7);
#pragma unroll
          for (int e2 = 0; e2 < 2; ++e2) {
            const int m = mb + (lm < 8 ? e2 : e2 + 2);
            const float val = lm < 8 ? r[e2] : r[e2 + 2];
            if (FULL || (m < p.M && nt < ntl && c < (p.N >> 1))) out[(long long)m * p.ldo + c] = from_f<OT>(val);
          }
        } else {
          const int n = nt * 16 + lm;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int m = mb + e;
            const float r = add ? res[i - i0][qd][e] + v[e] : v[e];
            if (FULL || (m < p.M && nt < ntl && n < p.N)) {
              out[(long long)m * p.ldo + n] = from_f<OT>(r);
              if constexpr (EPI == PF2_ADD_OUT2) p.out2[(long long)m * p.ldo2 + n] = f2bf(r);
              else if constexpr (EPI == PF2_GENERIC) { if (p.out2) p.out2[(long long)m * p.ldo2 + n] = f2bf(r); }
            }
          }
        }
      });
    });
  };
  if (m0 + BM <= p.M && (nt0 + NTB) * 16 <= p.N) run(std::true_type{});
  else run(std::false_type{});
  PF2_STAMP(2);
}

// split-K factor for a launch of nwg tiles: narrow (<= 2048-column) outputs whose tiles leave most CUs idle split K
// (>= 16 stages of 64 per split; wide outputs measured slower split: 1.7B q/k/v at 80 rows 15.5 -> 17.9 us) when the caller's workspace holds the split records (QT_PF2_SPLIT=0 disables, measurement)
template <int BM, int NTB, int WM, int WN>
int pf2_splits(const GemmP& p, int nwg) {
  static const int env = qt_knob("QT_PF2_SPLIT", 1);
  const int S = p.Klog / 64;
  if (!env || p.part == nullptr || p.cnt == nullptr || p.N > 2048 || nwg >= 192 || S < 32) return 1;
  int ks = std::min({PF2_KS_MAX, 256 / nwg, S / 16});
  constexpr int NW = WM * WN, MI = BM / WM / 16, CT = NTB / WN;
  const long long rec = (long long)NW * MI * CT * 256 + WN * BM;
  while (ks > 1 && (long long)nwg * ks * rec * 4 > p.part_bytes) --ks;
  return std::max(ks, 1);
}

template <typename OT, int BM, int NTB, int NS, int WM = 2, int WN = 2, bool AFL = true, int PP = 0>
void launch_pf2(const GemmP& p, hipStream_t s, int ks_pp = 1) {
  const int ntl = (p.N + 15) / 16;
  const int nwg = ((p.M + BM - 1) / BM) * ((ntl + NTB - 1) / NTB);
  const int ks = PP ? ks_pp : (BM <= 128 ? pf2_splits<BM, NTB, WM, WN>(p, nwg) : 1);
  const dim3 g(nwg, ks), b(WM * WN * 64);
  const bool plain = p.act == QT_ACT_NONE && p.bias == nullptr && p.colscale == nullptr;
  if constexpr (BM <= 128) {
    if (ks > 1) {  // narrow outputs: the split instantiations
      if constexpr (std::is_same<OT, bf16_t>::value) {
        if (plain && p.epi == QT_EPI_SWIGLU)
          { hipLaunchKernelGGL((gemm_pf2_k<OT, BM, NTB, NS, WM, WN, AFL, PF2_SWIGLU, 0, true, PP>), g, b, 0, s, p); return; }
      } else {
        if (plain && p.epi == QT_EPI_STORE && !p.out2)
          { hipLaunchKernelGGL((gemm_pf2_k<OT, BM, NTB, NS, WM, WN, AFL, PF2_STORE, 0, true, PP>), g, b, 0, s, p); return; }
        if (plain && p.epi == QT_EPI_ADD && !p.out2)
          { hipLaunchKernelGGL((gemm_pf2_k<OT, BM, NTB, NS, WM, WN, AFL, PF2_ADD, 0, true, PP>), g, b, 0, s, p); return; }
        if (plain && p.epi == QT_EPI_ADD && p.out2)
          { hipLaunchKernelGGL((gemm_pf2_k<OT, BM, NTB, NS, WM, WN, AFL, PF2_ADD_OUT2, 0, true, PP>), g, b, 0, s, p); return; }
      }
      hipLaunchKernelGGL((gemm_pf2_k<OT, BM, NTB, NS, WM, WN, AFL, PF2_GENERIC, 0, true, PP>), g, b, 0, s, p);
      return;
    }
  }
  if constexpr (std::is_same<OT, bf16_t>::value) {
    if (plain && p.epi == QT_EPI_SWIGLU)
      { hipLaunchKernelGGL((gemm_pf2_k<OT, BM, NTB, NS, WM, WN, AFL, PF2_SWIGLU, 0, false, PP>), g, b, 0, s, p); return; }
  } else {
    if (plain && p.epi == QT_EPI_STORE && !p.out2)
      { hipLaunchKernelGGL((gemm_pf2_k<OT, BM, NTB, NS, WM, WN, AFL, PF2_STORE, 0, false, PP>), g, b, 0, s, p); return; }
    if (plain && p.epi == QT_EPI_ADD && !p.out2)
      { hipLaunchKernelGGL((gemm_pf2_k<OT, BM, NTB, NS, WM, WN, AFL, PF2_ADD, 0, false, PP>), g, b, 0, s, p); return; }
    if (plain && p.epi == QT_EPI_ADD && p.out2)
      { hipLaunchKernelGGL((gemm_pf2_k<OT, BM, NTB, NS, WM, WN, AFL, PF2_ADD_OUT2, 0, false, PP>), g, b, 0, s, p); return; }
  }
  hipLaunchKernelGGL((gemm_pf2_k<OT, BM, NTB, NS, WM, WN, AFL, PF2_GENERIC, 0, false, PP>), g, b, 0, s, p);
}

#ifndef QT_PF2_PROBE
// Tile configuration (QT_PF2_CFG = 3 / 4 / 9 / 11 / 21 / 22 / 23 forces one, measurement; 0 = chosen by shape).
// tools/pf2_probe.hip timed every configuration on the 1.7B / 0.6B talker prefill shapes at M = 256 ... 4096
// (profiles/r03_pf2_probe_sweep.txt, profiles/r06_pf2_pingpong_probe.txt): a block's time is nearly independent of M
// and N (its loop runs K / 64 stages of a fixed tile), so launch time ~ ceil(blocks / resident slots) x block time,
// and the best tile is the one whose block count quantises best onto the 256 CUs.  Block cycles per 2048 of K and
// epilogue cycles below are those measurements; cfg 3 (72 KiB of LDS) runs 2 blocks per CU, the others 1.  The
// ping-pong configurations (pp, 8 waves in two staggered groups) are considered from 256 rows (long prefills: voice
// clone, non-streaming prompts); cfg 22 is cfg 21 with K split over two blocks (per-block K in its loop figure, its
// epilogue the record merge), only for <= 2048-column outputs whose two-fold grid fits the 256 CUs.
struct Pf2Cfg { int id, BM, BN, bpc; float loop1, loop2, epi; int pp, ks; };
constexpr Pf2Cfg PF2_CFGS[] = {
    {3, 128, 64, 2, 31000.f, 44000.f, 4000.f, 0, 1},   // 4 waves, wave tile 64 x 32
    {11, 64, 96, 1, 28000.f, 28000.f, 3000.f, 0, 1},   // 4 waves, wave tile 32 x 48
    {4, 256, 128, 1, 68000.f, 68000.f, 8000.f, 0, 1},  // 8 waves, wave tile 64 x 64
    {9, 256, 160, 1, 76500.f, 76500.f, 9000.f, 1, 1},  // ping-pong, 8 waves, wave tile 64 x 80 (4-wave form: 95000)
    {21, 128, 128, 1, 42600.f, 42600.f, 2500.f, 1, 1}, // ping-pong, 8 waves, wave tile 32 x 64
    {22, 128, 128, 1, 45000.f, 45000.f, 9500.f, 1, 2}, // cfg 21, split-K 2
    {23, 256, 256, 1, 97500.f, 97500.f, 10000.f, 1, 1}, // ping-pong, 8 waves, wave tile 64 x 128, 2 LDS stages
};
inline int pf2_cfg_env() {
  static const int v = qt_knob("QT_PF2_CFG", 0);
  return v;
}
inline bool pf2_split_fits(const GemmP& p, long long tiles, int ks) {  // cfg 22's records in the caller's workspace
  constexpr long long rec = 8ll * 2 * 4 * 256 + 2 * 128;  // NW x MI x CT x 256 + WN x BM floats
  return p.part != nullptr && p.cnt != nullptr && tiles <= 4096 && tiles * ks * rec * 4 <= p.part_bytes;
}
inline int pf2_pick(const GemmP& p) {
  static const int pp_env = qt_knob("QT_PF2_PP", 1);  // 0: without the ping-pong configurations (A/B)
  const int M = p.M, N = p.N, K = p.Klog;
  int best = 3;
  float best_t = 3.4e38f;
  for (const Pf2Cfg& c : PF2_CFGS) {
    if (c.pp && (M < 256 || !pp_env)) continue;
    const long long tiles = (long long)((M + c.BM - 1) / c.BM) * ((N + c.BN - 1) / c.BN);
    if (c.ks > 1 && (N > 2048 || tiles * c.ks > 256 || K / 64 < 32 || !pf2_split_fits(p, tiles, c.ks))) continue;
    const long long blocks = tiles * c.ks;
    const float kf = K / 2048.f / c.ks;
    float t;
    if (c.bpc == 2 && blocks > 256) t = (float)((blocks + 511) / 512) * (c.loop2 * kf + c.epi);
    else t = (float)((blocks + 255) / 256) * (c.loop1 * kf + c.epi);
    if (t < best_t) { best_t = t; best = c.id; }
  }
  return best;
}

template <typename OT>
void launch_pf2_auto(const GemmP& p, hipStream_t s) {
  int cfg = pf2_cfg_env();
  if (cfg == 0) cfg = pf2_pick(p);
  if (cfg == 22 && !pf2_split_fits(p, (long long)((p.M + 127) / 128) * ((p.N + 127) / 128), 2)) cfg = 21;
  // (deeper pipelines of the two small-tile configurations -- 7 stages of 64 x 96, 6 of 128 x 64, one block per CU --
  // measured slower at 24..680 rows: gate-up 160 rows 25.4 -> 37.9 us, qkv 680 rows 26.2 -> 37.1;
  // profiles/r04_pf2_deep_ab.txt)
  if (cfg == 4) launch_pf2<OT, 256, 8, 3, 4, 2>(p, s);
  else if (cfg == 9) launch_pf2<OT, 256, 10, 3, 4, 2, true, 3>(p, s);
  else if (cfg == 21) launch_pf2<OT, 128, 8, 4, 4, 2, true, 3>(p, s);
  else if (cfg == 22) launch_pf2<OT, 128, 8, 4, 4, 2, true, 3>(p, s, 2);
  else if (cfg == 23) launch_pf2<OT, 256, 16, 2, 4, 2, true, 3>(p, s);
  else if (cfg == 11) launch_pf2<OT, 64, 6, 4, 2, 2>(p, s);
  else launch_pf2<OT, 128, 4, 3>(p, s);
}
#endif  // QT_PF2_PROBE

}  // namespace

#ifndef QT_PF2_PROBE
namespace qt_gemm_impl {
void launch_pf2_auto_f32(const GemmP& p, hipStream_t s) { launch_pf2_auto<float>(p, s); }
void launch_pf2_auto_bf16(const GemmP& p, hipStream_t s) { launch_pf2_auto<bf16_t>(p, s); }
}  // namespace qt_gemm_impl
#endif  // QT_PF2_PROBE
