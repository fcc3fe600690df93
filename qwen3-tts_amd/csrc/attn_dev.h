// Device helpers shared by the decode attention kernels (attention.hip) and the code-predictor step engine
// (cp_engine.hip): hardware exp2, the lane-group softmax merge, RNE bf16 pair packing.
#pragma once
#include "common.h"

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;

// v_exp_f32 without the library's denormal-range scaling: arguments here are score differences <= 0, where
// results below 2^-126 (flushed) weigh nothing next to the row maximum's 1
QT_DEV float exp2_hw(float x) { return __builtin_amdgcn_exp2f(x); }

// Merge the online-softmax states (m, l, o[NREP][8]) of the lane groups of one wave (LPK lanes per group, each
// group's m uniform inside it): common max over the groups (readlane), rescale, then plain sums over the groups.
// Result: lane `lane` owns `cnt` consecutive output values starting at dim `d0` of head `jh` (totals of o) and
// that head's total l.  LPK == 16, NREP == 2 (the Qwen3 heads): a transpose-reduce over the four 16-lane rows
// -- two values share each VALU permlane swap, 12 swaps + 12 adds for the 16 o sums, every lane owns 4 outputs.
// Other shapes: xor butterflies, lane group 0 owns 8 outputs per head (cnt = 8 per head, looped by the caller).
template <int LPK, int NREP>
struct GroupMerge {
  static constexpr bool TR = LPK == 16 && NREP == 2;
  float mm[NREP];  // common max per head
  float t[TR ? 4 : NREP * 8];
  float lt[TR ? 1 : NREP];
  QT_DEV void run(float (&m)[NREP], float (&l)[NREP], float (&o)[NREP][8]) {
#pragma unroll
    for (int j = 0; j < NREP; ++j) {
      float x = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m[j]), 0));
#pragma unroll
      for (int g2 = LPK; g2 < 64; g2 += LPK)
        x = fmaxf(x, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m[j]), g2)));
      mm[j] = x;
      const float f = (m[j] == -INFINITY || x == -INFINITY) ? 0.f : exp2_hw(m[j] - x);
      l[j] *= f;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[j][i] *= f;
    }
    if constexpr (TR) {
      float v[16], s8[8];
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = o[i >> 3][i & 7];
#pragma unroll
      for (int i = 0; i < 8; ++i) {  // rows 0-1: v[i] half sums, rows 2-3: v[i + 8]
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[i]), __float_as_uint(v[i + 8]), false, false);
        s8[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {  // row rho: total of v[i + 4 rho]
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(s8[i]), __float_as_uint(s8[i + 4]), false, false);
        t[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
      }
      const auto rl = __builtin_amdgcn_permlane32_swap(__float_as_uint(l[0]), __float_as_uint(l[1]), false, false);
      const float lh = __uint_as_float(rl[0]) + __uint_as_float(rl[1]);
      const auto rl2 = __builtin_amdgcn_permlane16_swap(__float_as_uint(lh), __float_as_uint(lh), false, false);
      lt[0] = __uint_as_float(rl2[0]) + __uint_as_float(rl2[1]);  // rows 0-1: l[0], rows 2-3: l[1]
    } else {
      auto gsum = [](float x) {
        if constexpr (LPK <= 1) x += xor_lane<1>(x);
        if constexpr (LPK <= 2) x += xor_lane<2>(x);
        if constexpr (LPK <= 4) x += xor_lane<4>(x);
        if constexpr (LPK <= 8) x += xor_lane<8>(x);
        if constexpr (LPK <= 16) x += xor_lane<16>(x);
        x += xor_lane<32>(x);
        return x;
      };
#pragma unroll
      for (int j = 0; j < NREP; ++j) {
        lt[j] = gsum(l[j]);
#pragma unroll
        for (int i = 0; i < 8; ++i) t[j * 8 + i] = gsum(o[j][i]);
      }
    }
  }
  // visit (head, dim, total o, head total l, head max) for the outputs this lane owns
  template <typename F>
  QT_DEV void each(int lane, F&& f) const {
    const int sub = lane % LPK;
    if constexpr (TR) {
      const int rho = lane >> 4, jh = rho >> 1;
#pragma unroll
      for (int i = 0; i < 4; ++i) f(jh, sub * 8 + 4 * (rho & 1) + i, t[i], lt[0], mm[jh]);
    } else {
      if (lane / LPK != 0) return;
#pragma unroll
      for (int j = 0; j < NREP; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) f(j, sub * 8 + i, t[j * 8 + i], lt[j], mm[j]);
    }
  }
};

// two floats -> bf16 pair (low = a) by v_cvt_pk_bf16_f32 (round to nearest even; one instruction for f2bf's four)
QT_DEV unsigned pack2bf_rne(float a, float b) {
  typedef __attribute__((ext_vector_type(2))) float f32x2_t;
  const f32x2_t v = {a, b};
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2_t));
}
