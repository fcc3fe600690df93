// Internal to the GEMM sources (gemm.hip, gemm_pf2.hip): the kernel parameter block built by qt_gemm from
// qt_gemm_args, and the prefill GEMM launcher that lives in its own translation unit.
#pragma once
#include "common.h"

namespace qt_gemm_impl {

struct GemmP {
  int M, N, Kp, Klog;          // Kp = padded K (taps * cin_pad), Klog = RMSNorm length
  const void* A; long long lda;
  const int* a_index;
  const void* W;
  const float* gamma; float eps; int rms;
  const float* bias; const float* colscale;
  int act, epi;
  void* out; long long ldo;
  int taps, dil, cin, cin_pad, t_in, t_out, t_off;
  int ks;                       // split-K factor (gridDim.y), 1 = none
  int wpb_max;                  // waves-per-block cap of the decode GEMV (16, or 8 for wide grids)
  int no_igemm;                 // 1: keep large-M GEMMs on gemm_wt (A/B measurement)
  int ntl;                      // 1: non-temporal weight loads (decode GEMV over >= 16 MiB of weights)
  unsigned* cnt; float* part;   // split-K arrival counters [ntiles] + partials [ntiles][ks][64*4+16] (GEMV) /
  long long part_bytes;         //   gemm_pf2_k split records (17+ rows), part_bytes of room
  const float* sn_a; const float* sn_ib;  // optional SnakeBeta on A (per input channel)
  int a_elu;                    // ELU on A (tokenizer encoder convs)
  int mr;                       // decode GEMV rows per row group (gridDim.z = ceil(M / mr))
  bf16_t* out2; long long ldo2; // optional bf16 copy of the stored output (decode residual stream shadow)
  int sk;                       // 1: skinny GEMM (gemm_sk_k, 17..64 rows, every row in one block)
  int pf_small;                 // 1: gemm_pf2_k below its default row floor (17..256-row routing in qt_gemm)
};

// gemm_pf2_k (gemm_pf2.hip): prefill linears with bf16 A and bf16 pre-tiled W, K % 64 == 0, 16-byte aligned A
void launch_pf2_auto_f32(const GemmP& p, hipStream_t s);
void launch_pf2_auto_bf16(const GemmP& p, hipStream_t s);
// gemm_sk_k (gemm_sk.hip): 17..64 rows, bf16 A and bf16 pre-tiled W, K % 32 == 0, 16-byte aligned A rows
void launch_sk_f32(const GemmP& p, hipStream_t s);
void launch_sk_bf16(const GemmP& p, hipStream_t s);

}  // namespace qt_gemm_impl
