// Logits processing + token selection (transformers 4.57 semantics), one 256-thread block per row.
// Each thread keeps its V/256 (<= 16) scores in registers (strided, coalesced loads).
// Greedy: argmax with lowest-index tie break (torch.argmax).
// Sampling: Temperature -> TopK -> TopP -> softmax -> draw from a Philox-4x32-10 stream keyed by
// (seed, step, substep, row).  k <= 64 without top-p (the generate() defaults, k = 50): per-wave candidate lists and
// a Gumbel-max draw in one wave (see sample_k).  Otherwise: top-k threshold = exact k-th largest score, found by building its
// order-preserving 32-bit key MSB-first (<= 16 block-wide 2-bit steps, no sort); ties at the threshold are kept
// like TopKLogitsWarper.  The draw is an inverse CDF over a fixed category order (parallel prefix of
// per-thread masses), so it is an exact sample of the warped distribution; RNG streams differ from
// torch.multinomial, hence parity is distribution-level (tests/test_gpu_parity.py).
#include "common.h"
#include "sample_dev.h"
#include <cstdlib>

namespace {

using namespace qt_sample_dev;

struct SK {
  qt_sample_args a;
  int stop;  // measurement hook (QT_SAMPLE_STOP): end after phase 1..5; 0 = the full kernel
};

template <int PER>
__global__ __launch_bounds__(NT) void sample_k(SK pk) {
  __shared__ SampSh S;
  sample_row<PER>(pk.a, pk.stop, blockIdx.x, threadIdx.x, S, []() { __syncthreads(); });
}

}  // namespace

extern "C" int qt_sample(const qt_sample_args* a, void* stream) {
  if (!a || a->R <= 0 || a->V <= 0 || a->V > NT * 16 || !a->tok_out) return QT_ERR_SHAPE;
  if (a->do_sample && a->top_k > a->V) return QT_ERR_ARG;
  if (a->ctr_stride < 0) return QT_ERR_SHAPE;
  if (a->emb_table && (!a->emb_out || a->emb_dim % 4 || a->emb_ld % 4)) return QT_ERR_SHAPE;
  if (a->emb_out16 && (!a->emb_table || a->emb_ld16 % 4)) return QT_ERR_SHAPE;
  if (a->emb2_table && (!a->emb_table || !a->emb2_out || a->emb2_dim % 4 || a->emb2_ld % 4)) return QT_ERR_SHAPE;
  if (a->force && (!a->pick || !a->codes)) return QT_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  static const int stop = qt_knob("QT_SAMPLE_STOP", 0);
  const SK k{*a, stop};
  if (a->V <= NT * 8) hipLaunchKernelGGL(sample_k<8>, dim3(a->R), dim3(NT), 0, st, k);
  else if (a->V <= NT * 12) hipLaunchKernelGGL(sample_k<12>, dim3(a->R), dim3(NT), 0, st, k);
  else hipLaunchKernelGGL(sample_k<16>, dim3(a->R), dim3(NT), 0, st, k);
  return hipGetLastError() == hipSuccess ? 0 : QT_ERR_LAUNCH;
}
