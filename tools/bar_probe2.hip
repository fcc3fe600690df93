// Grid-synchronisation probe for a persistent code-predictor kernel (256 workgroups x 512 threads, one per CU):
// what does one all-to-all edge cost on MI355X?  Each phase: every block publishes a 64 B slice of a vector (sc1
// write-through stores), signals, waits for all 256 signals, then reads the whole 16 KiB vector (sc1 loads).
//   B1 xcd-tree : per-group counters (group = block % 8, 32 blocks each, agent-scope atomics), the last arriver of a
//                 group bumps the top counter, everyone polls the top counter (sc1 load + s_sleep)
//   B2 flags    : every block stores its epoch flag (sc1), one wave per block polls all 256 flags (one 1 KiB sc1 load)
//   B3 tagged   : no separate signal -- the 16 KiB vector is written as {value, epoch} 8-byte granules and every
//                 block polls the data itself until all 2048 granules carry the epoch
// Every spin is bounded (error flag, no hang).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bar_probe2.hip -o tools/bar_probe2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2_t;

__device__ __forceinline__ unsigned ld_sc1(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_sc1_64(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_64(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int NB = 256, VEC = 4096;  // 4096 fp32 values = 16 KiB vector, 16 per block
constexpr unsigned SPIN_MAX = 1u << 20;

template <int MODE>
__global__ __launch_bounds__(512) void k(unsigned* ctr, unsigned* flags, float* vec, unsigned long long* gran,
                                         int phases, float* sink, unsigned* err) {
  __shared__ unsigned s_ok;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  float acc = 0.f;
  for (int ph = 1; ph <= phases; ++ph) {
    // a timed-out wait anywhere ends every block at its next phase (block-uniform decision, no hang)
    if (tid == 0) s_ok = ld_sc1(err);
    __syncthreads();
    if (s_ok) return;
    __syncthreads();
    // publish this block's 16 values (wave 0, lanes 0..15)
    const float val = (float)(b * 16 + lane) + ph;
    if (MODE != 3) {
      if (w == 0 && lane < 16) st_sc1((unsigned*)vec + b * 16 + lane, __float_as_uint(val));
      __builtin_amdgcn_s_waitcnt(0);  // every storing wave drained before the signal
      __syncthreads();
    }
    if (MODE == 1) {
      if (tid == 0) {
        const int g = b & 7;
        const unsigned old = __hip_atomic_fetch_add(ctr + 64 * (1 + g), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old + 1 == (unsigned)ph * (NB / 8)) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned spins = 0;
        while (ld_sc1(ctr) < (unsigned)ph * 8) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > SPIN_MAX) { atomicOr(err, 1u); break; }
        }
      }
      __syncthreads();
    } else if (MODE == 2) {
      if (tid == 0) st_sc1(flags + b, (unsigned)ph);
      if (w == 0) {
        unsigned spins = 0;
        while (true) {
          unsigned f0 = ld_sc1(flags + lane * 4), f1 = ld_sc1(flags + lane * 4 + 1), f2 = ld_sc1(flags + lane * 4 + 2),
                   f3 = ld_sc1(flags + lane * 4 + 3);
          const bool mine = f0 >= (unsigned)ph && f1 >= (unsigned)ph && f2 >= (unsigned)ph && f3 >= (unsigned)ph;
          if (__all(mine)) break;
          __builtin_amdgcn_s_sleep(1);
          if (++spins > SPIN_MAX) { if (lane == 0) atomicOr(err, 2u); break; }
        }
      }
      __syncthreads();
    } else if (MODE == 3) {
      // tagged granules: value + epoch in one 8-byte sc1 store
      if (w == 0 && lane < 16)
        st_sc1_64(gran + b * 16 + lane, ((unsigned long long)ph << 32) | __float_as_uint(val));
    }
    // read the whole vector (all 512 threads, 8 values each)
    if (MODE == 3) {
      unsigned spins = 0;
      float s = 0.f;
      for (int i = tid; i < VEC; i += 512) {
        unsigned long long g;
        while (true) {
          g = ld_sc1_64(gran + i);
          if ((unsigned)(g >> 32) >= (unsigned)ph) break;
          __builtin_amdgcn_s_sleep(1);
          if (++spins > SPIN_MAX) { atomicOr(err, 4u); break; }
        }
        s += __uint_as_float((unsigned)g);
      }
      acc += s;
      __syncthreads();
    } else {
      float s = 0.f;
      for (int i = tid; i < VEC; i += 512) s += __uint_as_float(ld_sc1((const unsigned*)vec + i));
      acc += s;
      __syncthreads();  // everyone has read before the next phase overwrites
    }
  }
  if (acc == 1234.5f) sink[0] = acc;
}

int main() {
  unsigned *ctr, *flags, *err;
  float *vec, *sink;
  unsigned long long* gran;
  CK(hipMalloc(&ctr, 64 * 4 * 16)); CK(hipMalloc(&flags, NB * 4)); CK(hipMalloc(&err, 4));
  CK(hipMalloc(&vec, VEC * 4)); CK(hipMalloc(&sink, 4)); CK(hipMalloc(&gran, VEC * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto reset = [&] {
    CK(hipMemset(ctr, 0, 64 * 4 * 16)); CK(hipMemset(flags, 0, NB * 4)); CK(hipMemset(err, 0, 4));
    CK(hipMemset(gran, 0, VEC * 8));
  };
  for (int mode = 1; mode <= 3; ++mode) {
    for (int phases : {10, 1000}) {
      reset();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(NB), dim3(512), 0, 0, ctr, flags, vec, gran, phases, sink, err);
      if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(NB), dim3(512), 0, 0, ctr, flags, vec, gran, phases, sink, err);
      if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(NB), dim3(512), 0, 0, ctr, flags, vec, gran, phases, sink, err);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned he; CK(hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost));
      printf("mode %d (%s) phases %5d: %8.3f us total, %6.3f us per phase, err %u\n", mode,
             mode == 1 ? "xcd-tree" : mode == 2 ? "flags" : "tagged", phases, ms * 1e3, ms * 1e3 / phases, he);
      fflush(stdout);
    }
  }
  // reference: one kernel per phase (same publish + read, graph-captured chain of dependent launches)
  {
    const int n = 1000;
    hipStream_t st; CK(hipStreamCreate(&st));
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k<0>, dim3(NB), dim3(512), 0, st, ctr, flags, vec, gran, 1, sink, err);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st)); CK(hipStreamSynchronize(st));
    CK(hipEventRecord(e0, st));
    CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("mode 0 (kernel per phase, graph) phases %5d: %8.3f us total, %6.3f us per phase\n", n, ms * 1e3, ms * 1e3 / n);
  }
  printf("done\n");
  return 0;
}
