// Device helpers shared by the persistent engines (cp_engine.hip, talker_tail.hip): buffer-resource memory
// primitives, the agent-scope flag / granule hand-off stores and loads, MFMA and fragment addressing, LDS-DMA.
#pragma once
#include "common.h"

namespace qt_engine {

typedef unsigned long long u64;
typedef __amdgpu_buffer_rsrc_t rsrc_t;

// ---- memory primitives
QT_DEV rsrc_t mkr(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
constexpr int SC1 = 16;  // buffer-instruction cache policy: sc1 (agent-coherent, write-through)
QT_DEV u32x4_t bld(rsrc_t r, unsigned off) { return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0); }
QT_DEV u32x4_t bld_c(rsrc_t r, unsigned off) { return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, SC1); }
QT_DEV uint2 bld2_c(rsrc_t r, unsigned off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, SC1);
  return uint2{v[0], v[1]};
}
QT_DEV void bst_c(unsigned v, rsrc_t r, unsigned off) { __builtin_amdgcn_raw_buffer_store_b32(v, r, (int)off, 0, SC1); }
QT_DEV void bst4_c(u32x4_t v, rsrc_t r, unsigned off) { __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, SC1); }
QT_DEV void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
QT_DEV unsigned ld_flag(const unsigned* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
QT_DEV void st_flag(unsigned* p, unsigned v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
QT_DEV u64 ld_g(const u64* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
QT_DEV void st_g(u64* p, unsigned v, unsigned tag) {
  __hip_atomic_store(p, ((u64)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
QT_DEV f32x4_t mfma(u32x4_t a, u32x4_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c, 0,
                                                 0, 0);
}
// byte offset of lane `lane`'s 16 bytes of weight fragment (n tile, k tile) of a pre-tiled bf16 matrix with kt k tiles
QT_DEV unsigned fragoff(int nt, int ktile, int kt, int lane) { return ((unsigned)(nt * kt + ktile) << 10) + lane * 16; }
// keep issued loads where they are (not sunk to their first use)
#define CE_ISSUED() asm volatile("" ::: "memory")
// LDS-DMA (global_load_lds_dwordx4, no VGPR staging): lane l's 16 bytes land at lds + 16 l; hipcc does not count it,
// the issuing wave waits with its own s_waitcnt vmcnt before reading (vmcnt is in order, so every compiler wait on a
// later load also covers it)
QT_DEV void glds16(const void* g, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}
QT_DEV unsigned lds_u32(const void* p) {
  return __builtin_amdgcn_readfirstlane((unsigned)(size_t)(const __attribute__((address_space(3))) void*)p);
}
QT_DEV void vm_wait0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// the phase's MFMAs are issued before the next phase's weight loads (so the two weight sets are never live together)
// all four A fragments read (one LDS wait) before the first MFMA, instead of a wait per MFMA
QT_DEV void pin4(u32x4_t* a) { asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3])); }
#define CE_AFTER(acc) asm volatile("" : "+v"(acc)::"memory")


// ---- weight-ring engines (talker_tail.hip): loader waves, LDS-DMA with the non-temporal policy, consumer barrier
QT_DEV void glds16_nt(const void* g, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}
QT_DEV unsigned lds_ld(const unsigned* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
QT_DEV void lds_st(unsigned* p, unsigned v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }

// The consumer waves synchronise among themselves only: the loader waves run free, so a block-wide s_barrier cannot
// be used once they have split off.  The consumers meet through an LDS arrival counter instead (generation-counted,
// bounded spin: a give-up sets error bit 8).

struct CBar {
  unsigned* cnt;  // LDS: arrivals
  unsigned* gen;  // LDS: generation
};
template <int NWC>
QT_DEV void cons_sync(const CBar& cb, unsigned& g, int spin, int* err) {
  // every consumer wave's LDS writes before the barrier are visible after it: the wave's own LDS operations complete
  // (lgkmcnt(0)) before its arrival, an LDS atomic
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const int lane = threadIdx.x & 63;
  ++g;
  if (lane == 0) {
    const unsigned a = __hip_atomic_fetch_add(cb.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (a == g * NWC - 1) lds_st(cb.gen, g);
  }
  for (int spins = 0; __builtin_amdgcn_readfirstlane(lds_ld(cb.gen)) < g; ++spins) {
    if (spins > 64 * spin) { if (lane == 0) atomicOr(err, 8); break; }
    __builtin_amdgcn_s_sleep(0);
  }
}

}  // namespace qt_engine
