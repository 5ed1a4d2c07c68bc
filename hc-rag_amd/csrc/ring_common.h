// ring_common.h — device helpers of the LDS-DMA ring kernels (score v2/v3/v4, encoder GEMM):
// buffer descriptors, LDS-DMA pieces, explicit vmcnt / barrier control, LDS accesses the
// compiler must not order behind in-flight LDS-DMA, and the 64-byte-row LDS swizzle.
#pragma once
#include "device_common.h"

namespace hcr {

__device__ __forceinline__ float4 lds_read_f4_now(const char* p) {
  float4 v;
  const uint32_t a = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ uint32_t lds_read_u32_now(const char* p) {
  uint32_t v;
  const uint32_t a = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, char* lds_dst, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds_dst, 16,
                                           voff, soff, 0, 0);
}
__device__ __forceinline__ void* uniform_ptr(const void* p) {
  const uint64_t v = (uint64_t)p;
  // readfirstlane returns a signed int: go through uint32_t so an address whose low word has
  // bit 31 set is not sign-extended into the high word
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  return (void*)(((uint64_t)hi << 32) | (uint64_t)lo);
}

constexpr int V3_BK = 32;                 // K per stage
constexpr int V3_NT = 512;                // 8 waves
constexpr uint32_t V3_SWZ = 0x1320;       // f(q) = (V3_SWZ >> 4q) & 15 = {0, 2, 3, 1}

__device__ __forceinline__ int v3_slot(int chunk, int row) {
  return chunk ^ (int)((V3_SWZ >> (((row >> 2) & 3) * 4)) & 3u);
}

// s_waitcnt vmcnt(n) for a wave-uniform n (the immediate must be a constant)
__device__ __forceinline__ void v3_wait_vmcnt(int n) {
  switch (n) {
#define HCR_VMW(i) \
  case i: asm volatile("s_waitcnt vmcnt(" #i ")" ::: "memory"); break;
    HCR_VMW(0) HCR_VMW(1) HCR_VMW(2) HCR_VMW(3) HCR_VMW(4) HCR_VMW(5) HCR_VMW(6) HCR_VMW(7)
    HCR_VMW(8) HCR_VMW(9) HCR_VMW(10) HCR_VMW(11) HCR_VMW(12) HCR_VMW(13) HCR_VMW(14)
    HCR_VMW(15) HCR_VMW(16) HCR_VMW(17) HCR_VMW(18) HCR_VMW(19) HCR_VMW(20) HCR_VMW(21)
    HCR_VMW(22) HCR_VMW(23) HCR_VMW(24) HCR_VMW(25) HCR_VMW(26) HCR_VMW(27) HCR_VMW(28)
    HCR_VMW(29) HCR_VMW(30) HCR_VMW(31) HCR_VMW(32) HCR_VMW(33) HCR_VMW(34) HCR_VMW(35)
    HCR_VMW(36) HCR_VMW(37) HCR_VMW(38) HCR_VMW(39) HCR_VMW(40)
#undef HCR_VMW
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// Workgroup barrier WITHOUT the release fence of __syncthreads() (which makes the compiler
// drain vmcnt, i.e. every LDS-DMA stage in flight): LDS operations are drained here, global
// ones are the caller's business (per-wave vmcnt waits on the ring; full __syncthreads() where
// global stores of other waves are read).  One asm statement, so nothing moves across it.
__device__ __forceinline__ void v3_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// LDS helpers that the compiler cannot see as LDS accesses: it would otherwise order them
// behind every LDS-DMA write in flight (s_waitcnt vmcnt(0), draining the ring).
__device__ __forceinline__ uint32_t v3_lds_u32(const void* p) {
  uint32_t v;
  const uint32_t a = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ uint64_t v3_lds_u64(const void* p) {
  uint64_t v;
  const uint32_t a = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
  asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ int v3_lds_add_rtn(void* p, int x) {
  int v;
  const uint32_t a = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)p);
  asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=&v"(v) : "v"(a), "v"(x) : "memory");
  return v;
}
__device__ __forceinline__ void v3_lds_store_u32(void* p, uint32_t x) {
  const uint32_t a = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)p);
  asm volatile("ds_write_b32 %0, %1" : : "v"(a), "v"(x) : "memory");
}
__device__ __forceinline__ void v3_lds_store_u64(void* p, uint64_t x) {
  const uint32_t a = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)p);
  asm volatile("ds_write_b64 %0, %1" : : "v"(a), "v"(x) : "memory");
}

// the 12 MFMA fragments of a stage (8 row blocks at a, 4 query blocks at b, 1 KiB apart), one
// wait.  Inline asm: a compiler-visible LDS read after the loop's LDS-DMA would get a
// vmcnt(0) in front of it, draining the ring.
template <typename V>
__device__ __forceinline__ void v4_read_frags(uint32_t a, uint32_t b, V (&av)[8], V (&bq)[4]) {
  asm volatile(
      "ds_read_b128 %0, %12\n\t"
      "ds_read_b128 %1, %12 offset:1024\n\t"
      "ds_read_b128 %2, %12 offset:2048\n\t"
      "ds_read_b128 %3, %12 offset:3072\n\t"
      "ds_read_b128 %4, %12 offset:4096\n\t"
      "ds_read_b128 %5, %12 offset:5120\n\t"
      "ds_read_b128 %6, %12 offset:6144\n\t"
      "ds_read_b128 %7, %12 offset:7168\n\t"
      "ds_read_b128 %8, %13\n\t"
      "ds_read_b128 %9, %13 offset:1024\n\t"
      "ds_read_b128 %10, %13 offset:2048\n\t"
      "ds_read_b128 %11, %13 offset:3072\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(av[0]), "=&v"(av[1]), "=&v"(av[2]), "=&v"(av[3]), "=&v"(av[4]), "=&v"(av[5]),
        "=&v"(av[6]), "=&v"(av[7]), "=&v"(bq[0]), "=&v"(bq[1]), "=&v"(bq[2]), "=&v"(bq[3])
      : "v"(a), "v"(b)
      : "memory");
}

// Split form of v4_read_frags: issue the 4 query fragments, then the 8 row fragments, with no
// wait; v4_frag_wait<N>(x, y) then waits until at most N of them are outstanding (LDS reads
// complete in order) and re-defines x, y so no use of them is scheduled above the wait.
template <typename V>
__device__ __forceinline__ void v4_issue_frags(uint32_t a, uint32_t b, V (&av)[8], V (&bq)[4]) {
  asm volatile(
      "ds_read_b128 %8, %13\n\t"
      "ds_read_b128 %9, %13 offset:1024\n\t"
      "ds_read_b128 %10, %13 offset:2048\n\t"
      "ds_read_b128 %11, %13 offset:3072\n\t"
      "ds_read_b128 %0, %12\n\t"
      "ds_read_b128 %1, %12 offset:1024\n\t"
      "ds_read_b128 %2, %12 offset:2048\n\t"
      "ds_read_b128 %3, %12 offset:3072\n\t"
      "ds_read_b128 %4, %12 offset:4096\n\t"
      "ds_read_b128 %5, %12 offset:5120\n\t"
      "ds_read_b128 %6, %12 offset:6144\n\t"
      "ds_read_b128 %7, %12 offset:7168"
      : "=&v"(av[0]), "=&v"(av[1]), "=&v"(av[2]), "=&v"(av[3]), "=&v"(av[4]), "=&v"(av[5]),
        "=&v"(av[6]), "=&v"(av[7]), "=&v"(bq[0]), "=&v"(bq[1]), "=&v"(bq[2]), "=&v"(bq[3])
      : "v"(a), "v"(b)
      : "memory");
}
template <int N, typename V>
__device__ __forceinline__ void v4_frag_wait(V& x, V& y) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(x), "+v"(y) : "n"(N) : "memory");
}
template <int N, typename V>
__device__ __forceinline__ void v4_frag_wait6(V& x, V& y, V (&bq)[4]) {
  asm volatile("s_waitcnt lgkmcnt(%6)"
               : "+v"(x), "+v"(y), "+v"(bq[0]), "+v"(bq[1]), "+v"(bq[2]), "+v"(bq[3])
               : "n"(N) : "memory");
}

// 6 row-block fragments + 4 query/token fragments (gemm_v4 at 192-feature tiles), one wait
template <typename V>
__device__ __forceinline__ void v4_read_frags6(uint32_t a, uint32_t b, V (&av)[6], V (&bq)[4]) {
  asm volatile(
      "ds_read_b128 %0, %10\n\t"
      "ds_read_b128 %1, %10 offset:1024\n\t"
      "ds_read_b128 %2, %10 offset:2048\n\t"
      "ds_read_b128 %3, %10 offset:3072\n\t"
      "ds_read_b128 %4, %10 offset:4096\n\t"
      "ds_read_b128 %5, %10 offset:5120\n\t"
      "ds_read_b128 %6, %11\n\t"
      "ds_read_b128 %7, %11 offset:1024\n\t"
      "ds_read_b128 %8, %11 offset:2048\n\t"
      "ds_read_b128 %9, %11 offset:3072\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(av[0]), "=&v"(av[1]), "=&v"(av[2]), "=&v"(av[3]), "=&v"(av[4]), "=&v"(av[5]),
        "=&v"(bq[0]), "=&v"(bq[1]), "=&v"(bq[2]), "=&v"(bq[3])
      : "v"(a), "v"(b)
      : "memory");
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}

}  // namespace hcr
