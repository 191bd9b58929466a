// Device helpers shared by the LDS-DMA conv engines (bigconv2.hip, bigconv3.hip): counted vmcnt waits, the raw
// workgroup barrier that keeps LDS-DMAs in flight, LDS accesses the compiler cannot see (so it does not drain the
// in-flight DMAs before them), bf16 packing.
#pragma once
#include "common.h"

namespace {

// prologue kinds: AdaIN -> Snake (the generator resblocks, 5 coefficients per channel), or
// [AdaIN ->] LReLU (the decoder front-end's AdainResBlk1d convs, hifigan.py:359-403; 2 per
// channel; no prologue = a = 1, m = 0, slope 1)
enum { PK_SNAKE = 0, PK_LRELU = 1 };

template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void barrier_lds() {
  // publish this wave's LDS writes, then a raw barrier: LDS-DMAs stay in flight across it
  // (a __syncthreads() would drain vmcnt to 0)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// LDS byte address of a pointer into the kernel's dynamic LDS
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
// the five 16-byte coefficient vectors of 4 channels (rows stride_b bytes apart), read and waited
// for in ONE asm statement: hipcc otherwise drains every in-flight LDS-DMA (vmcnt(0)) before these
// reads, which are disjoint from every DMA destination
typedef float f32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void lds_coef5(unsigned a, f32x4v& c0, f32x4v& c1, f32x4v& c2, f32x4v& c3, f32x4v& c4,
                                          unsigned stride) {
  const unsigned a1 = a + stride, a2 = a + 2 * stride, a3 = a + 3 * stride, a4 = a + 4 * stride;
  asm volatile(
      "ds_read_b128 %0, %5\n\t"
      "ds_read_b128 %1, %6\n\t"
      "ds_read_b128 %2, %7\n\t"
      "ds_read_b128 %3, %8\n\t"
      "ds_read_b128 %4, %9\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(c0), "=&v"(c1), "=&v"(c2), "=&v"(c3), "=&v"(c4)
      : "v"(a), "v"(a1), "v"(a2), "v"(a3), "v"(a4)
      : "memory");
}

__device__ __forceinline__ void lds_coef2(unsigned a, f32x4v& c0, f32x4v& c1, unsigned stride) {
  const unsigned a1 = a + stride;
  asm volatile(
      "ds_read_b128 %0, %2\n\t"
      "ds_read_b128 %1, %3\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(c0), "=&v"(c1)
      : "v"(a), "v"(a1)
      : "memory");
}

// an LDS store hipcc cannot see: it drains every in-flight LDS-DMA (vmcnt(0)) before a visible
// ds_write, although the window units written here are never a pending DMA's destination (their
// own DMA was waited for by vm_wait)
__device__ __forceinline__ void lds_write_b64(unsigned a, const uint2& v) {
  asm volatile("ds_write_b64 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_write_b128(unsigned a, const uint4& v) {
  typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
  const u32x4v w = {v.x, v.y, v.z, v.w};
  asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(w) : "memory");
}

__device__ __forceinline__ void bf4_to_f32(const uint2& r, float (&v)[4]) {
  v[0] = __uint_as_float(r.x << 16);
  v[1] = __uint_as_float(r.x & 0xffff0000u);
  v[2] = __uint_as_float(r.y << 16);
  v[3] = __uint_as_float(r.y & 0xffff0000u);
}
__device__ __forceinline__ uint2 f32_to_bf4(const float (&v)[4]) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  bf16x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = (bf16_t)v[j];
  uint2 r;
  __builtin_memcpy(&r, &o, 8);
  return r;
}
__device__ __forceinline__ void bf8_to_f32v(const uint4& r, float* v) {
  const unsigned w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 f32_to_bf8v(const float* v) {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (bf16_t)v[j];
  uint4 r;
  __builtin_memcpy(&r, &o, 16);
  return r;
}

}  // namespace
