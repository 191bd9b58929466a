// Device helpers shared by the conv engines (conv1d.hip, conv_ring.hip).
#pragma once
#include "common.h"

namespace {

template <bool FAST>
__device__ __forceinline__ float snake_f(float v, float al, float inv_al) {
  const float s = FAST ? __sinf(al * v) : sinf(al * v);
  return v + inv_al * (s * s);
}

// Branch-free loads through a buffer descriptor: out-of-range offsets (negative rows wrap to
// huge unsigned values) return 0 from the hardware range check, so every prefetch is issued
// unconditionally and hipcc keeps counted vmcnt waits (a per-lane `if (ok) load` makes it
// branch around each load and drain vmcnt(0): cdna_hip_programming.md §5 trap (c)).
typedef __amdgpu_buffer_rsrc_t Rsrc;
__device__ __forceinline__ Rsrc make_rsrc(const void* base, unsigned bytes) {
  const unsigned long long a = (unsigned long long)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  void* pb = (void*)(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(pb, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
constexpr unsigned OOB = 0x80000000u;  // an offset beyond every descriptor used here
__device__ __forceinline__ uint4 bload16(Rsrc r, unsigned off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  uint4 o;
  __builtin_memcpy(&o, &v, 16);
  return o;
}

// Branch-free store through a buffer descriptor: out-of-range offsets (OOB, or a descriptor of 0 bytes)
// are dropped by the range check, so a tile's stores are issued unconditionally and later counted vmcnt
// waits stay exact (a predicated `if (valid) store` makes the waitcnt pass assume the stores may be
// missing and over-wait: every load issued before them then waits for them too)
__device__ __forceinline__ void bstore16(Rsrc r, unsigned off, const uint4& v) {
  __attribute__((ext_vector_type(4))) unsigned w;
  __builtin_memcpy(&w, &v, 16);
  __builtin_amdgcn_raw_buffer_store_b128(w, r, (int)off, 0, 0);
}

template <typename T> struct RawT;
template <> struct RawT<bf16_t> { using type = uint4; };
struct F8 { float4 a, b; };
template <> struct RawT<float> { using type = F8; };
__device__ __forceinline__ uint4 load_raw(const bf16_t* p) { return *reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ F8 load_raw(const float* p) {
  return F8{*reinterpret_cast<const float4*>(p), *reinterpret_cast<const float4*>(p + 4)};
}
// 8 elements at element offset `e` (OOB when e is out of range of the descriptor)
__device__ __forceinline__ void bload_raw(Rsrc r, unsigned e, uint4& out, const bf16_t*) {
  out = bload16(r, e >= OOB / 2 ? OOB : e * 2u);
}
__device__ __forceinline__ void bload_raw(Rsrc r, unsigned e, F8& out, const float*) {
  const unsigned o = e >= OOB / 4 ? OOB : e * 4u;
  const uint4 a = bload16(r, o), b = bload16(r, o + 16u);
  __builtin_memcpy(&out.a, &a, 16);
  __builtin_memcpy(&out.b, &b, 16);
}
__device__ __forceinline__ void raw_to_f32(const uint4& r, float (&v)[8]) {
  bf16x8 b;
  __builtin_memcpy(&b, &r, 16);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (float)b[j];
}
__device__ __forceinline__ void raw_to_f32(const F8& r, float (&v)[8]) {
  v[0] = r.a.x; v[1] = r.a.y; v[2] = r.a.z; v[3] = r.a.w; v[4] = r.b.x; v[5] = r.b.y; v[6] = r.b.z; v[7] = r.b.w;
}
template <typename R>
__device__ __forceinline__ void raw16_to_f32(const R& r, float (&v)[16]) {
  float a[8], b[8];
  raw_to_f32(r.a, a);
  raw_to_f32(r.b, b);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    v[j] = a[j];
    v[8 + j] = b[j];
  }
}
__device__ __forceinline__ void ld8_lds(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

template <typename T>
__device__ __forceinline__ void load16(const T* p, float (&v)[16]) {
  float a[8], b[8];
  load8(p, a);
  load8(p + 8, b);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    v[j] = a[j];
    v[8 + j] = b[j];
  }
}

__device__ __forceinline__ void store16(float* p, const float (&v)[16]) {
#pragma unroll
  for (int j = 0; j < 16; j += 4) *reinterpret_cast<float4*>(p + j) = make_float4(v[j], v[j + 1], v[j + 2], v[j + 3]);
}
__device__ __forceinline__ void store16(bf16_t* p, const float (&v)[16]) {
  bf16x8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = (bf16_t)v[j];
    b[j] = (bf16_t)v[8 + j];
  }
  *reinterpret_cast<bf16x8*>(p) = a;
  *reinterpret_cast<bf16x8*>(p + 8) = b;
}


// LDS-DMA: 64 lanes x 16 B from a buffer descriptor straight into LDS at the wave-uniform
// address `lds` (lane i lands at lds + 16 i).  Out-of-range offsets read 0.
__device__ __forceinline__ void glds16(Rsrc r, void* lds, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}

// the same with a wave-uniform byte offset in the instruction's SGPR offset (soff), so the per-lane VGPR part can be
// shared by every piece a loop issues
__device__ __forceinline__ void glds16s(Rsrc r, void* lds, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, (int)soff, 0, 0);
}

}  // namespace
