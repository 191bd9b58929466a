// Shared definitions for the StyleTTS2-lite MI355X (gfx950) synthesis kernels.
// Activations are time-major "frames" tensors: [B][L][ld] (channel fastest), so a
// convolution is an implicit GEMM whose K dimension (input channels) is contiguous —
// the layout the 64-lane MFMA operand maps want.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <map>
#include <mutex>
#include <tuple>

typedef __bf16 bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ST_SPLIT (accuracy mode): fp32 storage, every conv's operands split into bf16 hi + lo parts and
// multiplied as hi*hi + hi*lo + lo*hi on the bf16 MFMA (fp32 accumulation)
enum StDtype { ST_FP32 = 0, ST_BF16 = 1, ST_SPLIT = 2 };
constexpr int ST_NDTYPES = 3;
// internal (not a C-ABI dtype): bf16 MFMA operands staged from fp32 frames, fp32 outputs (the training
// step's convs on the general engine: no frames conversion passes around them)
constexpr int ST_BF16F = 3;

// hipOccupancyMaxActiveBlocksPerMultiprocessor per (kernel, block size, dynamic LDS), queried once per process
// (a host-side query on every launch otherwise: the training step makes ~5,000 launches a step); 0 on error
inline int occupancy_cached(const void* kern, int nt, size_t lds) {
  static std::mutex mu;
  static std::map<std::tuple<const void*, int, size_t>, int> cache;
  std::lock_guard<std::mutex> lk(mu);
  const auto key = std::make_tuple(kern, nt, lds);
  const auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, nt, lds) != hipSuccess) return 0;
  cache[key] = per_cu;
  return per_cu;
}

// domain error codes (negative; positive values are hipError_t)
enum StStatus {
  ST_OK = 0,
  ST_EINVAL = -1,      // bad argument / shape
  ST_EDTYPE = -2,      // unsupported dtype
  ST_EPARAMS = -3,     // parameter table incomplete / mismatched
  ST_EWORKSPACE = -4,  // workspace too small
  ST_ENOTPACKED = -5,  // forward before pack
};

#define ST_CHECK_HIP(expr)                                   \
  do {                                                       \
    hipError_t _e = (expr);                                  \
    if (_e != hipSuccess) return (int)_e;                    \
  } while (0)

#define ST_CHECK(expr)                                       \
  do {                                                       \
    int _r = (expr);                                         \
    if (_r != 0) return _r;                                  \
  } while (0)

__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(bf16_t v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16_t from_f32<bf16_t>(float v) { return (bf16_t)v; }

// Load 8 consecutive elements (16-byte aligned for bf16, 32-byte for fp32) as floats.
__device__ __forceinline__ void load8(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void load8(const bf16_t* p, float (&v)[8]) {
  const bf16x8 a = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (float)a[j];
}

// XCD-aware bijective block remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): consecutive logical tiles land on the same XCD (shared L2).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, k = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

// Prologue applied to every conv input element while it is staged into LDS:
//   AdaIN  : v = (x - mean) * a + beta,  a = (1 + gamma) * rstd   (reference hifigan.py:14-24)
//   Snake  : v = v + (1/alpha) * sin(alpha * v)^2                  (hifigan.py:68, 329)
//   LReLU  : v = v > 0 ? v : slope * v
enum ProMode { PRO_AFFINE = 1, PRO_SNAKE = 2, PRO_LRELU = 4 };

struct Prologue {
  int mode;              // bitmask of ProMode
  const double* stats;   // [B][stats_ld][ST_W] fixed-point (sum, sumsq) of the input, per (utterance, channel)
  int stats_ld;
  double inv_n;          // 1 / (time length) of the normalised tensor
  const float* gamma;    // AdaIN fc output: gamma = h[b][gb_off + c], beta = h[b][gb_off + C + c]
  int gb_ld;             // row stride of h (per utterance)
  int gb_C;              // C (offset of beta from gamma)
  const float* alpha;    // [C] snake alpha
  float slope;           // leaky-relu slope
  // the producer spread its statistics over `stats_slots` copies stats_slot_bs doubles apart
  // (small batches, ConvParams::stats_slots): the consumer sums them here, so no fold launch
  int stats_slots;
  long long stats_slot_bs;
};

// Deterministic InstanceNorm statistics (round 5).  The producers' partial sums reach the
// (utterance, channel) totals through device atomics from many workgroups in no fixed order; in fp64 those adds
// round, so repeat runs differed in the last bits.  Each total is now a fixed-point integer instead: a partial v is
// scaled by 2^48 and split into hi = floor(v 2^16) and lo = (v 2^48 - hi 2^32) in [0, 2^32), added with integer
// atomics (exact, so any order gives the same total), and read back as hi 2^-16 + lo 2^-48 (one rounding, the same
// every run).  Range |partial|, |sum| < 2^45, resolution 2^-48 per addend.  An entry is ST_W = 4 words: (hi, lo) of sum x, then
// of sum x^2.  A non-finite or out-of-range partial sets bit 63 of the lo word (ST_POISON, an atomic OR: idempotent,
// and the lo sums, < 2^32 per addend, never carry into it), read back as NaN.
constexpr int ST_W = 4;
constexpr unsigned long long ST_POISON = 0x8000000000000000ull;
__device__ __forceinline__ void fx_add(double* w, double v) {
  unsigned long long* u = reinterpret_cast<unsigned long long*>(w);
  if (!(v >= -0x1p45 && v <= 0x1p45)) {  // NaN, inf or out of range
    atomicOr(u + 1, ST_POISON);
    return;
  }
  const double q = v * 0x1p48;
  const double h = floor(q * 0x1p-32);
  const long long hi = (long long)h;
  const long long lo = (long long)floor(q - h * 0x1p32);
  atomicAdd(u, (unsigned long long)hi);
  atomicAdd(u + 1, (unsigned long long)lo);
}
// (the same for an fp32 partial, from its bits with integer shifts: no fp64 arithmetic in the MFMA engines'
// epilogues, where registers are scarce; truncation toward zero below 2^-48)
__device__ __forceinline__ void fx_add(double* w, float v) {
  unsigned long long* u = reinterpret_cast<unsigned long long*>(w);
  const unsigned bits = __float_as_uint(v);
  const int e = (int)((bits >> 23) & 255u);
  if (e >= 127 + 45) {  // NaN, inf or |v| >= 2^45
    atomicOr(u + 1, ST_POISON);
    return;
  }
  if (e == 0) return;  // zero (or a denormal, below the resolution)
  const unsigned long long m = (bits & 0x7fffffu) | 0x800000u;
  const int s = e - 127 - 23 + 48;  // v 2^48 = m 2^s, s <= 69
  unsigned long long hi, lo;
  if (s <= 0) {
    hi = 0;
    lo = s > -24 ? m >> -s : 0;
  } else if (s < 32) {
    const unsigned long long x = m << s;  // < 2^56
    hi = x >> 32;
    lo = x & 0xffffffffull;
  } else {
    hi = m << (s - 32);
    lo = 0;
  }
  if (bits >> 31) {  // -(hi 2^32 + lo) as (hi', lo') with lo' in [0, 2^32)
    hi = 0ull - hi - (lo != 0 ? 1ull : 0ull);
    lo = lo != 0 ? (1ull << 32) - lo : 0ull;
  }
  if (hi) atomicAdd(u, hi);
  if (lo) atomicAdd(u + 1, lo);
}
// Read back.  A total outside the range (|sum| >= 2^45: hi beyond +-2^61) reads as NaN too, like a poisoned entry: the
// int64 hi word only wraps once |sum| passes 2^47, so a total that grew past the range through many in-range partials
// reads as NaN, not as a wrong mean / variance (unless it ran past 2^47 and wrapped back into range: true |sum| within
// 2^45 of a non-zero multiple of 2^48, beyond 7 x 10^13)
__device__ __forceinline__ double fx_get(const double* w) {
  const long long* u = reinterpret_cast<const long long*>(w);
  const long long hi = u[0];
  const long long lo = u[1];
  if (lo < 0) return __builtin_nan("");  // poisoned (ST_POISON)
  if (hi >= (1ll << 61) || hi < -(1ll << 61)) return __builtin_nan("");  // out of range
  return (double)hi * 0x1p-16 + (double)lo * 0x1p-48;
}
// add the partial sums a = sum x, q = sum x^2 into the entry e (ST_W words)
__device__ __forceinline__ void stat_add(double* e, double a, double q) {
  fx_add(e, a);
  fx_add(e + 2, q);
}

// Reduce-scatter of a 32-lane half-wave's 16 per-lane partials v[r] (channels r = 0..15): 8 + 4 + 2 + 1
// exchanges leave lane l32 with channel l32 / 2 summed over 16 lanes, one exchange with lane l32 ^ 1 completes
// it (32 exchanges instead of the 80 of 16 butterflies).  v is clobbered.
__device__ __forceinline__ float rs16(float (&v)[16], int l32) {
#pragma unroll
  for (int m = 16, n = 16; m >= 2; m >>= 1, n >>= 1) {
    const bool up = (l32 & m) != 0;
#pragma unroll
    for (int i = 0; i < n / 2; ++i) {
      const float send = up ? v[i] : v[i + n / 2];
      const float keep = up ? v[i + n / 2] : v[i];
      v[i] = keep + __shfl_xor(send, m);
    }
  }
  return v[0] + __shfl_xor(v[0], 1);
}
// A half-wave's 16 channels' partial (sum, sumsq) -> lane r < 16 of the half holds channel r's totals in (a, q),
// the partials are zeroed: butterflies per channel (2 live values; the reduce-scatter above needs more registers
// than the 256-VGPR engines have left in their epilogues), the lanes then add 16 entries at once instead of lane 0
// adding all 16 in turn.
__device__ __forceinline__ void stat_bfly16(float (&s)[16], float (&q)[16], int l32, float& a, float& b) {
  a = b = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float x = s[r], y = q[r];
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) {
      x += __shfl_xor(x, o);
      y += __shfl_xor(y, o);
    }
    if (l32 == r) {
      a = x;
      b = y;
    }
    s[r] = q[r] = 0.f;
  }
}

// Per-(utterance, channel) AdaIN coefficients from raw stats: mean, a = (1+gamma)*rstd, beta.
__device__ __forceinline__ void adain_coeffs(const Prologue& p, int b, int c, float& m, float& a, float& be) {
  const size_t i = ((size_t)b * p.stats_ld + c) * ST_W;
  double s = fx_get(p.stats + i), ss = fx_get(p.stats + i + 2);
  for (int k = 1; k < p.stats_slots; ++k) {  // (slot order: fixed)
    s += fx_get(p.stats + (size_t)k * p.stats_slot_bs + i);
    ss += fx_get(p.stats + (size_t)k * p.stats_slot_bs + i + 2);
  }
  const double mean = s * p.inv_n;
  double var = ss * p.inv_n - mean * mean;
  if (var < 0) var = 0;
  const float rstd = (float)(1.0 / sqrt(var + 1e-5));
  const float g = p.gamma[(size_t)b * p.gb_ld + c];
  be = p.gamma[(size_t)b * p.gb_ld + p.gb_C + c];
  m = (float)mean;
  a = (1.0f + g) * rstd;
}
