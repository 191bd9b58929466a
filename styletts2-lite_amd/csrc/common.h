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
  const double* stats;   // [B][stats_ld][2] (sum, sumsq) of the input, per (utterance, channel)
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

// Per-(utterance, channel) AdaIN coefficients from raw stats: mean, a = (1+gamma)*rstd, beta.
__device__ __forceinline__ void adain_coeffs(const Prologue& p, int b, int c, float& m, float& a, float& be) {
  const size_t i = ((size_t)b * p.stats_ld + c) * 2;
  double s = p.stats[i], ss = p.stats[i + 1];
  for (int k = 1; k < p.stats_slots; ++k) {
    s += p.stats[(size_t)k * p.stats_slot_bs + i];
    ss += p.stats[(size_t)k * p.stats_slot_bs + i + 1];
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
