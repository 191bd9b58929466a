// Training-step pieces of the decoder / discriminator autograd graph that are not layer ops of the
// conv engines (include/stts2_train.h): the Generator's Snake with learned alphas, tanh, the sum /
// average of branch outputs, the SourceModuleHnNSF with its l_linear backward, the train-mode F0 / N
// box smoothing, the MSD's time expansion backward, the GAN loss terms with their gradients and the
// AdamW update.  All of them are HBM-streaming VALU kernels (a few bytes of traffic per flop): one
// pass over their operands, grid-stride loops, fixed-order fp64 reductions (per-block partials added
// in block order), so every result is bitwise reproducible.
#include <hip/hip_runtime.h>
#include <math.h>
#include <string.h>

#include <algorithm>

#include "../../include/stts2.h"
#include "../../include/stts2_train.h"
#include "common.h"
#include "kernels.h"

namespace {

constexpr int NT = 256;

inline unsigned grid_for(long long n, int per_thread = 1) {
  long long b = (n + (long long)NT * per_thread - 1) / ((long long)NT * per_thread);
  return (unsigned)std::max<long long>(1, std::min<long long>(b, 1 << 20));
}

inline size_t al(size_t n) { return (n + 255) & ~(size_t)255; }

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// fixed-order block sum of NT doubles (the tree shape never changes); every thread returns the total
template <int K>
__device__ __forceinline__ void block_sum(double (&v)[K], double (*red)[NT / 64]) {
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const double s = wave_sum(v[k]);
    if ((threadIdx.x & 63) == 0) red[k][w] = s;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < NT / 64; ++j) s += red[k][j];
    v[k] = s;
  }
  __syncthreads();
}

// ------------------------------------------------------------------ Snake with learned alpha
// reference hifigan.py:329 / :343: x + (1 / a) * sin(a * x) ** 2, alpha [1, C, 1]
__global__ void k_snake_fwd(const float* __restrict__ x, const float* __restrict__ alpha, int C, long long n,
                            float* __restrict__ y) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const float a = alpha[(int)(i % C)];
    const float v = x[i];
    const float s = sinf(a * v);
    y[i] = v + (1.0f / a) * (s * s);
  }
}

struct Slices {
  int S;
};

Slices slices_of(int B, int L, int C) {
  const int cblk = (C + 63) / 64;
  long long S = (2048 + (long long)B * cblk - 1) / ((long long)B * cblk);
  S = std::min<long long>(S, std::max(1, L / 16));
  return Slices{(int)std::max<long long>(1, std::min<long long>(S, 1024))};
}

// autograd's chain for y = x + inv * s^2 (inv = 1/a, s = sin(a x)):  gs = dy * inv * 2 s cos(a x);
// dx = dy + gs * a;  dalpha = sum(gs * x) - sum(dy * s^2) * inv^2.  One pass writes dx and fp64
// per-(utterance, slice, channel) partials of the dalpha terms.
__global__ __launch_bounds__(256) void k_snake_bwd(const float* __restrict__ x, const float* __restrict__ alpha,
                                                   const float* __restrict__ dy, int L, int C, int S,
                                                   float* __restrict__ dx, double* __restrict__ part) {
  __shared__ double red[4][64];
  const int l = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + l, s = blockIdx.y, b = blockIdx.z;
  const int r0 = (int)((long long)L * s / S), r1 = (int)((long long)L * (s + 1) / S);
  double acc = 0.0;
  if (c < C) {
    const float a = alpha[c], inv = 1.0f / a;
    const size_t base = (size_t)b * L * C + c;
    for (int r = r0 + rl; r < r1; r += 4) {
      const size_t i = base + (size_t)r * C;
      const float v = x[i], g = dy[i];
      float sn, cs;
      sincosf(a * v, &sn, &cs);
      const float gs = g * inv * 2.0f * sn * cs;
      if (dx) dx[i] = g + gs * a;
      acc += (double)(gs * v) - (double)(g * (sn * sn)) * ((double)inv * inv);
    }
  }
  red[rl][l] = acc;
  __syncthreads();
  if (rl == 0 && c < C) part[((size_t)b * S + s) * C + c] = ((red[0][l] + red[1][l]) + red[2][l]) + red[3][l];
}

// per channel (one wave, lanes stride the slices): dalpha[c] summed over utterances in order
__global__ __launch_bounds__(64) void k_snake_bwd_final(const double* __restrict__ part, int B, int C, int S,
                                                        float* __restrict__ dalpha) {
  const int c = blockIdx.x;
  double t = 0.0;
  for (int b = 0; b < B; ++b) {
    double v = 0.0;
    for (int s = threadIdx.x; s < S; s += 64) v += part[((size_t)b * S + s) * C + c];
    t += wave_sum(v);
  }
  if (threadIdx.x == 0) dalpha[c] = (float)t;
}

// ------------------------------------------------------------------ tanh, sums, scale
__global__ void k_tanh_fwd(const float* __restrict__ x, long long n, float* __restrict__ y) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) y[i] = tanhf(x[i]);
}

// torch's tanh_backward: dy * (1 - y * y)
__global__ void k_tanh_bwd(const float* __restrict__ y, const float* __restrict__ dy, long long n,
                           float* __restrict__ dx) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const float v = y[i];
    dx[i] = dy[i] * (1.0f - v * v);
  }
}

struct SumArgs {
  const float* x[8];
  int k;
};

__global__ void k_sum_div(SumArgs a, long long n, float div, int do_div, float* __restrict__ y) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    float v = a.x[0][i];
    for (int j = 1; j < a.k; ++j) v += a.x[j][i];
    y[i] = do_div ? v / div : v;
  }
}

// ------------------------------------------------------------------ SourceModuleHnNSF (training)
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

// the counter RNG of misc.hip's k_sine_source (same key schedule, so the training forward draws the
// same noise as the inference decoder for the same (seed, utterance))
__device__ __forceinline__ float rng_normal(unsigned long long seed, long long utt, int t, int h) {
  const unsigned long long key = splitmix64(seed ^ splitmix64((unsigned long long)utt * 0x632BE59BD9B4E019ULL));
  const unsigned long long z = splitmix64(key + (unsigned long long)t * 9ULL + (unsigned long long)h);
  const float u1 = ((float)(z >> 40) + 0.5f) * (1.0f / 16777216.0f);
  const float u2 = (float)((z >> 16) & 0xFFFFFF) * (1.0f / 16777216.0f);
  return sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
}

// hifigan.py:145-157 (x scale linear upsample of the phase, sin), :205-217 (uv, noise mix) -> sw, and
// :264 tanh(l_linear(sw)) -> har; the arithmetic is misc.hip's k_sine_source (PyTorch-CPU bit for bit)
__global__ void __launch_bounds__(256) k_source_train(const float* __restrict__ f0, const float* __restrict__ ph,
                                                      int n, int scale, const float* __restrict__ lw,
                                                      const float* __restrict__ lb, const float* __restrict__ noise,
                                                      unsigned long long seed, const unsigned long long* seed_dev,
                                                      long long utt_offset, float* __restrict__ sw,
                                                      float* __restrict__ har) {
  if (seed_dev) seed = *seed_dev;  // (the capturable form: the step's seed read from the device)
  const int b = blockIdx.y;
  const int L = n * scale;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= L) return;
  const float inv_sc = (float)(1.0 / (double)scale);
  int fi = (int)floorf((float)t * inv_sc);
  if (fi > n - 1) fi = n - 1;
  const float f0v = f0[(size_t)b * n + fi];
  const float uv = f0v > 10.0f ? 1.0f : 0.0f;
  float src = fmaf(inv_sc, (float)t + 0.5f, -0.5f);
  if (src < 0.f) src = 0.f;
  const int i0 = (int)src;
  const int i1 = i0 < n - 1 ? i0 + 1 : i0;
  const float l1 = src - (float)i0;
  const float l0 = 1.0f - l1;
  const float namp = uv * 0.003f + ((1.0f - uv) * 0.1f) / 3.0f;
  float acc = 0.f;
  const float* pb = ph + (size_t)b * 9 * n;
  float* swr = sw + ((size_t)b * L + t) * 9;
#pragma unroll
  for (int h = 0; h < 9; ++h) {
    const float x0 = pb[h * n + i0], x1 = pb[h * n + i1];
    const float phase = fmaf(l0, x0, l1 * x1);
    const float sine = sinf(phase) * 0.1f;
    const float z = noise ? noise[((size_t)b * L + t) * 9 + h] : rng_normal(seed, utt_offset + b, t, h);
    const float v = sine * uv + namp * z;
    swr[h] = v;
    acc = fmaf(lw[h], v, acc);
  }
  har[(size_t)b * L + t] = tanhf(acc + lb[0]);
}

// l_linear backward: dpre = dhar (1 - har^2); dW[h] = sum dpre sw[h], db = sum dpre.  Block partials
// over contiguous sample ranges (fixed split of R = B L rows), then k_source_bwd_final in block order.
constexpr int kSrcBlocks = 512;

__global__ __launch_bounds__(256) void k_source_bwd(const float* __restrict__ sw, const float* __restrict__ har,
                                                    const float* __restrict__ dhar, long long R,
                                                    double* __restrict__ part) {
  __shared__ double red[10][NT / 64];
  const long long r0 = R * blockIdx.x / gridDim.x, r1 = R * (blockIdx.x + 1) / gridDim.x;
  double v[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) v[k] = 0.0;
  for (long long r = r0 + threadIdx.x; r < r1; r += NT) {
    const float h = har[r];
    const float d = dhar[r] * (1.0f - h * h);
    const float* s = sw + r * 9;
#pragma unroll
    for (int k = 0; k < 9; ++k) v[k] += (double)d * s[k];
    v[9] += d;
  }
  block_sum<10>(v, red);
  if (threadIdx.x < 10) part[(size_t)blockIdx.x * 10 + threadIdx.x] = v[threadIdx.x];
}

__global__ void k_source_bwd_final(const double* __restrict__ part, int nb, float* __restrict__ dW,
                                   float* __restrict__ db) {
  const int k = threadIdx.x;
  if (k >= 10) return;
  double t = 0.0;
  for (int j = 0; j < nb; ++j) t += part[(size_t)j * 10 + k];
  if (k < 9) {
    if (dW) dW[k] = (float)t;
  } else if (db) {
    db[0] = (float)t;
  }
}

// ------------------------------------------------------------------ train-mode F0 / N smoothing
// y[j] = (sum_{i<k} x[j - k/2 + i]) / k (zero padding): conv1d(x, ones(1,1,k), padding=k//2) / k
__global__ void k_box_fwd(const float* __restrict__ x, int n, int k, long long total, float* __restrict__ y) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const long long b = i / n;
    const int j = (int)(i - b * n);
    const float* xr = x + b * n;
    float s = 0.f;
    for (int t = 0; t < k; ++t) {
      const int q = j - k / 2 + t;
      if (q >= 0 && q < n) s += xr[q];
    }
    y[i] = s / (float)k;
  }
}

// dx[i] = sum over the outputs j whose window holds i of dy[j] / k
__global__ void k_box_bwd(const float* __restrict__ dy, int n, int k, long long total, float* __restrict__ dx) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const long long b = i / n;
    const int q = (int)(i - b * n);
    const float* g = dy + b * n;
    float s = 0.f;
    for (int t = k - 1; t >= 0; --t) {
      const int j = q + k / 2 - t;
      if (j >= 0 && j < n) s += g[j] / (float)k;
    }
    dx[i] = s;
  }
}

// ------------------------------------------------------------------ MSD time expansion backward
__global__ void k_time_expand3_bwd(const float* __restrict__ dx3, int H, int W, int C, long long total,
                                   float* __restrict__ dy) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const int c = (int)(i % C);
    const long long shw = i / C;
    const int w = (int)(shw % W);
    const long long sh = shw / W;
    const int h = (int)(sh % H);
    const long long s = sh / H;
    float v = 0.f;
#pragma unroll
    for (int dh = 0; dh < 3; ++dh) {
      const int hh = h - dh + 1;  // x3 row hh reads y row hh + dh - 1 = h
      if (hh >= 0 && hh < H) v += dx3[(((size_t)s * H + hh) * W + w) * 3 * C + c * 3 + dh];
    }
    dy[i] = v;
  }
}

// ------------------------------------------------------------------ GAN loss terms
constexpr int kGanChunk = 32;   // terms per launch (kernel-argument table)
constexpr int kGanBlocks = 64;  // partial-sum blocks per term (fixed: the reduction order depends on n only)
constexpr int kGanRes = 8;      // per-term results: value, median, n_sel, mean, count_eq, sum_sel(d - m), n
constexpr float kTau = 0.04f;

struct GanChunk {
  const float* a[kGanChunk];
  const float* b[kGanChunk];
  float* da[kGanChunk];
  float* db[kGanChunk];
  long long n[kGanChunk];
  int kind[kGanChunk];
  int base;  // index of the chunk's first term
  int cnt;
};

__device__ __forceinline__ unsigned f2key(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// lower median of d = a - b for every TPRLS term of the chunk: one workgroup of 1024 threads per term,
// a 4-pass 8-bit radix select on the order-preserving key of each float (LDS histograms).
__global__ __launch_bounds__(1024) void k_gan_median(GanChunk c, double* __restrict__ res) {
  const int t = blockIdx.x;
  if (t >= c.cnt || c.kind[t] != STTS_GAN_TPRLS) return;
  __shared__ unsigned hist[256];
  __shared__ unsigned s_prefix, s_k;
  const float* a = c.a[t];
  const float* b = c.b[t];
  const long long n = c.n[t];
  if (threadIdx.x == 0) {
    s_prefix = 0;
    s_k = (unsigned)((n - 1) / 2);
  }
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    for (int j = threadIdx.x; j < 256; j += 1024) hist[j] = 0;
    __syncthreads();
    const unsigned prefix = s_prefix;
    const unsigned hmask = pass == 0 ? 0u : (0xFFFFFFFFu << (32 - 8 * pass));
    for (long long i = threadIdx.x; i < n; i += 1024) {
      const unsigned key = f2key(a[i] - b[i]);
      if ((key & hmask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned k = s_k, acc = 0;
      int d = 0;
      for (; d < 255; ++d) {
        if (acc + hist[d] > k) break;
        acc += hist[d];
      }
      s_k = k - acc;
      s_prefix = prefix | ((unsigned)d << shift);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) res[(size_t)(c.base + t) * kGanRes + 1] = (double)key2f(s_prefix);
}

// per (block, term) partial sums (fp64) of the term's reductions
__global__ __launch_bounds__(256) void k_gan_sums(GanChunk c, const double* __restrict__ res,
                                                  double* __restrict__ part) {
  __shared__ double red[4][NT / 64];
  const int t = blockIdx.y;
  if (t >= c.cnt) return;
  const float* a = c.a[t];
  const float* b = c.b[t];
  const long long n = c.n[t];
  const int kind = c.kind[t];
  const long long i0 = n * blockIdx.x / kGanBlocks, i1 = n * (blockIdx.x + 1) / kGanBlocks;
  double v[4] = {0.0, 0.0, 0.0, 0.0};
  const float m = kind == STTS_GAN_TPRLS ? (float)res[(size_t)(c.base + t) * kGanRes + 1] : 0.f;
  for (long long i = i0 + threadIdx.x; i < i1; i += NT) {
    if (kind == STTS_GAN_FEATURE) {
      v[0] += fabsf(a[i] - b[i]);
    } else if (kind == STTS_GAN_GEN) {
      const float q = 1.0f - b[i];
      v[0] += q * q;
    } else if (kind == STTS_GAN_DISC) {
      const float q = 1.0f - a[i], g = b[i];
      v[0] += q * q;
      v[1] += g * g;
    } else {
      const float av = a[i], bv = b[i];
      const float d = av - bv;
      if (av < bv + m) {  // the reference's mask `dr < dg + m_DG`
        const float e = d - m;
        v[0] += e * e;
        v[1] += 1.0;
        v[3] += e;
      }
      if (d == m) v[2] += 1.0;
    }
  }
  block_sum<4>(v, red);
  if (threadIdx.x < 4) part[(((size_t)(c.base + t)) * kGanBlocks + blockIdx.x) * 4 + threadIdx.x] = v[threadIdx.x];
}

// per term: add its partials in block order, finish the term value
__global__ void k_gan_term_final(GanChunk c, const double* __restrict__ part, double* __restrict__ res) {
  const int t = threadIdx.x;
  if (t >= c.cnt) return;
  const int g = c.base + t;
  double s[4] = {0.0, 0.0, 0.0, 0.0};
  for (int j = 0; j < kGanBlocks; ++j)
    for (int k = 0; k < 4; ++k) s[k] += part[((size_t)g * kGanBlocks + j) * 4 + k];
  const double n = (double)c.n[t];
  double* r = res + (size_t)g * kGanRes;
  double val;
  switch (c.kind[t]) {
    case STTS_GAN_FEATURE: val = 2.0 * (s[0] / n); break;
    case STTS_GAN_GEN: val = s[0] / n; break;
    case STTS_GAN_DISC: val = s[0] / n + s[1] / n; break;
    default: {
      const double mean = s[0] / s[1];  // NaN when nothing is selected, as the reference's empty mean
      const double inner = (double)kTau - mean;
      val = (double)kTau - (inner > 0.0 ? inner : (inner != inner ? inner : 0.0));
      r[2] = s[1];
      r[3] = mean;
      r[4] = s[2];
      r[5] = s[3];
    }
  }
  r[0] = val;
  r[6] = n;
}

__global__ void k_gan_total(const double* __restrict__ res, int nt, double* __restrict__ loss) {
  if (threadIdx.x != 0) return;
  double l = 0.0;
  for (int t = 0; t < nt; ++t) l += res[(size_t)t * kGanRes];
  loss[0] = l;
}

__global__ __launch_bounds__(256) void k_gan_bwd(GanChunk c, const float* __restrict__ go,
                                                 const double* __restrict__ res) {
  const int t = blockIdx.y;
  if (t >= c.cnt) return;
  const float* a = c.a[t];
  const float* b = c.b[t];
  float* da = c.da[t];
  float* db = c.db[t];
  if (!da && !db) return;
  const long long n = c.n[t];
  const int kind = c.kind[t];
  const float g = go ? go[0] : 1.0f;
  const double* r = res + (size_t)(c.base + t) * kGanRes;
  // torch: mean backward = g / n (fp32), then the elementwise chain
  const float gn = g / (float)n;
  float m = 0.f, gsel = 0.f, gmed = 0.f;
  bool active = false;
  if (kind == STTS_GAN_TPRLS) {
    m = (float)r[1];
    const double mean = r[3];
    active = ((double)kTau - mean) > 0.0;  // relu'(x) = (x > 0); NaN -> inactive
    if (active) {
      gsel = g / (float)r[2];                                            // mean over the selected elements
      gmed = (float)(-2.0 * r[5] * (double)gsel / r[4]);                  // median's share, evenly split
    }
  }
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    float ga = 0.f, gb = 0.f;
    if (kind == STTS_GAN_FEATURE) {
      const float d = a[i] - b[i];
      const float sg = (float)((d > 0.f) - (d < 0.f));
      const float v = (2.0f * gn) * sg;
      ga = v;
      gb = -v;
    } else if (kind == STTS_GAN_GEN) {
      gb = -(2.0f * (1.0f - b[i]) * gn);
    } else if (kind == STTS_GAN_DISC) {
      ga = -(2.0f * (1.0f - a[i]) * gn);
      gb = 2.0f * b[i] * gn;
    } else if (active) {
      const float av = a[i], bv = b[i];
      const float d = av - bv;
      float v = 0.f;
      if (av < bv + m) v = 2.0f * (d - m) * gsel;
      if (d == m) v += gmed;
      ga = v;
      gb = -v;
    }
    if (da) da[i] = ga;
    if (db) db[i] = gb;
  }
}

// ------------------------------------------------------------------ AdamW
constexpr int kAdamChunk = 32;
constexpr int kAdamPer = 2048;  // elements per block (8 per thread)

struct AdamTable {
  float* p[kAdamChunk];
  const float* g[kAdamChunk];
  float* m[kAdamChunk];
  float* v[kAdamChunk];
  long long n[kAdamChunk];
  int start[kAdamChunk + 1];  // first block of each tensor (prefix over ceil(n / kAdamPer))
  int cnt;
};

struct AdamScalars {
  float decay;      // 1 - lr * wd
  float w1;         // 1 - beta1 (lerp weight)
  float beta2;
  float omb2;       // 1 - beta2
  float bc2_sqrt;   // sqrt(1 - beta2^step)
  float eps;
  float neg_step;   // -lr / (1 - beta1^step)
};

__device__ __forceinline__ void adamw_body(const AdamTable& tb, const AdamScalars& s) {
  const int blk = blockIdx.x;
  int t = 0;
  while (t + 1 < tb.cnt && tb.start[t + 1] <= blk) ++t;
  const long long base = (long long)(blk - tb.start[t]) * kAdamPer;
  const long long n = tb.n[t];
  float* __restrict__ p = tb.p[t];
  const float* __restrict__ g = tb.g[t];
  float* __restrict__ m = tb.m[t];
  float* __restrict__ v = tb.v[t];
  for (int j = threadIdx.x; j < kAdamPer; j += NT) {
#pragma clang fp contract(off)  // torch's CPU AdamW rounds every product and sum separately
    const long long i = base + j;
    if (i >= n) break;
    const float gi = g[i];
    float pi = p[i] * s.decay;
    float mi = m[i];
    // ATen lerp: weight < 0.5 ? self + w (end - self) : end - (end - self) (1 - w)
    mi = s.w1 < 0.5f ? mi + s.w1 * (gi - mi) : gi - (gi - mi) * (1.0f - s.w1);
    float vi = v[i] * s.beta2;
    vi = vi + s.omb2 * gi * gi;
    const float den = sqrtf(vi) / s.bc2_sqrt + s.eps;
    pi = pi + s.neg_step * mi / den;
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
  }
}

__global__ __launch_bounds__(256) void k_adamw(AdamTable tb, AdamScalars s) { adamw_body(tb, s); }

// capturable form (stts_adamw_step_dev): the scalars come from device memory, formed by k_adamw_prep from the step
// count it advances there, so a hipGraph replay of the launch takes the next step's bias corrections
__global__ __launch_bounds__(256) void k_adamw_dev(AdamTable tb, const AdamScalars* __restrict__ sp) {
  const AdamScalars s = *sp;
  adamw_body(tb, s);
}

__global__ void k_adamw_prep(double* __restrict__ st, double lr, double beta1, double beta2, double eps, double wd,
                             AdamScalars* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const double step = st[0] + 1.0;
  st[0] = step;
  AdamScalars sc;
  sc.decay = (float)(1.0 - lr * wd);
  sc.w1 = (float)(1.0 - beta1);
  sc.beta2 = (float)beta2;
  sc.omb2 = (float)(1.0 - beta2);
  sc.bc2_sqrt = (float)sqrt(1.0 - pow(beta2, step));
  sc.eps = (float)eps;
  sc.neg_step = (float)(-(lr / (1.0 - pow(beta1, step))));
  *out = sc;
}

// ------------------------------------------------------------------ Dropout (train mode)
// keep element i when its counter draw u(seed, i) >= p; y = keep ? x / (1 - p) : 0 (torch's scaling).  The
// backward redraws the same mask from (seed, i): nothing is stored.
__device__ __forceinline__ bool drop_keep(unsigned long long seed, long long i, float p) {
  const unsigned long long z = splitmix64(seed ^ splitmix64((unsigned long long)i * 0xD1B54A32D192ED03ULL));
  return (float)(z >> 40) * (1.0f / 16777216.0f) >= p;
}

__global__ void __launch_bounds__(256) k_dropout(const float* __restrict__ x, long long n, float p, float scale,
                                                 unsigned long long seed, float* __restrict__ y) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT)
    y[i] = drop_keep(seed, i, p) ? x[i] * scale : 0.f;
}
// the same with the keep mask given (1 = kept): train-mode parity against the reference with injected masks
__global__ void __launch_bounds__(256) k_dropout_mask(const float* __restrict__ x, const float* __restrict__ mask,
                                                      long long n, float scale, float* __restrict__ y) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT)
    y[i] = mask[i] != 0.f ? x[i] * scale : 0.f;
}

}  // namespace

namespace {
// ------------------------------------------------------------------ smooth L1 (train.py:269-270)
// F.smooth_l1_loss(x, y) (beta 1, mean): one workgroup, fp64 per-lane sums reduced in a fixed tree order
__global__ void __launch_bounds__(256) k_smooth_l1(const float* __restrict__ x, const float* __restrict__ y,
                                                   long long n, double* __restrict__ loss) {
  __shared__ double red[256];
  double acc = 0.0;
  for (long long i = threadIdx.x; i < n; i += 256) {
    const float d = x[i] - y[i], ad = fabsf(d);
    acc += ad < 1.f ? 0.5 * (double)d * (double)d : (double)ad - 0.5;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = n ? red[0] / (double)n : 0.0;
}

// d/dx = g d / n (|d| < 1) or g sign(d) / n, d = x - y; dy = -dx.  g: the upstream gradient (a device scalar)
__global__ void __launch_bounds__(256) k_smooth_l1_bwd(const float* __restrict__ x, const float* __restrict__ y,
                                                       long long n, const float* __restrict__ g,
                                                       float* __restrict__ dx, float* __restrict__ dy) {
  const float s = g[0] / (float)n;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const float d = x[i] - y[i];
    const float v = (fabsf(d) < 1.f ? d : (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f))) * s;
    if (dx) dx[i] = v;
    if (dy) dy[i] = -v;
  }
}

}  // namespace

namespace {
}  // namespace

// ================================================================== C-ABI
extern "C" long long stts_snake_workspace_bytes(int B, int L, int C) {
  if (B <= 0 || L <= 0 || C <= 0) return ST_EINVAL;
  return (long long)al((size_t)B * slices_of(B, L, C).S * C * sizeof(double));
}

extern "C" int stts_snake_fwd(const float* x, const float* alpha, int B, int L, int C, float* y, void* stream) {
  if (!x || !alpha || !y || B <= 0 || L <= 0 || C <= 0) return ST_EINVAL;
  const long long n = (long long)B * L * C;
  hipLaunchKernelGGL(k_snake_fwd, dim3(grid_for(n, 4)), dim3(NT), 0, (hipStream_t)stream, x, alpha, C, n, y);
  return (int)hipGetLastError();
}

extern "C" int stts_snake_bwd(const float* x, const float* alpha, const float* dy, int B, int L, int C, float* dx,
                              float* dalpha, void* ws, long long ws_bytes, void* stream) {
  const long long need = stts_snake_workspace_bytes(B, L, C);
  if (need < 0) return (int)need;
  if (!x || !alpha || !dy) return ST_EINVAL;
  if (!dx && !dalpha) return 0;
  if (!ws || ws_bytes < need) return ST_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const Slices sl = slices_of(B, L, C);
  double* part = (double*)ws;
  hipLaunchKernelGGL(k_snake_bwd, dim3((C + 63) / 64, sl.S, B), dim3(256), 0, s, x, alpha, dy, L, C, sl.S, dx, part);
  ST_CHECK_HIP(hipGetLastError());
  if (dalpha) {
    hipLaunchKernelGGL(k_snake_bwd_final, dim3(C), dim3(64), 0, s, part, B, C, sl.S, dalpha);
    ST_CHECK_HIP(hipGetLastError());
  }
  return 0;
}

extern "C" int stts_tanh_fwd(const float* x, long long n, float* y, void* stream) {
  if (!x || !y || n < 0) return ST_EINVAL;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_tanh_fwd, dim3(grid_for(n, 4)), dim3(NT), 0, (hipStream_t)stream, x, n, y);
  return (int)hipGetLastError();
}

extern "C" int stts_tanh_bwd(const float* y, const float* dy, long long n, float* dx, void* stream) {
  if (!y || !dy || !dx || n < 0) return ST_EINVAL;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_tanh_bwd, dim3(grid_for(n, 4)), dim3(NT), 0, (hipStream_t)stream, y, dy, n, dx);
  return (int)hipGetLastError();
}

extern "C" int stts_sum_div(const float* const* xs, int k, long long n, float div, float* y, void* stream) {
  if (!xs || k < 1 || k > 8 || n < 0 || !y || !(div != 0.f)) return ST_EINVAL;
  SumArgs a;
  memset(&a, 0, sizeof(a));
  for (int j = 0; j < k; ++j) {
    if (!xs[j]) return ST_EINVAL;
    a.x[j] = xs[j];
  }
  a.k = k;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_sum_div, dim3(grid_for(n, 4)), dim3(NT), 0, (hipStream_t)stream, a, n, div, div != 1.0f ? 1 : 0,
                     y);
  return (int)hipGetLastError();
}

extern "C" int stts_div(const float* x, long long n, float div, float* y, void* stream) {
  const float* xs[1] = {x};
  if (!x) return ST_EINVAL;
  if (div == 1.0f) {  // an exact copy (x / 1)
    if (n > 0 && x != y) return (int)hipMemcpyAsync(y, x, (size_t)n * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream);
    return 0;
  }
  return stts_sum_div(xs, 1, n, div, y, stream);
}

extern "C" long long stts_source_workspace_bytes(int B, int n) {
  if (B <= 0 || n <= 0) return ST_EINVAL;
  return (long long)std::max(al((size_t)B * 9 * n * sizeof(float)), al((size_t)kSrcBlocks * 10 * sizeof(double)));
}

static int source_fwd(const float* f0_curve, const float* lw, const float* lb, const float* noise,
                      unsigned long long seed, const unsigned long long* seed_dev, long long utt_offset, int B, int n,
                      int scale, float* sw, float* har, void* ws, long long ws_bytes, void* stream) {
  const long long need = stts_source_workspace_bytes(B, n);
  if (need < 0) return (int)need;
  if (!f0_curve || !lw || !lb || !sw || !har || scale <= 0 || (long long)n * scale > (1LL << 31) - 1)
    return ST_EINVAL;
  if (!ws || ws_bytes < need) return ST_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  float* ph = (float*)ws;
  ST_CHECK(st_sine_phase(f0_curve, B, n, scale, ph, s));
  const int L = n * scale;
  hipLaunchKernelGGL(k_source_train, dim3((L + 255) / 256, B), dim3(256), 0, s, f0_curve, ph, n, scale, lw, lb, noise,
                     seed, seed_dev, utt_offset, sw, har);
  return (int)hipGetLastError();
}

extern "C" int stts_source_fwd(const float* f0_curve, const float* lw, const float* lb, const float* noise,
                               unsigned long long seed, long long utt_offset, int B, int n, int scale, float* sw,
                               float* har, void* ws, long long ws_bytes, void* stream) {
  return source_fwd(f0_curve, lw, lb, noise, seed, nullptr, utt_offset, B, n, scale, sw, har, ws, ws_bytes, stream);
}

extern "C" int stts_source_fwd_seed_dev(const float* f0_curve, const float* lw, const float* lb, const float* noise,
                                        const unsigned long long* seed_dev, long long utt_offset, int B, int n,
                                        int scale, float* sw, float* har, void* ws, long long ws_bytes,
                                        void* stream) {
  if (!seed_dev && !noise) return ST_EINVAL;
  return source_fwd(f0_curve, lw, lb, noise, 0ull, seed_dev, utt_offset, B, n, scale, sw, har, ws, ws_bytes, stream);
}

extern "C" int stts_source_bwd(const float* sw, const float* har, const float* dhar, int B, long long L, float* dW,
                               float* db, void* ws, long long ws_bytes, void* stream) {
  if (!sw || !har || !dhar || B <= 0 || L <= 0) return ST_EINVAL;
  if (!dW && !db) return 0;
  if (!ws || ws_bytes < (long long)al((size_t)kSrcBlocks * 10 * sizeof(double))) return ST_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  double* part = (double*)ws;
  hipLaunchKernelGGL(k_source_bwd, dim3(kSrcBlocks), dim3(NT), 0, s, sw, har, dhar, (long long)B * L, part);
  ST_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_source_bwd_final, dim3(1), dim3(64), 0, s, part, kSrcBlocks, dW, db);
  return (int)hipGetLastError();
}

extern "C" int stts_box_smooth_fwd(const float* x, int B, int n, int k, float* y, void* stream) {
  if (!x || !y || B <= 0 || n <= 0 || k <= 0 || (k & 1) == 0) return ST_EINVAL;
  const long long total = (long long)B * n;
  hipLaunchKernelGGL(k_box_fwd, dim3(grid_for(total)), dim3(NT), 0, (hipStream_t)stream, x, n, k, total, y);
  return (int)hipGetLastError();
}

extern "C" int stts_box_smooth_bwd(const float* dy, int B, int n, int k, float* dx, void* stream) {
  if (!dy || !dx || B <= 0 || n <= 0 || k <= 0 || (k & 1) == 0) return ST_EINVAL;
  const long long total = (long long)B * n;
  hipLaunchKernelGGL(k_box_bwd, dim3(grid_for(total)), dim3(NT), 0, (hipStream_t)stream, dy, n, k, total, dx);
  return (int)hipGetLastError();
}

extern "C" int stts_time_expand3(const float* y, int S, int H, int W, int C, float* x3, void* stream) {
  if (!y || !x3 || S <= 0 || H <= 0 || W <= 0 || C <= 0 || S > 65535) return ST_EINVAL;
  return st_time_expand(y, S, H, W, C, x3, ST_FP32, (hipStream_t)stream);
}

extern "C" int stts_time_expand3_bwd(const float* dx3, int S, int H, int W, int C, float* dy, void* stream) {
  if (!dx3 || !dy || S <= 0 || H <= 0 || W <= 0 || C <= 0) return ST_EINVAL;
  const long long total = (long long)S * H * W * C;
  hipLaunchKernelGGL(k_time_expand3_bwd, dim3(grid_for(total, 4)), dim3(NT), 0, (hipStream_t)stream, dx3, H, W, C,
                     total, dy);
  return (int)hipGetLastError();
}

extern "C" long long stts_gan_workspace_bytes(int n_terms) {
  if (n_terms <= 0 || n_terms > 256) return ST_EINVAL;
  return (long long)(al((size_t)n_terms * kGanRes * sizeof(double)) +
                     al((size_t)n_terms * kGanBlocks * 4 * sizeof(double)));
}

static int gan_chunk(const stts_gan_term* terms, float* const* da, float* const* db, int base, int cnt, GanChunk& c) {
  memset(&c, 0, sizeof(c));
  c.base = base;
  c.cnt = cnt;
  for (int j = 0; j < cnt; ++j) {
    const stts_gan_term& t = terms[base + j];
    if (!t.a || !t.b || t.n <= 0 || t.kind < 0 || t.kind > 3) return ST_EINVAL;
    if (t.kind == STTS_GAN_TPRLS && t.n > 0xFFFFFFFFLL) return ST_EINVAL;
    c.a[j] = t.a;
    c.b[j] = t.b;
    c.n[j] = t.n;
    c.kind[j] = t.kind;
    c.da[j] = da ? da[base + j] : nullptr;
    c.db[j] = db ? db[base + j] : nullptr;
  }
  return 0;
}

extern "C" int stts_gan_loss(const stts_gan_term* terms, int n_terms, double* loss, void* ws, long long ws_bytes,
                             void* stream) {
  const long long need = stts_gan_workspace_bytes(n_terms);
  if (need < 0) return (int)need;
  if (!terms || !loss) return ST_EINVAL;
  if (!ws || ws_bytes < need) return ST_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  double* res = (double*)ws;
  double* part = (double*)((char*)ws + al((size_t)n_terms * kGanRes * sizeof(double)));
  for (int base = 0; base < n_terms; base += kGanChunk) {
    GanChunk c;
    ST_CHECK(gan_chunk(terms, nullptr, nullptr, base, std::min(kGanChunk, n_terms - base), c));
    bool any_tprls = false;
    for (int j = 0; j < c.cnt; ++j) any_tprls |= c.kind[j] == STTS_GAN_TPRLS;
    if (any_tprls) {
      hipLaunchKernelGGL(k_gan_median, dim3(c.cnt), dim3(1024), 0, s, c, res);
      ST_CHECK_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(k_gan_sums, dim3(kGanBlocks, c.cnt), dim3(NT), 0, s, c, res, part);
    ST_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_gan_term_final, dim3(1), dim3(64), 0, s, c, part, res);
    ST_CHECK_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(k_gan_total, dim3(1), dim3(64), 0, s, res, n_terms, loss);
  return (int)hipGetLastError();
}

extern "C" int stts_gan_loss_bwd(const stts_gan_term* terms, float* const* da, float* const* db, int n_terms,
                                 const float* go, const void* ws, long long ws_bytes, void* stream) {
  const long long need = stts_gan_workspace_bytes(n_terms);
  if (need < 0) return (int)need;
  if (!terms) return ST_EINVAL;
  if (!ws || ws_bytes < need) return ST_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const double* res = (const double*)ws;
  for (int base = 0; base < n_terms; base += kGanChunk) {
    GanChunk c;
    ST_CHECK(gan_chunk(terms, da, db, base, std::min(kGanChunk, n_terms - base), c));
    long long nmax = 1;
    for (int j = 0; j < c.cnt; ++j) nmax = std::max(nmax, c.n[j]);
    const unsigned gx = (unsigned)std::min<long long>((nmax + NT * 4 - 1) / (NT * 4), 2048);
    hipLaunchKernelGGL(k_gan_bwd, dim3(gx, c.cnt), dim3(NT), 0, s, c, go, res);
    ST_CHECK_HIP(hipGetLastError());
  }
  return 0;
}

extern "C" int stts_adamw_step(const stts_adamw_tensor* tensors, int n_tensors, double lr, double beta1,
                               double beta2, double eps, double weight_decay, long long step, void* stream) {
  if (!tensors || n_tensors < 0 || step < 1 || !(beta1 >= 0.0 && beta1 < 1.0) || !(beta2 >= 0.0 && beta2 < 1.0))
    return ST_EINVAL;
  // the scalars as torch's single-tensor AdamW forms them: Python floats (double) combined in double, each
  // cast to fp32 by ATen where it meets the fp32 tensor
  const double dlr = lr, dwd = weight_decay, db1 = beta1, db2 = beta2;
  AdamScalars sc;
  sc.decay = (float)(1.0 - dlr * dwd);
  sc.w1 = (float)(1.0 - db1);
  sc.beta2 = (float)beta2;
  sc.omb2 = (float)(1.0 - db2);
  sc.bc2_sqrt = (float)sqrt(1.0 - pow(db2, (double)step));
  sc.eps = (float)eps;
  sc.neg_step = (float)(-(dlr / (1.0 - pow(db1, (double)step))));
  hipStream_t s = (hipStream_t)stream;
  for (int base = 0; base < n_tensors; base += kAdamChunk) {
    AdamTable tb;
    memset(&tb, 0, sizeof(tb));
    int blocks = 0;
    for (int j = 0; j < kAdamChunk && base + j < n_tensors; ++j) {
      const stts_adamw_tensor& t = tensors[base + j];
      if (t.n < 0 || (t.n > 0 && (!t.param || !t.grad || !t.exp_avg || !t.exp_avg_sq))) return ST_EINVAL;
      tb.p[j] = t.param;
      tb.g[j] = t.grad;
      tb.m[j] = t.exp_avg;
      tb.v[j] = t.exp_avg_sq;
      tb.n[j] = t.n;
      tb.start[j] = blocks;
      const long long nb = (t.n + kAdamPer - 1) / kAdamPer;
      if (blocks + nb > (1LL << 30)) return ST_EINVAL;
      blocks += (int)nb;
      tb.cnt = j + 1;
    }
    tb.start[tb.cnt] = blocks;
    if (blocks == 0) continue;
    hipLaunchKernelGGL(k_adamw, dim3(blocks), dim3(NT), 0, s, tb, sc);
    ST_CHECK_HIP(hipGetLastError());
  }
  return 0;
}

// the capturable AdamW step (include/stts2_train.h): state[0] = the step count (fp64, advanced on the device), the
// scalars of the step formed on the device in state[1..]
extern "C" int stts_adamw_step_dev(const stts_adamw_tensor* tensors, int n_tensors, double lr, double beta1,
                                   double beta2, double eps, double weight_decay, double* state, void* stream) {
  if (!tensors || n_tensors < 0 || !state || !(beta1 >= 0.0 && beta1 < 1.0) || !(beta2 >= 0.0 && beta2 < 1.0))
    return ST_EINVAL;
  static_assert(sizeof(AdamScalars) <= 7 * sizeof(double), "scalars fit state[1..8)");
  hipStream_t s = (hipStream_t)stream;
  AdamScalars* sc = reinterpret_cast<AdamScalars*>(state + 1);
  hipLaunchKernelGGL(k_adamw_prep, dim3(1), dim3(64), 0, s, state, lr, beta1, beta2, eps, weight_decay, sc);
  ST_CHECK_HIP(hipGetLastError());
  for (int base = 0; base < n_tensors; base += kAdamChunk) {
    AdamTable tb;
    memset(&tb, 0, sizeof(tb));
    int blocks = 0;
    for (int j = 0; j < kAdamChunk && base + j < n_tensors; ++j) {
      const stts_adamw_tensor& t = tensors[base + j];
      if (t.n < 0 || (t.n > 0 && (!t.param || !t.grad || !t.exp_avg || !t.exp_avg_sq))) return ST_EINVAL;
      tb.p[j] = t.param;
      tb.g[j] = t.grad;
      tb.m[j] = t.exp_avg;
      tb.v[j] = t.exp_avg_sq;
      tb.n[j] = t.n;
      tb.start[j] = blocks;
      const long long nb = (t.n + kAdamPer - 1) / kAdamPer;
      if (blocks + nb > (1LL << 30)) return ST_EINVAL;
      blocks += (int)nb;
      tb.cnt = j + 1;
    }
    tb.start[tb.cnt] = blocks;
    if (blocks == 0) continue;
    hipLaunchKernelGGL(k_adamw_dev, dim3(blocks), dim3(NT), 0, s, tb, (const AdamScalars*)sc);
    ST_CHECK_HIP(hipGetLastError());
  }
  return 0;
}

extern "C" int stts_dropout(const float* x, long long n, float p, unsigned long long seed, float* y, void* stream) {
  if (!x || !y || n < 0 || !(p >= 0.f && p < 1.f)) return ST_EINVAL;
  if (n == 0) return 0;
  const long long g = (n + NT - 1) / NT;
  hipLaunchKernelGGL(k_dropout, dim3((unsigned)(g < 65536 ? g : 65536)), dim3(NT), 0, (hipStream_t)stream, x, n, p,
                     1.0f / (1.0f - p), seed, y);
  return (int)hipGetLastError();
}

extern "C" int stts_dropout_mask(const float* x, const float* mask, long long n, float p, float* y, void* stream) {
  if (!x || !mask || !y || n < 0 || !(p >= 0.f && p < 1.f)) return ST_EINVAL;
  if (n == 0) return 0;
  const long long g = (n + NT - 1) / NT;
  hipLaunchKernelGGL(k_dropout_mask, dim3((unsigned)(g < 65536 ? g : 65536)), dim3(NT), 0, (hipStream_t)stream, x, mask,
                     n, 1.0f / (1.0f - p), y);
  return (int)hipGetLastError();
}

extern "C" int stts_smooth_l1_loss(const float* x, const float* y, long long n, double* loss, void* stream) {
  if (!x || !y || !loss || n < 0) return ST_EINVAL;
  hipLaunchKernelGGL(k_smooth_l1, dim3(1), dim3(256), 0, (hipStream_t)stream, x, y, n, loss);
  return (int)hipGetLastError();
}

extern "C" int stts_smooth_l1_loss_bwd(const float* x, const float* y, long long n, const float* g, float* dx,
                                       float* dy, void* stream) {
  if (!x || !y || !g || n < 0) return ST_EINVAL;
  if (n == 0) return 0;
  const long long gr = (n + NT - 1) / NT;
  hipLaunchKernelGGL(k_smooth_l1_bwd, dim3((unsigned)(gr < 4096 ? gr : 4096)), dim3(NT), 0, (hipStream_t)stream, x, y,
                     n, g, dx, dy);
  return (int)hipGetLastError();
}
