// Memory-bound / small kernels of the synthesis path (gfx950):
//   layout conversion + InstanceNorm statistics, the single-channel convs (F0_conv,
//   N_conv, HiFi-GAN noise_convs), the harmonic-plus-noise source (SineGen +
//   SourceModuleHnNSF), the depthwise x2 ConvTranspose "pool", the AdaIN style
//   projections, the iSTFTNet CustomSTFT transform / inverse, and weight-norm
//   folding + MFMA weight packing.
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace {



#define DISPATCH_DTYPE(dtype, T, ...)              \
  do {                                             \
    if ((dtype) == ST_FP32) {                      \
      using T = float;                             \
      __VA_ARGS__;                                 \
    } else if ((dtype) == ST_BF16) {               \
      using T = bf16_t;                            \
      __VA_ARGS__;                                 \
    } else {                                       \
      return ST_EDTYPE;                            \
    }                                              \
  } while (0)

// slots 1..S-1 of a spread statistics buffer folded into slot 0 and cleared (ConvParams::stats_slots)
__global__ void __launch_bounds__(256) k_stats_fold(double* __restrict__ st, int B, int ld, int C, int S,
                                                    long long slot_bs) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B * C) return;
  const int b = i / C, c = i % C;
  // integer (fixed-point) words: the fold is exact and order-free like the producers' atomics (common.h ST_W)
  long long* d = reinterpret_cast<long long*>(st + ((size_t)b * ld + c) * ST_W);
  // (the lo words' poison bit, ST_POISON, is OR-ed, not added: two poisoned words must not cancel it)
  unsigned long long w[ST_W] = {0, 0, 0, 0}, flag[ST_W] = {0, 0, 0, 0};
  unsigned long long* du = reinterpret_cast<unsigned long long*>(d);
  for (int k = 1; k < S; ++k) {
    unsigned long long* e = du + (size_t)k * slot_bs;
#pragma unroll
    for (int j = 0; j < ST_W; ++j) {
      const unsigned long long v = e[j];
      if (j & 1) {
        flag[j] |= v & ST_POISON;
        w[j] += v & ~ST_POISON;
      } else {
        w[j] += v;
      }
      e[j] = 0;
    }
  }
#pragma unroll
  for (int j = 0; j < ST_W; ++j) {
    if (j & 1) du[j] = ((du[j] & ~ST_POISON) + w[j]) | (du[j] & ST_POISON) | flag[j];
    else du[j] += w[j];
  }
}

__device__ __forceinline__ void atomic_stats(double* st, double a, double q) { stat_add(st, a, q); }

// ------------------------------------------------------------------ NCL -> frames
template <typename T>
__global__ void __launch_bounds__(256) k_ncl_to_frames(const float* __restrict__ src, int C, int L, T* dst, int ld,
                                                       int c0, long long dst_bs, double* stats, int stats_ld) {
  __shared__ float tile[64][65];
  const int b = blockIdx.z, ct = blockIdx.y * 64, lt = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
  const float* sb = src + (size_t)b * C * L;
  for (int i = ty; i < 64; i += 4) {
    const int c = ct + i, l = lt + tx;
    tile[i][tx] = (c < C && l < L) ? sb[(size_t)c * L + l] : 0.f;
  }
  __syncthreads();
  T* db = dst + (size_t)b * dst_bs;
  for (int i = ty; i < 64; i += 4) {
    const int l = lt + i, c = ct + tx;
    if (l < L && c < C) db[(size_t)l * ld + c0 + c] = from_f32<T>(tile[tx][i]);
  }
  if (stats && threadIdx.x < 64) {
    const int c = ct + threadIdx.x;
    if (c < C) {
      double a = 0, q = 0;
      for (int j = 0; j < 64; ++j) {
        if (lt + j < L) {
          const float v = to_f32(from_f32<T>(tile[threadIdx.x][j]));
          a += v;
          q += (double)v * v;
        }
      }
      atomic_stats(stats + ((size_t)b * stats_ld + c0 + c) * ST_W, a, q);
    }
  }
}

// ------------------------------------------------------------------ fp32 frames -> frames
template <typename T>
__global__ void __launch_bounds__(256) k_frames_convert(const float* __restrict__ src, int L, int C, int ld_in,
                                                        T* dst, int ld_out, double* stats, int stats_ld) {
  const int b = blockIdx.y;
  const int c = threadIdx.x + blockIdx.z * 256;
  if (c >= C) return;
  const int rows = 64, r0 = blockIdx.x * rows;
  double a = 0, q = 0;
  for (int r = r0; r < min(r0 + rows, L); ++r) {
    const float v = src[((size_t)b * L + r) * ld_in + c];
    const T t = from_f32<T>(v);
    dst[((size_t)b * L + r) * ld_out + c] = t;
    const float w = to_f32(t);
    a += w;
    q += (double)w * w;
  }
  if (stats) atomic_stats(stats + ((size_t)b * stats_ld + c) * ST_W, a, q);
}

// fp32 frames [rows][ld_in] -> bf16 frames [rows][ld_out] (ld_out % 8 == 0), no statistics: one thread per
// (row, 8-channel group), 32-B loads and one 16-B store; channels C .. ld_out - 1 written as 0 (the training
// path's conv inputs; k_frames_convert serves the statistics-producing plan conversions)
__global__ void __launch_bounds__(256) k_cvt_bf16_rows(const float* __restrict__ src, long long rows, int C, int ld_in,
                                                       bf16_t* __restrict__ dst, int ld_out) {
  const int ng = ld_out >> 3;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * ng) return;
  const long long r = i / ng;
  const int c = (int)(i - r * ng) * 8;
  const float* sp = src + r * ld_in + c;
  float v[8];
  if (c + 8 <= C && ((ld_in | c) & 3) == 0) {
    const float4 a = *reinterpret_cast<const float4*>(sp);
    const float4 b = *reinterpret_cast<const float4*>(sp + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = c + j < C ? sp[j] : 0.f;
  }
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (bf16_t)v[j];
  *reinterpret_cast<bf16x8*>(dst + r * ld_out + c) = o;
}

// bf16 frames [rows][ld] -> fp32 [rows][C] with C % 8 == 0: 16-B loads, 32-B stores
__global__ void __launch_bounds__(256) k_cvt_f32_rows(const bf16_t* __restrict__ src, long long rows, int C, int ld,
                                                      float* __restrict__ dst) {
  const int ng = C >> 3;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * ng) return;
  const long long r = i / ng;
  const int c = (int)(i - r * ng) * 8;
  const bf16x8 a = *reinterpret_cast<const bf16x8*>(src + r * ld + c);
  float4 o0, o1;
  o0.x = (float)a[0]; o0.y = (float)a[1]; o0.z = (float)a[2]; o0.w = (float)a[3];
  o1.x = (float)a[4]; o1.y = (float)a[5]; o1.z = (float)a[6]; o1.w = (float)a[7];
  float* dp = dst + r * C + c;
  *reinterpret_cast<float4*>(dp) = o0;
  *reinterpret_cast<float4*>(dp + 4) = o1;
}

template <typename T>
__global__ void __launch_bounds__(256) k_frames_to_f32(const T* __restrict__ src, int L, int C, int ld, float* dst) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const int b = blockIdx.y;
  if (i >= (size_t)L * C) return;
  const size_t r = i / C, c = i % C;
  dst[((size_t)b * L + r) * C + c] = to_f32(src[((size_t)b * L + r) * ld + c]);
}

// ------------------------------------------------------------------ Cin = 1 conv
// out[b][t][c] = bias[c] + sum_k w[c][k] * in[b][t*stride - pad + k]   (zero padded)
// reference hifigan.py:296-302 (noise_convs), :434-436 (F0_conv / N_conv).
// Each thread owns one channel (weights in registers); the input window is staged in LDS
// and read as a wave-wide broadcast; stores are channel-contiguous.
constexpr int C1_TT = 512;
template <typename T, int KC>
__global__ void __launch_bounds__(256) k_conv_cin1(const float* __restrict__ in, long long in_bs, int Lin,
                                                   const float* __restrict__ w, const float* __restrict__ bias,
                                                   int C, int Kr, int stride, int pad, int Lout, SmallConvDst d0,
                                                   SmallConvDst d1, SmallConvDst d2, int ndst) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* win = reinterpret_cast<float*>(smem);
  const int K = KC > 0 ? KC : Kr;
  const int b = blockIdx.y, t0 = blockIdx.x * C1_TT;
  const int nwin = (C1_TT - 1) * stride + K;
  const float* ib = in + (size_t)b * in_bs;
  for (int i = threadIdx.x; i < nwin; i += 256) {
    const int g = t0 * stride - pad + i;
    win[i] = (g >= 0 && g < Lin) ? ib[g] : 0.f;
  }
  float* wl = win + ((nwin + 3) & ~3);  // generic-K weights [C][K] (KC == 0 only)
  double* red = reinterpret_cast<double*>(wl + (KC > 0 ? 0 : ((C * K + 3) & ~3)));
  if (KC == 0)
    for (int i = threadIdx.x; i < C * K; i += 256) wl[i] = w[i];
  __syncthreads();
  const int cstr = C < 256 ? C : 256;
  const int tsplit = 256 / cstr;
  const int cl = threadIdx.x % cstr, ts = threadIdx.x / cstr;
  const SmallConvDst* ds[3] = {&d0, &d1, &d2};
  for (int cb = 0; cb < C; cb += cstr) {
    const int c = cb + cl;
    double a = 0, q = 0;
    if (ts < tsplit && c < C) {
      float wr[KC > 0 ? KC : 1];
      if constexpr (KC > 0) {
#pragma unroll
        for (int k = 0; k < KC; ++k) wr[k] = w[(size_t)c * KC + k];
      }
      const float bc = bias ? bias[c] : 0.f;
      float fa = 0.f, fq = 0.f;
      for (int tl = ts; tl < C1_TT; tl += tsplit) {
        const int t = t0 + tl;
        if (t >= Lout) break;
        const float* xw = win + tl * stride;
        float acc = 0.f;
        if constexpr (KC > 0) {
#pragma unroll
          for (int k = 0; k < KC; ++k) acc = fmaf(wr[k], xw[k], acc);
        } else {
          for (int k = 0; k < K; ++k) acc = fmaf(wl[c * K + k], xw[k], acc);
        }
        const float v = acc + bc;
        const T tv = from_f32<T>(v);
        for (int di = 0; di < ndst; ++di)
          reinterpret_cast<T*>(ds[di]->y)[(size_t)b * ds[di]->y_bs + (size_t)t * ds[di]->y_ld + ds[di]->c0 + c] = tv;
        const float vs = to_f32(tv);
        fa += vs;
        fq += vs * vs;
      }
      a = fa;
      q = fq;
    }
    if (d0.stats == nullptr && d1.stats == nullptr) continue;
    __syncthreads();
    red[(ts * cstr + cl) * 2] = a;
    red[(ts * cstr + cl) * 2 + 1] = q;
    __syncthreads();
    if (threadIdx.x < cstr && cb + threadIdx.x < C) {
      double A = 0, Q = 0;
      for (int s2 = 0; s2 < tsplit; ++s2) {
        A += red[(s2 * cstr + threadIdx.x) * 2];
        Q += red[(s2 * cstr + threadIdx.x) * 2 + 1];
      }
      for (int di = 0; di < ndst; ++di)
        if (ds[di]->stats)
          atomic_stats(ds[di]->stats + ((size_t)b * ds[di]->stats_ld + ds[di]->c0 + cb + threadIdx.x) * ST_W, A, Q);
    }
  }
}

// ------------------------------------------------------------------ SineGen
// reference hifigan.py:117-157: rad = (f0*h/sr) % 1; linear /scale downsample reads two
// equal samples of the nearest-upsampled curve (src = scale*j + (scale-1)/2), so the
// downsampled value is rad(f0[j]) exactly; cumsum accumulates in fp64 and rounds per
// element (PyTorch-CPU semantics); phase = (cum*2)*pi, then *scale.
// One block per utterance: the F0 row is staged in LDS (coalesced), then one thread per
// harmonic runs the serial fp64 prefix sum (PyTorch-CPU cumsum accumulates in fp64 and rounds
// each prefix: SURVEY.md App. B) out of LDS instead of a dependent global load per step.
__global__ void __launch_bounds__(64) k_sine_phase(const float* __restrict__ f0, int B, int n, int scale,
                                                   float* __restrict__ ph) {
  extern __shared__ float f0s[];
  const int b = blockIdx.x;
  for (int j = threadIdx.x; j < n; j += 64) f0s[j] = f0[(size_t)b * n + j];
  __syncthreads();
  const int h = threadIdx.x;
  if (h >= 9) return;
  const float hm = (float)(h + 1);
  const float pi_f = (float)3.14159265358979323846;
  const float sc = (float)scale;
  double cum = 0.0;
  float* out = ph + ((size_t)b * 9 + h) * n;
  for (int j = 0; j < n; ++j) {
    const float fn = f0s[j] * hm;
    float r = fn / 24000.0f;
    r = r - floorf(r);
    cum += (double)r;
    const float c = (float)cum;
    out[j] = ((c * 2.0f) * pi_f) * sc;
  }
}

__device__ __forceinline__ unsigned long long splitmix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

// counter RNG: N(0,1) keyed by (seed, global utterance, sample, harmonic) -> shard invariant
__device__ __forceinline__ float rng_normal(unsigned long long seed, long long utt, int t, int h) {
  const unsigned long long key = splitmix64(seed ^ splitmix64((unsigned long long)utt * 0x632BE59BD9B4E019ULL));
  const unsigned long long z = splitmix64(key + (unsigned long long)t * 9ULL + (unsigned long long)h);
  const float u1 = ((float)(z >> 40) + 0.5f) * (1.0f / 16777216.0f);
  const float u2 = (float)((z >> 16) & 0xFFFFFF) * (1.0f / 16777216.0f);
  return sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
}

// reference hifigan.py:155-157 (x scale linear upsample + sin), :189-218 (uv, noise),
// :254-264 (tanh(Linear 9->1)).  Upsample arithmetic follows PyTorch-CPU bit for bit:
// src = fma(1/scale, t+0.5, -0.5), out = fma(l0, x0, l1*x1).
__global__ void __launch_bounds__(256) k_sine_source(const float* __restrict__ f0, const float* __restrict__ ph,
                                                     int n, int scale, const float* __restrict__ lw,
                                                     const float* __restrict__ lb, const float* __restrict__ noise,
                                                     unsigned long long seed, long long utt_offset, float* har) {
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
#pragma unroll
  for (int h = 0; h < 9; ++h) {
    const float x0 = pb[h * n + i0], x1 = pb[h * n + i1];
    const float phase = fmaf(l0, x0, l1 * x1);
    const float sine = sinf(phase) * 0.1f;
    const float z = noise ? noise[((size_t)b * L + t) * 9 + h] : rng_normal(seed, utt_offset + b, t, h);
    const float sw = sine * uv + namp * z;
    acc = fmaf(lw[h], sw, acc);
  }
  har[(size_t)b * L + t] = tanhf(acc + lb[0]);
}

// ------------------------------------------------------------------ depthwise x2 ConvTranspose
// reference hifigan.py:373 (pool = ConvTranspose1d(C, C, 3, stride 2, groups=C, padding 1,
// output_padding 1)) applied after AdaIN(norm1) + LReLU(0.2) (hifigan.py:391-393).
template <typename T>
__global__ void __launch_bounds__(256) k_pool_dw(const T* __restrict__ x, long long x_bs, int x_ld, int Lin, int C,
                                                 const float* __restrict__ w, const float* __restrict__ bias,
                                                 Prologue pro, T* y, long long y_bs, int y_ld) {
  const int b = blockIdx.y;
  const int c = blockIdx.z * 256 + threadIdx.x;
  if (c >= C) return;
  float m = 0.f, a = 1.f, be = 0.f;
  if (pro.mode & PRO_AFFINE) adain_coeffs(pro, b, c, m, a, be);
  auto f = [&](int i) -> float {
    float v = to_f32(x[(size_t)b * x_bs + (size_t)i * x_ld + c]);
    if (pro.mode & PRO_AFFINE) v = (v - m) * a + be;
    if (pro.mode & PRO_LRELU) v = v > 0.f ? v : v * pro.slope;
    return v;
  };
  const float w0 = w[c * 3 + 0], w1 = w[c * 3 + 1], w2 = w[c * 3 + 2], bc = bias[c];
  const int rows = 16, i0 = blockIdx.x * rows;
  for (int i = i0; i < min(i0 + rows, Lin); ++i) {
    const float xi = f(i);
    // o = 2i:   k=1 from x[i]
    // o = 2i+1: k=0 from x[i+1] (if any) + k=2 from x[i]
    const float ve = xi * w1 + bc;
    float vo = xi * w2;
    if (i + 1 < Lin) vo = f(i + 1) * w0 + vo;
    vo = vo + bc;
    y[(size_t)b * y_bs + (size_t)(2 * i) * y_ld + c] = from_f32<T>(ve);
    y[(size_t)b * y_bs + (size_t)(2 * i + 1) * y_ld + c] = from_f32<T>(vo);
  }
}

// ------------------------------------------------------------------ style projections
// H[b][n] = bias[n] + sum_k s[b][k] * Wt[k][n]   (Wt packed [K][N] at load)
// H[b][n] = bias[n] + sum_k s[b][k] * Wt[k][n] for up to 32 utterances per block: 64 columns
// per block (one per lane), the 4 waves split K, the style rows sit in LDS, partial sums meet in LDS.
__global__ void __launch_bounds__(256) k_linear(const float* __restrict__ s, int B, int K,
                                                const float* __restrict__ Wt, const float* __restrict__ bias, int N,
                                                float* __restrict__ H) {
  extern __shared__ float ss[];  // [32][K] style rows, then [4][32][64] partial sums
  float* part = ss + 32 * K;
  const int b0 = blockIdx.y * 32, nb = min(32, B - b0);
  for (int i = threadIdx.x; i < 32 * K; i += 256) ss[i] = i < nb * K ? s[(size_t)b0 * K + i] : 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + lane;
  const int kq = (K + 3) / 4, k0 = wv * kq, k1 = min(K, k0 + kq);
  float acc[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) acc[i] = 0.f;
  if (n < N) {
#pragma unroll 4
    for (int k = k0; k < k1; ++k) {
      const float wv_ = Wt[(size_t)k * N + n];
#pragma unroll
      for (int i = 0; i < 32; ++i) acc[i] = fmaf(ss[i * K + k], wv_, acc[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < 32; ++i) part[(wv * 32 + i) * 64 + lane] = acc[i];
  __syncthreads();
  const float bv = (n < N && bias) ? bias[n] : 0.f;
  for (int i = wv; i < nb; i += 4) {
    const float h = part[(0 * 32 + i) * 64 + lane] + part[(1 * 32 + i) * 64 + lane] +
                    part[(2 * 32 + i) * 64 + lane] + part[(3 * 32 + i) * 64 + lane];
    if (n < N) H[(size_t)(b0 + i) * N + n] = h + bv;
  }
}

// ------------------------------------------------------------------ HiFi-GAN noise_convs
// Conv1d(1, C, K = 2S, stride S, padding P) over the harmonic source (hifigan.py:296-303).
// (a) small C*K (stages 1..3): one thread per (frame, 8 channels), weights in registers,
//     16-byte stores, statistics reduced in registers -> shuffles -> one atomic per channel.
template <typename T, int K>
__global__ void __launch_bounds__(256) k_noise_conv(const float* __restrict__ har, int L,
                                                    const float* __restrict__ w, const float* __restrict__ bias,
                                                    int C, int S, int P, int Lout, int fpb, T* __restrict__ y,
                                                    double* __restrict__ stats) {
  const int G = C >> 3;  // C % 8 == 0, 256 % G == 0
  const int b = blockIdx.y;
  const int g = threadIdx.x % G, fl = threadIdx.x / G, fstep = 256 / G;
  float wr[8][K], bb[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    bb[c] = bias ? bias[8 * g + c] : 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) wr[c][k] = w[(size_t)(8 * g + c) * K + k];
  }
  float sa[8], sq[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) sa[c] = sq[c] = 0.f;
  const float* hb = har + (size_t)b * L;
  T* yb = y + (size_t)b * Lout * C + 8 * g;
  const int f1 = min((blockIdx.x + 1) * fpb, Lout);
  for (int f = blockIdx.x * fpb + fl; f < f1; f += fstep) {
    float x[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = f * S - P + k;
      x[k] = (i >= 0 && i < L) ? hb[i] : 0.f;
    }
    float v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) a = fmaf(wr[c][k], x[k], a);
      v[c] = to_f32(from_f32<T>(a + bb[c]));  // statistics of the stored values
    }
    if constexpr (sizeof(T) == 2) {
      bf16x8 o;
#pragma unroll
      for (int c = 0; c < 8; ++c) o[c] = (bf16_t)v[c];
      *reinterpret_cast<bf16x8*>(yb + (size_t)f * C) = o;
    } else {
      *reinterpret_cast<float4*>(yb + (size_t)f * C) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(yb + (size_t)f * C + 4) = make_float4(v[4], v[5], v[6], v[7]);
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      sa[c] += v[c];
      sq[c] = fmaf(v[c], v[c], sq[c]);
    }
  }
  if (!stats) return;
  // lanes l, l+G, l+2G, ... of a wave share g; then the 4 waves combine in LDS and ONE atomic
  // pair per (block, channel) goes out (same-line atomics from many blocks serialise in L2)
  __shared__ float red[4][2][256];
#pragma unroll
  for (int c = 0; c < 8; ++c)
    for (int o = G; o < 64; o <<= 1) {
      sa[c] += __shfl_xor(sa[c], o);
      sq[c] += __shfl_xor(sq[c], o);
    }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) < G) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      red[wv][0][8 * g + c] = sa[c];
      red[wv][1][8 * g + c] = sq[c];
    }
  }
  __syncthreads();
  if (threadIdx.x < C) {
    const int c = threadIdx.x;
    const double a = (double)red[0][0][c] + red[1][0][c] + red[2][0][c] + red[3][0][c];
    const double q = (double)red[0][1][c] + red[1][1][c] + red[2][1][c] + red[3][1][c];
    atomic_stats(stats + ((size_t)b * C + c) * ST_W, a, q);
  }
}

// (b) large C*K (stage 0, K = 60): the source is cut into S-sample frames,
//     X[r][j] = har[S*r - P + j] (j < S, zero-padded to ld channels), so the strided conv is a
//     2-tap stride-1 conv with Cin = S that runs on the MFMA engine (weights: k_reframe_w).
template <typename T>
__global__ void __launch_bounds__(256) k_har_frames(const float* __restrict__ har, int L, int S, int P, int rows,
                                                    int ld, T* __restrict__ x) {
  const int b = blockIdx.y;
  const int gpr = ld >> 3;
  const long long u = (long long)blockIdx.x * 256 + threadIdx.x;
  if (u >= (long long)rows * gpr) return;
  const int r = (int)(u / gpr), j0 = (int)(u % gpr) * 8;
  const float* hb = har + (size_t)b * L;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int i = r * S - P + j0 + j;
    v[j] = (j0 + j < S && i >= 0 && i < L) ? hb[i] : 0.f;
  }
  T* dst = x + ((size_t)b * rows + r) * ld + j0;
#pragma unroll
  for (int j = 0; j < 8; ++j) dst[j] = from_f32<T>(v[j]);
}

// w [C][1][2S] (nn.Conv1d) -> w' [C][S][2]: w'[c][j][t] = w[c][t*S + j]
__global__ void k_reframe_w(const float* __restrict__ w, int C, int S, float* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= C * S * 2) return;
  const int t = i % 2, j = (i / 2) % S, c = i / (2 * S);
  out[i] = w[(size_t)c * 2 * S + t * S + j];
}

// ------------------------------------------------------------------ column statistics
template <typename T>
__global__ void __launch_bounds__(256) k_frames_stats(const T* __restrict__ x, long long x_bs, int x_ld, int L, int c0,
                                                      int C, double* stats, int stats_ld) {
  const int b = blockIdx.y, c = blockIdx.z * 256 + threadIdx.x;
  if (c >= C) return;
  const int rows = 256, r0 = blockIdx.x * rows;
  double a = 0, q = 0;
  for (int r = r0; r < min(r0 + rows, L); ++r) {
    const float v = to_f32(x[(size_t)b * x_bs + (size_t)r * x_ld + c0 + c]);
    a += v;
    q += (double)v * v;
  }
  atomic_stats(stats + ((size_t)b * stats_ld + c0 + c) * ST_W, a, q);
}

// ------------------------------------------------------------------ CustomSTFT
// reference istftnet.py:207-243: replicate pad n_fft/2, DFT-as-conv stride hop,
// mag = sqrt(re^2 + im^2 + 1e-14), phase = atan2(im, re) with (im==0 & re<0) -> pi.
template <typename T>
__global__ void __launch_bounds__(256) k_stft(const float* __restrict__ wave, int L, int n_fft, int hop,
                                              const float* __restrict__ wr, const float* __restrict__ wi, int F, T* y,
                                              int ld) {
  const int nb = n_fft / 2 + 1;
  const int b = blockIdx.y;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= F * nb) return;
  const int f = idx / nb, k = idx % nb;
  const int pad = n_fft / 2;
  const float* wb = wave + (size_t)b * L;
  float re = 0.f, im = 0.f;
  for (int n = 0; n < n_fft; ++n) {
    int g = f * hop + n - pad;
    g = g < 0 ? 0 : (g >= L ? L - 1 : g);
    const float xv = wb[g];
    re = fmaf(xv, wr[k * n_fft + n], re);
    im = fmaf(xv, wi[k * n_fft + n], im);
  }
  const float mag = sqrtf(re * re + im * im + 1e-14f);
  float phase = atan2f(im, re);
  if (im == 0.f && re < 0.f) phase = 3.14159265358979323846f;
  T* yr = y + ((size_t)b * F + f) * ld;
  yr[k] = from_f32<T>(mag);
  yr[nb + k] = from_f32<T>(phase);
}

// reference istftnet.py:571-573 + 246-293: spec = exp(x[:nb]), phase = sin(x[nb:]);
// re = spec*cos(phase), im = spec*sin(phase); wave = convT(re, Br) - convT(im, Bi), trim n_fft/2.
template <typename T>
__global__ void __launch_bounds__(256) k_istft(const T* __restrict__ post, int F, int ld, int n_fft, int hop,
                                               const float* __restrict__ br, const float* __restrict__ bi, float* out,
                                               int L) {
  const int nb = n_fft / 2 + 1;
  const int b = blockIdx.y;
  const int m = blockIdx.x * 256 + threadIdx.x;
  if (m >= L) return;
  const int pos = m + n_fft / 2;
  int flo = pos - n_fft + 1;
  flo = flo <= 0 ? 0 : (flo + hop - 1) / hop;
  int fhi = pos / hop;
  if (fhi > F - 1) fhi = F - 1;
  float rr = 0.f, ii = 0.f;
  for (int f = flo; f <= fhi; ++f) {
    const int kk = pos - f * hop;
    const T* xr = post + ((size_t)b * F + f) * ld;
    for (int k = 0; k < nb; ++k) {
      const float sp = expf(to_f32(xr[k]));
      const float phs = sinf(to_f32(xr[nb + k]));
      rr = fmaf(sp * cosf(phs), br[k * n_fft + kk], rr);
      ii = fmaf(sp * sinf(phs), bi[k * n_fft + kk], ii);
    }
  }
  out[(size_t)b * L + m] = rr - ii;
}

// ------------------------------------------------------------------ weight prep
__global__ void __launch_bounds__(256) k_wn_fold(const float* __restrict__ v, const float* __restrict__ g, int inner,
                                                 float* wout) {
  __shared__ double red[256];
  const int row = blockIdx.x;
  const float* vr = v + (size_t)row * inner;
  double a = 0;
  for (int i = threadIdx.x; i < inner; i += 256) a += (double)vr[i] * vr[i];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  const float factor = g ? g[row] / (float)sqrt(red[0]) : 1.0f;
  for (int i = threadIdx.x; i < inner; i += 256) wout[(size_t)row * inner + i] = vr[i] * factor;
}

template <typename MT>
__global__ void __launch_bounds__(256) k_pack_conv(const float* __restrict__ w, int Cin, int Cout, int K,
                                                   int transposed, int u, int taps, int nchunks, int N, int Np,
                                                   MT* out, MT* out_lo) {
  const size_t total = (size_t)nchunks * taps * 32 * Np;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  int c, tap, n, kl;
  if (std::is_same<MT, bf16_t>::value) {  // [chunk][tap][Np][32], 16-B units XOR-swizzled by (n>>2)&3
    const int kp = (int)(i % 32);
    size_t r = i / 32;
    n = (int)(r % Np);
    r /= Np;
    tap = (int)(r % taps);
    c = (int)(r / taps);
    kl = 8 * ((kp >> 3) ^ ((n >> 2) & 3)) + (kp & 7);  // physical unit kp>>3 holds logical unit kl>>3
  } else {  // [chunk][tap][32][Np]
    n = (int)(i % Np);
    size_t r = i / Np;
    kl = (int)(r % 32);
    r /= 32;
    tap = (int)(r % taps);
    c = (int)(r / taps);
  }
  // row permutation inside each 32-block: packed row m holds column 16*((m>>2)&1) + (m&3) + 4*(m>>3),
  // so the transposed MFMA output (C^T = W^T X^T) gives each lane 16 consecutive columns
  {
    const int m = n & 31;
    n = (n & ~31) + 16 * ((m >> 2) & 1) + (m & 3) + 4 * (m >> 3);
  }
  const int ci = c * 32 + kl;
  float val = 0.f;
  if (ci < Cin && n < N) {
    if (!transposed) {
      val = w[((size_t)n * Cin + ci) * K + tap];
    } else {
      const int p = n / Cout, co = n % Cout;
      const int k = p + (taps - 1 - tap) * u;
      if (k < K) val = w[((size_t)ci * Cout + co) * K + k];
    }
  }
  out[i] = (MT)val;
  if (out_lo) out_lo[i] = (MT)(val - (float)(MT)val);  // ST_SPLIT: the bf16 rounding residual (exact in fp32)
}


// ------------------------------------------------------------------ style encoder (models.py:13-150)
__device__ __forceinline__ size_t prow(int h, int w, int W) { return (size_t)h * (W + 2) + w; }

template <typename T>
__global__ void __launch_bounds__(256) k_mel_to_padded(const float* __restrict__ mel, int H, int W, T* dst) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= H * W) return;
  const int h = i / W, w = i % W;
  dst[((size_t)b * (H + 2) * (W + 2) + prow(h + 1, w + 1, W)) * 8] = from_f32<T>(mel[(size_t)b * H * W + i]);
}

// reference models.py:23 LearnedDownSample('half'): depthwise Conv2d k3 s2 p1 (+bias)
template <typename T>
__global__ void __launch_bounds__(256) k_dw_s2(const T* __restrict__ x, int H, int W, int C,
                                               const float* __restrict__ w, const float* __restrict__ bias, T* y) {
  const int b = blockIdx.z;
  const int Ho = H / 2, Wo = (W + 1) / 2;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)Ho * Wo * C) return;
  const int c = (int)(i % C);
  const size_t pix = i / C;
  const int oi = (int)(pix / Wo), oj = (int)(pix % Wo);
  const T* xb = x + (size_t)b * (H + 2) * (W + 2) * C;
  float acc = 0.f;
#pragma unroll
  for (int dy = 0; dy < 3; ++dy)
#pragma unroll
    for (int dx = 0; dx < 3; ++dx)
      acc = fmaf(w[c * 9 + dy * 3 + dx], to_f32(xb[prow(2 * oi + dy, 2 * oj + dx, W) * C + c]), acc);
  y[((size_t)b * (Ho + 2) * (Wo + 2) + prow(oi + 1, oj + 1, Wo)) * C + c] = from_f32<T>(acc + bias[c]);
}

// reference models.py:58-61 DownSample('half'): odd width -> repeat last column; avg_pool2d(2)
template <typename T>
__global__ void __launch_bounds__(256) k_avgpool_half(const T* __restrict__ x, int H, int W, int C, T* y) {
  const int b = blockIdx.z;
  const int Ho = H / 2, Wo = (W + 1) / 2;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)Ho * Wo * C) return;
  const int c = (int)(i % C);
  const size_t pix = i / C;
  const int oi = (int)(pix / Wo), oj = (int)(pix % Wo);
  const T* xb = x + (size_t)b * (H + 2) * (W + 2) * C;
  const int c0 = 2 * oj, c1 = (2 * oj + 1 < W) ? 2 * oj + 1 : W - 1;  // unpadded columns
  const float a00 = to_f32(xb[prow(2 * oi + 1, c0 + 1, W) * C + c]);
  const float a01 = to_f32(xb[prow(2 * oi + 1, c1 + 1, W) * C + c]);
  const float a10 = to_f32(xb[prow(2 * oi + 2, c0 + 1, W) * C + c]);
  const float a11 = to_f32(xb[prow(2 * oi + 2, c1 + 1, W) * C + c]);
  y[((size_t)b * (Ho + 2) * (Wo + 2) + prow(oi + 1, oj + 1, Wo)) * C + c] = from_f32<T>((((a00 + a01) + a10) + a11) / 4.0f);
}

// reference models.py:139-148: AdaptiveAvgPool2d(1) -> LeakyReLU(0.2) -> view -> Linear
template <typename T>
__global__ void __launch_bounds__(256) k_gap_linear(const T* __restrict__ z, int rows, int Wv, int C,
                                                    const float* __restrict__ w, const float* __restrict__ bias, int N,
                                                    float* out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* h = reinterpret_cast<float*>(smem);
  const int b = blockIdx.x;
  const T* zb = z + (size_t)b * rows * C;
  for (int c = threadIdx.x; c < C; c += 256) {
    float a = 0.f;
    for (int r = 0; r < Wv; ++r) a += to_f32(zb[(size_t)r * C + c]);
    a = a / (float)Wv;
    h[c] = a > 0.f ? a : 0.2f * a;
  }
  __syncthreads();
  for (int n = threadIdx.x; n < N; n += 256) {
    float a = 0.f;
    for (int c = 0; c < C; ++c) a = fmaf(w[(size_t)n * C + c], h[c], a);
    out[(size_t)b * N + n] = a + bias[n];
  }
}

}  // namespace

// ================================================================== launchers
int st_ncl_to_frames(const float* src, int B, int C, int L, void* dst, int ld, int c0, long long dst_bs,
                     double* stats, int stats_ld, int dtype, hipStream_t s) {
  dim3 grid((L + 63) / 64, (C + 63) / 64, B);
  DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_ncl_to_frames<T>, grid, dim3(256), 0, s, src, C, L,
                                              reinterpret_cast<T*>(dst), ld, c0, dst_bs, stats, stats_ld));
  return (int)hipGetLastError();
}

int st_frames_convert(const float* src, int B, int L, int C, int ld_in, void* dst, int ld_out, double* stats,
                      int stats_ld, int dtype, hipStream_t s) {
  if (dtype == ST_BF16 && !stats && ld_out % 8 == 0) {
    const long long n = (long long)B * L * (ld_out / 8);
    hipLaunchKernelGGL(k_cvt_bf16_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, (long long)B * L, C,
                       ld_in, reinterpret_cast<bf16_t*>(dst), ld_out);
    return (int)hipGetLastError();
  }
  dim3 grid((L + 63) / 64, B, (C + 255) / 256);
  DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_frames_convert<T>, grid, dim3(256), 0, s, src, L, C, ld_in,
                                              reinterpret_cast<T*>(dst), ld_out, stats, stats_ld));
  return (int)hipGetLastError();
}

// DiscriminatorP 1-d -> 2-d (Modules/discriminators.py:112-118): the waveform reflect-padded on the
// right to a multiple of the period p and viewed [B, 1, T/p, p]; its (k, 1) convs run along T/p
// for every column j, so column j of utterance b becomes frames row b*p + j: [B*p][L0][8]
// (channel 0 = the sample, channels 1..7 zero: the frames layout pads channels to 8)
template <typename T>
__global__ void __launch_bounds__(256) k_period_frames(const float* __restrict__ wave, int Tn, int p, int L0,
                                                       long long rows, T* __restrict__ dst) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * L0) return;
  const long long r = i / L0;
  const int t = (int)(i - r * L0);
  const int b = (int)(r / p), j = (int)(r - (long long)b * p);
  int k = t * p + j;
  if (k >= Tn) k = 2 * (Tn - 1) - k;  // F.pad(..., "reflect") on the right
  T o[8];
  o[0] = from_f32<T>(wave[(size_t)b * Tn + k]);
#pragma unroll
  for (int c = 1; c < 8; ++c) o[c] = from_f32<T>(0.f);
#pragma unroll
  for (int c = 0; c < 8; ++c) dst[i * 8 + c] = o[c];
}

int st_period_frames(const float* wave, int B, int Tn, int p, int L0, void* dst, int dtype, hipStream_t s) {
  if (B <= 0 || Tn <= 0 || p <= 0 || L0 * p < Tn || L0 * p - Tn >= Tn) return ST_EINVAL;
  const long long rows = (long long)B * p, n = rows * L0;
  dim3 grid((unsigned)((n + 255) / 256));
  DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_period_frames<T>, grid, dim3(256), 0, s, wave, Tn, p, L0, rows,
                                              reinterpret_cast<T*>(dst)));
  return (int)hipGetLastError();
}

// GAN losses over the MPD outputs (losses.py:97-128): each (period, layer) block of the engine's
// output holds the real half then the generated half (same element order), so
//   feature_loss = 2 sum_blocks mean|r - g|,  generator_loss = sum_periods mean((1 - g)^2),
//   discriminator_loss = sum_periods mean((1 - r)^2) + mean(g^2)   (scores = the conv_post blocks)
// Per-block sums: fp32 per thread, fp64 per workgroup, written as per-(segment, block) partials;
// k_mpd_loss_final adds the blocks of each segment in block order (deterministic run to run).

__global__ void __launch_bounds__(256) k_mpd_loss_sums(const float* __restrict__ out, MpdLossSegs sg,
                                                       double* __restrict__ part) {
  const int seg = blockIdx.y;
  if (seg >= sg.n) return;
  const long long half = sg.half[seg];
  const float* r = out + sg.off[seg];
  const float* g = r + half;
  float a = 0.f, q1 = 0.f, q2 = 0.f, q3 = 0.f;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < half; i += (long long)gridDim.x * 256) {
    const float x = r[i], y = g[i];
    a += fabsf(x - y);
    if (sg.score[seg]) {
      q1 += (1.f - x) * (1.f - x);
      q2 += (1.f - y) * (1.f - y);
      q3 += y * y;
    }
  }
  float v[4] = {a, q1, q2, q3};
  __shared__ float red[4][4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    for (int o = 32; o >= 1; o >>= 1) v[k] += __shfl_xor(v[k], o);
    if ((threadIdx.x & 63) == 0) red[k][threadIdx.x >> 6] = v[k];
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const int k = threadIdx.x;
    part[((size_t)seg * kMpdLossBlocks + blockIdx.x) * 4 + k] =
        (((double)red[k][0] + red[k][1]) + red[k][2]) + red[k][3];
  }
}

__global__ void k_mpd_loss_final(MpdLossSegs sg, const double* __restrict__ part, double* __restrict__ loss) {
  double fm = 0, gen = 0, disc = 0;
  for (int s = 0; s < sg.n; ++s) {
    double sums[4] = {0.0, 0.0, 0.0, 0.0};
    for (int j = 0; j < kMpdLossBlocks; ++j)
      for (int k = 0; k < 4; ++k) sums[k] += part[((size_t)s * kMpdLossBlocks + j) * 4 + k];
    const double n = (double)sg.half[s];
    fm += sums[0] / n;
    if (sg.score[s]) {
      gen += sums[2] / n;
      disc += (sums[1] + sums[3]) / n;
    }
  }
  loss[0] = 2.0 * fm;
  loss[1] = gen;
  loss[2] = disc;
}

int st_mpd_losses(const float* out, const MpdLossSegs& sg, double* part, double* loss, hipStream_t s) {
  if (sg.n <= 0 || sg.n > kMpdMaxSegs) return ST_EINVAL;
  hipLaunchKernelGGL(k_mpd_loss_sums, dim3(kMpdLossBlocks, sg.n), dim3(256), 0, s, out, sg, part);
  ST_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_mpd_loss_final, dim3(1), dim3(1), 0, s, sg, part, loss);
  return (int)hipGetLastError();
}

namespace {
// the resblock average of the concurrent branches (decoder_forward at small batches): acc = ((acc + r0) + r1 ...)
// / div in the running-sum epilogues' order; bf16 storage rounds each partial sum and divides by a reciprocal
// multiply, as the bf16 epilogues do (fp32: bit-identical to the running sum)
struct BranchRs {
  const void* r[4];
};
template <typename T>
__global__ void __launch_bounds__(256) k_branch_avg(T* __restrict__ acc, BranchRs rs, int nr, float div, long long n) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float a = to_f32(acc[i]);
  for (int j = 0; j < nr; ++j) {
    const float v = to_f32(reinterpret_cast<const T*>(rs.r[j])[i]);
    if (j + 1 < nr)
      a = to_f32(from_f32<T>(a + v));
    else if (std::is_same<T, float>::value)
      a = (a + v) / div;
    else
      a = (a + v) * (1.0f / div);
  }
  acc[i] = from_f32<T>(a);
}
}  // namespace

int g_opt_nbranch = 64;  // STTS_OPT_NBRANCH: the noise branches alone on a side stream up to this batch
int g_opt_branches = 8;  // STTS_OPT_BRANCHES (plan.cpp decoder_forward): concurrent resblocks up to this batch

int st_branch_avg(void* acc, const void* const* rs, int nr, float div, long long n, int dtype, hipStream_t s) {
  if (nr < 1 || nr > 4 || n < 0) return ST_EINVAL;
  BranchRs r = {};
  for (int j = 0; j < nr; ++j) r.r[j] = rs[j];
  const unsigned grid = (unsigned)((n + 255) / 256);
  if (!grid) return 0;
  DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_branch_avg<T>, dim3(grid), dim3(256), 0, s, reinterpret_cast<T*>(acc), r,
                                              nr, div, n));
  return (int)hipGetLastError();
}

int st_frames_to_f32(const void* src, int B, int L, int C, int ld, float* dst, int dtype, hipStream_t s) {
  if (dtype == ST_BF16 && C % 8 == 0 && ld % 8 == 0) {
    const long long n = (long long)B * L * (C / 8);
    hipLaunchKernelGGL(k_cvt_f32_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<const bf16_t*>(src), (long long)B * L, C, ld, dst);
    return (int)hipGetLastError();
  }
  dim3 grid((unsigned)(((size_t)L * C + 255) / 256), B);
  DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_frames_to_f32<T>, grid, dim3(256), 0, s,
                                              reinterpret_cast<const T*>(src), L, C, ld, dst));
  return (int)hipGetLastError();
}

int st_conv_cin1(const float* in, long long in_bs, int Lin, int B, const float* w, const float* bias, int C, int K,
                 int stride, int pad, int Lout, const SmallConvDst* dst, int ndst, int dtype, hipStream_t s) {
  if (ndst < 1 || ndst > 3 || C <= 0 || K <= 0) return ST_EINVAL;
  SmallConvDst d[3] = {dst[0], ndst > 1 ? dst[1] : dst[0], ndst > 2 ? dst[2] : dst[0]};
  if (ndst < 3) d[2].stats = nullptr;
  if (ndst < 2) d[1].stats = nullptr;
  const int nwin = (C1_TT - 1) * stride + K;
  const bool generic = !(K == 1 || K == 3 || K == 4 || K == 12 || K == 60);
  const size_t lds = ((nwin + 3) & ~3) * sizeof(float) + (generic ? ((C * K + 3) & ~3) * sizeof(float) : 0) +
                     256 * 2 * sizeof(double);
  if (lds > 160 * 1024) return ST_EINVAL;
  dim3 grid((Lout + C1_TT - 1) / C1_TT, B);
#define CIN1(KC)                                                                                                 \
  DISPATCH_DTYPE(dtype, T, {                                                                                     \
    auto kern = k_conv_cin1<T, KC>;                                                                              \
    if (lds > 64 * 1024)                                                                                         \
      ST_CHECK_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024)); \
    hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, in, in_bs, Lin, w, bias, C, K, stride, pad, Lout, d[0], d[1], \
                       d[2], ndst);                                                                              \
  })
  switch (K) {
    case 1: CIN1(1); break;
    case 3: CIN1(3); break;
    case 4: CIN1(4); break;
    case 12: CIN1(12); break;
    case 60: CIN1(60); break;
    default: CIN1(0); break;
  }
#undef CIN1
  return (int)hipGetLastError();
}

int st_sine_phase(const float* f0, int B, int n, int scale, float* ph, hipStream_t s) {
  const size_t lds = (size_t)n * 4;
  if (lds > 64 * 1024) {
    if (lds > 160 * 1024) return ST_EINVAL;
    ST_CHECK_HIP(hipFuncSetAttribute((const void*)k_sine_phase, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  }
  hipLaunchKernelGGL(k_sine_phase, dim3(B), dim3(64), lds, s, f0, B, n, scale, ph);
  return (int)hipGetLastError();
}

int st_sine_source(const float* f0, const float* ph, int B, int n, int scale, const float* lw, const float* lb,
                   const float* noise, unsigned long long seed, long long utt_offset, float* har, hipStream_t s) {
  const int L = n * scale;
  hipLaunchKernelGGL(k_sine_source, dim3((L + 255) / 256, B), dim3(256), 0, s, f0, ph, n, scale, lw, lb, noise, seed,
                     utt_offset, har);
  return (int)hipGetLastError();
}

int st_pool_dw(const void* x, long long x_bs, int x_ld, int B, int Lin, int C, const float* w, const float* bias,
               const Prologue& pro, void* y, long long y_bs, int y_ld, int dtype, hipStream_t s) {
  dim3 grid((Lin + 15) / 16, B, (C + 255) / 256);
  DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_pool_dw<T>, grid, dim3(256), 0, s, reinterpret_cast<const T*>(x),
                                              x_bs, x_ld, Lin, C, w, bias, pro, reinterpret_cast<T*>(y), y_bs, y_ld));
  return (int)hipGetLastError();
}

int st_linear(const float* s, int B, int K, const float* Wt, const float* bias, int N, float* H, hipStream_t st) {
  const size_t lds = ((size_t)32 * K + 4 * 32 * 64) * 4;
  if (lds > 64 * 1024) return ST_EINVAL;
  hipLaunchKernelGGL(k_linear, dim3((N + 63) / 64, (B + 31) / 32), dim3(256), lds, st, s, B, K, Wt, bias, N, H);
  return (int)hipGetLastError();
}

int st_frames_stats(const void* x, long long x_bs, int x_ld, int B, int L, int c0, int C, double* stats, int stats_ld,
                    int dtype, hipStream_t s) {
  dim3 grid((L + 255) / 256, B, (C + 255) / 256);
  DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_frames_stats<T>, grid, dim3(256), 0, s,
                                              reinterpret_cast<const T*>(x), x_bs, x_ld, L, c0, C, stats, stats_ld));
  return (int)hipGetLastError();
}

int st_stft(const float* wave, int B, int L, int n_fft, int hop, const float* wr, const float* wi, void* y, int ld,
            int dtype, hipStream_t s) {
  const int F = L / hop + 1;
  const int nb = n_fft / 2 + 1;
  dim3 grid((F * nb + 255) / 256, B);
  DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_stft<T>, grid, dim3(256), 0, s, wave, L, n_fft, hop, wr, wi, F,
                                              reinterpret_cast<T*>(y), ld));
  return (int)hipGetLastError();
}

int st_istft(const void* post, int B, int F, int ld, int n_fft, int hop, const float* br, const float* bi, float* out,
             int L, int dtype, hipStream_t s) {
  dim3 grid((L + 255) / 256, B);
  DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_istft<T>, grid, dim3(256), 0, s, reinterpret_cast<const T*>(post), F,
                                              ld, n_fft, hop, br, bi, out, L));
  return (int)hipGetLastError();
}

__global__ void k_stats_decode(const double* __restrict__ fx, long long n, double* __restrict__ out) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  out[2 * i] = fx_get(fx + i * ST_W);
  out[2 * i + 1] = fx_get(fx + i * ST_W + 2);
}

int st_stats_decode(const double* fx, long long n, double* out, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_stats_decode, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, fx, n, out);
  return (int)hipGetLastError();
}

int st_stats_fold(double* stats, int B, int ld, int C, int slots, long long slot_bs, hipStream_t s) {
  if (slots <= 1 || B * C == 0) return 0;
  hipLaunchKernelGGL(k_stats_fold, dim3((B * C + 255) / 256), dim3(256), 0, s, stats, B, ld, C, slots, slot_bs);
  return (int)hipGetLastError();
}

int st_wn_fold(const float* v, const float* g, int d0, int inner, float* wout, hipStream_t s) {
  hipLaunchKernelGGL(k_wn_fold, dim3(d0), dim3(256), 0, s, v, g, inner, wout);
  return (int)hipGetLastError();
}

size_t st_packed_conv_elems(int Cin, int Cout, int K, int transposed, int u) {
  const int taps = transposed ? (K + u - 1) / u : K;
  const int N = transposed ? u * Cout : Cout;
  const int Np = (N + 31) & ~31;
  const int nchunks = (Cin + 31) / 32;
  return (size_t)nchunks * taps * 32 * Np;
}

int st_pack_conv(const float* w, int Cin, int Cout, int K, int transposed, int u, void* out, int dtype,
                 hipStream_t s) {
  const int taps = transposed ? (K + u - 1) / u : K;
  const int N = transposed ? u * Cout : Cout;
  const int Np = (N + 31) & ~31;
  const int nchunks = (Cin + 31) / 32;
  const size_t total = st_packed_conv_elems(Cin, Cout, K, transposed, u);
  dim3 grid((unsigned)((total + 255) / 256));
  if (dtype == ST_FP32)
    hipLaunchKernelGGL(k_pack_conv<float>, grid, dim3(256), 0, s, w, Cin, Cout, K, transposed, u, taps, nchunks, N, Np,
                       reinterpret_cast<float*>(out), (float*)nullptr);
  else if (dtype == ST_BF16)
    hipLaunchKernelGGL(k_pack_conv<bf16_t>, grid, dim3(256), 0, s, w, Cin, Cout, K, transposed, u, taps, nchunks, N,
                       Np, reinterpret_cast<bf16_t*>(out), (bf16_t*)nullptr);
  else if (dtype == ST_SPLIT)  // bf16 layout, the hi parts then the lo parts (same bytes as fp32)
    hipLaunchKernelGGL(k_pack_conv<bf16_t>, grid, dim3(256), 0, s, w, Cin, Cout, K, transposed, u, taps, nchunks, N,
                       Np, reinterpret_cast<bf16_t*>(out), reinterpret_cast<bf16_t*>(out) + total);
  else
    return ST_EDTYPE;
  return (int)hipGetLastError();
}

int st_mel_to_padded(const float* mel, int B, int H, int W, void* dst, int dtype, hipStream_t s) {
  dim3 grid((H * W + 255) / 256, B);
  DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_mel_to_padded<T>, grid, dim3(256), 0, s, mel, H, W,
                                              reinterpret_cast<T*>(dst)));
  return (int)hipGetLastError();
}

int st_dw_s2(const void* x, int B, int H, int W, int C, const float* w, const float* bias, void* y, int dtype,
             hipStream_t s) {
  const size_t n = (size_t)(H / 2) * ((W + 1) / 2) * C;
  dim3 grid((unsigned)((n + 255) / 256), 1, B);
  DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_dw_s2<T>, grid, dim3(256), 0, s, reinterpret_cast<const T*>(x), H, W,
                                              C, w, bias, reinterpret_cast<T*>(y)));
  return (int)hipGetLastError();
}

int st_avgpool_half(const void* x, int B, int H, int W, int C, void* y, int dtype, hipStream_t s) {
  const size_t n = (size_t)(H / 2) * ((W + 1) / 2) * C;
  dim3 grid((unsigned)((n + 255) / 256), 1, B);
  DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_avgpool_half<T>, grid, dim3(256), 0, s,
                                              reinterpret_cast<const T*>(x), H, W, C, reinterpret_cast<T*>(y)));
  return (int)hipGetLastError();
}

int st_gap_linear(const void* z, int B, int rows, int Wv, int C, const float* w, const float* bias, int N, float* out,
                  int dtype, hipStream_t s) {
  DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_gap_linear<T>, dim3(B), dim3(256), C * sizeof(float), s,
                                              reinterpret_cast<const T*>(z), rows, Wv, C, w, bias, N, out));
  return (int)hipGetLastError();
}

int st_noise_conv(const float* har, int B, int L, const float* w, const float* bias, int C, int K, int S, int P,
                  int Lout, void* y, double* stats, int dtype, hipStream_t s) {
  if (C % 8 || 256 % (C / 8) || C > 256) return ST_EINVAL;
  // frames per block: about 2048 blocks over a 32-utterance batch (8 per CU), a multiple of the frames one
  // block covers per pass (256 / (C/8)); statistics cost one atomic pair per (block, channel).  From Lout alone,
  // not B, so each block's fp32 partial covers the same frames at every batch size (rank-count invariance, §8(e))
  const int fstep = 256 / (C / 8);
  long long fpb = ((long long)Lout * 32 + 2047) / 2048;
  fpb = (fpb + fstep - 1) / fstep * fstep;
  if (fpb < fstep) fpb = fstep;
  if (fpb > 8192) fpb = 8192;
  dim3 grid((unsigned)((Lout + fpb - 1) / fpb), B);
#define NCONV(KC)                                                                                              \
  DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((k_noise_conv<T, KC>), grid, dim3(256), 0, s, har, L, w, bias, C, S, \
                                              P, Lout, (int)fpb, reinterpret_cast<T*>(y), stats))
  switch (K) {
    case 1: NCONV(1); break;
    case 4: NCONV(4); break;
    case 12: NCONV(12); break;
    default: return ST_EINVAL;
  }
#undef NCONV
  return (int)hipGetLastError();
}

int st_har_frames(const float* har, int B, int L, int S, int P, int rows, int ld, void* x, int dtype, hipStream_t s) {
  if (ld % 8 || S > ld) return ST_EINVAL;
  const long long units = (long long)rows * (ld / 8);
  dim3 grid((unsigned)((units + 255) / 256), B);
  DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_har_frames<T>, grid, dim3(256), 0, s, har, L, S, P, rows, ld,
                                              reinterpret_cast<T*>(x)));
  return (int)hipGetLastError();
}

int st_reframe_w(const float* w, int C, int S, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_reframe_w, dim3((C * S * 2 + 255) / 256), dim3(256), 0, s, w, C, S, out);
  return (int)hipGetLastError();
}

// A stride-s Conv1d weight w [Cout][Cin][K] (padding pad) as the stride-1 conv over phase-folded frames
// (s consecutive input rows side by side, s Cin channels): out [Cout][s Cin][K2] with
// out[co][ph Cin + ci][k2] = w[co][ci][s (k2 - pad2) + ph + pad] (0 outside [0, K)).  MSD's stride-2 layers
// (plan.cpp msd_forward) run folded, on the stride-1 N = 32 conv tiles.
__global__ void k_fold_w(const float* __restrict__ w, int Cout, int Cin, int K, int st, int pad, int K2, int pad2,
                         float* __restrict__ out) {
  const long long n = (long long)Cout * st * Cin * K2;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int k2 = (int)(i % K2);
  const long long r = i / K2;
  const int cp = (int)(r % (st * Cin)), co = (int)(r / (st * Cin));
  const int ph = cp / Cin, ci = cp - ph * Cin;
  const int t = st * (k2 - pad2) + ph + pad;
  out[i] = (t >= 0 && t < K) ? w[((size_t)co * Cin + ci) * K + t] : 0.f;
}

int st_fold_w(const float* w, int Cout, int Cin, int K, int st, int pad, int K2, int pad2, float* out, hipStream_t s) {
  const long long n = (long long)Cout * st * Cin * K2;
  hipLaunchKernelGGL(k_fold_w, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, w, Cout, Cin, K, st, pad, K2, pad2,
                     out);
  return (int)hipGetLastError();
}
