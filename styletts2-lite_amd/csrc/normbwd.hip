// AdaIN1d + activation, forward and backward, and the style Linear's backward: the normalisation
// layers of the training step's decoder backward (config 5; train.py:272-327 backpropagates through
// Modules/hifigan.py's AdaIN1d (:14-24) + Snake (:68) in AdaINResBlock1 and AdaIN1d + LeakyReLU(0.2)
// in AdainResBlk1d (:359-403)).
//
//   z = (1 + gamma[b][c]) * (x - mean[b][c]) * rstd[b][c] + beta[b][c]      (InstanceNorm, eps 1e-5)
//   y = act(z): 0 identity, 1 Snake z + sin^2(alpha_c z) / alpha_c, 2 LeakyReLU(0.2)
//
// backward with dz = dy * act'(z), xhat = (x - mean) * rstd, over the L frames of (b, c):
//   dgamma = sum dz * xhat, dbeta = sum dz
//   dx = (1 + gamma) rstd (dz - dbeta / L - xhat dgamma / L)
//   dalpha_c = sum_(b,t) dy (z sin(2 alpha z) / alpha - sin^2(alpha z) / alpha^2)
// Frames layout [B][L][C] fp32.  Column sums: a workgroup = 64 channels x 4 row lanes over one row
// slice of one utterance writes fp64 partials; a per-channel pass adds the slices in order
// (deterministic).
#include <hip/hip_runtime.h>
#include <math.h>
#include <string.h>

#include <algorithm>

#include "../../include/stts2.h"
#include "common.h"
#include "kernels.h"

namespace {

constexpr double kEps = 1e-5;
constexpr float kSlope = 0.2f;

struct Cols {
  int S;  // row slices per utterance
};

Cols cols_of(int B, int L, int C) {
  const int cblk = (C + 63) / 64;
  long long S = (2048 + (long long)B * cblk - 1) / ((long long)B * cblk);
  S = std::min<long long>(S, std::max(1, L / 16));
  Cols c;
  c.S = (int)std::max<long long>(1, std::min<long long>(S, 1024));
  return c;
}

__device__ __forceinline__ float act_fwd(float z, int act, float a) {
  if (act == 1) {
    const float sn = sinf(a * z);
    return z + sn * sn / a;
  }
  if (act == 2) return z > 0.f ? z : kSlope * z;
  return z;
}

// (slice, b) rows of 64 channels: sums of x and x^2
__global__ __launch_bounds__(256) void k_stats_part(const float* __restrict__ x, int L, int C, int S,
                                                    double* __restrict__ part) {
  __shared__ double red[2][4][64];
  const int l = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + l, s = blockIdx.y, b = blockIdx.z;
  const int r0 = (int)((long long)L * s / S), r1 = (int)((long long)L * (s + 1) / S);
  double s1 = 0.0, s2 = 0.0;
  if (c < C) {
    const float* xb = x + (size_t)b * L * C + c;
    for (int r = r0 + rl; r < r1; r += 4) {
      const double v = xb[(size_t)r * C];
      s1 += v;
      s2 += v * v;
    }
  }
  red[0][rl][l] = s1;
  red[1][rl][l] = s2;
  __syncthreads();
  if (rl == 0 && c < C) {
    double* p = part + (((size_t)b * S + s) * C + c) * 2;
    p[0] = ((red[0][0][l] + red[0][1][l]) + red[0][2][l]) + red[0][3][l];
    p[1] = ((red[1][0][l] + red[1][1][l]) + red[1][2][l]) + red[1][3][l];
  }
}

__device__ __forceinline__ double wave_sum(double v) {
  // fixed butterfly: lane 0's result has the same association order on every run
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// mean / rstd per (b, c): mr[(b*C + c)*2 + {0, 1}]; one wave per (b, c), lanes stride the slices
__global__ __launch_bounds__(64) void k_stats_final(const double* __restrict__ part, int L, int C, int S,
                                                    float* __restrict__ mr) {
  const int i = blockIdx.x;
  const int b = i / C, c = i % C;
  double s1 = 0.0, s2 = 0.0;
  for (int s = threadIdx.x; s < S; s += 64) {
    const double* p = part + (((size_t)b * S + s) * C + c) * 2;
    s1 += p[0];
    s2 += p[1];
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  if (threadIdx.x == 0) {
    const double mean = s1 / L;
    const double var = fmax(s2 / L - mean * mean, 0.0);
    mr[2 * i] = (float)mean;
    mr[2 * i + 1] = (float)(1.0 / sqrt(var + kEps));
  }
}

__global__ void k_adain_act_fwd(const float* __restrict__ x, const float* __restrict__ gb,
                                const float* __restrict__ alpha, const float* __restrict__ mr, int L, int C, int act,
                                float* __restrict__ y, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int c = (int)(i % C);
  const int b = (int)(i / ((long long)L * C));
  const int bc = b * C + c;
  const float xh = (x[i] - mr[2 * bc]) * mr[2 * bc + 1];
  const float z = (1.f + gb[(size_t)b * 2 * C + c]) * xh + gb[(size_t)b * 2 * C + C + c];
  y[i] = act_fwd(z, act, act == 1 ? alpha[c] : 1.f);
}

struct Recomp {
  float xh, z, dz, da;
};

__device__ __forceinline__ Recomp recompute(float xv, float dyv, float mean, float rstd, float g1, float be, int act,
                                            float a) {
  Recomp o;
  o.xh = (xv - mean) * rstd;
  o.z = g1 * o.xh + be;
  o.da = 0.f;
  if (act == 1) {
    const float sn = sinf(a * o.z), s2 = sinf(2.f * a * o.z);
    o.dz = dyv * (1.f + s2);
    o.da = dyv * (o.z * s2 / a - sn * sn / (a * a));
  } else if (act == 2) {
    o.dz = o.z > 0.f ? dyv : kSlope * dyv;
  } else {
    o.dz = dyv;
  }
  return o;
}

// partials per (b, slice, c): sum dz, sum dz * xhat, sum dalpha terms
__global__ __launch_bounds__(256) void k_adain_bwd_part(const float* __restrict__ x, const float* __restrict__ dy,
                                                        const float* __restrict__ gb, const float* __restrict__ alpha,
                                                        const float* __restrict__ mr, int L, int C, int S, int act,
                                                        double* __restrict__ part) {
  __shared__ double red[3][4][64];
  const int l = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + l, s = blockIdx.y, b = blockIdx.z;
  const int r0 = (int)((long long)L * s / S), r1 = (int)((long long)L * (s + 1) / S);
  double a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if (c < C) {
    const int bc = b * C + c;
    const float mean = mr[2 * bc], rstd = mr[2 * bc + 1];
    const float g1 = 1.f + gb[(size_t)b * 2 * C + c], be = gb[(size_t)b * 2 * C + C + c];
    const float a = act == 1 ? alpha[c] : 1.f;
    const size_t base = (size_t)b * L * C + c;
    for (int r = r0 + rl; r < r1; r += 4) {
      const size_t i = base + (size_t)r * C;
      const Recomp o = recompute(x[i], dy[i], mean, rstd, g1, be, act, a);
      a1 += o.dz;
      a2 += (double)o.dz * o.xh;
      a3 += o.da;
    }
  }
  red[0][rl][l] = a1;
  red[1][rl][l] = a2;
  red[2][rl][l] = a3;
  __syncthreads();
  if (rl == 0 && c < C) {
    double* p = part + (((size_t)b * S + s) * C + c) * 3;
#pragma unroll
    for (int k = 0; k < 3; ++k) p[k] = ((red[k][0][l] + red[k][1][l]) + red[k][2][l]) + red[k][3][l];
  }
}

// per channel c (one wave; lanes stride the slices): dgb[b][c] = dgamma, dgb[b][C + c] = dbeta (and the
// fp64 sums for dx), dalpha[c] summed over utterances in order
__global__ __launch_bounds__(64) void k_adain_bwd_final(const double* __restrict__ part, int B, int C, int S,
                                                        float* __restrict__ dgb, double* __restrict__ sums,
                                                        float* __restrict__ dalpha) {
  const int c = blockIdx.x;
  double da = 0.0;
  for (int b = 0; b < B; ++b) {
    double s1 = 0.0, s2 = 0.0, s3 = 0.0;
    for (int s = threadIdx.x; s < S; s += 64) {
      const double* p = part + (((size_t)b * S + s) * C + c) * 3;
      s1 += p[0];
      s2 += p[1];
      s3 += p[2];
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    da += wave_sum(s3);
    if (threadIdx.x == 0) {
      sums[((size_t)b * C + c) * 2] = s1;
      sums[((size_t)b * C + c) * 2 + 1] = s2;
      if (dgb) {
        dgb[(size_t)b * 2 * C + c] = (float)s2;
        dgb[(size_t)b * 2 * C + C + c] = (float)s1;
      }
    }
  }
  if (dalpha && threadIdx.x == 0) dalpha[c] = (float)da;
}

__global__ void k_adain_bwd_dx(const float* __restrict__ x, const float* __restrict__ dy, const float* __restrict__ gb,
                               const float* __restrict__ alpha, const float* __restrict__ mr,
                               const double* __restrict__ sums, int L, int C, int act, float* __restrict__ dx,
                               long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int c = (int)(i % C);
  const int b = (int)(i / ((long long)L * C));
  const int bc = b * C + c;
  const float mean = mr[2 * bc], rstd = mr[2 * bc + 1];
  const float g1 = 1.f + gb[(size_t)b * 2 * C + c], be = gb[(size_t)b * 2 * C + C + c];
  const Recomp o = recompute(x[i], dy[i], mean, rstd, g1, be, act, act == 1 ? alpha[c] : 1.f);
  const float m1 = (float)(sums[2 * bc] / L), m2 = (float)(sums[2 * bc + 1] / L);
  dx[i] = g1 * rstd * (o.dz - m1 - o.xh * m2);
}

// Linear backward (h = s W^T + bias; s [B][K], W [N][K], dh [B][N]), fp64 sums in fixed order.
// ds[b][k] = sum_n dh[b][n] W[n][k]: one workgroup per (b, 64 k columns); its 16 waves stride n (a wave
// reads 64 consecutive k of one W row: coalesced), each with 8 independent fp64 partials (loads in flight
// instead of one dependent chain), then fixed-order sums (8-way in registers, 16-way in LDS): deterministic.
// (4 waves with one chain each took ~40 us a call; one thread per (b, k) over all N = 2 C rows, 150 us.)
__global__ __launch_bounds__(1024) void k_linear_bwd_ds(const float* __restrict__ W, const float* __restrict__ dh,
                                                        int B, int K, int N, float* __restrict__ ds) {
  // U = 32 loads in flight per thread (a 2,048-row W is 4 batches per wave): the call is latency-bound,
  // two blocks per 64 k columns, so the batch count, not the bytes, sets its time
  constexpr int NW = 16, U = 32, NA = 4;
  __shared__ double red[NW][64];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + l, b = blockIdx.y;
  double acc[NA];
#pragma unroll
  for (int u = 0; u < NA; ++u) acc[u] = 0.0;
  if (k < K) {
    const float* dhb = dh + (size_t)b * N;
    int n = w;
    for (; n + (U - 1) * NW < N; n += U * NW) {
      float hv[U], wv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        hv[u] = dhb[n + u * NW];
        wv[u] = W[(size_t)(n + u * NW) * K + k];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u % NA] += (double)hv[u] * wv[u];
    }
    for (; n < N; n += NW) acc[0] += (double)dhb[n] * W[(size_t)n * K + k];
  }
  double t = 0.0;
#pragma unroll
  for (int u = 0; u < NA; ++u) t += acc[u];
  red[w][l] = t;
  __syncthreads();
  if (w == 0 && k < K) {
    double r = 0.0;
#pragma unroll
    for (int i = 0; i < NW; ++i) r += red[i][l];
    ds[(size_t)b * K + k] = (float)r;
  }
}

__global__ void k_linear_bwd_dw(const float* __restrict__ s, const float* __restrict__ dh, int B, int K, int N,
                                float* __restrict__ dW, float* __restrict__ db) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * (K + 1)) return;
  const int n = i / (K + 1), k = i % (K + 1);
  double acc = 0.0;
  if (k < K) {
    for (int b = 0; b < B; ++b) acc += (double)dh[(size_t)b * N + n] * s[(size_t)b * K + k];
    if (dW) dW[(size_t)n * K + k] = (float)acc;
  } else {
    for (int b = 0; b < B; ++b) acc += dh[(size_t)b * N + n];
    if (db) db[n] = (float)acc;
  }
}

// h[b][n] = bias[n] + sum_k s[b][k] W[n][k]  (nn.Linear layout; fp64 sum)
// one wave per output row n: lanes stride over k (coalesced W row reads), fp64 lane partials reduced by
// shuffles in a fixed order, every utterance b from the same W row
__global__ __launch_bounds__(256) void k_linear_fwd(const float* __restrict__ s, const float* __restrict__ W,
                                                    const float* __restrict__ bias, int B, int K, int N,
                                                    float* __restrict__ h) {
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
  if (n >= N) return;  // uniform per wave
  const float* wr = W + (size_t)n * K;
  for (int b = 0; b < B; ++b) {
    const float* sb = s + (size_t)b * K;
    double acc = 0.0;
    for (int k = l; k < K; k += 64) acc += (double)sb[k] * wr[k];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
    if (l == 0) h[(size_t)b * N + n] = (float)(acc + (bias ? (double)bias[n] : 0.0));
  }
}

// weight_norm backward per row i of v [d0][inner] (w = g v / ||v||):
//   dg[i] = <dw, v> / ||v||,  dv = (g / ||v||) (dw - v <dw, v> / ||v||^2)
__global__ __launch_bounds__(256) void k_wn_bwd(const float* __restrict__ g, const float* __restrict__ v,
                                                const float* __restrict__ dw, int inner, float* __restrict__ dg,
                                                float* __restrict__ dv) {
  __shared__ double red[2][256];
  const int i = blockIdx.x;
  const float* vr = v + (size_t)i * inner;
  const float* dr = dw + (size_t)i * inner;
  double nn = 0.0, dot = 0.0;
  for (int k = threadIdx.x; k < inner; k += 256) {
    nn += (double)vr[k] * vr[k];
    dot += (double)dr[k] * vr[k];
  }
  red[0][threadIdx.x] = nn;
  red[1][threadIdx.x] = dot;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      red[0][threadIdx.x] += red[0][threadIdx.x + w];
      red[1][threadIdx.x] += red[1][threadIdx.x + w];
    }
    __syncthreads();
  }
  const double norm = sqrt(red[0][0]), d = red[1][0];
  if (threadIdx.x == 0 && dg) dg[i] = (float)(d / norm);
  if (dv) {
    const double sc = (g ? (double)g[i] : 1.0) / norm, pr = d / (norm * norm);
    for (int k = threadIdx.x; k < inner; k += 256) dv[(size_t)i * inner + k] = (float)(sc * (dr[k] - vr[k] * pr));
  }
}

// depthwise ConvTranspose1d(C, C, 3, stride 2, padding 1, output_padding 1, groups C) (AdainResBlk1d.pool,
// hifigan.py:375-377) on frames: y[2m] = b + w1 x[m], y[2m+1] = b + w2 x[m] + w0 x[m+1] (x[Lin] = 0)
__global__ void k_pool_fwd(const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
                           int Lin, int C, float* __restrict__ y, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;  // over B * 2Lin * C outputs
  if (i >= n) return;
  const int c = (int)(i % C);
  const long long bo = i / C;
  const int o = (int)(bo % (2 * Lin));
  const long long b = bo / (2 * Lin);
  const float* xb = x + b * Lin * C + c;
  const int m = o >> 1;
  float v = bias ? bias[c] : 0.f;
  if ((o & 1) == 0) {
    v += w[c * 3 + 1] * xb[(size_t)m * C];
  } else {
    v += w[c * 3 + 2] * xb[(size_t)m * C];
    if (m + 1 < Lin) v += w[c * 3 + 0] * xb[(size_t)(m + 1) * C];
  }
  y[i] = v;
}

// dx[m] = w1 dy[2m] + w2 dy[2m+1] + w0 dy[2m-1]
__global__ void k_pool_bwd_dx(const float* __restrict__ dy, const float* __restrict__ w, int Lin, int C,
                              float* __restrict__ dx, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int c = (int)(i % C);
  const long long bm = i / C;
  const int m = (int)(bm % Lin);
  const long long b = bm / Lin;
  const float* db_ = dy + b * 2 * Lin * C + c;
  float v = w[c * 3 + 1] * db_[(size_t)(2 * m) * C] + w[c * 3 + 2] * db_[(size_t)(2 * m + 1) * C];
  if (m > 0) v += w[c * 3 + 0] * db_[(size_t)(2 * m - 1) * C];
  dx[i] = v;
}

// partials per (b, slice, c) of dw0 = sum dy[2m-1] x[m], dw1 = sum dy[2m] x[m], dw2 = sum dy[2m+1] x[m],
// db = sum dy (rows m of the slice cover dy rows 2m, 2m+1)
__global__ __launch_bounds__(256) void k_pool_bwd_part(const float* __restrict__ x, const float* __restrict__ dy,
                                                       int Lin, int C, int S, double* __restrict__ part) {
  __shared__ double red[4][4][64];
  const int l = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + l, s = blockIdx.y, b = blockIdx.z;
  const int r0 = (int)((long long)Lin * s / S), r1 = (int)((long long)Lin * (s + 1) / S);
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if (c < C) {
    const float* xb = x + (size_t)b * Lin * C + c;
    const float* gb = dy + (size_t)b * 2 * Lin * C + c;
    for (int m = r0 + rl; m < r1; m += 4) {
      const double xv = xb[(size_t)m * C];
      const double g0 = gb[(size_t)(2 * m) * C], g1 = gb[(size_t)(2 * m + 1) * C];
      if (m > 0) a0 += (double)gb[(size_t)(2 * m - 1) * C] * xv;
      a1 += g0 * xv;
      a2 += g1 * xv;
      a3 += g0 + g1;
    }
  }
  red[0][rl][l] = a0;
  red[1][rl][l] = a1;
  red[2][rl][l] = a2;
  red[3][rl][l] = a3;
  __syncthreads();
  if (rl == 0 && c < C) {
    double* p = part + (((size_t)b * S + s) * C + c) * 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) p[k] = ((red[k][0][l] + red[k][1][l]) + red[k][2][l]) + red[k][3][l];
  }
}

// per channel (one wave): dw[c][0..2], db[c] summed over utterances and slices in fixed order
__global__ __launch_bounds__(64) void k_pool_bwd_final(const double* __restrict__ part, int B, int C, int S,
                                                       float* __restrict__ dw, float* __restrict__ db) {
  const int c = blockIdx.x;
  double t[4] = {0.0, 0.0, 0.0, 0.0};
  for (int b = 0; b < B; ++b) {
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    for (int s = threadIdx.x; s < S; s += 64) {
      const double* p = part + (((size_t)b * S + s) * C + c) * 4;
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] += p[k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) t[k] += wave_sum(v[k]);
  }
  if (threadIdx.x == 0) {
    if (dw) {
      dw[c * 3 + 0] = (float)t[0];
      dw[c * 3 + 1] = (float)t[1];
      dw[c * 3 + 2] = (float)t[2];
    }
    if (db) db[c] = (float)t[3];
  }
}

// nearest x2 upsample (UpSample1d 'half', hifigan.py:350-357) on frames and its backward
__global__ void k_up2(const float* __restrict__ x, int Lin, int C, float* __restrict__ y, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int c = (int)(i % C);
  const long long bo = i / C;
  const int o = (int)(bo % (2 * Lin));
  const long long b = bo / (2 * Lin);
  y[i] = x[(b * Lin + (o >> 1)) * C + c];
}

__global__ void k_up2_bwd(const float* __restrict__ dy, int Lin, int C, float* __restrict__ dx, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int c = (int)(i % C);
  const long long bm = i / C;
  const int m = (int)(bm % Lin);
  const long long b = bm / Lin;
  const float* g = dy + (b * 2 * Lin + 2 * m) * C + c;
  dx[i] = g[0] + g[C];
}

// LeakyReLU(slope) and its backward from the output (slope > 0 keeps the sign: y > 0 <=> x > 0)
__global__ void k_lrelu(const float* __restrict__ x, long long n, float slope, float* __restrict__ y) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = x[i] > 0.f ? x[i] : slope * x[i];
}

__global__ void k_lrelu_bwd(const float* __restrict__ y, const float* __restrict__ dy, long long n, float slope,
                            float* __restrict__ dx) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dx[i] = y[i] > 0.f ? dy[i] : slope * dy[i];
}

inline size_t al(size_t n) { return (n + 255) & ~(size_t)255; }

}  // namespace

extern "C" long long stts_adain_act_workspace_bytes(int B, int L, int C) {
  if (B <= 0 || L <= 0 || C <= 0) return ST_EINVAL;
  const Cols cl = cols_of(B, L, C);
  return (long long)(al((size_t)B * cl.S * C * 3 * sizeof(double)) + al((size_t)B * C * 2 * sizeof(double)));
}

extern "C" int stts_adain_act_fwd(const float* x, const float* gb, const float* alpha, int act, int B, int L, int C,
                                  float* y, float* mean_rstd, void* ws, long long ws_bytes, void* stream) {
  const long long need = stts_adain_act_workspace_bytes(B, L, C);
  if (need < 0) return (int)need;
  if (!x || !gb || !y || !mean_rstd || act < 0 || act > 2 || (act == 1 && !alpha)) return ST_EINVAL;
  if (!ws || ws_bytes < need) return ST_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const Cols cl = cols_of(B, L, C);
  double* part = (double*)ws;
  hipLaunchKernelGGL(k_stats_part, dim3((C + 63) / 64, cl.S, B), dim3(256), 0, s, x, L, C, cl.S, part);
  ST_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_stats_final, dim3(B * C), dim3(64), 0, s, part, L, C, cl.S, mean_rstd);
  ST_CHECK_HIP(hipGetLastError());
  const long long n = (long long)B * L * C;
  hipLaunchKernelGGL(k_adain_act_fwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, gb, alpha, mean_rstd, L,
                     C, act, y, n);
  return (int)hipGetLastError();
}

extern "C" int stts_adain_act_bwd(const float* x, const float* gb, const float* alpha, int act, const float* mean_rstd,
                                  const float* dy, int B, int L, int C, float* dx, float* dgb, float* dalpha, void* ws,
                                  long long ws_bytes, void* stream) {
  const long long need = stts_adain_act_workspace_bytes(B, L, C);
  if (need < 0) return (int)need;
  if (!x || !gb || !mean_rstd || !dy || act < 0 || act > 2 || (act == 1 && !alpha)) return ST_EINVAL;
  if (!ws || ws_bytes < need) return ST_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const Cols cl = cols_of(B, L, C);
  double* part = (double*)ws;
  double* sums = (double*)((char*)ws + al((size_t)B * cl.S * C * 3 * sizeof(double)));
  hipLaunchKernelGGL(k_adain_bwd_part, dim3((C + 63) / 64, cl.S, B), dim3(256), 0, s, x, dy, gb, alpha, mean_rstd, L,
                     C, cl.S, act, part);
  ST_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_adain_bwd_final, dim3(C), dim3(64), 0, s, part, B, C, cl.S, dgb, sums,
                     act == 1 ? dalpha : nullptr);
  ST_CHECK_HIP(hipGetLastError());
  if (dx) {
    const long long n = (long long)B * L * C;
    hipLaunchKernelGGL(k_adain_bwd_dx, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, dy, gb, alpha,
                       mean_rstd, sums, L, C, act, dx, n);
    ST_CHECK_HIP(hipGetLastError());
  }
  return 0;
}

extern "C" int stts_linear_fwd(const float* s_in, const float* W, const float* bias, int B, int K, int N, float* h,
                               void* stream) {
  if (!s_in || !W || !h || B <= 0 || K <= 0 || N <= 0) return ST_EINVAL;
  hipLaunchKernelGGL(k_linear_fwd, dim3((N + 3) / 4), dim3(256), 0, (hipStream_t)stream, s_in, W, bias, B, K, N, h);
  return (int)hipGetLastError();
}

extern "C" int stts_weight_norm_bwd(const float* g, const float* v, const float* dw, int d0, int inner, float* dg,
                                    float* dv, void* stream) {
  if (!v || !dw || d0 <= 0 || inner <= 0 || (dv && !g && dg)) return ST_EINVAL;
  hipLaunchKernelGGL(k_wn_bwd, dim3(d0), dim3(256), 0, (hipStream_t)stream, g, v, dw, inner, dg, dv);
  return (int)hipGetLastError();
}

extern "C" int stts_linear_bwd(const float* s_in, const float* W, const float* dh, int B, int K, int N, float* ds,
                               float* dW, float* db, void* stream) {
  if (!dh || B <= 0 || K <= 0 || N <= 0 || (ds && !W) || (dW && !s_in)) return ST_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (ds) {
    hipLaunchKernelGGL(k_linear_bwd_ds, dim3((K + 63) / 64, B), dim3(1024), 0, s, W, dh, B, K, N, ds);
    ST_CHECK_HIP(hipGetLastError());
  }
  if (dW || db) {
    hipLaunchKernelGGL(k_linear_bwd_dw, dim3((N * (K + 1) + 255) / 256), dim3(256), 0, s, s_in, dh, B, K, N, dW, db);
    ST_CHECK_HIP(hipGetLastError());
  }
  return 0;
}

extern "C" long long stts_pool_workspace_bytes(int B, int Lin, int C) {
  if (B <= 0 || Lin <= 0 || C <= 0) return ST_EINVAL;
  return (long long)al((size_t)B * cols_of(B, Lin, C).S * C * 4 * sizeof(double));
}

extern "C" int stts_pool_fwd(const float* x, const float* w, const float* bias, int B, int Lin, int C, float* y,
                             void* stream) {
  if (!x || !w || !y || B <= 0 || Lin <= 0 || C <= 0) return ST_EINVAL;
  const long long n = (long long)B * 2 * Lin * C;
  hipLaunchKernelGGL(k_pool_fwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, w, bias,
                     Lin, C, y, n);
  return (int)hipGetLastError();
}

extern "C" int stts_pool_bwd(const float* x, const float* w, const float* dy, int B, int Lin, int C, float* dx,
                             float* dw, float* db, void* ws, long long ws_bytes, void* stream) {
  const long long need = stts_pool_workspace_bytes(B, Lin, C);
  if (need < 0) return (int)need;
  if (!dy || (dx && !w) || (dw && !x)) return ST_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (dx) {
    const long long n = (long long)B * Lin * C;
    hipLaunchKernelGGL(k_pool_bwd_dx, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, dy, w, Lin, C, dx, n);
    ST_CHECK_HIP(hipGetLastError());
  }
  if (dw || db) {
    if (!x) return ST_EINVAL;
    if (!ws || ws_bytes < need) return ST_EWORKSPACE;
    const Cols cl = cols_of(B, Lin, C);
    double* part = (double*)ws;
    hipLaunchKernelGGL(k_pool_bwd_part, dim3((C + 63) / 64, cl.S, B), dim3(256), 0, s, x, dy, Lin, C, cl.S, part);
    ST_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_pool_bwd_final, dim3(C), dim3(64), 0, s, part, B, C, cl.S, dw, db);
    ST_CHECK_HIP(hipGetLastError());
  }
  return 0;
}

extern "C" int stts_upsample2(const float* x, int B, int Lin, int C, float* y, void* stream) {
  if (!x || !y || B <= 0 || Lin <= 0 || C <= 0) return ST_EINVAL;
  const long long n = (long long)B * 2 * Lin * C;
  hipLaunchKernelGGL(k_up2, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, Lin, C, y, n);
  return (int)hipGetLastError();
}

extern "C" int stts_upsample2_bwd(const float* dy, int B, int Lin, int C, float* dx, void* stream) {
  if (!dy || !dx || B <= 0 || Lin <= 0 || C <= 0) return ST_EINVAL;
  const long long n = (long long)B * Lin * C;
  hipLaunchKernelGGL(k_up2_bwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, dy, Lin, C, dx,
                     n);
  return (int)hipGetLastError();
}

extern "C" int stts_leaky_relu(const float* x, long long n, float slope, float* y, void* stream) {
  if (!x || !y || n < 0 || !(slope > 0.f)) return ST_EINVAL;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_lrelu, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, n, slope, y);
  return (int)hipGetLastError();
}

extern "C" int stts_leaky_relu_bwd(const float* y, const float* dy, long long n, float slope, float* dx,
                                   void* stream) {
  if (!y || !dy || !dx || n < 0 || !(slope > 0.f)) return ST_EINVAL;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_lrelu_bwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, y, dy, n,
                     slope, dx);
  return (int)hipGetLastError();
}
