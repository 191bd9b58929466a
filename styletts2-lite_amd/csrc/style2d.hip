// StyleEncoder (models.py:125-150) under train.py's G step (train.py:258, 318, 324): the 2-D pieces of its
// autograd path, on frames images [B][H][W][C] (channel fastest; H = mel bins, W = frames), fp32.
//   * Conv2d(k x k, pad p) = a row expansion xe[b][ho][w][c k + dh] = x[b][ho + dh - p][w][c] followed by the
//     conv1d engine over W with the reference weight [Cout][Cin][k][k] read as [Cout][Cin k][k] (the channel
//     order c k + dh makes it that tensor as it lies) -- stts_rowexp_fwd / _bwd here, the conv on convbwd.hip;
//   * LearnedDownSample 'half' (depthwise Conv2d 3x3, stride 2, pad 1, models.py:13-28): stts_dwconv2d_s2_*;
//   * DownSample 'half' (models.py:48-62: the last column repeated when W is odd, then avg_pool2d(2)):
//     stts_avgpool2_*;
//   * AdaptiveAvgPool2d(1) (models.py:139): stts_spatial_mean_*.
// Every reduction is in a fixed order (no atomics): gradients are bitwise reproducible.  These tensors are
// small (the style encoder sees B x 80 x ~300 mel frames): the kernels are plain VALU streams.
#include "common.h"
#include "stts2_train.h"

namespace {

constexpr int NT = 256;

__global__ void __launch_bounds__(NT) k_rowexp(const float* __restrict__ x, int B, int H, int W, int C, int k, int pad,
                                                int Ho, float* __restrict__ xe) {
  const long long n = (long long)B * Ho * W * C * k;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const int ck = (int)(i % ((long long)C * k));
    const long long r = i / ((long long)C * k);  // (b, ho, w)
    const int w = (int)(r % W), ho = (int)((r / W) % Ho), b = (int)(r / ((long long)W * Ho));
    const int c = ck / k, dh = ck - c * k, h = ho + dh - pad;
    xe[i] = (h >= 0 && h < H) ? x[(((long long)b * H + h) * W + w) * C + c] : 0.f;
  }
}

__global__ void __launch_bounds__(NT) k_rowexp_bwd(const float* __restrict__ dxe, int B, int H, int W, int C, int k,
                                                    int pad, int Ho, float* __restrict__ dx) {
  const long long n = (long long)B * H * W * C;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const int c = (int)(i % C);
    const long long r = i / C;
    const int w = (int)(r % W), h = (int)((r / W) % H), b = (int)(r / ((long long)W * H));
    float v = 0.f;
    for (int dh = 0; dh < k; ++dh) {  // in dh order
      const int ho = h - dh + pad;
      if (ho >= 0 && ho < Ho) v += dxe[((((long long)b * Ho + ho) * W + w) * C + c) * k + dh];
    }
    dx[i] = v;
  }
}

// depthwise 3x3 / stride 2 / pad 1: y[b][ho][wo][c] = bias[c] + sum_ij w[c][i][j] x[b][2ho+i-1][2wo+j-1][c]
__global__ void __launch_bounds__(NT) k_dw_s2(const float* __restrict__ x, const float* __restrict__ wt,
                                               const float* __restrict__ bias, int B, int H, int W, int C, int Ho,
                                               int Wo, float* __restrict__ y) {
  const long long n = (long long)B * Ho * Wo * C;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const int c = (int)(i % C);
    const long long r = i / C;
    const int wo = (int)(r % Wo), ho = (int)((r / Wo) % Ho), b = (int)(r / ((long long)Wo * Ho));
    float v = bias ? bias[c] : 0.f;
    for (int a = 0; a < 3; ++a) {
      const int h = 2 * ho + a - 1;
      if (h < 0 || h >= H) continue;
      for (int e = 0; e < 3; ++e) {
        const int w = 2 * wo + e - 1;
        if (w < 0 || w >= W) continue;
        v = fmaf(wt[c * 9 + a * 3 + e], x[(((long long)b * H + h) * W + w) * C + c], v);
      }
    }
    y[i] = v;
  }
}

__global__ void __launch_bounds__(NT) k_dw_s2_dx(const float* __restrict__ dy, const float* __restrict__ wt, int B,
                                                  int H, int W, int C, int Ho, int Wo, float* __restrict__ dx) {
  const long long n = (long long)B * H * W * C;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const int c = (int)(i % C);
    const long long r = i / C;
    const int w = (int)(r % W), h = (int)((r / W) % H), b = (int)(r / ((long long)W * H));
    float v = 0.f;
    for (int a = 0; a < 3; ++a) {
      const int t = h + 1 - a;
      if (t < 0 || (t & 1) || (t >> 1) >= Ho) continue;
      for (int e = 0; e < 3; ++e) {
        const int u = w + 1 - e;
        if (u < 0 || (u & 1) || (u >> 1) >= Wo) continue;
        v = fmaf(wt[c * 9 + a * 3 + e], dy[(((long long)b * Ho + (t >> 1)) * Wo + (u >> 1)) * C + c], v);
      }
    }
    dx[i] = v;
  }
}

// dw / db partials: block (channel group of 64, split s) sums its share of the output positions, one lane per
// channel (coalesced rows), the 4 waves over interleaved positions; partials [S][C][10] (9 taps + bias)
constexpr int DW_S = 32;
__global__ void __launch_bounds__(NT) k_dw_s2_dw(const float* __restrict__ x, const float* __restrict__ dy, int B,
                                                  int H, int W, int C, int Ho, int Wo, float* __restrict__ part) {
  __shared__ float red[4][64][10];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane, s = blockIdx.y;
  const long long P = (long long)B * Ho * Wo;
  const long long p0 = P * s / DW_S, p1 = P * (s + 1) / DW_S;
  float acc[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) acc[k] = 0.f;
  if (c < C) {
    for (long long p = p0 + wv; p < p1; p += 4) {
      const int wo = (int)(p % Wo), ho = (int)((p / Wo) % Ho), b = (int)(p / ((long long)Wo * Ho));
      const float g = dy[p * C + c];
      acc[9] += g;
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const int h = 2 * ho + a - 1;
        if (h < 0 || h >= H) continue;
#pragma unroll
        for (int e = 0; e < 3; ++e) {
          const int w = 2 * wo + e - 1;
          if (w < 0 || w >= W) continue;
          acc[a * 3 + e] = fmaf(g, x[(((long long)b * H + h) * W + w) * C + c], acc[a * 3 + e]);
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 10; ++k) red[wv][lane][k] = acc[k];
  __syncthreads();
  if (wv == 0 && c < C) {
#pragma unroll
    for (int k = 0; k < 10; ++k)
      part[((size_t)s * C + c) * 10 + k] = (red[0][lane][k] + red[1][lane][k]) + (red[2][lane][k] + red[3][lane][k]);
  }
}

__global__ void __launch_bounds__(NT) k_dw_s2_dw_reduce(const float* __restrict__ part, int C, float* __restrict__ dw,
                                                         float* __restrict__ db) {
  const int i = blockIdx.x * NT + threadIdx.x;
  if (i >= C * 10) return;
  const int c = i / 10, k = i - c * 10;
  float v = 0.f;
  for (int s = 0; s < DW_S; ++s) v += part[((size_t)s * C + c) * 10 + k];  // split order
  if (k < 9) {
    if (dw) dw[c * 9 + k] = v;
  } else if (db) {
    db[c] = v;
  }
}

// DownSample 'half': W odd -> the last column repeated, then 2 x 2 averages (H odd: the last row dropped)
__global__ void __launch_bounds__(NT) k_avgpool2(const float* __restrict__ x, int B, int H, int W, int C,
                                                  float* __restrict__ y) {
  const int Ho = H / 2, Wo = (W + 1) / 2;
  const long long n = (long long)B * Ho * Wo * C;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const int c = (int)(i % C);
    const long long r = i / C;
    const int wo = (int)(r % Wo), ho = (int)((r / Wo) % Ho), b = (int)(r / ((long long)Wo * Ho));
    const int w0 = 2 * wo, w1 = 2 * wo + 1 < W ? 2 * wo + 1 : W - 1;
    const float* r0 = x + (((long long)b * H + 2 * ho) * W) * C + c;
    const float* r1 = r0 + (long long)W * C;
    // avg_pool2d's order: the window's four values summed row by row, then / 4
    y[i] = (((r0[(long long)w0 * C] + r0[(long long)w1 * C]) + r1[(long long)w0 * C]) + r1[(long long)w1 * C]) / 4.f;
  }
}

__global__ void __launch_bounds__(NT) k_avgpool2_bwd(const float* __restrict__ dy, int B, int H, int W, int C,
                                                      float* __restrict__ dx) {
  const int Ho = H / 2, Wo = (W + 1) / 2;
  const long long n = (long long)B * H * W * C;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const int c = (int)(i % C);
    const long long r = i / C;
    const int w = (int)(r % W), h = (int)((r / W) % H), b = (int)(r / ((long long)W * H));
    const int ho = h / 2, wo = w / 2;
    float v = 0.f;
    if (ho < Ho) {
      const float g = dy[(((long long)b * Ho + ho) * Wo + wo) * C + c] / 4.f;
      // the repeated last column (W odd) takes part twice in its window
      v = (W & 1) && w == W - 1 ? g + g : g;
    }
    dx[i] = v;
  }
}

// AdaptiveAvgPool2d(1): y[b][c] = mean over the H W positions (position order)
__global__ void __launch_bounds__(NT) k_spatial_mean(const float* __restrict__ x, int B, int P, int C,
                                                      float* __restrict__ y) {
  const int i = blockIdx.x * NT + threadIdx.x;
  if (i >= B * C) return;
  const int b = i / C, c = i - b * C;
  float v = 0.f;
  for (int p = 0; p < P; ++p) v += x[((long long)b * P + p) * C + c];
  y[i] = v / (float)P;
}

__global__ void __launch_bounds__(NT) k_spatial_mean_bwd(const float* __restrict__ dy, int B, int P, int C,
                                                          float* __restrict__ dx) {
  const long long n = (long long)B * P * C;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const int c = (int)(i % C), b = (int)(i / ((long long)P * C));
    dx[i] = dy[b * C + c] / (float)P;
  }
}

unsigned grid_of(long long n) {
  const long long g = (n + NT - 1) / NT;
  return (unsigned)(g < 65536 ? (g > 0 ? g : 1) : 65536);
}

}  // namespace

extern "C" {

int stts_rowexp_fwd(const float* x, int B, int H, int W, int C, int k, int pad, float* xe, void* stream) {
  const int Ho = H + 2 * pad - k + 1;
  if (!x || !xe || B < 0 || H <= 0 || W <= 0 || C <= 0 || k <= 0 || pad < 0 || Ho <= 0) return ST_EINVAL;
  const long long n = (long long)B * Ho * W * C * k;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_rowexp, dim3(grid_of(n)), dim3(NT), 0, (hipStream_t)stream, x, B, H, W, C, k, pad, Ho, xe);
  return (int)hipGetLastError();
}

int stts_rowexp_bwd(const float* dxe, int B, int H, int W, int C, int k, int pad, float* dx, void* stream) {
  const int Ho = H + 2 * pad - k + 1;
  if (!dxe || !dx || B < 0 || H <= 0 || W <= 0 || C <= 0 || k <= 0 || pad < 0 || Ho <= 0) return ST_EINVAL;
  const long long n = (long long)B * H * W * C;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_rowexp_bwd, dim3(grid_of(n)), dim3(NT), 0, (hipStream_t)stream, dxe, B, H, W, C, k, pad, Ho,
                     dx);
  return (int)hipGetLastError();
}

int stts_dwconv2d_s2_fwd(const float* x, const float* w, const float* bias, int B, int H, int W, int C, float* y,
                         void* stream) {
  if (!x || !w || !y || B < 0 || H <= 0 || W <= 0 || C <= 0) return ST_EINVAL;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const long long n = (long long)B * Ho * Wo * C;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_dw_s2, dim3(grid_of(n)), dim3(NT), 0, (hipStream_t)stream, x, w, bias, B, H, W, C, Ho, Wo, y);
  return (int)hipGetLastError();
}

long long stts_dwconv2d_s2_workspace_bytes(int C) { return C <= 0 ? ST_EINVAL : (long long)DW_S * C * 10 * 4; }

int stts_dwconv2d_s2_bwd(const float* x, const float* w, const float* dy, int B, int H, int W, int C, float* dx,
                         float* dw, float* db, void* ws, long long ws_bytes, void* stream) {
  if (!x || !w || !dy || B < 0 || H <= 0 || W <= 0 || C <= 0) return ST_EINVAL;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  hipStream_t s = (hipStream_t)stream;
  if (dx) {
    const long long n = (long long)B * H * W * C;
    if (n) {
      hipLaunchKernelGGL(k_dw_s2_dx, dim3(grid_of(n)), dim3(NT), 0, s, dy, w, B, H, W, C, Ho, Wo, dx);
      ST_CHECK_HIP(hipGetLastError());
    }
  }
  if (dw || db) {
    if (!ws || ws_bytes < stts_dwconv2d_s2_workspace_bytes(C)) return ST_EWORKSPACE;
    float* part = (float*)ws;
    hipLaunchKernelGGL(k_dw_s2_dw, dim3((C + 63) / 64, DW_S), dim3(NT), 0, s, x, dy, B, H, W, C, Ho, Wo, part);
    ST_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_dw_s2_dw_reduce, dim3((C * 10 + NT - 1) / NT), dim3(NT), 0, s, part, C, dw, db);
    ST_CHECK_HIP(hipGetLastError());
  }
  return 0;
}

int stts_avgpool2_fwd(const float* x, int B, int H, int W, int C, float* y, void* stream) {
  if (!x || !y || B < 0 || H < 2 || W <= 0 || C <= 0) return ST_EINVAL;
  const long long n = (long long)B * (H / 2) * ((W + 1) / 2) * C;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_avgpool2, dim3(grid_of(n)), dim3(NT), 0, (hipStream_t)stream, x, B, H, W, C, y);
  return (int)hipGetLastError();
}

int stts_avgpool2_bwd(const float* dy, int B, int H, int W, int C, float* dx, void* stream) {
  if (!dy || !dx || B < 0 || H < 2 || W <= 0 || C <= 0) return ST_EINVAL;
  const long long n = (long long)B * H * W * C;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_avgpool2_bwd, dim3(grid_of(n)), dim3(NT), 0, (hipStream_t)stream, dy, B, H, W, C, dx);
  return (int)hipGetLastError();
}

int stts_spatial_mean_fwd(const float* x, int B, int P, int C, float* y, void* stream) {
  if (!x || !y || B < 0 || P <= 0 || C <= 0) return ST_EINVAL;
  if (B == 0) return 0;
  hipLaunchKernelGGL(k_spatial_mean, dim3((B * C + NT - 1) / NT), dim3(NT), 0, (hipStream_t)stream, x, B, P, C, y);
  return (int)hipGetLastError();
}

int stts_spatial_mean_bwd(const float* dy, int B, int P, int C, float* dx, void* stream) {
  if (!dy || !dx || B < 0 || P <= 0 || C <= 0) return ST_EINVAL;
  const long long n = (long long)B * P * C;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_spatial_mean_bwd, dim3(grid_of(n)), dim3(NT), 0, (hipStream_t)stream, dy, B, P, C, dx);
  return (int)hipGetLastError();
}

}  // extern "C"
