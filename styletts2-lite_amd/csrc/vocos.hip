// Vocos decoder kernels (reference Modules/vocos.py), gfx950:
//   k_dwconv7       ConvNeXtBlock.dwconv (:45): depthwise Conv1d(C, C, 7, pad 3) + bias over frames,
//                   with the InstanceNorm statistics of its output for the AdaIN that follows (:59)
//   k_frame_ln      Generator.final_layer_norm (:147, :160): LayerNorm over the channels of a frame
//   k_istft_frames  ISTFTHead (:271-296) + the irfft / window of ISTFT.forward (:210-212): one
//                   workgroup per STFT frame; the magnitude / phase channels of the head's Linear
//                   output become a Hermitian spectrum in LDS and a two-factor (N = N1 * N2)
//                   Cooley-Tukey DFT gives the real frame, scaled 1/N and windowed
//   k_istft_ola     the fold overlap-add, the folded squared-window envelope, the (win-hop)/2 trim
//                   and the division (:214-231), one output sample per thread
//   k_scale_rows    pack-time weight prep: layer-scale fold (gamma * W, gamma * b) and zero rows
//                   that pad the head's 2 * (n_fft/2 + 1) columns to the MFMA column multiple
// The pointwise convs (pwconv1 + GELU, pwconv2 + residual, ISTFTHead.out) run on conv1d_igemm.
#include "common.h"
#include "kernels.h"

namespace {

#define VDISPATCH(dtype, T, ...)                  \
  do {                                            \
    if ((dtype) == ST_FP32) {                     \
      using T = float;                            \
      __VA_ARGS__;                                \
    } else if ((dtype) == ST_BF16) {              \
      using T = bf16_t;                           \
      __VA_ARGS__;                                \
    } else {                                      \
      return ST_EDTYPE;                           \
    }                                             \
  } while (0)

constexpr int DW_ROWS = 32;  // output frames per thread

// y[b][t][c] = bias[c] + sum_k w[c][k] * x[b][t + k - 3][c]  (zero padded), stats of y.
// A thread owns one channel and DW_ROWS consecutive frames (sliding 7-tap window in registers);
// the 256 threads of a block cover 256 consecutive channels, so every row access is coalesced.
template <typename T>
__global__ void __launch_bounds__(256) k_dwconv7(const T* __restrict__ x, long long x_bs, int x_ld, int L, int C,
                                                 const float* __restrict__ w, const float* __restrict__ bias, T* y,
                                                 long long y_bs, int y_ld, double* stats, int stats_ld, int slots,
                                                 long long slot_bs) {
  const int b = blockIdx.y, c = blockIdx.z * 256 + threadIdx.x;
  if (c >= C) return;
  const int r0 = blockIdx.x * DW_ROWS;
  const T* xb = x + (size_t)b * x_bs + c;
  T* yb = y + (size_t)b * y_bs + c;
  float wk[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) wk[k] = w[c * 7 + k];
  const float bc = bias ? bias[c] : 0.f;
  float win[7];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const int r = r0 - 3 + k;
    win[k] = (r >= 0 && r < L) ? to_f32(xb[(size_t)r * x_ld]) : 0.f;
  }
  double a = 0.0, q = 0.0;
  const int r1 = min(r0 + DW_ROWS, L);
  for (int t = r0; t < r1; ++t) {
    const int r = t + 3;
    win[6] = r < L ? to_f32(xb[(size_t)r * x_ld]) : 0.f;
    float v = bc;
#pragma unroll
    for (int k = 0; k < 7; ++k) v = fmaf(wk[k], win[k], v);
    const T tv = from_f32<T>(v);
    yb[(size_t)t * y_ld] = tv;
    const float s = to_f32(tv);
    a += s;
    q += (double)s * s;
#pragma unroll
    for (int k = 0; k < 6; ++k) win[k] = win[k + 1];
  }
  if (stats) {
    double* d = stats + (size_t)(slots > 1 ? (blockIdx.x % slots) : 0) * slot_bs + ((size_t)b * stats_ld + c) * ST_W;
    stat_add(d, a, q);
  }
}

// LayerNorm(C, eps) over each frame row (torch layer_norm: biased variance, affine).  One wave per
// row; lane l holds channel groups l, l + 64, ... of 8 (C % 8 == 0, C <= 8 * 64 * LN_G).
constexpr int LN_G = 2;
template <typename T>
__global__ void __launch_bounds__(256) k_frame_ln(const T* __restrict__ x, int x_ld, long long rows, int C, float eps,
                                                  const float* __restrict__ g, const float* __restrict__ be, T* y,
                                                  int y_ld) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const T* xr = x + (size_t)row * x_ld;
  const int ng = C / 8;
  float v[LN_G][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LN_G; ++i) {
    const int grp = lane + 64 * i;
    if (grp < ng) {
      load8(xr + 8 * grp, v[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[i][j];
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
  const float mean = s / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < LN_G; ++i) {
    if (lane + 64 * i < ng) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[i][j] - mean;
        q = fmaf(d, d, q);
      }
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) q += __shfl_xor(q, o);
  const float rstd = 1.0f / sqrtf(q / (float)C + eps);
  T* yr = y + (size_t)row * y_ld;
#pragma unroll
  for (int i = 0; i < LN_G; ++i) {
    const int grp = lane + 64 * i;
    if (grp < ng) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = 8 * grp + j;
        yr[c] = from_f32<T>((v[i][j] - mean) * rstd * g[c] + be[c]);
      }
    }
  }
}

// e^{2 pi i m / M}
__device__ __forceinline__ float2 cis(int m, int M) {
  float sn, cs;
  sincospif(2.0f * (float)m / (float)M, &sn, &cs);
  return make_float2(cs, sn);
}

// One STFT frame: spec[k] = min(exp(h[k]), 100) * (cos h[nb + k] + i sin h[nb + k]), k < nb;
// x[n] = (1/N) sum_k X[k] e^{2 pi i k n / N} over the Hermitian extension (the imaginary parts of
// the DC and, N even, Nyquist bins dropped, as the C2R transform of torch.fft.irfft does);
// frame[n] = x[n] * window[n].   Index maps: k = k1 + N1 k2, n = N2 n1 + n2;
//   Y[k1][n2] = e^{2 pi i k1 n2 / N} sum_k2 X[k1 + N1 k2] e^{2 pi i k2 n2 / N2}
//   x[N2 n1 + n2] = Re sum_k1 Y[k1][n2] e^{2 pi i k1 n1 / N1}
template <typename T>
__global__ void __launch_bounds__(256) k_istft_frames(const T* __restrict__ h, int F, int ld, int N, int N1, int N2,
                                                      const float* __restrict__ window, float* __restrict__ fr) {
  extern __shared__ float2 sm[];
  float2* X = sm;            // [N]
  float2* Y = sm + N;        // [N1][N2]
  float2* t1 = Y + N;        // [N1]
  float2* t2 = t1 + N1;      // [N2]
  const int f = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int nb = N / 2 + 1;
  const T* hr = h + ((size_t)b * F + f) * ld;
  for (int k = tid; k < N; k += 256) {
    const bool mir = k > N / 2;
    const int src = mir ? N - k : k;
    const float mag = fminf(expf(to_f32(hr[src])), 100.0f);
    float sn, cs;
    sincosf(to_f32(hr[nb + src]), &sn, &cs);
    float re = mag * cs, im = mag * sn;
    if (src == 0 || 2 * src == N) im = 0.f;
    X[k] = make_float2(re, mir ? -im : im);
  }
  for (int m = tid; m < N1; m += 256) t1[m] = cis(m, N1);
  for (int m = tid; m < N2; m += 256) t2[m] = cis(m, N2);
  __syncthreads();
  for (int i = tid; i < N; i += 256) {
    const int k1 = i / N2, n2 = i - k1 * N2;
    float re = 0.f, im = 0.f;
    int e = 0;  // (k2 * n2) mod N2
    for (int k2 = 0; k2 < N2; ++k2) {
      const float2 xv = X[k1 + N1 * k2], tw = t2[e];
      re = fmaf(xv.x, tw.x, fmaf(-xv.y, tw.y, re));
      im = fmaf(xv.x, tw.y, fmaf(xv.y, tw.x, im));
      e += n2;
      if (e >= N2) e -= N2;
    }
    const float2 tw = cis((k1 * n2) % N, N);
    Y[i] = make_float2(re * tw.x - im * tw.y, re * tw.y + im * tw.x);
  }
  __syncthreads();
  const float invN = 1.0f / (float)N;
  float* fo = fr + ((size_t)b * F + f) * N;
  for (int n = tid; n < N; n += 256) {
    const int n1 = n / N2, n2 = n - n1 * N2;
    float re = 0.f;
    int e = 0;  // (k1 * n1) mod N1
    for (int k1 = 0; k1 < N1; ++k1) {
      const float2 yv = Y[k1 * N2 + n2], tw = t1[e];
      re = fmaf(yv.x, tw.x, fmaf(-yv.y, tw.y, re));
      e += n1;
      if (e >= N1) e -= N1;
    }
    fo[n] = re * invN * window[n];
  }
}

// out[b][j] = sum_t fr[b][t][p - t hop] / sum_t window[p - t hop]^2,  p = j + pad
__global__ void __launch_bounds__(256) k_istft_ola(const float* __restrict__ fr, int F, int N, int hop, int pad,
                                                   const float* __restrict__ window, float* __restrict__ out, int Lout) {
  const int j = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  if (j >= Lout) return;
  const int p = j + pad;
  int t0 = p - N + 1;
  t0 = t0 <= 0 ? 0 : (t0 + hop - 1) / hop;
  const int t1 = min(F - 1, p / hop);
  float y = 0.f, env = 0.f;
  for (int t = t0; t <= t1; ++t) {
    const int n = p - t * hop;
    y += fr[((size_t)b * F + t) * N + n];
    env = fmaf(window[n], window[n], env);
  }
  out[(size_t)b * Lout + j] = y / env;
}

// out[r][i] = r < rows_src ? src[r][i] * (scale ? scale[r] : 1) : 0,  r < rows_dst
__global__ void __launch_bounds__(256) k_scale_rows(const float* __restrict__ src, const float* __restrict__ scale,
                                                    int rows_src, long long inner, int rows_dst, float* out) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)rows_dst * inner) return;
  const int r = (int)(i / inner);
  out[i] = r < rows_src ? src[i] * (scale ? scale[r] : 1.0f) : 0.f;
}

}  // namespace

int st_dwconv7(const void* x, long long x_bs, int x_ld, int B, int L, int C, const float* w, const float* bias, void* y,
               long long y_bs, int y_ld, double* stats, int stats_ld, int slots, long long slot_bs, int dtype,
               hipStream_t s) {
  if (B <= 0 || L <= 0 || C <= 0) return ST_OK;
  dim3 grid((L + DW_ROWS - 1) / DW_ROWS, B, (C + 255) / 256);
  VDISPATCH(dtype, T,
            hipLaunchKernelGGL(k_dwconv7<T>, grid, dim3(256), 0, s, reinterpret_cast<const T*>(x), x_bs, x_ld, L, C, w,
                               bias, reinterpret_cast<T*>(y), y_bs, y_ld, stats, stats_ld, slots, slot_bs));
  return (int)hipGetLastError();
}

int st_frame_ln(const void* x, int x_ld, long long rows, int C, float eps, const float* g, const float* b, void* y,
                int y_ld, int dtype, hipStream_t s) {
  if (rows <= 0) return ST_OK;
  if (C % 8 || C > 8 * 64 * LN_G || x_ld % 8 || y_ld % 8) return ST_EINVAL;
  dim3 grid((unsigned)((rows + 3) / 4));
  VDISPATCH(dtype, T,
            hipLaunchKernelGGL(k_frame_ln<T>, grid, dim3(256), 0, s, reinterpret_cast<const T*>(x), x_ld, rows, C, eps,
                               g, b, reinterpret_cast<T*>(y), y_ld));
  return (int)hipGetLastError();
}

int st_istft_factor(int N, int* N1, int* N2) {
  int best = 0;
  for (int a = 1; a <= 64; ++a)
    if (N % a == 0 && N / a <= 64 && (best == 0 || abs(a * a - N) < abs(best * best - N))) best = a;
  if (!best) return ST_EINVAL;
  *N1 = best;
  *N2 = N / best;
  return ST_OK;
}

int st_istft_head(const void* h, int B, int F, int ld, int N, int hop, const float* window, float* fr, float* out,
                  int dtype, hipStream_t s) {
  if (B <= 0 || F <= 0) return ST_OK;
  int N1 = 0, N2 = 0;
  ST_CHECK(st_istft_factor(N, &N1, &N2));
  if (ld < 2 * (N / 2 + 1) || hop <= 0 || hop > N) return ST_EINVAL;
  const size_t lds = (size_t)(2 * N + N1 + N2) * sizeof(float2);
  if (lds > 64 * 1024) return ST_EINVAL;
  VDISPATCH(dtype, T,
            hipLaunchKernelGGL(k_istft_frames<T>, dim3(F, B), dim3(256), lds, s, reinterpret_cast<const T*>(h), F, ld, N,
                               N1, N2, window, fr));
  ST_CHECK_HIP(hipGetLastError());
  const int pad = (N - hop) / 2;
  const int Lout = (F - 1) * hop + N - 2 * pad;
  hipLaunchKernelGGL(k_istft_ola, dim3((Lout + 255) / 256, B), dim3(256), 0, s, fr, F, N, hop, pad, window, out, Lout);
  return (int)hipGetLastError();
}

int st_scale_rows(const float* src, const float* scale, int rows_src, long long inner, int rows_dst, float* out,
                  hipStream_t s) {
  const long long n = (long long)rows_dst * inner;
  if (n <= 0) return ST_OK;
  hipLaunchKernelGGL(k_scale_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, scale, rows_src, inner,
                     rows_dst, out);
  return (int)hipGetLastError();
}
