// Training-step spectral kernels, gfx950:
//   * the multi-resolution mel loss of losses.py:24-94 (MultiResolutionSTFTLoss / STFTLoss /
//     SpectralConvergengeLoss, train.py:282 `stft_loss(y_rec, wav)`): per resolution the torchaudio
//     MelSpectrogram(sample_rate, n_fft, win_length, hop_length, window_fn=hann) at its other
//     defaults (n_mels 128, f_min 0, f_max sr/2, power 2, center=True reflect, HTK, no norm) of both
//     signals, (log(1e-5 + mel) + 4) / 4, then ||y - x||_1 / ||y||_1, averaged over resolutions;
//   * the |STFT| front of SpecDiscriminator (Modules/discriminators.py:11-27, :57-60):
//     torch.stft(x, n_fft, hop, win, hann(win)) magnitude, written time-expanded for the Conv2d stack
//     (each (3, kw) Conv2d over (frames, bins) runs as a 1-D conv along the bins over 3 C channels).
// One workgroup walks a few frames of one signal: the n_fft reflect-padded, windowed samples go to
// LDS in bit-reversed order, an in-place radix-2 FFT runs log2(n_fft) stages (twiddles built per
// block in float64, rounded to fp32), then the bins are consumed from LDS.  n_fft is a power of two
// <= 2048, as every resolution of the reference is (512 / 1024 / 2048).
#include "common.h"
#include "kernels.h"

namespace {

constexpr int NT = 256, NMAX = 2048, MMAX = 128;

// torch.linspace(start, end, steps) in fp32 (aten RangeFactoriesKernel: two halves)
__device__ float lin_f32(float start, float end, int steps, int i) {
  const float step = (end - start) / (float)(steps - 1);
  const int half = steps / 2;
  return i < half ? start + step * (float)i : end - step * (float)(steps - i - 1);
}

__device__ __forceinline__ int brev(int n, int lg) { return (int)(__brev((unsigned)n) >> (32 - lg)); }

// Loads frame t of signal x (length L) into a[] bit-reversed, runs the FFT.  Requires tw[] (n/2
// entries, e^{-2 pi i j / n} as (cos, sin)) staged and a barrier-free a[] on entry; ends after a barrier.
__device__ void fft_frame(float2* a, const float2* tw, const float* x, long long L, int n, int lg, int hop,
                          int win, long long t) {
  const int tid = threadIdx.x, woff = (n - win) / 2;
  const long long base = t * hop - n / 2;
  for (int m = tid; m < n; m += NT) {
    const int s = brev(m, lg);
    float v = 0.f;
    if (s >= woff && s < woff + win) {
      long long j = base + s;
      if (j < 0) j = -j;
      if (j >= L) j = 2 * (L - 1) - j;
      // torch.hann_window(win) (periodic), zero-padded to n_fft in the centre (torch.stft)
      const float w = (float)(0.5 - 0.5 * cospi(2.0 * (s - woff) / win));
      v = x[j] * w;
    }
    a[m] = make_float2(v, 0.f);
  }
  __syncthreads();
  for (int l = 0; l < lg; ++l) {
    const int h = 1 << l;
    for (int j = tid; j < n / 2; j += NT) {
      const int pos = j & (h - 1), i0 = ((j >> l) << (l + 1)) + pos, i1 = i0 + h;
      const float2 w = tw[pos << (lg - 1 - l)];
      const float2 u = a[i0], v = a[i1];
      const float tr = w.x * v.x + w.y * v.y, ti = w.x * v.y - w.y * v.x;
      a[i0] = make_float2(u.x + tr, u.y + ti);
      a[i1] = make_float2(u.x - tr, u.y - ti);
    }
    __syncthreads();
  }
}

__device__ void stage_twiddles(float2* tw, int n) {
  for (int j = threadIdx.x; j < n / 2; j += NT) {
    double s, c;
    sincospi(2.0 * j / n, &s, &c);
    tw[j] = make_float2((float)c, (float)s);
  }
}

// log-mel of torchaudio MelSpectrogram (see the file comment) -> out [S][n_mels][F]
__global__ void __launch_bounds__(NT) k_logmel_g(const float* __restrict__ x, long long L, long long ld, int n,
                                                 int lg, int win, int hop, int F, int fpb, int n_mels, float sr,
                                                 float m_max, float* __restrict__ out) {
  __shared__ float2 a[NMAX];
  __shared__ float2 tw[NMAX / 2];
  __shared__ float pw[NMAX / 2 + 1];
  __shared__ float fe[MMAX][3];
  const int s = blockIdx.y, tid = threadIdx.x, nb = n / 2 + 1;
  const float fmax = sr * 0.5f;  // all_freqs = linspace(0, sr // 2, nb)
  for (int m = tid; m < n_mels; m += NT)
    for (int j = 0; j < 3; ++j) {
      const float mp = lin_f32(0.0f, m_max, n_mels + 2, m + j);
      fe[m][j] = 700.0f * (powf(10.0f, mp / 2595.0f) - 1.0f);
    }
  stage_twiddles(tw, n);
  const float* xs = x + (size_t)s * ld;
  const int t0 = blockIdx.x * fpb, t1 = min(F, t0 + fpb);
  for (int t = t0; t < t1; ++t) {
    fft_frame(a, tw, xs, L, n, lg, hop, win, t);
    for (int k = tid; k < nb; k += NT) {
      const float2 c = a[k];
      pw[k] = __builtin_fmaf(c.x, c.x, c.y * c.y);
    }
    __syncthreads();
    const float df = fmax / (float)(nb - 1);
    for (int m = tid; m < n_mels; m += NT) {
      const float* f = fe[m];
      const int lo = max(0, (int)floorf(f[0] / df) - 1), hi = min(nb - 1, (int)ceilf(f[2] / df) + 1);
      float acc = 0.f;
      for (int k = lo; k <= hi; ++k) {
        const float fk = lin_f32(0.0f, fmax, nb, k);
        const float down = -(f[0] - fk) / (f[1] - f[0]), up = (f[2] - fk) / (f[2] - f[1]);
        acc = __builtin_fmaf(pw[k], fmaxf(0.0f, fminf(down, up)), acc);
      }
      out[((size_t)s * n_mels + m) * F + t] = (logf(1e-5f + acc) + 4.0f) * 0.25f;
    }
    __syncthreads();  // pw[] / a[] reuse by the next frame
  }
}

// |STFT| -> the time-expanded input of the first (3, 9) conv: x3[s][h][k][dh] = |X(frame h + dh - 1, bin k)|
// (0 outside the frames), 8 channels per (h, k) with channels 3..7 left as the caller zeroed them
template <typename T>
__global__ void __launch_bounds__(NT) k_stft_mag(const float* __restrict__ x, long long L, long long ld, int n, int lg,
                                                 int win, int hop, int F, int fpb, T* x3) {
  __shared__ float2 a[NMAX];
  __shared__ float2 tw[NMAX / 2];
  const int s = blockIdx.y, tid = threadIdx.x, nb = n / 2 + 1;
  stage_twiddles(tw, n);
  const float* xs = x + (size_t)s * ld;
  T* im = x3 + (size_t)s * F * nb * 8;
  const int t0 = blockIdx.x * fpb, t1 = min(F, t0 + fpb);
  for (int t = t0; t < t1; ++t) {
    fft_frame(a, tw, xs, L, n, lg, hop, win, t);
    for (int k = tid; k < nb; k += NT) {
      const float2 c = a[k];
      const T v = from_f32<T>(sqrtf(__builtin_fmaf(c.x, c.x, c.y * c.y)));
#pragma unroll
      for (int dh = 0; dh < 3; ++dh) {
        const int h = t + 1 - dh;
        if (h >= 0 && h < F) im[((size_t)h * nb + k) * 8 + dh] = v;
      }
    }
    __syncthreads();
  }
}

// x3[s][h][w][c * 3 + dh] = y[s][h + dh - 1][w][c] (0 outside [0, H)): a (3, kw) Conv2d over (frames,
// bins) becomes a 1-D conv along the bins with 3 C input channels, whose weight is the reference's
// [Cout][C][3][kw] tensor read as [Cout][3C][kw]
template <typename T>
__global__ void __launch_bounds__(NT) k_time_expand(const T* __restrict__ y, int H, int W, int C, T* __restrict__ x3) {
  const long long i = (long long)blockIdx.x * NT + threadIdx.x;  // over H * W * C of utterance s
  const long long n = (long long)H * W * C;
  if (i >= n) return;
  const int s = blockIdx.y;
  const int c = (int)(i % C);
  const long long hw = i / C;
  const int w = (int)(hw % W), h = (int)(hw / W);
  const T* ys = y + (size_t)s * n;
  T* xs = x3 + (size_t)s * n * 3;
#pragma unroll
  for (int dh = 0; dh < 3; ++dh) {
    const int hh = h + dh - 1;
    xs[((size_t)h * W + w) * 3 * C + c * 3 + dh] = (hh >= 0 && hh < H) ? ys[((size_t)hh * W + w) * C + c] : from_f32<T>(0.f);
  }
}

// sums[0] += sum |y - x|, sums[1] += sum |y| over n elements (fixed-order per block, fp64 atomics)
__global__ void __launch_bounds__(NT) k_sc_sums(const float* __restrict__ xm, const float* __restrict__ ym,
                                                long long n, double* sums) {
  __shared__ double r0[NT], r1[NT];
  double a = 0.0, b = 0.0;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const float y = ym[i];
    a += fabsf(y - xm[i]);
    b += fabsf(y);
  }
  r0[threadIdx.x] = a;
  r1[threadIdx.x] = b;
  __syncthreads();
  for (int o = NT / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      r0[threadIdx.x] += r0[threadIdx.x + o];
      r1[threadIdx.x] += r1[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    atomicAdd(sums, r0[0]);
    atomicAdd(sums + 1, r1[0]);
  }
}

__global__ void k_sc_final(const double* __restrict__ sums, int nres, double* loss) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    double l = 0.0;
    for (int r = 0; r < nres; ++r) l += sums[2 * r] / sums[2 * r + 1];
    loss[0] = l / nres;
  }
}

int log2_exact(int n) {
  int lg = 0;
  while ((1 << lg) < n) ++lg;
  return (1 << lg) == n ? lg : -1;
}

int frames_per_block(long long S, long long F) {
  const long long want = S * F / 2048;
  return (int)(want < 1 ? 1 : want > 64 ? 64 : want);
}

}  // namespace

long long st_stft_frames(long long L, int hop) { return hop > 0 ? 1 + L / hop : 0; }

int st_logmel(const float* x, int S, long long L, long long ld, int n_fft, int win, int hop, int n_mels, float sr,
              float* out, hipStream_t s) {
  const int lg = log2_exact(n_fft);
  if (S <= 0) return ST_OK;
  if (lg < 1 || n_fft > NMAX || win <= 0 || win > n_fft || hop <= 0 || n_mels <= 0 || n_mels > MMAX ||
      L <= n_fft / 2 || ld < L || S > 65535)
    return ST_EINVAL;
  const long long F = st_stft_frames(L, hop);
  const int fpb = frames_per_block(S, F);
  // m_max = _hz_to_mel(sr / 2) in float64 (torchaudio computes it with math.log10), then fp32
  const float m_max = (float)(2595.0 * log10(1.0 + (double)sr * 0.5 / 700.0));
  hipLaunchKernelGGL(k_logmel_g, dim3((unsigned)((F + fpb - 1) / fpb), (unsigned)S), dim3(NT), 0, s, x, L, ld, n_fft,
                     lg, win, hop, (int)F, fpb, n_mels, sr, m_max, out);
  return (int)hipGetLastError();
}

int st_stft_mag_x3(const float* x, int S, long long L, long long ld, int n_fft, int win, int hop, void* x3, int dtype,
                   hipStream_t s) {
  const int lg = log2_exact(n_fft);
  if (S <= 0) return ST_OK;
  if (lg < 1 || n_fft > NMAX || win <= 0 || win > n_fft || hop <= 0 || L <= n_fft / 2 || ld < L || S > 65535)
    return ST_EINVAL;
  const long long F = st_stft_frames(L, hop);
  const int fpb = frames_per_block(S, F);
  dim3 grid((unsigned)((F + fpb - 1) / fpb), (unsigned)S);
  if (dtype == ST_FP32)
    hipLaunchKernelGGL(k_stft_mag<float>, grid, dim3(NT), 0, s, x, L, ld, n_fft, lg, win, hop, (int)F, fpb,
                       reinterpret_cast<float*>(x3));
  else if (dtype == ST_BF16)
    hipLaunchKernelGGL(k_stft_mag<bf16_t>, grid, dim3(NT), 0, s, x, L, ld, n_fft, lg, win, hop, (int)F, fpb,
                       reinterpret_cast<bf16_t*>(x3));
  else
    return ST_EDTYPE;
  return (int)hipGetLastError();
}

int st_time_expand(const void* y, int S, int H, int W, int C, void* x3, int dtype, hipStream_t s) {
  const long long n = (long long)H * W * C;
  if (S <= 0 || n <= 0) return ST_OK;
  dim3 grid((unsigned)((n + NT - 1) / NT), (unsigned)S);
  if (dtype == ST_FP32)
    hipLaunchKernelGGL(k_time_expand<float>, grid, dim3(NT), 0, s, reinterpret_cast<const float*>(y), H, W, C,
                       reinterpret_cast<float*>(x3));
  else if (dtype == ST_BF16)
    hipLaunchKernelGGL(k_time_expand<bf16_t>, grid, dim3(NT), 0, s, reinterpret_cast<const bf16_t*>(y), H, W, C,
                       reinterpret_cast<bf16_t*>(x3));
  else
    return ST_EDTYPE;
  return (int)hipGetLastError();
}

int st_sc_sums(const float* xm, const float* ym, long long n, double* sums, hipStream_t s) {
  if (n <= 0) return ST_OK;
  long long blocks = (n + NT - 1) / NT;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(k_sc_sums, dim3((unsigned)blocks), dim3(NT), 0, s, xm, ym, n, sums);
  return (int)hipGetLastError();
}

int st_sc_final(const double* sums, int nres, double* loss, hipStream_t s) {
  hipLaunchKernelGGL(k_sc_final, dim3(1), dim3(64), 0, s, sums, nres, loss);
  return (int)hipGetLastError();
}
