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
#include <algorithm>

#include "../../include/stts2_train.h"
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
__global__ void __launch_bounds__(NT) k_time_expand(const T* __restrict__ y, int H, int W, int C, T* __restrict__ x3,
                                                    int We) {
  // x3 rows per (signal, frame) sequence: We >= W (rows W .. We - 1 written as zeros: the even row count the
  // phase-folded stride-2 convs of msd_forward read)
  const long long i = (long long)blockIdx.x * NT + threadIdx.x;  // over H * We * C of utterance s
  const long long n = (long long)H * We * C;
  if (i >= n) return;
  const int s = blockIdx.y;
  const int c = (int)(i % C);
  const long long hw = i / C;
  const int w = (int)(hw % We), h = (int)(hw / We);
  const T* ys = y + (size_t)s * H * W * C;
  T* xs = x3 + (size_t)s * n * 3;
#pragma unroll
  for (int dh = 0; dh < 3; ++dh) {
    const int hh = h + dh - 1;
    xs[((size_t)h * We + w) * 3 * C + c * 3 + dh] =
        (hh >= 0 && hh < H && w < W) ? ys[((size_t)hh * W + w) * C + c] : from_f32<T>(0.f);
  }
}

// per-block partials of sum |y - x| and sum |y| over n elements (fixed split of n over kScBlocks blocks,
// fixed-order block tree): part[blk][0..1]; k_sc_final adds the blocks in order (deterministic)
__global__ void __launch_bounds__(NT) k_sc_sums(const float* __restrict__ xm, const float* __restrict__ ym,
                                                long long n, double* __restrict__ part) {
  __shared__ double r0[NT], r1[NT];
  const long long i0 = n * blockIdx.x / gridDim.x, i1 = n * (blockIdx.x + 1) / gridDim.x;
  double a = 0.0, b = 0.0;
  for (long long i = i0 + threadIdx.x; i < i1; i += NT) {
    const float y = ym[i];
    if (xm) a += fabsf(y - xm[i]);
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
    part[2 * blockIdx.x] = r0[0];
    part[2 * blockIdx.x + 1] = r1[0];
  }
}

// loss[0] = mean_r A_r / D_r with A_r, D_r the in-order sums of resolution r's partials
__global__ void k_sc_final(const double* __restrict__ part, int nres, int nblk, double* loss) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    double l = 0.0;
    for (int r = 0; r < nres; ++r) {
      double a = 0.0, d = 0.0;
      for (int j = 0; j < nblk; ++j) {
        a += part[((size_t)r * nblk + j) * 2];
        d += part[((size_t)r * nblk + j) * 2 + 1];
      }
      l += a / d;
    }
    loss[0] = l / nres;
  }
}

// ------------------------------------------------------------------ training backward (stts2_train.h)
// Inverse of fft_frame's butterflies: a[] holds Z (bit-reversed order) on entry; on exit
// a[n] = sum_k Z_k e^{+2 pi i k n / N} (after a barrier).
__device__ void ifft_inplace(float2* a, const float2* tw, int n, int lg) {
  const int tid = threadIdx.x;
  __syncthreads();
  for (int l = 0; l < lg; ++l) {
    const int h = 1 << l;
    for (int j = tid; j < n / 2; j += NT) {
      const int pos = j & (h - 1), i0 = ((j >> l) << (l + 1)) + pos, i1 = i0 + h;
      const float2 w = tw[pos << (lg - 1 - l)];
      const float2 u = a[i0], v = a[i1];
      const float tr = w.x * v.x - w.y * v.y, ti = w.x * v.y + w.y * v.x;
      a[i0] = make_float2(u.x + tr, u.y + ti);
      a[i1] = make_float2(u.x - tr, u.y - ti);
    }
    __syncthreads();
  }
}

__device__ __forceinline__ float hann_at(int i, int win) { return (float)(0.5 - 0.5 * cospi(2.0 * i / win)); }

// Frame t's adjoint: given dX_k (k < nb) in a[] bit-reversed (zeros above nb), the gradient of the
// windowed frame samples is Re(sum_k dX_k e^{+i theta}) (d Re X_k / d f_n = cos, d Im X_k / d f_n = -sin);
// times the window -> fb[i] for i < win (the window's support inside the n_fft frame).
__device__ void frame_adjoint_out(float2* a, const float2* tw, int n, int lg, int win, float* fb) {
  ifft_inplace(a, tw, n, lg);
  const int woff = (n - win) / 2;
  for (int i = threadIdx.x; i < win; i += NT) fb[i] = hann_at(i, win) * a[woff + i].x;
  __syncthreads();  // a[] is rewritten by the caller's next frame
}

// |torch.stft| image + the complex spectrum (training forward of SpecDiscriminator's input)
__global__ void __launch_bounds__(NT) k_stft_spec(const float* __restrict__ x, long long L, long long ld, int n, int lg,
                                                  int win, int hop, int F, int fpb, float* __restrict__ mag,
                                                  float2* __restrict__ spec) {
  __shared__ float2 a[NMAX];
  __shared__ float2 tw[NMAX / 2];
  const int s = blockIdx.y, tid = threadIdx.x, nb = n / 2 + 1;
  stage_twiddles(tw, n);
  const float* xs = x + (size_t)s * ld;
  const int t0 = blockIdx.x * fpb, t1 = min(F, t0 + fpb);
  for (int t = t0; t < t1; ++t) {
    fft_frame(a, tw, xs, L, n, lg, hop, win, t);
    const size_t row = ((size_t)s * F + t) * nb;
    for (int k = tid; k < nb; k += NT) {
      const float2 c = a[k];
      mag[row + k] = hypotf(c.x, c.y);  // torch.abs of a complex float = std::abs = hypot
      spec[row + k] = c;
    }
    __syncthreads();
  }
}

// per frame: dX = dmag * X / |X| (torch's abs backward, 0 at |X| = 0), then the adjoint -> fbuf[s][t][win]
__global__ void __launch_bounds__(NT) k_stft_adj(const float2* __restrict__ spec, const float* __restrict__ dmag,
                                                 int n, int lg, int win, int F, int fpb, float* __restrict__ fbuf) {
  __shared__ float2 a[NMAX];
  __shared__ float2 tw[NMAX / 2];
  const int s = blockIdx.y, tid = threadIdx.x, nb = n / 2 + 1;
  stage_twiddles(tw, n);
  const int t0 = blockIdx.x * fpb, t1 = min(F, t0 + fpb);
  for (int t = t0; t < t1; ++t) {
    const size_t row = ((size_t)s * F + t) * nb;
    for (int m = tid; m < n; m += NT) {
      const int k = brev(m, lg);
      float2 z = make_float2(0.f, 0.f);
      if (k < nb) {
        const float2 c = spec[row + k];
        const float ab = hypotf(c.x, c.y);
        if (ab != 0.f) {
          const float g = dmag[row + k];
          z = make_float2(g * (c.x / ab), g * (c.y / ab));
        }
      }
      a[m] = z;
    }
    frame_adjoint_out(a, tw, n, lg, win, fbuf + ((size_t)s * F + t) * win);
  }
}

// dx[s][j] (+)= sum over the padded positions p holding x[j] (centre p = j + n/2, and the reflect-pad
// copies p = n/2 - j, p = n/2 + 2(L-1) - j) of sum over the frames t covering p of fbuf[s][t][p - t hop - woff]
__global__ void __launch_bounds__(NT) k_ola_gather(const float* __restrict__ fbuf, long long L, int n, int win,
                                                   int hop, int F, int accumulate, float* __restrict__ dx,
                                                   long long dx_ld) {
  const int s = blockIdx.y;
  const long long j = (long long)blockIdx.x * NT + threadIdx.x;
  if (j >= L) return;
  const int woff = (n - win) / 2, half = n / 2;
  const float* fs = fbuf + (size_t)s * F * win;
  long long ps[3];
  int np = 0;
  ps[np++] = j + half;
  if (j >= 1 && j <= half) ps[np++] = half - j;
  if (j <= L - 2 && j >= L - 1 - half) ps[np++] = half + 2 * (L - 1) - j;
  float v = 0.f;
  for (int q = 0; q < np; ++q) {
    const long long p = ps[q] - woff;  // position inside the window support of frame t: p - t hop in [0, win)
    long long tlo = p - win + 1 <= 0 ? 0 : (p - win + 1 + hop - 1) / hop;
    long long thi = p < 0 ? -1 : p / hop;
    if (thi > F - 1) thi = F - 1;
    for (long long t = tlo; t <= thi; ++t) v += fs[(size_t)t * win + (p - t * hop)];
  }
  float* o = dx + (size_t)s * dx_ld + j;
  *o = accumulate ? *o + v : v;
}

// MR-STFT loss backward, one resolution, per frame of x: FFT, power, mel, the reference's
// (log(1e-5 + mel) + 4) / 4, d/dx_mag = -sign(y_mag - x_mag) * g0 (g0 = (go / n_res) / ||y_mag||_1), the
// log, filterbank (dP_k = sum_m fb[k][m] dmel_m) and power (dX = 2 X dP) adjoints, the frame adjoint
__global__ void __launch_bounds__(NT) k_mel_bwd(const float* __restrict__ x, long long L, long long ld, int n, int lg,
                                                int win, int hop, int F, int fpb, int n_mels, float sr, float m_max,
                                                const float* __restrict__ ym, const double* __restrict__ dsum,
                                                const float* __restrict__ go, float inv_nres,
                                                float* __restrict__ fbuf) {
  __shared__ float2 a[NMAX];
  __shared__ float2 tw[NMAX / 2];
  __shared__ float pw[NMAX / 2 + 1];
  __shared__ float dp[NMAX / 2 + 1];
  __shared__ float fe[MMAX][3];
  __shared__ float dmel[MMAX];
  const int s = blockIdx.y, tid = threadIdx.x, nb = n / 2 + 1;
  const float fmax = sr * 0.5f;
  for (int m = tid; m < n_mels; m += NT)
    for (int j = 0; j < 3; ++j) {
      const float mp = lin_f32(0.0f, m_max, n_mels + 2, m + j);
      fe[m][j] = 700.0f * (powf(10.0f, mp / 2595.0f) - 1.0f);
    }
  stage_twiddles(tw, n);
  const float g0 = ((go ? go[0] : 1.0f) * inv_nres) / (float)dsum[0];
  const float* xs = x + (size_t)s * ld;
  const float df = fmax / (float)(nb - 1);
  const int t0 = blockIdx.x * fpb, t1 = min(F, t0 + fpb);
  for (int t = t0; t < t1; ++t) {
    fft_frame(a, tw, xs, L, n, lg, hop, win, t);
    for (int k = tid; k < nb; k += NT) {
      const float2 c = a[k];
      pw[k] = __builtin_fmaf(c.x, c.x, c.y * c.y);
      dp[k] = 0.f;
    }
    __syncthreads();
    for (int m = tid; m < n_mels; m += NT) {
      const float* f = fe[m];
      const int lo = max(0, (int)floorf(f[0] / df) - 1), hi = min(nb - 1, (int)ceilf(f[2] / df) + 1);
      float acc = 0.f;
      for (int k = lo; k <= hi; ++k) {
        const float fk = lin_f32(0.0f, fmax, nb, k);
        const float down = -(f[0] - fk) / (f[1] - f[0]), up = (f[2] - fk) / (f[2] - f[1]);
        acc = __builtin_fmaf(pw[k], fmaxf(0.0f, fminf(down, up)), acc);
      }
      const float xm = (logf(1e-5f + acc) + 4.0f) * 0.25f;
      const float d = ym[((size_t)s * n_mels + m) * F + t] - xm;
      const float sg = (float)((d > 0.f) - (d < 0.f));
      dmel[m] = ((-sg * g0) * 0.25f) / (1e-5f + acc);
    }
    __syncthreads();
    // dP_k = sum_m fb[k][m] dmel_m: at most two filters are non-zero at a bin (adjacent triangles), so the
    // LDS float adds onto 0 are order independent
    for (int m = tid; m < n_mels; m += NT) {
      const float* f = fe[m];
      const int lo = max(0, (int)floorf(f[0] / df) - 1), hi = min(nb - 1, (int)ceilf(f[2] / df) + 1);
      for (int k = lo; k <= hi; ++k) {
        const float fk = lin_f32(0.0f, fmax, nb, k);
        const float down = -(f[0] - fk) / (f[1] - f[0]), up = (f[2] - fk) / (f[2] - f[1]);
        const float w = fmaxf(0.0f, fminf(down, up));
        if (w != 0.f) atomicAdd(&dp[k], w * dmel[m]);
      }
    }
    __syncthreads();
    // dX_k = 2 X_k dP_k into the bit-reversed slots of the inverse transform (X is read before any write:
    // each thread owns the slots it writes and reads them from a copy staged in pw's neighbour... use a
    // register pass: first read all, barrier, then write)
    float2 zr[NMAX / NT];
    int cnt = 0;
    for (int m = tid; m < n; m += NT, ++cnt) {
      const int k = brev(m, lg);
      float2 z = make_float2(0.f, 0.f);
      if (k < nb) {
        const float2 c = a[k];
        const float g2 = 2.0f * dp[k];
        z = make_float2(c.x * g2, c.y * g2);
      }
      zr[cnt] = z;
    }
    __syncthreads();
    cnt = 0;
    for (int m = tid; m < n; m += NT, ++cnt) a[m] = zr[cnt];
    frame_adjoint_out(a, tw, n, lg, win, fbuf + ((size_t)s * F + t) * win);
  }
}

__global__ void k_sum_d(const double* __restrict__ part, int nblk, double* __restrict__ d) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    double v = 0.0;
    for (int j = 0; j < nblk; ++j) v += part[2 * j + 1];
    d[0] = v;
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

int st_time_expand(const void* y, int S, int H, int W, int C, void* x3, int dtype, hipStream_t s, int We) {
  if (We < W) We = W;
  const long long n = (long long)H * We * C;
  if (S <= 0 || n <= 0) return ST_OK;
  dim3 grid((unsigned)((n + NT - 1) / NT), (unsigned)S);
  if (dtype == ST_FP32)
    hipLaunchKernelGGL(k_time_expand<float>, grid, dim3(NT), 0, s, reinterpret_cast<const float*>(y), H, W, C,
                       reinterpret_cast<float*>(x3), We);
  else if (dtype == ST_BF16)
    hipLaunchKernelGGL(k_time_expand<bf16_t>, grid, dim3(NT), 0, s, reinterpret_cast<const bf16_t*>(y), H, W, C,
                       reinterpret_cast<bf16_t*>(x3), We);
  else
    return ST_EDTYPE;
  return (int)hipGetLastError();
}

constexpr int kScBlocks = 1024;

int st_sc_sums(const float* xm, const float* ym, long long n, double* part, hipStream_t s) {
  if (n <= 0) return ST_EINVAL;
  hipLaunchKernelGGL(k_sc_sums, dim3(kScBlocks), dim3(NT), 0, s, xm, ym, n, part);
  return (int)hipGetLastError();
}

int st_sc_final(const double* part, int nres, double* loss, hipStream_t s) {
  hipLaunchKernelGGL(k_sc_final, dim3(1), dim3(64), 0, s, part, nres, kScBlocks, loss);
  return (int)hipGetLastError();
}

long long st_sc_part_bytes(int nres) { return (long long)nres * kScBlocks * 2 * sizeof(double); }

// ================================================================== training C-ABI (stts2_train.h)
extern "C" long long stts_stft_mag_workspace_bytes(int S, long long L, int n_fft, int win, int hop) {
  if (S <= 0 || L <= n_fft / 2 || log2_exact(n_fft) < 1 || n_fft > NMAX || win <= 0 || win > n_fft || hop <= 0)
    return ST_EINVAL;
  return (long long)S * st_stft_frames(L, hop) * win * sizeof(float);
}

extern "C" int stts_stft_mag_fwd(const float* wave, int S, long long L, long long ld, int n_fft, int win, int hop,
                                 float* mag, float* spec, void* stream) {
  if (stts_stft_mag_workspace_bytes(S, L, n_fft, win, hop) < 0 || !wave || !mag || !spec || ld < L || S > 65535)
    return ST_EINVAL;
  const int lg = log2_exact(n_fft);
  const long long F = st_stft_frames(L, hop);
  const int fpb = frames_per_block(S, F);
  hipLaunchKernelGGL(k_stft_spec, dim3((unsigned)((F + fpb - 1) / fpb), (unsigned)S), dim3(NT), 0, (hipStream_t)stream,
                     wave, L, ld, n_fft, lg, win, hop, (int)F, fpb, mag, reinterpret_cast<float2*>(spec));
  return (int)hipGetLastError();
}

extern "C" int stts_stft_mag_bwd(const float* spec, const float* dmag, int S, long long L, int n_fft, int win, int hop,
                                 float* dwave, void* ws, long long ws_bytes, void* stream) {
  const long long need = stts_stft_mag_workspace_bytes(S, L, n_fft, win, hop);
  if (need < 0) return (int)need;
  if (!spec || !dmag || !dwave || S > 65535) return ST_EINVAL;
  if (!ws || ws_bytes < need) return ST_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const int lg = log2_exact(n_fft);
  const long long F = st_stft_frames(L, hop);
  const int fpb = frames_per_block(S, F);
  float* fbuf = reinterpret_cast<float*>(ws);
  hipLaunchKernelGGL(k_stft_adj, dim3((unsigned)((F + fpb - 1) / fpb), (unsigned)S), dim3(NT), 0, s,
                     reinterpret_cast<const float2*>(spec), dmag, n_fft, lg, win, (int)F, fpb, fbuf);
  ST_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_ola_gather, dim3((unsigned)((L + NT - 1) / NT), (unsigned)S), dim3(NT), 0, s, fbuf, L, n_fft,
                     win, hop, (int)F, 0, dwave, L);
  return (int)hipGetLastError();
}

// workspace: [ym: B n_mels Fmax floats][partials: kScBlocks * 2 doubles][D: 1 double][fbuf: B Fmax win floats]
extern "C" long long stts_mrstft_bwd_workspace_bytes(int B, long long L, const int* n_ffts, const int* hops,
                                                     const int* wins, int n_res, int n_mels) {
  if (B <= 0 || L <= 0 || !n_ffts || !hops || !wins || n_res <= 0 || n_res > 16 || n_mels <= 0 || n_mels > MMAX)
    return ST_EINVAL;
  long long ym = 0, fb = 0;
  for (int r = 0; r < n_res; ++r) {
    if (hops[r] <= 0 || wins[r] <= 0 || wins[r] > n_ffts[r] || log2_exact(n_ffts[r]) < 1 || n_ffts[r] > NMAX ||
        L <= n_ffts[r] / 2)
      return ST_EINVAL;
    const long long F = st_stft_frames(L, hops[r]);
    ym = std::max(ym, (long long)B * n_mels * F * 4);
    fb = std::max(fb, (long long)B * F * wins[r] * 4);
  }
  auto al = [](long long v) { return (v + 255) & ~255LL; };
  return al(ym) + al(kScBlocks * 2 * 8) + 256 + al(fb);
}

extern "C" int stts_mrstft_loss_bwd(const float* x, const float* y, int B, long long L, long long ld, const int* n_ffts,
                                    const int* hops, const int* wins, int n_res, int sample_rate, int n_mels,
                                    const float* go, float* dx, void* ws, long long ws_bytes, void* stream) {
  const long long need = stts_mrstft_bwd_workspace_bytes(B, L, n_ffts, hops, wins, n_res, n_mels);
  if (need < 0) return (int)need;
  if (!x || !y || !dx || sample_rate <= 0 || ld < L || B > 65535) return ST_EINVAL;
  if (!ws || ws_bytes < need) return ST_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  auto al = [](long long v) { return (v + 255) & ~255LL; };
  long long ymb = 0;
  for (int r = 0; r < n_res; ++r) ymb = std::max(ymb, (long long)B * n_mels * st_stft_frames(L, hops[r]) * 4);
  char* base = reinterpret_cast<char*>(ws);
  float* ym = reinterpret_cast<float*>(base);
  double* part = reinterpret_cast<double*>(base + al(ymb));
  double* dsum = reinterpret_cast<double*>(base + al(ymb) + al(kScBlocks * 2 * 8));
  float* fbuf = reinterpret_cast<float*>(base + al(ymb) + al(kScBlocks * 2 * 8) + 256);
  const float sr = (float)sample_rate;
  const float m_max = (float)(2595.0 * log10(1.0 + (double)sr * 0.5 / 700.0));
  for (int r = 0; r < n_res; ++r) {
    const int n = n_ffts[r], lg = log2_exact(n), hop = hops[r], win = wins[r];
    const long long F = st_stft_frames(L, hop);
    ST_CHECK(st_logmel(y, B, L, ld, n, win, hop, n_mels, sr, ym, s));
    hipLaunchKernelGGL(k_sc_sums, dim3(kScBlocks), dim3(NT), 0, s, nullptr, ym, (long long)B * n_mels * F, part);
    ST_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_sum_d, dim3(1), dim3(64), 0, s, part, kScBlocks, dsum);
    ST_CHECK_HIP(hipGetLastError());
    const int fpb = frames_per_block(B, F);
    hipLaunchKernelGGL(k_mel_bwd, dim3((unsigned)((F + fpb - 1) / fpb), (unsigned)B), dim3(NT), 0, s, x, L, ld, n, lg,
                       win, hop, (int)F, fpb, n_mels, sr, m_max, ym, dsum, go, 1.0f / (float)n_res, fbuf);
    ST_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_ola_gather, dim3((unsigned)((L + NT - 1) / NT), (unsigned)B), dim3(NT), 0, s, fbuf, L, n, win,
                       hop, (int)F, r > 0 ? 1 : 0, dx, L);
    ST_CHECK_HIP(hipGetLastError());
  }
  return 0;
}
