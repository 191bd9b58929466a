// Style front-end: the log-mel spectrogram of Preprocess.wave_preprocess (reference
// inference.py:43-49), i.e. torchaudio MelSpectrogram(n_mels=80, n_fft=2048, win_length=1200,
// hop_length=300) at its defaults (sample_rate 16000 -> f_max 8000 over the 1025 one-sided bins,
// periodic Hann window zero-padded to n_fft, center=True with reflect padding, power 2, HTK mel
// scale, no filter normalisation), then (log(1e-5 + mel) - (-4)) / 4.
//
// A workgroup walks a few frames of one utterance: the frame's 2048 padded, windowed samples are
// transformed by a radix-2 FFT in LDS (twiddles from a float64-built table, so the rounding is
// that of an fp32 FFT, like torch.stft's), the power spectrum goes back to LDS and 80 threads
// apply their triangular filter (weights recomputed from the band edges) over its bin range.  The
// window and twiddle tables are built into the caller's workspace by a setup kernel on every
// call -- the library allocates nothing.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int NFFT = 2048, WIN = 1200, HOP = 300, NBIN = NFFT / 2 + 1, NMEL = 80;
constexpr int WOFF = (NFFT - WIN) / 2;  // torch.stft centres the shorter window in n_fft: 424
constexpr int NT = 256;

// workspace layout (floats / ints)
constexpr size_t T_WIN = 0;                      // [WIN]  periodic Hann
constexpr size_t T_COS = T_WIN + WIN;            // [NFFT] cos(2 pi j / NFFT)
constexpr size_t T_SIN = T_COS + NFFT;           // [NFFT] sin(2 pi j / NFFT)
constexpr size_t T_END = T_SIN + NFFT;

// torch.linspace(start, end, steps) in fp32: the first half counts up from start, the second
// half down from end (aten/src/ATen/native/cpu/RangeFactoriesKernel.cpp)
__device__ float linspace_f32(float start, float end, int steps, int i) {
  const float step = (end - start) / (float)(steps - 1);
  const int half = steps / 2;
  return i < half ? start + step * (float)i : end - step * (float)(steps - i - 1);
}

// mel band edges f[0..2] of filter m (HTK scale, 82 points linearly spaced in mel)
__device__ void mel_edges(int m, float (&f)[3]) {
  const float m_max = 2595.0f * log10f(1.0f + 8000.0f / 700.0f);
  for (int j = 0; j < 3; ++j) {
    const float mp = linspace_f32(0.0f, m_max, NMEL + 2, m + j);
    f[j] = 700.0f * (powf(10.0f, mp / 2595.0f) - 1.0f);
  }
}

// one thread per window / twiddle entry
__global__ void k_mel_tables(float* tab) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < WIN) {  // torch.hann_window(1200, periodic=True) = 0.5 - 0.5 cos(2 pi n / 1200)
    tab[T_WIN + i] = (float)(0.5 - 0.5 * cospi(2.0 * i / WIN));
  }
  if (i < NFFT) {
    double s, c;
    sincospi(2.0 * i / NFFT, &s, &c);
    tab[T_COS + i] = (float)c;
    tab[T_SIN + i] = (float)s;
  }
}

// weight of DFT bin k in mel filter m with band edges f[0..2]:
// torchaudio.functional.melscale_fbanks(1025, 0, 8000, 80, 16000, None, "htk")
__device__ __forceinline__ float mel_weight(const float* f, int k) {
  const float fk = linspace_f32(0.0f, 8000.0f, NBIN, k);  // = 7.8125 k exactly
  const float down = -(f[0] - fk) / (f[1] - f[0]), up = (f[2] - fk) / (f[2] - f[1]);
  return fmaxf(0.0f, fminf(down, up));
}

// bit reversal of an 11-bit index
__device__ __forceinline__ int brev11(int n) { return (int)(__brev((unsigned)n) >> 21); }

// FPB consecutive frames of one utterance per workgroup (the twiddle table is staged once).
// Per frame: the 2048 padded, windowed samples go to LDS in bit-reversed order, an in-place
// radix-2 decimation-in-time FFT runs 11 stages (4 butterflies per thread per stage, a barrier
// between stages), then |X[k]|^2 for k <= 1024 and the 80 triangular filters.
__global__ void __launch_bounds__(NT) k_logmel(const float* __restrict__ wave, long long L, long long ld, int F,
                                                int fpb, const float* __restrict__ tab, float* __restrict__ out) {
  __shared__ float2 a[NFFT];
  __shared__ float2 tw[NFFT / 2];
  __shared__ float pw[NBIN];
  __shared__ float fe[NMEL][3];
  const int b = blockIdx.y, tid = threadIdx.x;
  if (tid < NMEL) mel_edges(tid, fe[tid]);
  const float* x = wave + (size_t)b * ld;
  for (int j = tid; j < NFFT / 2; j += NT) tw[j] = make_float2(tab[T_COS + j], tab[T_SIN + j]);
  const int t0 = blockIdx.x * fpb, t1 = min(F, t0 + fpb);
  for (int t = t0; t < t1; ++t) {
    // frame t = padded samples [t*HOP, t*HOP + NFFT) of the signal reflect-padded by NFFT/2; the
    // window covers n in [WOFF, WOFF + WIN) of it, zeros elsewhere
    const long long base = (long long)t * HOP - NFFT / 2;
    for (int m = tid; m < NFFT; m += NT) {  // LDS slot m <- sample brev(m): conflict-free LDS
      const int n = brev11(m);                // writes, gathered (cached) global reads
      float v = 0.f;
      if (n >= WOFF && n < WOFF + WIN) {
        long long j = base + n;
        if (j < 0) j = -j;
        if (j >= L) j = 2 * (L - 1) - j;
        v = x[j] * tab[T_WIN + n - WOFF];
      }
      a[m] = make_float2(v, 0.f);
    }
    __syncthreads();
#pragma unroll 1
    for (int lg = 0; lg < 11; ++lg) {  // butterflies of span h = 2^lg
      const int h = 1 << lg;
      for (int j = tid; j < NFFT / 2; j += NT) {
        const int pos = j & (h - 1), i0 = ((j >> lg) << (lg + 1)) + pos, i1 = i0 + h;
        const float2 w = tw[pos << (10 - lg)];  // exp(-2 pi i pos / 2h) = cos - i sin
        const float2 u = a[i0], v = a[i1];
        const float tr = w.x * v.x + w.y * v.y, ti = w.x * v.y - w.y * v.x;
        a[i0] = make_float2(u.x + tr, u.y + ti);
        a[i1] = make_float2(u.x - tr, u.y - ti);
      }
      __syncthreads();
    }
    for (int k = tid; k < NBIN; k += NT) {
      const float2 c = a[k];
      pw[k] = __builtin_fmaf(c.x, c.x, c.y * c.y);
    }
    __syncthreads();
    if (tid < NMEL) {  // the weights are recomputed (no table reads): bins strictly inside the band
      const float* f = fe[tid];
      const int lo = max(0, (int)floorf(f[0] / 7.8125f) - 1), hi = min(NBIN - 1, (int)ceilf(f[2] / 7.8125f) + 1);
      float acc = 0.f;
      for (int k = lo; k <= hi; ++k) acc = __builtin_fmaf(pw[k], mel_weight(f, k), acc);
      out[((size_t)b * NMEL + tid) * F + t] = (logf(1e-5f + acc) + 4.0f) * 0.25f;
    }
    // the next frame's loads overwrite a[] only (pw[] is rewritten after two more barriers)
  }
}

}  // namespace

long long st_mel_frames(long long L) { return L > NFFT / 2 ? 1 + L / HOP : 0; }

long long st_mel_workspace_bytes() { return (long long)(T_END * sizeof(float)); }

int st_wave_preprocess(const float* wave, int B, long long L, long long ld, float* mel, void* ws, long long ws_bytes,
                       hipStream_t stream) {
  if (B <= 0) return ST_OK;
  if (!wave || !mel || L <= NFFT / 2 || ld < L) return ST_EINVAL;  // reflect padding needs L > 1024
  if (!ws || ws_bytes < st_mel_workspace_bytes()) return ST_EWORKSPACE;
  const long long F = st_mel_frames(L);
  if (F > 0x7fffffff || B > 65535) return ST_EINVAL;
  float* tab = static_cast<float*>(ws);
  hipLaunchKernelGGL(k_mel_tables, dim3((NFFT + NT - 1) / NT), dim3(NT), 0, stream, tab);
  ST_CHECK_HIP(hipGetLastError());
  // about 2048 workgroups in all, each reusing its staged twiddles over fpb frames
  const long long want = (long long)B * F / 2048;
  const int fpb = (int)(want < 1 ? 1 : want > 64 ? 64 : want);
  const unsigned gx = (unsigned)((F + fpb - 1) / fpb);
  hipLaunchKernelGGL(k_logmel, dim3(gx, (unsigned)B), dim3(NT), 0, stream, wave, L, ld, (int)F, fpb,
                     (const float*)tab, mel);
  return (int)hipGetLastError();
}
