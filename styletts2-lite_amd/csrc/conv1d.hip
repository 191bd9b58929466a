// Implicit-GEMM 1-D convolution on MFMA for gfx950 (both the dilated resblock convs,
// the AdainResBlk1d convs, the 1x1 shortcuts and — via a polyphase rewrite — the
// ConvTranspose1d upsamplers).  Reference ops restated: nn.Conv1d / nn.ConvTranspose1d
// inside Modules/hifigan.py:26-80, 272-347, 359-403 and Modules/istftnet.py:494-573.
//
// GEMM view (frames layout [B][L][C]):  out[q][n] = sum_{tap, ci} X[q*stride + tap*dil - pad][ci] * W[tap][ci][n]
//   rows M = output frames q, columns N = output channels (or (phase, channel) pairs for
//   a transposed conv), K = taps x input channels (contiguous in memory).
//
// One workgroup = 4 waves computes a BM x BN tile:
//   * per 32-channel chunk the input window [q0*stride - pad, ... + (BM-1)*stride + (KS-1)*dil]
//     is staged ONCE into LDS with the prologue (AdaIN / Snake / LReLU) applied on the way,
//     and re-read by every tap (dilated-conv halo reuse from LDS, not HBM);
//   * the packed weights of a group of taps are staged into LDS and shared by the waves;
//   * MFMA: bf16 -> v_mfma_f32_32x32x16_bf16, fp32 -> v_mfma_f32_32x32x2_f32 (exact f32 fma chain);
//   * epilogue fuses bias, residual add, 1/sqrt2 scale, the resblock average, tanh, the
//     iSTFTNet reflection pad, and the per-(utterance, channel) InstanceNorm statistics
//     (sum, sum of squares -> fp64 atomics) that the consumer's AdaIN prologue needs.
#include "common.h"
#include "kernels.h"
#include <type_traits>

namespace {

constexpr int BK = 32;

template <typename MT> struct Layout;
template <> struct Layout<bf16_t> {
  static constexpr int XP = 40;  // X row pitch (bf16 elements) = 80 B: conflict-free b128 reads
  static constexpr int WP = 40;  // W: [tap][n][WP]
};
template <> struct Layout<float> {
  static constexpr int XP = 33;  // odd pitch: conflict-free b32 column reads
  static constexpr int WP = 0;   // W: [tap][k][BN]
};

template <typename T, typename MT, int WAVES_M, int WAVES_N, int WM, int WN>
struct ConvCfg {
  static constexpr bool BF = std::is_same<MT, bf16_t>::value;
  static constexpr int BM = 32 * WM * WAVES_M;
  static constexpr int BN = 32 * WN * WAVES_N;
  static constexpr int XP = Layout<MT>::XP;
  static constexpr int WPITCH = BF ? Layout<MT>::WP : BN;
  static constexpr int W_TAP = BF ? BN * Layout<MT>::WP : BK * BN;  // elements per tap slice
  __host__ __device__ static int rows(const ConvParams& p) {
    return (BM - 1) * p.stride + ((p.KS - 1) / p.kw) * p.row_off + ((p.KS < p.kw ? p.KS : p.kw) - 1) * p.dil + 1;
  }
  __host__ __device__ static size_t xs_elems(const ConvParams& p) { return ((size_t)rows(p) * XP + 7) & ~(size_t)7; }
  static size_t lds_bytes(const ConvParams& p, int tg) {
    size_t b = (xs_elems(p) + (size_t)tg * W_TAP) * sizeof(MT) + 4 * BK * sizeof(float);
    const size_t red = (size_t)WAVES_M * BN * 2 * sizeof(double);
    return b > red ? b : red;
  }
};

__device__ __forceinline__ float snake_f(float v, float al, float inv_al) {
  const float s = sinf(al * v);
  return v + inv_al * (s * s);
}

template <typename T, typename MT, int WAVES_M, int WAVES_N, int WM, int WN>
__global__ void __launch_bounds__(256) conv1d_igemm_kernel(const ConvParams p) {
  using C = ConvCfg<T, MT, WAVES_M, WAVES_N, WM, WN>;
  constexpr int BM = C::BM, BN = C::BN, XP = C::XP, WPITCH = C::WPITCH, W_TAP = C::W_TAP;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int R = C::rows(p);
  MT* Xs = reinterpret_cast<MT*>(smem);
  MT* Ws = Xs + C::xs_elems(p);
  float* coef = reinterpret_cast<float*>(Ws + (size_t)p.tg * W_TAP);  // [4][BK]

  const int ntn = (p.N + BN - 1) / BN;
  const int ntm = (p.Lq + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int nt = t % ntn;
  const int mt = (t / ntn) % ntm;
  const int b = t / (ntn * ntm);
  const int q0 = mt * BM, n0 = nt * BN;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WAVES_N, wn = wid % WAVES_N;
  const int l32 = lane & 31, hi = lane >> 5;

  f32x16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const T* xb = reinterpret_cast<const T*>(p.x) + (size_t)b * p.x_bs;
  const int gr0 = q0 * p.stride - p.pad;
  const int Np = (p.N + 31) & ~31;
  const int mode = p.pro.mode;

  for (int c = 0; c < p.nchunks; ++c) {
    const int ci0 = c * BK;
    __syncthreads();  // previous chunk's LDS reads finished
    if (tid < BK) {
      const int ci = ci0 + tid;
      float m = 0.f, a = 1.f, be = 0.f, al = 1.f;
      if (ci < p.Cin) {
        if (mode & PRO_AFFINE) adain_coeffs(p.pro, b, ci, m, a, be);
        if (mode & PRO_SNAKE) al = p.pro.alpha[ci];
      }
      coef[tid] = m; coef[BK + tid] = a; coef[2 * BK + tid] = be; coef[3 * BK + tid] = al;
    }
    __syncthreads();
    // ---- stage the input window for this chunk (prologue applied) ----
    for (int u = tid; u < R * 4; u += 256) {
      const int r = u >> 2, g = u & 3;
      const int gr = gr0 + r, ch = ci0 + 8 * g;
      float v[8];
      if (gr >= 0 && gr < p.Lin && ch < p.Cin) {
        load8(xb + (size_t)gr * p.x_ld + ch, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int cl = 8 * g + j;
          float x = v[j];
          if (mode & PRO_AFFINE) x = (x - coef[cl]) * coef[BK + cl] + coef[2 * BK + cl];
          if (mode & PRO_SNAKE) { const float al = coef[3 * BK + cl]; x = snake_f(x, al, 1.0f / al); }
          if (mode & PRO_LRELU) x = x > 0.f ? x : x * p.pro.slope;
          v[j] = (ch + j < p.Cin) ? x : 0.f;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = 0.f;
      }
      MT* dst = Xs + r * XP + 8 * g;
      if constexpr (C::BF) {
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (bf16_t)v[j];
        *reinterpret_cast<bf16x8*>(dst) = o;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) dst[j] = v[j];
      }
    }
    // ---- taps, in groups whose packed weights fit the LDS budget ----
    for (int tap0 = 0; tap0 < p.KS; tap0 += p.tg) {
      const int ntap = min(p.tg, p.KS - tap0);
      if (tap0 > 0) __syncthreads();
      if constexpr (C::BF) {
        // packed bf16: [chunk][tap][Np][32]
        const int units = ntap * BN * 4;
        for (int u = tid; u < units; u += 256) {
          const int tl = u / (BN * 4), rem = u % (BN * 4), n = rem >> 2, g = rem & 3;
          const int gn = n0 + n;
          uint4 val = make_uint4(0, 0, 0, 0);
          if (gn < Np) {
            const bf16_t* src = reinterpret_cast<const bf16_t*>(p.w) +
                                (((size_t)c * p.KS + tap0 + tl) * Np + gn) * BK + 8 * g;
            val = *reinterpret_cast<const uint4*>(src);
          }
          *reinterpret_cast<uint4*>(Ws + (size_t)tl * W_TAP + n * WPITCH + 8 * g) = val;
        }
      } else {
        // packed fp32: [chunk][tap][32][Np]
        const int units = ntap * BK * (BN / 4);
        for (int u = tid; u < units; u += 256) {
          const int tl = u / (BK * (BN / 4)), rem = u % (BK * (BN / 4)), k = rem / (BN / 4), g = rem % (BN / 4);
          const int gn = n0 + 4 * g;
          float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
          if (gn < Np) {
            const float* src = reinterpret_cast<const float*>(p.w) + (((size_t)c * p.KS + tap0 + tl) * BK + k) * Np + gn;
            val = *reinterpret_cast<const float4*>(src);
          }
          *reinterpret_cast<float4*>(Ws + (size_t)tl * W_TAP + k * WPITCH + 4 * g) = val;
        }
      }
      __syncthreads();
      for (int tl = 0; tl < ntap; ++tl) {
        const int tap = tap0 + tl;
        const int toff = (tap / p.kw) * p.row_off + (tap % p.kw) * p.dil;
        const MT* wt = Ws + (size_t)tl * W_TAP;
        if constexpr (C::BF) {
#pragma unroll
          for (int kk = 0; kk < BK / 16; ++kk) {
            bf16x8 af[WM], bw[WN];
#pragma unroll
            for (int mi = 0; mi < WM; ++mi) {
              const int r = (wm * WM + mi) * 32 + l32;
              af[mi] = *reinterpret_cast<const bf16x8*>(Xs + (r * p.stride + toff) * XP + kk * 16 + hi * 8);
            }
#pragma unroll
            for (int ni = 0; ni < WN; ++ni) {
              const int n = (wn * WN + ni) * 32 + l32;
              bw[ni] = *reinterpret_cast<const bf16x8*>(wt + n * WPITCH + kk * 16 + hi * 8);
            }
#pragma unroll
            for (int mi = 0; mi < WM; ++mi)
#pragma unroll
              for (int ni = 0; ni < WN; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi], bw[ni], acc[mi][ni], 0, 0, 0);
          }
        } else {
#pragma unroll 4
          for (int kk = 0; kk < BK / 2; ++kk) {
            float af[WM], bw[WN];
#pragma unroll
            for (int mi = 0; mi < WM; ++mi) {
              const int r = (wm * WM + mi) * 32 + l32;
              af[mi] = Xs[(r * p.stride + toff) * XP + 2 * kk + hi];
            }
#pragma unroll
            for (int ni = 0; ni < WN; ++ni) {
              const int n = (wn * WN + ni) * 32 + l32;
              bw[ni] = wt[(2 * kk + hi) * WPITCH + n];
            }
#pragma unroll
            for (int mi = 0; mi < WM; ++mi)
#pragma unroll
              for (int ni = 0; ni < WN; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[mi], bw[ni], acc[mi][ni], 0, 0, 0);
          }
        }
      }
    }
  }

  // ---------------- epilogue ----------------
  const bool want_stats = p.stats != nullptr;
  double s_sum[WN], s_sq[WN];
  T* yT = reinterpret_cast<T*>(p.y) + (size_t)b * p.y_bs;
  float* yF = reinterpret_cast<float*>(p.y) + (size_t)b * p.y_bs;
  const T* resb = p.res ? reinterpret_cast<const T*>(p.res) + (size_t)b * p.res_bs : nullptr;
  const T* accb = p.accb ? reinterpret_cast<const T*>(p.accb) + (size_t)b * p.acc_bs : nullptr;
#pragma unroll
  for (int ni = 0; ni < WN; ++ni) {
    s_sum[ni] = 0.0;
    s_sq[ni] = 0.0;
    const int n = n0 + (wn * WN + ni) * 32 + l32;
    if (n >= p.N) continue;
    const int ph = n / p.Cout, co = n - ph * p.Cout;
    const float bias = p.bias ? p.bias[co] : 0.f;
    float ls = 0.f, lq = 0.f;
#pragma unroll
    for (int mi = 0; mi < WM; ++mi) {
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int q = q0 + (wm * WM + mi) * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * hi;
        if (q >= p.Lq) continue;
        const int o = q * p.up + ph - p.opad;
        if (o < 0 || o >= p.Lout) continue;
        const int orow = o + p.y_row_off;
        if (p.zc_period && (o % p.zc_period) >= p.zc_valid) {  // padded-image border column
          if (p.y_f32) yF[(size_t)orow * p.y_ld + co] = 0.f;
          else yT[(size_t)orow * p.y_ld + co] = from_f32<T>(0.f);
          continue;
        }
        const float v0 = acc[mi][ni][reg] + bias;
        float v = v0;
        if (resb) v += to_f32(resb[(size_t)(orow >> p.res_shift) * p.res_ld + co]);
        v *= p.out_scale;
        if (accb) {
          v = to_f32(accb[(size_t)orow * p.acc_ld + co]) + v;
          if (p.acc_div != 0.f) v = v / p.acc_div;
        }
        if (p.epi_tanh) v = tanhf(v);
        float vs;
        if (p.y_f32) {
          yF[(size_t)orow * p.y_ld + co] = v;
          vs = v;
        } else {
          const T tv = from_f32<T>(v);
          yT[(size_t)orow * p.y_ld + co] = tv;
          vs = to_f32(tv);
        }
        ls += vs;
        lq += vs * vs;
        if (p.reflect_front && o == 1) {  // iSTFTNet ReflectionPad1d((1,0)) (istftnet.py:538, 558-559)
          float w = v0;
          if (resb) w += to_f32(resb[(size_t)0 * p.res_ld + co]);
          const T tw = from_f32<T>(w);
          yT[co] = tw;
          const float ws = to_f32(tw);
          ls += ws;
          lq += ws * ws;
        }
      }
    }
    s_sum[ni] = ls;
    s_sq[ni] = lq;
  }
  if (!want_stats) return;
  // combine lane halves (same column), then waves along M via LDS, then fp64 atomics
  double* red = reinterpret_cast<double*>(smem);
  __syncthreads();
#pragma unroll
  for (int ni = 0; ni < WN; ++ni) {
    double a = s_sum[ni] + __shfl_xor(s_sum[ni], 32);
    double q = s_sq[ni] + __shfl_xor(s_sq[ni], 32);
    if (hi == 0) {
      const int nl = (wn * WN + ni) * 32 + l32;
      red[((size_t)wm * BN + nl) * 2 + 0] = a;
      red[((size_t)wm * BN + nl) * 2 + 1] = q;
    }
  }
  __syncthreads();
  if (tid < BN) {
    const int n = n0 + tid;
    if (n < p.N) {
      double a = 0.0, q = 0.0;
#pragma unroll
      for (int w = 0; w < WAVES_M; ++w) {
        a += red[((size_t)w * BN + tid) * 2 + 0];
        q += red[((size_t)w * BN + tid) * 2 + 1];
      }
      const int co = n % p.Cout;
      atomicAdd(p.stats + ((size_t)b * p.stats_ld + co) * 2 + 0, a);
      atomicAdd(p.stats + ((size_t)b * p.stats_ld + co) * 2 + 1, q);
    }
  }
}

template <typename T, typename MT, int WAVES_M, int WAVES_N, int WM, int WN>
int launch_cfg(ConvParams p, hipStream_t stream) {
  using C = ConvCfg<T, MT, WAVES_M, WAVES_N, WM, WN>;
  constexpr int LDS_MAX = 160 * 1024;
  constexpr int WBUDGET = 48 * 1024;
  const size_t wtap = (size_t)C::W_TAP * sizeof(MT);
  int tg = (int)(WBUDGET / wtap);
  if (tg < 1) tg = 1;
  if (tg > p.KS) tg = p.KS;
  while (tg > 1 && C::lds_bytes(p, tg) > (size_t)LDS_MAX) --tg;
  const size_t lds = C::lds_bytes(p, tg);
  if (lds > (size_t)LDS_MAX) return ST_EINVAL;
  p.tg = tg;
  static bool attr_set = false;
  auto kern = conv1d_igemm_kernel<T, MT, WAVES_M, WAVES_N, WM, WN>;
  if (!attr_set) {
    ST_CHECK_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX));
    attr_set = true;
  }
  const long long ntn = (p.N + C::BN - 1) / C::BN, ntm = (p.Lq + C::BM - 1) / C::BM;
  const long long grid = ntn * ntm * p.B;
  if (grid <= 0) return ST_OK;
  if (grid > 0x7fffffffLL) return ST_EINVAL;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(256), lds, stream, p);
  return (int)hipGetLastError();
}

template <typename T, typename MT>
int launch_typed(const ConvParams& p, hipStream_t stream) {
  if (p.stride > 1) return launch_cfg<T, MT, 2, 2, 1, 2>(p, stream);  // BM 64 x BN 128 (short window)
  if (p.N <= 32) return launch_cfg<T, MT, 4, 1, 2, 1>(p, stream);     // BM 256 x BN 32
  if (p.N <= 64) return launch_cfg<T, MT, 4, 1, 1, 2>(p, stream);     // BM 128 x BN 64
  return launch_cfg<T, MT, 2, 2, 2, 2>(p, stream);                    // BM 128 x BN 128
}

}  // namespace

int st_conv1d(const ConvParams& p, int dtype, hipStream_t stream) {
  if (p.B <= 0 || p.Lq <= 0 || p.N <= 0) return ST_OK;
  if (p.KS <= 0 || p.stride <= 0 || p.dil <= 0 || p.Cout <= 0 || p.up <= 0) return ST_EINVAL;
  ConvParams q = p;
  if (q.kw <= 0) q.kw = q.KS;
  if (p.x_ld % 8 != 0 || p.nchunks * BK < p.Cin) return ST_EINVAL;
  if (dtype == ST_FP32) return launch_typed<float, float>(q, stream);
  if (dtype == ST_BF16) return launch_typed<bf16_t, bf16_t>(q, stream);
  return ST_EDTYPE;
}
