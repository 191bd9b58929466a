// Pointwise (1x1) conv engine, bf16: y[b][q][n] = epi(sum_k pro(x[b][q][k]) * W[n][k]) — the
// AdainResBlk1d conv1x1 shortcuts (hifigan.py:380-383, 398-400) and the Vocos ConvNeXt pwconv1 /
// pwconv2 and ISTFTHead.out Linears (vocos.py:47-49, 268).  On conv1d_igemm these plain GEMMs ran at
// 0.06 of the bf16 MFMA peak, 87 us of a 252 us launch with every phase switched off
// (profiles/r02_vocos_phases.txt): that engine's per-step machinery (tap groups, window halos, two
// register prefetch sets) is dead weight at K = 1.
//
// Tile = 128 frames x 128 output channels, 4 waves (2 x 2, each 64 x 64 = 2 x 2 fragments of
// v_mfma_f32_32x32x16_bf16), K in 32-channel chunks through a 2-stage LDS ring with the next chunk
// prefetched in registers (one barrier per chunk), ~40 KB of LDS so several blocks share a CU.  The
// optional AdaIN prologue (per-(utterance, channel) affine from the producer's statistics) is applied
// while the frames chunk is staged; channels >= Cin are zero.  Epilogue from registers (lane = 16
// consecutive channels of one frame, the packed-row permutation of st_pack_conv): bias, residual x
// out_scale, erf-GELU, bf16 stores.  One tile per block; grid = tiles.
#include "common.h"
#include "conv_common.h"
#include "kernels.h"

namespace {

constexpr int BM = 128, BN = 128, NT = 256, XP = 40, WP = 40;

template <bool AFFINE>
__global__ void __launch_bounds__(NT) k_pwgemm(const ConvParams p, int ntm, int ntn) {
  __shared__ __attribute__((aligned(16))) bf16_t Xs[2][BM * XP];
  __shared__ __attribute__((aligned(16))) bf16_t Ws[2][BN * WP];
  extern __shared__ __attribute__((aligned(16))) float coef[];  // AFFINE: a[Cin_pad], m[Cin_pad]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, l32 = lane & 31, hi = lane >> 5;
  const int wm = wid >> 1, wn = wid & 1;
  // tile order: n fastest (consecutive blocks share the frames chunk in L2)
  const int bid = blockIdx.x;
  const int tn = bid % ntn, rest = bid / ntn, tm = rest % ntm, b = rest / ntm;
  const int q0 = tm * BM, n0 = tn * BN;
  const int nch = p.nchunks, cpad = nch * 32;
  if constexpr (AFFINE) {
    for (int c = tid; c < cpad; c += NT) {
      float mm = 0.f, aa = 0.f, be = 0.f;
      if (c < p.Cin) adain_coeffs(p.pro, b, c, mm, aa, be);
      coef[c] = aa;
      coef[cpad + c] = be - mm * aa;  // v * a + (beta - mean * a)
    }
  }
  const Rsrc rx = make_rsrc(reinterpret_cast<const bf16_t*>(p.x) + (size_t)b * p.x_bs,
                            (unsigned)((size_t)p.Lin * p.x_ld * 2));
  const Rsrc rw = make_rsrc(p.w, (unsigned)((size_t)nch * ((p.N + 31) & ~31) * 32 * 2));
  const int Np = (p.N + 31) & ~31;
  // staging units: 128 rows x 4 16-byte units for X and for W; thread tid owns units tid, tid + 256
  uint4 px[2], pw[2];
  auto issue = [&](int c) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int u = tid + k * NT, r = u >> 2, g = u & 3;
      const int q = q0 + r;
      px[k] = bload16(rx, q < p.Lin ? (unsigned)((q * p.x_ld + c * 32 + 8 * g) * 2) : OOB);
      const int n = n0 + r;
      pw[k] = bload16(rw, n < Np ? (unsigned)((((size_t)c * Np + n) * 32 + 8 * g) * 2) : OOB);
    }
  };
  auto stage = [&](int c, int s) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int u = tid + k * NT, r = u >> 2, g = u & 3;
      uint4 o = px[k];
      const int ch = c * 32 + 8 * g;
      if (AFFINE || ch + 8 > p.Cin) {
        bf16x8 v;
        __builtin_memcpy(&v, &o, 16);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float f = (float)v[j];
          if constexpr (AFFINE) f = __builtin_fmaf(f, coef[ch + j], coef[cpad + ch + j]);
          if (ch + j >= p.Cin) f = 0.f;
          v[j] = (bf16_t)f;
        }
        __builtin_memcpy(&o, &v, 16);
      }
      *reinterpret_cast<uint4*>(&Xs[s][r * XP + 8 * g]) = o;
      // packed weights: physical unit g of row n holds logical unit g ^ ((n >> 2) & 3)
      const int n = n0 + r;
      *reinterpret_cast<uint4*>(&Ws[s][r * WP + 8 * (g ^ ((n >> 2) & 3))]) = pw[k];
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;

  if constexpr (AFFINE) __syncthreads();  // coefficients
  issue(0);
  stage(0, 0);
  if (nch > 1) issue(1);
  __syncthreads();
  const bf16_t* xw0 = &Xs[0][(wm * 64 + l32) * XP + hi * 8];
  const bf16_t* ww0 = &Ws[0][(wn * 64 + l32) * WP + hi * 8];
  for (int c = 0; c < nch; ++c) {
    const int s = c & 1;
    const bf16_t* xw = xw0 + s * BM * XP;
    const bf16_t* ww = ww0 + s * BN * WP;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 wa[2], xb[2];
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) wa[ni] = *reinterpret_cast<const bf16x8*>(ww + ni * 32 * WP + kk * 16);
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) xb[mi] = *reinterpret_cast<const bf16x8*>(xw + mi * 32 * XP + kk * 16);
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[ni], xb[mi], acc[mi][ni], 0, 0, 0);
    }
    if (c + 1 < nch) {
      stage(c + 1, s ^ 1);  // the other buffer: every wave finished it before the last barrier
      if (c + 2 < nch) issue(c + 2);
    }
    __syncthreads();
  }

  // epilogue: lane = frame l32 of block mi, channels n0 + wn * 64 + ni * 32 + 16 * hi + r
  bf16_t* yb = reinterpret_cast<bf16_t*>(p.y) + (size_t)b * p.y_bs;
  const bf16_t* rb = p.res ? reinterpret_cast<const bf16_t*>(p.res) + (size_t)b * p.res_bs : nullptr;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    const int q = q0 + wm * 64 + mi * 32 + l32;
    if (q >= p.Lout) continue;
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int nb = n0 + wn * 64 + ni * 32 + 16 * hi;
      if (nb >= p.N) continue;
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = acc[mi][ni][r] + (p.bias ? p.bias[nb + r] : 0.f);
      if (rb) {
        float r16[16];
        load16(rb + (size_t)q * p.res_ld + nb, r16);
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = (v[r] + r16[r]) * p.out_scale;
      }
      if (p.epi_gelu) {
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = 0.5f * v[r] * (1.0f + erff(v[r] * 0.7071067811865476f));
      }
      store16(yb + (size_t)q * p.y_ld + nb, v);
    }
  }
}

}  // namespace

int g_opt_pw = 1;

bool st_pw_eligible(const ConvParams& p, int dtype) {
  if (!g_opt_pw || dtype != ST_BF16) return false;
  if (p.KS != 1 || p.stride != 1 || p.up != 1 || p.opad != 0 || p.pad != 0 || p.dil != 1 || p.row_off != 0) return false;
  if (p.kw != 0 && p.kw != 1) return false;
  if (p.N != p.Cout || p.N % 64 != 0 || p.Lq != p.Lin || p.Lout != p.Lq) return false;
  if (p.stats || p.accb || p.y_f32 || p.y_row_off || p.epi_tanh || p.epi_lrelu || p.reflect_front || p.zc_period ||
      p.res_shift)
    return false;
  if (p.pro.mode != 0 && p.pro.mode != PRO_AFFINE) return false;
  if (p.x_ld % 8 || p.y_ld % 8 || (p.res && p.res_ld % 8)) return false;
  return true;
}

int st_pw(const ConvParams& p, hipStream_t stream) {
  const int ntm = (p.Lq + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const long long blocks = (long long)ntm * ntn * p.B;
  if (blocks <= 0) return ST_OK;
  if (blocks > 0x7fffffffLL) return ST_EINVAL;
  if (p.pro.mode & PRO_AFFINE) {
    const size_t lds = (size_t)p.nchunks * 32 * 2 * sizeof(float);
    hipLaunchKernelGGL(k_pwgemm<true>, dim3((unsigned)blocks), dim3(NT), lds, stream, p, ntm, ntn);
  } else {
    hipLaunchKernelGGL(k_pwgemm<false>, dim3((unsigned)blocks), dim3(NT), 0, stream, p, ntm, ntn);
  }
  return (int)hipGetLastError();
}
