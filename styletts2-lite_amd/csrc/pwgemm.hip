// Short-conv GEMM engine, bf16: 1- and 2-tap convs as one GEMM each,
//   y[b][o(q, n)][n % Cout] = epi(sum_{t, k} pro(x[b][q + t - pad][k]) * W[t][n][k]),
// serving the AdainResBlk1d conv1x1 shortcuts (hifigan.py:380-383, 398-400), asr_res (:438-440),
// the Vocos ConvNeXt pwconv1 / pwconv2 and ISTFTHead.out Linears (vocos.py:47-49, 268), and the
// generator's ConvTranspose1d upsamplers (hifigan.py:292-294, istftnet.py:516-519) in their polyphase
// form (2 taps, N = u * Cout, output row o = q * u + n / Cout - opad).  On conv1d_igemm these ran at
// 0.06-0.25 of their roofline, with 87 of 252 us left when every phase was switched off
// (profiles/r02_vocos_phases.txt): that engine's tap-group / halo / two-register-set machinery is
// dead weight at one or two taps.
//
// Tile = 128 GEMM rows (input-rate frames) x 128 columns, 4 waves (2 x 2, each 64 x 64 = 2 x 2
// fragments of v_mfma_f32_32x32x16_bf16); K in 32-channel chunks through a 2-stage LDS ring (window of
// 128 + taps - 1 rows, all taps' weight slices), the next chunk prefetched in registers, one barrier
// per chunk, ~60 KB of LDS so two or more blocks share a CU.  The prologue (AdaIN affine / Snake /
// LeakyReLU, the per-(utterance, channel) coefficients in LDS) is applied while a chunk is staged;
// rows outside [0, Lin) and channels >= Cin are zero after it (the conv's zero padding).  Epilogue from
// registers (lane = 16 consecutive columns of one row, the packed-row permutation of st_pack_conv, so
// the 16 share one output row o): bias, residual x out_scale, erf-GELU, bf16 stores, and InstanceNorm
// statistics of the values (fp32, before the store) reduced across the wave's 32 rows, one fp64
// atomic pair per (wave, channel).  One tile per block; grid = tiles, columns fastest.
#include "common.h"
#include "conv_common.h"
#include "kernels.h"

namespace {

constexpr int BM = 128, BN = 128, NT = 256, XP = 40, WP = 40;

template <int TAPS>
__global__ void __launch_bounds__(NT, 2) k_pwgemm(const ConvParams p, int ntm, int ntn) {
  constexpr int XR = BM + TAPS - 1;                   // window rows
  constexpr int XU = (XR * 4 + NT - 1) / NT;          // 16-byte window units per thread
  __shared__ __attribute__((aligned(16))) bf16_t Xs[2][XR * XP];
  __shared__ __attribute__((aligned(16))) bf16_t Ws[2][TAPS * BN * WP];
  extern __shared__ __attribute__((aligned(16))) float coef[];  // [4][cpad]: m, a, alpha, 1/alpha
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, l32 = lane & 31, hi = lane >> 5;
  const int wm = wid >> 1, wn = wid & 1;
  const int nch = p.nchunks, cpad = nch * 32, mode = p.pro.mode;
  const int Np = (p.N + 31) & ~31;
  const Rsrc rw = make_rsrc(p.w, (unsigned)((size_t)nch * TAPS * Np * 32 * 2));
  // persistent: a contiguous range of tiles ordered (utterance, column tile, row tile), rows fastest,
  // so the statistics of a (utterance, column tile) accumulate in registers across many tiles and
  // leave as one atomic pair per channel (per-tile atomics all hitting the same few addresses
  // serialised: profiles/r02_layers_bf16_b32_pw1.txt)
  const long long total = (long long)ntm * ntn * p.B;
  // tile ranges (kernels.h tile_range: one per workgroup, or utterance-relative segments)
  const int nv = tile_nv(p, p.B);
  float st_s[2][16], st_q[2][16];
#pragma unroll
  for (int ni = 0; ni < 2; ++ni)
#pragma unroll
    for (int r = 0; r < 16; ++r) st_s[ni][r] = st_q[ni][r] = 0.f;
  int cur_b = -1, cur_key = -1;
  auto flush = [&](int b, int n0) __attribute__((always_inline)) {
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int nb = n0 + wn * 64 + ni * 32 + 16 * hi;
      const int co = nb % p.Cout;
      float a, q;
      stat_bfly16(st_s[ni], st_q[ni], l32, a, q);
      if (nb < p.N && l32 < 16) {
        double* d = stats_slot(p, blockIdx.x) + ((size_t)b * p.stats_ld + co + l32) * ST_W;
        fx_add(d, a);
        fx_add(d + 2, q);
      }
    }
  };
  for (int vb = blockIdx.x; vb < nv; vb += gridDim.x) {
  long long tbeg, tend;
  tile_range(p, vb, nv, total, (long long)ntm * ntn, tbeg, tend);
  for (long long t = tbeg; t < tend; ++t) {
    const int tm = (int)(t % ntm), tn = (int)((t / ntm) % ntn), b = (int)(t / ((long long)ntm * ntn));
    const int q0 = tm * BM, n0 = tn * BN;
    const int key = b * ntn + tn;
    if (key != cur_key) {
      if (cur_key >= 0 && p.stats) flush(cur_b, (cur_key % ntn) * BN);
      cur_key = key;
    }
    if (b != cur_b) {
      if (mode) {
        __syncthreads();  // every wave is done staging with the previous utterance's coefficients
        for (int c = tid; c < cpad; c += NT) {
          float mm = 0.f, aa = 1.f, be = 0.f, al = 1.f;
          if (c < p.Cin) {
            if (mode & PRO_AFFINE) adain_coeffs(p.pro, b, c, mm, aa, be);
            if (mode & PRO_SNAKE) al = p.pro.alpha[c];
          }
          coef[c] = be - mm * aa;  // v * a + (beta - mean * a)
          coef[cpad + c] = aa;
          coef[2 * cpad + c] = al;
          coef[3 * cpad + c] = 1.0f / al;  // the reference's (1 / alpha)
        }
        __syncthreads();
      }
      cur_b = b;
    }
    const Rsrc rx = make_rsrc(reinterpret_cast<const bf16_t*>(p.x) + (size_t)b * p.x_bs,
                              (unsigned)((size_t)p.Lin * p.x_ld * 2));
    const int r0 = q0 - p.pad;  // window row 0 = input row r0
    uint4 px[XU], pw[TAPS][2];
    auto issue = [&](int c) __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < XU; ++k) {
        const int u = tid + k * NT, r = u >> 2, g = u & 3, gr = r0 + r;
        px[k] = bload16(rx, (u < XR * 4 && gr >= 0 && gr < p.Lin) ? (unsigned)((gr * p.x_ld + c * 32 + 8 * g) * 2) : OOB);
      }
#pragma unroll
      for (int tp = 0; tp < TAPS; ++tp)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int u = tid + k * NT, r = u >> 2, g = u & 3, n = n0 + r;
          pw[tp][k] = bload16(rw, n < Np ? (unsigned)(((((size_t)c * TAPS + tp) * Np + n) * 32 + 8 * g) * 2) : OOB);
        }
    };
    auto stage = [&](int c, int s) __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < XU; ++k) {
        const int u = tid + k * NT, r = u >> 2, g = u & 3, gr = r0 + r;
        if (u >= XR * 4) continue;
        uint4 o = px[k];
        const int ch = c * 32 + 8 * g;
        const bool row_ok = gr >= 0 && gr < p.Lin;
        if (mode || ch + 8 > p.Cin || !row_ok) {
          bf16x8 v;
          __builtin_memcpy(&v, &o, 16);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float f = (float)v[j];
            if (mode & PRO_AFFINE) f = __builtin_fmaf(f, coef[cpad + ch + j], coef[ch + j]);
            if (mode & PRO_SNAKE) {
              const float sn = __sinf(coef[2 * cpad + ch + j] * f);
              f = __builtin_fmaf(sn * sn, coef[3 * cpad + ch + j], f);
            }
            if (mode & PRO_LRELU) f = f > 0.f ? f : f * p.pro.slope;
            if (ch + j >= p.Cin || !row_ok) f = 0.f;
            v[j] = (bf16_t)f;
          }
          __builtin_memcpy(&o, &v, 16);
        }
        *reinterpret_cast<uint4*>(&Xs[s][r * XP + 8 * g]) = o;
      }
      // packed weights: physical unit g of row n holds logical unit g ^ ((n >> 2) & 3)
#pragma unroll
      for (int tp = 0; tp < TAPS; ++tp)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int u = tid + k * NT, r = u >> 2, g = u & 3, n = n0 + r;
          *reinterpret_cast<uint4*>(&Ws[s][(tp * BN + r) * WP + 8 * (g ^ ((n >> 2) & 3))]) = pw[tp][k];
        }
    };

    f32x16 acc[2][2];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;

    issue(0);
    __syncthreads();  // every wave finished the previous tile's reads of both buffers
    stage(0, 0);
    if (nch > 1) issue(1);
    __syncthreads();
    const bf16_t* xw0 = &Xs[0][(wm * 64 + l32) * XP + hi * 8];
    const bf16_t* ww0 = &Ws[0][(wn * 64 + l32) * WP + hi * 8];
    for (int c = 0; c < nch; ++c) {
      const int s = c & 1;
      const bf16_t* xw = xw0 + s * XR * XP;
      const bf16_t* ww = ww0 + s * TAPS * BN * WP;
#pragma unroll
      for (int tp = 0; tp < TAPS; ++tp)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          bf16x8 wa[2], xb[2];
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
            wa[ni] = *reinterpret_cast<const bf16x8*>(ww + (tp * BN + ni * 32) * WP + kk * 16);
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
            xb[mi] = *reinterpret_cast<const bf16x8*>(xw + (mi * 32 + tp) * XP + kk * 16);
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[ni], xb[mi], acc[mi][ni], 0, 0, 0);
        }
      if (c + 1 < nch) {
        stage(c + 1, s ^ 1);  // the other buffer: every wave finished it before the last barrier
        if (c + 2 < nch) issue(c + 2);
        __syncthreads();
      }
    }

    // epilogue: lane = GEMM row q0 + wm*64 + mi*32 + l32, columns nb = n0 + wn*64 + ni*32 + 16*hi + r
    bf16_t* yb = reinterpret_cast<bf16_t*>(p.y) + (size_t)b * p.y_bs;
    const bf16_t* rb = p.res ? reinterpret_cast<const bf16_t*>(p.res) + (size_t)b * p.res_bs : nullptr;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const int q = q0 + wm * 64 + mi * 32 + l32;
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const int nb = n0 + wn * 64 + ni * 32 + 16 * hi;
        const int ph = nb / p.Cout, co = nb - ph * p.Cout;  // Cout % 16 == 0: one phase per lane
        const int o = q * p.up + ph - p.opad;
        if (q >= p.Lq || nb >= p.N || o < 0 || o >= p.Lout) continue;
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = acc[mi][ni][r] + (p.bias ? p.bias[co + r] : 0.f);
        if (rb) {
          float r16[16];
          load16(rb + (size_t)o * p.res_ld + co, r16);
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = (v[r] + r16[r]) * p.out_scale;
        }
        if (p.epi_gelu) {
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = 0.5f * v[r] * (1.0f + erff(v[r] * 0.7071067811865476f));
        }
        store16(yb + (size_t)o * p.y_ld + co, v);
        if (p.stats) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float sv = v[r];  // the fp32 value before the bf16 store, as conv1d_igemm's bf16 statistics
            st_s[ni][r] += sv;
            st_q[ni][r] = __builtin_fmaf(sv, sv, st_q[ni][r]);
          }
        }
      }
    }
  }
  if (cur_key >= 0 && p.stats) flush(cur_b, (cur_key % ntn) * BN);
  cur_key = -1;  // (flushed at every range end: a range's partial sums never join another range's)
  }  // tile ranges
}


// ---------------------------------------------------------------------------- split-K (small launches)
// At B = 1 the front-end / F0N k3 convs make 56 tiles for 256 CUs and each walks ~100 chunk steps on
// conv1d_igemm (120-132 us a launch, profiles/r02_layers_bf16_b1.txt).  Here the chunk range is split
// over S slices: block (tile, slice) writes its fp32 partial tile to the workspace, and k_pw_reduce sums
// the S partials in slice order (deterministic), then applies bias, residual (row >> res_shift) x
// out_scale, GELU, the bf16 store and the InstanceNorm statistics.
template <int TAPS>
__global__ void __launch_bounds__(NT) k_pwsplit(const ConvParams p, int ntm, int ntn, int S, float* __restrict__ part) {
  constexpr int XR = BM + TAPS - 1;
  constexpr int XU = (XR * 4 + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) bf16_t Xs[2][XR * XP];
  __shared__ __attribute__((aligned(16))) bf16_t Ws[2][TAPS * BN * WP];
  extern __shared__ __attribute__((aligned(16))) float coef[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, l32 = lane & 31, hi = lane >> 5;
  const int wm = wid >> 1, wn = wid & 1;
  const int slice = blockIdx.x % S, t = blockIdx.x / S;
  const int tn = t % ntn, tm = (t / ntn) % ntm, b = t / (ntn * ntm);
  const int q0 = tm * BM, n0 = tn * BN;
  const int nch = p.nchunks, cpad = nch * 32, mode = p.pro.mode;
  const int cb = (int)((long long)nch * slice / S), ce = (int)((long long)nch * (slice + 1) / S);
  const int Np = (p.N + 31) & ~31;
  if (mode) {
    for (int c = cb * 32 + tid; c < ce * 32; c += NT) {
      float mm = 0.f, aa = 1.f, be = 0.f, al = 1.f;
      if (c < p.Cin) {
        if (mode & PRO_AFFINE) adain_coeffs(p.pro, b, c, mm, aa, be);
        if (mode & PRO_SNAKE) al = p.pro.alpha[c];
      }
      coef[c] = be - mm * aa;
      coef[cpad + c] = aa;
      coef[2 * cpad + c] = al;
      coef[3 * cpad + c] = 1.0f / al;
    }
    __syncthreads();
  }
  const Rsrc rw = make_rsrc(p.w, (unsigned)((size_t)nch * TAPS * Np * 32 * 2));
  const Rsrc rx = make_rsrc(reinterpret_cast<const bf16_t*>(p.x) + (size_t)b * p.x_bs,
                            (unsigned)((size_t)p.Lin * p.x_ld * 2));
  const int r0 = q0 - p.pad;
  uint4 px[XU], pw[TAPS][2];
  auto issue = [&](int c) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < XU; ++k) {
      const int u = tid + k * NT, r = u >> 2, g = u & 3, gr = r0 + r;
      px[k] = bload16(rx, (u < XR * 4 && gr >= 0 && gr < p.Lin) ? (unsigned)((gr * p.x_ld + c * 32 + 8 * g) * 2) : OOB);
    }
#pragma unroll
    for (int tp = 0; tp < TAPS; ++tp)
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int u = tid + k * NT, r = u >> 2, g = u & 3, n = n0 + r;
        pw[tp][k] = bload16(rw, n < Np ? (unsigned)(((((size_t)c * TAPS + tp) * Np + n) * 32 + 8 * g) * 2) : OOB);
      }
  };
  auto stage = [&](int c, int s) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < XU; ++k) {
      const int u = tid + k * NT, r = u >> 2, g = u & 3, gr = r0 + r;
      if (u >= XR * 4) continue;
      uint4 o = px[k];
      const int ch = c * 32 + 8 * g;
      const bool row_ok = gr >= 0 && gr < p.Lin;
      if (mode || ch + 8 > p.Cin || !row_ok) {
        bf16x8 v;
        __builtin_memcpy(&v, &o, 16);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float f = (float)v[j];
          if (mode & PRO_AFFINE) f = __builtin_fmaf(f, coef[cpad + ch + j], coef[ch + j]);
          if (mode & PRO_SNAKE) {
            const float sn = __sinf(coef[2 * cpad + ch + j] * f);
            f = __builtin_fmaf(sn * sn, coef[3 * cpad + ch + j], f);
          }
          if (mode & PRO_LRELU) f = f > 0.f ? f : f * p.pro.slope;
          if (ch + j >= p.Cin || !row_ok) f = 0.f;
          v[j] = (bf16_t)f;
        }
        __builtin_memcpy(&o, &v, 16);
      }
      *reinterpret_cast<uint4*>(&Xs[s][r * XP + 8 * g]) = o;
    }
#pragma unroll
    for (int tp = 0; tp < TAPS; ++tp)
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int u = tid + k * NT, r = u >> 2, g = u & 3, n = n0 + r;
        *reinterpret_cast<uint4*>(&Ws[s][(tp * BN + r) * WP + 8 * (g ^ ((n >> 2) & 3))]) = pw[tp][k];
      }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;
  if (ce > cb) {
    issue(cb);
    stage(cb, 0);
    if (cb + 1 < ce) issue(cb + 1);
    __syncthreads();
    const bf16_t* xw0 = &Xs[0][(wm * 64 + l32) * XP + hi * 8];
    const bf16_t* ww0 = &Ws[0][(wn * 64 + l32) * WP + hi * 8];
    for (int c = cb; c < ce; ++c) {
      const int s = (c - cb) & 1;
      const bf16_t* xw = xw0 + s * XR * XP;
      const bf16_t* ww = ww0 + s * TAPS * BN * WP;
#pragma unroll
      for (int tp = 0; tp < TAPS; ++tp)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          bf16x8 wa[2], xb[2];
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
            wa[ni] = *reinterpret_cast<const bf16x8*>(ww + (tp * BN + ni * 32) * WP + kk * 16);
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
            xb[mi] = *reinterpret_cast<const bf16x8*>(xw + (mi * 32 + tp) * XP + kk * 16);
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[ni], xb[mi], acc[mi][ni], 0, 0, 0);
        }
      if (c + 1 < ce) {
        stage(c + 1, s ^ 1);
        if (c + 2 < ce) issue(c + 2);
        __syncthreads();
      }
    }
  }
  // fp32 partial tile -> part[slice][b][q][n]
  float* pb = part + ((size_t)slice * p.B + b) * (size_t)p.Lq * p.N;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    const int q = q0 + wm * 64 + mi * 32 + l32;
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int nb = n0 + wn * 64 + ni * 32 + 16 * hi;
      if (q >= p.Lq || nb >= p.N) continue;
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = acc[mi][ni][r];
      store16(pb + (size_t)q * p.N + nb, v);
    }
  }
}

// y[b][q][n] = epi(sum_s part[s][b][q][n]).  Block = 64 columns x RR rows; thread (column tx, row lane
// ty of 4) owns rows q0 + ty + 4 i, so the loads of a row are coalesced and a thread has RR / 4
// independent rows in flight; the statistics meet in LDS (fixed order) and leave as one atomic pair
// per (block, column).
constexpr int RR = 32;
__global__ void __launch_bounds__(256) k_pw_reduce(const ConvParams p, int S, const float* __restrict__ part) {
  __shared__ double red[2][4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + tx, b = blockIdx.z;
  const int q0 = blockIdx.y * RR;
  const size_t sb = (size_t)p.B * p.Lq * p.N;
  const float* pb = part + (size_t)b * p.Lq * p.N + n;
  bf16_t* yb = reinterpret_cast<bf16_t*>(p.y) + (size_t)b * p.y_bs;
  const bf16_t* rb = p.res ? reinterpret_cast<const bf16_t*>(p.res) + (size_t)b * p.res_bs : nullptr;
  const bool col = n < p.N;
  const float bias = (p.bias && col) ? p.bias[n] : 0.f;
  double a = 0.0, qq = 0.0;
#pragma unroll
  for (int i = 0; i < RR / 4; ++i) {
    const int q = q0 + ty + 4 * i;
    if (!col || q >= p.Lq) continue;
    float v = 0.f;
    for (int s = 0; s < S; ++s) v += pb[s * sb + (size_t)q * p.N];
    v += bias;
    if (rb) v = (v + (float)rb[(size_t)(q >> p.res_shift) * p.res_ld + n]) * p.out_scale;
    if (p.epi_gelu) v = 0.5f * v * (1.0f + erff(v * 0.7071067811865476f));
    yb[(size_t)q * p.y_ld + n] = (bf16_t)v;
    a += v;
    qq += (double)v * v;
  }
  if (!p.stats) return;
  red[0][ty][tx] = a;
  red[1][ty][tx] = qq;
  __syncthreads();
  if (ty == 0 && col) {
    const double sa = red[0][0][tx] + red[0][1][tx] + red[0][2][tx] + red[0][3][tx];
    const double sq = red[1][0][tx] + red[1][1][tx] + red[1][2][tx] + red[1][3][tx];
    double* d = stats_slot(p, blockIdx.y) + ((size_t)b * p.stats_ld + n) * ST_W;
    stat_add(d, sa, sq);
  }
}

}  // namespace

int g_opt_pw = 1;

bool st_pw_eligible(const ConvParams& p, int dtype) {
  if (!g_opt_pw || dtype != ST_BF16) return false;
  // 2-tap launches (the polyphase upsamplers) only with STTS_OPT_PW = 2: one tile at a time, load ->
  // stage -> MFMA -> epilogue, they measured slower than conv1d_igemm at their HBM-bound shapes
  // (ups3 892 vs 492 us, profiles/r02_layers_bf16_b32_pw2.txt)
  if (!(p.KS == 1 || (p.KS == 2 && g_opt_pw == 2)) || p.stride != 1 || p.dil != 1 || p.row_off != 0) return false;
  if (p.kw != 0 && p.kw != p.KS) return false;
  if (p.pad < 0 || p.pad > p.KS - 1) return false;  // window = rows [q0 - pad, q0 + 128 + taps - 1 - pad)
  if (p.N % 64 != 0 || p.Cout % 16 != 0 || p.N != p.up * p.Cout) return false;
  if (p.up == 1 && (p.Lq != p.Lin + 2 * p.pad - p.KS + 1 || p.opad != 0)) return false;
  if (p.accb || p.y_f32 || p.y_row_off || p.epi_tanh || p.epi_lrelu || p.reflect_front || p.zc_period || p.res_shift)
    return false;
  if (p.pro.mode & ~(PRO_AFFINE | PRO_SNAKE | PRO_LRELU)) return false;
  if (p.x_ld % 8 || p.y_ld % 8 || (p.res && p.res_ld % 8)) return false;
  return true;
}

int g_num_cu_pw = 0;

int st_pw(const ConvParams& p, hipStream_t stream) {
  const int ntm = (p.Lq + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const long long tiles = (long long)ntm * ntn * p.B;
  if (tiles <= 0) return ST_OK;
  if (!g_num_cu_pw) {
    int dev = 0;
    ST_CHECK_HIP(hipGetDevice(&dev));
    ST_CHECK_HIP(hipDeviceGetAttribute(&g_num_cu_pw, hipDeviceAttributeMultiprocessorCount, dev));
  }
  ConvParams q = p;
  q.seg = st_seg_choice(p, 1, g_num_cu_pw * 2);
  long long blocks = (long long)g_num_cu_pw * 2;  // 220-238 VGPRs: two 4-wave blocks per CU
  if (blocks > (q.seg ? (long long)p.B * q.seg : tiles)) blocks = q.seg ? (long long)p.B * q.seg : tiles;
  if (g_opt_grid_cap > 0 && blocks > g_opt_grid_cap) blocks = g_opt_grid_cap;
  const size_t lds = p.pro.mode ? (size_t)p.nchunks * 32 * 4 * sizeof(float) : 0;
  static bool attr = false;
  if (!attr) {  // static ring (<= 62 KB) + the coefficient table can exceed the 64 KB default
    ST_CHECK_HIP(hipFuncSetAttribute((const void*)k_pwgemm<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
    ST_CHECK_HIP(hipFuncSetAttribute((const void*)k_pwgemm<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
    attr = true;
  }
  if (lds > 96 * 1024) return ST_EINVAL;
  if (p.KS == 1)
    hipLaunchKernelGGL(k_pwgemm<1>, dim3((unsigned)blocks), dim3(NT), lds, stream, q, ntm, ntn);
  else
    hipLaunchKernelGGL(k_pwgemm<2>, dim3((unsigned)blocks), dim3(NT), lds, stream, q, ntm, ntn);
  return (int)hipGetLastError();
}

int g_opt_splitk = 1;

bool st_pw_split_eligible(const ConvParams& p, int dtype) {
  if (!g_opt_pw || !g_opt_splitk || dtype != ST_BF16 || !p.splitk_ws) return false;
  if (p.KS < 1 || p.KS > 3 || p.stride != 1 || p.dil != 1 || p.row_off != 0 || p.up != 1 || p.opad != 0) return false;
  if (p.kw != 0 && p.kw != p.KS) return false;
  if (p.pad != (p.KS - 1) / 2 || p.Lq != p.Lin || p.Lout != p.Lq) return false;
  if (p.N % 64 != 0 || p.Cout != p.N) return false;
  if (p.accb || p.y_f32 || p.y_row_off || p.epi_tanh || p.epi_lrelu || p.reflect_front || p.zc_period) return false;
  if (p.pro.mode & ~(PRO_AFFINE | PRO_SNAKE | PRO_LRELU)) return false;
  if (p.x_ld % 8 || p.y_ld % 8) return false;
  if (!g_num_cu_pw) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&g_num_cu_pw, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return false;
  }
  const long long tiles = (long long)((p.Lq + BM - 1) / BM) * ((p.N + BN - 1) / BN) * p.B;
  return tiles < g_num_cu_pw / 2 && p.nchunks >= 8;  // small launches with a long K only
}

int st_pw_split(const ConvParams& p, hipStream_t stream) {
  const int ntm = (p.Lq + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const long long tiles = (long long)ntm * ntn * p.B;
  // slices: about two blocks per CU, at least 4 chunks each, and the partials must fit the workspace
  int S = (int)((2LL * g_num_cu_pw + tiles - 1) / tiles);
  S = S < 1 ? 1 : S;
  if (S > p.nchunks / 4) S = p.nchunks / 4;
  while (S > 1 && (long long)S * p.B * p.Lq * p.N > p.splitk_ws_elems) --S;
  if (S < 1 || (long long)S * p.B * p.Lq * p.N > p.splitk_ws_elems) return ST_EWORKSPACE;
  const size_t lds = p.pro.mode ? (size_t)p.nchunks * 32 * 4 * sizeof(float) : 0;
  static bool attr = false;
  if (!attr) {
    ST_CHECK_HIP(hipFuncSetAttribute((const void*)k_pwsplit<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024));
    ST_CHECK_HIP(hipFuncSetAttribute((const void*)k_pwsplit<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024));
    ST_CHECK_HIP(hipFuncSetAttribute((const void*)k_pwsplit<3>, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024));
    attr = true;
  }
  if (lds > 64 * 1024) return ST_EINVAL;
  const dim3 grid((unsigned)(tiles * S));
  if (p.KS == 1)
    hipLaunchKernelGGL(k_pwsplit<1>, grid, dim3(NT), lds, stream, p, ntm, ntn, S, p.splitk_ws);
  else if (p.KS == 2)
    hipLaunchKernelGGL(k_pwsplit<2>, grid, dim3(NT), lds, stream, p, ntm, ntn, S, p.splitk_ws);
  else
    hipLaunchKernelGGL(k_pwsplit<3>, grid, dim3(NT), lds, stream, p, ntm, ntn, S, p.splitk_ws);
  ST_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_pw_reduce, dim3((p.N + 63) / 64, (p.Lq + RR - 1) / RR, p.B), dim3(256), 0, stream, p, S,
                     (const float*)p.splitk_ws);
  return (int)hipGetLastError();
}
