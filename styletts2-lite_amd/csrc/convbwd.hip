// Conv1d forward / backward on caller frames: the conv layers of the training step (config 5,
// train.py:272-327 runs loss.backward() through the decoder's and the discriminators' convs).
//
//   y  = conv1d(x, w, bias, stride, pad, dil)      x [B][Lin][Cin], y [B][Lq][Cout] (fp32 frames)
//   dx = conv_transpose1d(dy, w, stride, pad)      -> conv engine (st_conv1d) in the run's dtype:
//          stride 1: a forward conv of dy with w'[ci][co][t] = w[co][ci][K-1-t], pad' = dil(K-1) - pad
//          stride > 1 (dil 1): the engine's polyphase ConvTranspose with the weight as it is
//   dw[co][ci][t] = sum_(b,q) dy[b][q][co] * x[b][q*stride + t*dil - pad][ci]
//          -> k_wgrad: fp32-in MFMA (v_mfma_f32_32x32x2_f32), the (b, q) rows split into S slices,
//             one fp32 partial per slice, summed in slice order in fp64 (k_slice_reduce): deterministic
//   db[co] = sum_(b,q) dy[b][q][co]   -> k_colsum partials + the same reduction
//
// The wgrad GEMM is M = Cout, N = Cin (per tap), K = B*Lq (up to 3 M rows for a decoder stage):
// both operands are frames (rows = time, channels contiguous), which is exactly the f32 MFMA's
// operand map (lane l: A[m = l&31][k = l>>5], B[k = l>>5][n = l&31]), so 32 lanes read 128
// contiguous bytes of one row and no LDS transpose is needed.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>

#include "../../include/stts2.h"
#include "common.h"
#include "kernels.h"

int g_opt_bf16f = 0;  // STTS_OPT_BF16F: bf16 training convs on the general engine read / write fp32 frames
int g_opt_yf32 = 1;   // STTS_OPT_YF32: ... store fp32 output frames from the accumulators
int g_opt_cout1 = 1;  // STTS_OPT_COUT1: one-output-channel forwards as a GEMV (k_conv_cout1)
int g_opt_wgw = 1;  // k_wgrad_bf16w for the stride-1 convs (STTS_OPT_WGRAD); 0 = the per-tap kernel everywhere

namespace {

constexpr int kTargetWaves = 2048;  // 8 waves per CU on 256 CUs

// one wave: (32*NA co) x (32*NB ci) of tap t over rows [r0, r1) of the flattened (b, q) range
template <int NA, int NB, int UNR>
__global__ __launch_bounds__(64) void k_wgrad(const float* __restrict__ x, const float* __restrict__ dy, int Lin,
                                              int Cin, int Lq, int Cout, int K, int stride, int dil, int pad,
                                              long long R, int S, int ntco, int ntci, float* __restrict__ part) {
  const int lane = threadIdx.x;
  int tile = blockIdx.x;
  const int tci = tile % ntci;
  tile /= ntci;
  const int tco = tile % ntco;
  const int t = tile / ntco;
  const int s = blockIdx.y;
  const long long r0 = R * s / S, r1 = R * (s + 1) / S;
  const int col = lane & 31, h = lane >> 5;
  int co[NA], ci[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) co[i] = (tco * NA + i) * 32 + col;
#pragma unroll
  for (int j = 0; j < NB; ++j) ci[j] = (tci * NB + j) * 32 + col;
  f32x16 acc[NA][NB];
#pragma unroll
  for (int i = 0; i < NA; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  long long r = r0 + h;
  long long b = r / Lq;
  int q = (int)(r - b * Lq);
  const int toff = t * dil - pad;
  for (long long rb = r0; rb < r1; rb += 2 * UNR) {
    float a[UNR][NA], v[UNR][NB];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const bool vr = r < r1;
      const int xr = q * stride + toff;
      const bool vx = vr && xr >= 0 && xr < Lin;
      const float* yrow = dy + (b * Lq + q) * (long long)Cout;
      const float* xrow = x + (b * Lin + xr) * (long long)Cin;
#pragma unroll
      for (int i = 0; i < NA; ++i) a[u][i] = (vr && co[i] < Cout) ? yrow[co[i]] : 0.f;
#pragma unroll
      for (int j = 0; j < NB; ++j) v[u][j] = (vx && ci[j] < Cin) ? xrow[ci[j]] : 0.f;
      r += 2;
      q += 2;
      while (q >= Lq) {
        q -= Lq;
        ++b;
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u)
#pragma unroll
      for (int i = 0; i < NA; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u][i], v[u][j], acc[i][j], 0, 0, 0);
  }
  // C/D map: column = lane & 31 (ci), row = (e & 3) + 8 (e >> 2) + 4 h (co)
  float* pt = part + ((size_t)s * K + t) * (size_t)Cout * Cin;
#pragma unroll
  for (int i = 0; i < NA; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int cr = (tco * NA + i) * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
      if (cr >= Cout) continue;
#pragma unroll
      for (int j = 0; j < NB; ++j)
        if (ci[j] < Cin) pt[(size_t)cr * Cin + ci[j]] = acc[i][j][e];
    }
}

// bf16 weight gradient (the bf16 training mode): dw[co][ci][t] = sum_r dy[r][co] x[row(r, t)][ci] as
// v_mfma_f32_32x32x16_bf16 over 32-row chunks staged through LDS.  A workgroup = 64 co x 64 ci x up to 4
// taps (wave w computes tap 4 tg + w, 2 x 2 fragments) over one row slice; the dy chunk is staged once for
// its 4 taps.  Both operands are fp32 frames in HBM (rows = (utterance, frame), channels contiguous):
// staging converts them to bf16 in their natural [row][channel] layout (coalesced 32-B loads, 16-B LDS
// writes), and ds_read_b64_tr_b16 delivers the k (= row) -contiguous MFMA fragments (cdna_hip_programming
// T10): lane 4q + p of a 16-lane group addresses row q, channels 4p..4p+3 of a 4 x 16 block and receives
// its channel's 4 rows.  Rows are 192 B apart (64 bf16 + 64 B of padding): the 4 rows x 64 B a 32-lane half
// reads land in the 4 distinct 64-B bank quarters (conflict-free).  fp32 partials per slice, summed in
// slice order by k_slice_reduce (deterministic).
constexpr int WGB_ROWS = 32, WGB_STRIDE = 192;
typedef short s16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void ld8_f32_bf16(const float* __restrict__ src, int c, int C, bool ok, char* dst) {
  float v[8];
  if (ok && c + 8 <= C && (C & 3) == 0) {
    const float4 a = *reinterpret_cast<const float4*>(src + c);
    const float4 b = *reinterpret_cast<const float4*>(src + c + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (ok && c + j < C) ? src[c + j] : 0.f;
  }
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (bf16_t)v[j];
  *reinterpret_cast<bf16x8*>(dst) = o;
}

__device__ __forceinline__ bf16x8 tr_frag(const char* tile, int ks, int blk, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int row = ks * 16 + 8 * (g >> 1) + q, col = 32 * blk + 16 * (g & 1) + 4 * p;
  const char* a0 = tile + row * WGB_STRIDE + col * 2;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(a0 + 4 * WGB_STRIDE));
  bf16x8 f;
  __builtin_memcpy(&f, &lo, 8);
  __builtin_memcpy(reinterpret_cast<char*>(&f) + 8, &hi, 8);
  return f;
}

__global__ __launch_bounds__(256) void k_wgrad_bf16(const float* __restrict__ x, const float* __restrict__ dy, int Lin,
                                                    int Cin, int Lq, int Cout, int K, int stride, int dil, int pad,
                                                    int R, int S, int ntco, int ntci, int ntg,
                                                    float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) char lds[5 * WGB_ROWS * WGB_STRIDE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  int tile = blockIdx.x;
  const int tg = tile % ntg;
  tile /= ntg;
  const int tci = tile % ntci, tco = tile / ntci;
  const int s = blockIdx.y;
  const int r0 = (int)((long long)R * s / S), r1 = (int)((long long)R * (s + 1) / S);
  const int t = tg * 4 + w;
  const bool tap_ok = t < K;  // wave-uniform
  const int co0 = tco * 64, ci0 = tci * 64;
  char* At = lds;
  char* Xt = lds + (1 + w) * WGB_ROWS * WGB_STRIDE;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  const int toff = t * dil - pad;
  for (int rb = r0; rb < r1; rb += WGB_ROWS) {
    {  // dy chunk: thread -> row tid >> 3, channels 8 (tid & 7) .. + 8
      const int rr = tid >> 3, c8 = (tid & 7) * 8;
      const int r = rb + rr;
      const bool ok = r < r1;
      ld8_f32_bf16(dy + (size_t)(ok ? r : r0) * Cout, co0 + c8, Cout, ok, At + rr * WGB_STRIDE + c8 * 2);
    }
    {  // x chunk of this wave's tap: lane -> rows 4 (lane >> 3) .. + 4, channels 8 (lane & 7) .. + 8
      const int c8 = (lane & 7) * 8;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rr = (lane >> 3) * 4 + q;
        const int r = rb + rr;
        int xr = -1, b = 0;
        if (tap_ok && r < r1) {
          b = r / Lq;
          xr = (r - b * Lq) * stride + toff;
        }
        const bool ok = xr >= 0 && xr < Lin;
        ld8_f32_bf16(x + ((size_t)b * Lin + (ok ? xr : 0)) * Cin, ci0 + c8, Cin, ok, Xt + rr * WGB_STRIDE + c8 * 2);
      }
    }
    __syncthreads();
    if (tap_ok) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 a0 = tr_frag(At, ks, 0, lane), a1 = tr_frag(At, ks, 1, lane);
        const bf16x8 b0 = tr_frag(Xt, ks, 0, lane), b1 = tr_frag(Xt, ks, 1, lane);
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[1][1], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  if (!tap_ok) return;
  // C/D map of the 32x32 MFMAs: column = lane & 31 (ci), row = (e & 3) + 8 (e >> 2) + 4 (lane >> 5) (co)
  float* pt = part + ((size_t)s * K + t) * (size_t)Cout * Cin;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int co = co0 + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
      if (co >= Cout) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ci = ci0 + 32 * j + (lane & 31);
        if (ci < Cin) pt[(size_t)co * Cin + ci] = acc[i][j][e];
      }
    }
}

// Stride-1 convolutions (every decoder resblock / front-end conv, conv_post, the 1x1s): one workgroup owns a
// 64 co x 64 ci tile for ALL K taps over a slice of 64-row chunks (chunks never cross an utterance; a slice
// may span several short utterances, so the slice count and the partials stay small at any batch), and
// stages per chunk the dy rows
// and ONE x window of 64 + (K-1) dil rows, read at K row offsets (the per-tap kernel above stages K separate
// x chunks).  Wave w = (co half w >> 1, ci half w & 1) accumulates K 32 x 32 fragments.  The next chunk's fp32
// rows are loaded into registers while the current chunk's MFMAs run; LDS is double-buffered (one barrier per
// chunk).  Partials part[s][t][co][ci] with s = utterance x slice, summed in order by k_slice_reduce.
constexpr int WGW_CH = 64, WGW_DILMAX = 5;

// 4 fp32 channels c .. c + 3 of a row (zeros past C or when !ok)
__device__ __forceinline__ float4 ld4(const float* __restrict__ row, int c, int C, bool ok) {
  if (ok && c + 4 <= C && (C & 3) == 0) return *reinterpret_cast<const float4*>(row + c);
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = (ok && c + j < C) ? row[c + j] : 0.f;
  return make_float4(v[0], v[1], v[2], v[3]);
}

// ST > 1 (the discriminators' strided convs, dilation 1): the window is stored phase-split, ST blocks of PR
// rows, block ph holding window rows ph, ph + ST, ...; tap t then reads block (t mod ST) from row t / ST on,
// again consecutive rows for the transposed fragment reads.
// C32 (Cout <= 32: the MSD / MPD discriminator convs): the second output-channel block would be empty, so the
// fi = 1 waves take the odd taps of the fi = 0 block instead (each wave (K + 1) / 2 taps and accumulators)
// txH > 0: x is the MSD image [B = S H][Lin][32] time-expanded on the fly, channel ci = dh 32 + c reading
// utterance row b + dh - 1 (zero outside the signal's H rows), as stts_conv1d_fwd_tx
template <int K, int ST = 1, bool C32 = false>
__global__ __launch_bounds__(256) void k_wgrad_bf16w(const float* __restrict__ x, const float* __restrict__ dy, int Lin,
                                                     int Cin, int Lq, int Cout, int dil, int pad, int B, int S,
                                                     int ntci, float* __restrict__ part, int txH) {
  constexpr int DMAX = ST == 1 ? WGW_DILMAX : 1;
  constexpr int PR = WGW_CH + ((K - 1) * DMAX + ST - 1) / ST;  // rows per phase block
  constexpr int WMAX = ST * PR;                                // x window rows (LDS)
  constexpr int XPT = (WMAX + 63) / 64;                        // x window rows per thread (4 threads per row)
  constexpr int BUF = (WGW_CH + WMAX) * WGB_STRIDE;    // one stage: dy rows then the x window
  __shared__ __attribute__((aligned(16))) char lds[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fi = w >> 1, fj = w & 1;
  const int tci = blockIdx.x % ntci, tco = blockIdx.x / ntci;
  const int co0 = tco * 64, ci0 = tci * 64;
  const int sl = blockIdx.y;
  const int ncb = (Lq + WGW_CH - 1) / WGW_CH;  // chunks per utterance
  const long long U = (long long)B * ncb;      // chunk units (utterance, chunk), in order
  const int u0 = (int)(U * sl / S), u1 = (int)(U * (sl + 1) / S);
  const int WR = (WGW_CH - 1) * ST + (K - 1) * dil + 1;  // window rows the chunk reads
  // staging: thread -> row (tid >> 2) (+ 64 j for the window), channels 16 (tid & 3) .. + 16
  const int rr = tid >> 2, c16 = (tid & 3) * 16;
  float4 pd[4], px[XPT][4];
  auto load = [&](int u) __attribute__((always_inline)) {
    const int b = u / ncb, qc = (u - b * ncb) * WGW_CH;
    const float* dyb = dy + (size_t)b * Lq * Cout;
    const float* xb = x + (size_t)b * Lin * Cin;
    int xld = Cin, cb = 0;  // the source rows' channel count and this thread's channel base in them
    bool okt = true;
    if (txH) {  // this thread's 16 channels lie in one 32-channel row chunk dh
      const int dh = (ci0 + c16) >> 5, hh = b % txH + dh - 1;
      okt = (unsigned)hh < (unsigned)txH && ci0 + c16 < Cin;
      xb = x + (size_t)(okt ? b + dh - 1 : b) * Lin * 32;
      xld = 32;
      cb = 32 * dh;
    }
    const int q = qc + rr;
    const bool okd = q < Lq;
    const int cc = co0 + c16;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = cc + 4 * j;
      pd[j] = ld4(dyb + (size_t)(okd ? q : 0) * Cout, c, Cout, okd);
    }
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int wr = rr + 64 * i;                  // LDS row: phase block wr / PR, row wr % PR
      const int j = ST == 1 ? wr : (wr % PR) * ST + wr / PR;  // window row
      const int xr = qc * ST - pad + j;
      const bool ok = okt && wr < WMAX && j < WR && xr >= 0 && xr < Lin;
      const int c0 = ci0 + c16 - cb;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = c0 + 4 * j;
        px[i][j] = ld4(xb + (size_t)(ok ? xr : 0) * xld, c, xld, ok);
      }
    }
  };
  auto st8 = [&](char* dst, const float4& a, const float4& c) __attribute__((always_inline)) {
    bf16x8 o;
    o[0] = (bf16_t)a.x; o[1] = (bf16_t)a.y; o[2] = (bf16_t)a.z; o[3] = (bf16_t)a.w;
    o[4] = (bf16_t)c.x; o[5] = (bf16_t)c.y; o[6] = (bf16_t)c.z; o[7] = (bf16_t)c.w;
    *reinterpret_cast<bf16x8*>(dst) = o;
  };
  auto store = [&](char* buf) __attribute__((always_inline)) {
    char* d = buf + rr * WGB_STRIDE + c16 * 2;
    st8(d, pd[0], pd[1]);
    st8(d + 16, pd[2], pd[3]);
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int wr = rr + 64 * i;
      if (wr < WMAX) {
        char* e = buf + (WGW_CH + wr) * WGB_STRIDE + c16 * 2;
        st8(e, px[i][0], px[i][1]);
        st8(e + 16, px[i][2], px[i][3]);
      }
    }
  };
  constexpr int KA = C32 ? (K + 1) / 2 : K;  // accumulators (taps) per wave
  f32x16 acc[KA];
#pragma unroll
  for (int t = 0; t < KA; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
  const int cob = C32 ? 0 : fi;
  // a wave whose 32-channel block lies past Cout / Cin computes nothing (wave-uniform)
  const bool live = co0 + 32 * cob < Cout && ci0 + 32 * fj < Cin;
  const int nch = u1 - u0;
  if (nch > 0) {
    load(u0);
    store(lds);
  }
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    char* cur = lds + (c & 1) * BUF;
    if (c + 1 < nch) load(u0 + c + 1);  // in flight under this chunk's MFMAs
    if (live) {
#pragma unroll
      for (int ks = 0; ks < WGW_CH / 16; ++ks) {
        const bf16x8 a = tr_frag(cur, ks, cob, lane);
#pragma unroll
        for (int ta = 0; ta < KA; ++ta) {
          const int t = C32 ? 2 * ta + fi : ta;  // (C32: the wave's taps fi, fi + 2, ...)
          if (C32 && t >= K) continue;           // (wave-uniform)
          const int tj = t * dil;
          const int row = ST == 1 ? tj : (tj % ST) * PR + tj / ST;
          const bf16x8 bx = tr_frag(cur + (WGW_CH + row) * WGB_STRIDE, ks, fj, lane);
          acc[ta] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bx, acc[ta], 0, 0, 0);
        }
      }
    }
    if (c + 1 < nch) store(lds + ((c + 1) & 1) * BUF);
    __syncthreads();
  }
  if (!live) return;
  float* pt = part + (size_t)sl * K * Cout * Cin;
#pragma unroll
  for (int ta = 0; ta < KA; ++ta) {
    const int t = C32 ? 2 * ta + fi : ta;
    if (C32 && t >= K) continue;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int co = co0 + 32 * cob + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
      const int ci = ci0 + 32 * fj + (lane & 31);
      if (co < Cout && ci < Cin) pt[((size_t)t * Cout + co) * Cin + ci] = acc[ta][e];
    }
  }
}

// slices for k_wgrad_bf16w: about 256 workgroups, >= 2 chunks per slice
int wgw_slices(int B, int Lq, int Cin, int Cout, int K) {
  const long long tiles = (long long)((Cout + 63) / 64) * ((Cin + 63) / 64);
  const long long units = (long long)B * ((Lq + WGW_CH - 1) / WGW_CH);
  // ~256 workgroups: the fp32 partials (S x Cout x Cin x K) and their reduction scale with the slice count,
  // and at config-5 shapes 256 measured 30-50 % faster than 1,024 on the dw call (wgrad + reduction,
  // profiles/r03_ab_wgrad_slices.txt).  STTS_OPT_EXP bit 128 / 256 / 512: 512 / 1,024 / 128 (A/B).
  const long long target = (g_opt_exp & 512) ? 128 : (g_opt_exp & 256) ? 1024 : (g_opt_exp & 128) ? 512 : 256;
  long long S = (target + tiles - 1) / tiles;
  // (STTS_OPT_EXP bit 2048, off: few-input-channel convs over many rows get one slice per 16 chunks while the
  // partials stay under 32 MB; on the MSD first layer, Cin = 3 over 1.9 M rows, it measured slower, dw 0.59 ->
  // 0.75 ms, profiles/r03_ab_msd_conv.txt)
  if (Cin <= 16 && (g_opt_exp & 2048)) {
    const long long per = std::max<long long>(1, (long long)Cout * Cin * K * 4);
    S = std::max(S, std::min<long long>(units / 16, (32ll << 20) / per));
  }
  S = std::min<long long>(S, std::max<long long>(1, units / 2));
  return (int)std::max<long long>(1, std::min<long long>(S, 4096));
}

bool wgw_eligible(int K, int stride, int dil) {
  if (stride == 1)
    return dil >= 1 && dil <= WGW_DILMAX && (K == 1 || K == 2 || K == 3 || K == 5 || K == 7 || K == 9 || K == 11);
  if (dil != 1) return false;
  if (stride == 2) return K == 3 || K == 4 || K == 9;  // F0 / N convs, ups[3] dw, MSD
  if (stride == 3) return K == 5 || K == 6;            // MPD, ups[2] dw
  return false;
}

struct SlicesB {
  int ntco, ntci, ntg, S;
};

SlicesB slices_bf16(int B, int Lq, int Cin, int Cout, int K) {
  SlicesB sl;
  sl.ntco = (Cout + 63) / 64;
  sl.ntci = (Cin + 63) / 64;
  sl.ntg = (K + 3) / 4;
  const long long R = (long long)B * Lq;
  const long long tiles = (long long)sl.ntco * sl.ntci * sl.ntg;
  long long S = (1024 + tiles - 1) / tiles;
  S = std::min<long long>(S, std::max<long long>(1, R / 256));  // >= 8 row chunks per slice
  sl.S = (int)std::max<long long>(1, std::min<long long>(S, 4096));
  return sl;
}

// part[s][t][co][ci] -> out[co][ci][t] = sum over s in order (fp64); P = float (wgrad partials) or double
// (the bias column sums: a bias gradient often cancels to far below its slice partials, so those stay fp64)
template <typename P>
__global__ void k_slice_reduce(const P* __restrict__ part, int S, int K, int Cout, int Cin,
                               float* __restrict__ out) {
  const size_t per = (size_t)K * Cout * Cin;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= per) return;
  const int ci = (int)(i % Cin);
  const int co = (int)((i / Cin) % Cout);
  const int t = (int)(i / ((size_t)Cin * Cout));
  // eight independent loads in flight, added in slice order (the latency, not the bytes, bounds
  // a one-load-at-a-time loop)
  double sum = 0.0;
  int s = 0;
  for (; s + 8 <= S; s += 8) {
    P v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = part[(size_t)(s + k) * per + i];
#pragma unroll
    for (int k = 0; k < 8; ++k) sum += v[k];
  }
  for (; s < S; ++s) sum += part[(size_t)s * per + i];
  out[((size_t)co * Cin + ci) * K + t] = (float)sum;
}

// column sums of dy [R][C] over row slice s: part[s][c] (fp64)
__global__ __launch_bounds__(256) void k_colsum(const float* __restrict__ dy, long long R, int C, int S,
                                                double* __restrict__ part) {
  __shared__ double red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  const int s = blockIdx.y;
  const long long r0 = R * s / S, r1 = R * (s + 1) / S;
  double acc = 0.0;
  if (c < C) {
    // eight rows' loads in flight per thread (one load per add made the call latency-bound)
    long long r = r0 + rl;
    for (; r + 28 < r1; r += 32) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = dy[(r + 4 * u) * C + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; r < r1; r += 4) acc += dy[r * C + c];
  }
  red[rl][threadIdx.x & 63] = acc;
  __syncthreads();
  if (rl == 0 && c < C) {
    const int l = threadIdx.x;
    part[(size_t)s * C + c] = ((red[0][l] + red[1][l]) + red[2][l]) + red[3][l];
  }
}

// Cout = 1 forwards (MPD conv_post 1024 -> 1 (3, 1), the generator's conv_post, the F0 / N stride-2
// one-channel convs): a GEMV per output frame, which the MFMA engines run as a 16-column tile on a few dozen
// workgroups (~90 us a launch at config-5 sizes).  One wave per frame, lanes over the input channels, fp32 FMAs
// over the operands as the dtype rounds them (RB: bf16, as the bf16 MFMA sees them), a fixed-order wave reduction.
template <bool RB>
__global__ __launch_bounds__(256) void k_conv_cout1(const float* __restrict__ x, const float* __restrict__ w,
                                                    const float* __restrict__ bias, int B, int Lin, int Cin, int K,
                                                    int stride, int dil, int pad, int Lq, int lrelu, float slope,
                                                    float* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (long long)B * Lq) return;  // (wave-uniform)
  const int b = (int)(row / Lq), q = (int)(row - (long long)b * Lq);
  const float* xb = x + (size_t)b * Lin * Cin;
  auto rd = [](float v) __attribute__((always_inline)) { return RB ? (float)(bf16_t)v : v; };
  float acc = 0.f;
  for (int t = 0; t < K; ++t) {
    const int r = q * stride - pad + t * dil;
    if (r < 0 || r >= Lin) continue;  // (wave-uniform)
    const float* xr = xb + (size_t)r * Cin;
    for (int c = lane; c < Cin; c += 64) acc = fmaf(rd(w[(size_t)c * K + t]), rd(xr[c]), acc);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) {
    float v = acc + (bias ? bias[0] : 0.f);
    if (lrelu) v = v > 0.f ? v : v * slope;
    y[row] = v;
  }
}

// w [Cout][Cin][K] -> wt [Cin][Cout][K] with the taps reversed (the stride-1 dgrad weight)
__global__ void k_flip_transpose(const float* __restrict__ w, int Cout, int Cin, int K, float* __restrict__ wt) {
  const size_t n = (size_t)Cout * Cin * K;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int t = (int)(i % K);
  const int co = (int)((i / K) % Cout);
  const int ci = (int)(i / ((size_t)K * Cout));
  wt[i] = w[((size_t)co * Cin + ci) * K + (K - 1 - t)];
}

struct Geo {
  int B, Lin, Cin, Cout, K, stride, dil, pad, Lq;
};

inline int ldpad(int c) { return (c + 7) & ~7; }

bool geo_ok(const Geo& g) {
  if (g.B <= 0 || g.Lin <= 0 || g.Cin <= 0 || g.Cout <= 0 || g.K <= 0 || g.stride <= 0 || g.dil <= 0 || g.pad < 0)
    return false;
  const long long lq = ((long long)g.Lin + 2LL * g.pad - (long long)g.dil * (g.K - 1) - 1) / g.stride + 1;
  return lq == g.Lq && g.Lq > 0;
}

struct Slices {
  int NA, NB, ntco, ntci, S, S2;
};

Slices slices_of(const Geo& g) {
  Slices sl;
  sl.NA = g.Cout > 32 ? 2 : 1;
  sl.NB = g.Cin > 32 ? 2 : 1;
  sl.ntco = (g.Cout + 32 * sl.NA - 1) / (32 * sl.NA);
  sl.ntci = (g.Cin + 32 * sl.NB - 1) / (32 * sl.NB);
  const long long R = (long long)g.B * g.Lq;
  const long long tiles = (long long)g.K * sl.ntco * sl.ntci;
  long long S = (kTargetWaves + tiles - 1) / tiles;
  S = std::min<long long>(S, std::max<long long>(1, R / 64));  // >= 64 rows per slice
  sl.S = (int)std::max<long long>(1, std::min<long long>(S, 4096));
  const int cblk = (g.Cout + 63) / 64;
  long long S2 = (512 + cblk - 1) / cblk;
  S2 = std::min<long long>(S2, std::max<long long>(1, R / 256));
  sl.S2 = (int)std::max<long long>(1, std::min<long long>(S2, 1024));
  return sl;
}

int colsum_slices(int C, long long R) {
  const int cblk = (C + 63) / 64;
  long long S2 = (512 + cblk - 1) / cblk;
  S2 = std::min<long long>(S2, std::max<long long>(1, R / 256));
  return (int)std::max<long long>(1, std::min<long long>(S2, 1024));
}

// workspace pieces (bytes, each 256-aligned)
struct WsLayout {
  size_t xin, wstage, bpad, packed, yout, part, part2, total;
};

inline size_t al(size_t n) { return (n + 255) & ~(size_t)255; }

enum WMode { W_PLAIN = 0, W_FLIP = 1, W_TRANS = 2 };

// one engine launch as the caller sees it: ci_e -> co_e channels
struct EngineGeo {
  int Lin, ci, co, co_p, Lout, u, transposed, stride;
  WMode wm;
};

// the conv engine's narrow epilogue (Cout % 16 != 0) serves only N <= 32 at stride 1: other
// channel counts run with the output channels padded to 16 (zero weight rows) and are cropped
EngineGeo engine_geo(const Geo& g, bool fwd) {
  EngineGeo e;
  e.Lin = fwd ? g.Lin : g.Lq;
  e.Lout = fwd ? g.Lq : g.Lin;
  e.ci = fwd ? g.Cin : g.Cout;
  e.co = fwd ? g.Cout : g.Cin;
  e.transposed = !fwd && g.stride > 1;
  e.u = e.transposed ? g.stride : 1;
  e.stride = fwd ? g.stride : 1;
  e.wm = fwd ? W_PLAIN : (e.transposed ? W_TRANS : W_FLIP);
  const bool pad = e.co % 16 != 0 && (e.u * e.co > 32 || e.stride > 1);
  e.co_p = pad ? (e.co + 15) & ~15 : e.co;
  return e;
}

WsLayout ws_layout(const Geo& g, int dtype, bool fwd) {
  const size_t esz = dtype == ST_BF16 ? 2 : 4;  // ST_SPLIT: fp32 frames, bf16 hi + lo weights
  // bf16 runs on the general engine read / write fp32 frames directly (ST_BF16F): the padded input copy may be fp32
  const size_t xesz = 4;
  const EngineGeo e = engine_geo(g, fwd);
  WsLayout w;
  memset(&w, 0, sizeof(w));
  size_t off = 0;
  w.xin = off;
  off += al((size_t)g.B * e.Lin * ldpad(e.ci) * xesz);
  w.wstage = off;
  if (e.wm != W_PLAIN || e.co_p != e.co) off += al((size_t)e.co_p * e.ci * g.K * 4);
  w.bpad = off;
  if (e.co_p != e.co) off += al((size_t)e.co_p * 4);
  w.packed = off;
  off += al(st_packed_conv_elems(e.ci, e.co_p, g.K, e.transposed, e.u) * esz);
  w.yout = off;
  if (dtype == ST_BF16 || e.co_p != e.co) off += al((size_t)g.B * e.Lout * e.co_p * xesz);
  if (!fwd) {
    const Slices sl = slices_of(g);
    w.part = off;
    size_t ns = (size_t)sl.S;
    if (dtype == ST_BF16) {
      ns = std::max(ns, (size_t)slices_bf16(g.B, g.Lq, g.Cin, g.Cout, g.K).S);
      if (wgw_eligible(g.K, g.stride, g.dil))
        ns = std::max(ns, (size_t)wgw_slices(g.B, g.Lq, g.Cin, g.Cout, g.K));
    }
    off += al(ns * g.K * g.Cout * g.Cin * 4);
    w.part2 = off;
    off += al((size_t)sl.S2 * g.Cout * 8);
  }
  w.total = off;
  return w;
}

// db[co] = column sums of dy [B Lq][Cout]: per-slice fp64 partials, reduced in order
int bias_grad(const Geo& g, const float* dy, float* db, double* part2, hipStream_t s) {
  const Slices sl = slices_of(g);
  hipLaunchKernelGGL(k_colsum, dim3((unsigned)((g.Cout + 63) / 64), sl.S2), dim3(256), 0, s, dy,
                     (long long)g.B * g.Lq, g.Cout, sl.S2, part2);
  ST_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_slice_reduce<double>, dim3((unsigned)((g.Cout + 255) / 256)), dim3(256), 0, s, part2, sl.S2, 1,
                     g.Cout, 1, db);
  return (int)hipGetLastError();
}

// one engine launch: y fp32 [B][Lout][co] from xf fp32 frames [B][Lin][ci].  w is the forward
// weight [Cout][Cin][K]; wm says how the engine's weight derives from it (W_PLAIN: as is, W_FLIP:
// channel-transposed and tap-reversed, W_TRANS: as a ConvTranspose1d weight [in][out][K]).
int run_engine(int dtype, const Geo& g, bool fwd, const float* xf, const float* w, const float* bias, float* y,
               char* ws, hipStream_t s, const float* res = nullptr, float scale = 1.f, bool lrelu = false,
               float slope = 0.f, int tx_H = 0) {
  if (fwd && g.Cout == 1 && !tx_H && !res && g_opt_cout1) {  // the GEMV kernel (no workspace)
    const long long rows = (long long)g.B * g.Lq;
    if (dtype == ST_BF16)
      hipLaunchKernelGGL(k_conv_cout1<true>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, xf, w, bias, g.B, g.Lin,
                         g.Cin, g.K, g.stride, g.dil, g.pad, g.Lq, (int)lrelu, slope, y);
    else
      hipLaunchKernelGGL(k_conv_cout1<false>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, xf, w, bias, g.B,
                         g.Lin, g.Cin, g.K, g.stride, g.dil, g.pad, g.Lq, (int)lrelu, slope, y);
    return (int)hipGetLastError();
  }
  const EngineGeo e = engine_geo(g, fwd);
  const WsLayout L = ws_layout(g, dtype, fwd);
  const int K = g.K, B = g.B;
  // tx_H: xf is the MSD image [B = S H][Lin][32] that the engine time-expands to the ci = 96 channels itself
  const int cix = tx_H ? 32 : e.ci;
  const int ldx = tx_H ? 32 : ldpad(e.ci);
  void* xd = ws + L.xin;
  void* wd = ws + L.packed;
  const float* wsrc = w;
  if (e.wm != W_PLAIN || e.co_p != e.co) {
    float* wt = (float*)(ws + L.wstage);
    const size_t nst = (size_t)e.co_p * e.ci * K;
    const size_t n = (size_t)e.co * e.ci * K;
    if (e.wm == W_TRANS) {  // [ci][co][K] -> [ci][co_p][K]
      ST_CHECK_HIP(hipMemsetAsync(wt, 0, nst * 4, s));
      ST_CHECK_HIP(hipMemcpy2DAsync(wt, (size_t)e.co_p * K * 4, w, (size_t)e.co * K * 4, (size_t)e.co * K * 4, e.ci,
                                    hipMemcpyDeviceToDevice, s));
    } else {  // [co][ci][K] rows, then zero rows co .. co_p
      if (e.wm == W_FLIP) {
        hipLaunchKernelGGL(k_flip_transpose, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, w, g.Cout, g.Cin, K,
                           wt);
        ST_CHECK_HIP(hipGetLastError());
      } else {
        ST_CHECK_HIP(hipMemcpyAsync(wt, w, n * 4, hipMemcpyDeviceToDevice, s));
      }
      if (nst > n) ST_CHECK_HIP(hipMemsetAsync(wt + n, 0, (nst - n) * 4, s));
    }
    wsrc = wt;
  }
  const float* bsrc = bias;
  if (bias && e.co_p != e.co) {
    float* bp = (float*)(ws + L.bpad);
    ST_CHECK_HIP(hipMemsetAsync(bp, 0, (size_t)e.co_p * 4, s));
    ST_CHECK_HIP(hipMemcpyAsync(bp, bias, (size_t)e.co * 4, hipMemcpyDeviceToDevice, s));
    bsrc = bp;
  }
  ST_CHECK(st_pack_conv(wsrc, e.ci, e.co_p, K, e.transposed, e.u, wd, dtype, s));
  ConvParams p;
  memset(&p, 0, sizeof(p));
  p.x = xd;
  p.x_bs = (long long)e.Lin * ldx;
  p.x_ld = ldx;
  p.Lin = e.Lin;
  p.Cin = e.ci;
  p.B = B;
  p.w = wd;
  p.nchunks = (e.ci + 31) / 32;
  p.bias = bsrc;
  p.Cout = e.co_p;
  if (!e.transposed) {
    p.KS = K;
    p.dil = g.dil;
    p.stride = e.stride;
    p.pad = fwd ? g.pad : g.dil * (K - 1) - g.pad;
    p.N = e.co_p;
    p.up = 1;
    p.Lq = e.Lout;
  } else {
    const int taps = (K + e.u - 1) / e.u;
    p.KS = taps;
    p.dil = 1;
    p.stride = 1;
    p.pad = taps - 1;
    p.N = e.u * e.co_p;
    p.up = e.u;
    p.opad = g.pad;
    p.Lq = (e.Lout - 1 + g.pad) / e.u + 1;
  }
  p.Lout = e.Lout;
  p.y_bs = (long long)e.Lout * e.co_p;
  p.y_ld = e.co_p;
  p.out_scale = scale;
  p.tx_H = tx_H;
  if (lrelu) {  // leaky ReLU in the epilogue (the engines that lack it decline the launch: igemm takes it)
    p.epi_lrelu = 1;
    p.epi_slope = slope;
  }
  if (res) {  // y = conv + res (fp32 frames [B][Lout][co], the same layout as y)
    p.res = res;
    p.res_bs = (long long)e.Lout * e.co;
    p.res_ld = e.co;
  }
  // frames storage: bf16 runs whose launch goes to the general engine read and write the fp32 frames directly
  // (ST_BF16F: the window is rounded to bf16 while staged), saving the two conversion passes around the conv;
  // the specialised engines (resconv, pwgemm) take bf16 frames
  int edt = dtype;
  if (dtype == ST_BF16 && g_opt_bf16f && st_conv1d_engine(p, ST_BF16) == ST_ENGINE_IGEMM) edt = ST_BF16F;
  const int adt = (edt == ST_BF16) ? ST_BF16 : ST_FP32;
  if (res && (adt != ST_FP32 || e.co_p != e.co)) return ST_EINVAL;
  if (adt == ST_FP32 && ldx == cix)
    xd = (void*)xf;  // fp32 frames with 8-aligned rows are the engine's input as they are
  else
    ST_CHECK(st_frames_convert(xf, B, e.Lin, cix, cix, xd, ldx, nullptr, 0, adt, s));
  p.x = xd;
  // bf16 launches on the general engine write fp32 frames from the accumulators (y_f32, STTS_OPT_YF32): no
  // conversion pass after the conv; the specialised engines store bf16
  const bool yf = adt == ST_BF16 && e.co_p == e.co && !res && g_opt_yf32 && st_conv1d_engine(p, edt) == ST_ENGINE_IGEMM;
  const bool direct = (adt == ST_FP32 && e.co_p == e.co) || yf;
  void* yd = direct ? (void*)y : (void*)(ws + L.yout);
  p.y = yd;
  p.y_f32 = yf ? 1 : 0;
  ST_CHECK(st_conv1d(p, edt, s));
  if (!direct) ST_CHECK(st_frames_to_f32(yd, B, e.Lout, e.co, e.co_p, y, adt, s));
  return 0;
}

template <int K, int ST = 1>
void launch_wgw(const Geo& g, const float* x, const float* dy, float* part, int S, hipStream_t s, int txH) {
  const int ntci = (g.Cin + 63) / 64, ntco = (g.Cout + 63) / 64;
  if (g.Cout <= 32 && !(g_opt_exp & 4096))  // (STTS_OPT_EXP bit 4096: every tap on the fi = 0 waves, A/B)
    hipLaunchKernelGGL((k_wgrad_bf16w<K, ST, true>), dim3(ntco * ntci, S), dim3(256), 0, s, x, dy, g.Lin, g.Cin, g.Lq,
                       g.Cout, g.dil, g.pad, g.B, S, ntci, part, txH);
  else
    hipLaunchKernelGGL((k_wgrad_bf16w<K, ST>), dim3(ntco * ntci, S), dim3(256), 0, s, x, dy, g.Lin, g.Cin, g.Lq, g.Cout,
                       g.dil, g.pad, g.B, S, ntci, part, txH);
}

// dw as per-slice partials + the in-order reduction into dw [Cout][Cin][K] (txH: x time-expanded on the fly, the
// window kernel only)
int wgrad_bf16(const Geo& g, const float* x, const float* dy, float* part, float* dw, hipStream_t s, int txH = 0) {
  if (txH && !(g_opt_wgw && wgw_eligible(g.K, g.stride, g.dil))) return ST_EINVAL;
  if (g_opt_wgw && wgw_eligible(g.K, g.stride, g.dil)) {
    const int Sb = wgw_slices(g.B, g.Lq, g.Cin, g.Cout, g.K);
    if (g.stride == 2) {
      if (g.K == 3) launch_wgw<3, 2>(g, x, dy, part, Sb, s, txH);
      else if (g.K == 4) launch_wgw<4, 2>(g, x, dy, part, Sb, s, txH);
      else launch_wgw<9, 2>(g, x, dy, part, Sb, s, txH);
    } else if (g.stride == 3) {
      if (g.K == 5) launch_wgw<5, 3>(g, x, dy, part, Sb, s, txH);
      else launch_wgw<6, 3>(g, x, dy, part, Sb, s, txH);
    } else {
      switch (g.K) {
        case 1: launch_wgw<1>(g, x, dy, part, Sb, s, txH); break;
        case 2: launch_wgw<2>(g, x, dy, part, Sb, s, txH); break;
        case 3: launch_wgw<3>(g, x, dy, part, Sb, s, txH); break;
        case 5: launch_wgw<5>(g, x, dy, part, Sb, s, txH); break;
        case 7: launch_wgw<7>(g, x, dy, part, Sb, s, txH); break;
        case 9: launch_wgw<9>(g, x, dy, part, Sb, s, txH); break;
        default: launch_wgw<11>(g, x, dy, part, Sb, s, txH); break;
      }
    }
    ST_CHECK_HIP(hipGetLastError());
    const size_t n = (size_t)g.K * g.Cout * g.Cin;
    hipLaunchKernelGGL(k_slice_reduce<float>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, part, Sb, g.K,
                       g.Cout, g.Cin, dw);
    return (int)hipGetLastError();
  }
  const SlicesB sl = slices_bf16(g.B, g.Lq, g.Cin, g.Cout, g.K);
  const long long R = (long long)g.B * g.Lq;
  if (R > 0x7fffffffLL) return ST_EINVAL;
  hipLaunchKernelGGL(k_wgrad_bf16, dim3(sl.ntco * sl.ntci * sl.ntg, sl.S), dim3(256), 0, s, x, dy, g.Lin, g.Cin, g.Lq,
                     g.Cout, g.K, g.stride, g.dil, g.pad, (int)R, sl.S, sl.ntco, sl.ntci, sl.ntg, part);
  ST_CHECK_HIP(hipGetLastError());
  const size_t n = (size_t)g.K * g.Cout * g.Cin;
  hipLaunchKernelGGL(k_slice_reduce<float>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, part, sl.S, g.K,
                     g.Cout, g.Cin, dw);
  return (int)hipGetLastError();
}

template <int NA, int NB>
void launch_wgrad(const Geo& g, const Slices& sl, const float* x, const float* dy, float* part, hipStream_t s) {
  dim3 grid(g.K * sl.ntco * sl.ntci, sl.S);
  hipLaunchKernelGGL((k_wgrad<NA, NB, 4>), grid, dim3(64), 0, s, x, dy, g.Lin, g.Cin, g.Lq, g.Cout, g.K, g.stride,
                     g.dil, g.pad, (long long)g.B * g.Lq, sl.S, sl.ntco, sl.ntci, part);
}

}  // namespace

extern "C" long long stts_conv1d_fwd_workspace_bytes(int dtype, int B, int Lin, int Cin, int Cout, int K, int stride,
                                                     int dil, int pad, int Lq) {
  if (dtype != ST_FP32 && dtype != ST_BF16 && dtype != ST_SPLIT) return ST_EDTYPE;
  const Geo g{B, Lin, Cin, Cout, K, stride, dil, pad, Lq};
  if (!geo_ok(g)) return ST_EINVAL;
  return (long long)ws_layout(g, dtype, true).total;
}

extern "C" int stts_conv1d_fwd_res(int dtype, const float* x, const float* w, const float* bias, const float* res,
                                   float scale, int B, int Lin, int Cin, int Cout, int K, int stride, int dil, int pad, int Lq,
                                   float* y, void* workspace, long long ws_bytes, void* stream) {
  const long long need = stts_conv1d_fwd_workspace_bytes(dtype, B, Lin, Cin, Cout, K, stride, dil, pad, Lq);
  if (need < 0) return (int)need;
  if (!x || !w || !y) return ST_EINVAL;
  // the engines apply out_scale in their residual epilogue only: a scale without a residual would be
  // silently dropped (and the autograd backward would still scale dy), so it is refused
  if (!res && scale != 1.0f) return ST_EINVAL;
  if (!workspace || ws_bytes < need) return ST_EWORKSPACE;
  const Geo g{B, Lin, Cin, Cout, K, stride, dil, pad, Lq};
  return run_engine(dtype, g, true, x, w, bias, y, (char*)workspace, (hipStream_t)stream, res, scale);
}

extern "C" int stts_conv1d_fwd_act(int dtype, const float* x, const float* w, const float* bias, int B, int Lin,
                                   int Cin, int Cout, int K, int stride, int dil, int pad, int Lq, float slope, float* y,
                                   void* workspace, long long ws_bytes, void* stream) {
  const long long need = stts_conv1d_fwd_workspace_bytes(dtype, B, Lin, Cin, Cout, K, stride, dil, pad, Lq);
  if (need < 0) return (int)need;
  if (!x || !w || !y) return ST_EINVAL;
  if (!workspace || ws_bytes < need) return ST_EWORKSPACE;
  const Geo g{B, Lin, Cin, Cout, K, stride, dil, pad, Lq};
  return run_engine(dtype, g, true, x, w, bias, y, (char*)workspace, (hipStream_t)stream, nullptr, 1.f, true, slope);
}

extern "C" int stts_conv1d_fwd(int dtype, const float* x, const float* w, const float* bias, int B, int Lin, int Cin,
                               int Cout, int K, int stride, int dil, int pad, int Lq, float* y, void* workspace,
                               long long ws_bytes, void* stream) {
  const long long need = stts_conv1d_fwd_workspace_bytes(dtype, B, Lin, Cin, Cout, K, stride, dil, pad, Lq);
  if (need < 0) return (int)need;
  if (!x || !w || !y) return ST_EINVAL;
  if (!workspace || ws_bytes < need) return ST_EWORKSPACE;
  const Geo g{B, Lin, Cin, Cout, K, stride, dil, pad, Lq};
  return run_engine(dtype, g, true, x, w, bias, y, (char*)workspace, (hipStream_t)stream);
}

extern "C" long long stts_conv1d_fwd_tx_workspace_bytes(int dtype, int S, int H, int W, int C, int Cout, int K,
                                                        int stride, int pad, int Lq) {
  if (C != 32 || S < 1 || H < 1 || (long long)S * H > 0x7fffffffLL) return ST_EINVAL;
  return stts_conv1d_fwd_workspace_bytes(dtype, S * H, W, 3 * C, Cout, K, stride, 1, pad, Lq);
}

extern "C" int stts_conv1d_fwd_tx(int dtype, const float* x, const float* w, const float* bias, int S, int H, int W,
                                  int C, int Cout, int K, int stride, int pad, int Lq, int lrelu, float slope, float* y,
                                  void* workspace, long long ws_bytes, void* stream) {
  const long long need = stts_conv1d_fwd_tx_workspace_bytes(dtype, S, H, W, C, Cout, K, stride, pad, Lq);
  if (need < 0) return (int)need;
  if (!x || !w || !y) return ST_EINVAL;
  if (!workspace || ws_bytes < need) return ST_EWORKSPACE;
  const Geo g{S * H, W, 3 * C, Cout, K, stride, 1, pad, Lq};
  return run_engine(dtype, g, true, x, w, bias, y, (char*)workspace, (hipStream_t)stream, nullptr, 1.f, lrelu != 0,
                    slope, H);
}

extern "C" long long stts_conv1d_bwd_tx_workspace_bytes(int dtype, int S, int H, int W, int C, int Cout, int K,
                                                        int stride, int pad, int Lq) {
  if (Cout != 32 || S < 1 || H < 1 || (long long)S * H > 0x7fffffffLL) return ST_EINVAL;
  return stts_conv1d_bwd_workspace_bytes(dtype, S * H, W, C, 3 * Cout, K, stride, 1, pad, Lq);
}

extern "C" int stts_conv1d_bwd_tx(int dtype, const float* dy, const float* wd, int S, int H, int W, int C, int Cout,
                                  int K, int stride, int pad, int Lq, float* dx, void* workspace, long long ws_bytes,
                                  void* stream) {
  const long long need = stts_conv1d_bwd_tx_workspace_bytes(dtype, S, H, W, C, Cout, K, stride, pad, Lq);
  if (need < 0) return (int)need;
  if (!dy || !wd || !dx) return ST_EINVAL;
  if (!workspace || ws_bytes < need) return ST_EWORKSPACE;
  // the input gradient of the tx conv is the dx of the conv C -> 3 Cout whose output chunk j is dy's row
  // h + j - 1 (the expansion of dy, done by the engine's loads): weight chunk j = the Conv2d's row dh = 2 - j
  const Geo g{S * H, W, C, 3 * Cout, K, stride, 1, pad, Lq};
  return run_engine(dtype, g, false, dy, wd, nullptr, dx, (char*)workspace, (hipStream_t)stream, nullptr, 1.f, false,
                    0.f, H);
}

extern "C" long long stts_conv1d_bwd_workspace_bytes(int dtype, int B, int Lin, int Cin, int Cout, int K, int stride,
                                                     int dil, int pad, int Lq) {
  if (dtype != ST_FP32 && dtype != ST_BF16 && dtype != ST_SPLIT) return ST_EDTYPE;
  const Geo g{B, Lin, Cin, Cout, K, stride, dil, pad, Lq};
  if (!geo_ok(g)) return ST_EINVAL;
  if (g.stride > 1 && g.dil > 1) return ST_EINVAL;
  if (g.stride == 1 && g.dil * (g.K - 1) < g.pad) return ST_EINVAL;
  return (long long)ws_layout(g, dtype, false).total;
}

extern "C" int stts_conv1d_bwd(int dtype, const float* x, const float* w, const float* dy, int B, int Lin, int Cin,
                               int Cout, int K, int stride, int dil, int pad, int Lq, float* dx, float* dw,
                               float* db, void* workspace, long long ws_bytes, void* stream) {
  const long long need = stts_conv1d_bwd_workspace_bytes(dtype, B, Lin, Cin, Cout, K, stride, dil, pad, Lq);
  if (need < 0) return (int)need;
  if (!dy || (dx && !w) || (dw && !x)) return ST_EINVAL;
  if (!workspace || ws_bytes < need) return ST_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const Geo g{B, Lin, Cin, Cout, K, stride, dil, pad, Lq};
  const WsLayout L = ws_layout(g, dtype, false);
  char* ws = (char*)workspace;
  if (dx) ST_CHECK(run_engine(dtype, g, false, dy, w, nullptr, dx, ws, s));
  const Slices sl = slices_of(g);
  if (dw && dtype == ST_BF16) {
    ST_CHECK(wgrad_bf16(g, x, dy, (float*)(ws + L.part), dw, s));
  } else if (dw) {
    float* part = (float*)(ws + L.part);
    if (sl.NA == 2 && sl.NB == 2)
      launch_wgrad<2, 2>(g, sl, x, dy, part, s);
    else if (sl.NA == 2)
      launch_wgrad<2, 1>(g, sl, x, dy, part, s);
    else if (sl.NB == 2)
      launch_wgrad<1, 2>(g, sl, x, dy, part, s);
    else
      launch_wgrad<1, 1>(g, sl, x, dy, part, s);
    ST_CHECK_HIP(hipGetLastError());
    const size_t n = (size_t)K * Cout * Cin;
    hipLaunchKernelGGL(k_slice_reduce<float>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, part, sl.S, K, Cout,
                       Cin, dw);
    ST_CHECK_HIP(hipGetLastError());
  }
  if (db) ST_CHECK(bias_grad(g, dy, db, (double*)(ws + L.part2), s));
  return 0;
}

extern "C" int stts_conv1d_wgrad_tx(int dtype, const float* x, const float* dy, int S, int H, int W, int C, int Cout,
                                    int K, int stride, int pad, int Lq, float* dw, float* db, void* workspace,
                                    long long ws_bytes, void* stream) {
  if (dtype != ST_BF16) return ST_EDTYPE;
  const long long need = stts_conv1d_fwd_tx_workspace_bytes(dtype, S, H, W, C, Cout, K, stride, pad, Lq) < 0
                             ? ST_EINVAL
                             : stts_conv1d_bwd_workspace_bytes(dtype, S * H, W, 3 * C, Cout, K, stride, 1, pad, Lq);
  if (need < 0) return (int)need;
  if (!x || !dy || !dw) return ST_EINVAL;
  if (!workspace || ws_bytes < need) return ST_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const Geo g{S * H, W, 3 * C, Cout, K, stride, 1, pad, Lq};
  char* ws = (char*)workspace;
  const WsLayout L = ws_layout(g, dtype, false);
  ST_CHECK(wgrad_bf16(g, x, dy, (float*)(ws + L.part), dw, s, H));
  if (db) ST_CHECK(bias_grad(g, dy, db, (double*)(ws + L.part2), s));
  return 0;
}

// ConvTranspose1d(Cin_T -> Cout_T, K, stride, pad, output_padding implied by Lout) is the dx of the
// conv1d (Cout_T -> Cin_T) with the same weight; its backward is that conv's forward (dx) and wgrad
// with the operands' roles swapped (dw).  gc = the conv's geometry.
namespace {
Geo convT_geo(int B, int Lin, int Cin, int Cout, int K, int stride, int pad, int Lout) {
  return Geo{B, Lout, Cout, Cin, K, stride, 1, pad, Lin};
}
size_t convT_ws(const Geo& gc, int dtype) {
  const size_t a = ws_layout(gc, dtype, false).total, b = ws_layout(gc, dtype, true).total;
  const int S2 = colsum_slices(gc.Cin, (long long)gc.B * gc.Lin);
  return std::max(a, b) + al((size_t)S2 * gc.Cin * 8);
}
}  // namespace

extern "C" long long stts_conv_transpose1d_workspace_bytes(int dtype, int B, int Lin, int Cin, int Cout, int K,
                                                           int stride, int pad, int Lout) {
  if (dtype != ST_FP32 && dtype != ST_BF16 && dtype != ST_SPLIT) return ST_EDTYPE;
  const Geo gc = convT_geo(B, Lin, Cin, Cout, K, stride, pad, Lout);
  if (!geo_ok(gc)) return ST_EINVAL;
  if (stride == 1 && K - 1 < pad) return ST_EINVAL;
  return (long long)convT_ws(gc, dtype);
}

extern "C" int stts_conv_transpose1d_fwd(int dtype, const float* x, const float* w, const float* bias, int B, int Lin,
                                         int Cin, int Cout, int K, int stride, int pad, int Lout, float* y,
                                         void* workspace, long long ws_bytes, void* stream) {
  const long long need = stts_conv_transpose1d_workspace_bytes(dtype, B, Lin, Cin, Cout, K, stride, pad, Lout);
  if (need < 0) return (int)need;
  if (!x || !w || !y) return ST_EINVAL;
  if (!workspace || ws_bytes < need) return ST_EWORKSPACE;
  const Geo gc = convT_geo(B, Lin, Cin, Cout, K, stride, pad, Lout);
  return run_engine(dtype, gc, false, x, w, bias, y, (char*)workspace, (hipStream_t)stream);
}

extern "C" int stts_conv_transpose1d_bwd(int dtype, const float* x, const float* w, const float* dy, int B, int Lin,
                                         int Cin, int Cout, int K, int stride, int pad, int Lout, float* dx, float* dw,
                                         float* db, void* workspace, long long ws_bytes, void* stream) {
  const long long need = stts_conv_transpose1d_workspace_bytes(dtype, B, Lin, Cin, Cout, K, stride, pad, Lout);
  if (need < 0) return (int)need;
  if (!dy || (dx && !w) || (dw && !x)) return ST_EINVAL;
  if (!workspace || ws_bytes < need) return ST_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const Geo gc = convT_geo(B, Lin, Cin, Cout, K, stride, pad, Lout);
  char* ws = (char*)workspace;
  if (dx) ST_CHECK(run_engine(dtype, gc, true, dy, w, nullptr, dx, ws, s));
  if (dw && dtype == ST_BF16) {
    // wgrad of the conv with x := dy (Lout rows, Cout channels) and dy := x (Lin rows, Cin channels)
    ST_CHECK(wgrad_bf16(gc, dy, x, (float*)(ws + ws_layout(gc, dtype, false).part), dw, s));
  } else if (dw) {
    // wgrad of the conv with x := dy (Lout rows, Cout channels) and dy := x (Lin rows, Cin channels)
    const Slices sl = slices_of(gc);
    float* part = (float*)(ws + ws_layout(gc, dtype, false).part);
    if (sl.NA == 2 && sl.NB == 2)
      launch_wgrad<2, 2>(gc, sl, dy, x, part, s);
    else if (sl.NA == 2)
      launch_wgrad<2, 1>(gc, sl, dy, x, part, s);
    else if (sl.NB == 2)
      launch_wgrad<1, 2>(gc, sl, dy, x, part, s);
    else
      launch_wgrad<1, 1>(gc, sl, dy, x, part, s);
    ST_CHECK_HIP(hipGetLastError());
    const size_t n = (size_t)K * gc.Cout * gc.Cin;
    hipLaunchKernelGGL(k_slice_reduce<float>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, part, sl.S, K,
                       gc.Cout, gc.Cin, dw);
    ST_CHECK_HIP(hipGetLastError());
  }
  if (db) {
    const long long R = (long long)B * Lout;
    const int S2 = colsum_slices(Cout, R);
    double* part2 = (double*)(ws + convT_ws(gc, dtype) - al((size_t)S2 * Cout * 8));
    hipLaunchKernelGGL(k_colsum, dim3((unsigned)((Cout + 63) / 64), S2), dim3(256), 0, s, dy, R, Cout, S2, part2);
    ST_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_slice_reduce<double>, dim3((unsigned)((Cout + 255) / 256)), dim3(256), 0, s, part2, S2, 1,
                       Cout, 1, db);
    ST_CHECK_HIP(hipGetLastError());
  }
  return 0;
}
