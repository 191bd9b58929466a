// Fused AdaINResBlock1 iteration for the narrow generator stages (C = 32, and C = 64 at K = 3):
// one launch computes, per tile of output frames,
//     xt = conv1(Snake1(AdaIN1(x)))            dilated Conv1d(C, C, K, dil d)
//     x' = conv2(Snake2(AdaIN2(xt))) + x       Conv1d(C, C, K, dil 1)
// (Modules/hifigan.py:65-74) with xt kept in LDS: it never touches HBM.  AdaIN2 normalises xt
// over the whole utterance, so its statistics must exist before any tile can apply it; a
// statistics-only pass of conv1 (resconv.hip with no output, plan.cpp:resblock1) produces them
// first.  Per iteration that moves 3 activation tensors through HBM (x read twice, x' written)
// instead of 5 (x, xt, xt, x, x'), at the price of conv1's MFMAs twice plus a K-1 row halo.
//
// Tile = 32*(NB-1) output frames.  conv1 is evaluated on the NB 32-row blocks covering the
// tile plus conv2's (K-1)/2-row halo on each side; its epilogue (bias, AdaIN2, Snake2, bf16,
// conv2's zero padding outside [0, L)) writes straight into the LDS window that conv2 reads.
// Both layers' weights stay in LDS for the block's lifetime; the next tile's raw input window
// is prefetched into registers one tile ahead; the residual rows are prefetched before conv1.
// Two barriers per tile.  bf16 storage, v_mfma_f32_32x32x16_bf16, fp32 accumulation.
#include "common.h"
#include "conv_common.h"
#include "kernels.h"

namespace {

template <int C, int K, int DIL>
struct RF {
  static constexpr int NT = 512;                 // 8 waves, one block per CU
  static constexpr int WN = C / 32;              // waves along channels (one 32-channel block each)
  static constexpr int WMW = 8 / WN;             // waves along frames
  static constexpr int NB = 2 * WMW;             // conv1 row blocks per tile (two per wave)
  static constexpr int BM = 32 * (NB - 1);       // output frames per tile
  static constexpr int P1 = DIL * (K - 1) / 2;   // conv1 'same' padding
  static constexpr int P2 = (K - 1) / 2;         // conv2 'same' padding
  static constexpr int R2 = 32 * NB;             // conv1 output rows held for conv2
  static constexpr int R2A = R2 + 32;            // + slack rows read by a discarded conv2 block
  static constexpr int R1 = R2 + DIL * (K - 1);  // input window rows
  static constexpr int XP = C + 8, WP = 40;      // conflict-free ds_read_b128 pitches (bf16)
  static constexpr int NCH = C / 32, G8 = C / 8;
  static constexpr int UNITS = R1 * G8, MAXU = (UNITS + NT - 1) / NT;
  static constexpr int W_B = NCH * K * C * WP * 2;  // one layer's weights in LDS (bytes)
  static constexpr int OFF_C2 = 5 * C * 4;          // coef1 [5][C] f32, coef2 [5][C] f32
  static constexpr int OFF_B1 = OFF_C2 + 5 * C * 4;
  static constexpr int OFF_B2 = OFF_B1 + C * 4;
  static constexpr int OFF_W1 = OFF_B2 + C * 4;
  static constexpr int OFF_W2 = OFF_W1 + W_B;
  static constexpr int OFF_X1 = OFF_W2 + W_B;
  static constexpr int OFF_X2 = OFF_X1 + R1 * XP * 2;
  static constexpr int LDS = OFF_X2 + R2A * XP * 2;
  static_assert(2 * P2 <= 32, "conv2 halo must fit the extra conv1 row block");
  static_assert(NT % G8 == 0, "a thread's window units share one 8-channel group");
  static_assert(OFF_W1 % 16 == 0 && OFF_X1 % 16 == 0 && OFF_X2 % 16 == 0, "LDS carve alignment");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

__device__ __forceinline__ void bf8f(const uint4& r, float (&v)[8]) {
  const unsigned w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 f8bf(const float* v) {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (bf16_t)v[j];
  uint4 r;
  __builtin_memcpy(&r, &o, 16);
  return r;
}

// AdaIN -> Snake coefficients of one channel (resconv.hip:171-175):
//   y = fma(v, a, m1 + ia2) - ia2 * cos(fma(v, a*alpha/pi, m1*alpha/pi)),  m1 = beta - mean*a, ia2 = 1/(2 alpha)
__device__ __forceinline__ void put_coef(const Prologue& pro, int b, int ci, float* cf, int C) {
  float mm, aa, be;
  adain_coeffs(pro, b, ci, mm, aa, be);
  const float al = pro.alpha[ci];
  const float m1 = be - mm * aa, ia2 = 0.5f / al, alr = al * 0.31830988618379067f;
  cf[ci] = m1 + ia2;
  cf[C + ci] = aa;
  cf[2 * C + ci] = aa * alr;
  cf[3 * C + ci] = m1 * alr;
  cf[4 * C + ci] = -ia2;
}

// 8 consecutive channels ch.. of one frame through AdaIN -> Snake with coefficients cf
template <int C>
__device__ __forceinline__ void pro8(const float* cf, int ch, float (&v)[8]) {
  float m2[8], a[8], ar[8], mr[8], nia[8];
  ld8_lds(cf + ch, m2);
  ld8_lds(cf + C + ch, a);
  ld8_lds(cf + 2 * C + ch, ar);
  ld8_lds(cf + 3 * C + ch, mr);
  ld8_lds(cf + 4 * C + ch, nia);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float x2 = __builtin_fmaf(v[j], a[j], m2[j]);
    const float c = __builtin_amdgcn_cosf(__builtin_fmaf(v[j], ar[j], mr[j]));
    v[j] = __builtin_fmaf(c, nia[j], x2);
  }
}

template <int C, int K, int DIL, bool ACC>
__global__ void __launch_bounds__(512, 1) k_resfused(const ResFusedParams p) {
  using G = RF<C, K, DIL>;
  constexpr int NT = G::NT, WN = G::WN, WMW = G::WMW, NB = G::NB, BM = G::BM, XP = G::XP, WP = G::WP;
  constexpr int NCH = G::NCH, G8 = G::G8, UNITS = G::UNITS, MAXU = G::MAXU;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* coef1 = reinterpret_cast<float*>(smem);
  float* coef2 = reinterpret_cast<float*>(smem + G::OFF_C2);
  float* bias1 = reinterpret_cast<float*>(smem + G::OFF_B1);
  float* bias2 = reinterpret_cast<float*>(smem + G::OFF_B2);
  bf16_t* W1s = reinterpret_cast<bf16_t*>(smem + G::OFF_W1);  // [chunk][tap][n][WP], logical k order
  bf16_t* W2s = reinterpret_cast<bf16_t*>(smem + G::OFF_W2);
  bf16_t* X1s = reinterpret_cast<bf16_t*>(smem + G::OFF_X1);  // [R1][XP]: Snake1(AdaIN1(x)), zero padded
  bf16_t* X2s = reinterpret_cast<bf16_t*>(smem + G::OFF_X2);  // [R2A][XP]: Snake2(AdaIN2(xt)), zero padded

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, l32 = lane & 31, hi = lane >> 5;
  const int wn = wid % WN, wm = wid / WN;
  const int L = p.L;
  const int ntm = (L + BM - 1) / BM;
  const long long total = (long long)ntm * p.B;
  const int tbeg = (int)(total * blockIdx.x / gridDim.x);
  const int tend = (int)(total * (blockIdx.x + 1) / gridDim.x);
  if (tbeg >= tend) return;  // uniform over the block

  // ---- both layers' weights and biases -> LDS, once per block (packed layout: st_pack_conv)
  {
    const Rsrc r1 = make_rsrc(p.w1, (unsigned)((size_t)NCH * K * C * 32 * 2));
    const Rsrc r2 = make_rsrc(p.w2, (unsigned)((size_t)NCH * K * C * 32 * 2));
    constexpr int WU = NCH * K * C * 4;  // 16-byte units per layer
    for (int u = tid; u < WU; u += NT) {
      const int g = u & 3, n = (u >> 2) % C, ct = (u >> 2) / C;  // ct = chunk * K + tap
      const unsigned off = (unsigned)((((size_t)ct * C + n) * 32 + 8 * (g ^ ((n >> 2) & 3))) * 2);
      const size_t dst = ((size_t)ct * C + n) * WP + 8 * g;
      *reinterpret_cast<uint4*>(W1s + dst) = bload16(r1, off);
      *reinterpret_cast<uint4*>(W2s + dst) = bload16(r2, off);
    }
    for (int i = tid; i < C; i += NT) {
      bias1[i] = p.b1 ? p.b1[i] : 0.f;
      bias2[i] = p.b2 ? p.b2[i] : 0.f;
    }
  }

  // ---- raw input window of tile t -> registers (rows outside [0, L) read 0 / are zeroed later)
  const int g8 = tid % G8;
  uint4 pre[MAXU];
  auto issue = [&](int t) __attribute__((always_inline)) {
    const int b = t / ntm, mt = t - b * ntm;
    const Rsrc rx = make_rsrc(reinterpret_cast<const bf16_t*>(p.x) + (size_t)b * p.x_bs,
                              (unsigned)((size_t)L * p.x_ld * 2));
    const int gr0 = mt * BM - G::P2 - G::P1;
#pragma unroll
    for (int k = 0; k < MAXU; ++k) {
      const int u = tid + k * NT;
      const int e = (gr0 + u / G8) * p.x_ld + 8 * g8;
      const bool in = (k + 1) * NT <= UNITS || u < UNITS;
      pre[k] = bload16(rx, in && e >= 0 && !(p.dbg & 8) ? (unsigned)e * 2u : OOB);
    }
  };
  auto transform = [&](int t) __attribute__((always_inline)) {
    const int mt = t % ntm;
    const int gr0 = mt * BM - G::P2 - G::P1;
#pragma unroll
    for (int k = 0; k < MAXU; ++k) {
      const int u = tid + k * NT;
      if ((k + 1) * NT <= UNITS || u < UNITS) {
        const int r = u / G8;
        float v[8];
        bf8f(pre[k], v);
        if (!(p.dbg & 1)) pro8<C>(coef1, 8 * g8, v);
        uint4 o = f8bf(v);
        if ((unsigned)(gr0 + r) >= (unsigned)L) o = make_uint4(0, 0, 0, 0);  // conv1 zero padding
        *reinterpret_cast<uint4*>(X1s + r * XP + 8 * g8) = o;
      }
    }
  };

  // ---- conv2 output blocks of this wave: j = wm + WMW*mi (mi = 0, 1); j = NB-1 is discarded
  const int co0 = wn * 32 + hi * 16;  // this lane's 16 channels in every epilogue
  uint4 rres[2][2], racc[ACC ? 2 : 1][2];
  auto issue_epi = [&](int t) __attribute__((always_inline)) {
    const int b = t / ntm, mt = t - b * ntm;
    const Rsrc rr = make_rsrc(reinterpret_cast<const bf16_t*>(p.x) + (size_t)b * p.x_bs,
                              (unsigned)((size_t)L * p.x_ld * 2));
    const Rsrc ra = make_rsrc(ACC ? reinterpret_cast<const bf16_t*>(p.accb) + (size_t)b * p.acc_bs : nullptr,
                              ACC ? (unsigned)((size_t)L * p.acc_ld * 2) : 0u);
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const int q = mt * BM + (wm + WMW * mi) * 32 + l32;
      const unsigned er = (p.dbg & 4) ? OOB : (unsigned)(q * p.x_ld + co0) * 2u;
      rres[mi][0] = bload16(rr, er);
      rres[mi][1] = bload16(rr, er + 16u);
      if constexpr (ACC) {
        const unsigned ea = (unsigned)(q * p.acc_ld + co0) * 2u;
        racc[mi][0] = bload16(ra, ea);
        racc[mi][1] = bload16(ra, ea + 16u);
      }
    }
  };

  float st_s[16], st_q[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) st_s[r] = st_q[r] = 0.f;
  auto flush = [&](int b) __attribute__((always_inline)) {
    if constexpr (!ACC) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float a = st_s[r], q = st_q[r];
#pragma unroll
        for (int o = 16; o >= 1; o >>= 1) {
          a += __shfl_xor(a, o);
          q += __shfl_xor(q, o);
        }
        if (l32 == 0) {
          double* d = (p.stats_slots > 1 ? p.stats + (size_t)(blockIdx.x % p.stats_slots) * p.stats_slot_bs : p.stats) +
                      ((size_t)b * p.stats_ld + co0 + r) * 2;
          atomicAdd(d, (double)a);
          atomicAdd(d + 1, (double)q);
        }
        st_s[r] = st_q[r] = 0.f;
      }
    }
  };

  const bf16_t* x1w = X1s + (size_t)(2 * wm * 32 + l32) * XP + hi * 8;
  const bf16_t* x2w = X2s + (size_t)(wm * 32 + l32) * XP + hi * 8;
  const bf16_t* w1w = W1s + (size_t)(wn * 32 + l32) * WP + hi * 8;
  const bf16_t* w2w = W2s + (size_t)(wn * 32 + l32) * WP + hi * 8;
  const float adiv = (ACC && p.acc_div != 0.f) ? 1.0f / p.acc_div : 1.0f;

  int cur_b = -1;
  issue(tbeg);
  for (int t = tbeg; t < tend; ++t) {
    const int b = t / ntm, mt = t - b * ntm;
    // every wave is past barrier C of the previous tile: X1 and the coefficients are free
    if (b != cur_b) {
      if (cur_b >= 0 && p.stats) flush(cur_b);
      for (int ci = tid; ci < C; ci += NT) {
        put_coef(p.pro1, b, ci, coef1, C);
        put_coef(p.pro2, b, ci, coef2, C);
      }
      cur_b = b;
      __syncthreads();
    }
    transform(t);
    if (t + 1 < tend) issue(t + 1);
    issue_epi(t);
    __syncthreads();  // (B) window complete; every wave is done reading X2 of the previous tile

    // ---------------- conv1 over rows [q0 - P2, q0 - P2 + 32 NB): blocks 2 wm, 2 wm + 1
    f32x16 acc[2];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][r] = 0.f;
#pragma unroll 1
    for (int tap = 0; tap < ((p.dbg & 2) ? 0 : K); ++tap) {
      const bf16_t* xt = x1w + tap * DIL * XP;
      const bf16_t* wt = w1w + tap * C * WP;
#pragma unroll
      for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const bf16x8 wa = *reinterpret_cast<const bf16x8*>(wt + c * K * C * WP + kk * 16);
          bf16x8 xb[2];
#pragma unroll
          for (int mi = 0; mi < 2; ++mi) xb[mi] = *reinterpret_cast<const bf16x8*>(xt + mi * 32 * XP + c * 32 + kk * 16);
#pragma unroll
          for (int mi = 0; mi < 2; ++mi) acc[mi] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, xb[mi], acc[mi], 0, 0, 0);
        }
    }
    // epilogue 1: + bias1 -> AdaIN2 -> Snake2 -> bf16 into X2 (zero outside [0, L): conv2 padding)
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const int r = (2 * wm + mi) * 32 + l32;
      const int q = mt * BM - G::P2 + r;
      const bool in = (unsigned)q < (unsigned)L;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float v[8], bb[8];
        ld8_lds(bias1 + co0 + 8 * h, bb);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = acc[mi][8 * h + j] + bb[j];
        if (!(p.dbg & 1)) pro8<C>(coef2, co0 + 8 * h, v);
        uint4 o = f8bf(v);
        if (!in) o = make_uint4(0, 0, 0, 0);
        *reinterpret_cast<uint4*>(X2s + r * XP + co0 + 8 * h) = o;
      }
    }
    __syncthreads();  // (C) X2 complete

    // ---------------- conv2 over output blocks j = wm + WMW*mi
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][r] = 0.f;
#pragma unroll 1
    for (int tap = 0; tap < ((p.dbg & 2) ? 0 : K); ++tap) {
      const bf16_t* xt = x2w + tap * XP;
      const bf16_t* wt = w2w + tap * C * WP;
#pragma unroll
      for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const bf16x8 wa = *reinterpret_cast<const bf16x8*>(wt + c * K * C * WP + kk * 16);
          bf16x8 xb[2];
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
            xb[mi] = *reinterpret_cast<const bf16x8*>(xt + mi * WMW * 32 * XP + c * 32 + kk * 16);
#pragma unroll
          for (int mi = 0; mi < 2; ++mi) acc[mi] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, xb[mi], acc[mi], 0, 0, 0);
        }
    }
    // epilogue 2: + bias2 + x -> y (statistics) or the resblock running sum
    bf16_t* yb = reinterpret_cast<bf16_t*>(p.y) + (size_t)b * p.y_bs;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const int j = wm + WMW * mi;
      const int q = mt * BM + j * 32 + l32;
      if (j < NB - 1 && q < L) {
        float v[16], bb[16], r0[8], r1[8];
        ld8_lds(bias2 + co0, *reinterpret_cast<float(*)[8]>(&bb[0]));
        ld8_lds(bias2 + co0 + 8, *reinterpret_cast<float(*)[8]>(&bb[8]));
        bf8f(rres[mi][0], r0);
        bf8f(rres[mi][1], r1);
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          v[r] = acc[mi][r] + bb[r] + r0[r];
          v[8 + r] = acc[mi][8 + r] + bb[8 + r] + r1[r];
        }
        if constexpr (ACC) {
          bf8f(racc[mi][0], r0);
          bf8f(racc[mi][1], r1);
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            v[r] = (r0[r] + v[r]) * adiv;
            v[8 + r] = (r1[r] + v[8 + r]) * adiv;
          }
        }
        bf16_t* dst = yb + (size_t)q * p.y_ld + co0;
        if (!(p.dbg & 4)) {
          *reinterpret_cast<uint4*>(dst) = f8bf(&v[0]);
          *reinterpret_cast<uint4*>(dst + 8) = f8bf(&v[8]);
        }
        if constexpr (!ACC) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            st_s[r] += v[r];
            st_q[r] = __builtin_fmaf(v[r], v[r], st_q[r]);
          }
        }
      }
    }
  }
  if (p.stats) flush(cur_b);
}

int g_num_cu_rf = 0;

template <int C, int K, int DIL, bool ACC>
int launch_rf(const ResFusedParams& p, hipStream_t stream) {
  using G = RF<C, K, DIL>;
  auto kern = k_resfused<C, K, DIL, ACC>;
  static bool attr = false;
  if (!attr) {
    ST_CHECK_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
    attr = true;
  }
  if (!g_num_cu_rf) {
    int dev = 0;
    ST_CHECK_HIP(hipGetDevice(&dev));
    ST_CHECK_HIP(hipDeviceGetAttribute(&g_num_cu_rf, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const long long tiles = (long long)((p.L + G::BM - 1) / G::BM) * p.B;
  long long grid = g_num_cu_rf;
  if (grid > tiles) grid = tiles;
  if (g_opt_grid_cap > 0 && grid > g_opt_grid_cap) grid = g_opt_grid_cap;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(G::NT), G::LDS, stream, p);
  return (int)hipGetLastError();
}

template <int C, int K, int DIL>
int launch_rf_a(const ResFusedParams& p, hipStream_t s) {
  return p.accb ? launch_rf<C, K, DIL, true>(p, s) : launch_rf<C, K, DIL, false>(p, s);
}
template <int C, int K>
int launch_rf_d(const ResFusedParams& p, hipStream_t s) {
  switch (p.dil) {
    case 1: return launch_rf_a<C, K, 1>(p, s);
    case 3: return launch_rf_a<C, K, 3>(p, s);
    case 5: return launch_rf_a<C, K, 5>(p, s);
    default: return ST_EINVAL;
  }
}

}  // namespace

bool st_resfused_eligible(int C, int K, int dil, int dtype) {
  // the statistics-only conv1 launch runs on resconv.hip (the general engine has no y == null mode)
  if (!g_opt_resfused || !g_opt_resconv || dtype != ST_BF16) return false;
  if (!(dil == 1 || dil == 3 || dil == 5)) return false;
  if (C == 32) return K == 3 || K == 7 || K == 11;
  if (C == 64) return K == 3;
  return false;
}

int st_resfused(const ResFusedParams& pin, hipStream_t stream) {
  if (pin.B <= 0 || pin.L <= 0) return ST_OK;
  ResFusedParams p = pin;
  p.dbg = g_opt_debug;
  if (!st_resfused_eligible(p.C, p.K, p.dil, ST_BF16)) return ST_EINVAL;
  if (p.x_ld % 8 || p.y_ld % 8 || (p.accb && p.acc_ld % 8) || (p.accb && p.stats)) return ST_EINVAL;
  if (!p.pro1.stats || !p.pro1.gamma || !p.pro1.alpha || !p.pro2.stats || !p.pro2.gamma || !p.pro2.alpha)
    return ST_EINVAL;
  if (p.C == 32) {
    switch (p.K) {
      case 3: return launch_rf_d<32, 3>(p, stream);
      case 7: return launch_rf_d<32, 7>(p, stream);
      case 11: return launch_rf_d<32, 11>(p, stream);
    }
  } else if (p.C == 64 && p.K == 3) {
    return launch_rf_d<64, 3>(p, stream);
  }
  return ST_EINVAL;
}
