// Split-operand (STTS_SPLIT, the accuracy mode) resblock conv engine for the small-channel generator stages
// (C = 32 / 64): the dilated Conv1d(C, C, K, dilation d) of every AdaINResBlock1 iteration
// (Modules/hifigan.py:26-80, forward :65-74) with the AdaIN -> Snake prologue and the bias / residual /
// resblock-average / InstanceNorm-statistics epilogue fused, on fp32 activations.  Every operand is split into
// bf16 parts, v = hi + lo (hi = bf16(v) round-to-nearest-even, lo = bf16(v - hi)), and the product is formed as
// W_lo X_hi + W_hi X_lo + W_hi X_hi on v_mfma_f32_32x32x16_bf16 with fp32 accumulation (~16 significant bits
// per operand; the lo*lo term, ~2^-18 of a product, is dropped).  tests/test_gpu_split.py pins it.
//
// Structure (the lock-step resconv.hip tile loop): a block owns contiguous 256-frame tiles; the layer's weights
// (hi and lo copies) stay in LDS; the raw fp32 window of tile t+2 is prefetched into registers while tile t
// runs; the window is transformed (AdaIN -> Snake, sin^2 u = (1 - cos 2u) / 2 on v_cos) and written to LDS as
// a hi and a lo window; the epilogue works from registers (a lane owns 16 consecutive channels of one frame).
//
// C = 64: the hi + lo weights of a K = 11 layer (180 KB) do not fit the LDS next to two windows, so the conv
// runs as two passes over the input-channel halves: pass 1 (channels 0-31) writes its fp32 partial sums to a
// scratch buffer (p.splitk_ws), pass 2 (channels 32-63) adds them and runs the epilogue.  Each pass holds
// 90 KB of weights and transforms only its own 32 channels.
#include "common.h"
#include "conv_common.h"
#include "kernels.h"

namespace {

template <int NOUT, int K, int DIL>
struct RS {
  static constexpr int WAVES = NOUT == 32 ? 4 : 8;
  static constexpr int WAVES_N = NOUT / 32;
  static constexpr int NT = 64 * WAVES;
  static constexpr int FW = 64;                      // frames per wave
  static constexpr int MT = FW / 32;                 // 32-frame blocks per wave
  static constexpr int BM = (WAVES / WAVES_N) * FW;  // frames per tile (256)
  static constexpr int PAD = DIL * (K - 1) / 2;
  static constexpr int R = BM + DIL * (K - 1);       // window rows
  static constexpr int XP = 40;                      // window row pitch (bf16): 32 channels + 8
  static constexpr int WP = 40;                      // weight row pitch (bf16)
  static constexpr int UNITS = R * 4;                // 8-channel (32-B fp32) units per window
  static constexpr int MAXU = (UNITS + NT - 1) / NT;
  static constexpr int OFF_BIAS = 5 * 32 * 4;        // after coef [5][32] f32
  static constexpr int OFF_W = OFF_BIAS + NOUT * 4;
  static constexpr int W_EL = K * NOUT * WP;         // one copy (hi or lo), bf16 elements
  static constexpr int OFF_X = OFF_W + 2 * W_EL * 2;
  static constexpr int X_EL = R * XP;                // one window (hi or lo)
  static constexpr int LDS = OFF_X + 2 * X_EL * 2;
  static_assert(OFF_W % 16 == 0 && OFF_X % 16 == 0 && (X_EL * 2) % 16 == 0, "LDS carve alignment");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

struct U8 { uint4 a, b; };  // 8 fp32 values

__device__ __forceinline__ void u8_to_f32(const U8& r, float (&v)[8]) {
  float4 a, b;
  __builtin_memcpy(&a, &r.a, 16);
  __builtin_memcpy(&b, &r.b, 16);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
// 16 fp32 values at byte offset `off` (OOB: zeros)
__device__ __forceinline__ void bload64(Rsrc r, unsigned off, float (&v)[16]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint4 u = bload16(r, off == OOB ? OOB : off + 16u * i);
    float4 f;
    __builtin_memcpy(&f, &u, 16);
    v[4 * i] = f.x; v[4 * i + 1] = f.y; v[4 * i + 2] = f.z; v[4 * i + 3] = f.w;
  }
}
__device__ __forceinline__ void bstore64(Rsrc r, unsigned off, const float (&v)[16]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float4 f = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
    uint4 u;
    __builtin_memcpy(&u, &f, 16);
    bstore16(r, off == OOB ? OOB : off + 16u * i, u);
  }
}

// PASS: 0 = the whole conv (C = 32), 1 = input channels 0-31 of a C = 64 conv -> fp32 partials in
// p.splitk_ws, 2 = channels 32-63 + the partials + the epilogue.  ACC: the launch adds into the resblock
// running sum (p.accb / p.acc_div, hifigan.py:336-342) and keeps no statistics.
// PF: the epilogue's residual / running-sum / partial rows are loaded right after the window barrier, so their
// latency hides behind the tile's MFMAs instead of being exposed per fragment in the epilogue (default; STTS_OPT_EXP
// 16384 turns it off for A/B: bit-identical, accuracy-mode step 91.4 -> 90.5 ms, k11 residual launches 928 -> 776 us,
// profiles/r05_ab_ressplit_prefetch.txt)
// SEG: several tile ranges per workgroup (bigconv2.hip k_bigconv2: the plain instantiation runs one range)
template <int NOUT, int K, int DIL, int PASS, bool ACC, bool PF = false, bool SEG = false>
__global__ void __launch_bounds__(NOUT == 32 ? 256 : 512, NOUT == 32 ? 2 : 1) k_ressplit(const ConvParams p) {
  using G = RS<NOUT, K, DIL>;
  constexpr int NT = G::NT, BM = G::BM, MT = G::MT, XP = G::XP, WP = G::WP, FW = G::FW;
  constexpr int UNITS = G::UNITS, MAXU = G::MAXU, WAVES_N = G::WAVES_N;
  constexpr int NCHT = NOUT / 32;      // 32-channel chunks of the whole conv (packed weight layout)
  constexpr int CH = PASS == 2 ? 1 : 0;  // this pass's input chunk
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* coef = reinterpret_cast<float*>(smem);  // [5][32]
  float* bias_s = reinterpret_cast<float*>(smem + G::OFF_BIAS);
  bf16_t* Ws = reinterpret_cast<bf16_t*>(smem + G::OFF_W);  // [tap][n][WP] hi, then the lo copy
  bf16_t* Xs = reinterpret_cast<bf16_t*>(smem + G::OFF_X);  // [R][XP] hi, then the lo window

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, l32 = lane & 31, hi = lane >> 5;
  const int wn = wid % WAVES_N, wm = wid / WAVES_N;
  const int ntm = (p.Lq + BM - 1) / BM;
  const long long total = (long long)ntm * p.B;
  // tile ranges (kernels.h tile_range: one per workgroup, or utterance-relative segments); the lambdas
  // below read the current range by reference
  const int nv = SEG ? tile_nv(p, p.B) : (int)gridDim.x;
  if ((int)blockIdx.x >= nv) return;  // uniform over the block
  int tbeg = 0, tend = 0;

  {  // this pass's weights (hi and lo), in logical k order, and the bias
    const size_t copy = (size_t)NCHT * K * NOUT * 32;  // elements of one packed copy
    const Rsrc rw = make_rsrc(p.w, (unsigned)(2 * copy * 2));
    constexpr int WU = K * NOUT * 4;  // 16-byte units of one copy of this chunk
    for (int u = tid; u < 2 * WU; u += NT) {
      const int cp = u >= WU, uu = cp ? u - WU : u;
      const int g = uu & 3, n = (uu >> 2) % NOUT, tap = (uu >> 2) / NOUT;
      const size_t src = cp * copy + (((size_t)CH * K + tap) * NOUT + n) * 32 + 8 * (g ^ ((n >> 2) & 3));
      *reinterpret_cast<uint4*>(Ws + (size_t)cp * G::W_EL + ((size_t)tap * NOUT + n) * WP + 8 * g) =
          bload16(rw, (unsigned)(src * 2));
    }
    for (int i = tid; i < NOUT; i += NT) bias_s[i] = (PASS != 1 && p.bias) ? p.bias[i] : 0.f;
  }

  const int g8 = tid & 3;  // this thread's 8-channel group in every window unit (NT % 4 == 0)
  auto issue = [&](int t, U8 (&pre)[MAXU]) __attribute__((always_inline)) {
    const int b = t / ntm, mt = t - b * ntm;
    const Rsrc rx = make_rsrc(reinterpret_cast<const float*>(p.x) + (size_t)b * p.x_bs,
                              (unsigned)((size_t)p.Lin * p.x_ld * 4));
    const int gr0 = mt * BM - G::PAD;
#pragma unroll
    for (int k = 0; k < MAXU; ++k) {
      const int u = tid + k * NT;
      const int e = (gr0 + u / 4) * p.x_ld + CH * 32 + 8 * g8;  // rows past Lin read 0 (descriptor range)
      const bool in = (k + 1) * NT <= UNITS || u < UNITS;
      const unsigned off = in && e >= 0 ? (unsigned)e * 4u : OOB;
      pre[k].a = bload16(rx, off);
      pre[k].b = bload16(rx, off == OOB ? OOB : off + 16u);
    }
  };

  float st_s[ACC ? 1 : 16], st_q[ACC ? 1 : 16];
  if constexpr (!ACC) {
#pragma unroll
    for (int r = 0; r < 16; ++r) st_s[r] = st_q[r] = 0.f;
  }
  auto flush = [&](int b) __attribute__((always_inline)) {
    if constexpr (!ACC && PASS != 1) {
      float a, q;
      stat_bfly16(st_s, st_q, l32, a, q);
      if (l32 < 16) {
        double* d = stats_slot(p, blockIdx.x) + ((size_t)b * p.stats_ld + wn * 32 + hi * 16 + l32) * ST_W;
        fx_add(d, a);
        fx_add(d + 2, q);
      }
    }
  };

  // AdaIN -> Snake per element, as resconv.hip: y = fma(v, a, m2) - ia2 cos(2 alpha x), the cosine argument
  // in revolutions; then the hi / lo split
  auto transform = [&](int t, const U8 (&pre)[MAXU]) __attribute__((always_inline)) {
    const int mt = t % ntm;
    const int gr0 = mt * BM - G::PAD;
    float m2[8], a[8], ar[8], mr[8], nia[8];
    ld8_lds(coef + 8 * g8, m2);
    ld8_lds(coef + 32 + 8 * g8, a);
    ld8_lds(coef + 64 + 8 * g8, ar);
    ld8_lds(coef + 96 + 8 * g8, mr);
    ld8_lds(coef + 128 + 8 * g8, nia);
#pragma unroll
    for (int k = 0; k < MAXU; ++k) {
      const int u = tid + k * NT;
      if ((k + 1) * NT <= UNITS || u < UNITS) {
        const int r = u / 4;
        float v[8];
        u8_to_f32(pre[k], v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x2 = __builtin_fmaf(v[j], a[j], m2[j]);
          const float c = __builtin_amdgcn_cosf(__builtin_fmaf(v[j], ar[j], mr[j]));
          v[j] = __builtin_fmaf(c, nia[j], x2);
        }
        bf16x8 h, l;
        const bool pad = (unsigned)(gr0 + r) >= (unsigned)p.Lin;  // zero padding is post-prologue
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x = pad ? 0.f : v[j];
          h[j] = (bf16_t)x;
          l[j] = (bf16_t)(x - (float)h[j]);
        }
        *reinterpret_cast<bf16x8*>(Xs + r * XP + 8 * g8) = h;
        *reinterpret_cast<bf16x8*>(Xs + G::X_EL + r * XP + 8 * g8) = l;
      }
    }
  };

  int cur_b = -1;
  const Rsrc rpart = make_rsrc(p.splitk_ws, PASS ? (unsigned)((size_t)p.B * p.Lq * NOUT * 4) : 0u);
  auto step = [&](int t, U8 (&pre)[MAXU]) __attribute__((always_inline)) {
    const int b = t / ntm, mt = t - b * ntm;
    if (b != cur_b) {
      if (cur_b >= 0 && p.stats) flush(cur_b);
      // every wave is past its previous transform (barrier B of the previous step): coef is free
      for (int ci = tid; ci < 32; ci += NT) {
        float mm, aa, be;
        adain_coeffs(p.pro, b, CH * 32 + ci, mm, aa, be);
        const float al = p.pro.alpha[CH * 32 + ci];
        const float m1 = be - mm * aa, ia2 = 0.5f / al, alr = al * 0.31830988618379067f;  // alpha / pi
        coef[ci] = m1 + ia2;
        coef[32 + ci] = aa;
        coef[64 + ci] = aa * alr;
        coef[96 + ci] = m1 * alr;
        coef[128 + ci] = -ia2;
      }
      cur_b = b;
    }
    __syncthreads();  // (A) coef / weights visible; every wave done reading Xs of the previous tile
    transform(t, pre);
    if (t + 2 < tend) issue(t + 2, pre);
    __syncthreads();  // (B) windows complete

    // (PF) the epilogue's input rows of this tile, in flight during the MFMAs
    const int co0 = wn * 32 + hi * 16;
    const Rsrc rr = make_rsrc(p.res ? reinterpret_cast<const float*>(p.res) + (size_t)b * p.res_bs : nullptr,
                              p.res ? (unsigned)((size_t)p.Lq * p.res_ld * 4) : 0u);
    const Rsrc ra = make_rsrc(ACC ? reinterpret_cast<const float*>(p.accb) + (size_t)b * p.acc_bs : nullptr,
                              ACC ? (unsigned)((size_t)p.Lq * p.acc_ld * 4) : 0u);
    constexpr int NPF = PF ? MT : 1;
    float rv_pf[NPF][16], av_pf[NPF][16], pp_pf[NPF][16];
    if constexpr (PF) {
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) {
        const int q = mt * BM + wm * FW + mi * 32 + l32;
        const bool valid = q < p.Lq;
        if constexpr (PASS == 2) {
          const unsigned pe = valid ? (unsigned)((((size_t)b * p.Lq + q) * NOUT + co0) * 4) : OOB;
          bload64(rpart, pe, pp_pf[mi]);
        }
        if (p.res) bload64(rr, valid ? (unsigned)((q * p.res_ld + co0) * 4) : OOB, rv_pf[mi]);
        if constexpr (ACC) bload64(ra, valid ? (unsigned)((q * p.acc_ld + co0) * 4) : OOB, av_pf[mi]);
      }
    }

    f32x16 acc[MT];
#pragma unroll
    for (int mi = 0; mi < MT; ++mi)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][r] = 0.f;
    const bf16_t* xw = Xs + (size_t)(wm * FW + l32) * XP + hi * 8;
    const bf16_t* ww = Ws + (size_t)(wn * 32 + l32) * WP + hi * 8;
#pragma unroll
    for (int tap = 0; tap < K; ++tap) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const bf16_t* wt = ww + tap * NOUT * WP + kk * 16;
        const bf16x8 wh = *reinterpret_cast<const bf16x8*>(wt);
        const bf16x8 wl = *reinterpret_cast<const bf16x8*>(wt + G::W_EL);
#pragma unroll
        for (int mi = 0; mi < MT; ++mi) {
          const bf16_t* xt = xw + (tap * DIL + mi * 32) * XP + kk * 16;
          const bf16x8 xh = *reinterpret_cast<const bf16x8*>(xt);
          const bf16x8 xl = *reinterpret_cast<const bf16x8*>(xt + G::X_EL);
          acc[mi] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, xh, acc[mi], 0, 0, 0);
          acc[mi] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xl, acc[mi], 0, 0, 0);
          acc[mi] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xh, acc[mi], 0, 0, 0);
        }
      }
    }

    // ---- epilogue: lane = frame l32 of block mi, channels co0 + r
    const Rsrc ry = make_rsrc(reinterpret_cast<float*>(p.y) + (size_t)b * p.y_bs, (unsigned)((size_t)p.Lq * p.y_ld * 4));
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) {
      const int q = mt * BM + wm * FW + mi * 32 + l32;
      const bool valid = q < p.Lq;
      const unsigned pe = valid ? (unsigned)((((size_t)b * p.Lq + q) * NOUT + co0) * 4) : OOB;
      float v[16];
      if constexpr (PASS == 1) {
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = acc[mi][r];
        bstore64(rpart, pe, v);
        continue;
      }
      float bb[16];
      ld8_lds(bias_s + co0, *reinterpret_cast<float(*)[8]>(&bb[0]));
      ld8_lds(bias_s + co0 + 8, *reinterpret_cast<float(*)[8]>(&bb[8]));
      if constexpr (PASS == 2) {
        float pp[16];
        if constexpr (PF) {
#pragma unroll
          for (int r = 0; r < 16; ++r) pp[r] = pp_pf[mi][r];
        } else {
          bload64(rpart, pe, pp);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = (pp[r] + acc[mi][r]) + bb[r];
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = acc[mi][r] + bb[r];
      }
      if (p.res) {
        float rv[16];
        if constexpr (PF) {
#pragma unroll
          for (int r = 0; r < 16; ++r) rv[r] = rv_pf[mi][r];
        } else {
          bload64(rr, valid ? (unsigned)((q * p.res_ld + co0) * 4) : OOB, rv);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = (v[r] + rv[r]) * p.out_scale;
      }
      if constexpr (ACC) {
        float av[16];
        if constexpr (PF) {
#pragma unroll
          for (int r = 0; r < 16; ++r) av[r] = av_pf[mi][r];
        } else {
          bload64(ra, valid ? (unsigned)((q * p.acc_ld + co0) * 4) : OOB, av);
        }
        if (p.acc_div != 0.f) {
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = (av[r] + v[r]) / p.acc_div;  // the reference divides
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = av[r] + v[r];
        }
      }
      bstore64(ry, valid ? (unsigned)((q * p.y_ld + co0) * 4) : OOB, v);
      if constexpr (!ACC) {
        if (valid) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            st_s[r] += v[r];
            st_q[r] = __builtin_fmaf(v[r], v[r], st_q[r]);
          }
        }
      }
    }
  };

  for (int vb = blockIdx.x; vb < nv; vb += gridDim.x) {
  {
    long long tb_, te_;
    if constexpr (SEG) {
      tile_range(p, vb, nv, total, ntm, tb_, te_);
    } else {
      tb_ = total * vb / gridDim.x;
      te_ = total * (vb + 1) / gridDim.x;
    }
    tbeg = (int)tb_;
    tend = (int)te_;
  }
  if (tbeg >= tend) continue;  // uniform over the block
  U8 preA[MAXU], preB[MAXU];
  issue(tbeg, preA);
  if (tbeg + 1 < tend) issue(tbeg + 1, preB);
  for (int t = tbeg; t < tend; t += 2) {
    step(t, preA);
    if (t + 1 < tend) step(t + 1, preB);
  }
  if (p.stats) flush(cur_b);
  cur_b = -1;  // (flushed: the next range re-stages its coefficients)
  if constexpr (!SEG) break;  // (one range)
  __syncthreads();
  }  // tile ranges
}

int g_num_cu_rs = 0;

template <int NOUT, int K, int DIL, int PASS, bool ACC, bool PF = false>
int launch_rs_pf(const ConvParams& p, hipStream_t stream) {
  using G = RS<NOUT, K, DIL>;
  auto kern0 = k_ressplit<NOUT, K, DIL, PASS, ACC, PF, false>;
  auto kern1 = k_ressplit<NOUT, K, DIL, PASS, ACC, PF, true>;
  static bool attr = false;
  if (!attr) {
    ST_CHECK_HIP(hipFuncSetAttribute((const void*)kern0, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
    ST_CHECK_HIP(hipFuncSetAttribute((const void*)kern1, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
    attr = true;
  }
  if (!g_num_cu_rs) {
    int dev = 0;
    ST_CHECK_HIP(hipGetDevice(&dev));
    ST_CHECK_HIP(hipDeviceGetAttribute(&g_num_cu_rs, hipDeviceAttributeMultiprocessorCount, dev));
  }
  int per_cu = occupancy_cached((const void*)kern0, G::NT, G::LDS);
  if (per_cu < 1) per_cu = 1;
  const long long tiles = (long long)((p.Lq + G::BM - 1) / G::BM) * p.B;
  ConvParams q = p;
  const int seg = st_seg_choice(p, 1, g_num_cu_rs * per_cu);
  long long grid = (long long)g_num_cu_rs * per_cu;
  if (grid > (seg ? (long long)p.B * seg : tiles)) grid = seg ? (long long)p.B * seg : tiles;
  if (g_opt_grid_cap > 0 && grid > g_opt_grid_cap) grid = g_opt_grid_cap;
  const bool segk = seg > 0 && grid < (long long)p.B * seg;  // (one segment per workgroup = the plain even split)
  q.seg = segk ? seg : 0;
  hipLaunchKernelGGL(segk ? kern1 : kern0, dim3((unsigned)grid), dim3(G::NT), G::LDS, stream, q);
  return (int)hipGetLastError();
}

template <int NOUT, int K, int DIL, int PASS, bool ACC>
int launch_rs(const ConvParams& p, hipStream_t stream) {
  // (the prefetch only where the epilogue reads rows: a residual, a running sum or the pass-1 partials)
  if (!(g_opt_exp & 16384) && (p.res || ACC || PASS == 2)) return launch_rs_pf<NOUT, K, DIL, PASS, ACC, true>(p, stream);
  return launch_rs_pf<NOUT, K, DIL, PASS, ACC>(p, stream);
}

template <int NOUT, int K, int DIL>
int launch_rs_a(const ConvParams& p, hipStream_t s) {
  if constexpr (NOUT == 32) return p.accb ? launch_rs<32, K, DIL, 0, true>(p, s) : launch_rs<32, K, DIL, 0, false>(p, s);
  const int r = launch_rs<64, K, DIL, 1, false>(p, s);
  if (r) return r;
  return p.accb ? launch_rs<64, K, DIL, 2, true>(p, s) : launch_rs<64, K, DIL, 2, false>(p, s);
}

template <int NOUT, int K>
int launch_rs_d(const ConvParams& p, hipStream_t s) {
  switch (p.dil) {
    case 1: return launch_rs_a<NOUT, K, 1>(p, s);
    case 3: return launch_rs_a<NOUT, K, 3>(p, s);
    case 5: return launch_rs_a<NOUT, K, 5>(p, s);
    default: return ST_EINVAL;
  }
}

template <int NOUT>
int launch_rs_k(const ConvParams& p, hipStream_t s) {
  switch (p.KS) {
    case 3: return launch_rs_d<NOUT, 3>(p, s);
    case 7: return launch_rs_d<NOUT, 7>(p, s);
    case 11: return launch_rs_d<NOUT, 11>(p, s);
    default: return ST_EINVAL;
  }
}

}  // namespace

int g_opt_ressplit = 1;

bool st_ressplit_eligible(const ConvParams& p, int dtype) {
  if (!g_opt_ressplit || dtype != ST_SPLIT) return false;
  const int C = p.Cout;
  if (!(C == 32 || C == 64) || p.Cin != C || p.N != C || p.nchunks * 32 != C) return false;
  if (!(p.KS == 3 || p.KS == 7 || p.KS == 11) || !(p.dil == 1 || p.dil == 3 || p.dil == 5)) return false;
  if ((p.kw != 0 && p.kw != p.KS) || p.row_off != 0 || p.stride != 1 || p.up != 1 || p.opad != 0) return false;
  if (p.pad != p.dil * (p.KS - 1) / 2 || p.Lq != p.Lout || p.Lq != p.Lin) return false;
  if (p.y_row_off || p.y_f32 || p.epi_tanh || p.epi_lrelu || p.epi_gelu || p.reflect_front || p.zc_period || p.res_shift) return false;
  if (p.pro.mode != (PRO_AFFINE | PRO_SNAKE) || !p.pro.alpha || !p.pro.stats || !p.pro.gamma) return false;
  if (p.accb && p.stats) return false;
  if (!p.y || p.x_ld % 4 || p.y_ld % 4 || (p.res && p.res_ld % 4) || (p.accb && p.acc_ld % 4)) return false;
  // C = 64 runs in two passes through the fp32 partial scratch
  if (C == 64 && (!p.splitk_ws || p.splitk_ws_elems < (long long)p.B * p.Lq * 64)) return false;
  return true;
}

int st_ressplit(const ConvParams& p, hipStream_t stream) {
  if (p.Cout == 32) return launch_rs_k<32>(p, stream);
  if (p.Cout == 64) return launch_rs_k<64>(p, stream);
  return ST_EINVAL;
}
