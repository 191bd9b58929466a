// Resblock conv engine for the small-channel generator stages (C = 32 / 64; HBM-bound):
// the dilated Conv1d(C, C, K, dilation d, padding d(K-1)/2) of every AdaINResBlock1 iteration
// (Modules/hifigan.py:26-80, forward :65-74), with the AdaIN -> Snake prologue and the bias /
// residual / resblock-average / InstanceNorm-statistics epilogue fused.  bf16 storage, bf16 MFMA
// (v_mfma_f32_32x32x16_bf16), fp32 accumulation.  The general engine (conv1d.hip) serves every
// other conv; st_conv1d routes eligible launches here.
//
// What differs from the general engine (profiles/r01_pmc_*: waves parked ~45 % on s_waitcnt,
// ~950 VALU instructions per tile-wave):
//   * taps, dilation and channel count are template parameters: LDS operand addresses in the
//     MFMA loop are one base per tap + immediates;
//   * the raw input window is prefetched TWO tiles ahead (two named register sets, the tile
//     loop unrolled by two), so each load has a full tile of MFMA + epilogue time to land;
//   * the weights of the whole layer stay in LDS for the block's lifetime;
//   * statistics are accumulated per lane in registers (a lane owns 16 channels of one frame)
//     and reduced across lanes only when the block leaves an utterance.
#include "common.h"
#include "conv_common.h"
#include "kernels.h"

namespace {

// UPS: the HiFi-GAN ups[3] polyphase ConvTranspose1d (64 -> 32, x2; hifigan.py:292-294, 333-335) as the 2-tap
// GEMM of DESIGN §2: C = Cin = N = u Cout = 64 columns, tap t reads input row q + t - 1 (left pad 1), Snake
// prologue without AdaIN, and the epilogue maps row q / column n to output frame q u + n / Cout - opad,
// channel n % Cout (residual = the noise branch at the same position; statistics per channel n % Cout).
template <int C, int K, int DIL, int WAVES, int WAVES_N, bool UPS = false>
struct RC {
  static constexpr int NT = 64 * WAVES;              // threads per block
  static constexpr int FW = 64;                      // frames per wave
  static constexpr int MT = FW / 32;                 // 32-frame blocks per wave
  static constexpr int BM = (WAVES / WAVES_N) * FW;  // frames per tile
  static constexpr int NTL = C / 32 / WAVES_N;       // 32-channel output blocks per wave
  static constexpr int NCH = C / 32;                 // 32-channel K chunks
  static constexpr int PAD = UPS ? 1 : DIL * (K - 1) / 2;  // 'same' padding (UPS: rows q - 1, q)
  static constexpr int R = BM + DIL * (K - 1);       // window rows
  static constexpr int XP = C + 8;                   // window row pitch (bf16): conflict-free ds_read_b128
  static constexpr int WP = 40;                      // weight row pitch (bf16): 32 + 8
  static constexpr int G8 = C / 8;                   // 8-channel groups per window row
  static constexpr int UNITS = R * G8;               // 16-byte window units per tile
  static constexpr int MAXU = (UNITS + NT - 1) / NT;
  static constexpr int OFF_BIAS = 5 * C * 4;         // after coef [5][C] f32
  static constexpr int OFF_W = OFF_BIAS + C * 4;
  static constexpr int W_B = NCH * K * C * WP * 2;
  static constexpr int OFF_X = OFF_W + W_B;
  static constexpr int LDS = OFF_X + R * XP * 2;
  static_assert(NT % G8 == 0, "a thread's window units must share one 8-channel group");
  static_assert(OFF_W % 16 == 0 && OFF_X % 16 == 0, "LDS carve alignment");
  static_assert(NTL >= 1 && WAVES % WAVES_N == 0, "wave grid");
};

__device__ __forceinline__ void bf8_to_f32(const uint4& r, float (&v)[8]) {
  const unsigned w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 f32_to_bf8(const float* v) {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (bf16_t)v[j];
  uint4 r;
  __builtin_memcpy(&r, &o, 16);
  return r;
}

// ACC: the launch adds the output into the resblock running sum (p.accb, p.acc_div) and keeps
// no statistics (hifigan.py:336-342); otherwise statistics are kept when p.stats is set.
// RPF: the residual / running-sum rows of tile t+1 are loaded during tile t (two register sets,
// STTS_OPT_EXP bit 4), instead of at the start of the tile that consumes them
// PF: window prefetch depth in tiles (2; 3 keeps a third raw window in flight: one block per CU at
// C = 64 holds ~40 KB of loads in flight with two, below the ~70 KB an HBM-rate stream needs)
// IL: the epilogue of tile t - 1 is issued inside tile t's MFMA loop (one basic block: branch-free, the stores go
// through a buffer descriptor and rows that are not stored get an out-of-range offset), so its VALU work, residual
// adds and stores fill the gaps between the MFMAs instead of running after them with the MFMA pipe idle
// SEG: several tile ranges per workgroup (bigconv2.hip k_bigconv2: the plain instantiation runs one range)
// MINB: blocks per CU the register allocation is held to (0: 8 / WAVES, two waves per SIMD)
template <int C, int K, int DIL, int WAVES, int WAVES_N, bool ACC, bool RPF = false, int PF = 2, bool UPS = false,
          bool IL = false, bool SEG = false, int MINB = 0>
__global__ void __launch_bounds__(64 * WAVES, MINB ? MINB : 8 / WAVES) k_resconv(const ConvParams p) {
  using G = RC<C, K, DIL, WAVES, WAVES_N, UPS>;
  constexpr int NT = G::NT, BM = G::BM, MT = G::MT, NTL = G::NTL, NCH = G::NCH, XP = G::XP, WP = G::WP;
  constexpr int G8 = G::G8, UNITS = G::UNITS, MAXU = G::MAXU, FW = G::FW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* coef = reinterpret_cast<float*>(smem);  // [5][C]: prologue coefficients (see step)
  float* bias_s = reinterpret_cast<float*>(smem + G::OFF_BIAS);
  bf16_t* Ws = reinterpret_cast<bf16_t*>(smem + G::OFF_W);  // [chunk][tap][n][WP], logical k order
  bf16_t* Xs = reinterpret_cast<bf16_t*>(smem + G::OFF_X);  // [R][XP], prologue applied

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, l32 = lane & 31, hi = lane >> 5;
  const int wn = wid % WAVES_N, wm = wid / WAVES_N;
  const int ntm = (p.Lq + BM - 1) / BM;
  const long long total = (long long)ntm * p.B;
  // tile ranges (kernels.h tile_range: one per workgroup, or utterance-relative segments); the lambdas
  // below read the current range [tbeg, tend) by reference
  const int nv = SEG ? tile_nv(p, p.B) : (int)gridDim.x;
  if ((int)blockIdx.x >= nv) return;  // uniform over the block
  int tbeg = 0, tend = 0;

  // ---- layer constants -> LDS, once per block
  {
    const Rsrc rw = make_rsrc(p.w, (unsigned)((size_t)NCH * K * C * 32 * 2));
    constexpr int WU = NCH * K * C * 4;  // 16-byte units
    for (int u = tid; u < WU; u += NT) {
      const int g = u & 3, n = (u >> 2) % C, ct = (u >> 2) / C;  // ct = chunk * K + tap
      const unsigned off = (unsigned)((((size_t)ct * C + n) * 32 + 8 * (g ^ ((n >> 2) & 3))) * 2);
      *reinterpret_cast<uint4*>(Ws + ((size_t)ct * C + n) * WP + 8 * g) = bload16(rw, off);
    }
    for (int i = tid; i < C; i += NT) bias_s[i] = p.bias ? p.bias[UPS ? i % p.Cout : i] : 0.f;
  }

  const int g8 = tid % G8;  // this thread's 8-channel group in every window unit
  auto issue = [&](int t, uint4 (&pre)[MAXU]) __attribute__((always_inline)) {
    const int b = t / ntm, mt = t - b * ntm;
    const Rsrc rx = make_rsrc(reinterpret_cast<const bf16_t*>(p.x) + (size_t)b * p.x_bs,
                              (unsigned)((size_t)p.Lin * p.x_ld * 2));
    const int gr0 = mt * BM - G::PAD;
#pragma unroll
    for (int k = 0; k < MAXU; ++k) {
      const int u = tid + k * NT;
      const int e = (gr0 + u / G8) * p.x_ld + 8 * g8;  // rows past Lin read 0 (descriptor range)
      const bool in = (k + 1) * NT <= UNITS || u < UNITS;
      pre[k] = bload16(rx, in && e >= 0 ? (unsigned)e * 2u : OOB);
    }
  };

  // epilogue prefetch: residual rows of the tile (16 channels of one frame per lane)
  struct EpiRegs {
    uint4 rres[MT][NTL][2], racc[ACC ? MT : 1][ACC ? NTL : 1][2];
  };
  auto issue_epi = [&](int t, EpiRegs& er_) __attribute__((always_inline)) {
    auto& rres = er_.rres;
    auto& racc = er_.racc;
    const int b = t / ntm, mt = t - b * ntm;
    const bool hr = p.res != nullptr;
    const int Lrows = UPS ? p.Lout : p.Lq;
    const Rsrc rr = make_rsrc(hr ? reinterpret_cast<const bf16_t*>(p.res) + (size_t)b * p.res_bs : nullptr,
                              hr ? (unsigned)((size_t)Lrows * p.res_ld * 2) : 0u);
    const Rsrc ra = make_rsrc(ACC ? reinterpret_cast<const bf16_t*>(p.accb) + (size_t)b * p.acc_bs : nullptr,
                              ACC ? (unsigned)((size_t)p.Lq * p.acc_ld * 2) : 0u);
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) {
      const int q = mt * BM + wm * FW + mi * 32 + l32;
#pragma unroll
      for (int ni = 0; ni < NTL; ++ni) {
        const int co0 = (wn * NTL + ni) * 32 + hi * 16;
        // (UPS: output frame q u + phase - opad, channel co0 mod Cout; frames before 0 wrap past the range)
        const int ph = UPS ? co0 / p.Cout : 0;
        const int orow = UPS ? q * p.up + ph - p.opad : q, oc = UPS ? co0 - ph * p.Cout : co0;
        const unsigned er = (unsigned)(orow * p.res_ld + oc) * 2u;
        rres[mi][ni][0] = bload16(rr, er);
        rres[mi][ni][1] = bload16(rr, er + 16u);
        if constexpr (ACC) {
          const unsigned ea = (unsigned)(q * p.acc_ld + co0) * 2u;
          racc[mi][ni][0] = bload16(ra, ea);
          racc[mi][ni][1] = bload16(ra, ea + 16u);
        }
      }
    }
  };

  // per-lane statistics of the stored outputs: lane (frame l32, half hi) owns channels
  // (wn*NTL + ni)*32 + 16*hi + r of every frame it stores
  float st_s[ACC ? 1 : NTL][16], st_q[ACC ? 1 : NTL][16];
  if constexpr (!ACC) {
#pragma unroll
    for (int ni = 0; ni < NTL; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) st_s[ni][r] = st_q[ni][r] = 0.f;
  }
  auto flush = [&](int b) __attribute__((always_inline)) {
    if constexpr (!ACC) {
#pragma unroll
      for (int ni = 0; ni < NTL; ++ni)
      {
        float a, q;
        stat_bfly16(st_s[ni], st_q[ni], l32, a, q);
        const int ch = (wn * NTL + ni) * 32 + hi * 16 + l32;
        if (l32 < 16) {
          double* d = stats_slot(p, blockIdx.x) + ((size_t)b * p.stats_ld + (UPS ? ch % p.Cout : ch)) * ST_W;
          fx_add(d, a);
          fx_add(d + 2, q);
        }
      }
    }
  };

  // Prologue per element (AdaIN -> Snake), with sin^2(u) = (1 - cos 2u) / 2:
  //   x = v*a + (beta - mean*a)            (hifigan.py:14-24)
  //   y = x + sin^2(alpha x) / alpha        (hifigan.py:68)
  //     = fma(v, a, m2) - ia2 * cos(2 alpha x),   m2 = beta - mean*a + ia2,  ia2 = 1 / (2 alpha)
  // and the cosine argument (in revolutions, v_cos_f32) = fma(v, a*alpha/pi, (beta - mean*a)*alpha/pi).
  auto transform = [&](int t, const uint4 (&pre)[MAXU]) __attribute__((always_inline)) {
    const int mt = t % ntm;
    const int gr0 = mt * BM - G::PAD;
    float m2[8], a[8], ar[8], mr[8], nia[8];
    ld8_lds(coef + 8 * g8, m2);
    ld8_lds(coef + C + 8 * g8, a);
    ld8_lds(coef + 2 * C + 8 * g8, ar);
    ld8_lds(coef + 3 * C + 8 * g8, mr);
    ld8_lds(coef + 4 * C + 8 * g8, nia);
#pragma unroll
    for (int k = 0; k < MAXU; ++k) {
      const int u = tid + k * NT;
      if ((k + 1) * NT <= UNITS || u < UNITS) {
        const int r = u / G8;
        float v[8];
        bf8_to_f32(pre[k], v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x2 = __builtin_fmaf(v[j], a[j], m2[j]);
          const float c = __builtin_amdgcn_cosf(__builtin_fmaf(v[j], ar[j], mr[j]));
          v[j] = __builtin_fmaf(c, nia[j], x2);
        }
        uint4 o = (p.dbg & 1) ? pre[k] : f32_to_bf8(v);
        if ((unsigned)(gr0 + r) >= (unsigned)p.Lin) o = make_uint4(0, 0, 0, 0);  // zero padding is post-prologue
        *reinterpret_cast<uint4*>(Xs + r * XP + 8 * g8) = o;
      }
    }
  };

  // diagnostics (STTS_OPT_DEBUG bit 64 + a debug buffer): per-wave s_memtime sums of the step's phases
  // 0 coefficients / residual issue, 1 barrier A, 2 transform (with its window wait), 3 window issue,
  // 4 barrier B, 5 MFMA, 6 epilogue; 7 = total, [15] = blocks
  const bool stamp = (p.dbg & 64) && p.stamps;
  unsigned long long sacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const unsigned long long t_start = stamp ? __builtin_amdgcn_s_memtime() : 0;
  unsigned long long t_mark = t_start;
  auto mark = [&](int k) __attribute__((always_inline)) {
    if (stamp) {
      const unsigned long long tt = __builtin_amdgcn_s_memtime();
      sacc[k] += tt - t_mark;
      t_mark = tt;
    }
  };

  int cur_b = -1;
  auto step = [&](int t, uint4 (&pre)[MAXU], EpiRegs& er_, EpiRegs& er_next) __attribute__((always_inline)) {
    const int b = t / ntm, mt = t - b * ntm;
    auto& rres = er_.rres;
    auto& racc = er_.racc;
    if (b != cur_b) {
      if (cur_b >= 0 && p.stats) flush(cur_b);
      // every wave is past its previous transform (barrier B of the previous step): coef is free
      for (int ci = tid; ci < C; ci += NT) {
        if (p.pro.mode == 0) {  // plain conv (the training step's convs, normalised by their own kernel):
          coef[ci] = 0.f;       // x2 = v, cosine term times 0 -> the transform is exactly the identity
          coef[C + ci] = 1.f;
          coef[2 * C + ci] = coef[3 * C + ci] = coef[4 * C + ci] = 0.f;
          continue;
        }
        float mm = 0.f, aa = 1.f, be = 0.f;  // UPS: Snake alone
        if (!UPS) adain_coeffs(p.pro, b, ci, mm, aa, be);
        const float al = p.pro.alpha[ci];
        const float m1 = be - mm * aa, ia2 = 0.5f / al, alr = al * 0.31830988618379067f;  // alpha / pi
        coef[ci] = m1 + ia2;
        coef[C + ci] = aa;
        coef[2 * C + ci] = aa * alr;
        coef[3 * C + ci] = m1 * alr;
        coef[4 * C + ci] = -ia2;
      }
      cur_b = b;
    }
    if constexpr (RPF) {
      if (t + 1 < tend) issue_epi(t + 1, er_next);
    } else {
      issue_epi(t, er_);
    }
    mark(0);
    __syncthreads();  // (A) coef / weights visible; every wave done reading Xs of the previous tile
    mark(1);
    transform(t, pre);
    mark(2);
    if (t + PF < tend) issue(t + PF, pre);
    mark(3);
    __syncthreads();  // (B) window complete
    mark(4);

    f32x16 acc[MT][NTL];
#pragma unroll
    for (int mi = 0; mi < MT; ++mi)
#pragma unroll
      for (int ni = 0; ni < NTL; ++ni)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;
    const bf16_t* xw = Xs + (size_t)(wm * FW + l32) * XP + hi * 8;
    const bf16_t* ww = Ws + (size_t)(wn * NTL * 32 + l32) * WP + hi * 8;
    // the (tap, chunk, k-half) steps fully unrolled with double-buffered fragments: the reads of
    // step s+1 are issued before step s's MFMAs, so their LDS latency hides behind them (a read /
    // wait / MFMA sequence per step left the loop latency-bound at C = 64, k7 / k11)
    constexpr int S = K * NCH * 2;
    auto ldfr = [&](int st, bf16x8 (&wa)[NTL], bf16x8 (&xb)[MT]) __attribute__((always_inline)) {
      const int tap = st / (NCH * 2), c = (st / 2) % NCH, kk = st & 1;
      const bf16_t* xt = xw + tap * DIL * XP;
      const bf16_t* wt = ww + tap * C * WP;
#pragma unroll
      for (int ni = 0; ni < NTL; ++ni)
        wa[ni] = *reinterpret_cast<const bf16x8*>(wt + (c * K * C + ni * 32) * WP + kk * 16);
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
        xb[mi] = *reinterpret_cast<const bf16x8*>(xt + mi * 32 * XP + c * 32 + kk * 16);
    };
    if (!(p.dbg & 2)) {
      bf16x8 wa[2][NTL], xb[2][MT];
      ldfr(0, wa[0], xb[0]);
#pragma unroll
      for (int st = 0; st < S; ++st) {
        const int cb = st & 1;
        if (st + 1 < S) ldfr(st + 1, wa[cb ^ 1], xb[cb ^ 1]);
#pragma unroll
        for (int mi = 0; mi < MT; ++mi)
#pragma unroll
          for (int ni = 0; ni < NTL; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[cb][ni], xb[cb][mi], acc[mi][ni], 0, 0, 0);
      }
    }

    mark(5);
    // ---- epilogue: lane = frame l32 of block mi, channels (wn*NTL + ni)*32 + 16*hi + r
    if (p.dbg & 4) return;
    bf16_t* yb = reinterpret_cast<bf16_t*>(p.y) + (size_t)b * p.y_bs;
    const bool store = p.y != nullptr;
    const bool hr = p.res != nullptr;
    const float osc = p.out_scale;
    const float adiv = (ACC && p.acc_div != 0.f) ? 1.0f / p.acc_div : 1.0f;
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) {
      const int q = mt * BM + wm * FW + mi * 32 + l32;
#pragma unroll
      for (int ni = 0; ni < NTL; ++ni) {
        const int co0 = (wn * NTL + ni) * 32 + hi * 16;
        const int ph = UPS ? co0 / p.Cout : 0;
        const int orow = UPS ? q * p.up + ph - p.opad : q, oc = UPS ? co0 - ph * p.Cout : co0;
        const bool valid = q < p.Lq && (!UPS || (unsigned)orow < (unsigned)p.Lout);
        float v[16], bb[16];
        ld8_lds(bias_s + co0, *reinterpret_cast<float(*)[8]>(&bb[0]));
        ld8_lds(bias_s + co0 + 8, *reinterpret_cast<float(*)[8]>(&bb[8]));
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = acc[mi][ni][r] + bb[r];
        if (hr) {
          float r0[8], r1[8];
          bf8_to_f32(rres[mi][ni][0], r0);
          bf8_to_f32(rres[mi][ni][1], r1);
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            v[r] += r0[r];
            v[8 + r] += r1[r];
          }
          if (osc != 1.0f) {
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] *= osc;
          }
        }
        if (valid) {  // y == null: statistics-only pass (resfused.hip needs conv1's statistics)
          if constexpr (ACC) {
            float r0[8], r1[8];
            bf8_to_f32(racc[mi][ni][0], r0);
            bf8_to_f32(racc[mi][ni][1], r1);
#pragma unroll
            for (int r = 0; r < 8; ++r) {
              v[r] = (r0[r] + v[r]) * adiv;
              v[8 + r] = (r1[r] + v[8 + r]) * adiv;
            }
          }
          if (store) {
            bf16_t* dst = yb + (size_t)orow * p.y_ld + oc;
            *reinterpret_cast<uint4*>(dst) = f32_to_bf8(&v[0]);
            *reinterpret_cast<uint4*>(dst + 8) = f32_to_bf8(&v[8]);
          }
          if constexpr (!ACC) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              st_s[ni][r] += v[r];
              st_q[ni][r] = __builtin_fmaf(v[r], v[r], st_q[ni][r]);
            }
          }
        }
      }
    }
    mark(6);
  };

  // ---- IL: tile t's MFMAs with the epilogue of tile t - 1 (live = t - 1 is a tile of this range) in one block
  const float osc_il = p.res ? p.out_scale : 1.0f;  // (the residual of a launch without one reads as 0)
  const float adiv_il = (ACC && p.acc_div != 0.f) ? 1.0f / p.acc_div : 1.0f;
  // (a statistics-only launch, y == null, stores through a zero-range descriptor: every store dropped)
  const size_t ybs_il = p.y ? (size_t)p.y_bs * 2 : 0;
  const unsigned yrange_il = p.y ? (unsigned)((size_t)p.Lq * p.y_ld * 2) : 0u;
  // one epilogue unit: 8 channels (half hh of block (mi, ni)) of the lane's frame; NU units per tile
  constexpr int NU = MT * NTL * 2;
  auto epi_unit = [&](int t, bool live, const f32x16 (&accp)[MT][NTL], const EpiRegs& er_, int u)
                      __attribute__((always_inline)) {
    const int mi = u / (2 * NTL), ni = (u / 2) % NTL, hh = u & 1;
    const int b = t / ntm, mt = t - b * ntm;
    const Rsrc ry = make_rsrc(reinterpret_cast<const char*>(p.y) + (size_t)b * ybs_il, yrange_il);
    const int q = mt * BM + wm * FW + mi * 32 + l32;
    // (masks, not branches: the region must stay one basic block)
    const unsigned keep = (live && q < p.Lq) ? 0xffffffffu : 0u;
    const int co0 = (wn * NTL + ni) * 32 + hi * 16 + 8 * hh;
    float v[8], bb[8], r0[8];
    ld8_lds(bias_s + co0, bb);
    bf8_to_f32(er_.rres[mi][ni][hh], r0);
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = (accp[mi][ni][8 * hh + r] + bb[r] + r0[r]) * osc_il;
    if constexpr (ACC) {
      bf8_to_f32(er_.racc[mi][ni][hh], r0);
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = (r0[r] + v[r]) * adiv_il;
    }
    bstore16(ry, ((unsigned)(q * p.y_ld + co0) * 2u) | (~keep & OOB), f32_to_bf8(v));
    if constexpr (!ACC) {
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const float x = __uint_as_float(__float_as_uint(v[r]) & keep);
        st_s[ni][8 * hh + r] += x;
        st_q[ni][8 * hh + r] = __builtin_fmaf(x, x, st_q[ni][8 * hh + r]);
      }
    }
  };
  auto epi_il = [&](int t, bool live, const f32x16 (&accp)[MT][NTL], const EpiRegs& er_) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NU; ++u) epi_unit(t, live, accp, er_, u);
  };
  EpiRegs e_il;  // the residual rows of tile t - 1, loaded at the start of step t
  auto step_il = [&](int t, uint4 (&pre)[MAXU], f32x16 (&acc)[MT][NTL],
                     const f32x16 (&accp)[MT][NTL]) __attribute__((always_inline)) {
    const int b = t / ntm;
    if (b != cur_b) {  // tile t's coefficients (every wave is past its previous transform: barrier B)
      for (int ci = tid; ci < C; ci += NT) {
        if (p.pro.mode == 0) {
          coef[ci] = 0.f;
          coef[C + ci] = 1.f;
          coef[2 * C + ci] = coef[3 * C + ci] = coef[4 * C + ci] = 0.f;
          continue;
        }
        float mm = 0.f, aa = 1.f, be = 0.f;
        adain_coeffs(p.pro, b, ci, mm, aa, be);
        const float al = p.pro.alpha[ci];
        const float m1 = be - mm * aa, ia2 = 0.5f / al, alr = al * 0.31830988618379067f;
        coef[ci] = m1 + ia2;
        coef[C + ci] = aa;
        coef[2 * C + ci] = aa * alr;
        coef[3 * C + ci] = m1 * alr;
        coef[4 * C + ci] = -ia2;
      }
      cur_b = b;
    }
    issue_epi(t > tbeg ? t - 1 : t, e_il);
    __syncthreads();  // (A)
    transform(t, pre);
    if (t + PF < tend) issue(t + PF, pre);
    __syncthreads();  // (B)
#pragma unroll
    for (int mi = 0; mi < MT; ++mi)
#pragma unroll
      for (int ni = 0; ni < NTL; ++ni)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;
    const bf16_t* xw = Xs + (size_t)(wm * FW + l32) * XP + hi * 8;
    const bf16_t* ww = Ws + (size_t)(wn * NTL * 32 + l32) * WP + hi * 8;
    constexpr int S = K * NCH * 2;
    auto ldfr = [&](int st, bf16x8 (&wa)[NTL], bf16x8 (&xb)[MT]) __attribute__((always_inline)) {
      const int tap = st / (NCH * 2), c = (st / 2) % NCH, kk = st & 1;
      const bf16_t* xt = xw + tap * DIL * XP;
      const bf16_t* wt = ww + tap * C * WP;
#pragma unroll
      for (int ni = 0; ni < NTL; ++ni)
        wa[ni] = *reinterpret_cast<const bf16x8*>(wt + (c * K * C + ni * 32) * WP + kk * 16);
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
        xb[mi] = *reinterpret_cast<const bf16x8*>(xt + mi * 32 * XP + c * 32 + kk * 16);
    };
    bf16x8 wa[2][NTL], xb[2][MT];
    ldfr(0, wa[0], xb[0]);
#pragma unroll
    for (int st = 0; st < S; ++st) {
      const int cb = st & 1;
      if (st + 1 < S) ldfr(st + 1, wa[cb ^ 1], xb[cb ^ 1]);
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
#pragma unroll
        for (int ni = 0; ni < NTL; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[cb][ni], xb[cb][mi], acc[mi][ni], 0, 0, 0);
      // epilogue unit u of tile t - 1 after MFMA step (2 u + 1) S / (2 NU): its VALU work fills this step's gaps
#pragma unroll
      for (int u = 0; u < NU; ++u)
        if (st == ((2 * u + 1) * S) / (2 * NU)) epi_unit(t > tbeg ? t - 1 : t, t > tbeg, accp, e_il, u);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (t > tbeg && (t - 1) / ntm != b && p.stats) flush((t - 1) / ntm);  // tile t - 1 closed its utterance
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
  if constexpr (IL) {
    uint4 preA[MAXU], preB[MAXU];
    f32x16 accA[MT][NTL], accB[MT][NTL];
#pragma unroll
    for (int mi = 0; mi < MT; ++mi)
#pragma unroll
      for (int ni = 0; ni < NTL; ++ni)
#pragma unroll
        for (int r = 0; r < 16; ++r) accB[mi][ni][r] = 0.f;
    issue(tbeg, preA);
    if (tbeg + 1 < tend) issue(tbeg + 1, preB);
    for (int t = tbeg; t < tend; t += 2) {
      step_il(t, preA, accA, accB);
      if (t + 1 < tend) step_il(t + 1, preB, accB, accA);
    }
    // the range's last tile: its epilogue alone
    issue_epi(tend - 1, e_il);
    if ((tend - 1 - tbeg) % 2 == 0) epi_il(tend - 1, true, accA, e_il);
    else epi_il(tend - 1, true, accB, e_il);
    if (p.stats) flush(cur_b);
    cur_b = -1;
    if constexpr (!SEG) break;  // (one range)
    continue;
  }
  uint4 preA[MAXU], preB[MAXU];
  EpiRegs eA, eB;
  if constexpr (RPF) issue_epi(tbeg, eA);
  issue(tbeg, preA);
  if (tbeg + 1 < tend) issue(tbeg + 1, preB);
  if constexpr (PF == 3) {
    uint4 preC[MAXU];
    if (tbeg + 2 < tend) issue(tbeg + 2, preC);
    for (int t = tbeg; t < tend; t += 3) {
      step(t, preA, eA, eB);
      if (t + 1 < tend) step(t + 1, preB, eB, eA);
      if (t + 2 < tend) step(t + 2, preC, eA, eB);
    }
  } else {
    for (int t = tbeg; t < tend; t += 2) {
      step(t, preA, eA, eB);
      if (t + 1 < tend) step(t + 1, preB, eB, eA);
    }
  }
  if (p.stats) flush(cur_b);
  cur_b = -1;  // (the range's statistics are out: the next range re-stages its coefficients, flushes nothing twice)
  if constexpr (!SEG) break;  // (one range)
  }  // tile ranges
  if (stamp) {
    sacc[7] = __builtin_amdgcn_s_memtime() - t_start;
    if (lane == 0)
      for (int k = 0; k < 8; ++k) atomicAdd(p.stamps + k, sacc[k]);
    if (tid == 0) atomicAdd(p.stamps + 15, 1ull);
  }
}

int g_num_cu_rc = 0;

// WV / WN: block shape override (0 = the default: 4 x 1 waves at C = 32, 8 x 2 at C = 64)
template <int C, int K, int DIL, bool ACC, bool RPF = false, int PF = 2, bool UPS = false, int WV = 0, int WN = 0,
          bool IL = false, int MINB = 0>
int launch_rc(const ConvParams& p, hipStream_t stream) {
  constexpr int WAVES = WV ? WV : C == 32 ? 4 : 8;
  constexpr int WAVES_N = WN ? WN : C == 32 ? 1 : 2;
  using G = RC<C, K, DIL, WAVES, WAVES_N, UPS>;
  auto kern0 = k_resconv<C, K, DIL, WAVES, WAVES_N, ACC, RPF, PF, UPS, IL, false, MINB>;
  auto kern1 = k_resconv<C, K, DIL, WAVES, WAVES_N, ACC, RPF, PF, UPS, IL, true, MINB>;
  static bool attr = false;
  if (!attr) {
    ST_CHECK_HIP(hipFuncSetAttribute((const void*)kern0, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
    ST_CHECK_HIP(hipFuncSetAttribute((const void*)kern1, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
    attr = true;
  }
  if (!g_num_cu_rc) {
    int dev = 0;
    ST_CHECK_HIP(hipGetDevice(&dev));
    ST_CHECK_HIP(hipDeviceGetAttribute(&g_num_cu_rc, hipDeviceAttributeMultiprocessorCount, dev));
  }
  int per_cu = occupancy_cached((const void*)kern0, G::NT, G::LDS);
  if (per_cu < 1) per_cu = 1;
  const long long tiles = (long long)((p.Lq + G::BM - 1) / G::BM) * p.B;
  ConvParams q = p;
  const int seg = st_seg_choice(p, 1, g_num_cu_rc * per_cu);
  long long grid = (long long)g_num_cu_rc * per_cu;
  if (grid > (seg ? (long long)p.B * seg : tiles)) grid = seg ? (long long)p.B * seg : tiles;
  if (g_opt_grid_cap > 0 && grid > g_opt_grid_cap) grid = g_opt_grid_cap;
  const bool segk = seg > 0 && grid < (long long)p.B * seg;  // (one segment per workgroup = the plain even split)
  q.seg = segk ? seg : 0;
  hipLaunchKernelGGL(segk ? kern1 : kern0, dim3((unsigned)grid), dim3(G::NT), G::LDS, stream, q);
  return (int)hipGetLastError();
}

// ---- Ping-pong variant for C = 64 (STTS_OPT_RCPP): the block's 8 waves form two groups of 4 (one
// wave of each group per SIMD) that work on alternate 128-frame tiles half a step apart.  In every slot
// one group runs its tile's MFMAs while the other runs the previous tile's epilogue and the next tile's
// window transform, so the VALU / memory phases, which the lock-step kernel above runs after its MFMAs
// (profiles/r03_resconv_stamps.txt), overlap the partner's MFMAs (MI355X_MICROARCH.md "Two waves per
// SIMD").  Slot s of group g: compute tile j = (s - g) / 2 when s - g is even, else epilogue of tile
// (s - 1 - g) / 2 and transform of the next; one block barrier closes each slot, so a group's window is
// written in one slot and read in the next.  The weights are kept as packed (64-B rows, XOR-swizzled
// 16-B units), which makes room for the two windows next to the K = 11 weights.
template <int K, int DIL>
struct PP {
  static constexpr int C = 64, NT = 512, GT = 256, FW = 64, MT = 2, NCH = 2;
  static constexpr int BM = 128;                       // frames per group tile (2 wave rows x 64)
  static constexpr int PAD = DIL * (K - 1) / 2;
  static constexpr int R = BM + DIL * (K - 1);         // window rows
  static constexpr int XP = C + 8;                     // window row pitch (bf16)
  static constexpr int G8 = C / 8;
  static constexpr int UNITS = R * G8;
  static constexpr int MAXU = (UNITS + GT - 1) / GT;
  static constexpr int OFF_BIAS = 2 * 5 * C * 4;       // after coef [2 groups][5][C] f32
  static constexpr int OFF_W = OFF_BIAS + C * 4;
  static constexpr int W_B = NCH * K * C * 32 * 2;     // [chunk][tap][n][32] as packed
  static constexpr int OFF_X = OFF_W + W_B;
  static constexpr int X_B = R * XP * 2;               // one group's window
  static constexpr int LDS = OFF_X + 2 * X_B;
  static_assert(GT % G8 == 0 && OFF_W % 16 == 0 && OFF_X % 16 == 0 && X_B % 16 == 0, "carve");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

template <int K, int DIL, bool ACC>
__global__ void __launch_bounds__(512, 1) k_resconv_pp(const ConvParams p) {
  using G = PP<K, DIL>;
  constexpr int C = G::C, GT = G::GT, BM = G::BM, MT = G::MT, NCH = G::NCH, XP = G::XP, FW = G::FW;
  constexpr int G8 = G::G8, UNITS = G::UNITS, MAXU = G::MAXU;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, l32 = lane & 31, hi = lane >> 5;
  const int grp = wid >> 2, gw = wid & 3, gtid = tid & (GT - 1);
  const int wn = gw & 1, wm = gw >> 1;
  float* coef = reinterpret_cast<float*>(smem) + grp * 5 * C;  // this group's [5][C]
  float* bias_s = reinterpret_cast<float*>(smem + G::OFF_BIAS);
  bf16_t* Ws = reinterpret_cast<bf16_t*>(smem + G::OFF_W);
  bf16_t* Xs = reinterpret_cast<bf16_t*>(smem + G::OFF_X + grp * G::X_B);

  const int ntm = (p.Lq + BM - 1) / BM;
  const long long total = (long long)ntm * p.B;
  // tile ranges (kernels.h tile_range); the lambdas below read the current range by reference
  const int nv = tile_nv(p, p.B);
  if ((int)blockIdx.x >= nv) return;  // uniform over the block
  int tbeg = 0, tend = 0, n0 = 0, n1 = 0, ng = 0;  // ng: this group's tiles, tbeg + grp + 2 j
  auto utt = [&](int j) { return (tbeg + grp + 2 * j) / ntm; };

  {  // weights (copied as packed) and bias, once per block
    const Rsrc rw = make_rsrc(p.w, (unsigned)G::W_B);
    for (int u = tid; u < G::W_B / 16; u += G::NT) *reinterpret_cast<uint4*>(Ws + 8 * u) = bload16(rw, 16u * u);
    for (int i = tid; i < C; i += G::NT) bias_s[i] = p.bias ? p.bias[i] : 0.f;
  }
  auto set_coef = [&](int b) __attribute__((always_inline)) {
    for (int ci = gtid; ci < C; ci += GT) {
      if (p.pro.mode == 0) {
        coef[ci] = 0.f;
        coef[C + ci] = 1.f;
        coef[2 * C + ci] = coef[3 * C + ci] = coef[4 * C + ci] = 0.f;
        continue;
      }
      float mm, aa, be;
      adain_coeffs(p.pro, b, ci, mm, aa, be);
      const float al = p.pro.alpha[ci];
      const float m1 = be - mm * aa, ia2 = 0.5f / al, alr = al * 0.31830988618379067f;
      coef[ci] = m1 + ia2;
      coef[C + ci] = aa;
      coef[2 * C + ci] = aa * alr;
      coef[3 * C + ci] = m1 * alr;
      coef[4 * C + ci] = -ia2;
    }
  };

  const int g8 = gtid % G8;
  uint4 pre[MAXU];
  auto issue = [&](int j) __attribute__((always_inline)) {
    const int t = tbeg + grp + 2 * j;
    const int b = t / ntm, mt = t - b * ntm;
    const Rsrc rx = make_rsrc(reinterpret_cast<const bf16_t*>(p.x) + (size_t)b * p.x_bs,
                              (unsigned)((size_t)p.Lin * p.x_ld * 2));
    const int gr0 = mt * BM - G::PAD;
#pragma unroll
    for (int k = 0; k < MAXU; ++k) {
      const int u = gtid + k * GT;
      const int e = (gr0 + u / G8) * p.x_ld + 8 * g8;
      const bool in = (k + 1) * GT <= UNITS || u < UNITS;
      pre[k] = bload16(rx, in && e >= 0 ? (unsigned)e * 2u : OOB);
    }
  };
  auto transform = [&](int j) __attribute__((always_inline)) {
    const int t = tbeg + grp + 2 * j;
    const int mt = t % ntm;
    const int gr0 = mt * BM - G::PAD;
    float m2[8], a[8], ar[8], mr[8], nia[8];
    ld8_lds(coef + 8 * g8, m2);
    ld8_lds(coef + C + 8 * g8, a);
    ld8_lds(coef + 2 * C + 8 * g8, ar);
    ld8_lds(coef + 3 * C + 8 * g8, mr);
    ld8_lds(coef + 4 * C + 8 * g8, nia);
#pragma unroll
    for (int k = 0; k < MAXU; ++k) {
      const int u = gtid + k * GT;
      if ((k + 1) * GT <= UNITS || u < UNITS) {
        const int r = u / G8;
        float v[8];
        bf8_to_f32(pre[k], v);
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          const float x2 = __builtin_fmaf(v[jj], a[jj], m2[jj]);
          const float c = __builtin_amdgcn_cosf(__builtin_fmaf(v[jj], ar[jj], mr[jj]));
          v[jj] = __builtin_fmaf(c, nia[jj], x2);
        }
        uint4 o = f32_to_bf8(v);
        if ((unsigned)(gr0 + r) >= (unsigned)p.Lin) o = make_uint4(0, 0, 0, 0);
        *reinterpret_cast<uint4*>(Xs + r * XP + 8 * g8) = o;
      }
    }
  };

  // residual / running-sum rows of the tile being computed (read by its epilogue one slot later)
  uint4 rres[MT][2], racc[ACC ? MT : 1][2];
  auto issue_epi = [&](int j) __attribute__((always_inline)) {
    const int t = tbeg + grp + 2 * j;
    const int b = t / ntm, mt = t - b * ntm;
    const bool hr = p.res != nullptr;
    const Rsrc rr = make_rsrc(hr ? reinterpret_cast<const bf16_t*>(p.res) + (size_t)b * p.res_bs : nullptr,
                              hr ? (unsigned)((size_t)p.Lq * p.res_ld * 2) : 0u);
    const Rsrc ra = make_rsrc(ACC ? reinterpret_cast<const bf16_t*>(p.accb) + (size_t)b * p.acc_bs : nullptr,
                              ACC ? (unsigned)((size_t)p.Lq * p.acc_ld * 2) : 0u);
    const int co0 = wn * 32 + hi * 16;
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) {
      const int q = mt * BM + wm * FW + mi * 32 + l32;
      const unsigned er = (unsigned)(q * p.res_ld + co0) * 2u;
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
  int stat_b = -1;
  auto flush = [&](int b) __attribute__((always_inline)) {
    if constexpr (!ACC) {
      float a, q;
      stat_bfly16(st_s, st_q, l32, a, q);
      if (l32 < 16) {
        double* d = stats_slot(p, blockIdx.x) + ((size_t)b * p.stats_ld + wn * 32 + hi * 16 + l32) * ST_W;
        fx_add(d, a);
        fx_add(d + 2, q);
      }
    }
  };

  f32x16 acc[MT];
  // weight fragment: packed row n = wn * 32 + l32, 16-B unit g stored at g ^ ((n >> 2) & 3)
  const int swz = (l32 >> 2) & 3;
  const bf16_t* ww = Ws + (size_t)(wn * 32 + l32) * 32;
  const int wo0 = 8 * (hi ^ swz), wo1 = 8 * ((2 | hi) ^ swz);
  const bf16_t* xw = Xs + (size_t)(wm * FW + l32) * XP + hi * 8;
  constexpr int S = K * NCH * 2;
  auto ldfr = [&](int st, bf16x8& wa, bf16x8 (&xb)[MT]) __attribute__((always_inline)) {
    const int tap = st / (NCH * 2), c = (st / 2) % NCH, kk = st & 1;
    wa = *reinterpret_cast<const bf16x8*>(ww + (size_t)((c * K + tap) * C) * 32 + (kk ? wo1 : wo0));
#pragma unroll
    for (int mi = 0; mi < MT; ++mi)
      xb[mi] = *reinterpret_cast<const bf16x8*>(xw + (tap * DIL + mi * 32) * XP + c * 32 + kk * 16);
  };
  auto compute = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int mi = 0; mi < MT; ++mi)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][r] = 0.f;
    // fragments two steps ahead (one wave per SIMD computes: no partner wave covers the LDS latency)
    // (sched_group_barrier pins the order: hipcc otherwise sinks each read to one MFMA before its use)
    bf16x8 wa[3], xb[3][MT];
    ldfr(0, wa[0], xb[0]);
    ldfr(1, wa[1], xb[1]);
    __builtin_amdgcn_sched_group_barrier(0x100, 2 * (1 + MT), 0);
#pragma unroll
    for (int st = 0; st < S; ++st) {
      const int cb = st % 3;
      if (st + 2 < S) {
        ldfr(st + 2, wa[(st + 2) % 3], xb[(st + 2) % 3]);
        __builtin_amdgcn_sched_group_barrier(0x100, 1 + MT, 0);
      }
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
        acc[mi] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[cb], xb[cb][mi], acc[mi], 0, 0, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, MT, 0);
    }
  };
  auto epilogue = [&](int j) __attribute__((always_inline)) {
    const int t = tbeg + grp + 2 * j;
    const int b = t / ntm, mt = t - b * ntm;
    if (b != stat_b) {
      if (stat_b >= 0 && p.stats) flush(stat_b);
      stat_b = b;
    }
    bf16_t* yb = reinterpret_cast<bf16_t*>(p.y) + (size_t)b * p.y_bs;
    const bool store = p.y != nullptr;
    const bool hr = p.res != nullptr;
    const float osc = p.out_scale;
    const float adiv = (ACC && p.acc_div != 0.f) ? 1.0f / p.acc_div : 1.0f;
    const int co0 = wn * 32 + hi * 16;
    float bb[16];
    ld8_lds(bias_s + co0, *reinterpret_cast<float(*)[8]>(&bb[0]));
    ld8_lds(bias_s + co0 + 8, *reinterpret_cast<float(*)[8]>(&bb[8]));
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) {
      const int q = mt * BM + wm * FW + mi * 32 + l32;
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = acc[mi][r] + bb[r];
      if (hr) {
        float r0[8], r1[8];
        bf8_to_f32(rres[mi][0], r0);
        bf8_to_f32(rres[mi][1], r1);
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          v[r] += r0[r];
          v[8 + r] += r1[r];
        }
        if (osc != 1.0f) {
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] *= osc;
        }
      }
      if (q < p.Lq) {
        if constexpr (ACC) {
          float r0[8], r1[8];
          bf8_to_f32(racc[mi][0], r0);
          bf8_to_f32(racc[mi][1], r1);
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            v[r] = (r0[r] + v[r]) * adiv;
            v[8 + r] = (r1[r] + v[8 + r]) * adiv;
          }
        }
        if (store) {
          bf16_t* dst = yb + (size_t)q * p.y_ld + co0;
          *reinterpret_cast<uint4*>(dst) = f32_to_bf8(&v[0]);
          *reinterpret_cast<uint4*>(dst + 8) = f32_to_bf8(&v[8]);
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
  };

  for (int vb = blockIdx.x; vb < nv; vb += gridDim.x) {
  {
    long long tb_, te_;
    tile_range(p, vb, nv, total, ntm, tb_, te_);
    tbeg = (int)tb_;
    tend = (int)te_;
  }
  if (tbeg >= tend) continue;  // uniform over the block
  n0 = (tend - tbeg + 1) / 2;
  n1 = (tend - tbeg) / 2;
  ng = grp ? n1 : n0;
  // prologue: coefficients of each group's first tile, its window loads; group 0 transforms tile 0
  int coef_b = -1;
  if (ng > 0) {
    coef_b = utt(0);
    set_coef(coef_b);
    issue(0);
  }
  __syncthreads();  // weights, bias, coefficients visible
  if (grp == 0 && ng > 0) {
    transform(0);
    if (1 < ng) issue(1);
  }
  __syncthreads();
  const int nslots = (2 * n0 > 2 * n1 + 1) ? 2 * n0 : 2 * n1 + 1;
  for (int s = 0; s < nslots; ++s) {
    if (((s - grp) & 1) == 0) {  // compute slot: tile j
      const int j = (s - grp) >> 1;
      if (j < ng) {
        issue_epi(j);
        if (j + 1 < ng && utt(j + 1) != coef_b) {  // the next transform (next slot) needs its utterance
          coef_b = utt(j + 1);
          set_coef(coef_b);
        }
        compute();
      }
    } else {  // epilogue of tile j, transform of tile j + 1, loads of tile j + 2
      const int j = (s - 1 - grp) >> 1;
      if (j >= 0 && j < ng) epilogue(j);
      if (j + 1 < ng) {
        transform(j + 1);
        if (j + 2 < ng) issue(j + 2);
      }
    }
    __syncthreads();
  }
  if (p.stats && stat_b >= 0) flush(stat_b);
  stat_b = -1;
  __syncthreads();  // (the next range re-stages coefficients and windows)
  }  // tile ranges
}

int g_num_cu_pp = 0;

template <int K, int DIL, bool ACC>
int launch_pp(const ConvParams& p, hipStream_t stream) {
  using G = PP<K, DIL>;
  auto kern = k_resconv_pp<K, DIL, ACC>;
  static bool attr = false;
  if (!attr) {
    ST_CHECK_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
    attr = true;
  }
  if (!g_num_cu_pp) {
    int dev = 0;
    ST_CHECK_HIP(hipGetDevice(&dev));
    ST_CHECK_HIP(hipDeviceGetAttribute(&g_num_cu_pp, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const long long tiles = (long long)((p.Lq + G::BM - 1) / G::BM) * p.B;
  ConvParams q = p;
  q.seg = st_seg_choice(p, 1, g_num_cu_pp);
  long long grid = g_num_cu_pp;
  if (grid > (q.seg ? (long long)p.B * q.seg : tiles)) grid = q.seg ? (long long)p.B * q.seg : tiles;
  if (g_opt_grid_cap > 0 && grid > g_opt_grid_cap) grid = g_opt_grid_cap;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(G::NT), G::LDS, stream, q);
  return (int)hipGetLastError();
}

template <int C, int K, int DIL>
int launch_rc_a(const ConvParams& p, hipStream_t s) {
  if constexpr (DIL == 1) {  // (the residual launches: conv2 of an iteration, dilation 1)
    if ((g_opt_exp & 4) && (p.res || p.accb))
      return p.accb ? launch_rc<C, K, 1, true, true>(p, s) : launch_rc<C, K, 1, false, true>(p, s);
  }
  // STTS_OPT_RCPP: the two-group ping-pong kernel at C = 64 (1: residual / running-sum launches with K >= 7,
  // where the in-process A/B measured it faster, profiles/r03_ab_resconv_pp.txt; 2: every launch)
  // (3: those launches on the lock-step kernel with the interleaved epilogue instead, IL below)
  if constexpr (C == 64) {
    if (g_opt_rcpp == 2 || (g_opt_rcpp == 1 && K >= 7 && (p.res || p.accb)))
      return p.accb ? launch_pp<K, DIL, true>(p, s) : launch_pp<K, DIL, false>(p, s);
    if (g_opt_rcpp == 3 && K >= 7 && (p.res || p.accb))
      return p.accb ? launch_rc<C, K, DIL, true, false, 2, false, 0, 0, true>(p, s)
                    : launch_rc<C, K, DIL, false, false, 2, false, 0, 0, true>(p, s);
  }
  // STTS_OPT_RCOCC: C = 32, K >= 7, no residual: registers held to three 4-wave blocks per CU (168 VGPRs, three waves
  // per SIMD; 5-6 % faster per launch, profiles/r06_ab_rc3b.txt; the k3 and residual launches measured 0-3 % slower)
  if constexpr (C == 32 && K >= 7) {
    if (g_opt_rcocc && !p.res && !p.accb) return launch_rc<C, K, DIL, false, false, 2, false, 0, 0, false, 3>(p, s);
  }
  // STTS_OPT_EXP bit 32768: the interleaved epilogue (IL)
  if (g_opt_exp & 32768)
    return p.accb ? launch_rc<C, K, DIL, true, false, 2, false, 0, 0, true>(p, s)
                  : launch_rc<C, K, DIL, false, false, 2, false, 0, 0, true>(p, s);
  // STTS_OPT_EXP bit 262144 / 524288: C = 64 on 4-wave blocks (two or more per CU, each running its own tile loop,
  // so one block's MFMAs overlap the other's memory / VALU phases): 4 x 2 waves of 64 frames x 32 channels (128-frame
  // tiles) / 4 x 1 waves of 64 frames x 64 channels (256-frame tiles); bit 1048576 limits it to K = 3
  if constexpr (C == 64) {
    if ((g_opt_exp & (262144 | 524288)) && (K == 3 || !(g_opt_exp & 1048576))) {
      if (g_opt_exp & 262144)
        return p.accb ? launch_rc<C, K, DIL, true, false, 2, false, 4, 2>(p, s)
                      : launch_rc<C, K, DIL, false, false, 2, false, 4, 2>(p, s);
      return p.accb ? launch_rc<C, K, DIL, true, false, 2, false, 4, 1>(p, s)
                    : launch_rc<C, K, DIL, false, false, 2, false, 4, 1>(p, s);
    }
  }
  // STTS_OPT_EXP bit 8 / 16: window prefetch three tiles deep at C = 64 / C = 32 (register budget allows it:
  // 231-249 VGPRs, occupancy unchanged)
  if ((C == 64 && (g_opt_exp & 8)) || (C == 32 && (g_opt_exp & 16)))
    return p.accb ? launch_rc<C, K, DIL, true, false, 3>(p, s) : launch_rc<C, K, DIL, false, false, 3>(p, s);
  return p.accb ? launch_rc<C, K, DIL, true>(p, s) : launch_rc<C, K, DIL, false>(p, s);
}

template <int C, int K>
int launch_rc_d(const ConvParams& p, hipStream_t s) {
  switch (p.dil) {
    case 1: return launch_rc_a<C, K, 1>(p, s);
    case 3: return launch_rc_a<C, K, 3>(p, s);
    case 5: return launch_rc_a<C, K, 5>(p, s);
    default: return ST_EINVAL;
  }
}

template <int C>
int launch_rc_k(const ConvParams& p, hipStream_t s) {
  switch (p.KS) {
    case 3: return launch_rc_d<C, 3>(p, s);
    case 7: return launch_rc_d<C, 7>(p, s);
    case 11: return launch_rc_d<C, 11>(p, s);
    default: return ST_EINVAL;
  }
}

}  // namespace

int g_opt_plainrc = 1;
int g_opt_rcpp = 3;
int g_opt_rcocc = 1;

bool st_resconv_eligible(const ConvParams& p, int dtype) {
  if (dtype != ST_BF16) return false;
  const int C = p.Cout;
  if (!(C == 32 || C == 64) || p.Cin != C || p.N != C || p.nchunks * 32 != C) return false;
  if (!(p.KS == 3 || p.KS == 7 || p.KS == 11) || !(p.dil == 1 || p.dil == 3 || p.dil == 5)) return false;
  if ((p.kw != 0 && p.kw != p.KS) || p.row_off != 0 || p.stride != 1 || p.up != 1 || p.opad != 0) return false;
  if (p.pad != p.dil * (p.KS - 1) / 2 || p.Lq != p.Lout || p.Lq != p.Lin) return false;
  if (p.y_row_off || p.y_f32 || p.epi_tanh || p.epi_lrelu || p.epi_gelu || p.reflect_front || p.zc_period || p.res_shift) return false;
  // AdaIN -> Snake (the decoder), or no prologue (the training step's convs, STTS_OPT_PLAINRC)
  const bool snake = p.pro.mode == (PRO_AFFINE | PRO_SNAKE) && p.pro.alpha && p.pro.stats && p.pro.gamma;
  if (!snake && !(p.pro.mode == 0 && g_opt_plainrc)) return false;
  if (p.accb && p.stats) return false;  // the running-sum launch keeps no statistics
  if (p.x_ld % 8 || p.y_ld % 8 || (p.res && p.res_ld % 8) || (p.accb && p.acc_ld % 8)) return false;
  return true;
}

int st_resconv(const ConvParams& p, hipStream_t stream) {
  if (p.Cout == 32) return launch_rc_k<32>(p, stream);
  if (p.Cout == 64) return launch_rc_k<64>(p, stream);
  return ST_EINVAL;
}

// HiFi-GAN ups[3] (64 -> 32 channels, x2) on this engine (STTS_OPT_UPS with ups[0] / ups[1] on bigconv2)
bool st_resconv_ups_eligible(const ConvParams& p, int dtype) {
  if (!g_opt_ups || dtype != ST_BF16 || p.up != 2 || !p.res || p.accb) return false;
  return p.Cin == 64 && p.N == 64 && p.Cout == 32 && p.nchunks == 2 && p.KS == 2 && (p.kw == 0 || p.kw == 2) &&
         p.dil == 1 && p.stride == 1 && p.pad == 1 && p.row_off == 0 && p.pro.mode == PRO_SNAKE && p.pro.alpha &&
         p.res_shift == 0 && p.y_row_off == 0 && !p.reflect_front && !p.epi_tanh && !p.epi_lrelu && !p.epi_gelu &&
         !p.y_f32 && p.zc_period == 0 && p.x_ld % 8 == 0 && p.y_ld % 8 == 0 && p.res_ld % 8 == 0;
}

int st_resconv_ups(const ConvParams& p, hipStream_t stream) {
  return launch_rc<64, 2, 1, false, false, 2, true>(p, stream);
}
