// Resblock conv engine for the wide generator stages (C = 128 / 256; MFMA-bound): the dilated
// Conv1d(C, C, K, dilation d, padding d(K-1)/2) of every AdaINResBlock1 iteration
// (Modules/hifigan.py:26-80, forward :65-74) with the AdaIN -> Snake prologue and the bias /
// residual / resblock-average / InstanceNorm-statistics epilogue fused.  bf16 storage,
// v_mfma_f32_32x32x16_bf16, fp32 accumulation.  st_conv1d routes eligible launches here.
//
// The layer's weights (C*C*K bf16 = 0.2-1.4 MB) do not fit LDS, so a tile of 256 frames x C
// output channels walks a sequence of STEPS, one per (input-channel group, tap):
//   * the weight slice of a step (CG*32 input channels x C outputs = 16 KB) is loaded two steps
//     ahead into registers (two named sets, the step loop unrolled by two) and stored into a
//     2-slot LDS ring one step ahead: one barrier per step;
//   * the input window of the next channel group is loaded K steps ahead (at the group's first
//     tap) and transformed (AdaIN -> Snake -> bf16) into the other half of a 2-slot window ring
//     at the group's last tap;
//   * the pipeline runs across tile boundaries, so the chip never drains between tiles.
#include "common.h"
#include "conv_common.h"
#include "kernels.h"

namespace {

// One block of 8 waves per CU (two per SIMD, 256 registers each).
template <int C> struct BigCfg;
// C = 256: 2 x 4 waves, each 128 frames x 64 channels; one 32-channel group per step;
// statistics reduced across lanes once per tile (the tile is 88 steps long at K = 11)
template <> struct BigCfg<256> {
  static constexpr int WAVES_M = 2, WAVES_N = 4, MT = 4, NTL = 2, CG = 1;
  static constexpr bool SREG = false;
};
// C = 128: 2 x 4 waves, each 128 frames x 32 channels; two 32-channel groups per step;
// statistics kept per lane in registers and reduced when the block leaves an utterance
template <> struct BigCfg<128> {
  static constexpr int WAVES_M = 2, WAVES_N = 4, MT = 4, NTL = 1, CG = 2;
  static constexpr bool SREG = true;
};

template <int C, int K, int DIL>
struct BG {
  using F = BigCfg<C>;
  static constexpr int NT = 512, BM = 256;
  static constexpr int MT = F::MT, NTL = F::NTL, CG = F::CG;
  static constexpr int NCH = C / 32, NG = NCH / CG, CW = CG * 32, NS = NG * K;
  static constexpr int PAD = DIL * (K - 1) / 2, R = BM + DIL * (K - 1), XP = CW + 8;
  static constexpr int G8 = CW / 8, XUNITS = R * G8, MAXU = (XUNITS + NT - 1) / NT;
  static constexpr int WSLICE = CG * C * 32;        // bf16 elements per step
  static constexpr int WPT = WSLICE * 2 / 16 / NT;  // 16-byte units per thread per step
  static constexpr int OFF_BIAS = 2 * 5 * C * 4;    // coef [2][5][C] f32 (utterance parity)
  // stats [WAVES_M][C][2] f32 (per-tile reduction path): one copy per frame half, so every LDS word has one
  // writer and the flush adds the copies in a fixed order (deterministic statistics, common.h ST_W)
  static constexpr int OFF_ST = OFF_BIAS + C * 4;
  static constexpr int OFF_W = OFF_ST + F::WAVES_M * 2 * C * 4;
  static constexpr int OFF_X = OFF_W + 4 * WSLICE * 2;  // 4-slot weight ring
  static constexpr int LDS = OFF_X + 2 * R * XP * 2;
  static_assert(F::WAVES_M * MT * 32 == BM && F::WAVES_N * NTL * 32 == C, "wave grid");
  static_assert(WPT * 16 * NT == WSLICE * 2, "weight slice split");
  static_assert(NT % G8 == 0 && K >= 3, "pipeline shape");
  static_assert(NS % 2 == 0, "super-steps of two sub-steps must not straddle tiles");
  static_assert(LDS <= 160 * 1024, "LDS budget");
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

// SEG: several tile ranges per workgroup (bigconv2.hip k_bigconv2: the plain instantiation runs one range)
template <int C, int K, int DIL, bool ACC, bool SEG = false>
__global__ void __launch_bounds__(512, 1) k_bigconv(const ConvParams p) {
  using G = BG<C, K, DIL>;
  using F = typename G::F;
  constexpr int NT = G::NT, BM = G::BM, MT = G::MT, NTL = G::NTL, CG = G::CG, NG = G::NG, NS = G::NS;
  constexpr int XP = G::XP, G8 = G::G8, XUNITS = G::XUNITS, MAXU = G::MAXU, WPT = G::WPT;
  constexpr bool SREG = F::SREG && !ACC;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* coef = reinterpret_cast<float*>(smem);  // [2][5][C]
  float* bias_s = reinterpret_cast<float*>(smem + G::OFF_BIAS);
  float* st_lds = reinterpret_cast<float*>(smem + G::OFF_ST);
  bf16_t* Ws = reinterpret_cast<bf16_t*>(smem + G::OFF_W);  // [2][CG][C][32] (swizzled 16-B units)
  bf16_t* Xs = reinterpret_cast<bf16_t*>(smem + G::OFF_X);  // [2][R][XP]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, l32 = lane & 31, hi = lane >> 5;
  const int wn = wid % F::WAVES_N, wm = wid / F::WAVES_N;
  const int ntm = (p.Lq + BM - 1) / BM;
  const long long total = (long long)ntm * p.B;
  // tile ranges (kernels.h tile_range: one per workgroup, or utterance-relative segments)
  const int nv = SEG ? tile_nv(p, p.B) : (int)gridDim.x;
  for (int vb = blockIdx.x; vb < nv; vb += gridDim.x) {
  long long tb_, te_;
  if constexpr (SEG) {
    tile_range(p, vb, nv, total, ntm, tb_, te_);
  } else {
    tb_ = total * vb / gridDim.x;
    te_ = total * (vb + 1) / gridDim.x;
  }
  const int tbeg = (int)tb_, tend = (int)te_;
  if (tbeg >= tend) continue;  // uniform over the block
  const int nsteps = (tend - tbeg) * NS;

  for (int i = tid; i < C; i += NT) bias_s[i] = p.bias ? p.bias[i] : 0.f;
  for (int i = tid; i < F::WAVES_M * 2 * C; i += NT) st_lds[i] = 0.f;

  // ---------------- weights: global step g -> (group, tap) slice, 16-byte units u = tid + k*NT
  const Rsrc rw = make_rsrc(p.w, (unsigned)((size_t)G::NCH * K * C * 32 * 2));
  auto issue_w = [&](int g, uint4 (&wr)[WPT]) __attribute__((always_inline)) {
    const int s = g % NS, gi = s / K, tap = s - gi * K;
#pragma unroll
    for (int k = 0; k < WPT; ++k) {
      const int u = tid + k * NT;
      const int cg = u / (C * 4), rem = u - cg * (C * 4);
      const unsigned off = (unsigned)((((size_t)(gi * CG + cg) * K + tap) * C * 32) * 2 + (size_t)rem * 16);
      wr[k] = bload16(rw, g < nsteps ? off : OOB);
    }
  };
  auto store_w = [&](int slot, const uint4 (&wr)[WPT]) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < WPT; ++k)
      *reinterpret_cast<uint4*>(Ws + (size_t)slot * G::WSLICE + (size_t)(tid + k * NT) * 8) = wr[k];
  };

  // ---------------- input windows: global group index -> (tile, group)
  const int g8 = tid % G8;
  uint4 xr[MAXU];
  auto issue_x = [&](int gg) __attribute__((always_inline)) {
    const int t = tbeg + gg / NG, gi = gg % NG;
    const int b = t / ntm, mt = t - b * ntm;
    const Rsrc rx = make_rsrc(reinterpret_cast<const bf16_t*>(p.x) + (size_t)b * p.x_bs,
                              t < tend ? (unsigned)((size_t)p.Lin * p.x_ld * 2) : 0u);
    const int gr0 = mt * BM - G::PAD;
#pragma unroll
    for (int k = 0; k < MAXU; ++k) {
      const int u = tid + k * NT;
      const int e = (gr0 + u / G8) * p.x_ld + gi * G::CW + 8 * g8;
      const bool in = (k + 1) * NT <= XUNITS || u < XUNITS;
      xr[k] = bload16(rx, in && e >= 0 ? (unsigned)e * 2u : OOB);
    }
  };
  auto set_coef = [&](int b) __attribute__((always_inline)) {
    float* cf = coef + (b & 1) * 5 * C;
    for (int ci = tid; ci < C; ci += NT) {
      float mm, aa, be;
      adain_coeffs(p.pro, b, ci, mm, aa, be);
      const float al = p.pro.alpha[ci];
      const float m1 = be - mm * aa, ia2 = 0.5f / al, alr = al * 0.31830988618379067f;
      cf[ci] = m1 + ia2;
      cf[C + ci] = aa;
      cf[2 * C + ci] = aa * alr;
      cf[3 * C + ci] = m1 * alr;
      cf[4 * C + ci] = -ia2;
    }
  };
  // AdaIN -> Snake with sin^2(u) = (1 - cos 2u)/2 (see resconv.hip), zero padding post-prologue
  auto transform_x = [&](int gg) __attribute__((always_inline)) {
    const int t = tbeg + gg / NG, gi = gg % NG;
    const int b = t / ntm, mt = t - b * ntm;
    const int gr0 = mt * BM - G::PAD;
    const float* cf = coef + (b & 1) * 5 * C + gi * G::CW + 8 * g8;
    bf16_t* X = Xs + (size_t)(gg & 1) * G::R * XP;
#pragma unroll
    for (int k = 0; k < MAXU; ++k) {
      const int u = tid + k * NT;
      if ((k + 1) * NT <= XUNITS || u < XUNITS) {
        const int r = u / G8;
        float v[8];
        bf8_to_f32(xr[k], v);
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // 4 channels at a time: 20 coefficient registers
          const float4 m2 = *reinterpret_cast<const float4*>(cf + 4 * h);
          const float4 a = *reinterpret_cast<const float4*>(cf + C + 4 * h);
          const float4 ar = *reinterpret_cast<const float4*>(cf + 2 * C + 4 * h);
          const float4 mr = *reinterpret_cast<const float4*>(cf + 3 * C + 4 * h);
          const float4 nia = *reinterpret_cast<const float4*>(cf + 4 * C + 4 * h);
          const float am[4] = {m2.x, m2.y, m2.z, m2.w}, aa[4] = {a.x, a.y, a.z, a.w};
          const float aar[4] = {ar.x, ar.y, ar.z, ar.w}, amr[4] = {mr.x, mr.y, mr.z, mr.w};
          const float ani[4] = {nia.x, nia.y, nia.z, nia.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float x = v[4 * h + j];
            const float x2 = __builtin_fmaf(x, aa[j], am[j]);
            const float c = __builtin_amdgcn_cosf(__builtin_fmaf(x, aar[j], amr[j]));
            v[4 * h + j] = __builtin_fmaf(c, ani[j], x2);
          }
        }
        uint4 o = (p.dbg & 1) ? xr[k] : f32_to_bf8(v);
        if ((unsigned)(gr0 + r) >= (unsigned)p.Lin) o = make_uint4(0, 0, 0, 0);
        *reinterpret_cast<uint4*>(X + r * XP + 8 * g8) = o;
        asm volatile("" ::: "memory");  // reload the coefficients per unit (register budget)
      }
    }
  };

  // ---------------- epilogue state
  constexpr int NRES = (F::SREG ? 1 : 0);  // residual / running-sum prefetch only on the C = 128 path
  uint4 rres[NRES ? MT : 1][NRES ? NTL : 1][2];
  uint4 racc[NRES && ACC ? MT : 1][NRES && ACC ? NTL : 1][2];
  auto issue_epi = [&](int t) __attribute__((always_inline)) {
    if constexpr (NRES) {
      const int b = t / ntm, mt = t - b * ntm;
      const bool hr = p.res != nullptr;
      const Rsrc rr = make_rsrc(hr ? reinterpret_cast<const bf16_t*>(p.res) + (size_t)b * p.res_bs : nullptr,
                                hr ? (unsigned)((size_t)p.Lq * p.res_ld * 2) : 0u);
      const Rsrc ra = make_rsrc(ACC ? reinterpret_cast<const bf16_t*>(p.accb) + (size_t)b * p.acc_bs : nullptr,
                                ACC ? (unsigned)((size_t)p.Lq * p.acc_ld * 2) : 0u);
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) {
        const int q = mt * BM + (wm * MT + mi) * 32 + l32;
#pragma unroll
        for (int ni = 0; ni < NTL; ++ni) {
          const int co0 = (wn * NTL + ni) * 32 + hi * 16;
          const unsigned er = (unsigned)(q * p.res_ld + co0) * 2u;
          rres[mi][ni][0] = bload16(rr, er);
          rres[mi][ni][1] = bload16(rr, er + 16u);
          if constexpr (ACC) {
            const unsigned ea = (unsigned)(q * p.acc_ld + co0) * 2u;
            racc[mi][ni][0] = bload16(ra, ea);
            racc[mi][ni][1] = bload16(ra, ea + 16u);
          }
        }
      }
    }
  };
  float st_s[SREG ? NTL : 1][16], st_q[SREG ? NTL : 1][16];
  if constexpr (SREG) {
#pragma unroll
    for (int ni = 0; ni < NTL; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) st_s[ni][r] = st_q[ni][r] = 0.f;
  }
  // SREG: lane-register statistics -> global, when the block leaves utterance b
  auto flush_reg = [&](int b) __attribute__((always_inline)) {
    if constexpr (SREG) {
#pragma unroll
      for (int ni = 0; ni < NTL; ++ni)
      {
        float a, q;
        stat_bfly16(st_s[ni], st_q[ni], l32, a, q);
        if (l32 < 16) {
          double* d = stats_slot(p, blockIdx.x) + ((size_t)b * p.stats_ld + (wn * NTL + ni) * 32 + hi * 16 + l32) * ST_W;
          fx_add(d, a);
          fx_add(d + 2, q);
        }
      }
    }
  };
  // per-tile path: LDS accumulators -> global (after a barrier), when the block leaves utterance b
  auto flush_lds = [&](int b) __attribute__((always_inline)) {
    for (int ci = tid; ci < C; ci += NT) {
      double* d = stats_slot(p, blockIdx.x) + ((size_t)b * p.stats_ld + ci) * ST_W;
      float a = 0.f, q = 0.f;
#pragma unroll
      for (int m = 0; m < F::WAVES_M; ++m) {
        a += st_lds[(m * C + ci) * 2];
        q += st_lds[(m * C + ci) * 2 + 1];
        st_lds[(m * C + ci) * 2] = st_lds[(m * C + ci) * 2 + 1] = 0.f;
      }
      fx_add(d, a);
      fx_add(d + 2, q);
    }
  };

  f32x16 acc[MT][NTL];
  auto epilogue = [&](int t) __attribute__((always_inline)) {
    if (p.dbg & 4) return;
    const int b = t / ntm, mt = t - b * ntm;
    bf16_t* yb = reinterpret_cast<bf16_t*>(p.y) + (size_t)b * p.y_bs;
    const bf16_t* rb = p.res ? reinterpret_cast<const bf16_t*>(p.res) + (size_t)b * p.res_bs : nullptr;
    const bf16_t* ab = ACC ? reinterpret_cast<const bf16_t*>(p.accb) + (size_t)b * p.acc_bs : nullptr;
    const float osc = p.out_scale;
    const float adiv = (ACC && p.acc_div != 0.f) ? 1.0f / p.acc_div : 1.0f;
    const bool want_stats = !ACC && p.stats != nullptr;
#pragma unroll
    for (int ni = 0; ni < NTL; ++ni) {
      const int co0 = (wn * NTL + ni) * 32 + hi * 16;
      float ts[16], tq[16];  // per-tile path: this lane's sums over its MT frames
      if constexpr (!SREG) {
#pragma unroll
        for (int r = 0; r < 16; ++r) ts[r] = tq[r] = 0.f;
      }
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) {
        const int q = mt * BM + (wm * MT + mi) * 32 + l32;
        const bool valid = q < p.Lq;
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = acc[mi][ni][r];
        if (valid) {
          if (rb) {
            float r0[8], r1[8];
            if constexpr (NRES) {
              bf8_to_f32(rres[mi][ni][0], r0);
              bf8_to_f32(rres[mi][ni][1], r1);
            } else {
              const uint4* rp = reinterpret_cast<const uint4*>(rb + (size_t)q * p.res_ld + co0);
              bf8_to_f32(rp[0], r0);
              bf8_to_f32(rp[1], r1);
            }
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
          if constexpr (ACC) {
            float r0[8], r1[8];
            if constexpr (NRES) {
              bf8_to_f32(racc[mi][ni][0], r0);
              bf8_to_f32(racc[mi][ni][1], r1);
            } else {
              const uint4* ap = reinterpret_cast<const uint4*>(ab + (size_t)q * p.acc_ld + co0);
              bf8_to_f32(ap[0], r0);
              bf8_to_f32(ap[1], r1);
            }
#pragma unroll
            for (int r = 0; r < 8; ++r) {
              v[r] = (r0[r] + v[r]) * adiv;
              v[8 + r] = (r1[r] + v[8 + r]) * adiv;
            }
          }
          bf16_t* dst = yb + (size_t)q * p.y_ld + co0;
          *reinterpret_cast<uint4*>(dst) = f32_to_bf8(&v[0]);
          *reinterpret_cast<uint4*>(dst + 8) = f32_to_bf8(&v[8]);
          if constexpr (SREG) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              st_s[ni][r] += v[r];
              st_q[ni][r] = __builtin_fmaf(v[r], v[r], st_q[ni][r]);
            }
          } else if constexpr (!ACC) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              ts[r] += v[r];
              tq[r] = __builtin_fmaf(v[r], v[r], tq[r]);
            }
          }
        }
      }
      asm volatile("" ::: "memory");  // keep the next group's loads from being hoisted here
      if constexpr (!SREG && !ACC) {
        if (want_stats) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            float a = ts[r], q = tq[r];
#pragma unroll
            for (int o = 16; o >= 1; o >>= 1) {
              a += __shfl_xor(a, o);
              q += __shfl_xor(q, o);
            }
            if (l32 == 0) {
              st_lds[2 * (wm * C + co0 + r)] += a;
              st_lds[2 * (wm * C + co0 + r) + 1] += q;
            }
          }
        }
      }
    }
  };

  // ---------------- one step: MFMAs of global step g (slice slot g&1, window slot of its group)
  const int swz = (l32 >> 2) & 3;
  const bf16_t* wbase = Ws + (size_t)((wn * NTL) * 32 + l32) * 32;
  const bf16_t* xbase = Xs + (size_t)((wm * MT) * 32 + l32) * XP + hi * 8;
  auto mfma_step = [&](int g) __attribute__((always_inline)) {
    if (p.dbg & 2) return;
    const int s = g % NS, tap = s % K;
    const int gg = g / K;  // global group index
    const bf16_t* wt = wbase + (size_t)(g & 3) * G::WSLICE;
    const bf16_t* xt = xbase + (size_t)(gg & 1) * G::R * XP + tap * DIL * XP;
#pragma unroll
    for (int cg = 0; cg < CG; ++cg)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 wa[NTL], xb[MT];
        const int unit = (2 * kk + hi) ^ swz;
#pragma unroll
        for (int ni = 0; ni < NTL; ++ni)
          wa[ni] = *reinterpret_cast<const bf16x8*>(wt + (size_t)(cg * C + ni * 32) * 32 + unit * 8);
#pragma unroll
        for (int mi = 0; mi < MT; ++mi)
          xb[mi] = *reinterpret_cast<const bf16x8*>(xt + mi * 32 * XP + cg * 32 + kk * 16);
#pragma unroll
        for (int mi = 0; mi < MT; ++mi)
#pragma unroll
          for (int ni = 0; ni < NTL; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[ni], xb[mi], acc[mi][ni], 0, 0, 0);
      }
  };

  // ---------------- sub-step g (one (group, tap) slice), split into the staging it owns (for
  // later sub-steps) and its MFMAs + epilogue
  uint4 wr[2][WPT];  // weight slices of the next super-step (registers, one super-step of cover)
  int cur_b = tbeg / ntm;
  auto stage_sub = [&](int g, bool first) __attribute__((always_inline)) {
    const int tl = g / NS, s = g - tl * NS, t = tbeg + tl;
    const int gi = s / K, tap = s - gi * K;
    const int gg = tl * NG + gi;
    if (s == 0) {
      const int b = t / ntm;
      if (b != cur_b) {  // statistics of the utterance the block just left (every epilogue of its
        if constexpr (SREG) {  // last tile ran >= 1 barrier ago; the next one runs a tile later)
          if (p.stats) flush_reg(cur_b);
        } else if (!ACC) {
          if (p.stats) flush_lds(cur_b);
        }
        cur_b = b;
      }
      // the next tile opens another utterance: its coefficients (other parity slot), first read
      // by the transform at sub-step NS-2 of this tile, >= 1 barrier later
      if (t + 1 < tend && (t + 1) / ntm != b) set_coef((t + 1) / ntm);
    }
    if (first && !(p.dbg & 8)) {  // slices g+2, g+3 -> their ring slots (last read one super-step ago); load g+4, g+5
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (g + 2 + j < nsteps) store_w((g + 2 + j) & 3, wr[j]);
        issue_w(g + 4 + j, wr[j]);
      }
    }
    if (tap == K - 2) {
      // window of group gg+1 into the other window slot: its last reader (group gg-1) finished
      // >= 1 super-step ago, its first reader (group gg+1, sub-step s+2) runs >= 1 super-step later
      if (!(p.dbg & 16)) {
        transform_x(gg + 1);
        issue_x(gg + 2);  // the next window's raw loads: one full group (K sub-steps) of cover
      }
    }
  };
  auto mfma_sub = [&](int g) __attribute__((always_inline)) {
    const int tl = g / NS, s = g - tl * NS, t = tbeg + tl;
    if (s == 0) {
#pragma unroll
      for (int ni = 0; ni < NTL; ++ni) {  // the accumulators start at the bias
        float bb[16];
        const int co0 = (wn * NTL + ni) * 32 + hi * 16;
        ld8_lds(bias_s + co0, *reinterpret_cast<float(*)[8]>(&bb[0]));
        ld8_lds(bias_s + co0 + 8, *reinterpret_cast<float(*)[8]>(&bb[8]));
#pragma unroll
        for (int mi = 0; mi < MT; ++mi)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[mi][ni][r] = bb[r];
      }
    }
    if (s == NS - 1) issue_epi(t);  // residual rows (C = 128 path): this sub-step's MFMAs cover them
    mfma_step(g);
    if (s == NS - 1) epilogue(t);
  };

  // ---------------- prologue: slices 0, 1 in LDS, 2, 3 in registers; window 0 transformed,
  // window 1's raw loads in flight
  set_coef(cur_b);
  issue_x(0);
  issue_w(0, wr[0]);
  issue_w(1, wr[1]);
  store_w(0, wr[0]);
  store_w(1, wr[1]);
  issue_w(2, wr[0]);
  issue_w(3, wr[1]);
  __syncthreads();  // coef visible
  transform_x(0);
  issue_x(1);

  // super-steps of two sub-steps per barrier (NS is even: a tile never splits a super-step); the
  // weight ring has 4 slots, the window ring 2 (transform at tap K-2, see stage_sub).  stage(h)
  // writes only what MFMA(h+1..) reads and overwrites only what MFMA(h-1..) read.  (A ping-pong
  // variant, the two wave groups half a super-step apart so one stages while the other issues
  // MFMAs, measured no faster: the staging, not the MFMA pipe, is what the waves wait on.)
  for (int g = 0; g < nsteps; g += 2) {
    __syncthreads();  // slices g, g+1 and their windows visible; slots of g-2, g-1 free
    stage_sub(g, true);
    mfma_sub(g);
    stage_sub(g + 1, false);
    mfma_sub(g + 1);
  }
  __syncthreads();
  if constexpr (SREG) {
    if (p.stats) flush_reg(cur_b);
  } else if constexpr (!ACC) {
    if (p.stats) flush_lds(cur_b);
  }
  if constexpr (!SEG) break;  // (one range)
  __syncthreads();  // (the next range re-stages the LDS)
  }  // tile ranges
}

int g_num_cu_bc = 0;

template <int C, int K, int DIL, bool ACC>
int launch_bc(const ConvParams& p, hipStream_t stream) {
  using G = BG<C, K, DIL>;
  auto kern0 = k_bigconv<C, K, DIL, ACC, false>;
  auto kern1 = k_bigconv<C, K, DIL, ACC, true>;
  static bool attr = false;
  if (!attr) {
    ST_CHECK_HIP(hipFuncSetAttribute((const void*)kern0, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
    ST_CHECK_HIP(hipFuncSetAttribute((const void*)kern1, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
    attr = true;
  }
  if (!g_num_cu_bc) {
    int dev = 0;
    ST_CHECK_HIP(hipGetDevice(&dev));
    ST_CHECK_HIP(hipDeviceGetAttribute(&g_num_cu_bc, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const long long tiles = (long long)((p.Lq + G::BM - 1) / G::BM) * p.B;
  ConvParams q = p;
  const int seg = st_seg_choice(p, 1, g_num_cu_bc);
  long long grid = g_num_cu_bc;
  if (grid > (seg ? (long long)p.B * seg : tiles)) grid = seg ? (long long)p.B * seg : tiles;
  if (g_opt_grid_cap > 0 && grid > g_opt_grid_cap) grid = g_opt_grid_cap;
  const bool segk = seg > 0 && grid < (long long)p.B * seg;  // (one segment per workgroup = the plain even split)
  q.seg = segk ? seg : 0;
  hipLaunchKernelGGL(segk ? kern1 : kern0, dim3((unsigned)grid), dim3(G::NT), G::LDS, stream, q);
  return (int)hipGetLastError();
}

template <int C, int K, int DIL>
int launch_bc_a(const ConvParams& p, hipStream_t s) {
  return p.accb ? launch_bc<C, K, DIL, true>(p, s) : launch_bc<C, K, DIL, false>(p, s);
}
template <int C, int K>
int launch_bc_d(const ConvParams& p, hipStream_t s) {
  switch (p.dil) {
    case 1: return launch_bc_a<C, K, 1>(p, s);
    case 3: return launch_bc_a<C, K, 3>(p, s);
    case 5: return launch_bc_a<C, K, 5>(p, s);
    default: return ST_EINVAL;
  }
}
template <int C>
int launch_bc_k(const ConvParams& p, hipStream_t s) {
  switch (p.KS) {
    case 3: return launch_bc_d<C, 3>(p, s);
    case 7: return launch_bc_d<C, 7>(p, s);
    case 11: return launch_bc_d<C, 11>(p, s);
    default: return ST_EINVAL;
  }
}

}  // namespace

bool st_bigconv_eligible(const ConvParams& p, int dtype) {
  if (dtype != ST_BF16) return false;
  const int C = p.Cout;
  if (!(C == 128 || C == 256) || p.Cin != C || p.N != C || p.nchunks * 32 != C) return false;
  if (!(p.KS == 3 || p.KS == 7 || p.KS == 11) || !(p.dil == 1 || p.dil == 3 || p.dil == 5)) return false;
  if ((p.kw != 0 && p.kw != p.KS) || p.row_off != 0 || p.stride != 1 || p.up != 1 || p.opad != 0) return false;
  if (p.pad != p.dil * (p.KS - 1) / 2 || p.Lq != p.Lout || p.Lq != p.Lin) return false;
  if (p.y_row_off || p.y_f32 || p.epi_tanh || p.epi_lrelu || p.epi_gelu || p.reflect_front || p.zc_period || p.res_shift) return false;
  if (p.pro.mode != (PRO_AFFINE | PRO_SNAKE) || !p.pro.alpha || !p.pro.stats || !p.pro.gamma) return false;
  if (p.accb && p.stats) return false;
  if (p.x_ld % 8 || p.y_ld % 8 || (p.res && p.res_ld % 8) || (p.accb && p.acc_ld % 8)) return false;
  return true;
}

int st_bigconv(const ConvParams& p, hipStream_t stream) {
  if ((g_opt_big3 & 1) && (p.res ? p.dil == 1 : !p.accb)) return st_bigconv3(p, stream);  // bigconv3.hip
  if (st_bigconv2_eligible(p)) return st_bigconv2(p, stream);  // bigconv2.hip
  if (p.Cout == 128) return launch_bc_k<128>(p, stream);
  if (p.Cout == 256) return launch_bc_k<256>(p, stream);
  return ST_EINVAL;
}
