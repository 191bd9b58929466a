// Resblock conv engine v3: the work of bigconv2.hip — the dilated Conv1d of every C = 128 / 256 AdaINResBlock1
// iteration (Modules/hifigan.py:26-80, forward :65-74), the decoder front-end's k3 AdainResBlk1d convs
// (hifigan.py:359-403) and the wide polyphase upsamplers ups[0] / ups[1] (hifigan.py:292-294, 333-335) — with the
// same fused prologue (AdaIN -> Snake, or [AdaIN ->] LReLU) and epilogue (bias, residual, out_scale, resblock
// average, InstanceNorm statistics), on another MFMA tiling and weight staging:
//
//   * wave tile 64 output channels x 128 frames (2 x 4 accumulator fragments of v_mfma_f32_32x32x16_bf16) instead of
//     bigconv2's 32 x 256 (1 x 8).  A half-tap (16 input channels) then reads 2 weight + 4 window fragments for its
//     8 MFMAs instead of 1 + 8: 0.75 ds_read_b128 per MFMA instead of 1.125 (bigconv2's bare MFMA + fragment-read
//     loop ran at 0.50-0.64 of the dense peak, profiles/r05_phases_bf16.txt).
//   * weights: two waves (the two frame halves of a tile) now read each 64-channel weight slice, so bigconv2's
//     private per-wave DMA rings give way to a block-shared, double-buffered CHUNK of TC taps x the tile's output
//     channels x 32 input channels, DMA'd cooperatively (WPT 1-KiB LDS-DMA pieces per wave per tap, spread over the
//     previous chunk's taps) and published by the raw barrier that also publishes the window.  One barrier per chunk:
//     C = 256 holds 3 taps a chunk (k3: one barrier per 32-channel group, as bigconv2), C = 128 on 4-wave blocks 2.
//     The weight bytes moved per tap are bigconv2's (no slice is DMA'd twice).
//   * window (the next group's raw bf16 rows DMA'd into the other half of a 2-buffer ring, transformed in place by
//     the lane that DMA'd them during the group's last chunk) and the epilogue are bigconv2's;
//   * statistics: LDS words per frame slice (one writer each), converted to fixed point at EVERY tile boundary, so the
//     InstanceNorm totals do not depend on the tile -> workgroup split (grid, batch size, rank count: SURVEY §8(e)).
//
// Every output accumulates over (group, tap, half) in bigconv2's order on the same MFMA instruction, so a conv's
// output equals bigconv2's bit for bit on the same inputs; the statistics' fp32 partials are grouped differently
// (128-frame lane sums, one tile at a time), so a decode through both differs at the rounding of those partials
// (tests/test_gpu_decoder.py test_bigconv3_decoder_ab).
#include <type_traits>

#include "common.h"
#include "conv_common.h"
#include "kernels.h"
#include "lds_dma.h"

namespace {

// compile-time loop: f(integral_constant<I>) for I in [I0, N)
template <int I, int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}

// C: GEMM columns (the output channels; UPS: u Cout phase-major columns); CO: channels of the bias / statistics
template <int C, int NW, int K, int DIL, int PRO, int CINP, bool UPS, int CO>
struct B3 {
  static constexpr int NCOEF = PRO == PK_SNAKE ? 5 : 2;       // coefficient rows per input channel
  static constexpr int NCP = (C / 64 < NW / 2) ? C / 64 : NW / 2;  // 64-channel column pairs per tile
  static constexpr int FH = NW / NCP;                          // 128-frame slices per tile
  static constexpr int NCO = 64 * NCP;                         // output columns per tile
  static constexpr int NCH = C / NCO;                          // column parts per frame tile
  static constexpr int TM = 128 * FH;                          // tile rows (frames)
  static constexpr int PAD = UPS ? DIL * (K - 1) : DIL * (K - 1) / 2;
  static constexpr int R = TM + DIL * (K - 1);                 // window rows a group needs
  static constexpr int NWIN = (R * 4 + 64 * NW - 1) / (64 * NW);  // window DMA pieces per wave per group
  static constexpr int WROWS = NWIN * NW * 16;
  static constexpr int XBYTES = WROWS * 64;
  static constexpr int TAPB = NCO * 64;                        // one tap's weight slice (NCO x 32 bf16)
  static constexpr int WPT = TAPB / (NW * 1024);               // its DMA pieces per wave
  static constexpr int OFF_COEF = 0;                           // [2][NCOEF][CINP] f32 (utterance parity)
  static constexpr int OFF_BIAS = OFF_COEF + 2 * NCOEF * CINP * 4;
  static constexpr int OFF_ST = OFF_BIAS + CO * 4;             // [FH][CO][2] f32, one copy per frame slice
  static constexpr int OFF_W = (OFF_ST + FH * 2 * CO * 4 + 1023) / 1024 * 1024;
  static constexpr int BPC = NW == 4 ? 2 : 1;                  // blocks per CU
  static constexpr int TCMAX = (160 * 1024 / BPC - OFF_W - 2 * XBYTES) / (2 * TAPB);
  static constexpr int TC = TCMAX < K ? TCMAX : K;             // taps per weight chunk
  static constexpr int NCK = (K + TC - 1) / TC;                // chunks (barriers) per group
  static constexpr int OFF_X = OFF_W + 2 * TC * TAPB;          // [2][WROWS][64 B]
  static constexpr int LDS = OFF_X + 2 * XBYTES;
  static_assert(FH * NCP == NW && NCH * NCO == C && NCP >= 1, "wave grid");
  static_assert(WPT >= 1 && WPT * NW * 1024 == TAPB, "weight DMA pieces");
  static_assert(TC >= 1 && LDS * BPC <= 160 * 1024, "LDS budget");
  static_assert(!UPS || NCO <= CO, "one output phase per tile part");
  static_assert(OFF_W % 1024 == 0 && OFF_X % 1024 == 0, "DMA bases");
  static_assert(NW == 4 || NW == 8, "wave counts");
};

template <int C, int NW, int K, int DIL, bool RES, bool ACC, int PRO = PK_SNAKE, int CINP = C, bool UPS = false,
          int CO = C>
__global__ void __launch_bounds__(64 * NW, 2) k_bigconv3(const ConvParams p) {
  using G = B3<C, NW, K, DIL, PRO, CINP, UPS, CO>;
  constexpr int TM = G::TM, NWIN = G::NWIN, NCH = G::NCH, NCO = G::NCO, NCF = G::NCOEF;
  constexpr int TC = G::TC, NCK = G::NCK, WPT = G::WPT, TAPB = G::TAPB;
  // input-channel groups: C / 32 for the square resblock convs, ceil(Cin / 32) for the front-end and the upsamplers
  const int NG = (PRO == PK_SNAKE && CINP == C) ? C / 32 : (p.Cin + 31) / 32;
  constexpr int NT = 64 * NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* coef = reinterpret_cast<float*>(smem + G::OFF_COEF);
  float* bias_s = reinterpret_cast<float*>(smem + G::OFF_BIAS);
  float* st_lds = reinterpret_cast<float*>(smem + G::OFF_ST);
  char* const wbuf = smem + G::OFF_W;

  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hi = lane >> 5;
  const int wu = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave index, provably uniform
  const int cp = wu % G::NCP, fh = wu / G::NCP;               // column pair, frame slice
  const int ntm = (p.Lq + TM - 1) / TM;
  // tile t -> utterance t / (NCH ntm), column part (t / ntm) % NCH, frame tile t % ntm (bigconv2's order)
  const long long total = (long long)ntm * NCH * p.B;
  const int upb = ntm * NCH;
  const int tbeg = (int)(total * blockIdx.x / gridDim.x);
  const int tend = (int)(total * (blockIdx.x + 1) / gridDim.x);
  if (tbeg >= tend) return;  // uniform over the block
  const int NGG = (tend - tbeg) * NG;
  const bool want_stats = !ACC && p.stats != nullptr;

  for (int i = tid; i < CO; i += NT) bias_s[i] = p.bias ? p.bias[i] : 0.f;
  for (int i = tid; i < G::FH * 2 * CO; i += NT) st_lds[i] = 0.f;

  // ---------------- weights: piece i of tap t (group gi, column part ch) -> tap slot tl of chunk buffer cbuf.
  // The packed layout (stts_pack) holds a tap's C x 32 slice contiguously, 64 B a column, 16-B units XOR-swizzled
  // by (column >> 2) & 3; piece k of a part covers its columns 16 k .. 16 k + 15
  const Rsrc rw = make_rsrc(p.w, (unsigned)((size_t)NG * K * C * 32 * 2));
  const unsigned wlane = (unsigned)lane * 16u;
  auto issue_wp = [&](int cbuf, int tl, int gi, int ch, int t, int i) __attribute__((always_inline)) {
    const int piece = i * NW + wu;
    char* dst = wbuf + (cbuf * TC + tl) * TAPB + piece * 1024;
    // (lane part in one VGPR for every piece, the uniform part through the SGPR offset)
    const unsigned soff = (unsigned)((((size_t)gi * K + t) * C + (size_t)ch * NCO) * 64) + (unsigned)(piece * 1024);
    glds16s(rw, dst, wlane, __builtin_amdgcn_readfirstlane(soff));
    // (STTS_OPT_EXP bit 131072, a cost probe: every piece DMA'd twice, the same bytes to the same place)
    if (p.exp & 131072) glds16s(rw, dst, wlane, __builtin_amdgcn_readfirstlane(soff));
  };

  // ---------------- window: group gg -> raw rows [gr0, gr0 + WROWS) of its 32 channels, buffer gg & 1.
  // LDS unit pidx = row * 4 + u' holds logical 16-B unit u = u' ^ ((row >> 2) & 3) of that row
  auto issue_x = [&](int gg, int gi, int b, int mt) __attribute__((always_inline)) {
    const Rsrc rx = make_rsrc(reinterpret_cast<const char*>(p.x) + (size_t)b * p.x_bs * 2,
                              (unsigned)((size_t)p.Lin * p.x_ld * 2));
    const int gr0 = mt * TM - G::PAD;
    char* dst = smem + G::OFF_X + (gg & 1) * G::XBYTES;
#pragma unroll
    for (int j = 0; j < NWIN; ++j) {
      const int pidx = (j * NW + wu) * 64 + lane;
      const int r = pidx >> 2, u = (pidx & 3) ^ ((r >> 2) & 3);
      const int e = (gr0 + r) * p.x_ld + gi * 32 + 8 * u;
      // rows past the window (WROWS rounds R up to whole pieces) read out of range: no HBM traffic for them
      glds16(rx, dst + (j * NW + wu) * 1024, (e >= 0 && r < G::R) ? (unsigned)e * 2u : OOB);
    }
  };
  // AdaIN (+ Snake) coefficients of utterance b into parity slot b & 1 (bigconv2.hip)
  auto set_coef = [&](int b) __attribute__((always_inline)) {
    float* cf = coef + (b & 1) * NCF * CINP;
    if constexpr (PRO == PK_SNAKE) {
      for (int ci = tid; ci < CINP; ci += NT) {
        float mm = 0.f, aa = 1.f, be = 0.f;  // Snake alone (the upsamplers' prologue): a = 1, m = 0
        if (!UPS || (p.pro.mode & PRO_AFFINE)) adain_coeffs(p.pro, b, ci, mm, aa, be);
        const float al = p.pro.alpha[ci];
        const float m1 = be - mm * aa, ia2 = 0.5f / al, alr = al * 0.31830988618379067f;
        cf[ci] = m1 + ia2;
        cf[CINP + ci] = aa;
        cf[2 * CINP + ci] = aa * alr;
        cf[3 * CINP + ci] = m1 * alr;
        cf[4 * CINP + ci] = -ia2;
      }
    } else {  // x * a + m (AdaIN, or a = 1, m = 0 without it); channels >= Cin: a = m = 0 -> 0
      for (int ci = tid; ci < CINP; ci += NT) {
        float mm = 0.f, aa = 1.f, be = 0.f;
        if (ci < p.Cin && (p.pro.mode & PRO_AFFINE)) adain_coeffs(p.pro, b, ci, mm, aa, be);
        const bool ok = ci < p.Cin;
        cf[ci] = ok ? be - mm * aa : 0.f;
        cf[CINP + ci] = ok ? aa : 0.f;
      }
    }
  };
  // in-place transform of the units this lane DMA'd for group gg: x -> AdaIN -> Snake / LReLU -> bf16, 0 outside
  // [0, Lin) (Snake via sin^2(u) = (1 - cos 2u) / 2 on the hardware cosine, as bigconv2)
  const int my_u = (lane & 3) ^ ((lane >> 4) & 3);  // the lane's logical unit: the same in every row it owns
  auto transform = [&](int gg, int gi, int b, int mt) __attribute__((always_inline)) {
    const int gr0 = mt * TM - G::PAD;
    char* buf = smem + G::OFF_X + (gg & 1) * G::XBYTES;
    const float* cf = coef + (b & 1) * NCF * CINP + gi * 32 + 8 * my_u;
    if constexpr (PRO == PK_LRELU) {
      constexpr int JC = NWIN < 3 ? NWIN : 3;  // (in chunks of at most 3 units: more at once spill)
#pragma unroll
      for (int j0 = 0; j0 < NWIN; j0 += JC) {
        uint4 raw[JC];
#pragma unroll
        for (int jj = 0; jj < JC; ++jj)
          if (j0 + jj < NWIN) raw[jj] = *reinterpret_cast<const uint4*>(buf + (((j0 + jj) * NW + wu) * 64 + lane) * 16);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          f32x4v m2, a;
          lds_coef2(lds_addr(cf + 4 * h), m2, a, (unsigned)(CINP * 4));  // (its wait also covers raw[])
          const float am[4] = {m2.x, m2.y, m2.z, m2.w}, aa[4] = {a.x, a.y, a.z, a.w};
          const float slope = (p.pro.mode & PRO_LRELU) ? p.pro.slope : 1.0f;
          // channels >= Cin (the last group's padding, whose memory may hold anything) are forced to 0
          const int c0 = gi * 32 + 8 * my_u + 4 * h;
#pragma unroll
          for (int j = 0; j < JC; ++j) {
            if (j0 + j >= NWIN) continue;
            uint2 hv = h ? make_uint2(raw[j].z, raw[j].w) : make_uint2(raw[j].x, raw[j].y);
            float v[4];
            bf4_to_f32(hv, v);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float x2 = __builtin_fmaf(v[e], aa[e], am[e]);
              v[e] = c0 + e < p.Cin ? (x2 > 0.f ? x2 : x2 * slope) : 0.f;
            }
            hv = f32_to_bf4(v);
            if (h) { raw[j].z = hv.x; raw[j].w = hv.y; } else { raw[j].x = hv.x; raw[j].y = hv.y; }
          }
        }
#pragma unroll
        for (int j = 0; j < JC; ++j) {
          if (j0 + j >= NWIN) continue;
          const int pidx = ((j0 + j) * NW + wu) * 64 + lane;
          uint4 o = raw[j];
          if ((unsigned)(gr0 + (pidx >> 2)) >= (unsigned)p.Lin) o = make_uint4(0u, 0u, 0u, 0u);
          lds_write_b128(lds_addr(buf + pidx * 16), o);
        }
      }
      return;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      f32x4v m2, a, ar, mr, nia;
      lds_coef5(lds_addr(cf + 4 * h), m2, a, ar, mr, nia, (unsigned)(CINP * 4));
      const float am[4] = {m2.x, m2.y, m2.z, m2.w}, aa[4] = {a.x, a.y, a.z, a.w};
      const float aar[4] = {ar.x, ar.y, ar.z, ar.w}, amr[4] = {mr.x, mr.y, mr.z, mr.w};
      const float ani[4] = {nia.x, nia.y, nia.z, nia.w};
#pragma unroll
      for (int j = 0; j < NWIN; ++j) {
        const int pidx = (j * NW + wu) * 64 + lane;
        const int r = pidx >> 2;
        if (G::WROWS > G::R && r >= G::R) continue;  // padding rows: never read by a tap
        uint2* ptr = reinterpret_cast<uint2*>(buf + pidx * 16 + 8 * h);
        float v[4];
        bf4_to_f32(*ptr, v);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float x2 = __builtin_fmaf(v[e], aa[e], am[e]);
          const float c = __builtin_amdgcn_cosf(__builtin_fmaf(v[e], aar[e], amr[e]));
          v[e] = __builtin_fmaf(c, ani[e], x2);
        }
        uint2 o = f32_to_bf4(v);
        if ((unsigned)(gr0 + r) >= (unsigned)p.Lin) o = make_uint2(0u, 0u);
        lds_write_b64(lds_addr(ptr), o);
      }
    }
  };

  // ---------------- statistics: the LDS words of the tile that just closed -> fixed point, at every tile boundary.
  // Each tile's partial (per frame slice: the epilogue's lane reduction over its 128 frames; slices summed in a fixed
  // order here) is converted on its own and the fixed-point adds are exact, so the totals do not depend on which
  // workgroup ran which tiles: not on the grid, the batch size or the rank count (§8(e); bigconv2 accumulated a
  // block's tiles of an utterance in fp32 first, which tied the bits to the tile -> workgroup split).  LDS accesses
  // as asm: the compiler would otherwise drain the in-flight LDS-DMAs before them
  auto flush = [&](int b) __attribute__((always_inline)) {
    for (int ci = tid; ci < CO; ci += NT) {
      double* d = stats_slot(p, blockIdx.x) + ((size_t)b * p.stats_ld + ci) * ST_W;
      float a = 0.f, q = 0.f;
#pragma unroll
      for (int h = 0; h < G::FH; ++h) {  // (frame slices in a fixed order)
        const unsigned la = lds_addr(st_lds + (h * CO + ci) * 2);
        float2 v;
        asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(la) : "memory");
        a += v.x;
        q += v.y;
        lds_write_b64(la, make_uint2(0u, 0u));
      }
      fx_add(d, a);
      fx_add(d + 2, q);
    }
  };

  // ---------------- accumulators: acc[c * 4 + f] = columns 32 c .. 32 c + 31 of the wave's pair x frames 32 f ..
  f32x16 acc[8];
  auto epilogue = [&](int b, int mt, int ch) __attribute__((always_inline)) {
    const int q0 = mt * TM + fh * 128 + l32;
    const int Lrows = UPS ? p.Lout : p.Lq;
    const Rsrc ry = make_rsrc(reinterpret_cast<char*>(p.y) + (size_t)b * p.y_bs * 2, (unsigned)((size_t)Lrows * p.y_ld * 2));
    const Rsrc rr = make_rsrc(RES ? reinterpret_cast<const char*>(p.res) + (size_t)b * p.res_bs * 2 : nullptr,
                              RES ? (unsigned)((size_t)Lrows * p.res_ld * 2) : 0u);
    const Rsrc ra = make_rsrc(ACC ? reinterpret_cast<const char*>(p.accb) + (size_t)b * p.acc_bs * 2 : nullptr,
                              ACC ? (unsigned)((size_t)p.Lq * p.acc_ld * 2) : 0u);
    const float osc = p.out_scale;
    const float adiv = (ACC && p.acc_div != 0.f) ? 1.0f / p.acc_div : 1.0f;
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) in the compiler's model: the loads below are counted exactly
    sfor<0, 2>([&](auto CC) {  // (a compile-time column block: acc[] indices stay static)
      constexpr int c = decltype(CC)::value;
      // the lane's 16 consecutive output channels (packing permutation)
      const int co0 = ch * NCO + 64 * cp + 32 * c + 16 * hi;
      // UPS: the lane's 16 columns are channels c0.. of output phase ph; row q -> frame q u + ph - opad
      const int ph = UPS ? co0 / p.Cout : 0, c0 = UPS ? co0 - ph * p.Cout : co0;
      auto orow = [&](int q) __attribute__((always_inline)) { return UPS ? q * p.up + ph - p.opad : q; };
      float ts[16], tq[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) ts[r] = tq[r] = 0.f;
      // the residual / running-sum rows of the 4 fragments go out together: one load latency per column block
      uint4 rl[4][2], al[4][2];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const int q = q0 + 32 * f;
        if constexpr (RES) {
          const unsigned er = (unsigned)((UPS ? orow(q) : (q >> p.res_shift)) * p.res_ld + c0) * 2u;
          rl[f][0] = bload16(rr, er);
          rl[f][1] = bload16(rr, er + 16u);
        }
        if constexpr (ACC) {
          const unsigned ea = (unsigned)(q * p.acc_ld + co0) * 2u;
          al[f][0] = bload16(ra, ea);
          al[f][1] = bload16(ra, ea + 16u);
        }
      }
      asm volatile("" ::: "memory");
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        f32x16& v = acc[c * 4 + f];  // in place: the accumulators of a finished tile are the output
        const int q = q0 + 32 * f;
        if constexpr (RES) {
          float r0[16];
          bf8_to_f32v(rl[f][0], r0);
          bf8_to_f32v(rl[f][1], r0 + 8);
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = (v[r] + r0[r]) * osc;
        }
        if constexpr (ACC) {
          float a0[16];
          bf8_to_f32v(al[f][0], a0);
          bf8_to_f32v(al[f][1], a0 + 8);
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = (a0[r] + v[r]) * adiv;
        }
        float o[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) o[r] = v[r];
        // rows past the output (and UPS rows before frame 0: negative offsets) fall outside the descriptor
        const unsigned ey = (unsigned)(orow(q) * p.y_ld + c0) * 2u;
        bstore16(ry, ey, f32_to_bf8v(o));
        bstore16(ry, ey + 16u, f32_to_bf8v(o + 8));
        if (!ACC) {
          const float m = (unsigned)orow(q) < (unsigned)Lrows ? 1.f : 0.f;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float x = v[r] * m;
            ts[r] += x;
            tq[r] = __builtin_fmaf(x, x, tq[r]);
          }
        }
      }
      asm volatile("" ::: "memory");
      if (want_stats) {
        // reduce-scatter over the 32 lanes of the half (bigconv2): lane l32 ends with channel c0 + l32 / 2, the even
        // lane adds the sum, the odd one the sum of squares into this frame slice's word (one writer)
        const float s1 = rs16(ts, l32);
        const float s2 = rs16(tq, l32);
        atomicAdd(st_lds + 2 * (fh * CO + c0 + (l32 >> 1)) + (l32 & 1), (l32 & 1) ? s2 : s1);
      }
    });
  };
  auto init_acc = [&](int ch) __attribute__((always_inline)) {
    sfor<0, 2>([&](auto CC) {
      constexpr int c = decltype(CC)::value;
      const int co0 = (ch * NCO + 64 * cp + 32 * c + 16 * hi) % CO;  // (UPS: the bias of channel n % Cout)
      float bb[16];
      ld8_lds(bias_s + co0, *reinterpret_cast<float(*)[8]>(&bb[0]));
      ld8_lds(bias_s + co0 + 8, *reinterpret_cast<float(*)[8]>(&bb[8]));
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[c * 4 + f][r] = bb[r];
    });
  };

  // ---------------- fragments.  Weight fragment of column block c, half h of tap slot tl: 32 columns x 16 input
  // channels (logical units 2 h + hi of each column's 64 B); window fragment f of tap t, half h: frames
  // fh 128 + 32 f + l32 + t DIL, logical unit 2 h + hi
  const int swz = (l32 >> 2) & 3;
  auto rd_a = [&](int cbuf, int tl, int half, bf16x8 (&a)[2]) __attribute__((always_inline)) {
    const char* ws = wbuf + (cbuf * TC + tl) * TAPB + (64 * cp + l32) * 64 + ((2 * half + hi) ^ swz) * 16;
    a[0] = *reinterpret_cast<const bf16x8*>(ws);
    a[1] = *reinterpret_cast<const bf16x8*>(ws + 2048);
  };
  auto rd_b = [&](int xb, int t, int half, bf16x8 (&bq)[4]) __attribute__((always_inline)) {
    // (an opaque copy of the lane index: the address is formed at the tap, not hoisted as K live registers)
    int l = l32;
    asm volatile("" : "+v"(l));
    const int r0 = fh * 128 + l + t * DIL;
    const int u = ((2 * half + hi) ^ ((r0 >> 2) & 3)) * 16;  // rows r0 + 32 f share the swizzle
    const char* row = smem + G::OFF_X + xb * G::XBYTES + r0 * 64 + u;
#pragma unroll
    for (int f = 0; f < 4; ++f) bq[f] = *reinterpret_cast<const bf16x8*>(row + f * 2048);
  };
  // 8 MFMAs of one half-tap; the reads of the next half's 2 + 4 fragments go one per MFMA gap
  auto mfma8 = [&](const bf16x8 (&a)[2], const bf16x8 (&bq)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int c = 0; c < 2; ++c)
        acc[c * 4 + f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[c], bq[f], acc[c * 4 + f], 0, 0, 0);
  };
  auto interleave6 = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
  };

  // ---------------- group cursors (tile, group, utterance, frame tile, column part), advanced incrementally
  struct GCur { int tt, gi, b, mt, ch; };
  auto advance = [&](GCur c) __attribute__((always_inline)) {
    if (++c.gi == NG) {
      c.gi = 0;
      ++c.tt;
      if (++c.mt == ntm) {
        c.mt = 0;
        if (++c.ch == NCH) {
          c.ch = 0;
          ++c.b;
        }
      }
    }
    return c;
  };

  // ---------------- prologue: coefficients, group 0's window transformed, chunk 0 of group 0 in buffer 0
  GCur cur = {tbeg, 0, tbeg / upb, tbeg % ntm, NCH > 1 ? (tbeg / ntm) % NCH : 0};
  int cur_b = cur.b;
  set_coef(cur_b);
  __syncthreads();  // nothing in flight yet
  issue_x(0, 0, cur.b, cur.mt);
  sfor<0, TC>([&](auto TL) {
    sfor<0, WPT>([&](auto I) { issue_wp(0, decltype(TL)::value, 0, cur.ch, decltype(TL)::value, decltype(I)::value); });
  });
  vm_wait<0>();
  transform(0, 0, cur.b, cur.mt);
  init_acc(cur.ch);

  // ---------------- main loop: one iteration per 32-channel group, NCK chunks (barriers) unrolled inside.  Step
  // (group gg, chunk j) computes from chunk buffer cb and DMAs the next step's weights into cb ^ 1 (spread over its
  // taps); chunk 0 also DMAs the next group's window into buffer (gg + 1) & 1, which the last chunk transforms
  // STTS_OPT_DEBUG phase skipping (timing attribution only; outputs are wrong while set): 1 transform, 4 epilogue,
  // 8 weight DMAs, 16 window DMAs, 32 chunk barrier.  STTS_OPT_EXP bit 65536 (A/B): every chunk issues the next step's
  // weight pieces in one burst at its start and the window after them, so the end-of-chunk wait for the pieces does
  // not also wait for the window's HBM latency (LDS-DMAs retire in issue order); else the pieces are spread over the
  // chunk's taps, after the window
  const int dbg = p.dbg;
  const bool burst = (p.exp & 65536) != 0;
  int cb = 0;
  for (int gg = 0; gg < NGG; ++gg) {
    // the next group (past the end: the last group again, a harmless reload keeping the DMA counts uniform)
    const GCur nxt = gg + 1 < NGG ? advance(cur) : cur;
    const int xb = gg & 1;
    sfor<0, NCK>([&](auto J) {
      constexpr int j = decltype(J)::value;
      constexpr int t0 = j * TC;
      constexpr int t1 = (t0 + TC < K) ? t0 + TC : K;
      constexpr int tcur = t1 - t0;
      constexpr bool lastc = j == NCK - 1;
      // the next step's taps [n0, n1) (chunk j + 1 of this group, or chunk 0 of the next group)
      constexpr int n0 = lastc ? 0 : t1;
      constexpr int n1 = lastc ? TC : ((t1 + TC < K) ? t1 + TC : K);
      constexpr int NP = (n1 - n0) * WPT;
      if (!(dbg & 32)) barrier_lds();  // this chunk's weights (and at j = 0 the group's window) landed everywhere
      else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if constexpr (j == 0) {
        if (cur.gi == 0) {
          if (gg > 0 && want_stats) flush(cur_b);  // the previous tile's statistics (its epilogue ran before this barrier)
          cur_b = cur.b;
          // the next tile opens another utterance: its coefficients, first read by the transform of its group 0
          // during this tile's last group, >= 1 barrier from here (NG >= 4)
          if (cur.tt + 1 < tend && cur.mt == ntm - 1 && cur.ch == NCH - 1) set_coef(cur.b + 1);
        }
      }
      const int ngi = lastc ? nxt.gi : cur.gi, nch = lastc ? nxt.ch : cur.ch;
      if (burst && !(dbg & 8)) {
        sfor<0, NP>([&](auto PP) {
          constexpr int pc = decltype(PP)::value;
          issue_wp(cb ^ 1, pc / WPT, ngi, nch, n0 + pc / WPT, pc % WPT);
        });
      }
      // the next group's window: buffer (gg + 1) & 1, last read in group gg - 1
      if (j == 0 && !(dbg & 16)) issue_x(gg + 1, nxt.gi, nxt.b, nxt.mt);
      bf16x8 a0[2], a1[2], b0[4], b1[4];
      rd_a(cb, 0, 0, a0);
      rd_b(xb, t0, 0, b0);
      sfor<0, tcur>([&](auto TT) {
        constexpr int tl = decltype(TT)::value, t = t0 + tl;
        // this tap's share of the next step's weight pieces
        constexpr int P0 = tl * NP / tcur, P1 = (tl + 1) * NP / tcur;
        if (!burst && !(dbg & 8)) {
          sfor<P0, P1>([&](auto PP) {
            constexpr int pc = decltype(PP)::value;
            issue_wp(cb ^ 1, pc / WPT, ngi, nch, n0 + pc / WPT, pc % WPT);
          });
        }
        // half 0 of tap t; reads of half 1
        rd_a(cb, tl, 1, a1);
        rd_b(xb, t, 1, b1);
        mfma8(a0, b0);
        interleave6();
        // half 1; reads of the next tap's half 0
        if constexpr (tl + 1 < tcur) {
          rd_a(cb, tl + 1, 0, a0);
          rd_b(xb, t + 1, 0, b0);
          mfma8(a1, b1);
          interleave6();
        } else {
          mfma8(a1, b1);
        }
        // the next group's window: the last chunk transforms it, after this wave's DMA of it landed (younger: the
        // next-step pieces issued after it in this chunk).  With two waves per SIMD (NW = 8) the second half of the
        // waves transforms one tap earlier, so each SIMD's transforms run beside its partner's MFMAs
        if constexpr (lastc) {
          constexpr int TXA = t1 - 1;
          constexpr int TXB = (NW == 8 && t1 - 2 >= t0) ? t1 - 2 : t1 - 1;
          if ((t == TXA && (NW != 8 || wu < NW / 2)) || (t == TXB && NW == 8 && wu >= NW / 2)) {
            if (burst) {
              if constexpr (NCK == 1) vm_wait<0>();  // (the window went out after this chunk's pieces)
              else vm_wait<NP>();                    // (window of chunk 0; this chunk's pieces are younger)
            } else {
              vm_wait<P1>();
            }
            if (!(dbg & 1)) transform(gg + 1, nxt.gi, nxt.b, nxt.mt);
          }
        }
      });
      // this wave's pieces of the next step landed (burst, chunk 0: the window, younger, may still be in flight)
      if (burst && j == 0) vm_wait<NWIN>();
      else vm_wait<0>();
      if constexpr (lastc) {
        if (cur.gi == NG - 1) {
          if (!(dbg & 4)) epilogue(cur.b, cur.mt, cur.ch);
          init_acc(nxt.ch);
        }
      }
      cb ^= 1;
    });
    cur = nxt;
  }
  vm_wait<0>();  // nothing may land in LDS after the block's exit
  barrier_lds();
  if (want_stats) flush(cur_b);
}

template <int C, int NW, int K, int DIL, bool RES, bool ACC, int PRO = PK_SNAKE, int CINP = C, bool UPS = false,
          int CO = C>
int launch_b3(const ConvParams& p, hipStream_t stream) {
  using G = B3<C, NW, K, DIL, PRO, CINP, UPS, CO>;
  auto kern = k_bigconv3<C, NW, K, DIL, RES, ACC, PRO, CINP, UPS, CO>;
  static bool attr = false;
  if (!attr) {
    ST_CHECK_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
    attr = true;
  }
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    ST_CHECK_HIP(hipGetDevice(&dev));
    ST_CHECK_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  // shapes the kernel's tiling assumes (checked on the host: a mismatch would index outside the packed weights)
  if (p.N != C || (UPS ? p.Cout != CO : p.Cout != C) || p.KS != K || p.dil != DIL) return ST_EINVAL;
  if ((PRO == PK_SNAKE && CINP == C) ? p.Cin != C : (p.Cin > CINP || p.nchunks * 32 < p.Cin)) return ST_EINVAL;
  const long long tiles = (long long)((p.Lq + G::TM - 1) / G::TM) * G::NCH * p.B;
  long long grid = (long long)ncu * G::BPC;
  if (grid > tiles) grid = tiles;
  if (g_opt_grid_cap > 0 && grid > g_opt_grid_cap) grid = g_opt_grid_cap;
  ConvParams q = p;
  q.exp = g_opt_exp;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * NW), G::LDS, stream, q);
  return (int)hipGetLastError();
}

template <int C, int NW, int K>
int launch_b3_k(const ConvParams& p, hipStream_t s) {
  constexpr bool F = false, T = true;
  if (!p.res) {  // conv1 of an iteration: dilation 1 / 3 / 5, no residual
    if (p.accb) return ST_EINVAL;
    switch (p.dil) {
      case 1: return launch_b3<C, NW, K, 1, F, F>(p, s);
      case 3: return launch_b3<C, NW, K, 3, F, F>(p, s);
      case 5: return launch_b3<C, NW, K, 5, F, F>(p, s);
      default: return ST_EINVAL;
    }
  }
  if (p.dil != 1) return ST_EINVAL;  // conv2: dilation 1, residual, optionally the resblock sum
  if (p.accb) return launch_b3<C, NW, K, 1, T, T>(p, s);
  return launch_b3<C, NW, K, 1, T, F>(p, s);
}

template <int C, int NW>
int launch_b3_c(const ConvParams& p, hipStream_t s) {
  switch (p.KS) {
    case 3: return launch_b3_k<C, NW, 3>(p, s);
    case 7: return launch_b3_k<C, NW, 7>(p, s);
    case 11: return launch_b3_k<C, NW, 11>(p, s);
    default: return ST_EINVAL;
  }
}

int b3_num_cu() {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      ncu = 256;
  }
  return ncu;
}

}  // namespace

#ifndef B3_ONLY
// STTS_OPT_BIG3 (bit mask): 1 = the C = 128 / 256 resblock convs, 2 = the front-end k3 convs, 4 = ups[0] / ups[1] run
// on this engine instead of bigconv2 (and v1 for C = 128 k3); 8 = C = 128 on 8-wave blocks (512-frame tiles, 4-tap
// chunks) instead of two 4-wave blocks per CU (256-frame tiles, 2-tap chunks); 16 = C = 256 on two 4-wave blocks per CU
// (1-tap chunks) at every batch size
int g_opt_big3 = 0;

int st_bigconv3(const ConvParams& p, hipStream_t s) {
  // (the caller checked st_bigconv_eligible: square C = 128 / 256 'same' convs with the AdaIN -> Snake prologue)
  if (p.res ? p.dil != 1 : (p.accb != nullptr)) return ST_EINVAL;
  if (p.Cout == 128) return (g_opt_big3 & 8) ? launch_b3_c<128, 8>(p, s) : launch_b3_c<128, 4>(p, s);
  if (p.Cout == 256) {
    // (few tiles, small batches: 4-wave blocks, two per CU, as bigconv2 does)
    const long long tiles8 = (long long)((p.Lq + 255) / 256) * p.B;
    // (bit 16: 4-wave blocks, two per CU, at every size: one block's chunk barriers beside the other's MFMAs; A/B)
    return (tiles8 < b3_num_cu() || (g_opt_big3 & 16)) ? launch_b3_c<256, 4>(p, s) : launch_b3_c<256, 8>(p, s);
  }
  return ST_EINVAL;
}

int st_bigconv3_front(const ConvParams& p, hipStream_t s) {
  constexpr bool F = false, T = true;
  if (p.Cout == 1024)
    return p.res ? launch_b3<1024, 8, 3, 1, T, F, PK_LRELU, 1120>(p, s) : launch_b3<1024, 8, 3, 1, F, F, PK_LRELU, 1120>(p, s);
  if (p.Cout == 512)
    return p.res ? launch_b3<512, 8, 3, 1, T, F, PK_LRELU, 1120>(p, s) : launch_b3<512, 8, 3, 1, F, F, PK_LRELU, 1120>(p, s);
  return ST_EINVAL;
}

int st_bigconv3_ups(const ConvParams& p, hipStream_t s) {
  if (p.N == 2560 && p.Cout == 256) return launch_b3<2560, 8, 2, 1, true, false, PK_SNAKE, 512, true, 256>(p, s);
  if (p.N == 640 && p.Cout == 128) return launch_b3<640, 4, 2, 1, true, false, PK_SNAKE, 256, true, 128>(p, s);
  return ST_EINVAL;
}
#endif  // B3_ONLY
