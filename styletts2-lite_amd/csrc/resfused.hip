// Fused AdaINResBlock1 iteration for the narrow generator stages (C = 32 at K = 3 / 7 / 11, C = 64 at K = 3):
//     xt = conv1(Snake1(AdaIN1(x)))            dilated Conv1d(C, C, K, dil d)
//     x' = conv2(Snake2(AdaIN2(xt))) + x       Conv1d(C, C, K, dil 1)
// (Modules/hifigan.py:65-74).  AdaIN2 normalises xt over the whole utterance, so an iteration is two
// launches of this kernel: a statistics pass (MODE 0: conv1 over the output rows, only the per-(utterance,
// channel) sums of xt leave the chip) and the fused pass (MODE 1 / 2: conv1 over the output rows plus
// conv2's halo, AdaIN2 -> Snake2 into LDS, conv2, + x, the InstanceNorm sums of x' or the resblock running
// sum).  Per iteration that moves x twice and x' once through HBM instead of x, xt, xt, x, x' (the unfused
// pair of resconv launches): 3 activation passes instead of 5, for conv1's MFMAs twice.
//
// Wave-independent pipeline (the round-2 resfused kernel ran all 8 waves of one block per CU in lock
// step, three barriers per tile, and its skeleton alone was 2/3 of the fused iteration's HBM floor:
// DESIGN.md §3): every wave owns a contiguous range of 64-frame tiles and runs its own loop with no
// barrier after the block's one-time weight load.
//   * the raw windows of tiles t + 1 .. t + PFD are loaded into registers (buffer loads, unconditional,
//     out-of-range rows read 0) while tile t computes: PFD named register sets;
//   * the wave's private LDS buffer holds Snake1(AdaIN1(x)) (conv1's B operand), then, in place once conv1
//     has read it, Snake2(AdaIN2(xt)) (conv2's B operand): LDS ops of one wave retire in order;
//   * both layers' packed weights (st_pack_conv's [chunk][tap][n][32] bf16 rows, 16-B units XOR-swizzled
//     by (n >> 2) & 3) stay in LDS for the block's lifetime, shared by its waves;
//   * window rows are stored with their 16-B units XOR-swizzled by the row (conflict-free ds_read_b128
//     fragment reads), each lane keeping one logical unit (8 channels) in every row it stores, so its
//     AdaIN / Snake coefficients are one set per tile;
//   * the raw x rows of the tile's own frames (the residual) are kept in a second per-wave LDS buffer.
// With two waves per SIMD (C = 32: 8 waves), one wave's transform / epilogue overlaps the other's MFMAs
// without any hand-placed schedule.  bf16 storage, v_mfma_f32_32x32x16_bf16, fp32 accumulation.
#include "common.h"
#include "conv_common.h"
#include "kernels.h"

namespace {

// MODE: 0 statistics of conv1's output, 1 fused (x' + its statistics), 2 fused into the running sum
template <int C, int K, int DIL, int NW, int MODE>
struct RI {
  static constexpr bool FUSED = MODE != 0;
  static constexpr int NCB = C / 32;                 // 32-channel blocks: output blocks = input chunks
  static constexpr int U = C / 8;                    // 16-B units per frame row
  static constexpr int ROWB = C * 2;                 // bytes per frame row (bf16)
  static constexpr int TQ = 64;                      // output frames per wave tile
  static constexpr int P1 = DIL * (K - 1) / 2, P2 = (K - 1) / 2;
  static constexpr int M1 = FUSED ? 3 : 2;           // conv1 row blocks (fused: the tile + conv2's halo)
  // window rows that valid outputs need; window row 0 is global frame q0 - OFF1
  static constexpr int R1 = FUSED ? TQ + (K - 1) * (DIL + 1) : TQ + (K - 1) * DIL;
  static constexpr int OFF1 = FUSED ? P1 + P2 : P1;
  static constexpr int RPI = 64 / U;                 // rows per 64-lane load (1 KB)
  static constexpr int NJ = (R1 + RPI - 1) / RPI;    // 16-B window units per lane
  static constexpr int RW = NJ * RPI;
  static constexpr int BR = (FUSED && RW < 32 * M1) ? 32 * M1 : RW;  // buffer rows per wave
  static constexpr int BUFB = BR * ROWB;
  // conv1's discarded rows (fused: past TQ + 2 P2) read up to row 32 M1 - 1 + (K - 1) DIL: slack past the
  // last wave's buffer (the other waves' reads land in the next buffer: garbage that no kept row uses)
  static constexpr int SLACKB = (32 * M1 + (K - 1) * DIL > BR ? 32 * M1 + (K - 1) * DIL - BR : 0) * ROWB;
  static constexpr int WB = NCB * K * C * 64;        // one layer's packed weights
  static constexpr int NCF = FUSED ? 10 : 5;         // coefficient rows per wave: [layer][5][C]
  static constexpr int OFF_W1 = 0;
  static constexpr int OFF_W2 = WB;
  static constexpr int OFF_CF = OFF_W2 + (FUSED ? WB : 0);
  static constexpr int OFF_BIAS = OFF_CF + NW * NCF * C * 4;
  static constexpr int OFF_X = (OFF_BIAS + 2 * C * 4 + 1023) / 1024 * 1024;
  static constexpr int OFF_RES = OFF_X + NW * BUFB + SLACKB;  // [NW][TQ rows][ROWB]: raw x of the tile's frames
  static constexpr int LDS = OFF_RES + (FUSED ? NW * TQ * ROWB : 0);
  static_assert(2 * P2 <= 32, "conv2 halo within the third conv1 block");
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static_assert(U == 4 || U == 8, "C = 32 / 64");
};

// physical 16-B unit of logical unit u in window row r (C = 32: 4 units per 64-B row; C = 64: 8 per 128 B)
template <int U>
__device__ __forceinline__ int wswz(int r, int u) {
  return U == 4 ? (u ^ ((r >> 2) & 3)) : (u ^ ((r >> 1) & 7));
}

__device__ __forceinline__ void bf8v(const uint4& r, float (&v)[8]) {
  const unsigned w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 v8bf(const float* v) {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (bf16_t)v[j];
  uint4 r;
  __builtin_memcpy(&r, &o, 16);
  return r;
}

// AdaIN -> Snake coefficients of one channel (resconv.hip): y = fma(v, a, m1 + ia2) - ia2 cos(2 alpha x) with
// the cosine argument in revolutions fma(v, a alpha / pi, m1 alpha / pi), m1 = beta - mean a, ia2 = 1 / (2 alpha)
__device__ __forceinline__ void put_cf(const Prologue& pro, int b, int ci, float* cf, int C) {
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

// PFD: window prefetch distance in tiles (PFD register sets; the load of tile t + PFD is issued once tile t's
// window is in LDS)
template <int C, int K, int DIL, int NW, int MODE, int PFD>
__global__ void __launch_bounds__(64 * NW, NW / 4) k_resfused(const ResFusedParams p) {
  using G = RI<C, K, DIL, NW, MODE>;
  constexpr bool FUSED = G::FUSED, ACC = MODE == 2;
  constexpr int NCB = G::NCB, U = G::U, NJ = G::NJ, RPI = G::RPI, ROWB = G::ROWB, TQ = G::TQ;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hi = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int L = p.L;
  const int ntm = (L + TQ - 1) / TQ;
  const long long total = (long long)ntm * p.B;
  const long long nwt = (long long)gridDim.x * NW, gw = (long long)blockIdx.x * NW + wv;
  const int tbeg = (int)(total * gw / nwt), tend = (int)(total * (gw + 1) / nwt);

  // ---- the layers' packed weights and biases -> LDS, once per block (the only barrier)
  {
    const Rsrc r1 = make_rsrc(p.w1, (unsigned)G::WB);
    for (int u = tid; u < G::WB / 16; u += 64 * NW)
      *reinterpret_cast<uint4*>(smem + G::OFF_W1 + 16 * u) = bload16(r1, 16u * u);
    if constexpr (FUSED) {
      const Rsrc r2 = make_rsrc(p.w2, (unsigned)G::WB);
      for (int u = tid; u < G::WB / 16; u += 64 * NW)
        *reinterpret_cast<uint4*>(smem + G::OFF_W2 + 16 * u) = bload16(r2, 16u * u);
    }
    float* bs = reinterpret_cast<float*>(smem + G::OFF_BIAS);
    for (int i = tid; i < C; i += 64 * NW) {
      bs[i] = p.b1 ? p.b1[i] : 0.f;
      bs[C + i] = (FUSED && p.b2) ? p.b2[i] : 0.f;
    }
  }
  __syncthreads();
  if (tbeg >= tend) return;  // (per wave: no barrier follows)

  char* buf = smem + G::OFF_X + wv * G::BUFB;
  float* cf = reinterpret_cast<float*>(smem + G::OFF_CF) + wv * G::NCF * C;  // [layer][5][C]
  const float* bias = reinterpret_cast<const float*>(smem + G::OFF_BIAS);

  // ---- window loads: lane keeps logical unit ul of rows j * RPI + rl
  const int ul = lane & (U - 1), rl = lane / U;
  auto issue = [&](int t, uint4 (&pre)[NJ]) __attribute__((always_inline)) {
    const int b = t / ntm, mt = t - b * ntm;
    const Rsrc rx = make_rsrc(reinterpret_cast<const bf16_t*>(p.x) + (size_t)b * p.x_bs,
                              (unsigned)((size_t)L * p.x_ld * 2));
    const int gr0 = mt * TQ - G::OFF1;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int r = j * RPI + rl, g = gr0 + r;
      pre[j] = bload16(rx, (g >= 0 && r < G::R1 && !(p.dbg & 8)) ? (unsigned)(g * p.x_ld + 8 * ul) * 2u : OOB);
    }
  };
  // Snake1(AdaIN1(.)) of the window into the wave's buffer; rows outside [0, L) are conv1's zero padding
  // (fused: the raw rows of the tile's own frames also go to the wave's residual buffer, read by epilogue 2)
  char* resb = smem + G::OFF_RES + wv * TQ * ROWB;
  auto transform = [&](int t, uint4 (&pre)[NJ]) __attribute__((always_inline)) {
    const int gr0 = (t % ntm) * TQ - G::OFF1;
    if constexpr (FUSED) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int rr = j * RPI + rl - G::OFF1;
        if ((unsigned)rr < (unsigned)TQ) *reinterpret_cast<uint4*>(resb + rr * ROWB + 16 * wswz<U>(rr, ul)) = pre[j];
      }
    }
    // per 4-channel half, its coefficients (20 registers instead of 40 live)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float4 m2 = *reinterpret_cast<const float4*>(cf + 8 * ul + 4 * h);
      const float4 a = *reinterpret_cast<const float4*>(cf + C + 8 * ul + 4 * h);
      const float4 ar = *reinterpret_cast<const float4*>(cf + 2 * C + 8 * ul + 4 * h);
      const float4 mr = *reinterpret_cast<const float4*>(cf + 3 * C + 8 * ul + 4 * h);
      const float4 nia = *reinterpret_cast<const float4*>(cf + 4 * C + 8 * ul + 4 * h);
      const float cm2[4] = {m2.x, m2.y, m2.z, m2.w}, ca[4] = {a.x, a.y, a.z, a.w};
      const float car[4] = {ar.x, ar.y, ar.z, ar.w}, cmr[4] = {mr.x, mr.y, mr.z, mr.w};
      const float cni[4] = {nia.x, nia.y, nia.z, nia.w};
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        unsigned& w0 = h ? pre[j].z : pre[j].x;
        unsigned& w1 = h ? pre[j].w : pre[j].y;
        float v[4] = {__uint_as_float(w0 << 16), __uint_as_float(w0 & 0xffff0000u), __uint_as_float(w1 << 16),
                      __uint_as_float(w1 & 0xffff0000u)};
        if (!(p.dbg & 1)) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float x2 = __builtin_fmaf(v[e], ca[e], cm2[e]);
            const float c = __builtin_amdgcn_cosf(__builtin_fmaf(v[e], car[e], cmr[e]));
            v[e] = __builtin_fmaf(c, cni[e], x2);
          }
        }
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (bf16_t)v[e];
        uint2 ov;
        __builtin_memcpy(&ov, &o, 8);
        w0 = ov.x;
        w1 = ov.y;
      }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int r = j * RPI + rl;
      uint4 o = pre[j];
      if ((unsigned)(gr0 + r) >= (unsigned)L) o = make_uint4(0u, 0u, 0u, 0u);
      *reinterpret_cast<uint4*>(buf + r * ROWB + 16 * wswz<U>(r, ul)) = o;
    }
  };

  // ---- MFMA loop: acc[m][nb] += W[nb] x B rows (rb0 + 32 m + tap * dl), over (tap, chunk, k-half) steps,
  // the next step's fragments read before the current step's MFMAs
  const int swzw = (l32 >> 2) & 3;
  // acc[m][nb] (m < nm) for the row blocks m0 + m of the wave's buffer
  auto conv = [&](f32x16 (&acc)[2][NCB], const char* wbase, int m0, int nm, int dl) __attribute__((always_inline)) {
    constexpr int S = K * NCB * 2;
    auto rd = [&](int s, bf16x8 (&wa)[NCB], bf16x8 (&xb)[2]) __attribute__((always_inline)) {
      const int tap = s / (NCB * 2), c = (s >> 1) % NCB, kk = s & 1;
#pragma unroll
      for (int nb = 0; nb < NCB; ++nb)
        wa[nb] = *reinterpret_cast<const bf16x8*>(wbase + (((c * K + tap) * C + nb * 32 + l32) * 64) +
                                                  16 * ((2 * kk + hi) ^ swzw));
      // the window address from an opaque copy of the lane index, computed here at the step: hoisted out of
      // the tile loop, the K x 2 per-step addresses of both convs would stay live as registers
      int l = lane;
      asm volatile("" : "+v"(l));
      const int r0 = (l & 31) + tap * dl;  // (rows 32 m + r0 share the swizzle: 32 m leaves bits 1-3 alone)
      const char* xa = buf + (32 * m0 + r0) * ROWB + 16 * wswz<U>(r0, 4 * c + 2 * kk + (l >> 5));
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        if (m >= nm) continue;
        xb[m] = *reinterpret_cast<const bf16x8*>(xa + 32 * m * ROWB);
      }
    };
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int nb = 0; nb < NCB; ++nb)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[m][nb][r] = 0.f;
    if (p.dbg & 2) return;
    bf16x8 wa[2][NCB], xb[2][2];
    rd(0, wa[0], xb[0]);
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int cb = s & 1;
      if (s + 1 < S) rd(s + 1, wa[cb ^ 1], xb[cb ^ 1]);
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        if (m >= nm) continue;
#pragma unroll
        for (int nb = 0; nb < NCB; ++nb)
          acc[m][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[cb][nb], xb[cb][m], acc[m][nb], 0, 0, 0);
      }
    }
  };

  // ---- statistics: per-lane sums of the lane's 16 channels per block, reduced when the wave leaves an
  // utterance (reduce-scatter over the 32 lanes of a half: lane l32 ends with channel 16 hi + l32 / 2)
  const bool want_stats = !ACC && p.stats != nullptr;
  float st_s[NCB][16], st_q[NCB][16];
#pragma unroll
  for (int nb = 0; nb < NCB; ++nb)
#pragma unroll
    for (int r = 0; r < 16; ++r) st_s[nb][r] = st_q[nb][r] = 0.f;
  auto flush = [&](int b) __attribute__((always_inline)) {
    if (!want_stats) return;
    double* d = (p.stats_slots > 1 ? p.stats + (size_t)(blockIdx.x % p.stats_slots) * p.stats_slot_bs : p.stats) +
                (size_t)b * p.stats_ld * ST_W;
#pragma unroll
    for (int nb = 0; nb < NCB; ++nb) {
      const float s1 = rs16(st_s[nb], l32);
      const float s2 = rs16(st_q[nb], l32);
      const int ch = 32 * nb + 16 * hi + (l32 >> 1);
      fx_add(d + ST_W * ch + 2 * (l32 & 1), (l32 & 1) ? s2 : s1);
#pragma unroll
      for (int r = 0; r < 16; ++r) st_s[nb][r] = st_q[nb][r] = 0.f;
    }
  };
  auto acc_stats = [&](int nb, const float (&v)[16], bool valid) __attribute__((always_inline)) {
    const float mk = valid ? 1.f : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float x = v[r] * mk;
      st_s[nb][r] += x;
      st_q[nb][r] = __builtin_fmaf(x, x, st_q[nb][r]);
    }
  };

  const float adiv = (ACC && p.acc_div != 0.f) ? 1.0f / p.acc_div : 1.0f;
  auto step = [&](int t, uint4 (&pre)[NJ]) __attribute__((always_inline)) {
    const int b = t / ntm, mt = t - b * ntm;
    const int q0 = mt * TQ;
    transform(t, pre);
    // the tile's residual / running-sum rows (lane: frame q0 + 32 m + l32, channels 32 nb + 16 hi ..), before
    // the window loads of tile t + 2 so that their wait does not also wait for those
    uint4 racc[ACC ? 2 : 1][NCB][2];
    if constexpr (ACC) {
      const Rsrc ra = make_rsrc(reinterpret_cast<const bf16_t*>(p.accb) + (size_t)b * p.acc_bs,
                                (unsigned)((size_t)L * p.acc_ld * 2));
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int nb = 0; nb < NCB; ++nb) {
          const int q = q0 + 32 * m + l32, co = 32 * nb + 16 * hi;
          const unsigned ea = (unsigned)(q * p.acc_ld + co) * 2u;
          racc[m][nb][0] = bload16(ra, ea);
          racc[m][nb][1] = bload16(ra, ea + 16u);
        }
    }
    if (t + PFD < tend) issue(t + PFD, pre);

    f32x16 acc[2][NCB];
    if constexpr (!FUSED) {  // statistics of conv1 + bias over the tile's frames
      conv(acc, smem + G::OFF_W1, 0, 2, DIL);
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const bool valid = q0 + 32 * m + l32 < L;
#pragma unroll
        for (int nb = 0; nb < NCB; ++nb) {
          float v[16], bb[16];
          ld8_lds(bias + 32 * nb + 16 * hi, *reinterpret_cast<float(*)[8]>(&bb[0]));
          ld8_lds(bias + 32 * nb + 16 * hi + 8, *reinterpret_cast<float(*)[8]>(&bb[8]));
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = acc[m][nb][r] + bb[r];
          if (want_stats) acc_stats(nb, v, valid);
        }
      }
      return;
    } else {
      // ---- conv1 in two phases (row blocks 0-1, then block 2: conv2's far halo), each followed by
      // epilogue 1: + bias1 -> AdaIN2 -> Snake2 -> bf16, in place over the window rows of its blocks (block 2's
      // conv1 reads rows >= 64 only; a block's own reads have retired: its accumulators consumed them); rows
      // outside [0, L) are conv2's zero padding
      auto epi1 = [&](f32x16 (&a1)[2][NCB], int m0, int nm) __attribute__((always_inline)) {
#pragma unroll
        for (int nb = 0; nb < NCB; ++nb)
#pragma unroll
          for (int qd = 0; qd < 4; ++qd) {  // 4-channel quarters of the lane's 16 channels
            const int ch = 32 * nb + 16 * hi + 4 * qd;
            const float4 bb = *reinterpret_cast<const float4*>(bias + ch);
            const float4 m2 = *reinterpret_cast<const float4*>(cf + 5 * C + ch);
            const float4 a = *reinterpret_cast<const float4*>(cf + 6 * C + ch);
            const float4 ar = *reinterpret_cast<const float4*>(cf + 7 * C + ch);
            const float4 mr = *reinterpret_cast<const float4*>(cf + 8 * C + ch);
            const float4 nia = *reinterpret_cast<const float4*>(cf + 9 * C + ch);
            const float cb[4] = {bb.x, bb.y, bb.z, bb.w}, cm2[4] = {m2.x, m2.y, m2.z, m2.w};
            const float ca[4] = {a.x, a.y, a.z, a.w}, car[4] = {ar.x, ar.y, ar.z, ar.w};
            const float cmr[4] = {mr.x, mr.y, mr.z, mr.w}, cni[4] = {nia.x, nia.y, nia.z, nia.w};
#pragma unroll
            for (int m = 0; m < 2; ++m) {
              if (m >= nm) continue;
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                float v = a1[m][nb][4 * qd + e] + cb[e];
                if (!(p.dbg & 1)) {
                  const float x2 = __builtin_fmaf(v, ca[e], cm2[e]);
                  const float c = __builtin_amdgcn_cosf(__builtin_fmaf(v, car[e], cmr[e]));
                  v = __builtin_fmaf(c, cni[e], x2);
                }
                a1[m][nb][4 * qd + e] = v;
              }
            }
          }
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          if (m >= nm) continue;
          const int r = 32 * (m0 + m) + l32;
          const bool in = (unsigned)(q0 - G::P2 + r) < (unsigned)L;
#pragma unroll
          for (int nb = 0; nb < NCB; ++nb)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              float v[8];
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] = a1[m][nb][8 * h + j];
              uint4 o = v8bf(v);
              if (!in) o = make_uint4(0u, 0u, 0u, 0u);
              *reinterpret_cast<uint4*>(buf + r * ROWB + 16 * wswz<U>(r, 4 * nb + 2 * hi + h)) = o;
            }
        }
      };
      conv(acc, smem + G::OFF_W1, 0, 2, DIL);
      epi1(acc, 0, 2);
      conv(acc, smem + G::OFF_W1, 2, 1, DIL);
      epi1(acc, 2, 1);
      // ---- conv2 over the tile's two output blocks
      f32x16 (&acc2)[2][NCB] = acc;
      conv(acc2, smem + G::OFF_W2, 0, 2, 1);
      // ---- epilogue 2: + bias2 + x [-> running sum] -> y, statistics
      bf16_t* yb = reinterpret_cast<bf16_t*>(p.y) + (size_t)b * p.y_bs;
      const Rsrc ry = make_rsrc(yb, (unsigned)((size_t)L * p.y_ld * 2));
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int q = q0 + 32 * m + l32;
        const bool valid = q < L;
#pragma unroll
        for (int nb = 0; nb < NCB; ++nb)
#pragma unroll
          for (int h = 0; h < 2; ++h) {  // 8 channels at a time
            const int co = 32 * nb + 16 * hi + 8 * h;
            float v[8], bb[8], r0[8];
            ld8_lds(bias + C + co, bb);
            const int rr = 32 * m + l32;
            bf8v(*reinterpret_cast<const uint4*>(resb + rr * ROWB + 16 * wswz<U>(rr, 4 * nb + 2 * hi + h)), r0);
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] = acc2[m][nb][8 * h + r] + bb[r] + r0[r];
            if constexpr (ACC) {
              bf8v(racc[m][nb][h], r0);
#pragma unroll
              for (int r = 0; r < 8; ++r) v[r] = (r0[r] + v[r]) * adiv;
            }
            const unsigned ey = (valid && !(p.dbg & 4)) ? (unsigned)(q * p.y_ld + co) * 2u : OOB;
            bstore16(ry, ey, v8bf(v));
            if (want_stats) {
              const float mk = valid ? 1.f : 0.f;
#pragma unroll
              for (int r = 0; r < 8; ++r) {
                const float x = v[r] * mk;
                st_s[nb][8 * h + r] += x;
                st_q[nb][8 * h + r] = __builtin_fmaf(x, x, st_q[nb][8 * h + r]);
              }
            }
          }
      }
    }
  };

  auto set_cf = [&](int b) __attribute__((always_inline)) {
    for (int ci = lane; ci < C; ci += 64) {
      put_cf(p.pro1, b, ci, cf, C);
      if constexpr (FUSED) put_cf(p.pro2, b, ci, cf + 5 * C, C);
    }
  };
  // the wave's tiles, one utterance segment at a time (its coefficients at the start, its statistics flushed
  // at the end: one copy of each in the code); the tiles alternate between the two register sets, tile t of a
  // segment always in preA (an odd segment swaps the sets for the next one)
  // PFD register sets; set k holds tiles k, k + PFD, ... of a segment (a segment that ends after r < PFD tiles
  // of its last group rotates the sets by r, once)
  uint4 pre[PFD][NJ];
#pragma unroll
  for (int k = 0; k < PFD; ++k)
    if (tbeg + k < tend) issue(tbeg + k, pre[k]);
  auto rotate = [&](int r) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      uint4 v[PFD];
#pragma unroll
      for (int k = 0; k < PFD; ++k) v[k] = pre[k][j];
#pragma unroll
      for (int k = 0; k < PFD; ++k) pre[k][j] = v[(k + r) % PFD];
    }
  };
  int t = tbeg;
  while (t < tend) {
    const int b = t / ntm;
    const int t1 = (b + 1) * ntm < tend ? (b + 1) * ntm : tend;
    set_cf(b);
    bool more = true;
    while (more) {
#pragma unroll
      for (int k = 0; k < PFD; ++k) {
        step(t, pre[k]);
        if (++t == t1) {
          if (k + 1 < PFD) rotate(k + 1);
          more = false;
          break;
        }
      }
    }
    flush(b);
  }
}

int g_num_cu_ri = 0;

template <int C, int K, int DIL, int MODE>
int launch_ri(const ResFusedParams& p, hipStream_t stream) {
  // C = 32: two waves per SIMD (one wave transforms / stores while the other issues MFMAs); C = 64: one
  // (its register sets and both layers' weights leave room for four waves per CU)
  constexpr int NW = C == 32 ? 8 : 4;
  using G = RI<C, K, DIL, NW, MODE>;
  // window prefetch distance: the statistics pass holds three tiles of loads in flight, the fused pass two
  // (one at K = 11, whose longer tiles cover more of the latency; its registers are the limit)
  constexpr int PFD = MODE == 0 ? 3 : (K == 11 ? 1 : 2);
  auto kern = k_resfused<C, K, DIL, NW, MODE, PFD>;
  static bool attr = false;
  if (!attr) {
    ST_CHECK_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
    attr = true;
  }
  if (!g_num_cu_ri) {
    int dev = 0;
    ST_CHECK_HIP(hipGetDevice(&dev));
    ST_CHECK_HIP(hipDeviceGetAttribute(&g_num_cu_ri, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const long long tiles = (long long)((p.L + G::TQ - 1) / G::TQ) * p.B;
  long long grid = g_num_cu_ri;  // one block per CU
  if (grid * NW > tiles) grid = (tiles + NW - 1) / NW;
  if (g_opt_grid_cap > 0 && grid > g_opt_grid_cap) grid = g_opt_grid_cap;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * NW), G::LDS, stream, p);
  return (int)hipGetLastError();
}

template <int C, int K, int DIL>
int launch_ri_m(const ResFusedParams& p, hipStream_t s) {
  if (p.stats_only) return launch_ri<C, K, DIL, 0>(p, s);
  return p.accb ? launch_ri<C, K, DIL, 2>(p, s) : launch_ri<C, K, DIL, 1>(p, s);
}
template <int C, int K>
int launch_ri_d(const ResFusedParams& p, hipStream_t s) {
  switch (p.dil) {
    case 1: return launch_ri_m<C, K, 1>(p, s);
    case 3: return launch_ri_m<C, K, 3>(p, s);
    case 5: return launch_ri_m<C, K, 5>(p, s);
    default: return ST_EINVAL;
  }
}

}  // namespace

bool st_resfused_eligible(int C, int K, int dil, int dtype) {
  if (!g_opt_resfused || dtype != ST_BF16) return false;
  if (!(dil == 1 || dil == 3 || dil == 5)) return false;
  // (C = 64 needs one wave per SIMD here: measured slower than the unfused resconv pair, not routed)
  return C == 32 && (K == 3 || K == 7 || K == 11);
}

int st_resfused(const ResFusedParams& pin, hipStream_t stream) {
  if (pin.B <= 0 || pin.L <= 0) return ST_OK;
  ResFusedParams p = pin;
  p.dbg = g_opt_debug;
  if (!st_resfused_eligible(p.C, p.K, p.dil, ST_BF16)) return ST_EINVAL;
  if (p.x_ld % 8 || (!p.stats_only && p.y_ld % 8) || (p.accb && (p.acc_ld % 8 || p.stats))) return ST_EINVAL;
  if (!p.pro1.stats || !p.pro1.gamma || !p.pro1.alpha) return ST_EINVAL;
  if (!p.stats_only && (!p.y || !p.pro2.stats || !p.pro2.gamma || !p.pro2.alpha)) return ST_EINVAL;
  if (p.stats_only && !p.stats) return ST_EINVAL;
  if (p.C == 32) {
    switch (p.K) {
      case 3: return launch_ri_d<32, 3>(p, stream);
      case 7: return launch_ri_d<32, 7>(p, stream);
      case 11: return launch_ri_d<32, 11>(p, stream);
    }
  } else if (p.C == 64 && p.K == 3) {
    return launch_ri_d<64, 3>(p, stream);
  }
  return ST_EINVAL;
}
