// Resblock conv engine v2 for the wide generator stages (C = 128 / 256; MFMA-bound): the dilated
// Conv1d(C, C, K, dilation d, padding d(K-1)/2) of every AdaINResBlock1 iteration
// (Modules/hifigan.py:26-80, forward :65-74) with the AdaIN -> Snake prologue and the bias /
// residual / resblock-average / InstanceNorm-statistics epilogue fused.  bf16 storage,
// v_mfma_f32_32x32x16_bf16, fp32 accumulation.
//
// Why a v2: v1 staged weights and windows through registers shared by all 8 waves,
// so every step needed a workgroup barrier, 256 VGPRs held staging copies, and the measured
// phases (MFMA issue, weight staging, window staging) added up instead of overlapping.
//
// Layout of the work:
//   * 8 waves; wave w owns 32 output channels (co block w % (C/32)) x 256 frames (frame half
//     w / (C/32)): a tile is 256 (C = 256) or 512 (C = 128) frames x C channels, 128 fp32
//     accumulator registers per lane.  Weight bytes are not duplicated across waves.
//   * Weights: each wave streams ITS OWN 2 KB slice per step (32 co x 32 ci of one tap, the
//     packed layout's contiguous block, already XOR-swizzled at pack time) by LDS-DMA into a
//     private 3-slot ring, two steps ahead.  A wave waits only on its own vmcnt: no barrier.
//   * Window: the raw bf16 window of the next 32-channel group (tile rows + halo) is LDS-DMA'd
//     into the other half of a 2-buffer ring at the start of a group, and transformed IN PLACE
//     (AdaIN -> Snake -> bf16, zero outside the utterance) by the lane that DMA'd it (so only
//     that wave's vmcnt orders it), during the group's last tap.  One raw s_barrier per group
//     (K steps) publishes it; DMAs stay in flight across it (counted vmcnt, never 0 in the loop).
//   * Epilogue per tile from the accumulators: + residual, * out_scale, resblock average,
//     bf16 stores, per-lane statistics reduced across the wave and added into LDS, flushed to
//     the fp64 statistics when the workgroup leaves an utterance.
//
// SP (the split-operand accuracy mode, STTS_SPLIT): fp32 activations, every operand v = hi + lo
// with hi = bf16(v), lo = bf16(v - hi), products W_hi X_hi + W_lo X_hi + W_hi X_lo on the same MFMA.  A group
// is then 16 input channels instead of 32, and every LDS image keeps its byte layout: a window row holds
// [X_hi 0-7 | X_hi 8-15 | X_lo 0-7 | X_lo 8-15] where the bf16 kernel holds channels 0-31 (the raw fp32 window
// of 16 channels is the same 64 B a row, transformed in place into its hi / lo halves), and a weight slot
// [W_hi | W_lo] of 16 input channels where the bf16 kernel holds 32 (gathered by the LDS-DMA from the packed
// hi and lo copies).  So the fragment reads, the DMA counts and the LDS budget are the bf16 kernel's; a tap
// issues 24 MFMAs on the same 2 weight + 16 window fragments instead of 16, and the epilogue stores fp32.
#include "common.h"
#include "conv_common.h"
#include "kernels.h"
#include "lds_dma.h"

namespace {


// UPS: the polyphase ConvTranspose1d upsampler (hifigan.py:292-294, 333-335) as the 2-tap GEMM of
// C = N = u Cout columns, tap t reads input row q + t - 1 (left pad 1); the epilogue maps GEMM
// row q / column n to output frame q u + n / Cout - opad, channel n % Cout.
// CO: channels of the bias / statistics arrays (C; Cout for UPS)
// OFS: the second half of the waves (wu >= NW / 2) runs one group behind the first (3 window buffers), so the
// two waves of each SIMD reach their tile epilogues one group apart and one's epilogue runs beside the other's
// MFMAs (STTS_OPT_BIGCONV 5 / 6)
// LA: window lookahead 2 (3 window buffers): slot sl DMAs window sl + 2 instead of sl + 1, so a window lands a whole
// group (K taps) before its transform instead of K - 1 or K - 2 taps.  For K <= 3 those 1-2 taps (~1.5 us) are
// about one LDS-DMA latency under load, so the transform waited on the DMA (STTS_OPT_BIGLA)
// NF: 32-frame accumulator fragments per wave (8: 256 frames; 4: 128 frames, for C = 64, whose two 32-channel
// output blocks leave 4 frame slices per 8-wave tile: 512-frame windows instead of 1,024)
template <int C, int NW, int K, int DIL, int PRO = PK_SNAKE, int CINP = C, bool UPS = false, int CO = C, bool OFS = false,
          bool LA = false, int NF = 8, int NCB = 0>
struct B2 {
  static_assert(NF == 8 || NF == 4 || NF == 2, "fragments per wave");
  static_assert(!(OFS && LA), "one use of the third window buffer");
  static constexpr int NXB = (OFS || LA) ? 3 : 2;  // window buffers
  static constexpr int NCOEF = PRO == PK_SNAKE ? 5 : 2;  // coefficient rows per input channel
  // 32-channel output blocks per block tile (NCB: a smaller count, for column counts no power of two divides: ups[2])
  static constexpr int NCBW = NCB ? NCB : ((C / 32 < NW) ? C / 32 : NW);
  static constexpr int FH = NW / NCBW;   // frame halves per tile (waves per co block)
  static constexpr int NCO = 32 * NCBW;  // output channels per tile
  static constexpr int NCH = C / NCO;    // output-channel parts per frame tile (tiles per frame range)
  static constexpr int TM = 32 * NF * FH;  // tile rows (frames)
  // UPS tiles whose NCO columns span several output phases (ups[2] on 12-wave blocks: 192 = 3 x 64): the statistics
  // words of a channel then get one copy per phase too (one writer per word: deterministic sums)
  static constexpr int NPH = (UPS && NCO > CO) ? NCO / CO : 1;
  static constexpr int NG = CINP / 32;   // 32-channel input groups per tile (at most)
  static constexpr int PAD = UPS ? DIL * (K - 1) : DIL * (K - 1) / 2;
  static constexpr int R = TM + DIL * (K - 1);                    // window rows a group needs
  static constexpr int NWIN = (R * 4 + 64 * NW - 1) / (64 * NW);  // window DMA instructions per wave per group
  static constexpr int WROWS = NWIN * NW * 16;                    // rows the waves' DMAs cover
  // weight prefetch distance (steps): as deep as the LDS allows, up to K (the waits below assume a
  // target at most one group back) and 5.  It is also what covers the window DMA: vmcnt retires in
  // issue order, so the first wait for a weight slice issued after a group's window DMA (PD taps
  // later) also waits for that window (a DMA lands ~1.1 us after issue, MI355X_MICROARCH.md
  // ldsdma-fill, later from HBM under load; a tap is ~0.5 us of MFMA issue per SIMD)
  static constexpr int OFF_COEF = 0;                  // [2][NCOEF][CINP] f32 (utterance parity)
  static constexpr int OFF_BIAS = OFF_COEF + 2 * NCOEF * CINP * 4;
  // [FH][CO][2] f32: one copy per frame half, one writer per word, added in a fixed order by the flush
  // (deterministic statistics, common.h ST_W)
  static constexpr int OFF_ST = OFF_BIAS + CO * 4;
  static constexpr int OFF_W = (OFF_ST + FH * NPH * 2 * CO * 4 + 1023) / 1024 * 1024;  // [NW waves][RS][2 KB]
  static constexpr int BPC = NW == 4 ? 2 : 1;                     // blocks per CU
  static constexpr int PDMAX_LDS = ((160 * 1024 / BPC - OFF_W - NXB * WROWS * 64) / (NW * 2048)) - 1;
  static constexpr int PD0 = PDMAX_LDS < K ? PDMAX_LDS : K;
  static constexpr int PD = PD0 < 5 ? PD0 : 5, RS = PD + 1;
  static constexpr int OFF_X = OFF_W + NW * RS * 2048; // [NXB][WROWS][64 B]
  static constexpr int LDS = OFF_X + NXB * WROWS * 64;
  static_assert(FH * NCBW == NW && NCH * NCO == C, "wave grid");
  static_assert(!UPS || NCO <= CO || (NCO % CO == 0 && NCH == 1), "one writer per statistics word and tile");
  static_assert(NW == 4 || NW == 8 || (NW == 12 && UPS), "wave counts (12: the N = 192 upsampler)");
  static_assert(LDS * BPC <= 160 * 1024, "LDS budget");
  static_assert(K >= PD && PD >= 2, "weight prefetch stays within one group");
  static_assert(OFF_W % 1024 == 0 && OFF_X % 1024 == 0, "DMA bases");
};

// SEG: several tile ranges per workgroup (segmented partition, p.seg > 0, with fewer workgroups than segments); the
// plain instantiation runs the one-range code (a range loop in every launch measured ~0.5 % of the step)
template <int C, int NW, int K, int DIL, bool RES, bool ACC, int PRO = PK_SNAKE, int CINP = C, bool EPI1 = false,
          bool UPS = false, int CO = C, bool OFS = false, bool SP = false, bool LA = false, int NF = 8, int NCB = 0,
          bool SEG = false>
__global__ void __launch_bounds__(64 * NW, NW == 12 ? 3 : 2) k_bigconv2(const ConvParams p) {
  using G = B2<C, NW, K, DIL, PRO, CINP, UPS, CO, OFS, LA, NF, NCB>;
  constexpr int FW = 32 * NF;  // frames per wave
  constexpr int NXB = G::NXB;
  constexpr int TM = G::TM, NWIN = G::NWIN, PD = G::PD, RS = G::RS, NCH = G::NCH, NCO = G::NCO;
  constexpr int NCF = G::NCOEF;
  // input-channel groups: C / 32 for the square resblock convs, ceil(Cin / 32) for the front-end
  // (SP: 16-channel groups)
  constexpr int GW = SP ? 16 : 32;
  const int NG = (PRO == PK_SNAKE && CINP == C) ? C / GW : (p.Cin + GW - 1) / GW;
  constexpr int NT = 64 * NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* coef = reinterpret_cast<float*>(smem + G::OFF_COEF);
  float* bias_s = reinterpret_cast<float*>(smem + G::OFF_BIAS);
  float* st_lds = reinterpret_cast<float*>(smem + G::OFF_ST);

  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hi = lane >> 5;
  const int wu = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave index, provably uniform
  const int cb = wu % G::NCBW, fh = wu / G::NCBW;
  const int ntm = (p.Lq + TM - 1) / TM;
  // tile t -> utterance t / (NCH ntm), output-channel part (t / ntm) % NCH, frame tile t % ntm
  const long long total = (long long)ntm * NCH * p.B;
  const int upb = ntm * NCH;  // tiles per utterance
  // tile ranges (kernels.h tile_range: one per workgroup, or utterance-relative segments)
  const int nv = SEG ? tile_nv(p, p.B) : (int)gridDim.x;
  for (int vb = blockIdx.x; vb < nv; vb += gridDim.x) {
  long long tb_, te_;
  if constexpr (SEG) {
    tile_range(p, vb, nv, total, upb, tb_, te_);
  } else {
    tb_ = total * vb / gridDim.x;
    te_ = total * (vb + 1) / gridDim.x;
  }
  const int tbeg = (int)tb_, tend = (int)te_;
  if (tbeg >= tend) continue;  // uniform over the block
  const int NGG = (tend - tbeg) * NG;  // groups this block walks
  const bool want_stats = !ACC && p.stats != nullptr;
  // STTS_OPT_DEBUG phase skipping (timing attribution only; outputs are wrong while set):
  // 1 transform, 4 epilogue, 8 weight DMAs, 16 window DMAs, 32 group barrier, 128 epilogue stores,
  // 256 epilogue statistics (2, MFMAs, is not
  // honoured: a runtime branch around the pipelined taps keeps their fragments live everywhere)
  const int dbg = p.dbg;
  // diagnostics (dbg bit 64 + a debug buffer): per-wave s_memtime sums of the phases below
  const bool stamp = (dbg & 64) && p.stamps;
  // slots: 0 weight wait, 1 window wait, 2 barrier, 3 transform, 4 epilogue tail, 5 total, 6 the rest
  // (MFMA issue), 7 epilogue vmcnt(0), 8 epilogue loads + finish + stores, 9 epilogue statistics
  unsigned long long st_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long t_mark = stamp ? __builtin_amdgcn_s_memtime() : 0;
  auto lap = [&](int k) __attribute__((always_inline)) {
    if (stamp) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      st_acc[k] += t - t_mark;
      t_mark = t;
    }
  };
  const unsigned long long t_start = t_mark;

  // STTS_OPT_SKEW: half the workgroups start |skew| x 1024 cycles late (odd ones for skew > 0, the
  // second half of the grid for skew < 0), so that two workgroups sharing a CU run out of phase
  if (p.skew != 0 && (p.skew > 0 ? (blockIdx.x & 1) != 0 : blockIdx.x >= gridDim.x / 2)) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long d = (unsigned long long)(p.skew > 0 ? p.skew : -p.skew) * 1024ull;
    while (__builtin_amdgcn_s_memtime() - t0 < d) __builtin_amdgcn_s_sleep(8);
  }
  for (int i = tid; i < CO; i += NT) bias_s[i] = p.bias ? p.bias[i] : 0.f;
  for (int i = tid; i < G::FH * G::NPH * 2 * CO; i += NT) st_lds[i] = 0.f;

  // ---------------- weights: step s = (group, tap) -> this wave's 2 KB slice, slot s % RS
  char* wring = smem + G::OFF_W + wu * RS * 2048;
  // (SP: the packed hi copy, then the lo copy, each of p.nchunks 32-channel chunks)
  const unsigned wcopy = SP ? (unsigned)((size_t)p.nchunks * K * C * 32 * 2) : 0u;
  const Rsrc rw = make_rsrc(p.w, SP ? 2u * wcopy : (unsigned)((size_t)NG * K * C * 32 * 2));
  // (group index gi, output part ch and tap t of the step: from the group cursors below, so no
  // runtime division by the group count runs per step)
  auto issue_w = [&](int s, int gi, int ch, int t) __attribute__((always_inline)) {
    if (dbg & 8) return;
    char* dst = wring + (s % RS) * 2048;
    if constexpr (SP) {
      // slot byte P = lane's 16 B of half hf: row n = P / 64 (output channel 32 cb + n of part ch), physical
      // unit P / 16 % 4 = logical unit lu ^ sw (sw = (n >> 2) & 3, the packed layout's own swizzle), logical
      // unit lu = [hi 0-7, hi 8-15, lo 0-7, lo 8-15] of the group's 16 channels: 32-channel chunk gi / 2,
      // logical unit 2 (gi & 1) + (lu & 1) of the packed row in copy lu / 2
      const int c32 = gi >> 1, h16 = gi & 1;
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const int n = hf * 16 + (lane >> 2), sw = (n >> 2) & 3, lu = (lane & 3) ^ sw;
        const int pu = (2 * h16 + (lu & 1)) ^ sw;
        const unsigned off = ((lu >> 1) ? wcopy : 0u) +
                             (unsigned)((((size_t)c32 * K + t) * C + ch * NCO + 32 * cb + n) * 64 + pu * 16);
        glds16(rw, dst + hf * 1024, off);
      }
    } else {
      const unsigned base = (unsigned)((((size_t)gi * K + t) * C + ch * NCO + 32 * cb) * 64) + lane * 16;
      glds16(rw, dst, base);
      glds16(rw, dst + 1024, base + 1024);
    }
  };

  // ---------------- window: group gg -> raw rows [gr0, gr0 + WROWS) of its 32 channels, buffer gg & 1
  // LDS unit pidx = row * 4 + u' holds logical 16-B unit u = u' ^ ((row >> 2) & 3) of that row
  auto issue_x = [&](int gg, int gi, int b, int mt) __attribute__((always_inline)) {
    if (dbg & 16) return;
    constexpr unsigned ES = SP ? 4u : 2u;  // element bytes (SP: fp32 frames, 4 channels a 16-B unit)
    const Rsrc rx = make_rsrc(reinterpret_cast<const char*>(p.x) + (size_t)b * p.x_bs * ES,
                              (unsigned)((size_t)p.Lin * p.x_ld * ES));
    const int gr0 = mt * TM - G::PAD;
    char* dst = smem + G::OFF_X + (gg % NXB) * (G::WROWS * 64);
#pragma unroll
    for (int j = 0; j < NWIN; ++j) {
      const int pidx = (j * NW + wu) * 64 + lane;
      const int r = pidx >> 2, u = (pidx & 3) ^ ((r >> 2) & 3);
      const int e = (gr0 + r) * p.x_ld + gi * GW + (16 / (int)ES) * u;
      // rows past the window (WROWS rounds R up to whole DMA instructions) read out of range: no
      // HBM traffic for them (profiles/r02_pmc_bigconv.txt measured 1.5x the window bytes)
      glds16(rx, dst + (j * NW + wu) * 1024, (e >= 0 && r < G::R) ? (unsigned)e * ES : OOB);
    }
  };
  // AdaIN + Snake coefficients of utterance b into parity slot b & 1 (see bigconv.hip)
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
  // in-place transform of the units this lane DMA'd for group gg: x -> AdaIN -> Snake -> bf16
  // (Snake via sin^2(u) = (1 - cos 2u) / 2 on the hardware cosine, as resconv.hip), 0 outside [0, Lin)
  const int my_u = (lane & 3) ^ ((lane >> 4) & 3);  // the lane's logical unit: the same in every row it owns
  // The lane's NWIN units are read first (one LDS latency), transformed per 4-channel half with
  // that half's coefficients, and written back with one 16-B store each.  Padding rows past R
  // are transformed too (their DMA read zeros; no tap reads them): no per-unit branch.
  auto transform = [&](int gg, int gi, int b, int mt, int ja = 0, int jb = G::NWIN) __attribute__((always_inline)) {
    if (dbg & 1) return;
    const int gr0 = mt * TM - G::PAD;
    char* buf = smem + G::OFF_X + (gg % NXB) * (G::WROWS * 64);
    if constexpr (SP) {
      // the lane's unit holds fp32 channels 4 my_u .. 4 my_u + 3 of its row; after the prologue their hi parts go
      // to logical unit my_u / 2 and their lo parts to logical unit 2 + my_u / 2, at byte 8 (my_u & 1) of the unit
      // (the row's other three lanes write the rest of it: each lane reads its whole unit before the row's writes,
      // in program order of the one wave that owns the row)
      const int sw = (lane >> 4) & 3;  // the row's swizzle, (r >> 2) & 3 for every row this lane owns
      const unsigned o_hi = (unsigned)((((my_u >> 1) ^ sw) * 16) + (my_u & 1) * 8 - (lane & 3) * 16);
      const unsigned o_lo = (unsigned)((((2 + (my_u >> 1)) ^ sw) * 16) + (my_u & 1) * 8 - (lane & 3) * 16);
      const float* cf = coef + (b & 1) * NCF * CINP + gi * 16 + 4 * my_u;
      if constexpr (PRO == PK_LRELU) {
        f32x4v m2, a;
        lds_coef2(lds_addr(cf), m2, a, (unsigned)(CINP * 4));
        const float am[4] = {m2.x, m2.y, m2.z, m2.w}, aa[4] = {a.x, a.y, a.z, a.w};
        const float slope = (p.pro.mode & PRO_LRELU) ? p.pro.slope : 1.0f;
        const int c0 = gi * 16 + 4 * my_u;
#pragma unroll
        for (int j = ja; j < jb; ++j) {
          const int pidx = (j * NW + wu) * 64 + lane;
          const int r = pidx >> 2;
          const unsigned ua = lds_addr(buf + pidx * 16);
          const float4 raw = *reinterpret_cast<const float4*>(buf + pidx * 16);
          float v[4] = {raw.x, raw.y, raw.z, raw.w};
          const bool pad = (unsigned)(gr0 + r) >= (unsigned)p.Lin;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float x2 = __builtin_fmaf(v[e], aa[e], am[e]);
            // channels >= Cin (the last group's padding, whose memory may hold anything) are forced to 0
            v[e] = (c0 + e < p.Cin && !pad) ? (x2 > 0.f ? x2 : x2 * slope) : 0.f;
          }
          float h[4], l[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            h[e] = (float)(bf16_t)v[e];
            l[e] = v[e] - h[e];
          }
          lds_write_b64(ua + o_hi, f32_to_bf4(h));
          lds_write_b64(ua + o_lo, f32_to_bf4(l));
        }
      } else {
        f32x4v m2, a, ar, mr, nia;
        lds_coef5(lds_addr(cf), m2, a, ar, mr, nia, (unsigned)(CINP * 4));
        const float am[4] = {m2.x, m2.y, m2.z, m2.w}, aa[4] = {a.x, a.y, a.z, a.w};
        const float aar[4] = {ar.x, ar.y, ar.z, ar.w}, amr[4] = {mr.x, mr.y, mr.z, mr.w};
        const float ani[4] = {nia.x, nia.y, nia.z, nia.w};
#pragma unroll
        for (int j = ja; j < jb; ++j) {
          const int pidx = (j * NW + wu) * 64 + lane;
          const int r = pidx >> 2;
          if (G::WROWS > G::R && r >= G::R) continue;  // padding rows: never read by a tap
          const unsigned ua = lds_addr(buf + pidx * 16);
          const float4 raw = *reinterpret_cast<const float4*>(buf + pidx * 16);
          float v[4] = {raw.x, raw.y, raw.z, raw.w};
          const bool pad = (unsigned)(gr0 + r) >= (unsigned)p.Lin;
          float h[4], l[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float x2 = __builtin_fmaf(v[e], aa[e], am[e]);
            const float c = __builtin_amdgcn_cosf(__builtin_fmaf(v[e], aar[e], amr[e]));
            const float y = pad ? 0.f : __builtin_fmaf(c, ani[e], x2);  // zero padding is post-prologue
            h[e] = (float)(bf16_t)y;
            l[e] = y - h[e];
          }
          lds_write_b64(ua + o_hi, f32_to_bf4(h));
          lds_write_b64(ua + o_lo, f32_to_bf4(l));
        }
      }
      return;
    }
    const float* cf = coef + (b & 1) * NCF * CINP + gi * 32 + 8 * my_u;
    if constexpr (PRO == PK_LRELU) {
    // (in chunks of at most 3 units: C = 128's 5 units at once spill)
    constexpr int JC = NWIN < 3 ? NWIN : 3;
#pragma unroll
    for (int j0 = 0; j0 < NWIN; j0 += JC) {
    uint4 raw[JC];
#pragma unroll
    for (int jj = 0; jj < JC; ++jj)
      if (j0 + jj < NWIN) raw[jj] = *reinterpret_cast<const uint4*>(buf + (((j0 + jj) * NW + wu) * 64 + lane) * 16);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      {
        f32x4v m2, a;
        lds_coef2(lds_addr(cf + 4 * h), m2, a, (unsigned)(CINP * 4));  // (its wait also covers raw[])
        const float am[4] = {m2.x, m2.y, m2.z, m2.w}, aa[4] = {a.x, a.y, a.z, a.w};
        const float slope = (p.pro.mode & PRO_LRELU) ? p.pro.slope : 1.0f;
        // channels >= Cin (the last group's padding, whose memory may hold anything, NaN
        // included) are forced to 0 rather than multiplied by 0
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
    // Snake: per unit (measured faster for the resblock convs than the batched form above, which
    // spills at C = 128)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      f32x4v m2, a, ar, mr, nia;
      lds_coef5(lds_addr(cf + 4 * h), m2, a, ar, mr, nia, (unsigned)(CINP * 4));
      const float am[4] = {m2.x, m2.y, m2.z, m2.w}, aa[4] = {a.x, a.y, a.z, a.w};
      const float aar[4] = {ar.x, ar.y, ar.z, ar.w}, amr[4] = {mr.x, mr.y, mr.z, mr.w};
      const float ani[4] = {nia.x, nia.y, nia.z, nia.w};
#pragma unroll
      for (int j = ja; j < jb; ++j) {
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

  // ---------------- statistics: LDS per-block sums -> fp64 global when the block leaves an utterance
  auto flush = [&](int b) __attribute__((always_inline)) {
    for (int ci = tid; ci < CO; ci += NT) {
      double* d = stats_slot(p, blockIdx.x) + ((size_t)b * p.stats_ld + ci) * ST_W;
      float a = 0.f, q = 0.f;
#pragma unroll
      for (int h = 0; h < G::FH * G::NPH; ++h) {
        a += st_lds[(h * CO + ci) * 2];
        q += st_lds[(h * CO + ci) * 2 + 1];
        st_lds[(h * CO + ci) * 2] = st_lds[(h * CO + ci) * 2 + 1] = 0.f;
      }
      fx_add(d, a);
      fx_add(d + 2, q);
    }
  };

  f32x16 acc[NF];
  constexpr int NU = SP ? 4 : 2;  // 16-B units of a lane's 16 output channels (SP: fp32)
  constexpr unsigned OES = SP ? 4u : 2u;  // output / residual element bytes
  constexpr int NST = NF * NU;  // vector-memory stores of one epilogue (NF fragments x NU)
  auto epilogue = [&](int b, int mt, int ch) __attribute__((always_inline)) {
    const int q0 = mt * TM + fh * FW + l32;
    // the lane's 16 consecutive output channels (packing permutation)
    const int co0 = ch * NCO + 32 * cb + 16 * hi;
    // UPS: the lane's 16 columns are channels c0.. of output phase ph; row q -> frame q u + ph - opad
    const int ph = UPS ? co0 / p.Cout : 0, c0 = UPS ? co0 - ph * p.Cout : co0;
    const int Lrows = UPS ? p.Lout : p.Lq;
    auto orow = [&](int q) __attribute__((always_inline)) { return UPS ? q * p.up + ph - p.opad : q; };
    const Rsrc ry = make_rsrc(reinterpret_cast<char*>(p.y) + (size_t)b * p.y_bs * OES, (unsigned)((size_t)Lrows * p.y_ld * OES));
    const Rsrc rr = make_rsrc(RES ? reinterpret_cast<const char*>(p.res) + (size_t)b * p.res_bs * OES : nullptr,
                              RES ? (unsigned)((size_t)Lrows * p.res_ld * OES) : 0u);
    const Rsrc ra = make_rsrc(ACC ? reinterpret_cast<const char*>(p.accb) + (size_t)b * p.acc_bs * OES : nullptr,
                              ACC ? (unsigned)((size_t)p.Lq * p.acc_ld * OES) : 0u);
    const float osc = p.out_scale;
    const float adiv = (ACC && p.acc_div != 0.f) ? 1.0f / p.acc_div : 1.0f;
    float ts[16], tq[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) ts[r] = tq[r] = 0.f;
    // The residual / running-sum loads of a whole batch of fragments go out together (8 fragments
    // with a residual only, 2 x 4 with a residual and a running sum: the register budget), so a tile
    // pays one load latency per batch.  The builtin wait first retires this wave's in-flight weight
    // DMAs in the compiler's own model, so it counts the loads below precisely (with an LDS-DMA
    // pending it would wait vmcnt(0) at every use); the empty asm fences pin the issue order.
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), expcnt / lgkmcnt unconstrained
    lap(7);
    // (EPI1: a residual-only epilogue loads all 8 fragments in one batch, into the registers the dead
    // tap fragments held: one load latency per tile instead of two; STTS_OPT_EXP bit 2)
    // (SP: fp32 residual / running-sum rows, 64 B per fragment: 4 fragments a batch with a residual only, 2 with a
    // residual and a running sum)
    constexpr int NB0 = SP ? (RES ? (ACC ? 4 : 2) : 1) : ((RES && !(EPI1 && !ACC)) ? 2 : 1);
    constexpr int NB = NB0 * NF / 8 > 0 ? NB0 * NF / 8 : 1, FB = NF / NB;  // (the same batch size at NF = 4)
    uint4 rl[FB][NU], al[FB][NU];
    auto unpack16 = [&](const uint4 (&u)[NU], float (&o)[16]) __attribute__((always_inline)) {
      if constexpr (SP) {
        __builtin_memcpy(o, u, 64);
      } else {
        bf8_to_f32v(u[0], o);
        bf8_to_f32v(u[1], o + 8);
      }
    };
    auto finish = [&](int f, const uint4 (&r2)[NU], const uint4 (&a2)[NU]) __attribute__((always_inline)) {
      f32x16& v = acc[f];  // in place: the accumulators of a finished tile are the output
      const int q = q0 + 32 * f;
      if constexpr (RES) {
        float r0[16];
        unpack16(r2, r0);
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = (v[r] + r0[r]) * osc;
      }
      if constexpr (ACC) {
        float a0[16];
        unpack16(a2, a0);
        if constexpr (SP) {  // the reference divides (xs / num_kernels, hifigan.py:342), as the fp32 engines
          if (p.acc_div != 0.f) {
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] = (a0[r] + v[r]) / p.acc_div;
          } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] = a0[r] + v[r];
          }
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = (a0[r] + v[r]) * adiv;
        }
      }
      float o[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) o[r] = v[r];
      if (!(dbg & 128)) {
        // (an LDS-transposed variant writing 16 rows x 64 contiguous bytes per store measured the
        // same in the decoder: the stores are bound by the chip-wide write burst, not by requests)
        // rows past the output (and UPS rows before frame 0: negative offsets) fall outside the descriptor
        const unsigned ey = (unsigned)(orow(q) * p.y_ld + c0) * OES;
        if constexpr (SP) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            uint4 w;
            __builtin_memcpy(&w, o + 4 * i, 16);
            bstore16(ry, ey + 16u * i, w);
          }
        } else {
          bstore16(ry, ey, f32_to_bf8v(o));
          bstore16(ry, ey + 16u, f32_to_bf8v(o + 8));
        }
      }
      if (!ACC) {
        const float m = (unsigned)orow(q) < (unsigned)Lrows ? 1.f : 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float x = v[r] * m;
          ts[r] += x;
          tq[r] = __builtin_fmaf(x, x, tq[r]);
        }
      }
    };
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
#pragma unroll
      for (int k = 0; k < FB; ++k) {
        const int q = q0 + 32 * (nb * FB + k);
        if constexpr (RES) {
          const unsigned er = (unsigned)((UPS ? orow(q) : (q >> p.res_shift)) * p.res_ld + c0) * OES;
#pragma unroll
          for (int i = 0; i < NU; ++i) rl[k][i] = bload16(rr, er + 16u * i);
        }
        if constexpr (ACC) {
          const unsigned ea = (unsigned)(q * p.acc_ld + co0) * OES;
#pragma unroll
          for (int i = 0; i < NU; ++i) al[k][i] = bload16(ra, ea + 16u * i);
        }
      }
      asm volatile("" ::: "memory");
#pragma unroll
      for (int k = 0; k < FB; ++k) finish(nb * FB + k, rl[k], al[k]);
      asm volatile("" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);  // the tile's stores before the reduction: fewer live values
    lap(8);
    if (want_stats && !(dbg & 256)) {
      // reduce-scatter of the lane's 16 partial sums (then squares) over the 32 lanes of its half:
      // 8 + 4 + 2 + 1 exchanges leave lane l32 with channel co0 + l32 / 2 summed over 16 lanes, one
      // more exchange with lane l32 ^ 1 completes it; the even lane adds the sum, the odd one the
      // sum of squares (32 exchanges and one LDS add per lane instead of 160 and 32; the word is this frame
      // half's, so it has one writer and the totals do not depend on wave timing)
      const float s1 = rs16(ts, l32);
      const float s2 = rs16(tq, l32);
      const int sc = G::NPH > 1 ? fh * G::NPH + ph : fh;  // (this frame half's / phase's copy)
      atomicAdd(st_lds + 2 * (sc * CO + c0 + (l32 >> 1)) + (l32 & 1), (l32 & 1) ? s2 : s1);  // (ds_add: one writer)
    }
    lap(9);
  };

  // ---------------- MFMA taps, software-pipelined within a group.  Tap t = two 8-MFMA halves (input
  // channels 0-15 / 16-31 of the group: window fragments fb0 / fb1, weight fragments fa[t & 1][0 / 1]).
  // While one half's MFMAs issue, the reads of the next half's fragments are in flight (one ds_read
  // per MFMA gap, forced by sched_group_barrier), so the LDS latency is exposed once per group (its
  // first tap) instead of twice per tap.
  const int swz = (l32 >> 2) & 3;
  bf16x8 fa[2][2], fb0[NF], fb1[NF];
  auto rd_a = [&](int s, bf16x8 (&a)[2]) __attribute__((always_inline)) {
    const char* ws = wring + (s % RS) * 2048 + l32 * 64;
    a[0] = *reinterpret_cast<const bf16x8*>(ws + ((hi) ^ swz) * 16);
    a[1] = *reinterpret_cast<const bf16x8*>(ws + ((2 + hi) ^ swz) * 16);
  };
  auto brow = [&](int gg, int t, int half, int& u) __attribute__((always_inline)) {
    // an opaque copy of the lane index: the address is computed here, at the tap, instead of being
    // hoisted out of the loop as K loop-invariant registers (which spill at K = 11)
    int l = l32;
    asm volatile("" : "+v"(l));
    const int r0 = fh * FW + l + t * DIL;
    u = ((2 * half + hi) ^ ((r0 >> 2) & 3)) * 16;  // rows r0 + 32 f share the swizzle
    return smem + G::OFF_X + (gg % NXB) * (G::WROWS * 64) + r0 * 64;
  };
  auto rd_b = [&](bf16x8 (&fb)[NF], int gg, int t, int half) __attribute__((always_inline)) {
    int u;
    const char* row = brow(gg, t, half, u);
#pragma unroll
    for (int f = 0; f < NF; ++f) fb[f] = *reinterpret_cast<const bf16x8*>(row + f * 2048 + u);
  };
  // [MFMA, ds_read] x n in this order
  auto interleave = [&](int n) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < n; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
  };

  // ---------------- prologue: coefficients, group 0's window transformed, weights of steps 0..PD-1
  // group cursors: (tile, group, utterance, frame tile, output part) of the current and the next
  // group, advanced incrementally (tiles run frame tile fastest, then output part, then utterance)
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
  GCur cur = {tbeg, 0, tbeg / upb, tbeg % ntm, NCH > 1 ? (tbeg / ntm) % NCH : 0};
  int cur_b = cur.b;
  set_coef(cur_b);
  __syncthreads();  // nothing in flight yet
  issue_x(0, 0, cur.b, cur.mt);
#pragma unroll
  for (int s = 0; s < PD; ++s) issue_w(s, 0, cur.ch, s);
  if constexpr (LA) {  // window 1 as well (slot 0 DMAs window 2)
    const GCur c1 = NGG > 1 ? advance(cur) : cur;
    issue_x(1, c1.gi, c1.b, c1.mt);
    vm_wait<2 * PD + NWIN>();  // this wave's window DMA of group 0 landed
  } else {
    vm_wait<2 * PD>();
  }
  transform(0, 0, cur.b, cur.mt);

  // the accumulators of tile tt start at the bias.  Set right after the previous tile's epilogue
  // (not at the next group 0), so the compiler sees them dead while that epilogue reduces statistics
  auto init_acc = [&](int ch) __attribute__((always_inline)) {
    const int co0 = (ch * NCO + 32 * cb + 16 * hi) % CO;  // (UPS: the bias of channel n % Cout)
    float bb[16];
    ld8_lds(bias_s + co0, *reinterpret_cast<float(*)[8]>(&bb[0]));
    ld8_lds(bias_s + co0 + 8, *reinterpret_cast<float(*)[8]>(&bb[8]));
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[f][r] = bb[r];
  };

  // ---------------- main loop: one iteration (slot) per 32-channel group; K taps unrolled.  In slot sl every wave
  // DMAs and transforms its share of window sl + 1; a wave computes group gw = sl - off (OFS: off = 1 for the
  // second half of the waves, which so runs one slot behind on window buffers sl - 1; one extra slot at the end)
  init_acc(cur.ch);
  // STTS_OPT_EXP bit 1: static MFMA-issue priority for the second-dispatched half of the waves
  // (MI355X_MICROARCH.md, two waves per SIMD, item 4)
  if ((p.exp & 1) && wu >= NW / 2) __builtin_amdgcn_s_setprio(1);
  const int off = (OFS && wu >= NW / 2) ? 1 : 0;
  constexpr int XS = OFS ? 1 : 0;  // extra slots
  GCur prv = cur;  // the group of the previous slot (the lagging half's compute group)
  for (int sl = 0; sl < NGG + XS; ++sl) {
    lap(6);
    if (!(dbg & 32)) barrier_lds();  // window sl transformed by every wave; its reads of two slots back all done
    lap(2);
    if (sl > 0) {
      prv = cur;
      if (sl < NGG) cur = advance(cur);
    }
    // the next group (past the end: the last group again, a harmless reload keeping counts uniform)
    const GCur nxt = sl + 1 < NGG ? advance(cur) : cur;
    const int gw = sl - off;            // this wave's compute group
    const bool active = gw >= 0 && gw < NGG;
    const GCur me = off ? prv : cur;    // its cursor, and the group after it
    const GCur mnx = off ? cur : nxt;
    const int gi = me.gi;
    // utterance bookkeeping on the lagging half's cursor: it closes a tile one slot after the leading half, so
    // every epilogue of an utterance has run >= 1 barrier before this (OFS = false: both are `cur`)
    const GCur lag = OFS ? prv : cur;
    if (lag.gi == 0 && sl >= XS) {
      const int b = lag.b;
      if (b != cur_b) {  // the block left utterance cur_b
        if (want_stats) flush(cur_b);
        cur_b = b;
      }
    }
    if (cur.gi == 0 && sl < NGG) {
      // the next tile opens another utterance: its coefficients, first read by the transform of its group 0
      // during this tile's last group, >= 1 barrier from here (NG >= 4)
      if (cur.tt + 1 < tend && cur.mt == ntm - 1 && cur.ch == NCH - 1) set_coef(cur.b + 1);
    }
    // (the extra slot re-issues a harmless window DMA, untransformed and never read, so that every slot's
    // vmcnt waits count the same younger operations)
    const bool windows = sl < NGG;
    if constexpr (LA) {  // buffer (sl+2) % 3, last read in slot sl - 1 (before this slot's barrier)
      const GCur nn = sl + 2 < NGG ? advance(nxt) : nxt;
      issue_x(sl + 2, nn.gi, nn.b, nn.mt);
    } else {
      issue_x(sl + 1, nxt.gi, nxt.b, nxt.mt);  // buffer (sl+1) % NXB, last read NXB - 1 slots ago
    }
    if (!active) {  // the lagging half's first slot: only its share of window 1
      if (windows) {
        vm_wait<0>();
        transform(sl + 1, nxt.gi, nxt.b, nxt.mt);
      }
      continue;
    }
    // this wave's weights of step gw K: younger VMEM ops are the weight DMAs of the next PD - 1 steps
    // and the window DMAs just issued
    // (in the group after an epilogue, that epilogue's NST stores are younger too: counted, so the
    // wait does not also drain the stores' write acknowledgements)
    const bool post_epi = gi == 0 && gw > 0;
    lap(6);
    if (post_epi) vm_wait<2 * (PD - 1) + NWIN + NST>();
    else vm_wait<2 * (PD - 1) + NWIN>();
    lap(0);
    rd_a(gw * K, fa[0]);
    rd_b(fb0, gw, 0, 0);
#pragma unroll
    for (int t = 0; t < K; ++t) {
      const int s = gw * K + t;
      // into slot (s+PD) % RS = (s-1) % RS, whose fragments tap s-1 consumed; step s+PD is tap
      // t+PD of this group or tap t+PD-K of the next (PD <= K)
      if (t + PD < K) issue_w(s + PD, gi, me.ch, t + PD);
      else if (gw + 1 < NGG) issue_w(s + PD, mnx.gi, mnx.ch, t + PD - K);
      else issue_w(s + PD, gi, me.ch, K - 1);
      {
        const bf16x8(&a)[2] = fa[t & 1];
        // half 0 of tap t; reads of half 1
        // (SP: fb0 = X_hi, fb1 = X_lo, a[0] = W_hi, a[1] = W_lo: W_hi X_hi + W_lo X_hi here, W_hi X_lo in half 1)
        if constexpr (SP) {
          int u;
          const char* row = brow(gw, t, 1, u);
#pragma unroll
          for (int f = 0; f < NF; ++f) {
            acc[f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], fb0[f], acc[f], 0, 0, 0);
            acc[f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], fb0[f], acc[f], 0, 0, 0);
            fb1[f] = *reinterpret_cast<const bf16x8*>(row + f * 2048 + u);
          }
#pragma unroll
          for (int i = 0; i < NF; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          }
        } else {
          int u;
          const char* row = brow(gw, t, 1, u);
#pragma unroll
          for (int f = 0; f < NF; ++f) {
            acc[f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], fb0[f], acc[f], 0, 0, 0);
            fb1[f] = *reinterpret_cast<const bf16x8*>(row + f * 2048 + u);
          }
          interleave(NF);
        }
        const bf16x8& a1 = SP ? a[0] : a[1];  // the second half's weight fragment
        // half 1 of tap t; reads of half 0 of tap t+1 and, once its DMA is in, of its weights
        if (t + 1 < K) {
          int u;
          const char* row = brow(gw, t + 1, 0, u);
#pragma unroll
          for (int f = 0; f < NF / 2; ++f) {
            acc[f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, fb1[f], acc[f], 0, 0, 0);
            fb0[f] = *reinterpret_cast<const bf16x8*>(row + f * 2048 + u);
          }
          interleave(NF / 2);
          // weights of step s+1: younger VMEM ops are the weight DMAs of steps s+2..s+PD and, while
          // step s+1 precedes this slot's window DMAs (t + 1 < PD), those
          lap(6);
          if (t + 1 < PD) {
            if (post_epi) vm_wait<2 * (PD - 1) + NWIN + NST>();
            else vm_wait<2 * (PD - 1) + NWIN>();
          } else {
            vm_wait<2 * (PD - 1)>();
          }
          lap(0);
          rd_a(s + 1, fa[(t + 1) & 1]);
#pragma unroll
          for (int f = NF / 2; f < NF; ++f) {
            acc[f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, fb1[f], acc[f], 0, 0, 0);
            fb0[f] = *reinterpret_cast<const bf16x8*>(row + f * 2048 + u);
          }
          interleave(NF / 2);
        } else {
#pragma unroll
          for (int f = 0; f < NF; ++f) acc[f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, fb1[f], acc[f], 0, 0, 0);
        }
      }
      // the next window: this wave's DMAs of it are older than the weight DMAs of taps 0..t.  With two
      // waves per SIMD (NW = 8) the second half transforms one tap earlier, so each SIMD's transforms run
      // beside its partner's MFMAs instead of beside each other
      constexpr int TX = K - 1;
      constexpr int TX2 = (NW == 8) ? K - 2 : K - 1;
      if (windows && ((t == TX && (NW != 8 || wu < 4)) || (t == TX2 && NW == 8 && wu >= 4))) {
        lap(6);
        if constexpr (LA) {
          // window sl + 1 was DMA'd at the start of slot sl - 1 (slot 0: in the prologue).  Younger: slot sl - 1's K
          // weight steps (and its epilogue's NST stores when it closed a tile), window sl + 2's DMA, and this slot's
          // weight steps of taps 0..t
          constexpr int Y1 = NWIN + 2 * K, Y2 = NWIN + 2 * (K - 1);  // t = K - 1 / K - 2
          if (t == K - 1) {
            if (sl == 0) vm_wait<Y1>();
            else if (post_epi) vm_wait<Y1 + 2 * K + NST>();
            else vm_wait<Y1 + 2 * K>();
          } else {
            if (sl == 0) vm_wait<Y2>();
            else if (post_epi) vm_wait<Y2 + 2 * K + NST>();
            else vm_wait<Y2 + 2 * K>();
          }
        } else {
          if (t == K - 1) vm_wait<2 * K>();
          else vm_wait<2 * (K - 1)>();
        }
        lap(1);
        transform(sl + 1, nxt.gi, nxt.b, nxt.mt);
        lap(3);
      }
    }
    if (gi == NG - 1) {
      lap(6);
      if (!(dbg & 4)) epilogue(me.b, me.mt, me.ch);
      init_acc(mnx.ch);
      lap(4);
    }
  }
  vm_wait<0>();  // nothing may land in LDS after the block's exit
  barrier_lds();
  if (want_stats) flush(cur_b);
  if (stamp) {
    lap(6);
    st_acc[5] = __builtin_amdgcn_s_memtime() - t_start;
    if (lane == 0)
      for (int k = 0; k < 10; ++k) atomicAdd(p.stamps + k, st_acc[k]);
    if (lane == 0 && wu == 0) atomicAdd(p.stamps + 15, 1ull);
  }
  if constexpr (!SEG) break;  // (one range)
  }  // tile ranges
}

template <int C, int NW, int K, int DIL, bool RES, bool ACC, int PRO = PK_SNAKE, int CINP = C, bool EPI1 = false,
          bool UPS = false, int CO = C, bool OFS = false, bool SP = false, bool LA = false, int NF = 8, int NCB = 0>
int launch_b2(const ConvParams& p, hipStream_t stream) {
  using G = B2<C, NW, K, DIL, PRO, CINP, UPS, CO, OFS, LA, NF, NCB>;
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    ST_CHECK_HIP(hipGetDevice(&dev));
    ST_CHECK_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const long long tiles = (long long)((p.Lq + G::TM - 1) / G::TM) * G::NCH * p.B;
  ConvParams q = p;
  const int seg = st_seg_choice(p, 1, ncu * G::BPC);
  long long grid = (long long)ncu * G::BPC;
  if (grid > (seg ? (long long)p.B * seg : tiles)) grid = seg ? (long long)p.B * seg : tiles;
  if (g_opt_grid_cap > 0 && grid > g_opt_grid_cap) grid = g_opt_grid_cap;
  // one segment per workgroup: the segments are the even split of the plain kernel (every utterance has the same
  // tile count), so only a launch with more segments than workgroups needs the range loop
  const bool segk = seg > 0 && grid < (long long)p.B * seg;
  q.seg = segk ? seg : 0;
  auto kern = segk ? k_bigconv2<C, NW, K, DIL, RES, ACC, PRO, CINP, EPI1, UPS, CO, OFS, SP, LA, NF, NCB, true>
                   : k_bigconv2<C, NW, K, DIL, RES, ACC, PRO, CINP, EPI1, UPS, CO, OFS, SP, LA, NF, NCB, false>;
  static bool attr[2] = {false, false};
  if (!attr[segk]) {
    ST_CHECK_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
    attr[segk] = true;
  }
  q.skew = g_opt_skew;
  q.exp = g_opt_exp;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * NW), G::LDS, stream, q);
  return (int)hipGetLastError();
}

template <int C, int NW, int K, bool OFS = false, bool SP = false, bool LA = false, int NF = 8>
int launch_b2_k(const ConvParams& p, hipStream_t s) {
  constexpr bool F = false;
  if (!p.res) {  // conv1 of an iteration: dilation 1 / 3 / 5, no residual
    if (p.accb) return ST_EINVAL;
    switch (p.dil) {
      case 1: return launch_b2<C, NW, K, 1, F, F, PK_SNAKE, C, F, F, C, OFS, SP, LA, NF>(p, s);
      case 3: return launch_b2<C, NW, K, 3, F, F, PK_SNAKE, C, F, F, C, OFS, SP, LA, NF>(p, s);
      case 5: return launch_b2<C, NW, K, 5, F, F, PK_SNAKE, C, F, F, C, OFS, SP, LA, NF>(p, s);
      default: return ST_EINVAL;
    }
  }
  if (p.dil != 1) return ST_EINVAL;  // conv2: dilation 1, residual, optionally the resblock sum
  if (p.accb) return launch_b2<C, NW, K, 1, true, true, PK_SNAKE, C, F, F, C, OFS, SP, LA, NF>(p, s);
  if constexpr (!OFS && !SP && !LA && NF == 8)
    if (g_opt_exp & 2) return launch_b2<C, NW, K, 1, true, false, PK_SNAKE, C, true>(p, s);
  return launch_b2<C, NW, K, 1, true, F, PK_SNAKE, C, F, F, C, OFS, SP, LA, NF>(p, s);
}

template <int C, int NW, bool OFS = false, bool SP = false, int NF = 8>
int launch_b2_c(const ConvParams& p, hipStream_t s) {
  switch (p.KS) {
    case 3:
      if constexpr (NW == 8 && !OFS && C >= 256)  // the window lookahead (B2::LA) where it fits: 8-wave blocks, 3 taps
        // (C = 128: its 512-row windows leave no room for a third buffer)
        if (g_opt_bigla) return launch_b2_k<C, NW, 3, OFS, SP, true>(p, s);
      return launch_b2_k<C, NW, 3, OFS, SP, false, NF>(p, s);
    case 7: return launch_b2_k<C, NW, 7, OFS, SP, false, NF>(p, s);
    case 11: return launch_b2_k<C, NW, 11, OFS, SP, false, NF>(p, s);
    default: return ST_EINVAL;
  }
}

}  // namespace

// STTS_OPT_BIGCONV: 1 = bigconv.hip (v1, A/B); 2 = this engine, 8-wave blocks (one per CU);
// 3 = this engine, 4-wave blocks (two per CU, C = 256 split into two 128-channel output parts)
int g_opt_bigconv = 2;
// STTS_OPT_BIGLA: the 3-tap / 2-tap 8-wave launches with the window lookahead (B2::LA).  Off: measured neutral
// (profiles/r05_ab_bigla.txt: C = 256 k3 156 -> 161 us, the front-end and ups[0] within 2 %), so the window DMA's
// latency is not what the 3-tap launches wait on
int g_opt_bigla = 0;
int g_opt_skew = 0;
int g_opt_exp = 0;

bool st_bigconv2_eligible(const ConvParams& p) {
  if (g_opt_bigconv < 2) return false;
  if (p.res ? p.dil != 1 : (p.accb != nullptr)) return false;
  // mode 2 (default) keeps v1 where it measured faster: C = 128 with 3 taps (12 taps per tile, so
  // the per-tile window transform and epilogue dominate; profiles/r02_ab_bigconv_pipelined.txt)
  if ((g_opt_bigconv == 2 || g_opt_bigconv == 5) && p.Cout == 128 && p.KS == 3) return false;  // (modes 3 / 4: v2 everywhere)
  return true;  // on top of st_bigconv_eligible
}

static int b2_num_cu() {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      ncu = 256;
  }
  return ncu;
}

// ---- decoder front-end (AdainResBlk1d k3 convs, hifigan.py:359-403 / 427-432): C_out 1024 / 512
// in 256-channel output parts, C_in up to 1120 (the 1090-channel concat), [AdaIN ->] LReLU prologue
constexpr int FE_CINP = 1120;
int g_opt_front = 1;

bool st_front_eligible(const ConvParams& p, int dtype) {
  if (!g_opt_front || dtype != ST_BF16) return false;
  // few tiles (small batches: B = 1 has 8 at T = 400) leave the CUs idle behind long per-tile
  // group chains; the igemm engine's smaller tiles do better there (profiles/r02_ab_b1.txt)
  // (STTS_OPT_FRONT = 2 forces the engine at any size: tests)
  if (g_opt_front == 1 && (long long)((p.Lq + 255) / 256) * (p.Cout / 256) * p.B < b2_num_cu() / 2) return false;
  if (p.Cout != 1024 && p.Cout != 512) return false;
  const int mode = p.pro.mode;
  if (mode != 0 && mode != PRO_LRELU && mode != (PRO_AFFINE | PRO_LRELU) && mode != PRO_AFFINE) return false;
  return p.N == p.Cout && p.KS == 3 && p.dil == 1 && p.stride == 1 && p.up == 1 && p.pad == 1 && !p.epi_lrelu && !p.epi_gelu &&
         (p.kw == 0 || p.kw == p.KS) && p.row_off == 0 && p.Cin >= 128 && p.Cin <= FE_CINP &&
         p.Lin == p.Lq && p.Lout == p.Lq && !p.accb && !p.epi_tanh && !p.y_f32 && !p.reflect_front &&
         p.zc_period == 0 && p.y_row_off == 0 && p.x_ld % 8 == 0 && p.y_ld % 8 == 0 &&
         (!p.res || (p.res_ld % 8 == 0 && (p.res_shift == 0 || p.res_shift == 1)));
}

int st_bigconv2_front(const ConvParams& p, hipStream_t s) {
  if (g_opt_big3 & 2) return st_bigconv3_front(p, s);
  constexpr bool F = false;
  if (g_opt_bigla) {
    if (p.Cout == 1024)
      return p.res ? launch_b2<1024, 8, 3, 1, true, F, PK_LRELU, FE_CINP, F, F, 1024, F, F, true>(p, s)
                   : launch_b2<1024, 8, 3, 1, false, F, PK_LRELU, FE_CINP, F, F, 1024, F, F, true>(p, s);
    if (p.Cout == 512)
      return p.res ? launch_b2<512, 8, 3, 1, true, F, PK_LRELU, FE_CINP, F, F, 512, F, F, true>(p, s)
                   : launch_b2<512, 8, 3, 1, false, F, PK_LRELU, FE_CINP, F, F, 512, F, F, true>(p, s);
    return ST_EINVAL;
  }
  if (p.Cout == 1024)
    return p.res ? launch_b2<1024, 8, 3, 1, true, false, PK_LRELU, FE_CINP>(p, s)
                 : launch_b2<1024, 8, 3, 1, false, false, PK_LRELU, FE_CINP>(p, s);
  if (p.Cout == 512)
    return p.res ? launch_b2<512, 8, 3, 1, true, false, PK_LRELU, FE_CINP>(p, s)
                 : launch_b2<512, 8, 3, 1, false, false, PK_LRELU, FE_CINP>(p, s);
  return ST_EINVAL;
}


int st_bigconv2(const ConvParams& p, hipStream_t stream) {
  // STTS_OPT_BIGCONV 5: C = 256 on 8-wave blocks with the second half one group behind (OFS; a third window
  // buffer: C = 128's 512-row windows leave no room for it), the mode-2 choice elsewhere
  if (g_opt_bigconv == 5 && p.Cout == 256) return launch_b2_c<256, 8, true>(p, stream);
  // mode 3, or mode 2 with fewer 8-wave tiles than CUs (small batches: B = 1 at C = 256 has 32):
  // 4-wave blocks, two per CU, twice the tiles (profiles/r02_ab_b1.txt: C = 256 k11 75 -> 61 us)
  const int tm8 = p.Cout == 128 ? 512 : 256;
  const long long tiles8 = (long long)((p.Lq + tm8 - 1) / tm8) * p.B;
  // (mode 4 = 8-wave blocks at any size: tests).  Mode 2 also takes the 4-wave blocks for C = 128 with
  // 7 / 11 taps at every size: two blocks per CU overlap one block's window transform / epilogue with
  // the other's MFMAs, 371 -> 346 us (k7 conv1) and 445 -> 404 us (k7 conv2) at B = 32, while C = 256
  // and C = 128 k3 are faster with 8-wave blocks / v1 (profiles/r02_ab_bigconv_modes.txt)
  const bool two = g_opt_bigconv == 3 ||
                   ((g_opt_bigconv == 2 || g_opt_bigconv == 5) && (tiles8 < b2_num_cu() || (p.Cout == 128 && p.KS >= 7)));
  if (p.Cout == 128) return two ? launch_b2_c<128, 4>(p, stream) : launch_b2_c<128, 8>(p, stream);
  if (p.Cout == 256) return two ? launch_b2_c<256, 4>(p, stream) : launch_b2_c<256, 8>(p, stream);
  return ST_EINVAL;
}

// ---- the wide polyphase upsamplers (HiFi-GAN ups[0] 512 -> 256 x10, N = 2,560; ups[1] 256 -> 128 x5,
// N = 640; hifigan.py:292-294 with the Snake(alphas[i]) prologue of :333 and the noise-branch residual
// x + x_source of :335): 2 taps, on this engine instead of conv1d_igemm (STTS_OPT_UPS, default on)
int g_opt_ups = 1;

bool st_ups_eligible(const ConvParams& p, int dtype) {
  if (!g_opt_ups || dtype != ST_BF16 || p.up <= 1 || !p.res || p.accb) return false;
  // (ups[2], N = 192: STTS_OPT_UPS 1 takes it too, 2 = ups[0] / ups[1] only)
  const bool shape = (p.N == 2560 && p.Cin == 512 && p.Cout == 256) || (p.N == 640 && p.Cin == 256 && p.Cout == 128) ||
                     (g_opt_ups == 1 && p.N == 192 && p.Cin == 128 && p.Cout == 64);
  return shape && p.N == p.up * p.Cout && p.Cout % 16 == 0 && p.KS == 2 && (p.kw == 0 || p.kw == 2) &&
         p.dil == 1 && p.stride == 1 && p.pad == 1 && p.row_off == 0 && p.pro.mode == PRO_SNAKE && p.pro.alpha &&
         p.res_shift == 0 && p.y_row_off == 0 && !p.reflect_front && !p.epi_tanh && !p.epi_lrelu && !p.epi_gelu &&
         !p.y_f32 && p.zc_period == 0 && p.x_ld % 8 == 0 && p.y_ld % 8 == 0 && p.res_ld % 8 == 0 &&
         p.nchunks * 32 == p.Cin;
}

int st_bigconv2_ups(const ConvParams& p, hipStream_t s) {
  if ((g_opt_big3 & 4) && ((p.N == 2560 && p.Cout == 256) || (p.N == 640 && p.Cout == 128))) return st_bigconv3_ups(p, s);
  if (p.N == 2560 && p.Cout == 256)
    return g_opt_bigla ? launch_b2<2560, 8, 2, 1, true, false, PK_SNAKE, 512, false, true, 256, false, false, true>(p, s)
                       : launch_b2<2560, 8, 2, 1, true, false, PK_SNAKE, 512, false, true, 256>(p, s);
  if (p.N == 640 && p.Cout == 128) return launch_b2<640, 4, 2, 1, true, false, PK_SNAKE, 256, false, true, 128>(p, s);
  // ups[2]: 12-wave blocks (three per SIMD) of all 6 output blocks (the 3 phases) x 2 frame slices of 128 frames, so each
  // window is DMA'd and transformed once instead of once per phase: 668 -> 479 us (profiles/r05_ab_ups12.txt).
  // STTS_OPT_EXP bit 32: 4-wave blocks of 2 output blocks (one 64-column phase per tile part), as before (A/B)
  if (p.N == 192 && p.Cout == 64) {
    if (g_opt_exp & 32)
      return launch_b2<192, 4, 2, 1, true, false, PK_SNAKE, 128, false, true, 64, false, false, false, 4, 2>(p, s);
    return launch_b2<192, 12, 2, 1, true, false, PK_SNAKE, 128, false, true, 64, false, false, false, 4, 6>(p, s);
  }
  return ST_EINVAL;
}

// ---- C = 64 resblock convs (the generator's stage 2 and the 64-channel noise_res) on this engine with 128-frame
// wave slices (NF = 4): 4-wave blocks (two per CU) of 2 frame slices x 2 output blocks, 256-frame tiles (bit 4; else
// 8-wave blocks, 512-frame tiles).  STTS_OPT_BIG64 bit 1:
// the accuracy mode's (replacing the two-pass split resblock engine), bit 2: bf16 (replacing resconv)
int g_opt_big64 = 5;  // (SP on 4-wave blocks: 2-7 % faster per launch than 8-wave, profiles/r05_ab_big64.txt)

bool st_big64_eligible(const ConvParams& p, int dtype) {
  const int C = p.Cout;
  if (C == 32) {  // bit 8: the accuracy mode's C = 32 convs too (64-frame wave slices, NF = 2; A/B)
    if (!((g_opt_big64 & 8) && dtype == ST_SPLIT)) return false;
  } else if (!(((g_opt_big64 & 1) && dtype == ST_SPLIT) || ((g_opt_big64 & 2) && dtype == ST_BF16))) {
    return false;
  }
  if (!(C == 64 || C == 32) || p.Cin != C || p.N != C || p.nchunks * 32 != C) return false;
  if (!(p.KS == 3 || p.KS == 7 || p.KS == 11) || !(p.dil == 1 || p.dil == 3 || p.dil == 5)) return false;
  if ((p.kw != 0 && p.kw != p.KS) || p.row_off != 0 || p.stride != 1 || p.up != 1 || p.opad != 0) return false;
  if (p.pad != p.dil * (p.KS - 1) / 2 || p.Lq != p.Lout || p.Lq != p.Lin) return false;
  if (p.y_row_off || p.y_f32 || p.epi_tanh || p.epi_lrelu || p.epi_gelu || p.reflect_front || p.zc_period || p.res_shift) return false;
  if (p.pro.mode != (PRO_AFFINE | PRO_SNAKE) || !p.pro.alpha || !p.pro.stats || !p.pro.gamma) return false;
  if (p.accb && p.stats) return false;
  if (p.res ? p.dil != 1 : (p.accb != nullptr)) return false;
  if (!p.y || p.x_ld % 8 || p.y_ld % 8 || (p.res && p.res_ld % 8) || (p.accb && p.acc_ld % 8)) return false;
  return true;
}

int st_big64(const ConvParams& p, int dtype, hipStream_t s) {
  if (p.Cout == 32) return dtype == ST_SPLIT ? launch_b2_c<32, 4, false, true, 2>(p, s) : ST_EDTYPE;
  // (bit 4: 4-wave blocks, two per CU, 256-frame tiles; A/B)
  if (dtype == ST_SPLIT)
    return (g_opt_big64 & 4) ? launch_b2_c<64, 4, false, true, 4>(p, s) : launch_b2_c<64, 8, false, true, 4>(p, s);
  if (dtype == ST_BF16)
    return (g_opt_big64 & 4) ? launch_b2_c<64, 4, false, false, 4>(p, s) : launch_b2_c<64, 8, false, false, 4>(p, s);
  return ST_EDTYPE;
}

// ---- the split-operand accuracy mode (STTS_SPLIT, dtype ST_SPLIT: fp32 frames, bf16 hi + lo operands) on this
// engine (SP): the C = 128 / 256 resblock convs, the front-end k3 convs and ups[0] / ups[1], which ran on the split
// conv1d_igemm (STTS_OPT_BIGSPLIT, default on; 0 = the split igemm, A/B)
int g_opt_bigsplit = 1;

bool st_bigsplit_eligible(const ConvParams& p, int dtype) {
  if (!g_opt_bigsplit || dtype != ST_SPLIT) return false;
  // the bf16 engines' shape rules (frames ld multiples of 8 elements: 32-B aligned fp32 rows)
  // (and ups[3], which bf16 runs on resconv)
  return st_bigconv_eligible(p, ST_BF16) || st_front_eligible(p, ST_BF16) || st_ups_eligible(p, ST_BF16) ||
         (g_opt_ups == 1 && st_resconv_ups_eligible(p, ST_BF16));
}

int st_bigsplit(const ConvParams& p, hipStream_t s) {
  // ups[3] (64 -> 32, x2, N = 64): 4-wave blocks of 2 output blocks (both 32-column phases) x 2 frame slices of 64 frames
  // tiles of both phases, 2 output blocks x 2 frame slices of 64 frames, each window transformed once: 1076 -> 908 us
  // (profiles/r05_ab_ups12.txt; STTS_OPT_EXP bit 64: one phase per tile part, as before)
  if (g_opt_ups == 1 && st_resconv_ups_eligible(p, ST_BF16)) {
    if (g_opt_exp & 64)
      return launch_b2<64, 4, 2, 1, true, false, PK_SNAKE, 64, false, true, 32, false, true, false, 2, 1>(p, s);
    return launch_b2<64, 4, 2, 1, true, false, PK_SNAKE, 64, false, true, 32, false, true, false, 2, 2>(p, s);
  }
  if (st_ups_eligible(p, ST_BF16)) {
    if (p.N == 2560 && p.Cout == 256)
      return launch_b2<2560, 8, 2, 1, true, false, PK_SNAKE, 512, false, true, 256, false, true>(p, s);
    if (p.N == 640 && p.Cout == 128)
      return launch_b2<640, 4, 2, 1, true, false, PK_SNAKE, 256, false, true, 128, false, true>(p, s);
    if (p.N == 192 && p.Cout == 64) {  // (12-wave blocks as bf16: 1167 -> 926 us; bit 32: the 4-wave blocks)
      if (g_opt_exp & 32)
        return launch_b2<192, 4, 2, 1, true, false, PK_SNAKE, 128, false, true, 64, false, true, false, 4, 2>(p, s);
      return launch_b2<192, 12, 2, 1, true, false, PK_SNAKE, 128, false, true, 64, false, true, false, 4, 6>(p, s);
    }
    return ST_EINVAL;
  }
  if (st_front_eligible(p, ST_BF16)) {
    if (p.Cout == 1024)
      return p.res ? launch_b2<1024, 8, 3, 1, true, false, PK_LRELU, FE_CINP, false, false, 1024, false, true>(p, s)
                   : launch_b2<1024, 8, 3, 1, false, false, PK_LRELU, FE_CINP, false, false, 1024, false, true>(p, s);
    if (p.Cout == 512)
      return p.res ? launch_b2<512, 8, 3, 1, true, false, PK_LRELU, FE_CINP, false, false, 512, false, true>(p, s)
                   : launch_b2<512, 8, 3, 1, false, false, PK_LRELU, FE_CINP, false, false, 512, false, true>(p, s);
    return ST_EINVAL;
  }
  // resblock convs: 4-wave blocks (two per CU) where the bf16 engine takes them (few tiles, C = 128 k7 / k11)
  const int tm8 = p.Cout == 128 ? 512 : 256;
  const long long tiles8 = (long long)((p.Lq + tm8 - 1) / tm8) * p.B;
  // (STTS_OPT_BIGSPLIT 3 = 4-wave blocks everywhere, 4 = 8-wave blocks everywhere: tests)
  // (C = 128 takes them at every K: k3 548 vs 784 us on 8-wave blocks, profiles/r05_ab_bigsplit_modes.txt)
  const bool two = g_opt_bigsplit != 4 && (tiles8 < b2_num_cu() || p.Cout == 128 || g_opt_bigsplit == 3);
  if (p.Cout == 128) return two ? launch_b2_c<128, 4, false, true>(p, s) : launch_b2_c<128, 8, false, true>(p, s);
  if (p.Cout == 256) return two ? launch_b2_c<256, 4, false, true>(p, s) : launch_b2_c<256, 8, false, true>(p, s);
  return ST_EINVAL;
}
