// Implicit-GEMM 1-D convolution on MFMA for gfx950 (the dilated resblock convs, the
// AdainResBlk1d convs, the 1x1 shortcuts, the padded-image 2-D convs of the style encoder
// and — via a polyphase rewrite — the ConvTranspose1d upsamplers).  Reference ops restated:
// nn.Conv1d / nn.ConvTranspose1d inside Modules/hifigan.py:26-80, 272-347, 359-403,
// Modules/istftnet.py:494-573 and nn.Conv2d in models.py:82-150.
//
// GEMM view (frames layout [B][L][C]):
//   out[q][n] = sum_{tap, ci} X[q*stride + (tap/kw)*row_off + (tap%kw)*dil - pad][ci] * W[tap][ci][n]
//   rows M = output frames q, columns N = output channels (or (phase, channel) pairs for a
//   transposed conv), K = taps x input channels (contiguous in memory).
//
// Persistent workgroups (one launch fills the chip once; each workgroup walks a contiguous
// range of BM x BN tiles, time fastest):
//   * the per-(utterance, channel) AdaIN coefficients are computed once per utterance into LDS;
//   * when all packed weights of the column tile fit the LDS budget they are staged ONCE per
//     workgroup (small-channel stages) instead of once per tile — the weight re-reads, not HBM,
//     were the cost of the first version (profiles/r01_*);
//   * per 32-channel chunk the input window is staged once into LDS with the prologue
//     (AdaIN / Snake / LReLU) applied, and re-read by every tap;
//   * MFMA: bf16 -> v_mfma_f32_32x32x16_bf16, fp32 -> v_mfma_f32_32x32x2_f32 (exact f32 fma chain);
//   * epilogue: each wave transposes its 32x32 accumulator tiles through LDS so every lane
//     owns 16 consecutive channels of one frame (32/64-byte vector loads and stores), then
//     fuses bias, residual, 1/sqrt2, the resblock average, tanh, the iSTFTNet reflection pad
//     and the InstanceNorm statistics; statistics are kept in registers across the tiles of
//     one utterance and flushed with one fp64 atomic per (utterance, channel, workgroup).
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "conv_common.h"
#include "kernels.h"


namespace {

constexpr int BK = 32;
constexpr int EP = 36;  // stats scratch pitch (floats): conflict-free b128 row writes

template <typename MT> struct Layout;
template <> struct Layout<bf16_t> {
  static constexpr int XP = 40;  // X row pitch (bf16) = 80 B: conflict-free ds_read_b128
  static constexpr int WP = 40;  // W: [tap][n][WP]
};
template <> struct Layout<float> {
  static constexpr int XP = 33;  // odd pitch: conflict-free ds_read_b32 column reads
  static constexpr int WP = 0;   // W: [tap][k][BN]
};

// SPF: with fp32 frames on the bf16 MFMA path (T = float, MT = bf16), true = the split accuracy mode,
// false = plain bf16 operands converted while staging (ST_BF16F: the training step's fp32 frames)
template <typename T, typename MT, int WAVES_M, int WAVES_N, int WM, int WN, bool SPF = true>
struct ConvCfg {
  static constexpr bool BF = std::is_same<MT, bf16_t>::value;
  // ST_SPLIT (accuracy mode): fp32 activations on the bf16 MFMA path, every window and weight slice
  // staged twice (hi, lo) and multiplied as hi*hi + hi*lo + lo*hi
  static constexpr bool SPLIT = BF && std::is_same<T, float>::value && SPF;
  static constexpr bool LOWP = BF && !SPLIT;  // the bf16 throughput mode's shortcuts (v_sin, reciprocal)
  static constexpr int SPL = SPLIT ? 2 : 1;
  static constexpr int NW = WAVES_M * WAVES_N;
  static constexpr int NT = 64 * NW;
  static constexpr int BM = 32 * WM * WAVES_M;
  static constexpr int BN = 32 * WN * WAVES_N;
  static constexpr int XP = Layout<MT>::XP;
  static constexpr int WPITCH = BF ? Layout<MT>::WP : BN;
  static constexpr int W_TAP = BF ? BN * Layout<MT>::WP : BK * BN;  // elements per tap slice
  __host__ __device__ static int rows(const ConvParams& p) {
    return (BM - 1) * p.stride + ((p.KS - 1) / p.kw) * p.row_off + ((p.KS < p.kw ? p.KS : p.kw) - 1) * p.dil + 1;
  }
  // LDS carve (bytes): [coef 4 x cinp f32 | bias BN f32 | stats scratch NW x 32 x EP f32][X window][W slices]
  __host__ __device__ static int cinp(const ConvParams& p) { return p.nchunks * BK; }
  __host__ __device__ static size_t coef_bytes(const ConvParams& p) {
    return ((size_t)4 * cinp(p) + BN + (size_t)NW * 32 * EP) * 4;
  }
  __host__ __device__ static size_t xs_bytes(const ConvParams& p) {
    return (((size_t)rows(p) * XP * sizeof(MT)) + 15) & ~(size_t)15;
  }
  static size_t lds_bytes(const ConvParams& p, int nwslices, int nx = 1) {
    return coef_bytes(p) + (size_t)SPL * ((size_t)nx * xs_bytes(p) + (size_t)nwslices * W_TAP * sizeof(MT));
  }
};

typedef float f2v __attribute__((ext_vector_type(2)));
// bf16 frames: at least 2 waves per SIMD (<= 256 VGPRs); fp32 frames (the parity mode, the split accuracy
// mode, ST_BF16F) keep their registers (fp32 window prefetch sets) on 4-wave tiles
template <typename T, typename MT, bool SPF>
constexpr int kMinWaves = (std::is_same<MT, bf16_t>::value && std::is_same<T, bf16_t>::value) ? 2 : 1;

// 16 values <-> 8 packed pairs
__device__ __forceinline__ f2v pr(const float (&v)[16], int i) { return f2v{v[2 * i], v[2 * i + 1]}; }
__device__ __forceinline__ void pw(float (&v)[16], int i, f2v x) {
  v[2 * i] = x.x;
  v[2 * i + 1] = x.y;
}

// Accumulator orientation: the MFMA computes C^T = W^T X^T (A = weights, B = input window), so
// a lane's 16 accumulator registers are ONE output frame (column = lane & 31) and, because
// st_pack_conv permutes the packed rows inside each 32-block (row m holds channel
// 16*((m>>2)&1) + (m&3) + 4*(m>>3)), 16 CONSECUTIVE channels 16*(lane>>5) + r.  The epilogue
// therefore works straight from registers: no LDS transpose, 16-channel vector loads/stores,
// and per-lane statistics accumulated across tiles (reduced across lanes once per utterance).
// SEG: the launch runs segmented tile ranges (p.seg > 0, statistics launches of B = 32 k utterances); the plain
// instantiation keeps the one-range-per-workgroup code (a range loop in every launch had cost the training step's
// igemm convs 5-15 %: register allocation and hoisting across the loop)
template <typename T, typename MT, int WAVES_M, int WAVES_N, int WM, int WN, bool NARROW, int CPS, bool SPF = true,
          bool SEG = false>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N, (kMinWaves<T, MT, SPF>))
    conv1d_igemm_kernel(const ConvParams p) {
  using C = ConvCfg<T, MT, WAVES_M, WAVES_N, WM, WN, SPF>;
  constexpr int BM = C::BM, BN = C::BN, XP = C::XP, WPITCH = C::WPITCH, W_TAP = C::W_TAP, NT = C::NT;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int R = C::rows(p);
  const int cinp = C::cinp(p);
  float* coef = reinterpret_cast<float*>(smem);  // [4][cinp]: beta - mean*a, a, alpha (x 1/2pi in bf16), 1/alpha
  float* bias_s = coef + 4 * cinp;               // [BN]: bias of the column tile's (phase, channel) columns
  float* ws = bias_s + BN + (size_t)(threadIdx.x >> 6) * 32 * EP;  // this wave's stats scratch [frame][EP]
  MT* Xs = reinterpret_cast<MT*>(smem + C::coef_bytes(p));
  // chunks per step (set by the launcher): 2 = two 32-channel chunks (two windows, two weight
  // slices) per barrier pair, half the barriers and twice the MFMAs between them
  constexpr int cps = CPS;
  static_assert(!C::SPLIT || CPS == 1, "split mode stages one chunk per step (hi, lo windows)");
  MT* Ws = reinterpret_cast<MT*>(smem + C::coef_bytes(p) + (size_t)C::SPL * cps * C::xs_bytes(p));
  // the second window slot: chunk c+1 (cps == 2) or, in split mode, the lo parts of the window
  const size_t xs_el = C::xs_bytes(p) / sizeof(MT);
  // split mode: the lo weight slices follow the hi ones (resident: all of them; streamed: one tap group)
  const size_t wlo = C::SPLIT ? (p.w_resident ? (size_t)p.nchunks * p.KS * W_TAP : (size_t)p.tg * W_TAP) : 0;
  const unsigned wlo_bytes = C::SPLIT ? (unsigned)((size_t)p.nchunks * p.KS * BK * ((p.N + 31) & ~31) * sizeof(MT)) : 0u;

  const int ntn = (p.N + BN - 1) / BN;
  const int ntm = (p.Lq + BM - 1) / BM;
  const long long total = (long long)ntn * ntm * p.B;
  // XCD-aware: the tile ranges of consecutive logical blocks (same column tile, same weights)
  // land on one XCD, so each XCD's L2 holds the weights of ~1/8 of the column tiles
  // tile ranges (kernels.h tile_range: one per workgroup, or utterance-relative segments); the first is
  // the XCD-remapped one
  const int nv = SEG ? tile_nv(p, p.B) : (int)gridDim.x;
  for (int vb = xcd_remap(blockIdx.x, gridDim.x); vb < nv; vb += gridDim.x) {
  long long tb_, te_;
  if constexpr (SEG) {
    tile_range(p, vb, nv, total, (long long)ntn * ntm, tb_, te_);
  } else {
    tb_ = total * vb / gridDim.x;
    te_ = total * (vb + 1) / gridDim.x;
  }
  const int tbeg = (int)tb_, tend = (int)te_;
  if (SEG && tbeg >= tend) continue;  // uniform over the block

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WAVES_N, wn = wid % WAVES_N;
  const int l32 = lane & 31, hi = lane >> 5;
  const int Np = (p.N + 31) & ~31;
  const int mode = p.pro.mode;
  const bool resident = p.w_resident != 0;
  // tile t -> (row tile mt, utterance b, column tile nt), time fastest: a block's contiguous tile
  // range stays in one column tile.  (Column-tile-fastest orders, tried for the streamed-weight
  // upsamplers to re-read each input window from L2, measured 10-30 % slower: every tile then
  // re-stages its window's prologue and flushes statistics.)
  // (segmented ranges, p.seg > 0: utterance-major instead, (utterance, column tile, row tile), so that a range lies
  // inside one utterance whatever the column-tile count)
  auto t_mt = [&](int t) { return t % ntm; };
  auto t_b = [&](int t) { return SEG ? t / (ntm * ntn) : (t / ntm) % p.B; };
  auto t_nt = [&](int t) { return SEG ? (t / ntm) % ntn : t / (ntm * p.B); };
  constexpr bool FAST_SIN = C::BF;

  // statistics partials: lane = column l32 of tile ni, summed over the frames of its half (hi)
  float st_s[WN], st_q[WN];
#pragma unroll
  for (int ni = 0; ni < WN; ++ni) st_s[ni] = st_q[ni] = 0.f;

  int cur_nt = -1, cur_b = -1;

  // per-wave flush of the register statistics (no block barrier): the two frame halves
  // combine across lanes l and l^32, then one fp64 atomic pair per (wave, column)
  auto flush_stats = [&](int nt, int b) {
#pragma unroll
    for (int ni = 0; ni < WN; ++ni) {
      const float a = st_s[ni] + __shfl_xor(st_s[ni], 32);
      const float q = st_q[ni] + __shfl_xor(st_q[ni], 32);
      const int n = nt * BN + (wn * WN + ni) * 32 + l32;
      if (hi == 0 && n < p.N) {
        const int co = n % p.Cout;
        double* sb = stats_slot(p, blockIdx.x);
        fx_add(sb + ((size_t)b * p.stats_ld + co) * ST_W, a);
        fx_add(sb + ((size_t)b * p.stats_ld + co) * ST_W + 2, q);
      }
      st_s[ni] = st_q[ni] = 0.f;
    }
  };

  const Rsrc rw = make_rsrc(p.w, (unsigned)((size_t)C::SPL * p.nchunks * p.KS * BK * Np * sizeof(MT)));
  auto stage_w = [&](int c, int tap0, int ntap, MT* dst, int n0) {
    if constexpr (C::BF) {  // packed bf16: [chunk][tap][Np][32]
      const int units = ntap * BN * 4;
      for (int u = tid; u < units; u += NT) {
        const int tl = u / (BN * 4), rem = u % (BN * 4), n = rem >> 2, g = rem & 3;
        const int gn = n0 + n;
        const int gp = g ^ ((gn >> 2) & 3);  // swizzled packed layout (st_pack_conv)
        const unsigned off = gn < Np ? (unsigned)(((((size_t)c * p.KS + tap0 + tl) * Np + gn) * BK + 8 * gp) * 2) : OOB;
        *reinterpret_cast<uint4*>(dst + (size_t)tl * W_TAP + n * WPITCH + 8 * g) = bload16(rw, off);
        if constexpr (C::SPLIT)
          *reinterpret_cast<uint4*>(dst + wlo + (size_t)tl * W_TAP + n * WPITCH + 8 * g) =
              bload16(rw, off == OOB ? OOB : off + wlo_bytes);
      }
    } else {  // packed fp32: [chunk][tap][32][Np]
      const int units = ntap * BK * (BN / 4);
      for (int u = tid; u < units; u += NT) {
        const int tl = u / (BK * (BN / 4)), rem = u % (BK * (BN / 4)), k = rem / (BN / 4), g = rem % (BN / 4);
        const int gn = n0 + 4 * g;
        const unsigned off = gn < Np ? (unsigned)(((((size_t)c * p.KS + tap0 + tl) * BK + k) * Np + gn) * 4) : OOB;
        *reinterpret_cast<uint4*>(dst + (size_t)tl * W_TAP + k * WPITCH + 4 * g) = bload16(rw, off);
      }
    }
  };

  // ---- streamed weights (layers whose packed weights exceed the LDS budget): tap groups are
  // software-pipelined through registers like the input window — group g+1's loads are issued
  // right after group g is written to LDS, so the L2 latency hides under group g's MFMAs.
  constexpr int MAXW = 4;  // 16-byte W units per thread per group (launch_cfg sizes tg to fit)
  constexpr int MAXW2 = MAXW * C::SPL;  // split mode: the lo units follow
  auto issue_w = [&](int t, int c, int tap0, uint4 (&wpre)[MAXW2]) {
    const int n0 = t_nt(t) * BN;
    const int ntap = min(p.tg, p.KS - tap0);
#pragma unroll
    for (int k = 0; k < MAXW; ++k) {
      const int u = tid + k * NT;
      unsigned off = OOB;
      if constexpr (C::BF) {
        const int tl = u / (BN * 4), rem = u % (BN * 4), n = rem >> 2, g = rem & 3;
        const int gn = n0 + n;
        if (tl < ntap && gn < Np)
          off = (unsigned)(((((size_t)c * p.KS + tap0 + tl) * Np + gn) * BK + 8 * (g ^ ((gn >> 2) & 3))) * 2);
      } else {
        const int tl = u / (BK * (BN / 4)), rem = u % (BK * (BN / 4)), kq = rem / (BN / 4), g = rem % (BN / 4);
        const int gn = n0 + 4 * g;
        if (tl < ntap && gn < Np)
          off = (unsigned)(((((size_t)c * p.KS + tap0 + tl) * BK + kq) * Np + gn) * 4);
      }
      wpre[k] = bload16(rw, off);
      if constexpr (C::SPLIT) wpre[MAXW + k] = bload16(rw, off == OOB ? OOB : off + wlo_bytes);
    }
  };
  auto put_w = [&](int ntap, const uint4 (&wpre)[MAXW2], MT* Wd) {
#pragma unroll
    for (int k = 0; k < MAXW; ++k) {
      const int u = tid + k * NT;
      if constexpr (C::BF) {
        const int tl = u / (BN * 4), rem = u % (BN * 4), n = rem >> 2, g = rem & 3;
        if (tl < ntap) *reinterpret_cast<uint4*>(Wd + (size_t)tl * W_TAP + n * WPITCH + 8 * g) = wpre[k];
        if constexpr (C::SPLIT)
          if (tl < ntap) *reinterpret_cast<uint4*>(Wd + wlo + (size_t)tl * W_TAP + n * WPITCH + 8 * g) = wpre[MAXW + k];
      } else {
        const int tl = u / (BK * (BN / 4)), rem = u % (BK * (BN / 4)), kq = rem / (BN / 4), g = rem % (BN / 4);
        if (tl < ntap) *reinterpret_cast<uint4*>(Wd + (size_t)tl * W_TAP + kq * WPITCH + 4 * g) = wpre[k];
      }
    }
  };

  // ---- input-window staging, software-pipelined over (tile, chunk) steps: the raw loads of
  // step s+1 are issued into registers right after step s's window is written to LDS, so HBM
  // latency hides under step s's MFMAs and epilogue.
  // prefetched 8-channel units per thread (two sets in flight); the rest load synchronously.
  // Sized for a 'same' window of BM + a few rows; the strided config (iSTFTNet noise_convs)
  // has windows of ~6 BM rows.
  // (4, 1, 1, 1) is the stride-2 narrow-N tile (BM 128 x BN 32, windows of ~2 BM rows): 6 units as well.
  constexpr int MAXU = (!C::BF || (WAVES_M == 2 && WAVES_N == 2) || (WAVES_M == 4 && WAVES_N == 1 && WM == 1))
                           ? 6
                           : (BM * 4 + NT - 1) / NT + 1;
  const int units = R * 4;
  // every unit of a thread is the same 8-channel group: u = tid + k*NT, NT % 4 == 0
  const int g8 = tid & 3;

  // the utterance and channel offset chunk c of utterance b loads from (tx_H: the time-expanded MSD input)
  auto src_of = [&](int b, int c, int& bb, int& cx) __attribute__((always_inline)) {
    bb = b;
    cx = c * BK;
    if (p.tx_H) {
      const int h = b % p.tx_H + c - 1;
      const bool ok = (unsigned)h < (unsigned)p.tx_H;
      bb = ok ? b + c - 1 : b;
      cx = ok ? 0 : -1;  // -1: the whole chunk is the expansion's zero row
    }
  };
  auto issue = [&](int t, int c, typename RawT<T>::type (&pre)[MAXU]) {
    const int mt = t_mt(t), b = t_b(t);
    int bb, cx;
    src_of(b, c, bb, cx);
    const T* xb = reinterpret_cast<const T*>(p.x) + (size_t)bb * p.x_bs;
    const Rsrc rx = make_rsrc(xb, (unsigned)((size_t)p.Lin * p.x_ld * sizeof(T)));
    const int gr0 = mt * BM * p.stride - p.pad;
#pragma unroll
    for (int k = 0; k < MAXU; ++k) {
      const int u = tid + k * NT;
      const int r = u >> 2;
      const int gr = gr0 + r, ch = cx + 8 * g8;
      const unsigned e = (u < units && cx >= 0) ? (unsigned)(gr * p.x_ld + ch) : OOB;  // gr < 0 wraps: OOB
      bload_raw(rx, e, pre[k], (const T*)nullptr);
    }
  };

  // prologue coefficients of this thread's 8 channels, loaded once per step
  struct Coef8 { f2v a[4], m[4], al[4], ia[4]; };
  auto load_coef = [&](int ci0, Coef8& k) {
    const int ch = ci0 + 8 * g8;
    float t0[8], t1[8];
    if (mode & PRO_AFFINE) {
      ld8_lds(coef + ch, t0);
      ld8_lds(coef + cinp + ch, t1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        k.m[i] = f2v{t0[2 * i], t0[2 * i + 1]};
        k.a[i] = f2v{t1[2 * i], t1[2 * i + 1]};
      }
    }
    if (mode & PRO_SNAKE) {
      ld8_lds(coef + 2 * cinp + ch, t0);
      ld8_lds(coef + 3 * cinp + ch, t1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        k.al[i] = f2v{t0[2 * i], t0[2 * i + 1]};
        k.ia[i] = f2v{t1[2 * i], t1[2 * i + 1]};
      }
    }
  };

  auto put = [&](int u, float (&v)[8], bool ok, int ci0, const Coef8& k, MT* Xd) {
    const int r = u >> 2;
    const int ch = ci0 + 8 * g8;
    if (ok) {
      f2v x[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) x[i] = f2v{v[2 * i], v[2 * i + 1]};
      if (mode & PRO_AFFINE) {
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] = __builtin_elementwise_fma(x[i], k.a[i], k.m[i]);  // x*a + (beta - mean*a)
      }
      if (mode & PRO_SNAKE) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if constexpr (FAST_SIN) {  // v_sin_f32 takes revolutions: coef holds alpha / 2pi
            const f2v t = x[i] * k.al[i];
            const f2v sn = f2v{__builtin_amdgcn_sinf(t.x), __builtin_amdgcn_sinf(t.y)};
            x[i] = __builtin_elementwise_fma(sn * sn, k.ia[i], x[i]);
          } else {
            x[i] = f2v{snake_f<false>(x[i].x, k.al[i].x, k.ia[i].x), snake_f<false>(x[i].y, k.al[i].y, k.ia[i].y)};
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[2 * i] = x[i].x;
        v[2 * i + 1] = x[i].y;
      }
      if (mode & PRO_LRELU) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = v[j] > 0.f ? v[j] : v[j] * p.pro.slope;
      }
      if (ch + 8 > p.Cin) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (ch + j >= p.Cin) v[j] = 0.f;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = 0.f;
    }
    MT* dst = Xd + r * XP + 8 * g8;
    if constexpr (C::SPLIT) {  // hi = bf16(v) (round to nearest even), lo = bf16(v - hi): v - hi is exact
      bf16x8 o, ol;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o[j] = (bf16_t)v[j];
        ol[j] = (bf16_t)(v[j] - (float)o[j]);
      }
      *reinterpret_cast<bf16x8*>(dst) = o;
      *reinterpret_cast<bf16x8*>(dst + xs_el) = ol;
    } else if constexpr (C::BF) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16_t)v[j];
      *reinterpret_cast<bf16x8*>(dst) = o;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) dst[j] = v[j];
    }
  };

  auto write_x = [&](int t, int c, const typename RawT<T>::type (&pre)[MAXU], MT* Xd) {
    const int ci0 = c * BK;
    const int gr0 = t_mt(t) * BM * p.stride - p.pad;
    Coef8 k;
    load_coef(ci0, k);
#pragma unroll
    for (int kk = 0; kk < MAXU; ++kk) {
      const int u = tid + kk * NT;
      const int gr = gr0 + (u >> 2);
      float v[8];
      raw_to_f32(pre[kk], v);
      // conv zero padding applies to the post-prologue activation
      if (u < units) put(u, v, gr >= 0 && gr < p.Lin, ci0, k, Xd);
    }
    if (units > MAXU * NT) {  // large windows (2-D style convs): synchronous remainder
      int bb, cx;
      src_of(t_b(t), c, bb, cx);
      const T* xb = reinterpret_cast<const T*>(p.x) + (size_t)bb * p.x_bs;
      const Rsrc rx = make_rsrc(xb, (unsigned)((size_t)p.Lin * p.x_ld * sizeof(T)));
      for (int u = tid + MAXU * NT; u < units; u += NT) {
        const int r = u >> 2;
        const int gr = gr0 + r, ch = cx + 8 * g8;
        typename RawT<T>::type raw;
        bload_raw(rx, cx >= 0 ? (unsigned)(gr * p.x_ld + ch) : OOB, raw, (const T*)nullptr);
        float v[8];
        raw_to_f32(raw, v);
        put(u, v, gr >= 0 && gr < p.Lin, ci0, k, Xd);
      }
    }
  };

  f32x16 acc[WM][WN];
  constexpr bool PREF = !NARROW && WM * WN <= 2;
  struct Raw16 {
    typename RawT<T>::type a, b;
  };
  Raw16 rres[PREF ? WM : 1][PREF ? WN : 1], racc[PREF ? WM : 1][PREF ? WN : 1];
  const int npt = (p.nchunks + cps - 1) / cps;  // steps per tile
  const int nsteps = (tend - tbeg) * npt;
  // Two register sets (A, B).  cps == 1: the window / weight loads of step s+2 are issued while
  // step s is staged (A and B alternate).  cps == 2: a step stages chunks c (A) and c+1 (B) and
  // issues the next step's two chunks, so each load still has a full step of MFMAs to land.
  constexpr int PD = cps == 2 ? 1 : 2;
  auto st_tile = [&](int st) { return tbeg + st / npt; };
  auto st_chunk = [&](int st) { return (st % npt) * cps; };
  typename RawT<T>::type preA[MAXU], preB[MAXU];
  uint4 wpA[MAXW2], wpB[MAXW2];
  if (nsteps > 0) {
    issue(tbeg, 0, preA);
    if (!resident) issue_w(tbeg, 0, 0, wpA);
    if constexpr (cps == 2) {
      issue(tbeg, 1, preB);
      if (!resident) issue_w(tbeg, 1, 0, wpB);
    } else if (nsteps > 1) {
      issue(st_tile(1), st_chunk(1), preB);
      if (!resident) issue_w(st_tile(1), st_chunk(1), 0, wpB);
    }
  }
  // always_inline: left to itself the compiler outlines the fp32 instantiations' step into a
  // called function, which puts the register sets (passed by reference) in scratch memory
  auto step = [&](int st, typename RawT<T>::type (&pre)[MAXU], uint4 (&wpre)[MAXW2],
                  typename RawT<T>::type (&pre2)[MAXU], uint4 (&wpre2)[MAXW2]) __attribute__((always_inline)) {
    const int t = st_tile(st), c = st_chunk(st);
    const bool last = c + cps >= p.nchunks;     // the tile's epilogue follows this step
    const bool has2 = cps == 2 && c + 1 < p.nchunks;
    const int mt = t_mt(t);
    const int b = t_b(t);
    const int nt = t_nt(t);
    const int q0 = mt * BM, n0 = nt * BN;

    if (c == 0) {
      if (nt != cur_nt || b != cur_b) {
        if (cur_nt >= 0 && p.stats) flush_stats(cur_nt, cur_b);
        __syncthreads();
        if (b != cur_b) {  // AdaIN / Snake coefficients of this utterance, all input channels
          for (int ci = tid; ci < cinp; ci += NT) {
            float m = 0.f, a = 1.f, be = 0.f, al = 1.f;
            if (ci < p.Cin) {
              if (mode & PRO_AFFINE) adain_coeffs(p.pro, b, ci, m, a, be);
              if (mode & PRO_SNAKE) al = p.pro.alpha[ci];
            }
            coef[ci] = be - m * a;   // x * a + (beta - mean * a)  ==  (x - mean) * a + beta
            coef[cinp + ci] = a;
            coef[2 * cinp + ci] = FAST_SIN ? al * 0.15915494309189535f : al;  // bf16: alpha in revolutions
            coef[3 * cinp + ci] = 1.0f / al;  // the reference's (1 / alpha), once per channel
          }
        }
        if (nt != cur_nt) {
          for (int cc = tid; cc < BN; cc += NT) {
            const int n = n0 + cc;
            bias_s[cc] = (p.bias && n < p.N) ? p.bias[n % p.Cout] : 0.f;
          }
          if (resident)
            for (int cc = 0; cc < p.nchunks; ++cc) stage_w(cc, 0, p.KS, Ws + (size_t)cc * p.KS * W_TAP, n0);
        }
        cur_nt = nt;
        cur_b = b;
      }
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    }

    // residual / running-sum rows of this tile's epilogue: issued before the MFMAs so their
    // HBM latency hides under them (small-channel configs, where the epilogue dominates)
    if constexpr (PREF) {
      if (last) {
        const Rsrc rr = make_rsrc(p.res ? reinterpret_cast<const T*>(p.res) + (size_t)b * p.res_bs : (const T*)p.y,
                                  p.res ? (unsigned)(p.res_bs * sizeof(T)) : 0u);
        const Rsrc ra = make_rsrc(p.accb ? reinterpret_cast<const T*>(p.accb) + (size_t)b * p.acc_bs : (const T*)p.y,
                                  p.accb ? (unsigned)(p.acc_bs * sizeof(T)) : 0u);
#pragma unroll
        for (int mi = 0; mi < WM; ++mi)
#pragma unroll
          for (int ni = 0; ni < WN; ++ni) {
            const int q = q0 + (wm * WM + mi) * 32 + l32;
            const int nb = n0 + (wn * WN + ni) * 32 + hi * 16;
            const int ph = nb / p.Cout, co0 = nb - ph * p.Cout;
            const int o = q * p.up + ph - p.opad;
            const bool ok = q < p.Lq && nb < p.N && o >= 0 && o < p.Lout;
            const int orow = o + p.y_row_off;
            const unsigned er = ok ? (unsigned)((orow >> p.res_shift) * p.res_ld + co0) : OOB;
            const unsigned ea = ok ? (unsigned)(orow * p.acc_ld + co0) : OOB;
            bload_raw(rr, er, rres[mi][ni].a, (const T*)nullptr);
            bload_raw(rr, er + 8u, rres[mi][ni].b, (const T*)nullptr);
            bload_raw(ra, ea, racc[mi][ni].a, (const T*)nullptr);
            bload_raw(ra, ea + 8u, racc[mi][ni].b, (const T*)nullptr);
          }
      }
    }
    __syncthreads();  // previous readers of Xs (MFMA) are done; coef / bias / W visible
    // STTS_OPT_DEBUG (timing only, outputs wrong): 1 no window staging, 2 no MFMAs, 4 no
    // epilogue, 8 no window loads
    if (!(p.dbg & 1)) {
      write_x(t, c, pre, Xs);
      if (has2) write_x(t, c + 1, pre2, Xs + xs_el);
    }
    if (st + PD < nsteps && !(p.dbg & 8)) {
      issue(st_tile(st + PD), st_chunk(st + PD), pre);
      if (cps == 2) issue(st_tile(st + 1), st_chunk(st + 1) + 1, pre2);
    }
    // ---- taps (weights resident, or staged in groups that fit the budget) ----
    for (int tap0 = 0; tap0 < p.KS; tap0 += resident ? p.KS : p.tg) {
      const int ntap = resident ? p.KS : min(p.tg, p.KS - tap0);
      const MT* wbase;
      const MT* wbase2;  // chunk c+1 (cps == 2; the launcher allows it with one tap group only)
      if (resident) {
        wbase = Ws + (size_t)c * p.KS * W_TAP;
        wbase2 = wbase + (size_t)p.KS * W_TAP;
      } else {
        if (tap0 > 0) __syncthreads();  // every wave is done reading the previous group
        put_w(ntap, wpre, Ws);
        if (has2) put_w(ntap, wpre2, Ws + (size_t)p.tg * W_TAP);
        if (tap0 + p.tg < p.KS) {
          issue_w(t, c, tap0 + p.tg, wpre);
        } else if (st + PD < nsteps) {
          issue_w(st_tile(st + PD), st_chunk(st + PD), 0, wpre);
          if (cps == 2) issue_w(st_tile(st + 1), st_chunk(st + 1) + 1, 0, wpre2);
        }
        wbase = Ws;
        wbase2 = Ws + (size_t)p.tg * W_TAP;
      }
      __syncthreads();
      if (p.dbg & 2) continue;
      for (int half = 0; half < (has2 ? 2 : 1); ++half) {
      const MT* Xc = half ? Xs + xs_el : Xs;
      const MT* wb = half ? wbase2 : wbase;
#pragma unroll 1
      for (int tl = 0; tl < ntap; ++tl) {
        const int tap = tap0 + tl;
        // 1-D convs (row_off == 0): no per-tap division on the scalar unit
        const int toff = p.row_off == 0 ? tap * p.dil : (tap / p.kw) * p.row_off + (tap % p.kw) * p.dil;
        const MT* wt = wb + (size_t)tl * W_TAP;
        if constexpr (C::SPLIT) {
#pragma unroll
          for (int kk = 0; kk < BK / 16; ++kk) {
            bf16x8 af[WM], bw[WN], afl[WM], bwl[WN];
#pragma unroll
            for (int mi = 0; mi < WM; ++mi) {
              const int r = (wm * WM + mi) * 32 + l32;
              const MT* xa = Xc + (r * p.stride + toff) * XP + kk * 16 + hi * 8;
              af[mi] = *reinterpret_cast<const bf16x8*>(xa);
              afl[mi] = *reinterpret_cast<const bf16x8*>(xa + xs_el);
            }
#pragma unroll
            for (int ni = 0; ni < WN; ++ni) {
              const int n = (wn * WN + ni) * 32 + l32;
              const MT* wa = wt + n * WPITCH + kk * 16 + hi * 8;
              bw[ni] = *reinterpret_cast<const bf16x8*>(wa);
              bwl[ni] = *reinterpret_cast<const bf16x8*>(wa + wlo);
            }
            // the two small cross terms first, then hi*hi (lo*lo, ~2^-18 of the product, is dropped)
#pragma unroll
            for (int mi = 0; mi < WM; ++mi)
#pragma unroll
              for (int ni = 0; ni < WN; ++ni) {
                acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bw[ni], afl[mi], acc[mi][ni], 0, 0, 0);
                acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bwl[ni], af[mi], acc[mi][ni], 0, 0, 0);
                acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bw[ni], af[mi], acc[mi][ni], 0, 0, 0);
              }
          }
        } else if constexpr (C::BF) {
#pragma unroll
          for (int kk = 0; kk < BK / 16; ++kk) {
            bf16x8 af[WM], bw[WN];
#pragma unroll
            for (int mi = 0; mi < WM; ++mi) {
              const int r = (wm * WM + mi) * 32 + l32;
              af[mi] = *reinterpret_cast<const bf16x8*>(Xc + (r * p.stride + toff) * XP + kk * 16 + hi * 8);
            }
#pragma unroll
            for (int ni = 0; ni < WN; ++ni) {
              const int n = (wn * WN + ni) * 32 + l32;
              bw[ni] = *reinterpret_cast<const bf16x8*>(wt + n * WPITCH + kk * 16 + hi * 8);
            }
#pragma unroll
            for (int mi = 0; mi < WM; ++mi)
#pragma unroll
              for (int ni = 0; ni < WN; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bw[ni], af[mi], acc[mi][ni], 0, 0, 0);
          }
        } else {
#pragma unroll 4
          for (int kk = 0; kk < BK / 2; ++kk) {
            float af[WM], bw[WN];
#pragma unroll
            for (int mi = 0; mi < WM; ++mi) {
              const int r = (wm * WM + mi) * 32 + l32;
              af[mi] = Xc[(r * p.stride + toff) * XP + 2 * kk + hi];
            }
#pragma unroll
            for (int ni = 0; ni < WN; ++ni) {
              const int n = (wn * WN + ni) * 32 + l32;
              bw[ni] = wt[(2 * kk + hi) * WPITCH + n];
            }
#pragma unroll
            for (int mi = 0; mi < WM; ++mi)
#pragma unroll
              for (int ni = 0; ni < WN; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(bw[ni], af[mi], acc[mi][ni], 0, 0, 0);
          }
        }
      }
      }
    }
    if (!last || (p.dbg & 4)) return;

    // ---------------- epilogue, straight from registers: lane = (frame, 16 channels) ----------------
    T* yT = reinterpret_cast<T*>(p.y) + (size_t)b * p.y_bs;
    float* yF = reinterpret_cast<float*>(p.y) + (size_t)b * p.y_bs;
    const T* resb = p.res ? reinterpret_cast<const T*>(p.res) + (size_t)b * p.res_bs : nullptr;
    const T* accb = p.accb ? reinterpret_cast<const T*>(p.accb) + (size_t)b * p.acc_bs : nullptr;
#pragma unroll
    for (int mi = 0; mi < WM; ++mi) {
#pragma unroll
      for (int ni = 0; ni < WN; ++ni) {
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = acc[mi][ni][r];
        const int q = q0 + (wm * WM + mi) * 32 + l32;
        const int nl = (wn * WN + ni) * 32 + hi * 16;  // first of this lane's 16 columns, in the tile
        const int nb = n0 + nl;
        // v becomes the stored values (0 where nothing is stored) for the statistics
        bool stored = false;
        if (q < p.Lq && nb < p.N) {
          if constexpr (!NARROW) {
            // 16 consecutive channels of one output frame (Cout % 16 == 0, vector loads/stores)
            const int ph = nb / p.Cout, co0 = nb - ph * p.Cout;
            const int o = q * p.up + ph - p.opad;
            if (o >= 0 && o < p.Lout) {
              const int orow = o + p.y_row_off;
              if (p.zc_period && (o % p.zc_period) >= p.zc_valid) {  // padded-image border column
#pragma unroll
                for (int j = 0; j < 16; ++j) v[j] = 0.f;
                if (p.y_f32) store16(yF + (size_t)orow * p.y_ld + co0, v);
                else store16(yT + (size_t)orow * p.y_ld + co0, v);
              } else {
                {
                  float bb[16];
                  ld8_lds(bias_s + nl, *reinterpret_cast<float(*)[8]>(&bb[0]));
                  ld8_lds(bias_s + nl + 8, *reinterpret_cast<float(*)[8]>(&bb[8]));
#pragma unroll
                  for (int i = 0; i < 8; ++i) pw(v, i, pr(v, i) + pr(bb, i));
                }
                if (p.reflect_front && o == 1) {  // iSTFTNet ReflectionPad1d((1,0)) (istftnet.py:538, 558-559)
                  float r[16];
                  load16(resb + co0, r);
#pragma unroll
                  for (int j = 0; j < 16; ++j) r[j] += v[j];
                  store16(yT + co0, r);
                  if (p.stats) {  // once per (utterance, channel): direct atomics
                    for (int j = 0; j < 16; ++j) {
                      const double x = to_f32(from_f32<T>(r[j]));
                      stat_add(p.stats + ((size_t)b * p.stats_ld + co0 + j) * ST_W, x, x * x);
                    }
                  }
                }
                if (resb) {
                  float r[16];
                  if constexpr (PREF) raw16_to_f32(rres[PREF ? mi : 0][PREF ? ni : 0], r);
                  else load16(resb + (size_t)(orow >> p.res_shift) * p.res_ld + co0, r);
                  const f2v sc = f2v{p.out_scale, p.out_scale};
#pragma unroll
                  for (int i = 0; i < 8; ++i) pw(v, i, (pr(v, i) + pr(r, i)) * sc);
                }
                if (accb) {
                  float r[16];
                  if constexpr (PREF) raw16_to_f32(racc[PREF ? mi : 0][PREF ? ni : 0], r);
                  else load16(accb + (size_t)orow * p.acc_ld + co0, r);
                  if (p.acc_div != 0.f) {
                    if constexpr (C::LOWP) {  // bf16 mode multiplies by the reciprocal
                      const float id = 1.0f / p.acc_div;
                      const f2v inv = f2v{id, id};
#pragma unroll
                      for (int i = 0; i < 8; ++i) pw(v, i, (pr(r, i) + pr(v, i)) * inv);
                    } else {  // the reference divides (xs / num_kernels)
#pragma unroll
                      for (int j = 0; j < 16; ++j) v[j] = (r[j] + v[j]) / p.acc_div;
                    }
                  } else {
#pragma unroll
                    for (int i = 0; i < 8; ++i) pw(v, i, pr(r, i) + pr(v, i));
                  }
                }
                if (p.epi_lrelu) {
#pragma unroll
                  for (int j = 0; j < 16; ++j) v[j] = v[j] > 0.f ? v[j] : v[j] * p.epi_slope;
                }
                if (p.epi_gelu) {  // nn.GELU() (erf form), Modules/vocos.py:48
#pragma unroll
                  for (int j = 0; j < 16; ++j) v[j] = 0.5f * v[j] * (1.0f + erff(v[j] * 0.7071067811865476f));
                }
                // y_f32: fp32 frames straight from the accumulators (the bf16 training convs, no conversion pass)
                if (p.y_f32) store16(yF + (size_t)orow * p.y_ld + co0, v);
                else store16(yT + (size_t)orow * p.y_ld + co0, v);
                if constexpr (!C::BF) {
#pragma unroll
                  for (int j = 0; j < 16; ++j) v[j] = to_f32(from_f32<T>(v[j]));
                }
                stored = true;
              }
            }
          } else {
            // narrow heads (conv_post N = 1 / 22, F0/N projections): per-element path
            stored = true;
            for (int j = 0; j < 16; ++j) {
              const int n = nb + j;
              float x = 0.f;
              if (n < p.N) {
                const int ph = n / p.Cout, co = n - ph * p.Cout;
                const int o = q * p.up + ph - p.opad;
                if (o >= 0 && o < p.Lout) {
                  const int orow = o + p.y_row_off;
                  x = v[j] + bias_s[nl + j];
                  if (resb) x = (x + to_f32(resb[(size_t)(orow >> p.res_shift) * p.res_ld + co])) * p.out_scale;
                  if (p.epi_tanh) x = tanhf(x);
                  if (p.epi_lrelu) x = x > 0.f ? x : x * p.epi_slope;
                  if (p.epi_gelu) x = 0.5f * x * (1.0f + erff(x * 0.7071067811865476f));
                  if (p.y_f32) {
                    yF[(size_t)orow * p.y_ld + co] = x;
                  } else {
                    const T tx = from_f32<T>(x);
                    yT[(size_t)orow * p.y_ld + co] = tx;
                    x = to_f32(tx);
                  }
                }
              }
              v[j] = x;
            }
          }
        }
        if (p.stats) {  // column pass over the wave scratch: lane = column l32, frames of half hi
          if (!stored) {
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = 0.f;
          }
#pragma unroll
          for (int j = 0; j < 16; j += 4)
            *reinterpret_cast<float4*>(ws + l32 * EP + hi * 16 + j) = make_float4(v[j], v[j + 1], v[j + 2], v[j + 3]);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          f2v a2 = f2v{0.f, 0.f}, q2 = f2v{0.f, 0.f};
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const f2v x = f2v{ws[(hi * 16 + r) * EP + l32], ws[(hi * 16 + r + 1) * EP + l32]};
            a2 += x;
            q2 = __builtin_elementwise_fma(x, x, q2);
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          st_s[ni] += a2.x + a2.y;
          st_q[ni] += q2.x + q2.y;
        }
      }
    }
  };
  if constexpr (cps == 2) {
    for (int st = 0; st < nsteps; ++st) step(st, preA, wpA, preB, wpB);
  } else {
    for (int st = 0; st < nsteps; st += 2) {
      step(st, preA, wpA, preB, wpB);
      if (st + 1 < nsteps) step(st + 1, preB, wpB, preA, wpA);
    }
  }
  if (cur_nt >= 0 && p.stats) flush_stats(cur_nt, cur_b);
  if constexpr (!SEG) break;  // (one range)
  __syncthreads();  // (the next range re-stages the LDS)
  }  // tile ranges
}

int g_num_cu = 0;

template <typename T, typename MT, int WAVES_M, int WAVES_N, int WM, int WN, bool NARROW = false, bool SPF = true>
int launch_cfg(ConvParams p, hipStream_t stream) {
  using C = ConvCfg<T, MT, WAVES_M, WAVES_N, WM, WN, SPF>;
  constexpr int LDS_MAX = 160 * 1024;
  constexpr int WBUDGET = 48 * 1024;
  constexpr int WRES_BUDGET = 120 * 1024;
  const size_t wtap = (size_t)C::SPL * C::W_TAP * sizeof(MT);
  // weights resident across tiles when every chunk x tap slice of the column tile fits
  const int nres = p.nchunks * p.KS;
  if ((size_t)nres * wtap <= (size_t)WRES_BUDGET && C::lds_bytes(p, nres) <= (size_t)LDS_MAX) {
    p.w_resident = 1;
    p.tg = p.KS;
  } else {
    p.w_resident = 0;
    // a tap group must fit the per-thread W prefetch registers (MAXW 16-byte units per thread)
    const int units_per_tap = C::BF ? C::BN * 4 : BK * (C::BN / 4);
    int tg = 4 * C::NT / units_per_tap;
    if ((size_t)tg * wtap > (size_t)WBUDGET) tg = (int)(WBUDGET / wtap);
    if (tg < 1) return ST_EINVAL;
    if (tg > p.KS) tg = p.KS;
    while (tg > 1 && C::lds_bytes(p, tg) > (size_t)LDS_MAX) --tg;
    p.tg = tg;
  }
  // two chunks per step (bf16 wide configs with one tap group, when the second window and weight
  // slice fit the LDS): half the barriers and twice the MFMAs between them
  p.cps = 1;
  if (C::LOWP && !NARROW && p.nchunks >= 2 && (p.w_resident || p.tg >= p.KS) &&
      C::lds_bytes(p, p.w_resident ? nres : 2 * p.tg, 2) <= (size_t)LDS_MAX)
    p.cps = 2;
  const size_t lds = C::lds_bytes(p, p.w_resident ? nres : p.cps * p.tg, p.cps);
  if (lds > (size_t)LDS_MAX) return ST_EINVAL;
  const int sg = st_seg_choice(p, 1, 1 << 20) > 0 ? 1 : 0;  // (a segmented launch; its seg count below)
  auto kern = sg ? conv1d_igemm_kernel<T, MT, WAVES_M, WAVES_N, WM, WN, NARROW, 1, SPF, true>
                 : conv1d_igemm_kernel<T, MT, WAVES_M, WAVES_N, WM, WN, NARROW, 1, SPF, false>;
  if constexpr (C::LOWP && !NARROW) {
    if (p.cps == 2)
      kern = sg ? conv1d_igemm_kernel<T, MT, WAVES_M, WAVES_N, WM, WN, NARROW, 2, SPF, true>
                : conv1d_igemm_kernel<T, MT, WAVES_M, WAVES_N, WM, WN, NARROW, 2, SPF, false>;
  }
  static bool attr_set[2][2] = {{false, false}, {false, false}};
  if (!attr_set[sg][p.cps - 1]) {
    ST_CHECK_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX));
    attr_set[sg][p.cps - 1] = true;
  }
  if (!g_num_cu) {
    int dev = 0;
    ST_CHECK_HIP(hipGetDevice(&dev));
    ST_CHECK_HIP(hipDeviceGetAttribute(&g_num_cu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  int per_cu = occupancy_cached((const void*)kern, C::NT, lds);
  if (per_cu < 1) per_cu = 1;
  const long long ntn = (p.N + C::BN - 1) / C::BN, ntm = (p.Lq + C::BM - 1) / C::BM;
  const long long tiles = ntn * ntm * p.B;
  if (tiles <= 0) return ST_OK;
  if (tiles > 0x7fffffffLL) return ST_EINVAL;
  ConvParams q = p;
  q.seg = sg ? st_seg_choice(p, 1, g_num_cu * per_cu) : 0;
  const long long nvb = q.seg ? (long long)p.B * q.seg : tiles;
  long long grid = (long long)g_num_cu * per_cu;
  if (grid > nvb) grid = nvb;
  if (g_opt_grid_cap > 0 && grid > g_opt_grid_cap) grid = g_opt_grid_cap;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(C::NT), lds, stream, q);
  return (int)hipGetLastError();
}

template <typename T, typename MT, bool SPF = true>
int launch_typed(const ConvParams& p, hipStream_t stream) {
  const bool narrow = (p.Cout % 16 != 0) || (p.y_ld % 8 != 0) || (p.res && p.res_ld % 8 != 0) ||
                      (p.accb && p.acc_ld % 8 != 0);
  if (!narrow && p.y_f32 && p.reflect_front) return ST_EINVAL;  // the reflect row stores T
  if (narrow) {
    // per-element epilogue: residual/scale/tanh supported; accumulate/reflect/zero-columns are not
    if (p.accb || p.reflect_front || p.zc_period || p.N > 32 || p.stride > 1) return ST_EINVAL;
    return launch_cfg<T, MT, 4, 1, 2, 1, true, SPF>(p, stream);
  }
  if (p.epi_tanh) return ST_EINVAL;  // tanh only on narrow heads
  // stride 2 with N <= 32 (the MSD (3, 9) layers of the training step, N = 32): BM 128 x BN 32, every
  // column live, instead of the 64 x 128 tile with three quarters of its columns idle (STTS_OPT_EXP 1024:
  // the old tile, for A/B)
  if constexpr (ConvCfg<T, MT, 1, 1, 1, 1, SPF>::LOWP) {
    if (p.stride == 2 && p.N <= 32 && !(g_opt_exp & 1024)) return launch_cfg<T, MT, 4, 1, 1, 1, false, SPF>(p, stream);
  }
  if (p.stride > 1) return launch_cfg<T, MT, 2, 2, 1, 2, false, SPF>(p, stream);  // BM 64 x BN 128 (short window)
  if (p.N > 64 && g_opt_small_tiles) {
    // few tiles (small batches: the 400-frame front-end at B = 1 makes 16 tiles of 256 x 128 for 256
    // CUs): BM 64 x BN 128 tiles, 4x the workgroups
    const long long big = (long long)((p.N + 127) / 128) * ((p.Lq + 255) / 256) * p.B;
    const int ncu = g_num_cu ? g_num_cu : 256;
    if (big < ncu / 2) return launch_cfg<T, MT, 2, 2, 1, 2, false, SPF>(p, stream);
  }
  if (p.N <= 32) return launch_cfg<T, MT, 4, 1, 2, 1, false, SPF>(p, stream);     // BM 256 x BN 32, 4 waves
  if constexpr (std::is_same<T, float>::value) {
    // fp32 frames (parity mode, split, ST_BF16F): 4-wave tiles, so a wave may hold its fp32 windows and weight
    // slices (split: hi and lo) in up to 512 registers (the 8-wave tiles are capped at 256 and spill)
    if (p.N <= 64) return launch_cfg<T, MT, 2, 2, 2, 1, false, SPF>(p, stream);   // BM 128 x BN 64
    return launch_cfg<T, MT, 2, 2, 2, 2, false, SPF>(p, stream);                  // BM 128 x BN 128
  } else {
    // BM 256 x BN 64, 8 waves.  (N = 192 keeps BN 128: the window prologue is paid per tile, so
    // three 64-column tiles measured slower than a half-empty 128-column one.)
    if (p.N <= 64) return launch_cfg<T, MT, 8, 1, 1, 2, false, SPF>(p, stream);
    return launch_cfg<T, MT, 4, 2, 2, 2, false, SPF>(p, stream);                  // BM 256 x BN 128, 8 waves
  }
}

}  // namespace

int g_opt_resconv = 1;
int g_opt_small_tiles = 1;
int g_opt_resfused = 0;
int g_opt_grid_cap = 0;
int g_opt_segpart = 1;

// (only launches that keep InstanceNorm statistics: a conv's outputs do not depend on the tile -> workgroup split, its
// statistics' fp32 partials do.  A plain launch over many short rows — the discriminators' reshaped batches — would
// otherwise get mostly empty segments, each re-staging the layer's weights: 2.3x slower igemm in the training step)
int st_seg_choice(const ConvParams& p, int upu, int gmax) {
  const int B = p.B;
  if (!g_opt_segpart || !p.stats || B < 32 || B % 32 || upu <= 0) return 0;
  const int seg = gmax / (32 * upu);
  return seg >= 1 ? seg : 0;
}
int g_opt_debug = 0;
int g_opt_head = 1;
unsigned long long* g_dbg_stamps = nullptr;  // stts_set_debug_buffer

int st_conv1d_engine(const ConvParams& p, int dtype) {
  ConvParams q = p;
  if (q.kw <= 0) q.kw = q.KS;
  if (q.tx_H) return ST_ENGINE_IGEMM;
  if (g_opt_head && st_head_eligible(q)) return ST_ENGINE_HEAD;
  if (st_front_eligible(q, dtype) || st_ups_eligible(q, dtype)) return ST_ENGINE_BIGCONV;
  if (st_resconv_ups_eligible(q, dtype)) return ST_ENGINE_RESCONV;
  if (st_big64_eligible(q, dtype)) return dtype == ST_SPLIT ? ST_ENGINE_BIGSPLIT : ST_ENGINE_BIGCONV;
  if (g_opt_resconv && st_resconv_eligible(q, dtype)) return ST_ENGINE_RESCONV;
  if (g_opt_resconv && st_bigconv_eligible(q, dtype)) return ST_ENGINE_BIGCONV;
  if (st_pw_split_eligible(q, dtype) || st_pw_eligible(q, dtype)) return ST_ENGINE_PW;
  if (st_ressplit_eligible(q, dtype)) return ST_ENGINE_RESSPLIT;
  if (st_bigsplit_eligible(q, dtype)) return ST_ENGINE_BIGSPLIT;
  return ST_ENGINE_IGEMM;
}

int st_conv1d(const ConvParams& p, int dtype, hipStream_t stream) {
  if (p.B <= 0 || p.Lq <= 0 || p.N <= 0) return ST_OK;
  if (p.KS <= 0 || p.stride <= 0 || p.dil <= 0 || p.Cout <= 0 || p.up <= 0) return ST_EINVAL;
  if (p.x_ld % 8 != 0 || p.nchunks * BK < p.Cin) return ST_EINVAL;
  ConvParams q = p;
  if (q.kw <= 0) q.kw = q.KS;
  q.dbg = g_opt_debug;
  q.stamps = g_dbg_stamps;
  if (q.tx_H) {  // the time-expanded MSD input: general engine only (chunk dh = one 32-channel chunk)
    if (q.tx_H < 1 || q.nchunks != 3 || q.Cin != 96 || q.x_ld != 32 || q.B % q.tx_H) return ST_EINVAL;
    if (dtype == ST_FP32) return launch_typed<float, float>(q, stream);
    if (dtype == ST_BF16) return launch_typed<bf16_t, bf16_t>(q, stream);
    if (dtype == ST_SPLIT) return launch_typed<float, bf16_t, true>(q, stream);
    if (dtype == ST_BF16F) return launch_typed<float, bf16_t, false>(q, stream);
    return ST_EDTYPE;
  }
  if (g_opt_head && st_head_eligible(q)) return st_head(q, dtype, stream);
  if (st_front_eligible(q, dtype)) return st_bigconv2_front(q, stream);
  if (st_ups_eligible(q, dtype)) return st_bigconv2_ups(q, stream);
  if (st_resconv_ups_eligible(q, dtype)) return st_resconv_ups(q, stream);
  if (st_big64_eligible(q, dtype)) return st_big64(q, dtype, stream);
  if (g_opt_resconv && st_resconv_eligible(q, dtype)) return st_resconv(q, stream);
  if (g_opt_resconv && st_bigconv_eligible(q, dtype)) return st_bigconv(q, stream);
  if (st_pw_split_eligible(q, dtype)) return st_pw_split(q, stream);
  if (st_pw_eligible(q, dtype)) return st_pw(q, stream);
  if (st_ressplit_eligible(q, dtype)) return st_ressplit(q, stream);
  if (st_bigsplit_eligible(q, dtype)) return st_bigsplit(q, stream);
  if (dtype == ST_FP32) return launch_typed<float, float>(q, stream);
  if (dtype == ST_BF16) {
    return launch_typed<bf16_t, bf16_t>(q, stream);
  }
  if (dtype == ST_SPLIT) return launch_typed<float, bf16_t, true>(q, stream);
  if (dtype == ST_BF16F) return launch_typed<float, bf16_t, false>(q, stream);
  return ST_EDTYPE;
}
