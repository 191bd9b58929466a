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
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int BK = 32;
constexpr int EP = 36;  // epilogue transpose pitch (floats): conflict-free b128 row reads

template <typename MT> struct Layout;
template <> struct Layout<bf16_t> {
  static constexpr int XP = 40;  // X row pitch (bf16) = 80 B: conflict-free ds_read_b128
  static constexpr int WP = 40;  // W: [tap][n][WP]
};
template <> struct Layout<float> {
  static constexpr int XP = 33;  // odd pitch: conflict-free ds_read_b32 column reads
  static constexpr int WP = 0;   // W: [tap][k][BN]
};

template <typename T, typename MT, int WAVES_M, int WAVES_N, int WM, int WN>
struct ConvCfg {
  static constexpr bool BF = std::is_same<MT, bf16_t>::value;
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
  // LDS carve (bytes): [coef 4 x cinp f32][X window | epilogue scratch][W slices]
  __host__ __device__ static int cinp(const ConvParams& p) { return p.nchunks * BK; }
  __host__ __device__ static size_t coef_bytes(const ConvParams& p) { return (size_t)4 * cinp(p) * 4; }
  __host__ __device__ static size_t xs_bytes(const ConvParams& p) {
    size_t x = (((size_t)rows(p) * XP * sizeof(MT)) + 15) & ~(size_t)15;
    const size_t ep = (size_t)NW * 32 * EP * 4;
    const size_t red = (size_t)WAVES_M * BN * 2 * 4;
    x = x > ep ? x : ep;
    return x > red ? x : red;
  }
  static size_t lds_bytes(const ConvParams& p, int nwslices) {
    return coef_bytes(p) + xs_bytes(p) + (size_t)nwslices * W_TAP * sizeof(MT);
  }
};

template <bool FAST>
__device__ __forceinline__ float snake_f(float v, float al, float inv_al) {
  const float s = FAST ? __sinf(al * v) : sinf(al * v);
  return v + inv_al * (s * s);
}

// Branch-free loads through a buffer descriptor: out-of-range offsets (negative rows wrap to
// huge unsigned values) return 0 from the hardware range check, so every prefetch is issued
// unconditionally and hipcc keeps counted vmcnt waits (a per-lane `if (ok) load` makes it
// branch around each load and drain vmcnt(0): cdna_hip_programming.md §5 trap (c)).
typedef __amdgpu_buffer_rsrc_t Rsrc;
__device__ __forceinline__ Rsrc make_rsrc(const void* base, unsigned bytes) {
  const unsigned long long a = (unsigned long long)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  void* pb = (void*)(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(pb, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
constexpr unsigned OOB = 0x80000000u;  // an offset beyond every descriptor used here
__device__ __forceinline__ uint4 bload16(Rsrc r, unsigned off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  uint4 o;
  __builtin_memcpy(&o, &v, 16);
  return o;
}

template <typename T> struct RawT;
template <> struct RawT<bf16_t> { using type = uint4; };
struct F8 { float4 a, b; };
template <> struct RawT<float> { using type = F8; };
__device__ __forceinline__ uint4 load_raw(const bf16_t* p) { return *reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ F8 load_raw(const float* p) {
  return F8{*reinterpret_cast<const float4*>(p), *reinterpret_cast<const float4*>(p + 4)};
}
// 8 elements at element offset `e` (OOB when e is out of range of the descriptor)
__device__ __forceinline__ void bload_raw(Rsrc r, unsigned e, uint4& out, const bf16_t*) {
  out = bload16(r, e >= OOB / 2 ? OOB : e * 2u);
}
__device__ __forceinline__ void bload_raw(Rsrc r, unsigned e, F8& out, const float*) {
  const unsigned o = e >= OOB / 4 ? OOB : e * 4u;
  const uint4 a = bload16(r, o), b = bload16(r, o + 16u);
  __builtin_memcpy(&out.a, &a, 16);
  __builtin_memcpy(&out.b, &b, 16);
}
__device__ __forceinline__ void raw_to_f32(const uint4& r, float (&v)[8]) {
  bf16x8 b;
  __builtin_memcpy(&b, &r, 16);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (float)b[j];
}
__device__ __forceinline__ void raw_to_f32(const F8& r, float (&v)[8]) {
  v[0] = r.a.x; v[1] = r.a.y; v[2] = r.a.z; v[3] = r.a.w; v[4] = r.b.x; v[5] = r.b.y; v[6] = r.b.z; v[7] = r.b.w;
}
template <typename R>
__device__ __forceinline__ void raw16_to_f32(const R& r, float (&v)[16]) {
  float a[8], b[8];
  raw_to_f32(r.a, a);
  raw_to_f32(r.b, b);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    v[j] = a[j];
    v[8 + j] = b[j];
  }
}
__device__ __forceinline__ void ld8_lds(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

template <typename T>
__device__ __forceinline__ void load16(const T* p, float (&v)[16]) {
  float a[8], b[8];
  load8(p, a);
  load8(p + 8, b);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    v[j] = a[j];
    v[8 + j] = b[j];
  }
}

__device__ __forceinline__ void store16(float* p, const float (&v)[16]) {
#pragma unroll
  for (int j = 0; j < 16; j += 4) *reinterpret_cast<float4*>(p + j) = make_float4(v[j], v[j + 1], v[j + 2], v[j + 3]);
}
__device__ __forceinline__ void store16(bf16_t* p, const float (&v)[16]) {
  bf16x8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = (bf16_t)v[j];
    b[j] = (bf16_t)v[8 + j];
  }
  *reinterpret_cast<bf16x8*>(p) = a;
  *reinterpret_cast<bf16x8*>(p + 8) = b;
}

template <typename T, typename MT, int WAVES_M, int WAVES_N, int WM, int WN, bool NARROW>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N) conv1d_igemm_kernel(const ConvParams p) {
  using C = ConvCfg<T, MT, WAVES_M, WAVES_N, WM, WN>;
  constexpr int BM = C::BM, BN = C::BN, XP = C::XP, WPITCH = C::WPITCH, W_TAP = C::W_TAP, NT = C::NT;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int R = C::rows(p);
  const int cinp = C::cinp(p);
  float* coef = reinterpret_cast<float*>(smem);  // [4][cinp]: beta - mean*a, a, alpha, 1/alpha
  MT* Xs = reinterpret_cast<MT*>(smem + C::coef_bytes(p));
  float* scr = reinterpret_cast<float*>(Xs);     // epilogue scratch / stats reduction (aliases X)
  MT* Ws = reinterpret_cast<MT*>(smem + C::coef_bytes(p) + C::xs_bytes(p));

  const int ntn = (p.N + BN - 1) / BN;
  const int ntm = (p.Lq + BM - 1) / BM;
  const long long total = (long long)ntn * ntm * p.B;
  const int tbeg = (int)(total * blockIdx.x / gridDim.x);
  const int tend = (int)(total * (blockIdx.x + 1) / gridDim.x);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WAVES_N, wn = wid % WAVES_N;
  const int l32 = lane & 31, hi = lane >> 5;
  const int Np = (p.N + 31) & ~31;
  const int mode = p.pro.mode;
  const bool resident = p.w_resident != 0;
  constexpr bool FAST_SIN = C::BF;

  // statistics partials: lane = one output column (l32 of tile ni), rows of its half (hi)
  float st_s[WN], st_q[WN];
#pragma unroll
  for (int ni = 0; ni < WN; ++ni) st_s[ni] = st_q[ni] = 0.f;

  int cur_nt = -1, cur_b = -1;

  // flush the register statistics of column tile `nt` / utterance `b` (block-uniform call)
  auto flush_stats = [&](int nt, int b) {
    __syncthreads();
    // lanes l and l^32 hold the two row halves of the same column
#pragma unroll
    for (int ni = 0; ni < WN; ++ni) {
      const float a = st_s[ni] + __shfl_xor(st_s[ni], 32);
      const float q = st_q[ni] + __shfl_xor(st_q[ni], 32);
      if (hi == 0) {
        const int nl = (wn * WN + ni) * 32 + l32;
        scr[((size_t)wm * BN + nl) * 2 + 0] = a;
        scr[((size_t)wm * BN + nl) * 2 + 1] = q;
      }
      st_s[ni] = st_q[ni] = 0.f;
    }
    __syncthreads();
    for (int c = tid; c < BN; c += NT) {
      const int n = nt * BN + c;
      if (n < p.N) {
        double a = 0.0, q = 0.0;
#pragma unroll
        for (int w = 0; w < WAVES_M; ++w) {
          a += scr[((size_t)w * BN + c) * 2 + 0];
          q += scr[((size_t)w * BN + c) * 2 + 1];
        }
        const int co = n % p.Cout;
        atomicAdd(p.stats + ((size_t)b * p.stats_ld + co) * 2 + 0, a);
        atomicAdd(p.stats + ((size_t)b * p.stats_ld + co) * 2 + 1, q);
      }
    }
  };

  const Rsrc rw = make_rsrc(p.w, (unsigned)((size_t)p.nchunks * p.KS * BK * Np * sizeof(MT)));
  auto stage_w = [&](int c, int tap0, int ntap, MT* dst, int n0) {
    if constexpr (C::BF) {  // packed bf16: [chunk][tap][Np][32]
      const int units = ntap * BN * 4;
      for (int u = tid; u < units; u += NT) {
        const int tl = u / (BN * 4), rem = u % (BN * 4), n = rem >> 2, g = rem & 3;
        const int gn = n0 + n;
        const unsigned off = gn < Np ? (unsigned)(((((size_t)c * p.KS + tap0 + tl) * Np + gn) * BK + 8 * g) * 2) : OOB;
        *reinterpret_cast<uint4*>(dst + (size_t)tl * W_TAP + n * WPITCH + 8 * g) = bload16(rw, off);
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

  // ---- input-window staging, software-pipelined over (tile, chunk) steps: the raw loads of
  // step s+1 are issued into registers right after step s's window is written to LDS, so HBM
  // latency hides under step s's MFMAs and epilogue.
  constexpr int MAXU = 6;  // prefetched 8-channel units per thread; the rest load synchronously
  typename RawT<T>::type pre[MAXU];
  const int units = R * 4;

  auto issue = [&](int t, int c) {
    const int mt = t % ntm, b = (t / ntm) % p.B;
    const T* xb = reinterpret_cast<const T*>(p.x) + (size_t)b * p.x_bs;
    const Rsrc rx = make_rsrc(xb, (unsigned)((size_t)p.Lin * p.x_ld * sizeof(T)));
    const int gr0 = mt * BM * p.stride - p.pad, ci0 = c * BK;
#pragma unroll
    for (int k = 0; k < MAXU; ++k) {
      const int u = tid + k * NT;
      const int r = u >> 2, g = u & 3;
      const int gr = gr0 + r, ch = ci0 + 8 * g;
      const unsigned e = (u < units) ? (unsigned)(gr * p.x_ld + ch) : OOB;  // gr < 0 wraps: OOB
      bload_raw(rx, e, pre[k], (const T*)nullptr);
    }
  };

  auto put = [&](int u, float (&v)[8], bool ok, int ci0) {
    const int r = u >> 2, g = u & 3;
    const int ch = ci0 + 8 * g;
    if (ok) {
      float cm[8], ca[8];
      if (mode & PRO_AFFINE) {
        ld8_lds(coef + ch, cm);
        ld8_lds(coef + cinp + ch, ca);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = fmaf(v[j], ca[j], cm[j]);  // x*a + (beta - mean*a)
      }
      if (mode & PRO_SNAKE) {
        ld8_lds(coef + 2 * cinp + ch, cm);
        ld8_lds(coef + 3 * cinp + ch, ca);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = snake_f<FAST_SIN>(v[j], cm[j], ca[j]);
      }
      if (mode & PRO_LRELU) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = v[j] > 0.f ? v[j] : v[j] * p.pro.slope;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (ch + j >= p.Cin) v[j] = 0.f;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = 0.f;
    }
    MT* dst = Xs + r * XP + 8 * g;
    if constexpr (C::BF) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16_t)v[j];
      *reinterpret_cast<bf16x8*>(dst) = o;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) dst[j] = v[j];
    }
  };

  auto write_x = [&](int t, int c) {
    const int ci0 = c * BK;
    const int gr0 = (t % ntm) * BM * p.stride - p.pad;
#pragma unroll
    for (int k = 0; k < MAXU; ++k) {
      const int u = tid + k * NT;
      const int gr = gr0 + (u >> 2);
      float v[8];
      raw_to_f32(pre[k], v);
      // conv zero padding applies to the post-prologue activation
      if (u < units) put(u, v, gr >= 0 && gr < p.Lin, ci0);
    }
    if (units > MAXU * NT) {  // large windows (2-D style convs): synchronous remainder
      const int mt = t % ntm, b = (t / ntm) % p.B;
      const T* xb = reinterpret_cast<const T*>(p.x) + (size_t)b * p.x_bs;
      const Rsrc rx = make_rsrc(xb, (unsigned)((size_t)p.Lin * p.x_ld * sizeof(T)));
      (void)mt;
      for (int u = tid + MAXU * NT; u < units; u += NT) {
        const int r = u >> 2, g = u & 3;
        const int gr = gr0 + r, ch = ci0 + 8 * g;
        typename RawT<T>::type raw;
        bload_raw(rx, (unsigned)(gr * p.x_ld + ch), raw, (const T*)nullptr);
        float v[8];
        raw_to_f32(raw, v);
        put(u, v, gr >= 0 && gr < p.Lin, ci0);
      }
    }
  };

  f32x16 acc[WM][WN];
  constexpr bool PREF = !NARROW && WM * WN <= 2;
  struct Raw16 {
    typename RawT<T>::type a, b;
  };
  Raw16 rres[PREF ? WM : 1][PREF ? WN : 1], racc[PREF ? WM : 1][PREF ? WN : 1];
  const int nsteps = (tend - tbeg) * p.nchunks;
  if (nsteps > 0) issue(tbeg, 0);
  for (int st = 0; st < nsteps; ++st) {
    const int t = tbeg + st / p.nchunks, c = st % p.nchunks;
    const int mt = t % ntm;
    const int b = (t / ntm) % p.B;
    const int nt = t / (ntm * p.B);
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
            coef[2 * cinp + ci] = al;
            coef[3 * cinp + ci] = 1.0f / al;  // the reference's (1 / alpha), once per channel
          }
        }
        if (resident && nt != cur_nt)
          for (int cc = 0; cc < p.nchunks; ++cc) stage_w(cc, 0, p.KS, Ws + (size_t)cc * p.KS * W_TAP, n0);
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
      if (c == p.nchunks - 1) {
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
    __syncthreads();  // previous readers of Xs (MFMA / epilogue scratch) are done; coef / W visible
    write_x(t, c);
    if (st + 1 < nsteps) issue(tbeg + (st + 1) / p.nchunks, (st + 1) % p.nchunks);
    // ---- taps (weights resident, or staged in groups that fit the budget) ----
    for (int tap0 = 0; tap0 < p.KS; tap0 += resident ? p.KS : p.tg) {
      const int ntap = resident ? p.KS : min(p.tg, p.KS - tap0);
      const MT* wbase;
      if (resident) {
        wbase = Ws + (size_t)c * p.KS * W_TAP;
      } else {
        if (tap0 > 0) __syncthreads();
        stage_w(c, tap0, ntap, Ws, n0);
        wbase = Ws;
      }
      __syncthreads();
#pragma unroll 1
      for (int tl = 0; tl < ntap; ++tl) {
        const int tap = tap0 + tl;
        const int toff = (tap / p.kw) * p.row_off + (tap % p.kw) * p.dil;
        const MT* wt = wbase + (size_t)tl * W_TAP;
        if constexpr (C::BF) {
#pragma unroll
          for (int kk = 0; kk < BK / 16; ++kk) {
            bf16x8 af[WM], bw[WN];
#pragma unroll
            for (int mi = 0; mi < WM; ++mi) {
              const int r = (wm * WM + mi) * 32 + l32;
              af[mi] = *reinterpret_cast<const bf16x8*>(Xs + (r * p.stride + toff) * XP + kk * 16 + hi * 8);
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
                acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi], bw[ni], acc[mi][ni], 0, 0, 0);
          }
        } else {
#pragma unroll 4
          for (int kk = 0; kk < BK / 2; ++kk) {
            float af[WM], bw[WN];
#pragma unroll
            for (int mi = 0; mi < WM; ++mi) {
              const int r = (wm * WM + mi) * 32 + l32;
              af[mi] = Xs[(r * p.stride + toff) * XP + 2 * kk + hi];
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
                acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[mi], bw[ni], acc[mi][ni], 0, 0, 0);
          }
        }
      }
    }
    if (c != p.nchunks - 1) continue;

    // ---------------- epilogue: per-wave transpose, lane = (frame, 16 channels) ----------------
    __syncthreads();  // every wave is done reading Xs / Ws
    float* ws = scr + (size_t)wid * 32 * EP;
    T* yT = reinterpret_cast<T*>(p.y) + (size_t)b * p.y_bs;
    float* yF = reinterpret_cast<float*>(p.y) + (size_t)b * p.y_bs;
    const T* resb = p.res ? reinterpret_cast<const T*>(p.res) + (size_t)b * p.res_bs : nullptr;
    const T* accb = p.accb ? reinterpret_cast<const T*>(p.accb) + (size_t)b * p.acc_bs : nullptr;
#pragma unroll
    for (int mi = 0; mi < WM; ++mi) {
#pragma unroll
      for (int ni = 0; ni < WN; ++ni) {
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) ws[((reg & 3) + 8 * (reg >> 2) + 4 * hi) * EP + l32] = acc[mi][ni][reg];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        float v[16];
#pragma unroll
        for (int j = 0; j < 16; j += 4) {
          const float4 f = *reinterpret_cast<const float4*>(ws + l32 * EP + hi * 16 + j);
          v[j] = f.x; v[j + 1] = f.y; v[j + 2] = f.z; v[j + 3] = f.w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const int q = q0 + (wm * WM + mi) * 32 + l32;
        const int nb = n0 + (wn * WN + ni) * 32 + hi * 16;  // first of this lane's 16 columns
        // v becomes the stored values (0 where nothing is stored) for the statistics pass
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
                store16(yT + (size_t)orow * p.y_ld + co0, v);
              } else {
                if (p.bias) {
#pragma unroll
                  for (int j = 0; j < 16; j += 4) {
                    const float4 bb = *reinterpret_cast<const float4*>(p.bias + co0 + j);
                    v[j] += bb.x; v[j + 1] += bb.y; v[j + 2] += bb.z; v[j + 3] += bb.w;
                  }
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
                      atomicAdd(p.stats + ((size_t)b * p.stats_ld + co0 + j) * 2 + 0, x);
                      atomicAdd(p.stats + ((size_t)b * p.stats_ld + co0 + j) * 2 + 1, x * x);
                    }
                  }
                }
                if (resb) {
                  float r[16];
                  if constexpr (PREF) raw16_to_f32(rres[PREF ? mi : 0][PREF ? ni : 0], r);
                  else load16(resb + (size_t)(orow >> p.res_shift) * p.res_ld + co0, r);
#pragma unroll
                  for (int j = 0; j < 16; ++j) v[j] = (v[j] + r[j]) * p.out_scale;
                }
                if (accb) {
                  float r[16];
                  if constexpr (PREF) raw16_to_f32(racc[PREF ? mi : 0][PREF ? ni : 0], r);
                  else load16(accb + (size_t)orow * p.acc_ld + co0, r);
                  if (p.acc_div != 0.f) {
                    // the reference divides (xs / num_kernels); bf16 mode multiplies by the reciprocal
                    const float inv_div = 1.0f / p.acc_div;
#pragma unroll
                    for (int j = 0; j < 16; ++j) v[j] = C::BF ? (r[j] + v[j]) * inv_div : (r[j] + v[j]) / p.acc_div;
                  } else {
#pragma unroll
                    for (int j = 0; j < 16; ++j) v[j] = r[j] + v[j];
                  }
                }
                store16(yT + (size_t)orow * p.y_ld + co0, v);
#pragma unroll
                for (int j = 0; j < 16; ++j) v[j] = to_f32(from_f32<T>(v[j]));
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
                  x = v[j] + (p.bias ? p.bias[co] : 0.f);
                  if (resb) x = (x + to_f32(resb[(size_t)(orow >> p.res_shift) * p.res_ld + co])) * p.out_scale;
                  if (p.epi_tanh) x = tanhf(x);
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
        if (!stored) {
#pragma unroll
          for (int j = 0; j < 16; ++j) v[j] = 0.f;
        }
        if (p.stats) {  // column pass over the wave scratch: lane = column l32, rows of half hi
#pragma unroll
          for (int j = 0; j < 16; j += 4)
            *reinterpret_cast<float4*>(ws + l32 * EP + hi * 16 + j) = make_float4(v[j], v[j + 1], v[j + 2], v[j + 3]);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          float a = 0.f, q2 = 0.f;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float x = ws[(hi * 16 + r) * EP + l32];
            a += x;
            q2 += x * x;
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          st_s[ni] += a;
          st_q[ni] += q2;
        }
      }
    }
  }
  if (cur_nt >= 0 && p.stats) flush_stats(cur_nt, cur_b);
}

int g_num_cu = 0;

template <typename T, typename MT, int WAVES_M, int WAVES_N, int WM, int WN, bool NARROW = false>
int launch_cfg(ConvParams p, hipStream_t stream) {
  using C = ConvCfg<T, MT, WAVES_M, WAVES_N, WM, WN>;
  constexpr int LDS_MAX = 160 * 1024;
  constexpr int WBUDGET = 48 * 1024;
  constexpr int WRES_BUDGET = 120 * 1024;
  const size_t wtap = (size_t)C::W_TAP * sizeof(MT);
  // weights resident across tiles when every chunk x tap slice of the column tile fits
  const int nres = p.nchunks * p.KS;
  if ((size_t)nres * wtap <= (size_t)WRES_BUDGET && C::lds_bytes(p, nres) <= (size_t)LDS_MAX) {
    p.w_resident = 1;
    p.tg = p.KS;
  } else {
    p.w_resident = 0;
    int tg = (int)(WBUDGET / wtap);
    if (tg < 1) tg = 1;
    if (tg > p.KS) tg = p.KS;
    while (tg > 1 && C::lds_bytes(p, tg) > (size_t)LDS_MAX) --tg;
    p.tg = tg;
  }
  const size_t lds = C::lds_bytes(p, p.w_resident ? nres : p.tg);
  if (lds > (size_t)LDS_MAX) return ST_EINVAL;
  auto kern = conv1d_igemm_kernel<T, MT, WAVES_M, WAVES_N, WM, WN, NARROW>;
  static bool attr_set = false;
  if (!attr_set) {
    ST_CHECK_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX));
    attr_set = true;
  }
  if (!g_num_cu) {
    int dev = 0;
    ST_CHECK_HIP(hipGetDevice(&dev));
    ST_CHECK_HIP(hipDeviceGetAttribute(&g_num_cu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  int per_cu = 0;
  ST_CHECK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, C::NT, lds));
  if (per_cu < 1) per_cu = 1;
  const long long ntn = (p.N + C::BN - 1) / C::BN, ntm = (p.Lq + C::BM - 1) / C::BM;
  const long long tiles = ntn * ntm * p.B;
  if (tiles <= 0) return ST_OK;
  if (tiles > 0x7fffffffLL) return ST_EINVAL;
  long long grid = (long long)g_num_cu * per_cu;
  if (grid > tiles) grid = tiles;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(C::NT), lds, stream, p);
  return (int)hipGetLastError();
}

template <typename T, typename MT>
int launch_typed(const ConvParams& p, hipStream_t stream) {
  const bool narrow = (p.Cout % 16 != 0) || p.y_f32 || (p.y_ld % 8 != 0) || (p.res && p.res_ld % 8 != 0) ||
                      (p.accb && p.acc_ld % 8 != 0);
  if (narrow) {
    // per-element epilogue: residual/scale/tanh supported; accumulate/reflect/zero-columns are not
    if (p.accb || p.reflect_front || p.zc_period || p.N > 32 || p.stride > 1) return ST_EINVAL;
    return launch_cfg<T, MT, 4, 1, 2, 1, true>(p, stream);
  }
  if (p.epi_tanh) return ST_EINVAL;  // tanh only on narrow heads
  if (p.stride > 1) return launch_cfg<T, MT, 2, 2, 1, 2>(p, stream);  // BM 64 x BN 128 (short window)
  if (p.N <= 32) return launch_cfg<T, MT, 4, 1, 2, 1>(p, stream);     // BM 256 x BN 32, 4 waves
  if (p.N <= 64) return launch_cfg<T, MT, 8, 1, 1, 2>(p, stream);     // BM 256 x BN 64, 8 waves
  return launch_cfg<T, MT, 4, 2, 2, 2>(p, stream);                    // BM 256 x BN 128, 8 waves
}

}  // namespace

int st_conv1d(const ConvParams& p, int dtype, hipStream_t stream) {
  if (p.B <= 0 || p.Lq <= 0 || p.N <= 0) return ST_OK;
  if (p.KS <= 0 || p.stride <= 0 || p.dil <= 0 || p.Cout <= 0 || p.up <= 0) return ST_EINVAL;
  if (p.x_ld % 8 != 0 || p.nchunks * BK < p.Cin) return ST_EINVAL;
  ConvParams q = p;
  if (q.kw <= 0) q.kw = q.KS;
  if (dtype == ST_FP32) return launch_typed<float, float>(q, stream);
  if (dtype == ST_BF16) return launch_typed<bf16_t, bf16_t>(q, stream);
  return ST_EDTYPE;
}
