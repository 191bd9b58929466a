// Duration / text path of StyleTTS2-lite on gfx950, fp32.
//
// Reference computations replaced (thewh1teagle/StyleTTS2-lite @ 2025-06-14):
//   * nn.LSTM(bidirectional, batch_first) + pack_padded_sequence / pad_packed_sequence:
//       TextEncoder.lstm            models.py:267-279
//       DurationEncoder.lstms[2i]   models.py:510-518
//       ProsodyPredictor.lstm       models.py:420-430, inference.py:246
//       ProsodyPredictor.shared     models.py:449
//   * TextEncoder CNN  (weight-norm Conv1d k5 -> LayerNorm(gamma, beta) -> LeakyReLU 0.2 -> mask)
//                                   models.py:243-262
//   * AdaLayerNorm + style concat + mask (DurationEncoder)  models.py:372-392, 503-507
//   * embedding + mask (TextEncoder) models.py:257-260; duration_proj (LinearNorm) models.py:430;
//     the alignment products en = d^T @ aln / asr = t_en @ aln   models.py:432, inference.py:266-269
//
// All activations are "frames" [B][T][C] (channel fastest), the layout the reference's
// batch_first LSTMs use.  Everything here is latency-bound at text lengths (T <= a few
// hundred tokens): the kernels aim at few launches and no host round trips, not at MFMA.
#include "common.h"
#include "stts2.h"

// ---------------------------------------------------------------------------------------
// Strided batched "frames GEMM": a 1-D convolution over the T axis as an implicit GEMM
//   y[b][t][n] = bias[n] + bias2[n] + sum_{k<K} sum_{c<Cin} w(b, n, c, k) * x(b, t + k - pad, c)
// with every operand addressed by explicit strides, so one kernel serves Conv1d (K taps),
// Linear / LSTM input projections (K = 1) and batched matrix products (w strided per batch).
// 64 x 64 output tile per 256-thread workgroup, 4 x 4 per lane, K staged through LDS in 16s.
// ---------------------------------------------------------------------------------------
struct GemmArgs {
  const float* x;
  long long xs_b, xs_t, xs_c;
  int Tin, Cin;
  const float* w;
  long long ws_b, ws_n, ws_c, ws_k;
  int N, K, pad;
  const float* bias;
  const float* bias2;
  float* y;
  long long ys_b, ys_t, ys_n;
  int Tout;
  // split-K (few output tiles): blockIdx.z = b * splits + split; split k covers K rows
  // [k * kper, (k + 1) * kper) and writes its partial sums to part[k][b][t][n] (no bias); a fixed-order
  // reduction (k_splitk_reduce) then adds bias and stores y.  splits = 1: direct.
  int splits, kper;
  float* part;
};

__global__ void __launch_bounds__(256) k_frames_gemm(GemmArgs a) {
  __shared__ float As[16][68];  // [k][t]
  __shared__ float Bs[16][68];  // [k][n]
  const int sp = a.splits > 1 ? (int)blockIdx.z % a.splits : 0;
  const int b = a.splits > 1 ? (int)blockIdx.z / a.splits : (int)blockIdx.z;
  const int t0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int Kall = a.Cin * a.K;
  const int kbeg = a.splits > 1 ? sp * a.kper : 0;
  const int Ktot = a.splits > 1 ? (kbeg + a.kper < Kall ? kbeg + a.kper : Kall) : Kall;
  const float* xb = a.x + (size_t)b * a.xs_b;
  const float* wb = a.w + (size_t)b * a.ws_b;
  float acc[4][4] = {};
  for (int kk = kbeg; kk < Ktot; kk += 16) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int idx = tid + e * 256, kl = idx & 15, rl = idx >> 4;
      const int kg = kk + kl;
      float va = 0.f, vb = 0.f;
      if (kg < Ktot) {
        const int tap = kg / a.Cin, c = kg - tap * a.Cin;
        const int t = t0 + rl, ti = t + tap - a.pad;
        if (t < a.Tout && ti >= 0 && ti < a.Tin) va = xb[(size_t)ti * a.xs_t + (size_t)c * a.xs_c];
        const int n = n0 + rl;
        if (n < a.N) vb = wb[(size_t)n * a.ws_n + (size_t)c * a.ws_c + (size_t)tap * a.ws_k];
      }
      As[kl][rl] = va;
      Bs[kl][rl] = vb;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const float4 av = *reinterpret_cast<const float4*>(&As[k][ty * 4]);
      const float4 bv = *reinterpret_cast<const float4*>(&Bs[k][tx * 4]);
      const float ar[4] = {av.x, av.y, av.z, av.w}, br[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(ar[i], br[j], acc[i][j]);
    }
    __syncthreads();
  }
  if (a.splits > 1) {
    float* pp = a.part + (((size_t)sp * gridDim.z / a.splits + b) * a.Tout) * a.N;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tx * 4 + j;
      if (n >= a.N) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t = t0 + ty * 4 + i;
        if (t < a.Tout) pp[(size_t)t * a.N + n] = acc[i][j];
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + tx * 4 + j;
    if (n >= a.N) continue;
    const float bs = (a.bias ? a.bias[n] : 0.f) + (a.bias2 ? a.bias2[n] : 0.f);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = t0 + ty * 4 + i;
      if (t < a.Tout) a.y[(size_t)b * a.ys_b + (size_t)t * a.ys_t + (size_t)n * a.ys_n] = acc[i][j] + bs;
    }
  }
}

__global__ void __launch_bounds__(256) k_splitk_reduce(GemmArgs a, int B) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t per = (size_t)a.Tout * a.N;
  if (i >= (size_t)B * per) return;
  const int b = (int)(i / per), t = (int)((i % per) / a.N), n = (int)(i % a.N);
  float v = 0.f;
  for (int k = 0; k < a.splits; ++k) v += a.part[(size_t)k * B * per + i];  // fixed order
  v += (a.bias ? a.bias[n] : 0.f) + (a.bias2 ? a.bias2[n] : 0.f);
  a.y[(size_t)b * a.ys_b + (size_t)t * a.ys_t + (size_t)n * a.ys_n] = v;
}

// split count for a launch: enough workgroups for the chip when the output has few 64 x 64 tiles
// (the text path: 16 - 130 token rows), K chunks of >= 128, at most 16 splits
static int gemm_splits(int B, int Tout, int N, int Ktot) {
  const long long tiles = (long long)((Tout + 63) / 64) * ((N + 63) / 64) * B;
  int sp = 1;
  while (sp < 16 && tiles * sp * 2 <= 256 && Ktot / (sp * 2) >= 128) sp *= 2;
  return sp;
}

static int launch_gemm(const GemmArgs& a0, int B, hipStream_t s, float* part = nullptr, long long part_elems = 0) {
  if (B <= 0 || a0.Tout <= 0 || a0.N <= 0) return 0;
  if (a0.Cin <= 0 || a0.K <= 0 || !a0.x || !a0.w || !a0.y) return ST_EINVAL;
  GemmArgs a = a0;
  const int Kall = a.Cin * a.K;
  a.splits = part ? gemm_splits(B, a.Tout, a.N, Kall) : 1;
  while (a.splits > 1 && (long long)a.splits * B * a.Tout * a.N > part_elems) a.splits >>= 1;
  a.kper = ((Kall + a.splits - 1) / a.splits + 15) & ~15;
  a.part = part;
  dim3 grid((a.Tout + 63) / 64, (a.N + 63) / 64, B * a.splits);
  hipLaunchKernelGGL(k_frames_gemm, grid, dim3(256), 0, s, a);
  ST_CHECK_HIP(hipGetLastError());
  if (a.splits > 1) {
    const size_t n = (size_t)B * a.Tout * a.N;
    hipLaunchKernelGGL(k_splitk_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a, B);
    ST_CHECK_HIP(hipGetLastError());
  }
  return 0;
}

// ---------------------------------------------------------------------------------------
// BiLSTM recurrence (torch gate order i, f, g, o; c' = f c + i g; h' = o tanh(c')).
// G = x W_ih^T + b_ih + b_hh for every (direction, utterance, step) comes precomputed from
// k_frames_gemm.  One workgroup per (utterance, direction) with 4H lanes: lane j owns gate
// row j and streams column j of W_hh^T (coalesced over j, L2-resident across steps) against
// h_{t-1} broadcast from LDS.  pack_padded_sequence semantics: the forward direction runs
// t = 0 .. len-1, the reverse t = len-1 .. 0, both from zero state; rows t >= len are 0.
// ---------------------------------------------------------------------------------------
static int g_lstm_bg = 0;  // 0 = automatic, -1 = cooperative, 1/2/4 = per-workgroup (stts_set_lstm_group)

__device__ __forceinline__ float sigm(float v) { return 1.0f / (1.0f + expf(-v)); }

// BG utterances of one direction per workgroup: every W_hh element loaded from L2 feeds BG FMAs.
// Each step is a chain the workgroup cannot overlap with the next, so its cost is the latency of
// streaming the lane's 4H x H / 4H = H recurrent weights: W_hh is stored k-quad interleaved
// (WT4[q][j] = W_hh[j][4q .. 4q+3], one float4 per lane, 1 KB coalesced per wave) and streamed in
// chunks of 4 float4 with the next chunk in flight while the current one is consumed (measured:
// one dword per lane per load and a 4-deep loop spent ~8 us a step on L2 round trips).
// h_{t-1} sits in LDS as [q][BG][4] so one ds_read_b128 broadcasts 4 k of one utterance.
// cs (training, may be null): the cell state of every step, [2][B][T][H]
template <int BG>
__global__ void __launch_bounds__(1024) k_bilstm_rec(const float* __restrict__ G, const float4* __restrict__ WT4,
                                                     const int* __restrict__ lengths, int B, int T, int H,
                                                     float* __restrict__ y, float* __restrict__ hn,
                                                     float* __restrict__ cn, float* __restrict__ cs) {
  __shared__ float4 hs4[64 * BG];
  __shared__ float gs[BG][1024];
  float* hs = reinterpret_cast<float*>(hs4);
  const int b0 = blockIdx.x * BG, d = blockIdx.y, j = threadIdx.x, H4 = 4 * H;
  const int nch = H >> 4;  // chunks of 4 k-quads
  int len[BG], maxlen = 0;
#pragma unroll
  for (int i = 0; i < BG; ++i) {
    int l = 0;
    if (b0 + i < B) {
      l = lengths ? lengths[b0 + i] : T;
      l = l < 0 ? 0 : (l > T ? T : l);
    }
    len[i] = l;
    maxlen = l > maxlen ? l : maxlen;
  }
  if (j < H) {
#pragma unroll
    for (int i = 0; i < BG; ++i) {
      hs[((j >> 2) * BG + i) * 4 + (j & 3)] = 0.f;
      if (b0 + i >= B) continue;
      float* yb = y + (size_t)(b0 + i) * T * 2 * H + (size_t)d * H;
      for (int t = len[i]; t < T; ++t) yb[(size_t)t * 2 * H + j] = 0.f;
    }
  }
  float c[BG], h[BG];
#pragma unroll
  for (int i = 0; i < BG; ++i) c[i] = h[i] = 0.f;
  __syncthreads();
  const float4* W = WT4 + (size_t)d * (H >> 2) * H4 + j;
  for (int s = 0; s < maxlen; ++s) {
    float acc[BG][4];
#pragma unroll
    for (int i = 0; i < BG; ++i) {
      const int t = d == 0 ? s : len[i] - 1 - s;
      acc[i][0] = s < len[i] ? G[(((size_t)d * B + b0 + i) * T + t) * H4 + j] : 0.f;
      acc[i][1] = acc[i][2] = acc[i][3] = 0.f;
    }
    auto consume = [&](const float4 (&w)[4], int ch) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int q = ch * 4 + u;
#pragma unroll
        for (int i = 0; i < BG; ++i) {
          const float4 hv = hs4[q * BG + i];
          acc[i][0] = fmaf(w[u].x, hv.x, acc[i][0]);
          acc[i][1] = fmaf(w[u].y, hv.y, acc[i][1]);
          acc[i][2] = fmaf(w[u].z, hv.z, acc[i][2]);
          acc[i][3] = fmaf(w[u].w, hv.w, acc[i][3]);
        }
      }
    };
    float4 wa[4], wb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) wa[u] = W[(size_t)u * H4];
#pragma unroll 1
    for (int ch = 0; ch < nch; ch += 2) {
      if (ch + 1 < nch) {
#pragma unroll
        for (int u = 0; u < 4; ++u) wb[u] = W[(size_t)((ch + 1) * 4 + u) * H4];
      }
      consume(wa, ch);
      if (ch + 1 < nch) {
        if (ch + 2 < nch) {
#pragma unroll
          for (int u = 0; u < 4; ++u) wa[u] = W[(size_t)((ch + 2) * 4 + u) * H4];
        }
        consume(wb, ch + 1);
      }
    }
#pragma unroll
    for (int i = 0; i < BG; ++i) gs[i][j] = (acc[i][0] + acc[i][1]) + (acc[i][2] + acc[i][3]);
    __syncthreads();
    if (j < H) {
#pragma unroll
      for (int i = 0; i < BG; ++i) {
        if (s >= len[i]) continue;
        const int t = d == 0 ? s : len[i] - 1 - s;
        const float ig = sigm(gs[i][j]), fg = sigm(gs[i][H + j]), gg = tanhf(gs[i][2 * H + j]);
        const float og = sigm(gs[i][3 * H + j]);
        c[i] = fg * c[i] + ig * gg;
        h[i] = og * tanhf(c[i]);
        hs[((j >> 2) * BG + i) * 4 + (j & 3)] = h[i];
        y[((size_t)(b0 + i) * T + t) * 2 * H + (size_t)d * H + j] = h[i];
        if (cs) cs[(((size_t)d * B + b0 + i) * T + t) * H + j] = c[i];
      }
    }
    __syncthreads();
  }
  if (j < H) {
#pragma unroll
    for (int i = 0; i < BG; ++i) {
      if (b0 + i >= B) continue;
      if (hn) hn[((size_t)d * B + b0 + i) * H + j] = h[i];
      if (cn) cn[((size_t)d * B + b0 + i) * H + j] = c[i];
    }
  }
}

// ---------------------------------------------------------------------------------------
// Cooperative recurrence for H = 256 (the reference's every LSTM): the per-step floor of
// k_bilstm_rec is one CU streaming the whole 1 MB W_hh through its 64 B/clk L1 (~7 us a step).
// Here a direction's W_hh is split over COOP_NW = 8 workgroups, each holding the 4 gate rows of
// 32 hidden units resident in LDS (128 rows x 256, padded rows: 133 KB), so a step reads no weights
// from L2 at all.  Per step each workgroup computes its 128 gate rows (512 lanes: row = lane / 4,
// a quarter of k per lane, shuffle-reduced), updates its 32 (c, h), publishes h to an exchange
// buffer as (step tag, h) 64-bit words (double-buffered by step parity) and polls the 256 words of
// the step (agent-scope acquire loads): the data is its own arrival flag, one round trip a step.  Groups = (direction, utterance slot) run persistently over the utterances; the launch
// is a plain launch of at most 2B x 8 workgroups, admitted only when the occupancy query puts all of
// them on the chip at once (else k_bilstm_rec), and every spin is bounded: a timed-out wait sets
// *err (the host reads it: stts_bilstm_error_offset) and from then on the workgroup publishes NaN
// as its h, so y, h_n and c_n are all poisoned, never a hang.
// ---------------------------------------------------------------------------------------
#define COOP_H 256
#define COOP_NW 8
#define COOP_U (COOP_H / COOP_NW)  // hidden units per workgroup (32)
#define COOP_ROWS (4 * COOP_U)     // gate rows per workgroup (128)
#define COOP_LD 260                // padded LDS row stride (floats)
#define COOP_SPIN_LIMIT (1u << 22)
static unsigned g_coop_spin_limit = COOP_SPIN_LIMIT;  // stts_set_bilstm_debug (tests)
static int g_coop_drop = 0;                          // debug: member 0 of every group never publishes

struct CoopArgs {
  const float* G;     // [2][B][T][4H] input projections (+ both biases)
  const float* whh0;  // W_hh forward  [4H][H] (torch layout)
  const float* whh1;  // W_hh reverse
  const int* lengths;
  int B, T, groups;   // groups: even, group g -> direction g & 1, utterances g>>1, g>>1 + groups/2, ...
  float* y;           // [B][T][2H]
  float* hn;
  float* cn;
  unsigned long long* xe;  // exchange [groups][2][H] of (step tag << 32 | h bits), zeroed before launch
  int* err;
  unsigned spin_limit;
  int drop;  // debug: workgroup member 0 never publishes (every wait of its group times out)
};

__global__ void __launch_bounds__(512) k_bilstm_coop(CoopArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* Ws = lds;                           // [COOP_ROWS][COOP_LD]
  float* hb = lds + COOP_ROWS * COOP_LD;     // [H]
  float* gl = hb + COOP_H;                   // [COOP_ROWS]
  const int H = COOP_H, H4 = 4 * COOP_H;
  const int grp = blockIdx.x / COOP_NW, w = blockIdx.x % COOP_NW, tid = threadIdx.x;
  const int d = grp & 1, slot = grp >> 1, nslots = a.groups >> 1;
  const int r = tid >> 2, part = tid & 3;
  const int gate = r / COOP_U, unit = r % COOP_U;
  const int grow = gate * H + w * COOP_U + unit;  // global gate row of lane row r
  {  // resident W_hh slice: local row rr = (gate, unit) <- W_hh[gate * H + w * 32 + unit][:]
    const float* W = d ? a.whh1 : a.whh0;
    for (int i = tid; i < COOP_ROWS * (COOP_H / 4); i += 512) {
      const int rr = i / (COOP_H / 4), q = i % (COOP_H / 4);
      const int gr = (rr / COOP_U) * H + w * COOP_U + (rr % COOP_U);
      *reinterpret_cast<float4*>(&Ws[rr * COOP_LD + 4 * q]) = *reinterpret_cast<const float4*>(&W[(size_t)gr * H + 4 * q]);
    }
  }
  __shared__ int poisoned;  // a timed-out wait: stop waiting, poison the outputs
  if (tid == 0) poisoned = 0;
  unsigned gstep = 1;  // step tag, unique over the group's whole job sequence (words start zeroed)
  unsigned long long* xe = a.xe + (size_t)grp * 2 * H;
  for (int b = slot; b < a.B; b += nslots) {
    int len = a.lengths ? a.lengths[b] : a.T;
    len = len < 0 ? 0 : (len > a.T ? a.T : len);
    float* yb = a.y + (size_t)b * a.T * 2 * H + (size_t)d * H + w * COOP_U;
    if (tid < COOP_U)
      for (int t = len; t < a.T; ++t) yb[(size_t)t * 2 * H + tid] = 0.f;
    if (tid < H) hb[tid] = 0.f;
    float c = 0.f, h = 0.f;
    __syncthreads();
    const float* Gb = a.G + ((size_t)d * a.B + b) * a.T * H4;
    // the input projection of step s + 1 is loaded while step s computes (its HBM / L2 latency was
    // exposed once a step)
    float gnext = (part == 0 && len > 0) ? Gb[(size_t)(d == 0 ? 0 : len - 1) * H4 + grow] : 0.f;
    for (int s = 0; s < len; ++s) {
      const int t = d == 0 ? s : len - 1 - s;
      const float gcur = gnext;
      if (part == 0 && s + 1 < len) gnext = Gb[(size_t)(d == 0 ? s + 1 : len - 2 - s) * H4 + grow];
      float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
      const float* wr = Ws + r * COOP_LD + part * (COOP_H / 4);
      const float* hr = hb + part * (COOP_H / 4);
#pragma unroll
      for (int m = 0; m < COOP_H / 16; ++m) {
        const float4 wv = *reinterpret_cast<const float4*>(wr + 4 * m);
        const float4 hv = *reinterpret_cast<const float4*>(hr + 4 * m);
        acc0 = fmaf(wv.x, hv.x, acc0);
        acc1 = fmaf(wv.y, hv.y, acc1);
        acc2 = fmaf(wv.z, hv.z, acc2);
        acc3 = fmaf(wv.w, hv.w, acc3);
      }
      float v = (acc0 + acc1) + (acc2 + acc3);
      v += __shfl_xor(v, 1);
      v += __shfl_xor(v, 2);
      if (part == 0) gl[r] = v + gcur;
      __syncthreads();
      // publish (h, step tag) as one 64-bit word; every lane k < H then polls word k of this step
      unsigned long long* xo = xe + (size_t)(gstep & 1) * H;
      if (tid < COOP_U) {
        const float ig = sigm(gl[tid]), fg = sigm(gl[COOP_U + tid]), gg = tanhf(gl[2 * COOP_U + tid]);
        const float og = sigm(gl[3 * COOP_U + tid]);
        c = fg * c + ig * gg;
        h = og * tanhf(c);
        if (poisoned) c = h = __builtin_nanf("");  // a peer's h never arrived: everything after is NaN
        const unsigned long long word = ((unsigned long long)gstep << 32) | (unsigned long long)__float_as_uint(h);
        if (!(a.drop && w == 0)) __hip_atomic_store(&xo[w * COOP_U + tid], word, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        yb[(size_t)t * 2 * H + tid] = h;
      }
      if (tid < H) {  // hb is free: every lane finished this step's dot products (barrier above)
        unsigned long long v = 0;
        unsigned spins = 0;
        while (true) {
          v = __hip_atomic_load(&xo[tid], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
          if ((unsigned)(v >> 32) == gstep) break;
          if (poisoned || ++spins > a.spin_limit) {
            if (!poisoned) atomicOr(a.err, 1);
            poisoned = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        hb[tid] = poisoned ? __builtin_nanf("") : __uint_as_float((unsigned)v);
      }
      ++gstep;
      __syncthreads();
    }
    if (tid < COOP_U) {
      if (a.hn) a.hn[((size_t)d * a.B + b) * H + w * COOP_U + tid] = h;
      if (a.cn) a.cn[((size_t)d * a.B + b) * H + w * COOP_U + tid] = c;
    }
    __syncthreads();
  }
}

static int g_coop_groups_cap = -1;  // co-resident groups this device allows (-1 = not probed)
#define COOP_LDS_BYTES ((COOP_ROWS * COOP_LD + COOP_H + COOP_ROWS) * (int)sizeof(float))

// W_hh [4H][H] (torch) -> WT4 [H/4][4H][4] (k-quad interleaved), both directions.
__global__ void k_lstm_wt(const float* __restrict__ w0, const float* __restrict__ w1, int H, float* __restrict__ wt) {
  const int H4 = 4 * H;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)2 * H * H4) return;
  const int d = (int)(i / ((size_t)H * H4));
  const int r = (int)(i % ((size_t)H * H4));
  const int q = r / (H4 * 4), jj = (r >> 2) % H4, k = 4 * q + (r & 3);
  const float* w = d ? w1 : w0;
  wt[i] = w[(size_t)jj * H + k];
}

// ---------------------------------------------------------------------------------------
// Row norm over channels of frames rows, fused with what follows it in the reference:
//   mode 0 (LayerNorm, models.py:229-240):  v = xhat * gamma[c] + beta[c]
//   mode 1 (AdaLayerNorm, models.py:383-392): v = (1 + gb[b][c]) * xhat + gb[b][C + c]
//   mode 2 (no norm, the input concat of models.py:499-501): v = x
// then optional LeakyReLU(slope), then the row is zeroed for t >= len (masked_fill_), and
// `extra` [B][E] (the style vector) is appended as channels C .. C+E (the concat of
// models.py:505).  xhat = (x - mean) / sqrt(biased var + eps).  One wave64 per row.
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_row_norm(const float* __restrict__ x, long long xs_b, long long xs_t,
                                                  long long xs_c, int B,
                                                  int T, int C, int mode, const float* __restrict__ gamma,
                                                  const float* __restrict__ beta, long long gb_sb, float eps,
                                                  int lrelu, float slope, const int* __restrict__ lengths,
                                                  const float* __restrict__ extra, int E, float* __restrict__ y,
                                                  long long ys_b, long long ys_t) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (long long)B * T) return;
  const int b = (int)(row / T), t = (int)(row % T);
  const bool valid = !lengths || t < lengths[b];
  float* yr = y + (size_t)b * ys_b + (size_t)t * ys_t;
  if (!valid) {
    for (int c = lane; c < C + E; c += 64) yr[c] = 0.f;
    return;
  }
  const float* xr = x + (size_t)b * xs_b + (size_t)t * xs_t;
  if (mode == 2) {
    for (int c = lane; c < C; c += 64) yr[c] = xr[(size_t)c * xs_c];
    for (int e = lane; e < E; e += 64) yr[C + e] = extra[(size_t)b * E + e];
    return;
  }
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += xr[(size_t)c * xs_c];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const float mean = s / (float)C;
  float v2 = 0.f;
  for (int c = lane; c < C; c += 64) {
    const float dlt = xr[(size_t)c * xs_c] - mean;
    v2 += dlt * dlt;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v2 += __shfl_xor(v2, o);
  const float rstd = 1.0f / sqrtf(v2 / (float)C + eps);
  for (int c = lane; c < C; c += 64) {
    const float xh = (xr[(size_t)c * xs_c] - mean) * rstd;
    float v;
    if (mode == 0) {
      v = xh * gamma[c] + beta[c];
    } else {
      const float* gb = gamma + (size_t)b * gb_sb;
      v = (1.0f + gb[c]) * xh + gb[C + c];
    }
    if (lrelu) v = v > 0.f ? v : v * slope;
    yr[c] = v;
  }
  for (int e = lane; e < E; e += 64) yr[C + e] = extra[(size_t)b * E + e];
}

// Embedding gather + mask: y[b][t][:] = table[tokens[b][t]][:] for t < len, else 0.
__global__ void __launch_bounds__(256) k_embedding(const long long* __restrict__ tok, int B, int T,
                                                   const float* __restrict__ table, int n_symbols, int C,
                                                   const int* __restrict__ lengths, float* __restrict__ y,
                                                   int* __restrict__ err) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= (long long)B * T) return;
  const int b = (int)(row / T), t = (int)(row % T);
  const long long id = tok[row];
  const bool valid = (!lengths || t < lengths[b]);
  const bool in_range = id >= 0 && id < n_symbols;
  if (!in_range && lane == 0 && err) atomicOr(err, 1);
  float* yr = y + (size_t)row * C;
  for (int c = lane; c < C; c += 64) yr[c] = (valid && in_range) ? table[(size_t)id * C + c] : 0.f;
}

// ---------------------------------------------------------------------------------------
// Durations -> frame map (reference inference.py:247-263, StyleTTS2.__inference), one workgroup
// per utterance over its first len tokens:
//   dur   = sum_k sigmoid(logits[t][k])                                   (:247)
//   stats = (prev_mean != 0 ? prev_mean : mean(dur)) + std(dur) * z[t]    (:249-252, std unbiased)
//   dur   = dur * (1 - mix) + stats * mix                                 (:253)
//   dur[1:-2] = z-score outlier clamp (threshold 3, factor 0.95)          (:254, :134-148)
//   dur  /= speed; pred = max(round_half_even(dur), 1)                    (:256-258)
// and the frame -> token map of the alignment matrix (:259-263): frame_tok[b][f] = t for the
// pred[t] frames of token t, -1 past the utterance's total.  Sums are fixed-order tree reductions.
// ---------------------------------------------------------------------------------------
#define DUR_MAX_T 1024

__device__ float block_sum_1024(float v, float* red) {
  const int tid = threadIdx.x;
  red[tid] = v;
  __syncthreads();
  for (int s = 512; s > 0; s >>= 1) {
    if (tid < s) red[tid] += red[tid + s];
    __syncthreads();
  }
  const float r = red[0];
  __syncthreads();
  return r;
}

__global__ void __launch_bounds__(1024) k_durations(const float* __restrict__ logits, long long ls_b, long long ls_t,
                                                    int T, int K, const int* __restrict__ lengths,
                                                    const float* __restrict__ z, float mix, float prev_mean,
                                                    float speed, float* __restrict__ dur_out,
                                                    int* __restrict__ pred, int* __restrict__ total,
                                                    float* __restrict__ dur_mean) {
  __shared__ float red[1024];
  __shared__ int cum[DUR_MAX_T];
  const int b = blockIdx.x, t = threadIdx.x;
  int len = lengths ? lengths[b] : T;
  len = len < 0 ? 0 : (len > T ? T : len);
  const bool on = t < len;
  float d = 0.f;
  if (on) {
    const float* lr = logits + (size_t)b * ls_b + (size_t)t * ls_t;
    for (int k = 0; k < K; ++k) d += 1.0f / (1.0f + expf(-lr[k]));
  }
  // mean / unbiased std over the utterance's tokens (duration.mean(), duration.std())
  const float n = (float)len;
  float mean = block_sum_1024(on ? d : 0.f, red) / n;
  float dv = on ? (d - mean) : 0.f;
  float sd = sqrtf(block_sum_1024(dv * dv, red) / (n - 1.0f));
  {
    const float mu = prev_mean != 0.f ? prev_mean : mean;
    const float st = mu + sd * (z && on ? z[(size_t)b * T + t] : 0.f);
    if (on) d = d * (1.0f - mix) + st * mix;
  }
  // outliers over the slice [1, len-2)
  const int lo = 1, hi = len - 2;
  const bool in_sl = t >= lo && t < hi;
  const float ns = (float)(hi - lo);
  if (hi - lo > 0) {
    const float m2 = block_sum_1024(in_sl ? d : 0.f, red) / ns;
    const float dd = in_sl ? d - m2 : 0.f;
    const float s2 = sqrtf(block_sum_1024(dd * dd, red) / (ns - 1.0f));
    if (in_sl) {
      const float zz = (d - m2) / s2;
      if (fabsf(zz) > 3.0f) {
        const float sg = d > m2 ? 1.0f : (d < m2 ? -1.0f : 0.0f);
        d = m2 + sg * (3.0f * s2 * 0.95f);
      }
    }
  }
  d = d / speed;
  int p = 0;
  if (on) {
    p = (int)rintf(d);
    p = p < 1 ? 1 : p;
  }
  const float mfin = block_sum_1024(on ? d : 0.f, red) / n;
  if (on) {
    dur_out[(size_t)b * T + t] = d;
    pred[(size_t)b * T + t] = p;
  } else if (t < T) {
    dur_out[(size_t)b * T + t] = 0.f;
    pred[(size_t)b * T + t] = 0;
  }
  // inclusive scan of pred over tokens (Hillis-Steele in LDS)
  if (t < DUR_MAX_T) cum[t] = p;
  __syncthreads();
  for (int off = 1; off < DUR_MAX_T; off <<= 1) {
    const int v = (t < DUR_MAX_T && t >= off) ? cum[t - off] : 0;
    __syncthreads();
    if (t < DUR_MAX_T) cum[t] += v;
    __syncthreads();
  }
  if (t == 0) {
    total[b] = len > 0 ? cum[len - 1] : 0;
    if (dur_mean) dur_mean[b] = mfin;
  }
}

// frame_tok[b][f] for f < Fmax: the token whose run covers frame f (pred from k_durations), -1 past
// the utterance's total.  One workgroup per utterance; each token writes its own run.
__global__ void __launch_bounds__(1024) k_frame_map(const int* __restrict__ pred, int T, int Fmax,
                                                    int* __restrict__ frame_tok) {
  __shared__ int cum[DUR_MAX_T];
  const int b = blockIdx.x, t = threadIdx.x;
  const int p = t < T ? pred[(size_t)b * T + t] : 0;
  cum[t] = p;
  __syncthreads();
  for (int off = 1; off < DUR_MAX_T; off <<= 1) {
    const int v = t >= off ? cum[t - off] : 0;
    __syncthreads();
    cum[t] += v;
    __syncthreads();
  }
  const int end = cum[t], start = end - p;
  int* fr = frame_tok + (size_t)b * Fmax;
  for (int f = start; f < end && f < Fmax; ++f) fr[f] = t;
  const int tot = cum[DUR_MAX_T - 1];
  for (int f = tot + t; f < Fmax; f += DUR_MAX_T) fr[f] = -1;
}

// Alignment product as a gather (exact: a one-hot column picks one token):
//   y[b][c][f] = src(b, frame_tok[b][f], c), 0 where frame_tok = -1
// = (t_en @ aln)[b][c][f] (inference.py:268) or (d^T @ aln)[b][c][f] (models.py:432, inference.py:266).
__global__ void __launch_bounds__(256) k_expand_frames(const float* __restrict__ src, long long ss_b, long long ss_t,
                                                       long long ss_c, int C, const int* __restrict__ frame_tok,
                                                       int Fmax, float* __restrict__ y) {
  const int b = blockIdx.z, c = blockIdx.y;
  const int f = blockIdx.x * 256 + threadIdx.x;
  if (f >= Fmax) return;
  const int t = frame_tok[(size_t)b * Fmax + f];
  y[((size_t)b * C + c) * Fmax + f] = t < 0 ? 0.f : src[(size_t)b * ss_b + (size_t)t * ss_t + (size_t)c * ss_c];
}

// ---------------------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------------------
extern "C" {

int stts_frames_gemm(const float* x, long long xs_b, long long xs_t, long long xs_c, int B, int Tin, int Cin,
                     const float* w, long long ws_b, long long ws_n, long long ws_c, long long ws_k, int N, int K,
                     int pad, const float* bias, const float* bias2, float* y, long long ys_b, long long ys_t,
                     long long ys_n, int Tout, void* stream) {
  if (B < 0 || Tin < 0 || Tout < 0 || Cin < 0 || N < 0 || K <= 0 || pad < 0) return ST_EINVAL;
  GemmArgs a{x, xs_b, xs_t, xs_c, Tin, Cin, w, ws_b, ws_n, ws_c, ws_k, N, K, pad, bias, bias2, y, ys_b, ys_t, ys_n, Tout,
             1, 0, nullptr};
  return launch_gemm(a, B, (hipStream_t)stream);
}

int stts_frames_gemm_ws(const float* x, long long xs_b, long long xs_t, long long xs_c, int B, int Tin, int Cin,
                        const float* w, long long ws_b, long long ws_n, long long ws_c, long long ws_k, int N, int K,
                        int pad, const float* bias, const float* bias2, float* y, long long ys_b, long long ys_t,
                        long long ys_n, int Tout, void* workspace, long long ws_bytes, void* stream) {
  if (B < 0 || Tin < 0 || Tout < 0 || Cin < 0 || N < 0 || K <= 0 || pad < 0 || ws_bytes < 0) return ST_EINVAL;
  GemmArgs a{x, xs_b, xs_t, xs_c, Tin, Cin, w, ws_b, ws_n, ws_c, ws_k, N, K, pad, bias, bias2, y, ys_b, ys_t, ys_n, Tout,
             1, 0, nullptr};
  return launch_gemm(a, B, (hipStream_t)stream, (float*)workspace, workspace ? ws_bytes / (long long)sizeof(float) : 0);
}

// byte offset of the int error word in the BiLSTM workspace (after G and W_hh^T); the exchange
// words of the cooperative kernel follow it 8 bytes later
static long long lstm_err_off(int B, int T, int H) {
  return ((long long)2 * B * T * 4 * H + (long long)2 * H * 4 * H) * (long long)sizeof(float);
}

static long long lstm_part_elems(int B, int T, int H) {
  return (long long)B * T <= 256 ? 16LL * B * T * 4 * H : 0;
}

long long stts_bilstm_workspace_bytes(int B, int T, int H) {
  if (B < 0 || T < 0 || H <= 0) return -1;
  // G + W_hh^T (fp32), the cooperative kernel's exchange words (<= 2B groups x 2 x H) and flag, then
  // for text-length inputs (B T <= 256 rows) a split-K scratch for the input projections
  return lstm_err_off(B, T, H) + 8 + (long long)2 * B * 2 * H * 8 + lstm_part_elems(B, T, H) * (long long)sizeof(float);
}

long long stts_bilstm_error_offset(int B, int T, int H) {
  if (B < 0 || T < 0 || H <= 0) return -1;
  return lstm_err_off(B, T, H);
}

int stts_bilstm_fwd(const float* x, long long xs_b, long long xs_t, long long xs_c, int B, int T, int Cin,
                    const int* lengths, const float* const* params, int H, float* y, float* h_n, float* c_n,
                    void* workspace, long long ws_bytes, void* stream) {
  if (B < 0 || T < 0 || Cin <= 0 || !params || !y) return ST_EINVAL;
  if (H <= 0 || H > 256 || (H & 31)) return ST_EINVAL;  // 4H lanes per workgroup, chunks of 8 k-quads
  for (int i = 0; i < 8; ++i)
    if (!params[i]) return ST_EPARAMS;
  if (ws_bytes < stts_bilstm_workspace_bytes(B, T, H)) return ST_EWORKSPACE;
  if (B == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  int* err = (int*)((char*)workspace + lstm_err_off(B, T, H));
  ST_CHECK_HIP(hipMemsetAsync(err, 0, sizeof(int), s));  // the host reads it (stts_bilstm_error_offset)
  float* G = (float*)workspace;
  float* WT = G + (size_t)2 * B * T * 4 * H;
  const int H4 = 4 * H;
  {
    const size_t n = (size_t)2 * H * H4;
    hipLaunchKernelGGL(k_lstm_wt, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, params[1], params[5], H, WT);
    ST_CHECK_HIP(hipGetLastError());
  }
  if (T > 0) {
    for (int d = 0; d < 2; ++d) {
      const float* const* p = params + 4 * d;
      GemmArgs a{x, xs_b, xs_t, xs_c, T, Cin, p[0], 0, Cin, 1, 0, H4, 1, 0, p[2], p[3],
                 G + (size_t)d * B * T * H4, (long long)T * H4, H4, 1, T, 1, 0, nullptr};
      const long long pe = lstm_part_elems(B, T, H);
      float* part = pe ? (float*)((char*)workspace + (stts_bilstm_workspace_bytes(B, T, H) - pe * (long long)sizeof(float)))
                       : nullptr;
      ST_CHECK(launch_gemm(a, B, s, part, pe));
    }
  }
  // utterances per workgroup: 1 (measured fastest at every B from 1 to 64, tools/lstm_sweep.py);
  // 2 / 4 share each W_hh load between utterances (A/B knob stts_set_lstm_group)
  // cooperative path: B <= 4 by default (tools/lstm_sweep.py); -1 forces it
  if (H == COOP_H && (g_lstm_bg == -1 || (g_lstm_bg == 0 && B <= 4)) && B > 0 && T > 0) {
    if (g_coop_groups_cap < 0) {
      g_coop_groups_cap = 0;
      int dev = 0, ncu = 0, coop = 0, occ = 0;
      if (hipGetDevice(&dev) == hipSuccess &&
          hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev) == hipSuccess && coop &&
          hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
          hipFuncSetAttribute((const void*)k_bilstm_coop, hipFuncAttributeMaxDynamicSharedMemorySize,
                              COOP_LDS_BYTES) == hipSuccess &&
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_bilstm_coop, 512, COOP_LDS_BYTES) == hipSuccess)
        g_coop_groups_cap = ((occ * ncu) / COOP_NW) & ~1;
    }
    int groups = 2 * B < g_coop_groups_cap ? 2 * B : g_coop_groups_cap;
    if (groups >= 2) {
      unsigned long long* xe = (unsigned long long*)((char*)err + 8);
      ST_CHECK_HIP(hipMemsetAsync(xe, 0, sizeof(unsigned long long) * groups * 2 * H, s));
      CoopArgs ca{G, params[1], params[5], lengths, B, T, groups, y, h_n, c_n, xe, err, g_coop_spin_limit, g_coop_drop};
      // A plain launch: the grid (<= 2B x 8 = 64 workgroups, one per CU by LDS) was checked against the
      // occupancy query above, which is all hipLaunchCooperativeKernel adds (MI355X_MICROARCH.md
      // coop-launch: +15-19 us of host time per launch).  Under rocprofv3 the cooperative launch also
      // ended the process with a segfault at exit (round 1); the plain launch does not.
      hipLaunchKernelGGL(k_bilstm_coop, dim3(groups * COOP_NW), dim3(512), COOP_LDS_BYTES, s, ca);
      return (int)hipGetLastError();
    }
  }
  const int bg = g_lstm_bg > 0 ? g_lstm_bg : 1;  // (-1 with no co-residency: 1)
  if (bg == 4)
    hipLaunchKernelGGL(k_bilstm_rec<4>, dim3((B + 3) / 4, 2), dim3(H4), 0, s, G, reinterpret_cast<const float4*>(WT), lengths, B, T, H, y, h_n, c_n, nullptr);
  else if (bg == 2)
    hipLaunchKernelGGL(k_bilstm_rec<2>, dim3((B + 1) / 2, 2), dim3(H4), 0, s, G, reinterpret_cast<const float4*>(WT), lengths, B, T, H, y, h_n, c_n, nullptr);
  else
    hipLaunchKernelGGL(k_bilstm_rec<1>, dim3(B, 2), dim3(H4), 0, s, G, reinterpret_cast<const float4*>(WT), lengths, B, T, H, y, h_n, c_n, nullptr);
  return (int)hipGetLastError();
}

int stts_row_norm(const float* x, long long xs_b, long long xs_t, long long xs_c, int B, int T, int C, int mode,
                  const float* gamma, const float* beta, long long gb_sb, float eps, int lrelu, float slope,
                  const int* lengths, const float* extra, int E, float* y, long long ys_b, long long ys_t,
                  void* stream) {
  if (B < 0 || T < 0 || C <= 0 || E < 0 || (E > 0 && !extra) || !x || !y) return ST_EINVAL;
  if (mode < 0 || mode > 2 || (mode != 2 && !gamma) || (mode == 0 && !beta)) return ST_EINVAL;
  const long long rows = (long long)B * T;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(k_row_norm, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream, x, xs_b, xs_t,
                     xs_c, B, T, C, mode, gamma, beta, gb_sb, eps, lrelu, slope, lengths, extra, E, y, ys_b, ys_t);
  return (int)hipGetLastError();
}

int stts_embedding(const long long* tokens, int B, int T, const float* table, int n_symbols, int C,
                   const int* lengths, float* y, int* err_flag, void* stream) {
  if (B < 0 || T < 0 || C <= 0 || n_symbols <= 0 || !tokens || !table || !y) return ST_EINVAL;
  const long long rows = (long long)B * T;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(k_embedding, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream, tokens, B, T,
                     table, n_symbols, C, lengths, y, err_flag);
  return (int)hipGetLastError();
}

int stts_durations(const float* logits, long long ls_b, long long ls_t, int B, int T, int K, const int* lengths,
                   const float* z, float mix, float prev_mean, float speed, float* dur, int* pred, int* total,
                   float* dur_mean, void* stream) {
  if (B < 0 || T < 0 || T > DUR_MAX_T || K <= 0 || !logits || !dur || !pred || !total || !(speed > 0.f))
    return ST_EINVAL;
  if (B == 0) return 0;
  hipLaunchKernelGGL(k_durations, dim3(B), dim3(1024), 0, (hipStream_t)stream, logits, ls_b, ls_t, T, K, lengths, z,
                     mix, prev_mean, speed, dur, pred, total, dur_mean);
  return (int)hipGetLastError();
}

int stts_expand_frames(const float* src, long long ss_b, long long ss_t, long long ss_c, int B, int T, int C,
                       const int* pred, int Fmax, int* frame_tok, float* y, void* stream) {
  if (B < 0 || T < 0 || T > DUR_MAX_T || C <= 0 || Fmax < 0 || !src || !pred || !frame_tok || !y) return ST_EINVAL;
  if (B == 0 || Fmax == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_frame_map, dim3(B), dim3(DUR_MAX_T), 0, s, pred, T, Fmax, frame_tok);
  ST_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_expand_frames, dim3((Fmax + 255) / 256, C, B), dim3(256), 0, s, src, ss_b, ss_t, ss_c, C,
                     frame_tok, Fmax, y);
  return (int)hipGetLastError();
}

}  // extern "C"

int st_wn_fold(const float* v, const float* g, int d0, int inner, float* wout, hipStream_t s);

extern "C" int stts_weight_norm(const float* g, const float* v, int d0, int inner, float* w, void* stream) {
  if (d0 <= 0 || inner <= 0 || !v || !w) return ST_EINVAL;
  return st_wn_fold(v, g, d0, inner, w, (hipStream_t)stream);
}

extern "C" int stts_set_bilstm_debug(int spin_limit, int drop) {
  if (spin_limit < 0) return ST_EINVAL;
  g_coop_spin_limit = spin_limit ? (unsigned)spin_limit : COOP_SPIN_LIMIT;
  g_coop_drop = drop != 0;
  return 0;
}

extern "C" int stts_set_lstm_group(int bg) {
  if (bg != -1 && bg != 0 && bg != 1 && bg != 2 && bg != 4) return ST_EINVAL;
  g_lstm_bg = bg;
  return 0;
}

// ---------------------------------------------------------------------------------------
// BiLSTM training (ProsodyPredictor.shared under train.py's G step: models.py:449, train.py:265, 318, 323):
// full-length sequences (every row length T, as F0Ntrain feeds it), fp32.
//   forward: stts_bilstm_fwd's recurrence on the per-workgroup kernel, also writing every step's cell state;
//   backward (BPTT): the pre-activations Z = x W_ih^T + b_ih + b_hh + h_prev W_hh^T are recomputed for every
//   step at once (frames GEMMs: h_prev is the forward output shifted by one step), a sequential kernel walks
//   each (utterance, direction) backwards through the steps producing dZ (the gate gradients), and the
//   weight / input gradients are frames GEMMs over dZ:
//     dW_ih = dZ^T x, dW_hh = dZ^T h_prev, db_ih = db_hh = sum_t dZ, dx = sum_d dZ_d W_ih_d.
// ---------------------------------------------------------------------------------------
namespace {

// h_prev [B][T][2][H]: direction 0 the output of step t - 1, direction 1 that of step t + 1 (0 at the ends)
__global__ void __launch_bounds__(256) k_lstm_hprev(const float* __restrict__ y, int B, int T, int H,
                                                    float* __restrict__ hp) {
  const size_t n = (size_t)B * T * 2 * H;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int j = (int)(i % H), d = (int)((i / H) & 1);
  const size_t bt = i / (2 * H);
  const int t = (int)(bt % T), b = (int)(bt / T);
  const int tp = d == 0 ? t - 1 : t + 1;
  hp[i] = (tp >= 0 && tp < T) ? y[((size_t)b * T + tp) * 2 * H + (size_t)d * H + j] : 0.f;
}

// One workgroup per (utterance, direction), 4H lanes.  Per step (the direction's forward order reversed):
// lanes j < H turn dh = dy + W_hh^T dZ_{next} and the cell-gradient carry into the four gate gradients of
// hidden unit j; then every lane sums a quarter of k for W_hh^T dZ (coalesced rows of W_hh, dZ broadcast from
// LDS), reduced in fixed order.  Lane j also sums gate row j of dZ over the steps (the bias gradient, per
// utterance; summed over utterances in order by k_lstm_db).
// lengths (may be null): pack_padded_sequence semantics, the direction runs over the first lengths[b] steps only (the
// reverse one from step lengths[b] - 1 with a zero state); dZ rows t >= lengths[b] are zero (no gradient reaches the
// padded positions, as with the reference's packed sequences)
__global__ void __launch_bounds__(1024) k_bilstm_bwd_rec(const float* __restrict__ G, const float* __restrict__ HW,
                                                         const float* __restrict__ cs, const float* __restrict__ dy,
                                                         const float* __restrict__ W0, const float* __restrict__ W1,
                                                         const int* __restrict__ lengths, int B, int T, int H,
                                                         float* __restrict__ dZ, float* __restrict__ dbpart) {
  __shared__ float dz[1024];
  __shared__ float red[4][256];
  __shared__ float dhs[256];
  const int b = blockIdx.x, d = blockIdx.y, j = threadIdx.x, H4 = 4 * H;
  const float* __restrict__ W = d ? W1 : W0;  // [4H][H]
  const int part = j / H, jj = j - part * H;
  int len = lengths ? lengths[b] : T;
  len = len < 0 ? 0 : (len > T ? T : len);
  for (int t = len; t < T; ++t) dZ[(((size_t)b * T + t) * 2 + d) * H4 + j] = 0.f;
  float dc = 0.f, dbacc = 0.f;
  if (j < H) dhs[j] = 0.f;
  __syncthreads();
  for (int s = 0; s < len; ++s) {
    const int t = d == 0 ? len - 1 - s : s;
    if (j < H) {
      const size_t zb = (((size_t)d * B + b) * T + t) * H4;
      const float zi = G[zb + j] + HW[zb + j], zf = G[zb + H + j] + HW[zb + H + j];
      const float zg = G[zb + 2 * H + j] + HW[zb + 2 * H + j], zo = G[zb + 3 * H + j] + HW[zb + 3 * H + j];
      const float ig = sigm(zi), fg = sigm(zf), gg = tanhf(zg), og = sigm(zo);
      const size_t cb = ((size_t)d * B + b) * T;
      const float ct = cs[(cb + t) * H + j];
      const int tp = d == 0 ? t - 1 : t + 1;
      const float cp = (tp >= 0 && tp < len) ? cs[(cb + tp) * H + j] : 0.f;
      const float dh = dy[((size_t)b * T + t) * 2 * H + (size_t)d * H + j] + dhs[j];
      const float tc = tanhf(ct);
      const float dct = dc + dh * og * (1.f - tc * tc);
      const float di = dct * gg * ig * (1.f - ig), df = dct * cp * fg * (1.f - fg);
      const float dg = dct * ig * (1.f - gg * gg), dO = dh * tc * og * (1.f - og);
      dc = dct * fg;
      dz[j] = di;
      dz[H + j] = df;
      dz[2 * H + j] = dg;
      dz[3 * H + j] = dO;
      float* o = dZ + (((size_t)b * T + t) * 2 + d) * H4;
      o[j] = di;
      o[H + j] = df;
      o[2 * H + j] = dg;
      o[3 * H + j] = dO;
    }
    __syncthreads();
    dbacc += dz[j];
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    const float* __restrict__ wp = W + (size_t)part * H * H + jj;
#pragma unroll 8
    for (int k = 0; k < H; ++k) acc[k & 3] = fmaf(wp[(size_t)k * H], dz[part * H + k], acc[k & 3]);
    red[part][jj] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    __syncthreads();
    if (j < H) dhs[j] = (red[0][j] + red[1][j]) + (red[2][j] + red[3][j]);
    __syncthreads();
  }
  dbpart[((size_t)b * 2 + d) * H4 + j] = dbacc;
}

// db[d][k] = sum_b dbpart[b][d][k] in utterance order, into both bias gradients of the direction
__global__ void __launch_bounds__(256) k_lstm_db(const float* __restrict__ part, int B, int H, float* __restrict__ db_ih0,
                                                 float* __restrict__ db_hh0, float* __restrict__ db_ih1,
                                                 float* __restrict__ db_hh1) {
  const int H4 = 4 * H;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= 2 * H4) return;
  const int d = i / H4, k = i - d * H4;
  float v = 0.f;
  for (int b = 0; b < B; ++b) v += part[((size_t)b * 2 + d) * H4 + k];
  float* a = d ? db_ih1 : db_ih0;
  float* c = d ? db_hh1 : db_hh0;
  if (a) a[k] = v;
  if (c) c[k] = v;
}

struct LstmBwdWs {
  float *G, *HW, *hp, *dZ, *Wcat, *dbp;
  long long bytes;
};
LstmBwdWs lstm_bwd_ws(void* base, int B, int T, int Cin, int H) {
  LstmBwdWs w;
  const long long H4 = 4LL * H, bt = (long long)B * T;
  long long off = 0;
  auto take = [&](long long elems) {
    float* p = base ? (float*)((char*)base + off) : nullptr;
    off += (elems * 4 + 255) / 256 * 256;
    return p;
  };
  w.G = take(2 * bt * H4);
  w.HW = take(2 * bt * H4);
  w.hp = take(bt * 2 * H);
  w.dZ = take(bt * 2 * H4);
  w.Wcat = take(2 * H4 * Cin);
  w.dbp = take((long long)B * 2 * H4);
  w.bytes = off;
  return w;
}

}  // namespace

extern "C" int stts_bilstm_fwd_train(const float* x, long long xs_b, long long xs_t, long long xs_c, int B, int T,
                                     int Cin, const int* lengths, const float* const* params, int H, float* y,
                                     float* c_seq, void* workspace, long long ws_bytes, void* stream) {
  if (B < 0 || T < 0 || Cin <= 0 || !params || !y || !c_seq) return ST_EINVAL;
  if (H <= 0 || H > 256 || (H & 31)) return ST_EINVAL;
  for (int i = 0; i < 8; ++i)
    if (!params[i]) return ST_EPARAMS;
  if (ws_bytes < stts_bilstm_workspace_bytes(B, T, H)) return ST_EWORKSPACE;
  if (B == 0 || T == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  float* G = (float*)workspace;
  float* WT = G + (size_t)2 * B * T * 4 * H;
  const int H4 = 4 * H;
  {
    const size_t n = (size_t)2 * H * H4;
    hipLaunchKernelGGL(k_lstm_wt, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, params[1], params[5], H, WT);
    ST_CHECK_HIP(hipGetLastError());
  }
  for (int d = 0; d < 2; ++d) {
    const float* const* p = params + 4 * d;
    GemmArgs a{x, xs_b, xs_t, xs_c, T, Cin, p[0], 0, Cin, 1, 0, H4, 1, 0, p[2], p[3],
               G + (size_t)d * B * T * H4, (long long)T * H4, H4, 1, T, 1, 0, nullptr};
    ST_CHECK(launch_gemm(a, B, s));
  }
  hipLaunchKernelGGL(k_bilstm_rec<1>, dim3(B, 2), dim3(H4), 0, s, G, reinterpret_cast<const float4*>(WT), lengths, B,
                     T, H, y, nullptr, nullptr, c_seq);
  return (int)hipGetLastError();
}

extern "C" long long stts_bilstm_bwd_workspace_bytes(int B, int T, int Cin, int H) {
  if (B < 0 || T < 0 || Cin <= 0 || H <= 0) return ST_EINVAL;
  return lstm_bwd_ws(nullptr, B, T, Cin, H).bytes;
}

extern "C" int stts_bilstm_bwd(const float* x, int B, int T, int Cin, const int* lengths, const float* const* params,
                               int H, const float* y, const float* c_seq, const float* dy, float* dx,
                               float* const* grads, void* workspace, long long ws_bytes, void* stream) {
  if (B < 0 || T < 0 || Cin <= 0 || !params || !x || !y || !c_seq || !dy || !grads) return ST_EINVAL;
  if (H <= 0 || H > 256 || (H & 31)) return ST_EINVAL;
  for (int i = 0; i < 8; ++i)
    if (!params[i]) return ST_EPARAMS;
  const LstmBwdWs w = lstm_bwd_ws(workspace, B, T, Cin, H);
  if (!workspace || ws_bytes < w.bytes) return ST_EWORKSPACE;
  if (B == 0 || T == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int H4 = 4 * H;
  const long long bt = (long long)B * T;
  // h_prev, then Z = x W_ih^T + b_ih + b_hh (G) and h_prev W_hh^T (HW) per direction
  {
    const size_t n = (size_t)bt * 2 * H;
    hipLaunchKernelGGL(k_lstm_hprev, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, y, B, T, H, w.hp);
    ST_CHECK_HIP(hipGetLastError());
  }
  for (int d = 0; d < 2; ++d) {
    const float* const* p = params + 4 * d;
    GemmArgs a{x, (long long)T * Cin, Cin, 1, T, Cin, p[0], 0, Cin, 1, 0, H4, 1, 0, p[2], p[3],
               w.G + (size_t)d * bt * H4, (long long)T * H4, H4, 1, T, 1, 0, nullptr};
    ST_CHECK(launch_gemm(a, B, s));
    GemmArgs h{w.hp + (size_t)d * H, (long long)T * 2 * H, 2 * H, 1, T, H, p[1], 0, H, 1, 0, H4, 1, 0, nullptr, nullptr,
               w.HW + (size_t)d * bt * H4, (long long)T * H4, H4, 1, T, 1, 0, nullptr};
    ST_CHECK(launch_gemm(h, B, s));
  }
  hipLaunchKernelGGL(k_bilstm_bwd_rec, dim3(B, 2), dim3(H4), 0, s, w.G, w.HW, c_seq, dy, params[1], params[5], lengths,
                     B, T, H, w.dZ, w.dbp);
  ST_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_lstm_db, dim3((2 * H4 + 255) / 256), dim3(256), 0, s, w.dbp, B, H, grads[2], grads[3], grads[6],
                     grads[7]);
  ST_CHECK_HIP(hipGetLastError());
  for (int d = 0; d < 2; ++d) {
    const float* dzd = w.dZ + (size_t)d * H4;
    if (grads[4 * d + 0]) {  // dW_ih [4H][Cin] = sum over the B T rows of dZ_d (x) x
      GemmArgs a{dzd, 0, 1, 2LL * H4, H4, (int)bt, x, 0, 1, Cin, 0, Cin, 1, 0, nullptr, nullptr, grads[4 * d + 0], 0,
                 Cin, 1, H4, 1, 0, nullptr};
      ST_CHECK(launch_gemm(a, 1, s));
    }
    if (grads[4 * d + 1]) {  // dW_hh [4H][H] = sum over the rows of dZ_d (x) h_prev_d
      GemmArgs a{dzd, 0, 1, 2LL * H4, H4, (int)bt, w.hp + (size_t)d * H, 0, 1, 2 * H, 0, H, 1, 0, nullptr, nullptr,
                 grads[4 * d + 1], 0, H, 1, H4, 1, 0, nullptr};
      ST_CHECK(launch_gemm(a, 1, s));
    }
  }
  if (dx) {  // dx = [dZ_0 | dZ_1] [W_ih_0; W_ih_1]
    ST_CHECK_HIP(hipMemcpyAsync(w.Wcat, params[0], sizeof(float) * H4 * Cin, hipMemcpyDeviceToDevice, s));
    ST_CHECK_HIP(hipMemcpyAsync(w.Wcat + (size_t)H4 * Cin, params[4], sizeof(float) * H4 * Cin,
                                hipMemcpyDeviceToDevice, s));
    GemmArgs a{w.dZ, (long long)T * 2 * H4, 2 * H4, 1, T, 2 * H4, w.Wcat, 0, 1, Cin, 0, Cin, 1, 0, nullptr, nullptr,
               dx, (long long)T * Cin, Cin, 1, T, 1, 0, nullptr};
    ST_CHECK(launch_gemm(a, B, s));
  }
  return 0;
}
