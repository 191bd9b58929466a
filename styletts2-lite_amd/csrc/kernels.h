// Internal launcher interface (host side) for the gfx950 kernels.  Not part of the
// public C-ABI (include/stts2.h); the plan code in plan.cpp strings these together.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

// ---------------------------------------------------------------- conv1d_igemm
struct ConvParams {
  // input frames [B][Lin][x_ld] (dtype of the run); channels [0, Cin) used
  const void* x;
  long long x_bs;
  int x_ld, Lin, Cin;
  // geometry: input row of output frame q, tap t = q*stride + t*dil - pad
  int B, Lq, KS, dil, stride, pad;
  // GEMM columns and packed weights ([chunk][tap][Np][32] bf16 / [chunk][tap][32][Np] fp32)
  int N;
  const void* w;
  int nchunks;
  const float* bias;  // [Cout], column n uses bias[n % Cout]
  int Cout;
  Prologue pro;
  // epilogue: column n -> (phase n / Cout, channel n % Cout); output row o = q*up + phase - opad
  int up, opad, Lout;
  void* y;
  long long y_bs;
  int y_ld, y_row_off, y_f32;
  const void* res;  // residual, row (o + y_row_off) >> res_shift
  long long res_bs;
  int res_ld, res_shift;
  float out_scale;
  const void* accb;  // running sum buffer (resblock average)
  long long acc_bs;
  int acc_ld;
  float acc_div;
  int epi_tanh, reflect_front;
  int epi_lrelu;      // LeakyReLU(epi_slope) on the stored output (discriminator feature maps)
  float epi_slope;
  int epi_gelu;       // exact (erf) GELU on the stored output (Vocos ConvNeXt pwconv1 -> act)
  double* stats;  // [B][stats_ld][ST_W] accumulated statistics of the stored output (fixed point, common.h)
  int stats_ld;
  // small-batch atomic spreading: workgroup g accumulates into slot g % stats_slots, the slot
  // buffers lying stats_slot_bs doubles apart after `stats` (slot 0 = stats itself); the caller
  // folds slots 1.. into slot 0 after the launch (st_stats_fold).  0 / 1 = direct atomics.
  int stats_slots;
  long long stats_slot_bs;
  // 2-D taps on a zero-padded, row-flattened image (style encoder): tap t reads input row
  // q*stride + (t / kw) * row_off + (t % kw) * dil - pad.  1-D convs: kw = KS, row_off = 0.
  int kw, row_off;
  // zero columns: output rows o with (o % zc_period) >= zc_valid are written as 0 and excluded
  // from the statistics (keeps the padded image borders zero); zc_period = 0 disables.
  int zc_period, zc_valid;
  int dbg;         // phase-skipping timing knob (STTS_OPT_DEBUG; results are wrong when set)
  int skew;        // bigconv2 start skew of half the workgroups (STTS_OPT_SKEW, set by the launcher)
  int exp;         // experiment bits (STTS_OPT_EXP, set by the launchers that read them)
  unsigned long long* stamps;  // diagnostics: per-phase s_memtime cycle sums (stts_set_debug_buffer), or null
  int tg;          // taps per staged weight group (set by the launcher)
  int cps;         // 32-channel chunks per pipeline step, 1 or 2 (set by the launcher)
  int w_resident;  // weights of the column tile stay in LDS across tiles (set by the launcher)
  float* splitk_ws;          // fp32 scratch for split-K partials of small launches (plan workspace), or null
  long long splitk_ws_elems;
  // time expansion (the MSD's (3, kw) Conv2d over [S][H][W][C] frames, conv1d.hip only): with tx_H > 0 the
  // input is x [S H][Lin = W][C = 32] and 32-channel chunk dh (0..2) reads utterance b + dh - 1, zero when
  // (b mod tx_H) + dh - 1 falls outside [0, tx_H): the K dimension is dh-major (k = dh C + c), and the
  // time-expanded image x3[..][dh C + c] = x[b + dh - 1][..][c] is never materialised
  int tx_H;
  // segmented persistent partition (set by the launchers from st_seg_choice): seg > 0 splits every unit
  // (an utterance, or one column tile of an utterance) into seg tile ranges at unit-relative bounds, one virtual
  // workgroup each; 0 = the B x tiles split evenly over the grid
  int seg;
};

// Virtual workgroups of a persistent launch and the tile range [tb, te) of virtual workgroup v < nv.  Segmented: v ->
// (unit v / seg, segment v % seg), tiles [u upt + s upt / seg, u upt + (s + 1) upt / seg) with upt tiles per unit: a
// range never spans two units and its bounds are unit-relative, so the fp32 partial statistics a range accumulates
// (and with them every output bit) do not depend on the batch size, the rank count or the CU count.
__device__ __forceinline__ int tile_nv(const ConvParams& p, long long nunits) {
  return p.seg > 0 ? (int)(nunits * p.seg) : (int)gridDim.x;
}
__device__ __forceinline__ void tile_range(const ConvParams& p, int v, int nv, long long total, long long upt,
                                           long long& tb, long long& te) {
  if (p.seg > 0) {
    const long long u = v / p.seg, s = v % p.seg;
    tb = u * upt + upt * s / p.seg;
    te = u * upt + upt * (s + 1) / p.seg;
  } else {
    tb = total * v / nv;
    te = total * (v + 1) / nv;
  }
}
// host: segments per unit for a launch of B utterances with `upu` units each on a grid of up to gmax workgroups.
// Segmented when B is a multiple of 32 (every config-4 shard, 256 / W utterances): seg = gmax / (32 upu), so B = 32 k
// gives every workgroup k ranges of equal size; 0 (the even split) otherwise, or with STTS_OPT_SEGPART 0
int st_seg_choice(const ConvParams& p, int upu, int gmax);
extern int g_opt_segpart;

int st_conv1d(const ConvParams& p, int dtype, hipStream_t stream);
// slot base of workgroup `g` (see ConvParams::stats_slots)
__device__ __forceinline__ double* stats_slot(const ConvParams& p, int g) {
  return p.stats_slots > 1 ? p.stats + (size_t)(g % p.stats_slots) * p.stats_slot_bs : p.stats;
}
// stats[b][c] += sum of slots 1..S-1, and those slots are zeroed, for b < B, c < C
int st_stats_fold(double* stats, int B, int ld, int C, int slots, long long slot_bs, hipStream_t s);
// n fixed-point statistics entries (ST_W words) -> n (sum, sumsq) fp64 pairs (test hooks)
int st_stats_decode(const double* fx, long long n, double* out, hipStream_t s);
// which engine st_conv1d routes p to (profiling records; bench.py names the dominant kernel)
enum { ST_ENGINE_IGEMM = 0, ST_ENGINE_RESCONV = 1, ST_ENGINE_BIGCONV = 2, ST_ENGINE_RESFUSED = 3, ST_ENGINE_HEAD = 4,
       ST_ENGINE_PW = 5, ST_ENGINE_RESSPLIT = 6, ST_ENGINE_BIGSPLIT = 7 };
// split-operand (ST_SPLIT) resblock convs, C = 32 / 64 (ressplit.hip; C = 64 needs p.splitk_ws >= B Lq 64 floats)
bool st_ressplit_eligible(const ConvParams& p, int dtype);
int st_ressplit(const ConvParams& p, hipStream_t stream);
extern int g_opt_ressplit;
// split-operand (ST_SPLIT) C = 128 / 256 resblock convs, front-end k3 convs, ups[0] / ups[1] on the bigconv2
// engine (bigconv2.hip, SP)
bool st_bigsplit_eligible(const ConvParams& p, int dtype);
int st_bigsplit(const ConvParams& p, hipStream_t stream);
extern int g_opt_bigsplit;  // STTS_OPT_BIGSPLIT
extern int g_opt_bigla;     // STTS_OPT_BIGLA
// C = 64 resblock convs on the bigconv2 engine with 128-frame wave slices (bf16 and / or ST_SPLIT, STTS_OPT_BIG64)
bool st_big64_eligible(const ConvParams& p, int dtype);
int st_big64(const ConvParams& p, int dtype, hipStream_t stream);
extern int g_opt_big64;
int st_conv1d_engine(const ConvParams& p, int dtype);
// resblock conv engine (resconv.hip): bf16, C = 32 / 64, 1-D 'same' dilated conv with the
// AdaIN + Snake prologue.  st_conv1d routes eligible launches to it while g_opt_resconv != 0.
bool st_resconv_eligible(const ConvParams& p, int dtype);
int st_resconv(const ConvParams& p, hipStream_t stream);
extern int g_opt_rcpp;  // STTS_OPT_RCPP
extern int g_opt_rcocc;  // STTS_OPT_RCOCC
bool st_resconv_ups_eligible(const ConvParams& p, int dtype);
int st_resconv_ups(const ConvParams& p, hipStream_t stream);
extern int g_opt_resconv;
extern int g_opt_small_tiles;  // few-tile igemm launches use 64 x 128 tiles (STTS_OPT_SMALL_TILES)
extern int g_opt_grid_cap;  // > 0: cap persistent conv grids (tests: many tiles per block)
extern int g_opt_debug;     // resconv phase-skipping knob (timing experiments only)
extern unsigned long long* g_dbg_stamps;  // stts_set_debug_buffer (diagnostics only)
// wide-stage resblock conv engine (bigconv.hip): bf16, C = 128 / 256, same contract
bool st_bigconv_eligible(const ConvParams& p, int dtype);
int st_bigconv(const ConvParams& p, hipStream_t stream);
// v2 of that engine (bigconv2.hip: per-wave LDS-DMA weight rings, in-place window transform, one
// barrier per 32-channel group); st_bigconv routes to it while g_opt_bigconv == 2 (the default)
bool st_bigconv2_eligible(const ConvParams& p);
int st_bigconv2(const ConvParams& p, hipStream_t stream);
extern int g_opt_bigconv;
extern int g_opt_skew;  // STTS_OPT_SKEW (bigconv2.hip)
extern int g_opt_exp;   // STTS_OPT_EXP (bigconv2.hip, resconv.hip): A/B experiment bits
// the decoder front-end's k3 AdainResBlk1d convs on the bigconv2 engine (STTS_OPT_FRONT)
bool st_front_eligible(const ConvParams& p, int dtype);
int st_bigconv2_front(const ConvParams& p, hipStream_t stream);
// the HiFi-GAN ups[0] / ups[1] polyphase upsamplers on the bigconv2 engine (STTS_OPT_UPS)
extern int g_opt_ups;
extern int g_opt_wgw;
extern int g_opt_bf16f;
extern int g_opt_yf32;  // STTS_OPT_YF32 (convbwd.hip)
extern int g_opt_cout1;  // STTS_OPT_COUT1 (convbwd.hip)
extern int g_opt_plainrc;  // resconv.hip: prologue-free C = 32 / 64 convs (training step) on resconv (STTS_OPT_PLAINRC)  // convbwd.hip: bf16 weight gradient of stride-1 convs on k_wgrad_bf16w (STTS_OPT_WGRAD)
bool st_ups_eligible(const ConvParams& p, int dtype);
int st_bigconv2_ups(const ConvParams& p, hipStream_t stream);
// engine v3 of the same work (bigconv3.hip: 64-channel x 128-frame wave tiles, block-shared weight chunks), routed
// by STTS_OPT_BIG3 bits from st_bigconv / st_bigconv2_front / st_bigconv2_ups
int st_bigconv3(const ConvParams& p, hipStream_t stream);
int st_bigconv3_front(const ConvParams& p, hipStream_t stream);
int st_bigconv3_ups(const ConvParams& p, hipStream_t stream);
extern int g_opt_big3;
extern int g_opt_front;
// HiFi-GAN output head (head.hip): Snake -> conv_post (C -> 1, 7 taps) -> tanh as one streaming pass;
// st_conv1d routes eligible launches to it while g_opt_head != 0
bool st_head_eligible(const ConvParams& p);
int st_head(const ConvParams& p, int dtype, hipStream_t stream);
extern int g_opt_head;
// short-conv GEMM engine (pwgemm.hip): bf16, 1 tap (2 with g_opt_pw == 2), N % 64 == 0, [AdaIN / Snake /
// LReLU] prologue, bias / residual / GELU / statistics epilogue; st_conv1d routes eligible launches to it
bool st_pw_eligible(const ConvParams& p, int dtype);
int st_pw(const ConvParams& p, hipStream_t stream);
// its split-K path for small launches (tiles < CUs / 2, >= 8 chunks, 1-3 'same' taps): needs splitk_ws
bool st_pw_split_eligible(const ConvParams& p, int dtype);
extern int g_opt_splitk;  // STTS_OPT_SPLITK
int st_pw_split(const ConvParams& p, hipStream_t stream);
extern int g_opt_pw;

// fused AdaINResBlock1 iteration (resfused.hip): bf16, C = 32 (K = 3/7/11) or 64 (K = 3): a statistics pass
// (stats_only) then the fused conv1 -> AdaIN2 -> Snake2 -> conv2 -> + x pass.
//   y = conv2(Snake2(AdaIN2(conv1(Snake1(AdaIN1(x)))))) + x     (hifigan.py:65-74)
// pro2.stats must already hold the statistics of conv1's output (a statistics-only conv1 launch).
// y must not alias x (neighbouring tiles read x halos).  accb != null: y = (accb + .) / acc_div
// (acc_div 0 = no division) and no statistics; otherwise statistics of y when stats != null.
struct ResFusedParams {
  const void* x;
  long long x_bs;
  int x_ld, B, L, C, K, dil;
  const void* w1;
  const float* b1;
  Prologue pro1;
  const void* w2;
  const float* b2;
  Prologue pro2;
  void* y;
  long long y_bs;
  int y_ld;
  const void* accb;
  long long acc_bs;
  int acc_ld;
  float acc_div;
  double* stats;
  int stats_ld;
  int stats_slots;  // as ConvParams::stats_slots
  long long stats_slot_bs;
  int stats_only;  // 1: conv1 only over the output frames, its statistics into `stats` (no y, no conv2)
  int dbg;  // phase-skipping timing bits (STTS_OPT_DEBUG, set by st_resfused): 1 prologue math, 2 MFMAs,
            // 4 residual loads + stores, 8 window loads (results are wrong when set)
};
extern int g_opt_resfused;
bool st_resfused_eligible(int C, int K, int dil, int dtype);
int st_resfused(const ResFusedParams& p, hipStream_t stream);

// ---------------------------------------------------------------- misc kernels
// src [B][C][L] fp32 (torch NCL) -> dst frames [B][L][ld] at channel offset c0; optional stats.
int st_ncl_to_frames(const float* src, int B, int C, int L, void* dst, int ld, int c0, long long dst_bs,
                     double* stats, int stats_ld, int dtype, hipStream_t s);
// frames fp32 [B][L][ld_in] -> frames (dtype) [B][L][ld_out]; optional stats
int st_frames_convert(const float* src, int B, int L, int C, int ld_in, void* dst, int ld_out, double* stats,
                      int stats_ld, int dtype, hipStream_t s);
// single-input-channel conv (F0_conv / N_conv / HiFi-GAN noise_convs): in fp32 [B][in_bs]
// out[b][t][c0+c] = bias[c] + sum_k w[c][k] * in[b][t*stride - pad + k]; up to 3 destinations.
struct SmallConvDst {
  void* y;
  long long y_bs;
  int y_ld, c0;
  double* stats;
  int stats_ld;
};
int st_conv_cin1(const float* in, long long in_bs, int Lin, int B, const float* w, const float* bias, int C,
                 int K, int stride, int pad, int Lout, const SmallConvDst* dst, int ndst, int dtype,
                 hipStream_t s);
// HiFi-GAN noise_convs[s] = Conv1d(1, C, K, stride S, padding P) over har fp32 [B][L] ->
// frames (dtype) [B][Lout][C] + statistics (K in {1, 4, 12}; VALU kernel)
int st_noise_conv(const float* har, int B, int L, const float* w, const float* bias, int C, int K, int S, int P,
                  int Lout, void* y, double* stats, int dtype, hipStream_t s);
// har fp32 [B][L] -> S-sample frames (dtype) [B][rows][ld]: x[r][j] = har[S*r - P + j] (j < S), else 0
int st_har_frames(const float* har, int B, int L, int S, int P, int rows, int ld, void* x, int dtype, hipStream_t s);
// noise_convs weight [C][1][2S] -> [C][S][2] (the 2-tap conv over S-sample frames)
int st_reframe_w(const float* w, int C, int S, float* out, hipStream_t s);
int st_fold_w(const float* w, int Cout, int Cin, int K, int st, int pad, int K2, int pad2, float* out, hipStream_t s);
// SineGen phase: ph[b][h][j] = ((cumsum_f64(rad)[j] * 2) * pi) * scale  (fp32)
int st_sine_phase(const float* f0, int B, int n, int scale, float* ph, hipStream_t s);
// SineGen + SourceModuleHnNSF: har[b][t] (fp32), t < n*scale
int st_sine_source(const float* f0, const float* ph, int B, int n, int scale, const float* lw, const float* lb,
                   const float* noise, unsigned long long seed, long long utt_offset, float* har, hipStream_t s);
// depthwise ConvTranspose1d(C, C, 3, stride 2, pad 1, out_pad 1, groups=C) with prologue
int st_pool_dw(const void* x, long long x_bs, int x_ld, int B, int Lin, int C, const float* w, const float* bias,
               const Prologue& pro, void* y, long long y_bs, int y_ld, int dtype, hipStream_t s);
// H[b][n] = bias[n] + sum_k s[b][k] * W[n][k]
int st_linear(const float* s, int B, int K, const float* W, const float* bias, int N, float* H, hipStream_t st);
// column statistics of frames (dtype) [B][L][ld] channels [c0, c0+C) into stats[b][c0+c]
int st_frames_stats(const void* x, long long x_bs, int x_ld, int B, int L, int c0, int C, double* stats,
                    int stats_ld, int dtype, hipStream_t s);
// CustomSTFT.transform: wave fp32 [B][L] -> frames [B][F][ld] with mag (0..nb-1), phase (nb..2nb-1)
int st_stft(const float* wave, int B, int L, int n_fft, int hop, const float* wr, const float* wi, void* y,
            int ld, int dtype, hipStream_t s);
// exp/sin head + CustomSTFT.inverse: post frames [B][F][ld] -> wave fp32 [B][L]
int st_istft(const void* post, int B, int F, int ld, int n_fft, int hop, const float* br, const float* bi,
             float* out, int L, int dtype, hipStream_t s);
// weight-norm fold: wout[i] = v[i] * (g[row]/||v[row]||), rows = d0 of v ([d0][inner]); g may be null (copy)
int st_wn_fold(const float* v, const float* g, int d0, int inner, float* wout, hipStream_t s);
// pack a folded conv weight for conv1d_igemm.
//   transposed == 0: w [Cout][Cin][K]   (nn.Conv1d),           N = Cout,   taps = K
//   transposed == 1: w [Cin][Cout][K]   (nn.ConvTranspose1d),  N = u*Cout, taps = ceil(K/u)
int st_pack_conv(const float* w, int Cin, int Cout, int K, int transposed, int u, void* out, int dtype,
                 hipStream_t s);
size_t st_packed_conv_elems(int Cin, int Cout, int K, int transposed, int u);
// frames (dtype) [B][L][ld] -> fp32 frames [B][L][C]
int st_frames_to_f32(const void* src, int B, int L, int C, int ld, float* dst, int dtype, hipStream_t s);
// acc = ((acc + rs[0]) + rs[1] ...) / div over n contiguous elements (the concurrent resblock branches' average)
int st_branch_avg(void* acc, const void* const* rs, int nr, float div, long long n, int dtype, hipStream_t s);
extern int g_opt_branches;  // STTS_OPT_BRANCHES (plan.cpp)
extern int g_opt_nbranch;   // STTS_OPT_NBRANCH (plan.cpp)
// GAN losses over the MPD engine's outputs (misc.hip): per (period, layer) block, its offset, the
// size of its real half, and whether it is a score block (conv_post)
constexpr int kMpdMaxSegs = 64;
constexpr int kMpdLossBlocks = 64;  // per-segment partial blocks of st_mpd_losses (scratch: 4 doubles each)
struct MpdLossSegs {
  int n;
  long long off[kMpdMaxSegs], half[kMpdMaxSegs];
  int score[kMpdMaxSegs];
};
int st_mpd_losses(const float* out, const MpdLossSegs& sg, double* sums, double* loss, hipStream_t s);
// DiscriminatorP input: waveform [B][Tn] -> frames [B*p][L0][8] (reflect pad to L0*p)
int st_period_frames(const float* wave, int B, int Tn, int p, int L0, void* dst, int dtype, hipStream_t s);
// ---------------------------------------------------------------- style encoder (2-D, padded NHWC)
// An image [H][W] is stored zero-padded as rows (H+2)*(W+2) of ld channels ("padded frames").
// mel fp32 [B][1][H][W] -> padded frames (channel 0), ld = 8
int st_mel_to_padded(const float* mel, int B, int H, int W, void* dst, int dtype, hipStream_t s);
// depthwise Conv2d(C, C, 3, stride 2, pad 1, groups=C) + bias: padded [H][W] -> padded [H/2][ceil(W/2)]
int st_dw_s2(const void* x, int B, int H, int W, int C, const float* w, const float* bias, void* y, int dtype,
             hipStream_t s);
// DownSample('half'): replicate-pad odd W, avg_pool2d(2): padded [H][W] -> padded [H/2][ceil(W/2)]
int st_avgpool_half(const void* x, int B, int H, int W, int C, void* y, int dtype, hipStream_t s);
// AdaptiveAvgPool2d(1) over Wv valid rows of z [B][rows][C] -> LeakyReLU(0.2) -> Linear(C, N)
int st_gap_linear(const void* z, int B, int rows, int Wv, int C, const float* w, const float* bias, int N,
                  float* out, int dtype, hipStream_t s);
// ---------------------------------------------------------------- style front-end (mel.hip)
// Preprocess.wave_preprocess (inference.py:43-49): wave fp32 [B][ld] (L samples each) -> log-mel
// fp32 [B][80][F], F = 1 + L/300.  L must exceed 1024 (reflect padding).
long long st_mel_frames(long long L);
long long st_mel_workspace_bytes();
int st_wave_preprocess(const float* wave, int B, long long L, long long ld, float* mel, void* ws, long long ws_bytes,
                       hipStream_t stream);

// ---------------------------------------------------------------- Vocos decoder (vocos.hip)
// depthwise Conv1d(C, C, 7, pad 3) + bias over frames [B][L][x_ld] -> frames [B][L][y_ld], with the
// per-(utterance, channel) statistics of the output (slot = block % slots) for the next AdaIN
int st_dwconv7(const void* x, long long x_bs, int x_ld, int B, int L, int C, const float* w, const float* bias, void* y,
               long long y_bs, int y_ld, double* stats, int stats_ld, int slots, long long slot_bs, int dtype,
               hipStream_t s);
// LayerNorm(C, eps, affine g / b) over each of `rows` frame rows
int st_frame_ln(const void* x, int x_ld, long long rows, int C, float eps, const float* g, const float* b, void* y,
                int y_ld, int dtype, hipStream_t s);
// ISTFTHead + ISTFT('same'): head frames h [B][F][ld] (dtype; channels [0, nb) log-magnitude, [nb, 2nb)
// phase, nb = N/2 + 1) -> windowed irfft frames fr fp32 [B][F][N] -> out fp32 [B][(F-1) hop + N - 2 pad]
int st_istft_head(const void* h, int B, int F, int ld, int N, int hop, const float* window, float* fr, float* out,
                  int dtype, hipStream_t s);
int st_istft_factor(int N, int* N1, int* N2);
// out[r][i] = r < rows_src ? src[r][i] * (scale ? scale[r] : 1) : 0 for r < rows_dst (pack-time prep)
int st_scale_rows(const float* src, const float* scale, int rows_src, long long inner, int rows_dst, float* out,
                  hipStream_t s);

// ---------------------------------------------------------------- training-step spectra (spec.hip)
long long st_stft_frames(long long L, int hop);
// torchaudio MelSpectrogram(sr, n_fft, win, hop, hann, n_mels) -> (log(1e-5 + mel) + 4) / 4:
// x fp32 [S][ld] (L samples) -> out fp32 [S][n_mels][1 + L / hop]   (losses.py:44-54)
int st_logmel(const float* x, int S, long long L, long long ld, int n_fft, int win, int hop, int n_mels, float sr,
              float* out, hipStream_t s);
// |torch.stft(x, n_fft, hop, win, hann(win))| (Modules/discriminators.py:11-27) time-expanded:
// x3 [S][F][n_fft/2 + 1][8], channel dh = frame h + dh - 1 (channels 3..7 and out-of-range rows are not
// written: zero the buffer first)
int st_stft_mag_x3(const float* x, int S, long long L, long long ld, int n_fft, int win, int hop, void* x3, int dtype,
                   hipStream_t s);
// x3[s][h][w][c * 3 + dh] = y[s][h + dh - 1][w][c], 0 outside [0, H)
int st_time_expand(const void* y, int S, int H, int W, int C, void* x3, int dtype, hipStream_t s, int We = 0);
// SpectralConvergengeLoss numerator / denominator partials of one resolution: part[blk][0] = sum |y - x|,
// part[blk][1] = sum |y| over a fixed split of the n elements (st_sc_part_bytes(1) bytes per resolution)
int st_sc_sums(const float* xm, const float* ym, long long n, double* part, hipStream_t s);
// loss[0] = mean_r (sum of r's part[.][0]) / (sum of r's part[.][1]), partials added in block order
int st_sc_final(const double* part, int nres, double* loss, hipStream_t s);
long long st_sc_part_bytes(int nres);
