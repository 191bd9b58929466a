/*
 * stts2.h — C-ABI of the MI355X-native StyleTTS2-lite synthesis path (libstts2.so).
 *
 * The library replaces the compute under these reference interfaces (thewh1teagle/StyleTTS2-lite
 * @ 2025-06-14), keeping their argument meaning:
 *
 *   stts_decoder_fwd  <- Modules/hifigan.py:446  Decoder.forward(asr, F0_curve, N, s)
 *                        Modules/istftnet.py:692 Decoder.forward(asr, F0_curve, N, s)
 *                        Modules/vocos.py:392    Decoder.forward(asr, F0_curve, N, s)
 *   stts_f0n_fwd      <- models.py:448           ProsodyPredictor.F0Ntrain(x, s)  (conv stacks
 *                        after the shared BiLSTM, models.py:451-461)
 *   stts_style_fwd    <- models.py:145           StyleEncoder.forward(x)
 *   stts_wave_preprocess <- inference.py:43      Preprocess.wave_preprocess(wave)
 *   stts_model_create / stts_param_* / stts_set_param / stts_pack
 *                     <- the module constructors + load_state_dict (inference.py:93-124, 150-174)
 *
 * Conventions: every tensor argument is a raw DEVICE pointer (HIP, gfx950) to contiguous
 * float32 data in the reference's own layout; sizes are plain ints; `stream` is a hipStream_t
 * (0 = default stream).  The caller owns all memory: parameters (the state-dict tensors,
 * float32, contiguous), the packed-weight buffer and the workspace.  Nothing is allocated or
 * freed on the device by the library; calls are asynchronous on `stream` and re-entrant per
 * (model, workspace).  Return value: 0 on success, >0 a hipError_t, <0 an STTS_E* code below.
 */
#ifndef STTS2_H
#define STTS2_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct stts_model stts_model;

/* model kinds */
#define STTS_KIND_HIFIGAN 0  /* Modules/hifigan.py Decoder   */
#define STTS_KIND_ISTFTNET 1 /* Modules/istftnet.py Decoder  */
#define STTS_KIND_F0N 2      /* models.py ProsodyPredictor F0/N conv stacks */
#define STTS_KIND_STYLE 3    /* models.py StyleEncoder       */
#define STTS_KIND_MPD 4      /* Modules/discriminators.py MultiPeriodDiscriminator (training step, config 5);
                                cfg = {n, period_1 .. period_n}, the reference's {5, 2, 3, 5, 7, 11} */
#define STTS_KIND_MSD 6      /* Modules/discriminators.py MultiResSpecDiscriminator (training step, config 5);
                                cfg = {n, (fft_size, hop_size, win_length) x n}, the reference's
                                {3, 1024, 120, 600, 2048, 240, 1200, 512, 50, 240} */
#define STTS_KIND_VOCOS 5    /* Modules/vocos.py Decoder (front-end + ConvNeXt generator + ISTFTHead) */

/* compute / activation dtypes */
#define STTS_FP32 0 /* fp32 storage, exact-fp32 MFMA (parity mode)          */
#define STTS_BF16 1 /* bf16 storage, bf16 MFMA with fp32 accumulation      */
#define STTS_SPLIT 2 /* accuracy mode: fp32 storage, conv operands split into bf16 hi + lo,
                        hi*hi + hi*lo + lo*hi on the bf16 MFMA (fp32 accumulation)        */

/* error codes (negative) */
#define STTS_EINVAL (-1)
#define STTS_EDTYPE (-2)
#define STTS_EPARAMS (-3)
#define STTS_EWORKSPACE (-4)
#define STTS_ENOTPACKED (-5)

/*
 * cfg (ints) per kind:
 *   HIFIGAN : dim_in, style_dim, upsample_initial_channel, n_up, rates[n_up], kernels[n_up],
 *             n_rb, rb_kernels[n_rb], rb_dilations[n_rb*3]
 *             (reference Decoder(dim_in, style_dim, resblock_kernel_sizes, upsample_rates,
 *              upsample_initial_channel, resblock_dilation_sizes, upsample_kernel_sizes))
 *   ISTFTNET: as HIFIGAN, then gen_istft_n_fft, gen_istft_hop_size
 *   VOCOS   : dim_in (512), style_dim, intermediate_dim, num_layers, gen_istft_n_fft, gen_istft_hop_size
 *             (reference vocos.Decoder(dim_in, style_dim, dim_out, intermediate_dim, num_layers,
 *              gen_istft_n_fft, gen_istft_hop_size), inference.py:112-118; weight-norm parameters
 *              are named <layer>.parametrizations.weight.original0 / original1 there)
 *   F0N     : d_hid, style_dim                     (ProsodyPredictor(style_dim, d_hid, ...))
 *   STYLE   : dim_in, style_dim, max_conv_dim      (StyleEncoder(dim_in, style_dim, max_conv_dim))
 */
int stts_model_create(int kind, const int* cfg, int ncfg, stts_model** out);
void stts_model_destroy(stts_model* m);

/* Parameters the model reads, named exactly as the reference state-dict keys. */
int stts_param_count(const stts_model* m);
const char* stts_param_name(const stts_model* m, int i);
long long stts_param_numel(const stts_model* m, int i);
int stts_set_param(stts_model* m, int i, const float* dev_ptr);

/* Weight-norm folding + MFMA packing into a caller buffer (once per dtype after load). */
long long stts_packed_bytes(const stts_model* m, int dtype);
int stts_pack(stts_model* m, int dtype, void* packed, long long bytes, void* stream);

/* Workspace for one forward of B utterances of T frames (decoder: T = asr frames;
 * F0N: T = text-aligned frames; STYLE: T = mel frames). */
long long stts_workspace_bytes(const stts_model* m, int dtype, int B, int T);

/* Decoder: asr [B][dim_in][T], F0_curve [B][2T], N [B][2T], s [B][style_dim] -> out [B][1][600T]
 * (VOCOS: out [B][1][2T * gen_istft_hop_size]; it has no source, noise / seed are ignored).
 * noise: [B][600T][9] = the SineGen randn_like draw (hifigan.py:213), or NULL to draw it on the
 * device from a counter RNG keyed by (seed, utt_offset + b, sample, harmonic). */
int stts_decoder_fwd(stts_model* m, int dtype, const float* asr, const float* f0_curve, const float* n,
                     const float* s, const float* noise, unsigned long long seed, long long utt_offset, int B,
                     int T, float* out, void* workspace, long long ws_bytes, void* stream);

/* F0/N conv stacks: x = shared-BiLSTM output [B][T][d_hid] (batch_first, as nn.LSTM returns it),
 * s [B][style_dim] -> F0 [B][2T], N [B][2T]. */
int stts_f0n_fwd(stts_model* m, int dtype, const float* x, const float* s, int B, int T, float* F0, float* N,
                 void* workspace, long long ws_bytes, void* stream);

/* Style encoder: mel [B][1][80][T] -> style [B][style_dim]. */
int stts_style_fwd(stts_model* m, int dtype, const float* mel, int B, int T, float* out, void* workspace,
                   long long ws_bytes, void* stream);

/* MultiPeriodDiscriminator forward, <- Modules/discriminators.py:108-129 DiscriminatorP.forward for
 * every period (MultiPeriodDiscriminator.forward :143-156 calls it on y and y_hat: pass both as one
 * batch).  wave [B][T] fp32 (the reference's [B, 1, T]).  out (fp32, >= stts_mpd_out_elems) receives,
 * period by period, the 6 feature maps of fmap (:118-128, LeakyReLU(0.1) applied to the first 5) as
 * frames [B*p][L_j][C_j], row b*p + j = column j of utterance b: the reference's [B, C_j, L_j, p]
 * tensor is its permutation; the last map (C = 1) flattened is the score.  Workspace:
 * stts_workspace_bytes(m, dtype, B, T).  T must exceed each period's reflect pad, as in the reference. */
long long stts_mpd_out_elems(const stts_model* m, int B, int T);
int stts_mpd_fwd(stts_model* m, int dtype, const float* wave, int B, int T, float* out, long long out_elems,
                 void* workspace, long long ws_bytes, void* stream);
/* GAN losses over stts_mpd_fwd's output for a batch of 2B = B real then B generated waveforms,
 * <- losses.py:97-128 feature_loss(fmap_r, fmap_g), generator_loss(y_d_gs)[0] and
 * discriminator_loss(y_d_rs, y_d_gs)[0] over the MultiPeriodDiscriminator outputs.  loss (device,
 * 3 doubles) = {feature, generator, discriminator}; scratch (device) >= stts_gan_losses_scratch_bytes(m)
 * bytes = 64 * 4 * 6 * n_periods doubles
 * (per-block partial sums, added in block order: the result is bitwise reproducible). */
int stts_mpd_losses(const stts_model* m, int B, int T, const float* out, double* scratch,
                    long long scratch_bytes, double* loss, void* stream);
/* Bytes of `scratch` that stts_mpd_losses / stts_msd_losses need for model m (an MPD or MSD handle);
 * a smaller scratch_bytes returns ST_EWORKSPACE before anything is launched (ABI 4: the size argument
 * was added when the partials went from 4 to 64 blocks per segment). */
long long stts_gan_losses_scratch_bytes(const stts_model* m);

/* Multi-resolution mel loss, <- losses.py:55-94 MultiResolutionSTFTLoss(fft_sizes, hop_sizes, win_lengths)
 * .forward(x, y) as train.py:282 calls it (stft_loss(y_rec, wav)): per resolution r the torchaudio
 * MelSpectrogram(sample_rate, n_ffts[r], wins[r], hops[r], window_fn=hann) (n_mels = 128 at its default,
 * f_max sr/2, power 2, center/reflect, HTK) of x and y, (log(1e-5 + mel) + 4) / 4, and
 * SpectralConvergengeLoss = ||y_mag - x_mag||_1 / ||y_mag||_1 over the whole batch; loss (device, 1 double)
 * = the mean over the n_res resolutions.  x, y: [B][ld] fp32 (L samples each, L > n_fft / 2); n_ffts are
 * powers of two <= 2048 (the reference's 1024, 2048, 512); the int arrays are HOST pointers.
 * Workspace >= stts_mrstft_workspace_bytes(B, L, hops, n_res, n_mels). */
long long stts_mrstft_workspace_bytes(int B, long long L, const int* hops, int n_res, int n_mels);
int stts_mrstft_loss(const float* x, const float* y, int B, long long L, long long ld, const int* n_ffts,
                     const int* hops, const int* wins, int n_res, int sample_rate, int n_mels, double* loss,
                     void* workspace, long long ws_bytes, void* stream);

/* Conv1d forward / backward on caller frames: the conv layers of the training step (config 5).
 * train.py:272-327 calls loss.backward() through the decoder's and the discriminators' nn.Conv1d layers
 * (Modules/hifigan.py:26-80, 292-294, 427-432; Modules/discriminators.py:96-156, weight norm folded):
 * these compute y = conv1d(x, w, bias, stride, padding=pad, dilation=dil) and the gradients torch
 * autograd gives for it.  All tensors fp32 on the device, frames layout (channels contiguous):
 * x / dx [B][Lin][Cin], y / dy [B][Lq][Cout], w / dw [Cout][Cin][K] (nn.Conv1d layout), bias / db [Cout];
 * Lq = (Lin + 2 pad - dil (K - 1) - 1) / stride + 1 must hold (ST_EINVAL otherwise).
 * y and dx run on the conv engine in `dtype` (dx of a stride-1 conv = the forward conv of dy with the
 * channel-transposed, tap-reversed weight and padding dil (K - 1) - pad; of a strided conv (dil 1) = the
 * polyphase ConvTranspose1d of dy); dw / db always compute in fp32 (f32 MFMA over (utterance, frame)
 * row slices, fp64 fixed-order slice sums: deterministic).  dx, dw, db may each be null.
 * Every entry also takes STTS_SPLIT (fp32 frames; y and dx with split-operand MFMA, bf16 hi + lo, three MFMAs;
 * dw / db in fp32 as for STTS_FP32).  stts_conv_transpose1d_* likewise.
 * Workspace >= the matching *_workspace_bytes. */
long long stts_conv1d_fwd_workspace_bytes(int dtype, int B, int Lin, int Cin, int Cout, int K, int stride, int dil,
                                          int pad, int Lq);
int stts_conv1d_fwd(int dtype, const float* x, const float* w, const float* bias, int B, int Lin, int Cin, int Cout,
                    int K, int stride, int dil, int pad, int Lq, float* y, void* workspace, long long ws_bytes,
                    void* stream);
/* The same with a residual added in the epilogue: y = (conv1d(x, w, bias) + res) * scale (res fp32 [B][Lq][Cout];
 * dtype STTS_FP32 / STTS_SPLIT and Cout % 16 == 0 or Cout <= 32; ST_EINVAL otherwise, and for res = NULL with scale != 1).  AdaINResBlock1's x = xt + x
 * (hifigan.py:74) rides on convs2 this way; its gradient w.r.t. res is dy itself. */
int stts_conv1d_fwd_res(int dtype, const float* x, const float* w, const float* bias, const float* res, float scale, int B,
                        int Lin, int Cin, int Cout, int K, int stride, int dil, int pad, int Lq, float* y,
                        void* workspace, long long ws_bytes, void* stream);
/* The same forward with leaky_relu(., slope) applied in the conv epilogue (after the bias): the
 * discriminators' conv -> F.leaky_relu(x, 0.1) pairs (discriminators.py:59-61, 120-123) in one launch.
 * Its gradient is dy * (y > 0 ? 1 : slope) on the output y (slope > 0 keeps the sign), then
 * stts_conv1d_bwd.  Same workspace as stts_conv1d_fwd. */
int stts_conv1d_fwd_act(int dtype, const float* x, const float* w, const float* bias, int B, int Lin, int Cin, int Cout,
                        int K, int stride, int dil, int pad, int Lq, float slope, float* y, void* workspace,
                        long long ws_bytes, void* stream);
/* SpecDiscriminator's (3, kw) Conv2d(C = 32 -> Cout, stride (1, stride), padding (1, pad)) (discriminators.py:
 * 37-45, 58-61) over the image x [S][H frames][W bins][C] in one launch, the time expansion done by the engine's
 * window loads: the conv1d over W of x3 [S H][W][3 C] with x3[s][h][.][dh C + c] = x[s][h + dh - 1][.][c] (zero
 * outside 0 <= h + dh - 1 < H), which is never materialised.  w [Cout][3 C][K] is dh-major (the Conv2d weight
 * [Cout][C][3][K] permuted to [Cout][3][C][K]); y [S H][Lq][Cout]; lrelu != 0 applies leaky_relu(., slope) in
 * the epilogue (as stts_conv1d_fwd_act).  Its backward is stts_conv1d_bwd on the materialised c-major image
 * (stts_time_expand3: channel c 3 + dh) with the Conv2d weight as it lies ([Cout][3 C][K]), then
 * stts_time_expand3_bwd.  C must be 32 (ST_EINVAL). */
long long stts_conv1d_fwd_tx_workspace_bytes(int dtype, int S, int H, int W, int C, int Cout, int K, int stride,
                                             int pad, int Lq);
int stts_conv1d_fwd_tx(int dtype, const float* x, const float* w, const float* bias, int S, int H, int W, int C,
                       int Cout, int K, int stride, int pad, int Lq, int lrelu, float slope, float* y, void* workspace,
                       long long ws_bytes, void* stream);
/* Its input gradient without the expanded image: dx [S][H][W][C] from dy [S H][Lq][Cout] (Cout must be 32) as
 * the dx of a conv C -> 3 Cout whose output chunk j is dy's row h + j - 1, expanded by the engine's loads:
 * wd [3 Cout][C][K] with wd[j Cout + co][c][k] = w[co][c][2 - j][k] (the Conv2d weight's rows reversed, dh-major;
 * torch: w.flip(2).permute(2, 0, 1, 3)). */
long long stts_conv1d_bwd_tx_workspace_bytes(int dtype, int S, int H, int W, int C, int Cout, int K, int stride,
                                             int pad, int Lq);
int stts_conv1d_bwd_tx(int dtype, const float* dy, const float* wd, int S, int H, int W, int C, int Cout, int K,
                       int stride, int pad, int Lq, float* dx, void* workspace, long long ws_bytes, void* stream);
/* And its weight / bias gradient from the image x [S][H][W][C] (C = 32) without expanding it, STTS_BF16 only
 * (STTS_EDTYPE otherwise: the fp32 / split modes run stts_conv1d_bwd on the stts_time_expand3 image), and only
 * for the (K, stride) pairs of the window weight-gradient kernel ((3, 1), (9, 2) and the other stride-1 K <= 11;
 * STTS_EINVAL otherwise or with STTS_OPT_WGRAD 0).  dw [Cout][3 C][K] dh-major (dw[co][dh C + c][k] = the
 * Conv2d weight's gradient at [co][c][dh][k]); db [Cout] or NULL.  Workspace: stts_conv1d_bwd_workspace_bytes
 * (STTS_BF16, S H, W, 3 C, Cout, K, stride, 1, pad, Lq). */
int stts_conv1d_wgrad_tx(int dtype, const float* x, const float* dy, int S, int H, int W, int C, int Cout, int K,
                         int stride, int pad, int Lq, float* dw, float* db, void* workspace, long long ws_bytes,
                         void* stream);
long long stts_conv1d_bwd_workspace_bytes(int dtype, int B, int Lin, int Cin, int Cout, int K, int stride, int dil,
                                          int pad, int Lq);
int stts_conv1d_bwd(int dtype, const float* x, const float* w, const float* dy, int B, int Lin, int Cin, int Cout,
                    int K, int stride, int dil, int pad, int Lq, float* dx, float* dw, float* db, void* workspace,
                    long long ws_bytes, void* stream);

/* ConvTranspose1d forward / backward (the generator's weight-normed upsamplers, hifigan.py:292-294 /
 * 427-432, trained by train.py's backward): y = conv_transpose1d(x, w, bias, stride, padding=pad,
 * output_padding = Lout - ((Lin - 1) stride - 2 pad + K)), x / dx [B][Lin][Cin], y / dy [B][Lout][Cout],
 * w / dw [Cin][Cout][K] (the nn.ConvTranspose1d layout), groups 1, dilation 1.  It is the dx of the
 * conv1d Cout -> Cin with the same weight, so it runs on that path; its backward is that conv's
 * forward (dx) and wgrad with the operands' roles swapped (dw, fp32), db = column sums of dy. */
long long stts_conv_transpose1d_workspace_bytes(int dtype, int B, int Lin, int Cin, int Cout, int K, int stride,
                                                int pad, int Lout);
int stts_conv_transpose1d_fwd(int dtype, const float* x, const float* w, const float* bias, int B, int Lin, int Cin,
                              int Cout, int K, int stride, int pad, int Lout, float* y, void* workspace,
                              long long ws_bytes, void* stream);
int stts_conv_transpose1d_bwd(int dtype, const float* x, const float* w, const float* dy, int B, int Lin, int Cin,
                              int Cout, int K, int stride, int pad, int Lout, float* dx, float* dw, float* db,
                              void* workspace, long long ws_bytes, void* stream);

/* AdaIN1d + activation forward / backward (training step), <- Modules/hifigan.py:14-24 AdaIN1d followed by
 * Snake (:68, AdaINResBlock1) or LeakyReLU(0.2) (:385-395, AdainResBlk1d):
 *   z = (1 + gamma[b][c]) InstanceNorm(x)[b][t][c] + beta[b][c] (eps 1e-5, biased variance);
 *   y = act(z), act 0 identity, 1 Snake z + sin^2(alpha_c z) / alpha_c, 2 LeakyReLU(0.2).
 * x, y, dy, dx [B][L][C] fp32 frames; gb [B][2C] = fc(s) (gamma then beta, the reference's chunk order);
 * alpha [C] (act 1); mean_rstd [B][C][2] is written by the forward and read by the backward.
 * The backward writes dx (nullable), dgb [B][2C] (nullable) and dalpha [C] (act 1, nullable); its
 * column sums are fp64 row-slice partials added in fixed order.  Workspace >= stts_adain_act_workspace_bytes. */
long long stts_adain_act_workspace_bytes(int B, int L, int C);
int stts_adain_act_fwd(const float* x, const float* gb, const float* alpha, int act, int B, int L, int C, float* y,
                       float* mean_rstd, void* workspace, long long ws_bytes, void* stream);
int stts_adain_act_bwd(const float* x, const float* gb, const float* alpha, int act, const float* mean_rstd,
                       const float* dy, int B, int L, int C, float* dx, float* dgb, float* dalpha, void* workspace,
                       long long ws_bytes, void* stream);
/* nn.Linear (the AdaIN style projection fc, hifigan.py:18): h [B][N] = s [B][K] W^T + bias, W [N][K];
 * backward ds [B][K], dW [N][K], db [N] (each nullable; fp64 sums). */
int stts_linear_fwd(const float* s, const float* W, const float* bias, int B, int K, int N, float* h, void* stream);
int stts_linear_bwd(const float* s, const float* W, const float* dh, int B, int K, int N, float* ds, float* dW,
                    float* db, void* stream);
/* AdainResBlk1d's upsampling pieces (hifigan.py:350-403), frames fp32: the depthwise pool
 * ConvTranspose1d(C, C, 3, stride 2, padding 1, output_padding 1, groups C) with w [C][3] (the folded
 * [C][1][3] weight), x [B][Lin][C] -> y [B][2 Lin][C], its backward (dx, dw [C][3], db; fp64 row-slice
 * sums in fixed order, workspace >= stts_pool_workspace_bytes), and the shortcut's nearest x2 upsample
 * with its backward (dx[m] = dy[2m] + dy[2m+1]). */
long long stts_pool_workspace_bytes(int B, int Lin, int C);
int stts_pool_fwd(const float* x, const float* w, const float* bias, int B, int Lin, int C, float* y, void* stream);
int stts_pool_bwd(const float* x, const float* w, const float* dy, int B, int Lin, int C, float* dx, float* dw,
                  float* db, void* workspace, long long ws_bytes, void* stream);
int stts_upsample2(const float* x, int B, int Lin, int C, float* y, void* stream);
int stts_upsample2_bwd(const float* dy, int B, int Lin, int C, float* dx, void* stream);
/* LeakyReLU(slope) over n fp32 values and its backward from the output y (slope > 0), as the
 * discriminators apply it after every conv (discriminators.py:119, slope 0.1). */
int stts_leaky_relu(const float* x, long long n, float slope, float* y, void* stream);
int stts_leaky_relu_bwd(const float* y, const float* dy, long long n, float slope, float* dx, void* stream);
/* weight_norm backward (the training step's convs are weight-normed, hifigan.py:26-80): for w = g v / ||v||
 * per row of v [d0][inner]: dg [d0] = <dw, v> / ||v||, dv = (g / ||v||)(dw - v <dw, v> / ||v||^2). */
int stts_weight_norm_bwd(const float* g, const float* v, const float* dw, int d0, int inner, float* dg, float* dv,
                         void* stream);

/* MultiResSpecDiscriminator forward, <- Modules/discriminators.py:47-63 SpecDiscriminator.forward for every
 * resolution (MultiResSpecDiscriminator.forward :80-94 calls it on y and y_hat: pass both as one batch).
 * wave [B][T] fp32.  out (fp32, >= stts_msd_out_elems) receives, resolution by resolution, the 5
 * LeakyReLU(0.1)-activated feature maps as [B][H][W_j][32] (the reference's [B, 32, H, W_j] permuted;
 * H = 1 + T / hop frames, W = n_fft/2 + 1 bins halved by each stride-(1, 2) conv) and the out map
 * [B][H][W_5] (flattened = the score).  Workspace: stts_workspace_bytes(m, dtype, B, T). */
long long stts_msd_out_elems(const stts_model* m, int B, int T);
int stts_msd_fwd(stts_model* m, int dtype, const float* wave, int B, int T, float* out, long long out_elems,
                 void* workspace, long long ws_bytes, void* stream);
/* The GAN losses of stts_mpd_losses over stts_msd_fwd's output (losses.py:97-128 with the MSD outputs);
 * scratch >= stts_gan_losses_scratch_bytes(m) bytes. */
int stts_msd_losses(const stts_model* m, int B, int T, const float* out, double* scratch,
                    long long scratch_bytes, double* loss, void* stream);

/* Style front-end, <- inference.py:43-49 Preprocess.wave_preprocess(wave) (the torchaudio
 * MelSpectrogram(n_mels=80, n_fft=2048, win_length=1200, hop_length=300) it builds, then
 * (log(1e-5 + mel) + 4) / 4): wave [B][wave_ld] with L samples each (L > 1024) ->
 * mel [B][80][F], F = stts_mel_frames(L) = 1 + L/300 (0 if L <= 1024).  No model handle: the
 * window, twiddle and filterbank tables are rebuilt in the caller's workspace
 * (>= stts_mel_workspace_bytes()) on every call. */
long long stts_mel_frames(long long L);
long long stts_mel_workspace_bytes(void);
int stts_wave_preprocess(const float* wave, int B, long long L, long long wave_ld, float* mel, void* workspace,
                         long long ws_bytes, void* stream);

/* ---- Duration / text path, fp32, stateless (weights are the
 * state-dict tensors themselves).  Activations are frames [B][T][C] unless strides say otherwise;
 * `lengths` is a DEVICE int32 [B] (NULL = every row has length T), the lengths the reference
 * hands to pack_padded_sequence / length_to_mask. */

/* y[b][t][n] = bias[n] + bias2[n] + sum_{k<K, c<Cin} w[b*ws_b + n*ws_n + c*ws_c + k*ws_k] *
 *              x[b*xs_b + (t+k-pad)*xs_t + c*xs_c]      (x rows outside [0, Tin) read as 0)
 * for t < Tout.  Serves  Conv1d  <- models.py:245 (TextEncoder cnn, weight-norm folded),
 *                        Linear  <- models.py:430 duration_proj (LinearNorm, models.py:152-162),
 *                        en = d^T @ aln <- models.py:432 / inference.py:266, asr = t_en @ aln <- inference.py:268. */
int stts_frames_gemm(const float* x, long long xs_b, long long xs_t, long long xs_c, int B, int Tin, int Cin,
                     const float* w, long long ws_b, long long ws_n, long long ws_c, long long ws_k, int N, int K,
                     int pad, const float* bias, const float* bias2, float* y, long long ys_b, long long ys_t,
                     long long ys_n, int Tout, void* stream);
/* Same, with a scratch workspace: when the output has few 64 x 64 tiles (text-length rows) K is split
 * over up to 16 workgroups per tile, partial sums go to the workspace (splits x B x Tout x N floats,
 * fewer splits if it is smaller) and a fixed-order reduction adds them (deterministic). */
int stts_frames_gemm_ws(const float* x, long long xs_b, long long xs_t, long long xs_c, int B, int Tin, int Cin,
                        const float* w, long long ws_b, long long ws_n, long long ws_c, long long ws_k, int N, int K,
                        int pad, const float* bias, const float* bias2, float* y, long long ys_b, long long ys_t,
                        long long ys_n, int Tout, void* workspace, long long ws_bytes, void* stream);

/* Bidirectional single-layer nn.LSTM(batch_first=True) with pack_padded_sequence semantics
 * <- models.py:267-279 (TextEncoder.lstm), :420-430 (ProsodyPredictor.lstm), :449 (shared),
 *    :510-518 (DurationEncoder.lstms).  x(b, t, c) = x[b*xs_b + t*xs_t + c*xs_c], params = the 8
 * state-dict tensors {weight_ih_l0, weight_hh_l0, bias_ih_l0, bias_hh_l0, and the *_reverse four},
 * H = hidden_size (32 | H, H <= 256).  y [B][T][2H] (forward half first, rows t >= len zero);
 * h_n, c_n [2][B][H] or NULL.  Workspace >= stts_bilstm_workspace_bytes(B, T, H). */
long long stts_bilstm_workspace_bytes(int B, int T, int H);
/* Recurrence kernel choice: 0 = automatic (default: the cooperative kernel, W_hh split over 8 workgroups,
 * for H = 256 and B <= 4, else one workgroup per utterance and direction), -1 = cooperative whenever
 * H = 256, 1 / 2 / 4 = utterances per workgroup of the per-workgroup kernel (A/B testing). */
int stts_set_lstm_group(int bg);
int stts_bilstm_fwd(const float* x, long long xs_b, long long xs_t, long long xs_c, int B, int T, int Cin,
                    const int* lengths, const float* const* params, int H, float* y, float* h_n, float* c_n,
                    void* workspace, long long ws_bytes, void* stream);
/* Byte offset in that workspace of a device int the forward zeroes and the cooperative recurrence sets
 * to 1 when a wait for a peer workgroup timed out (y, h_n, c_n are then NaN from that step on): read it
 * after the stream reaches the call (a host sync the caller already makes) and treat non-zero as an
 * error.  Testing hook: stts_set_bilstm_debug(spin_limit (0 = default), drop) makes every wait give up
 * after spin_limit polls and, with drop != 0, one workgroup of each group never publish. */
long long stts_bilstm_error_offset(int B, int T, int H);
int stts_set_bilstm_debug(int spin_limit, int drop);

/* Channel norm of frames rows, fused with LeakyReLU, masking and a style concat:
 *   mode 0 LayerNorm(gamma[C], beta[C])       <- models.py:229-240 (TextEncoder cnn)
 *   mode 1 AdaLayerNorm: (1 + gb[b][c]) xhat + gb[b][C + c], gb = gamma, row stride gb_sb
 *                                             <- models.py:383-392, 503-507 (DurationEncoder)
 *   mode 2 no norm (copy)                     <- models.py:499-501 (the DurationEncoder input concat)
 * x(b, t, c) = x[b*xs_b + t*xs_t + c*xs_c];
 * y[b][t][0..C) = norm (LeakyReLU(slope) if lrelu), y[b][t][C..C+E) = extra[b][..]; rows t >= len = 0. */
int stts_row_norm(const float* x, long long xs_b, long long xs_t, long long xs_c, int B, int T, int C, int mode,
                  const float* gamma, const float* beta, long long gb_sb, float eps, int lrelu, float slope,
                  const int* lengths, const float* extra, int E, float* y, long long ys_b, long long ys_t,
                  void* stream);

/* nn.Embedding + masked_fill_ <- models.py:257-260: tokens int64 [B][T] -> y [B][T][C]; an id outside
 * [0, n_symbols) writes zeros and sets *err_flag |= 1 (device int, may be NULL). */
int stts_embedding(const long long* tokens, int B, int T, const float* table, int n_symbols, int C,
                   const int* lengths, float* y, int* err_flag, void* stream);

/* Durations -> integer frame counts <- inference.py:247-258 (StyleTTS2.__inference): per utterance
 * (its first lengths[b] <= T <= 1024 tokens), dur = sum_k sigmoid(logits[t][k]) over K logits
 * (logits(b, t, k) = logits[b*ls_b + t*ls_t + k]); stats = (prev_mean != 0 ? prev_mean : mean(dur)) +
 * std(dur) * z[b][t] (z = the standard-normal draw of :249-252, NULL = 0); dur = dur (1 - mix) + stats mix;
 * z-score outlier clamp of dur[1:-2] (threshold 3, factor 0.95, :134-148); dur /= speed;
 * pred = max(round_half_even(dur), 1).  Outputs dur [B][T], pred int32 [B][T] (0 past the length),
 * total int32 [B] = sum pred (the alignment width), dur_mean [B] (may be NULL) = the `duration.mean()`
 * the reference returns. */
int stts_durations(const float* logits, long long ls_b, long long ls_t, int B, int T, int K, const int* lengths,
                   const float* z, float mix, float prev_mean, float speed, float* dur, int* pred, int* total,
                   float* dur_mean, void* stream);

/* The alignment products of inference.py:259-268 / models.py:432 without the one-hot matrix: with
 * aln[b][t][f] = 1 for the pred[b][t] frames of token t (tokens in order, pred from stts_durations),
 * y[b][c][f] = sum_t src(b, t, c) aln[b][t][f] = src(b, token of f, c) exactly, 0 past the utterance's
 * total.  src(b, t, c) = src[b*ss_b + t*ss_t + c*ss_c]; y [B][C][Fmax]; frame_tok int32 [B][Fmax] scratch. */
int stts_expand_frames(const float* src, long long ss_b, long long ss_t, long long ss_c, int B, int T, int C,
                       const int* pred, int Fmax, int* frame_tok, float* y, void* stream);

/* weight_norm fold w = g * v / ||v|| (norm over all dims but 0) <- torch.nn.utils.weight_norm as used
 * at models.py:245; v, w [d0][inner], g [d0] (NULL = plain normalisation). */
int stts_weight_norm(const float* g, const float* v, int d0, int inner, float* w, void* stream);

const char* stts_error_string(int code);

/* ABI revision of this header and the library (STTS_ABI_VERSION).  Bumped on every incompatible change of an
 * entry point's signature or meaning (5: round 5; 4 changed stts_adamw_step's scalars to double and added
 * stts_mpd_losses / stts_msd_losses' scratch_bytes).  A caller binding by hand checks
 * stts_abi_version() == STTS_ABI_VERSION before any other call; stts2_mi355x.engine.lib() does. */
#define STTS_ABI_VERSION 5
int stts_abi_version(void);

/* Engine options (process-wide, take effect on the next launch):
 *   STTS_OPT_RESCONV  1 (default) = the specialised resblock conv engine serves the bf16
 *                     C = 32 / 64 dilated convs; 0 = the general implicit-GEMM engine serves them
 *                     (A/B measurement and cross-checking of the two engines). */
#define STTS_OPT_RESCONV 1
/*   STTS_OPT_GRID_CAP n > 0 caps the persistent conv grids at n workgroups (testing: forces many
 *                     tiles and utterance changes per workgroup); 0 (default) = one per CU. */
#define STTS_OPT_GRID_CAP 2
/*   STTS_OPT_RESFUSED 1 = bf16 AdaINResBlock1 iterations at C = 32 (and C = 64, K = 3) run as a
 *                     statistics-only conv1 launch + one fused conv1 -> conv2 launch (resfused.hip);
 *                     0 (default) = two conv launches per iteration (A/B, cross-checking). */
#define STTS_OPT_RESFUSED 3
/*   STTS_OPT_DEBUG    bit mask skipping phases of the resblock engine (1 prologue math, 2 MFMAs,
 *                     4 epilogue) for timing experiments; outputs are WRONG while set.  0 = off. */
#define STTS_OPT_DEBUG 4
/*   STTS_OPT_STATS_SLOTS n > 0: copies of every conv-statistics buffer the persistent grids spread their
 *                     fp64 atomics over (folded after each launch); 0 (default) = 16 for B <= 4, 4 for B <= 16, else 1. */
#define STTS_OPT_STATS_SLOTS 5
/*   STTS_OPT_SMALL_TILES 1 (default) = implicit-GEMM launches that would make fewer than half as many
 *                     256 x 128 tiles as there are CUs use 64 x 128 tiles; 0 = off (A/B). */
#define STTS_OPT_SMALL_TILES 6
/*   STTS_OPT_BIGCONV  2 (default) = the C = 128 / 256 resblock convs run on bigconv2.hip (per-wave
 *                     LDS-DMA weight rings, one barrier per 32-channel group): 8-wave blocks, or
 *                     4-wave blocks two per CU when a launch has fewer 8-wave tiles than CUs (small
 *                     batches) and for C = 128 with 7 / 11 taps; C = 128 with 3 taps on bigconv.hip
 *                     (measured faster); 1 =
 *                     bigconv.hip everywhere; 3 = bigconv2.hip, 4-wave blocks; 4 = bigconv2.hip,
 *                     8-wave blocks (A/B, tests); 5 = as 2, but C = 256 on 8-wave blocks whose second half runs
 *                     one 32-channel group behind the first (three window buffers), so the two waves of a SIMD
 *                     reach their tile epilogues a group apart. */
#define STTS_OPT_BIGCONV 7
/*   STTS_OPT_HEAD     1 (default) = the HiFi-GAN output head (Snake -> conv_post -> tanh) runs as one
 *                     streaming pass (head.hip); 0 = on the igemm engine (A/B). */
#define STTS_OPT_HEAD 8
/*   STTS_OPT_SKEW     0 (default) = every bigconv2 workgroup starts at once; v != 0: half of them
 *                     (odd ones for v > 0, the grid's second half for v < 0) start |v| x 1024 cycles
 *                     late, so two workgroups sharing a CU run out of phase (A/B experiments). */
#define STTS_OPT_SKEW 9
/*   STTS_OPT_FRONT    1 (default) = the decoder front-end's k3 AdainResBlk1d convs (C_out 1024 / 512)
 *                     run on the bigconv2 engine when the launch has at least half as many tiles as
 *                     CUs (else igemm: small batches); 2 = bigconv2 at any size (tests); 0 = igemm. */
#define STTS_OPT_FRONT 10
/*   STTS_OPT_PW       1 (default) = bf16 1x1 convs (the AdainResBlk1d shortcuts, asr_res, the Vocos pointwise
 *                     Linears) run on the short-conv GEMM engine (pwgemm.hip); 2 = the 2-tap polyphase
 *                     upsamplers too (measured slower); 0 = conv1d_igemm (A/B). */
#define STTS_OPT_PW 11
/*   STTS_OPT_SPLITK   1 (default) = small bf16 launches (fewer tiles than half the CUs, >= 8 input chunks,
 *                     1-3 taps: the front-end / F0N convs at B <= 4) run the short-conv engine split over K
 *                     (fp32 slice partials in the plan workspace, summed in slice order; B = 1 decoder
 *                     5.70 -> 4.92 ms); 0 = off. */
#define STTS_OPT_SPLITK 12
/*   STTS_OPT_EXP      bit mask of engine experiments under A/B (tools/ab_engine.py); 0 = the measured
 *                     defaults.  1: bigconv2 static MFMA priority for the second half of the waves;
 *                     2: bigconv2 residual epilogue in one load batch; 4: resconv residual prefetched
 *                     one tile ahead; 32: ups[2] (N = 192) on 4-wave bigconv2 blocks of one output phase per tile
 *                     part instead of 12-wave blocks of all three phases; 64: the accuracy mode's ups[3] with one
 *                     output phase per tile part instead of both. */
#define STTS_OPT_EXP 13
/*   STTS_OPT_UPS      1 = the HiFi-GAN ups[0] / ups[1] / ups[2] polyphase upsamplers (N = 2,560 / 640 / 192) on the
 *                     bigconv2 engine and ups[3] on resconv (default); 2 = ups[2] on conv1d_igemm (A/B); 0 = all on
 *                     conv1d_igemm. */
#define STTS_OPT_UPS 14
/*   STTS_OPT_WGRAD    1 = the bf16 weight gradient of stride-1 convs (stts_conv1d_bwd, training step) on the
 *                     all-taps window kernel k_wgrad_bf16w (default); 0 = the per-tap kernel. */
#define STTS_OPT_WGRAD 15
/*   STTS_OPT_PLAINRC  1 = prologue-free C = 32 / 64 'same' convs (the training step's conv forwards and dx) on the
 *                     resconv engine (default); 0 = on conv1d_igemm. */
#define STTS_OPT_PLAINRC 16
/*   STTS_OPT_MSDFOLD  1 = MultiResSpecDiscriminator models created from now on run their stride-2 layers as
 *                     stride-1 convs over phase-folded frames (weights folded at pack time; default); 0 = the
 *                     strided conv path.  Read at stts_model_create. */
#define STTS_OPT_MSDFOLD 17
/*   STTS_OPT_RCPP     resconv's two-group ping-pong kernel at C = 64 (one 4-wave group computes a 128-frame tile
 *                     while the other runs the previous tile's epilogue and the next window's transform):
 *                     1 = for the residual / running-sum launches with K >= 7 (where it measured faster than
 *                     the lock-step kernel), 2 = for every C = 64 launch, 0 = never; 3 (default, round 6) = those
 *                     launches on the lock-step kernel with the previous tile's epilogue interleaved into the
 *                     MFMA loop instead (3-5 % faster than the ping-pong kernel, profiles/r06_ab_rcpp3.txt). */
#define STTS_OPT_RCPP 18
/*   STTS_OPT_RESSPLIT 1 (default) = the accuracy mode's (STTS_SPLIT) C = 32 / 64 resblock convs run on the split
 *                     resblock engine (ressplit.hip; C = 64 in two input-channel passes); 0 = conv1d_igemm (A/B). */
#define STTS_OPT_RESSPLIT 19
/*   STTS_OPT_BF16F    1 = bf16 training-step convs (stts_conv1d_fwd / _bwd dx) that run on the general engine read
 *                     the caller's fp32 frames directly, rounding the window to bf16 while staging it (4-wave tiles);
 *                     0 (default) = fp32 -> bf16 frame conversion before each such conv (1 % slower step on). */
#define STTS_OPT_BF16F 20
/*   STTS_OPT_YF32     1 (default) = bf16 training-step convs on the general engine store the caller's fp32 output frames
 *                     from the accumulators (no bf16 rounding of y, no conversion pass); 0 = bf16 output + conversion. */
#define STTS_OPT_YF32 21
/*   STTS_OPT_COUT1    1 (default) = training-step conv forwards with one output channel (conv_post, MPD conv_post, the
 *                     F0 / N convs) run as a GEMV (one wave per output frame, fp32 FMAs over the dtype's operands);
 *                     0 = the MFMA engine's 16-column tile (A/B). */
#define STTS_OPT_COUT1 22
/*   STTS_OPT_BRANCHES 8 (default) = decoder forwards of at most this many utterances run a generator stage's resblocks
 *                     1 .. n-1 beside resblock 0 on side streams, and every stage's noise branch on a third, from the
 *                     start (fork / join events on the caller's stream, so they capture into a hipGraph); the
 *                     resblocks are averaged after instead of through the running sum; 0 = off.  (Measured: B = 1
 *                     -29 %, B = 4 -19 %, B = 8 -6 %, B = 16 even, B = 32 +5 % time.) */
#define STTS_OPT_BRANCHES 23
/*   STTS_OPT_NBRANCH  64 (default) = batches up to this size (beyond STTS_OPT_BRANCHES) run only the noise branches on
 *                     a side stream (measured: B = 16 -5 %, B = 32 -1.3 % time); 0 = off (bench.py's per-launch
 *                     profiled pass sets 0, so that the conv launches run alone and their hipEvent durations price
 *                     the kernels, not the overlap). */
#define STTS_OPT_NBRANCH 24
/*   STTS_OPT_BIGSPLIT 1 (default) = the accuracy mode's (STTS_SPLIT) C = 128 / 256 resblock convs, the front-end k3
 *                     convs and ups[0] / ups[1] run on the bigconv2 engine's split-operand variant (16-channel
 *                     groups, 3 MFMAs a product); 3 / 4 = the same on 4- / 8-wave blocks everywhere; 0 = the split
 *                     implicit-GEMM engine (A/B). */
#define STTS_OPT_BIGSPLIT 25
/*   STTS_OPT_BIGLA 1 = the bigconv2 engine's 3-tap (and ups[0]'s 2-tap) launches on 8-wave blocks DMA each window
 *                     two groups ahead into a third LDS buffer, so it lands before its transform; 0 (default) = one
 *                     group ahead (two buffers).  Bit-identical outputs; measured neutral (A/B). */
#define STTS_OPT_BIGLA 26
/*   STTS_OPT_BIG64 bit 1 = the accuracy mode's C = 64 resblock convs on the bigconv2 engine with 128-frame wave
 *                     slices (instead of the two-pass split resblock engine); bit 2 = the bf16 C = 64 resblock convs on it
 *                     too (instead of resconv); bit 4 = on 4-wave blocks, two per CU (else 8-wave); bit 8 = the accuracy mode's C = 32
 *                     convs as well (64-frame slices; slower than the split resblock engine, A/B); default 5; 0 = off. */
#define STTS_OPT_BIG64 27
/*   STTS_OPT_BIG3  bit mask: 1 = the bf16 C = 128 / 256 resblock convs, 2 = the front-end k3 convs, 4 = ups[0] / ups[1] run
 *                     on the v3 engine (64-channel x 128-frame wave tiles, block-shared weight chunks; bitwise equal to
 *                     bigconv2); 8 = its C = 128 convs on 8-wave blocks (else two 4-wave blocks per CU); 0 = off. */
#define STTS_OPT_BIG3 28
/*   STTS_OPT_SEGPART 1 (default) = batches of 32 k utterances split every persistent conv launch into utterance-relative
 *                     tile ranges (kernels.h tile_range), so each workgroup's fp32 partial statistics, and with them every
 *                     output bit, do not depend on the batch size: an N-rank job (256 / N utterances a rank) decodes
 *                     the same bits for every N; 0 = one even range per workgroup.  Only launches
 *                     that keep InstanceNorm statistics are split (no other result depends on the split); a launch
 *                     with one segment per workgroup runs the plain one-range kernel (the same ranges). */
#define STTS_OPT_SEGPART 29
/*   STTS_OPT_RCOCC  1 (default) = resconv's C = 32 launches with K >= 7 and no residual hold their registers to three
 *                     4-wave blocks per CU (168 VGPRs, three waves per SIMD: 5-6 % faster per launch, round 6); 0 = two. */
#define STTS_OPT_RCOCC 30
int stts_set_option(int key, int value);
/* Current value of an option (STTS_EINVAL for an unknown key). */
int stts_get_option(int key);
/* Diagnostics (not a product path): a device buffer of >= 16 uint64 that instrumented engines add
 * per-phase s_memtime cycle sums into (bigconv2.hip: set STTS_OPT_DEBUG bit 64); NULL = off. */
int stts_set_debug_buffer(void* buf);

/* Optional per-launch timing of the conv engines (conv1d_igemm, resconv, bigconv) with hipEvents
 * recorded on `stream` around each launch: enable, run, then read totals (ms, launches). */
int stts_profile_enable(int on);
int stts_profile_read(double* total_ms, long long* launches, double* alg_flops, double* alg_bytes);
/* Launch i of the timed region: shape = {B, rows, N, Cin, taps, dilation, Lout,
 * res | acc<<1 | engine<<4} with engine 0 = conv1d_igemm, 1 = resconv, 2 = bigconv, 3 = resfused,
 * ms_flops_bytes = {hipEvent ms, algorithmic flops, algorithmic bytes}. */
int stts_profile_launch(long long i, int* shape, double* ms_flops_bytes);

/* Diagnostics (not a product path): traffic-counter calibration kernels (csrc/calib.hip) that read or
 * write every byte of a bf16 frames buffer [rows][ld] exactly once (mode 3: plus `halo` rows per tile
 * side) with the conv engines' access patterns: 0 coalesced 16-B loads, 1 LDS-DMA 1 KiB per instruction,
 * 2 / 3 bigconv2's 64-B window row segments per 32-channel group (tile rows, halo), 4 coalesced 16-B
 * stores, 5 bigconv2's epilogue stores, 6 bigconv2's residual loads (the epilogue's per-lane pieces), 7 / 8 the
 * polyphase upsamplers' epilogue stores / residual loads (mode 5 / 6 pieces at rows `halo` apart, phase by phase).  `grid` workgroups of 256 threads; sink[grid] floats.
 * Used by tools/calib_traffic.py under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE. */
int stts_calib_traffic(int mode, void* buf, long long rows, int ld, int tile, int halo, int grid, float* sink,
                       void* stream);

/* ---- testing hook (not a product path): the InstanceNorm statistics entry of every engine (csrc/common.h fx_add /
 * fx_get) summing n parts (mode 0: float parts, the MFMA epilogues' form; 1: double parts), each added by its own
 * lane in no fixed order; out[0] = the total read back (NaN when a part or the total is outside the entry's range).
 * entry: 4 doubles of device scratch; out: 1 double on the device. */
int stts_test_fxsum(int mode, const void* parts, long long n, double* entry, double* out, void* stream);

/* ---- testing hook (not a product path): one conv1d_igemm launch on fp32 frames.
 * x [B][Lin][Cin] frames; w in nn.Conv1d [Cout][Cin][K] / nn.ConvTranspose1d [Cin][Cout][K] layout;
 * pro_mode bitmask 1 = AdaIN (instance stats of x, gamma_beta [B][2*Cin]), 2 = Snake (alpha [Cin]),
 * 4 = LeakyReLU(slope); y = (conv + bias + res) * out_scale, [B][Lout][Cout]; stats_out [B][Cout][2]. */
int stts_test_conv1d(int dtype, const float* x, int B, int Lin, int Cin, const float* w, const float* bias, int Cout,
                     int K, int transposed, int stride, int dil, int pad, int out_pad, int pro_mode,
                     const float* gamma_beta, const float* alpha, float slope, const float* res, float out_scale,
                     float* y, int Lout, double* stats_out);

#ifdef __cplusplus
}
#endif
#endif /* STTS2_H */
