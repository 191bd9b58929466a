/*
 * stts2_train.h — training-step (BASELINE config 5) entry points of libstts2.so, beyond the layer
 * forward / backward pairs already in stts2.h (conv1d, ConvTranspose1d, AdaIN1d + activation, Linear,
 * weight norm, pool, LeakyReLU).
 *
 * The reference's fine-tune step (train.py:267-327) runs, per batch: the decoder forward
 * (Modules/hifigan.py:446-475), DiscriminatorLoss (losses.py:170-190) + backward + AdamW on the MPD /
 * MSD (Modules/discriminators.py), then MultiResolutionSTFTLoss (losses.py:58-94) + GeneratorLoss
 * (:149-168) + backward + AdamW on the decoder (optimizers.py:65-73).  Everything below is one piece of
 * that autograd graph that stts2.h does not already cover; stts2_mi355x/training.py, losses.py and
 * optim.py string them together as torch.autograd.Functions.
 *
 * Conventions as stts2.h: DEVICE pointers to contiguous fp32 data, sizes as ints, `stream` a
 * hipStream_t (0 = default), caller-owned memory and workspaces, asynchronous, 0 = ok, >0 hipError_t,
 * <0 STTS_E*.  Every reduction is a fixed-order sum (fp64 partials, added in order): results are
 * bitwise reproducible run to run.  `go` arguments are DEVICE pointers to the autograd upstream
 * gradient of a scalar loss (read by the kernel, so no host synchronisation is needed).
 */
#ifndef STTS2_TRAIN_H
#define STTS2_TRAIN_H

#ifdef __cplusplus
extern "C" {
#endif

/* Snake with a learned per-channel alpha, the Generator's stage activations (hifigan.py:329, :343):
 * y = x + (1 / alpha_c) sin^2(alpha_c x) on frames x, y, dy, dx [B][L][C], alpha [C].  Backward: dx
 * and dalpha [C] (each nullable); workspace >= stts_snake_workspace_bytes(B, L, C). */
long long stts_snake_workspace_bytes(int B, int L, int C);
int stts_snake_fwd(const float* x, const float* alpha, int B, int L, int C, float* y, void* stream);
int stts_snake_bwd(const float* x, const float* alpha, const float* dy, int B, int L, int C, float* dx,
                   float* dalpha, void* ws, long long ws_bytes, void* stream);

/* tanh over n values (hifigan.py:345 after conv_post) and its backward from the output. */
int stts_tanh_fwd(const float* x, long long n, float* y, void* stream);
int stts_tanh_bwd(const float* y, const float* dy, long long n, float* dx, void* stream);

/* y = (xs[0] + xs[1] + ... + xs[k-1]) / div over n values, added left to right: `x + x_source`
 * (hifigan.py:334, div 1) and the resblock average `xs / num_kernels` (:337-342).  `xs` is a HOST array
 * of k <= 8 device pointers.  stts_div: y = x / div (the backward of the average). */
int stts_sum_div(const float* const* xs, int k, long long n, float div, float* y, void* stream);
int stts_div(const float* x, long long n, float div, float* y, void* stream);

/* SourceModuleHnNSF for training (hifigan.py:221-268): f0_curve [B][n] (the Decoder's F0_curve; the
 * Generator upsamples it x scale, :323) -> sw [B][n*scale][9] = the SineGen output sine_waves * uv + noise
 * (computed under no_grad in the reference, :262-263) and har [B][n*scale] = tanh(l_linear(sw)) (:264).
 * noise [B][n*scale][9] = the randn_like draw of :213, or NULL for the counter RNG keyed by
 * (seed, utt_offset + b, sample, harmonic) as stts_decoder_fwd.  Backward: dW [9] and db [1] of l_linear
 * from dhar (the only parameters with a gradient there).  Workspace >= stts_source_workspace_bytes(B, n). */
long long stts_source_workspace_bytes(int B, int n);
int stts_source_fwd(const float* f0_curve, const float* lw, const float* lb, const float* noise,
                    unsigned long long seed, long long utt_offset, int B, int n, int scale, float* sw, float* har,
                    void* ws, long long ws_bytes, void* stream);
/* The same with the seed read from DEVICE memory (seed_dev, or noise given): a hipGraph capture of the training step
 * replays with the seed the caller writes there before each replay (round 5). */
int stts_source_fwd_seed_dev(const float* f0_curve, const float* lw, const float* lb, const float* noise,
                             const unsigned long long* seed_dev, long long utt_offset, int B, int n, int scale,
                             float* sw, float* har, void* ws, long long ws_bytes, void* stream);
int stts_source_bwd(const float* sw, const float* har, const float* dhar, int B, long long L, float* dW, float* db,
                    void* ws, long long ws_bytes, void* stream);

/* Decoder.forward's train-mode F0 / N smoothing (hifigan.py:447-455):
 * y = conv1d(x, ones(1, 1, k), padding k // 2) / k per row of x [B][n], k odd; and its backward. */
int stts_box_smooth_fwd(const float* x, int B, int n, int k, float* y, void* stream);
int stts_box_smooth_bwd(const float* dy, int B, int n, int k, float* dx, void* stream);

/* A (3, kw) Conv2d over (frames, bins) (SpecDiscriminator, discriminators.py:39-47) as a 1-D conv
 * along the bins over 3 C channels: x3[s][h][w][c * 3 + dh] = y[s][h + dh - 1][w][c] (0 outside
 * [0, H)), so the reference's [Cout][C][3][kw] weight is the [Cout][3C][kw] conv1d weight.  Backward:
 * dy[s][h][w][c] = sum_dh dx3[s][h - dh + 1][w][c * 3 + dh]. */
int stts_time_expand3(const float* y, int S, int H, int W, int C, float* x3, void* stream);
int stts_time_expand3_bwd(const float* dx3, int S, int H, int W, int C, float* dy, void* stream);

/* |torch.stft(x, n_fft, hop, win, hann(win), center, reflect, onesided)| (discriminators.py:11-27,
 * :53): wave [S][ld] (L > n_fft / 2 samples) -> mag [S][F][nb] (F = 1 + L / hop, nb = n_fft / 2 + 1:
 * the reference's [S, 1, F, nb] image) and spec [S][F][nb][2] (re, im, kept for the backward).
 * Backward: dwave [S][L] = the stft adjoint (per frame an inverse FFT in LDS, window, then a fixed-order
 * overlap-add gather that folds the reflect padding back) of dspec = dmag * spec / |spec|
 * (0 where |spec| = 0, as torch.abs).  n_fft a power of two <= 2048.
 * Workspace >= stts_stft_mag_workspace_bytes(S, L, n_fft, win, hop). */
long long stts_stft_mag_workspace_bytes(int S, long long L, int n_fft, int win, int hop);
int stts_stft_mag_fwd(const float* wave, int S, long long L, long long ld, int n_fft, int win, int hop, float* mag,
                      float* spec, void* stream);
int stts_stft_mag_bwd(const float* spec, const float* dmag, int S, long long L, int n_fft, int win, int hop,
                      float* dwave, void* ws, long long ws_bytes, void* stream);

/* MultiResolutionSTFTLoss backward (losses.py:24-94; stts_mrstft_loss is the forward): dx [B][L]
 * = go * d loss / d x for x the predicted signal (train.py:281 stft_loss(y_rec, wav)) and y the target.
 * Per resolution: log-mel of y, ||y_mag||_1, then per frame of x the FFT, mel, d|mag| = -sign(y - x) /
 * (n_res ||y_mag||_1), the log / filterbank / power adjoints and the inverse FFT; the frames are
 * overlap-added in fixed order.  The int arrays are HOST pointers.
 * Workspace >= stts_mrstft_bwd_workspace_bytes(B, L, n_ffts, hops, wins, n_res, n_mels). */
long long stts_mrstft_bwd_workspace_bytes(int B, long long L, const int* n_ffts, const int* hops, const int* wins,
                                          int n_res, int n_mels);
int stts_mrstft_loss_bwd(const float* x, const float* y, int B, long long L, long long ld, const int* n_ffts,
                         const int* hops, const int* wins, int n_res, int sample_rate, int n_mels, const float* go,
                         float* dx, void* ws, long long ws_bytes, void* stream);

/* GAN loss terms: the sums GeneratorLoss / DiscriminatorLoss form (losses.py:97-190).  A term reads
 * two equally laid out tensors a, b of n values (a = the real side, b = the generated side):
 *   STTS_GAN_FEATURE  2 mean|a - b|                    feature_loss (:97-103, fmap_r, fmap_g)
 *   STTS_GAN_GEN      mean((1 - b)^2)                  generator_loss (:120-128, b = D(y_hat))
 *   STTS_GAN_DISC     mean((1 - a)^2) + mean(b^2)      discriminator_loss (:106-117)
 *   STTS_GAN_TPRLS    tau - relu(tau - mean(((a - b) - m)^2 over a < b + m)),  m = median(a - b)
 *                     (the lower median, as torch.median), tau = 0.04: discriminator_TPRLS_loss(dr, dg)
 *                     with (a, b) = (dr, dg) and generator_TPRLS_loss(dr, dg) with (a, b) = (dg, dr)
 *                     (:131-147; the latter's loop swaps the names).
 * stts_gan_loss: loss (device, 1 double) = the sum of the terms in order; it also leaves per-term
 * results (median, selected count, mean) in the workspace for the backward.  stts_gan_loss_bwd (after
 * the forward, same terms and workspace): da[i] / db[i] (device, n values each, nullable) = go * the
 * term's gradient w.r.t. a / b (torch's: sign(0) = 0; the median's gradient shared evenly by the
 * elements equal to it; relu'(0) = 0).  `terms`, `da`, `db` are HOST arrays; n_terms <= 256.
 * Workspace >= stts_gan_workspace_bytes(n_terms). */
typedef struct {
  const float* a;
  const float* b;
  long long n;
  int kind;
} stts_gan_term;
#define STTS_GAN_FEATURE 0
#define STTS_GAN_GEN 1
#define STTS_GAN_DISC 2
#define STTS_GAN_TPRLS 3
long long stts_gan_workspace_bytes(int n_terms);
int stts_gan_loss(const stts_gan_term* terms, int n_terms, double* loss, void* ws, long long ws_bytes, void* stream);
int stts_gan_loss_bwd(const stts_gan_term* terms, float* const* da, float* const* db, int n_terms, const float* go,
                      const void* ws, long long ws_bytes, void* stream);

/* AdamW step (torch.optim.AdamW, single-tensor arithmetic order, amsgrad off), as build_optimizer makes it
 * (optimizers.py:65-73: betas (0.0, 0.99), eps 1e-9, weight_decay 1e-4): for every tensor
 *   p *= 1 - lr wd;  m = lerp(m, g, 1 - beta1);  v = v beta2 + (1 - beta2) g g;
 *   p += (-lr / (1 - beta1^step)) m / (sqrt(v) / sqrt(1 - beta2^step) + eps)
 * with `step` the tensor's step count after the increment (1 on the first call).  `tensors` is a HOST
 * array; any number of tensors (one launch per 32).  The hyper-parameters are doubles (Python floats): the
 * scalars 1 - lr wd, 1 - beta1, 1 - beta2, the bias corrections and lr / bc1 are formed in double and rounded
 * to fp32 once, as torch forms them, so the update is bitwise torch's. */
typedef struct {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  long long n;
} stts_adamw_tensor;
int stts_adamw_step(const stts_adamw_tensor* tensors, int n_tensors, double lr, double beta1, double beta2,
                    double eps, double weight_decay, long long step, void* stream);
/* Capturable form (round 5; torch's `capturable=True`): the step count lives in DEVICE memory, state[0] (fp64,
 * >= 8 doubles of state), advanced and turned into the step's scalars by a one-thread launch on the stream, so a
 * hipGraph replay of the call takes the next step's bias corrections without the host.  The scalars are formed in
 * device fp64 (pow: the device library's), so an update may differ from the host form in the last fp32 bit. */
int stts_adamw_step_dev(const stts_adamw_tensor* tensors, int n_tensors, double lr, double beta1, double beta2,
                        double eps, double weight_decay, double* state, void* stream);

/* ---- ProsodyPredictor.F0Ntrain under train.py's G step (train.py:265, 318, 323; models.py:448-461) */

/* Training forward of the bidirectional nn.LSTM(batch_first) layers under train.py's G step: ProsodyPredictor.shared
 * (models.py:449, full-length rows) and, with `lengths` (device int32 [B], NULL = every row has length T; ABI 5), the
 * packed-sequence LSTMs of TextEncoder (models.py:267-279), DurationEncoder (:510-518) and ProsodyPredictor.lstm
 * (:421-430): stts_bilstm_fwd's output y [B][T][2H] (rows t >= len zero; same params, same workspace size) plus
 * every step's cell state c_seq [2][B][T][H] for the backward. */
int stts_bilstm_fwd_train(const float* x, long long xs_b, long long xs_t, long long xs_c, int B, int T, int Cin,
                          const int* lengths, const float* const* params, int H, float* y, float* c_seq,
                          void* workspace, long long ws_bytes, void* stream);
/* Its backward (what autograd computes for nn.LSTM over a packed sequence): x frames [B][T][Cin] contiguous, the same
 * lengths, y and c_seq from the training forward, dy [B][T][2H] -> dx [B][T][Cin] (NULL: not computed; rows t >= len
 * zero) and grads[8] in torch's parameter order (weight_ih_l0, weight_hh_l0, bias_ih_l0, bias_hh_l0, then the
 * _reverse four; NULL entries skipped).  Deterministic (no atomics; the bias gradients summed over utterances in
 * order). */
long long stts_bilstm_bwd_workspace_bytes(int B, int T, int Cin, int H);
int stts_bilstm_bwd(const float* x, int B, int T, int Cin, const int* lengths, const float* const* params, int H,
                    const float* y, const float* c_seq, const float* dy, float* dx, float* const* grads,
                    void* workspace, long long ws_bytes, void* stream);

/* ---- The text / duration path under train.py's G step (train.py:217, 230-233, 286-299, 318, 323, 327; round 5) */

/* Backward of stts_row_norm (include/stts2.h: mode 0 LayerNorm(gamma, beta) + optional LeakyReLU(slope) <- models.py
 * :229-240, 246-249; mode 1 AdaLayerNorm with gb [b][2C] rows gb_sb apart <- :372-392, 503-507; mode 2 the copy of
 * the DurationEncoder's input concat <- :497-501), each with the row mask t >= lengths[b] and E concatenated style
 * columns: x, gamma, beta, gb_sb, eps, lrelu, slope, lengths as the forward; dy [b][t][C + E] (rows dys_b / dys_t
 * apart).  Writes (each nullable) dx [B][T][C] contiguous (masked rows 0), dgamma / dbeta [C] (mode 0),
 * dgb [B][2C] (mode 1: the gradient of the style projection fc(s), gamma half then beta half) and
 * dextra [B][E] = sum_{t < len} dy[b][t][C + e].  Parameter sums are fp64 in row order (deterministic); they need a
 * workspace >= stts_row_norm_bwd_workspace_bytes(B, T, C). */
long long stts_row_norm_bwd_workspace_bytes(int B, int T, int C);
int stts_row_norm_bwd(const float* x, long long xs_b, long long xs_t, long long xs_c, int B, int T, int C, int mode,
                      const float* gamma, const float* beta, long long gb_sb, float eps, int lrelu, float slope,
                      const int* lengths, const float* dy, long long dys_b, long long dys_t, int E, float* dx,
                      float* dgamma, float* dbeta, float* dgb, float* dextra, void* workspace, long long ws_bytes,
                      void* stream);
/* nn.Embedding backward with the masked_fill_ of TextEncoder.forward (models.py:257-260): dW [n_symbols][C] (C <=
 * 1024) = the sum of dy rows (b, t < len) per token id, in row order (deterministic); ids outside range add nothing. */
int stts_embedding_bwd(const long long* tokens, int B, int T, const int* lengths, const float* dy, long long dys_b,
                       long long dys_t, int n_symbols, int C, float* dW, void* stream);
/* The duration losses of train.py:286-299 over the predictor's logits d [B][T][K] (rows ls_b / ls_t apart), the
 * text lengths and d_gt [B][T] (s2s_attn_mono.sum(-1), integer-valued, rows dg_b apart): loss[0] = loss_dur =
 * mean_b l1(sum_k sigmoid(d[b][p]), d_gt[b][p]) over 1 <= p < len - 1, loss[1] = loss_ce = mean_b BCEWithLogits(d[b][:len],
 * trg) with trg[p][k] = k < d_gt[b][p] (fp64, utterance order).  With dlogits [B][T][K] (nullable) also the gradient of
 * g_dur loss_dur + g_ce loss_ce, the two upstream scalars read from DEVICE floats (nullable: 0), so the call needs no
 * host sync.  Workspace >= stts_dur_losses_workspace_bytes(B); T <= 4096. */
long long stts_dur_losses_workspace_bytes(int B);
int stts_dur_losses(const float* logits, long long ls_b, long long ls_t, int B, int T, int K, const int* lengths,
                    const float* d_gt, long long dg_b, double* loss, float* dlogits, const float* g_dur,
                    const float* g_ce, void* workspace, long long ws_bytes, void* stream);

/* nn.Dropout(p) in train mode (the predictor's AdainResBlk1d dropout, models.py:335, 358-367): y = x / (1 - p) where
 * a counter draw u(seed, i) >= p, else 0.  The backward is the same call on dy with the same seed (the mask is
 * redrawn, not stored).  The draws are not torch's (no implementation reproduces those); the seed comes from
 * torch's default generator in the Python layer, so torch.manual_seed governs them. */
int stts_dropout(const float* x, long long n, float p, unsigned long long seed, float* y, void* stream);
/* The same with the keep mask given: y[i] = mask[i] != 0 ? x[i] / (1 - p) : 0 (backward: the same call on dy).  Used
 * when a caller injects the masks (training.set_dropout_masks: train-mode parity against the reference run with the
 * same masks, tests/golden/make_golden_train_text.py). */
int stts_dropout_mask(const float* x, const float* mask, long long n, float p, float* y, void* stream);

/* ---- StyleEncoder under train.py's G step (train.py:258, 324; models.py:125-150), frames images [B][H][W][C] */
/* Row expansion for a k x k Conv2d with padding `pad` in H: xe[b][ho][w][c k + dh] = x[b][ho + dh - pad][w][c]
 * (0 outside), Ho = H + 2 pad - k + 1; the conv then runs as conv1d over W (stts_conv1d_fwd / _bwd) with the
 * reference weight [Cout][Cin][k][k] read as [Cout][Cin k][k].  _bwd: its adjoint (sums over dh in order). */
int stts_rowexp_fwd(const float* x, int B, int H, int W, int C, int k, int pad, float* xe, void* stream);
int stts_rowexp_bwd(const float* dxe, int B, int H, int W, int C, int k, int pad, float* dx, void* stream);
/* LearnedDownSample('half') = depthwise Conv2d(C, C, 3, stride 2, pad 1, groups C) (models.py:13-28):
 * y [B][(H-1)/2+1][(W-1)/2+1][C]; w [C][1][3][3]; bias [C] or NULL.  _bwd: dx, dw, db (each may be NULL), dw / db
 * as fixed-order split sums (workspace >= stts_dwconv2d_s2_workspace_bytes(C)). */
int stts_dwconv2d_s2_fwd(const float* x, const float* w, const float* bias, int B, int H, int W, int C, float* y,
                         void* stream);
long long stts_dwconv2d_s2_workspace_bytes(int C);
int stts_dwconv2d_s2_bwd(const float* x, const float* w, const float* dy, int B, int H, int W, int C, float* dx,
                         float* dw, float* db, void* ws, long long ws_bytes, void* stream);
/* DownSample('half') (models.py:48-62): W odd -> the last column repeated, then avg_pool2d(2):
 * y [B][H/2][(W+1)/2][C]; _bwd its adjoint. */
int stts_avgpool2_fwd(const float* x, int B, int H, int W, int C, float* y, void* stream);
int stts_avgpool2_bwd(const float* dy, int B, int H, int W, int C, float* dx, void* stream);
/* AdaptiveAvgPool2d(1) (models.py:139) over the P = H W positions: y [B][C]; _bwd: dx = dy / P. */
int stts_spatial_mean_fwd(const float* x, int B, int P, int C, float* y, void* stream);
int stts_spatial_mean_bwd(const float* dy, int B, int P, int C, float* dx, void* stream);

/* F.smooth_l1_loss(x, y) (beta 1, mean) <- train.py:269-270 (loss_F0_rec, loss_norm_rec): loss (device, 1 double)
 * from one workgroup's fixed-order fp64 sum; _bwd: dx = g dL/dx, dy = -dx (either may be NULL), g a device float. */
int stts_smooth_l1_loss(const float* x, const float* y, long long n, double* loss, void* stream);
int stts_smooth_l1_loss_bwd(const float* x, const float* y, long long n, const float* g, float* dx, float* dy,
                            void* stream);

#ifdef __cplusplus
}
#endif
#endif /* STTS2_TRAIN_H */
