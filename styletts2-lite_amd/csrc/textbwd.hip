// Backward kernels of the text / duration path under train.py's G step (train.py:217, 230-233, 286-299, 318, 323,
// 327): the TextEncoder (models.py:238-299), the DurationEncoder (:468-533) and ProsodyPredictor.forward (:422-446)
// differentiate through
//   * the channel norms of their rows: LayerNorm (+ LeakyReLU + mask) and AdaLayerNorm (+ style concat + mask),
//     the inverse of stts_row_norm (prosody.hip),
//   * the embedding table (nn.Embedding + masked_fill_),
//   * and the duration losses loss_dur / loss_ce of train.py:286-299.
// Everything is deterministic: per-row partials written to scratch, then reduced in a fixed (row) order in fp64.
#include "common.h"
#include "kernels.h"

namespace {

// One wave per (b, t) row, as k_row_norm.  Recomputes the row's mean / rstd exactly as the forward does (same
// summation order), then
//   dv    = dy[0..C) * LeakyReLU'(v)      (v = the forward's pre-activation: xhat gamma + beta, or (1 + gb) xhat + gb')
//   dxhat = dv * g,  g = gamma[c] (mode 0) or 1 + gb[b][c] (mode 1)
//   dx    = rstd (dxhat - sum(dxhat) / C - xhat sum(dxhat xhat) / C)          (mode 2: dx = dy[0..C))
// and the per-row partials p1 = dv xhat, p2 = dv of the affine parameters.  Masked rows (t >= len) write zeros.
__global__ void __launch_bounds__(256) k_row_norm_bwd(const float* __restrict__ x, long long xs_b, long long xs_t,
                                                      long long xs_c, int B, int T, int C, int mode,
                                                      const float* __restrict__ gamma, const float* __restrict__ beta,
                                                      long long gb_sb, float eps, int lrelu, float slope,
                                                      const int* __restrict__ lengths, const float* __restrict__ dy,
                                                      long long dys_b, long long dys_t, float* __restrict__ dx,
                                                      float* __restrict__ p1, float* __restrict__ p2) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (long long)B * T) return;
  const int b = (int)(row / T), t = (int)(row % T);
  const bool valid = !lengths || t < lengths[b];
  float* dxr = dx ? dx + (size_t)row * C : nullptr;
  float* p1r = p1 ? p1 + (size_t)row * C : nullptr;
  float* p2r = p2 ? p2 + (size_t)row * C : nullptr;
  if (!valid) {
    for (int c = lane; c < C; c += 64) {
      if (dxr) dxr[c] = 0.f;
      if (p1r) p1r[c] = 0.f;
      if (p2r) p2r[c] = 0.f;
    }
    return;
  }
  const float* xr = x + (size_t)b * xs_b + (size_t)t * xs_t;
  const float* dyr = dy + (size_t)b * dys_b + (size_t)t * dys_t;
  if (mode == 2) {
    if (dxr)
      for (int c = lane; c < C; c += 64) dxr[c] = dyr[c];
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
  const float* gb = mode == 1 ? gamma + (size_t)b * gb_sb : nullptr;
  // (xhat, dv, dxhat) of channel c
  auto chan = [&](int c, float& xh, float& dv, float& dxh) __attribute__((always_inline)) {
    xh = (xr[(size_t)c * xs_c] - mean) * rstd;
    float g, v;
    if (mode == 0) {
      g = gamma[c];
      v = xh * g + beta[c];
    } else {
      g = 1.0f + gb[c];
      v = g * xh + gb[C + c];
    }
    dv = dyr[c];
    if (lrelu && !(v > 0.f)) dv *= slope;  // torch: grad * (self > 0 ? 1 : negative_slope)
    dxh = dv * g;
  };
  float s1 = 0.f, s2 = 0.f;
  for (int c = lane; c < C; c += 64) {
    float xh, dv, dxh;
    chan(c, xh, dv, dxh);
    s1 += dxh;
    s2 += dxh * xh;
    if (p1r) p1r[c] = dv * xh;
    if (p2r) p2r[c] = dv;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o);
    s2 += __shfl_xor(s2, o);
  }
  if (!dxr) return;
  const float m1 = s1 / (float)C, m2 = s2 / (float)C;
  for (int c = lane; c < C; c += 64) {
    float xh, dv, dxh;
    chan(c, xh, dv, dxh);
    dxr[c] = rstd * (dxh - m1 - xh * m2);
  }
}

// out[b * out_bs + c] = sum over rows r < min(R, len_b) (len_b = lengths[b], or R) of p[b * p_bs + r * p_rs + c],
// in row order, in fp64; one thread per (b, c).  Serves the LayerNorm parameter sums (Bn = 1 over all rows), the
// AdaLayerNorm's per-utterance gamma / beta sums and the style-concat gradient (a strided view of dy).
__global__ void __launch_bounds__(256) k_rows_sum(const float* __restrict__ p, long long p_bs, long long p_rs, int R,
                                                  int C, int Bn, const int* __restrict__ lengths,
                                                  float* __restrict__ out, long long out_bs) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)Bn * C) return;
  const int b = (int)(i / C), c = (int)(i % C);
  int n = R;
  if (lengths) {
    n = lengths[b];
    n = n < 0 ? 0 : (n > R ? R : n);
  }
  const float* q = p + (size_t)b * p_bs + c;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;  // four interleaved chains, added in a fixed order
  int r = 0;
  for (; r + 4 <= n; r += 4) {
    a0 += (double)q[(size_t)r * p_rs];
    a1 += (double)q[(size_t)(r + 1) * p_rs];
    a2 += (double)q[(size_t)(r + 2) * p_rs];
    a3 += (double)q[(size_t)(r + 3) * p_rs];
  }
  for (; r < n; ++r) a0 += (double)q[(size_t)r * p_rs];
  out[(size_t)b * out_bs + c] = (float)((a0 + a1) + (a2 + a3));
}

// nn.Embedding backward with the reference's masked_fill_ (models.py:257-260): dW[sym][c] = sum of dy[b][t][c] over
// the rows (b, t < len_b) whose token is sym, in row order (one workgroup per symbol: the rows' tokens are staged
// 256 at a time in LDS, every thread adds its channels of the matching rows).  Ids outside [0, n_symbols) add nothing.
constexpr int EMB_CPT = 4;  // channels per thread (C <= 1024)
__global__ void __launch_bounds__(256) k_embedding_bwd(const long long* __restrict__ tok, int B, int T,
                                                       const int* __restrict__ lengths, const float* __restrict__ dy,
                                                       long long dys_b, long long dys_t, int C,
                                                       float* __restrict__ dW) {
  __shared__ int rows[256];
  const int sym = blockIdx.x, tid = threadIdx.x;
  float acc[EMB_CPT];
#pragma unroll
  for (int k = 0; k < EMB_CPT; ++k) acc[k] = 0.f;
  const long long n = (long long)B * T;
  for (long long base = 0; base < n; base += 256) {
    const long long r = base + tid;
    int ok = 0;
    if (r < n) {
      const int b = (int)(r / T), t = (int)(r % T);
      ok = tok[r] == (long long)sym && (!lengths || t < lengths[b]);
    }
    rows[tid] = ok;
    __syncthreads();
    const int m = (int)(n - base < 256 ? n - base : 256);
    for (int i = 0; i < m; ++i) {
      if (!rows[i]) continue;
      const long long rr = base + i;
      const int b = (int)(rr / T), t = (int)(rr % T);
      const float* d = dy + (size_t)b * dys_b + (size_t)t * dys_t;
#pragma unroll
      for (int k = 0; k < EMB_CPT; ++k) {
        const int c = tid + 256 * k;
        if (c < C) acc[k] += d[c];
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < EMB_CPT; ++k) {
    const int c = tid + 256 * k;
    if (c < C) dW[(size_t)sym * C + c] = acc[k];
  }
}

// train.py:286-299, per utterance b (one workgroup), with L = text length, z = logits[b][:L][:K], dg = d_gt[b][:L]
// as integers (.long() truncation):
//   trg[p][k] = k < dg[p];  dur[p] = sum_k sigmoid(z[p][k])
//   loss_dur_b = mean_{1 <= p < L-1} |dur[p] - dg[p]|          (F.l1_loss; NaN when L <= 2, as torch's empty mean)
//   loss_ce_b  = mean_{p < L, k} BCEWithLogits(z[p][k], trg[p][k])
// part[b] = (loss_dur_b, loss_ce_b) in fp64.  With dz: the gradient of g_dur / B * sum_b loss_dur_b +
// g_ce / B * sum_b loss_ce_b (rows p >= L zero), g_dur / g_ce read from the device (nullable: 0).
__global__ void __launch_bounds__(256) k_dur_losses(const float* __restrict__ z, long long zs_b, long long zs_t, int B,
                                                    int T, int K, const int* __restrict__ lengths,
                                                    const float* __restrict__ dgt, long long dg_b,
                                                    double* __restrict__ part, float* __restrict__ dz,
                                                    const float* __restrict__ gp_dur, const float* __restrict__ gp_ce) {
  extern __shared__ double sh[];  // [T] dur sums, [T] bce row sums
  double* dur = sh;
  double* bce = sh + T;
  const int b = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int L = lengths ? lengths[b] : T;
  L = L < 0 ? 0 : (L > T ? T : L);
  const float* zb = z + (size_t)b * zs_b;
  for (int p = w; p < L; p += 4) {
    const float* zr = zb + (size_t)p * zs_t;
    const long long dgi = (long long)dgt[(size_t)b * dg_b + p];
    double sd = 0.0, sb = 0.0;
    for (int k = lane; k < K; k += 64) {
      const double v = (double)zr[k];
      const double sg = 1.0 / (1.0 + exp(-v));
      const double y = k < dgi ? 1.0 : 0.0;
      const double mx = v < 0.0 ? -v : 0.0;  // torch: (1 - y) z + max(-z, 0) + log(exp(-max) + exp(-z - max))
      sd += sg;
      sb += (1.0 - y) * v + mx + log(exp(-mx) + exp(-v - mx));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      sd += __shfl_xor(sd, o);
      sb += __shfl_xor(sb, o);
    }
    if (lane == 0) {
      dur[p] = sd;
      bce[p] = sb;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double ld = 0.0, lc = 0.0;
    for (int p = 1; p < L - 1; ++p) {
      const double dg = (double)(long long)dgt[(size_t)b * dg_b + p];
      ld += fabs((double)(float)dur[p] - dg);
    }
    for (int p = 0; p < L; ++p) lc += bce[p];
    part[2 * b] = ld / (double)(L - 2);  // (0 / 0 = NaN for L <= 2, as F.l1_loss over no elements)
    part[2 * b + 1] = lc / ((double)L * K);
  }
  if (!dz) return;
  const float g_dur = gp_dur ? *gp_dur : 0.f, g_ce = gp_ce ? *gp_ce : 0.f;
  const double gc = (double)g_ce / B / ((double)L * K), gd = (double)g_dur / B / (double)(L - 2);
  float* dzb = dz + (size_t)b * T * K;
  for (long long i = threadIdx.x; i < (long long)T * K; i += 256) {
    const int p = (int)(i / K), k = (int)(i % K);
    float g = 0.f;
    if (p < L) {
      const double v = (double)zb[(size_t)p * zs_t + k];
      const double sg = 1.0 / (1.0 + exp(-v));
      const long long dgi = (long long)dgt[(size_t)b * dg_b + p];
      double d = gc * (sg - (k < dgi ? 1.0 : 0.0));
      if (p >= 1 && p < L - 1) {
        const double diff = (double)(float)dur[p] - (double)dgi;
        const double sgn = diff > 0.0 ? 1.0 : (diff < 0.0 ? -1.0 : 0.0);  // torch's l1 backward: sign, 0 at 0
        d += gd * sgn * sg * (1.0 - sg);
      }
      g = (float)d;
    }
    dzb[i] = g;
  }
}

// loss[0] = sum_b part[b][0] / B (loss_dur), loss[1] = sum_b part[b][1] / B (loss_ce), in utterance order
__global__ void k_dur_final(const double* __restrict__ part, int B, double* __restrict__ loss) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double a = 0.0, c = 0.0;
  for (int b = 0; b < B; ++b) {
    a += part[2 * b];
    c += part[2 * b + 1];
  }
  loss[0] = a / B;
  loss[1] = c / B;
}

}  // namespace

extern "C" long long stts_row_norm_bwd_workspace_bytes(int B, int T, int C) {
  if (B < 0 || T < 0 || C <= 0) return ST_EINVAL;
  return 2LL * B * T * C * 4;
}

extern "C" int stts_row_norm_bwd(const float* x, long long xs_b, long long xs_t, long long xs_c, int B, int T, int C,
                                 int mode, const float* gamma, const float* beta, long long gb_sb, float eps, int lrelu,
                                 float slope, const int* lengths, const float* dy, long long dys_b, long long dys_t,
                                 int E, float* dx, float* dgamma, float* dbeta, float* dgb, float* dextra,
                                 void* workspace, long long ws_bytes, void* stream) {
  if (B < 0 || T < 0 || C <= 0 || E < 0 || mode < 0 || mode > 2 || !dy) return ST_EINVAL;
  if (mode != 2 && !x) return ST_EINVAL;
  if (mode == 0 && (!gamma || !beta)) return ST_EINVAL;
  if (mode == 1 && !gamma) return ST_EINVAL;
  const long long rows = (long long)B * T;
  if (rows == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const bool params = (mode == 0 && (dgamma || dbeta)) || (mode == 1 && dgb);
  float *p1 = nullptr, *p2 = nullptr;
  if (params) {
    if (!workspace || ws_bytes < stts_row_norm_bwd_workspace_bytes(B, T, C)) return ST_EWORKSPACE;
    p1 = (float*)workspace;
    p2 = p1 + (size_t)rows * C;
  }
  if (dx || params) {
    hipLaunchKernelGGL(k_row_norm_bwd, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, x, xs_b, xs_t, xs_c, B, T, C,
                       mode, gamma, beta, gb_sb, eps, lrelu, slope, lengths, dy, dys_b, dys_t, dx, p1, p2);
    ST_CHECK_HIP(hipGetLastError());
  }
  if (mode == 0 && params) {
    const unsigned g = (unsigned)((C + 255) / 256);
    if (dgamma) hipLaunchKernelGGL(k_rows_sum, dim3(g), dim3(256), 0, s, p1, 0LL, (long long)C, (int)rows, C, 1,
                                   (const int*)nullptr, dgamma, 0LL);
    if (dbeta) hipLaunchKernelGGL(k_rows_sum, dim3(g), dim3(256), 0, s, p2, 0LL, (long long)C, (int)rows, C, 1,
                                  (const int*)nullptr, dbeta, 0LL);
    ST_CHECK_HIP(hipGetLastError());
  }
  if (mode == 1 && dgb) {  // dgb[b][0..C) = sum_t dv xhat (gamma), dgb[b][C..2C) = sum_t dv (beta)
    const unsigned g = (unsigned)(((long long)B * C + 255) / 256);
    hipLaunchKernelGGL(k_rows_sum, dim3(g), dim3(256), 0, s, p1, (long long)T * C, (long long)C, T, C, B,
                       (const int*)nullptr, dgb, 2LL * C);
    hipLaunchKernelGGL(k_rows_sum, dim3(g), dim3(256), 0, s, p2, (long long)T * C, (long long)C, T, C, B,
                       (const int*)nullptr, dgb + C, 2LL * C);
    ST_CHECK_HIP(hipGetLastError());
  }
  if (E > 0 && dextra) {  // the concatenated style columns: dextra[b][e] = sum_{t < len} dy[b][t][C + e]
    const unsigned g = (unsigned)(((long long)B * E + 255) / 256);
    hipLaunchKernelGGL(k_rows_sum, dim3(g), dim3(256), 0, s, dy + C, dys_b, dys_t, T, E, B, lengths, dextra, (long long)E);
    ST_CHECK_HIP(hipGetLastError());
  }
  return 0;
}

extern "C" int stts_embedding_bwd(const long long* tokens, int B, int T, const int* lengths, const float* dy,
                                  long long dys_b, long long dys_t, int n_symbols, int C, float* dW, void* stream) {
  if (B < 0 || T < 0 || C <= 0 || C > 256 * EMB_CPT || n_symbols <= 0 || !tokens || !dy || !dW) return ST_EINVAL;
  hipLaunchKernelGGL(k_embedding_bwd, dim3(n_symbols), dim3(256), 0, (hipStream_t)stream, tokens, B, T, lengths, dy,
                     dys_b, dys_t, C, dW);
  return (int)hipGetLastError();
}

extern "C" long long stts_dur_losses_workspace_bytes(int B) { return B < 0 ? ST_EINVAL : 16LL * (B > 0 ? B : 1); }

extern "C" int stts_dur_losses(const float* logits, long long ls_b, long long ls_t, int B, int T, int K,
                               const int* lengths, const float* d_gt, long long dg_b, double* loss, float* dlogits,
                               const float* g_dur, const float* g_ce, void* workspace, long long ws_bytes,
                               void* stream) {
  if (B <= 0 || T <= 0 || K <= 0 || !logits || !d_gt || !loss) return ST_EINVAL;
  if (T > 4096) return ST_EINVAL;  // (the per-row sums live in LDS)
  if (!workspace || ws_bytes < stts_dur_losses_workspace_bytes(B)) return ST_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  double* part = (double*)workspace;
  hipLaunchKernelGGL(k_dur_losses, dim3(B), dim3(256), (size_t)2 * T * sizeof(double), s, logits, ls_b, ls_t, B, T, K,
                     lengths, d_gt, dg_b, part, dlogits, g_dur, g_ce);
  ST_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_dur_final, dim3(1), dim3(64), 0, s, part, B, loss);
  return (int)hipGetLastError();
}
