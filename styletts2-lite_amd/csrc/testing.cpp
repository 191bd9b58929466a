// Test hooks (include/stts2.h, "testing" section): run ONE conv1d_igemm launch on caller
// data so tests can check the conv engine (dilation, stride, polyphase ConvTranspose,
// AdaIN/Snake/LReLU prologues, residual/scale/accumulate epilogues, statistics) against
// torch.nn.functional on the CPU.  Allocates its own scratch (not a product path).
#include <hip/hip_runtime.h>
#include <string.h>

#include "../../include/stts2.h"
#include "common.h"
#include "kernels.h"

extern "C" int stts_test_conv1d(int dtype, const float* x, int B, int Lin, int Cin, const float* w,
                                const float* bias, int Cout, int K, int transposed, int stride, int dil, int pad,
                                int out_pad, int pro_mode, const float* gamma_beta, const float* alpha, float slope,
                                const float* res, float out_scale, float* y, int Lout, double* stats_out) {
  if (dtype != ST_FP32 && dtype != ST_BF16) return ST_EDTYPE;
  const size_t esz = dtype == ST_FP32 ? 4 : 2;
  const int ldx = (Cin + 7) & ~7;
  hipStream_t s = 0;
  char *xd = nullptr, *wd = nullptr, *yd = nullptr, *rd = nullptr;
  double* sx = nullptr;
  const int u = transposed ? stride : 1;
  const size_t wel = st_packed_conv_elems(Cin, Cout, K, transposed, u);
  ST_CHECK_HIP(hipMalloc(&xd, (size_t)B * Lin * ldx * esz));
  ST_CHECK_HIP(hipMemset(xd, 0, (size_t)B * Lin * ldx * esz));
  ST_CHECK_HIP(hipMalloc(&wd, wel * esz));
  ST_CHECK_HIP(hipMalloc(&yd, (size_t)B * Lout * Cout * esz));
  double* so = nullptr;  // the engine's fixed-point statistics (common.h ST_W), decoded into stats_out below
  ST_CHECK_HIP(hipMalloc(&sx, (size_t)B * Cin * ST_W * sizeof(double)));
  ST_CHECK_HIP(hipMemset(sx, 0, (size_t)B * Cin * ST_W * sizeof(double)));
  if (stats_out) {
    ST_CHECK_HIP(hipMalloc(&so, (size_t)B * Cout * ST_W * sizeof(double)));
    ST_CHECK_HIP(hipMemset(so, 0, (size_t)B * Cout * ST_W * sizeof(double)));
  }
  if (res) {
    ST_CHECK_HIP(hipMalloc(&rd, (size_t)B * Lout * Cout * esz));
    ST_CHECK(st_frames_convert(res, B, Lout, Cout, Cout, rd, Cout, nullptr, 0, dtype, s));
  }
  ST_CHECK(st_frames_convert(x, B, Lin, Cin, Cin, xd, ldx, sx, Cin, dtype, s));
  ST_CHECK(st_pack_conv(w, Cin, Cout, K, transposed, u, wd, dtype, s));
  ConvParams p;
  memset(&p, 0, sizeof(p));
  p.x = xd;
  p.x_bs = (long long)Lin * ldx;
  p.x_ld = ldx;
  p.Lin = Lin;
  p.Cin = Cin;
  p.B = B;
  p.w = wd;
  p.nchunks = (Cin + 31) / 32;
  p.bias = bias;
  p.Cout = Cout;
  p.pro.mode = pro_mode;
  p.pro.stats = sx;
  p.pro.stats_ld = Cin;
  p.pro.inv_n = 1.0 / Lin;
  p.pro.gamma = gamma_beta;
  p.pro.gb_ld = 2 * Cin;
  p.pro.gb_C = Cin;
  p.pro.alpha = alpha;
  p.pro.slope = slope;
  if (!transposed) {
    p.KS = K;
    p.dil = dil;
    p.stride = stride;
    p.pad = pad;
    p.N = Cout;
    p.up = 1;
    p.Lq = Lout;
  } else {
    const int taps = (K + u - 1) / u;
    p.KS = taps;
    p.dil = 1;
    p.stride = 1;
    p.pad = taps - 1;
    p.N = u * Cout;
    p.up = u;
    p.opad = pad;
    p.Lq = (Lout - 1 + pad) / u + 1;
  }
  (void)out_pad;
  p.Lout = Lout;
  p.y = yd;
  p.y_bs = (long long)Lout * Cout;
  p.y_ld = Cout;
  p.res = rd;
  p.res_bs = (long long)Lout * Cout;
  p.res_ld = Cout;
  p.out_scale = out_scale;
  p.stats = so;
  p.stats_ld = Cout;
  ST_CHECK(st_conv1d(p, dtype, s));
  if (stats_out) ST_CHECK(st_stats_decode(so, (long long)B * Cout, stats_out, s));
  ST_CHECK(st_frames_to_f32(yd, B, Lout, Cout, Cout, y, dtype, s));
  ST_CHECK_HIP(hipDeviceSynchronize());
  (void)hipFree(xd);
  (void)hipFree(wd);
  (void)hipFree(yd);
  (void)hipFree(sx);
  if (so) (void)hipFree(so);
  if (rd) (void)hipFree(rd);
  return 0;
}
