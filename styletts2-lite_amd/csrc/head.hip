// HiFi-GAN output head: Snake(alpha_last) -> conv_post (Conv1d(C, 1, 7, padding 3)) -> tanh
// (Modules/hifigan.py:343-345), one pass over the last stage's frames.
//
// Why not the igemm engine: a 1-column GEMM leaves 31 of 32 MFMA columns idle and re-reads every
// input row 7 times through its tap loop (446 us per 10-s x 32 batch, profiles/r02_ab_*), while the
// head is a pure stream: read C channels of every frame once (64 B / frame at C = 32 bf16), write
// one fp32 sample.  HBM floor at 32 x 240,000 frames: 522 MB -> ~95 us.
//
// Work split: a workgroup of 256 threads owns 256 input rows [r0, r0 + 256) of one utterance and
// writes the 250 outputs whose 7-row window lies inside them.  Thread r loads its row (C channels,
// contiguous across threads: coalesced), applies Snake in fp32 and produces the row's 7 tap
// partials z_k(r) = sum_c w[c][k] * snake(x[r][c]) (packed-fp32 FMAs over channel pairs); output
// q = sum_k z_k(q + k - 3) + bias, read back from LDS (stride 7 floats: conflict-free).
#include "common.h"
#include "conv_common.h"
#include "kernels.h"

namespace {

constexpr int HT = 256;      // rows per workgroup
constexpr int HQ = HT - 6;   // outputs per workgroup
typedef float f2 __attribute__((ext_vector_type(2)));

// weights: the packed conv buffer's column 0 (packing in misc.hip k_pack_conv; 32-channel chunks,
// 7 taps, Np = 32): bf16 [chunk][tap][Np][32] whose row 0 is column 0 with unit swizzle
// (0 >> 2) & 3 = 0 (ST_SPLIT: the hi copy, then the lo copy), or fp32 [chunk][tap][32][Np]
// WL: weight layout 0 = fp32, 1 = bf16, 2 = ST_SPLIT (bf16 hi parts, then the lo parts: hi + lo in fp32)
template <int WL, int C>
__device__ __forceinline__ float wcol0(const void* w, int tap, int ci) {
  const size_t ct = (size_t)(ci / 32) * 7 + tap;
  if constexpr (WL == 0) return reinterpret_cast<const float*>(w)[(ct * 32 + ci % 32) * 32];
  const bf16_t* wb = reinterpret_cast<const bf16_t*>(w);
  float v = (float)wb[ct * 32 * 32 + ci % 32];
  if constexpr (WL == 2) v += (float)wb[(size_t)(C / 32) * 7 * 32 * 32 + ct * 32 * 32 + ci % 32];
  return v;
}

template <typename T, int C, int WL>
__global__ void __launch_bounds__(HT) k_conv_post(const T* __restrict__ x, long long x_bs, int x_ld, int L,
                                                  const void* __restrict__ w, const float* __restrict__ bias,
                                                  const float* __restrict__ alpha, float* __restrict__ y) {
  __shared__ __attribute__((aligned(8))) float wl[7][C];  // weights [tap][channel]
  __shared__ float al[2][C];      // Snake: alpha (bf16: in revolutions), 1 / alpha
  __shared__ float z[HT * 7 + 1];
  const int tid = threadIdx.x, b = blockIdx.y;
  for (int i = tid; i < 7 * C; i += HT) wl[i / C][i % C] = wcol0<WL, C>(w, i / C, i % C);
  for (int i = tid; i < C; i += HT) {
    const float a = alpha[i];
    al[0][i] = std::is_same<T, bf16_t>::value ? a * 0.15915494309189535f : a;
    al[1][i] = 1.0f / a;
  }
  __syncthreads();
  const int q0 = blockIdx.x * HQ;          // first output of this workgroup
  const int r = q0 - 3 + tid;              // this thread's input row
  const bool in = r >= 0 && r < L;
  f2 acc[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) acc[k] = f2{0.f, 0.f};
  if (in) {
    const T* row = x + (size_t)b * x_bs + (size_t)r * x_ld;
#pragma unroll
    for (int c8 = 0; c8 < C / 8; ++c8) {
      float v[8];
      raw_to_f32(load_raw(row + 8 * c8), v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = 8 * c8 + j;
        float s;
        if constexpr (std::is_same<T, bf16_t>::value)
          s = __builtin_amdgcn_sinf(v[j] * al[0][c]);  // v_sin_f32 takes revolutions
        else
          s = sinf(v[j] * al[0][c]);
        v[j] = __builtin_fmaf(s * s, al[1][c], v[j]);
      }
#pragma unroll
      for (int k = 0; k < 7; ++k)
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const int c = 8 * c8 + j;
          acc[k] = __builtin_elementwise_fma(f2{v[j], v[j + 1]}, *reinterpret_cast<const f2*>(&wl[k][c]), acc[k]);
        }
    }
  }
  // rows outside [0, L) are the conv's zero padding: their partials stay 0
#pragma unroll
  for (int k = 0; k < 7; ++k) z[tid * 7 + k] = acc[k].x + acc[k].y;
  __syncthreads();
  if (tid < HQ) {
    const int q = q0 + tid;
    if (q < L) {
      // output q reads rows q - 3 + k = thread tid + k's row, tap k
      float o = bias ? bias[0] : 0.f;
#pragma unroll
      for (int k = 0; k < 7; ++k) o += z[(tid + k) * 7 + k];
      y[(size_t)b * L + q] = tanhf(o);
    }
  }
}

template <typename T, int C, int WL>
int launch_head(const ConvParams& p, hipStream_t s) {
  dim3 grid((p.Lq + HQ - 1) / HQ, p.B);
  hipLaunchKernelGGL((k_conv_post<T, C, WL>), grid, dim3(HT), 0, s, reinterpret_cast<const T*>(p.x), p.x_bs, p.x_ld,
                     p.Lq, p.w, p.bias, p.pro.alpha, reinterpret_cast<float*>(p.y));
  return (int)hipGetLastError();
}

}  // namespace

bool st_head_eligible(const ConvParams& p) {
  return p.N == 1 && p.Cout == 1 && p.KS == 7 && p.pad == 3 && p.dil == 1 && p.stride == 1 && p.up == 1 &&
         (p.Cin == 32 || p.Cin == 64) && p.pro.mode == PRO_SNAKE && p.y_f32 && p.y_ld == 1 && p.y_bs == p.Lq &&
         p.epi_tanh && !p.epi_lrelu && !p.epi_gelu && !p.res && !p.accb && !p.stats && p.Lin == p.Lq && p.Lout == p.Lq && p.y_row_off == 0 &&
         p.x_ld >= p.Cin && p.x_ld % 8 == 0;
}

int st_head(const ConvParams& p, int dtype, hipStream_t s) {
  if (dtype == ST_BF16) return p.Cin == 32 ? launch_head<bf16_t, 32, 1>(p, s) : launch_head<bf16_t, 64, 1>(p, s);
  if (dtype == ST_FP32) return p.Cin == 32 ? launch_head<float, 32, 0>(p, s) : launch_head<float, 64, 0>(p, s);
  if (dtype == ST_SPLIT) return p.Cin == 32 ? launch_head<float, 32, 2>(p, s) : launch_head<float, 64, 2>(p, s);
  return ST_EDTYPE;
}
