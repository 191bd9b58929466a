// Traffic-counter calibration (diagnostics; VERDICT r2 item 4, MI355X_MICROARCH.md HBM section): kernels
// that read or write a KNOWN number of bytes with the access patterns of the conv engines, so that the
// rocprofv3 FETCH_SIZE / WRITE_SIZE counters can be converted to bytes for exactly those patterns
// (the guide calibrates only 16-B-per-lane coalesced streams; other widths are "uncalibrated").
//
// The buffer is a frames tensor [rows][ld] bf16 (ld = C channels).  Modes:
//   0  coalesced read: 16 B per lane, consecutive lanes consecutive 16-B units (1 KiB per wave load)
//   1  the same bytes by LDS-DMA (buffer_load ... lds, 1 KiB per wave instruction)
//   2  bigconv2's window pattern, no halo: per tile of `tile` rows and per 32-channel group, the
//      group's 64-B row segments by LDS-DMA (4 lanes per row, 16 rows per instruction), groups in
//      order inside the tile (bigconv2.hip issue_x); every byte read once
//   3  mode 2 with a halo of `halo` rows on each side (the rows bigconv2 re-reads between tiles)
//   4  coalesced write: 16 B per lane, 1 KiB per wave store
//   5  bigconv2's epilogue store pattern: per 32-channel block and 32-frame fragment, lane
//      (frame l32, half hi) stores 16 B at channels 16 hi + {0, 8} (two instructions fill a 64-B
//      row segment); every byte written once
//   6  bigconv2's residual loads: the same per-lane 16-B pieces as mode 5, loaded
//   7  the polyphase upsamplers' epilogue stores (bigconv2 UPS): mode 5's per-lane pieces at rows q up + ph, the 32
//      frames of a fragment `up` rows apart (up = the `halo` argument), one output phase ph at a time
//   8  the upsamplers' residual loads: mode 7's pieces, loaded
// Each workgroup (256 threads) walks a contiguous range of tiles; the reads are summed into one
// word per workgroup so nothing is optimised away.
#include "common.h"
#include "conv_common.h"
#include "kernels.h"

namespace {

__global__ void __launch_bounds__(256) k_calib(int mode, char* buf, long long rows, int ld, int tile, int halo,
                                              float* sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const long long row_bytes = (long long)ld * 2;
  const Rsrc r = make_rsrc(buf, (unsigned)(rows * row_bytes));
  float acc = 0.f;
  if (mode == 0 || mode == 1 || mode == 4) {
    const long long units = rows * row_bytes / 16;  // 16-B units
    const long long per = (units + gridDim.x - 1) / gridDim.x;
    const long long u0 = per * blockIdx.x, u1 = u0 + per < units ? u0 + per : units;
    for (long long u = u0 + tid; u < u1; u += 256) {
      const unsigned off = (unsigned)(u * 16);
      if (mode == 0) {
        const uint4 v = bload16(r, off);
        acc += __uint_as_float(v.x & 0x3fffffffu) * 1e-30f;
      } else if (mode == 1) {
        // one DMA per wave instruction; the wave-uniform LDS address is the wave's 1 KiB slot
        glds16(r, smem + wv * 1024, off);
      } else {
        const uint4 v = make_uint4((unsigned)u, 1u, 2u, 3u);
        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const __attribute__((ext_vector_type(4))) unsigned*>(&v),
                                               r, (int)off, 0, 0);
      }
    }
  } else if (mode == 2 || mode == 3) {
    const int hl = mode == 3 ? halo : 0;
    const int ng = ld / 32;
    const long long ntile = (rows + tile - 1) / tile;
    const long long t0 = ntile * blockIdx.x / gridDim.x, t1 = ntile * (blockIdx.x + 1) / gridDim.x;
    const int wrows = tile + 2 * hl;
    const int ninst = (wrows * 4 + 255) / 256;  // DMA instructions per wave per group (4 waves)
    for (long long t = t0; t < t1; ++t) {
      const long long gr0 = t * tile - hl;
      for (int g = 0; g < ng; ++g) {
        for (int j = 0; j < ninst; ++j) {
          const int pidx = (j * 4 + wv) * 64 + lane;
          const int rr = pidx >> 2, u = pidx & 3;
          const long long row = gr0 + rr;
          const bool in = rr < wrows && row >= 0 && row < rows;
          const unsigned off = in ? (unsigned)(row * row_bytes + g * 64 + u * 16) : OOB;
          glds16(r, smem + ((j * 4 + wv) & 7) * 1024, off);
        }
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      }
    }
  } else if (mode == 7 || mode == 8) {
    const int up = halo, ncb = ld / 32;
    const long long nq = rows / up;              // rows = nq up: q = 0 .. nq - 1, phases 0 .. up - 1
    const long long nfrag = (nq + 31) / 32;
    const long long items = nfrag * ncb * up;    // (phase, fragment, channel block)
    const long long i0 = items * (blockIdx.x * 4 + wv) / (gridDim.x * 4);
    const long long i1 = items * (blockIdx.x * 4 + wv + 1) / (gridDim.x * 4);
    const int l32 = lane & 31, hi = lane >> 5;
    for (long long it = i0; it < i1; ++it) {
      const int ph = (int)(it / (nfrag * ncb));
      const long long rem = it % (nfrag * ncb);
      const long long q = (rem / ncb) * 32 + l32;
      const int co0 = (int)(rem % ncb) * 32 + 16 * hi;
      const unsigned ey = q < nq ? (unsigned)(((q * up + ph) * ld + co0) * 2) : OOB;
      if (mode == 8) {
        const uint4 a = bload16(r, ey), b = bload16(r, ey == OOB ? OOB : ey + 16u);
        acc += __uint_as_float((a.x ^ b.y) & 0x3fffffffu) * 1e-30f;
        continue;
      }
      const uint4 v = make_uint4((unsigned)it, 1u, 2u, 3u);
      const auto vv = *reinterpret_cast<const __attribute__((ext_vector_type(4))) unsigned*>(&v);
      __builtin_amdgcn_raw_buffer_store_b128(vv, r, (int)ey, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(vv, r, (int)(ey == OOB ? OOB : ey + 16u), 0, 0);
    }
  } else if (mode == 5 || mode == 6) {
    const int ncb = ld / 32;
    const long long nfrag = (rows + 31) / 32;  // 32-frame fragments
    const long long items = nfrag * ncb;
    const long long i0 = items * (blockIdx.x * 4 + wv) / (gridDim.x * 4);
    const long long i1 = items * (blockIdx.x * 4 + wv + 1) / (gridDim.x * 4);
    const int l32 = lane & 31, hi = lane >> 5;
    for (long long it = i0; it < i1; ++it) {
      const long long q = (it / ncb) * 32 + l32;
      const int co0 = (int)(it % ncb) * 32 + 16 * hi;
      const unsigned ey = (unsigned)((q * ld + co0) * 2);
      if (mode == 6) {
        const uint4 a = bload16(r, q < rows ? ey : OOB), b = bload16(r, q < rows ? ey + 16u : OOB);
        acc += __uint_as_float((a.x ^ b.y) & 0x3fffffffu) * 1e-30f;
        continue;
      }
      const uint4 v = make_uint4((unsigned)it, 1u, 2u, 3u);
      const auto vv = *reinterpret_cast<const __attribute__((ext_vector_type(4))) unsigned*>(&v);
      __builtin_amdgcn_raw_buffer_store_b128(vv, r, (int)(q < rows ? ey : OOB), 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(vv, r, (int)(q < rows ? ey + 16u : OOB), 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  acc += __shfl_xor(acc, 1);
  if (tid == 0) sink[blockIdx.x] = acc;
}

// fixed-point statistics entry (common.h fx_add / fx_get): every part added by its own lane, then read back
__global__ void k_fx_add(int mode, const void* parts, long long n, double* entry) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    if (mode == 0) fx_add(entry, reinterpret_cast<const float*>(parts)[i]);
    else fx_add(entry, reinterpret_cast<const double*>(parts)[i]);
  }
}
__global__ void k_fx_get(const double* entry, double* out) {
  if (threadIdx.x == 0) out[0] = fx_get(entry);
}

}  // namespace

// testing hook (include/stts2.h): the total of n parts through one fixed-point entry
extern "C" int stts_test_fxsum(int mode, const void* parts, long long n, double* entry, double* out, void* stream) {
  if ((mode != 0 && mode != 1) || !parts || n <= 0 || !entry || !out) return ST_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  ST_CHECK_HIP(hipMemsetAsync(entry, 0, ST_W * sizeof(double), s));
  const long long g = (n + 255) / 256;
  hipLaunchKernelGGL(k_fx_add, dim3((unsigned)(g < 1024 ? g : 1024)), dim3(256), 0, s, mode, parts, n, entry);
  hipLaunchKernelGGL(k_fx_get, dim3(1), dim3(64), 0, s, entry, out);
  return (int)hipGetLastError();
}

extern "C" int stts_calib_traffic(int mode, void* buf, long long rows, int ld, int tile, int halo, int grid,
                                  float* sink, void* stream) {
  if (mode < 0 || mode > 8 || !buf || !sink || rows <= 0 || ld <= 0 || ld % 32 || grid <= 0) return ST_EINVAL;
  if ((mode == 7 || mode == 8) && (halo < 1 || rows % halo)) return ST_EINVAL;  // (halo = the row stride up)
  if ((mode == 2 || mode == 3) && (tile <= 0 || tile + 2 * halo > 2048)) return ST_EINVAL;
  if (rows * (long long)ld * 2 >= (long long)OOB) return ST_EINVAL;  // buffer offsets are 32-bit
  hipLaunchKernelGGL(k_calib, dim3((unsigned)grid), dim3(256), 8192, (hipStream_t)stream, mode, (char*)buf, rows, ld,
                     tile, halo, sink);
  return (int)hipGetLastError();
}
