// EXPERIMENT (not product code): the product's direct-gather bilinear warp against an LDS-staged variant.
// Result (profiles/r01/exp/warp_staged_vs_direct.log, (8, 3, 436, 1024) frames): staged 54-58 us vs direct 79 us on
// the SURVEY workload (i.i.d. N(0, 8^2) px flow), but 48-50 us vs 32-44 us on zero / smooth flows (48 KB of LDS per
// 16 x 64 tile leaves 12 waves per CU for the gathers) -- not adopted; see DESIGN.md §4.
#include "../../torch-optical-flow_amd/csrc/grid_warp.hip"

namespace oflow {
namespace {
// Bilinear fast path: one workgroup = a 16 x 64 output tile (a wave = one 64-pixel row segment, 4 rows per thread).
// The tap coordinates of the tile are computed once (registers), their bounding box is reduced over the workgroup,
// and when it fits kBoxFloats the source box of each channel is staged in LDS with coalesced row reads, so every
// bilinear tap is an LDS read instead of a scattered 128-B line fetch (flows whose taps spread wider than the
// budget take the direct-gather loop for that tile). Same arithmetic as grid_warp_kernel: bit-identical results.
constexpr int kWThreads = 256, kWWaves = kWThreads / 64;
constexpr int kWTY = 16, kWTX = 64, kWRows = kWTY / kWWaves;
constexpr int kStageMin = 0;  // stage every tile whose box fits (the hybrid threshold did not pay: occupancy)
constexpr int kBoxFloats = 12288;  // 48 KB: a 16 x 64 tile with a +-32 px margin fits

template <bool FLOW>
__global__ __launch_bounds__(kWThreads) void warp_bilinear_lds_kernel(WarpArgs a, int tiles_x, int tiles_y) {
  __shared__ __attribute__((aligned(16))) float sBox[kBoxFloats];
  __shared__ int sRed[kWWaves][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // XCD-aware order: dispatch is round-robin over the 8 XCDs, so block ids equal mod 8 share an L2; give each XCD a
  // contiguous run of tiles, ordered column-major (ty fastest) so consecutive tiles are vertical neighbours whose
  // staged boxes overlap most (speed only; the remap is a bijection for any grid size)
  const int nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, xcd = blockIdx.x % 8;
  int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + blockIdx.x / 8;
  const int ty = t % tiles_y;
  t /= tiles_y;
  const int tx = t % tiles_x;
  const int b = t / tiles_x;
  const int HW = a.H * a.W, HWo = a.Ho * a.Wo;
  const int xo = tx * kWTX + lane;

  int o00[kWRows];  // (x0 << 16) | (y0 & 0xffff) of the top-left tap (x0, y0 >= -1)
  float wnw[kWRows], wne[kWRows], wsw[kWRows], wse[kWRows];
  unsigned vmask = 0u;  // 4 tap-valid bits per row + an in-tile bit (bit 16 + k)
  int xmin = 0x7fffffff, ymin = 0x7fffffff, xmax = -1, ymax = -1;
#pragma unroll
  for (int k = 0; k < kWRows; ++k) {
    const int yo = ty * kWTY + wave + kWWaves * k;
    o00[k] = 0;
    wnw[k] = wne[k] = wsw[k] = wse[k] = 0.f;
    if (xo < a.Wo && yo < a.Ho) {
      const int pix = yo * a.Wo + xo;
      float gx, gy;
      if constexpr (FLOW) {
        gx = linspace_m1_p1(xo, a.Wo) + a.flow[(size_t)(2 * b) * HWo + pix];
        gy = linspace_m1_p1(yo, a.Ho) + a.flow[(size_t)(2 * b + 1) * HWo + pix];
      } else {
        const float2 g = *reinterpret_cast<const float2*>(a.flow + 2 * ((size_t)b * HWo + pix));
        gx = g.x;
        gy = g.y;
      }
      const float ix = pad_coord(unnormalize(gx, a.W, a.ac), a.W, a.pad, a.ac);
      const float iy = pad_coord(unnormalize(gy, a.H, a.ac), a.H, a.pad, a.ac);
      const float fx = floorf(ix), fy = floorf(iy);
      const int x0 = to_index(fx), y0 = to_index(fy);
      const float wx = ix - fx, wy = iy - fy;
      const float ex = 1.0f - wx, ey = 1.0f - wy;
      wnw[k] = ey * ex;
      wne[k] = ey * wx;
      wsw[k] = wy * ex;
      wse[k] = wy * wx;
      const unsigned m = (inb(x0, y0, a.W, a.H) ? 1u : 0u) | (inb(x0 + 1, y0, a.W, a.H) ? 2u : 0u) |
                         (inb(x0, y0 + 1, a.W, a.H) ? 4u : 0u) | (inb(x0 + 1, y0 + 1, a.W, a.H) ? 8u : 0u);
      vmask |= (m << (4 * k)) | (1u << (16 + k));
      if (m) {  // bounding box of the taps actually read
        xmin = min(xmin, (m & 5u) ? x0 : x0 + 1);
        xmax = max(xmax, (m & 10u) ? x0 + 1 : x0);
        ymin = min(ymin, (m & 3u) ? y0 : y0 + 1);
        ymax = max(ymax, (m & 12u) ? y0 + 1 : y0);
        o00[k] = static_cast<int>((static_cast<unsigned>(x0) << 16) | (static_cast<unsigned>(y0) & 0xffffu));
      }
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    xmin = min(xmin, __shfl_xor(xmin, o));
    ymin = min(ymin, __shfl_xor(ymin, o));
    xmax = max(xmax, __shfl_xor(xmax, o));
    ymax = max(ymax, __shfl_xor(ymax, o));
  }
  if (lane == 0) {
    sRed[wave][0] = xmin;
    sRed[wave][1] = ymin;
    sRed[wave][2] = xmax;
    sRed[wave][3] = ymax;
  }
  __syncthreads();
  xmin = sRed[0][0];
  ymin = sRed[0][1];
  xmax = sRed[0][2];
  ymax = sRed[0][3];
#pragma unroll
  for (int w = 1; w < kWWaves; ++w) {
    xmin = min(xmin, sRed[w][0]);
    ymin = min(ymin, sRed[w][1]);
    xmax = max(xmax, sRed[w][2]);
    ymax = max(ymax, sRed[w][3]);
  }
  // 16-B staging when the frame rows are 16-B aligned: widen the box to 4-float boundaries
  const bool vec4 = (a.W & 3) == 0 && (reinterpret_cast<uintptr_t>(a.frame) & 15) == 0;
  if (vec4 && xmax >= xmin) {
    xmin &= ~3;
    xmax |= 3;
  }
  const int bw = xmax - xmin + 1, bh = ymax - ymin + 1;
  // (scalar staging would need 4x the per-thread registers: frames with W % 4 != 0 take the direct gathers)
  // Taps spread over a box under kStageMin floats (smooth flow): neighbouring lanes already share lines, direct
  // gathers are cheaper than staging (measured: tools/exp/run_warp_exp.py).
  const bool staged = vec4 && xmax >= xmin && (long long)bw * bh <= kBoxFloats && (long long)bw * bh > kStageMin;
  const float* __restrict__ src = a.frame + (size_t)b * a.C * HW;
  float* __restrict__ dst = a.out + (size_t)b * a.C * HWo;

  if (!staged) {
    // direct gathers, pixel-major: 4 channels' 16 taps of a pixel in flight before any store (grid_warp_kernel's loop)
#pragma unroll
    for (int k = 0; k < kWRows; ++k) {
      if (!((vmask >> (16 + k)) & 1u)) continue;
      const int yo = ty * kWTY + wave + kWWaves * k;
      const unsigned m = (vmask >> (4 * k)) & 15u;
      const int y0 = static_cast<int>(static_cast<short>(o00[k] & 0xffff)), x0 = o00[k] >> 16;
      const int o = y0 * a.W + x0;
      float* __restrict__ d = dst + yo * a.Wo + xo;
      for (int c0 = 0; c0 < a.C; c0 += 4) {
        float v[4][4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float* sp = src + (size_t)(c0 + q) * HW + o;
          const bool ok = c0 + q < a.C;
          v[q][0] = (ok && (m & 1u)) ? sp[0] : 0.0f;
          v[q][1] = (ok && (m & 2u)) ? sp[1] : 0.0f;
          v[q][2] = (ok && (m & 4u)) ? sp[a.W] : 0.0f;
          v[q][3] = (ok && (m & 8u)) ? sp[a.W + 1] : 0.0f;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (c0 + q < a.C) d[(size_t)(c0 + q) * HWo] = v[q][0] * wnw[k] + v[q][1] * wne[k] + v[q][2] * wsw[k] + v[q][3] * wse[k];
      }
    }
    return;
  }
  for (int c = 0; c < a.C; ++c) {
    const float* __restrict__ sc = src + (size_t)c * HW;
    {
      if (c) __syncthreads();  // every thread is done reading channel c-1's box
      // flat index over 16-B chunks of the box rows (i = tid + kWThreads j -> (row, chunk), stepped incrementally);
      // 8 chunks in flight per thread; the box starts on a 4-float boundary and rows are 16-B aligned
      const int cw = bw >> 2, n = cw * bh, dr = kWThreads / cw, dc = kWThreads - dr * cw;
      const float* base = sc + (size_t)ymin * a.W + xmin;
      int r = tid / cw, col = tid - r * cw;
      for (int i0 = tid; i0 < n; i0 += 8 * kWThreads) {
        float4 v[8];
        int off[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          off[j] = r * bw + col * 4;
          if (i0 + kWThreads * j < n) {
            const int x = xmin + col * 4;
            const float* q = base + (size_t)r * a.W + col * 4;
            v[j] = x + 3 < a.W ? *reinterpret_cast<const float4*>(q)  // never read past the row's end
                               : make_float4(q[0], x + 1 < a.W ? q[1] : 0.f, x + 2 < a.W ? q[2] : 0.f, 0.f);
          }
          r += dr;
          col += dc;
          if (col >= cw) {
            col -= cw;
            ++r;
          }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (i0 + kWThreads * j < n) *reinterpret_cast<float4*>(&sBox[off[j]]) = v[j];
      }
      __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < kWRows; ++k) {
      if (!((vmask >> (16 + k)) & 1u)) continue;
      const int yo = ty * kWTY + wave + kWWaves * k;
      const unsigned m = (vmask >> (4 * k)) & 15u;
      const int y0 = static_cast<int>(static_cast<short>(o00[k] & 0xffff)), x0 = o00[k] >> 16;
      float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
      if (m) {
        const float* p = sBox + (y0 - ymin) * bw + (x0 - xmin);
        if (m & 1u) v0 = p[0];
        if (m & 2u) v1 = p[1];
        if (m & 4u) v2 = p[bw];
        if (m & 8u) v3 = p[bw + 1];
      }
      dst[(size_t)c * HWo + yo * a.Wo + xo] = v0 * wnw[k] + v1 * wne[k] + v2 * wsw[k] + v3 * wse[k];
    }
  }
}

}  // namespace
}  // namespace oflow

extern "C" int exp_warp(int which, const float* d_frame, const float* d_flow, int B, int C, int H, int W, float* d_out,
                        void* stream) {
  oflow::WarpArgs a{d_frame, d_flow, d_out, B, C, H, W, H, W, OFLOW_PAD_BORDER, 0};
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (which == 0) {
    const long long want = ((long long)B * H * W + 255) / 256;
    hipLaunchKernelGGL((oflow::grid_warp_kernel<OFLOW_INTERP_BILINEAR, true>), dim3((unsigned)(want < 65535 ? want : 65535)),
                       dim3(256), 0, s, a);
  } else {
    const int tx = (W + oflow::kWTX - 1) / oflow::kWTX, ty = (H + oflow::kWTY - 1) / oflow::kWTY;
    hipLaunchKernelGGL((oflow::warp_bilinear_lds_kernel<true>), dim3(B * tx * ty), dim3(oflow::kWThreads), 0, s, a, tx, ty);
  }
  return hipGetLastError();
}
