// Inverse warp by a flow field = F.grid_sample(frame, linspace-grid + flow) (gfx950).
//
// Replaces optical_flow/operator/operator.py:8-56 (warp -> warp_grid -> grid_sample). Every arithmetic step is the
// one ATen's CPU kernels perform on the reference path, so results are bit-identical to it (pinned by
// tools/exp/gridsample_emul.py, a numpy model of those kernels that matches torch bit for bit). The CPU kernels are
// compiled with FP contraction, which fixes where the fused multiply-adds sit:
//   base grid  torch.linspace(-1, 1, n): fma(step, i, -1) below n/2, fma(-step, n-1-i, 1) from it (step = 2/(n-1))
//   unnormalize  align_corners: (g+1) * ((n-1)/2);  else fma(g+1, n/2, -0.5)
//   reflection   ATen's vectorised form: extra = fma(-trunc(|x-low|/2span), 2span, |x-low|), min(extra, 2span-extra)
//   bilinear     fma(v_se, se, fma(v_sw, sw, fma(v_ne, ne, v_nw * nw)))  with nw = (1-ty)(1-tx) ...
//   bicubic      A = -0.75 coefficients (inner polynomials fused), x-sums per padding instantiation (see row4), y-sum
//                fma(c3, r3, fma(c2, r2, fma(c1, r1, c0 r0)))
//   nearest      round half to even
// Bilinear (the default mode): warp_bilinear_lds_kernel stages each 16 x 64 output tile's source box in LDS (below).
// Other modes, and frames whose rows are not 16-B multiples: one thread per output pixel, flow read and output
// writes coalesced along W; the gathered taps of neighbouring lanes are neighbours too for smooth flow.
#include <algorithm>
#include <type_traits>

#include "oflow_internal.h"

#pragma clang fp contract(off)

namespace oflow {
namespace {

struct WarpArgs {
  const float* frame;  // (B, C, H, W)
  const float* flow;   // FLOW: (B, 2, Ho, Wo) normalized flow; else the grid (B, Ho, Wo, 2)
  float* out;          // (B, C, Ho, Wo)
  int B, C, H, W;      // input sizes
  int Ho, Wo;          // output sizes (== H, W for warp)
  int pad;
  int ac;
};

__device__ __forceinline__ float linspace_m1_p1(int i, int n) {
  if (n == 1) return -1.0f;
  const float step = 2.0f / static_cast<float>(n - 1);
  return i < n / 2 ? fmaf(step, static_cast<float>(i), -1.0f) : fmaf(-step, static_cast<float>(n - 1 - i), 1.0f);
}

__device__ __forceinline__ float unnormalize(float g, int n, int ac) {
  return ac ? (g + 1.0f) * (static_cast<float>(n - 1) / 2.0f) : fmaf(g + 1.0f, static_cast<float>(n) / 2.0f, -0.5f);
}

__device__ __forceinline__ float clip(float x, int n) { return fminf(static_cast<float>(n - 1), fmaxf(x, 0.0f)); }

// ATen's vectorised reflect_coordinates: reflection about low and low + span, span = n-1 (align_corners, low = 0)
// or n (low = -0.5)
__device__ __forceinline__ float reflect(float x, int n, int ac) {
  if (ac) {
    if (n <= 1) return 0.0f;
    const float ts = static_cast<float>(2 * (n - 1));
    const float a = fabsf(x);
    const float extra = fmaf(-truncf(a / ts), ts, a);
    return fminf(extra, ts - extra);
  }
  const float ts = static_cast<float>(2 * n);
  const float a = fabsf(x + 0.5f);
  const float extra = fmaf(-truncf(a / ts), ts, a);
  return fminf(extra, ts - extra) - 0.5f;
}

// padding applied to an unnormalized coordinate (ATen compute_coordinates)
__device__ __forceinline__ float pad_coord(float x, int n, int pad, int ac) {
  if (pad == OFLOW_PAD_BORDER) {
    x = clip(x, n);
  } else if (pad == OFLOW_PAD_REFLECTION) {
    x = reflect(x, n, ac);
    x = clip(x, n);
  }
  return x;
}

// keeps float->int conversion defined for huge / non-finite coordinates (those taps are out of bounds)
__device__ __forceinline__ int to_index(float x) {
  return (x > -1048576.0f && x < 1048576.0f) ? static_cast<int>(x) : -1048576;
}

__device__ __forceinline__ bool inb(int x, int y, int W, int H) {
  return static_cast<unsigned>(x) < static_cast<unsigned>(W) && static_cast<unsigned>(y) < static_cast<unsigned>(H);
}

__device__ __forceinline__ void cubic_coeffs(float t, float c[4]) {
  const float A = -0.75f;
  float x = t + 1.0f;
  c[0] = ((A * x - 5.0f * A) * x + 8.0f * A) * x - 4.0f * A;
  x = t;
  c[1] = fmaf(fmaf(A + 2.0f, x, -(A + 3.0f)) * x, x, 1.0f);
  x = 1.0f - t;
  c[2] = fmaf(fmaf(A + 2.0f, x, -(A + 3.0f)) * x, x, 1.0f);
  x = 2.0f - t;
  c[3] = ((A * x - 5.0f * A) * x + 8.0f * A) * x - 4.0f * A;
}

// ATen: (nw_val * nw) + (ne_val * ne) + (sw_val * sw) + (se_val * se), contracted
__device__ __forceinline__ float bilerp(const float v[4], float nw, float ne, float sw, float se) {
  return fmaf(v[3], se, fmaf(v[2], sw, fmaf(v[1], ne, v[0] * nw)));
}

template <int MODE, bool FLOW>
__global__ __launch_bounds__(256) void grid_warp_kernel(WarpArgs a) {
  const int HW = a.H * a.W;
  const int HWo = a.Ho * a.Wo;
  const long long total = (long long)a.B * HWo;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int b = static_cast<int>(t / HWo);
    const int pix = static_cast<int>(t - (long long)b * HWo);
    float gx, gy;
    if constexpr (FLOW) {  // warp_grid fused: linspace base grid + normalized flow (operator.py:49-55)
      const int y = pix / a.Wo, x = pix - y * a.Wo;
      gx = linspace_m1_p1(x, a.Wo) + a.flow[(size_t)(2 * b) * HWo + pix];
      gy = linspace_m1_p1(y, a.Ho) + a.flow[(size_t)(2 * b + 1) * HWo + pix];
    } else {
      const float2 g = *reinterpret_cast<const float2*>(a.flow + 2 * ((size_t)b * HWo + pix));
      gx = g.x;
      gy = g.y;
    }
    // restrict: frame and out never alias, so the gathers of a channel chunk can all be in flight together
    const float* __restrict__ src = a.frame + (size_t)b * a.C * HW;
    float* __restrict__ dst = a.out + (size_t)b * a.C * HWo + pix;

    if constexpr (MODE == OFLOW_INTERP_BICUBIC) {
      const float ix = unnormalize(gx, a.W, a.ac), iy = unnormalize(gy, a.H, a.ac);
      const float fx = floorf(ix), fy = floorf(iy);
      float cx[4], cy[4];
      cubic_coeffs(ix - fx, cx);
      cubic_coeffs(iy - fy, cy);
      int xi[4], yi[4];
      bool xv[4], yv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float px = pad_coord(fx - 1.0f + k, a.W, a.pad, a.ac);
        const float py = pad_coord(fy - 1.0f + k, a.H, a.pad, a.ac);
        xi[k] = to_index(px);
        yi[k] = to_index(py);
        xv[k] = static_cast<unsigned>(xi[k]) < static_cast<unsigned>(a.W);
        yv[k] = static_cast<unsigned>(yi[k]) < static_cast<unsigned>(a.H);
      }
      for (int c = 0; c < a.C; ++c) {
        const float* s = src + (size_t)c * HW;
        float acc = 0.0f;
        float rows[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = (xv[j] && yv[i]) ? s[yi[i] * a.W + xi[j]] : 0.0f;
          // the x-direction sum as ATen's instantiations evaluate it: reflection fuses the whole chain; zeros and
          // border fuse only the first product
          rows[i] = a.pad == OFLOW_PAD_REFLECTION
                        ? fmaf(cx[3], v[3], fmaf(cx[2], v[2], fmaf(cx[1], v[1], cx[0] * v[0])))
                        : (fmaf(cx[0], v[0], cx[1] * v[1]) + cx[2] * v[2]) + cx[3] * v[3];
        }
        acc = fmaf(cy[3], rows[3], fmaf(cy[2], rows[2], fmaf(cy[1], rows[1], cy[0] * rows[0])));
        dst[(size_t)c * HWo] = acc;
      }
    } else {
      const float ix = pad_coord(unnormalize(gx, a.W, a.ac), a.W, a.pad, a.ac);
      const float iy = pad_coord(unnormalize(gy, a.H, a.ac), a.H, a.pad, a.ac);
      if constexpr (MODE == OFLOW_INTERP_NEAREST) {
        const int xn = to_index(rintf(ix)), yn = to_index(rintf(iy));
        const bool ok = inb(xn, yn, a.W, a.H);
        for (int c0 = 0; c0 < a.C; c0 += 4) {
          float v[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) v[k] = (ok && c0 + k < a.C) ? src[(size_t)(c0 + k) * HW + yn * a.W + xn] : 0.0f;
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (c0 + k < a.C) dst[(size_t)(c0 + k) * HWo] = v[k];
        }
      } else {
        const float fx = floorf(ix), fy = floorf(iy);
        const int x0 = to_index(fx), y0 = to_index(fy);
        const float wx = ix - fx, wy = iy - fy;
        const float ex = 1.0f - wx, ey = 1.0f - wy;
        const float nw = ey * ex, ne = ey * wx, sw = wy * ex, se = wy * wx;
        const bool bnw = inb(x0, y0, a.W, a.H), bne = inb(x0 + 1, y0, a.W, a.H);
        const bool bsw = inb(x0, y0 + 1, a.W, a.H), bse = inb(x0 + 1, y0 + 1, a.W, a.H);
        const int o00 = y0 * a.W + x0;
        for (int c0 = 0; c0 < a.C; c0 += 4) {  // 4 channels' 16 gathers issued before any store
          float v[4][4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float* s = src + (size_t)(c0 + k) * HW;
            const bool ok = c0 + k < a.C;
            v[k][0] = (ok && bnw) ? s[o00] : 0.0f;
            v[k][1] = (ok && bne) ? s[o00 + 1] : 0.0f;
            v[k][2] = (ok && bsw) ? s[o00 + a.W] : 0.0f;
            v[k][3] = (ok && bse) ? s[o00 + a.W + 1] : 0.0f;
          }
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (c0 + k < a.C) dst[(size_t)(c0 + k) * HWo] = bilerp(v[k], nw, ne, sw, se);
        }
      }
    }
  }
}

// Bilinear fast path: one workgroup = a 16 x 64 output tile (a wave = one 64-pixel row segment, 4 rows per thread).
// The tap coordinates of the tile are computed once (registers), their bounding box is reduced over the workgroup,
// and when it fits kBoxFloats the source box of each channel is staged in LDS with coalesced row reads, so every
// bilinear tap is an LDS read instead of a scattered 128-B line fetch (flows whose taps spread wider than the
// budget take the direct-gather loop for that tile). Same arithmetic as grid_warp_kernel: bit-identical results.
constexpr int kWThreads = 256, kWWaves = kWThreads / 64;
constexpr int kWTY = 16, kWTX = 64, kWRows = kWTY / kWWaves;
constexpr int kBoxFloats = 9216;  // 36 KB (4 workgroups per CU): a 16 x 64 tile with a +-27 px margin (N(0, 8^2) px flow) fits
constexpr int kWChunks = kBoxFloats / 4 / kWThreads;  // 16-B box chunks per thread (12)

template <bool FLOW>
__global__ __launch_bounds__(kWThreads) void warp_bilinear_lds_kernel(WarpArgs a, int tiles_x, int tiles_y, int cpw) {
  __shared__ __attribute__((aligned(16))) float sBox[kBoxFloats];
  __shared__ int sRed[kWWaves][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // XCD-aware order: dispatch is round-robin over the 8 XCDs, so block ids equal mod 8 share an L2; give each XCD a
  // contiguous run of tiles, ordered column-major (ty fastest) so consecutive tiles are vertical neighbours whose
  // staged boxes overlap most (speed only; the remap is a bijection for any grid size)
  const int nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, xcd = blockIdx.x % 8;
  int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + blockIdx.x / 8;
  // channel chunks of one tile are consecutive in that order (one XCD: the flow is read from HBM once)
  const int nch = (a.C + cpw - 1) / cpw;
  const int cb = (t % nch) * cpw, ce = min(a.C, cb + cpw);
  t /= nch;
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
  const bool staged = vec4 && xmax >= xmin && (long long)bw * bh <= kBoxFloats;
  const float* __restrict__ src = a.frame + (size_t)b * a.C * HW;
  float* __restrict__ dst = a.out + (size_t)b * a.C * HWo;

  if (!staged) {
    // direct gathers, pixel-major: 4 channels' 16 taps of a pixel in flight before any store (grid_warp_kernel's loop)
    // (this workgroup's channel chunk [cb, ce))
#pragma unroll
    for (int k = 0; k < kWRows; ++k) {
      if (!((vmask >> (16 + k)) & 1u)) continue;
      const int yo = ty * kWTY + wave + kWWaves * k;
      const unsigned m = (vmask >> (4 * k)) & 15u;
      const int y0 = static_cast<int>(static_cast<short>(o00[k] & 0xffff)), x0 = o00[k] >> 16;
      const int o = y0 * a.W + x0;
      float* __restrict__ d = dst + yo * a.Wo + xo;
      for (int c0 = cb; c0 < ce; c0 += 4) {
        float v[4][4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float* sp = src + (size_t)(c0 + q) * HW + o;
          const bool ok = c0 + q < ce;
          v[q][0] = (ok && (m & 1u)) ? sp[0] : 0.0f;
          v[q][1] = (ok && (m & 2u)) ? sp[1] : 0.0f;
          v[q][2] = (ok && (m & 4u)) ? sp[a.W] : 0.0f;
          v[q][3] = (ok && (m & 8u)) ? sp[a.W + 1] : 0.0f;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (c0 + q < ce) d[(size_t)(c0 + q) * HWo] = bilerp(v[q], wnw[k], wne[k], wsw[k], wse[k]);
      }
    }
    return;
  }
  // Channel pipeline: the box of channel c + 1 is loaded into registers (16-B chunks, kWChunks per thread, all in
  // flight) while channel c is interpolated from LDS, then written over it: one L2 round trip per channel is hidden
  // behind the previous channel's taps instead of serialised with them.
  const int cw = bw >> 2, n = cw * bh, dr = kWThreads / cw, dc = kWThreads - dr * cw;
  float4 stage[kWChunks];
  // chunk j of this thread -> (box row, 16-B column), stepped incrementally from tid
  auto chunk_walk = [&](auto&& fn) {
    int r = tid / cw, col = tid - r * cw;
#pragma unroll
    for (int j = 0; j < kWChunks; ++j) {
      if (tid + kWThreads * j < n) fn(j, r, col);
      r += dr;
      col += dc;
      if (col >= cw) {
        col -= cw;
        ++r;
      }
    }
  };
  auto load_box = [&](int c) {
    const float* base = src + (size_t)c * HW + (size_t)ymin * a.W + xmin;
    chunk_walk([&](int j, int r, int col) {
      const int x = xmin + col * 4;
      const float* q = base + (size_t)r * a.W + col * 4;
      stage[j] = x + 3 < a.W ? *reinterpret_cast<const float4*>(q)  // never read past the row's end
                             : make_float4(q[0], x + 1 < a.W ? q[1] : 0.f, x + 2 < a.W ? q[2] : 0.f, 0.f);
    });
  };
  load_box(cb);
  for (int c = cb; c < ce; ++c) {
    if (c > cb) __syncthreads();  // every thread is done reading channel c-1's box
    chunk_walk([&](int j, int r, int col) { *reinterpret_cast<float4*>(&sBox[r * bw + col * 4]) = stage[j]; });
    __syncthreads();
    if (c + 1 < ce) load_box(c + 1);
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
      const float v[4] = {v0, v1, v2, v3};
      dst[(size_t)c * HWo + yo * a.Wo + xo] = bilerp(v, wnw[k], wne[k], wsw[k], wse[k]);
    }
  }
}

// Warp fast path (flow given, bilinear, C <= 3, 16-B frame rows): a workgroup walks down a 64-column strip of one
// image in 16-row steps and keeps the source rows its taps can reach in an LDS ring: rows y - kSM .. y + 16 + kSM and
// columns x0 - kSM .. x0 + 64 + kSM of every channel (kSM = 28 px: |flow| of an i.i.d. N(0, 8^2) field stays inside for
// all but ~0.1 % of pixels). Each step brings in only the 16 new rows (loaded one step ahead into registers), so every
// source byte is read ~1.9x from L2 (the strip's side margins and a segment's first rows) instead of ~8x with per-tile
// bounding boxes, and with coalesced 16-B row reads. Taps outside the ring (a larger flow) are gathered from global
// memory by that lane. Same arithmetic as grid_warp_kernel: bit-identical results.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kSThreads = 1024, kSWaves = kSThreads / 64;
constexpr int kSX = 64, kSY = 16, kSM = 28;           // strip width, rows per step, margin
constexpr int kSRows = kSY / kSWaves;                 // output rows per thread per step
constexpr int kSR = 2 * kSY + 2 * kSM;                // ring rows (88: one step of slack, see the loop)
constexpr int kSC = kSX + 2 * kSM;                    // ring columns (120 = 30 float4)
constexpr int kSC4 = kSC / 4;
constexpr int kSMaxC = 3;
constexpr int kSPre = (kSY * kSC4 * kSMaxC + kSThreads - 1) / kSThreads;  // float4 of a step's new rows per thread

// BUF (r06, the default below 2^29 frame elements): every row and flow load unconditional -- buffer loads whose offset
// is a sentinel past the frame's buffer for rows / chunks outside the image (the load returns zeros, no memory access)
// -- no branch around a step's loads (past the segment's end they fetch rows nobody reads), the flow prefetched as many
// steps ahead as the rows, and pixels whose taps leave the ring deferred to the segment's end (an LDS list), so no load
// of a step waits for the ones issued after it. The r03 form loaded under exec-masked branches, after which the
// compiler cannot count the outstanding loads and waits for all of them (s_waitcnt vmcnt(0), stores included) inside the
// step loop: the rows prefetched kSD steps ahead were waited for one step later. In-process A/B at (8, 3, 436, 1024)
// (tools/exp/run_warp_ab.py, profiles/r06/r6s16_warp_ab.log): i.i.d. N(0, 8^2) flow 33.34 -> 31.14 us, smooth 32.78 ->
// 30.90, zero 31.70 -> 29.96; bit-identical.
template <bool BUF>
__global__ __launch_bounds__(kSThreads) void warp_strip_kernel(WarpArgs a, int strips, int segs, int seg_h) {
  __shared__ __attribute__((aligned(16))) float sRing[kSMaxC * kSR * kSC];
  constexpr int kFbCap = BUF ? 1024 : 1;  // deferred out-of-ring pixels (BUF)
  __shared__ int sFb[kFbCap];
  __shared__ int sFbN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) sFbN = 0;  // (published by the first step's barrier, before any append)
  // XCD-aware order: block ids equal mod 8 share an L2; each XCD takes a contiguous run of (image, strip, segment)
  const int nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, xcd = blockIdx.x % 8;
  int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + blockIdx.x / 8;
  const int seg = t % segs;
  t /= segs;
  const int strip = t % strips;
  const int b = t / strips;
  const int C = a.C, H = a.H, W = a.W, HW = H * W;
  const int x0 = strip * kSX, xb = x0 - kSM;
  const int ys = seg * seg_h, ye = min(H, ys + seg_h);
  const float* __restrict__ src = a.frame + (size_t)b * C * HW;
  float* __restrict__ dst = a.out + (size_t)b * C * HW;
  const float* __restrict__ fxp = a.flow + (size_t)(2 * b) * HW;
  const float* __restrict__ fyp = a.flow + (size_t)(2 * b + 1) * HW;

  // one float4 of image row yy (ring slot yy mod kSR), column chunk j, channel c; rows / chunks outside the image: 0
  // (chunks are 4-float aligned and W % 4 == 0: a chunk is wholly inside or outside a row)
  const __amdgpu_buffer_rsrc_t rsF =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0, C * HW * 4, 0x00020000);
  auto fetch = [&](int c, int yy, int j) {
    const int xx = xb + 4 * j;
    const bool in = yy >= 0 && yy < H && xx >= 0 && xx < W;
    if constexpr (BUF) {
      const unsigned off = in ? static_cast<unsigned>(((c * H + yy) * W + xx) * 4) : 0x80000000u;  // sentinel: zeros
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsF, static_cast<int>(off), 0, 0);
      return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
    } else {
      if (in) return *reinterpret_cast<const float4*>(src + (size_t)c * HW + (size_t)yy * W + xx);
      return make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto put = [&](int c, int yy, int j, float4 v) {
    const int slot = static_cast<int>(static_cast<unsigned>(yy + kSR) % kSR);  // (yy >= -kSM > -kSR)
    *reinterpret_cast<float4*>(&sRing[(c * kSR + slot) * kSC + 4 * j]) = v;
  };
  // rows [y, y + kSY) of every channel: item e -> (c, row, chunk)
  const int nitems = C * kSY * kSC4;
  // a step's new rows are loaded kSD steps ahead into one of kSD register sets (static index: the step loop is
  // unrolled kSD times), so each load has kSD steps of work to land behind
  constexpr int kSD = 3;
  float4 pre[kSD][kSPre];
  auto load_rows = [&](float4 (&dst)[kSPre], int y) {
#pragma unroll
    for (int k = 0; k < kSPre; ++k) {
      const int e = BUF ? min(tid + k * kSThreads, nitems - 1) : tid + k * kSThreads;  // (BUF: past nitems unused)
      const int c = e / (kSY * kSC4), rem = e - c * (kSY * kSC4);
      const int rr = rem / kSC4, j = rem - rr * kSC4;
      if constexpr (BUF)
        dst[k] = fetch(c, y + rr, j);
      else
        dst[k] = e < nitems ? fetch(c, y + rr, j) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_rows = [&](const float4 (&v)[kSPre], int y) {
#pragma unroll
    for (int k = 0; k < kSPre; ++k) {
      const int e = tid + k * kSThreads;
      const int c = e / (kSY * kSC4), rem = e - c * (kSY * kSC4);
      const int rr = rem / kSC4, j = rem - rr * kSC4;
      if (e < nitems) put(c, y + rr, j, v[k]);
    }
  };
  // prologue: the first step's kSR rows (ys - kSM ..): every load issued before the first LDS store; then the next
  // step's new rows in registers
  {
    constexpr int R0 = kSY + 2 * kSM;  // the first step's rows
    constexpr int NP = (R0 * kSC4 * kSMaxC + kSThreads - 1) / kSThreads;
    const int ni = C * R0 * kSC4;
    float4 pv[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int e = BUF ? min(tid + k * kSThreads, ni - 1) : tid + k * kSThreads;
      const int c = e / (R0 * kSC4), rem = e - c * (R0 * kSC4);
      const int rr = rem / kSC4, j = rem - rr * kSC4;
      if constexpr (BUF)
        pv[k] = fetch(c, ys - kSM + rr, j);
      else
        pv[k] = e < ni ? fetch(c, ys - kSM + rr, j) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int e = tid + k * kSThreads;
      const int c = e / (R0 * kSC4), rem = e - c * (R0 * kSC4);
      const int rr = rem / kSC4, j = rem - rr * kSC4;
      if (e < ni) put(c, ys - kSM + rr, j, pv[k]);
    }
  }
  // new rows of steps 1 .. kSD (step k needs rows ys + k*kSY + kSM .. + kSY - 1), set k % kSD
#pragma unroll
  for (int k = 1; k <= kSD; ++k) load_rows(pre[k % kSD], ys + k * kSY + kSM);
  const int xo = x0 + lane;
  // the step's flow (wave w: rows y + w + kSWaves * h), loaded FD steps ahead into FD register sets (step k: set
  // k % FD); BUF: as far ahead as the rows (a step's flow wait then leaves the later steps' loads in flight)
  constexpr int FD = BUF ? kSD : 1;
  float fl[FD][kSRows][2];
  auto load_flow = [&](float (&f)[kSRows][2], int y) {
#pragma unroll
    for (int h = 0; h < kSRows; ++h) {
      const int yo = min(y + wave + kSWaves * h, H - 1), xc = min(xo, W - 1);
      f[h][0] = fxp[yo * W + xc];
      f[h][1] = fyp[yo * W + xc];
    }
  };
#pragma unroll
  for (int k = 0; k < FD; ++k) load_flow(fl[k], ys + k * kSY);

  // taps outside the ring: gathered from the frame (global memory)
  auto gather_global = [&](int pix, int tx0, int ty0, unsigned m, float nw, float ne, float sw, float se) {
    const int o = ty0 * W + tx0;
    for (int c = 0; c < C; ++c) {
      const float* sp = src + (size_t)c * HW + o;
      const float v[4] = {(m & 1u) ? sp[0] : 0.f, (m & 2u) ? sp[1] : 0.f, (m & 4u) ? sp[W] : 0.f,
                          (m & 8u) ? sp[W + 1] : 0.f};
      dst[(size_t)c * HW + pix] = bilerp(v, nw, ne, sw, se);
    }
  };
  // one step at row y; Q = the register set holding step y + kSY's new rows (refilled with step y + (kSD+1)*kSY's)
  // One barrier per step: the ring holds one step of slack (kSR = the 72 rows a step reads + 16), so the rows step
  // s + 1 adds (y + kSY + kSM ..) go to the slots of rows y - kSY - kSM .., which step s - 1 read last: after this
  // step's barrier they are free, and the barrier of step s + 1 publishes them.
  auto step = [&](int y, auto Qc) -> bool {
    constexpr int Q = decltype(Qc)::value;
    constexpr int F = ((Q + kSD - 1) % kSD) % FD;  // (step k of the segment: Q = (k + 1) % kSD)
    if (y >= ye) return false;
    __syncthreads();
    if (BUF || y + kSY < ye) {
      store_rows(pre[Q], y + kSY + kSM);
      load_rows(pre[Q], y + (kSD + 1) * kSY + kSM);
    }
    float cur[kSRows][2];
#pragma unroll
    for (int h = 0; h < kSRows; ++h) {
      cur[h][0] = fl[F][h][0];
      cur[h][1] = fl[F][h][1];
    }
    if (BUF || y + kSY < ye) load_flow(fl[F], y + FD * kSY);
    // ---- the step's 16 rows: wave w takes rows y + w + kSWaves * h ----
#pragma unroll
    for (int h = 0; h < kSRows; ++h) {
      const int yo = y + wave + kSWaves * h;
      if (yo < ye && xo < W) {
        const int pix = yo * W + xo;
        const float gx = linspace_m1_p1(xo, W) + cur[h][0];
        const float gy = linspace_m1_p1(yo, H) + cur[h][1];
        const float ix = pad_coord(unnormalize(gx, W, a.ac), W, a.pad, a.ac);
        const float iy = pad_coord(unnormalize(gy, H, a.ac), H, a.pad, a.ac);
        const float fx = floorf(ix), fy = floorf(iy);
        const int tx0 = to_index(fx), ty0 = to_index(fy);
        const float wx = ix - fx, wy = iy - fy;
        const float ex = 1.0f - wx, ey = 1.0f - wy;
        const float nw = ey * ex, ne = ey * wx, sw = wy * ex, se = wy * wx;
        const unsigned m = (inb(tx0, ty0, W, H) ? 1u : 0u) | (inb(tx0 + 1, ty0, W, H) ? 2u : 0u) |
                           (inb(tx0, ty0 + 1, W, H) ? 4u : 0u) | (inb(tx0 + 1, ty0 + 1, W, H) ? 8u : 0u);
        // every tap read lies in the ring: rows y - kSM .. y + kSY + kSM - 1, columns xb .. xb + kSC - 1
        const int ylo = (m & 3u) ? ty0 : ty0 + 1, yhi = (m & 12u) ? ty0 + 1 : ty0;
        const int xlo = (m & 5u) ? tx0 : tx0 + 1, xhi = (m & 10u) ? tx0 + 1 : tx0;
        const bool ring = m == 0u || (ylo >= y - kSM && yhi < y + kSY + kSM && xlo >= xb && xhi < xb + kSC);
        if (ring) {
          // every channel's taps read before any is combined (C <= kSMaxC: a static loop)
          const int s0 = ((ty0 % kSR) + kSR) % kSR, s1 = s0 + 1 == kSR ? 0 : s0 + 1;
          const int cx = tx0 - xb;
          float v[kSMaxC][4];
#pragma unroll
          for (int c = 0; c < kSMaxC; ++c) {
            const float* r0 = sRing + (c * kSR + s0) * kSC + cx;
            const float* r1 = sRing + (c * kSR + s1) * kSC + cx;
            const bool ok = c < C;
            v[c][0] = (ok && (m & 1u)) ? r0[0] : 0.f;
            v[c][1] = (ok && (m & 2u)) ? r0[1] : 0.f;
            v[c][2] = (ok && (m & 4u)) ? r1[0] : 0.f;
            v[c][3] = (ok && (m & 8u)) ? r1[1] : 0.f;
          }
#pragma unroll
          for (int c = 0; c < kSMaxC; ++c)
            if (c < C) dst[(size_t)c * HW + pix] = bilerp(v[c], nw, ne, sw, se);
        } else {
          // BUF: deferred to the end of the segment (an LDS list of pixels), so that no load of the step waits here
          // for every load issued before it (vector-memory loads retire in order); a full list gathers at once
          int slot = kFbCap;
          if constexpr (BUF) slot = atomicAdd(&sFbN, 1);
          if (slot < kFbCap)
            sFb[slot] = pix;
          else
            gather_global(pix, tx0, ty0, m, nw, ne, sw, se);
        }
      }
    }
    return true;
  };
  for (int y = ys; y < ye; y += kSD * kSY) {
    if (!step(y, std::integral_constant<int, 1>{})) break;
    if (!step(y + kSY, std::integral_constant<int, 2>{})) break;
    if (!step(y + 2 * kSY, std::integral_constant<int, 0>{})) break;
  }
  if constexpr (BUF) {
    // the deferred pixels: the step's arithmetic from their flow again, taps gathered from the frame
    __syncthreads();
    const int n = min(sFbN, kFbCap);
    for (int i = tid; i < n; i += kSThreads) {
      const int pix = sFb[i], yo = pix / W, xo2 = pix - yo * W;
      const float gx = linspace_m1_p1(xo2, W) + fxp[pix];
      const float gy = linspace_m1_p1(yo, H) + fyp[pix];
      const float ix = pad_coord(unnormalize(gx, W, a.ac), W, a.pad, a.ac);
      const float iy = pad_coord(unnormalize(gy, H, a.ac), H, a.pad, a.ac);
      const float fx = floorf(ix), fy = floorf(iy);
      const int tx0 = to_index(fx), ty0 = to_index(fy);
      const float wx = ix - fx, wy = iy - fy;
      const float ex = 1.0f - wx, ey = 1.0f - wy;
      const unsigned m = (inb(tx0, ty0, W, H) ? 1u : 0u) | (inb(tx0 + 1, ty0, W, H) ? 2u : 0u) |
                         (inb(tx0, ty0 + 1, W, H) ? 4u : 0u) | (inb(tx0 + 1, ty0 + 1, W, H) ? 8u : 0u);
      gather_global(pix, tx0, ty0, m, ey * ex, ey * wx, wy * ex, wy * wx);
    }
  }
}

}  // namespace
}  // namespace oflow

using namespace oflow;

namespace {
int g_warp_cpw = 0;  // channels per staged-tile workgroup (0: all; experiment hook oflow_exp_set_warp_cpw)
int g_warp_strip = 1;  // warp (flow given) on the strip-walking kernel (0: the per-tile boxes; oflow_exp_set_warp_strip)

template <bool FLOW>
int launch_warp(const WarpArgs& a, int mode, hipStream_t s) {
  const long long total = (long long)a.B * a.Ho * a.Wo;
  const long long want = (total + 255) / 256;
  dim3 grid(static_cast<unsigned>(want < 65535 ? want : 65535));
  switch (mode) {
    case OFLOW_INTERP_BILINEAR: {
      // LDS-staged tiles need 16-B frame rows for the box staging and H, W < 32768 for the packed tap coordinates
      const int tiles_x = (a.Wo + kWTX - 1) / kWTX, tiles_y = (a.Ho + kWTY - 1) / kWTY;
      const int cpw = g_warp_cpw > 0 ? std::min(g_warp_cpw, a.C) : a.C;
      const long long nb = (long long)a.B * tiles_x * tiles_y * ((a.C + cpw - 1) / cpw);
      if (FLOW && g_warp_strip && a.C <= kSMaxC && (a.W & 3) == 0 && (reinterpret_cast<uintptr_t>(a.frame) & 15) == 0 &&
          a.W >= kSX && a.H >= 2 * kSY && a.W < 32768 && a.H < 32768) {
        // strip walk: one round of at most one workgroup per CU (256 CUs; 135 KB of LDS each), segments >= 8 steps
        const int strips = (a.W + kSX - 1) / kSX;
        const long long cols = (long long)a.B * strips;
        int segs = static_cast<int>(std::max(1ll, std::min(256 / cols, (long long)a.H / (8 * kSY))));
        const int seg_h = (((a.H + segs - 1) / segs) + kSY - 1) / kSY * kSY;
        segs = (a.H + seg_h - 1) / seg_h;
        if (cols * segs < (1ll << 31)) {
          const dim3 g(static_cast<unsigned>(cols * segs));
          if ((long long)a.C * a.H * a.W < (1ll << 29))  // (BUF: the frame's byte offsets < 2^31)
            hipLaunchKernelGGL((warp_strip_kernel<true>), g, dim3(kSThreads), 0, s, a, strips, segs, seg_h);
          else
            hipLaunchKernelGGL((warp_strip_kernel<false>), g, dim3(kSThreads), 0, s, a, strips, segs, seg_h);
          break;
        }
      }
      if ((a.W & 3) == 0 && (reinterpret_cast<uintptr_t>(a.frame) & 15) == 0 && a.W < 32768 && a.H < 32768 &&
          nb < (1ll << 31)) {
        hipLaunchKernelGGL((warp_bilinear_lds_kernel<FLOW>), dim3(static_cast<unsigned>(nb)), dim3(kWThreads), 0, s, a,
                           tiles_x, tiles_y, cpw);
      } else {
        hipLaunchKernelGGL((grid_warp_kernel<OFLOW_INTERP_BILINEAR, FLOW>), grid, dim3(256), 0, s, a);
      }
      break;
    }
    case OFLOW_INTERP_NEAREST:
      hipLaunchKernelGGL((grid_warp_kernel<OFLOW_INTERP_NEAREST, FLOW>), grid, dim3(256), 0, s, a);
      break;
    case OFLOW_INTERP_BICUBIC:
      hipLaunchKernelGGL((grid_warp_kernel<OFLOW_INTERP_BICUBIC, FLOW>), grid, dim3(256), 0, s, a);
      break;
    default:
      return OFLOW_E_MODE;
  }
  return launch_status();
}
}  // namespace

extern "C" int oflow_grid_warp_f32(const float* d_frame, const float* d_flow, int B, int C, int H, int W, int mode,
                                   int padding_mode, int align_corners, float* d_out, void* stream) {
  if (!d_frame || !d_flow || !d_out) return OFLOW_E_NULL;
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0) return OFLOW_E_SHAPE;
  if ((long long)C * H * W >= (1ll << 31) || (long long)B * H * W >= (1ll << 40)) return OFLOW_E_SHAPE;
  if (padding_mode < OFLOW_PAD_ZEROS || padding_mode > OFLOW_PAD_REFLECTION) return OFLOW_E_MODE;
  WarpArgs a{d_frame, d_flow, d_out, B, C, H, W, H, W, padding_mode, align_corners ? 1 : 0};
  return launch_warp<true>(a, mode, static_cast<hipStream_t>(stream));
}

extern "C" int oflow_grid_sample_f32(const float* d_input, const float* d_grid, int B, int C, int H, int W, int Ho,
                                     int Wo, int mode, int padding_mode, int align_corners, float* d_out,
                                     void* stream) {
  if (!d_input || !d_grid || !d_out) return OFLOW_E_NULL;
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || Ho <= 0 || Wo <= 0) return OFLOW_E_SHAPE;
  if ((long long)C * H * W >= (1ll << 31) || (long long)C * Ho * Wo >= (1ll << 31)) return OFLOW_E_SHAPE;
  if ((reinterpret_cast<uintptr_t>(d_grid) & 7) != 0) return OFLOW_E_ALIGN;
  if (padding_mode < OFLOW_PAD_ZEROS || padding_mode > OFLOW_PAD_REFLECTION) return OFLOW_E_MODE;
  WarpArgs a{d_input, d_grid, d_out, B, C, H, W, Ho, Wo, padding_mode, align_corners ? 1 : 0};
  return launch_warp<false>(a, mode, static_cast<hipStream_t>(stream));
}

// experiment hook (not part of include/oflow.h): channels per LDS-staged warp workgroup (0 = all of the frame's)
extern "C" void oflow_exp_set_warp_cpw(int cpw) { g_warp_cpw = cpw; }
extern "C" void oflow_exp_set_warp_strip(int on) { g_warp_strip = on; }
