// Backward of the flow warp / grid_sample (gfx950).
//
// Replaces the autograd of optical_flow/operator/operator.py:30-33 (`F.grid_sample(frame, warp_grid(flow), ...)`, whose
// grid = linspace base + flow, operator.py:36-56) and of the explicit-grid `bilinear_sampler` path: given dL/dout
// (B, C, Ho, Wo) it forms dL/dframe (B, C, H, W) and dL/dflow (B, 2, Ho, Wo) (warp) or dL/dgrid (B, Ho, Wo, 2)
// (grid_sample), for every interpolation mode (bilinear, nearest, bicubic A = -0.75) and padding mode (zeros, border,
// reflection), align_corners either way -- the formulas of ATen's grid_sampler_2d_backward:
//   * source coordinate = padding(unnormalize(g)), with the chain-rule multiplier of each step (unnormalize: (n-1)/2 or
//     n/2; border clip: 0 outside [0, n-1]; reflection: +-1 by the fold), the coordinate itself computed exactly as the
//     forward kernel (grid_warp.hip) computes it;
//   * dL/dframe: every tap's weight x dL/dout added to its source pixel. One thread per output pixel adds its taps with
//     no-return fp32 atomics (the scatter of a data-dependent map; several output pixels can share a source pixel);
//   * dL/dgrid: sum over channels of dL/dout x (d out / d coordinate), i.e. the taps' values times the weights'
//     derivatives, times the multiplier.
// One thread per output pixel: the flow / grid read and the dL/dflow write are coalesced along W, the channel loop reads
// dL/dout planes coalesced, the tap reads and atomics follow the flow.
#include <algorithm>

#include "oflow_internal.h"

namespace oflow {
namespace {

struct WarpBwdArgs {
  const float* gout;   // (B, C, Ho, Wo)
  const float* frame;  // (B, C, H, W)
  const float* flow;   // FLOW: (B, 2, Ho, Wo) normalized flow; else the grid (B, Ho, Wo, 2)
  float* gframe;       // (B, C, H, W), zero-filled by the caller; null: not wanted
  float* gflow;        // FLOW: (B, 2, Ho, Wo); else (B, Ho, Wo, 2); null: not wanted
  int B, C, H, W, Ho, Wo;
  int pad, ac;
};

__device__ __forceinline__ float linspace_m1_p1(int i, int n) {  // torch.linspace(-1, 1, n)[i] (grid_warp.hip)
  if (n == 1) return -1.0f;
  const float step = 2.0f / static_cast<float>(n - 1);
  return i < n / 2 ? fmaf(step, static_cast<float>(i), -1.0f) : fmaf(-step, static_cast<float>(n - 1 - i), 1.0f);
}

// source coordinate of a normalized grid value and d(coordinate)/d(grid) (ATen grid_sampler_compute_source_index_
// set_grad), the coordinate in the forward kernel's arithmetic
__device__ __forceinline__ float source_index_set_grad(float g, int n, int pad, int ac, float& mult) {
  float x;
  if (ac) {
    mult = static_cast<float>(n - 1) / 2.0f;
    x = (g + 1.0f) * (static_cast<float>(n - 1) / 2.0f);
  } else {
    mult = static_cast<float>(n) / 2.0f;
    x = fmaf(g + 1.0f, static_cast<float>(n) / 2.0f, -0.5f);
  }
  if (pad == OFLOW_PAD_REFLECTION) {
    float s = 1.0f;
    if (ac) {
      if (n <= 1) {
        x = 0.0f;
        s = 0.0f;
      } else {
        const float ts = static_cast<float>(2 * (n - 1));
        const float a = fabsf(x);
        const float extra = fmaf(-truncf(a / ts), ts, a);
        s = (x < 0.0f ? -1.0f : 1.0f) * (extra <= ts - extra ? 1.0f : -1.0f);
        x = fminf(extra, ts - extra);
      }
    } else {
      const float ts = static_cast<float>(2 * n);
      const float a = fabsf(x + 0.5f);
      const float extra = fmaf(-truncf(a / ts), ts, a);
      s = (x + 0.5f < 0.0f ? -1.0f : 1.0f) * (extra <= ts - extra ? 1.0f : -1.0f);
      x = fminf(extra, ts - extra) - 0.5f;
    }
    mult *= s;
  }
  if (pad == OFLOW_PAD_BORDER || pad == OFLOW_PAD_REFLECTION) {  // clip_coordinates_set_grad
    const float hi = static_cast<float>(n - 1);
    if (x <= 0.0f) {
      x = 0.0f;
      mult = 0.0f;
    } else if (x >= hi) {
      x = hi;
      mult = 0.0f;
    }
  }
  return x;
}

__device__ __forceinline__ int to_index(float x) {
  return (x > -1048576.0f && x < 1048576.0f) ? static_cast<int>(x) : -1048576;
}

__device__ __forceinline__ bool inb(int x, int y, int W, int H) {
  return static_cast<unsigned>(x) < static_cast<unsigned>(W) && static_cast<unsigned>(y) < static_cast<unsigned>(H);
}

// padding of one bicubic tap coordinate, given as the float ATen forms (ix_nw - 1 + k; add_value_bounded /
// get_value_bounded pad the float, then cast): returns the in-range index or -1 (zeros padding, outside). Far-out
// coordinates (|x| >= 2^20) still land on the border / reflected pixel under border and reflection padding, as in the
// forward (grid_warp.hip)
__device__ __forceinline__ int tap_index(float x, int n, int pad, int ac) {
  if (pad == OFLOW_PAD_ZEROS) {
    const int i = to_index(x);
    return (static_cast<unsigned>(i) < static_cast<unsigned>(n)) ? i : -1;
  }
  if (pad == OFLOW_PAD_REFLECTION) {
    if (ac) {
      if (n <= 1) return 0;
      const float ts = static_cast<float>(2 * (n - 1));
      const float a = fabsf(x);
      const float extra = fmaf(-truncf(a / ts), ts, a);
      x = fminf(extra, ts - extra);
    } else {
      const float ts = static_cast<float>(2 * n);
      const float a = fabsf(x + 0.5f);
      const float extra = fmaf(-truncf(a / ts), ts, a);
      x = fminf(extra, ts - extra) - 0.5f;
    }
  }
  x = fminf(static_cast<float>(n - 1), fmaxf(x, 0.0f));
  return static_cast<int>(x);
}

__device__ __forceinline__ void cubic_coeffs(float t, float c[4]) {
  const float A = -0.75f;
  float x = t + 1.0f;
  c[0] = ((A * x - 5.0f * A) * x + 8.0f * A) * x - 4.0f * A;
  x = t;
  c[1] = ((A + 2.0f) * x - (A + 3.0f)) * x * x + 1.0f;
  x = 1.0f - t;
  c[2] = ((A + 2.0f) * x - (A + 3.0f)) * x * x + 1.0f;
  x = 2.0f - t;
  c[3] = ((A * x - 5.0f * A) * x + 8.0f * A) * x - 4.0f * A;
}

// d(coefficient)/dt (ATen get_cubic_coefficients_grad)
__device__ __forceinline__ void cubic_coeffs_grad(float t, float c[4]) {
  const float A = -0.75f;
  float x = -1.0f - t;
  c[0] = (-3.0f * A * x - 10.0f * A) * x - 8.0f * A;
  x = -t;
  c[1] = (-3.0f * (A + 2.0f) * x - 2.0f * (A + 3.0f)) * x;
  x = 1.0f - t;
  c[2] = (3.0f * (A + 2.0f) * x - 2.0f * (A + 3.0f)) * x;
  x = 2.0f - t;
  c[3] = (3.0f * A * x - 10.0f * A) * x + 8.0f * A;
}

template <int MODE, bool FLOW>
__global__ __launch_bounds__(256) void warp_backward_kernel(WarpBwdArgs a) {
  const long long HW = (long long)a.H * a.W, HWo = (long long)a.Ho * a.Wo;
  const long long total = (long long)a.B * HWo;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const int b = static_cast<int>(t / HWo);
    const int pix = static_cast<int>(t - (long long)b * HWo);
    float gx, gy;
    if constexpr (FLOW) {
      const int y = pix / a.Wo, x = pix - y * a.Wo;
      gx = linspace_m1_p1(x, a.Wo) + a.flow[(size_t)(2 * b) * HWo + pix];
      gy = linspace_m1_p1(y, a.Ho) + a.flow[(size_t)(2 * b + 1) * HWo + pix];
    } else {
      const float2 g = *reinterpret_cast<const float2*>(a.flow + 2 * ((size_t)b * HWo + pix));
      gx = g.x;
      gy = g.y;
    }
    const float* go = a.gout + (size_t)b * a.C * HWo + pix;
    const float* src = a.frame + (size_t)b * a.C * HW;
    float* gin = a.gframe ? a.gframe + (size_t)b * a.C * HW : nullptr;
    float gix = 0.0f, giy = 0.0f, mx = 0.0f, my = 0.0f;
    if constexpr (MODE == OFLOW_INTERP_BILINEAR) {
      const float ix = source_index_set_grad(gx, a.W, a.pad, a.ac, mx);
      const float iy = source_index_set_grad(gy, a.H, a.pad, a.ac, my);
      const float fx = floorf(ix), fy = floorf(iy);
      const int x0 = to_index(fx), y0 = to_index(fy);
      const float e = fx + 1.0f - ix, w = ix - fx, s = fy + 1.0f - iy, n = iy - fy;  // ix_se - ix, ix - ix_nw, ...
      const float nw = e * s, ne = w * s, sw = e * n, se = w * n;
      const bool bnw = inb(x0, y0, a.W, a.H), bne = inb(x0 + 1, y0, a.W, a.H);
      const bool bsw = inb(x0, y0 + 1, a.W, a.H), bse = inb(x0 + 1, y0 + 1, a.W, a.H);
      const long long o = (long long)y0 * a.W + x0;
      for (int c = 0; c < a.C; ++c) {
        const float g = go[(size_t)c * HWo];
        const float* sc = src + (size_t)c * HW;
        if (bnw) {
          if (gin) atomicAdd(gin + (size_t)c * HW + o, nw * g);
          const float v = sc[o];
          gix -= v * s * g;
          giy -= v * e * g;
        }
        if (bne) {
          if (gin) atomicAdd(gin + (size_t)c * HW + o + 1, ne * g);
          const float v = sc[o + 1];
          gix += v * s * g;
          giy -= v * w * g;
        }
        if (bsw) {
          if (gin) atomicAdd(gin + (size_t)c * HW + o + a.W, sw * g);
          const float v = sc[o + a.W];
          gix -= v * n * g;
          giy += v * e * g;
        }
        if (bse) {
          if (gin) atomicAdd(gin + (size_t)c * HW + o + a.W + 1, se * g);
          const float v = sc[o + a.W + 1];
          gix += v * n * g;
          giy += v * w * g;
        }
      }
    } else if constexpr (MODE == OFLOW_INTERP_NEAREST) {
      const float ix = source_index_set_grad(gx, a.W, a.pad, a.ac, mx);
      const float iy = source_index_set_grad(gy, a.H, a.pad, a.ac, my);
      const int xn = to_index(rintf(ix)), yn = to_index(rintf(iy));
      if (gin && inb(xn, yn, a.W, a.H)) {
        const long long o = (long long)yn * a.W + xn;
        for (int c = 0; c < a.C; ++c) atomicAdd(gin + (size_t)c * HW + o, go[(size_t)c * HWo]);
      }
      mx = my = 0.0f;  // nearest: no gradient w.r.t. the grid
    } else {  // bicubic: the coordinate is unnormalized only; padding applies to each tap (ATen)
      float ix, iy;
      if (a.ac) {
        mx = static_cast<float>(a.W - 1) / 2.0f;
        my = static_cast<float>(a.H - 1) / 2.0f;
        ix = (gx + 1.0f) * mx;
        iy = (gy + 1.0f) * my;
      } else {
        mx = static_cast<float>(a.W) / 2.0f;
        my = static_cast<float>(a.H) / 2.0f;
        ix = fmaf(gx + 1.0f, mx, -0.5f);
        iy = fmaf(gy + 1.0f, my, -0.5f);
      }
      const float fx = floorf(ix), fy = floorf(iy);
      const float tx = ix - fx, ty = iy - fy;
      float cx[4], cy[4], dx[4], dy[4];
      cubic_coeffs(tx, cx);
      cubic_coeffs(ty, cy);
      cubic_coeffs_grad(tx, dx);
      cubic_coeffs_grad(ty, dy);
      int xi[4], yi[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        xi[k] = tap_index(fx - 1.0f + static_cast<float>(k), a.W, a.pad, a.ac);
        yi[k] = tap_index(fy - 1.0f + static_cast<float>(k), a.H, a.pad, a.ac);
      }
      for (int c = 0; c < a.C; ++c) {
        const float g = go[(size_t)c * HWo];
        const float* sc = src + (size_t)c * HW;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (xi[i] < 0 || yi[j] < 0) continue;
            const long long o = (long long)yi[j] * a.W + xi[i];
            if (gin) atomicAdd(gin + (size_t)c * HW + o, g * cx[i] * cy[j]);
            const float v = sc[o];
            gix -= v * dx[i] * cy[j] * g;
            giy -= v * dy[j] * cx[i] * g;
          }
        }
      }
      // (cubic_coeffs_grad is -d(coefficient)/dt, as ATen's get_cubic_coefficients_grad: hence the -=)
    }
    if (a.gflow) {
      if constexpr (FLOW) {
        a.gflow[(size_t)(2 * b) * HWo + pix] = mx * gix;
        a.gflow[(size_t)(2 * b + 1) * HWo + pix] = my * giy;
      } else {
        *reinterpret_cast<float2*>(a.gflow + 2 * ((size_t)b * HWo + pix)) = make_float2(mx * gix, my * giy);
      }
    }
  }
}

template <bool FLOW>
int launch_bwd(const WarpBwdArgs& a, int mode, hipStream_t s) {
  const long long total = (long long)a.B * a.Ho * a.Wo;
  const int blocks = static_cast<int>(std::min<long long>((total + 255) / 256, 1ll << 20));
  if (blocks <= 0) return OFLOW_OK;
  if (mode == OFLOW_INTERP_BILINEAR)
    hipLaunchKernelGGL((warp_backward_kernel<OFLOW_INTERP_BILINEAR, FLOW>), dim3(blocks), dim3(256), 0, s, a);
  else if (mode == OFLOW_INTERP_NEAREST)
    hipLaunchKernelGGL((warp_backward_kernel<OFLOW_INTERP_NEAREST, FLOW>), dim3(blocks), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((warp_backward_kernel<OFLOW_INTERP_BICUBIC, FLOW>), dim3(blocks), dim3(256), 0, s, a);
  return launch_status();
}

int check_bwd(const float* gout, const float* frame, const float* flow, int B, int C, int H, int W, int Ho, int Wo,
              int mode, int pad, int ac) {
  if (!gout || !frame || !flow) return OFLOW_E_NULL;
  if (B < 0 || C <= 0 || H <= 0 || W <= 0 || Ho < 0 || Wo < 0) return OFLOW_E_SHAPE;
  if (mode < OFLOW_INTERP_BILINEAR || mode > OFLOW_INTERP_BICUBIC) return OFLOW_E_MODE;
  if (pad < OFLOW_PAD_ZEROS || pad > OFLOW_PAD_REFLECTION || (ac != 0 && ac != 1)) return OFLOW_E_MODE;
  return OFLOW_OK;
}

}  // namespace
}  // namespace oflow

using namespace oflow;

extern "C" int oflow_grid_warp_backward_f32(const float* d_grad_out, const float* d_frame, const float* d_flow, int B,
                                            int C, int H, int W, int mode, int padding_mode, int align_corners,
                                            float* d_grad_frame, float* d_grad_flow, void* stream) {
  const int st = check_bwd(d_grad_out, d_frame, d_flow, B, C, H, W, H, W, mode, padding_mode, align_corners);
  if (st != OFLOW_OK) return st;
  WarpBwdArgs a{d_grad_out, d_frame, d_flow, d_grad_frame, d_grad_flow, B, C, H, W, H, W, padding_mode, align_corners};
  return launch_bwd<true>(a, mode, static_cast<hipStream_t>(stream));
}

extern "C" int oflow_grid_sample_backward_f32(const float* d_grad_out, const float* d_input, const float* d_grid, int B,
                                              int C, int H, int W, int Ho, int Wo, int mode, int padding_mode,
                                              int align_corners, float* d_grad_input, float* d_grad_grid, void* stream) {
  const int st = check_bwd(d_grad_out, d_input, d_grid, B, C, H, W, Ho, Wo, mode, padding_mode, align_corners);
  if (st != OFLOW_OK) return st;
  if ((uintptr_t)d_grid & 7 || (d_grad_grid && ((uintptr_t)d_grad_grid & 7))) return OFLOW_E_ALIGN;
  WarpBwdArgs a{d_grad_out, d_input, d_grid, d_grad_input, d_grad_grid, B, C, H, W, Ho, Wo, padding_mode, align_corners};
  return launch_bwd<false>(a, mode, static_cast<hipStream_t>(stream));
}
