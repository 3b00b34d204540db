// Producers of the S32 split-fp16 activation format (conv_s32.hip) around the RAFT update loop (gfx950).
//
//   oflow_pack_s32_f32  : NCHW fp32 -> act -> S32 slice(s) (+ optional NHWC fp32 copy). Feeds the context
//                         features into the GRU buffers: net = tanh(cnet[:, :hdim]), inp = relu(cnet[:, hdim:])
//                         (methods/raft/model/raft.py:115-118).
//   oflow_flow_prep_s32 : flow = coords1 - coords0 (raft.py:129; coords0 is the pixel grid, exact) written as
//                         (a) the two flow channels of the GRU input buffers (update.py:127-128: cat([out, flow]))
//                         and (b) the 7x7 patch matrix of convf1 (update.py:116), channel t*2 + c = flow channel c
//                         at tap t = ky*7 + kx, zero padded (so convf1 runs as a 1x1 split-fp16 GEMM, K = 98 -> 128).
#include "oflow_internal.h"

namespace oflow {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float act_fn(float v, int act) {
  if (act == 1) return v < 0.f ? 0.f : v;
  if (act == 2) return 1.0f / (1.0f + expf(-v));
  if (act == 3) return tanhf(v);
  return v;
}

__device__ __forceinline__ void put8(uint8_t* line, const float* v) {
  half8 hi, lo;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    _Float16 h_, l_;
    split_f16(v[j], h_, l_);
    hi[j] = h_;
    lo[j] = l_;
  }
  *reinterpret_cast<half8*>(line) = hi;
  *reinterpret_cast<half8*>(line + 64) = lo;
}

// one thread = one pixel x 8 channels; consecutive threads = consecutive pixels (coalesced NCHW reads). Source channel
// c goes to destination channel yc0 + c (yc0 % 8 == 0); the chunk's channels beyond C are written as zeros.
__global__ __launch_bounds__(256) void pack_s32_kernel(const float* __restrict__ x, long long xbs, int C, int B, int HW,
                                                       int act, int yc0, uint8_t* y0, long long y0ps, uint8_t* y1,
                                                       long long y1ps, float* f, int fcs) {
  const long long P = (long long)B * HW;
  const int C8 = (C + 7) / 8;
  const long long item = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= P * C8) return;
  const int c8 = static_cast<int>(item / P);
  const long long p = item - (long long)c8 * P;
  const int b = static_cast<int>(p / HW);
  const int pix = static_cast<int>(p - (long long)b * HW);
  const int c0 = c8 * 8;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = c0 + j;
    v[j] = c < C ? act_fn(x[b * xbs + (long long)c * HW + pix], act) : 0.f;
  }
  const int cd = yc0 + c0;  // destination channel (multiple of 8)
  const long long off = (long long)(cd >> 5) * 128 + ((cd & 31) >> 3) * 16;
  put8(y0 + p * y0ps + off, v);
  if (y1) put8(y1 + p * y1ps + off, v);
  if (f) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (c0 + j < C) f[p * fcs + c0 + j] = v[j];
  }
}

// one thread = one pixel x one 32-channel group of the 7x7 patch matrix (4 groups: 98 channels + 30 zeros);
// group 0 also writes the flow channels of the GRU inputs.
__global__ __launch_bounds__(256) void flow_prep_kernel(const float* __restrict__ coords, int B, int H, int W,
                                                        uint8_t* pm, uint8_t* d0, long long d0ps, uint8_t* d1,
                                                        long long d1ps) {
  constexpr int KS = 7, R = 3, G = 4;
  const long long HW = (long long)H * W;
  const long long P = B * HW;
  const long long item = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= P * G) return;
  const int g = static_cast<int>(item % G);
  const long long p = item / G;
  const int b = static_cast<int>(p / HW);
  const int pix = static_cast<int>(p - b * HW);
  const int y = pix / W, x = pix - y * W;
  const float* cx = coords + (long long)b * 2 * HW;
  const float* cy = cx + HW;
  float v[32];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int t = g * 16 + k;
    float fx = 0.f, fy = 0.f;
    if (t < KS * KS) {
      const int yy = y + t / KS - R, xx = x + t % KS - R;
      if (static_cast<unsigned>(yy) < static_cast<unsigned>(H) && static_cast<unsigned>(xx) < static_cast<unsigned>(W)) {
        const long long q = (long long)yy * W + xx;
        fx = cx[q] - static_cast<float>(xx);
        fy = cy[q] - static_cast<float>(yy);
      }
    }
    v[2 * k] = fx;
    v[2 * k + 1] = fy;
  }
  uint8_t* line = pm + (p * G + g) * 128;
#pragma unroll
  for (int c = 0; c < 4; ++c) put8(line + c * 16, v + 8 * c);
  if (g == 0 && d0) {
    const float fx = cx[pix] - static_cast<float>(x), fy = cy[pix] - static_cast<float>(y);
    _Float16 hx, lx, hy, ly;
    split_f16(fx, hx, lx);
    split_f16(fy, hy, ly);
    for (int d = 0; d < 2; ++d) {
      uint8_t* dst = d == 0 ? d0 + p * d0ps : (d1 ? d1 + p * d1ps : nullptr);
      if (!dst) continue;
      _Float16* h = reinterpret_cast<_Float16*>(dst);
      h[0] = hx;
      h[1] = hy;
      h[32] = lx;
      h[33] = ly;
    }
  }
}

}  // namespace
}  // namespace oflow

using namespace oflow;

extern "C" int oflow_pack_s32_f32(const float* d_x, long long x_batch_stride, int C, int B, int H, int W, int activation,
                                  int dst_channel, void* d_y0, long long y0_pixel_stride, void* d_y1,
                                  long long y1_pixel_stride, float* d_nhwc, int nhwc_pixel_stride, void* stream) {
  if (!d_x || !d_y0) return OFLOW_E_NULL;
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || dst_channel < 0 || (dst_channel & 7)) return OFLOW_E_SHAPE;
  if (activation < 0 || activation > 3) return OFLOW_E_MODE;
  if ((y0_pixel_stride & 127) || ((uintptr_t)d_y0 & 15) || (d_y1 && ((y1_pixel_stride & 127) || ((uintptr_t)d_y1 & 15))))
    return OFLOW_E_ALIGN;
  const long long items = (long long)B * H * W * ((C + 7) / 8);
  hipLaunchKernelGGL(pack_s32_kernel, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     d_x, x_batch_stride, C, B, H * W, activation, dst_channel, static_cast<uint8_t*>(d_y0), y0_pixel_stride,
                     static_cast<uint8_t*>(d_y1), y1_pixel_stride, d_nhwc, nhwc_pixel_stride);
  return launch_status();
}

extern "C" int oflow_flow_prep_s32(const float* d_coords, int B, int H, int W, void* d_patches, void* d_flow0,
                                   long long flow0_pixel_stride, void* d_flow1, long long flow1_pixel_stride,
                                   void* stream) {
  if (!d_coords || !d_patches) return OFLOW_E_NULL;
  if (B <= 0 || H <= 0 || W <= 0) return OFLOW_E_SHAPE;
  if (((uintptr_t)d_patches & 15) || (d_flow0 && ((uintptr_t)d_flow0 & 3)) || (d_flow1 && ((uintptr_t)d_flow1 & 3)))
    return OFLOW_E_ALIGN;
  const long long items = (long long)B * H * W * 4;
  hipLaunchKernelGGL(flow_prep_kernel, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     d_coords, B, H, W, static_cast<uint8_t*>(d_patches), static_cast<uint8_t*>(d_flow0),
                     flow0_pixel_stride, static_cast<uint8_t*>(d_flow1), flow1_pixel_stride);
  return launch_status();
}
