// Inference I/O kernels (gfx950), SURVEY.md §8(f) row 4: flow visualisation and file-layout packing.
//
// flow2rgb replaces optical_flow/visualization/flow2rgb.py:19-73 with its three colour maps
// (methods/baker.py:32-78 + colorwheel_baker :81-146, methods/hsv.py:8-36, methods/meister.py:30-55, and the
// shared hsv_to_rgb of visualization/utils.py:19-61). The reference runs ~25 (baker) to ~40 (hsv) ATen passes over
// the field, each re-reading and re-writing a (B, H, W)-sized tensor; here it is two passes:
//   1. flow_stats: per (batch, chunk) partial maxima of |flow| (the default max_norm, flow2rgb.py:60-62) and of the
//      raw flow values (meister's max_flow, meister.py:46) after the optional clip / y inversion.
//   2. flow2rgb:   every workgroup folds its batch's partials (L2-resident), then one thread per pixel computes
//      the colour from the clipped, inverted, normalised vector and writes (B, 3, H, W) fp32.
// Both are HBM-bound: 8 B read per pixel (pass 1) and 8 B read + 12 B written per pixel (pass 2).
//
// The arithmetic is the reference's op-for-op in fp32 (each ATen op is its own kernel there, so nothing is fused:
// this file is compiled with contraction off, see the pragma below) so that colours agree to the last 1/255 step
// except where the GPU's atan2f / sqrtf differ from the host libm by an ulp at a quantisation boundary.
//
// flow_pack replaces the host-side re-layouts of the file writers: Middlebury .flo rows are (H, W, 2) interleaved
// fp32 (io/middlebury.py:64-71), PFM rows are (H, W, 3) with a zero third channel, bottom row first
// (io/pfm.py:95-98). One launch turns the (2, H, W) planar field into the file's payload on the device, so the
// D2H copy moves exactly the bytes that go into the file.
#include "oflow_internal.h"

#pragma clang fp contract(off)

namespace oflow {
namespace {

constexpr int kStatsChunks = 128;  // partials per image (include/oflow.h OFLOW_FLOW_STATS_CHUNKS)
constexpr int kThreads = 256;
constexpr float kEps = 1e-5f;       // flow2rgb.py:10
constexpr float kPi = 3.14159265358979323846f;
constexpr float kTwoPi = 6.28318530717958647692f;

// colorwheel_baker (methods/baker.py:81-146): 55 hues in six segments RY 15, YG 6, GC 4, CB 11, BM 13, MR 6; in
// each one channel is held at 255 and one ramps by floor(255 * i / n) (up, or 255 minus it). Evaluated in
// registers (integer arithmetic, so exactly the table's integers) instead of a per-lane indexed table load.
__device__ inline void wheel_entry(int k, float& r, float& g, float& b) {
  int n, i, full, ramp, up;
  if (k < 15) { n = 15; i = k; full = 0; ramp = 1; up = 1; }
  else if (k < 21) { n = 6; i = k - 15; full = 1; ramp = 0; up = 0; }
  else if (k < 25) { n = 4; i = k - 21; full = 1; ramp = 2; up = 1; }
  else if (k < 36) { n = 11; i = k - 25; full = 2; ramp = 1; up = 0; }
  else if (k < 49) { n = 13; i = k - 36; full = 2; ramp = 0; up = 1; }
  else { n = 6; i = k - 49; full = 0; ramp = 2; up = 0; }
  const int q = (255 * i) / n;
  const float rv = (float)(up ? q : 255 - q);
  float c[3] = {0.f, 0.f, 0.f};
  c[full] = 255.f;
  c[ramp] = rv;
  r = c[0];
  g = c[1];
  b = c[2];
}

__device__ inline float clip_val(float x, float lo, float hi) {
  // torch.clip: max then min, NaN propagates
  x = x < lo ? lo : x;
  return x > hi ? hi : x;
}

// torch.remainder for a float divisor b > 0 (ATen: fmod, then shift into [0, b))
__device__ inline float rem_pos(float a, float b) {
  float m = fmodf(a, b);
  if (m != 0.f && m < 0.f) m += b;
  return m;
}

// kornia-style hsv_to_rgb (visualization/utils.py:19-61) for one pixel
__device__ inline void hsv_to_rgb(float h, float s, float v, float& r, float& g, float& b) {
  const float h6 = h * 6.f;
  const float hi = rem_pos(floorf(h6), 6.f);
  const float f = rem_pos(h6, 6.f) - hi;
  const float p = v * (1.f - s);
  const float q = v * (1.f - f * s);
  const float t = v * (1.f - (1.f - f) * s);
  switch ((int)hi) {
    case 0: r = v; g = t; b = p; break;
    case 1: r = q; g = v; b = p; break;
    case 2: r = p; g = v; b = t; break;
    case 3: r = p; g = q; b = v; break;
    case 4: r = t; g = p; b = v; break;
    default: r = v; g = p; b = q; break;
  }
}

__device__ inline float wave_max(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o, 64));
  return x;
}

// The colour of one flow vector (u, v): clip, y inversion, division by d, then the method's map. mf = meister's
// max_flow (the largest normalised flow value of the image).
__device__ inline void pixel_rgb(float x, float y, int method, int clip, float lo, float hi, int invert_y, float d,
                                 float mf, const float* sW, const float* sQ, float& r, float& g, float& bl) {
  if (clip) {
    x = clip_val(x, lo, hi);
    y = clip_val(y, lo, hi);
  }
  if (invert_y) y = -y;
  x = x / d;
  y = y / d;
  if (method == 0) {
    // methods/baker.py:54-74
    const float a = atan2f(-y, -x) / kPi;
    const float fk = (a + 1.f) / 2.f * 54.f;
    const float k0f = floorf(fk);
    int k0 = (int)k0f;
    k0 = k0 < 0 ? 0 : (k0 > 54 ? 54 : k0);  // NaN flow: the reference indexes out of range; clamp instead
    const int k1 = k0 + 1 == 55 ? 0 : k0 + 1;
    const float f = fk - k0f;
    const float rad = sqrtf(x * x + y * y);
    float c[3];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      // sW = colorwheel / 255 and sQ[n] = n / 255, both correctly rounded fp32 quotients (the reference's divisions)
      const float c0 = sW[k0 * 3 + ch], c1 = sW[k1 * 3 + ch];
      float col = (1.f - f) * c0 + f * c1;
      col = rad <= 1.f ? 1.f - rad * (1.f - col) : col * 0.75f;
      const float n = floorf(255.f * col);
      c[ch] = n >= 0.f && n <= 255.f ? sQ[(int)n] : n / 255.f;
    }
    r = c[0];
    g = c[1];
    bl = c[2];
  } else if (method == 1) {
    // methods/hsv.py:21-35 (the method flips y itself)
    const float dx = x, dy = -y;
    float angle = atan2f(dy, dx);
    angle = angle < 0.f ? angle + kTwoPi : angle;
    const float sc = sqrtf(dx * dx + dy * dy);
    const float s = clip_val(sc, 0.f, 1.f);
    hsv_to_rgb(angle / kTwoPi, s, 1.f, r, g, bl);
  } else {
    // methods/meister.py:43-54
    const float mag = sqrtf(x * x + y * y);
    const float angle = atan2f(y, x);
    const float h = rem_pos(angle / kTwoPi + 1.f, 1.f);
    const float s = clip_val(mag * 8.f / mf, 0.f, 1.f);
    const float v = clip_val(8.f - s, 0.f, 1.f);
    hsv_to_rgb(h, s, v, r, g, bl);
  }
}

// grid (kStatsChunks, B); partials[b][chunk] = {max |flow|, max flow value}
__global__ __launch_bounds__(kThreads) void flow_stats_kernel(const float* __restrict__ flow, long long HW, int clip,
                                                              float lo, float hi, int invert_y, int vec4,
                                                              float* __restrict__ partials) {
  __shared__ float sN[kThreads / 64], sV[kThreads / 64];
  const int b = blockIdx.y;
  const float* u = flow + (long long)b * 2 * HW;
  const float* v = u + HW;
  float mn = 0.f, mv = -INFINITY;
  auto acc = [&](float x, float y) {
    if (clip) {
      x = clip_val(x, lo, hi);
      y = clip_val(y, lo, hi);
    }
    if (invert_y) y = -y;
    mn = fmaxf(mn, sqrtf(x * x + y * y));
    mv = fmaxf(mv, fmaxf(x, y));
  };
  // chunk = a multiple of 4 pixels so that 16-B loads stay aligned when vec4 (HW % 4 == 0)
  const long long per = ((HW + kStatsChunks - 1) / kStatsChunks + 3) & ~3LL;
  const long long p0 = (long long)blockIdx.x * per, p1 = p0 + per < HW ? p0 + per : HW;
  if (vec4) {
    for (long long p = p0 + 4 * threadIdx.x; p < p1; p += 4 * kThreads) {
      const float4 a = *reinterpret_cast<const float4*>(u + p);
      const float4 c = *reinterpret_cast<const float4*>(v + p);
      acc(a.x, c.x);
      acc(a.y, c.y);
      acc(a.z, c.z);
      acc(a.w, c.w);
    }
  } else {
    for (long long p = p0 + threadIdx.x; p < p1; p += kThreads) acc(u[p], v[p]);
  }
  mn = wave_max(mn);
  mv = wave_max(mv);
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sN[wave] = mn;
    sV[wave] = mv;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float n = sN[0], m = sV[0];
    for (int i = 1; i < kThreads / 64; ++i) {
      n = fmaxf(n, sN[i]);
      m = fmaxf(m, sV[i]);
    }
    float* o = partials + ((long long)b * kStatsChunks + blockIdx.x) * 2;
    o[0] = n;
    o[1] = m;
  }
}

// grid (ceil(HW / 1024), B), 4 pixels per thread (16-B accesses when vec4: HW % 4 == 0). method 0 = baker, 1 = hsv, 2 = meister. have_denom: denom is the caller's
// max_norm + EPS; otherwise max |flow| + EPS from the partials. Partials are always read for meister's max_flow.
__global__ __launch_bounds__(kThreads) void flow2rgb_kernel(const float* __restrict__ flow, long long HW, int method,
                                                            int clip, float lo, float hi, int invert_y, int have_denom,
                                                            float denom,
                                                            const float* __restrict__ partials, int vec4, float* __restrict__ rgb) {
  __shared__ float sD, sMax;
  __shared__ float sW[55 * 3], sQ[256];
  const int b = blockIdx.y;
  if (method == 0) {
    // baker's per-workgroup quotient tables: 421 divisions here instead of 9 per pixel
    const int t = threadIdx.x;
    sQ[t] = (float)t / 255.f;
    if (t < 55) {
      float w[3];
      wheel_entry(t, w[0], w[1], w[2]);
      sW[3 * t] = w[0] / 255.f;
      sW[3 * t + 1] = w[1] / 255.f;
      sW[3 * t + 2] = w[2] / 255.f;
    }
  }
  if (threadIdx.x < 64) {
    float n = 0.f, m = -INFINITY;
    if (partials) {
      const float* pp = partials + (long long)b * kStatsChunks * 2;
      for (int i = threadIdx.x; i < kStatsChunks; i += 64) {
        n = fmaxf(n, pp[2 * i]);
        m = fmaxf(m, pp[2 * i + 1]);
      }
      n = wave_max(n);
      m = wave_max(m);
    }
    if (threadIdx.x == 0) {
      const float d = have_denom ? denom : n + kEps;  // flow / (max_norm + EPS), flow2rgb.py:63
      sD = d;
      sMax = m / d;  // max(flow / d) == max(flow) / d: division by d > 0 is monotone
    }
  }
  __syncthreads();
  const float d = sD, mf = sMax;
  const float* fu = flow + (long long)b * 2 * HW;
  float* o = rgb + (long long)b * 3 * HW;
  const long long p0 = ((long long)blockIdx.x * kThreads + threadIdx.x) * 4;
  if (p0 >= HW) return;
  if (vec4 && p0 + 4 <= HW) {
    // 4 consecutive pixels: 16-B loads of u and v, 16-B stores of each colour plane
    const float4 u4 = *reinterpret_cast<const float4*>(fu + p0);
    const float4 v4 = *reinterpret_cast<const float4*>(fu + HW + p0);
    const float us[4] = {u4.x, u4.y, u4.z, u4.w}, vs[4] = {v4.x, v4.y, v4.z, v4.w};
    float r[4], g[4], bl[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) pixel_rgb(us[k], vs[k], method, clip, lo, hi, invert_y, d, mf, sW, sQ, r[k], g[k], bl[k]);
    *reinterpret_cast<float4*>(o + p0) = make_float4(r[0], r[1], r[2], r[3]);
    *reinterpret_cast<float4*>(o + HW + p0) = make_float4(g[0], g[1], g[2], g[3]);
    *reinterpret_cast<float4*>(o + 2 * HW + p0) = make_float4(bl[0], bl[1], bl[2], bl[3]);
  } else {
    for (long long p = p0; p < p0 + 4 && p < HW; ++p) {
      float r, g, bl;
      pixel_rgb(fu[p], fu[HW + p], method, clip, lo, hi, invert_y, d, mf, sW, sQ, r, g, bl);
      o[p] = r;
      o[HW + p] = g;
      o[2 * HW + p] = bl;
    }
  }
}

// grid (ceil(W / 256), H, B): planar (B, 2, H, W) -> per image (H, W, C) rows, C = 2 (.flo) or 3 (PFM: zero third
// channel, rows bottom-up when flip)
__global__ __launch_bounds__(kThreads) void flow_pack_kernel(const float* __restrict__ flow, int H, int W, int C,
                                                             int flip, float* __restrict__ out) {
  const int x = blockIdx.x * kThreads + threadIdx.x;
  const int y = blockIdx.y, b = blockIdx.z;
  if (x >= W) return;
  const long long HW = (long long)H * W;
  const float* fu = flow + (long long)b * 2 * HW + (long long)y * W + x;
  const int yo = flip ? H - 1 - y : y;
  float* o = out + (long long)b * C * HW + ((long long)yo * W + x) * C;
  if (C == 2) {
    *reinterpret_cast<float2*>(o) = make_float2(fu[0], fu[HW]);
  } else {
    o[0] = fu[0];
    o[1] = fu[HW];
    o[2] = 0.f;
  }
}

}  // namespace
}  // namespace oflow

using namespace oflow;

extern "C" int oflow_flow_stats_f32(const float* d_flow, int B, int H, int W, int clip, float clip_lo, float clip_hi,
                                    int invert_y, float* d_partials, void* stream) {
  if (!d_flow || !d_partials) return OFLOW_E_NULL;
  if (B <= 0 || H <= 0 || W <= 0 || B > 65535) return OFLOW_E_SHAPE;
  hipLaunchKernelGGL(flow_stats_kernel, dim3(kStatsChunks, B), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                     d_flow, (long long)H * W, clip, clip_lo, clip_hi, invert_y,
                     (int)(((long long)H * W) % 4 == 0 && reinterpret_cast<uintptr_t>(d_flow) % 16 == 0), d_partials);
  return launch_status();
}

extern "C" int oflow_flow2rgb_f32(const float* d_flow, int B, int H, int W, int method, int clip, float clip_lo,
                                  float clip_hi, int invert_y, int have_denom, float denom, const float* d_partials,
                                  float* d_rgb, void* stream) {
  if (!d_flow || !d_rgb) return OFLOW_E_NULL;
  if (B <= 0 || H <= 0 || W <= 0 || B > 65535) return OFLOW_E_SHAPE;
  if (method < 0 || method > 2) return OFLOW_E_MODE;
  if ((method == 2 || !have_denom) && !d_partials) return OFLOW_E_NULL;
  const long long HW = (long long)H * W;
  const long long blocks = (HW + 4 * kThreads - 1) / (4 * kThreads);
  const int vec4 = (HW % 4 == 0) && (reinterpret_cast<uintptr_t>(d_flow) % 16 == 0) &&
                   (reinterpret_cast<uintptr_t>(d_rgb) % 16 == 0);
  if (blocks > 0x7fffffffLL) return OFLOW_E_SHAPE;
  hipLaunchKernelGGL(flow2rgb_kernel, dim3((unsigned)blocks, B), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                     d_flow, HW, method, clip, clip_lo, clip_hi, invert_y, have_denom, denom, d_partials, vec4,
                     d_rgb);
  return launch_status();
}

extern "C" int oflow_flow_pack_f32(const float* d_flow, int B, int H, int W, int channels, int flip_rows, float* d_out,
                                   void* stream) {
  if (!d_flow || !d_out) return OFLOW_E_NULL;
  if (B <= 0 || H <= 0 || W <= 0 || B > 65535 || H > 65535) return OFLOW_E_SHAPE;
  if (channels != 2 && channels != 3) return OFLOW_E_MODE;
  hipLaunchKernelGGL(flow_pack_kernel, dim3((W + kThreads - 1) / kThreads, H, B), dim3(kThreads), 0,
                     static_cast<hipStream_t>(stream), d_flow, H, W, channels, flip_rows, d_out);
  return launch_status();
}
