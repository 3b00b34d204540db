// Fused elementwise stages of the RAFT update block (methods/raft/model/update.py:69-161), gfx950.
//
// The convolutions stay on MIOpen (run without bias); what PyTorch would run as separate passes around them —
// bias add, ReLU / sigmoid / tanh, r*h, the GRU blend (1-z)*h + z*q, the x0.25 mask scale and the torch.cat
// copies that rebuild [h, x] / [r*h, x] — is done here in one pass each, writing straight into persistent
// channel-concatenated buffers. Arithmetic follows the reference op by op (bias added to the conv sum, then
// the activation; blend as (1-z)*h + z*q with each product rounded), so results track it to ulp level.
//   oflow_bias_act_f32 : y[b, c, p] = act(x[b, c, p] + bias[c]) * scale, optionally to two destinations
//   oflow_gru_reset_f32: rh = sigmoid(r_pre + br) * h                (update.py:94-96 / 101-103, r and r*h)
//   oflow_gru_blend_f32: h  = (1 - z) * h + z * tanh(q_pre + bq), z = sigmoid(z_pre + bz)   (update.py:97, 104)
// Tensors are (B, C, P) slices of larger buffers: every pointer comes with its batch stride (in floats).
#include "oflow_internal.h"

#pragma clang fp contract(off)

namespace oflow {
namespace {

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

__device__ __forceinline__ float act(float v, int a) {
  if (a == 1) return fmaxf(v, 0.0f);  // relu (torch: NaN-propagating clamp; inputs here are finite)
  if (a == 2) return sigmoidf_(v);
  if (a == 3) return tanhf(v);
  return v;
}

// One workgroup per (b, c) row of P pixels; float4 along the row when every base is 16-B aligned and P % 4 == 0.
template <bool V4>
__global__ __launch_bounds__(256) void bias_act_kernel(const float* __restrict__ x, long long sx, const float* __restrict__ bias,
                                                        float* __restrict__ y0, long long sy0, float* __restrict__ y1,
                                                        long long sy1, int C, int P, int a, float scale) {
  const int b = blockIdx.x / C, c = blockIdx.x - (blockIdx.x / C) * C;
  const float* xr = x + b * sx + (long long)c * P;
  float* r0 = y0 + b * sy0 + (long long)c * P;
  float* r1 = y1 ? y1 + b * sy1 + (long long)c * P : nullptr;
  const float bb = bias ? bias[c] : 0.0f;
  if constexpr (V4) {
    for (int p = threadIdx.x; p < P / 4; p += blockDim.x) {
      float4 v = reinterpret_cast<const float4*>(xr)[p];
      v.x = act(v.x + bb, a); v.y = act(v.y + bb, a); v.z = act(v.z + bb, a); v.w = act(v.w + bb, a);
      if (scale != 1.0f) { v.x = v.x * scale; v.y = v.y * scale; v.z = v.z * scale; v.w = v.w * scale; }
      reinterpret_cast<float4*>(r0)[p] = v;
      if (r1) reinterpret_cast<float4*>(r1)[p] = v;
    }
  } else {
    for (int p = threadIdx.x; p < P; p += blockDim.x) {
      float v = act(xr[p] + bb, a);
      if (scale != 1.0f) v = v * scale;
      r0[p] = v;
      if (r1) r1[p] = v;
    }
  }
}

// zr: [z | r] pre-bias conv output (2*CH channels); rh = sigmoid(r + br) * h
template <bool V4>
__global__ __launch_bounds__(256) void gru_reset_kernel(const float* __restrict__ zr, long long szr, const float* __restrict__ br,
                                                         const float* __restrict__ h, long long sh, float* __restrict__ rh,
                                                         long long srh, int CH, int P) {
  const int b = blockIdx.x / CH, c = blockIdx.x - (blockIdx.x / CH) * CH;
  const float* rr = zr + b * szr + (long long)(CH + c) * P;
  const float* hr = h + b * sh + (long long)c * P;
  float* o = rh + b * srh + (long long)c * P;
  const float bb = br[c];
  if constexpr (V4) {
    for (int p = threadIdx.x; p < P / 4; p += blockDim.x) {
      const float4 r4 = reinterpret_cast<const float4*>(rr)[p];
      const float4 h4 = reinterpret_cast<const float4*>(hr)[p];
      reinterpret_cast<float4*>(o)[p] = make_float4(sigmoidf_(r4.x + bb) * h4.x, sigmoidf_(r4.y + bb) * h4.y,
                                                    sigmoidf_(r4.z + bb) * h4.z, sigmoidf_(r4.w + bb) * h4.w);
    }
  } else {
    for (int p = threadIdx.x; p < P; p += blockDim.x) o[p] = sigmoidf_(rr[p] + bb) * hr[p];
  }
}

__device__ __forceinline__ float blend(float zp, float bz, float qp, float bq, float hv) {
  const float z = sigmoidf_(zp + bz);
  const float q = tanhf(qp + bq);
  return (1.0f - z) * hv + z * q;
}

// h <- (1 - z) * h + z * tanh(q + bq), z = sigmoid(z_pre + bz); in place
template <bool V4>
__global__ __launch_bounds__(256) void gru_blend_kernel(const float* __restrict__ zr, long long szr, const float* __restrict__ bz,
                                                         const float* __restrict__ q, long long sq, const float* __restrict__ bq,
                                                         float* h, long long sh, int CH, int P) {
  const int b = blockIdx.x / CH, c = blockIdx.x - (blockIdx.x / CH) * CH;
  const float* zrow = zr + b * szr + (long long)c * P;
  const float* qrow = q + b * sq + (long long)c * P;
  float* hrow = h + b * sh + (long long)c * P;
  const float z0 = bz[c], q0 = bq[c];
  if constexpr (V4) {
    for (int p = threadIdx.x; p < P / 4; p += blockDim.x) {
      const float4 z4 = reinterpret_cast<const float4*>(zrow)[p];
      const float4 q4 = reinterpret_cast<const float4*>(qrow)[p];
      const float4 h4 = reinterpret_cast<const float4*>(hrow)[p];
      reinterpret_cast<float4*>(hrow)[p] = make_float4(blend(z4.x, z0, q4.x, q0, h4.x), blend(z4.y, z0, q4.y, q0, h4.y),
                                                       blend(z4.z, z0, q4.z, q0, h4.z), blend(z4.w, z0, q4.w, q0, h4.w));
    }
  } else {
    for (int p = threadIdx.x; p < P; p += blockDim.x) hrow[p] = blend(zrow[p], z0, qrow[p], q0, hrow[p]);
  }
}

inline bool a16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
inline bool s4(long long s) { return (s & 3) == 0; }

}  // namespace
}  // namespace oflow

using namespace oflow;

extern "C" int oflow_bias_act_f32(const float* d_x, long long sx, const float* d_bias, float* d_y0, long long sy0,
                                  float* d_y1, long long sy1, int B, int C, int P, int activation, float scale,
                                  void* stream) {
  if (!d_x || !d_y0) return OFLOW_E_NULL;
  if (B <= 0 || C <= 0 || P <= 0) return OFLOW_E_SHAPE;
  if (activation < 0 || activation > 3) return OFLOW_E_MODE;
  const bool v4 = P % 4 == 0 && a16(d_x) && a16(d_y0) && (!d_y1 || a16(d_y1)) && s4(sx) && s4(sy0) && s4(sy1);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (v4)
    hipLaunchKernelGGL(bias_act_kernel<true>, dim3(B * C), dim3(256), 0, s, d_x, sx, d_bias, d_y0, sy0, d_y1, sy1, C, P,
                       activation, scale);
  else
    hipLaunchKernelGGL(bias_act_kernel<false>, dim3(B * C), dim3(256), 0, s, d_x, sx, d_bias, d_y0, sy0, d_y1, sy1, C,
                       P, activation, scale);
  return launch_status();
}

extern "C" int oflow_gru_reset_f32(const float* d_zr, long long szr, const float* d_br, const float* d_h, long long sh,
                                   float* d_rh, long long srh, int B, int CH, int P, void* stream) {
  if (!d_zr || !d_br || !d_h || !d_rh) return OFLOW_E_NULL;
  if (B <= 0 || CH <= 0 || P <= 0) return OFLOW_E_SHAPE;
  const bool v4 = P % 4 == 0 && a16(d_zr) && a16(d_h) && a16(d_rh) && s4(szr) && s4(sh) && s4(srh);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (v4)
    hipLaunchKernelGGL(gru_reset_kernel<true>, dim3(B * CH), dim3(256), 0, s, d_zr, szr, d_br, d_h, sh, d_rh, srh, CH, P);
  else
    hipLaunchKernelGGL(gru_reset_kernel<false>, dim3(B * CH), dim3(256), 0, s, d_zr, szr, d_br, d_h, sh, d_rh, srh, CH, P);
  return launch_status();
}

extern "C" int oflow_gru_blend_f32(const float* d_zr, long long szr, const float* d_bz, const float* d_q, long long sq,
                                   const float* d_bq, float* d_h, long long sh, int B, int CH, int P, void* stream) {
  if (!d_zr || !d_bz || !d_q || !d_bq || !d_h) return OFLOW_E_NULL;
  if (B <= 0 || CH <= 0 || P <= 0) return OFLOW_E_SHAPE;
  const bool v4 = P % 4 == 0 && a16(d_zr) && a16(d_q) && a16(d_h) && s4(szr) && s4(sq) && s4(sh);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (v4)
    hipLaunchKernelGGL(gru_blend_kernel<true>, dim3(B * CH), dim3(256), 0, s, d_zr, szr, d_bz, d_q, sq, d_bq, d_h, sh, CH, P);
  else
    hipLaunchKernelGGL(gru_blend_kernel<false>, dim3(B * CH), dim3(256), 0, s, d_zr, szr, d_bz, d_q, sq, d_bq, d_h, sh, CH, P);
  return launch_status();
}
