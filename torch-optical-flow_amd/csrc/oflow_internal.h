// Internal helpers shared by the liboflow_hip kernels (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "oflow.h"

namespace oflow {

// Lane exchange inside 4-lane quads via DPP (no LDS traffic): quad_perm [1,0,3,2] and [2,3,0,1].
__device__ __forceinline__ float dpp_xor1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float dpp_xor2(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
}
// xor-4 within 32-lane groups: ds_swizzle bit mode (and 0x1F, or 0, xor 4); crossbar only, no LDS memory.
__device__ __forceinline__ float swz_xor4(float v) {
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x1F | (4 << 10)));
}

// avg_pool2d(2, stride=2) of one output: ATen sums the 2x2 window row by row into a zero-initialised
// accumulator and divides by 4 (exact), i.e. (((a + b) + c) + d) / 4 with a,b the upper pair.
__device__ __forceinline__ float pool4(float a, float b, float c, float d) {
  float s = __fadd_rn(__fadd_rn(__fadd_rn(a, b), c), d);
  return s * 0.25f;
}

// fp32 -> split fp16 pair (hi, lo): hi = fp16(v), lo = fp16(v - hi), so hi + lo holds v to ~22 bits (the S32 format).
// v is pinned to a VGPR first (empty asm) and contraction is off: otherwise the multiply that produced v (the GRU
// epilogue's r * h) is folded into the conversions -- hi as v_fma_mix (fp16(r * h), one rounding) and the residual
// from a second, double-rounded fp16(fp32(r * h)) -- and where the two roundings differ hi + lo is one fp16 ulp off
// (seen at 2 of 9216 elements, tests/test_gpu_conv_s32.py::test_conv_s32_gru_epilogues).
__device__ __forceinline__ void split_f16(float v, _Float16& hi, _Float16& lo) {
#pragma clang fp contract(off)
  asm volatile("" : "+v"(v));
  const _Float16 a = static_cast<_Float16>(v);
  hi = a;
  lo = static_cast<_Float16>(v - static_cast<float>(a));
}

// The lo halves of two values whose hi halves are packed in hi2 (hi2 = v_cvt_pk_f16_f32(v0, v1), RNE):
// fp16(v0 - hi0) | fp16(v1 - hi1) << 16 by v_fma_mixlo/mixhi_f16 (-hi * 1 + v, one rounding). v - hi is exact in fp32
// (|v - hi| <= half an fp16 ulp of v, a multiple of v's fp32 ulp), so the result equals split_f16's
// fp16(v - fp32(hi)) bit for bit, in 2 VALU per pair instead of 6. The callers pin v to a VGPR before converting
// (split_f16's note: a multiply producing v must not fold into the conversion).
__device__ __forceinline__ unsigned split_lo_pair(unsigned hi2, float v0, float v1) {
  unsigned lo;
  asm("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, -%1, 1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(lo)
      : "v"(hi2), "v"(v0), "v"(v1));
  return lo;
}

// split_f16 of two values at once: hi pair by v_cvt_pk_f16_f32 (RNE, as the scalar conversion), lo pair by
// split_lo_pair; bit for bit split_f16's halves, ~3 VALU per pair instead of ~8.
__device__ __forceinline__ void split_pair(float v0, float v1, unsigned& hi, unsigned& lo) {
  asm volatile("" : "+v"(v0), "+v"(v1));  // (split_f16's note: no folding of the producer into the conversions)
  typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
  const h2_t hp = {static_cast<_Float16>(v0), static_cast<_Float16>(v1)};
  hi = __builtin_bit_cast(unsigned, hp);
  lo = split_lo_pair(hi, v0, v1);
}
// 8 / 4 consecutive values -> their hi and lo halves as packed vectors (H, L: 16-B / 8-B vector types of fp16)
template <class H>
__device__ __forceinline__ void split_vec(const float* v, H& hi, H& lo) {
  constexpr int NP = sizeof(H) / 4;
  typedef unsigned uv_t __attribute__((ext_vector_type(NP)));
  uv_t hw, lw;
#pragma unroll
  for (int e = 0; e < NP; ++e) {
    unsigned h_, l_;
    split_pair(v[2 * e], v[2 * e + 1], h_, l_);
    hw[e] = h_;
    lw[e] = l_;
  }
  hi = __builtin_bit_cast(H, hw);
  lo = __builtin_bit_cast(H, lw);
}

// Range guard of the split-fp16 operands (S32, include/oflow.h): a value whose hi half would overflow fp16 (|v| >= 65520
// rounds to inf; inf included, NaN not) sets the device flag registered by oflow_set_range_flag (sticky; the host reads
// it once per forward and raises). Every translation unit that splits holds its own copy of the flag pointer
// (internal linkage); OFLOW_RANGE_FLAG_SETTER(name) defines that unit's setter, which oflow_set_range_flag calls.
namespace {
__device__ unsigned int* g_range_flag = nullptr;
}
__device__ __forceinline__ void range_guard(float max_abs) {
  if (__builtin_expect(max_abs >= 65520.0f, 0)) {
    unsigned int* f = g_range_flag;
    if (f != nullptr) atomicOr(f, 1u);
  }
}
__device__ __forceinline__ void range_guard8(const float* v) {
  range_guard(fmaxf(fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))),
                    fmaxf(fmaxf(fabsf(v[4]), fabsf(v[5])), fmaxf(fabsf(v[6]), fabsf(v[7])))));
}
#define OFLOW_RANGE_FLAG_SETTER(name)                                                              \
  int range_flag_set_##name(unsigned int* d_flag) {                                                \
    return static_cast<int>(hipMemcpyToSymbol(HIP_SYMBOL(g_range_flag), &d_flag, sizeof(d_flag)));     \
  }
int range_flag_set_conv(unsigned int* d_flag);
int range_flag_set_encoder(unsigned int* d_flag);
int range_flag_set_s32io(unsigned int* d_flag);
int range_flag_set_convc1(unsigned int* d_flag);

// Bilinear tap of the lookup: nw*w.x + ne*w.y + sw*w.z + se*w.w in one fixed rounding order, shared by every lookup
// kernel (corr_lookup.hip, corr_convc1.hip) so that they agree bit for bit.
__device__ __forceinline__ float bilinear4(float nw, float ne, float sw, float se, float4 w) {
  return fmaf(se, w.w, fmaf(sw, w.z, fmaf(ne, w.y, __fmul_rn(nw, w.x))));
}

// Window origin and bilinear weights of one (query, level) (corr.py:63-70 in pixel space): centre
// c = coords / 2^l; origin floor(c) - r; weights (nw, ne, sw, se) as grid_sample's CPU kernel forms them. |c| >= 2^22
// (or NaN / inf) puts every tap far outside any level: origin far away, all-zero window.
__device__ __forceinline__ void window_origin(float cx, float cy, float inv, int r, int& xs, int& ys, float4& w) {
  cx *= inv;
  cy *= inv;
  xs = -(1 << 28);
  ys = -(1 << 28);
  w = make_float4(0.f, 0.f, 0.f, 0.f);
  if (fabsf(cx) < 4194304.0f && fabsf(cy) < 4194304.0f) {
    const float fx = floorf(cx), fy = floorf(cy);
    const float wx = cx - fx, wy = cy - fy;  // exact
    const float ex = 1.0f - wx, ey = 1.0f - wy;
    xs = static_cast<int>(fx) - r;
    ys = static_cast<int>(fy) - r;
    w = make_float4(ey * ex, ey * wx, wy * ex, wy * wx);
  }
}

inline int launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? OFLOW_OK : static_cast<int>(e);
}

}  // namespace oflow
