// EXPERIMENT: sustained v_mfma_f32_32x32x16_f16 rate on this chip with the conv kernel's issue pattern (4 accumulators,
// 3 dependent MFMAs each per operand set), operands from registers, random data; 2 and 1 waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ __launch_bounds__(256) void mfma_loop(const half8* __restrict__ src, float* __restrict__ out, int iters) {
  const int lane = threadIdx.x;
  half8 a0 = src[lane], a1 = src[lane + 256], b0 = src[lane + 512], b1 = src[lane + 768];
  f32x16 acc[NACC];
#pragma unroll
  for (int j = 0; j < NACC; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < NACC; ++j) {
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, acc[j], 0, 0, 0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NACC; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) s += acc[j][e];
  out[blockIdx.x * 256 + lane] = s;
}

// fp32 form (corr_pyramid's instruction): 8 independent accumulators
__global__ __launch_bounds__(256) void mfma_loop_f32(const float* __restrict__ src, float* __restrict__ out, int iters) {
  const int lane = threadIdx.x;
  float a0 = src[lane], a1 = src[lane + 256];
  f32x16 acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(j & 1 ? a0 : a1, a0, acc[j], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) s += acc[j][e];
  out[blockIdx.x * 256 + lane] = s;
}

extern "C" int exp_mfma_f32(const void* src, float* out, int blocks, int iters, void* stream) {
  hipLaunchKernelGGL(mfma_loop_f32, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream), (const float*)src, out, iters);
  return hipGetLastError();
}

extern "C" int exp_mfma(int nacc, const void* src, float* out, int blocks, int iters, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (nacc == 4)
    hipLaunchKernelGGL((mfma_loop<4>), dim3(blocks), dim3(256), 0, s, (const half8*)src, out, iters);
  else
    hipLaunchKernelGGL((mfma_loop<8>), dim3(blocks), dim3(256), 0, s, (const half8*)src, out, iters);
  return hipGetLastError();
}
