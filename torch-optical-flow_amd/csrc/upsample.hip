// Convex upsampling of the low-resolution flow (gfx950), SURVEY.md §8(f) row 2.
//
// Replaces methods/raft/model/raft.py:73-85 (RAFT.upsample_flow): softmax over the 9 neighbour weights of each of the
// 8x8 sub-pixels (mask.view(N, 1, 9, 8, 8, H, W), dim 2), F.unfold(8 * flow, 3x3, padding 1), the weighted sum, the
// permute and the reshape -- five ATen passes -- as one kernel:
//   out[n, c, 8y + i, 8x + j] = sum_k softmax_k(mask[n, k*64 + i*8 + j, y, x]) * 8 * flow[n, c, y + k/3 - 1, x + k%3 - 1]
// (zero padding outside the low-resolution grid).
//
// One workgroup = one low-res row segment of 32 pixels, looping over the 8 sub-pixel rows i: the 9 x 8 x 32 mask
// values of row i are read as 72 coalesced 128-B rows (lanes along x) into LDS and consumed with lanes along
// (x, j), so both the mask reads and the (B, 2, 8H, 8W) output rows (256 consecutive floats per channel) are
// coalesced. Bound: HBM, (576 + 2*64) * 4 B per low-res pixel + the flow.
#include "oflow_internal.h"

namespace oflow {
namespace {

constexpr int kUX = 32;  // low-res pixels per workgroup

__global__ __launch_bounds__(256) void convex_upsample_kernel(const float* __restrict__ flow,
                                                              const float* __restrict__ mask, int H, int W,
                                                              float* __restrict__ out) {
  __shared__ float sM[9][8][kUX + 1];
  __shared__ float sF[2][3][kUX + 2];
  const int tid = threadIdx.x;
  const int xb = blockIdx.x, y = blockIdx.y, n = blockIdx.z;
  const int x0 = xb * kUX;
  const long long HW = (long long)H * W;
  const float* fl = flow + (long long)n * 2 * HW;
  const float* mk = mask + (long long)n * 576 * HW + (long long)y * W;
  // 8 * flow on the 3 x (32 + 2) neighbourhood, zeros outside (unfold's padding)
  for (int e = tid; e < 2 * 3 * (kUX + 2); e += 256) {
    const int c = e / (3 * (kUX + 2)), rem = e - c * 3 * (kUX + 2);
    const int dy = rem / (kUX + 2), dx = rem - dy * (kUX + 2);
    const int yy = y + dy - 1, xx = x0 + dx - 1;
    float v = 0.f;
    if (yy >= 0 && yy < H && xx >= 0 && xx < W) v = 8.0f * fl[c * HW + (long long)yy * W + xx];
    sF[c][dy][dx] = v;
  }
  // output mapping: lane -> (x, j) with j fastest: 256 consecutive output floats per channel row
  const int xo = tid >> 3, j = tid & 7;
  const bool live = x0 + xo < W;
  for (int i = 0; i < 8; ++i) {
    __syncthreads();  // sF ready (i = 0) / every thread is done with row i-1's mask
    // 9 k x 8 j rows of 32 x: lanes along x
    for (int e = tid; e < 9 * 8 * kUX; e += 256) {
      const int row = e / kUX, xl = e - row * kUX;
      const int k = row >> 3, jj = row & 7;
      float v = 0.f;
      if (x0 + xl < W) v = mk[(long long)(k * 64 + i * 8 + jj) * HW + x0 + xl];
      sM[k][jj][xl] = v;
    }
    __syncthreads();
    if (live) {
      float m[9];
      float mx = sM[0][j][xo];
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        m[k] = sM[k][j][xo];
        mx = fmaxf(mx, m[k]);
      }
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        m[k] = expf(m[k] - mx);
        s += m[k];
      }
      float o0 = 0.f, o1 = 0.f;
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const float w = m[k] / s;
        const int dy = k / 3, dx = k % 3;
        o0 += w * sF[0][dy][xo + dx];
        o1 += w * sF[1][dy][xo + dx];
      }
      const long long W8 = 8LL * W, H8W8 = 64LL * HW;
      float* op = out + (long long)n * 2 * H8W8 + (long long)(8 * y + i) * W8 + 8LL * (x0 + xo) + j;
      op[0] = o0;
      op[H8W8] = o1;
    }
  }
}

}  // namespace
}  // namespace oflow

using namespace oflow;

extern "C" int oflow_convex_upsample_f32(const float* d_flow, const float* d_mask, int B, int H, int W, float* d_out,
                                         void* stream) {
  if (!d_flow || !d_mask || !d_out) return OFLOW_E_NULL;
  if (B <= 0 || H <= 0 || W <= 0 || B > 65535 || H > 65535) return OFLOW_E_SHAPE;
  dim3 grid((W + kUX - 1) / kUX, H, B);
  hipLaunchKernelGGL(convex_upsample_kernel, grid, dim3(256), 0, static_cast<hipStream_t>(stream), d_flow, d_mask, H,
                     W, d_out);
  return launch_status();
}
