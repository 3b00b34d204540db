// All-pairs correlation pyramid on fp32 MFMA (gfx950).
//
// Replaces methods/raft/model/corr.py:79-87 (corr = fmap1^T fmap2 / sqrt(C)) and corr.py:46-54 (reshape to
// (B*H*W, 1, H, W) then num_levels-1 avg_pool2d(2, stride=2)).
//
// GEMM view per batch b:  M = queries i (flattened H*W), N = targets j (flattened H*W), K = channels C.
// Both operands are stored K-major in the NCHW fmaps (A^T = fmap1[b] is [C][H*W], B = fmap2[b] is [C][H*W]),
// so a K-slab of either is a set of contiguous rows: staged global -> registers -> LDS as float4.
//
// Workgroup tile: 128 queries x (8 target rows x 32 target cols) = 128 x 256, 4 waves, each wave 32 queries
// x 256 targets = eight 32x32 accumulators of v_mfma_f32_32x32x2_f32 (exact fp32 fma chain, 128 acc VGPRs).
// The target tile is 8x8-aligned in (row, col) of the target grid, so every level-1..3 pooled pixel's whole
// footprint lies in one tile: the epilogue pools in registers and level 0 is never re-read from HBM.
//   accumulator n  <-> target row ty0 + n;  lane & 31 <-> target col tx0 + (lane & 31)
//   register r     <-> query i0 + 32*wave + (r & 3) + 8*(r >> 2) + 4*(lane >> 5)      (32x32 C/D map)
// Level-1 pooling pairs accumulators (2m, 2m+1) and lanes (x, x^1); level 2 pairs level-1 rows and lanes
// x^2; level 3 level-2 rows and lanes x^4 — DPP / ds_swizzle exchanges, no LDS round trip.
#include <type_traits>

#include "../../torch-optical-flow_amd/csrc/oflow_internal.h"

namespace oflow {
namespace {

constexpr int kBM = 128;        // queries per workgroup
constexpr int kTR = 8;          // target rows per tile
constexpr int kTC = 32;         // target cols per tile
constexpr int kBN = kTR * kTC;  // targets per tile
constexpr int kBK = 16;         // channels per LDS stage
constexpr int kThreads = 256;

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct PyramidArgs {
  const float* f1;
  const float* f2;
  float* lv[4];
  int C, H, W, N;
  int Hl[4], Wl[4];
  int nlev;         // levels written by the fused kernel (1..4)
  int tiles_x;      // ceil(W / 32)
  float scale;      // sqrt(C) as torch computes it (float sqrt of float(C))
  float inv_scale;  // exact 1/scale when scale is a power of two (multiply == divide bit-for-bit)
  int scale_pow2;
};

template <bool VEC, int B64 = 0>
struct Stage {
  // VEC: float4 loads (H*W % 4 == 0, W % 4 == 0, 16-B aligned bases); else scalar loads.
  static constexpr int kA = VEC ? (kBK * kBM / 4) / kThreads : (kBK * kBM) / kThreads;  // 2 or 8
  static constexpr int kB = VEC ? (kBK * kBN / 4) / kThreads : (kBK * kBN) / kThreads;  // 4 or 16
  typedef typename std::conditional<VEC, float4, float>::type T;
  T a[kA];
  T b[kB];

  __device__ __forceinline__ void load(const PyramidArgs& p, const float* F1, const float* F2, int k0, int i0,
                                       int ty0, int tx0) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int s = 0; s < kA; ++s) {
      const int idx = tid + kThreads * s;
      const int k = VEC ? (idx >> 5) : (idx >> 7);
      const int m = VEC ? ((idx & 31) << 2) : (idx & 127);
      const int kk = k0 + k, ii = i0 + m;
      if constexpr (VEC) {
        a[s] = (kk < p.C && ii < p.N) ? *reinterpret_cast<const float4*>(F1 + (size_t)kk * p.N + ii)
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        a[s] = (kk < p.C && ii < p.N) ? F1[(size_t)kk * p.N + ii] : 0.f;
      }
    }
#pragma unroll
    for (int s = 0; s < kB; ++s) {
      const int idx = tid + kThreads * s;
      const int k = VEC ? (idx >> 6) : (idx >> 8);
      const int rem = VEC ? (idx & 63) : (idx & 255);
      const int n = VEC ? (rem >> 3) : (rem >> 5);
      const int c = VEC ? ((rem & 7) << 2) : (rem & 31);
      const int kk = k0 + k, y = ty0 + n, x = tx0 + c;
      const bool ok = kk < p.C && y < p.H && x < p.W;
      if constexpr (VEC) {
        b[s] = ok ? *reinterpret_cast<const float4*>(F2 + (size_t)kk * p.N + (size_t)y * p.W + x)
                  : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        b[s] = ok ? F2[(size_t)kk * p.N + (size_t)y * p.W + x] : 0.f;
      }
    }
  }

  __device__ __forceinline__ void store(float (*sA)[kBM], float (*sB)[kBN]) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int s = 0; s < kA; ++s) {
      const int idx = tid + kThreads * s;
      if constexpr (VEC && B64) {
        const int k = idx >> 5, m = (idx & 31) << 2;
        float* base = &sA[0][0] + (k >> 1) * kBM * 2 + (k & 1);
        base[(m + 0) * 2] = a[s].x; base[(m + 1) * 2] = a[s].y; base[(m + 2) * 2] = a[s].z; base[(m + 3) * 2] = a[s].w;
      } else if constexpr (VEC) {
        *reinterpret_cast<float4*>(&sA[idx >> 5][(idx & 31) << 2]) = a[s];
      } else {
        sA[idx >> 7][idx & 127] = a[s];
      }
    }
#pragma unroll
    for (int s = 0; s < kB; ++s) {
      const int idx = tid + kThreads * s;
      if constexpr (VEC && B64) {
        const int rem = idx & 63, k = idx >> 6, n = ((rem >> 3) << 5) + ((rem & 7) << 2);
        float* base = &sB[0][0] + (k >> 1) * kBN * 2 + (k & 1);
        base[(n + 0) * 2] = b[s].x; base[(n + 1) * 2] = b[s].y; base[(n + 2) * 2] = b[s].z; base[(n + 3) * 2] = b[s].w;
      } else if constexpr (VEC) {
        const int rem = idx & 63;
        *reinterpret_cast<float4*>(&sB[idx >> 6][((rem >> 3) << 5) + ((rem & 7) << 2)]) = b[s];
      } else {
        sB[idx >> 8][idx & 255] = b[s];
      }
    }
  }
};

template <bool VEC, int NOSTORE, int B64>
__global__ __launch_bounds__(kThreads, 2) void corr_pyramid_kernel(PyramidArgs p) {
  __shared__ __attribute__((aligned(16))) float sA[2][kBK][kBM];
  __shared__ __attribute__((aligned(16))) float sB[2][kBK][kBN];
  // B64 view: [buf][k/2][m][2] over the same bytes (the stage writer below fills it in that order when B64)
  auto sAp = reinterpret_cast<float (*)[kBK / 2][kBM][2]>(&sA[0][0][0]);
  auto sBp = reinterpret_cast<float (*)[kBK / 2][kBN][2]>(&sB[0][0][0]);

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int tile = blockIdx.x;
  const int ty0 = (tile / p.tiles_x) * kTR;
  const int tx0 = (tile % p.tiles_x) * kTC;
  const int i0 = blockIdx.y * kBM;
  const int b = blockIdx.z;
  const float* F1 = p.f1 + (size_t)b * p.C * p.N;
  const float* F2 = p.f2 + (size_t)b * p.C * p.N;

  f32x16 acc[kTR];
#pragma unroll
  for (int n = 0; n < kTR; ++n) acc[n] = f32x16{0};

  Stage<VEC, B64> st;
  const int nk = (p.C + kBK - 1) / kBK;
  st.load(p, F1, F2, 0, i0, ty0, tx0);
  st.store(sA[0], sB[0]);
  __syncthreads();

  const int kl = lane >> 5;          // k within an MFMA k-step (32x32x2: lanes 32-63 hold k = 1)
  const int ml = wave * 32 + (lane & 31);
  const int nl = lane & 31;
  for (int c = 0; c < nk; ++c) {
    const int buf = c & 1;
    if (c + 1 < nk) st.load(p, F1, F2, (c + 1) * kBK, i0, ty0, tx0);
    if (B64) {
#pragma unroll
      for (int kk = 0; kk < kBK; kk += 4) {
        // k-order permuted: lanes 0-31 take k = kk, kk+1; lanes 32-63 take kk+2, kk+3 (same for A and B)
        const float2 av = *reinterpret_cast<const float2*>(&sAp[buf][(kk >> 1) + kl][ml][0]);
#pragma unroll
        for (int n = 0; n < kTR; ++n) {
          const float2 bv = *reinterpret_cast<const float2*>(&sBp[buf][(kk >> 1) + kl][n * kTC + nl][0]);
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, bv.x, acc[n], 0, 0, 0);
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, bv.y, acc[n], 0, 0, 0);
        }
      }
    } else {
#pragma unroll
    for (int kk = 0; kk < kBK; kk += 2) {
      const float av = sA[buf][kk + kl][ml];
#pragma unroll
      for (int n = 0; n < kTR; ++n) {
        const float bv = sB[buf][kk + kl][n * kTC + nl];
        acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[n], 0, 0, 0);
      }
    }
    }
    if (c + 1 < nk) st.store(sA[buf ^ 1], sB[buf ^ 1]);
    __syncthreads();
  }

  // ---- epilogue: scale, level-0 store, in-register pooled levels 1..3 ----
  const int tx = lane & 31;
  const int qbase = i0 + wave * 32 + 4 * (lane >> 5);
  const size_t Nn = (size_t)p.N;
#pragma unroll
  for (int n = 0; n < kTR; ++n) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[n][r] = p.scale_pow2 ? acc[n][r] * p.inv_scale : acc[n][r] / p.scale;
  }

  {  // level 0: (B*N, H, W)
    float* L0 = p.lv[0];
    const int gx = tx0 + tx;
#pragma unroll
    for (int n = 0; n < kTR; ++n) {
      const int gy = ty0 + n;
      const bool ok = gx < p.W && gy < p.H;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = qbase + (r & 3) + 8 * (r >> 2);
        if (!NOSTORE && ok && i < p.N) L0[((size_t)b * Nn + i) * Nn + (size_t)gy * p.W + gx] = acc[n][r];
      }
    }
  }
  if (p.nlev < 2) return;

  float v2[2][16];
  const int H1 = p.Hl[1], W1 = p.Wl[1];
  const int x1 = (tx0 >> 1) + (tx >> 1);
  const bool lane1 = (tx & 1) == 0 && x1 < W1;
  const int H2 = p.Hl[2], W2 = p.Wl[2];
  const int x2 = (tx0 >> 2) + (tx >> 2);
  const bool lane2 = (tx & 3) == 0 && x2 < W2;
#pragma unroll
  for (int pr = 0; pr < 2; ++pr) {
    float v1[2][16];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int m = 2 * pr + h;
      const int y1 = (ty0 >> 1) + m;
      const bool ok = lane1 && y1 < H1;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float a0 = acc[2 * m][r], c0 = acc[2 * m + 1][r];
        v1[h][r] = pool4(a0, dpp_xor1(a0), c0, dpp_xor1(c0));
        const int i = qbase + (r & 3) + 8 * (r >> 2);
        if ((!NOSTORE || v1[h][r] == 1234.5f) && ok && i < p.N) p.lv[1][((size_t)b * Nn + i) * (size_t)(H1 * W1) + (size_t)y1 * W1 + x1] = v1[h][r];
      }
    }
    if (p.nlev >= 3) {
      const int y2 = (ty0 >> 2) + pr;
      const bool ok = lane2 && y2 < H2;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float a0 = v1[0][r], c0 = v1[1][r];
        v2[pr][r] = pool4(a0, dpp_xor2(a0), c0, dpp_xor2(c0));
        const int i = qbase + (r & 3) + 8 * (r >> 2);
        if ((!NOSTORE || v2[pr][r] == 1234.5f) && ok && i < p.N) p.lv[2][((size_t)b * Nn + i) * (size_t)(H2 * W2) + (size_t)y2 * W2 + x2] = v2[pr][r];
      }
    }
  }
  if (p.nlev < 4) return;
  {
    const int H3 = p.Hl[3], W3 = p.Wl[3];
    const int x3 = (tx0 >> 3) + (tx >> 3);
    const int y3 = ty0 >> 3;
    const bool ok = (tx & 7) == 0 && x3 < W3 && y3 < H3;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float a0 = v2[0][r], c0 = v2[1][r];
      const float v3 = pool4(a0, swz_xor4(a0), c0, swz_xor4(c0));
      const int i = qbase + (r & 3) + 8 * (r >> 2);
      if ((!NOSTORE || v3 == 1234.5f) && ok && i < p.N) p.lv[3][((size_t)b * Nn + i) * (size_t)(H3 * W3) + (size_t)y3 * W3 + x3] = v3;
    }
  }
}

// Levels >= 4 (num_levels > 4 only): plain floor 2x2 average pool of the level above.
__global__ __launch_bounds__(256) void avgpool2x2_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                          long long planes, int Hin, int Win, int Hout, int Wout) {
  const long long total = planes * Hout * Wout;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const long long pl = t / ((long long)Hout * Wout);
    const int rem = (int)(t - pl * Hout * Wout);
    const int y = rem / Wout, x = rem - y * Wout;
    const float* s = in + pl * Hin * Win + (size_t)(2 * y) * Win + 2 * x;
    out[t] = pool4(s[0], s[1], s[Win], s[Win + 1]);
  }
}

}  // namespace
}  // namespace oflow

using namespace oflow;
extern "C" int exp_pyramid(const float* f1, const float* f2, int B, int C, int H, int W, float* const* lv, int nostore, int b64, void* stream) {
  PyramidArgs p{};
  p.f1 = f1; p.f2 = f2; p.C = C; p.H = H; p.W = W; p.N = H * W; p.nlev = 4;
  int h = H, w = W;
  for (int l = 0; l < 4; ++l) { p.lv[l] = lv[l]; p.Hl[l] = h; p.Wl[l] = w; h /= 2; w /= 2; }
  p.tiles_x = (W + kTC - 1) / kTC; p.scale = 16.0f; p.scale_pow2 = 1; p.inv_scale = 1.0f / 16.0f;
  dim3 grid(p.tiles_x * ((H + kTR - 1) / kTR), (p.N + kBM - 1) / kBM, B);
  hipStream_t s = (hipStream_t)stream;
  if (nostore == 0 && b64 == 0) hipLaunchKernelGGL((corr_pyramid_kernel<true, 0, 0>), grid, dim3(kThreads), 0, s, p);
  else if (nostore == 1 && b64 == 0) hipLaunchKernelGGL((corr_pyramid_kernel<true, 1, 0>), grid, dim3(kThreads), 0, s, p);
  else if (nostore == 0 && b64 == 1) hipLaunchKernelGGL((corr_pyramid_kernel<true, 0, 1>), grid, dim3(kThreads), 0, s, p);
  else if (nostore == 1 && b64 == 1) hipLaunchKernelGGL((corr_pyramid_kernel<true, 1, 1>), grid, dim3(kThreads), 0, s, p);
  return (int)hipGetLastError();
}
