// On-the-fly ("alternate") correlation lookup in fp16 for large frames (BASELINE configs[4]: 1080p), gfx950.
//
// Same output as CorrBlock(fmap1, fmap2)(coords) (methods/raft/model/corr.py:38-87, utils.py:64-80) without the
// O((HW)^2) volume. By linearity of the pooling (corr.py:53) in the target dims,
//     corr_l[q, y, x] = < fmap1[:, q], pool_l(fmap2)[:, y, x] > / sqrt(C)
// where pool_l is the floor 2^l x 2^l average of fmap2 (= l iterated floor 2x2 pools). So the lookup needs only
// fmap1 and a 4-level fmap2 pyramid (SURVEY.md §5 "Long-context analogue"): per (query, level) the (2r+2)^2
// window of dot products, then the same shared-weight bilinear stencil as the dense lookup.
//
// Storage: fmap1 pre-scaled by 1/sqrt(C) and every fmap2 level in NHWC fp16 (a pixel's C channels contiguous:
// one MFMA operand fragment = 16 B). Pooling is done in fp32 before the fp16 rounding.
//
// Lookup kernel: a workgroup takes a segment of queries (2 query rows x 16 query cols = 32 queries, one
// level). The union of their windows is a bounding box of T targets (T <= kTMax for smooth flow). The box is
// computed as a small GEMM on v_mfma_f32_16x16x32_f16: C[32 q x T] = f1[32 x C] . F2[C x T] (fp32 accumulate),
// written to LDS, and each query's 81 outputs are sampled from its own window of that tile. Segments whose box
// exceeds kTMax (divergent flow) fall back to one query per pass (box = its own window, T <= (2r+2)^2).
#include <hip/hip_fp16.h>

#include "oflow_internal.h"

namespace oflow {
namespace {

constexpr int kQR = 2;                 // query rows per segment
constexpr int kQC = 16;                // query cols per segment
constexpr int kQ = kQR * kQC;          // 32 queries
constexpr int kTMax = 384;             // max targets per box (24 N-tiles)
constexpr int kNT = kTMax / 16;        // 24
constexpr int kNTW = kNT / 4;          // N-tiles per wave (6)
constexpr int kCS = kTMax + 4;         // LDS row stride of the corr tile
constexpr int kThreads = 256;

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---- fmap (B, C, H, W) fp32 -> (B, H, W, C) fp16 * scale ----
__global__ __launch_bounds__(256) void to_nhwc_f16_kernel(const float* __restrict__ in, __half* __restrict__ out, int B,
                                                          int C, int HW, float scale) {
  // 64 pixels x 64 channels per block through LDS: coalesced reads along pixels, 128-B writes along channels
  __shared__ float tile[64][65];
  const int b = blockIdx.z;
  const int p0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int c = c0 + r, p = p0 + tx;
    tile[r][tx] = (c < C && p < HW) ? in[((size_t)b * C + c) * HW + p] * scale : 0.0f;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int p = p0 + r, c = c0 + tx;
    if (p < HW && c < C) out[((size_t)b * HW + p) * C + c] = __float2half_rn(tile[tx][r]);
  }
}

// floor 2x2 average pool of (planes, Hin, Win) fp32 -> (planes, Hout, Wout), ATen's summation order
__global__ __launch_bounds__(256) void otf_pool_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                        long long planes, int Hin, int Win, int Hout, int Wout) {
  const long long total = planes * Hout * Wout;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const long long pl = t / ((long long)Hout * Wout);
    const int rem = (int)(t - pl * Hout * Wout);
    const int y = rem / Wout, x = rem - y * Wout;
    const float* src = in + pl * Hin * Win + (size_t)(2 * y) * Win + 2 * x;
    out[t] = pool4(src[0], src[1], src[Win], src[Win + 1]);
  }
}

struct OtfArgs {
  const __half* f1;              // (B, H, W, C)
  const __half* f2[OFLOW_MAX_LEVELS];  // (B, H_l, W_l, C)
  int Hl[OFLOW_MAX_LEVELS], Wl[OFLOW_MAX_LEVELS];
  const float* coords;           // (B, 2, H, W)
  float* out;                    // (B, L*K*K, H, W)
  int B, C, H, W, segx, segy, cout;
};

template <int R>
__global__ __launch_bounds__(kThreads) void corr_otf_kernel(OtfArgs a) {
  constexpr int PK = 2 * R + 2, K = 2 * R + 1;
  __shared__ float sC[kQ * kCS];          // corr tile: [query][target]
  __shared__ int sXs[kQ], sYs[kQ];        // window origin (level pixels), or huge when invalid
  __shared__ float4 sW[kQ];

  const int lvl = blockIdx.y;
  const int seg = blockIdx.x;
  const int b = seg / (a.segx * a.segy);
  const int sr = seg - b * a.segx * a.segy;
  const int qy0 = (sr / a.segx) * kQR, qx0 = (sr % a.segx) * kQC;
  const int Hl = a.Hl[lvl], Wl = a.Wl[lvl];
  const __half* __restrict__ F2 = a.f2[lvl];
  const int N = a.H * a.W;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // provably wave-uniform for the MFMA guards

  if (threadIdx.x < kQ) {
    const int qy = qy0 + threadIdx.x / kQC, qx = qx0 + threadIdx.x % kQC;
    int xs = 1 << 28, ys = 1 << 28;
    float4 w = make_float4(0.f, 0.f, 0.f, 0.f);
    if (qy < a.H && qx < a.W) {
      const float inv = 1.0f / static_cast<float>(1 << lvl);
      const float cx = a.coords[((size_t)(2 * b) * a.H + qy) * a.W + qx] * inv;
      const float cy = a.coords[((size_t)(2 * b + 1) * a.H + qy) * a.W + qx] * inv;
      if (fabsf(cx) < 4194304.0f && fabsf(cy) < 4194304.0f) {
        const float fx = floorf(cx), fy = floorf(cy);
        const float wx = cx - fx, wy = cy - fy, ex = 1.0f - wx, ey = 1.0f - wy;
        xs = static_cast<int>(fx) - R;
        ys = static_cast<int>(fy) - R;
        w = make_float4(ey * ex, ey * wx, wy * ex, wy * wx);
      }
    }
    sXs[threadIdx.x] = xs;
    sYs[threadIdx.x] = ys;
    sW[threadIdx.x] = w;
  }
  __syncthreads();

  // Box of the whole segment, clipped to the level (taps outside the level are zero padding).
  int by0 = 1 << 29, bx0 = 1 << 29, by1 = -(1 << 29), bx1 = -(1 << 29);
  for (int q = 0; q < kQ; ++q) {
    const int ys = sYs[q], xs = sXs[q];
    if (ys < (1 << 27) && ys + PK > 0 && ys < Hl && xs + PK > 0 && xs < Wl) {
      by0 = min(by0, ys);
      bx0 = min(bx0, xs);
      by1 = max(by1, ys + PK - 1);
      bx1 = max(bx1, xs + PK - 1);
    }
  }
  by0 = max(by0, 0);
  bx0 = max(bx0, 0);
  by1 = min(by1, Hl - 1);
  bx1 = min(bx1, Wl - 1);
  const bool any = by1 >= by0 && bx1 >= bx0;
  const bool fits = any && (by1 - by0 + 1) * (bx1 - bx0 + 1) <= kTMax;
  const int passes = !any ? 0 : (fits ? 1 : kQ);

  for (int pass = 0; pass < passes; ++pass) {
    // queries of this pass: all (fits) or query `pass` alone
    int y0 = by0, x0 = bx0, bh = by1 - by0 + 1, bw = bx1 - bx0 + 1;
    if (!fits) {
      const int ys = sYs[pass], xs = sXs[pass];
      y0 = max(ys, 0);
      x0 = max(xs, 0);
      bh = min(ys + PK - 1, Hl - 1) - y0 + 1;
      bw = min(xs + PK - 1, Wl - 1) - x0 + 1;
    }
    // a lone query whose window misses the level only needs its zero outputs (uniform across the workgroup)
    const bool gemm = fits || (sYs[pass] < (1 << 27) && bh > 0 && bw > 0);
    const int T = gemm ? bh * bw : 0;
    const int nT = (T + 15) >> 4;

    // ---- GEMM: rows = 32 queries (2 M-tiles), cols = T targets; wave w takes N-tiles w, w+4, ... ----
    f32x4 acc[kNTW][2];
#pragma unroll
    for (int j = 0; j < kNTW; ++j) acc[j][0] = acc[j][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int kg = 8 * (lane >> 4);  // this lane's channel offset inside a 32-channel step
    const __half* arow[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int qi = m * 16 + (lane & 15);
      const int qy = qy0 + qi / kQC, qx = qx0 + qi % kQC;
      const bool ok = (fits || qi == pass) && qy < a.H && qx < a.W;
      arow[m] = ok ? a.f1 + ((size_t)b * N + (size_t)qy * a.W + qx) * a.C + kg : nullptr;
    }
    const __half* bcol[kNTW];
#pragma unroll
    for (int j = 0; j < kNTW; ++j) {
      const int t = (wave + 4 * j) * 16 + (lane & 15);
      bcol[j] = nullptr;
      if (t < T) {
        const int ty = y0 + t / bw, tx = x0 + t % bw;
        bcol[j] = F2 + (((size_t)b * Hl + ty) * Wl + tx) * a.C + kg;
      }
    }
    for (int k0 = 0; gemm && k0 < a.C; k0 += 32) {
      half8 af[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        af[m] = half8{};
        if (arow[m]) af[m] = *reinterpret_cast<const half8*>(arow[m] + k0);
      }
#pragma unroll
      for (int j = 0; j < kNTW; ++j) {
        if (wave + 4 * j < nT) {  // wave-uniform
          half8 bf = half8{};
          if (bcol[j]) bf = *reinterpret_cast<const half8*>(bcol[j] + k0);
          acc[j][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[0], bf, acc[j][0], 0, 0, 0);
          acc[j][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[1], bf, acc[j][1], 0, 0, 0);
        }
      }
    }
    // C/D map of 16x16 MFMA: col = lane & 15, row = 4*(lane >> 4) + reg
#pragma unroll
    for (int j = 0; j < kNTW; ++j) {
      const int n = wave + 4 * j;
      if (n < nT) {
        const int t = n * 16 + (lane & 15);
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int r = 0; r < 4; ++r) sC[(m * 16 + 4 * (lane >> 4) + r) * kCS + t] = acc[j][m][r];
      }
    }
    __syncthreads();

    // ---- bilinear sampling of each query's window from the tile ----
    const int nq = fits ? kQ : 1;
    for (int o = threadIdx.x; o < nq * K * K; o += kThreads) {
      const int c = o / nq;
      const int qi = fits ? o - c * nq : pass;
      const int qy = qy0 + qi / kQC, qx = qx0 + qi % kQC;
      if (qy >= a.H || qx >= a.W) continue;
      const int i = c / K, j = c - i * K;
      const int ys = sYs[qi], xs = sXs[qi];
      float val = 0.0f;
      if (ys < (1 << 27)) {
        const float4 w = sW[qi];
        const float* row = &sC[qi * kCS];
        float v[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const int y = ys + j + (d >> 1), x = xs + i + (d & 1);
          v[d] = (static_cast<unsigned>(y) < static_cast<unsigned>(Hl) && static_cast<unsigned>(x) < static_cast<unsigned>(Wl))
                     ? row[(y - y0) * bw + (x - x0)]
                     : 0.0f;
        }
        val = v[0] * w.x + v[1] * w.y + v[2] * w.z + v[3] * w.w;
      }
      a.out[(((size_t)b * a.cout + lvl * K * K + c) * a.H + qy) * a.W + qx] = val;
    }
    __syncthreads();
  }

  if (passes == 0) {  // every window of the segment is outside the level: zeros
    for (int o = threadIdx.x; o < kQ * K * K; o += kThreads) {
      const int c = o / kQ, qi = o - c * kQ;
      const int qy = qy0 + qi / kQC, qx = qx0 + qi % kQC;
      if (qy < a.H && qx < a.W) a.out[(((size_t)b * a.cout + lvl * K * K + c) * a.H + qy) * a.W + qx] = 0.0f;
    }
  }
}

template <int R>
int launch_otf(const OtfArgs& a, int nlev, hipStream_t s) {
  dim3 grid(a.B * a.segx * a.segy, nlev);
  hipLaunchKernelGGL(corr_otf_kernel<R>, grid, dim3(kThreads), 0, s, a);
  return launch_status();
}

}  // namespace
}  // namespace oflow

using namespace oflow;

// level 0 of fmap2 and fmap1 -> NHWC fp16; levels 1.. pooled in fp32 (scratch, NCHW) then converted.
extern "C" int oflow_corr_otf_prepare_f16(const float* d_fmap1, const float* d_fmap2, int B, int C, int H, int W,
                                          int num_levels, void* d_f1h, void* const* d_f2h, float* d_scratch,
                                          void* stream) {
  if (!d_fmap1 || !d_fmap2 || !d_f1h || !d_f2h) return OFLOW_E_NULL;
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || C % 32 != 0) return OFLOW_E_SHAPE;
  int hl[OFLOW_MAX_LEVELS], wl[OFLOW_MAX_LEVELS];
  int st = oflow_corr_pyramid_dims(H, W, num_levels, hl, wl);
  if (st != OFLOW_OK) return st;
  for (int l = 0; l < num_levels; ++l) {
    if (hl[l] < 1 || wl[l] < 1) return OFLOW_E_TINY;
    if (!d_f2h[l]) return OFLOW_E_NULL;
  }
  if (num_levels > 1 && !d_scratch) return OFLOW_E_NULL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const float scale = 1.0f / sqrtf(static_cast<float>(C));
  auto conv = [&](const float* src, void* dst, int hw, float sc) {
    dim3 grid((hw + 63) / 64, (C + 63) / 64, B);
    hipLaunchKernelGGL(to_nhwc_f16_kernel, grid, dim3(256), 0, s, src, static_cast<__half*>(dst), B, C, hw, sc);
    return launch_status();
  };
  if ((st = conv(d_fmap1, d_f1h, H * W, scale)) != OFLOW_OK) return st;
  if ((st = conv(d_fmap2, d_f2h[0], H * W, 1.0f)) != OFLOW_OK) return st;
  const float* prev = d_fmap2;
  float* cur = d_scratch;
  for (int l = 1; l < num_levels; ++l) {
    const long long planes = (long long)B * C;
    const long long total = planes * hl[l] * wl[l];
    const int blocks = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
    hipLaunchKernelGGL(otf_pool_kernel, dim3(blocks), dim3(256), 0, s, prev, cur, planes, hl[l - 1], wl[l - 1], hl[l], wl[l]);
    if ((st = launch_status()) != OFLOW_OK) return st;
    if ((st = conv(cur, d_f2h[l], hl[l] * wl[l], 1.0f)) != OFLOW_OK) return st;
    prev = cur;
    cur += planes * hl[l] * wl[l];
  }
  return OFLOW_OK;
}

extern "C" int oflow_corr_lookup_otf_f16(const void* d_f1h, const void* const* d_f2h, const int* level_h,
                                         const int* level_w, int num_levels, const float* d_coords, int B, int C,
                                         int H, int W, int radius, float* d_out, void* stream) {
  if (!d_f1h || !d_f2h || !level_h || !level_w || !d_coords || !d_out) return OFLOW_E_NULL;
  if (B <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 32 != 0) return OFLOW_E_SHAPE;
  if (num_levels < 1 || num_levels > OFLOW_MAX_LEVELS) return OFLOW_E_LEVELS;
  if (radius < 0 || radius > 4) return OFLOW_E_RADIUS;  // (2r+2)^2 <= 100 <= kTMax keeps the fallback exact
  OtfArgs a{};
  a.f1 = static_cast<const __half*>(d_f1h);
  for (int l = 0; l < num_levels; ++l) {
    if (!d_f2h[l]) return OFLOW_E_NULL;
    if (level_h[l] < 2 || level_w[l] < 2) return OFLOW_E_TINY;
    a.f2[l] = static_cast<const __half*>(d_f2h[l]);
    a.Hl[l] = level_h[l];
    a.Wl[l] = level_w[l];
  }
  a.coords = d_coords;
  a.out = d_out;
  a.B = B;
  a.C = C;
  a.H = H;
  a.W = W;
  a.segx = (W + kQC - 1) / kQC;
  a.segy = (H + kQR - 1) / kQR;
  const int K = 2 * radius + 1;
  a.cout = num_levels * K * K;
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (radius) {
    case 0: return launch_otf<0>(a, num_levels, s);
    case 1: return launch_otf<1>(a, num_levels, s);
    case 2: return launch_otf<2>(a, num_levels, s);
    case 3: return launch_otf<3>(a, num_levels, s);
    case 4: return launch_otf<4>(a, num_levels, s);
    default: return OFLOW_E_RADIUS;
  }
}
