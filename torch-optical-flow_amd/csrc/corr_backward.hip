// Backward of the correlation pyramid and its windowed lookup (gfx950), SURVEY.md §8(f) row 3: what the reference's
// training step (methods/raft/model/raft.py:149-175) differentiates through corr.py:38-87 and utils.py:64-80.
//
//   oflow_corr_lookup_backward_f32 : grad of the (B, L*(2r+1)^2, H, W) lookup output -> += grad of each canonical level
//       (B*H*W, H_l, W_l). The forward (corr_lookup.hip) samples S[j][i] = nw*P[j][i] + ne*P[j][i+1] + sw*P[j+1][i] +
//       se*P[j+1][i+1] over the (2r+2)^2 patch P at the query's level-l window; its transpose in gather form is
//       dP[u][v] = nw*g[u][v] + ne*g[u][v-1] + sw*g[u-1][v] + se*g[u-1][v-1] (g[j][i] = grad of channel i*(2r+1) + j,
//       out-of-range terms dropped), added to the level's row of the query -- every (query, cell) is owned by one
//       thread, so no atomics. Coordinates get no gradient (the reference detaches coords1, raft.py:127).
//   oflow_corr_pyramid_grad_combine_f32 : the levels' gradients folded into level 0 through the floor 2x2 average
//       pools (corr.py:53): g0[q, y, x] += sum_l g_l[q, y >> l, x >> l] / 4^l where (y >> l, x >> l) is inside level l.
//   oflow_corr_fmap_grad_f32 : the two fmap gradients, grad_f1 = f2 . g0^T / sqrt(C) and grad_f2 = f1 . g0 / sqrt(C)
//       (the transpose of corr.py:85's matmul), as batched GEMMs on the fp32 matrix cores (v_mfma_f32_32x32x2_f32:
//       exact fp32 fma chains, fixed k order per output: deterministic).
#include "oflow_internal.h"

namespace oflow {
namespace {

constexpr int kBQ = 64;  // queries per workgroup
constexpr int kBThreads = 256;

template <int R>
__global__ __launch_bounds__(kBThreads) void corr_lookup_backward_kernel(const float* __restrict__ gout,
                                                                         const float* __restrict__ coords, int N,
                                                                         int total, int cout, int lvl, int Hl, int Wl,
                                                                         float* __restrict__ gl) {
  constexpr int K = 2 * R + 1, KK = K * K, PK = 2 * R + 2, PS = PK * PK;
  constexpr int GS = KK + 1;  // odd LDS stride per query
  __shared__ float sG[kBQ * GS];
  __shared__ int sX[kBQ], sY[kBQ];
  __shared__ float4 sW[kBQ];
  const int q0 = blockIdx.x * kBQ;
  const float inv = 1.0f / static_cast<float>(1 << lvl);
  if (threadIdx.x < kBQ) {
    const int q = q0 + threadIdx.x;
    int xs = -(1 << 28), ys = -(1 << 28);
    float4 w = make_float4(0.f, 0.f, 0.f, 0.f);
    if (q < total) {
      const int b = q / N, pix = q - b * N;
      const float cx = coords[(size_t)(2 * b) * N + pix] * inv;
      const float cy = coords[(size_t)(2 * b + 1) * N + pix] * inv;
      if (fabsf(cx) < 4194304.0f && fabsf(cy) < 4194304.0f) {
        const float fx = floorf(cx), fy = floorf(cy);
        const float wx = cx - fx, wy = cy - fy, ex = 1.0f - wx, ey = 1.0f - wy;
        xs = static_cast<int>(fx) - R;
        ys = static_cast<int>(fy) - R;
        w = make_float4(ey * ex, ey * wx, wy * ex, wy * wx);
      }
    }
    sX[threadIdx.x] = xs;
    sY[threadIdx.x] = ys;
    sW[threadIdx.x] = w;
  }
  // the 64 queries' K*K output gradients of this level: lanes along queries (coalesced NCHW rows)
  for (int e = threadIdx.x; e < kBQ * KK; e += kBThreads) {
    const int c = e / kBQ, qi = e - c * kBQ, q = q0 + qi;
    float g = 0.f;
    if (q < total) {
      const int b = q / N, pix = q - b * N;
      g = gout[((size_t)b * cout + lvl * KK + c) * N + pix];
    }
    sG[qi * GS + c] = g;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < kBQ * PS; e += kBThreads) {
    const int qi = e / PS, cell = e - qi * PS;
    const int q = q0 + qi;
    if (q >= total) continue;
    const int u = cell / PK, v = cell - u * PK;  // patch row (y) / column (x)
    const int y = sY[qi] + u, x = sX[qi] + v;
    if (static_cast<unsigned>(y) >= static_cast<unsigned>(Hl) || static_cast<unsigned>(x) >= static_cast<unsigned>(Wl))
      continue;
    const float4 w = sW[qi];
    const float* g = &sG[qi * GS];
    // channel k = i*K + j samples (x: i, y: j); g[j][i] = g[i*K + j]
    float d = 0.f;
    if (u < K && v < K) d += w.x * g[v * K + u];
    if (u < K && v >= 1) d += w.y * g[(v - 1) * K + u];
    if (u >= 1 && v < K) d += w.z * g[v * K + (u - 1)];
    if (u >= 1 && v >= 1) d += w.w * g[(v - 1) * K + (u - 1)];
    float* dst = gl + ((size_t)q * Hl + y) * Wl + x;
    *dst += d;
  }
}

struct LevelTable {
  const float* p[OFLOW_MAX_LEVELS];
  int h[OFLOW_MAX_LEVELS];
  int w[OFLOW_MAX_LEVELS];
};

__global__ __launch_bounds__(256) void pyramid_grad_combine_kernel2(float* __restrict__ g0, LevelTable t, int nlev,
                                                                    long long Q, int H0, int W0) {
  const long long per = (long long)H0 * W0;
  const long long total = Q * per;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const long long q = e / per;
    const int rem = static_cast<int>(e - q * per);
    const int y = rem / W0, x = rem - y * W0;
    float acc = g0[e];
    float scale = 1.0f;
#pragma unroll
    for (int l = 1; l < OFLOW_MAX_LEVELS; ++l) {
      if (l >= nlev) break;
      scale *= 0.25f;  // exact
      const int yl = y >> l, xl = x >> l;
      if (yl < t.h[l] && xl < t.w[l]) acc += t.p[l][(q * t.h[l] + yl) * t.w[l] + xl] * scale;
    }
    g0[e] = acc;
  }
}

// ---- fmap gradients: batched fp32 MFMA GEMM ----
// C[b][m][n] = scale * sum_k A[b][m][k] * Bop[k][n], A row-major [M][K] (K contiguous: a feature map [C][N]); Bop = G^T
// (TB: G [N][K] row-major, K contiguous) or G ([K][N] row-major, N contiguous). Workgroup tile 64 x 64, 4 waves as 2 x 2
// of 32 x 32 (one v_mfma_f32_32x32x2_f32 accumulator each); K in chunks of 16 through LDS as [k][m] / [k][n] (the
// MFMA reads lane l: A[m = l & 31][k = l >> 5], B[k = l >> 5][n = l & 31]: consecutive lanes, consecutive words);
// global -> registers -> LDS one chunk ahead. Ragged M / N / K edges stage zeros.
constexpr int kGT = 64, kGK = 16, kGThreads = 256;
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <bool TB>
__global__ __launch_bounds__(kGThreads) void fmap_grad_gemm_kernel(const float* __restrict__ A, const float* __restrict__ G,
                                                                   float* __restrict__ C, int M, int N, int K, float scale,
                                                                   int tiles_n) {
  __shared__ float sA[2][kGK][kGT + 4];
  __shared__ float sB[2][kGK][kGT + 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int b = blockIdx.y;
  const int m0 = (blockIdx.x / tiles_n) * kGT, n0 = (blockIdx.x % tiles_n) * kGT;
  const float* Ab = A + (size_t)b * M * K;
  const float* Gb = G + (size_t)b * (size_t)N * K;  // G is [N][K] (TB) or [K][N]: N * K elements either way
  // staging: A (and TB's G) as 64 rows x 16 k = 256 float4 along k; non-TB G as 16 k x 64 n = 256 float4 along n
  const int ar = tid >> 2, ac4 = (tid & 3) * 4;
  const int br = tid >> 4, bc4 = (tid & 15) * 4;
  float4 ra, rb;
  auto load = [&](int k0) {
    float av[4], bv[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = k0 + ac4 + e;
      av[e] = (m0 + ar < M && k < K) ? Ab[(size_t)(m0 + ar) * K + k] : 0.f;
      if constexpr (TB) {
        bv[e] = (n0 + ar < N && k < K) ? Gb[(size_t)(n0 + ar) * K + k] : 0.f;
      } else {
        const int n = n0 + bc4 + e, kk = k0 + br;
        bv[e] = (n < N && kk < K) ? Gb[(size_t)kk * N + n] : 0.f;
      }
    }
    ra = make_float4(av[0], av[1], av[2], av[3]);
    rb = make_float4(bv[0], bv[1], bv[2], bv[3]);
  };
  auto store = [&](int buf) {
    sA[buf][ac4 + 0][ar] = ra.x;
    sA[buf][ac4 + 1][ar] = ra.y;
    sA[buf][ac4 + 2][ar] = ra.z;
    sA[buf][ac4 + 3][ar] = ra.w;
    if constexpr (TB) {
      sB[buf][ac4 + 0][ar] = rb.x;
      sB[buf][ac4 + 1][ar] = rb.y;
      sB[buf][ac4 + 2][ar] = rb.z;
      sB[buf][ac4 + 3][ar] = rb.w;
    } else {
      *reinterpret_cast<float4*>(&sB[buf][br][bc4]) = rb;
    }
  };
  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
  const int nk = (K + kGK - 1) / kGK;
  load(0);
  store(0);
  __syncthreads();
  for (int kc = 0; kc < nk; ++kc) {
    const int buf = kc & 1;
    if (kc + 1 < nk) load((kc + 1) * kGK);
#pragma unroll
    for (int kk = 0; kk < kGK; kk += 2) {
      const float av = sA[buf][kk + (lane >> 5)][wm * 32 + (lane & 31)];
      const float bv = sB[buf][kk + (lane >> 5)][wn * 32 + (lane & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
    }
    if (kc + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }
  // C/D map: acc[e] <-> row m = 4 * (lane >> 5) + (e & 3) + 8 * (e >> 2), column n = lane & 31
  float* Cb = C + (size_t)b * M * N;
  const int n = n0 + wn * 32 + (lane & 31);
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int m = m0 + wm * 32 + 4 * (lane >> 5) + (e & 3) + 8 * (e >> 2);
    if (m < M && n < N) Cb[(size_t)m * N + n] = acc[e] * scale;
  }
}

}  // namespace
}  // namespace oflow

using namespace oflow;

extern "C" int oflow_corr_lookup_backward_f32(const float* d_grad_out, const float* d_coords, int B, int H, int W,
                                              int radius, float* const* d_grad_levels, const int* level_h,
                                              const int* level_w, int num_levels, void* stream) {
  if (!d_grad_out || !d_coords || !d_grad_levels || !level_h || !level_w) return OFLOW_E_NULL;
  if (B <= 0 || H <= 0 || W <= 0) return OFLOW_E_SHAPE;
  if (num_levels < 1 || num_levels > OFLOW_MAX_LEVELS) return OFLOW_E_LEVELS;
  if (radius < 0 || radius > OFLOW_MAX_RADIUS) return OFLOW_E_RADIUS;
  const long long total = (long long)B * H * W;
  if (total >= (1ll << 31) / 64) return OFLOW_E_SHAPE;
  const int K = 2 * radius + 1, cout = num_levels * K * K;
  hipStream_t s = static_cast<hipStream_t>(stream);
  dim3 grid(static_cast<unsigned>((total + kBQ - 1) / kBQ));
  for (int l = 0; l < num_levels; ++l) {
    if (!d_grad_levels[l]) return OFLOW_E_NULL;
    if (level_h[l] < 2 || level_w[l] < 2) return OFLOW_E_TINY;
    switch (radius) {
#define OFLOW_CASE(RR)                                                                                                \
  case RR:                                                                                                            \
    hipLaunchKernelGGL((corr_lookup_backward_kernel<RR>), grid, dim3(kBThreads), 0, s, d_grad_out, d_coords, H * W,   \
                       static_cast<int>(total), cout, l, level_h[l], level_w[l], d_grad_levels[l]);                   \
    break;
      OFLOW_CASE(0) OFLOW_CASE(1) OFLOW_CASE(2) OFLOW_CASE(3) OFLOW_CASE(4) OFLOW_CASE(5) OFLOW_CASE(6) OFLOW_CASE(7)
#undef OFLOW_CASE
      default: return OFLOW_E_RADIUS;
    }
    const int st = launch_status();
    if (st) return st;
  }
  return OFLOW_OK;
}

extern "C" int oflow_corr_pyramid_grad_combine_f32(float* const* d_grad_levels, const int* level_h, const int* level_w,
                                                   int num_levels, long long Q, void* stream) {
  if (!d_grad_levels || !level_h || !level_w) return OFLOW_E_NULL;
  if (num_levels < 1 || num_levels > OFLOW_MAX_LEVELS || Q <= 0) return OFLOW_E_SHAPE;
  LevelTable t{};
  for (int l = 0; l < num_levels; ++l) {
    if (!d_grad_levels[l]) return OFLOW_E_NULL;
    t.p[l] = d_grad_levels[l];
    t.h[l] = level_h[l];
    t.w[l] = level_w[l];
  }
  if (num_levels == 1) return OFLOW_OK;
  const long long total = Q * level_h[0] * level_w[0];
  const long long want = (total + 255) / 256;
  dim3 grid(static_cast<unsigned>(want < 1048576 ? want : 1048576));
  hipLaunchKernelGGL(pyramid_grad_combine_kernel2, grid, dim3(256), 0, static_cast<hipStream_t>(stream), d_grad_levels[0], t,
                     num_levels, Q, level_h[0], level_w[0]);
  return launch_status();
}

extern "C" int oflow_corr_fmap_grad_f32(const float* d_fmap1, const float* d_fmap2, const float* d_g0, int B, int C, int N,
                                        float scale, float* d_grad_f1, float* d_grad_f2, void* stream) {
  if (!d_fmap1 || !d_fmap2 || !d_g0 || (!d_grad_f1 && !d_grad_f2)) return OFLOW_E_NULL;
  if (B < 0 || C <= 0 || N < 0) return OFLOW_E_SHAPE;
  if (B == 0 || N == 0) return OFLOW_OK;
  if ((long long)N * N >= (1ll << 40) || B > 65535) return OFLOW_E_SHAPE;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int tm = (C + kGT - 1) / kGT, tn = (N + kGT - 1) / kGT;
  const dim3 grid(tm * tn, B);
  // grad_f1[c][q] = scale * sum_t f2[c][t] g0[q][t]; grad_f2[c][t] = scale * sum_q f1[c][q] g0[q][t]
  if (d_grad_f1) hipLaunchKernelGGL((fmap_grad_gemm_kernel<true>), grid, dim3(kGThreads), 0, s, d_fmap2, d_g0, d_grad_f1, C, N, N, scale, tn);
  if (d_grad_f2) hipLaunchKernelGGL((fmap_grad_gemm_kernel<false>), grid, dim3(kGThreads), 0, s, d_fmap1, d_g0, d_grad_f2, C, N, N, scale, tn);
  return launch_status();
}
