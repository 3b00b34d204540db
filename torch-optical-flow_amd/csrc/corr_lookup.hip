// Multi-level windowed bilinear lookup into the correlation pyramid (gfx950).
//
// Replaces methods/raft/model/corr.py:56-77 (CorrBlock.__call__) and utils.py:64-80 (bilinear_sampler ->
// F.grid_sample(align_corners=True, padding_mode='zeros')), including the window channel order of the
// reference (Q1): channel l*(2r+1)^2 + i*(2r+1) + j samples (x/2^l + i - r, y/2^l + j - r).
//
// Pixel-space formulation: for one (query, level) every window tap shares the fractional
// offset (wx, wy) of the centre, so the lookup is a (2r+2)^2 patch gather plus one fixed 2x2 stencil. The
// normalise -> unnormalise round trip of the reference (x -> 2x/(W-1)-1 -> x) is skipped; it only adds
// ulp-level noise (<= 2.2e-5 abs measured).
//
// Two kernels: corr_lookup_tiled_kernel over the tiled pyramid CorrBlock keeps (NCHW for CorrBlock.__call__, NHWC rows
// for the RAFT forward's convc1), and corr_lookup_kernel over canonical (B*H*W, H_l, W_l) rows (the reference's
// corr_pyramid list, once it has been materialised or assigned).
#include "oflow_internal.h"

namespace oflow {
namespace {

constexpr int kQ = 64;  // queries per workgroup (canonical kernel)
constexpr int kThreads = 256;

struct LookupArgs {
  const float* lv[OFLOW_MAX_LEVELS];
  int nqb;              // query blocks
  int nlev;
  int Hl[OFLOW_MAX_LEVELS];
  int Wl[OFLOW_MAX_LEVELS];
  const float* coords;  // (B, 2, N)
  float* out;           // (B, nlev*K*K, N)
  int N;                // query pixels per batch element
  int total;            // B * N
  int cout;             // nlev * K * K
};

// Canonical rows. Workgroup = 64 queries x 1 level, 256 threads: 64 lanes decode the centres into LDS; all threads
// gather the 64 patches into LDS (odd per-query stride: conflict-free compute reads); 64 consecutive lanes write 64
// consecutive query pixels of one output channel.
template <int R>
__global__ __launch_bounds__(kThreads) void corr_lookup_kernel(LookupArgs a) {
  constexpr int PK = 2 * R + 2;   // patch side
  constexpr int K = 2 * R + 1;    // window side
  constexpr int PS = PK * PK;     // patch size
  constexpr int QS = PS + 1;      // LDS stride per query (odd)
  constexpr int ITEMS = kQ * PS;
  constexpr int PER = (ITEMS + kThreads - 1) / kThreads;
  constexpr int OUTS = kQ * K * K;
  constexpr int PERO = (OUTS + kThreads - 1) / kThreads;

  __shared__ float sP[kQ * QS];
  __shared__ int sX[kQ], sY[kQ];
  __shared__ float4 sW[kQ];
  __shared__ long long sO[kQ];

  const int grp = blockIdx.x / (8 * a.nlev), rem = blockIdx.x - grp * 8 * a.nlev;
  const int lvl = rem >> 3;
  const int qb = grp * 8 + (rem & 7);
  if (qb >= a.nqb) return;
  const int q0 = qb * kQ;
  const int Hl = a.Hl[lvl], Wl = a.Wl[lvl];
  const float* __restrict__ L = a.lv[lvl];
  const float inv = 1.0f / static_cast<float>(1 << lvl);  // exact power of two (corr.py:68)

  if (threadIdx.x < kQ) {
    const int q = q0 + threadIdx.x;
    int xs = -(1 << 28), ys = -(1 << 28);
    float4 w = make_float4(0.f, 0.f, 0.f, 0.f);
    long long off = -1;
    if (q < a.total) {
      const int b = q / a.N;
      const int pix = q - b * a.N;
      const float cx = a.coords[(size_t)(2 * b) * a.N + pix] * inv;
      const float cy = a.coords[(size_t)(2 * b + 1) * a.N + pix] * inv;
      // |c| >= 2^22 (or NaN/inf) puts every tap far outside any level: all-zero window.
      if (fabsf(cx) < 4194304.0f && fabsf(cy) < 4194304.0f) {
        const float fx = floorf(cx), fy = floorf(cy);
        const float wx = cx - fx, wy = cy - fy;  // exact
        const float ex = 1.0f - wx, ey = 1.0f - wy;
        xs = static_cast<int>(fx) - R;
        ys = static_cast<int>(fy) - R;
        w = make_float4(ey * ex, ey * wx, wy * ex, wy * wx);  // nw, ne, sw, se (grid_sample CPU weights)
      }
      off = (long long)b * a.cout * a.N + (long long)lvl * K * K * a.N + pix;
    }
    sX[threadIdx.x] = xs;
    sY[threadIdx.x] = ys;
    sW[threadIdx.x] = w;
    sO[threadIdx.x] = off;
  }
  __syncthreads();

  float v[PER];
#pragma unroll
  for (int s = 0; s < PER; ++s) {
    const int item = threadIdx.x + kThreads * s;
    v[s] = 0.0f;
    if (item < ITEMS) {
      const int q = item / PS;
      const int rem = item - q * PS;
      const int row = rem / PK;
      const int col = rem - row * PK;
      const int y = sY[q] + row, x = sX[q] + col;
      if (q0 + q < a.total && static_cast<unsigned>(y) < static_cast<unsigned>(Hl) &&
          static_cast<unsigned>(x) < static_cast<unsigned>(Wl))
        v[s] = L[(size_t)(q0 + q) * (size_t)Hl * Wl + (size_t)y * Wl + x];
    }
  }
#pragma unroll
  for (int s = 0; s < PER; ++s) {
    const int item = threadIdx.x + kThreads * s;
    if (item < ITEMS) {
      const int q = item / PS;
      sP[q * QS + (item - q * PS)] = v[s];
    }
  }
  __syncthreads();

#pragma unroll
  for (int s = 0; s < PERO; ++s) {
    const int o = threadIdx.x + kThreads * s;
    if (o < OUTS) {
      const int c = o / kQ;
      const int q = o - c * kQ;
      const long long off = sO[q];
      if (off >= 0) {
        const int i = c / K;           // moves x
        const int j = c - i * K;       // moves y
        const float* p = &sP[q * QS + j * PK + i];
        const float4 w = sW[q];
        a.out[off + (long long)c * a.N] = bilinear4(p[0], p[1], p[PK], p[PK + 1], w);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------------------------
// Lookup over the tiled pyramid ([q][H_l/4][W_l/8][4][8] fp32, corr_pyramid.hip lvl_off): a 4x8 tile is one 128-B
// line, so a (2r+2)^2 window touches ~7 lines (r = 4) instead of ~13 in row-major storage.
//
// Workgroup = 64 consecutive queries x ONE level, 256 threads (levels never mix inside a workgroup: every gather
// address uses the same level geometry). Block g -> (query block, level) puts the L levels of one query block on
// blocks g, g + 8, g + 16, ... (one XCD under round-robin dispatch; speed only), so the NHWC row segments that share a
// 128-B line are merged in that XCD's L2.
// 1. threads < 64 decode their query's window origin and bilinear weights;
// 2. all threads gather the 64 patches: consecutive threads take consecutive columns of one patch row, so a wave
//    instruction covers ~6 patch rows of ~1 patch, a handful of lines (scalar 4-B loads, 25 in flight per thread);
//    the patches go to LDS with an odd per-query stride;
// 3. thread = (query, window column i): columns i and i + 1 of the patch (conflict-free: consecutive queries are an
//    odd stride apart) -> the 2r+1 outputs of that column, in registers;
// 4. the outputs become an LDS image over the dead patches ([k][64 queries] for NCHW, [query][K*K] for NHWC; both
//    written conflict-free) and are stored coalesced: NCHW 256-B channel runs; NHWC the level's K*K-float segment of
//    each query's row (row = the reference's channel order l*K*K + k, i.e. corr.permute(0, 2, 3, 1)).
// (Measured alternatives, tools/exp/run_lookup_ab.py: LDS-DMA segment gathers, persistent double-buffered waves and
// 16-B piece gathers with 8 threads per query were all slower on Sintel x8)
// Bilinear arithmetic: bilinear4, shared with the canonical kernel (bit-identical results).
// ---------------------------------------------------------------------------------------------------------------
struct TiledArgs {
  const float* lv[OFLOW_MAX_LEVELS];
  int Hl[OFLOW_MAX_LEVELS];
  int Wl[OFLOW_MAX_LEVELS];
  int WB[OFLOW_MAX_LEVELS];  // ceil(W_l / 8)
  int LF[OFLOW_MAX_LEVELS];  // floats per query of a level (tiles * 32)
  int nlev;
  int nqb;              // 64-query blocks
  const float* coords;  // (B, 2, N)
  float* out;
  int N;       // query pixels per batch element
  int total;   // B * N
  int row;     // NHWC row pitch (floats)
};

template <int R, int OUT, bool BUF>
__global__ __launch_bounds__(kThreads) void corr_lookup_tiled_kernel(TiledArgs a) {
  constexpr int PK = 2 * R + 2, K = 2 * R + 1, KK = K * K, PS = PK * PK;
  constexpr int QS = PS + 1;  // odd query stride
  constexpr int ITEMS = kQ * PS, PER = (ITEMS + kThreads - 1) / kThreads;
  constexpr int CI = (kQ * K + kThreads - 1) / kThreads;  // (query, column) items per thread
  constexpr int IMG = kQ * KK;
  static_assert(IMG <= kQ * QS, "output image must fit over the patches");
  __shared__ float sP[kQ * QS];
  __shared__ int sX[kQ], sY[kQ];
  __shared__ float4 sW[kQ];

  // block -> (query block, level): levels of a query block 8 blocks apart
  const int L = a.nlev;
  const int grp = blockIdx.x / (8 * L), rem = blockIdx.x - grp * 8 * L;
  const int lvl = rem >> 3;
  const int qb = grp * 8 + (rem & 7);
  if (qb >= a.nqb) return;
  const int q0 = qb * kQ;
  const int nq = min(kQ, a.total - q0);
  int Hl = a.Hl[0], Wl = a.Wl[0], WB = a.WB[0], LF = a.LF[0];
  const float* base = a.lv[0];
#pragma unroll
  for (int j = 1; j < OFLOW_MAX_LEVELS; ++j)
    if (j == lvl) { Hl = a.Hl[j]; Wl = a.Wl[j]; WB = a.WB[j]; LF = a.LF[j]; base = a.lv[j]; }
  const int tid = threadIdx.x;

  // ---- 1. decode ----
  if (tid < kQ) {
    int xs = -(1 << 28), ys = -(1 << 28);
    float4 w = make_float4(0.f, 0.f, 0.f, 0.f);
    if (tid < nq) {
      const int q = q0 + tid;
      const int b = q / a.N, pix = q - b * a.N;
      const float inv = 1.0f / static_cast<float>(1 << lvl);  // exact power of two (corr.py:68)
      const float cx = a.coords[(size_t)(2 * b) * a.N + pix] * inv;
      const float cy = a.coords[(size_t)(2 * b + 1) * a.N + pix] * inv;
      // |c| >= 2^22 (or NaN/inf) puts every tap far outside any level: all-zero window
      if (fabsf(cx) < 4194304.0f && fabsf(cy) < 4194304.0f) {
        const float fx = floorf(cx), fy = floorf(cy);
        const float wx = cx - fx, wy = cy - fy;  // exact
        const float ex = 1.0f - wx, ey = 1.0f - wy;
        xs = static_cast<int>(fx) - R;
        ys = static_cast<int>(fy) - R;
        w = make_float4(ey * ex, ey * wx, wy * ex, wy * wx);  // nw, ne, sw, se (grid_sample CPU weights)
      }
    }
    sX[tid] = xs;
    sY[tid] = ys;
    sW[tid] = w;
  }
  __syncthreads();

  // ---- 2. gather ----
  // BUF (r06, launch_tiled): every load unconditional -- a buffer load whose offset is a sentinel past this block's
  // window reads for taps outside the level (and items past the last query) returns 0 without a memory access --
  // instead of one exec-masked branch per load
  const float* __restrict__ Lq = base + (size_t)q0 * LF;
  float v[PER];
  if constexpr (!BUF) {
#pragma unroll
  for (int s = 0; s < PER; ++s) {
    const int item = tid + kThreads * s;
    v[s] = 0.0f;
    if (item < ITEMS) {
      const int q = item / PS;
      const int rm = item - q * PS;
      const int u = rm / PK, c = rm - u * PK;
      const int y = sY[q] + u, x = sX[q] + c;
      if (q < nq && static_cast<unsigned>(y) < static_cast<unsigned>(Hl) && static_cast<unsigned>(x) < static_cast<unsigned>(Wl))
        v[s] = Lq[(size_t)q * LF + ((y >> 2) * WB + (x >> 3)) * 32 + ((y & 3) << 3) + (x & 7)];
    }
  }
  } else {
  const __amdgpu_buffer_rsrc_t rsL =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Lq), (short)0, nq * LF * 4, 0x00020000);
#pragma unroll
  for (int s = 0; s < PER; ++s) {
    const int item = min(tid + kThreads * s, ITEMS - 1);  // (items past ITEMS: loaded, never stored)
    const int q = item / PS;
    const int rm = item - q * PS;
    const int u = rm / PK, c = rm - u * PK;
    const int y = sY[q] + u, x = sX[q] + c;
    const bool in = q < nq && static_cast<unsigned>(y) < static_cast<unsigned>(Hl) &&
                    static_cast<unsigned>(x) < static_cast<unsigned>(Wl);
    const unsigned off = in ? static_cast<unsigned>((q * LF + ((y >> 2) * WB + (x >> 3)) * 32 + ((y & 3) << 3) + (x & 7)) * 4)
                            : 0x80000000u;
    v[s] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsL, static_cast<int>(off), 0, 0));
  }
  }
#pragma unroll
  for (int s = 0; s < PER; ++s) {
    const int item = tid + kThreads * s;
    if (item < ITEMS) {
      const int q = item / PS;
      sP[q * QS + (item - q * PS)] = v[s];
    }
  }
  __syncthreads();

  // ---- 3. thread = (query, column i) -> K outputs ----
  float res[CI][K];
#pragma unroll
  for (int s = 0; s < CI; ++s) {
    const int it = tid + kThreads * s;
    const int q = it & (kQ - 1), i = it / kQ;
    if (it < kQ * K) {
      const float* p = &sP[q * QS + i];
      const float4 w = sW[q];
      float c0[PK], c1[PK];
#pragma unroll
      for (int u = 0; u < PK; ++u) {
        c0[u] = p[u * PK];
        c1[u] = p[u * PK + 1];
      }
#pragma unroll
      for (int j = 0; j < K; ++j) res[s][j] = bilinear4(c0[j], c1[j], c0[j + 1], c1[j + 1], w);
    }
  }
  __syncthreads();  // every patch read has returned: the buffer becomes the output image
#pragma unroll
  for (int s = 0; s < CI; ++s) {
    const int it = tid + kThreads * s;
    const int q = it & (kQ - 1), i = it / kQ;
    if (it < kQ * K) {
#pragma unroll
      for (int j = 0; j < K; ++j) {
        if constexpr (OUT == 0) sP[(i * K + j) * kQ + q] = res[s][j];  // [k][64 queries]
        else sP[q * KK + i * K + j] = res[s][j];                       // [query][K*K]
      }
    }
  }
  __syncthreads();

  // ---- 4. coalesced stores ----
  if constexpr (OUT == 0) {
    const int ql = tid & (kQ - 1);  // fixed per thread: e += 256 keeps e % 64
    if (ql < nq) {
      const int q = q0 + ql;
      const int b = q / a.N, pix = q - b * a.N;
      float* dst = a.out + ((size_t)b * L * KK + (size_t)lvl * KK) * a.N + pix;
      for (int e = tid; e < IMG; e += kThreads) dst[(size_t)(e / kQ) * a.N] = sP[e];
    }
  } else {
    float* dst = a.out + (size_t)q0 * a.row + (size_t)lvl * KK;
    int ql = tid / KK, k = tid - ql * KK;
    constexpr int DQ = kThreads / KK, DK = kThreads - DQ * KK;  // e += 256 -> (ql, k) += (DQ, DK) with carry
    for (int e = tid; e < nq * KK; e += kThreads) {
      dst[(size_t)ql * a.row + k] = sP[e];
      ql += DQ;
      k += DK;
      if (k >= KK) { k -= KK; ++ql; }
    }
  }
}

template <int R>
int launch_lookup(const LookupArgs& a, hipStream_t s) {
  dim3 grid(((a.nqb + 7) / 8) * 8 * a.nlev);
  hipLaunchKernelGGL((corr_lookup_kernel<R>), grid, dim3(kThreads), 0, s, a);
  return launch_status();
}

// The unconditional buffer-load gathers (BUF) wherever a block's window reads fit 32-bit byte offsets (every
// practical level: LF < 2^23 floats). r06 in-process A/B at the bench workload (tools/exp/run_lookup_buf_ab.py,
// profiles/r06/r6s16_lookup_ab.log): cold 44.42 -> 41.79 us, hot 39.08 -> 38.15, bit-identical.
template <int R>
int launch_tiled(const TiledArgs& a, int out_form, hipStream_t s) {
  const dim3 grid(((a.nqb + 7) / 8) * 8 * a.nlev);
  bool buf = true;
  for (int l = 0; l < a.nlev; ++l) buf = buf && (long long)kQ * a.LF[l] * 4 < (1ll << 31);
  if (buf) {
    if (out_form == 0)
      hipLaunchKernelGGL((corr_lookup_tiled_kernel<R, 0, true>), grid, dim3(kThreads), 0, s, a);
    else
      hipLaunchKernelGGL((corr_lookup_tiled_kernel<R, 1, true>), grid, dim3(kThreads), 0, s, a);
  } else {
    if (out_form == 0)
      hipLaunchKernelGGL((corr_lookup_tiled_kernel<R, 0, false>), grid, dim3(kThreads), 0, s, a);
    else
      hipLaunchKernelGGL((corr_lookup_tiled_kernel<R, 1, false>), grid, dim3(kThreads), 0, s, a);
  }
  return launch_status();
}

}  // namespace
}  // namespace oflow

using namespace oflow;

static int lookup_common_checks(const float* const* d_levels, const int* level_h, const int* level_w, int num_levels,
                                const float* d_coords, int B, int H, int W, int radius, const float* d_out) {
  if (!d_levels || !level_h || !level_w || !d_coords || !d_out) return OFLOW_E_NULL;
  if (B <= 0 || H <= 0 || W <= 0) return OFLOW_E_SHAPE;
  if (num_levels < 1 || num_levels > OFLOW_MAX_LEVELS) return OFLOW_E_LEVELS;
  if (radius < 0 || radius > OFLOW_MAX_RADIUS) return OFLOW_E_RADIUS;
  if ((long long)B * H * W >= (1ll << 31) / 64) return OFLOW_E_SHAPE;
  for (int l = 0; l < num_levels; ++l) {
    if (!d_levels[l]) return OFLOW_E_NULL;
    // the reference normalises by (W_l - 1), (H_l - 1): a level under 2 px gives inf/NaN there (Q3)
    if (level_h[l] < 2 || level_w[l] < 2) return OFLOW_E_TINY;
  }
  return OFLOW_OK;
}

extern "C" int oflow_corr_lookup_f32(const float* const* d_levels, const int* level_h, const int* level_w,
                                     int num_levels, const float* d_coords, int B, int H, int W, int radius,
                                     float* d_out, void* stream) {
  const int st = lookup_common_checks(d_levels, level_h, level_w, num_levels, d_coords, B, H, W, radius, d_out);
  if (st != OFLOW_OK) return st;
  LookupArgs a{};
  for (int l = 0; l < num_levels; ++l) {
    a.lv[l] = d_levels[l];
    a.Hl[l] = level_h[l];
    a.Wl[l] = level_w[l];
  }
  const int K = 2 * radius + 1;
  a.coords = d_coords;
  a.out = d_out;
  a.N = H * W;
  a.total = B * H * W;
  a.cout = num_levels * K * K;
  a.nqb = (a.total + kQ - 1) / kQ;
  a.nlev = num_levels;
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (radius) {
    case 0: return launch_lookup<0>(a, s);
    case 1: return launch_lookup<1>(a, s);
    case 2: return launch_lookup<2>(a, s);
    case 3: return launch_lookup<3>(a, s);
    case 4: return launch_lookup<4>(a, s);
    case 5: return launch_lookup<5>(a, s);
    case 6: return launch_lookup<6>(a, s);
    case 7: return launch_lookup<7>(a, s);
    default: return OFLOW_E_RADIUS;
  }
}

static int tiled_lookup(const float* const* d_levels, const int* level_h, const int* level_w, int num_levels,
                        const float* d_coords, int B, int H, int W, int radius, float* d_out, int out_form, int row,
                        void* stream) {
  const int st = lookup_common_checks(d_levels, level_h, level_w, num_levels, d_coords, B, H, W, radius, d_out);
  if (st != OFLOW_OK) return st;
  TiledArgs a{};
  for (int l = 0; l < num_levels; ++l) {
    a.lv[l] = d_levels[l];
    a.Hl[l] = level_h[l];
    a.Wl[l] = level_w[l];
    a.WB[l] = (level_w[l] + 7) / 8;
    a.LF[l] = ((level_h[l] + 3) / 4) * a.WB[l] * 32;
  }
  a.nlev = num_levels;
  a.coords = d_coords;
  a.out = d_out;
  a.N = H * W;
  a.total = B * H * W;
  a.nqb = (a.total + kQ - 1) / kQ;
  a.row = row;
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (radius) {
    case 0: return launch_tiled<0>(a, out_form, s);
    case 1: return launch_tiled<1>(a, out_form, s);
    case 2: return launch_tiled<2>(a, out_form, s);
    case 3: return launch_tiled<3>(a, out_form, s);
    case 4: return launch_tiled<4>(a, out_form, s);
    case 5: return launch_tiled<5>(a, out_form, s);
    case 6: return launch_tiled<6>(a, out_form, s);
    case 7: return launch_tiled<7>(a, out_form, s);
    default: return OFLOW_E_RADIUS;
  }
}

extern "C" int oflow_corr_lookup_tiled_f32(const float* const* d_levels, const int* level_h, const int* level_w,
                                           int num_levels, const float* d_coords, int B, int H, int W, int radius,
                                           float* d_out, void* stream) {
  return tiled_lookup(d_levels, level_h, level_w, num_levels, d_coords, B, H, W, radius, d_out, 0, 0, stream);
}

extern "C" int oflow_corr_lookup_tiled_nhwc_f32(const float* const* d_levels, const int* level_h, const int* level_w,
                                                int num_levels, const float* d_coords, int B, int H, int W, int radius,
                                                float* d_out, int row_floats, void* stream) {
  const int K = 2 * radius + 1;
  if (row_floats < num_levels * K * K) return OFLOW_E_SHAPE;
  if ((long long)B * H * W * row_floats >= (1ll << 31)) return OFLOW_E_SHAPE;
  if (((uintptr_t)d_out & 15) != 0) return OFLOW_E_ALIGN;
  return tiled_lookup(d_levels, level_h, level_w, num_levels, d_coords, B, H, W, radius, d_out, 1, row_floats, stream);
}
