// EXPERIMENT (not product): the round-1 lookup kernels (git 98a97cd csrc/corr_lookup.hip), exported as r01_* for
// in-process A/B timing against the product kernels (tools/exp/run_lookup_ab.py).
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
// Workgroup = 64 queries x 1 level, 256 threads:
//   phase 0: 64 lanes decode the query centres (floor, weights, output offsets) into LDS;
//   phase 1: all 256 threads gather the 64 patches (consecutive threads read consecutive columns of one
//            patch row: each wave instruction touches ~6 row segments) into LDS, stride (2r+2)^2+1 floats
//            (odd: the compute phase's per-query reads are bank-conflict free);
//   phase 2: each thread emits outputs channel-major so that 64 consecutive lanes write 64 consecutive
//            query pixels of one output channel (256-B coalesced stores of the NCHW output).
#include "../../torch-optical-flow_amd/csrc/oflow_internal.h"

namespace oflow {
namespace {

constexpr int kQ = 64;  // queries per workgroup
constexpr int kThreads = 256;

struct LookupArgs {
  const float* lv[OFLOW_MAX_LEVELS];
  uint8_t* s32;         // S32 output (OUT == 1) and its pixel stride in bytes
  long long s32ps;
  int nqb;              // query blocks
  int nlev;
  int Hl[OFLOW_MAX_LEVELS];
  int Wl[OFLOW_MAX_LEVELS];
  int HB[OFLOW_MAX_LEVELS];  // TILED: ceil(H_l / 4)
  int WB[OFLOW_MAX_LEVELS];  // TILED: ceil(W_l / 8)
  const float* coords;  // (B, 2, N)
  float* out;           // (B, nlev*K*K, N)
  int N;                // query pixels per batch element
  int total;            // B * N
  int cout;             // nlev * K * K
};

// TILED: level l stored as [q][H_l/4][W_l/8][4][8] (corr_pyramid.hip, lvl_off): one 4x8 tile = one 128-B line,
// so a window's row segments share lines with the rows above/below them (fetched once into L2 by this workgroup).
// S32 output (OUT = 1; split-fp16 NHWC feeding the update block's convc1, conv_s32.hip): level l occupies channels
// [l*LS, l*LS + (2r+1)^2), LS = (2r+1)^2 rounded up to 8 (r = 4: 88; 4 levels = 352 = 11 groups), the channels up to
// the next multiple of 8 are written as zeros; convc1's weights are permuted to match on the host. Every 8-channel
// chunk belongs to one (query, level): a thread computes 8 window taps and stores one 16-B hi and one 16-B lo half.
// The 128-B lines straddling two levels are completed by two workgroups: the block -> (query block, level) map puts the
// levels of one query block on blocks b, b+8, b+16, ... (one XCD under round-robin dispatch, speed only) so that the
// XCD's L2 merges the two halves before write-back.
template <int R, bool TILED, int OUT>
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
  const int HB = a.HB[lvl], WB = a.WB[lvl];
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
      {
        if constexpr (TILED)
          v[s] = L[(((size_t)(q0 + q) * HB + (y >> 2)) * WB + (x >> 3)) * 32 + ((y & 3) << 3) + (x & 7)];
        else
          v[s] = L[(size_t)(q0 + q) * (size_t)Hl * Wl + (size_t)y * Wl + x];
      }
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

  if constexpr (OUT == 0) {
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
          const float val = p[0] * w.x + p[1] * w.y + p[PK] * w.z + p[PK + 1] * w.w;
          a.out[off + (long long)c * a.N] = val;
        }
      }
    }
  } else {
    typedef _Float16 half8 __attribute__((ext_vector_type(8)));
    constexpr int KK = K * K, LS = (KK + 7) / 8 * 8, NCH = LS / 8;
    for (int item = threadIdx.x; item < kQ * NCH; item += kThreads) {
      const int q = item / NCH;
      const int ch = item - q * NCH;
      if (sO[q] < 0) continue;
      const float4 w = sW[q];
      half8 hi, lo;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = ch * 8 + e;
        float val = 0.f;
        if (k < KK) {
          const int i = k / K;  // moves x (Q1)
          const int j = k - i * K;
          const float* p = &sP[q * QS + j * PK + i];
          val = p[0] * w.x + p[1] * w.y + p[PK] * w.z + p[PK + 1] * w.w;
        }
        const _Float16 h = static_cast<_Float16>(val);
        hi[e] = h;
        lo[e] = static_cast<_Float16>(val - static_cast<float>(h));
      }
      const int c0 = lvl * LS + ch * 8;
      uint8_t* line = a.s32 + (long long)(q0 + q) * a.s32ps + (c0 >> 5) * 128 + ((c0 & 31) >> 3) * 16;
      *reinterpret_cast<half8*>(line) = hi;
      *reinterpret_cast<half8*>(line + 64) = lo;
    }
  }
}


// NHWC fp32 form for the RAFT forward (oflow_corr_lookup_tiled_nhwc_f32): row q = [level l at l*LS .. l*LS + K^2,
// zeros elsewhere] of row_floats fp32 (the permuted channel order convc1's packed weights expect). Query-major
// workgroups: QB = 64 / nlev queries x all levels, so a workgroup owns QB consecutive output rows = one contiguous
// region, written with consecutive lanes on consecutive floats (full 128-B lines, pads included).
template <int R>
__global__ __launch_bounds__(kThreads) void corr_lookup_nhwc_kernel(LookupArgs a, int QB, int row_floats) {
  constexpr int PK = 2 * R + 2, K = 2 * R + 1, PS = PK * PK, QS = PS + 1;
  constexpr int ITEMS = kQ * PS, PER = (ITEMS + kThreads - 1) / kThreads;
  constexpr int KK = K * K, LS = (KK + 7) / 8 * 8;
  __shared__ float sP[kQ * QS];
  __shared__ int sX[kQ], sY[kQ], sHl[kQ], sWl[kQ], sWB[kQ];
  __shared__ float4 sW[kQ];
  __shared__ const float* sL[kQ];
  const int pairs = QB * a.nlev;
  const int q0 = blockIdx.x * QB;
  if (threadIdx.x < pairs) {
    const int pr = threadIdx.x, lvl = pr / QB, q = q0 + pr - lvl * QB;
    int xs = -(1 << 28), ys = -(1 << 28), hl = 0, wl = 0, wb = 1;
    float4 w = make_float4(0.f, 0.f, 0.f, 0.f);
    const float* base = nullptr;
    if (q < a.total) {
      const int b = q / a.N, pix = q - b * a.N;
      const float inv = 1.0f / static_cast<float>(1 << lvl);  // exact power of two (corr.py:68)
      const float cx = a.coords[(size_t)(2 * b) * a.N + pix] * inv;
      const float cy = a.coords[(size_t)(2 * b + 1) * a.N + pix] * inv;
      if (fabsf(cx) < 4194304.0f && fabsf(cy) < 4194304.0f) {
        const float fx = floorf(cx), fy = floorf(cy);
        const float wx = cx - fx, wy = cy - fy, ex = 1.0f - wx, ey = 1.0f - wy;
        xs = static_cast<int>(fx) - R;
        ys = static_cast<int>(fy) - R;
        w = make_float4(ey * ex, ey * wx, wy * ex, wy * wx);
      }
      // level parameters through a switch: kernel-argument arrays indexed by a lane value would go to scratch
      hl = a.Hl[0]; wl = a.Wl[0]; wb = a.WB[0]; base = a.lv[0];
      for (int l = 1; l < OFLOW_MAX_LEVELS; ++l)
        if (l == lvl) { hl = a.Hl[l]; wl = a.Wl[l]; wb = a.WB[l]; base = a.lv[l]; }
      base += (size_t)q * ((hl + 3) >> 2) * wb * 32;
    }
    sX[pr] = xs;
    sY[pr] = ys;
    sW[pr] = w;
    sHl[pr] = hl;
    sWl[pr] = wl;
    sWB[pr] = wb;
    sL[pr] = base;
  }
  __syncthreads();
  float v[PER];
#pragma unroll
  for (int s = 0; s < PER; ++s) {
    const int item = threadIdx.x + kThreads * s;
    v[s] = 0.0f;
    if (item < pairs * PS) {
      const int pr = item / PS, rem = item - pr * PS;
      const int row = rem / PK, col = rem - row * PK;
      const int y = sY[pr] + row, x = sX[pr] + col;
      if (static_cast<unsigned>(y) < static_cast<unsigned>(sHl[pr]) && static_cast<unsigned>(x) < static_cast<unsigned>(sWl[pr]))
        v[s] = sL[pr][((y >> 2) * sWB[pr] + (x >> 3)) * 32 + ((y & 3) << 3) + (x & 7)];
    }
  }
#pragma unroll
  for (int s = 0; s < PER; ++s) {
    const int item = threadIdx.x + kThreads * s;
    if (item < pairs * PS) {
      const int pr = item / PS;
      sP[pr * QS + (item - pr * PS)] = v[s];
    }
  }
  __syncthreads();
  // a thread owns channels ch = tid, tid + 256, ... of every row: the channel -> (level, window tap) decode is done
  // once, then the QB rows are written with 64 lanes on 64 consecutive floats per store
  const int nq = min(QB, a.total - q0);
  float* dst = a.out + (long long)q0 * row_floats;
  for (int ch = threadIdx.x; ch < row_floats; ch += kThreads) {
    const int lvl = ch / LS, k = ch - lvl * LS;
    const bool real = lvl < a.nlev && k < KK;
    const int i = k / K, j = k - i * K;  // i moves x, j moves y (Q1)
    const int poff = j * PK + i;
    for (int qi = 0; qi < nq; ++qi) {
      float val = 0.f;
      if (real) {
        const int pr = lvl * QB + qi;
        const float* p = &sP[pr * QS + poff];
        const float4 w = sW[pr];
        val = p[0] * w.x + p[1] * w.y + p[PK] * w.z + p[PK + 1] * w.w;
      }
      dst[(long long)qi * row_floats + ch] = val;
    }
  }
}

template <int R>
int launch_lookup(const LookupArgs& a, hipStream_t s, bool tiled, bool s32) {
  dim3 grid(((a.nqb + 7) / 8) * 8 * a.nlev);
  if (s32)
    hipLaunchKernelGGL((corr_lookup_kernel<R, true, 1>), grid, dim3(kThreads), 0, s, a);
  else if (tiled)
    hipLaunchKernelGGL((corr_lookup_kernel<R, true, 0>), grid, dim3(kThreads), 0, s, a);
  else
    hipLaunchKernelGGL((corr_lookup_kernel<R, false, 0>), grid, dim3(kThreads), 0, s, a);
  return launch_status();
}

}  // namespace
}  // namespace oflow

using namespace oflow;

static int corr_lookup_impl(const float* const* d_levels, const int* level_h, const int* level_w, int num_levels,
                            const float* d_coords, int B, int H, int W, int radius, float* d_out, void* stream,
                            bool tiled, uint8_t* s32 = nullptr, long long s32ps = 0) {
  if (!d_levels || !level_h || !level_w || !d_coords || (!d_out && !s32)) return OFLOW_E_NULL;
  if (B <= 0 || H <= 0 || W <= 0) return OFLOW_E_SHAPE;
  if (num_levels < 1 || num_levels > OFLOW_MAX_LEVELS) return OFLOW_E_LEVELS;
  if (radius < 0 || radius > OFLOW_MAX_RADIUS) return OFLOW_E_RADIUS;
  if ((long long)B * H * W >= (1ll << 31) / 64) return OFLOW_E_SHAPE;
  LookupArgs a{};
  for (int l = 0; l < num_levels; ++l) {
    if (!d_levels[l]) return OFLOW_E_NULL;
    // the reference normalises by (W_l - 1), (H_l - 1): a level under 2 px gives inf/NaN there (Q3)
    if (level_h[l] < 2 || level_w[l] < 2) return OFLOW_E_TINY;
    a.lv[l] = d_levels[l];
    a.Hl[l] = level_h[l];
    a.Wl[l] = level_w[l];
    a.HB[l] = (level_h[l] + 3) / 4;
    a.WB[l] = (level_w[l] + 7) / 8;
  }
  const int K = 2 * radius + 1;
  a.coords = d_coords;
  a.out = d_out;
  a.s32 = s32;
  a.s32ps = s32ps;
  a.N = H * W;
  a.total = B * H * W;
  a.cout = num_levels * K * K;
  a.nqb = (a.total + kQ - 1) / kQ;
  a.nlev = num_levels;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool os = s32 != nullptr;
  switch (radius) {
    case 0: return launch_lookup<0>(a, s, tiled, os);
    case 1: return launch_lookup<1>(a, s, tiled, os);
    case 2: return launch_lookup<2>(a, s, tiled, os);
    case 3: return launch_lookup<3>(a, s, tiled, os);
    case 4: return launch_lookup<4>(a, s, tiled, os);
    case 5: return launch_lookup<5>(a, s, tiled, os);
    case 6: return launch_lookup<6>(a, s, tiled, os);
    case 7: return launch_lookup<7>(a, s, tiled, os);
    default: return OFLOW_E_RADIUS;
  }
}

extern "C" int r01_corr_lookup_f32(const float* const* d_levels, const int* level_h, const int* level_w,
                                     int num_levels, const float* d_coords, int B, int H, int W, int radius,
                                     float* d_out, void* stream) {
  return corr_lookup_impl(d_levels, level_h, level_w, num_levels, d_coords, B, H, W, radius, d_out, stream, false);
}

extern "C" int r01_corr_lookup_tiled_f32(const float* const* d_levels, const int* level_h, const int* level_w,
                                           int num_levels, const float* d_coords, int B, int H, int W, int radius,
                                           float* d_out, void* stream) {
  return corr_lookup_impl(d_levels, level_h, level_w, num_levels, d_coords, B, H, W, radius, d_out, stream, true);
}

extern "C" int r01_corr_lookup_tiled_s32(const float* const* d_levels, const int* level_h, const int* level_w,
                                           int num_levels, const float* d_coords, int B, int H, int W, int radius,
                                           void* d_out, long long out_pixel_stride, void* stream) {
  if (!d_out) return OFLOW_E_NULL;
  if (radius < 0 || radius > OFLOW_MAX_RADIUS) return OFLOW_E_RADIUS;
  if (num_levels < 1 || num_levels > OFLOW_MAX_LEVELS) return OFLOW_E_LEVELS;
  const int K = 2 * radius + 1;
  if (out_pixel_stride < (long long)((num_levels * ((K * K + 7) / 8 * 8) + 31) / 32) * 128) return OFLOW_E_SHAPE;
  if ((out_pixel_stride & 127) || ((uintptr_t)d_out & 15)) return OFLOW_E_ALIGN;
  return corr_lookup_impl(d_levels, level_h, level_w, num_levels, d_coords, B, H, W, radius, nullptr, stream, true,
                          static_cast<uint8_t*>(d_out), out_pixel_stride);
}

extern "C" int r01_corr_lookup_tiled_nhwc_f32(const float* const* d_levels, const int* level_h, const int* level_w,
                                                int num_levels, const float* d_coords, int B, int H, int W, int radius,
                                                float* d_out, int row_floats, void* stream) {
  if (!d_levels || !level_h || !level_w || !d_coords || !d_out) return OFLOW_E_NULL;
  if (B <= 0 || H <= 0 || W <= 0) return OFLOW_E_SHAPE;
  if (num_levels < 1 || num_levels > OFLOW_MAX_LEVELS) return OFLOW_E_LEVELS;
  if (radius < 0 || radius > OFLOW_MAX_RADIUS) return OFLOW_E_RADIUS;
  const int K = 2 * radius + 1, LS = (K * K + 7) / 8 * 8;
  if (row_floats < num_levels * LS || (row_floats & 31) || ((uintptr_t)d_out & 15)) return OFLOW_E_SHAPE;
  if ((long long)B * H * W * row_floats >= (1ll << 31)) return OFLOW_E_SHAPE;
  LookupArgs a{};
  for (int l = 0; l < num_levels; ++l) {
    if (!d_levels[l]) return OFLOW_E_NULL;
    if (level_h[l] < 2 || level_w[l] < 2) return OFLOW_E_TINY;  // Q3
    a.lv[l] = d_levels[l];
    a.Hl[l] = level_h[l];
    a.Wl[l] = level_w[l];
    a.HB[l] = (level_h[l] + 3) / 4;
    a.WB[l] = (level_w[l] + 7) / 8;
  }
  a.coords = d_coords;
  a.out = d_out;
  a.N = H * W;
  a.total = B * H * W;
  a.nlev = num_levels;
  const int QB = kQ / num_levels;
  dim3 grid((a.total + QB - 1) / QB);
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (radius) {
#define OFLOW_CASE(RR) \
  case RR: hipLaunchKernelGGL((corr_lookup_nhwc_kernel<RR>), grid, dim3(kThreads), 0, s, a, QB, row_floats); break;
    OFLOW_CASE(0) OFLOW_CASE(1) OFLOW_CASE(2) OFLOW_CASE(3) OFLOW_CASE(4) OFLOW_CASE(5) OFLOW_CASE(6) OFLOW_CASE(7)
#undef OFLOW_CASE
    default: return OFLOW_E_RADIUS;
  }
  return launch_status();
}
