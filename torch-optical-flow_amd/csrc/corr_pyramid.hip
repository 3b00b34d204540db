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

#include "oflow_internal.h"

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
  int HB[4], WB[4];  // tiled layout: tile rows / cols per level (ceil(H_l/4), ceil(W_l/8))
  int nlev;         // levels written by the fused kernel (1..4)
  int tiles_x;      // ceil(W / 32)
  float scale;      // sqrt(C) as torch computes it (float sqrt of float(C))
  float inv_scale;  // exact 1/scale when scale is a power of two (multiply == divide bit-for-bit)
  int scale_pow2;
  int stagger_cycles, stagger_mode;  // experiments only (oflow_exp_set_pyramid_stagger); 0 in the product
};

template <bool VEC>
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
      if constexpr (VEC) {
        *reinterpret_cast<float4*>(&sA[idx >> 5][(idx & 31) << 2]) = a[s];
      } else {
        sA[idx >> 7][idx & 127] = a[s];
      }
    }
#pragma unroll
    for (int s = 0; s < kB; ++s) {
      const int idx = tid + kThreads * s;
      if constexpr (VEC) {
        const int rem = idx & 63;
        *reinterpret_cast<float4*>(&sB[idx >> 6][((rem >> 3) << 5) + ((rem & 7) << 2)]) = b[s];
      } else {
        sB[idx >> 8][idx & 255] = b[s];
      }
    }
  }
};

// Offset of (query q, row y, col x) in level l: canonical (q, H_l, W_l) rows, or TILED [q][H_l/4][W_l/8][4][8]
// (one 4x8 tile = one 128-B line: a (2r+2)^2 lookup window then touches ~7 lines instead of ~13).
template <bool TILED>
__device__ __forceinline__ size_t lvl_off(const PyramidArgs& p, int l, size_t q, int y, int x) {
  if constexpr (TILED) {
    return ((q * p.HB[l] + (y >> 2)) * p.WB[l] + (x >> 3)) * 32 + ((y & 3) << 3) + (x & 7);
  } else {
    return q * (size_t)(p.Hl[l] * p.Wl[l]) + (size_t)y * p.Wl[l] + x;
  }
}

// TILED: a workgroup's first query's base pointer in level l (64-bit, once, in scalar registers) and 32-bit offsets
// from it for its 128 queries (the per-store 64-bit index products were ~180 v_mul_lo_u32 / 86 v_mad_u64_u32 per
// wave in the epilogue)
__device__ __forceinline__ float* lvl_base(const PyramidArgs& p, int l, size_t q0) {
  return p.lv[l] + q0 * (size_t)(p.HB[l] * p.WB[l] * 32);
}
__device__ __forceinline__ int lvl_off32(const PyramidArgs& p, int l, int dq, int y, int x) {
  // 24-bit products (full-rate v_mul_u32_u24): dq < 128, a level's 4x8 tiles per query < 2^16 (checked on the host)
  const unsigned t = __umul24(__umul24(static_cast<unsigned>(dq), static_cast<unsigned>(p.HB[l])) + (y >> 2),
                              static_cast<unsigned>(p.WB[l])) + (x >> 3);
  return static_cast<int>(t * 32u) + ((y & 3) << 3) + (x & 7);
}

// Workgroup -> (target tile, query block) for one image's Mt x Nt GEMM tiles, L2-aware: dispatch is round-robin over
// the 8 XCDs (4 MB L2 each), so each XCD is given a contiguous run of the tile order, and the order walks bands of
// kGM query blocks (A: kGM x 128 KB) across the target tiles (B: 256 KB each) -- the ~64 workgroups an XCD runs at
// once then share about kGM query blocks and 64 / kGM target tiles (~3 MB) instead of streaming all of A or B through
// its L2. Speed only: a bijection on [0, Mt * Nt).
constexpr int kGM = 8;
__device__ __forceinline__ void gemm_tile(int Mt, int Nt, int& tile, int& qblk) {
  const int nwg = Mt * Nt, q8 = nwg / 8, r8 = nwg % 8, id = blockIdx.x, xcd = id % 8;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + id / 8;
  const int band = t / (kGM * Nt), in_band = t - band * (kGM * Nt);
  const int rows = min(kGM, Mt - band * kGM);
  tile = in_band / rows;
  qblk = band * kGM + (in_band - (in_band / rows) * rows);
}

// level-0 staging: tiles 2, 3 of a tile row swap their row pairs (bit 3 of the float offset) so that the 32 lanes of
// one accumulator row write 32 different banks (tiles 0 and 2 are 64 floats apart); 16-B chunks stay whole
__device__ __forceinline__ int l0swz(int e) { return e ^ (((e >> 6) & 1) << 3); }

// Epilogue shared by the fp32 and split-fp16 kernels (both leave the same 32x32 C/D accumulator map): scale by 1/sqrt(C),
// level-0 store, levels 1..3 pooled in registers.
template <bool TILED>
__device__ __forceinline__ void pyramid_epilogue(const PyramidArgs& p, f32x16 (&acc)[kTR], int i0, int ty0, int tx0, int b,
                                                 float* sbuf) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  // ---- epilogue: scale, level-0 store, in-register pooled levels 1..3 ----
  const int tx = lane & 31;
  const int qbase = i0 + wave * 32 + 4 * (lane >> 5);
  const size_t Nn = (size_t)p.N;
#pragma unroll
  for (int n = 0; n < kTR; ++n) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[n][r] = p.scale_pow2 ? acc[n][r] * p.inv_scale : acc[n][r] / p.scale;
  }

  if constexpr (TILED) {
    // level 0 through LDS as whole tiles: a wave's 32 queries x (8 rows x 32 cols) are, per query, 2 tile rows x 4
    // 4x8 tiles = 2 runs of 512 contiguous bytes of the tiled level. Four passes of 8 queries: the accumulators go to
    // the wave's 8 KB of LDS in the tiled byte order, then each lane stores 16-B chunks, a wave instruction writing
    // 2 x 512 B (whole 128-B lines) instead of 8 scattered 32-B row pieces.
    float* sw = sbuf + wave * 2048;
    const int tb = p.WB[0] - (tx0 >> 3);  // tiles of this tile row that exist in the level (>= 1)
    float* const L0b = lvl_base(p, 0, (size_t)b * Nn + i0);
    __syncthreads();  // the main loop's LDS operand reads are done (the scratch aliases them)
    // experiment (mode bit 4): level-0 stores straight from the accumulators, same addresses, unstaged values
    const bool direct = (p.stagger_mode & 16) != 0;
#pragma unroll
    for (int ps = 0; ps < 4; ++ps) {
      if (direct) {
        const int tr = lane >> 5, ch = lane & 31;
        const int y0 = ty0 + 4 * tr;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int i = i0 + wave * 32 + 8 * ps + j;
          const float4 v = make_float4(acc[j][4 * ps], acc[j][4 * ps + 1], acc[j][4 * ps + 2], acc[j][4 * ps + 3]);
          if (i < p.N && (y0 >> 2) < p.HB[0] && (ch >> 3) < tb)
            *reinterpret_cast<float4*>(&L0b[lvl_off32(p, 0, i - i0, y0, tx0) + ch * 4]) = v;
        }
        continue;
      }
#pragma unroll
      for (int n = 0; n < kTR; ++n)
#pragma unroll
        for (int k = 0; k < 4; ++k)  // query wave*32 + 8ps + k + 4hh <- acc[n][4ps + k]
          sw[(k + 4 * (lane >> 5)) * 256 + l0swz((n >> 2) * 128 + (tx >> 3) * 32 + (n & 3) * 8 + (tx & 7))] = acc[n][4 * ps + k];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int tr = lane >> 5, ch = lane & 31;  // tile row, 16-B chunk of its 512 B
      const int y0 = ty0 + 4 * tr;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = i0 + wave * 32 + 8 * ps + j;
        const float4 v = *reinterpret_cast<const float4*>(&sw[j * 256 + l0swz(tr * 128 + ch * 4)]);
        if (i < p.N && (y0 >> 2) < p.HB[0] && (ch >> 3) < tb)
          *reinterpret_cast<float4*>(&L0b[lvl_off32(p, 0, i - i0, y0, tx0) + ch * 4]) = v;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();  // every lane's reads of this pass are done before the next pass overwrites
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  } else {  // level 0: (B*N, H, W)
    float* L0 = p.lv[0];
    const int gx = tx0 + tx;
#pragma unroll
    for (int n = 0; n < kTR; ++n) {
      const int gy = ty0 + n;
      const bool ok = gx < p.W && gy < p.H;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = qbase + (r & 3) + 8 * (r >> 2);
        if (ok && i < p.N) L0[lvl_off<TILED>(p, 0, (size_t)b * Nn + i, gy, gx)] = acc[n][r];
      }
    }
  }
  if (p.nlev < 2 || (p.stagger_mode & 8)) return;  // (mode bit 3, experiment: level 0 alone)

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
        if constexpr (TILED) {
          // staged: this wave's 32 queries x (4 rows x 16 cols) = per query one tile row of 2 tiles (256 B)
          if ((tx & 1) == 0)
            sbuf[wave * 2048 + ((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * 64 + (tx >> 4) * 32 + m * 8 + ((tx >> 1) & 7)] = v1[h][r];
        } else {
          if (ok && i < p.N) p.lv[1][lvl_off<TILED>(p, 1, (size_t)b * Nn + i, y1, x1)] = v1[h][r];
        }
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
        if (!TILED && ok && i < p.N) p.lv[2][lvl_off<TILED>(p, 2, (size_t)b * Nn + i, y2, x2)] = v2[pr][r];
      }
    }
  }
  if constexpr (TILED) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const float* sw = sbuf + wave * 2048;
    const int y1 = ty0 >> 1, tb1 = p.WB[1] - (tx0 >> 4), ch = lane & 15;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ql = 4 * j + (lane >> 4);
      const int i = i0 + wave * 32 + ql;
      const float4 v = *reinterpret_cast<const float4*>(&sw[ql * 64 + ch * 4]);
      if (i < p.N && (y1 >> 2) < p.HB[1] && (ch >> 3) < tb1 && !(p.stagger_mode & 64))
        *reinterpret_cast<float4*>(&lvl_base(p, 1, (size_t)b * Nn + i0)[lvl_off32(p, 1, i - i0, y1, tx0 >> 1) + ch * 4]) = v;
    }
    if (p.nlev < 3) return;
    // levels 2 and 3 through LDS as well: per query, level 2 of this tile is 2 rows x 8 columns = 64 contiguous bytes
    // of one 4x8 tile (ty0 / 4 is even, tx0 / 4 a multiple of 8) and level 3 one row x 4 columns = 16 contiguous bytes,
    // so a wave writes 16-B chunks (3 store instructions) instead of 48 scalar stores of 8 or 16 lanes
    float v3[16];
    if (p.nlev >= 4) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float a0 = v2[0][r], c0 = v2[1][r];
        v3[r] = pool4(a0, swz_xor4(a0), c0, swz_xor4(c0));
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();  // level 1's LDS reads are done before the scratch is reused
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float* s2 = sbuf + wave * 2048;  // level 2: [query 32][row 2][col 8]; level 3 at +512: [query 32][col 4]
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ql = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if ((tx & 3) == 0) {
        s2[ql * 16 + (tx >> 2)] = v2[0][r];
        s2[ql * 16 + 8 + (tx >> 2)] = v2[1][r];
      }
      if (p.nlev >= 4 && (tx & 7) == 0) s2[512 + ql * 4 + (tx >> 3)] = v3[r];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int y2 = ty0 >> 2, x2 = tx0 >> 2;
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int c = lane + 64 * it, ql = c >> 2, part = c & 3;
      const int i = i0 + wave * 32 + ql;
      const float4 v = *reinterpret_cast<const float4*>(&s2[ql * 16 + part * 4]);
      if (i < p.N && (y2 >> 2) < p.HB[2] && (x2 >> 3) < p.WB[2] && !(p.stagger_mode & 64))
        *reinterpret_cast<float4*>(&lvl_base(p, 2, (size_t)b * Nn + i0)[lvl_off32(p, 2, i - i0, y2, x2) + part * 4]) = v;
    }
    if (p.nlev >= 4 && lane < 32 && !(p.stagger_mode & 96)) {
      const int y3 = ty0 >> 3, x3 = tx0 >> 3;
      const int i = i0 + wave * 32 + lane;
      const float4 v = *reinterpret_cast<const float4*>(&s2[512 + lane * 4]);
      if (i < p.N && (y3 >> 2) < p.HB[3] && (x3 >> 3) < p.WB[3])
        *reinterpret_cast<float4*>(&lvl_base(p, 3, (size_t)b * Nn + i0)[lvl_off32(p, 3, i - i0, y3, x3)]) = v;
    }
    return;
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
      if (ok && i < p.N) p.lv[3][lvl_off<TILED>(p, 3, (size_t)b * Nn + i, y3, x3)] = v3;
    }
  }
}

template <bool VEC, bool TILED>
__global__ __launch_bounds__(kThreads, 2) void corr_pyramid_kernel(PyramidArgs p) {
  __shared__ __attribute__((aligned(16))) float sA[2][kBK][kBM];
  __shared__ __attribute__((aligned(16))) float sB[2][kBK][kBN];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  int tile, qblk;
  gemm_tile((p.N + kBM - 1) / kBM, p.tiles_x * ((p.H + kTR - 1) / kTR), tile, qblk);
  const int ty0 = (tile / p.tiles_x) * kTR;
  const int tx0 = (tile % p.tiles_x) * kTC;
  const int i0 = qblk * kBM;
  const int b = blockIdx.z;
  const float* F1 = p.f1 + (size_t)b * p.C * p.N;
  const float* F2 = p.f2 + (size_t)b * p.C * p.N;

  f32x16 acc[kTR];
#pragma unroll
  for (int n = 0; n < kTR; ++n) acc[n] = f32x16{0};

  Stage<VEC> st;
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
#pragma unroll
    for (int kk = 0; kk < kBK; kk += 2) {
      const float av = sA[buf][kk + kl][ml];
#pragma unroll
      for (int n = 0; n < kTR; ++n) {
        const float bv = sB[buf][kk + kl][n * kTC + nl];
        acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[n], 0, 0, 0);
      }
    }
    if (c + 1 < nk) st.store(sA[buf ^ 1], sB[buf ^ 1]);
    __syncthreads();
  }

  pyramid_epilogue<TILED>(p, acc, i0, ty0, tx0, b, &sB[0][0][0]);
}

// ---------------------------------------------------------------------------------------------------------------
// Split-fp16 variant (the RAFT forward's pyramid): both feature maps come as S32 rows (include/oflow.h: per pixel
// C/32 groups of hi[32] | lo[32] fp16, written directly by the feature encoder's last convolution), and every product
// is three v_mfma_f32_32x32x16_f16 (hi*lo + lo*hi + hi*hi, fp32 accumulate; conv_s32.hip's arithmetic: 22-bit operands,
// the lo*lo term below fp32 rounding) instead of fp32 MFMAs at 1/16 of the f16 rate. Same workgroup tile, wave map and
// 32x32 C/D accumulator map as corr_pyramid_kernel, so the fused pooling epilogue is the same code.
// Per k32 group: A = 128 query rows x 128 B, B = 256 target rows x 128 B staged in LDS (16-B slots XOR-swizzled as in
// conv_s32.hip: conflict-free ds_read_b128), the next group register-staged behind the MFMAs; rows outside the image
// load a clamped pixel and stage as zeros.
__device__ __forceinline__ int swz8(int row) { return (row >> 1) & 7; }

template <bool TILED>
__global__ __launch_bounds__(kThreads, 2) void corr_pyramid_s32_kernel(PyramidArgs p, const uint8_t* F1s, const uint8_t* F2s) {
  typedef _Float16 half8 __attribute__((ext_vector_type(8)));
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  constexpr int AP = kBM * 8 / kThreads;  // 16-B chunks per thread: A 4, B 8
  constexpr int BP = kBN * 8 / kThreads;
  __shared__ __attribute__((aligned(16))) uint8_t sA[kBM * 128];
  __shared__ __attribute__((aligned(16))) uint8_t sB[kBN * 128];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (p.stagger_cycles > 0 && blockIdx.z == 0) {  // experiment: start some of the first wave of workgroups late
    const unsigned id = blockIdx.x;
    const bool late = (p.stagger_mode & 3) == 1 ? (id >= 256u && id < 512u) : ((id & 1u) && id < 512u);
    if (late) {
      const unsigned long long t0 = __builtin_amdgcn_s_memtime();
      while (__builtin_amdgcn_s_memtime() - t0 < static_cast<unsigned long long>(p.stagger_cycles)) __builtin_amdgcn_s_sleep(8);
    }
  }
  int tile, qblk;
  gemm_tile((p.N + kBM - 1) / kBM, p.tiles_x * ((p.H + kTR - 1) / kTR), tile, qblk);
  const int ty0 = (tile / p.tiles_x) * kTR;
  const int tx0 = (tile % p.tiles_x) * kTC;
  const int i0 = qblk * kBM;
  const int b = blockIdx.z;
  const int ps = (p.C >> 5) * 128;  // bytes per pixel row
  const int G = (p.stagger_mode & 4) ? 0 : (p.C >> 5);  // experiment (mode bit 2): no main loop, epilogue alone
  const uint8_t* A0 = F1s + (size_t)b * p.N * ps;
  const uint8_t* B0 = F2s + (size_t)b * p.N * ps;

  int aoff[AP], boff[BP];
  unsigned okm = 0u;
#pragma unroll
  for (int s = 0; s < AP; ++s) {
    const int c = tid + kThreads * s, row = c >> 3, sl = c & 7;
    const int i = i0 + row;
    okm |= (i < p.N ? 1u : 0u) << s;
    aoff[s] = min(i, p.N - 1) * ps + sl * 16;
  }
#pragma unroll
  for (int s = 0; s < BP; ++s) {
    const int c = tid + kThreads * s, row = c >> 3, sl = c & 7;
    const int y = ty0 + (row >> 5), x = tx0 + (row & 31);
    const bool ok = y < p.H && x < p.W;
    okm |= (ok ? 1u : 0u) << (AP + s);
    boff[s] = (min(y, p.H - 1) * p.W + min(x, p.W - 1)) * ps + sl * 16;
  }
  u32x4 ra[AP], rb[BP];
  auto load = [&](int g) {
#pragma unroll
    for (int s = 0; s < AP; ++s) ra[s] = *reinterpret_cast<const u32x4*>(A0 + aoff[s] + g * 128);
#pragma unroll
    for (int s = 0; s < BP; ++s) rb[s] = *reinterpret_cast<const u32x4*>(B0 + boff[s] + g * 128);
  };
  auto write = [&]() {
    const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int s = 0; s < AP; ++s) {
      const int c = tid + kThreads * s, row = c >> 3, sl = c & 7;
      *reinterpret_cast<u32x4*>(sA + row * 128 + ((sl ^ swz8(row)) << 4)) = ((okm >> s) & 1u) ? ra[s] : z;
    }
#pragma unroll
    for (int s = 0; s < BP; ++s) {
      const int c = tid + kThreads * s, row = c >> 3, sl = c & 7;
      *reinterpret_cast<u32x4*>(sB + row * 128 + ((sl ^ swz8(row)) << 4)) = ((okm >> (AP + s)) & 1u) ? rb[s] : z;
    }
  };

  f32x16 acc[kTR];
#pragma unroll
  for (int n = 0; n < kTR; ++n) acc[n] = f32x16{0};
  const int r = lane & 31, hh = lane >> 5;
  const int arow = wave * 32 + r;
  load(0);
  for (int g = 0; g < G; ++g) {
    if (g) __syncthreads();  // every wave is done reading group g-1
    write();
    __syncthreads();
    if (g + 1 < G) load(g + 1);
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int chi = 2 * sub + hh, clo = 4 + 2 * sub + hh;
      const half8 ah = *reinterpret_cast<const half8*>(sA + arow * 128 + ((chi ^ swz8(arow)) << 4));
      const half8 al = *reinterpret_cast<const half8*>(sA + arow * 128 + ((clo ^ swz8(arow)) << 4));
#pragma unroll
      for (int n = 0; n < kTR; ++n) {
        const int brow = n * kTC + r;
        const half8 bh = *reinterpret_cast<const half8*>(sB + brow * 128 + ((chi ^ swz8(brow)) << 4));
        const half8 bl = *reinterpret_cast<const half8*>(sB + brow * 128 + ((clo ^ swz8(brow)) << 4));
        acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc[n], 0, 0, 0);
        acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc[n], 0, 0, 0);
        acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[n], 0, 0, 0);
      }
    }
  }
  pyramid_epilogue<TILED>(p, acc, i0, ty0, tx0, b, reinterpret_cast<float*>(sB));
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

// tiled level -> canonical (q, H, W) rows (the reference's corr_pyramid[l] view)
__global__ __launch_bounds__(256) void untile_kernel(const float* __restrict__ in, float* __restrict__ out, long long Q,
                                                      int H, int W, int HB, int WB) {
  const long long total = Q * H * W;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const long long q = t / ((long long)H * W);
    const int rem = (int)(t - q * H * W);
    const int y = rem / W, x = rem - y * W;
    out[t] = in[((q * HB + (y >> 2)) * WB + (x >> 3)) * 32 + ((y & 3) << 3) + (x & 7)];
  }
}

// tiled floor 2x2 pool for levels >= 4
__global__ __launch_bounds__(256) void avgpool2x2_tiled_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                                long long planes, int HBi, int WBi, int Hout, int Wout,
                                                                int HBo, int WBo) {
  const long long total = planes * Hout * Wout;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const long long q = t / ((long long)Hout * Wout);
    const int rem = (int)(t - q * Hout * Wout);
    const int y = rem / Wout, x = rem - y * Wout;
    auto at = [&](int yy, int xx) { return in[((q * HBi + (yy >> 2)) * WBi + (xx >> 3)) * 32 + ((yy & 3) << 3) + (xx & 7)]; };
    out[((q * HBo + (y >> 2)) * WBo + (x >> 3)) * 32 + ((y & 3) << 3) + (x & 7)] =
        pool4(at(2 * y, 2 * x), at(2 * y, 2 * x + 1), at(2 * y + 1, 2 * x), at(2 * y + 1, 2 * x + 1));
  }
}

}  // namespace
}  // namespace oflow

using namespace oflow;

static int g_pyr_stagger_cycles = 0, g_pyr_stagger_mode = 1;
// experiment hook (not part of include/oflow.h): delay part of the split pyramid's first workgroups by `cycles`
// (mode & 3: which ones); ablations: mode & 4 no main loop, & 8 level 0 alone, & 16 level 0 stored unstaged, & 32 no
// level-3 stores, & 64 no level 1-3 stores (pooled and staged all the same)
extern "C" void oflow_exp_set_pyramid_stagger(int cycles, int mode) {
  g_pyr_stagger_cycles = cycles;
  g_pyr_stagger_mode = mode;
}

extern "C" long long oflow_corr_tiled_level_floats(int H_l, int W_l) {
  if (H_l <= 0 || W_l <= 0) return 0;
  return (long long)((H_l + 3) / 4) * ((W_l + 7) / 8) * 32;
}

extern "C" int oflow_corr_untile_f32(const float* d_tiled, float* d_out, long long Q, int H_l, int W_l, void* stream) {
  if (!d_tiled || !d_out) return OFLOW_E_NULL;
  if (Q <= 0 || H_l <= 0 || W_l <= 0) return OFLOW_E_SHAPE;
  const long long total = Q * H_l * W_l;
  const long long want = (total + 255) / 256;
  hipLaunchKernelGGL(untile_kernel, dim3((unsigned)(want < 16384 ? want : 16384)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), d_tiled, d_out, Q, H_l, W_l, (H_l + 3) / 4, (W_l + 7) / 8);
  return launch_status();
}

extern "C" int oflow_corr_pyramid_dims(int H, int W, int num_levels, int* level_h, int* level_w) {
  if (!level_h || !level_w) return OFLOW_E_NULL;
  if (H <= 0 || W <= 0) return OFLOW_E_SHAPE;
  if (num_levels < 1 || num_levels > OFLOW_MAX_LEVELS) return OFLOW_E_LEVELS;
  int h = H, w = W;
  for (int l = 0; l < num_levels; ++l) {
    level_h[l] = h;
    level_w[l] = w;
    h /= 2;
    w /= 2;
  }
  return OFLOW_OK;
}

static int corr_pyramid_impl(const float* d_fmap1, const float* d_fmap2, int B, int C, int H, int W, int num_levels,
                             float* const* d_levels, void* stream, bool tiled) {
  if (!d_fmap1 || !d_fmap2 || !d_levels) return OFLOW_E_NULL;
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0) return OFLOW_E_SHAPE;
  if ((long long)H * W > (1ll << 30)) return OFLOW_E_SHAPE;
  int hl[OFLOW_MAX_LEVELS], wl[OFLOW_MAX_LEVELS];
  int st = oflow_corr_pyramid_dims(H, W, num_levels, hl, wl);
  if (st != OFLOW_OK) return st;
  for (int l = 0; l < num_levels; ++l) {
    if (hl[l] < 1 || wl[l] < 1) return OFLOW_E_TINY;  // avg_pool2d would have no output pixel
    if (!d_levels[l]) return OFLOW_E_NULL;
    if ((reinterpret_cast<uintptr_t>(d_levels[l]) & 3) != 0) return OFLOW_E_ALIGN;
  }
  if (((reinterpret_cast<uintptr_t>(d_fmap1) | reinterpret_cast<uintptr_t>(d_fmap2)) & 3) != 0) return OFLOW_E_ALIGN;
  hipStream_t s = static_cast<hipStream_t>(stream);

  PyramidArgs p{};
  p.f1 = d_fmap1;
  p.f2 = d_fmap2;
  p.C = C;
  p.H = H;
  p.W = W;
  p.N = H * W;
  p.nlev = num_levels < 4 ? num_levels : 4;
  for (int l = 0; l < 4; ++l) {
    p.lv[l] = l < num_levels ? d_levels[l] : nullptr;
    p.Hl[l] = l < num_levels ? hl[l] : 1;
    p.Wl[l] = l < num_levels ? wl[l] : 1;
    p.HB[l] = (p.Hl[l] + 3) / 4;
    p.WB[l] = (p.Wl[l] + 7) / 8;
  }
  if ((long long)p.HB[0] * p.WB[0] >= (1ll << 17)) return OFLOW_E_SHAPE;  // lvl_off32's 24-bit products
  p.tiles_x = (W + kTC - 1) / kTC;
  p.scale = sqrtf(static_cast<float>(C));
  int e2 = 0;
  const float m = frexpf(p.scale, &e2);
  p.scale_pow2 = (m == 0.5f) ? 1 : 0;
  p.inv_scale = p.scale_pow2 ? 1.0f / p.scale : 0.0f;

  const int tiles_y = (H + kTR - 1) / kTR;
  dim3 grid(p.tiles_x * tiles_y * ((p.N + kBM - 1) / kBM), 1, B);
  const bool vec = (W % 4 == 0) &&
                   (((reinterpret_cast<uintptr_t>(d_fmap1) | reinterpret_cast<uintptr_t>(d_fmap2)) & 15) == 0);
  if (vec && tiled) hipLaunchKernelGGL((corr_pyramid_kernel<true, true>), grid, dim3(kThreads), 0, s, p);
  else if (vec) hipLaunchKernelGGL((corr_pyramid_kernel<true, false>), grid, dim3(kThreads), 0, s, p);
  else if (tiled) hipLaunchKernelGGL((corr_pyramid_kernel<false, true>), grid, dim3(kThreads), 0, s, p);
  else hipLaunchKernelGGL((corr_pyramid_kernel<false, false>), grid, dim3(kThreads), 0, s, p);
  st = launch_status();
  if (st != OFLOW_OK) return st;
  for (int l = 4; l < num_levels; ++l) {
    const long long planes = (long long)B * p.N;
    const long long total = planes * hl[l] * wl[l];
    const int blocks = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
    if (tiled)
      hipLaunchKernelGGL(avgpool2x2_tiled_kernel, dim3(blocks), dim3(256), 0, s, d_levels[l - 1], d_levels[l], planes,
                         (hl[l - 1] + 3) / 4, (wl[l - 1] + 7) / 8, hl[l], wl[l], (hl[l] + 3) / 4, (wl[l] + 7) / 8);
    else
      hipLaunchKernelGGL(avgpool2x2_kernel, dim3(blocks), dim3(256), 0, s, d_levels[l - 1], d_levels[l], planes,
                         hl[l - 1], wl[l - 1], hl[l], wl[l]);
    st = launch_status();
    if (st != OFLOW_OK) return st;
  }
  return OFLOW_OK;
}

extern "C" int oflow_corr_pyramid_tiled_s32(const void* d_fmap1_s32, const void* d_fmap2_s32, int B, int C, int H, int W,
                                            int num_levels, float* const* d_levels, void* stream) {
  if (!d_fmap1_s32 || !d_fmap2_s32 || !d_levels) return OFLOW_E_NULL;
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || C % 32) return OFLOW_E_SHAPE;
  if ((long long)H * W * (C / 32) * 128 >= (1ll << 31)) return OFLOW_E_SHAPE;  // 32-bit row offsets per image
  if (((reinterpret_cast<uintptr_t>(d_fmap1_s32) | reinterpret_cast<uintptr_t>(d_fmap2_s32)) & 15) != 0) return OFLOW_E_ALIGN;
  int hl[OFLOW_MAX_LEVELS], wl[OFLOW_MAX_LEVELS];
  int st = oflow_corr_pyramid_dims(H, W, num_levels, hl, wl);
  if (st != OFLOW_OK) return st;
  for (int l = 0; l < num_levels; ++l) {
    if (hl[l] < 1 || wl[l] < 1) return OFLOW_E_TINY;
    if (!d_levels[l]) return OFLOW_E_NULL;
    if ((reinterpret_cast<uintptr_t>(d_levels[l]) & 3) != 0) return OFLOW_E_ALIGN;
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  PyramidArgs p{};
  p.C = C;
  p.H = H;
  p.W = W;
  p.N = H * W;
  p.nlev = num_levels < 4 ? num_levels : 4;
  for (int l = 0; l < 4; ++l) {
    p.lv[l] = l < num_levels ? d_levels[l] : nullptr;
    p.Hl[l] = l < num_levels ? hl[l] : 1;
    p.Wl[l] = l < num_levels ? wl[l] : 1;
    p.HB[l] = (p.Hl[l] + 3) / 4;
    p.WB[l] = (p.Wl[l] + 7) / 8;
  }
  if ((long long)p.HB[0] * p.WB[0] >= (1ll << 17)) return OFLOW_E_SHAPE;  // lvl_off32's 24-bit products
  p.tiles_x = (W + kTC - 1) / kTC;
  p.scale = sqrtf(static_cast<float>(C));
  int e2 = 0;
  p.scale_pow2 = (frexpf(p.scale, &e2) == 0.5f) ? 1 : 0;
  p.inv_scale = p.scale_pow2 ? 1.0f / p.scale : 0.0f;
  p.stagger_cycles = g_pyr_stagger_cycles;
  p.stagger_mode = g_pyr_stagger_mode;
  const dim3 grid(p.tiles_x * ((H + kTR - 1) / kTR) * ((p.N + kBM - 1) / kBM), 1, B);
  hipLaunchKernelGGL((corr_pyramid_s32_kernel<true>), grid, dim3(kThreads), 0, s, p,
                     static_cast<const uint8_t*>(d_fmap1_s32), static_cast<const uint8_t*>(d_fmap2_s32));
  st = launch_status();
  if (st != OFLOW_OK) return st;
  for (int l = 4; l < num_levels; ++l) {
    const long long planes = (long long)B * p.N;
    const long long total = planes * hl[l] * wl[l];
    const int blocks = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
    hipLaunchKernelGGL(avgpool2x2_tiled_kernel, dim3(blocks), dim3(256), 0, s, d_levels[l - 1], d_levels[l], planes,
                       (hl[l - 1] + 3) / 4, (wl[l - 1] + 7) / 8, hl[l], wl[l], (hl[l] + 3) / 4, (wl[l] + 7) / 8);
    st = launch_status();
    if (st != OFLOW_OK) return st;
  }
  return OFLOW_OK;
}

extern "C" int oflow_corr_pyramid_f32(const float* d_fmap1, const float* d_fmap2, int B, int C, int H, int W,
                                      int num_levels, float* const* d_levels, void* stream) {
  return corr_pyramid_impl(d_fmap1, d_fmap2, B, C, H, W, num_levels, d_levels, stream, false);
}

extern "C" int oflow_corr_pyramid_tiled_f32(const float* d_fmap1, const float* d_fmap2, int B, int C, int H, int W,
                                            int num_levels, float* const* d_levels, void* stream) {
  return corr_pyramid_impl(d_fmap1, d_fmap2, B, C, H, W, num_levels, d_levels, stream, true);
}
