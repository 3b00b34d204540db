// Correlation lookup fused into the motion encoder's first convolution (gfx950).
//
// Replaces, in the RAFT forward, `corr = corr_fn(coords1)` (methods/raft/model/raft.py:128 -> corr.py:56-77) followed
// by `F.relu(self.convc1(corr))` (update.py:120-121, a 1x1 conv L*(2r+1)^2 -> 256): the (B, 324, H, W) lookup volume
// never reaches HBM. A workgroup (4 waves, two workgroups per CU) owns 64 query pixels and all 256 output channels and
// runs the levels as a pipeline (details at the kernel): level l+1's window gathers fly while level l's bilinear taps
// (bilinear4: the lookup kernels' arithmetic, bit for bit) become the split-fp16 A operand in LDS and its k32 groups
// run on v_mfma_f32_32x32x16_f16 (hi*lo + lo*hi + hi*hi, fp32 accumulate: conv_s32.hip's arithmetic), with the weights
// streamed from L2 straight into the MFMA operand registers. Epilogue: accumulators -> LDS [pixel][channel] fp32 ->
// per-channel weight scale, bias, ReLU -> S32 store of the 256 output channels (convc2's input).
//
// Weights (include/oflow.h): oflow_conv_s32's packing of convc1 with its input channels regrouped per level (level l's
// tap k at packed channel l*G*32 + k, G = ceil((2r+1)^2 / 32), zeros elsewhere; radius 3: G = 2, radius 4: G = 3),
// stored fragment-major: [k32 group][wave 4][n tile 2][sub 2][hi, lo][lane 64][16 B], lane (r, hh) of wave w and
// n tile nt holding channel w*64 + nt*32 + r, k = 16*sub + 8*hh .. +7 -- the MFMA's B fragment, so that one wave
// instruction loads 1 KB contiguous.
// LDS: patches 44.3 KB + A G*8 KB (epilogue tile overlay 66.5 KB) + 5.5 KB: two workgroups per CU.
#include <type_traits>

#include "oflow_internal.h"

namespace oflow {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kQM = 64;   // query pixels per workgroup
constexpr int kNT = 256;  // threads: 4 waves, one per 64-channel quarter (64 pixels x 64 channels each)
constexpr int kN = 256;   // convc1 output channels (update.py:114)

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }


struct C1Args {
  const float* lv[OFLOW_MAX_LEVELS];  // tiled levels: [query][tiles_l * 32] fp32
  int Hl[OFLOW_MAX_LEVELS];
  int Wl[OFLOW_MAX_LEVELS];
  int WB[OFLOW_MAX_LEVELS];  // ceil(W_l / 8)
  int LF[OFLOW_MAX_LEVELS];  // floats per query of a level
  int nlev;
  const float* coords;  // (B, 2, N)
  int N;                // query pixels per batch element
  int total;            // B * N
  const uint8_t* wf;    // weights, fragment-major [nlev * G][4][2][2][2][64][16 B]
  const float* wsc;     // [256] inverse weight scale
  const float* bias;    // [256] or null
  uint8_t* y;           // S32 destination (8 groups of one pixel from y + P * yps)
  long long yps;
  unsigned long long* stamps;  // diagnostics only (experiment hook): per workgroup 16 clock stamps, or null
};

// exact n / D for 0 <= n < LIM as (n * M) >> 16 with M = ceil(65536 / D) (checked at compile time)
constexpr unsigned magic16(unsigned d) { return (65536u + d - 1) / d; }
constexpr bool magic16_ok(unsigned d, unsigned lim) {
  for (unsigned n = 0; n < lim; ++n)
    if (((n * magic16(d)) >> 16) != n / d) return false;
  return true;
}

// Per workgroup (64 queries, 4 waves; wave w = output channels 64w..64w+63), level by level:
//   * gathers: lane = (query qi of a group of 4, row phase uo, chunk column k); a wave covers its 16 queries in 4
//     groups, rows uo + 4m, so one buffer_load_dwordx4 instruction reads 4 queries x 4 consecutive window rows x 4
//     16-B chunk columns (a chunk never crosses a 4x8 tile: tile rows are 32 B; ~18 lines of 128 B per instruction).
//     A chunk column's byte offset (query base folded in) is formed once per (query, level), or set to a sentinel past
//     the buffer when the column lies outside the level or the window; each row adds its tile-row part (rows m and
//     m+1 are one tile row apart: one add) and takes the sentinel when outside the level. A sentinel load returns
//     zeros without a memory access: the zero padding of Q4.
//   * patches in LDS: row u of query q at sP[q*QS + u*RW], the window's cells at +3 .. +3+PK-1; a chunk's 4 floats go
//     to +3 + 4k + e - dx (dx = x0 & 3) by four ds_write_b32 at immediate offsets from one per-(query, level) base; the
//     chunks of a row cover disjoint cells, the ones outside the window land in the row's slack (RW >= 4*NCH, the
//     last one at most 2 floats into the next row's slack). A level whose width is not a multiple of 4 masks the cells
//     of the one chunk column crossing its right edge (tile padding).
//   * level l+1's gathers are issued right after level l's patches are in LDS, so they fly during level l's taps and
//     MFMAs;
//   * taps: bilinear4 per tap, hi by v_cvt_pk_f16_f32 (two taps, RNE), lo = fp16(v - hi) by v_fma_mixlo/mixhi_f16
//     (split_lo_pair: v - hi is exact in fp32, so the one rounding equals the cvt(sub) pair's);
//   * B (weights, fragment-major: one wave instruction = 1 KB contiguous, L2-resident) goes straight into the MFMA
//     operand registers through a 2-deep ring of k32 groups, each group's load issued right after the MFMAs of the
//     group two before it. Vector-memory loads retire in issue order, so only a group whose load follows the next
//     level's gathers waits for them (G = 3: the level's last group).
// r05 (tools/exp/corr_convc1_variants.hip variant 7, profiles/r05/s13-s14): the r04 kernel's chunk items were decoded
// per item (query, row, chunk) with per-element masks and selects -- ~680 of 1,190 VALU per wave and level; this
// mapping and the mix split take the static VALU count from 4,471 to ~2,590, 37.2 -> 35.8 us per 4-pair launch alone.
// Taps, split values, MFMA order and epilogue are unchanged: bit for bit the r04 kernel's output.
template <int R>
__global__ __launch_bounds__(kNT, 2) void corr_convc1_kernel(C1Args a) {
  constexpr int PK = 2 * R + 2, K = 2 * R + 1, KK = K * K;
  constexpr int NCH = (PK + 6) / 4;
  constexpr int RW = ((4 * NCH > PK + 3) ? 4 * NCH : PK + 3) | 1;
  constexpr int QS = ((PK * RW + 3) | 1);
  constexpr int G = (KK + 31) / 32;
  constexpr int NSLOT = (KK + 7) / 8;
  constexpr int A_BYTES = G * kQM * 128;
  constexpr int P_BYTES = kQM * QS * 4;
  constexpr int TS = kN + 4;
  constexpr int EPI_BYTES = kQM * TS * 4;
  constexpr int MAIN = A_BYTES + P_BYTES;
  constexpr int LDS_BYTES = MAIN > EPI_BYTES ? MAIN : EPI_BYTES;
  constexpr int NS = 4;
  constexpr unsigned SENT = 0x80000000u;  // past any workgroup's buffer (< 2^31 bytes): the load returns zeros
  static_assert(NCH <= 4 && kNT == 4 * kQM, "thread = (query, chunk column)");
  static_assert(3 + 4 * NCH - 1 + (PK - 1) * RW < QS, "a row's chunks stay inside the query's patch");
  __shared__ __attribute__((aligned(16))) uint8_t smem[LDS_BYTES];
  __shared__ float2 sSB[kN];
  __shared__ float2 sC[kQM];
  __shared__ int4 sO[NS][kQM];    // window origin x0, y0, (unused), dx
  __shared__ float4 sW[NS][kQM];  // bilinear weights (nw, ne, sw, se)
  uint8_t* sA = smem;  // the taps (A operand); the patches follow at float offset A_BYTES / 4

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave;
  const int r = lane & 31, hh = lane >> 5;
  const int q0 = blockIdx.x * kQM;
  const int nq = min(kQM, a.total - q0);
  // the gather role: lane = (query of a group of 4 qi, row phase uo, chunk column gk); the wave's 16 queries in 4 groups
  const int gk = lane & 3, uo = (lane >> 2) & 3, qi = lane >> 4;
  constexpr int MR = (PK + 3) / 4;  // rows uo + 4m, m < MR
  int nst = 0;
  auto stamp = [&]() {
    if (a.stamps != nullptr) {
      if (tid == 0) a.stamps[(size_t)blockIdx.x * 16 + nst] = __builtin_amdgcn_s_memtime();
      ++nst;
    }
  };
  stamp();
  auto level = [&](int l, int& Hl, int& Wl, int& WB, int& LF, const float*& base) {
    Hl = a.Hl[0]; Wl = a.Wl[0]; WB = a.WB[0]; LF = a.LF[0]; base = a.lv[0];
#pragma unroll
    for (int j = 1; j < OFLOW_MAX_LEVELS; ++j)
      if (j == l) { Hl = a.Hl[j]; Wl = a.Wl[j]; WB = a.WB[j]; LF = a.LF[j]; base = a.lv[j]; }
  };
  const int qd = tid & (kQM - 1);
  const bool dwave = tid >= (kNT - kQM);
  auto decode = [&](int l, float cx, float cy) {
    int xs, ys;
    float4 w4;
    window_origin(cx, cy, __int_as_float((127 - l) << 23), R, xs, ys, w4);  // 1/2^l exactly (corr.py:68)
    sO[l & (NS - 1)][qd] = make_int4(xs, ys, 0, xs & 3);
    sW[l & (NS - 1)][qd] = w4;
  };

  for (int c = tid; c < kN; c += kNT) sSB[c] = make_float2(a.wsc[c], a.bias ? a.bias[c] : 0.f);
  if (wave < 2) {
    float2 c = make_float2(1e30f, 1e30f);  // past the last query: all-zero window
    if (qd < nq) {
      const int q = q0 + qd;
      const int b = q / a.N, pix = q - b * a.N;
      c = make_float2(a.coords[(size_t)(2 * b) * a.N + pix], a.coords[(size_t)(2 * b + 1) * a.N + pix]);
    }
    if (wave == 0) sC[qd] = c;
    if (wave < a.nlev) decode(wave, c.x, c.y);
  }
  for (int e = tid; e < A_BYTES / 16; e += kNT) reinterpret_cast<u32x4*>(sA)[e] = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();

  u32x4 rv[4][MR];
  auto gather = [&](int l) {
    int Hl, Wl, WB, LF;
    const float* base;
    level(l, Hl, Wl, WB, LF, base);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(base + (size_t)q0 * LF), (short)0, nq * LF * 4, 0x00020000);
    if (NCH == 4 || gk < NCH) {
      const int WB128 = WB * 128;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int gq = wave * 16 + qq * 4 + qi;
        const int4 o = sO[l & (NS - 1)][gq];
        const int xc = o.x - o.w + 4 * gk;
        const bool cv = static_cast<unsigned>(xc) < static_cast<unsigned>(Wl) && 4 * gk < o.w + PK;
        const int y0 = o.y + uo;
        unsigned off = cv ? static_cast<unsigned>(__umul24(gq, LF) * 4 + ((xc >> 3) << 7) + ((xc & 7) << 2)) : SENT;
        off += static_cast<unsigned>(__mul24(y0 >> 2, WB128) + ((y0 & 3) << 5));
#pragma unroll
        for (int m = 0; m < MR; ++m) {
          if (PK % 4 == 0 || m < MR - 1 || uo + 4 * m < PK) {
            const int y = y0 + 4 * m;
            const unsigned o2 = static_cast<unsigned>(y) < static_cast<unsigned>(Hl) ? off + m * WB128 : SENT;
            rv[qq][m] = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(o2), 0, 0);
          }
        }
      }
    }
  };
  const __amdgpu_buffer_rsrc_t rsW =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.wf), (short)0, a.nlev * G * kN * 128, 0x00020000);
  const int wbase = wn * 8192 + lane * 16;
  u32x4 bq[2][8];
  auto load_b = [&](int t, u32x4 (&dst)[8]) {
    const int so = t * (kN * 128);
#pragma unroll
    for (int e = 0; e < 8; ++e) dst[e] = __builtin_amdgcn_raw_buffer_load_b128(rsW, wbase, so + e * 1024, 0);
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nlg = a.nlev * G;
  load_b(0, bq[0]);
  if (nlg > 1) load_b(1, bq[1]);
  gather(0);
  stamp();
  auto body = [&](int l, auto Pc) {
    constexpr int P = decltype(Pc)::value;
    // ---- 1. chunks -> LDS patches ----
    if (NCH == 4 || gk < NCH) {
      int Hl, Wl, WB, LF;
      const float* base;
      level(l, Hl, Wl, WB, LF, base);
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int gq = wave * 16 + qq * 4 + qi;
        const int4 o = sO[l & (NS - 1)][gq];
        int dofs = (A_BYTES / 4) + gq * QS + 3 - o.w + 4 * gk + uo * RW;
        asm volatile("" : "+v"(dofs));  // one base register, immediate offsets
        float* dst = reinterpret_cast<float*>(smem) + dofs;
        const int nv = (Wl & 3) ? Wl - (o.x - o.w + 4 * gk) : 4;  // the chunk column crossing a ragged right edge
#pragma unroll
        for (int m = 0; m < MR; ++m) {
          if (PK % 4 == 0 || m < MR - 1 || uo + 4 * m < PK) {
            const float* fv = reinterpret_cast<const float*>(&rv[qq][m]);
            if (Wl & 3) {
              dst[4 * m * RW + 0] = fv[0];
              dst[4 * m * RW + 1] = nv > 1 ? fv[1] : 0.f;
              dst[4 * m * RW + 2] = nv > 2 ? fv[2] : 0.f;
              dst[4 * m * RW + 3] = nv > 3 ? fv[3] : 0.f;
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e) dst[4 * m * RW + e] = fv[e];
            }
          }
        }
      }
    }
    __syncthreads();
    stamp();
    // ---- 2. next level's gathers, the level after next's windows ----
    if (l + 1 < a.nlev) gather(l + 1);
    if (dwave && l + 2 < a.nlev) decode(l + 2, sC[qd].x, sC[qd].y);
    // ---- 3. bilinear taps -> split-fp16 A operand ----
    {
      const int q = tid & (kQM - 1), set = __builtin_amdgcn_readfirstlane(tid / kQM);
      const float4 w4 = sW[l & (NS - 1)][q];
      int pofs = (A_BYTES / 4) + q * QS + 3;
      asm volatile("" : "+v"(pofs));  // one base register: the taps' offsets fit ds_read2_b32's immediates
      const float* p = reinterpret_cast<const float*>(smem) + pofs;
#pragma unroll
      for (int S = 0; S < NSLOT; ++S) {
        if ((S & 3) != set) continue;
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int k = 8 * S + e;
          v[e] = 0.f;
          if (k < KK) {
            const int i = k / K, j = k - (k / K) * K;
            v[e] = bilinear4(p[j * RW + i], p[j * RW + i + 1], p[(j + 1) * RW + i], p[(j + 1) * RW + i + 1], w4);
          }
          asm volatile("" : "+v"(v[e]));  // the conversions below must not fold the tap's last fma
        }
        range_guard8(v);
        u32x4 hw, lw;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          typedef _Float16 h2 __attribute__((ext_vector_type(2)));
          const h2 hp = {static_cast<_Float16>(v[2 * e]), static_cast<_Float16>(v[2 * e + 1])};
          hw[e] = __builtin_bit_cast(unsigned, hp);
          lw[e] = split_lo_pair(hw[e], v[2 * e], v[2 * e + 1]);
        }
        uint8_t* row = sA + (S >> 2) * (kQM * 128) + q * 128;
        *reinterpret_cast<u32x4*>(row + (((S & 3) ^ swz(q)) << 4)) = hw;
        *reinterpret_cast<u32x4*>(row + (((4 + (S & 3)) ^ swz(q)) << 4)) = lw;
      }
    }
    __syncthreads();
    stamp();
    // ---- 4. the level's MFMAs ----
#pragma unroll
    for (int g = 0; g < G; ++g) {
      u32x4 (&bc)[8] = bq[(P + g) & 1];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        half8 ah[2], al[2];
        const int chi = 2 * sub + hh, clo = 4 + 2 * sub + hh;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const int pr = mt * 32 + r;
          const uint8_t* row = sA + g * (kQM * 128) + pr * 128;
          ah[mt] = *reinterpret_cast<const half8*>(row + ((chi ^ swz(pr)) << 4));
          al[mt] = *reinterpret_cast<const half8*>(row + ((clo ^ swz(pr)) << 4));
        }
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) {
            const half8 bh = __builtin_bit_cast(half8, bc[(nt * 2 + sub) * 2 + 0]);
            const half8 bl = __builtin_bit_cast(half8, bc[(nt * 2 + sub) * 2 + 1]);
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[mt], bl, acc[mt][nt], 0, 0, 0);
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[mt], bh, acc[mt][nt], 0, 0, 0);
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[mt], bh, acc[mt][nt], 0, 0, 0);
          }
      }
      const int t2 = l * G + g + 2;
      if (t2 < nlg) load_b(t2, bc);
    }
    stamp();
  };
  for (int l = 0; l < a.nlev; l += 2) {
    body(l, std::integral_constant<int, 0>{});
    if (l + 1 < a.nlev) body(l + 1, std::integral_constant<int, G & 1>{});
  }

  // ---- epilogue (the r04 kernel's) ----
  __syncthreads();
  float* sT = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int n = wn * 64 + nt * 32 + r;
      const int pbase = mt * 32;
#pragma unroll
      for (int e = 0; e < 16; ++e) sT[(pbase + (e & 3) + 8 * (e >> 2) + 4 * hh) * TS + n] = acc[mt][nt][e];
    }
  const int n = (tid % (kN / 8)) * 8;
  float2 sbv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sbv[j] = sSB[n + j];
  __syncthreads();
#pragma unroll
  for (int it = 0; it < kQM * (kN / 8) / kNT; ++it) {
    const int pl = (tid + it * kNT) / (kN / 8);
    if (pl >= nq) continue;
    const float4 t0 = *reinterpret_cast<const float4*>(&sT[pl * TS + n]);
    const float4 t1 = *reinterpret_cast<const float4*>(&sT[pl * TS + n + 4]);
    const float v[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
    float x[8];
    float mx = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float2 sb = sbv[j];
      x[j] = v[j] * sb.x + sb.y;
      x[j] = x[j] < 0.f ? 0.f : x[j];  // relu (update.py:120); NaN propagates like ATen
      asm volatile("" : "+v"(x[j]));
      mx = fmaxf(mx, x[j]);
    }
    u32x4 hw, lw;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      typedef _Float16 h2 __attribute__((ext_vector_type(2)));
      const h2 hp = {static_cast<_Float16>(x[2 * e]), static_cast<_Float16>(x[2 * e + 1])};
      hw[e] = __builtin_bit_cast(unsigned, hp);
      lw[e] = split_lo_pair(hw[e], x[2 * e], x[2 * e + 1]);
    }
    range_guard(mx);
    uint8_t* line = a.y + (long long)(q0 + pl) * a.yps + (n >> 5) * 128 + ((n & 31) >> 3) * 16;
    *reinterpret_cast<u32x4*>(line) = hw;
    *reinterpret_cast<u32x4*>(line + 64) = lw;
  }
  if (a.stamps != nullptr) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  stamp();
}

unsigned long long* g_convc1_stamps = nullptr;  // diagnostics (experiment hook): per-workgroup clock stamps

}  // namespace
OFLOW_RANGE_FLAG_SETTER(convc1)
}  // namespace oflow

using namespace oflow;

extern "C" int oflow_corr_lookup_convc1_s32(const float* const* d_levels, const int* level_h, const int* level_w,
                                            int num_levels, const float* d_coords, int B, int H, int W, int radius,
                                            const void* d_wpack, const float* d_wscale, const float* d_bias, void* d_y,
                                            long long y_pixel_stride, void* stream) {
  if (!d_levels || !level_h || !level_w || !d_coords || !d_wpack || !d_wscale || !d_y) return OFLOW_E_NULL;
  if (B <= 0 || H <= 0 || W <= 0) return OFLOW_E_SHAPE;
  if (num_levels < 1 || num_levels > OFLOW_MAX_LEVELS) return OFLOW_E_LEVELS;
  if (radius != 3 && radius != 4) return OFLOW_E_RADIUS;
  if ((long long)B * H * W >= (1ll << 31) / 64) return OFLOW_E_SHAPE;
  if ((y_pixel_stride & 127) || ((uintptr_t)d_y & 15) || ((uintptr_t)d_wpack & 15)) return OFLOW_E_ALIGN;
  C1Args a{};
  for (int l = 0; l < num_levels; ++l) {
    if (!d_levels[l]) return OFLOW_E_NULL;
    if (level_h[l] < 2 || level_w[l] < 2) return OFLOW_E_TINY;  // Q3, as the lookup
    a.lv[l] = d_levels[l];
    a.Hl[l] = level_h[l];
    a.Wl[l] = level_w[l];
    a.WB[l] = (level_w[l] + 7) / 8;
    a.LF[l] = ((level_h[l] + 3) / 4) * a.WB[l] * 32;
    if ((long long)kQM * a.LF[l] * 4 >= (1ll << 31)) return OFLOW_E_SHAPE;  // a workgroup's window reads: 32-bit offsets
  }
  a.nlev = num_levels;
  a.coords = d_coords;
  a.N = H * W;
  a.total = B * H * W;
  a.wf = static_cast<const uint8_t*>(d_wpack);
  a.wsc = d_wscale;
  a.bias = d_bias;
  a.y = static_cast<uint8_t*>(d_y);
  a.yps = y_pixel_stride;
  const dim3 grid((a.total + kQM - 1) / kQM);
  hipStream_t s = static_cast<hipStream_t>(stream);
  a.stamps = g_convc1_stamps;
  if (radius == 4)
    hipLaunchKernelGGL((corr_convc1_kernel<4>), grid, dim3(kNT), 0, s, a);
  else
    hipLaunchKernelGGL((corr_convc1_kernel<3>), grid, dim3(kNT), 0, s, a);
  return launch_status();
}

// experiment hook (not part of include/oflow.h): a device buffer of 16 clock stamps per workgroup, or null
extern "C" void oflow_exp_set_convc1_stamps(void* stamps) {
  oflow::g_convc1_stamps = static_cast<unsigned long long*>(stamps);
}
