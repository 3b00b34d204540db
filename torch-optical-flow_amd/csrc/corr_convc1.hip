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
//   * gathers: a window row of PK cells starting at x0 lies inside NCH 16-B aligned chunks from xa = x0 & ~3 (a chunk
//     never crosses a 4x8 tile: tile rows are 32 B), one buffer_load_dwordx4 per chunk; per-(query, level) window
//     origin and row / column validity masks come from LDS (decoded two levels ahead), offsets are branch-free (a chunk
//     not needed loads the workgroup's first 16 B);
//   * patches in LDS: row u of query q at sP[q*QS + u*RW], the window's cells at +3 .. +3+PK-1; a chunk's 4 floats go
//     to +3 + 4k + e - dx (dx = x0 - xa), the ones outside the window into the row's slack (RW >= 4*NCH: never another
//     row's cells); cells outside the level (zero padding, Q4) are written as 0 from the masks;
//   * level l+1's gathers are issued right after level l's patches are in LDS, so they fly during level l's taps and
//     MFMAs;
//   * B (weights, fragment-major: one wave instruction = 1 KB contiguous, L2-resident) goes straight into the MFMA
//     operand registers through a 2-deep ring of k32 groups, each group's load issued right after the MFMAs of the
//     group two before it. Vector-memory loads retire in issue order, so only a group whose load follows the next
//     level's gathers waits for them (G = 3: the level's last group).
// Taps, split and MFMA order are those of the round-2 kernel (LDS-staged weights, dword gathers; git history and
// tools/build_rev.sh for A/B): the output is bit for bit the same.
template <int R>
__global__ __launch_bounds__(kNT, 2) void corr_convc1_kernel(C1Args a) {
  constexpr int PK = 2 * R + 2, K = 2 * R + 1, KK = K * K;
  constexpr int NCH = (PK + 6) / 4;                          // chunks per window row (dx <= 3)
  constexpr int RW = ((4 * NCH > PK + 3) ? 4 * NCH : PK + 3) | 1;  // LDS row pitch (floats; odd: spreads the
                                                                    // chunk writes of consecutive rows over banks)
  constexpr int QS = ((PK * RW + 3) | 1);                    // per-query pitch: odd -> conflict-free tap reads
  constexpr int G = (KK + 31) / 32;
  constexpr int NSLOT = (KK + 7) / 8;
  constexpr int A_BYTES = G * kQM * 128;
  constexpr int P_BYTES = kQM * QS * 4;
  constexpr int TS = kN + 4;
  constexpr int EPI_BYTES = kQM * TS * 4;
  constexpr int MAIN = A_BYTES + P_BYTES;
  constexpr int LDS_BYTES = MAIN > EPI_BYTES ? MAIN : EPI_BYTES;
  constexpr int CITEMS = kQM * PK * NCH;                     // chunk items per level
  constexpr int NI = (CITEMS + kNT - 1) / kNT;
  constexpr int NS = 4;                                      // decode slots (level & 3)
  static_assert(4 * NCH <= 16 && PK <= 16, "mask widths");
  __shared__ __attribute__((aligned(16))) uint8_t smem[LDS_BYTES];
  __shared__ float2 sSB[kN];
  __shared__ float2 sC[kQM];
  __shared__ int4 sO[NS][kQM];    // window origin x0, y0, masks (x: bits 0-15, y: bits 16-31), dx
  __shared__ float4 sW[NS][kQM];  // bilinear weights (nw, ne, sw, se)
  uint8_t* sA = smem;
  float* sP = reinterpret_cast<float*>(smem + A_BYTES);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave;
  const int r = lane & 31, hh = lane >> 5;
  const int q0 = blockIdx.x * kQM;
  const int nq = min(kQM, a.total - q0);
  int nst = 0;
  auto stamp = [&]() {  // diagnostics (experiment hook): per-workgroup clock stamps
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
  const int qd = tid & (kQM - 1);            // the query a decoding thread handles
  const bool dwave = tid >= (kNT - kQM);      // wave 3: decodes levels 2.. inside the loop
  // window of query qd at level l -> sO / sW[l & 3]
  auto decode = [&](int l, float cx, float cy) {
    int Hl, Wl, WB, LF;
    const float* base;
    level(l, Hl, Wl, WB, LF, base);
    int xs, ys;
    float4 w4;
    window_origin(cx, cy, __int_as_float((127 - l) << 23), R, xs, ys, w4);  // 1/2^l exactly (corr.py:68)
    const int dx = xs & 3, xa = xs - dx;
    const int xl = max(0, -xa), xh = min(4 * NCH, Wl - xa);
    const int yl = max(0, -ys), yh = min(PK, Hl - ys);
    const unsigned xm = xh > xl ? (((1u << (xh - xl)) - 1u) << xl) : 0u;
    const unsigned ym = yh > yl ? (((1u << (yh - yl)) - 1u) << yl) : 0u;
    sO[l & (NS - 1)][qd] = make_int4(xs, ys, static_cast<int>(xm | (ym << 16)), dx);
    sW[l & (NS - 1)][qd] = w4;
  };

  for (int c = tid; c < kN; c += kNT) sSB[c] = make_float2(a.wsc[c], a.bias ? a.bias[c] : 0.f);
  // the query's coordinates; waves 0 and 1 decode levels 0 and 1 (wave 3, the one with the fewest tap slots, decodes
  // the later levels inside the loop)
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
  // A's taps past KK (the last group's tail) are never written again: zero the whole A buffer once
  for (int e = tid; e < A_BYTES / 16; e += kNT) reinterpret_cast<u32x4*>(sA)[e] = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();
  // chunk item s of this thread -> (query, window row, chunk): recomputed per use (a few full-rate ops; no live
  // registers across the level)
  static_assert(magic16_ok(PK * NCH, CITEMS) && magic16_ok(NCH, PK * NCH), "chunk item decode");
  auto item_of = [&](int s, int& q, int& u, int& k) {
    int t_ = tid;
    asm volatile("" : "+v"(t_));
    const unsigned item = static_cast<unsigned>(min(t_ + kNT * s, CITEMS - 1));
    q = static_cast<int>(__umul24(item, magic16(PK * NCH)) >> 16);
    const unsigned rm = item - static_cast<unsigned>(q) * (PK * NCH);
    u = static_cast<int>(__umul24(rm, magic16(NCH)) >> 16);
    k = static_cast<int>(rm - static_cast<unsigned>(u) * NCH);
  };

  u32x4 rv[NI];
  auto gather = [&](int l) {
    int Hl, Wl, WB, LF;
    const float* base;
    level(l, Hl, Wl, WB, LF, base);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(base + (size_t)q0 * LF), (short)0, nq * LF * 4, 0x00020000);
    constexpr int HB = (NI + 1) / 2;  // two batches of window reads: fewer live registers
#pragma unroll
    for (int s0 = 0; s0 < NI; s0 += HB) {
      int4 o[NI];
      int qs[NI], us[NI], ks[NI];
#pragma unroll
      for (int s = s0; s < (NI < s0 + HB ? NI : s0 + HB); ++s) {
        item_of(s, qs[s], us[s], ks[s]);
        o[s] = sO[l & (NS - 1)][qs[s]];
      }
#pragma unroll
      for (int s = s0; s < (NI < s0 + HB ? NI : s0 + HB); ++s) {
        const int q = qs[s], u = us[s], k = ks[s];
        const int y = o[s].y + u, xc = (o[s].x - o[s].w) + 4 * k;
        // the chunk holds a needed, in-level cell: row u valid, one of its 4 columns valid and inside the window
        const unsigned need = ((static_cast<unsigned>(o[s].z) >> 16) >> u) & 1u &
                              (((static_cast<unsigned>(o[s].z) & 0xffffu) >> (4 * k)) & 15u ? 1u : 0u) &
                              (4 * k < o[s].w + PK ? 1u : 0u);
        int off = (__umul24(q, LF) + (__umul24(static_cast<unsigned>(y) >> 2, WB) + (xc >> 3)) * 32 + ((y & 3) << 3) + (xc & 7)) * 4;
        asm volatile("" : "+v"(off));  // computed unconditionally: a select, not an exec branch around it
        off = need ? off : 0;
        rv[s] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
      }
    }
  };
  const __amdgpu_buffer_rsrc_t rsW =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.wf), (short)0, a.nlev * G * kN * 128, 0x00020000);
  const int wbase = wn * 8192 + lane * 16;
  u32x4 bq[2][8];  // B ring: global k32 group t in bq[t & 1]; [(nt * 2 + sub) * 2 + hi/lo]
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
  // one level; P = (l * G) & 1: the ring slot of the level's first group
  auto body = [&](int l, auto Pc) {
    constexpr int P = decltype(Pc)::value;
    // ---- 1. chunks -> LDS patches (cells outside the level zeroed) ----
#pragma unroll
    for (int s = 0; s < NI; ++s) {
      if (CITEMS % kNT == 0 || tid + kNT * s < CITEMS) {
        int q, u, k;
        item_of(s, q, u, k);
        const int4 o = sO[l & (NS - 1)][q];
        const unsigned m = (((static_cast<unsigned>(o.z) >> 16) >> u) & 1u) ? ((static_cast<unsigned>(o.z) >> (4 * k)) & 15u) : 0u;
        const float* fv = reinterpret_cast<const float*>(&rv[s]);
        float* dst = sP + q * QS + u * RW + 3 + 4 * k - o.w;
#pragma unroll
        for (int e = 0; e < 4; ++e) dst[e] = ((m >> e) & 1u) ? fv[e] : 0.0f;
      }
    }
    __syncthreads();  // patches complete; every wave is past level l-1's MFMAs (A free)
    stamp();
    // ---- 2. next level's gathers (rv is free), the level after next's windows ----
    if (l + 1 < a.nlev) gather(l + 1);
    if (dwave && l + 2 < a.nlev) decode(l + 2, sC[qd].x, sC[qd].y);
    // ---- 3. bilinear taps -> split-fp16 A operand; the slot set is the wave index (a scalar branch per slot) ----
    {
      const int q = tid & (kQM - 1), set = __builtin_amdgcn_readfirstlane(tid / kQM);
      const float4 w4 = sW[l & (NS - 1)][q];
      const float* p = sP + q * QS + 3;
#pragma unroll
      for (int S = 0; S < NSLOT; ++S) {
        if ((S & 3) != set) continue;
        float v[8];  // all 8 taps first (the shared cells are read once), then the splits
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int k = 8 * S + e;  // reference channel order within the level: k = i*K + j, i moves x, j moves y
          v[e] = 0.f;
          if (k < KK) {
            const int i = k / K, j = k - (k / K) * K;
            v[e] = bilinear4(p[j * RW + i], p[j * RW + i + 1], p[(j + 1) * RW + i], p[(j + 1) * RW + i + 1], w4);
          }
        }
        range_guard8(v);
        half8 hi, lo;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          _Float16 h_, l_;
          split_f16(v[e], h_, l_);
          hi[e] = h_;
          lo[e] = l_;
        }
        uint8_t* row = sA + (S >> 2) * (kQM * 128) + q * 128;
        *reinterpret_cast<half8*>(row + (((S & 3) ^ swz(q)) << 4)) = hi;
        *reinterpret_cast<half8*>(row + (((4 + (S & 3)) ^ swz(q)) << 4)) = lo;
      }
    }
    __syncthreads();  // A complete; the patches consumed
    stamp();
    // ---- 4. the level's MFMAs ----
#pragma unroll
    for (int g = 0; g < G; ++g) {
      constexpr int dummy = 0;
      (void)dummy;
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
      const int t2 = l * G + g + 2;  // the ring slot is free: the group two ahead
      if (t2 < nlg) load_b(t2, bc);
    }
    stamp();
  };
  for (int l = 0; l < a.nlev; l += 2) {
    body(l, std::integral_constant<int, 0>{});  // (l * G) & 1 = 0 for even l
    if (l + 1 < a.nlev) body(l + 1, std::integral_constant<int, G & 1>{});
  }

  // ---- epilogue: accumulators -> LDS tile [pixel][channel] -> scale, bias, ReLU -> S32 ----
  __syncthreads();  // every wave is past its last A read (the tile overlays A and the patches)
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
  // each thread's 8 channels are the same for every item (kNT is a multiple of kN / 8): their (scale, bias) once
  static_assert(kNT % (kN / 8) == 0, "fixed channel octet per thread");
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
    half8 hi, lo;
    float mx = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float2 sb = sbv[j];
      float x = v[j] * sb.x + sb.y;
      x = x < 0.f ? 0.f : x;  // relu (update.py:120); NaN propagates like ATen
      mx = fmaxf(mx, x);
      _Float16 h_, l_;
      split_f16(x, h_, l_);
      hi[j] = h_;
      lo[j] = l_;
    }
    range_guard(mx);
    uint8_t* line = a.y + (long long)(q0 + pl) * a.yps + (n >> 5) * 128 + ((n & 31) >> 3) * 16;
    *reinterpret_cast<half8*>(line) = hi;
    *reinterpret_cast<half8*>(line + 64) = lo;
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
