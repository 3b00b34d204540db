// Experiment variants of the fused lookup + convc1 kernel (r05), measured against the product kernel
// (torch-optical-flow_amd/csrc/corr_convc1.hip, corr_convc1_kernel) and not adopted; results and reasoning in DESIGN.md §4
// ("corr_convc1 ... r05") and profiles/r05/s2-s7. Built as a separate library (tools/exp/build_c1var.sh ->
// build/exp/libc1var.so) with one C entry point taking the product ABI's arguments plus the variant number, so that the
// A/B scripts (tools/exp/run_c1_variant_ab.py, run_c1_stamps_variants.py) time them in one process beside the product.
// Variants: 2 = 8 waves; 3 = phase-pipelined; 4 = VALU-lean (offset tables, register epilogue); 5 = hybrid; 6 = rowmap; 7 = quad; 8 = 128 queries per workgroup. Every one is
// bit-identical to the product kernel (checked by the A/B script on three pyramids).
#include <type_traits>
#include <utility>

#include "../../torch-optical-flow_amd/csrc/oflow_internal.h"

namespace oflow {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kQM = 64;   // query pixels per workgroup
constexpr int kNT = 256;  // threads: 4 waves, one per 64-channel quarter (64 pixels x 64 channels each)
constexpr int kN = 256;   // convc1 output channels (update.py:114)

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

// f(std::integral_constant<int, 0>{}) ... f(std::integral_constant<int, N - 1>{}), in order
template <class F, int... S>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, S...>) {
  (f(std::integral_constant<int, S>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

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



// r05 kernel: 8 waves per workgroup (64 queries, wave w = output channels 32w..32w+31 = S32 group w), two workgroups
// per CU (<= 128 VGPRs, <= 80 KB of LDS). Against the 4-wave kernel above, each wave's share of a level's serial chain
// halves (chunk items 10 -> 5 per thread, tap slots 3 -> 2, MFMAs 72 -> 36) while a CU still holds 128 queries.
// The MFMA runs with the operands swapped (weights as A, taps as B: the same fragments, the same three products in the
// same order), so the accumulators hold [channel][pixel] and each lane owns 16 channels of one pixel: the epilogue
// (scale, bias, ReLU, split) stores its 8-B runs of the pixel's S32 line straight from the registers -- no LDS tile,
// no transpose, no extra barriers. Every level's window origin is decoded in the prologue (waves 0..L-1).
template <int R>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void corr_convc1_w8_kernel(C1Args a) {
  constexpr int NT = 512;
  constexpr int PK = 2 * R + 2, K = 2 * R + 1, KK = K * K;
  constexpr int NCH = (PK + 6) / 4;
  constexpr int RW = ((4 * NCH > PK + 3) ? 4 * NCH : PK + 3) | 1;
  constexpr int QS = ((PK * RW + 3) | 1);
  constexpr int G = (KK + 31) / 32;
  constexpr int NSLOT = (KK + 7) / 8;
  constexpr int A_BYTES = G * kQM * 128;
  constexpr int P_BYTES = kQM * QS * 4;
  constexpr int CITEMS = kQM * PK * NCH;
  constexpr int NI = (CITEMS + NT - 1) / NT;
  static_assert(4 * NCH <= 16 && PK <= 16, "mask widths");
  static_assert(NT / 64 * 32 == kN, "one S32 group per wave");
  __shared__ __attribute__((aligned(16))) uint8_t smem[A_BYTES + P_BYTES];
  __shared__ float2 sSB[kN];
  constexpr int NS = 4;                // decode slots (level & 3)
  __shared__ int4 sO[NS][kQM];         // window origin x0, y0, masks (x: bits 0-15, y: bits 16-31), dx
  __shared__ float4 sW[NS][kQM];       // bilinear weights (nw, ne, sw, se)
  __shared__ float2 sC[kQM];           // coordinates (levels past NS are decoded inside the loop)
  uint8_t* sA = smem;
  float* sP = reinterpret_cast<float*>(smem + A_BYTES);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int q0 = blockIdx.x * kQM;
  const int nq = min(kQM, a.total - q0);
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
  // window of query `lane` at level l -> sO / sW[l & 3]
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
    sO[l & (NS - 1)][lane] = make_int4(xs, ys, static_cast<int>(xm | (ym << 16)), dx);
    sW[l & (NS - 1)][lane] = w4;
  };
  // prologue: wave l < min(L, 4) decodes level l's windows of the 64 queries (lane = query)
  for (int c = tid; c < kN; c += NT) sSB[c] = make_float2(a.wsc[c], a.bias ? a.bias[c] : 0.f);
  if (wave < a.nlev && wave < NS) {
    float cx = 1e30f, cy = 1e30f;  // past the last query: all-zero window
    if (lane < nq) {
      const int q = q0 + lane;
      const int b = q / a.N, pix = q - b * a.N;
      cx = a.coords[(size_t)(2 * b) * a.N + pix];
      cy = a.coords[(size_t)(2 * b + 1) * a.N + pix];
    }
    if (wave == 0) sC[lane] = make_float2(cx, cy);
    decode(wave, cx, cy);
  }
  for (int e = tid; e < A_BYTES / 16; e += NT) reinterpret_cast<u32x4*>(sA)[e] = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();
  static_assert(magic16_ok(PK * NCH, CITEMS) && magic16_ok(NCH, PK * NCH), "chunk item decode");
  auto item_of = [&](int s, int& q, int& u, int& k) {
    int t_ = tid;
    asm volatile("" : "+v"(t_));
    const unsigned item = static_cast<unsigned>(min(t_ + NT * s, CITEMS - 1));
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
      const unsigned need = ((static_cast<unsigned>(o[s].z) >> 16) >> u) & 1u &
                            (((static_cast<unsigned>(o[s].z) & 0xffffu) >> (4 * k)) & 15u ? 1u : 0u) &
                            (4 * k < o[s].w + PK ? 1u : 0u);
      int off = (__umul24(q, LF) + (__umul24(static_cast<unsigned>(y) >> 2, WB) + (xc >> 3)) * 32 + ((y & 3) << 3) + (xc & 7)) * 4;
      asm volatile("" : "+v"(off));
      off = need ? off : 0;
      rv[s] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
    }
    }
  };
  const __amdgpu_buffer_rsrc_t rsW =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.wf), (short)0, a.nlev * G * kN * 128, 0x00020000);
  const int wbase = wave * 4096 + lane * 16;  // [group][wave 8][sub 2][hi, lo][lane 64][16 B] of the fragment-major pack
  u32x4 bq[2][4];  // A-operand (weights) ring: global k32 group t in bq[t & 1]; [sub * 2 + hi/lo]
  auto load_b = [&](int t, u32x4 (&dst)[4]) {
    const int so = t * (kN * 128);
#pragma unroll
    for (int e = 0; e < 4; ++e) dst[e] = __builtin_amdgcn_raw_buffer_load_b128(rsW, wbase, so + e * 1024, 0);
  };
  f32x16 acc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;

  const int nlg = a.nlev * G;
  load_b(0, bq[0]);
  if (nlg > 1) load_b(1, bq[1]);
  gather(0);
  stamp();
  auto body = [&](int l, auto Pc) {
    constexpr int P = decltype(Pc)::value;
    // ---- 1. chunks -> LDS patches (cells outside the level zeroed), the window shifted by dx ----
#pragma unroll
    for (int s = 0; s < NI; ++s) {
      if (CITEMS % NT == 0 || tid + NT * s < CITEMS) {
        int q, u, k;
        item_of(s, q, u, k);
        const int4 o = sO[l & (NS - 1)][q];
        const unsigned m = (((static_cast<unsigned>(o.z) >> 16) >> u) & 1u) ? ((static_cast<unsigned>(o.z) >> (4 * k)) & 15u) : 0u;
        const float4 f4 = __builtin_bit_cast(float4, rv[s]);
        const float fv[4] = {f4.x, f4.y, f4.z, f4.w};
        float* dst = sP + q * QS + u * RW + 3 + 4 * k - o.w;
#pragma unroll
        for (int e = 0; e < 4; ++e) dst[e] = ((m >> e) & 1u) ? fv[e] : 0.0f;
      }
    }
    __syncthreads();  // patches complete; every wave is past level l-1's MFMAs (A free)
    stamp();
    // ---- 2. next level's gathers (rv is free) ----
    if (l + 1 < a.nlev) gather(l + 1);
    // ---- 3. bilinear taps -> split-fp16 tap operand; slot set = wave (waves 0..NSLOT-9 take two slots) ----
    {
      const int q = lane, set = wave;
      const float4 w4 = sW[l & (NS - 1)][q];
      const float* p = sP + q * QS + 3;
#pragma unroll
      for (int S = 0; S < NSLOT; ++S) {
        if ((S & 7) != set) continue;
        float v[8];
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
    __syncthreads();  // taps complete; the patches consumed
    stamp();
    if (wave == 0 && l + NS < a.nlev) decode(l + NS, sC[lane].x, sC[lane].y);  // slot l & 3 is free now
    // ---- 4. the level's MFMAs: C[channel][pixel] += W[channel][k] * T[k][pixel] ----
#pragma unroll
    for (int g = 0; g < G; ++g) {
      u32x4 (&wc)[4] = bq[(P + g) & 1];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        half8 th[2], tl[2];
        const int chi = 2 * sub + hh, clo = 4 + 2 * sub + hh;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const int pr = mt * 32 + r;
          const uint8_t* row = sA + g * (kQM * 128) + pr * 128;
          th[mt] = *reinterpret_cast<const half8*>(row + ((chi ^ swz(pr)) << 4));
          tl[mt] = *reinterpret_cast<const half8*>(row + ((clo ^ swz(pr)) << 4));
        }
        const half8 wh = __builtin_bit_cast(half8, wc[sub * 2 + 0]);
        const half8 wl = __builtin_bit_cast(half8, wc[sub * 2 + 1]);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, th[mt], acc[mt], 0, 0, 0);
          acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, tl[mt], acc[mt], 0, 0, 0);
          acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, th[mt], acc[mt], 0, 0, 0);
        }
      }
      const int t2 = l * G + g + 2;
      if (t2 < nlg) load_b(t2, wc);
    }
    stamp();
  };
  for (int l = 0; l < a.nlev; l += 2) {
    body(l, std::integral_constant<int, 0>{});
    if (l + 1 < a.nlev) body(l + 1, std::integral_constant<int, G & 1>{});
  }

  // ---- epilogue from the accumulators: lane (pixel r, half hh) holds channels 8j + 4hh + e of its wave's group ----
  typedef _Float16 half4 __attribute__((ext_vector_type(4)));
  float2 sbv[16];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) sbv[j * 4 + e] = sSB[wave * 32 + 8 * j + 4 * hh + e];
  float mx = 0.f;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int pl = mt * 32 + r;
    if (pl >= nq) continue;
    uint8_t* line = a.y + (long long)(q0 + pl) * a.yps + wave * 128;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      half4 hi, lo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float2 sb = sbv[j * 4 + e];
        float x = acc[mt][j * 4 + e] * sb.x + sb.y;
        x = x < 0.f ? 0.f : x;  // relu (update.py:120); NaN propagates like ATen
        mx = fmaxf(mx, x);
        _Float16 h_, l_;
        split_f16(x, h_, l_);
        hi[e] = h_;
        lo[e] = l_;
      }
      *reinterpret_cast<half4*>(line + (8 * j + 4 * hh) * 2) = hi;
      *reinterpret_cast<half4*>(line + 64 + (8 * j + 4 * hh) * 2) = lo;
    }
  }
  range_guard(mx);
  if (a.stamps != nullptr) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  stamp();
}

// r05 pipelined kernel (4 waves, 64 queries, two workgroups per CU). The kernels above run each level as serial phases
// (patch writes -> taps -> MFMAs) and the two workgroups of a CU, started together on identical code, stay in step: the
// matrix cores idle while the taps and patch writes run and the VALU / LDS idle during the MFMAs (r03 stamps: per level
// gather wait + patch writes 3-4 k cycles, taps 5 k, MFMAs 4 k). Here the next level's patch writes and taps run in the
// same phases as this level's MFMAs:
//   phase 0 of level l: MFMAs of k32 group 0 of l  | patch writes of level l+1 (its gathers landed), then the gathers
//                                                     of level l+2 are issued
//   phase g >= 1:       MFMAs of group g of l      | taps of level l+1 for group g (phase 1 also group 0)
// with one barrier per phase. The tap operand lives in a ring of G+1 group slots (global group t = l*G + g in slot
// t % (G+1)): the taps of level l+1's group g' overwrite the slot of group l*G + g' - 1, whose MFMAs ran in the phase
// before. Inside a phase each wave alternates blocks of MFMAs with tap / patch work (sched_barrier-separated), so one
// wave's VALU / LDS work fills the gaps of the other waves' MFMAs on its SIMD.
// The patch keeps only the window's cells (row pitch PK | 1, query pitch PK*RW | 1: odd, conflict-free tap reads); a
// chunk's cells outside the window are not written. The MFMA runs with the operands swapped (weights as A, taps as B)
// and the epilogue stores from the accumulators, as in the 8-wave kernel. Same taps, same products in the same order:
// bit-identical to the kernels above.
template <int R>
__global__ __launch_bounds__(256, 2) void corr_convc1_pipe_kernel(C1Args a) {
  constexpr int NT = 256;
  constexpr int PK = 2 * R + 2, K = 2 * R + 1, KK = K * K;
  constexpr int NCH = (PK + 6) / 4;
  constexpr int RW = PK | 1;                   // patch row pitch (floats): the window's PK cells
  constexpr int QS = (PK * RW) | 1;            // per-query pitch: odd -> conflict-free tap reads (lane = query)
  constexpr int G = (KK + 31) / 32;
  constexpr int NU = 4 * G;                    // tap units (8 taps each) per level, zero units past KK included
  constexpr int NR = G + 1;                    // tap-operand ring slots
  constexpr int SLOT = kQM * 128;              // one k32 group of the tap operand: [pixel][hi 64 B | lo 64 B]
  constexpr int A_BYTES = NR * SLOT;
  constexpr int P_BYTES = kQM * QS * 4;
  constexpr int CITEMS = kQM * PK * NCH;
  constexpr int NI = (CITEMS + NT - 1) / NT;
  constexpr int NS = 4;
  static_assert(4 * NCH <= 16 && PK <= 16, "mask widths");
  __shared__ __attribute__((aligned(16))) uint8_t smem[A_BYTES + P_BYTES];
  __shared__ float2 sSB[kN];
  __shared__ int4 sO[NS][kQM];
  __shared__ float4 sW[NS][kQM];
  __shared__ float2 sC[kQM];
  uint8_t* sA = smem;
  float* sP = reinterpret_cast<float*>(smem + A_BYTES);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int q0 = blockIdx.x * kQM;
  const int nq = min(kQM, a.total - q0);
  const int L = a.nlev;
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
    sO[l & (NS - 1)][lane] = make_int4(xs, ys, static_cast<int>(xm | (ym << 16)), dx);
    sW[l & (NS - 1)][lane] = w4;
  };
  for (int c = tid; c < kN; c += NT) sSB[c] = make_float2(a.wsc[c], a.bias ? a.bias[c] : 0.f);
  if (wave < L) {  // waves 0..3: levels 0..3 (4 waves = NS slots)
    float cx = 1e30f, cy = 1e30f;  // past the last query: all-zero window
    if (lane < nq) {
      const int q = q0 + lane;
      const int b = q / a.N, pix = q - b * a.N;
      cx = a.coords[(size_t)(2 * b) * a.N + pix];
      cy = a.coords[(size_t)(2 * b + 1) * a.N + pix];
    }
    if (wave == 0) sC[lane] = make_float2(cx, cy);
    decode(wave, cx, cy);
  }
  __syncthreads();
  static_assert(magic16_ok(PK * NCH, CITEMS) && magic16_ok(NCH, PK * NCH), "chunk item decode");
  auto item_of = [&](int s, int& q, int& u, int& k) {
    int t_ = tid;
    asm volatile("" : "+v"(t_));
    const unsigned item = static_cast<unsigned>(min(t_ + NT * s, CITEMS - 1));
    q = static_cast<int>(__umul24(item, magic16(PK * NCH)) >> 16);
    const unsigned rm = item - static_cast<unsigned>(q) * (PK * NCH);
    u = static_cast<int>(__umul24(rm, magic16(NCH)) >> 16);
    k = static_cast<int>(rm - static_cast<unsigned>(u) * NCH);
  };
  u32x4 rv[NI];
  auto gather = [&](int l) __attribute__((always_inline)) {
    int Hl, Wl, WB, LF;
    const float* base;
    level(l, Hl, Wl, WB, LF, base);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(base + (size_t)q0 * LF), (short)0, nq * LF * 4, 0x00020000);
    constexpr int HB = (NI + 1) / 2;
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
        const unsigned need = ((static_cast<unsigned>(o[s].z) >> 16) >> u) & 1u &
                              (((static_cast<unsigned>(o[s].z) & 0xffffu) >> (4 * k)) & 15u ? 1u : 0u) &
                              (4 * k < o[s].w + PK ? 1u : 0u);
        int off = (__umul24(q, LF) + (__umul24(static_cast<unsigned>(y) >> 2, WB) + (xc >> 3)) * 32 + ((y & 3) << 3) + (xc & 7)) * 4;
        asm volatile("" : "+v"(off));
        off = need ? off : 0;
        rv[s] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
      }
    }
  };
  // chunks -> LDS patch: window cell p = 4k - dx + e of row u at sP[q*QS + u*RW + p] for 0 <= p < PK (cells outside
  // the level zeroed from the masks; a chunk's cells outside the window are not written)
  auto patch_write = [&](int l) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < NI; ++s) {
      if (CITEMS % NT == 0 || tid + NT * s < CITEMS) {
        int q, u, k;
        item_of(s, q, u, k);
        const int4 o = sO[l & (NS - 1)][q];
        const unsigned m = (((static_cast<unsigned>(o.z) >> 16) >> u) & 1u) ? ((static_cast<unsigned>(o.z) >> (4 * k)) & 15u) : 0u;
        const float4 f4 = __builtin_bit_cast(float4, rv[s]);
        const float fv[4] = {f4.x, f4.y, f4.z, f4.w};
        const int p0 = 4 * k - o.w;
        float* dst = sP + q * QS + u * RW + p0;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (static_cast<unsigned>(p0 + e) < static_cast<unsigned>(PK)) dst[e] = ((m >> e) & 1u) ? fv[e] : 0.0f;
      }
    }
  };
  // tap unit S of level l (8 taps k = 8S..8S+7 of every query; wave S % 4; lane = query) -> the tap operand's slot
  auto tap_unit = [&](int l, auto Sc) __attribute__((always_inline)) {
    constexpr int S = decltype(Sc)::value;
    if ((S & 3) != wave) return;
    const int q = lane;
    uint8_t* row = sA + ((l * G + (S >> 2)) % NR) * SLOT + q * 128;
    half8 hi, lo;
    if constexpr (8 * S >= KK) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { hi[e] = 0; lo[e] = 0; }
    } else {
      const float4 w4 = sW[l & (NS - 1)][q];
      const float* p = sP + q * QS;
      float v[8];
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
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        _Float16 h_, l_;
        split_f16(v[e], h_, l_);
        hi[e] = h_;
        lo[e] = l_;
      }
    }
    *reinterpret_cast<half8*>(row + (((S & 3) ^ swz(q)) << 4)) = hi;
    *reinterpret_cast<half8*>(row + (((4 + (S & 3)) ^ swz(q)) << 4)) = lo;
  };
  const __amdgpu_buffer_rsrc_t rsW =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.wf), (short)0, L * G * kN * 128, 0x00020000);
  const int wbase = wave * 8192 + lane * 16;
  u32x4 bq[2][8];  // weight ring: global k32 group t in bq[t & 1]; [(nt * 2 + sub) * 2 + hi/lo]
  auto load_b = [&](int t, u32x4 (&dst)[8]) {
    const int so = t * (kN * 128);
#pragma unroll
    for (int e = 0; e < 8; ++e) dst[e] = __builtin_amdgcn_raw_buffer_load_b128(rsW, wbase, so + e * 1024, 0);
  };
  f32x16 acc[2][2];  // [nt][mt]: C[channel][pixel]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  // MFMAs of one sub-step (16 k) of global group t: weights from the ring, taps from the operand slot
  auto mfma_sub = [&](int t, int sub, u32x4 (&wc)[8]) __attribute__((always_inline)) {
    const uint8_t* slot = sA + (t % NR) * SLOT;
    half8 th[2], tl[2];
    const int chi = 2 * sub + hh, clo = 4 + 2 * sub + hh;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int pr = mt * 32 + r;
      th[mt] = *reinterpret_cast<const half8*>(slot + pr * 128 + ((chi ^ swz(pr)) << 4));
      tl[mt] = *reinterpret_cast<const half8*>(slot + pr * 128 + ((clo ^ swz(pr)) << 4));
    }
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const half8 wh = __builtin_bit_cast(half8, wc[(nt * 2 + sub) * 2 + 0]);
      const half8 wl = __builtin_bit_cast(half8, wc[(nt * 2 + sub) * 2 + 1]);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        acc[nt][mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, th[mt], acc[nt][mt], 0, 0, 0);
        acc[nt][mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, tl[mt], acc[nt][mt], 0, 0, 0);
        acc[nt][mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, th[mt], acc[nt][mt], 0, 0, 0);
      }
    }
  };
  const int nlg = L * G;
  load_b(0, bq[0]);
  if (nlg > 1) load_b(1, bq[1]);
  gather(0);
  patch_write(0);
  __syncthreads();  // patch 0 complete
  if (L > 1) gather(1);
  static_for<NU>([&](auto Sc) __attribute__((always_inline)) { tap_unit(0, Sc); });
  __syncthreads();  // level 0's tap operand complete; patch 0 consumed
  stamp();
  // one phase: MFMAs of global group t (two sub-steps) interleaved with the work of the next level
  auto phase = [&](int l, auto gc, auto Pc) __attribute__((always_inline)) {
    constexpr int g = decltype(gc)::value;
    constexpr int P = decltype(Pc)::value;  // ring slot parity of group t = l*G + g
    const int t = l * G + g;
    u32x4 (&wc)[8] = bq[P];
    const bool nxt = l + 1 < L;
    mfma_sub(t, 0, wc);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (g == 0) {
      if (nxt) patch_write(l + 1);
      __builtin_amdgcn_sched_barrier(0);
      mfma_sub(t, 1, wc);
      __builtin_amdgcn_sched_barrier(0);
      // (the ring's next weights before the gathers: only loads issued after a gather wait for it)
      if (t + 2 < nlg) load_b(t + 2, wc);
      if (l + 2 < L) gather(l + 2);
      if (wave == 0 && l + NS < L) decode(l + NS, sC[lane].x, sC[lane].y);  // slot l & 3 is free (taps of l done)
    } else {
      // taps of level l+1 for group g (phase 1: groups 0 and 1)
      if (nxt) {
        if constexpr (g == 1) {
          tap_unit(l + 1, std::integral_constant<int, 0>{});
          tap_unit(l + 1, std::integral_constant<int, 1>{});
          tap_unit(l + 1, std::integral_constant<int, 2>{});
          tap_unit(l + 1, std::integral_constant<int, 3>{});
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      mfma_sub(t, 1, wc);
      __builtin_amdgcn_sched_barrier(0);
      if (nxt) {
        static_for<4>([&](auto Sc) __attribute__((always_inline)) { tap_unit(l + 1, std::integral_constant<int, 4 * g + decltype(Sc)::value>{}); });
      }
    }
    if constexpr (g != 0)
      if (t + 2 < nlg) load_b(t + 2, wc);
    __syncthreads();
    stamp();
  };
  auto level_phases = [&](int l, auto P0) __attribute__((always_inline)) {  // P0 = (l*G) & 1
    constexpr int p0 = decltype(P0)::value;
    static_for<G>([&](auto gc) __attribute__((always_inline)) { phase(l, gc, std::integral_constant<int, (p0 + decltype(gc)::value) & 1>{}); });
  };
  for (int l = 0; l < L; l += 2) {
    level_phases(l, std::integral_constant<int, 0>{});
    if (l + 1 < L) level_phases(l + 1, std::integral_constant<int, G & 1>{});
  }

  // ---- epilogue from the accumulators: lane (pixel r of tile mt, half hh) holds channels 8j + 4hh + e of tile nt ----
  typedef _Float16 half4 __attribute__((ext_vector_type(4)));
  float mx = 0.f;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int cb = wave * 64 + nt * 32;  // S32 group 2 * wave + nt
    float2 sbv[16];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) sbv[j * 4 + e] = sSB[cb + 8 * j + 4 * hh + e];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int pl = mt * 32 + r;
      if (pl >= nq) continue;
      uint8_t* line = a.y + (long long)(q0 + pl) * a.yps + (cb >> 5) * 128;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        half4 hi, lo;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float2 sb = sbv[j * 4 + e];
          float x = acc[nt][mt][j * 4 + e] * sb.x + sb.y;
          x = x < 0.f ? 0.f : x;  // relu (update.py:120); NaN propagates like ATen
          mx = fmaxf(mx, x);
          _Float16 h_, l_;
          split_f16(x, h_, l_);
          hi[e] = h_;
          lo[e] = l_;
        }
        *reinterpret_cast<half4*>(line + (8 * j + 4 * hh) * 2) = hi;
        *reinterpret_cast<half4*>(line + 64 + (8 * j + 4 * hh) * 2) = lo;
      }
    }
  }
  range_guard(mx);
  if (a.stamps != nullptr) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  stamp();
}

// r05 VALU-lean kernel (4 waves, 64 queries, two workgroups per CU; the r04 kernel's level pipeline). PMC of the r04
// kernel (profiles/r05/s4_pmc_mfma.json): 4,751 VALU instructions per wave, ~1,190 per level, against 72 MFMAs per
// level; a wave64 VALU instruction occupies its SIMD for ~4 cycles, so with two waves per SIMD the VALU alone is ~9.5 k
// of a level's ~12 k cycles (stamps, s4_stamps.log) -- the kernel was VALU-issue bound, not gather or MFMA bound. ISA
// count: ~32 VALU to address each 16-B window chunk load and ~36 to write it to the patch (item decode, window origin,
// tile arithmetic, validity masks, the zero selects), i.e. ~680 of the ~1,190 per level. Here:
//   * the decoding wave writes, per (query, level), the byte offset of each of the window's PK rows in the tiled level
//     (query base folded in) and of each of its NCH chunk columns, with a sentinel (2^30) for rows / chunks outside the
//     level or the window: a chunk's offset is one add of two LDS words, and an outside chunk's offset lies past the
//     buffer's size, so the buffer load returns zeros without touching memory (the zero padding of Q4 for free);
//   * every thread's chunk items (query, row, chunk) are decoded once into one packed register per item;
//   * the patch write is then the item's constant offset + the query's window base, and four stores, no selects (only
//     levels whose width is not a multiple of 4 -- a chunk partly past the level's right edge -- take a masked path);
//   * the MFMA runs with the operands swapped and the epilogue stores from the accumulators (no LDS tile).
// Same chunk data, taps, products and order: bit-identical to the r04 kernel.
template <int R>
__global__ __launch_bounds__(256, 2) void corr_convc1_lean_kernel(C1Args a) {
  constexpr int NT = 256;
  constexpr int PK = 2 * R + 2, K = 2 * R + 1, KK = K * K;
  constexpr int NCH = (PK + 6) / 4;
  constexpr int RW = ((4 * NCH > PK + 3) ? 4 * NCH : PK + 3) | 1;
  constexpr int QS = ((PK * RW + 3) | 1);
  constexpr int G = (KK + 31) / 32;
  constexpr int NSLOT = (KK + 7) / 8;
  constexpr int A_BYTES = G * kQM * 128;
  constexpr int P_BYTES = kQM * QS * 4;
  constexpr int CITEMS = kQM * PK * NCH;
  constexpr int NI = (CITEMS + NT - 1) / NT;
  constexpr int NS = 2;                      // decode slots (level & 1): level l+1 decoded while level l's patch is written
  constexpr int SENT = 1 << 30;              // offset sentinel: past any workgroup's buffer size
  static_assert(kQM * PK <= 1024 && kQM * NCH <= 256 && 9 * RW + 4 * NCH <= 255, "packed item fields");
  __shared__ __attribute__((aligned(16))) uint8_t smem[A_BYTES + P_BYTES];
  __shared__ int sRow[NS][kQM * PK];   // byte offset of window row u of query q in the level (+ q * LF * 4), or SENT
  __shared__ int sCol[NS][kQM * NCH];  // byte offset of window chunk column k, or SENT
  __shared__ int sPB[NS][kQM];         // the query's patch base: q * QS + 3 - dx
  __shared__ int sXA[NS][kQM];         // the window's first chunk column x0 & ~3 (masked path only)
  __shared__ float4 sW[NS][kQM];       // bilinear weights (nw, ne, sw, se)
  __shared__ float2 sC[kQM];
  uint8_t* sA = smem;
  float* sP = reinterpret_cast<float*>(smem + A_BYTES);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int q0 = blockIdx.x * kQM;
  const int nq = min(kQM, a.total - q0);
  const int L = a.nlev;
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
  // window of query `lane` at level l -> the offset tables of slot l & 1 (one wave; lane = query)
  auto decode = [&](int l, float cx, float cy) __attribute__((always_inline)) {
    int Hl, Wl, WB, LF;
    const float* base;
    level(l, Hl, Wl, WB, LF, base);
    int xs, ys;
    float4 w4;
    window_origin(cx, cy, __int_as_float((127 - l) << 23), R, xs, ys, w4);  // 1/2^l exactly (corr.py:68)
    const int dx = xs & 3, xa = xs - dx;
    const int sl = l & (NS - 1), q = lane;
    const int qb = q * LF * 4;
#pragma unroll
    for (int u = 0; u < PK; ++u) {
      const int y = ys + u;
      sRow[sl][q * PK + u] = static_cast<unsigned>(y) < static_cast<unsigned>(Hl)
                                 ? qb + (y >> 2) * (WB * 128) + ((y & 3) << 5) : SENT;
    }
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int xc = xa + 4 * k;
      sCol[sl][q * NCH + k] = (static_cast<unsigned>(xc) < static_cast<unsigned>(Wl) && 4 * k < dx + PK)
                                  ? ((xc >> 3) << 7) + ((xc & 7) << 2) : SENT;
    }
    sPB[sl][q] = q * QS + 3 - dx;
    sXA[sl][q] = xa;
    sW[sl][q] = w4;
  };
  if (wave == 0) {
    float cx = 1e30f, cy = 1e30f;  // past the last query: all-zero window
    if (lane < nq) {
      const int qq = q0 + lane;
      const int b = qq / a.N, pix = qq - b * a.N;
      cx = a.coords[(size_t)(2 * b) * a.N + pix];
      cy = a.coords[(size_t)(2 * b + 1) * a.N + pix];
    }
    sC[lane] = make_float2(cx, cy);
    decode(0, cx, cy);
  }
  for (int e = tid; e < A_BYTES / 16; e += NT) reinterpret_cast<u32x4*>(sA)[e] = u32x4{0u, 0u, 0u, 0u};
  // chunk item s of this thread -> bits 0-9 q*PK + u, 10-17 q*NCH + k, 18-25 u*RW + 4k (recomputed per use from an
  // opaque copy of tid: a few full-rate ops, no registers held across the level)
  static_assert(magic16_ok(PK * NCH, CITEMS) && magic16_ok(NCH, PK * NCH), "chunk item decode");
  auto item_word = [&](int s) __attribute__((always_inline)) {
    int t_ = tid;
    asm volatile("" : "+v"(t_));
    const unsigned item = static_cast<unsigned>(min(t_ + NT * s, CITEMS - 1));
    const unsigned q = __umul24(item, magic16(PK * NCH)) >> 16;
    const unsigned rm = item - q * (PK * NCH);
    const unsigned u = (NCH == 4) ? (rm >> 2) : (__umul24(rm, magic16(NCH)) >> 16);
    const unsigned k = rm - u * NCH;
    return (q * PK + u) | ((q * NCH + k) << 10) | ((u * RW + 4 * k) << 18);
  };
  __syncthreads();
  u32x4 rv[NI];
  auto gather = [&](int l) __attribute__((always_inline)) {
    int Hl, Wl, WB, LF;
    const float* base;
    level(l, Hl, Wl, WB, LF, base);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(base + (size_t)q0 * LF), (short)0, nq * LF * 4, 0x00020000);
    const int sl = l & (NS - 1);
    int ro[NI], co[NI];  // all table reads first (one LDS round trip), then the loads
#pragma unroll
    for (int s = 0; s < NI; ++s) {
      const unsigned w = item_word(s);
      ro[s] = sRow[sl][w & 1023u];
      co[s] = sCol[sl][(w >> 10) & 255u];
    }
#pragma unroll
    for (int s = 0; s < NI; ++s) rv[s] = __builtin_amdgcn_raw_buffer_load_b128(rs, ro[s] + co[s], 0, 0);
  };
  // chunks -> patch row u of query q at sP[q*QS + u*RW], the window's cells at +3 .. (a chunk's cells at
  // +3 + 4k - dx + e; outside chunks arrived as zeros). A level whose width is not a multiple of 4 masks the cells of a
  // chunk past its right edge (tile padding).
  auto patch_write = [&](int l) __attribute__((always_inline)) {
    int Hl, Wl, WB, LF;
    const float* base;
    level(l, Hl, Wl, WB, LF, base);
    const int sl = l & (NS - 1);
    const bool ragged = (Wl & 3) != 0;
    int pb[NI];  // the queries' patch bases first (one LDS round trip)
#pragma unroll
    for (int s = 0; s < NI; ++s) pb[s] = sPB[sl][(item_word(s) & 1023u) / PK];
#pragma unroll
    for (int s = 0; s < NI; ++s) {
      if (CITEMS % NT == 0 || tid + NT * s < CITEMS) {
        const unsigned w = item_word(s);
        const unsigned q = (w & 1023u) / PK;
        float4 f4 = __builtin_bit_cast(float4, rv[s]);
        if (ragged) {
          const int k = static_cast<int>((w >> 10) & 255u) - static_cast<int>(q) * NCH;
          const int nv = Wl - (sXA[sl][q] + 4 * k);
          f4.y = nv > 1 ? f4.y : 0.f;
          f4.z = nv > 2 ? f4.z : 0.f;
          f4.w = nv > 3 ? f4.w : 0.f;
        }
        float* dst = sP + pb[s] + (w >> 18);
        dst[0] = f4.x;
        dst[1] = f4.y;
        dst[2] = f4.z;
        dst[3] = f4.w;
      }
    }
  };
  const __amdgpu_buffer_rsrc_t rsW =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.wf), (short)0, L * G * kN * 128, 0x00020000);
  const int wbase = wave * 8192 + lane * 16;
  u32x4 bq[2][8];
  auto load_b = [&](int t, u32x4 (&dst)[8]) __attribute__((always_inline)) {
    const int so = t * (kN * 128);
#pragma unroll
    for (int e = 0; e < 8; ++e) dst[e] = __builtin_amdgcn_raw_buffer_load_b128(rsW, wbase, so + e * 1024, 0);
  };
  f32x16 acc[2][2];  // [nt][mt]: C[channel][pixel]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nlg = L * G;
  load_b(0, bq[0]);
  if (nlg > 1) load_b(1, bq[1]);
  gather(0);
  stamp();
  auto body = [&](int l, auto Pc) __attribute__((always_inline)) {
    constexpr int P = decltype(Pc)::value;
    // ---- 1. chunks -> LDS patches; the next level's windows decoded (slot (l+1) & 1: level l-1's, free) ----
    patch_write(l);
    if (wave == 3 && l + 1 < L) decode(l + 1, sC[lane].x, sC[lane].y);
    __syncthreads();  // patches and level l+1's tables complete; every wave is past level l-1's MFMAs (A free)
    stamp();
    // ---- 2. next level's gathers (rv is free) ----
    if (l + 1 < L) gather(l + 1);
    // ---- 3. bilinear taps -> split-fp16 tap operand; the slot set is the wave index ----
    {
      const int q = lane, set = __builtin_amdgcn_readfirstlane(wave);
      const float4 w4 = sW[l & (NS - 1)][q];
      const float* p = sP + q * QS + 3;
#pragma unroll
      for (int S = 0; S < NSLOT; ++S) {
        if ((S & 3) != set) continue;
        float v[8];
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
    __syncthreads();  // tap operand complete; the patches consumed
    stamp();
    // ---- 4. the level's MFMAs: C[channel][pixel] += W[channel][k] * T[k][pixel] ----
#pragma unroll
    for (int g = 0; g < G; ++g) {
      u32x4 (&wc)[8] = bq[(P + g) & 1];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        half8 th[2], tl[2];
        const int chi = 2 * sub + hh, clo = 4 + 2 * sub + hh;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const int pr = mt * 32 + r;
          const uint8_t* row = sA + g * (kQM * 128) + pr * 128;
          th[mt] = *reinterpret_cast<const half8*>(row + ((chi ^ swz(pr)) << 4));
          tl[mt] = *reinterpret_cast<const half8*>(row + ((clo ^ swz(pr)) << 4));
        }
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const half8 wh = __builtin_bit_cast(half8, wc[(nt * 2 + sub) * 2 + 0]);
          const half8 wl = __builtin_bit_cast(half8, wc[(nt * 2 + sub) * 2 + 1]);
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) {
            acc[nt][mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, th[mt], acc[nt][mt], 0, 0, 0);
            acc[nt][mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, tl[mt], acc[nt][mt], 0, 0, 0);
            acc[nt][mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, th[mt], acc[nt][mt], 0, 0, 0);
          }
        }
      }
      const int t2 = l * G + g + 2;
      if (t2 < nlg) load_b(t2, wc);
    }
    stamp();
  };
  for (int l = 0; l < L; l += 2) {
    body(l, std::integral_constant<int, 0>{});
    if (l + 1 < L) body(l + 1, std::integral_constant<int, G & 1>{});
  }

  // ---- epilogue from the accumulators: lane (pixel r of tile mt, half hh) holds channels 8j + 4hh + e of tile nt ----
  typedef _Float16 half4 __attribute__((ext_vector_type(4)));
  float mx = 0.f;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int cb = wave * 64 + nt * 32;  // S32 group 2 * wave + nt
    float4 sc[4], bi[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sc[j] = *reinterpret_cast<const float4*>(a.wsc + cb + 8 * j + 4 * hh);
      bi[j] = a.bias ? *reinterpret_cast<const float4*>(a.bias + cb + 8 * j + 4 * hh) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int pl = mt * 32 + r;
      if (pl >= nq) continue;
      uint8_t* line = a.y + (long long)(q0 + pl) * a.yps + (cb >> 5) * 128;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float s4[4] = {sc[j].x, sc[j].y, sc[j].z, sc[j].w};
        const float b4[4] = {bi[j].x, bi[j].y, bi[j].z, bi[j].w};
        half4 hi, lo;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = acc[nt][mt][j * 4 + e] * s4[e] + b4[e];
          x = x < 0.f ? 0.f : x;  // relu (update.py:120); NaN propagates like ATen
          mx = fmaxf(mx, x);
          _Float16 h_, l_;
          split_f16(x, h_, l_);
          hi[e] = h_;
          lo[e] = l_;
        }
        *reinterpret_cast<half4*>(line + (8 * j + 4 * hh) * 2) = hi;
        *reinterpret_cast<half4*>(line + 64 + (8 * j + 4 * hh) * 2) = lo;
      }
    }
  }
  range_guard(mx);
  if (a.stamps != nullptr) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  stamp();
}

// r05 hybrid (variant 5): the lean kernel's offset tables and chunk addressing with the r04 kernel's MFMA orientation
// and LDS-tile epilogue (the lean kernel's register epilogue of 8-B stores measured 10.8 k vs 6.5 k cycles, s5_stamps),
// and the next level's windows decoded by all four waves (16 queries each, 4 lanes per query) instead of one.
// Lean kernel notes follow.
// r05 VALU-lean kernel (4 waves, 64 queries, two workgroups per CU; the r04 kernel's level pipeline). PMC of the r04
// kernel (profiles/r05/s4_pmc_mfma.json): 4,751 VALU instructions per wave, ~1,190 per level, against 72 MFMAs per
// level; a wave64 VALU instruction occupies its SIMD for ~4 cycles, so with two waves per SIMD the VALU alone is ~9.5 k
// of a level's ~12 k cycles (stamps, s4_stamps.log) -- the kernel was VALU-issue bound, not gather or MFMA bound. ISA
// count: ~32 VALU to address each 16-B window chunk load and ~36 to write it to the patch (item decode, window origin,
// tile arithmetic, validity masks, the zero selects), i.e. ~680 of the ~1,190 per level. Here:
//   * the decoding wave writes, per (query, level), the byte offset of each of the window's PK rows in the tiled level
//     (query base folded in) and of each of its NCH chunk columns, with a sentinel (2^30) for rows / chunks outside the
//     level or the window: a chunk's offset is one add of two LDS words, and an outside chunk's offset lies past the
//     buffer's size, so the buffer load returns zeros without touching memory (the zero padding of Q4 for free);
//   * every thread's chunk items (query, row, chunk) are decoded once into one packed register per item;
//   * the patch write is then the item's constant offset + the query's window base, and four stores, no selects (only
//     levels whose width is not a multiple of 4 -- a chunk partly past the level's right edge -- take a masked path);
//   * the MFMA runs with the operands swapped and the epilogue stores from the accumulators (no LDS tile).
// Same chunk data, taps, products and order: bit-identical to the r04 kernel.
template <int R>
__global__ __launch_bounds__(256, 2) void corr_convc1_hyb_kernel(C1Args a) {
  constexpr int NT = 256;
  constexpr int PK = 2 * R + 2, K = 2 * R + 1, KK = K * K;
  constexpr int NCH = (PK + 6) / 4;
  constexpr int RW = ((4 * NCH > PK + 3) ? 4 * NCH : PK + 3) | 1;
  constexpr int QS = ((PK * RW + 3) | 1);
  constexpr int G = (KK + 31) / 32;
  constexpr int NSLOT = (KK + 7) / 8;
  constexpr int A_BYTES = G * kQM * 128;
  constexpr int P_BYTES = kQM * QS * 4;
  constexpr int CITEMS = kQM * PK * NCH;
  constexpr int NI = (CITEMS + NT - 1) / NT;
  constexpr int NS = 2;                      // decode slots (level & 1): level l+1 decoded while level l's patch is written
  constexpr int SENT = 1 << 30;              // offset sentinel: past any workgroup's buffer size
  static_assert(kQM * PK <= 1024 && kQM * NCH <= 256 && 9 * RW + 4 * NCH <= 255, "packed item fields");
  constexpr int TS = kN + 4;
  constexpr int EPI_BYTES = kQM * TS * 4;
  constexpr int LDS_BYTES = (A_BYTES + P_BYTES) > EPI_BYTES ? (A_BYTES + P_BYTES) : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) uint8_t smem[LDS_BYTES];
  __shared__ float2 sSB[kN];
  __shared__ int sRow[NS][kQM * PK];   // byte offset of window row u of query q in the level (+ q * LF * 4), or SENT
  __shared__ int sCol[NS][kQM * NCH];  // byte offset of window chunk column k, or SENT
  __shared__ int sPB[NS][kQM];         // the query's patch base: q * QS + 3 - dx
  __shared__ int sXA[NS][kQM];         // the window's first chunk column x0 & ~3 (masked path only)
  __shared__ float4 sW[NS][kQM];       // bilinear weights (nw, ne, sw, se)
  __shared__ float2 sC[kQM];
  uint8_t* sA = smem;
  float* sP = reinterpret_cast<float*>(smem + A_BYTES);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int q0 = blockIdx.x * kQM;
  const int nq = min(kQM, a.total - q0);
  const int L = a.nlev;
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
  // windows of level l -> the offset tables of slot l & 1: wave w decodes queries 16w .. 16w+15, four lanes per query
  // (lane part p writes rows p, p+4, p+8 and chunk column p)
  auto decode = [&](int l) __attribute__((always_inline)) {
    int Hl, Wl, WB, LF;
    const float* base;
    level(l, Hl, Wl, WB, LF, base);
    const int q = wave * 16 + (lane >> 2), part = lane & 3;
    const float2 c = sC[q];
    int xs, ys;
    float4 w4;
    window_origin(c.x, c.y, __int_as_float((127 - l) << 23), R, xs, ys, w4);  // 1/2^l exactly (corr.py:68)
    const int dx = xs & 3, xa = xs - dx;
    const int sl = l & (NS - 1);
    const int qb = q * LF * 4;
#pragma unroll
    for (int uu = 0; uu < PK; uu += 4) {
      const int u = uu + part;
      const int y = ys + u;
      if (u < PK)
        sRow[sl][q * PK + u] = static_cast<unsigned>(y) < static_cast<unsigned>(Hl)
                                   ? qb + (y >> 2) * (WB * 128) + ((y & 3) << 5) : SENT;
    }
    if (part < NCH) {
      const int k = part, xc = xa + 4 * k;
      sCol[sl][q * NCH + k] = (static_cast<unsigned>(xc) < static_cast<unsigned>(Wl) && 4 * k < dx + PK)
                                  ? ((xc >> 3) << 7) + ((xc & 7) << 2) : SENT;
    }
    if (part == 0) {
      sPB[sl][q] = q * QS + 3 - dx;
      sXA[sl][q] = xa;
      sW[sl][q] = w4;
    }
  };
  if (wave == 0) {
    float cx = 1e30f, cy = 1e30f;  // past the last query: all-zero window
    if (lane < nq) {
      const int qq = q0 + lane;
      const int b = qq / a.N, pix = qq - b * a.N;
      cx = a.coords[(size_t)(2 * b) * a.N + pix];
      cy = a.coords[(size_t)(2 * b + 1) * a.N + pix];
    }
    sC[lane] = make_float2(cx, cy);
  }
  __syncthreads();
  decode(0);
  for (int e = tid; e < A_BYTES / 16; e += NT) reinterpret_cast<u32x4*>(sA)[e] = u32x4{0u, 0u, 0u, 0u};
  // chunk item s of this thread -> bits 0-9 q*PK + u, 10-17 q*NCH + k, 18-25 u*RW + 4k (recomputed per use from an
  // opaque copy of tid: a few full-rate ops, no registers held across the level)
  static_assert(magic16_ok(PK * NCH, CITEMS) && magic16_ok(NCH, PK * NCH), "chunk item decode");
  auto item_word = [&](int s) __attribute__((always_inline)) {
    int t_ = tid;
    asm volatile("" : "+v"(t_));
    const unsigned item = static_cast<unsigned>(min(t_ + NT * s, CITEMS - 1));
    const unsigned q = __umul24(item, magic16(PK * NCH)) >> 16;
    const unsigned rm = item - q * (PK * NCH);
    const unsigned u = (NCH == 4) ? (rm >> 2) : (__umul24(rm, magic16(NCH)) >> 16);
    const unsigned k = rm - u * NCH;
    return (q * PK + u) | ((q * NCH + k) << 10) | ((u * RW + 4 * k) << 18);
  };
  __syncthreads();
  u32x4 rv[NI];
  auto gather = [&](int l) __attribute__((always_inline)) {
    int Hl, Wl, WB, LF;
    const float* base;
    level(l, Hl, Wl, WB, LF, base);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(base + (size_t)q0 * LF), (short)0, nq * LF * 4, 0x00020000);
    const int sl = l & (NS - 1);
    int ro[NI], co[NI];  // all table reads first (one LDS round trip), then the loads
#pragma unroll
    for (int s = 0; s < NI; ++s) {
      const unsigned w = item_word(s);
      ro[s] = sRow[sl][w & 1023u];
      co[s] = sCol[sl][(w >> 10) & 255u];
    }
#pragma unroll
    for (int s = 0; s < NI; ++s) rv[s] = __builtin_amdgcn_raw_buffer_load_b128(rs, ro[s] + co[s], 0, 0);
  };
  // chunks -> patch row u of query q at sP[q*QS + u*RW], the window's cells at +3 .. (a chunk's cells at
  // +3 + 4k - dx + e; outside chunks arrived as zeros). A level whose width is not a multiple of 4 masks the cells of a
  // chunk past its right edge (tile padding).
  auto patch_write = [&](int l) __attribute__((always_inline)) {
    int Hl, Wl, WB, LF;
    const float* base;
    level(l, Hl, Wl, WB, LF, base);
    const int sl = l & (NS - 1);
    const bool ragged = (Wl & 3) != 0;
    int pb[NI];  // the queries' patch bases first (one LDS round trip)
#pragma unroll
    for (int s = 0; s < NI; ++s) pb[s] = sPB[sl][(item_word(s) & 1023u) / PK];
#pragma unroll
    for (int s = 0; s < NI; ++s) {
      if (CITEMS % NT == 0 || tid + NT * s < CITEMS) {
        const unsigned w = item_word(s);
        const unsigned q = (w & 1023u) / PK;
        float4 f4 = __builtin_bit_cast(float4, rv[s]);
        if (ragged) {
          const int k = static_cast<int>((w >> 10) & 255u) - static_cast<int>(q) * NCH;
          const int nv = Wl - (sXA[sl][q] + 4 * k);
          f4.y = nv > 1 ? f4.y : 0.f;
          f4.z = nv > 2 ? f4.z : 0.f;
          f4.w = nv > 3 ? f4.w : 0.f;
        }
        float* dst = sP + pb[s] + (w >> 18);
        dst[0] = f4.x;
        dst[1] = f4.y;
        dst[2] = f4.z;
        dst[3] = f4.w;
      }
    }
  };
  const __amdgpu_buffer_rsrc_t rsW =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.wf), (short)0, L * G * kN * 128, 0x00020000);
  const int wbase = wave * 8192 + lane * 16;
  u32x4 bq[2][8];
  auto load_b = [&](int t, u32x4 (&dst)[8]) __attribute__((always_inline)) {
    const int so = t * (kN * 128);
#pragma unroll
    for (int e = 0; e < 8; ++e) dst[e] = __builtin_amdgcn_raw_buffer_load_b128(rsW, wbase, so + e * 1024, 0);
  };
  for (int c = tid; c < kN; c += NT) sSB[c] = make_float2(a.wsc[c], a.bias ? a.bias[c] : 0.f);
  f32x16 acc[2][2];  // [mt][nt]: C[pixel][channel]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nlg = L * G;
  load_b(0, bq[0]);
  if (nlg > 1) load_b(1, bq[1]);
  gather(0);
  stamp();
  auto body = [&](int l, auto Pc) __attribute__((always_inline)) {
    constexpr int P = decltype(Pc)::value;
    // ---- 1. chunks -> LDS patches; the next level's windows decoded (slot (l+1) & 1: level l-1's, free) ----
    patch_write(l);
    if (l + 1 < L) decode(l + 1);
    __syncthreads();  // patches and level l+1's tables complete; every wave is past level l-1's MFMAs (A free)
    stamp();
    // ---- 2. next level's gathers (rv is free) ----
    if (l + 1 < L) gather(l + 1);
    // ---- 3. bilinear taps -> split-fp16 tap operand; the slot set is the wave index ----
    {
      const int q = lane, set = __builtin_amdgcn_readfirstlane(wave);
      const float4 w4 = sW[l & (NS - 1)][q];
      const float* p = sP + q * QS + 3;
#pragma unroll
      for (int S = 0; S < NSLOT; ++S) {
        if ((S & 3) != set) continue;
        float v[8];
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
    __syncthreads();  // tap operand complete; the patches consumed
    stamp();
    // ---- 4. the level's MFMAs: C[channel][pixel] += W[channel][k] * T[k][pixel] ----
#pragma unroll
    for (int g = 0; g < G; ++g) {
      u32x4 (&wc)[8] = bq[(P + g) & 1];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        half8 th[2], tl[2];
        const int chi = 2 * sub + hh, clo = 4 + 2 * sub + hh;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const int pr = mt * 32 + r;
          const uint8_t* row = sA + g * (kQM * 128) + pr * 128;
          th[mt] = *reinterpret_cast<const half8*>(row + ((chi ^ swz(pr)) << 4));
          tl[mt] = *reinterpret_cast<const half8*>(row + ((clo ^ swz(pr)) << 4));
        }
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) {
            const half8 wh = __builtin_bit_cast(half8, wc[(nt * 2 + sub) * 2 + 0]);
            const half8 wl = __builtin_bit_cast(half8, wc[(nt * 2 + sub) * 2 + 1]);
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(th[mt], wl, acc[mt][nt], 0, 0, 0);
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(tl[mt], wh, acc[mt][nt], 0, 0, 0);
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(th[mt], wh, acc[mt][nt], 0, 0, 0);
          }
      }
      const int t2 = l * G + g + 2;
      if (t2 < nlg) load_b(t2, wc);
    }
    stamp();
  };
  for (int l = 0; l < L; l += 2) {
    body(l, std::integral_constant<int, 0>{});
    if (l + 1 < L) body(l + 1, std::integral_constant<int, G & 1>{});
  }

  // ---- epilogue: accumulators -> LDS tile [pixel][channel] -> scale, bias, ReLU -> S32 (the r04 kernel's) ----
  __syncthreads();  // every wave is past its last tap-operand read (the tile overlays the operand and the patches)
  float* sT = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int n = wave * 64 + nt * 32 + r;
#pragma unroll
      for (int e = 0; e < 16; ++e) sT[(mt * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh) * TS + n] = acc[mt][nt][e];
    }
  static_assert(NT % (kN / 8) == 0, "fixed channel octet per thread");
  const int n8 = (tid % (kN / 8)) * 8;
  float2 sbv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sbv[j] = sSB[n8 + j];
  __syncthreads();
  float mx = 0.f;
#pragma unroll
  for (int itr = 0; itr < kQM * (kN / 8) / NT; ++itr) {
    const int pl = (tid + itr * NT) / (kN / 8);
    if (pl >= nq) continue;
    const float4 t0 = *reinterpret_cast<const float4*>(&sT[pl * TS + n8]);
    const float4 t1 = *reinterpret_cast<const float4*>(&sT[pl * TS + n8 + 4]);
    const float v[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
    half8 hi, lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float x = v[j] * sbv[j].x + sbv[j].y;
      x = x < 0.f ? 0.f : x;  // relu (update.py:120); NaN propagates like ATen
      mx = fmaxf(mx, x);
      _Float16 h_, l_;
      split_f16(x, h_, l_);
      hi[j] = h_;
      lo[j] = l_;
    }
    uint8_t* line = a.y + (long long)(q0 + pl) * a.yps + (n8 >> 5) * 128 + ((n8 & 31) >> 3) * 16;
    *reinterpret_cast<half8*>(line) = hi;
    *reinterpret_cast<half8*>(line + 64) = lo;
  }
  range_guard(mx);
  if (a.stamps != nullptr) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  stamp();
}


// r05 variant 6 ("rowmap"): the r04 kernel with the two VALU-heavy parts rebuilt (PMC: 4,751 VALU per wave, ~680 of a
// level's ~1,190 for chunk addressing and patch writes, ~8 per tap for the hi/lo split):
//   * chunk gathers mapped as thread = (query q = tid / 4, chunk column k = tid % 4) x every window row u: the column's
//     byte offset (query base folded in, or a sentinel past the buffer when the column is outside the level or not
//     needed) is formed once per level, each row adds its tile-row / row-in-tile part and is replaced by the sentinel
//     when outside the level (the buffer load then returns zeros without a memory access: Q4's zero padding); the patch
//     write of row u is four ds_write_b32 at immediate offsets from one per-level base (q*QS + 3 - dx + 4k). A level
//     whose width is not a multiple of 4 masks the cells of the one chunk column that crosses its right edge.
//   * split: hi pairs by v_cvt_pk_f16_f32 (RNE), lo = fp16(v - hi) by v_fma_mixlo/mixhi_f16 (v - hi is exact in fp32,
//     so one rounding of the exact difference = the cvt(sub) pair's result), three VALU per two taps instead of ~8.
// Taps, products, order and epilogue as the r04 kernel: bit-identical.
// split_lo_pair: oflow_internal.h

template <int R>
__global__ __launch_bounds__(kNT, 2) void corr_convc1_rowmap_kernel(C1Args a) {
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
  uint8_t* sA = smem;
  float* sP = reinterpret_cast<float*>(smem + A_BYTES);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave;
  const int r = lane & 31, hh = lane >> 5;
  const int q0 = blockIdx.x * kQM;
  const int nq = min(kQM, a.total - q0);
  const int gq = tid >> 2, gk = tid & 3;  // the gather role: query, chunk column
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

  u32x4 rv[PK];
  auto gather = [&](int l) {
    int Hl, Wl, WB, LF;
    const float* base;
    level(l, Hl, Wl, WB, LF, base);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(base + (size_t)q0 * LF), (short)0, nq * LF * 4, 0x00020000);
    if (NCH == 4 || gk < NCH) {
      const int4 o = sO[l & (NS - 1)][gq];
      const int xc = o.x - o.w + 4 * gk;
      const bool cv = static_cast<unsigned>(xc) < static_cast<unsigned>(Wl) && 4 * gk < o.w + PK;
      const unsigned cb = cv ? static_cast<unsigned>(__umul24(gq, LF) * 4 + ((xc >> 3) << 7) + ((xc & 7) << 2)) : SENT;
      const int WB128 = WB * 128;
#pragma unroll
      for (int u = 0; u < PK; ++u) {
        const int y = o.y + u;
        unsigned off = cb + static_cast<unsigned>(__mul24(y >> 2, WB128) + ((y & 3) << 5));
        off = static_cast<unsigned>(y) < static_cast<unsigned>(Hl) ? off : SENT;
        rv[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(off), 0, 0);
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
      const int4 o = sO[l & (NS - 1)][gq];
      int dofs = (A_BYTES / 4) + gq * QS + 3 - o.w + 4 * gk;
      asm volatile("" : "+v"(dofs));  // one base register, immediate offsets
      float* dst = reinterpret_cast<float*>(smem) + dofs;
      if (Wl & 3) {  // the chunk column crossing the right edge: cells past it are tile padding
        const int nv = Wl - (o.x - o.w + 4 * gk);
#pragma unroll
        for (int u = 0; u < PK; ++u) {
          const float* fv = reinterpret_cast<const float*>(&rv[u]);
          dst[u * RW + 0] = fv[0];
          dst[u * RW + 1] = nv > 1 ? fv[1] : 0.f;
          dst[u * RW + 2] = nv > 2 ? fv[2] : 0.f;
          dst[u * RW + 3] = nv > 3 ? fv[3] : 0.f;
        }
      } else {
#pragma unroll
        for (int u = 0; u < PK; ++u) {
          const float* fv = reinterpret_cast<const float*>(&rv[u]);
#pragma unroll
          for (int e = 0; e < 4; ++e) dst[u * RW + e] = fv[e];
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


// r05 variant 7 ("quad"): variant 6 with a gather mapping that keeps each load instruction on few tile lines: lane =
// (query qi of a group of 4, row phase uo, chunk column k), the wave's 16 queries in 4 groups, rows uo + 4m: one
// instruction covers 4 queries x 4 consecutive window rows x 4 chunk columns (~18 lines of 128 B against ~40 for
// variant 6's 16 queries x 1 row), rows m and m+1 of a thread differ by one tile row (one add).
template <int R>
__global__ __launch_bounds__(kNT, 2) void corr_convc1_quad_kernel(C1Args a) {
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
  uint8_t* sA = smem;
  float* sP = reinterpret_cast<float*>(smem + A_BYTES);

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

// r05 variant 8 ("q128"): variant 7 on 128 queries per workgroup (8 waves, one workgroup per CU), each wave 32 output
// channels x all 128 queries (4 m tiles). PMC of the product kernel (profiles/r05/s14_pmc_c1.json): 70 % of its
// vector-memory instructions and ~69 % of its L1->L2 requests are the weight stream (every 64-query workgroup reads
// all 384 KB of convc1's packed weights), and the texture data path is busy 63 % of the kernel; 128 queries per
// workgroup halve the weight stream per query. LDS 154 KB (patches 88.6 + taps 48 + tables 19), epilogue tile
// overlaid. Same products in the same order per accumulator: bit-identical.
template <int R>
__global__ __launch_bounds__(512, 1) void corr_convc1_q128_kernel(C1Args a) {
  constexpr int kNT = 512, kQM = 128;  // 8 waves, 128 queries, one workgroup per CU
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
  static_assert(NCH <= 4, "chunk columns");
  static_assert(3 + 4 * NCH - 1 + (PK - 1) * RW < QS, "a row's chunks stay inside the query's patch");
  __shared__ __attribute__((aligned(16))) uint8_t smem[LDS_BYTES];
  __shared__ float2 sSB[kN];
  __shared__ float2 sC[kQM];
  __shared__ int4 sO[NS][kQM];    // window origin x0, y0, (unused), dx
  __shared__ float4 sW[NS][kQM];  // bilinear weights (nw, ne, sw, se)
  uint8_t* sA = smem;
  float* sP = reinterpret_cast<float*>(smem + A_BYTES);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
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
  if (tid < 2 * kQM) {  // threads 0-127 decode level 0, 128-255 level 1
    float2 c = make_float2(1e30f, 1e30f);  // past the last query: all-zero window
    if (qd < nq) {
      const int q = q0 + qd;
      const int b = q / a.N, pix = q - b * a.N;
      c = make_float2(a.coords[(size_t)(2 * b) * a.N + pix], a.coords[(size_t)(2 * b + 1) * a.N + pix]);
    }
    if (tid < kQM) sC[qd] = c;
    if ((tid >> 7) < a.nlev) decode(tid >> 7, c.x, c.y);
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
  const int wbase = wave * 4096 + lane * 16;  // wave = 32 channels = (64-channel quarter wave / 2, n tile wave & 1)
  u32x4 bq[2][4];
  auto load_b = [&](int t, u32x4 (&dst)[4]) {
    const int so = t * (kN * 128);
#pragma unroll
    for (int e = 0; e < 4; ++e) dst[e] = __builtin_amdgcn_raw_buffer_load_b128(rsW, wbase, so + e * 1024, 0);
  };
  f32x16 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;

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
      u32x4 (&bc)[4] = bq[(P + g) & 1];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        half8 ah[4], al[4];
        const int chi = 2 * sub + hh, clo = 4 + 2 * sub + hh;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const int pr = mt * 32 + r;
          const uint8_t* row = sA + g * (kQM * 128) + pr * 128;
          ah[mt] = *reinterpret_cast<const half8*>(row + ((chi ^ swz(pr)) << 4));
          al[mt] = *reinterpret_cast<const half8*>(row + ((clo ^ swz(pr)) << 4));
        }
        const half8 bh = __builtin_bit_cast(half8, bc[sub * 2 + 0]);
        const half8 bl = __builtin_bit_cast(half8, bc[sub * 2 + 1]);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[mt], bl, acc[mt], 0, 0, 0);
          acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[mt], bh, acc[mt], 0, 0, 0);
          acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[mt], bh, acc[mt], 0, 0, 0);
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
  for (int mt = 0; mt < 4; ++mt) {
    const int n = wave * 32 + r;
    const int pbase = mt * 32;
#pragma unroll
    for (int e = 0; e < 16; ++e) sT[(pbase + (e & 3) + 8 * (e >> 2) + 4 * hh) * TS + n] = acc[mt][e];
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

}  // namespace
// keeps the range guards' flag pointer (and so their code) alive, as in the product library
OFLOW_RANGE_FLAG_SETTER(c1var)
}  // namespace oflow

using namespace oflow;

// the product ABI's arguments (include/oflow.h oflow_corr_lookup_convc1_s32) + the variant and an optional stamp buffer
extern "C" int oflow_exp_convc1_variant(int variant, const float* const* d_levels, const int* level_h, const int* level_w,
                                        int num_levels, const float* d_coords, int B, int H, int W, int radius,
                                        const void* d_wpack, const float* d_wscale, const float* d_bias, void* d_y,
                                        long long y_pixel_stride, void* stamps, void* stream) {
  if (!d_levels || !level_h || !level_w || !d_coords || !d_wpack || !d_wscale || !d_y) return OFLOW_E_NULL;
  if (B <= 0 || H <= 0 || W <= 0) return OFLOW_E_SHAPE;
  if (num_levels < 1 || num_levels > OFLOW_MAX_LEVELS) return OFLOW_E_LEVELS;
  if (radius != 3 && radius != 4) return OFLOW_E_RADIUS;
  C1Args a{};
  for (int l = 0; l < num_levels; ++l) {
    if (level_h[l] < 2 || level_w[l] < 2) return OFLOW_E_TINY;
    a.lv[l] = d_levels[l];
    a.Hl[l] = level_h[l];
    a.Wl[l] = level_w[l];
    a.WB[l] = (level_w[l] + 7) / 8;
    a.LF[l] = ((level_h[l] + 3) / 4) * a.WB[l] * 32;
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
  a.stamps = static_cast<unsigned long long*>(stamps);
  const dim3 grid((a.total + kQM - 1) / kQM);
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (variant * 10 + radius) {
    case 24: hipLaunchKernelGGL((corr_convc1_w8_kernel<4>), grid, dim3(512), 0, s, a); break;
    case 23: hipLaunchKernelGGL((corr_convc1_w8_kernel<3>), grid, dim3(512), 0, s, a); break;
    case 34: hipLaunchKernelGGL((corr_convc1_pipe_kernel<4>), grid, dim3(256), 0, s, a); break;
    case 33: hipLaunchKernelGGL((corr_convc1_pipe_kernel<3>), grid, dim3(256), 0, s, a); break;
    case 44: hipLaunchKernelGGL((corr_convc1_lean_kernel<4>), grid, dim3(256), 0, s, a); break;
    case 43: hipLaunchKernelGGL((corr_convc1_lean_kernel<3>), grid, dim3(256), 0, s, a); break;
    case 54: hipLaunchKernelGGL((corr_convc1_hyb_kernel<4>), grid, dim3(256), 0, s, a); break;
    case 53: hipLaunchKernelGGL((corr_convc1_hyb_kernel<3>), grid, dim3(256), 0, s, a); break;
    case 64: hipLaunchKernelGGL((corr_convc1_rowmap_kernel<4>), grid, dim3(256), 0, s, a); break;
    case 63: hipLaunchKernelGGL((corr_convc1_rowmap_kernel<3>), grid, dim3(256), 0, s, a); break;
    case 74: hipLaunchKernelGGL((corr_convc1_quad_kernel<4>), grid, dim3(256), 0, s, a); break;
    case 73: hipLaunchKernelGGL((corr_convc1_quad_kernel<3>), grid, dim3(256), 0, s, a); break;
    case 84: hipLaunchKernelGGL((corr_convc1_q128_kernel<4>), dim3((a.total + 127) / 128), dim3(512), 0, s, a); break;
    case 83: hipLaunchKernelGGL((corr_convc1_q128_kernel<3>), dim3((a.total + 127) / 128), dim3(512), 0, s, a); break;
    default: return OFLOW_E_MODE;
  }
  return launch_status();
}
