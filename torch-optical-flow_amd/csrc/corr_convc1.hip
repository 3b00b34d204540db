// Correlation lookup fused into the motion encoder's first convolution (gfx950).
//
// Replaces, in the RAFT forward, `corr = corr_fn(coords1)` (methods/raft/model/raft.py:128 -> corr.py:56-77) followed
// by `F.relu(self.convc1(corr))` (update.py:120-121, a 1x1 conv L*(2r+1)^2 -> 256): the (B, 324, H, W) lookup volume
// never reaches HBM. Per workgroup of 64 query pixels (4 waves; two workgroups per CU, so one's gather / tap phases
// overlap the other's MFMAs), level by level:
//   1. the (2r+2)^2 window patches of the level, gathered from the tiled pyramid (4x8 tiles = 128-B lines, the
//      layout corr_lookup.hip reads; 25 scalar loads per thread, issued during the previous level's last MFMAs), are
//      written to LDS (odd per-query stride);
//   2. the (2r+1)^2 bilinear taps of each query (bilinear4: the lookup kernels' arithmetic, bit for bit) become the
//      level's split-fp16 A operand in LDS: [k32 group][pixel][hi 32 | lo 32], 16-B slots XOR-swizzled, one thread per
//      (pixel, 8-tap slot) writing whole 16-B slots; taps past (2r+1)^2 in the level's last group stay zero;
//   3. each wave (64 pixels x 64 output channels) runs the level's G k32 groups as split-fp16 products on
//      v_mfma_f32_32x32x16_f16 (hi*lo + lo*hi + hi*hi, fp32 accumulate: conv_s32.hip's arithmetic); the weights
//      stream one k32 group (256 channels x 128 B) at a time through LDS over the dead patches, register-staged one
//      group ahead.
// Epilogue: accumulators -> LDS [pixel][channel] fp32 -> per-channel weight scale, bias, ReLU -> S32 store of the 256
// output channels (convc2's input).
//
// Weights: oflow_conv_s32's packing of convc1 with its input channels regrouped per level: level l's tap k at packed
// channel l*G*32 + k (G = ceil((2r+1)^2 / 32)); the other channels are zero. Radius 3 (G = 2) and 4 (G = 3).
// LDS: A G*8 KB + weights/patches 32 KB, epilogue tile overlay 66.5 KB, + 5.5 KB (two workgroups per CU).
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
  const uint8_t* w;     // packed weights [nlev * G][256][hi | lo]
  const float* wsc;     // [256] inverse weight scale
  const float* bias;    // [256] or null
  uint8_t* y;           // S32 destination (8 groups of one pixel from y + P * yps)
  long long yps;
};

template <int R>
__global__ __launch_bounds__(kNT, 2) void corr_convc1_kernel(C1Args a) {
  constexpr int PK = 2 * R + 2, K = 2 * R + 1, KK = K * K, PS = PK * PK, QS = PS + 1;
  constexpr int G = (KK + 31) / 32;      // k32 groups per level
  constexpr int NSLOT = (KK + 7) / 8;    // 8-tap slots that hold taps
  constexpr int A_BYTES = G * kQM * 128;
  constexpr int B_BYTES = kN * 128;      // one k32 weight group
  constexpr int P_BYTES = kQM * QS * 4;
  constexpr int TS = kN + 4;             // epilogue tile row (floats)
  constexpr int EPI_BYTES = kQM * TS * 4;
  constexpr int MAIN = A_BYTES + B_BYTES;
  constexpr int LDS_BYTES = MAIN > EPI_BYTES ? MAIN : EPI_BYTES;
  constexpr int GI = (kQM * PS + kNT - 1) / kNT;  // gather items per thread
  constexpr int BI = kN * 128 / (16 * kNT);        // 16-B weight chunks per thread and group
  static_assert(P_BYTES <= B_BYTES, "patches alias the weight buffer");
  static_assert(kN * 128 % (16 * kNT) == 0, "weight chunks");
  __shared__ __attribute__((aligned(16))) uint8_t smem[LDS_BYTES];
  __shared__ float2 sSB[kN];      // per channel (inverse weight scale, bias) for the epilogue
  __shared__ float2 sC[kQM];      // the queries' coordinates
  __shared__ int2 sO[2][kQM];     // per level parity: window origin (x, y)
  __shared__ float4 sW[2][kQM];   // bilinear weights (nw, ne, sw, se)
  uint8_t* sA = smem;
  uint8_t* sB = smem + A_BYTES;
  float* sP = reinterpret_cast<float*>(sB);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave;
  const int r = lane & 31, hh = lane >> 5;
  const int q0 = blockIdx.x * kQM;
  const int nq = min(kQM, a.total - q0);

  for (int c = tid; c < kN; c += kNT) sSB[c] = make_float2(a.wsc[c], a.bias ? a.bias[c] : 0.f);
  if (tid < kQM) {
    float2 c = make_float2(1e30f, 1e30f);  // past the last query: all-zero window
    if (tid < nq) {
      const int q = q0 + tid;
      const int b = q / a.N, pix = q - b * a.N;
      c = make_float2(a.coords[(size_t)(2 * b) * a.N + pix], a.coords[(size_t)(2 * b + 1) * a.N + pix]);
    }
    sC[tid] = c;
  }
  // window origin + bilinear weights of each query at level l -> sO / sW[l & 1] (threads < kQM; coords from sC, so the
  // caller orders this after a barrier that follows the sC stores)
  auto decode = [&](int l) {
    if (tid < kQM) {
      int xs, ys;
      float4 w4;
      window_origin(sC[tid].x, sC[tid].y, 1.0f / static_cast<float>(1 << l), R, xs, ys, w4);  // 1/2^l exact (corr.py:68)
      sO[l & 1][tid] = make_int2(xs, ys);
      sW[l & 1][tid] = w4;
    }
  };
  decode(0);
  // A's taps past KK (the last group's tail) are never written again: zero the whole A buffer once
  for (int e = tid; e < A_BYTES / 16; e += kNT) reinterpret_cast<u32x4*>(sA)[e] = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();

  // level geometry without dynamic indexing of the kernel arguments
  auto level = [&](int l, int& Hl, int& Wl, int& WB, int& LF, const float*& base) {
    Hl = a.Hl[0]; Wl = a.Wl[0]; WB = a.WB[0]; LF = a.LF[0]; base = a.lv[0];
#pragma unroll
    for (int j = 1; j < OFLOW_MAX_LEVELS; ++j)
      if (j == l) { Hl = a.Hl[j]; Wl = a.Wl[j]; WB = a.WB[j]; LF = a.LF[j]; base = a.lv[j]; }
  };
  float rv[GI];
  unsigned okm = 0u;  // bit s: gather item s is inside its level
  static_assert(GI <= 32, "okm bits");
  u32x4 rb[BI];
  // gather level l's patches into rv (item = (query, patch row u, patch column c))
  auto gather = [&](int l) {
    int Hl, Wl, WB, LF;
    const float* base;
    level(l, Hl, Wl, WB, LF, base);
    // the workgroup's queries of the level as one buffer; a tap outside the level loads the query block's first
    // float and is zeroed through okm when staged (no exec branches: vmcnt is counted exactly; the buffer's
    // out-of-range zero fill is not relied on)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(base + (size_t)q0 * LF), (short)0, nq * LF * 4, 0x00020000);
    int t = tid;
    asm volatile("" : "+v"(t));  // opaque per call: the item decode below is recomputed, not hoisted into 25 live regs
    okm = 0u;
#pragma unroll
    for (int s = 0; s < GI; ++s) {
      const int item = min(t + kNT * s, kQM * PS - 1);
      const int q = item / PS;
      const int rm = item - q * PS;
      const int u = rm / PK, c = rm - u * PK;
      const int2 o = sO[l & 1][q];
      const int y = o.y + u, x = o.x + c;
      const bool ok = static_cast<unsigned>(y) < static_cast<unsigned>(Hl) && static_cast<unsigned>(x) < static_cast<unsigned>(Wl);
      const int off = ok ? (q * LF + ((y >> 2) * WB + (x >> 3)) * 32 + ((y & 3) << 3) + (x & 7)) * 4 : 0;
      okm |= (ok ? 1u : 0u) << s;
      rv[s] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
    }
  };
  // one k32 group of weights (256 channels x 128 B) per step: chunk c -> channel c / 8, 16-B slot c % 8
  auto load_w = [&](int l, int g) {
    const uint8_t* wg = a.w + (size_t)(l * G + g) * (kN * 128);
#pragma unroll
    for (int s = 0; s < BI; ++s) rb[s] = *reinterpret_cast<const u32x4*>(wg + (size_t)(tid + kNT * s) * 16);
  };
  auto write_w = [&]() {
#pragma unroll
    for (int s = 0; s < BI; ++s) {
      const int c = tid + kNT * s, n = c >> 3, sl = c & 7;
      *reinterpret_cast<u32x4*>(sB + n * 128 + ((sl ^ swz(n)) << 4)) = rb[s];
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  load_w(0, 0);
  gather(0);
  for (int l = 0; l < a.nlev; ++l) {
    // ---- 1. patches -> LDS (over the weight buffer: the previous level's MFMAs are done) ----
#pragma unroll
    for (int s = 0; s < GI; ++s) {
      const int item = tid + kNT * s;
      if (item < kQM * PS) {
        const int q = item / PS;
        sP[q * QS + (item - q * PS)] = ((okm >> s) & 1u) ? rv[s] : 0.0f;
      }
    }
    __syncthreads();
    // ---- 2. bilinear taps -> split-fp16 A operand: thread = (pixel q, slots S = set, set + 4, ...) ----
    {
      const int q = tid & (kQM - 1), set = tid / kQM;  // set (= wave) is uniform per wave
      const float4 w4 = sW[l & 1][q];
      const float* p = sP + q * QS;
#pragma unroll
      for (int S = 0; S < NSLOT; ++S) {
        if ((S & 3) != set) continue;
        half8 hi, lo;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int k = 8 * S + e;  // reference channel order within the level: k = i*K + j, i moves x, j moves y
          float v = 0.f;
          if (k < KK) {
            const int i = k / K, j = k - (k / K) * K;
            v = bilinear4(p[j * PK + i], p[j * PK + i + 1], p[(j + 1) * PK + i], p[(j + 1) * PK + i + 1], w4);
          }
          _Float16 h_, l_;
          split_f16(v, h_, l_);
          hi[e] = h_;
          lo[e] = l_;
        }
        uint8_t* row = sA + (S >> 2) * (kQM * 128) + q * 128;
        *reinterpret_cast<half8*>(row + (((S & 3) ^ swz(q)) << 4)) = hi;
        *reinterpret_cast<half8*>(row + (((4 + (S & 3)) ^ swz(q)) << 4)) = lo;
      }
    }
    if (l + 1 < a.nlev) decode(l + 1);
    __syncthreads();  // patches dead (the weight buffer is free), A complete, the next level's windows decoded
    // ---- 3. the level's k32 groups: weights (held in rb since the previous group) -> LDS, the next group's (or the
    // next level's first) weights loaded, then the group's MFMAs. The next level's gathers are issued after the
    // level's last weight load (vmcnt retires in order: a weight wait never waits for them) and fly during the last
    // group's MFMAs; the other workgroup on the CU covers what they do not hide. ----
    half8 ah[2][2], al[2][2], bh[2][2], bl[2][2];  // [sub-step][tile]
    auto read_ops = [&](int g, int sub) {
      const int chi = 2 * sub + hh, clo = 4 + 2 * sub + hh;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int pr = mt * 32 + r;
        const uint8_t* row = sA + g * (kQM * 128) + pr * 128;
        ah[sub][mt] = *reinterpret_cast<const half8*>(row + ((chi ^ swz(pr)) << 4));
        al[sub][mt] = *reinterpret_cast<const half8*>(row + ((clo ^ swz(pr)) << 4));
      }
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int n = wn * 64 + nt * 32 + r;
        const uint8_t* row = sB + n * 128;
        bh[sub][nt] = *reinterpret_cast<const half8*>(row + ((chi ^ swz(n)) << 4));
        bl[sub][nt] = *reinterpret_cast<const half8*>(row + ((clo ^ swz(n)) << 4));
      }
    };
#pragma unroll
    for (int g = 0; g < G; ++g) {
      write_w();
      if (g + 1 < G) {
        load_w(l, g + 1);
      } else if (l + 1 < a.nlev) {
        load_w(l + 1, 0);
        gather(l + 1);
      }
      __syncthreads();  // group g's weights visible
      read_ops(g, 0);
      read_ops(g, 1);
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) {
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[sub][mt], bl[sub][nt], acc[mt][nt], 0, 0, 0);
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[sub][mt], bh[sub][nt], acc[mt][nt], 0, 0, 0);
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[sub][mt], bh[sub][nt], acc[mt][nt], 0, 0, 0);
          }
      __syncthreads();  // group g's operand reads done: the weight buffer (and at the level's end the patch / A
                        // buffers) may be overwritten
    }
  }

  // ---- epilogue: accumulators -> LDS tile [pixel][channel] -> scale, bias, ReLU -> S32 ----
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
  __syncthreads();
  for (int item = tid; item < kQM * (kN / 8); item += kNT) {
    const int pl = item / (kN / 8), n = (item - pl * (kN / 8)) * 8;
    if (pl >= nq) continue;
    const float4 t0 = *reinterpret_cast<const float4*>(&sT[pl * TS + n]);
    const float4 t1 = *reinterpret_cast<const float4*>(&sT[pl * TS + n + 4]);
    const float v[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
    half8 hi, lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float2 sb = sSB[n + j];
      float x = v[j] * sb.x + sb.y;
      x = x < 0.f ? 0.f : x;  // relu (update.py:120); NaN propagates like ATen
      _Float16 h_, l_;
      split_f16(x, h_, l_);
      hi[j] = h_;
      lo[j] = l_;
    }
    uint8_t* line = a.y + (long long)(q0 + pl) * a.yps + (n >> 5) * 128 + ((n & 31) >> 3) * 16;
    *reinterpret_cast<half8*>(line) = hi;
    *reinterpret_cast<half8*>(line + 64) = lo;
  }
}

}  // namespace
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
  }
  a.nlev = num_levels;
  a.coords = d_coords;
  a.N = H * W;
  a.total = B * H * W;
  a.w = static_cast<const uint8_t*>(d_wpack);
  a.wsc = d_wscale;
  a.bias = d_bias;
  a.y = static_cast<uint8_t*>(d_y);
  a.yps = y_pixel_stride;
  const dim3 grid((a.total + kQM - 1) / kQM);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (radius == 4)
    hipLaunchKernelGGL((corr_convc1_kernel<4>), grid, dim3(kNT), 0, s, a);
  else
    hipLaunchKernelGGL((corr_convc1_kernel<3>), grid, dim3(kNT), 0, s, a);
  return launch_status();
}
