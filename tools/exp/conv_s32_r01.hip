// EXPERIMENT RECORD (not product code): the round-1 conv_s32 kernel with its VAR schedule hooks and ablations
// (BREG register-direct weights, PADL rows, setprio, no-load / no-barrier ablations), kept for A/B runs
// (tools/exp/conv_exp.hip, run_conv_exp.py). The product kernel is torch-optical-flow_amd/csrc/conv_s32.hip.
//
// Split-fp16 implicit-GEMM convolution for the RAFT update block (gfx950).
//
// Replaces the nn.Conv2d layers of methods/raft/model/update.py:40-161 (BasicMotionEncoder, SepConvGRU,
// FlowHead, mask head) at fp32 accuracy on the fp16 matrix cores.
//
// Numerics. Every operand is carried as an unevaluated sum of two fp16 values, x = hi + lo (hi = fp16(x),
// lo = fp16(x - hi): 22 significant bits), and every product as three v_mfma_f32_32x32x16_f16:
// hi*hi + hi*lo + lo*hi (the lo*lo term is below fp32 rounding), accumulated in fp32. Weights are scaled per
// output channel by a power of two (max |w| -> 2^14, undone exactly in the epilogue) so that their lo parts stay
// normal fp16. tools/exp/split_numerics.py measured RAFT at Sintel size with this arithmetic: 3.7e-6 px mean
// EPE against the reference's fp32 CPU flow, the same as fp32 reordering noise.
//
// Activation format "S32" (include/oflow.h): NHWC by groups of 32 channels, one group of one pixel = one 128-B
// line = hi[32] fp16 then lo[32] fp16. A channel slice of a wider S32 buffer is (base + g0 * 128, pixel stride).
// Packed weights: [input groups][taps][n_pad][hi[32] | lo[32]] fp16 (the same line format, one line per output
// channel and k32 chunk), so both MFMA operands stage as whole lines.
//
// Workgroup tile: 4 output rows x 32 output columns (128 pixels) x BN output channels; 4 waves as WM x WN.
// Loop: input groups (k32) outer, taps inner. Per group the (4 + KH - 1) x (32 + KW - 1) input halo is staged in
// LDS once and read by every tap at a shifted offset; per (group, tap) a BN x 128-B weight slab is staged (double
// buffered). Both are register-staged one step ahead. LDS lines are 16-B-slot swizzled (slot ^= (row >> 1) & 7)
// so that the 32 rows of an MFMA operand read by ds_read_b128 are bank-conflict free from any starting row.
// Epilogue: accumulators -> LDS tile [pixel][channel] fp32 -> per-channel scale, bias, activation and the fused
// consumer (S32 stores with 16-B chunks, GRU gates, fp32 NCHW store/accumulate).
#include "oflow_internal.h"

namespace oflow {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));  // native vector: stays in VGPRs (HIP uint4 is copied by memcpy)

constexpr int kTY = 4, kTX = 32, kThreads = 256;  // default tile: kTY rows x kTX columns
constexpr int kAinGroups = 4;                      // AIN inputs: up to 128 channels (the encoders' 64 / 96 / 128)

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

struct ConvArgs {
  const uint8_t* x;        // S32 input, first group of the slice
  long long xps;           // input pixel stride (bytes)
  int kg;                  // input groups (k32 chunks)
  const uint8_t* w;        // packed weights
  int npad;                // padded output channels in the packing
  const float* wsc;        // [npad] inverse weight scale
  const float* bias;       // [N] or null
  int N;                   // real output channels
  int B, H, W, tiles_x, tiles_y;
  int act;                 // 0 none, 1 relu, 2 sigmoid, 3 tanh
  float oscale;            // applied after the activation
  uint8_t* y0;             // S32 destination 0 (first group) or null
  long long y0ps;
  uint8_t* y1;             // S32 destination 1 or null
  long long y1ps;
  float* f;                // fp32 NCHW destination or null
  long long fbs, fcs;      // its batch / channel strides (floats)
  int faccum;              // 1: f += value
  // GRU (EPI 1 = z|r gates, EPI 2 = candidate + blend); NHWC fp32 [P][gch]
  float* h;
  float* z;
  int gch;
  // encoder options (EPI 0)
  float* fn;               // fp32 NHWC destination [P][fnps] (pre-activation value when stats are taken) or null
  int fnps;
  float* stats;            // per-tile (count, mean, M2) partials [B][tiles][npad][3] of the conv output, or null
  const uint8_t* res;      // S32 residual added after the activation (then res_act), or null
  long long resps;
  int res_act;
  int s2d;                 // S32 destinations in space-to-depth layout: pixel (y/2, x/2), channel + ((y&1)*2+(x&1))*N
  // fp32 NHWC input normalised on load (AIN): x = relu(raw * ia[b, c] + ib[b, c]) -- the previous conv's instance
  // norm + ReLU (extractor.py:75-76) folded into this conv's operand staging; [B][kg*32] each, or null (S32 input)
  const float* ia;
  const float* ib;
  int ain;                 // input format: kInS32 / kInF32Norm / kInF32
  int cin;                 // kInF32: real input channels (row pitch cin * 4 B); channels >= cin stage as zeros
};
// input formats of oflow_conv_s32_ex2
constexpr int kInS32 = OFLOW_IN_S32, kInF32Norm = OFLOW_IN_F32_NORM, kInF32 = OFLOW_IN_F32;

__device__ __forceinline__ float act_fn(float v, int act) {
  if (act == 1) return v < 0.f ? 0.f : v;  // relu; NaN propagates like ATen
  if (act == 2) return 1.0f / (1.0f + expf(-v));
  if (act == 3) return tanhf(v);
  return v;
}

__device__ __forceinline__ void split8(const float* v, half8& hi, half8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const _Float16 a = static_cast<_Float16>(v[j]);
    hi[j] = a;
    lo[j] = static_cast<_Float16>(v[j] - static_cast<float>(a));
  }
}

// store channels [n, n + 8) of pixel P (n % 8 == 0) into an S32 destination, only those < N
__device__ __forceinline__ void store_s32(uint8_t* y, long long ps, long long P, int n, int N, const float* v) {
  uint8_t* line = y + P * ps + (long long)(n >> 5) * 128 + ((n & 31) >> 3) * 16;
  if (n + 8 <= N) {
    half8 hi, lo;
    split8(v, hi, lo);
    *reinterpret_cast<half8*>(line) = hi;
    *reinterpret_cast<half8*>(line + 64) = lo;
  } else {
    _Float16* hp = reinterpret_cast<_Float16*>(line);
    _Float16* lp = reinterpret_cast<_Float16*>(line + 64);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (n + j < N) {
        const _Float16 a = static_cast<_Float16>(v[j]);
        hp[j] = a;
        lp[j] = static_cast<_Float16>(v[j] - static_cast<float>(a));
      }
    }
  }
}

// VAR (experiment hooks, 0 in the product): bit 0 s_setprio(1) around each MFMA block; bit 1 issue both K-halves'
// LDS operand reads before the MFMAs; bit 2 ask for 3 waves per SIMD; bit 3 (launcher) 8-row tiles for BN 64;
// bits 4-6 see BREG / PADL / launch_128. Ablations (wrong results, timing only): bit 7 no global loads in the loop,
// bit 9 no per-step barrier.
// BREG: the weight fragments go straight from global memory (L2) into registers, one step of lead, instead of
// through LDS: no weight slab in LDS and no per-step barrier (A changes once per group); waves as 1 x 4.
// AIN: kInF32Norm = fp32 NHWC [P][kg*32] input normalised + ReLU'd while staged (ConvArgs.ia / .ib, kg <= kAinGroups);
// kInF32 = fp32 NHWC input split into hi + lo while staged (the NHWC corr lookup feeding convc1).
template <int KH, int KW, int BN, int WM, int WN, int EPI, int VAR = 0, int TY = kTY, bool BREG = false, int AIN = kInS32>
__global__ __launch_bounds__(kThreads, (VAR & 4) ? 3 : 2) void conv_s32_kernel(ConvArgs a) {
  constexpr int T = KH * KW;
  constexpr int BM = TY * kTX;  // output pixels per workgroup (TY rows x 32 columns)
  constexpr int PH = KH / 2, PW = KW / 2;
  constexpr int HY = TY + KH - 1, HX = kTX + KW - 1, NPIX = HY * HX;
  constexpr int AITEMS = NPIX * 8, APER = (AITEMS + kThreads - 1) / kThreads;
  constexpr int BITEMS = BN * 8, BPER = (BITEMS + kThreads - 1) / kThreads;
  constexpr int MT = TY / WM;            // 32-pixel row tiles per wave
  constexpr int NT = BN / WN / 32;        // 32-channel column tiles per wave
  static_assert(WM * WN == 4 && MT >= 1 && NT >= 1, "bad wave grid");
  // T == 1 (1x1 convs): the input tile changes every K-step, so A is staged like B (double buffered in LDS).
  constexpr bool ADB = (T == 1);
  // LDS row format: PADL (VAR bit 5) = 144-B rows (128 B + 16 B pad: rows r and r+1 start 9 slots apart, so any 16
  // consecutive rows of a ds_read_b128 cover distinct bank groups) with affine addressing; else 128-B rows with the
  // 16-B slot XOR swizzle (slot ^= (row >> 1) & 7), whose per-lane address math is redone every step.
  constexpr bool PADL = (VAR & 32) != 0;
  constexpr int RS = PADL ? 144 : 128;
  constexpr int A_BYTES = NPIX * RS, B_BYTES = BN * RS;
  constexpr int MAIN_BYTES = (ADB ? 2 : 1) * A_BYTES + (BREG ? 0 : 2 * B_BYTES);
  constexpr int TS = BN + 4;              // epilogue tile row stride (floats)
  constexpr int EPI_BYTES = BM * TS * 4;
  constexpr int LDS_BYTES = MAIN_BYTES > EPI_BYTES ? MAIN_BYTES : EPI_BYTES;
  constexpr int AFF_BYTES = AIN == kInF32Norm ? kAinGroups * 32 * 8 : 0;  // float2 (scale, shift) per input channel
  __shared__ __attribute__((aligned(16))) uint8_t smem[LDS_BYTES + AFF_BYTES];
  float2* sAff = reinterpret_cast<float2*>(smem + LDS_BYTES);
  uint8_t* sA = smem;
  uint8_t* sB = smem + (ADB ? 2 : 1) * A_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int r = lane & 31, hh = lane >> 5;

  int tile = blockIdx.x;
  const int tx0 = (tile % a.tiles_x) * kTX;
  tile /= a.tiles_x;
  const int ty0 = (tile % a.tiles_y) * TY;
  const int b = tile / a.tiles_y;
  const int n0 = blockIdx.y * BN;
  const long long pix0 = (long long)b * a.H * a.W;

  // Software pipeline. B (weights of one (group, tap) step) is register-staged TWO steps ahead in two register sets
  // (rb0 / rb1, alternating by step parity: the loop is unrolled by two so that every register index is static) and
  // double buffered in LDS. A (the input halo of one group) is loaded at the group's first tap and written to LDS at
  // its last (T steps of lead); for 1x1 convs A follows B's two-step scheme.
  u32x4 ra0[APER], ra1[APER], rb0[BPER], rb1[BPER];
  // Every global load of the loop is unconditional (no exec branches around it), so that the compiler can count
  // vmcnt precisely instead of draining the queue: halo pixels outside the image load a clamped in-image pixel and
  // are zeroed when written to LDS (the in/out mask and the per-item offsets do not depend on the group).
  long long aoff[APER];
  int acol[APER];  // kInF32: byte offset of the item's 4 channels within a 32-channel group (added per group, clamped)
  unsigned aok = 0u;
#pragma unroll
  for (int s_ = 0; s_ < APER; ++s_) {
    const int item = (AITEMS % kThreads == 0) ? tid + s_ * kThreads : min(tid + s_ * kThreads, AITEMS - 1);
    const int p = item >> 3, c = item & 7;
    const int gy = ty0 - PH + p / HX, gx = tx0 - PW + p % HX;
    const bool ok = static_cast<unsigned>(gy) < static_cast<unsigned>(a.H) && static_cast<unsigned>(gx) < static_cast<unsigned>(a.W);
    const int cy = min(max(gy, 0), a.H - 1), cx = min(max(gx, 0), a.W - 1);
    aoff[s_] = (pix0 + (long long)cy * a.W + cx) * a.xps + (AIN == kInF32 ? 0 : c * 16);
    acol[s_] = c * 16;
    aok |= (ok ? 1u : 0u) << s_;
  }
#define OFLOW_LOAD_A(RA, G)                                                                                          \
  _Pragma("unroll") for (int s_ = 0; s_ < APER; ++s_) {                                                              \
    if constexpr (AIN == kInF32) /* rows of cin floats: channels past cin re-read the row's last 16 B (zeroed) */   \
      RA[s_] = *reinterpret_cast<const u32x4*>(a.x + aoff[s_] + min((G) * 128 + acol[s_], a.cin * 4 - 16));        \
    else                                                                                                             \
      RA[s_] = *reinterpret_cast<const u32x4*>(a.x + aoff[s_] + (long long)(G) * 128);                              \
  }
#define OFLOW_WRITE_A(RA, BUF, G)                                                                                    \
  _Pragma("unroll") for (int s_ = 0; s_ < APER; ++s_) {                                                              \
    const int item = tid + s_ * kThreads;                                                                            \
    const int p = item >> 3, c = item & 7;                                                                           \
    if (AITEMS % kThreads == 0 || item < AITEMS) {                                                                   \
      if constexpr (AIN != kInS32) {                                                                                 \
        /* 4 fp32 channels (G*32 + 4c ..) [-> relu(x * scale + shift)] -> 4 hi + 4 lo halves (8 B each) */           \
        typedef _Float16 half4_ __attribute__((ext_vector_type(4)));                                                 \
        half4_ h4 = {0, 0, 0, 0}, l4 = {0, 0, 0, 0};                                                                 \
        if (((aok >> s_) & 1u) && (AIN != kInF32 || (G) * 32 + 4 * c < a.cin)) {                                    \
          const float* fv = reinterpret_cast<const float*>(&RA[s_]);                                                 \
          _Pragma("unroll") for (int e_ = 0; e_ < 4; ++e_) {                                                         \
            float v_ = fv[e_];                                                                                       \
            if constexpr (AIN == kInF32Norm) {                                                                       \
              const float2 af = sAff[(G) * 32 + 4 * c + e_];                                                         \
              v_ = v_ * af.x + af.y;                                                                                 \
              v_ = v_ < 0.f ? 0.f : v_;                                                                              \
            }                                                                                                        \
            const _Float16 hv = static_cast<_Float16>(v_);                                                           \
            h4[e_] = hv;                                                                                             \
            l4[e_] = static_cast<_Float16>(v_ - static_cast<float>(hv));                                             \
          }                                                                                                          \
        }                                                                                                            \
        uint8_t* rw_ = sA + (BUF) * A_BYTES + p * RS + (c & 1) * 8;                                                  \
        *reinterpret_cast<half4_*>(rw_ + ((PADL ? (c >> 1) : ((c >> 1) ^ swz(p))) << 4)) = h4;                       \
        *reinterpret_cast<half4_*>(rw_ + ((PADL ? 4 + (c >> 1) : ((4 + (c >> 1)) ^ swz(p))) << 4)) = l4;             \
      } else {                                                                                                       \
        *reinterpret_cast<u32x4*>(sA + (BUF) * A_BYTES + p * RS + ((PADL ? c : (c ^ swz(p))) << 4)) =               \
            ((aok >> s_) & 1u) ? RA[s_] : u32x4{0u, 0u, 0u, 0u};                                                     \
      }                                                                                                              \
    }                                                                                                                \
  }
#define OFLOW_LOAD_B(RB, STEP)                                                                                       \
  _Pragma("unroll") for (int s_ = 0; s_ < BPER; ++s_) {                                                              \
    const int item = tid + s_ * kThreads;                                                                            \
    if (BITEMS % kThreads == 0 || item < BITEMS)                                                                     \
      RB[s_] = *reinterpret_cast<const u32x4*>(a.w + ((long long)(STEP) * a.npad + n0) * 128 + item * 16);           \
  }
#define OFLOW_WRITE_B(RB, BUF)                                                                                       \
  _Pragma("unroll") for (int s_ = 0; s_ < BPER; ++s_) {                                                              \
    const int item = tid + s_ * kThreads;                                                                            \
    const int n = item >> 3, c = item & 7;                                                                           \
    if (BITEMS % kThreads == 0 || item < BITEMS)                                                                     \
      *reinterpret_cast<u32x4*>(sB + (BUF) * B_BYTES + n * RS + ((PADL ? c : (c ^ swz(n))) << 4)) = RB[s_];         \
  }

  f32x16 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int S = a.kg * T;
  // BREG fragment sets: [sub-step][nt], set 0 = even steps, set 1 = odd steps
  half8 f0h[2][NT], f0l[2][NT], f1h[2][NT], f1l[2][NT];
#define OFLOW_LOAD_F(FH, FL, STEP)                                                                                   \
  _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_)                                                                   \
    _Pragma("unroll") for (int nt_ = 0; nt_ < NT; ++nt_) {                                                           \
      const uint8_t* row_ = a.w + ((long long)(STEP) * a.npad + n0 + wn * (BN / WN) + nt_ * 32 + r) * 128;          \
      FH[s_][nt_] = *reinterpret_cast<const half8*>(row_ + (2 * s_ + hh) * 16);                                      \
      FL[s_][nt_] = *reinterpret_cast<const half8*>(row_ + (4 + 2 * s_ + hh) * 16);                                  \
    }
  if constexpr (AIN == kInF32Norm) {
    for (int e = tid; e < a.kg * 32; e += kThreads)
      sAff[e] = make_float2(a.ia[(long long)b * a.kg * 32 + e], a.ib[(long long)b * a.kg * 32 + e]);
    __syncthreads();
  }
  OFLOW_LOAD_A(ra0, 0);
  if constexpr (BREG) {
    OFLOW_LOAD_F(f0h, f0l, 0);
    OFLOW_LOAD_F(f1h, f1l, S > 1 ? 1 : 0);
  } else {
    OFLOW_LOAD_B(rb0, 0);
  }
  OFLOW_WRITE_A(ra0, 0, 0);
  if constexpr (!BREG) { OFLOW_WRITE_B(rb0, 0); }
  if (S > 1) {
    if constexpr (!BREG) { OFLOW_LOAD_B(rb1, 1); }
    if constexpr (ADB) { OFLOW_LOAD_A(ra1, 1); }
  }
  __syncthreads();

#define OFLOW_MFMA_BLOCK(S_)                                                                                         \
  {                                                                                                                  \
    if constexpr ((VAR & 1) != 0) __builtin_amdgcn_s_setprio(1);                                                     \
    _Pragma("unroll") for (int mt = 0; mt < MT; ++mt)                                                                \
      _Pragma("unroll") for (int nt = 0; nt < NT; ++nt) {                                                            \
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi[S_][mt], blo[S_][nt], acc[mt][nt], 0, 0, 0);        \
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(alo[S_][mt], bhi[S_][nt], acc[mt][nt], 0, 0, 0);        \
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi[S_][mt], bhi[S_][nt], acc[mt][nt], 0, 0, 0);        \
      }                                                                                                              \
    if constexpr ((VAR & 1) != 0) __builtin_amdgcn_s_setprio(0);                                                     \
  }

  // one K-step: B(i) is in LDS buffer i&1, the register set RBN holds B(i+1), RBF is free (its B(i) is in LDS)
#define OFLOW_STEP(I, RAF, RAN, RBF, RBN, FH, FL)                                                                    \
  {                                                                                                                  \
    const int i_ = (I);                                                                                              \
    const int g = i_ / T, t = i_ - g * T;                                                                            \
    {                                                                                                                \
      const int i2 = i_ + 2 < S ? i_ + 2 : S - 1; /* past the end: a harmless re-load */                           \
      if constexpr (!BREG && !(VAR & 128)) { OFLOW_LOAD_B(RBF, i2); }                                                \
      if constexpr (ADB && !(VAR & 128)) { OFLOW_LOAD_A(RAF, i2); }                                                  \
    }                                                                                                                \
    if constexpr (!ADB) {                                                                                            \
      if (t == 0 && !(VAR & 128)) { OFLOW_LOAD_A(ra0, g + 1 < a.kg ? g + 1 : g); }                                   \
    }                                                                                                                \
    const int ky = t / KW, kx = t - ky * KW;                                                                         \
    const uint8_t* bufA = sA + (ADB ? (i_ & 1) * A_BYTES : 0);                                                       \
    const uint8_t* bufB = sB + (i_ & 1) * B_BYTES;                                                                   \
    half8 ahi[2][MT], alo[2][MT], bhi[2][NT], blo[2][NT];                                                          \
    _Pragma("unroll") for (int s = 0; s < 2; ++s) {                                                                  \
      const int chi = 2 * s + hh, clo = 4 + 2 * s + hh;                                                              \
      _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) {                                                            \
        const int p = (wm * MT + mt + ky) * HX + r + kx;                                                             \
        const uint8_t* row = bufA + p * RS;                                                                          \
        ahi[s][mt] = *reinterpret_cast<const half8*>(row + ((PADL ? chi : (chi ^ swz(p))) << 4));                    \
        alo[s][mt] = *reinterpret_cast<const half8*>(row + ((PADL ? clo : (clo ^ swz(p))) << 4));                    \
      }                                                                                                              \
      _Pragma("unroll") for (int nt = 0; nt < NT; ++nt) {                                                            \
        if constexpr (BREG) {                                                                                        \
          bhi[s][nt] = FH[s][nt];                                                                                    \
          blo[s][nt] = FL[s][nt];                                                                                    \
        } else {                                                                                                     \
          const int n = wn * (BN / WN) + nt * 32 + r;                                                                \
          const uint8_t* row = bufB + n * RS;                                                                        \
          bhi[s][nt] = *reinterpret_cast<const half8*>(row + ((PADL ? chi : (chi ^ swz(n))) << 4));                  \
          blo[s][nt] = *reinterpret_cast<const half8*>(row + ((PADL ? clo : (clo ^ swz(n))) << 4));                  \
        }                                                                                                            \
      }                                                                                                              \
      if constexpr (!(VAR & 2)) { OFLOW_MFMA_BLOCK(s); }                                                             \
    }                                                                                                                \
    if constexpr ((VAR & 2) != 0) { OFLOW_MFMA_BLOCK(0); OFLOW_MFMA_BLOCK(1); }                                      \
    if constexpr (BREG) { /* this step's fragment set is consumed: refill it two steps ahead */                    \
      OFLOW_LOAD_F(FH, FL, i_ + 2 < S ? i_ + 2 : S - 1);                                                             \
    }                                                                                                                \
    if constexpr (!ADB) {                                                                                            \
      if (t == T - 1 && g + 1 < a.kg) {                                                                              \
        __syncthreads(); /* every wave is done with A(g) */                                                          \
        OFLOW_WRITE_A(ra0, 0, g + 1);                                                                                \
        if constexpr (BREG) __syncthreads(); /* A(g+1) visible to every wave */                                     \
      }                                                                                                              \
    }                                                                                                                \
    if (i_ + 1 < S) {                                                                                                \
      if constexpr (!BREG) { OFLOW_WRITE_B(RBN, (i_ + 1) & 1); }                                                     \
      if constexpr (ADB) { OFLOW_WRITE_A(RAN, (i_ + 1) & 1, i_ + 1); }                                               \
    }                                                                                                                \
    if constexpr ((!BREG || ADB) && !(VAR & 512)) __syncthreads();                                                   \
  }

  if constexpr (BREG && !ADB && (VAR & 1024) != 0) {
    // Pipelined register-direct loop (VAR bit 10): the A operands of tap t+1 are read from LDS into the other
    // register set BEFORE tap t's MFMAs, so the MFMA chain covers the LDS latency; the halo changes (barrier) only at
    // group boundaries, where the next tap's reads are issued after the new halo is visible.
    // operand sets per K-half (sub-step): set 0 feeds sub-step 0 of every tap, set 1 sub-step 1
    half8 p0h[MT], p0l[MT], p1h[MT], p1l[MT];
#define OFLOW_READ_OPS(XH, XL, J, S_)                                                                                \
  {                                                                                                                  \
    const int tj_ = (J) % T, ky_ = tj_ / KW, kx_ = tj_ - ky_ * KW;                                                   \
    _Pragma("unroll") for (int mt_ = 0; mt_ < MT; ++mt_) {                                                           \
      const int p_ = (wm * MT + mt_ + ky_) * HX + r + kx_;                                                           \
      const uint8_t* row_ = sA + p_ * RS;                                                                            \
      const int ch_ = 2 * (S_) + hh, cl_ = 4 + 2 * (S_) + hh;                                                        \
      XH[mt_] = *reinterpret_cast<const half8*>(row_ + ((PADL ? ch_ : (ch_ ^ swz(p_))) << 4));                       \
      XL[mt_] = *reinterpret_cast<const half8*>(row_ + ((PADL ? cl_ : (cl_ ^ swz(p_))) << 4));                       \
    }                                                                                                                \
  }
#define OFLOW_MFMA_SUB(XH, XL, FH, FL, S_)                                                                           \
  _Pragma("unroll") for (int mt = 0; mt < MT; ++mt)                                                                  \
    _Pragma("unroll") for (int nt = 0; nt < NT; ++nt) {                                                              \
      acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(XH[mt], FL[S_][nt], acc[mt][nt], 0, 0, 0);                \
      acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(XL[mt], FH[S_][nt], acc[mt][nt], 0, 0, 0);                \
      acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(XH[mt], FH[S_][nt], acc[mt][nt], 0, 0, 0);                \
    }
#define OFLOW_PSTEP(I, FH, FL)                                                                                       \
  {                                                                                                                  \
    const int i_ = (I);                                                                                              \
    const int g = i_ / T, t = i_ - g * T;                                                                            \
    if (t == 0) { OFLOW_LOAD_A(ra0, g + 1 < a.kg ? g + 1 : g); }                                                     \
    OFLOW_READ_OPS(p1h, p1l, i_, 1); /* sub-step 1 operands in flight during sub-step 0 */                          \
    OFLOW_MFMA_SUB(p0h, p0l, FH, FL, 0);                                                                             \
    const bool same_ = t != T - 1 && i_ + 1 < S;                                                                     \
    if (same_) OFLOW_READ_OPS(p0h, p0l, i_ + 1, 0); /* next tap, same halo */                                       \
    OFLOW_MFMA_SUB(p1h, p1l, FH, FL, 1);                                                                             \
    OFLOW_LOAD_F(FH, FL, i_ + 2 < S ? i_ + 2 : S - 1);                                                               \
    if (t == T - 1 && i_ + 1 < S) {                                                                                  \
      __syncthreads(); /* every wave is done with A(g) */                                                            \
      OFLOW_WRITE_A(ra0, 0, g + 1);                                                                                  \
      __syncthreads(); /* A(g+1) visible */                                                                          \
      OFLOW_READ_OPS(p0h, p0l, i_ + 1, 0);                                                                           \
    }                                                                                                                \
  }
    OFLOW_READ_OPS(p0h, p0l, 0, 0);
    for (int i = 0; i < S; i += 2) {
      OFLOW_PSTEP(i, f0h, f0l);
      if (i + 1 < S) OFLOW_PSTEP(i + 1, f1h, f1l);
    }
#undef OFLOW_PSTEP
#undef OFLOW_MFMA_SUB
#undef OFLOW_READ_OPS
  } else {
    for (int i = 0; i < S; i += 2) {
      OFLOW_STEP(i, ra0, ra1, rb0, rb1, f0h, f0l);
      if (i + 1 < S) OFLOW_STEP(i + 1, ra1, ra0, rb1, rb0, f1h, f1l);
    }
  }
#undef OFLOW_STEP
#undef OFLOW_MFMA_BLOCK

#undef OFLOW_LOAD_A
#undef OFLOW_WRITE_A
#undef OFLOW_LOAD_B
#undef OFLOW_WRITE_B
#undef OFLOW_LOAD_F

  if constexpr ((VAR & 256) != 0) {  // ablation: no epilogue (accumulators kept live)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) asm volatile("" ::"v"(acc[mt][nt]));
    return;
  }
  // ---- epilogue: accumulators -> LDS tile [pixel][channel] ----
  if constexpr (BREG && !ADB) __syncthreads();  // every wave is done reading A before the tile overwrites it
  float* sT = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int nl = wn * (BN / WN) + nt * 32 + r;
      const int pbase = (wm * MT + mt) * kTX;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = (e & 3) + 8 * (e >> 2) + 4 * hh;
        sT[(pbase + m) * TS + nl] = acc[mt][nt][e];
      }
    }
  __syncthreads();

  if (a.f != nullptr) {
    // fp32 NCHW: lanes = consecutive pixels of one tile row (128-B rows of the destination)
    for (int item = tid; item < BM * BN; item += kThreads) {
      const int nl = item / BM, pl = item - nl * BM;
      const int n = n0 + nl;
      const int y = ty0 + pl / kTX, x = tx0 + (pl % kTX);
      if (n < a.N && y < a.H && x < a.W) {
        float v = sT[pl * TS + nl] * a.wsc[n];
        if (a.bias) v += a.bias[n];
        v = act_fn(v, a.act) * a.oscale;
        float* d = a.f + b * a.fbs + n * a.fcs + (long long)y * a.W + x;
        if (a.faccum)
          *d = *d + v;
        else
          *d = v;
      }
    }
  }
  if constexpr (EPI == 0) {
    if (a.stats != nullptr) {
      // per-tile instance-norm partials of the conv output (merged by oflow_norm_stats_finalize): SL = 256 / BN
      // adjacent lanes share a channel and take interleaved slices of the tile's pixels (two-pass mean / M2 in
      // fp32); the slices are merged across those lanes with xor shuffles (Chan et al.).
      constexpr int SL = kThreads / BN >= 4 ? 4 : kThreads / BN >= 2 ? 2 : 1;
      const int c = tid / SL, sl = tid % SL;
      const int n = n0 + c;
      const bool on = c < BN && n < a.N;
      const float ws = on ? a.wsc[n] : 0.f, bi = (on && a.bias) ? a.bias[n] : 0.f;
      int cnt = 0;
      float sum = 0.f;
      if (on) {
        for (int pl = sl; pl < BM; pl += SL) {
          const int y = ty0 + pl / kTX, x = tx0 + (pl % kTX);
          if (y < a.H && x < a.W) {
            sum += sT[pl * TS + c] * ws + bi;
            ++cnt;
          }
        }
      }
      float N0 = static_cast<float>(cnt), M0 = cnt ? sum / N0 : 0.f, Q0 = 0.f;
      if (on) {
        for (int pl = sl; pl < BM; pl += SL) {
          const int y = ty0 + pl / kTX, x = tx0 + (pl % kTX);
          if (y < a.H && x < a.W) {
            const float d = sT[pl * TS + c] * ws + bi - M0;
            Q0 += d * d;
          }
        }
      }
#pragma unroll
      for (int m = 1; m < SL; m <<= 1) {
        const float nb = __shfl_xor(N0, m), mb = __shfl_xor(M0, m), qb = __shfl_xor(Q0, m);
        const float nn = N0 + nb;
        if (nb > 0.f) {
          // symmetric form: both lanes of a pair compute the identical merged value
          const float lo_n = (sl & m) ? nb : N0, hi_n = (sl & m) ? N0 : nb;
          const float lo_m = (sl & m) ? mb : M0, hi_m = (sl & m) ? M0 : mb;
          const float lo_q = (sl & m) ? qb : Q0, hi_q = (sl & m) ? Q0 : qb;
          if (lo_n > 0.f) {
            const float d = hi_m - lo_m;
            M0 = lo_m + d * (hi_n / nn);
            Q0 = lo_q + hi_q + d * d * (lo_n * hi_n / nn);
          } else {
            M0 = hi_m;
            Q0 = hi_q;
          }
          N0 = nn;
        }
      }
      if (on && sl == 0) {
        const int tile_in_img = (ty0 / TY) * a.tiles_x + tx0 / kTX;
        float* st = a.stats + (((long long)b * a.tiles_x * a.tiles_y + tile_in_img) * a.npad + n) * 3;
        st[0] = N0;
        st[1] = M0;
        st[2] = Q0;
      }
    }
    if (a.y0 == nullptr && a.fn == nullptr) return;
  }

  // S32 / GRU consumers: one thread = one pixel x 8 consecutive channels
  constexpr int C8 = BN / 8;
  for (int item = tid; item < BM * C8; item += kThreads) {
    const int pl = item / C8, c8 = item - pl * C8;
    const int nl = c8 * 8, n = n0 + nl;
    const int y = ty0 + pl / kTX, x = tx0 + (pl % kTX);
    if (n >= a.N || y >= a.H || x >= a.W) continue;
    const long long P = pix0 + (long long)y * a.W + x;
    const float4 t0 = *reinterpret_cast<const float4*>(&sT[pl * TS + nl]);
    const float4 t1 = *reinterpret_cast<const float4*>(&sT[pl * TS + nl + 4]);
    float v[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int nj = n + j < a.N ? n + j : a.N - 1;
      v[j] = v[j] * a.wsc[nj] + (a.bias ? a.bias[nj] : 0.f);
    }
    if constexpr (EPI == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = act_fn(v[j], a.act) * a.oscale;
      if (a.res) {
        const uint8_t* rl = a.res + P * a.resps + (long long)(n >> 5) * 128 + ((n & 31) >> 3) * 16;
        const half8 rh = *reinterpret_cast<const half8*>(rl), rlo = *reinterpret_cast<const half8*>(rl + 64);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[j] = v[j] + (static_cast<float>(rh[j]) + static_cast<float>(rlo[j]));
          if (a.res_act) v[j] = act_fn(v[j], a.res_act);
        }
      }
      if (a.fn) {
        float* fp = a.fn + P * a.fnps + n;
        if (n + 8 <= a.N) {
          *reinterpret_cast<float4*>(fp) = make_float4(v[0], v[1], v[2], v[3]);
          *reinterpret_cast<float4*>(fp + 4) = make_float4(v[4], v[5], v[6], v[7]);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (n + j < a.N) fp[j] = v[j];
        }
      }
      if (a.y0) {
        long long Pd = P;
        int nd = n;
        if (a.s2d) {
          const int W2 = a.W >> 1, H2 = a.H >> 1;
          Pd = ((long long)b * H2 + (y >> 1)) * W2 + (x >> 1);
          nd = n + ((y & 1) * 2 + (x & 1)) * a.N;
        }
        store_s32(a.y0, a.y0ps, Pd, nd, a.s2d ? 4 * a.N : a.N, v);
        if (a.y1) store_s32(a.y1, a.y1ps, Pd, nd, a.s2d ? 4 * a.N : a.N, v);
      }
    } else if constexpr (EPI == 1) {
      // [z | r] gates (update.py:91-96): z = sigmoid -> a.z; r*h = sigmoid(r) * h -> S32 y0 (channel n - gch)
      if (n < a.gch) {
        float* zp = a.z + P * a.gch + n;
#pragma unroll
        for (int j = 0; j < 8; ++j) zp[j] = 1.0f / (1.0f + expf(-v[j]));
      } else {
        const float* hp = a.h + P * a.gch + (n - a.gch);
        float rh[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) rh[j] = (1.0f / (1.0f + expf(-v[j]))) * hp[j];
        store_s32(a.y0, a.y0ps, P, n - a.gch, a.gch, rh);
      }
    } else {
      // candidate + blend (update.py:96-97): h = (1 - z) * h + z * tanh(q); h (fp32) in place + S32 y0
      float* hp = a.h + P * a.gch + n;
      const float* zp = a.z + P * a.gch + n;
      float hn[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float q = tanhf(v[j]);
        const float z = zp[j];
        hn[j] = (1.0f - z) * hp[j] + z * q;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) hp[j] = hn[j];
      store_s32(a.y0, a.y0ps, P, n, a.N, hn);
    }
  }
}

template <int KH, int KW, int BN, int WM, int WN, int EPI, int VAR, int TY = kTY, bool BREG = false>
int launch_conv(const ConvArgs& a0, hipStream_t s) {
  ConvArgs a = a0;
  a.tiles_y = (a.H + TY - 1) / TY;
  dim3 grid(a.tiles_x * a.tiles_y * a.B, a.npad / BN);
  if constexpr (KH == 3 && KW == 3 && EPI == 0 && !BREG) {  // the encoders' second block convs
    if (a.ain == kInF32Norm) {
      hipLaunchKernelGGL((conv_s32_kernel<KH, KW, BN, WM, WN, EPI, VAR, TY, BREG, kInF32Norm>), grid, dim3(kThreads), 0, s,
                         a);
      return launch_status();
    }
  }
  if constexpr (KH == 1 && KW == 1 && EPI == 0 && BN == 128 && !BREG) {  // convc1 on the NHWC corr lookup
    if (a.ain == kInF32) {
      hipLaunchKernelGGL((conv_s32_kernel<KH, KW, BN, WM, WN, EPI, VAR, TY, BREG, kInF32>), grid, dim3(kThreads), 0, s, a);
      return launch_status();
    }
  }
  if (a.ain != kInS32) return OFLOW_E_MODE;
  hipLaunchKernelGGL((conv_s32_kernel<KH, KW, BN, WM, WN, EPI, VAR, TY, BREG>), grid, dim3(kThreads), 0, s, a);
  return launch_status();
}

// BN 128: the LDS-staged weight slab (2 x 2 waves) or, with VAR bit 4 (16), register-direct fragments (1 x 4 waves)
template <int KH, int KW, int EPI, int VAR>
int launch_128(const ConvArgs& a, hipStream_t s) {
  // VAR bit 6 (64): 256-channel workgroups (1 x 4 waves of 128 px x 64 ch, register-direct weights) where N allows
  if constexpr ((VAR & 64) != 0)
    if (a.npad % 256 == 0) return launch_conv<KH, KW, 256, 1, 4, EPI, VAR, kTY, true>(a, s);
  if constexpr ((VAR & 16) != 0) return launch_conv<KH, KW, 128, 1, 4, EPI, VAR, kTY, true>(a, s);
  return launch_conv<KH, KW, 128, 2, 2, EPI, VAR>(a, s);
}

template <int KH, int KW, int EPI, int VAR>
int launch_bn(const ConvArgs& a, int bn, hipStream_t s) {
  switch (bn) {
    case 128: return launch_128<KH, KW, EPI, VAR>(a, s);
    case 96: return launch_conv<KH, KW, 96, 4, 1, EPI, VAR>(a, s);
    case 64:
      // 8-row tiles (each wave 64 px x 64 ch: 8 operand reads per 12 MFMAs instead of 6 per 6): 4-5 % faster
      // (tools/exp/run_conv_exp.py), except with instance-norm partials, whose layout is 4-row tiles
      if ((VAR & 8) != 0 || a.stats == nullptr) return launch_conv<KH, KW, 64, 4, 1, EPI, VAR, 8>(a, s);
      return launch_conv<KH, KW, 64, 2, 2, EPI, VAR>(a, s);
    case 32: return launch_conv<KH, KW, 32, 4, 1, EPI, VAR>(a, s);
    default: return OFLOW_E_SHAPE;
  }
}

template <int VAR>
int dispatch_conv(const ConvArgs& a, int kh, int kw, int block_n, int epilogue, hipStream_t s) {
  const int key = kh * 16 + kw;
  switch (epilogue) {
    case 0:
      switch (key) {
        case 0x11: return launch_bn<1, 1, 0, VAR>(a, block_n, s);
        case 0x22: return launch_bn<2, 2, 0, VAR>(a, block_n, s);
        case 0x33: return launch_bn<3, 3, 0, VAR>(a, block_n, s);
        case 0x15: return launch_bn<1, 5, 0, VAR>(a, block_n, s);
        case 0x51: return launch_bn<5, 1, 0, VAR>(a, block_n, s);
        default: return OFLOW_E_SHAPE;
      }
    case 1:
      if (block_n != 128) return OFLOW_E_SHAPE;
      if (key == 0x15) return launch_128<1, 5, 1, VAR>(a, s);
      if (key == 0x51) return launch_128<5, 1, 1, VAR>(a, s);
      return OFLOW_E_SHAPE;
    default:
      if (block_n != 128) return OFLOW_E_SHAPE;
      if (key == 0x15) return launch_128<1, 5, 2, VAR>(a, s);
      if (key == 0x51) return launch_128<5, 1, 2, VAR>(a, s);
      return OFLOW_E_SHAPE;
  }
}

// argument checks + ConvArgs for oflow_conv_s32_ex (shared with the tools/exp variant harness)
int build_conv_args(ConvArgs& a, const void* d_x, long long x_pixel_stride, int in_groups, const void* d_wpack,
                    int n_pad, const float* d_wscale, const float* d_bias, int N, int B, int H, int W, int kh, int kw,
                    int block_n, int epilogue, int activation, float out_scale, void* d_y0, long long y0_pixel_stride,
                    void* d_y1, long long y1_pixel_stride, float* d_f32, long long f32_batch_stride,
                    long long f32_channel_stride, int f32_accumulate, float* d_gru_h, float* d_gru_z, int gru_channels,
                    float* d_nhwc, int nhwc_pixel_stride, float* d_stats, const void* d_res, long long res_pixel_stride,
                    int res_activation, int s2d) {
  if (!d_x || !d_wpack || !d_wscale) return OFLOW_E_NULL;
  if (B <= 0 || H <= 0 || W <= 0 || N <= 0 || in_groups <= 0 || n_pad < N || n_pad % block_n) return OFLOW_E_SHAPE;
  if (activation < 0 || activation > 3 || res_activation < 0 || res_activation > 3 || epilogue < 0 || epilogue > 2)
    return OFLOW_E_MODE;
  if ((x_pixel_stride & 15) || ((uintptr_t)d_x & 15) || ((uintptr_t)d_wpack & 15)) return OFLOW_E_ALIGN;
  if (epilogue == 0 && !d_y0 && !d_f32 && !d_nhwc && !d_stats) return OFLOW_E_NULL;
  if (epilogue != 0 && (!d_y0 || !d_gru_h || !d_gru_z || gru_channels <= 0 || gru_channels % 8)) return OFLOW_E_NULL;
  if (epilogue == 1 && N != 2 * gru_channels) return OFLOW_E_SHAPE;
  if (epilogue == 2 && N != gru_channels) return OFLOW_E_SHAPE;
  if (epilogue != 0 && (d_nhwc || d_stats || d_res || s2d)) return OFLOW_E_MODE;
  if (s2d && ((H | W) & 1 || N % 8)) return OFLOW_E_SHAPE;
  if (d_nhwc && (nhwc_pixel_stride < N || ((uintptr_t)d_nhwc & 15) || (nhwc_pixel_stride & 3))) return OFLOW_E_ALIGN;
  if ((d_y0 && ((y0_pixel_stride & 127) || ((uintptr_t)d_y0 & 15))) ||
      (d_y1 && ((y1_pixel_stride & 127) || ((uintptr_t)d_y1 & 15))) ||
      (d_res && ((res_pixel_stride & 127) || ((uintptr_t)d_res & 15))))
    return OFLOW_E_ALIGN;
  a = ConvArgs{};
  a.x = static_cast<const uint8_t*>(d_x);
  a.xps = x_pixel_stride;
  a.kg = in_groups;
  a.w = static_cast<const uint8_t*>(d_wpack);
  a.npad = n_pad;
  a.wsc = d_wscale;
  a.bias = d_bias;
  a.N = N;
  a.B = B;
  a.H = H;
  a.W = W;
  a.tiles_x = (W + kTX - 1) / kTX;
  a.tiles_y = (H + kTY - 1) / kTY;
  a.act = activation;
  a.oscale = out_scale;
  a.y0 = static_cast<uint8_t*>(d_y0);
  a.y0ps = y0_pixel_stride;
  a.y1 = static_cast<uint8_t*>(d_y1);
  a.y1ps = y1_pixel_stride;
  a.f = d_f32;
  a.fbs = f32_batch_stride;
  a.fcs = f32_channel_stride;
  a.faccum = f32_accumulate;
  a.h = d_gru_h;
  a.z = d_gru_z;
  a.gch = gru_channels;
  a.fn = d_nhwc;
  a.fnps = nhwc_pixel_stride;
  a.stats = d_stats;
  a.res = static_cast<const uint8_t*>(d_res);
  a.resps = res_pixel_stride;
  a.res_act = res_activation;
  a.s2d = s2d;
  a.cin = in_groups * 32;
  (void)kh;
  (void)kw;
  (void)block_n;
  return OFLOW_OK;
}

}  // namespace
}  // namespace oflow

using namespace oflow;

extern "C" int oflow_conv_s32_ex2(const void* d_x, long long x_pixel_stride, int in_groups, const void* d_wpack,
                                  int n_pad, const float* d_wscale, const float* d_bias, int N, int B, int H, int W, int kh,
                                  int kw, int block_n, int epilogue, int activation, float out_scale, void* d_y0,
                                  long long y0_pixel_stride, void* d_y1, long long y1_pixel_stride, float* d_f32,
                                  long long f32_batch_stride, long long f32_channel_stride, int f32_accumulate,
                                  float* d_gru_h, float* d_gru_z, int gru_channels, float* d_nhwc, int nhwc_pixel_stride,
                                  float* d_stats, const void* d_res, long long res_pixel_stride, int res_activation,
                                  int s2d, int in_format, const float* d_in_scale, const float* d_in_shift,
                                  void* stream) {
  ConvArgs a;
  const int st = build_conv_args(a, d_x, x_pixel_stride, in_groups, d_wpack, n_pad, d_wscale, d_bias, N, B, H, W, kh, kw,
                                 block_n, epilogue, activation, out_scale, d_y0, y0_pixel_stride, d_y1, y1_pixel_stride,
                                 d_f32, f32_batch_stride, f32_channel_stride, f32_accumulate, d_gru_h, d_gru_z,
                                 gru_channels, d_nhwc, nhwc_pixel_stride, d_stats, d_res, res_pixel_stride,
                                 res_activation, s2d);
  if (st != OFLOW_OK) return st;
  if (in_format < kInS32 || in_format > kInF32) return OFLOW_E_MODE;
  if (in_format != kInF32 && (x_pixel_stride & 127)) return OFLOW_E_ALIGN;  // S32 / dense fp32: whole 128-B groups
  if (in_format == kInF32Norm && x_pixel_stride != (long long)in_groups * 128) return OFLOW_E_SHAPE;  // dense [P][kg*32]
  if (in_format == kInF32) {  // rows of cin fp32 channels, (kg - 1) * 32 < cin <= kg * 32, cin % 4 == 0
    const long long cin = x_pixel_stride / 4;
    if ((x_pixel_stride & 15) || cin > (long long)in_groups * 32 || cin <= (long long)(in_groups - 1) * 32) return OFLOW_E_SHAPE;
    a.cin = static_cast<int>(cin);
  }
  if (in_format == kInF32Norm) {  // normalised + ReLU'd on load
    if (!d_in_scale || !d_in_shift) return OFLOW_E_NULL;
    if (kh != 3 || kw != 3 || epilogue != 0 || in_groups > kAinGroups) return OFLOW_E_MODE;
    a.ia = d_in_scale;
    a.ib = d_in_shift;
  } else if (in_format == kInF32) {
    if (kh != 1 || kw != 1 || epilogue != 0 || block_n != 128) return OFLOW_E_MODE;
  }
  a.ain = in_format;
  return dispatch_conv<0>(a, kh, kw, block_n, epilogue, static_cast<hipStream_t>(stream));
}

extern "C" int oflow_conv_s32_ex(const void* d_x, long long x_pixel_stride, int in_groups, const void* d_wpack,
                                 int n_pad, const float* d_wscale, const float* d_bias, int N, int B, int H, int W, int kh,
                                 int kw, int block_n, int epilogue, int activation, float out_scale, void* d_y0,
                                 long long y0_pixel_stride, void* d_y1, long long y1_pixel_stride, float* d_f32,
                                 long long f32_batch_stride, long long f32_channel_stride, int f32_accumulate,
                                 float* d_gru_h, float* d_gru_z, int gru_channels, float* d_nhwc, int nhwc_pixel_stride,
                                 float* d_stats, const void* d_res, long long res_pixel_stride, int res_activation,
                                 int s2d, void* stream) {
  return oflow_conv_s32_ex2(d_x, x_pixel_stride, in_groups, d_wpack, n_pad, d_wscale, d_bias, N, B, H, W, kh, kw,
                            block_n, epilogue, activation, out_scale, d_y0, y0_pixel_stride, d_y1, y1_pixel_stride,
                            d_f32, f32_batch_stride, f32_channel_stride, f32_accumulate, d_gru_h, d_gru_z, gru_channels,
                            d_nhwc, nhwc_pixel_stride, d_stats, d_res, res_pixel_stride, res_activation, s2d, kInS32,
                            nullptr, nullptr, stream);
}

extern "C" int oflow_conv_s32(const void* d_x, long long x_pixel_stride, int in_groups, const void* d_wpack, int n_pad,
                              const float* d_wscale, const float* d_bias, int N, int B, int H, int W, int kh, int kw,
                              int block_n, int epilogue, int activation, float out_scale, void* d_y0,
                              long long y0_pixel_stride, void* d_y1, long long y1_pixel_stride, float* d_f32,
                              long long f32_batch_stride, long long f32_channel_stride, int f32_accumulate,
                              float* d_gru_h, float* d_gru_z, int gru_channels, void* stream) {
  return oflow_conv_s32_ex(d_x, x_pixel_stride, in_groups, d_wpack, n_pad, d_wscale, d_bias, N, B, H, W, kh, kw,
                           block_n, epilogue, activation, out_scale, d_y0, y0_pixel_stride, d_y1, y1_pixel_stride,
                           d_f32, f32_batch_stride, f32_channel_stride, f32_accumulate, d_gru_h, d_gru_z, gru_channels,
                           nullptr, 0, nullptr, nullptr, 0, 0, 0, stream);
}
