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
// buffered). Both are register-staged (B one step, the halo one group ahead). LDS lines are 16-B-slot swizzled
// (slot ^= (row >> 1) & 7) so that the 32 rows of an MFMA operand read by ds_read_b128 are bank-conflict free.
// Epilogue: accumulators -> LDS tile [pixel][channel] fp32 -> per-channel scale, bias, activation and the fused
// consumer (S32 stores with 16-B chunks, GRU gates, fp32 NCHW store/accumulate).
#include "oflow_internal.h"

namespace oflow {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));  // native vector: stays in VGPRs (HIP uint4 is copied by memcpy)

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }
// operand rows in LDS: 144-B padded rows (1) or 128-B rows with XOR-swizzled 16-B slots (0; build with
// VECFLAGS+=-DOFLOW_PAD_ROWS=0 for A/B). Both are conflict-free for the ds_read_b128 operand reads; the padded rows
// make every read address one per-lane base plus an immediate (no per-read swizzle arithmetic).
// register-direct weights: steps of B fragments in flight (2 or 3: measured neutral, profiles/r04/s18_*; default 2)
#ifndef OFLOW_BREG_RING
#define OFLOW_BREG_RING 2
#endif
// register-direct weights, vertical taps: halo-row operands reused across taps (1; 0 = re-read per tap, for A/B)
#ifndef OFLOW_VSLIDE
#define OFLOW_VSLIDE 1
#endif
// XCD-aware workgroup order (1) or the 2D grid (tile, channel block) (0, default): measured no faster -- per layer
// alone 977.9 (2D) vs 986.8 us per update iteration, benches 422.0 / 423.4 vs 421.2 / 420.7 pairs/s alternated on one
// box (profiles/r04/s21_*): the halo re-reads of a tile's second channel block already hit the Infinity Cache
#ifndef OFLOW_XCD_MAP
#define OFLOW_XCD_MAP 0
#endif
#ifndef OFLOW_STEM_SINGLE_A
#define OFLOW_STEM_SINGLE_A 1
#endif
#ifndef OFLOW_PAD_ROWS
#define OFLOW_PAD_ROWS 1
#endif
// register-direct weights: the halo double-buffered in LDS (1): group g+1's halo is written into the buffer group g-1
// used while group g's MFMAs run, one barrier per group instead of two around a single buffer's swap. Bit-identical,
// but the step is 0.1-0.3 ms slower (the doubled halo, up to 74 KB per workgroup, crowds the other lane's workgroups
// off the CUs: profiles/r05/s25_step_ab.log), so the single buffer (0) stays the default.
#ifndef OFLOW_HALO_DB
#define OFLOW_HALO_DB 0
#endif

constexpr int kTY = 4, kTX = 32;  // default tile: kTY rows x kTX columns

// ablation build (tools/exp: -DOFLOW_ABLATE): exp_flags bits drop parts of the kernel to time the rest (2 MFMAs, 4 A
// staging writes, 8 instance-norm partials, 16 epilogue stores, 32 B staging writes, 64 the main loop's per-step
// barrier); the product build compiles every test to false
#ifdef OFLOW_ABLATE
#define OFLOW_ABL(bit) ((a.exp_flags & (bit)) != 0)
#else
#define OFLOW_ABL(bit) false
#endif
constexpr int kAinGroups = 4;                      // AIN inputs: up to 128 channels (the encoders' 64 / 96 / 128)


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
  // fp32 NHWC addend [P][addps] added to the pre-activation value (after scale and bias), or null: the GRU's
  // loop-invariant context term, computed once per forward (EPI 1, 2)
  const float* add;
  long long addps;
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
  int wbytes;              // bytes of the packed weights (kg * taps * npad * 128)
  const uint8_t* wf;       // the same weights fragment-major (register-direct B, BREG kernels), or null
  int exp_flags;           // experiments only (oflow_exp_set_conv_flags): bit 0 = the stem's element-wise window loop
  // split-K (BREG kernels only, oflow_conv_s32_ex5): gridDim.z = 2 workgroups per tile, each summing half of the input
  // groups (kg above is the half); per tile a BM x BN fp32 partial slab and two counters [ticket, published]
  float* ks_slab;
  unsigned* ks_ctr;
  long long ks_tiles;      // tiles (x channel blocks) the slab and counters hold
};
// input formats of oflow_conv_s32_ex2
constexpr int kInS32 = OFLOW_IN_S32, kInF32Norm = OFLOW_IN_F32_NORM, kInF32 = OFLOW_IN_F32, kInImg = OFLOW_IN_IMG7S2,
              kInFlow = OFLOW_IN_FLOW7;
// kInImg: the stem's 7x7/2 pad-3 window of a 3-channel image, staged per tile (TY = 4 rows x 32 columns)
constexpr int kImgC = 3, kImgK = 7, kImgRows = (kTY - 1) * 2 + kImgK, kImgCols = (kTX - 1) * 2 + kImgK;
// the window in LDS: [c][row][column parity][column / 2] (row pitch kImgPitch floats): output column x reads window
// column 2x + kx at (kx & 1) * kImgHalf + x + (kx >> 1), so the 32 lanes of one output row read 32 consecutive floats
// (conflict-free ds_read_b32; the column-interleaved [c][row][col] image gave each 32-lane group 2- to 4-way conflicts:
// 50 % of the stem's LDS cycles, profiles/r04/s1_pmc_mfma.json)
constexpr int kImgHalf = (kImgCols + 1) / 2, kImgPitch = 2 * kImgHalf, kImgPlane = kImgRows * kImgPitch;

// the GRU gates' sigmoid / tanh (update.py:91-97) from the hardware exp2 and reciprocal (v_exp_f32, v_rcp_f32: 1 ulp each; a few
// instructions instead of libm's expf + IEEE division / tanhf, ~25-30 VALU per value in an epilogue of 64 values per
// lane). Absolute error <= ~2e-7 for both (tanh near 0 through 1 - 2 / (e^2v + 1)); NaN propagates, +-inf saturate.
__device__ __forceinline__ float sigmoid_hw(float v) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(v * -1.4426950408889634f));
}
__device__ __forceinline__ float tanh_hw(float v) {
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(v * 2.8853900817779268f) + 1.0f);
}

__device__ __forceinline__ float act_fn(float v, int act) {
  if (act == 1) return v < 0.f ? 0.f : v;  // relu; NaN propagates like ATen
  if (act == 2) return 1.0f / (1.0f + expf(-v));
  if (act == 3) return tanhf(v);
  return v;
}

__device__ __forceinline__ void split8(const float* v, half8& hi, half8& lo) { split_vec(v, hi, lo); }

// store channels [n, n + 8) of pixel P (n % 8 == 0) into an S32 destination, only those < N; the max |x| of the stored
// values goes into gm (the caller range-guards once per epilogue: one branch instead of one per item)
__device__ __forceinline__ void store_s32(uint8_t* y, long long ps, long long P, int n, int N, const float* v, float& gm) {
  uint8_t* line = y + P * ps + (long long)(n >> 5) * 128 + ((n & 31) >> 3) * 16;
  if (n + 8 <= N) {
    half8 hi, lo;
    split8(v, hi, lo);
    gm = fmaxf(gm, fmaxf(fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))),
                         fmaxf(fmaxf(fabsf(v[4]), fabsf(v[5])), fmaxf(fabsf(v[6]), fabsf(v[7])))));
    *reinterpret_cast<half8*>(line) = hi;
    *reinterpret_cast<half8*>(line + 64) = lo;
  } else {
    _Float16* hp = reinterpret_cast<_Float16*>(line);
    _Float16* lp = reinterpret_cast<_Float16*>(line + 64);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (n + j < N) {
        gm = fmaxf(gm, fabsf(v[j]));
        _Float16 h_, l_;
        split_f16(v[j], h_, l_);
        hp[j] = h_;
        lp[j] = l_;
      }
    }
  }
}

// AIN: kInF32Norm = fp32 NHWC [P][kg*32] input normalised + ReLU'd while staged (ConvArgs.ia / .ib, kg <= kAinGroups);
// kInF32 = fp32 NHWC input split into hi + lo while staged (the NHWC corr lookup feeding convc1).
//
// Main loop (one K-step = one (input group, tap) pair = 32 input channels = two 16-deep MFMA sub-steps):
//   1. write B(i+1) [1x1: and A(i+1)] from registers into its LDS buffer (loaded one step earlier)
//   2. issue the global loads of B(i+2) [A(i+2)] (and, at a group's first tap, of the next group's halo)
//   3. read sub-step 1's operands of step i from LDS                     -> in flight during 4
//   4. 3 x MT x NT MFMAs of sub-step 0 (operands read during step i-1)
//   5. barrier (at a group's last tap: first a barrier, then the next halo is written)
//   6. read sub-step 0's operands of step i+1                            -> in flight during 7
//   7. MFMAs of sub-step 1
// so every LDS read has a block of MFMAs to hide behind, and the one barrier per step sits between two MFMA blocks.
//
// BREG (register-direct weights, T > 1, 4 waves as 1 x 4: each wave all 128 pixels x one 32-channel tile): B comes from
// the fragment-major copy of the weights (ConvArgs.wf: per step and channel tile [sub-step 2][hi, lo][lane 64][16 B],
// one wave instruction = 1 KB contiguous = the MFMA's B fragment) straight into a 2-deep ring of operand registers --
// no B staging through LDS, and the only barriers are the two around each input group's halo swap (T steps per group
// instead of one barrier per step). No two waves load the same fragment. Same MFMAs in the same order per accumulator
// as the LDS-staged kernel: bit-identical outputs.
// BD (LDS-staged B, r06): steps of operand prefetch in registers -- B(i + BD) is loaded at step i into one of BD
// register sets (1x1 convs: A too). With BD = 1 the load issued just before a step's barrier was written to LDS a
// few MFMAs into the next step (an L2 round trip of ~0.3-0.5 us waited out in most steps: s_waitcnt vmcnt(0) in the
// main loop's ISA); BD = 2 (launch_staged, the default) gives it a whole step more.
template <int KH, int KW, int BN, int WM, int WN, int EPI, int TY = kTY, int AIN = kInS32, bool BREG = false, int BD = 1>
// (the second bound is HIP's minimum waves per SIMD: 2 -> <= 256 VGPRs)
__global__ __launch_bounds__(64 * WM * WN, WM * WN == 8 ? 1 : 2) void conv_s32_kernel(ConvArgs a) {
  constexpr int NTH = 64 * WM * WN;  // 4 waves (two workgroups per CU) or 8 (one)
  constexpr int T = KH * KW;
  constexpr int BM = TY * kTX;  // output pixels per workgroup (TY rows x 32 columns)
  constexpr int PH = KH / 2, PW = KW / 2;
  constexpr int HY = TY + KH - 1, HX = kTX + KW - 1, NPIX = HY * HX;
  constexpr int AITEMS = NPIX * 8, APER = (AITEMS + NTH - 1) / NTH;
  constexpr int BITEMS = BN * 8, BPER = (BITEMS + NTH - 1) / NTH;
  constexpr int MT = TY / WM;            // 32-pixel row tiles per wave
  constexpr int NT = BN / WN / 32;        // 32-channel column tiles per wave
  static_assert((WM * WN == 4 || WM * WN == 8) && MT >= 1 && NT >= 1, "bad wave grid");
  static_assert(NTH % 8 == 0, "an A item's 16-B chunk is tid & 7");
  // T == 1 (1x1 convs): the input tile changes every K-step, so A is staged like B (double buffered in LDS).
  // The stem (kInImg) builds A from the image window already in LDS, so nothing is gained by building A(i+1) beside
  // A(i): one A buffer and the halo-swap schedule (a barrier before each rebuild) -- 50.5 instead of 68.9 KB of LDS,
  // three workgroups per CU instead of two (OFLOW_STEM_SINGLE_A=0: the double buffer, for A/B).
  // input windows (the stem's image, convf1's flow): the patch operand is built per tile from a window staged in LDS
  constexpr bool WIN = AIN == kInImg || AIN == kInFlow;
  constexpr int WC = AIN == kInFlow ? 2 : kImgC, WS = AIN == kInFlow ? 1 : 2;  // window channels, stride
  constexpr int WROWS = (kTY - 1) * WS + kImgK, WCOLS = (kTX - 1) * WS + kImgK;
  // stride 2: [c][row][column parity][column / 2] (kImgHalf); stride 1: [c][row][column]
  constexpr int WHALF = WS == 2 ? (WCOLS + 1) / 2 : WCOLS, WPITCH = WS == 2 ? 2 * WHALF : WCOLS;
  constexpr int WPLANE = WROWS * WPITCH;
  constexpr int WKPAD = AIN == kInFlow ? 128 : 160;  // patch channels staged (>= 49 * WC: zeros past it)
  constexpr int WAPER = WIN ? BM * 4 / NTH : 1;      // window input: (pixel, 8 patch channels) items per thread
  static_assert(!WIN || (BM * 4) % NTH == 0, "window items");
  static_assert(AIN != kInImg || (WHALF == kImgHalf && WPITCH == kImgPitch && WPLANE == kImgPlane), "stem window");
  constexpr bool ADB = (T == 1) && !(WIN && OFLOW_STEM_SINGLE_A);
  // 128-B LDS rows, 16-B slots XOR-swizzled (slot ^= (row >> 1) & 7): the 32 rows of an MFMA operand read by
  // ds_read_b128 are bank-conflict free from any starting row (padded 144-B rows with affine addressing measured the
  // same speed, tools/exp/conv_s32_dma.hip's history)
  constexpr int RS = 128;
  // BREG: the halo rows padded to 144 B instead of swizzled (consecutive rows start 36 banks apart: the 16 rows of a
  // ds_read_b128 phase are conflict-free), so every A read is one per-lane base plus an immediate offset (the swizzle
  // costs ~4 VALU per read, 16 reads per step with 4 row tiles per wave)
  constexpr int RSA = (BREG || OFLOW_PAD_ROWS) ? 144 : RS, RSB = OFLOW_PAD_ROWS ? 144 : RS;
  constexpr int A_BYTES = NPIX * RSA, B_BYTES = BN * RSB;
  static_assert(!BREG || (T > 1 && (WM == 1 || WM == 2 || WM == 4) && BN == 32 * WN && AIN == kInS32),
                "register-direct B: T > 1, WM x WN waves of one 32-channel tile each");
  constexpr bool HDB = BREG && OFLOW_HALO_DB;  // double-buffered halo (register-direct kernels)
  constexpr int MAIN_BYTES = ((ADB || HDB) ? 2 : 1) * A_BYTES + (BREG ? 0 : 2 * B_BYTES);
  constexpr int TS = BN + 4;              // epilogue tile row stride (floats)
  constexpr int EPI_BYTES = BM * TS * 4;
  constexpr int LDS_BYTES = MAIN_BYTES > EPI_BYTES ? MAIN_BYTES : EPI_BYTES;
  // windows: the input window + one zero float, then the patch channels' window offsets
  constexpr int kImgZero = WC * WPLANE;
  constexpr int IMG_FLOATS = (kImgZero + 1 + 3) & ~3;
  constexpr int AFF_BYTES = AIN == kInF32Norm ? kAinGroups * 32 * 8  // float2 (scale, shift) per input channel
                            : WIN ? IMG_FLOATS * 4 + WKPAD * 4
                            : 0;
  static_assert(!WIN || (T == 1 && TY == kTY), "window input: 1x1 geometry over the patch channels, 4-row tiles");
  __shared__ __attribute__((aligned(16))) uint8_t smem[LDS_BYTES + AFF_BYTES];
  // the block's per-channel (inverse weight scale, bias), staged once for the epilogue (whose loops would otherwise
  // wait on a global-load round trip per iteration)
  __shared__ float2 sSB[BN];
  // instance-norm partials per (row of waves, channel): (count, mean, M2)
  __shared__ float3 sStat[EPI == 0 ? WM * BN : 1];
  float2* sAff = reinterpret_cast<float2*>(smem + LDS_BYTES);
  float* sImg = reinterpret_cast<float*>(smem + LDS_BYTES);  // kInImg: [c][row][parity][col/2], zero at kImgZero
  int* sKoff = reinterpret_cast<int*>(smem + LDS_BYTES + (WIN ? IMG_FLOATS * 4 : 0));
  uint8_t* sA = smem;
  uint8_t* sB = smem + (ADB ? 2 : 1) * A_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int r = lane & 31, hh = lane >> 5;
  if constexpr (BREG) {
    if (a.ks_slab != nullptr) {  // split-K: this workgroup's half of the input groups (a.kg is the half count)
      const int z = blockIdx.z;
      a.x += (long long)z * a.kg * 128;                 // S32 channel slice: + 128 B per group
      a.wf += (long long)z * a.kg * T * a.npad * 128;   // fragment-major weights are step-major, step = (group, tap)
    }
  }
  auto aswz = [](int p) { return (BREG || OFLOW_PAD_ROWS) ? 0 : swz(p); };  // row slot swizzles (none with padded rows)
  auto bswz = [](int n) { return OFLOW_PAD_ROWS ? 0 : swz(n); };

  // workgroup -> (tile, channel block). XCD-aware (OFLOW_XCD_MAP): workgroups are dealt round-robin over the 8 XCDs
  // (each with its own L2), so ids 8 apart share one; the channel blocks of a tile take ids 8 apart within a group of
  // 8 * nblk ids and run on one XCD close together in time -- the second reads the tile's halo from that L2 instead of
  // from the fabric (a 2D grid runs every tile's block 0 before any block 1)
  int tile, cblk;
  if constexpr (OFLOW_XCD_MAP) {
    const int nblk = a.npad / BN, ntiles = a.tiles_x * a.tiles_y * a.B, bid = blockIdx.x;
    const int full = (ntiles >> 3) * 8 * nblk;
    if (bid < full) {
      const int grp = bid / (8 * nblk), rem = bid - grp * 8 * nblk;
      cblk = rem >> 3;
      tile = grp * 8 + (rem & 7);
    } else {
      const int ntail = ntiles & 7, rem = bid - full;
      cblk = rem / ntail;
      tile = (ntiles & ~7) + (rem - cblk * ntail);
    }
  } else {
    tile = blockIdx.x;
    cblk = blockIdx.y;
  }
  const int tx0 = (tile % a.tiles_x) * kTX;
  tile /= a.tiles_x;
  const int ty0 = (tile % a.tiles_y) * TY;
  const int b = tile / a.tiles_y;
  const int n0 = cblk * BN;
  const long long pix0 = (long long)b * a.H * a.W;

  // Register staging: one register set per operand; B(i+1) is written to LDS at step i's start and the set reloaded
  // with B(i+2) right after. A (one group's halo) is loaded at the group's first tap and written at its last; for 1x1
  // convs A follows B's scheme.
  u32x4 ra[APER], rb[BPER];
  // Global loads are raw buffer loads: a per-lane 32-bit offset (fixed for the whole loop) plus the step's uniform
  // byte offset in an SGPR, so the loop spends no vector instructions on addresses. Every load is unconditional (no
  // exec branches), so the compiler counts vmcnt precisely: halo pixels outside the image load a clamped in-image
  // pixel that is zeroed when staged (not the buffer's out-of-range zero fill: that gave nondeterministic halos).
  // B loads precede A loads in every step, so waiting for B never waits for the (HBM-latency) halo prefetch.
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(a.x + pix0 * a.xps), (short)0, (int)((long long)a.H * a.W * a.xps), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.w), (short)0, a.wbytes, 0x00020000);
  // the halo item offsets are recomputed at each load from an opaque copy of tid (a few VALU per group) rather than
  // kept in APER live registers (the 3x3 BN64 8-row variant spilled them to scratch inside the main loop)
  auto a_off = [&](int s_, int& col) {
    int t_ = tid;
    asm volatile("" : "+v"(t_));
    const int item = (AITEMS % NTH == 0) ? t_ + s_ * NTH : min(t_ + s_ * NTH, AITEMS - 1);
    const int p = item >> 3, c = item & 7;
    const int gy = ty0 - PH + p / HX, gx = tx0 - PW + p % HX;
    const int cy = min(max(gy, 0), a.H - 1), cx = min(max(gx, 0), a.W - 1);
    col = c * 16;
    return (cy * a.W + cx) * (int)a.xps + (AIN == kInF32 ? 0 : c * 16);
  };
  unsigned aok = 0u;
#pragma unroll
  for (int s_ = 0; s_ < APER; ++s_) {
    const int item = (AITEMS % NTH == 0) ? tid + s_ * NTH : min(tid + s_ * NTH, AITEMS - 1);
    const int p = item >> 3;
    const int gy = ty0 - PH + p / HX, gx = tx0 - PW + p % HX;
    const bool ok = static_cast<unsigned>(gy) < static_cast<unsigned>(a.H) && static_cast<unsigned>(gx) < static_cast<unsigned>(a.W);
    aok |= (ok ? 1u : 0u) << s_;
  }
  int boff[BPER];
#pragma unroll
  for (int s_ = 0; s_ < BPER; ++s_) boff[s_] = (n0 + (tid + s_ * NTH) / 8) * 128 + ((tid + s_ * NTH) & 7) * 16;
#define OFLOW_LOAD_A(RA, G)                                                                                          \
  if constexpr (!WIN) _Pragma("unroll") for (int s_ = 0; s_ < APER; ++s_) {                                        \
    int col_;                                                                                                        \
    const int off_ = a_off(s_, col_);                                                                                \
    if constexpr (AIN == kInF32) /* rows of cin floats: channels past cin re-read the row's last 16 B (zeroed) */   \
      RA[s_] = __builtin_amdgcn_raw_buffer_load_b128(rsA, off_ + min((G) * 128 + col_, a.cin * 4 - 16), 0, 0);      \
    else                                                                                                             \
      RA[s_] = __builtin_amdgcn_raw_buffer_load_b128(rsA, off_, (G) * 128, 0);                                      \
  }
// (one range-guard branch per call: the max |x| of all the thread's split values; the normalising affine of the
// thread's 4 channels read once: an item's chunk is tid & 7 for every item, NTH being a multiple of 8)
#define OFLOW_WRITE_A(RA, BUF, G)                                                                                    \
  if (!OFLOW_ABL(4)) {                                                                                               \
  float amx_ = 0.f;                                                                                                  \
  float2 af4_[4];                                                                                                    \
  if constexpr (AIN == kInF32Norm) _Pragma("unroll") for (int e_ = 0; e_ < 4; ++e_)                                  \
    af4_[e_] = sAff[(G) * 32 + 4 * (tid & 7) + e_];                                                                  \
  if constexpr (WIN) {                                                                                               \
    /* window input: item = (pixel p, 8 patch channels G*32 + 8cp ..), consecutive lanes on consecutive pixels       \
       (conflict-free window reads); hi and lo each one 16-B slot of the pixel's row: with 144-B rows the 8 lanes of \
       a ds_write_b128 phase cover the 32 banks once (4-channel items wrote 8-B halves: 2-way conflicts, twice the   \
       writes) */                                                                                                    \
    _Pragma("unroll") for (int s_ = 0; s_ < WAPER; ++s_) {                                                           \
      const int item = tid + s_ * NTH;                                                                               \
      const int p = item % BM, cp = item / BM;                                                                       \
      const int pb_ = WS * (p >> 5) * WPITCH + (p & 31);                                                             \
      const int4 k0_ = *reinterpret_cast<const int4*>(sKoff + (G) * 32 + 8 * cp);                                    \
      const int4 k1_ = *reinterpret_cast<const int4*>(sKoff + (G) * 32 + 8 * cp + 4);                                \
      const int kov_[8] = {k0_.x, k0_.y, k0_.z, k0_.w, k1_.x, k1_.y, k1_.z, k1_.w};                                  \
      float v8_[8];                                                                                                  \
      _Pragma("unroll") for (int e_ = 0; e_ < 8; ++e_) {                                                             \
        v8_[e_] = sImg[kov_[e_] < 0 ? kImgZero : pb_ + kov_[e_]];                                                    \
        amx_ = fmaxf(amx_, fabsf(v8_[e_]));                                                                          \
      }                                                                                                              \
      half8 h8_, l8_;                                                                                                \
      split_vec(v8_, h8_, l8_);                                                                                      \
      uint8_t* rw_ = sA + (BUF) * A_BYTES + p * RSA;                                                                 \
      *reinterpret_cast<half8*>(rw_ + ((cp ^ aswz(p)) << 4)) = h8_;                                                  \
      *reinterpret_cast<half8*>(rw_ + (((4 + cp) ^ aswz(p)) << 4)) = l8_;                                            \
    }                                                                                                                \
  } else                                                                                                             \
  _Pragma("unroll") for (int s_ = 0; s_ < APER; ++s_) {                                                              \
    const int item = tid + s_ * NTH;                                                                            \
    /* the 8 chunks of a pixel (whole 128-B LDS rows per 8 lanes) */                                                 \
    const int p = item >> 3, c = item & 7;                                                                           \
    if (AITEMS % NTH == 0 || item < AITEMS) {                                                                   \
      if constexpr (AIN != kInS32) {                                                                                 \
        /* 4 fp32 channels (G*32 + 4c ..) [-> relu(x * scale + shift)] -> 4 hi + 4 lo halves (8 B each) */           \
        typedef _Float16 half4_ __attribute__((ext_vector_type(4)));                                                 \
        half4_ h4 = {0, 0, 0, 0}, l4 = {0, 0, 0, 0};                                                                 \
        if (((aok >> s_) & 1u) && (AIN != kInF32 || (G) * 32 + 4 * c < a.cin)) {                                     \
          const float* fv = reinterpret_cast<const float*>(&RA[s_]);                                                 \
          float mx_ = 0.f, v4_[4];                                                                                   \
          _Pragma("unroll") for (int e_ = 0; e_ < 4; ++e_) {                                                         \
            float v_ = fv[e_];                                                                                       \
            if constexpr (AIN == kInF32Norm) {                                                                       \
              const float2 af = af4_[e_];                                                                            \
              v_ = v_ * af.x + af.y;                                                                                 \
              v_ = v_ < 0.f ? 0.f : v_;                                                                              \
            }                                                                                                        \
            mx_ = fmaxf(mx_, fabsf(v_));                                                                             \
            v4_[e_] = v_;                                                                                            \
          }                                                                                                          \
          split_vec(v4_, h4, l4);                                                                                    \
          amx_ = fmaxf(amx_, mx_);                                                                                   \
        }                                                                                                            \
        uint8_t* rw_ = sA + (BUF) * A_BYTES + p * RSA + (c & 1) * 8;                                                 \
        *reinterpret_cast<half4_*>(rw_ + (((c >> 1) ^ aswz(p)) << 4)) = h4;                                          \
        *reinterpret_cast<half4_*>(rw_ + (((4 + (c >> 1)) ^ aswz(p)) << 4)) = l4;                                    \
      } else {                                                                                                       \
        *reinterpret_cast<u32x4*>(sA + (BUF) * A_BYTES + p * RSA + ((c ^ aswz(p)) << 4)) =                          \
            ((aok >> s_) & 1u) ? RA[s_] : u32x4{0u, 0u, 0u, 0u};                                                     \
      }                                                                                                              \
    }                                                                                                                \
  }                                                                                                                  \
  if constexpr (AIN != kInS32) range_guard(amx_);                                                                    \
  }
#define OFLOW_LOAD_B(RB, STEP)                                                                                       \
  _Pragma("unroll") for (int s_ = 0; s_ < BPER; ++s_) {                                                              \
    const int item = tid + s_ * NTH;                                                                            \
    if (BITEMS % NTH == 0 || item < BITEMS)                                                                     \
      RB[s_] = __builtin_amdgcn_raw_buffer_load_b128(rsB, boff[s_], (STEP) * a.npad * 128, 0);                      \
  }
#define OFLOW_WRITE_B(RB, BUF)                                                                                       \
  if (!OFLOW_ABL(32)) _Pragma("unroll") for (int s_ = 0; s_ < BPER; ++s_) {                                          \
    const int item = tid + s_ * NTH;                                                                            \
    const int n = item >> 3, c = item & 7;                                                                           \
    if (BITEMS % NTH == 0 || item < BITEMS)                                                                     \
      *reinterpret_cast<u32x4*>(sB + (BUF) * B_BYTES + n * RSB + ((c ^ bswz(n)) << 4)) = RB[s_];                    \
  }
  // operands of one 16-deep sub-step S_ of step I: A rows of this wave's pixel tiles at the step's tap offset, B rows
  // of its channel tiles; hi and lo halves
#define OFLOW_READ_OPS(AH, AL, BH, BL, I, S_)                                                                        \
  {                                                                                                                  \
    const int ii_ = (I);                                                                                              \
    const int t_ = ii_ % T, ky_ = t_ / KW, kx_ = t_ - ky_ * KW;                                                       \
    const uint8_t* bufA_ = sA + (ADB ? (ii_ & 1) * A_BYTES : 0);                                                      \
    const uint8_t* bufB_ = sB + (ii_ & 1) * B_BYTES;                                                                  \
    const int chi_ = 2 * (S_) + hh, clo_ = 4 + 2 * (S_) + hh;                                                        \
    _Pragma("unroll") for (int mt_ = 0; mt_ < MT; ++mt_) {                                                           \
      const int p_ = (wm * MT + mt_ + ky_) * HX + r + kx_;                                                           \
      const uint8_t* row_ = bufA_ + p_ * RSA;                                                                        \
      AH[mt_] = *reinterpret_cast<const half8*>(row_ + ((chi_ ^ aswz(p_)) << 4));                                    \
      AL[mt_] = *reinterpret_cast<const half8*>(row_ + ((clo_ ^ aswz(p_)) << 4));                                    \
    }                                                                                                                \
    _Pragma("unroll") for (int nt_ = 0; nt_ < NT; ++nt_) {                                                           \
      const int n_ = wn * (BN / WN) + nt_ * 32 + r;                                                                  \
      const uint8_t* row_ = bufB_ + n_ * RSB;                                                                        \
      BH[nt_] = *reinterpret_cast<const half8*>(row_ + ((chi_ ^ bswz(n_)) << 4));                                    \
      BL[nt_] = *reinterpret_cast<const half8*>(row_ + ((clo_ ^ bswz(n_)) << 4));                                    \
    }                                                                                                                \
  }
  // hi*lo + lo*hi + hi*hi per (pixel tile, channel tile): the lo*lo term is below fp32 rounding
#define OFLOW_MFMAS(AH, AL, BH, BL)                                                                                  \
  if (!OFLOW_ABL(2)) _Pragma("unroll") for (int mt = 0; mt < MT; ++mt)                                               \
    _Pragma("unroll") for (int nt = 0; nt < NT; ++nt) {                                                              \
      acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(AH[mt], BL[nt], acc[mt][nt], 0, 0, 0);                    \
      acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(AL[mt], BH[nt], acc[mt][nt], 0, 0, 0);                    \
      acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(AH[mt], BH[nt], acc[mt][nt], 0, 0, 0);                    \
    }

  f32x16 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int S = a.kg * T;
  for (int c = tid; c < BN; c += NTH) {
    const int n = min(n0 + c, a.N - 1);
    sSB[c] = make_float2(a.wsc[n], a.bias ? a.bias[n] : 0.f);
  }
  if constexpr (AIN == kInF32Norm) {
    for (int e = tid; e < a.kg * 32; e += NTH)
      sAff[e] = make_float2(a.ia[(long long)b * a.kg * 32 + e], a.ib[(long long)b * a.kg * 32 + e]);
    __syncthreads();
  }
  if constexpr (AIN == kInImg) {
    // the tile's input window (rows 2*ty0 - 3 .., columns 2*tx0 - 3 ..), zero padded (extractor.py:186 padding=3)
    const float* img = reinterpret_cast<const float*>(a.x) + (long long)b * kImgC * (2 * a.H) * (2 * a.W);
    const int iy0 = 2 * ty0 - kImgK / 2, ix0 = 2 * tx0 - kImgK / 2;
    // every load of the window issued before the first LDS store (clamped in-image addresses, zero selected after):
    // a load -> store loop waited out one memory round trip per element (the stem ran 0.6 ms per 8 images)
    constexpr int IMG_N = kImgC * kImgRows * kImgCols, IMG_PER = (IMG_N + NTH - 1) / NTH;
    if (a.exp_flags & 1) {  // experiment: the element-wise load -> store loop
      for (int e = tid; e < IMG_N; e += NTH) {
        const int ch = e / (kImgRows * kImgCols), rem = e - ch * (kImgRows * kImgCols);
        const int ry = rem / kImgCols, rx = rem - ry * kImgCols;
        const int iy = iy0 + ry, ix = ix0 + rx;
        float v = 0.f;
        if (static_cast<unsigned>(iy) < static_cast<unsigned>(2 * a.H) && static_cast<unsigned>(ix) < static_cast<unsigned>(2 * a.W))
          v = img[((long long)ch * (2 * a.H) + iy) * (2 * a.W) + ix];
        sImg[ch * kImgPlane + ry * kImgPitch + (rx & 1) * kImgHalf + (rx >> 1)] = v;
      }
    } else {
    float iv[IMG_PER];
    int io[IMG_PER];
#pragma unroll
    for (int s_ = 0; s_ < IMG_PER; ++s_) {
      const int e = min(tid + s_ * NTH, IMG_N - 1);
      const int ch = e / (kImgRows * kImgCols), rem = e - ch * (kImgRows * kImgCols);
      const int ry = rem / kImgCols, rx = rem - ry * kImgCols;
      const int iy = iy0 + ry, ix = ix0 + rx;
      const bool in = static_cast<unsigned>(iy) < static_cast<unsigned>(2 * a.H) && static_cast<unsigned>(ix) < static_cast<unsigned>(2 * a.W);
      const int cy = min(max(iy, 0), 2 * a.H - 1), cx = min(max(ix, 0), 2 * a.W - 1);
      const float v = img[((long long)ch * (2 * a.H) + cy) * (2 * a.W) + cx];
      iv[s_] = in ? v : 0.f;
      io[s_] = ch * kImgPlane + ry * kImgPitch + (rx & 1) * kImgHalf + (rx >> 1);
    }
#pragma unroll
    for (int s_ = 0; s_ < IMG_PER; ++s_)
      if (tid + s_ * NTH < IMG_N) sImg[io[s_]] = iv[s_];
    }
  }
  if constexpr (AIN == kInFlow) {
    // convf1's input: the tile's flow window (rows ty0 - 3 .., columns tx0 - 3 ..) from coords1 (B, 2, H, W):
    // flow = coords1 - (x, y) as oflow_flow_prep_s32 forms it (raft.py:129), zeros outside the image (padding=3);
    // every load issued before the first LDS store
    const float* co = reinterpret_cast<const float*>(a.x) + (long long)b * 2 * a.H * a.W;
    const int iy0 = ty0 - kImgK / 2, ix0 = tx0 - kImgK / 2;
    constexpr int FL_N = 2 * WROWS * WCOLS, FL_PER = (FL_N + NTH - 1) / NTH;
    float iv[FL_PER];
    int io[FL_PER];
#pragma unroll
    for (int s_ = 0; s_ < FL_PER; ++s_) {
      const int e = min(tid + s_ * NTH, FL_N - 1);
      const int ch = e / (WROWS * WCOLS), rem = e - ch * (WROWS * WCOLS);
      const int ry = rem / WCOLS, rx = rem - ry * WCOLS;
      const int iy = iy0 + ry, ix = ix0 + rx;
      const bool in = static_cast<unsigned>(iy) < static_cast<unsigned>(a.H) && static_cast<unsigned>(ix) < static_cast<unsigned>(a.W);
      const int cy = min(max(iy, 0), a.H - 1), cx = min(max(ix, 0), a.W - 1);
      const float v = co[((long long)ch * a.H + cy) * a.W + cx] - static_cast<float>(ch == 0 ? ix : iy);
      iv[s_] = in ? v : 0.f;
      io[s_] = ch * WPLANE + ry * WPITCH + rx;
    }
#pragma unroll
    for (int s_ = 0; s_ < FL_PER; ++s_)
      if (tid + s_ * NTH < FL_N) sImg[io[s_]] = iv[s_];
  }
  if constexpr (WIN) {
    // patch channel k = t*WC + ch, t = ky*7 + kx -> window offset (-1: zero, k >= 49 * WC)
    for (int k = tid; k < WKPAD; k += NTH) {
      const int t = k / WC, ch = k - t * WC;
      const int ky = t / kImgK, kx = t - ky * kImgK;
      sKoff[k] = t < kImgK * kImgK
                     ? ch * WPLANE + ky * WPITCH + (WS == 2 ? (kx & 1) * WHALF + (kx >> 1) : kx)
                     : -1;
    }
    if (tid == 0) sImg[kImgZero] = 0.f;
    __syncthreads();
  }
  if constexpr (BREG) {
  // ---- register-direct B: the wave's channel tile of every step from the fragment-major weights ----
  const __amdgpu_buffer_rsrc_t rsW =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.wf), (short)0, a.wbytes, 0x00020000);
  const int wlane = ((n0 >> 5) + wn) * 4096 + lane * 16;
  const int wstep = a.npad * 128;  // bytes per (group, tap) step
  // ring of RING steps' B fragments: step i in bq[i % RING]; [sub-step * 2 + (hi, lo)]. Vector-memory loads retire in
  // issue order, so the loads of B issued after a group's halo prefetch (HBM latency) cannot be consumed before it:
  // the ring depth is how many steps the prefetch has before a B wait covers it. 3 where the registers allow it.
  constexpr int RING = (T == 5 && KH == 5 && EPI == 0) ? 2 : OFLOW_BREG_RING;  // (the 5x1 context conv: 255 VGPRs at 2)
  u32x4 bq[RING][4];
  auto load_b = [&](u32x4 (&d)[4], int step) {
#pragma unroll
    for (int e = 0; e < 4; ++e) d[e] = __builtin_amdgcn_raw_buffer_load_b128(rsW, wlane + e * 1024, step * wstep, 0);
  };
#define OFLOW_READ_A(AH, AL, I, S_)                                                                                   \
  {                                                                                                                  \
    const int ii_ = (I);                                                                                              \
    const int t_ = ii_ % T, ky_ = t_ / KW, kx_ = t_ - ky_ * KW;                                                       \
    const int chi_ = 2 * (S_) + hh, clo_ = 4 + 2 * (S_) + hh;                                                        \
    const uint8_t* sAb_ = sA + (HDB && ((ii_ / T) & 1) ? A_BYTES : 0); /* group (I / T)'s halo buffer */          \
    _Pragma("unroll") for (int mt_ = 0; mt_ < MT; ++mt_) {                                                           \
      const int p_ = (wm * MT + mt_ + ky_) * HX + r + kx_;                                                           \
      const uint8_t* row_ = sAb_ + p_ * RSA;                                                                         \
      AH[mt_] = *reinterpret_cast<const half8*>(row_ + (chi_ << 4));                                                 \
      AL[mt_] = *reinterpret_cast<const half8*>(row_ + (clo_ << 4));                                                 \
    }                                                                                                                \
  }
#define OFLOW_MFMAS_R(AH, AL, BC, S_)                                                                                 \
  if (!OFLOW_ABL(2)) _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) {                                             \
    const half8 bh_ = __builtin_bit_cast(half8, BC[2 * (S_)]), bl_ = __builtin_bit_cast(half8, BC[2 * (S_) + 1]);     \
    acc[mt][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(AH[mt], bl_, acc[mt][0], 0, 0, 0);                           \
    acc[mt][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(AL[mt], bh_, acc[mt][0], 0, 0, 0);                           \
    acc[mt][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(AH[mt], bh_, acc[mt][0], 0, 0, 0);                           \
  }
#pragma unroll
  for (int q = 0; q < RING; ++q) load_b(bq[q], q < S ? q : S - 1);
  OFLOW_LOAD_A(ra, 0);
  OFLOW_WRITE_A(ra, 0, 0);
  OFLOW_LOAD_A(ra, a.kg > 1 ? 1 : 0);
  __syncthreads();
  // a loop body of a multiple of RING steps keeps the ring slot of every step static: GPB groups per body
  constexpr int GPB = (T % RING == 0) ? 1 : RING;  // (RING 2 or 3, both prime)
  // Vertical taps (KH x 1): tap ky of row tile mt reads halo row mt + ky, so consecutive taps share MT - 1 of their MT
  // rows: the operands live in registers per halo row and each step reads only its newest row (one row tile's 4 reads
  // instead of MT's 16; LDS operand reads were ~30 of a GRU conv's ~145 us, profiles/r04/s18_abl.log).
  constexpr bool VSLIDE = OFLOW_VSLIDE && KW == 1 && KH > 1 && WM == 1 && !(EPI == 0 && KH == 5);  // (5x1 EPI 0: VGPRs)
  if constexpr (VSLIDE) {
    constexpr int NR = MT + KH - 1;  // halo rows per group
    half8 V[NR][2][2];               // [halo row][sub-step][hi, lo]
    auto rd = [&](int hr, int sub, int grp) {
      const uint8_t* row_ = sA + (HDB && (grp & 1) ? A_BYTES : 0) + (hr * HX + r) * RSA;
      V[hr][sub][0] = *reinterpret_cast<const half8*>(row_ + ((2 * sub + hh) << 4));
      V[hr][sub][1] = *reinterpret_cast<const half8*>(row_ + ((4 + 2 * sub + hh) << 4));
    };
    auto mf = [&](int ky, int sub, u32x4 (&bc)[4]) {
      if (OFLOW_ABL(2)) return;
      const half8 bh_ = __builtin_bit_cast(half8, bc[2 * sub]), bl_ = __builtin_bit_cast(half8, bc[2 * sub + 1]);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        acc[mt][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(V[mt + ky][sub][0], bl_, acc[mt][0], 0, 0, 0);
        acc[mt][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(V[mt + ky][sub][1], bh_, acc[mt][0], 0, 0, 0);
        acc[mt][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(V[mt + ky][sub][0], bh_, acc[mt][0], 0, 0, 0);
      }
    };
#pragma unroll
    for (int m = 0; m < MT; ++m) rd(m, 0, 0);
    for (int g0 = 0; g0 < a.kg; g0 += GPB) {
#pragma unroll
      for (int j = 0; j < GPB * T; ++j) {
        const int gg = g0 + j / T, t = j % T;
        if (GPB > 1 && j > 0 && t == 0 && gg >= a.kg) break;
        const int i_ = gg * T + t;
        u32x4 (&bc)[4] = bq[j % RING];
        if (t == 0) {
#pragma unroll
          for (int m = 0; m < MT; ++m) rd(m, 1, gg);
        } else {
          rd(t + MT - 1, 1, gg);
        }
        mf(t, 0, bc);
        if (t == T - 1) {
          if constexpr (HDB) {
            // group gg+1's halo into the other buffer (last read in group gg-1, before the previous barrier)
            OFLOW_WRITE_A(ra, (gg + 1) & 1, gg + 1 < a.kg ? gg + 1 : gg);
          } else {
            __syncthreads();
            OFLOW_WRITE_A(ra, 0, gg + 1 < a.kg ? gg + 1 : gg);
          }
          const int g2 = gg + 2 < a.kg ? gg + 2 : a.kg - 1;
          OFLOW_LOAD_A(ra, g2);
          __syncthreads();
#pragma unroll
          for (int m = 0; m < MT; ++m) rd(m, 0, gg + 1);  // the next group's first tap (rows 0 .. MT-1: free since tap MT-1)
        } else {
          rd(t + MT, 0, gg);  // the next tap's new row
        }
        mf(t, 1, bc);
        load_b(bc, i_ + RING < S ? i_ + RING : S - 1);
      }
    }
  } else {
  half8 xah[MT], xal[MT], yah[MT], yal[MT];
  OFLOW_READ_A(xah, xal, 0, 0);
  for (int g0 = 0; g0 < a.kg; g0 += GPB) {
#pragma unroll
    for (int j = 0; j < GPB * T; ++j) {
      const int gg = g0 + j / T, t = j % T;
      if (GPB > 1 && j > 0 && t == 0 && gg >= a.kg) break;  // the last body's missing groups (uniform branch)
      const int i_ = gg * T + t;
      u32x4 (&bc)[4] = bq[j % RING];
      OFLOW_READ_A(yah, yal, i_, 1);
      OFLOW_MFMAS_R(xah, xal, bc, 0);
      if (t == T - 1) {  // the halo swap: every wave done reading A(g); A(g+1) visible before its first read
        if constexpr (HDB) {
          OFLOW_WRITE_A(ra, (gg + 1) & 1, gg + 1 < a.kg ? gg + 1 : gg);  // the other buffer (read last in group g-1)
        } else {
          __syncthreads();
          OFLOW_WRITE_A(ra, 0, gg + 1 < a.kg ? gg + 1 : gg);
        }
        const int g2 = gg + 2 < a.kg ? gg + 2 : a.kg - 1;
        OFLOW_LOAD_A(ra, g2);
        __syncthreads();
      }
      OFLOW_READ_A(xah, xal, i_ + 1, 0);
      OFLOW_MFMAS_R(yah, yal, bc, 1);
      load_b(bc, i_ + RING < S ? i_ + RING : S - 1);  // step i+RING into the slot step i used
    }
  }
  }  // VSLIDE
#undef OFLOW_READ_A
#undef OFLOW_MFMAS_R
  } else {
  // prologue: step 0 in LDS, steps 1 .. BD in registers (set d % BD), sub-step 0 operands of step 0 read
  u32x4 rbr[BD][BPER];
  u32x4 rar[ADB ? BD : 1][APER];
  OFLOW_LOAD_B(rbr[0], 0);
  OFLOW_LOAD_A(rar[0], 0);
  OFLOW_WRITE_A(rar[0], 0, 0);
  OFLOW_WRITE_B(rbr[0], 0);
#pragma unroll
  for (int d = 1; d <= BD; ++d) {
    const int id = d < S ? d : S - 1;
    OFLOW_LOAD_B(rbr[d % BD], id);
    if constexpr (ADB) { OFLOW_LOAD_A(rar[d % BD], id); }
  }
  if constexpr (!ADB) { OFLOW_LOAD_A(rar[0], a.kg > 1 ? 1 : 0); }
  __syncthreads();
  half8 xah[MT], xal[MT], xbh[NT], xbl[NT];  // sub-step 0 operands
  half8 yah[MT], yal[MT], ybh[NT], ybl[NT];  // sub-step 1 operands
  OFLOW_READ_OPS(xah, xal, xbh, xbl, 0, 0);

  // The loop body is one input group with its T taps unrolled (static tap index), and nothing in it is conditional:
  // past the last step it re-loads / re-writes the last step's data into buffers no longer read, so the compiler
  // sees every load and counts vmcnt exactly (a halo prefetch from HBM is never waited for by a weight write).
  // (a body of GPB2 groups keeps the register set of every step static: (i + 1) % BD = (j + 1) % BD)
  constexpr int GPB2 = (BD > 1 && (T % BD) != 0) ? BD : 1;
  for (int g0 = 0; g0 < a.kg; g0 += GPB2) {
#pragma unroll
    for (int j = 0; j < GPB2 * T; ++j) {
      const int g = g0 + j / T, t = j % T;
      if (GPB2 > 1 && j > 0 && t == 0 && g >= a.kg) break;  // the last body's missing groups (uniform branch)
      const int i_ = g * T + t;
      u32x4 (&rb)[BPER] = rbr[(j + 1) % BD];
      // 1-2: step i+1's operands into the LDS buffers step i-1 used (free since step i-1's barrier); reload the
      // register set with step i+1+BD's
      OFLOW_WRITE_B(rb, (i_ + 1) & 1);
      if constexpr (ADB) { OFLOW_WRITE_A(rar[(j + 1) % BD], (i_ + 1) & 1, i_ + 1 < S ? i_ + 1 : S - 1); }
      {
        const int i2 = i_ + 1 + BD < S ? i_ + 1 + BD : S - 1;
        OFLOW_LOAD_B(rb, i2);
        if constexpr (ADB) { OFLOW_LOAD_A(rar[(j + 1) % BD], i2); }
      }
      // 3-4
      OFLOW_READ_OPS(yah, yal, ybh, ybl, i_, 1);
      OFLOW_MFMAS(xah, xal, xbh, xbl);
      // 5: at the group's last tap the next group's halo replaces this one (loaded at the group's first tap)
      if constexpr (!ADB) {
        if (t == T - 1) {
          __syncthreads(); /* every wave is done reading A(g) */
          OFLOW_WRITE_A(rar[0], 0, g + 1 < a.kg ? g + 1 : g);
          const int g2 = g + 2 < a.kg ? g + 2 : a.kg - 1;
          OFLOW_LOAD_A(rar[0], g2);
        }
      }
      if (!OFLOW_ABL(64)) __syncthreads(); /* B(i+1) [A] visible; every read of step i done before step i+1 overwrites its buffers */
      // 6-7
      OFLOW_READ_OPS(xah, xal, xbh, xbl, i_ + 1, 0);
      OFLOW_MFMAS(yah, yal, ybh, ybl);
    }
  }
  }  // LDS-staged B
#undef OFLOW_MFMAS
#undef OFLOW_READ_OPS
#undef OFLOW_LOAD_A
#undef OFLOW_WRITE_A
#undef OFLOW_LOAD_B
#undef OFLOW_WRITE_B

  if constexpr (BREG) {
    if (a.ks_slab != nullptr) {
      // Split-K hand-off (MI355X_MICROARCH.md "inter-workgroup visibility"; cdna_hip_programming.md Guideline 16 R1):
      // the tile's two workgroups take tickets from one counter; the first publishes its partial sums write-through
      // (16-B sc1 stores: no release fence), drains them, and one lane bumps the tile's "published" counter; the second
      // polls that counter (relaxed agent-scope loads), drops its L1 with one agent acquire and adds the partials to its
      // own before running the epilogue. fp32 addition is commutative, so acc_0 + acc_1 is the same bits whichever
      // workgroup arrives second. Counters only grow (two tickets and one publication per tile and launch), so they
      // need no reset between launches or graph replays; the host zeroes them once. The second arriver polls only after
      // the first took its ticket (it is resident and past its main loop): no dependence on dispatch order. The poll is
      // bounded (a hang would hold the GPU): past the bound it proceeds without the partials (the results are then
      // wrong, which the parity tests see).
      typedef __attribute__((address_space(1))) unsigned gu32;
      __shared__ unsigned sTicket;
      const int tile_id = blockIdx.y * gridDim.x + blockIdx.x;
      gu32* ctr = (gu32*)(a.ks_ctr) + 2 * tile_id;  // (global address space: no flat atomics)
      if (tid == 0) sTicket = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const unsigned ticket = sTicket;
      // slab of the tile: [wave][mt][nt][16-B quarter of the accumulator][lane 64][16 B] (one wave instruction = 1 KB)
      const __amdgpu_buffer_rsrc_t rsS = __builtin_amdgcn_make_buffer_rsrc(
          a.ks_slab + (size_t)tile_id * (BM * BN), (short)0, BM * BN * 4, 0x00020000);
      const int sbase = wave * (MT * NT * 4096) + lane * 16;
      if ((ticket & 1u) == 0u) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int e4 = 0; e4 < 4; ++e4) {
              const u32x4 v = {__float_as_uint(acc[mt][nt][4 * e4]), __float_as_uint(acc[mt][nt][4 * e4 + 1]),
                               __float_as_uint(acc[mt][nt][4 * e4 + 2]), __float_as_uint(acc[mt][nt][4 * e4 + 3])};
              __builtin_amdgcn_raw_buffer_store_b128(v, rsS, sbase + ((mt * NT + nt) * 4 + e4) * 1024, 0, 16);  // sc1
            }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its write-through stores
        __syncthreads();
        if (tid == 0) __hip_atomic_fetch_add(ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
      if (tid == 0) {
        const unsigned want = (ticket >> 1) + 1u;
        for (unsigned spin = 0; spin < (1u << 24); ++spin) {
          if (static_cast<int>(__hip_atomic_load(ctr + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - want) >= 0) break;
          __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          u32x4 pv[4];
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4)
            pv[e4] = __builtin_amdgcn_raw_buffer_load_b128(rsS, sbase + ((mt * NT + nt) * 4 + e4) * 1024, 0, 0);
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[mt][nt][4 * e4 + j] += __uint_as_float(pv[e4][j]);
        }
    }
  }

  // ---- epilogue: accumulators -> LDS tile [pixel][channel] ----
  constexpr int C8 = BN / 8;
  constexpr int KIT = (BM * C8 + NTH - 1) / NTH;  // epilogue items (pixel x 8 channels) per thread
  // GRU addend (the hoisted context term): its loads are issued here, so they fly while the accumulators go to LDS,
  // and it is folded into the tile (with the scale and bias) before the GRU state is prefetched -- never both sets
  // of registers live at once
  const bool has_add = EPI != 0 && a.add != nullptr;
  u32x4 ad[EPI == 0 ? 1 : KIT][2];
  if (has_add) {
#pragma unroll
    for (int k = 0; k < (EPI == 0 ? 0 : KIT); ++k) {
      const int item = tid + k * NTH;
      const int pl = item / C8, n = n0 + (item - pl * C8) * 8;
      const int y = ty0 + pl / kTX, x = tx0 + (pl % kTX);
      if (item >= BM * C8 || n >= a.N || y >= a.H || x >= a.W) continue;
      const u32x4* ap = reinterpret_cast<const u32x4*>(a.add + (pix0 + (long long)y * a.W + x) * a.addps + n);
      ad[k][0] = ap[0];
      ad[k][1] = ap[1];
    }
  }
  __syncthreads();  // the tile overwrites the operand buffers: every wave is past its last LDS operand read
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
  if constexpr (EPI == 0 && TY >= kTY) {
    if (a.stats != nullptr && !OFLOW_ABL(8)) {
      // instance-norm partials of the conv output (merged by oflow_norm_stats_finalize), from the accumulators: each
      // lane holds one channel of this wave's MT rows (16 pixels per row and lane half); two-pass mean / M2 over its
      // values in fp32, merged with the other lane half (xor 32) and then, per 4-row sub-tile, across the waves that
      // cover it (sStat, after the barrier)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int nl = wn * (BN / WN) + nt * 32 + r;
        const float2 sb = sSB[nl];
        float cnt = 0.f, sum = 0.f, q = 0.f;
        // a tile wholly inside the image (every tile of the 8 / 4-aligned encoder grids) skips the per-value bounds
        // selects: the same sums in the same order (cnt = 16 * MT exactly)
        const bool full = ty0 + TY <= a.H && tx0 + kTX <= a.W;
        if (full) {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int e = 0; e < 16; ++e) sum += acc[mt][nt][e] * sb.x + sb.y;
          cnt = 16.f * MT;
        } else {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            const bool yok = ty0 + wm * MT + mt < a.H;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const bool ok = yok && tx0 + (e & 3) + 8 * (e >> 2) + 4 * hh < a.W;
              sum += ok ? acc[mt][nt][e] * sb.x + sb.y : 0.f;
              cnt += ok ? 1.f : 0.f;
            }
          }
        }
        const float mean = cnt > 0.f ? sum / cnt : 0.f;
        if (full) {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const float d = (acc[mt][nt][e] * sb.x + sb.y) - mean;
              float dd = d * d;
              asm volatile("" : "+v"(dd));  // no fma contraction: the checked form below rounds d * d before the add
              q += dd;
            }
        } else {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            const bool yok = ty0 + wm * MT + mt < a.H;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const bool ok = yok && tx0 + (e & 3) + 8 * (e >> 2) + 4 * hh < a.W;
              const float d = (acc[mt][nt][e] * sb.x + sb.y) - mean;
              q += ok ? d * d : 0.f;
            }
          }
        }
        // merge with lane ^ 32 (symmetric: both lanes compute the same value; lane half 0 first)
        const float nb = __shfl_xor(cnt, 32), mb = __shfl_xor(mean, 32), qb = __shfl_xor(q, 32);
        const float n0_ = hh ? nb : cnt, m0_ = hh ? mb : mean, q0_ = hh ? qb : q;
        const float n1_ = hh ? cnt : nb, m1_ = hh ? mean : mb, q1_ = hh ? q : qb;
        const float nn = n0_ + n1_;
        float M = m0_, Q = q0_;
        if (n1_ > 0.f) {
          if (n0_ > 0.f) {
            const float d = m1_ - m0_;
            M = m0_ + d * (n1_ / nn);
            Q = q0_ + q1_ + d * d * (n0_ * n1_ / nn);
          } else {
            M = m1_;
            Q = q1_;
          }
        }
        if (hh == 0) sStat[wm * BN + nl] = make_float3(nn, M, Q);
      }
    }
  }
  __syncthreads();
  if (has_add) {
    // pre-activation value = acc * scale + bias + addend, in place (each thread rewrites only its own items, which it
    // alone reads below: no barrier). r05: the item's 8 tile values as two 16-B LDS accesses each way (the main
    // epilogue loop's conflict-free pattern) and the channel octet's (scale, bias) read once -- the scalar form (8 + 8
    // dword accesses per item, 16 lanes of a pixel 8 floats apart: 4-way bank conflicts) was the GRU kernels' 0.14 /
    // 0.20 LDS-conflict rate (profiles/r04/s28_pmc_mfma.json)
    constexpr bool FIXED_OCT_ADD = NTH % C8 == 0;
    float2 sba[8];
    if constexpr (FIXED_OCT_ADD) {
#pragma unroll
      for (int j = 0; j < 8; ++j) sba[j] = sSB[(tid % C8) * 8 + j];
    }
#pragma unroll
    for (int k = 0; k < (EPI == 0 ? 0 : KIT); ++k) {
      const int item = tid + k * NTH;
      const int pl = item / C8, nl = (item - pl * C8) * 8, n = n0 + nl;
      const int y = ty0 + pl / kTX, x = tx0 + (pl % kTX);
      if (item >= BM * C8 || n >= a.N || y >= a.H || x >= a.W) continue;
      const float* av = reinterpret_cast<const float*>(&ad[k][0]);
      float4* tp4 = reinterpret_cast<float4*>(&sT[pl * TS + nl]);
      const float4 t0 = tp4[0], t1 = tp4[1];
      float t[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float2 sb = FIXED_OCT_ADD ? sba[j] : sSB[nl + j];
        t[j] = (t[j] * sb.x + sb.y) + av[j];
      }
      tp4[0] = make_float4(t[0], t[1], t[2], t[3]);
      tp4[1] = make_float4(t[4], t[5], t[6], t[7]);
    }
  }

  if (a.f != nullptr) {
    // fp32 NCHW: lanes = consecutive pixels of one tile row (128-B rows of the destination)
    for (int item = tid; item < BM * BN; item += NTH) {
      const int nl = item / BM, pl = item - nl * BM;
      const int n = n0 + nl;
      const int y = ty0 + pl / kTX, x = tx0 + (pl % kTX);
      if (n < a.N && y < a.H && x < a.W) {
        const float2 sb = sSB[nl];
        float v = sT[pl * TS + nl] * sb.x + sb.y;
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
    if (a.stats != nullptr && !OFLOW_ABL(8)) {
      // per-4-row-sub-tile partials from the waves' (count, mean, M2) in sStat, merged in wave order (Chan et al.)
      if constexpr (TY >= kTY) {
        constexpr int NSUB = TY / kTY, WPS = kTY / MT;  // sub-tiles per tile, waves (rows of waves) per sub-tile
        if (tid < BN * NSUB) {
          const int c = tid % BN, sub = tid / BN, n = n0 + c;
          float N0 = 0.f, M0 = 0.f, Q0 = 0.f;
#pragma unroll
          for (int j = 0; j < WPS; ++j) {
            const float3 t = sStat[(sub * WPS + j) * BN + c];
            const float nn = N0 + t.x;
            if (t.x > 0.f) {
              if (N0 > 0.f) {
                const float d = t.y - M0;
                M0 = M0 + d * (t.x / nn);
                Q0 = Q0 + t.z + d * d * (N0 * t.x / nn);
              } else {
                M0 = t.y;
                Q0 = t.z;
              }
              N0 = nn;
            }
          }
          if (n < a.N && ty0 + sub * kTY < a.H) {
            const int tiles4_y = (a.H + kTY - 1) / kTY;
            const int tile_in_img = (ty0 / kTY + sub) * a.tiles_x + tx0 / kTX;
            float* st = a.stats + (((long long)b * a.tiles_x * tiles4_y + tile_in_img) * a.npad + n) * 3;
            st[0] = N0;
            st[1] = M0;
            st[2] = Q0;
          }
        }
      }
    }
    if ((a.y0 == nullptr && a.fn == nullptr) || OFLOW_ABL(16)) return;
  }

  if (OFLOW_ABL(16)) return;
  // S32 / GRU consumers: one thread = one pixel x 8 consecutive channels, KIT items per thread. The GRU state operands
  // of every item (h; z) are loaded first, all in flight at once, then consumed: one memory round trip per epilogue
  // instead of one per item.
  u32x4 pre[EPI == 0 ? 1 : KIT][EPI == 2 ? 4 : 2];
#pragma unroll
  for (int k = 0; k < (EPI == 0 ? 0 : KIT); ++k) {
    const int item = tid + k * NTH;
    const int pl = item / C8, nl = (item - pl * C8) * 8, n = n0 + nl;
    const int y = ty0 + pl / kTX, x = tx0 + (pl % kTX);
    if (item >= BM * C8 || n >= a.N || y >= a.H || x >= a.W) continue;
    const long long P = pix0 + (long long)y * a.W + x;
    if constexpr (EPI == 1) {
      if (n >= a.gch) {
        const u32x4* hp = reinterpret_cast<const u32x4*>(a.h + P * a.gch + (n - a.gch));
        pre[k][0] = hp[0];
        pre[k][1] = hp[1];
      }
    } else if constexpr (EPI == 2) {
      const u32x4* hp = reinterpret_cast<const u32x4*>(a.h + P * a.gch + n);
      const u32x4* zp = reinterpret_cast<const u32x4*>(a.z + P * a.gch + n);
      pre[k][0] = hp[0];
      pre[k][1] = hp[1];
      pre[k][2] = zp[0];
      pre[k][3] = zp[1];
    }
  }
  // the gates from the hardware exp2 / reciprocal (default; in-process step A/B 19.31 -> 19.05 ms, flows within
  // 2.8e-5 px, profiles/r04/s15_ab.log); exp flag 256: libm expf / tanhf and IEEE division (A/B only)
  const bool hwx = (a.exp_flags & 256) == 0;
  constexpr int UNR = EPI == 0 ? 1 : KIT;  // GRU: unrolled (pre[k] in registers); EPI 0: a plain loop
  float gmx = 0.f;  // max |x| of every S32 value this thread stores (one range-guard branch, after the loop)
  // where every item of a thread has the same channel octet (NTH a multiple of BN / 8), its (scale, bias) pairs are
  // read once: in the plain loop each item would otherwise wait on 8 dependent LDS round trips
  constexpr bool FIXED_OCT = NTH % C8 == 0;
  float2 sbv[8];
  if constexpr (FIXED_OCT) {
#pragma unroll
    for (int j = 0; j < 8; ++j) sbv[j] = sSB[(tid % C8) * 8 + j];
  }
#pragma unroll UNR
  for (int k = 0; k < KIT; ++k) {
    const int item = tid + k * NTH;
    const int pl = item / C8, c8 = item - pl * C8;
    const int nl = c8 * 8, n = n0 + nl;
    const int y = ty0 + pl / kTX, x = tx0 + (pl % kTX);
    if (item >= BM * C8 || n >= a.N || y >= a.H || x >= a.W) continue;
    const long long P = pix0 + (long long)y * a.W + x;
    const float* pf = reinterpret_cast<const float*>(&pre[EPI == 0 ? 0 : k][0]);  // GRU: [0..7] h, [8..15] z
    const float4 t0 = *reinterpret_cast<const float4*>(&sT[pl * TS + nl]);
    const float4 t1 = *reinterpret_cast<const float4*>(&sT[pl * TS + nl + 4]);
    float v[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
    if (!has_add) {  // (with the addend the tile already holds the pre-activation value)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float2 sb = FIXED_OCT ? sbv[j] : sSB[nl + j];
        v[j] = v[j] * sb.x + sb.y;
      }
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
        store_s32(a.y0, a.y0ps, Pd, nd, a.s2d ? 4 * a.N : a.N, v, gmx);
        if (a.y1) store_s32(a.y1, a.y1ps, Pd, nd, a.s2d ? 4 * a.N : a.N, v, gmx);
      }
    } else if constexpr (EPI == 1) {
      // [z | r] gates (update.py:91-96): z = sigmoid -> a.z; r*h = sigmoid(r) * h -> S32 y0 (channel n - gch)
      if (n < a.gch) {
        // two 16-B stores per item (a.z rows of gch = 128 floats, n % 8 == 0: 32-B aligned); as 8 dword stores the
        // compiler could not prove the alignment and each wave instruction wrote 64 lanes' 4 B, 32 B apart
        float4* zp = reinterpret_cast<float4*>(a.z + P * a.gch + n);
        float zv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) zv[j] = hwx ? sigmoid_hw(v[j]) : 1.0f / (1.0f + expf(-v[j]));
        zp[0] = make_float4(zv[0], zv[1], zv[2], zv[3]);
        zp[1] = make_float4(zv[4], zv[5], zv[6], zv[7]);
      } else {
        float rh[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) rh[j] = (hwx ? sigmoid_hw(v[j]) : 1.0f / (1.0f + expf(-v[j]))) * pf[j];
        store_s32(a.y0, a.y0ps, P, n - a.gch, a.gch, rh, gmx);
      }
    } else {
      // candidate + blend (update.py:96-97): h = (1 - z) * h + z * tanh(q); h (fp32) in place + S32 y0
      float* hp = a.h + P * a.gch + n;
      float hn[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float q = hwx ? tanh_hw(v[j]) : tanhf(v[j]);
        const float z = pf[8 + j];
        hn[j] = (1.0f - z) * pf[j] + z * q;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) hp[j] = hn[j];
      store_s32(a.y0, a.y0ps, P, n, a.N, hn, gmx);
    }
  }
  range_guard(gmx);
}

inline dim3 conv_grid(const ConvArgs& a, int bn) {
  const int ntiles = a.tiles_x * a.tiles_y * a.B;
  return OFLOW_XCD_MAP ? dim3(ntiles * (a.npad / bn)) : dim3(ntiles, a.npad / bn);
}

// LDS-staged kernels: operands prefetched two steps ahead (BD 2). r06 in-process A/B on the replayed 8-pair graph,
// alternated (tools/exp/run_graph_ab.py, profiles/r06/r6s16_ab.log): 17.883 (BD 1) -> 17.720 ms/step, bit-identical
// (the same MFMAs in the same order; only the loads move). The loop's ISA has no s_waitcnt vmcnt(0) left (7-9 per
// input group with BD 1).
template <int KH, int KW, int BN, int WM, int WN, int EPI, int TY, int AIN>
void launch_staged(const ConvArgs& a, dim3 grid, hipStream_t s) {
  hipLaunchKernelGGL((conv_s32_kernel<KH, KW, BN, WM, WN, EPI, TY, AIN, false, 2>), grid, dim3(64 * WM * WN), 0, s, a);
}

template <int KH, int KW, int BN, int WM, int WN, int EPI, int TY = kTY, bool BREG = false>
int launch_conv(const ConvArgs& a0, hipStream_t s) {
  ConvArgs a = a0;
  if constexpr (BREG) {
    a.tiles_y = (a.H + TY - 1) / TY;
    dim3 grid = conv_grid(a, BN);
    if (a.ks_slab != nullptr) {
      if (OFLOW_XCD_MAP || (long long)grid.x * grid.y > a.ks_tiles) return OFLOW_E_SHAPE;
      grid.z = 2;
    }
    hipLaunchKernelGGL((conv_s32_kernel<KH, KW, BN, WM, WN, EPI, TY, kInS32, true>), grid, dim3(64 * WM * WN), 0, s, a);
    return launch_status();
  } else {
  a.tiles_y = (a.H + TY - 1) / TY;
  dim3 grid = conv_grid(a, BN);
  if constexpr (KH == 3 && KW == 3 && EPI == 0) {  // the encoders' second block convs
    if (a.ain == kInF32Norm) {
      launch_staged<KH, KW, BN, WM, WN, EPI, TY, kInF32Norm>(a, grid, s);
      return launch_status();
    }
  }
  if constexpr (KH == 1 && KW == 1 && EPI == 0 && BN == 64 && TY == kTY) {  // the encoders' stem from the image
    if (a.ain == kInImg) {
      launch_staged<KH, KW, BN, WM, WN, EPI, TY, kInImg>(a, grid, s);
      return launch_status();
    }
  }
  if constexpr (KH == 1 && KW == 1 && EPI == 0 && BN == 128 && TY == kTY) {  // convf1 from coords1's flow window
    if (a.ain == kInFlow) {
      launch_staged<KH, KW, BN, WM, WN, EPI, TY, kInFlow>(a, grid, s);
      return launch_status();
    }
  }
  if constexpr (KH == 1 && KW == 1 && EPI == 0 && BN == 128) {  // convc1 on the NHWC corr lookup
    if (a.ain == kInF32) {
      launch_staged<KH, KW, BN, WM, WN, EPI, TY, kInF32>(a, grid, s);
      return launch_status();
    }
  }
  if (a.ain != kInS32) return OFLOW_E_MODE;
  launch_staged<KH, KW, BN, WM, WN, EPI, TY, kInS32>(a, grid, s);
  return launch_status();
  }
}

// Small grids (batch 1 and other small images: under 16384 output pixels, e.g. every update-block conv of one Sintel
// pair launches 28-112 workgroups on 256 CUs at the default tiles): 2-row x 32-column tiles and 64-channel blocks, up
// to 4x the workgroups. Same k order per output element, so the results are bit-identical to the default tiles.
// In-process A/B (tools/exp/run_small_grid_ab.py): batch 1 x 24 iterations 12.9 -> 8.8 ms; a pixel threshold keeps
// the 4-pair lanes of the 8-pair step (28160 px) on the default tiles, where the small ones cost +1.5-3 %.
int g_small_grid_px = 16384;  // output-pixel count under which the small tiles are used (0: never; experiments only)
// instance-norm convs (encoders, BN 64) on 8-row tiles too (outputs bit-identical). Alone the 8-row tiles are 0-12 %
// faster per layer; r03 measured the eager step slower with them (fnet's halves and cnet share the chip and their
// 71 KB of LDS per workgroup crowded the other streams' workgroups: 20.40 (4-row) vs 20.69-20.90 ms,
// profiles/r03/exp/s8b_ab_enc.log). r05, on the replayed graph with the r05 kernels: 457.5 / 457.4 vs 453.6 / 453.9
// pairs/s (profiles/r05/s58_*.log), so on by default (oflow_exp_set_stats_8row(0) restores the 4-row tiles).
int g_stats_8row = 1;
int g_conv_exp_flags = 0;
// BN 64 convs without instance-norm partials (cnet's layer1, convc2, the motion conv) on 8-row tiles (experiments
// only). r02 adopted them from per-layer timings; in the step (concurrent streams) the 4-row tiles win: interleaved
// in-process A/B 20.36 vs 20.53-20.55 ms (profiles/r03/exp/s9_ab_bn64.log).
int g_bn64_8row = 0;
// r04 register-direct workgroup shapes measured against the 1 x 4 waves of 4 row tiles (bit-identical, not kept):
// 256-channel 8-wave workgroups (1 x 8, one per CU, the halo staged once for all 256 channels): GRU z|r 139.6 / 138.0
// -> 144.8 / 149.9 us, step 18.96 -> 19.74 ms (profiles/r04/s26_*) -- with one workgroup per CU each halo-swap
// barrier idles the CU's matrix cores; 128-channel 8-wave workgroups (2 x 4 of 2 row tiles, <= 128 VGPRs, four waves
// per SIMD): z|r 141.0 / 141.1 -> 148.9 / 150.3 us, step 19.07 -> 19.65 ms (s27_*).
// (a split-K call always takes the default tiles: the caller decides the split from its whole batch, so that pair
// lanes of a forward compute what one lane computes, bit for bit, whatever their own sizes)
inline bool small_grid(const ConvArgs& a, int bn) {
  return (long long)a.B * a.H * a.W < g_small_grid_px && a.stats == nullptr && a.ain == kInS32 && a.npad % 64 == 0 &&
         bn >= 64 && a.ks_slab == nullptr;
}

// register-direct weights (BREG): 128-channel blocks of T > 1 convs on S32 input, given the fragment-major weights.
// r04 A/B (profiles/r04/s16_*): the same for 64-channel 3x3 blocks as two-wave workgroups (four per CU) was slower
// (convc2 170 -> 179 us, convf2 35 -> 49 us alone; step -0.9 % instead of -4 %), and with instance-norm partials one
// wave per 4-row sub-tile changes the partials' summation order (not bit-identical to the LDS-staged kernel): neither
// kept.
inline bool use_breg(const ConvArgs& a, int bn, int taps) {
  return a.wf != nullptr && (bn == 128 || bn == 64 || bn == 32) && taps > 1 && a.ain == kInS32 && a.stats == nullptr &&
         !small_grid(a, bn);
}

template <int KH, int KW, int EPI>
int launch_bn(const ConvArgs& a, int bn, hipStream_t s) {
  if (small_grid(a, bn)) return launch_conv<KH, KW, 64, 2, 2, EPI, 2>(a, s);
  if constexpr (KH * KW > 1 && KH * KW != 4)  // (the 2x2 instance spills)
    if (use_breg(a, bn, KH * KW)) {
      if (bn == 128) return launch_conv<KH, KW, 128, 1, 4, EPI, kTY, true>(a, s);
      // 64-channel blocks: 2 x 2 waves, each 2 row tiles x one 32-channel tile (3x3 only)
      if constexpr (KH == 3 && KW == 3) {
        if (bn == 64) return launch_conv<KH, KW, 64, 2, 2, EPI, kTY, true>(a, s);
        // 32-channel blocks (the flow head's 256 -> 2 output conv): 4 x 1 waves, one row tile each, all four loading
        // the same B fragments (no per-step B staging or barrier)
        return launch_conv<KH, KW, 32, 4, 1, EPI, kTY, true>(a, s);
      }
    }
  switch (bn) {
    case 128: return launch_conv<KH, KW, 128, 2, 2, EPI>(a, s);
    case 96: return launch_conv<KH, KW, 96, 4, 1, EPI>(a, s);
    case 64:
      // 8-row tiles (each wave 64 px x 64 ch: 8 operand reads per 12 MFMAs instead of 6 per 6); instance-norm
      // partials are written per 4-row half
      // (1x1 convs double-buffer the 8-row halo: 4-row tiles keep two workgroups per CU within the LDS)
      if constexpr (KH * KW > 1)
        if (a.stats == nullptr ? g_bn64_8row != 0 : g_stats_8row != 0) return launch_conv<KH, KW, 64, 4, 1, EPI, 8>(a, s);
      return launch_conv<KH, KW, 64, 2, 2, EPI>(a, s);
    case 32: return launch_conv<KH, KW, 32, 4, 1, EPI>(a, s);
    default: return OFLOW_E_SHAPE;
  }
}

int dispatch_conv(const ConvArgs& a, int kh, int kw, int block_n, int epilogue, hipStream_t s) {
  const int key = kh * 16 + kw;
  switch (epilogue) {
    case 0:
      switch (key) {
        case 0x11: return launch_bn<1, 1, 0>(a, block_n, s);
        case 0x22: return launch_bn<2, 2, 0>(a, block_n, s);
        case 0x33: return launch_bn<3, 3, 0>(a, block_n, s);
        case 0x15: return launch_bn<1, 5, 0>(a, block_n, s);
        case 0x51: return launch_bn<5, 1, 0>(a, block_n, s);
        default: return OFLOW_E_SHAPE;
      }
    case 1:
      if (block_n != 128) return OFLOW_E_SHAPE;
      if (small_grid(a, block_n)) {
        if (key == 0x15) return launch_conv<1, 5, 64, 2, 2, 1, 2>(a, s);
        if (key == 0x51) return launch_conv<5, 1, 64, 2, 2, 1, 2>(a, s);
      }
      if (use_breg(a, block_n, kh * kw)) {
        if (key == 0x15) return launch_conv<1, 5, 128, 1, 4, 1, kTY, true>(a, s);
        if (key == 0x51) return launch_conv<5, 1, 128, 1, 4, 1, kTY, true>(a, s);
      }
      if (key == 0x15) return launch_conv<1, 5, 128, 2, 2, 1>(a, s);
      if (key == 0x51) return launch_conv<5, 1, 128, 2, 2, 1>(a, s);
      return OFLOW_E_SHAPE;
    default:
      if (block_n != 128) return OFLOW_E_SHAPE;
      if (small_grid(a, block_n)) {
        if (key == 0x15) return launch_conv<1, 5, 64, 2, 2, 2, 2>(a, s);
        if (key == 0x51) return launch_conv<5, 1, 64, 2, 2, 2, 2>(a, s);
      }
      if (use_breg(a, block_n, kh * kw)) {
        if (key == 0x15) return launch_conv<1, 5, 128, 1, 4, 2, kTY, true>(a, s);
        if (key == 0x51) return launch_conv<5, 1, 128, 1, 4, 2, kTY, true>(a, s);
      }
      if (key == 0x15) return launch_conv<1, 5, 128, 2, 2, 2>(a, s);
      if (key == 0x51) return launch_conv<5, 1, 128, 2, 2, 2>(a, s);
      return OFLOW_E_SHAPE;
  }
}

// argument checks + ConvArgs for oflow_conv_s32_ex
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
  // the GRU epilogues read h / z and write z as 16-B vectors (rows of gru_channels floats, n % 8 == 0)
  if (epilogue != 0 && (((uintptr_t)d_gru_h & 15) || ((uintptr_t)d_gru_z & 15))) return OFLOW_E_ALIGN;
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
  // the loads address the weights and one image of the input with 32-bit offsets
  const long long wbytes = (long long)in_groups * kh * kw * n_pad * 128;
  if (wbytes >= (1ll << 31) || (long long)H * W * x_pixel_stride >= (1ll << 31)) return OFLOW_E_SHAPE;
  a.wbytes = static_cast<int>(wbytes);
  a.exp_flags = g_conv_exp_flags;
  (void)block_n;
  return OFLOW_OK;
}

}  // namespace
OFLOW_RANGE_FLAG_SETTER(conv)
}  // namespace oflow

using namespace oflow;

extern "C" int oflow_conv_s32_ex5(const void* d_x, long long x_pixel_stride, int in_groups, const void* d_wpack,
                                  int n_pad, const float* d_wscale, const float* d_bias, int N, int B, int H, int W, int kh,
                                  int kw, int block_n, int epilogue, int activation, float out_scale, void* d_y0,
                                  long long y0_pixel_stride, void* d_y1, long long y1_pixel_stride, float* d_f32,
                                  long long f32_batch_stride, long long f32_channel_stride, int f32_accumulate,
                                  float* d_gru_h, float* d_gru_z, int gru_channels, float* d_nhwc, int nhwc_pixel_stride,
                                  float* d_stats, const void* d_res, long long res_pixel_stride, int res_activation,
                                  int s2d, int in_format, const float* d_in_scale, const float* d_in_shift,
                                  const float* d_addend, long long addend_pixel_stride, const void* d_wfrag,
                                  float* d_ksplit_slab, unsigned* d_ksplit_ctr, long long ksplit_tiles, void* stream);

extern "C" int oflow_conv_s32_ex4(const void* d_x, long long x_pixel_stride, int in_groups, const void* d_wpack,
                                  int n_pad, const float* d_wscale, const float* d_bias, int N, int B, int H, int W, int kh,
                                  int kw, int block_n, int epilogue, int activation, float out_scale, void* d_y0,
                                  long long y0_pixel_stride, void* d_y1, long long y1_pixel_stride, float* d_f32,
                                  long long f32_batch_stride, long long f32_channel_stride, int f32_accumulate,
                                  float* d_gru_h, float* d_gru_z, int gru_channels, float* d_nhwc, int nhwc_pixel_stride,
                                  float* d_stats, const void* d_res, long long res_pixel_stride, int res_activation,
                                  int s2d, int in_format, const float* d_in_scale, const float* d_in_shift,
                                  const float* d_addend, long long addend_pixel_stride, const void* d_wfrag, void* stream) {
  return oflow_conv_s32_ex5(d_x, x_pixel_stride, in_groups, d_wpack, n_pad, d_wscale, d_bias, N, B, H, W, kh, kw,
                            block_n, epilogue, activation, out_scale, d_y0, y0_pixel_stride, d_y1, y1_pixel_stride,
                            d_f32, f32_batch_stride, f32_channel_stride, f32_accumulate, d_gru_h, d_gru_z, gru_channels,
                            d_nhwc, nhwc_pixel_stride, d_stats, d_res, res_pixel_stride, res_activation, s2d, in_format,
                            d_in_scale, d_in_shift, d_addend, addend_pixel_stride, d_wfrag, nullptr, nullptr, 0, stream);
}

extern "C" int oflow_conv_s32_ex5(const void* d_x, long long x_pixel_stride, int in_groups, const void* d_wpack,
                                  int n_pad, const float* d_wscale, const float* d_bias, int N, int B, int H, int W, int kh,
                                  int kw, int block_n, int epilogue, int activation, float out_scale, void* d_y0,
                                  long long y0_pixel_stride, void* d_y1, long long y1_pixel_stride, float* d_f32,
                                  long long f32_batch_stride, long long f32_channel_stride, int f32_accumulate,
                                  float* d_gru_h, float* d_gru_z, int gru_channels, float* d_nhwc, int nhwc_pixel_stride,
                                  float* d_stats, const void* d_res, long long res_pixel_stride, int res_activation,
                                  int s2d, int in_format, const float* d_in_scale, const float* d_in_shift,
                                  const float* d_addend, long long addend_pixel_stride, const void* d_wfrag,
                                  float* d_ksplit_slab, unsigned* d_ksplit_ctr, long long ksplit_tiles, void* stream) {
  ConvArgs a;
  const int st = build_conv_args(a, d_x, x_pixel_stride, in_groups, d_wpack, n_pad, d_wscale, d_bias, N, B, H, W, kh, kw,
                                 block_n, epilogue, activation, out_scale, d_y0, y0_pixel_stride, d_y1, y1_pixel_stride,
                                 d_f32, f32_batch_stride, f32_channel_stride, f32_accumulate, d_gru_h, d_gru_z,
                                 gru_channels, d_nhwc, nhwc_pixel_stride, d_stats, d_res, res_pixel_stride,
                                 res_activation, s2d);
  if (st != OFLOW_OK) return st;
  if (d_wfrag) {  // the fragment-major copy of d_wpack (same size; n_pad a multiple of 32)
    if ((uintptr_t)d_wfrag & 15) return OFLOW_E_ALIGN;
    if (n_pad % 32) return OFLOW_E_SHAPE;
    a.wf = static_cast<const uint8_t*>(d_wfrag);
  }
  if (in_format < kInS32 || in_format > kInFlow) return OFLOW_E_MODE;
  if (in_format == kInFlow) {  // convf1 from coords1: 1x1 geometry over 4 patch groups, BN 128, epilogue 0
    if (kh != 1 || kw != 1 || epilogue != 0 || block_n != 128 || in_groups != (kImgK * kImgK * 2 + 31) / 32)
      return OFLOW_E_MODE;
    if ((long long)2 * B * H * W >= (1ll << 31) || d_addend) return OFLOW_E_SHAPE;
    a.ain = in_format;
    return dispatch_conv(a, kh, kw, block_n, epilogue, static_cast<hipStream_t>(stream));
  }
  if (in_format == kInImg) {  // the stem from the image: 1x1 geometry over 5 patch groups, BN 64, epilogue 0
    if (kh != 1 || kw != 1 || epilogue != 0 || block_n != 64 || in_groups != (kImgK * kImgK * kImgC + 31) / 32)
      return OFLOW_E_MODE;
    if ((long long)kImgC * 4 * H * W >= (1ll << 31)) return OFLOW_E_SHAPE;
    a.ain = in_format;
    if (d_addend) return OFLOW_E_MODE;
    return dispatch_conv(a, kh, kw, block_n, epilogue, static_cast<hipStream_t>(stream));
  }
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
  if (d_addend) {  // GRU epilogues only; 16-B aligned rows of >= N floats
    if (epilogue == 0) return OFLOW_E_MODE;
    // the epilogue reads whole 8-float octets of every row: N a multiple of 8 keeps them inside the row
    if (N % 8) return OFLOW_E_SHAPE;
    if (((uintptr_t)d_addend & 15) || (addend_pixel_stride & 3) || addend_pixel_stride < N) return OFLOW_E_ALIGN;
    a.add = d_addend;
    a.addps = addend_pixel_stride;
  }
  if (d_ksplit_slab || d_ksplit_ctr) {
    // split-K over the input groups: only the register-direct kernels (S32 input, fragment-major weights, multi-tap,
    // 4-row tiles) take it; any other path this call would dispatch to runs unsplit (same results up to the order of
    // one fp32 addition per output)
    if (!d_ksplit_slab || !d_ksplit_ctr) return OFLOW_E_NULL;
    if (((uintptr_t)d_ksplit_slab & 15) || ((uintptr_t)d_ksplit_ctr & 7)) return OFLOW_E_ALIGN;
    if (ksplit_tiles <= 0) return OFLOW_E_SHAPE;
    // (the register-direct instances: launch_bn / dispatch_conv -- 128-channel blocks of any multi-tap kernel but 2x2,
    // 64- and 32-channel blocks of 3x3 ones; the GRU epilogues 1x5 / 5x1 only -- at the default tiles whatever the
    // grid's size, see small_grid)
    a.ks_slab = d_ksplit_slab;
    const bool breg = in_format == kInS32 && a.wf != nullptr && use_breg(a, block_n, kh * kw) && kh * kw != 4 &&
                      (block_n == 128 || (kh == 3 && kw == 3)) && (epilogue == 0 || kh * kw == 5);
    a.ks_slab = nullptr;
    if (breg && (in_groups % 2) == 0) {
      // ksplit_tiles: the slab's capacity in (4 x 32-pixel tile, block_n channels) units of 128 * block_n floats
      if ((long long)B * ((H + kTY - 1) / kTY) * ((W + kTX - 1) / kTX) * (n_pad / block_n) > ksplit_tiles)
        return OFLOW_E_SHAPE;
      a.ks_slab = d_ksplit_slab;
      a.ks_ctr = d_ksplit_ctr;
      a.ks_tiles = ksplit_tiles;
      a.kg = in_groups / 2;
      a.wbytes /= 2;
    }
  }
  return dispatch_conv(a, kh, kw, block_n, epilogue, static_cast<hipStream_t>(stream));
}

extern "C" int oflow_conv_s32_ex3(const void* d_x, long long x_pixel_stride, int in_groups, const void* d_wpack,
                                  int n_pad, const float* d_wscale, const float* d_bias, int N, int B, int H, int W, int kh,
                                  int kw, int block_n, int epilogue, int activation, float out_scale, void* d_y0,
                                  long long y0_pixel_stride, void* d_y1, long long y1_pixel_stride, float* d_f32,
                                  long long f32_batch_stride, long long f32_channel_stride, int f32_accumulate,
                                  float* d_gru_h, float* d_gru_z, int gru_channels, float* d_nhwc, int nhwc_pixel_stride,
                                  float* d_stats, const void* d_res, long long res_pixel_stride, int res_activation,
                                  int s2d, int in_format, const float* d_in_scale, const float* d_in_shift,
                                  const float* d_addend, long long addend_pixel_stride, void* stream) {
  return oflow_conv_s32_ex4(d_x, x_pixel_stride, in_groups, d_wpack, n_pad, d_wscale, d_bias, N, B, H, W, kh, kw,
                            block_n, epilogue, activation, out_scale, d_y0, y0_pixel_stride, d_y1, y1_pixel_stride,
                            d_f32, f32_batch_stride, f32_channel_stride, f32_accumulate, d_gru_h, d_gru_z, gru_channels,
                            d_nhwc, nhwc_pixel_stride, d_stats, d_res, res_pixel_stride, res_activation, s2d, in_format,
                            d_in_scale, d_in_shift, d_addend, addend_pixel_stride, nullptr, stream);
}

extern "C" int oflow_conv_s32_ex2(const void* d_x, long long x_pixel_stride, int in_groups, const void* d_wpack,
                                  int n_pad, const float* d_wscale, const float* d_bias, int N, int B, int H, int W, int kh,
                                  int kw, int block_n, int epilogue, int activation, float out_scale, void* d_y0,
                                  long long y0_pixel_stride, void* d_y1, long long y1_pixel_stride, float* d_f32,
                                  long long f32_batch_stride, long long f32_channel_stride, int f32_accumulate,
                                  float* d_gru_h, float* d_gru_z, int gru_channels, float* d_nhwc, int nhwc_pixel_stride,
                                  float* d_stats, const void* d_res, long long res_pixel_stride, int res_activation,
                                  int s2d, int in_format, const float* d_in_scale, const float* d_in_shift,
                                  void* stream) {
  return oflow_conv_s32_ex3(d_x, x_pixel_stride, in_groups, d_wpack, n_pad, d_wscale, d_bias, N, B, H, W, kh, kw,
                            block_n, epilogue, activation, out_scale, d_y0, y0_pixel_stride, d_y1, y1_pixel_stride,
                            d_f32, f32_batch_stride, f32_channel_stride, f32_accumulate, d_gru_h, d_gru_z, gru_channels,
                            d_nhwc, nhwc_pixel_stride, d_stats, d_res, res_pixel_stride, res_activation, s2d, in_format,
                            d_in_scale, d_in_shift, nullptr, 0, stream);
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

// experiment hook (not part of include/oflow.h): the small-grid pixel threshold, for in-process A/B runs (tools/exp)
extern "C" void oflow_exp_set_small_grid_px(int pixels) { oflow::g_small_grid_px = pixels; }
extern "C" void oflow_exp_set_stats_8row(int on) { oflow::g_stats_8row = on; }
extern "C" void oflow_exp_set_conv_flags(int flags) { oflow::g_conv_exp_flags = flags; }
extern "C" void oflow_exp_set_bn64_8row(int on) { oflow::g_bn64_8row = on; }
