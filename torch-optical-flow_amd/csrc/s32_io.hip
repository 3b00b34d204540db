// Producers of the S32 split-fp16 activation format (conv_s32.hip) around the RAFT update loop (gfx950).
//
//   oflow_pack_s32_f32  : NCHW fp32 -> act -> S32 slice(s) (+ optional NHWC fp32 copy). Feeds the context
//                         features into the GRU buffers: net = tanh(cnet[:, :hdim]), inp = relu(cnet[:, hdim:])
//                         (methods/raft/model/raft.py:115-118).
//   oflow_flow_prep_s32 : flow = coords1 - coords0 (raft.py:129; coords0 is the pixel grid, exact) written as
//                         (a) the two flow channels of the GRU input buffers (update.py:127-128: cat([out, flow]))
//                         and (b) the 7x7 patch matrix of convf1 (update.py:116), channel t*2 + c = flow channel c
//                         at tap t = ky*7 + kx, zero padded (so convf1 runs as a 1x1 split-fp16 GEMM, K = 98 -> 128).
#include "oflow_internal.h"

namespace oflow {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float act_fn(float v, int act) {
  if (act == 1) return v < 0.f ? 0.f : v;
  if (act == 2) return 1.0f / (1.0f + expf(-v));
  if (act == 3) return tanhf(v);
  return v;
}

__device__ __forceinline__ void put8(uint8_t* line, const float* v) {
  range_guard8(v);
  half8 hi, lo;
  split_vec(v, hi, lo);
  *reinterpret_cast<half8*>(line) = hi;
  *reinterpret_cast<half8*>(line + 64) = lo;
}

// one thread = one pixel x 32 channels (4 octets); consecutive threads = consecutive pixels (coalesced NCHW reads).
// Source channel c goes to destination channel yc0 + c (yc0 % 8 == 0); an octet's channels beyond C are written as
// zeros. A thread writes its 4 octets back to back (with yc0 % 32 == 0: the whole 128-B S32 line of the group; one
// thread per octet wrote 16-B pieces of each line at far-apart times: 49 us per 4-pair launch in the step).
__global__ __launch_bounds__(256) void pack_s32_kernel(const float* __restrict__ x, long long xbs, int C, int B, int HW,
                                                       int act, int yc0, uint8_t* y0, long long y0ps, uint8_t* y1,
                                                       long long y1ps, float* f, int fcs) {
  // 32-bit indexing (the host checks P * C8 < 2^31): 64-bit divisions dominated these memory-bound kernels
  const int P = B * HW;
  const int C32 = (C + 31) / 32;
  const int item = blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= P * C32) return;
  const int c32 = item / P;
  const long long p = item - c32 * P;
  const int b = static_cast<int>(p) / HW;
  const int pix = static_cast<int>(p) - b * HW;
  const bool f16b = f != nullptr && (fcs & 3) == 0 && (reinterpret_cast<uintptr_t>(f) & 15) == 0;
#pragma unroll
  for (int o = 0; o < 4; ++o) {
    const int c0 = c32 * 32 + o * 8;
    if (c0 >= C) break;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      v[j] = c < C ? act_fn(x[b * xbs + (long long)c * HW + pix], act) : 0.f;
    }
    const int cd = yc0 + c0;  // destination channel (multiple of 8)
    const long long off = (long long)(cd >> 5) * 128 + ((cd & 31) >> 3) * 16;
    put8(y0 + p * y0ps + off, v);
    if (y1) put8(y1 + p * y1ps + off, v);
    if (f) {
      float* fp = f + p * fcs + c0;
      if (f16b && c0 + 8 <= C) {  // two 16-B stores (was 8 dword stores 4 * fcs bytes apart across the lanes)
        reinterpret_cast<float4*>(fp)[0] = make_float4(v[0], v[1], v[2], v[3]);
        reinterpret_cast<float4*>(fp)[1] = make_float4(v[4], v[5], v[6], v[7]);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (c0 + j < C) fp[j] = v[j];
      }
    }
  }
}

// one thread = one pixel x one 32-channel group of the 7x7 patch matrix (4 groups: 98 channels + 30 zeros);
// group 0 also writes the flow channels of the GRU inputs.
__global__ __launch_bounds__(256) void flow_prep_kernel(const float* __restrict__ coords, int B, int H, int W,
                                                        uint8_t* pm, uint8_t* d0, long long d0ps, uint8_t* d1,
                                                        long long d1ps) {
  constexpr int KS = 7, R = 3, G = 4;
  const int HW = H * W;
  const int P = B * HW;  // 32-bit indexing: the host checks P * G < 2^31
  const int item = blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= P * G) return;
  const int g = item % G;
  const long long p = item / G;
  const int b = static_cast<int>(p) / HW;
  const int pix = static_cast<int>(p) - b * HW;
  const int y = pix / W, x = pix - y * W;
  const float* cx = coords + (long long)b * 2 * HW;
  const float* cy = cx + HW;
  float v[32];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int t = g * 16 + k;
    float fx = 0.f, fy = 0.f;
    if (t < KS * KS) {
      const int yy = y + t / KS - R, xx = x + t % KS - R;
      if (static_cast<unsigned>(yy) < static_cast<unsigned>(H) && static_cast<unsigned>(xx) < static_cast<unsigned>(W)) {
        const long long q = (long long)yy * W + xx;
        fx = cx[q] - static_cast<float>(xx);
        fy = cy[q] - static_cast<float>(yy);
      }
    }
    v[2 * k] = fx;
    v[2 * k + 1] = fy;
  }
  uint8_t* line = pm + (p * G + g) * 128;
#pragma unroll
  for (int c = 0; c < 4; ++c) put8(line + c * 16, v + 8 * c);
  if (g == 0 && d0) {
    const float fx = cx[pix] - static_cast<float>(x), fy = cy[pix] - static_cast<float>(y);
    _Float16 hx, lx, hy, ly;
    range_guard(fmaxf(fabsf(fx), fabsf(fy)));
    split_f16(fx, hx, lx);
    split_f16(fy, hy, ly);
    for (int d = 0; d < 2; ++d) {
      uint8_t* dst = d == 0 ? d0 + p * d0ps : (d1 ? d1 + p * d1ps : nullptr);
      if (!dst) continue;
      _Float16* h = reinterpret_cast<_Float16*>(dst);
      h[0] = hx;
      h[1] = hy;
      h[32] = lx;
      h[33] = ly;
    }
  }
}

// The same outputs from a 4 x 32-pixel tile per workgroup: the tile's flow window (10 x 38 pixels, flow = coords1 -
// coords0 with zeros outside the image, the same fp32 subtraction as above) staged once in LDS, then each thread
// builds one pixel's patch groups from it (lanes = consecutive pixels: conflict-free float2 reads). The per-thread
// form above read its 49 taps' coordinates from global memory one dword at a time (2 x 16 loads per item): 24 us per
// 4-pair launch in the step for 14 MB of output.
constexpr int kFpTH = 4, kFpTW = 32, kFpWH = kFpTH + 6, kFpWW = kFpTW + 6;
__global__ __launch_bounds__(256) void flow_prep_tiled_kernel(const float* __restrict__ coords, int B, int H, int W,
                                                              int tiles_x, int tiles_y, uint8_t* pm, uint8_t* d0,
                                                              long long d0ps, uint8_t* d1, long long d1ps) {
  constexpr int KS = 7, R = 3, G = 4;
  __shared__ float2 sF[kFpWH * kFpWW];
  int t = blockIdx.x;
  const int tx0 = (t % tiles_x) * kFpTW;
  t /= tiles_x;
  const int ty0 = (t % tiles_y) * kFpTH;
  const int b = t / tiles_y;
  const int HW = H * W;
  const float* cx = coords + (long long)b * 2 * HW;
  const float* cy = cx + HW;
  for (int e = threadIdx.x; e < kFpWH * kFpWW; e += blockDim.x) {
    const int wy = e / kFpWW, wx = e - wy * kFpWW;
    const int yy = ty0 - R + wy, xx = tx0 - R + wx;
    float2 f = make_float2(0.f, 0.f);
    if (static_cast<unsigned>(yy) < static_cast<unsigned>(H) && static_cast<unsigned>(xx) < static_cast<unsigned>(W)) {
      const int q = yy * W + xx;
      f = make_float2(cx[q] - static_cast<float>(xx), cy[q] - static_cast<float>(yy));
    }
    sF[e] = f;
  }
  __syncthreads();
  // r05: the tile's output (128 pixels x 4 groups = 512 lines of 128 B, pixel-major, contiguous within a tile row) as
  // 16-B chunks with consecutive lanes on consecutive chunks: a wave store instruction writes 8 whole lines (1 KB
  // contiguous) instead of 64 scattered 16-B pieces of 64 lines. Chunk c of line (pixel, group g): c < 4 the hi halves
  // of the group's values 8c .. 8c+7 (taps 16g + 4c .. +3, x and y), c >= 4 the lo halves of values 8(c-4) ..
  float gm = 0.f;
#pragma unroll 4
  for (int i = 0; i < (pm ? (kFpTH * kFpTW * G * 8) / 256 : 0); ++i) {
    const int k = threadIdx.x + 256 * i, line = k >> 3, c = k & 7;
    const int pl = line >> 2, g = line & 3, py = pl / kFpTW, px = pl - py * kFpTW;
    const int y = ty0 + py, x = tx0 + px;
    if (y >= H || x >= W) continue;
    float v[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int tt = g * 16 + (c & 3) * 4 + e;
      float2 f = make_float2(0.f, 0.f);
      if (tt < KS * KS) f = sF[(py + tt / KS) * kFpWW + px + tt % KS];
      v[2 * e] = f.x;
      v[2 * e + 1] = f.y;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) gm = fmaxf(gm, fabsf(v[j]));
    half8 hi, lo;
    split_vec(v, hi, lo);
    const long long p = (long long)b * HW + (long long)y * W + x;
    *reinterpret_cast<half8*>(pm + (p * G + g) * 128 + (c & 3) * 16 + (c >> 2) * 64) = (c >> 2) ? lo : hi;
  }
  range_guard(gm);  // (the centre tap is among the patch values: the flow channels below are covered)
  const int pl = threadIdx.x & (kFpTH * kFpTW - 1), py = pl / kFpTW, px = pl - py * kFpTW;
  if (!pm && threadIdx.x < 128) {  // no patch matrix: guard the flow channels themselves
    const float2 f = sF[(py + 3) * kFpWW + px + 3];
    if (ty0 + py < H && tx0 + px < W) range_guard(fmaxf(fabsf(f.x), fabsf(f.y)));
  }
  const int y = ty0 + py, x = tx0 + px;
  if (y >= H || x >= W) return;
  const long long p = (long long)b * HW + (long long)y * W + x;
  if (threadIdx.x < 128 && d0) {
    const float2 f = sF[(py + R) * kFpWW + px + R];
    _Float16 hx, lx, hy, ly;
    split_f16(f.x, hx, lx);
    split_f16(f.y, hy, ly);
    for (int d = 0; d < 2; ++d) {
      uint8_t* dst = d == 0 ? d0 + p * d0ps : (d1 ? d1 + p * d1ps : nullptr);
      if (!dst) continue;
      _Float16* h = reinterpret_cast<_Float16*>(dst);
      h[0] = hx;
      h[1] = hy;
      h[32] = lx;
      h[33] = ly;
    }
  }
}

// RAFT.forward's input scaling `2 * (image / 255.0) - 1.0` (methods/raft/model/raft.py:104-105) for both frames in
// one pass (ATen runs it as three elementwise kernels per frame, on the step's critical path ahead of the encoders).
// The reference's operations in its order -- a correctly rounded fp32 division, an exact doubling, a rounded
// subtraction -- so the result is bit-identical to the reference on the CPU; ATen on the GPU divides by a scalar as a
// multiplication by fl(1/255), which differs from the true quotient in 1 ulp for ~74 % of the values
// (profiles/r04/s36_div.log).
__global__ __launch_bounds__(256) void normalize_images_kernel(const float4* __restrict__ x0, const float4* __restrict__ x1,
                                                               float4* __restrict__ y0, float4* __restrict__ y1,
                                                               long long n4) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < 2 * n4; i += stride) {
    const bool second = i >= n4;
    const long long j = second ? i - n4 : i;
    const float4 v = second ? x1[j] : x0[j];
    float4 r;
    r.x = 2.0f * (v.x / 255.0f) - 1.0f;
    r.y = 2.0f * (v.y / 255.0f) - 1.0f;
    r.z = 2.0f * (v.z / 255.0f) - 1.0f;
    r.w = 2.0f * (v.w / 255.0f) - 1.0f;
    (second ? y1 : y0)[j] = r;
  }
}

// any size / alignment: one element per thread-iteration
__global__ __launch_bounds__(256) void normalize_images_scalar_kernel(const float* __restrict__ x0, const float* __restrict__ x1,
                                                                      float* __restrict__ y0, float* __restrict__ y1,
                                                                      long long n) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < 2 * n; i += stride) {
    const bool second = i >= n;
    const long long j = second ? i - n : i;
    (second ? y1 : y0)[j] = 2.0f * ((second ? x1 : x0)[j] / 255.0f) - 1.0f;
  }
}

// InputPadder.pad (methods/raft/model/utils.py:38-61, F.pad mode="replicate") of up to 4 same-shape tensors in one
// launch: out[t][n][y][x] = in[t][n][clamp(y - top)][clamp(x - left)] -- a copy, bit-exact. One thread = 4 output
// columns of one row (a 16-B store when the row pitch allows it).
struct PadArgs {
  const float* src[4];
  float* dst[4];
};
__global__ __launch_bounds__(256) void replicate_pad_kernel(PadArgs a, int count, long long planes, int H, int W, int Ho,
                                                            int Wo, int top, int left) {
  const int qw = (Wo + 3) / 4;
  const long long per = planes * Ho * qw;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < per * count; i += stride) {
    const int t = static_cast<int>(i / per);
    long long r = i - t * per;
    const int xq = static_cast<int>(r % qw);
    r /= qw;
    const int yo = static_cast<int>(r % Ho);
    const long long n = r / Ho;
    const int ys = min(max(yo - top, 0), H - 1);
    const float* srow = a.src[t] + (n * H + ys) * W;
    float* drow = a.dst[t] + (n * Ho + yo) * Wo;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = srow[min(max(4 * xq + e - left, 0), W - 1)];
    if ((Wo & 3) == 0 && (((uintptr_t)drow) & 15) == 0) {
      *reinterpret_cast<float4*>(drow + 4 * xq) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (4 * xq + e < Wo) drow[4 * xq + e] = v[e];
    }
  }
}

// Flow head output conv (update.py:35-36, `self.conv2`: 3x3, 256 -> 2, + coords1 in place, raft.py:133) for small
// grids. Two output channels fill a matrix-core tile 1/16 (oflow_conv_s32 pads them to N = 32) and that conv's
// LDS-staged K loop is latency-bound when the grid is one image (24.8 us at 55x128), so here the conv runs as fp32
// FMAs with one memory round trip: a workgroup covers 32 pixels x 32 chunks of 8 channels, lane l of wave w taking
// pixel l & 31 and chunk 2w + (l >> 5), and issues all 18 of its loads (the chunk's hi and lo 16-B slots of the 9
// neighbours) plus its share of the weights at once. x = hi + lo exactly and the conv is linear, so hi and lo meet
// the same fp32 weight (staged tap-major in LDS), packed two outputs per FMA. The 32 partial sums per pixel meet in
// LDS in a fixed order. Every pixel reads its neighbours' lines 9 times (through L1/L2), which is why large grids stay
// on oflow_conv_s32 (13 us vs 25 us at 55x128, but no faster at 4 x 55x128).
// r05: the same conv (3x3, C -> 2, + coords1) for large grids as an LDS-tiled fp32-FMA kernel: a workgroup covers a
// 4 x 32 output tile and stages, per 32-channel group, its 6 x 34 halo as fp32 (hi + lo, exact) in LDS (144-B pixel
// stride: the 32 lanes of an output row read 16-B slots 144 B apart, conflict-free); 512 threads = 128 output pixels x
// 4 channel quarters (8 channels of every group, two independent FMA chains per output), the weights from a
// host-repacked [group][4-channel chunk][tap][output][4] copy through scalar loads, the next pass's halos prefetched
// into registers behind the FMAs; the quarters meet in LDS in a fixed order. Each input pixel is read once per tile
// (1.6x with the halo) instead of 9 times through L1/L2 (flow_head2_kernel).
constexpr int kF2TH = 4, kF2TW = 32, kF2HR = kF2TH + 2, kF2HC = kF2TW + 2, kF2HP = kF2HR * kF2HC, kF2PS = 9;
constexpr int kF2NT = 512;  // threads: 128 output pixels x 4 channel quarters (8 channels of each group)
// groups staged per pass (two halo buffers, 58.8 KB): half the barriers, and each prefetch has two groups' FMAs to
// hide behind; same FMA order per chain as one group per pass (bit-identical)
constexpr int kF2GP = 2;
__global__ __launch_bounds__(kF2NT) void flow_head2_tiled_kernel(const uint8_t* __restrict__ x, long long xps, int G, int H,
                                                                 int W, int tiles_x, int tiles_y, const float* __restrict__ wr,
                                                                 const float* __restrict__ bias, float* __restrict__ coords) {
  typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
  typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
  __shared__ float4 sX[kF2GP][kF2HP * kF2PS];
  __shared__ float2 sPart[3][kF2TH * kF2TW];
  int t = blockIdx.x;
  const int tx0 = (t % tiles_x) * kF2TW;
  t /= tiles_x;
  const int ty0 = (t % tiles_y) * kF2TH;
  const int b = t / tiles_y;
  const int tid = threadIdx.x, pl = tid & 127, qq = __builtin_amdgcn_readfirstlane(tid >> 7);
  const int py = pl >> 5, px = pl & 31;
  constexpr int NIT = (kF2HP * 4 + kF2NT - 1) / kF2NT;  // staging items (halo pixel, 8-channel chunk) per thread
  u32x4_t rh[kF2GP][NIT], rl[kF2GP][NIT];
  unsigned inm = 0u;  // staging items inside the image (the others load a clamped pixel and stage zeros: padding 1)
#pragma unroll
  for (int s_ = 0; s_ < NIT; ++s_) {
    const int hp = min(tid + kF2NT * s_, kF2HP * 4 - 1) >> 2;
    const int hy = ty0 - 1 + hp / kF2HC, hx = tx0 - 1 + hp % kF2HC;
    const bool in = static_cast<unsigned>(hy) < static_cast<unsigned>(H) && static_cast<unsigned>(hx) < static_cast<unsigned>(W);
    inm |= (in ? 1u : 0u) << s_;
  }
  auto load = [&](int g, int k) {
#pragma unroll
    for (int s_ = 0; s_ < NIT; ++s_) {
      const int item = min(tid + kF2NT * s_, kF2HP * 4 - 1), hp = item >> 2, q = item & 3;
      const int hy = ty0 - 1 + hp / kF2HC, hx = tx0 - 1 + hp % kF2HC;
      const int cy = min(max(hy, 0), H - 1), cx = min(max(hx, 0), W - 1);
      const uint8_t* line = x + ((long long)(b * H + cy) * W + cx) * xps + g * 128 + q * 16;
      rh[k][s_] = *reinterpret_cast<const u32x4_t*>(line);
      rl[k][s_] = *reinterpret_cast<const u32x4_t*>(line + 64);
    }
  };
  float acc[2][2] = {{0.f, 0.f}, {0.f, 0.f}};  // [channel chunk of the quarter][output]: independent FMA chains
#pragma unroll
  for (int k = 0; k < kF2GP; ++k)
    if (k < G) load(k, k);
  for (int g0 = 0; g0 < G; g0 += kF2GP) {
    __syncthreads();  // every thread is done reading the previous pass's halos
#pragma unroll
    for (int k = 0; k < kF2GP; ++k) {
      if (g0 + k >= G) break;
#pragma unroll
      for (int s_ = 0; s_ < NIT; ++s_) {
        const int item = tid + kF2NT * s_;
        if (item < kF2HP * 4) {
          const int hp = item >> 2, q = item & 3;
          const half8_t hv = __builtin_bit_cast(half8_t, rh[k][s_]), lv = __builtin_bit_cast(half8_t, rl[k][s_]);
          const bool in = (inm >> s_) & 1u;
          float f[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = in ? static_cast<float>(hv[j]) + static_cast<float>(lv[j]) : 0.f;
          sX[k][hp * kF2PS + 2 * q] = make_float4(f[0], f[1], f[2], f[3]);
          sX[k][hp * kF2PS + 2 * q + 1] = make_float4(f[4], f[5], f[6], f[7]);
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kF2GP; ++k)
      if (g0 + kF2GP + k < G) load(g0 + kF2GP + k, k);
#pragma unroll
    for (int k = 0; k < kF2GP; ++k) {
      const int g = g0 + k;
      if (g >= G) break;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int ky = tap / 3, kx = tap - ky * 3;
#pragma unroll
        for (int cl = 0; cl < 2; ++cl) {
          const int c4 = qq * 2 + cl;
          const float4 v = sX[k][((py + ky) * kF2HC + px + kx) * kF2PS + c4];
          const float4* wq = reinterpret_cast<const float4*>(wr) + ((g * 8 + c4) * 9 + tap) * 2;
          const float4 w0 = wq[0], w1 = wq[1];
          float a0 = acc[cl][0], a1 = acc[cl][1];
          a0 = fmaf(v.x, w0.x, a0);
          a0 = fmaf(v.y, w0.y, a0);
          a0 = fmaf(v.z, w0.z, a0);
          a0 = fmaf(v.w, w0.w, a0);
          a1 = fmaf(v.x, w1.x, a1);
          a1 = fmaf(v.y, w1.y, a1);
          a1 = fmaf(v.z, w1.z, a1);
          a1 = fmaf(v.w, w1.w, a1);
          acc[cl][0] = a0;
          acc[cl][1] = a1;
        }
      }
    }
  }
  const float s0 = acc[0][0] + acc[1][0], s1 = acc[0][1] + acc[1][1];
  if (qq) sPart[qq - 1][pl] = make_float2(s0, s1);
  __syncthreads();
  if (!qq) {
    const float2 o1 = sPart[0][pl], o2 = sPart[1][pl], o3 = sPart[2][pl];
    const int y = ty0 + py, xx = tx0 + px;
    if (y < H && xx < W) {
      float* cb = coords + (long long)b * 2 * H * W + (long long)y * W + xx;
      // the quarters in a fixed order; delta_flow = conv2(.) incl. its bias; coords1 += delta_flow (raft.py:133)
      cb[0] += (((s0 + o1.x) + o2.x) + o3.x) + bias[0];
      cb[(long long)H * W] += (((s1 + o1.y) + o2.y) + o3.y) + bias[1];
    }
  }
}

constexpr int kFhPx = 32;
__global__ __launch_bounds__(1024) void flow_head2_kernel(const uint8_t* __restrict__ x, long long xps, int G, int B, int H,
                                                          int W, const float* __restrict__ w, const float* __restrict__ bias,
                                                          float* __restrict__ coords) {
  typedef _Float16 half8 __attribute__((ext_vector_type(8)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  __shared__ float2 sw[9 * 256];     // [tap][channel] (w_out0, w_out1)
  __shared__ float2 red[32][kFhPx];  // [chunk][pixel]
  const int tid = threadIdx.x, lane = tid & 63;
  const int C = G * 32;
  const int HW = H * W, P = B * HW;  // < 2^31: checked at the entry
  const int px = lane & (kFhPx - 1);
  const int k = (tid >> 6) * 2 + (lane >> 5);  // chunk: channels 8k .. 8k+7, group k / 4, slot k % 4
  const int p = blockIdx.x * kFhPx + px;
  const int pc = p < P ? p : P - 1;
  const int b = pc / HW;
  const int pix = pc - b * HW;
  const int y = pix / W, xx = pix - y * W;
  float v[5];  // this thread's weights, loaded before the neighbours and stored to LDS after them
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int i = tid + j * 1024;
    v[j] = w[i < 2 * C * 9 ? i : 0];
  }
  half8 hv[9], lv[9];
  if (k < G * 4) {
    const uint8_t* base = x + (long long)b * HW * xps + (k >> 2) * 128 + (k & 3) * 16;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ny = y + t / 3 - 1, nx = xx + t % 3 - 1;  // zero padding: load the clamped neighbour, then zero it
      const bool ok = static_cast<unsigned>(ny) < static_cast<unsigned>(H) && static_cast<unsigned>(nx) < static_cast<unsigned>(W);
      const uint8_t* line = base + ((long long)min(max(ny, 0), H - 1) * W + min(max(nx, 0), W - 1)) * xps;
      hv[t] = *reinterpret_cast<const half8*>(line);
      lv[t] = *reinterpret_cast<const half8*>(line + 64);
      if (!ok) {
        hv[t] = half8{};
        lv[t] = half8{};
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 5; ++j) {  // (o, c, t) as nn.Conv2d stores the weight -> [t][c].o
    const int i = tid + j * 1024;
    if (i >= 2 * C * 9) break;
    const int o = i >= C * 9, r = i - o * C * 9, c = r / 9, t = r - c * 9;
    reinterpret_cast<float*>(sw)[(t * C + c) * 2 + o] = v[j];
  }
  __syncthreads();
  f2 ah = {0.f, 0.f}, al = {0.f, 0.f};  // (out0, out1) over the hi and the lo halves
  if (k < G * 4) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float2 u = sw[t * C + k * 8 + e];
        const f2 uw = {u.x, u.y};
        const float h = static_cast<float>(hv[t][e]), l = static_cast<float>(lv[t][e]);
        ah = __builtin_elementwise_fma(f2{h, h}, uw, ah);
        al = __builtin_elementwise_fma(f2{l, l}, uw, al);
      }
  }
  red[k][px] = make_float2(ah.x + al.x, ah.y + al.y);
  __syncthreads();
  if (tid < 2 * kFhPx) {
    const int q = tid & (kFhPx - 1), o = tid >> 5;
    const int pq = blockIdx.x * kFhPx + q;
    if (pq < P) {
      const float* rf = reinterpret_cast<const float*>(&red[0][q]) + o;
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 32; ++j) s += rf[j * kFhPx * 2];
      const int bq = pq / HW;
      coords[(long long)bq * 2 * HW + (long long)o * HW + (pq - bq * HW)] += s + bias[o];
    }
  }
}

// coords (B, 2, H, W) += bias + sum over the 9 taps of the 3x3 conv's per-tap products y (B, 18, H, W) gathered at the
// tap's neighbour (zero padding): the second half of the flow head's output conv (update.py:35-36 conv2, 3x3 C -> 2)
// computed as a 1x1 conv C -> 18 (channel (ky*3+kx)*2 + c = the tap's contribution, evaluated at the INPUT pixel) and
// this col2im. One thread per output pixel; the plane reads are coalesced along x.
__global__ __launch_bounds__(256) void flow_head_col2im_kernel(const float* __restrict__ y, int B, int H, int W,
                                                               const float* __restrict__ bias, float* __restrict__ coords) {
  const int HW = H * W;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * HW) return;
  const int b = t / HW, p = t - b * HW, py = p / W, px = p - py * W;
  const float* yb = y + (size_t)b * 18 * HW;
  float s[2] = {0.f, 0.f};
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int yy = py + ky - 1;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int xx = px + kx - 1;
      const bool in = static_cast<unsigned>(yy) < static_cast<unsigned>(H) && static_cast<unsigned>(xx) < static_cast<unsigned>(W);
      const int q = in ? yy * W + xx : p;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float v = yb[(size_t)((ky * 3 + kx) * 2 + c) * HW + q];
        s[c] += in ? v : 0.f;
      }
    }
  }
  float* cb = coords + (size_t)b * 2 * HW + p;
  cb[0] += s[0] + bias[0];  // delta_flow = conv2(.) incl. its bias; coords1 = coords1 + delta_flow (raft.py:133)
  cb[HW] += s[1] + bias[1];
}

}  // namespace
OFLOW_RANGE_FLAG_SETTER(s32io)
}  // namespace oflow

using namespace oflow;

extern "C" int oflow_pack_s32_f32(const float* d_x, long long x_batch_stride, int C, int B, int H, int W, int activation,
                                  int dst_channel, void* d_y0, long long y0_pixel_stride, void* d_y1,
                                  long long y1_pixel_stride, float* d_nhwc, int nhwc_pixel_stride, void* stream) {
  if (!d_x || !d_y0) return OFLOW_E_NULL;
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || dst_channel < 0 || (dst_channel & 7)) return OFLOW_E_SHAPE;
  if (activation < 0 || activation > 3) return OFLOW_E_MODE;
  if ((y0_pixel_stride & 127) || ((uintptr_t)d_y0 & 15) || (d_y1 && ((y1_pixel_stride & 127) || ((uintptr_t)d_y1 & 15))))
    return OFLOW_E_ALIGN;
  const long long items = (long long)B * H * W * ((C + 31) / 32);
  if ((items + 255) / 256 * 256 >= (1ll << 31)) return OFLOW_E_SHAPE;  // 32-bit indexing over the rounded-up grid
  hipLaunchKernelGGL(pack_s32_kernel, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     d_x, x_batch_stride, C, B, H * W, activation, dst_channel, static_cast<uint8_t*>(d_y0), y0_pixel_stride,
                     static_cast<uint8_t*>(d_y1), y1_pixel_stride, d_nhwc, nhwc_pixel_stride);
  return launch_status();
}

extern "C" int oflow_normalize_images_f32(const float* d_x0, const float* d_x1, long long n, float* d_y0, float* d_y1,
                                          void* stream) {
  if (!d_x0 || !d_x1 || !d_y0 || !d_y1) return OFLOW_E_NULL;
  if (n <= 0) return OFLOW_E_SHAPE;
  if (((uintptr_t)d_x0 | (uintptr_t)d_x1 | (uintptr_t)d_y0 | (uintptr_t)d_y1) & 3) return OFLOW_E_ALIGN;
  if ((n & 3) || (((uintptr_t)d_x0 | (uintptr_t)d_x1 | (uintptr_t)d_y0 | (uintptr_t)d_y1) & 15)) {
    const long long blocks = (2 * n + 255) / 256;
    hipLaunchKernelGGL(normalize_images_scalar_kernel, dim3((unsigned)(blocks < 16384 ? blocks : 16384)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), d_x0, d_x1, d_y0, d_y1, n);
    return launch_status();
  }
  const long long n4 = n / 4;
  const long long blocks = (2 * n4 + 255) / 256;
  hipLaunchKernelGGL(normalize_images_kernel, dim3((unsigned)(blocks < 16384 ? blocks : 16384)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), reinterpret_cast<const float4*>(d_x0),
                     reinterpret_cast<const float4*>(d_x1), reinterpret_cast<float4*>(d_y0), reinterpret_cast<float4*>(d_y1),
                     n4);
  return launch_status();
}

extern "C" int oflow_replicate_pad_f32(const float* const* d_src, float* const* d_dst, int count, long long planes, int H,
                                       int W, int top, int bottom, int left, int right, void* stream) {
  if (!d_src || !d_dst) return OFLOW_E_NULL;
  if (count < 1 || count > 4 || planes <= 0 || H <= 0 || W <= 0 || top < 0 || bottom < 0 || left < 0 || right < 0)
    return OFLOW_E_SHAPE;
  PadArgs a{};
  for (int t = 0; t < count; ++t) {
    if (!d_src[t] || !d_dst[t]) return OFLOW_E_NULL;
    a.src[t] = d_src[t];
    a.dst[t] = d_dst[t];
  }
  const int Ho = H + top + bottom, Wo = W + left + right;
  const long long items = planes * Ho * ((Wo + 3) / 4) * count;
  const long long blocks = (items + 255) / 256;
  hipLaunchKernelGGL(replicate_pad_kernel, dim3((unsigned)(blocks < 16384 ? blocks : 16384)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), a, count, planes, H, W, Ho, Wo, top, left);
  return launch_status();
}

namespace oflow {
int g_flow_prep_untiled = 0;  // experiments only: the per-thread form (oflow_exp_set_flow_prep_untiled)
}
extern "C" void oflow_exp_set_flow_prep_untiled(int on) { oflow::g_flow_prep_untiled = on; }

extern "C" int oflow_flow_prep_s32(const float* d_coords, int B, int H, int W, void* d_patches, void* d_flow0,
                                   long long flow0_pixel_stride, void* d_flow1, long long flow1_pixel_stride,
                                   void* stream) {
  // d_patches may be null (only the flow channels: convf1 then reads coords1 itself, OFLOW_IN_FLOW7)
  if (!d_coords || (!d_patches && !d_flow0) || (!d_patches && g_flow_prep_untiled)) return OFLOW_E_NULL;
  if (B <= 0 || H <= 0 || W <= 0) return OFLOW_E_SHAPE;
  if (((uintptr_t)d_patches & 15) || (d_flow0 && ((uintptr_t)d_flow0 & 3)) || (d_flow1 && ((uintptr_t)d_flow1 & 3)))
    return OFLOW_E_ALIGN;
  if ((long long)H * W >= (1ll << 31) / 2) return OFLOW_E_SHAPE;  // 32-bit pixel index within an image
  if (!g_flow_prep_untiled) {
    const int tiles_x = (W + kFpTW - 1) / kFpTW, tiles_y = (H + kFpTH - 1) / kFpTH;
    const long long blocks = (long long)tiles_x * tiles_y * B;
    if (blocks >= (1ll << 31)) return OFLOW_E_SHAPE;
    hipLaunchKernelGGL(flow_prep_tiled_kernel, dim3((unsigned)blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                       d_coords, B, H, W, tiles_x, tiles_y, static_cast<uint8_t*>(d_patches), static_cast<uint8_t*>(d_flow0),
                       flow0_pixel_stride, static_cast<uint8_t*>(d_flow1), flow1_pixel_stride);
    return launch_status();
  }
  const long long items = (long long)B * H * W * 4;
  if ((items + 255) / 256 * 256 >= (1ll << 31)) return OFLOW_E_SHAPE;  // 32-bit indexing over the rounded-up grid
  hipLaunchKernelGGL(flow_prep_kernel, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     d_coords, B, H, W, static_cast<uint8_t*>(d_patches), static_cast<uint8_t*>(d_flow0),
                     flow0_pixel_stride, static_cast<uint8_t*>(d_flow1), flow1_pixel_stride);
  return launch_status();
}

extern "C" int oflow_flow_head_col2im_f32(const float* d_y, const float* d_bias, int B, int H, int W, float* d_coords,
                                          void* stream) {
  if (!d_y || !d_bias || !d_coords) return OFLOW_E_NULL;
  if (B <= 0 || H <= 0 || W <= 0 || (long long)B * H * W * 18 >= (1LL << 31)) return OFLOW_E_SHAPE;
  const int P = B * H * W;
  hipLaunchKernelGGL(flow_head_col2im_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     d_y, B, H, W, d_bias, d_coords);
  return launch_status();
}

extern "C" int oflow_flow_head2_tiled_s32(const void* d_x, long long x_pixel_stride, int in_groups, const float* d_wr,
                                          const float* d_bias, int B, int H, int W, float* d_coords, void* stream) {
  if (!d_x || !d_wr || !d_bias || !d_coords) return OFLOW_E_NULL;
  if (B <= 0 || H <= 0 || W <= 0 || in_groups <= 0 || in_groups > 8 || (long long)B * H * W >= (1LL << 31))
    return OFLOW_E_SHAPE;
  if ((x_pixel_stride & 127) || ((uintptr_t)d_x & 15) || ((uintptr_t)d_wr & 15) || x_pixel_stride < 128LL * in_groups)
    return OFLOW_E_ALIGN;
  const int tiles_x = (W + kF2TW - 1) / kF2TW, tiles_y = (H + kF2TH - 1) / kF2TH;
  const long long blocks = (long long)tiles_x * tiles_y * B;
  if (blocks >= (1ll << 31)) return OFLOW_E_SHAPE;
  hipLaunchKernelGGL(flow_head2_tiled_kernel, dim3((unsigned)blocks), dim3(kF2NT), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint8_t*>(d_x), x_pixel_stride, in_groups, H, W, tiles_x, tiles_y, d_wr, d_bias,
                     d_coords);
  return launch_status();
}

extern "C" int oflow_flow_head2_s32(const void* d_x, long long x_pixel_stride, int in_groups, const float* d_weight,
                                    const float* d_bias, int B, int H, int W, float* d_coords, void* stream) {
  if (!d_x || !d_weight || !d_bias || !d_coords) return OFLOW_E_NULL;
  if (B <= 0 || H <= 0 || W <= 0 || in_groups <= 0 || in_groups > 8 || (long long)B * H * W >= (1LL << 31))
    return OFLOW_E_SHAPE;
  if ((x_pixel_stride & 127) || ((uintptr_t)d_x & 15) || x_pixel_stride < 128LL * in_groups) return OFLOW_E_ALIGN;
  const long long P = (long long)B * H * W;
  hipLaunchKernelGGL(flow_head2_kernel, dim3((unsigned)((P + kFhPx - 1) / kFhPx)), dim3(1024), 0,
                     static_cast<hipStream_t>(stream), static_cast<const uint8_t*>(d_x), x_pixel_stride, in_groups, B, H, W,
                     d_weight, d_bias, d_coords);
  return launch_status();
}
