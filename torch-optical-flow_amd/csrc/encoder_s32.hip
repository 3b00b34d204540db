// Feature / context encoder stages around the split-fp16 convolution (conv_s32.hip) (gfx950).
//
// Replaces the non-convolution parts of methods/raft/model/extractor.py:35-231 (BasicEncoder, ResidualBlock):
//   oflow_stem_patches_s32   : the 7x7 / stride 2 / pad 3 stem's patch matrix (extractor.py:186) as S32, channel
//                              t*C + c = input channel c at tap t = ky*7 + kx (C = 3: 147 channels, zero padded to 160),
//                              so the stem runs as a 1x1 split-fp16 GEMM.
//   oflow_norm_stats_finalize: instance-norm statistics (nn.InstanceNorm2d, extractor.py:22, biased variance, eps) of a
//                              convolution output from the per-tile (count, mean, M2) partials its epilogue wrote,
//                              merged as fp64 sums, as the affine form the reference applies:
//                              y = x * invstd + (-mean * invstd)  (ATen batch_norm_cpu_transform_input).
//   oflow_norm_apply_s32     : y = act(x * alpha[b,c] + beta[b,c]) [+ residual, act2] -> S32 (optionally space-to-depth),
//                              i.e. relu(norm(conv)) and the block tail relu(x + y) / relu(norm3(down) + y)
//                              (extractor.py:76-90).
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

// One workgroup = 64 consecutive output pixels of one output row: the 7 input rows x (2*64 + 5) input columns x C
// channels they read are staged in LDS once (coalesced row reads, zero padding applied there), then each thread
// assembles (pixel, 32-channel group) lines from LDS; the workgroup's output is one contiguous run of 64 * G lines.
constexpr int kStemPX = 64, kStemMaxC = 4;
template <int C>  // input channels: compile-time, so the channel / tap decode of every patch entry is constant folded
__global__ __launch_bounds__(256) void stem_patches_kernel(const float* __restrict__ img, int B, int H, int W, int Ho,
                                                           int Wo, int G, uint8_t* out) {
  constexpr int KS = 7, PAD = 3, ST = 2, IX = ST * kStemPX + KS - ST;  // 133 input columns
  __shared__ float sImg[C][KS][IX];
  const int xb = blockIdx.x, oy = blockIdx.y, b = blockIdx.z;
  const int ox0 = xb * kStemPX;
  const int iy0 = oy * ST - PAD, ix0 = ox0 * ST - PAD;
  const float* src = img + (long long)b * C * H * W;
  for (int e = threadIdx.x; e < C * KS * IX; e += 256) {
    const int c = e / (KS * IX), rem = e - c * (KS * IX);
    const int ky = rem / IX, xx = rem - ky * IX;
    const int iy = iy0 + ky, ix = ix0 + xx;
    float v = 0.f;
    if (static_cast<unsigned>(iy) < static_cast<unsigned>(H) && static_cast<unsigned>(ix) < static_cast<unsigned>(W))
      v = src[((long long)c * H + iy) * W + ix];
    sImg[c][ky][xx] = v;
  }
  __syncthreads();
  const int npx = min(kStemPX, Wo - ox0);
  uint8_t* dst = out + (((long long)b * Ho + oy) * Wo + ox0) * G * 128;
  // lane = one 16-B piece of a line (8 hi or 8 lo halves): 8 consecutive lanes fill one 128-B line, so every store
  // instruction writes 8 whole consecutive lines
  for (int item = threadIdx.x; item < npx * G * 8; item += 256) {
    const int line = item >> 3, piece = item & 7, q = piece & 3;
    const int px = line / G, g = line - px * G;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = 0.f;
    // the (group, quarter) of a lane is divergent within a wave, the 8 entries it needs are not: one body per pair
#pragma unroll
    for (int gg = 0; gg < (KS * KS * C + 31) / 32; ++gg) {
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        if (g == gg && q == qq) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int k = gg * 32 + qq * 8 + e;
            const int t = k / C, c = k - t * C;
            if (t < KS * KS) v[e] = sImg[c][t / KS][px * ST + t % KS];
          }
        }
      }
    }
    half8 h;
    if (piece < 4) range_guard8(v);  // (the lo pieces split the same values)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      _Float16 h_, l_;
      split_f16(v[e], h_, l_);
      h[e] = piece < 4 ? h_ : l_;
    }
    *reinterpret_cast<half8*>(dst + (long long)line * 128 + (piece < 4 ? q * 16 : 64 + q * 16)) = h;
  }
}

// one workgroup = one image x 64 channels, 1024 threads: lane = channel (coalesced 12-B partials), the 16 waves stride
// over the tiles with 4 partials in flight per lane. Each (count, mean, M2) partial becomes fp64 (n, sum, sum of squares)
// terms -- sum += n*mean, sq += M2 + n*mean^2 -- so the merge is a plain fp64 sum (no dependent divisions); the 16 wave
// sums are added through LDS in a fixed order (deterministic). var = sq/n - mean^2 in fp64 keeps ~1e-12 relative
// accuracy for the conv outputs here (mean^2/var << 1e4), far below the fp32 result's rounding.
constexpr int kStatWaves = 16;
__global__ __launch_bounds__(64 * kStatWaves) void norm_stats_kernel(const float* __restrict__ part, int B, int tiles,
                                                                     int npad, int C, double eps, float* alpha,
                                                                     float* beta) {
  __shared__ double sN[kStatWaves][64], sS[kStatWaves][64], sQ[kStatWaves][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int cblocks = (C + 63) / 64;
  const int b = blockIdx.x / cblocks, c = (blockIdx.x - b * cblocks) * 64 + lane;
  double n = 0.0, s = 0.0, q = 0.0;
  if (c < C) {
    const float* base = part + ((long long)b * tiles * npad + c) * 3;
    const long long tstride = (long long)npad * 3;
    int t = wave;
    for (; t + 3 * kStatWaves < tiles; t += 4 * kStatWaves) {
      float pv[4][3];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float* p = base + (t + u * kStatWaves) * tstride;
        pv[u][0] = p[0];
        pv[u][1] = p[1];
        pv[u][2] = p[2];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const double nb = pv[u][0], mb = pv[u][1];
        n += nb;
        s += nb * mb;
        q += static_cast<double>(pv[u][2]) + nb * mb * mb;
      }
    }
    for (; t < tiles; t += kStatWaves) {
      const float* p = base + t * tstride;
      const double nb = p[0], mb = p[1];
      n += nb;
      s += nb * mb;
      q += static_cast<double>(p[2]) + nb * mb * mb;
    }
  }
  sN[wave][lane] = n;
  sS[wave][lane] = s;
  sQ[wave][lane] = q;
  __syncthreads();
  if (wave == 0 && c < C) {
    for (int w = 1; w < kStatWaves; ++w) {
      n += sN[w][lane];
      s += sS[w][lane];
      q += sQ[w][lane];
    }
    const double mean = n > 0.0 ? s / n : 0.0;
    double var = n > 0.0 ? q / n - mean * mean : 0.0;
    if (var < 0.0) var = 0.0;
    const float invstd = static_cast<float>(1.0 / sqrt(var + eps));
    alpha[(long long)b * C + c] = invstd;
    beta[(long long)b * C + c] = -static_cast<float>(mean) * invstd;
  }
}

// one thread = one pixel x 8 channels; every operand as 16-B loads (the per-channel affines too), 32-bit indexing
// (the host checks P * C / 8 < 2^31)
__global__ __launch_bounds__(256) void norm_apply_kernel(const float* __restrict__ x, int C, int B, int H, int W,
                                                         const float* __restrict__ alpha, const float* __restrict__ beta,
                                                         int act, int res_mode, const uint8_t* res, long long resps,
                                                         const float* __restrict__ x2, const float* __restrict__ alpha2,
                                                         const float* __restrict__ beta2, int res_act, int s2d,
                                                         uint8_t* y, long long yps) {
  const int C8 = C / 8;
  const int HW = H * W, P = B * HW;
  const int item = blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= P * C8) return;
  const int p = item / C8, c8 = item - p * C8;
  const int b = p / HW;
  const int c0 = c8 * 8;
  auto ld8 = [](const float* q, float (&o)[8]) {
    const float4 u0 = reinterpret_cast<const float4*>(q)[0], u1 = reinterpret_cast<const float4*>(q)[1];
    o[0] = u0.x; o[1] = u0.y; o[2] = u0.z; o[3] = u0.w; o[4] = u1.x; o[5] = u1.y; o[6] = u1.z; o[7] = u1.w;
  };
  float v[8], al[8], be[8];
  ld8(x + (long long)p * C + c0, v);
  ld8(alpha + b * C + c0, al);
  ld8(beta + b * C + c0, be);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = act_fn(v[j] * al[j] + be[j], act);
  if (res_mode == 1) {  // S32 residual (identity shortcut)
    const uint8_t* rl = res + p * resps + (long long)(c0 >> 5) * 128 + ((c0 & 31) >> 3) * 16;
    const half8 rh = *reinterpret_cast<const half8*>(rl), rlo = *reinterpret_cast<const half8*>(rl + 64);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = act_fn(v[j] + (static_cast<float>(rh[j]) + static_cast<float>(rlo[j])), res_act);
  } else if (res_mode >= 2) {  // normalised raw residual: 2 = the downsample branch norm3(conv1x1(x)); 3 = a block
                                // input kept raw, relu(norm(x)) (the stem's output feeding layer1's first block)
    float r[8], a2[8], b2[8];
    ld8(x2 + (long long)p * C + c0, r);
    ld8(alpha2 + b * C + c0, a2);
    ld8(beta2 + b * C + c0, b2);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float rn = r[j] * a2[j] + b2[j];
      if (res_mode == 3) rn = act_fn(rn, 1);
      v[j] = act_fn(rn + v[j], res_act);
    }
  }
  long long pd = p;
  int cd = c0;
  if (s2d) {
    const int pix = p - b * HW;
    const int yy = pix / W, xx = pix - yy * W;
    pd = ((long long)b * (H >> 1) + (yy >> 1)) * (W >> 1) + (xx >> 1);
    cd = c0 + ((yy & 1) * 2 + (xx & 1)) * C;
  }
  put8(y + pd * yps + (long long)(cd >> 5) * 128 + ((cd & 31) >> 3) * 16, v);
}

}  // namespace
OFLOW_RANGE_FLAG_SETTER(encoder)
}  // namespace oflow

using namespace oflow;

extern "C" int oflow_stem_patches_s32(const float* d_img, int B, int C, int H, int W, void* d_out, int out_groups,
                                      void* stream) {
  if (!d_img || !d_out) return OFLOW_E_NULL;
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || out_groups * 32 < 49 * C) return OFLOW_E_SHAPE;
  if ((uintptr_t)d_out & 15) return OFLOW_E_ALIGN;
  if (C > kStemMaxC || B > 65535) return OFLOW_E_SHAPE;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;  // (H + 2*3 - 7) / 2 + 1
  if (Ho > 65535) return OFLOW_E_SHAPE;
  const dim3 grid((Wo + kStemPX - 1) / kStemPX, Ho, B);
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint8_t* o = static_cast<uint8_t*>(d_out);
  switch (C) {
    case 1: hipLaunchKernelGGL(stem_patches_kernel<1>, grid, dim3(256), 0, s, d_img, B, H, W, Ho, Wo, out_groups, o); break;
    case 2: hipLaunchKernelGGL(stem_patches_kernel<2>, grid, dim3(256), 0, s, d_img, B, H, W, Ho, Wo, out_groups, o); break;
    case 3: hipLaunchKernelGGL(stem_patches_kernel<3>, grid, dim3(256), 0, s, d_img, B, H, W, Ho, Wo, out_groups, o); break;
    default: hipLaunchKernelGGL(stem_patches_kernel<4>, grid, dim3(256), 0, s, d_img, B, H, W, Ho, Wo, out_groups, o); break;
  }
  return launch_status();
}

extern "C" int oflow_norm_stats_finalize(const float* d_partials, int B, int tiles, int n_pad, int C, double eps,
                                         float* d_alpha, float* d_beta, void* stream) {
  if (!d_partials || !d_alpha || !d_beta) return OFLOW_E_NULL;
  if (B <= 0 || tiles <= 0 || C <= 0 || n_pad < C) return OFLOW_E_SHAPE;
  hipLaunchKernelGGL(norm_stats_kernel, dim3(B * ((C + 63) / 64)), dim3(64 * kStatWaves), 0, static_cast<hipStream_t>(stream),
                     d_partials, B, tiles, n_pad, C, eps, d_alpha, d_beta);
  return launch_status();
}

extern "C" int oflow_norm_apply_s32(const float* d_x, int C, int B, int H, int W, const float* d_alpha,
                                    const float* d_beta, int activation, int res_mode, const void* d_res,
                                    long long res_pixel_stride, const float* d_x2, const float* d_alpha2,
                                    const float* d_beta2, int res_activation, int s2d, void* d_y,
                                    long long y_pixel_stride, void* stream) {
  if (!d_x || !d_alpha || !d_beta || !d_y) return OFLOW_E_NULL;
  if (B <= 0 || C <= 0 || C % 8 || H <= 0 || W <= 0) return OFLOW_E_SHAPE;
  if (activation < 0 || activation > 3 || res_activation < 0 || res_activation > 3 || res_mode < 0 || res_mode > 3)
    return OFLOW_E_MODE;
  if (res_mode == 1 && !d_res) return OFLOW_E_NULL;
  if (res_mode >= 2 && (!d_x2 || !d_alpha2 || !d_beta2)) return OFLOW_E_NULL;
  if (s2d && ((H | W) & 1)) return OFLOW_E_SHAPE;
  if (((uintptr_t)d_x & 15) || ((uintptr_t)d_y & 15) || (y_pixel_stride & 127) ||
      (d_res && (((uintptr_t)d_res & 15) || (res_pixel_stride & 127))) || (d_x2 && ((uintptr_t)d_x2 & 15)) ||
      (((uintptr_t)d_alpha | (uintptr_t)d_beta) & 15) || (((uintptr_t)d_alpha2 | (uintptr_t)d_beta2) & 15))
    return OFLOW_E_ALIGN;
  const long long items = (long long)B * H * W * (C / 8);
  if ((items + 255) / 256 * 256 >= (1ll << 31)) return OFLOW_E_SHAPE;  // 32-bit indexing over the rounded-up grid
  hipLaunchKernelGGL(norm_apply_kernel, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     d_x, C, B, H, W, d_alpha, d_beta, activation, res_mode, static_cast<const uint8_t*>(d_res),
                     res_pixel_stride, d_x2, d_alpha2, d_beta2, res_activation, s2d, static_cast<uint8_t*>(d_y),
                     y_pixel_stride);
  return launch_status();
}
