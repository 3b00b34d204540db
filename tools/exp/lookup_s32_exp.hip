// EXPERIMENT (not product code): S32 lookup organised query-major -- one workgroup = 16 queries x all levels, so each
// query's 11 output lines are written whole by one workgroup -- against the product's level-per-workgroup kernel.
#include "../../torch-optical-flow_amd/csrc/corr_lookup.hip"

namespace oflow {
namespace {

template <int R, int L, bool NT>
__global__ __launch_bounds__(256) void lookup_s32_qmajor(LookupArgs a) {
  constexpr int QB = 64 / L;      // queries per workgroup
  constexpr int PK = 2 * R + 2, K = 2 * R + 1, PS = PK * PK, QS = PS + 1;
  constexpr int ITEMS = 64 * PS, PER = (ITEMS + 255) / 256;
  constexpr int KK = K * K, LS = (KK + 7) / 8 * 8, NCH = L * LS / 8;
  __shared__ float sP[64 * QS];
  __shared__ int sX[64], sY[64];
  __shared__ float4 sW[64];
  __shared__ const float* sL[64];
  __shared__ int sHl[64], sWl[64], sHB[64], sWB[64];
  const int q0 = blockIdx.x * QB;
  if (threadIdx.x < 64) {
    const int pr = threadIdx.x, lvl = pr / QB, q = q0 + pr % QB;
    int xs = -(1 << 28), ys = -(1 << 28);
    float4 w = make_float4(0.f, 0.f, 0.f, 0.f);
    if (q < a.total) {
      const int b = q / a.N, pix = q - b * a.N;
      const float inv = 1.0f / static_cast<float>(1 << lvl);
      const float cx = a.coords[(size_t)(2 * b) * a.N + pix] * inv;
      const float cy = a.coords[(size_t)(2 * b + 1) * a.N + pix] * inv;
      if (fabsf(cx) < 4194304.0f && fabsf(cy) < 4194304.0f) {
        const float fx = floorf(cx), fy = floorf(cy);
        const float wx = cx - fx, wy = cy - fy, ex = 1.0f - wx, ey = 1.0f - wy;
        xs = static_cast<int>(fx) - R;
        ys = static_cast<int>(fy) - R;
        w = make_float4(ey * ex, ey * wx, wy * ex, wy * wx);
      }
    }
    sX[pr] = xs;
    sY[pr] = ys;
    sW[pr] = w;
    const float* base = lvl == 0 ? a.lv[0] : lvl == 1 ? a.lv[1] : lvl == 2 ? a.lv[2] : a.lv[3];
    const int hl = lvl == 0 ? a.Hl[0] : lvl == 1 ? a.Hl[1] : lvl == 2 ? a.Hl[2] : a.Hl[3];
    const int wl = lvl == 0 ? a.Wl[0] : lvl == 1 ? a.Wl[1] : lvl == 2 ? a.Wl[2] : a.Wl[3];
    const int hb = (hl + 3) >> 2, wb = (wl + 7) >> 3;
    sL[pr] = base + (size_t)q * hb * wb * 32;
    sHl[pr] = q < a.total ? hl : 0;
    sWl[pr] = wl;
    sHB[pr] = hb;
    sWB[pr] = wb;
  }
  __syncthreads();
  float v[PER];
#pragma unroll
  for (int s = 0; s < PER; ++s) {
    const int item = threadIdx.x + 256 * s;
    v[s] = 0.0f;
    if (item < ITEMS) {
      const int pr = item / PS, rem = item - pr * PS;
      const int row = rem / PK, col = rem - row * PK;
      const int y = sY[pr] + row, x = sX[pr] + col;
      if (static_cast<unsigned>(y) < static_cast<unsigned>(sHl[pr]) && static_cast<unsigned>(x) < static_cast<unsigned>(sWl[pr])) {
        const float* p = sL[pr] + ((y >> 2) * sWB[pr] + (x >> 3)) * 32 + ((y & 3) << 3) + (x & 7);
        v[s] = NT ? __builtin_nontemporal_load(p) : *p;
      }
    }
  }
#pragma unroll
  for (int s = 0; s < PER; ++s) {
    const int item = threadIdx.x + 256 * s;
    if (item < ITEMS) {
      const int pr = item / PS;
      sP[pr * QS + (item - pr * PS)] = v[s];
    }
  }
  __syncthreads();
  typedef _Float16 half8 __attribute__((ext_vector_type(8)));
  for (int item = threadIdx.x; item < QB * NCH; item += 256) {
    const int qi = item / NCH, k = item - qi * NCH;
    if (q0 + qi >= a.total) continue;
    const int c0 = k * 8, lvl = c0 / LS, ch = (c0 - lvl * LS) / 8;
    const int pr = lvl * QB + qi;
    const float4 w = sW[pr];
    half8 hi, lo;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int kk = ch * 8 + e;
      float val = 0.f;
      if (kk < KK) {
        const int i = kk / K, j = kk - i * K;
        const float* p = &sP[pr * QS + j * PK + i];
        val = p[0] * w.x + p[1] * w.y + p[PK] * w.z + p[PK + 1] * w.w;
      }
      const _Float16 h = static_cast<_Float16>(val);
      hi[e] = h;
      lo[e] = static_cast<_Float16>(val - static_cast<float>(h));
    }
    uint8_t* line = a.s32 + (long long)(q0 + qi) * a.s32ps + (c0 >> 5) * 128 + ((c0 & 31) >> 3) * 16;
    *reinterpret_cast<half8*>(line) = hi;
    *reinterpret_cast<half8*>(line + 64) = lo;
  }
}

}  // namespace
}  // namespace oflow

extern "C" int exp_lookup_s32_qmajor(const float* const* d_levels, const int* level_h, const int* level_w, const float* d_coords,
                                     int B, int H, int W, void* d_out, long long ps, int nt, void* stream) {
  LookupArgs a{};
  for (int l = 0; l < 4; ++l) {
    a.lv[l] = d_levels[l];
    a.Hl[l] = level_h[l];
    a.Wl[l] = level_w[l];
    a.HB[l] = (level_h[l] + 3) / 4;
    a.WB[l] = (level_w[l] + 7) / 8;
  }
  a.coords = d_coords;
  a.s32 = static_cast<uint8_t*>(d_out);
  a.s32ps = ps;
  a.N = H * W;
  a.total = B * H * W;
  a.nlev = 4;
  dim3 grid((a.total + 15) / 16);
  if (nt)
    hipLaunchKernelGGL((lookup_s32_qmajor<4, 4, true>), grid, dim3(256), 0, static_cast<hipStream_t>(stream), a);
  else
    hipLaunchKernelGGL((lookup_s32_qmajor<4, 4, false>), grid, dim3(256), 0, static_cast<hipStream_t>(stream), a);
  return launch_status();
}
