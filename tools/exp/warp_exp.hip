// EXPERIMENT (not product code): the direct-gather bilinear warp (grid_warp_kernel) against the LDS-staged tile kernel
// the product launches for bilinear (warp_bilinear_lds_kernel), same inputs, in one process.
// Result (profiles/r01/exp/warp_staged_vs_direct.log, (8, 3, 436, 1024) frames, direct -> staged, us): i.i.d.
// N(0, 8^2) px flow 79.2 -> 51.7; sigma 4: 57.1 -> 45.6; sigma 2: 49.6 -> 43.8; smooth +-20 px: 43.8 -> 43.7;
// zero flow 31.4 -> 41.7.
#include "../../torch-optical-flow_amd/csrc/grid_warp.hip"

extern "C" int exp_warp(int which, const float* d_frame, const float* d_flow, int B, int C, int H, int W, float* d_out,
                        void* stream) {
  oflow::WarpArgs a{d_frame, d_flow, d_out, B, C, H, W, H, W, OFLOW_PAD_BORDER, 0};
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (which == 0) {
    const long long want = ((long long)B * H * W + 255) / 256;
    hipLaunchKernelGGL((oflow::grid_warp_kernel<OFLOW_INTERP_BILINEAR, true>), dim3((unsigned)(want < 65535 ? want : 65535)),
                       dim3(256), 0, s, a);
  } else {
    const int tx = (W + oflow::kWTX - 1) / oflow::kWTX, ty = (H + oflow::kWTY - 1) / oflow::kWTY;
    hipLaunchKernelGGL((oflow::warp_bilinear_lds_kernel<true>), dim3(B * tx * ty), dim3(oflow::kWThreads), 0, s, a, tx, ty);
  }
  return hipGetLastError();
}
