// EXPERIMENT (not product code): the product conv_s32 kernel launched as 8-wave workgroups (8-row x 32-column
// pixel tiles, one workgroup per CU) for the BN = 128 layers, vs the product's 4-wave workgroups.
#include "../../torch-optical-flow_amd/csrc/conv_s32.hip"

namespace {
int wg8_launch(const oflow::ConvArgs& a, int kh, int kw, int bn, int epi, hipStream_t s) {
  using namespace oflow;
  const int key = kh * 16 + kw;
  if (bn == 128) {
    if (epi == 1 && key == 0x15) return launch_conv<1, 5, 128, 4, 2, 1, 8>(a, s);
    if (epi == 1 && key == 0x51) return launch_conv<5, 1, 128, 4, 2, 1, 8>(a, s);
    if (epi == 2 && key == 0x15) return launch_conv<1, 5, 128, 4, 2, 2, 8>(a, s);
    if (epi == 2 && key == 0x51) return launch_conv<5, 1, 128, 4, 2, 2, 8>(a, s);
    if (epi == 0 && key == 0x33) return launch_conv<3, 3, 128, 4, 2, 0, 8>(a, s);
    if (epi == 0 && key == 0x11) return launch_conv<1, 1, 128, 4, 2, 0, 8>(a, s);
  }
  return dispatch_conv(a, kh, kw, bn, epi, s);
}
}  // namespace

extern "C" int exp_conv_s32_var(int var, const void* d_x, long long x_pixel_stride, int in_groups, const void* d_wpack,
                                int n_pad, const float* d_wscale, const float* d_bias, int N, int B, int H, int W, int kh,
                                int kw, int block_n, int epilogue, int activation, float out_scale, void* d_y0,
                                long long y0_pixel_stride, void* d_y1, long long y1_pixel_stride, float* d_f32,
                                long long f32_batch_stride, long long f32_channel_stride, int f32_accumulate,
                                float* d_gru_h, float* d_gru_z, int gru_channels, float* d_nhwc, int nhwc_pixel_stride,
                                float* d_stats, const void* d_res, long long res_pixel_stride, int res_activation,
                                int s2d, void* stream) {
  oflow::ConvArgs a;
  const int st = oflow::build_conv_args(a, d_x, x_pixel_stride, in_groups, d_wpack, n_pad, d_wscale, d_bias, N, B, H, W,
                                        kh, kw, block_n, epilogue, activation, out_scale, d_y0, y0_pixel_stride, d_y1,
                                        y1_pixel_stride, d_f32, f32_batch_stride, f32_channel_stride, f32_accumulate,
                                        d_gru_h, d_gru_z, gru_channels, d_nhwc, nhwc_pixel_stride, d_stats, d_res,
                                        res_pixel_stride, res_activation, s2d);
  if (st != OFLOW_OK) return st;
  a.ain = oflow::kInS32;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (var == 8) return wg8_launch(a, kh, kw, block_n, epilogue, s);
  return oflow::dispatch_conv(a, kh, kw, block_n, epilogue, s);
}
