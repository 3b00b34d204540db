// EXPERIMENT (not product code): the product conv_s32 kernel with its VAR schedule hooks, for A/B timing in one process.
#include "conv_s32_r01.hip"

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
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (var) {
    case 0: return oflow::dispatch_conv<0>(a, kh, kw, block_n, epilogue, s);
    case 1040: return oflow::dispatch_conv<1040>(a, kh, kw, block_n, epilogue, s);
    case 1072: return oflow::dispatch_conv<1072>(a, kh, kw, block_n, epilogue, s);
    case 640: return oflow::dispatch_conv<640>(a, kh, kw, block_n, epilogue, s);
    default: return OFLOW_E_MODE;
  }
}
