/*
 * oflow.h — C ABI of liboflow_hip.so, the MI355X (gfx950) implementation of the RAFT inference hot path of
 * awaelchli/torch-optical-flow. Plain pointers and sizes only: no torch or C++ types cross this boundary.
 *
 * All pointers named d_* are DEVICE pointers (HBM), contiguous, fp32 unless stated. Every entry point only
 * ENQUEUES work on `stream` (hipStream_t passed as void*; NULL = the null stream of the current device) and
 * returns without synchronising; it never allocates. Callers set the current device to the one owning the
 * buffers (the Python host layer does this with a torch device guard).
 *
 * Return value: OFLOW_OK (0), a negative OFLOW_E_* argument error (nothing was enqueued), or a positive
 * hipError_t from the launch. oflow_status_string() turns either into text; the Python layer raises
 * RuntimeError/ValueError with it, the exception types the reference's ATen ops raise.
 *
 * Replaces (reference file:line, /root/reference):
 *   oflow_corr_pyramid_f32  <- methods/raft/model/corr.py:38-54 (CorrBlock.__init__) + 79-87 (CorrBlock.corr)
 *   oflow_corr_lookup_f32   <- methods/raft/model/corr.py:56-77 (CorrBlock.__call__)
 *                              + methods/raft/model/utils.py:64-80 (bilinear_sampler)
 *   oflow_grid_warp_f32     <- optical_flow/operator/operator.py:8-56 (warp, warp_grid -> F.grid_sample)
 *   oflow_conv_s32 & co.    <- methods/raft/model/update.py:40-161 (update-block convolutions)
 *   oflow_stem_patches_s32, oflow_norm_*, oflow_conv_s32_ex <- methods/raft/model/extractor.py:35-231 (encoders)
 *   oflow_convex_upsample_f32 <- methods/raft/model/raft.py:73-85 (RAFT.upsample_flow)
 *   oflow_flow_stats_f32, oflow_flow2rgb_f32 <- optical_flow/visualization/flow2rgb.py:19-73 (+ visualization/methods/)
 *   oflow_flow_pack_f32     <- optical_flow/io/middlebury.py:43-71, optical_flow/io/pfm.py:79-104 (file payloads)
 */
#ifndef OFLOW_H_
#define OFLOW_H_

#ifdef __cplusplus
extern "C" {
#endif

#define OFLOW_ABI_VERSION 1

#define OFLOW_OK 0
#define OFLOW_E_NULL (-1)      /* a required pointer is NULL */
#define OFLOW_E_SHAPE (-2)     /* a size is <= 0 or inconsistent */
#define OFLOW_E_LEVELS (-3)    /* num_levels outside [1, OFLOW_MAX_LEVELS] */
#define OFLOW_E_TINY (-4)      /* a pyramid level is < 2 pixels in H or W (reference divides by 0: Q3) */
#define OFLOW_E_RADIUS (-5)    /* radius outside [0, OFLOW_MAX_RADIUS] */
#define OFLOW_E_MODE (-6)      /* unknown interpolation or padding mode */
#define OFLOW_E_ALIGN (-7)     /* a pointer is not 4-byte aligned */

#define OFLOW_MAX_LEVELS 8
#define OFLOW_MAX_RADIUS 7

/* grid_sample modes (torch.nn.functional.grid_sample names) */
#define OFLOW_INTERP_BILINEAR 0
#define OFLOW_INTERP_NEAREST 1
#define OFLOW_INTERP_BICUBIC 2
#define OFLOW_PAD_ZEROS 0
#define OFLOW_PAD_BORDER 1
#define OFLOW_PAD_REFLECTION 2

/* oflow_conv_s32_ex2 input formats */
#define OFLOW_IN_S32 0
#define OFLOW_IN_F32_NORM 1
#define OFLOW_IN_F32 2
#define OFLOW_IN_IMG7S2 3
#define OFLOW_IN_FLOW7 4

int oflow_abi_version(void);
const char* oflow_status_string(int status);

/*
 * Pyramid level sizes for a (H, W) query grid: level 0 = (H, W), level l = floor-halves of level l-1
 * (avg_pool2d(2, stride=2) semantics, corr.py:53). Writes num_levels entries to level_h / level_w (host).
 */
int oflow_corr_pyramid_dims(int H, int W, int num_levels, int* level_h, int* level_w);

/*
 * All-pairs correlation pyramid (CorrBlock.__init__).
 *   d_fmap1, d_fmap2 : (B, C, H, W) fp32
 *   d_levels[l]      : host array of num_levels device pointers; level l is (B*H*W, H_l, W_l) fp32,
 *                      i.e. the reference's corr_pyramid[l] of shape (B*H*W, 1, H_l, W_l).
 *   level 0 = (fmap1^T fmap2) / sqrt(C) on fp32 MFMA (v_mfma_f32_32x32x2f32); levels 1.. are the floor
 *   2x2 average pools of the level above, fused in the GEMM epilogue (level 0 is never re-read).
 */
int oflow_corr_pyramid_f32(const float* d_fmap1, const float* d_fmap2, int B, int C, int H, int W,
                           int num_levels, float* const* d_levels, void* stream);

/*
 * Windowed multi-level bilinear lookup (CorrBlock.__call__).
 *   d_levels[l] : as produced above (H_l, W_l from oflow_corr_pyramid_dims)
 *   d_coords    : (B, 2, H, W) fp32 pixel coordinates, channel 0 = x, 1 = y
 *   d_out       : (B, num_levels*(2r+1)^2, H, W) fp32; channel l*(2r+1)^2 + i*(2r+1) + j samples level l
 *                 at (x/2^l + i - r, y/2^l + j - r), bilinear, zero outside the level (grid_sample
 *                 align_corners=True, padding_mode='zeros').
 */
int oflow_corr_lookup_f32(const float* const* d_levels, const int* level_h, const int* level_w,
                          int num_levels, const float* d_coords, int B, int H, int W, int radius,
                          float* d_out, void* stream);

/*
 * Tiled pyramid storage (what CorrBlock uses internally): level l of each query is stored as
 * [ceil(H_l/4)][ceil(W_l/8)][4][8] fp32 tiles, one 4x8 tile = one 128-B line, so a (2r+2)^2 lookup window
 * touches ~7 lines instead of ~13 with canonical rows. oflow_corr_tiled_level_floats(H_l, W_l) = floats per query
 * of a level; levels are otherwise produced and read exactly like the canonical ones above, and
 * oflow_corr_untile_f32 rebuilds the canonical (Q, H_l, W_l) view bit-for-bit.
 */
long long oflow_corr_tiled_level_floats(int H_l, int W_l);
int oflow_corr_pyramid_tiled_f32(const float* d_fmap1, const float* d_fmap2, int B, int C, int H, int W,
                                 int num_levels, float* const* d_levels, void* stream);
/* oflow_corr_pyramid_tiled_s32: oflow_corr_pyramid_tiled_f32's levels (same tiled layout) from feature maps given as
 * S32 rows (B, H, W, C/32 groups of hi[32] | lo[32] fp16; C % 32 == 0; 16-B aligned) -- the RAFT forward's pyramid,
 * fed by the feature encoder's last convolution: products as three fp16 MFMAs on the hi/lo split (22-bit operands,
 * fp32 accumulation), not fp32 MFMAs. Within SURVEY §8(c)'s pyramid tolerance of the fp32 result (tested). */
int oflow_corr_pyramid_tiled_s32(const void* d_fmap1_s32, const void* d_fmap2_s32, int B, int C, int H, int W,
                                 int num_levels, float* const* d_levels, void* stream);
int oflow_corr_lookup_tiled_f32(const float* const* d_levels, const int* level_h, const int* level_w,
                                int num_levels, const float* d_coords, int B, int H, int W, int radius,
                                float* d_out, void* stream);
int oflow_corr_untile_f32(const float* d_tiled, float* d_out, long long Q, int H_l, int W_l, void* stream);

/*
 * Inverse warp (optical_flow.warp): out = grid_sample(frame, linspace-grid + flow, mode, padding_mode,
 * align_corners). d_frame, d_out: (B, C, H, W); d_flow: (B, 2, H, W) already normalized to [-1, 1] units.
 */
int oflow_grid_warp_f32(const float* d_frame, const float* d_flow, int B, int C, int H, int W, int mode,
                        int padding_mode, int align_corners, float* d_out, void* stream);

/*
 * Explicit-grid sampling (F.grid_sample): d_input (B, C, H, W), d_grid (B, Ho, Wo, 2) in [-1, 1] units
 * (x, y), d_out (B, C, Ho, Wo). Replaces the grid_sample inside methods/raft/model/utils.py:64-80
 * (bilinear_sampler, called there with align_corners=True, zeros padding) for callers outside CorrBlock.
 */
int oflow_grid_sample_f32(const float* d_input, const float* d_grid, int B, int C, int H, int W, int Ho, int Wo,
                          int mode, int padding_mode, int align_corners, float* d_out, void* stream);

/*
 * On-the-fly fp16 correlation (memory-efficient path for large frames; BASELINE configs[4], no volume).
 * Same output as oflow_corr_lookup_f32 on the dense pyramid of (fmap1, fmap2), by linearity of the pooling:
 * level-l correlations are dot products of fmap1 with the floor 2^l-pooled fmap2 (corr.py:38-54, 79-87).
 *   prepare: d_f1h = fmap1 / sqrt(C) as (B, H, W, C) fp16; d_f2h[l] = pool_l(fmap2) as (B, H_l, W_l, C) fp16,
 *            pooled in fp32 (d_scratch: B*C*sum_{l>=1} H_l*W_l floats) then rounded. C % 32 == 0.
 *   lookup:  d_out (B, L*(2r+1)^2, H, W) fp32, radius <= 4; window dot products on v_mfma_f32_16x16x32_f16.
 */
int oflow_corr_otf_prepare_f16(const float* d_fmap1, const float* d_fmap2, int B, int C, int H, int W,
                               int num_levels, void* d_f1h, void* const* d_f2h, float* d_scratch, void* stream);
int oflow_corr_lookup_otf_f16(const void* d_f1h, const void* const* d_f2h, const int* level_h, const int* level_w,
                              int num_levels, const float* d_coords, int B, int C, int H, int W, int radius,
                              float* d_out, void* stream);

/*
 * Fused elementwise stages of the update block around its (bias-free) MIOpen convolutions
 * (methods/raft/model/update.py:69-161). Tensors are (B, C, P) with contiguous (C, P)
 * parts and an explicit batch stride in floats, so they can be channel slices of concatenated buffers.
 *   bias_act : y0[b,c,p] (and y1 if not NULL) = act(x[b,c,p] + bias[c]) * scale; act 0 none, 1 relu,
 *              2 sigmoid, 3 tanh; bias may be NULL; y0 may alias x.
 *   gru_reset: rh = sigmoid(zr[:, CH + c] + br[c]) * h          (zr = [z | r] pre-bias gate convolution)
 *   gru_blend: h = (1 - z) * h + z * tanh(q + bq[c]), z = sigmoid(zr[:, c] + bz[c]); h updated in place
 */
int oflow_bias_act_f32(const float* d_x, long long sx, const float* d_bias, float* d_y0, long long sy0, float* d_y1,
                       long long sy1, int B, int C, int P, int activation, float scale, void* stream);
int oflow_gru_reset_f32(const float* d_zr, long long szr, const float* d_br, const float* d_h, long long sh,
                        float* d_rh, long long srh, int B, int CH, int P, void* stream);
int oflow_gru_blend_f32(const float* d_zr, long long szr, const float* d_bz, const float* d_q, long long sq,
                        const float* d_bq, float* d_h, long long sh, int B, int CH, int P, void* stream);

/*
 * Split-fp16 ("S32") update-block path: fp32-accurate convolutions on the fp16 matrix cores
 * (methods/raft/model/update.py:40-161; csrc/conv_s32.hip).
 *
 * S32 activation format: NHWC by groups of 32 channels; element (pixel p, channel c) of a buffer with G groups
 * is hi = fp16(v) at byte p*G*128 + (c/32)*128 + (c%32)*2 and lo = fp16(v - hi) 64 bytes further (v ~ hi + lo,
 * 22 significant bits). A channel slice starting at group g0 is (base + g0*128, pixel stride G*128).
 * Padding channels (beyond the real ones, up to a multiple of 32) must hold zeros.
 *
 * oflow_conv_s32: stride-1 'same' convolution, kernel kh x kw in {1x1, 3x3, 1x5, 5x1}, over in_groups*32 input
 *   channels. d_wpack = weights packed as [in_groups][kh*kw][n_pad][hi[32] | lo[32]] fp16 after scaling output
 *   channel n by 2^s_n (|w| <= 2^14); d_wscale[n] = 2^-s_n. block_n in {32, 64, 128} divides n_pad.
 *   value = act(acc * wscale[n] + bias[n]) * out_scale, act 0 none, 1 relu, 2 sigmoid, 3 tanh, then
 *   epilogue 0: stored to S32 d_y0 (and d_y1 if not NULL) for channels n < N, and/or to fp32 NCHW d_f32
 *               (batch / channel strides in floats; f32_accumulate = 1 adds to it);
 *   epilogue 1 (GRU gates, N = 2*CH): n < CH -> z = sigmoid(.) into d_gru_z ([P][CH] fp32);
 *               n >= CH -> sigmoid(.) * d_gru_h[p][n-CH] into S32 d_y0 channel n-CH   (update.py:91-96)
 *   epilogue 2 (GRU candidate, N = CH): h = (1 - z) * h + z * tanh(.), in place in d_gru_h and into S32 d_y0
 *               (update.py:96-97). (act is ignored by epilogues 1 and 2.) Epilogues 1 and 2 read / write d_gru_h
 *               and d_gru_z as 16-B vectors: both must be 16-byte aligned (else OFLOW_E_ALIGN).
 * oflow_pack_s32_f32: d_x (B, C, H, W) fp32 with batch stride x_batch_stride -> act -> S32 d_y0 (and d_y1) channels
 *   dst_channel + c (dst_channel % 8 == 0; the last 8-channel chunk is zero-filled past C), and optionally a
 *   [P][nhwc_pixel_stride] fp32 copy.                                     (raft.py:115-118: tanh / relu of cnet)
 * oflow_flow_prep_s32: flow = coords1 - pixel grid (raft.py:129) as the 7x7 patch matrix of convf1
 *   (d_patches: S32 with 4 groups; channel t*2 + c = flow c at tap t = ky*7 + kx, zero padded) and, if not NULL,
 *   the 2 flow channels at d_flow0 / d_flow1 (byte address of the hi half of the x channel; y follows).
 */
int oflow_conv_s32(const void* d_x, long long x_pixel_stride, int in_groups, const void* d_wpack, int n_pad,
                   const float* d_wscale, const float* d_bias, int N, int B, int H, int W, int kh, int kw, int block_n,
                   int epilogue, int activation, float out_scale, void* d_y0, long long y0_pixel_stride, void* d_y1,
                   long long y1_pixel_stride, float* d_f32, long long f32_batch_stride, long long f32_channel_stride,
                   int f32_accumulate, float* d_gru_h, float* d_gru_z, int gru_channels, void* stream);
int oflow_pack_s32_f32(const float* d_x, long long x_batch_stride, int C, int B, int H, int W, int activation,
                       int dst_channel, void* d_y0, long long y0_pixel_stride, void* d_y1, long long y1_pixel_stride,
                       float* d_nhwc, int nhwc_pixel_stride, void* stream);
int oflow_flow_prep_s32(const float* d_coords, int B, int H, int W, void* d_patches, void* d_flow0,
                        long long flow0_pixel_stride, void* d_flow1, long long flow1_pixel_stride, void* stream);
/* oflow_flow_head2_s32: the flow head's output conv (update.py:35-36 conv2: 3x3, C -> 2, zero padding) added into
 * coords (B, 2, H, W) fp32 in place (raft.py:133 `coords1 = coords1 + delta_flow`), from an S32 input of in_groups
 * groups (1..8): fp32 FMAs on the exact S32 values; d_weight (2, C, 3, 3) fp32 as the nn.Conv2d stores it, d_bias [2].
 * Built for small grids (one image at 1/8 resolution); larger ones run faster as oflow_conv_s32 with n_pad 32. */
/* oflow_flow_head_col2im_f32: d_coords (B, 2, H, W) += d_bias[c] + sum_{ky,kx} d_y[b][(ky*3+kx)*2 + c][y+ky-1][x+kx-1]
 * (zero outside the image): the flow head's output conv (update.py:35-36, conv2 3x3 C -> 2, raft.py:133 coords1 +=
 * delta_flow) as a 1x1 conv C -> 18 per-tap products (oflow_conv_s32 with an fp32 NCHW destination d_y (B, 18, H, W))
 * followed by this gather. */
int oflow_flow_head_col2im_f32(const float* d_y, const float* d_bias, int B, int H, int W, float* d_coords, void* stream);

/* oflow_normalize_images_f32: y = 2 * (x / 255) - 1 for two frames of n fp32 values each (4-B aligned; vector loads
 * when n % 4 == 0 and 16-B aligned): RAFT.forward's input scaling (methods/raft/model/raft.py:104-105), the reference's
 * fp32 operations (a correctly rounded division) in one pass -- bit-identical to the reference on the CPU. */
int oflow_normalize_images_f32(const float* d_x0, const float* d_x1, long long n, float* d_y0, float* d_y1, void* stream);

/* oflow_replicate_pad_f32: InputPadder.pad (methods/raft/model/utils.py:38-61, F.pad(x, [left, right, top, bottom],
 * mode="replicate")) of `count` (1..4) tensors of `planes` x H x W fp32 values each (host arrays of device pointers),
 * into planes x (H + top + bottom) x (W + left + right): a copy, bit-exact, one launch. */
int oflow_replicate_pad_f32(const float* const* d_src, float* const* d_dst, int count, long long planes, int H, int W,
                            int top, int bottom, int left, int right, void* stream);

/* oflow_set_range_flag: register d_flag (one unsigned int in device memory of the current device; NULL: off) as the
 * range flag of the split-fp16 operands. Every kernel that writes or stages S32 values (the conv epilogues and staging,
 * norm_apply, pack / flow_prep, the fused lookup + convc1) sets it to 1 (atomic or) when a value's hi half overflows
 * fp16 (|x| >= 65520 or inf); it is never cleared by the library. Synchronous (a copy to each kernel module's symbol). */
int oflow_set_range_flag(unsigned int* d_flag);

/* oflow_range_flag_exchange: *d_out = the range flag's value, and the flag cleared, in one device atomic exchange on
 * `stream` (enqueued after a forward's kernels: that forward's snapshot; an overflow set concurrently by a forward on
 * another stream lands in this snapshot or the next one, never lost). d_flag: the pointer given to
 * oflow_set_range_flag; d_out: one unsigned int of device memory. Replaces nothing in the reference (the split-fp16
 * range guard of RAFT.forward, methods/raft/model/raft.py:87-147, is this build's addition). */
int oflow_range_flag_exchange(unsigned int* d_flag, unsigned int* d_out, void* stream);

/* Instrumentation (bench.py's per-kernel timings; replaces nothing in the reference): HIP timing events that can be
 * recorded inside a stream capture as external event-record nodes (external != 0), so every replay of the graph
 * re-records them; oflow_timing_event_elapsed_ms = hipEventElapsedTime(end - start). Status OFLOW_OK or a HIP error. */
int oflow_timing_event_create(void** ev);
int oflow_timing_event_destroy(void* ev);
int oflow_timing_event_record(void* ev, void* stream, int external);
int oflow_timing_event_elapsed_ms(void* start, void* end, float* ms);

int oflow_flow_head2_s32(const void* d_x, long long x_pixel_stride, int in_groups, const float* d_weight,
                         const float* d_bias, int B, int H, int W, float* d_coords, void* stream);
/* oflow_flow_head2_tiled_s32: oflow_flow_head2_s32 for large grids (update.py:36 FlowHead.conv2 + raft.py:133): each
 * workgroup stages a 4 x 32 output tile's 6 x 34 halo per 32-channel group in LDS as fp32 (hi + lo) and runs the
 * 3x3 x C -> 2 products as fp32 FMAs. d_wr: the weight (2, C, 3, 3) repacked [group][4-channel chunk][tap][output][4]
 * (16-B aligned); coords1 (B, 2, H, W) += conv + bias. */
int oflow_flow_head2_tiled_s32(const void* d_x, long long x_pixel_stride, int in_groups, const float* d_wr,
                               const float* d_bias, int B, int H, int W, float* d_coords, void* stream);
/* oflow_corr_lookup_tiled_nhwc_f32: the tiled lookup as fp32 NHWC rows [B*H*W][row_floats] (d_out 16-B aligned) in the
 * reference's channel order: row q, channel l*(2r+1)^2 + k = oflow_corr_lookup_tiled_f32's (b, l*(2r+1)^2 + k, y, x) bit for
 * bit; row_floats >= num_levels*(2r+1)^2, channels past that are not written. With row_floats = num_levels*(2r+1)^2 (324)
 * it is the RAFT forward's convc1 input (oflow_conv_s32_ex2, OFLOW_IN_F32). Replaces corr.py:56-77 + the permute feeding
 * update.py:120-121. */
int oflow_corr_lookup_tiled_nhwc_f32(const float* const* d_levels, const int* level_h, const int* level_w, int num_levels,
                                     const float* d_coords, int B, int H, int W, int radius, float* d_out, int row_floats,
                                     void* stream);
/* oflow_corr_lookup_convc1_s32: the tiled lookup fused into the motion encoder's first convolution -- S32 output
 * y = relu(convc1(corr_fn(coords))) (256 channels: d_y + P * y_pixel_stride, 8 groups), the lookup volume never
 * written. Replaces raft.py:128 (corr.py:56-77) + update.py:120-121 (`F.relu(self.convc1(corr))`) in the forward.
 * Weights: oflow_conv_s32's packing (1x1, n_pad 256) of convc1 with its input channels regrouped per level -- level l's
 * tap k at channel l*G*32 + k, G = ceil((2r+1)^2/32), zeros elsewhere (num_levels*G k32 groups) -- stored
 * fragment-major: [group][wave 4][n tile 2][sub 2][hi, lo][lane 64][8 fp16], where lane = hh*32 + r holds output channel
 * wave*64 + ntile*32 + r, inputs k = 16*sub + 8*hh .. +7 of the group (the same bytes as the conv packing
 * [group][256][hi 32 | lo 32], permuted); d_wscale [256], d_bias [256] or NULL. radius 3 or 4 (else OFLOW_E_RADIUS),
 * y_pixel_stride % 128 == 0. */
int oflow_corr_lookup_convc1_s32(const float* const* d_levels, const int* level_h, const int* level_w, int num_levels,
                                 const float* d_coords, int B, int H, int W, int radius, const void* d_wpack,
                                 const float* d_wscale, const float* d_bias, void* d_y, long long y_pixel_stride,
                                 void* stream);

/*
 * Encoders on the split-fp16 path (methods/raft/model/extractor.py:35-231; csrc/encoder_s32.hip).
 *
 * oflow_conv_s32_ex: oflow_conv_s32 plus (epilogue 0 only)
 *   d_nhwc        : fp32 [P][nhwc_pixel_stride] copy of the value (after activation / residual);
 *   d_stats       : per-tile instance-norm partials (count, mean, M2) of the pre-activation conv output, layout
 *                   [B][ceil(H/4)*ceil(W/32)][n_pad][3] floats (reduced by oflow_norm_stats_finalize);
 *   d_res         : S32 residual added after the activation, then res_activation (relu(x + y), extractor.py:90);
 *   s2d           : S32 destinations in space-to-depth layout (pixel (y/2, x/2), channel + ((y%2)*2 + x%2) * N), the
 *                   input form of the next stage's stride-2 convolutions (a 3x3/2 conv = a 2x2/1 conv on s2d input,
 *                   a 1x1/2 conv = a 1x1 conv over the first N channels of it).  kh x kw also allows 2x2 (taps at
 *                   offsets -1, 0), block_n also 96.
 * oflow_conv_s32_ex2: oflow_conv_s32_ex with an input format: OFLOW_IN_S32 (as _ex); OFLOW_IN_F32_NORM: the raw fp32
 *   NHWC output [P][in_groups*32] of the previous convolution (x_pixel_stride = in_groups*128), normalised and ReLU'd
 *   while staged, x = max(0, raw * d_in_scale[b, c] + d_in_shift[b, c]) ([B][in_groups*32] each) -- the instance
 *   norm + ReLU between a residual block's two 3x3 convs (extractor.py:75-76) never materialises (3x3, epilogue 0,
 *   in_groups <= 4); OFLOW_IN_F32: an fp32 NHWC input of cin = x_pixel_stride/4 channels per pixel
 *   ((in_groups-1)*32 < cin <= in_groups*32, x_pixel_stride % 16 == 0; channels past cin stage as zeros) split into
 *   hi + lo while staged (1x1, epilogue 0, block_n 128: convc1 reading oflow_corr_lookup_tiled_nhwc_f32's rows).
 *   OFLOW_IN_IMG7S2: the encoders' stem (extractor.py:186, a 7x7 / stride 2 / pad 3 conv of a 3-channel image) straight
 *   from the fp32 NCHW image d_x (B, 3, 2H, 2W) for an output of H x W (x_pixel_stride ignored): each 4 x 32 output tile
 *   stages its 13 x 69 x 3 input window in LDS and builds the patch-matrix operand (channel t*3 + c, t = ky*7 + kx,
 *   in_groups 5 = 160 channels, weights packed with patches=True as for oflow_stem_patches_s32's matrix) from it, so
 *   no patch matrix is written (1x1 geometry, epilogue 0, block_n 64).
 *   OFLOW_IN_FLOW7: the motion encoder's convf1 (update.py:116, a 7x7 / stride 1 / pad 3 conv of the 2-channel flow)
 *   straight from coords1 d_x (B, 2, H, W) fp32 (x_pixel_stride ignored): flow = coords1 - the pixel grid (raft.py:129,
 *   the fp32 subtraction of oflow_flow_prep_s32), each 4 x 32 output tile stages its 10 x 38 x 2 flow window in LDS
 *   and builds the patch operand (channel t*2 + c, t = ky*7 + kx, in_groups 4 = 128 channels, weights packed with
 *   patches=True as for oflow_flow_prep_s32's matrix) from it: bit for bit the conv of that matrix, which is then not
 *   written (1x1 geometry, epilogue 0, block_n 128).
 * oflow_stem_patches_s32: 7x7/2 pad-3 patch matrix of a (B, C, H, W) fp32 image: S32 (B, ceil(H/2), ceil(W/2),
 *   out_groups) with channel t*C + c (t = ky*7 + kx), zeros past 49*C.
 * oflow_norm_stats_finalize: merge the partials (fp64 sums) -> alpha = 1/sqrt(var + eps), beta = -mean * alpha, [B][C].
 * oflow_norm_apply_s32: y = act(x*alpha + beta) for x [P][C] fp32 (C % 8 == 0); res_mode 1: y = res_act(y + S32 res),
 *   res_mode 2: y = res_act((x2*alpha2 + beta2) + y); res_mode 3: y = res_act(relu(x2*alpha2 + beta2) + y) (a block
 *   input kept as raw fp32 + its norm); written as S32 (s2d: space-to-depth as above).
 */
int oflow_conv_s32_ex(const void* d_x, long long x_pixel_stride, int in_groups, const void* d_wpack, int n_pad,
                      const float* d_wscale, const float* d_bias, int N, int B, int H, int W, int kh, int kw,
                      int block_n, int epilogue, int activation, float out_scale, void* d_y0, long long y0_pixel_stride,
                      void* d_y1, long long y1_pixel_stride, float* d_f32, long long f32_batch_stride,
                      long long f32_channel_stride, int f32_accumulate, float* d_gru_h, float* d_gru_z,
                      int gru_channels, float* d_nhwc, int nhwc_pixel_stride, float* d_stats, const void* d_res,
                      long long res_pixel_stride, int res_activation, int s2d, void* stream);
int oflow_conv_s32_ex2(const void* d_x, long long x_pixel_stride, int in_groups, const void* d_wpack, int n_pad,
                       const float* d_wscale, const float* d_bias, int N, int B, int H, int W, int kh, int kw,
                       int block_n, int epilogue, int activation, float out_scale, void* d_y0, long long y0_pixel_stride,
                       void* d_y1, long long y1_pixel_stride, float* d_f32, long long f32_batch_stride,
                       long long f32_channel_stride, int f32_accumulate, float* d_gru_h, float* d_gru_z,
                       int gru_channels, float* d_nhwc, int nhwc_pixel_stride, float* d_stats, const void* d_res,
                       long long res_pixel_stride, int res_activation, int s2d, int in_format,
                       const float* d_in_scale, const float* d_in_shift, void* stream);
/* oflow_conv_s32_ex3: oflow_conv_s32_ex2 plus an fp32 NHWC addend d_addend[P * addend_pixel_stride + n] added to the
 * pre-activation value after the scale and bias (GRU epilogues 1 and 2 only; 16-B aligned, addend_pixel_stride >= N,
 * a multiple of 4; NULL = none). It carries the GRU's loop-invariant context term: x = [inp | motion] (update.py:153-154)
 * and inp never changes across iterations (raft.py:115-118), so W_inp * inp + bias is computed once per forward and the
 * per-iteration z / r / q convolutions (update.py:92-105) run over [h | motion | flow] only. */
int oflow_conv_s32_ex3(const void* d_x, long long x_pixel_stride, int in_groups, const void* d_wpack, int n_pad,
                       const float* d_wscale, const float* d_bias, int N, int B, int H, int W, int kh, int kw,
                       int block_n, int epilogue, int activation, float out_scale, void* d_y0, long long y0_pixel_stride,
                       void* d_y1, long long y1_pixel_stride, float* d_f32, long long f32_batch_stride,
                       long long f32_channel_stride, int f32_accumulate, float* d_gru_h, float* d_gru_z,
                       int gru_channels, float* d_nhwc, int nhwc_pixel_stride, float* d_stats, const void* d_res,
                       long long res_pixel_stride, int res_activation, int s2d, int in_format,
                       const float* d_in_scale, const float* d_in_shift, const float* d_addend,
                       long long addend_pixel_stride, void* stream);
/* oflow_conv_s32_ex4: oflow_conv_s32_ex3 plus d_wfrag, an optional fragment-major copy of d_wpack (same bytes, reordered
 * [group][tap][n/32][slice][hi|lo][k half][row][8] so that one wave's 32x16 MFMA B fragment is 1 KB contiguous and is
 * loaded straight into registers, skipping the LDS staging of B). Used, on S32 input without instance-norm partials
 * outside the small-grid tiles, by every multi-tap convolution with block_n 128 and by 3x3 convolutions with block_n 64
 * or 32; other shapes ignore it. The block_n 64 / 32 register-direct variants measured slower in the RAFT step
 * (DESIGN.md §4, r04): pass NULL for them unless comparing (the Python layer passes d_wfrag for them only under
 * OFLOW_CONV_BREG64 / OFLOW_CONV_BREG32). NULL = ex3. */
int oflow_conv_s32_ex4(const void* d_x, long long x_pixel_stride, int in_groups, const void* d_wpack, int n_pad,
                       const float* d_wscale, const float* d_bias, int N, int B, int H, int W, int kh, int kw,
                       int block_n, int epilogue, int activation, float out_scale, void* d_y0, long long y0_pixel_stride,
                       void* d_y1, long long y1_pixel_stride, float* d_f32, long long f32_batch_stride,
                       long long f32_channel_stride, int f32_accumulate, float* d_gru_h, float* d_gru_z,
                       int gru_channels, float* d_nhwc, int nhwc_pixel_stride, float* d_stats, const void* d_res,
                       long long res_pixel_stride, int res_activation, int s2d, int in_format,
                       const float* d_in_scale, const float* d_in_shift, const float* d_addend,
                       long long addend_pixel_stride, const void* d_wfrag, void* stream);
/* oflow_conv_s32_ex5: oflow_conv_s32_ex4 plus split-K over the input groups for the register-direct kernels (S32 input,
 * d_wfrag given, in_groups even; the 224-workgroup GRU q / motion convs of a 4-pair lane fill 224 of 512 two-per-CU
 * slots unsplit). Each 4 x 32-pixel tile (x block_n channels) runs as two workgroups, each summing half of the input
 * groups; the first to finish hands its fp32 partials to the second through d_ksplit_slab (write-through stores, an
 * agent-scope counter, an acquire on the reader), which adds them and runs the epilogue. Results differ from ex4 only
 * in the order of one fp32 addition per output (and do not depend on which workgroup finishes first).
 *   d_ksplit_slab: >= ksplit_tiles * 128 * block_n floats, 16-B aligned, any contents;
 *   d_ksplit_ctr: 2 * ksplit_tiles uint32, 8-B aligned, ZEROED ONCE before the first call; the counters only grow (two
 *     tickets and one publication per tile and call), so successive calls and graph replays need no reset -- but
 *     calls that share a buffer pair must be stream-ordered (never in flight together);
 *   ksplit_tiles: capacity; OFLOW_E_SHAPE if the call needs B * ceil(H/4) * ceil(W/32) * n_pad / block_n more.
 * A split call always runs the default 4-row tiles, small grids included (so that a caller deciding the split from its
 * whole batch gets the same bits from any partition of it into calls); calls of other shapes (not register-direct, odd
 * in_groups) run unsplit. Both NULL = ex4. */
int oflow_conv_s32_ex5(const void* d_x, long long x_pixel_stride, int in_groups, const void* d_wpack, int n_pad,
                       const float* d_wscale, const float* d_bias, int N, int B, int H, int W, int kh, int kw,
                       int block_n, int epilogue, int activation, float out_scale, void* d_y0, long long y0_pixel_stride,
                       void* d_y1, long long y1_pixel_stride, float* d_f32, long long f32_batch_stride,
                       long long f32_channel_stride, int f32_accumulate, float* d_gru_h, float* d_gru_z,
                       int gru_channels, float* d_nhwc, int nhwc_pixel_stride, float* d_stats, const void* d_res,
                       long long res_pixel_stride, int res_activation, int s2d, int in_format,
                       const float* d_in_scale, const float* d_in_shift, const float* d_addend,
                       long long addend_pixel_stride, const void* d_wfrag, float* d_ksplit_slab,
                       unsigned* d_ksplit_ctr, long long ksplit_tiles, void* stream);
int oflow_stem_patches_s32(const float* d_img, int B, int C, int H, int W, void* d_out, int out_groups, void* stream);
int oflow_norm_stats_finalize(const float* d_partials, int B, int tiles, int n_pad, int C, double eps, float* d_alpha,
                              float* d_beta, void* stream);
int oflow_norm_apply_s32(const float* d_x, int C, int B, int H, int W, const float* d_alpha, const float* d_beta,
                         int activation, int res_mode, const void* d_res, long long res_pixel_stride, const float* d_x2,
                         const float* d_alpha2, const float* d_beta2, int res_activation, int s2d, void* d_y,
                         long long y_pixel_stride, void* stream);

/*
 * Convex upsampling (methods/raft/model/raft.py:73-85, RAFT.upsample_flow; csrc/upsample.hip).
 * oflow_convex_upsample_f32: flow (B, 2, H, W), mask (B, 576, H, W) (the mask head output, already x0.25) ->
 *   out (B, 2, 8H, 8W): softmax over the 9 neighbours of each 8x8 sub-pixel, convex combination of 8*flow over the
 *   zero-padded 3x3 neighbourhood. B, H <= 65535.
 */
int oflow_convex_upsample_f32(const float* d_flow, const float* d_mask, int B, int H, int W, float* d_out, void* stream);

/*
 * Backward of the correlation (methods/raft/model/corr.py:38-87 + utils.py:64-80 under autograd, the training step
 * raft.py:149-175; csrc/corr_backward.hip). Canonical levels (B*H*W, H_l, W_l) fp32.
 * oflow_corr_lookup_backward_f32: d_grad_out (B, L*(2r+1)^2, H, W) -> d_grad_levels[l] += its gradient (same window
 *   and weights as the forward; coordinates get none: the reference detaches them, raft.py:127).
 * oflow_corr_pyramid_grad_combine_f32: d_grad_levels[0] += sum_{l>0} of level l's gradient pushed back through the
 *   floor 2x2 average pools (value / 4^l on every level-0 cell it averaged).
 */
int oflow_corr_lookup_backward_f32(const float* d_grad_out, const float* d_coords, int B, int H, int W, int radius,
                                   float* const* d_grad_levels, const int* level_h, const int* level_w, int num_levels,
                                   void* stream);
int oflow_corr_pyramid_grad_combine_f32(float* const* d_grad_levels, const int* level_h, const int* level_w,
                                        int num_levels, long long Q, void* stream);
/* oflow_corr_fmap_grad_f32: the feature-map gradients of corr.py:85 (corr = f1^T f2 / sqrt(C)) from the level-0-folded
 *   gradient g0 (B, N, N) (query-major): d_grad_f1 (B, C, N) = scale * f2 . g0^T, d_grad_f2 (B, C, N) = scale * f1 . g0
 *   (scale = 1/sqrt(C)), fmaps (B, C, N) fp32; fp32 MFMA GEMMs, deterministic. Either output may be NULL. */
int oflow_corr_fmap_grad_f32(const float* d_fmap1, const float* d_fmap2, const float* d_g0, int B, int C, int N,
                             float scale, float* d_grad_f1, float* d_grad_f2, void* stream);

/*
 * Backward of the warp / grid_sample (optical_flow/operator/operator.py:8-56, utils.py:64-80 under autograd; SURVEY
 * §8(f) row 3; csrc/warp_backward.hip): ATen grid_sampler_2d_backward's formulas for every mode / padding /
 * align_corners. d_grad_frame / d_grad_input must be zero-filled by the caller (taps are added with fp32 atomics);
 * either output may be NULL.
 * oflow_grid_warp_backward_f32: d_grad_out (B, C, H, W), frame (B, C, H, W), normalized flow (B, 2, H, W) ->
 *   d_grad_frame (B, C, H, W) += ..., d_grad_flow (B, 2, H, W) = dL/d(grid) (grid = linspace base + flow).
 * oflow_grid_sample_backward_f32: d_grad_out (B, C, Ho, Wo), input (B, C, H, W), grid (B, Ho, Wo, 2) ->
 *   d_grad_input += ..., d_grad_grid (B, Ho, Wo, 2).
 */
int oflow_grid_warp_backward_f32(const float* d_grad_out, const float* d_frame, const float* d_flow, int B, int C, int H,
                                 int W, int mode, int padding_mode, int align_corners, float* d_grad_frame,
                                 float* d_grad_flow, void* stream);
int oflow_grid_sample_backward_f32(const float* d_grad_out, const float* d_input, const float* d_grid, int B, int C,
                                   int H, int W, int Ho, int Wo, int mode, int padding_mode, int align_corners,
                                   float* d_grad_input, float* d_grad_grid, void* stream);

/*
 * Inference I/O (csrc/flow_io.hip).
 * oflow_flow_stats_f32: flow (B, 2, H, W) -> d_partials (B, OFLOW_FLOW_STATS_CHUNKS, 2): per-chunk maxima of |flow|
 *   and of the flow values, after clip to [clip_lo, clip_hi] (when clip != 0) and y negation (when invert_y != 0).
 * oflow_flow2rgb_f32: flow (B, 2, H, W) -> d_rgb (B, 3, H, W) in [0, 1], the reference's flow2rgb
 *   (optical_flow/visualization/flow2rgb.py:19-73). method OFLOW_FLOW2RGB_{BAKER,HSV,MEISTER}. The flow is divided
 *   by denom (= max_norm + 1e-5, the caller's max_norm) when have_denom != 0, else by max|flow| + 1e-5 taken from
 *   d_partials (which oflow_flow_stats_f32 must have filled with the same clip / invert_y, earlier on the stream).
 *   d_partials is also required for MEISTER (its max_flow). Same clip / invert_y semantics as above.
 * oflow_flow_pack_f32: planar flow (B, 2, H, W) -> per image the file payload (H, W, channels) fp32:
 *   channels 2 = Middlebury .flo rows (io/middlebury.py:64-71); channels 3 = PFM rows with a zero third channel,
 *   written bottom row first when flip_rows != 0 (io/pfm.py:95-98). B, H <= 65535.
 */
#define OFLOW_FLOW_STATS_CHUNKS 128
#define OFLOW_FLOW2RGB_BAKER 0
#define OFLOW_FLOW2RGB_HSV 1
#define OFLOW_FLOW2RGB_MEISTER 2
int oflow_flow_stats_f32(const float* d_flow, int B, int H, int W, int clip, float clip_lo, float clip_hi,
                         int invert_y, float* d_partials, void* stream);
int oflow_flow2rgb_f32(const float* d_flow, int B, int H, int W, int method, int clip, float clip_lo, float clip_hi,
                       int invert_y, int have_denom, float denom, const float* d_partials, float* d_rgb, void* stream);
int oflow_flow_pack_f32(const float* d_flow, int B, int H, int W, int channels, int flip_rows, float* d_out,
                        void* stream);

#ifdef __cplusplus
}
#endif

#endif /* OFLOW_H_ */
