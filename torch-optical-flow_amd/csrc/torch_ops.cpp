// PyTorch operator registration of the correlation / warp path: TORCH_LIBRARY(oflow) -> torch.ops.oflow.*.
//
// Each op's HIP-key (PyTorch-ROCm's "CUDA" dispatch key) kernel validates its tensors and calls the C ABI of
// liboflow_hip.so (include/oflow.h) on PyTorch's current HIP stream; the Meta kernel computes output shapes only,
// which is what torch.compile's fake-tensor tracing runs. Autograd formulas are registered from Python
// (optical_flow/_ops.py) on top of these ops, so CorrBlock / warp trace into a single graph with no breaks.
//
// Ops (reference interface each one implements):
//   corr_pyramid(fmap1, fmap2, num_levels) -> Tensor[]            CorrBlock.__init__  (corr.py:38-54, 79-87)
//   corr_pyramid_tiled(fmap1, fmap2, num_levels) -> Tensor[]      same values, tiled lookup layout
//   corr_lookup(levels, coords, radius) -> Tensor                 CorrBlock.__call__  (corr.py:56-77)
//   corr_lookup_tiled(levels, coords, radius) -> Tensor           same, over the tiled levels
//   corr_lookup_tiled_nhwc(levels, coords, radius, out!) -> ()    same, fp32 NHWC rows (convc1 input)
//   corr_otf_prepare(fmap1, fmap2, num_levels) -> (Tensor, Tensor[])  AlternateCorrBlock.__init__ (fp16 features)
//   corr_lookup_otf(f1h, f2h, coords, radius) -> Tensor           AlternateCorrBlock.__call__ (corr.py:90-110)
//   grid_warp(frame, flow, mode, padding_mode, align_corners)     optical_flow.warp   (operator.py:8-33)
//   grid_sample(input, grid, mode, padding_mode, align_corners)   bilinear_sampler    (utils.py:64-80)
//   corr_lookup_backward(grad_out, coords, radius, H0, W0, L)     transpose of corr_lookup (training, §8(f) row 3)
//   corr_pyramid_backward(level_grads, fmap1, fmap2) -> (g1, g2)  pool transpose + two fp32-MFMA GEMMs
//   grid_warp_backward(grad_out, frame, flow, mode, pad, ac, mask) -> (grad_frame, grad_flow)     warp's autograd
//   grid_sample_backward(grad_out, input, grid, mode, pad, ac, mask) -> (grad_input, grad_grid)   grid_sample's autograd
#include <array>
#include <torch/library.h>
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>

#include <cmath>
#include <vector>

#include "oflow.h"

namespace {

using at::Tensor;

void check_status(int st, const char* what) {
  if (st == OFLOW_OK) return;
  // Q3 (a level under 2 px): the reference returns NaN; this build raises ValueError, as the Python layer did
  TORCH_CHECK_VALUE(st != OFLOW_E_TINY, what, ": ", oflow_status_string(st));
  TORCH_CHECK(false, what, " failed (", st, "): ", oflow_status_string(st));
}

void* cur_stream() { return (void*)c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

Tensor gpu_f32(const Tensor& t, const char* name, const char* what) {
  TORCH_CHECK(t.is_cuda(), what, ": ", name, " is on ", t.device(),
              "; this MI355X build runs only on ROCm GPU tensors (no CPU fallback)");
  return t.to(at::kFloat).contiguous();
}

std::vector<std::pair<int, int>> dims_of(int64_t h, int64_t w, int64_t nl, const char* what) {
  TORCH_CHECK(nl >= 1 && nl <= OFLOW_MAX_LEVELS, what, ": number of pyramid levels ", nl, " outside [1, ",
              OFLOW_MAX_LEVELS, "]");
  int hs[OFLOW_MAX_LEVELS], ws[OFLOW_MAX_LEVELS];
  check_status(oflow_corr_pyramid_dims((int)h, (int)w, (int)nl, hs, ws), what);
  std::vector<std::pair<int, int>> d;
  for (int l = 0; l < nl; ++l) d.emplace_back(hs[l], ws[l]);
  return d;
}

void check_fmaps(const Tensor& f1, const Tensor& f2, const char* what) {
  TORCH_CHECK(f1.dim() == 4 && f1.sizes() == f2.sizes(), what, ": fmap1 ", f1.sizes(), " and fmap2 ", f2.sizes(),
              " must be equal (B, C, H, W)");
  TORCH_CHECK(f1.device() == f2.device(), what, ": fmap1 and fmap2 are on different devices");
}

void check_pool_dims(const std::vector<std::pair<int, int>>& d, int64_t nl, const char* what) {
  for (auto& p : d)
    TORCH_CHECK(p.first >= 1 && p.second >= 1, what, ": ", nl, " levels of 2x2 pooling need H, W >= ",
                1 << (nl - 1));
}

void check_radius(int64_t r, int64_t rmax, const char* what) {
  TORCH_CHECK(r >= 0 && r <= rmax, what, ": radius ", r, " outside [0, ", rmax, "]");
}

void check_coords(const Tensor& co, const char* what) {
  TORCH_CHECK(co.dim() == 4 && co.size(1) == 2, what, ": coords must be (B, 2, H, W), got ", co.sizes());
}

// ---------------------------------------------------------------- pyramid
std::vector<Tensor> corr_pyramid_hip(const Tensor& fmap1, const Tensor& fmap2, int64_t num_levels) {
  const char* what = "corr_pyramid";
  check_fmaps(fmap1, fmap2, what);
  Tensor f1 = gpu_f32(fmap1, "fmap1", what), f2 = gpu_f32(fmap2, "fmap2", what);
  const int64_t b = f1.size(0), c = f1.size(1), h = f1.size(2), w = f1.size(3);
  auto d = dims_of(h, w, num_levels, what);
  std::vector<Tensor> levels;
  for (auto& p : d) levels.push_back(at::empty({b * h * w, 1, p.first, p.second}, f1.options()));
  if (b == 0) return levels;
  check_pool_dims(d, num_levels, what);
  c10::hip::HIPGuardMasqueradingAsCUDA g(f1.device());
  float* ptrs[OFLOW_MAX_LEVELS];
  for (int l = 0; l < num_levels; ++l) ptrs[l] = levels[l].data_ptr<float>();
  check_status(oflow_corr_pyramid_f32(f1.data_ptr<float>(), f2.data_ptr<float>(), (int)b, (int)c, (int)h, (int)w,
                                      (int)num_levels, ptrs, cur_stream()),
               what);
  return levels;
}

std::vector<Tensor> corr_pyramid_meta(const Tensor& fmap1, const Tensor& fmap2, int64_t num_levels) {
  check_fmaps(fmap1, fmap2, "corr_pyramid");
  const int64_t b = fmap1.size(0), h = fmap1.size(2), w = fmap1.size(3);
  std::vector<Tensor> levels;
  for (auto& p : dims_of(h, w, num_levels, "corr_pyramid"))
    levels.push_back(at::empty({b * h * w, 1, p.first, p.second}, fmap1.options().dtype(at::kFloat)));
  return levels;
}

std::vector<Tensor> corr_pyramid_tiled_hip(const Tensor& fmap1, const Tensor& fmap2, int64_t num_levels) {
  const char* what = "corr_pyramid";
  check_fmaps(fmap1, fmap2, what);
  Tensor f1 = gpu_f32(fmap1, "fmap1", what), f2 = gpu_f32(fmap2, "fmap2", what);
  const int64_t b = f1.size(0), c = f1.size(1), h = f1.size(2), w = f1.size(3), q = b * h * w;
  auto d = dims_of(h, w, num_levels, what);
  check_pool_dims(d, num_levels, what);
  std::vector<Tensor> levels;
  for (auto& p : d) levels.push_back(at::empty({q, oflow_corr_tiled_level_floats(p.first, p.second)}, f1.options()));
  if (q == 0) return levels;
  c10::hip::HIPGuardMasqueradingAsCUDA g(f1.device());
  float* ptrs[OFLOW_MAX_LEVELS];
  for (int l = 0; l < num_levels; ++l) ptrs[l] = levels[l].data_ptr<float>();
  check_status(oflow_corr_pyramid_tiled_f32(f1.data_ptr<float>(), f2.data_ptr<float>(), (int)b, (int)c, (int)h,
                                            (int)w, (int)num_levels, ptrs, cur_stream()),
               what);
  return levels;
}

std::vector<Tensor> corr_pyramid_tiled_meta(const Tensor& fmap1, const Tensor& fmap2, int64_t num_levels) {
  check_fmaps(fmap1, fmap2, "corr_pyramid");
  const int64_t q = fmap1.size(0) * fmap1.size(2) * fmap1.size(3);
  std::vector<Tensor> levels;
  for (auto& p : dims_of(fmap1.size(2), fmap1.size(3), num_levels, "corr_pyramid"))
    levels.push_back(at::empty({q, oflow_corr_tiled_level_floats(p.first, p.second)},
                               fmap1.options().dtype(at::kFloat)));
  return levels;
}

// ---------------------------------------------------------------- lookups
struct LevelArgs {
  const float* ptr[OFLOW_MAX_LEVELS];
  int h[OFLOW_MAX_LEVELS], w[OFLOW_MAX_LEVELS];
  int n = 0;
};

// canonical levels: (B*H*W, 1, H_l, W_l)
LevelArgs canonical_levels(const std::vector<Tensor>& lv, std::vector<Tensor>& keep, const Tensor& co,
                           const char* what) {
  const int64_t n = (int64_t)lv.size();
  TORCH_CHECK(n >= 1 && n <= OFLOW_MAX_LEVELS, what, ": number of pyramid levels ", n, " outside [1, ",
              OFLOW_MAX_LEVELS, "]");
  const int64_t q = co.size(0) * co.size(2) * co.size(3);
  LevelArgs a;
  a.n = (int)n;
  for (int64_t i = 0; i < n; ++i) {
    Tensor t = gpu_f32(lv[i], "corr_pyramid level", what);
    TORCH_CHECK(t.device() == co.device(), what, ": corr_pyramid[", i, "] and coords are on different devices");
    TORCH_CHECK(t.dim() == 4 && t.size(0) == q && t.size(1) == 1, what, ": corr_pyramid[", i, "] shape ", t.sizes(),
                " != (", q, ", 1, H_l, W_l)");
    keep.push_back(t);
    a.ptr[i] = t.data_ptr<float>();
    a.h[i] = (int)t.size(2);
    a.w[i] = (int)t.size(3);
  }
  return a;
}

// tiled levels: (B*H*W, floats_l), level dims from the query grid
LevelArgs tiled_levels(const std::vector<Tensor>& lv, const Tensor& co, const char* what) {
  const int64_t n = (int64_t)lv.size();
  auto d = dims_of(co.size(2), co.size(3), n, what);
  const int64_t q = co.size(0) * co.size(2) * co.size(3);
  LevelArgs a;
  a.n = (int)n;
  for (int64_t i = 0; i < n; ++i) {
    const Tensor& t = lv[i];
    TORCH_CHECK(t.is_cuda() && t.device() == co.device(), what, ": tiled level ", i, " and coords are on different devices");
    TORCH_CHECK(t.scalar_type() == at::kFloat && t.is_contiguous() && t.dim() == 2 && t.size(0) == q &&
                    t.size(1) == oflow_corr_tiled_level_floats(d[i].first, d[i].second),
                what, ": tiled level ", i, " ", t.sizes(), " does not match coords ", co.sizes(),
                " (expected a contiguous fp32 (", q, ", ", oflow_corr_tiled_level_floats(d[i].first, d[i].second), "))");
    a.ptr[i] = t.data_ptr<float>();
    a.h[i] = d[i].first;
    a.w[i] = d[i].second;
  }
  return a;
}

Tensor lookup_out(const Tensor& co, int64_t nl, int64_t radius) {
  const int64_t k = 2 * radius + 1;
  return at::empty({co.size(0), nl * k * k, co.size(2), co.size(3)}, co.options().dtype(at::kFloat));
}

Tensor corr_lookup_hip(const std::vector<Tensor>& levels, const Tensor& coords, int64_t radius) {
  const char* what = "corr_lookup";
  check_coords(coords, what);
  check_radius(radius, OFLOW_MAX_RADIUS, what);
  Tensor co = gpu_f32(coords, "coords", what);
  std::vector<Tensor> keep;
  LevelArgs a = canonical_levels(levels, keep, co, what);
  Tensor out = lookup_out(co, a.n, radius);
  if (out.numel() == 0) return out;
  c10::hip::HIPGuardMasqueradingAsCUDA g(co.device());
  check_status(oflow_corr_lookup_f32(a.ptr, a.h, a.w, a.n, co.data_ptr<float>(), (int)co.size(0), (int)co.size(2),
                                     (int)co.size(3), (int)radius, out.data_ptr<float>(), cur_stream()),
               what);
  return out;
}

Tensor corr_lookup_meta(const std::vector<Tensor>& levels, const Tensor& coords, int64_t radius) {
  check_coords(coords, "corr_lookup");
  check_radius(radius, OFLOW_MAX_RADIUS, "corr_lookup");
  return lookup_out(coords, (int64_t)levels.size(), radius);
}

Tensor corr_lookup_tiled_hip(const std::vector<Tensor>& levels, const Tensor& coords, int64_t radius) {
  const char* what = "corr_lookup";
  check_coords(coords, what);
  check_radius(radius, OFLOW_MAX_RADIUS, what);
  Tensor co = gpu_f32(coords, "coords", what);
  LevelArgs a = tiled_levels(levels, co, what);
  Tensor out = lookup_out(co, a.n, radius);
  if (out.numel() == 0) return out;
  c10::hip::HIPGuardMasqueradingAsCUDA g(co.device());
  check_status(oflow_corr_lookup_tiled_f32(a.ptr, a.h, a.w, a.n, co.data_ptr<float>(), (int)co.size(0),
                                           (int)co.size(2), (int)co.size(3), (int)radius, out.data_ptr<float>(),
                                           cur_stream()),
               what);
  return out;
}

void corr_lookup_tiled_nhwc_hip(const std::vector<Tensor>& levels, const Tensor& coords, int64_t radius,
                                const Tensor& out) {
  const char* what = "corr_lookup";
  check_coords(coords, what);
  check_radius(radius, OFLOW_MAX_RADIUS, what);
  Tensor co = gpu_f32(coords, "coords", what);
  LevelArgs a = tiled_levels(levels, co, what);
  const int64_t q = co.size(0) * co.size(2) * co.size(3);
  TORCH_CHECK(out.is_cuda() && out.device() == co.device() && out.scalar_type() == at::kFloat && out.is_contiguous() &&
                  out.dim() == 2 && out.size(0) == q,
              what, ": NHWC output must be a contiguous fp32 [B*H*W, row] on the coords' device, got ", out.sizes());
  if (q == 0) return;
  c10::hip::HIPGuardMasqueradingAsCUDA g(co.device());
  check_status(oflow_corr_lookup_tiled_nhwc_f32(a.ptr, a.h, a.w, a.n, co.data_ptr<float>(), (int)co.size(0),
                                                (int)co.size(2), (int)co.size(3), (int)radius, out.data_ptr<float>(),
                                                (int)out.size(1), cur_stream()),
               what);
}

void corr_lookup_tiled_nhwc_meta(const std::vector<Tensor>&, const Tensor& coords, int64_t radius, const Tensor&) {
  check_coords(coords, "corr_lookup");
  check_radius(radius, OFLOW_MAX_RADIUS, "corr_lookup");
}

// ---------------------------------------------------------------- on-the-fly (fp16 feature) correlation
std::tuple<Tensor, std::vector<Tensor>> otf_prepare_impl(const Tensor& fmap1, const Tensor& fmap2, int64_t num_levels,
                                                         bool run) {
  const char* what = "corr_otf_prepare";
  check_fmaps(fmap1, fmap2, what);
  if (run) TORCH_CHECK(fmap1.is_cuda(), what, ": fmap1 is on ", fmap1.device(),
                       "; this MI355X build runs only on ROCm GPU tensors (no CPU fallback)");
  const int64_t b = fmap1.size(0), c = fmap1.size(1), h = fmap1.size(2), w = fmap1.size(3);
  TORCH_CHECK(c % 32 == 0, what, ": the fp16 MFMA path needs C % 32 == 0, got C=", c);
  auto d = dims_of(h, w, num_levels, what);
  check_pool_dims(d, num_levels, what);
  auto o16 = fmap1.options().dtype(at::kHalf);
  Tensor f1h = at::empty({b, h, w, c}, o16);
  std::vector<Tensor> f2h;
  int64_t pooled = 0;
  for (int l = 0; l < num_levels; ++l) {
    f2h.push_back(at::empty({b, d[l].first, d[l].second, c}, o16));
    if (l) pooled += (int64_t)d[l].first * d[l].second;
  }
  if (!run || b == 0) return {f1h, f2h};
  Tensor f1 = gpu_f32(fmap1, "fmap1", what), f2 = gpu_f32(fmap2, "fmap2", what);
  Tensor scratch = at::empty({std::max<int64_t>(1, b * c * pooled)}, f1.options());
  c10::hip::HIPGuardMasqueradingAsCUDA g(f1.device());
  void* ptrs[OFLOW_MAX_LEVELS];
  for (int l = 0; l < num_levels; ++l) ptrs[l] = f2h[l].data_ptr();
  check_status(oflow_corr_otf_prepare_f16(f1.data_ptr<float>(), f2.data_ptr<float>(), (int)b, (int)c, (int)h, (int)w,
                                          (int)num_levels, f1h.data_ptr(), ptrs, scratch.data_ptr<float>(),
                                          cur_stream()),
               what);
  return {f1h, f2h};
}

std::tuple<Tensor, std::vector<Tensor>> otf_prepare_hip(const Tensor& f1, const Tensor& f2, int64_t nl) {
  return otf_prepare_impl(f1, f2, nl, true);
}
std::tuple<Tensor, std::vector<Tensor>> otf_prepare_meta(const Tensor& f1, const Tensor& f2, int64_t nl) {
  return otf_prepare_impl(f1, f2, nl, false);
}

Tensor corr_lookup_otf_impl(const Tensor& f1h, const std::vector<Tensor>& f2h, const Tensor& coords, int64_t radius,
                            bool run) {
  const char* what = "corr_lookup_otf";
  check_coords(coords, what);
  if (run) TORCH_CHECK(coords.is_cuda(), what, ": coords is on ", coords.device(),
                       "; this MI355X build runs only on ROCm GPU tensors (no CPU fallback)");
  check_radius(radius, 4, what);
  const int64_t b = coords.size(0), h = coords.size(2), w = coords.size(3);
  TORCH_CHECK(f1h.scalar_type() == at::kHalf && f1h.dim() == 4 && f1h.size(0) == b && f1h.size(1) == h &&
                  f1h.size(2) == w && f1h.is_contiguous(),
              what, ": f1h ", f1h.sizes(), " must be contiguous fp16 (", b, ", ", h, ", ", w, ", C)");
  const int64_t c = f1h.size(3), nl = (int64_t)f2h.size();
  TORCH_CHECK(nl >= 1 && nl <= OFLOW_MAX_LEVELS, what, ": number of pyramid levels ", nl, " outside [1, ",
              OFLOW_MAX_LEVELS, "]");
  const void* ptrs[OFLOW_MAX_LEVELS];
  int hs[OFLOW_MAX_LEVELS], ws[OFLOW_MAX_LEVELS];
  for (int64_t i = 0; i < nl; ++i) {
    const Tensor& t = f2h[i];
    TORCH_CHECK(t.scalar_type() == at::kHalf && t.dim() == 4 && t.size(0) == b && t.size(3) == c && t.is_contiguous(),
                what, ": fmap2 level ", i, " ", t.sizes(), " must be contiguous fp16 (", b, ", H_l, W_l, ", c, ")");
    TORCH_CHECK(t.device() == coords.device(), what, ": fmap2 level ", i, " and coords are on different devices");
    ptrs[i] = t.data_ptr();
    hs[i] = (int)t.size(1);
    ws[i] = (int)t.size(2);
  }
  Tensor out = lookup_out(coords, nl, radius);
  if (!run || out.numel() == 0) return out;
  Tensor co = gpu_f32(coords, "coords", what);
  c10::hip::HIPGuardMasqueradingAsCUDA g(co.device());
  check_status(oflow_corr_lookup_otf_f16(f1h.data_ptr(), ptrs, hs, ws, (int)nl, co.data_ptr<float>(), (int)b, (int)c,
                                         (int)h, (int)w, (int)radius, out.data_ptr<float>(), cur_stream()),
               what);
  return out;
}

Tensor corr_lookup_otf_hip(const Tensor& f1h, const std::vector<Tensor>& f2h, const Tensor& co, int64_t r) {
  return corr_lookup_otf_impl(f1h, f2h, co, r, true);
}
Tensor corr_lookup_otf_meta(const Tensor& f1h, const std::vector<Tensor>& f2h, const Tensor& co, int64_t r) {
  return corr_lookup_otf_impl(f1h, f2h, co, r, false);
}

// ---------------------------------------------------------------- warp / grid_sample
void check_modes(int64_t mode, int64_t pad, const char* what) {
  TORCH_CHECK_VALUE(mode >= 0 && mode <= 2, what, ": interpolation mode ", mode, " is not 0 (bilinear), 1 (nearest) or 2 (bicubic)");
  TORCH_CHECK_VALUE(pad >= 0 && pad <= 2, what, ": padding mode ", pad, " is not 0 (zeros), 1 (border) or 2 (reflection)");
}

void check_warp(const Tensor& fr, const Tensor& fl, const char* what) {
  TORCH_CHECK(fr.dim() == 4 && fl.dim() == 4 && fl.size(1) == 2 && fl.size(0) == fr.size(0) && fl.size(2) == fr.size(2) &&
                  fl.size(3) == fr.size(3),
              what, ": frame ", fr.sizes(), " must be (B, C, H, W) and flow ", fl.sizes(), " (B, 2, H, W)");
  TORCH_CHECK(fr.device() == fl.device(), what, ": frame and flow are on different devices");
}

Tensor grid_warp_hip(const Tensor& frame, const Tensor& flow, int64_t mode, int64_t pad, bool align_corners) {
  const char* what = "warp";
  check_modes(mode, pad, what);
  check_warp(frame, flow, what);
  Tensor fr = gpu_f32(frame, "frame", what), fl = gpu_f32(flow, "flow", what);
  Tensor out = at::empty_like(fr);
  if (out.numel() == 0) return out;
  c10::hip::HIPGuardMasqueradingAsCUDA g(fr.device());
  check_status(oflow_grid_warp_f32(fr.data_ptr<float>(), fl.data_ptr<float>(), (int)fr.size(0), (int)fr.size(1),
                                   (int)fr.size(2), (int)fr.size(3), (int)mode, (int)pad, align_corners ? 1 : 0,
                                   out.data_ptr<float>(), cur_stream()),
               what);
  return out;
}

Tensor grid_warp_meta(const Tensor& frame, const Tensor& flow, int64_t mode, int64_t pad, bool) {
  check_modes(mode, pad, "warp");
  check_warp(frame, flow, "warp");
  return at::empty(frame.sizes(), frame.options().dtype(at::kFloat));
}

void check_sample(const Tensor& x, const Tensor& g, const char* what) {
  TORCH_CHECK(x.dim() == 4 && g.dim() == 4 && g.size(3) == 2 && g.size(0) == x.size(0), what, ": input ", x.sizes(),
              " must be (B, C, H, W) and grid ", g.sizes(), " (B, Ho, Wo, 2)");
  TORCH_CHECK(x.device() == g.device(), what, ": input and grid are on different devices");
}

Tensor grid_sample_hip(const Tensor& input, const Tensor& grid, int64_t mode, int64_t pad, bool align_corners) {
  const char* what = "grid_sample";
  check_modes(mode, pad, what);
  check_sample(input, grid, what);
  Tensor x = gpu_f32(input, "input", what), gr = gpu_f32(grid, "grid", what);
  Tensor out = at::empty({x.size(0), x.size(1), gr.size(1), gr.size(2)}, x.options());
  if (out.numel() == 0) return out;
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  check_status(oflow_grid_sample_f32(x.data_ptr<float>(), gr.data_ptr<float>(), (int)x.size(0), (int)x.size(1),
                                     (int)x.size(2), (int)x.size(3), (int)gr.size(1), (int)gr.size(2), (int)mode,
                                     (int)pad, align_corners ? 1 : 0, out.data_ptr<float>(), cur_stream()),
               what);
  return out;
}

Tensor grid_sample_meta(const Tensor& input, const Tensor& grid, int64_t mode, int64_t pad, bool) {
  check_modes(mode, pad, "grid_sample");
  check_sample(input, grid, "grid_sample");
  return at::empty({input.size(0), input.size(1), grid.size(1), grid.size(2)}, input.options().dtype(at::kFloat));
}

// warp / grid_sample backward (warp_backward.hip): (grad_frame, grad_flow) / (grad_input, grad_grid)
// output_mask (ATen grid_sampler_2d_backward's): an output not wanted is returned as an empty (0-element) tensor and
// the kernel gets a null pointer for it (no zero fill, no atomics for grad_frame)
std::tuple<Tensor, Tensor> grid_warp_backward_impl(const Tensor& gout, const Tensor& frame, const Tensor& flow,
                                                   int64_t mode, int64_t pad, bool ac, std::array<bool, 2> mask, bool run) {
  const char* what = "warp backward";
  check_modes(mode, pad, what);
  check_warp(frame, flow, what);
  TORCH_CHECK(gout.sizes() == frame.sizes(), what, ": grad_out ", gout.sizes(), " must match the frame ", frame.sizes());
  const auto fopt = frame.options().dtype(at::kFloat), lopt = flow.options().dtype(at::kFloat);
  if (!run)
    return {at::empty(mask[0] ? frame.sizes() : at::IntArrayRef{0}, fopt), at::empty(mask[1] ? flow.sizes() : at::IntArrayRef{0}, lopt)};
  Tensor go = gpu_f32(gout, "grad_out", what), fr = gpu_f32(frame, "frame", what), fl = gpu_f32(flow, "flow", what);
  Tensor gfr = mask[0] ? at::zeros_like(fr) : at::empty({0}, fopt), gfl = mask[1] ? at::empty_like(fl) : at::empty({0}, lopt);
  if (fr.numel() == 0) return {gfr, gfl.zero_()};
  if (!mask[0] && !mask[1]) return {gfr, gfl};
  c10::hip::HIPGuardMasqueradingAsCUDA g(fr.device());
  check_status(oflow_grid_warp_backward_f32(go.data_ptr<float>(), fr.data_ptr<float>(), fl.data_ptr<float>(), (int)fr.size(0),
                                            (int)fr.size(1), (int)fr.size(2), (int)fr.size(3), (int)mode, (int)pad, ac ? 1 : 0,
                                            mask[0] ? gfr.data_ptr<float>() : nullptr,
                                            mask[1] ? gfl.data_ptr<float>() : nullptr, cur_stream()),
               what);
  return {gfr, gfl};
}
std::tuple<Tensor, Tensor> grid_warp_backward_hip(const Tensor& go, const Tensor& fr, const Tensor& fl, int64_t m, int64_t p, bool ac,
                                                  std::array<bool, 2> mask) {
  return grid_warp_backward_impl(go, fr, fl, m, p, ac, mask, true);
}
std::tuple<Tensor, Tensor> grid_warp_backward_meta(const Tensor& go, const Tensor& fr, const Tensor& fl, int64_t m, int64_t p, bool ac,
                                                   std::array<bool, 2> mask) {
  return grid_warp_backward_impl(go, fr, fl, m, p, ac, mask, false);
}

std::tuple<Tensor, Tensor> grid_sample_backward_impl(const Tensor& gout, const Tensor& input, const Tensor& grid,
                                                     int64_t mode, int64_t pad, bool ac, std::array<bool, 2> mask, bool run) {
  const char* what = "grid_sample backward";
  check_modes(mode, pad, what);
  check_sample(input, grid, what);
  TORCH_CHECK(gout.dim() == 4 && gout.size(0) == input.size(0) && gout.size(1) == input.size(1) &&
                  gout.size(2) == grid.size(1) && gout.size(3) == grid.size(2),
              what, ": grad_out ", gout.sizes(), " must be (B, C, Ho, Wo)");
  const auto xopt = input.options().dtype(at::kFloat), gopt = grid.options().dtype(at::kFloat);
  if (!run)
    return {at::empty(mask[0] ? input.sizes() : at::IntArrayRef{0}, xopt), at::empty(mask[1] ? grid.sizes() : at::IntArrayRef{0}, gopt)};
  Tensor go = gpu_f32(gout, "grad_out", what), x = gpu_f32(input, "input", what), gr = gpu_f32(grid, "grid", what);
  Tensor gx = mask[0] ? at::zeros_like(x) : at::empty({0}, xopt), gg = mask[1] ? at::empty_like(gr) : at::empty({0}, gopt);
  if (go.numel() == 0) return {gx, gg.zero_()};
  if (!mask[0] && !mask[1]) return {gx, gg};
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  check_status(oflow_grid_sample_backward_f32(go.data_ptr<float>(), x.data_ptr<float>(), gr.data_ptr<float>(), (int)x.size(0),
                                              (int)x.size(1), (int)x.size(2), (int)x.size(3), (int)gr.size(1), (int)gr.size(2),
                                              (int)mode, (int)pad, ac ? 1 : 0, mask[0] ? gx.data_ptr<float>() : nullptr,
                                              mask[1] ? gg.data_ptr<float>() : nullptr, cur_stream()),
               what);
  return {gx, gg};
}
std::tuple<Tensor, Tensor> grid_sample_backward_hip(const Tensor& go, const Tensor& x, const Tensor& gr, int64_t m, int64_t p, bool ac,
                                                    std::array<bool, 2> mask) {
  return grid_sample_backward_impl(go, x, gr, m, p, ac, mask, true);
}
std::tuple<Tensor, Tensor> grid_sample_backward_meta(const Tensor& go, const Tensor& x, const Tensor& gr, int64_t m, int64_t p, bool ac,
                                                     std::array<bool, 2> mask) {
  return grid_sample_backward_impl(go, x, gr, m, p, ac, mask, false);
}

// ---------------------------------------------------------------- backward (training path, §8(f) row 3)
std::vector<Tensor> lookup_backward_impl(const Tensor& grad_out, const Tensor& coords, int64_t radius, int64_t h0,
                                         int64_t w0, int64_t nl, bool run) {
  const char* what = "corr_lookup_backward";
  check_coords(coords, what);
  check_radius(radius, OFLOW_MAX_RADIUS, what);
  const int64_t b = coords.size(0), h = coords.size(2), w = coords.size(3), k = 2 * radius + 1;
  TORCH_CHECK(grad_out.dim() == 4 && grad_out.size(0) == b && grad_out.size(1) == nl * k * k && grad_out.size(2) == h &&
                  grad_out.size(3) == w,
              what, ": grad_out ", grad_out.sizes(), " does not match coords / levels");
  auto d = dims_of(h0, w0, nl, what);
  if (run) TORCH_CHECK(coords.is_cuda(), what, ": coords is on ", coords.device(),
                       "; this MI355X build runs only on ROCm GPU tensors (no CPU fallback)");
  std::vector<Tensor> grads;
  auto opt = coords.options().dtype(at::kFloat);
  for (auto& p : d) grads.push_back(run ? at::zeros({b * h * w, 1, p.first, p.second}, opt)
                                        : at::empty({b * h * w, 1, p.first, p.second}, opt));
  if (!run || b * h * w == 0) return grads;
  Tensor go = gpu_f32(grad_out, "grad_out", what), co = gpu_f32(coords, "coords", what);
  c10::hip::HIPGuardMasqueradingAsCUDA g(co.device());
  float* ptrs[OFLOW_MAX_LEVELS];
  int hs[OFLOW_MAX_LEVELS], ws[OFLOW_MAX_LEVELS];
  for (int64_t l = 0; l < nl; ++l) {
    ptrs[l] = grads[l].data_ptr<float>();
    hs[l] = d[l].first;
    ws[l] = d[l].second;
  }
  check_status(oflow_corr_lookup_backward_f32(go.data_ptr<float>(), co.data_ptr<float>(), (int)b, (int)h, (int)w,
                                              (int)radius, ptrs, hs, ws, (int)nl, cur_stream()),
               what);
  return grads;
}

std::vector<Tensor> lookup_backward_hip(const Tensor& go, const Tensor& co, int64_t r, int64_t h0, int64_t w0,
                                        int64_t nl) {
  return lookup_backward_impl(go, co, r, h0, w0, nl, true);
}
std::vector<Tensor> lookup_backward_meta(const Tensor& go, const Tensor& co, int64_t r, int64_t h0, int64_t w0,
                                         int64_t nl) {
  return lookup_backward_impl(go, co, r, h0, w0, nl, false);
}

// grads[0] += every coarser level's gradient pushed back through the floor 2x2 pools (native kernel), then
// grad_f1 = f2 . G^T / sqrt(C), grad_f2 = f1 . G / sqrt(C) as batched GEMMs on the fp32 matrix cores
// (oflow_corr_fmap_grad_f32, csrc/corr_backward.hip)
std::tuple<Tensor, Tensor> pyramid_backward_impl(const std::vector<Tensor>& level_grads, const Tensor& fmap1,
                                                 const Tensor& fmap2, bool run) {
  const char* what = "corr_pyramid_backward";
  check_fmaps(fmap1, fmap2, what);
  const int64_t b = fmap1.size(0), c = fmap1.size(1), h = fmap1.size(2), w = fmap1.size(3), n = h * w;
  const int64_t nl = (int64_t)level_grads.size();
  auto d = dims_of(h, w, nl, what);
  if (!run) return {at::empty_like(fmap1), at::empty_like(fmap2)};
  std::vector<Tensor> gl;
  for (int64_t l = 0; l < nl; ++l) {
    Tensor t = gpu_f32(level_grads[l], "level gradient", what);
    TORCH_CHECK(t.numel() == b * n * d[l].first * d[l].second, what, ": level ", l, " gradient ", t.sizes(),
                " does not match the pyramid");
    gl.push_back(l == 0 ? t.clone() : t);  // level 0 is accumulated in place
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(fmap1.device());
  if (b * n > 0) {
    float* ptrs[OFLOW_MAX_LEVELS];
    int hs[OFLOW_MAX_LEVELS], ws[OFLOW_MAX_LEVELS];
    for (int64_t l = 0; l < nl; ++l) {
      ptrs[l] = gl[l].data_ptr<float>();
      hs[l] = d[l].first;
      ws[l] = d[l].second;
    }
    check_status(oflow_corr_pyramid_grad_combine_f32(ptrs, hs, ws, (int)nl, b * n, cur_stream()), what);
  }
  // the fmap gradients on the fp32 matrix cores (corr_backward.hip): scale as the forward, 1/sqrt(float(C))
  const float s = 1.0f / std::sqrt(static_cast<float>(c));
  Tensor f1m = fmap1.to(at::kFloat).contiguous(), f2m = fmap2.to(at::kFloat).contiguous();
  Tensor g1 = at::empty({b, c, h, w}, f1m.options()), g2 = at::empty({b, c, h, w}, f2m.options());
  check_status(oflow_corr_fmap_grad_f32(f1m.data_ptr<float>(), f2m.data_ptr<float>(), gl[0].data_ptr<float>(), (int)b,
                                        (int)c, (int)n, s, g1.data_ptr<float>(), g2.data_ptr<float>(), cur_stream()),
               what);
  return {g1.to(fmap1.scalar_type()), g2.to(fmap2.scalar_type())};
}

std::tuple<Tensor, Tensor> pyramid_backward_hip(const std::vector<Tensor>& g, const Tensor& f1, const Tensor& f2) {
  return pyramid_backward_impl(g, f1, f2, true);
}
std::tuple<Tensor, Tensor> pyramid_backward_meta(const std::vector<Tensor>& g, const Tensor& f1, const Tensor& f2) {
  return pyramid_backward_impl(g, f1, f2, false);
}

}  // namespace

TORCH_LIBRARY(oflow, m) {
  m.def("corr_pyramid(Tensor fmap1, Tensor fmap2, int num_levels) -> Tensor[]");
  m.def("corr_pyramid_tiled(Tensor fmap1, Tensor fmap2, int num_levels) -> Tensor[]");
  m.def("corr_lookup(Tensor[] levels, Tensor coords, int radius) -> Tensor");
  m.def("corr_lookup_tiled(Tensor[] levels, Tensor coords, int radius) -> Tensor");
  m.def("corr_lookup_tiled_nhwc(Tensor[] levels, Tensor coords, int radius, Tensor(a!) out) -> ()");
  m.def("corr_otf_prepare(Tensor fmap1, Tensor fmap2, int num_levels) -> (Tensor, Tensor[])");
  m.def("corr_lookup_otf(Tensor f1h, Tensor[] f2h, Tensor coords, int radius) -> Tensor");
  m.def("grid_warp(Tensor frame, Tensor flow, int mode, int padding_mode, bool align_corners) -> Tensor");
  m.def("grid_sample(Tensor input, Tensor grid, int mode, int padding_mode, bool align_corners) -> Tensor");
  m.def("corr_lookup_backward(Tensor grad_out, Tensor coords, int radius, int H, int W, int num_levels) -> Tensor[]");
  m.def("corr_pyramid_backward(Tensor[] level_grads, Tensor fmap1, Tensor fmap2) -> (Tensor, Tensor)");
  m.def("grid_warp_backward(Tensor grad_out, Tensor frame, Tensor flow, int mode, int padding_mode, bool align_corners, bool[2] output_mask) -> (Tensor, Tensor)");
  m.def("grid_sample_backward(Tensor grad_out, Tensor input, Tensor grid, int mode, int padding_mode, bool align_corners, bool[2] output_mask) -> (Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(oflow, CUDA, m) {
  m.impl("corr_pyramid", &corr_pyramid_hip);
  m.impl("corr_pyramid_tiled", &corr_pyramid_tiled_hip);
  m.impl("corr_lookup", &corr_lookup_hip);
  m.impl("corr_lookup_tiled", &corr_lookup_tiled_hip);
  m.impl("corr_lookup_tiled_nhwc", &corr_lookup_tiled_nhwc_hip);
  m.impl("corr_otf_prepare", &otf_prepare_hip);
  m.impl("corr_lookup_otf", &corr_lookup_otf_hip);
  m.impl("grid_warp", &grid_warp_hip);
  m.impl("grid_sample", &grid_sample_hip);
  m.impl("corr_lookup_backward", &lookup_backward_hip);
  m.impl("corr_pyramid_backward", &pyramid_backward_hip);
  m.impl("grid_warp_backward", &grid_warp_backward_hip);
  m.impl("grid_sample_backward", &grid_sample_backward_hip);
}

// CPU tensors reach the same kernels, whose first check raises "no CPU fallback" (there is no CPU path)
TORCH_LIBRARY_IMPL(oflow, CPU, m) {
  m.impl("corr_pyramid", &corr_pyramid_hip);
  m.impl("corr_pyramid_tiled", &corr_pyramid_tiled_hip);
  m.impl("corr_lookup", &corr_lookup_hip);
  m.impl("corr_lookup_tiled", &corr_lookup_tiled_hip);
  m.impl("corr_lookup_tiled_nhwc", &corr_lookup_tiled_nhwc_hip);
  m.impl("corr_otf_prepare", &otf_prepare_hip);
  m.impl("corr_lookup_otf", &corr_lookup_otf_hip);
  m.impl("grid_warp", &grid_warp_hip);
  m.impl("grid_sample", &grid_sample_hip);
  m.impl("corr_lookup_backward", &lookup_backward_hip);
  m.impl("corr_pyramid_backward", &pyramid_backward_hip);
  m.impl("grid_warp_backward", &grid_warp_backward_hip);
  m.impl("grid_sample_backward", &grid_sample_backward_hip);
}

TORCH_LIBRARY_IMPL(oflow, Meta, m) {
  m.impl("corr_pyramid", &corr_pyramid_meta);
  m.impl("corr_pyramid_tiled", &corr_pyramid_tiled_meta);
  m.impl("corr_lookup", &corr_lookup_meta);
  m.impl("corr_lookup_tiled", &corr_lookup_meta);
  m.impl("corr_lookup_tiled_nhwc", &corr_lookup_tiled_nhwc_meta);
  m.impl("corr_otf_prepare", &otf_prepare_meta);
  m.impl("corr_lookup_otf", &corr_lookup_otf_meta);
  m.impl("grid_warp", &grid_warp_meta);
  m.impl("grid_sample", &grid_sample_meta);
  m.impl("corr_lookup_backward", &lookup_backward_meta);
  m.impl("corr_pyramid_backward", &pyramid_backward_meta);
  m.impl("grid_warp_backward", &grid_warp_backward_meta);
  m.impl("grid_sample_backward", &grid_sample_backward_meta);
}
