// chamfer_3D and emd_cuda / emd_ext as torch C++ extensions over the C ABI
// (include/pcfm.h), one source (-DPCFM_TORCH_MODULE=1: chamfer, 2: EMD; the EMD
// module is built under both names: the reference's setup.py and backend.py
// build `emd_ext`, PyTorchEMD/setup.py:26-29 and backend.py:11-12, and emd.py
// imports it as emd_cuda).
//
// chamfer_3D replaces third_party/ChamferDistancePytorch/chamfer3D/chamfer_cuda.cpp:17-32
// (forward / backward into caller-allocated tensors, int status: 1 ok, 0 after
// printing the error, as chamfer3D.cu:145-151 / :219-225); emd_cuda replaces
// third_party/PyTorchEMD/cuda/emd.cpp:8-27 (approxmatch_forward, matchcost_forward,
// matchcost_backward; float and double).  HIP tensors only: the CPU backend of
// config 1 is pcfm.cpu_ops through the default ctypes bindings (pcfm.ops).
// Built by csrc/build_torch_backend.py with plain g++ (no device code here).
#include <torch/extension.h>

#include <c10/hip/HIPStream.h>

#include <cstdio>
#include <initializer_list>
#include <vector>

#include "../../include/pcfm.h"

namespace {

void* stream_of(const at::Tensor& t) {
  return (void*)c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

void check_hip(const at::Tensor& t, const char* name, at::ScalarType dt) {
  TORCH_CHECK(t.is_cuda(), name, " must be a HIP tensor (the CPU backend is pcfm.cpu_ops)");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(t.scalar_type() == dt, name, " has the wrong dtype");
}

void check_rc(int rc, const char* op) {
  TORCH_CHECK(rc == PCFM_OK, op, " failed (", rc, "): ", pcfm_last_error());
}

// shape and device checks matching pcfm.ops' (a caller mistake is a
// TORCH_CHECK error, never an out-of-bounds kernel access)
void check_shape(const at::Tensor& t, const char* name, std::initializer_list<int64_t> shape) {
  TORCH_CHECK(t.dim() == (int64_t)shape.size(), name, " must have ", shape.size(),
              " dimensions, got ", t.sizes());
  int64_t d = 0;
  for (int64_t want : shape) {
    TORCH_CHECK(want < 0 || t.size(d) == want, name, " has shape ", t.sizes(), ": dimension ", d,
                " must be ", want);
    ++d;
  }
}

void check_same_device(const at::Tensor& a, const at::Tensor& b, const char* name) {
  TORCH_CHECK(a.device() == b.device(), name, " is on ", b.device(), ", expected ", a.device());
}

at::Tensor workspace(size_t bytes, const at::Tensor& like) {
  return at::empty({(int64_t)std::max<size_t>(bytes, 1)}, like.options().dtype(at::kByte));
}

#if PCFM_TORCH_MODULE == 1
// chamfer_cuda.cpp:17-24
int chamfer_forward(at::Tensor xyz1, at::Tensor xyz2, at::Tensor dist1, at::Tensor dist2,
                    at::Tensor idx1, at::Tensor idx2) {
  try {
    check_hip(xyz1, "xyz1", at::kFloat);
    check_hip(xyz2, "xyz2", at::kFloat);
    check_hip(dist1, "dist1", at::kFloat);
    check_hip(dist2, "dist2", at::kFloat);
    check_hip(idx1, "idx1", at::kInt);
    check_hip(idx2, "idx2", at::kInt);
    check_shape(xyz1, "xyz1", {-1, -1, 3});
    const int64_t B = xyz1.size(0), N = xyz1.size(1);
    check_shape(xyz2, "xyz2", {B, -1, 3});
    const int64_t M = xyz2.size(1);
    check_shape(dist1, "dist1", {B, N});
    check_shape(dist2, "dist2", {B, M});
    check_shape(idx1, "idx1", {B, N});
    check_shape(idx2, "idx2", {B, M});
    for (const at::Tensor* t : {&xyz2, &dist1, &dist2, &idx1, &idx2})
      check_same_device(xyz1, *t, "an output or xyz2");
    const int b = xyz1.size(0), n = xyz1.size(1), m = xyz2.size(1);
    auto ws = workspace(pcfm_chamfer_workspace_bytes(b, n, m), xyz1);
    check_rc(pcfm_chamfer_fwd(xyz1.data_ptr<float>(), xyz2.data_ptr<float>(), b, n, m,
                              dist1.data_ptr<float>(), dist2.data_ptr<float>(),
                              idx1.data_ptr<int>(), idx2.data_ptr<int>(), ws.data_ptr(),
                              (size_t)ws.numel(), stream_of(xyz1)),
             "chamfer forward");
  } catch (const c10::Error& e) {
    std::printf("error in nnd updateOutput: %s\n", e.what_without_backtrace());
    return 0;
  }
  return 1;
}

// chamfer_cuda.cpp:26-32
int chamfer_backward(at::Tensor xyz1, at::Tensor xyz2, at::Tensor gradxyz1, at::Tensor gradxyz2,
                     at::Tensor graddist1, at::Tensor graddist2, at::Tensor idx1,
                     at::Tensor idx2) {
  try {
    check_hip(xyz1, "xyz1", at::kFloat);
    check_hip(xyz2, "xyz2", at::kFloat);
    check_hip(gradxyz1, "gradxyz1", at::kFloat);
    check_hip(gradxyz2, "gradxyz2", at::kFloat);
    check_hip(graddist1, "graddist1", at::kFloat);
    check_hip(graddist2, "graddist2", at::kFloat);
    check_hip(idx1, "idx1", at::kInt);
    check_hip(idx2, "idx2", at::kInt);
    check_shape(xyz1, "xyz1", {-1, -1, 3});
    const int64_t B = xyz1.size(0), N = xyz1.size(1);
    check_shape(xyz2, "xyz2", {B, -1, 3});
    const int64_t M = xyz2.size(1);
    check_shape(gradxyz1, "gradxyz1", {B, N, 3});
    check_shape(gradxyz2, "gradxyz2", {B, M, 3});
    check_shape(graddist1, "graddist1", {B, N});
    check_shape(graddist2, "graddist2", {B, M});
    check_shape(idx1, "idx1", {B, N});
    check_shape(idx2, "idx2", {B, M});
    for (const at::Tensor* t : {&xyz2, &gradxyz1, &gradxyz2, &graddist1, &graddist2, &idx1, &idx2})
      check_same_device(xyz1, *t, "a gradient, index or xyz2");
    const int b = xyz1.size(0), n = xyz1.size(1), m = xyz2.size(1);
    check_rc(pcfm_chamfer_bwd(xyz1.data_ptr<float>(), xyz2.data_ptr<float>(), b, n, m,
                              graddist1.data_ptr<float>(), graddist2.data_ptr<float>(),
                              idx1.data_ptr<int>(), idx2.data_ptr<int>(),
                              gradxyz1.data_ptr<float>(), gradxyz2.data_ptr<float>(),
                              stream_of(xyz1)),
             "chamfer backward");
  } catch (const c10::Error& e) {
    std::printf("error in nnd get grad: %s\n", e.what_without_backtrace());
    return 0;
  }
  return 1;
}
#else
void emd_check(const at::Tensor& xyz1, const at::Tensor& xyz2) {
  TORCH_CHECK(xyz1.is_cuda() && xyz2.is_cuda(), "emd: HIP tensors expected");
  TORCH_CHECK(xyz1.dim() == 3 && xyz2.dim() == 3 && xyz1.size(0) == xyz2.size(0) &&
                  xyz1.size(2) == 3 && xyz2.size(2) == 3,
              "emd: expected (B,N,3) and (B,M,3)");
  TORCH_CHECK((xyz1.scalar_type() == at::kFloat || xyz1.scalar_type() == at::kDouble) &&
                  xyz2.scalar_type() == xyz1.scalar_type(),
              "emd: xyz1/xyz2 must both be float32 or both float64");
  check_same_device(xyz1, xyz2, "xyz2");
}

// match (B, M, N) of the same dtype and device as the points
void emd_check_match(const at::Tensor& xyz1, const at::Tensor& xyz2, const at::Tensor& match) {
  check_shape(match, "match", {xyz1.size(0), xyz2.size(1), xyz1.size(1)});
  TORCH_CHECK(match.scalar_type() == xyz1.scalar_type(), "emd: match must have the points' dtype");
  check_same_device(xyz1, match, "match");
}

at::Tensor emd_ws(const at::Tensor& xyz1, int b, int n, int m) {
  return workspace(pcfm_emd_workspace_bytes(b, n, m, (int)xyz1.element_size()), xyz1);
}

// emd_kernel.cu:169-191
at::Tensor approxmatch_forward(const at::Tensor& xyz1_, const at::Tensor& xyz2_) {
  const at::Tensor xyz1 = xyz1_.contiguous(), xyz2 = xyz2_.contiguous();
  emd_check(xyz1, xyz2);
  const int b = xyz1.size(0), n = xyz1.size(1), m = xyz2.size(1);
  auto match = at::empty({b, m, n}, xyz1.options());
  if (n == 0 || m == 0) return match.zero_();
  auto ws = emd_ws(xyz1, b, n, m);
  if (xyz1.scalar_type() == at::kFloat)
    check_rc(pcfm_emd_approxmatch_f32(xyz1.data_ptr<float>(), xyz2.data_ptr<float>(), b, n, m,
                                      match.data_ptr<float>(), ws.data_ptr(), (size_t)ws.numel(),
                                      stream_of(xyz1)),
             "approxmatch_forward");
  else
    check_rc(pcfm_emd_approxmatch_f64(xyz1.data_ptr<double>(), xyz2.data_ptr<double>(), b, n, m,
                                      match.data_ptr<double>(), ws.data_ptr(),
                                      (size_t)ws.numel(), stream_of(xyz1)),
             "approxmatch_forward");
  return match;
}

// emd_kernel.cu:255-277
at::Tensor matchcost_forward(const at::Tensor& xyz1_, const at::Tensor& xyz2_,
                             const at::Tensor& match_) {
  const at::Tensor xyz1 = xyz1_.contiguous(), xyz2 = xyz2_.contiguous(),
                   match = match_.contiguous();
  emd_check(xyz1, xyz2);
  emd_check_match(xyz1, xyz2, match);
  const int b = xyz1.size(0), n = xyz1.size(1), m = xyz2.size(1);
  auto cost = at::empty({b}, xyz1.options());
  auto ws = emd_ws(xyz1, b, n, m);
  if (xyz1.scalar_type() == at::kFloat)
    check_rc(pcfm_emd_matchcost_f32(xyz1.data_ptr<float>(), xyz2.data_ptr<float>(),
                                    match.data_ptr<float>(), b, n, m, cost.data_ptr<float>(),
                                    ws.data_ptr(), (size_t)ws.numel(), stream_of(xyz1)),
             "matchcost_forward");
  else
    check_rc(pcfm_emd_matchcost_f64(xyz1.data_ptr<double>(), xyz2.data_ptr<double>(),
                                    match.data_ptr<double>(), b, n, m, cost.data_ptr<double>(),
                                    ws.data_ptr(), (size_t)ws.numel(), stream_of(xyz1)),
             "matchcost_forward");
  return cost;
}

// emd_kernel.cu:371-396
std::vector<at::Tensor> matchcost_backward(const at::Tensor& grad_cost_, const at::Tensor& xyz1_,
                                           const at::Tensor& xyz2_, const at::Tensor& match_) {
  const at::Tensor xyz1 = xyz1_.contiguous(), xyz2 = xyz2_.contiguous(),
                   match = match_.contiguous();
  emd_check(xyz1, xyz2);
  emd_check_match(xyz1, xyz2, match);
  check_shape(grad_cost_, "grad_cost", {xyz1.size(0)});
  check_same_device(xyz1, grad_cost_, "grad_cost");
  const at::Tensor grad_cost = grad_cost_.contiguous().to(xyz1.scalar_type());
  const int b = xyz1.size(0), n = xyz1.size(1), m = xyz2.size(1);
  auto g1 = at::empty({b, n, 3}, xyz1.options());
  auto g2 = at::empty({b, m, 3}, xyz1.options());
  auto ws = emd_ws(xyz1, b, n, m);
  if (xyz1.scalar_type() == at::kFloat)
    check_rc(pcfm_emd_matchcost_bwd_f32(grad_cost.data_ptr<float>(), xyz1.data_ptr<float>(),
                                        xyz2.data_ptr<float>(), match.data_ptr<float>(), b, n, m,
                                        g1.data_ptr<float>(), g2.data_ptr<float>(), ws.data_ptr(),
                                        (size_t)ws.numel(), stream_of(xyz1)),
             "matchcost_backward");
  else
    check_rc(pcfm_emd_matchcost_bwd_f64(grad_cost.data_ptr<double>(), xyz1.data_ptr<double>(),
                                        xyz2.data_ptr<double>(), match.data_ptr<double>(), b, n,
                                        m, g1.data_ptr<double>(), g2.data_ptr<double>(),
                                        ws.data_ptr(), (size_t)ws.numel(), stream_of(xyz1)),
             "matchcost_backward");
  return {g1, g2};
}
#endif

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
#if PCFM_TORCH_MODULE == 1
  m.def("forward", &chamfer_forward, "chamfer forward (gfx950)");
  m.def("backward", &chamfer_backward, "chamfer backward (gfx950)");
#else
  m.def("approxmatch_forward", &approxmatch_forward, "ApproxMatch forward (gfx950)");
  m.def("matchcost_forward", &matchcost_forward, "MatchCost forward (gfx950)");
  m.def("matchcost_backward", &matchcost_backward, "MatchCost backward (gfx950)");
#endif
}
