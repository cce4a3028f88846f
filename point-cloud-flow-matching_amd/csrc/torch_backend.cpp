// _pvcnn_backend as a torch C++ extension over the C ABI (include/pcfm.h).
//
// The reference builds its PVCNN backend with torch.utils.cpp_extension.load
// (third_party/pvcnn/modules/functional/backend.py:6-24) and binds 12 functions
// (src/bindings.cpp:10-44).  This module exports the same 12 names with the
// same arguments and return values; the seven the flow model uses call the
// gfx950 kernels of libpcfm_hip.so on torch's current HIP stream, the five
// PointNet++ operators outside this build's hot path raise (as
// pcfm.ops.backend does).  Tensors must be HIP tensors:
// the CPU backend of config 1 is pcfm.cpu_ops, reached through the default
// ctypes binding (modules/functional/backend.py), never from here.
//
// Built by g++ against torch's headers (no hipify, no device code here):
// csrc/build_torch_backend.py, run by __graft_entry__.build().
#include <torch/extension.h>

#include <c10/hip/HIPStream.h>

#include <initializer_list>
#include <string>
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

// vox.cpp:17-43
std::vector<at::Tensor> avg_voxelize_forward(const at::Tensor& features, const at::Tensor& coords,
                                             const int resolution) {
  check_hip(features, "features", at::kFloat);
  check_hip(coords, "coords", at::kInt);
  check_shape(features, "features", {-1, -1, -1});
  check_shape(coords, "coords", {features.size(0), 3, features.size(2)});
  check_same_device(features, coords, "coords");
  TORCH_CHECK(resolution > 0 && resolution <= 1024, "resolution must be in [1, 1024]");
  const int b = features.size(0), c = features.size(1), n = features.size(2);
  const int r = resolution, s = r * r * r;
  auto out = at::empty({b, c, s}, features.options());
  auto ind = at::empty({b, n}, coords.options());
  auto cnt = at::empty({b, s}, coords.options());
  auto ws = workspace(pcfm_avg_voxelize_fwd_workspace_bytes(b, c, n, r), features);
  check_rc(pcfm_avg_voxelize_fwd(features.data_ptr<float>(), coords.data_ptr<int>(), b, c, n, r,
                                 out.data_ptr<float>(), ind.data_ptr<int>(), cnt.data_ptr<int>(),
                                 ws.data_ptr(), (size_t)ws.numel(), stream_of(features)),
           "avg_voxelize_forward");
  return {out, ind, cnt};
}

// vox.cpp:54-76
at::Tensor avg_voxelize_backward(const at::Tensor& grad_y, const at::Tensor& indices,
                                 const at::Tensor& cnt) {
  check_hip(grad_y, "grad_y", at::kFloat);
  check_hip(indices, "indices", at::kInt);
  check_hip(cnt, "cnt", at::kInt);
  check_shape(grad_y, "grad_y", {-1, -1, -1});
  check_shape(indices, "indices", {grad_y.size(0), -1});
  check_shape(cnt, "cnt", {grad_y.size(0), grad_y.size(2)});
  check_same_device(grad_y, indices, "indices");
  check_same_device(grad_y, cnt, "cnt");
  const int b = grad_y.size(0), c = grad_y.size(1), s = grad_y.size(2);
  const int n = indices.size(1);
  auto grad_x = at::empty({b, c, n}, grad_y.options());
  check_rc(pcfm_avg_voxelize_bwd(grad_y.data_ptr<float>(), indices.data_ptr<int>(),
                                 cnt.data_ptr<int>(), b, c, n, s, grad_x.data_ptr<float>(),
                                 stream_of(grad_y)),
           "avg_voxelize_backward");
  return grad_x;
}

// trilinear_devox.cpp:18-55
std::vector<at::Tensor> trilinear_devoxelize_forward(const int r, const bool is_training,
                                                     const at::Tensor& coords,
                                                     const at::Tensor& features) {
  check_hip(features, "features", at::kFloat);
  check_hip(coords, "coords", at::kFloat);
  TORCH_CHECK(r > 0 && r <= 1024, "r must be in [1, 1024]");
  check_shape(features, "features", {-1, -1, (int64_t)r * r * r});
  check_shape(coords, "coords", {features.size(0), 3, -1});
  check_same_device(features, coords, "coords");
  const int b = features.size(0), c = features.size(1), n = coords.size(2);
  auto outs = at::empty({b, c, n}, features.options());
  at::Tensor inds, wgts;
  if (is_training) {
    inds = at::empty({b, 8, n}, features.options().dtype(at::kInt));
    wgts = at::empty({b, 8, n}, features.options());
  } else {
    inds = at::zeros({1}, features.options().dtype(at::kInt));
    wgts = at::zeros({1}, features.options());
  }
  check_rc(pcfm_trilinear_devoxelize_fwd(coords.data_ptr<float>(), features.data_ptr<float>(), b,
                                         c, n, r, is_training ? 1 : 0, outs.data_ptr<float>(),
                                         is_training ? inds.data_ptr<int>() : nullptr,
                                         is_training ? wgts.data_ptr<float>() : nullptr,
                                         stream_of(features)),
           "trilinear_devoxelize_forward");
  return {outs, inds, wgts};
}

// trilinear_devox.cpp:67-91
at::Tensor trilinear_devoxelize_backward(const at::Tensor& grad_y, const at::Tensor& indices,
                                         const at::Tensor& weights, const int r) {
  check_hip(grad_y, "grad_y", at::kFloat);
  check_hip(indices, "indices", at::kInt);
  check_hip(weights, "weights", at::kFloat);
  TORCH_CHECK(r > 0 && r <= 1024, "r must be in [1, 1024]");
  check_shape(grad_y, "grad_y", {-1, -1, -1});
  check_shape(indices, "indices", {grad_y.size(0), 8, grad_y.size(2)});
  check_shape(weights, "weights", {grad_y.size(0), 8, grad_y.size(2)});
  check_same_device(grad_y, indices, "indices");
  check_same_device(grad_y, weights, "weights");
  const int b = grad_y.size(0), c = grad_y.size(1), n = grad_y.size(2);
  auto grad_x = at::empty({b, c, (int64_t)r * r * r}, grad_y.options());
  auto ws = workspace(pcfm_trilinear_devoxelize_bwd_workspace_bytes(b, c, n, r), grad_y);
  check_rc(pcfm_trilinear_devoxelize_bwd(grad_y.data_ptr<float>(), indices.data_ptr<int>(),
                                         weights.data_ptr<float>(), b, c, n, r,
                                         grad_x.data_ptr<float>(), ws.data_ptr(),
                                         (size_t)ws.numel(), stream_of(grad_y)),
           "trilinear_devoxelize_backward");
  return grad_x;
}

// ball_query.cpp:6-30
at::Tensor ball_query(const at::Tensor& centers_coords, const at::Tensor& points_coords,
                      const float radius, const int num_neighbors) {
  check_hip(centers_coords, "centers_coords", at::kFloat);
  check_hip(points_coords, "points_coords", at::kFloat);
  check_shape(centers_coords, "centers_coords", {-1, 3, -1});
  check_shape(points_coords, "points_coords", {centers_coords.size(0), 3, -1});
  check_same_device(centers_coords, points_coords, "points_coords");
  TORCH_CHECK(num_neighbors >= 0, "num_neighbors must be >= 0");
  const int b = centers_coords.size(0), m = centers_coords.size(2), n = points_coords.size(2);
  auto idx = at::zeros({b, m, num_neighbors}, centers_coords.options().dtype(at::kInt));
  check_rc(pcfm_ball_query(centers_coords.data_ptr<float>(), points_coords.data_ptr<float>(), b,
                           m, n, radius, num_neighbors, idx.data_ptr<int>(),
                           stream_of(centers_coords)),
           "ball_query");
  return idx;
}

// grouping.cpp:6-22
at::Tensor grouping_forward(const at::Tensor& features, const at::Tensor& indices) {
  check_hip(features, "features", at::kFloat);
  check_hip(indices, "indices", at::kInt);
  check_shape(features, "features", {-1, -1, -1});
  check_shape(indices, "indices", {features.size(0), -1, -1});
  check_same_device(features, indices, "indices");
  const int b = features.size(0), c = features.size(1), n = features.size(2);
  const int m = indices.size(1), u = indices.size(2);
  auto out = at::empty({b, c, m, u}, features.options());
  check_rc(pcfm_grouping_fwd(features.data_ptr<float>(), indices.data_ptr<int>(), b, c, n, m, u,
                             out.data_ptr<float>(), stream_of(features)),
           "grouping_forward");
  return out;
}

// grouping.cpp:24-44
at::Tensor grouping_backward(const at::Tensor& grad_y, const at::Tensor& indices, const int n) {
  check_hip(grad_y, "grad_y", at::kFloat);
  check_hip(indices, "indices", at::kInt);
  check_shape(grad_y, "grad_y", {-1, -1, -1, -1});
  check_shape(indices, "indices", {grad_y.size(0), grad_y.size(2), grad_y.size(3)});
  check_same_device(grad_y, indices, "indices");
  TORCH_CHECK(n >= 0, "n must be >= 0");
  const int b = grad_y.size(0), c = grad_y.size(1);
  const int m = indices.size(1), u = indices.size(2);
  auto grad_x = at::empty({b, c, n}, grad_y.options());
  auto ws = workspace(pcfm_grouping_bwd_workspace_bytes(b, c, n, m, u), grad_y);
  check_rc(pcfm_grouping_bwd(grad_y.data_ptr<float>(), indices.data_ptr<int>(), b, c, n, m, u,
                             grad_x.data_ptr<float>(), ws.data_ptr(), (size_t)ws.numel(),
                             stream_of(grad_y)),
           "grouping_backward");
  return grad_x;
}

[[noreturn]] void out_of_scope(const char* name) {
  TORCH_CHECK(false, "_pvcnn_backend.", name,
              ": PointNet++ operator outside this build's hot path (SURVEY.md section 2.2: "
              "FPS / gather / 3-NN are used only by PointNet SA/FP modules, which the flow "
              "model never calls)");
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.def("gather_features_forward",
        [](const at::Tensor&, const at::Tensor&) -> at::Tensor {
          out_of_scope("gather_features_forward");
        });
  m.def("gather_features_backward",
        [](const at::Tensor&, const at::Tensor&, const int) -> at::Tensor {
          out_of_scope("gather_features_backward");
        });
  m.def("furthest_point_sampling",
        [](const at::Tensor&, const int) -> at::Tensor { out_of_scope("furthest_point_sampling"); });
  m.def("ball_query", &ball_query, "Ball Query (gfx950)");
  m.def("grouping_forward", &grouping_forward, "Grouping Features forward (gfx950)");
  m.def("grouping_backward", &grouping_backward, "Grouping Features backward (gfx950)");
  m.def("three_nearest_neighbors_interpolate_forward",
        [](const at::Tensor&, const at::Tensor&, const at::Tensor&) -> std::vector<at::Tensor> {
          out_of_scope("three_nearest_neighbors_interpolate_forward");
        });
  m.def("three_nearest_neighbors_interpolate_backward",
        [](const at::Tensor&, const at::Tensor&, const at::Tensor&, const int) -> at::Tensor {
          out_of_scope("three_nearest_neighbors_interpolate_backward");
        });
  m.def("trilinear_devoxelize_forward", &trilinear_devoxelize_forward,
        "Trilinear Devoxelization forward (gfx950)");
  m.def("trilinear_devoxelize_backward", &trilinear_devoxelize_backward,
        "Trilinear Devoxelization backward (gfx950)");
  m.def("avg_voxelize_forward", &avg_voxelize_forward,
        "Voxelization forward with average pooling (gfx950)");
  m.def("avg_voxelize_backward", &avg_voxelize_backward, "Voxelization backward (gfx950)");
}
