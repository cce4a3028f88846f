// Store-pattern probe (dev tool): how fast can the pointwise GEMM's output tile
// (256 channel rows x 128 points of a (B, C, N) fp32 tensor, N = 20000, rows
// 80 KB apart) be written, by pattern?  Each kernel writes the same 164 MB.
//   acc32   : the 32x32 MFMA accumulator layout as pw_gemm256 stores it -- per
//             store instruction two 128-B row segments (lanes 0-31 / 32-63)
//   row4    : the same tile, each wave-instruction 64 float4 = two 512-B rows
//   quad4   : the accumulator after a 4x4 lane transpose: float4 per lane, each
//             instruction eight 128-B row segments (4x fewer instructions
//             than acc32, the same 128-B pieces)
//   seq4    : the same bytes as one contiguous float4 stream
// hipcc --offload-arch=gfx950 -O3 tools/store_probe.hip -o tools/store_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int B = 8, C = 256, N = 20000, TM = 256, TN = 128;

template <bool NT>
__device__ __forceinline__ void st1(float* p, float v) {
  if (NT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

template <bool NT>
__global__ void __launch_bounds__(512) acc32(float* __restrict__ y, float val) {
  const int b = blockIdx.z, m0 = blockIdx.y * TM, p0 = blockIdx.x * TN;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w >> 1, wc = w & 1, r = lane & 31, h = lane >> 5;
  const int pw0 = p0 + wc * 64;
  for (int i = 0; i < 2; ++i) {
    const int mg = m0 + wr * 64 + i * 32;
    float* yr = y + ((size_t)b * C + mg) * N;
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int dm = (e & 3) + 8 * (e >> 2) + 4 * h;
        const int p = pw0 + j * 32 + r;
        if (p < N) st1<NT>(yr + (size_t)dm * N + p, val + e);
      }
  }
}

template <bool NT>
__global__ void __launch_bounds__(512) row4(float* __restrict__ y, float val) {
  const int b = blockIdx.z, m0 = blockIdx.y * TM, p0 = blockIdx.x * TN;
  const int t = threadIdx.x;
  // 256 rows x 32 float4; thread t: float4 (t & 31) of rows (t >> 5) + 16 k
  const int q = t & 31, r0 = t >> 5;
  const int p = p0 + 4 * q;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int m = m0 + r0 + 16 * k;
    float4* dst = reinterpret_cast<float4*>(y + ((size_t)b * C + m) * N + p);
    const float4 v = make_float4(val, val + 1, val + 2, val + k);
    if (p + 3 < N) {
      if (NT) {
        typedef float v4f __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(v4f{v.x, v.y, v.z, v.w}, reinterpret_cast<v4f*>(dst));
      } else {
        *dst = v;
      }
    }
  }
}

template <bool NT>
__global__ void __launch_bounds__(512) quad4(float* __restrict__ y, float val) {
  const int b = blockIdx.z, m0 = blockIdx.y * TM, p0 = blockIdx.x * TN;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w >> 1, wc = w & 1, r = lane & 31, h = lane >> 5;
  const int pw0 = p0 + wc * 64;
  for (int i = 0; i < 2; ++i) {
    const int mg = m0 + wr * 64 + i * 32;
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = mg + 8 * q + (r & 3) + 4 * h;
        const int p = pw0 + j * 32 + (r & ~3);
        float4* dst = reinterpret_cast<float4*>(y + ((size_t)b * C + row) * N + p);
        if (p + 3 < N) {
          typedef float v4f __attribute__((ext_vector_type(4)));
          const v4f v{val, val + 1, val + 2, val + q};
          if (NT)
            __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(dst));
          else
            *reinterpret_cast<v4f*>(dst) = v;
        }
      }
  }
}

__global__ void __launch_bounds__(256) seq4(float4* __restrict__ y, size_t n4, float val) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
    y[i] = make_float4(val, val, val, val);
}

int main() {
  const size_t n = (size_t)B * C * N;
  float* y;
  if (hipMalloc(&y, n * sizeof(float)) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const dim3 grid((N + TN - 1) / TN, C / TM, B);
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    hipDeviceSynchronize();
    const int iters = 20;
    hipEventRecord(e0);
    for (int i = 0; i < iters; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / iters;
    printf("{\"pattern\": \"%s\", \"us\": %.2f, \"TBps\": %.3f}\n", name, us,
           n * 4.0 / (us * 1e-6) / 1e12);
  };
  run("acc32_nt", [&] { hipLaunchKernelGGL(acc32<true>, grid, dim3(512), 0, 0, y, 1.0f); });
  run("acc32_plain", [&] { hipLaunchKernelGGL(acc32<false>, grid, dim3(512), 0, 0, y, 1.0f); });
  run("row4_nt", [&] { hipLaunchKernelGGL(row4<true>, grid, dim3(512), 0, 0, y, 1.0f); });
  run("row4_plain", [&] { hipLaunchKernelGGL(row4<false>, grid, dim3(512), 0, 0, y, 1.0f); });
  run("quad4_nt", [&] { hipLaunchKernelGGL(quad4<true>, grid, dim3(512), 0, 0, y, 1.0f); });
  run("quad4_plain", [&] { hipLaunchKernelGGL(quad4<false>, grid, dim3(512), 0, 0, y, 1.0f); });
  run("seq4", [&] {
    hipLaunchKernelGGL(seq4, dim3(4096), dim3(256), 0, 0, reinterpret_cast<float4*>(y), n / 4,
                       1.0f);
  });
  hipFree(y);
  return 0;
}
