// Stable segment sort of the PVConv scatters (segsum.hpp step 1) on rocPRIM's
// device radix sort.
//
// Items (b, i) are sorted by the composite key b * (V + 1) + key, where keys
// outside [0, V) become the batch's sentinel V (sorted after its valid keys).
// rocprim::radix_sort_pairs is stable, so inside one key the items keep their
// index order: rank[b, i] = start[b, key_i] + #{j < i : key_j = key_i}, and
// every float sum downstream runs in a fixed order (deterministic scatters).
// A full-chip LSD radix sort over B * n items replaces a per-key-range
// counting sort whose blocks each had to scan all n keys of their batch
// element.
#include <cstring>  // rocprim's host code uses memset

#include <rocprim/rocprim.hpp>

#include "segsum.hpp"

namespace pcfm {
namespace {

__global__ void __launch_bounds__(256)
    ss_keys_kernel(const int* __restrict__ key, long long key_bstride, int n, int V,
                   unsigned* __restrict__ ck, int* __restrict__ val) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int k = key[(size_t)b * key_bstride + i];
  const size_t o = (size_t)b * n + i;
  ck[o] = (unsigned)b * (unsigned)(V + 1) + ((unsigned)k < (unsigned)V ? (unsigned)k : (unsigned)V);
  val[o] = (int)o;
}

// start[v'] for every composite key v' in [0, B (V + 1)): the first sorted
// position whose key is >= v' (a lower-bound search of the sorted keys, one
// thread per key), minus the batch's base b * n (batch-local).
__global__ void __launch_bounds__(256)
    ss_bounds_kernel(const unsigned* __restrict__ sk, long long total, int n, int V, int B,
                     int* __restrict__ start) {
  const long long v = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long nkeys = (long long)B * (V + 1);
  if (v >= nkeys) return;
  long long lo = 0, hi = total;  // first p with sk[p] >= v
  while (lo < hi) {
    const long long mid = (lo + hi) >> 1;
    if ((long long)sk[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  start[v] = (int)(lo - (v / (V + 1)) * n);
}

__global__ void __launch_bounds__(256)
    ss_rank_kernel(const unsigned* __restrict__ sk, const int* __restrict__ perm, long long total,
                   int n, int V, int* __restrict__ rank) {
  const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
  if (p >= total) return;
  const int o = perm[p];
  const int b = o / n;
  const bool valid = (sk[p] % (unsigned)(V + 1)) != (unsigned)V;
  rank[o] = valid ? (int)(p - (long long)b * n) : -1;
}

__global__ void __launch_bounds__(256)
    ss_counts_kernel(const int* __restrict__ start, int V, int B, int* __restrict__ cnt_out,
                     float* __restrict__ vinv) {
  const int b = blockIdx.y;
  const int v = blockIdx.x * 256 + threadIdx.x;
  if (v >= V) return;
  const int* sb = start + (size_t)b * (V + 1);
  const int c = sb[v + 1] - sb[v];
  if (cnt_out != nullptr) cnt_out[(size_t)b * V + v] = c;
  if (vinv != nullptr) vinv[(size_t)b * V + v] = c > 0 ? (float)(1.0 / (double)c) : 0.0f;
}

unsigned key_bits(int B, int V) {
  const unsigned long long top = (unsigned long long)B * (V + 1);
  unsigned bits = 1;
  while ((1ull << bits) < top) ++bits;
  return bits;
}

size_t rp_temp_bytes(int B, int n, int V) {
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs((void*)nullptr, bytes, (const unsigned*)nullptr, (unsigned*)nullptr,
                            (const int*)nullptr, (int*)nullptr, (size_t)B * n, 0,
                            key_bits(B, V));
  return bytes;
}

}  // namespace

size_t seg_sort_stable_ws(int B, int n, int V) {
  const size_t t = (size_t)B * n;
  return 2 * align256(t * 4) + 2 * align256(t * 4) + align256(rp_temp_bytes(B, n, V));
}

int seg_sort_stable(const int* key, long long key_bstride, int B, int n, int V, int* start,
                    int* cnt_out, float* vinv, int* rank, void* ws, hipStream_t st) {
  const long long total = (long long)B * n;
  // composite keys are 32-bit unsigned, values / permutation 32-bit int
  PCFM_CHECK_ARG((unsigned long long)B * ((unsigned long long)V + 1) <= 0xffffffffull,
                 "segment sort: B * (V + 1) = %llu exceeds 32-bit keys",
                 (unsigned long long)B * ((unsigned long long)V + 1));
  PCFM_CHECK_ARG(total <= 0x7fffffffll, "segment sort: B * n = %lld exceeds int indices", total);
  char* p = (char*)ws;
  auto take = [&p](size_t bytes) {
    char* q = p;
    p += align256(bytes);
    return q;
  };
  unsigned* ck = (unsigned*)take(total * 4);
  unsigned* sk = (unsigned*)take(total * 4);
  int* val = (int*)take(total * 4);
  int* perm = (int*)take(total * 4);
  size_t tb = rp_temp_bytes(B, n, V);
  void* tmp = take(tb);
  if (n > 0) {
    hipLaunchKernelGGL(ss_keys_kernel, dim3(ceil_div(n, 256), B), dim3(256), 0, st, key,
                       key_bstride, n, V, ck, val);
    hipError_t e = rocprim::radix_sort_pairs(tmp, tb, ck, sk, val, perm, (size_t)total, 0,
                                             key_bits(B, V), st);
    if (e != hipSuccess) {
      set_error("segment sort: rocprim::radix_sort_pairs: %s", hipGetErrorString(e));
      return (int)e;
    }
    hipLaunchKernelGGL(ss_rank_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, st, sk, perm,
                       total, n, V, rank);
  }
  hipLaunchKernelGGL(ss_bounds_kernel, dim3(ceil_div((long long)B * (V + 1), 256)), dim3(256), 0,
                     st, sk, total, n, V, B, start);
  if (cnt_out != nullptr || vinv != nullptr)
    hipLaunchKernelGGL(ss_counts_kernel, dim3(ceil_div(V, 256), B), dim3(256), 0, st, start, V, B,
                       cnt_out, vinv);
  return PCFM_OK;
}

}  // namespace pcfm
