// Microbenchmark: rocprim radix sort of (u32 key, u32 value) pairs at the pick list's sizes
// (fanout_kernels.hip, launch_fanout_resolve): which onesweep configuration sorts 0.2-3 M pairs
// on 20-24 key bits fastest on gfx950.  Prints one JSON line per (config, n, bits).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/sort_bench tools/sort_bench.hip
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

using rocprim::default_config;
using rocprim::kernel_config;
template <unsigned B, unsigned I, unsigned R>
using OS = rocprim::radix_sort_config<
    default_config, default_config,
    rocprim::radix_sort_onesweep_config<kernel_config<B, I>, kernel_config<B, I>, R,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;
using DefaultOnesweep = rocprim::radix_sort_config<default_config, default_config, default_config, 0>;

template <class Config>
float run(const char* name, uint32_t* k, uint32_t* v, uint32_t* ko, uint32_t* vo, size_t n, unsigned bits) {
  size_t tb = 0;
  CK(rocprim::radix_sort_pairs<Config>(nullptr, tb, k, ko, v, vo, n, 0u, bits));
  void* tmp = nullptr;
  CK(hipMalloc(&tmp, tb));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) CK(rocprim::radix_sort_pairs<Config>(tmp, tb, k, ko, v, vo, n, 0u, bits));
  const int reps = 20;
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) CK(rocprim::radix_sort_pairs<Config>(tmp, tb, k, ko, v, vo, n, 0u, bits));
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  // check sortedness on the host
  std::vector<uint32_t> h(n);
  CK(hipMemcpy(h.data(), ko, n * 4, hipMemcpyDeviceToHost));
  bool ok = true;
  const uint32_t mask = bits >= 32 ? ~0u : ((1u << bits) - 1);
  for (size_t i = 1; i < n && ok; ++i) ok = (h[i - 1] & mask) <= (h[i] & mask);
  printf("{\"config\": \"%s\", \"n\": %zu, \"bits\": %u, \"us\": %.1f, \"sorted\": %s}\n", name, n, bits,
         1e3f * ms / reps, ok ? "true" : "false");
  CK(hipFree(tmp));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / reps;
}

int main() {
  const size_t nmax = 3u << 20;
  uint32_t *k, *v, *ko, *vo;
  CK(hipMalloc(&k, nmax * 4));
  CK(hipMalloc(&v, nmax * 4));
  CK(hipMalloc(&ko, nmax * 4));
  CK(hipMalloc(&vo, nmax * 4));
  std::vector<uint32_t> hk(nmax), hv(nmax);
  uint64_t x = 88172645463325252ull;
  for (size_t i = 0; i < nmax; ++i) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    hk[i] = static_cast<uint32_t>(x);
    hv[i] = static_cast<uint32_t>(i);
  }
  CK(hipMemcpy(k, hk.data(), nmax * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(v, hv.data(), nmax * 4, hipMemcpyHostToDevice));
  for (size_t n : {size_t(200000), size_t(800000), size_t(3000000)})
    for (unsigned bits : {20u, 24u}) {
      run<DefaultOnesweep>("default_onesweep", k, v, ko, vo, n, bits);
      run<rocprim::default_config>("default", k, v, ko, vo, n, bits);
      run<OS<256, 12, 8>>("os_256x12_r8", k, v, ko, vo, n, bits);
      run<OS<256, 8, 8>>("os_256x8_r8", k, v, ko, vo, n, bits);
      run<OS<512, 8, 8>>("os_512x8_r8", k, v, ko, vo, n, bits);
      run<OS<256, 8, 10>>("os_256x8_r10", k, v, ko, vo, n, bits);
      run<OS<256, 12, 11>>("os_256x12_r11", k, v, ko, vo, n, bits);
      run<OS<512, 8, 11>>("os_512x8_r11", k, v, ko, vo, n, bits);
    }
  return 0;
}
