// Random-access ceiling for the match kernel's access pattern on MI355X (gfx950):
// 16-byte records (one dwordx4 load per lane, the EdgeSlot size) at random addresses of a
// table from L2-resident to far larger than the Infinity Cache.  Two shapes:
//   indep  every lane issues R independent random record loads (throughput ceiling)
//   chase  every lane follows its own chain of R dependent loads (latency x concurrency)
// Prints one JSON line per (shape, table size, waves per CU).  Used to price the roofline of
// match_fast_kernel against random-access HBM rather than the streaming 8 TB/s figure.
// `gather_bench cal`: FETCH_SIZE / WRITE_SIZE calibration kernels instead — a 1 GiB buffer read
// once with 4-B lanes (stream_dword_kernel), once with 16-B lanes (stream_x4_kernel) and written
// once with 4-B lanes (write_dword_kernel): known byte counts for the fan-out's access widths.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/gather_bench tools/gather_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

struct alignas(16) Rec {
  uint32_t next, a, b, c;
};

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__global__ void init_kernel(Rec* t, uint32_t n, uint32_t stride) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    Rec r;
    r.next = (uint32_t)(((uint64_t)i * stride + 1) % n);  // stride coprime with n: one long cycle
    r.a = i; r.b = i ^ 1; r.c = i ^ 2;
    t[i] = r;
  }
}

__global__ void indep_kernel(const Rec* __restrict__ t, uint32_t n, uint32_t iters, uint32_t* out) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  uint32_t h = mix(gid * 0x9e3779b9u + 12345u);
  for (uint32_t k = 0; k < iters; ++k) {
    h = mix(h + k);
    const Rec* p = t + (h % n);
    const uint4 x = *reinterpret_cast<const uint4*>(p);
    acc ^= x.x + x.y + x.z + x.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// Two 16-B loads per lane per iteration (`gather_bench pair`): in one 64-B line (SAME = 1) or in
// two random lines (SAME = 0).  Prices the '+' probe sharing the literal probe's line: does the
// second load of a line cost an L2 request and a miss of its own?
template <int SAME>
__global__ void pair_kernel(const Rec* __restrict__ t, uint32_t n, uint32_t iters, uint32_t* out) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  uint32_t h = mix(gid * 0x9e3779b9u + 4321u);
  for (uint32_t k = 0; k < iters; ++k) {
    h = mix(h + k);
    const uint32_t i = (h % n) & ~3u;
    const uint32_t j = SAME ? (i | (1u + (h >> 30))) : (mix(h ^ 0x5bd1e995u) % n);
    const uint4 x = *reinterpret_cast<const uint4*>(t + i);
    const uint4 y = *reinterpret_cast<const uint4*>(t + j);
    acc ^= x.x + x.y + y.z + y.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void chase_kernel(const Rec* __restrict__ t, uint32_t n, uint32_t iters, uint32_t* out) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t i = mix(gid * 0x9e3779b9u + 777u) % n;
  uint32_t acc = 0;
  for (uint32_t k = 0; k < iters; ++k) {
    const Rec* p = t + i;
    const uint4 x = *reinterpret_cast<const uint4*>(p);
    acc ^= x.y + x.w;
    i = x.x;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void stream_dword_kernel(const uint32_t* __restrict__ a, uint64_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    acc += a[i];
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void stream_x4_kernel(const uint4* __restrict__ a, uint64_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 x = a[i];
    acc += x.x ^ x.y ^ x.z ^ x.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void write_dword_kernel(uint32_t* __restrict__ a, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    a[i] = (uint32_t)i;
}

static int calibrate() {
  const uint64_t bytes = 1ull << 30;
  uint32_t* buf;
  uint32_t* out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 64));
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(write_dword_kernel, dim3(8192), dim3(256), 0, 0, buf, bytes / 4);
    hipLaunchKernelGGL(stream_dword_kernel, dim3(8192), dim3(256), 0, 0, buf, bytes / 4, out);
    hipLaunchKernelGGL(stream_x4_kernel, dim3(8192), dim3(256), 0, 0, reinterpret_cast<const uint4*>(buf), bytes / 16,
                       out);
  }
  CK(hipDeviceSynchronize());
  printf("{\"calibration\": \"1 GiB per kernel: write_dword_kernel writes it, stream_dword_kernel and "
         "stream_x4_kernel read it\", \"bytes_per_dispatch\": %llu}\n", (unsigned long long)bytes);
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}

static int pairs() {
  const uint64_t bytes = 1ull << 30;
  const uint32_t n = (uint32_t)(bytes / sizeof(Rec));
  Rec* t;
  uint32_t* out;
  CK(hipMalloc(&t, bytes));
  CK(hipMalloc(&out, 64));
  hipLaunchKernelGGL(init_kernel, dim3(4096), dim3(256), 0, 0, t, n, 2654435761u % n | 1u);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const uint32_t blocks = 256u * 24 / 4u, iters = 256;
  for (int rep = 0; rep < 3; ++rep) {
    for (int v = 0; v < 3; ++v) {
      CK(hipEventRecord(e0));
      if (v == 0) hipLaunchKernelGGL(indep_kernel, dim3(blocks), dim3(256), 0, 0, t, n, iters, out);
      if (v == 1) hipLaunchKernelGGL(pair_kernel<1>, dim3(blocks), dim3(256), 0, 0, t, n, iters, out);
      if (v == 2) hipLaunchKernelGGL(pair_kernel<0>, dim3(blocks), dim3(256), 0, 0, t, n, iters, out);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep == 2)
        printf("{\"pair\": \"%s\", \"ms\": %.4f, \"iters_per_s\": %.4g}\n",
               v == 0 ? "one load" : v == 1 ? "two loads, one 64-B line" : "two loads, two lines", ms,
               (double)blocks * 256 * iters / (ms * 1e-3));
    }
  }
  CK(hipFree(t));
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && argv[1][0] == 'c') return calibrate();
  if (argc > 1 && argv[1][0] == 'p') return pairs();
  const uint64_t sizes_mb[] = {2, 64, 1024};
  const int wpc[] = {8, 16, 24, 32};
  uint32_t* out;
  CK(hipMalloc(&out, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (uint64_t mb : sizes_mb) {
    const uint32_t n = (uint32_t)(mb * 1024 * 1024 / sizeof(Rec));
    Rec* t;
    CK(hipMalloc(&t, (uint64_t)n * sizeof(Rec)));
    hipLaunchKernelGGL(init_kernel, dim3(4096), dim3(256), 0, 0, t, n, 2654435761u % n | 1u);
    CK(hipDeviceSynchronize());
    for (int shape = 0; shape < 2; ++shape) {
      for (int w : wpc) {
        const uint32_t blocks = 256u * w / 4u;  // 256 threads = 4 waves per block
        const uint32_t iters = shape == 0 ? 256 : 128;
        for (int rep = 0; rep < 2; ++rep) {  // rep 0 = warm-up
          CK(hipEventRecord(e0));
          if (shape == 0)
            hipLaunchKernelGGL(indep_kernel, dim3(blocks), dim3(256), 0, 0, t, n, iters, out);
          else
            hipLaunchKernelGGL(chase_kernel, dim3(blocks), dim3(256), 0, 0, t, n, iters, out);
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          if (rep == 1) {
            const double loads = (double)blocks * 256 * iters;
            printf("{\"shape\": \"%s\", \"table_mb\": %llu, \"waves_per_cu\": %d, \"ms\": %.4f, "
                   "\"records_per_s\": %.4g, \"gb_per_s_16B\": %.1f, \"gb_per_s_128B_lines\": %.1f, "
                   "\"ns_per_dependent_load\": %.1f}\n",
                   shape == 0 ? "indep" : "chase", (unsigned long long)mb, w, ms, loads / (ms * 1e-3),
                   loads * 16 / (ms * 1e-3) / 1e9, loads * 128 / (ms * 1e-3) / 1e9,
                   shape == 1 ? ms * 1e6 / iters : 0.0);
          }
        }
      }
    }
    CK(hipFree(t));
  }
  return 0;
}
