// Walk order (emqx_set_tuning "order"): a batch is matched in an order that groups topics by
// prefix, so tiles that run together on one XCD walk the same subtrees and share its L2.
//
// The reference matches each published topic on its own (emqx_broker.erl:213 ->
// emqx_router:match_routes/1, emqx_router.erl:128-133); the order in which a batch is walked
// changes nothing in any topic's match set, and the CSR comes back in the caller's order.
//
//   order_key_kernel     per topic: a 64-bit prefix key (per level, the top `lbits` bits of a
//                        hash of the word, first level in the highest bits) and its index
//   radix sort           (rocprim) keys -> the topic indices in key order: perm[p] = topic
//   order_len_kernel     lens[p] = length of topic perm[p]; a scan gives the new offsets
//   order_gather_kernel  the topic bytes in the new order (one contiguous buffer again, as the
//                        fast kernel's tokenizer wants)
//   order_counts_kernel  after the walk: per-topic counts back to the caller's order, whose
//                        scan is the output CSR's offsets (the scatter kernels write each
//                        topic's ids at out_off[perm[p]])
// The fast kernel also deals logical tiles to XCDs in contiguous ranges (MatchArgs::deal), so
// each XCD walks one slice of the key space.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include "kernels.h"

namespace emqx {

namespace {

template <class K>
__global__ __launch_bounds__(256) void order_key_kernel(const uint8_t* __restrict__ tbytes,
                                                        const uint64_t* __restrict__ toffs, uint64_t n,
                                                        uint32_t lbits, uint32_t sort_bits, K* __restrict__ keys,
                                                        uint32_t* __restrict__ idx) {
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint64_t s = toffs[i], e = toffs[i + 1], lim = toffs[n];
    uint64_t key = 0;
    uint32_t room = 64, h = 0x811C9DC5u;
    // the topic's bytes in 16-B aligned windows (a window holding a topic byte lies inside the
    // buffer's allocation), then one byte step per position; position e is the final '/'
    const uintptr_t a0 = reinterpret_cast<uintptr_t>(tbytes + s) & ~static_cast<uintptr_t>(15);
    const uintptr_t aend = reinterpret_cast<uintptr_t>(tbytes + e);
    const uintptr_t abeg = reinterpret_cast<uintptr_t>(tbytes + s);
    const uintptr_t alim = reinterpret_cast<uintptr_t>(tbytes + lim);  // bytes below are readable
    for (uintptr_t c0 = a0; c0 <= aend && room; c0 += 16) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (c0 + 16 <= alim) {
        v = *reinterpret_cast<const uint4*>(c0);
      } else if (c0 < aend) {  // the batch's last window: only its readable bytes
        uint32_t t4[4] = {0, 0, 0, 0};
        for (uint32_t b = 0; b < 16 && c0 + b < alim; ++b)
          t4[b >> 2] |= static_cast<uint32_t>(*reinterpret_cast<const uint8_t*>(c0 + b)) << (8u * (b & 3u));
        v = make_uint4(t4[0], t4[1], t4[2], t4[3]);
      }
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (uint32_t b = 0; b < 16; ++b) {
        const uintptr_t p = c0 + b;
        if (p < abeg || p > aend || !room) continue;
        const uint32_t c = p < aend ? (w[b >> 2] >> (8u * (b & 3u))) & 0xFFu : static_cast<uint32_t>('/');
        if (c == '/') {
          const uint32_t take = min(lbits, room);
          room -= take;
          key |= static_cast<uint64_t>(mix32(h) >> (32u - take)) << room;
          h = 0x811C9DC5u;
        } else {
          h = (h ^ c) * 0x01000193u;
        }
      }
    }
    keys[i] = static_cast<K>(key >> (64u - sort_bits));  // the sort orders bits [0, sort_bits)
    idx[i] = static_cast<uint32_t>(i);
  }
}

__global__ __launch_bounds__(256) void order_len_kernel(const uint64_t* __restrict__ toffs,
                                                        const uint32_t* __restrict__ perm, uint64_t n,
                                                        uint32_t* __restrict__ lens) {
  for (uint64_t p = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; p < n;
       p += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint32_t t = perm[p];
    lens[p] = static_cast<uint32_t>(toffs[t + 1] - toffs[t]);
  }
}

// 16 lanes per topic, 16 topics per block; bytes beyond `cap` flag the call for a rerun with
// a larger buffer (nothing is written then, and the match kernels skip the call).
__global__ __launch_bounds__(256) void order_gather_kernel(const uint8_t* __restrict__ tbytes,
                                                           const uint64_t* __restrict__ toffs,
                                                           const uint32_t* __restrict__ perm, uint64_t n,
                                                           const uint64_t* __restrict__ noffs,
                                                           uint8_t* __restrict__ obytes, uint64_t cap,
                                                           uint32_t* ctrl) {
  if (noffs[n] > cap) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(&ctrl[CTRL_ERROR], CTRL_ERR_ORDER_CAP);
    return;
  }
  const uint32_t sub = threadIdx.x & 15u;
  for (uint64_t p = (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 4; p < n;
       p += (static_cast<uint64_t>(gridDim.x) * blockDim.x) >> 4) {
    const uint32_t t = perm[p];
    const uint64_t s = toffs[t], len = toffs[t + 1] - s, d = noffs[p];
    for (uint64_t j = sub; j < len; j += 16) obytes[d + j] = tbytes[s + j];
  }
}

__global__ __launch_bounds__(256) void order_counts_kernel(const uint32_t* __restrict__ counts,
                                                           const uint32_t* __restrict__ perm, uint64_t n,
                                                           uint32_t* __restrict__ corig) {
  for (uint64_t p = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; p < n;
       p += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    corig[perm[p]] = counts[p];
}

// 16 lanes per topic: received topic k's ids (at recv_off[k]) to its batch position's slot
// of the output CSR (out_off[perm[k]]).
__global__ __launch_bounds__(256) void csr_unpermute_kernel(const uint32_t* __restrict__ counts,
                                                            const uint64_t* __restrict__ recv_off,
                                                            const uint32_t* __restrict__ ids,
                                                            const uint32_t* __restrict__ perm, uint64_t n,
                                                            const uint64_t* __restrict__ out_off,
                                                            uint32_t* __restrict__ out_ids) {
  const uint32_t sub = threadIdx.x & 15u;
  for (uint64_t k = (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 4; k < n;
       k += (static_cast<uint64_t>(gridDim.x) * blockDim.x) >> 4) {
    const uint32_t c = counts[k];
    const uint64_t s = recv_off[k], d = out_off[perm[k]];
    for (uint32_t j = sub; j < c; j += 16) out_ids[d + j] = ids[s + j];
  }
}

uint32_t grid_for(uint64_t n, uint32_t per_block) {
  return static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>((n + per_block - 1) / per_block, 8192)));
}

}  // namespace

// Keys of at most 32 bits sort as u32 (rocprim's radix sort then runs its one-sweep passes
// over half the bytes; 64-bit keys take its merge sort at these sizes).
template <class K>
hipError_t sort_pairs(void* temp, size_t& bytes, K* keys, K* keys_out, uint32_t* idx, uint32_t* perm, uint64_t n,
                      uint32_t sort_bits, hipStream_t s) {
  return rocprim::radix_sort_pairs(temp, bytes, keys, keys_out, idx, perm, static_cast<size_t>(n), 0u, sort_bits, s);
}

// Scratch of the radix sort over n pairs on `sort_bits` key bits (the size depends on the bit
// range, not only on n: fewer bits can take another algorithm).
uint64_t order_sort_temp_bytes(uint64_t n, uint32_t sort_bits) {
  size_t bytes = 0;
  if (sort_bits <= 32)
    (void)sort_pairs<uint32_t>(nullptr, bytes, nullptr, nullptr, nullptr, nullptr, n, sort_bits, nullptr);
  else
    (void)sort_pairs<uint64_t>(nullptr, bytes, nullptr, nullptr, nullptr, nullptr, n, sort_bits, nullptr);
  return bytes;
}

template <class K>
hipError_t launch_order_t(const OrderArgs& o, hipStream_t s) {
  K* keys = reinterpret_cast<K*>(o.keys);
  K* keys_out = reinterpret_cast<K*>(o.keys_out);
  hipLaunchKernelGGL(order_key_kernel<K>, dim3(grid_for(o.n, 256)), dim3(256), 0, s, o.tbytes, o.toffs, o.n,
                     o.level_bits, o.sort_bits, keys, o.idx);
  size_t tb = 0;
  (void)sort_pairs<K>(nullptr, tb, keys, keys_out, o.idx, o.perm, o.n, o.sort_bits, s);
  if (tb > o.temp_bytes) return hipErrorInvalidValue;  // the caller sized the scratch for fewer bytes
  hipError_t err = sort_pairs<K>(o.temp, tb, keys, keys_out, o.idx, o.perm, o.n, o.sort_bits, s);
  if (err != hipSuccess) return err;
  hipLaunchKernelGGL(order_len_kernel, dim3(grid_for(o.n, 256)), dim3(256), 0, s, o.toffs, o.perm, o.n, o.lens);
  err = launch_scan(o.lens, o.n, o.noffs, o.partials, s);
  if (err != hipSuccess) return err;
  hipLaunchKernelGGL(order_gather_kernel, dim3(grid_for(o.n, 16)), dim3(256), 0, s, o.tbytes, o.toffs, o.perm, o.n,
                     o.noffs, o.obytes, o.cap_bytes, o.ctrl);
  return hipGetLastError();
}

hipError_t launch_order(const OrderArgs& o, hipStream_t s) {
  if (o.n == 0) return hipSuccess;
  return o.sort_bits <= 32 ? launch_order_t<uint32_t>(o, s) : launch_order_t<uint64_t>(o, s);
}

// Scratch of the batch (un)permute entry points: u32 [n] lengths / counts, u64 [n + 1]
// offsets, the scan's partials, one control word block.
namespace {
uint64_t align16(uint64_t x) { return (x + 15) & ~15ull; }
}  // namespace

uint64_t permute_scratch_bytes(uint64_t n) {
  return align16(4 * std::max<uint64_t>(n, 1)) + align16(8 * (n + 1)) + align16(8 * scan_partials(n)) +
         align16(4 * CTRL_WORDS);
}

hipError_t launch_batch_permute(const uint8_t* tbytes, const uint64_t* toffs, uint64_t n, const uint32_t* perm,
                                uint8_t* obytes, uint64_t* ooffs, void* scratch, hipStream_t s) {
  uint8_t* p = static_cast<uint8_t*>(scratch);
  uint32_t* lens = reinterpret_cast<uint32_t*>(p);
  p += align16(4 * std::max<uint64_t>(n, 1)) + align16(8 * (n + 1));
  uint64_t* partials = reinterpret_cast<uint64_t*>(p);
  p += align16(8 * scan_partials(n));
  uint32_t* ctrl = reinterpret_cast<uint32_t*>(p);
  if (n) hipLaunchKernelGGL(order_len_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, toffs, perm, n, lens);
  hipError_t err = launch_scan(lens, n, ooffs, partials, s);
  if (err != hipSuccess || n == 0) return err;
  hipLaunchKernelGGL(order_gather_kernel, dim3(grid_for(n, 16)), dim3(256), 0, s, tbytes, toffs, perm, n, ooffs,
                     obytes, ~0ull, ctrl);
  return hipGetLastError();
}

hipError_t launch_csr_unpermute(const uint32_t* counts, const uint32_t* ids, uint64_t n, const uint32_t* perm,
                                uint64_t* out_off, uint32_t* out_ids, void* scratch, hipStream_t s) {
  uint8_t* p = static_cast<uint8_t*>(scratch);
  uint32_t* corig = reinterpret_cast<uint32_t*>(p);
  p += align16(4 * std::max<uint64_t>(n, 1));
  uint64_t* recv_off = reinterpret_cast<uint64_t*>(p);
  p += align16(8 * (n + 1));
  uint64_t* partials = reinterpret_cast<uint64_t*>(p);
  if (n) hipLaunchKernelGGL(order_counts_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, counts, perm, n, corig);
  hipError_t err = launch_scan(corig, n, out_off, partials, s);  // batch order
  if (err == hipSuccess) err = launch_scan(counts, n, recv_off, partials, s);  // received order
  if (err != hipSuccess || n == 0) return err;
  hipLaunchKernelGGL(csr_unpermute_kernel, dim3(grid_for(n, 16)), dim3(256), 0, s, counts, recv_off, ids, perm, n,
                     out_off, out_ids);
  return hipGetLastError();
}

// Stable sort of a batch's topics by owner rank (the sharded layout's partition): a radix sort
// of (owner, index) pairs over the owner's bits only — one pass for up to 256 ranks.
namespace {
__global__ __launch_bounds__(256) void iota_kernel(uint32_t* __restrict__ idx, uint64_t n) {
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    idx[i] = static_cast<uint32_t>(i);
}
uint32_t owner_bits(uint32_t world) {
  uint32_t b = 1;
  while (b < 32 && (1ull << b) < world) ++b;
  return b;
}
}  // namespace

uint64_t owner_sort_scratch_bytes(uint64_t n, uint32_t world) {
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, bytes, static_cast<const uint32_t*>(nullptr),
                                  static_cast<uint32_t*>(nullptr), static_cast<const uint32_t*>(nullptr),
                                  static_cast<uint32_t*>(nullptr), static_cast<size_t>(n), 0u, owner_bits(world));
  return align16(bytes) + 2 * align16(4 * std::max<uint64_t>(n, 1));
}

hipError_t launch_owner_sort(const uint32_t* owner, uint64_t n, uint32_t world, uint32_t* perm, void* scratch,
                             hipStream_t s) {
  if (n == 0) return hipSuccess;
  size_t tb = 0;
  const uint32_t bits = owner_bits(world);
  (void)rocprim::radix_sort_pairs(nullptr, tb, owner, static_cast<uint32_t*>(nullptr), static_cast<const uint32_t*>(nullptr),
                                  perm, static_cast<size_t>(n), 0u, bits, s);
  uint8_t* p = static_cast<uint8_t*>(scratch);
  void* temp = p;
  p += align16(tb);
  uint32_t* keys_out = reinterpret_cast<uint32_t*>(p);
  p += align16(4 * n);
  uint32_t* idx = reinterpret_cast<uint32_t*>(p);
  hipLaunchKernelGGL(iota_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, idx, n);
  return rocprim::radix_sort_pairs(temp, tb, owner, keys_out, idx, perm, static_cast<size_t>(n), 0u, bits, s);
}

hipError_t launch_order_counts(const uint32_t* counts, const uint32_t* perm, uint64_t n, uint32_t* corig,
                               hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(order_counts_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, counts, perm, n, corig);
  return hipGetLastError();
}

}  // namespace emqx
