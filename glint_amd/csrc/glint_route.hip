// glint_route.hip -- device-side client bucketing: the exchange step in front of the shards.
//
// AsyncBigVector.mapPartitions (src/main/scala/glint/models/client/async/AsyncBigVector.scala:96-98)
// groups a batch's record indices by owning partition, each group in the caller's order, and sends
// one message per partition. On the GPU this is a stable counting sort by partition index:
//   route_hist     per 4096-record block, a histogram of owners (RangePartitioner.partition,
//                  RangePartitioner.scala:27-43, bit for bit incl. its Int truncations, or the
//                  cyclic key % P of CyclicPartitioner.scala:19-22), stored
//                  partition-major so that one exclusive scan yields every (partition, block) offset;
//   (rocPRIM exclusive scan over the histogram)
//   route_scatter  each block writes its record indices to their partition's range, in order: a
//                  wave finds its same-owner lanes with one ballot per owner bit, the waves of a
//                  256-record round then claim slots in wave order from per-owner LDS counters --
//                  the result is stable.
// Out-of-range keys (IndexOutOfBoundsException in the reference, :30-32) are reported as the first
// bad record index; the routing of the other records is unaffected.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_scan.hpp>
#include <stdint.h>
#include <algorithm>
#include <mutex>
#include "../../include/glint_gpu.h"

namespace {

typedef int64_t i64;
typedef uint64_t u64;
typedef unsigned int u32;

constexpr int kRT = 256;         // threads per block
constexpr int kMinRounds = 16;   // a block's chunk: >= 16 rounds of 256 records (4096)
constexpr int kMaxParts = 8192;  // LDS counters (32 KiB)

struct RangeDesc {
  i64 nkeys;      // RangePartitioner.size / CyclicPartitioner.keys
  i64 small_keys; // numberOfSmallPartitions * smallPartitionSize
  int32_t n_small;
  int32_t q;      // smallPartitionSize
  int32_t nparts;
  int32_t cyclic; // GLINT_ROUTE_CYCLIC
};

// RangePartitioner.partition (RangePartitioner.scala:27-43) or CyclicPartitioner.partition
// (CyclicPartitioner.scala:19-22); -1 where the reference throws
__device__ __forceinline__ int32_t owner_of(const RangeDesc& d, i64 key) {
  if (key < 0 || key >= d.nkeys) return -1;
  if (d.cyclic) return (int32_t)(key % d.nparts);
  // .toInt of the index; a partitioner whose Int sizes overflowed yields an index outside the
  // partition array (ArrayIndexOutOfBoundsException in the reference) -> rejected like a bad key
  const int32_t o = key < d.small_keys ? (int32_t)(key / d.q)
                                       : (int32_t)((i64)d.n_small + (key - d.small_keys) / ((i64)d.q + 1));
  return o < d.nparts ? o : -1;
}

// Lanes of the wave whose owner equals this lane's: one ballot per owner bit (owners < 2^nbits,
// the sentinel `nparts` included) instead of a loop over the distinct owners of the wave.
__device__ __forceinline__ u64 match_owner(int32_t o, int nbits) {
  u64 m = ~0ull;
  for (int k = 0; k < nbits; ++k) {
    const bool bit = (o >> k) & 1;
    const u64 b = __ballot(bit);
    m &= bit ? b : ~b;
  }
  return m;
}

// The block's chunk is `rounds` x 256 consecutive records; owners outside [0, nparts) count as bad.
__global__ __launch_bounds__(kRT) void route_hist(const i64* __restrict__ keys, i64 n, RangeDesc d, int nbits,
                                                  int rounds, u32* __restrict__ hist, i64 nblocks,
                                                  u64* __restrict__ bad) {
  __shared__ u32 h[kMaxParts];
  const int lane = threadIdx.x & 63;
  for (int p = threadIdx.x; p < d.nparts; p += kRT) h[p] = 0;
  __syncthreads();
  const i64 base = (i64)blockIdx.x * rounds * kRT;
  for (int r = 0; r < rounds; ++r) {
    const i64 i = base + (i64)r * kRT + threadIdx.x;
    int32_t o = d.nparts;  // sentinel: past the end
    if (i < n) {
      o = owner_of(d, keys[i]);
      if (o < 0) { atomicMax(bad, ~(u64)i); o = d.nparts; }
    }
    const u64 m = match_owner(o, nbits);
    // the group's lowest lane adds the group size: one LDS atomic per distinct owner per wave
    if (o < d.nparts && (m & ((1ull << lane) - 1)) == 0) atomicAdd(&h[o], (u32)__popcll(m));
  }
  __syncthreads();
  for (int p = threadIdx.x; p < d.nparts; p += kRT) hist[(i64)p * nblocks + blockIdx.x] = h[p];  // partition-major
}

__global__ __launch_bounds__(kRT) void route_scatter(const i64* __restrict__ keys, i64 n, RangeDesc d, int nbits,
                                                     int rounds, const u32* __restrict__ offs, i64 nblocks,
                                                     i64* __restrict__ order) {
  __shared__ u32 cnt[kMaxParts];  // records of each owner this block has placed so far
  __shared__ u32 grp_base[kRT];   // per group leader: the group's first slot within its owner
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int p = threadIdx.x; p < d.nparts; p += kRT) cnt[p] = 0;
  __syncthreads();
  const i64 base = (i64)blockIdx.x * rounds * kRT;
  for (int r = 0; r < rounds; ++r) {
    const i64 i = base + (i64)r * kRT + threadIdx.x;  // 256 consecutive records per round
    int32_t o = d.nparts;
    if (i < n) {
      o = owner_of(d, keys[i]);
      if (o < 0) o = d.nparts;
    }
    const u64 m = match_owner(o, nbits);
    const u64 below = m & ((1ull << lane) - 1);
    const bool leader = below == 0 && o < d.nparts;
    // waves claim their slots in order (wave 0 holds the round's earliest records): stable
    for (int w = 0; w < kRT / 64; ++w) {
      if (wid == w && leader) {
        grp_base[threadIdx.x] = cnt[o];
        cnt[o] += (u32)__popcll(m);
      }
      __syncthreads();
    }
    if (o < d.nparts) {
      const int lead = __ffsll((long long)m) - 1;
      order[(i64)offs[(i64)o * nblocks + blockIdx.x] + grp_base[wid * 64 + lead] + __popcll(below)] = i;
    }
    __syncthreads();  // grp_base is rewritten next round
  }
}

// records per partition: the distance between consecutive partitions' first offsets; the last
// partition ends at the scan's total (its last block's offset + count)
__global__ void route_counts(const u32* __restrict__ offs, const u32* __restrict__ hist, i64 nblocks,
                             int32_t nparts, i64* __restrict__ counts) {
  const i64 total = (i64)offs[(i64)nparts * nblocks - 1] + hist[(i64)nparts * nblocks - 1];
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < nparts; p += gridDim.x * blockDim.x) {
    const i64 end = p + 1 < nparts ? (i64)offs[(i64)(p + 1) * nblocks] : total;
    counts[p] = end - (i64)offs[(i64)p * nblocks];
  }
}

std::mutex g_route_mu;
void* g_tmp = nullptr;
size_t g_tmp_bytes = 0;

}  // namespace

extern "C" int glint_route_dev(const int64_t* keys, int64_t n, int kind, int32_t nparts, int64_t nkeys,
                               int64_t* counts, int64_t* order, int64_t* first_bad, void* stream) {
  if (kind != GLINT_ROUTE_RANGE && kind != GLINT_ROUTE_CYCLIC) return GLINT_EINVAL;
  if (nparts <= 0 || nparts > kMaxParts || n < 0 || nkeys < 0 || !counts || !first_bad) return GLINT_EINVAL;
  if (n > 0 && (!keys || !order)) return GLINT_EINVAL;
  if (n >= ((i64)1 << 32)) return GLINT_EINVAL;  // 32-bit offsets
  hipStream_t st = (hipStream_t)stream;
  // RangePartitioner.apply (RangePartitioner.scala:62-84) -- same Int truncation of the sizes
  RangeDesc d{};
  const int32_t n_large = (int32_t)(nkeys % nparts);
  d.n_small = nparts - n_large;
  d.q = (int32_t)((nkeys - nkeys % nparts) / nparts);
  d.small_keys = (i64)d.n_small * (i64)d.q;
  d.nkeys = nkeys;
  d.nparts = nparts;
  d.cyclic = kind == GLINT_ROUTE_CYCLIC;
  // chunk per block grows with nparts so the (partition x block) histogram stays <= n/4 entries
  const int rounds = std::max<int>(kMinRounds, (4 * nparts + kRT - 1) / kRT);
  const i64 chunk = (i64)rounds * kRT;
  const i64 nblocks = std::max<i64>(1, (n + chunk - 1) / chunk);
  int nbits = 1;
  while ((1 << nbits) <= nparts) ++nbits;  // owners and the sentinel nparts fit in nbits
  std::lock_guard<std::mutex> lk(g_route_mu);
  const size_t hist_bytes = (size_t)nparts * nblocks * 4;
  size_t scan_bytes = 0;
  if (rocprim::exclusive_scan(nullptr, scan_bytes, (u32*)nullptr, (u32*)nullptr, 0u, (size_t)nparts * nblocks,
                              rocprim::plus<u32>(), st) != hipSuccess)
    return GLINT_EDEVICE;
  const size_t need = 2 * ((hist_bytes + 255) & ~(size_t)255) + 256 + scan_bytes;
  if (g_tmp_bytes < need) {
    if (g_tmp) (void)hipFree(g_tmp);
    g_tmp = nullptr;
    g_tmp_bytes = 0;
    if (hipMalloc(&g_tmp, need) != hipSuccess) { (void)hipGetLastError(); return GLINT_ENOMEM; }
    g_tmp_bytes = need;
  }
  char* b = (char*)g_tmp;
  u32* hist = (u32*)b;
  u32* offs = (u32*)(b + ((hist_bytes + 255) & ~(size_t)255));
  u64* bad = (u64*)(b + 2 * ((hist_bytes + 255) & ~(size_t)255));
  void* scan_tmp = b + 2 * ((hist_bytes + 255) & ~(size_t)255) + 256;
  if (hipMemsetAsync(bad, 0, 8, st) != hipSuccess) return GLINT_EDEVICE;
  if (n == 0) {
    if (hipMemsetAsync(counts, 0, (size_t)nparts * 8, st) != hipSuccess) return GLINT_EDEVICE;
  } else {
    route_hist<<<(unsigned)nblocks, kRT, 0, st>>>(keys, n, d, nbits, rounds, hist, nblocks, bad);
    if (rocprim::exclusive_scan(scan_tmp, scan_bytes, hist, offs, 0u, (size_t)nparts * nblocks,
                                rocprim::plus<u32>(), st) != hipSuccess)
      return GLINT_EDEVICE;
    route_scatter<<<(unsigned)nblocks, kRT, 0, st>>>(keys, n, d, nbits, rounds, offs, nblocks, order);
    route_counts<<<(unsigned)((nparts + 255) / 256), 256, 0, st>>>(offs, hist, nblocks, nparts, counts);
  }
  // first bad record: enc = ~index (0 = none); returned through the host word *first_bad
  u64 enc = 0;
  if (hipMemcpyAsync(&enc, bad, 8, hipMemcpyDeviceToHost, st) != hipSuccess) return GLINT_EDEVICE;
  if (hipStreamSynchronize(st) != hipSuccess) return GLINT_EDEVICE;
  *first_bad = enc ? (int64_t)~enc : -1;
  if (hipGetLastError() != hipSuccess) return GLINT_EDEVICE;
  return enc ? GLINT_EOUTOFRANGE : GLINT_OK;
}
