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
//                  wave ranks its 64 records per owner with ballots, waves and 256-record rounds are
//                  chained through per-owner counters in LDS -- the result is stable.
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

constexpr int kRT = 256;                // threads per block
constexpr int kRPerThread = 16;         // records per thread per block chunk
constexpr int kRChunk = kRT * kRPerThread;  // 4096 records per block
constexpr int kMaxParts = 8192;         // LDS counters (32 KiB)

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

__global__ __launch_bounds__(kRT) void route_hist(const i64* __restrict__ keys, i64 n, RangeDesc d,
                                                  u32* __restrict__ hist, i64 nblocks, u64* __restrict__ bad) {
  __shared__ u32 h[kMaxParts];
  for (int p = threadIdx.x; p < d.nparts; p += kRT) h[p] = 0;
  __syncthreads();
  const i64 base = (i64)blockIdx.x * kRChunk;
  for (int q = threadIdx.x; q < kRChunk; q += kRT) {
    const i64 i = base + q;
    if (i >= n) break;
    const int32_t o = owner_of(d, keys[i]);
    if (o < 0) { atomicMax(bad, ~(u64)i); continue; }
    atomicAdd(&h[o], 1u);
  }
  __syncthreads();
  for (int p = threadIdx.x; p < d.nparts; p += kRT) hist[(i64)p * nblocks + blockIdx.x] = h[p];  // partition-major
}

__global__ __launch_bounds__(kRT) void route_scatter(const i64* __restrict__ keys, i64 n, RangeDesc d,
                                                     const u32* __restrict__ offs, i64 nblocks,
                                                     i64* __restrict__ order) {
  __shared__ u32 cnt[kMaxParts];       // records of each owner already placed by this block
  __shared__ u32 wave_cnt[4][64];      // per round: per wave, count of each of its (<= 64) owners
  __shared__ int32_t wave_own[4][64];  // the owners each wave saw this round
  __shared__ int wave_n[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int p = threadIdx.x; p < d.nparts; p += kRT) cnt[p] = 0;
  __syncthreads();
  const i64 base = (i64)blockIdx.x * kRChunk;
  for (int round = 0; round < kRPerThread; ++round) {
    const i64 i = base + (i64)round * kRT + threadIdx.x;  // 256 consecutive records per round
    const int32_t o = i < n ? owner_of(d, keys[i]) : -1;
    // rank among the same-owner lanes of this wave, lane order = record order
    u64 pending = __ballot(o >= 0);
    int my_rank = 0, nslots = 0;
    while (pending) {
      const int leader = __ffsll((long long)pending) - 1;
      const int32_t lo = __shfl(o, leader);
      const u64 m = __ballot(o == lo);
      if (o == lo) {
        my_rank = __popcll(m & ((1ull << lane) - 1));
      }
      if (lane == 0) { wave_own[wid][nslots] = lo; wave_cnt[wid][nslots] = (u32)__popcll(m); }
      ++nslots;
      pending &= ~m;
    }
    if (lane == 0) wave_n[wid] = nslots;
    __syncthreads();
    if (o >= 0) {
      // earlier waves' records of the same owner in this round come first
      u32 before = cnt[o];
      for (int w = 0; w < wid; ++w)
        for (int s = 0; s < wave_n[w]; ++s)
          if (wave_own[w][s] == o) before += wave_cnt[w][s];
      order[(i64)offs[(i64)o * nblocks + blockIdx.x] + before + my_rank] = i;
    }
    __syncthreads();
    // advance the block's per-owner counters by this round's totals (one writer per owner)
    if (threadIdx.x < 64 * 4) {
      const int w = threadIdx.x >> 6, s = threadIdx.x & 63;
      if (s < wave_n[w]) {
        const int32_t ow = wave_own[w][s];
        bool first = true;  // the first wave that saw this owner sums every wave's count
        for (int w2 = 0; w2 < w; ++w2)
          for (int s2 = 0; s2 < wave_n[w2]; ++s2)
            if (wave_own[w2][s2] == ow) first = false;
        if (first) {
          u32 tot = 0;
          for (int w2 = w; w2 < 4; ++w2)
            for (int s2 = 0; s2 < wave_n[w2]; ++s2)
              if (wave_own[w2][s2] == ow) tot += wave_cnt[w2][s2];
          cnt[ow] += tot;
        }
      }
    }
    __syncthreads();
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
  const i64 nblocks = std::max<i64>(1, (n + kRChunk - 1) / kRChunk);
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
    route_hist<<<(unsigned)nblocks, kRT, 0, st>>>(keys, n, d, hist, nblocks, bad);
    if (rocprim::exclusive_scan(scan_tmp, scan_bytes, hist, offs, 0u, (size_t)nparts * nblocks,
                                rocprim::plus<u32>(), st) != hipSuccess)
      return GLINT_EDEVICE;
    route_scatter<<<(unsigned)nblocks, kRT, 0, st>>>(keys, n, d, offs, nblocks, order);
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
