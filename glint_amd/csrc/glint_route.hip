// glint_route.hip -- device-side client bucketing: the exchange step in front of the shards.
//
// AsyncBigVector.mapPartitions (src/main/scala/glint/models/client/async/AsyncBigVector.scala:96-98)
// groups a batch's record indices by owning partition, each group in the caller's order, and sends
// one message per partition. On the GPU this is a stable counting sort by partition index:
//   route_hist     per 4096-record block, a histogram of owners (RangePartitioner.partition,
//                  RangePartitioner.scala:27-43, bit for bit incl. its Int truncations, or the
//                  cyclic key % P of CyclicPartitioner.scala:19-22), stored
//                  partition-major so that one exclusive scan yields every (partition, block) offset;
//   route_row_sums / route_row_scan
//                  the (partition, block) offsets: each partition's total, then per partition its
//                  first slot (the totals before it) plus the exclusive scan of its row;
//   route_scatter  each block writes its record indices to their partition's range, in order: a
//                  wave finds its same-owner lanes with one ballot per owner bit, the waves of a
//                  256-record round then claim slots in wave order from per-owner LDS counters --
//                  the result is stable.
// Out-of-range keys (IndexOutOfBoundsException in the reference, :30-32) are reported as the first
// bad record index; the routing of the other records is unaffected.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <map>
#include <memory>
#include <mutex>
#include <utility>
#include <type_traits>
#include <cstdlib>
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
  int32_t fastdiv;  // nkeys <= 2^52: the quotients below by a double reciprocal and one correction
  double inv_q, inv_large, inv_p;  // 1 / smallPartitionSize, 1 / largePartitionSize, 1 / nparts
};

// floor(x / dv) for 0 <= x < 2^52 and 0 < dv < 2^31, from inv = 1.0 / dv: the estimate is within one of
// the quotient (both roundings are relative 2^-53), and one step each way fixes it, in place of an i64
// division's ~100-instruction sequence per record (the route kernels timed the same either way: they
// are bound by their memory traffic, not by this).
__device__ __forceinline__ i64 div_fast(i64 x, i64 dv, double inv) {
  i64 o = (i64)((double)x * inv);
  const i64 r = x - o * dv;
  o += r < 0 ? -1 : (r >= dv ? 1 : 0);
  return o;
}

// RangePartitioner.partition (RangePartitioner.scala:27-43) or CyclicPartitioner.partition
// (CyclicPartitioner.scala:19-22); -1 where the reference throws
__device__ __forceinline__ int32_t owner_of(const RangeDesc& d, i64 key) {
  if (key < 0 || key >= d.nkeys) return -1;
  if (d.cyclic) return (int32_t)(d.fastdiv ? key - div_fast(key, d.nparts, d.inv_p) * d.nparts : key % d.nparts);
  // largePartitionSize is an Int (smallPartitionSize + 1, :18): it wraps to Int.MinValue when
  // small partitions hold 2^31-1 keys, as on the JVM. .toInt of the index; a partitioner whose Int
  // sizes overflowed yields an index outside the partition array (ArrayIndexOutOfBoundsException
  // in the reference) -> rejected like a bad key
  const i64 large = (int32_t)((uint32_t)d.q + 1u);
  if (d.fastdiv) {  // (large > 0 here: fastdiv is off when the Int sum wrapped)
    const int32_t o = (int32_t)(uint32_t)(u64)(key < d.small_keys ? div_fast(key, d.q, d.inv_q)
                                                                   : (i64)d.n_small + div_fast(key - d.small_keys, large, d.inv_large));
    return o >= 0 && o < d.nparts ? o : -1;
  }
  const int32_t o = (int32_t)(uint32_t)(u64)(key < d.small_keys ? key / d.q : (i64)d.n_small + (key - d.small_keys) / large);
  return o >= 0 && o < d.nparts ? o : -1;
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

// Group ("slot") of a record: its owning partition, or slot_of[partition] when the caller orders
// the partitions differently (e.g. by hosting rank); nparts (the sentinel) for a bad key.
__device__ __forceinline__ int32_t slot_of_key(const RangeDesc& d, const int32_t* slot_of, i64 key) {
  const int32_t o = owner_of(d, key);
  if (o < 0) return -1;
  return slot_of ? slot_of[o] : o;
}

// The block's chunk is `rounds` x 256 consecutive records; owners outside [0, nparts) count as bad.
// (LDS: nparts counters, launch-sized, so small routes fit many blocks per CU; the chunk's keys are
// loaded kMinRounds at a time, all in flight together, before any is used)
__global__ __launch_bounds__(kRT) void route_hist(const i64* __restrict__ keys, i64 n, RangeDesc d,
                                                  const int32_t* __restrict__ slot_of, int nbits, int rounds,
                                                  u32* __restrict__ hist, i64 nblocks, u64* __restrict__ bad) {
  extern __shared__ u32 h[];
  const int lane = threadIdx.x & 63;
  for (int p = threadIdx.x; p < d.nparts; p += kRT) h[p] = 0;
  __syncthreads();
  const i64 base = (i64)blockIdx.x * rounds * kRT;
  for (int r0 = 0; r0 < rounds; r0 += kMinRounds) {
    i64 k[kMinRounds];
#pragma unroll
    for (int r = 0; r < kMinRounds; ++r) {  // clamped, unconditional: every load in flight at once
      const i64 i = base + (i64)(r0 + r) * kRT + threadIdx.x;
      k[r] = keys[i < n ? i : n - 1];
    }
#pragma unroll
    for (int r = 0; r < kMinRounds; ++r) {
      const i64 i = base + (i64)(r0 + r) * kRT + threadIdx.x;
      int32_t o = d.nparts;  // sentinel: past the end
      if (r0 + r < rounds && i < n) {
        o = slot_of_key(d, slot_of, k[r]);
        if (o < 0) { atomicMax(bad, ~(u64)i); o = d.nparts; }
      }
      const u64 m = match_owner(o, nbits);
      // the group's lowest lane adds the group size: one LDS atomic per distinct owner per wave
      if (o < d.nparts && (m & ((1ull << lane) - 1)) == 0) atomicAdd(&h[o], (u32)__popcll(m));
    }
  }
  __syncthreads();
  for (int p = threadIdx.x; p < d.nparts; p += kRT) hist[(i64)p * nblocks + blockIdx.x] = h[p];  // partition-major
}

// Send-order outputs of the fused route (each may be null): the record indices (order) and the
// records themselves -- keys, cols, and values of vsize bytes -- so no separate gather pass runs.
struct RouteOut {
  i64* order;
  i64* keys;
  int32_t* cols;
  void* vals;
  const int32_t* in_cols;
  const void* in_vals;
  int vsize;  // 4 or 8
  // added to each key written out, per slot (nullable): a partition's keys rebased to its place in
  // the receiving rank's slab (glint_route_gather_rebased_dev)
  const i64* key_delta;
};

__global__ __launch_bounds__(kRT) void route_scatter(const i64* __restrict__ keys, i64 n, RangeDesc d,
                                                     const int32_t* __restrict__ slot_of, int nbits, int rounds,
                                                     const u32* __restrict__ offs, i64 nblocks, RouteOut out) {
  extern __shared__ u32 cnt[];    // records of each owner this block has placed so far (nparts, launch-sized)
  __shared__ u32 grp_base[kRT];   // per group leader: the group's first slot within its owner
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int p = threadIdx.x; p < d.nparts; p += kRT) cnt[p] = 0;
  __syncthreads();
  const i64 base = (i64)blockIdx.x * rounds * kRT;
  for (int r = 0; r < rounds; ++r) {
    const i64 i = base + (i64)r * kRT + threadIdx.x;  // 256 consecutive records per round
    int32_t o = d.nparts;
    i64 key = 0;
    if (i < n) {
      key = keys[i];
      o = slot_of_key(d, slot_of, key);
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
      const i64 pos = (i64)offs[(i64)o * nblocks + blockIdx.x] + grp_base[wid * 64 + lead] + __popcll(below);
      if (out.order) out.order[pos] = i;
      if (out.keys) out.keys[pos] = key + (out.key_delta ? out.key_delta[o] : 0);
      if (out.cols) out.cols[pos] = out.in_cols[i];
      if (out.vals) {
        if (out.vsize == 8) reinterpret_cast<u64*>(out.vals)[pos] = reinterpret_cast<const u64*>(out.in_vals)[i];
        else reinterpret_cast<u32*>(out.vals)[pos] = reinterpret_cast<const u32*>(out.in_vals)[i];
      }
    }
    __syncthreads();  // grp_base is rewritten next round
  }
}

// route_scatter for nparts <= 64 (the exchange's shapes: P = world x partitions per rank): a block's
// 4096 records (16 rounds of 256, rounds == kMinRounds) are sorted by owner in LDS, stably, and each
// owner's run is written out contiguously -- the per-lane stores of route_scatter left one 8-64-byte
// segment per owner per wave instruction, and its wave-ordered claims took 5 barriers per round.
// Per (round, wave) each owner group's size goes into a table [owner][round x 4 + wave]; one exclusive
// scan of the table in that (owner-major) order gives every group its first position in the block's
// sorted order, so a record's position is its group's plus its rank in the group -- the order of
// (round, wave, lane) = the caller's order. The records then go through one LDS staging buffer per
// output (keys, values, cols, record indices).
constexpr int kSmallParts = 64;
constexpr int kSChunk = kMinRounds * kRT;  // 4096
__global__ __launch_bounds__(kRT) void route_scatter_small(const i64* __restrict__ keys, i64 n, RangeDesc d,
                                                           const int32_t* __restrict__ slot_of, int nbits,
                                                           const u32* __restrict__ offs, i64 nblocks, RouteOut out) {
  constexpr int R = kMinRounds, RW = R * (kRT / 64);  // (round, wave) groups per owner: 64
  static_assert(RW == 64, "one table row of 64 per owner");
  __shared__ u32 wc[kSmallParts * RW];
  __shared__ __attribute__((aligned(16))) u64 stage[kSChunk];
  __shared__ uint8_t ob[kSChunk];        // owner of each sorted position
  __shared__ u32 goff[kSmallParts + 1];  // per owner: its first output slot minus its first sorted position
  __shared__ u32 wt[kRT / 64];
  __shared__ i64 kd[kSmallParts];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const i64 base = (i64)blockIdx.x * kSChunk;
  const int np = d.nparts;
  if (tid < np) kd[tid] = out.key_delta ? out.key_delta[tid] : 0;
  i64 k[R];
  u64 v[R];
  int32_t c[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {  // every load of the chunk in flight at once (clamped, unconditional)
    const i64 i = base + (i64)r * kRT + tid;
    const i64 ic = i < n ? i : n - 1;
    k[r] = keys[ic];
    v[r] = 0;
    c[r] = 0;
    if (out.vals)  // (launch-uniform)
      v[r] = out.vsize == 8 ? reinterpret_cast<const u64*>(out.in_vals)[ic] : (u64)reinterpret_cast<const u32*>(out.in_vals)[ic];
    if (out.cols) c[r] = out.in_cols[ic];
  }
  for (int e = tid; e < np * RW; e += kRT) wc[e] = 0;
  __syncthreads();
  int32_t o[R];
  u32 rk[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const i64 i = base + (i64)r * kRT + tid;
    o[r] = np;  // sentinel: past the end, or a bad key (route_hist reported it)
    if (i < n) {
      const int32_t x = slot_of_key(d, slot_of, k[r]);
      if (x >= 0) o[r] = x;
    }
    const u64 m = match_owner(o[r], nbits);
    const u64 below = m & ((1ull << lane) - 1);
    rk[r] = (u32)__popcll(below);
    if (o[r] < np && below == 0) wc[o[r] * RW + r * (kRT / 64) + wid] = (u32)__popcll(m);
  }
  __syncthreads();
  // exclusive scan of the np x 64 table, owner-major: 16 entries per thread
  const int E = np * RW, per = (E + kRT - 1) / kRT, e0 = tid * per;
  u32 sum = 0;
  for (int j = 0; j < per; ++j) sum += e0 + j < E ? wc[e0 + j] : 0u;
  u32 incl = sum;
#pragma unroll
  for (int dd = 1; dd < 64; dd <<= 1) {
    const u32 y = __shfl_up(incl, dd);
    if (lane >= dd) incl += y;
  }
  if (lane == 63) wt[wid] = incl;
  __syncthreads();
  u32 run = incl - sum;
  for (int w = 0; w < wid; ++w) run += wt[w];
  for (int j = 0; j < per; ++j) {
    if (e0 + j < E) {
      const u32 x = wc[e0 + j];
      wc[e0 + j] = run;
      run += x;
    }
  }
  __syncthreads();
  u32 total = 0;
  for (int w = 0; w < kRT / 64; ++w) total += wt[w];
  if (tid < np) goff[tid] = offs[(i64)tid * nblocks + blockIdx.x] - wc[tid * RW];
  u32 pos[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    pos[r] = o[r] < np ? wc[o[r] * RW + r * (kRT / 64) + wid] + rk[r] : 0u;
    if (o[r] < np) ob[pos[r]] = (uint8_t)o[r];
  }
  __syncthreads();
  // one output at a time: the chunk's records into their sorted positions, then each owner's run
  // written out as it lies (consecutive threads, consecutive slots)
  auto emit = [&](auto val, auto* dst) {
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (o[r] < np) stage[pos[r]] = (u64)val(r);
    __syncthreads();
    for (u32 x = tid; x < total; x += kRT) {
      typedef typename std::remove_pointer<decltype(dst)>::type T;
      dst[goff[ob[x]] + x] = (T)stage[x];
    }
    __syncthreads();
  };
  if (out.keys) emit([&](int r) { return (u64)(k[r] + kd[o[r]]); }, out.keys);
  if (out.vals) {
    if (out.vsize == 8) emit([&](int r) { return v[r]; }, reinterpret_cast<u64*>(out.vals));
    else emit([&](int r) { return v[r]; }, reinterpret_cast<u32*>(out.vals));
  }
  if (out.cols) emit([&](int r) { return (u64)(u32)c[r]; }, out.cols);
  if (out.order) emit([&](int r) { return (u64)(base + (i64)r * kRT + tid); }, out.order);
}

// ---- the (partition, block) offsets -------------------------------------------------------------
// hist is partition-major: row p = the records of partition p in each block. The offset of (p, b) is
// the records of partitions < p plus those of p in blocks < b: a row total per partition, then per
// partition a base (the totals before it) and the exclusive scan of its row. Two small launches, no
// scan library; every value stays on the device.
constexpr int kST = 1024;  // threads of the offset kernels

__device__ __forceinline__ u32 block_reduce_u32(u32 x) {
  __shared__ u32 ws[kST / 64];
  for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = x;
  __syncthreads();
  u32 t = 0;
#pragma unroll
  for (int w = 0; w < kST / 64; ++w) t += ws[w];
  __syncthreads();
  return t;
}

// tot[p] = records of partition p (the route's counts, too)
__global__ __launch_bounds__(kST) void route_row_sums(const u32* __restrict__ hist, i64 nblocks, u32* __restrict__ tot,
                                                      i64* __restrict__ counts) {
  const u32* row = hist + (i64)blockIdx.x * nblocks;
  u32 x = 0;
  for (i64 b = threadIdx.x; b < nblocks; b += kST) x += row[b];
  x = block_reduce_u32(x);
  if (threadIdx.x == 0) {
    tot[blockIdx.x] = x;
    counts[blockIdx.x] = x;
  }
}

// offs[p][b] = sum(tot[0..p)) + sum(hist[p][0..b)): one block per partition, the row in tiles of
// kST x 4 values (each thread scans its 4, a wave scan, the waves' totals, then the carry)
__global__ __launch_bounds__(kST) void route_row_scan(const u32* __restrict__ hist, i64 nblocks,
                                                      const u32* __restrict__ tot, u32* __restrict__ offs) {
  __shared__ u32 wt[kST / 64];
  const int p = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  u32 base = 0;
  for (int q = tid; q < p; q += kST) base += tot[q];
  base = block_reduce_u32(base);
  const u32* row = hist + (i64)p * nblocks;
  u32* out = offs + (i64)p * nblocks;
  constexpr int PER = 4;
  u32 carry = base;
  for (i64 t0 = 0; t0 < nblocks; t0 += (i64)kST * PER) {
    const i64 b0 = t0 + (i64)tid * PER;
    u32 v[PER], sum = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      v[j] = b0 + j < nblocks ? row[b0 + j] : 0u;
      sum += v[j];
    }
    u32 incl = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const u32 y = __shfl_up(incl, d);
      if (lane >= d) incl += y;
    }
    if (lane == 63) wt[wid] = incl;
    __syncthreads();
    u32 run = carry + incl - sum, all = 0;
#pragma unroll
    for (int w = 0; w < kST / 64; ++w) {
      const u32 y = wt[w];
      run += w < wid ? y : 0u;
      all += y;
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (b0 + j < nblocks) out[b0 + j] = run;
      run += v[j];
    }
    carry += all;
    __syncthreads();
  }
}

// ---- route scratch: one per (device, stream) ------------------------------------------------------
// Routes on one stream run in stream order, so they can share a buffer once their kernels are on the
// stream; routes on different streams of one device may run at the same time and get their own. A
// caller holds its buffer's lock from taking it until its kernels are enqueued (host threads sharing
// a stream would otherwise interleave their launches on one buffer). A buffer grows only after its
// stream has drained. At most kMaxScratch streams per device keep a buffer: the least recently used
// idle one is released to make room, after the event its last route recorded (never a device-wide
// sync: that would stall every shard's pushes on the device, and the victim's stream may be gone).
constexpr int kMaxDevices = 64;
constexpr size_t kMaxScratch = 64;
constexpr size_t kBadWordOffset = 0;  // the synchronous route's status word: the buffer's first 256 B
struct RouteScratch {
  std::mutex use;  // held while a caller enqueues work on this buffer
  void* tmp = nullptr;
  size_t bytes = 0;
  u64 used = 0;    // last use (LRU)
  hipEvent_t done = nullptr;  // recorded after the last route's kernels on this buffer
  bool recorded = false;
};
std::mutex g_scratch_mu;
std::map<std::pair<int, hipStream_t>, std::unique_ptr<RouteScratch>> g_scratch;
u64 g_scratch_clock = 0;

// The scratch of (dev, st), at least `need` bytes past its status word, LOCKED for the caller (who
// unlocks it once its kernels are enqueued); nullptr on failure (unlocked).
RouteScratch* route_scratch(int dev, hipStream_t st, size_t need) {
  RouteScratch* sc;
  {
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    auto& slot = g_scratch[{dev, st}];
    if (!slot) slot.reset(new RouteScratch());
    sc = slot.get();
    sc->used = ++g_scratch_clock;
    size_t on_dev = 0;
    for (auto& kv : g_scratch) on_dev += kv.first.first == dev;
    if (on_dev > kMaxScratch) {  // release the least recently used idle buffer of this device
      auto victim = g_scratch.end();
      for (auto it = g_scratch.begin(); it != g_scratch.end(); ++it)
        if (it->first.first == dev && it->second.get() != sc &&
            (victim == g_scratch.end() || it->second->used < victim->second->used))
          victim = it;
      if (victim != g_scratch.end() && victim->second->use.try_lock()) {
        RouteScratch* v = victim->second.get();
        if (v->recorded) (void)hipEventSynchronize(v->done);  // its last route has finished with it
        (void)hipFree(v->tmp);
        if (v->done) (void)hipEventDestroy(v->done);
        (void)hipGetLastError();
        v->use.unlock();
        g_scratch.erase(victim);
      }
    }
  }
  sc->use.lock();
  need += 256;  // the status word
  if (sc->bytes < need) {
    if (sc->tmp) {  // earlier routes on this stream may still read the old buffer
      (void)hipStreamSynchronize(st);
      (void)hipFree(sc->tmp);
    }
    sc->tmp = nullptr;
    sc->bytes = 0;
    if (hipMalloc(&sc->tmp, need) != hipSuccess) {
      (void)hipGetLastError();
      sc->use.unlock();
      return nullptr;
    }
    sc->bytes = need;
  }
  return sc;
}

struct DevGuard {
  int prev = -1;
  bool ok = false;
  explicit DevGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DevGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// One partition and no output: the batch is its own send buffer, so the pass only checks the keys
// (owner_of: 0 <= key < nkeys for either kind when nparts == 1) -- a streaming read -- and sets
// counts[0] = n (the exchange sends nothing when a key is bad, so the count matters only when all
// are good).
__global__ __launch_bounds__(256) void route_validate(const i64* __restrict__ keys, i64 n, i64 nkeys,
                                                      i64* counts, u64* bad) {
  u64 b = 0;
  const i64 stride = (i64)gridDim.x * 256 * 2;
  for (i64 i = ((i64)blockIdx.x * 256 + threadIdx.x) * 2; i < n; i += stride) {
    if (i + 1 < n) {
      typedef __attribute__((ext_vector_type(2))) long long KP;
      const KP k = __builtin_nontemporal_load(reinterpret_cast<const KP*>(keys + i));
      if (k.y < 0 || k.y >= nkeys) b = max(b, ~(u64)(i + 1));
      if (k.x < 0 || k.x >= nkeys) b = max(b, ~(u64)i);
    } else {
      const i64 k = keys[i];
      if (k < 0 || k >= nkeys) b = max(b, ~(u64)i);
    }
  }
  for (int d = 32; d > 0; d >>= 1) b = max(b, (u64)__shfl_xor((unsigned long long)b, d));
  if ((threadIdx.x & 63) == 0 && b) atomicMax((unsigned long long*)bad, (unsigned long long)b);
  if (blockIdx.x == 0 && threadIdx.x == 0) counts[0] = n;
}

// Launches the route (histogram, scan, scatter, counts) on `st`; the first bad record (~index, 0 =
// none) lands in the device word *bad_dev (nullptr: the scratch's own status word, and the scratch
// stays locked for the caller, who reads the word after a sync and unlocks `*held`). No host
// synchronisation.
int route_launch(const int64_t* keys, int64_t n, int kind, int32_t nparts, int64_t nkeys, const int32_t* slot_of,
                 int64_t* counts, const RouteOut& out, uint64_t* bad_dev, hipStream_t st,
                 RouteScratch** held = nullptr) {
  if (kind != GLINT_ROUTE_RANGE && kind != GLINT_ROUTE_CYCLIC) return GLINT_EINVAL;
  if (nparts <= 0 || nparts > kMaxParts || n < 0 || nkeys < 0 || !counts || (!bad_dev && !held)) return GLINT_EINVAL;
  if (n > 0 && !keys) return GLINT_EINVAL;
  if (n >= ((i64)1 << 32)) return GLINT_EINVAL;  // 32-bit offsets
  if (out.vals && out.vsize != 4 && out.vsize != 8) return GLINT_EINVAL;
  if (n > 0 && ((out.vals && !out.in_vals) || (out.cols && !out.in_cols))) return GLINT_EINVAL;
  int dev = 0;
  if (st ? hipStreamGetDevice(st, &dev) != hipSuccess : hipGetDevice(&dev) != hipSuccess) {
    (void)hipGetLastError();
    return GLINT_EDEVICE;
  }
  if (dev < 0 || dev >= kMaxDevices) return GLINT_EDEVICE;
  DevGuard guard(dev);
  if (!guard.ok) return GLINT_EDEVICE;
  // RangePartitioner.apply (RangePartitioner.scala:62-84) -- same Int truncation of the sizes
  RangeDesc d{};
  const int32_t n_large = (int32_t)(nkeys % nparts);
  d.n_small = nparts - n_large;
  d.q = (int32_t)((nkeys - nkeys % nparts) / nparts);
  d.small_keys = (i64)d.n_small * (i64)d.q;
  d.nkeys = nkeys;
  d.nparts = nparts;
  d.cyclic = kind == GLINT_ROUTE_CYCLIC;
  {
    const i64 large = (int32_t)((uint32_t)d.q + 1u);
    d.fastdiv = nkeys <= ((i64)1 << 52) && (d.cyclic || (d.q > 0 && large > 0)) ? 1 : 0;
    d.inv_q = d.q > 0 ? 1.0 / (double)d.q : 0.0;
    d.inv_large = large > 0 ? 1.0 / (double)large : 0.0;
    d.inv_p = 1.0 / (double)nparts;
  }
  // chunk per block grows with nparts so the (partition x block) histogram stays <= n/4 entries
  const int rounds = std::max<int>(kMinRounds, (4 * nparts + kRT - 1) / kRT);
  const i64 chunk = (i64)rounds * kRT;
  const i64 nblocks = std::max<i64>(1, (n + chunk - 1) / chunk);
  int nbits = 1;
  while ((1 << nbits) <= nparts) ++nbits;  // owners and the sentinel nparts fit in nbits
  const size_t hist_bytes = ((size_t)nparts * nblocks * 4 + 255) & ~(size_t)255;
  const size_t need = 2 * hist_bytes + (size_t)kMaxParts * 4;
  RouteScratch* sc = route_scratch(dev, st, need);
  if (!sc) return GLINT_ENOMEM;
  // the buffer stays locked until this call's kernels are on the stream (or, held, for the caller);
  // its event marks the end of this call's use, for an eviction from another stream
  struct Unlock {
    RouteScratch* sc;
    hipStream_t st;
    bool keep;
    ~Unlock() {
      if (!sc->done && hipEventCreateWithFlags(&sc->done, hipEventDisableTiming) != hipSuccess) sc->done = nullptr;
      sc->recorded = sc->done && hipEventRecord(sc->done, st) == hipSuccess;
      (void)hipGetLastError();
      if (!keep) sc->use.unlock();
    }
  } unlock{sc, st, held != nullptr};
  if (held) *held = sc;
  char* b = (char*)sc->tmp + 256;
  if (!bad_dev) bad_dev = (uint64_t*)((char*)sc->tmp + kBadWordOffset);
  u32* hist = (u32*)b;
  u32* offs = (u32*)(b + hist_bytes);
  u32* tot = (u32*)(b + 2 * hist_bytes);
  if (hipMemsetAsync(bad_dev, 0, 8, st) != hipSuccess) return GLINT_EDEVICE;
  if (nparts == 1 && !out.order && !out.keys && !out.cols && !out.vals && n > 0 &&
      ((uintptr_t)keys & 15) == 0) {
    const unsigned g = (unsigned)std::max<i64>(1, std::min<i64>((n / 2 + 255) / 256, 1024));
    route_validate<<<g, 256, 0, st>>>(keys, n, nkeys, counts, bad_dev);
    return hipGetLastError() == hipSuccess ? GLINT_OK : GLINT_EDEVICE;
  }
  if (n == 0) {
    if (hipMemsetAsync(counts, 0, (size_t)nparts * 8, st) != hipSuccess) return GLINT_EDEVICE;
  } else {
    route_hist<<<(unsigned)nblocks, kRT, (size_t)nparts * 4, st>>>(keys, n, d, slot_of, nbits, rounds, hist, nblocks,
                                                                 bad_dev);
    route_row_sums<<<(unsigned)nparts, kST, 0, st>>>(hist, nblocks, tot, counts);
    // no output requested (a single partition: the batch is its own send buffer): counts and the
    // status word only
    if (out.order || out.keys || out.cols || out.vals) {
      route_row_scan<<<(unsigned)nparts, kST, 0, st>>>(hist, nblocks, tot, offs);
      static const bool small_off = [] {
        const char* e = getenv("GLINT_ROUTE_SMALL");  // 0: the general scatter at every size (A/B)
        return e && atoi(e) == 0;
      }();
      if (nparts <= kSmallParts && rounds == kMinRounds && !small_off)
        route_scatter_small<<<(unsigned)nblocks, kRT, 0, st>>>(keys, n, d, slot_of, nbits, offs, nblocks, out);
      else
        route_scatter<<<(unsigned)nblocks, kRT, (size_t)nparts * 4, st>>>(keys, n, d, slot_of, nbits, rounds, offs,
                                                                           nblocks, out);
    }
  }
  if (hipGetLastError() != hipSuccess) return GLINT_EDEVICE;
  return GLINT_OK;
}

}  // namespace

extern "C" int glint_route_dev(const int64_t* keys, int64_t n, int kind, int32_t nparts, int64_t nkeys,
                               int64_t* counts, int64_t* order, int64_t* first_bad, void* stream) {
  if (!first_bad || (n > 0 && !order)) return GLINT_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  RouteOut out{};
  out.order = order;
  // the status word is the scratch's own; the scratch stays locked until the call has read it
  RouteScratch* held = nullptr;
  int rc = route_launch(keys, n, kind, nparts, nkeys, nullptr, counts, out, nullptr, st, &held);
  if (!held) return rc;
  uint64_t enc = 0;
  if (rc == GLINT_OK && (hipMemcpyAsync(&enc, held->tmp, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
                         hipStreamSynchronize(st) != hipSuccess)) {
    (void)hipGetLastError();
    rc = GLINT_EDEVICE;
  }
  held->use.unlock();
  if (rc) return rc;
  *first_bad = enc ? (int64_t)~enc : -1;
  return enc ? GLINT_EOUTOFRANGE : GLINT_OK;
}

extern "C" int glint_route_gather_rebased_dev(const int64_t* keys, const int32_t* cols, const void* vals, int vsize,
                                              int64_t n, int kind, int32_t nparts, int64_t nkeys, const int32_t* slot_of,
                                              const int64_t* key_delta, int64_t* counts, int64_t* order,
                                              int64_t* out_keys, int32_t* out_cols, void* out_vals, uint64_t* bad_dev,
                                              void* stream) {
  if (!key_delta || (!out_keys && n > 0) || nparts <= 1) return GLINT_EINVAL;  // (one partition: no scatter pass to rebase in)
  RouteOut out{};
  out.order = order;
  out.keys = out_keys;
  out.cols = out_cols;
  out.vals = out_vals;
  out.in_cols = cols;
  out.in_vals = vals;
  out.vsize = vsize;
  out.key_delta = key_delta;
  return route_launch(keys, n, kind, nparts, nkeys, slot_of, counts, out, bad_dev, (hipStream_t)stream);
}

extern "C" int glint_route_gather_dev(const int64_t* keys, const int32_t* cols, const void* vals, int vsize, int64_t n,
                                      int kind, int32_t nparts, int64_t nkeys, const int32_t* slot_of, int64_t* counts,
                                      int64_t* order, int64_t* out_keys, int32_t* out_cols, void* out_vals,
                                      uint64_t* bad_dev, void* stream) {
  RouteOut out{};
  out.order = order;
  out.keys = out_keys;
  out.cols = out_cols;
  out.vals = out_vals;
  out.in_cols = cols;
  out.in_vals = vals;
  out.vsize = vsize;
  return route_launch(keys, n, kind, nparts, nkeys, slot_of, counts, out, bad_dev, (hipStream_t)stream);
}
