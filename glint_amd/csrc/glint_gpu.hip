// glint_gpu.hip -- MI355X (gfx950) implementation of include/glint_gpu.h.
//
// Device side: the shard loops of Glint's partial models
//   PartialVector.update / get          src/main/scala/glint/models/server/PartialVector.scala:35-60
//   PartialMatrix.update / get / getRows src/main/scala/glint/models/server/PartialMatrix.scala:37-83
// as hand-written HIP kernels (see glint_kernels.h for the push design).
// Host side: the C ABI (shard lifetime, host-pointer and device-pointer entry points, wire
// ingest of RequestSerializer payloads, src/main/scala/glint/serialization/RequestSerializer.scala).
//
// There is no CPU fallback anywhere in this library: without a GPU every entry point that touches
// a shard returns GLINT_EDEVICE.
#include "glint_kernels.h"
#include "../../include/glint_gpu.h"
#include "glint_device.h"

#include <mutex>
#include <vector>
#include <utility>
#include <new>
#include <chrono>
#include <cstring>
#include <sched.h>
#include <time.h>
#include <cstdio>
#include <algorithm>
#include <cstdlib>

namespace glint {

// ------------------------------------------------------------------------------------------------
// push, ordered part: push_check + push_apply
// ------------------------------------------------------------------------------------------------
// addresses are element indices: int32 for vectors (Partition.globalToLocal is an Int), int64 for
// matrices (row * pitch + col)
template <bool MAT> struct AddrT { typedef int32_t T; };
template <> struct AddrT<true> { typedef i64 T; };

template <bool MAT, int KIND = -1>
__device__ __forceinline__ bool rec_addr_t(const PartDesc& p, i64 key, int32_t col, typename AddrT<MAT>::T& addr) {
  i64 ad;
  const bool ok = rec_addr<MAT, KIND>(p, key, col, ad);
  addr = (typename AddrT<MAT>::T)ad;
  return ok;
}

// push_check: reads every key (and col) once, 8 (12) B/record, and per wave tile of kTile records
//   - finds the first tile whose record addresses stop being strictly increasing (within the tile
//     or against the record before it) -> LaunchCtl.brk_enc;
//   - writes the tile's descriptor: its first address when the tile is AFFINE (record r of the tile
//     hits element base + r, every record in range), else kNotAffine.
// Waves work independently (no barriers) and stop once a break before their tile is known, so an
// unordered push costs about one wave tile of reads per wave. Full tiles take a branch-free path
// (a per-element bounds test would make hipcc wait for each load before issuing the next).
template <bool MAT, bool FULL, int KIND>
__device__ __forceinline__ bool check_tile(const i64* __restrict__ keys, const int32_t* __restrict__ cols, i64 n,
                                           const PartDesc& part, LaunchCtl* ctl, i64* __restrict__ desc,
                                           u32 ntiles, u32 t, int lane, bool validate, bool read_all) {
  typedef typename AddrT<MAT>::T A;
  const i64 pbase = (i64)t * (kTile / 2);
  K2 k[kPPT];
  C2 c[kPPT];
#pragma unroll
  for (int j = 0; j < kPPT; ++j) {
    const i64 p = pbase + lane + (i64)j * 64;
    const i64 r = 2 * p;
    if (FULL || r + 1 < n) {
      k[j] = __builtin_nontemporal_load(reinterpret_cast<const K2*>(keys) + p);
      if (MAT) c[j] = __builtin_nontemporal_load(reinterpret_cast<const C2*>(cols) + p);
    } else {
      k[j] = K2{r < n ? keys[r] : 0, 0};
      if (MAT) c[j] = C2{r < n ? cols[r] : 0, 0};
    }
  }
  const i64 r_first = 2 * pbase;
  const i64 kb = r_first > 0 ? keys[r_first - 1] : 0;  // the record before this tile
  const int32_t cb = (MAT && r_first > 0) ? cols[r_first - 1] : 0;
  // stop once a break before this tile is known (read after the loads are in flight)
  // (a validating push reads every tile: its records are checked before anything is applied; a tile
  // past a known break is only validated -- its order and descriptor no longer matter, and every such
  // tile adding to brk_enc would serialise on that one word)
  const u32 brk = __builtin_amdgcn_readfirstlane(ld_relaxed(&ctl->brk_enc));
  const bool after = brk != 0u && ntiles - brk < t;
  if (!read_all && after) return false;
  A before = 0;
  if (r_first > 0) rec_addr_t<MAT, KIND>(part, kb, cb, before);
  bool mono = true, affine = true;
  A a_first = 0;
  A last = before;
#pragma unroll
  for (int j = 0; j < kPPT; ++j) {
    const i64 r = 2 * (pbase + lane + (i64)j * 64);
    const bool h0 = FULL || r < n, h1 = FULL || r + 1 < n;
    A a0, a1;
    const bool o0 = rec_addr_t<MAT, KIND>(part, k[j].x, MAT ? c[j].x : 0, a0);
    const bool o1 = rec_addr_t<MAT, KIND>(part, k[j].y, MAT ? c[j].y : 0, a1);
    if (j == 0) a_first = __shfl(a0, 0);
    if (h1) mono = mono && (a1 > a0);
    A prev = __shfl_up(a1, 1);
    if (lane == 0) prev = last;
    if (h0 && r > 0) mono = mono && (a0 > prev);
    last = __shfl(a1, 63);
    const A off = (A)(r - r_first);
    affine = affine && (!h0 || (o0 && a0 == a_first + off)) && (!h1 || (o1 && a1 == a_first + off + 1));
    if (validate) {  // the raw keys too (no Int wrap); rare: one atomic per lane with a rejected record
      const bool b0 = h0 && (!o0 || !key_in_part<KIND>(part, k[j].x));
      const bool b1 = h1 && (!o1 || !key_in_part<KIND>(part, k[j].y));
      if (b0 || b1) atomicMax(&ctl->bad, ~(u64)(b0 ? r : r + 1));
    }
  }
  const bool any_bad = __any(!mono);  // wave-wide votes, outside any lane-divergent branch
  const bool all_affine = __all(affine);
  if (lane == 0 && !after) {
    if (any_bad) {  // (an earlier break already recorded: no atomic -- every wave of an unordered push gets here)
      if (ld_relaxed(&ctl->brk_enc) < ntiles - t) atomicMax(&ctl->brk_enc, ntiles - t);
    } else {
      desc[t] = all_affine ? (i64)a_first : kNotAffine;
      // the push is ONE affine run iff every tile is affine and continues its predecessor; only a
      // tile that breaks the run writes the shared flag (after a relaxed read: it flips once)
      const bool linked = all_affine && (r_first == 0 || (i64)a_first == (i64)before + 1);
      if (!linked && ld_relaxed(&ctl->nonaffine) == 0u) atomicOr(&ctl->nonaffine, 1u);
    }
  }
  return true;
}

// One launch covers the wave tiles [t_begin, t_end) (a push is checked in windows of tiles, see
// sweep_window_tiles); the first window's launch also zeroes the next push's control words.
// validate: 0 none; 1 every record of the push (every tile is read); 2 the records of the tiles it
// reads, which stop after the break as for an ordinary push (a binned tail is validated by its count
// pass, bin_count_kernel<..., VALIDATE>)
template <bool MAT, int KIND>
__global__ __launch_bounds__(kTPB) void push_check_kernel(const i64* __restrict__ keys,
                                                          const int32_t* __restrict__ cols, i64 n,
                                                          PartDesc part, LaunchCtl* ctl, LaunchCtl* next,
                                                          i64* __restrict__ desc, u32 ntiles, u32 t_begin,
                                                          u32 t_end, int validate) {
  const int lane = threadIdx.x & 63;
  if (t_begin == 0 && blockIdx.x == 0 && threadIdx.x == 0) {  // the next push's control words (no kernel of this push reads them)
    next->brk_enc = 0u;
    next->nonaffine = 0u;
    next->cancel = 0u;
    next->bad = 0ull;
  }
  if (ctl->cancel) return;  // a cancelled gated push: brk_enc stays 0, so no tail either
  const u32 w0 = blockIdx.x * (kTPB / 64) + (threadIdx.x >> 6);
  const u32 nw = gridDim.x * (kTPB / 64);
  for (u32 t = t_begin + w0; t < t_end; t += nw) {
    const bool full = 2 * ((i64)t * (kTile / 2)) + kTile <= n;
    const bool go = full ? check_tile<MAT, true, KIND>(keys, cols, n, part, ctl, desc, ntiles, t, lane, validate != 0,
                                                       validate == 1)
                         : check_tile<MAT, false, KIND>(keys, cols, n, part, ctl, desc, ntiles, t, lane, validate != 0,
                                                        validate == 1);
    if (!go) return;
  }
}

// push_apply: wave tiles before the break, plain read-modify-write. Their addresses are strictly
// increasing across the whole prefix, hence unique, so no two lanes touch one element.
//   affine tile: the addresses are base + r -- values and shard elements are streamed with no
//                dependent load (the keys were read once, by push_check); 16 B per lane per pair
//                when base is even;
//   other tiles: keys re-read, addresses recomputed (range errors recorded here), dependent RMW,
//                16 B per pair of adjacent aligned elements.
template <typename V, bool MAT, bool FULL>
__device__ __forceinline__ void apply_affine(const PushArgs<V>& a, i64 pbase, i64 base, int lane) {
  typedef typename Vec2<V>::T V2;
  const i64 n = a.n;
  const i64 r_first = 2 * pbase;
  V2 v[kPPT], d[kPPT];
  if ((base & 1) == 0) {
    V2* dp = reinterpret_cast<V2*>(a.data + base);  // tile pair q -> element pair base + 2q
#pragma unroll
    for (int j = 0; j < kPPT; ++j) {
      const i64 q = lane + (i64)j * 64;
      if (FULL || 2 * (pbase + q) + 1 < n) {
        v[j] = __builtin_nontemporal_load(reinterpret_cast<const V2*>(a.vals) + pbase + q);
        d[j] = dp[q];
      }
    }
#pragma unroll
    for (int j = 0; j < kPPT; ++j) {
      const i64 q = lane + (i64)j * 64;
      const i64 r = 2 * (pbase + q);
      if (FULL || r + 1 < n) dp[q] = as2<V>(vadd((V)d[j].x, (V)v[j].x), vadd((V)d[j].y, (V)v[j].y));
      else if (r < n) a.data[base + (r - r_first)] = vadd(a.data[base + (r - r_first)], a.vals[r]);
    }
  } else {
#pragma unroll
    for (int j = 0; j < kPPT; ++j) {
      const i64 p = pbase + lane + (i64)j * 64;
      const i64 r = 2 * p;
      const i64 e = base + (r - r_first);
      if (FULL || r + 1 < n) {
        v[j] = __builtin_nontemporal_load(reinterpret_cast<const V2*>(a.vals) + p);
        d[j] = as2<V>(a.data[e], a.data[e + 1]);
      } else {
        v[j] = as2<V>(r < n ? a.vals[r] : V(0), V(0));
        d[j] = as2<V>(r < n ? a.data[e] : V(0), V(0));
      }
    }
#pragma unroll
    for (int j = 0; j < kPPT; ++j) {
      const i64 r = 2 * (pbase + lane + (i64)j * 64);
      const i64 e = base + (r - r_first);
      if (FULL || r < n) a.data[e] = vadd((V)d[j].x, (V)v[j].x);
      if (FULL || r + 1 < n) a.data[e + 1] = vadd((V)d[j].y, (V)v[j].y);
    }
  }
}

template <typename V, bool MAT, bool FULL>
__device__ __forceinline__ void apply_general(const PushArgs<V>& a, i64 pbase, int lane) {
  typedef typename Vec2<V>::T V2;
  typedef typename AddrT<MAT>::T A;
  const i64 n = a.n;
  K2 k[kPPT];
  C2 c[kPPT];
  V2 v[kPPT];
#pragma unroll
  for (int j = 0; j < kPPT; ++j) {
    const i64 p = pbase + lane + (i64)j * 64;
    const i64 r = 2 * p;
    if (FULL || r + 1 < n) {
      k[j] = __builtin_nontemporal_load(reinterpret_cast<const K2*>(a.keys) + p);
      if (MAT) c[j] = __builtin_nontemporal_load(reinterpret_cast<const C2*>(a.cols) + p);
      v[j] = __builtin_nontemporal_load(reinterpret_cast<const V2*>(a.vals) + p);
    } else {
      k[j] = K2{r < n ? a.keys[r] : 0, 0};
      if (MAT) c[j] = C2{r < n ? a.cols[r] : 0, 0};
      v[j] = as2<V>(r < n ? a.vals[r] : V(0), V(0));
    }
  }
#pragma unroll
  for (int j = 0; j < kPPT; ++j) {
    const i64 r = 2 * (pbase + lane + (i64)j * 64);
    A a0, a1;
    const bool h0 = FULL || r < n, h1 = FULL || r + 1 < n;
    const bool o0 = rec_addr_t<MAT>(a.part, k[j].x, MAT ? c[j].x : 0, a0) && h0;
    const bool o1 = rec_addr_t<MAT>(a.part, k[j].y, MAT ? c[j].y : 0, a1) && h1;
    if (h0 && !o0) record_error(a.err, r);
    if (h1 && !o1) record_error(a.err, r + 1);
    if (o0 && o1 && a1 == a0 + 1 && (a0 & 1) == 0) {
      V2* dp = reinterpret_cast<V2*>(a.data + a0);
      const V2 d = *dp;
      *dp = as2<V>(vadd((V)d.x, (V)v[j].x), vadd((V)d.y, (V)v[j].y));
    } else {
      if (o0) a.data[a0] = vadd(a.data[a0], (V)v[j].x);
      if (o1) a.data[a1] = vadd(a.data[a1], (V)v[j].y);
    }
  }
}

// The whole push is one affine run (element = record + delta): a grid-stride sweep over record
// pairs, so the grid reads one compact window of the value and shard streams at a time and no
// load depends on another (the keys were read once, by push_check). Only the first
// a.sweep_blocks blocks take part (about one per CU): this 2-read + 1-write stream runs fastest
// with ~16 KiB of loads in flight per CU and every access non-temporal (tools/microbench_stream.hip:
// 6.2 TB/s, against 5.7 TB/s at twice the waves with cached shard accesses).
constexpr int kSweepU = 2;  // record pairs per lane per iteration
template <typename V, bool EVEN>
__device__ __forceinline__ void apply_sweep(const PushArgs<V>& a, i64 delta, i64 p_begin, i64 p_end, bool last) {
  typedef typename Vec2<V>::T V2;
  if (blockIdx.x >= a.sweep_blocks) return;
  const i64 npairs = p_end;
  const i64 stride = (i64)a.sweep_blocks * kTPB;
  const V2* vp = reinterpret_cast<const V2*>(a.vals);
  i64 p = p_begin + (i64)blockIdx.x * kTPB + threadIdx.x;
  if (EVEN) {
    V2* dp = reinterpret_cast<V2*>(a.data + delta);  // pair p -> element pair delta + 2p
    for (; p + (kSweepU - 1) * stride < npairs; p += kSweepU * stride) {
      V2 v[kSweepU], d[kSweepU];
#pragma unroll
      for (int j = 0; j < kSweepU; ++j) {
        v[j] = __builtin_nontemporal_load(vp + p + j * stride);
        d[j] = __builtin_nontemporal_load(dp + p + j * stride);
      }
#pragma unroll
      for (int j = 0; j < kSweepU; ++j)
        __builtin_nontemporal_store(as2<V>(vadd((V)d[j].x, (V)v[j].x), vadd((V)d[j].y, (V)v[j].y)), dp + p + j * stride);
    }
    for (; p < npairs; p += stride) {
      const V2 v = __builtin_nontemporal_load(vp + p);
      const V2 d = __builtin_nontemporal_load(dp + p);
      __builtin_nontemporal_store(as2<V>(vadd((V)d.x, (V)v.x), vadd((V)d.y, (V)v.y)), dp + p);
    }
  } else {
    for (; p < npairs; p += stride) {
      const V2 v = __builtin_nontemporal_load(vp + p);
      const i64 e = 2 * p + delta;
      const V d0 = a.data[e], d1 = a.data[e + 1];
      a.data[e] = vadd(d0, (V)v.x);
      a.data[e + 1] = vadd(d1, (V)v.y);
    }
  }
  // the odd record belongs to the last window only: with n = k * 2^26 + 1 an earlier window also
  // ends at pair n >> 1 (its tiles cover every pair), so p_end alone cannot tell them apart
  if ((a.n & 1) && last && blockIdx.x == 0 && threadIdx.x == 0) {
    const i64 e = a.n - 1 + delta;
    a.data[e] = vadd(a.data[e], a.vals[a.n - 1]);
  }
}

// One launch covers the wave tiles [t_begin, t_end) of the push (a window, see sweep_window_tiles).
template <typename V, bool MAT>
__global__ __launch_bounds__(kTPB) void push_apply_kernel(PushArgs<V> a, const i64* __restrict__ desc, u32 t_begin,
                                                          u32 t_end) {
  if (a.ctl->cancel) return;  // a gated push whose gate was set applies nothing (and leaves the hint)
  const u32 brk = a.ctl->brk_enc;  // written by push_check; ordered by the kernel boundary
  if (t_begin == 0 && blockIdx.x == 0 && threadIdx.x == 0 && a.hint) {  // for the host's next push: how unordered was this one?
    __hip_atomic_store(a.hint, brk == 0u ? 0ull : (u64)(a.n - (i64)(a.ntiles - brk) * kTile), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(a.hint + 3, brk == 0u ? (u64)a.n : (u64)(a.ntiles - brk) * kTile, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);  // ... and where its tail started
  }
  if (brk == 0u && a.ctl->nonaffine == 0u) {
    const i64 delta = desc[0];  // tile 0 starts the run at record 0
    const i64 p0 = (i64)t_begin * (kTile / 2), p1 = min((i64)t_end * (kTile / 2), a.n >> 1);
    const bool last = t_end >= a.ntiles;
    if ((delta & 1) == 0) apply_sweep<V, true>(a, delta, p0, p1, last);
    else apply_sweep<V, false>(a, delta, p0, p1, last);
    return;
  }
  const u32 tiles = min(t_end, brk == 0u ? a.ntiles : a.ntiles - brk);
  const int lane = threadIdx.x & 63;
  const u32 w0 = blockIdx.x * (kTPB / 64) + (threadIdx.x >> 6);
  const u32 nw = gridDim.x * (kTPB / 64);
  i64 dbatch = kNotAffine;  // descriptors of this wave's next 64 tiles, one per lane
  for (u32 t = t_begin + w0, it = 0; t < tiles; t += nw, ++it) {
    if ((it & 63) == 0) {  // one load per 64 tiles instead of a dependent load per tile
      const i64 tt = (i64)t + (i64)lane * nw;
      dbatch = tt < (i64)tiles ? desc[tt] : kNotAffine;
    }
    const i64 pbase = (i64)t * (kTile / 2);
    const i64 base = __shfl(dbatch, (int)(it & 63));  // wave-uniform
    const bool full = 2 * pbase + kTile <= a.n;
    if (base != kNotAffine) {
      if (full) apply_affine<V, MAT, true>(a, pbase, base, lane);
      else apply_affine<V, MAT, false>(a, pbase, base, lane);
    } else {
      if (full) apply_general<V, MAT, true>(a, pbase, lane);
      else apply_general<V, MAT, false>(a, pbase, lane);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// push_scatter: LDS-binned aggregation + device atomics for records [break*TILE, n)
// ------------------------------------------------------------------------------------------------

constexpr u64 kEmpty = ~0ull;

// force_all: every record (unaligned caller pointers, no push_check ran); otherwise the records
// from the first non-increasing tile push_check found (none when the push was increasing).
template <typename V, bool MAT>
// force_all: 0 the records from push_check's break; 1 every record; 2 every record of a whole-push
// scatter, which also writes the hint words as push_apply would for a push that broke in its first tile
__global__ __launch_bounds__(kTPB) void push_scatter_kernel(PushArgs<V> a, int force_all) {
  i64 r0 = 0;
  if (force_all == 2 && blockIdx.x == 0 && threadIdx.x == 0 && a.hint) {
    __hip_atomic_store(a.hint, (u64)a.n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(a.hint + 3, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (!force_all) {
    const u32 brk = a.ctl->brk_enc;  // written by push_check; ordered by the kernel boundary
    if (brk == 0u) return;
    r0 = (i64)(a.ntiles - brk) * kTile;
  }
  if (r0 >= a.n) return;
  const i64 rem = a.n - r0;
  const i64 nchunks = (rem + kScatterChunk - 1) / kScatterChunk;
  if ((i64)blockIdx.x >= nchunks) return;

  typedef typename LdsAcc<V>::T A;
  __shared__ u64 hk[kHashSlots];
  __shared__ A hv[kHashSlots];
  const int tid = threadIdx.x;
  for (int s = tid; s < kHashSlots; s += kTPB) { hk[s] = kEmpty; hv[s] = A(0); }
  __syncthreads();

  for (i64 ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const i64 cbase = r0 + ch * kScatterChunk;
#pragma unroll 2
    for (int q = tid; q < kScatterChunk; q += kTPB) {
      const i64 i = cbase + q;
      if (i >= a.n) break;
      const i64 key = a.keys[i];
      const int32_t col = MAT ? a.cols[i] : 0;
      const V val = a.vals[i];
      i64 addr;
      if (!rec_addr<MAT>(a.part, key, col, addr)) { record_error(a.err, i); continue; }
      const u64 ua = (u64)addr;
      u32 h = (u32)((ua * 0x9E3779B97F4A7C15ull) >> (64 - 12));
      for (;;) {
        const u64 cur = __hip_atomic_load(&hk[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (cur == ua) break;
        if (cur == kEmpty) {
          const u64 prev = atomicCAS(&hk[h], kEmpty, ua);
          if (prev == kEmpty || prev == ua) break;
        }
        h = (h + 1) & (kHashSlots - 1);
      }
      lds_add(&hv[h], (A)val);
    }
    __syncthreads();
    for (int s = tid; s < kHashSlots; s += kTPB) {
      const u64 key = hk[s];
      if (key != kEmpty) {
        gadd(a.data + key, (V)hv[s]);
        hk[s] = kEmpty;
        hv[s] = A(0);
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------
// several range shards in one push (glint_vec_push_dev_shards): the partitions one server hosts, as
// one launch sequence -- a validation pass over the keys, then one scatter that sends each record's
// aggregate to the shard whose range holds its key
// ------------------------------------------------------------------------------------------------
constexpr int kMaxSetShards = 64;
template <typename V>
struct ShardSet {
  int n;
  i64 start[kMaxSetShards];  // ascending, ranges disjoint
  i64 end[kMaxSetShards];
  V* data[kMaxSetShards];
};

// index of the shard whose [start, end) holds key, or -1 (RangePartitioner.partition restated over the
// shards' own ranges: the first start > key, one back)
__device__ __forceinline__ int set_find(const i64* st, const i64* en, int n, i64 key) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (st[mid] <= key) lo = mid + 1;
    else hi = mid;
  }
  return lo > 0 && key < en[lo - 1] ? lo - 1 : -1;
}

// *bad = ~(first record whose key is in no shard), 0 if none (atomicMax of ~index)
template <typename V>
__global__ __launch_bounds__(kTPB) void set_validate_kernel(const i64* __restrict__ keys, i64 n, ShardSet<V> set,
                                                            u64* bad) {
  __shared__ i64 st[kMaxSetShards], en[kMaxSetShards];
  if (threadIdx.x < set.n) {
    st[threadIdx.x] = set.start[threadIdx.x];
    en[threadIdx.x] = set.end[threadIdx.x];
  }
  __syncthreads();
  u64 b = 0;
  if (((uintptr_t)keys & 15) == 0) {  // two keys per 16-B load, four loads in flight per lane
    typedef __attribute__((ext_vector_type(2))) long long KP;
    const i64 np = n >> 1, stride = (i64)gridDim.x * kTPB;
    i64 p = (i64)blockIdx.x * kTPB + threadIdx.x;
    for (; p + 3 * stride < np; p += 4 * stride) {
      KP k[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) k[u] = __builtin_nontemporal_load(reinterpret_cast<const KP*>(keys) + p + u * stride);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const i64 i = 2 * (p + u * stride);
        if (set_find(st, en, set.n, k[u].y) < 0) b = max(b, ~(u64)(i + 1));
        if (set_find(st, en, set.n, k[u].x) < 0) b = max(b, ~(u64)i);
      }
    }
    for (; p < np; p += stride) {
      const KP k = __builtin_nontemporal_load(reinterpret_cast<const KP*>(keys) + p);
      if (set_find(st, en, set.n, k.y) < 0) b = max(b, ~(u64)(2 * p + 1));
      if (set_find(st, en, set.n, k.x) < 0) b = max(b, ~(u64)(2 * p));
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0 && set_find(st, en, set.n, keys[n - 1]) < 0)
      b = max(b, ~(u64)(n - 1));
  } else {
    const i64 stride = (i64)gridDim.x * kTPB;
    for (i64 i = (i64)blockIdx.x * kTPB + threadIdx.x; i < n; i += stride)
      if (set_find(st, en, set.n, keys[i]) < 0) b = max(b, ~(u64)i);
  }
  for (int d = 32; d > 0; d >>= 1) b = max(b, (u64)__shfl_xor((unsigned long long)b, d));
  if ((threadIdx.x & 63) == 0 && b) atomicMax((unsigned long long*)bad, (unsigned long long)b);
}

__global__ void set_gate_kernel(const u64* bad, u64* gate) {
  if (threadIdx.x == 0) *gate = *bad;
}

// push_scatter over the set: the LDS hash aggregates by key, and each aggregate goes to its shard
template <typename V>
__global__ __launch_bounds__(kTPB) void set_scatter_kernel(const i64* __restrict__ keys, const V* __restrict__ vals,
                                                           i64 n, ShardSet<V> set, const u64* bad) {
  if (*bad != 0ull) return;  // a key outside every shard: nothing is applied
  const i64 nchunks = (n + kScatterChunk - 1) / kScatterChunk;
  typedef typename LdsAcc<V>::T A;
  __shared__ u64 hk[kHashSlots];
  __shared__ A hv[kHashSlots];
  __shared__ i64 st[kMaxSetShards], en[kMaxSetShards];
  __shared__ V* dp[kMaxSetShards];
  const int tid = threadIdx.x;
  if (tid < set.n) {
    st[tid] = set.start[tid];
    en[tid] = set.end[tid];
    dp[tid] = set.data[tid];
  }
  for (int q = tid; q < kHashSlots; q += kTPB) { hk[q] = kEmpty; hv[q] = A(0); }
  __syncthreads();
  for (i64 ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const i64 cbase = ch * kScatterChunk;
#pragma unroll 2
    for (int q = tid; q < kScatterChunk; q += kTPB) {
      const i64 i = cbase + q;
      if (i >= n) break;
      const u64 ua = (u64)keys[i];  // in some shard (validated)
      const V val = vals[i];
      u32 h = (u32)((ua * 0x9E3779B97F4A7C15ull) >> (64 - 12));
      for (;;) {
        const u64 cur = __hip_atomic_load(&hk[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (cur == ua) break;
        if (cur == kEmpty) {
          const u64 prev = atomicCAS(&hk[h], kEmpty, ua);
          if (prev == kEmpty || prev == ua) break;
        }
        h = (h + 1) & (kHashSlots - 1);
      }
      lds_add(&hv[h], (A)val);
    }
    __syncthreads();
    for (int q = tid; q < kHashSlots; q += kTPB) {
      const u64 key = hk[q];
      if (key != kEmpty) {
        const int j = set_find(st, en, set.n, (i64)key);
        if (j >= 0) gadd(dp[j] + ((i64)key - st[j]), (V)hv[q]);  // (validated: always found)
        hk[q] = kEmpty;
        hv[q] = A(0);
      }
    }
    __syncthreads();
  }
}

// A gated push (glint_vec_push_dev_gated): its LaunchCtl learns, on the device, whether the gate word
// is set; push_check and push_apply then do nothing, and the tail is empty (brk_enc stays 0).
__global__ void push_gate_kernel(const u64* gate, LaunchCtl* ctl) {
  if (threadIdx.x == 0) ctl->cancel = *gate != 0ull ? 1u : 0u;
}

// A validating gated push (GLINT_PUSH_VALIDATE): push_check has checked every record; its verdict goes
// to the caller's gate word, and a rejected batch is cancelled (no head: push_apply sees cancel; no
// tail: the break is cleared) before anything is applied.
__global__ void push_validate_gate_kernel(LaunchCtl* ctl, u64* gate) {
  if (threadIdx.x == 0) {
    const u64 b = ctl->bad;
    *gate = b;
    if (b != 0ull) {
      ctl->cancel = 1u;
      ctl->brk_enc = 0u;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// pulls
// ------------------------------------------------------------------------------------------------
// PartialVector.get (PartialVector.scala:51-60): out[i] = data(globalToLocal(keys(i)))
// PAIRS: records [2 * p_begin, min(n, 2 * p_end)) (a large pull runs one launch per window), one pair
// per lane per iteration at 4 blocks per CU. (2 or 4 pairs per lane per iteration -- every key load,
// then every gather, then every store -- and 1 / 2 / 8 blocks per CU all measured slower:
// profiles/r06/ab_pull_unroll.txt.)
constexpr int kPullBlocksPerCu = 4;
template <typename V>
__device__ __forceinline__ typename Vec2<V>::T pull_pair(const K2& k, const V* data, const PartDesc& part, ErrState* err,
                                                         i64 r) {
  typedef typename Vec2<V>::T V2;
  i64 l0, l1;
  const bool o0 = rec_addr<false>(part, k.x, 0, l0);
  const bool o1 = rec_addr<false>(part, k.y, 0, l1);
  if (o0 && o1 && l1 == l0 + 1 && (l0 & 1) == 0)  // adjacent pair: a streamed (dense) pull -- non-temporal
    return __builtin_nontemporal_load(reinterpret_cast<const V2*>(data + l0));
  if (!o0) record_error(err, r);
  if (!o1) record_error(err, r + 1);
  return as2<V>(o0 ? data[l0] : V(0), o1 ? data[l1] : V(0));
}
// the gather of record pairs [p_begin, p_end), grid-stride over the first `blocks` blocks
template <typename V>
__device__ __forceinline__ void pull_pairs(const i64* keys, i64 n, const V* data, const PartDesc& part, V* out,
                                           ErrState* err, i64 p_begin, i64 p_end, i64 blocks) {
  typedef typename Vec2<V>::T V2;
  const i64 stride = blocks * kTPB;
  for (i64 p = p_begin + (i64)blockIdx.x * kTPB + threadIdx.x; p < p_end; p += stride) {
    const i64 r = 2 * p;
    if (r + 1 < n) {
      const K2 k = __builtin_nontemporal_load(reinterpret_cast<const K2*>(keys) + p);
      __builtin_nontemporal_store(pull_pair<V>(k, data, part, err, r), reinterpret_cast<V2*>(out + r));
    } else {
      i64 l0;
      const bool o0 = rec_addr<false>(part, keys[r], 0, l0);
      if (!o0) record_error(err, r);
      out[r] = o0 ? data[l0] : V(0);
    }
  }
}

template <typename V, bool PAIRS>
__global__ __launch_bounds__(kTPB) void vec_pull_kernel(const i64* keys, i64 n, const V* data, PartDesc part,
                                                        V* out, ErrState* err, MsgSig sig, i64 p_begin, i64 p_end) {
  const i64 stride = (i64)gridDim.x * kTPB;
  if (PAIRS) {
    pull_pairs<V>(keys, n, data, part, out, err, p_begin, p_end, gridDim.x);
  } else {
    for (i64 i = (i64)blockIdx.x * kTPB + threadIdx.x; i < n; i += stride) {
      i64 l;
      const bool o = rec_addr<false>(part, keys[i], 0, l);
      if (!o) record_error(err, i);
      out[i] = o ? data[l] : V(0);
    }
  }
  msg_signal(sig, err);
}

// A ring pull (one signalling workgroup, <= kRingPullMax records, keys read from the mapped slot
// over PCIe): 1024 threads, up to four records each (record j * 1024 + thread: every load
// instruction of a wave reads 64 consecutive keys), every key load issued before any gather and every
// gather before any store -- one PCIe round trip and one HBM round trip. The grid-stride kernels
// above ran 8 dependent iterations per thread at 256 threads (their stores may alias the keys, so the
// next iteration's loads could not move above them). Batches of 16 384 records (16 per thread,
// GLINT_RING_PULL_PER=16) were measured and not kept: the actor-model cfg4a pulls ran 695-759 M
// records/s against 800-879 with 4 096 (profiles/r04/ab_ring_pull_per.txt): fewer launches, but one
// workgroup reading 128 KB of keys over PCIe per launch, and the GPU waits for 16 messages.
// With a destination table (a coalesced batch whose callers answer from glint_host_alloc buffers),
// each record's answer goes to its own message's destination: the table (<= kPullDirectMax entries,
// read over PCIe beside the keys) is staged in LDS and a record finds its message by binary search.
constexpr int kRingPullTPB = 1024;
#ifndef GLINT_RING_PULL_PER
#define GLINT_RING_PULL_PER 4  // (a build-time experiment knob: records per thread of a ring pull)
#endif
constexpr int kRingPullPer = GLINT_RING_PULL_PER;
constexpr i64 kRingPullMax = (i64)kRingPullTPB * kRingPullPer;
template <typename V, bool MAT>
__global__ __launch_bounds__(kRingPullTPB) void ring_pull_kernel(const i64* __restrict__ keys,
                                                                const int32_t* __restrict__ cols, i64 n,
                                                                const V* __restrict__ data, PartDesc part,
                                                                V* __restrict__ out, ErrState* err, MsgSig sig,
                                                                const PullDst* __restrict__ tab, int nm) {
  __shared__ u32 s_off[kPullDirectMax + 1];
  __shared__ V* s_dst[kPullDirectMax];
  // records per thread actually present (launch-uniform bound: no loads past the batch)
  const int per = (int)min<i64>(kRingPullPer, (n + kRingPullTPB - 1) / kRingPullTPB);
  i64 k[kRingPullPer];
  int32_t c[kRingPullPer];
#pragma unroll
  for (int j = 0; j < kRingPullPer; ++j) {  // clamped, branch-free: all loads in flight together
    if (j < per) {
      const i64 r0 = (i64)j * kRingPullTPB + threadIdx.x;
      const i64 r = r0 < n ? r0 : n - 1;
      k[j] = keys[r];
      c[j] = MAT ? cols[r] : 0;
    }
  }
  if (tab) {  // launch-uniform
    for (int i = threadIdx.x; i < nm; i += kRingPullTPB) {
      s_off[i] = tab[i].off;
      s_dst[i] = reinterpret_cast<V*>(tab[i].dst);
    }
    if (threadIdx.x == 0) s_off[nm] = (u32)n;
  }
  V v[kRingPullPer];
#pragma unroll
  for (int j = 0; j < kRingPullPer; ++j) {
    if (j < per) {
      const i64 r = (i64)j * kRingPullTPB + threadIdx.x;
      i64 l;
      const bool ok = rec_addr<MAT>(part, k[j], c[j], l);
      v[j] = ok ? data[l] : V(0);
      if (!ok && r < n) record_error(err, r);
    }
  }
  if (tab) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kRingPullPer; ++j) {
      const i64 r = (i64)j * kRingPullTPB + threadIdx.x;
      if (j >= per || r >= n) continue;
      int lo = 0, hi = nm - 1;  // the last message starting at or before r
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((i64)s_off[mid] <= r) lo = mid;
        else hi = mid - 1;
      }
      s_dst[lo][r - (i64)s_off[lo]] = v[j];
    }
  } else {
#pragma unroll
    for (int j = 0; j < kRingPullPer; ++j) {
      const i64 r = (i64)j * kRingPullTPB + threadIdx.x;
      if (j < per && r < n) out[r] = v[j];
    }
  }
  msg_signal(sig, err);
}

// PartialMatrix.get (PartialMatrix.scala:55-65)
template <typename V>
__global__ __launch_bounds__(kTPB) void mat_pull_kernel(const i64* rows, const int32_t* cols, i64 n, const V* data,
                                                        PartDesc part, V* out, ErrState* err, MsgSig sig) {
  for (i64 i = (i64)blockIdx.x * kTPB + threadIdx.x; i < n; i += (i64)gridDim.x * kTPB) {
    i64 ad;
    const bool o = rec_addr<true>(part, rows[i], cols[i], ad);
    if (!o) record_error(err, i);
    out[i] = o ? data[ad] : V(0);
  }
  msg_signal(sig, err);
}

// PartialMatrix.getRows (PartialMatrix.scala:37-46) + the row flattening of ResponseSerializer
// (ResponseSerializer.scala:52-61): one wave per requested row, 16 B per lane when rows allow.
template <typename V, bool VEC16>
__global__ __launch_bounds__(kTPB) void mat_pull_rows_kernel(const i64* rows, i64 n, const V* data, PartDesc part,
                                                             V* out, ErrState* err, MsgSig sig) {
  const int lane = threadIdx.x & 63;
  const i64 w0 = (i64)blockIdx.x * (kTPB / 64) + (threadIdx.x >> 6);
  const i64 nw = (i64)gridDim.x * (kTPB / 64);
  const i64 cols = part.cols;
  for (i64 i = w0; i < n; i += nw) {
    const int32_t l = g2l(part, rows[i]);
    const bool ok = l >= 0 && l < part.size;
    if (!ok && lane == 0) record_error(err, i);
    if (VEC16) {
      typedef __attribute__((ext_vector_type(4))) unsigned int U4;
      const i64 chunks = cols * (i64)sizeof(V) / 16;
      const U4* src = reinterpret_cast<const U4*>(data + (ok ? (i64)l : 0) * part.pitch);
      U4* dst = reinterpret_cast<U4*>(out + i * cols);
#pragma unroll 4
      for (i64 c = lane; c < chunks; c += 64) dst[c] = ok ? src[c] : U4{0, 0, 0, 0};
    } else {
      const V* src = data + (ok ? (i64)l : 0) * part.pitch;
      V* dst = out + i * cols;
      for (i64 c = lane; c < cols; c += 64) dst[c] = ok ? src[c] : V(0);
    }
  }
  msg_signal(sig, err);
}

}  // namespace glint

// ================================================================================================
// host side
// ================================================================================================
using namespace glint;

#include "glint_host.h"

namespace {

// ---- push -------------------------------------------------------------------------------------
// blocks per CU in the affine sweep (1 measured best on MI355X)
constexpr int kSweepBlocksPerCu = 1;

// The apply of a large push runs as one launch per window of 2^26 records. A grid-stride sweep over a
// whole 2^30-record push lets its blocks drift apart across gigabytes, and the 2-read + 1-write stream
// then runs 6-11 % slower than the same bytes swept window by window (tools/microbench_stream.hip mode
// 6: 2^30 records whole 5.90 TB/s, in 2^26-record launches 6.56 TB/s; 2^28 whole 6.21 TB/s;
// profiles/r03/micro_stream_2p30.txt).
constexpr u32 kSweepWindowTiles = ((u32)1 << 26) / kTile;

// GLINT_BINNED: 0 = never bin, 1 = bin every large push, unset = bin when the previous push on the
// shard left a large unordered tail (read from the host-mapped word push_apply writes)
int binned_mode() {
  static EnvKnob k("GLINT_BINNED");
  return (int)k.get([](const char* e) -> long long {
    if (!e || !*e) return -1;
    return atoi(e) != 0 ? 1 : 0;
  });
}
constexpr i64 kBinMin = (i64)1 << 20;  // records: below this the LDS-hash scatter wins
// ... and below this many records per 4096-element slab of the shard (GLINT_BIN_DENSITY): the binned
// pipeline's passes cost about the same whatever the density, the atomic scatter's time grows with
// the records. Measured crossover (tools/tail_ab.py, profiles/r05/tail_ab.jsonl, uniform keys into a
// 2^28-element shard): scatter 0.55 / 1.02 / 1.98 / 3.83 ms against binned 0.88 / 1.27 / 1.99 / 2.24 ms
// at 128 / 256 / 512 / 1024 records per slab; 8 shards pushed on 8 concurrent streams at 128 per slab
// (the cfg4 key space's local pushes) 3.70 against 4.69 ms
i64 bin_density() {
  static EnvKnob k("GLINT_BIN_DENSITY");
  return k.get([](const char* e) -> long long { return e ? std::max(0ll, atoll(e)) : 512ll; });
}
// records: up to this many, a (non-deterministic) push is the single scatter launch
constexpr i64 kSmallPushMax = 4096;

template <typename V, bool MAT>
int launch_push(glint_shard* s, const i64* keys, const int32_t* cols, const void* vals, i64 n, int flags,
                hipStream_t st) {
  if (n <= 0) return GLINT_OK;
  if (!keys || !vals || (MAT && !cols)) return GLINT_EINVAL;
  PushArgs<V> a;
  a.keys = keys;
  a.cols = cols;
  a.vals = (const V*)vals;
  a.n = n;
  a.data = (V*)s->data;
  a.part = s->part;
  a.err = err_of(s);
  a.elems = s->elems;
  a.hint = s->d_hint;
  a.sig = s->sig;
  a.sweep_blocks = 0;
  const i64 ntiles = (n + kTile - 1) / kTile;
  if (ntiles >= (i64)0xFFFFFFF0ll) return GLINT_EINVAL;
  a.ntiles = (u32)ntiles;
  const bool vec_ok = aligned(keys, 16) && aligned(vals, 2 * sizeof(V)) && (!MAT || aligned(cols, 8));
  const bool fp = s->dtype == GLINT_F32 || s->dtype == GLINT_F64;
  const bool det = (flags & GLINT_PUSH_DETERMINISTIC) && fp;
  const bool unordered = (flags & GLINT_PUSH_UNORDERED) != 0;
  // Message-sized Float/Double pushes that must keep the reference's summation order -- every
  // deterministic one, and host-pointer / wire pushes unless the caller said UNORDERED -- are one
  // launch of the order-preserving fold (glint_ordered.hip). Int/Long sums are exact in any order.
  const bool seq = det || (fp && (flags & kPushHostSequential) && !unordered);
  // a gated push takes check + apply (+ its tail from the break): those kernels read the gate's
  // verdict from the LaunchCtl (the ordered fold, the unordered hint and the one-launch small push
  // have no such step)
  const bool gated = s->gate != nullptr;
  if (gated && (det || !vec_ok)) return GLINT_EINVAL;
  // a ring launch (one workgroup that signals its own completion) is always the ordered fold: for
  // Int/Long it is one more exact summation order
  if (a.sig.done || (seq && n <= kOrderedMax && s->elems < ((i64)1 << 32))) return push_ordered<V, MAT>(s, a, st);
  // control region: [LaunchCtl slot 0 | slot 1 | pad to 256][tile descriptors i64 x ntiles]. An
  // ordered push uses one slot while its push_check zeroes the other for the next push, so no
  // memset runs per push (pushes on one shard are stream-ordered, as the actor's messages are).
  const size_t ctl_need = 256 + (size_t)ntiles * sizeof(i64);
  const void* ctl_old = s->d_ctl;
  int rc = grow(&s->d_ctl, &s->ctl_bytes, ctl_need);
  if (rc) return rc;
  if (s->d_ctl != ctl_old) {  // fresh region: both slots zero
    HIPCHK(hipMemsetAsync(s->d_ctl, 0, 2 * sizeof(LaunchCtl), st));
    s->ctl_par = 0;
  }
  LaunchCtl* const slots = (LaunchCtl*)s->d_ctl;
  a.ctl = slots + s->ctl_par;
  i64* desc = (i64*)((char*)s->d_ctl + 256);

  const int bmode = binned_mode();
  const i64 last_tail = (i64)s->hint_tail;  // the previous push's unordered tail, as of the last sync point
  const i64 slabs = (s->elems + 4095) / 4096;
  const bool binned = !det && vec_ok && push_binnable(s, n) && bmode != 0 &&
                      (unordered || (n >= kBinMin && (bmode == 1 || (last_tail >= kBinMin &&
                                                                     last_tail >= bin_density() * slabs))));
  if (binned && unordered && !gated) return push_binned<V, MAT>(s, a, false, st);
  const bool validate = gated && (flags & GLINT_PUSH_VALIDATE) != 0;
  // Whole-push bin: when the last push (as of the last sync point) broke order in its first tile, the
  // binned pipeline takes this one from record 0 with no push_check (the unordered push's check found
  // only that, at one contended atomic per wave tile) and no head. Sums are the same in any order (this
  // is not a deterministic push); bin_count validates every record of a validating push, zeroes the
  // next push's LaunchCtl slot as push_check does, and notes whether two adjacent records were ever out
  // of order, so an ordered push is followed by the checked path again. GLINT_BIN_WHOLE=0: always check.
  static EnvKnob whole_knob("GLINT_BIN_WHOLE");
  const bool whole = binned && (!gated || validate) && s->hint_tail > 0 && s->hint_head == 0 &&
                     whole_knob.get([](const char* e) -> long long { return e ? atoi(e) != 0 : 1; }) != 0;
  if (whole) {
    LaunchCtl* const next = slots + (s->ctl_par ^ 1);
    const BinHook hook = [&](void* bc, u32* T, u32 nb) -> int {
      return launch_validate_gate_binned(a.ctl, s->gate, bc, T, nb, st);
    };
    rc = push_binned<V, MAT>(s, a, false, st, validate ? &hook : nullptr, next);
    if (rc == GLINT_OK) s->ctl_par ^= 1;  // bin_count zeroed the other slot
    return rc;
  }
  // Small pushes (an Akka message is ~1000 records, GranularBigVectorSpec.scala:21) are one launch:
  // the scatter handles every record, instead of check + apply + scatter. Launch latency is the
  // whole cost at this size, so two fewer launches is the win; results are those of the scatter
  // path (bit-exact for unique keys and for Int/Long, unordered sums otherwise).
  const bool small = !det && !gated && n <= kSmallPushMax;
  // Whole-push scatter: the sparse counterpart of the whole-push bin. When the last checked push broke
  // order in its first tile and this one stays below the binned density, the scatter takes every record
  // from 0 with no push_check / push_apply in front (they found only that). Its hint words say so (the
  // push's size, a tail from record 0) without looking, so every 8th such push is checked again (its
  // push_apply writes the measured words: an ordered push returns the shard to the checked path).
  const bool whole_scatter = !binned && !det && !gated && vec_ok && !small && s->hint_tail > 0 &&
                             s->hint_head == 0 && (s->whole_probe++ & 7u) != 7u &&
                             whole_knob.get([](const char* e) -> long long { return e ? atoi(e) != 0 : 1; }) != 0;
  if (!vec_ok || small || whole_scatter) {  // unaligned caller pointers or a small push: the scatter for everything
    if (det) return push_det_tail<V, MAT>(s, a, false, st);
    const unsigned g2 = grid_for(n, kScatterChunk, (i64)s->cus * 2);
    HIPCHK(launch_k(s, GLINT_K_PUSH_SCATTER, push_scatter_kernel<V, MAT>, g2, kTPB, st, a, whole_scatter ? 2 : 1));
    return GLINT_OK;
  }
  const u64 win = std::min<u64>(kSweepWindowTiles, a.ntiles);
  // a validating push whose tail is binned reads its keys once: push_check validates the records up to
  // the break, the tail's count pass the rest, and the verdict comes after that count (BinHook)
  const bool fuse = validate && binned && !det;
  {
    LaunchCtl* const next = slots + (s->ctl_par ^ 1);
    if (gated && !validate) {
      push_gate_kernel<<<1, 64, 0, st>>>(s->gate, a.ctl);
      HIPCHK(hipGetLastError());
    }
    // one launch: the key stream alone lost 3-6 % when windowed (each short launch ramps up and drains)
    const unsigned gc =
        grid_for(a.ntiles, kTPB / 64, (i64)s->cus * blocks_per_cu<push_check_kernel<MAT, 0>>(2));
    HIPCHK(a.part.kind == 0 ? launch_k(s, GLINT_K_PUSH_CHECK, push_check_kernel<MAT, 0>, gc, kTPB, st, keys, cols, n,
                                       a.part, a.ctl, next, desc, a.ntiles, 0u, a.ntiles, validate ? (fuse ? 2 : 1) : 0)
                            : launch_k(s, GLINT_K_PUSH_CHECK, push_check_kernel<MAT, 1>, gc, kTPB, st, keys, cols, n,
                                       a.part, a.ctl, next, desc, a.ntiles, 0u, a.ntiles, validate ? (fuse ? 2 : 1) : 0));
    if (validate && !fuse) {
      push_validate_gate_kernel<<<1, 64, 0, st>>>(a.ctl, s->gate);
      HIPCHK(hipGetLastError());
    }
    s->ctl_par ^= 1;  // only once the check that zeroes the other slot is on the stream
  }
  auto apply_head = [&]() -> int {  // the records before the break (every record of an ordered push)
    const i64 bpc = blocks_per_cu<push_apply_kernel<V, MAT>>(2);
    for (u64 t0 = 0; t0 < a.ntiles; t0 += win) {
      const u32 t1 = (u32)std::min<u64>(a.ntiles, t0 + win);
      const unsigned ga = grid_for(t1 - t0, kTPB / 64, (i64)s->cus * bpc);
      a.sweep_blocks = std::min<u32>(ga, (u32)((i64)s->cus * kSweepBlocksPerCu));
      HIPCHK(launch_k(s, GLINT_K_PUSH_APPLY, push_apply_kernel<V, MAT>, ga, kTPB, st, a, (const i64*)desc, (u32)t0, t1));
    }
    return GLINT_OK;
  };
  if (fuse) {  // verdict, cancel and the head, behind the tail's validating count
    const BinHook hook = [&](void* bc, u32* T, u32 nb) -> int {
      const int rc2 = launch_validate_gate_binned(a.ctl, s->gate, bc, T, nb, st);
      return rc2 ? rc2 : apply_head();
    };
    return push_binned<V, MAT>(s, a, true, st, &hook);
  }
  rc = apply_head();
  if (rc) return rc;
  if (det) return push_det_tail<V, MAT>(s, a, true, st);
  if (binned) return push_binned<V, MAT>(s, a, true, st);
  const unsigned g2 = grid_for(n, kScatterChunk, (i64)s->cus * 2);
  HIPCHK(launch_k(s, GLINT_K_PUSH_SCATTER, push_scatter_kernel<V, MAT>, g2, kTPB, st, a, 0));
  return GLINT_OK;
}

// ---- pulls ------------------------------------------------------------------------------------
// A ring launch (s->sig.done set) is one workgroup that signals its own completion. (A dense pull
// checked first -- a key pass flagging any record off one run, then a 16-B streaming copy of the run --
// measured no faster than the gather, which is itself a dense stream for such keys: 1.006-1.054 against
// 0.992-1.044 ms kernel time at 2^28, profiles/r06/ab_pull_checked.txt.)
template <typename V>
int launch_vec_pull(glint_shard* s, const i64* keys, void* out, i64 n, hipStream_t st) {
  if (n <= 0) return GLINT_OK;
  if (!keys || !out) return GLINT_EINVAL;
  const MsgSig sig = s->sig;
  if (sig.done && n <= kRingPullMax) {
    HIPCHK(launch_k(s, GLINT_K_VEC_PULL, ring_pull_kernel<V, false>, 1u, kRingPullTPB, st, keys, (const int32_t*)nullptr,
                    n, (const V*)s->data, s->part, (V*)out, err_of(s), sig, s->pull_tab, s->pull_nm));
    return GLINT_OK;
  }
  const bool pairs = aligned(keys, 16) && aligned(out, 2 * sizeof(V));
  if (pairs) {
    // 4 blocks per CU: the dense gather's best (tools/microbench_stream.hip mode 5); one launch per
    // window of records, as the push's apply sweep (kSweepWindowTiles)
    const i64 npairs = (n + 1) / 2;
    const i64 win = sig.done ? npairs : std::min<i64>(npairs, (i64)kSweepWindowTiles * (kTile / 2));
    for (i64 p0 = 0; p0 < npairs; p0 += win) {
      const i64 p1 = std::min<i64>(npairs, p0 + win);
      const unsigned g = sig.done ? 1u : grid_for(p1 - p0, kTPB, (i64)s->cus * kPullBlocksPerCu);
      HIPCHK(launch_k(s, GLINT_K_VEC_PULL, vec_pull_kernel<V, true>, g, kTPB, st, keys, n, (const V*)s->data, s->part,
                      (V*)out, err_of(s), sig, p0, p1));
    }
  } else {
    const unsigned g = sig.done ? 1u : grid_for(n, kTPB, (i64)s->cus * 8);
    HIPCHK(launch_k(s, GLINT_K_VEC_PULL, vec_pull_kernel<V, false>, g, kTPB, st, keys, n, (const V*)s->data, s->part,
                    (V*)out, err_of(s), sig, (i64)0, (i64)0));
  }
  return GLINT_OK;
}

template <typename V>
int launch_mat_pull(glint_shard* s, const i64* rows, const int32_t* cols, void* out, i64 n, hipStream_t st) {
  if (n <= 0) return GLINT_OK;
  if (!rows || !cols || !out) return GLINT_EINVAL;
  const MsgSig sig = s->sig;
  if (sig.done && n <= kRingPullMax) {
    HIPCHK(launch_k(s, GLINT_K_MAT_PULL, ring_pull_kernel<V, true>, 1u, kRingPullTPB, st, rows, cols, n,
                    (const V*)s->data, s->part, (V*)out, err_of(s), sig, s->pull_tab, s->pull_nm));
    return GLINT_OK;
  }
  const unsigned g = sig.done ? 1u : grid_for(n, kTPB, (i64)s->cus * 8);
  HIPCHK(launch_k(s, GLINT_K_MAT_PULL, mat_pull_kernel<V>, g, kTPB, st, rows, cols, n, (const V*)s->data, s->part,
                  (V*)out, err_of(s), sig));
  return GLINT_OK;
}

template <typename V>
int launch_mat_pull_rows(glint_shard* s, const i64* rows, void* out, i64 n, hipStream_t st) {
  if (n <= 0) return GLINT_OK;
  if (!rows || !out) return GLINT_EINVAL;
  const MsgSig sig = s->sig;
  const bool v16 = ((i64)s->part.cols * (i64)sizeof(V)) % 16 == 0 && aligned(out, 16);
  const unsigned g = sig.done ? 1u : grid_for(n, kTPB / 64, (i64)s->cus * 8);
  HIPCHK(launch_k(s, GLINT_K_MAT_PULL_ROWS, v16 ? mat_pull_rows_kernel<V, true> : mat_pull_rows_kernel<V, false>, g,
                  kTPB, st, rows, n, (const V*)s->data, s->part, (V*)out, err_of(s), sig));
  return GLINT_OK;
}

// dtype dispatch
#define GLINT_DISPATCH(dt, FN, ...)                            \
  switch (dt) {                                                \
    case GLINT_F64: return FN<double>(__VA_ARGS__);            \
    case GLINT_F32: return FN<float>(__VA_ARGS__);             \
    case GLINT_I64: return FN<long long>(__VA_ARGS__);         \
    case GLINT_I32: return FN<int>(__VA_ARGS__);               \
    default: return GLINT_EINVAL;                              \
  }

template <typename V>
int push_vec_t(glint_shard* s, const i64* k, const int32_t*, const void* v, i64 n, int f, hipStream_t st) {
  return launch_push<V, false>(s, k, nullptr, v, n, f, st);
}
template <typename V>
int push_mat_t(glint_shard* s, const i64* k, const int32_t* c, const void* v, i64 n, int f, hipStream_t st) {
  return launch_push<V, true>(s, k, c, v, n, f, st);
}

// glint_vec_push_dev_shards' launches: the set's ranges and data pointers by value, its verdict in the
// first shard's scratch word for this stream (under the locks of every member)
template <typename V>
int launch_set_push(glint_shard* const* sh, int m, const i64* keys, const void* vals, i64 n, u64* gate,
                    hipStream_t st) {
  glint_shard* s0 = sh[0];
  ShardSet<V> set{};
  set.n = m;
  for (int j = 0; j < m; ++j) {
    set.start[j] = sh[j]->part.start;
    set.end[j] = sh[j]->part.start + sh[j]->part.size;
    set.data[j] = (V*)sh[j]->data;
  }
  u64* word = nullptr;
  for (auto& sw : s0->set_words)
    if (sw.first == st) word = sw.second;
  if (!word) {
    if (hipMalloc((void**)&word, sizeof(u64)) != hipSuccess) {
      (void)hipGetLastError();
      return GLINT_ENOMEM;
    }
    s0->set_words.emplace_back(st, word);
  }
  HIPCHK(hipMemsetAsync(word, 0, sizeof(u64), st));
  const unsigned gv = grid_for(n, (i64)kTPB * 16, (i64)s0->cus * 4);
  HIPCHK(launch_k(s0, GLINT_K_PUSH_CHECK, set_validate_kernel<V>, gv, kTPB, st, keys, n, set, word));
  set_gate_kernel<<<1, 64, 0, st>>>(word, gate);
  HIPCHK(hipGetLastError());
  const unsigned g2 = grid_for(n, kScatterChunk, (i64)s0->cus * 2);
  HIPCHK(launch_k(s0, GLINT_K_PUSH_SCATTER, set_scatter_kernel<V>, g2, kTPB, st, keys, (const V*)vals, n, set,
                  (const u64*)word));
  return GLINT_OK;
}

int create_common(glint_shard* s, int device, int dtype, int32_t cols, void* view_data = nullptr) {
  if (dtype < GLINT_I32 || dtype > GLINT_F64 || cols < 0) return GLINT_EINVAL;
  static EnvKnob hprof_knob("GLINT_HOST_PROF");
  s->hprof = hprof_knob.pos_or(0) != 0;
  if (s->part.size < 0) return GLINT_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
    (void)hipGetLastError();
    return GLINT_EDEVICE;
  }
  DeviceGuard g(device);
  if (!g.ok) return GLINT_EDEVICE;
  s->device = device;
  s->dtype = dtype;
  s->vsize = dtype_size(dtype);
  s->part.cols = cols;
  const i64 per16 = 16 / (i64)s->vsize;
  s->part.pitch = cols > 0 ? ((i64)cols + per16 - 1) / per16 * per16 : 1;
  s->elems = cols > 0 ? (i64)s->part.size * s->part.pitch : (i64)s->part.size;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    s->cus = prop.multiProcessorCount;
  HIPCHK(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
  // +16 B: a slab-wide pair load may touch one element past an odd-sized shard's end
  const size_t bytes = (size_t)s->elems * s->vsize + 16;
  if (view_data) {
    s->data = view_data;  // a slab's elements, as they are (glint_shard_create_in)
  } else if (hipMalloc(&s->data, bytes) != hipSuccess) {
    (void)hipGetLastError();
    return GLINT_ENOMEM;
  }
  if (hipMalloc((void**)&s->d_err, sizeof(ErrState)) != hipSuccess ||
      hipMalloc((void**)&s->d_err_host, sizeof(ErrState)) != hipSuccess) {
    (void)hipGetLastError();
    return GLINT_ENOMEM;
  }
  if (hipHostMalloc((void**)&s->h_hint, 64, hipHostMallocMapped) == hipSuccess) {
    s->h_hint[0] = 0;  // unordered-tail size of the last push (push_apply)
    s->h_hint[1] = 0;  // (m << 32 | tail) of the last binned push (bin_fpart)
    s->h_hint[2] = 0;  // cold records of the last binned push (bin_fpart)
    s->h_hint[3] = 0;  // where the last push's unordered tail started (push_apply; bin_fsort for a whole-push bin)
    if (hipHostGetDevicePointer((void**)&s->d_hint, s->h_hint, 0) != hipSuccess) s->d_hint = nullptr;
  } else {
    s->h_hint = nullptr;
  }
  (void)hipGetLastError();
  if (!s->d_hint && s->h_hint) { (void)hipHostFree(s->h_hint); s->h_hint = nullptr; }
  if (hipHostMalloc((void**)&s->h_err, sizeof(ErrState), hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    s->h_err = nullptr;  // host calls then read the error state with a pageable copy
  }
  if (!view_data) HIPCHK(hipMemsetAsync(s->data, 0, bytes, s->stream));  // new Array[V](size) is zeroed
  HIPCHK(hipMemsetAsync(s->d_err, 0, sizeof(ErrState), s->stream));
  HIPCHK(hipMemsetAsync(s->d_err_host, 0, sizeof(ErrState), s->stream));
  HIPCHK(hipStreamSynchronize(s->stream));
  return GLINT_OK;
}

void free_shard(glint_shard* s) {
  if (!s) return;
  if (s->hprof) {
    const auto& p = s->hp;
    fprintf(stderr,
            "glint_host_prof {\"device\": %d, \"locks\": %llu, \"lock_wait_s\": %.6f, \"lock_hold_s\": %.6f, "
            "\"launches\": %llu, \"launch_s\": %.6f, \"retire_waits\": %llu, \"retire_wait_s\": %.6f, "
            "\"copy_s\": %.6f, \"tickets\": %llu}\n",
            s->device, (unsigned long long)p.nlock.load(), 1e-9 * (double)p.lock_wait.load(),
            1e-9 * (double)p.lock_hold.load(), (unsigned long long)p.nlaunch.load(), 1e-9 * (double)p.launch.load(),
            (unsigned long long)p.nretire_wait.load(), 1e-9 * (double)p.retire_wait.load(),
            1e-9 * (double)p.copy.load(), (unsigned long long)s->ticket_next);
  }
  {
    DeviceGuard g(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    prof_drain(s);
    if (s->data && !s->slab) (void)hipFree(s->data);
    if (s->d_err) (void)hipFree(s->d_err);
    if (s->d_err_host) (void)hipFree(s->d_err_host);
    if (s->d_ctl) (void)hipFree(s->d_ctl);
    if (s->d_scratch) (void)hipFree(s->d_scratch);
    if (s->d_det) (void)hipFree(s->d_det);
    if (s->det_stream) {
      (void)hipStreamSynchronize(s->det_stream);
      (void)hipStreamDestroy(s->det_stream);
    }
    for (auto& e : s->det_ev)
      if (e) (void)hipEventDestroy(e);
    if (s->d_bin) (void)hipFree(s->d_bin);
    for (auto& sw : s->set_words) (void)hipFree(sw.second);
    if (s->d_binctl) (void)hipFree(s->d_binctl);
    if (s->d_hot) (void)hipFree(s->d_hot);
    if (s->h_hint) (void)hipHostFree(s->h_hint);
    if (s->h_stage) (void)hipHostFree(s->h_stage);
    if (s->h_err) (void)hipHostFree(s->h_err);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    if (s->order_ev) (void)hipEventDestroy(s->order_ev);
    for (auto& r : s->ring) {
      if (r.h) (void)hipHostFree(r.h);
      if (r.d) (void)hipFree(r.d);
      if (r.herr) (void)hipHostFree(r.herr);
      if (r.done) (void)hipEventDestroy(r.done);
    }
    if (s->h_done) (void)hipHostFree(s->h_done);
    if (s->host_ev) (void)hipEventDestroy(s->host_ev);
    (void)hipGetLastError();
  }
  delete s;
}

// wire constants (src/main/scala/glint/serialization/SerializationConstants.scala:24-38)
enum : uint8_t {
  W_PULL_MATRIX = 0x00, W_PULL_MATRIX_ROWS = 0x01, W_PULL_VECTOR = 0x02,
  W_PUSH_MAT_D = 0x03, W_PUSH_MAT_F = 0x04, W_PUSH_MAT_I = 0x05, W_PUSH_MAT_L = 0x06,
  W_PUSH_VEC_D = 0x07, W_PUSH_VEC_F = 0x08, W_PUSH_VEC_I = 0x09, W_PUSH_VEC_L = 0x0A,
  W_RESP_D = 0x10, W_RESP_F = 0x11, W_RESP_I = 0x12, W_RESP_L = 0x13
};

int wire_dtype_of_push(uint8_t t, bool* mat) {
  switch (t) {
    case W_PUSH_MAT_D: *mat = true; return GLINT_F64;
    case W_PUSH_MAT_F: *mat = true; return GLINT_F32;
    case W_PUSH_MAT_I: *mat = true; return GLINT_I32;
    case W_PUSH_MAT_L: *mat = true; return GLINT_I64;
    case W_PUSH_VEC_D: *mat = false; return GLINT_F64;
    case W_PUSH_VEC_F: *mat = false; return GLINT_F32;
    case W_PUSH_VEC_I: *mat = false; return GLINT_I32;
    case W_PUSH_VEC_L: *mat = false; return GLINT_I64;
    default: return -1;
  }
}
uint8_t wire_response_type(int dtype) {
  switch (dtype) {
    case GLINT_F64: return W_RESP_D;
    case GLINT_F32: return W_RESP_F;
    case GLINT_I32: return W_RESP_I;
    default: return W_RESP_L;
  }
}

// defined with the ring below: device-resident calls are ordered after the ring's entries
int dev_order_after_host(glint_shard* s, hipStream_t st);
void* host_dev_ptr(const void* p, size_t bytes, size_t align, HostHold* hold = nullptr);  // glint_host_alloc buffers (below)
int ring_flush_locked(glint_shard* s);
int ring_retire_through(glint_shard* s, u64 t);

}  // namespace

// ================================================================================================
// C ABI
// ================================================================================================
std::atomic<unsigned> g_env_gen{1};

extern "C" {

int glint_version(void) { return 100; }

int glint_reload_env(void) {
  g_env_gen.fetch_add(1, std::memory_order_acq_rel);
  return GLINT_OK;
}

int glint_push_flags_supported(void) {
  return GLINT_PUSH_DETERMINISTIC | GLINT_PUSH_UNORDERED | GLINT_PUSH_VALIDATE;
}

int glint_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

const char* glint_strerror(int status) {
  switch (status) {
    case GLINT_OK: return "ok";
    case GLINT_EOUTOFRANGE: return "key outside the shard (ArrayIndexOutOfBoundsException in the reference)";
    case GLINT_EDEVICE: return "HIP device error (or no GPU)";
    case GLINT_EINVAL: return "invalid argument";
    case GLINT_ENOMEM: return "out of memory";
    default: return "unknown status";
  }
}

int glint_shard_create(int device, int dtype, int64_t start, int64_t end, int32_t cols, glint_shard_t* out) {
  if (!out) return GLINT_EINVAL;
  *out = nullptr;
  glint_shard* s = new (std::nothrow) glint_shard();
  if (!s) return GLINT_ENOMEM;
  s->part.kind = 0;
  s->part.start = start;
  s->part.size = (int32_t)(end - start);  // RangePartition.size, RangePartition.scala:24
  int rc = create_common(s, device, dtype, cols);
  if (rc) { free_shard(s); return rc; }
  *out = s;
  return GLINT_OK;
}

int glint_shard_create_cyclic(int device, int dtype, int32_t index, int32_t num_partitions, int64_t num_keys,
                              int32_t cols, glint_shard_t* out) {
  if (!out || num_partitions <= 0 || index < 0 || index >= num_partitions || num_keys <= 0) return GLINT_EINVAL;
  *out = nullptr;
  glint_shard* s = new (std::nothrow) glint_shard();
  if (!s) return GLINT_ENOMEM;
  s->part.kind = 1;
  s->part.cidx = index;
  s->part.cparts = num_partitions;
  // CyclicPartition.size (CyclicPartition.scala:30-36): local index of the last key it owns + 1
  int32_t size = 0;
  for (int64_t i = 1; i <= (int64_t)num_partitions && num_keys - i >= 0; ++i) {
    const int64_t k = num_keys - i;
    if ((int32_t)(k % num_partitions) == index) { size = (int32_t)((k - index) / num_partitions) + 1; break; }
  }
  s->part.size = size;
  int rc = create_common(s, device, dtype, cols);
  if (rc) { free_shard(s); return rc; }
  *out = s;
  return GLINT_OK;
}

int glint_shard_create_in(glint_shard_t slab, int64_t offset, int64_t start, int64_t end, glint_shard_t* out) {
  if (!out) return GLINT_EINVAL;
  *out = nullptr;
  if (!slab || slab->slab || offset < 0 || end < start || end - start > INT32_MAX) return GLINT_EINVAL;
  ShardLock lk(slab);
  if (slab->dying) return GLINT_EINVAL;
  const i64 rows = end - start;
  if (offset + rows > (i64)slab->part.size) return GLINT_EINVAL;
  const i64 first = offset * (slab->part.cols > 0 ? slab->part.pitch : 1);  // the view's first element
  if ((first * (i64)slab->vsize) % 256 != 0) return GLINT_EINVAL;  // kernels take 256 B-aligned shards
  glint_shard* s = new (std::nothrow) glint_shard();
  if (!s) return GLINT_ENOMEM;
  s->part.kind = 0;
  s->part.start = start;
  s->part.size = (int32_t)rows;
  s->slab = slab;  // set first: a failed create does not free the slab's memory
  int rc = create_common(s, slab->device, slab->dtype, slab->part.cols, (char*)slab->data + first * (i64)slab->vsize);
  if (rc == GLINT_OK) {
    try {
      slab->views.push_back(s);
    } catch (...) {
      rc = GLINT_ENOMEM;
    }
  }
  if (rc) { free_shard(s); return rc; }
  *out = s;
  return GLINT_OK;
}

// (destroying a shard while another thread still calls into it is the caller's error, as for any handle;
// a slab marks itself dying under its lock, so a view created after the check is refused)
int glint_shard_destroy(glint_shard_t s) {
  if (!s) return GLINT_EINVAL;
  if (s->slab) {  // a view: off its slab's list first
    ShardLock lk(s->slab);
    auto& v = s->slab->views;
    v.erase(std::remove(v.begin(), v.end(), s), v.end());
  } else {
    ShardLock lk(s);
    if (!s->views.empty()) return GLINT_EINVAL;  // its views read and write its memory: destroy them first
    s->dying = true;
  }
  free_shard(s);
  return GLINT_OK;
}

int glint_shard_zero(glint_shard_t s) {
  if (!s) return GLINT_EINVAL;
  ShardLock lk(s);
  DeviceGuard g(s->device);
  int rc = refuse_slab(s);
  if (rc == GLINT_OK) rc = ring_flush_locked(s);  // the restart comes after every message enqueued before it
  if (rc == GLINT_OK) rc = order_after_dev(s);
  if (rc) return rc;
  HIPCHK(hipMemsetAsync(s->data, 0, (size_t)s->elems * s->vsize, s->stream));
  HIPCHK(hipMemsetAsync(s->d_err, 0, sizeof(ErrState), s->stream));
  HIPCHK(hipMemsetAsync(s->d_err_host, 0, sizeof(ErrState), s->stream));
  HIPCHK(hipStreamSynchronize(s->stream));
  rc = ring_retire_through(s, s->ticket_next);  // all complete: pulls get their answers
  s->failed.clear();  // a fresh shard: nothing before the restart is reported any more
  s->host_pending = false;
  return rc;
}

int glint_shard_info(glint_shard_t s, int32_t* size, int32_t* cols, int* dtype, int* device) {
  if (!s) return GLINT_EINVAL;
  if (size) *size = s->part.size;
  if (cols) *cols = s->part.cols;
  if (dtype) *dtype = s->dtype;
  if (device) *device = s->device;
  return GLINT_OK;
}

int glint_shard_data(glint_shard_t s, void** p) {
  if (!s || !p) return GLINT_EINVAL;
  *p = s->data;
  return GLINT_OK;
}

int glint_shard_pitch(glint_shard_t s, int64_t* e) {
  if (!s || !e) return GLINT_EINVAL;
  *e = s->part.cols > 0 ? s->part.pitch : 1;
  return GLINT_OK;
}

int glint_shard_last_error(glint_shard_t s, int64_t* first_bad) {
  if (!s || !first_bad) return GLINT_EINVAL;
  *first_bad = s->last_bad;
  return GLINT_OK;
}

int glint_prof_enable(glint_shard_t s, int on) {
  if (!s) return GLINT_EINVAL;
  ShardLock lk(s);
  s->prof = on != 0;
  return GLINT_OK;
}

int glint_prof_read(glint_shard_t s, int kernel_id, double* total_ms, int64_t* launches) {
  if (!s || kernel_id < 0 || kernel_id >= GLINT_K_COUNT) return GLINT_EINVAL;
  ShardLock lk(s);
  DeviceGuard g(s->device);
  prof_drain(s);
  if (total_ms) *total_ms = s->prof_ms[kernel_id];
  if (launches) *launches = s->prof_n[kernel_id];
  return GLINT_OK;
}

int glint_prof_reset(glint_shard_t s) {
  if (!s) return GLINT_EINVAL;
  ShardLock lk(s);
  DeviceGuard g(s->device);
  prof_drain(s);
  for (int k = 0; k < GLINT_K_COUNT; ++k) { s->prof_ms[k] = 0; s->prof_n[k] = 0; }
  return GLINT_OK;
}

int glint_shards_sync(glint_shard_t* shards, void** streams, int n, int* rcs, int64_t* first_bad) {
  if (n < 0 || (n > 0 && (!shards || !streams || !rcs))) return GLINT_EINVAL;
  std::vector<glint_shard*> order(shards, shards + n);
  std::sort(order.begin(), order.end());
  if (n > 0 && (!order[0] || std::adjacent_find(order.begin(), order.end()) != order.end())) return GLINT_EINVAL;
  lock_order(order);
  struct Locks {  // every shard's lock, in lock_order, for the whole call
    std::vector<glint_shard*>& v;
    size_t k = 0;
    ~Locks() {
      for (size_t i = 0; i < k; ++i) v[i]->mu.unlock();
    }
  } locks{order};
  for (; locks.k < order.size(); ++locks.k) order[locks.k]->mu.lock();
  std::vector<ErrState> local((size_t)n);
  std::vector<ErrState*> h((size_t)n);
  for (int i = 0; i < n; ++i) {  // the error states ride behind each stream's work
    glint_shard* s = shards[i];
    DeviceGuard g(s->device);
    h[i] = s->h_err ? s->h_err : &local[i];
    rcs[i] = hipMemcpyAsync(h[i], s->d_err, sizeof(ErrState), hipMemcpyDeviceToHost, (hipStream_t)streams[i]) ==
                     hipSuccess ? GLINT_OK : GLINT_EDEVICE;
  }
  {
    // a query submits what the runtime holds back for the stream, so every copy is on its queue
    // before the first wait (without it the copies of streams sharing a hardware queue went out one
    // per wait, ~25 us apart, after the last push)
    for (int i = 0; i < n; ++i) {
      DeviceGuard g(shards[i]->device);
      (void)hipStreamQuery((hipStream_t)streams[i]);
    }
    (void)hipGetLastError();
  }
  int rc = GLINT_OK;
  for (int i = 0; i < n; ++i) {
    glint_shard* s = shards[i];
    DeviceGuard g(s->device);
    hipStream_t st = (hipStream_t)streams[i];
    if (rcs[i] == GLINT_OK && hipStreamSynchronize(st) != hipSuccess) rcs[i] = GLINT_EDEVICE;
    if (rcs[i] == GLINT_OK) {
      if (st == s->last_dev_stream) {
        s->dev_dirty = false;
        latch_hints(s);
      }
      if (h[i]->min_bad_enc != 0) {
        s->last_bad = (i64)~h[i]->min_bad_enc;
        if (first_bad) first_bad[i] = s->last_bad;
        rcs[i] = hipMemsetAsync(s->d_err, 0, sizeof(ErrState), st) == hipSuccess && hipStreamSynchronize(st) == hipSuccess
                     ? GLINT_EOUTOFRANGE : GLINT_EDEVICE;
      }
    }
    if (rcs[i] != GLINT_OK) (void)hipGetLastError();
    if (rc == GLINT_OK) rc = rcs[i];
  }
  return rc;
}

int glint_shard_sync(glint_shard_t s, void* stream, int64_t* first_bad) {
  if (!s) return GLINT_EINVAL;
  ShardLock lk(s);
  DeviceGuard g(s->device);
  hipStream_t st = (hipStream_t)stream;
  // the error state rides back behind the stream's work (pinned, async): one synchronisation
  ErrState local{};
  ErrState* h = s->h_err ? s->h_err : &local;
  HIPCHK(hipMemcpyAsync(h, s->d_err, sizeof(ErrState), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (st == s->last_dev_stream) {
    s->dev_dirty = false;  // everything enqueued there has completed
    latch_hints(s);        // a sync point: later pushes decide from the pushes up to here
  }
  if (h->min_bad_enc == 0) return GLINT_OK;
  s->last_bad = (i64)~h->min_bad_enc;
  if (first_bad) *first_bad = s->last_bad;
  HIPCHK(hipMemsetAsync(s->d_err, 0, sizeof(ErrState), st));
  HIPCHK(hipStreamSynchronize(st));
  return GLINT_EOUTOFRANGE;
}

// ---- device-resident ---------------------------------------------------------------------------
int glint_vec_push_dev(glint_shard_t s, const int64_t* keys, const void* vals, int64_t n, int flags, void* stream) {
  if (!s || n < 0) return GLINT_EINVAL;
  if (s->part.cols != 0) return GLINT_EINVAL;
  ShardLock lk(s);
  DeviceGuard g(s->device);
  if (int rc = dev_order_after_host(s, (hipStream_t)stream)) return rc;
  GLINT_DISPATCH(s->dtype, push_vec_t, s, (const i64*)keys, nullptr, vals, n, flags, pick(s, stream));
}

int glint_mat_push_dev(glint_shard_t s, const int64_t* rows, const int32_t* cols, const void* vals, int64_t n,
                       int flags, void* stream) {
  if (!s || n < 0) return GLINT_EINVAL;
  if (s->part.cols == 0) return GLINT_EINVAL;
  ShardLock lk(s);
  DeviceGuard g(s->device);
  if (int rc = dev_order_after_host(s, (hipStream_t)stream)) return rc;
  GLINT_DISPATCH(s->dtype, push_mat_t, s, (const i64*)rows, cols, vals, n, flags, pick(s, stream));
}

int glint_vec_push_dev_gated(glint_shard_t s, const int64_t* keys, const void* vals, int64_t n, int flags,
                             uint64_t* gate, void* stream) {
  if (!s || n < 0 || !gate) return GLINT_EINVAL;
  if (s->part.cols != 0) return GLINT_EINVAL;
  ShardLock lk(s);
  DeviceGuard g(s->device);
  if (int rc = dev_order_after_host(s, (hipStream_t)stream)) return rc;
  struct Gate {
    glint_shard* s;
    ~Gate() { s->gate = nullptr; }
  } reset{s};
  // a gate word in glint_host_alloc memory is read / written by the kernels through its device
  // address, and the caller reads the verdict straight from host memory after its wait
  u64* gd = (u64*)host_dev_ptr(gate, sizeof(u64), sizeof(u64));
  s->gate = gd ? gd : (u64*)gate;
  if (n == 0 && (flags & GLINT_PUSH_VALIDATE)) {  // nothing to check: the verdict is "none rejected"
    HIPCHK(hipMemsetAsync(s->gate, 0, sizeof(u64), pick(s, stream)));
    return GLINT_OK;
  }
  GLINT_DISPATCH(s->dtype, push_vec_t, s, (const i64*)keys, nullptr, vals, n, flags, pick(s, stream));
}

int glint_mat_push_dev_gated(glint_shard_t s, const int64_t* rows, const int32_t* cols, const void* vals, int64_t n,
                             int flags, uint64_t* gate, void* stream) {
  if (!s || n < 0 || !gate) return GLINT_EINVAL;
  if (s->part.cols == 0) return GLINT_EINVAL;
  ShardLock lk(s);
  DeviceGuard g(s->device);
  if (int rc = dev_order_after_host(s, (hipStream_t)stream)) return rc;
  struct Gate {
    glint_shard* s;
    ~Gate() { s->gate = nullptr; }
  } reset{s};
  // a gate word in glint_host_alloc memory is read / written by the kernels through its device
  // address, and the caller reads the verdict straight from host memory after its wait
  u64* gd = (u64*)host_dev_ptr(gate, sizeof(u64), sizeof(u64));
  s->gate = gd ? gd : (u64*)gate;
  if (n == 0 && (flags & GLINT_PUSH_VALIDATE)) {  // nothing to check: the verdict is "none rejected"
    HIPCHK(hipMemsetAsync(s->gate, 0, sizeof(u64), pick(s, stream)));
    return GLINT_OK;
  }
  GLINT_DISPATCH(s->dtype, push_mat_t, s, (const i64*)rows, cols, vals, n, flags, pick(s, stream));
}

int glint_vec_push_dev_shards(glint_shard_t* shards, int m, const int64_t* keys, const void* vals, int64_t n,
                              uint64_t* gate, void* stream) {
  if (!shards || m <= 0 || m > kMaxSetShards || n < 0 || !gate || (n > 0 && (!keys || !vals))) return GLINT_EINVAL;
  std::vector<glint_shard*> v(shards, shards + m);
  for (glint_shard* s : v)
    if (!s || s->part.cols != 0 || s->part.kind != 0 || s->dtype != v[0]->dtype || s->device != v[0]->device)
      return GLINT_EINVAL;
  std::sort(v.begin(), v.end(), [](const glint_shard* a, const glint_shard* b) { return a->part.start < b->part.start; });
  for (int j = 1; j < m; ++j)  // disjoint ranges (each once)
    if (v[j - 1]->part.start + v[j - 1]->part.size > v[j]->part.start || v[j - 1] == v[j]) return GLINT_EINVAL;
  std::vector<glint_shard*> order(v);  // every shard's lock, in lock_order, for the whole call
  lock_order(order);
  struct Locks {
    std::vector<glint_shard*>& o;
    size_t k = 0;
    ~Locks() {
      for (size_t i = 0; i < k; ++i) o[i]->mu.unlock();
    }
  } locks{order};
  for (; locks.k < order.size(); ++locks.k) order[locks.k]->mu.lock();
  for (glint_shard* s : v)  // a slab with views orders itself through their locks (held here if in the set)
    if (!s->views.empty()) return GLINT_EINVAL;
  DeviceGuard g(v[0]->device);
  hipStream_t st = (hipStream_t)stream;
  for (glint_shard* s : v) {
    if (int rc = dev_order_after_host(s, st)) return rc;
    (void)pick(s, stream);
  }
  u64* gd = (u64*)host_dev_ptr(gate, sizeof(u64), sizeof(u64));
  if (!gd) gd = (u64*)gate;
  if (n == 0) {
    HIPCHK(hipMemsetAsync(gd, 0, sizeof(u64), st));
    return GLINT_OK;
  }
  switch (v[0]->dtype) {
    case GLINT_F64: return launch_set_push<double>(v.data(), m, (const i64*)keys, vals, n, gd, st);
    case GLINT_F32: return launch_set_push<float>(v.data(), m, (const i64*)keys, vals, n, gd, st);
    case GLINT_I64: return launch_set_push<long long>(v.data(), m, (const i64*)keys, vals, n, gd, st);
    case GLINT_I32: return launch_set_push<int>(v.data(), m, (const i64*)keys, vals, n, gd, st);
    default: return GLINT_EINVAL;
  }
}

int glint_vec_pull_dev(glint_shard_t s, const int64_t* keys, void* out, int64_t n, void* stream) {
  if (!s || n < 0) return GLINT_EINVAL;
  if (s->part.cols != 0) return GLINT_EINVAL;
  ShardLock lk(s);
  DeviceGuard g(s->device);
  if (int rc = dev_order_after_host(s, (hipStream_t)stream)) return rc;
  GLINT_DISPATCH(s->dtype, launch_vec_pull, s, (const i64*)keys, out, n, pick(s, stream));
}

int glint_mat_pull_dev(glint_shard_t s, const int64_t* rows, const int32_t* cols, void* out, int64_t n,
                       void* stream) {
  if (!s || n < 0) return GLINT_EINVAL;
  if (s->part.cols == 0) return GLINT_EINVAL;
  ShardLock lk(s);
  DeviceGuard g(s->device);
  if (int rc = dev_order_after_host(s, (hipStream_t)stream)) return rc;
  GLINT_DISPATCH(s->dtype, launch_mat_pull, s, (const i64*)rows, cols, out, n, pick(s, stream));
}

int glint_mat_pull_rows_dev(glint_shard_t s, const int64_t* rows, void* out, int64_t n, void* stream) {
  if (!s || n < 0) return GLINT_EINVAL;
  if (s->part.cols == 0) return GLINT_EINVAL;
  ShardLock lk(s);
  DeviceGuard g(s->device);
  if (int rc = dev_order_after_host(s, (hipStream_t)stream)) return rc;
  GLINT_DISPATCH(s->dtype, launch_mat_pull_rows, s, (const i64*)rows, out, n, pick(s, stream));
}

}  // extern "C"

// ---- host-pointer entry points --------------------------------------------------------------------
namespace {

// Host arrays up to this size are staged through the shard's pinned buffer: one CPU memcpy per
// section, then ONE DMA for the whole message (a pageable hipMemcpy costs a driver-side bounce and a
// fence per section, which dominated small Akka-sized messages: ~1000 records per push,
// GranularBigVectorSpec.scala:21). Larger arrays go straight from pageable memory at PCIe rate.
// GLINT_PINNED_STAGE_MAX (bytes) overrides the crossover; tools/host_latency.py measures it.
size_t pinned_stage_max() {
  static EnvKnob k("GLINT_PINNED_STAGE_MAX");
  return (size_t)k.get([](const char* e) -> long long {
    return e ? (long long)std::strtoull(e, nullptr, 10) : (2ll << 20);
  });
}

// stage host arrays into the shard's device scratch: returns device pointers to each section and,
// when the call is small enough, the pinned host block that mirrors the scratch (pinned = true)
struct Staged {
  char* p[3] = {nullptr, nullptr, nullptr};
  bool pinned = false;
  size_t in_bytes = 0;  // bytes of the staged input sections (the pinned block's first part)
};

int stage(glint_shard* s, const void* const* src, const size_t* bytes, int count, Staged& out, size_t extra,
          char** extra_ptr) {
  size_t need = 0;
  for (int i = 0; i < count; ++i) need += pad256(bytes[i]);
  out.in_bytes = need;
  need += pad256(extra);
  int rc = grow(&s->d_scratch, &s->scratch_bytes, need);
  if (rc) return rc;
  out.pinned = need <= pinned_stage_max() && grow_pinned(&s->h_stage, &s->h_stage_bytes, need) == GLINT_OK;
  char* b = (char*)s->d_scratch;
  char* h = (char*)s->h_stage;
  for (int i = 0; i < count; ++i) {
    out.p[i] = b;
    if (bytes[i]) {
      if (out.pinned) std::memcpy(h, src[i], bytes[i]);
      else HIPCHK(hipMemcpyAsync(b, src[i], bytes[i], hipMemcpyHostToDevice, s->stream));
    }
    b += pad256(bytes[i]);
    h += pad256(bytes[i]);
  }
  if (out.pinned && out.in_bytes) {
    HIPCHK(hipMemcpyAsync(s->d_scratch, s->h_stage, out.in_bytes, hipMemcpyHostToDevice, s->stream));
  }
  if (extra_ptr) *extra_ptr = b;
  return GLINT_OK;
}

// Ends a host call: the device error state rides back with the call's last copy (pinned, async),
// so a clean call costs one stream synchronisation.
int finish(glint_shard* s) {
  ErrState local{};
  ErrState* h = s->h_err ? s->h_err : &local;
  HIPCHK(hipMemcpyAsync(h, s->d_err_host, sizeof(ErrState), hipMemcpyDeviceToHost, s->stream));
  HIPCHK(hipStreamSynchronize(s->stream));
  if (!s->dev_dirty) latch_hints(s);  // a sync point (the shard's pushes all ran on this stream)
  if (h->min_bad_enc == 0) return GLINT_OK;
  s->last_bad = (i64)~h->min_bad_enc;
  HIPCHK(hipMemsetAsync(s->d_err_host, 0, sizeof(ErrState), s->stream));
  HIPCHK(hipStreamSynchronize(s->stream));
  return GLINT_EOUTOFRANGE;
}

// ---- host-side validation of ring messages ------------------------------------------------------
// The first record of a message the reference would reject -- RangePartition.globalToLocal /
// CyclicPartition.globalToLocal (`.toInt` included) outside [0, size), or a column outside [0, cols)
// (PartialVector.scala:37-41, PartialMatrix.scala:77-81 throw ArrayIndexOutOfBoundsException there)
// -- or -1. The arrays are host memory the call copies anyway (any alignment: wire sections start at
// odd offsets). A ring message is checked here, before it is enqueued, so its error belongs to the
// call that enqueues it -- the Push or Pull message itself, as in the reference -- and a rejected
// message is not applied at all.
i64 host_first_bad(const glint_shard* s, const void* keys, const void* cols, i64 n) {
  const PartDesc& p = s->part;
  const char* kb = (const char*)keys;
  const char* cb = (const char*)cols;
  if (p.kind == 0) {
    // the common case (range layout): one branch-free pass the compiler vectorises -- (key - start)
    // .toInt in [0, size) is one unsigned compare -- and a scalar search only when something failed
    u32 any = 0;
    const u32 size = (u32)p.size, ncols = (u32)p.cols;
    for (i64 i = 0; i < n; ++i) {
      int64_t k;
      std::memcpy(&k, kb + 8 * i, 8);
      any |= (u32)((u32)(int32_t)(k - p.start) >= size);
      if (cb) {
        int32_t c;
        std::memcpy(&c, cb + 4 * i, 4);
        any |= (u32)((u32)c >= ncols);
      }
    }
    if (!any) return -1;
  }
  for (i64 i = 0; i < n; ++i) {
    int64_t k;
    std::memcpy(&k, kb + 8 * i, 8);
    const int32_t l = p.kind == 0 ? (int32_t)(k - p.start) : (int32_t)((k - (i64)p.cidx) / (i64)p.cparts);
    bool ok = l >= 0 && l < p.size;
    if (cb) {
      int32_t c;
      std::memcpy(&c, cb + 4 * i, 4);
      ok = ok && c >= 0 && c < p.cols;
    }
    if (!ok) return i;
  }
  return -1;
}

// GLINT_EOUTOFRANGE with the record index for glint_shard_last_error when a message has a bad record
inline int reject_if_bad(glint_shard* s, const void* keys, const void* cols, i64 n) {
  const i64 bad = host_first_bad(s, keys, cols, n);
  if (bad < 0) return GLINT_OK;
  s->last_bad = bad;
  return GLINT_EOUTOFRANGE;
}

// ---- pinned ring (pipelined ingest) -------------------------------------------------------------
constexpr i64 kRingMaxRecords = (i64)1 << 20;
// an async pull whose answer is larger than this is answered synchronously (staged copies) instead of
// through a ring slot, and a slot grown above kSlotKeepBytes is released when its entry retires: the
// ring's pinned memory stays bounded by what message-sized traffic needs
constexpr size_t kRingAnswerMax = (size_t)16 << 20;
constexpr size_t kSlotKeepBytes = (size_t)4 << 20;

struct StageLayout {
  size_t kb, cb, vb, total;  // keys | cols (matrix) | values, each section 256-aligned
};
StageLayout stage_layout(const glint_shard* s, i64 n) {
  StageLayout L;
  L.kb = pad256((size_t)n * 8);
  L.cb = s->part.cols != 0 ? pad256((size_t)n * 4) : 0;
  L.vb = pad256((size_t)n * s->vsize);
  L.total = L.kb + L.cb + L.vb;
  return L;
}

// Polls a host-mapped ticket word until it reaches `ticket` or `budget_us` has passed: a busy spin
// for the first few microseconds (a message-sized launch completes in about that), then
// sched_yield between polls, so that a server with many more waiting threads than cores (one
// thread per client connection) hands the CPU to the threads that have work instead of spinning
// against them.
// After a short spin a lone waiter yields (a message's round trip stays ~10 us: window-1 clients);
// when more than kBusyWaiters threads of the process are waiting at once, each sleeps between polls
// instead (50 us), leaving the cores to the threads that have work: the loopback servers run hundreds
// of connection threads on a 16-core share, and yielding waiters there cost the cfg4a / cfg4b pull rows
// 16 % / 10 % (profiles/r04/loopback_wait_sleep.txt).
std::atomic<int> g_waiters{0};
constexpr int kBusyWaiters = 8;
constexpr long long kWaitSleepUs = 50;
bool poll_word(const u64* word, u64 ticket, double budget_us) {
  constexpr double kSpinUs = 4.0;
  struct Count {
    Count() { g_waiters.fetch_add(1, std::memory_order_relaxed); }
    ~Count() { g_waiters.fetch_sub(1, std::memory_order_relaxed); }
  } count;
  const auto t0 = std::chrono::steady_clock::now();
  for (u32 i = 0;; ++i) {
    if (__atomic_load_n(word, __ATOMIC_ACQUIRE) >= ticket) return true;
    if ((i & 15) == 15) {
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      if (us > budget_us) return false;
      if (us > kSpinUs) {
        if (g_waiters.load(std::memory_order_relaxed) > kBusyWaiters) {
          const struct timespec ts = {0, (long)kWaitSleepUs * 1000};
          nanosleep(&ts, nullptr);
        } else {
          sched_yield();
        }
        continue;
      }
    }
    __builtin_ia32_pause();
  }
}

// Waits until the launch that carries `ticket` has written it to h_done (tickets complete in stream
// order, so a later ticket there covers this one). Polls briefly, then lets HIP block on the
// stream, which also surfaces a device error.
int wait_done(glint_shard* s, u64 ticket) {
  if (poll_word(s->h_done, ticket, 200.0)) return GLINT_OK;
  HIPCHK(hipStreamSynchronize(s->stream));
  return __atomic_load_n(s->h_done, __ATOMIC_ACQUIRE) >= ticket ? GLINT_OK : GLINT_EDEVICE;
}

// Retires a slot: waits for its entry and hands an async pull its answer. Ring messages were
// validated on the host before they were enqueued, so their kernels reject nothing: a rejected
// record here means the device and the host check disagree, a device fault.
int ring_retire(glint_shard* s, glint_shard::RingSlot& r) {
  if (!r.inflight) return GLINT_OK;
  const u64 tw = s->hprof ? host_ns() : 0;
  if (r.sig) {
    const int rc = wait_done(s, r.ticket);
    if (rc) return rc;
  } else {
    HIPCHK(hipEventSynchronize(r.done));
  }
  const u64 tc = s->hprof ? host_ns() : 0;
  if (tw) {
    s->hp.retire_wait.fetch_add(tc - tw, std::memory_order_relaxed);
    s->hp.nretire_wait.fetch_add(1, std::memory_order_relaxed);
  }
  r.inflight = false;
  const int err = __atomic_load_n(&r.herr->min_bad_enc, __ATOMIC_ACQUIRE) != 0 ? GLINT_EDEVICE : GLINT_OK;
  if (r.out) {
    std::memcpy(r.out, r.h + r.out_off, r.out_bytes);
    r.out = nullptr;
  }
  if (r.pull_batch) {
    for (const auto& m : r.msgs)
      if (!m.dout) std::memcpy(m.out, r.h + r.out_off + (size_t)m.off * s->vsize, (size_t)m.n * s->vsize);
    for (auto& m : r.msgs) m.hold.reset();  // the kernel's writes into caller buffers are complete
    r.pull_batch = false;
  }
  if (tc) s->hp.copy.fetch_add(host_ns() - tc, std::memory_order_relaxed);
  if (r.hcap > kSlotKeepBytes) {  // a large entry's slot: give the pinned memory back
    (void)hipHostFree(r.h);
    r.h = r.hd = nullptr;
    r.hcap = 0;
  }
  if (r.dcap > kSlotKeepBytes) {
    (void)hipFree(r.d);
    r.d = nullptr;
    r.dcap = 0;
  }
  return err;
}

// Retires, oldest first, every in-flight entry that covers a ticket <= t (errors then belong to
// the earliest message that saw them).
int ring_retire_through(glint_shard* s, u64 t) {
  for (;;) {
    glint_shard::RingSlot* next = nullptr;
    for (auto& r : s->ring)
      if (r.inflight && r.ticket_lo <= t && (!next || r.ticket_lo < next->ticket_lo)) next = &r;
    if (!next) return GLINT_OK;
    const int rc = ring_retire(s, *next);
    if (rc) return rc;
  }
}

// the pinned bytes a coalesced pull batch needs (keys, cols, answers, destination table): every
// slot is pinned at least this large from the start
inline size_t pull_slot_min(const glint_shard* s) {
  const StageLayout L = stage_layout(s, kRingPullMax);
  return L.kb + L.cb + pad256((size_t)kRingPullMax * s->vsize) + sizeof(PullDst) * kPullDirectMax;
}

// Hands out a free slot sized for n records (and, for a pull, an answer of out_bytes behind the
// key sections). Retires the slot's previous entry (and every older one) first.
int ring_acquire_locked(glint_shard* s, i64 n, int* slot, size_t out_bytes = 0) {
  if (n < 0 || n > kRingMaxRecords) return GLINT_EINVAL;
  const StageLayout L = stage_layout(s, n);
  const size_t need = std::max(L.total, L.kb + L.cb + pad256(out_bytes));
  if (!s->h_done) {
    if (hipHostMalloc((void**)&s->h_done, 256, hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer((void**)&s->d_done, s->h_done, 0) != hipSuccess) {
      (void)hipGetLastError();
      if (s->h_done) (void)hipHostFree(s->h_done);
      s->h_done = s->d_done = nullptr;
      return GLINT_ENOMEM;
    }
    __atomic_store_n(s->h_done, (u64)0, __ATOMIC_RELEASE);
  }
  for (int tries = 0; tries < GLINT_RING_SLOTS; ++tries) {
    const int idx = s->ring_next;
    s->ring_next = (idx + 1) % GLINT_RING_SLOTS;
    glint_shard::RingSlot& r = s->ring[idx];
    if (r.acquired) continue;  // handed out (or an open batch) and not launched yet
    if (r.inflight) {
      const int rc = ring_retire_through(s, r.ticket_lo);
      if (rc) return rc;
    }
    if (r.hcap < need) {
      if (r.h) (void)hipHostFree(r.h);
      r.h = r.hd = nullptr;
      r.hcap = 0;
      // at least a coalesced batch of either kind: a slot first sized for a push batch (keys + values,
      // 64 KiB of Double) and later taken by a pull batch (keys + answers + destination table) would
      // otherwise be freed and re-pinned in the middle of the traffic (cfg1 pulls 124 -> 62 M/s)
      size_t cap = std::max<size_t>((size_t)1 << 17, pull_slot_min(s));
      while (cap < need) cap <<= 1;
      if (hipHostMalloc((void**)&r.h, cap, hipHostMallocMapped) != hipSuccess ||
          hipHostGetDevicePointer((void**)&r.hd, r.h, 0) != hipSuccess) {
        (void)hipGetLastError();
        if (r.h) (void)hipHostFree(r.h);
        r.h = r.hd = nullptr;
        return GLINT_ENOMEM;
      }
      r.hcap = cap;
    }
    if (!r.done && hipEventCreateWithFlags(&r.done, hipEventDisableTiming) != hipSuccess) {
      (void)hipGetLastError();
      r.done = nullptr;
      return GLINT_EDEVICE;
    }
    if (!r.herr) {
      if (hipHostMalloc((void**)&r.herr, sizeof(ErrState), hipHostMallocMapped) != hipSuccess ||
          hipHostGetDevicePointer((void**)&r.herr_d, r.herr, 0) != hipSuccess) {
        (void)hipGetLastError();
      if (r.herr) (void)hipHostFree(r.herr);
        r.herr = r.herr_d = nullptr;
        return GLINT_ENOMEM;
      }
    }
    r.acquired = true;
    r.n = n;
    r.cap_need = need;
    r.out = nullptr;
    r.fill = 0;
    r.msgs.clear();
    r.pull_batch = false;
    *slot = idx;
    return GLINT_OK;
  }
  return GLINT_ENOMEM;  // every slot handed out and not pushed
}

// ---- caller buffers the kernels can write (glint_host_alloc) -----------------------------------
// Pinned, device-mapped host memory handed to a server for its response images: a coalesced pull
// whose destination lies in one is answered by the kernel straight into it.
struct HostRange {
  char* h;
  size_t n;
  char* d;
  std::shared_ptr<std::atomic<long>> pending;  // kernel writes enqueued into it and not yet retired
};
std::mutex g_host_mu;
std::vector<HostRange> g_host;  // sorted by h

// p's device address if [p, p + bytes) lies in one glint_host_alloc buffer and p is aligned to
// `align`, else nullptr; with `hold`, the buffer is held (glint_host_free refuses it) until *hold resets
void* host_dev_ptr(const void* p, size_t bytes, size_t align, HostHold* hold) {
  if (!p || (uintptr_t)p % align) return nullptr;
  std::lock_guard<std::mutex> lk(g_host_mu);
  if (g_host.empty()) return nullptr;
  const char* c = (const char*)p;
  auto it = std::upper_bound(g_host.begin(), g_host.end(), c,
                             [](const char* x, const HostRange& r) { return x < r.h; });
  if (it == g_host.begin()) return nullptr;
  --it;
  if (c + bytes > it->h + it->n) return nullptr;
  if (hold) *hold = HostHold(it->pending);
  return it->d + (c - it->h);
}

// smallest answer (bytes) a pull writes straight into a glint_host_alloc buffer (GLINT_DIRECT_MIN_BYTES)
size_t direct_min_bytes() {
  static EnvKnob k("GLINT_DIRECT_MIN_BYTES");
  return (size_t)k.get([](const char* e) -> long long { return e ? atoll(e) : 4096ll; });
}

// a coalesced pull batch's destination table: behind the answer section of its slot
inline size_t pull_tab_off(const glint_shard* s, const StageLayout& L) {
  return L.kb + L.cb + pad256((size_t)kRingPullMax * s->vsize);  // (kPullBatch, below)
}

// whether an entry of n records is one signalling launch reading (and answering) in the mapped slot
inline bool ring_direct(const glint_shard* s, i64 n) { return n <= GLINT_ZERO_COPY_MAX && s->elems < ((i64)1 << 32); }

// Runs `launch` (the entry's kernels on s->stream) for slot r, covering tickets [lo, hi]: a direct
// entry is one workgroup that signals hi itself; any other entry ends with an error-state copy and
// an event.
// A launch that fails after the entry's tickets were handed out drops the entry: its tickets are
// remembered as failed, so the wait that covers them reports the failure.
void drop_entry(glint_shard* s, glint_shard::RingSlot& r, u64 lo, u64 hi, int rc) {
  r.acquired = false;
  r.out = nullptr;
  r.pull_batch = false;
  r.msgs.clear();
  if (hi >= lo && lo > 0) s->failed.push_back({lo, hi, rc});
}

template <typename F>
int ring_dispatch(glint_shard* s, glint_shard::RingSlot& r, bool direct, u64 lo, u64 hi, F launch) {
  if (direct) s->sig = MsgSig{s->d_done, hi, r.herr_d};
  int rc;
  {
    HostCall hc(s);  // ring messages are host-pointer calls: their kernels use the host error state
    rc = launch();
  }
  s->sig = MsgSig{nullptr, 0, nullptr};
  if (rc == GLINT_OK && !direct &&
      (hipMemcpyAsync(r.herr, s->d_err_host, sizeof(ErrState), hipMemcpyDeviceToHost, s->stream) != hipSuccess ||
       hipEventRecord(r.done, s->stream) != hipSuccess)) {
    (void)hipGetLastError();
    rc = GLINT_EDEVICE;
  }
  if (rc) {
    (void)hipStreamSynchronize(s->stream);
    drop_entry(s, r, lo, hi, rc);
    return rc;
  }
  r.ticket_lo = lo;
  r.ticket = hi;
  r.sig = direct;
  r.inflight = true;
  r.acquired = false;
  s->host_pending = true;
  return GLINT_OK;
}

// ---- message coalescing -------------------------------------------------------------------------
// Consecutive message-sized pushes with the same flags are appended to one open ring slot and go to
// the GPU as ONE single-workgroup ordered push when the slot is full or anything else needs the
// stream (another entry, a wait, a device call). The fold runs over the concatenation in arrival
// order -- each message applied after the one before it, the actor's own sequence -- so results
// are those of one launch per message. Every message keeps its ticket; the launch signals the last.
constexpr i64 kBatchMax = GLINT_ZERO_COPY_MAX;
constexpr i64 kPullBatch = kRingPullMax;  // records per coalesced pull batch (= kBatchMax)

int launch_push_entry(glint_shard* s, glint_shard::RingSlot& r, const char* base, const StageLayout& L, i64 n,
                      int flags, bool direct, u64 lo, u64 hi) {
  const bool mat = s->part.cols != 0;
  const i64* keys = (const i64*)base;
  const int32_t* cols = mat ? (const int32_t*)(base + L.kb) : nullptr;
  const void* vals = base + L.kb + L.cb;
  const int hflags = flags | kPushHostSequential;  // the actor's update: message order by default
  return ring_dispatch(s, r, direct && n > 0, lo, hi, [&]() -> int {
    if (n == 0) return GLINT_OK;
    if (mat) {
      GLINT_DISPATCH(s->dtype, push_mat_t, s, keys, cols, vals, n, hflags, s->stream);
    }
    GLINT_DISPATCH(s->dtype, push_vec_t, s, keys, nullptr, vals, n, hflags, s->stream);
  });
}

int launch_pull_batch(glint_shard* s, glint_shard::RingSlot& r, int kind);

// launches the open batch, if any
int ring_flush_locked(glint_shard* s) {
  if (s->open_slot < 0) return GLINT_OK;
  glint_shard::RingSlot& r = s->ring[s->open_slot];
  s->open_slot = -1;
  int rc = order_after_dev(s);
  if (rc) {
    drop_entry(s, r, r.msgs.front().ticket, r.msgs.back().ticket, rc);
    return rc;
  }
  if (s->open_kind >= 0) return launch_pull_batch(s, r, s->open_kind);
  return launch_push_entry(s, r, r.hd, stage_layout(s, kBatchMax), r.fill, s->open_flags, true,
                           r.msgs.front().ticket, r.msgs.back().ticket);
}

inline bool batchable(const glint_shard* s, i64 n) { return n > 0 && n <= kBatchMax && s->elems < ((i64)1 << 32); }

// Appends one message-sized push (sections: keys, cols for matrices, values; any alignment) to the
// open batch, opening one if needed; *ticket = the message's own ticket.
int ring_append_locked(glint_shard* s, i64 n, int flags, const void* k, const void* c, const void* v, u64* ticket,
                       bool checked = false) {
  int rc = checked ? GLINT_OK : reject_if_bad(s, k, s->part.cols != 0 ? c : nullptr, n);
  if (rc) return rc;
  if (s->open_slot >= 0 &&
      (s->open_kind >= 0 || flags != s->open_flags || s->ring[s->open_slot].fill + n > kBatchMax)) {
    rc = ring_flush_locked(s);
    if (rc) return rc;
  }
  if (s->open_slot < 0) {
    int slot = -1;
    rc = ring_acquire_locked(s, kBatchMax, &slot);
    if (rc) return rc;
    s->open_slot = slot;
    s->open_flags = flags;
    s->open_kind = -1;
  }
  glint_shard::RingSlot& r = s->ring[s->open_slot];
  const StageLayout L = stage_layout(s, kBatchMax);
  std::memcpy(r.h + (size_t)r.fill * 8, k, (size_t)n * 8);
  if (s->part.cols != 0) std::memcpy(r.h + L.kb + (size_t)r.fill * 4, c, (size_t)n * 4);
  std::memcpy(r.h + L.kb + L.cb + (size_t)r.fill * s->vsize, v, (size_t)n * s->vsize);
  const u64 t = ++s->ticket_next;
  r.msgs.push_back({r.fill, n, t});
  r.fill += n;
  if (ticket) *ticket = t;
  if (r.fill == kBatchMax) return ring_flush_locked(s);
  return GLINT_OK;
}

// Enqueues the push staged in slot idx. Message-sized pushes join the open batch (one copy inside
// pinned memory); larger ones are copied to the device with one DMA and launched at once.
int ring_push_locked(glint_shard* s, int idx, i64 n, int flags, u64* ticket) {
  if (idx < 0 || idx >= GLINT_RING_SLOTS || idx == s->open_slot) return GLINT_EINVAL;
  glint_shard::RingSlot& r = s->ring[idx];
  if (!r.acquired || n < 0 || n > r.n) return GLINT_EINVAL;
  const StageLayout L = stage_layout(s, r.n);  // the sections as handed out
  if (batchable(s, n)) {
    // the records move to the batch; the slot stays acquired until they are copied (the batch's
    // slot search then cannot pick it), and is free again after
    const int rc = ring_append_locked(s, n, flags, r.h, r.h + L.kb, r.h + L.kb + L.cb, ticket);
    r.acquired = false;
    return rc;
  }
  int rc = reject_if_bad(s, r.h, s->part.cols != 0 ? r.h + L.kb : nullptr, n);
  if (rc == GLINT_OK) rc = ring_flush_locked(s);
  if (rc == GLINT_OK) rc = order_after_dev(s);
  const bool direct = ring_direct(s, n);
  const char* base = r.hd;
  if (rc == GLINT_OK && !direct) {
    rc = grow((void**)&r.d, &r.dcap, L.total);
    if (rc == GLINT_OK && hipMemcpyAsync(r.d, r.h, L.total, hipMemcpyHostToDevice, s->stream) != hipSuccess) {
      (void)hipGetLastError();
      rc = GLINT_EDEVICE;
    }
    base = r.d;
  }
  if (rc) {
    r.acquired = false;  // nothing enqueued: the slot is free again
    return rc;
  }
  const u64 t = ++s->ticket_next;
  r.msgs.assign(1, glint_shard::RingSlot::Msg{0, n, t});
  rc = launch_push_entry(s, r, base, L, n, flags, direct, t, t);
  if (rc) return rc;
  if (ticket) *ticket = t;
  return GLINT_OK;
}

// Enqueues a pull whose keys (and cols) are in slot idx; kind 0 vector get, 1 matrix get, 2 rows.
// The answer is written into the slot behind the key sections and copied to `out` when the slot
// retires (glint_shard_wait, or the slot's reuse).
int ring_pull_locked(glint_shard* s, int idx, int kind, i64 n, void* out, size_t out_bytes, u64* ticket) {
  glint_shard::RingSlot& r = s->ring[idx];
  int rc = ring_flush_locked(s);  // the pull sees every push enqueued before it
  if (rc == GLINT_OK) rc = order_after_dev(s);
  if (rc) {
    r.acquired = false;
    return rc;
  }
  const StageLayout L = stage_layout(s, n);
  const bool direct = n > 0 && ring_direct(s, n) && (kind != 2 || out_bytes <= ((size_t)1 << 20));
  const char* base = r.hd;
  char* ans = r.hd + L.kb + L.cb;
  if (!direct) {  // keys over by DMA, the answer back by DMA into the slot
    rc = grow((void**)&r.d, &r.dcap, L.kb + L.cb + pad256(out_bytes));
    if (rc) {
      r.acquired = false;
      return rc;
    }
    if (hipMemcpyAsync(r.d, r.h, L.kb + L.cb, hipMemcpyHostToDevice, s->stream) != hipSuccess) {
      (void)hipGetLastError();
      r.acquired = false;
      return GLINT_EDEVICE;
    }
    base = r.d;
    ans = r.d + L.kb + L.cb;
  }
  const i64* keys = (const i64*)base;
  const int32_t* cols = (const int32_t*)(base + L.kb);
  r.out = out;
  r.out_bytes = out_bytes;
  r.out_off = L.kb + L.cb;
  const u64 t = ++s->ticket_next;
  r.msgs.assign(1, glint_shard::RingSlot::Msg{0, n, t});
  rc = ring_dispatch(s, r, direct, t, t, [&]() -> int {
    int e;
    if (kind == 0) {
      e = [&]() -> int { GLINT_DISPATCH(s->dtype, launch_vec_pull, s, keys, ans, n, s->stream); }();
    } else if (kind == 1) {
      e = [&]() -> int { GLINT_DISPATCH(s->dtype, launch_mat_pull, s, keys, cols, ans, n, s->stream); }();
    } else {
      e = [&]() -> int { GLINT_DISPATCH(s->dtype, launch_mat_pull_rows, s, keys, ans, n, s->stream); }();
    }
    if (e || direct) return e;
    return hipMemcpyAsync(r.h + L.kb + L.cb, ans, out_bytes, hipMemcpyDeviceToHost, s->stream) == hipSuccess
               ? GLINT_OK
               : GLINT_EDEVICE;
  });
  if (rc) return rc;
  if (ticket) *ticket = t;
  return GLINT_OK;
}

// A coalesced pull batch: consecutive message-sized element pulls of one kind share one launch;
// each answer is copied to its own destination when the batch retires.
int launch_pull_batch(glint_shard* s, glint_shard::RingSlot& r, int kind) {
  const StageLayout L = stage_layout(s, kPullBatch);
  const i64* keys = (const i64*)r.hd;
  const int32_t* cols = (const int32_t*)(r.hd + L.kb);
  char* ans = r.hd + L.kb + L.cb;
  const i64 n = r.fill;
  r.out = nullptr;
  r.out_off = L.kb + L.cb;
  // messages answering into glint_host_alloc buffers: the kernel writes there itself, through a
  // destination table behind the answer section (the others keep their answer in the slot)
  bool direct = false;
  for (const auto& m : r.msgs) direct = direct || m.dout != nullptr;
  if (direct && r.msgs.size() <= (size_t)kPullDirectMax) {
    const size_t toff = pull_tab_off(s, L);
    PullDst* tab = reinterpret_cast<PullDst*>(r.h + toff);
    for (size_t i = 0; i < r.msgs.size(); ++i) {
      const auto& m = r.msgs[i];
      tab[i].off = (unsigned)m.off;
      tab[i].n = (unsigned)m.n;
      tab[i].dst = (unsigned long long)(uintptr_t)(m.dout ? (char*)m.dout : ans + (size_t)m.off * s->vsize);
    }
    s->pull_tab = reinterpret_cast<const PullDst*>(r.hd + toff);
    s->pull_nm = (int)r.msgs.size();
  } else {
    for (auto& m : r.msgs) {  // answered through the slot, copied out at retire
      m.dout = nullptr;
      m.hold.reset();
    }
  }
  const int rc = ring_dispatch(s, r, true, r.msgs.front().ticket, r.msgs.back().ticket, [&]() -> int {
    if (kind == 0) {
      GLINT_DISPATCH(s->dtype, launch_vec_pull, s, keys, ans, n, s->stream);
    }
    GLINT_DISPATCH(s->dtype, launch_mat_pull, s, keys, cols, ans, n, s->stream);
  });
  s->pull_tab = nullptr;
  s->pull_nm = 0;
  if (rc == GLINT_OK) r.pull_batch = true;
  return rc;
}

int ring_append_pull_locked(glint_shard* s, int kind, i64 n, const int64_t* keys, const int32_t* cols, void* out,
                            u64* ticket, bool checked) {
  int rc = checked ? GLINT_OK : reject_if_bad(s, keys, kind == 1 ? cols : nullptr, n);
  if (rc) return rc;
  if (s->open_slot >= 0 && (s->open_kind != kind || s->ring[s->open_slot].fill + n > kPullBatch)) {
    rc = ring_flush_locked(s);
    if (rc) return rc;
  }
  if (s->open_slot < 0) {
    int slot = -1;
    // the answer section, then the destination table (pull_tab_off)
    rc = ring_acquire_locked(s, kPullBatch, &slot, pad256((size_t)kPullBatch * s->vsize) + sizeof(PullDst) * kPullDirectMax);
    if (rc) return rc;
    s->open_slot = slot;
    s->open_kind = kind;
    s->open_flags = 0;
  }
  glint_shard::RingSlot& r = s->ring[s->open_slot];
  const StageLayout L = stage_layout(s, kPullBatch);
  std::memcpy(r.h + (size_t)r.fill * 8, keys, (size_t)n * 8);
  if (kind == 1) std::memcpy(r.h + L.kb + (size_t)r.fill * 4, cols, (size_t)n * 4);
  const u64 t = ++s->ticket_next;
  glint_shard::RingSlot::Msg m{r.fill, n, t};
  m.out = out;
  // answered in place only from a page of answer on: each message's destination costs the kernel's
  // stores a host-page translation, so small answers are cheaper copied out of the contiguous slot
  // (cfg4b's ~125-record pulls ran at half the rate in place; cfg4a's 1000-record ones 1.4x faster)
  m.dout = (size_t)n * s->vsize >= direct_min_bytes() ? host_dev_ptr(out, (size_t)n * s->vsize, s->vsize, &m.hold)
                                                       : nullptr;
  r.msgs.push_back(m);
  r.fill += n;
  if (ticket) *ticket = t;
  if (r.fill == kPullBatch) return ring_flush_locked(s);
  return GLINT_OK;
}

int ring_wait_locked(glint_shard* s, u64 ticket, i64* first_bad) {
  if (s->open_slot >= 0 && s->ring[s->open_slot].msgs.front().ticket <= ticket) {
    const int rc = ring_flush_locked(s);
    if (rc) return rc;
  }
  int rc = ring_retire_through(s, ticket);
  if (rc) return rc;
  // entries whose launch failed after their tickets were handed out: reported once, by the first
  // wait that covers them (rejected records never reach the ring: their calls returned the error)
  for (size_t i = 0; i < s->failed.size(); ++i) {
    if (s->failed[i].lo <= ticket) {
      rc = s->failed[i].rc;
      s->failed.erase(s->failed.begin() + (long)i);
      return rc;
    }
  }
  if (first_bad) *first_bad = -1;
  return GLINT_OK;
}

// A device-resident call runs on the caller's stream: it first waits for the ring entries enqueued
// on the shard's stream (they share the data array and the error state).
int dev_order_after_host(glint_shard* s, hipStream_t st) {
  // a slab's call reads or writes its views' elements: it waits for their host-pointer work, and
  // their later host-pointer calls wait for it (lock order: slab, then view)
  for (glint_shard* v : s->views) {
    ShardLock lv(v);
    if (int rc = dev_order_after_host(v, st)) return rc;
    v->last_dev_stream = st;
    v->dev_dirty = true;
  }
  int rc = ring_flush_locked(s);
  if (rc) return rc;
  if (!s->host_pending) return GLINT_OK;
  if (!s->host_ev && hipEventCreateWithFlags(&s->host_ev, hipEventDisableTiming) != hipSuccess) {
    (void)hipGetLastError();
    s->host_ev = nullptr;
    return GLINT_EDEVICE;
  }
  HIPCHK(hipEventRecord(s->host_ev, s->stream));
  HIPCHK(hipStreamWaitEvent(st, s->host_ev, 0));
  s->host_pending = false;
  return GLINT_OK;
}

// pull answer bytes: n values, or n rows of cols values
inline size_t pull_bytes(const glint_shard* s, int kind, i64 n) {
  return (size_t)n * s->vsize * (kind == 2 ? (size_t)s->part.cols : 1);
}

// Copies a pull's keys (and cols) into a fresh slot and enqueues it. The slot's answer reaches `out`
// when the slot retires.
int pull_enqueue_locked(glint_shard* s, int kind, const int64_t* keys, const int32_t* cols, void* out, int64_t n,
                        u64* ticket, bool checked = false) {
  if (kind != 2 && batchable(s, n)) return ring_append_pull_locked(s, kind, n, keys, cols, out, ticket, checked);
  int rc = checked ? GLINT_OK : reject_if_bad(s, keys, kind == 1 ? cols : nullptr, n);
  if (rc) return rc;
  int slot = -1;
  const size_t ob = pull_bytes(s, kind, n);
  rc = ring_acquire_locked(s, n, &slot, ob);
  if (rc) return rc;
  glint_shard::RingSlot& r = s->ring[slot];
  const StageLayout L = stage_layout(s, n);
  std::memcpy(r.h, keys, (size_t)n * 8);
  if (kind == 1) std::memcpy(r.h + L.kb, cols, (size_t)n * 4);
  return ring_pull_locked(s, slot, kind, n, out, ob, ticket);
}

int host_push(glint_shard* s, bool mat, const int64_t* keys, const int32_t* cols, const void* vals, int64_t n,
              int flags) {
  if (n < 0 || (n > 0 && (!keys || !vals || (mat && !cols)))) return GLINT_EINVAL;
  if (mat != (s->part.cols != 0)) return GLINT_EINVAL;
  if (n == 0) return GLINT_OK;
  ShardLock lk(s);
  DeviceGuard g(s->device);
  int rc = refuse_slab(s);
  if (rc == GLINT_OK) rc = order_after_dev(s);
  if (rc) return rc;
  if (batchable(s, n)) {  // Akka-sized: into the open batch (read in place by the kernel), then wait
    u64 ticket = 0;
    rc = ring_append_locked(s, n, flags, keys, cols, vals, &ticket);
    if (rc) return rc;
    return ring_wait_locked(s, ticket, nullptr);
  }
  rc = ring_flush_locked(s);
  if (rc) return rc;
  Staged st;
  const void* src[3] = {keys, mat ? (const void*)cols : vals, vals};
  size_t bytes[3] = {(size_t)n * 8, mat ? (size_t)n * 4 : (size_t)n * s->vsize, (size_t)n * s->vsize};
  rc = stage(s, src, bytes, mat ? 3 : 2, st, 0, nullptr);
  if (rc) return rc;
  const int hflags = flags | kPushHostSequential;  // the actor's update: message order by default
  HostCall hc(s);  // this call's rejected records are its own (d_err_host, read by finish)
  if (mat) {
    rc = [&]() -> int {
      GLINT_DISPATCH(s->dtype, push_mat_t, s, (const i64*)st.p[0], (const int32_t*)st.p[1], st.p[2], n, hflags,
                     s->stream);
    }();
  } else {
    rc = [&]() -> int {
      GLINT_DISPATCH(s->dtype, push_vec_t, s, (const i64*)st.p[0], nullptr, st.p[1], n, hflags, s->stream);
    }();
  }
  if (rc) {
    (void)hipStreamSynchronize(s->stream);  // the staging buffers stay busy until the stream drains
    return rc;
  }
  return finish(s);
}

// kind: 0 vector get, 1 matrix get, 2 matrix rows
int host_pull(glint_shard* s, int kind, const int64_t* keys, const int32_t* cols, void* out, int64_t n) {
  if (n < 0 || (n > 0 && (!keys || !out || (kind == 1 && !cols)))) return GLINT_EINVAL;
  if ((kind == 0) != (s->part.cols == 0)) return GLINT_EINVAL;
  if (n == 0) return GLINT_OK;
  ShardLock lk(s);
  DeviceGuard g(s->device);
  int rc = refuse_slab(s);
  if (rc == GLINT_OK) rc = ring_flush_locked(s);
  if (rc == GLINT_OK) rc = order_after_dev(s);
  if (rc) return rc;
  if (n <= GLINT_ZERO_COPY_MAX && pull_bytes(s, kind, n) <= kRingAnswerMax) {
    // Akka-sized: one workgroup reads the keys from a mapped pinned ring slot, writes the answer into
    // it and signals its ticket, so the call is one launch and a wait on host memory. The keys are
    // checked first: a rejected pull enqueues nothing and throws, as get() does in the reference.
    u64 ticket = 0;
    rc = pull_enqueue_locked(s, kind, keys, cols, out, n, &ticket);
    if (rc) return rc;
    return ring_wait_locked(s, ticket, nullptr);
  }
  const size_t out_bytes = (size_t)n * s->vsize * (kind == 2 ? (size_t)s->part.cols : 1);
  Staged st;
  const void* src[2] = {keys, cols};
  size_t bytes[2] = {(size_t)n * 8, kind == 1 ? (size_t)n * 4 : 0};
  char* d_out = nullptr;
  rc = stage(s, src, bytes, kind == 1 ? 2 : 1, st, out_bytes, &d_out);
  if (rc) return rc;
  HostCall hc(s);  // this call's rejected records are its own (d_err_host, read by finish)
  if (kind == 0) {
    rc = [&]() -> int { GLINT_DISPATCH(s->dtype, launch_vec_pull, s, (const i64*)st.p[0], d_out, n, s->stream); }();
  } else if (kind == 1) {
    rc = [&]() -> int {
      GLINT_DISPATCH(s->dtype, launch_mat_pull, s, (const i64*)st.p[0], (const int32_t*)st.p[1], d_out, n,
                     s->stream);
    }();
  } else {
    rc = [&]() -> int {
      GLINT_DISPATCH(s->dtype, launch_mat_pull_rows, s, (const i64*)st.p[0], d_out, n, s->stream);
    }();
  }
  if (rc) {
    (void)hipStreamSynchronize(s->stream);
    return rc;
  }
  if (st.pinned) {  // answer into the pinned block behind the inputs, then one CPU copy out
    char* h_out = (char*)s->h_stage + st.in_bytes;
    HIPCHK(hipMemcpyAsync(h_out, d_out, out_bytes, hipMemcpyDeviceToHost, s->stream));
    rc = finish(s);
    if (rc == GLINT_OK) std::memcpy(out, h_out, out_bytes);
    return rc;
  }
  HIPCHK(hipMemcpyAsync(out, d_out, out_bytes, hipMemcpyDeviceToHost, s->stream));
  return finish(s);
}

}  // namespace

extern "C" {

int glint_vec_push(glint_shard_t s, const int64_t* keys, const void* vals, int64_t n, int flags) {
  if (!s) return GLINT_EINVAL;
  return host_push(s, false, keys, nullptr, vals, n, flags);
}

int glint_vec_pull(glint_shard_t s, const int64_t* keys, void* out, int64_t n) {
  if (!s) return GLINT_EINVAL;
  return host_pull(s, 0, keys, nullptr, out, n);
}

int glint_mat_push(glint_shard_t s, const int64_t* rows, const int32_t* cols, const void* vals, int64_t n,
                   int flags) {
  if (!s) return GLINT_EINVAL;
  return host_push(s, true, rows, cols, vals, n, flags);
}

int glint_mat_pull(glint_shard_t s, const int64_t* rows, const int32_t* cols, void* out, int64_t n) {
  if (!s) return GLINT_EINVAL;
  return host_pull(s, 1, rows, cols, out, n);
}

int glint_mat_pull_rows(glint_shard_t s, const int64_t* rows, void* out, int64_t n) {
  if (!s) return GLINT_EINVAL;
  return host_pull(s, 2, rows, nullptr, out, n);
}

// RequestSerializer.fromBinary (RequestSerializer.scala:59-130) for the push messages, applied
// straight to the shard: the unaligned key/col/value sections are copied to the device as they lie.
int glint_push_wire(glint_shard_t s, const uint8_t* payload, size_t len, int32_t* id, int flags) {
  if (!s || !payload || len < 9) return GLINT_EINVAL;
  bool mat = false;
  const int dt = wire_dtype_of_push(payload[0], &mat);
  if (dt < 0 || dt != s->dtype || mat != (s->part.cols != 0)) return GLINT_EINVAL;
  int32_t n = 0, mid = 0;
  std::memcpy(&n, payload + 1, 4);
  std::memcpy(&mid, payload + 5, 4);
  if (n < 0) return GLINT_EINVAL;
  const size_t want = 9 + (size_t)n * (8 + (mat ? 4 : 0) + s->vsize);
  if (len != want) return GLINT_EINVAL;
  if (id) *id = mid;
  const uint8_t* keys = payload + 9;
  const uint8_t* cols = keys + (size_t)n * 8;
  const uint8_t* vals = cols + (mat ? (size_t)n * 4 : 0);
  return host_push(s, mat, (const int64_t*)keys, (const int32_t*)cols, vals, n, flags);
}

int glint_stage_acquire(glint_shard_t s, int64_t n, void** keys, void** cols, void** vals, int* slot) {
  if (!s || !keys || !vals || !slot) return GLINT_EINVAL;
  ShardLock lk(s);
  DeviceGuard g(s->device);
  int rc = refuse_slab(s);
  if (rc == GLINT_OK) rc = ring_acquire_locked(s, n, slot);
  if (rc) return rc;
  glint_shard::RingSlot& r = s->ring[*slot];
  const StageLayout L = stage_layout(s, n);
  *keys = r.h;
  if (cols) *cols = s->part.cols != 0 ? r.h + L.kb : nullptr;
  *vals = r.h + L.kb + L.cb;
  return GLINT_OK;
}

int glint_push_staged(glint_shard_t s, int slot, int64_t n, int flags, uint64_t* ticket) {
  if (!s) return GLINT_EINVAL;
  ShardLock lk(s);
  DeviceGuard g(s->device);
  if (int rc = refuse_slab(s)) return rc;
  return ring_push_locked(s, slot, n, flags, (u64*)ticket);
}

int glint_push_wire_async(glint_shard_t s, const uint8_t* payload, size_t len, int32_t* id, int flags,
                          uint64_t* ticket) {
  if (!s || !payload || len < 9) return GLINT_EINVAL;
  bool mat = false;
  const int dt = wire_dtype_of_push(payload[0], &mat);
  if (dt < 0 || dt != s->dtype || mat != (s->part.cols != 0)) return GLINT_EINVAL;
  int32_t n = 0, mid = 0;
  std::memcpy(&n, payload + 1, 4);
  std::memcpy(&mid, payload + 5, 4);
  if (n < 0) return GLINT_EINVAL;
  if (len != 9 + (size_t)n * (8 + (mat ? 4 : 0) + s->vsize)) return GLINT_EINVAL;
  if (id) *id = mid;
  const uint8_t* kp = payload + 9;  // unaligned sections, copied as they lie
  if (!batchable(s, n) && stage_layout(s, n).total > kSlotKeepBytes) {
    // larger than a ring slot is kept at (never an Akka message: the frame cap is 79 999 records):
    // applied now through the staged copies, so no pinned slot is allocated and released per message.
    // Checked on the host first, so a rejected message applies nothing, as every enqueued one; the
    // ticket is that of everything enqueued so far (complete on return).
    {
      ShardLock lk(s);
      const int rc = reject_if_bad(s, kp, mat ? kp + (size_t)n * 8 : nullptr, n);
      if (rc) return rc;
    }
    const int rc = host_push(s, mat, (const int64_t*)kp, (const int32_t*)(kp + (size_t)n * 8),
                             kp + (size_t)n * (8 + (mat ? 4 : 0)), n, flags);
    ShardLock lk(s);
    if (ticket) *ticket = s->ticket_next;
    return rc;
  }
  // the key check before the lock (it reads only the shard's fixed geometry), as in glint_pull_async
  const bool small = batchable(s, n);
  const i64 bad = small ? host_first_bad(s, kp, mat ? kp + (size_t)n * 8 : nullptr, n) : -1;
  ShardLock lk(s);
  DeviceGuard g(s->device);
  if (int rc = refuse_slab(s)) return rc;
  if (bad >= 0) {
    s->last_bad = bad;
    return GLINT_EOUTOFRANGE;
  }
  if (small)
    return ring_append_locked(s, n, flags, kp, kp + (size_t)n * 8, kp + (size_t)n * (8 + (mat ? 4 : 0)),
                              (u64*)ticket, true);
  int slot = -1;
  int rc = ring_acquire_locked(s, n, &slot);
  if (rc) return rc;
  glint_shard::RingSlot& r = s->ring[slot];
  const StageLayout L = stage_layout(s, n);
  std::memcpy(r.h, kp, (size_t)n * 8);
  if (mat) std::memcpy(r.h + L.kb, kp + (size_t)n * 8, (size_t)n * 4);
  std::memcpy(r.h + L.kb + L.cb, kp + (size_t)n * (8 + (mat ? 4 : 0)), (size_t)n * s->vsize);
  return ring_push_locked(s, slot, n, flags, (u64*)ticket);
}

int glint_shard_wait(glint_shard_t s, uint64_t ticket, int64_t* first_bad) {
  if (!s) return GLINT_EINVAL;
  // Launch the open batch if it holds this ticket, then wait WITHOUT the shard lock, so other
  // threads of the server keep enqueueing meanwhile (one connection per client in the actor
  // model): on the ticket word when the entry carrying the ticket signals it, else on its event.
  bool sig = false;
  hipEvent_t ev = nullptr;
  {
    ShardLock lk(s);
    DeviceGuard g(s->device);
    if (s->open_slot >= 0 && s->ring[s->open_slot].msgs.front().ticket <= ticket) {
      const int rc = ring_flush_locked(s);
      if (rc) return rc;
    }
    const glint_shard::RingSlot* cover = nullptr;  // the newest in-flight entry at or below the ticket
    for (const auto& r : s->ring)
      if (r.inflight && r.ticket_lo <= ticket && (!cover || r.ticket_lo > cover->ticket_lo)) cover = &r;
    if (cover) {
      sig = cover->sig;
      ev = cover->done;
    }
  }
  if (sig) {
    (void)poll_word(s->h_done, ticket, 5000.0);
  } else if (ev) {
    // a DMA'd entry completes by its event; a slot reused meanwhile only re-records it later, so
    // this never returns early (the locked wait below settles the entries either way)
    (void)hipEventSynchronize(ev);
    (void)hipGetLastError();
  }
  ShardLock lk(s);
  DeviceGuard g(s->device);
  return ring_wait_locked(s, (u64)ticket, (i64*)first_bad);
}

int glint_pull_async(glint_shard_t s, int kind, const int64_t* keys, const int32_t* cols, void* out, int64_t n,
                     uint64_t* ticket) {
  if (!s || !ticket || kind < 0 || kind > 2) return GLINT_EINVAL;
  if (n < 0 || (n > 0 && (!keys || !out || (kind == 1 && !cols)))) return GLINT_EINVAL;
  if ((kind == 0) != (s->part.cols == 0)) return GLINT_EINVAL;
  if (n > 0 && pull_bytes(s, kind, n) > kRingAnswerMax) {
    // an answer too large for a ring slot (row pulls of wide matrices): answered now, through the
    // staged copies; the ticket is that of everything enqueued so far (complete on return)
    const int rc = host_pull(s, kind, keys, cols, out, n);
    ShardLock lk(s);
    *ticket = s->ticket_next;
    return rc;
  }
  // the key check reads only the shard's fixed geometry: done before the lock, so the threads
  // enqueueing on one shard hold it only for the copy into the batch
  const i64 bad = n > 0 ? host_first_bad(s, keys, kind == 1 ? cols : nullptr, n) : -1;
  ShardLock lk(s);
  DeviceGuard g(s->device);
  if (int rc = refuse_slab(s)) return rc;
  if (bad >= 0) {
    s->last_bad = bad;
    return GLINT_EOUTOFRANGE;
  }
  if (n == 0) {  // nothing to enqueue: the ticket of everything so far
    *ticket = s->ticket_next;
    return GLINT_OK;
  }
  return pull_enqueue_locked(s, kind, keys, cols, out, n, (u64*)ticket, true);
}

// RequestSerializer.fromBinary for the pull messages + ResponseSerializer.toBinary of the answer
// (ResponseSerializer.scala:43-117; row answers are flattened rows x cols, :52-61).
static int pull_wire(glint_shard_t s, const uint8_t* payload, size_t len, uint8_t* response, size_t cap,
                     size_t* out_len, uint64_t* ticket) {
  if (!s || !payload || len < 5 || !out_len) return GLINT_EINVAL;
  const uint8_t t = payload[0];
  int32_t n = 0;
  std::memcpy(&n, payload + 1, 4);
  if (n < 0) return GLINT_EINVAL;
  int kind;
  size_t want;
  if (t == W_PULL_VECTOR) { kind = 0; want = 5 + (size_t)n * 8; }
  else if (t == W_PULL_MATRIX) { kind = 1; want = 5 + (size_t)n * 12; }
  else if (t == W_PULL_MATRIX_ROWS) { kind = 2; want = 5 + (size_t)n * 8; }
  else return GLINT_EINVAL;
  if (len != want) return GLINT_EINVAL;
  if ((kind == 0) != (s->part.cols == 0)) return GLINT_EINVAL;
  const int64_t count = kind == 2 ? (int64_t)n * s->part.cols : (int64_t)n;
  if (count > INT32_MAX) return GLINT_EINVAL;  // the response header carries an Int count
  const size_t resp = 5 + (size_t)count * s->vsize;
  *out_len = resp;
  if (!response || cap < resp) return GLINT_EINVAL;
  response[0] = wire_response_type(s->dtype);
  const int32_t c32 = (int32_t)count;
  std::memcpy(response + 1, &c32, 4);
  const uint8_t* keys = payload + 5;
  const uint8_t* cols = keys + (size_t)n * 8;
  if (ticket) {
    *ticket = 0;
    return glint_pull_async(s, kind, (const int64_t*)keys, kind == 1 ? (const int32_t*)cols : nullptr,
                            response + 5, n, ticket);
  }
  return host_pull(s, kind, (const int64_t*)keys, kind == 1 ? (const int32_t*)cols : nullptr, response + 5, n);
}

int glint_pull_wire(glint_shard_t s, const uint8_t* payload, size_t len, uint8_t* response, size_t cap,
                    size_t* out_len) {
  return pull_wire(s, payload, len, response, cap, out_len, nullptr);
}

int glint_pull_wire_async(glint_shard_t s, const uint8_t* payload, size_t len, uint8_t* response, size_t cap,
                          size_t* out_len, uint64_t* ticket) {
  if (!ticket) return GLINT_EINVAL;
  return pull_wire(s, payload, len, response, cap, out_len, ticket);
}

int glint_host_alloc(size_t bytes, void** p) {
  if (!p || bytes == 0) return GLINT_EINVAL;
  *p = nullptr;
  char* h = nullptr;
  char* d = nullptr;
  if (hipHostMalloc((void**)&h, bytes, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess ||
      hipHostGetDevicePointer((void**)&d, h, 0) != hipSuccess) {
    (void)hipGetLastError();
    if (h) (void)hipHostFree(h);
    return GLINT_ENOMEM;
  }
  {
    std::lock_guard<std::mutex> lk(g_host_mu);
    const HostRange r{h, bytes, d, std::make_shared<std::atomic<long>>(0)};
    g_host.insert(std::upper_bound(g_host.begin(), g_host.end(), r,
                                   [](const HostRange& a, const HostRange& b) { return a.h < b.h; }),
                  r);
  }
  *p = h;
  return GLINT_OK;
}

int glint_host_free(void* p) {
  if (!p) return GLINT_OK;
  {
    std::lock_guard<std::mutex> lk(g_host_mu);
    auto it = std::find_if(g_host.begin(), g_host.end(), [p](const HostRange& r) { return r.h == (char*)p; });
    if (it == g_host.end()) return GLINT_EINVAL;
    // a pull enqueued to answer into it has not retired: its kernel would write into freed memory
    if (it->pending->load(std::memory_order_acquire) != 0) return GLINT_EINVAL;
    g_host.erase(it);
  }
  return hipHostFree(p) == hipSuccess ? GLINT_OK : GLINT_EDEVICE;
}

}  // extern "C"
