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

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <mutex>
#include <vector>
#include <utility>
#include <new>
#include <cstring>
#include <cstdio>
#include <algorithm>
#include <cstdlib>

namespace glint {

// ------------------------------------------------------------------------------------------------
// small device helpers
// ------------------------------------------------------------------------------------------------
template <typename V> struct Vec2;
template <> struct Vec2<double> { typedef __attribute__((ext_vector_type(2))) double T; };
template <> struct Vec2<float> { typedef __attribute__((ext_vector_type(2))) float T; };
template <> struct Vec2<long long> { typedef __attribute__((ext_vector_type(2))) unsigned long long T; };
template <> struct Vec2<int> { typedef __attribute__((ext_vector_type(2))) unsigned int T; };

typedef __attribute__((ext_vector_type(2))) long long K2;
typedef __attribute__((ext_vector_type(2))) int C2;

// Semiring `+` of spire on JVM primitives: IEEE round-to-nearest for Float/Double, two's-complement
// wrap for Int/Long (PartialVector.scala:39 `data(key) += values(i)`).
__device__ __forceinline__ double vadd(double a, double b) { return a + b; }
__device__ __forceinline__ float vadd(float a, float b) { return a + b; }
__device__ __forceinline__ long long vadd(long long a, long long b) { return (long long)((u64)a + (u64)b); }
__device__ __forceinline__ int vadd(int a, int b) { return (int)((u32)a + (u32)b); }

template <typename V> __device__ __forceinline__ typename Vec2<V>::T as2(V x, V y);
template <> __device__ __forceinline__ Vec2<double>::T as2(double x, double y) { return {x, y}; }
template <> __device__ __forceinline__ Vec2<float>::T as2(float x, float y) { return {x, y}; }
template <> __device__ __forceinline__ Vec2<long long>::T as2(long long x, long long y) { return {(u64)x, (u64)y}; }
template <> __device__ __forceinline__ Vec2<int>::T as2(int x, int y) { return {(u32)x, (u32)y}; }

// device-scope atomic add, no return (global_atomic_add_f64 / _f32 / _x2 / plain)
__device__ __forceinline__ void gadd(double* p, double v) { unsafeAtomicAdd(p, v); }
__device__ __forceinline__ void gadd(float* p, float v) { unsafeAtomicAdd(p, v); }
__device__ __forceinline__ void gadd(long long* p, long long v) { atomicAdd((u64*)p, (u64)v); }
__device__ __forceinline__ void gadd(int* p, int v) { atomicAdd((u32*)p, (u32)v); }

__device__ __forceinline__ u32 ld_relaxed(const u32* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_relaxed(u32* p, u32 v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void record_error(ErrState* e, i64 idx) {
  atomicMax(&e->min_bad_enc, ~(u64)idx);
  atomicAdd(&e->count, 1ull);
}

// address of a record; false when the JVM would throw ArrayIndexOutOfBoundsException
template <bool MAT>
__device__ __forceinline__ bool rec_addr(const PartDesc& p, i64 key, int32_t col, i64& addr) {
  const int32_t l = g2l(p, key);
  bool ok = l >= 0 && l < p.size;
  if (MAT) {
    ok = ok && col >= 0 && col < p.cols;
    addr = (i64)l * p.pitch + (i64)col;
  } else {
    addr = (i64)l;
  }
  return ok;
}

// ------------------------------------------------------------------------------------------------
// push, ordered part: push_check + push_apply
// ------------------------------------------------------------------------------------------------
// addresses are element indices: int32 for vectors (Partition.globalToLocal is an Int), int64 for
// matrices (row * pitch + col)
template <bool MAT> struct AddrT { typedef int32_t T; };
template <> struct AddrT<true> { typedef i64 T; };

template <bool MAT>
__device__ __forceinline__ bool rec_addr_t(const PartDesc& p, i64 key, int32_t col, typename AddrT<MAT>::T& addr) {
  i64 ad;
  const bool ok = rec_addr<MAT>(p, key, col, ad);
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
template <bool MAT, bool FULL>
__device__ __forceinline__ bool check_tile(const i64* __restrict__ keys, const int32_t* __restrict__ cols, i64 n,
                                           const PartDesc& part, LaunchCtl* ctl, i64* __restrict__ desc,
                                           u32 ntiles, u32 t, int lane) {
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
  const u32 brk = __builtin_amdgcn_readfirstlane(ld_relaxed(&ctl->brk_enc));
  if (brk != 0u && ntiles - brk < t) return false;
  A before = 0;
  if (r_first > 0) rec_addr_t<MAT>(part, kb, cb, before);
  bool mono = true, affine = true;
  A a_first = 0;
  A last = before;
#pragma unroll
  for (int j = 0; j < kPPT; ++j) {
    const i64 r = 2 * (pbase + lane + (i64)j * 64);
    const bool h0 = FULL || r < n, h1 = FULL || r + 1 < n;
    A a0, a1;
    const bool o0 = rec_addr_t<MAT>(part, k[j].x, MAT ? c[j].x : 0, a0);
    const bool o1 = rec_addr_t<MAT>(part, k[j].y, MAT ? c[j].y : 0, a1);
    if (j == 0) a_first = __shfl(a0, 0);
    if (h1) mono = mono && (a1 > a0);
    A prev = __shfl_up(a1, 1);
    if (lane == 0) prev = last;
    if (h0 && r > 0) mono = mono && (a0 > prev);
    last = __shfl(a1, 63);
    const A off = (A)(r - r_first);
    affine = affine && (!h0 || (o0 && a0 == a_first + off)) && (!h1 || (o1 && a1 == a_first + off + 1));
  }
  const bool any_bad = __any(!mono);  // wave-wide votes, outside any lane-divergent branch
  const bool all_affine = __all(affine);
  if (lane == 0) {
    if (any_bad) {
      atomicMax(&ctl->brk_enc, ntiles - t);
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

template <bool MAT>
__global__ __launch_bounds__(kTPB) void push_check_kernel(const i64* __restrict__ keys,
                                                          const int32_t* __restrict__ cols, i64 n,
                                                          PartDesc part, LaunchCtl* ctl, i64* __restrict__ desc,
                                                          u32 ntiles) {
  const int lane = threadIdx.x & 63;
  const u32 w0 = blockIdx.x * (kTPB / 64) + (threadIdx.x >> 6);
  const u32 nw = gridDim.x * (kTPB / 64);
  for (u32 t = w0; t < ntiles; t += nw) {
    const bool full = 2 * ((i64)t * (kTile / 2)) + kTile <= n;
    const bool go = full ? check_tile<MAT, true>(keys, cols, n, part, ctl, desc, ntiles, t, lane)
                         : check_tile<MAT, false>(keys, cols, n, part, ctl, desc, ntiles, t, lane);
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
__device__ __forceinline__ void apply_sweep(const PushArgs<V>& a, i64 delta) {
  typedef typename Vec2<V>::T V2;
  if (blockIdx.x >= a.sweep_blocks) return;
  const i64 npairs = a.n >> 1;
  const i64 stride = (i64)a.sweep_blocks * kTPB;
  const V2* vp = reinterpret_cast<const V2*>(a.vals);
  i64 p = (i64)blockIdx.x * kTPB + threadIdx.x;
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
  if ((a.n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const i64 e = a.n - 1 + delta;
    a.data[e] = vadd(a.data[e], a.vals[a.n - 1]);
  }
}

template <typename V, bool MAT>
__global__ __launch_bounds__(kTPB) void push_apply_kernel(PushArgs<V> a, const i64* __restrict__ desc) {
  const u32 brk = a.ctl->brk_enc;  // written by push_check; ordered by the kernel boundary
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.hint)  // for the host's next push: how unordered was this one?
    __hip_atomic_store(a.hint, brk == 0u ? 0ull : (u64)(a.n - (i64)(a.ntiles - brk) * kTile), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  if (brk == 0u && a.ctl->nonaffine == 0u) {
    const i64 delta = desc[0];  // tile 0 starts the run at record 0
    if ((delta & 1) == 0) apply_sweep<V, true>(a, delta);
    else apply_sweep<V, false>(a, delta);
    return;
  }
  const u32 tiles = brk == 0u ? a.ntiles : a.ntiles - brk;
  const int lane = threadIdx.x & 63;
  const u32 w0 = blockIdx.x * (kTPB / 64) + (threadIdx.x >> 6);
  const u32 nw = gridDim.x * (kTPB / 64);
  i64 dbatch = kNotAffine;  // descriptors of this wave's next 64 tiles, one per lane
  for (u32 t = w0, it = 0; t < tiles; t += nw, ++it) {
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
__device__ __forceinline__ void lds_add(double* p, double v) { unsafeAtomicAdd(p, v); }
__device__ __forceinline__ void lds_add(float* p, float v) { unsafeAtomicAdd(p, v); }
__device__ __forceinline__ void lds_add(long long* p, long long v) { atomicAdd((u64*)p, (u64)v); }
__device__ __forceinline__ void lds_add(int* p, int v) { atomicAdd((u32*)p, (u32)v); }

constexpr u64 kEmpty = ~0ull;

// force_all: every record (unaligned caller pointers, no push_check ran); otherwise the records
// from the first non-increasing tile push_check found (none when the push was increasing).
template <typename V, bool MAT>
__global__ __launch_bounds__(kTPB) void push_scatter_kernel(PushArgs<V> a, int force_all) {
  i64 r0 = 0;
  if (!force_all) {
    const u32 brk = a.ctl->brk_enc;  // written by push_check; ordered by the kernel boundary
    if (brk == 0u) return;
    r0 = (i64)(a.ntiles - brk) * kTile;
  }
  if (r0 >= a.n) return;
  const i64 rem = a.n - r0;
  const i64 nchunks = (rem + kScatterChunk - 1) / kScatterChunk;
  if ((i64)blockIdx.x >= nchunks) return;

  __shared__ u64 hk[kHashSlots];
  __shared__ V hv[kHashSlots];
  const int tid = threadIdx.x;
  for (int s = tid; s < kHashSlots; s += kTPB) { hk[s] = kEmpty; hv[s] = V(0); }
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
      lds_add(&hv[h], val);
    }
    __syncthreads();
    for (int s = tid; s < kHashSlots; s += kTPB) {
      const u64 key = hk[s];
      if (key != kEmpty) {
        gadd(a.data + key, hv[s]);
        hk[s] = kEmpty;
        hv[s] = V(0);
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------
// binned push: the unordered tail of a large push, without per-record global atomics
// ------------------------------------------------------------------------------------------------
// Element-granular device atomics run at ~17 G/s here (each lane's add is its own 64-B memory-side
// request). A large unordered tail is instead binned by shard slab -- a rocPRIM radix sort of
// (u32 element address, value) on the address bits above kSlabBits (two 8-bit passes for a 2^28
// shard) -- and each slab's records are summed in LDS (ds_add) and written back with one coalesced
// read-modify-write of the slab's touched element pairs. Slabs with more than kBinItem records are
// split into several work items, which then flush with device atomics, so a hot slab never
// serialises on one workgroup. (A single-pass counting sort into the 32768 slabs measured slower:
// 1.4-2.1 ms for 2^26 records against 1.2 ms here -- its per-record writes scatter over too many
// output segments for L2 to merge.)
constexpr int kSlabBits = 12;
constexpr int kSlab = 1 << kSlabBits;  // elements accumulated in LDS per work item (32 KiB of Double:
                                       // 4 workgroups per CU keep enough item phases overlapping)
constexpr i64 kBinItem = 16384;        // records per apply work item at most
constexpr u32 kBinSentinel = 0xFFFFFFFFu;

// u32 element address of every record from the tail start on (records before it and rejected
// ones: the sentinel); from_break: the tail starts at push_check's break, otherwise at 0
template <bool MAT>
__global__ __launch_bounds__(kTPB) void bin_prepare_kernel(const i64* __restrict__ keys,
                                                           const int32_t* __restrict__ cols, i64 n, PartDesc part,
                                                           const LaunchCtl* ctl, u32 ntiles, int from_break,
                                                           u32* __restrict__ addr, ErrState* err) {
  i64 r0 = 0;
  if (from_break) {
    const u32 brk = ctl->brk_enc;
    r0 = brk == 0u ? n : (i64)(ntiles - brk) * kTile;
  }
  for (i64 i = (i64)blockIdx.x * kTPB + threadIdx.x; i < n; i += (i64)gridDim.x * kTPB) {
    u32 out = kBinSentinel;
    if (i >= r0) {
      i64 ad;
      if (rec_addr<MAT>(part, keys[i], MAT ? cols[i] : 0, ad)) out = (u32)ad;
      else record_error(err, i);
    }
    addr[i] = out;
  }
}

// Duplicate-heavy tails: each workgroup first sums its chunk's records per element in an LDS hash
// table and emits one (address, sum) per distinct element, so the sort and the apply see only
// those. Output order is arbitrary (the default mode's contract); the count goes to *m_out.
constexpr int kDedupSlots = 4096;   // u32 keys + V sums: 48 KiB for Double
constexpr int kDedupChunk = 2048;   // records per table fill (load factor <= 0.5)
template <typename V, bool MAT>
__global__ __launch_bounds__(kTPB) void bin_dedup_kernel(const i64* __restrict__ keys, const int32_t* __restrict__ cols,
                                                         const V* __restrict__ vals, i64 n, PartDesc part,
                                                         const LaunchCtl* ctl, u32 ntiles, int from_break,
                                                         u32* __restrict__ addr_out, V* __restrict__ val_out,
                                                         u32* __restrict__ m_out, ErrState* err) {
  __shared__ u32 hk[kDedupSlots];
  __shared__ V hv[kDedupSlots];
  __shared__ u32 wsum[kTPB / 64];
  __shared__ u32 obase;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  i64 r0 = 0;
  if (from_break) {
    const u32 brk = ctl->brk_enc;
    r0 = brk == 0u ? n : (i64)(ntiles - brk) * kTile;
  }
  if (blockIdx.x == 0 && tid == 0) m_out[1] = (u32)(n - r0);  // the tail size, for the host's ratio
  for (int sl = tid; sl < kDedupSlots; sl += kTPB) { hk[sl] = kBinSentinel; hv[sl] = V(0); }
  __syncthreads();
  const i64 nchunks = (n - r0 + kDedupChunk - 1) / kDedupChunk;
  for (i64 ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const i64 c0 = r0 + ch * kDedupChunk, c1 = min(n, c0 + kDedupChunk);
    constexpr int kPer = kDedupChunk / kTPB;
    i64 k[kPer];
    int32_t cl[kPer];
    V v[kPer];
#pragma unroll
    for (int q = 0; q < kPer; ++q) {  // clamped, branch-free loads
      const i64 i = c0 + q * kTPB + tid;
      const i64 ii = i < c1 ? i : c1 - 1;
      k[q] = keys[ii];
      cl[q] = MAT ? cols[ii] : 0;
      v[q] = vals[ii];
    }
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const i64 i = c0 + q * kTPB + tid;
      if (i >= c1) continue;
      i64 ad64;
      if (!rec_addr<MAT>(part, k[q], cl[q], ad64)) { record_error(err, i); continue; }
      const u32 ad = (u32)ad64;
      u32 h = (ad * 0x9E3779B1u) >> (32 - 12);
      for (;;) {
        const u32 cur = hk[h];
        if (cur == ad) break;
        if (cur == kBinSentinel) {
          const u32 prev = atomicCAS(&hk[h], kBinSentinel, ad);
          if (prev == kBinSentinel || prev == ad) break;
        }
        h = (h + 1) & (kDedupSlots - 1);
      }
      lds_add(&hv[h], v[q]);
    }
    __syncthreads();
    // compact: count this thread's occupied slots, scan across the block, reserve, write
    constexpr int kSlotsPer = kDedupSlots / kTPB;
    u32 cnt = 0;
#pragma unroll
    for (int q = 0; q < kSlotsPer; ++q) cnt += hk[tid * kSlotsPer + q] != kBinSentinel;
    u32 incl = cnt;  // wave-inclusive scan
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const u32 y = __shfl_up(incl, d);
      if (lane >= d) incl += y;
    }
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    if (tid == 0) {
      u32 t = 0;
      for (int w = 0; w < kTPB / 64; ++w) { const u32 x = wsum[w]; wsum[w] = t; t += x; }
      obase = atomicAdd(m_out, t);
    }
    __syncthreads();
    u32 pos = obase + wsum[wid] + incl - cnt;
#pragma unroll
    for (int q = 0; q < kSlotsPer; ++q) {
      const int sl = tid * kSlotsPer + q;
      const u32 key = hk[sl];
      if (key != kBinSentinel) {
        addr_out[pos] = key;
        val_out[pos] = hv[sl];
        ++pos;
        hk[sl] = kBinSentinel;
        hv[sl] = V(0);
      }
    }
    __syncthreads();
  }
}

__device__ __forceinline__ u32 slab_of(u32 a, u32 mask) { return (a >> kSlabBits) & mask; }

// per slab s < nslabs: start[s] = first sorted record of slab s (the sort orders by slab_of, so the
// sentinels share the all-ones slab with its real records), items[s] = its apply work items;
// start[nslabs] = n, items[nslabs] = 0 (an exclusive scan of items then ends in the total)
__global__ void bin_bounds_kernel(const u32* __restrict__ addr, i64 n, u32 nslabs, u32 mask, u32* __restrict__ start,
                                  u32* __restrict__ items) {
  for (i64 s = (i64)blockIdx.x * blockDim.x + threadIdx.x; s <= (i64)nslabs; s += (i64)gridDim.x * blockDim.x) {
    i64 lo = 0, hi = n;  // first record with slab_of >= s
    while (lo < hi) {
      const i64 mid = (lo + hi) >> 1;
      if (slab_of(addr[mid], mask) < (u32)s) lo = mid + 1;
      else hi = mid;
    }
    start[s] = (u32)lo;
    if (s == (i64)nslabs) {
      items[s] = 0u;
    } else {
      i64 lo2 = lo, hi2 = n;  // first record with slab_of > s
      while (lo2 < hi2) {
        const i64 mid = (lo2 + hi2) >> 1;
        if (slab_of(addr[mid], mask) <= (u32)s) lo2 = mid + 1;
        else hi2 = mid;
      }
      items[s] = (u32)((lo2 - lo + kBinItem - 1) / kBinItem);
    }
  }
}

// One descriptor per apply work item {slab, first record, end record, exclusive}: an apply
// workgroup finds its work with one 16-B load instead of a search
__global__ void bin_item_map_kernel(const u32* __restrict__ start, const u32* __restrict__ items,
                                    const u32* __restrict__ item_off, u32 nslabs, uint4* __restrict__ item_desc) {
  for (u32 s = blockIdx.x * blockDim.x + threadIdx.x; s < nslabs; s += gridDim.x * blockDim.x) {
    const u32 o = item_off[s], m = items[s], r0 = start[s], r1 = start[s + 1];
    for (u32 k = 0; k < m; ++k) {
      const u32 lo = r0 + k * (u32)kBinItem;
      item_desc[o + k] = make_uint4(s, lo, min(r1, lo + (u32)kBinItem), m == 1u ? 1u : 0u);
    }
  }
}

constexpr int kBinTPB = 256;  // 4 waves share one LDS slab
constexpr int kBinRB = 4;     // records per thread per batch: loads issue together, then the LDS adds

// One work item = up to kBinItem records of one slab
template <typename V>
__global__ __launch_bounds__(kBinTPB) void bin_apply_kernel(const u32* __restrict__ addr, const V* __restrict__ val,
                                                            const uint4* __restrict__ item_desc,
                                                            const u32* __restrict__ item_off, u32 nslabs,
                                                            i64 elems, V* __restrict__ data) {
  typedef typename Vec2<V>::T V2;
  __shared__ V acc[kSlab];
  __shared__ uint8_t touched[kSlab];  // plain byte stores: no atomic serialisation on hot elements
  constexpr int kPairsPerThread = kSlab / 2 / kBinTPB;
  const int tid = threadIdx.x;
  const u32 total = item_off[nslabs];
  for (u32 it = blockIdx.x; it < total; it += gridDim.x) {
    const uint4 d4 = item_desc[it];
    const u32 slab = d4.x;
    const bool exclusive = d4.w != 0u;
    const i64 r_lo = d4.y, r_hi = d4.z;
    const i64 sbase_g = (i64)slab << kSlabBits;
    for (int e = tid; e < kSlab; e += kBinTPB) acc[e] = V(0);
    for (int w = tid; w < kSlab / 16; w += kBinTPB) reinterpret_cast<uint4*>(touched)[w] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    for (i64 j0 = r_lo; j0 < r_hi; j0 += (i64)kBinTPB * kBinRB) {
      u32 ad[kBinRB];
      V v[kBinRB];
#pragma unroll
      for (int q = 0; q < kBinRB; ++q) {  // clamped, branch-free loads
        const i64 j = j0 + q * kBinTPB + tid;
        const i64 jj = j < r_hi ? j : r_hi - 1;
        ad[q] = addr[jj];
        v[q] = val[jj];
        if (j >= r_hi) ad[q] = kBinSentinel;
      }
#pragma unroll
      for (int q = 0; q < kBinRB; ++q) {
        if (ad[q] == kBinSentinel) continue;
        const u32 e = ad[q] & (kSlab - 1);
        lds_add(&acc[e], v[q]);
        touched[e] = 1;
      }
    }
    __syncthreads();
    V* const sbase = data + sbase_g;
    if (exclusive) {
      // one coalesced RMW of the touched pairs; untouched lanes load the slab's first pair
      // instead (one cached line), so all loads issue back to back without a branch
      V2 d[kPairsPerThread];
      u32 t[kPairsPerThread];
#pragma unroll
      for (int q = 0; q < kPairsPerThread; ++q) {
        const int e0 = 2 * (tid + q * kBinTPB);
        t[q] = (u32)touched[e0] | ((u32)touched[e0 + 1] << 1);
        const bool vec = t[q] != 0u && sbase_g + e0 + 1 < elems;
        d[q] = *reinterpret_cast<const V2*>(vec ? sbase + e0 : sbase);
      }
#pragma unroll
      for (int q = 0; q < kPairsPerThread; ++q) {
        if (t[q] == 0u) continue;
        const int e0 = 2 * (tid + q * kBinTPB);
        if (sbase_g + e0 + 1 < elems) {
          V2 r = d[q];
          if (t[q] & 1u) r.x = vadd(r.x, acc[e0]);
          if (t[q] & 2u) r.y = vadd(r.y, acc[e0 + 1]);
          *reinterpret_cast<V2*>(sbase + e0) = r;
        } else {  // the shard's last element, odd count
          sbase[e0] = vadd(sbase[e0], acc[e0]);
        }
      }
    } else {
      for (int e = tid; e < kSlab; e += kBinTPB)
        if (touched[e]) gadd(sbase + e, acc[e]);
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------
// deterministic tail: stable sort by address, then an in-order fold per address starting from the
// shard's current value -- the reference's sequential `+=` order, bit for bit
// ------------------------------------------------------------------------------------------------
template <typename V, bool MAT>
__global__ __launch_bounds__(kTPB) void det_prepare_kernel(const i64* keys, const int32_t* cols, const V* vals, i64 r0,
                                                           i64 m, PartDesc part, u64 sentinel, u64* addr, V* val,
                                                           ErrState* err) {
  for (i64 i = (i64)blockIdx.x * kTPB + threadIdx.x; i < m; i += (i64)gridDim.x * kTPB) {
    i64 ad;
    const bool ok = rec_addr<MAT>(part, keys[r0 + i], MAT ? cols[r0 + i] : 0, ad);
    if (!ok) record_error(err, r0 + i);
    addr[i] = ok ? (u64)ad : sentinel;
    val[i] = vals[r0 + i];
  }
}

// After the stable sort by address, each run of equal addresses holds that element's values in
// push order. A run is folded into the shard strictly left to right, starting from the shard's
// current value -- the reference's `data(k) += v` sequence, rounding for rounding.
constexpr int kDetShort = 64;  // runs up to this length: one thread; longer: one wave

template <typename V>
__global__ __launch_bounds__(kTPB) void det_fold_short_kernel(const u64* addr, const V* val, i64 m, u64 sentinel,
                                                              V* data, u32* long_count, u32* long_list) {
  for (i64 i = (i64)blockIdx.x * kTPB + threadIdx.x; i < m; i += (i64)gridDim.x * kTPB) {
    const u64 ad = addr[i];
    if (ad == sentinel) continue;
    if (i > 0 && addr[i - 1] == ad) continue;  // not the head of its run
    i64 j = i;
    while (j < m && j - i < kDetShort && addr[j] == ad) ++j;
    if (j < m && j - i == kDetShort && addr[j] == ad) {  // a long run: leave it to a whole wave
      long_list[atomicAdd(long_count, 1u)] = (u32)i;
      continue;
    }
    V acc = data[ad];
    for (i64 q = i; q < j; ++q) acc = vadd(acc, val[q]);
    data[ad] = acc;
  }
}

// value of lane l (wave-uniform l) through v_readlane -> SGPR: no LDS round trip per element
__device__ __forceinline__ double lane_value(double x, int l) {
  const u64 b = __double_as_longlong(x);
  const u32 lo = __builtin_amdgcn_readlane((u32)b, l), hi = __builtin_amdgcn_readlane((u32)(b >> 32), l);
  return __longlong_as_double((long long)(((u64)hi << 32) | lo));
}
__device__ __forceinline__ float lane_value(float x, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l));
}
__device__ __forceinline__ long long lane_value(long long x, int l) {
  const u64 b = (u64)x;
  return (long long)(((u64)__builtin_amdgcn_readlane((u32)(b >> 32), l) << 32) | __builtin_amdgcn_readlane((u32)b, l));
}
__device__ __forceinline__ int lane_value(int x, int l) { return __builtin_amdgcn_readlane(x, l); }

// End (exclusive) of the run of `ad` that starts at i in the sorted addresses: a 64-way gallop,
// then 64-way refinement -- O(log64 len) dependent probe rounds instead of a compare per element.
__device__ __forceinline__ i64 run_end(const u64* addr, i64 m, i64 i, u64 ad, int lane) {
  i64 lo = i, hi;  // addr[lo] == ad; the end lies in (lo, hi]
  for (i64 step = 1;; step *= 64) {
    const i64 p = lo + (i64)(lane + 1) * step;
    const int c = __popcll(__ballot(p < m && addr[p] == ad));  // equal probes form a prefix
    if (c < 64) {
      hi = lo + (i64)(c + 1) * step;
      lo += (i64)c * step;
      break;
    }
    lo += 64 * step;
  }
  if (hi > m) hi = m;
  while (hi - lo > 1) {
    const i64 step = (hi - lo + 63) / 64;
    const i64 p = lo + (i64)(lane + 1) * step;
    const int c = __popcll(__ballot(p < hi && addr[p] == ad));
    const i64 nh = lo + (i64)(c + 1) * step;
    lo += (i64)c * step;
    if (nh < hi) hi = nh;
  }
  return lo + 1;
}

// One wave per long run. The fold is one strictly sequential chain of adds, so its speed is the
// dependent v_add latency: the values are loaded *transposed* -- lane L holds kDetK consecutive
// values of the run in VGPRs -- and lane L alone (exec = one lane) folds them into the running sum
// with register operands, then hands the sum to lane L+1 (v_readlane). Two buffers alternate so
// the next 64 x kDetK values are in flight while the current ones are folded. Padding is -0.0, the
// exact identity of IEEE addition (x + -0.0 == x for every x, signed zeros included).
constexpr int kDetK = 32;
template <typename V>
__device__ __forceinline__ void det_load(V (&x)[kDetK], const V* val, i64 start, i64 e, int lane) {
  const i64 q0 = start + (i64)lane * kDetK;
#pragma unroll
  for (int j = 0; j < kDetK; ++j) {
    const i64 q = q0 + j;
    const V v = val[q < e ? q : e - 1];  // clamped, branch-free: all loads issue back to back
    x[j] = q < e ? v : V(-0.0);
  }
}
template <typename V>
__device__ __forceinline__ V det_fold(const V (&x)[kDetK], V acc, i64 start, i64 e, int lane) {
  if (start >= e) return acc;
  const i64 left = e - start;
  const int nl = left >= 64 * kDetK ? 64 : (int)((left + kDetK - 1) / kDetK);
  for (int L = 0; L < nl; ++L) {
    if (lane == L) {
#pragma unroll
      for (int j = 0; j < kDetK; ++j) acc = vadd(acc, x[j]);
    }
    acc = lane_value(acc, L);
  }
  return acc;
}

template <typename V>
__global__ __launch_bounds__(kTPB) void det_fold_long_kernel(const u64* addr, const V* val, i64 m,
                                                             const u32* long_count, const u32* long_list, V* data) {
  const int lane = threadIdx.x & 63;
  const u32 w0 = blockIdx.x * (kTPB / 64) + (threadIdx.x >> 6);
  const u32 nw = gridDim.x * (kTPB / 64);
  const u32 cnt = *long_count;
  constexpr i64 kB = 64 * kDetK;
  for (u32 w = w0; w < cnt; w += nw) {
    const i64 i = long_list[w];
    const u64 ad = addr[i];
    const i64 e = run_end(addr, m, i, ad, lane);
    V acc = data[ad];
    V A[kDetK], B[kDetK];
    det_load(A, val, i, e, lane);
    for (i64 base = i; base < e; base += 2 * kB) {
      det_load(B, val, base + kB, e, lane);
      acc = det_fold(A, acc, base, e, lane);
      det_load(A, val, base + 2 * kB, e, lane);
      acc = det_fold(B, acc, base + kB, e, lane);
    }
    if (lane == 0) data[ad] = acc;
  }
}

// ------------------------------------------------------------------------------------------------
// pulls
// ------------------------------------------------------------------------------------------------
// PartialVector.get (PartialVector.scala:51-60): out[i] = data(globalToLocal(keys(i)))
template <typename V, bool PAIRS>
__global__ __launch_bounds__(kTPB) void vec_pull_kernel(const i64* keys, i64 n, const V* data, PartDesc part,
                                                        V* out, ErrState* err) {
  typedef typename Vec2<V>::T V2;
  const i64 stride = (i64)gridDim.x * kTPB;
  if (PAIRS) {
    const i64 npairs = (n + 1) >> 1;
    for (i64 p = (i64)blockIdx.x * kTPB + threadIdx.x; p < npairs; p += stride) {
      const i64 r = 2 * p;
      if (r + 1 < n) {
        const K2 k = __builtin_nontemporal_load(reinterpret_cast<const K2*>(keys) + p);
        i64 l0, l1;
        const bool o0 = rec_addr<false>(part, k.x, 0, l0);
        const bool o1 = rec_addr<false>(part, k.y, 0, l1);
        V2 o;
        if (o0 && o1 && l1 == l0 + 1 && (l0 & 1) == 0) {
          // adjacent pair: a streamed (dense) pull -- non-temporal, like the push sweep
          o = __builtin_nontemporal_load(reinterpret_cast<const V2*>(data + l0));
        } else {
          if (!o0) record_error(err, r);
          if (!o1) record_error(err, r + 1);
          o = as2<V>(o0 ? data[l0] : V(0), o1 ? data[l1] : V(0));
        }
        __builtin_nontemporal_store(o, reinterpret_cast<V2*>(out + r));
      } else {
        i64 l0;
        const bool o0 = rec_addr<false>(part, keys[r], 0, l0);
        if (!o0) record_error(err, r);
        out[r] = o0 ? data[l0] : V(0);
      }
    }
  } else {
    for (i64 i = (i64)blockIdx.x * kTPB + threadIdx.x; i < n; i += stride) {
      i64 l;
      const bool o = rec_addr<false>(part, keys[i], 0, l);
      if (!o) record_error(err, i);
      out[i] = o ? data[l] : V(0);
    }
  }
}

// PartialMatrix.get (PartialMatrix.scala:55-65)
template <typename V>
__global__ __launch_bounds__(kTPB) void mat_pull_kernel(const i64* rows, const int32_t* cols, i64 n, const V* data,
                                                        PartDesc part, V* out, ErrState* err) {
  for (i64 i = (i64)blockIdx.x * kTPB + threadIdx.x; i < n; i += (i64)gridDim.x * kTPB) {
    i64 ad;
    const bool o = rec_addr<true>(part, rows[i], cols[i], ad);
    if (!o) record_error(err, i);
    out[i] = o ? data[ad] : V(0);
  }
}

// PartialMatrix.getRows (PartialMatrix.scala:37-46) + the row flattening of ResponseSerializer
// (ResponseSerializer.scala:52-61): one wave per requested row, 16 B per lane when rows allow.
template <typename V, bool VEC16>
__global__ __launch_bounds__(kTPB) void mat_pull_rows_kernel(const i64* rows, i64 n, const V* data, PartDesc part,
                                                             V* out, ErrState* err) {
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
}

}  // namespace glint

// ================================================================================================
// host side
// ================================================================================================
using namespace glint;

struct glint_shard {
  int device = 0;
  int dtype = 0;
  size_t vsize = 0;
  PartDesc part{};
  i64 elems = 0;  // allocated elements (size * pitch for matrices)
  void* data = nullptr;
  hipStream_t stream = nullptr;
  int cus = 256;
  // per-launch control words (LaunchCtl), zeroed before each ordered push
  void* d_ctl = nullptr;
  size_t ctl_bytes = 0;
  ErrState* d_err = nullptr;
  // grow-only device scratch for host-pointer calls and the deterministic path
  void* d_scratch = nullptr;
  size_t scratch_bytes = 0;
  void* d_det = nullptr;
  size_t det_bytes = 0;
  void* d_bin = nullptr;  // binned-push scratch
  size_t bin_bytes = 0;
  double bin_dedup_ratio = 0.0;  // distinct/records of the last deduplicating binned push
  uint32_t bin_pushes = 0;
  u64* h_hint = nullptr;  // host-mapped: unordered-tail size of the last push (written by push_apply)
  u64* d_hint = nullptr;
  i64 last_bad = -1;
  // kernel timing (glint_prof_*): HIP event pairs recorded on the launch stream, summed lazily
  bool prof = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_ev[GLINT_K_COUNT];
  double prof_ms[GLINT_K_COUNT] = {0};
  int64_t prof_n[GLINT_K_COUNT] = {0};
  std::mutex mu;
};

namespace {

struct DeviceGuard {
  int prev = -1;
  bool ok = false;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

#define HIPCHK(x)                                   \
  do {                                              \
    hipError_t e_ = (x);                            \
    if (e_ != hipSuccess) {                         \
      (void)hipGetLastError();                      \
      return GLINT_EDEVICE;                         \
    }                                               \
  } while (0)

size_t dtype_size(int dt) { return (dt == GLINT_I32 || dt == GLINT_F32) ? 4 : 8; }
size_t pad256(size_t b) { return (b + 255) & ~(size_t)255; }
bool aligned(const void* p, size_t a) { return ((uintptr_t)p % a) == 0; }

int grow(void** buf, size_t* cap, size_t need) {
  if (*cap >= need) return GLINT_OK;
  if (*buf) (void)hipFree(*buf);
  *buf = nullptr;
  *cap = 0;
  size_t sz = std::max(need, (size_t)1 << 20);
  if (hipMalloc(buf, sz) != hipSuccess) {
    (void)hipGetLastError();
    *buf = nullptr;
    return GLINT_ENOMEM;
  }
  *cap = sz;
  return GLINT_OK;
}

// device-resident calls run on the caller's stream exactly as given (NULL = the HIP null stream,
// as in every HIP API), so they order with the caller's producers and consumers of the buffers
hipStream_t pick(glint_shard*, void* stream) { return (hipStream_t)stream; }

// Brackets one kernel launch with events on its stream when profiling is on.
struct ProfScope {
  glint_shard* s;
  int id;
  hipStream_t st;
  hipEvent_t b = nullptr, e = nullptr;
  ProfScope(glint_shard* s_, int id_, hipStream_t st_) : s(s_), id(id_), st(st_) {
    if (!s->prof) return;
    if (hipEventCreate(&b) != hipSuccess || hipEventCreate(&e) != hipSuccess) {
      (void)hipGetLastError();
      b = e = nullptr;
      return;
    }
    (void)hipEventRecord(b, st);
  }
  ~ProfScope() {
    if (!b) return;
    (void)hipEventRecord(e, st);
    s->prof_ev[id].emplace_back(b, e);
  }
};

void prof_drain(glint_shard* s) {
  for (int k = 0; k < GLINT_K_COUNT; ++k) {
    for (auto& pr : s->prof_ev[k]) {
      float ms = 0.f;
      if (hipEventSynchronize(pr.second) == hipSuccess && hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) {
        s->prof_ms[k] += ms;
        s->prof_n[k] += 1;
      }
      (void)hipEventDestroy(pr.first);
      (void)hipEventDestroy(pr.second);
    }
    s->prof_ev[k].clear();
  }
  (void)hipGetLastError();
}

unsigned grid_for(i64 units, i64 per_block, i64 cap) {
  i64 g = (units + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// resident blocks per CU for a kernel (occupancy query), capped at the measured best; the
// environment variable `knob` (e.g. GLINT_CHECK_BPC) overrides it for tuning sweeps
template <typename K>
int blocks_per_cu(K kernel, int cap, const char* knob = nullptr) {
  int b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kernel, kTPB, 0) != hipSuccess || b < 1) {
    (void)hipGetLastError();
    b = 2;
  }
  b = std::min(b, cap);
  const char* env = knob ? getenv(knob) : nullptr;
  if (env && atoi(env) > 0) b = atoi(env);
  return b;
}

// ---- push -------------------------------------------------------------------------------------
template <typename V, bool MAT>
int push_det_tail(glint_shard* s, const PushArgs<V>& a, bool from_break, hipStream_t st) {
  // where does the non-increasing tail start? (a host round trip: this is the strict-order path)
  i64 r0 = 0;
  if (from_break) {
    LaunchCtl h{};
    HIPCHK(hipMemcpyAsync(&h, s->d_ctl, sizeof(h), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (h.brk_enc == 0u) return GLINT_OK;
    r0 = (i64)(a.ntiles - h.brk_enc) * kTile;
  }
  if (r0 >= a.n) return GLINT_OK;
  const i64 m = a.n - r0;
  const u64 sentinel = (u64)s->elems;
  int end_bit = 1;
  while (end_bit < 64 && ((u64)1 << end_bit) <= sentinel) ++end_bit;
  size_t tmp_bytes = 0;
  u64* nul64 = nullptr;
  V* nulv = nullptr;
  HIPCHK(rocprim::radix_sort_pairs(nullptr, tmp_bytes, nul64, nul64, nulv, nulv, (size_t)m, 0, end_bit, st));
  const size_t b_addr = pad256((size_t)m * 8), b_val = pad256((size_t)m * sizeof(V));
  const size_t b_list = pad256(((size_t)m / kDetShort + 2) * 4);
  const size_t need = 2 * b_addr + 2 * b_val + b_list + pad256(tmp_bytes);
  int rc = grow(&s->d_det, &s->det_bytes, need);
  if (rc) return rc;
  char* base = (char*)s->d_det;
  u64* addr_in = (u64*)base;
  u64* addr_out = (u64*)(base + b_addr);
  V* val_in = (V*)(base + 2 * b_addr);
  V* val_out = (V*)(base + 2 * b_addr + b_val);
  u32* long_count = (u32*)(base + 2 * b_addr + 2 * b_val);
  u32* long_list = long_count + 1;
  void* tmp = base + 2 * b_addr + 2 * b_val + b_list;
  const unsigned g = grid_for(m, kTPB, (i64)s->cus * 8);
  det_prepare_kernel<V, MAT><<<g, kTPB, 0, st>>>(a.keys, a.cols, a.vals, r0, m, a.part, sentinel, addr_in, val_in,
                                                 a.err);
  HIPCHK(hipGetLastError());
  // stable LSD radix sort: equal addresses keep their push order
  HIPCHK(rocprim::radix_sort_pairs(tmp, tmp_bytes, addr_in, addr_out, val_in, val_out, (size_t)m, 0, end_bit, st));
  HIPCHK(hipMemsetAsync(long_count, 0, 4, st));
  det_fold_short_kernel<V><<<g, kTPB, 0, st>>>(addr_out, val_out, m, sentinel, a.data, long_count, long_list);
  HIPCHK(hipGetLastError());
  det_fold_long_kernel<V><<<(unsigned)s->cus * 2, kTPB, 0, st>>>(addr_out, val_out, m, long_count, long_list, a.data);
  HIPCHK(hipGetLastError());
  return GLINT_OK;
}

// The binned tail pipeline over the whole push (records before push_check's break are masked on
// the device, so no host round trip is needed): prepare -> radix sort by slab -> slab bounds ->
// item scan -> item map -> LDS slab apply.
template <typename V, bool MAT>
int push_binned(glint_shard* s, const PushArgs<V>& a, bool from_break, hipStream_t st) {
  const i64 n = a.n;
  if (n >= ((i64)1 << 32) || s->elems >= ((i64)1 << 32) - 1) return GLINT_EINVAL;  // u32 addresses
  int end_bit = kSlabBits + 1;
  while (end_bit < 32 && ((i64)1 << end_bit) < s->elems) ++end_bit;
  const u32 nslabs = 1u << (end_bit - kSlabBits);
  const u32 mask = nslabs - 1u;
  // dedup when the last probe found < 60 % distinct records per chunk; re-probe every 16 pushes
  const bool dedup = s->bin_dedup_ratio < 0.6 || (++s->bin_pushes & 15) == 0;
  size_t sort_bytes = 0, scan_bytes = 0;
  HIPCHK(rocprim::radix_sort_pairs(nullptr, sort_bytes, (u32*)nullptr, (u32*)nullptr, (const V*)nullptr, (V*)nullptr,
                                   (size_t)n, kSlabBits, end_bit, st));
  HIPCHK(rocprim::exclusive_scan(nullptr, scan_bytes, (u32*)nullptr, (u32*)nullptr, 0u, (size_t)nslabs + 1,
                                 rocprim::plus<u32>(), st));
  const i64 max_items = (i64)nslabs + (n + kBinItem - 1) / kBinItem;
  const size_t b_a = pad256((size_t)n * 4), b_v = pad256((size_t)n * sizeof(V));
  const size_t b_s = pad256(((size_t)nslabs + 1) * 4), b_m = pad256((size_t)max_items * 16);
  const size_t need = 2 * b_a + 2 * b_v + 3 * b_s + b_m + 256 + pad256(sort_bytes) + pad256(scan_bytes);
  int rc = grow(&s->d_bin, &s->bin_bytes, need);
  if (rc) return rc;
  char* p = (char*)s->d_bin;
  u32* addr_in = (u32*)p;
  u32* addr_out = (u32*)(p + b_a);
  V* val_in = (V*)(p + 2 * b_a);
  V* val_out = (V*)(p + 2 * b_a + b_v);
  u32* start = (u32*)(p + 2 * b_a + 2 * b_v);
  u32* items = (u32*)(p + 2 * b_a + 2 * b_v + b_s);
  u32* item_off = (u32*)(p + 2 * b_a + 2 * b_v + 2 * b_s);
  uint4* item_desc = (uint4*)(p + 2 * b_a + 2 * b_v + 3 * b_s);
  u32* m_dev = (u32*)(p + 2 * b_a + 2 * b_v + 3 * b_s + b_m);
  void* sort_tmp = p + 2 * b_a + 2 * b_v + 3 * b_s + b_m + 256;
  void* scan_tmp = (char*)sort_tmp + pad256(sort_bytes);
  const unsigned gs = grid_for((i64)nslabs + 1, 256, 8192);
  ProfScope ps(s, GLINT_K_PUSH_BINNED, st);
  i64 m = n;
  const V* sort_vals = a.vals;
  if (dedup) {
    HIPCHK(hipMemsetAsync(m_dev, 0, 8, st));
    bin_dedup_kernel<V, MAT><<<grid_for(n, kDedupChunk, (i64)s->cus * 3), kTPB, 0, st>>>(
        a.keys, a.cols, a.vals, n, a.part, a.ctl, a.ntiles, from_break ? 1 : 0, addr_in, val_in, m_dev, a.err);
    HIPCHK(hipGetLastError());
    u32 mh[2] = {0, 0};  // the sort needs its size on the host: one round trip, only on this path
    HIPCHK(hipMemcpyAsync(mh, m_dev, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    m = mh[0];
    sort_vals = val_in;
    if (mh[1] > 0) s->bin_dedup_ratio = (double)mh[0] / (double)mh[1];
    if (m == 0) return GLINT_OK;
  } else {
    bin_prepare_kernel<MAT><<<grid_for(n, kTPB, (i64)s->cus * 8), kTPB, 0, st>>>(
        a.keys, a.cols, n, a.part, a.ctl, a.ntiles, from_break ? 1 : 0, addr_in, a.err);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(rocprim::radix_sort_pairs(sort_tmp, sort_bytes, addr_in, addr_out, sort_vals, val_out, (size_t)m, kSlabBits,
                                   end_bit, st));
  bin_bounds_kernel<<<gs, 256, 0, st>>>(addr_out, m, nslabs, mask, start, items);
  HIPCHK(hipGetLastError());
  HIPCHK(rocprim::exclusive_scan(scan_tmp, scan_bytes, items, item_off, 0u, (size_t)nslabs + 1, rocprim::plus<u32>(),
                                 st));
  bin_item_map_kernel<<<gs, 256, 0, st>>>(start, items, item_off, nslabs, item_desc);
  HIPCHK(hipGetLastError());
  const i64 mi = (i64)nslabs + (m + kBinItem - 1) / kBinItem;
  bin_apply_kernel<V><<<(unsigned)std::min<i64>(mi, (i64)s->cus * 8), kBinTPB, 0, st>>>(
      addr_out, val_out, item_desc, item_off, nslabs, s->elems, a.data);
  HIPCHK(hipGetLastError());
  return GLINT_OK;
}

// blocks per CU in the affine sweep (GLINT_SWEEP_BPC overrides; 1 measured best on MI355X)
int sweep_blocks_per_cu() {
  static const int v = [] {
    const char* e = getenv("GLINT_SWEEP_BPC");
    return (e && atoi(e) > 0) ? atoi(e) : 1;
  }();
  return v;
}

// GLINT_BINNED: 0 = never bin, 1 = bin every large push, unset = bin when the previous push on the
// shard left a large unordered tail (read from the host-mapped word push_apply writes)
int binned_mode() {
  const char* e = getenv("GLINT_BINNED");
  if (!e || !*e) return -1;
  return atoi(e) != 0 ? 1 : 0;
}
constexpr i64 kBinMin = (i64)1 << 20;  // records: below this the LDS-hash scatter wins

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
  a.err = s->d_err;
  a.elems = s->elems;
  a.hint = s->d_hint;
  a.sweep_blocks = 0;
  const i64 ntiles = (n + kTile - 1) / kTile;
  if (ntiles >= (i64)0xFFFFFFF0ll) return GLINT_EINVAL;
  a.ntiles = (u32)ntiles;
  const bool vec_ok = aligned(keys, 16) && aligned(vals, 2 * sizeof(V)) && (!MAT || aligned(cols, 8));
  const bool det = (flags & GLINT_PUSH_DETERMINISTIC) && (s->dtype == GLINT_F32 || s->dtype == GLINT_F64);
  // control region: [LaunchCtl | pad to 256][tile descriptors i64 x ntiles]
  const size_t ctl_need = 256 + (size_t)ntiles * sizeof(i64);
  int rc = grow(&s->d_ctl, &s->ctl_bytes, ctl_need);
  if (rc) return rc;
  a.ctl = (LaunchCtl*)s->d_ctl;
  i64* desc = (i64*)((char*)s->d_ctl + 256);

  const int bmode = binned_mode();
  const bool unordered = (flags & GLINT_PUSH_UNORDERED) != 0;
  const i64 last_tail = s->h_hint ? (i64)__atomic_load_n(s->h_hint, __ATOMIC_RELAXED) : 0;
  const bool binned = !det && vec_ok && n < ((i64)1 << 32) && s->elems < ((i64)1 << 32) - 1 && bmode != 0 &&
                      (unordered || (n >= kBinMin && (bmode == 1 || last_tail >= kBinMin)));
  if (binned && unordered) return push_binned<V, MAT>(s, a, false, st);
  if (!vec_ok) {  // unaligned caller pointers: the scalar-load scatter for everything
    if (det) return push_det_tail<V, MAT>(s, a, false, st);
    const unsigned g2 = grid_for(n, kScatterChunk, (i64)s->cus * 2);
    ProfScope ps(s, GLINT_K_PUSH_SCATTER, st);
    push_scatter_kernel<V, MAT><<<g2, kTPB, 0, st>>>(a, 1);
    HIPCHK(hipGetLastError());
    return GLINT_OK;
  }
  HIPCHK(hipMemsetAsync(s->d_ctl, 0, sizeof(LaunchCtl), st));
  {
    const unsigned gc =
        grid_for(ntiles, kTPB / 64, (i64)s->cus * blocks_per_cu(push_check_kernel<MAT>, 2, "GLINT_CHECK_BPC"));
    ProfScope pc(s, GLINT_K_PUSH_CHECK, st);
    push_check_kernel<MAT><<<gc, kTPB, 0, st>>>(keys, cols, n, a.part, a.ctl, desc, a.ntiles);
    HIPCHK(hipGetLastError());
  }
  {
    const unsigned ga =
        grid_for(ntiles, kTPB / 64, (i64)s->cus * blocks_per_cu(push_apply_kernel<V, MAT>, 2, "GLINT_APPLY_BPC"));
    a.sweep_blocks = std::min<u32>(ga, (u32)((i64)s->cus * sweep_blocks_per_cu()));
    ProfScope ps(s, GLINT_K_PUSH_APPLY, st);
    push_apply_kernel<V, MAT><<<ga, kTPB, 0, st>>>(a, desc);
    HIPCHK(hipGetLastError());
  }
  if (det) return push_det_tail<V, MAT>(s, a, true, st);
  if (binned) return push_binned<V, MAT>(s, a, true, st);
  const unsigned g2 = grid_for(n, kScatterChunk, (i64)s->cus * 2);
  ProfScope ps(s, GLINT_K_PUSH_SCATTER, st);
  push_scatter_kernel<V, MAT><<<g2, kTPB, 0, st>>>(a, 0);
  HIPCHK(hipGetLastError());
  return GLINT_OK;
}

// ---- pulls ------------------------------------------------------------------------------------
template <typename V>
int launch_vec_pull(glint_shard* s, const i64* keys, void* out, i64 n, hipStream_t st) {
  if (n <= 0) return GLINT_OK;
  if (!keys || !out) return GLINT_EINVAL;
  const bool pairs = aligned(keys, 16) && aligned(out, 2 * sizeof(V));
  ProfScope ps(s, GLINT_K_VEC_PULL, st);
  if (pairs) {
    // 4 blocks per CU: the dense gather's best (tools/microbench_stream.hip mode 5)
    const unsigned g = grid_for((n + 1) / 2, kTPB, (i64)s->cus * 4);
    vec_pull_kernel<V, true><<<g, kTPB, 0, st>>>(keys, n, (const V*)s->data, s->part, (V*)out, s->d_err);
  } else {
    const unsigned g = grid_for(n, kTPB, (i64)s->cus * 8);
    vec_pull_kernel<V, false><<<g, kTPB, 0, st>>>(keys, n, (const V*)s->data, s->part, (V*)out, s->d_err);
  }
  HIPCHK(hipGetLastError());
  return GLINT_OK;
}

template <typename V>
int launch_mat_pull(glint_shard* s, const i64* rows, const int32_t* cols, void* out, i64 n, hipStream_t st) {
  if (n <= 0) return GLINT_OK;
  if (!rows || !cols || !out) return GLINT_EINVAL;
  const unsigned g = grid_for(n, kTPB, (i64)s->cus * 8);
  ProfScope ps(s, GLINT_K_MAT_PULL, st);
  mat_pull_kernel<V><<<g, kTPB, 0, st>>>(rows, cols, n, (const V*)s->data, s->part, (V*)out, s->d_err);
  HIPCHK(hipGetLastError());
  return GLINT_OK;
}

template <typename V>
int launch_mat_pull_rows(glint_shard* s, const i64* rows, void* out, i64 n, hipStream_t st) {
  if (n <= 0) return GLINT_OK;
  if (!rows || !out) return GLINT_EINVAL;
  const bool v16 = ((i64)s->part.cols * (i64)sizeof(V)) % 16 == 0 && aligned(out, 16);
  const unsigned g = grid_for(n, kTPB / 64, (i64)s->cus * 8);
  ProfScope ps(s, GLINT_K_MAT_PULL_ROWS, st);
  if (v16)
    mat_pull_rows_kernel<V, true><<<g, kTPB, 0, st>>>(rows, n, (const V*)s->data, s->part, (V*)out, s->d_err);
  else
    mat_pull_rows_kernel<V, false><<<g, kTPB, 0, st>>>(rows, n, (const V*)s->data, s->part, (V*)out, s->d_err);
  HIPCHK(hipGetLastError());
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

// read and clear the device error state (caller has synchronised the stream)
int collect_errors(glint_shard* s, hipStream_t st, int64_t* first_bad) {
  ErrState h{};
  HIPCHK(hipMemcpyAsync(&h, s->d_err, sizeof(h), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (h.min_bad_enc != 0) {
    HIPCHK(hipMemsetAsync(s->d_err, 0, sizeof(ErrState), st));
    HIPCHK(hipStreamSynchronize(st));
    s->last_bad = (i64)~h.min_bad_enc;
    if (first_bad) *first_bad = s->last_bad;
    return GLINT_EOUTOFRANGE;
  }
  return GLINT_OK;
}

int create_common(glint_shard* s, int device, int dtype, int32_t cols) {
  if (dtype < GLINT_I32 || dtype > GLINT_F64 || cols < 0) return GLINT_EINVAL;
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
  if (hipMalloc(&s->data, bytes) != hipSuccess) {
    (void)hipGetLastError();
    return GLINT_ENOMEM;
  }
  if (hipMalloc((void**)&s->d_err, sizeof(ErrState)) != hipSuccess) {
    (void)hipGetLastError();
    return GLINT_ENOMEM;
  }
  if (hipHostMalloc((void**)&s->h_hint, 64, hipHostMallocMapped) == hipSuccess) {
    *s->h_hint = 0;
    if (hipHostGetDevicePointer((void**)&s->d_hint, s->h_hint, 0) != hipSuccess) s->d_hint = nullptr;
  } else {
    s->h_hint = nullptr;
  }
  (void)hipGetLastError();
  if (!s->d_hint && s->h_hint) { (void)hipHostFree(s->h_hint); s->h_hint = nullptr; }
  HIPCHK(hipMemsetAsync(s->data, 0, bytes, s->stream));  // new Array[V](size) is zeroed
  HIPCHK(hipMemsetAsync(s->d_err, 0, sizeof(ErrState), s->stream));
  HIPCHK(hipStreamSynchronize(s->stream));
  return GLINT_OK;
}

void free_shard(glint_shard* s) {
  if (!s) return;
  {
    DeviceGuard g(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    prof_drain(s);
    if (s->data) (void)hipFree(s->data);
    if (s->d_err) (void)hipFree(s->d_err);
    if (s->d_ctl) (void)hipFree(s->d_ctl);
    if (s->d_scratch) (void)hipFree(s->d_scratch);
    if (s->d_det) (void)hipFree(s->d_det);
    if (s->d_bin) (void)hipFree(s->d_bin);
    if (s->h_hint) (void)hipHostFree(s->h_hint);
    if (s->stream) (void)hipStreamDestroy(s->stream);
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

}  // namespace

// ================================================================================================
// C ABI
// ================================================================================================
extern "C" {

int glint_version(void) { return 100; }

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

int glint_shard_destroy(glint_shard_t s) {
  if (!s) return GLINT_EINVAL;
  free_shard(s);
  return GLINT_OK;
}

int glint_shard_zero(glint_shard_t s) {
  if (!s) return GLINT_EINVAL;
  std::lock_guard<std::mutex> lk(s->mu);
  DeviceGuard g(s->device);
  HIPCHK(hipMemsetAsync(s->data, 0, (size_t)s->elems * s->vsize, s->stream));
  HIPCHK(hipMemsetAsync(s->d_err, 0, sizeof(ErrState), s->stream));
  HIPCHK(hipStreamSynchronize(s->stream));
  return GLINT_OK;
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
  std::lock_guard<std::mutex> lk(s->mu);
  s->prof = on != 0;
  return GLINT_OK;
}

int glint_prof_read(glint_shard_t s, int kernel_id, double* total_ms, int64_t* launches) {
  if (!s || kernel_id < 0 || kernel_id >= GLINT_K_COUNT) return GLINT_EINVAL;
  std::lock_guard<std::mutex> lk(s->mu);
  DeviceGuard g(s->device);
  prof_drain(s);
  if (total_ms) *total_ms = s->prof_ms[kernel_id];
  if (launches) *launches = s->prof_n[kernel_id];
  return GLINT_OK;
}

int glint_prof_reset(glint_shard_t s) {
  if (!s) return GLINT_EINVAL;
  std::lock_guard<std::mutex> lk(s->mu);
  DeviceGuard g(s->device);
  prof_drain(s);
  for (int k = 0; k < GLINT_K_COUNT; ++k) { s->prof_ms[k] = 0; s->prof_n[k] = 0; }
  return GLINT_OK;
}

int glint_shard_sync(glint_shard_t s, void* stream, int64_t* first_bad) {
  if (!s) return GLINT_EINVAL;
  std::lock_guard<std::mutex> lk(s->mu);
  DeviceGuard g(s->device);
  hipStream_t st = pick(s, stream);
  HIPCHK(hipStreamSynchronize(st));
  return collect_errors(s, st, first_bad);
}

// ---- device-resident ---------------------------------------------------------------------------
int glint_vec_push_dev(glint_shard_t s, const int64_t* keys, const void* vals, int64_t n, int flags, void* stream) {
  if (!s || n < 0) return GLINT_EINVAL;
  if (s->part.cols != 0) return GLINT_EINVAL;
  std::lock_guard<std::mutex> lk(s->mu);
  DeviceGuard g(s->device);
  GLINT_DISPATCH(s->dtype, push_vec_t, s, (const i64*)keys, nullptr, vals, n, flags, pick(s, stream));
}

int glint_mat_push_dev(glint_shard_t s, const int64_t* rows, const int32_t* cols, const void* vals, int64_t n,
                       int flags, void* stream) {
  if (!s || n < 0) return GLINT_EINVAL;
  if (s->part.cols == 0) return GLINT_EINVAL;
  std::lock_guard<std::mutex> lk(s->mu);
  DeviceGuard g(s->device);
  GLINT_DISPATCH(s->dtype, push_mat_t, s, (const i64*)rows, cols, vals, n, flags, pick(s, stream));
}

int glint_vec_pull_dev(glint_shard_t s, const int64_t* keys, void* out, int64_t n, void* stream) {
  if (!s || n < 0) return GLINT_EINVAL;
  if (s->part.cols != 0) return GLINT_EINVAL;
  std::lock_guard<std::mutex> lk(s->mu);
  DeviceGuard g(s->device);
  GLINT_DISPATCH(s->dtype, launch_vec_pull, s, (const i64*)keys, out, n, pick(s, stream));
}

int glint_mat_pull_dev(glint_shard_t s, const int64_t* rows, const int32_t* cols, void* out, int64_t n,
                       void* stream) {
  if (!s || n < 0) return GLINT_EINVAL;
  if (s->part.cols == 0) return GLINT_EINVAL;
  std::lock_guard<std::mutex> lk(s->mu);
  DeviceGuard g(s->device);
  GLINT_DISPATCH(s->dtype, launch_mat_pull, s, (const i64*)rows, cols, out, n, pick(s, stream));
}

int glint_mat_pull_rows_dev(glint_shard_t s, const int64_t* rows, void* out, int64_t n, void* stream) {
  if (!s || n < 0) return GLINT_EINVAL;
  if (s->part.cols == 0) return GLINT_EINVAL;
  std::lock_guard<std::mutex> lk(s->mu);
  DeviceGuard g(s->device);
  GLINT_DISPATCH(s->dtype, launch_mat_pull_rows, s, (const i64*)rows, out, n, pick(s, stream));
}

}  // extern "C"

// ---- host-pointer entry points --------------------------------------------------------------------
namespace {

// stage host arrays into the shard's device scratch: returns device pointers to each section
struct Staged {
  char* p[3] = {nullptr, nullptr, nullptr};
};

int stage(glint_shard* s, const void* const* src, const size_t* bytes, int count, Staged& out, size_t extra,
          char** extra_ptr) {
  size_t need = 0;
  for (int i = 0; i < count; ++i) need += pad256(bytes[i]);
  need += pad256(extra);
  int rc = grow(&s->d_scratch, &s->scratch_bytes, need);
  if (rc) return rc;
  char* b = (char*)s->d_scratch;
  for (int i = 0; i < count; ++i) {
    out.p[i] = b;
    if (bytes[i]) HIPCHK(hipMemcpyAsync(b, src[i], bytes[i], hipMemcpyHostToDevice, s->stream));
    b += pad256(bytes[i]);
  }
  if (extra_ptr) *extra_ptr = b;
  return GLINT_OK;
}

int finish(glint_shard* s) {
  HIPCHK(hipStreamSynchronize(s->stream));
  return collect_errors(s, s->stream, nullptr);
}

int host_push(glint_shard* s, bool mat, const int64_t* keys, const int32_t* cols, const void* vals, int64_t n,
              int flags) {
  if (n < 0 || (n > 0 && (!keys || !vals || (mat && !cols)))) return GLINT_EINVAL;
  if (mat != (s->part.cols != 0)) return GLINT_EINVAL;
  if (n == 0) return GLINT_OK;
  std::lock_guard<std::mutex> lk(s->mu);
  DeviceGuard g(s->device);
  Staged st;
  const void* src[3] = {keys, mat ? (const void*)cols : vals, vals};
  size_t bytes[3] = {(size_t)n * 8, mat ? (size_t)n * 4 : (size_t)n * s->vsize, (size_t)n * s->vsize};
  int rc = stage(s, src, bytes, mat ? 3 : 2, st, 0, nullptr);
  if (rc) return rc;
  if (mat) {
    rc = [&]() -> int {
      GLINT_DISPATCH(s->dtype, push_mat_t, s, (const i64*)st.p[0], (const int32_t*)st.p[1], st.p[2], n, flags,
                     s->stream);
    }();
  } else {
    rc = [&]() -> int {
      GLINT_DISPATCH(s->dtype, push_vec_t, s, (const i64*)st.p[0], nullptr, st.p[1], n, flags, s->stream);
    }();
  }
  if (rc) return rc;
  return finish(s);
}

// kind: 0 vector get, 1 matrix get, 2 matrix rows
int host_pull(glint_shard* s, int kind, const int64_t* keys, const int32_t* cols, void* out, int64_t n) {
  if (n < 0 || (n > 0 && (!keys || !out || (kind == 1 && !cols)))) return GLINT_EINVAL;
  if ((kind == 0) != (s->part.cols == 0)) return GLINT_EINVAL;
  if (n == 0) return GLINT_OK;
  std::lock_guard<std::mutex> lk(s->mu);
  DeviceGuard g(s->device);
  const size_t out_bytes = (size_t)n * s->vsize * (kind == 2 ? (size_t)s->part.cols : 1);
  Staged st;
  const void* src[2] = {keys, cols};
  size_t bytes[2] = {(size_t)n * 8, kind == 1 ? (size_t)n * 4 : 0};
  char* d_out = nullptr;
  int rc = stage(s, src, bytes, kind == 1 ? 2 : 1, st, out_bytes, &d_out);
  if (rc) return rc;
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
  if (rc) return rc;
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

// RequestSerializer.fromBinary for the pull messages + ResponseSerializer.toBinary of the answer
// (ResponseSerializer.scala:43-117; row answers are flattened rows x cols, :52-61).
int glint_pull_wire(glint_shard_t s, const uint8_t* payload, size_t len, uint8_t* response, size_t cap,
                    size_t* out_len) {
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
  return host_pull(s, kind, (const int64_t*)keys, kind == 1 ? (const int32_t*)cols : nullptr, response + 5, n);
}

}  // extern "C"
