// glint_sort.hip -- the sort-based tails of a push:
//   binned push     large unordered tails: rocPRIM radix sort by shard slab, LDS slab accumulation,
//                   one coalesced read-modify-write per touched element pair;
//   deterministic   stable rocPRIM sort by address, then an in-order fold per address starting from
//                   the shard's value -- PartialVector.update's sequential `+=` order
//                   (src/main/scala/glint/models/server/PartialVector.scala:35-43), bit for bit.
// Kept apart from glint_gpu.hip so that the rocPRIM instantiations compile once.
#include "glint_device.h"
#include "glint_host.h"

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <cstring>

namespace glint {

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
constexpr int kDedupSlots = 4096;   // u32 keys + 64-bit sums (LdsAcc): 48 KiB
constexpr int kDedupChunk = 2048;   // records per table fill (load factor <= 0.5)
template <typename V, bool MAT>
__global__ __launch_bounds__(kTPB) void bin_dedup_kernel(const i64* __restrict__ keys, const int32_t* __restrict__ cols,
                                                         const V* __restrict__ vals, i64 n, PartDesc part,
                                                         const LaunchCtl* ctl, u32 ntiles, int from_break,
                                                         u32* __restrict__ addr_out, V* __restrict__ val_out,
                                                         u32* __restrict__ m_out, ErrState* err) {
  typedef typename LdsAcc<V>::T A;
  __shared__ u32 hk[kDedupSlots];
  __shared__ A hv[kDedupSlots];
  // slots claimed in this chunk, in claim order: the compaction walks only these (distinct <=
  // kDedupChunk) instead of scanning and re-zeroing the whole table
  __shared__ uint16_t used[kDedupChunk];
  __shared__ u32 nused, obase, olen;
  const int tid = threadIdx.x, lane = tid & 63;
  i64 r0 = 0;
  if (from_break) {
    const u32 brk = ctl->brk_enc;
    r0 = brk == 0u ? n : (i64)(ntiles - brk) * kTile;
  }
  if (blockIdx.x == 0 && tid == 0) m_out[1] = (u32)(n - r0);  // the tail size, for the host's ratio
  for (int sl = tid; sl < kDedupSlots; sl += kTPB) { hk[sl] = kBinSentinel; hv[sl] = A(0); }
  if (tid == 0) nused = 0;
  __syncthreads();
  const u64 below = (1ull << lane) - 1ull;
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
      bool claimed = false;
      u32 h = 0;
      if (i < c1) {
        i64 ad64;
        if (!rec_addr<MAT>(part, k[q], cl[q], ad64)) {
          record_error(err, i);
        } else {
          const u32 ad = (u32)ad64;
          h = (ad * 0x9E3779B1u) >> (32 - 12);
          for (;;) {
            const u32 cur = hk[h];
            if (cur == ad) break;
            if (cur == kBinSentinel) {
              const u32 prev = atomicCAS(&hk[h], kBinSentinel, ad);
              if (prev == kBinSentinel) { claimed = true; break; }
              if (prev == ad) break;
            }
            h = (h + 1) & (kDedupSlots - 1);
          }
          lds_add(&hv[h], (A)v[q]);
        }
      }
      // the wave's new slots join the list with one LDS atomic (every lane reaches the ballot)
      const u64 b = __ballot(claimed);
      if (b) {
        u32 base = 0;
        if (lane == 0) base = atomicAdd(&nused, (u32)__popcll(b));
        base = __shfl(base, 0);
        if (claimed) used[base + (u32)__popcll(b & below)] = (uint16_t)h;
      }
    }
    __syncthreads();
    if (tid == 0) {
      olen = nused;
      obase = atomicAdd(m_out, olen);
      nused = 0;
    }
    __syncthreads();
    const u32 len = olen, ob = obase;
    for (u32 j = tid; j < len; j += kTPB) {  // contiguous, coalesced output of the chunk's sums
      const u32 sl = used[j];
      addr_out[ob + j] = hk[sl];
      val_out[ob + j] = (V)hv[sl];
      hk[sl] = kBinSentinel;
      hv[sl] = A(0);
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
                                                            i64 elems, V* __restrict__ data, u32 pre_min) {
  typedef typename Vec2<V>::T V2;
  typedef typename LdsAcc<V>::T A;
  __shared__ A acc[kSlab];
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
    V* const sbase = data + sbase_g;
    // A slab item with many records touches most of its lines: pull the slab into L2 now (one
    // dword per 128-B line), so the fetch overlaps the record phase and the RMW's loads below hit
    // in cache. Into registers it would cost the kernel its occupancy (246 VGPRs, measured).
    const bool pre = exclusive && (u32)(r_hi - r_lo) >= pre_min;
    u32 warm = 0;
    if (pre) {
      constexpr int kLines = kSlab * (int)sizeof(V) / 128;
      constexpr int kPerLine = 128 / (int)sizeof(V);
      for (int l = tid; l < kLines; l += kBinTPB)
        if (sbase_g + (i64)l * kPerLine < elems) warm ^= *reinterpret_cast<const u32*>(sbase + (i64)l * kPerLine);
    }
    for (int e = tid; e < kSlab; e += kBinTPB) acc[e] = A(0);
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
        lds_add(&acc[e], (A)v[q]);
        touched[e] = 1;
      }
    }
    asm volatile("" ::"v"(warm));  // the warm-up loads complete here, after the record phase
    __syncthreads();
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
          if (t[q] & 1u) r.x = acc_add(r.x, acc[e0]);
          if (t[q] & 2u) r.y = acc_add(r.y, acc[e0 + 1]);
          *reinterpret_cast<V2*>(sbase + e0) = r;
        } else {  // the shard's last element, odd count
          sbase[e0] = acc_add(sbase[e0], acc[e0]);
        }
      }
    } else {
      for (int e = tid; e < kSlab; e += kBinTPB)
        if (touched[e]) gadd(sbase + e, (V)acc[e]);
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------
// deterministic tail: stable sort by address, then an in-order fold per address starting from the
// shard's current value -- the reference's sequential `+=` order, bit for bit
// ------------------------------------------------------------------------------------------------
// Records before the tail start (push_check's break, read here on the device: no host round trip)
// and rejected records get the sentinel address, which sorts behind every element and is skipped.
template <typename V, bool MAT>
__global__ __launch_bounds__(kTPB) void det_prepare_kernel(const i64* keys, const int32_t* cols, const V* vals, i64 m,
                                                           const LaunchCtl* ctl, u32 ntiles, int from_break,
                                                           PartDesc part, u64 sentinel, u64* addr, V* val,
                                                           ErrState* err) {
  i64 r0 = 0;
  if (from_break) {
    const u32 brk = ctl->brk_enc;
    r0 = brk == 0u ? m : (i64)(ntiles - brk) * kTile;
  }
  for (i64 i = (i64)blockIdx.x * kTPB + threadIdx.x; i < m; i += (i64)gridDim.x * kTPB) {
    u64 out = sentinel;
    if (i >= r0) {
      i64 ad;
      if (rec_addr<MAT>(part, keys[i], MAT ? cols[i] : 0, ad)) out = (u64)ad;
      else record_error(err, i);
    }
    addr[i] = out;
    val[i] = vals[i];
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

// ---- host side ----------------------------------------------------------------------------------
template <typename V, bool MAT>
int push_det_tail(glint_shard* s, const PushArgs<V>& a, bool from_break, hipStream_t st) {
  // the whole push is sorted; records before push_check's break are masked on the device, so the
  // call stays stream-ordered with no host synchronisation
  const i64 m = a.n;
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
  det_prepare_kernel<V, MAT><<<g, kTPB, 0, st>>>(a.keys, a.cols, a.vals, m, a.ctl, a.ntiles, from_break ? 1 : 0,
                                                 a.part, sentinel, addr_in, val_in, a.err);
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

// records per slab item from which bin_apply prefetches the whole slab (GLINT_BIN_PREFETCH_MIN;
// 0xFFFFFFFF disables)
u32 bin_prefetch_min() {
  static const u32 v = [] {
    const char* e = getenv("GLINT_BIN_PREFETCH_MIN");
    return e ? (u32)strtoul(e, nullptr, 10) : (u32)(kSlab / 4);
  }();
  return v;
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
  // dedup when the last probe found < 60 % distinct records per chunk; re-probe every 16 pushes.
  // GLINT_BIN_FRONT = dedup | prep forces one front end (tests, tuning).
  bool dedup = s->bin_dedup_ratio < 0.6 || (++s->bin_pushes & 15) == 0;
  if (const char* e = getenv("GLINT_BIN_FRONT")) {
    if (!strcmp(e, "dedup")) dedup = true;
    else if (!strcmp(e, "prep")) dedup = false;
  }
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
  static const int apply_bpc = [] {  // GLINT_BIN_APPLY_BPC: work-item blocks per CU (tuning knob)
    const char* e = getenv("GLINT_BIN_APPLY_BPC");
    return (e && atoi(e) > 0) ? atoi(e) : 64;  // swept 4..all: 32-128 best (profiles/r01/bin_apply_bpc.txt)
  }();
  bin_apply_kernel<V><<<(unsigned)std::min<i64>(mi, (i64)s->cus * apply_bpc), kBinTPB, 0, st>>>(
      addr_out, val_out, item_desc, item_off, nslabs, s->elems, a.data, bin_prefetch_min());
  HIPCHK(hipGetLastError());
  return GLINT_OK;
}

#define GLINT_INST(V, MAT)                                                                         \
  template int push_det_tail<V, MAT>(glint_shard*, const PushArgs<V>&, bool, hipStream_t);        \
  template int push_binned<V, MAT>(glint_shard*, const PushArgs<V>&, bool, hipStream_t);
GLINT_INST(int, false)
GLINT_INST(int, true)
GLINT_INST(long long, false)
GLINT_INST(long long, true)
GLINT_INST(float, false)
GLINT_INST(float, true)
GLINT_INST(double, false)
GLINT_INST(double, true)
#undef GLINT_INST

}  // namespace glint
