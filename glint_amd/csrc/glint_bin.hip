// glint_bin.hip -- the binned push: large unordered pushes summed per shard slab in LDS, with no
// per-record device atomics, no sort library and no host round trip (every size and count stays on
// the device). PartialVector.update / PartialMatrix.update (src/main/scala/glint/models/server/
// PartialVector.scala:35-43, PartialMatrix.scala:74-83) for records in no particular order.
//
// A slab is 4096 consecutive shard elements: the unit one workgroup sums in LDS. Records are moved
// into slab order by a two-level MSD partition on the slab index -- a coarse digit (<= 1024
// buckets) and a fine digit (<= 1024 slabs per bucket) -- and each slab's records are then summed
// in LDS and written back with one coalesced read-modify-write of the touched element pairs:
//
//   bin_count   raw records per (region, coarse bucket), region = chunk % 8 (one per XCD); the last
//               workgroup turns the counts into capacity offsets of the (bucket, region) segments.
//   bin_part    per 2048-record chunk: (optionally) sums duplicate elements in an LDS hash table,
//               then appends the chunk's records to its region's segment of each bucket (one
//               returning atomic per bucket per chunk), staged in LDS so the stores are runs.
//               Segments of one region are written only by workgroups of one XCD, so partial lines
//               merge in that XCD's L2 before they reach HBM.
//   bin_bitems  segment lengths -> fine-partition work items (<= 2048 records each).
//   bin_fhist   per item: records per slab (exact, after dedup) -> H[slab].
//   bin_cscan   one workgroup: slab starts (exclusive scan of H) and the apply work items (slabs with
//               more than 16384 records are cut into several items, which flush with atomics).
//   bin_fpart   per item: records moved to their slab's range (LDS-staged runs).
//   bin_apply   per apply item: LDS accumulation of the slab, coalesced RMW of touched pairs.
//
// Capacities come from the raw counts, so dedup can only leave holes at segment ends; the fine
// partition counts exactly, so the slab ranges it writes are dense.
#include "glint_device.h"
#include "glint_host.h"

#include <cstring>

namespace glint {

constexpr int kSlabBits = 12;
constexpr int kSlab = 1 << kSlabBits;
constexpr int kRegions = 8;            // partition regions: one per XCD
constexpr int kMaxDigit = 1024;        // coarse buckets and fine slabs per bucket, at most
constexpr int kATPB = 256;
constexpr int kAChunk = 2048;          // records per partition chunk (and dedup table fill)
constexpr int kAPer = kAChunk / kATPB;
constexpr int kASlots = 4096;          // dedup hash slots (load <= 0.5)
constexpr int kBItem = 2048;           // records per fine-partition item
constexpr int kBPer = kBItem / kATPB;
constexpr u32 kCItem = 16384;          // records per apply item at most
constexpr u32 kEmptySlot = 0xFFFFFFFFu;
constexpr int kScanTPB = 1024;

struct BinGeom {
  u32 fb;     // fine digit bits
  u32 nb;     // coarse buckets (power of two)
  u32 nf;     // fine slabs per bucket (power of two)
  u32 nslab;  // nb * nf
};
__device__ __forceinline__ u32 bucket_of(u32 a, const BinGeom& g) { return a >> (kSlabBits + g.fb); }

struct BinCtl {
  u32 done_count;  // bin_count workgroups finished (last-block detection)
  u32 nb_items;    // fine-partition items
  u32 nc_items;    // apply items
  u32 tail;        // valid records in the tail
  u32 m;           // records after dedup
  u32 pad_[3];
};

// ---- small block-level helpers ------------------------------------------------------------------
// Exclusive scan over N values by one workgroup of TPB threads; value(i) may be called twice;
// write(i, exclusive prefix) is called once per i in increasing i per thread. Returns the total.
template <int TPB, typename F, typename W>
__device__ __forceinline__ u32 block_scan(u32 N, F value, W write) {
  __shared__ u32 wt[TPB / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const u32 per = (N + TPB - 1) / TPB;
  const u32 b0 = min(N, (u32)tid * per), b1 = min(N, b0 + per);
  u32 s = 0;
  for (u32 i = b0; i < b1; ++i) s += value(i);
  u32 incl = s;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const u32 y = __shfl_up(incl, d);
    if (lane >= d) incl += y;
  }
  if (lane == 63) wt[wid] = incl;
  __syncthreads();
  u32 run = incl - s, tot = 0;
#pragma unroll
  for (int w = 0; w < TPB / 64; ++w) {
    const u32 x = wt[w];
    run += w < wid ? x : 0u;
    tot += x;
  }
  for (u32 i = b0; i < b1; ++i) {
    const u32 v = value(i);
    write(i, run);
    run += v;
  }
  __syncthreads();
  return tot;
}

template <bool MAT>
__device__ __forceinline__ i64 tail_start(const LaunchCtl* lctl, u32 ntiles, int from_break, i64 n) {
  if (!from_break) return 0;
  const u32 brk = lctl->brk_enc;  // written by push_check; ordered by the kernel boundary
  return brk == 0u ? n : (i64)(ntiles - brk) * kTile;
}

// ---- bin_count ------------------------------------------------------------------------------------
template <bool MAT>
__global__ __launch_bounds__(kATPB) void bin_count_kernel(const i64* __restrict__ keys, const int32_t* __restrict__ cols,
                                                          i64 n, PartDesc part, const LaunchCtl* lctl, u32 ntiles,
                                                          int from_break, BinGeom g, u32* __restrict__ R,
                                                          u32* __restrict__ cap_off, BinCtl* bc) {
  __shared__ u32 h[kMaxDigit];
  __shared__ bool last;
  const int tid = threadIdx.x;
  const i64 r0 = tail_start<MAT>(lctl, ntiles, from_break, n);
  for (u32 b = tid; b < g.nb; b += kATPB) h[b] = 0;
  __syncthreads();
  const u32 region = blockIdx.x % kRegions;  // gridDim.x is a multiple of kRegions: chunk c -> c % 8
  const i64 nchunks = (n - r0 + kAChunk - 1) / kAChunk;
  for (i64 c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const i64 c0 = r0 + c * kAChunk, c1 = min(n, c0 + kAChunk);
    i64 k[kAPer];
    int32_t cl[kAPer];
#pragma unroll
    for (int q = 0; q < kAPer; ++q) {  // clamped, branch-free loads
      const i64 i = c0 + q * kATPB + tid;
      const i64 ii = i < c1 ? i : c1 - 1;
      k[q] = keys[ii];
      cl[q] = MAT ? cols[ii] : 0;
    }
#pragma unroll
    for (int q = 0; q < kAPer; ++q) {
      i64 ad;
      if (c0 + q * kATPB + tid < c1 && rec_addr<MAT>(part, k[q], cl[q], ad)) atomicAdd(&h[bucket_of((u32)ad, g)], 1u);
    }
  }
  __syncthreads();
  for (u32 b = tid; b < g.nb; b += kATPB)
    if (h[b]) atomicAdd(&R[region * g.nb + b], h[b]);
  __threadfence();
  __syncthreads();
  if (tid == 0) last = atomicAdd(&bc->done_count, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  __threadfence();
  // capacity offsets, bucket-major: segment (b, x) = e = b * 8 + x holds R[x][b] records at most
  const u32 ne = g.nb * kRegions;
  const u32 tot = block_scan<kATPB>(
      ne,
      [&](u32 e) { return __hip_atomic_load(&R[(e % kRegions) * g.nb + e / kRegions], __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT); },
      [&](u32 e, u32 x) { cap_off[e] = x; });
  if (tid == 0) {
    cap_off[ne] = tot;
    bc->tail = tot;
  }
}

// ---- bin_part -------------------------------------------------------------------------------------
// Appends a chunk's records (P per thread in registers, `valid` bit mask) to their bucket's segment
// of this workgroup's region. dcnt must be zero on entry and is zero again on exit.
template <typename A, int P>
__device__ __forceinline__ void part_emit(const u32 (&ad)[P], const A (&va)[P], u32 valid, const BinGeom& g,
                                          u32 region, u32* dcnt, u32* dgo, const u32* cap, u32* __restrict__ cur,
                                          u32* st_a, A* st_v, u32* __restrict__ addr_out, A* __restrict__ val_out) {
  const int tid = threadIdx.x;
  u32 rank[P];
#pragma unroll
  for (int j = 0; j < P; ++j)
    if (valid & (1u << j)) rank[j] = atomicAdd(&dcnt[bucket_of(ad[j], g)], 1u);
  __syncthreads();
  const u32 total = block_scan<kATPB>(
      g.nb, [&](u32 d) { return dcnt[d]; },
      [&](u32 d, u32 excl) {
        const u32 c = dcnt[d];
        u32 go = 0;
        if (c) go = cap[d] + atomicAdd(&cur[region * g.nb + d], c);
        dgo[d] = go - excl;  // global slot of local staging position p (digit d) = dgo[d] + p
        dcnt[d] = excl;
      });
#pragma unroll
  for (int j = 0; j < P; ++j) {
    if (valid & (1u << j)) {
      const u32 p = dcnt[bucket_of(ad[j], g)] + rank[j];
      st_a[p] = ad[j];
      st_v[p] = va[j];
    }
  }
  __syncthreads();
  for (u32 p = tid; p < total; p += kATPB) {  // consecutive threads: consecutive slots of one run
    const u32 a = st_a[p];
    const u32 pos = dgo[bucket_of(a, g)] + p;
    addr_out[pos] = a;
    val_out[pos] = st_v[p];
  }
  __syncthreads();
  for (u32 d = tid; d < g.nb; d += kATPB) dcnt[d] = 0;
  __syncthreads();
}

template <typename V, bool MAT>
__device__ __forceinline__ void load_chunk(const i64* __restrict__ keys, const int32_t* __restrict__ cols,
                                           const V* __restrict__ vals, i64 c0, i64 c1, i64 (&k)[kAPer],
                                           int32_t (&cl)[kAPer], V (&v)[kAPer]) {
#pragma unroll
  for (int q = 0; q < kAPer; ++q) {  // clamped, branch-free loads
    const i64 i = c0 + q * kATPB + threadIdx.x;
    const i64 ii = i < c1 ? i : c1 - 1;
    k[q] = keys[ii];
    cl[q] = MAT ? cols[ii] : 0;
    v[q] = vals[ii];
  }
}

// Plain front end: every valid record is appended as it is.
template <typename V, bool MAT>
__global__ __launch_bounds__(kATPB) void bin_part_kernel(const i64* __restrict__ keys, const int32_t* __restrict__ cols,
                                                         const V* __restrict__ vals, i64 n, PartDesc part,
                                                         const LaunchCtl* lctl, u32 ntiles, int from_break, BinGeom g,
                                                         const u32* __restrict__ cap_off, u32* __restrict__ cur,
                                                         u32* __restrict__ addr_out,
                                                         typename LdsAcc<V>::T* __restrict__ val_out, ErrState* err) {
  typedef typename LdsAcc<V>::T A;
  __shared__ u32 dcnt[kMaxDigit], dgo[kMaxDigit], cap[kMaxDigit];
  __shared__ u32 st_a[kAChunk];
  __shared__ A st_v[kAChunk];
  const int tid = threadIdx.x;
  const u32 region = blockIdx.x % kRegions;
  const i64 r0 = tail_start<MAT>(lctl, ntiles, from_break, n);
  for (u32 d = tid; d < g.nb; d += kATPB) {
    dcnt[d] = 0;
    cap[d] = cap_off[d * kRegions + region];
  }
  __syncthreads();
  const i64 nchunks = (n - r0 + kAChunk - 1) / kAChunk;
  i64 k[kAPer];
  int32_t cl[kAPer];
  V v[kAPer];
  i64 c = blockIdx.x;
  if (c < nchunks) load_chunk<V, MAT>(keys, cols, vals, r0 + c * kAChunk, min(n, r0 + (c + 1) * kAChunk), k, cl, v);
  for (; c < nchunks; c += gridDim.x) {
    const i64 c0 = r0 + c * kAChunk, c1 = min(n, c0 + kAChunk);
    u32 ad[kAPer];
    A va[kAPer];
    u32 valid = 0;
#pragma unroll
    for (int q = 0; q < kAPer; ++q) {
      const i64 i = c0 + q * kATPB + tid;
      i64 a64;
      ad[q] = 0;
      va[q] = (A)v[q];
      if (i < c1) {
        if (rec_addr<MAT>(part, k[q], cl[q], a64)) {
          ad[q] = (u32)a64;
          valid |= 1u << q;
        } else {
          record_error(err, i);
        }
      }
    }
    const i64 cn = c + gridDim.x;  // next chunk's loads overlap this chunk's partition
    if (cn < nchunks) load_chunk<V, MAT>(keys, cols, vals, r0 + cn * kAChunk, min(n, r0 + (cn + 1) * kAChunk), k, cl, v);
    part_emit<A, kAPer>(ad, va, valid, g, region, dcnt, dgo, cap, cur, st_a, st_v, addr_out, val_out);
  }
}

// Dedup front end for duplicate-heavy tails: per chunk, equal elements are summed in an LDS hash
// table first, so one record per distinct element of the chunk moves on. The staging buffer of the
// append overlays the table's value array.
template <typename V, bool MAT>
__global__ __launch_bounds__(kATPB) void bin_part_dedup_kernel(
    const i64* __restrict__ keys, const int32_t* __restrict__ cols, const V* __restrict__ vals, i64 n, PartDesc part,
    const LaunchCtl* lctl, u32 ntiles, int from_break, BinGeom g, const u32* __restrict__ cap_off,
    u32* __restrict__ cur, u32* __restrict__ addr_out, typename LdsAcc<V>::T* __restrict__ val_out, ErrState* err) {
  typedef typename LdsAcc<V>::T A;
  static_assert(kAChunk * (4 + sizeof(A)) <= kASlots * sizeof(A), "staging must fit the value table");
  __shared__ u32 hk[kASlots];
  __shared__ A hv[kASlots];
  __shared__ uint16_t used[kAChunk];
  __shared__ u32 dcnt[kMaxDigit], dgo[kMaxDigit], cap[kMaxDigit];
  __shared__ u32 nused;
  const int tid = threadIdx.x, lane = tid & 63;
  const u32 region = blockIdx.x % kRegions;
  const i64 r0 = tail_start<MAT>(lctl, ntiles, from_break, n);
  A* const st_v = hv;
  u32* const st_a = reinterpret_cast<u32*>(hv + kAChunk);
  constexpr int kStageA = (kAChunk * (4 + (int)sizeof(A)) + (int)sizeof(A) - 1) / (int)sizeof(A);  // hv entries staging uses
  for (int sl = tid; sl < kASlots; sl += kATPB) {
    hk[sl] = kEmptySlot;
    hv[sl] = A(0);
  }
  for (u32 d = tid; d < g.nb; d += kATPB) {
    dcnt[d] = 0;
    cap[d] = cap_off[d * kRegions + region];
  }
  if (tid == 0) nused = 0;
  __syncthreads();
  const u64 below = (1ull << lane) - 1ull;
  const i64 nchunks = (n - r0 + kAChunk - 1) / kAChunk;
  i64 k[kAPer];
  int32_t cl[kAPer];
  V v[kAPer];
  i64 c = blockIdx.x;
  if (c < nchunks) load_chunk<V, MAT>(keys, cols, vals, r0 + c * kAChunk, min(n, r0 + (c + 1) * kAChunk), k, cl, v);
  for (; c < nchunks; c += gridDim.x) {
    const i64 c0 = r0 + c * kAChunk, c1 = min(n, c0 + kAChunk);
#pragma unroll
    for (int q = 0; q < kAPer; ++q) {
      const i64 i = c0 + q * kATPB + tid;
      bool claimed = false;
      u32 h = 0;
      if (i < c1) {
        i64 a64;
        if (!rec_addr<MAT>(part, k[q], cl[q], a64)) {
          record_error(err, i);
        } else {
          const u32 a = (u32)a64;
          h = (a * 0x9E3779B1u) >> (32 - 12);
          for (;;) {  // the compare-and-swap is the probe: one LDS round trip per slot tried
            const u32 prev = atomicCAS(&hk[h], kEmptySlot, a);
            if (prev == kEmptySlot) { claimed = true; break; }
            if (prev == a) break;
            h = (h + 1) & (kASlots - 1);
          }
          lds_add(&hv[h], (A)v[q]);
        }
      }
      const u64 b = __ballot(claimed);  // the wave's new slots join the list with one LDS atomic
      if (b) {
        u32 base = 0;
        if (lane == 0) base = atomicAdd(&nused, (u32)__popcll(b));
        base = __shfl(base, 0);
        if (claimed) used[base + (u32)__popcll(b & below)] = (uint16_t)h;
      }
    }
    const i64 cn = c + gridDim.x;  // next chunk's loads overlap the append below
    if (cn < nchunks) load_chunk<V, MAT>(keys, cols, vals, r0 + cn * kAChunk, min(n, r0 + (cn + 1) * kAChunk), k, cl, v);
    __syncthreads();
    const u32 D = nused;
    u32 ad[kAPer];
    A va[kAPer];
    u32 valid = 0;
#pragma unroll
    for (int j = 0; j < kAPer; ++j) {  // the chunk's distinct elements, out of the table
      const u32 e = tid + j * kATPB;
      ad[j] = 0;
      va[j] = A(0);
      if (e < D) {
        const u32 sl = used[e];
        ad[j] = hk[sl];
        va[j] = hv[sl];
        hk[sl] = kEmptySlot;
        valid |= 1u << j;
      }
    }
    __syncthreads();
    if (tid == 0) nused = 0;
    part_emit<A, kAPer>(ad, va, valid, g, region, dcnt, dgo, cap, cur, st_a, st_v, addr_out, val_out);
    for (int sl = tid; sl < kStageA; sl += kATPB) hv[sl] = A(0);  // staging overlaid these
    for (int j = 0; j < kAPer; ++j) {  // and the table's own slots of this chunk
      const u32 e = tid + j * kATPB;
      if (e < D) {
        const u32 sl = used[e];
        if (sl >= (u32)kStageA) hv[sl] = A(0);
      }
    }
    __syncthreads();
  }
}

// ---- fine partition ---------------------------------------------------------------------------------
// segments -> items of <= kBItem records: {bucket, first, end}
__global__ __launch_bounds__(kATPB) void bin_bitems_kernel(BinGeom g, const u32* __restrict__ cap_off,
                                                           const u32* __restrict__ cur, uint4* __restrict__ bdesc,
                                                           BinCtl* bc, u64* hint) {
  const u32 ne = g.nb * kRegions;
  auto len = [&](u32 e) { return cur[(e % kRegions) * g.nb + e / kRegions]; };
  const u32 tot = block_scan<kATPB>(
      ne, [&](u32 e) { return (len(e) + (u32)kBItem - 1) / (u32)kBItem; },
      [&](u32 e, u32 x) {
        const u32 l = len(e), s0 = cap_off[e], b = e / kRegions;
        for (u32 q = 0; q * (u32)kBItem < l; ++q)
          bdesc[x + q] = make_uint4(b, s0 + q * (u32)kBItem, s0 + min(l, (q + 1) * (u32)kBItem), 0u);
      });
  const u32 m = block_scan<kATPB>(ne, len, [](u32, u32) {});
  if (threadIdx.x == 0) {
    bc->nb_items = tot;
    bc->m = m;
    if (hint)  // for the host's next binned push: how much did dedup keep? (m << 32 | tail)
      __hip_atomic_store(hint, ((u64)m << 32) | (u64)bc->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// records per slab of each item -> H[slab]
__global__ __launch_bounds__(kATPB) void bin_fhist_kernel(BinGeom g, const uint4* __restrict__ bdesc,
                                                          const BinCtl* bc, const u32* __restrict__ addr,
                                                          u32* __restrict__ H) {
  __shared__ u32 fh[kMaxDigit];
  const int tid = threadIdx.x;
  const u32 nit = bc->nb_items;
  for (u32 f = tid; f < g.nf; f += kATPB) fh[f] = 0;
  __syncthreads();
  for (u32 it = blockIdx.x; it < nit; it += gridDim.x) {
    const uint4 d = bdesc[it];
    u32 a[kBPer];
#pragma unroll
    for (int q = 0; q < kBPer; ++q) {
      const u32 r = d.y + q * kATPB + tid;
      a[q] = addr[r < d.z ? r : d.z - 1];
    }
#pragma unroll
    for (int q = 0; q < kBPer; ++q)
      if (d.y + q * kATPB + tid < d.z) atomicAdd(&fh[(a[q] >> kSlabBits) & (g.nf - 1)], 1u);
    __syncthreads();
    for (u32 f = tid; f < g.nf; f += kATPB) {
      const u32 c = fh[f];
      if (c) {
        atomicAdd(&H[d.x * g.nf + f], c);
        fh[f] = 0;
      }
    }
    __syncthreads();
  }
}

// One workgroup: slab starts (exclusive scan of H; cur2 starts there for bin_fpart) and the apply
// items {slab, first, end, exclusive}.
__global__ __launch_bounds__(kScanTPB) void bin_cscan_kernel(BinGeom g, const u32* __restrict__ H,
                                                             u32* __restrict__ cur2, uint4* __restrict__ cdesc,
                                                             BinCtl* bc) {
  __shared__ u32 wt[kScanTPB / 64], wi[kScanTPB / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const u32 N = g.nslab;
  const u32 per = (N + kScanTPB - 1) / kScanTPB;
  const u32 b0 = min(N, (u32)tid * per), b1 = min(N, b0 + per);
  u32 sr = 0, si = 0;
  for (u32 s = b0; s < b1; ++s) {
    const u32 h = H[s];
    sr += h;
    si += (h + kCItem - 1) / kCItem;
  }
  u32 ir = sr, ii = si;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const u32 yr = __shfl_up(ir, d), yi = __shfl_up(ii, d);
    if (lane >= d) {
      ir += yr;
      ii += yi;
    }
  }
  if (lane == 63) {
    wt[wid] = ir;
    wi[wid] = ii;
  }
  __syncthreads();
  u32 rr = ir - sr, ri = ii - si, ti = 0;
#pragma unroll
  for (int w = 0; w < kScanTPB / 64; ++w) {
    rr += w < wid ? wt[w] : 0u;
    ri += w < wid ? wi[w] : 0u;
    ti += wi[w];
  }
  for (u32 s = b0; s < b1; ++s) {
    const u32 h = H[s];
    cur2[s] = rr;
    const u32 m = (h + kCItem - 1) / kCItem;
    for (u32 q = 0; q < m; ++q)
      cdesc[ri + q] = make_uint4(s, rr + q * kCItem, rr + min(h, (q + 1) * kCItem), m == 1u ? 1u : 0u);
    rr += h;
    ri += m;
  }
  if (tid == 0) bc->nc_items = ti;
}

// per item: records moved to their slab's range (cur2[slab] = next free slot of the slab)
template <typename A>
__global__ __launch_bounds__(kATPB) void bin_fpart_kernel(BinGeom g, const uint4* __restrict__ bdesc, const BinCtl* bc,
                                                          const u32* __restrict__ addr_in, const A* __restrict__ val_in,
                                                          u32* __restrict__ cur2, u32* __restrict__ addr_out,
                                                          A* __restrict__ val_out) {
  __shared__ u32 fcnt[kMaxDigit], fgo[kMaxDigit];
  __shared__ u32 st_a[kBItem];
  __shared__ A st_v[kBItem];
  const int tid = threadIdx.x;
  const u32 nit = bc->nb_items;
  for (u32 f = tid; f < g.nf; f += kATPB) fcnt[f] = 0;
  __syncthreads();
  for (u32 it = blockIdx.x; it < nit; it += gridDim.x) {
    const uint4 d = bdesc[it];
    u32 a[kBPer], rank[kBPer];
    A v[kBPer];
    u32 valid = 0;
#pragma unroll
    for (int q = 0; q < kBPer; ++q) {
      const u32 r = d.y + q * kATPB + tid;
      const u32 rr = r < d.z ? r : d.z - 1;
      a[q] = addr_in[rr];
      v[q] = val_in[rr];
      if (r < d.z) valid |= 1u << q;
    }
#pragma unroll
    for (int q = 0; q < kBPer; ++q)
      if (valid & (1u << q)) rank[q] = atomicAdd(&fcnt[(a[q] >> kSlabBits) & (g.nf - 1)], 1u);
    __syncthreads();
    const u32 total = block_scan<kATPB>(
        g.nf, [&](u32 f) { return fcnt[f]; },
        [&](u32 f, u32 excl) {
          const u32 c = fcnt[f];
          u32 go = 0;
          if (c) go = atomicAdd(&cur2[d.x * g.nf + f], c);
          fgo[f] = go - excl;
          fcnt[f] = excl;
        });
#pragma unroll
    for (int q = 0; q < kBPer; ++q) {
      if (valid & (1u << q)) {
        const u32 p = fcnt[(a[q] >> kSlabBits) & (g.nf - 1)] + rank[q];
        st_a[p] = a[q];
        st_v[p] = v[q];
      }
    }
    __syncthreads();
    for (u32 p = tid; p < total; p += kATPB) {
      const u32 x = st_a[p];
      const u32 pos = fgo[(x >> kSlabBits) & (g.nf - 1)] + p;
      addr_out[pos] = x;
      val_out[pos] = st_v[p];
    }
    __syncthreads();
    for (u32 f = tid; f < g.nf; f += kATPB) fcnt[f] = 0;
    __syncthreads();
  }
}

// ---- slab apply ----------------------------------------------------------------------------------------
constexpr int kCRB = 4;  // records per thread per batch: loads issue together, then the LDS adds

// One work item = up to kCItem records of one slab: summed in LDS (A, a byte flag per touched
// element), then one coalesced read-modify-write of the touched pairs (exclusive items) or device
// atomics (items of a slab that was cut into several).
template <typename V>
__global__ __launch_bounds__(kATPB) void bin_apply_kernel(const u32* __restrict__ addr,
                                                          const typename LdsAcc<V>::T* __restrict__ val,
                                                          const uint4* __restrict__ cdesc, const BinCtl* bc, i64 elems,
                                                          V* __restrict__ data, u32 pre_min) {
  typedef typename Vec2<V>::T V2;
  typedef typename LdsAcc<V>::T A;
  __shared__ A acc[kSlab];
  __shared__ uint8_t touched[kSlab];  // plain byte stores: no atomic serialisation on hot elements
  constexpr int kPairsPerThread = kSlab / 2 / kATPB;
  const int tid = threadIdx.x;
  const u32 total = bc->nc_items;
  for (u32 it = blockIdx.x; it < total; it += gridDim.x) {
    const uint4 d4 = cdesc[it];
    const u32 slab = d4.x;
    const bool exclusive = d4.w != 0u;
    const u32 r_lo = d4.y, r_hi = d4.z;
    const i64 sbase_g = (i64)slab << kSlabBits;
    V* const sbase = data + sbase_g;
    // an item with many records touches most of the slab's lines: pull the slab into L2 now (one
    // dword per 128-B line), so the fetch overlaps the record phase and the RMW's loads hit
    const bool pre = exclusive && r_hi - r_lo >= pre_min;
    u32 warm = 0;
    if (pre) {
      constexpr int kLines = kSlab * (int)sizeof(V) / 128;
      constexpr int kPerLine = 128 / (int)sizeof(V);
      for (int l = tid; l < kLines; l += kATPB)
        if (sbase_g + (i64)l * kPerLine < elems) warm ^= *reinterpret_cast<const u32*>(sbase + (i64)l * kPerLine);
    }
    for (int e = tid; e < kSlab; e += kATPB) acc[e] = A(0);
    for (int w = tid; w < kSlab / 16; w += kATPB) reinterpret_cast<uint4*>(touched)[w] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    for (u32 j0 = r_lo; j0 < r_hi; j0 += (u32)kATPB * kCRB) {
      u32 ad[kCRB];
      A v[kCRB];
#pragma unroll
      for (int q = 0; q < kCRB; ++q) {  // clamped, branch-free loads
        const u32 j = j0 + q * kATPB + tid;
        const u32 jj = j < r_hi ? j : r_hi - 1;
        ad[q] = addr[jj];
        v[q] = val[jj];
        if (j >= r_hi) ad[q] = kEmptySlot;
      }
#pragma unroll
      for (int q = 0; q < kCRB; ++q) {
        if (ad[q] == kEmptySlot) continue;
        const u32 e = ad[q] & (kSlab - 1);
        lds_add(&acc[e], v[q]);
        touched[e] = 1;
      }
    }
    asm volatile("" ::"v"(warm));  // the warm-up loads complete here, after the record phase
    __syncthreads();
    if (exclusive) {
      // one coalesced RMW of the touched pairs; untouched lanes load the slab's first pair instead
      // (one cached line), so all loads issue back to back without a branch
      V2 dd[kPairsPerThread];
      u32 t[kPairsPerThread];
#pragma unroll
      for (int q = 0; q < kPairsPerThread; ++q) {
        const int e0 = 2 * (tid + q * kATPB);
        t[q] = (u32)touched[e0] | ((u32)touched[e0 + 1] << 1);
        const bool vec = t[q] != 0u && sbase_g + e0 + 1 < elems;
        dd[q] = *reinterpret_cast<const V2*>(vec ? sbase + e0 : sbase);
      }
#pragma unroll
      for (int q = 0; q < kPairsPerThread; ++q) {
        if (t[q] == 0u) continue;
        const int e0 = 2 * (tid + q * kATPB);
        if (sbase_g + e0 + 1 < elems) {
          V2 r = dd[q];
          if (t[q] & 1u) r.x = acc_add((V)r.x, acc[e0]);
          if (t[q] & 2u) r.y = acc_add((V)r.y, acc[e0 + 1]);
          *reinterpret_cast<V2*>(sbase + e0) = r;
        } else {  // the shard's last element, odd count
          sbase[e0] = acc_add(sbase[e0], acc[e0]);
        }
      }
    } else {
      for (int e = tid; e < kSlab; e += kATPB)
        if (touched[e]) gadd(sbase + e, (V)acc[e]);
    }
    __syncthreads();
  }
}

// ---- host side ----------------------------------------------------------------------------------------
// records per slab item from which bin_apply warms the whole slab into L2 (GLINT_BIN_PREFETCH_MIN;
// 0xFFFFFFFF disables)
u32 bin_prefetch_min() {
  static const u32 v = [] {
    const char* e = getenv("GLINT_BIN_PREFETCH_MIN");
    return e ? (u32)strtoul(e, nullptr, 10) : (u32)(kSlab / 4);
  }();
  return v;
}

BinGeom bin_geometry(i64 elems) {
  const i64 slabs = (elems + kSlab - 1) / kSlab;
  u32 sb = 0;
  while (((i64)1 << sb) < slabs) ++sb;
  // coarse bits: all of them up to 8; above that half (rounded up), so both digits stay <= 1024
  const u32 cb = sb <= 8 ? sb : std::max<u32>(8u, (sb + 1) / 2);
  BinGeom g;
  g.fb = sb - cb;
  g.nb = 1u << cb;
  g.nf = 1u << g.fb;
  g.nslab = g.nb * g.nf;
  return g;
}

template <typename V, bool MAT>
int push_binned(glint_shard* s, const PushArgs<V>& a, bool from_break, hipStream_t st) {
  typedef typename LdsAcc<V>::T A;
  const i64 n = a.n;
  if (n >= ((i64)1 << 32) - kAChunk || s->elems >= ((i64)1 << 32) - 1) return GLINT_EINVAL;  // u32 addresses
  const BinGeom g = bin_geometry(s->elems);
  // front end: dedup when the last probe kept < 60 % of the records (the device reports m and the
  // tail size of each push through a host-mapped word; read without a sync, so it may be one push
  // old); re-probe every 16 pushes. GLINT_BIN_FRONT = dedup | prep forces one (tests, tuning).
  if (s->h_hint) {
    const u64 w = __atomic_load_n(s->h_hint + 1, __ATOMIC_RELAXED);
    const u32 m = (u32)(w >> 32), tail = (u32)w;
    if (tail > 0 && s->bin_last_dedup) s->bin_dedup_ratio = (double)m / (double)tail;
  }
  bool dedup = s->bin_dedup_ratio < 0.6 || (++s->bin_pushes & 15) == 0;
  if (const char* e = getenv("GLINT_BIN_FRONT")) {
    if (!strcmp(e, "dedup")) dedup = true;
    else if (!strcmp(e, "prep")) dedup = false;
  }
  s->bin_last_dedup = dedup;
  const u32 ne = g.nb * kRegions;
  const i64 max_bitems = n / kBItem + ne + 1;
  const i64 max_citems = (i64)g.nslab + n / kCItem + 1;
  // zeroed block: [BinCtl | R | cur | H], then cap_off, cur2, bdesc, cdesc, record buffers
  const size_t b_ctl = 256, b_R = pad256((size_t)ne * 4), b_H = pad256((size_t)g.nslab * 4);
  const size_t b_zero = b_ctl + 2 * b_R + b_H;
  const size_t b_cap = pad256(((size_t)ne + 1) * 4);
  const size_t b_bd = pad256((size_t)max_bitems * 16), b_cd = pad256((size_t)max_citems * 16);
  const size_t b_a = pad256((size_t)n * 4), b_v = pad256((size_t)n * sizeof(A));
  const size_t need = b_zero + b_cap + b_H + b_bd + b_cd + 2 * (b_a + b_v);
  int rc = grow(&s->d_bin, &s->bin_bytes, need);
  if (rc) return rc;
  char* p = (char*)s->d_bin;
  BinCtl* bc = (BinCtl*)p;
  u32* R = (u32*)(p + b_ctl);
  u32* cur = (u32*)(p + b_ctl + b_R);
  u32* H = (u32*)(p + b_ctl + 2 * b_R);
  p += b_zero;
  u32* cap_off = (u32*)p;
  p += b_cap;
  u32* cur2 = (u32*)p;
  p += b_H;
  uint4* bdesc = (uint4*)p;
  p += b_bd;
  uint4* cdesc = (uint4*)p;
  p += b_cd;
  u32* addr_a = (u32*)p;
  A* val_a = (A*)(p + b_a);
  u32* addr_b = (u32*)(p + b_a + b_v);
  A* val_b = (A*)(p + 2 * b_a + b_v);

  ProfScope ps(s, GLINT_K_PUSH_BINNED, st);
  HIPCHK(hipMemsetAsync(s->d_bin, 0, b_zero, st));
  const i64 nchunks = (n + kAChunk - 1) / kAChunk;
  auto grid8 = [](i64 want, i64 cap) {  // a multiple of kRegions (chunk c -> region c % 8)
    i64 g8 = std::min(want, cap);
    g8 = (g8 + kRegions - 1) / kRegions * kRegions;
    return (unsigned)std::max<i64>(g8, kRegions);
  };
  const int fb = from_break ? 1 : 0;
  bin_count_kernel<MAT><<<grid8(nchunks, (i64)s->cus * 4), kATPB, 0, st>>>(a.keys, a.cols, n, a.part, a.ctl, a.ntiles,
                                                                           fb, g, R, cap_off, bc);
  HIPCHK(hipGetLastError());
  if (dedup) {
    bin_part_dedup_kernel<V, MAT><<<grid8(nchunks, (i64)s->cus * 2), kATPB, 0, st>>>(
        a.keys, a.cols, a.vals, n, a.part, a.ctl, a.ntiles, fb, g, cap_off, cur, addr_a, val_a, a.err);
  } else {
    bin_part_kernel<V, MAT><<<grid8(nchunks, (i64)s->cus * 4), kATPB, 0, st>>>(
        a.keys, a.cols, a.vals, n, a.part, a.ctl, a.ntiles, fb, g, cap_off, cur, addr_a, val_a, a.err);
  }
  HIPCHK(hipGetLastError());
  bin_bitems_kernel<<<1, kATPB, 0, st>>>(g, cap_off, cur, bdesc, bc, s->d_hint ? s->d_hint + 1 : nullptr);
  HIPCHK(hipGetLastError());
  const unsigned gb = (unsigned)std::min<i64>(max_bitems, (i64)s->cus * 8);
  bin_fhist_kernel<<<gb, kATPB, 0, st>>>(g, bdesc, bc, addr_a, H);
  HIPCHK(hipGetLastError());
  bin_cscan_kernel<<<1, kScanTPB, 0, st>>>(g, H, cur2, cdesc, bc);
  HIPCHK(hipGetLastError());
  bin_fpart_kernel<A><<<gb, kATPB, 0, st>>>(g, bdesc, bc, addr_a, val_a, cur2, addr_b, val_b);
  HIPCHK(hipGetLastError());
  static const int apply_bpc = [] {  // GLINT_BIN_APPLY_BPC: work-item blocks per CU (tuning knob)
    const char* e = getenv("GLINT_BIN_APPLY_BPC");
    return (e && atoi(e) > 0) ? atoi(e) : 64;
  }();
  bin_apply_kernel<V><<<(unsigned)std::min<i64>(max_citems, (i64)s->cus * apply_bpc), kATPB, 0, st>>>(
      addr_b, val_b, cdesc, bc, s->elems, a.data, bin_prefetch_min());
  HIPCHK(hipGetLastError());
  return GLINT_OK;
}

#define GLINT_INST(V, MAT) template int push_binned<V, MAT>(glint_shard*, const PushArgs<V>&, bool, hipStream_t);
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
