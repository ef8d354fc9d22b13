// glint_page.hip -- the binned push, paged: large unordered pushes summed per shard slab in LDS with
// every intermediate store a whole line. PartialVector.update / PartialMatrix.update
// (src/main/scala/glint/models/server/PartialVector.scala:35-43, PartialMatrix.scala:74-83) for
// records in no particular order.
//
// A slab is 4096 consecutive shard elements (one workgroup sums it in LDS). Records reach slab order
// through at most two partition levels of at most 256 buckets each -- the coarse digit, then the
// slab within its bucket -- and both levels write PAGES: 32 records (32 addresses = one 128-B line,
// 32 values = two lines) that are filled in LDS and stored once complete. A workgroup keeps one open
// page per bucket across its chunks, so what it stores is whole pages -- every line written in one
// short window, merged in L2 -- however its records spread; only each (workgroup, bucket) pair's last
// page is partial. Pages come from a private pool per workgroup, so nothing is counted or reserved
// across workgroups beforehand:
//
//   pg_part<1>   per workgroup: a contiguous range of the push's records, checked and turned into
//                element addresses, (optionally) summed per 2048-record chunk in an LDS hash table,
//                then paged by coarse bucket. At the end the workgroup sorts its page list by bucket
//                (stable), so bucket b's pages are one run per workgroup: seg[b][w] = (first
//                directory entry, pages, records of the last page).
//   pg_plan      one workgroup: pages per bucket, and the fine items -- each bucket's page list cut
//                into pieces of at most 512 pages (16384 records).
//   pg_part<2>   per fine item: its pages paged again by slab within the bucket -> seg[i][d].
//   pg_apply     per slab: its pages (one run per fine item of its bucket) summed in LDS, then one
//                read-modify-write of the touched element pairs. A slab with more records than one
//                workgroup should take is queued for pg_apply_hot, which splits it over workgroups
//                that flush their partial sums with device atomics.
// Every size stays on the device (no host round trip).
#include "glint_device.h"
#include "glint_host.h"

#include <atomic>
#include <cstring>

namespace glint {

constexpr int kPgSlabBits = 12;
constexpr int kPgSlab = 1 << kPgSlabBits;
constexpr int kPage = 32;             // records per page
constexpr int kPgDigit = 256;         // buckets per partition level, at most
constexpr int kPT = 512;              // partition workgroup size (1024 spills at its 128-VGPR budget)
constexpr int kPW = kPT / 64;         // its waves
constexpr int kPPer = 4;              // records per thread per batch
constexpr int kPChunk = kPT * kPPer;  // 2048 records (64 pages) per batch
constexpr int kPSlots = 2 * kPChunk;  // dedup hash slots (load <= 0.5)
constexpr int kPSlotBits = 12;
static_assert((1 << kPSlotBits) == kPSlots, "dedup table size");
constexpr u32 kFItemPages = 512;      // pages per fine item at most (16384 records)
constexpr int kPgMaxG = 256;          // level-1 workgroups at most
constexpr int kAT = 256;              // apply workgroup size
constexpr int kAPer = 4;              // records per thread per apply round: kAT * kAPer = 32 pages
constexpr int kAPages = kAT * kAPer / kPage;
constexpr int kMaxPieces = 256;       // runs of pages per slab one apply workgroup takes
constexpr u32 kPgHot = 1u << 18;      // records of one slab above which pg_apply_hot splits it
constexpr u32 kEmptyA = 0xFFFFFFFFu;

// Page p of a pool: [32 addresses (u32) | 32 values (A)] = 128 + 32 * sizeof(A) bytes, line-aligned.
template <typename A> __host__ __device__ constexpr size_t page_bytes() { return 128 + kPage * sizeof(A); }
template <typename A> __device__ __forceinline__ u32* pg_a(char* pool, u32 p) {
  return reinterpret_cast<u32*>(pool + (size_t)p * page_bytes<A>());
}
template <typename A> __device__ __forceinline__ A* pg_v(char* pool, u32 p) {
  return reinterpret_cast<A*>(pool + (size_t)p * page_bytes<A>() + 128);
}

// digit of an element address at one level: (a >> shift) & (nd - 1), nd a power of two <= 256
struct PgLevel {
  u32 shift, nd;
  __device__ __forceinline__ u32 digit(u32 a) const { return (a >> shift) & (nd - 1); }
};

struct PgCtl {
  u32 m;       // records level 1 emitted (after dedup)
  u32 tail;    // valid records of the tail
  u32 nitems;  // fine items (pg_plan)
  u32 nhot;    // hot slabs queued for pg_apply_hot
};

// Where a level's output pages are: directory entries (pool page ids) grouped by digit, one run per
// producing work item; run (item i, digit d) at index i * nd + d (level 2) or d * G + i (level 1).
struct PgSegs {
  u32* off;   // first directory entry of the run
  u32* np;    // pages in the run
  u32* last;  // records in its last page (1..32)
};

__device__ __forceinline__ i64 pg_tail_start(const LaunchCtl* lctl, u32 ntiles, int from_break, i64 n) {
  if (!from_break) return 0;
  const u32 brk = lctl->brk_enc;  // written by push_check; ordered by the kernel boundary
  return brk == 0u ? n : (i64)(ntiles - brk) * kTile;
}

// Exclusive scan of one value per thread of a kPT workgroup; returns the total.
__device__ __forceinline__ u32 pg_scan(u32 v, u32& excl, u32* wt) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  u32 incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const u32 y = __shfl_up(incl, d);
    if (lane >= d) incl += y;
  }
  if (lane == 63) wt[wid] = incl;
  __syncthreads();
  u32 run = incl - v, tot = 0;
#pragma unroll
  for (int w = 0; w < kPW; ++w) {
    const u32 x = wt[w];
    run += w < wid ? x : 0u;
    tot += x;
  }
  __syncthreads();
  excl = run;
  return tot;
}

// the lanes of this wave whose digit equals this lane's (digits < 2^nbits): one ballot per bit
__device__ __forceinline__ u64 pg_match(u32 d, int nbits) {
  u64 m = ~0ull;
  for (int k = 0; k < nbits; ++k) {
    const bool bit = (d >> k) & 1u;
    const u64 b = __ballot(bit);
    m &= bit ? b : ~b;
  }
  return m;
}

// ---- the partition workgroup's LDS --------------------------------------------------------------------
template <typename A>
struct PgLds {
  u32 buf_a[kPgDigit * kPage];  // the open page of each bucket
  A buf_v[kPgDigit * kPage];
  u32 fill[kPgDigit];   // records in the open page
  u32 npg[kPgDigit];    // pages completed (the level's output)
  u32 cnt[kPgDigit];    // this batch: records per bucket (zero between batches)
  u32 runp[kPgDigit];   // this batch: staging run start
  u32 pg0[kPgDigit];    // this batch: first page id it completes
  u32 nfull[kPgDigit];  // this batch: pages it completes
  u32 wt[kPW];
  u32 nused;
  u32 segpre[kPgMaxG + 1];  // level 2: the bucket's runs of input pages (page prefix, directory
  u32 segst[kPgMaxG];       //          offset, records of the last page)
  u32 segl[kPgMaxG];
  union {
    struct {  // the batch's dedup table
      u32 hk[kPSlots];
      A hv[kPSlots];
    } h;
    struct {  // the batch in staging order (grouped by bucket)
      A st_v[kPChunk];
      u32 st_a[kPChunk];
    } s;
    u32 hist[kPW * kPgDigit];  // end: per-wave page counts of the directory sort
  } u;
  uint16_t used[kPChunk];  // dedup: the slots claimed this batch
};

// Places one batch of entries (up to kPPer per thread: ad[j], va[j], bit j of `valid`) into the open
// pages; completed pages go to the workgroup's pool. `npages` = pages this workgroup has completed.
template <typename A>
__device__ __forceinline__ void pg_place(PgLds<A>& L, const PgLevel lv, const u32 (&ad)[kPPer], const A (&va)[kPPer],
                                         u32 valid, char* pool, u32 pbase, u32* __restrict__ dig, u32& npages) {
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  u32 rank[kPPer];
#pragma unroll
  for (int j = 0; j < kPPer; ++j)
    if (valid & (1u << j)) rank[j] = atomicAdd(&L.cnt[lv.digit(ad[j])], 1u);
  __syncthreads();
  // per bucket: its run in the staging order, and the pages this batch completes (ids from the pool)
  u32 c = 0, f = 0, full = 0;
  if (tid < (int)lv.nd) {
    c = L.cnt[tid];
    f = L.fill[tid];
    full = (f + c) >> 5;
  }
  u32 excl;
  const u32 tot = pg_scan(c | (full << 16), excl, L.wt);
  const u32 nent = tot & 0xFFFFu, newpages = tot >> 16;
  if (tid < (int)lv.nd) {
    L.runp[tid] = excl & 0xFFFFu;
    L.pg0[tid] = npages + (excl >> 16);
    L.nfull[tid] = full;
    L.npg[tid] += full;
    for (u32 k = 0; k < full; ++k) dig[pbase + npages + (excl >> 16) + k] = (u32)tid;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kPPer; ++j) {
    if (valid & (1u << j)) {
      const u32 p = L.runp[lv.digit(ad[j])] + rank[j];
      L.u.s.st_a[p] = ad[j];
      L.u.s.st_v[p] = va[j];
    }
  }
  __syncthreads();
  // staging position p -> slot (fill + index within its run) of the bucket's page stream: page 0 is
  // the open page (completed into LDS and flushed below), pages 1.. of a completing batch are written
  // straight to the pool, and the records of the last, partial page wait until the flush has read
  // the open page
  u32 dfr_slot[kPPer], dfr_a[kPPer];
  A dfr_v[kPPer];
  u32 dfr = 0;
#pragma unroll
  for (int j = 0; j < kPPer; ++j) {
    const u32 p = (u32)tid + (u32)j * kPT;
    if (p >= nent) break;
    const u32 a = L.u.s.st_a[p];
    const A v = L.u.s.st_v[p];
    const u32 d = lv.digit(a);
    const u32 vv = L.fill[d] + (p - L.runp[d]);
    const u32 pj = vv >> 5, slot = vv & 31u, nf = L.nfull[d];
    if (pj == 0 && nf > 0) {
      L.buf_a[d * kPage + slot] = a;
      L.buf_v[d * kPage + slot] = v;
    } else if (pj < nf) {
      const u32 page = pbase + L.pg0[d] + pj;
      pg_a<A>(pool, page)[slot] = a;
      pg_v<A>(pool, page)[slot] = v;
    } else if (nf == 0) {  // the open page is not completed: the record extends it in place
      L.buf_a[d * kPage + slot] = a;
      L.buf_v[d * kPage + slot] = v;
    } else {
      dfr_slot[j] = d * kPage + slot;
      dfr_a[j] = a;
      dfr_v[j] = v;
      dfr |= 1u << j;
    }
  }
  __syncthreads();
  // flush the completed open pages: one wave per bucket, 32 addresses and 32 values
  for (u32 d = (u32)wid; d < lv.nd; d += kPW) {
    if (L.nfull[d] == 0) continue;
    const u32 page = pbase + L.pg0[d];
    if (lane < kPage) {
      pg_a<A>(pool, page)[lane] = L.buf_a[d * kPage + lane];
      pg_v<A>(pool, page)[lane] = L.buf_v[d * kPage + lane];
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kPPer; ++j) {
    if (dfr & (1u << j)) {
      L.buf_a[dfr_slot[j]] = dfr_a[j];
      L.buf_v[dfr_slot[j]] = dfr_v[j];
    }
  }
  if (tid < (int)lv.nd) {
    L.fill[tid] = (f + c) & 31u;
    L.cnt[tid] = 0;
  }
  npages += newpages;
  __syncthreads();
}

// End of a partition workgroup: the partial open pages go to the pool, then the workgroup's pages are
// sorted by bucket (stable: each wave owns a contiguous range of page ids) into the directory, and
// each bucket's run is published.
template <typename A>
__device__ __forceinline__ void pg_finish(PgLds<A>& L, const PgLevel lv, char* pool, u32 pbase, u32* __restrict__ dig,
                                          u32* __restrict__ dir, u32 npages, PgSegs out, u32 seg_base,
                                          u32 seg_stride) {
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const u32 nd = lv.nd;
  const u32 f = tid < (int)nd ? L.fill[tid] : 0u;
  u32 excl;
  const u32 npart = pg_scan(f > 0 ? 1u : 0u, excl, L.wt);
  if (tid < (int)nd) {
    L.pg0[tid] = npages + excl;  // the partial page's id (if any)
    if (f > 0) {
      dig[pbase + npages + excl] = (u32)tid;
      L.npg[tid] += 1;
    }
  }
  __syncthreads();
  for (u32 d = (u32)wid; d < nd; d += kPW) {
    const u32 fd = L.fill[d];
    if (fd == 0) continue;
    const u32 page = pbase + L.pg0[d];
    if (lane < (int)fd) {
      pg_a<A>(pool, page)[lane] = L.buf_a[d * kPage + lane];
      pg_v<A>(pool, page)[lane] = L.buf_v[d * kPage + lane];
    }
  }
  const u32 P = npages + npart;
  // the page -> bucket map was written by this workgroup's own stores: drain them, then read it back
  // past L1
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __syncthreads();
  const int nbits = 32 - __clz((int)nd);  // digits and the sentinel nd fit
  const u32 per = (P + kPW - 1) / kPW;
  const u32 p0 = min(P, (u32)wid * per), p1 = min(P, p0 + per);
  u32* hw = L.u.hist + wid * kPgDigit;
  for (u32 d = lane; d < nd; d += 64) hw[d] = 0;
  for (u32 b = p0; b < p1; b += 64) {
    const u32 p = b + (u32)lane;
    const u32 d = p < p1 ? __hip_atomic_load(dig + pbase + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : nd;
    const u64 m = pg_match(d, nbits);
    if (d < nd && (m & ((1ull << lane) - 1)) == 0) hw[d] += (u32)__popcll(m);
  }
  __syncthreads();
  // exclusive scan over (bucket, wave), bucket-major: the first directory slot of each
  const int per_t = kPW * kPgDigit / kPT;  // 4
  u32 v[per_t], s = 0;
#pragma unroll
  for (int k = 0; k < per_t; ++k) {
    const u32 i = (u32)tid * per_t + k;  // bucket i / kPW, wave i % kPW
    v[k] = (i / kPW) < nd ? L.u.hist[(i % kPW) * kPgDigit + i / kPW] : 0u;
    s += v[k];
  }
  u32 ex;
  pg_scan(s, ex, L.wt);
#pragma unroll
  for (int k = 0; k < per_t; ++k) {
    const u32 i = (u32)tid * per_t + k;
    if ((i / kPW) < nd) {
      if (i % kPW == 0) {
        const u32 d = i / kPW;
        out.off[seg_base + d * seg_stride] = pbase + ex;
        out.np[seg_base + d * seg_stride] = L.npg[d];
        out.last[seg_base + d * seg_stride] = L.fill[d] ? L.fill[d] : (L.npg[d] ? (u32)kPage : 0u);
      }
      L.u.hist[(i % kPW) * kPgDigit + i / kPW] = ex;
    }
    ex += v[k];
  }
  __syncthreads();
  for (u32 b = p0; b < p1; b += 64) {
    const u32 p = b + (u32)lane;
    const u32 d = p < p1 ? __hip_atomic_load(dig + pbase + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : nd;
    const u64 m = pg_match(d, nbits);
    if (d < nd) {
      const u64 below = m & ((1ull << lane) - 1);
      dir[pbase + hw[d] + (u32)__popcll(below)] = pbase + p;
      if (below == 0) hw[d] += (u32)__popcll(m);  // the group's lowest lane advances the cursor
    }
  }
}

// ---- level 1: the push's records -> pages by coarse bucket ----------------------------------------------
template <typename V, bool MAT>
struct PgIn {
  i64 k[kPPer];
  int32_t c[kPPer];
  V v[kPPer];
};

template <typename V, bool MAT>
__device__ __forceinline__ void pg_load(const i64* __restrict__ keys, const int32_t* __restrict__ cols,
                                        const V* __restrict__ vals, i64 c0, i64 c1, PgIn<V, MAT>& r) {
#pragma unroll
  for (int q = 0; q < kPPer; ++q) {  // clamped, branch-free loads
    const i64 i = c0 + q * kPT + threadIdx.x;
    const i64 ii = i < c1 ? i : c1 - 1;
    r.k[q] = keys[ii];
    r.c[q] = MAT ? cols[ii] : 0;
    r.v[q] = vals[ii];
  }
}

template <typename V, bool MAT, bool DEDUP>
__global__ __launch_bounds__(kPT) void pg_part1_kernel(const i64* __restrict__ keys, const int32_t* __restrict__ cols,
                                                       const V* __restrict__ vals, i64 n, PartDesc part,
                                                       const LaunchCtl* lctl, u32 ntiles, int from_break, PgLevel lv,
                                                       char* pool, u32 PW, u32* __restrict__ dig,
                                                       u32* __restrict__ dir, PgSegs out, ErrState* err, PgCtl* pc) {
  typedef typename LdsAcc<V>::T A;
  __shared__ PgLds<A> L;
  const int tid = threadIdx.x, lane = tid & 63;
  const u32 w = blockIdx.x, G = gridDim.x;
  const i64 r0 = pg_tail_start(lctl, ntiles, from_break, n);
  const i64 nchunks = (n - r0 + kPChunk - 1) / kPChunk;
  // contiguous chunk ranges (the pages of a bucket, workgroup after workgroup, are in push order)
  const i64 q = nchunks / G, rm = nchunks % G;
  const i64 cb = (i64)w * q + min((i64)w, rm), ce = cb + q + ((i64)w < rm ? 1 : 0);
  const u32 pbase = w * PW;
  for (u32 d = tid; d < (u32)kPgDigit; d += kPT) {
    L.fill[d] = 0;
    L.npg[d] = 0;
    L.cnt[d] = 0;
  }
  if (DEDUP)
    for (int sl = tid; sl < kPSlots; sl += kPT) {
      L.u.h.hk[sl] = kEmptyA;
      L.u.h.hv[sl] = A(0);
    }
  if (tid == 0) L.nused = 0;
  __syncthreads();
  const u64 below = (1ull << lane) - 1ull;
  u32 npages = 0, emitted = 0, nvalid = 0;
  i64 bad_first = -1;
  u32 bad_count = 0;
  PgIn<V, MAT> ra, rb;
  auto load = [&](i64 c, PgIn<V, MAT>& r) {
    const i64 cc = min(c, ce - 1);
    pg_load<V, MAT>(keys, cols, vals, r0 + cc * kPChunk, min(n, r0 + (cc + 1) * kPChunk), r);
  };
  auto step = [&](i64 c, PgIn<V, MAT>& r) {
    const i64 c0 = r0 + c * kPChunk, c1 = c < ce ? min(n, c0 + kPChunk) : c0;
    u32 ad[kPPer];
    A va[kPPer];
    u32 valid = 0;
#pragma unroll
    for (int j = 0; j < kPPer; ++j) {
      const i64 i = c0 + j * kPT + tid;
      i64 a64;
      ad[j] = 0;
      va[j] = (A)r.v[j];
      if (i < c1) {
        if (rec_addr<MAT>(part, r.k[j], r.c[j], a64)) {
          ad[j] = (u32)a64;
          valid |= 1u << j;
        } else {
          bad_first = bad_count ? min(bad_first, i) : i;
          ++bad_count;
        }
      }
    }
    nvalid += (u32)__popc(valid);
    load(c + 2, r);  // two chunks ahead, into the registers just consumed
    if (DEDUP) {
      // equal elements of the batch summed in the hash table: one entry per distinct element moves on
#pragma unroll
      for (int j = 0; j < kPPer; ++j) {
        bool claimed = false;
        u32 h = 0;
        if (valid & (1u << j)) {
          h = (ad[j] * 0x9E3779B1u) >> (32 - kPSlotBits);
          for (;;) {
            const u32 prev = atomicCAS(&L.u.h.hk[h], kEmptyA, ad[j]);
            if (prev == kEmptyA) { claimed = true; break; }
            if (prev == ad[j]) break;
            h = (h + 1) & (kPSlots - 1);
          }
          lds_add(&L.u.h.hv[h], va[j]);
        }
        const u64 b = __ballot(claimed);
        if (b) {
          u32 base = 0;
          if (lane == 0) base = atomicAdd(&L.nused, (u32)__popcll(b));
          base = __shfl(base, 0);
          if (claimed) L.used[base + (u32)__popcll(b & below)] = (uint16_t)h;
        }
      }
      __syncthreads();
      const u32 D = L.nused;
      valid = 0;
#pragma unroll
      for (int j = 0; j < kPPer; ++j) {
        const u32 e = tid + j * kPT;
        if (e < D) {
          const u32 sl = L.used[e];
          ad[j] = L.u.h.hk[sl];
          va[j] = L.u.h.hv[sl];
          valid |= 1u << j;
        }
      }
      __syncthreads();
      if (tid == 0) L.nused = 0;
    }
    emitted += (u32)__popc(valid);
    pg_place<A>(L, lv, ad, va, valid, pool, pbase, dig, npages);
    if (DEDUP) {  // the staging overlaid the table: reset it for the next batch
      for (int sl = tid; sl < kPSlots; sl += kPT) {
        L.u.h.hk[sl] = kEmptyA;
        L.u.h.hv[sl] = A(0);
      }
      __syncthreads();
    }
  };
  if (cb < ce) {
    load(cb, ra);
    load(cb + 1, rb);
    for (i64 c = cb; c < ce; c += 2) {
      step(c, ra);
      step(c + 1, rb);  // past the end: no valid record, nothing placed
    }
  }
  pg_finish<A>(L, lv, pool, pbase, dig, dir, npages, out, w, G);
  if (bad_count) {
    atomicMax(&err->min_bad_enc, ~(u64)bad_first);
    atomicAdd(&err->count, (unsigned long long)bad_count);
  }
  // totals for the host's next binned push (the dedup decision)
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    emitted += __shfl_xor(emitted, d);
    nvalid += __shfl_xor(nvalid, d);
  }
  if (lane == 0) {
    if (emitted) atomicAdd(&pc->m, emitted);
    if (nvalid) atomicAdd(&pc->tail, nvalid);
  }
}

// ---- plan: fine items ------------------------------------------------------------------------------------
// One workgroup. Bucket b's pages (level 1: the runs seg[b][w], w < G) are cut into items of at most
// kFItemPages pages; ib0[b] = its first item, items[i] = {b, first page, end page} in run order.
__global__ __launch_bounds__(kPT) void pg_plan_kernel(PgLevel lv1, u32 G, PgSegs s1, uint4* __restrict__ items,
                                                      u32* __restrict__ ib0, PgCtl* pc, u64* hint) {
  __shared__ u32 wt[kPW];
  const int tid = threadIdx.x;
  u32 pages = 0;
  if (tid < (int)lv1.nd)
    for (u32 w = 0; w < G; ++w) pages += s1.np[tid * G + w];
  const u32 J = tid < (int)lv1.nd ? max(1u, (pages + kFItemPages - 1) / kFItemPages) : 0u;
  u32 excl;
  const u32 tot = pg_scan(J, excl, wt);
  if (tid < (int)lv1.nd) {
    ib0[tid] = excl;
    for (u32 j = 0; j < J; ++j)
      items[excl + j] = make_uint4((u32)tid, j * kFItemPages, min(pages, (j + 1) * kFItemPages), 0u);
  }
  if (tid == 0) {
    ib0[lv1.nd] = tot;
    pc->nitems = tot;
    if (hint)  // for the host's next binned push: how much did dedup keep?
      __hip_atomic_store(hint, ((u64)pc->m << 32) | (u64)pc->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---- level 2: a bucket's pages -> pages by slab -----------------------------------------------------------
template <typename A, bool DEDUP>
__global__ __launch_bounds__(kPT) void pg_part2_kernel(PgLevel lv, u32 G, const uint4* __restrict__ items,
                                                       const PgCtl* pc, PgSegs s1, const u32* __restrict__ dir1,
                                                       char* pool1, char* pool, u32 PW, u32* __restrict__ dig,
                                                       u32* __restrict__ dir, PgSegs out) {
  __shared__ PgLds<A> L;
  const int tid = threadIdx.x, lane = tid & 63;
  const u64 below = (1ull << lane) - 1ull;
  const u32 nit = pc->nitems;
  for (u32 it = blockIdx.x; it < nit; it += gridDim.x) {
    const uint4 d4 = items[it];
    const u32 b = d4.x, k0 = d4.y, k1 = d4.z;
    const u32 pbase = it * PW;
    for (u32 d = tid; d < (u32)kPgDigit; d += kPT) {
      L.fill[d] = 0;
      L.npg[d] = 0;
      L.cnt[d] = 0;
    }
    // the bucket's runs of level-1 pages
    {
      const u32 np = tid < (int)G ? s1.np[b * G + tid] : 0u;
      u32 excl;
      const u32 tot = pg_scan(np, excl, L.wt);
      if (tid < (int)G) {
        L.segpre[tid] = excl;
        L.segst[tid] = s1.off[b * G + tid];
        L.segl[tid] = s1.last[b * G + tid];
      }
      if (tid == 0) {
        L.segpre[G] = tot;
        L.nused = 0;
      }
    }
    if (DEDUP)
      for (int sl = tid; sl < kPSlots; sl += kPT) {
        L.u.h.hk[sl] = kEmptyA;
        L.u.h.hv[sl] = A(0);
      }
    __syncthreads();
    u32 npages = 0;
    u32 s = 0;  // this thread's run cursor (its pages only move forward)
    for (u32 t0 = k0; t0 < k1; t0 += kPChunk / kPage) {
      u32 ad[kPPer];
      A va[kPPer];
      u32 valid = 0;
#pragma unroll
      for (int j = 0; j < kPPer; ++j) {
        const u32 qq = (u32)tid + (u32)j * kPT;
        const u32 k = t0 + (qq >> 5), slot = qq & 31u;
        ad[j] = 0;
        va[j] = A(0);
        if (k < k1) {
          while (L.segpre[s + 1] <= k) ++s;
          const u32 within = k - L.segpre[s];
          const u32 page = dir1[L.segst[s] + within];
          const u32 cntp = within + 1 == L.segpre[s + 1] - L.segpre[s] ? L.segl[s] : (u32)kPage;
          if (slot < cntp) {
            ad[j] = pg_a<A>(pool1, page)[slot];
            va[j] = pg_v<A>(pool1, page)[slot];
            valid |= 1u << j;
          }
        }
      }
      if (DEDUP) {
#pragma unroll
        for (int j = 0; j < kPPer; ++j) {
          bool claimed = false;
          u32 h = 0;
          if (valid & (1u << j)) {
            h = (ad[j] * 0x9E3779B1u) >> (32 - kPSlotBits);
            for (;;) {
              const u32 prev = atomicCAS(&L.u.h.hk[h], kEmptyA, ad[j]);
              if (prev == kEmptyA) { claimed = true; break; }
              if (prev == ad[j]) break;
              h = (h + 1) & (kPSlots - 1);
            }
            lds_add(&L.u.h.hv[h], va[j]);
          }
          const u64 bb = __ballot(claimed);
          if (bb) {
            u32 base = 0;
            if (lane == 0) base = atomicAdd(&L.nused, (u32)__popcll(bb));
            base = __shfl(base, 0);
            if (claimed) L.used[base + (u32)__popcll(bb & below)] = (uint16_t)h;
          }
        }
        __syncthreads();
        const u32 D = L.nused;
        valid = 0;
#pragma unroll
        for (int j = 0; j < kPPer; ++j) {
          const u32 e = tid + j * kPT;
          if (e < D) {
            const u32 sl = L.used[e];
            ad[j] = L.u.h.hk[sl];
            va[j] = L.u.h.hv[sl];
            valid |= 1u << j;
          }
        }
        __syncthreads();
        if (tid == 0) L.nused = 0;
      }
      pg_place<A>(L, lv, ad, va, valid, pool, pbase, dig, npages);
      if (DEDUP) {
        for (int sl = tid; sl < kPSlots; sl += kPT) {
          L.u.h.hk[sl] = kEmptyA;
          L.u.h.hv[sl] = A(0);
        }
        __syncthreads();
      }
    }
    pg_finish<A>(L, lv, pool, pbase, dig, dir, npages, out, it * lv.nd, 1);
    __syncthreads();
  }
}

// ---- apply ------------------------------------------------------------------------------------------------
// The runs of pages of slab s: level 2 -> one per fine item of its bucket (index i * nd2 + d); one level
// -> one per level-1 workgroup (index s * G + w).
struct PgSlabRuns {
  u32 base, stride, count;
};
__device__ __forceinline__ PgSlabRuns pg_runs_of(u32 s, bool two, u32 fbits, u32 nd2, u32 G,
                                                 const u32* __restrict__ ib0) {
  if (!two) return PgSlabRuns{s * G, 1u, G};
  const u32 b = s >> fbits, d = s & (nd2 - 1);
  const u32 i0 = ib0[b], i1 = ib0[b + 1];
  return PgSlabRuns{i0 * nd2 + d, nd2, i1 - i0};
}

template <typename V>
__global__ __launch_bounds__(kAT) void pg_apply_kernel(PgSegs sg, const u32* __restrict__ dir, char* pool,
                                                       const u32* __restrict__ ib0, u32 nslab, int two, u32 fbits,
                                                       u32 nd2, u32 G, i64 elems, V* __restrict__ data,
                                                       u32* __restrict__ hot, PgCtl* pc, u32 pre_min, u64* hint) {
  typedef typename Vec2<V>::T V2;
  typedef typename LdsAcc<V>::T A;
  __shared__ A acc[kPgSlab];
  __shared__ uint8_t touched[kPgSlab];
  __shared__ u32 rpre[kMaxPieces + 1], rst[kMaxPieces], rl[kMaxPieces];
  __shared__ u32 wt4[kAT / 64];
  constexpr int kPairsPerThread = kPgSlab / 2 / kAT;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (hint && blockIdx.x == 0 && tid == 0)  // one level (no plan kernel): the dedup hint from here
    __hip_atomic_store(hint, ((u64)pc->m << 32) | (u64)pc->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (int e = tid; e < kPgSlab; e += kAT) acc[e] = A(0);
  for (int e = tid; e < kPgSlab / 16; e += kAT) reinterpret_cast<uint4*>(touched)[e] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  for (u32 s = blockIdx.x; s < nslab; s += gridDim.x) {
    const PgSlabRuns R = pg_runs_of(s, two != 0, fbits, nd2, G, ib0);
    if (R.count > (u32)kMaxPieces) {  // too many runs for this workgroup's table: split it instead
      if (tid == 0) hot[atomicAdd(&pc->nhot, 1u)] = s;
      continue;
    }
    // the slab's runs: page prefix, directory offset, records of the last page
    u32 np = 0, recs = 0;
    if (tid < (int)R.count) {
      const u32 ix = R.base + (u32)tid * R.stride;
      np = sg.np[ix];
      rst[tid] = sg.off[ix];
      rl[tid] = sg.last[ix];
      recs = np ? (np - 1) * kPage + sg.last[ix] : 0u;
    }
    // block scan of np over kAT threads
    u32 incl = np;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const u32 y = __shfl_up(incl, d);
      if (lane >= d) incl += y;
    }
    u32 rsum = recs;
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) rsum += __shfl_xor(rsum, d);
    if (lane == 63) wt4[wid] = incl;
    __syncthreads();
    u32 ex = incl - np, P = 0;
#pragma unroll
    for (int w = 0; w < kAT / 64; ++w) {
      ex += w < wid ? wt4[w] : 0u;
      P += wt4[w];
    }
    if (tid < (int)R.count) rpre[tid] = ex;
    if (tid == 0) rpre[R.count] = P;
    __syncthreads();
    if (lane == 0) wt4[wid] = rsum;
    __syncthreads();
    const u32 total = wt4[0] + wt4[1] + wt4[2] + wt4[3];
    __syncthreads();
    if (total == 0) continue;
    if (total > kPgHot) {
      if (tid == 0) hot[atomicAdd(&pc->nhot, 1u)] = s;
      continue;
    }
    const i64 sbase_g = (i64)s << kPgSlabBits;
    V* const sbase = data + sbase_g;
    u32 warm = 0;
    if (total >= pre_min) {  // most lines will be touched: pull the slab into L2 meanwhile
      constexpr int kLines = kPgSlab * (int)sizeof(V) / 128;
      constexpr int kPerLine = 128 / (int)sizeof(V);
      for (int l = tid; l < kLines; l += kAT)
        if (sbase_g + (i64)l * kPerLine < elems) warm ^= *reinterpret_cast<const u32*>(sbase + (i64)l * kPerLine);
    }
    u32 r = 0;  // this thread's run cursor
    for (u32 g0 = 0; g0 < P; g0 += kAPages) {
      u32 ca[kAPer];
      A cv[kAPer];
#pragma unroll
      for (int j = 0; j < kAPer; ++j) {
        const u32 qq = (u32)tid + (u32)j * kAT;
        const u32 g = g0 + (qq >> 5), slot = qq & 31u;
        ca[j] = kEmptyA;
        cv[j] = A(0);
        if (g < P) {
          while (rpre[r + 1] <= g) ++r;
          const u32 within = g - rpre[r];
          const u32 page = dir[rst[r] + within];
          const u32 cntp = within + 1 == rpre[r + 1] - rpre[r] ? rl[r] : (u32)kPage;
          if (slot < cntp) {
            ca[j] = pg_a<A>(pool, page)[slot];
            cv[j] = pg_v<A>(pool, page)[slot];
          }
        }
      }
#pragma unroll
      for (int j = 0; j < kAPer; ++j) {
        if (ca[j] == kEmptyA) continue;
        const u32 e = ca[j] & (kPgSlab - 1);
        lds_add(&acc[e], cv[j]);
        touched[e] = 1;
      }
    }
    asm volatile("" ::"v"(warm));
    __syncthreads();
    // one coalesced read-modify-write of the touched pairs; untouched lanes load the slab's first
    // pair instead (one cached line), so all loads issue back to back
    V2 dd[kPairsPerThread];
    u32 t[kPairsPerThread];
#pragma unroll
    for (int qd = 0; qd < kPairsPerThread; ++qd) {
      const int e0 = 2 * (tid + qd * kAT);
      t[qd] = (u32)touched[e0] | ((u32)touched[e0 + 1] << 1);
      const bool vec = t[qd] != 0u && sbase_g + e0 + 1 < elems;
      dd[qd] = *reinterpret_cast<const V2*>(vec ? sbase + e0 : sbase);
      if (t[qd]) *reinterpret_cast<uint16_t*>(touched + e0) = 0;
    }
#pragma unroll
    for (int qd = 0; qd < kPairsPerThread; ++qd) {
      if (t[qd] == 0u) continue;
      const int e0 = 2 * (tid + qd * kAT);
      if (sbase_g + e0 + 1 < elems) {
        V2 rr = dd[qd];
        if (t[qd] & 1u) rr.x = acc_add((V)rr.x, acc[e0]);
        if (t[qd] & 2u) rr.y = acc_add((V)rr.y, acc[e0 + 1]);
        *reinterpret_cast<V2*>(sbase + e0) = rr;
      } else {  // the shard's last element, odd count
        sbase[e0] = acc_add(sbase[e0], acc[e0]);
      }
      acc[e0] = A(0);
      acc[e0 + 1] = A(0);
    }
    __syncthreads();
  }
}

// Hot slabs: every (slab, run) pair is a work unit of its own (a run holds at most one fine item's
// records -- or one level-1 workgroup's), summed in LDS and added with device atomics.
template <typename V>
__global__ __launch_bounds__(kAT) void pg_apply_hot_kernel(PgSegs sg, const u32* __restrict__ dir, char* pool,
                                                           const u32* __restrict__ ib0, int two, u32 fbits, u32 nd2,
                                                           u32 G, u32 maxruns, V* __restrict__ data,
                                                           const u32* __restrict__ hot, const PgCtl* pc) {
  typedef typename LdsAcc<V>::T A;
  __shared__ A acc[kPgSlab];
  __shared__ uint8_t touched[kPgSlab];
  const int tid = threadIdx.x;
  const u32 nh = pc->nhot;
  if (nh == 0) return;
  for (int e = tid; e < kPgSlab; e += kAT) {
    acc[e] = A(0);
    touched[e] = 0;
  }
  __syncthreads();
  const u64 units = (u64)nh * maxruns;
  for (u64 u = blockIdx.x; u < units; u += gridDim.x) {
    const u32 s = hot[u / maxruns], k = (u32)(u % maxruns);
    const PgSlabRuns R = pg_runs_of(s, two != 0, fbits, nd2, G, ib0);
    if (k >= R.count) continue;
    const u32 ix = R.base + k * R.stride;
    const u32 np = sg.np[ix], off = sg.off[ix], last = sg.last[ix];
    if (np == 0) continue;
    for (u32 g0 = 0; g0 < np; g0 += kAPages) {
#pragma unroll
      for (int j = 0; j < kAPer; ++j) {
        const u32 qq = (u32)tid + (u32)j * kAT;
        const u32 g = g0 + (qq >> 5), slot = qq & 31u;
        if (g < np && slot < (g + 1 == np ? last : (u32)kPage)) {
          const u32 page = dir[off + g];
          const u32 e = pg_a<A>(pool, page)[slot] & (kPgSlab - 1);
          lds_add(&acc[e], pg_v<A>(pool, page)[slot]);
          touched[e] = 1;
        }
      }
    }
    __syncthreads();
    V* const sbase = data + ((i64)s << kPgSlabBits);
    for (int e = tid; e < kPgSlab; e += kAT) {
      if (touched[e]) {
        gadd(sbase + e, (V)acc[e]);
        acc[e] = A(0);
        touched[e] = 0;
      }
    }
    __syncthreads();
  }
}

// ---- host side ----------------------------------------------------------------------------------------------
struct PgGeom {
  bool two;     // two levels (else level 1 is the slab)
  PgLevel l1, l2;
  u32 fbits;    // log2 of l2.nd
  u32 nslab;
};

// nullopt-style: false when the shard has more than 2^16 slabs (the paged path needs <= two levels)
bool pg_geometry(i64 elems, PgGeom& g) {
  const i64 slabs = (elems + kPgSlab - 1) / kPgSlab;
  u32 sb = 0;
  while (((i64)1 << sb) < slabs) ++sb;
  if (sb > 16) return false;
  g.nslab = (u32)slabs;
  if (sb <= 8) {
    g.two = false;
    g.l1 = PgLevel{(u32)kPgSlabBits, 1u << sb};
    g.l2 = PgLevel{0u, 1u};
    g.fbits = 0;
  } else {
    g.two = true;
    g.fbits = sb - 8;
    g.l1 = PgLevel{(u32)kPgSlabBits + g.fbits, 256u};
    g.l2 = PgLevel{(u32)kPgSlabBits, 1u << g.fbits};
  }
  return true;
}

bool paged_available(const glint_shard* s) {
  PgGeom g;
  return s->elems < ((i64)1 << 32) - 1 && pg_geometry(s->elems, g);
}

// records per slab from which pg_apply warms the whole slab into L2 (GLINT_BIN_PREFETCH_MIN)
u32 pg_prefetch_min() {
  static const u32 v = [] {
    const char* e = getenv("GLINT_BIN_PREFETCH_MIN");
    return e ? (u32)strtoul(e, nullptr, 10) : (u32)(kPgSlab / 4);
  }();
  return v;
}

template <typename V, bool MAT>
int push_paged(glint_shard* s, const PushArgs<V>& a, bool from_break, hipStream_t st) {
  typedef typename LdsAcc<V>::T A;
  const i64 n = a.n;
  if (n >= ((i64)1 << 32) - 2 * kPChunk || s->elems >= ((i64)1 << 32) - 1) return GLINT_EINVAL;  // u32 addresses
  PgGeom g;
  if (!pg_geometry(s->elems, g)) return GLINT_EINVAL;
  // front end: dedup when the last probe kept < 60 % of the records (the hints as of the last sync
  // point); re-probe every 16 pushes. GLINT_BIN_FRONT = dedup | prep forces one (tests, tuning).
  {
    const u64 w = s->hint_bin;
    const u32 m = (u32)(w >> 32), tail = (u32)w;
    if (tail > 0 && s->hint_bin_dedup) s->bin_dedup_ratio = (double)m / (double)tail;
  }
  bool dedup = s->bin_dedup_ratio < 0.6 || (++s->bin_pushes & 15) == 0;
  if (const char* e = getenv("GLINT_BIN_FRONT")) {
    if (!strcmp(e, "dedup")) dedup = true;
    else if (!strcmp(e, "prep")) dedup = false;
  }
  s->bin_last_dedup = dedup;
  const i64 nchunks = (n + kPChunk - 1) / kPChunk;  // an upper bound (the tail may start later)
  // level-1 workgroups: one per CU (the LDS holds one), fewer for small pushes so that each
  // (workgroup, bucket) pair fills some whole pages
  const u32 G = (u32)std::max<i64>(1, std::min<i64>({(i64)s->cus, (i64)kPgMaxG, nchunks, (n + 16383) / 16384}));
  const i64 chunks_w = (nchunks + G - 1) / G;
  const u32 PW = (u32)(chunks_w * (kPChunk / kPage) + g.l1.nd + 1);  // full pages + one partial per bucket
  const i64 pages1 = (i64)G * PW;
  const i64 max_items = g.two ? (i64)g.l1.nd + pages1 / kFItemPages + 1 : 0;
  const u32 FPW = kFItemPages + g.l2.nd + 1;
  const i64 pages2 = max_items * FPW;
  const size_t PB = page_bytes<A>();
  const size_t nseg1 = (size_t)g.l1.nd * G, nseg2 = (size_t)max_items * g.l2.nd;
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off += pad256(bytes); return o; };
  const size_t o_ctl = take(sizeof(PgCtl));
  const size_t o_pool1 = take((size_t)pages1 * PB), o_dir1 = take((size_t)pages1 * 4), o_dig1 = take((size_t)pages1 * 4);
  const size_t o_seg1 = take(nseg1 * 12);
  const size_t o_items = take((size_t)max_items * 16), o_ib0 = take(((size_t)g.l1.nd + 1) * 4);
  const size_t o_pool2 = take((size_t)pages2 * PB), o_dir2 = take((size_t)pages2 * 4), o_dig2 = take((size_t)pages2 * 4);
  const size_t o_seg2 = take(nseg2 * 12);
  const size_t o_hot = take((size_t)g.nslab * 4);
  int rc = grow(&s->d_bin, &s->bin_bytes, off);
  if (rc) return rc;
  char* base = (char*)s->d_bin;
  PgCtl* pc = (PgCtl*)(base + o_ctl);
  char* pool1 = base + o_pool1;
  u32* dir1 = (u32*)(base + o_dir1);
  u32* dig1 = (u32*)(base + o_dig1);
  PgSegs s1{(u32*)(base + o_seg1), (u32*)(base + o_seg1) + nseg1, (u32*)(base + o_seg1) + 2 * nseg1};
  uint4* items = (uint4*)(base + o_items);
  u32* ib0 = (u32*)(base + o_ib0);
  char* pool2 = base + o_pool2;
  u32* dir2 = (u32*)(base + o_dir2);
  u32* dig2 = (u32*)(base + o_dig2);
  PgSegs s2{(u32*)(base + o_seg2), (u32*)(base + o_seg2) + nseg2, (u32*)(base + o_seg2) + 2 * nseg2};
  u32* hot = (u32*)(base + o_hot);

  ProfScope ps(s, GLINT_K_PUSH_BINNED, st);
  HIPCHK(hipMemsetAsync(pc, 0, sizeof(PgCtl), st));
  const int fb = from_break ? 1 : 0;
  u64* hint = s->d_hint ? s->d_hint + 1 : nullptr;
  if (dedup)
    pg_part1_kernel<V, MAT, true><<<G, kPT, 0, st>>>(a.keys, a.cols, a.vals, n, a.part, a.ctl, a.ntiles, fb, g.l1, pool1,
                                                      PW, dig1, dir1, s1, a.err, pc);
  else
    pg_part1_kernel<V, MAT, false><<<G, kPT, 0, st>>>(a.keys, a.cols, a.vals, n, a.part, a.ctl, a.ntiles, fb, g.l1,
                                                       pool1, PW, dig1, dir1, s1, a.err, pc);
  HIPCHK(hipGetLastError());
  PgSegs sa = s1;
  const u32* dira = dir1;
  char* poola = pool1;
  if (g.two) {
    pg_plan_kernel<<<1, kPT, 0, st>>>(g.l1, G, s1, items, ib0, pc, hint);
    HIPCHK(hipGetLastError());
    const unsigned g2 = (unsigned)std::min<i64>(max_items, (i64)s->cus);
    pg_part2_kernel<A, false><<<g2, kPT, 0, st>>>(g.l2, G, items, pc, s1, dir1, pool1, pool2, FPW, dig2, dir2, s2);
    HIPCHK(hipGetLastError());
    sa = s2;
    dira = dir2;
    poola = pool2;
  }
  // apply workgroups: exactly the resident ones (4 per CU at ~39 KB of LDS); GLINT_BIN_APPLY_BPC overrides
  static const int apply_bpc = [] {
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, pg_apply_kernel<V>, kAT, 0) != hipSuccess || b < 1) {
      (void)hipGetLastError();
      b = 4;
    }
    const char* e = getenv("GLINT_BIN_APPLY_BPC");
    return (e && atoi(e) > 0) ? atoi(e) : b;
  }();
  const unsigned ga = (unsigned)std::min<i64>(g.nslab, (i64)s->cus * apply_bpc);
  pg_apply_kernel<V><<<ga, kAT, 0, st>>>(sa, dira, poola, ib0, g.nslab, g.two ? 1 : 0, g.fbits, g.l2.nd, G, s->elems,
                                          a.data, hot, pc, pg_prefetch_min(), g.two ? nullptr : hint);
  HIPCHK(hipGetLastError());
  const u32 maxruns = g.two ? (u32)std::max<i64>(1, max_items) : G;
  pg_apply_hot_kernel<V><<<(unsigned)s->cus * 2, kAT, 0, st>>>(sa, dira, poola, ib0, g.two ? 1 : 0, g.fbits, g.l2.nd,
                                                                G, maxruns, a.data, hot, pc);
  HIPCHK(hipGetLastError());
  return GLINT_OK;
}

// The binned tail: the paged pipeline above, or glint_bin.hip's for shards of more than 2^16 slabs
// (GLINT_BIN_IMPL=v1 forces the latter: A/B runs on one box).
template <typename V, bool MAT>
int push_binned_tail(glint_shard* s, const PushArgs<V>& a, bool from_break, hipStream_t st) {
  static const bool v1 = [] {
    const char* e = getenv("GLINT_BIN_IMPL");
    return e && !strcmp(e, "v1");
  }();
  if (!v1 && paged_available(s)) return push_paged<V, MAT>(s, a, from_break, st);
  return push_binned<V, MAT>(s, a, from_break, st);
}

#define GLINT_INST(V, MAT)                                                                          \
  template int push_paged<V, MAT>(glint_shard*, const PushArgs<V>&, bool, hipStream_t);            \
  template int push_binned_tail<V, MAT>(glint_shard*, const PushArgs<V>&, bool, hipStream_t);
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
