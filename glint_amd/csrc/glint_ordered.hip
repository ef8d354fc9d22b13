// glint_ordered.hip -- the order-preserving push for message-sized pushes: PartialVector.update's
// strictly sequential `data(k) += v` (src/main/scala/glint/models/server/PartialVector.scala:35-43;
// PartialMatrix.scala:74-83 for matrices), rounding for rounding, in one launch and with no sort
// library and no host round trip.
//
// An Akka message holds at most 79 999 Double records (the 1 280 000-byte frame cap,
// src/main/resources/glint.conf:143, RequestSerializer.scala:166-167) and usually ~1000
// (GranularBigVectorSpec.scala:21). For such pushes the order-preserving fold costs about what the
// unordered LDS-hash scatter costs, so the host-pointer and wire entry points (what the JNI shim
// calls) use it by default for Float/Double, and device calls use it under GLINT_PUSH_DETERMINISTIC.
//
// Design: the shard's elements are dealt to the grid's workgroups by a hash of the element address,
// so every element has exactly one owner. Every workgroup streams the whole message (from L2: a
// frame-cap message is 1.3 MB) in record order, 4096 records at a time, and appends the records it
// owns to an LDS list -- order preserved by a block-wide prefix sum over the owned flags. When the
// list would overflow (and at the end) it is flushed: a bitonic sort of (address << 12 | position)
// keys, which orders each element's records by message position, then one thread per run folds the
// run into the shard strictly left to right, starting from the shard's current value. Later flushes
// of the same workgroup see the earlier flushes' stores, so an element's chain stays in message
// order across flushes.
#include "glint_device.h"
#include "glint_host.h"

namespace glint {

constexpr int kOrdTPB = 1024;                  // 16 waves: one workgroup per CU-sized share of the work
constexpr int kOrdR = 4;                       // consecutive records per thread per chunk
constexpr int kOrdChunk = kOrdTPB * kOrdR;     // records streamed per step (4096)
constexpr int kOrdCap = 4096;                  // LDS list capacity (records)
static_assert(kOrdCap % kOrdTPB == 0, "a flush holds at most kOrdCap / kOrdTPB records per thread");
constexpr int kOrdPosBits = 12;                // list position bits in a sort key
constexpr u64 kOrdPad = ~0ull;                 // sort padding (above every real key: keys < 2^44)
constexpr int kOrdHashBits = 13;               // distinctness table: 8192 slots (load <= 0.5)
constexpr int kOrdHash = 1 << kOrdHashBits;
constexpr u32 kOrdEmpty = 0xFFFFFFFFu;         // no address: shards hold < 2^32 - 1 elements

__device__ __forceinline__ u32 ordered_owner(u64 addr, u32 nwg) {
  const u64 h = addr * 0x9E3779B97F4A7C15ull;
  return (u32)(((h >> 32) * (u64)nwg) >> 32);
}

// the shard value a fold starts from: an L1-bypassing load, so a flush sees the stores of an
// earlier flush of its own workgroup made by another wave
__device__ __forceinline__ double ld_shard(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load((const u64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ float ld_shard(const float* p) {
  return __int_as_float((int)__hip_atomic_load((const u32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ long long ld_shard(const long long* p) {
  return (long long)__hip_atomic_load((const u64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_shard(const int* p) {
  return (int)__hip_atomic_load((const u32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// distinctness-table slot of an address: murmur3's fmix32, low bits. It must not correlate with
// ordered_owner: a multiplicative hash with a golden-ratio constant did (both took top bits of nearly
// the same product), so a workgroup's addresses crowded 1/nwg of the table into long probe chains
__device__ __forceinline__ u32 ord_hash(u32 x) {
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x & (kOrdHash - 1);
}

// Sorts list[0, cnt) and folds each element's run in message order. Block-uniform cnt.
// Only elements that occur more than once in the list need the sort: every address is inserted into
// an LDS hash table (htab, all empty on entry and on return), a repeated address marks its slot in
// dupbits, and records whose slot is unmarked -- runs of one record, the usual message is all of
// them -- are added to the shard directly. The marked records (the repeated elements' whole runs)
// are compacted to the list's front and bitonic-sorted by (address, position) as before.
template <typename V>
__device__ void ordered_flush(u64* skey, const V* sval, u32 cnt, V* data, u32* htab, u32* dupbits, u32* s_dcnt) {
  const u32 tid = threadIdx.x;
  constexpr int kPer = kOrdCap / kOrdTPB;
  for (u32 i = tid; i < cnt; i += kOrdTPB) {
    const u32 ad = (u32)(skey[i] >> kOrdPosBits);
    u32 h = ord_hash(ad);
    for (;;) {
      const u32 prev = atomicCAS(&htab[h], kOrdEmpty, ad);
      if (prev == kOrdEmpty) break;
      if (prev == ad) {
        atomicOr(&dupbits[h >> 5], 1u << (h & 31));
        break;
      }
      h = (h + 1) & (kOrdHash - 1);
    }
  }
  __syncthreads();
  u64 dk[kPer];
  u32 dmask = 0;
#pragma unroll
  for (int r = 0; r < kPer; ++r) {  // list position i holds record position i
    const u32 i = tid + (u32)r * kOrdTPB;
    dk[r] = 0;
    if (i < cnt) {
      const u64 key = skey[i];
      const u32 ad = (u32)(key >> kOrdPosBits);
      u32 h = ord_hash(ad);
      while (htab[h] != ad) h = (h + 1) & (kOrdHash - 1);
      if (dupbits[h >> 5] & (1u << (h & 31))) {
        dk[r] = key;
        dmask |= 1u << r;
      } else {
        data[ad] = vadd(ld_shard(data + ad), sval[i]);
      }
    }
  }
  if (tid == 0) *s_dcnt = 0;
  __syncthreads();  // every record is read (skey is free) and the table's lookups are done
  for (u32 h = tid; h < (u32)kOrdHash; h += kOrdTPB) htab[h] = kOrdEmpty;
  for (u32 w = tid; w < (u32)kOrdHash / 32; w += kOrdTPB) dupbits[w] = 0;
#pragma unroll
  for (int r = 0; r < kPer; ++r)
    if (dmask & (1u << r)) skey[atomicAdd(s_dcnt, 1u)] = dk[r];
  __syncthreads();
  cnt = *s_dcnt;  // the repeated elements' records, in no particular order: the sort orders them
  if (cnt == 0) {
    __syncthreads();  // every thread has read the count before the caller refills the list
    return;
  }
  u32 P = 64;
  while (P < cnt) P <<= 1;
  for (u32 i = cnt + tid; i < P; i += kOrdTPB) skey[i] = kOrdPad;
  __syncthreads();
  for (u32 k = 2; k <= P; k <<= 1) {
    for (u32 j = k >> 1; j > 0; j >>= 1) {
      for (u32 t = tid; t < P / 2; t += kOrdTPB) {
        const u32 i = ((t & ~(j - 1)) << 1) | (t & (j - 1));
        const u32 l = i + j;
        const u64 x = skey[i], y = skey[l];
        if ((x > y) == ((i & k) == 0)) {
          skey[i] = y;
          skey[l] = x;
        }
      }
      __syncthreads();
    }
  }
  for (u32 i = tid; i < cnt; i += kOrdTPB) {
    const u64 key = skey[i];
    const u64 ad = key >> kOrdPosBits;
    if (i > 0 && (skey[i - 1] >> kOrdPosBits) == ad) continue;  // not the head of its run
    V acc = ld_shard(data + ad);
    u32 j = i;
    do {
      acc = vadd(acc, sval[(u32)skey[j] & (kOrdCap - 1)]);
      ++j;
    } while (j < cnt && (skey[j] >> kOrdPosBits) == ad);
    data[ad] = acc;
  }
  __syncthreads();
}

template <typename V, bool MAT>
__global__ __launch_bounds__(kOrdTPB) void push_ordered_kernel(PushArgs<V> a, int vec) {
  typedef typename Vec2<V>::T V2;
  __shared__ u64 skey[kOrdCap];
  __shared__ V sval[kOrdCap];
  __shared__ u32 wsum[kOrdTPB / 64];
  __shared__ u32 s_cnt, s_dcnt;
  __shared__ u32 htab[kOrdHash];
  __shared__ u32 dupbits[kOrdHash / 32];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const u32 nwg = gridDim.x, me = blockIdx.x;
  const i64 n = a.n;
  if (tid == 0) s_cnt = 0;
  for (u32 h = tid; h < (u32)kOrdHash; h += kOrdTPB) htab[h] = kOrdEmpty;
  for (u32 w = tid; w < (u32)kOrdHash / 32; w += kOrdTPB) dupbits[w] = 0;
  for (i64 base = 0; base < n; base += kOrdChunk) {
    const i64 r0 = base + (i64)tid * kOrdR;
    i64 k[kOrdR];
    int32_t c[kOrdR];
    V v[kOrdR];
    if (vec && r0 + kOrdR <= n) {
#pragma unroll
      for (int h = 0; h < kOrdR / 2; ++h) {
        const K2 kk = reinterpret_cast<const K2*>(a.keys + r0)[h];
        const V2 vv = reinterpret_cast<const V2*>(a.vals + r0)[h];
        k[2 * h] = kk.x;
        k[2 * h + 1] = kk.y;
        v[2 * h] = (V)vv.x;
        v[2 * h + 1] = (V)vv.y;
        if (MAT) {
          const C2 cc = reinterpret_cast<const C2*>(a.cols + r0)[h];
          c[2 * h] = cc.x;
          c[2 * h + 1] = cc.y;
        } else {
          c[2 * h] = c[2 * h + 1] = 0;
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < kOrdR; ++j) {
        const i64 r = r0 + j < n ? r0 + j : n - 1;
        k[j] = a.keys[r];
        c[j] = MAT ? a.cols[r] : 0;
        v[j] = a.vals[r];
      }
    }
    u32 own = 0;
    u32 ad[kOrdR];
#pragma unroll
    for (int j = 0; j < kOrdR; ++j) {
      ad[j] = 0;
      if (r0 + j < n) {
        i64 a64;
        if (rec_addr<MAT>(a.part, k[j], c[j], a64)) {
          ad[j] = (u32)a64;
          if (ordered_owner((u64)a64, nwg) == me) own |= 1u << j;
        } else if (me == 0) {
          record_error(a.err, r0 + j);
        }
      }
    }
    // block-wide exclusive prefix of the owned counts: the list keeps message order
    const u32 cnt_t = (u32)__popc(own);
    u32 incl = cnt_t;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const u32 y = __shfl_up(incl, d);
      if (lane >= d) incl += y;
    }
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    u32 woff = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kOrdTPB / 64; ++w) {
      const u32 x = wsum[w];
      woff += w < wid ? x : 0u;
      total += x;
    }
    u32 cur = s_cnt;
    if (cur + total > (u32)kOrdCap) {  // block-uniform
      ordered_flush<V>(skey, sval, cur, a.data, htab, dupbits, &s_dcnt);
      cur = 0;
    }
    u32 p = cur + woff + incl - cnt_t;
#pragma unroll
    for (int j = 0; j < kOrdR; ++j) {
      if (own & (1u << j)) {
        skey[p] = ((u64)ad[j] << kOrdPosBits) | p;
        sval[p] = v[j];
        ++p;
      }
    }
    __syncthreads();
    if (tid == 0) s_cnt = cur + total;
  }
  __syncthreads();
  ordered_flush<V>(skey, sval, s_cnt, a.data, htab, dupbits, &s_dcnt);
  msg_signal(a.sig, a.err);
}

template <typename V, bool MAT>
int push_ordered(glint_shard* s, const PushArgs<V>& a, hipStream_t st) {
  if (a.n <= 0) return GLINT_OK;
  if (a.n > kOrderedMax || s->elems >= ((i64)1 << 32)) return GLINT_EINVAL;
  if (a.sig.done && a.n > kOrdCap) return GLINT_EINVAL;  // a ring launch is one workgroup: one list
  const unsigned g = a.sig.done ? 1u : grid_for(a.n, 1024, (i64)s->cus);
  const int vec = aligned(a.keys, 16) && aligned(a.vals, 2 * sizeof(V)) && (!MAT || aligned(a.cols, 8));
  HIPCHK(launch_k(s, GLINT_K_PUSH_ORDERED, push_ordered_kernel<V, MAT>, g, kOrdTPB, st, a, vec));
  return GLINT_OK;
}

#define GLINT_INST(V, MAT) template int push_ordered<V, MAT>(glint_shard*, const PushArgs<V>&, hipStream_t);
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
