// glint_sort.hip -- the deterministic tail of a large push: a stable
// radix sort by address (hand-written, LSD, 8-bit digits), then an in-order fold per address starting
// from the shard's value -- PartialVector.update's sequential `+=` order (src/main/scala/glint/models/
// server/PartialVector.scala:35-43), bit for bit. (Pushes of up to kOrderedMax records take the
// one-launch fold of glint_ordered.hip instead; the binned unordered path is glint_bin.hip.)
#include "glint_device.h"
#include "glint_host.h"

#include <cstring>

namespace glint {

// ------------------------------------------------------------------------------------------------
// deterministic tail: stable sort by address, then an in-order fold per address starting from the
// shard's current value -- the reference's sequential `+=` order, bit for bit
// ------------------------------------------------------------------------------------------------
// Records before the tail start (push_check's break, read here on the device: no host round trip)
// and rejected records get the sentinel address, which sorts behind every element and is skipped.
template <typename K, typename V, bool MAT>
__global__ __launch_bounds__(kTPB) void det_prepare_kernel(const i64* keys, const int32_t* cols, const V* vals, i64 m,
                                                           const LaunchCtl* ctl, u32 ntiles, int from_break,
                                                           PartDesc part, K sentinel, K* addr, V* val,
                                                           ErrState* err) {
  i64 r0 = 0;
  if (from_break) {
    const u32 brk = ctl->brk_enc;
    r0 = brk == 0u ? m : (i64)(ntiles - brk) * kTile;
  }
  for (i64 i = (i64)blockIdx.x * kTPB + threadIdx.x; i < m; i += (i64)gridDim.x * kTPB) {
    K out = sentinel;
    if (i >= r0) {
      i64 ad;
      if (rec_addr<MAT>(part, keys[i], MAT ? cols[i] : 0, ad)) out = (K)ad;
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

template <typename K, typename V>
__global__ __launch_bounds__(kTPB) void det_fold_short_kernel(const K* addr, const V* val, i64 m, K sentinel,
                                                              V* data, u32* long_count, u32* long_list) {
  for (i64 i = (i64)blockIdx.x * kTPB + threadIdx.x; i < m; i += (i64)gridDim.x * kTPB) {
    const K ad = addr[i];
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
template <typename K>
__device__ __forceinline__ i64 run_end(const K* addr, i64 m, i64 i, K ad, int lane) {
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

template <typename K, typename V>
__global__ __launch_bounds__(kTPB) void det_fold_long_kernel(const K* addr, const V* val, i64 m,
                                                             const u32* long_count, const u32* long_list, V* data) {
  const int lane = threadIdx.x & 63;
  const u32 w0 = blockIdx.x * (kTPB / 64) + (threadIdx.x >> 6);
  const u32 nw = gridDim.x * (kTPB / 64);
  const u32 cnt = *long_count;
  constexpr i64 kB = 64 * kDetK;
  for (u32 w = w0; w < cnt; w += nw) {
    const i64 i = long_list[w];
    const K ad = addr[i];
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

// ---- stable LSD radix sort of (address, value) pairs --------------------------------------------
// One pass per 8-bit digit, three launches each:
//   rs_hist     per 2048-key tile, the digit counts -> hist[digit][tile];
//   rs_sums / rs_scan  per digit its total, then offs[digit][tile] = keys of smaller digits + keys of
//               this digit in earlier tiles (the route's offset kernels, one block per digit);
//   rs_scatter  per tile, stable ranks (lanes and waves in key order: one ballot per digit bit, then
//               per-(round, wave) counts), the tile staged in LDS grouped by digit, and written out
//               in runs -- consecutive threads, consecutive slots.
constexpr int kST = 256;               // threads of the sort kernels
constexpr int kSPer = 8;               // keys per thread per tile
constexpr int kSTile = kST * kSPer;    // 2048
constexpr int kSSegs = kSPer * (kST / 64);  // (round, wave) segments of a tile: 32

template <typename K>
__global__ __launch_bounds__(kST) void rs_hist(const K* __restrict__ keys, i64 n, int shift, u32* __restrict__ hist,
                                               u32 ntiles) {
  __shared__ u32 h[kST / 64][256];
  const int tid = threadIdx.x, wid = tid >> 6;
  for (int d = tid; d < 4 * 256; d += kST) (&h[0][0])[d] = 0;
  __syncthreads();
  const i64 t0 = (i64)blockIdx.x * kSTile;
  K k[kSPer];
#pragma unroll
  for (int j = 0; j < kSPer; ++j) {
    const i64 i = t0 + j * kST + tid;
    k[j] = keys[i < n ? i : n - 1];
  }
  const int lane = tid & 63;
#pragma unroll
  for (int j = 0; j < kSPer; ++j) {  // one LDS add per distinct digit of the wave (a hot key is one)
    const u32 d = t0 + j * kST + tid < n ? ((u32)(k[j] >> shift) & 255u) : 256u;
    u64 m = ~0ull;
#pragma unroll
    for (int b = 0; b < 9; ++b) {
      const bool bit = (d >> b) & 1u;
      const u64 bb = __ballot(bit);
      m &= bit ? bb : ~bb;
    }
    if (d < 256u && (m & ((1ull << lane) - 1ull)) == 0) h[wid][d] += (u32)__popcll(m);
  }
  __syncthreads();
  hist[(i64)tid * ntiles + blockIdx.x] = h[0][tid] + h[1][tid] + h[2][tid] + h[3][tid];
}

__device__ __forceinline__ u32 rs_block_sum(u32 x) {
  __shared__ u32 ws[1024 / 64];
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = x;
  __syncthreads();
  u32 t = 0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += ws[w];
  __syncthreads();
  return t;
}

// tot[d] = keys with digit d (one block per digit)
__global__ __launch_bounds__(1024) void rs_sums(const u32* __restrict__ hist, u32 ntiles, u32* __restrict__ tot) {
  const u32* row = hist + (i64)blockIdx.x * ntiles;
  u32 x = 0;
  for (u32 b = threadIdx.x; b < ntiles; b += 1024) x += row[b];
  x = rs_block_sum(x);
  if (threadIdx.x == 0) tot[blockIdx.x] = x;
}

// offs[d][t] = sum(tot[0..d)) + sum(hist[d][0..t)) (one block per digit)
__global__ __launch_bounds__(1024) void rs_scan(const u32* __restrict__ hist, u32 ntiles, const u32* __restrict__ tot,
                                                u32* __restrict__ offs) {
  __shared__ u32 wt[16];
  const int d = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  u32 base = tid < d ? tot[tid] : 0u;
  base = rs_block_sum(base);
  const u32* row = hist + (i64)d * ntiles;
  u32* out = offs + (i64)d * ntiles;
  u32 carry = base;
  for (u32 t0 = 0; t0 < ntiles; t0 += 1024 * 4) {
    const u32 b0 = t0 + (u32)tid * 4;
    u32 v[4], sum = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = b0 + j < ntiles ? row[b0 + j] : 0u;
      sum += v[j];
    }
    u32 incl = sum;
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
      const u32 y = __shfl_up(incl, s);
      if (lane >= s) incl += y;
    }
    if (lane == 63) wt[wid] = incl;
    __syncthreads();
    u32 run = carry + incl - sum, all = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) {
      const u32 y = wt[w];
      run += w < wid ? y : 0u;
      all += y;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (b0 + j < ntiles) out[b0 + j] = run;
      run += v[j];
    }
    carry += all;
    __syncthreads();
  }
}

template <typename K, typename V>
__global__ __launch_bounds__(kST) void rs_scatter(const K* __restrict__ kin, const V* __restrict__ vin, i64 n, int shift,
                                                  const u32* __restrict__ offs, u32 ntiles, K* __restrict__ kout,
                                                  V* __restrict__ vout) {
  __shared__ uint16_t seg[256][kSSegs];  // per digit: counts, then first staging slot, of each segment
  __shared__ u32 dbase[256];             // per digit: first staging slot
  __shared__ u32 wt[kST / 64];
  __shared__ K sk[kSTile];
  __shared__ V sv[kSTile];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const u64 below = (1ull << lane) - 1ull;
  const i64 t0 = (i64)blockIdx.x * kSTile;
  K k[kSPer];
  V v[kSPer];
  u32 d[kSPer], wr[kSPer];
#pragma unroll
  for (int j = 0; j < kSPer; ++j) {  // clamped, branch-free loads; key order = (round j, thread)
    const i64 i = t0 + j * kST + tid;
    const i64 ii = i < n ? i : n - 1;
    k[j] = kin[ii];
    v[j] = vin[ii];
    d[j] = i < n ? ((u32)(k[j] >> shift) & 255u) : 256u;  // 256: past the end
  }
  for (int x = tid; x < 256 * kSSegs / 2; x += kST) reinterpret_cast<u32*>(&seg[0][0])[x] = 0;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kSPer; ++j) {  // lanes with equal digits: one ballot per digit bit
    u64 m = ~0ull;
#pragma unroll
    for (int b = 0; b < 9; ++b) {
      const bool bit = (d[j] >> b) & 1u;
      const u64 bb = __ballot(bit);
      m &= bit ? bb : ~bb;
    }
    wr[j] = (u32)__popcll(m & below);
    if (d[j] < 256u && wr[j] == 0) seg[d[j]][j * (kST / 64) + wid] = (uint16_t)__popcll(m);
  }
  __syncthreads();
  // per digit (one thread each): segment prefixes in key order, then the digits' bases
  u32 tot = 0;
  {
    for (int q = 0; q < kSSegs; ++q) {
      const u32 c = seg[tid][q];
      seg[tid][q] = (uint16_t)tot;
      tot += c;
    }
    u32 incl = tot;
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
      const u32 y = __shfl_up(incl, s);
      if (lane >= s) incl += y;
    }
    if (lane == 63) wt[wid] = incl;
    __syncthreads();
    u32 ex = incl - tot;
#pragma unroll
    for (int w = 0; w < kST / 64; ++w) ex += w < wid ? wt[w] : 0u;
    dbase[tid] = ex;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kSPer; ++j) {
    if (d[j] < 256u) {
      const u32 p = dbase[d[j]] + seg[d[j]][j * (kST / 64) + wid] + wr[j];
      sk[p] = k[j];
      sv[p] = v[j];
    }
  }
  __syncthreads();
  const i64 valid = n - t0 < kSTile ? n - t0 : kSTile;
#pragma unroll
  for (int j = 0; j < kSPer; ++j) {
    const int p = tid + j * kST;
    if (p < valid) {
      const K kk = sk[p];
      const u32 dd = (u32)(kk >> shift) & 255u;
      const u32 dst = offs[(i64)dd * ntiles + blockIdx.x] + ((u32)p - dbase[dd]);
      kout[dst] = kk;
      vout[dst] = sv[p];
    }
  }
}

// Sorts m (key, value) pairs by the low end_bit bits of the key, stably; the result is in (k1, v1)
// when the number of passes is odd, else back in (k0, v0). Returns the buffer index (0 or 1).
template <typename K, typename V>
int rs_sort(K* k0, V* v0, K* k1, V* v1, i64 m, int end_bit, u32* hist, u32* offs, u32* tot, hipStream_t st,
            int* where) {
  const u32 ntiles = (u32)((m + kSTile - 1) / kSTile);
  int cur = 0;
  for (int shift = 0; shift < end_bit; shift += 8) {
    const K* ki = cur ? k1 : k0;
    const V* vi = cur ? v1 : v0;
    K* ko = cur ? k0 : k1;
    V* vo = cur ? v0 : v1;
    rs_hist<K><<<ntiles, kST, 0, st>>>(ki, m, shift, hist, ntiles);
    rs_sums<<<256, 1024, 0, st>>>(hist, ntiles, tot);
    rs_scan<<<256, 1024, 0, st>>>(hist, ntiles, tot, offs);
    rs_scatter<K, V><<<ntiles, kST, 0, st>>>(ki, vi, m, shift, offs, ntiles, ko, vo);
    HIPCHK(hipGetLastError());
    cur ^= 1;
  }
  *where = cur;
  return GLINT_OK;
}

// ---- hot chains ---------------------------------------------------------------------------------
// An element with hundreds of thousands of records is a fold chain of that many dependent adds (the
// cfg3 batch's hottest key: 7.3 M records, ~33 ms); nothing can shorten it, but nothing needs to wait
// for it either. The elements with the most records in a sample are split off first: their records,
// in push order, go to one buffer per element (a stable compaction) and leave the main sort (their
// address becomes the sentinel). One wave per hot element folds its chain on a second stream while
// the main stream sorts and folds everything else.
constexpr int kHotMax = 8;          // hot elements split off, at most
constexpr int kHotSample = 16384;   // records sampled
constexpr i64 kHotMinRecords = 1 << 16;  // estimated records an element needs to be split off
constexpr int kHotTile = 4096;      // records per block of the compaction

// One block: sample every (m / kHotSample)-th address, count them in an LDS hash table, keep the up
// to kHotMax most frequent ones whose estimated record count reaches kHotMinRecords.
template <typename K>
__global__ __launch_bounds__(1024) void det_hot_pick(const K* __restrict__ addr, i64 m, K sentinel, u32 thresh,
                                                     K* __restrict__ hot, u32* __restrict__ nhot) {
  constexpr int kSlots = sizeof(K) == 4 ? 16384 : 8192;
  constexpr int kSlotShift = sizeof(K) == 4 ? 50 : 51;
  __shared__ K hk[kSlots];
  __shared__ u32 hc[kSlots];
  __shared__ u32 best_c[1024 / 64];
  __shared__ int best_i[1024 / 64];
  __shared__ u32 taken;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int i = tid; i < kSlots; i += 1024) {
    hk[i] = sentinel;
    hc[i] = 0;
  }
  if (tid == 0) taken = 0;
  __syncthreads();
  const i64 stride = m / kHotSample > 0 ? m / kHotSample : 1;
  for (i64 j = tid; j < kHotSample && j * stride < m; j += 1024) {
    const K a = addr[j * stride];
    if (a == sentinel) continue;
    u32 h = (u32)(((u64)a * 0x9E3779B97F4A7C15ull) >> kSlotShift);
    // bounded probing: with more distinct samples than slots a sample may go uncounted -- a hot
    // element is among the first ones seen and is counted
    for (int probe = 0; probe < 64; ++probe) {
      const K prev = atomicCAS(&hk[h], sentinel, a);
      if (prev == sentinel || prev == a) {
        atomicAdd(&hc[h], 1u);
        break;
      }
      h = (h + 1) & (kSlots - 1);
    }
  }
  __syncthreads();
  for (int r = 0; r < kHotMax; ++r) {  // repeated block-wide arg-max
    u32 c = 0;
    int idx = -1;
    for (int i = tid; i < kSlots; i += 1024)
      if (hc[i] > c) { c = hc[i]; idx = i; }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
      const u32 oc = __shfl_xor(c, d);
      const int oi = __shfl_xor(idx, d);
      if (oc > c || (oc == c && oi > idx)) { c = oc; idx = oi; }
    }
    if (lane == 0) { best_c[wid] = c; best_i[wid] = idx; }
    __syncthreads();
    if (tid == 0) {
      u32 bc = 0;
      int bi = -1;
      for (int w = 0; w < 1024 / 64; ++w)
        if (best_c[w] > bc) { bc = best_c[w]; bi = best_i[w]; }
      if (bi >= 0 && bc >= thresh) {
        hot[taken++] = hk[bi];
        hc[bi] = 0;
      }
    }
    __syncthreads();
  }
  if (tid == 0) *nhot = taken;
}

__device__ __forceinline__ int hot_index(u64 a, const u64* hot, u32 nh) {
  int h = -1;
#pragma unroll
  for (int q = 0; q < kHotMax; ++q) h = ((u32)q < nh && a == hot[q]) ? q : h;
  return h;
}

// per block (kHotTile records): records of each hot element -> cnt[h * nblocks + block]
template <typename K>
__global__ __launch_bounds__(kTPB) void det_hot_count(const K* __restrict__ addr, i64 m, const K* __restrict__ hot,
                                                      const u32* __restrict__ nhot, u32* __restrict__ cnt, u32 nblocks) {
  __shared__ u32 c[kHotMax];
  const u32 nh = *nhot;
  if (threadIdx.x < kHotMax) c[threadIdx.x] = 0;
  __syncthreads();
  if (nh == 0) return;
  u64 hv[kHotMax];
#pragma unroll
  for (int q = 0; q < kHotMax; ++q) hv[q] = (u32)q < nh ? (u64)hot[q] : ~0ull;
  const i64 t0 = (i64)blockIdx.x * kHotTile;
  u32 mine[kHotMax] = {0};
  for (int j = threadIdx.x; j < kHotTile; j += kTPB) {
    const i64 i = t0 + j;
    if (i >= m) break;
    const int h = hot_index((u64)addr[i], hv, nh);
    if (h >= 0) ++mine[h];
  }
#pragma unroll
  for (int q = 0; q < kHotMax; ++q)
    if (mine[q]) atomicAdd(&c[q], mine[q]);
  __syncthreads();
  if (threadIdx.x < kHotMax) cnt[(i64)threadIdx.x * nblocks + blockIdx.x] = c[threadIdx.x];
}

// per block, in record order: each hot record's value to the hot buffer at offs[h][block] (the
// element's run, then its block) + its rank among the block's earlier records of that element (waves
// in order, lanes in order); its address becomes the sentinel, so the main sort leaves it out
template <typename K, typename V>
__global__ __launch_bounds__(kTPB) void det_hot_scatter(K* __restrict__ addr, const V* __restrict__ val, i64 m,
                                                        K sentinel, const K* __restrict__ hot,
                                                        const u32* __restrict__ nhot, const u32* __restrict__ offs,
                                                        u32 nblocks, V* __restrict__ hbuf) {
  __shared__ u32 base[kHotMax];
  __shared__ u32 wc[kTPB / 64][kHotMax];
  const u32 nh = *nhot;
  if (nh == 0) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const u64 below = (1ull << lane) - 1ull;
  u64 hv[kHotMax];
#pragma unroll
  for (int q = 0; q < kHotMax; ++q) hv[q] = (u32)q < nh ? (u64)hot[q] : ~0ull;
  if (tid < kHotMax) base[tid] = (u32)tid < nh ? offs[(i64)tid * nblocks + blockIdx.x] : 0u;
  const i64 t0 = (i64)blockIdx.x * kHotTile;
  for (int r0 = 0; r0 < kHotTile; r0 += kTPB) {  // rounds of kTPB records
    const i64 i = t0 + r0 + tid;
    const int h = i < m ? hot_index((u64)addr[i], hv, nh) : -1;
    u32 rank = 0;
#pragma unroll
    for (int q = 0; q < kHotMax; ++q) {
      const u64 b = __ballot(h == q);
      if (h == q) rank = (u32)__popcll(b & below);
      if (lane == 0) wc[wid][q] = (u32)__popcll(b);
    }
    __syncthreads();
    if (h >= 0) {
      u32 pos = base[h] + rank;
      for (int w = 0; w < wid; ++w) pos += wc[w][h];
      hbuf[pos] = val[i];
      addr[i] = sentinel;
    }
    __syncthreads();
    if (tid < kHotMax)
      for (int w = 0; w < kTPB / 64; ++w) base[tid] += wc[w][tid];
    __syncthreads();
  }
}

// one wave per hot element: its whole chain, starting from the shard's value (det_fold's transposed
// loads and lane hand-off)
template <typename K, typename V>
__global__ __launch_bounds__(kTPB) void det_fold_hot(const K* __restrict__ hot, const u32* __restrict__ nhot,
                                                     const u32* __restrict__ tot, const u32* __restrict__ offs,
                                                     u32 nblocks, const V* __restrict__ hbuf, V* data) {
  const int lane = threadIdx.x & 63;
  const u32 w = blockIdx.x * (kTPB / 64) + (threadIdx.x >> 6);
  if (w >= *nhot) return;
  const K ad = hot[w];
  const V* v = hbuf + offs[(i64)w * nblocks];  // the element's run starts at its first block's offset
  const i64 e = tot[w];
  constexpr i64 kB = 64 * kDetK;
  V acc = data[ad];
  V A[kDetK], B[kDetK];
  det_load(A, v, 0, e, lane);
  for (i64 b = 0; b < e; b += 2 * kB) {
    det_load(B, v, b + kB, e, lane);
    acc = det_fold(A, acc, b, e, lane);
    det_load(A, v, b + 2 * kB, e, lane);
    acc = det_fold(B, acc, b + kB, e, lane);
  }
  if (lane == 0) data[ad] = acc;
}

// ---- host side ----------------------------------------------------------------------------------
template <typename K, typename V, bool MAT>
int det_tail_k(glint_shard* s, const PushArgs<V>& a, bool from_break, hipStream_t st) {
  // the whole push is sorted; records before push_check's break are masked on the device, so the
  // call stays stream-ordered with no host synchronisation
  const i64 m = a.n;
  const K sentinel = (K)s->elems;
  int end_bit = 1;
  while (end_bit < (int)(8 * sizeof(K)) && ((u64)1 << end_bit) <= (u64)sentinel) ++end_bit;
  const u32 ntiles = (u32)((m + kSTile - 1) / kSTile);
  const size_t b_addr = pad256((size_t)m * sizeof(K)), b_val = pad256((size_t)m * sizeof(V));
  const size_t b_list = pad256(((size_t)m / kDetShort + 2) * 4);
  const size_t b_hist = pad256((size_t)ntiles * 256 * 4);
  // hot chains: up to kHotMax buffers of m values each (a hot element may own any share of the push)
  const bool split = m >= 8 * kHotMinRecords;
  const u32 hblocks = (u32)((m + kHotTile - 1) / kHotTile);
  const size_t b_hot = split ? pad256((size_t)m * sizeof(V)) + 2 * pad256((size_t)kHotMax * hblocks * 4) + 1024 : 0;
  const size_t need = 2 * b_addr + 2 * b_val + b_list + 2 * b_hist + 1024 + b_hot;
  int rc = grow(&s->d_det, &s->det_bytes, need);
  if (rc) return rc;
  char* base = (char*)s->d_det;
  K* addr0 = (K*)base;
  K* addr1 = (K*)(base + b_addr);
  V* val0 = (V*)(base + 2 * b_addr);
  V* val1 = (V*)(base + 2 * b_addr + b_val);
  u32* long_count = (u32*)(base + 2 * b_addr + 2 * b_val);
  u32* long_list = long_count + 1;
  u32* hist = (u32*)(base + 2 * b_addr + 2 * b_val + b_list);
  u32* offs = (u32*)((char*)hist + b_hist);
  u32* tot = (u32*)((char*)offs + b_hist);
  const unsigned g = grid_for(m, kTPB, (i64)s->cus * 8);
  det_prepare_kernel<K, V, MAT><<<g, kTPB, 0, st>>>(a.keys, a.cols, a.vals, m, a.ctl, a.ntiles, from_break ? 1 : 0,
                                                    a.part, sentinel, addr0, val0, a.err);
  HIPCHK(hipGetLastError());
  if (split) {
    if (!s->det_stream) {
      if (hipStreamCreateWithFlags(&s->det_stream, hipStreamNonBlocking) != hipSuccess ||
          hipEventCreateWithFlags(&s->det_ev[0], hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&s->det_ev[1], hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        return GLINT_EDEVICE;
      }
    }
    char* hb = (char*)tot + 1024;
    V* hbuf = (V*)hb;
    u32* hcnt = (u32*)(hb + pad256((size_t)m * sizeof(V)));
    u32* hoffs = hcnt + pad256((size_t)kHotMax * hblocks * 4) / 4;
    K* hot = (K*)(hoffs + pad256((size_t)kHotMax * hblocks * 4) / 4);
    u32* nhot = (u32*)(hot + kHotMax);
    u32* htot = nhot + 1;
    const u32 thresh = (u32)std::max<i64>(2, kHotMinRecords * kHotSample / m);
    det_hot_pick<K><<<1, 1024, 0, st>>>(addr0, m, sentinel, thresh, hot, nhot);
    det_hot_count<K><<<hblocks, kTPB, 0, st>>>(addr0, m, hot, nhot, hcnt, hblocks);
    // per hot element its records, then per block its offset (the elements' runs one after another)
    rs_sums<<<kHotMax, 1024, 0, st>>>(hcnt, hblocks, htot);
    rs_scan<<<kHotMax, 1024, 0, st>>>(hcnt, hblocks, htot, hoffs);
    det_hot_scatter<K, V><<<hblocks, kTPB, 0, st>>>(addr0, val0, m, sentinel, hot, nhot, hoffs, hblocks, hbuf);
    HIPCHK(hipGetLastError());
    // the hot chains on the second stream, from here; the push's stream joins them at its end
    HIPCHK(hipEventRecord(s->det_ev[0], st));
    HIPCHK(hipStreamWaitEvent(s->det_stream, s->det_ev[0], 0));
    det_fold_hot<K, V><<<(kHotMax + kTPB / 64 - 1) / (kTPB / 64), kTPB, 0, s->det_stream>>>(hot, nhot, htot, hoffs,
                                                                                              hblocks, hbuf, a.data);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(s->det_ev[1], s->det_stream));
  }
  // stable LSD radix sort: equal addresses keep their push order
  int where = 0;
  rc = rs_sort<K, V>(addr0, val0, addr1, val1, m, end_bit, hist, offs, tot, st, &where);
  if (rc) return rc;
  const K* addr = where ? addr1 : addr0;
  const V* val = where ? val1 : val0;
  HIPCHK(hipMemsetAsync(long_count, 0, 4, st));
  det_fold_short_kernel<K, V><<<g, kTPB, 0, st>>>(addr, val, m, sentinel, a.data, long_count, long_list);
  HIPCHK(hipGetLastError());
  det_fold_long_kernel<K, V><<<(unsigned)s->cus * 2, kTPB, 0, st>>>(addr, val, m, long_count, long_list, a.data);
  HIPCHK(hipGetLastError());
  if (split) HIPCHK(hipStreamWaitEvent(st, s->det_ev[1], 0));  // the push ends when its hot chains have
  return GLINT_OK;
}

template <typename V, bool MAT>
int push_det_tail(glint_shard* s, const PushArgs<V>& a, bool from_break, hipStream_t st) {
  // 32-bit addresses (and 32-bit offsets) while the shard's element count and the push fit them
  if (s->elems < ((i64)1 << 32) - 1 && a.n < ((i64)1 << 32) - kSTile) return det_tail_k<u32, V, MAT>(s, a, from_break, st);
  if (a.n >= ((i64)1 << 32) - kSTile) return GLINT_EINVAL;
  return det_tail_k<u64, V, MAT>(s, a, from_break, st);
}

#define GLINT_INST(V, MAT) template int push_det_tail<V, MAT>(glint_shard*, const PushArgs<V>&, bool, hipStream_t);
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
