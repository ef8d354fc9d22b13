// glint_sort.hip -- the deterministic tail of a large push: a stable
// rocPRIM radix sort by address, then an in-order fold per address starting from the shard's value --
// PartialVector.update's sequential `+=` order (src/main/scala/glint/models/server/
// PartialVector.scala:35-43), bit for bit. (Pushes of up to kOrderedMax records take the one-launch
// fold of glint_ordered.hip instead; the binned unordered path is glint_bin.hip.)
// Kept apart from glint_gpu.hip so that the rocPRIM instantiations compile once.
#include "glint_device.h"
#include "glint_host.h"

#include <rocprim/device/device_radix_sort.hpp>

#include <cstring>

namespace glint {

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
