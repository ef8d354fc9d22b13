// glint_device.h -- device helpers shared by the push/pull kernels (glint_gpu.hip) and the
// sort-based push tails (glint_sort.hip): paired vector types, the reference's `+` on JVM
// primitives, device/LDS atomics and the record -> element address map with its range test.
#pragma once
#include "glint_kernels.h"

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

// End of a single-workgroup ring launch (MsgSig). Every wave first waits for its own stores
// (answers written into mapped host memory, error atomics) to reach L2; then one lane publishes the
// error state and, behind a system-scope release (the L2 writes back what those stores left in it,
// and the lane waits for the write-backs -- plain stores to mapped host memory can sit in L2 until
// then), the ticket. Once the host sees the ticket, everything before it is in host memory. Called
// by every thread (workgroup-uniform `done`).
__device__ __forceinline__ void msg_signal(const MsgSig& g, const ErrState* err) {
  if (!g.done) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const u64 enc = __hip_atomic_load(&err->min_bad_enc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const u64 cnt = __hip_atomic_load(&err->count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&g.herr->min_bad_enc, enc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&g.herr->count, cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(g.done, g.ticket, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// address of a record; false when the JVM would throw ArrayIndexOutOfBoundsException
template <bool MAT, int KIND = -1>
__device__ __forceinline__ bool rec_addr(const PartDesc& p, i64 key, int32_t col, i64& addr) {
  const int32_t l = g2l<KIND>(p, key);
  bool ok = l >= 0 && l < p.size;
  if (MAT) {
    ok = ok && col >= 0 && col < p.cols;
    addr = (i64)l * p.pitch + (i64)col;
  } else {
    addr = (i64)l;
  }
  return ok;
}


// The 64-bit key itself lies in the partition's key range (no Int wrap): what RangePartitioner.partition
// checks (key < 0 || key >= size, RangePartitioner.scala:30) before the shard's (key - start).toInt
// (RangePartition.scala:33) could alias a key 2^32 away onto element key - start - 2^32. A validating
// push (GLINT_PUSH_VALIDATE) stands in for that check, so it tests the raw key too.
template <int KIND = -1>
__device__ __forceinline__ bool key_in_part(const PartDesc& p, i64 key) {
  if (KIND == 0 || (KIND < 0 && p.kind == 0)) return key >= p.start && key - p.start < (i64)p.size;
  return key >= (i64)p.cidx && (key - (i64)p.cidx) / (i64)p.cparts < (i64)p.size;
}

__device__ __forceinline__ void lds_add(double* p, double v) { unsafeAtomicAdd(p, v); }
__device__ __forceinline__ void lds_add(float* p, float v) { unsafeAtomicAdd(p, v); }
__device__ __forceinline__ void lds_add(long long* p, long long v) { atomicAdd((u64*)p, (u64)v); }
__device__ __forceinline__ void lds_add(int* p, int v) { atomicAdd((u32*)p, (u32)v); }

// Type of an LDS partial sum of V. Float shards accumulate in double: ds_add_f32 runs ~20x slower
// than ds_add_f64 on gfx950 (2.6 vs 0.12 cycles per lane per CU, tools/microbench_lds.hip,
// profiles/r01/mb_lds.txt), and a single record's sum stays exact, so a key pushed once still
// gets data + value rounded once, as PartialVector.scala:39 does.
template <typename V> struct LdsAcc { typedef V T; };
template <> struct LdsAcc<float> { typedef double T; };

// d + (LDS partial sum a), rounded once: float((double)d + a) equals the float sum d + v when a
// holds one float v (double carries > 2*24+2 bits, so the double rounding is innocuous)
__device__ __forceinline__ double acc_add(double d, double a) { return d + a; }
__device__ __forceinline__ float acc_add(float d, double a) { return (float)((double)d + a); }
__device__ __forceinline__ long long acc_add(long long d, long long a) { return vadd(d, a); }
__device__ __forceinline__ int acc_add(int d, int a) { return vadd(d, a); }

}  // namespace glint
