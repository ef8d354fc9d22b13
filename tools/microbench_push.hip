// Design-space microbenchmark for the push scatter-add (SURVEY.md §7 hard part (i)).
// Not part of the product: it measures, on gfx950, the primitives the push kernel can be built
// from, so the shipped kernel's structure is chosen from numbers rather than guesses.
//
//   copy        : 16 B/rec read + 16 B/rec write           (stream peak, calibration)
//   read_kv     : keys + values read only                  (16 B/rec)
//   rmw_plain   : keys+values read, data[k] += v plain RMW (32 B/rec)  -- requires unique keys
//   rmw_atomic  : same with global_atomic_add_f64          (32 B/rec algorithmic)
//   check       : keys read, strictly-increasing reduction (8 B/rec)
//   atomic_perm : atomic add with a random permutation of keys (scattered, unique)
//   atomic_zipf-like hot key: all records to 64 distinct keys (contention)
//
// Build: hipcc --offload-arch=gfx950 -O3 -o microbench_push tools/microbench_push.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <algorithm>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

typedef long long i64;
typedef __attribute__((ext_vector_type(2))) long long i64x2;
typedef __attribute__((ext_vector_type(2))) double f64x2;

template <int RPT>
__global__ __launch_bounds__(256) void k_copy(const f64x2* __restrict__ a, f64x2* __restrict__ b, i64 n2) {
  i64 tid = (i64)blockIdx.x * 256 + threadIdx.x;
  i64 stride = (i64)gridDim.x * 256;
  for (i64 i = tid; i < n2; i += stride) b[i] = __builtin_nontemporal_load(&a[i]);
}

template <int U>
__global__ __launch_bounds__(256) void k_read_kv(const i64x2* __restrict__ keys, const f64x2* __restrict__ vals,
                                                i64 n2, double* __restrict__ sink) {
  i64 tid = (i64)blockIdx.x * 256 + threadIdx.x;
  i64 stride = (i64)gridDim.x * 256;
  double acc = 0;
  for (i64 i = tid; i < n2; i += stride) {
    i64x2 k = __builtin_nontemporal_load(&keys[i]);
    f64x2 v = __builtin_nontemporal_load(&vals[i]);
    acc += (double)(k.x + k.y) + v.x + v.y;
  }
  if (acc == 12345.678) sink[0] = acc;
}

// plain RMW, 2 records per lane per iteration, contiguous fast path with 16-B data access
template <bool ATOMIC, bool NT>
__global__ __launch_bounds__(256) void k_rmw(const i64x2* __restrict__ keys, const f64x2* __restrict__ vals,
                                            i64 n2, double* __restrict__ data, i64 start) {
  i64 tid = (i64)blockIdx.x * 256 + threadIdx.x;
  i64 stride = (i64)gridDim.x * 256;
  for (i64 i = tid; i < n2; i += stride) {
    i64x2 k; f64x2 v;
    if (NT) { k = __builtin_nontemporal_load(&keys[i]); v = __builtin_nontemporal_load(&vals[i]); }
    else { k = keys[i]; v = vals[i]; }
    int l0 = (int)(k.x - start), l1 = (int)(k.y - start);
    if (ATOMIC) {
      unsafeAtomicAdd(&data[l0], v.x);
      unsafeAtomicAdd(&data[l1], v.y);
    } else {
      if (l1 == l0 + 1 && (l0 & 1) == 0) {
        f64x2* p = reinterpret_cast<f64x2*>(data + l0);
        f64x2 d = *p;
        d.x += v.x; d.y += v.y;
        *p = d;
      } else {
        data[l0] += v.x;
        data[l1] += v.y;
      }
    }
  }
}

// 4 records per lane per iteration (two 16-B loads each of keys/vals), more bytes in flight
template <bool ATOMIC>
__global__ __launch_bounds__(256) void k_rmw4(const i64x2* __restrict__ keys, const f64x2* __restrict__ vals,
                                             i64 n2, double* __restrict__ data, i64 start) {
  i64 tid = (i64)blockIdx.x * 256 + threadIdx.x;
  i64 stride = (i64)gridDim.x * 256;
  i64 i = tid;
  for (; i + stride < n2; i += 2 * stride) {
    i64x2 ka = __builtin_nontemporal_load(&keys[i]);
    i64x2 kb = __builtin_nontemporal_load(&keys[i + stride]);
    f64x2 va = __builtin_nontemporal_load(&vals[i]);
    f64x2 vb = __builtin_nontemporal_load(&vals[i + stride]);
    int a0 = (int)(ka.x - start), a1 = (int)(ka.y - start);
    int b0 = (int)(kb.x - start), b1 = (int)(kb.y - start);
    if (ATOMIC) {
      unsafeAtomicAdd(&data[a0], va.x); unsafeAtomicAdd(&data[a1], va.y);
      unsafeAtomicAdd(&data[b0], vb.x); unsafeAtomicAdd(&data[b1], vb.y);
    } else {
      if (a1 == a0 + 1 && (a0 & 1) == 0 && b1 == b0 + 1 && (b0 & 1) == 0) {
        f64x2* pa = reinterpret_cast<f64x2*>(data + a0);
        f64x2* pb = reinterpret_cast<f64x2*>(data + b0);
        f64x2 da = *pa, db = *pb;
        da += va; db += vb;
        *pa = da; *pb = db;
      } else {
        data[a0] += va.x; data[a1] += va.y; data[b0] += vb.x; data[b1] += vb.y;
      }
    }
  }
  for (; i < n2; i += stride) {
    i64x2 k = keys[i]; f64x2 v = vals[i];
    int l0 = (int)(k.x - start), l1 = (int)(k.y - start);
    if (ATOMIC) { unsafeAtomicAdd(&data[l0], v.x); unsafeAtomicAdd(&data[l1], v.y); }
    else { data[l0] += v.x; data[l1] += v.y; }
  }
}

__global__ __launch_bounds__(256) void k_check(const i64x2* __restrict__ keys, i64 n2, int* __restrict__ flag) {
  i64 tid = (i64)blockIdx.x * 256 + threadIdx.x;
  i64 stride = (i64)gridDim.x * 256;
  int bad = 0;
  const i64* k1 = reinterpret_cast<const i64*>(keys);
  for (i64 i = tid; i < n2; i += stride) {
    i64x2 k = __builtin_nontemporal_load(&keys[i]);
    i64 prev = i > 0 ? k1[2 * i - 1] : (i64)-1 << 62;
    bad |= (k.y <= k.x) | (k.x <= prev);
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

// scalar record-per-lane atomic (for scattered keys)
__global__ __launch_bounds__(256) void k_atomic1(const i64* __restrict__ keys, const double* __restrict__ vals,
                                                i64 n, double* __restrict__ data, i64 start) {
  i64 tid = (i64)blockIdx.x * 256 + threadIdx.x;
  i64 stride = (i64)gridDim.x * 256;
  for (i64 i = tid; i < n; i += stride) unsafeAtomicAdd(&data[(int)(keys[i] - start)], vals[i]);
}
__global__ __launch_bounds__(256) void k_plain1(const i64* __restrict__ keys, const double* __restrict__ vals,
                                               i64 n, double* __restrict__ data, i64 start) {
  i64 tid = (i64)blockIdx.x * 256 + threadIdx.x;
  i64 stride = (i64)gridDim.x * 256;
  for (i64 i = tid; i < n; i += stride) data[(int)(keys[i] - start)] += vals[i];
}

__global__ void k_fill_keys(i64* keys, i64 n, int mode, unsigned long long seed) {
  i64 tid = (i64)blockIdx.x * blockDim.x + threadIdx.x;
  i64 stride = (i64)gridDim.x * blockDim.x;
  for (i64 i = tid; i < n; i += stride) {
    if (mode == 0) keys[i] = i;
    else if (mode == 1) {  // bijective scatter: multiply by odd constant mod 2^m (n power of 2)
      unsigned long long x = (unsigned long long)i * 0x9E3779B97F4A7C15ull + seed;
      keys[i] = (i64)(x & (unsigned long long)(n - 1));  // not a permutation in general; fine for timing
    } else {
      keys[i] = (i * 2654435761ll) & 63;
    }
  }
}
__global__ void k_fill_vals(double* v, i64 n) {
  i64 tid = (i64)blockIdx.x * blockDim.x + threadIdx.x;
  i64 stride = (i64)gridDim.x * blockDim.x;
  for (i64 i = tid; i < n; i += stride) v[i] = (double)((i * 7919) % 1000) * 1e-3 - 0.5;
}

struct Timer {
  hipEvent_t a, b;
  Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
  float run(auto fn, int reps) {
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(a)); fn(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b)); t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
  }
};

int main(int argc, char** argv) {
  int lg = argc > 1 ? atoi(argv[1]) : 28;
  int reps = argc > 2 ? atoi(argv[2]) : 10;
  i64 n = 1ll << lg, n2 = n / 2;
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  printf("device %s CUs %d  n=2^%d\n", prop.gcnArchName, prop.multiProcessorCount, lg);
  i64 *keys; double *vals, *data, *sink; int* flag;
  CK(hipMalloc(&keys, n * 8)); CK(hipMalloc(&vals, n * 8)); CK(hipMalloc(&data, n * 8));
  CK(hipMalloc(&sink, 64)); CK(hipMalloc(&flag, 64));
  k_fill_keys<<<4096, 256>>>(keys, n, 0, 1); k_fill_vals<<<4096, 256>>>(vals, n);
  CK(hipMemset(data, 0, n * 8)); CK(hipDeviceSynchronize());
  Timer T;
  const double GB = 1e9;
  for (int grid : {1024, 2048, 4096, 8192, 16384}) {
    float t;
    t = T.run([&] { k_copy<1><<<grid, 256>>>((const f64x2*)vals, (f64x2*)data, n2); }, reps);
    printf("grid %5d copy        %8.3f ms %7.0f GB/s (16B/rec)\n", grid, t, 16.0 * n / t / 1e6);
    t = T.run([&] { k_read_kv<1><<<grid, 256>>>((const i64x2*)keys, (const f64x2*)vals, n2, sink); }, reps);
    printf("grid %5d read_kv     %8.3f ms %7.0f GB/s (16B/rec)\n", grid, t, 16.0 * n / t / 1e6);
    t = T.run([&] { k_rmw<false, true><<<grid, 256>>>((const i64x2*)keys, (const f64x2*)vals, n2, data, 0); }, reps);
    printf("grid %5d rmw_plainNT %8.3f ms %7.0f GB/s (32B/rec)\n", grid, t, 32.0 * n / t / 1e6);
    t = T.run([&] { k_rmw<false, false><<<grid, 256>>>((const i64x2*)keys, (const f64x2*)vals, n2, data, 0); }, reps);
    printf("grid %5d rmw_plain   %8.3f ms %7.0f GB/s (32B/rec)\n", grid, t, 32.0 * n / t / 1e6);
    t = T.run([&] { k_rmw4<false><<<grid, 256>>>((const i64x2*)keys, (const f64x2*)vals, n2, data, 0); }, reps);
    printf("grid %5d rmw4_plain  %8.3f ms %7.0f GB/s (32B/rec)\n", grid, t, 32.0 * n / t / 1e6);
    t = T.run([&] { k_rmw<true, true><<<grid, 256>>>((const i64x2*)keys, (const f64x2*)vals, n2, data, 0); }, reps);
    printf("grid %5d rmw_atomic  %8.3f ms %7.0f GB/s (32B/rec)\n", grid, t, 32.0 * n / t / 1e6);
    t = T.run([&] { k_rmw4<true><<<grid, 256>>>((const i64x2*)keys, (const f64x2*)vals, n2, data, 0); }, reps);
    printf("grid %5d rmw4_atomic %8.3f ms %7.0f GB/s (32B/rec)\n", grid, t, 32.0 * n / t / 1e6);
    t = T.run([&] { k_check<<<grid, 256>>>((const i64x2*)keys, n2, flag); }, reps);
    printf("grid %5d check       %8.3f ms %7.0f GB/s (8B/rec)\n", grid, t, 8.0 * n / t / 1e6);
  }
  // scattered
  k_fill_keys<<<4096, 256>>>(keys, n, 1, 7); CK(hipDeviceSynchronize());
  for (int grid : {2048, 8192}) {
    float t = T.run([&] { k_atomic1<<<grid, 256>>>(keys, vals, n, data, 0); }, reps);
    printf("grid %5d atomic_scat %8.3f ms %7.0f GB/s (32B/rec) %7.2f Gop/s\n", grid, t, 32.0 * n / t / 1e6, n / t / 1e6);
    t = T.run([&] { k_plain1<<<grid, 256>>>(keys, vals, n, data, 0); }, reps);
    printf("grid %5d plain_scat  %8.3f ms %7.0f GB/s (32B/rec) %7.2f Gop/s\n", grid, t, 32.0 * n / t / 1e6, n / t / 1e6);
  }
  k_fill_keys<<<4096, 256>>>(keys, n, 2, 7); CK(hipDeviceSynchronize());
  {
    i64 nn = n / 16;
    float t = T.run([&] { k_atomic1<<<2048, 256>>>(keys, vals, nn, data, 0); }, 3);
    printf("atomic_hot64 (n/16) %8.3f ms %7.2f Gop/s\n", t, nn / t / 1e6);
  }
  CK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
