// Design-space microbenchmark for push_apply (the ordered plain-RMW push): which structure gets
// closest to the HBM roofline for 32 B/record (key 8 + value 8 + shard read 8 + shard write 8)?
// Not part of the product. Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o tools/microbench_apply tools/microbench_apply.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

typedef long long i64;
typedef __attribute__((ext_vector_type(2))) long long K2;
typedef __attribute__((ext_vector_type(2))) double D2;

// stream4: no dependent load -- the address is the record index (upper bound for the access mix)
__global__ __launch_bounds__(256) void k_stream4(const K2* __restrict__ keys, const D2* __restrict__ vals,
                                                D2* __restrict__ data, i64 n2) {
  const i64 stride = (i64)gridDim.x * 256;
  for (i64 i = (i64)blockIdx.x * 256 + threadIdx.x; i < n2; i += stride) {
    const K2 k = __builtin_nontemporal_load(&keys[i]);
    const D2 v = __builtin_nontemporal_load(&vals[i]);
    D2 d = data[i];
    d += v;
    d.x += (double)(k.x & 1) * 0.0;
    data[i] = d;
  }
}

// stream3: values + shard RMW only (the affine apply: no keys read)
__global__ __launch_bounds__(256) void k_stream3(const D2* __restrict__ vals, D2* __restrict__ data, i64 n2) {
  const i64 stride = (i64)gridDim.x * 256;
  for (i64 i = (i64)blockIdx.x * 256 + threadIdx.x; i < n2; i += stride) {
    const D2 v = __builtin_nontemporal_load(&vals[i]);
    D2 d = data[i];
    d += v;
    data[i] = d;
  }
}
// stream3 with two pairs per iteration (the product's apply_stream)
__global__ __launch_bounds__(256) void k_stream3x2(const D2* __restrict__ vals, D2* __restrict__ data, i64 n2) {
  const i64 stride = (i64)gridDim.x * 256;
  i64 p = (i64)blockIdx.x * 256 + threadIdx.x;
  for (; p + stride < n2; p += 2 * stride) {
    const D2 v0 = __builtin_nontemporal_load(&vals[p]);
    const D2 v1 = __builtin_nontemporal_load(&vals[p + stride]);
    const D2 d0 = data[p];
    const D2 d1 = data[p + stride];
    data[p] = d0 + v0;
    data[p + stride] = d1 + v1;
  }
  for (; p < n2; p += stride) data[p] = data[p] + __builtin_nontemporal_load(&vals[p]);
}
// pure read of one stream (push_check's traffic)
__global__ __launch_bounds__(256) void k_read1(const K2* __restrict__ keys, i64 n2, i64* sink) {
  const i64 stride = (i64)gridDim.x * 256;
  i64 acc = 0;
  for (i64 i = (i64)blockIdx.x * 256 + threadIdx.x; i < n2; i += stride) {
    const K2 k = __builtin_nontemporal_load(&keys[i]);
    acc += k.x ^ k.y;
  }
  if (acc == 42) sink[0] = acc;
}

// grid-stride, PPT pairs per thread per iteration, dependent shard access
template <int PPT, bool NTST>
__global__ __launch_bounds__(256) void k_rmw(const K2* __restrict__ keys, const D2* __restrict__ vals,
                                            double* __restrict__ data, i64 n2) {
  const i64 stride = (i64)gridDim.x * 256;
  for (i64 i0 = (i64)blockIdx.x * 256 + threadIdx.x; i0 < n2; i0 += stride * PPT) {
    K2 k[PPT];
    D2 v[PPT];
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
      const i64 i = i0 + j * stride;
      if (i < n2) { k[j] = __builtin_nontemporal_load(&keys[i]); v[j] = __builtin_nontemporal_load(&vals[i]); }
      else { k[j] = K2{-1, -1}; v[j] = D2{0, 0}; }
    }
    D2 d[PPT];
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
      const int a0 = (int)k[j].x;
      if (k[j].x >= 0) d[j] = *reinterpret_cast<const D2*>(data + a0);
    }
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
      const int a0 = (int)k[j].x;
      if (k[j].x >= 0) {
        D2 r = d[j] + v[j];
        if (NTST) __builtin_nontemporal_store(r, reinterpret_cast<D2*>(data + a0));
        else *reinterpret_cast<D2*>(data + a0) = r;
      }
    }
  }
}

// tile-based (the product's push_apply layout): tile = 256 threads x PPT pairs, block-strided
template <int PPT>
__global__ __launch_bounds__(256) void k_tile(const K2* __restrict__ keys, const D2* __restrict__ vals,
                                             double* __restrict__ data, i64 n2) {
  const i64 ntiles = (n2 + 256 * PPT - 1) / (256 * PPT);
  for (i64 t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const i64 base = t * 256 * PPT + threadIdx.x;
    K2 k[PPT];
    D2 v[PPT];
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
      const i64 i = base + j * 256;
      if (i < n2) { k[j] = __builtin_nontemporal_load(&keys[i]); v[j] = __builtin_nontemporal_load(&vals[i]); }
      else { k[j] = K2{-1, -1}; v[j] = D2{0, 0}; }
    }
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
      const int a0 = (int)k[j].x;
      if (k[j].x >= 0) {
        D2* p = reinterpret_cast<D2*>(data + a0);
        D2 d = *p;
        *p = d + v[j];
      }
    }
  }
}

__global__ void k_fill(i64* keys, double* v, i64 n) {
  const i64 stride = (i64)gridDim.x * blockDim.x;
  for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    keys[i] = i;
    v[i] = (double)((i * 7919) % 1000) * 1e-3 - 0.5;
  }
}

template <class F>
float timeit(F fn, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  std::vector<float> t;
  fn();
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a)); fn(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 28;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  const i64 n = 1ll << lg, n2 = n / 2;
  i64* keys; double *vals, *data;
  CK(hipMalloc(&keys, n * 8)); CK(hipMalloc(&vals, n * 8)); CK(hipMalloc(&data, n * 8));
  k_fill<<<4096, 256>>>(keys, vals, n);
  CK(hipMemset(data, 0, n * 8));
  CK(hipDeviceSynchronize());
  const double B = 32.0 * n;
  auto rep = [&](const char* name, int grid, float ms) {
    printf("%-14s grid %6d  %8.3f ms  %7.0f GB/s\n", name, grid, ms, B / ms / 1e6);
  };
  const K2* K = (const K2*)keys;
  const D2* Vv = (const D2*)vals;
  for (int g : {512, 1024, 2048}) {
    rep("stream4", g, timeit([&] { k_stream4<<<g, 256>>>(K, Vv, (D2*)data, n2); }, reps));
  }
  for (int g : {256, 512, 1024, 2048}) {
    const float ms = timeit([&] { k_stream3<<<g, 256>>>(Vv, (D2*)data, n2); }, reps);
    printf("%-14s grid %6d  %8.3f ms  %7.0f GB/s actual (24B/rec)\n", "stream3", g, ms, 24.0 * n / ms / 1e6);
    const float ms2 = timeit([&] { k_stream3x2<<<g, 256>>>(Vv, (D2*)data, n2); }, reps);
    printf("%-14s grid %6d  %8.3f ms  %7.0f GB/s actual (24B/rec)\n", "stream3x2", g, ms2, 24.0 * n / ms2 / 1e6);
    const float ms3 = timeit([&] { k_read1<<<g, 256>>>(K, n2, keys); }, reps);
    printf("%-14s grid %6d  %8.3f ms  %7.0f GB/s actual (8B/rec)\n", "read1", g, ms3, 8.0 * n / ms3 / 1e6);
  }
  for (int g : {512, 1024, 2048, 4096}) {
    rep("rmw_p1", g, timeit([&] { k_rmw<1, false><<<g, 256>>>(K, Vv, data, n2); }, reps));
    rep("rmw_p2", g, timeit([&] { k_rmw<2, false><<<g, 256>>>(K, Vv, data, n2); }, reps));
    rep("rmw_p4", g, timeit([&] { k_rmw<4, false><<<g, 256>>>(K, Vv, data, n2); }, reps));
    rep("rmw_p1_ntst", g, timeit([&] { k_rmw<1, true><<<g, 256>>>(K, Vv, data, n2); }, reps));
    rep("rmw_p2_ntst", g, timeit([&] { k_rmw<2, true><<<g, 256>>>(K, Vv, data, n2); }, reps));
  }
  for (int g : {512, 1024, 2048}) {
    rep("tile_p2", g, timeit([&] { k_tile<2><<<g, 256>>>(K, Vv, data, n2); }, reps));
    rep("tile_p4", g, timeit([&] { k_tile<4><<<g, 256>>>(K, Vv, data, n2); }, reps));
    rep("tile_p8", g, timeit([&] { k_tile<8><<<g, 256>>>(K, Vv, data, n2); }, reps));
  }
  printf("done\n");
  return 0;
}
