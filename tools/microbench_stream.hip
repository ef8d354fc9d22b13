// Streaming-shape sweep for the dense push (push_check = 1 read stream, push_apply sweep = 2 reads +
// 1 write stream): pairs per lane in flight, blocks per CU, grid-stride vs per-block chunking, and
// the cache policy of each access. Not part of the product. Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/microbench_stream tools/microbench_stream.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

typedef long long i64;
typedef __attribute__((ext_vector_type(2))) double D2;
typedef __attribute__((ext_vector_type(2))) long long K2;

// load/store policy: 0 default, 1 nontemporal
template <int P, typename T> __device__ __forceinline__ T ld(const T* p) {
  if (P == 1) return __builtin_nontemporal_load(p);
  return *p;
}
template <int P, typename T> __device__ __forceinline__ void st(T* p, T v) {
  if (P == 1) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// 2 reads + 1 write: data[p] += vals[p]   (16 B per lane per access)
// CHUNK=0: grid-stride, the U pairs of one iteration are one grid stride apart
// CHUNK=1: per-block tiles of 256*U pairs, block-strided
template <int U, int CHUNK, int LV, int LD, int SD, int TPB = 256>
__global__ __launch_bounds__(TPB) void k_apply(const D2* __restrict__ vals, D2* __restrict__ data, i64 n2) {
  if (CHUNK == 0) {
    const i64 stride = (i64)gridDim.x * TPB;
    i64 p = (i64)blockIdx.x * TPB + threadIdx.x;
    for (; p + (U - 1) * stride < n2; p += U * stride) {
      D2 v[U], d[U];
#pragma unroll
      for (int j = 0; j < U; ++j) { v[j] = ld<LV>(vals + p + j * stride); d[j] = ld<LD>(data + p + j * stride); }
#pragma unroll
      for (int j = 0; j < U; ++j) st<SD>(data + p + j * stride, d[j] + v[j]);
    }
    for (; p < n2; p += stride) data[p] = data[p] + vals[p];
  } else {
    const i64 ntile = n2 / (TPB * U);
    for (i64 t = blockIdx.x; t < ntile; t += gridDim.x) {
      const i64 b = t * TPB * U + threadIdx.x;
      D2 v[U], d[U];
#pragma unroll
      for (int j = 0; j < U; ++j) { v[j] = ld<LV>(vals + b + j * TPB); d[j] = ld<LD>(data + b + j * TPB); }
#pragma unroll
      for (int j = 0; j < U; ++j) st<SD>(data + b + j * TPB, d[j] + v[j]);
    }
  }
}

// fused speculative push: keys + values + shard RMW in one pass (32 B/record); a tile is applied
// only if its keys are affine (key = key0 + record); else a flag is raised for a fallback pass
template <int U, int TPB>
__global__ __launch_bounds__(TPB) void k_fused(const K2* __restrict__ keys, const D2* __restrict__ vals,
                                               D2* __restrict__ data, i64 n2, unsigned* flag) {
  const i64 k0 = reinterpret_cast<const i64*>(keys)[0];
  const i64 stride = (i64)gridDim.x * TPB;
  i64 p = (i64)blockIdx.x * TPB + threadIdx.x;
  for (; p + (U - 1) * stride < n2; p += U * stride) {
    K2 k[U];
    D2 v[U], d[U];
#pragma unroll
    for (int j = 0; j < U; ++j) k[j] = __builtin_nontemporal_load(keys + p + j * stride);
#pragma unroll
    for (int j = 0; j < U; ++j) {
      v[j] = __builtin_nontemporal_load(vals + p + j * stride);
      d[j] = __builtin_nontemporal_load(data + p + j * stride);
    }
    bool ok = true;
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const i64 r = 2 * (p + j * stride);
      ok = ok && k[j].x == k0 + r && k[j].y == k0 + r + 1;
    }
    if (__all(ok)) {
#pragma unroll
      for (int j = 0; j < U; ++j) __builtin_nontemporal_store(d[j] + v[j], data + p + j * stride);
    } else if ((threadIdx.x & 63) == 0) {
      atomicOr(flag, 1u);
    }
  }
}

// 1 read: the key stream of push_check
template <int U, int CHUNK, int LK>
__global__ __launch_bounds__(256) void k_read(const K2* __restrict__ keys, i64 n2, i64* sink) {
  i64 acc = 0;
  if (CHUNK == 0) {
    const i64 stride = (i64)gridDim.x * 256;
    for (i64 p = (i64)blockIdx.x * 256 + threadIdx.x; p + (U - 1) * stride < n2; p += U * stride) {
      K2 k[U];
#pragma unroll
      for (int j = 0; j < U; ++j) k[j] = ld<LK>(keys + p + j * stride);
#pragma unroll
      for (int j = 0; j < U; ++j) acc += k[j].x ^ k[j].y;
    }
  } else {
    const i64 ntile = n2 / (256 * U);
    for (i64 t = blockIdx.x; t < ntile; t += gridDim.x) {
      const i64 b = t * 256 * U + threadIdx.x;
      K2 k[U];
#pragma unroll
      for (int j = 0; j < U; ++j) k[j] = ld<LK>(keys + b + j * 256);
#pragma unroll
      for (int j = 0; j < U; ++j) acc += k[j].x ^ k[j].y;
    }
  }
  if (acc == 42) sink[0] = acc;
}

// 1 read, block tiles of TPB*U pairs (push_check's shape)
template <int U, int TPB>
__global__ __launch_bounds__(TPB) void k_read3(const K2* __restrict__ keys, i64 n2, i64* sink) {
  i64 acc = 0;
  const i64 ntile = n2 / (TPB * U);
  for (i64 t = blockIdx.x; t < ntile; t += gridDim.x) {
    const i64 b = t * TPB * U + threadIdx.x;
    K2 k[U];
#pragma unroll
    for (int j = 0; j < U; ++j) k[j] = __builtin_nontemporal_load(keys + b + j * TPB);
#pragma unroll
    for (int j = 0; j < U; ++j) acc += k[j].x ^ k[j].y;
  }
  if (acc == 42) sink[0] = acc;
}

// dense pull: out[p] = data[key[p] - k0] (dependent gather, 24 B/record)
template <int U, int LD, int SO>
__global__ __launch_bounds__(256) void k_pull(const K2* __restrict__ keys, const double* __restrict__ data,
                                              D2* __restrict__ out, i64 n2, i64 k0) {
  const i64 stride = (i64)gridDim.x * 256;
  i64 p = (i64)blockIdx.x * 256 + threadIdx.x;
  for (; p + (U - 1) * stride < n2; p += U * stride) {
    K2 k[U];
    D2 o[U];
#pragma unroll
    for (int j = 0; j < U; ++j) k[j] = __builtin_nontemporal_load(keys + p + j * stride);
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const i64 l0 = k[j].x - k0, l1 = k[j].y - k0;
      if (l1 == l0 + 1 && (l0 & 1) == 0) o[j] = ld<LD>(reinterpret_cast<const D2*>(data + l0));
      else o[j] = D2{data[l0], data[l1]};
    }
#pragma unroll
    for (int j = 0; j < U; ++j) st<SO>(out + p + j * stride, o[j]);
  }
}

// copy (1R + 1W) for the guide's float4-copy comparison
template <int U, int LV, int SD>
__global__ __launch_bounds__(256) void k_copy(const D2* __restrict__ src, D2* __restrict__ dst, i64 n2) {
  const i64 stride = (i64)gridDim.x * 256;
  for (i64 p = (i64)blockIdx.x * 256 + threadIdx.x; p + (U - 1) * stride < n2; p += U * stride) {
    D2 v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = ld<LV>(src + p + j * stride);
#pragma unroll
    for (int j = 0; j < U; ++j) st<SD>(dst + p + j * stride, v[j]);
  }
}

__global__ void k_iota(i64* keys, i64 n) {
  for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x) keys[i] = i + 5;
}

template <class F>
float timeit(F fn, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  std::vector<float> t;
  fn(); fn();
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a)); fn(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 28;
  const int reps = argc > 2 ? atoi(argv[2]) : 9;
  const i64 n = 1ll << lg, n2 = n / 2;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  double *vals, *data;
  i64* keys;
  CK(hipMalloc(&keys, n * 8)); CK(hipMalloc(&vals, n * 8)); CK(hipMalloc(&data, n * 8));
  CK(hipMemset(keys, 1, n * 8)); CK(hipMemset(vals, 0, n * 8)); CK(hipMemset(data, 0, n * 8));
  CK(hipDeviceSynchronize());
  printf("cus %d, n 2^%d\n", cus, lg);
  const D2* V = (const D2*)vals;
  D2* Dd = (D2*)data;
  const int mode = argc > 3 ? atoi(argv[3]) : 0;
#define APPLY(U, C, LV, LD, SD)                                                                   \
  for (int bpc : {1, 2, 4, 8}) {                                                                  \
    const int g = cus * bpc;                                                                      \
    const float ms = timeit([&] { k_apply<U, C, LV, LD, SD><<<g, 256>>>(V, Dd, n2); }, reps);      \
    printf("apply U%d chunk%d lv%d ld%d sd%d bpc %d: %7.3f ms %6.0f GB/s\n", U, C, LV, LD, SD, bpc, \
           ms, 24.0 * n / ms / 1e6);                                                              \
  }
#define APPLY2(U, C, TPB)                                                                         \
  for (int g : {cus / 2, cus * 3 / 4, cus, cus * 3 / 2, cus * 2}) {                               \
    const float ms = timeit([&] { k_apply<U, C, 1, 1, 1, TPB><<<g, TPB>>>(V, Dd, n2); }, reps);   \
    printf("apply-nt U%d chunk%d tpb %d grid %d: %7.3f ms %6.0f GB/s\n", U, C, TPB, g, ms,         \
           24.0 * n / ms / 1e6);                                                                  \
  }
#define FUSED(U, TPB)                                                                             \
  for (int g : {cus / 2, cus * 3 / 4, cus, cus * 3 / 2, cus * 2, cus * 4}) {                      \
    const float ms = timeit([&] { k_fused<U, TPB><<<g, TPB>>>((const K2*)keys, V, Dd, n2, flag); }, reps); \
    printf("fused U%d tpb %d grid %d: %7.3f ms %6.0f GB/s\n", U, TPB, g, ms, 32.0 * n / ms / 1e6);  \
  }
  if (mode == 2) {
    unsigned* flag;
    CK(hipMalloc(&flag, 4));
    k_iota<<<4096, 256>>>(keys, n);
    FUSED(1, 256) FUSED(2, 256) FUSED(4, 256) FUSED(8, 256)
    FUSED(2, 512) FUSED(4, 512) FUSED(2, 1024) FUSED(4, 128) FUSED(8, 128)
    unsigned h = 0;
    CK(hipMemcpy(&h, flag, 4, hipMemcpyDeviceToHost));
    printf("flag %u\ndone\n", h);
    return 0;
  }
#define APPLY3(U, TPB, LV, LD, SD)                                                                \
  for (int g : {cus / 2, cus, cus * 2}) {                                                         \
    const float ms = timeit([&] { k_apply<U, 0, LV, LD, SD, TPB><<<g, TPB>>>(V, Dd, n2); }, reps); \
    printf("apply U%d tpb %d grid %d pol %d%d%d: %7.3f ms %6.0f GB/s\n", U, TPB, g, LV, LD, SD, ms,  \
           24.0 * n / ms / 1e6);                                                                  \
  }
#define APPLY3P(U, TPB) APPLY3(U, TPB, 1, 0, 0) APPLY3(U, TPB, 1, 1, 1) APPLY3(U, TPB, 1, 0, 1)
  if (mode == 3) {
    APPLY3P(2, 64) APPLY3P(4, 64) APPLY3P(8, 64)
    APPLY3P(2, 128) APPLY3P(4, 128) APPLY3P(8, 128)
    APPLY3P(2, 256) APPLY3P(4, 256) APPLY3P(8, 256)
    printf("done\n");
    return 0;
  }
#define READ3(U, TPB)                                                                             \
  for (int g : {cus / 2, cus, cus * 2, cus * 4, cus * 8}) {                                       \
    const float ms = timeit([&] { k_read3<U, TPB><<<g, TPB>>>((const K2*)keys, n2, keys); }, reps); \
    printf("read U%d tpb %d grid %d: %7.3f ms %6.0f GB/s\n", U, TPB, g, ms, 8.0 * n / ms / 1e6);   \
  }
  if (mode == 4) {
    READ3(4, 64) READ3(8, 64) READ3(16, 64)
    READ3(4, 128) READ3(8, 128) READ3(16, 128)
    READ3(4, 256) READ3(8, 256) READ3(16, 256)
    READ3(4, 512) READ3(8, 512)
    printf("done\n");
    return 0;
  }
#define PULL(U, LD, SO)                                                                           \
  for (int g : {cus, cus * 2, cus * 4, cus * 8}) {                                                \
    const float ms = timeit([&] { k_pull<U, LD, SO><<<g, 256>>>((const K2*)keys, data, (D2*)vals, n2, 5); }, reps); \
    printf("pull U%d ld%d so%d grid %d: %7.3f ms %6.0f GB/s\n", U, LD, SO, g, ms, 24.0 * n / ms / 1e6); \
  }
  if (mode == 5) {
    k_iota<<<4096, 256>>>(keys, n);
    PULL(1, 0, 0) PULL(1, 1, 1) PULL(1, 0, 1) PULL(2, 0, 0) PULL(2, 1, 1) PULL(2, 0, 1)
    PULL(4, 0, 0) PULL(4, 1, 1) PULL(4, 0, 1) PULL(4, 1, 0)
    printf("done\n");
    return 0;
  }
  if (mode == 6) {
    // the push_apply sweep's shape (2 pairs per lane, all non-temporal, one 256-thread block per
    // CU) at 2^26..2^lg records: whole, in 2^28-record launches, and with the value stream shifted
    // against the shard stream -- why does 2^30 run slower per byte than 2^28?
    double *v2, *d2;
    CK(hipMalloc(&v2, n * 8 + (64 << 20)));
    CK(hipMalloc(&d2, n * 8 + (64 << 20)));
    CK(hipMemset(v2, 0, n * 8 + (64 << 20)));
    CK(hipMemset(d2, 0, n * 8 + (64 << 20)));
    CK(hipDeviceSynchronize());
    printf("vals %p data %p (delta %lld MiB)\n", (void*)v2, (void*)d2, (long long)(((char*)d2 - (char*)v2) >> 20));
    for (int l = 26; l <= lg; ++l) {
      const i64 m2 = (1ll << l) / 2;
      const float ms = timeit([&] { k_apply<2, 0, 1, 1, 1, 256><<<cus, 256>>>((const D2*)v2, (D2*)d2, m2); }, reps);
      printf("sweep 2^%d whole: %7.3f ms %6.0f GB/s\n", l, ms, 24.0 * (2 * m2) / ms / 1e6);
    }
    for (int cl : {26, 27, 28, 29}) {
      if (cl >= lg) continue;
      const i64 c2 = (1ll << cl) / 2;
      const float ms = timeit([&] {
        for (i64 o = 0; o < n2; o += c2)
          k_apply<2, 0, 1, 1, 1, 256><<<cus, 256>>>((const D2*)v2 + o, (D2*)d2 + o, std::min(c2, n2 - o));
      }, reps);
      printf("sweep 2^%d in 2^%d launches: %7.3f ms %6.0f GB/s\n", lg, cl, ms, 24.0 * n / ms / 1e6);
    }
    for (i64 shift : {4096ll, 65536ll, 1ll << 20, (2ll << 20) + 4096, (16ll << 20) + 65536}) {
      const float ms = timeit([&] {
        k_apply<2, 0, 1, 1, 1, 256><<<cus, 256>>>((const D2*)((char*)v2 + shift), (D2*)d2, n2);
      }, reps);
      printf("sweep 2^%d vals shifted +%lld B: %7.3f ms %6.0f GB/s\n", lg, (long long)shift, ms, 24.0 * n / ms / 1e6);
    }
    for (int g : {cus / 2, cus, cus * 2}) {
      const float ms = timeit([&] { k_apply<4, 0, 1, 1, 1, 256><<<g, 256>>>((const D2*)v2, (D2*)d2, n2); }, reps);
      printf("sweep 2^%d U4 grid %d: %7.3f ms %6.0f GB/s\n", lg, g, ms, 24.0 * n / ms / 1e6);
    }
    printf("done\n");
    return 0;
  }
  if (mode == 1) {
    APPLY2(2, 0, 256) APPLY2(4, 0, 256) APPLY2(8, 0, 256) APPLY2(16, 0, 256)
    APPLY2(4, 1, 256) APPLY2(8, 1, 256) APPLY2(16, 1, 256)
    APPLY2(4, 0, 128) APPLY2(8, 0, 128) APPLY2(16, 0, 128)
    APPLY2(2, 0, 512) APPLY2(4, 0, 512) APPLY2(8, 0, 512)
    APPLY2(2, 0, 1024) APPLY2(4, 0, 1024)
    APPLY2(4, 1, 512) APPLY2(8, 1, 512) APPLY2(4, 1, 1024)
    printf("done\n");
    return 0;
  }

  APPLY(1, 0, 1, 0, 0)
  APPLY(2, 0, 1, 0, 0)
  APPLY(4, 0, 1, 0, 0)
  APPLY(8, 0, 1, 0, 0)
  APPLY(2, 1, 1, 0, 0)
  APPLY(4, 1, 1, 0, 0)
  APPLY(8, 1, 1, 0, 0)
  APPLY(4, 0, 0, 0, 0)
  APPLY(4, 0, 1, 1, 0)
  APPLY(4, 0, 1, 0, 1)
  APPLY(4, 0, 1, 1, 1)
  APPLY(1, 0, 1, 0, 1)
  APPLY(2, 0, 1, 0, 1)
  APPLY(4, 1, 1, 0, 1)
#define READ(U, C, LK)                                                                          \
  for (int bpc : {2, 4, 8, 16}) {                                                               \
    const int g = cus * bpc;                                                                    \
    const float ms = timeit([&] { k_read<U, C, LK><<<g, 256>>>((const K2*)keys, n2, keys); }, reps); \
    printf("read U%d chunk%d lk%d bpc %d: %7.3f ms %6.0f GB/s\n", U, C, LK, bpc, ms, 8.0 * n / ms / 1e6); \
  }
  READ(2, 0, 1)
  READ(4, 0, 1)
  READ(8, 0, 1)
  READ(16, 0, 1)
  READ(4, 1, 1)
  READ(8, 1, 1)
  READ(16, 1, 1)
  READ(8, 0, 0)
#define COPY(U, LV, SD)                                                                          \
  for (int bpc : {2, 4, 8}) {                                                                    \
    const int g = cus * bpc;                                                                     \
    const float ms = timeit([&] { k_copy<U, LV, SD><<<g, 256>>>(V, Dd, n2); }, reps);            \
    printf("copy U%d lv%d sd%d bpc %d: %7.3f ms %6.0f GB/s\n", U, LV, SD, bpc, ms, 16.0 * n / ms / 1e6); \
  }
  COPY(1, 1, 0)
  COPY(4, 1, 0)
  COPY(4, 1, 1)
  COPY(4, 0, 0)
  printf("done\n");
  return 0;
}
