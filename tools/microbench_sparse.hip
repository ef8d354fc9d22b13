// Practical floors for the sparse pushes (cfg3 / cfg4b / cfg5), measured on the box -- not part of the
// product. A binned push must at least (a) stream its records once and (b) read-modify-write every
// distinct element it touches once. This times both parts in their best shapes:
//   read      n records of 16 B (key + value), streamed once (non-temporal 16-B loads)
//   rmw_sorted  U distinct random elements of the shard, visited in ascending order, data[e] += v
//              (plain RMW: the best locality a perfect sort could give -- lines shared by touched
//              elements are fetched once)
//   rmw_random  the same U elements in random order (what an unsorted scatter pays)
// floor = read + rmw_sorted: the time a binned push would take if partitioning were free.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench_sparse tools/microbench_sparse.hip
// Run:   tools/microbench_sparse   (cfg3: 2^26 records, 7.78 M distinct of 2^28; cfg4b: 2^26 / 59.2 M
//        of 2^28; cfg5: 2^23 / 3.54 M of 2^26 -- U from the bench lines' post-run checks; cfg4_mps8_shard:
//        one of the eight 2^23-record shard pushes of the cfg4 key space on one GPU, 8.26 M of 2^28)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

typedef long long i64;
typedef __attribute__((ext_vector_type(2))) long long i64x2;
typedef __attribute__((ext_vector_type(2))) double f64x2;

__global__ __launch_bounds__(256) void k_read(const i64x2* __restrict__ k, const f64x2* __restrict__ v, i64 n2,
                                              double* sink) {
  double acc = 0;
  for (i64 i = (i64)blockIdx.x * 256 + threadIdx.x; i < n2; i += (i64)gridDim.x * 256) {
    const i64x2 a = __builtin_nontemporal_load(&k[i]);
    const f64x2 b = __builtin_nontemporal_load(&v[i]);
    acc += (double)(a.x ^ a.y) * 1e-30 + b.x + b.y;
  }
  if (acc == 12345.678) sink[0] = acc;  // keeps the loads
}

__global__ __launch_bounds__(256) void k_rmw(const uint32_t* __restrict__ e, const double* __restrict__ v, i64 u,
                                             double* __restrict__ data) {
  for (i64 i = (i64)blockIdx.x * 256 + threadIdx.x; i < u; i += (i64)gridDim.x * 256) {
    const uint32_t x = __builtin_nontemporal_load(&e[i]);
    data[x] += __builtin_nontemporal_load(&v[i]);
  }
}

struct Timer {
  hipEvent_t a, b;
  Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
  template <typename F> float run(F f, int reps) {
    f();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(a));
      f();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      best = std::min(best, ms);
    }
    return best;
  }
};

static void run_case(const char* name, int lg_shard, i64 n, i64 u, int cus) {
  const i64 size = 1ll << lg_shard;
  // U distinct elements, chosen uniformly (Bernoulli by a hash), ascending
  std::vector<uint32_t> el;
  el.reserve((size_t)(u * 1.01) + 16);
  const double p = (double)u / (double)size;
  const uint64_t thr = (uint64_t)(p * 4294967296.0);
  for (i64 x = 0; x < size; ++x) {
    uint64_t h = (uint64_t)x * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 32;
    if ((h & 0xFFFFFFFFull) < thr) el.push_back((uint32_t)x);
  }
  const i64 U = (i64)el.size();
  std::vector<uint32_t> shuf(el);
  std::mt19937_64 rng(42);
  std::shuffle(shuf.begin(), shuf.end(), rng);
  i64* keys;
  double *vals, *data, *sink;
  uint32_t *e_sorted, *e_random;
  CK(hipMalloc(&keys, n * 8));
  CK(hipMalloc(&vals, std::max(n, U) * 8));
  CK(hipMalloc(&data, size * 8));
  CK(hipMalloc(&sink, 64));
  CK(hipMalloc(&e_sorted, U * 4));
  CK(hipMalloc(&e_random, U * 4));
  CK(hipMemset(keys, 1, n * 8));
  CK(hipMemset(vals, 0, std::max(n, U) * 8));
  CK(hipMemset(data, 0, size * 8));
  CK(hipMemcpy(e_sorted, el.data(), U * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(e_random, shuf.data(), U * 4, hipMemcpyHostToDevice));
  Timer T;
  const unsigned grid = (unsigned)cus * 8;
  const float t_read = T.run([&] { k_read<<<grid, 256>>>((const i64x2*)keys, (const f64x2*)vals, n / 2, sink); }, 5);
  const float t_sorted = T.run([&] { k_rmw<<<grid, 256>>>(e_sorted, vals, U, data); }, 5);
  const float t_random = T.run([&] { k_rmw<<<grid, 256>>>(e_random, vals, U, data); }, 5);
  printf("{\"case\": \"%s\", \"shard_elems\": %lld, \"records\": %lld, \"distinct\": %lld, \"read_ms\": %.4f, "
         "\"read_GBps\": %.0f, \"rmw_sorted_ms\": %.4f, \"rmw_sorted_Gelem_per_s\": %.2f, \"rmw_random_ms\": %.4f, "
         "\"rmw_random_Gelem_per_s\": %.2f, \"floor_ms\": %.4f}\n",
         name, (long long)size, (long long)n, (long long)U, t_read, 16.0 * n / t_read / 1e6, t_sorted,
         U / t_sorted / 1e6, t_random, U / t_random / 1e6, t_read + t_sorted);
  CK(hipFree(keys));
  CK(hipFree(vals));
  CK(hipFree(data));
  CK(hipFree(sink));
  CK(hipFree(e_sorted));
  CK(hipFree(e_random));
}

int main() {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  run_case("cfg3", 28, 1ll << 26, 7780619, prop.multiProcessorCount);
  run_case("cfg4b", 28, 1ll << 26, 59236000, prop.multiProcessorCount);
  run_case("cfg5", 26, 1ll << 23, 3540048, prop.multiProcessorCount);
  // one of the 8 shard pushes of the cfg4 key space on one GPU (bench --pattern exchange
  // --parts-per-gpu 8): 2^23 uniform records into a 2^28-element shard, U = 2^28 (1 - e^-(1/32))
  run_case("cfg4_mps8_shard", 28, 1ll << 23, 8259000, prop.multiProcessorCount);
  return 0;
}
