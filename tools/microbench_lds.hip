// LDS atomic-add throughput on gfx950 by address pattern and type: what the binned tail's dedup and
// slab-apply kernels pay per record. Not part of the product. Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/microbench_lds tools/microbench_lds.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int kSlots = 4096;
constexpr int kIters = 4096;

__device__ __forceinline__ unsigned hash(unsigned x) { x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; return x ^ (x >> 16); }

// PAT 0: lane-distinct, consecutive slots (no conflict); 1: random slots in the table;
// 2: 8 lanes per address (Zipf-like hot key); 3: all lanes one address.
// OP 0: atomic add (ds_add_*); 1: plain read + write (non-atomic RMW, wrong under conflicts: timing only)
template <typename V, int PAT, int OP>
__global__ __launch_bounds__(256) void k_lds(V* out, unsigned seed) {
  __shared__ V t[kSlots];
  for (int i = threadIdx.x; i < kSlots; i += 256) t[i] = V(0);
  __syncthreads();
  const unsigned lane = threadIdx.x & 63, tid = threadIdx.x;
  unsigned h = hash(seed ^ (blockIdx.x * 256 + tid));
  for (int it = 0; it < kIters; ++it) {
    unsigned a;
    if (PAT == 0) a = (tid + it * 256) & (kSlots - 1);
    else if (PAT == 1) { h = hash(h + it); a = h & (kSlots - 1); }
    else if (PAT == 2) a = ((lane >> 3) * 97 + it * 13 + (threadIdx.x >> 6) * 7) & (kSlots - 1);
    else a = (it * 5) & (kSlots - 1);
    if (OP == 0) atomicAdd(&t[a], V(1));
    else t[a] = t[a] + V(1);
  }
  __syncthreads();
  V s = V(0);
  for (int i = threadIdx.x; i < kSlots; i += 256) s += t[i];
  if (s == V(-1)) out[0] = s;
}

template <class F>
float timeit(F fn, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  std::vector<float> v;
  fn();
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a)); fn(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); v.push_back(ms);
  }
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  double* out;
  CK(hipMalloc(&out, 64));
  const int bpc = 3;
  const double ops = (double)cus * bpc * 256 * kIters;
#define RUN(V, PAT, OP, NAME)                                                                        \
  {                                                                                                  \
    const float ms = timeit([&] { k_lds<V, PAT, OP><<<cus * bpc, 256>>>((V*)out, 7); }, 5);          \
    printf("%-8s pat %d op %d: %8.3f ms  %7.1f G lane-ops/s  %5.2f cyc/lane/CU\n", NAME, PAT, OP, ms,     \
           ops / ms / 1e6, (ms * 1e-3 * 2.1e9) / (ops / cus));                                         \
  }
  RUN(double, 0, 0, "f64") RUN(double, 1, 0, "f64") RUN(double, 2, 0, "f64") RUN(double, 3, 0, "f64")
  RUN(double, 0, 1, "f64") RUN(double, 1, 1, "f64")
  RUN(float, 0, 0, "f32") RUN(float, 1, 0, "f32") RUN(float, 2, 0, "f32")
  RUN(unsigned, 0, 0, "u32") RUN(unsigned, 1, 0, "u32") RUN(unsigned, 2, 0, "u32")
  RUN(unsigned long long, 0, 0, "u64") RUN(unsigned long long, 1, 0, "u64")
  printf("done\n");
  return 0;
}
