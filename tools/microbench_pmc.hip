// PMC calibration: kernels with KNOWN HBM byte counts, one per access shape the push kernels use,
// so that FETCH_SIZE / WRITE_SIZE can be converted to bytes per shape (MI355X_MICROARCH.md §HBM: the
// gfx950 factor of 2 on FETCH_SIZE is calibrated only for 16-B-per-lane streaming reads; "other access
// widths are uncalibrated"). Every buffer is 2 GiB, far past the 256 MiB Infinity Cache, and every
// shape covers every line of its buffer exactly once, so the true bytes are the buffer size.
// Not part of the product. Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/build/microbench_pmc tools/microbench_pmc.hip
// Run under separate passes:  rocprofv3 --pmc FETCH_SIZE -- tools/build/microbench_pmc
//                             rocprofv3 --pmc WRITE_SIZE -- tools/build/microbench_pmc
// It prints one JSON line per kernel: {"kernel", "read_bytes", "write_bytes"} (the known counts);
// tools/pmc_calibrate.py joins them with the counter CSVs.
//
// Shapes (as in the push kernels):
//   ld16      16 B per lane, coalesced (push_check keys, push_apply sweep)        -- the guide's case
//   ld8       8 B per lane, coalesced (binned record values, route keys)
//   ld4       4 B per lane, coalesced (binned u32 addresses)
//   ld4s8     4 B per lane at a stride of 8 B: the low words of i64 keys (bin_count, bin_part)
//   st16/st8/st4   coalesced stores of those widths
//   rmw16     16-B pairs read and written back (bin_apply's dense item write-back, the sweep)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

typedef long long i64;
typedef unsigned int u32;
typedef __attribute__((ext_vector_type(4))) unsigned int U4;
typedef __attribute__((ext_vector_type(2))) unsigned int U2;

constexpr int TPB = 256;

template <typename T>
__device__ __forceinline__ u32 fold(T v) {
  if constexpr (sizeof(T) == 16) return v.x ^ v.y ^ v.z ^ v.w;
  else if constexpr (sizeof(T) == 8) return v.x ^ v.y;
  else return v;
}

// grid-stride coalesced loads of n elements of T (STRIDE elements apart: 2 = every other word)
template <typename T, int STRIDE>
__device__ __forceinline__ void k_load(const T* __restrict__ p, i64 n, u32* __restrict__ sink) {
  u32 acc = 0;
  const i64 stride = (i64)gridDim.x * TPB;
  for (i64 i = (i64)blockIdx.x * TPB + threadIdx.x; i < n; i += stride)
    acc ^= fold(__builtin_nontemporal_load(p + i * STRIDE));
  if (acc == 0x12345679u) sink[0] = acc;  // keeps the loads; never true for the fill below
}

template <typename T>
__device__ __forceinline__ void k_store(T* __restrict__ p, i64 n, u32 v) {
  const i64 stride = (i64)gridDim.x * TPB;
  for (i64 i = (i64)blockIdx.x * TPB + threadIdx.x; i < n; i += stride) {
    T x;
    if constexpr (sizeof(T) == 16) x = U4{v, v, v, (u32)i};
    else if constexpr (sizeof(T) == 8) x = U2{v, (u32)i};
    else x = v ^ (u32)i;
    __builtin_nontemporal_store(x, p + i);
  }
}

__global__ __launch_bounds__(TPB) void rmw16(U4* __restrict__ p, i64 n) {
  const i64 stride = (i64)gridDim.x * TPB;
  for (i64 i = (i64)blockIdx.x * TPB + threadIdx.x; i < n; i += stride) {
    U4 x = p[i];
    x.x += 1u;
    p[i] = x;
  }
}

// plain kernel names: the counter CSVs are joined by name
__global__ __launch_bounds__(TPB) void ld16(const U4* p, i64 n, u32* s) { k_load<U4, 1>(p, n, s); }
__global__ __launch_bounds__(TPB) void ld8(const U2* p, i64 n, u32* s) { k_load<U2, 1>(p, n, s); }
__global__ __launch_bounds__(TPB) void ld4(const u32* p, i64 n, u32* s) { k_load<u32, 1>(p, n, s); }
__global__ __launch_bounds__(TPB) void ld4s8(const u32* p, i64 n, u32* s) { k_load<u32, 2>(p, n, s); }
__global__ __launch_bounds__(TPB) void st16(U4* p, i64 n, u32 v) { k_store<U4>(p, n, v); }
__global__ __launch_bounds__(TPB) void st8(U2* p, i64 n, u32 v) { k_store<U2>(p, n, v); }
__global__ __launch_bounds__(TPB) void st4(u32* p, i64 n, u32 v) { k_store<u32>(p, n, v); }

int main(int argc, char** argv) {
  const i64 bytes = (i64)(argc > 1 ? atoll(argv[1]) : 2) << 30;  // GiB
  int cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) == hipSuccess) cus = prop.multiProcessorCount;
  const unsigned grid = (unsigned)cus * 8;
  char* buf;
  u32* sink;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(buf, 0x5A, bytes));
  CK(hipDeviceSynchronize());
  auto report = [&](const char* name, i64 rd, i64 wr) {
    CK(hipDeviceSynchronize());
    printf("{\"kernel\": \"%s\", \"read_bytes\": %lld, \"write_bytes\": %lld}\n", name, rd, wr);
    fflush(stdout);
  };
  for (int rep = 0; rep < 2; ++rep) {  // two dispatches of each: the calibration averages them
    ld16<<<grid, TPB>>>((const U4*)buf, bytes / 16, sink);
    report("ld16", bytes, 0);
    ld8<<<grid, TPB>>>((const U2*)buf, bytes / 8, sink);
    report("ld8", bytes, 0);
    ld4<<<grid, TPB>>>((const u32*)buf, bytes / 4, sink);
    report("ld4", bytes, 0);
    ld4s8<<<grid, TPB>>>((const u32*)buf, bytes / 8, sink);  // every line, half its bytes used
    report("ld4s8", bytes, 0);
    st16<<<grid, TPB>>>((U4*)buf, bytes / 16, 7u);
    report("st16", 0, bytes);
    st8<<<grid, TPB>>>((U2*)buf, bytes / 8, 7u);
    report("st8", 0, bytes);
    st4<<<grid, TPB>>>((u32*)buf, bytes / 4, 7u);
    report("st4", 0, bytes);
    rmw16<<<grid, TPB>>>((U4*)buf, bytes / 16);
    report("rmw16", bytes, bytes);
  }
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
