// launch_latency.hip -- the floor under a message-sized host push/pull on this box: one kernel
// launch and its completion, measured several ways (stream sync, event sync, a host-mapped word
// the kernel writes, pipelined launches, a 16-B D2H copy). Prints one JSON line per variant.
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/build/launch_latency tools/launch_latency.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

typedef unsigned long long u64;

__global__ void k_empty() {}

__global__ void k_flag(u64* f, u64 t) {
  if (threadIdx.x == 0) __hip_atomic_store(f, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// a message-sized gather from mapped host memory into mapped host memory, then the flag
__global__ void k_gather(const long long* keys, const double* data, double* out, int n, u64* f, u64 t) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) out[i] = data[keys[i]];
  __syncthreads();
  if (threadIdx.x == 0) {
    __atomic_thread_fence(__ATOMIC_RELEASE);
    __hip_atomic_store(f, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void spin(volatile u64* f, u64 t) {
  while (__atomic_load_n(f, __ATOMIC_ACQUIRE) < t) {
  }
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 2000;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  u64* h = nullptr;
  u64* hd = nullptr;
  CK(hipHostMalloc((void**)&h, 4096, hipHostMallocMapped));
  CK(hipHostGetDevicePointer((void**)&hd, h, 0));
  *h = 0;
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const int n = 1000;
  long long* hk = nullptr;
  double* ho = nullptr;
  CK(hipHostMalloc((void**)&hk, n * 8, hipHostMallocMapped));
  CK(hipHostMalloc((void**)&ho, n * 8, hipHostMallocMapped));
  long long *dk, *dko;
  double* dout;
  CK(hipHostGetDevicePointer((void**)&dk, hk, 0));
  CK(hipHostGetDevicePointer((void**)&dout, ho, 0));
  (void)dko;
  double* data = nullptr;
  CK(hipMalloc((void**)&data, (size_t)1 << 23));
  CK(hipMemset(data, 0, (size_t)1 << 23));
  for (int i = 0; i < n; ++i) hk[i] = (i * 7919) % (1 << 20);
  u64* dh16 = nullptr;
  CK(hipMalloc((void**)&dh16, 64));
  for (int i = 0; i < 200; ++i) k_empty<<<1, 64, 0, s>>>();
  CK(hipStreamSynchronize(s));

  u64 t = 0;
  auto report = [&](const char* what, double us) { std::printf("{\"variant\": \"%s\", \"us\": %.2f, \"reps\": %d}\n", what, us, reps); };
  double t0 = now_us();
  for (int i = 0; i < reps; ++i) {
    k_empty<<<1, 64, 0, s>>>();
    CK(hipStreamSynchronize(s));
  }
  report("launch+stream_sync", (now_us() - t0) / reps);
  t0 = now_us();
  for (int i = 0; i < reps; ++i) {
    k_empty<<<1, 64, 0, s>>>();
    CK(hipEventRecord(ev, s));
    CK(hipEventSynchronize(ev));
  }
  report("launch+event_sync", (now_us() - t0) / reps);
  t0 = now_us();
  for (int i = 0; i < reps; ++i) {
    k_flag<<<1, 64, 0, s>>>(hd, ++t);
    spin(h, t);
  }
  report("launch+mapped_flag_spin", (now_us() - t0) / reps);
  t0 = now_us();
  for (int i = 0; i < reps; ++i) {
    k_gather<<<1, 1024, 0, s>>>(dk, data, dout, n, hd, ++t);
    spin(h, t);
  }
  report("gather1000_zero_copy+flag_spin", (now_us() - t0) / reps);
  t0 = now_us();
  for (int i = 0; i < reps; ++i) {
    k_empty<<<1, 64, 0, s>>>();
    CK(hipMemcpyAsync(h + 8, dh16, 16, hipMemcpyDeviceToHost, s));
    CK(hipEventRecord(ev, s));
    CK(hipEventSynchronize(ev));
  }
  report("launch+d2h16+event_sync", (now_us() - t0) / reps);
  t0 = now_us();
  for (int i = 0; i < reps; ++i) k_empty<<<1, 64, 0, s>>>();
  CK(hipStreamSynchronize(s));
  report("pipelined_launch", (now_us() - t0) / reps);
  t0 = now_us();
  for (int i = 0; i < reps; ++i) {
    k_empty<<<1, 64, 0, s>>>();
    CK(hipEventRecord(ev, s));
  }
  CK(hipStreamSynchronize(s));
  report("pipelined_launch+event_record", (now_us() - t0) / reps);
  t0 = now_us();
  for (int i = 0; i < reps; ++i) {
    k_empty<<<1, 64, 0, s>>>();
    CK(hipMemcpyAsync(h + 8, dh16, 16, hipMemcpyDeviceToHost, s));
    CK(hipEventRecord(ev, s));
  }
  CK(hipStreamSynchronize(s));
  report("pipelined_launch+d2h16+event_record", (now_us() - t0) / reps);
  t0 = now_us();
  for (int i = 0; i < reps; ++i) k_flag<<<1, 64, 0, s>>>(hd, ++t);
  spin(h, t);
  report("pipelined_flag_launch", (now_us() - t0) / reps);
  CK(hipStreamSynchronize(s));
  return 0;
}
