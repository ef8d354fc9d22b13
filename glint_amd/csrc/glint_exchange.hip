// glint_exchange.hip -- the exchange glue between the collective and the caller's tensors.
//
// AsyncBigVector.pull (src/main/scala/glint/models/client/async/AsyncBigVector.scala:61-79) sends one
// Pull message per partition and writes each partition's answer back to the positions its keys
// came from (`result(indices(i)) = response.values(i)`); AsyncBigMatrix.pull(rows)
// (AsyncBigMatrix.scala:53-86) does the same with whole rows. On the GPU the routed batch keeps the
// record indices (`order`, written by the route, glint_route.hip), and the answers come back grouped
// by partition:
//   scatter_rows   dst[order[i]] = src[i], rows of row_bytes (8 B elements, 4 KiB matrix rows ...);
//   copy_segments  a multi-range copy in one launch: a local partition's records that arrived from
//                  several source ranks gathered into one contiguous buffer (and the inverse, its
//                  answers put back into the response buffer's ranges);
//   send_matrix    the (rank, local partition) count matrix a rank sends in the split exchange, from
//                  the route's per-partition counts -- all zero when the batch had a bad key (the
//                  rank still joins the collectives, sending nothing).
// The copies are plain HBM streams: reads coalesced, writes coalesced per row (scatter_rows' element
// case writes one 8-B word per record at a random position -- the caller's order is arbitrary).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include "../../include/glint_gpu.h"

namespace {

typedef int64_t i64;
typedef unsigned int u32;
typedef __attribute__((ext_vector_type(4))) unsigned int U4;

constexpr int kXT = 256;

// one record per thread: 4- or 8-byte rows
template <typename W>
__global__ __launch_bounds__(kXT) void scatter_words(const W* __restrict__ src, const i64* __restrict__ order, i64 n,
                                                     W* __restrict__ dst) {
  const i64 stride = (i64)gridDim.x * kXT;
  for (i64 i = (i64)blockIdx.x * kXT + threadIdx.x; i < n; i += stride) {
    const i64 o = __builtin_nontemporal_load(order + i);
    dst[o] = __builtin_nontemporal_load(src + i);
  }
}

// one wave per record: wide rows (matrix row pulls), 16 B per lane when the rows allow it, else 4 B
template <bool VEC16>
__global__ __launch_bounds__(kXT) void scatter_wide(const char* __restrict__ src, const i64* __restrict__ order, i64 n,
                                                    i64 row_bytes, char* __restrict__ dst) {
  const int lane = threadIdx.x & 63;
  const i64 w0 = (i64)blockIdx.x * (kXT / 64) + (threadIdx.x >> 6);
  const i64 nw = (i64)gridDim.x * (kXT / 64);
  for (i64 i = w0; i < n; i += nw) {
    const i64 o = order[i];
    if (VEC16) {
      const U4* s = reinterpret_cast<const U4*>(src + i * row_bytes);
      U4* d = reinterpret_cast<U4*>(dst + o * row_bytes);
      const i64 m = row_bytes / 16;
#pragma unroll 4
      for (i64 c = lane; c < m; c += 64) d[c] = __builtin_nontemporal_load(s + c);
    } else {
      const u32* s = reinterpret_cast<const u32*>(src + i * row_bytes);
      u32* d = reinterpret_cast<u32*>(dst + o * row_bytes);
      const i64 m = row_bytes / 4;
      for (i64 c = lane; c < m; c += 64) d[c] = s[c];
    }
  }
}

// up to kMaxSeg (src offset, dst offset, bytes) segments per launch, by value
constexpr int kMaxSeg = 64;
struct Segs {
  i64 src[kMaxSeg], dst[kMaxSeg], end[kMaxSeg];  // end = inclusive prefix of the lengths, in units
  int n;
};

// grid-stride over the concatenated units; a unit finds its segment by a scan of the (few) prefixes
template <typename W>
__global__ __launch_bounds__(kXT) void copy_segs(const W* __restrict__ src, W* __restrict__ dst, Segs s) {
  const i64 total = s.end[s.n - 1];
  const i64 stride = (i64)gridDim.x * kXT;
  int k = 0;
  for (i64 u = (i64)blockIdx.x * kXT + threadIdx.x; u < total; u += stride) {
    while (s.end[k] <= u) ++k;  // u only grows: the cursor moves forward
    const i64 begin = k ? s.end[k - 1] : 0;
    dst[s.dst[k] + (u - begin)] = __builtin_nontemporal_load(src + s.src[k] + (u - begin));
  }
}

// send[cell[p]] = counts[p] (every other cell 0), or all zero when *bad != 0; one workgroup
__global__ __launch_bounds__(kXT) void send_matrix(const i64* __restrict__ counts, const i64* __restrict__ cell,
                                                   int nparts, int ncells, const unsigned long long* bad,
                                                   i64* __restrict__ send) {
  const bool ok = bad == nullptr || *bad == 0ull;
  for (int c = threadIdx.x; c < ncells; c += kXT) send[c] = 0;
  __syncthreads();
  if (ok)
    for (int p = threadIdx.x; p < nparts; p += kXT) send[cell[p]] = counts[p];
}

unsigned grid_of(i64 units, i64 per_block) {
  i64 g = (units + per_block - 1) / per_block;
  return (unsigned)std::max<i64>(1, std::min<i64>(g, 256 * 16));
}

}  // namespace

extern "C" int glint_scatter_rows_dev(const void* src, const int64_t* order, int64_t n, int64_t row_bytes, void* dst,
                                      void* stream) {
  if (n < 0 || row_bytes <= 0 || row_bytes % 4) return GLINT_EINVAL;
  if (n == 0) return GLINT_OK;
  if (!src || !order || !dst) return GLINT_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const uintptr_t al = (uintptr_t)src | (uintptr_t)dst;
  if (row_bytes == 8 && al % 8 == 0) {
    scatter_words<unsigned long long><<<grid_of(n, kXT), kXT, 0, st>>>((const unsigned long long*)src, order, n,
                                                                         (unsigned long long*)dst);
  } else if (row_bytes == 4) {
    scatter_words<u32><<<grid_of(n, kXT), kXT, 0, st>>>((const u32*)src, order, n, (u32*)dst);
  } else if (row_bytes % 16 == 0 && al % 16 == 0) {
    scatter_wide<true><<<grid_of(n, kXT / 64), kXT, 0, st>>>((const char*)src, order, n, row_bytes, (char*)dst);
  } else {
    scatter_wide<false><<<grid_of(n, kXT / 64), kXT, 0, st>>>((const char*)src, order, n, row_bytes, (char*)dst);
  }
  return hipGetLastError() == hipSuccess ? GLINT_OK : GLINT_EDEVICE;
}

extern "C" int glint_copy_segments_dev(const void* src, void* dst, const int64_t* segs, int nseg, void* stream) {
  if (nseg < 0 || (nseg > 0 && !segs)) return GLINT_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  // 16-B units when every offset and length allows it, else 4-B
  uintptr_t al = (uintptr_t)src | (uintptr_t)dst;
  for (int k = 0; k < nseg; ++k) {
    if (segs[3 * k] < 0 || segs[3 * k + 1] < 0 || segs[3 * k + 2] < 0) return GLINT_EINVAL;
    al |= (uintptr_t)(segs[3 * k] | segs[3 * k + 1] | segs[3 * k + 2]);
  }
  if (al % 4) return GLINT_EINVAL;
  const int ub = al % 16 == 0 ? 16 : 4;
  for (int k = 0; k < nseg;) {
    Segs s{};
    i64 tot = 0;
    for (; k < nseg && s.n < kMaxSeg; ++k) {  // up to kMaxSeg nonempty segments per launch
      if (segs[3 * k + 2] == 0) continue;
      s.src[s.n] = segs[3 * k] / ub;
      s.dst[s.n] = segs[3 * k + 1] / ub;
      tot += segs[3 * k + 2] / ub;
      s.end[s.n] = tot;
      ++s.n;
    }
    if (!s.n) continue;
    if (!src || !dst) return GLINT_EINVAL;
    if (ub == 16)
      copy_segs<U4><<<grid_of(tot, kXT), kXT, 0, st>>>((const U4*)src, (U4*)dst, s);
    else
      copy_segs<u32><<<grid_of(tot, kXT), kXT, 0, st>>>((const u32*)src, (u32*)dst, s);
    if (hipGetLastError() != hipSuccess) return GLINT_EDEVICE;
  }
  return GLINT_OK;
}

extern "C" int glint_send_matrix_dev(const int64_t* counts, const int64_t* cells, int32_t nparts, int32_t ncells,
                                     const uint64_t* bad_dev, int64_t* send, void* stream) {
  if (nparts < 0 || ncells <= 0 || !send || (nparts > 0 && (!counts || !cells))) return GLINT_EINVAL;
  send_matrix<<<1, kXT, 0, (hipStream_t)stream>>>(counts, cells, nparts, ncells,
                                                  (const unsigned long long*)bad_dev, send);
  return hipGetLastError() == hipSuccess ? GLINT_OK : GLINT_EDEVICE;
}
