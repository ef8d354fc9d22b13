// glint_kernels.h -- gfx950 kernels of the push/pull reduction plane.
//
// The shard is the HBM image of a Glint partial model's `data` array
// (src/main/scala/glint/models/server/PartialVector.scala:27, PartialMatrix.scala:28):
// vector shard = V[size], matrix shard = row-major V[size][pitch] (pitch = cols rounded up to
// 16 B so every row starts 16-B aligned; Array[Array[V]] has no cross-row layout to preserve).
//
// Record "address" = the element a record touches:
//   vector: (int)(key - start)                 RangePartition.globalToLocal (RangePartition.scala:33)
//           (int)((key - index) / P)           CyclicPartition.globalToLocal (CyclicPartition.scala:45-47)
//   matrix: globalToLocal(row) * pitch + col   PartialMatrix.update (PartialMatrix.scala:77-79)
// A record is rejected (GLINT_EOUTOFRANGE) exactly when the JVM would throw
// ArrayIndexOutOfBoundsException: local index outside [0, size) or col outside [0, cols).
//
// Push = two stream-ordered kernels:
//   push_seq      persistent, ticketed tiles; a decoupled look-back computes, per tile, whether
//                 every record address from the start of the call up to the end of the tile is
//                 strictly increasing. Such a prefix has unique addresses, so those tiles apply
//                 their records with PLAIN coalesced read-modify-write (16-B accesses when two
//                 consecutive records hit adjacent elements). The first tile whose prefix is not
//                 increasing records itself as the break point and is NOT applied; neither is any
//                 later tile.
//   push_scatter  applies records [break*TILE, n) -- nothing when the whole call was increasing --
//                 by LDS hash aggregation (duplicate addresses within a chunk are summed in LDS)
//                 followed by one device-scope atomic add per distinct address.
// The kernel boundary between the two orders every plain store before every atomic.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace glint {

typedef long long i64;
typedef unsigned long long u64;
typedef unsigned int u32;

constexpr int kTPB = 256;          // threads per block (4 waves)
constexpr int kSeqPPT = 8;         // record pairs per thread in push_seq
constexpr int kSeqTile = kTPB * kSeqPPT * 2;  // 4096 records per tile
constexpr int kHashSlots = 4096;   // LDS hash table slots in push_scatter (64 KiB for 8-B V)
constexpr int kScatterChunk = 2048;  // records per block iteration in push_scatter (load <= 0.5)
static_assert(kSeqTile % kScatterChunk == 0, "a scatter chunk must lie inside one push_seq tile");

// tile status words (published with agent-scope relaxed atomics; the word IS the payload)
constexpr u32 ST_EMPTY = 0, ST_A_OK = 1, ST_A_BAD = 2, ST_P_OK = 3, ST_P_BAD = 4;
constexpr u32 kLookbackSpinLimit = 1u << 22;

// per-launch control words, zeroed by one hipMemsetAsync together with the status array
struct LaunchCtl {
  u32 ticket;    // next tile ticket
  u32 brk_enc;   // max over prefix-bad tiles of (ntiles - t); 0 = whole call increasing
  u32 bad_enc;   // max over locally-bad tiles of (ntiles - t)
  u32 timeouts;  // look-back spins that hit the limit (treated as a break: conservative)
};

// persistent error state, cleared by glint_shard_sync / host-pointer calls
struct ErrState {
  u64 min_bad_enc;  // max of ~index over rejected records; 0 = none
  u64 count;        // number of rejected records
};

// Partition -> local index, for both partitioner kinds (kind is launch-uniform)
struct PartDesc {
  int32_t kind;   // 0 range, 1 cyclic
  int32_t size;   // Partition.size: vector elements or matrix rows
  int64_t start;  // RangePartition.start
  int32_t cidx;   // CyclicPartition.index
  int32_t cparts; // CyclicPartition.numberOfPartitions
  int32_t cols;   // 0 = vector
  int32_t pad_;
  int64_t pitch;  // elements per row (matrix)
};

__device__ __forceinline__ int32_t g2l(const PartDesc& p, i64 key) {
  return p.kind == 0 ? (int32_t)(key - p.start) : (int32_t)((key - (i64)p.cidx) / (i64)p.cparts);
}

template <typename V>
struct PushArgs {
  const i64* keys;      // keys (vector) or rows (matrix)
  const int32_t* cols;  // matrix only
  const V* vals;
  i64 n;
  V* data;
  PartDesc part;
  LaunchCtl* ctl;
  u32* status;
  u32 ntiles;
  ErrState* err;
};

}  // namespace glint
