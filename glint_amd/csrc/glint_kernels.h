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
// Push = up to three stream-ordered kernels:
//   push_check    reads the keys once; finds the first 1024-record wave tile whose record addresses
//                 stop being strictly increasing (within the tile or across its left edge), and
//                 marks AFFINE tiles (record r hits element base + r), whose addresses push_apply
//                 then knows without reading the keys again.
//   push_apply    every tile before that break: the prefix's addresses are strictly increasing,
//                 hence unique, so records are applied with PLAIN coalesced read-modify-write
//                 (16-B accesses when two consecutive records hit adjacent elements) -- bit-exact
//                 with the reference's sequential loop.
//   push_scatter  records [break*TILE, n) -- nothing when the whole call was increasing -- by LDS
//                 hash aggregation (duplicate addresses within a chunk summed in LDS) followed by one
//                 device-scope atomic add per distinct address; or, in deterministic mode, a stable
//                 sort by address and an in-order fold per address.
// Kernel boundaries order check -> apply -> scatter: every plain store precedes every atomic.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace glint {

typedef long long i64;
typedef unsigned long long u64;
typedef unsigned int u32;

constexpr int kTPB = 256;          // threads per block (4 waves)
constexpr int kPPT = 8;            // record pairs per lane per wave tile (push_check / push_apply)
constexpr int kTile = 64 * kPPT * 2;  // 1024 records per wave tile
constexpr i64 kNotAffine = (i64)0x8000000000000000ll;  // tile descriptor: addresses not base + r
constexpr int kHashSlots = 4096;   // LDS hash table slots in push_scatter (64 KiB for 8-B V)
constexpr int kScatterChunk = 2048;  // records per block iteration in push_scatter (load <= 0.5)
// pushes of up to this many records can take the one-launch order-preserving fold (glint_ordered.hip):
// above the reference's frame cap of 79 999 Double records per message (glint.conf:143)
constexpr i64 kOrderedMax = (i64)1 << 17;
// internal push flag (not in the ABI): the call comes from a host-pointer / wire entry point, i.e.
// from the actor's update(), and keeps the message's summation order unless GLINT_PUSH_UNORDERED
constexpr int kPushHostSequential = 1 << 16;

// per-launch control words, zeroed by one hipMemsetAsync before push_check
struct LaunchCtl {
  u32 brk_enc;    // max over tiles that break the increasing order of (ntiles - t); 0 = none
  u32 nonaffine;  // some tile is not affine or does not continue its predecessor's affine run
  u32 cancel;     // a gated push whose gate word was set: it applies nothing (push_gate_kernel)
  u32 pad_;
  u64 bad;        // a validating gated push: max of ~index over its out-of-range records (push_check)
};

// persistent error state, cleared by glint_shard_sync / host-pointer calls
struct ErrState {
  u64 min_bad_enc;  // max of ~index over rejected records; 0 = none
  u64 count;        // number of rejected records
};

// Completion of a single-workgroup launch on the pinned-ring path (message-sized host calls): the
// kernel itself writes the shard's error state and then its ticket to host-mapped words, so the
// host waits on memory -- no event marker and no error copy in the stream (glint_gpu.hip, ring_*).
struct MsgSig {
  u64* done;       // host-mapped ticket word; nullptr = an ordinary launch
  u64 ticket;
  ErrState* herr;  // host-mapped: the error state after this launch
};

// A coalesced ring pull's answer destinations, one per message (the table sits in the slot, after
// the answer section): records [off, off + n) of the batch are written to dst -- a glint_host_alloc
// buffer the caller answers from, or the slot's own answer section.
struct PullDst {
  unsigned int off, n;
  unsigned long long dst;  // device address
};
constexpr int kPullDirectMax = 256;  // messages per batch with a destination table, at most

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

// KIND: 0 range, 1 cyclic (a kernel specialised per layout keeps the cyclic 64-bit division out of
// the range hot path), -1 = read p.kind at run time
template <int KIND = -1>
__device__ __forceinline__ int32_t g2l(const PartDesc& p, i64 key) {
  if (KIND == 0 || (KIND < 0 && p.kind == 0)) return (int32_t)(key - p.start);
  return (int32_t)((key - (i64)p.cidx) / (i64)p.cparts);
}

template <typename V>
struct PushArgs {
  const i64* keys;      // keys (vector) or rows (matrix)
  const int32_t* cols;  // matrix only
  const V* vals;
  i64 n;
  V* data;
  i64 elems;  // elements allocated in the shard
  PartDesc part;
  LaunchCtl* ctl;
  u32 ntiles;
  ErrState* err;
  u32 sweep_blocks;  // blocks of push_apply that take part in the affine sweep (<= grid)
  u64* hint;  // host-mapped word: the unordered-tail size push_apply saw (binned-path heuristic)
  MsgSig sig;  // ring launches only (one workgroup)
};

}  // namespace glint
