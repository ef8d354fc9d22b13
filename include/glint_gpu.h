/*
 * glint_gpu.h -- C ABI of the MI355X push/pull reduction plane for Glint's parameter server.
 *
 * A "shard" is the device-resident replacement of one Glint partial model: the JVM array
 * `data` of PartialVector[V] (src/main/scala/glint/models/server/PartialVector.scala:27) or
 * PartialMatrix[V] (src/main/scala/glint/models/server/PartialMatrix.scala:28), now held in HBM
 * of one MI355X. The entry points below are exactly the methods of those classes that the
 * server actors call (PartialVectorDouble.scala:17-23, PartialMatrixDouble.scala:21-28), plus
 * shard lifetime, device-resident variants for stream-ordered callers, and a raw wire-format
 * ingest of the reference's RequestSerializer payloads.
 *
 * Plain C: pointers, sizes and status codes only. Thread-safety: calls on DIFFERENT shards may
 * run concurrently from any threads; calls on ONE shard are serialized internally (the Akka
 * actor already serializes them, PartialVector.scala:16-17). Every host-pointer call is
 * synchronous: when it returns, its effect is visible to the next call on the same shard.
 */
#ifndef GLINT_GPU_H
#define GLINT_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Value types of the typed partial models (PartialVector{Int,Long,Float,Double}.scala,
 * PartialMatrix{Int,Long,Float,Double}.scala). */
enum glint_dtype { GLINT_I32 = 0, GLINT_I64 = 1, GLINT_F32 = 2, GLINT_F64 = 3 };

/* Status codes. GLINT_EOUTOFRANGE is where the reference throws
 * ArrayIndexOutOfBoundsException inside update/get (a key whose local index falls outside the
 * partition array); the JNI shim raises that exception type so Akka supervision behaves as in
 * the reference (restart => the actor re-creates a zeroed shard). */
enum glint_status {
  GLINT_OK = 0,
  GLINT_EOUTOFRANGE = 1, /* a key/row/col outside the shard; see glint_shard_last_error */
  GLINT_EDEVICE = 2,     /* HIP runtime error */
  GLINT_EINVAL = 3,      /* bad argument (null handle, wrong dtype, malformed payload ...) */
  GLINT_ENOMEM = 4       /* device or pinned-host allocation failed */
};

/* Push flags. */
enum glint_push_flags {
  GLINT_PUSH_DEFAULT = 0,
  /* Bit-exact reproduction of the reference's strictly sequential `data(k) += v` order for
   * Float/Double even when keys repeat (PartialVector.scala:37-41). Without it, repeated keys in
   * a device-resident push are summed in arbitrary order (<= 1e-6 relative for Double; Int and
   * Long are exact either way). Unique-key pushes are bit-exact in both modes.
   * Host-pointer and wire pushes (glint_vec_push, glint_mat_push, glint_push_wire: what the actor's
   * update() calls) of up to 131 072 records -- above the 79 999-record frame cap, glint.conf:143 --
   * keep the message's order WITHOUT this flag too (one launch, glint_ordered.hip), unless
   * GLINT_PUSH_UNORDERED is given. */
  GLINT_PUSH_DETERMINISTIC = 1,
  /* Hint: the keys are in no particular order and the caller does not need the reference's
   * summation order. A large push skips the order check and sums the records per shard slab in
   * LDS (partition by slab + one read-modify-write per touched element pair) instead of per-record
   * device atomics; a host-pointer push takes the unordered LDS-hash scatter instead of the
   * order-preserving fold. Without the hint, a large push takes the binned path by itself when the
   * shard's previous push was unordered (environment GLINT_BINNED=0 disables that, =1 forces it
   * for pushes >= 2^20 records). The adaptive choices (binned or not, and the binned front end)
   * follow what earlier pushes measured on the device as of the shard's last sync point
   * (glint_shard_sync, or the end of a host-pointer call): a device-resident caller that never
   * syncs gets the no-history defaults. */
  GLINT_PUSH_UNORDERED = 2,
  /* glint_*_push_dev_gated only: the gate word is the push's OUTPUT. The push checks every record
   * itself before applying any (its order check reads all keys), writes 0 or ~(index of the first
   * out-of-range record) to *gate, and applies nothing when there is one -- the route's validation
   * pass in front of a one-partition push, folded into the push. */
  GLINT_PUSH_VALIDATE = 4
};

typedef struct glint_shard* glint_shard_t;

/* ---- lifetime ------------------------------------------------------------------------------ */

/* Range-partitioned shard = `new PartialVector*(RangePartition(index, start, end))`
 * (RangePartition.scala:8; PartialVectorDouble.scala:15 allocates Array[Double](size), zeroed).
 * cols == 0 creates a vector shard of size (int)(end - start) elements (RangePartition.scala:24);
 * cols > 0 creates a matrix shard of (int)(end - start) rows x cols (PartialMatrixDouble.scala:19).
 * Replaces `Props(classOf[PartialVectorDouble], partition)` (src/main/scala/glint/Client.scala:178)
 * and `Props(classOf[PartialMatrixDouble], partition, cols)` (Client.scala:130). */
int glint_shard_create(int device, int dtype, int64_t start, int64_t end, int32_t cols,
                       glint_shard_t* out);

/* Cyclic-partitioned shard (CyclicPartition(index, numberOfPartitions, numberOfKeys),
 * src/main/scala/glint/partitioning/cyclic/CyclicPartition.scala:12). */
int glint_shard_create_cyclic(int device, int dtype, int32_t index, int32_t num_partitions,
                              int64_t num_keys, int32_t cols, glint_shard_t* out);

/* One device-resident push into several range vector shards of one device and type at once (up to
 * 64, disjoint ranges, any order): each record goes to the shard whose range holds its key -- the
 * partitions one server hosts, applied by one launch sequence where the reference sends a message per
 * partition (AsyncBigVector.scala:96-98) and each partition's actor applies its own
 * (PartialVector.scala:35-43). The batch is checked first: a key in no shard's range applies NOTHING
 * (mapPartitions throws before sending, AsyncBigVector.scala:96-98) and *gate receives ~(first such
 * record), else 0 -- gate is a device word or a glint_host_alloc word the caller reads after waiting on
 * `stream`. Unordered sums (as GLINT_PUSH_UNORDERED; exact for Int/Long). Every shard's lock is held
 * for the call; each is ordered after its host-pointer work and marked for the next sync like any
 * device-resident call (glint_shards_sync / glint_shard_sync on `stream`). A slab with views is not
 * a member (GLINT_EINVAL): push to its views, or to the slab alone. */
int glint_vec_push_dev_shards(glint_shard_t* shards, int n_shards, const int64_t* keys, const void* vals,
                              int64_t n, uint64_t* gate, void* stream);

/* Slabs: the partitions one server hosts, kept in one allocation. A range shard (vector, or matrix
 * rows of the slab's width) over RangePartition(start, end) whose elements are the slab's rows
 * [offset, offset + end - start) -- a view: it reads and writes them as they are, and is a shard like
 * any other (its own partition, key check, stream, error state). The slab keeps its own partition, so
 * a batch whose records all fall in the views can be pushed or pulled as ONE device-resident call on
 * the slab when the views' partitions lie side by side in key order (the Client's partitions of one
 * rank at world size 1: DistributedClient's slab) -- one launch sequence for all of them, where the
 * reference sends one message per partition (AsyncBigVector.scala:96-98, one actor per partition,
 * Client.scala:71-85). The view's first element must be 256-byte aligned in the slab. While it has
 * views the slab takes device-resident calls only (its host-pointer calls, and glint_shard_zero,
 * return GLINT_EINVAL), each ordered after the views' host-pointer work and before their later
 * host-pointer calls; device-resident calls on the slab and its views are ordered by their streams,
 * as for any shard. A view is destroyed before its slab (GLINT_EINVAL until then). */
int glint_shard_create_in(glint_shard_t slab, int64_t offset, int64_t start, int64_t end,
                          glint_shard_t* out);

/* Frees the device memory (actor postStop / `destroy()`, AsyncBigVector.scala:135-140). */
int glint_shard_destroy(glint_shard_t shard);

/* Zeroes the shard: what an Akka restart of the partial-model actor produces. */
int glint_shard_zero(glint_shard_t shard);

/* Shape: size = Partition.size (elements for a vector, rows for a matrix), cols (0 = vector),
 * dtype, device. Any out-pointer may be NULL. */
int glint_shard_info(glint_shard_t shard, int32_t* size, int32_t* cols, int* dtype, int* device);

/* ---- host-pointer hot path (what the JNI shim calls) ---------------------------------------- */

/* PartialVector.update(keys, values) -- PartialVector.scala:35-43. vals: n elements of dtype. */
int glint_vec_push(glint_shard_t shard, const int64_t* keys, const void* vals, int64_t n, int flags);

/* PartialVector.get(keys) -- PartialVector.scala:51-60. out: n elements of dtype. */
int glint_vec_pull(glint_shard_t shard, const int64_t* keys, void* out, int64_t n);

/* PartialMatrix.update(rows, cols, values) -- PartialMatrix.scala:74-83. */
int glint_mat_push(glint_shard_t shard, const int64_t* rows, const int32_t* cols, const void* vals,
                   int64_t n, int flags);

/* PartialMatrix.get(rows, cols) -- PartialMatrix.scala:55-65. */
int glint_mat_pull(glint_shard_t shard, const int64_t* rows, const int32_t* cols, void* out, int64_t n);

/* PartialMatrix.getRows(rows) -- PartialMatrix.scala:37-46, written flattened row-major
 * (n x cols) the way ResponseSerializer sends ResponseRows* (ResponseSerializer.scala:52-61). */
int glint_mat_pull_rows(glint_shard_t shard, const int64_t* rows, void* out, int64_t n);

/* After GLINT_EOUTOFRANGE: index (within the failing call) of the first rejected record. */
int glint_shard_last_error(glint_shard_t shard, int64_t* first_bad_record);

/* ---- device-resident variants (stream-ordered, no host synchronisation) --------------------- *
 * All pointers are device pointers on the shard's device; `stream` is a hipStream_t used exactly
 * as given (NULL = the HIP null stream, as in the HIP API). All device-resident calls on one shard
 * must be ordered (one stream, or event-ordered streams), as the actor model orders its messages.
 * Errors are accumulated on the device and reported by glint_shard_sync. */
int glint_vec_push_dev(glint_shard_t shard, const int64_t* keys, const void* vals, int64_t n,
                       int flags, void* stream);
int glint_vec_pull_dev(glint_shard_t shard, const int64_t* keys, void* out, int64_t n, void* stream);
int glint_mat_push_dev(glint_shard_t shard, const int64_t* rows, const int32_t* cols,
                       const void* vals, int64_t n, int flags, void* stream);
int glint_mat_pull_dev(glint_shard_t shard, const int64_t* rows, const int32_t* cols, void* out,
                       int64_t n, void* stream);
int glint_mat_pull_rows_dev(glint_shard_t shard, const int64_t* rows, void* out, int64_t n,
                            void* stream);

/* glint_vec_push_dev / glint_mat_push_dev behind a device-side gate: the push is enqueued at once,
 * and when it runs it applies NOTHING if the 64-bit device word *gate is nonzero (a route status word,
 * glint_route_gather_dev's bad_dev: a batch with a key outside the partitioner is not applied, as
 * AsyncBigVector.mapPartitions throws before any message is sent, AsyncBigVector.scala:96-98). The
 * client reads the word after its one wait, so no host synchronisation separates the route from the
 * push. The push takes the check + apply path (GLINT_PUSH_UNORDERED is ignored); deterministic pushes
 * and unaligned arrays (keys not 16-B aligned, values not 2-element aligned) are GLINT_EINVAL. */
/* With GLINT_PUSH_VALIDATE the push writes *gate itself (see the flag): no route in front. The gate
 * word may be device memory or lie in a glint_host_alloc buffer (the caller then reads the verdict
 * from host memory after its wait, with no copy). */
int glint_vec_push_dev_gated(glint_shard_t shard, const int64_t* keys, const void* vals, int64_t n,
                             int flags, uint64_t* gate, void* stream);
int glint_mat_push_dev_gated(glint_shard_t shard, const int64_t* rows, const int32_t* cols,
                             const void* vals, int64_t n, int flags, uint64_t* gate, void* stream);

/* Waits for the shard's pending device work on `stream` and returns GLINT_EOUTOFRANGE if any
 * device-resident call since the last sync saw an out-of-range record (first_bad_record = its
 * index within the call that saw it, may be NULL). Clears the device error state. */
int glint_shard_sync(glint_shard_t shard, void* stream, int64_t* first_bad_record);
/* glint_shard_sync for n DISTINCT shards at once, shard i's calls on streams[i] (the local pushes of one
 * exchange step, each on a stream of its own): every error-state copy is enqueued before the first
 * wait, so the n waits overlap. rcs[i] / first_bad[i] (may be NULL): what glint_shard_sync(shards[i],
 * streams[i], ...) returns and reports. Returns GLINT_OK when every rcs[i] is, else the first other
 * code (GLINT_EINVAL for a NULL or repeated shard, before anything is waited for). */
int glint_shards_sync(glint_shard_t* shards, void** streams, int n, int* rcs, int64_t* first_bad);

/* Device pointer to the shard's data (row-major, row pitch from glint_shard_pitch) for
 * stream-ordered consumers (RCCL exchange buffers, checkpoint dumps, tests). */
int glint_shard_data(glint_shard_t shard, void** device_ptr);
int glint_shard_pitch(glint_shard_t shard, int64_t* elements_per_row);

/* ---- wire ingest (RequestSerializer / ResponseSerializer byte images) ----------------------- *
 * payload is the exact byte image RequestSerializer.toBinary produces
 * (src/main/scala/glint/serialization/RequestSerializer.scala:92-205): native-endian
 * [u8 type][i32 n]([i32 id])[i64 keys x n]([i32 cols x n])([V values x n]); keys start at the
 * unaligned offset 5 or 9. */

/* Applies a Push{Vector,Matrix}{Int,Long,Float,Double} message; *id receives its id. */
int glint_push_wire(glint_shard_t shard, const uint8_t* payload, size_t len, int32_t* id, int flags);

/* Answers a PullVector / PullMatrix / PullMatrixRows message with the ResponseSerializer image
 * [u8 type][i32 n][V x n] (ResponseSerializer.scala:43-117). *out_len receives the image size;
 * if cap is too small nothing is written, *out_len is set and GLINT_EINVAL returned. */
int glint_pull_wire(glint_shard_t shard, const uint8_t* payload, size_t len, uint8_t* response,
                    size_t cap, size_t* out_len);

/* ---- pipelined host ingest ----------------------------------------------------------------------- *
 * For servers whose messages arrive faster than one at a time (GranularBigVector/AsyncBigVector send
 * a batch's messages without waiting for one another, GranularBigVector.scala:39-50): a push is put
 * in one of the shard's GLINT_RING_SLOTS pinned host slots and enqueued on the shard's stream without
 * waiting. Pushes of up to GLINT_ZERO_COPY_MAX records are read by the kernel straight from the
 * pinned slot (no copy command); larger ones cross PCIe in one DMA. Tickets number the enqueued
 * pushes of a shard; glint_shard_wait(ticket) returns once that push and every push enqueued before
 * it are applied -- what the actor needs before it answers AcknowledgeReceipt
 * (PushLogic.scala:40-66). Every other call on the shard is ordered after the enqueued pushes.
 * Errors belong to the call that enqueues a message, as the reference's update/get throw while the
 * actor handles the Push/Pull message itself (PartialVectorDouble.scala:17-23): the enqueueing call
 * checks every record first and returns GLINT_EOUTOFRANGE (first bad record via
 * glint_shard_last_error) with nothing of that message enqueued; a wait reports only a launch that
 * failed on the device (GLINT_EDEVICE, once, to the first wait covering it).
 * Flags as for glint_vec_push (message order kept for Float/Double unless GLINT_PUSH_UNORDERED).
 * An entry of up to GLINT_ZERO_COPY_MAX records is ONE single-workgroup kernel that signals its own
 * completion through a host-mapped word (no event, no copy command): a few microseconds of stream
 * time per message. Pulls can be enqueued the same way (glint_pull_async), so a server answering a
 * burst of Pull messages waits once for all of them. Consecutive message-sized pushes with the same
 * flags, and consecutive message-sized element pulls, are coalesced into one launch per batch (the
 * batch goes to the GPU when it is full or anything else needs the stream); every message keeps its
 * own ticket and its own errors. Tickets number pushes and pulls together. */
#ifndef GLINT_RING_SLOTS
#define GLINT_RING_SLOTS 16
#endif
#define GLINT_ZERO_COPY_MAX 4096

/* A free slot for a push of n records, with the section pointers the caller fills: keys (i64 x n),
 * cols (i32 x n, matrix shards only, else NULL) and vals (n values of the shard's type). Waits for
 * the slot's previous push if it is still in flight. The JNI shim copies the JVM arrays straight in
 * (Get<T>ArrayRegion): no critical region, no second copy. n <= 2^20. */
int glint_stage_acquire(glint_shard_t shard, int64_t n, void** keys, void** cols, void** vals, int* slot);
/* Enqueues the push of the n records staged in `slot`; *ticket receives its ticket. */
int glint_push_staged(glint_shard_t shard, int slot, int64_t n, int flags, uint64_t* ticket);
/* glint_push_wire, enqueued: the payload is copied into a slot before the call returns. A push of more
 * than 4 MiB of records (far above the 79 999-record frame cap) is applied before the call returns
 * instead, through the staged copies, so the ring's pinned memory stays bounded. */
int glint_push_wire_async(glint_shard_t shard, const uint8_t* payload, size_t len, int32_t* id, int flags,
                          uint64_t* ticket);
/* Waits for the entry with this ticket and every earlier one and completes their pulls' answers;
 * GLINT_EDEVICE if one of them failed to launch. */
int glint_shard_wait(glint_shard_t shard, uint64_t ticket, int64_t* first_bad);
/* glint_vec_pull (kind 0), glint_mat_pull (1) or glint_mat_pull_rows (2), enqueued: the keys (and
 * cols) are checked and copied before the call returns; `out` receives the answer by the time
 * glint_shard_wait(*ticket) returns and must stay valid until then. n <= 2^20. An answer of more than
 * 16 MiB (row pulls of wide matrices) is produced before the call returns instead, so the ring's pinned
 * memory stays bounded. */
int glint_pull_async(glint_shard_t shard, int kind, const int64_t* keys, const int32_t* cols, void* out,
                     int64_t n, uint64_t* ticket);
/* glint_pull_wire, enqueued: the response header is written at once, its values by the time
 * glint_shard_wait(*ticket) returns (the response buffer must stay valid until then). */
int glint_pull_wire_async(glint_shard_t shard, const uint8_t* payload, size_t len, uint8_t* response,
                          size_t cap, size_t* out_len, uint64_t* ticket);

/* ---- client routing (device) -------------------------------------------------------------- *
 * Replaces the client-side grouping in AsyncBigVector/AsyncBigMatrix.mapPartitions
 * (src/main/scala/glint/models/client/async/AsyncBigVector.scala:96-98, AsyncBigMatrix.scala:
 * 150-152): a stable counting sort of the n device-resident keys by owning partition under
 * RangePartitioner.apply(nparts, nkeys) (RangePartitioner.scala:27-84) or
 * CyclicPartitioner.apply(nparts, nkeys) (CyclicPartitioner.scala:19-22, 41-50). On return (the
 * call synchronises `stream`): order[0..n) holds the record indices grouped by partition, each
 * group in the caller's order; counts[0..nparts) (device) the group sizes. Out-of-range keys
 * (IndexOutOfBoundsException in partition()) -> GLINT_EOUTOFRANGE with the first bad record index
 * in *first_bad (host), else *first_bad = -1. nparts <= 8192, n < 2^32. */
enum glint_route_kind { GLINT_ROUTE_RANGE = 0, GLINT_ROUTE_CYCLIC = 1 };
int glint_route_dev(const int64_t* keys, int64_t n, int kind, int32_t nparts, int64_t nkeys,
                    int64_t* counts, int64_t* order, int64_t* first_bad, void* stream);

/* The exchange's send buffers in one pass, with no host synchronisation (AsyncBigVector.scala:96-116,
 * AsyncBigMatrix.scala:141-156): records grouped as glint_route_dev groups them -- by partition, or
 * by slot_of[partition] (device array of nparts group indices, e.g. partitions ordered by hosting
 * rank; NULL = identity) -- each group in the caller's order, and written in that order into every
 * non-NULL output: order (record indices), out_keys, out_cols (from cols), out_vals (vsize = 4 or 8
 * bytes per value, from vals). counts[0..nparts) (device) receives the group sizes. The first bad
 * record is left in the device word *bad_dev as ~index (0 = none); bad records are in no group.
 * With every output NULL only counts and *bad_dev are produced (a one-partition batch is its own
 * send buffer). Stream-ordered on `stream`; the caller reads counts and *bad_dev when it needs them. */
int glint_route_gather_dev(const int64_t* keys, const int32_t* cols, const void* vals, int vsize, int64_t n,
                           int kind, int32_t nparts, int64_t nkeys, const int32_t* slot_of, int64_t* counts,
                           int64_t* order, int64_t* out_keys, int32_t* out_cols, void* out_vals,
                           uint64_t* bad_dev, void* stream);

/* glint_route_gather_dev with every key written to out_keys as key + key_delta[group] (device array
 * of nparts int64, indexed like the groups): a partition's keys rebased to their rows in the slab of
 * the rank that hosts it (glint_shard_create_in), so the receiving rank pushes everything it receives
 * as ONE call on its slab instead of one per partition (the reference's one message per partition,
 * AsyncBigVector.scala:96-116). out_keys and key_delta non-NULL, nparts >= 2. */
int glint_route_gather_rebased_dev(const int64_t* keys, const int32_t* cols, const void* vals, int vsize,
                                   int64_t n, int kind, int32_t nparts, int64_t nkeys, const int32_t* slot_of,
                                   const int64_t* key_delta, int64_t* counts, int64_t* order,
                                   int64_t* out_keys, int32_t* out_cols, void* out_vals, uint64_t* bad_dev,
                                   void* stream);

/* ---- exchange glue (device) ----------------------------------------------------------------- *
 * The client side of a routed pull: AsyncBigVector.pull writes each partition's answer back to the
 * positions its keys came from (`result(indices(i)) = values(i)`, AsyncBigVector.scala:61-79;
 * whole rows in AsyncBigMatrix.pull(rows), AsyncBigMatrix.scala:53-86). Stream-ordered on `stream`,
 * no host synchronisation; device pointers.
 * dst[order[i]] = src[i] for i < n, rows of row_bytes bytes (a multiple of 4); order is the record
 * index array glint_route_gather_dev wrote (or a sub-range of it). */
int glint_scatter_rows_dev(const void* src, const int64_t* order, int64_t n, int64_t row_bytes, void* dst,
                           void* stream);
/* A multi-range copy in one launch: segs is a HOST array of nseg (src_offset, dst_offset, bytes)
 * triples (byte offsets, multiples of 4); segment k copies src + src_offset to dst + dst_offset. Used to
 * gather a local partition's records that arrived from several source ranks into one buffer, and to
 * put its answers back into the response buffer's ranges. */
int glint_copy_segments_dev(const void* src, void* dst, const int64_t* segs, int nseg, void* stream);
/* The (rank, local partition) count matrix of a split exchange, from the route's per-partition counts:
 * send[cells[p]] = counts[p] for p < nparts and every other of the ncells entries 0; all ncells
 * entries 0 when the route's status word *bad_dev is nonzero (NULL: no status word) -- a rank with an
 * out-of-range key sends nothing but still joins the collectives. Device arrays, one launch. */
int glint_send_matrix_dev(const int64_t* counts, const int64_t* cells, int32_t nparts, int32_t ncells,
                          const uint64_t* bad_dev, int64_t* send, void* stream);

/* ---- kernel timing ------------------------------------------------------------------------- *
 * With profiling on, every kernel launch of the shard is bracketed by HIP events recorded on the
 * stream it is launched on; glint_prof_read waits for them and returns the summed device time and
 * launch count of one kernel kind since the last reset. Used by bench.py for the roofline figure. */
enum glint_kernel_id {
  GLINT_K_PUSH_APPLY = 0,   /* plain-RMW push of the increasing prefix (the dense hot path) */
  GLINT_K_PUSH_SCATTER = 1, /* LDS-aggregated atomic push of the unordered tail */
  GLINT_K_VEC_PULL = 2,
  GLINT_K_MAT_PULL = 3,
  GLINT_K_MAT_PULL_ROWS = 4,
  GLINT_K_PUSH_CHECK = 5,   /* order / affinity check over the keys in front of push_apply */
  GLINT_K_PUSH_BINNED = 6,  /* the binned unordered-push pipeline (count, partition, apply) */
  GLINT_K_PUSH_ORDERED = 7, /* the order-preserving push of message-sized pushes (one launch) */
  GLINT_K_COUNT = 8
};
int glint_prof_enable(glint_shard_t shard, int on);
int glint_prof_read(glint_shard_t shard, int kernel_id, double* total_ms, int64_t* launches);
int glint_prof_reset(glint_shard_t shard);

/* ---- misc ---------------------------------------------------------------------------------- */
const char* glint_strerror(int status);
/* Number of visible devices (0 without a GPU; never fails). */
int glint_device_count(void);
/* Library version (major*10000 + minor*100 + patch). */
int glint_version(void);
/* The library reads its GLINT_* environment overrides (tuning and test knobs) once and caches them;
 * this makes the next call re-read them (tests that change the environment between calls). */
int glint_reload_env(void);

/* Pinned, device-mapped host memory for the buffers a server answers from (the response images it
 * sends). A message-sized pull (glint_pull_async, glint_pull_wire_async) whose answer destination
 * lies in such a buffer, is aligned to the value size and is at least a page (GLINT_DIRECT_MIN_BYTES,
 * default 4096) is answered by the kernel straight into it: no copy out of the ring slot when the
 * entry retires. Free with glint_host_free: it returns GLINT_EINVAL (and frees nothing) while a pull
 * enqueued to answer into the buffer has not retired (glint_shard_wait for its ticket first). */
int glint_host_alloc(size_t bytes, void** host_ptr);
int glint_host_free(void* host_ptr);

/* The glint_push_flags this library implements (a client built against a newer header checks
 * before relying on a flag an older library would ignore, e.g. GLINT_PUSH_VALIDATE). */
int glint_push_flags_supported(void);

#ifdef __cplusplus
}
#endif
#endif /* GLINT_GPU_H */
