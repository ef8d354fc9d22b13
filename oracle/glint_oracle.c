/*
 * glint_oracle.c -- CPU restatement of rjagerman/glint's push/pull hot path.
 *
 * TEST INFRASTRUCTURE ONLY. This file is the parity checker for the HIP path in glint_amd/csrc.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The product
 * (libglint_gpu.so) never links it and has no CPU fallback.
 *
 * Parity pinning: the reference is Scala/Akka and cannot be built or run in this image (no JVM;
 * SURVEY.md §8c). This restatement is pinned against the reference's own known-answer tests,
 * transcribed as fixtures in tests/golden/ (BigVectorSpec, BigMatrixSpec, BufferedBigMatrixSpec,
 * GranularBigVectorSpec, GranularBigMatrixSpec, PartitioningSpec, SerializationSpec).
 *
 * Every function is a line-by-line restatement of the cited reference code, including its
 * integer-width quirks (Scala `.toInt` truncation of longs).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>
#include <pthread.h>

enum { O_I32 = 0, O_I64 = 1, O_F32 = 2, O_F64 = 3 };

static size_t dsize(int dt) { return (dt == O_I32 || dt == O_F32) ? 4 : 8; }

/* ----------------------------------------------------------------------------------------------
 * Partitioning
 * --------------------------------------------------------------------------------------------*/

/* RangePartitioner.apply -- src/main/scala/glint/partitioning/range/RangePartitioner.scala:62-84.
 * Fills starts/ends (length P) and returns the partitioner's (numberOfSmallPartitions,
 * smallPartitionSize) pair used by partition(). `keysPerSmallPartition` is `.toInt` truncated
 * exactly as at :66. */
void oracle_range_partitioner(int32_t P, int64_t N, int64_t* starts, int64_t* ends,
                              int32_t* n_small_out, int32_t* small_size_out) {
  int32_t n_large = (int32_t)(N % P);                    /* :64 */
  int32_t n_small = P - n_large;                         /* :65 */
  int32_t q = (int32_t)((N - (N % P)) / P);              /* :66 (.toInt) */
  int64_t start = 0, end = start + (int64_t)q;           /* :68-69 */
  for (int32_t i = 0; i < P; ++i) {                      /* :70 */
    if (i < n_small) {                                   /* :71 */
      starts[i] = start; ends[i] = end;                  /* :72 */
      start += q; end += q;                              /* :73-74 */
    } else {
      end += 1;                                          /* :76 */
      starts[i] = start; ends[i] = end;                  /* :77 */
      start += (int32_t)((uint32_t)q + 1u);              /* :78 (Int + 1 wraps, then widens) */
      end += q;                                          /* :79 */
    }
  }
  *n_small_out = n_small;
  *small_size_out = q;
}

/* RangePartitioner.partition -- RangePartitioner.scala:27-43. Returns -1 where the reference
 * throws IndexOutOfBoundsException (:30-32) or indexes the partition array below 0. All Int
 * arithmetic wraps as on the JVM: largePartitionSize = smallPartitionSize + 1 is an Int (:18), so a
 * partitioner with 2^31-1 keys per small partition divides by Int.MinValue, exactly like the
 * reference. */
int32_t oracle_range_partition(int64_t key, int32_t n_small, int32_t small_size, int64_t N) {
  if (key < 0 || key >= N) return -1;                                   /* :30-32 */
  int64_t n_small_keys = (int64_t)n_small * (int64_t)small_size;        /* RangePartitioner.scala:17 */
  int64_t large = (int32_t)((uint32_t)small_size + 1u);                /* :18 (Int + 1, wraps) */
  int64_t idx = key < n_small_keys ? key / small_size                   /* :37 */
                                   : (int64_t)n_small + (key - n_small_keys) / large; /* :39 */
  int32_t o = (int32_t)(uint32_t)(uint64_t)idx;                         /* .toInt */
  return o >= 0 ? o : -1;  /* an index >= P: the caller rejects it (partitions(idx) throws) */
}

/* RangePartition -- src/main/scala/glint/partitioning/range/RangePartition.scala:17,24,33 */
int32_t oracle_range_size(int64_t start, int64_t end) { return (int32_t)(end - start); }          /* :24 */
int32_t oracle_range_local(int64_t key, int64_t start) { return (int32_t)(key - start); }          /* :33 */
int oracle_range_contains(int64_t key, int64_t start, int64_t end) { return key >= start && key < end; } /* :17 */

/* CyclicPartition -- src/main/scala/glint/partitioning/cyclic/CyclicPartition.scala:21-47 */
int oracle_cyclic_contains(int64_t key, int32_t index, int32_t P) { return (int32_t)(key % P) == index; } /* :21-23 */
int32_t oracle_cyclic_local(int64_t key, int32_t index, int32_t P) { return (int32_t)((key - index) / P); } /* :45-47 */
int32_t oracle_cyclic_size(int32_t index, int32_t P, int64_t N) {                                  /* :30-36 */
  int64_t i = 1;
  while (!oracle_cyclic_contains(N - i, index, P)) {
    i += 1;
    /* the reference loops forever for a partition that owns no key; Client.create never builds
     * one (P = min(keys, ...), Client.scala:71), so report an empty partition instead */
    if (i > (int64_t)P + 1) return 0;
  }
  return oracle_cyclic_local(N - i, index, P) + 1;
}
/* CyclicPartitioner.partition -- CyclicPartitioner.scala:19-22. -1 where the reference throws
 * (key >= keys explicitly; negative keys through the negative array index at :21). */
int32_t oracle_cyclic_partition(int64_t key, int32_t P, int64_t N) {
  if (key >= N) return -1;
  int32_t idx = (int32_t)(key % P);
  if (idx < 0) return -1;
  return idx;
}

/* Shard layout descriptor: the Partition a partial model is constructed with. */
typedef struct {
  int32_t kind;   /* 0 range, 1 cyclic */
  int64_t start;  /* range */
  int64_t end;    /* range */
  int32_t index;  /* cyclic */
  int32_t nparts; /* cyclic */
  int64_t nkeys;  /* cyclic */
} oracle_partition;

static inline int32_t g2l(const oracle_partition* p, int64_t key) {
  return p->kind == 0 ? oracle_range_local(key, p->start) : oracle_cyclic_local(key, p->index, p->nparts);
}
int32_t oracle_partition_size(const oracle_partition* p) {
  return p->kind == 0 ? oracle_range_size(p->start, p->end) : oracle_cyclic_size(p->index, p->nparts, p->nkeys);
}

/* ----------------------------------------------------------------------------------------------
 * Server-side shard loops (the hot path)
 * --------------------------------------------------------------------------------------------*/

/* PartialVector.update -- src/main/scala/glint/models/server/PartialVector.scala:35-43.
 * Sequential, in message order: data(globalToLocal(k_i)) += v_i, with spire's Semiring `+` on JVM
 * primitives (IEEE-754 round-to-nearest for Float/Double, two's-complement wrap for Int/Long).
 * Returns -1 on success, else the index of the record whose local index is outside [0,size): the
 * JVM throws ArrayIndexOutOfBoundsException there, after records [0,i) were applied. */
int64_t oracle_vec_update(const oracle_partition* p, int dt, void* data, int32_t size,
                          const int64_t* keys, const void* vals, int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    int32_t k = g2l(p, keys[i]);                            /* :38 */
    if (k < 0 || k >= size) return i;                       /* JVM array bounds check */
    switch (dt) {                                           /* :39 */
      case O_F64: ((double*)data)[k] += ((const double*)vals)[i]; break;
      case O_F32: ((float*)data)[k] += ((const float*)vals)[i]; break;
      case O_I64: ((uint64_t*)data)[k] += ((const uint64_t*)vals)[i]; break;
      case O_I32: ((uint32_t*)data)[k] += ((const uint32_t*)vals)[i]; break;
    }
  }
  return -1;
}

/* PartialVector.get -- PartialVector.scala:51-60 */
int64_t oracle_vec_get(const oracle_partition* p, int dt, const void* data, int32_t size,
                       const int64_t* keys, void* out, int64_t n) {
  size_t s = dsize(dt);
  for (int64_t i = 0; i < n; ++i) {
    int32_t k = g2l(p, keys[i]);                            /* :55 */
    if (k < 0 || k >= size) return i;
    memcpy((char*)out + i * s, (const char*)data + (size_t)k * s, s);   /* :56 */
  }
  return -1;
}

/* PartialMatrix.update -- src/main/scala/glint/models/server/PartialMatrix.scala:74-83.
 * data is the row-major image of Array[Array[V]] (rows x cols). */
int64_t oracle_mat_update(const oracle_partition* p, int dt, void* data, int32_t rows, int32_t cols,
                          const int64_t* r, const int32_t* c, const void* vals, int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    int32_t row = g2l(p, r[i]);                             /* :77 */
    int32_t col = c[i];                                     /* :78 */
    if (row < 0 || row >= rows || col < 0 || col >= cols) return i;
    size_t at = (size_t)row * (size_t)cols + (size_t)col;
    switch (dt) {                                           /* :79 */
      case O_F64: ((double*)data)[at] += ((const double*)vals)[i]; break;
      case O_F32: ((float*)data)[at] += ((const float*)vals)[i]; break;
      case O_I64: ((uint64_t*)data)[at] += ((const uint64_t*)vals)[i]; break;
      case O_I32: ((uint32_t*)data)[at] += ((const uint32_t*)vals)[i]; break;
    }
  }
  return -1;
}

/* PartialMatrix.get -- PartialMatrix.scala:55-65 */
int64_t oracle_mat_get(const oracle_partition* p, int dt, const void* data, int32_t rows, int32_t cols,
                       const int64_t* r, const int32_t* c, void* out, int64_t n) {
  size_t s = dsize(dt);
  for (int64_t i = 0; i < n; ++i) {
    int32_t row = g2l(p, r[i]);
    int32_t col = c[i];
    if (row < 0 || row >= rows || col < 0 || col >= cols) return i;
    memcpy((char*)out + i * s, (const char*)data + ((size_t)row * cols + col) * s, s);
  }
  return -1;
}

/* PartialMatrix.getRows -- PartialMatrix.scala:37-46, flattened row-major the way
 * ResponseSerializer writes ResponseRows* (ResponseSerializer.scala:52-61). */
int64_t oracle_mat_get_rows(const oracle_partition* p, int dt, const void* data, int32_t rows, int32_t cols,
                            const int64_t* r, void* out, int64_t n) {
  size_t s = dsize(dt);
  for (int64_t i = 0; i < n; ++i) {
    int32_t row = g2l(p, r[i]);
    if (row < 0 || row >= rows) return i;
    memcpy((char*)out + (size_t)i * cols * s, (const char*)data + (size_t)row * cols * s, (size_t)cols * s);
  }
  return -1;
}

/* ----------------------------------------------------------------------------------------------
 * Client-side bucketing (the exchange step in front of the shards)
 * --------------------------------------------------------------------------------------------*/

/* AsyncBigVector.mapPartitions -- src/main/scala/glint/models/client/async/AsyncBigVector.scala:96-98
 * `keys.indices.groupBy(i => partitioner.partition(keys(i)))`: each bucket keeps its indices in
 * the caller's order (groupBy appends in traversal order). Restated as a stable counting sort by
 * partition index. Output: counts[P], offsets[P+1], order[n] (caller indices, bucket-major).
 * Returns -1, or the index of the first key the partitioner rejects (the reference throws
 * IndexOutOfBoundsException synchronously, before any message is sent). */
int64_t oracle_bucket_range(const int64_t* keys, int64_t n, int32_t P, int32_t n_small, int32_t small_size,
                            int64_t N, int64_t* counts, int64_t* offsets, int64_t* order) {
  int32_t* owner = (int32_t*)malloc((size_t)(n > 0 ? n : 1) * sizeof(int32_t));
  for (int32_t p = 0; p < P; ++p) counts[p] = 0;
  for (int64_t i = 0; i < n; ++i) {
    int32_t o = oracle_range_partition(keys[i], n_small, small_size, N);
    if (o < 0 || o >= P) { free(owner); return i; }
    owner[i] = o;
    counts[o]++;
  }
  offsets[0] = 0;
  for (int32_t p = 0; p < P; ++p) offsets[p + 1] = offsets[p] + counts[p];
  int64_t* cur = (int64_t*)malloc((size_t)P * sizeof(int64_t));
  for (int32_t p = 0; p < P; ++p) cur[p] = offsets[p];
  for (int64_t i = 0; i < n; ++i) order[cur[owner[i]]++] = i;
  free(cur); free(owner);
  return -1;
}

/* ----------------------------------------------------------------------------------------------
 * CPU baseline helper: one scalar thread per shard, as one actor per partition processes its
 * mailbox serially (PartialVector.scala:16-17, Akka's one-message-at-a-time guarantee).
 * --------------------------------------------------------------------------------------------*/
typedef struct {
  oracle_partition part; double* data; int32_t size; const int64_t* keys; const double* vals; int64_t n;
  int64_t rc;
} oracle_job;

static void* job_main(void* arg) {
  oracle_job* j = (oracle_job*)arg;
  j->rc = oracle_vec_update(&j->part, O_F64, j->data, j->size, j->keys, j->vals, j->n);
  return NULL;
}

/* Runs `nshards` independent PartialVector[Double].update loops on `nthreads` POSIX threads
 * (nthreads == nshards or 1). Shard s: range [starts[s], ends[s]), its own data array and its own
 * record stream. Returns the number of failed shards. */
typedef struct {
  oracle_job* jobs;
  int32_t first, step, count;
} oracle_worker;

static void* worker_main(void* arg) {
  oracle_worker* w = (oracle_worker*)arg;
  for (int32_t s = w->first; s < w->count; s += w->step) job_main(&w->jobs[s]);
  return NULL;
}

int oracle_vec_update_f64_parallel(int32_t nshards, const int64_t* starts, const int64_t* ends,
                                   double** datas, const int64_t** keys, const double** vals,
                                   const int64_t* ns, int32_t nthreads) {
  oracle_job* jobs = (oracle_job*)calloc((size_t)nshards, sizeof(oracle_job));
  for (int32_t s = 0; s < nshards; ++s) {
    jobs[s].part.kind = 0; jobs[s].part.start = starts[s]; jobs[s].part.end = ends[s];
    jobs[s].data = datas[s]; jobs[s].size = oracle_range_size(starts[s], ends[s]);
    jobs[s].keys = keys[s]; jobs[s].vals = vals[s]; jobs[s].n = ns[s];
  }
  if (nthreads <= 1) {
    for (int32_t s = 0; s < nshards; ++s) job_main(&jobs[s]);
  } else {
    /* nthreads workers; worker w runs the actors (shards) w, w + nthreads, ... one after another */
    if (nthreads > nshards) nthreads = nshards;
    oracle_worker* ws = (oracle_worker*)calloc((size_t)nthreads, sizeof(oracle_worker));
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
    for (int32_t w = 0; w < nthreads; ++w) {
      ws[w].jobs = jobs; ws[w].first = w; ws[w].step = nthreads; ws[w].count = nshards;
      pthread_create(&th[w], NULL, worker_main, &ws[w]);
    }
    for (int32_t w = 0; w < nthreads; ++w) pthread_join(th[w], NULL);
    free(th);
    free(ws);
  }
  int bad = 0;
  for (int32_t s = 0; s < nshards; ++s) bad += jobs[s].rc >= 0;
  free(jobs);
  return bad;
}
