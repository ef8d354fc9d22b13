/*
 * glint_jni.c -- JNI shim between Glint's server actors (Scala) and libglint_gpu.so.
 *
 * Binds the native methods of glint.models.server.gpu.GpuShard (integration/scala/GpuShard.scala) to
 * the C ABI in include/glint_gpu.h, one typed entry point per value type of the reference's partial
 * models (PartialVector{Double,Float,Long,Int}.scala, PartialMatrix{Double,Float,Long,Int}.scala).
 *
 * No JVM array is pinned across a GPU call. A push copies the message's arrays straight into one of
 * the shard's pinned ring slots with Get<T>ArrayRegion (glint_stage_acquire: no critical region, no
 * second copy) and is enqueued (glint_push_staged); the returned ticket is waited on
 * (glint_shard_wait) before the actor acknowledges the push (AcknowledgeReceipt, PushLogic.scala:40-66).
 * Pulls copy the keys out with Get<T>ArrayRegion and the answer in with Set<T>ArrayRegion.
 *
 * Argument checks mirror the reference: update(keys, values) loops over keys.length and reads
 * values(i), so a shorter values array throws ArrayIndexOutOfBoundsException
 * (PartialVector.scala:37-41) -- as does a shorter cols array for matrices (PartialMatrix.scala:77-81);
 * extra values are ignored. A value type that does not match the shard's is an
 * IllegalArgumentException. Library status codes become the exceptions the reference throws, so
 * Akka supervision behaves as with PartialVector/PartialMatrix.
 *
 * Build (needs a JDK):
 *   gcc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -I../../include \
 *       glint_jni.c -L../../glint_amd/lib -lglint_gpu -Wl,-rpath,'$ORIGIN' -o libglint_jni.so
 * tests/c/ compiles this same file against a minimal JNI environment and drives it on the GPU.
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include "glint_gpu.h"

static void throw_named(JNIEnv* env, const char* cls, const char* msg) {
  jclass c = (*env)->FindClass(env, cls);
  if (c) (*env)->ThrowNew(env, c, msg);
}

/* status -> the reference's exception types; returns nonzero when an exception is pending */
static int raise(JNIEnv* env, int rc, glint_shard_t s) {
  if (rc == GLINT_OK) return 0;
  if (rc == GLINT_EOUTOFRANGE) {
    int64_t bad = -1;
    if (s) glint_shard_last_error(s, &bad);
    char msg[96];
    snprintf(msg, sizeof msg, "record %lld is outside the partition", (long long)bad);
    throw_named(env, "java/lang/ArrayIndexOutOfBoundsException", msg);
  } else if (rc == GLINT_ENOMEM) {
    throw_named(env, "java/lang/OutOfMemoryError", glint_strerror(rc));
  } else if (rc == GLINT_EINVAL) {
    throw_named(env, "java/lang/IllegalArgumentException", glint_strerror(rc));
  } else {
    throw_named(env, "java/lang/RuntimeException", glint_strerror(rc));
  }
  return 1;
}

#define SHARD(h) ((glint_shard_t)(intptr_t)(h))

static int check_dtype(JNIEnv* env, glint_shard_t s, int want, int matrix) {
  int dt = -1;
  int32_t cols = 0;
  if (raise(env, glint_shard_info(s, NULL, &cols, &dt, NULL), s)) return 1;
  if (dt != want || (cols != 0) != matrix) {
    throw_named(env, "java/lang/IllegalArgumentException", "value type or model kind does not match the shard");
    return 1;
  }
  return 0;
}

/* values(i) for i < n must exist (the reference reads them in its loop) */
static int check_len(JNIEnv* env, jarray a, jsize n, const char* what) {
  if ((*env)->GetArrayLength(env, a) < n) {
    throw_named(env, "java/lang/ArrayIndexOutOfBoundsException", what);
    return 1;
  }
  return 0;
}

JNIEXPORT jlong JNICALL Java_glint_models_server_gpu_GpuShard_createRange(JNIEnv* env, jclass c, jint device,
                                                                          jint dtype, jlong start, jlong end,
                                                                          jint cols) {
  glint_shard_t s = NULL;
  if (raise(env, glint_shard_create(device, dtype, start, end, cols, &s), NULL)) return 0;
  return (jlong)(intptr_t)s;
}

JNIEXPORT jlong JNICALL Java_glint_models_server_gpu_GpuShard_createCyclic(JNIEnv* env, jclass c, jint device,
                                                                           jint dtype, jint index, jint parts,
                                                                           jlong keys, jint cols) {
  glint_shard_t s = NULL;
  if (raise(env, glint_shard_create_cyclic(device, dtype, index, parts, keys, cols, &s), NULL)) return 0;
  return (jlong)(intptr_t)s;
}

JNIEXPORT void JNICALL Java_glint_models_server_gpu_GpuShard_destroy(JNIEnv* env, jclass c, jlong h) {
  glint_shard_destroy(SHARD(h));
}

JNIEXPORT void JNICALL Java_glint_models_server_gpu_GpuShard_zero(JNIEnv* env, jclass c, jlong h) {
  raise(env, glint_shard_zero(SHARD(h)), SHARD(h));
}

/* Waits for the push with this ticket (and every earlier one) before the actor acknowledges it. */
JNIEXPORT void JNICALL Java_glint_models_server_gpu_GpuShard_await(JNIEnv* env, jclass c, jlong h, jlong ticket) {
  int64_t bad = -1;
  raise(env, glint_shard_wait(SHARD(h), (uint64_t)ticket, &bad), SHARD(h));
}

/* Pushes of more records than a ring slot is kept at (a few MiB; never an Akka message: the frame cap
 * is 79 999) go through the synchronous host-pointer entry points with a private copy of the arrays,
 * so no pinned slot is allocated and released per message. */
#define RING_MAX ((jsize)1 << 17)

/* ---- typed pushes: PartialVector.update / PartialMatrix.update -> ticket ------------------------- */
#define VEC_PUSH(SUF, JT, JARR, REGION, GLDT)                                                              \
  JNIEXPORT jlong JNICALL Java_glint_models_server_gpu_GpuShard_vecPush##SUF(                               \
      JNIEnv* env, jclass c, jlong h, jlongArray keys, JARR values, jint flags) {                            \
    glint_shard_t s = SHARD(h);                                                                             \
    if (check_dtype(env, s, GLDT, 0)) return 0;                                                             \
    const jsize n = (*env)->GetArrayLength(env, keys);                                                       \
    if (check_len(env, values, n, "values shorter than keys")) return 0;                                   \
    if (n > RING_MAX) {                                                                                     \
      jlong* k = (jlong*)malloc((size_t)n * 8);                                                             \
      JT* v = (JT*)malloc((size_t)n * sizeof(JT));                                                          \
      if (!k || !v) { free(k); free(v); raise(env, GLINT_ENOMEM, s); return 0; }                           \
      (*env)->GetLongArrayRegion(env, keys, 0, n, k);                                                       \
      (*env)->Get##REGION##ArrayRegion(env, values, 0, n, v);                                               \
      const int rc = glint_vec_push(s, (const int64_t*)k, v, n, flags);                                    \
      free(k);                                                                                              \
      free(v);                                                                                              \
      raise(env, rc, s);                                                                                    \
      return 0;                                                                                             \
    }                                                                                                       \
    void *kp, *vp;                                                                                          \
    int slot;                                                                                               \
    if (raise(env, glint_stage_acquire(s, n, &kp, NULL, &vp, &slot), s)) return 0;                         \
    (*env)->GetLongArrayRegion(env, keys, 0, n, (jlong*)kp);                                                \
    (*env)->Get##REGION##ArrayRegion(env, values, 0, n, (JT*)vp);                                           \
    uint64_t ticket = 0;                                                                                    \
    raise(env, glint_push_staged(s, slot, n, flags, &ticket), s);                                           \
    return (jlong)ticket;                                                                                   \
  }

#define MAT_PUSH(SUF, JT, JARR, REGION, GLDT)                                                              \
  JNIEXPORT jlong JNICALL Java_glint_models_server_gpu_GpuShard_matPush##SUF(                               \
      JNIEnv* env, jclass c, jlong h, jlongArray rows, jintArray cols, JARR values, jint flags) {             \
    glint_shard_t s = SHARD(h);                                                                             \
    if (check_dtype(env, s, GLDT, 1)) return 0;                                                             \
    const jsize n = (*env)->GetArrayLength(env, rows);                                                       \
    if (check_len(env, cols, n, "cols shorter than rows")) return 0;                                       \
    if (check_len(env, values, n, "values shorter than rows")) return 0;                                   \
    if (n > RING_MAX) {                                                                                     \
      jlong* r = (jlong*)malloc((size_t)n * 8);                                                             \
      jint* cc = (jint*)malloc((size_t)n * 4);                                                              \
      JT* v = (JT*)malloc((size_t)n * sizeof(JT));                                                          \
      if (!r || !cc || !v) { free(r); free(cc); free(v); raise(env, GLINT_ENOMEM, s); return 0; }          \
      (*env)->GetLongArrayRegion(env, rows, 0, n, r);                                                       \
      (*env)->GetIntArrayRegion(env, cols, 0, n, cc);                                                       \
      (*env)->Get##REGION##ArrayRegion(env, values, 0, n, v);                                               \
      const int rc = glint_mat_push(s, (const int64_t*)r, (const int32_t*)cc, v, n, flags);                \
      free(r);                                                                                              \
      free(cc);                                                                                             \
      free(v);                                                                                              \
      raise(env, rc, s);                                                                                    \
      return 0;                                                                                             \
    }                                                                                                       \
    void *rp, *cp, *vp;                                                                                     \
    int slot;                                                                                               \
    if (raise(env, glint_stage_acquire(s, n, &rp, &cp, &vp, &slot), s)) return 0;                          \
    (*env)->GetLongArrayRegion(env, rows, 0, n, (jlong*)rp);                                                \
    (*env)->GetIntArrayRegion(env, cols, 0, n, (jint*)cp);                                                  \
    (*env)->Get##REGION##ArrayRegion(env, values, 0, n, (JT*)vp);                                           \
    uint64_t ticket = 0;                                                                                    \
    raise(env, glint_push_staged(s, slot, n, flags, &ticket), s);                                           \
    return (jlong)ticket;                                                                                   \
  }

/* ---- typed pulls: PartialVector.get, PartialMatrix.get / getRows (flattened rows x cols) -------- */
#define PULLS(SUF, JT, JARR, REGION, GLDT)                                                                 \
  JNIEXPORT void JNICALL Java_glint_models_server_gpu_GpuShard_vecPull##SUF(JNIEnv* env, jclass c, jlong h, \
                                                                          jlongArray keys, JARR out) {       \
    glint_shard_t s = SHARD(h);                                                                             \
    if (check_dtype(env, s, GLDT, 0)) return;                                                               \
    const jsize n = (*env)->GetArrayLength(env, keys);                                                       \
    if (check_len(env, out, n, "result array shorter than keys")) return;                                  \
    jlong* k = (jlong*)malloc((size_t)n * 8 + 8);                                                           \
    JT* o = (JT*)malloc((size_t)n * sizeof(JT) + 8);                                                        \
    if (!k || !o) { free(k); free(o); raise(env, GLINT_ENOMEM, s); return; }                               \
    (*env)->GetLongArrayRegion(env, keys, 0, n, k);                                                         \
    const int rc = glint_vec_pull(s, (const int64_t*)k, o, n);                                             \
    if (rc == GLINT_OK) (*env)->Set##REGION##ArrayRegion(env, out, 0, n, o);                                \
    free(k);                                                                                                \
    free(o);                                                                                                \
    raise(env, rc, s);                                                                                      \
  }                                                                                                         \
  JNIEXPORT void JNICALL Java_glint_models_server_gpu_GpuShard_matPull##SUF(                                 \
      JNIEnv* env, jclass c, jlong h, jlongArray rows, jintArray cols, JARR out) {                           \
    glint_shard_t s = SHARD(h);                                                                             \
    if (check_dtype(env, s, GLDT, 1)) return;                                                               \
    const jsize n = (*env)->GetArrayLength(env, rows);                                                       \
    if (check_len(env, cols, n, "cols shorter than rows")) return;                                         \
    if (check_len(env, out, n, "result array shorter than rows")) return;                                  \
    jlong* r = (jlong*)malloc((size_t)n * 8 + 8);                                                           \
    jint* cc = (jint*)malloc((size_t)n * 4 + 8);                                                            \
    JT* o = (JT*)malloc((size_t)n * sizeof(JT) + 8);                                                        \
    if (!r || !cc || !o) { free(r); free(cc); free(o); raise(env, GLINT_ENOMEM, s); return; }              \
    (*env)->GetLongArrayRegion(env, rows, 0, n, r);                                                         \
    (*env)->GetIntArrayRegion(env, cols, 0, n, cc);                                                         \
    const int rc = glint_mat_pull(s, (const int64_t*)r, (const int32_t*)cc, o, n);                         \
    if (rc == GLINT_OK) (*env)->Set##REGION##ArrayRegion(env, out, 0, n, o);                                \
    free(r);                                                                                                \
    free(cc);                                                                                               \
    free(o);                                                                                                \
    raise(env, rc, s);                                                                                      \
  }                                                                                                         \
  JNIEXPORT void JNICALL Java_glint_models_server_gpu_GpuShard_matPullRows##SUF(                             \
      JNIEnv* env, jclass c, jlong h, jlongArray rows, JARR out) {                                           \
    glint_shard_t s = SHARD(h);                                                                             \
    if (check_dtype(env, s, GLDT, 1)) return;                                                               \
    int32_t ncols = 0;                                                                                      \
    glint_shard_info(s, NULL, &ncols, NULL, NULL);                                                          \
    const jsize n = (*env)->GetArrayLength(env, rows);                                                       \
    const int64_t total = (int64_t)n * ncols;                                                               \
    if (total > 0x7fffffff || check_len(env, out, (jsize)total, "result array shorter than rows x cols"))  \
      return;                                                                                               \
    jlong* r = (jlong*)malloc((size_t)n * 8 + 8);                                                           \
    JT* o = (JT*)malloc((size_t)total * sizeof(JT) + 8);                                                    \
    if (!r || !o) { free(r); free(o); raise(env, GLINT_ENOMEM, s); return; }                               \
    (*env)->GetLongArrayRegion(env, rows, 0, n, r);                                                         \
    const int rc = glint_mat_pull_rows(s, (const int64_t*)r, o, n);                                        \
    if (rc == GLINT_OK) (*env)->Set##REGION##ArrayRegion(env, out, 0, (jsize)total, o);                     \
    free(r);                                                                                                \
    free(o);                                                                                                \
    raise(env, rc, s);                                                                                      \
  }

/* ---- pipelined pulls: the actor enqueues a Pull and answers the burst's pulls after one wait -------
 * pullAsync copies the keys (and cols) out of the JVM arrays and enqueues the pull (glint_pull_async)
 * into a native answer buffer; it returns a handle. pullFinish<T> waits for that pull's ticket, copies
 * the answer into the result array and frees the handle. kind: 0 PartialVector.get, 1
 * PartialMatrix.get, 2 PartialMatrix.getRows (flattened rows x cols). An out-of-partition key throws
 * from pullAsync (the Pull message itself), with nothing enqueued. */
typedef struct {
  glint_shard_t s;
  uint64_t ticket;
  int64_t count; /* answer elements */
  int dtype;
  void* buf;
} pending_pull;

#define PULL_ASYNC_MAX ((jsize)1 << 20) /* glint_pull_async's bound; larger pulls are answered at once */

JNIEXPORT jlong JNICALL Java_glint_models_server_gpu_GpuShard_pullAsync(JNIEnv* env, jclass c, jlong h, jint kind,
                                                                        jlongArray rows, jintArray cols) {
  glint_shard_t s = SHARD(h);
  int dt = -1;
  int32_t ncols = 0;
  if (raise(env, glint_shard_info(s, NULL, &ncols, &dt, NULL), s)) return 0;
  if (kind < 0 || kind > 2 || (kind == 0) != (ncols == 0)) {
    throw_named(env, "java/lang/IllegalArgumentException", "pull kind does not match the shard");
    return 0;
  }
  const jsize n = (*env)->GetArrayLength(env, rows);
  if (kind == 1 && check_len(env, cols, n, "cols shorter than rows")) return 0;
  const int64_t count = kind == 2 ? (int64_t)n * ncols : (int64_t)n;
  if (count > 0x7fffffff) {
    throw_named(env, "java/lang/IllegalArgumentException", "answer larger than a JVM array");
    return 0;
  }
  const size_t vsize = (dt == GLINT_F64 || dt == GLINT_I64) ? 8 : 4;
  pending_pull* p = (pending_pull*)calloc(1, sizeof(pending_pull));
  jlong* r = (jlong*)malloc((size_t)n * 8 + 8);
  jint* cc = kind == 1 ? (jint*)malloc((size_t)n * 4 + 8) : NULL;
  void* buf = malloc((size_t)count * vsize + 8);
  if (!p || !r || (kind == 1 && !cc) || !buf) {
    free(p); free(r); free(cc); free(buf);
    raise(env, GLINT_ENOMEM, s);
    return 0;
  }
  (*env)->GetLongArrayRegion(env, rows, 0, n, r);
  if (kind == 1) (*env)->GetIntArrayRegion(env, cols, 0, n, cc);
  int rc;
  uint64_t ticket = 0;
  if (n > PULL_ASYNC_MAX) {
    rc = kind == 0   ? glint_vec_pull(s, (const int64_t*)r, buf, n)
         : kind == 1 ? glint_mat_pull(s, (const int64_t*)r, (const int32_t*)cc, buf, n)
                     : glint_mat_pull_rows(s, (const int64_t*)r, buf, n);
  } else {
    rc = glint_pull_async(s, kind, (const int64_t*)r, (const int32_t*)cc, buf, n, &ticket);
  }
  free(r);
  free(cc);
  if (raise(env, rc, s)) {
    free(buf);
    free(p);
    return 0;
  }
  p->s = s;
  p->ticket = ticket;
  p->count = count;
  p->dtype = dt;
  p->buf = buf;
  return (jlong)(intptr_t)p;
}

#define PULL_FINISH(SUF, JT, JARR, REGION, GLDT)                                                           \
  JNIEXPORT void JNICALL Java_glint_models_server_gpu_GpuShard_pullFinish##SUF(JNIEnv* env, jclass c,         \
                                                                             jlong pending, JARR out) {    \
    pending_pull* p = (pending_pull*)(intptr_t)pending;                                                     \
    if (!p) return;                                                                                         \
    int rc = glint_shard_wait(p->s, p->ticket, NULL);                                                       \
    if (rc == GLINT_OK && p->dtype != GLDT) {                                                               \
      throw_named(env, "java/lang/IllegalArgumentException", "value type does not match the shard");       \
    } else if (rc == GLINT_OK && !check_len(env, out, (jsize)p->count, "result array shorter than answer")) { \
      (*env)->Set##REGION##ArrayRegion(env, out, 0, (jsize)p->count, (const JT*)p->buf);                    \
    }                                                                                                       \
    const glint_shard_t s = p->s;                                                                           \
    free(p->buf);                                                                                           \
    free(p);                                                                                                \
    raise(env, rc, s);                                                                                      \
  }

PULL_FINISH(D, jdouble, jdoubleArray, Double, GLINT_F64)
PULL_FINISH(F, jfloat, jfloatArray, Float, GLINT_F32)
PULL_FINISH(L, jlong, jlongArray, Long, GLINT_I64)
PULL_FINISH(I, jint, jintArray, Int, GLINT_I32)

VEC_PUSH(D, jdouble, jdoubleArray, Double, GLINT_F64)
VEC_PUSH(F, jfloat, jfloatArray, Float, GLINT_F32)
VEC_PUSH(L, jlong, jlongArray, Long, GLINT_I64)
VEC_PUSH(I, jint, jintArray, Int, GLINT_I32)
MAT_PUSH(D, jdouble, jdoubleArray, Double, GLINT_F64)
MAT_PUSH(F, jfloat, jfloatArray, Float, GLINT_F32)
MAT_PUSH(L, jlong, jlongArray, Long, GLINT_I64)
MAT_PUSH(I, jint, jintArray, Int, GLINT_I32)
PULLS(D, jdouble, jdoubleArray, Double, GLINT_F64)
PULLS(F, jfloat, jfloatArray, Float, GLINT_F32)
PULLS(L, jlong, jlongArray, Long, GLINT_I64)
PULLS(I, jint, jintArray, Int, GLINT_I32)
