/*
 * glint_jni.c -- JNI shim between Glint's server actors (Scala) and libglint_gpu.so.
 *
 * Binds the native methods of glint.models.server.gpu.GpuShard (integration/scala/GpuShard.scala)
 * to the C ABI in include/glint_gpu.h. Arrays are pinned with GetPrimitiveArrayCritical for the
 * duration of the (synchronous) call -- the library copies them to HBM before returning -- and
 * status codes become the exceptions the reference throws, so Akka supervision behaves as with
 * PartialVector/PartialMatrix (M/models/server/PartialVector.scala:35-60).
 *
 * Build (needs a JDK; not part of this image's CI):
 *   gcc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -I../../include \
 *       glint_jni.c -L../../glint_amd/lib -lglint_gpu -Wl,-rpath,'$ORIGIN' -o libglint_jni.so
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include "glint_gpu.h"

static void raise(JNIEnv* env, int rc, glint_shard_t s) {
  if (rc == GLINT_OK) return;
  if (rc == GLINT_EOUTOFRANGE) {
    int64_t bad = -1;
    glint_shard_last_error(s, &bad);
    char msg[96];
    snprintf(msg, sizeof msg, "record %lld is outside the partition", (long long)bad);
    (*env)->ThrowNew(env, (*env)->FindClass(env, "java/lang/ArrayIndexOutOfBoundsException"), msg);
  } else if (rc == GLINT_ENOMEM) {
    (*env)->ThrowNew(env, (*env)->FindClass(env, "java/lang/OutOfMemoryError"), glint_strerror(rc));
  } else if (rc == GLINT_EINVAL) {
    (*env)->ThrowNew(env, (*env)->FindClass(env, "java/lang/IllegalArgumentException"), glint_strerror(rc));
  } else {
    (*env)->ThrowNew(env, (*env)->FindClass(env, "java/lang/RuntimeException"), glint_strerror(rc));
  }
}

#define SHARD(h) ((glint_shard_t)(intptr_t)(h))

JNIEXPORT jlong JNICALL Java_glint_models_server_gpu_GpuShard_createRange(JNIEnv* env, jclass c, jint device,
                                                                          jint dtype, jlong start, jlong end,
                                                                          jint cols) {
  glint_shard_t s = NULL;
  int rc = glint_shard_create(device, dtype, start, end, cols, &s);
  if (rc) { raise(env, rc, NULL); return 0; }
  return (jlong)(intptr_t)s;
}

JNIEXPORT jlong JNICALL Java_glint_models_server_gpu_GpuShard_createCyclic(JNIEnv* env, jclass c, jint device,
                                                                           jint dtype, jint index, jint parts,
                                                                           jlong keys, jint cols) {
  glint_shard_t s = NULL;
  int rc = glint_shard_create_cyclic(device, dtype, index, parts, keys, cols, &s);
  if (rc) { raise(env, rc, NULL); return 0; }
  return (jlong)(intptr_t)s;
}

JNIEXPORT void JNICALL Java_glint_models_server_gpu_GpuShard_destroy(JNIEnv* env, jclass c, jlong h) {
  glint_shard_destroy(SHARD(h));
}

JNIEXPORT void JNICALL Java_glint_models_server_gpu_GpuShard_zero(JNIEnv* env, jclass c, jlong h) {
  raise(env, glint_shard_zero(SHARD(h)), SHARD(h));
}

/* PartialVector.update(keys, values): values is a jdoubleArray / jfloatArray / jlongArray / jintArray
 * matching the shard's dtype (checked on the Scala side). */
JNIEXPORT void JNICALL Java_glint_models_server_gpu_GpuShard_vecPush(JNIEnv* env, jclass c, jlong h,
                                                                     jlongArray keys, jarray values,
                                                                     jint deterministic) {
  const jsize n = (*env)->GetArrayLength(env, keys);
  jlong* k = (*env)->GetPrimitiveArrayCritical(env, keys, NULL);
  void* v = (*env)->GetPrimitiveArrayCritical(env, values, NULL);
  int rc = glint_vec_push(SHARD(h), (const int64_t*)k, v, n, deterministic ? GLINT_PUSH_DETERMINISTIC : 0);
  (*env)->ReleasePrimitiveArrayCritical(env, values, v, JNI_ABORT);
  (*env)->ReleasePrimitiveArrayCritical(env, keys, k, JNI_ABORT);
  raise(env, rc, SHARD(h));
}

/* PartialVector.get(keys) into a caller-allocated result array (the new Array[V] of get). */
JNIEXPORT void JNICALL Java_glint_models_server_gpu_GpuShard_vecPull(JNIEnv* env, jclass c, jlong h,
                                                                     jlongArray keys, jarray out) {
  const jsize n = (*env)->GetArrayLength(env, keys);
  jlong* k = (*env)->GetPrimitiveArrayCritical(env, keys, NULL);
  void* o = (*env)->GetPrimitiveArrayCritical(env, out, NULL);
  int rc = glint_vec_pull(SHARD(h), (const int64_t*)k, o, n);
  (*env)->ReleasePrimitiveArrayCritical(env, out, o, 0);
  (*env)->ReleasePrimitiveArrayCritical(env, keys, k, JNI_ABORT);
  raise(env, rc, SHARD(h));
}

/* PartialMatrix.update(rows, cols, values) */
JNIEXPORT void JNICALL Java_glint_models_server_gpu_GpuShard_matPush(JNIEnv* env, jclass c, jlong h,
                                                                     jlongArray rows, jintArray cols,
                                                                     jarray values, jint deterministic) {
  const jsize n = (*env)->GetArrayLength(env, rows);
  jlong* r = (*env)->GetPrimitiveArrayCritical(env, rows, NULL);
  jint* cc = (*env)->GetPrimitiveArrayCritical(env, cols, NULL);
  void* v = (*env)->GetPrimitiveArrayCritical(env, values, NULL);
  int rc = glint_mat_push(SHARD(h), (const int64_t*)r, (const int32_t*)cc, v, n,
                          deterministic ? GLINT_PUSH_DETERMINISTIC : 0);
  (*env)->ReleasePrimitiveArrayCritical(env, values, v, JNI_ABORT);
  (*env)->ReleasePrimitiveArrayCritical(env, cols, cc, JNI_ABORT);
  (*env)->ReleasePrimitiveArrayCritical(env, rows, r, JNI_ABORT);
  raise(env, rc, SHARD(h));
}

/* PartialMatrix.get(rows, cols) */
JNIEXPORT void JNICALL Java_glint_models_server_gpu_GpuShard_matPull(JNIEnv* env, jclass c, jlong h,
                                                                     jlongArray rows, jintArray cols, jarray out) {
  const jsize n = (*env)->GetArrayLength(env, rows);
  jlong* r = (*env)->GetPrimitiveArrayCritical(env, rows, NULL);
  jint* cc = (*env)->GetPrimitiveArrayCritical(env, cols, NULL);
  void* o = (*env)->GetPrimitiveArrayCritical(env, out, NULL);
  int rc = glint_mat_pull(SHARD(h), (const int64_t*)r, (const int32_t*)cc, o, n);
  (*env)->ReleasePrimitiveArrayCritical(env, out, o, 0);
  (*env)->ReleasePrimitiveArrayCritical(env, cols, cc, JNI_ABORT);
  (*env)->ReleasePrimitiveArrayCritical(env, rows, r, JNI_ABORT);
  raise(env, rc, SHARD(h));
}

/* PartialMatrix.getRows(rows), flattened rows x cols (what ResponseSerializer sends,
 * M/serialization/ResponseSerializer.scala:52-61) */
JNIEXPORT void JNICALL Java_glint_models_server_gpu_GpuShard_matPullRows(JNIEnv* env, jclass c, jlong h,
                                                                         jlongArray rows, jarray out) {
  const jsize n = (*env)->GetArrayLength(env, rows);
  jlong* r = (*env)->GetPrimitiveArrayCritical(env, rows, NULL);
  void* o = (*env)->GetPrimitiveArrayCritical(env, out, NULL);
  int rc = glint_mat_pull_rows(SHARD(h), (const int64_t*)r, o, n);
  (*env)->ReleasePrimitiveArrayCritical(env, out, o, 0);
  (*env)->ReleasePrimitiveArrayCritical(env, rows, r, JNI_ABORT);
  raise(env, rc, SHARD(h));
}
