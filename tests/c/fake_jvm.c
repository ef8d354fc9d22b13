/* The JNIEnv of tests/c/jni.h over plain C arrays, plus a driver that calls the shim's native
 * methods in the order the GPU actors (integration/scala/GpuShard.scala) call them:
 * create -> push (ticket) -> await -> pull; an order-sensitive Double push; an out-of-partition
 * push throws ArrayIndexOutOfBoundsException at the Push message itself (as update() throws inside
 * receive, PartialVectorDouble.scala:17-23) and applies nothing, while earlier pushes' awaits and a
 * pull stay clean; an out-of-partition pull throws the same way; pipelined pulls (pullAsync, then
 * pullFinish after the burst) see the pushes enqueued before them; zero (the Akka restart) -> push again;
 * argument errors (value type, short arrays); a matrix shard's element and row pulls; destroy; and
 * MatrixBenchmark's update -> get -> getRows sequence on a range and a cyclic Double matrix, getRows
 * restated from the Scala override (a flat row pull cut into cols-long rows).
 * Exit status 0 and "ok" on stdout when every check passes. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jni.h"

typedef struct {
  jsize len;
  size_t esize;
  char* data;
} Arr;

static char pending[256];  /* the exception the shim raised: "Class: message" */

static jclass FindClass(JNIEnv* e, const char* n) { (void)e; return (jclass)n; }
static jint ThrowNew(JNIEnv* e, jclass c, const char* m) {
  (void)e;
  snprintf(pending, sizeof pending, "%s: %s", (const char*)c, m);
  return 0;
}
static jsize GetArrayLength(JNIEnv* e, jarray a) { (void)e; return ((Arr*)a)->len; }
static void get_region(jarray a, jsize s, jsize n, void* buf) {
  Arr* x = (Arr*)a;
  if (s < 0 || n < 0 || s + n > x->len) { fprintf(stderr, "region out of bounds\n"); exit(3); }
  memcpy(buf, x->data + (size_t)s * x->esize, (size_t)n * x->esize);
}
static void set_region(jarray a, jsize s, jsize n, const void* buf) {
  Arr* x = (Arr*)a;
  if (s < 0 || n < 0 || s + n > x->len) { fprintf(stderr, "region out of bounds\n"); exit(3); }
  memcpy(x->data + (size_t)s * x->esize, buf, (size_t)n * x->esize);
}
static void GL(JNIEnv* e, jlongArray a, jsize s, jsize n, jlong* b) { (void)e; get_region(a, s, n, b); }
static void GI(JNIEnv* e, jintArray a, jsize s, jsize n, jint* b) { (void)e; get_region(a, s, n, b); }
static void GF(JNIEnv* e, jfloatArray a, jsize s, jsize n, jfloat* b) { (void)e; get_region(a, s, n, b); }
static void GD(JNIEnv* e, jdoubleArray a, jsize s, jsize n, jdouble* b) { (void)e; get_region(a, s, n, b); }
static void SL(JNIEnv* e, jlongArray a, jsize s, jsize n, const jlong* b) { (void)e; set_region(a, s, n, b); }
static void SI(JNIEnv* e, jintArray a, jsize s, jsize n, const jint* b) { (void)e; set_region(a, s, n, b); }
static void SF(JNIEnv* e, jfloatArray a, jsize s, jsize n, const jfloat* b) { (void)e; set_region(a, s, n, b); }
static void SD(JNIEnv* e, jdoubleArray a, jsize s, jsize n, const jdouble* b) { (void)e; set_region(a, s, n, b); }

static const struct JNINativeInterface_ table = {FindClass, ThrowNew, GetArrayLength, GL, GI, GF, GD, SL, SI, SF, SD};
static JNIEnv env_ptr = &table;
static JNIEnv* env = &env_ptr;

static Arr* arr(jsize n, size_t es) {
  Arr* a = (Arr*)calloc(1, sizeof(Arr));
  a->len = n;
  a->esize = es;
  a->data = (char*)calloc((size_t)(n > 0 ? n : 1), es);
  return a;
}

/* the shim's native methods (integration/jni/glint_jni.c) */
#define NAT(name) Java_glint_models_server_gpu_GpuShard_##name
jlong NAT(createRange)(JNIEnv*, jclass, jint, jint, jlong, jlong, jint);
void NAT(destroy)(JNIEnv*, jclass, jlong);
void NAT(zero)(JNIEnv*, jclass, jlong);
void NAT(await)(JNIEnv*, jclass, jlong, jlong);
jlong NAT(vecPushD)(JNIEnv*, jclass, jlong, jlongArray, jdoubleArray, jint);
jlong NAT(vecPushF)(JNIEnv*, jclass, jlong, jlongArray, jfloatArray, jint);
void NAT(vecPullD)(JNIEnv*, jclass, jlong, jlongArray, jdoubleArray);
jlong NAT(matPushI)(JNIEnv*, jclass, jlong, jlongArray, jintArray, jintArray, jint);
void NAT(matPullI)(JNIEnv*, jclass, jlong, jlongArray, jintArray, jintArray);
void NAT(matPullRowsI)(JNIEnv*, jclass, jlong, jlongArray, jintArray);
jlong NAT(pullAsync)(JNIEnv*, jclass, jlong, jint, jlongArray, jintArray);
void NAT(pullFinishD)(JNIEnv*, jclass, jlong, jdoubleArray);
void NAT(pullFinishI)(JNIEnv*, jclass, jlong, jintArray);
jlong NAT(createCyclic)(JNIEnv*, jclass, jint, jint, jint, jint, jlong, jint);
jlong NAT(matPushD)(JNIEnv*, jclass, jlong, jlongArray, jintArray, jdoubleArray, jint);
void NAT(matPullD)(JNIEnv*, jclass, jlong, jlongArray, jintArray, jdoubleArray);
void NAT(matPullRowsD)(JNIEnv*, jclass, jlong, jlongArray, jdoubleArray);

static int failures = 0;
#define CHECK(cond, what)                                            \
  do {                                                               \
    if (!(cond)) { fprintf(stderr, "FAILED: %s\n", what); ++failures; } \
  } while (0)
static int took(const char* cls) {
  const int hit = strncmp(pending, cls, strlen(cls)) == 0;
  pending[0] = 0;
  return hit;
}

/* GpuPartialMatrixDouble.getRows (integration/scala/GpuShard.scala): getRowsFlat -- one flat row pull
 * (matPullRowsD) -- cut into cols-long rows, each its own array, as PartialMatrix.getRows returns
 * Array[Array[Double]] (PartialMatrix.scala:37-46) */
static Arr** get_rows(jlong h, Arr* rows, int cols) {
  Arr* flat = arr(rows->len * cols, 8);
  NAT(matPullRowsD)(env, NULL, h, rows, flat);
  Arr** out = (Arr**)calloc((size_t)rows->len, sizeof(Arr*));
  for (jsize i = 0; i < rows->len; ++i) {
    out[i] = arr(cols, 8);
    memcpy(out[i]->data, flat->data + (size_t)i * cols * 8, (size_t)cols * 8);
  }
  return out;
}

/* MatrixBenchmark.scala:24-47,54-101 on one shard: update, then get, then getRows, for its range
 * (RangePartition(1, 10000, 20000)) and cyclic (CyclicPartition(3, 10, 100000)) PartialMatrixDouble of
 * 300 cols, `size` records row x + 10000 (range) / 10 x + 3 (cyclic), col x % 300, value 0.25 x + 1 */
static void matrix_benchmark(int dev, int cyclic, int size) {
  const int cols = 300;
  const jlong h = cyclic ? NAT(createCyclic)(env, NULL, dev, 3, 3, 10, (jlong)(10000 - 1) * 10 + 3 + 1, cols)
                         : NAT(createRange)(env, NULL, dev, 3, 10000, 20000, cols);
  CHECK(h != 0 && !pending[0], "MatrixBenchmark shard");
  Arr* r = arr(size, 8);
  Arr* c = arr(size, 4);
  Arr* v = arr(size, 8);
  for (int x = 0; x < size; ++x) {
    ((jlong*)r->data)[x] = cyclic ? 10L * x + 3 : (jlong)x + 10000;
    ((jint*)c->data)[x] = x % cols;
    ((jdouble*)v->data)[x] = 0.25 * x + 1.0;
  }
  NAT(await)(env, NULL, h, NAT(matPushD)(env, NULL, h, r, c, v, 0));  /* update */
  CHECK(!pending[0], "MatrixBenchmark update");
  Arr* o = arr(size, 8);
  NAT(matPullD)(env, NULL, h, r, c, o);  /* get */
  CHECK(!pending[0] && !memcmp(o->data, v->data, (size_t)size * 8), "MatrixBenchmark get");
  Arr** rows = get_rows(h, r, cols);  /* getRows: row x holds 0.25 x + 1 at col x % 300, zeros elsewhere */
  int ok = !pending[0];
  for (int x = 0; x < size && ok; ++x)
    for (int j = 0; j < cols; ++j)
      ok &= ((jdouble*)rows[x]->data)[j] == (j == x % cols ? 0.25 * x + 1.0 : 0.0);
  CHECK(ok, cyclic ? "MatrixBenchmark getRows (cyclic)" : "MatrixBenchmark getRows (range)");
  /* a row outside the partition: getRows throws as data(row) would (ArrayIndexOutOfBoundsException) */
  Arr* bad = arr(1, 8);
  ((jlong*)bad->data)[0] = cyclic ? 100003 : 20000;
  free(get_rows(h, bad, cols));
  CHECK(took("java/lang/ArrayIndexOutOfBoundsException"), "getRows of a row outside the partition");
  NAT(destroy)(env, NULL, h);
}

int main(int argc, char** argv) {
  const int dev = argc > 1 ? atoi(argv[1]) : 0;
  /* a PartialVectorDouble of RangePartition(0, 1000, 2000) */
  jlong h = NAT(createRange)(env, NULL, dev, 3, 1000, 2000, 0);
  CHECK(h != 0 && !pending[0], "createRange");
  Arr* k = arr(1000, 8);
  Arr* v = arr(1000, 8);
  for (int i = 0; i < 1000; ++i) {
    ((jlong*)k->data)[i] = 1000 + i;
    ((jdouble*)v->data)[i] = 0.5 * i;
  }
  jlong t = NAT(vecPushD)(env, NULL, h, k, v, 0);
  CHECK(t > 0 && !pending[0], "vecPushD ticket");
  NAT(await)(env, NULL, h, t);
  CHECK(!pending[0], "await");
  Arr* out = arr(1000, 8);
  NAT(vecPullD)(env, NULL, h, k, out);
  int same = 1;
  for (int i = 0; i < 1000; ++i) same &= ((jdouble*)out->data)[i] == 0.5 * i;
  CHECK(same && !pending[0], "pull after push");
  /* one message, one key three times: the JVM's ((d + 1e16) + 1) + 1, not d + (1e16 + 2) */
  Arr* k3 = arr(3, 8);
  Arr* v3 = arr(3, 8);
  for (int i = 0; i < 3; ++i) ((jlong*)k3->data)[i] = 1000;
  ((jdouble*)v3->data)[0] = 1e16;
  ((jdouble*)v3->data)[1] = 1.0;
  ((jdouble*)v3->data)[2] = 1.0;
  NAT(await)(env, NULL, h, NAT(vecPushD)(env, NULL, h, k3, v3, 0));
  Arr* o1 = arr(3, 8);
  NAT(vecPullD)(env, NULL, h, k3, o1);
  CHECK(!pending[0], "pull of a repeated key");
  volatile double seq = 0.0;
  seq = seq + 1e16;
  seq = seq + 1.0;
  seq = seq + 1.0;
  CHECK(((jdouble*)o1->data)[0] == seq && ((jdouble*)o1->data)[2] == seq, "sequential Double order");
  /* an out-of-partition key: the Push itself throws ArrayIndexOutOfBoundsException and nothing of it
   * is applied; a push enqueued before it and a pull after it are clean; restart = zero */
  Arr* kb = arr(2, 8);
  Arr* vb = arr(2, 8);
  ((jlong*)kb->data)[0] = 1001;
  ((jlong*)kb->data)[1] = 2000;
  ((jdouble*)vb->data)[0] = 7.0;
  Arr* k1 = arr(1, 8);
  Arr* v1 = arr(1, 8);
  ((jlong*)k1->data)[0] = 1002;
  ((jdouble*)v1->data)[0] = 0.25;
  const jlong t_before = NAT(vecPushD)(env, NULL, h, k1, v1, 0);
  CHECK(t_before > 0 && !pending[0], "push before the bad one");
  NAT(vecPushD)(env, NULL, h, kb, vb, 0);
  CHECK(took("java/lang/ArrayIndexOutOfBoundsException"), "out-of-partition key raises at the Push");
  NAT(await)(env, NULL, h, t_before);
  CHECK(!pending[0], "the earlier push's await is clean");
  Arr* k2 = arr(2, 8);
  ((jlong*)k2->data)[0] = 1001;
  ((jlong*)k2->data)[1] = 1002;
  Arr* o2 = arr(2, 8);
  NAT(vecPullD)(env, NULL, h, k2, o2);
  CHECK(!pending[0] && ((jdouble*)o2->data)[0] == 0.5 && ((jdouble*)o2->data)[1] == 1.0 + 0.25,
        "clean pull after the bad push; the bad push applied nothing");
  NAT(vecPullD)(env, NULL, h, kb, o2);
  CHECK(took("java/lang/ArrayIndexOutOfBoundsException"), "out-of-partition pull raises");
  /* pipelined pulls (the actor's burst): a push enqueued, two pulls enqueued behind it, then answered */
  const jlong tp = NAT(vecPushD)(env, NULL, h, k1, v1, 0);
  const jlong pa = NAT(pullAsync)(env, NULL, h, 0, k2, NULL);
  const jlong pb = NAT(pullAsync)(env, NULL, h, 0, k, NULL);
  CHECK(tp > 0 && pa != 0 && pb != 0 && !pending[0], "pulls enqueued behind a push");
  Arr* oa = arr(2, 8);
  NAT(pullFinishD)(env, NULL, pa, oa);
  NAT(pullFinishD)(env, NULL, pb, out);
  CHECK(!pending[0] && ((jdouble*)oa->data)[0] == 0.5 && ((jdouble*)oa->data)[1] == 1.0 + 0.5,
        "async pull sees the push enqueued before it");
  CHECK(((jdouble*)out->data)[0] == seq && ((jdouble*)out->data)[999] == 0.5 * 999, "async pull of 1000 keys");
  CHECK(NAT(pullAsync)(env, NULL, h, 0, kb, NULL) == 0 && took("java/lang/ArrayIndexOutOfBoundsException"),
        "out-of-partition async pull raises at the Pull");
  NAT(pullAsync)(env, NULL, h, 2, k2, NULL);
  CHECK(took("java/lang/IllegalArgumentException"), "row pull of a vector shard");
  NAT(zero)(env, NULL, h);
  NAT(await)(env, NULL, h, NAT(vecPushD)(env, NULL, h, k3, v3, 0));
  NAT(vecPullD)(env, NULL, h, k3, o1);
  CHECK(((jdouble*)o1->data)[0] == seq && !pending[0], "push after restart");
  /* argument errors */
  Arr* vf = arr(1000, 4);
  NAT(vecPushF)(env, NULL, h, k, vf, 0);
  CHECK(took("java/lang/IllegalArgumentException"), "value type mismatch");
  Arr* vs = arr(999, 8);
  NAT(vecPushD)(env, NULL, h, k, vs, 0);
  CHECK(took("java/lang/ArrayIndexOutOfBoundsException"), "short values");
  NAT(destroy)(env, NULL, h);

  /* a PartialMatrixInt of 10 rows x 7 cols */
  jlong m = NAT(createRange)(env, NULL, dev, 0, 0, 10, 7);
  Arr* r = arr(70, 8);
  Arr* c = arr(70, 4);
  Arr* mv = arr(70, 4);
  for (int i = 0; i < 70; ++i) {
    ((jlong*)r->data)[i] = i / 7;
    ((jint*)c->data)[i] = i % 7;
    ((jint*)mv->data)[i] = 3 * i - 100;
  }
  NAT(await)(env, NULL, m, NAT(matPushI)(env, NULL, m, r, c, mv, 0));
  Arr* mo = arr(70, 4);
  NAT(matPullI)(env, NULL, m, r, c, mo);
  CHECK(!memcmp(mo->data, mv->data, 280), "matrix element pull");
  Arr* rows = arr(10, 8);
  for (int i = 0; i < 10; ++i) ((jlong*)rows->data)[i] = i;
  Arr* ro = arr(70, 4);
  NAT(matPullRowsI)(env, NULL, m, rows, ro);
  CHECK(!memcmp(ro->data, mv->data, 280) && !pending[0], "matrix row pull (flattened)");
  const jlong pr = NAT(pullAsync)(env, NULL, m, 2, rows, NULL);
  const jlong pe = NAT(pullAsync)(env, NULL, m, 1, r, c);
  Arr* ro2 = arr(70, 4);
  Arr* mo2 = arr(70, 4);
  NAT(pullFinishI)(env, NULL, pr, ro2);
  NAT(pullFinishI)(env, NULL, pe, mo2);
  CHECK(!pending[0] && !memcmp(ro2->data, mv->data, 280) && !memcmp(mo2->data, mv->data, 280),
        "async matrix row and element pulls");
  Arr* cs = arr(69, 4);
  NAT(matPushI)(env, NULL, m, r, cs, mv, 0);
  CHECK(took("java/lang/ArrayIndexOutOfBoundsException"), "short cols");
  NAT(destroy)(env, NULL, m);
  for (int size = 4000; size <= 10000; size += 2000) {  /* Gen.range("size")(4000, 10000, 2000) */
    matrix_benchmark(dev, 0, size);
    matrix_benchmark(dev, 1, size);
  }
  if (failures) return 1;
  printf("ok\n");
  return 0;
}
