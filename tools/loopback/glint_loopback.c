/*
 * glint_loopback.c -- BASELINE.json configs[0] over loopback TCP: 1 client + S parameter servers,
 * a Double vector of N keys range-partitioned over the servers, a dense push of keys 0..N-1 with
 * java.util.Random(42).nextDouble() values in messages of <= M records, then a pull of every key
 * and an exact check. It restates the message flow of the reference's Akka path:
 *
 *   client  GranularBigVector.push (src/main/scala/glint/models/client/granular/GranularBigVector.scala:72-81)
 *           slices the keys into <= M-record chunks; AsyncBigVector.push (.../async/AsyncBigVector.scala:96-121)
 *           groups each chunk by partition (RangePartitioner.partition, RangePartitioner.scala:27-43);
 *           PushFSM (.../async/PushFSM.scala:55-141) runs the exactly-once protocol per message:
 *             GetUniqueID -> UniqueID(id); PushVectorDouble(id, keys, values);
 *             AcknowledgeReceipt(id) -> AcknowledgeReceipt(id) | NotAcknowledgeReceipt(id) (resend);
 *             Forget(id) -> Forget(id)
 *   server  PartialVectorDouble.receive (src/main/scala/glint/models/server/PartialVectorDouble.scala:17-23):
 *           push -> update(keys, values); updateFinished(id); pull -> ResponseDouble(get(keys));
 *           PushLogic.handleLogic (src/main/scala/glint/models/server/PushLogic.scala:40-66)
 *
 * Push and pull payloads are the exact RequestSerializer / ResponseSerializer byte images
 * (RequestSerializer.scala:150-173, ResponseSerializer.scala:45-61); the logic messages, which Akka
 * serialises with Java serialisation, are 5-byte frames here. Every frame is [u32 length][payload].
 * Each client connection runs its protocol synchronously (one message in flight per server).
 *
 * The server's shard is a backend loaded at run time:
 *   --backend oracle --lib oracle/build/libglint_oracle.so  the CPU restatement of the server loop
 *            (deserialise into arrays as FastPrimitiveDeserializer does, then the scalar update):
 *            the CPU baseline, run only from bench.py's cpu_baseline leg;
 *   --backend gpu --lib glint_amd/lib/libglint_gpu.so       an HBM shard fed the raw wire image
 *            through glint_push_wire / glint_pull_wire (include/glint_gpu.h): the drop-in, end to end.
 *
 * Output: one JSON line.
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <dlfcn.h>
#include <errno.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

enum {
  W_PULL_VECTOR = 0x02, W_PUSH_VEC_D = 0x07, W_RESP_D = 0x10, /* SerializationConstants.scala:24-38 */
  L_GET_UID = 0x20, L_UID = 0x21, L_ACK = 0x22, L_NACK = 0x23, L_FORGET = 0x24, L_STOP = 0x7F
};

static void die(const char* what) {
  fprintf(stderr, "glint_loopback: %s: %s\n", what, strerror(errno));
  exit(2);
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* ---- framing ---------------------------------------------------------------------------------- */
static void write_all(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n) {
    ssize_t w = send(fd, c, n, MSG_NOSIGNAL);
    if (w <= 0) { if (w < 0 && errno == EINTR) continue; die("send"); }
    c += w;
    n -= (size_t)w;
  }
}
static int read_all(int fd, void* p, size_t n) {
  char* c = (char*)p;
  while (n) {
    ssize_t r = recv(fd, c, n, 0);
    if (r == 0) return 0;
    if (r < 0) { if (errno == EINTR) continue; die("recv"); }
    c += r;
    n -= (size_t)r;
  }
  return 1;
}
static void send_frame(int fd, const uint8_t* payload, uint32_t len) {
  write_all(fd, &len, 4);
  write_all(fd, payload, len);
}
/* returns payload length (0 on EOF); *buf grows as needed */
static uint32_t recv_frame(int fd, uint8_t** buf, size_t* cap) {
  uint32_t len;
  if (!read_all(fd, &len, 4)) return 0;
  if (len > *cap) {
    *cap = len;
    *buf = (uint8_t*)realloc(*buf, *cap);
    if (!*buf) die("realloc");
  }
  if (!read_all(fd, *buf, len)) return 0;
  return len;
}
static void send_logic(int fd, uint8_t type, int32_t id) {
  uint8_t m[5];
  m[0] = type;
  memcpy(m + 1, &id, 4);
  send_frame(fd, m, 5);
}

/* ---- backends ----------------------------------------------------------------------------------- */
typedef struct {
  int gpu;
  /* oracle (CPU restatement) */
  struct { int32_t kind; int32_t pad; int64_t start, end; int32_t cidx, cparts; int64_t ckeys; } opart;
  int64_t (*o_update)(const void*, int, void*, int32_t, const int64_t*, const void*, int64_t);
  int64_t (*o_get)(const void*, int, const void*, int32_t, const int64_t*, void*, int64_t);
  double* data;
  int32_t size;
  /* gpu */
  void* shard;
  int (*g_create)(int, int, int64_t, int64_t, int32_t, void**);
  int (*g_push_wire)(void*, const uint8_t*, size_t, int32_t*, int);
  int (*g_pull_wire)(void*, const uint8_t*, size_t, uint8_t*, size_t, size_t*);
  int (*g_destroy)(void*);
} backend;

static void* dl;
static int use_gpu;
static int gpu_device;

static void backend_open(const char* kind, const char* path) {
  dl = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!dl) { fprintf(stderr, "glint_loopback: dlopen %s: %s\n", path, dlerror()); exit(2); }
  use_gpu = strcmp(kind, "gpu") == 0;
}

static void backend_init(backend* b, int64_t start, int64_t end) {
  memset(b, 0, sizeof(*b));
  b->gpu = use_gpu;
  if (b->gpu) {
    *(void**)&b->g_create = dlsym(dl, "glint_shard_create");
    *(void**)&b->g_push_wire = dlsym(dl, "glint_push_wire");
    *(void**)&b->g_pull_wire = dlsym(dl, "glint_pull_wire");
    *(void**)&b->g_destroy = dlsym(dl, "glint_shard_destroy");
    if (!b->g_create || !b->g_push_wire || !b->g_pull_wire || !b->g_destroy) die("dlsym glint_*");
    int rc = b->g_create(gpu_device, 3 /* GLINT_F64 */, start, end, 0, &b->shard);
    if (rc) { fprintf(stderr, "glint_loopback: glint_shard_create failed (%d)\n", rc); exit(3); }
    /* actor start-up (preStart): one push of +0.0 and one pull, so the first timed message does not
     * pay the HIP runtime's lazy code-object load; x + 0.0 leaves every (zeroed) element unchanged */
    if (end > start) {
      uint8_t w[25] = {W_PUSH_VEC_D, 1, 0, 0, 0, 0, 0, 0, 0};
      const double zero = 0.0;
      memcpy(w + 9, &start, 8);
      memcpy(w + 17, &zero, 8);
      int32_t id;
      uint8_t q[13] = {W_PULL_VECTOR, 1, 0, 0, 0};
      memcpy(q + 5, &start, 8);
      uint8_t r[13];
      size_t rl;
      if (b->g_push_wire(b->shard, w, sizeof(w), &id, 0) || b->g_pull_wire(b->shard, q, sizeof(q), r, sizeof(r), &rl))
        die("warm-up");
    }
  } else {
    *(void**)&b->o_update = dlsym(dl, "oracle_vec_update");
    *(void**)&b->o_get = dlsym(dl, "oracle_vec_get");
    if (!b->o_update || !b->o_get) die("dlsym oracle_*");
    b->opart.kind = 0;
    b->opart.start = start;
    b->opart.end = end;
    b->size = (int32_t)(end - start); /* RangePartition.size, RangePartition.scala:24 */
    b->data = (double*)calloc((size_t)(b->size > 0 ? b->size : 1), 8); /* new Array[Double](size) */
  }
}

/* a PushVectorDouble image: [0x07][n:i32][id:i32][keys i64 x n][values f64 x n] */
static int backend_push(backend* b, const uint8_t* msg, uint32_t len, int32_t* id) {
  if (b->gpu) return b->g_push_wire(b->shard, msg, len, id, 0);
  int32_t n;
  memcpy(&n, msg + 1, 4);
  memcpy(id, msg + 5, 4);
  /* FastPrimitiveDeserializer.readArrayLong/readArrayDouble: copy out of the frame into arrays */
  int64_t* keys = (int64_t*)malloc((size_t)n * 8 + 8);
  double* vals = (double*)malloc((size_t)n * 8 + 8);
  memcpy(keys, msg + 9, (size_t)n * 8);
  memcpy(vals, msg + 9 + (size_t)n * 8, (size_t)n * 8);
  const int64_t bad = b->o_update(&b->opart, 3, b->data, b->size, keys, vals, n);
  free(keys);
  free(vals);
  return bad >= 0 ? 1 : 0;
}

/* a PullVector image [0x02][n][keys] -> a ResponseDouble image [0x10][n][values] */
static int backend_pull(backend* b, const uint8_t* msg, uint32_t len, uint8_t* out, size_t cap, size_t* out_len) {
  if (b->gpu) return b->g_pull_wire(b->shard, msg, len, out, cap, out_len);
  int32_t n;
  memcpy(&n, msg + 1, 4);
  int64_t* keys = (int64_t*)malloc((size_t)n * 8 + 8);
  memcpy(keys, msg + 5, (size_t)n * 8);
  const int64_t bad = b->o_get(&b->opart, 3, b->data, b->size, keys, out + 5, n);
  free(keys);
  out[0] = W_RESP_D;
  memcpy(out + 1, &n, 4);
  *out_len = 5 + (size_t)n * 8;
  return bad >= 0 ? 1 : 0;
}

static void backend_close(backend* b) {
  if (b->gpu) b->g_destroy(b->shard);
  else free(b->data);
}

/* ---- server: PartialVectorDouble.receive + PushLogic ------------------------------------------- */
typedef struct {
  int64_t start, end;
  int listen_fd;
  int port;
  int64_t records_applied;
  int errors;
} server_arg;

static pthread_barrier_t servers_ready;

static void* server_main(void* p) {
  server_arg* a = (server_arg*)p;
  backend b;
  backend_init(&b, a->start, a->end);
  pthread_barrier_wait(&servers_ready); /* the client's clock starts once every shard exists */
  int fd = accept(a->listen_fd, NULL, NULL);
  if (fd < 0) die("accept");
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  int32_t uid = 0;                       /* PushLogic.uid */
  size_t rcap = 1 << 16;                 /* PushLogic.receipt, indexed by id */
  uint8_t* receipt = (uint8_t*)calloc(rcap, 1);
  uint8_t* buf = NULL;
  size_t cap = 0;
  size_t ocap = 1 << 20;
  uint8_t* out = (uint8_t*)malloc(ocap);
  for (;;) {
    const uint32_t len = recv_frame(fd, &buf, &cap);
    if (len == 0) break;
    const uint8_t t = buf[0];
    int32_t id = 0;
    if (len >= 5 && t >= L_GET_UID && t <= L_FORGET) memcpy(&id, buf + 1, 4);
    if (t == W_PUSH_VEC_D) {
      int32_t mid = 0;
      if (backend_push(&b, buf, len, &mid) != 0) a->errors++;
      int32_t n;
      memcpy(&n, buf + 1, 4);
      a->records_applied += n;
      if ((size_t)mid >= rcap) {                         /* updateFinished(id) */
        size_t nc = rcap;
        while ((size_t)mid >= nc) nc *= 2;
        receipt = (uint8_t*)realloc(receipt, nc);
        memset(receipt + rcap, 0, nc - rcap);
        rcap = nc;
      }
      receipt[mid] = 1;
    } else if (t == W_PULL_VECTOR) {
      int32_t n;
      memcpy(&n, buf + 1, 4);
      const size_t need = 5 + (size_t)n * 8;
      if (need > ocap) { ocap = need; out = (uint8_t*)realloc(out, ocap); }
      size_t olen = 0;
      if (backend_pull(&b, buf, len, out, ocap, &olen) != 0) a->errors++;
      send_frame(fd, out, (uint32_t)olen);
    } else if (t == L_GET_UID) {
      send_logic(fd, L_UID, ++uid);                      /* sender ! UniqueID(nextId()) */
    } else if (t == L_ACK) {
      const int got = (size_t)id < rcap && receipt[id];
      send_logic(fd, got ? L_ACK : L_NACK, id);
    } else if (t == L_FORGET) {
      if ((size_t)id < rcap) receipt[id] = 0;
      send_logic(fd, L_FORGET, id);
    } else if (t == L_STOP) {
      break;
    } else {
      a->errors++;
    }
  }
  close(fd);
  free(buf);
  free(out);
  free(receipt);
  backend_close(&b);
  return NULL;
}

/* ---- client ------------------------------------------------------------------------------------ */
/* java.util.Random(42).nextDouble() -- the values of GranularBigVectorSpec.scala:14-35 */
typedef struct { uint64_t seed; } jrandom;
static void jr_init(jrandom* r, int64_t s) { r->seed = ((uint64_t)s ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1); }
static int32_t jr_next(jrandom* r, int bits) {
  r->seed = (r->seed * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
  return (int32_t)(int64_t)(r->seed >> (48 - bits));
}
static double jr_double(jrandom* r) {
  return (double)(((int64_t)jr_next(r, 26) << 27) + jr_next(r, 27)) * (1.0 / (double)(1LL << 53));
}

typedef struct {
  int fd;
  int part;
  const int64_t* keys;
  const double* vals;
  const int32_t* owner;
  int64_t nkeys;
  int msg;
  int64_t messages, resends;
  double* pulled;
  int mode; /* 0 push, 1 pull */
} client_arg;

static void* client_main(void* p) {
  client_arg* c = (client_arg*)p;
  uint8_t* buf = NULL;
  size_t cap = 0;
  uint8_t* m = (uint8_t*)malloc(9 + (size_t)c->msg * 16);
  int64_t* idx = (int64_t*)malloc((size_t)c->msg * 8);
  /* GranularBigVector: <= msg-record slices of the caller's keys; AsyncBigVector groups each slice
   * by partition, one message per partition -- this thread sends partition `part`'s messages */
  for (int64_t i = 0; i < c->nkeys; i += c->msg) {
    const int64_t end = i + c->msg < c->nkeys ? i + c->msg : c->nkeys;
    int32_t n = 0;
    for (int64_t j = i; j < end; ++j)
      if (c->owner[j] == c->part) idx[n++] = j;
    if (n == 0) continue;
    if (c->mode == 0) {
      send_logic(c->fd, L_GET_UID, 0);                       /* prepare(): GetUniqueID */
      uint32_t len = recv_frame(c->fd, &buf, &cap);
      int32_t id;
      if (len != 5 || buf[0] != L_UID) die("protocol: UniqueID");
      memcpy(&id, buf + 1, 4);
      m[0] = W_PUSH_VEC_D;                                   /* RequestSerializer.scala:165-173 */
      memcpy(m + 1, &n, 4);
      memcpy(m + 5, &id, 4);
      for (int32_t q = 0; q < n; ++q) {
        memcpy(m + 9 + (size_t)q * 8, &c->keys[idx[q]], 8);
        memcpy(m + 9 + (size_t)n * 8 + (size_t)q * 8, &c->vals[idx[q]], 8);
      }
      for (;;) {
        send_frame(c->fd, m, 9 + (uint32_t)n * 16);          /* execute(): actorRef ! message(id) */
        c->messages++;
        send_logic(c->fd, L_ACK, id);                        /* acknowledge() */
        len = recv_frame(c->fd, &buf, &cap);
        if (len != 5) die("protocol: ack");
        if (buf[0] == L_ACK) break;
        c->resends++;                                        /* NotAcknowledgeReceipt: execute() again */
      }
      send_logic(c->fd, L_FORGET, id);                       /* forget() */
      len = recv_frame(c->fd, &buf, &cap);
      if (len != 5 || buf[0] != L_FORGET) die("protocol: forget");
    } else {
      m[0] = W_PULL_VECTOR;                                  /* RequestSerializer.scala:150-155 */
      memcpy(m + 1, &n, 4);
      for (int32_t q = 0; q < n; ++q) memcpy(m + 5 + (size_t)q * 8, &c->keys[idx[q]], 8);
      send_frame(c->fd, m, 5 + (uint32_t)n * 8);
      c->messages++;
      const uint32_t len = recv_frame(c->fd, &buf, &cap);
      int32_t rn;
      if (len < 5 || buf[0] != W_RESP_D) die("protocol: response");
      memcpy(&rn, buf + 1, 4);
      if (rn != n || len != 5 + (uint32_t)n * 8) die("protocol: response size");
      for (int32_t q = 0; q < n; ++q) memcpy(&c->pulled[idx[q]], buf + 5 + (size_t)q * 8, 8);
    }
  }
  free(m);
  free(idx);
  free(buf);
  return NULL;
}

int main(int argc, char** argv) {
  const char* kind = "oracle";
  const char* lib = NULL;
  int S = 2, msg = 1000;
  int64_t N = 1000000;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--backend") && i + 1 < argc) kind = argv[++i];
    else if (!strcmp(argv[i], "--lib") && i + 1 < argc) lib = argv[++i];
    else if (!strcmp(argv[i], "--servers") && i + 1 < argc) S = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--keys") && i + 1 < argc) N = atoll(argv[++i]);
    else if (!strcmp(argv[i], "--msg") && i + 1 < argc) msg = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--device") && i + 1 < argc) gpu_device = atoi(argv[++i]);
    else { fprintf(stderr, "usage: %s --backend oracle|gpu --lib PATH [--servers S] [--keys N] [--msg M] [--device D]\n", argv[0]); return 2; }
  }
  if (!lib || S <= 0 || N <= 0 || msg <= 0) { fprintf(stderr, "glint_loopback: bad arguments\n"); return 2; }
  backend_open(kind, lib);

  /* RangePartitioner.apply(S, N) (RangePartitioner.scala:62-84) and partition() (:27-43) */
  const int32_t n_large = (int32_t)(N % S), n_small = S - n_large;
  const int32_t q = (int32_t)((N - N % S) / S);
  int64_t* starts = (int64_t*)malloc(sizeof(int64_t) * S);
  int64_t* ends = (int64_t*)malloc(sizeof(int64_t) * S);
  {
    int64_t start = 0, end = q;
    for (int i = 0; i < S; ++i) {
      if (i < n_small) { starts[i] = start; ends[i] = end; start += q; end += q; }
      else { end += 1; starts[i] = start; ends[i] = end; start += q + 1; end += q; }
    }
  }
  const int64_t small_keys = (int64_t)n_small * q;
  int64_t* keys = (int64_t*)malloc((size_t)N * 8);
  double* vals = (double*)malloc((size_t)N * 8);
  double* pulled = (double*)calloc((size_t)N, 8);
  int32_t* owner = (int32_t*)malloc((size_t)N * 4);
  jrandom jr;
  jr_init(&jr, 42);
  for (int64_t k = 0; k < N; ++k) {
    keys[k] = k;
    vals[k] = jr_double(&jr);
    owner[k] = k < small_keys ? (int32_t)(k / q) : (int32_t)(n_small + (k - small_keys) / ((int64_t)q + 1));
  }

  server_arg* sa = (server_arg*)calloc((size_t)S, sizeof(server_arg));
  pthread_t* st = (pthread_t*)malloc(sizeof(pthread_t) * S);
  pthread_barrier_init(&servers_ready, NULL, (unsigned)S + 1);
  for (int i = 0; i < S; ++i) {
    sa[i].start = starts[i];
    sa[i].end = ends[i];
    sa[i].listen_fd = socket(AF_INET, SOCK_STREAM, 0);
    if (sa[i].listen_fd < 0) die("socket");
    struct sockaddr_in ad;
    memset(&ad, 0, sizeof(ad));
    ad.sin_family = AF_INET;
    ad.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    ad.sin_port = 0;
    if (bind(sa[i].listen_fd, (struct sockaddr*)&ad, sizeof(ad)) < 0) die("bind");
    if (listen(sa[i].listen_fd, 1) < 0) die("listen");
    socklen_t sl = sizeof(ad);
    getsockname(sa[i].listen_fd, (struct sockaddr*)&ad, &sl);
    sa[i].port = ntohs(ad.sin_port);
    pthread_create(&st[i], NULL, server_main, &sa[i]);
  }
  pthread_barrier_wait(&servers_ready);
  client_arg* ca = (client_arg*)calloc((size_t)S, sizeof(client_arg));
  for (int i = 0; i < S; ++i) {
    ca[i].fd = socket(AF_INET, SOCK_STREAM, 0);
    struct sockaddr_in ad;
    memset(&ad, 0, sizeof(ad));
    ad.sin_family = AF_INET;
    ad.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    ad.sin_port = htons((uint16_t)sa[i].port);
    if (connect(ca[i].fd, (struct sockaddr*)&ad, sizeof(ad)) < 0) die("connect");
    int one = 1;
    setsockopt(ca[i].fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    ca[i].part = i;
    ca[i].keys = keys;
    ca[i].vals = vals;
    ca[i].owner = owner;
    ca[i].nkeys = N;
    ca[i].msg = msg;
    ca[i].pulled = pulled;
  }
  pthread_t* ct = (pthread_t*)malloc(sizeof(pthread_t) * S);
  double t[3];
  int64_t msgs[2] = {0, 0};
  for (int mode = 0; mode < 2; ++mode) {
    t[mode] = now_s();
    for (int i = 0; i < S; ++i) {
      ca[i].mode = mode;
      ca[i].messages = 0;
      pthread_create(&ct[i], NULL, client_main, &ca[i]);
    }
    for (int i = 0; i < S; ++i) {
      pthread_join(ct[i], NULL);
      msgs[mode] += ca[i].messages;
    }
  }
  t[2] = now_s();
  for (int i = 0; i < S; ++i) {
    uint8_t stop[5] = {L_STOP, 0, 0, 0, 0};
    send_frame(ca[i].fd, stop, 5);
  }
  int errors = 0;
  int64_t resends = 0;
  for (int i = 0; i < S; ++i) {
    pthread_join(st[i], NULL);
    errors += sa[i].errors;
    resends += ca[i].resends;
    close(ca[i].fd);
    close(sa[i].listen_fd);
  }
  /* GranularBigVectorSpec: the pulled values equal the pushed ones exactly (one add onto 0.0) */
  int ok = errors == 0;
  for (int64_t k = 0; k < N && ok; ++k) ok = memcmp(&pulled[k], &vals[k], 8) == 0;
  const double tp = t[1] - t[0], tl = t[2] - t[1];
  printf("{\"backend\": \"%s\", \"servers\": %d, \"keys\": %lld, \"max_records_per_message\": %d, "
         "\"push_messages\": %lld, \"pull_messages\": %lld, \"resends\": %lld, \"push_s\": %.6f, \"pull_s\": %.6f, "
         "\"push_records_per_s\": %.1f, \"pull_records_per_s\": %.1f, \"push_payload_MBps\": %.2f, "
         "\"pull_payload_MBps\": %.2f, \"first_values\": [%.17g, %.17g, %.17g], \"check\": %s}\n",
         kind, S, (long long)N, msg, (long long)msgs[0], (long long)msgs[1], (long long)resends, tp, tl,
         (double)N / tp, (double)N / tl, 16.0 * (double)N / tp / 1e6, 16.0 * (double)N / tl / 1e6,
         vals[0], N > 1 ? vals[1] : 0.0, N > 2 ? vals[2] : 0.0, ok ? "true" : "false");
  free(keys); free(vals); free(pulled); free(owner); free(sa); free(st); free(ca); free(ct);
  free(starts); free(ends);
  return ok ? 0 : 1;
}
