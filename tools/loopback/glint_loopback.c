/*
 * glint_loopback.c -- Glint's push/pull message flow over loopback TCP, C clients x S parameter
 * servers, with the server's shard as a pluggable backend. It restates the reference's Akka path:
 *
 *   client  GranularBigVector.push/pull (src/main/scala/glint/models/client/granular/
 *           GranularBigVector.scala:26-50) slices the caller's keys into <= M-record chunks and issues
 *           every chunk at once (one future each); AsyncBigVector.push/pull (.../async/
 *           AsyncBigVector.scala:49-121) groups each chunk by partition (RangePartitioner.partition,
 *           RangePartitioner.scala:27-43) and sends one message per partition. Each push runs the
 *           exactly-once PushFSM (.../async/PushFSM.scala:55-141):
 *             GetUniqueID -> UniqueID(id); PushVector*(id, keys, values); AcknowledgeReceipt(id) ->
 *             AcknowledgeReceipt(id) | NotAcknowledgeReceipt(id) (resend); Forget(id) -> Forget(id)
 *           Here every (client, server) connection keeps up to W messages in flight (-window).
 *   server  PartialVector{Double,Long}.receive (src/main/scala/glint/models/server/
 *           PartialVectorDouble.scala:17-23) -- one message at a time per server, whatever connection
 *           it came from -- with PushLogic (PushLogic.scala:40-66) for the ids and receipts.
 *
 * Push and pull payloads are the exact RequestSerializer / ResponseSerializer byte images
 * (RequestSerializer.scala:150-173, ResponseSerializer.scala:45-61); the logic messages, which Akka
 * serialises with Java serialisation, are 5-byte frames here. Every frame is [u32 length][payload].
 *
 * Backends (loaded at run time):
 *   --backend oracle --lib oracle/build/libglint_oracle.so   the CPU restatement of the server loop:
 *            deserialise into arrays as FastPrimitiveDeserializer does, then the scalar update
 *            (the CPU baseline, run only from bench.py's cpu_baseline leg and the tests);
 *   --backend gpu --lib glint_amd/lib/libglint_gpu.so        an HBM shard per server fed the raw wire
 *            images: pushes are enqueued (glint_push_wire_async) and the server waits for them
 *            (glint_shard_wait) only when it has drained the messages that have arrived and owes an
 *            AcknowledgeReceipt or a Response -- what PushLogic needs, one wait per burst; pulls are
 *            enqueued the same way (glint_pull_wire_async, ordered after the enqueued pushes) and
 *            their Responses are sent, in request order, after that wait.
 *
 * Workloads (--pattern): dense -- client c pushes then pulls its own contiguous key range
 * (BASELINE configs[0] at C = 1: GranularBigVectorSpec's 1M keys with java.util.Random(42)
 * values; configs[3] 4a at C = 64: each client owns N / C keys); uniform -- every client pushes R
 * uniform keys over the whole space and pulls them back (configs[3] 4b). Checks: dense, every pulled
 * value equals the pushed one bit for bit; uniform, the pulled sums equal the sequential sum over all
 * clients' records (Long: bit-exact; Double: within 1e-9 of the sum of magnitudes, since concurrent
 * clients' messages reach a server in no fixed order, as with Akka).
 *
 * Client bucketing (--bucket), the mapPartitions step (AsyncBigVector.scala:96-98) in front of the
 * links, done once per client batch for the push and again for the pull, and timed on its own:
 *   groupby  the reference's algorithm restated: per GranularBigVector slice, one pass over its
 *            records appending each index to its partition's list (keys.indices.groupBy(partition));
 *   device   offloaded: the client's whole batch (in pinned memory) routed on the GPU by
 *            glint_route_gather_dev (a stable counting sort by partition, no synchronisation inside), the
 *            order, counts and status word read back with the one wait, then each partition's ordered
 *            index list is cut at the slice boundaries. Each client holds its device buffers, pinned
 *            memory and its own stream from before the timed region. Both give the same messages, record
 *            for record.
 *
 * Output: one JSON line.
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <dlfcn.h>
#include <errno.h>
#include <math.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/ioctl.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

enum {
  W_PULL_VECTOR = 0x02, W_PUSH_VEC_D = 0x07, W_PUSH_VEC_L = 0x0A, /* SerializationConstants.scala:24-38 */
  W_RESP_D = 0x10, W_RESP_L = 0x13,
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

/* an output buffer of frames, sent with one write */
typedef struct { uint8_t* p; size_t len, cap; } obuf;
static void ob_put(obuf* o, const void* d, size_t n) {
  if (o->len + n > o->cap) {
    o->cap = (o->len + n) * 2 + 4096;
    o->p = (uint8_t*)realloc(o->p, o->cap);
    if (!o->p) die("realloc");
  }
  memcpy(o->p + o->len, d, n);
  o->len += n;
}
static void ob_frame(obuf* o, const void* payload, uint32_t len) { ob_put(o, &len, 4); ob_put(o, payload, len); }
static void ob_logic(obuf* o, uint8_t type, int32_t id) {
  uint8_t m[5];
  m[0] = type;
  memcpy(m + 1, &id, 4);
  ob_frame(o, m, 5);
}
static void ob_flush(obuf* o, int fd) {
  if (o->len) write_all(fd, o->p, o->len);
  o->len = 0;
}

static void tune_socket(int fd) {
  int one = 1, big = 8 << 20;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &big, sizeof(big));
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &big, sizeof(big));
}

/* ---- backends ----------------------------------------------------------------------------------- */
static void* dl;
static int use_gpu;
/* --answers direct (the default when the library has glint_host_alloc): each connection answers
 * pulls from a pinned, device-mapped arena, so the GPU writes the answers straight into the response
 * images (no copy out of the ring slot); --answers copy: malloc'd response buffers */
static int answers_direct = -1;
static size_t arena_bytes; /* per connection: W responses of up to M records */
static int (*g_host_alloc)(size_t, void**);
static int (*g_host_free)(void*);
static int gpu_device;
static int dtype_long; /* 0: Double values, 1: Long values */

typedef struct {
  /* oracle (CPU restatement) */
  struct { int32_t kind; int32_t pad; int64_t start, end; int32_t cidx, cparts; int64_t ckeys; } opart;
  int64_t (*o_update)(const void*, int, void*, int32_t, const int64_t*, const void*, int64_t);
  int64_t (*o_get)(const void*, int, const void*, int32_t, const int64_t*, void*, int64_t);
  void* data;
  int32_t size;
  /* gpu */
  void* shard;
  int (*g_create)(int, int, int64_t, int64_t, int32_t, void**);
  int (*g_push_async)(void*, const uint8_t*, size_t, int32_t*, int, uint64_t*);
  int (*g_wait)(void*, uint64_t, int64_t*);
  int (*g_pull_wire)(void*, const uint8_t*, size_t, uint8_t*, size_t, size_t*);
  int (*g_pull_async)(void*, const uint8_t*, size_t, uint8_t*, size_t, size_t*, uint64_t*);
  int (*g_destroy)(void*);
} backend;

static void backend_open(const char* kind, const char* path) {
  dl = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!dl) { fprintf(stderr, "glint_loopback: dlopen %s: %s\n", path, dlerror()); exit(2); }
  use_gpu = strcmp(kind, "gpu") == 0;
}

static int value_code(void) { return dtype_long ? 1 /* GLINT_I64 / O_I64 */ : 3 /* F64 */; }

static void backend_init(backend* b, int64_t start, int64_t end) {
  memset(b, 0, sizeof(*b));
  if (use_gpu) {
    *(void**)&b->g_create = dlsym(dl, "glint_shard_create");
    *(void**)&b->g_push_async = dlsym(dl, "glint_push_wire_async");
    *(void**)&b->g_wait = dlsym(dl, "glint_shard_wait");
    *(void**)&b->g_pull_wire = dlsym(dl, "glint_pull_wire");
    *(void**)&b->g_pull_async = dlsym(dl, "glint_pull_wire_async");
    *(void**)&b->g_destroy = dlsym(dl, "glint_shard_destroy");
    if (!b->g_create || !b->g_push_async || !b->g_wait || !b->g_pull_wire || !b->g_pull_async || !b->g_destroy)
      die("dlsym glint_*");
    int rc = b->g_create(gpu_device, value_code(), start, end, 0, &b->shard);
    if (rc) { fprintf(stderr, "glint_loopback: glint_shard_create failed (%d)\n", rc); exit(3); }
    /* actor start-up (preStart): one push of +0 and one pull, so the first timed message does not pay
     * the HIP runtime's lazy code-object load; x + 0 leaves every (zeroed) element unchanged */
    if (end > start) {
      uint8_t w[25] = {dtype_long ? W_PUSH_VEC_L : W_PUSH_VEC_D, 1, 0, 0, 0, 0, 0, 0, 0};
      memcpy(w + 9, &start, 8);
      memset(w + 17, 0, 8);
      int32_t id;
      uint64_t t;
      uint8_t q[13] = {W_PULL_VECTOR, 1, 0, 0, 0};
      memcpy(q + 5, &start, 8);
      uint8_t r[13];
      size_t rl;
      if (b->g_push_async(b->shard, w, sizeof(w), &id, 0, &t) || b->g_wait(b->shard, t, NULL) ||
          b->g_pull_wire(b->shard, q, sizeof(q), r, sizeof(r), &rl))
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
    b->data = calloc((size_t)(b->size > 0 ? b->size : 1), 8); /* new Array[V](size) */
  }
}

static void backend_close(backend* b) {
  if (use_gpu) b->g_destroy(b->shard);
  else free(b->data);
}

/* ---- server: PartialVector*.receive + PushLogic, one thread per client connection ---------------- */
typedef struct {
  int64_t start, end;
  int listen_fd, port;
  backend b;
  pthread_mutex_t mu; /* one message at a time per server (the actor) + PushLogic's state */
  int32_t uid;        /* PushLogic.uid */
  uint8_t* receipt;   /* PushLogic.receipt, indexed by id */
  size_t rcap;
  int errors;
  double cpu[8]; /* --cpu-stats: server thread CPU s in enqueue / update (push, pull), in waits (push,
                    pull), wall s in waits (push, pull) and in enqueue / update (push, pull) */
} server;

static void receipt_set(server* s, int32_t id, uint8_t v) {
  if ((size_t)id >= s->rcap) {
    size_t nc = s->rcap ? s->rcap : 1024;
    while ((size_t)id >= nc) nc *= 2;
    s->receipt = (uint8_t*)realloc(s->receipt, nc);
    memset(s->receipt + s->rcap, 0, nc - s->rcap);
    s->rcap = nc;
  }
  s->receipt[id] = v;
}
static int receipt_has(server* s, int32_t id) { return (size_t)id < s->rcap && s->receipt[id]; }

typedef struct {
  server* s;
  int fd;
} conn_arg;

/* Replies leave a connection in request order. A reply is either ready (its frame is in `out`), an
 * AcknowledgeReceipt of a push still on the GPU, or the Response of a pull still on the GPU; the
 * held ones are answered after one wait per drained burst. */
typedef struct {
  size_t end;      /* out[prev end .. end) is ready, then this reply */
  int32_t ack_id;  /* an AcknowledgeReceipt, or */
  uint8_t* resp;   /* a pull's Response frame (filled by the wait) */
  size_t resp_len;
  int owned;       /* resp was malloc'd (else it lies in the connection's arena) */
} hold;

/* --cpu-stats: the servers' thread CPU time around the backend calls (one clock read each side) */
static int cpu_stats;
static double tcpu(void) {
  struct timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}
static double pcpu(void) { /* the whole process: user + system */
  struct rusage ru;
  getrusage(RUSAGE_SELF, &ru);
  return (double)ru.ru_utime.tv_sec + 1e-6 * (double)ru.ru_utime.tv_usec + (double)ru.ru_stime.tv_sec +
         1e-6 * (double)ru.ru_stime.tv_usec;
}

static int readable_now(int fd) {
  int avail = 0;
  if (ioctl(fd, FIONREAD, &avail) < 0) return 0;
  return avail > 0;
}

/* --replies async: a connection's receive loop never waits for the GPU. It enqueues every push and
 * pull on the shard and hands each reply, in request order, to the connection's reply thread; that
 * thread takes whatever has queued up, waits ONCE for the highest ticket among it (tickets complete
 * in order), then writes the replies with one send (the actor equivalent: pipeTo from a completion
 * thread). --replies burst (the default): one blocking wait per drained burst, then the replies.
 * Measured on one box (profiles/r03/loopback_gpu_async.jsonl against loopback_gpu.jsonl): async loses
 * everywhere there are many connections (cfg4b push 48 -> 23 M, pull 108 -> 24-30 M records/s): a
 * reply thread per connection doubles the threads on the box's CPU share, and each waits on a
 * smaller batch. Kept as an option for the comparison. */
static int replies_async = 0;

enum { R_FRAME, R_ACK, R_RESP, R_STOP };
typedef struct {
  int kind;
  int32_t id;       /* R_ACK */
  uint64_t ticket;  /* R_ACK (0: not a push of this connection), R_RESP */
  uint8_t* buf;     /* R_FRAME / R_RESP payload (owned) */
  uint32_t len;
} rentry;
typedef struct {
  server* s;
  int fd;
  pthread_mutex_t mu;
  pthread_cond_t cv;
  rentry* q;
  size_t n, cap;
} rqueue;

static void rq_put(rqueue* r, rentry e) {
  pthread_mutex_lock(&r->mu);
  if (r->n == r->cap) {
    r->cap = r->cap ? 2 * r->cap : 256;
    r->q = (rentry*)realloc(r->q, r->cap * sizeof(rentry));
    if (!r->q) die("realloc");
  }
  r->q[r->n++] = e;
  pthread_cond_signal(&r->cv);
  pthread_mutex_unlock(&r->mu);
}
static void rq_frame_logic(rqueue* r, uint8_t type, int32_t id) {
  rentry e = {R_FRAME, 0, 0, (uint8_t*)malloc(5), 5};
  e.buf[0] = type;
  memcpy(e.buf + 1, &id, 4);
  rq_put(r, e);
}

static void* reply_main(void* p) {
  rqueue* r = (rqueue*)p;
  server* s = r->s;
  obuf out = {0};
  rentry* batch = NULL;
  size_t bcap = 0;
  for (int stop = 0; !stop;) {
    pthread_mutex_lock(&r->mu);
    while (r->n == 0) pthread_cond_wait(&r->cv, &r->mu);
    /* swap the queue out: the receive loop keeps appending to the (empty) other array */
    rentry* q = r->q;
    const size_t n = r->n, qcap = r->cap;
    r->q = batch;
    r->cap = bcap;
    r->n = 0;
    pthread_mutex_unlock(&r->mu);
    batch = q;
    bcap = qcap;
    uint64_t tmax = 0;
    for (size_t i = 0; i < n; ++i)
      if (batch[i].ticket > tmax) tmax = batch[i].ticket;
    const int rc = tmax ? s->b.g_wait(s->b.shard, tmax, NULL) : 0;
    pthread_mutex_lock(&s->mu);
    if (rc != 0) s->errors++;
    for (size_t i = 0; i < n; ++i) {
      rentry* e = &batch[i];
      if (e->kind == R_FRAME || e->kind == R_RESP) {
        ob_frame(&out, e->buf, e->len);
        free(e->buf);
      } else if (e->kind == R_ACK) {
        if (e->ticket && rc == 0) receipt_set(s, e->id, 1); /* updateFinished(id), once the push ran */
        ob_logic(&out, receipt_has(s, e->id) ? L_ACK : L_NACK, e->id);
      } else {
        stop = 1;
      }
    }
    pthread_mutex_unlock(&s->mu);
    ob_flush(&out, r->fd);
  }
  free(out.p);
  free(batch);
  return NULL;
}

static void* conn_main_async(conn_arg* a) {
  server* s = a->s;
  const int fd = a->fd;
  rqueue r;
  memset(&r, 0, sizeof(r));
  r.s = s;
  r.fd = fd;
  pthread_mutex_init(&r.mu, NULL);
  pthread_cond_init(&r.cv, NULL);
  pthread_t th;
  if (pthread_create(&th, NULL, reply_main, &r)) die("pthread_create");
  uint8_t* buf = NULL;
  size_t cap = 0;
  struct { int32_t id; uint64_t ticket; }* pend = NULL; /* this connection's pushes, not acked yet */
  size_t npend = 0, pcap = 0;
  for (;;) {
    const uint32_t len = recv_frame(fd, &buf, &cap);
    if (len == 0) break;
    const uint8_t t = buf[0];
    int32_t id = 0;
    if (len >= 5 && t >= L_GET_UID && t <= L_FORGET) memcpy(&id, buf + 1, 4);
    if (t == W_PUSH_VEC_D || t == W_PUSH_VEC_L) {
      int32_t mid = 0;
      uint64_t ticket = 0;
      if (s->b.g_push_async(s->b.shard, buf, len, &mid, 0, &ticket) != 0) {
        pthread_mutex_lock(&s->mu);
        s->errors++;
        pthread_mutex_unlock(&s->mu);
        continue; /* rejected: never updateFinished, the ack becomes a NotAcknowledgeReceipt */
      }
      if (npend == pcap) {
        pcap = pcap ? 2 * pcap : 64;
        pend = realloc(pend, pcap * sizeof(*pend));
        if (!pend) die("realloc");
      }
      pend[npend].id = mid;
      pend[npend].ticket = ticket;
      ++npend;
    } else if (t == W_PULL_VECTOR) {
      int32_t n;
      memcpy(&n, buf + 1, 4);
      const size_t need = 5 + (size_t)n * 8;
      rentry e = {R_RESP, 0, 0, (uint8_t*)malloc(need), 0};
      size_t olen = 0;
      if (s->b.g_pull_async(s->b.shard, buf, len, e.buf, need, &olen, &e.ticket) != 0) {
        pthread_mutex_lock(&s->mu);
        s->errors++;
        pthread_mutex_unlock(&s->mu);
      }
      e.len = (uint32_t)olen;
      rq_put(&r, e);
    } else if (t == L_GET_UID) {
      pthread_mutex_lock(&s->mu);
      const int32_t u = ++s->uid; /* sender ! UniqueID(nextId()) */
      pthread_mutex_unlock(&s->mu);
      rq_frame_logic(&r, L_UID, u);
    } else if (t == L_ACK) {
      rentry e = {R_ACK, id, 0, NULL, 0};
      for (size_t i = 0; i < npend; ++i)
        if (pend[i].id == id) {
          e.ticket = pend[i].ticket;
          pend[i] = pend[--npend];
          break;
        }
      rq_put(&r, e);
    } else if (t == L_FORGET) {
      pthread_mutex_lock(&s->mu);
      if (receipt_has(s, id)) receipt_set(s, id, 0);
      pthread_mutex_unlock(&s->mu);
      rq_frame_logic(&r, L_FORGET, id);
    } else if (t == L_STOP) {
      break;
    } else {
      pthread_mutex_lock(&s->mu);
      s->errors++;
      pthread_mutex_unlock(&s->mu);
    }
  }
  rentry stop = {R_STOP, 0, 0, NULL, 0};
  rq_put(&r, stop);
  pthread_join(th, NULL);
  close(fd);
  free(buf);
  free(pend);
  free(r.q);
  pthread_mutex_destroy(&r.mu);
  pthread_cond_destroy(&r.cv);
  free(a);
  return NULL;
}

/* One connection's server-side state: the replies owed, in request order, and the GPU work enqueued
 * for it since its last settle. */
typedef struct {
  int fd;
  obuf out;
  uint8_t* resp; /* the oracle's response scratch */
  size_t rcap;
  int32_t* pending; /* ids of this connection's pushes enqueued on the GPU since the last settle */
  size_t npend, pcap;
  uint64_t last_ticket;
  hold* holds; /* held replies, in reply order */
  size_t nhold, hcap;
  int enqueued; /* GPU work enqueued since the last settle */
  double cs[8]; /* --cpu-stats, as server.cpu */
  int wmode;    /* the kind (0 push, 1 pull) of the work a wait covers */
  int dirty;    /* --server actor: owes replies (in the actor's settle list) */
  uint8_t* arena; /* --answers direct: the pinned response arena, reset after every settle */
  size_t aused;
} cstate;

/* connections whose server side is set up (arena allocated): the timed phases start only once all
 * are, so no pinned allocation overlaps them */
static int conns_ready;
static void cstate_arena(cstate* c) {
  if (use_gpu && answers_direct && arena_bytes && g_host_alloc((size_t)arena_bytes, (void**)&c->arena) != 0)
    c->arena = NULL;
  __atomic_add_fetch(&conns_ready, 1, __ATOMIC_RELEASE);
}

/* PartialVector*.receive + PushLogic for one message of connection c; returns 1 on L_STOP */
static int handle_msg(server* s, cstate* c, const uint8_t* buf, uint32_t len) {
  const uint8_t t = buf[0];
  int32_t id = 0;
  if (len >= 5 && t >= L_GET_UID && t <= L_FORGET) memcpy(&id, buf + 1, 4);
  const double c0 = cpu_stats ? tcpu() : 0.0, cw0 = cpu_stats ? now_s() : 0.0;
  int cmode = -1;
  if (t == W_PUSH_VEC_D || t == W_PUSH_VEC_L) {
    int32_t mid = 0;
    cmode = 0;
    c->wmode = 0;
    if (use_gpu) { /* enqueued: update runs on the GPU in arrival order; no reply */
      uint64_t ticket = 0;
      if (s->b.g_push_async(s->b.shard, buf, len, &mid, 0, &ticket) != 0) s->errors++;
      if (c->npend == c->pcap) {
        c->pcap = c->pcap ? 2 * c->pcap : 64;
        c->pending = (int32_t*)realloc(c->pending, c->pcap * 4);
      }
      c->pending[c->npend++] = mid;
      if (ticket > c->last_ticket) c->last_ticket = ticket;
      c->enqueued = 1;
    } else {
      int32_t n;
      memcpy(&n, buf + 1, 4);
      memcpy(&mid, buf + 5, 4);
      /* FastPrimitiveDeserializer.readArrayLong/readArray*: copy out of the frame into arrays */
      int64_t* keys = (int64_t*)malloc((size_t)n * 8 + 8);
      void* vals = malloc((size_t)n * 8 + 8);
      memcpy(keys, buf + 9, (size_t)n * 8);
      memcpy(vals, buf + 9 + (size_t)n * 8, (size_t)n * 8);
      pthread_mutex_lock(&s->mu);
      if (s->b.o_update(&s->b.opart, value_code(), s->b.data, s->b.size, keys, vals, n) >= 0) s->errors++;
      receipt_set(s, mid, 1); /* updateFinished(id) */
      pthread_mutex_unlock(&s->mu);
      free(keys);
      free(vals);
    }
  } else if (t == W_PULL_VECTOR) {
    int32_t n;
    cmode = 1;
    c->wmode = 1;
    memcpy(&n, buf + 1, 4);
    const size_t need = 5 + (size_t)n * 8;
    if (need > c->rcap) {
      c->rcap = need;
      c->resp = (uint8_t*)realloc(c->resp, c->rcap);
    }
    size_t olen = 0;
    if (use_gpu) { /* enqueued after every push on the shard; its Response is held until the wait */
      /* the answer (r + 5) 8-aligned in the arena when it fits and is answered in place (a page of
       * answer or more, as the library decides: GLINT_DIRECT_MIN_BYTES), else a malloc'd buffer --
       * smaller answers are copied out of the ring slot, and copied into ordinary memory faster */
      size_t pos = c->aused + ((8 - ((uintptr_t)c->arena + c->aused + 5) % 8) % 8);
      uint8_t* r;
      int owned = 0;
      if (c->arena && (size_t)n * 8 >= 4096 && pos + need <= arena_bytes) {
        r = c->arena + pos;
        c->aused = pos + need;
      } else {
        r = (uint8_t*)malloc(need);
        owned = 1;
      }
      uint64_t ticket = 0;
      if (s->b.g_pull_async(s->b.shard, buf, len, r, need, &olen, &ticket) != 0) s->errors++;
      if (ticket > c->last_ticket) c->last_ticket = ticket;
      c->enqueued = 1;
      if (c->nhold == c->hcap) {
        c->hcap = c->hcap ? 2 * c->hcap : 64;
        c->holds = (hold*)realloc(c->holds, c->hcap * sizeof(hold));
      }
      c->holds[c->nhold].end = c->out.len;
      c->holds[c->nhold].ack_id = 0;
      c->holds[c->nhold].resp = r;
      c->holds[c->nhold].resp_len = olen;
      c->holds[c->nhold].owned = owned;
      ++c->nhold;
    } else {
      int64_t* keys = (int64_t*)malloc((size_t)n * 8 + 8);
      memcpy(keys, buf + 5, (size_t)n * 8);
      pthread_mutex_lock(&s->mu);
      if (s->b.o_get(&s->b.opart, value_code(), s->b.data, s->b.size, keys, c->resp + 5, n) >= 0) s->errors++;
      pthread_mutex_unlock(&s->mu);
      free(keys);
      c->resp[0] = dtype_long ? W_RESP_L : W_RESP_D;
      memcpy(c->resp + 1, &n, 4);
      olen = need;
      ob_frame(&c->out, c->resp, (uint32_t)olen);
    }
  } else if (t == L_GET_UID) {
    pthread_mutex_lock(&s->mu);
    const int32_t u = ++s->uid; /* sender ! UniqueID(nextId()) */
    pthread_mutex_unlock(&s->mu);
    ob_logic(&c->out, L_UID, u);
  } else if (t == L_ACK) {
    int mine = 0;
    for (size_t i = 0; i < c->npend && !mine; ++i) mine = c->pending[i] == id;
    if (mine) { /* its push is still on the GPU: answered after the settle's wait */
      if (c->nhold == c->hcap) {
        c->hcap = c->hcap ? 2 * c->hcap : 64;
        c->holds = (hold*)realloc(c->holds, c->hcap * sizeof(hold));
      }
      c->holds[c->nhold].end = c->out.len;
      c->holds[c->nhold].ack_id = id;
      c->holds[c->nhold].resp = NULL;
      ++c->nhold;
    } else {
      pthread_mutex_lock(&s->mu);
      ob_logic(&c->out, receipt_has(s, id) ? L_ACK : L_NACK, id);
      pthread_mutex_unlock(&s->mu);
    }
  } else if (t == L_FORGET) {
    pthread_mutex_lock(&s->mu);
    if (receipt_has(s, id)) receipt_set(s, id, 0);
    pthread_mutex_unlock(&s->mu);
    ob_logic(&c->out, L_FORGET, id);
  } else if (t == L_STOP) {
    return 1;
  } else {
    s->errors++;
  }
  if (cpu_stats && cmode >= 0) {
    c->cs[cmode] += tcpu() - c0;
    c->cs[6 + cmode] += now_s() - cw0;
  }
  return 0;
}

/* After the wait that covered c's enqueued work (rc: its status): the pushes' receipts, then the held
 * replies spliced into the reply stream at their places, then one send. */
static void answer(server* s, cstate* c, int rc) {
  if (c->enqueued) {
    pthread_mutex_lock(&s->mu);
    for (size_t i = 0; i < c->npend; ++i)
      if (rc == 0) receipt_set(s, c->pending[i], 1); /* updateFinished(id) */
    pthread_mutex_unlock(&s->mu);
    if (rc != 0) s->errors++;
    c->npend = 0;
    c->enqueued = 0;
    c->last_ticket = 0;
  }
  if (c->nhold) {
    obuf merged = {0};
    size_t from = 0;
    pthread_mutex_lock(&s->mu);
    for (size_t i = 0; i < c->nhold; ++i) {
      ob_put(&merged, c->out.p + from, c->holds[i].end - from);
      from = c->holds[i].end;
      if (c->holds[i].resp) {
        ob_frame(&merged, c->holds[i].resp, (uint32_t)c->holds[i].resp_len);
        if (c->holds[i].owned) free(c->holds[i].resp);
      } else {
        ob_logic(&merged, receipt_has(s, c->holds[i].ack_id) ? L_ACK : L_NACK, c->holds[i].ack_id);
      }
    }
    pthread_mutex_unlock(&s->mu);
    ob_put(&merged, c->out.p + from, c->out.len - from);
    free(c->out.p);
    c->out = merged;
    c->nhold = 0;
    c->aused = 0; /* every answer in the arena has been sent */
  }
  ob_flush(&c->out, c->fd);
}

/* the wait for everything a settle covers (ticket: the highest), timed for --cpu-stats */
static int settle_wait(server* s, uint64_t ticket, double* cs, int wmode) {
  const double w0 = cpu_stats ? tcpu() : 0.0, ww0 = cpu_stats ? now_s() : 0.0;
  const int rc = s->b.g_wait(s->b.shard, ticket, NULL);
  if (cpu_stats) {
    cs[2 + wmode] += tcpu() - w0;
    cs[4 + wmode] += now_s() - ww0;
  }
  return rc;
}

static void cstate_free(server* s, cstate* c) {
  if (cpu_stats) {
    pthread_mutex_lock(&s->mu);
    for (int i = 0; i < 8; ++i) s->cpu[i] += c->cs[i];
    pthread_mutex_unlock(&s->mu);
  }
  close(c->fd);
  if (c->arena) g_host_free(c->arena);
  free(c->resp);
  free(c->out.p);
  free(c->pending);
  free(c->holds);
}

/* --server threads (the default): each connection's thread runs the server loop for its messages
 * (the actor's one-at-a-time update under the server's mutex), with one wait per drained burst */
static void* conn_main(void* p) {
  conn_arg* a = (conn_arg*)p;
  if (use_gpu && replies_async) return conn_main_async(a);
  server* s = a->s;
  cstate c;
  memset(&c, 0, sizeof(c));
  c.fd = a->fd;
  cstate_arena(&c);
  uint8_t* buf = NULL;
  size_t cap = 0;
  for (;;) {
    const uint32_t len = recv_frame(c.fd, &buf, &cap);
    if (len == 0) break;
    if (handle_msg(s, &c, buf, len)) break;
    if (!readable_now(c.fd)) { /* the burst is drained: one wait for the enqueued work, then reply */
      const int rc = c.enqueued ? settle_wait(s, c.last_ticket, c.cs, c.wmode) : 0;
      answer(s, &c, rc);
    }
  }
  ob_flush(&c.out, c.fd);
  cstate_free(s, &c);
  free(buf);
  free(a);
  return NULL;
}

/* --server actor: the Akka model. Connection threads only receive frames into the server's mailbox;
 * ONE thread per server (the PartialVector actor) takes them in arrival order and runs the update /
 * get for each, enqueueing on the GPU without waiting. When the mailbox is empty it settles: one wait
 * for the highest ticket it enqueued, then every connection's held replies (GpuShard.scala's
 * FlushPulls, integration/scala). */
typedef struct {
  cstate* c; /* NULL: the sender's connection closed */
  uint8_t* buf;
  uint32_t len;
} mitem;
typedef struct {
  server* s;
  int nconn;
  pthread_mutex_t mu;
  pthread_cond_t cv;
  mitem* q;
  size_t n, cap;
  int closed; /* connections whose receive loop ended */
} mailbox;

static void mb_put(mailbox* m, mitem it) {
  pthread_mutex_lock(&m->mu);
  if (m->n == m->cap) {
    m->cap = m->cap ? 2 * m->cap : 1024;
    m->q = (mitem*)realloc(m->q, m->cap * sizeof(mitem));
    if (!m->q) die("realloc");
  }
  m->q[m->n++] = it;
  if (m->n == 1) pthread_cond_signal(&m->cv);
  pthread_mutex_unlock(&m->mu);
}

typedef struct {
  mailbox* m;
  cstate* c;
} aconn_arg;

static void* aconn_main(void* p) { /* receive only: each frame (owned) into the mailbox */
  aconn_arg* a = (aconn_arg*)p;
  for (;;) {
    uint8_t* buf = NULL;
    size_t cap = 0;
    const uint32_t len = recv_frame(a->c->fd, &buf, &cap);
    if (len == 0) {
      free(buf);
      break;
    }
    const int stop = buf[0] == L_STOP;  /* read before the hand-off: the actor frees the frame */
    mitem it = {a->c, buf, len};
    mb_put(a->m, it);
    if (stop) break;
  }
  mitem end = {NULL, NULL, 0};
  mb_put(a->m, end);
  free(a);
  return NULL;
}

static void actor_loop(mailbox* m, cstate* conns) {
  server* s = m->s;
  cstate** dirty = (cstate**)malloc(sizeof(cstate*) * (size_t)m->nconn);
  size_t ndirty = 0;
  mitem* batch = NULL;
  size_t bcap = 0;
  int closed = 0;
  double cs[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int wmode = 0;
  while (closed < m->nconn) {
    pthread_mutex_lock(&m->mu);
    if (m->n == 0 && ndirty) { /* the mailbox is empty: settle before sleeping */
      pthread_mutex_unlock(&m->mu);
      uint64_t tmax = 0;
      for (size_t i = 0; i < ndirty; ++i)
        if (dirty[i]->last_ticket > tmax) tmax = dirty[i]->last_ticket;
      const int rc = tmax ? settle_wait(s, tmax, cs, wmode) : 0;
      for (size_t i = 0; i < ndirty; ++i) {
        answer(s, dirty[i], rc);
        dirty[i]->dirty = 0;
      }
      ndirty = 0;
      continue;
    }
    while (m->n == 0) pthread_cond_wait(&m->cv, &m->mu);
    mitem* q = m->q; /* swap the mailbox out: the receivers keep appending to the other array */
    const size_t n = m->n, qcap = m->cap;
    m->q = batch;
    m->cap = bcap;
    m->n = 0;
    pthread_mutex_unlock(&m->mu);
    batch = q;
    bcap = qcap;
    for (size_t i = 0; i < n; ++i) {
      cstate* c = batch[i].c;
      if (!c) {
        ++closed;
        continue;
      }
      if (batch[i].buf[0] != L_STOP) {
        handle_msg(s, c, batch[i].buf, batch[i].len);
        wmode = c->wmode;
        if (!c->dirty) {
          c->dirty = 1;
          dirty[ndirty++] = c;
        }
      }
      free(batch[i].buf);
    }
  }
  for (size_t i = 0; i < ndirty; ++i) answer(s, dirty[i], 0);
  for (int i = 0; i < 8; ++i) conns[0].cs[i] += cs[i];
  free(dirty);
  free(batch);
}

static int server_actor; /* --server actor */

typedef struct {
  server* s;
  int nconn;
} acceptor_arg;

static void* acceptor_main(void* p) {
  acceptor_arg* a = (acceptor_arg*)p;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)a->nconn);
  if (server_actor) { /* receivers per connection, this thread runs the server's actor */
    mailbox m;
    memset(&m, 0, sizeof(m));
    m.s = a->s;
    m.nconn = a->nconn;
    pthread_mutex_init(&m.mu, NULL);
    pthread_cond_init(&m.cv, NULL);
    cstate* conns = (cstate*)calloc((size_t)a->nconn, sizeof(cstate));
    for (int i = 0; i < a->nconn; ++i) {
      int fd = accept(a->s->listen_fd, NULL, NULL);
      if (fd < 0) die("accept");
      tune_socket(fd);
      conns[i].fd = fd;
      cstate_arena(&conns[i]);
      aconn_arg* c = (aconn_arg*)malloc(sizeof(aconn_arg));
      c->m = &m;
      c->c = &conns[i];
      pthread_create(&th[i], NULL, aconn_main, c);
    }
    actor_loop(&m, conns);
    for (int i = 0; i < a->nconn; ++i) pthread_join(th[i], NULL);
    for (int i = 0; i < a->nconn; ++i) {
      ob_flush(&conns[i].out, conns[i].fd);
      cstate_free(a->s, &conns[i]);
    }
    free(conns);
    free(m.q);
    pthread_mutex_destroy(&m.mu);
    pthread_cond_destroy(&m.cv);
    free(th);
    return NULL;
  }
  for (int i = 0; i < a->nconn; ++i) {
    int fd = accept(a->s->listen_fd, NULL, NULL);
    if (fd < 0) die("accept");
    tune_socket(fd);
    conn_arg* c = (conn_arg*)malloc(sizeof(conn_arg));
    c->s = a->s;
    c->fd = fd;
    pthread_create(&th[i], NULL, conn_main, c);
  }
  for (int i = 0; i < a->nconn; ++i) pthread_join(th[i], NULL);
  free(th);
  return NULL;
}

/* ---- clients ------------------------------------------------------------------------------------ */
/* java.util.Random -- the values of GranularBigVectorSpec.scala:14-35 (seed 42) */
typedef struct { uint64_t seed; } jrandom;
static void jr_init(jrandom* r, int64_t s) { r->seed = ((uint64_t)s ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1); }
static int32_t jr_next(jrandom* r, int bits) {
  r->seed = (r->seed * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
  return (int32_t)(int64_t)(r->seed >> (48 - bits));
}
static double jr_double(jrandom* r) {
  return (double)(((int64_t)jr_next(r, 26) << 27) + jr_next(r, 27)) * (1.0 / (double)(1LL << 53));
}
static uint64_t splitmix(uint64_t* x) {
  uint64_t z = (*x += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

static int S, C, M, W;
static int64_t N;
static int32_t n_small, q_small;
static int64_t small_keys;
static int32_t owner_of(int64_t k) {
  const int64_t large = (int32_t)((uint32_t)q_small + 1u); /* an Int, wraps (RangePartitioner.scala:18) */
  return (int32_t)(uint32_t)(uint64_t)(k < small_keys ? k / q_small : n_small + (k - small_keys) / large);
}

typedef struct {
  int32_t id;
  int32_t n;
  int64_t* idx; /* record positions of the message */
} fsm;

typedef struct {
  int c;               /* client index */
  int part;            /* server / partition */
  int fd;
  const int64_t* keys; /* the client's records */
  const void* vals;
  int64_t n;
  void* pulled;        /* values pulled back, at the records' positions */
  int mode;            /* 0 push, 1 pull */
  int64_t messages, resends;
  fsm* msgs;           /* this link's messages, in slice order (set by the client's bucketing) */
  int64_t nmsg;
} link_arg;

/* ---- client bucketing (mapPartitions, AsyncBigVector.scala:96-98) ------------------------------------ */
static int bucket_device;  /* --bucket device (1) or auto (2) */
/* --bucket auto: a batch is routed on the device while fewer than auto_max clients are (the one GPU
 * and its PCIe link are shared by every client of the loopback; past a few concurrent routes each
 * waits behind the others' transfers), else grouped on the host */
static int auto_max = 4;
static int dev_routes;     /* clients routing on the device right now */
static int dev_batches;    /* batches routed on the device (--bucket auto reports it) */
static void* hip_dl;
static int (*hip_malloc)(void**, size_t);
static int (*hip_free)(void*);
static int (*hip_memcpy_async)(void*, const void*, size_t, int, void*);
static int (*hip_stream_create)(void**, unsigned);
static int (*hip_stream_sync)(void*);
static int (*hip_host_malloc)(void**, size_t, unsigned);
static int (*route_gather_dev)(const int64_t*, const int32_t*, const void*, int, int64_t, int, int32_t, int64_t,
                               const int32_t*, int64_t*, int64_t*, int64_t*, int32_t*, void*, uint64_t*, void*);

/* per partition: its record indices in record order (idx[p][0..cnt[p])) -> the link's messages, cut at
 * the GranularBigVector slice boundaries (every M records) */
static void cut_messages(link_arg* l, int64_t* idx, int64_t cnt) {
  const int64_t nslices = (l->n + M - 1) / M;
  l->msgs = (fsm*)calloc((size_t)(nslices > 0 ? nslices : 1), sizeof(fsm));
  l->nmsg = 0;
  int64_t a = 0;
  while (a < cnt) {
    const int64_t slice = idx[a] / M;
    int64_t b = a;
    while (b < cnt && idx[b] / M == slice) ++b;
    l->msgs[l->nmsg].n = (int32_t)(b - a);
    l->msgs[l->nmsg].idx = idx + a;
    ++l->nmsg;
    a = b;
  }
}

/* A client's device context for the offloaded bucketing, set up before the timed region (a client
 * process holds its GPU buffers and stream for its lifetime): keys in, counts and order out, the order
 * read back into pinned host memory, all on the client's own stream. The client's batch itself lives
 * in pinned memory (a JVM client would fill a direct buffer), so it crosses PCIe in one DMA with no
 * staging copy; the route (glint_route_gather_dev) does not synchronise, so the whole offload is one
 * wait: keys over, route, order + counts + status word back. */
typedef struct {
  void *dk, *dc, *dord, *dbad, *stream;
  int64_t* order; /* pinned */
  int64_t* cnt;   /* pinned: S counts, then the status word */
  int64_t* keys;  /* pinned: the client's batch */
} client_dev;

static void client_dev_init(client_dev* d, const int64_t* keys, int64_t n) {
  const size_t b = (size_t)(n > 0 ? n : 1) * 8;
  if (hip_malloc(&d->dk, b) || hip_malloc(&d->dc, (size_t)S * 8 + 8) || hip_malloc(&d->dord, b)) die("hipMalloc");
  d->dbad = (char*)d->dc + (size_t)S * 8;
  if (hip_stream_create(&d->stream, 1 /* hipStreamNonBlocking */)) die("hipStreamCreateWithFlags");
  if (hip_host_malloc((void**)&d->order, b, 0) || hip_host_malloc((void**)&d->cnt, (size_t)S * 8 + 8, 0) ||
      hip_host_malloc((void**)&d->keys, b, 0))
    die("hipHostMalloc");
  memcpy(d->keys, keys, (size_t)n * 8);
  /* one route of the batch on the new stream, before the timed region: the stream's first use (its
   * hardware queue) and the route's scratch, sized by the batch, are paid here, as a client process
   * pays them once for its batches */
  if (n > 0) {
    if (hip_memcpy_async(d->dk, d->keys, (size_t)n * 8, 1, d->stream) ||
        route_gather_dev((const int64_t*)d->dk, NULL, NULL, 0, n, 0, S, N, NULL, (int64_t*)d->dc, (int64_t*)d->dord,
                         NULL, NULL, NULL, (uint64_t*)d->dbad, d->stream) ||
        hip_memcpy_async(d->cnt, d->dc, (size_t)S * 8 + 8, 2, d->stream) || hip_stream_sync(d->stream))
      die("client warm-up route");
  }
}

/* Buckets client c's batch for its S links; returns the seconds it took. `store` receives the S
 * index arrays (freed by the caller). */
static double bucket_client(link_arg* links, const int64_t* keys, int64_t n, int64_t** store, client_dev* d) {
  const double t0 = now_s();
  int64_t* cnt = (int64_t*)calloc((size_t)S, 8);
  int on_dev = bucket_device == 1 && n > 0;
  if (bucket_device == 2 && n > 0) {
    if (__atomic_add_fetch(&dev_routes, 1, __ATOMIC_ACQ_REL) <= auto_max) on_dev = 1;
    else __atomic_sub_fetch(&dev_routes, 1, __ATOMIC_ACQ_REL);
  }
  if (on_dev) {
    /* offloaded: one stable route of the whole batch on the GPU, on the client's stream, one wait */
    if (hip_memcpy_async(d->dk, d->keys, (size_t)n * 8, 1 /* hipMemcpyHostToDevice */, d->stream)) die("hipMemcpyAsync");
    if (route_gather_dev((const int64_t*)d->dk, NULL, NULL, 0, n, 0 /* GLINT_ROUTE_RANGE */, S, N, NULL,
                         (int64_t*)d->dc, (int64_t*)d->dord, NULL, NULL, NULL, (uint64_t*)d->dbad, d->stream))
      die("glint_route_gather_dev");
    if (hip_memcpy_async(d->order, d->dord, (size_t)n * 8, 2 /* DeviceToHost */, d->stream) ||
        hip_memcpy_async(d->cnt, d->dc, (size_t)S * 8 + 8, 2, d->stream) || hip_stream_sync(d->stream))
      die("hipMemcpyAsync");
    if (d->cnt[S] != 0) die("glint_route_gather_dev: key outside the partitioner");
    memcpy(cnt, d->cnt, (size_t)S * 8);
    /* each partition's ordered index list is read where it landed (the pinned order buffer, the
     * client's for its lifetime): no copy */
    int64_t o = 0;
    for (int p = 0; p < S; ++p) {
      cut_messages(&links[p], d->order + o, cnt[p]);
      store[p] = NULL;
      o += cnt[p];
    }
    if (bucket_device == 2) {
      __atomic_sub_fetch(&dev_routes, 1, __ATOMIC_ACQ_REL);
      __atomic_add_fetch(&dev_batches, 1, __ATOMIC_ACQ_REL);
    }
    free(cnt);
    return now_s() - t0;
  } else {
    /* the reference's groupBy, slice by slice: one pass per slice, each index appended to its
     * partition's list (lists grow as the groupBy's buffers do) */
    int64_t* capv = (int64_t*)calloc((size_t)S, 8);
    for (int p = 0; p < S; ++p) {
      capv[p] = 1024;
      store[p] = (int64_t*)malloc((size_t)capv[p] * 8);
    }
    for (int64_t s0 = 0; s0 < n; s0 += M) {
      const int64_t s1 = s0 + M < n ? s0 + M : n;
      for (int64_t j = s0; j < s1; ++j) {
        const int32_t p = owner_of(keys[j]);
        if (cnt[p] == capv[p]) {
          capv[p] *= 2;
          store[p] = (int64_t*)realloc(store[p], (size_t)capv[p] * 8);
          if (!store[p]) die("realloc");
        }
        store[p][cnt[p]++] = j;
      }
    }
    free(capv);
  }
  for (int p = 0; p < S; ++p) cut_messages(&links[p], store[p], cnt[p]);
  free(cnt);
  return now_s() - t0;
}

typedef struct {
  link_arg* links; /* this client's S links */
  double bucket_s;
  client_dev dev;  /* --bucket device */
} client_arg;

static void* link_main(void* p);

/* one client: bucket its batch (timed), then run its S links (one connection per server) */
static void* client_main(void* p) {
  client_arg* ca = (client_arg*)p;
  link_arg* l = ca->links;
  int64_t** store = (int64_t**)calloc((size_t)S, sizeof(int64_t*));
  ca->bucket_s = bucket_client(l, l[0].keys, l[0].n, store, &ca->dev);
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)S);
  for (int i = 0; i < S; ++i) pthread_create(&th[i], NULL, link_main, &l[i]);
  for (int i = 0; i < S; ++i) pthread_join(th[i], NULL);
  for (int i = 0; i < S; ++i) {
    free(l[i].msgs);
    l[i].msgs = NULL;
    free(store[i]);
  }
  free(store);
  free(th);
  return NULL;
}

static void* link_main(void* p) {
  link_arg* l = (link_arg*)p;
  uint8_t* buf = NULL;
  size_t cap = 0;
  obuf out = {0};
  /* the messages of this link, in slice order (empty slices send nothing), from the client's bucketing */
  fsm* msgs = l->msgs;
  const int64_t nmsg = l->nmsg;
  uint8_t* m = (uint8_t*)malloc(9 + (size_t)M * 16);
  /* replies come back in request order on a connection: a FIFO of (kind, message) */
  int64_t* fifo_msg = (int64_t*)malloc(sizeof(int64_t) * (size_t)(4 * W + 8));
  uint8_t* fifo_kind = (uint8_t*)malloc((size_t)(4 * W + 8));
  size_t fh = 0, ft = 0;
  const size_t fcap = (size_t)(4 * W + 8);
#define FPUSH(kind, mi) do { fifo_kind[ft % fcap] = (kind); fifo_msg[ft % fcap] = (mi); ++ft; } while (0)
  int64_t started = 0, done = 0;
  const uint8_t ptype = dtype_long ? W_PUSH_VEC_L : W_PUSH_VEC_D;
  while (done < nmsg) {
    while (started < nmsg && started - done < W) { /* issue: GetUniqueID (push) or the pull itself */
      if (l->mode == 0) {
        ob_logic(&out, L_GET_UID, 0);
        FPUSH(L_UID, started);
      } else {
        fsm* f = &msgs[started];
        m[0] = W_PULL_VECTOR; /* RequestSerializer.scala:150-155 */
        memcpy(m + 1, &f->n, 4);
        for (int32_t q = 0; q < f->n; ++q) memcpy(m + 5 + (size_t)q * 8, &l->keys[f->idx[q]], 8);
        ob_frame(&out, m, 5 + (uint32_t)f->n * 8);
        l->messages++;
        FPUSH(W_PULL_VECTOR, started);
      }
      ++started;
    }
    ob_flush(&out, l->fd);
    const uint32_t len = recv_frame(l->fd, &buf, &cap);
    if (len == 0) die("protocol: connection closed");
    if (fh == ft) die("protocol: unexpected reply");
    const uint8_t kind = fifo_kind[fh % fcap];
    const int64_t mi = fifo_msg[fh % fcap];
    ++fh;
    fsm* f = &msgs[mi];
    if (kind == L_UID) {
      if (len != 5 || buf[0] != L_UID) die("protocol: UniqueID");
      memcpy(&f->id, buf + 1, 4);
      goto execute;
    } else if (kind == L_ACK) {
      if (len != 5) die("protocol: ack");
      if (buf[0] == L_ACK) {
        ob_logic(&out, L_FORGET, f->id); /* forget() */
        FPUSH(L_FORGET, mi);
      } else {
        l->resends++; /* NotAcknowledgeReceipt: execute() again */
        goto execute;
      }
    } else if (kind == L_FORGET) {
      if (len != 5 || buf[0] != L_FORGET) die("protocol: forget");
      ++done;
    } else { /* a pull response */
      int32_t rn;
      if (len < 5 || buf[0] != (dtype_long ? W_RESP_L : W_RESP_D)) die("protocol: response");
      memcpy(&rn, buf + 1, 4);
      if (rn != f->n || len != 5 + (uint32_t)f->n * 8) die("protocol: response size");
      for (int32_t q = 0; q < f->n; ++q) memcpy((char*)l->pulled + (size_t)f->idx[q] * 8, buf + 5 + (size_t)q * 8, 8);
      ++done;
    }
    continue;
  execute:
    m[0] = ptype; /* RequestSerializer.scala:157-173 */
    memcpy(m + 1, &f->n, 4);
    memcpy(m + 5, &f->id, 4);
    for (int32_t q = 0; q < f->n; ++q) {
      memcpy(m + 9 + (size_t)q * 8, &l->keys[f->idx[q]], 8);
      memcpy(m + 9 + (size_t)f->n * 8 + (size_t)q * 8, (const char*)l->vals + (size_t)f->idx[q] * 8, 8);
    }
    ob_frame(&out, m, 9 + (uint32_t)f->n * 16); /* execute(): actorRef ! message(id) */
    l->messages++;
    ob_logic(&out, L_ACK, f->id); /* acknowledge() */
    FPUSH(L_ACK, mi);
  }
  ob_flush(&out, l->fd);
  free(m);
  free(fifo_msg);
  free(fifo_kind);
  free(buf);
  free(out.p);
  return NULL;
}

int main(int argc, char** argv) {
  const char* kind = "oracle";
  const char* lib = NULL;
  const char* pattern = "dense";
  S = 2;
  C = 1;
  M = 1000;
  W = 64;
  N = 1000000;
  int64_t R = 0;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--backend") && i + 1 < argc) kind = argv[++i];
    else if (!strcmp(argv[i], "--lib") && i + 1 < argc) lib = argv[++i];
    else if (!strcmp(argv[i], "--servers") && i + 1 < argc) S = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--clients") && i + 1 < argc) C = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--keys") && i + 1 < argc) N = atoll(argv[++i]);
    else if (!strcmp(argv[i], "--records") && i + 1 < argc) R = atoll(argv[++i]);
    else if (!strcmp(argv[i], "--msg") && i + 1 < argc) M = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--window") && i + 1 < argc) W = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--pattern") && i + 1 < argc) pattern = argv[++i];
    else if (!strcmp(argv[i], "--dtype") && i + 1 < argc) dtype_long = !strcmp(argv[++i], "long");
    else if (!strcmp(argv[i], "--device") && i + 1 < argc) gpu_device = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--bucket") && i + 1 < argc) {
      ++i;
      bucket_device = !strcmp(argv[i], "device") ? 1 : !strcmp(argv[i], "auto") ? 2 : 0;
    } else if (!strcmp(argv[i], "--auto-max") && i + 1 < argc) auto_max = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--cpu-stats")) cpu_stats = 1;
    else if (!strcmp(argv[i], "--answers") && i + 1 < argc) answers_direct = !strcmp(argv[++i], "direct");
    else if (!strcmp(argv[i], "--server") && i + 1 < argc) server_actor = !strcmp(argv[++i], "actor");
    else if (!strcmp(argv[i], "--replies") && i + 1 < argc) replies_async = !strcmp(argv[++i], "async");
    else {
      fprintf(stderr, "usage: %s --backend oracle|gpu --lib PATH [--servers S] [--clients C] [--keys N] "
                      "[--pattern dense|uniform] [--records R] [--msg M] [--window W] [--dtype double|long] "
                      "[--device D] [--bucket groupby|device|auto] [--auto-max K] [--replies async|burst] [--server threads|actor] [--answers direct|copy] [--cpu-stats]\n", argv[0]);
      return 2;
    }
  }
  const int uniform = !strcmp(pattern, "uniform");
  if (!lib || S <= 0 || C <= 0 || N <= 0 || M <= 0 || W <= 0) { fprintf(stderr, "glint_loopback: bad arguments\n"); return 2; }
  if (uniform && R <= 0) R = N / C;
  backend_open(kind, lib);
  if (use_gpu) {
    *(void**)&g_host_alloc = dlsym(dl, "glint_host_alloc");
    *(void**)&g_host_free = dlsym(dl, "glint_host_free");
    if (answers_direct < 0) answers_direct = g_host_alloc && g_host_free;
    if (answers_direct && (!g_host_alloc || !g_host_free)) die("dlsym glint_host_alloc");
    arena_bytes = (size_t)W * ((size_t)M * 8 + 16);
  } else {
    answers_direct = 0;
  }
  if (bucket_device) { /* the device route of libglint_gpu.so and the HIP runtime it runs on */
    if (!use_gpu) { fprintf(stderr, "glint_loopback: --bucket device needs --backend gpu\n"); return 2; }
    hip_dl = dlopen("libamdhip64.so", RTLD_NOW | RTLD_LOCAL);
    if (!hip_dl) hip_dl = dlopen("/opt/rocm/lib/libamdhip64.so", RTLD_NOW | RTLD_LOCAL);
    if (!hip_dl) { fprintf(stderr, "glint_loopback: dlopen libamdhip64.so: %s\n", dlerror()); return 2; }
    *(void**)&hip_malloc = dlsym(hip_dl, "hipMalloc");
    *(void**)&hip_free = dlsym(hip_dl, "hipFree");
    *(void**)&hip_memcpy_async = dlsym(hip_dl, "hipMemcpyAsync");
    *(void**)&hip_stream_create = dlsym(hip_dl, "hipStreamCreateWithFlags");
    *(void**)&hip_stream_sync = dlsym(hip_dl, "hipStreamSynchronize");
    *(void**)&hip_host_malloc = dlsym(hip_dl, "hipHostMalloc");
    *(void**)&route_gather_dev = dlsym(dl, "glint_route_gather_dev");
    if (!hip_malloc || !hip_free || !hip_memcpy_async || !hip_stream_create || !hip_stream_sync || !hip_host_malloc ||
        !route_gather_dev)
      die("dlsym hip*/glint_route_gather_dev");
  }

  /* RangePartitioner.apply(S, N) (RangePartitioner.scala:62-84) and partition() (:27-43) */
  const int32_t n_large = (int32_t)(N % S);
  n_small = S - n_large;
  q_small = (int32_t)((N - N % S) / S);
  small_keys = (int64_t)n_small * q_small;
  server* sv = (server*)calloc((size_t)S, sizeof(server));
  {
    int64_t start = 0, end = q_small;                                         /* :68-69 */
    for (int i = 0; i < S; ++i) {
      if (i >= n_small) end += 1;                                              /* :76 */
      sv[i].start = start;
      sv[i].end = end;
      start += i < n_small ? q_small : (int32_t)((uint32_t)q_small + 1u);     /* :73,:78 (Int + 1 wraps) */
      end += q_small;                                                          /* :74,:79 */
    }
  }
  /* the clients' records */
  int64_t* cn = (int64_t*)calloc((size_t)C, 8);
  int64_t** ck = (int64_t**)calloc((size_t)C, sizeof(int64_t*));
  void** cv = (void**)calloc((size_t)C, sizeof(void*));
  void** cp = (void**)calloc((size_t)C, sizeof(void*));
  for (int c = 0; c < C; ++c) {
    int64_t lo = 0, n;
    if (uniform) n = R;
    else { lo = N * c / C; n = N * (c + 1) / C - lo; }
    cn[c] = n;
    ck[c] = (int64_t*)malloc((size_t)(n > 0 ? n : 1) * 8);
    cv[c] = malloc((size_t)(n > 0 ? n : 1) * 8);
    cp[c] = calloc((size_t)(n > 0 ? n : 1), 8);
    jrandom jr;
    jr_init(&jr, 42 + c); /* client 0: GranularBigVectorSpec's java.util.Random(42) */
    uint64_t sm = 0x5EED0000ULL + (uint64_t)c;
    for (int64_t j = 0; j < n; ++j) {
      ck[c][j] = uniform ? (int64_t)(splitmix(&sm) % (uint64_t)N) : lo + j;
      if (dtype_long) ((int64_t*)cv[c])[j] = (int64_t)(splitmix(&sm) % 2001) - 1000;
      else ((double*)cv[c])[j] = jr_double(&jr);
    }
  }

  /* servers: one acceptor per server, one thread per client connection */
  pthread_t* at = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)S);
  acceptor_arg* aa = (acceptor_arg*)calloc((size_t)S, sizeof(acceptor_arg));
  for (int i = 0; i < S; ++i) {
    backend_init(&sv[i].b, sv[i].start, sv[i].end);
    pthread_mutex_init(&sv[i].mu, NULL);
    sv[i].listen_fd = socket(AF_INET, SOCK_STREAM, 0);
    if (sv[i].listen_fd < 0) die("socket");
    struct sockaddr_in ad;
    memset(&ad, 0, sizeof(ad));
    ad.sin_family = AF_INET;
    ad.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (bind(sv[i].listen_fd, (struct sockaddr*)&ad, sizeof(ad)) < 0) die("bind");
    if (listen(sv[i].listen_fd, C + 8) < 0) die("listen");
    socklen_t sl = sizeof(ad);
    getsockname(sv[i].listen_fd, (struct sockaddr*)&ad, &sl);
    sv[i].port = ntohs(ad.sin_port);
    aa[i].s = &sv[i];
    aa[i].nconn = C;
    pthread_create(&at[i], NULL, acceptor_main, &aa[i]);
  }
  const int L = C * S;
  link_arg* la = (link_arg*)calloc((size_t)L, sizeof(link_arg));
  for (int c = 0; c < C; ++c)
    for (int i = 0; i < S; ++i) {
      link_arg* l = &la[c * S + i];
      l->fd = socket(AF_INET, SOCK_STREAM, 0);
      struct sockaddr_in ad;
      memset(&ad, 0, sizeof(ad));
      ad.sin_family = AF_INET;
      ad.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
      ad.sin_port = htons((uint16_t)sv[i].port);
      if (connect(l->fd, (struct sockaddr*)&ad, sizeof(ad)) < 0) die("connect");
      tune_socket(l->fd);
      l->c = c;
      l->part = i;
      l->keys = ck[c];
      l->vals = cv[c];
      l->n = cn[c];
      l->pulled = cp[c];
    }
  pthread_t* ct = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)C);
  client_arg* cargs = (client_arg*)calloc((size_t)C, sizeof(client_arg));
  if (bucket_device)
    for (int c = 0; c < C; ++c) client_dev_init(&cargs[c].dev, ck[c], cn[c]);
  if (!(use_gpu && replies_async)) /* every connection's server side is set up (conn_main_async has no arena) */
    while (__atomic_load_n(&conns_ready, __ATOMIC_ACQUIRE) < S * C) usleep(1000);
  double t[3], pc[3], bucket_s[2] = {0, 0}, bucket_max[2] = {0, 0};
  int64_t msgs[2] = {0, 0}, resends = 0;
  for (int mode = 0; mode < 2; ++mode) {
    t[mode] = now_s();
    pc[mode] = pcpu();
    for (int c = 0; c < C; ++c) {
      for (int i = 0; i < S; ++i) {
        la[c * S + i].mode = mode;
        la[c * S + i].messages = 0;
      }
      cargs[c].links = &la[c * S];
      pthread_create(&ct[c], NULL, client_main, &cargs[c]);
    }
    for (int c = 0; c < C; ++c) {
      pthread_join(ct[c], NULL);
      bucket_s[mode] += cargs[c].bucket_s / C;
      if (cargs[c].bucket_s > bucket_max[mode]) bucket_max[mode] = cargs[c].bucket_s;
    }
    for (int x = 0; x < L; ++x) {
      msgs[mode] += la[x].messages;
      resends += la[x].resends;
    }
  }
  t[2] = now_s();
  pc[2] = pcpu();
  for (int x = 0; x < L; ++x) {
    uint8_t stop[9] = {5, 0, 0, 0, L_STOP, 0, 0, 0, 0};
    write_all(la[x].fd, stop, 9);
  }
  int errors = 0;
  double scpu[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < S; ++i) {
    pthread_join(at[i], NULL);
    errors += sv[i].errors;
    for (int j = 0; j < 8; ++j) scpu[j] += sv[i].cpu[j];
    close(sv[i].listen_fd);
  }
  for (int x = 0; x < L; ++x) close(la[x].fd);

  /* checks */
  int ok = errors == 0;
  int64_t total = 0;
  for (int c = 0; c < C; ++c) total += cn[c];
  if (!uniform) { /* each key pushed once: pulled == pushed, bit for bit */
    for (int c = 0; c < C && ok; ++c) ok = memcmp(cp[c], cv[c], (size_t)cn[c] * 8) == 0;
  } else { /* the sequential sum over every client's records, then compared per pulled record */
    void* sum = calloc((size_t)N, 8);
    double* mag = dtype_long ? NULL : (double*)calloc((size_t)N, 8);
    for (int c = 0; c < C; ++c)
      for (int64_t j = 0; j < cn[c]; ++j) {
        const int64_t k = ck[c][j];
        if (dtype_long) ((int64_t*)sum)[k] = (int64_t)((uint64_t)((int64_t*)sum)[k] + (uint64_t)((int64_t*)cv[c])[j]);
        else { ((double*)sum)[k] += ((double*)cv[c])[j]; mag[k] += fabs(((double*)cv[c])[j]); }
      }
    for (int c = 0; c < C && ok; ++c)
      for (int64_t j = 0; j < cn[c] && ok; ++j) {
        const int64_t k = ck[c][j];
        if (dtype_long) ok = ((int64_t*)cp[c])[j] == ((int64_t*)sum)[k];
        else ok = fabs(((double*)cp[c])[j] - ((double*)sum)[k]) <= 1e-9 * mag[k] + 1e-300;
      }
    free(sum);
    free(mag);
  }
  for (int i = 0; i < S; ++i) backend_close(&sv[i].b);
  const double tp = t[1] - t[0], tl = t[2] - t[1];
  printf("{\"backend\": \"%s\", \"pattern\": \"%s\", \"dtype\": \"%s\", \"servers\": %d, \"clients\": %d, "
         "\"keys\": %lld, \"records\": %lld, \"max_records_per_message\": %d, \"window\": %d, "
         "\"push_messages\": %lld, \"pull_messages\": %lld, \"resends\": %lld, \"push_s\": %.6f, \"pull_s\": %.6f, "
         "\"push_records_per_s\": %.1f, \"pull_records_per_s\": %.1f, \"push_payload_MBps\": %.2f, "
         "\"pull_payload_MBps\": %.2f, \"server\": \"%s\", \"answers\": \"%s\", \"replies\": \"%s\", \"bucket\": \"%s\", \"bucket_s_per_client\": [%.6f, %.6f], "
         "\"bucket_s_max\": [%.6f, %.6f], \"device_batches\": %d, \"process_cpu_s\": [%.4f, %.4f], \"server_call_cpu_s\": [%.4f, %.4f], "
         "\"server_wait_cpu_s\": [%.4f, %.4f], \"server_wait_wall_s\": [%.4f, %.4f], \"server_call_wall_s\": [%.4f, %.4f], "
         "\"first_values\": [%.17g, %.17g, %.17g], \"check\": %s}\n",
         kind, pattern, dtype_long ? "long" : "double", S, C, (long long)N, (long long)total, M, W,
         (long long)msgs[0], (long long)msgs[1], (long long)resends, tp, tl, (double)total / tp, (double)total / tl,
         16.0 * (double)total / tp / 1e6, 16.0 * (double)total / tl / 1e6,
         server_actor ? "actor" : "threads", answers_direct ? "direct" : "copy", !use_gpu ? "inline" : replies_async ? "async" : "burst", bucket_device == 1 ? "device" : bucket_device == 2 ? "auto" : "groupby", bucket_s[0], bucket_s[1], bucket_max[0], bucket_max[1],
         bucket_device == 1 ? 2 * C : dev_batches, pc[1] - pc[0], pc[2] - pc[1], scpu[0], scpu[1], scpu[2], scpu[3], scpu[4], scpu[5], scpu[6], scpu[7],
         dtype_long ? 0.0 : ((double*)cv[0])[0], (!dtype_long && cn[0] > 1) ? ((double*)cv[0])[1] : 0.0,
         (!dtype_long && cn[0] > 2) ? ((double*)cv[0])[2] : 0.0, ok ? "true" : "false");
  return ok ? 0 : 1;
}
