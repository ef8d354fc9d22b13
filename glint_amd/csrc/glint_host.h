// glint_host.h -- host-side state of a shard (the handle behind glint_shard_t) and the helpers
// shared by the C ABI (glint_gpu.hip) and the sort-based push tails (glint_sort.hip).
#pragma once
#include "glint_kernels.h"
#include "../../include/glint_gpu.h"

#include <hip/hip_ext.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <utility>
#include <vector>

using namespace glint;

// One pending kernel write into a glint_host_alloc buffer (a pull answering in place): the buffer's
// pending count is held from enqueue until the entry retires, and glint_host_free refuses the buffer
// while it is non-zero.
struct HostHold {
  std::shared_ptr<std::atomic<long>> c;
  HostHold() = default;
  explicit HostHold(std::shared_ptr<std::atomic<long>> p) : c(std::move(p)) {
    if (c) c->fetch_add(1, std::memory_order_acq_rel);
  }
  HostHold(const HostHold& o) : c(o.c) {
    if (c) c->fetch_add(1, std::memory_order_acq_rel);
  }
  HostHold(HostHold&& o) noexcept : c(std::move(o.c)) {}
  HostHold& operator=(const HostHold& o) {
    if (this != &o) {
      reset();
      c = o.c;
      if (c) c->fetch_add(1, std::memory_order_acq_rel);
    }
    return *this;
  }
  HostHold& operator=(HostHold&& o) noexcept {
    if (this != &o) {
      reset();
      c = std::move(o.c);
    }
    return *this;
  }
  ~HostHold() { reset(); }
  void reset() {
    if (c) c->fetch_sub(1, std::memory_order_acq_rel);
    c.reset();
  }
};

struct glint_shard {
  int device = 0;
  int dtype = 0;
  size_t vsize = 0;
  PartDesc part{};
  i64 elems = 0;  // allocated elements (size * pitch for matrices)
  void* data = nullptr;
  hipStream_t stream = nullptr;
  int cus = 256;
  // per-launch control words (LaunchCtl), zeroed before each ordered push
  void* d_ctl = nullptr;
  size_t ctl_bytes = 0;
  int ctl_par = 0;  // which of the two LaunchCtl slots the next ordered push uses
  ErrState* d_err = nullptr;       // device-resident calls' error state: reported by glint_shard_sync
  ErrState* d_err_host = nullptr;  // host-pointer calls' own (read and cleared by the call itself)
  bool host_call = false;          // set while a host-pointer call launches: its kernels use d_err_host
  // grow-only device scratch for host-pointer calls and the deterministic path
  void* d_scratch = nullptr;
  size_t scratch_bytes = 0;
  void* d_det = nullptr;
  size_t det_bytes = 0;
  // the deterministic tail folds the chains of its hottest elements on a second stream while the rest
  // of the push is sorted (glint_sort.hip); created on first use
  hipStream_t det_stream = nullptr;
  hipEvent_t det_ev[2] = {nullptr, nullptr};
  void* d_bin = nullptr;  // binned-push scratch
  // v2 binned push: two [BinCtl | T] headers, used by alternate pushes; each push's bin_count zeroes
  // the other one for the next push (no memset per push). Zeroed once when allocated.
  void* d_binctl = nullptr;
  int bin_par = 0;
  // the hot front end's global sample table and picks, emptied by their last reader (bin_hot_select,
  // bin_hot_reduce) for the next push instead of by memsets; initialised once when allocated
  void* d_hot = nullptr;
  size_t bin_bytes = 0;
  // binned front end (glint_bin.hip push_binned): 0 plain, 1 plain + hot-element split, 2 chunk dedup
  // (+ hot split). What the last dedup push measured decides: chunk_ratio = records it kept of the cold
  // records that entered its hash table (1.0 = dedup merged nothing), hot_frac = share of the tail
  // taken by the hot elements. A dedup push re-measures every 16 pushes. The measurements reach the
  // host only at sync points (latch_hints), so a device-resident caller that never calls
  // glint_shard_sync keeps the no-history default: the plain front end (ratio 1.0: dedup merged
  // nothing), with a dedup probe every 16 pushes.
  double bin_chunk_ratio = 1.0;
  double bin_hot_frac = 0.0;
  uint32_t bin_pushes = 0;
  int bin_last_front = 0;        // the front end of the last binned push
  u32 hot_age = 0;               // binned pushes since the wide hot table was last sampled (0: never)
  // pinned host staging for host-pointer calls (grow-only, <= pinned_stage_max()): the caller's
  // arrays are memcpy'd in and cross PCIe in one DMA; pull answers come back the same way
  void* h_stage = nullptr;
  size_t h_stage_bytes = 0;
  ErrState* h_err = nullptr;  // pinned: the device error state lands here with the push's last copy
  // pipelined ingest (glint_stage_acquire / glint_push_staged / glint_push_wire_async / glint_pull_async /
  // glint_shard_wait): a ring of pinned, device-mapped host slots; each in-flight entry owns one until it
  // completes. Message-sized entries are one single-workgroup kernel that reads its input from the
  // slot (and writes a pull's answer into it) and then writes its ticket to h_done.
  struct RingSlot {
    char* h = nullptr;       // pinned host memory, mapped (small pushes are read in place by the kernel)
    char* hd = nullptr;      // its device-side address
    size_t hcap = 0;
    char* d = nullptr;       // device copy target for larger pushes
    size_t dcap = 0;
    hipEvent_t done = nullptr;  // completion of a multi-kernel (DMA) entry
    ErrState* herr = nullptr;   // pinned, mapped: the shard's error state right after this entry
    ErrState* herr_d = nullptr;
    uint64_t ticket = 0;
    int64_t n = 0;
    size_t cap_need = 0;        // bytes this entry's layout uses
    void* out = nullptr;        // an async pull's destination: filled from the slot when retired
    size_t out_bytes = 0, out_off = 0;
    bool inflight = false, acquired = false;
    bool sig = false;           // one-workgroup launch that signals through h_done (no event)
    uint64_t ticket_lo = 0;     // first ticket the entry covers (a coalesced batch covers several)
    struct Msg {
      int64_t off, n;
      uint64_t ticket;
      void* out = nullptr;  // a coalesced pull's destination (its answer sits at off in the slot)
      void* dout = nullptr; // out's device address when out is glint_host_alloc memory: the kernel
                            // writes the answer there itself (no copy out of the slot)
      HostHold hold;        // dout's buffer stays allocated until the entry retires
    };
    std::vector<Msg> msgs;      // the messages of this entry, for error attribution
    int64_t fill = 0;           // records appended to an open batch
    bool pull_batch = false;    // a coalesced pull batch: answers go to msgs[i].out when retired
  } ring[GLINT_RING_SLOTS];
  int open_slot = -1;     // the batch that message-sized pushes (or pulls) are appended to, not launched yet
  int open_flags = 0;
  int open_kind = -1;     // -1: a push batch; 0 / 1: a vector / matrix element pull batch
  bool host_pending = false;     // ring entries enqueued on `stream` since a device call last waited for them
  hipEvent_t host_ev = nullptr;
  u64* h_done = nullptr;  // host-mapped: ticket of the last completed signalling launch
  u64* d_done = nullptr;
  MsgSig sig{};           // set only while a ring entry dispatches its one launch
  const PullDst* pull_tab = nullptr;  // set only while a pull batch with direct answers dispatches
  int pull_nm = 0;
  u64* gate = nullptr;  // set only while a gated device push launches (glint_*_push_dev_gated)
  // device scratch of glint_vec_push_dev_shards (the set's verdict word), one per caller stream: calls
  // on one stream are ordered, calls on two streams never share a word (one would clear the other's)
  std::vector<std::pair<hipStream_t, u64*>> set_words;
  int ring_next = 0;
  uint64_t ticket_next = 0;
  // tickets of ring entries whose launch failed after their tickets were handed out: a wait that
  // covers one returns the failure (once)
  struct Failed {
    uint64_t lo, hi;
    int rc;
  };
  std::vector<Failed> failed;
  u64* h_hint = nullptr;  // host-mapped: unordered-tail size of the last push (written by push_apply)
  u64* d_hint = nullptr;
  // the hints as of the shard's last sync point (glint_shard_sync, the end of a host call): what the
  // adaptive tail switch and the binned front end decide from, so a given sequence of calls and
  // syncs takes the same path every run
  u64 hint_tail = 0;  // h_hint[0]
  u64 hint_bin = 0;   // h_hint[1]
  u64 hint_bin_cold = 0;  // h_hint[2]
  u64 hint_head = 0;  // h_hint[3]: where the last push's unordered tail started (records before it were ordered)
  u32 whole_probe = 0;  // whole-push scatters so far (every 8th is checked: launch_push)
  int hint_bin_front = -1;  // the front end of the binned push that wrote hint_bin (-1: none yet)
  i64 last_bad = -1;
  // ordering of host-pointer calls (private stream) after device-resident calls (caller's stream):
  // the last stream a *_dev call used; a host call records an event there and waits on it
  hipStream_t last_dev_stream = nullptr;
  bool dev_dirty = false;
  hipEvent_t order_ev = nullptr;
  // kernel timing (glint_prof_*): HIP event pairs recorded on the launch stream, summed lazily
  bool prof = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_ev[GLINT_K_COUNT];
  double prof_ms[GLINT_K_COUNT] = {0};
  int64_t prof_n[GLINT_K_COUNT] = {0};
  // host-side time accounting (GLINT_HOST_PROF=1, read at create; printed to stderr at destroy as
  // one "glint_host_prof {...}" line): what the message path's calls spend where
  bool hprof = false;
  struct HostProf {
    std::atomic<u64> lock_wait{0}, lock_hold{0}, nlock{0};  // ns waiting for / holding mu
    std::atomic<u64> launch{0}, nlaunch{0};                   // ns inside kernel launches
    std::atomic<u64> retire_wait{0}, nretire_wait{0};         // ns waiting for an entry to retire
    std::atomic<u64> copy{0};                                  // ns copying answers out of ring slots
  } hp;
  // slabs (glint_shard_create_in): a view's elements live inside its slab's allocation (not owned);
  // the slab lists its views (under its mu) so that its device-resident calls are ordered after the
  // views' host-pointer work and the views' later host-pointer calls after them
  glint_shard* slab = nullptr;
  std::vector<glint_shard*> views;
  bool dying = false;  // a slab being destroyed: no new views
  std::mutex mu;
};

// The order a call that locks several shards takes their locks in: shards that are not views (slabs
// among them) before views, each group by address -- a slab's own device calls lock the slab, then
// each of its views (dev_order_after_host), so every caller takes a slab's lock before its views'.
inline void lock_order(std::vector<glint_shard*>& v) {
  std::sort(v.begin(), v.end(), [](const glint_shard* a, const glint_shard* b) {
    const bool va = a->slab != nullptr, vb = b->slab != nullptr;
    return va != vb ? vb : a < b;
  });
}

// ---- environment knobs ----------------------------------------------------------------------------
// Test and policy overrides (GLINT_BINNED, GLINT_BIN_FRONT, ...; DESIGN.md §8 lists them) are read once per
// generation, so the push paths that several actor threads reach never call getenv. A test that
// changes the environment between calls starts a new generation with glint_reload_env().
extern std::atomic<unsigned> g_env_gen;  // glint_gpu.hip

struct EnvKnob {
  const char* name;
  std::atomic<unsigned> gen{0};
  std::atomic<long long> val{0};
  explicit EnvKnob(const char* n) : name(n) {}
  // parse(getenv(name)) -- the string may be NULL -- cached until the next glint_reload_env()
  template <typename F>
  long long get(F parse) {
    const unsigned g = g_env_gen.load(std::memory_order_acquire);
    if (gen.load(std::memory_order_acquire) == g) return val.load(std::memory_order_relaxed);
    const long long v = parse(getenv(name));
    val.store(v, std::memory_order_relaxed);
    gen.store(g, std::memory_order_release);
    return v;
  }
  // an integer knob: its value if set to a positive integer, else dflt
  long long pos_or(long long dflt) {
    return get([dflt](const char* e) { return (e && atoll(e) > 0) ? atoll(e) : dflt; });
  }
};

namespace {

inline u64 host_ns() {
  return (u64)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

// The shard's lock (one message at a time per shard, as the actor); with GLINT_HOST_PROF it also
// accounts the time spent waiting for it and holding it.
struct ShardLock {
  glint_shard* s;
  u64 t1 = 0;
  explicit ShardLock(glint_shard* s_) : s(s_) {
    if (!s->hprof) {
      s->mu.lock();
      return;
    }
    const u64 t0 = host_ns();
    s->mu.lock();
    t1 = host_ns();
    s->hp.lock_wait.fetch_add(t1 - t0, std::memory_order_relaxed);
    s->hp.nlock.fetch_add(1, std::memory_order_relaxed);
  }
  ~ShardLock() {
    if (t1) s->hp.lock_hold.fetch_add(host_ns() - t1, std::memory_order_relaxed);
    s->mu.unlock();
  }
  ShardLock(const ShardLock&) = delete;
  ShardLock& operator=(const ShardLock&) = delete;
};

struct DeviceGuard {
  int prev = -1;
  bool ok = false;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

#define HIPCHK(x)                                   \
  do {                                              \
    hipError_t e_ = (x);                            \
    if (e_ != hipSuccess) {                         \
      (void)hipGetLastError();                      \
      return GLINT_EDEVICE;                         \
    }                                               \
  } while (0)

inline size_t dtype_size(int dt) { return (dt == GLINT_I32 || dt == GLINT_F32) ? 4 : 8; }
inline size_t pad256(size_t b) { return (b + 255) & ~(size_t)255; }
inline bool aligned(const void* p, size_t a) { return ((uintptr_t)p % a) == 0; }

inline int grow(void** buf, size_t* cap, size_t need) {
  if (*cap >= need) return GLINT_OK;
  if (*buf) (void)hipFree(*buf);
  *buf = nullptr;
  *cap = 0;
  size_t sz = std::max(need, (size_t)1 << 20);
  if (hipMalloc(buf, sz) != hipSuccess) {
    (void)hipGetLastError();
    *buf = nullptr;
    return GLINT_ENOMEM;
  }
  *cap = sz;
  return GLINT_OK;
}

// pinned host buffer, grow-only (hipHostFree of the old one after the caller's stream sync)
inline int grow_pinned(void** buf, size_t* cap, size_t need) {
  if (*cap >= need) return GLINT_OK;
  if (*buf) (void)hipHostFree(*buf);
  *buf = nullptr;
  *cap = 0;
  size_t sz = (size_t)1 << 20;
  while (sz < need) sz <<= 1;
  if (hipHostMalloc(buf, sz, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    *buf = nullptr;
    return GLINT_ENOMEM;
  }
  *cap = sz;
  return GLINT_OK;
}

// device-resident calls run on the caller's stream exactly as given (NULL = the HIP null stream,
// as in every HIP API), so they order with the caller's producers and consumers of the buffers
inline hipStream_t pick(glint_shard* s, void* stream) {
  s->last_dev_stream = (hipStream_t)stream;
  s->dev_dirty = true;
  return (hipStream_t)stream;
}

// A host-pointer call runs on the shard's private stream: it first waits for everything the
// caller has enqueued on the last device-resident call's stream (that call's kernels share the
// shard's data, control words and error state with this one).
// A slab with views (glint_shard_create_in) takes device-resident calls only: host-pointer work on
// its private stream would not be ordered with the views' (they take that traffic). Under s->mu.
inline int refuse_slab(const glint_shard* s) { return s->views.empty() ? GLINT_OK : GLINT_EINVAL; }

inline int order_after_dev(glint_shard* s) {
  if (!s->dev_dirty) return GLINT_OK;
  if (!s->order_ev && hipEventCreateWithFlags(&s->order_ev, hipEventDisableTiming) != hipSuccess) {
    (void)hipGetLastError();
    return GLINT_EDEVICE;
  }
  if (hipEventRecord(s->order_ev, s->last_dev_stream) != hipSuccess ||
      hipStreamWaitEvent(s->stream, s->order_ev, 0) != hipSuccess) {
    (void)hipGetLastError();
    return GLINT_EDEVICE;
  }
  s->dev_dirty = false;
  return GLINT_OK;
}

// Brackets one kernel launch with events on its stream when profiling is on.
struct ProfScope {
  glint_shard* s;
  int id;
  hipStream_t st;
  hipEvent_t b = nullptr, e = nullptr;
  ProfScope(glint_shard* s_, int id_, hipStream_t st_) : s(s_), id(id_), st(st_) {
    if (!s->prof) return;
    if (hipEventCreate(&b) != hipSuccess || hipEventCreate(&e) != hipSuccess) {
      (void)hipGetLastError();
      b = e = nullptr;
      return;
    }
    (void)hipEventRecord(b, st);
  }
  ~ProfScope() {
    if (!b) return;
    (void)hipEventRecord(e, st);
    s->prof_ev[id].emplace_back(b, e);
  }
};

// Launches one kernel. With profiling on, its start/stop events ride on the kernel's own dispatch
// packet (hipExtLaunchKernel), so timing adds no marker packets and no gaps to the stream; a
// bracketing hipEventRecord pair costs ~8 us of stream time per kernel here.
template <typename... KArgs, typename... Args>
inline hipError_t launch_k(glint_shard* s, int id, void (*kernel)(KArgs...), unsigned grid, unsigned block,
                           hipStream_t st, Args... args) {
  hipEvent_t b = nullptr, e = nullptr;
  if (s->prof && (hipEventCreate(&b) != hipSuccess || hipEventCreate(&e) != hipSuccess)) {
    (void)hipGetLastError();
    b = e = nullptr;
  }
  const u64 t0 = s->hprof ? host_ns() : 0;
  hipExtLaunchKernelGGL(kernel, dim3(grid), dim3(block), 0, st, b, e, 0, static_cast<KArgs>(args)...);
  const hipError_t err = hipGetLastError();
  if (t0) {
    s->hp.launch.fetch_add(host_ns() - t0, std::memory_order_relaxed);
    s->hp.nlaunch.fetch_add(1, std::memory_order_relaxed);
  }
  if (b) s->prof_ev[id].emplace_back(b, e);
  return err;
}

inline void prof_drain(glint_shard* s) {
  for (int k = 0; k < GLINT_K_COUNT; ++k) {
    for (auto& pr : s->prof_ev[k]) {
      float ms = 0.f;
      if (hipEventSynchronize(pr.second) == hipSuccess && hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) {
        s->prof_ms[k] += ms;
        s->prof_n[k] += 1;
      }
      (void)hipEventDestroy(pr.first);
      (void)hipEventDestroy(pr.second);
    }
    s->prof_ev[k].clear();
  }
  (void)hipGetLastError();
}

// At a sync point (the stream that carried the shard's pushes has drained): the hint words the last
// push wrote become the ones the next pushes decide from.
inline void latch_hints(glint_shard* s) {
  if (!s->h_hint) return;
  s->hint_tail = __atomic_load_n(s->h_hint, __ATOMIC_ACQUIRE);
  s->hint_bin = __atomic_load_n(s->h_hint + 1, __ATOMIC_ACQUIRE);
  s->hint_bin_cold = __atomic_load_n(s->h_hint + 2, __ATOMIC_ACQUIRE);
  s->hint_head = __atomic_load_n(s->h_hint + 3, __ATOMIC_ACQUIRE);
  s->hint_bin_front = s->bin_last_front;  // the stream has drained: the hint is the last binned push's
}

// The error state a launch of this call records into: a host-pointer call's own, or the one
// glint_shard_sync reports for device-resident calls.
inline ErrState* err_of(const glint_shard* s) { return s->host_call ? s->d_err_host : s->d_err; }

// Marks the launches of a host-pointer call (their rejected records are the call's own errors).
struct HostCall {
  glint_shard* s;
  explicit HostCall(glint_shard* s_) : s(s_) { s->host_call = true; }
  ~HostCall() { s->host_call = false; }
};

inline unsigned grid_for(i64 units, i64 per_block, i64 cap) {
  i64 g = (units + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// resident blocks per CU for a kernel (occupancy query, once per kernel), capped at the measured best
template <auto Kernel>
inline int blocks_per_cu(int cap) {
  static std::atomic<int> occ{0};  // one per kernel
  int b = occ.load(std::memory_order_relaxed);
  if (!b) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, Kernel, kTPB, 0) != hipSuccess || b < 1) {
      (void)hipGetLastError();
      b = 2;
    }
    occ.store(b, std::memory_order_relaxed);
  }
  return std::min(b, cap);
}

}  // namespace

namespace glint {
// sort-based tails of a push (glint_sort.hip), instantiated for V in {int, long long, float, double}
// and MAT in {false, true}
template <typename V, bool MAT>
int push_det_tail(glint_shard* s, const PushArgs<V>& a, bool from_break, hipStream_t st);
// Work a caller slots into a binned push right after its count pass, given the push's [BinCtl | T]
// header (the validating gated push: its verdict, cancel and head apply; see push_binned_v2)
typedef std::function<int(void* bc, u32* T, u32 nb)> BinHook;
template <typename V, bool MAT>
int push_binned(glint_shard* s, const PushArgs<V>& a, bool from_break, hipStream_t st, const BinHook* hook = nullptr,
                LaunchCtl* whole_next = nullptr);
// whole_next: a whole-push bin (from_break false, no push_check ran): bin_count zeroes this LaunchCtl slot
// for the next push as push_check would, and reports through the hint words whether the push was ordered.
// whether a push of n records can be binned (u32 record indices and element addresses)
bool push_binnable(const glint_shard* s, i64 n);
// the verdict of a validating gated push whose tail is binned (glint_bin.hip)
int launch_validate_gate_binned(LaunchCtl* ctl, u64* gate, void* bc, u32* T, u32 nb, hipStream_t st);
// one-launch order-preserving push (glint_ordered.hip): n <= kOrderedMax, elems < 2^32
template <typename V, bool MAT>
int push_ordered(glint_shard* s, const PushArgs<V>& a, hipStream_t st);
}  // namespace glint
