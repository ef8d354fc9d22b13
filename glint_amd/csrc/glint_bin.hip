// glint_bin.hip -- the binned push: large unordered pushes summed per shard slab in LDS, with no
// per-record device atomics, no sort library and no host round trip (every size and count stays on
// the device). PartialVector.update / PartialMatrix.update (src/main/scala/glint/models/server/
// PartialVector.scala:35-43, PartialMatrix.scala:74-83) for records in no particular order.
//
// A slab is 4096 consecutive shard elements: the unit one workgroup sums in LDS. Records are moved
// into slab order by a two-level MSD partition on the slab index -- a coarse digit (<= 1024
// buckets) and a fine digit (<= 1024 slabs per bucket) -- and each slab's records are then summed
// in LDS and written back with one coalesced read-modify-write of the touched element pairs.
// Nothing is reserved across workgroups at run time: every writer owns its output range.
//
//   bin_part    per 4096- or 8192-record chunk c of the tail (optionally after summing duplicate
//               elements in an LDS hash table): the chunk's records ranked by bucket in LDS and stored
//               to the chunk's own range of the partition buffer (u32 address + value), grouped by
//               bucket, with the chunk's column of the chunk table ct[b][c] (run start | length). No
//               count pass: every chunk's output is one contiguous range.
//   bin_scan    per bucket: its chunk prefixes P[b][c] and places Q[b][c] (record v of the bucket is at
//               Q[b][c] + v), its total, output range and fine items (each with the chunks of its first
//               and last records).
//   bin_fsort   per fine item (<= 12288 records of one bucket, gathered from its chunks' runs): ranked by
//               slab in LDS and written slab-sorted (u16 slab offset + value) to the item's own range,
//               with the item's per-slab offsets (off2).
//   bin_plan    per bucket: every slab's runs (one per item) cut into apply units (fused into
//               bin_fsort for small pushes).
//   bin_apply2  per apply unit: LDS accumulation of the slab, coalesced RMW of the touched lines
//               (units of a slab cut into several flush with device atomics instead).
// Record indices are u32 (a push of < 2^32 records); a partition chunk's stores go through a buffer
// window at its own range, and the fine sort's gathers are 64-bit addressed, so buffers may pass 4 GiB.
#include "glint_device.h"
#include "glint_host.h"

#include <atomic>
#include <cstring>
#include <type_traits>

namespace glint {

#ifndef GLINT_SLAB_BITS
#define GLINT_SLAB_BITS 12
#endif
constexpr int kSlabBits = GLINT_SLAB_BITS;  // (a build-time experiment knob; 12 = 32 KiB of Double per slab)
constexpr int kSlab = 1 << kSlabBits;
constexpr int kMaxDigit = 1024;        // coarse buckets and fine slabs per bucket, at most
#ifndef GLINT_PART_TPB
#define GLINT_PART_TPB 1024
#endif
constexpr int kATPB = GLINT_PART_TPB;  // partition workgroup size (build-time knob: 1024 or 512)
#ifndef GLINT_PART_PER
#define GLINT_PART_PER 4
#endif
constexpr int kAPer = GLINT_PART_PER;  // records per thread per chunk (build-time knob)
#ifndef GLINT_PART_PER_PLAIN
#define GLINT_PART_PER_PLAIN 8
#endif
// The plain front end of a large push takes chunks of 8 records per thread (no hot or dedup table
// beside its staging in LDS): runs of 64 records per bucket and half the barriers per record. Same box,
// two rounds (profiles/r06/ab_part_per_plain.txt): cfg4b 2.20 -> 2.16 ms; cfg5 (a small push) 0.311 ->
// 0.314, so a small push keeps 4
constexpr int kAPerPlain = GLINT_PART_PER_PLAIN;
constexpr int kAChunk = kATPB * kAPer; // records per partition chunk (and dedup table fill)
constexpr int kASlots = 2 * kAChunk;   // dedup hash slots (load <= 0.5)
constexpr int kASlotBits = kASlots == 8192 ? 13 : kASlots == 4096 ? 12 : 11;
static_assert((1 << kASlotBits) == kASlots, "dedup table size");
// partition workgroups per CU: LDS-bound (the dedup table; the plain front end's staging)
constexpr int kPartWgPerCuDedup = kATPB == 1024 ? 1 : 2;
#ifndef GLINT_PART_WPC
#define GLINT_PART_WPC (kATPB == 1024 ? 1 : 2)
#endif
#ifndef GLINT_PART_AHEAD
#define GLINT_PART_AHEAD 2
#endif
constexpr int kPartAhead = GLINT_PART_AHEAD;  // partition chunks in flight per workgroup (build-time knob)
constexpr int kPartWgPerCuPlain = GLINT_PART_WPC;  // what fits (VGPRs): a second round of
                                                           // workgroups measured 3-9 % slower
#ifndef GLINT_APPLY_TPB
#define GLINT_APPLY_TPB 256
#endif
constexpr int kCTPB = GLINT_APPLY_TPB;  // slab-apply workgroup size (build-time knob)
constexpr u32 kEmptySlot = 0xFFFFFFFFu;

struct BinGeom {
  u32 fb;     // fine digit bits
  u32 nb;     // coarse buckets (power of two)
  u32 nf;     // fine slabs per bucket (power of two)
  u32 nslab;  // nb * nf
};
__device__ __forceinline__ u32 bucket_of(u32 a, const BinGeom& g) { return a >> (kSlabBits + g.fb); }
__device__ __forceinline__ u32 fine_of(u32 a, const BinGeom& g) { return (a >> kSlabBits) & (g.nf - 1); }

struct BinCtl {
  u32 m;       // records the partition emitted (after dedup)
  u32 tail;    // valid records in the tail
  u32 nfitems; // fine items (written by bin_part's workgroup 0)
  u32 cold;    // valid records that were not hot (the dedup front end's input; m for the others)
  u32 nunits;  // apply units written by bin_plan (each bucket takes its range with one atomic)
  u32 disorder;  // a whole-push bin (no push_check): some wave saw two adjacent records out of order
  u32 rbase;   // bin_scan: records of the buckets placed so far (each bucket takes its range with one atomic)
  u32 nch;     // bin_scan: partition chunks of the tail
};

// Phase timing for tuning (tools/bin_phases.py): built with -DGLINT_BIN_PROF, thread 0 of every
// workgroup sums clock64() deltas per phase into g_bin_prof; the product build compiles it away.
#ifdef GLINT_BIN_PROF
__device__ unsigned long long g_bin_prof[64];
struct PhaseClock {  // slots base .. base + 11 of g_bin_prof
  u64 last, acc[12];
  int base;
  __device__ explicit PhaseClock(int b) : last((u64)clock64()), base(b) {
    for (int i = 0; i < 12; ++i) acc[i] = 0;
  }
  __device__ void mark(int slot) {  // scheduling barriers: the clock read stays where it is written
    __builtin_amdgcn_sched_barrier(0);
    const u64 t = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
    if (threadIdx.x == 0) {
      acc[slot - base] += t - last;
      last = t;
    }
  }
  __device__ void flush(int n) {
    if (threadIdx.x != 0) return;
    for (int i = 0; i < n; ++i) atomicAdd(&g_bin_prof[base + i], acc[i]);
  }
};
#else
struct PhaseClock {
  __device__ explicit PhaseClock(int) {}
  __device__ void mark(int) {}
  __device__ void flush(int) {}
};
#endif

// Streaming inputs (records read once by a pass) load non-temporally (GLINT_BIN_NT, default 1), so
// they do not evict the partially written output runs and slab lines the passes revisit. Same box,
// two runs each (profiles/r03/ab_nt.txt): cfg3 1.43-1.50 -> 1.33-1.40 ms, cfg4b exchange -2-4 %.
// The intermediates (the partition's output read by bin_fsort, the fine sort's read by bin_apply2) load
// cached (GLINT_BIN_NT_MID=0): a slab's runs are gathered from every item of its bucket, and the lines
// two neighbouring runs share stay in L2 for the unit of the next slab (XCD-grouped unit order). Same box,
// two rounds (profiles/r06/ab_nt_mid.txt), with the per-push fine item size below: cfg4b exchange 2.42 ms
// non-temporal -> 2.20 cached (round 5: 2.37), cfg3 1.055 -> 1.046, cfg5 0.318 -> 0.315.
// (build-time knobs: GLINT_BIN_NT for the push's own records, read by bin_part;
// GLINT_BIN_NT_MID for the intermediates)
#ifndef GLINT_BIN_NT
#define GLINT_BIN_NT 1
#endif
#ifndef GLINT_BIN_NT_MID
#define GLINT_BIN_NT_MID 0
#endif
template <typename T>
__device__ __forceinline__ T ld_in(const T* p) {
#if GLINT_BIN_NT
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}
template <typename T>
__device__ __forceinline__ T ld_mid(const T* p) {
#if GLINT_BIN_NT_MID
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}

// ---- counted memory operations --------------------------------------------------------------------
// On gfx9 loads and stores share one counter (vmcnt), and the compiler can keep loads of a later
// chunk in flight across a wait only if every path issues the same number of memory instructions.
// So the hot loops have no data-dependent stores: a lane with nothing to store writes through a
// buffer descriptor at an out-of-range offset, which the buffer unit drops, and rejected records
// are counted in registers and reported once at the end instead of by an atomic per record.
typedef u32 v2u32 __attribute__((ext_vector_type(2)));
struct BufOut {
  __amdgpu_buffer_rsrc_t r;
  u32 oob;  // the descriptor's size: a store at this offset is dropped
};
// base and bytes must be workgroup-uniform; readfirstlane makes that provable to the compiler, which
// otherwise wraps every buffer store in a waterfall loop
__device__ __forceinline__ BufOut buf_out(const void* base, u32 bytes) {
  const u64 b = (u64)base;
  const u32 lo = __builtin_amdgcn_readfirstlane((u32)b), hi = __builtin_amdgcn_readfirstlane((u32)(b >> 32));
  const u32 nb = __builtin_amdgcn_readfirstlane(bytes);
  void* p = (void*)(((u64)hi << 32) | lo);
  return BufOut{__builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)nb, 0x00020000), nb};
}
template <typename T>
__device__ __forceinline__ void bput(const BufOut& b, u32 off, bool on, T v) {
  const int o = (int)(on ? off : b.oob);
  if constexpr (sizeof(T) == 4) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(u32, v), b.r, o, 0, 0);
  } else {
    static_assert(sizeof(T) == 8, "4- or 8-byte stores");
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u32, v), b.r, o, 0, 0);
  }
}
// A load through a buffer window: 0 past its end (no memory access), non-temporal as ld_mid
template <typename T>
__device__ __forceinline__ T bget(const BufOut& b, u32 off) {
  constexpr int kAux = GLINT_BIN_NT_MID ? 2 : 0;  // gfx950 buffer cache policy: bit 1 = nt
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(b.r, (int)off, 0, kAux));
  } else {
    static_assert(sizeof(T) == 8, "4- or 8-byte loads");
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(b.r, (int)off, 0, kAux));
  }
}
__device__ __forceinline__ void bput16(const BufOut& b, u32 off, bool on, uint16_t v) {
  __builtin_amdgcn_raw_buffer_store_b16(v, b.r, (int)(on ? off : b.oob), 0, 0);
}
// A record array of T through one buffer window: element `rel` at byte rel * sizeof(T) (< 2^32 bytes).
template <typename T>
struct RecOut {
  BufOut b;
  __device__ __forceinline__ void put(u32 rel, bool on, T v) const { bput(b, rel * (u32)sizeof(T), on, v); }
};
struct BadRecs {  // this thread's rejected records: the first one and how many
  i64 first = -1;
  u32 count = 0;
  __device__ void add(i64 i) {
    first = count ? min(first, i) : i;
    ++count;
  }
  __device__ void report(ErrState* err) const {
    if (count) {
      atomicMax(&err->min_bad_enc, ~(u64)first);
      atomicAdd(&err->count, (unsigned long long)count);
    }
  }
};

// ---- block-level helpers ------------------------------------------------------------------------
// The per-wave totals of a workgroup (wt[0..NW), NW <= 16 waves): lane l < NW reads wt[l], an inclusive
// scan across the lanes of the first DPP row (row_shr 1, 2, 4, 8: register-to-register, no LDS round
// trip) -> the waves before wave `wid` (exclusive) and all of them, both workgroup-uniform. Two registers,
// one LDS read.
template <int NW>
__device__ __forceinline__ void wave_totals(const u32* wt, int lane, int wid, u32& pre, u32& tot) {
  static_assert(NW >= 1 && NW <= 16, "one DPP row");
  u32 x = lane < NW ? wt[lane] : 0u;
  x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  if (NW > 2) x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  if (NW > 4) x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  if (NW > 8) x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  const int w = __builtin_amdgcn_readfirstlane(wid);
  pre = w > 0 ? (u32)__builtin_amdgcn_readlane((int)x, w - 1) : 0u;
  tot = (u32)__builtin_amdgcn_readlane((int)x, NW - 1);
}

// Exclusive scan over N values by one workgroup of TPB threads, in tiles of TPB x PER: each thread
// loads a run of PER values into registers (all loads in flight together), scans them and calls
// write(i, exclusive prefix) once per i. Returns the total.
template <int TPB, int PER, typename F, typename W>
__device__ __forceinline__ u32 block_scan(u32 N, F value, W write) {
  __shared__ u32 wt[TPB / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  u32 carry = 0;
  for (u32 base = 0; base < N; base += (u32)TPB * PER) {
    const u32 b0 = base + (u32)tid * PER;
    u32 v[PER];
    u32 s = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      v[j] = b0 + j < N ? value(b0 + j) : 0u;
      s += v[j];
    }
    u32 incl = s;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const u32 y = __shfl_up(incl, d);
      if (lane >= d) incl += y;
    }
    if (lane == 63) wt[wid] = incl;
    __syncthreads();
    u32 pre, tot;  // the waves before this one and all of them
    wave_totals<TPB / 64>(wt, lane, wid, pre, tot);
    u32 run = carry + incl - s + pre;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (b0 + j < N) write(b0 + j, run);
      run += v[j];
    }
    carry += tot;
    __syncthreads();
  }
  return carry;
}

template <int TPB>
__device__ __forceinline__ u32 block_sum(u32 x) {
  __shared__ u32 ws[TPB / 64];
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = x;
  __syncthreads();
  u32 pre, t;
  wave_totals<TPB / 64>(ws, threadIdx.x & 63, threadIdx.x >> 6, pre, t);
  __syncthreads();
  return t;
}

template <int TPB>
__device__ __forceinline__ u32 block_max(u32 x) {
  __shared__ u32 wm[TPB / 64];
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) x = max(x, (u32)__shfl_xor(x, d));
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = x;
  __syncthreads();
  u32 m = 0;
  for (int w = 0; w < TPB / 64; ++w) m = max(m, wm[w]);
  __syncthreads();
  return m;
}

// from_break: 0 the whole push; 1 from push_check's break; 2 the whole push unless its gate cancelled it
// (a validating whole-push bin: the kernels after its verdict see an empty tail, as a cancelled break)
__device__ __forceinline__ i64 tail_start(const LaunchCtl* lctl, u32 ntiles, int from_break, i64 n) {
  if (!from_break) return 0;
  if (from_break == 2) return lctl->cancel ? n : 0;
  const u32 brk = lctl->brk_enc;  // written by push_check; ordered by the kernel boundary
  return brk == 0u ? n : (i64)(ntiles - brk) * kTile;
}

// One partition chunk's records, kAPer per thread, in registers. The partition kernels keep two of
// these in flight (chunks c + G and c + 2G load while chunk c is partitioned): one chunk of loads per
// workgroup left too little in flight per CU to cover HBM latency.
template <typename V, bool MAT, int PER = kAPer>
struct RecRegs {
  i64 k[PER];
  int32_t cl[PER];
  V v[PER];
};

template <typename V, bool MAT, bool VALS = true, int PER = kAPer>
__device__ __forceinline__ void load_recs(const i64* __restrict__ keys, const int32_t* __restrict__ cols,
                                          const V* __restrict__ vals, i64 c0, i64 c1, RecRegs<V, MAT, PER>& r) {
#pragma unroll
  for (int q = 0; q < PER; ++q) {  // clamped, branch-free loads
    const i64 i = c0 + q * kATPB + threadIdx.x;
    const i64 ii = i < c1 ? i : c1 - 1;
    r.k[q] = ld_in(keys + ii);
    r.cl[q] = MAT ? ld_in(cols + ii) : 0;
    if (VALS) r.v[q] = ld_in(vals + ii);
  }
}

// KIND: the partition layout (0 range, -1 read at run time), as push_check is specialised
__device__ __forceinline__ u32 hot_mix(u32 x) {  // murmur3 fmix32
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}

constexpr int kWideSlots = 8192;  // the plain + hot front end's hot table (see bin_hot_select)
__device__ __forceinline__ u32 wide_slot(u32 a) { return hot_mix(a) & (kWideSlots - 1); }
// The verdict of a validating gated push whose tail is binned (after bin_part validated the tail and
// push_check the records before the break): 0 or ~(first rejected record) to the caller's gate word; a
// rejected batch is cancelled before anything is applied -- no head (push_apply sees cancel), no tail
// (the break is cleared / cancel set, so bin_scan sees an empty tail and every bucket empty, and
// bin_hot_reduce drops the partition's hot sums). T is zeroed here too (bin_scan rewrites it).
__global__ __launch_bounds__(256) void push_validate_gate_binned_kernel(LaunchCtl* ctl, u64* gate, BinCtl* bc,
                                                                        u32* __restrict__ T, u32 nb) {
  const u64 b = ctl->bad;
  if (b == 0ull) {
    if (threadIdx.x == 0) *gate = 0ull;
    return;
  }
  for (u32 x = threadIdx.x; x < nb; x += 256) T[x] = 0;
  if (threadIdx.x == 0) {
    *gate = b;
    ctl->cancel = 1u;
    ctl->brk_enc = 0u;
    bc->tail = 0u;
  }
}

// ---- hot elements ----------------------------------------------------------------------------------
// A Zipf-like tail sends its most frequent elements through every partition chunk: the dedup table
// merges them within a chunk, but each chunk still emits one record per hot element, and those
// records cross both partition levels and the apply. The hot elements are picked per push from a
// sample of the tail (bin_hot_pick) into a direct-mapped table of kHotSlots elements; the dedup
// front end sums their records in per-workgroup LDS accumulators over ALL its chunks and adds each
// sum to the shard once at the end (one device atomic per hot element per workgroup), so only the
// cold elements are partitioned. Any choice of hot set gives the same sums; the sample only decides
// how much work moves off the partition path.
constexpr int kHotSlots = 2048;     // direct-mapped hot table (per dedup workgroup: tags + sums in LDS)
constexpr int kHotSample = 16384;   // records sampled per push, as kHotRuns runs of kHotRun records
constexpr int kHotRun = 128;
constexpr int kHotRuns = kHotSample / kHotRun;
constexpr int kHotCount = 16384;    // sampler's LDS count table (load <= ~0.5: short probe chains)
constexpr int kHotTPB = 1024;

__device__ __forceinline__ u32 hot_slot(u32 a) { return hot_mix(a) & (kHotSlots - 1); }



// One workgroup: kHotSample records (kHotRuns runs spread evenly over the tail) are counted per
// element in LDS; every element seen at least min_count times (2: frequency >= ~2 / kHotSample of
// the tail) competes for its direct-mapped slot, the most frequent one wins. Writes hot_tags[kHotSlots] (kEmptySlot = none).
template <bool MAT>
__global__ __launch_bounds__(kHotTPB) void bin_hot_pick_kernel(const i64* __restrict__ keys,
                                                               const int32_t* __restrict__ cols, i64 n,
                                                               PartDesc part, const LaunchCtl* lctl, u32 ntiles,
                                                               int from_break, u32 min_count,
                                                               u32* __restrict__ hot_tags) {
  __shared__ u32 ck[kHotCount];
  __shared__ u32 cc[kHotCount];
  __shared__ unsigned long long best[kHotSlots];
  const int tid = threadIdx.x;
  for (int i = tid; i < kHotCount; i += kHotTPB) {
    ck[i] = kEmptySlot;
    cc[i] = 0;
  }
  for (int i = tid; i < kHotSlots; i += kHotTPB) best[i] = 0ull;
  __syncthreads();
  const i64 r0 = tail_start(lctl, ntiles, from_break, n);
  const i64 m = n - r0;
  if (m > 0) {
    // kHotRuns runs of kHotRun consecutive records, spread evenly over the tail: whole-line reads
    // (one workgroup reading 32768 scattered 8-B keys took ~150 us, bound by its lines in flight;
    // 32768 samples in this table took 87 us, bound by divergent probe chains at load ~0.75)
    const i64 ns = min((i64)kHotSample, m);
    const i64 run_stride = m >= (i64)kHotSample ? m / kHotRuns : kHotRun;  // a short tail: read it all
    auto rec_of = [&](i64 sidx) { return r0 + (sidx / kHotRun) * run_stride + (sidx % kHotRun); };
    constexpr int kBatch = 16;  // samples per thread whose loads are in flight together
    for (i64 s0 = 0; s0 < ns; s0 += (i64)kBatch * kHotTPB) {
      i64 k[kBatch];
      int32_t c[kBatch];
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {  // clamped, branch-free loads
        const i64 i = rec_of(min(s0 + (i64)j * kHotTPB + tid, ns - 1));
        k[j] = keys[i];
        c[j] = MAT ? cols[i] : 0;
      }
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {
        i64 a64;
        if (s0 + (i64)j * kHotTPB + tid >= ns || !rec_addr<MAT>(part, k[j], c[j], a64)) continue;
        const u32 a = (u32)a64;
        u32 h = hot_mix(a * 0x9E3779B1u) & (kHotCount - 1);
        for (int probe = 0; probe < 64; ++probe) {  // bounded: a full neighbourhood drops the sample
          const u32 prev = atomicCAS(&ck[h], kEmptySlot, a);
          if (prev == kEmptySlot || prev == a) {
            atomicAdd(&cc[h], 1u);
            break;
          }
          h = (h + 1) & (kHotCount - 1);
        }
      }
    }
  }
  __syncthreads();
  for (int h = tid; h < kHotCount; h += kHotTPB)
    if (cc[h] >= min_count) atomicMax(&best[hot_slot(ck[h])], ((unsigned long long)cc[h] << 32) | ck[h]);
  __syncthreads();
  for (int i = tid; i < kHotSlots; i += kHotTPB) hot_tags[i] = best[i] ? (u32)best[i] : kEmptySlot;
}

// a hot sum's initial value: adding it to the first record is exact (x + -0.0 == x), and a slot still
// holding it at the end got no record (or only -0.0 ones, which leave the element as it is)
template <typename A> __device__ __forceinline__ A hot_zero() { return A(0); }
template <> __device__ __forceinline__ double hot_zero<double>() { return -0.0; }
template <typename A> __device__ __forceinline__ bool hot_untouched(A x) { return x == A(0); }
template <> __device__ __forceinline__ bool hot_untouched<double>(double x) {
  return __double_as_longlong(x) == (long long)0x8000000000000000ull;
}
__device__ __forceinline__ void hot_flush(double* p, double x) { gadd(p, x); }
__device__ __forceinline__ void hot_flush(float* p, double x) { gadd(p, (float)x); }
__device__ __forceinline__ void hot_flush(long long* p, long long x) { gadd(p, x); }
__device__ __forceinline__ void hot_flush(int* p, int x) { gadd(p, x); }

// ---- bin_part -------------------------------------------------------------------------------------
// Chunk-local partition: chunk c of the tail (kChunk records) is written to the partition buffer's own
// range [c * kChunk, c * kChunk + total) with its records grouped by coarse bucket, and its column of
// the chunk table ct[b][c] = (where bucket b's run starts in the chunk) | (its length << 16). No count pass
// runs first: the stores are one contiguous range per chunk, and bin_scan turns the table into each
// bucket's chunk prefix afterwards. ad / va: P records per thread in registers, `valid` bit mask; dcnt
// and gcnt are scratch (dcnt zero on entry and exit). OA / OV: the chunk's output windows.
template <typename A, int P>
__device__ __forceinline__ u32 part_emit(const u32 (&ad)[P], const A (&va)[P], u32 valid, const BinGeom& g,
                                         u32* dcnt, u32* gcnt, u32* st_a, A* st_v, const BufOut& ctb, u32 ctcol,
                                         u32 ctstride, u32* __restrict__ out_a, A* __restrict__ out_v, PhaseClock& ph,
                                         int pb) {
  const int tid = threadIdx.x;
  u32 rank[P];
#pragma unroll
  for (int j = 0; j < P; ++j)
    if (valid & (1u << j)) rank[j] = atomicAdd(&dcnt[bucket_of(ad[j], g)], 1u);
  __syncthreads();
  ph.mark(pb);
  const u32 total = block_scan<kATPB, 1>(
      g.nb, [&](u32 d) { return dcnt[d]; },
      [&](u32 d, u32 excl) {
        gcnt[d] = dcnt[d];
        dcnt[d] = excl;
      });
  ph.mark(pb + 1);
  static_assert(kATPB <= kMaxDigit, "one chunk-table entry per thread");
  // the chunk's column of the table (bucket-major rows of ctstride): one counted store per thread
  bput(ctb, ((u32)tid * ctstride + ctcol) * 4u, (u32)tid < g.nb, dcnt[tid] | (gcnt[tid] << 16));
#pragma unroll
  for (int j = 0; j < P; ++j) {
    if (valid & (1u << j)) {
      const u32 p = dcnt[bucket_of(ad[j], g)] + rank[j];
      st_a[p] = ad[j];
      st_v[p] = va[j];
    }
  }
  __syncthreads();
  ph.mark(pb + 2);
  const RecOut<u32> oa{buf_out(out_a, total * 4u)};
  const RecOut<A> ov{buf_out(out_v, total * (u32)sizeof(A))};
#pragma unroll
  for (int j = 0; j < P; ++j) {  // consecutive threads: consecutive slots of the chunk's range
    if ((u32)(j * kATPB) >= total) break;  // workgroup-uniform: no store instructions past the chunk
    const u32 p = tid + j * kATPB;
    const bool on = p < total;
    oa.put(p, on, st_a[p]);
    ov.put(p, on, st_v[p]);
  }
  __syncthreads();
  ph.mark(pb + 3);
  for (u32 d = tid; d < g.nb; d += kATPB) dcnt[d] = 0;
  __syncthreads();
  ph.mark(pb + 4);
  return total;
}

// Workgroup 0 of the partition: the next push's header (the previous push used it; it is done) and,
// for a whole-push bin (no push_check ran), the next push's control words as push_check zeroes them.
__device__ __forceinline__ void part_next_header(const BinGeom& g, BinCtl* next_bc, u32* __restrict__ next_T,
                                                 LaunchCtl* next_ctl) {
  const int tid = threadIdx.x;
  for (u32 b = tid; b < kMaxDigit; b += kATPB) {  // (every slot: the next push may have more buckets)
    next_T[b] = 0;
    next_T[kMaxDigit + b] = 0;  // the fused plan's per-bucket item counters
  }
  if (tid < (int)(sizeof(BinCtl) / 4)) reinterpret_cast<u32*>(next_bc)[tid] = 0;
  if (next_ctl && tid == 0) {
    next_ctl->brk_enc = 0u;
    next_ctl->nonaffine = 0u;
    next_ctl->cancel = 0u;
    next_ctl->bad = 0ull;
  }
}

// fine items of a bucket of t records: ceil(t / item), at least one (an empty bucket's one item writes
// its empty offset row)
__device__ __forceinline__ u32 bucket_items(u32 t, u32 item) { return max(1u, (t + item - 1) / item); }

// The plain + hot front end keeps a wider hot table (kWideSlots tags + sums fit the plain partition
// kernel's LDS next to its staging). Its hot elements come from a sample 16x larger than
// bin_hot_pick's, counted in a global hash table by many workgroups (bin_hot_sample) and picked per
// slot by bin_hot_select; the partition workgroups' per-slot sums are stored (not added with atomics:
// kWideSlots x G of them would cost more than the split saves) and bin_hot_reduce adds each hot
// element's sum over the workgroups to the shard in workgroup order.
constexpr int kWideHashBits = 20;           // global count table: 2^20 slots
constexpr int kWideRunsPerWg = 8;           // sampled runs of kHotRun records per sampling workgroup
constexpr int kWideSampleWgs = 256;         // 256 x 8 x 128 = 262 144 sampled records per push

// Each workgroup reads kWideRunsPerWg runs of kHotRun consecutive records (spread evenly over the
// tail), counts them in LDS, then adds its (element, count) pairs to the global hash table.
template <bool MAT>
__global__ __launch_bounds__(256) void bin_hot_sample_kernel(const i64* __restrict__ keys, const int32_t* __restrict__ cols,
                                                             i64 n, PartDesc part, const LaunchCtl* lctl, u32 ntiles,
                                                             int from_break, u32* __restrict__ gkey,
                                                             u32* __restrict__ gcnt) {
  constexpr int kLocal = 2048;  // LDS count table (1024 samples per workgroup: load <= 0.5)
  __shared__ u32 lk[kLocal], lc[kLocal];
  const int tid = threadIdx.x;
  for (int i = tid; i < kLocal; i += 256) {
    lk[i] = kEmptySlot;
    lc[i] = 0;
  }
  __syncthreads();
  const i64 r0 = tail_start(lctl, ntiles, from_break, n);
  const i64 m = n - r0;
  const i64 runs = (i64)kWideSampleWgs * kWideRunsPerWg;
  if (m > 0) {
    const i64 stride = m >= runs * kHotRun ? m / runs : kHotRun;
    constexpr int kPer = kWideRunsPerWg * kHotRun / 256;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int s = j * 256 + tid;  // sample s of this workgroup: run s / kHotRun, offset s % kHotRun
      const i64 run = (i64)blockIdx.x * kWideRunsPerWg + s / kHotRun;
      const i64 i = r0 + run * stride + s % kHotRun;
      if (i >= n) continue;
      i64 a64;
      if (!rec_addr<MAT>(part, keys[i], MAT ? cols[i] : 0, a64)) continue;
      const u32 a = (u32)a64;
      u32 h = hot_mix(a * 0x9E3779B1u) & (kLocal - 1);
      for (int probe = 0; probe < 64; ++probe) {
        const u32 prev = atomicCAS(&lk[h], kEmptySlot, a);
        if (prev == kEmptySlot || prev == a) {
          atomicAdd(&lc[h], 1u);
          break;
        }
        h = (h + 1) & (kLocal - 1);
      }
    }
  }
  __syncthreads();
  constexpr u32 kMask = (1u << kWideHashBits) - 1u;
  for (int i = tid; i < kLocal; i += 256) {
    const u32 a = lk[i];
    if (a == kEmptySlot) continue;
    u32 h = hot_mix(a) & kMask;
    for (int probe = 0; probe < 64; ++probe) {
      const u32 prev = atomicCAS(&gkey[h], kEmptySlot, a);
      if (prev == kEmptySlot || prev == a) {
        atomicAdd(&gcnt[h], lc[i]);
        break;
      }
      h = (h + 1) & kMask;
    }
  }
}

// Every counted element with >= min_count samples competes for its wide slot; the most sampled wins
// (best[slot] = count << 32 | element; zeroed per push). The partition kernel reads the tags from it.
__global__ __launch_bounds__(256) void bin_hot_select_kernel(u32* __restrict__ gkey, u32* __restrict__ gcnt,
                                                             u32 min_count, unsigned long long* __restrict__ best) {
  const u32 i = blockIdx.x * 256u + threadIdx.x;
  const u32 a = gkey[i], c = gcnt[i];
  gkey[i] = kEmptySlot;  // the table's last reader empties it for the next push (no memset)
  gcnt[i] = 0;
  if (a != kEmptySlot && c >= min_count) atomicMax(&best[wide_slot(a)], ((unsigned long long)c << 32) | a);
}

// Each hot element's sum over the partition workgroups (partial[w][slot]), added to the shard once: a
// plain read-modify-write (the element's records all went to the hot sums, so no other kernel of the
// push touches it). A workgroup of kRedTPB threads takes kRedSlots slots; its kRedGroups lane groups
// each sum a contiguous range of workgroups (coalesced rows, loads issued back to back), then the
// group sums are added in group order -- the result is the same on every run.
constexpr int kRedSlots = 64, kRedTPB = 1024, kRedGroups = kRedTPB / kRedSlots;
// (the picks stay for the next pushes: push_binned clears them itself before it samples again)
// (run by bin_scan's workgroups past its buckets, blk = which kRedSlots slots: one launch fewer)
template <typename V>
__device__ __forceinline__ void hot_reduce_block(u32 blk, const unsigned long long* __restrict__ best, u32 G,
                                                 const typename LdsAcc<V>::T* __restrict__ partial,
                                                 V* __restrict__ data, const LaunchCtl* gated) {
  typedef typename LdsAcc<V>::T A;
  if (gated && gated->cancel) return;  // a validating push its verdict rejected: nothing is applied
  __shared__ A gs[kRedGroups][kRedSlots];
  __shared__ u32 gany[kRedGroups][kRedSlots];
  const int tid = threadIdx.x, ls = tid % kRedSlots, grp = tid / kRedSlots;
  const u32 sl = blk * (u32)kRedSlots + (u32)ls;
  const u32 per = (G + kRedGroups - 1) / kRedGroups;
  const u32 w0 = grp * per, w1 = min(G, w0 + per);
  A sum = hot_zero<A>();
  u32 any = 0;
  constexpr int kUnroll = 8;
  for (u32 w = w0; w < w1; w += kUnroll) {
    A x[kUnroll];
#pragma unroll
    for (int j = 0; j < kUnroll; ++j) x[j] = partial[(size_t)min(w + (u32)j, w1 - 1u) * kWideSlots + sl];
#pragma unroll
    for (int j = 0; j < kUnroll; ++j) {
      if (w + (u32)j < w1 && !hot_untouched<A>(x[j])) {
        sum = any ? vadd(sum, x[j]) : x[j];
        any = 1;
      }
    }
  }
  gs[grp][ls] = sum;
  gany[grp][ls] = any;
  __syncthreads();
  if (grp != 0) return;
  const unsigned long long b = best[sl];
  if (!b) return;
  A tot = hot_zero<A>();
  bool seen = false;
  for (int q = 0; q < kRedGroups; ++q) {
    if (!gany[q][ls]) continue;
    tot = seen ? vadd(tot, gs[q][ls]) : gs[q][ls];
    seen = true;
  }
  const u32 a = (u32)b;
  if (seen) data[a] = acc_add(data[a], tot);
}

// Plain front end: every valid record is appended as it is. HOT: the push's hot elements (the wide
// table, bin_hot_select) are summed in LDS over all of the workgroup's chunks and stored per
// workgroup for bin_hot_reduce; only the cold records are appended. Once the hot elements are off,
// a Zipf-like tail has almost no duplicates left inside a chunk (cfg3: the chunk dedup would merge
// 0.6 % of the cold records), so the hash table is not worth its time there.
// VALIDATE (a validating gated push, GLINT_PUSH_VALIDATE, whose tail is binned): every tail record is
// also checked -- the key itself in the partition's key range, as key_in_part -- and the first rejected
// one goes to the push's LaunchCtl (vctl->bad), as push_check does for the records before the break; the
// verdict and cancel come after this kernel (push_validate_gate_binned_kernel), before anything is
// applied (this kernel writes only the partition buffers and, HOT, its per-workgroup hot sums, which
// bin_hot_reduce drops for a cancelled push). next_ctl (a whole-push bin): workgroup 0 zeroes the next
// push's control words, and any wave that sees two adjacent records out of order says so (bc->disorder).
#ifndef GLINT_PART_WAVES
#define GLINT_PART_WAVES 4  // bin_part's register budget: waves per SIMD (build-time knob)
#endif
template <typename V, bool MAT, bool HOT, int KIND, bool VALIDATE, int PER = kAPer>
__global__ __launch_bounds__(kATPB) __attribute__((amdgpu_waves_per_eu(HOT ? 4 : GLINT_PART_WAVES))) void bin_part_kernel(
    const i64* __restrict__ keys, const int32_t* __restrict__ cols, const V* __restrict__ vals, i64 n, PartDesc part,
    const LaunchCtl* lctl, u32 ntiles, int from_break, BinGeom g, u32* __restrict__ addr_out,
    typename LdsAcc<V>::T* __restrict__ val_out, ErrState* err, BinCtl* bc, u32* __restrict__ ct, u32 ctstride,
    const unsigned long long* __restrict__ hot_best, typename LdsAcc<V>::T* __restrict__ hot_partial,
    BinCtl* next_bc, u32* __restrict__ next_T, LaunchCtl* vctl, LaunchCtl* next_ctl) {
  typedef typename LdsAcc<V>::T A;
  constexpr int kChunk = kATPB * PER;  // records per chunk
  __shared__ u32 dcnt[kMaxDigit], gcnt[kMaxDigit];
  __shared__ u32 st_a[kChunk];
  __shared__ A st_v[kChunk];
  constexpr int kHS = HOT ? kWideSlots : 1;
  __shared__ u32 htag[kHS];
  __shared__ A hacc[kHS];
  const int tid = threadIdx.x;
  const u32 w = blockIdx.x;
  const i64 r0 = tail_start(lctl, ntiles, from_break, n);
  const i64 nchunks = (n - r0 + kChunk - 1) / kChunk;
  // chunks in flight: the hot front end runs one workgroup per CU (its LDS tables), two chunks ahead;
  // the plain one kPartAhead
  constexpr int kAhead = HOT ? 2 : kPartAhead;
  if constexpr (HOT) {
    for (int sl = tid; sl < kWideSlots; sl += kATPB) {
      const unsigned long long b = hot_best[sl];
      htag[sl] = b ? (u32)b : kEmptySlot;
      hacc[sl] = hot_zero<A>();
    }
  }
  for (u32 d = tid; d < g.nb; d += kATPB) dcnt[d] = 0;
  if (w == 0) part_next_header(g, next_bc, next_T, next_ctl);
  __syncthreads();
  PhaseClock ph(0);
  const i64 G = gridDim.x;
  const BufOut ctb = buf_out(ct, g.nb * ctstride * 4u);  // (< 2^32 bytes: push_binnable)
  BadRecs bad;
  u32 emitted = 0;
  bool dis = false;  // (a whole-push bin) two adjacent records of one wave out of order
  // chunk loads are unconditional (index clamped; a step past the end sees no valid record), so the
  // compiler can wait for one chunk's loads while the next chunk's stay in flight
  auto load_chunk = [&](i64 c, RecRegs<V, MAT, PER>& r) {
    const i64 cc = min(c, nchunks - 1);
    const i64 c0 = r0 + cc * kChunk, c1 = min(n, r0 + (cc + 1) * kChunk);
    if constexpr (KIND == 0 && !VALIDATE) {  // (key - start).toInt needs the low words only
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const i64 i = c0 + q * kATPB + threadIdx.x;
        const i64 ii = i < c1 ? i : c1 - 1;
        r.k[q] = (i64)(u64)ld_in(reinterpret_cast<const u32*>(keys) + 2 * ii);
        r.cl[q] = MAT ? ld_in(cols + ii) : 0;
        r.v[q] = ld_in(vals + ii);
      }
    } else {
      load_recs<V, MAT, true, PER>(keys, cols, vals, c0, c1, r);
    }
  };
  auto step = [&](i64 c, RecRegs<V, MAT, PER>& r) {
    const i64 c0 = r0 + c * kChunk, c1 = c < nchunks ? min(n, c0 + kChunk) : c0;
    u32 ad[PER];
    A va[PER];
    u32 valid = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const i64 i = c0 + q * kATPB + tid;
      const bool in = i < c1;
      i64 a64;
      bool ok = in && rec_addr<MAT, KIND>(part, r.k[q], r.cl[q], a64);
      if constexpr (VALIDATE) ok = ok && key_in_part<KIND>(part, r.k[q]);
      ad[q] = ok ? (u32)a64 : 0u;
      va[q] = (A)r.v[q];
      if (ok) valid |= 1u << q;
      else if (in) bad.add(i);
      if (next_ctl && q == 0) {  // a wave's records are consecutive: are they strictly increasing? (one
        // record per thread per chunk is sample enough: an unordered push shows it in every wave, a sorted
        // one nowhere; a record before this one is in the push whenever this one is)
        const u32 a32 = ok ? (u32)a64 : 0xFFFFFFFFu, prev = __shfl_up(a32, 1);
        dis = dis || (in && (!ok || ((threadIdx.x & 63) && prev >= a32)));
      }
    }
    if constexpr (HOT) {
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const u32 hs = wide_slot(ad[q]);
        if ((valid & (1u << q)) && htag[hs] == ad[q]) {  // hot: summed over all of this workgroup's chunks
          lds_add(&hacc[hs], va[q]);
          valid &= ~(1u << q);
        }
      }
    }
    ph.mark(1);
    const i64 cs = c < nchunks ? c : 0;  // (a step past the end emits nothing: its table row and stores land
    // on chunk 0's, all of them dropped -- total 0 -- but its table column, which would overwrite chunk
    // 0's: past the end the column goes to the spare one at nchunks instead)
    const u32 crow = (u32)(c < nchunks ? c : nchunks);
    emitted += part_emit<A, PER>(ad, va, valid, g, dcnt, gcnt, st_a, st_v, ctb, crow, ctstride,
                                 addr_out + (size_t)cs * kChunk, val_out + (size_t)cs * kChunk, ph, 3);
    // kAhead chunks ahead, into the registers just consumed: in flight across the next chunks' work
    load_chunk(c + kAhead * G, r);
    ph.mark(2);
  };
  RecRegs<V, MAT, PER> r[kAhead];
  i64 c = w;
  if (c < nchunks) {
#pragma unroll
    for (int j = 0; j < kAhead; ++j) load_chunk(c + j * G, r[j]);
    for (; c < nchunks; c += kAhead * G) {
#pragma unroll
      for (int j = 0; j < kAhead; ++j) step(c + j * G, r[j]);  // past the end: no valid record
    }
  }
  if (tid == 0 && emitted) {  // (emitted is workgroup-uniform: the sum of the chunks' totals)
    atomicAdd(&bc->m, emitted);
    atomicAdd(&bc->cold, emitted);  // cold records: all of them were appended
    atomicAdd(&bc->tail, emitted);  // valid records of the tail (the hot front end's hot ones not counted)
  }
  if (next_ctl && __syncthreads_or(dis) && tid == 0) atomicOr(&bc->disorder, 1u);
  if constexpr (VALIDATE) {
    if (bad.count) atomicMax(&vctl->bad, ~(u64)bad.first);  // rare: one atomic per thread
  } else {
    bad.report(err);
  }
  if constexpr (HOT) {
    __syncthreads();  // every chunk's hot sums are in; bin_hot_reduce adds them up
    for (int sl = tid; sl < kWideSlots; sl += kATPB) hot_partial[(size_t)w * kWideSlots + sl] = hacc[sl];
  }
  ph.flush(8);
}

// Dedup front end for duplicate-heavy tails: per chunk, equal elements are summed in an LDS hash
// table first, so one record per distinct element of the chunk moves on. The staging buffer of the
// append overlays the table's value array. Records of the push's hot elements (hot_tags) are summed
// in LDS across all of the workgroup's chunks instead and added to the shard at the end (never for a
// validating push: its verdict comes after this kernel, so the host passes no hot tags and every record
// is partitioned). VALIDATE, next_ctl: as bin_part_kernel.

// KIND: the partition layout (0 range: only the keys' low words are loaded -- the register budget of
// this kernel is tight; -1 read at run time)
template <typename V, bool MAT, int KIND, bool VALIDATE>
__global__ __launch_bounds__(kATPB) void bin_part_dedup_kernel(
    const i64* __restrict__ keys, const int32_t* __restrict__ cols, const V* __restrict__ vals, i64 n, PartDesc part,
    const LaunchCtl* lctl, u32 ntiles, int from_break, BinGeom g, u32* __restrict__ addr_out,
    typename LdsAcc<V>::T* __restrict__ val_out, ErrState* err, BinCtl* bc, u32* __restrict__ ct, u32 ctstride,
    const u32* __restrict__ hot_tags, V* __restrict__ data, BinCtl* next_bc, u32* __restrict__ next_T,
    LaunchCtl* vctl, LaunchCtl* next_ctl) {
  typedef typename LdsAcc<V>::T A;
  static_assert(kAChunk * (4 + sizeof(A)) <= kASlots * sizeof(A), "staging must fit the value table");
  __shared__ u32 hk[kASlots];
  __shared__ A hv[kASlots];
  __shared__ u32 htag[kHotSlots];
  __shared__ A hacc[kHotSlots];
  __shared__ uint16_t used[kAChunk];
  __shared__ u32 dcnt[kMaxDigit], gcnt[kMaxDigit];
  __shared__ u32 nused;
  const int tid = threadIdx.x, lane = tid & 63;
  const u32 w = blockIdx.x;
  const i64 r0 = tail_start(lctl, ntiles, from_break, n);
  const i64 nchunks = (n - r0 + kAChunk - 1) / kAChunk;
  A* const st_v = hv;
  u32* const st_a = reinterpret_cast<u32*>(hv + kAChunk);
  constexpr int kStageA = (kAChunk * (4 + (int)sizeof(A)) + (int)sizeof(A) - 1) / (int)sizeof(A);  // hv entries staging uses
  for (int sl = tid; sl < kASlots; sl += kATPB) {
    hk[sl] = kEmptySlot;
    hv[sl] = A(0);
  }
  for (int sl = tid; sl < kHotSlots; sl += kATPB) {
    htag[sl] = hot_tags ? hot_tags[sl] : kEmptySlot;
    hacc[sl] = hot_zero<A>();
  }
  for (u32 d = tid; d < g.nb; d += kATPB) dcnt[d] = 0;
  if (tid == 0) nused = 0;
  if (w == 0) part_next_header(g, next_bc, next_T, next_ctl);
  __syncthreads();
  PhaseClock ph(8);
  ph.mark(8);
  const u64 below = (1ull << lane) - 1ull;
  const i64 G = gridDim.x;
  const BufOut ctb = buf_out(ct, g.nb * ctstride * 4u);  // (< 2^32 bytes: push_binnable)
  BadRecs bad;
  u32 emitted = 0, ncold = 0, nvalid = 0;
  bool dis = false;
  // chunk loads are unconditional (index clamped; a step past the end sees no valid record), so the
  // compiler can wait for one chunk's loads while the next chunk's stay in flight
  auto load_chunk = [&](i64 c, RecRegs<V, MAT>& r) {
    const i64 cc = min(c, nchunks - 1);
    const i64 c0 = r0 + cc * kAChunk, c1 = min(n, r0 + (cc + 1) * kAChunk);
    if constexpr (KIND == 0 && !VALIDATE) {  // (key - start).toInt needs the low words only
#pragma unroll
      for (int q = 0; q < kAPer; ++q) {
        const i64 i = c0 + q * kATPB + threadIdx.x;
        const i64 ii = i < c1 ? i : c1 - 1;
        r.k[q] = (i64)(u64)ld_in(reinterpret_cast<const u32*>(keys) + 2 * ii);
        r.cl[q] = MAT ? ld_in(cols + ii) : 0;
        r.v[q] = ld_in(vals + ii);
      }
    } else {
      load_recs<V, MAT>(keys, cols, vals, c0, c1, r);
    }
  };
  auto step = [&](i64 c, RecRegs<V, MAT>& r) {
    const i64 c0 = r0 + c * kAChunk, c1 = c < nchunks ? min(n, c0 + kAChunk) : c0;
    // the chunk's addresses, rejected records and hot hits first: the hot-table reads of all kAPer
    // records are in flight together, and a hot record is summed here and leaves the chunk
    u32 ca[kAPer];
    u32 cold = 0;
#pragma unroll
    for (int q = 0; q < kAPer; ++q) {
      const i64 i = c0 + q * kATPB + tid;
      const bool in = i < c1;
      i64 a64;
      bool ok = in && rec_addr<MAT, KIND>(part, r.k[q], r.cl[q], a64);
      if constexpr (VALIDATE) ok = ok && key_in_part<KIND>(part, r.k[q]);
      ca[q] = ok ? (u32)a64 : 0u;
      if (ok) cold |= 1u << q;
      else if (in) bad.add(i);
      if (next_ctl && q == 0) {  // (as bin_part_kernel)
        const u32 a32 = ok ? (u32)a64 : 0xFFFFFFFFu, prev = __shfl_up(a32, 1);
        dis = dis || (in && (!ok || ((threadIdx.x & 63) && prev >= a32)));
      }
    }
    nvalid += (u32)__popc(cold);
#pragma unroll
    for (int q = 0; q < kAPer; ++q) {
      const u32 hs = hot_slot(ca[q]);
      if ((cold & (1u << q)) && htag[hs] == ca[q]) {  // hot: summed over all of this workgroup's chunks
        lds_add(&hacc[hs], (A)r.v[q]);
        cold &= ~(1u << q);
      }
    }
    ncold += (u32)__popc(cold);
#pragma unroll
    for (int q = 0; q < kAPer; ++q) {
      bool claimed = false;
      u32 h = 0;
      if (cold & (1u << q)) {
        const u32 a = ca[q];
        h = (a * 0x9E3779B1u) >> (32 - kASlotBits);
        for (;;) {  // the compare-and-swap is the probe: one LDS round trip per slot tried
          const u32 prev = atomicCAS(&hk[h], kEmptySlot, a);
          if (prev == kEmptySlot) { claimed = true; break; }
          if (prev == a) break;
          h = (h + 1) & (kASlots - 1);
        }
        lds_add(&hv[h], (A)r.v[q]);
      }
      const u64 b = __ballot(claimed);  // the wave's new slots join the list with one LDS atomic
      if (b) {
        u32 base = 0;
        if (lane == 0) base = atomicAdd(&nused, (u32)__popcll(b));
        base = __shfl(base, 0);
        if (claimed) used[base + (u32)__popcll(b & below)] = (uint16_t)h;
      }
    }
    ph.mark(9);
    load_chunk(c + 2 * G, r);  // two chunks ahead: in flight across this chunk and the next
    ph.mark(10);
    __syncthreads();
    const u32 D = nused;
    u32 ad[kAPer];
    A va[kAPer];
    u32 valid = 0;
#pragma unroll
    for (int j = 0; j < kAPer; ++j) {  // the chunk's distinct elements, out of the table
      const u32 e = tid + j * kATPB;
      ad[j] = 0;
      va[j] = A(0);
      if (e < D) {
        const u32 sl = used[e];
        ad[j] = hk[sl];
        va[j] = hv[sl];
        hk[sl] = kEmptySlot;
        valid |= 1u << j;
      }
    }
    __syncthreads();
    if (tid == 0) nused = 0;
    ph.mark(11);
    const i64 cs = c < nchunks ? c : 0;  // (as bin_part_kernel)
    const u32 crow = (u32)(c < nchunks ? c : nchunks);
    emitted += part_emit<A, kAPer>(ad, va, valid, g, dcnt, gcnt, st_a, st_v, ctb, crow, ctstride,
                                   addr_out + (size_t)cs * kAChunk, val_out + (size_t)cs * kAChunk, ph, 12);
    for (int sl = tid; sl < kStageA; sl += kATPB) hv[sl] = A(0);  // staging overlaid these
#pragma unroll
    for (int j = 0; j < kAPer; ++j) {  // and the table's own slots of this chunk
      const u32 e = tid + j * kATPB;
      if (e < D) {
        const u32 sl = used[e];
        if (sl >= (u32)kStageA) hv[sl] = A(0);
      }
    }
    __syncthreads();
    ph.mark(17);
  };
  RecRegs<V, MAT> r[2];
  i64 c = w;
  if (c < nchunks) {
#pragma unroll
    for (int j = 0; j < 2; ++j) load_chunk(c + j * G, r[j]);
    for (; c < nchunks; c += 2 * G) {
#pragma unroll
      for (int j = 0; j < 2; ++j) step(c + j * G, r[j]);  // past the end: no valid record, nothing stored
    }
  }
  if (tid == 0 && emitted) atomicAdd(&bc->m, emitted);
  if constexpr (VALIDATE) {
    if (bad.count) atomicMax(&vctl->bad, ~(u64)bad.first);
  } else {
    bad.report(err);
  }
  {  // records that entered the hash table (valid, not hot): the host's measure of what chunk dedup merges
    const u32 tot = block_sum<kATPB>(ncold);
    if (tid == 0 && tot) atomicAdd(&bc->cold, tot);
    const u32 tv = block_sum<kATPB>(nvalid);  // valid records of the tail, hot ones included
    if (tid == 0 && tv) atomicAdd(&bc->tail, tv);
  }
  if (next_ctl && __syncthreads_or(dis) && tid == 0) atomicOr(&bc->disorder, 1u);
  __syncthreads();  // every chunk's hot sums are in
  for (int sl = tid; sl < kHotSlots; sl += kATPB) {
    const u32 a = htag[sl];
    if (a != kEmptySlot && !hot_untouched<A>(hacc[sl])) hot_flush(data + a, hacc[sl]);
  }
  ph.flush(10);
}

// ---- bin_scan ---------------------------------------------------------------------------------------
// One workgroup per coarse bucket b, after the partition (and a validating push's verdict: a cancelled
// push's tail is empty here, so every bucket is): bucket b's records are its runs in chunk order, the
// run of chunk c at partition-buffer index c * kChunk + start(c, b). The bucket's chunk prefix
// P[b][c] = records of b in chunks < c (P[b][nch] = T[b]) and Q[b][c] = c * kChunk + start - P[b][c]
// (so record v of the bucket, in chunk c, is at Q[b][c] + v), its range [Bb[b], Bb[b] + T[b]) of the
// fine sort's output and its items [Ib[b], Ib[b] + items) -- each bucket takes both with one atomic, in
// any order -- with cwin[item] = the chunks holding the item's first and last records. Two passes over
// the bucket's row of the chunk table (the second one hits in cache): its total, then the prefixes.
// The hot split's sums (bin_hot_reduce) ride along as workgroups past the buckets (best != nullptr).
constexpr int kScanTPB = 1024;
constexpr int kScanPer = 8;
static_assert(kScanTPB == kRedTPB, "one launch for both");
template <typename V>
__global__ __launch_bounds__(kScanTPB) void bin_scan_kernel(BinGeom g, const u32* __restrict__ ct, u32 ctstride, i64 n,
                                                            const LaunchCtl* lctl, u32 ntiles, int from_break,
                                                            u32 kchunk, u32 nstride, BinCtl* bc, u32* __restrict__ T,
                                                            u32* __restrict__ Bb, u32* __restrict__ Ib,
                                                            uint2* __restrict__ fitems, uint2* __restrict__ cwin,
                                                            u32* __restrict__ P, u32* __restrict__ Q, u32 item,
                                                            const unsigned long long* __restrict__ best, u32 G,
                                                            const typename LdsAcc<V>::T* __restrict__ partial,
                                                            V* __restrict__ data, const LaunchCtl* gated) {
  if (blockIdx.x >= g.nb) {
    hot_reduce_block<V>(blockIdx.x - g.nb, best, G, partial, data, gated);
    return;
  }
  __shared__ u32 base2[2];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const u32 b = blockIdx.x;
  const i64 r0 = tail_start(lctl, ntiles, from_break, n);
  const u32 nch = (u32)((n - r0 + kchunk - 1) / kchunk);
  if (b == 0 && tid == 0) bc->nch = nch;
  const u32* const row = ct + (size_t)b * ctstride;
  u32 s = 0;
  for (u32 base = 0; base < nch; base += (u32)kScanTPB * kScanPer) {  // kScanPer loads in flight
    u32 w[kScanPer];
#pragma unroll
    for (int k = 0; k < kScanPer; ++k)  // (clamped, unconditional loads: all in flight together)
      w[k] = row[min(base + (u32)k * kScanTPB + tid, nch - 1u)];
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) s += base + (u32)k * kScanTPB + tid < nch ? w[k] >> 16 : 0u;
  }
  const u32 tb = block_sum<kScanTPB>(s);
  const u32 J = bucket_items(tb, item);
  if (tid == 0) {
    T[b] = tb;
    base2[0] = atomicAdd(&bc->rbase, tb);
    base2[1] = atomicAdd(&bc->nfitems, J);
    Bb[b] = base2[0];
    Ib[b] = base2[1];
  }
  __syncthreads();
  const u32 ib = base2[1];
  u32* const Pb = P + (size_t)b * (nstride + 1);
  u32* const Qb = Q + (size_t)b * nstride;
  // tiles of kScanTPB x kScanPer chunks, column k of a tile = chunks base + k kScanTPB + tid (coalesced
  // loads and stores): every column's entries in registers, each column scanned across the workgroup
  // (one barrier for all of them), then only stores (a load between stores would wait for them: one
  // counter for both)
  __shared__ u32 wtk[kScanPer][kScanTPB / 64];
  u32 carry = 0, clast = 0;
  for (u32 base = 0; base < nch; base += (u32)kScanTPB * kScanPer) {
    u32 w[kScanPer], incl[kScanPer];
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) w[k] = row[min(base + (u32)k * kScanTPB + tid, nch - 1u)];
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
      if (base + (u32)k * kScanTPB + tid >= nch) w[k] = 0u;
      const u32 cnt = w[k] >> 16;
      incl[k] = cnt;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const u32 y = __shfl_up(incl[k], d);
        if (lane >= d) incl[k] += y;
      }
      if (lane == 63) wtk[k][wid] = incl[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
      u32 pre, tot;
      wave_totals<kScanTPB / 64>(wtk[k], lane, wid, pre, tot);
      const u32 c = base + (u32)k * kScanTPB + tid, cnt = w[k] >> 16;
      const u32 run = carry + pre + incl[k] - cnt;
      if (c < nch) {
        Pb[c] = run;
        Qb[c] = c * kchunk + (w[k] & 0xFFFFu) - run;
      }
      if (cnt) {
        clast = c;
        // items whose first record is in this run; items whose last one ((j + 1) item - 1) is
        for (u32 j = (run + item - 1) / item; j * item < run + cnt; ++j) {
          fitems[ib + j] = make_uint2(b, j);
          cwin[ib + j].x = c;
        }
        for (u32 k1 = (run + item) / item; k1 * item <= run + cnt; ++k1) cwin[ib + k1 - 1].y = c;
      }
      carry += tot;
    }
    __syncthreads();
  }
  const u32 cl = block_max<kScanTPB>(clast);  // the bucket's last chunk with records
  if (tid == 0) {
    Pb[nch] = tb;
    if (tb == 0) {  // an empty bucket's one item
      fitems[ib] = make_uint2(b, 0u);
      cwin[ib] = make_uint2(0u, 0u);
    } else {
      cwin[ib + J - 1].y = cl;  // the bucket's last record closes its last item
    }
  }
}

// ==== v2 fine stage: one sort pass per fine item, a plan per bucket, an apply that gathers runs =========
// After the chunk-local partition and bin_scan (bucket b = its runs in chunk order, one per chunk;
// record v of the bucket at partition index Q[b][c] + v), bucket b is cut into fine items of 12 x 1024
// records in bucket order. bin_fsort gathers one item's records from its chunks' runs with every load in
// flight, ranks them by fine digit (slab of the bucket) in LDS and writes them to the item's own range
// [Bb[b] + j item, ...) of the fine buffers, sorted by slab, with the item's slab offsets
// off2[item][0..nf] -- no global cursor, whole-wave stores. A slab's records are then one run per item
// of its bucket. bin_plan (one workgroup per bucket) reads the bucket's off2 rows and cuts every slab's
// runs into apply units of <= kUnitCap records at item boundaries (a slab with one unit is exclusive:
// plain read-modify-write; a hot slab's units flush with device atomics). bin_apply2 sums a unit's runs
// in LDS and writes the slab back.
#ifndef GLINT_FSORT_TPB
#define GLINT_FSORT_TPB 1024
#endif
// Records per thread of a fine item: 12 for every push, the values held in registers from their load to
// their staging round (two rounds of 8192 through the 64 KiB stage), at two workgroups per CU (64
// VGPRs). Same boxes (profiles/r06/ab_chunk_local.txt): 16 per thread with the values loaded again in
// each staging round measured cfg4b 2.10 against 1.89 ms, cfg3 1.06 against 0.99; 8 per thread 1.92 /
// 0.99 / cfg5 0.339 against 0.328. (Before the chunk-local partition, with contiguous items, 16 late
// had been the best: ab_fsort_per16.txt.) Build-time knobs GLINT_FSORT_PER_SMALL / _LARGE (small: the
// pushes with the plan fused in, see push_binned).
#ifndef GLINT_PLAN_SPLIT
#define GLINT_PLAN_SPLIT 2
#endif
#ifndef GLINT_FSORT_PER_SMALL
#define GLINT_FSORT_PER_SMALL 12
#endif
#ifndef GLINT_FSORT_PER_LARGE
#define GLINT_FSORT_PER_LARGE 12
#endif
constexpr int kSTPB = GLINT_FSORT_TPB;
constexpr int kSPerSmall = GLINT_FSORT_PER_SMALL, kSPerLarge = GLINT_FSORT_PER_LARGE;
constexpr u32 kSItemMax = (u32)kSTPB * (kSPerSmall > kSPerLarge ? kSPerSmall : kSPerLarge);
static_assert(kSItemMax <= 32768, "u16 slab offsets and the u16 staging of one item");
constexpr u32 kUnitExcl = 1u;  // apply unit descriptor {slab, runs, records, flags}: the slab's only unit
constexpr u32 kSparseCap2 = 1024;  // bin_apply2's touched list (4 workgroups per CU fit in LDS)
// An exclusive slab unit of at most kSparseMax2 records lists its touched elements (first touch) and
// writes back those alone -- unless it touched more than kListMax distinct elements: at 768 of a slab's
// 4096 ~95 % of its lines are touched, and the whole-line sweep beats byte-masked element stores
// (cfg4b exchange 2.91 -> 2.84-2.88 ms, profiles/r04/ab_apply_writeback.txt; 256 / 512 slowed cfg5)
constexpr u32 kSparseMax2 = kSparseCap2;
constexpr u32 kListMax = 768;

// One workgroup per bucket: every slab's runs (one per item of the bucket, from the bucket's off2 rows,
// staged in LDS) cut into apply units of <= kUnitCap records and <= kRunMax runs (a run longer than
// what is left of a unit is split). A unit is a descriptor {slab, runs, records, flags} and a
// fixed-stride run table {start, records before it}, so bin_apply2 reads both in one round trip. A slab
// with one unit is exclusive (plain read-modify-write); the units of a hot slab flush with device
// atomics. Sparse neighbours are merged: an aligned group of 2..16 slabs whose records total at most
// min(kGroupCap, 512 per slab) is ONE unit (one run per item covers all of them: fsort sorted the item
// by slab), summed in an LDS hash table -- a sparse slab alone would hold a whole 32 KB accumulator for
// a few hundred records and one element round trip. Each bucket takes its range of the dense unit list
// with one atomic.
constexpr int kPlanTPB = 1024;
// The plan's LDS: ROWB bytes of the bucket's off2 rows staged at once, PTAB u32 run prefixes (items x
// (slabs + 1)) of the wave emit. The plan launch takes the large one; the plan fused into bin_fsort the
// small one, so that the fine sort keeps two workgroups per CU (a fused push has few items per bucket
// and <= 128 slabs per bucket: cfg5's 641 items, nf = 128)
constexpr u32 kPlanLds = 65536, kPlanPTab = 16640;
constexpr u32 kPlanLdsFused = 32768, kPlanPTabFused = 8320;
constexpr int kRunMax = 128;     // runs per apply unit at most
#ifndef GLINT_UNIT_CAP
#define GLINT_UNIT_CAP 4096
#endif
constexpr u32 kUnitCap = GLINT_UNIT_CAP;  // records per apply unit at most
static_assert(kUnitCap <= 65535, "a unit's record prefix is staged as u16");
#ifndef GLINT_GROUP_SLAB_AVG
#define GLINT_GROUP_SLAB_AVG 512
#endif
constexpr u32 kGroupCap = 2048;      // records per grouped unit (= its LDS hash slots: never full)
constexpr u32 kGroupSlabAvg = GLINT_GROUP_SLAB_AVG;  // ... and per slab of the group on average, at most
constexpr u32 kGroupMax = 16;        // slabs per group (the record's u16 carries its slab's low 4 bits)
static_assert(kSlabBits + 4 <= 16, "a slab offset and 4 slab bits in one u16");
constexpr u32 kUnitGroup = 2u;       // unit flag: a group of sparse slabs (hash-table path)
static_assert(kGroupCap <= kUnitCap && kGroupMax <= 64, "a group is one unit, inside one wave's lanes");
template <u32 ROWB, u32 PTAB, u32 NSLAB = kMaxDigit>
struct PlanLds {
  static constexpr u32 kRowBytes = ROWB, kPTab = PTAB;
  uint16_t rows[ROWB / 2];
  u32 ptab[PTAB];  // (wave emit) records of the slab (group) before each item's run
  u32 nunit[NSLAB];  // (indexed by the slab within the workgroup's range)
  u32 utot[NSLAB];
  uint8_t spanv[NSLAB];
  u32 ubase;
};
// The plan of bucket b by one workgroup of kPlanTPB threads. SC1: the bucket's off2 rows were written by
// other workgroups of this launch (bin_fsort's fused plan, the last item of the bucket plans it), so
// they are read with sc1 loads, as they were stored (the hand-off of the MI355X guide's sc1 table: each
// storing workgroup waits for its stores, then adds to the bucket's counter; the last adder reads).
// The slabs [f_lo, f_hi) of the bucket (at most TPB of them, f_lo a multiple of 64: one slab per thread,
// a wave's lanes on consecutive slabs); the plan launch splits a bucket of many slabs over several
// workgroups, each taking its range of the unit list with one atomic.
template <bool SC1, typename PL, int TPB>
__device__ __forceinline__ void plan_bucket(u32 b, const BinGeom& g, const u32* __restrict__ T, const u32* __restrict__ Bb,
                                            const u32* __restrict__ Ib, const u32* off2, BinCtl* bc,
                                            uint4* __restrict__ units, uint2* __restrict__ runs, int group_on,
                                            PL& L, u32 item, u32 f_lo, u32 f_hi) {
  uint16_t* const rows = L.rows;
  u32* const ptab = L.ptab;
  u32* const nunit = L.nunit;
  u32* const utot = L.utot;
  uint8_t* const spanv = L.spanv;
  u32& ubase = L.ubase;
  const int tid = threadIdx.x;
  const u32 J = bucket_items(T[b], item), I = Ib[b], nf1 = g.nf + 1, bb = Bb[b];
  // the staged rows hold this workgroup's columns only: slabs [f_lo, f_hi] (a run's end is the next
  // slab's offset), nl u16 per item
  const u32 nl = f_hi - f_lo + 1;
  const u32 jt = PL::kRowBytes / 2 / nl;  // items per staged tile (>= 31 for 1024 slabs at 64 KiB)
  const u32 f = f_lo + (u32)tid;      // this thread's slab
  auto stage = [&](u32 j0, u32 j1) {  // rows of items [j0, j1): every load of a round in flight together
    const u32 nx = (j1 - j0) * nl;
    const u32* src = off2 + (size_t)(I + j0) * nf1 + f_lo;
    constexpr int U = 8;
    for (u32 x0 = 0; x0 < nx; x0 += TPB * U) {
      uint16_t t[U];
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const u32 x = x0 + q * TPB + tid;
        const u32 xx = x < nx ? x : nx - 1;
        const u32* ps = src + (size_t)(xx / nl) * nf1 + xx % nl;
        t[q] = (uint16_t)(SC1 ? __hip_atomic_load(ps, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *ps);
      }
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const u32 x = x0 + q * TPB + tid;
        if (x < nx) rows[x] = t[q];
      }
    }
  };
  // The units of slabs [f, f + span) (span 0: this slab belongs to a group another thread emits).
  // emit = false counts them (and *tot = the records); emit = true writes them from unit `base` on.
  auto walk = [&](bool emit, u32 base, u32 flags, u32 span, u32* tot) -> u32 {
    u32 acc = 0, nr = 0, nu = 0, t = 0;
    for (u32 j0 = 0; j0 < J; j0 += jt) {
      const u32 j1 = min(J, j0 + jt);
      if (!emit || J > jt) {  // block-uniform: the rows are staged once when they fit
        __syncthreads();
        stage(j0, j1);
        __syncthreads();
      }
      if (f >= f_hi || span == 0) continue;
      for (u32 j = j0; j < j1; ++j) {
        const uint16_t* r = rows + (j - j0) * nl + (f - f_lo);
        const u32 o0 = r[0];
        u32 c = (u32)r[span] - o0;
        u32 st = bb + j * item + o0;
        t += c;
        while (c) {
          const u32 take = min(c, kUnitCap - acc);
          if (emit) runs[(size_t)(base + nu) * kRunMax + nr] = make_uint2(st, acc);
          acc += take;
          st += take;
          c -= take;
          ++nr;
          if (acc == kUnitCap || nr == (u32)kRunMax) {
            if (emit) units[base + nu] = make_uint4(b * g.nf + f, nr, acc, flags);
            ++nu;
            acc = 0;
            nr = 0;
          }
        }
      }
    }
    if (f < f_hi && span && acc) {
      if (emit) units[base + nu] = make_uint4(b * g.nf + f, nr, acc, flags);
      ++nu;
    }
    if (tot) *tot = t;
    return nu;
  };
  PhaseClock ph(48);
  // A bucket of at most 64 items whose rows fit in LDS at once (every shape measured) is planned with
  // its rows staged once: a thread per slab sums its runs and notes each run's prefix (ptab), so a
  // slab's units are ceil(records / kUnitCap) (a unit never reaches kRunMax runs with <= 64 items); the
  // units are then written by lanes of one wave per slab (2 or 4 slabs per wave for <= 32 / 16 items),
  // a lane per item, so the run-table stores are contiguous (the per-thread walk stored one 8-byte run
  // per lane into 64 different run tables per instruction). Larger buckets take the walk.
  // ptab row stride: this workgroup's slabs + 1 (so the lanes of one slab's column hit different banks)
  const u32 ps = f_hi - f_lo + 1;
  const bool wave_emit = J <= 64u && J <= jt && J * ps <= PL::kPTab;  // block-uniform
  u32 h = 0, nu1 = 0;
  if (wave_emit) {
    stage(0, J);
    __syncthreads();
    if (f < f_hi) {
      const uint16_t* r = rows + (f - f_lo);
#pragma unroll 8
      for (u32 j = 0; j < J; ++j) {
        ptab[j * ps + (f - f_lo)] = h;
        h += (u32)r[j * nl + 1] - (u32)r[j * nl];
      }
    }
    nu1 = (h + kUnitCap - 1) / kUnitCap;
  } else {
    nu1 = walk(false, 0, 0, 1, &h);
  }
  ph.mark(48);
  // sparse neighbours: the largest aligned group (lanes f..f+gs-1 of one wave) within the caps
  u32 span = 1;
  if (group_on && J <= (u32)kRunMax) {
    u32 s = f < f_hi ? h : 0u;
    for (u32 gs = 2; gs <= kGroupMax && gs <= g.nf; gs <<= 1) {
      s += __shfl_xor(s, (int)(gs >> 1));  // the sum over the aligned group of gs slabs
      if (s > 0 && s <= min(kGroupCap, gs * kGroupSlabAvg)) span = gs;
    }
    if (span > 1 && (f & (span - 1))) span = 0;  // a member: its group's first slab emits it
  }
  // (a group's units: at most one, exclusive; a single slab's: the cut above)
  const u32 nu = span > 1 ? 1u : span == 1 ? nu1 : 0u;  // a group (records > 0, <= kGroupCap): one unit
  u32 tot_f = h;
  if (wave_emit && span > 1 && f < f_hi) {  // a group's leader: its column over the group's slabs
    const uint16_t* r = rows + (f - f_lo);
    tot_f = 0;
    for (u32 j = 0; j < J; ++j) {
      ptab[j * ps + (f - f_lo)] = tot_f;
      tot_f += (u32)r[j * nl + span] - (u32)r[j * nl];
    }
  }
  if (f < f_hi) {
    nunit[f - f_lo] = nu;
    spanv[f - f_lo] = (uint8_t)span;
    utot[f - f_lo] = tot_f;
  }
  __syncthreads();
  const u32 used = block_scan<TPB, 1>(f_hi - f_lo, [&](u32 x) { return nunit[x]; },
                                      [&](u32 x, u32 excl) { nunit[x] = excl; });
  ph.mark(49);
  if (tid == 0) ubase = used ? atomicAdd(&bc->nunits, used) : 0u;
  __syncthreads();
  ph.mark(50);
  if (wave_emit) {
    const u32 lane = (u32)tid & 63u;
    const u32 spw = J <= 16u ? 4u : J <= 32u ? 2u : 1u;  // slabs per wave pass, 64 / spw lanes each
    const u32 lpw = 64u / spw, sub = lane / lpw, j = lane % lpw;
    const u64 gmask = lpw == 64u ? ~0ull : ((1ull << lpw) - 1ull) << (sub * lpw);
    const u64 below = (1ull << lane) - 1ull;
    for (u32 f0 = f_lo + (u32)(tid >> 6) * spw; f0 < f_hi; f0 += (TPB / 64) * spw) {
      const u32 ff = f0 + sub;
      u32 sp = 0, base = 0, tot = 0;
      if (ff < f_hi) {
        sp = spanv[ff - f_lo];
        base = ubase + nunit[ff - f_lo];
        tot = utot[ff - f_lo];
      }
      const bool on = sp != 0u && j < J;
      u32 c = 0, st = 0, P = 0;
      if (on) {  // this item's run of the slab (or of the group's slabs: fsort sorted the item by slab)
        const uint16_t* r = rows + j * nl + (ff - f_lo);
        const u32 o0 = r[0];
        c = (u32)r[sp] - o0;
        st = bb + j * item + o0;
        P = ptab[j * ps + (ff - f_lo)];
      }
      const u32 nus = sp == 0u ? 0u : sp > 1u ? 1u : (tot + kUnitCap - 1) / kUnitCap;
      const u32 fl = sp > 1u ? (kUnitExcl | kUnitGroup) : (nus == 1u ? kUnitExcl : 0u);
      for (u32 u = 0; __ballot(u < nus); ++u) {  // unit u: records [u * cap, min(tot, (u + 1) * cap)) of the slab
        const u32 lo = u * kUnitCap, hi = min(tot, lo + kUnitCap);
        const bool in = on && u < nus && c > 0u && P < hi && P + c > lo;
        const u64 m = __ballot(in) & gmask;
        if (in) {
          const u32 from = max(P, lo);
          runs[(size_t)(base + u) * kRunMax + (u32)__popcll(m & below)] = make_uint2(st + (from - P), from - lo);
        }
        if (j == 0u && u < nus) units[base + u] = make_uint4(b * g.nf + ff, (u32)__popcll(m), hi - lo, fl);
      }
    }
  } else {
    const u32 flags = span > 1 ? (kUnitExcl | kUnitGroup) : (nu == 1 ? kUnitExcl : 0u);
    walk(true, ubase + (f < f_hi ? nunit[f - f_lo] : 0u), flags, span, nullptr);
  }
  __syncthreads();
  ph.mark(51);
  ph.flush(4);
}

// The plan launch: one workgroup of kPlanTPB threads per bucket, a slab per thread. (Split over
// 256-slab ranges, four workgroups per bucket of 512 slabs with lighter LDS, it measured no faster:
// cfg3 1.033 -> 1.047 ms, cfg4b 2.170 -> 2.164, profiles/r06/ab_plan_split.txt.)
__global__ __launch_bounds__(kPlanTPB) void bin_plan_kernel(BinGeom g, const u32* __restrict__ T, const u32* __restrict__ Bb,
                                                            const u32* __restrict__ Ib, const u32* __restrict__ off2,
                                                            BinCtl* bc, uint4* __restrict__ units, uint2* __restrict__ runs,
                                                            int group_on, u32 item) {
  typedef PlanLds<kPlanLds, kPlanPTab> PL;
  __shared__ PL L;
  constexpr u32 kS = GLINT_PLAN_SPLIT;  // workgroups per bucket, each planning a range of its slabs
  // (plan_bucket's ranges start at multiples of 64 slabs: a bucket of fewer than 64 kS slabs has fewer
  // ranges, the spare workgroups return)
  const u32 b = blockIdx.x / kS, s = blockIdx.x % kS, fs = max(64u, g.nf / kS);
  if (s * fs >= g.nf) return;
  plan_bucket<false, PL, kPlanTPB>(b, g, T, Bb, Ib, off2, bc, units, runs, group_on, L, item, s * fs,
                                   min(g.nf, (s + 1) * fs));
}

// FUSED: the plan runs here too -- the workgroup of a bucket's last item to finish plans the bucket
// (plan_bucket<true>), so no plan launch follows and the buckets' plans overlap the other items' sorts.
constexpr u32 kStage = 65536;  // bin_fsort: bytes of the item's u16 offsets, then its values in rounds
// A value the compiler must recompute where it is used (not hoist and hold in a register across a loop)
__device__ __forceinline__ u32 opaque(u32 x) {
  asm volatile("" : "+v"(x));
  return x;
}
// Forward fill of rid[0, x1) (<= TPB * 16 entries, 0 = no mark; the array holds whole blocks of 16):
// every entry becomes the last mark at or before it (marks increase with x, so this is an inclusive
// max-scan). 16 entries per thread, read and written as two 16-byte LDS accesses.
template <int TPB>
__device__ __forceinline__ void fill_forward(uint16_t* rid, u32 x1) {
  constexpr int kPer = 16;
  __shared__ u32 wmax[TPB / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const u32 b0 = (u32)tid * kPer;
  const bool mine = b0 < x1;
  uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;
  if (mine) {
    q0 = reinterpret_cast<const uint4*>(rid + b0)[0];
    q1 = reinterpret_cast<const uint4*>(rid + b0)[1];
  }
  u32 h[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};  // two u16 per word, low first
  u32 m = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) m = max(m, max(h[k] & 0xFFFFu, h[k] >> 16));
  u32 incl = m;
#pragma unroll
  for (int dd = 1; dd < 64; dd <<= 1) {
    const u32 y = __shfl_up(incl, dd);
    if (lane >= dd) incl = max(incl, y);
  }
  if (lane == 63) wmax[wid] = incl;
  __syncthreads();
  u32 run = __shfl_up(incl, 1);
  if (lane == 0) run = 0;
  for (int w2 = 0; w2 < wid; ++w2) run = max(run, wmax[w2]);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const u32 lo = run = max(run, h[k] & 0xFFFFu);
    const u32 hi = run = max(run, h[k] >> 16);
    h[k] = lo | (hi << 16);
  }
  if (mine) {
    reinterpret_cast<uint4*>(rid + b0)[0] = make_uint4(h[0], h[1], h[2], h[3]);
    reinterpret_cast<uint4*>(rid + b0)[1] = make_uint4(h[4], h[5], h[6], h[7]);
  }
  __syncthreads();
}
constexpr u32 kFWin = 2048;  // bin_fsort: chunks per window of the item's run table
template <typename A, bool FUSED, int kSPer>
__global__ __launch_bounds__(kSTPB) __attribute__((amdgpu_waves_per_eu(8))) void bin_fsort_kernel(BinGeom g, const uint2* __restrict__ fitems, BinCtl* bc,
                                                          const u32* __restrict__ T, const u32* __restrict__ Bb,
                                                          const u32* __restrict__ addr_in, const A* __restrict__ val_in,
                                                          uint16_t* __restrict__ e_out, A* __restrict__ v_out,
                                                          u32* __restrict__ off2, u64* hint, u64* whole_hint,
                                                          u32 whole_n, const u32* __restrict__ Ib, u32* done,
                                                          uint4* __restrict__ units, uint2* __restrict__ runs,
                                                          int group_on, u32 item, const uint2* __restrict__ cwin,
                                                          const u32* __restrict__ P, const u32* __restrict__ Q,
                                                          u32 nstride) {
  constexpr u32 kStageV = kStage / (u32)sizeof(A);   // values per round
  // [hist | stage]; until the ranking the stage holds the item's window of chunk prefixes P and places Q
  // and its run marks (u16 per record)
  constexpr size_t kSortLds = 4 * kMaxDigit + kStage;
  constexpr u32 kOffQ = ((kFWin + 1) * 4 + 255) / 256 * 256, kOffRid = kOffQ + 4 * kFWin;
  static_assert(kOffRid + 2 * kSItemMax <= kStage, "the window and the marks overlay the stage");
  typedef PlanLds<kPlanLdsFused, kPlanPTabFused> FusedPlanLds;
  constexpr size_t kLds = FUSED && sizeof(FusedPlanLds) > kSortLds ? sizeof(FusedPlanLds) : kSortLds;
  __shared__ __attribute__((aligned(16))) unsigned char smem[kLds];
  __shared__ u32 last_flag;
  u32* const hist = reinterpret_cast<u32*>(smem);
  unsigned char* const stage = smem + 4 * kMaxDigit;
  const int tid = threadIdx.x;
  if (blockIdx.x == 0 && tid == 0 && hint) {  // for the host's next binned push: how much did dedup keep?
    __hip_atomic_store(hint, ((u64)bc->m << 32) | (u64)bc->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(hint + 1, (u64)bc->cold, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (whole_hint) {  // a whole-push bin, in push_apply's words: an unordered push has its tail from record
      const bool dis = bc->disorder != 0u;  // 0 on (so the next push bins whole again); an ordered one none
      __hip_atomic_store(whole_hint, dis ? (u64)whole_n : 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(whole_hint + 3, dis ? 0ull : ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  const u32 it = blockIdx.x;
  if (it >= bc->nfitems) return;  // the grid is the item count's upper bound
  const uint2 d = fitems[it];
  const uint2 cw = cwin[it];  // the chunks of the item's first and last records
  const u32 b = d.x;
  const u32* const Pb = P + (size_t)b * (nstride + 1);
  const u32* const Qb = Q + (size_t)b * nstride;
  const u32 span = cw.y - cw.x + 1;
  const bool slow = span > kFWin;  // workgroup-uniform: the item spans more chunks than the window holds
  u32* const Pw = reinterpret_cast<u32*>(stage);  // (the stage is free until the ranking)
  u32* const Qw = reinterpret_cast<u32*>(stage + kOffQ);
  uint16_t* const rid = reinterpret_cast<uint16_t*>(stage + kOffRid);
  static_assert(kFWin == 2 * kSTPB, "two window entries per thread");
  {  // the window's loads first (in flight with the bucket's T and Bb); clamped, unconditional
    const u32 t0 = tid, t1 = tid + kSTPB, sp = min(span, kFWin);
    const u32 p0 = Pb[cw.x + min(t0, sp)], p1 = Pb[cw.x + min(t1, sp)];  // (P[b][c] up to c = nch)
    const u32 q0 = Qb[cw.x + min(t0, sp - 1)], q1 = Qb[cw.x + min(t1, sp - 1)];
    if (t0 <= sp) Pw[t0] = p0;
    if (t1 <= sp) Pw[t1] = p1;
    if (t0 < sp) Qw[t0] = q0;
    if (t1 < sp) Qw[t1] = q1;
  }
  const u32 s0 = Bb[b] + d.y * item, s1 = Bb[b] + min(T[b], (d.y + 1) * item);
  const u32 nf1 = g.nf + 1;
  u32* const orow = off2 + (size_t)it * nf1;
  auto put_row = [&](u32 f, u32 x) {  // (fused: sc1 stores, read by the bucket's planner with sc1 loads)
    if (FUSED) __hip_atomic_store(orow + f, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else orow[f] = x;
  };
  auto finish = [&]() {  // fused: count this item in; the bucket's last one plans it
    if (!FUSED) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its stores done
    __syncthreads();
    if (tid == 0) last_flag = atomicAdd(&done[b], 1u) + 1u == bucket_items(T[b], item);
    __syncthreads();
    if (last_flag)
      plan_bucket<true, FusedPlanLds, kSTPB>(b, g, T, Bb, Ib, off2, bc, units, runs, group_on,
                                             *reinterpret_cast<FusedPlanLds*>(smem), item, 0u, g.nf);
  };
  for (u32 f = tid; f < g.nf; f += kSTPB) hist[f] = 0;
  if (s1 == s0) {  // an empty bucket's one item
    for (u32 f = tid; f < nf1; f += kSTPB) put_row(f, 0u);
    finish();
    return;
  }
  PhaseClock ph(32);
  // (the item's outputs go through buffer windows over its own ranges: workgroup-uniform descriptors,
  // 32-bit offsets, a store at the window's end dropped -- counted stores, see BufOut)
  const u32 cnt = s1 - s0;
  // Where the item's records are: record v of the bucket lies in the run of the chunk c with
  // P[b][c] <= v < P[b][c + 1], at partition index Q[b][c] + v. The prefixes of the item's chunks (cwin:
  // those of its first and last records, at most kFWin) go to LDS; every chunk's run marks its first record
  // of the item with its window slot, a forward fill gives every record its run, and the record's index
  // follows. (Marks past the item's last record are never cleared: a forward fill carries them only to
  // later places, which no record reads.)
  static_assert(kSItemMax <= 16 * kSTPB && kFWin < 65536 && kSItemMax % 16 == 0,
                "fill_forward's 16 per thread; u16 marks and window slots");
  const u32 v0 = d.y * item;
  if (!slow) {
    for (u32 x = tid * 8u; x < cnt; x += kSTPB * 8u) reinterpret_cast<uint4*>(rid + x)[0] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    ph.mark(32);
    for (u32 t = tid; t < span; t += kSTPB) {
      const u32 lo = max(Pw[t], v0), hi = min(Pw[t + 1], v0 + cnt);
      if (lo < hi) rid[lo - v0] = (uint16_t)(t + 1);
    }
    __syncthreads();
    fill_forward<kSTPB>(rid, cnt);
    ph.mark(33);
  }
  // record x of the item: its index in the partition buffer (slow: a binary search over the bucket's
  // prefix row between the item's first and last chunks, for an item spread so thin over the chunks that
  // its window would not hold it). The two are separate code paths (a search loop's loads in the same
  // path would make every record wait for the loads of the one before).
  auto pos_fast = [&](u32 x) -> u32 { return Qw[rid[x] - 1u] + v0 + x; };
  auto pos_slow = [&](u32 x) -> u32 {
    const u32 v = v0 + x;
    u32 lo = cw.x, hi = cw.y + 1;  // P[lo] <= v < P[hi]
    while (hi - lo > 1) {
      const u32 m = (lo + hi) >> 1;
      if (Pb[m] <= v) lo = m;
      else hi = m;
    }
    return Qb[lo] + v;
  };
  u32 a[kSPer];
  A v[kSPer];
  auto load_item = [&](auto pos_of) {
#pragma unroll
    for (int q = 0; q < kSPer; ++q) {  // the whole item in flight at once
      const u32 x = q * kSTPB + opaque(tid);
      const bool on = (u32)q * kSTPB < item && x < cnt;
      const u32 ps = on ? pos_of(x) : 0u;
      a[q] = on ? ld_mid(addr_in + ps) : kEmptySlot;
      v[q] = on ? ld_mid(val_in + ps) : A(0);
    }
  };
  if (slow) load_item(pos_slow);
  else load_item(pos_fast);
  __syncthreads();
  ph.mark(34);
  // the slab counts, then (after the scan) each record's place in the item's slab order from a second
  // LDS atomic: a place taken in the first pass would hold a register per record through the scan
  // (within a slab the order is any; kEmptySlot: no record)
#pragma unroll
  for (int q = 0; q < kSPer; ++q)
    if (a[q] != kEmptySlot) atomicAdd(&hist[fine_of(a[q], g)], 1u);
  __syncthreads();
  ph.mark(35);
  const u32 total = block_scan<kSTPB, 1>(
      g.nf, [&](u32 f) { return hist[f]; },
      [&](u32 f, u32 excl) {
        hist[f] = excl;
        put_row(f, excl);
      });
  if (tid == 0) put_row(g.nf, total);
  ph.mark(36);
  // the slab offsets (and the slab's low 4 bits: bin_apply2's groups of sparse slabs), staged as u16
  // and stored as whole-wave runs
  uint16_t* const ste = reinterpret_cast<uint16_t*>(stage);
  u32 p[kSPer];
#pragma unroll
  for (int q = 0; q < kSPer; ++q) {
    p[q] = kEmptySlot;
    if (a[q] == kEmptySlot) continue;
    const u32 f = fine_of(a[q], g);
    p[q] = atomicAdd(&hist[f], 1u);
    ste[p[q]] = (uint16_t)((a[q] & (kSlab - 1)) | ((f & 15u) << kSlabBits));
  }
  __syncthreads();
  const BufOut eo = buf_out(e_out + s0, total * 2u), vo = buf_out(v_out + s0, total * (u32)sizeof(A));
#pragma unroll
  for (int q = 0; q < kSPer; ++q) {  // total <= item <= kSPer * kSTPB
    const u32 x = q * kSTPB + opaque(tid);
    if ((u32)q * kSTPB >= item) break;  // launch-uniform
    bput16(eo, x * 2u, x < total, ste[x]);
  }
  __syncthreads();
  ph.mark(37);
  A* const stv = reinterpret_cast<A*>(stage);
  for (u32 r0 = 0; r0 < total; r0 += kStageV) {  // the values, kStageV per round
#pragma unroll
    for (int q = 0; q < kSPer; ++q)
      if (p[q] != kEmptySlot && p[q] - r0 < kStageV) stv[p[q] - r0] = v[q];
    __syncthreads();
    constexpr int kRound = (int)(kStageV / kSTPB);
#pragma unroll
    for (int q = 0; q < kRound; ++q) {
      const u32 x = r0 + q * kSTPB + tid;
      bput(vo, x * (u32)sizeof(A), x < total, stv[x - r0]);
    }
    __syncthreads();
  }
  ph.mark(38);
  ph.flush(7);
  finish();
}

// Per apply unit: the records of its runs (record r lives in run i = the last one whose prefix is <= r:
// a binary search over the unit's run table in LDS), kCRB2 per thread per batch. A slab unit sums them
// in LDS and is written back (exclusive: one coalesced RMW of the touched 128-B lines, or the touched
// list of a sparse unit; shared: device atomics). A group unit (several sparse slabs) sums them
// in an LDS hash table keyed by element (overlaying the slab accumulator) and read-modify-writes each
// distinct element. Element write-backs issue all their loads before any store (a loop of dependent
// load / store pairs would wait one round trip per element). Software-pipelined per workgroup: the
// descriptor and run table of the unit two ahead load during this one, and the next unit's run table
// and first record batch are issued before this unit's write-back.
#ifndef GLINT_APPLY2_WAVES
#define GLINT_APPLY2_WAVES 4  // bin_apply2's register budget: waves per SIMD (4 workgroups per CU fit in LDS)
#endif
#ifndef GLINT_CRB2
#define GLINT_CRB2 4  // (8: 18 spilled VGPRs; A/B profiles/r05: cfg5 0.383 vs 0.403 ms, cfg3 1.130 vs 1.136, cfg4b 2.508 vs 2.501)
#endif
constexpr int kCRB2 = GLINT_CRB2;  // records per thread per batch
template <typename V>
__global__ __launch_bounds__(kCTPB) __attribute__((amdgpu_waves_per_eu(GLINT_APPLY2_WAVES))) void bin_apply2_kernel(
    const uint16_t* __restrict__ e_in, const typename LdsAcc<V>::T* __restrict__ v_in, const uint4* __restrict__ units,
    const uint2* __restrict__ runs, const BinCtl* bc, i64 elems, V* __restrict__ data, int xcd_map, u32 nf) {
  typedef typename Vec2<V>::T V2;
  typedef typename LdsAcc<V>::T A;
  static_assert(kRunMax <= kCTPB, "one run per loading thread");
  static_assert(kGroupCap * (4 + sizeof(A)) <= kSlab * sizeof(A), "the group table overlays the slab accumulator");
  static_assert(kGroupCap * 2 <= kSlab, "the group's slot list overlays the touched flags");
  __shared__ A acc[kSlab];
  __shared__ uint8_t touched[kSlab];
  __shared__ uint16_t tlist[kSparseCap2];
  __shared__ u32 ntl[2];
  __shared__ u32 rs[2][kRunMax];
  __shared__ uint16_t rp[2][kRunMax + 1];
  u32* const hk = reinterpret_cast<u32*>(acc);  // group units: element + 1 (0 = empty slot)
  A* const hv = reinterpret_cast<A*>(reinterpret_cast<char*>(acc) + kGroupCap * 4);
  uint16_t* const hused = reinterpret_cast<uint16_t*>(touched);  // the group's claimed slots, in order
  constexpr int kPairsPerThread = kSlab / 2 / kCTPB;
  constexpr int kListPer = (kGroupCap + kCTPB - 1) / kCTPB;  // element write-backs per thread at most
  constexpr int kListPass = 4;                                // ... in passes of this many
  static_assert(kSparseCap2 <= kGroupCap, "the touched list fits the element write-back");
  const int tid = threadIdx.x, lane = tid & 63;
  const u64 below = (1ull << lane) - 1ull;
  for (int e = tid; e < kSlab; e += kCTPB) acc[e] = A(0);
  for (int w = tid; w < kSlab / 16; w += kCTPB) reinterpret_cast<uint4*>(touched)[w] = make_uint4(0, 0, 0, 0);
  if (tid < 2) ntl[tid] = 0;
  const u32 nunits = bc->nunits;
  const u32 G = gridDim.x;
  // this workgroup's i-th unit: blockIdx + i G, or (xcd_map) a contiguous eighth of the units per group
  // of workgroups that dispatch to one XCD (blockIdx % 8), so the workgroups of an XCD take neighbouring
  // slabs together and share in its L2 the lines where one item's runs for them meet
  const u32 xk = blockIdx.x >> 3, xK = G >> 3, xC = (nunits + 7) >> 3, xbase = (blockIdx.x & 7u) * xC;
  auto unit_of = [&](u32 i) -> u32 {
    if (!xcd_map) return blockIdx.x + i * G;
    const u32 k = xk + i * xK;
    return k < xC ? xbase + k : 0xFFFFFFFFu;
  };
  const uint4 kNone = make_uint4(0u, 0u, 0u, 0u);
  auto load_unit = [&](u32 uu, uint4& d, uint2& r) {
    d = uu < nunits ? units[uu] : kNone;
    r = make_uint2(0u, 0u);
    if (uu < nunits && tid < kRunMax) r = runs[(size_t)uu * kRunMax + tid];
  };
  auto publish = [&](int slot, const uint4& d, const uint2& r) {  // the unit's run table into LDS
    if ((u32)tid < d.y) {
      rs[slot][tid] = r.x;
      rp[slot][tid] = (uint16_t)r.y;
    }
    if (tid == 0) rp[slot][d.y] = (uint16_t)d.z;  // (d.y == 0 only for a missing unit: count 0)
  };
  // a batch's records: record rr lives in run lo = the last one whose prefix is <= rr, found by a
  // fixed-step search (kRunMax = 2^7: seven steps, the kCRB2 searches in lockstep -- a data-dependent
  // loop ran them one after another, ~40 % of the workgroup's clocks); runs past nr are never chosen
  // (the prefix array holds the unit's count at nr, and rr < count)
  static_assert((kRunMax & (kRunMax - 1)) == 0, "fixed-step search over a power of two");
  // returns which of the thread's kCRB2 records are valid as a mask: selecting on the loaded registers
  // would make the compiler wait for the loads right there (and the prefetch would not overlap anything)
  auto fetch = [&](int slot, const uint4& d, u32 r0, u32 (&ca)[kCRB2], A (&cv)[kCRB2]) -> u32 {
    const u32 cnt = d.z, nr = d.y;
    if (cnt == 0) return 0u;  // block-uniform: a missing unit
    u32 rr[kCRB2], lo[kCRB2];
#pragma unroll
    for (int q = 0; q < kCRB2; ++q) {
      const u32 r = r0 + q * kCTPB + tid;
      rr[q] = r < cnt ? r : cnt - 1;  // clamped, branch-free loads
      lo[q] = 0;
    }
#pragma unroll
    for (u32 step = kRunMax / 2; step > 0; step >>= 1) {
#pragma unroll
      for (int q = 0; q < kCRB2; ++q) {
        const u32 m = lo[q] + step;
        if (m < nr && (u32)rp[slot][m] <= rr[q]) lo[q] = m;
      }
    }
    u32 valid = 0;
#pragma unroll
    for (int q = 0; q < kCRB2; ++q) {
      const u32 idx = rs[slot][lo[q]] + (rr[q] - (u32)rp[slot][lo[q]]);
      ca[q] = ld_mid(e_in + idx);
      cv[q] = ld_mid(v_in + idx);
      valid |= (r0 + q * kCTPB + tid < cnt ? 1u : 0u) << q;
    }
    return valid;
  };
  // a wave's claimed list entries: one LDS atomic per wave for all its lanes' new entries
  auto list_append = [&](bool first, u32 val, u32 par_, uint16_t* list) {
    const u64 bl = __ballot(first);
    if (bl) {
      u32 base = 0;
      if (lane == 0) base = atomicAdd(&ntl[par_], (u32)__popcll(bl));
      base = __shfl(base, 0);
      if (first) list[base + (u32)__popcll(bl & below)] = (uint16_t)val;
    }
  };
  // prologue: unit u published, its first batch in flight; unit u + G loaded
  uint4 dcur, dnext;
  uint2 rcur, rnext;
  u32 i = 0, u = unit_of(0);
  load_unit(u, dcur, rcur);
  load_unit(unit_of(1), dnext, rnext);
  publish(0, dcur, rcur);
  __syncthreads();
  u32 pa[kCRB2];
  A pv[kCRB2];
  u32 pvalid = fetch(0, dcur, 0u, pa, pv);
  int cs = 0;  // LDS table slot of unit u
  u32 par = 0;
  PhaseClock ph(56);
  for (; u < nunits; u = unit_of(++i)) {
    const uint4 d = dcur;
    const u32 slab = d.x, cnt = d.z;
    const bool group = (d.w & kUnitGroup) != 0;
    const bool exclusive = (d.w & kUnitExcl) != 0;
    const i64 sbase_g = (i64)slab << kSlabBits;
    V* const sbase = data + sbase_g;
    const bool sparse = !group && exclusive && cnt <= kSparseMax2;
    u32 ca[kCRB2];
    A cv[kCRB2];
    u32 valid = pvalid;
#pragma unroll
    for (int q = 0; q < kCRB2; ++q) {
      ca[q] = pa[q];
      cv[q] = pv[q];
    }
    for (u32 r0 = 0;;) {  // the first batch came with the prefetch
      if (group) {
#pragma unroll
        for (int q = 0; q < kCRB2; ++q) {
          bool first = false;
          u32 h = 0;
          if ((valid >> q) & 1u) {
            // the record's slab: the group's first slab + the difference of their fine digits' low 4 bits
            // (a group of <= 16 aligned slabs lies in one 16-aligned block of its bucket's fine digits)
            const u32 ad = ((slab + (ca[q] >> kSlabBits) - ((slab & (nf - 1)) & (kGroupMax - 1))) << kSlabBits) |
                           (ca[q] & (kSlab - 1));
            const u32 key = ad + 1u;
            h = (ad * 0x9E3779B1u) >> (32 - 11);
            static_assert(kGroupCap == 2048, "11-bit slot hash");
            for (;;) {  // <= kGroupCap distinct keys in kGroupCap slots: an insert always finds one
              const u32 prev = atomicCAS(&hk[h], 0u, key);
              if (prev == 0u) { first = true; break; }
              if (prev == key) break;
              h = (h + 1) & (kGroupCap - 1);
            }
            lds_add(&hv[h], cv[q]);
          }
          list_append(first, h, par, hused);
        }
      } else if (sparse) {
#pragma unroll
        for (int q = 0; q < kCRB2; ++q) {
          bool first = false;
          u32 e = 0;
          if ((valid >> q) & 1u) {
            e = ca[q] & (kSlab - 1);
            lds_add(&acc[e], cv[q]);
            const u32 sh = 8u * (e & 3u);
            first = ((atomicOr(reinterpret_cast<u32*>(touched) + (e >> 2), 1u << sh) >> sh) & 0xFFu) == 0u;
          }
          list_append(first, e, par, tlist);
        }
      } else {
#pragma unroll
        for (int q = 0; q < kCRB2; ++q) {
          if (!((valid >> q) & 1u)) continue;
          const u32 e = ca[q] & (kSlab - 1);
          lds_add(&acc[e], cv[q]);
          touched[e] = 1;
        }
      }
      r0 += (u32)kCTPB * kCRB2;
      if (r0 >= cnt) break;
      valid = fetch(cs, d, r0, ca, cv);
    }
    ph.mark(56);
    // the next unit's run table into the other slot; the one after it starts loading
    publish(cs ^ 1, dnext, rnext);
    dcur = dnext;
    load_unit(unit_of(i + 2), dnext, rnext);
    __syncthreads();
    ph.mark(57);
    if (tid == 0) ntl[par ^ 1u] = 0;  // the next list unit's count (the last one read it before a barrier)
    // the next unit's first batch: in flight during this unit's write-back
    pvalid = fetch(cs ^ 1, dcur, 0u, pa, pv);
    ph.mark(58);
    bool sweep_wb = exclusive && !sparse && !group;
    if (group || sparse) {
      const u32 L = ntl[par];  // block-uniform (read after the barrier)
      par ^= 1u;
      if (sparse && L > kListMax) {
        sweep_wb = true;  // many distinct elements: whole-line write-back
      } else {
        // element read-modify-writes: every load of a pass (kListPass per thread, 1024 elements)
        // issued before any store
        for (int k0 = 0; k0 < kListPer; k0 += kListPass) {
          if ((u32)(k0 * kCTPB) >= L) break;  // block-uniform
        u32 ad[kListPass];
        V old[kListPass];
#pragma unroll
        for (int k = 0; k < kListPass; ++k) {
          const u32 x = tid + (k0 + k) * kCTPB;
          ad[k] = 0xFFFFFFFFu;
          if (x < L) {
            const u32 s2 = group ? hused[x] : tlist[x];
            ad[k] = group ? hk[s2] - 1u : (u32)(sbase_g + s2);
            if ((i64)ad[k] < elems) old[k] = data[ad[k]];
          }
        }
#pragma unroll
        for (int k = 0; k < kListPass; ++k) {
          if (ad[k] == 0xFFFFFFFFu) continue;
          const u32 x = tid + (k0 + k) * kCTPB;
          const u32 s2 = group ? hused[x] : tlist[x];
          if (group) {
            if ((i64)ad[k] < elems) data[ad[k]] = acc_add(old[k], hv[s2]);
            hk[s2] = 0u;
            hv[s2] = A(0);
            hused[x] = 0;
          } else {
            if ((i64)ad[k] < elems) data[ad[k]] = acc_add(old[k], acc[s2]);
            acc[s2] = A(0);
            touched[s2] = 0;
          }
        }
        }
      }
    }
    if (sweep_wb) {
      // one coalesced RMW of the slab's touched 128-B lines: every pair of a line with a touched
      // element is read and written back (the untouched ones unchanged -- the slab is this unit's), so
      // the stores are whole lines, not byte-masked pairs. Lanes of a line-less pair load the slab's
      // first pair instead (one cached line), so all loads issue back to back without a branch.
      constexpr int kPPL = 128 / (2 * (int)sizeof(V));
      const u64 gmask = (kPPL >= 64 ? ~0ull : ((1ull << kPPL) - 1ull)) << (lane & ~(kPPL - 1));
      V2 dd[kPairsPerThread];
      u32 t[kPairsPerThread];
      bool wb[kPairsPerThread];
#pragma unroll
      for (int q = 0; q < kPairsPerThread; ++q) {
        const int e0 = 2 * (tid + q * kCTPB);
        t[q] = (u32)touched[e0] | ((u32)touched[e0 + 1] << 1);
        wb[q] = (__ballot(t[q] != 0u) & gmask) != 0ull;  // wave-uniform per line
      }
#pragma unroll
      for (int q = 0; q < kPairsPerThread; ++q) {
        const int e0 = 2 * (tid + q * kCTPB);
        const bool vec = wb[q] && sbase_g + e0 + 1 < elems;
        dd[q] = *reinterpret_cast<const V2*>(vec ? sbase + e0 : sbase);
        if (t[q]) *reinterpret_cast<uint16_t*>(touched + e0) = 0;
      }
#pragma unroll
      for (int q = 0; q < kPairsPerThread; ++q) {
        if (!wb[q]) continue;
        const int e0 = 2 * (tid + q * kCTPB);
        if (sbase_g + e0 + 1 < elems) {
          V2 r = dd[q];
          if (t[q] & 1u) r.x = acc_add((V)r.x, acc[e0]);
          if (t[q] & 2u) r.y = acc_add((V)r.y, acc[e0 + 1]);
          *reinterpret_cast<V2*>(sbase + e0) = r;
        } else if (t[q]) {
          sbase[e0] = acc_add(sbase[e0], acc[e0]);
        }
        if (t[q]) {
          acc[e0] = A(0);
          acc[e0 + 1] = A(0);
        }
      }
    } else if (!exclusive) {
      for (int e = tid; e < kSlab; e += kCTPB) {
        if (touched[e]) {
          gadd(sbase + e, (V)acc[e]);
          acc[e] = A(0);
          touched[e] = 0;
        }
      }
    }
    ph.mark(59);
    __syncthreads();
    ph.mark(60);
    cs ^= 1;
  }
  ph.flush(5);
}

// ---- host side ----------------------------------------------------------------------------------------
// resident blocks per CU of a kernel at its block size (occupancy query)
template <typename K>
int resident_per_cu(K kernel, int tpb, size_t dyn_lds = 0) {
  int b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kernel, tpb, dyn_lds) != hipSuccess || b < 1) {
    (void)hipGetLastError();
    b = 1;
  }
  return b;
}

// 128 coarse buckets (few enough that a partition chunk's records form runs per bucket, and a fine
// item's runs per slab stay as long: 32 records each way for uniform keys into 2^28), more only when
// the fine digit would exceed 10 bits (slabs < 2^20 for u32 addresses). Same box, two runs each
// (profiles/r03/bench_binned_cb.txt): 2^7 against 2^8 buckets cfg5 0.418 -> 0.398 ms, cfg3 1.648 ->
// 1.636 ms, cfg4b exchange 3.005 -> 3.005 ms; 2^6 slower on all
#ifndef GLINT_BIN_CB
#define GLINT_BIN_CB 7  // (build-time knob: coarse digit bits at least)
#endif
constexpr u32 kCoarseBitsMin = GLINT_BIN_CB;
BinGeom bin_geometry(i64 elems, u32 cbmin) {
  const i64 slabs = (elems + kSlab - 1) / kSlab;
  u32 sb = 0;
  while (((i64)1 << sb) < slabs) ++sb;
  const u32 cb = std::min<u32>(sb, std::max<u32>(cbmin, sb > 10u ? sb - 10u : 0u));
  BinGeom g;
  g.fb = sb - cb;
  g.nb = 1u << cb;
  g.nf = 1u << g.fb;
  g.nslab = g.nb * g.nf;
  return g;
}

// u32 record indices and element addresses. (Then the chunk table -- nb <= 1024 rows of
// ceil(n / 4096) + 1 u32 -- stays below 2^32 bytes: one buffer window in bin_part.)
constexpr u64 kBinMaxRecs = (1ull << 32) - 2ull * kATPB * (kAPer > kAPerPlain ? kAPer : kAPerPlain);
static_assert((u64)kATPB * (u64)kAPer >= 4096 && (u64)kMaxDigit * ((kBinMaxRecs + 4095) / 4096 + 1) * 4 < (1ull << 32),
              "the chunk table's window: chunks of >= 4096 records");
bool push_binnable(const glint_shard* s, i64 n) {
  return (u64)n < kBinMaxRecs && s->elems < ((i64)1 << 32) - 1;
}

int launch_validate_gate_binned(LaunchCtl* ctl, u64* gate, void* bc, u32* T, u32 nb, hipStream_t st) {
  push_validate_gate_binned_kernel<<<1, 256, 0, st>>>(ctl, gate, (BinCtl*)bc, T, nb);
  HIPCHK(hipGetLastError());
  return GLINT_OK;
}

// Front end of a binned push (0 plain, 1 plain + hot split, 2 chunk dedup + hot split), from what the
// last dedup push measured (the device reports m, the tail size and the cold records of each push
// through host-mapped words, taken at the shard's last sync point, so the choice does not depend on
// timing): chunk dedup when it kept < 80 % of the cold records it saw; otherwise the plain front end,
// with the hot-element split when the hot elements took >= 25 % of the tail (cfg3 ~65 %; cfg5's ~10 %
// does not pay for the sampling launch and the per-record check). A dedup push re-measures every 16
// pushes (and the first one). GLINT_BIN_FRONT = dedup | hot | prep forces one (tests).
int bin_front(glint_shard* s) {
  {
    const u64 w = s->hint_bin;
    const u32 m = (u32)(w >> 32), tail = (u32)w;
    const u32 cold = (u32)s->hint_bin_cold;
    if (tail > 0 && s->hint_bin_front == 2) {
      s->bin_chunk_ratio = cold ? (double)m / (double)cold : 1.0;
      s->bin_hot_frac = 1.0 - (double)cold / (double)tail;
    }
  }
  const bool probe = (s->bin_pushes++ & 15) == 0;
  const int front = probe || s->bin_chunk_ratio < 0.8 ? 2 : (s->bin_hot_frac >= 0.25 ? 1 : 0);
  static EnvKnob front_knob("GLINT_BIN_FRONT");
  const int forced = (int)front_knob.get([](const char* e) -> long long {
    if (!e) return -1;
    if (!strcmp(e, "dedup")) return 2;
    if (!strcmp(e, "hot")) return 1;
    if (!strcmp(e, "prep")) return 0;
    return -1;
  });
  return forced >= 0 ? forced : front;
}

// The wide hot table (front 1) is sampled every kHotEvery-th push and kept in between: a push's hot
// set only decides how much work leaves the partition path (any set gives the same sums), and a
// Zipf-like stream keeps its hot elements from push to push. A shard coming from another front end
// samples at once. (tests/test_gpu_parity.py::test_binned_stream_of_batches pushes a stream of
// different batches through the kept table.)
constexpr u32 kHotEvery = 8;
constexpr u32 kWideMin = 3;  // samples (of 262 144) that make an element hot in the wide table
constexpr u32 kHotMin = 2;   // samples (of 16 384) that make an element hot in the dedup front end's table

template <typename V, bool MAT>
int push_binned(glint_shard* s, const PushArgs<V>& a, bool from_break, hipStream_t st, const BinHook* hook,
                LaunchCtl* whole_next) {
  typedef typename LdsAcc<V>::T A;
  const i64 n = a.n;
  if (!push_binnable(s, n)) return GLINT_EINVAL;
  const int front = bin_front(s);
  const bool dedup = front == 2;
  bool hot_refresh = true;
  if (front == 1) {
    hot_refresh = s->bin_last_front != 1 || s->hot_age == 0 || s->hot_age >= kHotEvery;
    s->hot_age = hot_refresh ? 1u : s->hot_age + 1u;
  }
  s->bin_last_front = front;
  // a small push (at most ~4 fine items per CU, cfg5) plans its buckets inside bin_fsort
  const bool small_push =
      (i64)bin_geometry(s->elems, kCoarseBitsMin).nb + n / ((i64)kSTPB * kSPerSmall) + 1 <= (i64)4 * s->cus;
  // records per thread of a partition chunk: 8 for a large push's plain front end, 4 otherwise (the hot
  // and dedup tables share the LDS; a small push wants more chunks)
  const int per = front == 0 && !small_push ? kAPerPlain : kAPer;
  // Coarse buckets: 128 for chunks of 8 records per thread, 64 for chunks of 4 -- runs of ~64 records
  // per bucket and chunk either way, which the fine sort gathers. Same box, 2 rounds
  // (profiles/r06/ab_chunk_local.txt): 64 buckets for every push took cfg5 0.316 -> 0.303 ms and cfg3
  // 0.965 -> 0.956, but cfg4b (8-record chunks) 1.85 -> 1.93.
  const BinGeom g = bin_geometry(s->elems, per == kAPerPlain ? kCoarseBitsMin : kCoarseBitsMin - 1u);
  const u32 kchunk = (u32)kATPB * (u32)per;
  const i64 nchunks_max = (n + kchunk - 1) / kchunk;
  // partition workgroups per CU: what fits at once (the hot front end's LDS table allows fewer)
  static const int hot_occ = resident_per_cu(bin_part_kernel<V, MAT, true, 0, false>, kATPB);
  const int wpc = dedup ? kPartWgPerCuDedup : front == 1 ? std::min(kPartWgPerCuPlain, hot_occ) : kPartWgPerCuPlain;
  const u32 G = (u32)std::max<i64>(1, std::min<i64>(nchunks_max, (i64)s->cus * wpc));
  const u32 item = (u32)kSTPB * (small_push ? kSPerSmall : kSPerLarge);
  const i64 max_fitems = (i64)g.nb + n / item + 1;
  // apply units: a slab's units close at kUnitCap records or kRunMax runs, so at most
  // floor(H / cap) + floor(runs / kRunMax) + 1 per non-empty slab
  const i64 max_units = (i64)g.nslab + n / kUnitCap + std::min<i64>(n, max_fitems * g.nf) / kRunMax + 1;
  // The chunk table (a spare row past the last chunk), the buckets' chunk prefixes P and places Q, Bb,
  // Ib, the fine items and their first chunks, off2, the apply units, the dedup front end's hot tags and
  // the record buffers (coarse: u32 address + A value; fine: u16 slab offset + A value). The
  // [BinCtl | T] headers and the hot front end's tables live in buffers of their own (stable
  // addresses: emptied by the kernels of the push before, not by memsets)
  const u32 nstride = (u32)nchunks_max, ctstride = nstride + 1;  // (a spare column past the last chunk)
  const size_t b_ct = pad256((size_t)ctstride * g.nb * 4);
  const size_t b_pq = pad256((size_t)g.nb * (nstride + 1) * 4) + pad256((size_t)g.nb * nstride * 4);
  const size_t b_nb = pad256((size_t)g.nb * 4);
  const size_t b_fit = 2 * pad256((size_t)max_fitems * 8);
  const size_t b_off2 = pad256((size_t)max_fitems * (g.nf + 1) * 4);
  const size_t b_units = pad256((size_t)max_units * 16) + pad256((size_t)max_units * kRunMax * 8);
  const size_t b_hot = pad256((size_t)kHotSlots * 4);
  const size_t b_wpart = front == 1 ? pad256((size_t)G * kWideSlots * sizeof(A)) : 0;
  const size_t b_a = pad256((size_t)n * 4), b_v = pad256((size_t)n * sizeof(A)), b_e = pad256((size_t)n * 2);
  const size_t need = b_ct + b_pq + 2 * b_nb + b_fit + b_off2 + b_units + b_hot + b_wpart + b_a + 2 * b_v + b_e;
  int rc = grow(&s->d_bin, &s->bin_bytes, need);
  if (rc) return rc;
  constexpr size_t kHdr = 12288;  // one [BinCtl (256 B) | T (<= kMaxDigit u32) | done (<= kMaxDigit u32)] header
  static_assert(256 + 8 * kMaxDigit <= kHdr && sizeof(BinCtl) <= 256, "header slot");
  if (!s->d_binctl) {
    if (hipMalloc(&s->d_binctl, 2 * kHdr) != hipSuccess) {
      (void)hipGetLastError();
      s->d_binctl = nullptr;
      return GLINT_ENOMEM;
    }
    HIPCHK(hipMemsetAsync(s->d_binctl, 0, 2 * kHdr, st));
    s->bin_par = 0;
  }
  const size_t b_wk = ((size_t)4 << kWideHashBits), b_wbest = (size_t)kWideSlots * 8;
  if (front == 1 && !s->d_hot) {  // keys empty, counts and picks zero; their readers keep them so
    if (hipMalloc(&s->d_hot, 2 * b_wk + b_wbest) != hipSuccess) {
      (void)hipGetLastError();
      s->d_hot = nullptr;
      return GLINT_ENOMEM;
    }
    HIPCHK(hipMemsetAsync(s->d_hot, 0xFF, b_wk, st));
    HIPCHK(hipMemsetAsync((char*)s->d_hot + b_wk, 0, b_wk + b_wbest, st));
  }
  char* const hdr = (char*)s->d_binctl + (size_t)s->bin_par * kHdr;
  char* const nhdr = (char*)s->d_binctl + (size_t)(s->bin_par ^ 1) * kHdr;
  BinCtl* bc = (BinCtl*)hdr;
  u32* T = (u32*)(hdr + 256);
  u32* done = T + kMaxDigit;  // the fused plan: items of each bucket sorted so far
  char* p = (char*)s->d_bin;
  u32* ct = (u32*)p;
  p += b_ct;
  u32* P = (u32*)p;
  u32* Q = (u32*)(p + pad256((size_t)g.nb * (nstride + 1) * 4));
  p += b_pq;
  u32* Bb = (u32*)p;
  u32* Ib = (u32*)(p + b_nb);
  p += 2 * b_nb;
  uint2* fitems = (uint2*)p;
  uint2* cwin = (uint2*)(p + pad256((size_t)max_fitems * 8));
  p += b_fit;
  u32* off2 = (u32*)p;
  p += b_off2;
  uint4* units = (uint4*)p;
  uint2* runs = (uint2*)(p + pad256((size_t)max_units * 16));
  p += b_units;
  u32* hot_tags = (u32*)p;
  p += b_hot;
  u32* wkey = front == 1 ? (u32*)s->d_hot : nullptr;
  u32* wcnt = front == 1 ? (u32*)((char*)s->d_hot + b_wk) : nullptr;
  unsigned long long* wbest = front == 1 ? (unsigned long long*)((char*)s->d_hot + 2 * b_wk) : nullptr;
  A* wpart = (A*)p;
  p += b_wpart;
  u32* addr_a = (u32*)p;
  A* val_a = (A*)(p + b_a);
  A* val_b = (A*)(p + b_a + b_v);
  uint16_t* e_b = (uint16_t*)(p + b_a + 2 * b_v);

  ProfScope ps(s, GLINT_K_PUSH_BINNED, st);
  const int fb = from_break ? 1 : (hook && whole_next ? 2 : 0);
  if (front == 1 && hot_refresh) {  // the wide hot table: sample, count, pick (the count table starts empty)
    HIPCHK(hipMemsetAsync(wbest, 0, b_wbest, st));  // the picks of the pushes before (kept for reuse)
    bin_hot_sample_kernel<MAT><<<kWideSampleWgs, 256, 0, st>>>(a.keys, a.cols, n, a.part, a.ctl, a.ntiles, fb, wkey,
                                                                wcnt);
    HIPCHK(hipGetLastError());
    bin_hot_select_kernel<<<(1u << kWideHashBits) / 256u, 256, 0, st>>>(wkey, wcnt, kWideMin, wbest);
    HIPCHK(hipGetLastError());
  }
  // (a validating push's dedup front end sums no hot elements: they would reach the shard before its
  // verdict)
  const bool dedup_hot = dedup && !hook;
  if (dedup_hot) {
    bin_hot_pick_kernel<MAT><<<1, kHotTPB, 0, st>>>(a.keys, a.cols, n, a.part, a.ctl, a.ntiles, fb, kHotMin, hot_tags);
    HIPCHK(hipGetLastError());
  }
  BinCtl* const nbc = (BinCtl*)nhdr;
  u32* const nT = (u32*)(nhdr + 256);
  LaunchCtl* const vctl = hook ? a.ctl : nullptr;
  // (hook: a validating gated push, whose partition validates the tail records)
  if (dedup) {
    auto kern = a.part.kind == 0 ? (hook ? bin_part_dedup_kernel<V, MAT, 0, true> : bin_part_dedup_kernel<V, MAT, 0, false>)
                                 : (hook ? bin_part_dedup_kernel<V, MAT, -1, true> : bin_part_dedup_kernel<V, MAT, -1, false>);
    kern<<<G, kATPB, 0, st>>>(a.keys, a.cols, a.vals, n, a.part, a.ctl, a.ntiles, fb, g, addr_a, val_a, a.err, bc, ct, ctstride,
                              dedup_hot ? hot_tags : nullptr, a.data, nbc, nT, vctl, whole_next);
  } else {
    auto pick = [&](auto pp, auto vv) {
      constexpr int PP = decltype(pp)::value;
      constexpr bool VV = decltype(vv)::value;
      return a.part.kind == 0 ? (front == 1 ? bin_part_kernel<V, MAT, true, 0, VV> : bin_part_kernel<V, MAT, false, 0, VV, PP>)
                              : (front == 1 ? bin_part_kernel<V, MAT, true, -1, VV> : bin_part_kernel<V, MAT, false, -1, VV, PP>);
    };
    auto pick2 = [&](auto vv) {
      return per == kAPerPlain ? pick(std::integral_constant<int, kAPerPlain>{}, vv) : pick(std::integral_constant<int, kAPer>{}, vv);
    };
    auto kern = hook ? pick2(std::true_type{}) : pick2(std::false_type{});
    kern<<<G, kATPB, 0, st>>>(a.keys, a.cols, a.vals, n, a.part, a.ctl, a.ntiles, fb, g, addr_a, val_a, a.err, bc, ct, ctstride,
                              wbest, wpart, nbc, nT, vctl, whole_next);
  }
  HIPCHK(hipGetLastError());
  s->bin_par ^= 1;  // this push's header is [hdr]; bin_part zeroed the other one for the next push
  if (hook) {  // the verdict (and a rejected batch's cancel) and the head's apply, before anything is applied
    rc = (*hook)(bc, T, g.nb);
    if (rc) return rc;
  }
  // (front 1: the hot split's sums added by the same launch's workgroups past the buckets)
  const u32 red = front == 1 ? (u32)(kWideSlots / kRedSlots) : 0u;
  bin_scan_kernel<V><<<g.nb + red, kScanTPB, 0, st>>>(g, ct, ctstride, n, a.ctl, a.ntiles, fb, kchunk, nstride, bc, T,
                                                      Bb, Ib, fitems, cwin, P, Q, item, wbest, G, wpart, a.data, vctl);
  HIPCHK(hipGetLastError());
  // Groups of sparse slabs for vector shards; a matrix shard's sparse slabs stay units of their own: its
  // records cluster in a slab's few hot rows, and grouping cost cfg5 0.309 -> 0.337 ms while it takes
  // cfg3 1.077 -> 1.038 (profiles/r05/ab_group_unitcap.txt).
  const int group_on = MAT ? 0 : 1;
  // The plan fused into bin_fsort for a push of at most ~4 items per CU (cfg5's 641), where the plan
  // launch and its tail are a real share of the push; with many items per CU every item's wait for its
  // stores before counting itself in costs more: cfg3 1.067 -> 1.078, cfg4b 2.375 -> 2.44 ms, cfg5
  // 0.347 -> 0.335 (profiles/r05/ab_fused_plan.txt)
  // (fused for every push, with the fine sort at two workgroups per CU: cfg4b 2.15 -> 2.50 ms, cfg3 1.02
  // -> 1.04, profiles/r06/ab_fuse_all.txt; again with 16-record items at two per CU: cfg4b 2.14 -> 2.35,
  // cfg3 1.029 -> 1.028)
  const bool fused = small_push;
  u64* const bhint = s->d_hint ? s->d_hint + 1 : nullptr;
  u64* const whint = whole_next ? s->d_hint : nullptr;
  if (fused) {
    bin_fsort_kernel<A, true, kSPerSmall><<<(unsigned)max_fitems, kSTPB, 0, st>>>(g, fitems, bc, T, Bb, addr_a, val_a, e_b, val_b,
                                                                      off2, bhint, whint, (u32)n, Ib, done, units, runs,
                                                                      group_on, item, cwin, P, Q, nstride);
    HIPCHK(hipGetLastError());
  } else {
    bin_fsort_kernel<A, false, kSPerLarge><<<(unsigned)max_fitems, kSTPB, 0, st>>>(g, fitems, bc, T, Bb, addr_a, val_a, e_b, val_b,
                                                                       off2, bhint, whint, (u32)n, Ib, done, units, runs,
                                                                       group_on, item, cwin, P, Q, nstride);
    HIPCHK(hipGetLastError());
    bin_plan_kernel<<<g.nb * GLINT_PLAN_SPLIT, kPlanTPB, 0, st>>>(g, T, Bb, Ib, off2, bc, units, runs, group_on, item);
    HIPCHK(hipGetLastError());
  }
  // a persistent grid of the resident workgroups: each pipelines its units two deep, in XCD-grouped
  // order (see bin_apply2_kernel)
  static const int apply2_occ = resident_per_cu(bin_apply2_kernel<V>, kCTPB);
  const unsigned apply2_grid = (unsigned)std::min<i64>(max_units, (i64)s->cus * apply2_occ);
  bin_apply2_kernel<V><<<apply2_grid, kCTPB, 0, st>>>(e_b, val_b, units, runs, bc, s->elems, a.data,
                                                      apply2_grid % 8 == 0 ? 1 : 0, g.nf);
  HIPCHK(hipGetLastError());
  return GLINT_OK;
}

#define GLINT_INST(V, MAT) \
  template int push_binned<V, MAT>(glint_shard*, const PushArgs<V>&, bool, hipStream_t, const BinHook*, LaunchCtl*);
GLINT_INST(int, false)
GLINT_INST(int, true)
GLINT_INST(long long, false)
GLINT_INST(long long, true)
GLINT_INST(float, false)
GLINT_INST(float, true)
GLINT_INST(double, false)
GLINT_INST(double, true)
#undef GLINT_INST

}  // namespace glint

#ifdef GLINT_BIN_PROF
// tuning build only: the summed phase clocks (and reset)
extern "C" int glint_debug_bin_prof(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(glint::g_bin_prof), sizeof(glint::g_bin_prof)) != hipSuccess) return 1;
  if (reset) {
    static unsigned long long z[64] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(glint::g_bin_prof), z, sizeof(z)) != hipSuccess) return 1;
  }
  return 0;
}
#endif
