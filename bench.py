#!/usr/bin/env python3
"""Device-resident push scatter-add benchmark (BASELINE.json metric).

One step = one push of a batch of (key, value) records that is already resident in HBM into the
rank's HBM shard: `glint_vec_push_dev` (include/glint_gpu.h), i.e. PartialVector.update
(src/main/scala/glint/models/server/PartialVector.scala:35-43) on the GPU.

Workload (default): BASELINE.json north_star -- 1 GPU, 2^30-key Double vector, dense contiguous
push scatter-add (keys[i] = start + i, values U[-1,1) from seed 42): the configuration its >= 70 %
of HBM roofline target is quoted on. With N GPUs (torchrun), the key space is
RangePartitioner(N, N * 2^30) and every rank pushes its own dense range (cfg4a: clients own
contiguous key ranges, no exchange step) -- weak scaling, no collective in the timed region.
The default 1-GPU run also measures BASELINE.json configs[1] (2^28 keys, the extra key `cfg2_2p28`).

Algorithmic bytes per record: 8 (key) + 8 (value) + 8 + 8 (shard read + write)
= 32 B; value = all ranks' algorithmic bytes / max-over-ranks wall time of the K timed steps.
The roofline figure uses the push kernels' own device time from HIP events carried on each launch
on its stream (glint_prof_*); PMC HBM traffic comes from profiles/ when present.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--log2-keys 30]
                    [--pattern dense|zipf|matrix|exchange|pull|rowpull] [--scaling weak|strong]

--gpus N without torchrun starts N worker processes itself (one per GPU, before touching any GPU);
under torchrun (WORLD_SIZE set) every process is one rank.

--pattern matrix is BASELINE.json configs[4] per GPU (weak scaling): a 2^17-row x 512-col Double
shard of RangePartitioner(N, N * 2^17) rows (8 x 2^17 = the 2^20-row matrix at N = 8), pushed
2^23 triplets (2^26 / 8) with rows Zipf(1.0) and cols uniform: PartialMatrix.update
(PartialMatrix.scala:74-83) through glint_mat_push_dev. Algorithmic bytes n(8+4+8) + 16U.

--pattern exchange is cfg4b: every rank pushes 2^26 uniform keys of the whole key space through
DistributedBigVector.push (route + all-to-all + local push, AsyncBigVector.scala:96-121); the
post-run check regenerates every rank's batches and compares the rank's shard with a torch fp64
segment sum, and U (distinct elements a shard receives) is counted, not estimated.

--batches K (push patterns): K batches of the same distribution from distinct seeds (the same
permutation of the shard, fresh Zipf / uniform samples and values), pre-generated in HBM and rotated
per step -- every push is a new message, as a server sees them (AsyncBigVector.scala:107-121) -- so
no state the binned push keeps across pushes (the hot table, the latched front-end and whole-push
hints) meets the same batch twice in a row. The post-run check replays all K batches.

At N > 1 the line carries `devices`: every rank's device index and PCI address (all-gathered), and a
run over RCCL fails if two ranks share a GPU.
"""
from __future__ import annotations

import argparse
import ctypes as C
import glob
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--log2-keys", type=int, default=None,
                    help="keys per GPU shard (default: 30 -- the north star -- for the weak-scaling dense push, "
                         "28 for every other pattern: cfg2 / cfg3 / cfg4b's shard)")
    ap.add_argument("--pattern", choices=["dense", "zipf", "matrix", "exchange", "pull", "rowpull"], default="dense",
                    help="dense: cfg2/cfg4a push; zipf: cfg3 push; matrix: cfg5 push per GPU (2^17 x 512 Double "
                         "rows, 2^23 Zipf(1.0)-row x uniform-col triplets); exchange: cfg4b push through the "
                         "route + all-to-all layer; pull: dense vector get (24 B/record); rowpull: cfg5 row pull "
                         "of 2^16 Zipf(1.0) rows (8200 B/row)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                    help="weak: 2^k keys per GPU (cfg4a); strong: one 2^k-key vector split over the GPUs")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline sample length")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-north-star", action="store_true",
                    help="skip the extra cfg2 (2^28) leg of the default 1-GPU run")
    ap.add_argument("--no-check", action="store_true", help="skip the post-run shard check")
    ap.add_argument("--batches", type=int, default=1,
                    help="push patterns: K different batches of the same distribution, rotated per step")
    ap.add_argument("--parts-per-gpu", type=int, default=1,
                    help="exchange only: range partitions hosted per GPU (modelsPerServer, Client.scala:63); "
                         "8 at one GPU is cfg4's own key space, RangePartitioner(8, 2^31)")
    return ap.parse_args()


def pmc_traffic(workload_tag: str):
    """Per-launch HBM bytes of the step's kernels, REPLAYED from the newest committed PMC summary for
    this workload (tools/pmc_traffic.py writes profiles/<round>/pmc_<tag>.json from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this same command); (None, None) without one.
    PMC counters cannot be read inside the timed run itself, so the source file is named."""
    files = sorted(glob.glob(str(ROOT / "profiles" / "*" / f"pmc_{workload_tag}.json")))
    if not files:
        return None, None, None
    try:
        d = json.loads(Path(files[-1]).read_text())
        return (d.get("hbm_bytes_per_launch"), "replayed from " + str(Path(files[-1]).relative_to(ROOT)),
                d.get("records_per_push"))
    except Exception:
        return None, None, None


def sparse_floor(workload_tag: str, ms_per_step: float):
    """The practical floor of a binned line, REPLAYED from the newest committed
    tools/microbench_sparse measurement (profiles/<round>/micro_sparse_floor.json): the time to stream
    the records once plus read-modify-write each distinct element once in ascending order, as if
    partitioning were free. frac = floor / ms_per_step; None for lines without one."""
    # (case, shard pushes per step): the 8-partition line's step is eight shard pushes, each floored alone
    case, per_step = {"zipf_2p28": ("cfg3", 1), "exchange_2p28": ("cfg4b", 1), "matrix_2p17x512": ("cfg5", 1),
                      "exchange_2p28_mps8": ("cfg4_mps8_shard", 8),
                      # the eight partitions in one slab: one push of the whole batch, cfg4b's floor
                      "exchange_2p28_mps8_slab": ("cfg4b", 1)}.get(workload_tag, (None, 1))
    files = [f for f in sorted(glob.glob(str(ROOT / "profiles" / "*" / "micro_sparse_floor.json")))
             if case and f'"{case}"' in Path(f).read_text()]
    if not case or not files:
        return None
    try:
        for d in json.loads(Path(files[-1]).read_text())["cases"]:
            if d.get("case") == case:
                floor = d["floor_ms"] * per_step
                return {"floor_ms": round(floor, 4), "frac": round(floor / ms_per_step, 4),
                        "read_ms": round(d["read_ms"] * per_step, 4),
                        "rmw_sorted_ms": round(d["rmw_sorted_ms"] * per_step, 4),
                        "shard_pushes_per_step": per_step,
                        "source": "replayed from " + str(Path(files[-1]).relative_to(ROOT))}
    except Exception:
        return None
    return None


def cpu_baseline(log2_keys: int, seconds: float):
    """The oracle's scalar PartialVector.update loop (one thread = one actor) on a bounded sample of
    the same dense workload, timed on this host."""
    import numpy as np
    from oracle import oracle as O
    n = 1 << min(log2_keys, 26)
    keys = np.arange(n, dtype=np.int64)
    vals = np.random.default_rng(42).uniform(-1, 1, n)
    data = np.zeros(n, np.float64)
    O.vec_update_f64_parallel([0], [n], [data], [keys], [vals], 1)  # warm (page-in)
    passes, t0 = 0, time.perf_counter()
    while True:
        O.vec_update_f64_parallel([0], [n], [data], [keys], [vals], 1)
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    gbs = 32.0 * n * passes / el / 1e9
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    out = {"value": round(gbs, 3), "unit": "GB/s", "cores": 1, "kind": "port",
           "host_cores": os.cpu_count(), "cores_available_to_process": avail,
           "sample": f"{passes} x PartialVector[Double].update of 2^{min(log2_keys, 26)} dense records "
                     f"(oracle/glint_oracle.c scalar loop, 1 thread = 1 actor), {el:.1f} s"}
    # the same sample as P = 8 range shards (cfg4's partition count), one actor thread per shard on
    # min(P, host cores) threads
    P = 8
    threads = max(1, min(P, avail))
    q = n // P
    starts, ends = [i * q for i in range(P)], [(i + 1) * q for i in range(P)]
    datas = [data[i * q:(i + 1) * q] for i in range(P)]
    ks = [keys[i * q:(i + 1) * q] for i in range(P)]
    vs = [vals[i * q:(i + 1) * q] for i in range(P)]
    O.vec_update_f64_parallel(starts, ends, datas, ks, vs, threads)
    passes, t0 = 0, time.perf_counter()
    while True:
        O.vec_update_f64_parallel(starts, ends, datas, ks, vs, threads)
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds / 2:
            break
    # BASELINE.json configs[0]: 1 client + 2 loopback servers, 1M-key Double vector, dense push in
    # <= 1000-record messages with the exactly-once protocol, then a pull of every key
    # (tools/loopback/glint_loopback.c with the oracle's server loop as the shard)
    try:
        import subprocess
        from glint_amd.build import LOOPBACK_BIN, ORACLE_LIB
        r = subprocess.run([str(LOOPBACK_BIN), "--backend", "oracle", "--lib", str(ORACLE_LIB)],
                           capture_output=True, text=True, timeout=120)
        out["cfg1_loopback"] = json.loads(r.stdout.strip().splitlines()[-1])
    except Exception as e:  # the baseline is reported, never required
        out["cfg1_loopback"] = {"error": str(e)[:200]}
    out["parallel"] = {"value": round(32.0 * q * P * passes / el / 1e9, 3), "unit": "GB/s", "cores": threads,
                       "sample": f"{passes} x 2^{min(log2_keys, 26)} dense records over {P} shards, "
                                 f"one thread per shard on {threads} threads, {el:.1f} s"}
    return out


def spawn_ranks(n: int) -> int:
    """`python bench.py --gpus N` without a launcher: start N worker processes (one per GPU, the
    torchrun environment contract: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*) before this process
    touches any GPU, relay their output (rank 0 prints the JSON line) and exit with the worst code."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:], env=env))
    codes = [p.wait() for p in procs]
    return max(codes, key=abs)


def zipf_rows(rng, n: int, count: int):
    """Zipf(1.0) ranks over [0, n) (word frequency; inverse CDF of the 1/k law)."""
    import numpy as np
    return np.minimum(np.floor(np.power(float(n), rng.random(count))).astype(np.int64) - 1, n - 1)


def segment_sums(v, counts, chunk: int = 1 << 22):
    """torch.segment_reduce(v, "sum", lengths=counts), in pieces of at most 2^22 segments: on this
    ROCm build one call over ~59 M segments (cfg4b) returned zeros past the first ~9 M."""
    import torch
    out, o = [], 0
    for i in range(0, counts.numel(), chunk):
        c = counts[i:i + chunk]
        m = int(c.sum())
        out.append(torch.segment_reduce(v[o:o + m], "sum", lengths=c))
        o += m
    return torch.cat(out) if out else v[:0]


def run_line(ctx, pat: str, log2_keys: int, scaling: str, steps: int, warmup: int, check: bool,
             mps: int = 1, nb: int = 1) -> dict:
    """Builds the workload of one bench line, times `steps` pushes (or pulls) after `warmup`, checks
    the shard afterwards and returns the line's fields (without the CPU baseline)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from glint_amd import PartialMatrix, PartialVector, RangePartitioner
    from glint_amd import _native as N

    lib, dev, world, rank, backend = ctx["lib"], ctx["dev"], ctx["world"], ctx["rank"], ctx["backend"]
    local = dev.index
    exch = pat == "exchange"
    mat = pat in ("matrix", "rowpull")
    strong = scaling == "strong"
    cols_n = 512
    if mat:
        partitioner = RangePartitioner.apply(world, world * (1 << 17))
    elif exch:  # modelsPerServer partitions per rank (rank r hosts r, r + W, ...: Client.scala:71-85)
        partitioner = RangePartitioner.apply(world * mps, world * mps * (1 << log2_keys))
    elif strong:  # total work fixed: one 2^k-key vector range-sharded over the ranks
        partitioner = RangePartitioner.apply(world, 1 << log2_keys)
    else:
        partitioner = RangePartitioner.apply(world, world * (1 << log2_keys))
    if exch:
        from glint_amd.dist import Router
        my_parts = [partitioner.all()[p] for p in Router(partitioner, world).rank_parts[rank]]
    else:
        my_parts = [partitioner.all()[rank]]
    part = my_parts[0]
    slab = None
    if exch and mps > 1:  # the rank's partitions as views of one slab (dist.slab_shards)
        from glint_amd.dist import slab_shards
        sv = slab_shards("vector", my_parts, 0, "double", local)
        if sv is not None:
            slab, shards = sv
    if slab is None:
        shards = [PartialMatrix(p, cols_n, "double", device=local) if mat else PartialVector(p, "double", device=local)
                  for p in my_parts]
    handles = shards + ([slab] if slab is not None else [])  # every shard a push may launch on
    shard = shards[0]
    n = part.size
    gen = torch.Generator(device=dev)
    gen.manual_seed(42 + rank)
    cols = out = None
    push = pat in ("dense", "zipf", "matrix", "exchange")
    how = ""  # the exchange line's push path (named below)
    scope = "per GPU" if not strong else f"1/{world} of the vector per GPU"
    fill_v = None
    u_note = ""
    batches = []  # [(keys, cols, vals, distinct elements)] of --batches K
    if pat == "matrix":
        # cfg5: rows Zipf(1.0) through a seeded permutation of the shard's rows, cols uniform [0, 512)
        rng = np.random.default_rng(42 + rank)
        nrec = 1 << 23
        perm = rng.permutation(n)
        for b in range(nb):
            rb = rng if b == 0 else np.random.default_rng(100042 + 1000 * b + rank)
            r = perm[zipf_rows(rb, n, nrec)].astype(np.int64)
            c = rb.integers(0, cols_n, nrec).astype(np.int32)
            batches.append((torch.from_numpy(r + part.start).to(dev), torch.from_numpy(c).to(dev),
                            torch.rand(nrec, dtype=torch.float64, device=dev, generator=gen) * 2 - 1,
                            int(np.unique(r * cols_n + c).size)))
        keys, cols, vals, uniq = batches[0]
        uniq = int(np.mean([bt[3] for bt in batches]))
        tag = "matrix_2p17x512"
        bytes_per_step = 20.0 * nrec + 16.0 * uniq  # n(8+4+8) + U(8+8)
        workload = (f"cfg5 per GPU: {nrec} Zipf(1.0)-row x uniform-col triplets into a 2^17 x 512 Double "
                    f"matrix shard of RangePartitioner({world}, {world}x2^17) rows")
    elif pat == "rowpull":
        # cfg5 row pull: r = 2^16 Zipf(1.0) rows (PartialMatrix.getRows, PartialMatrix.scala:37-46)
        # from a 2^17 x 512 Double shard filled by one dense row-major push beforehand
        rng = np.random.default_rng(42 + rank)
        nrec = 1 << 16
        keys = torch.from_numpy(rng.permutation(n)[zipf_rows(rng, n, nrec)].astype(np.int64) + part.start).to(dev)
        fill_r = torch.arange(part.start, part.end, dtype=torch.int64, device=dev).repeat_interleave(cols_n)
        fill_c = torch.arange(cols_n, dtype=torch.int32, device=dev).repeat(n)
        fill_v = torch.rand(n * cols_n, dtype=torch.float64, device=dev, generator=gen)
        shard.update(fill_r, fill_c, fill_v)
        del fill_r, fill_c
        out = torch.empty((nrec, cols_n), dtype=torch.float64, device=dev)
        vals = None
        uniq = nrec
        tag = "rowpull_2p17x512"
        bytes_per_step = (8.0 + 2.0 * cols_n * 8) * nrec  # 8 200 B per row
        workload = (f"cfg5 row pull per GPU: {nrec} Zipf(1.0) rows of a 2^17 x 512 Double matrix shard "
                    f"(getRows, flattened rows x cols)")
    elif exch:
        # cfg4b: every rank's batch holds keys of every rank's range (uniform over the whole key
        # space), so each push is route + gather (glint_route_gather_dev) + all_to_all_single + the
        # local push. Keys and values come from per-rank generators that every rank can replay.
        from glint_amd.dist import DistributedBigVector
        dv = DistributedBigVector(partitioner, shards, partitioner.size, np.float64, None, dev, slab=slab)
        nrec = 1 << 26

        def batch(src, b=0):
            kg = torch.Generator(device=dev)
            kg.manual_seed(1042 + src + 100000 * b)
            vg = torch.Generator(device=dev)
            vg.manual_seed(2042 + src + 100000 * b)
            k = torch.randint(0, partitioner.size, (nrec,), dtype=torch.int64, device=dev, generator=kg)
            return k, torch.rand(nrec, dtype=torch.float64, device=dev, generator=vg) * 2 - 1

        for b in range(nb):
            kb, vb = batch(rank, b)
            batches.append((kb, None, vb, None))
        keys, vals = batches[0][0], batches[0][2]
        # distinct elements a rank receives per push: counted over all ranks' batches by the check,
        # the expected value until then
        P = world * mps
        uniq = int(mps * n * (1.0 - np.exp(-nrec / (P * n) * world)))
        u_note = " (U estimated)"
        tag = f"exchange_2p{log2_keys}" + (f"_mps{mps}" if mps > 1 else "")
        bytes_per_step = 16.0 * nrec + 16.0 * uniq
        # the path DistributedBigVector.push takes (dist.py: _push_gated, _push_set, _push_slab, the route)
        set_path = slab is None and 1 < mps <= 64 and nrec * 8 < mps * n
        if world == 1 and mps == 1:
            how = "one validating push (the push checks the keys), no route"
        elif slab is not None and world == 1:
            how = f"the rank's {mps} partitions in one slab: one validating push, no route"
        elif slab is not None:
            how = f"route (keys rebased into each rank's slab) + RCCL all-to-all + one slab push per rank"
        elif set_path and world == 1:
            how = f"one validated scatter over the {mps} local shards (glint_vec_push_dev_shards), no route"
        elif set_path:
            how = (f"route + RCCL all-to-all + one validated scatter over the rank's {mps} shards "
                   f"(glint_vec_push_dev_shards)")
        else:
            how = "route + gather + RCCL all-to-all + local push" + ("es" if mps > 1 else "")
        workload = (f"cfg4b: {world} GPU(s), {nrec} uniform keys per rank over RangePartitioner({P}, "
                    f"{partitioner.size}), {mps} partition(s) per GPU; {how}")
    elif pat in ("dense", "pull"):
        keys = torch.arange(part.start, part.end, dtype=torch.int64, device=dev)
        vals = torch.rand(n, dtype=torch.float64, device=dev, generator=gen) * 2 - 1
        nrec, uniq = n, n
        if pat == "dense":  # K batches: the same keys, fresh values
            batches = [(keys, None, vals, n)] + [
                (keys, None, torch.rand(n, dtype=torch.float64, device=dev, generator=gen) * 2 - 1, n)
                for _ in range(nb - 1)]
        if pat == "pull":  # PartialVector.get (PartialVector.scala:51-60) of every key of the shard
            shard.update(keys, vals)
            out = torch.empty(n, dtype=torch.float64, device=dev)
            tag = f"pull_2p{log2_keys}"
            bytes_per_step = 24.0 * nrec  # key 8 + element 8 + out 8
            workload = f"dense pull (get) of every key, 2^{n.bit_length() - 1}-key Double shard {scope}"
        else:
            tag = f"dense_2p{log2_keys}"
            bytes_per_step = 32.0 * nrec  # key 8 + value 8 + element read 8 + write 8
            if strong:
                workload = (f"strong scaling: one 2^{log2_keys}-key Double vector, RangePartitioner({world}, "
                            f"2^{log2_keys}); each rank pushes its own dense range")
            elif world == 1 and log2_keys == 30:
                workload = ("north star: dense contiguous-range push scatter-add, 2^30-key Double vector per GPU "
                            "(BASELINE.json north_star's 1-GPU target configuration)")
            elif world == 1:
                workload = f"cfg2: dense contiguous-range push, 2^{log2_keys}-key Double vector per GPU"
            else:
                workload = (f"cfg4a: {world} GPUs, RangePartitioner({world}, {world}x2^{log2_keys}), "
                            f"each rank pushes its own dense range")
    else:
        # cfg3: Zipf(1.1) ranks mapped through a seeded permutation of the shard, n = N/4 records
        rng = np.random.default_rng(42 + rank)
        nrec = n // 4
        ranks = rng.zipf(1.1, size=int(nrec * 1.3))
        ranks = ranks[ranks <= n][:nrec] - 1
        nrec = ranks.size
        perm = rng.permutation(n)
        for b in range(nb):
            if b:  # a fresh sample of the same law, the same number of records
                rb = np.random.default_rng(100042 + 1000 * b + rank)
                ranks = rb.zipf(1.1, size=int(nrec * 1.4))
                ranks = ranks[ranks <= n][:nrec] - 1
                assert ranks.size == nrec
            k = perm[ranks].astype(np.int64) + part.start
            batches.append((torch.from_numpy(k).to(dev), None,
                            torch.rand(nrec, dtype=torch.float64, device=dev, generator=gen) * 2 - 1,
                            int(np.unique(k).size)))
        keys, _, vals, _ = batches[0]
        uniq = int(np.mean([bt[3] for bt in batches]))
        tag = f"zipf_2p{log2_keys}"
        bytes_per_step = 16.0 * nrec + 16.0 * uniq
        workload = f"cfg3: Zipf(1.1) push of {nrec} records into a 2^{log2_keys}-key Double shard"
    stream = torch.cuda.current_stream(dev).cuda_stream
    h = shard.handle
    nstep = [0]  # pushes so far: step s pushes batch s % K

    def step():
        nonlocal keys, cols, vals
        if batches:
            keys, cols, vals = batches[nstep[0] % len(batches)][:3]
        nstep[0] += 1
        if exch:
            dv.push(keys, vals)
            return
        if pat == "matrix":
            rc = lib.glint_mat_push_dev(h, keys.data_ptr(), cols.data_ptr(), vals.data_ptr(), nrec, 0, stream)
        elif pat == "rowpull":
            rc = lib.glint_mat_pull_rows_dev(h, keys.data_ptr(), out.data_ptr(), nrec, stream)
        elif pat == "pull":
            rc = lib.glint_vec_pull_dev(h, keys.data_ptr(), out.data_ptr(), nrec, stream)
        else:
            rc = lib.glint_vec_push_dev(h, keys.data_ptr(), vals.data_ptr(), nrec, 0, stream)
        if rc:
            raise RuntimeError(N.strerror(rc))

    for _ in range(warmup):
        step()
        # one push at a time, each ended by the shard's sync point: the adaptive tail switch decides
        # from the previous push's tail as published at its sync, so the timed pushes take the path
        # the warm-up settled on (and its one-time scratch allocation lands in the warm-up)
        for sh in handles:
            sh.sync(stream)
    for sh in handles:
        sh.sync(stream)
        lib.glint_prof_reset(sh.handle)
        lib.glint_prof_enable(sh.handle, 1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    for sh in handles:
        lib.glint_prof_enable(sh.handle, 0)
        sh.sync(stream)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    def kernel_avg(kid):
        """Device time of one kernel kind per step (a large push runs its check and apply as one
        launch per window of records: the launches of a step are summed) and its launch count."""
        tot_ms, tot_n = 0.0, 0
        for sh in handles:  # every local shard's launches of this kind (the exchange line may host several)
            ms, cnt = C.c_double(), C.c_int64()
            lib.glint_prof_read(sh.handle, kid, C.byref(ms), C.byref(cnt))
            tot_ms, tot_n = tot_ms + ms.value, tot_n + cnt.value
        return tot_ms / steps, tot_n

    # post-run check. Dense push: the shard holds (W+K) additions of each record, bit-exact (each
    # key once per push, the ordered path). Zipf / matrix / exchange: repeated keys sum in an
    # unordered way, so the check is a torch fp64 segment sum of one push (of every rank's batch,
    # for the exchange) times (W+K), within the north star's 1e-6 relative. Pulls: the pulled values
    # equal what was pushed, bit for bit (a row pull: the dense fill's rows).
    ok = None
    reps = warmup + steps
    # pushes of each batch: step s pushed batch s % K
    times = [len(range(b, reps, len(batches))) for b in range(len(batches))] if batches else [reps]
    recv = nrec  # records this rank's shard takes per push
    if check:
        if pat == "dense":
            acc = torch.zeros_like(vals)
            for s_ in range(reps):  # (in push order: the same rounding as the shard's ordered adds)
                acc += batches[s_ % len(batches)][2]
            ok = bool(torch.equal(shard.get(keys), acc))
            del acc
        elif pat == "pull":
            ok = bool(torch.equal(out, vals))
        elif pat == "rowpull":
            ok = bool(torch.equal(out, fill_v.view(n, cols_n)[keys - part.start]))
        else:
            # every batch's records (value x the times it was pushed), in addresses local to the shard
            # (exchange: to the concatenation of the rank's shards, shard j's elements at j * n ...)
            addr_l, val_l = [], []
            recv_b = []
            for b, tb in enumerate(times):
                if exch:
                    # every rank's batch b, replayed: the records of this rank's partitions
                    r0 = sum(int(x.numel()) for x in addr_l)
                    for src in range(world):
                        k_s, v_s = (batches[b][0], batches[b][2]) if src == rank else batch(src, b)
                        for j, p in enumerate(my_parts):
                            m = (k_s >= p.start) & (k_s < p.end)
                            addr_l.append(k_s[m] - p.start + j * n)
                            val_l.append(v_s[m] * tb)
                        del k_s, v_s, m
                    recv_b.append(sum(int(x.numel()) for x in addr_l) - r0)
                else:
                    kb, cb, vb = batches[b][:3] if batches else (keys, cols, vals)
                    addr_l.append((kb - part.start) * cols_n + cb.to(torch.int64) if mat else kb - part.start)
                    val_l.append(vb * tb)
            addr, v_all = torch.cat(addr_l), torch.cat(val_l)
            mag_all = torch.cat([v.abs() for v in val_l])
            del addr_l, val_l
            if exch:
                recv = int(np.mean(recv_b))
                got = torch.cat([sh.get(torch.arange(p.start, p.end, dtype=torch.int64, device=dev))
                                 for sh, p in zip(shards, my_parts)])
            elif mat:
                got = shard.getRows(torch.arange(part.start, part.end, dtype=torch.int64, device=dev)).reshape(-1)
            else:
                got = shard.get(torch.arange(part.start, part.end, dtype=torch.int64, device=dev))
            # segment sums over the sorted addresses (an atomic index_add_ serialises on Zipf's hot key)
            a, order = torch.sort(addr)
            uq, counts = torch.unique_consecutive(a, return_counts=True)
            sums = segment_sums(v_all[order], counts)
            # 1e-9 of each element's sum of magnitudes: the scale any summation order of a Double sum
            # is accurate to (~n eps sum |v|), far inside the north star's 1e-6 relative, while a lost
            # or duplicated record cannot pass
            mags = segment_sums(mag_all[order], counts)
            close = (got[uq] - sums).abs() <= 1e-9 * mags
            ok = bool(close.all())
            if not ok:
                bad = (~close).nonzero().reshape(-1)[:5]
                print(f"check: {int((~close).sum())} of {uq.numel()} elements differ, e.g. addr "
                      f"{uq[bad].tolist()} got {got[uq[bad]].tolist()} want {sums[bad].tolist()}", file=sys.stderr)
            got[uq] = 0
            if bool(got.any()):  # nothing outside the pushed addresses
                ok = False
                print(f"check: {int((got != 0).sum())} elements outside the pushed addresses are nonzero",
                      file=sys.stderr)
            if exch and len(times) == 1:
                uniq, u_note = int(uq.numel()), ""
                bytes_per_step = 16.0 * recv + 16.0 * uniq
            del a, order, uq, counts, sums, mags, addr, v_all, mag_all, got
    if check and world > 1:  # every rank's verdict: the line's check holds for all of them
        t = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        ok = bool(t.item() == 1.0)
    if check and not ok:
        raise SystemExit(f"post-run shard check FAILED ({pat}, 2^{log2_keys}, rank {rank})")

    total_bytes = bytes_per_step
    if world > 1:  # every rank's algorithmic bytes (exchange: its own recv and U)
        t = torch.tensor([bytes_per_step], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        total_bytes = float(t.item())
    value = total_bytes * steps / dt / 1e9
    if push:
        # The push is push_check (reads the keys) + push_apply (values and shard for the ordered
        # prefix) + the unordered tail (push_scatter, or the binned pipeline for large tails).
        # Together they move the algorithmic bytes once, so the roofline is taken over their summed
        # device time (each kernel's share below).
        apply_ms, apply_n = kernel_avg(N.GLINT_K_PUSH_APPLY)
        check_ms, _ = kernel_avg(N.GLINT_K_PUSH_CHECK)
        scat_ms, _ = kernel_avg(N.GLINT_K_PUSH_SCATTER)
        bin_ms, _ = kernel_avg(N.GLINT_K_PUSH_BINNED)
        kern = "push_check+push_apply+push_scatter+push_binned"
        kern_ms = check_ms + apply_ms + scat_ms + bin_ms
        launches = apply_n
        shares = {"push_check": round(check_ms, 4), "push_apply": round(apply_ms, 4),
                  "push_scatter": round(scat_ms, 4), "push_binned": round(bin_ms, 4)}
        metric = "device-resident push scatter-add GB/s (and % HBM peak) at 1/2/4/8 GPUs"
    else:
        kid = N.GLINT_K_MAT_PULL_ROWS if pat == "rowpull" else N.GLINT_K_VEC_PULL
        kern = "mat_pull_rows" if pat == "rowpull" else "vec_pull"
        kern_ms, launches = kernel_avg(kid)
        shares = {kern: round(kern_ms, 4)}
        metric = "device-resident pull gather GB/s (and % HBM peak)"
    overlap = len(shards) > 1 and kern_ms > dt / steps * 1e3
    if overlap:  # the local shards' pushes run on concurrent streams: their summed device time exceeds the
        kern_ms = dt / steps * 1e3  # step, so the roofline is taken over the step's wall time instead
    achieved = bytes_per_step / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0
    traffic, traffic_src, traffic_recs = pmc_traffic(tag)
    if traffic is not None and traffic_recs and push:
        # the summary is per profiled shard push: scaled to the records this step's pushes take (the
        # 8-partition exchange line's step is eight shard pushes of ~2^23 records each)
        step_recs = recv if exch else nrec
        if abs(step_recs / traffic_recs - 1.0) > 0.01:
            traffic = traffic * step_recs / traffic_recs
            traffic_src += f" (x {step_recs / traffic_recs:.3f}: {step_recs} records per step / {traffic_recs} per push)"
    line = {
        "metric": metric,
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(dt / steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (keys per BASELINE.md config, values U[-1,1) seed 42+rank), resident in HBM",
        "config": {"workload": workload + u_note, "keys_per_gpu": n * (cols_n if mat else 1) * len(shards),
                   "records_per_step_per_gpu": nrec, "records_received_per_step_per_gpu": recv,
                   "distinct_keys_per_step_per_gpu": uniq, "key_dtype": "i64", "value_dtype": "f64",
                   "parallelism": f"range-sharded x{world}, " + (
                       "route + all-to-all exchange" if exch and world > 1 else
                       "no exchange (world 1: " + how.split(",")[0] + ")" if exch else "no exchange")},
        "pct_hbm_peak_per_gpu": round(100.0 * value / world / HBM_PEAK_GBS, 2),
        "roofline": {"bound": "hbm", "kernel": kern, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_src, "kernel_ms": round(kern_ms, 4),
                     "algorithmic_bytes_per_launch": bytes_per_step,
                     "launches_timed": launches, "kernels_ms": shares,
                     "kernel_time": "wall time of the step (concurrent shard streams)" if overlap
                     else "summed device time of the step's kernels"},
        "check": ok,
    }
    if batches and len(batches) > 1:
        line["batches"] = {"k": len(batches), "rotation": "step s pushes batch s % K",
                           "distinct_keys_per_batch": [bt[3] for bt in batches] if not exch else None,
                           "check": "every batch replayed (value x times pushed) into one fp64 segment sum"}
    floor = sparse_floor(tag + ("_slab" if slab is not None else ""), dt / steps * 1e3)
    if floor is not None:
        line["practical_floor"] = floor
    for sh in shards:
        sh.destroy()
    if slab is not None:  # after its views
        slab.destroy()
    return line


def rank_devices(dev, backend: str, local_pinned: bool) -> dict:
    """Every rank's GPU as the ranks see it (all-gathered to every rank): device index, PCI address and
    UUID. Over RCCL two ranks on one GPU are an error -- the line would not be N GPUs' throughput; the
    gloo rehearsal (GLINT_BENCH_DEVICE pins every rank to one GPU) is marked as such."""
    import torch
    import torch.distributed as dist
    p = torch.cuda.get_device_properties(dev)
    me = {"rank": dist.get_rank(), "device": torch.cuda.current_device(),
          "pci": f"{getattr(p, 'pci_domain_id', 0):04x}:{getattr(p, 'pci_bus_id', 0):02x}:"
                 f"{getattr(p, 'pci_device_id', 0):02x}",
          "uuid": str(getattr(p, "uuid", ""))}
    allr = [None] * dist.get_world_size()
    dist.all_gather_object(allr, me)
    distinct = len({(d["pci"], d["uuid"]) for d in allr})
    if backend == "nccl" and distinct != len(allr):
        raise SystemExit(f"{len(allr)} ranks on {distinct} distinct GPUs: {allr}")
    return {"ranks": allr, "distinct_gpus": distinct, "backend": backend,
            "rehearsal": bool(local_pinned or backend != "nccl")}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    import torch
    import torch.distributed as dist
    import glint_amd  # noqa: F401  (loads libglint_gpu.so; fails loudly without it)
    from glint_amd import _native as N

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # rehearsal hooks (not used by the driver): GLINT_BENCH_DEVICE pins every rank to one GPU and
    # GLINT_BENCH_BACKEND=gloo replaces RCCL, so the N > 1 path can run on a one-GPU box
    local = int(os.environ.get("GLINT_BENCH_DEVICE", local))
    backend = os.environ.get("GLINT_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    exch = args.pattern == "exchange"
    if world > 1 or exch:
        if world == 1:  # the exchange path needs a process group even alone (RCCL world 1)
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29561")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    ctx = {"lib": N.load(), "dev": dev, "world": world, "rank": rank, "backend": backend}
    if args.parts_per_gpu > 1 and not exch:
        raise SystemExit("--parts-per-gpu applies to --pattern exchange")
    headline = args.log2_keys is None and args.pattern == "dense" and args.scaling == "weak"
    log2_keys = args.log2_keys if args.log2_keys is not None else (30 if headline else 28)
    if args.batches > 1 and args.pattern not in ("dense", "zipf", "matrix", "exchange"):
        raise SystemExit("--batches applies to the push patterns")
    line = run_line(ctx, args.pattern, log2_keys, args.scaling, args.steps, args.warmup, not args.no_check,
                    args.parts_per_gpu, max(1, args.batches))
    if world > 1:
        line["world_size"] = dist.get_world_size()
        line["devices"] = rank_devices(dev, backend, local_pinned="GLINT_BENCH_DEVICE" in os.environ)
    # BASELINE.json configs[1] (cfg2: 2^28 keys) beside the north-star line, with its own roofline and check
    if world == 1 and headline and not args.no_north_star:
        torch.cuda.empty_cache()
        c2 = run_line(ctx, "dense", 28, "weak", args.steps, args.warmup, not args.no_check)
        line["cfg2_2p28"] = {k: c2[k] for k in ("value", "unit", "ms_per_step", "steps", "warmup",
                                                "pct_hbm_peak_per_gpu", "roofline", "check")}
        line["cfg2_2p28"]["workload"] = c2["config"]["workload"]
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(log2_keys, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1 or exch:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
