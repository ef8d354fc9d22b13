"""World-1 pulls through DistributedBigVector with the partitions in one slab: the route's key check plus
one gather (_pull_slab) against route + per-partition pulls + scatter back (GLINT_DIST_SLAB_PULL=0).

    python tools/ab_slab_pull.py [--log2-keys 25] [--parts 8] [--records 26] [--steps 20]

cfg4b's key space as 8 partitions of 2^25 keys on one GPU, 2^26 uniform keys pulled per step; prints
one JSON line per mode (ms per pull, and whether both modes returned the same values)."""
import argparse
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2-keys", type=int, default=25)
    ap.add_argument("--parts", type=int, default=8)
    ap.add_argument("--records", type=int, default=26)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    from glint_amd.dist import DistributedClient
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29577")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    dev = torch.device("cuda", 0)
    nkeys = a.parts << a.log2_keys
    vec = DistributedClient(device=dev).vector(nkeys, "double", modelsPerServer=a.parts)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    fill = torch.arange(nkeys, device=dev)
    vec.push(fill, torch.rand(nkeys, dtype=torch.float64, device=dev, generator=g))
    keys = torch.randint(0, nkeys, (1 << a.records,), device=dev, generator=g)
    outs = {}
    for mode in ("slab", "route"):
        os.environ["GLINT_DIST_SLAB_PULL"] = "1" if mode == "slab" else "0"
        for _ in range(3):
            out = vec.pull(keys)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            out = vec.pull(keys)
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) / a.steps * 1e3
        outs[mode] = out
        print(json.dumps({"mode": mode, "slab": vec.slab is not None, "keyed": bool(vec._slab_keyed),
                          "keys": nkeys, "records": 1 << a.records, "ms_per_pull": round(ms, 4),
                          "GBps_keys_and_values": round(16.0 * (1 << a.records) / ms / 1e6, 1)}), flush=True)
    print(json.dumps({"same_values": bool(torch.equal(outs["slab"], outs["route"]))}), flush=True)
    vec.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
