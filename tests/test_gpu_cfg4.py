"""BASELINE.json configs[3] at its own key space: RangePartitioner(8, 2^31) = eight 2^28-key shards
(16 GiB of Long) on the one GPU of the box, behind DistributedClient / DistributedBigVector at world 1
with modelsPerServer = 8, fed 64 client batches of 2^25 uniform keys (cfg4's 64 loopback clients x
2^25 records). Every batch goes through the device route (glint_route_gather_dev, 8 partitions) and
the exchange's per-partition split (AsyncBigVector.scala:96-121, Client.scala:71-85). Long sums are
exact in any order: each shard must equal a torch.index_add_ int64 reference bit for bit, and two
sampled key windows are replayed through the oracle's sequential update loop."""
import socket

import pytest

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_cfg4_key_space_64_clients(gpu):
    import torch.multiprocessing as mp
    import dist_workers
    mp.spawn(dist_workers.run_cfg4, args=(1, _port(), "nccl", 64, 25), nprocs=1, join=True)
