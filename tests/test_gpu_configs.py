"""BASELINE.json configs[3] and configs[4] at their own shapes on one GPU.

configs[3]: RangePartitioner(8, 2^31) = eight 2^28-key shards
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


@pytest.mark.parametrize("dtype", ["long", "double"])
def test_cfg4_key_space_64_clients(gpu, dtype):
    """Long: bit-exact against index_add_; Double (the config's own type): within 1e-6 of fp64 segment
    sums relative to each element's sum of magnitudes (dist_workers._check_close)."""
    import torch.multiprocessing as mp
    import dist_workers
    mp.spawn(dist_workers.run_cfg4, args=(1, _port(), "nccl", 64, 25, dtype), nprocs=1, join=True)


@pytest.mark.parametrize("dtype", ["long", "double"])
def test_cfg5_full_shape(gpu, dtype):
    """BASELINE.json configs[4] at its own shape: a 2^20 x 512 matrix over 8 range partitions behind
    DistributedClient at world 1 (modelsPerServer = 8), 2^26 Zipf(1.0)-row triplets in 8 client
    batches of 2^23, then a 2^16-row Zipf pull and an element pull (dist_workers.run_cfg5)."""
    import torch.multiprocessing as mp
    import dist_workers
    mp.spawn(dist_workers.run_cfg5, args=(1, _port(), "nccl", dtype), nprocs=1, join=True)
