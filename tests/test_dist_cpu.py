"""Multi-process tests of the exchange layer (glint_amd.dist) on CPU: world_size 1, 2 and 3 over gloo,
with oracle-backed shards standing in for the HBM shards (tests/dist_workers.py). Covers range and
cyclic placement, several partitions per rank (Client.scala:63, 75-84), fewer keys than partitions,
matrices, out-of-range keys and empty batches."""
import socket

import pytest
import torch.multiprocessing as mp

import dist_workers


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [1, 2, 3])
@pytest.mark.parametrize("case", sorted(dist_workers.CASES))
def test_exchange_matches_sequential_oracle(case, world):
    mp.spawn(dist_workers.run_case, args=(world, free_port(), "gloo", case, False), nprocs=world, join=True)
