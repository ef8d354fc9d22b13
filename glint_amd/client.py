"""In-process client over HBM shards: the exchange step in front of the shard kernels.

Mirrors the reference's client factory and asynchronous models, minus the Akka transport:

* ``Client.vector`` / ``Client.matrix`` -- glint.Client.vector/matrix/create
  (src/main/scala/glint/Client.scala:53-94, 105-196): P = min(keys, modelsPerServer x servers)
  partitions, partition i placed on "server" (here: GPU) i % servers.
* ``BigVector.push/pull`` -- AsyncBigVector.push/pull (AsyncBigVector.scala:49-121): records are
  bucketed by partition preserving their order inside each bucket (``mapPartitions``, :96-98),
  one shard call per partition, and pulled values scattered back to the caller's order (:61-79).
* ``BigMatrix.push/pull`` -- AsyncBigMatrix (AsyncBigMatrix.scala:53-170), including the row pull.

Out-of-range keys raise ``IndexOutOfBoundsException`` before any shard is touched, as the
reference's ``partitioner.partition`` does synchronously inside ``mapPartitions``.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import numpy as np

from .errors import ModelCreationException
from .partitioning import CyclicPartitioner, RangePartitioner
from .shard import PartialMatrix, PartialVector, resolve_dtype


def bucket(owner: np.ndarray, nparts: int):
    """Stable grouping of record indices by owning partition (AsyncBigVector.scala:96-98).
    Returns (order, offsets): records of partition p are order[offsets[p]:offsets[p+1]], in the
    caller's order."""
    order = np.argsort(owner, kind="stable")
    counts = np.bincount(owner, minlength=nparts)
    offsets = np.zeros(nparts + 1, dtype=np.int64)
    np.cumsum(counts, out=offsets[1:])
    return order, offsets


class BigVector:
    """AsyncBigVector over PartialVector shards (one per partition)."""

    def __init__(self, partitioner, shards: Sequence[PartialVector], size: int):
        self.partitioner = partitioner
        self.shards = list(shards)
        self.size = int(size)

    @property
    def nrOfPartitions(self) -> int:  # AsyncBigVector.scala:126-128
        return len(self.partitioner.all())

    def push(self, keys, values, deterministic: bool = False) -> bool:
        keys = np.ascontiguousarray(keys, dtype=np.int64)
        values = np.ascontiguousarray(values, dtype=self.shards[0].np_dtype)
        owner = self.partitioner.partition_indices(keys)
        order, off = bucket(owner, len(self.shards))
        for p, sh in enumerate(self.shards):
            idx = order[off[p]:off[p + 1]]
            if idx.size:
                sh.update(keys[idx], values[idx], deterministic=deterministic)
        return True

    def pull(self, keys) -> np.ndarray:
        keys = np.ascontiguousarray(keys, dtype=np.int64)
        owner = self.partitioner.partition_indices(keys)
        order, off = bucket(owner, len(self.shards))
        out = np.zeros(keys.shape, dtype=self.shards[0].np_dtype)
        for p, sh in enumerate(self.shards):
            idx = order[off[p]:off[p + 1]]
            if idx.size:
                out[idx] = sh.get(keys[idx])
        return out

    def destroy(self) -> bool:
        for sh in self.shards:
            sh.destroy()
        return True


class BigMatrix:
    """AsyncBigMatrix over PartialMatrix shards."""

    def __init__(self, partitioner, shards: Sequence[PartialMatrix], rows: int, cols: int):
        self.partitioner = partitioner
        self.shards = list(shards)
        self.rows = int(rows)
        self.cols = int(cols)

    @property
    def nrOfPartitions(self) -> int:
        return len(self.partitioner.all())

    def push(self, rows, cols, values, deterministic: bool = False) -> bool:
        rows = np.ascontiguousarray(rows, dtype=np.int64)
        cols = np.ascontiguousarray(cols, dtype=np.int32)
        values = np.ascontiguousarray(values, dtype=self.shards[0].np_dtype)
        owner = self.partitioner.partition_indices(rows)
        order, off = bucket(owner, len(self.shards))
        for p, sh in enumerate(self.shards):
            idx = order[off[p]:off[p + 1]]
            if idx.size:
                sh.update(rows[idx], cols[idx], values[idx], deterministic=deterministic)
        return True

    def pull(self, rows, cols=None) -> np.ndarray:
        """pull(rows, cols): elements (AsyncBigMatrix.scala:96-130); pull(rows): whole rows as an
        (n, cols) array (AsyncBigMatrix.scala:53-86)."""
        rows = np.ascontiguousarray(rows, dtype=np.int64)
        owner = self.partitioner.partition_indices(rows)
        order, off = bucket(owner, len(self.shards))
        if cols is None:
            out = np.zeros((rows.size, self.cols), dtype=self.shards[0].np_dtype)
            for p, sh in enumerate(self.shards):
                idx = order[off[p]:off[p + 1]]
                if idx.size:
                    out[idx] = sh.getRows(rows[idx])
            return out
        cols = np.ascontiguousarray(cols, dtype=np.int32)
        out = np.zeros(rows.shape, dtype=self.shards[0].np_dtype)
        for p, sh in enumerate(self.shards):
            idx = order[off[p]:off[p + 1]]
            if idx.size:
                out[idx] = sh.get(rows[idx], cols[idx])
        return out

    def destroy(self) -> bool:
        for sh in self.shards:
            sh.destroy()
        return True


class Client:
    """glint.Client's model factory with MI355X GPUs in the role of parameter servers."""

    def __init__(self, devices: Optional[Sequence[int]] = None):
        if devices is None:
            from . import _native as N
            devices = list(range(N.load().glint_device_count()))
        self.devices = list(devices)

    def _create(self, keys: int, modelsPerServer: int, createPartitioner: Callable, make_shard: Callable):
        # Client.create (Client.scala:53-94)
        if not self.devices:
            raise ModelCreationException("Cannot create a model without active parameter servers")
        nparts = int(min(keys, modelsPerServer * len(self.devices)))
        partitioner = createPartitioner(nparts, keys)
        shards = [make_shard(part, self.devices[i % len(self.devices)])
                  for i, part in enumerate(partitioner.all())]
        return partitioner, shards

    def vector(self, keys: int, dtype="double", modelsPerServer: int = 1,
               createPartitioner: Callable = RangePartitioner.apply) -> BigVector:
        resolve_dtype(dtype)  # ModelCreationException analogue for unsupported types: ValueError
        partitioner, shards = self._create(keys, modelsPerServer, createPartitioner,
                                           lambda part, dev: PartialVector(part, dtype, dev))
        return BigVector(partitioner, shards, keys)

    def matrix(self, rows: int, cols: int, dtype="double", modelsPerServer: int = 1,
               createPartitioner: Callable = RangePartitioner.apply) -> BigMatrix:
        resolve_dtype(dtype)
        partitioner, shards = self._create(rows, modelsPerServer, createPartitioner,
                                           lambda part, dev: PartialMatrix(part, cols, dtype, dev))
        return BigMatrix(partitioner, shards, rows, cols)


__all__ = ["Client", "BigVector", "BigMatrix", "bucket", "RangePartitioner", "CyclicPartitioner"]
