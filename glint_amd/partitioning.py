"""Key-space partitioning: the layout that decides which shard (and GPU) owns a key.

Mirrors glint.partitioning (src/main/scala/glint/partitioning/) -- same class and method names,
argument meaning and failure behaviour (``IndexOutOfBoundsException`` for keys outside the key
space) -- plus vectorised forms used to route whole record batches at once.
"""
from __future__ import annotations

import numpy as np

from .errors import IndexOutOfBoundsException


def _to_int(x: int) -> int:
    """Scala's Long.toInt: keep the low 32 bits, two's complement."""
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= (1 << 31) else x


def _jdiv(a: int, b: int) -> int:
    """Java/Scala Long division: truncates toward zero."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


class Partition:
    """glint.partitioning.Partition (Partition.scala:8-35)."""

    def __init__(self, index: int):
        self.index = int(index)

    def contains(self, key: int) -> bool:  # pragma: no cover - abstract
        raise NotImplementedError

    def globalToLocal(self, key: int) -> int:  # pragma: no cover - abstract
        raise NotImplementedError

    @property
    def size(self) -> int:  # pragma: no cover - abstract
        raise NotImplementedError


class RangePartition(Partition):
    """glint.partitioning.range.RangePartition (RangePartition.scala:8-35)."""

    kind = 0

    def __init__(self, index: int, start: int, end: int):
        super().__init__(index)
        self.start = int(start)
        self.end = int(end)

    def contains(self, key: int) -> bool:  # :17
        return self.start <= key < self.end

    @property
    def size(self) -> int:  # :24  (end - start).toInt
        return _to_int(self.end - self.start)

    def globalToLocal(self, key: int) -> int:  # :33  (key - start).toInt
        return _to_int(int(key) - self.start)

    def __repr__(self) -> str:
        return f"RangePartition({self.index}, {self.start}, {self.end})"


class RangePartitioner:
    """glint.partitioning.range.RangePartitioner (RangePartitioner.scala:8-84)."""

    def __init__(self, partitions, numberOfSmallPartitions: int, smallPartitionSize: int, size: int):
        self.partitions = list(partitions)
        self.numberOfSmallPartitions = int(numberOfSmallPartitions)
        self.smallPartitionSize = int(smallPartitionSize)
        self.size = int(size)
        self.numberOfSmallKeys = self.numberOfSmallPartitions * self.smallPartitionSize  # :17
        self.largePartitionSize = _to_int(self.smallPartitionSize + 1)  # :18 (an Int: wraps)

    @classmethod
    def apply(cls, numberOfPartitions: int, numberOfKeys: int) -> "RangePartitioner":
        """RangePartitioner.apply (RangePartitioner.scala:62-84)."""
        P, N = int(numberOfPartitions), int(numberOfKeys)
        if P <= 0:
            raise ValueError("numberOfPartitions must be positive")
        n_large = _to_int(N % P)
        n_small = P - n_large
        q = _to_int((N - N % P) // P)
        parts = []
        start, end = 0, q
        for i in range(P):
            if i < n_small:
                parts.append(RangePartition(i, start, end))
                start += q
                end += q
            else:
                end += 1
                parts.append(RangePartition(i, start, end))
                start += _to_int(q + 1)  # :78 Int + 1 wraps before widening
                end += q
        return cls(parts, n_small, q, N)

    def partition(self, key: int) -> RangePartition:
        """RangePartitioner.partition (RangePartitioner.scala:27-43)."""
        key = int(key)
        if key < 0 or key >= self.size:
            raise IndexOutOfBoundsException(f"key {key} outside [0, {self.size})")
        if key < self.numberOfSmallKeys:
            idx = _jdiv(key, self.smallPartitionSize)
        else:
            idx = self.numberOfSmallPartitions + _jdiv(key - self.numberOfSmallKeys, self.largePartitionSize)
        idx = _to_int(idx)
        if not 0 <= idx < len(self.partitions):  # partitions(idx): ArrayIndexOutOfBoundsException
            raise IndexOutOfBoundsException(f"key {key} maps to partition index {idx} of {len(self.partitions)}")
        return self.partitions[idx]

    def partition_indices(self, keys: np.ndarray) -> np.ndarray:
        """Vectorised `partition(k).index` over an int64 array; raises like `partition` for the first
        key outside the key space (AsyncBigVector.mapPartitions evaluates keys in order)."""
        keys = np.asarray(keys, dtype=np.int64)
        bad = (keys < 0) | (keys >= self.size)
        if bad.any():
            i = int(np.argmax(bad))
            raise IndexOutOfBoundsException(f"key {int(keys[i])} (record {i}) outside [0, {self.size})")
        out = np.empty(keys.shape, dtype=np.int64)
        small = keys < self.numberOfSmallKeys
        if self.smallPartitionSize > 0:
            out[small] = keys[small] // self.smallPartitionSize  # both operands >= 0: floor == trunc
        rest = keys[~small] - self.numberOfSmallKeys
        L = self.largePartitionSize
        out[~small] = self.numberOfSmallPartitions + (rest // L if L > 0 else -(rest // -L))  # Java truncation
        out = ((out & 0xFFFFFFFF) ^ 0x80000000) - 0x80000000  # .toInt
        oob = (out < 0) | (out >= len(self.partitions))
        if oob.any():
            i = int(np.argmax(oob))
            raise IndexOutOfBoundsException(f"key {int(keys[i])} (record {i}) maps to partition index {int(out[i])}")
        return out

    def all(self):
        return self.partitions


class CyclicPartition(Partition):
    """glint.partitioning.cyclic.CyclicPartition (CyclicPartition.scala:12-49)."""

    kind = 1

    def __init__(self, index: int, numberOfPartitions: int, numberOfKeys: int):
        super().__init__(index)
        self.numberOfPartitions = int(numberOfPartitions)
        self.numberOfKeys = int(numberOfKeys)

    @staticmethod
    def _jmod(a: int, b: int) -> int:
        """Java/Scala `%` (sign of the dividend)."""
        r = abs(a) % abs(b)
        return -r if a < 0 else r

    def contains(self, key: int) -> bool:  # :21-23
        return _to_int(self._jmod(int(key), self.numberOfPartitions)) == self.index

    @property
    def size(self) -> int:  # :30-36
        i = 1
        while not self.contains(self.numberOfKeys - i):
            i += 1
            if i > self.numberOfPartitions + 1:
                return 0
        return self.globalToLocal(self.numberOfKeys - i) + 1

    def globalToLocal(self, key: int) -> int:  # :45-47 (Long division truncates toward zero)
        d = int(key) - self.index
        q = abs(d) // self.numberOfPartitions
        return _to_int(-q if d < 0 else q)

    def __repr__(self) -> str:
        return f"CyclicPartition({self.index}, {self.numberOfPartitions}, {self.numberOfKeys})"


class CyclicPartitioner:
    """glint.partitioning.cyclic.CyclicPartitioner (CyclicPartitioner.scala:12-49)."""

    def __init__(self, partitions, keys: int):
        self.partitions = list(partitions)
        self.keys = int(keys)

    @classmethod
    def apply(cls, numberOfPartitions: int, numberOfKeys: int) -> "CyclicPartitioner":
        P = int(numberOfPartitions)
        return cls([CyclicPartition(i, P, numberOfKeys) for i in range(P)], numberOfKeys)

    def partition(self, key: int) -> CyclicPartition:  # :19-22
        key = int(key)
        if key >= self.keys:
            raise IndexOutOfBoundsException(f"key {key} >= {self.keys}")
        idx = _to_int(CyclicPartition._jmod(key, len(self.partitions)))
        if idx < 0:  # negative array index in the reference
            raise IndexOutOfBoundsException(f"key {key} is negative")
        return self.partitions[idx]

    def partition_indices(self, keys: np.ndarray) -> np.ndarray:
        keys = np.asarray(keys, dtype=np.int64)
        bad = (keys < 0) | (keys >= self.keys)
        if bad.any():
            i = int(np.argmax(bad))
            raise IndexOutOfBoundsException(f"key {int(keys[i])} (record {i}) outside [0, {self.keys})")
        return keys % len(self.partitions)

    def all(self):
        return self.partitions
