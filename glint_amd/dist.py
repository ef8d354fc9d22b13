"""Models spread over a process group: one process per GPU, records exchanged with all-to-all.

The reference's client fans a push/pull out as one Akka message per partition
(AsyncBigVector.push/pull, src/main/scala/glint/models/client/async/AsyncBigVector.scala:49-121;
AsyncBigMatrix.scala:53-170) to the server that hosts it -- partition i lives on server
i % servers (Client.create, Client.scala:75-84). Here every rank of a ``torch.distributed`` group
is both a client and a server driving one GPU:

1. route   -- the batch's record indices are grouped by owning partition, stable
              (``glint_route_dev`` on the GPU; the same grouping on host for CPU tensors), and the
              partition groups are ordered by hosting rank;
2. exchange -- per-rank record counts, then keys (+ cols) and values, with ``all_to_all_single``
              (RCCL over xGMI for the ``nccl`` backend, gloo on CPU);
3. apply   -- each local shard gets its records ordered by source rank, each source's records in
              that caller's order, and runs the push / pull kernels;
4. answer  -- (pull) values travel back along the reversed splits and are scattered to the
              caller's order (AsyncBigVector.scala:61-79).

Out-of-range keys raise ``IndexOutOfBoundsException`` on the calling rank before anything is sent
-- the reference throws inside ``mapPartitions`` before any message leaves -- so a caller that
catches it must not enter the collective (every rank of the group takes part in every exchange).

The bench's weak-scaling line does not come through here: there every rank pushes the records of
the partition it hosts, which needs no exchange.
"""
from __future__ import annotations

import ctypes as C
from typing import Callable, List, Optional

import numpy as np
import torch
import torch.distributed as dist

from . import _native as N
from .client import bucket
from .errors import IndexOutOfBoundsException, ModelCreationException
from .partitioning import CyclicPartitioner, RangePartitioner
from .shard import PartialMatrix, PartialVector, check, resolve_dtype

_TORCH_DTYPES = {np.dtype(np.int32): torch.int32, np.dtype(np.int64): torch.int64,
                 np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64}


class Router:
    """Stable grouping of a batch by partition, partitions ordered by hosting rank."""

    def __init__(self, partitioner, world: int):
        self.partitioner = partitioner
        self.nparts = len(partitioner.all())
        self.world = int(world)
        if isinstance(partitioner, RangePartitioner):
            self.kind, self.nkeys = N.GLINT_ROUTE_RANGE, partitioner.size
        elif isinstance(partitioner, CyclicPartitioner):
            self.kind, self.nkeys = N.GLINT_ROUTE_CYCLIC, partitioner.keys
        else:
            raise TypeError(f"unsupported partitioner {type(partitioner).__name__}")
        # rank r hosts partitions r, r + W, r + 2W, ... (Client.scala:75-84)
        self.rank_parts: List[List[int]] = [list(range(r, self.nparts, self.world)) for r in range(self.world)]
        self.perm = [p for r in range(self.world) for p in self.rank_parts[r]]
        self.maxp = max(len(p) for p in self.rank_parts)
        self.identity = self.perm == list(range(self.nparts))

    def group(self, keys: torch.Tensor):
        """-> (order, counts): order = record indices grouped by partition in ``perm`` order (each
        group in the caller's order), counts = host int64 array of the group sizes (perm order)."""
        n = keys.numel()
        if keys.is_cuda:
            lib = N.load()
            counts_d = torch.empty(self.nparts, dtype=torch.int64, device=keys.device)
            order = torch.empty(n, dtype=torch.int64, device=keys.device)
            bad = C.c_int64(-1)
            stream = torch.cuda.current_stream(keys.device).cuda_stream
            rc = lib.glint_route_dev(keys.data_ptr(), n, self.kind, self.nparts, self.nkeys, counts_d.data_ptr(),
                                     order.data_ptr(), C.byref(bad), stream)
            if rc == N.GLINT_EOUTOFRANGE:
                i = bad.value
                raise IndexOutOfBoundsException(f"key {int(keys[i])} (record {i}) outside [0, {self.nkeys})")
            check(rc)
            counts = counts_d.cpu().numpy()
        else:
            owner = self.partitioner.partition_indices(keys.numpy())  # raises IndexOutOfBoundsException
            o, off = bucket(owner, self.nparts)
            order, counts = torch.from_numpy(o), np.diff(off)
        if not self.identity:
            off = np.zeros(self.nparts + 1, dtype=np.int64)
            np.cumsum(counts, out=off[1:])
            order = torch.cat([order[off[p]:off[p + 1]] for p in self.perm])
            counts = counts[self.perm]
        return order, counts


class _Exchange:
    """The all-to-all legs of one routed call (send splits, receive splits, local layout)."""

    def __init__(self, router: Router, rank: int, counts: np.ndarray, group, device):
        W, maxp = router.world, router.maxp
        self.group, self.device = group, device
        send = np.zeros((W, maxp), dtype=np.int64)
        i = 0
        for r in range(W):
            k = len(router.rank_parts[r])
            send[r, :k] = counts[i:i + k]
            i += k
        recv = torch.empty((W, maxp), dtype=torch.int64, device=device)
        dist.all_to_all_single(recv, torch.from_numpy(send).to(device), group=group)
        self.recv_counts = recv.cpu().numpy()  # [source rank, local partition j]
        self.in_splits = send.sum(axis=1).tolist()
        self.out_splits = self.recv_counts.sum(axis=1).tolist()
        self.nlocal = len(router.rank_parts[rank])

    def forward(self, t: torch.Tensor) -> torch.Tensor:
        out = torch.empty((sum(self.out_splits),) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_to_all_single(out, t.contiguous(), self.out_splits, self.in_splits, group=self.group)
        return out

    def backward(self, t: torch.Tensor) -> torch.Tensor:
        out = torch.empty((sum(self.in_splits),) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_to_all_single(out, t.contiguous(), self.in_splits, self.out_splits, group=self.group)
        return out

    def local_index(self, j: int) -> Optional[torch.Tensor]:
        """Positions in the received buffer of local partition j's records (source-rank order);
        None when the local shard owns the whole buffer."""
        if self.nlocal == 1:
            return None
        seg = np.concatenate([[0], np.cumsum(self.recv_counts.sum(axis=1))])
        parts = []
        for s in range(self.recv_counts.shape[0]):
            a = seg[s] + self.recv_counts[s, :j].sum()
            parts.append(np.arange(a, a + self.recv_counts[s, j], dtype=np.int64))
        return torch.from_numpy(np.concatenate(parts)).to(self.device)


class _Distributed:
    def __init__(self, partitioner, shards, group, device):
        self.partitioner = partitioner
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.router = Router(partitioner, self.world)
        self.shards = list(shards)  # local shards, in rank_parts[rank] order
        self.device = device

    @property
    def nrOfPartitions(self) -> int:
        return self.router.nparts

    def _comm_device(self, t: torch.Tensor) -> torch.Tensor:
        # gloo exchanges host tensors; nccl (RCCL) device tensors
        if dist.get_backend(self.group) == "gloo":
            return t.cpu()
        return t

    def _begin(self, keys: torch.Tensor):
        order, counts = self.router.group(keys)
        comm = torch.device("cpu") if dist.get_backend(self.group) == "gloo" else keys.device
        return order, _Exchange(self.router, self.rank, counts, self.group, comm)

    def _to_shard(self, t: torch.Tensor) -> torch.Tensor:
        return t.to(self.device) if t.device != self.device else t

    def _split(self, ex: _Exchange, *bufs):
        for j, sh in enumerate(self.shards):
            idx = ex.local_index(j)
            yield j, sh, [b if idx is None else b.index_select(0, idx.to(b.device)) for b in bufs]

    def destroy(self) -> bool:
        for sh in self.shards:
            sh.destroy()
        return True


class DistributedBigVector(_Distributed):
    """AsyncBigVector over the ranks of a process group (push / pull of any keys from any rank)."""

    def __init__(self, partitioner, shards, size: int, np_dtype, group=None, device=None):
        super().__init__(partitioner, shards, group, device)
        self.size = int(size)
        self.dtype = _TORCH_DTYPES[np.dtype(np_dtype)]

    def push(self, keys: torch.Tensor, values: torch.Tensor, deterministic: bool = False) -> bool:
        keys = keys.reshape(-1).to(torch.int64)
        values = values.reshape(-1).to(self.dtype)
        if keys.numel() != values.numel():
            raise ValueError("keys and values differ in length")
        order, ex = self._begin(keys)
        rk = ex.forward(self._comm_device(keys.index_select(0, order)))
        rv = ex.forward(self._comm_device(values.index_select(0, order.to(values.device))))
        for _, sh, (k, v) in self._split(ex, rk, rv):
            if k.numel():
                sh.update(self._to_shard(k), self._to_shard(v), deterministic=deterministic)
        return True

    def pull(self, keys: torch.Tensor) -> torch.Tensor:
        keys = keys.reshape(-1).to(torch.int64)
        order, ex = self._begin(keys)
        rk = ex.forward(self._comm_device(keys.index_select(0, order)))
        resp = torch.empty(rk.numel(), dtype=self.dtype, device=rk.device)
        for j, sh, (k,) in self._split(ex, rk):
            if k.numel():
                got = sh.get(self._to_shard(k)).to(resp.device)
                idx = ex.local_index(j)
                if idx is None:
                    resp = got
                else:
                    resp.index_copy_(0, idx.to(resp.device), got)
        back = ex.backward(resp).to(keys.device)
        out = torch.empty(keys.numel(), dtype=self.dtype, device=keys.device)
        out.index_copy_(0, order.to(keys.device), back)
        return out


class DistributedBigMatrix(_Distributed):
    """AsyncBigMatrix over the ranks of a process group."""

    def __init__(self, partitioner, shards, rows: int, cols: int, np_dtype, group=None, device=None):
        super().__init__(partitioner, shards, group, device)
        self.rows, self.cols = int(rows), int(cols)
        self.dtype = _TORCH_DTYPES[np.dtype(np_dtype)]

    def push(self, rows: torch.Tensor, cols: torch.Tensor, values: torch.Tensor,
             deterministic: bool = False) -> bool:
        rows = rows.reshape(-1).to(torch.int64)
        cols = cols.reshape(-1).to(torch.int32)
        values = values.reshape(-1).to(self.dtype)
        if not rows.numel() == cols.numel() == values.numel():
            raise ValueError("rows, cols and values differ in length")
        order, ex = self._begin(rows)
        rr = ex.forward(self._comm_device(rows.index_select(0, order)))
        rc = ex.forward(self._comm_device(cols.index_select(0, order.to(cols.device))))
        rv = ex.forward(self._comm_device(values.index_select(0, order.to(values.device))))
        for _, sh, (r, c, v) in self._split(ex, rr, rc, rv):
            if r.numel():
                sh.update(self._to_shard(r), self._to_shard(c), self._to_shard(v), deterministic=deterministic)
        return True

    def pull(self, rows: torch.Tensor, cols: Optional[torch.Tensor] = None) -> torch.Tensor:
        """pull(rows, cols): elements (AsyncBigMatrix.scala:96-130); pull(rows): whole rows as an
        (n, cols) tensor (AsyncBigMatrix.scala:53-86)."""
        rows = rows.reshape(-1).to(torch.int64)
        order, ex = self._begin(rows)
        rr = ex.forward(self._comm_device(rows.index_select(0, order)))
        if cols is None:
            shape = (rr.numel(), self.cols)
            bufs = (rr,)
        else:
            cols = cols.reshape(-1).to(torch.int32)
            rc = ex.forward(self._comm_device(cols.index_select(0, order.to(cols.device))))
            shape = (rr.numel(),)
            bufs = (rr, rc)
        resp = torch.empty(shape, dtype=self.dtype, device=rr.device)
        for j, sh, parts in self._split(ex, *bufs):
            if parts[0].numel():
                got = (sh.getRows(self._to_shard(parts[0])) if cols is None
                       else sh.get(self._to_shard(parts[0]), self._to_shard(parts[1])))
                got = got.to(resp.device).reshape((-1,) + shape[1:])
                idx = ex.local_index(j)
                if idx is None:
                    resp = got
                else:
                    resp.index_copy_(0, idx.to(resp.device), got)
        back = ex.backward(resp).to(rows.device)
        out = torch.empty((rows.numel(),) + shape[1:], dtype=self.dtype, device=rows.device)
        out.index_copy_(0, order.to(rows.device), back)
        return out


class DistributedClient:
    """glint.Client's model factory over a process group: rank r hosts partitions r, r + W, ...

    ``shard_factory(kind, partition, cols, dtype, device)`` builds a local shard; the default makes
    ``PartialVector`` / ``PartialMatrix`` HBM shards on ``device`` (this rank's GPU)."""

    def __init__(self, group=None, device=None, shard_factory: Optional[Callable] = None):
        if not dist.is_initialized():
            raise ModelCreationException("torch.distributed is not initialised")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        self.shard_factory = shard_factory or self._hbm_shard

    @staticmethod
    def _hbm_shard(kind, partition, cols, dtype, device):
        if device.type != "cuda":
            raise ModelCreationException("HBM shards need a GPU device")
        if kind == "vector":
            return PartialVector(partition, dtype, device.index)
        return PartialMatrix(partition, cols, dtype, device.index)

    def _create(self, keys: int, modelsPerServer: int, createPartitioner: Callable, kind, cols, dtype):
        nparts = int(min(keys, modelsPerServer * self.world))  # Client.scala:63
        partitioner = createPartitioner(nparts, keys)
        mine = Router(partitioner, self.world).rank_parts[self.rank]
        parts = partitioner.all()
        shards = [self.shard_factory(kind, parts[p], cols, dtype, self.device) for p in mine]
        return partitioner, shards

    def vector(self, keys: int, dtype="double", modelsPerServer: int = 1,
               createPartitioner: Callable = RangePartitioner.apply) -> DistributedBigVector:
        _, np_dtype = resolve_dtype(dtype)
        partitioner, shards = self._create(keys, modelsPerServer, createPartitioner, "vector", 0, dtype)
        return DistributedBigVector(partitioner, shards, keys, np_dtype, self.group, self.device)

    def matrix(self, rows: int, cols: int, dtype="double", modelsPerServer: int = 1,
               createPartitioner: Callable = RangePartitioner.apply) -> DistributedBigMatrix:
        _, np_dtype = resolve_dtype(dtype)
        partitioner, shards = self._create(rows, modelsPerServer, createPartitioner, "matrix", cols, dtype)
        return DistributedBigMatrix(partitioner, shards, rows, cols, np_dtype, self.group, self.device)


__all__ = ["Router", "DistributedClient", "DistributedBigVector", "DistributedBigMatrix"]
