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

Out-of-range keys raise ``IndexOutOfBoundsException`` on the calling rank, and nothing of that
rank's batch is applied -- the reference throws inside ``mapPartitions`` before any message leaves.
For device batches the bad rank still joins the call's collectives (with nothing to send, so the
other ranks' pushes and pulls complete) and raises after them; host (CPU) batches raise before the
exchange, so there a caller that catches it must not enter the collective.

The bench's weak-scaling line does not come through here: there every rank pushes the records of
the partition it hosts, which needs no exchange.
"""
from __future__ import annotations

import ctypes as C
import math
import threading
from typing import Callable, List, Optional

import numpy as np
import torch
import torch.distributed as dist

from . import _native as N
from .client import bucket
from .errors import ArrayIndexOutOfBoundsException, IndexOutOfBoundsException, ModelCreationException
from .partitioning import CyclicPartitioner, RangePartition, RangePartitioner
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
        # group ("slot") of partition p in send order, and the slot's cell in the (rank, j) count matrix
        slot_of = np.empty(self.nparts, np.int32)
        slot_of[self.perm] = np.arange(self.nparts, dtype=np.int32)
        self.slot_of = slot_of
        self.slot_cell = np.array([r * self.maxp + j for r in range(self.world)
                                   for j in range(len(self.rank_parts[r]))], np.int64)
        self._dev = {}

    def _device_tables(self, device):
        t = self._dev.get(device)
        if t is None:
            slot_of = None if self.identity else torch.from_numpy(self.slot_of).to(device)
            t = (slot_of, torch.from_numpy(self.slot_cell).to(device))
            self._dev[device] = t
        return t

    def route(self, keys: torch.Tensor, cols=None, vals=None, want_order: bool = False, key_delta=None):
        """Device batch -> records in send order, in ONE kernel pass (glint_route_gather_dev) with no
        host synchronisation: (counts, order, keys, cols, vals, bad), all device tensors; counts in
        slot (send) order, bad = ~first bad record index or 0. key_delta (device int64 per slot, with
        nparts >= 2): keys written as key + key_delta[slot] (glint_route_gather_rebased_dev)."""
        n = keys.numel()
        dev = keys.device
        slot_of, _ = self._device_tables(dev)
        counts = torch.empty(self.nparts, dtype=torch.int64, device=dev)
        bad = torch.empty(1, dtype=torch.int64, device=dev)
        if self.nparts == 1:
            # one partition: the batch, in the caller's order, is the send buffer (order = identity,
            # None); the pass only validates the keys and counts them
            rc = N.load().glint_route_gather_dev(
                keys.data_ptr(), None, None, 0, n, self.kind, 1, self.nkeys, None, counts.data_ptr(), None,
                None, None, None, bad.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
            check(rc)
            return counts, None, keys, cols, vals, bad
        order = torch.empty(n, dtype=torch.int64, device=dev) if want_order else None
        sk = torch.empty(n, dtype=torch.int64, device=dev)
        sc = torch.empty(n, dtype=torch.int32, device=dev) if cols is not None else None
        sv = torch.empty(n, dtype=vals.dtype, device=dev) if vals is not None else None
        ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        vsize = vals.element_size() if vals is not None else 0
        st = torch.cuda.current_stream(dev).cuda_stream
        if key_delta is not None:
            rc = N.load().glint_route_gather_rebased_dev(
                keys.data_ptr(), ptr(cols), ptr(vals), vsize, n, self.kind, self.nparts, self.nkeys, ptr(slot_of),
                key_delta.data_ptr(), counts.data_ptr(), ptr(order), sk.data_ptr(), ptr(sc), ptr(sv), bad.data_ptr(), st)
        else:
            rc = N.load().glint_route_gather_dev(
                keys.data_ptr(), ptr(cols), ptr(vals), vsize, n, self.kind, self.nparts, self.nkeys, ptr(slot_of),
                counts.data_ptr(), ptr(order), sk.data_ptr(), ptr(sc), ptr(sv), bad.data_ptr(), st)
        check(rc)
        return counts, order, sk, sc, sv, bad

    def group(self, keys: torch.Tensor):
        """-> (order, counts): order = record indices grouped by partition in ``perm`` order (each
        group in the caller's order), counts = host int64 array of the group sizes (perm order)."""
        if keys.is_cuda:
            counts, order, _, _, _, bad = self.route(keys, want_order=True)
            if order is None:  # one partition: the identity
                order = torch.arange(keys.numel(), dtype=torch.int64, device=keys.device)
            host = torch.cat([counts, bad]).cpu().numpy()
            if host[-1] != 0:
                i = int(~host[-1])
                raise IndexOutOfBoundsException(f"key {int(keys[i])} (record {i}) outside [0, {self.nkeys})")
            return order, host[:-1]
        owner = self.partitioner.partition_indices(keys.numpy())  # raises IndexOutOfBoundsException
        o, off = bucket(owner, self.nparts)
        order, counts = torch.from_numpy(o), np.diff(off)
        if not self.identity:
            off = np.zeros(self.nparts + 1, dtype=np.int64)
            np.cumsum(counts, out=off[1:])
            order = torch.cat([order[off[p]:off[p + 1]] for p in self.perm])
            counts = counts[self.perm]
        return order, counts


def _row_bytes(t: torch.Tensor) -> int:
    return t.element_size() * (t[0].numel() if t.dim() > 1 else 1)


def copy_ranges(src: torch.Tensor, dst: torch.Tensor, ranges) -> None:
    """dst[d:d + c] = src[s:s + c] for every (s, d, c) in ranges (rows): one launch of
    glint_copy_segments_dev for device tensors; plain slices on the host."""
    ranges = [(int(a), int(b), int(c)) for a, b, c in ranges if c]
    if not ranges:
        return
    if src.is_cuda:
        rb = _row_bytes(src)
        segs = np.array([(a * rb, b * rb, c * rb) for a, b, c in ranges], dtype=np.int64).reshape(-1)
        check(N.load().glint_copy_segments_dev(src.data_ptr(), dst.data_ptr(),
                                               segs.ctypes.data_as(N.C.POINTER(N.C.c_int64)), len(ranges),
                                               torch.cuda.current_stream(src.device).cuda_stream))
        return
    for a, b, c in ranges:
        dst[b:b + c] = src[a:a + c]


def scatter_rows(src: torch.Tensor, order: torch.Tensor, out: torch.Tensor) -> None:
    """out[order[i]] = src[i] (rows): the answer's way back to the caller's order
    (AsyncBigVector.scala:61-79). Device tensors: one launch of glint_scatter_rows_dev; host tensors:
    index_copy_."""
    n = src.shape[0]
    if n == 0:
        return
    if src.is_cuda:
        check(N.load().glint_scatter_rows_dev(src.data_ptr(), order.data_ptr(), n, _row_bytes(src), out.data_ptr(),
                                              torch.cuda.current_stream(src.device).cuda_stream))
        return
    out.index_copy_(0, order, src)


class _Exchange:
    """The all-to-all legs of one routed call (send splits, receive splits, local layout).

    One code path for every backend: the (rank, partition) count matrix is built where the counts
    are (on the device for a device route, on the host for the host route), exchanged with one
    ``all_to_all_single``, and read by the host ONCE together with the route's status word; that
    single read gives both the send and the receive splits. Only the transport differs (``_a2a``):
    RCCL (``nccl``) exchanges device tensors, gloo host tensors. A batch with an out-of-range key
    sends nothing (every rank still joins the collectives) and raises after them, so the other
    ranks' pushes complete."""

    def __init__(self, router: Router, rank: int, counts: torch.Tensor, group, comm_device, bad=None,
                 bad_exc=None):
        W, maxp = router.world, router.maxp
        self.group, self.comm, self.world = group, comm_device, W
        self.bad = -1
        self.bad_exc = bad_exc
        if W == 1:
            # a world of one exchanges nothing: the counts (and the status word) are read as they are,
            # one small copy, and the send matrix is built on the host
            host = (torch.cat([counts, bad]) if bad is not None else counts).cpu().numpy()
            send_h = np.zeros((1, maxp), dtype=np.int64)
            if bad_exc is None and (bad is None or host[-1] == 0):
                send_h[0, router.slot_cell] = host[:counts.numel()]
            recv_h = send_h
        else:
            _, cell = router._device_tables(counts.device)
            if counts.is_cuda:  # one launch: the counts into their cells, all zero after a bad key
                send = torch.empty(W * maxp, dtype=torch.int64, device=counts.device)
                n = 0 if bad_exc is not None else counts.numel()
                check(N.load().glint_send_matrix_dev(counts.data_ptr(), cell.data_ptr(), n, W * maxp,
                                                     None if bad is None else bad.data_ptr(), send.data_ptr(),
                                                     torch.cuda.current_stream(counts.device).cuda_stream))
            else:
                send = torch.zeros(W * maxp, dtype=torch.int64, device=counts.device)
                if bad_exc is None:
                    send[cell] = counts
                if bad is not None:
                    send = torch.where(bad == 0, send, torch.zeros_like(send))
            recv = self._a2a(send)
            parts = [send, recv] + ([bad] if bad is not None else [])
            host = torch.cat(parts).cpu().numpy()  # the call's one host synchronisation
            send_h, recv_h = host[:W * maxp].reshape(W, maxp), host[W * maxp:2 * W * maxp].reshape(W, maxp)
        if bad is not None and host[-1] != 0:
            self.bad = int(~host[-1])
        self.recv_counts = recv_h  # [source rank, local partition j]
        self.in_splits = send_h.sum(axis=1).tolist()
        self.out_splits = recv_h.sum(axis=1).tolist()
        self.nlocal = len(router.rank_parts[rank])
        # start of each source rank's block in the received buffer, and of partition j inside it
        self._src_off = np.concatenate([[0], np.cumsum(recv_h.sum(axis=1))])
        self._part_off = np.concatenate([np.zeros((W, 1), np.int64), np.cumsum(recv_h, axis=1)], axis=1)

    def _a2a(self, t: torch.Tensor, out_splits=None, in_splits=None) -> torch.Tensor:
        """all_to_all_single on the backend's side of the bus, result on t's device: the only part
        of the exchange that depends on the backend."""
        src = t if t.device == self.comm else t.to(self.comm)
        rows = sum(out_splits) if out_splits is not None else t.shape[0]
        out = torch.empty((rows,) + tuple(t.shape[1:]), dtype=t.dtype, device=self.comm)
        dist.all_to_all_single(out, src.contiguous(), out_splits, in_splits, group=self.group)
        return out if out.device == t.device else out.to(t.device)

    def forward(self, t: torch.Tensor) -> torch.Tensor:
        if self.world == 1:  # a world of one exchanges with itself: the send buffer is the receive buffer
            return t[:self.out_splits[0]]
        return self._a2a(t[:sum(self.in_splits)], self.out_splits, self.in_splits)

    def backward(self, t: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return t
        return self._a2a(t, self.in_splits, self.out_splits)

    def raise_if_bad(self, keys: torch.Tensor, nkeys: int):
        if self.bad_exc is not None:
            raise self.bad_exc
        if self.bad >= 0:
            i = self.bad
            raise IndexOutOfBoundsException(f"key {int(keys[i])} (record {i}) outside [0, {nkeys})")

    def local_ranges(self, j: int):
        """Local partition j's records in the received buffer: one (start, length) range per source
        rank, in source-rank order (each source's records in its caller's order)."""
        return [(int(self._src_off[s] + self._part_off[s, j]), int(self.recv_counts[s, j]))
                for s in range(self.recv_counts.shape[0]) if self.recv_counts[s, j]]

    def take(self, buf: torch.Tensor, j: int) -> torch.Tensor:
        """Local partition j's records of a received buffer: a view when they are one range (one
        source, or one local partition), else the ranges gathered into one buffer by one
        multi-range copy (glint_copy_segments_dev) -- no index array."""
        if self.nlocal == 1:
            return buf
        rs = self.local_ranges(j)
        if not rs:
            return buf[:0]
        if len(rs) == 1:
            return buf[rs[0][0]:rs[0][0] + rs[0][1]]
        out = torch.empty((sum(c for _, c in rs),) + tuple(buf.shape[1:]), dtype=buf.dtype, device=buf.device)
        copy_ranges(buf, out, [(a, o, c) for (a, c), o in zip(rs, np.cumsum([0] + [c for _, c in rs]))])
        return out

    def single_range(self, j: int):
        """(start, length) of local partition j's records in the received buffer when they are one
        range (their answers can then be written in place), else None."""
        if self.nlocal == 1:
            return (0, int(self._src_off[-1]))
        rs = self.local_ranges(j)
        return rs[0] if len(rs) == 1 else None

    def put(self, resp: torch.Tensor, j: int, got: torch.Tensor) -> torch.Tensor:
        """Writes local partition j's answers into the response buffer (the inverse of take)."""
        if self.nlocal == 1:
            return got
        rs = self.local_ranges(j)
        copy_ranges(got, resp, [(o, a, c) for (a, c), o in zip(rs, np.cumsum([0] + [c for _, c in rs]))])
        return resp


def slab_layout(parts, cols: int, dtype):
    """Where a rank's partitions sit in its slab -> (start, end, rows), or None when they do not
    qualify (fewer than two, not all RangePartitions, more than an Int of rows): the slab is
    RangePartition(start, end) and partition j's first row in it is rows[j], each 256-byte aligned.
    * Side by side in key order (a rank's partitions at world 1), aligned: the slab spans their keys,
      so a key is its own slab key (delta 0) and a batch needs no route at all.
    * Otherwise (rank r of W hosts r, r + W, ...): one after another from row 0, each at the next
      256-byte boundary; the route rebases keys into it (glint_route_gather_rebased_dev).
    The same function of (parts, cols, dtype) on every rank, so each rank knows every slab's layout."""
    if len(parts) < 2 or not all(isinstance(p, RangePartition) for p in parts):
        return None
    _, np_dtype = resolve_dtype(dtype)
    vsize = np.dtype(np_dtype).itemsize
    pitch = -(-int(cols) // (16 // vsize)) * (16 // vsize) if cols else 1  # the library's row pitch
    step = 256 // math.gcd(256, pitch * vsize)  # rows per 256-byte boundary
    rows = [p.start - parts[0].start for p in parts]
    if all(a.end == b.start for a, b in zip(parts, parts[1:])) and all(r % step == 0 for r in rows):
        start, end = parts[0].start, parts[-1].end
    else:
        rows, r = [], 0
        for p in parts:
            rows.append(r)
            r = -(-(r + p.end - p.start) // step) * step
        start, end = 0, rows[-1] + parts[-1].end - parts[-1].start
    if end - start >= 2 ** 31:
        return None
    return start, end, rows


def slab_shards(kind: str, parts, cols: int, dtype, device: int):
    """The partitions one rank hosts as views of ONE slab (glint_shard_create_in, laid out by
    slab_layout) -> (slab, views), or None. A push whose records all belong to the rank is then one
    device-resident call on the slab -- one launch sequence for all of its partitions, where the
    reference sends a message per partition (AsyncBigVector.scala:96-98): _Distributed._push_gated
    (world 1, the slab spans the key space) and DistributedBigVector._push_slab (the route rebases
    keys into every rank's slab). Vectors only: a matrix keeps per-partition pushes (_slab_plan), so a
    matrix slab would buy nothing but alignment padding and one large allocation."""
    if kind != "vector":
        return None
    lay = slab_layout(parts, cols, dtype)
    if lay is None:
        return None
    start, end, rows = lay
    whole = RangePartition(parts[0].index, start, end)
    slab = PartialVector(whole, dtype, device) if kind == "vector" else PartialMatrix(whole, cols, dtype, device)
    views = [type(slab).view(slab, p, r) for p, r in zip(parts, rows)]
    return slab, views


class _Distributed:
    def __init__(self, partitioner, shards, group, device, slab=None):
        self.partitioner = partitioner
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.router = Router(partitioner, self.world)
        self.shards = list(shards)  # local shards, in rank_parts[rank] order
        self.device = device
        # the slab the local shards are views of (slab_shards), or None
        self.slab = slab

    @property
    def nrOfPartitions(self) -> int:
        return self.router.nparts

    def _comm(self, t: torch.Tensor) -> torch.device:
        # the transport's side of the bus: gloo exchanges host tensors, RCCL (nccl) device tensors
        return torch.device("cpu") if dist.get_backend(self.group) == "gloo" else t.device

    def _begin(self, keys: torch.Tensor):
        """Host route (CPU keys): order + counts on the host, records gathered by index. A batch with
        an out-of-range key sends nothing and raises after the collectives (raise_if_bad)."""
        exc = None
        try:
            order, counts = self.router.group(keys)
        except IndexOutOfBoundsException as e:
            exc = e
            order = torch.zeros(0, dtype=torch.int64, device=keys.device)
            counts = np.zeros(self.router.nparts, dtype=np.int64)
        ex = _Exchange(self.router, self.rank, torch.from_numpy(np.ascontiguousarray(counts, np.int64)), self.group,
                       self._comm(keys), bad_exc=exc)
        return order, ex

    def _begin_fused(self, keys, cols=None, vals=None, want_order=False, rebase=False):
        """Device route: the fused route writes the send buffers; one host read for the splits.
        rebase: keys written as their slab keys (_slab_plan's deltas)."""
        delta = None
        if rebase:
            if getattr(self, "_delta_dev", None) is None or self._delta_dev.device != keys.device:
                self._delta_dev = torch.from_numpy(self._delta).to(keys.device)
            delta = self._delta_dev
        counts, order, sk, sc, sv, bad = self.router.route(keys, cols, vals, want_order, key_delta=delta)
        ex = _Exchange(self.router, self.rank, counts, self.group, self._comm(keys), bad)
        return ex, order, sk, sc, sv

    def _to_shard(self, t: torch.Tensor) -> torch.Tensor:
        return t.to(self.device) if t.device != self.device else t

    def _split(self, ex: _Exchange, *bufs):
        for j, sh in enumerate(self.shards):
            yield j, sh, [ex.take(b, j) for b in bufs]

    def _on_shard_device(self, t: torch.Tensor) -> bool:
        return t.is_cuda and self.device.type == "cuda" and t.device == self.device

    def _nosync(self, t: torch.Tensor, out=None) -> dict:
        """Device-resident shard calls are enqueued without a wait (_sync waits once at the end), and
        a pull may write its answer straight into `out`."""
        kw = {"sync": False} if self._on_shard_device(t) else {}
        if out is not None:
            kw["out"] = out
        return kw

    @staticmethod
    def _sync(touched) -> None:
        for sh, t in touched:
            if t.is_cuda and hasattr(sh, "sync"):
                sh.sync(torch.cuda.current_stream(t.device).cuda_stream)

    def _stream(self, j: int) -> "torch.cuda.Stream":
        if not hasattr(self, "_streams"):
            self._streams = {}
        st = self._streams.get(j)
        if st is None:
            st = self._streams[j] = torch.cuda.Stream(self.device)
        return st

    def _run_local(self, ops) -> None:
        """The local shards' calls of one push: ops = [(j, shard, first tensor, call)]. Several device
        shards run concurrently, each on a stream of its own behind the caller's stream (the shards are
        independent, so one push's short kernels -- counts, scans, tails -- overlap another's), and the
        caller's stream waits for all of them; then one wait per shard (its errors)."""
        if len(ops) > 1 and all(self._on_shard_device(t) and hasattr(sh, "handle") for _, sh, t, _ in ops):
            cur = torch.cuda.current_stream(self.device)
            ready = torch.cuda.Event()
            ready.record(cur)
            done = []
            for j, sh, _, call in ops:
                st = self._stream(j)
                st.wait_event(ready)
                with torch.cuda.stream(st):
                    call()
                ev = torch.cuda.Event()
                ev.record(st)
                cur.wait_event(ev)
                done.append((sh, st))
            self._sync_all(done)
            return
        touched = []
        for _, sh, t, call in ops:
            call()
            touched.append((sh, t))
        self._sync(touched)

    @staticmethod
    def _sync_all(done) -> None:
        """Each (shard, stream)'s sync, with one library call for all of them (glint_shards_sync: every
        error-state copy enqueued before the first wait), raising as the first failing shard's sync."""
        lib = N.load()
        if len(done) < 2 or getattr(lib, "glint_shards_sync", None) is None:
            for sh, st in done:
                sh.sync(st.cuda_stream)
            return
        n = len(done)
        hs = (C.c_void_p * n)(*[sh.handle for sh, _ in done])
        ss = (C.c_void_p * n)(*[st.cuda_stream for _, st in done])
        rcs = (C.c_int * n)()
        bad = (C.c_int64 * n)(*([-1] * n))
        lib.glint_shards_sync(hs, ss, n, rcs, bad)
        for i, (sh, _) in enumerate(done):
            if rcs[i] == N.GLINT_EOUTOFRANGE:
                raise ArrayIndexOutOfBoundsException(f"record {bad[i]} is outside the partition", bad[i])
            check(rcs[i], sh.handle)

    def _gated_shard(self):
        """The one shard a world-of-one push goes to as it is: the only partition's, or the slab that
        holds every partition side by side (its range is the key space, so its key check is the
        route's; vectors only, _slab_plan)."""
        if self.world != 1:
            return None
        if self.router.nparts == 1:
            return self.shards[0]
        return self.slab if getattr(self, "_slab_keyed", False) else None

    def _slab_plan(self, np_dtype) -> None:
        """Vectors: whether pushes go to slabs, and the route's per-slot key deltas (key -> the key of
        its row in the hosting rank's slab, slab_layout). Decided the same way on every rank: the
        layouts are a function of the partitioner, and at world > 1 the ranks agree by one MIN
        all-reduce that every rank joins (a rank without a slab -- another shard factory, or
        slabs=False -- turns it off for all). (A matrix keeps per-partition pushes: a batch with
        a bad column fails only that partition's message in the reference.)"""
        self._delta, self._slab_keyed = None, False
        if not isinstance(self.partitioner, RangePartitioner) or self.router.maxp < 2:
            return
        parts = self.partitioner.all()
        lays = [slab_layout([parts[p] for p in self.router.rank_parts[r]], 0, np_dtype) for r in range(self.world)]
        if any(lay is None for lay in lays):
            return
        ok = self.slab is not None and self.slab.partition.start == lays[self.rank][0] and \
            self.slab.partition.end == lays[self.rank][1]
        if self.world > 1:
            t = torch.tensor([1 if ok else 0], dtype=torch.int64,
                             device="cpu" if dist.get_backend(self.group) == "gloo" else self.device)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
            ok = bool(t.item())
        if not ok:
            return
        d = np.zeros(self.router.nparts, np.int64)
        for r, (start, _, rows) in enumerate(lays):
            for j, p in enumerate(self.router.rank_parts[r]):
                d[self.router.slot_of[p]] = start + rows[j] - parts[p].start
        self._slab_keyed = self.world == 1 and not d.any()
        self._delta = d

    def _gate(self):
        """(address, int64 view) of the pinned host word a gated push writes its verdict into: one per
        model, used under _gate_lock."""
        if getattr(self, "_gate_buf", None) is None:
            from .shard import HostBuffer
            self._gate_lock = threading.Lock()
            self._gate_buf = HostBuffer(64)
            self._gate_arr = self._gate_buf.array(np.int64, 1)
        return self._gate_buf.ptr, self._gate_arr

    def _push_gated(self, keys: torch.Tensor, args: tuple, deterministic: bool) -> bool:
        """A world of one with one partition (or a slab holding all of them, slab_shards): the batch
        is the shard's push as it is. The key check
        (the route's validation pass) and the push are enqueued back to back -- the push gated on the
        route's status word on the device (glint_*_push_dev_gated: a batch with an out-of-range key
        applies nothing, as mapPartitions throws before sending, AsyncBigVector.scala:96-98) -- and the
        host reads the word after the one wait, so no synchronisation sits between them. The push checks
        the keys itself (GLINT_PUSH_VALIDATE: its order check reads them all) and writes the word, so no
        route pass reads them first. The word lives in pinned host memory (a HostBuffer): read after the
        one wait, with no device-to-host copy. Returns False when the call does not qualify (the general
        path then runs)."""
        sh = self._gated_shard()
        if not (sh is not None and keys.is_cuda and not deterministic
                and self._on_shard_device(keys) and hasattr(sh, "handle")):
            return False
        esz = args[-1].element_size()
        if keys.data_ptr() % 16 or args[-1].data_ptr() % (2 * esz) or (len(args) == 3 and args[1].data_ptr() % 8):
            return False
        gptr, word = self._gate()
        with self._gate_lock:  # one word per model: one gated push at a time
            sh.update(*args, gate=gptr, validate=True, sync=False)
            sh.sync(torch.cuda.current_stream(keys.device).cuda_stream)
            b = int(word[0])
        if b != 0:
            i = ~b
            k = int(keys[i])
            if len(args) == 3 and 0 <= k < self.router.nkeys:
                # the row is in range, so the column failed: what the general path's shard reports
                # (PartialMatrix.update indexes data(row)(col), PartialMatrix.scala:77-79)
                raise ArrayIndexOutOfBoundsException(
                    f"record {i}: column {int(args[1][i])} outside [0, {self.cols})", i)
            raise IndexOutOfBoundsException(f"key {k} (record {i}) outside [0, {self.router.nkeys})")
        return True

    def _answer(self, ex: _Exchange, order, bufs: tuple, caller: torch.Tensor, tail: tuple, get):
        """The pull's answer path: each local shard answers its records (get(shard, parts, out)), the
        answers travel back along the reversed splits and land in the caller's order
        (AsyncBigVector.scala:61-79, AsyncBigMatrix.scala:53-86).
        * world 1, device batch: each shard's answer is scattered straight to the caller's positions
          (glint_scatter_rows_dev over its range of `order`): no response buffer, no collective;
        * otherwise: answers are written into the response buffer (in place when a partition's records
          are one range, else by one multi-range copy), sent back, and scattered by `order`."""
        rk = bufs[0]
        n = caller.shape[0]
        out_shape = (n,) + tail
        touched = []
        if ex.world == 1 and order is not None and self._on_shard_device(rk):
            out = torch.empty(out_shape, dtype=self.dtype, device=caller.device)
            for j, sh, parts in self._split(ex, *bufs):
                if parts[0].numel():
                    a, c = ex.single_range(j)
                    got = get(sh, parts, None)
                    touched.append((sh, parts[0]))
                    scatter_rows(got, order[a:a + c], out)
            self._sync(touched)
            ex.raise_if_bad(caller, self.router.nkeys)
            return out
        resp = torch.empty((rk.shape[0],) + tail, dtype=self.dtype, device=rk.device)
        for j, sh, parts in self._split(ex, *bufs):
            if parts[0].numel():
                rng = ex.single_range(j)
                k = [self._to_shard(p) for p in parts]
                if rng is not None and self._on_shard_device(rk):  # answered in place
                    get(sh, k, resp[rng[0]:rng[0] + rng[1]])
                else:
                    got = get(sh, k, None)
                    resp = ex.put(resp, j, got.to(resp.device).reshape((-1,) + tail))
                touched.append((sh, k[0]))
        self._sync(touched)
        back = ex.backward(resp).to(caller.device)
        ex.raise_if_bad(caller, self.router.nkeys)  # after the collectives: this rank asked for nothing
        if order is None:  # one partition: the answer is already in the caller's order
            return back
        out = torch.empty(out_shape, dtype=self.dtype, device=caller.device)
        scatter_rows(back, order.to(caller.device), out)
        return out

    def destroy(self) -> bool:
        for sh in self.shards:
            sh.destroy()
        if self.slab is not None:  # after its views
            self.slab.destroy()
        if getattr(self, "_gate_buf", None) is not None:
            self._gate_buf.free()
            self._gate_buf = None
        return True


class DistributedBigVector(_Distributed):
    """AsyncBigVector over the ranks of a process group (push / pull of any keys from any rank)."""

    def __init__(self, partitioner, shards, size: int, np_dtype, group=None, device=None, slab=None):
        super().__init__(partitioner, shards, group, device, slab)
        self.size = int(size)
        self.dtype = _TORCH_DTYPES[np.dtype(np_dtype)]
        self._slab_plan(np_dtype)


    def _set_ok(self, n: int) -> bool:
        """Whether a sparse batch of n records (fewer than 1/8 of this rank's keys, where every shard
        push would take the atomic scatter anyway) can go to all local shards in ONE launch sequence
        (glint_vec_push_dev_shards): range vector shards on this GPU, 2..64 of them."""
        m = len(self.shards)
        if not (1 < m <= 64 and isinstance(self.partitioner, RangePartitioner) and self.device.type == "cuda"
                and all(hasattr(sh, "handle") for sh in self.shards)):
            return False
        return n * 8 < sum(sh.size for sh in self.shards)

    def _set_push(self, keys: torch.Tensor, values: torch.Tensor) -> int:
        """glint_vec_push_dev_shards over the local shards, then one wait for all of them
        (glint_shards_sync: each member's error state, hints latched): -> the verdict word (0, or ~ the
        first record whose key is in no local shard; nothing applied then)."""
        n = keys.numel()
        m = len(self.shards)
        for sh in self.shards:  # (their dtype and device: the library checks the set agrees)
            sh._check_dev(n, keys, values=values)
        hs = getattr(self, "_set_handles", None)
        if hs is None:
            hs = self._set_handles = (C.c_void_p * m)(*[sh.handle for sh in self.shards])
        stream = torch.cuda.current_stream(self.device).cuda_stream
        gptr, word = self._gate()
        with self._gate_lock:
            check(N.load().glint_vec_push_dev_shards(hs, m, keys.data_ptr(), values.data_ptr(), n, gptr, stream))
            cur = torch.cuda.current_stream(self.device)
            self._sync_all([(sh, cur) for sh in self.shards])
            return int(word[0])

    def _push_set(self, keys: torch.Tensor, values: torch.Tensor) -> bool:
        """World 1, several partitions, no key-spanning slab, a sparse batch: one call for all local
        shards (_set_push) -- the keys checked against the shards' ranges, then one scatter sending each
        aggregate to its shard -- in place of the route, the split and a push per partition. A key
        outside the key space applies nothing and raises as the route would."""
        if not (self.world == 1 and keys.is_cuda and self._on_shard_device(keys) and values.device == keys.device
                and self._set_ok(keys.numel())):
            return False
        keys = keys.contiguous()
        b = self._set_push(keys, values.contiguous())
        if b != 0:
            i = ~b
            raise IndexOutOfBoundsException(f"key {int(keys[i])} (record {i}) outside [0, {self.router.nkeys})")
        return True

    def _push_slab(self, keys: torch.Tensor, values: torch.Tensor) -> bool:
        """Every rank's partitions in one slab (_slab_plan): the route writes each key rebased into
        the hosting rank's slab (glint_route_gather_rebased_dev), the exchange sends the records as
        usual, and each rank pushes ALL it received as one unordered call on its slab -- no
        per-partition split, no per-partition push. Keys were checked by the route (a batch with a bad
        one sends nothing and raises after the collectives), so the slab push cannot reject any."""
        if self._delta is None or not (keys.is_cuda and self._on_shard_device(keys) and values.device == keys.device):
            return False
        ex, _, sk, _, sv = self._begin_fused(keys, vals=values.contiguous(), rebase=True)
        rk, rv = ex.forward(sk), ex.forward(sv)
        if rk.numel():
            stream = torch.cuda.current_stream(self.device).cuda_stream
            self.slab.update(self._to_shard(rk), self._to_shard(rv), sync=False, unordered=True)
            self.slab.sync(stream)
        ex.raise_if_bad(keys, self.router.nkeys)
        return True

    def push(self, keys: torch.Tensor, values: torch.Tensor, deterministic: bool = False) -> bool:
        keys = keys.reshape(-1).to(torch.int64)
        values = values.reshape(-1).to(self.dtype)
        if keys.numel() != values.numel():
            raise ValueError("keys and values differ in length")
        if values.device == keys.device and self._push_gated(keys, (keys, values.contiguous()), deterministic):
            return True
        if not deterministic and (self._push_set(keys, values) or self._push_slab(keys, values)):
            return True
        if keys.is_cuda and values.device == keys.device:
            ex, _, sk, _, sv = self._begin_fused(keys, vals=values.contiguous())
            rk, rv = ex.forward(sk), ex.forward(sv)
        else:
            order, ex = self._begin(keys)
            rk = ex.forward(keys.index_select(0, order))
            rv = ex.forward(values.index_select(0, order.to(values.device)))
        if not deterministic and self._set_ok(rk.numel()) and rk.numel():
            # a sparse receive: every local partition's records in one call, no split (keys validated by
            # the route, so the verdict is 0)
            if self._set_push(self._to_shard(rk).contiguous(), self._to_shard(rv).contiguous()) != 0:
                raise RuntimeError("routed records outside the local shards")
            ex.raise_if_bad(keys, self.router.nkeys)
            return True
        ops = []
        for j, sh, (k, v) in self._split(ex, rk, rv):
            if k.numel():
                # every local push is enqueued before the first wait (keys are validated by the route)
                ops.append((j, sh, k, lambda sh=sh, k=k, v=v: sh.update(
                    self._to_shard(k), self._to_shard(v), deterministic=deterministic, **self._nosync(k))))
        self._run_local(ops)
        ex.raise_if_bad(keys, self.router.nkeys)
        return True

    def _pull_slab(self, keys: torch.Tensor) -> torch.Tensor:
        """World 1 with every partition side by side in one slab (_slab_keyed): the batch's keys are
        checked as the route checks them (glint_route_gather_dev with one partition: a read of the
        keys, the raw 64-bit range) and the slab answers them in the caller's order in one gather --
        no grouping, no per-partition pulls, no scatter back. A bad key raises the route's exception
        (the slab's own check, which the gather makes on its (key - start).toInt, is not the one
        reported)."""
        keys = keys.contiguous()
        n, dev = keys.numel(), keys.device
        st = torch.cuda.current_stream(dev).cuda_stream
        counts = torch.empty(1, dtype=torch.int64, device=dev)
        bad = torch.empty(1, dtype=torch.int64, device=dev)
        check(N.load().glint_route_gather_dev(keys.data_ptr(), None, None, 0, n, N.GLINT_ROUTE_RANGE, 1,
                                              self.router.nkeys, None, counts.data_ptr(), None, None, None, None,
                                              bad.data_ptr(), st))
        out = torch.empty(n, dtype=self.dtype, device=dev)
        try:
            self.slab.get(keys, out=out)  # (one wait, on this stream: the check above is done too)
        except ArrayIndexOutOfBoundsException:
            # outside the slab = outside the key space, and the route's word names the record; a slab
            # that rejects a key the route passed would leave `out` partly unwritten
            if int(bad.item()) == 0:
                raise RuntimeError("the slab rejected a key inside the key space") from None
        b = int(bad.item())
        if b != 0:
            i = ~b
            raise IndexOutOfBoundsException(f"key {int(keys[i])} (record {i}) outside [0, {self.router.nkeys})")
        return out

    def pull(self, keys: torch.Tensor) -> torch.Tensor:
        keys = keys.reshape(-1).to(torch.int64)
        if keys.is_cuda and self._slab_keyed and self._on_shard_device(keys):
            return self._pull_slab(keys)
        if keys.is_cuda:
            ex, order, sk, _, _ = self._begin_fused(keys, want_order=True)
            rk = ex.forward(sk)
        else:
            order, ex = self._begin(keys)
            rk = ex.forward(keys.index_select(0, order))
        return self._answer(ex, order, (rk,), keys, (), lambda sh, p, out: sh.get(p[0], **self._nosync(p[0], out)))


class DistributedBigMatrix(_Distributed):
    """AsyncBigMatrix over the ranks of a process group."""

    def __init__(self, partitioner, shards, rows: int, cols: int, np_dtype, group=None, device=None, slab=None):
        super().__init__(partitioner, shards, group, device, slab)
        self.rows, self.cols = int(rows), int(cols)
        self.dtype = _TORCH_DTYPES[np.dtype(np_dtype)]

    def push(self, rows: torch.Tensor, cols: torch.Tensor, values: torch.Tensor,
             deterministic: bool = False) -> bool:
        rows = rows.reshape(-1).to(torch.int64)
        cols = cols.reshape(-1).to(torch.int32)
        values = values.reshape(-1).to(self.dtype)
        if not rows.numel() == cols.numel() == values.numel():
            raise ValueError("rows, cols and values differ in length")
        if cols.device == rows.device and values.device == rows.device and \
                self._push_gated(rows, (rows, cols.contiguous(), values.contiguous()), deterministic):
            return True
        if rows.is_cuda and cols.device == rows.device and values.device == rows.device:
            ex, _, sr, sc, sv = self._begin_fused(rows, cols=cols.contiguous(), vals=values.contiguous())
            rr, rc, rv = (ex.forward(t) for t in (sr, sc, sv))
        else:
            order, ex = self._begin(rows)
            rr = ex.forward(rows.index_select(0, order))
            rc = ex.forward(cols.index_select(0, order.to(cols.device)))
            rv = ex.forward(values.index_select(0, order.to(values.device)))
        ops = []
        for j, sh, (r, c, v) in self._split(ex, rr, rc, rv):
            if r.numel():
                ops.append((j, sh, r, lambda sh=sh, r=r, c=c, v=v: sh.update(
                    self._to_shard(r), self._to_shard(c), self._to_shard(v), deterministic=deterministic,
                    **self._nosync(r))))
        self._run_local(ops)
        ex.raise_if_bad(rows, self.router.nkeys)
        return True

    def pull(self, rows: torch.Tensor, cols: Optional[torch.Tensor] = None) -> torch.Tensor:
        """pull(rows, cols): elements (AsyncBigMatrix.scala:96-130); pull(rows): whole rows as an
        (n, cols) tensor (AsyncBigMatrix.scala:53-86)."""
        rows = rows.reshape(-1).to(torch.int64)
        if cols is not None:
            cols = cols.reshape(-1).to(torch.int32)
        if rows.is_cuda and (cols is None or cols.device == rows.device):
            ex, order, sr, sc, _ = self._begin_fused(rows, cols=None if cols is None else cols.contiguous(),
                                                     want_order=True)
            rr = ex.forward(sr)
            rc = None if cols is None else ex.forward(sc)
        else:
            order, ex = self._begin(rows)
            rr = ex.forward(rows.index_select(0, order))
            rc = None if cols is None else ex.forward(cols.index_select(0, order.to(cols.device)))
        if cols is None:
            return self._answer(ex, order, (rr,), rows, (self.cols,),
                                lambda sh, p, out: sh.getRows(p[0], **self._nosync(p[0], out)))
        return self._answer(ex, order, (rr, rc), rows, (),
                            lambda sh, p, out: sh.get(p[0], p[1], **self._nosync(p[0], out)))


class DistributedClient:
    """glint.Client's model factory over a process group: rank r hosts partitions r, r + W, ...

    ``shard_factory(kind, partition, cols, dtype, device)`` builds a local shard; the default makes
    ``PartialVector`` / ``PartialMatrix`` HBM shards on ``device`` (this rank's GPU). ``slabs=False``
    keeps a vector's local partitions in shards of their own instead of views of one slab
    (slab_shards)."""

    def __init__(self, group=None, device=None, shard_factory: Optional[Callable] = None, slabs: bool = True):
        if not dist.is_initialized():
            raise ModelCreationException("torch.distributed is not initialised")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        self.shard_factory = shard_factory or self._hbm_shard
        self.slabs = bool(slabs)

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
        if self.slabs and self.shard_factory == self._hbm_shard and self.device.type == "cuda":
            sv = slab_shards(kind, [parts[p] for p in mine], cols, dtype, self.device.index)
            if sv is not None:  # the rank's partitions side by side in one slab
                return partitioner, sv[1], sv[0]
        shards = [self.shard_factory(kind, parts[p], cols, dtype, self.device) for p in mine]
        return partitioner, shards, None

    def vector(self, keys: int, dtype="double", modelsPerServer: int = 1,
               createPartitioner: Callable = RangePartitioner.apply) -> DistributedBigVector:
        _, np_dtype = resolve_dtype(dtype)
        partitioner, shards, slab = self._create(keys, modelsPerServer, createPartitioner, "vector", 0, dtype)
        return DistributedBigVector(partitioner, shards, keys, np_dtype, self.group, self.device, slab)

    def matrix(self, rows: int, cols: int, dtype="double", modelsPerServer: int = 1,
               createPartitioner: Callable = RangePartitioner.apply) -> DistributedBigMatrix:
        _, np_dtype = resolve_dtype(dtype)
        partitioner, shards, slab = self._create(rows, modelsPerServer, createPartitioner, "matrix", cols, dtype)
        return DistributedBigMatrix(partitioner, shards, rows, cols, np_dtype, self.group, self.device, slab)


__all__ = ["Router", "DistributedClient", "DistributedBigVector", "DistributedBigMatrix", "slab_shards"]
