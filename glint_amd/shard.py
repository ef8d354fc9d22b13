"""Host-side mirror of Glint's server-side partial models, backed by HBM shards.

``PartialVector`` / ``PartialMatrix`` keep the reference's method names and argument meaning
(src/main/scala/glint/models/server/PartialVector.scala:16-64, PartialMatrix.scala:17-87):

    vec = PartialVector(RangePartition(0, 0, 1000), "double")
    vec.update(keys, values)      # PartialVector.update  -> True
    vec.get(keys)                 # PartialVector.get     -> array of values

Every operation runs the HIP kernels through the C ABI (include/glint_gpu.h). Arguments may be
numpy arrays (host path: staged H2D, synchronous like the actor's ``update``) or torch CUDA tensors
on the shard's device (device-resident path, stream-ordered on torch's current stream; the call
synchronises only when ``sync=True``).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import _native as N
from .errors import ArrayIndexOutOfBoundsException, GlintDeviceError
from .partitioning import CyclicPartition, Partition, RangePartition

_DTYPES = {
    "int": (N.GLINT_I32, np.int32), "int32": (N.GLINT_I32, np.int32), "i32": (N.GLINT_I32, np.int32),
    "long": (N.GLINT_I64, np.int64), "int64": (N.GLINT_I64, np.int64), "i64": (N.GLINT_I64, np.int64),
    "float": (N.GLINT_F32, np.float32), "float32": (N.GLINT_F32, np.float32), "f32": (N.GLINT_F32, np.float32),
    "double": (N.GLINT_F64, np.float64), "float64": (N.GLINT_F64, np.float64), "f64": (N.GLINT_F64, np.float64),
}


def resolve_dtype(dtype) -> tuple:
    """Map a value type ('double', np.float64, 'Int', ...) to (GLINT_* code, numpy dtype)."""
    if isinstance(dtype, str):
        key = dtype.lower()
    else:
        key = np.dtype(dtype).name
    if key not in _DTYPES:
        raise ValueError(f"unsupported value type {dtype!r} (Int, Long, Float or Double)")
    return _DTYPES[key]


def check(rc: int, handle=None) -> None:
    """Translate a C ABI status into the reference's exception types."""
    if rc == N.GLINT_OK:
        return
    if rc == N.GLINT_EOUTOFRANGE:
        rec = -1
        if handle is not None:
            v = C.c_int64(-1)
            N.load().glint_shard_last_error(handle, C.byref(v))
            rec = v.value
        raise ArrayIndexOutOfBoundsException(f"record {rec} is outside the partition", rec)
    if rc == N.GLINT_EDEVICE:
        raise GlintDeviceError(N.strerror(rc))
    if rc == N.GLINT_ENOMEM:
        raise MemoryError(N.strerror(rc))
    raise ValueError(N.strerror(rc))


def _flags(deterministic: bool, unordered: bool) -> int:
    return (N.GLINT_PUSH_DETERMINISTIC if deterministic else 0) | (N.GLINT_PUSH_UNORDERED if unordered else 0)


def _addr(x) -> int:
    """A raw address (int) as it is, else the tensor's data pointer."""
    return x if isinstance(x, int) else x.data_ptr()


def _is_torch_cuda(x) -> bool:
    return type(x).__module__.startswith("torch") and getattr(x, "is_cuda", False)


def _host(x, dtype) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x, dtype=dtype))


class HostBuffer:
    """Pinned, device-mapped host memory from glint_host_alloc: the buffers a server answers pulls
    from. A message-sized pull whose ``out`` lies in one is answered by the kernel straight into it
    (no copy out of the ring slot when it retires). ``array(dtype, count, offset)`` views a part of it
    as a numpy array; free() (or leaving the ``with`` block) only once no pull into it is pending."""

    def __init__(self, nbytes: int):
        self.lib = N.load()
        p = C.c_void_p()
        check(self.lib.glint_host_alloc(int(nbytes), C.byref(p)))
        self.ptr, self.nbytes = p.value, int(nbytes)

    def array(self, dtype, count: int, offset: int = 0) -> np.ndarray:
        dt = np.dtype(dtype)
        if offset < 0 or offset + count * dt.itemsize > self.nbytes:
            raise ValueError("outside the buffer")
        raw = (C.c_char * (count * dt.itemsize)).from_address(self.ptr + offset)
        return np.frombuffer(raw, dtype=dt, count=count)

    def free(self) -> None:
        if self.ptr:
            check(self.lib.glint_host_free(self.ptr))
            self.ptr = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.free()


class _Shard:
    def __init__(self, partition: Partition, dtype, cols: int = 0, device: int = 0):
        self.lib = N.load()
        self.partition = partition
        self.code, self.np_dtype = resolve_dtype(dtype)
        self.device = int(device)
        self._h = C.c_void_p()
        if isinstance(partition, RangePartition):
            rc = self.lib.glint_shard_create(self.device, self.code, partition.start, partition.end, int(cols),
                                             C.byref(self._h))
        elif isinstance(partition, CyclicPartition):
            rc = self.lib.glint_shard_create_cyclic(self.device, self.code, partition.index,
                                                    partition.numberOfPartitions, partition.numberOfKeys,
                                                    int(cols), C.byref(self._h))
        else:
            raise TypeError(f"unsupported partition type {type(partition).__name__}")
        check(rc)
        sz, cl = C.c_int32(), C.c_int32()
        check(self.lib.glint_shard_info(self._h, C.byref(sz), C.byref(cl), None, None), self._h)
        self.size = sz.value
        self.cols = cl.value

    @classmethod
    def view(cls, slab: "_Shard", partition: RangePartition, offset: int):
        """A shard over ``partition`` whose elements are rows [offset, offset + size) of ``slab``
        (glint_shard_create_in): the partitions a server hosts, kept in one allocation so that one
        device-resident call on the slab serves all of them. Destroy views before their slab."""
        if not isinstance(partition, RangePartition):
            raise TypeError("a slab view takes a RangePartition")
        self = cls.__new__(cls)
        self.lib, self.partition, self.device = slab.lib, partition, slab.device
        self.code, self.np_dtype = slab.code, slab.np_dtype
        self._h = C.c_void_p()
        check(self.lib.glint_shard_create_in(slab.handle, int(offset), partition.start, partition.end, C.byref(self._h)))
        sz, cl = C.c_int32(), C.c_int32()
        check(self.lib.glint_shard_info(self._h, C.byref(sz), C.byref(cl), None, None), self._h)
        self.size, self.cols = sz.value, cl.value
        if cl.value:
            self.rows = self.size
        self.slab = slab
        return self

    # lifetime -------------------------------------------------------------------------------
    @property
    def handle(self) -> C.c_void_p:
        if not self._h:
            raise ValueError("shard already destroyed")
        return self._h

    def destroy(self) -> None:
        if self._h:
            check(self.lib.glint_shard_destroy(self._h))  # (a slab with live views refuses: EINVAL)
            self._h = C.c_void_p()

    close = destroy

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.destroy()

    def zero(self) -> None:
        """What an Akka restart produces: a freshly constructed, zeroed partial model."""
        check(self.lib.glint_shard_zero(self.handle), self.handle)

    def data_ptr(self) -> int:
        p = C.c_void_p()
        check(self.lib.glint_shard_data(self.handle, C.byref(p)), self.handle)
        return p.value or 0

    # pipelined host ingest (include/glint_gpu.h): enqueue now, wait for the ticket before acknowledging
    def push_async(self, *arrays, deterministic: bool = False, unordered: bool = False) -> int:
        """Stage (keys, values) -- or (rows, cols, values) for a matrix -- in a pinned ring slot and
        enqueue the push; returns its ticket (glint_stage_acquire + glint_push_staged). A record outside
        the partition raises ArrayIndexOutOfBoundsException here, at the message (as update() throws in
        the reference), and nothing of the message is applied."""
        mat = self.cols != 0
        if len(arrays) != (3 if mat else 2):
            raise ValueError("push_async(keys, values) for vectors, (rows, cols, values) for matrices")
        keys = _host(arrays[0], np.int64).reshape(-1)
        cols = _host(arrays[1], np.int32).reshape(-1) if mat else None
        vals = _host(arrays[-1], self.np_dtype).reshape(-1)
        if keys.size != vals.size or (mat and cols.size != keys.size):
            raise ValueError("argument lengths differ")
        n = keys.size
        kp, cp, vp, slot = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_int(-1)
        check(self.lib.glint_stage_acquire(self.handle, n, C.byref(kp), C.byref(cp), C.byref(vp), C.byref(slot)),
              self.handle)
        if n:
            C.memmove(kp.value, keys.ctypes.data, keys.nbytes)
            if mat:
                C.memmove(cp.value, cols.ctypes.data, cols.nbytes)
            C.memmove(vp.value, vals.ctypes.data, vals.nbytes)
        ticket = C.c_uint64()
        check(self.lib.glint_push_staged(self.handle, slot.value, n, _flags(deterministic, unordered),
                                         C.byref(ticket)), self.handle)
        return ticket.value

    def push_wire_async(self, payload: bytes, deterministic: bool = False):
        """Enqueue a RequestSerializer push image; returns (message id, ticket)."""
        buf = (C.c_uint8 * len(payload)).from_buffer_copy(payload)
        mid, ticket = C.c_int32(), C.c_uint64()
        flags = N.GLINT_PUSH_DETERMINISTIC if deterministic else N.GLINT_PUSH_DEFAULT
        check(self.lib.glint_push_wire_async(self.handle, buf, len(payload), C.byref(mid), flags, C.byref(ticket)),
              self.handle)
        return mid.value, ticket.value

    def pull_async(self, *arrays, rows: bool = False, out=None):
        """Enqueue a pull -- get(keys) for vectors, get(rows, cols) or getRows(rows) (rows=True) for
        matrices -- behind everything enqueued before it (glint_pull_async). Returns (ticket, out):
        `out` holds the answer once wait(ticket) has returned; keep it alive until then."""
        mat = self.cols != 0
        kind = 0 if not mat else (2 if rows else 1)
        if len(arrays) != (2 if kind == 1 else 1):
            raise ValueError("pull_async(keys) for vectors and row pulls, (rows, cols) for matrix elements")
        keys = _host(arrays[0], np.int64).reshape(-1)
        cols = _host(arrays[1], np.int32).reshape(-1) if kind == 1 else None
        if kind == 1 and cols.size != keys.size:
            raise ValueError("argument lengths differ")
        out = self._host_out(out, (keys.size, self.cols) if kind == 2 else (keys.size,))
        ticket = C.c_uint64()
        check(self.lib.glint_pull_async(self.handle, kind, keys.ctypes.data, None if cols is None else cols.ctypes.data,
                                        out.ctypes.data, keys.size, C.byref(ticket)), self.handle)
        return ticket.value, out

    def wait(self, ticket: int) -> None:
        """Until the push with this ticket (and every earlier one) is applied; raises GlintDeviceError if
        one of them failed to launch (rejected records raise at the enqueueing call instead)."""
        bad = C.c_int64(-1)
        rc = self.lib.glint_shard_wait(self.handle, ticket, C.byref(bad))
        if rc == N.GLINT_EOUTOFRANGE:
            raise ArrayIndexOutOfBoundsException(f"record {bad.value} is outside the partition", bad.value)
        check(rc, self.handle)

    def sync(self, stream: Optional[int] = None) -> None:
        """Wait for device-resident calls and raise if any of them rejected a record."""
        bad = C.c_int64(-1)
        rc = self.lib.glint_shard_sync(self.handle, stream, C.byref(bad))
        if rc == N.GLINT_EOUTOFRANGE:
            raise ArrayIndexOutOfBoundsException(f"record {bad.value} is outside the partition", bad.value)
        check(rc, self.handle)

    @staticmethod
    def _stream_of(t) -> int:
        import torch
        return torch.cuda.current_stream(t.device).cuda_stream

    @property
    def torch_dtype(self):
        import torch
        return getattr(torch, np.dtype(self.np_dtype).name)

    def _check_dev(self, n: int, keys, cols=None, values=None, out=None, out_elems=None) -> None:
        """Device-resident arguments: every tensor on the shard's GPU, contiguous, of the dtype the
        kernels read (keys/rows int64, cols int32, values/out the shard's type) and long enough --
        the kernels take raw pointers, so a mismatch would read or write past a buffer."""
        import torch
        spec = [("keys", keys, torch.int64, n)]
        if cols is not None:
            spec.append(("cols", cols, torch.int32, n))
        if values is not None:
            spec.append(("values", values, self.torch_dtype, n))
        if out is not None:
            spec.append(("out", out, self.torch_dtype, n if out_elems is None else out_elems))
        for name, t, dt, want in spec:
            if not _is_torch_cuda(t):
                raise TypeError(f"{name}: expected a CUDA tensor (mixing host arrays and device tensors)")
            if t.device.index != self.device:
                raise ValueError(f"{name} on cuda:{t.device.index}, shard on cuda:{self.device}")
            if not t.is_contiguous():
                raise ValueError(f"{name}: device tensors must be contiguous")
            if t.dtype != dt:
                raise TypeError(f"{name}: dtype {t.dtype}, expected {dt}")
            if t.numel() != want:
                raise ValueError(f"{name}: {t.numel()} elements, expected {want}")

    def _host_out(self, out, shape) -> np.ndarray:
        """A caller-provided host result buffer must be a writable C-contiguous array of the shard's
        type and exact shape (the library writes n x sizeof(V) bytes into it)."""
        if out is None:
            return np.empty(shape, dtype=self.np_dtype)
        if not isinstance(out, np.ndarray) or out.dtype != self.np_dtype or out.shape != tuple(shape) \
                or not out.flags.c_contiguous or not out.flags.writeable:
            raise ValueError(f"out must be a writable C-contiguous {np.dtype(self.np_dtype).name} array of shape "
                             f"{tuple(shape)}")
        return out


class PartialVector(_Shard):
    """glint.models.server.PartialVector (PartialVector.scala:16-64) on one MI355X."""

    def __init__(self, partition: Partition, dtype="double", device: int = 0):
        super().__init__(partition, dtype, 0, device)

    def update(self, keys, values, deterministic: bool = False, sync: bool = True, unordered: bool = False,
               gate=None, validate: bool = False) -> bool:
        """PartialVector.update (PartialVector.scala:35-43): data(globalToLocal(k)) += v.
        ``unordered`` is a performance hint (GLINT_PUSH_UNORDERED): skip the order check, bin by slab.
        ``gate`` (device tensors only): a one-element int64 device tensor, or the address of a word in a
        HostBuffer; the push applies nothing if it is nonzero when the push runs
        (glint_vec_push_dev_gated). With ``validate`` the push writes the gate itself
        (GLINT_PUSH_VALIDATE): 0, or ~(first out-of-range record), which cancels it."""
        flags = _flags(deterministic, unordered) | (N.GLINT_PUSH_VALIDATE if validate else 0)
        if _is_torch_cuda(keys):
            self._check_dev(keys.numel(), keys, values=values)
            if gate is not None:
                rc = self.lib.glint_vec_push_dev_gated(self.handle, keys.data_ptr(), values.data_ptr(), keys.numel(),
                                                       flags, _addr(gate), self._stream_of(keys))
            else:
                rc = self.lib.glint_vec_push_dev(self.handle, keys.data_ptr(), values.data_ptr(), keys.numel(), flags,
                                                 self._stream_of(keys))
            check(rc, self.handle)
            if sync:
                self.sync(self._stream_of(keys))
            return True
        k = _host(keys, np.int64)
        v = _host(values, self.np_dtype)
        if k.shape != v.shape:
            raise ValueError("keys and values differ in length")
        check(self.lib.glint_vec_push(self.handle, k.ctypes.data, v.ctypes.data, k.size, flags), self.handle)
        return True

    def get(self, keys, out=None, sync: bool = True):
        """PartialVector.get (PartialVector.scala:51-60): a new array of data(globalToLocal(k))."""
        if _is_torch_cuda(keys):
            import torch
            if out is None:
                out = torch.empty(keys.numel(), dtype=self.torch_dtype, device=keys.device)
            self._check_dev(keys.numel(), keys, out=out)
            rc = self.lib.glint_vec_pull_dev(self.handle, keys.data_ptr(), out.data_ptr(), keys.numel(),
                                             self._stream_of(keys))
            check(rc, self.handle)
            if sync:
                self.sync(self._stream_of(keys))
            return out
        k = _host(keys, np.int64)
        res = self._host_out(out, k.shape)
        check(self.lib.glint_vec_pull(self.handle, k.ctypes.data, res.ctypes.data, k.size), self.handle)
        return res

    def push_wire(self, payload: bytes, deterministic: bool = False) -> int:
        """Apply a RequestSerializer Push*Vector* byte image; returns its message id."""
        buf = (C.c_uint8 * len(payload)).from_buffer_copy(payload)
        mid = C.c_int32()
        flags = N.GLINT_PUSH_DETERMINISTIC if deterministic else N.GLINT_PUSH_DEFAULT
        check(self.lib.glint_push_wire(self.handle, buf, len(payload), C.byref(mid), flags), self.handle)
        return mid.value

    def pull_wire(self, payload: bytes) -> bytes:
        """Answer a RequestSerializer PullVector byte image with the ResponseSerializer image."""
        return _pull_wire(self, payload)

    def to_numpy(self) -> np.ndarray:
        """Whole shard to host (a pull of every local key through the product path)."""
        p = self.partition
        if isinstance(p, RangePartition):
            keys = np.arange(p.start, p.start + self.size, dtype=np.int64)
        else:
            keys = np.arange(self.size, dtype=np.int64) * p.numberOfPartitions + p.index
        return self.get(keys)


class PartialMatrix(_Shard):
    """glint.models.server.PartialMatrix (PartialMatrix.scala:17-87) on one MI355X."""

    def __init__(self, partition: Partition, cols: int, dtype="double", device: int = 0):
        if int(cols) <= 0:
            raise ValueError("a matrix shard needs cols > 0")
        super().__init__(partition, dtype, int(cols), device)
        self.rows = self.size

    def update(self, rows, cols, values, deterministic: bool = False, sync: bool = True,
               unordered: bool = False, gate=None, validate: bool = False) -> bool:
        """PartialMatrix.update (PartialMatrix.scala:74-83); ``gate`` and ``validate`` as for
        PartialVector.update."""
        flags = _flags(deterministic, unordered) | (N.GLINT_PUSH_VALIDATE if validate else 0)
        if _is_torch_cuda(rows):
            self._check_dev(rows.numel(), rows, cols=cols, values=values)
            if gate is not None:
                rc = self.lib.glint_mat_push_dev_gated(self.handle, rows.data_ptr(), cols.data_ptr(),
                                                       values.data_ptr(), rows.numel(), flags, _addr(gate),
                                                       self._stream_of(rows))
            else:
                rc = self.lib.glint_mat_push_dev(self.handle, rows.data_ptr(), cols.data_ptr(), values.data_ptr(),
                                                 rows.numel(), flags, self._stream_of(rows))
            check(rc, self.handle)
            if sync:
                self.sync(self._stream_of(rows))
            return True
        r = _host(rows, np.int64)
        c = _host(cols, np.int32)
        v = _host(values, self.np_dtype)
        if not (r.shape == c.shape == v.shape):
            raise ValueError("rows, cols and values differ in length")
        check(self.lib.glint_mat_push(self.handle, r.ctypes.data, c.ctypes.data, v.ctypes.data, r.size, flags),
              self.handle)
        return True

    def get(self, rows, cols, out=None, sync: bool = True):
        """PartialMatrix.get (PartialMatrix.scala:55-65)."""
        if _is_torch_cuda(rows):
            import torch
            if out is None:
                out = torch.empty(rows.numel(), dtype=self.torch_dtype, device=rows.device)
            self._check_dev(rows.numel(), rows, cols=cols, out=out)
            rc = self.lib.glint_mat_pull_dev(self.handle, rows.data_ptr(), cols.data_ptr(), out.data_ptr(),
                                             rows.numel(), self._stream_of(rows))
            check(rc, self.handle)
            if sync:
                self.sync(self._stream_of(rows))
            return out
        r = _host(rows, np.int64)
        c = _host(cols, np.int32)
        if r.shape != c.shape:
            raise ValueError("rows and cols differ in length")
        res = self._host_out(out, r.shape)
        check(self.lib.glint_mat_pull(self.handle, r.ctypes.data, c.ctypes.data, res.ctypes.data, r.size),
              self.handle)
        return res

    def getRows(self, rows, out=None, sync: bool = True):
        """PartialMatrix.getRows (PartialMatrix.scala:37-46) as one (n, cols) array -- the flattened
        row-major image ResponseSerializer sends (ResponseSerializer.scala:52-61)."""
        if _is_torch_cuda(rows):
            import torch
            if out is None:
                out = torch.empty((rows.numel(), self.cols), dtype=self.torch_dtype, device=rows.device)
            self._check_dev(rows.numel(), rows, out=out, out_elems=rows.numel() * self.cols)
            rc = self.lib.glint_mat_pull_rows_dev(self.handle, rows.data_ptr(), out.data_ptr(), rows.numel(),
                                                  self._stream_of(rows))
            check(rc, self.handle)
            if sync:
                self.sync(self._stream_of(rows))
            return out
        r = _host(rows, np.int64).reshape(-1)
        res = self._host_out(out, (r.size, self.cols))
        check(self.lib.glint_mat_pull_rows(self.handle, r.ctypes.data, res.ctypes.data, r.size), self.handle)
        return res

    def push_wire(self, payload: bytes, deterministic: bool = False) -> int:
        buf = (C.c_uint8 * len(payload)).from_buffer_copy(payload)
        mid = C.c_int32()
        flags = N.GLINT_PUSH_DETERMINISTIC if deterministic else N.GLINT_PUSH_DEFAULT
        check(self.lib.glint_push_wire(self.handle, buf, len(payload), C.byref(mid), flags), self.handle)
        return mid.value

    def pull_wire(self, payload: bytes) -> bytes:
        return _pull_wire(self, payload)

    def to_numpy(self) -> np.ndarray:
        p = self.partition
        if isinstance(p, RangePartition):
            rows = np.arange(p.start, p.start + self.size, dtype=np.int64)
        else:
            rows = np.arange(self.size, dtype=np.int64) * p.numberOfPartitions + p.index
        return self.getRows(rows)


def _pull_wire(shard: _Shard, payload: bytes) -> bytes:
    lib = shard.lib
    buf = (C.c_uint8 * len(payload)).from_buffer_copy(payload)
    need = C.c_size_t(0)
    rc = lib.glint_pull_wire(shard.handle, buf, len(payload), None, 0, C.byref(need))
    if rc != N.GLINT_OK and need.value == 0:
        check(rc, shard.handle)
    out = (C.c_uint8 * need.value)()
    check(lib.glint_pull_wire(shard.handle, buf, len(payload), out, need.value, C.byref(need)), shard.handle)
    return bytes(out)
