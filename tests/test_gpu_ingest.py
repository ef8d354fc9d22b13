"""Pipelined host ingest (pinned ring slots, enqueue without waiting, ticketed waits): results equal
the sequential oracle over the pushes in enqueue order -- PartialVector.update per message, messages
applied one at a time as an actor does (PartialVectorDouble.scala:17-23) -- and a wait reports the
rejected records of the pushes it covers (PushLogic.scala:40-66 acknowledges only applied pushes)."""
import zlib

import numpy as np
import pytest

from glint_amd import ArrayIndexOutOfBoundsException, PartialMatrix, PartialVector, RangePartition
from glint_amd import _native as N
from oracle import oracle as O

pytestmark = pytest.mark.gpu
DT = ["double", "float", "long", "int"]


def _vals(rng, dtype, n):
    npd = {"double": np.float64, "float": np.float32, "long": np.int64, "int": np.int32}[dtype]
    if np.issubdtype(npd, np.floating):
        return (rng.uniform(-1, 1, n) * 10.0 ** rng.integers(-6, 6, n)).astype(npd)
    return rng.integers(-1000, 1000, n).astype(npd)


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("sizes", [[1000] * 37, [1, 4096, 4097, 79_999, 12, 3000]])
def test_async_pushes_equal_sequential_oracle(gpu, dtype, sizes):
    """More pushes in flight than ring slots; small ones read in place, large ones copied."""
    rng = np.random.default_rng(zlib.crc32(f"ring/{dtype}/{len(sizes)}".encode()))
    start, size = 1 << 34, 60_000
    ref = O.OracleVector(O.part_range(start, start + size), O.CODE[dtype])
    with PartialVector(RangePartition(0, start, start + size), dtype, gpu) as sh:
        tickets = []
        for n in sizes:
            keys = (np.minimum(rng.zipf(1.3, n) - 1, size - 1) + start).astype(np.int64)
            vals = _vals(rng, dtype, n)
            tickets.append(sh.push_async(keys, vals))
            assert ref.update(keys, vals) == -1
        assert tickets == sorted(tickets) and len(set(tickets)) == len(tickets)
        sh.wait(tickets[-1])
        np.testing.assert_array_equal(sh.to_numpy(), ref.data)


def test_wire_async_and_pull_ordering(gpu):
    """Wire images enqueued without waiting; a pull issued before any wait sees every push."""
    rng = np.random.default_rng(5)
    size = 20_000
    ref = O.OracleVector(O.part_range(0, size), O.O_F64)
    with PartialVector(RangePartition(0, 0, size), "double", gpu) as sh:
        last = 0
        for mid in range(50):
            keys = rng.integers(0, size, 1000).astype(np.int64)
            vals = rng.uniform(-1, 1, 1000)
            got_id, last = sh.push_wire_async(O.encode_push_vector(O.O_F64, mid + 100, keys, vals))
            assert got_id == mid + 100
            ref.update(keys, vals)
        q = np.arange(size, dtype=np.int64)
        np.testing.assert_array_equal(sh.get(q), ref.data)  # ordered after the enqueued pushes
        sh.wait(last)


def test_large_wire_async_push_applied_at_once(gpu):
    """A wire push of more than 4 MiB of records (far above the 79 999 frame cap) is applied through
    the synchronous path before glint_push_wire_async returns: it lands between the enqueued messages
    around it in order, its ticket covers everything before it, and a bad key in it applies nothing."""
    rng = np.random.default_rng(17)
    size = 1 << 20
    ref = O.OracleVector(O.part_range(0, size), O.O_F64)
    with PartialVector(RangePartition(0, 0, size), "double", gpu) as sh:
        msgs = [(rng.integers(0, size, n).astype(np.int64), rng.uniform(-1, 1, n)) for n in (1000, 300_000, 1000)]
        ts = []
        for i, (k, v) in enumerate(msgs):
            _, t = sh.push_wire_async(O.encode_push_vector(O.O_F64, i, k, v))
            ts.append(t)
            ref.update(k, v)
        assert ts[0] == ts[1] < ts[2]  # the large push's ticket: everything enqueued before it
        bad_k = msgs[1][0].copy()
        bad_k[123_456] = size
        with pytest.raises(ArrayIndexOutOfBoundsException) as ei:
            sh.push_wire_async(O.encode_push_vector(O.O_F64, 9, bad_k, msgs[1][1]))
        assert ei.value.record == 123_456
        sh.wait(ts[2])
        # above 131 072 records a Double push is not folded in message order: repeated
        # keys of the large message may differ from the JVM loop in the last bit
        np.testing.assert_allclose(sh.to_numpy(), ref.data, rtol=1e-12, atol=0)


@pytest.mark.parametrize("dtype", ["double", "int"])
def test_async_matrix_pushes(gpu, dtype):
    rng = np.random.default_rng(9)
    rows_n, cols_n = 500, 129
    ref = O.OracleMatrix(O.part_range(0, rows_n), cols_n, O.CODE[dtype])
    with PartialMatrix(RangePartition(0, 0, rows_n), cols_n, dtype, gpu) as sh:
        t = 0
        for n in (1000, 3000, 5000, 10):
            r = rng.integers(0, rows_n, n).astype(np.int64)
            c = rng.integers(0, cols_n, n).astype(np.int32)
            v = _vals(rng, dtype, n)
            t = sh.push_async(r, c, v)
            ref.update(r, c, v)
        sh.wait(t)
        np.testing.assert_array_equal(sh.to_numpy(), ref.data)


def test_async_push_error_belongs_to_its_message(gpu):
    """A rejected record raises at the Push message itself (PartialVectorDouble.scala:17-23: update
    throws inside receive), with nothing of that message applied; the pushes around it, later waits
    and a pull are clean -- no earlier push's error surfaces at another call."""
    size = 1000
    with PartialVector(RangePartition(0, 0, size), "long", gpu) as sh:
        t1 = sh.push_async(np.array([1, 2], np.int64), np.array([1, 1], np.int64))
        with pytest.raises(ArrayIndexOutOfBoundsException) as ei:
            sh.push_async(np.array([3, size + 9, 4], np.int64), np.array([1, 1, 1], np.int64))
        assert ei.value.record == 1
        t3 = sh.push_async(np.array([5], np.int64), np.array([1], np.int64))
        assert sh.get(np.array([1, 5], np.int64)).tolist() == [1, 1]  # a clean pull after the bad push
        with pytest.raises(ArrayIndexOutOfBoundsException) as ei:  # a second bad message: its own error
            sh.push_async(np.array([size], np.int64), np.array([1], np.int64))
        assert ei.value.record == 0
        sh.wait(t1)
        sh.wait(t3)
        t4 = sh.push_async(np.array([6], np.int64), np.array([1], np.int64))
        sh.wait(t4)
        got = sh.get(np.arange(8, dtype=np.int64))
        assert got.tolist() == [0, 1, 1, 0, 0, 1, 1, 0]
        assert t1 < t3 < t4


def test_stage_acquire_rejects_bad_arguments(gpu):
    import ctypes as C
    lib = N.load()
    with PartialVector(RangePartition(0, 0, 10), "double", gpu) as sh:
        kp, cp, vp, slot = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_int()
        assert lib.glint_stage_acquire(sh.handle, (1 << 20) + 1, C.byref(kp), C.byref(cp), C.byref(vp),
                                       C.byref(slot)) == N.GLINT_EINVAL
        assert lib.glint_push_staged(sh.handle, 99, 1, 0, None) == N.GLINT_EINVAL
        assert lib.glint_stage_acquire(sh.handle, 5, C.byref(kp), C.byref(cp), C.byref(vp), C.byref(slot)) == 0
        assert cp.value is None  # no cols section for a vector shard
        assert lib.glint_push_staged(sh.handle, slot.value, 6, 0, None) == N.GLINT_EINVAL  # more than staged
        assert lib.glint_push_staged(sh.handle, slot.value, 0, 0, None) == 0


def test_jni_shim_end_to_end(gpu):
    """The shim's native methods, called in the actors' order through a minimal JNI environment
    (tests/c/fake_jvm.c): push -> await -> pull, sequential Double order, restart after an
    out-of-partition key, argument errors, matrix element and row pulls."""
    import subprocess
    from glint_amd.build import build_jni_driver
    r = subprocess.run([str(build_jni_driver()), str(gpu)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr


@pytest.mark.parametrize("dtype", DT)
def test_async_pulls_interleaved_with_pushes(gpu, dtype):
    """Pulls enqueued between pushes see exactly the pushes enqueued before them (the actor's
    mailbox order); small pulls run in place in the mapped slot, large ones through DMA; more
    entries in flight than ring slots."""
    rng = np.random.default_rng(zlib.crc32(f"pull-async/{dtype}".encode()))
    size = 50_000
    ref = O.OracleVector(O.part_range(0, size), O.CODE[dtype])
    with PartialVector(RangePartition(0, 0, size), dtype, gpu) as sh:
        want, got = [], []
        t = 0
        for step, n in enumerate([1000, 1, 4096, 4097, 30_000, 777] * 4):
            keys = rng.integers(0, size, n).astype(np.int64)
            if step % 2 == 0:
                vals = _vals(rng, dtype, n)
                t = sh.push_async(keys, vals)
                ref.update(keys, vals)
            else:
                t, out = sh.pull_async(keys)
                got.append(out)
                want.append(ref.data[keys].copy())
        sh.wait(t)
        for w, g in zip(want, got):
            np.testing.assert_array_equal(g, w)


@pytest.mark.parametrize("dtype", ["double", "int"])
def test_async_matrix_pulls(gpu, dtype):
    rng = np.random.default_rng(21)
    rows_n, cols_n = 300, 65
    ref = O.OracleMatrix(O.part_range(0, rows_n), cols_n, O.CODE[dtype])
    with PartialMatrix(RangePartition(0, 0, rows_n), cols_n, dtype, gpu) as sh:
        r = rng.integers(0, rows_n, 5000).astype(np.int64)
        c = rng.integers(0, cols_n, 5000).astype(np.int32)
        v = _vals(rng, dtype, 5000)
        sh.push_async(r, c, v)
        ref.update(r, c, v)
        qr = rng.integers(0, rows_n, 999).astype(np.int64)
        qc = rng.integers(0, cols_n, 999).astype(np.int32)
        t1, elems = sh.pull_async(qr, qc)
        t2, rows_small = sh.pull_async(qr[:200], rows=True)     # 200 x 65 values: in place
        t3, rows_big = sh.pull_async(qr, rows=True)            # 999 x 65 values
        sh.wait(t3)
        assert t1 < t2 < t3
        np.testing.assert_array_equal(elems, ref.data.reshape(rows_n, cols_n)[qr, qc])
        np.testing.assert_array_equal(rows_small, ref.data.reshape(rows_n, cols_n)[qr[:200]])
        np.testing.assert_array_equal(rows_big, ref.data.reshape(rows_n, cols_n)[qr])


@pytest.mark.parametrize("n", [4095, 4096, 4097])
def test_async_matrix_element_pulls_at_the_ring_bound(gpu, n):
    """Element pulls of up to 4096 records run as one 1024-thread signalling kernel reading the
    mapped slot; 4097 goes through DMA. Both answer like the oracle, and a bad column is reported
    as its record index."""
    rng = np.random.default_rng(n)
    rows_n, cols_n = 700, 33
    ref = O.OracleMatrix(O.part_range(0, rows_n), cols_n, O.CODE["double"])
    with PartialMatrix(RangePartition(0, 0, rows_n), cols_n, "double", gpu) as sh:
        r = rng.integers(0, rows_n, 20_000).astype(np.int64)
        c = rng.integers(0, cols_n, 20_000).astype(np.int32)
        v = _vals(rng, "double", 20_000)
        sh.push_async(r, c, v)
        ref.update(r, c, v)
        qr = rng.integers(0, rows_n, n).astype(np.int64)
        qc = rng.integers(0, cols_n, n).astype(np.int32)
        t, elems = sh.pull_async(qr, qc)
        sh.wait(t)
        np.testing.assert_array_equal(elems, ref.data.reshape(rows_n, cols_n)[qr, qc])
        qc[n - 2] = cols_n  # out of range: the JVM throws at record n - 2, at the Pull message
        with pytest.raises(ArrayIndexOutOfBoundsException) as ei:
            sh.pull_async(qr, qc)
        assert ei.value.record == n - 2


def test_async_pull_bad_key_and_wire(gpu):
    size = 1000
    with PartialVector(RangePartition(0, 0, size), "double", gpu) as sh:
        sh.update(np.arange(size, dtype=np.int64), np.arange(size, dtype=np.float64))
        with pytest.raises(ArrayIndexOutOfBoundsException) as ei:
            sh.pull_async(np.array([5, size + 3, 7], np.int64))
        assert ei.value.record == 1
        # the wire form: header at once, values after the wait
        import ctypes as C
        keys = np.array([9, 1, 9], np.int64)
        req = O.encode_pull_vector(keys)
        buf = (C.c_uint8 * len(req)).from_buffer_copy(req)
        resp = (C.c_uint8 * 64)()
        olen, ticket = C.c_size_t(), C.c_uint64()
        assert sh.lib.glint_pull_wire_async(sh.handle, buf, len(req), resp, 64, C.byref(olen), C.byref(ticket)) == 0
        assert olen.value == 5 + 24
        sh.wait(ticket.value)
        assert np.frombuffer(bytes(resp)[5:29], np.float64).tolist() == [9.0, 1.0, 9.0]
        t0, empty = sh.pull_async(np.zeros(0, np.int64))
        sh.wait(t0)
        assert empty.size == 0


def test_coalesced_batch_attributes_errors_to_their_message(gpu):
    """Message-sized pushes are coalesced into one launch; a rejected record is reported as record i
    of ITS message, by the call that enqueues that message, and the message is not applied."""
    size = 5000
    rng = np.random.default_rng(77)
    ref = O.OracleVector(O.part_range(0, size), O.O_F64)
    with PartialVector(RangePartition(0, 0, size), "double", gpu) as sh:
        tickets = []
        for m in range(6):
            keys = rng.integers(0, size, 300).astype(np.int64)
            vals = rng.uniform(-1, 1, 300)
            if m in (3, 4):
                keys[7 + m] = size + 1  # out of the partition: record 10 of message 3, 11 of message 4
                with pytest.raises(ArrayIndexOutOfBoundsException) as ei:
                    sh.push_async(keys, vals)
                assert ei.value.record == 7 + m
                continue
            ref.update(keys, vals)
            tickets.append(sh.push_async(keys, vals))
        sh.wait(tickets[2])  # messages 0..2
        sh.wait(tickets[-1])
        np.testing.assert_array_equal(sh.to_numpy(), ref.data)


def test_coalescing_keeps_order_across_flags_pulls_and_device_calls(gpu):
    """Batches break on a flag change, a pull or a device-resident call; every call still sees the
    pushes enqueued before it, and the Double sums keep the message order bit for bit."""
    import torch
    size = 3000
    rng = np.random.default_rng(78)
    ref = O.OracleVector(O.part_range(0, size), O.O_F64)
    dev = torch.device("cuda", gpu)
    with PartialVector(RangePartition(0, 0, size), "double", gpu) as sh:
        want, got = [], []
        for step in range(40):
            keys = np.minimum(rng.zipf(1.5, 200) - 1, size - 1).astype(np.int64)
            vals = rng.uniform(-1, 1, 200) * 10.0 ** rng.integers(-8, 8, 200)
            if step % 10 == 9:  # a device-resident push on the caller's stream, no sync
                sh.update(torch.from_numpy(keys).to(dev), torch.from_numpy(vals).to(dev), sync=False,
                          deterministic=True)
                ref.update(keys, vals)
            elif step % 7 == 6:
                t, out = sh.pull_async(keys)
                got.append(out)
                want.append(ref.data[keys].copy())
            else:  # DETERMINISTIC on every 5th: another flags value, so the batch breaks there
                sh.push_async(keys, vals, deterministic=(step % 5 == 4))
                ref.update(keys, vals)
        sh.sync()
        t, final = sh.pull_async(np.arange(size, dtype=np.int64))
        sh.wait(t)
        np.testing.assert_array_equal(final, ref.data)
        for w, g in zip(want, got):
            np.testing.assert_array_equal(g, w)


@pytest.mark.parametrize("dtype", ["double", "int"])
def test_coalesced_pulls_answer_each_message(gpu, dtype):
    """Consecutive message-sized pulls share one launch; every message gets its own answer, and a
    bad key is reported as record i of its own message."""
    size = 20_000
    rng = np.random.default_rng(91)
    with PartialVector(RangePartition(0, 0, size), dtype, gpu) as sh:
        base = _vals(rng, dtype, size)
        sh.update(np.arange(size, dtype=np.int64), base)
        outs, want, tickets = [], [], []
        for m in range(40):
            n = int(rng.integers(1, 300))
            q = rng.integers(0, size, n).astype(np.int64)
            t, out = sh.pull_async(q)
            outs.append(out)
            want.append(base[q])
            tickets.append(t)
        sh.wait(tickets[-1])
        for w, g in zip(want, outs):
            np.testing.assert_array_equal(g, w)
        q1 = np.array([1, 2, 3], np.int64)
        q2 = np.array([4, size + 2, 6, 7], np.int64)
        t1, o1 = sh.pull_async(q1)
        with pytest.raises(ArrayIndexOutOfBoundsException) as ei:
            sh.pull_async(q2)
        assert ei.value.record == 1
        sh.wait(t1)  # the first message is answered
        np.testing.assert_array_equal(o1, base[q1])


def test_host_free_refuses_a_buffer_with_pending_pulls(gpu):
    """glint_host_free of a buffer that an enqueued, not yet retired pull answers into would let the
    kernel write into freed pinned memory: it returns GLINT_EINVAL and frees nothing; once the pull's
    ticket has been waited for, the buffer frees normally."""
    from glint_amd.shard import HostBuffer
    lib = N.load()
    size = 10_000
    with PartialVector(RangePartition(0, 0, size), "double", gpu) as sh:
        base = np.arange(size, dtype=np.float64) * 0.5
        sh.update(np.arange(size, dtype=np.int64), base)
        hb = HostBuffer(1 << 16)
        q = np.arange(0, 2 * 1024, 2, dtype=np.int64)  # 1024 doubles: a page of answer, in place
        t, got = sh.pull_async(q, out=hb.array(np.float64, q.size))
        assert lib.glint_host_free(hb.ptr) == N.GLINT_EINVAL
        sh.wait(t)
        np.testing.assert_array_equal(got, base[q])
        assert lib.glint_host_free(hb.ptr) == N.GLINT_OK
        hb.ptr = None


@pytest.mark.parametrize("dtype", ["double", "int"])
@pytest.mark.parametrize("min_bytes", ["0", None])
def test_pulls_answer_straight_into_host_buffers(gpu, dtype, min_bytes, monkeypatch):
    """Answers whose destination is glint_host_alloc memory (HostBuffer) are written by the kernel
    itself through the batch's destination table; in the same batch, messages answering into ordinary
    memory, at a misaligned address or below GLINT_DIRECT_MIN_BYTES (default one page; "0": every
    message in place) still get theirs through the slot; a batch of more messages than the table holds
    (kPullDirectMax) falls back to the copies; matrix element pulls likewise."""
    from glint_amd.shard import HostBuffer
    if min_bytes is not None:
        monkeypatch.setenv("GLINT_DIRECT_MIN_BYTES", min_bytes)
    N.reload_env()
    size = 20_000
    rng = np.random.default_rng(93)
    npd = np.dtype(np.float64 if dtype == "double" else np.int32)
    with PartialVector(RangePartition(0, 0, size), dtype, gpu) as sh, HostBuffer(1 << 22) as hb:
        base = _vals(rng, dtype, size)
        sh.update(np.arange(size, dtype=np.int64), base)
        for rnd in range(3):
            outs, want, tickets, off = [], [], [], 0
            for m in range(60):
                n = int(rng.integers(1, 400 if min_bytes == "0" else 1500))
                q = rng.integers(0, size, n).astype(np.int64)
                kind = m % 4
                if kind == 3:  # ordinary numpy memory: through the slot
                    out = np.empty(n, npd)
                else:
                    off = (off + 7) // 8 * 8
                    if kind == 2 and npd.itemsize == 8:
                        off += 4  # misaligned for 8-B values: through the slot
                    out = hb.array(npd, n, off)
                    off += n * npd.itemsize
                t, got = sh.pull_async(q, out=out)
                outs.append(got)
                want.append(base[q])
                tickets.append(t)
            sh.wait(tickets[-1])
            for w, g in zip(want, outs):
                np.testing.assert_array_equal(g, w)
        # more one-record messages in one batch than the destination table holds
        outs, want = [], []
        for m in range(300):
            q = np.array([m * 7 % size], np.int64)
            t, got = sh.pull_async(q, out=hb.array(npd, 1, 8 * m))
            outs.append(got)
            want.append(base[q])
        sh.wait(t)
        for w, g in zip(want, outs):
            np.testing.assert_array_equal(g, w)
    with PartialMatrix(RangePartition(0, 0, 300), 37, dtype, gpu) as mt, HostBuffer(1 << 20) as hb:
        full = _vals(rng, dtype, 300 * 37).reshape(300, 37)
        r = np.repeat(np.arange(300, dtype=np.int64), 37)
        c = np.tile(np.arange(37, dtype=np.int32), 300)
        mt.update(r, c, full.reshape(-1))
        outs, want, off = [], [], 0
        for m in range(20):
            n = int(rng.integers(1, 500))
            qr = rng.integers(0, 300, n).astype(np.int64)
            qc = rng.integers(0, 37, n).astype(np.int32)
            t, got = mt.pull_async(qr, qc, out=hb.array(npd, n, off))
            off += (n * npd.itemsize + 7) // 8 * 8
            outs.append(got)
            want.append(full[qr, qc])
        mt.wait(t)
        for w, g in zip(want, outs):
            np.testing.assert_array_equal(g, w)


def test_wide_row_pull_answers_bypass_the_ring(gpu):
    """A row pull of a few rows of a very wide matrix (an answer > 16 MiB) is produced through the
    staged copies -- synchronous and async alike -- instead of growing a pinned ring slot to the
    answer's size; the answers are the rows."""
    rows_n, cols_n = 64, 100_000
    rng = np.random.default_rng(5)
    with PartialMatrix(RangePartition(0, 0, rows_n), cols_n, "double", gpu) as sh:
        r = np.repeat(np.arange(rows_n, dtype=np.int64), 50)
        c = rng.integers(0, cols_n, r.size).astype(np.int32)
        v = rng.uniform(-1, 1, r.size)
        sh.update(r, c, v)
        full = sh.to_numpy().reshape(rows_n, cols_n)
        q = rng.integers(0, rows_n, 40).astype(np.int64)  # 40 x 800 KB = 32 MB of answer
        np.testing.assert_array_equal(sh.getRows(q), full[q])
        t, out = sh.pull_async(q, rows=True)
        sh.wait(t)
        np.testing.assert_array_equal(out, full[q])


def test_shards_sync_reports_each_shard(gpu):
    """glint_shards_sync: the syncs of several shards, each on its own stream, in one call (the
    exchange layer's local pushes): each shard's result is what its own glint_shard_sync reports --
    the rejected record of the one bad push, nothing for the others -- the error state is cleared,
    and a repeated shard is refused before anything is waited for."""
    import ctypes as C
    import torch
    lib = N.load()
    d = torch.device("cuda", gpu)
    shards = [PartialVector(RangePartition(i, i * 1000, (i + 1) * 1000), "long", gpu) for i in range(3)]
    streams = [torch.cuda.Stream(d) for _ in shards]
    try:
        for i, (sh, st) in enumerate(zip(shards, streams)):
            k = torch.arange(i * 1000, (i + 1) * 1000, dtype=torch.int64, device=d)
            if i == 1:
                k[17] = 5  # shard 0's key: outside shard 1
            with torch.cuda.stream(st):
                sh.update(k, torch.ones(1000, dtype=torch.int64, device=d), sync=False)
        n = len(shards)
        hs = (C.c_void_p * n)(*[sh.handle for sh in shards])
        ss = (C.c_void_p * n)(*[st.cuda_stream for st in streams])
        rcs, bad = (C.c_int * n)(), (C.c_int64 * n)(*([-1] * n))
        assert lib.glint_shards_sync(hs, ss, n, rcs, bad) == N.GLINT_EOUTOFRANGE
        assert list(rcs) == [0, N.GLINT_EOUTOFRANGE, 0] and bad[1] == 17 and bad[0] == -1
        assert lib.glint_shards_sync(hs, ss, n, rcs, bad) == 0 and list(rcs) == [0, 0, 0]  # cleared
        want = np.ones(1000, np.int64)
        np.testing.assert_array_equal(shards[0].to_numpy(), want)
        np.testing.assert_array_equal(shards[2].to_numpy(), want)
        got1 = shards[1].to_numpy()  # in-range records applied, as the reference's loop did before it threw
        assert got1[17] == 0 and got1.sum() == 999
        dup = (C.c_void_p * 2)(shards[0].handle, shards[0].handle)
        assert lib.glint_shards_sync(dup, (C.c_void_p * 2)(ss[0], ss[1]), 2, (C.c_int * 2)(), None) == N.GLINT_EINVAL
    finally:
        for sh in shards:
            sh.destroy()
