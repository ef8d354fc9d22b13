"""CPU tests of the host side: the C-ABI library loads and exports every declared symbol, fails loudly
without a GPU, and the Python mirror of the partitioners / client bucketing agrees with the oracle."""
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

import glint_amd
from glint_amd import _native as N
from glint_amd.client import bucket
from glint_amd.errors import IndexOutOfBoundsException
from glint_amd.partitioning import CyclicPartitioner, RangePartitioner
from oracle import oracle as O

ROOT = Path(__file__).resolve().parent.parent


def header_symbols():
    text = (ROOT / "include" / "glint_gpu.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(glint_[a-z_]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    lib = N.load()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(N.SIGNATURES), "binding and header disagree"


def test_library_is_gfx950_only():
    """Every code object in the offload bundle targets gfx950 (the bundle ids are
    'hipv4-amdgcn-amd-amdhsa--<arch>'; rocPRIM's host-side arch-name tables are not code objects)."""
    data = N.LIB_PATH.read_bytes()
    targets = set(re.findall(rb"hipv4-amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", data))
    assert targets == {b"gfx950"}


def test_no_gpu_fails_loudly():
    lib = N.load()
    if lib.glint_device_count() > 0:
        pytest.skip("a GPU is visible")
    h = C.c_void_p()
    rc = lib.glint_shard_create(0, N.GLINT_F64, 0, 100, 0, C.byref(h))
    assert rc == N.GLINT_EDEVICE and not h.value
    with pytest.raises(glint_amd.GlintDeviceError):
        glint_amd.PartialVector(glint_amd.RangePartition(0, 0, 100))


def test_abi_argument_checks_without_gpu():
    lib = N.load()
    assert lib.glint_vec_push(None, None, None, 0, 0) == N.GLINT_EINVAL
    assert lib.glint_shard_destroy(None) == N.GLINT_EINVAL
    assert lib.glint_strerror(N.GLINT_EOUTOFRANGE).startswith(b"key outside")
    assert lib.glint_version() >= 100


@pytest.mark.parametrize("P,Nk", [(5, 109), (20, 50), (13, 13), (33, 12), (15, 97), (8, 1 << 31), (7, 1000003)])
def test_range_partitioner_matches_oracle(P, Nk):
    mine = RangePartitioner.apply(P, Nk)
    starts, ends, ns, q = O.range_partitioner(P, Nk)
    assert [p.start for p in mine.all()] == list(starts)
    assert [p.end for p in mine.all()] == list(ends)
    assert mine.numberOfSmallPartitions == ns and mine.smallPartitionSize == q
    rng = np.random.default_rng(P * 7 + Nk % 1000)
    keys = rng.integers(0, Nk, size=2000, dtype=np.int64)
    idx = mine.partition_indices(keys)
    for k, i in zip(keys[:200], idx[:200]):
        assert O.range_partition_of(int(k), ns, q, Nk) == i
        assert mine.partition(int(k)).index == i
        part = mine.all()[i]
        assert part.contains(int(k)) and 0 <= part.globalToLocal(int(k)) < part.size
    with pytest.raises(IndexOutOfBoundsException):
        mine.partition(Nk)
    with pytest.raises(IndexOutOfBoundsException):
        mine.partition(-2)
    with pytest.raises(IndexOutOfBoundsException):
        mine.partition_indices(np.array([0, Nk], np.int64))


@pytest.mark.parametrize("P,Nk", [(5, 37), (20, 50), (13, 13), (17, 137)])
def test_cyclic_partitioner_matches_oracle(P, Nk):
    mine = CyclicPartitioner.apply(P, Nk)
    for k in range(Nk):
        assert mine.partition(k).index == O.cyclic_partition_of(k, P, Nk)
    for p in mine.all():
        assert p.size == O.lib().oracle_cyclic_size(p.index, P, Nk)
    with pytest.raises(IndexOutOfBoundsException):
        mine.partition(Nk)
    with pytest.raises(IndexOutOfBoundsException):
        mine.partition(-2)


def test_client_bucketing_matches_reference_groupby():
    """AsyncBigVector.mapPartitions keeps each bucket in caller order (AsyncBigVector.scala:96-98)."""
    rng = np.random.default_rng(3)
    Nk, P = 10_000, 7
    keys = rng.integers(0, Nk, size=5000, dtype=np.int64)
    part = RangePartitioner.apply(P, Nk)
    order, off = bucket(part.partition_indices(keys), P)
    counts, ooff, oorder = O.bucket_range(keys, P, Nk)
    np.testing.assert_array_equal(off, ooff)
    np.testing.assert_array_equal(order, oorder)


def test_loopback_harness_cpu_backend():
    """configs[0] restated over loopback TCP (tools/loopback/glint_loopback.c) with the oracle's
    server loop: the exactly-once push protocol, ragged partitions and message sizes, and the
    GranularBigVectorSpec values (java.util.Random(42))."""
    import json
    import subprocess
    from glint_amd.build import LOOPBACK_BIN, ORACLE_LIB, build_loopback
    build_loopback()
    for servers, keys, msg in [(2, 100_000, 1000), (3, 10_007, 77), (5, 3, 1)]:
        r = subprocess.run([str(LOOPBACK_BIN), "--backend", "oracle", "--lib", str(ORACLE_LIB), "--servers",
                            str(servers), "--keys", str(keys), "--msg", str(msg)],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        d = json.loads(r.stdout)
        assert d["check"] is True and d["resends"] == 0
        assert d["push_messages"] >= -(-keys // msg)
        first = O.JavaRandom(42).nextDoubles(3)
        assert d["first_values"][:min(3, keys)] == list(first[:min(3, keys)])


def test_jni_shim_compiles_and_links():
    """integration/jni/glint_jni.c builds (-Wall -Werror) against the minimal JNI environment of
    tests/c/jni.h and links with libglint_gpu.so: every native method of GpuShard.scala exists."""
    import subprocess
    from glint_amd.build import JNI_DRIVER, build_jni_driver
    build_jni_driver()
    syms = subprocess.run(["nm", "-D", "--defined-only", str(JNI_DRIVER)], capture_output=True, text=True).stdout
    syms += subprocess.run(["nm", "--defined-only", str(JNI_DRIVER)], capture_output=True, text=True).stdout
    scala = (Path(__file__).resolve().parent.parent / "integration" / "scala" / "GpuShard.scala").read_text()
    import re
    natives = re.findall(r"@native def (\w+)", scala)
    assert len(natives) == 30  # lifetime 5, typed pushes 8, typed pulls 12, pipelined pulls 5
    for name in natives:
        assert f"Java_glint_models_server_gpu_GpuShard_{name}" in syms, name


@pytest.mark.parametrize("args", [
    ["--clients", "16", "--servers", "4", "--keys", "200003", "--msg", "777"],             # 4a: owned ranges
    ["--clients", "8", "--servers", "3", "--keys", "50000", "--pattern", "uniform", "--records", "20000",
     "--dtype", "long"],                                                                        # 4b: Long exact
    ["--clients", "8", "--servers", "3", "--keys", "50000", "--pattern", "uniform", "--records", "20000"],
    ["--clients", "2", "--servers", "2", "--keys", "30000", "--window", "1"],                  # one in flight
])
@pytest.mark.parametrize("server", ["threads", "actor"])
def test_loopback_concurrent_clients_cpu_backend(args, server):
    """configs[3]'s shape over loopback TCP with the oracle's server loop: many clients, each with up
    to W messages in flight per server (GranularBigVector issues every chunk at once), messages of
    different clients interleaving at the servers. `--server actor`: one thread per server takes the
    messages of every connection from a mailbox, as the Akka actor does."""
    import json
    import subprocess
    from glint_amd.build import LOOPBACK_BIN, ORACLE_LIB, build_loopback
    build_loopback()
    r = subprocess.run([str(LOOPBACK_BIN), "--backend", "oracle", "--lib", str(ORACLE_LIB), "--server", server] + args,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout)
    assert d["check"] is True and d["resends"] == 0 and d["server"] == server


@pytest.mark.parametrize("args", [[], ["--clients", "8", "--servers", "3", "--keys", "100003", "--pattern", "uniform",
                                       "--records", "20000", "--dtype", "long"]])
def test_loopback_harness_oracle_backend(args):
    """The loopback harness (tools/loopback/glint_loopback.c) with the oracle's CPU loop as the server
    backend: the message flow, PushLogic's exactly-once protocol and the harness's own checks run on
    the CPU (the GPU backend is exercised by the -m gpu tests)."""
    import json
    import subprocess
    from glint_amd.build import LOOPBACK_BIN, ORACLE_LIB
    r = subprocess.run([str(LOOPBACK_BIN), "--backend", "oracle", "--lib", str(ORACLE_LIB)] + args,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout)
    assert d["check"] is True and d["resends"] == 0 and d["replies"] == "inline"
