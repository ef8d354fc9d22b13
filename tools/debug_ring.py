"""Which side of a ring entry is wrong: pushes (async, direct or DMA) checked through a large,
non-ring element pull; direct row pulls and direct element pulls checked against it."""
import numpy as np

from glint_amd import PartialMatrix, RangePartition
from oracle import oracle as O

rng = np.random.default_rng(9)
rows_n, cols_n = 500, 129
for mode in ("sync", "async"):
    ref = O.OracleMatrix(O.part_range(0, rows_n), cols_n, O.O_F64)
    with PartialMatrix(RangePartition(0, 0, rows_n), cols_n, "double", 0) as sh:
        t = 0
        for n in (1000, 3000, 5000, 10):
            r = rng.integers(0, rows_n, n).astype(np.int64)
            c = rng.integers(0, cols_n, n).astype(np.int32)
            v = rng.uniform(-1, 1, n)
            if mode == "async":
                t = sh.push_async(r, c, v)
            else:
                sh.update(r, c, v)
            ref.update(r, c, v)
        if mode == "async":
            sh.wait(t)
        want = ref.data.reshape(rows_n, cols_n)
        rr = np.repeat(np.arange(rows_n, dtype=np.int64), cols_n)
        cc = np.tile(np.arange(cols_n, dtype=np.int32), rows_n)
        big = sh.get(rr, cc).reshape(rows_n, cols_n)          # 64500 elements: staged path
        print(mode, "element pull (staged) mismatches:", int((big != want).sum()))
        small = np.concatenate([sh.get(rr[i:i + 4000], cc[i:i + 4000]) for i in range(0, rr.size, 4000)])
        print(mode, "element pull (ring, 4000) mismatches:", int((small.reshape(rows_n, cols_n) != want).sum()))
        rows = sh.getRows(np.arange(rows_n, dtype=np.int64))
        print(mode, "row pull (ring) mismatches:", int((rows != want).sum()))
        rows2 = np.concatenate([sh.getRows(np.arange(i, min(rows_n, i + 50), dtype=np.int64)) for i in range(0, rows_n, 50)])
        print(mode, "row pull (ring, 50 rows) mismatches:", int((rows2 != want).sum()))
