"""CPU side of the read_batch slice rules: the one-column test file writer (tests/_minifile.py) is
read back page for page by the host file reader and by pyarrow, and the oracle's read_batch with
the reference's slice lengths (column/reader.rs:170-205) and without def levels (SURVEY A.2,
:212-226, 247-250) behaves as the reference's loop does on hand-checked cases."""
import numpy as np
import pytest

import _minifile


def _page(oracle, lv, body, enc):
    return oracle.PageSpec(oracle.PAGE_DATA, oracle.level_encode(np.asarray(lv, np.int16), 1) + body, len(lv), enc)


def test_minifile_pages_read_back(oracle):
    import pqgpu
    rng = np.random.default_rng(0)
    pages = []
    for n in (10, 0, 300):
        lv = (rng.random(n) > 0.2).astype(np.int16)
        pages.append(_page(oracle, lv, np.arange(int(lv.sum()), dtype=np.int32).tobytes(), oracle.PLAIN))
    data = _minifile.one_column_file(oracle.INT32, pages)
    fr = pqgpu.FileReader(data=data)
    blob, arr, n = fr.chunk_pages(0, 0)
    assert n == 3 and [arr[i].num_values for i in range(3)] == [10, 0, 300]
    for i, p in enumerate(pages):
        assert bytes(blob[arr[i].offset:arr[i].offset + arr[i].nbytes]) == p.buf
    fr.close()
    pq = pytest.importorskip("pyarrow.parquet")
    import io
    t = pq.read_table(io.BytesIO(data))
    assert t.num_rows == 310
    ref = oracle.read_column(oracle.INT32, pages, max_def=1)
    got = np.asarray(t.column("c").drop_null(), dtype=np.int32)
    np.testing.assert_array_equal(got, ref["values"])


def test_oracle_slice_clamps():
    """Hand-checked: pages of 130 and 90 levels without nulls, batch 100, def slice 1000 (no rep
    slice): call 1 reads 100; call 2 reads the 30 left of page 1, then iter = min(100, 90,
    1000 - 30) = 90 of page 2: 120 levels; the def slice of 50 clamps every call to 50; a rep slice
    of 100 (given although max_rep = 0) clamps like the def slice."""
    import pyoracle as oracle
    lv1, lv2 = np.ones(130, np.int16), np.ones(90, np.int16)
    pages = [_page(oracle, lv1, np.zeros(130, np.int32).tobytes(), oracle.PLAIN),
             _page(oracle, lv2, np.zeros(90, np.int32).tobytes(), oracle.PLAIN)]
    r = oracle.read_column(oracle.INT32, pages, max_def=1, batch_size=100, def_cap=1000, values_cap=1000,
                           want_rep=False)
    assert r["status"] == 0 and r["counts"] == [(100, 100), (120, 120)]
    r = oracle.read_column(oracle.INT32, pages, max_def=1, batch_size=100, def_cap=50, values_cap=1000,
                           want_rep=False)
    assert r["counts"] == [(50, 50)] * 4 + [(20, 20)]
    r = oracle.read_column(oracle.INT32, pages, max_def=1, batch_size=100, def_cap=1000, values_cap=1000,
                           rep_cap=100)
    assert r["counts"] == [(100, 100), (100, 100), (20, 20)]


def test_oracle_no_def_levels():
    """A.2: 10 levels, 7 values, PLAIN INT32, def = None, batch 4: calls read 4 values, then 3 are
    left for the next 4 (num_values left 6 of the 10 set): EOF on the second call."""
    import pyoracle as oracle
    lv = np.array([1, 1, 0, 1, 0, 1, 1, 0, 1, 1], np.int16)
    p = _page(oracle, lv, np.arange(7, dtype=np.int32).tobytes(), oracle.PLAIN)
    r = oracle.read_column(oracle.INT32, [p], max_def=1, batch_size=4, want_def=False)
    assert r["status"] == oracle.EOF and r["counts"] == [(4, 0)]
    r = oracle.read_column(oracle.INT32, [p], max_def=1, batch_size=7, want_def=False)
    # call 1 reads all 7 values; call 2 asks min(7, 10 - 7) = 3 more of a used-up value section
    assert r["status"] == oracle.EOF and r["counts"] == [(7, 0)]
