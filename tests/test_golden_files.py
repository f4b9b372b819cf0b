"""The reference's data files, end to end on the host: footer/page reader (product host code,
no GPU) + the CPU oracle, checked against pyarrow-generated golden vectors
(tests/golden/make_golden.py) and the reference's own file/triplet KATs.

GPU counterpart: tests/test_gpu_files.py (same files through the GPU column reader).
"""
import json
import os

import numpy as np
import pytest

import pqgpu

HERE = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(HERE, "golden", "data")
VEC = os.path.join(HERE, "golden", "vectors")

with open(os.path.join(VEC, "manifest.json")) as fh:
    MANIFEST = {m["file"]: m for m in json.load(fh)["files"]}


def golden(fname):
    return np.load(os.path.join(VEC, fname.replace(".parquet", ".npz")))


def cases():
    for f, m in sorted(MANIFEST.items()):
        for rg in range(len(m["row_groups"])):
            for j in range(len(m["columns"])):
                yield f, rg, j


class Spec:
    def __init__(self, blob, p):
        self.page_type, self.num_values, self.encoding = p.page_type, p.num_values, p.encoding
        self.def_encoding, self.rep_encoding = p.def_encoding, p.rep_encoding
        self.def_len, self.rep_len = p.def_len, p.rep_len
        self.buf = blob[p.offset:p.offset + p.nbytes]


def oracle_read(oracle, fr, rg, j, batch_size=1024):
    path, col = fr.column(j)
    blob, pages, n = fr.chunk_pages(rg, j)
    specs = [Spec(blob, pages[i]) for i in range(n)]
    return oracle.read_column(col.physical_type, [oracle.PageSpec(s.page_type, s.buf, s.num_values, s.encoding,
                                                                  s.def_encoding, s.rep_encoding, s.def_len, s.rep_len)
                                                  for s in specs],
                              col.max_def, col.max_rep, col.type_length, batch_size, True, True)


def expected_bytes(g, j, rg):
    return g[f"{j}_{rg}_val"].tobytes()


def test_schema_matches_manifest():
    for f, m in MANIFEST.items():
        fr = pqgpu.FileReader(os.path.join(DATA, f))
        assert fr.num_row_groups == len(m["row_groups"])
        assert fr.num_columns == len(m["columns"])
        for rg, nrows in enumerate(m["row_groups"]):
            assert fr.row_group_num_rows(rg) == nrows
        for j, c in enumerate(m["columns"]):
            path, col = fr.column(j)
            assert path == c["path"], (f, j)
            assert (col.physical_type, col.max_def, col.max_rep) == (c["physical_type"], c["max_def"], c["max_rep"])


@pytest.mark.parametrize("fname,rg,j", list(cases()))
def test_oracle_matches_golden(oracle, fname, rg, j):
    fr = pqgpu.FileReader(os.path.join(DATA, fname))
    g = golden(fname)
    c = MANIFEST[fname]["columns"][j]
    res = oracle_read(oracle, fr, rg, j)
    assert res["status"] == oracle.OK, res["message"]
    exp_def, exp_rep = g[f"{j}_{rg}_def"], g[f"{j}_{rg}_rep"]
    if c["max_def"] > 0:
        np.testing.assert_array_equal(res["def"], exp_def)
    if c["max_rep"] > 0:
        np.testing.assert_array_equal(res["rep"], exp_rep)
    if c["physical_type"] in (pqgpu.BYTE_ARRAY, pqgpu.FIXED_LEN_BYTE_ARRAY):
        lens = np.diff(np.asarray(res["offsets"], dtype=np.int64))
        np.testing.assert_array_equal(lens, g[f"{j}_{rg}_len"])
        got = res["bytes"]
    else:
        got = np.ascontiguousarray(res["values"]).tobytes()
    assert got == expected_bytes(g, j, rg)


# ---- reference KATs (file/reader.rs:699-800, record/triplet.rs:362-439), restated as data

def test_alltypes_plain_pages():
    fr = pqgpu.FileReader(os.path.join(DATA, "alltypes_plain.parquet"))
    assert fr.num_rows == 8 and fr.num_row_groups == 1 and fr.num_columns == 11
    blob, pages, n = fr.chunk_pages(0, 0)
    assert n == 2
    assert (pages[0].page_type, pages[0].nbytes, pages[0].num_values, pages[0].encoding) == \
        (pqgpu.PAGE_DICTIONARY, 32, 8, pqgpu.PLAIN_DICTIONARY)
    assert (pages[1].page_type, pages[1].nbytes, pages[1].num_values, pages[1].encoding,
            pages[1].def_encoding, pages[1].rep_encoding) == \
        (pqgpu.PAGE_DATA, 11, 8, pqgpu.PLAIN_DICTIONARY, pqgpu.RLE, pqgpu.BIT_PACKED)
    # every column's first page is readable (test_reuse_file_chunk)
    for j in range(11):
        assert fr.chunk_pages(0, j)[2] >= 1


def test_datapage_v2_pages():
    fr = pqgpu.FileReader(os.path.join(DATA, "test_datapage_v2.snappy.parquet"))
    assert fr.num_rows == 5
    blob, pages, n = fr.chunk_pages(0, 0)
    assert n == 2
    assert (pages[0].page_type, pages[0].nbytes, pages[0].num_values, pages[0].encoding) == \
        (pqgpu.PAGE_DICTIONARY, 7, 1, pqgpu.PLAIN)
    p = pages[1]
    assert (p.page_type, p.num_values, p.encoding, p.def_len, p.rep_len) == \
        (pqgpu.PAGE_DATA_V2, 5, pqgpu.RLE_DICTIONARY, 2, 0)
    assert p.nbytes == 4  # buf.len(): level bytes (kept uncompressed) + decompressed values


TRIPLET_KATS = [
    ("nulls.snappy.parquet", "b_struct.b_c_int", [], [1] * 8, [0] * 8),
    ("nonnullable.impala.parquet", "ID", [8], [0], [0]),
    ("nullable.impala.parquet", "nested_struct.A", [1, 7], [2, 1, 1, 1, 1, 0, 2], [0] * 7),
    ("nested_lists.snappy.parquet", "a.list.element.list.element.list.element",
     [b"a", b"b", b"c", b"d", b"a", b"b", b"c", b"d", b"e", b"a", b"b", b"c", b"d", b"e", b"f"],
     [7, 7, 7, 4, 7, 7, 7, 7, 7, 4, 7, 7, 7, 7, 7, 7, 4, 7],
     [0, 3, 2, 1, 2, 0, 3, 2, 3, 1, 2, 0, 3, 2, 3, 2, 1, 2]),
    ("nested_maps.snappy.parquet", "a.key_value.value.key_value.key", [1, 2, 1, 1, 3, 4, 5],
     [4, 4, 4, 2, 3, 4, 4, 4, 4], [0, 2, 0, 0, 0, 0, 0, 2, 2]),
]


def _col_index(fname, path):
    return [c["path"] for c in MANIFEST[fname]["columns"]].index(path)


@pytest.mark.parametrize("fname,path,values,defs,reps", TRIPLET_KATS)
def test_triplet_kats_pin_golden(fname, path, values, defs, reps):
    """The golden generator's record shredding agrees with the reference's triplet KATs."""
    j = _col_index(fname, path)
    g = golden(fname)
    np.testing.assert_array_equal(g[f"{j}_0_def"], defs)
    np.testing.assert_array_equal(g[f"{j}_0_rep"], reps)
    raw = g[f"{j}_0_val"].tobytes()
    if values and isinstance(values[0], bytes):
        assert raw == b"".join(values)
    elif values:
        w = 8 if MANIFEST[fname]["columns"][j]["physical_type"] == pqgpu.INT64 else 4
        assert raw == b"".join(int(v).to_bytes(w, "little", signed=True) for v in values)
    else:
        assert raw == b""


@pytest.mark.parametrize("fname,path,values,defs,reps", TRIPLET_KATS)
@pytest.mark.parametrize("batch", [1, 2, 3, 7, 10, 128])
def test_triplet_kats_oracle_batches(oracle, fname, path, values, defs, reps, batch):
    """Oracle read_batch loop at the reference's batch sizes (triplet.rs:450-456)."""
    fr = pqgpu.FileReader(os.path.join(DATA, fname))
    j = _col_index(fname, path)
    res = oracle_read(oracle, fr, 0, j, batch_size=batch)
    assert res["status"] == oracle.OK
    if MANIFEST[fname]["columns"][j]["max_def"] > 0:  # triplets report 0 for required leaves
        np.testing.assert_array_equal(res["def"], defs)
    if MANIFEST[fname]["columns"][j]["max_rep"] > 0:
        np.testing.assert_array_equal(res["rep"], reps)


def test_open_errors():
    with pytest.raises(pqgpu.PqgError):
        pqgpu.FileReader(os.path.join(DATA, "does-not-exist.parquet"))
    with pytest.raises(pqgpu.PqgError) as e:
        pqgpu.FileReader(data=b"PAR1")
    assert "smaller than footer" in str(e.value)
    with pytest.raises(pqgpu.PqgError) as e:
        pqgpu.FileReader(data=b"PAR1\0\0\0\0PAR2")
    assert "Corrupt footer" in str(e.value)
    with pytest.raises(pqgpu.PqgError) as e:
        pqgpu.FileReader(data=b"PAR1" + (100).to_bytes(4, "little") + b"PAR1")
    assert "Metadata start is less than zero" in str(e.value)


def test_truncated_chunk_is_an_error():
    data = open(os.path.join(DATA, "alltypes_plain.parquet"), "rb").read()
    fr = pqgpu.FileReader(data=data)
    blob, pages, n = fr.chunk_pages(0, 0)
    assert n == 2
    # chop the first data page out of the file but keep the footer: the page header now
    # points at garbage -> a thrift/EOF error from the page reader, never a crash
    bad = bytearray(data)
    for k in range(4, 200):
        bad[k] = 0xFF
    fr2 = pqgpu.FileReader(data=bytes(bad))
    with pytest.raises(pqgpu.PqgError):
        for j in range(fr2.num_columns):
            fr2.chunk_pages(0, j)


def test_malformed_dictionary_file(oracle):
    """nation.dict-malformed.parquet: the reader must report an error or decode, never crash."""
    fr = pqgpu.FileReader(os.path.join(DATA, "nation.dict-malformed.parquet"))
    for j in range(fr.num_columns):
        try:
            res = oracle_read(oracle, fr, 0, j)
        except pqgpu.PqgError:
            continue
        assert res["status"] in range(8)
