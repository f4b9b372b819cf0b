"""The reference's data files through the GPU column reader (pqg_column_reader_*), checked
against the pyarrow golden vectors and the reference's triplet KATs at its batch sizes."""
import os

import numpy as np
import pytest

from test_golden_files import DATA, MANIFEST, TRIPLET_KATS, _col_index, cases, golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    import pqgpu
    c = pqgpu.Context(0)
    yield c
    c.close()


def read_all(cr, batch):
    vals, defs, reps = [], [], []
    while True:
        v, d, r, nv, nl = cr.read_batch(batch)
        if nv == 0 and nl == 0:
            break
        vals.append(v)
        if d is not None:
            defs.append(d)
        if r is not None:
            reps.append(r)
    return vals, defs, reps


def _flat_bytes(vals, ptype):
    import pqgpu
    if ptype in (pqgpu.BYTE_ARRAY, pqgpu.FIXED_LEN_BYTE_ARRAY):
        items = [x for v in vals for x in v]
        return b"".join(items), np.array([len(x) for x in items], np.uint32)
    return b"".join(np.ascontiguousarray(v).tobytes() for v in vals), None


@pytest.mark.parametrize("fname,rg,j", list(cases()))
def test_gpu_column_reader_matches_golden(ctx, fname, rg, j):
    import pqgpu
    fr = pqgpu.FileReader(os.path.join(DATA, fname))
    c = MANIFEST[fname]["columns"][j]
    g = golden(fname)
    cr = fr.column_reader(rg, j, ctx)
    vals, defs, reps = read_all(cr, 1024)
    if c["max_def"] > 0:
        np.testing.assert_array_equal(np.concatenate(defs) if defs else np.zeros(0, np.int16), g[f"{j}_{rg}_def"])
    if c["max_rep"] > 0:
        np.testing.assert_array_equal(np.concatenate(reps) if reps else np.zeros(0, np.int16), g[f"{j}_{rg}_rep"])
    raw, lens = _flat_bytes(vals, c["physical_type"])
    if lens is not None:
        np.testing.assert_array_equal(lens, g[f"{j}_{rg}_len"])
    assert raw == g[f"{j}_{rg}_val"].tobytes()


@pytest.mark.parametrize("fname,path,values,defs,reps", TRIPLET_KATS)
@pytest.mark.parametrize("batch", [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 128, 256])
def test_gpu_triplet_kats(ctx, fname, path, values, defs, reps, batch):
    """triplet.rs:442-456: the same levels at every batch size the reference tries."""
    import pqgpu
    fr = pqgpu.FileReader(os.path.join(DATA, fname))
    j = _col_index(fname, path)
    c = MANIFEST[fname]["columns"][j]
    cr = fr.column_reader(0, j, ctx)
    vals, d, r = read_all(cr, batch)
    if c["max_def"] > 0:
        np.testing.assert_array_equal(np.concatenate(d), defs)
        for k in range(len(d) - 1):
            assert len(d[k]) == batch  # every call but the last returns exactly batch levels
    if c["max_rep"] > 0:
        np.testing.assert_array_equal(np.concatenate(r), reps)
    raw, _ = _flat_bytes(vals, c["physical_type"])
    if values and isinstance(values[0], bytes):
        assert raw == b"".join(values)
    elif values:
        w = 8 if c["physical_type"] == pqgpu.INT64 else 4
        assert raw == b"".join(int(v).to_bytes(w, "little", signed=True) for v in values)


def test_gpu_malformed_dictionary_file(ctx):
    """nation.dict-malformed.parquet must surface a status, never crash the device."""
    import pqgpu
    fr = pqgpu.FileReader(os.path.join(DATA, "nation.dict-malformed.parquet"))
    for j in range(fr.num_columns):
        try:
            cr = fr.column_reader(0, j, ctx)
            read_all(cr, 7)
        except pqgpu.PqgError as e:
            assert 1 <= e.status <= 7


@pytest.mark.parametrize("fname,path,values,defs,reps", TRIPLET_KATS)
@pytest.mark.parametrize("batch", [1, 2, 3, 5, 7, 10, 128, 256])
def test_gpu_triplet_iter_kats(ctx, fname, path, values, defs, reps, batch):
    """TypedTripletIter over the GPU-decoded chunk (record/triplet.rs:270-318, tests :442-456):
    the triplet sequence is the KAT's levels, values sit on the max_def slots, and reading a
    value on a null slot is refused as the reference asserts."""
    import pqgpu
    fr = pqgpu.FileReader(os.path.join(DATA, fname))
    j = _col_index(fname, path)
    c = MANIFEST[fname]["columns"][j]
    cr = fr.column_reader(0, j, ctx)
    it = pqgpu.TripletIter(cr, batch)
    got_d, got_r, got_v = [], [], []
    while it.read_next():
        d, r = it.current_def_level(), it.current_rep_level()
        got_d.append(d)
        got_r.append(r)
        if d == c["max_def"]:
            v = it.current_value()
            got_v.append(v if isinstance(v, bytes) else int(v))
        else:
            assert it.is_null()
            with pytest.raises(pqgpu.PqgError):
                it.current_value()
    assert not it.has_next()
    if c["max_def"] > 0:
        assert got_d == list(defs)
    if c["max_rep"] > 0:
        assert got_r == list(reps)
    if values:
        assert got_v == [v if isinstance(v, bytes) else int(v) for v in values]
    it.close()
    cr.close()
