"""read_batch through the C ABI column reader (pqg_column_reader_read_batch_caps over a chunk
decoded on the GPU) against the oracle's ColumnReaderImpl::read_batch (column/reader.rs:159-265)
call by call: the (values_read, levels_read) of every call, the levels and values, and the status
and call at which a read fails.

Covers the reference's slice rules (the batch clamped to def_levels.len() / rep_levels.len() /
values.len(), every page iteration clamped again, :170-205: a def slice shorter than the batch, and
one longer, where a call crossing a page returns more levels than batch_size), read_batch without
def levels on an OPTIONAL column (:212-226, 247-250: iter_batch_size values per page
iteration from the value decoder, out of step with the levels, with the value decoder's own end:
PLAIN EOF, PLAIN BYTE_ARRAY panic, DELTA short reads then no progress), and an empty data page
(has_next returns false on it, :416-430, so the call ends short)."""
import numpy as np
import pytest

import _minifile

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    import pqgpu
    c = pqgpu.Context(0)
    yield c
    c.close()


def _page(oracle, rng, n, p_null, body_of, encoding):
    lv = (rng.random(n) >= p_null).astype(np.int16)
    nn = int(lv.sum())
    return oracle.PageSpec(oracle.PAGE_DATA, oracle.level_encode(lv, 1) + body_of(nn), n, encoding)


def _gpu_calls(ctx, ptype, pages, batch, want_def, def_cap=None, values_cap=None, optional=True,
               type_length=-1, max_calls=100000):
    """Every read_batch call of a GPU column reader over a one-column file of `pages`: the list
    of (values, def, values_read, levels_read) and the status that ended the reads (0 at the end)."""
    import pqgpu
    fr = pqgpu.FileReader(data=_minifile.one_column_file(ptype, pages, optional=optional,
                                                         type_length=type_length))
    cr = pqgpu.ColumnReader(fr, 0, 0, ctx)
    calls, st = [], 0
    try:
        for _ in range(max_calls):
            try:
                v, d, _, nv, nl = cr.read_batch(batch, want_def=want_def, want_rep=False, def_cap=def_cap,
                                                values_cap=values_cap)
            except pqgpu.PqgError as e:
                st = e.status
                break
            if nv == 0 and nl == 0:
                break
            calls.append((v, d, nv, nl))
    finally:
        cr.close()
        fr.close()
    return calls, st


def _check(oracle, ctx, ptype, pages, batch, want_def, def_cap=None, values_cap=None, optional=True,
           type_length=-1, expect_status=None):
    ref = oracle.read_column(ptype, pages, max_def=1 if optional else 0, type_length=type_length,
                             batch_size=batch, want_def=want_def, want_rep=False, def_cap=def_cap,
                             values_cap=values_cap)
    calls, st = _gpu_calls(ctx, ptype, pages, batch, want_def, def_cap, values_cap, optional, type_length)
    if expect_status is not None:
        assert ref["status"] == expect_status, ref["message"]
    assert st == ref["status"], (st, ref["status"], ref["message"])
    assert [(c[2], c[3]) for c in calls] == ref["counts"][:len(calls)]
    assert len(calls) == ref["batches"]
    ba = ptype in (oracle.BYTE_ARRAY, oracle.FIXED_LEN_BYTE_ARRAY)
    if ba:
        got = [x for c in calls for x in c[0]]
        assert got == ref["values"]
    else:
        got = b"".join(np.asarray(c[0]).tobytes() for c in calls)
        assert got == np.asarray(ref["values"]).tobytes()
    if want_def and optional:
        got_def = np.concatenate([c[1] for c in calls]) if calls else np.zeros(0, np.int16)
        np.testing.assert_array_equal(got_def, ref["def"])
    return ref, calls


def _i32(rng):
    return lambda nn: rng.integers(-2 ** 31, 2 ** 31, nn, dtype=np.int64).astype(np.int32).tobytes()


@pytest.mark.parametrize("batch", [16, 17, 512, 1024])
def test_no_def_levels_nullable_plain_no_nulls(oracle, ctx, batch):
    """OPTIONAL PLAIN INT32 without nulls read with def = None: every level slot a value, the
    calls and values the reference's (A.2 on a column whose pages hold every value)."""
    rng = np.random.default_rng(1)
    pages = [_page(oracle, rng, n, 0.0, _i32(rng), oracle.PLAIN) for n in (3000, 1, 4097, 700)]
    ref, calls = _check(oracle, ctx, oracle.INT32, pages, batch, want_def=False, expect_status=0)
    assert all(c[3] == 0 for c in calls)  # levels_read 0 without def / rep levels
    assert sum(c[2] for c in calls) == 3000 + 1 + 4097 + 700


@pytest.mark.parametrize("batch", [16, 100, 1024])
def test_no_def_levels_nullable_plain_with_nulls(oracle, ctx, batch):
    """OPTIONAL PLAIN INT32 with nulls read with def = None: iter_batch_size values per page
    iteration until a page's value bytes run out, then the reference's EOF, at the same call."""
    rng = np.random.default_rng(2)
    pages = [_page(oracle, rng, n, 0.05, _i32(rng), oracle.PLAIN) for n in (5000, 3000)]
    _check(oracle, ctx, oracle.INT32, pages, batch, want_def=False, expect_status=oracle.EOF)


def test_no_def_levels_nullable_int64_and_int96_with_nulls(oracle, ctx):
    rng = np.random.default_rng(3)
    i64 = lambda nn: rng.integers(-2 ** 62, 2 ** 62, nn, dtype=np.int64).tobytes()  # noqa: E731
    i96 = lambda nn: rng.integers(0, 256, nn * 12, dtype=np.uint8).tobytes()  # noqa: E731
    _check(oracle, ctx, oracle.INT64, [_page(oracle, rng, 2000, 0.3, i64, oracle.PLAIN)], 64, False,
           expect_status=oracle.EOF)
    _check(oracle, ctx, oracle.INT96, [_page(oracle, rng, 900, 0.01, i96, oracle.PLAIN)], 128, False,
           expect_status=oracle.EOF)


def test_no_def_levels_plain_byte_array_with_nulls_panics(oracle, ctx):
    """PLAIN BYTE_ARRAY read past the page's values: the length read panics (read_num_bytes!)."""
    rng = np.random.default_rng(4)
    strs = lambda nn: oracle.plain_encode_ba([b"x" * int(k) for k in rng.integers(0, 9, nn)])  # noqa: E731
    pages = [_page(oracle, rng, 1500, 0.02, strs, oracle.PLAIN)]
    _check(oracle, ctx, oracle.BYTE_ARRAY, pages, 100, False, expect_status=oracle.PANIC)
    _check(oracle, ctx, oracle.BYTE_ARRAY, [_page(oracle, rng, 1500, 0.0, strs, oracle.PLAIN)], 100, False,
           expect_status=0)


def test_no_def_levels_delta_with_nulls_short_then_hang(oracle, ctx):
    """DELTA_BINARY_PACKED read with def = None past the page's values: a short read (the
    header's count), then no progress: the reference loops forever (PQG_ERR_HANG)."""
    rng = np.random.default_rng(5)
    delta = lambda nn: oracle.delta_encode(oracle.INT64, np.cumsum(rng.integers(-999, 999, nn)))  # noqa: E731
    pages = [_page(oracle, rng, 3000, 0.1, delta, oracle.DELTA_BINARY_PACKED)]
    _check(oracle, ctx, oracle.INT64, pages, 256, False, expect_status=oracle.HANG)
    pages = [_page(oracle, rng, n, 0.0, delta, oracle.DELTA_BINARY_PACKED) for n in (3000, 129)]
    _check(oracle, ctx, oracle.INT64, pages, 256, False, expect_status=0)


def test_no_def_levels_dictionary_with_nulls_is_nyi(oracle, ctx):
    """Dictionary pages read with def = None past their values: the reference decodes the index
    stream's padding there; the GPU reader does not replay it (PQG_ERR_NYI).
    Without nulls the reads match the reference."""
    import pqgpu
    rng = np.random.default_rng(6)
    dvals = np.arange(100, dtype=np.int64) * 7
    dpage = oracle.PageSpec(oracle.PAGE_DICTIONARY, oracle.plain_encode(oracle.INT64, dvals), 100, oracle.PLAIN)
    idx = lambda nn: bytes([7]) + oracle.rle_encode(rng.integers(0, 100, nn).astype(np.uint64), 7)  # noqa: E731
    _check(oracle, ctx, oracle.INT64, [dpage, _page(oracle, rng, 5000, 0.0, idx, oracle.RLE_DICTIONARY)], 333,
           False, expect_status=0)
    pages = [dpage, _page(oracle, rng, 5000, 0.2, idx, oracle.RLE_DICTIONARY)]
    calls, st = _gpu_calls(ctx, oracle.INT64, pages, 333, False)
    assert st == pqgpu.NYI
    ref = oracle.read_column(oracle.INT64, pages, max_def=1, batch_size=333, want_def=False)
    assert ref["status"] != 0  # the reference reaches the padding, then loops forever
    got = b"".join(np.asarray(c[0]).tobytes() for c in calls)
    assert got == np.asarray(ref["values"]).tobytes()[:len(got)]


@pytest.mark.parametrize("batch,def_cap", [(1024, 100), (512, 511), (64, 1), (1000, 1000)])
def test_def_slice_shorter_than_batch(oracle, ctx, batch, def_cap):
    """A def slice shorter than batch_size clamps the batch (:172-174) and every iteration."""
    rng = np.random.default_rng(7)
    pages = [_page(oracle, rng, n, 0.3, _i32(rng), oracle.PLAIN) for n in (2500, 77, 4096)]
    _check(oracle, ctx, oracle.INT32, pages, batch, want_def=True, def_cap=def_cap, expect_status=0)


@pytest.mark.parametrize("batch,def_cap,values_cap", [(100, 1000, 1000), (100, 150, 1000), (100, 1000, 120)])
def test_slices_longer_than_batch_cross_pages(oracle, ctx, batch, def_cap, values_cap):
    """Slices longer than batch_size: an iteration after a page boundary is clamped by batch_size
    and the slices' room, not by what is left of the batch (:187-205), so a call can return more
    than batch_size levels."""
    rng = np.random.default_rng(8)
    pages = [_page(oracle, rng, n, 0.25, _i32(rng), oracle.PLAIN) for n in (130, 90, 1000, 33)]
    ref, calls = _check(oracle, ctx, oracle.INT32, pages, batch, want_def=True, def_cap=def_cap,
                        values_cap=values_cap, expect_status=0)
    if def_cap > batch and values_cap > batch:
        assert max(c[3] for c in calls) > batch


def test_values_slice_shorter_required(oracle, ctx):
    """REQUIRED column: values.len() < batch_size clamps the batch (:171)."""
    rng = np.random.default_rng(9)
    i32 = _i32(rng)
    pages = [oracle.PageSpec(oracle.PAGE_DATA, i32(n), n, oracle.PLAIN) for n in (1000, 2000)]
    _check(oracle, ctx, oracle.INT32, pages, 1024, want_def=False, values_cap=300, optional=False,
           expect_status=0)
    _check(oracle, ctx, oracle.INT32, pages, 1024, want_def=True, values_cap=300, def_cap=50, optional=False,
           expect_status=0)


def test_empty_data_page_ends_the_call(oracle, ctx):
    """A data page of 0 values: has_next returns false on it (:416-430), the call ends short, the
    next call goes on with the page after it."""
    rng = np.random.default_rng(10)
    pages = [_page(oracle, rng, 300, 0.1, _i32(rng), oracle.PLAIN),
             oracle.PageSpec(oracle.PAGE_DATA, oracle.level_encode(np.zeros(0, np.int16), 1), 0, oracle.PLAIN),
             _page(oracle, rng, 500, 0.1, _i32(rng), oracle.PLAIN)]
    for want_def in (True, False):
        ref, calls = _check(oracle, ctx, oracle.INT32, pages, 1024, want_def=want_def,
                            expect_status=0 if want_def else None)
        if want_def:
            assert len(calls) == 2 and calls[0][3] == 300
