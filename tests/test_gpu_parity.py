"""GPU parity: the HIP path (through the C ABI) against the C oracle on the same pages.

Inputs are produced with the restated reference writers (oracle encoders), so every page is
byte-identical to what parquet-rs would write. The bar is bit-exact equality of def/rep
levels and dense values with the oracle's ColumnReaderImpl::read_batch concatenation.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    import pqgpu
    c = pqgpu.Context(0)
    yield c
    c.close()


def _check(oracle, ctx, ptype, pages, max_def=0, max_rep=0, type_length=-1, want_def=True,
           want_rep=True):
    import pqgpu
    ref = oracle.read_column(ptype, pages, max_def=max_def, max_rep=max_rep,
                             type_length=type_length, batch_size=1024, want_def=want_def,
                             want_rep=want_rep)
    got = pqgpu.decode_column(ctx, ptype, pages, max_def=max_def, max_rep=max_rep,
                              type_length=type_length, want_def=want_def, want_rep=want_rep)
    assert ref["status"] == 0, ref["message"]
    assert got["status"] == 0, got["message"]
    if want_def and max_def > 0:
        np.testing.assert_array_equal(got["def"], ref["def"])
    if want_rep and max_rep > 0:
        np.testing.assert_array_equal(got["rep"], ref["rep"])
    assert got["num_values"] == len(ref["values"])
    if ptype == oracle.INT96:
        assert got["values"].tobytes() == ref["values"].tobytes()
    else:
        np.testing.assert_array_equal(got["values"].view(np.uint8), ref["values"].view(np.uint8))
    return got, ref


def _levels_plain_pages(oracle, rng, sizes, p_null, v2=False, ptype=None, dtype=np.int32,
                        def_enc=None):
    ptype = oracle.INT32 if ptype is None else ptype
    pages = []
    for n in sizes:
        lv = (rng.random(n) >= p_null).astype(np.int16)
        nn = int(lv.sum())
        if dtype == np.uint8:
            vals = rng.integers(0, 2, size=nn).astype(np.uint8)
        elif np.issubdtype(dtype, np.floating):
            vals = rng.standard_normal(nn).astype(dtype)
        else:
            info = np.iinfo(dtype)
            vals = rng.integers(info.min, info.max, size=nn, dtype=dtype, endpoint=True)
        body = oracle.plain_encode(ptype, vals)
        if v2:
            lev = oracle.level_encode(lv, 1, oracle.RLE, v2=True)
            pages.append(oracle.PageSpec(oracle.PAGE_DATA_V2, lev + body, n, oracle.PLAIN,
                                         def_len=len(lev)))
        else:
            e = oracle.RLE if def_enc is None else def_enc
            lev = oracle.level_encode(lv, 1, e)
            pages.append(oracle.PageSpec(oracle.PAGE_DATA, lev + body, n, oracle.PLAIN,
                                         def_encoding=e))
    return pages


@pytest.mark.parametrize("p_null", [0.0, 0.1, 0.5, 0.97, 1.0])
def test_def_levels_plain_int32(oracle, ctx, p_null):
    rng = np.random.default_rng(int(p_null * 100) + 1)
    sizes = [1, 7, 8, 9, 63, 64, 65, 1000, 4096, 20000, 65536 + 3]
    _check(oracle, ctx, oracle.INT32, _levels_plain_pages(oracle, rng, sizes, p_null), max_def=1)


def test_def_levels_v2_and_bitpacked(oracle, ctx):
    rng = np.random.default_rng(2)
    pages = _levels_plain_pages(oracle, rng, [1000, 77, 5000], 0.3, v2=True)
    _check(oracle, ctx, oracle.INT32, pages, max_def=1)
    pages = _levels_plain_pages(oracle, rng, [1000, 5000], 0.3, def_enc=oracle.BIT_PACKED)
    _check(oracle, ctx, oracle.INT32, pages, max_def=1)


@pytest.mark.parametrize("ptype,dtype", [("INT64", np.int64), ("FLOAT", np.float32),
                                         ("DOUBLE", np.float64), ("BOOLEAN", np.uint8)])
def test_plain_types(oracle, ctx, ptype, dtype):
    rng = np.random.default_rng(3)
    t = getattr(oracle, ptype)
    pages = _levels_plain_pages(oracle, rng, [3, 1000, 33333], 0.2, ptype=t, dtype=dtype)
    _check(oracle, ctx, t, pages, max_def=1)


def test_plain_int96_required(oracle, ctx):
    rng = np.random.default_rng(4)
    pages = []
    for n in (5, 1001):
        words = rng.integers(0, 2 ** 32, size=(n, 3), dtype=np.uint64).astype(np.uint32)
        pages.append(oracle.PageSpec(oracle.PAGE_DATA, words.tobytes(), n, oracle.PLAIN))
    _check(oracle, ctx, oracle.INT96, pages)


def test_required_levels_ignored(oracle, ctx):
    rng = np.random.default_rng(5)
    vals = rng.integers(-100, 100, size=5000).astype(np.int64)
    pages = [oracle.PageSpec(oracle.PAGE_DATA, oracle.plain_encode(oracle.INT64, vals), 5000, oracle.PLAIN)]
    got, ref = _check(oracle, ctx, oracle.INT64, pages)
    assert got["num_levels"] == 0


@pytest.mark.parametrize("max_def,max_rep", [(2, 1), (3, 2), (7, 3)])
def test_nested_levels(oracle, ctx, max_def, max_rep):
    rng = np.random.default_rng(max_def * 10 + max_rep)
    pages = []
    for n, v2 in ((3000, False), (2500, True), (10, False)):
        d = rng.integers(0, max_def + 1, size=n).astype(np.int16)
        r = rng.integers(0, max_rep + 1, size=n).astype(np.int16)
        nn = int((d == max_def).sum())
        vals = rng.integers(-5, 5, size=nn).astype(np.int32)
        body = oracle.plain_encode(oracle.INT32, vals)
        if v2:
            rl = oracle.level_encode(r, max_rep, oracle.RLE, v2=True)
            dl = oracle.level_encode(d, max_def, oracle.RLE, v2=True)
            pages.append(oracle.PageSpec(oracle.PAGE_DATA_V2, rl + dl + body, n, oracle.PLAIN,
                                         rep_len=len(rl), def_len=len(dl)))
        else:
            rl = oracle.level_encode(r, max_rep, oracle.RLE)
            dl = oracle.level_encode(d, max_def, oracle.RLE)
            pages.append(oracle.PageSpec(oracle.PAGE_DATA, rl + dl + body, n, oracle.PLAIN))
    _check(oracle, ctx, oracle.INT32, pages, max_def=max_def, max_rep=max_rep)


@pytest.mark.parametrize("ptype,dtype,ndict", [("INT32", np.int32, 1), ("INT32", np.int32, 1000),
                                               ("INT64", np.int64, 65536), ("FLOAT", np.float32, 37),
                                               ("DOUBLE", np.float64, 300)])
def test_dictionary(oracle, ctx, ptype, dtype, ndict):
    rng = np.random.default_rng(ndict)
    t = getattr(oracle, ptype)
    if np.issubdtype(dtype, np.floating):
        dvals = rng.standard_normal(ndict).astype(dtype)
    else:
        dvals = np.unique(rng.integers(np.iinfo(dtype).min, np.iinfo(dtype).max, size=ndict * 2,
                                       dtype=dtype))[:ndict]
        rng.shuffle(dvals)
    dvals = dvals[:ndict]
    pages = [oracle.PageSpec(oracle.PAGE_DICTIONARY, oracle.plain_encode(t, dvals), len(dvals),
                             oracle.PLAIN_DICTIONARY)]
    bw = 1 if len(dvals) == 1 else int(oracle.lib().or_log2(len(dvals)))
    for n, mode in ((1000, "random"), (5000, "runs"), (70000, "random"), (1, "random")):
        if mode == "runs":
            idx = np.repeat(rng.integers(0, len(dvals), size=n // 50 + 1), 50)[:n]
        else:
            idx = rng.integers(0, len(dvals), size=n)
        lv = (rng.random(n) < 0.85).astype(np.int16)
        nn = int(lv.sum())
        body = bytes([bw]) + oracle.rle_encode(idx[:nn], bw)
        lev = oracle.level_encode(lv, 1, oracle.RLE)
        pages.append(oracle.PageSpec(oracle.PAGE_DATA, lev + body, n, oracle.RLE_DICTIONARY))
    _check(oracle, ctx, t, pages, max_def=1)
    # required column, PLAIN_DICTIONARY id on the data page (column/reader.rs:391-393)
    req = [pages[0]]
    idx = rng.integers(0, len(dvals), size=12345)
    req.append(oracle.PageSpec(oracle.PAGE_DATA, bytes([bw]) + oracle.rle_encode(idx, bw), 12345,
                               oracle.PLAIN_DICTIONARY))
    _check(oracle, ctx, t, req)


def test_dictionary_fallback_to_plain(oracle, ctx):
    rng = np.random.default_rng(8)
    dvals = np.arange(50, dtype=np.int32) * 3
    pages = [oracle.PageSpec(oracle.PAGE_DICTIONARY, oracle.plain_encode(oracle.INT32, dvals), 50, oracle.PLAIN)]
    for k in range(4):
        n = 3000 + k
        if k < 2:
            idx = rng.integers(0, 50, size=n)
            body = bytes([6]) + oracle.rle_encode(idx, 6)
            pages.append(oracle.PageSpec(oracle.PAGE_DATA, body, n, oracle.RLE_DICTIONARY))
        else:
            v = rng.integers(-1000, 1000, size=n).astype(np.int32)
            pages.append(oracle.PageSpec(oracle.PAGE_DATA, oracle.plain_encode(oracle.INT32, v), n, oracle.PLAIN))
    _check(oracle, ctx, oracle.INT32, pages)


@pytest.mark.parametrize("ptype", ["INT32", "INT64"])
def test_delta_binary_packed(oracle, ctx, ptype):
    t = getattr(oracle, ptype)
    dt = np.int32 if ptype == "INT32" else np.int64
    info = np.iinfo(dt)
    rng = np.random.default_rng(21)
    pages = []
    for n, mode in ((1, "r"), (2, "r"), (129, "r"), (5000, "small"), (40000, "wide"), (777, "ext")):
        if mode == "small":
            v = np.cumsum(rng.integers(-1000, 1000, size=n)).astype(dt)
        elif mode == "wide":
            v = rng.integers(info.min, info.max, size=n, dtype=dt, endpoint=True)
        elif mode == "ext":
            v = rng.choice(np.array([info.min, info.max, 0, -1, 1], dt), size=n)
        else:
            v = rng.integers(-10, 10, size=n).astype(dt)
        pages.append(oracle.PageSpec(oracle.PAGE_DATA, oracle.delta_encode(t, v), n,
                                     oracle.DELTA_BINARY_PACKED))
    _check(oracle, ctx, t, pages)
    # optional column with nulls, v2 pages
    pages = []
    for n in (3000, 4100):
        lv = (rng.random(n) < 0.7).astype(np.int16)
        nn = int(lv.sum())
        v = np.cumsum(rng.integers(-50, 50, size=nn)).astype(dt)
        lev = oracle.level_encode(lv, 1, oracle.RLE, v2=True)
        pages.append(oracle.PageSpec(oracle.PAGE_DATA_V2, lev + oracle.delta_encode(t, v), n,
                                     oracle.DELTA_BINARY_PACKED, def_len=len(lev)))
    _check(oracle, ctx, t, pages, max_def=1)


def test_rle_bool_v2(oracle, ctx):
    rng = np.random.default_rng(31)
    pages = []
    for n in (100, 5000, 65537):
        lv = (rng.random(n) < 0.9).astype(np.int16)
        nn = int(lv.sum())
        vals = (rng.random(nn) < 0.2).astype(np.uint8)
        lev = oracle.level_encode(lv, 1, oracle.RLE, v2=True)
        pages.append(oracle.PageSpec(oracle.PAGE_DATA_V2, lev + oracle.rle_bool_encode(vals), n,
                                     oracle.RLE, def_len=len(lev)))
    _check(oracle, ctx, oracle.BOOLEAN, pages, max_def=1)


def test_kat_vectors_on_gpu(oracle, ctx):
    """The reference's RLE KATs (rle.rs:524-623) as one-page chunks."""
    import pqgpu
    # dict page [10,20,30], RLE runs 3x0 4x1 5x2, bit width 3 (rle.rs:595-609)
    d = oracle.PageSpec(oracle.PAGE_DICTIONARY, np.array([10, 20, 30], np.int32).tobytes(), 3, oracle.PLAIN)
    p = oracle.PageSpec(oracle.PAGE_DATA, bytes([3, 0x06, 0x00, 0x08, 0x01, 0x0A, 0x02]), 12,
                        oracle.RLE_DICTIONARY)
    got = pqgpu.decode_column(ctx, oracle.INT32, [d, p])
    assert got["status"] == 0 and got["values"].tolist() == [10] * 3 + [20] * 4 + [30] * 5
    # bit-packed 0..7 at width 3 (rle.rs:524-535) as dictionary indices into 0..7
    d = oracle.PageSpec(oracle.PAGE_DICTIONARY, np.arange(8, dtype=np.int32).tobytes(), 8, oracle.PLAIN)
    p = oracle.PageSpec(oracle.PAGE_DATA, bytes([3, 0x03, 0x88, 0xC6, 0xFA]), 8, oracle.RLE_DICTIONARY)
    got = pqgpu.decode_column(ctx, oracle.INT32, [d, p])
    assert got["status"] == 0 and got["values"].tolist() == list(range(8))
    # levels v2 KAT (levels.rs:487-506)
    buf = bytes([5, 198, 2, 5, 42, 168, 10, 0, 2, 3, 36, 73])
    page = oracle.PageSpec(oracle.PAGE_DATA_V2, buf, 10, oracle.PLAIN, rep_len=3, def_len=5)
    got = pqgpu.decode_column(ctx, oracle.BOOLEAN, [page], max_def=2, max_rep=1)
    assert got["rep"].tolist() == [0, 1, 1, 0, 0, 0, 1, 1, 0, 1]
    assert got["def"].tolist() == [2, 2, 2, 0, 0, 2, 2, 2, 2, 2]


@pytest.mark.parametrize("case", ["trunc_bp", "trunc_plain", "bad_dict_idx", "no_dict",
                                  "bad_prefix", "delta_trunc", "trunc_dict_plain"])
def test_errors_match_reference_class(oracle, ctx, case):
    """Malformed pages: the GPU path reports an error wherever the reference errors, panics
    or hangs; it never returns data there."""
    import pqgpu
    rng = np.random.default_rng(1)
    ptype, max_def = oracle.INT32, 0
    if case == "trunc_bp":
        pages = [oracle.PageSpec(oracle.PAGE_DATA, oracle.level_encode(np.ones(100, np.int16), 1)[:4] + b"\x03\x01", 100, oracle.PLAIN)]
        lv = (rng.random(200) < .5).astype(np.int16)
        enc = oracle.level_encode(lv, 1)
        enc = enc[:4] + enc[4:-3]
        pages = [oracle.PageSpec(oracle.PAGE_DATA, enc, 200, oracle.PLAIN)]
        max_def = 1
    elif case == "trunc_plain":
        pages = [oracle.PageSpec(oracle.PAGE_DATA, np.arange(10, dtype=np.int32).tobytes()[:-1], 10, oracle.PLAIN)]
    elif case == "bad_dict_idx":
        d = oracle.PageSpec(oracle.PAGE_DICTIONARY, np.arange(3, dtype=np.int32).tobytes(), 3, oracle.PLAIN)
        pages = [d, oracle.PageSpec(oracle.PAGE_DATA, bytes([3, 0x03, 0x88, 0xC6, 0xFA]), 8, oracle.RLE_DICTIONARY)]
    elif case == "no_dict":
        pages = [oracle.PageSpec(oracle.PAGE_DATA, bytes([1, 0x10, 0x01]), 8, oracle.RLE_DICTIONARY)]
    elif case == "trunc_dict_plain":
        # a dictionary page cut short, then PLAIN pages only: configure_dictionary still decodes
        # the dictionary (column/reader.rs:463-481, decoding.rs:145-147) and returns EOF
        d = oracle.PageSpec(oracle.PAGE_DICTIONARY, np.arange(5, dtype=np.int32).tobytes()[:-2], 5, oracle.PLAIN)
        pages = [d, oracle.PageSpec(oracle.PAGE_DATA, np.arange(10, dtype=np.int32).tobytes(), 10, oracle.PLAIN)]
    elif case == "bad_prefix":
        pages = [oracle.PageSpec(oracle.PAGE_DATA, b"\xff\x00\x00\x00\x02\x01", 1, oracle.PLAIN)]
        max_def = 1
    else:
        enc = oracle.delta_encode(oracle.INT32, np.arange(1000, dtype=np.int32) * 7)
        pages = [oracle.PageSpec(oracle.PAGE_DATA, enc[:len(enc) // 2], 1000, oracle.DELTA_BINARY_PACKED)]
    ref = oracle.read_column(ptype, pages, max_def=max_def)
    got = pqgpu.decode_column(ctx, ptype, pages, max_def=max_def)
    assert ref["status"] != 0
    assert got["status"] != 0, "GPU decoded a page the reference rejects"
    if case == "trunc_dict_plain":
        assert ref["status"] == oracle.EOF and got["status"] == pqgpu.EOF and got["page"] == 0


def test_large_chunk_properties(oracle, ctx):
    """Size-independent checks at scale: decode(encode(x)) == x over 8M levels."""
    import pqgpu
    rng = np.random.default_rng(99)
    pages, exp_def, exp_val = [], [], []
    for k in range(8):
        n = 1 << 20
        lv = (rng.random(n) >= 0.1).astype(np.int16)
        nn = int(lv.sum())
        v = rng.integers(-2 ** 31, 2 ** 31, size=nn, dtype=np.int64).astype(np.int32)
        lev = oracle.level_encode(lv, 1, oracle.RLE)
        pages.append(oracle.PageSpec(oracle.PAGE_DATA, lev + oracle.plain_encode(oracle.INT32, v), n, oracle.PLAIN))
        exp_def.append(lv)
        exp_val.append(v)
    got = pqgpu.decode_column(ctx, oracle.INT32, pages, max_def=1)
    assert got["status"] == 0, got["message"]
    np.testing.assert_array_equal(got["def"], np.concatenate(exp_def))
    np.testing.assert_array_equal(got["values"], np.concatenate(exp_val))


@pytest.mark.parametrize("ptype,dtype", [(None, np.int32), ("int64", np.int64), ("int96", None), ("bool", None)])
def test_space_values_matches_levels(oracle, ctx, ptype, dtype):
    """pqg_space_values: the decoded dense values spread onto the def == max_def level slots,
    zeros elsewhere (record/triplet.rs:300-318 over a whole chunk)."""
    import torch

    import pqgpu
    rng = np.random.default_rng(7)
    n = 300_000
    t = {None: oracle.INT32, "int64": oracle.INT64, "int96": oracle.INT96, "bool": oracle.BOOLEAN}[ptype]
    es = {oracle.INT32: 4, oracle.INT64: 8, oracle.INT96: 12, oracle.BOOLEAN: 1}[t]
    d = (rng.random(n) > 0.3).astype(np.int16)
    nn = int(d.sum())
    raw = rng.integers(0, 256, size=nn * es, dtype=np.uint8)
    if t == oracle.BOOLEAN:
        raw = (raw & 1).astype(np.uint8)
    dev = torch.device("cuda")
    d_def = torch.from_numpy(d).to(dev)
    d_val = torch.from_numpy(raw).to(dev)
    d_sp = torch.full((n * es + 16,), 0x5A, dtype=torch.uint8, device=dev)
    st = pqgpu.lib().pqg_space_values(ctx.h, d_def.data_ptr(), n, 1, d_val.data_ptr(), es, d_sp.data_ptr(), None)
    assert st == 0
    torch.cuda.synchronize()
    got = d_sp[: n * es].cpu().numpy().reshape(n, es)
    want = np.zeros((n, es), np.uint8)
    want[d == 1] = raw.reshape(nn, es)
    np.testing.assert_array_equal(got, want)
