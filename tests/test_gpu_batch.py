"""Batched decode (pqg_decode_chunks): many column chunks of different types, encodings, level
widths and dictionary sizes in one pass must each decode exactly as the oracle decodes them alone
(every chunk is what one ColumnReaderImpl reads, column/reader.rs:159-488; the chunks share
nothing, file/reader.rs:252-260). Also: failures are reported per chunk and call."""
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


def _strings(rng, n, lo=0, hi=30, alphabet=b"abcdefghijklmnop"):
    a = np.frombuffer(alphabet, np.uint8)
    return [bytes(a[rng.integers(0, len(a), l)]) for l in rng.integers(lo, hi + 1, n)]


def _opt(oracle, rng, n, p_null, body_of, encoding, v2=False, max_def=1):
    lv = (rng.random(n) >= p_null).astype(np.int16) * max_def
    nn = int((lv == max_def).sum())
    body = body_of(nn)
    if v2:
        lev = oracle.level_encode(lv, max_def, oracle.RLE, v2=True)
        return oracle.PageSpec(oracle.PAGE_DATA_V2, lev + body, n, encoding, def_len=len(lev))
    return oracle.PageSpec(oracle.PAGE_DATA, oracle.level_encode(lv, max_def) + body, n, encoding)


def _dict_chunk(oracle, rng, ptype, dvals, sizes, p_null, ba=False, fixed=False, required=False):
    if ba:
        dbytes = oracle.plain_encode_ba(dvals, fixed=fixed)
    else:
        dbytes = oracle.plain_encode(ptype, dvals)
    d = oracle.PageSpec(oracle.PAGE_DICTIONARY, dbytes, len(dvals), oracle.PLAIN_DICTIONARY)
    bw = max(1, int(np.ceil(np.log2(len(dvals)))))
    enc = lambda nn: bytes([bw]) + oracle.rle_encode(rng.integers(0, len(dvals), nn).astype(np.uint64), bw)  # noqa: E731
    if required:
        return [d] + [oracle.PageSpec(oracle.PAGE_DATA, enc(n), n, oracle.RLE_DICTIONARY) for n in sizes]
    return [d] + [_opt(oracle, rng, n, p_null, enc, oracle.RLE_DICTIONARY) for n in sizes]


def _zoo(oracle, seed=11):
    """(name, ptype, pages, max_def, max_rep, type_length, want_def) of one chunk each."""
    rng = np.random.default_rng(seed)
    z = []
    i32 = lambda nn: rng.integers(-2 ** 31, 2 ** 31, nn, dtype=np.int64).astype(np.int32).tobytes()  # noqa: E731
    z.append(("int32_plain", oracle.INT32, [_opt(oracle, rng, n, 0.3, i32, oracle.PLAIN) for n in (5000, 70001, 3)],
              1, 0, -1, True))
    z.append(("int64_dict_small", oracle.INT64,
              _dict_chunk(oracle, rng, oracle.INT64, np.unique(rng.integers(-10 ** 12, 10 ** 12, 400))[:250],
                          (9000, 40000), 0.2), 1, 0, -1, True))
    z.append(("int64_dict_large", oracle.INT64,
              _dict_chunk(oracle, rng, oracle.INT64, np.unique(rng.integers(-10 ** 15, 10 ** 15, 80000))[:70000],
                          (100000, 20000), 0.0, required=True), 0, 0, -1, True))
    i96 = np.frombuffer(rng.integers(0, 256, 100 * 12, dtype=np.uint8).tobytes(), dtype=np.uint8).reshape(100, 12)
    z.append(("int96_dict", oracle.INT96, _dict_chunk(oracle, rng, oracle.INT96, i96, (3000,), 0.1), 1, 0, -1, True))
    z.append(("bool_plain", oracle.BOOLEAN,
              [_opt(oracle, rng, n, 0.2, lambda nn: oracle.plain_encode(oracle.BOOLEAN, rng.integers(0, 2, nn).astype(np.uint8)),
                    oracle.PLAIN) for n in (777, 20000)], 1, 0, -1, True))
    z.append(("bool_rle_v2", oracle.BOOLEAN,
              [_opt(oracle, rng, n, 0.1, lambda nn: oracle.rle_bool_encode((rng.random(nn) < 0.3).astype(np.uint8)),
                    oracle.RLE, v2=True) for n in (5000, 65537)], 1, 0, -1, True))
    z.append(("double_dict", oracle.DOUBLE,
              _dict_chunk(oracle, rng, oracle.DOUBLE, rng.standard_normal(200), (30000,), 0.5), 1, 0, -1, True))
    z.append(("int32_delta", oracle.INT32,
              [oracle.PageSpec(oracle.PAGE_DATA, oracle.delta_encode(oracle.INT32, np.cumsum(rng.integers(-99, 99, n)).astype(np.int32)),
                               n, oracle.DELTA_BINARY_PACKED) for n in (4000, 129)], 0, 0, -1, True))
    z.append(("int64_delta", oracle.INT64,
              [_opt(oracle, rng, n, 0.25, lambda nn: oracle.delta_encode(oracle.INT64, np.cumsum(rng.integers(-9999, 9999, nn))),
                    oracle.DELTA_BINARY_PACKED, v2=True) for n in (10000, 4097)], 1, 0, -1, True))
    z.append(("ba_plain", oracle.BYTE_ARRAY,
              [_opt(oracle, rng, n, 0.3, lambda nn: oracle.plain_encode_ba(_strings(rng, nn)), oracle.PLAIN) for n in (6000, 10)],
              1, 0, -1, True))
    z.append(("ba_dict_small", oracle.BYTE_ARRAY,
              _dict_chunk(oracle, rng, oracle.BYTE_ARRAY, list(dict.fromkeys(_strings(rng, 600, 1, 20)))[:500],
                          (12000, 3), 0.2, ba=True), 1, 0, -1, True))
    z.append(("ba_dict_large", oracle.BYTE_ARRAY,
              _dict_chunk(oracle, rng, oracle.BYTE_ARRAY, [b"v%06d" % i for i in range(70000)], (50000,), 0.1, ba=True),
              1, 0, -1, True))
    z.append(("ba_delta_length", oracle.BYTE_ARRAY,
              [_opt(oracle, rng, n, 0.3, lambda nn: oracle.delta_length_encode(_strings(rng, nn)), oracle.DELTA_LENGTH_BYTE_ARRAY)
               for n in (3000,)], 1, 0, -1, True))
    z.append(("ba_delta_byte_array", oracle.BYTE_ARRAY,
              [_opt(oracle, rng, n, 0.1, lambda nn: oracle.delta_byte_array_encode(sorted(_strings(rng, nn, 3, 25))),
                    oracle.DELTA_BYTE_ARRAY) for n in (2500, 77)], 1, 0, -1, True))
    z.append(("flba_dict_v2", oracle.FIXED_LEN_BYTE_ARRAY,
              [_dict_chunk(oracle, rng, oracle.FIXED_LEN_BYTE_ARRAY, list(dict.fromkeys(_strings(rng, 300, 16, 16))),
                           (), 0, ba=True, fixed=True)[0]] +
              [_opt(oracle, rng, 4000, 0.3,
                    lambda nn: bytes([9]) + oracle.rle_encode(rng.integers(0, 290, nn).astype(np.uint64), 9),
                    oracle.RLE_DICTIONARY, v2=True)], 1, 0, 16, True))
    for md, mr in ((3, 2), (7, 3)):  # nested columns: level streams of bit widths 2, 3 beside width 1
        pages = []
        for n in (3000, 2500):
            d = rng.integers(0, md + 1, n).astype(np.int16)
            r = rng.integers(0, mr + 1, n).astype(np.int16)
            body = oracle.plain_encode(oracle.INT32, rng.integers(-5, 5, int((d == md).sum())).astype(np.int32))
            pages.append(oracle.PageSpec(oracle.PAGE_DATA, oracle.level_encode(r, mr) + oracle.level_encode(d, md) + body,
                                         n, oracle.PLAIN))
        z.append((f"nested_{md}_{mr}", oracle.INT32, pages, md, mr, -1, True))
    # def levels not read (read_batch(None, ..), column/reader.rs:247-250): every level slot a value
    z.append(("int32_levels_not_read", oracle.INT32,
              [_opt(oracle, rng, n, 0.0, i32, oracle.PLAIN) for n in (300000,)], 1, 0, -1, False))
    z.append(("float_plain_dictionary_required", oracle.FLOAT,
              _dict_chunk(oracle, rng, oracle.FLOAT, rng.standard_normal(37).astype(np.float32), (5000,), 0, required=True),
              0, 0, -1, True))
    return z


def _decode_batch(ctx, zoo, order=None):
    """One pqg_decode_chunks over the zoo's chunks (in `order`): every page in one blob."""
    import torch

    import pqgpu
    order = list(range(len(zoo))) if order is None else order
    parts, off, arrays, cols, outs, keep = [], 0, [], [], [], []
    for j in order:
        name, pt, specs, md, mr, tl, wdef = zoo[j]
        arr = (pqgpu.Page * max(len(specs), 1))()
        for i, s in enumerate(specs):
            pad = (-off) % 64
            parts.append(b"\0" * pad)
            off += pad
            arr[i] = pqgpu.Page(off, len(s.buf), s.num_values, s.page_type, s.encoding, s.def_encoding,
                                s.rep_encoding, s.def_len, s.rep_len)
            parts.append(s.buf)
            off += len(s.buf)
        arrays.append(arr)
    blob = b"".join(parts) + b"\0" * 64
    d_blob = torch.frombuffer(bytearray(blob), dtype=torch.uint8).cuda()
    for j in order:
        name, pt, specs, md, mr, tl, wdef = zoo[j]
        nlev = sum(s.num_values for s in specs if s.page_type != pqgpu.PAGE_DICTIONARY)
        ba = pt in (pqgpu.BYTE_ARRAY, pqgpu.FIXED_LEN_BYTE_ARRAY)
        es = pqgpu.VALUE_SIZE.get(pt, 1)
        cap = len(blob) + 64 if ba else max(nlev, 1) * es
        d_def = torch.empty(nlev + 8, dtype=torch.int16, device="cuda") if (md > 0 and wdef) else None
        d_rep = torch.empty(nlev + 8, dtype=torch.int16, device="cuda") if mr > 0 else None
        d_val = torch.empty(cap + 64, dtype=torch.uint8, device="cuda")
        d_off = torch.empty(nlev + 2, dtype=torch.int64, device="cuda") if ba else None
        cols.append(pqgpu.Column(pt, tl, md, mr))
        outs.append(pqgpu.Output(d_def.data_ptr() if d_def is not None else None,
                                 d_rep.data_ptr() if d_rep is not None else None, d_val.data_ptr(), cap,
                                 d_off.data_ptr() if ba else None, nlev + 1 if ba else 0, 0, 0, 0))
        keep.append((d_def, d_rep, d_val, d_off))
    oa = ctx.decode_chunks_async(cols, d_blob.data_ptr(), len(blob), [arrays[k] for k in range(len(order))], outs,
                                 torch.cuda.current_stream().cuda_stream)
    st = ctx.sync_detail()
    res = []
    for k, j in enumerate(order):
        d_def, d_rep, d_val, d_off = keep[k]
        o = oa[k]
        r = {"num_levels": o.num_levels, "num_values": o.num_values, "num_bytes": o.num_bytes}
        if st[0] == 0:
            r["def"] = d_def[:o.num_levels].cpu().numpy() if d_def is not None else None
            r["rep"] = d_rep[:o.num_levels].cpu().numpy() if d_rep is not None else None
            if d_off is not None:
                r["offsets"] = d_off[:o.num_values + 1].cpu().numpy()
                r["bytes"] = d_val[:o.num_bytes].cpu().numpy().tobytes()
            else:
                es = pqgpu.VALUE_SIZE.get(zoo[j][1], 1)
                r["raw"] = d_val[:o.num_values * es].cpu().numpy().tobytes()
        res.append(r)
    return st, res


def _check_zoo(oracle, zoo, st, res, order):
    assert st[0] == 0, st
    for k, j in enumerate(order):
        name, pt, specs, md, mr, tl, wdef = zoo[j]
        ref = oracle.read_column(pt, specs, max_def=md, max_rep=mr, type_length=tl, want_def=wdef)
        assert ref["status"] == 0, (name, ref["message"])
        got = res[k]
        assert got["num_values"] == len(ref["values"]), name
        if md > 0 and wdef:
            np.testing.assert_array_equal(got["def"], ref["def"], err_msg=name)
        if mr > 0:
            np.testing.assert_array_equal(got["rep"], ref["rep"], err_msg=name)
        if "bytes" in got:
            assert got["bytes"] == ref["bytes"], name
            np.testing.assert_array_equal(got["offsets"], ref["offsets"], err_msg=name)
        else:
            assert got["raw"] == ref["values"].tobytes(), name


def test_batch_of_every_kind(oracle, ctx):
    """Every chunk of the zoo in one pass, in file order and reversed."""
    zoo = _zoo(oracle)
    for order in (list(range(len(zoo))), list(reversed(range(len(zoo))))):
        st, res = _decode_batch(ctx, zoo, order)
        _check_zoo(oracle, zoo, st, res, order)


def test_batch_equals_chunk_by_chunk(oracle, ctx):
    """The batch's outputs are byte-identical to pqg_decode_chunk of each chunk alone."""
    import pqgpu
    zoo = _zoo(oracle, seed=5)
    order = list(range(len(zoo)))
    st, res = _decode_batch(ctx, zoo, order)
    assert st[0] == 0, st
    for k, (name, pt, specs, md, mr, tl, wdef) in enumerate(zoo):
        one = pqgpu.decode_column(ctx, pt, specs, max_def=md, max_rep=mr, type_length=tl, want_def=wdef)
        assert one["status"] == 0, (name, one["message"])
        assert one["num_values"] == res[k]["num_values"], name
        if "bytes" in res[k]:
            assert one["bytes"] == res[k]["bytes"], name
        else:
            assert np.asarray(one["values"]).tobytes() == res[k]["raw"], name


def test_batch_reports_failing_chunk(oracle, ctx):
    """Chunks 3 and 7 of a batch fail (a PLAIN page cut short, a dictionary index past the
    dictionary): sync_detail names call 0, chunk 3 and its page; the others still decode."""
    import pqgpu
    zoo = _zoo(oracle, seed=9)[:10]
    name, pt, specs, md, mr, tl, wdef = zoo[3]  # int96_dict: cut its data page
    specs = list(specs)
    specs[1] = oracle.PageSpec(specs[1].page_type, specs[1].buf[:len(specs[1].buf) // 3], specs[1].num_values,
                               specs[1].encoding)
    zoo[3] = (name, pt, specs, md, mr, tl, wdef)
    name7, pt7, specs7, md7, mr7, tl7, wdef7 = zoo[7]  # int32_delta: truncate its stream
    s7 = list(specs7)
    s7[0] = oracle.PageSpec(s7[0].page_type, s7[0].buf[:20], s7[0].num_values, s7[0].encoding)
    zoo[7] = (name7, pt7, s7, md7, mr7, tl7, wdef7)
    st, res = _decode_batch(ctx, zoo)
    ref3 = oracle.read_column(pt, specs, max_def=md)
    assert ref3["status"] != 0
    assert st[0] != 0 and st[1] == 0 and st[2] == 3 and st[3] == 1, st
    # the healthy chunks were decoded all the same (their counters filled)
    assert res[0]["num_values"] == len(oracle.read_column(zoo[0][1], zoo[0][2], max_def=1)["values"])
    assert pqgpu.OK == 0


def _plain_zoo(oracle, seed=21):
    """Chunks whose data pages are all PLAIN behind def levels (the speculative copy's chunks),
    one with trailing bytes after its values (the reference reads the non-null values only), one
    whose first page holds fewer value bytes than its non-null values need (EOF)."""
    rng = np.random.default_rng(seed)
    i32 = lambda nn: rng.integers(-2 ** 31, 2 ** 31, nn, dtype=np.int64).astype(np.int32).tobytes()  # noqa: E731
    i64 = lambda nn: rng.integers(-2 ** 62, 2 ** 62, nn, dtype=np.int64).tobytes()  # noqa: E731
    f64 = lambda nn: rng.standard_normal(nn).tobytes()  # noqa: E731
    i96 = lambda nn: rng.integers(0, 256, nn * 12, dtype=np.uint8).tobytes()  # noqa: E731
    z = [("int32_plain", oracle.INT32, [_opt(oracle, rng, n, 0.3, i32, oracle.PLAIN) for n in (5000, 70001, 3)],
          1, 0, -1, True),
         ("double_plain_v2", oracle.DOUBLE, [_opt(oracle, rng, n, 0.0, f64, oracle.PLAIN, v2=True) for n in (4096, 9)],
          1, 0, -1, True),
         ("int96_plain", oracle.INT96, [_opt(oracle, rng, n, 0.2, i96, oracle.PLAIN) for n in (1000, 2000)],
          1, 0, -1, True)]
    pages = [_opt(oracle, rng, n, 0.1, i64, oracle.PLAIN) for n in (3000, 6000, 50)]
    pages[1] = oracle.PageSpec(pages[1].page_type, pages[1].buf + b"\x07" * 21, pages[1].num_values, pages[1].encoding)
    z.append(("int64_plain_trailing", oracle.INT64, pages, 1, 0, -1, True))
    return z


@pytest.mark.parametrize("overlap", [2, 1, 0])
def test_speculative_plain_copy(oracle, ctx, overlap):
    """PLAIN values behind def levels, copied beside the level decode at the value sections'
    offsets (pqg_ctx_set_overlap 1: from the start, 2: beside the emit) or after it (0): identical
    to the oracle, including a chunk whose speculative offsets are wrong (trailing value bytes:
    re-copied at the true offsets)."""
    zoo = _plain_zoo(oracle)
    ctx.set_overlap(overlap)
    try:
        for order in (list(range(len(zoo))), [3, 0, 2, 1]):
            st, res = _decode_batch(ctx, zoo, order)
            _check_zoo(oracle, zoo, st, res, order)
    finally:
        ctx.set_overlap(0)


def test_speculative_plain_copy_short_section(oracle, ctx):
    """A PLAIN page whose value section is shorter than its non-null values: EOF on that page, the
    same with the speculative copy as without (eof_err!, decoding.rs:138-186)."""
    zoo = _plain_zoo(oracle, seed=22)
    name, pt, pages, md, mr, tl, wdef = zoo[0]
    pages = list(pages)
    pages[1] = oracle.PageSpec(pages[1].page_type, pages[1].buf[:-9], pages[1].num_values, pages[1].encoding)
    zoo[0] = (name, pt, pages, md, mr, tl, wdef)
    ref = oracle.read_column(pt, pages, max_def=md)
    assert ref["status"] != 0
    for overlap in (2, 1, 0):
        ctx.set_overlap(overlap)
        try:
            st, res = _decode_batch(ctx, zoo)
        finally:
            ctx.set_overlap(0)
        assert st[0] == ref["status"] and st[2] == 0 and st[3] == 1, (overlap, st)
