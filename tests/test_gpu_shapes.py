"""GPU parity at the shapes the benchmark and the reference's decoders accept, beyond the
reference writer's defaults:

- DELTA_BINARY_PACKED at BASELINE config 4's block shape (512-value blocks of 4 x 128-value
  mini-blocks) and the other shapes DeltaBitPackDecoder accepts (any values_per_mini_block % 8
  == 0, /root/reference/src/encodings/decoding.rs:501-533), including blocks that do not divide
  the decoder's 4096-value tile;
- the RLE/bit-packing hybrid at every bit width 0..32 (RleDecoder::reload, rle.rs:490-508; the
  dictionary decoder accepts any width byte, decoding.rs:292-300);
- the reference quirks of SURVEY Appendix A.3 (1024-index re-loop) and A.5 (BIT_PACKED v1
  levels read at a doubled offset, levels.rs:191-211).

Every case compares the HIP path (through the C ABI) with the C oracle bit for bit.
"""
import zlib

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


def _same(oracle, ctx, ptype, pages, max_def=0, max_rep=0, batch_size=1024, expect_ok=True):
    import pqgpu
    ref = oracle.read_column(ptype, pages, max_def=max_def, max_rep=max_rep, batch_size=batch_size)
    got = pqgpu.decode_column(ctx, ptype, pages, max_def=max_def, max_rep=max_rep)
    if expect_ok:
        assert ref["status"] == 0, ref["message"]
    assert (got["status"] == 0) == (ref["status"] == 0), (got["status"], got["message"],
                                                          ref["status"], ref["message"])
    if ref["status"]:
        return got, ref
    if max_def > 0:
        np.testing.assert_array_equal(got["def"], ref["def"])
    if max_rep > 0:
        np.testing.assert_array_equal(got["rep"], ref["rep"])
    assert got["num_values"] == len(ref["values"])
    assert got["values"].tobytes() == ref["values"].tobytes()
    return got, ref


def _delta_values(rng, dt, n, mode):
    info = np.iinfo(dt)
    if mode == "d16":  # config 4: deltas uniform in [-2^15, 2^15)
        first = rng.integers(info.min, info.max, dtype=dt, endpoint=True)
        d = rng.integers(-(1 << 15), 1 << 15, size=n).astype(dt)
        d[0] = first
        with np.errstate(over="ignore"):
            return np.cumsum(d, dtype=dt)
    if mode == "ext":
        return rng.choice(np.array([info.min, info.max, 0, -1, 1], dt), size=n)
    if mode == "wide":
        return rng.integers(info.min, info.max, size=n, dtype=dt, endpoint=True)
    if mode == "const":
        return np.full(n, 42, dt)
    return rng.integers(-3, 4, size=n).astype(dt)


# (block size, mini-blocks): config 4's shape first; (384, 3) and (192, 3) blocks do not
# divide the 4096-value tile; (64, 8) has 8-value mini-blocks (the smallest the decoder takes)
DELTA_SHAPES = [(512, 4), (256, 8), (1024, 16), (128, 4), (384, 3), (192, 3), (64, 8), (2048, 4)]


@pytest.mark.parametrize("shape", DELTA_SHAPES)
@pytest.mark.parametrize("ptype", ["INT32", "INT64"])
def test_delta_block_shapes(oracle, ctx, ptype, shape):
    bs, nmb = shape
    t = getattr(oracle, ptype)
    dt = np.int32 if ptype == "INT32" else np.int64
    rng = np.random.default_rng(bs * 31 + nmb + (7 if ptype == "INT64" else 0))
    pages, vals = [], []
    for n, mode in ((1, "d16"), (2, "d16"), (129, "d16"), (4097, "d16"), (65537, "d16"),
                    (5000, "ext"), (3001, "wide"), (700, "const"), (4096 * 3 + 5, "small")):
        v = _delta_values(rng, dt, n, mode)
        vals.append(v)
        pages.append(oracle.PageSpec(oracle.PAGE_DATA, oracle.delta_encode(t, v, bs, nmb), n,
                                     oracle.DELTA_BINARY_PACKED))
    expect = np.concatenate(vals)
    got, ref = _same(oracle, ctx, t, pages)
    np.testing.assert_array_equal(got["values"], expect)  # decode(encode(x)) == x as well


# Blocks of many mini-blocks: DeltaBitPackDecoder::init_block reads num_mini_blocks width bytes
# into a Vec, any count (decoding.rs:448-468). 128 and 1024 mini-blocks of 8 values; 32 768
# mini-blocks put a block's width bytes (32 KiB) past the decoder's 16 KiB staged region.
MANY_MB_SHAPES = [(1024, 128), (8192, 1024), (32768, 1024), (262144, 32768)]


@pytest.mark.parametrize("shape", MANY_MB_SHAPES)
@pytest.mark.parametrize("ptype", ["INT32", "INT64"])
def test_delta_many_mini_blocks(oracle, ctx, ptype, shape):
    bs, nmb = shape
    t = getattr(oracle, ptype)
    dt = np.int32 if ptype == "INT32" else np.int64
    rng = np.random.default_rng(bs + nmb + (3 if ptype == "INT64" else 0))
    pages, vals = [], []
    for n, mode in ((1, "d16"), (2, "d16"), (9, "small"), (bs + 1, "d16"), (3 * bs + 77, "small"),
                    (70001, "d16"), (5000, "ext"), (3001, "wide")):
        v = _delta_values(rng, dt, n, mode)
        vals.append(v)
        pages.append(oracle.PageSpec(oracle.PAGE_DATA, oracle.delta_encode(t, v, bs, nmb), n,
                                     oracle.DELTA_BINARY_PACKED))
    got, _ = _same(oracle, ctx, t, pages)
    np.testing.assert_array_equal(got["values"], np.concatenate(vals))


@pytest.mark.parametrize("ptype", ["INT32", "INT64"])
def test_delta_config4_page(oracle, ctx, ptype):
    """One full benchmark page: 2^20 values, 16-bit deltas, 512 / 4 x 128 (bench.py config 4),
    plus a nullable v2 variant at the same shape."""
    t = getattr(oracle, ptype)
    dt = np.int32 if ptype == "INT32" else np.int64
    rng = np.random.default_rng(404)
    v = _delta_values(rng, dt, 1 << 20, "d16")
    pages = [oracle.PageSpec(oracle.PAGE_DATA, oracle.delta_encode(t, v, 512, 4), len(v),
                             oracle.DELTA_BINARY_PACKED)]
    got, _ = _same(oracle, ctx, t, pages)
    np.testing.assert_array_equal(got["values"], v)
    pages = []
    for n in (70000, 4099):
        lv = (rng.random(n) < 0.8).astype(np.int16)
        vals = _delta_values(rng, dt, int(lv.sum()), "d16")
        lev = oracle.level_encode(lv, 1, oracle.RLE, v2=True)
        pages.append(oracle.PageSpec(oracle.PAGE_DATA_V2, lev + oracle.delta_encode(t, vals, 512, 4), n,
                                     oracle.DELTA_BINARY_PACKED, def_len=len(lev)))
    _same(oracle, ctx, t, pages, max_def=1)


def _hybrid(values, w):
    """RLE/bit-packed hybrid through the reference writer (RleEncoder, rle.rs:55-317)."""
    import pyoracle
    return pyoracle.rle_encode(np.asarray(values, np.uint64), w)


@pytest.mark.parametrize("w", list(range(1, 33)))
def test_dictionary_index_width_sweep(oracle, ctx, w):
    """Dictionary indices at bit width w: a 2^w-entry dictionary up to w = 16, beyond that a
    70 000-entry dictionary with indices written at width w (the reader takes any width byte)."""
    rng = np.random.default_rng(1000 + w)
    ndict = (1 << w) if w <= 16 else 70000
    dvals = rng.integers(-2 ** 31, 2 ** 31, size=ndict, dtype=np.int64).astype(np.int32)
    pages = [oracle.PageSpec(oracle.PAGE_DICTIONARY, dvals.tobytes(), ndict, oracle.PLAIN)]
    for n, mode in ((1, "random"), (4103, "random"), (9000, "runs"), (20000, "mixed")):
        if mode == "random":
            idx = rng.integers(0, ndict, size=n)
        elif mode == "runs":
            idx = np.repeat(rng.integers(0, ndict, size=n // 40 + 1), 40)[:n]
        else:
            idx = np.where(rng.random(n) < 0.5, ndict - 1, rng.integers(0, ndict, size=n))
        pages.append(oracle.PageSpec(oracle.PAGE_DATA, bytes([w]) + _hybrid(idx, w), n,
                                     oracle.RLE_DICTIONARY))
    got, _ = _same(oracle, ctx, oracle.INT32, pages)
    assert got["num_values"] == 1 + 4103 + 9000 + 20000


def test_dictionary_index_width_zero(oracle, ctx):
    """Width byte 0: RLE runs carry a 0-byte value and bit-packed groups no payload, so every
    index is 0 (rle.rs:490-508)."""
    d = oracle.PageSpec(oracle.PAGE_DICTIONARY, np.array([77, 88], np.int32).tobytes(), 2, oracle.PLAIN)
    # RLE run of 5 (header 10), bit-packed 2 groups (header 5), RLE run of 300 (varint 0xD8 0x04)
    body = bytes([0, 10, 5, 0xD8, 0x04])
    p = oracle.PageSpec(oracle.PAGE_DATA, body, 5 + 16 + 300, oracle.RLE_DICTIONARY)
    got, ref = _same(oracle, ctx, oracle.INT32, [d, p])
    assert got["values"].tolist() == [77] * 321


@pytest.mark.parametrize("max_def", [1, 2, 3, 7, 15, 100, 255, 1000, 32767])
def test_level_width_sweep(oracle, ctx, max_def):
    """Def levels at every level bit width the reader derives (log2(max_def + 1), levels.rs:163),
    with and without long runs, v1 and v2 pages."""
    rng = np.random.default_rng(max_def)
    pages = []
    for n, v2, mode in ((5000, False, "random"), (70000, True, "runs"), (33, False, "random"),
                        (9000, False, "skew")):
        if mode == "random":
            d = rng.integers(0, max_def + 1, size=n)
        elif mode == "runs":
            d = np.repeat(rng.integers(0, max_def + 1, size=n // 100 + 1), 100)[:n]
        else:
            d = np.where(rng.random(n) < 0.8, max_def, rng.integers(0, max_def + 1, size=n))
        d = d.astype(np.int16)
        nn = int((d == max_def).sum())
        body = oracle.plain_encode(oracle.INT64, rng.integers(-9, 9, size=nn).astype(np.int64))
        if v2:
            lev = oracle.level_encode(d, max_def, oracle.RLE, v2=True)
            pages.append(oracle.PageSpec(oracle.PAGE_DATA_V2, lev + body, n, oracle.PLAIN, def_len=len(lev)))
        else:
            lev = oracle.level_encode(d, max_def, oracle.RLE)
            pages.append(oracle.PageSpec(oracle.PAGE_DATA, lev + body, n, oracle.PLAIN))
    _same(oracle, ctx, oracle.INT64, pages, max_def=max_def)


@pytest.mark.parametrize("rep_enc,def_enc", [("RLE", "BIT_PACKED"), ("BIT_PACKED", "BIT_PACKED"),
                                             ("BIT_PACKED", "RLE")])
def test_bit_packed_v1_double_offset(oracle, ctx, rep_enc, def_enc):
    """a v1 BIT_PACKED level stream is sliced with data.range(data.start(), ..)
    (levels.rs:206) on an already offset buffer, so def levels after rep levels are read from
    twice the offset. GPU and oracle must agree on status and every level and value."""
    rng = np.random.default_rng(55)
    re, de = getattr(oracle, rep_enc), getattr(oracle, def_enc)
    for n in (64, 1000, 4100):
        r = rng.integers(0, 2, size=n).astype(np.int16)
        d = rng.integers(0, 4, size=n).astype(np.int16)
        rl = oracle.level_encode(r, 1, re)
        dl = oracle.level_encode(d, 3, de)
        # enough trailing bytes that the doubled offset stays inside the page
        tail = rng.integers(0, 256, size=len(rl) + len(dl) + 4 * n, dtype=np.uint8).tobytes()
        page = oracle.PageSpec(oracle.PAGE_DATA, rl + dl + tail, n, oracle.PLAIN, def_encoding=de,
                               rep_encoding=re)
        _same(oracle, ctx, oracle.INT32, [page], max_def=3, max_rep=1, expect_ok=False)


def _long_bitpacked_run(idx, w):
    """A bit-packed run of len(idx) values (a multiple of 8) in one header: longer than the
    reference writer's 504-value runs (rle.rs:49-50), as a foreign writer may emit."""
    groups = len(idx) // 8
    h = (groups << 1) | 1
    hdr = bytearray()
    while True:
        b = h & 0x7F
        h >>= 7
        hdr.append(b | (0x80 if h else 0))
        if not h:
            break
    bits = np.zeros(len(idx) * w, np.uint8)
    for b in range(w):
        bits[b::w] = (np.asarray(idx) >> b) & 1
    return bytes(hdr) + np.packbits(bits, bitorder="little").tobytes()


@pytest.mark.parametrize("batch_size", [1, 16, 512, 1000, 2000, 4096])
def test_long_bitpacked_dict_runs(oracle, ctx, batch_size):
    """get_batch_with_dict re-loops without re-clamping once it has read exactly
    1024 indices (rle.rs:466-477). The GPU decode is batch-independent and matches the
    reference at every batch size where that re-loop cannot fire; at batch 1024 the reference
    panics on a >= 1024-value run (asserted below), which DESIGN.md lists as a deviation on
    foreign files only (the reference writer never emits runs over 504 values)."""
    import pqgpu
    rng = np.random.default_rng(3)
    w = 5
    idx = rng.integers(0, 32, size=2000)
    d = oracle.PageSpec(oracle.PAGE_DICTIONARY, (np.arange(32, dtype=np.int64) * 11).tobytes(), 32, oracle.PLAIN)
    p = oracle.PageSpec(oracle.PAGE_DATA, bytes([w]) + _long_bitpacked_run(idx, w), 2000,
                        oracle.RLE_DICTIONARY)
    got, ref = _same(oracle, ctx, oracle.INT64, [d, p], batch_size=batch_size)
    assert got["values"].tolist() == (idx * 11).tolist()
    assert oracle.read_column(oracle.INT64, [d, p], batch_size=1024)["status"] == oracle.PANIC
    assert pqgpu.decode_column(ctx, oracle.INT64, [d, p])["status"] == 0


def test_rejected_call_keeps_pending_decode(oracle, ctx):
    """A call rejected for its arguments (BYTE_ARRAY output without offsets) must not disturb
    the decode still in flight on the same context: pqg_sync then reports that decode."""
    import torch
    import pqgpu
    rng = np.random.default_rng(12)
    vals = rng.integers(-2 ** 31, 2 ** 31, size=5000, dtype=np.int64).astype(np.int32)
    spec = oracle.PageSpec(oracle.PAGE_DATA, vals.tobytes(), len(vals), oracle.PLAIN)
    blob, pages = pqgpu.make_pages([spec])
    d_blob = torch.frombuffer(bytearray(blob), dtype=torch.uint8).cuda()
    d_val = torch.zeros(len(vals) * 4 + 64, dtype=torch.uint8, device="cuda")
    out = pqgpu.Output(None, None, d_val.data_ptr(), len(vals) * 4, None, 0, 0, 0, 0)
    s = torch.cuda.current_stream().cuda_stream
    ctx.decode_async(pqgpu.Column(pqgpu.INT32, -1, 0, 0), d_blob.data_ptr(), len(blob), pages, out, s)
    bad_out = pqgpu.Output(None, None, d_val.data_ptr(), len(vals) * 4, None, 0, 0, 0, 0)
    with pytest.raises(pqgpu.PqgError) as e:
        ctx.decode_async(pqgpu.Column(pqgpu.BYTE_ARRAY, -1, 0, 0), d_blob.data_ptr(), len(blob),
                         pages, bad_out, s)
    assert e.value.status == pqgpu.INVALID
    st, bad = ctx.sync()
    assert st == 0 and bad == -1
    assert out.num_values == len(vals)
    assert d_val[: len(vals) * 4].cpu().numpy().view(np.int32).tolist() == vals.tolist()


@pytest.mark.gpu
@pytest.mark.parametrize("ptype,es", [("INT32", 4), ("INT64", 8), ("INT96", 12), ("DOUBLE", 8)])
@pytest.mark.parametrize("extra", [[0, 0, 0, 0], [0, 3, 0, 0], [0, 0, 1, 0], [5, 0, 0, 7], [0, -1, 0, 0]])
def test_plain_values_behind_def_levels(oracle, ctx, ptype, es, extra):
    """PLAIN values behind def levels go through the speculative copy (value counts implied by
    each value section, copied beside the level decode) and its fix-up: sections with trailing
    values or bytes (the reader takes the first non-null count, decoding.rs:138-186) and a short
    section (EOF on that page) must give the oracle's result."""
    rng = np.random.default_rng(zlib.crc32(repr((ptype, extra)).encode()))
    t = getattr(oracle, ptype)
    pages = []
    for k, x in enumerate(extra):
        n = 3000 + 1000 * k
        defs = (rng.random(n) > 0.3).astype(np.int16)
        nn = int(defs.sum())
        vals = rng.integers(0, 256, size=(nn + max(x, 0)) * es, dtype=np.uint8).tobytes()
        if x < 0:
            vals = vals[:len(vals) - es]  # one value short: EOF on this page
        elif k == 2 and x:
            vals += b"\x01"  # a section that is not a whole number of values
        pages.append(oracle.PageSpec(oracle.PAGE_DATA, oracle.level_encode(defs, 1) + vals, n, oracle.PLAIN))
    _same(oracle, ctx, t, pages, max_def=1, expect_ok=min(extra) >= 0)


def _leb_padded(x, nbytes):
    """x as a non-minimal LEB128 varint of exactly nbytes bytes (the reference's reader accepts
    them, bit_util.rs get_vlq_int; the level path's fast parse takes up to 4 bytes)."""
    out = []
    for i in range(nbytes):
        b = (x >> (7 * i)) & 0x7F
        out.append(b | (0x80 if i < nbytes - 1 else 0))
    return bytes(out)


@pytest.mark.gpu
@pytest.mark.parametrize("nbytes", [5, 7, 10])
def test_level_streams_the_level_path_hands_back(oracle, ctx, nbytes):
    """Def-level streams whose first run header is a 5..10-byte varint: the level path hands the
    page back and the fallback kernel (index walk + tile expand + non-null count, one workgroup
    per page) decodes it; the page's non-null count places the PLAIN values of every later page.
    Pages taken by the level path are mixed in."""
    rng = np.random.default_rng(nbytes)
    pages = []
    for k in range(6):
        n = 5000 + 731 * k
        defs = (rng.random(n) > 0.25).astype(np.int16)
        if k % 2 == 0:  # an RLE run of 300 ones with a padded header, then the writer's encoding
            defs[:300] = 1
            rest = oracle.rle_encode(defs[300:].astype(np.uint64), 1)
            body = _leb_padded(300 << 1, nbytes) + b"\x01" + rest
            lev = len(body).to_bytes(4, "little") + body
        else:
            lev = oracle.level_encode(defs, 1)
        nn = int(defs.sum())
        vals = rng.integers(-2 ** 31, 2 ** 31, size=nn, dtype=np.int64).astype(np.int32)
        pages.append(oracle.PageSpec(oracle.PAGE_DATA, lev + vals.tobytes(), n, oracle.PLAIN))
    _same(oracle, ctx, oracle.INT32, pages, max_def=1)


@pytest.mark.gpu
@pytest.mark.parametrize("long_run", [3000, 70000, 200000])
def test_dense_level_windows_with_long_runs(oracle, ctx, long_run):
    """Dense one-bit def-level streams (10% nulls: a header every few bytes, the window path) with
    one long RLE run in the middle: the window holding it writes tens of thousands of outputs
    from one run among hundreds of short ones. Runs of ones and of zeros; a dense page without a
    long run after them."""
    rng = np.random.default_rng(long_run)
    pages = []
    for k in range(4):
        d1 = (rng.random(8 * (2500 + 125 * k)) > 0.1).astype(np.int16)
        d3 = (rng.random(8 * 1875) > 0.1).astype(np.int16)
        d1[-16:] = 1  # the prefix's encoding ends in an RLE run (no padded bit-packed group)
        if k == 3:  # a dense page without a long run
            defs = np.concatenate([d1, d3])
            lev = oracle.level_encode(defs, 1)
        else:
            v = k % 2
            body = (oracle.rle_encode(d1.astype(np.uint64), 1) + _leb_padded(long_run << 1, 3) + bytes([v]) +
                    oracle.rle_encode(d3.astype(np.uint64), 1))
            defs = np.concatenate([d1, np.full(long_run, v, np.int16), d3])
            lev = len(body).to_bytes(4, "little") + body
        n = len(defs)
        nn = int(defs.sum())
        vals = rng.integers(-2 ** 31, 2 ** 31, size=nn, dtype=np.int64).astype(np.int32)
        pages.append(oracle.PageSpec(oracle.PAGE_DATA, lev + vals.tobytes(), n, oracle.PLAIN))
    _same(oracle, ctx, oracle.INT32, pages, max_def=1)


@pytest.mark.parametrize("shape", [(512, 4), (128, 4)])
@pytest.mark.parametrize("ptype", ["INT32", "INT64"])
def test_delta_bench_pages_lookback(oracle, ctx, ptype, shape):
    """Config 4's pages at the bench shape and at the reference writer's default (128 / 4 x 32,
    encoding.rs:508-509), several pages of 2^20 values and a ragged one, from the bench's own
    generator: every tile of every page goes through the header pass (k_delta_hdr) and the
    look-back tile kernel (k_delta_lb), whose running values chain across 256 tiles per page."""
    import ctypes as C

    import pqgpu
    import pqgtools
    L = pqgtools.lib()
    info = pqgtools.WorkloadInfo()
    n, page = 3 * (1 << 20) + 77_777, 1 << 20
    bits = 16 if ptype == "INT64" else 12
    assert L.pqg_gen_delta_int64(n, bits, page, shape[0], shape[1], 0x5EED0004, 8, None, 0, None, 0, C.byref(info)) == 0
    host = np.zeros(info.blob_len + 64, np.uint8)
    pages = (pqgpu.Page * info.npages)()
    assert L.pqg_gen_delta_int64(n, bits, page, shape[0], shape[1], 0x5EED0004, 8, host.ctypes.data_as(C.c_void_p),
                                 info.blob_len, pages, info.npages, C.byref(info)) == 0
    specs = [oracle.PageSpec(p.page_type, host[p.offset:p.offset + p.nbytes].tobytes(), p.num_values, p.encoding)
             for p in (pages[i] for i in range(info.npages))]
    t = getattr(oracle, ptype)
    if ptype == "INT32":  # the generator writes INT64 pages: re-encode the same values as INT32
        vals = oracle.read_column(oracle.INT64, specs)["values"].astype(np.int32)
        specs, o = [], 0
        for i in range(info.npages):
            k = pages[i].num_values
            specs.append(oracle.PageSpec(oracle.PAGE_DATA, oracle.delta_encode(t, vals[o:o + k], *shape), k,
                                         oracle.DELTA_BINARY_PACKED))
            o += k
    got, ref = _same(oracle, ctx, t, specs)
    assert got["num_values"] == n


@pytest.mark.parametrize("misalign", [1, 3, 8, 13])
def test_unaligned_payloads(oracle, ctx, misalign):
    """The C ABI takes any payload offset (pqgpu.h pqg_page.offset): every page here starts
    `misalign` bytes past a 64-byte boundary. Windowed dictionary gathers (5 000 INT64 / 3 000
    INT32 entries: the window realigned in LDS), PLAIN copies, DELTA and byte arrays."""
    import pqgpu
    rng = np.random.default_rng(500 + misalign)
    cases = []
    for ptype, dt, nd in (("INT64", np.int64, 5000), ("INT32", np.int32, 3000)):
        t = getattr(oracle, ptype)
        dvals = np.unique(rng.integers(-2**30, 2**30, 2 * nd).astype(dt))[:nd]
        bw = int(np.ceil(np.log2(len(dvals))))
        pages = [oracle.PageSpec(oracle.PAGE_DICTIONARY, dvals.tobytes(), len(dvals), oracle.PLAIN)]
        for n in (50000, 4099):
            body = bytes([bw]) + _hybrid(rng.integers(0, len(dvals), n), bw)
            pages.append(oracle.PageSpec(oracle.PAGE_DATA, body, n, oracle.RLE_DICTIONARY))
        cases.append((t, pages, pqgpu.PATH_DICT_WINDOW))
    v = rng.integers(-2**31, 2**31, 30001, dtype=np.int64).astype(np.int32)
    cases.append((oracle.INT32, [oracle.PageSpec(oracle.PAGE_DATA, v.tobytes(), len(v), oracle.PLAIN)],
                  pqgpu.PATH_PLAIN))
    v = _delta_values(rng, np.int64, 20001, "d16")
    cases.append((oracle.INT64, [oracle.PageSpec(oracle.PAGE_DATA, oracle.delta_encode(oracle.INT64, v, 512, 4),
                                                 len(v), oracle.DELTA_BINARY_PACKED)], pqgpu.PATH_DELTA))
    for t, pages, path in cases:
        ref = oracle.read_column(t, pages)
        got = pqgpu.decode_column(ctx, t, pages, misalign=misalign)
        assert ref["status"] == 0 and got["status"] == 0, (got["message"], ref["message"])
        assert ctx.last_paths() & path, (path, ctx.last_paths())
        assert got["values"].tobytes() == ref["values"].tobytes()
