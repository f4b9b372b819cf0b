"""GPU parity for BYTE_ARRAY / FIXED_LEN_BYTE_ARRAY columns against the C oracle: PLAIN
(decoding.rs:206-247), dictionary (:256-315), DELTA_LENGTH_BYTE_ARRAY (:629-712) and
DELTA_BYTE_ARRAY (:722-835), including the error classes the reference raises."""
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


def rand_strings(rng, n, lo=0, hi=40, alphabet=b"abcdefghij"):
    lens = rng.integers(lo, hi + 1, n)
    a = np.frombuffer(alphabet, np.uint8)
    return [bytes(a[rng.integers(0, len(a), l)]) for l in lens]


def sorted_strings(rng, n):
    """Shared prefixes, the case DELTA_BYTE_ARRAY exists for."""
    base = [b"http://www.example.com/" + b"/".join(rand_strings(rng, 3, 1, 6)) for _ in range(n)]
    return sorted(base)


def check(oracle, ctx, ptype, pages, max_def=0, type_length=-1, expect=0):
    import pqgpu
    ref = oracle.read_column(ptype, pages, max_def=max_def, type_length=type_length)
    got = pqgpu.decode_column(ctx, ptype, pages, max_def=max_def, type_length=type_length)
    assert ref["status"] == expect, ref["message"]
    assert got["status"] == expect, got["message"]
    if expect:
        return got, ref
    if max_def:
        np.testing.assert_array_equal(got["def"], ref["def"])
    assert got["num_values"] == len(ref["values"])
    assert got["bytes"] == ref["bytes"]
    np.testing.assert_array_equal(got["offsets"], ref["offsets"])
    return got, ref


def optional_pages(oracle, rng, sizes, p_null, make_values, encode, encoding, v2=False):
    pages = []
    for n in sizes:
        lv = (rng.random(n) >= p_null).astype(np.int16)
        vals = make_values(int(lv.sum()))
        body = encode(vals)
        if v2:
            lev = oracle.level_encode(lv, 1, oracle.RLE, v2=True)
            pages.append(oracle.PageSpec(oracle.PAGE_DATA_V2, lev + body, n, encoding, def_len=len(lev)))
        else:
            lev = oracle.level_encode(lv, 1)
            pages.append(oracle.PageSpec(oracle.PAGE_DATA, lev + body, n, encoding))
    return pages


@pytest.mark.parametrize("p_null", [0.0, 0.3, 1.0])
def test_plain_byte_array(oracle, ctx, p_null):
    rng = np.random.default_rng(1)
    pages = optional_pages(oracle, rng, [1, 100, 5000, 20000], p_null,
                           lambda n: rand_strings(rng, n), oracle.plain_encode_ba, oracle.PLAIN)
    check(oracle, ctx, oracle.BYTE_ARRAY, pages, max_def=1)


def test_plain_byte_array_long_values(oracle, ctx):
    rng = np.random.default_rng(2)
    vals = rand_strings(rng, 300, 0, 70000)
    pages = [oracle.PageSpec(oracle.PAGE_DATA, oracle.plain_encode_ba(vals), len(vals), oracle.PLAIN)]
    check(oracle, ctx, oracle.BYTE_ARRAY, pages)


@pytest.mark.parametrize("tl", [1, 12, 16, 37])
def test_plain_flba(oracle, ctx, tl):
    rng = np.random.default_rng(tl)
    pages = optional_pages(oracle, rng, [10, 3000], 0.2, lambda n: rand_strings(rng, n, tl, tl),
                           lambda v: oracle.plain_encode_ba(v, fixed=True), oracle.PLAIN)
    check(oracle, ctx, oracle.FIXED_LEN_BYTE_ARRAY, pages, max_def=1, type_length=tl)


def _dict_pages(oracle, rng, ptype, distinct, sizes, p_null, fixed=False, v2=False):
    dict_vals = list(dict.fromkeys(distinct))
    dpage = oracle.PageSpec(oracle.PAGE_DICTIONARY, oracle.plain_encode_ba(dict_vals, fixed=fixed),
                            len(dict_vals), oracle.PLAIN)
    bw = max(1, int(np.ceil(np.log2(len(dict_vals)))))

    def enc(vals):
        return bytes([bw]) + oracle.rle_encode(np.array(vals, np.uint64), bw)

    pages = optional_pages(oracle, rng, sizes, p_null,
                           lambda n: rng.integers(0, len(dict_vals), n).tolist(), enc,
                           oracle.RLE_DICTIONARY, v2=v2)
    return [dpage] + pages


def test_dictionary_byte_array(oracle, ctx):
    rng = np.random.default_rng(3)
    pages = _dict_pages(oracle, rng, oracle.BYTE_ARRAY, rand_strings(rng, 500, 0, 30), [100, 7000, 1], 0.25)
    check(oracle, ctx, oracle.BYTE_ARRAY, pages, max_def=1)


def _leb_padded(x, nbytes):
    """x as a non-minimal LEB128 varint of nbytes bytes (bit_util.rs get_vlq_int accepts it; the
    level path's fast parse takes up to 4 bytes)."""
    return bytes(((x >> (7 * i)) & 0x7F) | (0x80 if i < nbytes - 1 else 0) for i in range(nbytes))


@pytest.mark.parametrize("nbytes", [5, 9])
def test_dictionary_byte_array_pages_handed_back(oracle, ctx, nbytes):
    """A small byte-array dictionary (the level path's dictionary emit) over pages of which every
    other one holds a padded 5..10-byte RLE run header inside its index stream: the level path
    hands those pages back and the general decoder's fallback writes their indices and byte
    totals; the emitted pages' totals are their tiles' sums (PageWork::tile_bytes). Offsets and
    bytes of every page must be the oracle's."""
    import pqgpu
    rng = np.random.default_rng(40 + nbytes)
    d = list(dict.fromkeys(rand_strings(rng, 120, 1, 9)))[:80]
    dpage = oracle.PageSpec(oracle.PAGE_DICTIONARY, oracle.plain_encode_ba(d), len(d), oracle.PLAIN)
    bw = max(1, int(np.ceil(np.log2(len(d)))))
    pages = [dpage]
    for k in range(6):
        n = 6000 + 517 * k
        lv = (rng.random(n) >= 0.2).astype(np.int16)
        nn = int(lv.sum())
        idx = rng.integers(0, len(d), nn).astype(np.uint64)
        if k % 2 == 0:
            cut = (nn // 3) & ~7
            idx[cut - 16:cut] = idx[cut - 16]  # (the prefix's encoding ends in an RLE run)
            run = 200
            idx[cut:cut + run] = idx[cut]
            body = (bytes([bw]) + oracle.rle_encode(idx[:cut], bw) + _leb_padded(run << 1, nbytes) +
                    int(idx[cut]).to_bytes((bw + 7) // 8, "little") + oracle.rle_encode(idx[cut + run:], bw))
        else:
            body = bytes([bw]) + oracle.rle_encode(idx, bw)
        pages.append(oracle.PageSpec(oracle.PAGE_DATA, oracle.level_encode(lv, 1) + body, n, oracle.RLE_DICTIONARY))
    check(oracle, ctx, oracle.BYTE_ARRAY, pages, max_def=1)
    assert ctx.last_paths() & pqgpu.PATH_DICT_LEVEL, "the small dictionary takes the level path"


def test_dictionary_flba_v2(oracle, ctx):
    rng = np.random.default_rng(4)
    pages = _dict_pages(oracle, rng, oracle.FIXED_LEN_BYTE_ARRAY, rand_strings(rng, 300, 16, 16),
                        [4000, 900], 0.1, fixed=True, v2=True)
    check(oracle, ctx, oracle.FIXED_LEN_BYTE_ARRAY, pages, max_def=1, type_length=16)


@pytest.mark.parametrize("p_null", [0.0, 0.4])
def test_delta_length_byte_array(oracle, ctx, p_null):
    rng = np.random.default_rng(5)
    pages = optional_pages(oracle, rng, [1, 129, 6000, 30000], p_null,
                           lambda n: rand_strings(rng, n, 0, 50), oracle.delta_length_encode,
                           oracle.DELTA_LENGTH_BYTE_ARRAY)
    check(oracle, ctx, oracle.BYTE_ARRAY, pages, max_def=1)


@pytest.mark.parametrize("p_null", [0.0, 0.4])
def test_delta_byte_array(oracle, ctx, p_null):
    rng = np.random.default_rng(6)
    pages = optional_pages(oracle, rng, [1, 200, 5000], p_null, lambda n: sorted_strings(rng, n),
                           oracle.delta_byte_array_encode, oracle.DELTA_BYTE_ARRAY, v2=True)
    check(oracle, ctx, oracle.BYTE_ARRAY, pages, max_def=1)


def test_delta_byte_array_long_values(oracle, ctx):
    """Values of any length (the reference builds a Vec per value, decoding.rs:794-822): 40 KiB
    and 1 MiB values sharing long prefixes, between short ones."""
    rng = np.random.default_rng(61)
    big = bytes(rng.integers(0, 256, 1 << 20, dtype=np.uint8))
    mid = bytes(rng.integers(0, 256, 40 << 10, dtype=np.uint8))
    vals = [b"a", mid, mid + b"x", mid[:30000] + b"yz", big, big[:700000] + mid, big + b"!", b"b",
            big[:5] + mid, mid + big]
    pages = [oracle.PageSpec(oracle.PAGE_DATA, oracle.delta_byte_array_encode(vals), len(vals),
                             oracle.DELTA_BYTE_ARRAY)]
    got, _ = check(oracle, ctx, oracle.BYTE_ARRAY, pages)
    offs = got["offsets"]
    assert [got["bytes"][offs[i]:offs[i + 1]] for i in range(len(vals))] == vals


def test_delta_byte_array_many_long_slices(oracle, ctx):
    """More long slices in one 4096-value tile than k_dba_copy queues (DBA_QCAP = 512 slices over
    DBA_LONG = 256 bytes; past that its per-lane copy): 600 values of ~1.1 KiB, each the previous
    value's first 400 bytes (one 400-byte slice back to value 0) and a fresh 700-byte suffix, so
    1200 long slices."""
    rng = np.random.default_rng(63)
    vals = [bytes(rng.integers(0, 256, 1100, dtype=np.uint8))]
    for _ in range(599):
        vals.append(vals[-1][:400] + bytes(rng.integers(0, 256, 700, dtype=np.uint8)))
    pages = [oracle.PageSpec(oracle.PAGE_DATA, oracle.delta_byte_array_encode(vals), len(vals),
                             oracle.DELTA_BYTE_ARRAY)]
    got, _ = check(oracle, ctx, oracle.BYTE_ARRAY, pages)
    offs = got["offsets"]
    assert [got["bytes"][offs[i]:offs[i + 1]] for i in range(len(vals))] == vals


def _prefix_chain_values(n):
    """Value i = 'a' * (i % 3000 + 1) and similar: prefix lengths rising by one, so every byte
    of a value comes from a different earlier suffix (chains as long as the values)."""
    return [b"a" * (i % 3000 + 1) + bytes([98 + (i % 3000 == 2999)]) for i in range(n)]


@pytest.mark.parametrize("shape", ["rising", "common_prefix", "million"])
def test_delta_byte_array_prefix_chains(oracle, ctx, shape):
    """Prefix-length shapes for the slice rebuild: prefix lengths rising by one (chains of
    thousands of slices), one 23-byte prefix shared by every value across many 4096-value tiles
    (each value's chain jumps back to value 0), and a 1 M-value page of sorted URL-like strings."""
    rng = np.random.default_rng(62)
    if shape == "rising":
        vals = _prefix_chain_values(7000)
    elif shape == "common_prefix":
        vals = [b"http://www.example.com/" + b"%07d" % int(x) for x in rng.integers(0, 10 ** 7, 50000)]
    else:
        xs = np.sort(rng.integers(0, 10 ** 12, 1 << 20))
        vals = [b"http://www.example.com/%d/%012d" % (x % 7, x) + b"/q" * int(x % 5) for x in xs]
    pages = [oracle.PageSpec(oracle.PAGE_DATA, oracle.delta_byte_array_encode(vals), len(vals),
                             oracle.DELTA_BYTE_ARRAY)]
    got, _ = check(oracle, ctx, oracle.BYTE_ARRAY, pages)
    assert got["bytes"] == b"".join(vals)


def test_delta_byte_array_flba(oracle, ctx):
    rng = np.random.default_rng(7)
    vals = sorted(rand_strings(rng, 3000, 10, 10, b"ab"))
    pages = [oracle.PageSpec(oracle.PAGE_DATA, oracle.delta_byte_array_encode(vals), len(vals),
                             oracle.DELTA_BYTE_ARRAY)]
    check(oracle, ctx, oracle.FIXED_LEN_BYTE_ARRAY, pages, type_length=10)


def test_mixed_encodings_in_one_chunk(oracle, ctx):
    """Dictionary pages, then fallback pages in other encodings (writer fallback)."""
    rng = np.random.default_rng(8)
    pages = _dict_pages(oracle, rng, oracle.BYTE_ARRAY, rand_strings(rng, 100), [3000], 0.2)
    pages += optional_pages(oracle, rng, [2000], 0.2, lambda n: rand_strings(rng, n), oracle.plain_encode_ba, oracle.PLAIN)
    pages += optional_pages(oracle, rng, [2000], 0.2, lambda n: rand_strings(rng, n), oracle.delta_length_encode,
                            oracle.DELTA_LENGTH_BYTE_ARRAY)
    pages += optional_pages(oracle, rng, [2000], 0.2, lambda n: sorted_strings(rng, n), oracle.delta_byte_array_encode,
                            oracle.DELTA_BYTE_ARRAY)
    check(oracle, ctx, oracle.BYTE_ARRAY, pages, max_def=1)


# ---- errors: same status class and page as the oracle

def _err(oracle, ctx, ptype, pages, **kw):
    import pqgpu
    ref = oracle.read_column(ptype, pages, **kw)
    got = pqgpu.decode_column(ctx, ptype, pages, **kw)
    assert ref["status"] != 0
    assert got["status"] == ref["status"], (got["message"], ref["message"])
    return got


def test_plain_ba_truncated_length_prefix(oracle, ctx):
    body = oracle.plain_encode_ba([b"abc", b"de"])[:-4]  # second value's length cut
    _err(oracle, ctx, oracle.BYTE_ARRAY, [oracle.PageSpec(oracle.PAGE_DATA, body, 2, oracle.PLAIN)])


def test_plain_ba_truncated_value(oracle, ctx):
    body = oracle.plain_encode_ba([b"abc", b"defgh"])[:-2]
    _err(oracle, ctx, oracle.BYTE_ARRAY, [oracle.PageSpec(oracle.PAGE_DATA, body, 2, oracle.PLAIN)])


def test_dlba_lengths_past_data(oracle, ctx):
    body = oracle.delta_length_encode([b"abcdef", b"ghijkl"])[:-3]
    _err(oracle, ctx, oracle.BYTE_ARRAY, [oracle.PageSpec(oracle.PAGE_DATA, body, 2, oracle.DELTA_LENGTH_BYTE_ARRAY)])


def test_dba_prefix_longer_than_previous(oracle, ctx):
    # prefix lengths [0, 9] with a 3-byte first value: previous_value[0..9] panics
    prefixes = oracle.delta_encode(oracle.INT32, np.array([0, 9], np.int32))
    suffixes = oracle.delta_length_encode([b"abc", b"x"])
    _err(oracle, ctx, oracle.BYTE_ARRAY, [oracle.PageSpec(oracle.PAGE_DATA, prefixes + suffixes, 2, oracle.DELTA_BYTE_ARRAY)])


def test_dba_suffix_reuse(oracle, ctx):
    """More prefixes than suffixes: the reference reuses the last suffix (decoding.rs:796-801)."""
    prefixes = oracle.delta_encode(oracle.INT32, np.array([0, 1, 2], np.int32))
    suffixes = oracle.delta_length_encode([b"ab"])
    pages = [oracle.PageSpec(oracle.PAGE_DATA, prefixes + suffixes, 3, oracle.DELTA_BYTE_ARRAY)]
    got, ref = check(oracle, ctx, oracle.BYTE_ARRAY, pages)
    assert ref["values"] == [b"ab", b"aab", b"aaab"]


def test_bad_dictionary_index_ba(oracle, ctx):
    dpage = oracle.PageSpec(oracle.PAGE_DICTIONARY, oracle.plain_encode_ba([b"a", b"b"]), 2, oracle.PLAIN)
    body = bytes([2]) + oracle.rle_encode(np.array([0, 3, 1], np.uint64), 2)
    _err(oracle, ctx, oracle.BYTE_ARRAY, [dpage, oracle.PageSpec(oracle.PAGE_DATA, body, 3, oracle.RLE_DICTIONARY)])


def test_truncated_dictionary_page_ba(oracle, ctx):
    dbytes = oracle.plain_encode_ba([b"abc", b"defg"])[:-1]
    dpage = oracle.PageSpec(oracle.PAGE_DICTIONARY, dbytes, 2, oracle.PLAIN)
    body = bytes([1]) + oracle.rle_encode(np.array([0, 1], np.uint64), 1)
    _err(oracle, ctx, oracle.BYTE_ARRAY, [dpage, oracle.PageSpec(oracle.PAGE_DATA, body, 2, oracle.RLE_DICTIONARY)])


@pytest.mark.parametrize("odd", [None, 0, 2500, 4999])
def test_plain_byte_array_one_length(oracle, ctx, odd):
    """Values of one length take the workgroup's fixed-stride check instead of the chain walk;
    one value of another length (first, middle, last) sends the page back to the walk."""
    rng = np.random.default_rng(11)
    vals = rand_strings(rng, 5000, 8, 8)
    if odd is not None:
        vals[odd] = vals[odd] + b"x"
    pages = [oracle.PageSpec(oracle.PAGE_DATA, oracle.plain_encode_ba(vals), len(vals), oracle.PLAIN)]
    check(oracle, ctx, oracle.BYTE_ARRAY, pages)


def test_dictionary_byte_array_one_length(oracle, ctx):
    rng = np.random.default_rng(12)
    pages = _dict_pages(oracle, rng, oracle.BYTE_ARRAY, rand_strings(rng, 700, 8, 8), [3000, 9000], 0.2)
    check(oracle, ctx, oracle.BYTE_ARRAY, pages, max_def=1)


@pytest.mark.parametrize("cut", [1, 4, 9])
def test_plain_ba_one_length_truncated(oracle, ctx, cut):
    """Equal lengths but the section cut short: the fixed-stride check fails and the walk reports
    the reference's error (panic on a cut length, EOF on cut bytes)."""
    body = oracle.plain_encode_ba([b"abcdefgh"] * 50)[:-cut]
    _err(oracle, ctx, oracle.BYTE_ARRAY, [oracle.PageSpec(oracle.PAGE_DATA, body, 50, oracle.PLAIN)])


# ------------------------------------------------------------------ large pages: pqg_balen.hpp
def _prefixes(vals):
    import os.path
    pre, prev = [], b""
    for v in vals:
        pre.append(len(os.path.commonprefix([prev, v])))
        prev = v
    return pre


def _dba_body(oracle, vals, shape=(128, 4), pre=None, suf=None):
    """DELTA_BYTE_ARRAY with the length streams in a chosen block shape (prefix / suffix lengths
    may be given to write malformed pages)."""
    pre = _prefixes(vals) if pre is None else pre
    sufs = [v[k:] for v, k in zip(vals, pre)] if suf is None else suf
    return (oracle.delta_encode(oracle.INT32, np.array(pre, np.int32), *shape) +
            oracle.delta_encode(oracle.INT32, np.array([len(s) for s in sufs], np.int32), *shape) + b"".join(sufs))


def _dlba_body(oracle, vals, shape=(128, 4), lens=None):
    lens = [len(v) for v in vals] if lens is None else lens
    return oracle.delta_encode(oracle.INT32, np.array(lens, np.int32), *shape) + b"".join(vals)


@pytest.mark.parametrize("shape", [(128, 4), (256, 8), (512, 4), (4096, 8), (1024, 1), (64, 2)])
def test_large_length_streams(oracle, ctx, shape):
    """Pages of at least 65536 values (BL_MIN): their length streams decoded by the multi-workgroup
    kernels (k_bl_walk's block chain, per-tile sums, scans and expands, pqg_balen.hpp) for block
    shapes the decoder accepts (decoding.rs:501-533); blocks of 64 values are not that path's
    shape and stay with k_ba_index. DELTA_LENGTH_BYTE_ARRAY (random lengths 0..40) and
    DELTA_BYTE_ARRAY (sorted strings with shared prefixes), every byte and offset against the
    oracle."""
    rng = np.random.default_rng(70 + shape[0] + shape[1])
    vals = rand_strings(rng, 150_000, 0, 40)
    p = oracle.PageSpec(oracle.PAGE_DATA, _dlba_body(oracle, vals, shape), len(vals), oracle.DELTA_LENGTH_BYTE_ARRAY)
    check(oracle, ctx, oracle.BYTE_ARRAY, [p])
    svals = sorted_strings(rng, 100_000)
    p = oracle.PageSpec(oracle.PAGE_DATA, _dba_body(oracle, svals, shape), len(svals), oracle.DELTA_BYTE_ARRAY)
    got, _ = check(oracle, ctx, oracle.BYTE_ARRAY, [p])
    assert got["values"][:3] == svals[:3] and got["values"][-1] == svals[-1]


def test_large_length_streams_optional(oracle, ctx):
    """Nullable pages: 100 000 levels of which ~80 000 values, so the page's value count (its
    non-null levels) decides the path, beside a small page (k_ba_index) in the same chunk."""
    rng = np.random.default_rng(80)
    for enc, encode in ((oracle.DELTA_LENGTH_BYTE_ARRAY, lambda v: _dlba_body(oracle, v)),
                        (oracle.DELTA_BYTE_ARRAY, lambda v: _dba_body(oracle, v))):
        pages = optional_pages(oracle, rng, (100_000, 3000, 90_000), 0.2,
                               lambda k: sorted_strings(rng, k), encode, enc)
        check(oracle, ctx, oracle.BYTE_ARRAY, pages, max_def=1)


@pytest.mark.parametrize("case", ["negative_length", "past_data", "prefix_too_long", "negative_prefix",
                                  "short_suffix_stream", "count_mismatch"])
def test_large_length_streams_errors(oracle, ctx, case):
    """Malformed large pages: the multi-workgroup path hands the page back and k_ba_index reports
    what the reference reports (data.range's assert on a negative length or one past the data;
    previous_value[0..prefix_len] past the previous value, decoding.rs:804; a suffix stream with
    fewer values than the prefix stream, :796-801; a length stream whose count is not the page's)."""
    rng = np.random.default_rng(90)
    n = 80_000
    if case in ("negative_length", "past_data", "count_mismatch"):
        vals = rand_strings(rng, n, 1, 30)
        lens = [len(v) for v in vals]
        if case == "negative_length":
            lens[70_001] = -3
        body = _dlba_body(oracle, vals, lens=lens)
        if case == "past_data":
            body = body[:-7]
        npage = n if case != "count_mismatch" else n + 5
        p = oracle.PageSpec(oracle.PAGE_DATA, body, npage, oracle.DELTA_LENGTH_BYTE_ARRAY)
    else:
        vals = sorted_strings(rng, n)
        pre = _prefixes(vals)
        sufs = [v[k:] for v, k in zip(vals, pre)]
        if case == "prefix_too_long":
            pre[66_000] = len(vals[65_999]) + 4
        if case == "negative_prefix":
            pre[75_000] = -1
        if case == "short_suffix_stream":
            sufs = sufs[:-3]
        p = oracle.PageSpec(oracle.PAGE_DATA, _dba_body(oracle, vals, pre=pre, suf=sufs), n, oracle.DELTA_BYTE_ARRAY)
    import pqgpu
    ref = oracle.read_column(oracle.BYTE_ARRAY, [p])
    got = pqgpu.decode_column(ctx, pqgpu.BYTE_ARRAY, [p])
    assert got["status"] == ref["status"], (case, got["message"], ref["message"])
    if ref["status"] == 0:
        assert got["bytes"] == ref["bytes"]
        np.testing.assert_array_equal(got["offsets"], ref["offsets"])
