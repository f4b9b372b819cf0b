"""Producer -> consumer kernel pairs on malformed input (fault-class audit).

A chunk's status is read only when the decode is synced, so every kernel after a failing stage
still runs: it must never follow scratch the failed stage did not write. Each pair gets one
malformed page (the failing stage) beside well-formed ones (whose later kernels run), and the
result must be the oracle's: the same status, the same failing page, no device fault.

  (1) DELTA_BYTE_ARRAY: k_ba_index (prefix and suffix streams -> per-value prefix / source /
      length) -> k_scan_bytes -> k_dba_copy (the prefix rebuild), decoding.rs:722-835;
  (2) fixed-width dictionary: k_prepare's dictionary check -> the level path's dictionary emit
      (LvDictOut: the dictionary copied into LDS) / k_dict_fallback, decoding.rs:282-309;
  (3) DELTA_BINARY_PACKED: k_delta_page (the per-page pass, which hands a page back at the first
      irregular block) -> k_delta_index / k_delta_sums / k_delta_expand -> k_delta_rest,
      decoding.rs:448-572;
  (4) byte-array dictionary: k_ba_dict_prep -> k_ba_copy / k_ba_copy_sd (covered by
      test_gpu_bytes.py::test_truncated_dictionary_page_ba; here with a nullable page on the
      level path's small-dictionary copy)."""
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


def _same_error(oracle, ctx, ptype, pages, **kw):
    import pqgpu
    ref = oracle.read_column(ptype, pages, **kw)
    got = pqgpu.decode_column(ctx, ptype, pages, **kw)
    assert ref["status"] != 0, "the malformed page must fail in the reference"
    assert got["status"] == ref["status"], (got["message"], ref["message"])
    return got, ref


def _opt(oracle, n, body_of, encoding, rng, p_null=0.2):
    lv = (rng.random(n) >= p_null).astype(np.int16)
    return oracle.PageSpec(oracle.PAGE_DATA, oracle.level_encode(lv, 1) + body_of(int(lv.sum())), n, encoding)


def _strings(rng, n, lo=0, hi=40):
    a = np.frombuffer(b"abcdefghij", np.uint8)
    return [bytes(a[rng.integers(0, 10, l)]) for l in rng.integers(lo, hi + 1, n)]


# ---- (1) DELTA_BYTE_ARRAY prefix rebuild

@pytest.mark.parametrize("cut", ["suffix_data", "suffix_lengths"])
def test_dba_failed_index_then_good_pages(oracle, ctx, cut):
    """Page 1's suffix section is cut (its bytes, or inside its length stream): k_ba_index fails
    there with no per-value scratch written; the good pages before and after still run the byte
    scan and the prefix rebuild."""
    rng = np.random.default_rng(21)

    def dba(n):
        return oracle.delta_byte_array_encode(sorted(_strings(rng, n, 5, 30)))

    good0 = _opt(oracle, 3000, dba, oracle.DELTA_BYTE_ARRAY, rng)
    vals = sorted(_strings(rng, 2000, 5, 30))
    pre = oracle.delta_encode(oracle.INT32, np.zeros(len(vals), np.int32))
    suf = oracle.delta_length_encode(vals)
    body = pre + (suf[:-7] if cut == "suffix_data" else suf[:12])
    bad = oracle.PageSpec(oracle.PAGE_DATA, body, len(vals), oracle.DELTA_BYTE_ARRAY)
    good2 = _opt(oracle, 4000, dba, oracle.DELTA_BYTE_ARRAY, rng)
    _same_error(oracle, ctx, oracle.BYTE_ARRAY, [good0, bad, good2], max_def=1)


# ---- (2) fixed-width dictionary emit after a bad dictionary page

@pytest.mark.parametrize("ptype,nd", [("INT64", 200), ("INT32", 40), ("INT64", 5000)])
@pytest.mark.parametrize("p_null", [0.0, 0.3])
def test_truncated_fixed_dictionary_then_data_pages(oracle, ctx, ptype, nd, p_null):
    """A PLAIN dictionary page holding fewer bytes than num_values entries (DictDecoder::set_dict
    fails, decoding.rs:282-288) followed by long data pages: small dictionaries are the level
    path's (its emit copies the dictionary into LDS), 5000 entries the general decoder's."""
    rng = np.random.default_rng(22)
    t = getattr(oracle, ptype)
    dt = np.int64 if ptype == "INT64" else np.int32
    dvals = np.unique(rng.integers(-2**30, 2**30, nd * 2).astype(dt))[:nd]
    dbytes = dvals.tobytes()[: len(dvals) * dvals.itemsize // 3]
    dpage = oracle.PageSpec(oracle.PAGE_DICTIONARY, dbytes, len(dvals), oracle.PLAIN)
    bw = max(1, int(np.ceil(np.log2(len(dvals)))))

    def idx(n):
        return bytes([bw]) + oracle.rle_encode(rng.integers(0, len(dvals), n).astype(np.uint64), bw)

    pages = [dpage] + [_opt(oracle, n, idx, oracle.RLE_DICTIONARY, rng, p_null) for n in (70_000, 300)]
    _same_error(oracle, ctx, t, pages, max_def=1)


def test_truncated_small_ba_dictionary_nullable(oracle, ctx):
    """(4) A byte-array dictionary of short strings (the level path's small-dictionary copy,
    k_ba_copy_sd) cut short: every entry is left empty by k_ba_dict_prep, nothing follows a
    stale entry."""
    rng = np.random.default_rng(23)
    d = list(dict.fromkeys(_strings(rng, 300, 1, 12)))
    dpage = oracle.PageSpec(oracle.PAGE_DICTIONARY, oracle.plain_encode_ba(d)[:-5], len(d), oracle.PLAIN)
    bw = max(1, int(np.ceil(np.log2(len(d)))))

    def idx(n):
        return bytes([bw]) + oracle.rle_encode(rng.integers(0, len(d), n).astype(np.uint64), bw)

    pages = [dpage] + [_opt(oracle, n, idx, oracle.RLE_DICTIONARY, rng) for n in (50_000, 7)]
    _same_error(oracle, ctx, oracle.BYTE_ARRAY, pages, max_def=1)


@pytest.mark.parametrize("nd", [300, 60000])
def test_failing_ba_dictionary_after_stale_in_range_indices(oracle, ctx, nd):
    """The per-value index slots are scratch reused across decodes. Two good decodes (one per
    context slot) first fill them with in-range indices of another dictionary; then a chunk whose
    dictionary page is cut decodes. No kernel may read those slots (dict_usable: the producers
    skip the chunk's data pages, so the consumers do too): the status is the oracle's, and a good
    decode afterwards is still exact."""
    import pqgpu
    rng = np.random.default_rng(24)
    d = list(dict.fromkeys(_strings(rng, nd + nd // 2, 4, 16)))[:nd]
    bw = max(1, int(np.ceil(np.log2(len(d)))))

    def idx(n):
        return bytes([bw]) + oracle.rle_encode(rng.integers(0, len(d), n).astype(np.uint64), bw)

    good = [oracle.PageSpec(oracle.PAGE_DICTIONARY, oracle.plain_encode_ba(d), len(d), oracle.PLAIN)]
    good += [_opt(oracle, n, idx, oracle.RLE_DICTIONARY, rng) for n in (90_000, 40_000)]
    ref_good = oracle.read_column(oracle.BYTE_ARRAY, good, max_def=1)
    for _ in range(2):
        got = pqgpu.decode_column(ctx, oracle.BYTE_ARRAY, good, max_def=1)
        assert got["status"] == 0 and got["bytes"] == ref_good["bytes"]
    bad = [oracle.PageSpec(oracle.PAGE_DICTIONARY, oracle.plain_encode_ba(d)[:-3], len(d), oracle.PLAIN)]
    bad += [_opt(oracle, n, idx, oracle.RLE_DICTIONARY, rng) for n in (90_000, 40_000)]
    for _ in range(2):
        _same_error(oracle, ctx, oracle.BYTE_ARRAY, bad, max_def=1)
    got = pqgpu.decode_column(ctx, oracle.BYTE_ARRAY, good, max_def=1)
    assert got["status"] == 0 and got["bytes"] == ref_good["bytes"]
    np.testing.assert_array_equal(got["offsets"], ref_good["offsets"])


# ---- (3) DELTA_BINARY_PACKED page pass -> tiled fallback

def _delta_blocks(buf):
    """Stream offsets of each block's (min delta, bit widths) in a DELTA_BINARY_PACKED page
    (header: block size, mini-blocks, total, first value; decoding.rs:501-533, 535-572)."""
    def vlq(i):
        v = s = 0
        while True:
            b = buf[i]
            i += 1
            v |= (b & 0x7F) << s
            s += 7
            if not b & 0x80:
                return v, i
    bs, i = vlq(0)
    nmb, i = vlq(i)
    total, i = vlq(i)
    _, i = vlq(i)
    vpmb = bs // nmb
    out, left = [], total - 1
    while left > 0 and i < len(buf):
        _, j = vlq(i)  # min delta
        widths = list(buf[j:j + nmb])
        out.append((i, j))
        i = j + nmb + sum(vpmb * w // 8 for w in widths)
        left -= bs
    return out


@pytest.mark.parametrize("es", [4, 8])
@pytest.mark.parametrize("what", ["width", "truncated"])
def test_delta_page_pass_hands_back_a_bad_block(oracle, ctx, es, what):
    """A 20 000-value DELTA page whose 70th block (the third 4096-delta tile of k_delta_page) has a
    bit width wider than the type, or whose payload is cut inside that tile: k_delta_page has
    already written the first tiles when it hands the page to the tiled path, which must report
    the reference's error; a good page after it decodes in the page pass."""
    rng = np.random.default_rng(24 + es)
    t = oracle.INT64 if es == 8 else oracle.INT32
    dt = np.int64 if es == 8 else np.int32
    v = np.cumsum(rng.integers(-2**12, 2**12, 20_000)).astype(dt)
    body = bytearray(oracle.delta_encode(t, v))
    blocks = _delta_blocks(body)
    b = blocks[70]
    if what == "width":
        body[b[1]] = 8 * es + 1
    else:
        body = body[:b[1] + 40]
    bad = oracle.PageSpec(oracle.PAGE_DATA, bytes(body), len(v), oracle.DELTA_BINARY_PACKED)
    good = oracle.PageSpec(oracle.PAGE_DATA, oracle.delta_encode(t, v[:9000]), 9000, oracle.DELTA_BINARY_PACKED)
    import pqgpu
    ref = oracle.read_column(t, [good, bad, good])
    got = pqgpu.decode_column(ctx, t, [good, bad, good])
    assert got["status"] == ref["status"], (got["message"], ref["message"])
    if ref["status"] == 0:  # (a width the reference accepts: every value must match)
        np.testing.assert_array_equal(got["values"], ref["values"])
