"""Full-size parity of the level path's multi-segment shapes and of a config-5 row group.

- The headline shape: 2^20-level pages from the bench's own generator (pqg_gen_levels_plain,
  reference RleEncoder, rle.rs:152-316) at p_null 0.5 (every page ~134 KB of level stream: ~8
  segments of 16 KiB through k_lv_bound -> k_lv_segwalk -> k_lv_segscan), 0.1 and 0.05 (dense
  streams: the window path) and 0, against the oracle's read_batch concatenation
  (column/reader.rs:159-265, rle.rs:398-434).
- Crafted sparse streams whose segment starts k_lv_bound cannot place on the true header chain:
  payload bytes that are themselves a chain of valid headers (a "decoy" track) outvote the true
  chain, so the segment walks never land on their successor and k_lv_segscan's serial fallback
  (and past LW_SCAP runs, the window path) decides the page; and a segment whose first window has
  no exit of the writer's form (LV_BX_NONE -> LS_NOSTART).
- One config-5 row group at the bench's size (2^23 rows, dictionary columns are single 8 M-value
  pages: k_lv_stitch over ~11 chunks of window tables) against the generator's cells.
"""
import numpy as np
import pytest

import pqgtools

pytestmark = pytest.mark.gpu

PAGE = 1 << 20


@pytest.fixture(scope="module")
def ctx():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    import pqgpu
    c = pqgpu.Context(0)
    yield c
    c.close()


def _gen_levels_plain(n, p_null, seed):
    import ctypes as C

    import pqgpu
    L = pqgtools.lib()
    info = pqgtools.WorkloadInfo()
    assert L.pqg_gen_levels_plain(n, p_null, PAGE, seed, 8, None, 0, None, 0, C.byref(info)) == 0
    host = np.zeros(info.blob_len + 64, np.uint8)
    pages = (pqgpu.Page * info.npages)()
    assert L.pqg_gen_levels_plain(n, p_null, PAGE, seed, 8, host.ctypes.data_as(C.c_void_p), info.blob_len,
                                  pages, info.npages, C.byref(info)) == 0
    return host, pages, info


def _specs(oracle, host, pages, n):
    return [oracle.PageSpec(p.page_type, host[p.offset:p.offset + p.nbytes].tobytes(), p.num_values, p.encoding,
                            p.def_encoding, p.rep_encoding, p.def_len, p.rep_len)
            for p in (pages[i] for i in range(n))]


def _check(oracle, ctx, specs, max_def=1):
    import pqgpu
    ref = oracle.read_column(oracle.INT32, specs, max_def=max_def, batch_size=1024)
    got = pqgpu.decode_column(ctx, pqgpu.INT32, specs, max_def=max_def)
    assert ref["status"] == 0, ref["message"]
    assert got["status"] == 0, got["message"]
    np.testing.assert_array_equal(got["def"], ref["def"])
    assert got["num_values"] == len(ref["values"])
    np.testing.assert_array_equal(got["values"], ref["values"])
    return got, ref


@pytest.mark.parametrize("p_null", [0.5, 0.3, 0.2, 0.1, 0.05, 0.0])
def test_headline_pages_full_size(oracle, ctx, p_null):
    """Six 2^20-level pages and a ragged seventh, written by the bench's generator at the bench's
    seed, against the oracle: every level and every value. p_null 0.2-0.3: dense windows whose
    speculative chain walk needs several repair rounds or falls back to the serial walk (payload
    bytes parsed out of phase for a whole window); p_null 0: one RLE run per page, its outputs
    written by 16 waves per window in slices."""
    n = 6 * PAGE + 12345
    host, pages, info = _gen_levels_plain(n, p_null, 0x5EED0002 + int(p_null * 1000))
    assert info.npages == 7
    if p_null == 0.5:  # the multi-segment sparse walk: > 8 segments of 16 KiB per page
        assert min(pages[i].nbytes for i in range(6)) > 8 * 16384
    _check(oracle, ctx, _specs(oracle, host, pages, info.npages))


def test_dictionary_pages_bench_shape(oracle, ctx):
    """Config 3's page shape (bench.py `dict`): a 65 536-entry INT64 dictionary page and 2^20-index
    data pages of bit width 16, written by the bench's own generator (pqg_gen_dict_int64: reference
    DictEncoder + RleEncoder, rle.rs:152-316), four full pages and a ragged fifth, against the
    oracle's read_batch (get_batch_with_dict, rle.rs:437-487; DictDecoder, decoding.rs:282-309):
    every value. This is the windowed dictionary path the benchmark times (k_run_index's 64-run
    fast-forward, k_tile_desc, then k_dict_win: each workgroup decodes its 8 tiles' indices from
    their run records and payload in LDS and gathers them through 128 KiB dictionary windows);
    the test asserts that this path ran (pqg_ctx_last_paths)."""
    import ctypes as C

    import pqgpu
    L = pqgtools.lib()
    n = 4 * PAGE + 54321
    info = pqgtools.WorkloadInfo()
    seed = 0x5EED0003
    assert L.pqg_gen_dict_int64(n, 65536, PAGE, seed, 8, None, 0, None, 0, C.byref(info)) == 0
    host = np.zeros(info.blob_len + 64, np.uint8)
    pages = (pqgpu.Page * info.npages)()
    assert L.pqg_gen_dict_int64(n, 65536, PAGE, seed, 8, host.ctypes.data_as(C.c_void_p), info.blob_len, pages,
                                info.npages, C.byref(info)) == 0
    assert info.npages == 6 and pages[0].page_type == oracle.PAGE_DICTIONARY and pages[0].num_values == 65536
    assert host[pages[1].offset] == 16  # the data page's bit width byte
    specs = _specs(oracle, host, pages, info.npages)
    ref = oracle.read_column(oracle.INT64, specs, batch_size=1024)
    got = pqgpu.decode_column(ctx, pqgpu.INT64, specs)
    assert ref["status"] == 0, ref["message"]
    assert got["status"] == 0, got["message"]
    assert ctx.last_paths() & pqgpu.PATH_DICT_WINDOW, ctx.last_paths()
    assert got["num_values"] == n == len(ref["values"])
    np.testing.assert_array_equal(got["values"], ref["values"])
    # and the generator's own truth for the ragged last page
    last = np.zeros(pages[5].num_values, np.int64)
    L.pqg_truth_dict_int64(n, 65536, PAGE, seed, 4, last.ctypes.data)
    np.testing.assert_array_equal(got["values"][4 * PAGE:], last)


# ------------------------------------------------------------------------------ crafted streams
# A one-bit level stream of the writer's full bit-packed runs (header 0x7F: 63 groups, 504 levels,
# 64 bytes apart), whose payload bytes are chosen so that chains entering a window on payload
# bytes converge on a decoy track of valid headers that never meets the true chain.

def _parse(buf, p, w=1):
    """Header at p the way the level path's fast parse reads it (pqg_levels.hip lv_parse_xy):
    (next offset, ok)."""
    slen = len(buf)
    if p >= slen:
        return p, False
    h, hl = 0, 0
    for k in range(4):
        b = buf[p + k] if p + k < slen else 0
        h |= (b & 0x7F) << (7 * k)
        hl += 1
        if not b & 0x80:
            break
    else:
        return p, False  # a fifth varint byte: the fast parse refuses it
    g = h >> 1
    ln = hl + g * w if h & 1 else hl + (w + 7) // 8
    return p + ln, ln <= slen - p


def _bound_pick(buf, W0, w=1):
    """k_lv_bound's choice for the segment starting at W0 (non-wide streams): every chain entering
    the first window at [0, 64) walked over 2 KiB (<= 128 headers, hops out of the first window of
    the writer's form), the exit most chains share (ties: the lowest), None when no chain exits."""
    span = min(2048, len(buf) - W0)
    near = span + 8 + 64 * w
    votes = {}
    for e in range(64):
        o, ok = e, True
        for _ in range(128):
            if not (ok and o < span):
                break
            nx, ok = _parse(buf, W0 + o, w)
            o2 = nx - W0
            if o < 1024 and o2 >= 1024 + 8 + 64 * w:
                ok = False
            o = o2
        if ok and span <= o < near:
            votes[o] = votes.get(o, 0) + 1
    if not votes:
        return None
    top = max(votes.values())
    return W0 + min(o for o, c in votes.items() if c == top)


def _decoy_runs(nruns, rng, decoy=True):
    """nruns full bit-packed runs; with `decoy`, payload byte 33 of each run is 0x7F (a decoy
    header 64 bytes on, always at offset 33 of the next run) and every other payload byte 0x01 (a
    bit-packed header of 0 groups: one-byte hops, so that chains entering before byte 33 funnel
    into the decoy track and those entering after it into the next true header); without
    `decoy` the payload is random."""
    out = bytearray()
    for _ in range(nruns):
        run = bytearray([0x7F]) + bytearray(rng.integers(0, 256, 63, dtype=np.uint8).tobytes())
        if decoy:
            run[1:33] = b"\x01" * 32
            run[33] = 0x7F
            run[34:64] = b"\x01" * 30
        out += run
    return bytes(out)


def _page_from_stream(oracle, rng, stream, n):
    """A v1 data page: [i32 len][stream] + PLAIN INT32 values of its non-null levels (the
    oracle decodes the level stream to count them)."""
    st, lv = oracle.rle_decode(stream, 1, n, type_size=2)
    assert st == 0 and len(lv) == n
    nn = int((lv == 1).sum())
    vals = rng.integers(-2 ** 31, 2 ** 31, size=nn, dtype=np.int64).astype(np.int32)
    body = len(stream).to_bytes(4, "little") + stream + vals.tobytes()
    return oracle.PageSpec(oracle.PAGE_DATA, body, n, oracle.PLAIN, def_encoding=oracle.RLE)


@pytest.mark.parametrize("nruns", [1024, 2000, 10240])
def test_decoy_segment_starts(oracle, ctx, nruns):
    """Every segment start k_lv_bound picks is on the decoy track (checked with a model of its
    vote), so no segment walk lands on its successor: segment 0's walk follows the true chain to
    the page's end (k_lv_segscan's serial fallback), or past LW_SCAP recorded runs the page goes
    to the window path (10240 runs)."""
    rng = np.random.default_rng(nruns)
    stream = _decoy_runs(nruns, rng)
    for W0 in range(16384, len(stream) - 4096, 16384):
        pick = _bound_pick(stream, W0)
        assert pick is not None and (pick % 64) == 33, (W0, pick)  # a decoy header, not a true one
    n = nruns * 504 - 77  # the last run is read in part (levels.rs:255, rle.rs:398-434)
    _check(oracle, ctx, [_page_from_stream(oracle, rng, stream, n)])


def test_decoy_then_true_segments(oracle, ctx):
    """Decoy segments followed by ordinary ones: segment 0's walk passes the decoy starts and lands
    on a later segment's (true) start, so its successor is not j + 1 (the serial scan follows
    LvSeg::next); two such pages and a plain one in one chunk."""
    rng = np.random.default_rng(5)
    pages = []
    for lead in (3, 7):
        stream = _decoy_runs(256 * lead, rng) + _decoy_runs(256 * 5, rng, decoy=False)
        picks = [_bound_pick(stream, W0) for W0 in range(16384, len(stream) - 4096, 16384)]
        assert any(p is not None and p % 64 == 33 for p in picks)
        assert any(p is not None and p % 64 == 0 for p in picks)
        pages.append(_page_from_stream(oracle, rng, stream, len(stream) // 64 * 504))
    lv = (rng.random(300_000) >= 0.5).astype(np.int16)
    nn = int(lv.sum())
    pages.append(oracle.PageSpec(oracle.PAGE_DATA, oracle.level_encode(lv, 1) +
                                 rng.integers(-9, 9, nn).astype(np.int32).tobytes(), len(lv), oracle.PLAIN))
    _check(oracle, ctx, pages)


def test_segment_without_exit(oracle, ctx):
    """Segment 1's first window holds a bit-packed run of 255 groups (2040 levels: longer than the
    writer's 504, legal for the reader) that crosses out of the window, and every chain entering the
    window meets the true chain before it: no chain leaves of the writer's form, k_lv_bound records
    no start (LS_NOSTART) and segment 0's walk goes on to segment 2's start."""
    rng = np.random.default_rng(9)
    filler = lambda k: (b"\x7F" + b"\x01" * 63) * k  # noqa: E731  (payload: one-byte hops)
    head = filler(256)                    # segment 0: [0, 16384)
    pre = filler(14)                      # segment 1's window up to offset 896
    long_run = b"\xFF\x03" + b"\x01" * 255  # h = 511: bit-packed, 255 groups
    body = head + pre + long_run
    stream = body + filler((16384 * 3 - len(body)) // 64 + 1)
    assert _bound_pick(stream, 16384) is None
    n = (len(stream) - len(long_run)) // 64 * 504 + 2040
    _check(oracle, ctx, [_page_from_stream(oracle, rng, stream, n)])


# ------------------------------------------------------------------------------ config 5, full size

def test_alltypes_row_group_full_size():
    """One config-5 row group at the bench's size (2^23 rows, p_null 0.05, the reference writer's
    defaults: each dictionary column a single 8 M-value page) through pqg_rg_decode (one batched
    decode of the 11 chunks on the caller's stream), every column (levels, values, BYTE_ARRAY offsets) against the generator's cells."""
    import torch

    import pqgpu
    rows, row0, p_null, seed = 1 << 23, 3 << 23, 0.05, 0x5EED0005
    blob, pages, info = pqgtools.alltypes_row_group(rows, row0, p_null, seed, threads=16)
    assert info.chunk_first[3] - info.chunk_first[2] == 2  # tinyint_col: dictionary + one data page
    d_blob = torch.from_numpy(np.ascontiguousarray(blob[:info.blob_len + 64])).cuda()
    del blob
    cols = [pqgpu.Column(pt, -1, 1, 0) for _, pt in pqgtools.ALLTYPES]
    parr = [(pqgpu.Page * (info.chunk_first[j + 1] - info.chunk_first[j]))(
        *[pages[i] for i in range(info.chunk_first[j], info.chunk_first[j + 1])]) for j in range(11)]
    keep, outs = [], []
    for j, (_, pt) in enumerate(pqgtools.ALLTYPES):
        d_def = torch.empty(rows + 64, dtype=torch.int16, device="cuda")
        d_val = torch.empty(info.value_bytes[j] + 64, dtype=torch.uint8, device="cuda")
        d_off = torch.empty(rows + 8, dtype=torch.int64, device="cuda") if pt == 6 else None
        outs.append(pqgpu.Output(d_def.data_ptr(), None, d_val.data_ptr(), info.value_bytes[j] + 64,
                                 d_off.data_ptr() if d_off is not None else None, rows + 1 if pt == 6 else 0,
                                 0, 0, 0))
        keep.append((d_def, d_val, d_off))
    rgd = pqgpu.RowGroupDecoder(0, 16)
    try:
        oa = rgd.decode_async(cols, d_blob.data_ptr(), info.blob_len, parr, outs,
                              torch.cuda.current_stream().cuda_stream)
        st, bcol, bad = rgd.sync()
        assert st == 0, (st, bcol, bad, rgd.error_message())
        torch.cuda.current_stream().synchronize()
        for j, (name, pt) in enumerate(pqgtools.ALLTYPES):
            lv, vals, offs = pqgtools.alltypes_truth(row0, rows, j, p_null, seed, info.value_bytes[j])
            d_def, d_val, d_off = keep[j]
            assert oa[j].num_levels == rows and oa[j].num_values == info.num_values[j], name
            np.testing.assert_array_equal(d_def[:rows].cpu().numpy(), lv, err_msg=name)
            assert d_val[:info.value_bytes[j]].cpu().numpy().tobytes() == vals.tobytes(), name
            if offs is not None:
                np.testing.assert_array_equal(d_off[:len(offs)].cpu().numpy(), offs, err_msg=name)
    finally:
        rgd.close()
