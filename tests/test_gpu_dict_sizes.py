"""RLE_DICTIONARY chunks of 4- and 8-byte values whose dictionary is larger than the level path's
(2^8 entries): the windowed gather (indices to a buffer or decoded in the gather kernel, then the
dictionary streamed through 128 KiB LDS windows: k_dict_win). Values must be the oracle's
(get_batch_with_dict, rle.rs:437-487; DictDecoder, decoding.rs:282-315) for dictionaries of 257 to
65536 entries at any byte alignment inside the blob, for chunks of several dictionaries in one
batch, for tiles of many short runs, and an index past the dictionary is the reference's panic."""
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


def _dvals(rng, ptype, oracle, nd):
    if ptype in (oracle.INT32, oracle.FLOAT):
        v = np.unique(rng.integers(0, 2 ** 32, nd * 2, dtype=np.uint64).astype(np.uint32))[:nd]
        rng.shuffle(v)
        return v.view(np.int32) if ptype == oracle.INT32 else v.view(np.float32)
    v = np.unique(rng.integers(0, 2 ** 63, nd * 2, dtype=np.uint64))[:nd]
    rng.shuffle(v)
    return v.view(np.int64) if ptype == oracle.INT64 else v.view(np.float64)


def _chunk(oracle, rng, ptype, nd, sizes, p_null, hi=None):
    dv = _dvals(rng, ptype, oracle, nd)
    d = oracle.PageSpec(oracle.PAGE_DICTIONARY, oracle.plain_encode(ptype, dv), len(dv), oracle.PLAIN_DICTIONARY)
    hi = nd if hi is None else hi
    bw = max(1, int(np.ceil(np.log2(max(hi, 2)))))

    def body(nn):
        return bytes([bw]) + oracle.rle_encode(rng.integers(0, hi, nn).astype(np.uint64), bw)

    pages = [d]
    for n in sizes:
        lv = (rng.random(n) >= p_null).astype(np.int16)
        pages.append(oracle.PageSpec(oracle.PAGE_DATA, oracle.level_encode(lv, 1) + body(int(lv.sum())), n,
                                     oracle.RLE_DICTIONARY))
    return pages


def _same(oracle, ctx, ptype, pages):
    import pqgpu
    ref = oracle.read_column(ptype, pages, max_def=1)
    got = pqgpu.decode_column(ctx, ptype, pages, max_def=1)
    assert got["status"] == ref["status"], (got["message"], ref["message"])
    if ref["status"] == 0:
        np.testing.assert_array_equal(got["def"], ref["def"])
        assert np.asarray(got["values"]).tobytes() == ref["values"].tobytes()
    return got, ref


@pytest.mark.parametrize("ptype", ["INT32", "INT64", "FLOAT", "DOUBLE"])
@pytest.mark.parametrize("nd", [300, 16385, 40000, 65536])
def test_dictionary_sizes(oracle, ctx, ptype, nd):
    """Ragged pages (a partial last tile, a 3-value page) beside long ones."""
    rng = np.random.default_rng(nd + len(ptype))
    t = getattr(oracle, ptype)
    _same(oracle, ctx, t, _chunk(oracle, rng, t, nd, (70_001, 3, 9000, 4096, 4097), 0.25))


@pytest.mark.parametrize("p_null", [0.0, 0.6])
def test_dictionary_required_and_sparse(oracle, ctx, p_null):
    rng = np.random.default_rng(31)
    _same(oracle, ctx, oracle.INT64, _chunk(oracle, rng, oracle.INT64, 30000, (200_000, 12_345), p_null))


@pytest.mark.parametrize("ptype", ["INT32", "INT64"])
def test_dictionary_index_past_the_end(oracle, ctx, ptype):
    """Indices drawn up to 1023 against a 1000-entry dictionary: the reference panics."""
    rng = np.random.default_rng(32)
    t = getattr(oracle, ptype)
    got, ref = _same(oracle, ctx, t, _chunk(oracle, rng, t, 1000, (50_000,), 0.1, hi=1024))
    assert ref["status"] != 0


def test_dictionaries_of_several_chunks(oracle, ctx):
    """A batch of chunks with different dictionaries (sizes, value widths) and short pages: the
    tiles of several chunks side by side in one tile list."""
    from test_gpu_batch import _check_zoo, _decode_batch
    rng = np.random.default_rng(33)
    zoo = []
    for k, (pt, nd) in enumerate([("INT64", 3000), ("INT64", 50000), ("INT32", 700), ("DOUBLE", 20000),
                                   ("INT64", 65536), ("FLOAT", 40000)]):
        t = getattr(oracle, pt)
        sizes = (5000, 300, 9000) if k % 2 else (4096, 1, 12000)
        zoo.append((f"{pt}_{nd}", t, _chunk(oracle, rng, t, nd, sizes, 0.2), 1, 0, -1, True))
    for order in (list(range(len(zoo))), list(reversed(range(len(zoo))))):
        st, res = _decode_batch(ctx, zoo, order)
        _check_zoo(oracle, zoo, st, res, order)


@pytest.mark.parametrize("mean_run", [3, 12, 40, 400])
@pytest.mark.parametrize("ptype", ["INT32", "INT64"])
def test_dictionary_index_runs(oracle, ctx, ptype, mean_run):
    """Indices in runs of equal values (RLE runs beside bit-packed ones): tiles of few records
    (their indices read from the stream by the gather kernel), of many (kept by the tile expand)
    and of more than one index batch (re-walked)."""
    rng = np.random.default_rng(34 + mean_run)
    t = getattr(oracle, ptype)
    nd = 5000
    dv = _dvals(rng, t, oracle, nd)
    d = oracle.PageSpec(oracle.PAGE_DICTIONARY, oracle.plain_encode(t, dv), nd, oracle.PLAIN_DICTIONARY)
    bw = 13
    pages = [d]
    for n in (60_000, 4097, 30_001):
        lens = rng.geometric(1.0 / mean_run, n)
        vals = rng.integers(0, nd, len(lens))
        idx = np.repeat(vals, lens)[:n]
        lv = np.ones(n, np.int16)
        lv[rng.random(n) < 0.1] = 0
        body = bytes([bw]) + oracle.rle_encode(idx[:int(lv.sum())].astype(np.uint64), bw)
        pages.append(oracle.PageSpec(oracle.PAGE_DATA, oracle.level_encode(lv, 1) + body, n, oracle.RLE_DICTIONARY))
    _same(oracle, ctx, t, pages)


@pytest.mark.parametrize("nd", [257, 4097, 65536])
@pytest.mark.parametrize("ptype", ["INT32", "INT64"])
def test_dictionary_hard_tiles_mixed(oracle, ctx, ptype, nd):
    """Windowed-gather tiles that k_dict_win does not decode itself -- 4096-index tiles of short
    RLE runs (each index repeated 9..12 times: ~380 run records, more than DF_RC = 128) -- beside
    easy tiles of random indices, alternating along one long page and a ragged second: 320 hard
    tiles, more than one k_didx_mark workgroup's 256 list entries, expanded by k_texpand_didx's
    grid-strided list, then gathered with their easy neighbours by one k_dict_win
    workgroup. Values against the oracle (get_batch_with_dict, rle.rs:437-487)."""
    rng = np.random.default_rng(nd + 7 * len(ptype))
    t = getattr(oracle, ptype)
    dv = _dvals(rng, t, oracle, nd)
    d = oracle.PageSpec(oracle.PAGE_DICTIONARY, oracle.plain_encode(t, dv), nd, oracle.PLAIN_DICTIONARY)
    bw = max(1, int(np.ceil(np.log2(nd))))
    pages = [d]
    for ntiles in (640, 37):
        parts = []
        for k in range(ntiles):
            if k % 2 == 0:
                lens = rng.integers(9, 13, 500)
                parts.append(np.repeat(rng.integers(0, nd, 500), lens)[:4096])
            else:
                parts.append(rng.integers(0, nd, 4096))
        idx = np.concatenate(parts)[:ntiles * 4096 - 1000]
        n = len(idx)
        body = bytes([bw]) + oracle.rle_encode(idx.astype(np.uint64), bw)
        pages.append(oracle.PageSpec(oracle.PAGE_DATA, oracle.level_encode(np.ones(n, np.int16), 1) + body, n,
                                     oracle.RLE_DICTIONARY))
    _same(oracle, ctx, t, pages)
