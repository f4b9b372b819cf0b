"""CPU tests: the tooling's reference-identical writers and workload generators
(tools/gen/pqg_gen.cpp, libpqgtools.so) against the oracle's restated writers/decoders."""
import ctypes as C

import numpy as np
import pytest


@pytest.fixture(scope="module")
def pq():
    import pqgpu
    import pqgtools
    pqgtools.Page = pqgpu.Page
    return pqgtools


def _enc(fn, *args, cap):
    out = np.zeros(cap, np.uint8)
    n = fn(*args, out.ctypes.data_as(C.c_void_p), cap)
    assert n > 0
    return out[:n].tobytes()


@pytest.mark.parametrize("w", [1, 2, 3, 8, 15, 16, 20, 32])
def test_rle_writer_matches_oracle(pq, oracle, w):
    rng = np.random.default_rng(w)
    for mode in ("random", "runs", "mixed"):
        n = 5003
        if mode == "random":
            v = rng.integers(0, 1 << w, size=n, dtype=np.uint64)
        elif mode == "runs":
            v = np.repeat(rng.integers(0, 1 << w, size=n // 37 + 1, dtype=np.uint64), 37)[:n]
        else:
            v = np.where(rng.random(n) < 0.7, 1, rng.integers(0, 1 << w, size=n)).astype(np.uint64)
        got = _enc(pq.lib().pqg_encode_rle, v.ctypes.data_as(C.c_void_p), n, w, cap=n * 9 + 64)
        assert got == oracle.rle_encode(v, w)


def test_level_writer_matches_oracle(pq, oracle):
    rng = np.random.default_rng(1)
    for max_level in (1, 2, 7):
        lv = rng.integers(0, max_level + 1, size=10000).astype(np.int16)
        got = _enc(pq.lib().pqg_encode_levels_v1, lv.ctypes.data_as(C.c_void_p), len(lv), max_level,
                   cap=len(lv) * 4 + 64)
        assert got == oracle.level_encode(lv, max_level)


@pytest.mark.parametrize("ptype", ["INT32", "INT64"])
def test_delta_writer_matches_oracle(pq, oracle, ptype):
    t = getattr(oracle, ptype)
    dt = np.int32 if ptype == "INT32" else np.int64
    rng = np.random.default_rng(2)
    for n in (0, 1, 2, 128, 129, 5000):
        v = rng.integers(np.iinfo(dt).min, np.iinfo(dt).max, size=n, dtype=dt)
        got = _enc(pq.lib().pqg_encode_delta, t, v.ctypes.data_as(C.c_void_p), n, 128, 4,
                   cap=n * 10 + 256)
        assert got == oracle.delta_encode(t, v)
    # other block shapes decode to the same values through the oracle's decoder
    v = np.cumsum(rng.integers(-5000, 5000, size=3000)).astype(dt)
    for bs, nmb in ((512, 4), (256, 8), (64, 1), (1024, 16)):
        enc = _enc(pq.lib().pqg_encode_delta, t, v.ctypes.data_as(C.c_void_p), len(v), bs, nmb,
                   cap=len(v) * 10 + 1024)
        st, dec, off, tot = oracle.delta_decode(t, enc, len(v))
        assert st == 0 and dec.tolist() == v.tolist()


def _gen(pq, kind, **kw):
    L = pq.lib()
    info = pq.WorkloadInfo()
    args = {"levels": lambda b, c, p, pc: L.pqg_gen_levels_plain(kw["n"], kw["p"], kw["pv"], 7, 4, b, c, p, pc, C.byref(info)),
            "dict": lambda b, c, p, pc: L.pqg_gen_dict_int64(kw["n"], kw["dict"], kw["pv"], 7, 4, b, c, p, pc, C.byref(info)),
            "delta": lambda b, c, p, pc: L.pqg_gen_delta_int64(kw["n"], 16, kw["pv"], kw.get("bs", 512), kw.get("nmb", 4), 7, 4, b, c, p, pc, C.byref(info))}[kind]
    assert args(None, 0, None, 0) == 0
    blob = np.zeros(info.blob_len + 64, np.uint8)
    pages = (pq.Page * info.npages)()
    assert args(blob.ctypes.data_as(C.c_void_p), info.blob_len, pages, info.npages) == 0
    return blob, pages, info


def _specs(oracle, blob, pages):
    return [oracle.PageSpec(p.page_type, blob[p.offset:p.offset + p.nbytes].tobytes(), p.num_values,
                            p.encoding, p.def_encoding, p.rep_encoding, p.def_len, p.rep_len)
            for p in pages]


@pytest.mark.parametrize("p_null", [0.0, 0.1, 0.5])
def test_gen_levels_plain(pq, oracle, p_null):
    blob, pages, info = _gen(pq, "levels", n=300000, p=p_null, pv=65536)
    specs = _specs(oracle, blob, pages)
    r = oracle.read_column(oracle.INT32, specs, max_def=1)
    assert r["status"] == 0
    assert len(r["def"]) == info.total_levels == 300000
    assert len(r["values"]) == info.total_values
    frac = 1 - info.total_values / info.total_levels
    assert abs(frac - p_null) < 0.01
    # writer parity: re-encoding the decoded levels reproduces the page bytes
    off = 0
    for s, p in zip(specs, pages):
        lv = r["def"][off:off + p.num_values]
        off += p.num_values
        enc = oracle.level_encode(lv, 1)
        assert s.buf[:len(enc)] == enc


def test_gen_dict(pq, oracle):
    blob, pages, info = _gen(pq, "dict", n=200000, dict=65536, pv=65536)
    specs = _specs(oracle, blob, pages)
    assert pages[0].page_type == oracle.PAGE_DICTIONARY and pages[0].num_values == 65536
    d = np.frombuffer(specs[0].buf, np.int64)
    assert len(np.unique(d)) == 65536
    r = oracle.read_column(oracle.INT64, specs)
    assert r["status"] == 0 and len(r["values"]) == 200000
    for s in specs[1:]:
        assert s.buf[0] == 16
        st, idx = oracle.rle_decode(s.buf[1:], 16, s.num_values, 4)
        assert st == 0 and oracle.rle_encode(idx.astype(np.uint64), 16) == s.buf[1:]


@pytest.mark.parametrize("bs,nmb", [(512, 4), (128, 4)])
def test_gen_delta(pq, oracle, bs, nmb):
    blob, pages, info = _gen(pq, "delta", n=150000, pv=65536, bs=bs, nmb=nmb)
    specs = _specs(oracle, blob, pages)
    r = oracle.read_column(oracle.INT64, specs)
    assert r["status"] == 0 and len(r["values"]) == 150000
    d = np.diff(r["values"][:65536])
    assert d.min() >= -(1 << 15) and d.max() < (1 << 15)
    if bs == 128:  # the reference writer's own block shape: bytes must match exactly
        for s in specs:
            st, v, off, tot = oracle.delta_decode(oracle.INT64, s.buf, s.num_values)
            assert oracle.delta_encode(oracle.INT64, v) == s.buf


@pytest.mark.parametrize("kind", ["levels", "dict", "delta"])
def test_truth_matches_generated_pages(pq, oracle, kind):
    """pqg_truth_* (the bench's value check) regenerates exactly what the generator encoded:
    the oracle's decode of generated page k equals the truth of page k."""
    L = pq.lib()
    n, pv = 200000, 65536
    if kind == "levels":
        blob, pages, info = _gen(pq, "levels", n=n, p=0.3, pv=pv)
    elif kind == "dict":
        blob, pages, info = _gen(pq, "dict", n=n, dict=4096, pv=pv)
    else:
        blob, pages, info = _gen(pq, "delta", n=n, pv=pv)
    specs = _specs(oracle, blob, pages)
    first = 1 if kind == "dict" else 0
    for k in (0, len(specs) - first - 1):
        sel = ([specs[0]] if first else []) + [specs[first + k]]
        r = oracle.read_column(oracle.INT32 if kind == "levels" else oracle.INT64, sel,
                               max_def=1 if kind == "levels" else 0)
        assert r["status"] == 0
        cnt = specs[first + k].num_values
        if kind == "levels":
            lv = np.zeros(cnt, np.int16)
            vals = np.zeros(cnt, np.int32)
            nn = L.pqg_truth_levels_plain(n, 0.3, pv, 7, k, lv.ctypes.data, vals.ctypes.data)
            np.testing.assert_array_equal(r["def"], lv)
            np.testing.assert_array_equal(r["values"], vals[:nn])
        else:
            vals = np.zeros(cnt, np.int64)
            if kind == "dict":
                got = L.pqg_truth_dict_int64(n, 4096, pv, 7, k, vals.ctypes.data)
            else:
                got = L.pqg_truth_delta_int64(n, 16, pv, 7, k, vals.ctypes.data)
            assert got == cnt
            np.testing.assert_array_equal(r["values"], vals)
