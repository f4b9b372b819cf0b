"""Pins the C oracle against every known-answer test the reference holds for the path.

Each test cites the reference test it ports (path:line into /root/reference). The
reference's own random round-trip tests (unseeded thread_rng) are ported with fixed seeds.
"""
import numpy as np
import pytest


# ------------------------------------------------------------------ util/bit_util.rs

def test_ceil(oracle):  # bit_util.rs:627-639
    L = oracle.lib()
    for v, d, e in [(0, 1, 0), (1, 1, 1), (1, 2, 1), (1, 8, 1), (7, 8, 1), (8, 8, 1), (9, 8, 2),
                    (9, 9, 1), (10000000000, 10, 1000000000), (10, 10000000000, 1),
                    (10000000000, 1000000000, 10)]:
        assert L.or_ceil(v, d) == e


def test_log2_and_required_bits(oracle):  # bit_util.rs:727-750
    L = oracle.lib()
    for x, e in [(0, 0), (1, 1), (2, 2), (4, 3), (8, 4), (10, 4), (12, 4), (16, 5)]:
        assert L.or_num_required_bits(x) == e
    for x, e in [(1, 0), (2, 1), (3, 2), (4, 2), (5, 3), (6, 3), (7, 3), (8, 3), (9, 4)]:
        assert L.or_log2(x) == e


def test_bit_reader_get_byte_offset(oracle):  # bit_util.rs:641-654
    r = oracle.BitReaderPy([255] * 10)
    assert r.get_byte_offset() == 0
    r.get_value(6, 4)
    assert r.get_byte_offset() == 1
    r.get_value(10, 4)
    assert r.get_byte_offset() == 2
    r.get_value(20, 4)
    assert r.get_byte_offset() == 5
    r.get_value(30, 4)
    assert r.get_byte_offset() == 9


def test_bit_reader_get_value(oracle):  # bit_util.rs:656-664
    r = oracle.BitReaderPy([255, 0])
    assert [r.get_value(1, 4), r.get_value(2, 4), r.get_value(3, 4), r.get_value(4, 4)] == [1, 3, 7, 3]


def test_bit_reader_get_value_boundary(oracle):  # bit_util.rs:666-674
    r = oracle.BitReaderPy([10, 0, 0, 0, 20, 0, 30, 0, 0, 0, 40, 0])
    assert [r.get_value(32), r.get_value(16), r.get_value(32), r.get_value(16)] == [10, 20, 30, 40]


def test_bit_reader_get_aligned(oracle):  # bit_util.rs:676-686
    r = oracle.BitReaderPy([0x75, 0xCB])
    assert r.get_value(3, 4) == 5
    assert r.get_aligned(1) == 203
    assert r.get_value(1, 4) is None
    r = oracle.BitReaderPy([0x75, 0xCB])
    assert r.get_aligned(3) is None


def test_bit_reader_vlq(oracle):  # bit_util.rs:688-695
    r = oracle.BitReaderPy([0x89, 0x01, 0xF2, 0xB5, 0x06])
    assert r.get_vlq_int() == 137
    assert r.get_vlq_int() == 105202


def test_bit_reader_zigzag(oracle):  # bit_util.rs:697-705
    r = oracle.BitReaderPy([0, 1, 2, 3])
    assert [r.get_zigzag_vlq_int() for _ in range(4)] == [0, -1, 1, -2]


def test_vlq_max_len_panics(oracle):  # bit_util.rs:570-574 (assert on > 10 bytes)
    r = oracle.BitReaderPy([0x80] * 10 + [0x01])
    assert r.get_vlq_int() is None and r.r.status == oracle.PANIC
    r = oracle.BitReaderPy([0xFF] * 9 + [0x01])
    assert r.get_vlq_int() == -1  # 10-byte varint is accepted


@pytest.mark.parametrize("num_bits", list(range(0, 33)))
def test_get_batch_roundtrip(oracle, num_bits):  # bit_util.rs:888-935 (seeded)
    rng = np.random.default_rng(1000 + num_bits)
    for total in (1, 31, 32, 33, 100, 1000):
        hi = 1 << num_bits
        vals = rng.integers(0, hi, size=total, dtype=np.uint64) if num_bits else np.zeros(total, np.uint64)
        # BitWriter::put_value stream == RLE-free bit packing: build it directly
        acc, nb, out = 0, 0, bytearray()
        for v in vals:
            acc |= int(v) << nb
            nb += num_bits
            while nb >= 8:
                out.append(acc & 0xFF)
                acc >>= 8
                nb -= 8
        if nb:
            out.append(acc & 0xFF)
        for ts in (4, 2, 8) if num_bits <= 16 else (4, 8):
            r = oracle.BitReaderPy(bytes(out))
            got = r.get_batch(total, num_bits, ts)
            assert len(got) == total
            if ts == 8:
                # 8-byte T through unpack32 writes only the low 4 bytes (bit_util.rs:498-503);
                # buffers start zeroed so the value still matches.
                assert (got.astype(np.uint64) & 0xFFFFFFFF).tolist() == vals.tolist()
            else:
                mask = (1 << (8 * ts)) - 1
                assert [int(x) & mask for x in got] == [int(v) & mask for v in vals]


# ------------------------------------------------------------------ encodings/rle.rs

def test_rle_decode_int32(oracle):  # rle.rs:524-535
    st, v = oracle.rle_decode(bytes([0x03, 0x88, 0xC6, 0xFA]), 3, 8)
    assert st == 0 and v.tolist() == list(range(8))


def test_rle_decode_bool(oracle):  # rle.rs:552-592
    st, v = oracle.rle_decode(bytes([0x64, 0x01, 0x64, 0x00]), 1, 100, 1)
    assert st == 0 and v.tolist() == [1] * 50 + [0] * 50
    data2 = bytes([0x1B] + [0xAA] * 12 + [0x0A])
    st, v = oracle.rle_decode(data2, 1, 100, 1)
    assert st == 0 and v.tolist() == [i % 2 for i in range(100)]


def test_rle_decode_with_dict(oracle):  # rle.rs:595-623
    st, v = oracle.rle_decode_dict(bytes([0x06, 0x00, 0x08, 0x01, 0x0A, 0x02]), 3,
                                   np.array([10, 20, 30], np.int32), 12)
    assert st == 0 and v.tolist() == [10] * 3 + [20] * 4 + [30] * 5
    words = np.array([b"aaa", b"bbb", b"ccc", b"ddd", b"eee", b"fff"], dtype="S3")
    st, v = oracle.rle_decode_dict(bytes([0x03, 0x63, 0xC7, 0x8E, 0x03, 0x65, 0x0B]), 3, words, 12)
    assert st == 0
    assert [x.decode() for x in v] == ["ddd", "eee", "fff", "ddd", "eee", "fff", "ddd", "eee",
                                       "fff", "eee", "fff", "fff"]


def _validate_rle(oracle, values, bit_width, expected=None, expected_len=-1):  # rle.rs:625-665
    enc = oracle.rle_encode(values, bit_width)
    if expected_len != -1:
        assert len(enc) == expected_len
    if expected is not None:
        assert enc == bytes(expected)
    st, dec = oracle.rle_decode(enc, bit_width, len(values), 8)
    assert st == 0
    mask = (1 << 32) - 1  # 8-byte T: unpack32 path writes 4 bytes; values here fit
    assert [int(x) & mask for x in dec] == [int(v) & mask for v in values]


def test_rle_specific_sequences(oracle):  # rle.rs:668-722
    values = [0] * 50 + [1] * 50
    exp = [50 << 1, 0, 50 << 1, 1]
    for w in range(1, 9):
        _validate_rle(oracle, values, w, exp, 4)
    for w in range(9, 33):
        _validate_rle(oracle, values, w, None, 2 * (1 + (w + 7) // 8))
    values = [i % 2 for i in range(101)]
    ng = (100 + 7) // 8
    exp = [(ng << 1) | 1] + [0b10101010] * (100 // 8) + [0b00001010]
    _validate_rle(oracle, values, 1, exp, 1 + ng)
    for w in range(2, 33):
        nv = ng * 8
        _validate_rle(oracle, values, w, None, 1 + (w * nv + 7) // 8)


@pytest.mark.parametrize("width", list(range(1, 33)))
def test_rle_values(oracle, width):  # rle.rs:724-749
    mod = 1 << width
    for n, val in ((1, -1), (1024, -1), (1024, 0), (1024, 1)):
        vals = [(v % mod) if val == -1 else val for v in range(n)]
        _validate_rle(oracle, vals, width)


def test_rle_specific_roundtrip(oracle):  # rle.rs:751-767
    vals = [0, 1, 1, 1, 1, 0, 0, 0, 0, 1]
    enc = oracle.rle_encode(vals, 1)
    st, dec = oracle.rle_decode(enc, 1, len(vals), 2)
    assert st == 0 and dec.tolist() == vals


def test_rle_random(oracle):  # rle.rs:796-835 (seeded instead of thread_rng)
    for it in range(50):
        rng = np.random.default_rng(7000 + it)
        vals, parity = [], 0
        for _ in range(1000):
            g = int(rng.integers(1, 20))
            if g > 15:
                g = 1
            vals += [parity] * g
            parity ^= 1
        bw = int(oracle.lib().or_num_required_bits(len(vals)))
        enc = oracle.rle_encode(vals, bw)
        st, dec = oracle.rle_decode(enc, bw, len(vals), 4)
        assert st == 0 and dec.tolist() == vals


def test_rle_truncated_bitpacked_reports_hang(oracle):
    st, v = oracle.rle_decode(bytes([0x03, 0x88]), 3, 8)
    assert st == oracle.HANG


# ------------------------------------------------------------------ encodings/levels.rs

def test_levels_set_data_range(oracle):  # levels.rs:487-506
    buf = bytes([5, 198, 2, 5, 42, 168, 10, 0, 2, 3, 36, 73])
    st, rep = oracle.rle_decode(buf[0:3], 1, 10, 2)
    assert st == 0 and rep.tolist() == [0, 1, 1, 0, 0, 0, 1, 1, 0, 1]
    st, d = oracle.rle_decode(buf[3:8], 2, 10, 2)
    assert st == 0 and d.tolist() == [2, 2, 2, 0, 0, 2, 2, 2, 2, 2]
    # through the column reader with a v2 page: rep from bytes 0..3, def from 3..8
    page = oracle.PageSpec(oracle.PAGE_DATA_V2, buf, 10, oracle.PLAIN, rep_len=3, def_len=5)
    r = oracle.read_column(oracle.BOOLEAN, [page], max_def=2, max_rep=1)
    assert r["rep"].tolist() == [0, 1, 1, 0, 0, 0, 1, 1, 0, 1]
    assert r["def"].tolist() == [2, 2, 2, 0, 0, 2, 2, 2, 2, 2]


@pytest.mark.parametrize("enc", ["RLE", "BIT_PACKED", "RLE_V2"])
@pytest.mark.parametrize("max_level", [1, 3, 10, 1000, 32767])
def test_levels_roundtrip(oracle, enc, max_level):  # levels.rs:279-419 (seeded)
    rng = np.random.default_rng(max_level)
    for n in (1, 7, 8, 9, 100, 1000, 4097):
        levels = rng.integers(0, max_level + 1, size=n).astype(np.int16)
        if enc == "RLE_V2":
            data = oracle.level_encode(levels, max_level, oracle.RLE, v2=True)
            page = oracle.PageSpec(oracle.PAGE_DATA_V2, data + oracle.plain_encode(oracle.INT32, np.zeros(0, np.int32)), n,
                                   oracle.PLAIN, def_len=len(data))
        else:
            e = oracle.RLE if enc == "RLE" else oracle.BIT_PACKED
            data = oracle.level_encode(levels, max_level, e)
            page = oracle.PageSpec(oracle.PAGE_DATA, data, n, oracle.PLAIN, def_encoding=e)
        nn = int((levels == max_level).sum())
        page.buf += oracle.plain_encode(oracle.INT32, np.arange(nn, dtype=np.int32))
        for bs in (16, 17, 1024):
            r = oracle.read_column(oracle.INT32, [page], max_def=max_level, batch_size=bs)
            assert r["status"] == 0, r["message"]
            assert r["def"].tolist() == levels.tolist()
            assert r["values"].tolist() == list(range(nn))


def test_bit_packed_level_set_data_size(oracle):  # levels.rs:521-530
    # max size is ceil(n*w/8) bounded by the buffer
    buf = bytes([1, 2, 3, 4, 5])
    page = oracle.PageSpec(oracle.PAGE_DATA, buf, 3, oracle.PLAIN, def_encoding=oracle.BIT_PACKED)
    r = oracle.read_column(oracle.BOOLEAN, [page], max_def=1)
    # 1 byte of levels (0b00000001 -> 1,0,0), then PLAIN bools from byte 1 (0x02 -> 0)
    assert r["def"].tolist() == [1, 0, 0]
    assert r["values"].tolist() == [0]


# ------------------------------------------------------------------ encodings/decoding.rs

def test_plain_decode_fixed(oracle):  # decoding.rs:875-955
    for pt, data in ((oracle.INT32, np.array([42, 18, 52], np.int32)),
                     (oracle.INT64, np.array([42, 18, 52], np.int64)),
                     (oracle.FLOAT, np.array([3.14, 2.414, 12.51], np.float32)),
                     (oracle.DOUBLE, np.array([3.14, 2.414, 12.51], np.float64))):
        st, v = oracle.plain_decode(pt, data.tobytes(), 3, 3)
        assert st == 0 and v.tobytes() == data.tobytes()


def test_plain_decode_int96(oracle):  # decoding.rs:915-929, data_type.rs:381-383
    words = np.array([[11, 22, 33], [44, 55, 66], [10, 20, 30], [40, 50, 60]], np.uint32)
    st, v = oracle.plain_decode(oracle.INT96, words.tobytes(), 4, 4)
    assert st == 0 and v.tobytes() == words.tobytes()


def test_plain_decode_bool(oracle):  # decoding.rs:931-943
    data = [0, 1, 0, 0, 1, 0, 1, 1, 0, 1]
    enc = oracle.plain_encode(oracle.BOOLEAN, np.array(data, np.uint8))
    st, v = oracle.plain_decode(oracle.BOOLEAN, enc, 10, 10)
    assert st == 0 and v.tolist() == data


def test_plain_decode_byte_array_and_flba(oracle):  # decoding.rs:945-975
    enc = oracle.plain_encode_ba([b"hello", b"parquet"])
    assert enc == b"\x05\x00\x00\x00hello\x07\x00\x00\x00parquet"
    page = oracle.PageSpec(oracle.PAGE_DATA, enc, 2, oracle.PLAIN)
    r = oracle.read_column(oracle.BYTE_ARRAY, [page])
    assert r["values"] == [b"hello", b"parquet"]
    enc = oracle.plain_encode_ba([b"bird", b"come", b"flow"], fixed=True)
    page = oracle.PageSpec(oracle.PAGE_DATA, enc, 3, oracle.PLAIN)
    r = oracle.read_column(oracle.FIXED_LEN_BYTE_ARRAY, [page], type_length=4)
    assert r["values"] == [b"bird", b"come", b"flow"]


def test_plain_decode_eof(oracle):  # decoding.rs:145-147
    st, v = oracle.plain_decode(oracle.INT32, b"\x01\x00\x00\x00\x02", 2, 2)
    assert st == oracle.EOF


def test_delta_bit_packed_decoder_sample(oracle):  # decoding.rs:1152-1167
    data = bytes([128, 1, 4, 3, 58, 28, 6, 0, 0, 0, 0, 8] + [0] * 22)
    st, v, off, tot = oracle.delta_decode(oracle.INT32, data, 0)
    assert st == 0 and off == 5 and tot == 3
    st, v, off, tot = oracle.delta_decode(oracle.INT32, data, 3)
    assert st == 0 and v.tolist() == [29, 43, 89] and off == 34


@pytest.mark.parametrize("pt", ["INT32", "INT64"])
def test_delta_roundtrip(oracle, pt):  # decoding.rs:1060-1150 (seeded)
    t = getattr(oracle, pt)
    dt = np.int32 if pt == "INT32" else np.int64
    info = np.iinfo(dt)
    rng = np.random.default_rng(11)
    cases = [np.zeros(0, dt), np.array([5], dt), np.arange(129, dtype=dt),
             rng.integers(info.min, info.max, size=1000, dtype=dt, endpoint=True),
             rng.integers(-1000, 1000, size=4097).astype(dt),
             np.array([info.max, info.min, info.max, 0, info.min], dt)]
    for vals in cases:
        enc = oracle.delta_encode(t, vals)
        st, dec, off, tot = oracle.delta_decode(t, enc, len(vals))
        assert st == 0 and tot == len(vals)
        assert dec.tolist() == vals.tolist()


def test_dict_roundtrip_column(oracle):  # decoding.rs:1200-1236 + reader.rs make_pages
    rng = np.random.default_rng(5)
    vals = rng.integers(0, 1000, size=5000).astype(np.int64)
    dpage, ipage, nu = oracle.dict_encode(vals)
    assert nu == len(np.unique(vals))
    assert ipage[0] == int(oracle.lib().or_log2(nu))
    pages = [oracle.PageSpec(oracle.PAGE_DICTIONARY, dpage, nu, oracle.PLAIN),
             oracle.PageSpec(oracle.PAGE_DATA, ipage, len(vals), oracle.PLAIN_DICTIONARY)]
    r = oracle.read_column(oracle.INT64, pages)
    assert r["status"] == 0 and r["values"].tolist() == vals.tolist()


def test_delta_length_and_byte_array(oracle):  # decoding.rs:1168-1236 (seeded)
    rng = np.random.default_rng(3)
    words = [b"", b"a", b"ab", b"abc", b"abd", b"b", b"bbbbbbbb", b"bbbbbbbc"]
    vals = [words[int(i)] for i in rng.integers(0, len(words), size=777)]
    for enc_fn, enc in ((oracle.delta_length_encode, oracle.DELTA_LENGTH_BYTE_ARRAY),
                        (oracle.delta_byte_array_encode, oracle.DELTA_BYTE_ARRAY)):
        data = enc_fn(vals)
        page = oracle.PageSpec(oracle.PAGE_DATA, data, len(vals), enc)
        for bs in (1, 16, 1024):
            r = oracle.read_column(oracle.BYTE_ARRAY, [page], batch_size=bs)
            assert r["status"] == 0, r["message"]
            assert r["values"] == vals


def test_rle_bool_value_decoder(oracle):  # decoding.rs:339-384 + encoding.rs:475-500
    rng = np.random.default_rng(9)
    vals = (rng.random(3000) < 0.3).astype(np.uint8)
    data = oracle.rle_bool_encode(vals)
    page = oracle.PageSpec(oracle.PAGE_DATA_V2, data, len(vals), oracle.RLE)
    r = oracle.read_column(oracle.BOOLEAN, [page])
    assert r["status"] == 0 and r["values"].tolist() == vals.tolist()


def test_as_bytes_layouts():  # data_type.rs:348-389
    assert np.array([555], np.int32).tobytes() == bytes([43, 2, 0, 0])
    assert np.array([-2 ** 31], np.int32).tobytes() == bytes([0, 0, 0, 128])
    assert np.array([3.14], np.float32).tobytes() == bytes([195, 245, 72, 64])
    assert np.array([3.14], np.float64).tobytes() == bytes([31, 133, 235, 81, 184, 30, 9, 64])
    assert np.array([1, 2, 3], np.uint32).tobytes() == bytes([1, 0, 0, 0, 2, 0, 0, 0, 3, 0, 0, 0])


# ------------------------------------------------------------------ column/reader.rs

def test_column_reader_mixed_pages(oracle):  # reader.rs:571-896 pattern (seeded make_pages)
    rng = np.random.default_rng(17)
    max_def = 1
    pages, exp_def, exp_val = [], [], []
    dict_vals = np.arange(100, 200, dtype=np.int32)
    dpage = oracle.plain_encode(oracle.INT32, dict_vals)
    pages.append(oracle.PageSpec(oracle.PAGE_DICTIONARY, dpage, len(dict_vals), oracle.PLAIN))
    for pi in range(6):
        n = int(rng.integers(1, 3000))
        lv = (rng.random(n) < 0.8).astype(np.int16)
        nn = int(lv.sum())
        v2 = pi % 2 == 1
        if pi % 3 == 0:
            idx = rng.integers(0, len(dict_vals), size=nn)
            vals = dict_vals[idx]
            bw = int(oracle.lib().or_log2(len(dict_vals)))
            body = bytes([bw]) + oracle.rle_encode(idx, bw)
            enc = oracle.RLE_DICTIONARY
        elif pi % 3 == 1:
            vals = rng.integers(-2 ** 31, 2 ** 31, size=nn).astype(np.int32)
            body = oracle.plain_encode(oracle.INT32, vals)
            enc = oracle.PLAIN
        else:
            vals = rng.integers(-50, 50, size=nn).astype(np.int32).cumsum().astype(np.int32)
            body = oracle.delta_encode(oracle.INT32, vals)
            enc = oracle.DELTA_BINARY_PACKED
        if v2:
            lev = oracle.level_encode(lv, max_def, oracle.RLE, v2=True)
            pages.append(oracle.PageSpec(oracle.PAGE_DATA_V2, lev + body, n, enc, def_len=len(lev)))
        else:
            lev = oracle.level_encode(lv, max_def, oracle.RLE)
            pages.append(oracle.PageSpec(oracle.PAGE_DATA, lev + body, n, enc))
        exp_def += lv.tolist()
        exp_val += vals.tolist()
    for bs in (16, 17, 512):
        r = oracle.read_column(oracle.INT32, pages, max_def=max_def, batch_size=bs)
        assert r["status"] == 0, r["message"]
        assert r["def"].tolist() == exp_def
        assert r["values"].tolist() == exp_val


def test_second_dictionary_is_error(oracle):  # reader.rs:469-471
    dpage = oracle.plain_encode(oracle.INT32, np.arange(4, dtype=np.int32))
    pages = [oracle.PageSpec(oracle.PAGE_DICTIONARY, dpage, 4, oracle.PLAIN)] * 2
    r = oracle.read_column(oracle.INT32, pages)
    assert r["status"] == oracle.GENERAL
