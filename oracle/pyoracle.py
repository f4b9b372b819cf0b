"""ctypes binding of the C parity oracle (oracle/pq_oracle.c). TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / CPU baseline. The product path never touches it.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libpqoracle.so")

OK, GENERAL, NYI, EOF, PANIC, HANG = range(6)
BOOLEAN, INT32, INT64, INT96, FLOAT, DOUBLE, BYTE_ARRAY, FIXED_LEN_BYTE_ARRAY = range(8)
PLAIN, PLAIN_DICTIONARY, RLE, BIT_PACKED = 0, 2, 3, 4
DELTA_BINARY_PACKED, DELTA_LENGTH_BYTE_ARRAY, DELTA_BYTE_ARRAY, RLE_DICTIONARY = 5, 6, 7, 8
PAGE_DATA, PAGE_DICTIONARY, PAGE_DATA_V2 = 0, 2, 3

TYPE_SIZE = {BOOLEAN: 1, INT32: 4, INT64: 8, INT96: 12, FLOAT: 4, DOUBLE: 8}
NP_DTYPE = {BOOLEAN: np.uint8, INT32: np.int32, INT64: np.int64, FLOAT: np.float32,
            DOUBLE: np.float64}


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = C.CDLL(_LIB_PATH)
        _declare(_lib)
    return _lib


class Page(C.Structure):
    _fields_ = [("page_type", C.c_int), ("buf", C.c_void_p), ("len", C.c_size_t),
                ("num_values", C.c_uint32), ("encoding", C.c_int), ("def_encoding", C.c_int),
                ("rep_encoding", C.c_int), ("def_len", C.c_uint32), ("rep_len", C.c_uint32)]


class Column(C.Structure):
    _fields_ = [("physical_type", C.c_int), ("type_length", C.c_int32),
                ("max_def", C.c_int16), ("max_rep", C.c_int16)]


class ColumnResult(C.Structure):
    _fields_ = [("status", C.c_int), ("message", C.c_char * 256),
                ("def_levels", C.POINTER(C.c_int16)), ("rep_levels", C.POINTER(C.c_int16)),
                ("values", C.POINTER(C.c_uint8)), ("offsets", C.POINTER(C.c_int64)),
                ("bytes", C.POINTER(C.c_uint8)), ("num_levels", C.c_size_t),
                ("num_values", C.c_size_t), ("num_bytes", C.c_size_t),
                ("num_batches", C.c_size_t)]


class BitReader(C.Structure):
    _fields_ = [("buf", C.c_void_p), ("total_bytes", C.c_size_t), ("byte_offset", C.c_size_t),
                ("bit_offset", C.c_size_t), ("buffered", C.c_uint64), ("status", C.c_int)]


def _declare(L):
    sz, vp, u8p = C.c_size_t, C.c_void_p, C.c_char_p
    szp = C.POINTER(C.c_size_t)
    L.or_ceil.restype = C.c_int64
    L.or_ceil.argtypes = [C.c_int64, C.c_int64]
    L.or_log2.argtypes = [C.c_uint64]
    L.or_num_required_bits.restype = sz
    L.or_num_required_bits.argtypes = [C.c_uint64]
    L.or_br_init.argtypes = [C.POINTER(BitReader), vp, sz]
    L.or_br_get_value.argtypes = [C.POINTER(BitReader), C.c_int, C.c_int, C.POINTER(C.c_uint64)]
    L.or_br_get_batch.restype = sz
    L.or_br_get_batch.argtypes = [C.POINTER(BitReader), vp, sz, C.c_int, C.c_int]
    L.or_br_get_aligned.argtypes = [C.POINTER(BitReader), sz, C.POINTER(C.c_uint64)]
    L.or_br_get_vlq_int.argtypes = [C.POINTER(BitReader), C.POINTER(C.c_int64)]
    L.or_br_get_zigzag_vlq_int.argtypes = [C.POINTER(BitReader), C.POINTER(C.c_int64)]
    L.or_br_get_byte_offset.restype = sz
    L.or_br_get_byte_offset.argtypes = [C.POINTER(BitReader)]
    L.or_rle_decode.argtypes = [vp, sz, C.c_int, C.c_int, vp, sz, szp]
    L.or_rle_decode_dict.argtypes = [vp, sz, C.c_int, vp, sz, sz, vp, sz, szp]
    L.or_plain_decode.argtypes = [C.c_int, C.c_int32, vp, sz, sz, vp, sz, szp]
    L.or_delta_decode.argtypes = [C.c_int, vp, sz, vp, sz, szp, szp, szp]
    L.or_read_column.argtypes = [C.POINTER(Column), C.POINTER(Page), sz, sz, C.c_int, C.c_int,
                                 C.POINTER(ColumnResult)]
    L.or_read_column_caps.argtypes = [C.POINTER(Column), C.POINTER(Page), sz, sz, sz, sz, sz, C.c_int,
                                      C.c_int, vp, sz, C.POINTER(ColumnResult)]
    L.or_column_result_free.argtypes = [C.POINTER(ColumnResult)]
    for name, args in [
        ("or_rle_encode", [vp, sz, C.c_int, vp, sz]),
        ("or_level_encode", [C.c_int, C.c_int, C.c_int16, vp, sz, vp, sz]),
        ("or_plain_encode", [C.c_int, vp, sz, vp, sz]),
        ("or_delta_encode", [C.c_int, vp, sz, vp, sz]),
        ("or_delta_encode_shape", [C.c_int, vp, sz, sz, sz, vp, sz]),
        ("or_dict_encode", [vp, sz, sz, vp, sz, szp, vp, sz, szp]),
        ("or_rle_bool_encode", [vp, sz, vp, sz]),
        ("or_plain_encode_ba", [vp, vp, sz, C.c_int, vp, sz]),
        ("or_delta_length_encode", [vp, vp, sz, vp, sz]),
        ("or_delta_byte_array_encode", [vp, vp, sz, vp, sz]),
    ]:
        f = getattr(L, name)
        f.restype = sz
        f.argtypes = args


_FAIL = (1 << 64) - 1


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def _bytes_arr(b):
    return np.frombuffer(bytes(b), dtype=np.uint8).copy() if len(b) else np.zeros(1, np.uint8)


# --------------------------------------------------------------------------- decoders

def rle_decode(data, bit_width, n, type_size=4):
    """RleDecoder::set_data + get_batch::<T> (rle.rs:352-434). Returns (status, values)."""
    d = _bytes_arr(data)
    dt = {1: np.uint8, 2: np.int16, 4: np.int32, 8: np.int64}[type_size]
    out = np.zeros(max(n, 1), dtype=dt)
    r = C.c_size_t(0)
    st = lib().or_rle_decode(_ptr(d), len(data), bit_width, type_size, _ptr(out), n, C.byref(r))
    return st, out[: r.value]


def rle_decode_dict(data, bit_width, dictionary, n):
    """RleDecoder::get_batch_with_dict (rle.rs:437-487) over a numpy dictionary."""
    d = _bytes_arr(data)
    dic = np.ascontiguousarray(dictionary)
    out = np.zeros(max(n, 1), dtype=dic.dtype)
    r = C.c_size_t(0)
    st = lib().or_rle_decode_dict(_ptr(d), len(data), bit_width, _ptr(dic), len(dic),
                                  dic.dtype.itemsize, _ptr(out), n, C.byref(r))
    return st, out[: r.value]


def plain_decode(ptype, data, num_values, n, type_length=-1):
    d = _bytes_arr(data)
    if ptype in NP_DTYPE:
        out = np.zeros(max(n, 1), dtype=NP_DTYPE[ptype])
    else:
        out = np.zeros(max(n, 1) * TYPE_SIZE[ptype], dtype=np.uint8)
    r = C.c_size_t(0)
    st = lib().or_plain_decode(ptype, type_length, _ptr(d), len(data), num_values, _ptr(out), n,
                               C.byref(r))
    if ptype == INT96:
        return st, out[: r.value * 12].reshape(-1, 12)
    return st, out[: r.value]


def delta_decode(ptype, data, n):
    """DeltaBitPackDecoder set_data + get (decoding.rs:501-572).
    Returns (status, values, get_offset, header_count)."""
    d = _bytes_arr(data)
    out = np.zeros(max(n, 1), dtype=np.int32 if ptype == INT32 else np.int64)
    r, off, tot = C.c_size_t(0), C.c_size_t(0), C.c_size_t(0)
    st = lib().or_delta_decode(ptype, _ptr(d), len(data), _ptr(out), n, C.byref(r), C.byref(off),
                               C.byref(tot))
    return st, out[: r.value], off.value, tot.value


class BitReaderPy:
    """Thin wrapper over the restated BitReader (bit_util.rs:369-608)."""

    def __init__(self, data):
        self._buf = _bytes_arr(data)
        self.r = BitReader()
        lib().or_br_init(C.byref(self.r), _ptr(self._buf), len(data))

    def get_value(self, bits, type_size=8):
        v = C.c_uint64(0)
        ok = lib().or_br_get_value(C.byref(self.r), bits, type_size, C.byref(v))
        return v.value if ok else None

    def get_aligned(self, nbytes):
        v = C.c_uint64(0)
        ok = lib().or_br_get_aligned(C.byref(self.r), nbytes, C.byref(v))
        return v.value if ok else None

    def get_vlq_int(self):
        v = C.c_int64(0)
        return v.value if lib().or_br_get_vlq_int(C.byref(self.r), C.byref(v)) else None

    def get_zigzag_vlq_int(self):
        v = C.c_int64(0)
        return v.value if lib().or_br_get_zigzag_vlq_int(C.byref(self.r), C.byref(v)) else None

    def get_byte_offset(self):
        return lib().or_br_get_byte_offset(C.byref(self.r))

    def get_batch(self, n, bits, type_size=4):
        dt = {1: np.uint8, 2: np.int16, 4: np.int32, 8: np.int64}[type_size]
        out = np.zeros(max(n, 1), dtype=dt)
        r = lib().or_br_get_batch(C.byref(self.r), _ptr(out), n, type_size, bits)
        return out[:r]


# --------------------------------------------------------------------------- encoders

def _enc(fn, *args, cap):
    out = np.zeros(cap, dtype=np.uint8)
    n = fn(*args, _ptr(out), cap)
    if n == _FAIL:
        raise ValueError("encoder overflow")
    return out[:n].tobytes()


def rle_encode(values, bit_width, cap=None):
    v = np.ascontiguousarray(values, dtype=np.uint64)
    cap = cap or (len(v) * 9 + 64)
    return _enc(lib().or_rle_encode, _ptr(v), len(v), bit_width, cap=cap)


def level_encode(levels, max_level, encoding=RLE, v2=False):
    v = np.ascontiguousarray(levels, dtype=np.int16)
    cap = len(v) * 4 + 64
    return _enc(lib().or_level_encode, encoding, int(v2), max_level, _ptr(v), len(v), cap=cap)


def plain_encode(ptype, values):
    v = np.ascontiguousarray(values)
    cap = v.nbytes + 64
    return _enc(lib().or_plain_encode, ptype, _ptr(v), len(v), cap=cap)


def delta_encode(ptype, values, block_size=128, mini_blocks=4):
    """DeltaBitPackEncoder (encoding.rs:534-714); the reference writes 128 / 4 x 32 blocks,
    other shapes exercise what the decoder accepts (decoding.rs:501-533)."""
    v = np.ascontiguousarray(values, dtype=np.int32 if ptype == INT32 else np.int64)
    cap = len(v) * 10 + 256 + (16 + mini_blocks) * (len(v) // max(block_size, 1) + 2)
    if (block_size, mini_blocks) == (128, 4):
        return _enc(lib().or_delta_encode, ptype, _ptr(v), len(v), cap=cap)
    return _enc(lib().or_delta_encode_shape, ptype, _ptr(v), len(v), block_size, mini_blocks, cap=cap)


def dict_encode(values):
    """Returns (dict_page_bytes, index_page_bytes, num_uniques)."""
    v = np.ascontiguousarray(values)
    es = v.dtype.itemsize
    dcap = v.nbytes + 64
    icap = len(v) * 9 + 64
    dout = np.zeros(dcap, np.uint8)
    iout = np.zeros(icap, np.uint8)
    dl, il = C.c_size_t(0), C.c_size_t(0)
    nu = lib().or_dict_encode(_ptr(v), len(v), es, _ptr(dout), dcap, C.byref(dl), _ptr(iout),
                              icap, C.byref(il))
    if nu == _FAIL:
        raise ValueError("dict encoder overflow")
    return dout[: dl.value].tobytes(), iout[: il.value].tobytes(), nu


def rle_bool_encode(values):
    v = np.ascontiguousarray(values, dtype=np.uint8)
    return _enc(lib().or_rle_bool_encode, _ptr(v), len(v), cap=len(v) + 64)


def _ba_args(values):
    lens = np.array([len(x) for x in values], dtype=np.int64)
    offs = np.zeros(len(values) + 1, dtype=np.int64)
    np.cumsum(lens, out=offs[1:])
    data = _bytes_arr(b"".join(values))
    return data, offs


def plain_encode_ba(values, fixed=False):
    data, offs = _ba_args(values)
    cap = int(offs[-1]) + 4 * len(values) + 64
    return _enc(lib().or_plain_encode_ba, _ptr(data), _ptr(offs), len(values), int(fixed), cap=cap)


def delta_length_encode(values):
    data, offs = _ba_args(values)
    cap = int(offs[-1]) + 10 * len(values) + 256
    return _enc(lib().or_delta_length_encode, _ptr(data), _ptr(offs), len(values), cap=cap)


def delta_byte_array_encode(values):
    data, offs = _ba_args(values)
    cap = int(offs[-1]) + 20 * len(values) + 512
    return _enc(lib().or_delta_byte_array_encode, _ptr(data), _ptr(offs), len(values), cap=cap)


# --------------------------------------------------------------------------- column chunk

class PageSpec:
    """An uncompressed page, as Page in column/page.rs:28-57."""

    def __init__(self, page_type, buf, num_values, encoding, def_encoding=RLE,
                 rep_encoding=RLE, def_len=0, rep_len=0):
        self.page_type, self.buf, self.num_values = page_type, bytes(buf), num_values
        self.encoding, self.def_encoding, self.rep_encoding = encoding, def_encoding, rep_encoding
        self.def_len, self.rep_len = def_len, rep_len


def read_column(ptype, pages, max_def=0, max_rep=0, type_length=-1, batch_size=1024,
                want_def=True, want_rep=True, values_cap=None, def_cap=None, rep_cap=None):
    """ColumnReaderImpl::read_batch over all pages (column/reader.rs:159-265), every call with
    slices of values_cap / def_cap / rep_cap elements (default batch_size).

    Returns dict(status, message, def, rep, values, offsets, bytes, batches, counts: the
    (values_read, levels_read) of each call)."""
    col = Column(ptype, type_length, max_def, max_rep)
    keep = []
    arr = (Page * max(len(pages), 1))()
    for i, p in enumerate(pages):
        b = _bytes_arr(p.buf)
        keep.append(b)
        arr[i] = Page(p.page_type, b.ctypes.data, len(p.buf), p.num_values, p.encoding,
                      p.def_encoding, p.rep_encoding, p.def_len, p.rep_len)
    res = ColumnResult()
    bs = batch_size or 1024
    caps = [bs] + [c for c in (values_cap, def_cap, rep_cap) if c]
    ccap = 2 * min(sum(p.num_values for p in pages) // max(1, min(caps)) + 2 * len(pages) + 8, 1 << 20)
    counts = np.zeros(ccap, np.uint64)
    st = lib().or_read_column_caps(C.byref(col), arr, len(pages), bs,
                                   bs if values_cap is None else values_cap,
                                   bs if def_cap is None else def_cap,
                                   bs if rep_cap is None else rep_cap, int(want_def),
                                   int(want_rep), counts.ctypes.data, ccap, C.byref(res))
    out = {"status": st, "message": res.message.decode(errors="replace"),
           "batches": res.num_batches,
           "counts": [(int(counts[2 * k]), int(counts[2 * k + 1])) for k in range(min(res.num_batches, ccap // 2))]}
    nl, nv = res.num_levels, res.num_values
    out["def"] = (np.ctypeslib.as_array(res.def_levels, (nl,)).copy()
                  if res.def_levels and nl else np.zeros(0, np.int16))
    out["rep"] = (np.ctypeslib.as_array(res.rep_levels, (nl,)).copy()
                  if res.rep_levels and nl else np.zeros(0, np.int16))
    if ptype in (BYTE_ARRAY, FIXED_LEN_BYTE_ARRAY):
        offs = np.ctypeslib.as_array(res.offsets, (nv + 1,)).copy() if res.offsets else np.zeros(1, np.int64)
        nb = res.num_bytes
        out["offsets"] = offs
        out["bytes"] = (np.ctypeslib.as_array(res.bytes, (nb,)).copy().tobytes()
                        if res.bytes and nb else b"")
        out["values"] = [out["bytes"][offs[i]:offs[i + 1]] for i in range(nv)]
    else:
        es = TYPE_SIZE[ptype]
        raw = (np.ctypeslib.as_array(res.values, (nv * es,)).copy()
               if res.values and nv else np.zeros(0, np.uint8))
        if ptype == INT96:
            out["values"] = raw.reshape(-1, 12)
        else:
            out["values"] = raw.view(NP_DTYPE[ptype])
    lib().or_column_result_free(C.byref(res))
    return out
