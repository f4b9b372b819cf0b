"""ctypes binding of libpqgtools.so: the reference-identical page writers and BASELINE.json
workload generators used by bench.py and the tests (tools/gen/pqg_gen.h). Not part of the
decode library (parquet-rs_amd/lib/libpqgpu.so)."""
import ctypes as C
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libpqgtools.so")

EXPORTS = ["pqg_encode_rle", "pqg_encode_levels_v1", "pqg_encode_delta", "pqg_encode_dict_indices",
           "pqg_gen_levels_plain", "pqg_gen_dict_int64", "pqg_gen_delta_int64",
           "pqg_truth_levels_plain", "pqg_truth_dict_int64", "pqg_truth_delta_int64",
           "pqg_gen_alltypes", "pqg_alltypes_copy", "pqg_alltypes_free", "pqg_truth_alltypes",
           "pqg_write_alltypes_file", "pqg_gen_levels_plain_pages", "pqg_gen_dict_int64_pages",
           "pqg_gen_delta_int64_pages"]

# alltypes_plain schema (data/alltypes_plain.parquet): 11 OPTIONAL leaves, physical types
ALLTYPES = [("id", 1), ("bool_col", 0), ("tinyint_col", 1), ("smallint_col", 1), ("int_col", 1),
            ("bigint_col", 2), ("float_col", 4), ("double_col", 5), ("date_string_col", 6),
            ("string_col", 6), ("timestamp_col", 3)]


class WorkloadInfo(C.Structure):
    _fields_ = [("blob_len", C.c_uint64), ("npages", C.c_uint32), ("total_levels", C.c_uint64),
                ("total_values", C.c_uint64)]


class AlltypesInfo(C.Structure):
    _fields_ = [("blob_len", C.c_uint64), ("rows", C.c_uint64), ("npages", C.c_uint32),
                ("chunk_first", C.c_uint32 * 12), ("chunk_offset", C.c_uint64 * 12),
                ("num_values", C.c_uint64 * 11), ("value_bytes", C.c_uint64 * 11)]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        import pqgpu  # Page layout
        Page = pqgpu.Page
        L = C.CDLL(LIB_PATH)
        vp, u64, i32, u32 = C.c_void_p, C.c_uint64, C.c_int, C.c_uint32
        L.pqg_gen_levels_plain.argtypes = [u64, C.c_double, u32, u64, i32, vp, u64,
                                           C.POINTER(Page), u32, C.POINTER(WorkloadInfo)]
        L.pqg_gen_dict_int64.argtypes = [u64, u32, u32, u64, i32, vp, u64, C.POINTER(Page), u32,
                                         C.POINTER(WorkloadInfo)]
        L.pqg_gen_delta_int64.argtypes = [u64, i32, u32, i32, i32, u64, i32, vp, u64,
                                          C.POINTER(Page), u32, C.POINTER(WorkloadInfo)]
        L.pqg_gen_levels_plain_pages.argtypes = [u64, C.c_double, u32, u64, u32, u32, i32, vp, u64,
                                                 C.POINTER(Page), u32, C.POINTER(WorkloadInfo)]
        L.pqg_gen_dict_int64_pages.argtypes = [u64, u32, u32, u64, u32, u32, i32, vp, u64, C.POINTER(Page), u32,
                                               C.POINTER(WorkloadInfo)]
        L.pqg_gen_delta_int64_pages.argtypes = [u64, i32, u32, i32, i32, u64, u32, u32, i32, vp, u64,
                                                C.POINTER(Page), u32, C.POINTER(WorkloadInfo)]
        L.pqg_truth_levels_plain.argtypes = [u64, C.c_double, u32, u64, u32, vp, vp]
        L.pqg_truth_levels_plain.restype = u64
        L.pqg_truth_dict_int64.argtypes = [u64, u32, u32, u64, u32, vp]
        L.pqg_truth_dict_int64.restype = u64
        L.pqg_truth_delta_int64.argtypes = [u64, i32, u32, u64, u32, vp]
        L.pqg_truth_delta_int64.restype = u64
        L.pqg_encode_rle.restype = u64
        L.pqg_encode_rle.argtypes = [vp, u64, i32, vp, u64]
        L.pqg_encode_levels_v1.restype = u64
        L.pqg_encode_levels_v1.argtypes = [vp, u64, C.c_int16, vp, u64]
        L.pqg_encode_delta.restype = u64
        L.pqg_encode_delta.argtypes = [i32, vp, u64, i32, i32, vp, u64]
        L.pqg_encode_dict_indices.restype = u64
        L.pqg_encode_dict_indices.argtypes = [vp, u64, i32, vp, u64]
        L.pqg_gen_alltypes.restype = vp
        L.pqg_gen_alltypes.argtypes = [u64, u64, C.c_double, u64, i32, C.POINTER(AlltypesInfo)]
        L.pqg_alltypes_copy.argtypes = [vp, vp, u64, C.POINTER(Page), u32]
        L.pqg_alltypes_free.argtypes = [vp]
        L.pqg_truth_alltypes.restype = u64
        L.pqg_truth_alltypes.argtypes = [u64, u64, i32, C.c_double, u64, vp, vp, vp]
        L.pqg_write_alltypes_file.argtypes = [C.c_char_p, u64, u32, u64, C.c_double, u64, i32, i32]
        _lib = L
    return _lib


def alltypes_row_group(rows, row0, p_null, seed, threads=16, out=None):
    """One alltypes row group: (host bytes as numpy uint8, pqgpu.Page array, AlltypesInfo).
    `out`, if given, is a uint8 array (e.g. pinned) the pages are laid out into."""
    import numpy as np
    import pqgpu
    L = lib()
    info = AlltypesInfo()
    h = L.pqg_gen_alltypes(rows, row0, p_null, seed, threads, C.byref(info))
    if not h:
        raise RuntimeError("pqg_gen_alltypes failed")
    try:
        blob = np.zeros(info.blob_len + 64, np.uint8) if out is None else out
        assert blob.nbytes >= info.blob_len
        pages = (pqgpu.Page * info.npages)()
        st = L.pqg_alltypes_copy(h, blob.ctypes.data, blob.nbytes, pages, info.npages)
        assert st == 0, st
    finally:
        L.pqg_alltypes_free(h)
    return blob, pages, info


def alltypes_truth(row0, rows, col, p_null, seed, value_bytes):
    """Raw content of one alltypes column over rows [row0, row0 + rows): (levels, values bytes,
    offsets or None)."""
    import numpy as np
    L = lib()
    lv = np.zeros(rows, np.int16)
    vals = np.zeros(max(value_bytes, 1), np.uint8)
    ba = ALLTYPES[col][1] == 6
    offs = np.zeros(rows + 1, np.int64) if ba else None
    nv = L.pqg_truth_alltypes(row0, rows, col, p_null, seed, lv.ctypes.data, vals.ctypes.data,
                              offs.ctypes.data if ba else None)
    return lv, vals[:value_bytes], (offs[:nv + 1] if ba else None)


def write_alltypes_file(path, rows_per_group, row_groups, row0=0, p_null=0.0, seed=0x5EED0005, codec=0,
                        threads=16):
    """The alltypes workload's row groups as a parquet file (codec 0 none, 1 SNAPPY, 2 GZIP)."""
    st = lib().pqg_write_alltypes_file(os.fsencode(path), rows_per_group, row_groups, row0, p_null, seed,
                                       codec, threads)
    if st:
        raise RuntimeError("pqg_write_alltypes_file failed: %d" % st)


def _delta_i32(vals):
    """DeltaBitPackEncoder<Int32Type> of vals (encoding.rs:534-714, the writer's 128 / 4 blocks)."""
    import numpy as np
    v = np.ascontiguousarray(vals, dtype=np.int32)
    cap = 64 + 8 * len(v) + 1024
    out = (C.c_uint8 * cap)()
    n = lib().pqg_encode_delta(1, v.ctypes.data, len(v), 128, 4, out, cap)
    assert n > 0
    return bytes(out[:n])


def url_values(n, seed):
    """n sorted URL-like byte strings ('http://www.example.com/' + a path of digits and letters of
    2..24 bytes), the DELTA_BYTE_ARRAY bench shape: long shared prefixes, short suffixes."""
    import numpy as np
    rng = np.random.default_rng(seed)
    keys = np.sort(rng.integers(0, 10 ** 12, n))
    tails = rng.integers(0, 10 ** 6, n)
    return [b"http://www.example.com/%012d/%x" % (int(k), int(t)) for k, t in zip(keys, tails)]


def delta_byte_array_body(vals):
    """DeltaByteArrayEncoder (encoding.rs:813-889): prefix lengths against the previous value,
    suffix lengths (both DELTA_BINARY_PACKED INT32), then the suffixes."""
    import os.path
    pre = [0] * len(vals)
    prev = b""
    for i, v in enumerate(vals):
        k = len(os.path.commonprefix([prev, v]))
        pre[i] = k
        prev = v
    sufs = [v[k:] for v, k in zip(vals, pre)]
    return _delta_i32(pre) + _delta_i32([len(s) for s in sufs]) + b"".join(sufs)


def delta_length_body(vals):
    """DeltaLengthByteArrayEncoder (encoding.rs:735-800): lengths (DELTA_BINARY_PACKED INT32)
    then the values' bytes."""
    return _delta_i32([len(v) for v in vals]) + b"".join(vals)
