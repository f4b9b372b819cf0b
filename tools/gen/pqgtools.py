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
           "pqg_truth_levels_plain", "pqg_truth_dict_int64", "pqg_truth_delta_int64"]


class WorkloadInfo(C.Structure):
    _fields_ = [("blob_len", C.c_uint64), ("npages", C.c_uint32), ("total_levels", C.c_uint64),
                ("total_values", C.c_uint64)]


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
        _lib = L
    return _lib
