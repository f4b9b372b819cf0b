"""The C-ABI library loads on a GPU-less host and exports every symbol include/*.h declares."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    inc = os.path.join(ROOT, "include")
    for f in os.listdir(inc):
        if not f.endswith(".h"):
            continue
        src = open(os.path.join(inc, f)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"\b(pqg_\w+)\s*\(", src):
            names.add(m.group(1))
    return sorted(names)


def test_header_declares_entry_points():
    names = declared_functions()
    assert "pqg_decode_chunk" in names and "pqg_column_reader_read_batch" in names
    assert len(names) >= 25


def test_library_exports_every_declared_symbol():
    import pqgpu
    lib = ctypes.CDLL(pqgpu.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(pqgpu.EXPORTS) <= set(declared_functions())


def test_status_codes_match_header():
    import pqgpu
    src = open(os.path.join(ROOT, "include", "pqgpu.h")).read()
    codes = dict(re.findall(r"#define (PQG_(?:OK|ERR_\w+)) (\d+)", src))
    assert int(codes["PQG_OK"]) == pqgpu.OK
    assert int(codes["PQG_ERR_EOF"]) == pqgpu.EOF
    assert int(codes["PQG_ERR_CAPACITY"]) == pqgpu.CAPACITY
    assert int(codes["PQG_ERR_HIP"]) == pqgpu.HIP


def test_no_gpu_needed_for_host_entry_points():
    """Host-only entry points (writers, file reader) run without a device."""
    import numpy as np
    import pqgpu
    L = pqgpu.lib()
    vals = np.arange(100, dtype=np.uint64) % 4
    out = np.zeros(256, np.uint8)
    n = L.pqg_encode_rle(vals.ctypes.data, 100, 2, out.ctypes.data, 256)
    assert 0 < n < 256
