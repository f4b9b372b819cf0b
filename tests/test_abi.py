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
    assert len(names) >= 20
    # bench/test writers live in the tools library, not in the decode library's ABI
    assert not any(n.startswith(("pqg_gen_", "pqg_encode_", "pqg_truth_")) for n in names)


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


def test_decode_library_has_no_tooling_symbols():
    """Workload generators and writers are tooling (tools/gen/libpqgtools.so): the product
    library neither exports nor links them."""
    import pqgpu
    lib = ctypes.CDLL(pqgpu.LIB_PATH)
    for name in ("pqg_gen_levels_plain", "pqg_encode_rle", "pqg_truth_delta_int64"):
        assert not hasattr(lib, name), name


def test_tools_library_exports():
    import pqgtools
    lib = pqgtools.lib()
    for name in pqgtools.EXPORTS:
        assert hasattr(lib, name), name


def test_no_gpu_needed_for_host_entry_points():
    """Host-only entry points (writers, file reader) run without a device."""
    import numpy as np
    import pqgtools
    L = pqgtools.lib()
    vals = np.arange(100, dtype=np.uint64) % 4
    out = np.zeros(256, np.uint8)
    n = L.pqg_encode_rle(vals.ctypes.data, 100, 2, out.ctypes.data, 256)
    assert 0 < n < 256
