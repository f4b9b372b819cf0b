"""Diagnostics: per-page cycle stamps of the level-path page walker (k_lv_walk) from a PQG_DIAG
build (make -C parquet-rs_amd DIAG=1 -> lib_diag/libpqgpu.so). Not part of the product or the
bench: PQG_DEBUG is read only by the diagnostic library.

    PQG_DEBUG=64 python tools/diag_walk.py --p-null 0.5 [--n 2e8]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parquet-rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools", "gen"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--p-null", type=float, default=0.5)
    ap.add_argument("--n", type=float, default=2e8)
    a = ap.parse_args()
    import torch
    import pqgpu
    pqgpu.LIB_PATH = os.path.join(ROOT, "parquet-rs_amd", "lib_diag", "libpqgpu.so")
    L = pqgpu.lib()
    L.pqg_debug_read.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    import bench
    args = bench.parse(["--n", str(a.n), "--p-null", str(a.p_null)])
    w = bench.Workload(pqgpu, args, 0, "levels", a.p_null)
    ctx = pqgpu.Context(torch.cuda.current_device(), timing=True)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(2):
        bench.decode_once(ctx, w, s)
        st, bad = ctx.sync()
        assert st == 0, (st, bad)
    buf = np.zeros(8 * w.npages, np.uint64)
    assert L.pqg_debug_read(ctx.h, buf.ctypes.data, buf.size) == 0
    d = buf.reshape(w.npages, 8).astype(np.float64)
    reg, hop, bat, nh, status = d[:, 0], d[:, 1], d[:, 2], d[:, 3], d[:, 4]
    tot = reg + hop + bat
    print(f"pages {w.npages}  status counts {np.bincount(status.astype(int))}")
    print(f"headers/page mean {nh.mean():.0f}")
    for name, v in (("region", reg), ("hops", hop), ("batch", bat), ("total", tot)):
        print(f"{name:8s} mean {v.mean():10.0f}  max {v.max():10.0f} cycles   per header {v.mean() / max(nh.mean(), 1):8.1f}")
    tm = ctx.timings()
    print("levels_kernel_ms", tm.levels_kernel_ms)


if __name__ == "__main__":
    main()
