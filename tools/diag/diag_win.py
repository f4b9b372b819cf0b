"""Diagnostics: where k_lv_win's waves spend their cycles on one-bit dense windows (PQG_DIAG
build, PQG_DEBUG=2048): stage wait, segment tables, the chain from 0 and the entry walks, the
reference choice (with the second chain when entry 0 is not on the majority chain), table writes.

    make -C parquet-rs_amd DIAG=1 && PQG_DEBUG=2048 python tools/diag/diag_win.py --p-null 0.1
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "parquet-rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools", "gen"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--p-null", type=float, default=0.1)
    ap.add_argument("--n", type=float, default=1e9)
    a = ap.parse_args()
    import torch
    import pqgpu
    pqgpu.LIB_PATH = os.path.join(ROOT, "parquet-rs_amd", os.environ.get("PQG_DIAG_LIBDIR", "lib_diag"),
                                  "libpqgpu.so")
    L = pqgpu.lib()
    L.pqg_debug_read.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    import bench
    args = bench.parse(["--n", str(a.n), "--p-null", str(a.p_null)])
    w = bench.Workload(pqgpu, args, 0, "levels", a.p_null)
    ctx = pqgpu.Context(torch.cuda.current_device())
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(2):
        bench.decode_once(ctx, w, s)
        st, bad = ctx.sync()
        assert st == 0, (st, bad)
    n = 2048 * 16
    buf = np.zeros(8 * n, np.uint64)
    assert L.pqg_debug_read(ctx.h, buf.ctypes.data, buf.size) == 0
    raw = buf.reshape(n, 8)
    raw = raw[raw[:, 5] > 0]
    d = raw.astype(np.float64)
    win, sec = d[:, 5].sum(), d[:, 6].sum()
    steps, tried, two = (raw[:, 7] & 0xFFFFFF).sum(), ((raw[:, 7] >> 24) & 0xFFFFF).sum(), (raw[:, 7] >> 44).sum()
    print(f"waves {len(d)} windows {win:.0f}, reference not from 0 {sec / win:.3f}, "
          f"entry-walk steps {steps / win:.1f} per window, chain from 0 failed {tried / win:.3f}, "
          f"second entry chain {two / win:.3f}")
    for k, name in enumerate(("stage wait", "segment tables", "chain + entries", "reference", "writes")):
        print(f"  {name:15s} {d[:, k].sum() / win:9.0f} cycles per window")


if __name__ == "__main__":
    main()
