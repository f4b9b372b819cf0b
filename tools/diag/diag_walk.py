"""Diagnostics: per-page verdicts of the level-path segment walks (k_lv_segscan) from a PQG_DIAG
build (make -C parquet-rs_amd DIAG=1 -> lib_diag/libpqgpu.so). Not part of the product or the
bench: PQG_DEBUG is read only by the diagnostic library.

    PQG_DEBUG=64 python tools/diag/diag_walk.py --p-null 0.5 [--n 2e8]     # page verdicts
    PQG_DEBUG=128 python tools/diag/diag_walk.py --p-null 0.5 --stamps      # segment walk cycles
"""
import argparse
import collections
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
    ap.add_argument("--p-null", type=float, default=0.5)
    ap.add_argument("--n", type=float, default=2e8)
    ap.add_argument("--stamps", action="store_true")
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
    ctx = pqgpu.Context(torch.cuda.current_device(), timing=True)
    s = torch.cuda.current_stream().cuda_stream
    bench.decode_once(ctx, w, s)
    st, bad = ctx.sync()
    assert st == 0, (st, bad)
    if a.stamps:
        nwin = sum((w.pages[i].nbytes + 1023) // 1024 for i in range(w.npages))
        nseg = nwin // 16 + w.npages + 1
        buf = np.zeros(4 * nseg, np.uint64)
        assert L.pqg_debug_read(ctx.h, buf.ctypes.data, buf.size) == 0
        d = buf.reshape(nseg, 4).astype(np.float64)
        d = d[d[:, 3] > 0]
        nh = d[:, 3]
        print(f"segments walked {len(d)}  headers/segment mean {nh.mean():.0f} max {nh.max():.0f}")
        med = np.median(nh)
        print("walk length / median:", {f">{r}x": int((nh > r * med).sum()) for r in (1.3, 1.8, 2.5)})
        for k, name in enumerate(("region", "hops", "batch")):
            print(f"{name:8s} mean {d[:, k].mean():10.0f} max {d[:, k].max():10.0f} cycles  per header {d[:, k].sum() / nh.sum():7.1f}")
        tm = ctx.timings()
        print("levels_kernel_ms", tm.levels_kernel_ms)
        return
    buf = np.zeros(8 * w.npages, np.uint64)
    assert L.pqg_debug_read(ctx.h, buf.ctypes.data, buf.size) == 0
    d = buf.reshape(w.npages, 8)
    print("verdicts", collections.Counter(d[:, 0].tolist()))
    print("deciding segment status", collections.Counter(d[:, 2].tolist()))
    for i in range(min(8, w.npages)):
        print("page", i, "verdict", d[i, 0], "seg", d[i, 1], "status", d[i, 2], "runs", d[i, 3], "out", d[i, 4],
              "nseg", d[i, 5], "lastpos", d[i, 6], "next bexit", d[i, 7])


if __name__ == "__main__":
    main()
