"""Diagnostics: where the dense one-bit level kernels (pqg_lvd1.hpp: k_d1_tab, k_d1_emit) spend their
cycles (PQG_DIAG build, PQG_DEBUG=8192): thread 0's s_memtime per phase, summed over each
workgroup's segments, and the settle rounds (serial fallbacks count 1000 each).

    make -C parquet-rs_amd DIAG=1 && PQG_DEBUG=8192 python tools/diag/diag_d1.py [--p-null 0.1]
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

PHASES = {0: ("stage", "chunk-0 entries", "guess walks", "settle", "scan + R store", "table walks", "-", "idle/next"),
          1: ("stage", "load R + chunk 0", "settle", "generate", "stores", "count", "-", "idle/next")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--p-null", type=float, default=0.1)
    a = ap.parse_args()
    import torch
    import pqgpu
    pqgpu.LIB_PATH = os.path.join(ROOT, "parquet-rs_amd", os.environ.get("PQG_DIAG_LIBDIR", "lib_diag"), "libpqgpu.so")
    L = pqgpu.lib()
    L.pqg_debug_read.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    import bench
    args = bench.parse(["--config", "levels", "--p-null", str(a.p_null)])
    w = bench.Workload(pqgpu, args, 0, "levels", p_null=a.p_null)
    ctx = pqgpu.Context(torch.cuda.current_device())
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(2):
        bench.decode_once(ctx, w, s)
        st, bad = ctx.sync()
        assert st == 0, (st, bad)
    buf = np.zeros(2 * 2048 * 8, np.uint64)
    assert L.pqg_debug_read(ctx.h, buf.ctypes.data, buf.size) == 0
    raw = buf.reshape(2, 2048, 8)
    for k in (0, 1):
        r = raw[k]
        segs = (r[:, 6] >> 32).sum()
        rounds = (r[:, 6] & 0xFFFF).sum()
        fb = ((r[:, 6] >> 16) & 0xFFFF).sum()
        print(f"{'k_d1_tab' if k == 0 else 'k_d1_emit'}: segments {segs}, settle rounds {rounds / max(segs, 1):.2f} per segment, "
              f"serial fallbacks {fb}")
        tot = r[:, [0, 1, 2, 3, 4, 5, 7]].astype(np.float64).sum()
        for j in (7, 0, 1, 2, 3, 4, 5):
            v = r[:, j].astype(np.float64).sum()
            print(f"  {PHASES[k][j]:18s} {v / max(segs, 1):9.0f} cycles per segment ({v / tot:.2f})")


if __name__ == "__main__":
    main()
