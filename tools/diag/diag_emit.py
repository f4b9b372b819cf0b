"""Diagnostics: where k_lv_emit's waves spend their cycles (PQG_DIAG build, PQG_DEBUG=256):
per window, the staging wait, chain / run placement, bitmap generation and output stores
(s_memtime stamps).

    make -C parquet-rs_amd DIAG=1 && PQG_DEBUG=256 python tools/diag/diag_emit.py --p-null 0.1
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
    ctx = pqgpu.Context(torch.cuda.current_device(), timing=True)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(2):
        bench.decode_once(ctx, w, s)
        st, bad = ctx.sync()
        assert st == 0, (st, bad)
    n = 2048 * 64
    buf = np.zeros(8 * n, np.uint64)
    assert L.pqg_debug_read(ctx.h, buf.ctypes.data, buf.size) == 0
    raw = buf.reshape(n, 8)
    raw = raw[raw[:, 4] > 0]
    cnt = raw[:, 4]
    miss = raw[:, 5].sum()
    tspec, nspec = raw[:, 6].astype(np.float64).sum(), raw[:, 7].sum()
    via, bmw = ((cnt >> 20) & 0xFFFFF).sum(), (cnt >> 40).sum()
    d = raw.astype(np.float64)
    d[:, 4] = (cnt & 0xFFFFF).astype(np.float64)
    tot = d[:, 4].sum()
    print(f"waves {len(d)} windows {tot:.0f}: via the reference chain {via / tot:.3f} (missed {miss / tot:.5f}), "
          f"bitmap writes {bmw / tot:.3f}")
    for k, name in enumerate(("stage wait", "placement", "bitmap gen", "stores")):
        print(f"  {name:11s} {d[:, k].sum() / tot:9.0f} cycles per window (wave mean {d[:, k].mean():10.0f})")
    allc = d[:, :4].sum()
    print(f"  windows through the segment tables: {nspec / tot:.3f} of them, {tspec / max(nspec, 1):.0f} cycles each, "
          f"{tspec / allc:.2f} of all cycles")
    print("levels_kernel_ms", ctx.timings().levels_kernel_ms)


if __name__ == "__main__":
    main()
