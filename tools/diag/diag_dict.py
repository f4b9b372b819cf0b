"""Diagnostics: where k_dict_win's workgroups spend their cycles on config 3 (PQG_DIAG build,
PQG_DEBUG=4096): thread 0's s_memtime per phase -- run records, block descriptors, the first
fill issued + index decode (its loads wait for that fill too),
window fills (issue to the barrier after the wait), gathers, stores.

    make -C parquet-rs_amd DIAG=1 && PQG_DEBUG=4096 python tools/diag/diag_dict.py
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "parquet-rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools", "gen"))
sys.path.insert(0, ROOT)


def main():
    import torch
    import pqgpu
    pqgpu.LIB_PATH = os.path.join(ROOT, "parquet-rs_amd", os.environ.get("PQG_DIAG_LIBDIR", "lib_diag"),
                                  "libpqgpu.so")
    L = pqgpu.lib()
    L.pqg_debug_read.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    import bench
    args = bench.parse(["--config", "dict"])
    w = bench.Workload(pqgpu, args, 0, "dict", 0.0)
    ctx = pqgpu.Context(torch.cuda.current_device())
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        bench.decode_once(ctx, w, s)
        st, bad = ctx.sync()
        assert st == 0, (st, bad)
    n = int(args.n) // 4096 // 8 + 64  # (the buffer: one 64-byte record per workgroup)
    buf = np.zeros(8 * n, np.uint64)
    assert L.pqg_debug_read(ctx.h, buf.ctypes.data, buf.size) == 0
    raw = buf.reshape(n, 8)
    raw = raw[raw[:, 7] > 0].astype(np.float64)
    nb = raw[:, 7].sum()
    print(f"workgroups {len(raw)}, workgroups of 8 tiles {nb:.0f}")
    tot = raw[:, :6].sum(axis=1)
    for k, name in enumerate(("run records", "block descriptors", "fill 1 + decode", "window fills", "gathers", "stores")):
        print(f"  {name:18s} {raw[:, k].sum() / nb:9.0f} cycles per workgroup ({raw[:, k].sum() / tot.sum():.2f})")
    print(f"  {'total':18s} {tot.sum() / nb:9.0f} cycles per workgroup")


if __name__ == "__main__":
    main()
