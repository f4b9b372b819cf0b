"""Diagnostics: where k_delta_page's workgroups spend their cycles on config 4 (PQG_DIAG build,
PQG_DEBUG=32): thread 0's s_memtime per tile phase -- stage install, header scan, unpack (with the
next tile's load issue), workgroup scan, stores.

    make -C parquet-rs_amd DIAG=1 && PQG_DEBUG=32 python tools/diag/diag_delta.py [--block 128]
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
    ap.add_argument("--block", type=int, default=0, help="128: the writer-default 128-value blocks of 4 x 32")
    a = ap.parse_args()
    import torch
    import pqgpu
    pqgpu.LIB_PATH = os.path.join(ROOT, "parquet-rs_amd", os.environ.get("PQG_DIAG_LIBDIR", "lib_diag"),
                                  "libpqgpu.so")
    L = pqgpu.lib()
    L.pqg_debug_read.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    import bench
    args = bench.parse(["--config", "delta"])
    blk = (128, 4) if a.block == 128 else None
    w = bench.Workload(pqgpu, args, 0, "delta", None, block=blk) if blk else bench.Workload(pqgpu, args, 0, "delta")
    ctx = pqgpu.Context(torch.cuda.current_device())
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        bench.decode_once(ctx, w, s)
        st, bad = ctx.sync()
        assert st == 0, (st, bad)
    n = 954 + 64
    buf = np.zeros(8 * n, np.uint64)
    assert L.pqg_debug_read(ctx.h, buf.ctypes.data, buf.size) == 0
    raw = buf.reshape(n, 8).astype(np.float64)
    raw = raw[raw[:, 7] > 0]
    nt = raw[:, 7].sum()
    tot = raw[:, :5].sum()
    print(f"pages {len(raw)}, tiles {nt:.0f}")
    for k, name in enumerate(("stage install", "header scan", "unpack", "scan", "stores")):
        print(f"  {name:14s} {raw[:, k].sum() / nt:8.0f} cycles per tile ({raw[:, k].sum() / tot:.2f})")
    print(f"  {'total':14s} {tot / nt:8.0f} cycles per tile; page max/mean {raw[:, :5].sum(1).max() / raw[:, :5].sum(1).mean():.2f}")


if __name__ == "__main__":
    main()
