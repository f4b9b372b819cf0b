"""Diagnostics: where the walked-page dictionary emit (k_lv_emit_walk<LvDictOut>) spends its
cycles on config 5 (PQG_DIAG build, PQG_DEBUG=1024): per wave s_memtime cycles in the run bounds
and records, the payload staging and the writes by value size, per unit and per output.

    make -C parquet-rs_amd DIAG=1 && PQG_DEBUG=1024 python tools/diag/diag_walkemit.py [--rowgroups 2]
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
    ap.add_argument("--rowgroups", type=int, default=2)
    a = ap.parse_args()
    import torch
    import pqgpu
    pqgpu.LIB_PATH = os.path.join(ROOT, "parquet-rs_amd", os.environ.get("PQG_DIAG_LIBDIR", "lib_diag"),
                                  "libpqgpu.so")
    L = pqgpu.lib()
    L.pqg_debug_read.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    import bench
    args = bench.parse(["--config", "alltypes", "--rowgroups", str(a.rowgroups)])
    w = bench.AlltypesWorkload(pqgpu, args, 0, 1)
    ctx = pqgpu.Context(torch.cuda.current_device())
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(2):
        w.decode_step(ctx, s)
        r = ctx.sync_detail()
        assert r[0] == 0, r
    n = 2048 * 16
    buf = np.zeros(8 * n, np.uint64)
    assert L.pqg_debug_read(ctx.h, buf.ctypes.data, buf.size) == 0
    d = buf.reshape(n, 8).astype(np.float64)
    d_keep = d[:, 5] > 0
    d = d[d_keep]
    f4 = (buf.reshape(n, 8)[:, 6] & 0xFFFFFFFF).astype(np.float64)[d_keep]
    f8 = (buf.reshape(n, 8)[:, 6] >> 32).astype(np.float64)[d_keep]
    d[:, 6] = f4 + f8
    units, of, ob = d[:, 5].sum(), d[:, 6].sum(), d[:, 7].sum()
    print(f"waves {len(d)} units {units:.0f} outputs fixed {of:.0f} byte-array {ob:.0f}")
    tot = d[:, :5].sum()
    for k, name in enumerate(("bounds+records", "staging", "writes BA", "writes 4 B", "writes 8 B")):
        print(f"  {name:15s} {d[:, k].sum() / units:9.0f} cycles per unit  ({d[:, k].sum() / tot:.2f} of the stamped)")
    print(f"  per output: fixed {(d[:, 3].sum() + d[:, 4].sum()) / max(of, 1):.2f} (4 B {d[:, 3].sum() / max(f4.sum(), 1):.2f}, "
          f"8 B {d[:, 4].sum() / max(f8.sum(), 1):.2f}), BA {d[:, 2].sum() / max(ob, 1):.2f} cycles")
    busy = d[:, :5].sum(1)
    outs = d[:, 6] + d[:, 7]
    print(f"  wave busy cycles: mean {busy.mean():.0f} p50 {np.percentile(busy, 50):.0f} "
          f"p90 {np.percentile(busy, 90):.0f} max {busy.max():.0f}")
    print(f"  wave outputs: mean {outs.mean():.0f} p50 {np.percentile(outs, 50):.0f} "
          f"p90 {np.percentile(outs, 90):.0f} max {outs.max():.0f}; units: mean {d[:, 5].mean():.1f} max {d[:, 5].max():.0f}")
    top = np.argsort(busy)[-5:]
    for i in top:
        print(f"    busy {busy[i]:.0f}: units {d[i, 5]:.0f} outputs {outs[i]:.0f} (BA {d[i, 7]:.0f}) "
              + " ".join(f"{d[i, k]:.0f}" for k in range(5)))
    c = np.corrcoef(busy, outs)[0, 1]
    print(f"  correlation busy ~ outputs {c:.2f}")


if __name__ == "__main__":
    main()
