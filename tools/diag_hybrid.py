"""Diagnostic: phase shares of the RLE hybrid decoder (walker vs expanders vs barrier) from
in-kernel s_memtime stamps (debug mode 4), plus timings with expansion skipped (mode 1).
Not part of the product path; prints one JSON object per workload."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "parquet-rs_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import pqgpu  # noqa: E402
import bench  # noqa: E402

L = pqgpu.lib()
L.pqg_debug_set.argtypes = [C.c_int]
L.pqg_debug_read.argtypes = [C.c_void_p]
NAMES = ["walk_cyc", "exp_cyc", "exp_bar_cyc", "walk_bar_cyc", "batches", "hops", "windows",
         "loads", "tiles", "load_cyc", "wgs"]


def run(kind, p_null, n, mode, steps=3):
    class A:
        pass
    a = A()
    a.n, a.page_values, a.dict_size, a.delta_bits, a.block_size, a.mini_blocks = n, 1 << 20, 65536, 16, 512, 4
    a.threads, a.seed = 16, 0x5EED0000
    ctx = pqgpu.Context(0, timing=True)
    w = bench.Workload(pqgpu, a, 0, kind, p_null=p_null)
    stream = torch.cuda.current_stream().cuda_stream
    out = {}
    for m in mode:
        L.pqg_debug_set(m)
        per, tm = bench.time_steps(pqgpu, ctx, w, stream, steps, 1)
        st = np.zeros(16, np.uint64)
        L.pqg_debug_read(st.ctypes.data)
        d = {"mode": m, "ms": per * 1e3, "levels_ms": tm.levels_ms, "values_ms": tm.values_ms}
        if m & 4:
            wg = max(int(st[10]), 1)
            d.update({k: float(st[i]) / wg for i, k in enumerate(NAMES) if k != "wgs"})
            d["wgs_total"] = int(st[10])
        out[m] = d
    L.pqg_debug_set(0)
    ctx.close()
    return out


if __name__ == "__main__":
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else int(2e8)
    res = {}
    for kind, p in (("levels", 0.5), ("dict", None), ("levels", 0.1)):
        res[f"{kind}-{p}"] = run(kind, p, n, [0, 8, 4])
        print(json.dumps({f"{kind}-{p}": res[f"{kind}-{p}"]}), flush=True)
