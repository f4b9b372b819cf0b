"""Host-side cost of pqg_decode_chunk per column of an alltypes row group (enqueue only, the
GPU idle and the staging slot free: a sync after each call). Not part of the product."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for d in ("", "parquet-rs_amd", os.path.join("tools", "gen")):
    sys.path.insert(0, os.path.join(ROOT, d))


def main():
    import torch
    import pqgpu
    import pqgtools
    import bench
    args = bench.parse(["--config", "alltypes", "--rowgroups", "1", "--rg-rows", str(1 << 23)])
    w = bench.AlltypesWorkload(pqgpu, args, 0)
    ctx = pqgpu.Context(torch.cuda.current_device())
    s = torch.cuda.current_stream().cuda_stream
    for j, (name, pt) in enumerate(pqgtools.ALLTYPES):
        ch = w.chunks[0][j]
        ts = []
        for r in range(8):
            t0 = time.perf_counter()
            ctx.decode_async(w.cols[j], w.d_blob.data_ptr() + w.base[0], w.info[0].blob_len, ch, w.out[0][j][3], s)
            ts.append(time.perf_counter() - t0)
            ctx.sync()
        print(f"{name:16s} host us per decode call: {sorted(ts)[len(ts) // 2] * 1e6:8.1f}", flush=True)
    # raw HIP launch cost for comparison: an empty torch op (one kernel)
    x = torch.zeros(16, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(1000):
        x.add_(1)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"torch add_ launch: {(t1 - t0) * 1e3:.1f} us per call")


if __name__ == "__main__":
    main()
