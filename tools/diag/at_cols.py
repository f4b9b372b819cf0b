"""Per-column decode time of one alltypes row group (bench.py's AlltypesWorkload), HIP events
around each column's decode_async. Not part of the product or the bench.

    python tools/diag/at_cols.py [--rg-rows 8388608] [--reps 5]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for d in ("", "parquet-rs_amd", os.path.join("tools", "gen")):
    sys.path.insert(0, os.path.join(ROOT, d))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rg-rows", type=int, default=1 << 23)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    assert torch.cuda.is_available()
    import pqgpu
    import pqgtools
    import bench
    args = bench.parse(["--config", "alltypes", "--rowgroups", "1", "--rg-rows", str(a.rg_rows)])
    w = bench.AlltypesWorkload(pqgpu, args, 0, 1)
    ctx = pqgpu.Context(torch.cuda.current_device())
    stream = torch.cuda.current_stream()
    s = stream.cuda_stream
    rgd = pqgpu.RowGroupDecoder(torch.cuda.current_device())
    bench.alltypes_check(rgd, w, s)
    rgd.close()
    tot = 0.0
    for j, (name, pt) in enumerate(pqgtools.ALLTYPES):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ch = w.chunks[0][j]
        encs = sorted({(p.page_type, p.encoding) for p in ch})
        for r in range(a.reps + 1):
            if r == 1:
                ev[0].record(stream)
            ctx.decode_async(w.cols[j], w.d_blob.data_ptr() + w.base[0], w.info[0].blob_len, ch, w.out[0][j][3], s)
        ev[1].record(stream)
        st, bad = ctx.sync()
        assert st == 0, (name, st, bad)
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / a.reps
        tot += ms
        print(f"{name:16s} pages {len(ch):5d} {encs}  {ms:8.3f} ms", flush=True)
    print(f"total {tot:.3f} ms per row group")


if __name__ == "__main__":
    main()
