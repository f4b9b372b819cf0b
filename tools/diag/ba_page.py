"""Times bench.py's 2^20-value DELTA_BYTE_ARRAY / DELTA_LENGTH_BYTE_ARRAY pages alone (for
rocprofv3 kernel stats of the byte-array path): python tools/diag/ba_page.py [dba|dlba ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    import pqgpu
    ctx = pqgpu.Context(torch.cuda.current_device())
    s = torch.cuda.current_stream().cuda_stream
    for enc in sys.argv[1:] or ["dba", "dlba"]:
        r = bench.run_bytes_page(pqgpu, ctx, s, enc, 5, 2)
        print(enc, json.dumps({k: r[k] for k in ("ms_per_step", "values_per_s", "page_bytes", "value_bytes")}),
              "frac", r["roofline"]["frac"], flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
