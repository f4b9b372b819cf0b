"""DELTA_BYTE_ARRAY decode of one 1 M-value page (sorted URL-like strings, the shape of
tests/test_gpu_bytes.py::test_delta_byte_array_prefix_chains "million"): GPU (pqg_decode_chunk,
device-resident page, HIP events) against the C oracle's read_batch (one thread), values compared.
Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-rs_amd"), os.path.join(ROOT, "oracle")]


def main():
    import torch

    import pqgpu
    import pyoracle as oracle  # the checker and the CPU baseline only
    rng = np.random.default_rng(62)
    xs = np.sort(rng.integers(0, 10 ** 12, 1 << 20))
    vals = [b"http://www.example.com/%d/%012d" % (x % 7, x) + b"/q" * int(x % 5) for x in xs]
    body = oracle.delta_byte_array_encode(vals)
    spec = oracle.PageSpec(oracle.PAGE_DATA, body, len(vals), oracle.DELTA_BYTE_ARRAY)
    t = time.perf_counter()
    ref = oracle.read_column(oracle.BYTE_ARRAY, [spec])
    cpu_s = time.perf_counter() - t
    ctx = pqgpu.Context(0)
    blob, pages = pqgpu.make_pages([spec])
    dev = torch.device("cuda", 0)
    d_blob = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
    nbytes = sum(len(v) for v in vals)
    d_val = torch.empty(nbytes + 64, dtype=torch.uint8, device=dev)
    d_off = torch.empty(len(vals) + 2, dtype=torch.int64, device=dev)
    col = pqgpu.Column(pqgpu.BYTE_ARRAY, -1, 0, 0)
    s = torch.cuda.current_stream(dev).cuda_stream

    def once():
        out = pqgpu.Output(None, None, d_val.data_ptr(), nbytes + 64, d_off.data_ptr(), len(vals) + 1, 0, 0, 0)
        ctx.decode_async(col, d_blob.data_ptr(), len(blob), pages, out, s, npages=1)
        st, _ = ctx.sync()
        assert st == 0, ctx.error_message()
        return out

    for _ in range(3):
        once()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        once()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    same = d_val[:nbytes].cpu().numpy().tobytes() == ref["bytes"] and \
        np.array_equal(d_off[:len(vals) + 1].cpu().numpy(), ref["offsets"])
    print(json.dumps({"what": "DELTA_BYTE_ARRAY, one page of 2^20 values", "values": len(vals), "bytes_out": nbytes,
                      "page_bytes": len(body), "gpu_ms_per_decode": ms,
                      "gpu_values_per_s": len(vals) / (ms * 1e-3), "cpu_port_s": cpu_s,
                      "cpu_values_per_s": len(vals) / cpu_s, "identical_to_oracle": bool(same),
                      "note": "gpu time: one pqg_decode_chunk + pqg_sync per decode (host enqueue included)"}))
    ctx.close()


if __name__ == "__main__":
    main()
