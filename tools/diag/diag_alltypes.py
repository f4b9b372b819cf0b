"""Diagnostics: decode one alltypes column chunk with the diagnostic library (PQG_DEBUG modes) and
compare levels / value count / values with the generator. Not part of the product or the bench.

    PQG_DEBUG=256 python tools/diag/diag_alltypes.py --col 6
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for d in ("parquet-rs_amd", os.path.join("tools", "gen"), "oracle"):
    sys.path.insert(0, os.path.join(ROOT, d))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--col", type=int, default=6)
    ap.add_argument("--rows", type=int, default=300_000)
    ap.add_argument("--row0", type=int, default=4_000_000)
    ap.add_argument("--p-null", type=float, default=0.05)
    ap.add_argument("--seed", type=int, default=0xA11)
    a = ap.parse_args()
    import torch
    assert torch.cuda.is_available()
    import pqgpu
    import pqgtools
    import pyoracle
    pqgpu.LIB_PATH = os.path.join(ROOT, "parquet-rs_amd", "lib_diag", "libpqgpu.so")
    blob, pages, info = pqgtools.alltypes_row_group(a.rows, a.row0, a.p_null, a.seed, threads=8)
    j = a.col
    name, pt = pqgtools.ALLTYPES[j]
    specs = [pyoracle.PageSpec(p.page_type, blob[p.offset:p.offset + p.nbytes].tobytes(), p.num_values,
                               p.encoding, p.def_encoding, p.rep_encoding)
             for p in (pages[i] for i in range(info.chunk_first[j], info.chunk_first[j + 1]))]
    lv, vals, offs = pqgtools.alltypes_truth(a.row0, a.rows, j, a.p_null, a.seed, info.value_bytes[j])
    ctx = pqgpu.Context(0)
    got = pqgpu.decode_column(ctx, pt, specs, max_def=1)
    print(name, "status", got["status"], got["message"], "num_values", got["num_values"], "truth", info.num_values[j])
    if len(got["def"]):
        d = got["def"] != lv
        print("def mismatches", int(d.sum()), "first", int(np.argmax(d)) if d.any() else -1)
    got2 = pqgpu.decode_column(ctx, pt, specs, max_def=1, want_def=False)
    print("without def levels: status", got2["status"], got2["message"], "num_values", got2["num_values"])
    if got2["status"] == 0 and pt != 6:
        g = got2["values"].view(np.uint8)
        diff = np.nonzero(g != vals[:len(g)])[0]
        print("value byte mismatches", len(diff), "first", diff[:5])
    ctx.close()


if __name__ == "__main__":
    main()
