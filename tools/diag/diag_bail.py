"""Diagnostics: which pages of an alltypes row group the level path hands back to the general
decoder, and where (PQG_DIAG build, PQG_DEBUG=512; sites in pqg_levels.hip LV_BAIL).

    make -C parquet-rs_amd DIAG=1 && PQG_DEBUG=512 python tools/diag/diag_bail.py [--rows 8388608]
"""
import argparse
import collections
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for d in ("parquet-rs_amd", os.path.join("tools", "gen"), "oracle"):
    sys.path.insert(0, os.path.join(ROOT, d))

SITES = {1: "segment scan", 2: "stitch", 3: "emit: entry chain missed the reference", 4: "emit: chain/run check",
         5: "emit: bitmap run check", 6: "walked emit (a)", 7: "walked emit (b)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 23)
    ap.add_argument("--row0", type=int, default=0)
    ap.add_argument("--p-null", type=float, default=0.05)
    ap.add_argument("--seed", type=int, default=0xA11)
    a = ap.parse_args()
    import torch
    assert torch.cuda.is_available()
    import pqgpu
    import pqgtools
    import pyoracle
    pqgpu.LIB_PATH = os.path.join(ROOT, "parquet-rs_amd", "lib_diag", "libpqgpu.so")
    L = pqgpu.lib()
    L.pqg_debug_read.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    blob, pages, info = pqgtools.alltypes_row_group(a.rows, a.row0, a.p_null, a.seed, threads=8)
    ctx = pqgpu.Context(0)
    for j, (name, pt) in enumerate(pqgtools.ALLTYPES):
        idx = list(range(info.chunk_first[j], info.chunk_first[j + 1]))
        specs = [pyoracle.PageSpec(p.page_type, blob[p.offset:p.offset + p.nbytes].tobytes(), p.num_values,
                                   p.encoding, p.def_encoding, p.rep_encoding) for p in (pages[i] for i in idx)]
        got = pqgpu.decode_column(ctx, pt, specs, max_def=1)
        np_ = len(specs)
        buf = np.zeros((np_ * 20 + 7) // 8, np.uint64)
        assert L.pqg_debug_read(ctx.h, buf.ctypes.data, buf.size) == 0
        u = buf.view(np.uint32)
        site = u[:np_]
        win = u[np_:np_ + 4 * np_].reshape(np_, 4)
        c = collections.Counter(int(x) for x in site if x)
        desc = ", ".join(f"{SITES.get(k, k)}: {v}" for k, v in sorted(c.items())) or "none"
        sizes = [s.num_values for s in specs]
        print(f"{name:16s} status {got['status']} pages {len(specs)} (levels {min(sizes)}..{max(sizes)}) "
              f"handed back: {desc}")
        bad = [i for i, x in enumerate(site) if x]
        if bad:
            print("   first:", [(i, int(site[i]), specs[i].num_values, len(specs[i].buf)) for i in bad[:6]])
            for i in bad[:3]:
                k, wx, wy = int(win[i, 0]), int(win[i, 1]), int(win[i, 2])
                if not k:
                    continue
                k -= 1
                sp = specs[i]
                import struct
                ln = struct.unpack_from("<i", sp.buf, 0)[0]
                stream = sp.buf[4:4 + ln]
                w0 = k * 1024
                print(f"   page {i}: window {k} of {(ln + 1023) // 1024}, stream {ln} bytes, entry {wx & 0xFFFF}, "
                      f"meeting {wx >> 16}, first output {wy}")
                np.save(os.path.join(ROOT, "gpurun_out", f"bail_{name}_p{i}_w{k}.npy"),
                        np.frombuffer(stream[max(0, w0 - 2048):w0 + 3072], np.uint8))
    ctx.close()


if __name__ == "__main__":
    main()
