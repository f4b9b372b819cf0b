#!/usr/bin/env python3
"""Device-resident Parquet page-decode benchmark (BASELINE.json metric) on MI355X.

  python bench.py [--gpus N --steps K --warmup W] [--config all|levels|dict|delta|alltypes] [...]

A step is one decode of the whole synthetic workload through the C ABI with the page bytes
already resident in HBM:
  configs[1] (headline, `levels`): 1e9 one-bit def levels + 1e9 PLAIN INT32 values (p_null 0,
      the literal config), 954 pages of 2^20 levels; p_null 0.5 / 0.1 variants alongside;
  configs[2] (`dict`): RLE_DICTIONARY INT64, 65 536-entry dictionary, 1e9 indices;
  configs[3] (`delta`): DELTA_BINARY_PACKED INT64, 1e9 values, 128-value mini-blocks;
  configs[4] (`alltypes`): this GPU's share of the alltypes_plain-schema file (88 row groups of
      2^23 rows, ~64 GiB decoded): row groups partitioned over the ranks.
The default (`all`) times every config in one run; the JSON line's top level is configs[1], the
others are under "configs". With --gpus N > 1 and no WORLD_SIZE in the environment, this process
starts N ranks through torch.distributed.run (before touching the GPU) and exits with their
status; every rank decodes its own partition: weak scaling, no collective on the data path (gloo
carries the barrier and the max-over-ranks step time). Rank 0 prints one JSON line.

ms_per_step is timed on the production kernel sequence with stage timing off; a second, shorter
pass with HIP events on the decode stream (pqg_ctx_set_timing) gives the dominant kernel's time
for the roofline. The CPU baseline is the C restatement of parquet-rs's decode loop (oracle/,
kind "port") on a bounded sample, one decoder per thread, at 1 thread and at the host threads
this process may use, batch sizes 32/64/128/1024 (benches/decoding.rs:103-123,
record/reader.rs:33).
"""
import argparse
import ctypes as C
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "parquet-rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools", "gen"))

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
HBM_ACHIEVABLE_GBS = 6290.0  # MI355X_MICROARCH.md: float4 copy, measured
METRIC = "decoded values/s + GB/s, device-resident page decode, 1/2/4/8 MI355X"
FILE_ROW_GROUPS = 8          # config 5's file = FILE_ROW_GROUPS x --rowgroups row groups


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="all", choices=["all", "levels", "dict", "delta", "alltypes"])
    ap.add_argument("--n", type=float, default=1e9, help="levels/values per GPU")
    ap.add_argument("--p-null", type=float, default=0.0, help="configs[1]: null fraction of the def levels")
    ap.add_argument("--page-values", type=int, default=1 << 20)
    ap.add_argument("--dict-size", type=int, default=65536)
    ap.add_argument("--delta-bits", type=int, default=16)
    ap.add_argument("--block-size", type=int, default=512)
    ap.add_argument("--mini-blocks", type=int, default=4)
    ap.add_argument("--variants", type=int, default=1,
                    help="also time the p_null 0.5 / 0.1 variants (config 2) and the writer-default DELTA "
                         "block shape, 128 values in 4 mini-blocks of 32 (config 4, encoding.rs:508-509)")
    ap.add_argument("--split", default="auto", choices=["auto", "weak", "strong"],
                    help="configs 2-4 over N ranks: weak = every rank decodes its own 1e9-value stream; "
                         "strong = the ranks split one 1e9-value stream into contiguous page ranges "
                         "(SURVEY 8(e)); auto = weak, plus a strong-scaling line per config when N > 1")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--pcie", type=int, default=1, help="also time the host-to-host (PCIe) rate")
    ap.add_argument("--cpu-seconds", type=float, default=16.0, help="CPU baseline budget of the headline")
    ap.add_argument("--threads", type=int, default=16, help="host threads at most (box CPU share: 16)")
    ap.add_argument("--seed", type=int, default=0x5EED0000)
    ap.add_argument("--rowgroups", type=int, default=11,
                    help="alltypes: row groups per GPU (11 x 2^23 rows ~ 8 GiB decoded: 1/8 of config 5)")
    ap.add_argument("--rg-rows", type=int, default=1 << 23, help="alltypes: rows per row group")
    ap.add_argument("--at-p-null", type=float, default=0.05, help="alltypes: null fraction per column")
    ap.add_argument("--streams", type=int, default=1,
                    help="alltypes: pqg_rg_ctx_create's reserved nstreams (1..16, ignored by the library)")
    ap.add_argument("--at-batch", default="step", choices=["step", "rg"],
                    help="alltypes: one pqg_decode_chunks over every chunk of the step (step) or one "
                         "pqg_rg_decode per row group on two alternating streams (rg)")
    ap.add_argument("--overlap", type=int, default=0,
                    help="speculative PLAIN copy beside the level decode (pqg_ctx_set_overlap)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / partition / reduction plumbing only (gloo, no GPU, no value)")
    return ap.parse_args(argv)


from sharding import max_over_ranks, pages_for_rank, row_groups_for_rank, shard_seed  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n, argv):
    """One process per GPU through torch.distributed.run, started before this process touches
    the GPU; returns their exit status (rank 0 prints the JSON line)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def host_threads(cap):
    """Threads the CPU legs use: at most `cap` (the box's CPU share) and at most the CPUs this
    process may run on; with the affinity and cgroup quota that bound them, for the record."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    n = max(1, min(cap, aff, int(quota) if quota else aff))
    return n, {"affinity_cpus": aff, "cgroup_cpu_quota": quota, "nproc": os.cpu_count(), "cap": cap}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


class Workload:
    """Synthetic pages generated on the host by the reference-identical writers of
    libpqgtools.so (tools/gen) and uploaded once to HBM."""

    def __init__(self, pqgpu, args, rank, kind, p_null=None, block=None, world=1, strong=False):
        import torch
        import pqgtools
        L = pqgtools.lib()
        info = pqgtools.WorkloadInfo()
        n = int(args.n)
        self.n = n
        self.kind = kind
        self.p_null = p_null
        self.page_values = args.page_values
        self.dict_size, self.delta_bits = args.dict_size, args.delta_bits
        self.block = block or (args.block_size, args.mini_blocks)
        th = host_threads(args.threads)[0]
        # weak: this rank's own stream (seeded per rank), every page of it; strong: pages
        # [first, first + count) of the one stream every rank shares (rank 0's seed)
        srank = 0 if strong else rank
        npages_all = (n + args.page_values - 1) // args.page_values
        self.first, cnt = pages_for_rank(npages_all, world, rank) if strong else (0, npages_all)
        self.strong = strong
        first = self.first
        if kind == "levels":
            self.seed = shard_seed(args.seed + 2, srank)
            gen = lambda blob, cap, pages, pcap: L.pqg_gen_levels_plain_pages(
                n, p_null, args.page_values, self.seed, first, cnt, th, blob, cap, pages, pcap, C.byref(info))
            self.col = pqgpu.Column(pqgpu.INT32, -1, 1, 0)
            self.es = 4
        elif kind == "dict":
            self.seed = shard_seed(args.seed + 3, srank)
            gen = lambda blob, cap, pages, pcap: L.pqg_gen_dict_int64_pages(
                n, args.dict_size, args.page_values, self.seed, first, cnt, th, blob, cap, pages, pcap,
                C.byref(info))
            self.col = pqgpu.Column(pqgpu.INT64, -1, 0, 0)
            self.es = 8
        else:
            self.seed = shard_seed(args.seed + 4, srank)
            gen = lambda blob, cap, pages, pcap: L.pqg_gen_delta_int64_pages(
                n, args.delta_bits, args.page_values, self.block[0], self.block[1], self.seed, first, cnt,
                th, blob, cap, pages, pcap, C.byref(info))
            self.col = pqgpu.Column(pqgpu.INT64, -1, 0, 0)
            self.es = 8
        st = gen(None, 0, None, 0)
        assert st == 0, st
        cap, npg = info.blob_len, info.npages
        self.host = np.zeros(cap + 64, dtype=np.uint8)
        self.pages = (pqgpu.Page * npg)()
        t0 = time.time()
        st = gen(self.host.ctypes.data_as(C.c_void_p), cap, self.pages, npg)
        assert st == 0, f"generator failed: {st}"
        self.gen_s = time.time() - t0
        self.npages = npg
        self.levels = info.total_levels
        self.values = info.total_values
        self.in_bytes = sum(self.pages[i].nbytes for i in range(npg))
        dev = torch.device("cuda", torch.cuda.current_device())
        self.d_blob = torch.from_numpy(self.host).to(dev)
        self.blob_len = cap
        nlev = self.levels
        self.d_def = torch.empty(nlev + 64, dtype=torch.int16, device=dev) if self.col.max_def > 0 else None
        self.d_val = torch.empty(self.values * self.es + 64, dtype=torch.uint8, device=dev)
        self.out = pqgpu.Output(self.d_def.data_ptr() if self.d_def is not None else None, None,
                                self.d_val.data_ptr(), self.values * self.es, None, 0, 0, 0, 0)
        # algorithmic bytes per step: encoded page bytes in, decoded bytes out
        self.level_bytes_in = 0
        if kind == "levels":
            for i in range(npg):
                self.level_bytes_in += int.from_bytes(self.host[self.pages[i].offset:self.pages[i].offset + 4].tobytes(), "little") + 4
        self.out_bytes = (2 * nlev if self.col.max_def > 0 else 0) + self.values * self.es

    def page_specs(self, count, first=0):
        """Pages [first, first + count) as oracle page specs (CPU baseline leg only)."""
        import pyoracle
        specs = []
        for i in range(first, first + count):
            p = self.pages[i]
            buf = self.host[p.offset:p.offset + p.nbytes].tobytes()
            specs.append(pyoracle.PageSpec(p.page_type, buf, p.num_values, p.encoding, p.def_encoding,
                                           p.rep_encoding, p.def_len, p.rep_len))
        return specs


def decode_once(ctx, w, stream):
    ctx.decode_async(w.col, w.d_blob.data_ptr(), w.blob_len, w.pages, w.out, stream, npages=w.npages)


def check_values(ctx, w, stream):
    """Decode once and compare sampled pages (first, middle, last) with the generator's own
    content (pqg_truth_*: the levels and values the pages were written from), plus the status
    and the value count. Parity itself is established by tests/ against the oracle."""
    import pqgtools
    L = pqgtools.lib()
    decode_once(ctx, w, stream)
    st, bad = ctx.sync()
    assert st == 0, (st, bad, ctx.error_message())
    assert w.out.num_values == w.values, (w.out.num_values, w.values)
    first = 1 if w.kind == "dict" else 0
    ndata = w.npages - first
    checked = 0
    for k in sorted({0, ndata // 2, ndata - 1}):
        cnt = w.pages[first + k].num_values
        lo = k * w.page_values  # every page but the last holds page_values levels/values
        gk = w.first + k        # the page's index in the stream (strong scaling: this rank's range)
        if w.kind == "levels":
            lv = np.zeros(cnt, np.int16)
            vals = np.zeros(cnt, np.int32)
            nn = L.pqg_truth_levels_plain(w.n, w.p_null, w.page_values, w.seed, gk, lv.ctypes.data, vals.ctypes.data)
            got_lv = w.d_def[lo:lo + cnt].cpu().numpy()
            assert np.array_equal(got_lv, lv), f"def levels of page {k} differ from the generator"
            voff = int((w.d_def[:lo] == 1).sum().item())
            got_v = w.d_val[4 * voff:4 * (voff + nn)].cpu().numpy().view(np.int32)
            assert np.array_equal(got_v, vals[:nn]), f"values of page {k} differ from the generator"
        else:
            vals = np.zeros(cnt, np.int64)
            if w.kind == "dict":
                L.pqg_truth_dict_int64(w.n, w.dict_size, w.page_values, w.seed, gk, vals.ctypes.data)
            else:
                L.pqg_truth_delta_int64(w.n, w.delta_bits, w.page_values, w.seed, gk, vals.ctypes.data)
            got_v = w.d_val[8 * lo:8 * (lo + cnt)].cpu().numpy().view(np.int64)
            assert np.array_equal(got_v, vals), f"values of page {k} differ from the generator"
        checked += 1
    if w.d_def is not None:
        nn = int((w.d_def[: w.levels] == 1).sum().item())
        assert nn == w.values, (nn, w.values)
    return {"pages_checked": checked, "status": st, "values": int(w.out.num_values)}


def time_steps(ctx, w, stream, steps, warmup, dist=None):
    """Seconds per step over `steps` decodes, production path (no stage events)."""
    import torch
    for _ in range(warmup):
        decode_once(ctx, w, stream)
    ctx.sync()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        decode_once(ctx, w, stream)
    st, bad = ctx.sync()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist is not None:
        dist.barrier()
    assert st == 0, (st, bad, ctx.error_message())
    return (t1 - t0) / steps


def time_stages(pqgpu, ctx, w, stream, n, overlap):
    """Average stage / dominant-kernel device times over n decodes with HIP events on the decode
    stream. The stages are timed one after the other (pqg_ctx_set_overlap 0: the PLAIN copy after
    the level path, not beside it on the side stream), so that each kernel's time and roofline are
    its own; the step time (`value`) is the production path with the overlap."""
    ctx.set_timing(True)
    ctx.set_overlap(False)
    pqgpu.lib().pqg_reset_timings(ctx.h)
    for _ in range(n):
        decode_once(ctx, w, stream)
    st, bad = ctx.sync()
    assert st == 0, (st, bad, ctx.error_message())
    tm = ctx.timings()
    ctx.set_timing(False)
    ctx.set_overlap(overlap)
    return tm


def cpu_baseline(w, seconds, threads, thr_info):
    """parquet-rs's decode loop restated in C (oracle, kind "port"): ColumnReaderImpl::
    read_batch(batch) per reader, one reader per thread over disjoint pages (the reference's Rc
    types are !Send, so one reader per row group / thread is its only parallelism). Timed at 1
    thread and at `threads` threads, batch sizes 32/64/128/1024, on a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from concurrent.futures import ThreadPoolExecutor
    first = 1 if w.kind == "dict" else 0
    dict_spec = w.page_specs(1)[0] if w.kind == "dict" else None
    batches = (32, 64, 128, 1024)
    legs = [(1, b) for b in batches] + [(threads, b) for b in batches]
    budget = seconds / len(legs)

    def run(g, b):
        pages = ([dict_spec] if dict_spec else []) + g
        rr = pyoracle.read_column(w.col.physical_type, pages, max_def=w.col.max_def, batch_size=b)
        assert rr["status"] == 0, rr["message"]
        return sum(p.num_values for p in g)

    one = {}
    for b in batches:  # time one page per batch size to size the samples
        sp = w.page_specs(1, first)
        t0 = time.perf_counter()
        run(sp, b)
        one[b] = time.perf_counter() - t0
    res = {}
    for th, b in legs:
        npg = max(th, min(w.npages - first, int(budget * th / max(one[b], 1e-6))))
        npg = min(npg, w.npages - first)
        specs = w.page_specs(npg, first)
        groups = [specs[i::th] for i in range(th)]
        t0 = time.perf_counter()
        with ThreadPoolExecutor(th) as ex:
            n = sum(ex.map(lambda g: run(g, b), groups))
        dt = time.perf_counter() - t0
        res[(th, b)] = (n / dt, npg, n, dt)
    head = res[(threads, 1024)]
    return {"value": head[0], "unit": "values/s" if w.kind != "levels" else "levels/s",
            "cores": threads, "kind": "port", "cpu_model": cpu_model(), "host_cpus": thr_info,
            "sample": f"{head[1]} of {w.npages} pages ({head[2]} levels/values), read_batch(1024), "
                      f"one reader per thread, {head[3]:.1f}s wall",
            "by_threads_batch": {f"{th}t_b{b}": round(v[0], 1) for (th, b), v in res.items()}}


def pcie_inclusive(ctx, w, stream, iters=3):
    """Host-to-host rate of the same decode (north_star): pinned page bytes -> HBM, decode,
    decoded levels/values -> pinned host memory, all on the decode stream."""
    import torch
    h_blob = torch.from_numpy(w.host).pin_memory()
    h_def = torch.empty(w.levels, dtype=torch.int16).pin_memory() if w.d_def is not None else None
    h_val = torch.empty(w.values * w.es, dtype=torch.uint8).pin_memory()
    s = torch.cuda.ExternalStream(stream)
    best = None
    for _ in range(iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            w.d_blob.copy_(h_blob, non_blocking=True)
            decode_once(ctx, w, stream)
            if h_def is not None:
                h_def.copy_(w.d_def[: w.levels], non_blocking=True)
            h_val.copy_(w.d_val[: w.values * w.es], non_blocking=True)
        st, bad = ctx.sync()
        s.synchronize()
        dt = time.perf_counter() - t0
        assert st == 0, (st, bad)
        best = dt if best is None else min(best, dt)
    units = w.levels if w.kind == "levels" else w.values
    moved = w.blob_len + (2 * w.levels if h_def is not None else 0) + w.values * w.es
    return {"values_per_s": units / best, "ms": best * 1e3, "pcie_bytes": moved,
            "note": "pinned H2D of page bytes + decode + D2H of decoded levels/values, best of %d" % iters}


LEVEL_PATH = ("k_lv_", "k_d1_", "k_run_index", "k_tile_desc", "k_texpand_levels", "k_page_counts")
DELTA_STAGE = ("k_delta_",)  # k_delta_page, the tiled path's kernels
# the dictionary values: tile descriptors, the tile expand (16-bit indices kept, or gathered from
# L2) and the windowed gather (k_dict_win)
DICT_STAGE = ("k_tile_desc", "k_texpand_d", "k_dict_win")


def pmc_traffic(kind, kernel, variant=None):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes of this config
    (profiles/<round>/<config>[_<variant>]/kernels.json, written by tools/pmc_traffic.py:
    FETCH_SIZE x2 + WRITE_SIZE, the MI355X_MICROARCH.md gfx950 corrections). The def-level path
    is a chain of kernels timed as one (HIP events around pqg_launch_levels): its traffic is their
    sum per step (each kernel's per-launch bytes x its launches per step). None when not profiled."""
    base = kernel.split("<")[0]
    sub = kind if variant is None else f"{kind}_{variant}"
    for rnd in sorted(os.listdir(os.path.join(ROOT, "profiles")), reverse=True):
        path = os.path.join(ROOT, "profiles", rnd, sub, "kernels.json")
        if not os.path.exists(path):
            continue
        try:
            ks = json.load(open(path))["kernels"]
        except (OSError, ValueError, KeyError):
            continue
        names = {k.replace("pqg::", ""): e for k, e in ks.items() if "traffic_bytes" in e}
        # per step: a kernel launched more than once per step (config 5 runs the level-path chain
        # for its def streams twice) weighs calls / steps, steps = the fewest calls of a decode kernel
        steps = min([e.get("calls", 1) for k, e in ks.items() if k.startswith("pqg::")] or [1])

        def per_step(e):
            return e["traffic_bytes"] * max(e.get("calls", steps), 1) / max(steps, 1)

        if kernel == "whole step":  # config 5: every decode kernel of the step
            tot = [per_step(e) for k, e in ks.items() if k.startswith("pqg::") and "traffic_bytes" in e]
            if tot:
                return sum(tot), os.path.relpath(path, ROOT)
            continue
        if kernel in ("level path", "DELTA stage", "dictionary stage"):  # kernels timed as one: their sum
            pre = {"level path": LEVEL_PATH, "DELTA stage": DELTA_STAGE, "dictionary stage": DICT_STAGE}[kernel]
            tot = [per_step(e) for k, e in names.items() if k.startswith(pre)]
            if tot:
                return sum(tot), os.path.relpath(path, ROOT)
            continue
        for k, e in names.items():
            if k.split("<")[0] == base:
                return e["traffic_bytes"], os.path.relpath(path, ROOT)
    return None, None


def copy_ceiling_gbs(nbytes=4 << 30):
    """Achievable HBM rate on this device: a 16-byte-per-lane copy kernel
    (tools/ubench/copy_ceiling.hip), best of plain and non-temporal."""
    L = C.CDLL(os.path.join(ROOT, "tools", "ubench", "libpqgcopy.so"))
    L.pqg_copy_ceiling_gbs.restype = C.c_double
    L.pqg_copy_ceiling_gbs.argtypes = [C.c_uint64, C.c_int]
    return L.pqg_copy_ceiling_gbs(nbytes, 10)


def roofline(name, ms, nbytes, traffic, traffic_src, note=None):
    achieved = nbytes / (ms * 1e-3) / 1e9 if ms else None
    return {"bound": "hbm", "kernel": name, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS if achieved else None, "traffic": traffic,
            "traffic_source": traffic_src, "bytes_per_launch": nbytes, "avg_ms": ms,
            "frac_of_achievable": achieved / HBM_ACHIEVABLE_GBS if achieved else None, "note": note}


LEVEL_NOTE = ("HIP events around pqg_launch_levels: the def-level kernel chain (k_lv_plan, k_lv_bound, "
              "k_lv_segwalk, k_lv_segscan, k_lv_compact, the dense one-bit pages' k_d1_tab, k_d1_stitch, k_d1_emit, "
              "the window path's k_lv_win, k_lv_stitch, k_lv_emit, k_lv_emit_walk, k_lv_fallback + the fused "
              "value-offset scan), one launch each per step; traffic = their PMC sum")


def run_fixed(pqgpu, ctx, args, world, rank, dist, stream, kind, p_null=None, steps=None, warmup=None,
              cpu_seconds=None, extras=True, block=None, variant=None, strong=False):
    """One of configs[1..3]: generate, check, time (production path), stage times, roofline, and
    on rank 0 of a 1-GPU run the PCIe-inclusive rate and the CPU baseline. strong: the ranks split
    one stream into contiguous page ranges (value = the stream's units / the slowest rank's time)."""
    import torch
    steps = args.steps if steps is None else steps
    warmup = args.warmup if warmup is None else warmup
    w = Workload(pqgpu, args, rank, kind, p_null=p_null, block=block, world=world, strong=strong)
    checked = check_values(ctx, w, stream)
    per_step = max_over_ranks(time_steps(ctx, w, stream, steps, warmup, dist), dist)
    tm = time_stages(pqgpu, ctx, w, stream, max(3, steps // 4), args.overlap)
    units = w.levels if kind == "levels" else w.values
    step_bytes = w.in_bytes + w.out_bytes
    if kind == "levels":
        lev_b = w.level_bytes_in + 2 * w.levels   # level stream in + int16 levels out
        val_b = 2 * w.values * w.es               # PLAIN values in + out
        variant = f"p{int(round(p_null * 100)):02d}"
        stages = [("level path", tm.levels_kernel_ms, lev_b, w.level_bytes_in),
                  ("k_plain_copy", tm.values_kernel_ms, val_b, w.values * w.es)]
    elif kind == "dict":   # indices in + values out (HIP events around the dictionary kernels: the
        # tile expand keeping 16-bit indices and the windowed gather; their index round trip and
        # the dictionary windows are traffic above these algorithmic bytes)
        stages = [("dictionary stage", tm.values_kernel_ms, w.in_bytes + w.out_bytes, w.in_bytes)]
    else:                  # deltas in + values out (HIP events around the DELTA kernels: the page
        # pass, and the tiled path for pages it leaves)
        stages = [("DELTA stage", tm.values_kernel_ms, w.in_bytes + w.out_bytes, w.in_bytes)]
        if tuple(w.block) != (512, 4):
            variant = f"b{w.block[0]}x{w.block[1]}"
    rl = []
    for name, ms, nb, nin in stages:
        tr, src = pmc_traffic(kind, name, variant)
        r = roofline(name, ms, nb, tr, src, LEVEL_NOTE if name == "level path" else None)
        r["read_bytes_per_launch"] = nin
        r["read_gbs"] = nin / (ms * 1e-3) / 1e9 if ms else None  # In / time
        rl.append(r)
    # the dominant kernel by time; for the nullable level variants (p_null > 0) the level path, the
    # decode those variants exist to measure (the PLAIN copy beside it is the same memcpy at every p_null)
    dom = max(rl, key=lambda r: r["avg_ms"] or 0)
    if kind == "levels" and p_null:
        dom = rl[0]
    # the stream each rank decodes: its own (weak) or its page range of the shared one (strong)
    job_units = (w.n if strong else units * world)
    res = {
        "value": job_units / per_step,
        "unit": "levels/s" if kind == "levels" else "values/s",
        "ms_per_step": per_step * 1e3,
        "gbps": step_bytes / per_step / 1e9 * world,
        # read-only rate (encoded page bytes / step time) and the reference bench's
        # unit, encoded MB/s (benches/decoding.rs:111 sets Throughput::Bytes of the encoded buffer)
        "read_gbps": w.in_bytes / per_step / 1e9 * world,
        "encoded_mb_per_s": w.in_bytes / per_step / 1e6 * world,
        "config": {"workload": {"levels": "configs[1]: RLE/bit-packed def levels (max_def 1) + PLAIN INT32",
                                "dict": "configs[2]: RLE_DICTIONARY INT64, 64K dictionary",
                                "delta": "configs[3]: DELTA_BINARY_PACKED INT64"}[kind],
                   "levels_per_gpu": w.levels, "values_per_gpu": w.values,
                   "pages_per_gpu": w.npages, "page_values": args.page_values,
                   "p_null": w.p_null, "in_bytes_per_gpu": w.in_bytes, "out_bytes_per_gpu": w.out_bytes,
                   "block_size": w.block[0] if kind == "delta" else None,
                   "mini_blocks": w.block[1] if kind == "delta" else None,
                   "values_per_mini_block": w.block[0] // w.block[1] if kind == "delta" else None,
                   "gen_seconds": round(w.gen_s, 1),
                   "parallelism": (f"one stream split into contiguous page ranges x{world}, no collective"
                                   if strong else f"row-group partitions x{world}, no collective")},
        "roofline": dom,
        "roofline_stages": rl if len(rl) > 1 else None,
        # the whole step beside the dominant kernel: every algorithmic byte of the step / ms_per_step
        "roofline_whole_step": {"bound": "hbm", "achieved": step_bytes / per_step / 1e9, "peak": HBM_PEAK_GBS,
                                "unit": "GB/s", "frac": step_bytes / per_step / 1e9 / HBM_PEAK_GBS,
                                "bytes_per_step": step_bytes},
        "stages_note": ("stage and kernel times from HIP events with the stages one after the other "
                        "(pqg_ctx_set_overlap 0); ms_per_step is the production path, PLAIN copy beside "
                        "the level decode" if kind == "levels" and args.overlap else None),
        "stages_ms": {"prepare": tm.prepare_ms, "levels": tm.levels_ms, "scan": tm.scan_ms,
                      "values": tm.values_ms, "total": tm.total_ms,
                      "levels_kernel": tm.levels_kernel_ms, "values_kernel": tm.values_kernel_ms},
        "value_check": checked,
    }
    if strong:  # the job's bytes (sum of the ranks' shares) over the slowest rank's time
        tot = [float(w.in_bytes), float(w.out_bytes)]
        if dist is not None:
            t = torch.tensor(tot, dtype=torch.float64)
            dist.all_reduce(t)
            tot = [float(x) for x in t]
        res["gbps"] = (tot[0] + tot[1]) / per_step / 1e9
        res["read_gbps"] = tot[0] / per_step / 1e9
        res["encoded_mb_per_s"] = tot[0] / per_step / 1e6
        res["config"]["first_page"] = w.first
    if extras and rank == 0 and world == 1:
        if args.pcie:
            res["pcie_inclusive"] = pcie_inclusive(ctx, w, stream)
        if args.cpu_baseline:
            th, info = host_threads(args.threads)
            res["cpu_baseline"] = cpu_baseline(w, args.cpu_seconds if cpu_seconds is None else cpu_seconds, th, info)
    del w
    torch.cuda.empty_cache()
    return res


def run_bytes_page(pqgpu, ctx, stream, enc, steps, warmup):
    """One REQUIRED BYTE_ARRAY page of 2^20 values, DELTA_BYTE_ARRAY (sorted URL-like strings:
    prefix lengths, suffix lengths, suffixes; decoding.rs:768-835) or DELTA_LENGTH_BYTE_ARRAY
    (random lengths 0..48; decoding.rs:682-712), written by tools/gen's restated encoders, decoded
    whole by the production path (k_ba_index's length streams, the value-offset scan, the slice
    copy / prefix rebuild) and checked byte for byte against the values written. Roofline: the
    page's bytes in + the values' bytes and int64 offsets out, over the decode time."""
    import torch
    import pqgtools
    n = 1 << 20
    if enc == "dba":
        vals = pqgtools.url_values(n, 0x5EED0006)
        body, code = pqgtools.delta_byte_array_body(vals), pqgpu.DELTA_BYTE_ARRAY
    else:
        rng = np.random.default_rng(0x5EED0007)
        lens = rng.integers(0, 49, n)
        raw = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8).tobytes()
        offs0 = np.concatenate([[0], np.cumsum(lens)])
        vals = [raw[offs0[i]:offs0[i + 1]] for i in range(n)]
        body, code = pqgtools.delta_length_body(vals), pqgpu.DELTA_LENGTH_BYTE_ARRAY
    flat = b"".join(vals)
    pages = (pqgpu.Page * 1)()
    pages[0] = pqgpu.Page(0, len(body), n, pqgpu.PAGE_DATA, code, pqgpu.RLE, pqgpu.RLE, 0, 0)
    d_blob = torch.frombuffer(bytearray(body + b"\0" * 64), dtype=torch.uint8).cuda()
    d_val = torch.empty(len(flat) + 64, dtype=torch.uint8, device="cuda")
    d_off = torch.empty(n + 2, dtype=torch.int64, device="cuda")
    col = pqgpu.Column(pqgpu.BYTE_ARRAY, -1, 0, 0)
    out = pqgpu.Output(None, None, d_val.data_ptr(), len(flat), d_off.data_ptr(), n + 1, 0, 0, 0)

    def once():
        ctx.decode_async(col, d_blob.data_ptr(), len(body) + 64, pages, out, stream, npages=1)

    once()
    st, bad = ctx.sync()
    assert st == 0, (st, bad, ctx.error_message())
    offs = d_off[:n + 1].cpu().numpy()
    ok = (out.num_values == n and offs[-1] == len(flat) and
          np.array_equal(offs, np.concatenate([[0], np.cumsum([len(v) for v in vals])])) and
          d_val[:len(flat)].cpu().numpy().tobytes() == flat)
    assert ok, "byte-array page decode differs from the values written"
    for _ in range(warmup):
        once()
    ctx.sync()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        once()
    st, bad = ctx.sync()
    e1.record()
    torch.cuda.synchronize()
    assert st == 0, (st, bad)
    ms = e0.elapsed_time(e1) / steps
    nb = len(body) + len(flat) + 8 * (n + 1)
    return {"values_per_s": n / (ms * 1e-3), "ms_per_step": ms, "values_per_gpu": n,
            "page_bytes": len(body), "value_bytes": len(flat), "value_check": "every byte and offset",
            "roofline": roofline("byte-array page decode (whole step)", ms, nb, None, None,
                                 "HIP events on the decode stream around whole decodes (the host "
                                 "enqueue of each decode included); bytes = page in + values and "
                                 "int64 offsets out")}


def dry_run(args, world, rank, dist):
    """Launcher / partition / reduction plumbing without a GPU: every rank derives its own
    partition (seed, config-5 row groups), the max-over-ranks step time is reduced over gloo,
    rank 0 prints a line marked dry_run with no value."""
    seed = shard_seed(args.seed + 2, rank)
    mine = alltypes_partition(args, world, rank)
    t0 = time.perf_counter()
    time.sleep(0.01 * (rank + 1))
    per_step = max_over_ranks(time.perf_counter() - t0, dist)
    seeds, parts = [seed], [mine]
    if dist is not None:
        seeds, parts = [None] * world, [None] * world
        dist.all_gather_object(seeds, seed)
        dist.all_gather_object(parts, mine)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "levels/s", "n_gpus": world,
                          "steps": 0, "warmup": 0, "ms_per_step": per_step * 1e3, "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dry_run": True,
                          "config": {"workload": args.config, "partition_seeds": seeds,
                                     "alltypes_row_groups": parts,
                                     "parallelism": f"row-group partitions x{world}, no collective"}}),
              flush=True)


def alltypes_partition(args, world, rank):
    """Row groups of config 5's file this rank decodes. The file has FILE_ROW_GROUPS x --rowgroups
    row groups of --rg-rows rows (88 x 2^23 rows, ~64 GiB decoded); a run on `world` GPUs decodes
    its first --rowgroups x world (all of it at 8 GPUs: weak scaling), split over the ranks by
    sharding.row_groups_for_rank (contiguous, balanced by bytes; the synthetic row groups have
    equal row counts and the same column mix, so rows stand in for their bytes)."""
    file_rgs = FILE_ROW_GROUPS * args.rowgroups
    job = min(file_rgs, args.rowgroups * world)
    return row_groups_for_rank([args.rg_rows] * job, world, rank)


class AlltypesWorkload:
    """Config 5 (one GPU's share): the row groups alltypes_partition assigns this rank, written by
    the reference writer's defaults (tools/gen pqg_gen_alltypes), pages of all row groups in one
    pinned host buffer and one device buffer; one pqg_rg_decode per row group."""

    def __init__(self, pqgpu, args, rank, world):
        import torch
        import pqgtools
        self.rows, self.p_null = args.rg_rows, args.at_p_null
        self.seed = shard_seed(args.seed + 5, 0)  # one file: every rank generates from the same seed
        self.rg_index = alltypes_partition(args, world, rank)
        self.R = len(self.rg_index)
        self.row0s = [g * self.rows for g in self.rg_index]
        self.job_rgs = min(FILE_ROW_GROUPS * args.rowgroups, args.rowgroups * world)
        self.cols = [pqgpu.Column(pt, -1, 1, 0) for _, pt in pqgtools.ALLTYPES]
        th = host_threads(args.threads)[0]
        t0 = time.time()
        rgs = [pqgtools.alltypes_row_group(self.rows, r0, self.p_null, self.seed, th) for r0 in self.row0s]
        self.gen_s = time.time() - t0
        self.base = []
        off = 0
        for blob, pages, info in rgs:
            self.base.append(off)
            off += (info.blob_len + 255) & ~255
        self.blob_len = off
        self.h_blob = torch.empty(off + 64, dtype=torch.uint8).pin_memory()
        hb = self.h_blob.numpy()
        self.info, self.chunks = [], []
        for g, (blob, pages, info) in enumerate(rgs):
            hb[self.base[g]:self.base[g] + info.blob_len] = blob[:info.blob_len]
            self.info.append(info)
            per = []
            for j in range(len(self.cols)):
                lo, hi = info.chunk_first[j], info.chunk_first[j + 1]
                arr = (pqgpu.Page * (hi - lo))(*[pages[i] for i in range(lo, hi)])
                per.append(arr)
            self.chunks.append(per)
        del rgs
        dev = torch.device("cuda", torch.cuda.current_device())
        self.d_blob = torch.empty(off + 64, dtype=torch.uint8, device=dev)
        self.d_blob.copy_(self.h_blob)
        # pages of every row group with offsets into the one device blob (the batched step)
        self.shifted = []
        for g in range(self.R):
            per = []
            for arr in self.chunks[g]:
                sh = (pqgpu.Page * len(arr))()
                for i in range(len(arr)):
                    sh[i] = arr[i]
                    sh[i].offset = arr[i].offset + self.base[g]
                per.append(sh)
            self.shifted.append(per)
        # outputs: one set per row group for the batched step; the row-group path and the PCIe
        # pipeline use sets 0 and 1 (row group g + 1 decodes while g drains)
        self.vcap = [max(i.value_bytes[j] for i in self.info) + 64 for j in range(len(self.cols))]
        self.ncap = [self.rows + 1] * len(self.cols)  # BYTE_ARRAY offsets: num_levels + 1 (pqgpu.h)
        self.out = []
        for _ in range(max(2, self.R) if args.at_batch == "step" else 2):
            o = []
            for j, (name, pt) in enumerate(pqgtools.ALLTYPES):
                d_def = torch.empty(self.rows + 64, dtype=torch.int16, device=dev)
                d_val = torch.empty(self.vcap[j], dtype=torch.uint8, device=dev)
                d_off = torch.empty(self.ncap[j] + 8, dtype=torch.int64, device=dev) if pt == 6 else None
                st = pqgpu.Output(d_def.data_ptr(), None, d_val.data_ptr(), self.vcap[j],
                                  d_off.data_ptr() if d_off is not None else None,
                                  self.ncap[j] if d_off is not None else 0, 0, 0, 0)
                o.append((d_def, d_val, d_off, st))
            self.out.append(o)
        self.levels = self.R * self.rows * len(self.cols)  # cells: one level per row and column
        self.in_bytes = sum(i.blob_len for i in self.info)
        self.out_bytes = 0
        for i in self.info:
            for j, (_, pt) in enumerate(pqgtools.ALLTYPES):
                self.out_bytes += 2 * self.rows + i.value_bytes[j] + (8 * (i.num_values[j] + 1) if pt == 6 else 0)

    def decode_rg(self, rgd, g, stream, oset=0):
        """pqg_rg_decode of row group g: its 11 column chunks in one batched decode."""
        return rgd.decode_async(self.cols, self.d_blob.data_ptr() + self.base[g], self.info[g].blob_len,
                                self.chunks[g], [o[3] for o in self.out[oset]], stream)

    def decode_step(self, ctx, stream):
        """Every column chunk of every row group of the share in one pqg_decode_chunks (row group
        g into output set g)."""
        cols, arrays, outs = [], [], []
        for g in range(self.R):
            for j, col in enumerate(self.cols):
                cols.append(col)
                arrays.append(self.shifted[g][j])
                outs.append(self.out[g][j][3])
        return ctx.decode_chunks_async(cols, self.d_blob.data_ptr(), self.blob_len, arrays, outs, stream)


def alltypes_check(ctx, w, stream, batch_ctx=None):
    """Decode this rank's row groups and compare every column (levels, values, BYTE_ARRAY
    offsets) of the first and the last with the generator's own cells (pqg_truth_alltypes):
    through the batched step when batch_ctx is given, else row group 0 through pqg_rg_decode."""
    import pqgtools
    if batch_ctx is not None:
        oa_all = w.decode_step(batch_ctx, stream)
        st, call, chunk, bad = batch_ctx.sync_detail()
        assert st == 0, (st, call, chunk, bad, batch_ctx.error_message())
        groups = sorted({0, w.R - 1})
    else:
        oa_all = w.decode_rg(ctx, 0, stream)
        st, bcol, bad = ctx.sync()
        assert st == 0, (st, bcol, bad, ctx.error_message())
        groups = [0]
    nc = len(pqgtools.ALLTYPES)
    for g in groups:
        for j, (name, pt) in enumerate(pqgtools.ALLTYPES):
            o = oa_all[g * nc + j] if batch_ctx is not None else oa_all[j]
            nv, nb = w.info[g].num_values[j], w.info[g].value_bytes[j]
            assert o.num_values == nv and o.num_levels == w.rows, (g, name, o.num_values, nv)
            lv, vals, offs = pqgtools.alltypes_truth(w.row0s[g], w.rows, j, w.p_null, w.seed, nb)
            d_def, d_val, d_off, _ = w.out[g][j]
            assert np.array_equal(d_def[:w.rows].cpu().numpy(), lv), f"{name}: def levels differ"
            assert np.array_equal(d_val[:nb].cpu().numpy(), vals), f"{name}: values differ"
            if offs is not None:
                assert np.array_equal(d_off[:nv + 1].cpu().numpy(), offs), f"{name}: offsets differ"
    return {"row_groups_checked": len(groups), "columns": nc, "status": st,
            "path": "pqg_decode_chunks (whole step)" if batch_ctx is not None else "pqg_rg_decode"}


def alltypes_steps(ctx, w, stream, steps, warmup, dist=None, batch_ctx=None):
    """Every row group of the share per step: one batched decode of all their column chunks
    (batch_ctx), or one row-group decode per row group alternating between two launch streams and
    two output sets, so that row group g + 1's kernels start while g's still run."""
    import torch
    lanes = [stream, torch.cuda.Stream().cuda_stream]

    def one_pass():
        if batch_ctx is not None:
            w.decode_step(batch_ctx, stream)
            return
        for g in range(w.R):
            w.decode_rg(ctx, g, lanes[g % 2], g % 2)

    sync = (lambda: batch_ctx.sync_detail()) if batch_ctx is not None else (lambda: ctx.sync())
    for _ in range(warmup):
        one_pass()
    sync()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        one_pass()
    th = time.perf_counter()
    r = sync()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist is not None:
        dist.barrier()
    assert r[0] == 0, r
    alltypes_steps.host_ms = (th - t0) / steps * 1e3  # enqueue time per step (host side)
    # the enqueue alone: with the GPU idle, no wait for a staging slot is inside it
    enq = []
    for _ in range(3):
        torch.cuda.synchronize()
        te = time.perf_counter()
        one_pass()
        enq.append(time.perf_counter() - te)
        sync()
    alltypes_steps.enqueue_ms = min(enq) * 1e3
    return (t1 - t0) / steps


def alltypes_file_pipeline(pqgpu, w, args, groups=6):
    """PCIe-inclusive rate through the product API (pqg_rgr_*, csrc/host/rg_reader.cpp): `groups`
    row groups of this workload written as an uncompressed parquet file, then read file -> pinned
    staging (host threads) -> H2D -> batched decode -> D2H into pinned host buffers, two row groups
    in flight. The file is in the page cache (just written): the rate excludes disk."""
    import tempfile
    import pqgtools
    th = host_threads(args.threads)[0]
    path = os.path.join(tempfile.gettempdir(), f"pqg_bench_alltypes_{os.getpid()}.parquet")
    groups = min(groups, max(2, w.R))
    t0 = time.perf_counter()
    pqgtools.write_alltypes_file(path, w.rows, groups, row0=w.row0s[0], p_null=w.p_null, seed=w.seed, codec=0,
                                 threads=th)
    write_s = time.perf_counter() - t0
    res = {"row_groups": groups, "rows_per_group": w.rows, "file_bytes": os.path.getsize(path),
           "write_seconds": round(write_s, 1), "host_threads": th}
    try:
        r = pqgpu.FileReader(path)
        for host_output in (True, False):
            rd = pqgpu.RowGroupReader(r, host_threads=th, host_output=host_output)
            rd.submit(0)  # warm: buffers sized, pages faulted in
            assert rd.wait()[0] == 0, rd.error()
            s0 = rd.stats()
            t0 = time.perf_counter()
            nxt = 0
            for _ in range(min(2, groups)):
                rd.submit(nxt)
                nxt += 1
            for g in range(groups):
                st, rg, col, page = rd.wait()
                assert st == 0 and rg == g, (st, rg, col, page, rd.error())
                if nxt < groups:
                    rd.submit(nxt)
                    nxt += 1
            dt = time.perf_counter() - t0
            s1 = rd.stats()
            if host_output:  # the last row group's columns against the generator's cells
                g = groups - 1
                for j, (name, pt) in enumerate(pqgtools.ALLTYPES):
                    out = rd.host_arrays(j, pt)
                    nb = out["num_bytes"] if pt == 6 else out["values"].nbytes
                    lv, vals, offs = pqgtools.alltypes_truth(w.row0s[0] + g * w.rows, w.rows, j, w.p_null, w.seed,
                                                             max(nb, 1))
                    assert np.array_equal(out["def_levels"], lv), name
                    assert out["values"].tobytes() == vals[:nb].tobytes(), name
            key = "to_host" if host_output else "to_device"
            fb = s1["file_bytes"] - s0["file_bytes"]
            ob = s1["output_bytes"] - s0["output_bytes"]
            res[key] = {"values_per_s": groups * w.rows * len(w.cols) / dt, "ms": dt * 1e3,
                        "ms_per_row_group": dt * 1e3 / groups,
                        "file_gbps": fb / dt / 1e9, "output_gbps": ob / dt / 1e9,
                        "host_ms_per_row_group": (s1["host_ms"] - s0["host_ms"]) / groups,
                        "per_row_group_ms": {k: round((s1[k] - s0[k]) / groups, 3)
                                             for k in ("plan_ms", "fill_ms", "enqueue_ms", "sync_ms",
                                                       "d2h_wait_ms")},
                        "checked": host_output}
            rd.close()
        r.close()
    finally:
        os.unlink(path)
    res["note"] = ("pqg_rgr: headers + page fill into pinned staging on host threads, async H2D, one "
                   "pqg_decode_chunks per row group, async D2H (to_host) into pinned buffers; row group "
                   "g+1 staged while g decodes")
    return res


def alltypes_cpu_baseline(w, threads, thr_info):
    """The C restatement of read_batch(1024) (oracle, kind "port") over the first row group's 11
    column chunks: one reader per chunk, at 1 thread and at `threads` threads."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    import pqgtools
    from concurrent.futures import ThreadPoolExecutor
    hb = w.h_blob.numpy()
    specs = []
    for j, (_, pt) in enumerate(pqgtools.ALLTYPES):
        ps = [pyoracle.PageSpec(p.page_type, hb[w.base[0] + p.offset:w.base[0] + p.offset + p.nbytes].tobytes(),
                                p.num_values, p.encoding, p.def_encoding, p.rep_encoding)
              for p in w.chunks[0][j]]
        specs.append((pt, ps))

    def run(t):
        rr = pyoracle.read_column(t[0], t[1], max_def=1, batch_size=1024)
        assert rr["status"] == 0, rr["message"]
        return w.rows

    res = {}
    for th in (1, threads):
        t0 = time.perf_counter()
        with ThreadPoolExecutor(th) as ex:
            n = sum(ex.map(run, specs))
        res[th] = (n / (time.perf_counter() - t0), time.perf_counter() - t0)
    return {"value": res[threads][0], "unit": "values/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus": thr_info,
            "sample": f"row group 0 ({w.rows} rows x 11 columns), read_batch(1024), one reader per column "
                      f"chunk, {res[threads][1]:.1f}s wall",
            "by_threads": {f"{th}t_b1024": round(v[0], 1) for th, v in res.items()}}


def run_alltypes(pqgpu, args, world, rank, dist, stream, extras=True):
    import torch
    w = AlltypesWorkload(pqgpu, args, rank, world)
    ctx = pqgpu.RowGroupDecoder(torch.cuda.current_device(), args.streams)
    bctx = pqgpu.Context(torch.cuda.current_device()) if args.at_batch == "step" else None
    if bctx is not None:
        bctx.set_overlap(args.overlap)
    checked = alltypes_check(ctx, w, stream, bctx)
    if bctx is not None:
        checked["row_group_path"] = alltypes_check(ctx, w, stream)  # the row-group decoder too
    per_step = max_over_ranks(alltypes_steps(ctx, w, stream, args.steps, args.warmup, dist, bctx), dist)
    step_bytes = w.in_bytes + w.out_bytes
    achieved = step_bytes / per_step / 1e9
    # traffic: the PMC bytes of every decode kernel of one step (one pqg_decode_chunks per step)
    at_traffic, at_src = pmc_traffic("alltypes", "whole step") if bctx is not None else (None, None)
    res = {
        "value": w.job_rgs * w.rows * len(w.cols) / per_step, "unit": "values/s (cells: one level + its value)",
        "ms_per_step": per_step * 1e3, "gbps": step_bytes / per_step / 1e9 * world,
        "dtype": "int16 levels + native values (i32/i64/f32/f64/int96/bool bytes/byte arrays)",
        "config": {"workload": "configs[4]: alltypes_plain schema, this GPU's share of an "
                               f"{FILE_ROW_GROUPS * args.rowgroups}-row-group file of {w.rows}-row row groups",
                   "row_groups": w.rg_index, "row_groups_per_gpu": w.R, "job_row_groups": w.job_rgs,
                   "rows_per_gpu": w.R * w.rows, "cells_per_gpu": w.levels, "p_null": w.p_null,
                   "in_bytes_per_gpu": w.in_bytes, "out_bytes_per_gpu": w.out_bytes,
                   "chunk_decodes_per_step": w.R * len(w.cols), "gen_seconds": round(w.gen_s, 1),
                   "decode_calls_per_step": 1 if bctx is not None else w.R,
                   "batch": "pqg_decode_chunks of every chunk of the step" if bctx is not None
                            else "pqg_rg_decode per row group, two streams",
                   "parallelism": f"row-group partitions x{world}, no collective"},
        "roofline": {"bound": "hbm", "kernel": "whole step (every chunk decode)", "achieved": achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": at_traffic, "traffic_source": at_src,
                     "bytes_per_launch": step_bytes, "avg_ms": per_step * 1e3,
                     "frac_of_achievable": achieved / HBM_ACHIEVABLE_GBS},
        "value_check": checked,
        "host_enqueue_ms_per_step": getattr(alltypes_steps, "enqueue_ms", None),
        "host_ms_per_step_in_loop": getattr(alltypes_steps, "host_ms", None),
    }
    if extras and rank == 0 and world == 1:
        if args.pcie:
            res["pcie_inclusive"] = alltypes_file_pipeline(pqgpu, w, args)
        if args.cpu_baseline:
            th, info = host_threads(args.threads)
            res["cpu_baseline"] = alltypes_cpu_baseline(w, th, info)
    ctx.close()
    if bctx is not None:
        bctx.close()
    del w
    torch.cuda.empty_cache()
    return res


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if os.environ.get("PQG_DEBUG"):
        sys.exit("bench.py: PQG_DEBUG is set; diagnostic modes are not a valid measurement")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:  # barrier + max over ranks: two host scalars, gloo (no RCCL on this path)
        import torch.distributed as td
        # (gloo prints its connection report on stdout: kept off it, which carries only the JSON line)
        sys.stdout.flush()
        keep = os.dup(1)
        os.dup2(2, 1)
        try:
            td.init_process_group("gloo")
        finally:
            os.dup2(keep, 1)
            os.close(keep)
        dist = td
    if args.dry_run:
        dry_run(args, world, rank, dist)
        if dist is not None:
            dist.destroy_process_group()
        return
    import torch
    # PQG_BENCH_DEVICE: every rank on one device (rehearsing the multi-rank path on a 1-GPU box)
    torch.cuda.set_device(int(os.environ.get("PQG_BENCH_DEVICE", local if world > 1 else 0)))
    import pqgpu
    stream = torch.cuda.current_stream().cuda_stream
    head = {"metric": METRIC, "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "higher_is_better": True, "scaling": "strong" if args.split == "strong" else "weak", "vs_baseline": None,
            "data": "synthetic pages from reference-identical writers (SplitMix64 seeded)"}
    sub = {}
    kinds = ["levels", "dict", "delta", "alltypes"] if args.config == "all" else [args.config]
    ctx = pqgpu.Context(torch.cuda.current_device())
    ctx.set_overlap(args.overlap)
    short_steps = max(5, args.steps // 2)
    strong = args.split == "strong"

    def brief(r, key):
        return {key: r["value"], "ms_per_step": r["ms_per_step"], "gbps": r["gbps"], "read_gbps": r["read_gbps"],
                "encoded_mb_per_s": r["encoded_mb_per_s"], "values_per_gpu": r["config"]["values_per_gpu"],
                "config": {k: r["config"][k] for k in ("block_size", "mini_blocks", "values_per_mini_block",
                                                       "pages_per_gpu", "parallelism") if k in r["config"]},
                "roofline": r["roofline"], "roofline_stages": r["roofline_stages"],
                "roofline_whole_step": r["roofline_whole_step"], "stages_ms": r["stages_ms"],
                "value_check": r["value_check"]}

    for kind in kinds:
        if kind == "alltypes":
            sub[kind] = run_alltypes(pqgpu, args, world, rank, dist, stream)
            continue
        unit_key = "levels_per_s" if kind == "levels" else "values_per_s"
        if kind == "levels":
            sub[kind] = run_fixed(pqgpu, ctx, args, world, rank, dist, stream, "levels", p_null=args.p_null,
                                  strong=strong)
            if args.variants:
                var = {}
                for p in (0.5, 0.1):
                    r = run_fixed(pqgpu, ctx, args, world, rank, dist, stream, "levels", p_null=p,
                                  steps=short_steps, warmup=2, extras=False, strong=strong)
                    var[f"p_null={p}"] = brief(r, unit_key)
                sub[kind]["variants"] = var
        else:
            sub[kind] = run_fixed(pqgpu, ctx, args, world, rank, dist, stream, kind, cpu_seconds=6.0, strong=strong)
            if kind == "delta" and args.variants:
                # the reference writer's default block (DeltaBitPackEncoder: 128 values, 4 mini-blocks
                # of 32, encoding.rs:508-509): the shape real parquet-rs files carry
                r = run_fixed(pqgpu, ctx, args, world, rank, dist, stream, "delta", steps=short_steps, warmup=2,
                              extras=False, block=(128, 4), strong=strong)
                sub[kind]["variants"] = {"block128_4x32": brief(r, unit_key)}
                # DELTA_BYTE_ARRAY / DELTA_LENGTH_BYTE_ARRAY: one 2^20-value page each
                for enc in ("dba", "dlba"):
                    sub[kind]["variants"][f"{enc}_page_1M"] = run_bytes_page(pqgpu, ctx, stream, enc, short_steps, 2)
        if args.split == "auto" and world > 1:
            # strong scaling alongside: the ranks split one 1e9-value stream into page ranges
            r = run_fixed(pqgpu, ctx, args, world, rank, dist, stream, kind,
                          p_null=args.p_null if kind == "levels" else None, steps=short_steps, warmup=2,
                          extras=False, strong=True)
            sub[kind]["strong_scaling"] = dict(brief(r, unit_key), scaling="strong")
    ctx.close()
    top = kinds[0]
    result = dict(head)
    result.update(sub[top])
    result.setdefault("dtype", {"levels": "int16 levels + int32 values", "dict": "uint16 indices -> int64",
                                "delta": "int64 (wrapping)"}.get(top))
    if len(kinds) > 1:
        result["configs"] = {k: sub[k] for k in kinds[1:]}
    if rank == 0:
        try:
            result["copy_ceiling_gbs"] = copy_ceiling_gbs()
        except Exception as e:  # pragma: no cover
            result["copy_ceiling_gbs"] = str(e)
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
