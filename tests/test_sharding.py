"""Multi-GPU layout on CPU: row-group partition over ranks and the max-over-ranks step time,
run with world_size 2 over gloo (the nccl/RCCL path is the same code with GPU tensors)."""
import os

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import sharding


def test_partition_covers_every_row_group_once():
    for n in (0, 1, 2, 7, 64, 1000):
        sizes = [((i * 7919) % 13 + 1) * 1000 for i in range(n)]
        for world in (1, 2, 3, 8):
            got = [sharding.row_groups_for_rank(sizes, world, r) for r in range(world)]
            flat = [i for g in got for i in g]
            assert flat == list(range(n)), (n, world)


def test_partition_is_balanced():
    sizes = [1000] * 64
    parts = [sharding.row_groups_for_rank(sizes, 8, r) for r in range(8)]
    assert all(len(p) == 8 for p in parts)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sizes = [100 + 17 * i for i in range(33)]
        mine = sharding.row_groups_for_rank(sizes, world, rank)
        allp = [None] * world
        dist.all_gather_object(allp, mine)
        t = sharding.max_over_ranks(0.010 * (rank + 1), dist)
        seeds = [None] * world
        dist.all_gather_object(seeds, sharding.shard_seed(5, rank))
        q.put((rank, allp, t, seeds))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gloo_world2_partition_and_max():
    world = 2
    port = 29500 + os.getpid() % 2000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    for rank, allp, t, seeds in res:
        flat = [i for part in allp for i in part]
        assert flat == list(range(33))
        assert abs(t - 0.020) < 1e-12  # slowest rank
        assert len(set(seeds)) == world


@pytest.mark.timeout(240)
def test_bench_launches_n_ranks_dry_run():
    """bench.py --gpus 2 starts two ranks itself (torch.distributed.run, 127.0.0.1) when no
    WORLD_SIZE is set; on the gloo dry path rank 0 prints one line with n_gpus 2 and both
    ranks' distinct partition seeds."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=220, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["dry_run"] is True and res["value"] is None
    assert len(set(res["config"]["partition_seeds"])) == 2
    # config 5: the two ranks split the first 22 row groups of the one 88-row-group file
    assert res["config"]["alltypes_row_groups"] == [list(range(11)), list(range(11, 22))]


def test_bench_alltypes_partition_is_one_file():
    """bench.alltypes_partition: at N GPUs the ranks split the first 11 N row groups of config 5's
    88-row-group file (weak scaling), contiguous, each exactly once; at 8 GPUs the whole file."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    args = bench.parse([])
    for world in (1, 2, 4, 8):
        parts = [bench.alltypes_partition(args, world, r) for r in range(world)]
        assert [g for p in parts for g in p] == list(range(11 * world))
        assert all(len(p) == 11 for p in parts)
    assert bench.alltypes_partition(args, 8, 7)[-1] == bench.FILE_ROW_GROUPS * 11 - 1


def test_bench_refuses_debug_env():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PQG_DEBUG="256")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "PQG_DEBUG" in r.stderr


# ---- shards decode independently: the concatenation of per-rank decodes is the whole decode


def _rg_decode_oracle(rg_index, rows):
    """Oracle decode of alltypes row group `rg_index` (columns id and date_string_col)."""
    import pyoracle
    import pqgtools
    blob, pages, info = pqgtools.alltypes_row_group(rows, rg_index * rows, 0.1, 77, threads=2)
    out = []
    for j in (0, 8):
        specs = [pyoracle.PageSpec(p.page_type, blob[p.offset:p.offset + p.nbytes].tobytes(), p.num_values,
                                   p.encoding, p.def_encoding, p.rep_encoding)
                 for p in (pages[i] for i in range(info.chunk_first[j], info.chunk_first[j + 1]))]
        r = pyoracle.read_column(pqgtools.ALLTYPES[j][1], specs, max_def=1)
        assert r["status"] == 0, r["message"]
        out.append((r["def"].tobytes(), r["values"].tobytes() if j == 0 else r["bytes"]))
    return info.blob_len, out


def _shard_worker(rank, world, port, q, nrg, rows):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "gen"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sizes = [rows * (1 + (i % 3)) for i in range(nrg)]  # uneven byte sizes
        mine = sharding.row_groups_for_rank(sizes, world, rank)
        dec = {g: _rg_decode_oracle(g, rows)[1] for g in mine}
        allp = [None] * world
        dist.all_gather_object(allp, dec)
        q.put((rank, allp))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_gloo_world2_shards_concatenate_to_whole():
    world, nrg, rows = 2, 5, 20_000
    port = 31500 + os.getpid() % 2000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, q, nrg, rows)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=200) for _ in range(world)]
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    _, allp = res[0]
    merged = {}
    for part in allp:
        assert not (set(part) & set(merged))  # every row group decoded by exactly one rank
        merged.update(part)
    assert sorted(merged) == list(range(nrg))
    for g in range(nrg):  # the unsharded decode, row group by row group in file order
        assert merged[g] == _rg_decode_oracle(g, rows)[1], g


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["levels", "dict"])
def test_gpu_page_shards_concatenate_to_whole(kind):
    """Configs 2-3 shard a chunk's pages across GPUs (the dictionary page goes to
    every shard). Decoding 4 contiguous page ranges in sequence gives the whole chunk's decode."""
    import ctypes as C

    import numpy as np
    import torch

    import pqgpu
    import pqgtools
    L = pqgtools.lib()
    info = pqgtools.WorkloadInfo()
    n, pv = 3_000_000, 1 << 18
    if kind == "levels":
        gen = lambda b, cap, pg, pc: L.pqg_gen_levels_plain(n, 0.3, pv, 99, 8, b, cap, pg, pc, C.byref(info))
        col = pqgpu.Column(pqgpu.INT32, -1, 1, 0)
    else:
        gen = lambda b, cap, pg, pc: L.pqg_gen_dict_int64(n, 4096, pv, 99, 8, b, cap, pg, pc, C.byref(info))
        col = pqgpu.Column(pqgpu.INT64, -1, 0, 0)
    assert gen(None, 0, None, 0) == 0
    host = np.zeros(info.blob_len + 64, np.uint8)
    pages = (pqgpu.Page * info.npages)()
    assert gen(host.ctypes.data_as(C.c_void_p), info.blob_len, pages, info.npages) == 0
    d_blob = torch.from_numpy(host).cuda()
    es = 4 if kind == "levels" else 8
    ctx = pqgpu.Context(0)

    def decode(idx):
        sel = (pqgpu.Page * len(idx))(*[pages[i] for i in idx])
        nlev = sum(pages[i].num_values for i in idx if pages[i].page_type == pqgpu.PAGE_DATA)
        d_def = torch.empty(nlev + 8, dtype=torch.int16, device="cuda")
        d_val = torch.empty(nlev * es + 64, dtype=torch.uint8, device="cuda")
        out = pqgpu.Output(d_def.data_ptr() if col.max_def else None, None, d_val.data_ptr(), nlev * es, None, 0, 0, 0, 0)
        ctx.decode_async(col, d_blob.data_ptr(), info.blob_len, sel, out, torch.cuda.current_stream().cuda_stream)
        st, bad = ctx.sync()
        assert st == 0, (st, bad, ctx.error_message())
        return (d_def[:out.num_levels].cpu().numpy().tobytes() if col.max_def else b"",
                d_val[:out.num_values * es].cpu().numpy().tobytes())

    try:
        first = 1 if kind == "dict" else 0
        data = list(range(first, info.npages))
        whole = decode(list(range(info.npages)))
        parts = [decode(list(range(first)) + data[r * len(data) // 4:(r + 1) * len(data) // 4]) for r in range(4)]
    finally:
        ctx.close()
    assert b"".join(p[0] for p in parts) == whole[0]
    assert b"".join(p[1] for p in parts) == whole[1]


# ---- strong scaling: N ranks split ONE stream into contiguous page ranges


def test_page_ranges_cover_the_stream_once():
    for npages in (1, 2, 7, 954):
        for world in (1, 2, 3, 8):
            rs = [sharding.pages_for_rank(npages, world, r) for r in range(world)]
            assert rs[0][0] == 0 and all(a[0] + a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert sum(c for _, c in rs) == npages and max(c for _, c in rs) - min(c for _, c in rs) <= 1


STREAM_N, STREAM_PV = 5 * 65536 + 777, 65536  # six pages, the last ragged


def _stream_pages(kind, first, count):
    """Pages [first, first + count) of one config-2/3/4 stream from the bench's page-range
    generators (the dictionary page first for config 3)."""
    import ctypes as C

    import numpy as np
    import pqgpu
    import pqgtools
    L = pqgtools.lib()
    info = pqgtools.WorkloadInfo()
    if kind == "levels":
        gen = lambda b, cap, pg, pc: L.pqg_gen_levels_plain_pages(STREAM_N, 0.1, STREAM_PV, 0x5EED0002, first, count,
                                                                  2, b, cap, pg, pc, C.byref(info))
    elif kind == "dict":
        gen = lambda b, cap, pg, pc: L.pqg_gen_dict_int64_pages(STREAM_N, 65536, STREAM_PV, 0x5EED0003, first, count,
                                                                2, b, cap, pg, pc, C.byref(info))
    else:
        gen = lambda b, cap, pg, pc: L.pqg_gen_delta_int64_pages(STREAM_N, 16, STREAM_PV, 128, 4, 0x5EED0004, first,
                                                                 count, 2, b, cap, pg, pc, C.byref(info))
    assert gen(None, 0, None, 0) == 0
    host = np.zeros(info.blob_len + 64, np.uint8)
    pages = (pqgpu.Page * info.npages)()
    assert gen(host.ctypes.data_as(C.c_void_p), info.blob_len, pages, info.npages) == 0
    return host, pages, info


def _stream_decode_oracle(kind, first, count):
    import pyoracle
    host, pages, info = _stream_pages(kind, first, count)
    specs = [pyoracle.PageSpec(p.page_type, host[p.offset:p.offset + p.nbytes].tobytes(), p.num_values, p.encoding,
                               p.def_encoding, p.rep_encoding) for p in (pages[i] for i in range(info.npages))]
    ptype = {"levels": pyoracle.INT32, "dict": pyoracle.INT64, "delta": pyoracle.INT64}[kind]
    r = pyoracle.read_column(ptype, specs, max_def=1 if kind == "levels" else 0)
    assert r["status"] == 0, r["message"]
    return (r["def"].tobytes() if kind == "levels" else b""), r["values"].tobytes()


def _stream_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "oracle"))
    sys.path.insert(0, os.path.join(root, "tools", "gen"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        npages = (STREAM_N + STREAM_PV - 1) // STREAM_PV
        first, count = sharding.pages_for_rank(npages, world, rank)
        mine = {k: _stream_decode_oracle(k, first, count) for k in ("levels", "dict", "delta")}
        allp = [None] * world
        dist.all_gather_object(allp, (first, count, mine))
        q.put((rank, allp))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_gloo_world2_stream_split_concatenates_to_whole():
    """bench.py --split strong: each of 2 ranks generates and decodes its contiguous page range of
    one stream (configs 2-4, the dictionary page replicated); the ranks' outputs in rank order are
    the single-rank decode of the whole stream, byte for byte."""
    world = 2
    port = 33500 + os.getpid() % 2000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_stream_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=200) for _ in range(world)]
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    _, allp = res[0]
    assert [a[0] for a in allp] == [0, allp[0][1]]
    npages = (STREAM_N + STREAM_PV - 1) // STREAM_PV
    for kind in ("levels", "dict", "delta"):
        whole = _stream_decode_oracle(kind, 0, npages)
        assert b"".join(a[2][kind][0] for a in allp) == whole[0], kind
        assert b"".join(a[2][kind][1] for a in allp) == whole[1], kind


def test_page_range_generator_is_the_whole_streams_pages():
    """A page range from the generator holds exactly those pages of the whole stream."""
    for kind in ("levels", "dict", "delta"):
        hw, pw, iw = _stream_pages(kind, 0, 6)
        hr, pr, ir = _stream_pages(kind, 2, 3)
        d = 1 if kind == "dict" else 0
        for i in range(ir.npages - d):
            a, b = pr[d + i], pw[d + 2 + i]
            assert (a.num_values, a.nbytes) == (b.num_values, b.nbytes)
            assert hr[a.offset:a.offset + a.nbytes].tobytes() == hw[b.offset:b.offset + b.nbytes].tobytes()
