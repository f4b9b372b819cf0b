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


def test_bench_refuses_debug_env():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PQG_DEBUG="256")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "PQG_DEBUG" in r.stderr
