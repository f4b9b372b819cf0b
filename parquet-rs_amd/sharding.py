"""Row-group and page-range partitioning across GPUs (one process per GPU).

parquet-rs reads row groups independently (file/reader.rs:252-260 hands each RowGroupReader
its own file handle), so the multi-GPU layout is a partition of row groups over ranks with no
exchange on the data path. The only collectives are the bench's barrier and the max-over-ranks
reduction of the step time.
"""


def row_groups_for_rank(sizes, world, rank):
    """Contiguous, byte-balanced split of row groups (sizes = bytes per row group) over
    `world` ranks; returns this rank's row-group indices. Every row group lands on exactly one
    rank, in file order."""
    n = len(sizes)
    if world <= 1:
        return list(range(n))
    total = float(sum(sizes)) or 1.0
    bounds, acc, r = [0], 0.0, 1
    for i, s in enumerate(sizes):
        acc += s
        while r < world and acc >= total * r / world and len(bounds) < world:
            bounds.append(i + 1)
            r += 1
    while len(bounds) < world:
        bounds.append(n)
    bounds.append(n)
    return list(range(bounds[rank], bounds[rank + 1]))


def pages_for_rank(npages, world, rank):
    """Contiguous page range [first, first + count) of one column-chunk stream for `rank` (strong
    scaling: N ranks split the same stream; pages are independent decode units once the dictionary
    page is replicated, and DELTA state resets per page, decoding.rs:501-533). Ranks differ by at
    most one page."""
    if world <= 1:
        return 0, npages
    q, r = divmod(npages, world)
    first = rank * q + min(rank, r)
    return first, q + (1 if rank < r else 0)


def shard_seed(base, rank):
    """Seed of rank `rank`'s synthetic partition (distinct row groups per rank)."""
    return base + 1000003 * rank


def max_over_ranks(x, dist=None, device="cpu"):
    """Step time of the slowest rank (the whole job finishes when it does)."""
    if dist is None:
        return float(x)
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
