"""Config 5 (alltypes_plain schema written with the reference writer's defaults): the generator's
pages decode, through the oracle (CPU) and through pqg_decode_chunk (GPU), to the generator's own
cells; row-group shards decode independently (the multi-GPU partition)."""
import os

import numpy as np
import pytest

import pqgtools

ROWS = 300_000   # > 262 144: `id` and `timestamp_col` fall back to PLAIN past the 1 MiB dictionary
ROW0 = 4_000_000
P_NULL = 0.05
SEED = 0xA11


@pytest.fixture(scope="module")
def rowgroup():
    return pqgtools.alltypes_row_group(ROWS, ROW0, P_NULL, SEED, threads=8)


def _specs(oracle, blob, pages, info, j):
    return [oracle.PageSpec(p.page_type, blob[p.offset:p.offset + p.nbytes].tobytes(), p.num_values,
                            p.encoding, p.def_encoding, p.rep_encoding)
            for p in (pages[i] for i in range(info.chunk_first[j], info.chunk_first[j + 1]))]


def test_writer_page_layout(rowgroup):
    blob, pages, info = rowgroup
    enc = lambda j: [(pages[i].page_type, pages[i].encoding)
                     for i in range(info.chunk_first[j], info.chunk_first[j + 1])]
    # dictionary columns: dictionary page first, then one buffered data page (column/writer.rs:406-420)
    for j in (2, 3, 4, 5, 6, 7, 8, 9):
        assert enc(j) == [(2, 2), (0, 2)], pqgtools.ALLTYPES[j][0]
    # bool_col: PLAIN, no dictionary support (:744-756)
    assert enc(1) == [(0, 0)]
    # id / timestamp_col: dictionary fallback past 1 MiB, then PLAIN pages cut at 1 MiB
    for j in (0, 10):
        e = enc(j)
        assert e[0] == (2, 2) and e[1] == (0, 2) and all(x == (0, 0) for x in e[2:]) and len(e) >= 3


@pytest.mark.parametrize("j", range(11))
def test_oracle_decodes_generator_cells(oracle, rowgroup, j):
    blob, pages, info = rowgroup
    name, pt = pqgtools.ALLTYPES[j]
    ref = oracle.read_column(pt, _specs(oracle, blob, pages, info, j), max_def=1, batch_size=1024)
    assert ref["status"] == 0, ref["message"]
    lv, vals, offs = pqgtools.alltypes_truth(ROW0, ROWS, j, P_NULL, SEED, info.value_bytes[j])
    np.testing.assert_array_equal(ref["def"], lv)
    if pt == oracle.BYTE_ARRAY:
        assert ref["bytes"] == vals.tobytes()
        np.testing.assert_array_equal(ref["offsets"], offs)
    else:
        assert ref["values"].tobytes() == vals.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("j", range(11))
def test_gpu_decodes_alltypes_chunks(oracle, rowgroup, j):
    import pqgpu
    import torch
    assert torch.cuda.is_available()
    blob, pages, info = rowgroup
    name, pt = pqgtools.ALLTYPES[j]
    ctx = pqgpu.Context(0)
    try:
        got = pqgpu.decode_column(ctx, pt, _specs(oracle, blob, pages, info, j), max_def=1)
    finally:
        ctx.close()
    assert got["status"] == 0, got["message"]
    lv, vals, offs = pqgtools.alltypes_truth(ROW0, ROWS, j, P_NULL, SEED, info.value_bytes[j])
    np.testing.assert_array_equal(got["def"], lv)
    if pt == oracle.BYTE_ARRAY:
        assert got["bytes"] == vals.tobytes()
        np.testing.assert_array_equal(got["offsets"], offs)
    else:
        assert got["values"].view(np.uint8).tobytes() == vals.tobytes()
