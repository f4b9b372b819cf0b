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


def _rg_outputs(torch, info, rows):
    import pqgpu
    keep, outs = [], []
    for j, (_, pt) in enumerate(pqgtools.ALLTYPES):
        d_def = torch.empty(rows + 64, dtype=torch.int16, device="cuda")
        d_val = torch.empty(info.value_bytes[j] + 64, dtype=torch.uint8, device="cuda")
        d_off = torch.empty(rows + 8, dtype=torch.int64, device="cuda") if pt == 6 else None
        outs.append(pqgpu.Output(d_def.data_ptr(), None, d_val.data_ptr(), info.value_bytes[j] + 64,
                                 d_off.data_ptr() if d_off is not None else None, rows + 1 if pt == 6 else 0,
                                 0, 0, 0))
        keep.append((d_def, d_val, d_off))
    return keep, outs


def _rg_pages(pqgpu, pages, info):
    return [(pqgpu.Page * (info.chunk_first[j + 1] - info.chunk_first[j]))(
        *[pages[i] for i in range(info.chunk_first[j], info.chunk_first[j + 1])]) for j in range(11)]


@pytest.mark.gpu
@pytest.mark.parametrize("nstreams", [1, 4])
def test_gpu_row_group_decoder(rowgroup, nstreams):
    """pqg_rg_decode: all 11 column chunks of the row group over `nstreams` streams, twice in a
    row (the second decode into other outputs) before one pqg_rg_sync; every column matches the
    generator's cells and its counters are filled."""
    import pqgpu
    import torch
    blob, pages, info = rowgroup
    d_blob = torch.from_numpy(np.ascontiguousarray(blob[:info.blob_len + 64])).cuda()
    cols = [pqgpu.Column(pt, -1, 1, 0) for _, pt in pqgtools.ALLTYPES]
    parr = _rg_pages(pqgpu, pages, info)
    rgd = pqgpu.RowGroupDecoder(0, nstreams)
    try:
        s = torch.cuda.current_stream().cuda_stream
        sets = [_rg_outputs(torch, info, ROWS) for _ in range(2)]
        oas = [rgd.decode_async(cols, d_blob.data_ptr(), info.blob_len, parr, outs, s) for _, outs in sets]
        st, bcol, bad = rgd.sync()
        assert st == 0, (st, bcol, bad, rgd.error_message())
        torch.cuda.current_stream().synchronize()
        for (keep, _), oa in zip(sets, oas):
            for j, (name, pt) in enumerate(pqgtools.ALLTYPES):
                lv, vals, offs = pqgtools.alltypes_truth(ROW0, ROWS, j, P_NULL, SEED, info.value_bytes[j])
                d_def, d_val, d_off = keep[j]
                assert oa[j].num_levels == ROWS and oa[j].num_values == info.num_values[j], name
                np.testing.assert_array_equal(d_def[:ROWS].cpu().numpy(), lv)
                assert d_val[:info.value_bytes[j]].cpu().numpy().tobytes() == vals.tobytes(), name
                if offs is not None:
                    assert oa[j].num_bytes == info.value_bytes[j]
                    np.testing.assert_array_equal(d_off[:len(offs)].cpu().numpy(), offs)
    finally:
        rgd.close()


@pytest.mark.gpu
def test_gpu_row_group_decoder_reports_failing_column(rowgroup):
    """A column chunk whose data page is cut short fails with EOF-class status; pqg_rg_sync names
    that column (the lowest failing one) and its page while the other columns still decode."""
    import pqgpu
    import torch
    blob, pages, info = rowgroup
    d_blob = torch.from_numpy(np.ascontiguousarray(blob[:info.blob_len + 64])).cuda()
    cols = [pqgpu.Column(pt, -1, 1, 0) for _, pt in pqgtools.ALLTYPES]
    parr = _rg_pages(pqgpu, pages, info)
    # bool_col (column 1): one PLAIN data page; drop most of its value bytes
    parr[1][0].nbytes = 64
    rgd = pqgpu.RowGroupDecoder(0, 4)
    try:
        keep, outs = _rg_outputs(torch, info, ROWS)
        rgd.decode_async(cols, d_blob.data_ptr(), info.blob_len, parr, outs, torch.cuda.current_stream().cuda_stream)
        st, bcol, bad = rgd.sync()
        assert st != 0 and bcol == 1 and bad == 0, (st, bcol, bad)
        lv, vals, _ = pqgtools.alltypes_truth(ROW0, ROWS, 0, P_NULL, SEED, info.value_bytes[0])
        assert keep[0][1][:info.value_bytes[0]].cpu().numpy().tobytes() == vals.tobytes()
    finally:
        rgd.close()


@pytest.mark.gpu
def test_gpu_row_group_decoder_reports_earliest_row_group():
    """Two row groups in flight before one sync: the first fails on column 5 (bigint_col's data
    page cut short), the second on column 1. The reference reads row group 0 first and stops at
    its column 5, so pqg_rg_sync_call names call 0, column 5 (not the lower column of call 1)."""
    import pqgpu
    import torch
    blob, pages, info = pqgtools.alltypes_row_group(70_000, ROW0, P_NULL, SEED, threads=8)
    d_blob = torch.from_numpy(np.ascontiguousarray(blob[:info.blob_len + 64])).cuda()
    cols = [pqgpu.Column(pt, -1, 1, 0) for _, pt in pqgtools.ALLTYPES]
    first, second = _rg_pages(pqgpu, pages, info), _rg_pages(pqgpu, pages, info)
    first[5][1].nbytes = 40      # bigint_col: dictionary page, then its one data page
    second[1][0].nbytes = 64     # bool_col: its PLAIN data page
    rgd = pqgpu.RowGroupDecoder(0, 4)
    try:
        s = torch.cuda.current_stream().cuda_stream
        sets = [_rg_outputs(torch, info, 70_000) for _ in range(2)]
        rgd.decode_async(cols, d_blob.data_ptr(), info.blob_len, first, sets[0][1], s)
        rgd.decode_async(cols, d_blob.data_ptr(), info.blob_len, second, sets[1][1], s)
        st, call, bcol, bad = rgd.sync_call()
        assert st != 0 and (call, bcol, bad) == (0, 5, 1), (st, call, bcol, bad, rgd.error_message())
        # one row group failing alone: call 0, its column
        rgd.decode_async(cols, d_blob.data_ptr(), info.blob_len, _rg_pages(pqgpu, pages, info), sets[0][1], s)
        rgd.decode_async(cols, d_blob.data_ptr(), info.blob_len, second, sets[1][1], s)
        st, call, bcol, bad = rgd.sync_call()
        assert st != 0 and (call, bcol, bad) == (1, 1, 0), (st, call, bcol, bad)
    finally:
        rgd.close()


@pytest.mark.gpu
def test_gpu_row_group_pipeline():
    """The bench's config-5 loop at small scale: four row groups decoded by one row-group decoder
    (16 streams), alternating two launch streams and two output sets, so that row group g + 1 is
    enqueued while g still runs and every column context cycles through both staging slots; each
    row group's columns are checked against the generator's cells once its decode is known done."""
    import pqgpu
    import torch
    rows, nrg = 70_000, 4
    rgs = [pqgtools.alltypes_row_group(rows, ROW0 + g * rows, P_NULL, SEED, threads=8) for g in range(nrg)]
    cols = [pqgpu.Column(pt, -1, 1, 0) for _, pt in pqgtools.ALLTYPES]
    blobs = [torch.from_numpy(np.ascontiguousarray(b[:i.blob_len + 64])).cuda() for b, _, i in rgs]
    parrs = [_rg_pages(pqgpu, p, i) for _, p, i in rgs]
    vcap = max(max(i.value_bytes) for _, _, i in rgs)

    class Info:  # one output set sized for every row group
        value_bytes = [vcap] * 11
    sets = [_rg_outputs(torch, Info, rows) for _ in range(2)]
    lanes = [torch.cuda.current_stream(), torch.cuda.Stream()]
    rgd = pqgpu.RowGroupDecoder(0, 16)
    try:
        done = [torch.cuda.Event() for _ in range(nrg)]
        oas = []
        for g in range(nrg):
            lane = lanes[g % 2]
            if g >= 2:  # output set g % 2 is free once row group g - 2 was checked
                lane.wait_event(done[g - 2])
            oas.append(rgd.decode_async(cols, blobs[g].data_ptr(), rgs[g][2].blob_len, parrs[g], sets[g % 2][1],
                                        lane.cuda_stream))
            done[g].record(lane)
            if g >= 1:  # check row group g - 1 while g runs
                _check_rg(torch, rgs, sets, done, oas, g - 1, rows)
        st, bcol, bad = rgd.sync()
        assert st == 0, (st, bcol, bad, rgd.error_message())
        _check_rg(torch, rgs, sets, done, oas, nrg - 1, rows)
    finally:
        rgd.close()


def _check_rg(torch, rgs, sets, done, oas, g, rows):
    done[g].synchronize()
    keep = sets[g % 2][0]
    info = rgs[g][2]
    for j, (name, pt) in enumerate(pqgtools.ALLTYPES):
        lv, vals, offs = pqgtools.alltypes_truth(ROW0 + g * rows, rows, j, P_NULL, SEED, info.value_bytes[j])
        d_def, d_val, d_off = keep[j]
        np.testing.assert_array_equal(d_def[:rows].cpu().numpy(), lv)
        assert d_val[:info.value_bytes[j]].cpu().numpy().tobytes() == vals.tobytes(), (g, name)
        if offs is not None:
            np.testing.assert_array_equal(d_off[:len(offs)].cpu().numpy(), offs)
