"""The file-to-device product path (pqg_rgr_*, csrc/host/rg_reader.cpp): alltypes row groups written
as parquet files (pqgtools.write_alltypes_file: uncompressed, SNAPPY, GZIP), read by the host reader
(headers, parallel page fill / decompression into pinned staging) and decoded on the GPU, two row
groups in flight, compared with the generator's cells (pqgtools.alltypes_truth).

The writer itself is pinned on the CPU against pyarrow's reader, and the host page walk against
the generator's own pages (file/reader.rs:420-522 yields exactly the pages the writer wrote)."""
import numpy as np
import pytest

import pqgtools

ROWS = 100_000      # > 87 381: timestamp_col's 1 MiB dictionary falls back to PLAIN pages
GROUPS = 3
ROW0 = 7_000_000
P_NULL = 0.05
SEED = 0x5EED0F11
CODECS = {0: "none", 1: "snappy", 2: "gzip"}


@pytest.fixture(scope="module", params=[0, 1, 2], ids=lambda c: CODECS[c])
def alltypes_file(request, tmp_path_factory):
    path = str(tmp_path_factory.mktemp("rgr") / f"alltypes_{CODECS[request.param]}.parquet")
    pqgtools.write_alltypes_file(path, ROWS, GROUPS, row0=ROW0, p_null=P_NULL, seed=SEED, codec=request.param,
                                 threads=8)
    return path, request.param


def _truth(g, j):
    r0 = ROW0 + g * ROWS
    lv, vals, offs = pqgtools.alltypes_truth(r0, ROWS, j, P_NULL, SEED, ROWS * 16)  # room for any cell
    nv = int(np.count_nonzero(lv))
    pt = pqgtools.ALLTYPES[j][1]
    nb = int(offs[-1]) if offs is not None else nv * {0: 1, 1: 4, 2: 8, 3: 12, 4: 4, 5: 8}[pt]
    return lv, vals[:nb], offs


def test_pyarrow_reads_the_written_file(alltypes_file):
    pq = pytest.importorskip("pyarrow.parquet")
    path, codec = alltypes_file
    f = pq.ParquetFile(path)
    assert f.metadata.num_row_groups == GROUPS and f.metadata.num_rows == ROWS * GROUPS
    assert f.metadata.row_group(0).column(0).compression == {0: "UNCOMPRESSED", 1: "SNAPPY", 2: "GZIP"}[codec]
    t = f.read_row_group(1)
    for j, (name, pt) in enumerate(pqgtools.ALLTYPES):
        lv, vals, offs = _truth(1, j)
        col = t.column(name)
        valid = np.asarray(col.is_valid())
        np.testing.assert_array_equal(valid, lv == 1, err_msg=name)
        if pt == 6:  # BYTE_ARRAY
            got = b"".join(x for x in col.to_pylist() if x is not None)
            assert got == vals.tobytes(), name
        elif pt == 3:  # INT96 is read as timestamps; checked through the host page walk below
            continue
        elif pt == 0:
            got = np.asarray(col.drop_null(), dtype=np.uint8)
            np.testing.assert_array_equal(got, vals, err_msg=name)
        else:
            got = np.asarray(col.drop_null()).tobytes()
            assert got == vals.tobytes(), name


def test_host_page_walk_yields_the_generator_pages(alltypes_file):
    import pqgpu
    path, _ = alltypes_file
    r = pqgpu.FileReader(path)
    assert r.num_row_groups == GROUPS and r.num_columns == 11
    blob, pages, info = pqgtools.alltypes_row_group(ROWS, ROW0 + 2 * ROWS, P_NULL, SEED, threads=8)
    for j in range(11):
        hb, hp, n = r.chunk_pages(2, j)
        first, last = info.chunk_first[j], info.chunk_first[j + 1]
        assert n == last - first
        for i in range(n):
            a, b = hp[i], pages[first + i]
            assert (a.page_type, a.num_values, a.encoding, a.nbytes) == (b.page_type, b.num_values, b.encoding,
                                                                          b.nbytes)
            assert hb[a.offset:a.offset + a.nbytes] == blob[b.offset:b.offset + b.nbytes].tobytes()
    r.close()


def _check_row_group(rd, g):
    for j, (name, pt) in enumerate(pqgtools.ALLTYPES):
        res = rd.host_arrays(j, pt)
        assert res["status"] == 0, name
        lv, vals, offs = _truth(g, j)
        assert res["num_levels"] == ROWS
        np.testing.assert_array_equal(res["def_levels"], lv, err_msg=name)
        assert res["num_values"] == int(np.count_nonzero(lv)), name
        if pt == 6:
            np.testing.assert_array_equal(res["offsets"], offs, err_msg=name)
            assert res["values"].tobytes() == vals.tobytes(), name
        else:
            assert res["values"].tobytes() == vals.tobytes(), name


@pytest.mark.gpu
def test_row_groups_pipelined_from_file(alltypes_file):
    import pqgpu
    path, _ = alltypes_file
    r = pqgpu.FileReader(path)
    rd = pqgpu.RowGroupReader(r, device=0, host_threads=8, host_output=True)
    rd.submit(0)
    rd.submit(1)
    with pytest.raises(pqgpu.PqgError):
        rd.submit(2)  # two in flight
    for g in range(GROUPS):
        st, rg, col, page = rd.wait()
        assert (st, rg, col, page) == (0, g, -1, -1), rd.error()
        if g + 2 < GROUPS:
            rd.submit(g + 2)
        _check_row_group(rd, g)
    # row groups again, reusing the staging and outputs, in another order
    for g in (2, 0):
        rd.submit(g)
        assert rd.wait()[:2] == (0, g)
        _check_row_group(rd, g)
    s = rd.stats()
    assert s["row_groups"] == GROUPS + 2 and s["staged_bytes"] > 0 and s["output_bytes"] > 0
    rd.close()
    r.close()


@pytest.mark.gpu
def test_device_outputs_without_host_copies(alltypes_file):
    import ctypes as C
    import pqgpu
    path, _ = alltypes_file
    r = pqgpu.FileReader(path)
    rd = pqgpu.RowGroupReader(r, host_output=False)
    rd.submit(1)
    assert rd.wait()[0] == 0
    st, o = rd.column(0)  # id: int32
    assert st == 0 and not o.host_values
    lv, vals, _ = _truth(1, 0)
    got = np.zeros(o.num_values * 4, np.uint8)
    hip = C.CDLL("libamdhip64.so")  # the library's own runtime (no torch in this process's path)
    assert hip.hipMemcpy(C.c_void_p(got.ctypes.data), C.c_void_p(o.values), C.c_size_t(got.nbytes), 2) == 0
    assert got.tobytes() == vals.tobytes()
    rd.close()
    r.close()


@pytest.mark.gpu
def test_corrupt_page_fails_at_its_column(tmp_path):
    """A damaged page in column 3 of row group 1: that row group reports column 3, the other row
    groups decode in full (the reference fails reading that column chunk, file/reader.rs:420-461)."""
    import pqgpu
    pq = pytest.importorskip("pyarrow.parquet")
    path = str(tmp_path / "bad.parquet")
    pqgtools.write_alltypes_file(path, ROWS, GROUPS, row0=ROW0, p_null=P_NULL, seed=SEED, codec=1, threads=8)
    cc = pq.ParquetFile(path).metadata.row_group(1).column(3)
    at = cc.data_page_offset + 64  # inside the data page's compressed payload
    data = bytearray(open(path, "rb").read())
    for k in range(64):
        data[at + k] = 0xFF
    open(path, "wb").write(bytes(data))
    r = pqgpu.FileReader(path)
    rd = pqgpu.RowGroupReader(r)
    for g in range(GROUPS):
        rd.submit(g)
        st, rg, col, page = rd.wait()
        if g == 1:
            assert st != 0 and (rg, col) == (1, 3) and page >= 0, (st, rg, col, page)
            assert rd.column(2)[0] == 0
            assert rd.column(3)[0] != 0
        else:
            assert st == 0, rd.error()
            _check_row_group(rd, g)
    rd.close()
    r.close()


def _damaged_file(tmp_path, payload_page=None, header_page=None, col=10, rg=1):
    """The alltypes file (SNAPPY) with page `payload_page` of (rg, col) given a garbled compressed
    payload and/or page `header_page`'s header overwritten. timestamp_col holds three pages at
    ROWS rows: its dictionary page, a dictionary-encoded page, the PLAIN fallback page."""
    import _pagewalk
    pq = pytest.importorskip("pyarrow.parquet")
    path = str(tmp_path / f"bad_{payload_page}_{header_page}.parquet")
    pqgtools.write_alltypes_file(path, ROWS, GROUPS, row0=ROW0, p_null=P_NULL, seed=SEED, codec=1, threads=8)
    cc = pq.ParquetFile(path).metadata.row_group(rg).column(col)
    start = cc.dictionary_page_offset if cc.has_dictionary_page else cc.data_page_offset
    data = bytearray(open(path, "rb").read())
    pages = _pagewalk.chunk_pages(data, start, cc.total_compressed_size)
    assert len(pages) == 3
    if payload_page is not None:
        _, at, n, _ = pages[payload_page]
        for k in range(4):  # the snappy preamble (uncompressed length): the page fails to decompress
            data[at + k] = 0xFF
    if header_page is not None:
        at = pages[header_page][0]
        for k in range(6):
            data[at + k] = 0xFF
    open(path, "wb").write(bytes(data))
    return path


def test_decompression_failure_before_a_bad_header_is_reported_first(tmp_path):
    """Pages are read in order (SerializedPageReader::get_next_page reads and decompresses one page
    before parsing the next header, file/reader.rs:420-461): a garbled payload on page 1 is the
    chunk's error even though page 2's header is damaged too."""
    import pqgpu
    both = pqgpu.FileReader(_damaged_file(tmp_path, payload_page=1, header_page=2))
    one = pqgpu.FileReader(_damaged_file(tmp_path, payload_page=1))
    hdr = pqgpu.FileReader(_damaged_file(tmp_path, header_page=2))
    errs = []
    for r in (both, one, hdr):
        with pytest.raises(pqgpu.PqgError) as e:
            r.chunk_pages(1, 10)
        errs.append((e.value.status, str(e.value)))
    assert errs[0] == errs[1] and errs[0] != errs[2], errs
    for r in (both, one, hdr):
        r.close()


@pytest.mark.gpu
def test_row_group_reader_reports_the_earliest_host_failure(tmp_path):
    """pqg_rgr: a damaged payload on page 1 and a damaged header on page 2 of timestamp_col report
    page 1; a damaged header alone reports page 2 after the pages before it decoded."""
    import pqgpu
    for payload, header, want in ((1, 2, 1), (None, 2, 2)):
        r = pqgpu.FileReader(_damaged_file(tmp_path, payload_page=payload, header_page=header))
        rd = pqgpu.RowGroupReader(r)
        rd.submit(1)
        st, rg, col, page = rd.wait()
        assert st != 0 and (rg, col, page) == (1, 10, want), (st, rg, col, page, rd.error())
        assert all(rd.column(j)[0] == 0 for j in range(10))
        assert rd.column(10)[0] != 0
        rd.close()
        r.close()


@pytest.mark.gpu
def test_column_reader_serves_the_pages_before_a_bad_header(tmp_path):
    """read_batch over a chunk whose third page header is damaged: the levels and values of the
    pages before it come back as decoded, the batch that reaches the damaged page fails
    (read_new_page -> get_next_page, column/reader.rs:269-275)."""
    import pqgpu
    r = pqgpu.FileReader(_damaged_file(tmp_path, header_page=2))
    ctx = pqgpu.Context(0)
    cr = r.column_reader(1, 10, ctx)
    lv, vals, _ = _truth(1, 10)
    good = pqgpu.FileReader(_damaged_file(tmp_path))  # the same file undamaged: page 1's level count
    _, hp, n = good.chunk_pages(1, 10)
    n1 = hp[1].num_values
    got_d, got_v = [], []
    with pytest.raises(pqgpu.PqgError):
        while True:
            v, d, _, _, _ = cr.read_batch(1000)
            assert len(d) == 1000  # only whole batches succeed: the one reaching the page fails
            got_d.append(d)
            got_v.append(v)
    d = np.concatenate(got_d)
    k = (n1 // 1000) * 1000
    assert len(d) == k
    np.testing.assert_array_equal(d, lv[:k])
    nv = int(np.count_nonzero(lv[:k]))
    assert np.concatenate(got_v).tobytes() == vals[:12 * nv].tobytes()
    cr.close()
    ctx.close()
    good.close()
    r.close()
