"""Python binding of the MI355X decode library (lib/libpqgpu.so) over its C ABI.

This mirrors the reference's column-reader interface for the decode path (column/reader.rs,
encodings/decoding.rs): a Column descriptor, a list of uncompressed Pages, and decode results
of (def levels, rep levels, dense values). PyTorch provides device memory and streams only.

The library must be built (`make -C parquet-rs_amd`); loading fails loudly otherwise. There
is no CPU fallback on this path.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# PQG_LIBDIR selects an experiment build (Makefile VARIANT=...) for A/B timing; default lib/
LIB_PATH = os.path.join(_HERE, os.environ.get("PQG_LIBDIR", "lib"), "libpqgpu.so")

OK, GENERAL, NYI, EOF, PANIC, HANG, CAPACITY, INVALID, HIP = range(9)
STATUS_NAMES = ["OK", "General", "NYI", "EOF", "Panic", "Hang", "Capacity", "Invalid", "HIP"]
BOOLEAN, INT32, INT64, INT96, FLOAT, DOUBLE, BYTE_ARRAY, FIXED_LEN_BYTE_ARRAY = range(8)
PLAIN, PLAIN_DICTIONARY, RLE, BIT_PACKED = 0, 2, 3, 4
DELTA_BINARY_PACKED, DELTA_LENGTH_BYTE_ARRAY, DELTA_BYTE_ARRAY, RLE_DICTIONARY = 5, 6, 7, 8
PAGE_DATA, PAGE_DICTIONARY, PAGE_DATA_V2 = 0, 2, 3
VALUE_SIZE = {BOOLEAN: 1, INT32: 4, INT64: 8, INT96: 12, FLOAT: 4, DOUBLE: 8}
NP_DTYPE = {BOOLEAN: np.uint8, INT32: np.int32, INT64: np.int64, FLOAT: np.float32,
            DOUBLE: np.float64}


class PqgError(RuntimeError):
    def __init__(self, status, message, page=-1):
        super().__init__(f"{STATUS_NAMES[status] if 0 <= status < 9 else status}: {message}"
                         + (f" (page {page})" if page >= 0 else ""))
        self.status, self.page = status, page


class Page(C.Structure):
    _fields_ = [("offset", C.c_uint64), ("nbytes", C.c_uint32), ("num_values", C.c_uint32),
                ("page_type", C.c_int32), ("encoding", C.c_int32), ("def_encoding", C.c_int32),
                ("rep_encoding", C.c_int32), ("def_len", C.c_uint32), ("rep_len", C.c_uint32)]


class Column(C.Structure):
    _fields_ = [("physical_type", C.c_int32), ("type_length", C.c_int32),
                ("max_def", C.c_int16), ("max_rep", C.c_int16)]


class Output(C.Structure):
    _fields_ = [("def_levels", C.c_void_p), ("rep_levels", C.c_void_p), ("values", C.c_void_p),
                ("values_capacity", C.c_uint64), ("offsets", C.c_void_p),
                ("offsets_capacity", C.c_uint64), ("num_levels", C.c_uint64),
                ("num_values", C.c_uint64), ("num_bytes", C.c_uint64)]


class Timings(C.Structure):
    _fields_ = [("prepare_ms", C.c_float), ("levels_ms", C.c_float), ("scan_ms", C.c_float),
                ("values_ms", C.c_float), ("total_ms", C.c_float), ("values_kernel", C.c_uint32),
                ("levels_kernel_ms", C.c_float), ("values_kernel_ms", C.c_float)]


class RgrOutput(C.Structure):
    _fields_ = [("def_levels", C.c_void_p), ("rep_levels", C.c_void_p), ("values", C.c_void_p),
                ("offsets", C.c_void_p), ("host_def_levels", C.c_void_p), ("host_rep_levels", C.c_void_p),
                ("host_values", C.c_void_p), ("host_offsets", C.c_void_p), ("num_levels", C.c_uint64),
                ("num_values", C.c_uint64), ("num_bytes", C.c_uint64)]


class RgrStats(C.Structure):
    _fields_ = [("row_groups", C.c_uint64), ("file_bytes", C.c_uint64), ("staged_bytes", C.c_uint64),
                ("output_bytes", C.c_uint64), ("host_ms", C.c_double), ("plan_ms", C.c_double),
                ("fill_ms", C.c_double), ("enqueue_ms", C.c_double), ("sync_ms", C.c_double),
                ("d2h_wait_ms", C.c_double)]


RGR_HOST_OUTPUT = 1

EXPORTS = [
    "pqg_ctx_create", "pqg_ctx_destroy", "pqg_ctx_set_timing", "pqg_ctx_set_overlap", "pqg_decode_chunk",
    "pqg_decode_chunks",
    "pqg_sync", "pqg_sync_detail",
    "pqg_get_timings", "pqg_reset_timings", "pqg_ctx_last_paths", "pqg_error_message", "pqg_file_open", "pqg_file_open_memory",
    "pqg_file_close", "pqg_file_error", "pqg_file_num_rows", "pqg_file_num_row_groups",
    "pqg_file_num_columns", "pqg_file_column", "pqg_row_group_num_rows", "pqg_chunk_pages",
    "pqg_chunk_blob", "pqg_column_reader_open", "pqg_column_reader_close",
    "pqg_column_reader_read_batch", "pqg_column_reader_read_batch_caps", "pqg_triplet_iter_open", "pqg_triplet_iter_close",
    "pqg_triplet_iter_read_next", "pqg_triplet_iter_has_next", "pqg_triplet_iter_def_level",
    "pqg_triplet_iter_rep_level", "pqg_triplet_iter_is_null", "pqg_triplet_iter_value",
    "pqg_space_values", "pqg_rg_ctx_create", "pqg_rg_ctx_destroy", "pqg_rg_decode", "pqg_rg_sync",
    "pqg_rg_sync_call", "pqg_rg_error_message", "pqg_rgr_open", "pqg_rgr_close", "pqg_rgr_submit",
    "pqg_rgr_wait", "pqg_rgr_column", "pqg_rgr_get_stats", "pqg_rgr_error", "pqg_row_iter_open",
    "pqg_row_iter_open_fields", "pqg_row_iter_close", "pqg_row_iter_next", "pqg_row_iter_error",
]

_lib = None


def lib():
    """Load lib/libpqgpu.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `make -C {_HERE}`")
        L = C.CDLL(LIB_PATH)
        vp, u64, i32 = C.c_void_p, C.c_uint64, C.c_int
        L.pqg_ctx_create.argtypes = [i32, C.POINTER(vp)]
        L.pqg_ctx_destroy.argtypes = [vp]
        L.pqg_ctx_set_timing.argtypes = [vp, i32]
        L.pqg_ctx_set_overlap.argtypes = [vp, i32]
        L.pqg_decode_chunk.argtypes = [vp, C.POINTER(Column), vp, u64, C.POINTER(Page), C.c_uint32,
                                       C.POINTER(Output), vp]
        L.pqg_decode_chunks.argtypes = [vp, C.c_uint32, C.POINTER(Column), vp, u64, C.POINTER(C.POINTER(Page)),
                                        C.POINTER(C.c_uint32), C.POINTER(Output), vp]
        L.pqg_sync.argtypes = [vp, C.POINTER(C.c_int)]
        L.pqg_sync_detail.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.pqg_get_timings.argtypes = [vp, C.POINTER(Timings)]
        L.pqg_reset_timings.argtypes = [vp]
        L.pqg_ctx_last_paths.argtypes = [vp, C.POINTER(C.c_uint32)]
        L.pqg_error_message.argtypes = [vp]
        L.pqg_error_message.restype = C.c_char_p
        L.pqg_file_open.argtypes = [C.c_char_p, C.POINTER(vp)]
        L.pqg_file_open_memory.argtypes = [vp, u64, C.POINTER(vp)]
        L.pqg_file_close.argtypes = [vp]
        L.pqg_file_close.restype = None
        L.pqg_file_error.argtypes = [vp]
        L.pqg_file_error.restype = C.c_char_p
        for name in ("pqg_file_num_rows",):
            getattr(L, name).argtypes = [vp]
            getattr(L, name).restype = C.c_int64
        L.pqg_file_num_row_groups.argtypes = [vp]
        L.pqg_file_num_columns.argtypes = [vp]
        L.pqg_file_column.argtypes = [vp, i32, C.POINTER(Column), C.c_char_p, C.c_size_t]
        L.pqg_row_group_num_rows.argtypes = [vp, i32]
        L.pqg_row_group_num_rows.restype = C.c_int64
        L.pqg_chunk_pages.argtypes = [vp, i32, i32, C.POINTER(Page), C.c_uint32]
        L.pqg_chunk_blob.argtypes = [vp, i32, i32, C.POINTER(vp), C.POINTER(u64)]
        L.pqg_column_reader_open.argtypes = [vp, i32, i32, vp, C.POINTER(vp)]
        L.pqg_column_reader_close.argtypes = [vp]
        L.pqg_column_reader_close.restype = None
        L.pqg_column_reader_read_batch.argtypes = [vp, C.c_size_t, vp, vp, vp, u64, vp,
                                                   C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]
        L.pqg_column_reader_read_batch_caps.argtypes = [vp, C.c_size_t, vp, C.c_size_t, vp, C.c_size_t, vp,
                                                        C.c_size_t, u64, vp, C.POINTER(C.c_size_t),
                                                        C.POINTER(C.c_size_t)]
        L.pqg_triplet_iter_open.argtypes = [vp, C.c_size_t, C.POINTER(vp)]
        L.pqg_triplet_iter_close.argtypes = [vp]
        L.pqg_triplet_iter_read_next.argtypes = [vp, C.POINTER(C.c_int)]
        for f in ("has_next", "is_null"):
            getattr(L, "pqg_triplet_iter_" + f).argtypes = [vp]
        for f in ("def_level", "rep_level"):
            getattr(L, "pqg_triplet_iter_" + f).argtypes = [vp]
            getattr(L, "pqg_triplet_iter_" + f).restype = C.c_int16
        L.pqg_triplet_iter_value.argtypes = [vp, vp, C.c_size_t, C.POINTER(C.c_size_t)]
        L.pqg_space_values.argtypes = [vp, vp, u64, C.c_int16, vp, i32, vp, vp]
        L.pqg_rg_ctx_create.argtypes = [i32, i32, C.POINTER(vp)]
        L.pqg_rg_ctx_destroy.argtypes = [vp]
        L.pqg_rg_decode.argtypes = [vp, C.c_uint32, C.POINTER(Column), vp, u64, C.POINTER(C.POINTER(Page)),
                                    C.POINTER(C.c_uint32), C.POINTER(Output), vp]
        L.pqg_rg_sync.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.pqg_rg_sync_call.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.pqg_rg_error_message.argtypes = [vp]
        L.pqg_rg_error_message.restype = C.c_char_p
        L.pqg_rgr_open.argtypes = [vp, i32, i32, i32, C.POINTER(vp)]
        L.pqg_rgr_close.argtypes = [vp]
        L.pqg_rgr_submit.argtypes = [vp, i32]
        L.pqg_rgr_wait.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.pqg_rgr_column.argtypes = [vp, i32, C.POINTER(RgrOutput)]
        L.pqg_rgr_get_stats.argtypes = [vp, C.POINTER(RgrStats)]
        L.pqg_rgr_error.argtypes = [vp]
        L.pqg_rgr_error.restype = C.c_char_p
        L.pqg_row_iter_open.argtypes = [vp, i32, vp, C.c_size_t, C.POINTER(vp)]
        L.pqg_row_iter_open_fields.argtypes = [vp, i32, vp, C.c_size_t, C.POINTER(C.c_char_p), C.c_uint32,
                                               C.POINTER(vp)]
        L.pqg_row_iter_close.argtypes = [vp]
        L.pqg_row_iter_close.restype = None
        L.pqg_row_iter_next.argtypes = [vp, i32, vp, C.c_size_t, C.POINTER(C.c_size_t), C.POINTER(C.c_int)]
        L.pqg_row_iter_error.argtypes = [vp]
        L.pqg_row_iter_error.restype = C.c_char_p
        _lib = L
    return _lib


def _torch():
    import torch
    return torch


class Context:
    """pqg_ctx: one per GPU (pqgpu.h)."""

    def __init__(self, device=0, timing=False):
        self.device = device
        h = C.c_void_p()
        st = lib().pqg_ctx_create(device, C.byref(h))
        if st:
            raise PqgError(st, "pqg_ctx_create failed")
        self.h = h
        if timing:
            lib().pqg_ctx_set_timing(self.h, 1)

    def close(self):
        if self.h:
            lib().pqg_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def error_message(self):
        return lib().pqg_error_message(self.h).decode(errors="replace")

    def set_timing(self, enabled):
        """HIP events around the decode stages (pqg_get_timings); call with no decode pending."""
        lib().pqg_ctx_set_timing(self.h, 1 if enabled else 0)

    def set_overlap(self, enabled):
        """Speculative PLAIN copy beside the level decode (pqg_ctx_set_overlap), a mode: 0 off (default),
        1 early fork (one workgroup per page on a side stream), 2 late fork (full grid); values above 2
        are taken as 2."""
        lib().pqg_ctx_set_overlap(self.h, int(enabled))

    def decode_async(self, column, blob, blob_len, pages, out, stream=0, npages=None):
        """Enqueue pqg_decode_chunk. `blob` is a device pointer (int), `pages` a ctypes Page
        array, `out` an Output struct with device pointers."""
        n = len(pages) if npages is None else npages
        st = lib().pqg_decode_chunk(self.h, C.byref(column), C.c_void_p(blob), blob_len, pages,
                                    n, C.byref(out), C.c_void_p(stream))
        if st:
            raise PqgError(st, self.error_message())

    def decode_chunks_async(self, columns, blob, blob_len, page_arrays, outs, stream=0):
        """Enqueue pqg_decode_chunks: a batch of column chunks (Column, ctypes Page array, Output
        per chunk), every page in the device blob at `blob`. Returns the Output array the
        library fills at sync (keep it alive until then)."""
        n = len(columns)
        cols = (Column * n)(*columns)
        pp = (C.POINTER(Page) * n)(*[C.cast(a, C.POINTER(Page)) for a in page_arrays])
        npg = (C.c_uint32 * n)(*[len(a) for a in page_arrays])
        oa = (Output * n)(*outs)
        st = lib().pqg_decode_chunks(self.h, n, cols, C.c_void_p(blob), blob_len, pp, npg, oa, C.c_void_p(stream))
        self._keep = getattr(self, "_keep", []) + [(cols, pp, npg, oa, page_arrays)]
        if st:
            raise PqgError(st, self.error_message())
        return oa

    def sync(self):
        bad = C.c_int(-1)
        st = lib().pqg_sync(self.h, C.byref(bad))
        self._keep = getattr(self, "_keep", [])[-2:]
        return st, bad.value

    def sync_detail(self):
        """(status, failing call since the last sync, its chunk, that chunk's page)."""
        call, chunk, page = C.c_int(-1), C.c_int(-1), C.c_int(-1)
        st = lib().pqg_sync_detail(self.h, C.byref(call), C.byref(chunk), C.byref(page))
        self._keep = getattr(self, "_keep", [])[-2:]
        return st, call.value, chunk.value, page.value

    def timings(self):
        t = Timings()
        lib().pqg_get_timings(self.h, C.byref(t))
        return t

    def last_paths(self):
        """PATH_* mask of the value-kernel families the last decode enqueued."""
        m = C.c_uint32(0)
        lib().pqg_ctx_last_paths(self.h, C.byref(m))
        return m.value


class RowGroupDecoder:
    """pqg_rg_ctx: the column chunks of a row group decoded together by one batched decode on the
    caller's stream (pqgpu.h, file/reader.rs:252-260). `nstreams` is reserved (1..16, ignored)."""

    def __init__(self, device=0, nstreams=1):
        self.device = device
        h = C.c_void_p()
        st = lib().pqg_rg_ctx_create(device, nstreams, C.byref(h))
        if st:
            raise PqgError(st, "pqg_rg_ctx_create failed")
        self.h = h
        self._keep = []  # argument arrays of the decodes not yet synced (the library fills oa)

    def close(self):
        if self.h:
            lib().pqg_rg_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def error_message(self):
        return lib().pqg_rg_error_message(self.h).decode(errors="replace")

    def decode_async(self, columns, blob, blob_len, page_arrays, outs, stream=0):
        """Enqueue pqg_rg_decode: columns[j] (Column), page_arrays[j] (ctypes Page array) and
        outs[j] (Output) per column chunk, every page in the device blob at `blob`."""
        n = len(columns)
        cols = (Column * n)(*columns)
        pp = (C.POINTER(Page) * n)(*[C.cast(a, C.POINTER(Page)) for a in page_arrays])
        npg = (C.c_uint32 * n)(*[len(a) for a in page_arrays])
        oa = (Output * n)(*outs)
        st = lib().pqg_rg_decode(self.h, n, cols, C.c_void_p(blob), blob_len, pp, npg, oa, C.c_void_p(stream))
        self._keep.append((cols, pp, npg, oa, page_arrays))
        if st:
            raise PqgError(st, self.error_message())
        return oa

    def sync(self):
        """(status, bad column, bad page); the Output array the last decode_async returned
        holds the counters."""
        col, page = C.c_int(-1), C.c_int(-1)
        st = lib().pqg_rg_sync(self.h, C.byref(col), C.byref(page))
        self._keep = self._keep[-1:]
        return st, col.value, page.value

    def sync_call(self):
        """(status, failing decode call since the last sync, bad column, bad page)."""
        call, col, page = C.c_int(-1), C.c_int(-1), C.c_int(-1)
        st = lib().pqg_rg_sync_call(self.h, C.byref(call), C.byref(col), C.byref(page))
        self._keep = self._keep[-1:]
        return st, call.value, col.value, page.value


# pqg_ctx_last_paths bits (pqgpu.h PQG_PATH_*)
PATH_PLAIN, PATH_DICT_LEVEL, PATH_DICT_WINDOW, PATH_DICT_TILES = 1, 2, 4, 8
PATH_BYTES, PATH_DELTA_BYTES, PATH_DELTA, PATH_RLE_BOOL = 16, 32, 64, 128


def make_pages(specs, misalign=0):
    """Pack page specs (objects with page_type, buf, num_values, encoding, def_encoding,
    rep_encoding, def_len, rep_len) into a host blob with 64-byte aligned payloads (at
    `misalign` bytes past a 64-byte boundary: the C ABI takes any payload offset)."""
    arr = (Page * max(len(specs), 1))()
    parts, off = [], 0
    for i, s in enumerate(specs):
        pad = (misalign - off) % 64
        if pad:
            parts.append(b"\0" * pad)
            off += pad
        arr[i] = Page(off, len(s.buf), s.num_values, s.page_type, s.encoding,
                      getattr(s, "def_encoding", RLE), getattr(s, "rep_encoding", RLE),
                      getattr(s, "def_len", 0), getattr(s, "rep_len", 0))
        parts.append(bytes(s.buf))
        off += len(s.buf)
    blob = b"".join(parts) + b"\0" * 64
    return blob, arr


def decode_column(ctx, ptype, specs, max_def=0, max_rep=0, type_length=-1, want_def=True,
                  want_rep=True, device=None, stream=None, values_capacity=None, misalign=0):
    """Decode one column chunk on the GPU; returns a dict with numpy def/rep/values.

    Equivalent to reading every batch of ColumnReaderImpl::read_batch (column/reader.rs
    :159-265) and concatenating: def/rep levels are the full level streams, values the
    dense non-null values (BYTE_ARRAY/FLBA: list of bytes, plus "offsets" and "bytes")."""
    torch = _torch()
    dev = device if device is not None else torch.device("cuda", ctx.device)
    blob, pages = make_pages(specs, misalign)
    d_blob = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
    nlev = sum(s.num_values for s in specs if s.page_type in (PAGE_DATA, PAGE_DATA_V2))
    ba = ptype in (BYTE_ARRAY, FIXED_LEN_BYTE_ARRAY)
    es = VALUE_SIZE.get(ptype, max(type_length, 1))
    if values_capacity is not None:
        cap_vals = values_capacity
    elif ba:
        cap_vals = max(len(blob), 64)
    else:
        cap_vals = max(nlev, 1) * es
    d_def = torch.empty(max(nlev, 1) + 8, dtype=torch.int16, device=dev) if (want_def and max_def > 0) else None
    d_rep = torch.empty(max(nlev, 1) + 8, dtype=torch.int16, device=dev) if (want_rep and max_rep > 0) else None
    d_off = torch.empty(nlev + 2, dtype=torch.int64, device=dev) if ba else None
    col = Column(ptype, type_length, max_def, max_rep)
    s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    for attempt in range(2):
        d_val = torch.empty(cap_vals + 64, dtype=torch.uint8, device=dev)
        out = Output(d_def.data_ptr() if d_def is not None else None,
                     d_rep.data_ptr() if d_rep is not None else None,
                     d_val.data_ptr(), cap_vals, d_off.data_ptr() if ba else None,
                     nlev + 1 if ba else 0, 0, 0, 0)
        ctx.decode_async(col, d_blob.data_ptr(), len(blob), pages, out, s, npages=len(specs))
        st, bad = ctx.sync()
        if st == CAPACITY and ba and attempt == 0 and values_capacity is None and out.num_bytes > cap_vals:
            cap_vals = int(out.num_bytes)
            continue
        break
    res = {"status": st, "page": bad, "message": ctx.error_message() if st else "",
           "num_levels": out.num_levels, "num_values": out.num_values, "num_bytes": out.num_bytes}
    nl, nv = out.num_levels, out.num_values
    res["def"] = d_def[:nl].cpu().numpy() if (d_def is not None and not st) else np.zeros(0, np.int16)
    res["rep"] = d_rep[:nl].cpu().numpy() if (d_rep is not None and not st) else np.zeros(0, np.int16)
    if st:
        res["values"] = np.zeros(0, np.uint8)
    elif ba:
        offs = d_off[: nv + 1].cpu().numpy()
        raw = d_val[: out.num_bytes].cpu().numpy().tobytes()
        res["offsets"], res["bytes"] = offs, raw
        res["values"] = [raw[offs[i]:offs[i + 1]] for i in range(nv)]
    else:
        raw = d_val[: nv * es].cpu().numpy()
        if ptype == INT96:
            res["values"] = raw.reshape(-1, 12)
        elif ptype in NP_DTYPE:
            res["values"] = raw.view(NP_DTYPE[ptype])
        else:
            res["values"] = raw
    return res


class FileReader:
    """SerializedFileReader over the host-side footer/page reader (file/reader.rs:140-330).
    Host-only: opening a file and listing pages needs no GPU."""

    def __init__(self, path=None, data=None):
        h = C.c_void_p()
        if data is not None:
            buf = (C.c_uint8 * len(data)).from_buffer_copy(data)
            st = lib().pqg_file_open_memory(buf, len(data), C.byref(h))
        else:
            st = lib().pqg_file_open(os.fsencode(path), C.byref(h))
        self.h = h
        if st:
            msg = lib().pqg_file_error(h).decode(errors="replace") if h else ""
            self.close()
            raise PqgError(st, msg)

    def close(self):
        if getattr(self, "h", None):
            lib().pqg_file_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def error(self):
        return lib().pqg_file_error(self.h).decode(errors="replace")

    @property
    def num_rows(self):
        return lib().pqg_file_num_rows(self.h)

    @property
    def num_row_groups(self):
        return lib().pqg_file_num_row_groups(self.h)

    @property
    def num_columns(self):
        return lib().pqg_file_num_columns(self.h)

    def row_group_num_rows(self, rg):
        return lib().pqg_row_group_num_rows(self.h, rg)

    def column(self, j):
        """(dot-joined path, Column descriptor) of leaf j."""
        col = Column()
        buf = C.create_string_buffer(1024)
        st = lib().pqg_file_column(self.h, j, C.byref(col), buf, 1024)
        if st:
            raise PqgError(st, "bad column index")
        return buf.value.decode(), col

    def chunk_pages(self, rg, j):
        """(host blob bytes, ctypes Page array) of one column chunk, uncompressed."""
        n = lib().pqg_chunk_pages(self.h, rg, j, None, 0)
        if n < 0:
            raise PqgError(-n, self.error())
        arr = (Page * max(n, 1))()
        lib().pqg_chunk_pages(self.h, rg, j, arr, n)
        p, ln = C.c_void_p(), C.c_uint64()
        st = lib().pqg_chunk_blob(self.h, rg, j, C.byref(p), C.byref(ln))
        if st:
            raise PqgError(st, self.error())
        return C.string_at(p, ln.value), arr, n

    def column_reader(self, rg, j, ctx):
        return ColumnReader(self, rg, j, ctx)


class RowGroupReader:
    """pqg_rgr_*: whole row groups from a FileReader to device memory (and, with host_output, to
    pinned host memory), pipelined: submit(g + 1) before wait() overlaps g + 1's page reading,
    decompression and H2D copy with g's decode (file/reader.rs:252-260, 306-330, 420-522)."""

    def __init__(self, reader, device=0, host_threads=8, host_output=True):
        self.reader = reader  # keeps the file open while the pqg_rgr lives
        self.h = C.c_void_p()
        st = lib().pqg_rgr_open(reader.h, device, host_threads, RGR_HOST_OUTPUT if host_output else 0,
                                C.byref(self.h))
        if st:
            raise PqgError(st, "pqg_rgr_open failed")
        self.host_output = host_output

    def close(self):
        if getattr(self, "h", None):
            lib().pqg_rgr_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def error(self):
        return lib().pqg_rgr_error(self.h).decode(errors="replace")

    def submit(self, rg):
        st = lib().pqg_rgr_submit(self.h, rg)
        if st:
            raise PqgError(st, self.error())

    def wait(self):
        """(status, row group, bad column, bad page) of the oldest row group in flight."""
        rg, col, page = C.c_int(), C.c_int(), C.c_int()
        st = lib().pqg_rgr_wait(self.h, C.byref(rg), C.byref(col), C.byref(page))
        if st == INVALID or st == HIP:
            raise PqgError(st, self.error())
        return st, rg.value, col.value, page.value

    def column(self, j):
        """(status, RgrOutput) of column j of the current (last waited) row group."""
        o = RgrOutput()
        st = lib().pqg_rgr_column(self.h, j, C.byref(o))
        return st, o

    def host_arrays(self, j, ptype):
        """Column j's host outputs as numpy arrays: {levels, values, offsets} (copies)."""
        import numpy as np
        st, o = self.column(j)
        res = {"status": st, "num_levels": o.num_levels, "num_values": o.num_values, "num_bytes": o.num_bytes}

        def arr(ptr, n, dt):
            if not ptr or n == 0:
                return np.zeros(0, dt)
            return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(np.ctypeslib.as_ctypes_type(dt))),
                                         shape=(n,)).copy()
        res["def_levels"] = arr(o.host_def_levels, o.num_levels, np.int16) if o.host_def_levels else None
        res["rep_levels"] = arr(o.host_rep_levels, o.num_levels, np.int16) if o.host_rep_levels else None
        if ptype in (BYTE_ARRAY, FIXED_LEN_BYTE_ARRAY):
            res["offsets"] = arr(o.host_offsets, o.num_values + 1, np.int64)
            res["values"] = arr(o.host_values, o.num_bytes, np.uint8)
        else:
            nb = o.num_values * VALUE_SIZE[ptype]
            res["values"] = arr(o.host_values, nb, np.uint8)
        return res

    def stats(self):
        s = RgrStats()
        lib().pqg_rgr_get_stats(self.h, C.byref(s))
        return {k: getattr(s, k) for k, _ in RgrStats._fields_}


class RowIter:
    """RowIter (record/reader.rs:588-717) over GPU-decoded column chunks: iterate to get rows as
    parsed JSON ([[name, field], ...], fields {"Kind": value} or None) or, with display=True, the
    reference's Display text."""

    def __init__(self, reader, ctx, row_group=-1, batch_size=1024, display=False, fields=None):
        self.reader = reader
        self.h = C.c_void_p()
        if fields is None:
            st = lib().pqg_row_iter_open(reader.h, row_group, ctx.h, batch_size, C.byref(self.h))
        else:
            arr = (C.c_char_p * max(len(fields), 1))(*[f.encode() for f in fields])
            st = lib().pqg_row_iter_open_fields(reader.h, row_group, ctx.h, batch_size, arr, len(fields),
                                                C.byref(self.h))
        if st:
            raise PqgError(st, reader.error() if fields is not None else "pqg_row_iter_open")
        self.fmt = 0 if display else 1
        self.buf = C.create_string_buffer(1 << 16)

    def close(self):
        if getattr(self, "h", None):
            lib().pqg_row_iter_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __iter__(self):
        return self

    def __next__(self):
        import json
        n, has = C.c_size_t(), C.c_int()
        st = lib().pqg_row_iter_next(self.h, self.fmt, self.buf, len(self.buf), C.byref(n), C.byref(has))
        if st == CAPACITY:
            self.buf = C.create_string_buffer(n.value + 1)
            st = lib().pqg_row_iter_next(self.h, self.fmt, self.buf, len(self.buf), C.byref(n), C.byref(has))
        if st:
            raise PqgError(st, lib().pqg_row_iter_error(self.h).decode(errors="replace"))
        if not has.value:
            raise StopIteration
        text = self.buf.raw[:n.value].decode("utf-8", errors="surrogateescape")
        return text if self.fmt == 0 else json.loads(text)


class ColumnReader:
    """ColumnReaderImpl::read_batch over a chunk decoded on the GPU (column/reader.rs:159-265)."""

    def __init__(self, fr, rg, j, ctx):
        self.fr = fr
        self.path, self.col = fr.column(j)
        h = C.c_void_p()
        st = lib().pqg_column_reader_open(fr.h, rg, j, ctx.h, C.byref(h))
        if st:
            raise PqgError(st, fr.error())
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            lib().pqg_column_reader_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def read_batch(self, batch_size, want_def=True, want_rep=True, def_cap=None, rep_cap=None,
                   values_cap=None):
        """Returns (values, def, rep, values_read, levels_read). For BYTE_ARRAY/FLBA values
        is a list of bytes objects; otherwise a numpy array in the reference layout. The caps are
        the lengths of the reference's def / rep / values slices (default batch_size each,
        column/reader.rs:170-205); want_def / want_rep False pass None for that slice."""
        t = self.col.physical_type
        es = VALUE_SIZE.get(t, 0)
        ba = t in (BYTE_ARRAY, FIXED_LEN_BYTE_ARRAY)
        dcap = batch_size if def_cap is None else def_cap
        rcap = batch_size if rep_cap is None else rep_cap
        vcap = batch_size if values_cap is None else values_cap
        d = np.zeros(max(dcap, 1), np.int16) if want_def else None
        r = np.zeros(max(rcap, 1), np.int16) if want_rep else None
        cap = vcap * es if not ba else 1 << 16
        while True:
            vals = np.zeros(max(cap, 1), np.uint8)
            lens = np.zeros(max(vcap, 1), np.uint32) if ba else None
            vr, lr = C.c_size_t(), C.c_size_t()
            st = lib().pqg_column_reader_read_batch_caps(
                self.h, batch_size, d.ctypes.data if d is not None else None, dcap,
                r.ctypes.data if r is not None else None, rcap, vals.ctypes.data, vcap, cap,
                lens.ctypes.data if lens is not None else None, C.byref(vr), C.byref(lr))
            if st == CAPACITY and ba:
                cap *= 4
                continue
            break
        if st:
            raise PqgError(st, self.fr.error())
        nv, nl = vr.value, lr.value
        if ba:
            out, o = [], 0
            for k in range(nv):
                out.append(bytes(vals[o:o + lens[k]]))
                o += int(lens[k])
            values = out
        else:
            raw = vals[: nv * es]
            values = raw.reshape(-1, 12) if t == INT96 else raw.view(NP_DTYPE[t])
        return (values, d[:nl] if d is not None and self.col.max_def > 0 else None,
                r[:nl] if r is not None and self.col.max_rep > 0 else None, nv, nl)


class TripletIter:
    """TypedTripletIter (record/triplet.rs:168-330) over a ColumnReader: read_next() advances one
    (definition level, repetition level, value) triplet; values are spaced onto the levels whose
    def == max_def. current_value() raises (the reference asserts) on a null slot."""

    def __init__(self, reader, batch_size=1024):
        self.reader = reader  # kept alive: the iterator reads through it
        self.col = reader.col
        h = C.c_void_p()
        st = lib().pqg_triplet_iter_open(reader.h, batch_size, C.byref(h))
        if st:
            raise PqgError(st, "pqg_triplet_iter_open failed")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            lib().pqg_triplet_iter_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def read_next(self):
        hn = C.c_int(0)
        st = lib().pqg_triplet_iter_read_next(self.h, C.byref(hn))
        if st:
            raise PqgError(st, self.reader.fr.error())
        return bool(hn.value)

    def has_next(self):
        return bool(lib().pqg_triplet_iter_has_next(self.h))

    def current_def_level(self):
        return int(lib().pqg_triplet_iter_def_level(self.h))

    def current_rep_level(self):
        return int(lib().pqg_triplet_iter_rep_level(self.h))

    def is_null(self):
        return bool(lib().pqg_triplet_iter_is_null(self.h))

    def current_value(self):
        """bytes for BYTE_ARRAY/FLBA, else the value in the reference's numpy layout."""
        n = C.c_size_t(0)
        buf = np.zeros(16, np.uint8)
        st = lib().pqg_triplet_iter_value(self.h, buf.ctypes.data, buf.nbytes, C.byref(n))
        if st == CAPACITY:
            buf = np.zeros(n.value, np.uint8)
            st = lib().pqg_triplet_iter_value(self.h, buf.ctypes.data, buf.nbytes, C.byref(n))
        if st:
            raise PqgError(st, "current_value on a triplet below the max definition level")
        raw = buf[: n.value]
        t = self.col.physical_type
        if t in (BYTE_ARRAY, FIXED_LEN_BYTE_ARRAY):
            return raw.tobytes()
        if t == INT96:
            return raw.copy()
        return raw.view(NP_DTYPE[t])[0]
