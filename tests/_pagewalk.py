"""Test helper: file positions of a column chunk's pages, from a minimal thrift compact-protocol
walk of the page headers (format of parquet.thrift's PageHeader: 1 type, 2 uncompressed size,
3 compressed size, 5.. the per-type headers; file/reader.rs:420-522 reads the same sequence).
Used to damage one page's header or payload in a written file."""


def _varint(b, i):
    v = s = 0
    while True:
        x = b[i]
        i += 1
        v |= (x & 0x7F) << s
        s += 7
        if not x & 0x80:
            return v, i


def _zz(v):
    return (v >> 1) ^ -(v & 1)


def _skip(b, i, t):
    if t in (1, 2):           # bool in the type nibble
        return i
    if t == 3:                # byte
        return i + 1
    if t in (4, 5, 6):        # i16 / i32 / i64: zigzag varint
        return _varint(b, i)[1]
    if t == 7:                # double
        return i + 8
    if t == 8:                # binary
        n, i = _varint(b, i)
        return i + n
    if t in (9, 10):          # list / set
        h = b[i]
        i += 1
        n, et = h >> 4, h & 15
        if n == 15:
            n, i = _varint(b, i)
        for _ in range(n):
            i = _skip(b, i, et)
        return i
    if t == 12:               # struct
        return _struct(b, i)[1]
    raise ValueError(f"thrift type {t}")


def _struct(b, i, want=()):
    fid, got = 0, {}
    while True:
        h = b[i]
        i += 1
        if h == 0:
            return got, i
        t, d = h & 15, h >> 4
        if d:
            fid += d
        else:
            v, i = _varint(b, i)
            fid = _zz(v)
        if fid in want and t in (5, 6):
            v, i = _varint(b, i)
            got[fid] = _zz(v)
        else:
            i = _skip(b, i, t)


def chunk_pages(data, start, nbytes):
    """[(header_pos, payload_pos, compressed_size, page_type)] of the pages in [start, start + nbytes)."""
    out, i, end = [], start, start + nbytes
    while i < end:
        got, j = _struct(data, i, want=(1, 3))
        out.append((i, j, got[3], got[1]))
        i = j + got[3]
    return out
