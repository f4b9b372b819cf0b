"""Test helper: a one-column parquet file (uncompressed) holding exactly the given pages, so that
hand-built pages can be read through the host file reader and the GPU column reader
(pqg_file_open_memory + pqg_column_reader_*). Layout as SerializedFileWriter writes it
(file/writer.rs): "PAR1", per page a thrift-compact PageHeader + payload, the thrift-compact
FileMetaData, its length, "PAR1". Test infrastructure only."""
import struct


class _Tw:
    """Thrift compact protocol writer (field deltas, zigzag varints, list headers)."""

    def __init__(self):
        self.b = bytearray()
        self.last = [0]

    def varint(self, v):
        while v >= 0x80:
            self.b.append((v & 0x7F) | 0x80)
            v >>= 7
        self.b.append(v)

    def zz(self, v):
        self.varint(((v << 1) ^ (v >> 63)) & ((1 << 64) - 1))

    def field(self, fid, t):
        d = fid - self.last[-1]
        if 0 < d <= 15:
            self.b.append((d << 4) | t)
        else:
            self.b.append(t)
            self.zz(fid)
        self.last[-1] = fid

    def i32(self, fid, v):
        self.field(fid, 5)
        self.zz(v)

    def i64(self, fid, v):
        self.field(fid, 6)
        self.zz(v)

    def boolean(self, fid, v):
        self.field(fid, 1 if v else 2)

    def string(self, fid, s):
        self.field(fid, 8)
        s = s.encode()
        self.varint(len(s))
        self.b += s

    def lst(self, fid, elem, n):
        self.field(fid, 9)
        if n < 15:
            self.b.append((n << 4) | elem)
        else:
            self.b.append(0xF0 | elem)
            self.varint(n)

    def begin(self):
        self.last.append(0)

    def end(self):
        self.b.append(0)
        self.last.pop()

    def struct(self, fid):
        self.field(fid, 12)
        self.begin()


PAGE_DATA, PAGE_DICTIONARY, PAGE_DATA_V2 = 0, 2, 3


def one_column_file(ptype, pages, optional=True, type_length=-1, name="c"):
    """pages: objects with page_type, buf, num_values, encoding, def_encoding, rep_encoding,
    def_len, rep_len (the oracle's PageSpec). Returns the file bytes."""
    out = bytearray(b"PAR1")
    start = len(out)
    data_off, dict_off, rows, encs = -1, -1, 0, []
    for p in pages:
        w = _Tw()
        w.i32(1, p.page_type)
        w.i32(2, len(p.buf))
        w.i32(3, len(p.buf))
        if p.page_type == PAGE_DICTIONARY:
            w.struct(7)
            w.i32(1, p.num_values)
            w.i32(2, p.encoding)
            w.end()
            dict_off = len(out)
        elif p.page_type == PAGE_DATA_V2:
            w.struct(8)
            w.i32(1, p.num_values)
            w.i32(2, 0)
            w.i32(3, p.num_values)
            w.i32(4, p.encoding)
            w.i32(5, p.def_len)
            w.i32(6, p.rep_len)
            w.boolean(7, False)
            w.end()
            if data_off < 0:
                data_off = len(out)
            rows += p.num_values
        else:
            w.struct(5)
            w.i32(1, p.num_values)
            w.i32(2, p.encoding)
            w.i32(3, p.def_encoding)
            w.i32(4, p.rep_encoding)
            w.end()
            if data_off < 0:
                data_off = len(out)
            rows += p.num_values
        w.b.append(0)
        if p.encoding not in encs:
            encs.append(p.encoding)
        out += w.b + bytes(p.buf)
    size = len(out) - start
    if data_off < 0:
        data_off = len(out)
    w = _Tw()  # FileMetaData
    w.i32(1, 1)
    w.lst(2, 12, 2)
    w.begin()
    w.string(4, "schema")
    w.i32(5, 1)
    w.end()
    w.begin()
    w.i32(1, ptype)
    if type_length > 0:
        w.i32(2, type_length)
    w.i32(3, 1 if optional else 0)
    w.string(4, name)
    w.end()
    w.i64(3, rows)
    w.lst(4, 12, 1)
    w.begin()  # RowGroup
    w.lst(1, 12, 1)
    w.begin()  # ColumnChunk
    w.i64(2, start)
    w.struct(3)  # ColumnMetaData
    w.i32(1, ptype)
    w.lst(2, 5, len(encs))
    for e in encs:
        w.zz(e)
    w.lst(3, 8, 1)
    w.varint(len(name))
    w.b += name.encode()
    w.i32(4, 0)
    w.i64(5, rows)
    w.i64(6, size)
    w.i64(7, size)
    w.i64(9, data_off)
    if dict_off >= 0:
        w.i64(11, dict_off)
    w.end()
    w.end()
    w.i64(2, size)
    w.i64(3, rows)
    w.end()
    w.string(6, "tests one-column writer")
    w.b.append(0)
    out += w.b + struct.pack("<I", len(w.b)) + b"PAR1"
    return bytes(out)
