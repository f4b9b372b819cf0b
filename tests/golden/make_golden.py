"""Generate golden column vectors for the reference's data files (tests/golden/data/*.parquet).

The data files are the reference's own test fixtures (/root/reference/data, copied verbatim).
The expected outputs are produced independently of this repo's decoder and of the reference
(Rust is not available here): pyarrow (Arrow C++'s Parquet reader) reads each file, and the
Dremel record shredding below turns its rows back into exactly what parquet-rs's
ColumnReaderImpl::read_batch returns per leaf column (column/reader.rs:159-265):

    def levels (i16), rep levels (i16), dense non-null values in the reference layout
    (INT32/FLOAT 4 B, INT64/DOUBLE 8 B, INT96 12 B, BOOLEAN 1 B, BYTE_ARRAY/FLBA bytes+lengths).

The shredding is itself pinned by the reference's triplet KATs (record/triplet.rs:362-439),
checked in tests/test_golden_files.py. Output: one .npz per file (no pickles) + manifest.json.

Run:  python tests/golden/make_golden.py
"""
import json
import os
import re
import struct
import sys

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

HERE = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(HERE, "data")
OUT = os.path.join(HERE, "vectors")

PTYPES = {"BOOLEAN": 0, "INT32": 1, "INT64": 2, "INT96": 3, "FLOAT": 4, "DOUBLE": 5,
          "BYTE_ARRAY": 6, "FIXED_LEN_BYTE_ARRAY": 7}

# Files whose pages the reference itself rejects; no golden values (tested as errors).
SKIP = {"nation.dict-malformed.parquet"}

# Arrow converts INT96 to int64 ns and cannot represent Julian day 0: 10k-v2's int96_field has a
# one-entry dictionary page of 12 zero bytes (see `xxd` of the chunk) that Arrow reports as 0 ns,
# which would invert to the Unix epoch. For these (file, column) pairs 0 ns maps to zero bytes.
INT96_ZERO = {("10k-v2.parquet", "int96_field")}


class Node:
    def __init__(self, rep, kind, name, ann):
        self.rep, self.kind, self.name, self.ann = rep, kind, name, ann
        self.children = []
        self.leaf_index = None


_LINE = re.compile(r"^\s*(required|optional|repeated)\s+(\S+)\s+field_id=\S+\s+([^\s;{(]+)"
                   r"(?:\s*\(([^)]*)\))?\s*([{;])")


def parse_schema(pf):
    """Schema tree with repetitions from ParquetSchema's text form."""
    lines = str(pf.schema).splitlines()[1:]
    root = None
    stack = []
    for ln in lines:
        if ln.strip() == "}":
            stack.pop()
            continue
        m = _LINE.match(ln)
        if not m:
            continue
        rep, kind, name, ann, tail = m.groups()
        n = Node(rep, kind, name, (ann or "").split("(")[0].strip())
        if root is None:
            root = n
        else:
            stack[-1].children.append(n)
        if tail == "{":
            stack.append(n)
    leaves = []

    def number(n):
        if not n.children:
            n.leaf_index = len(leaves)
            leaves.append(n)
        for c in n.children:
            number(c)

    for c in root.children:
        number(c)
    return root, leaves


def shred_row(root, row, leaves, out):
    """Dremel shredding of one record (dict of top-level values) into per-leaf triplets."""

    def emit_null(node, r, d):
        if not node.children:
            out[node.leaf_index].append((r, d, None))
            return
        for c in node.children:
            emit_null(c, r, d)

    def content(node, v, r, d, rlev, parent_ann):
        if not node.children:
            out[node.leaf_index].append((r, d, v))
            return
        if node.ann in ("List", "Map") and len(node.children) == 1 and node.children[0].rep == "repeated":
            shred(node.children[0], v, r, d, rlev, node.ann)
            return
        if node.rep == "repeated" and parent_ann == "List" and len(node.children) == 1:
            shred(node.children[0], v, r, d, rlev, None)
            return
        if node.rep == "repeated" and parent_ann == "Map":
            k, val = v
            shred(node.children[0], k, r, d, rlev, None)
            shred(node.children[1], val, r, d, rlev, None)
            return
        for c in node.children:
            shred(c, None if v is None else v.get(c.name), r, d, rlev, None)

    def shred(node, v, r, d, rlev, parent_ann):
        if node.rep == "repeated":
            if not v:
                emit_null(node, r, d)
                return
            for i, e in enumerate(v):
                content(node, e, r if i == 0 else rlev + 1, d + 1, rlev + 1, parent_ann)
        elif node.rep == "optional":
            if v is None:
                emit_null(node, r, d)
            else:
                content(node, v, r, d + 1, rlev, parent_ann)
        else:
            content(node, v, r, d, rlev, parent_ann)

    for c in root.children:
        shred(c, row.get(c.name), 0, 0, 0, None)


def encode_value(ptype, v, int96_zero=False):
    if ptype == 0:
        return b"\x01" if v else b"\x00"
    if ptype == 1:
        return struct.pack("<I", int(v) & 0xFFFFFFFF)
    if ptype == 2:
        return struct.pack("<Q", int(v) & 0xFFFFFFFFFFFFFFFF)
    if ptype == 3:  # INT96 from Arrow's ns timestamp: [nanos of day u64][julian day u32]
        ns = int(v)
        if int96_zero and ns == 0:
            return bytes(12)
        day, nod = divmod(ns, 86400 * 10**9)
        return struct.pack("<QI", nod, (day + 2440588) & 0xFFFFFFFF)
    if ptype == 4:
        return struct.pack("<f", v)
    if ptype == 5:
        return struct.pack("<d", v)
    return v.encode("utf-8") if isinstance(v, str) else bytes(v)


def storage_table(t):
    """Replace logical types with their stored integers (dates, timestamps)."""
    cols = []
    for name, col in zip(t.column_names, t.columns):
        ty = col.type
        if pa.types.is_timestamp(ty):
            col = col.cast(pa.int64())
        elif pa.types.is_date32(ty):
            col = col.cast(pa.int32())
        cols.append(col)
    return pa.table(cols, names=t.column_names)


def golden_for(path):
    pf = pq.ParquetFile(path)
    root, leaves = parse_schema(pf)
    md = pf.metadata
    assert len(leaves) == md.num_columns, (path, len(leaves), md.num_columns)
    arrays = {}
    cols = []
    for j in range(md.num_columns):
        sc = pf.schema.column(j)
        cols.append({"path": sc.path, "physical_type": PTYPES[sc.physical_type],
                     "type_length": sc.length or 0, "max_def": sc.max_definition_level,
                     "max_rep": sc.max_repetition_level})
    for rg in range(md.num_row_groups):
        rows = storage_table(pf.read_row_group(rg)).to_pylist()
        out = [[] for _ in leaves]
        for row in rows:
            shred_row(root, row, leaves, out)
        for j, trip in enumerate(out):
            ptype = cols[j]["physical_type"]
            md_, mr_ = cols[j]["max_def"], cols[j]["max_rep"]
            dense = [v for (r, d, v) in trip if d == md_]
            arrays[f"{j}_{rg}_def"] = np.array([d for (_, d, _) in trip], dtype=np.int16)
            arrays[f"{j}_{rg}_rep"] = np.array([r for (r, _, _) in trip], dtype=np.int16)
            z = (os.path.basename(path), cols[j]["path"]) in INT96_ZERO
            enc = [encode_value(ptype, v, z) for v in dense]
            arrays[f"{j}_{rg}_val"] = np.frombuffer(b"".join(enc), dtype=np.uint8).copy()
            if ptype in (6, 7):
                arrays[f"{j}_{rg}_len"] = np.array([len(e) for e in enc], dtype=np.uint32)
            assert mr_ > 0 or all(r == 0 for (r, _, _) in trip)
    meta = {"file": os.path.basename(path), "num_rows": md.num_rows,
            "row_groups": [md.row_group(i).num_rows for i in range(md.num_row_groups)],
            "columns": cols}
    return meta, arrays


def main():
    os.makedirs(OUT, exist_ok=True)
    manifest = []
    for f in sorted(os.listdir(DATA)):
        if not f.endswith(".parquet") or f in SKIP:
            continue
        meta, arrays = golden_for(os.path.join(DATA, f))
        np.savez_compressed(os.path.join(OUT, f.replace(".parquet", ".npz")), **arrays)
        manifest.append(meta)
        print(f, meta["num_rows"], len(meta["columns"]), file=sys.stderr)
    with open(os.path.join(OUT, "manifest.json"), "w") as fh:
        json.dump({"generator": "pyarrow " + pa.__version__, "files": manifest}, fh, indent=1)


if __name__ == "__main__":
    main()
