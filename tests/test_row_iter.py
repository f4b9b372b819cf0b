"""Record assembly into rows (pqg_row_iter_*, csrc/host/record_reader.cpp): RowIter / Reader tree
over the GPU-decoded leaf columns (record/reader.rs:38-717).

Expected rows: (1) the reference's own record-reader tests (reader.rs:774-1434), transcribed here
as data in the iterator's JSON form, for the reference data files they read; (2) pyarrow's rows of
every golden data file (tests/golden/data), field by field."""
import datetime
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DATA = os.path.join(os.path.dirname(__file__), "golden", "data")


@pytest.fixture(scope="module")
def ctx():
    import pqgpu
    c = pqgpu.Context(0)
    yield c
    c.close()


# ---- the iterator's JSON form of record/api.rs Field / Row
def Int(v): return {"Int": v}            # noqa: E302,E704
def Long(v): return {"Long": v}          # noqa: E302,E704
def Double(v): return {"Double": v}      # noqa: E302,E704
def Bool(v): return {"Bool": v}          # noqa: E302,E704
def Str(v): return {"Str": v}            # noqa: E302,E704
Null = None


def lst(*e): return {"List": list(e)}                          # noqa: E302,E704
def mp(*kv): return {"Map": [[k, v] for k, v in kv]}           # noqa: E302,E704
def grp(*f): return {"Group": [[n, v] for n, v in f]}          # noqa: E302,E704
def row(*f): return [[n, v] for n, v in f]                     # noqa: E302,E704


def rows_of(ctx, name, fields=None, row_group=-1, batch_size=1024):
    import pqgpu
    r = pqgpu.FileReader(os.path.join(DATA, name))
    it = pqgpu.RowIter(r, ctx, row_group=row_group, batch_size=batch_size, fields=fields)
    out = list(it)
    it.close()
    r.close()
    return out


def test_rows_nulls(ctx):  # reader.rs:774-812
    exp = [row(("b_struct", grp(("b_c_int", Null))))] * 8
    assert rows_of(ctx, "nulls.snappy.parquet") == exp


def test_rows_nonnullable(ctx):  # reader.rs:814-857
    exp = [row(
        ("ID", Long(8)),
        ("Int_Array", lst(Int(-1))),
        ("int_array_array", lst(lst(Int(-1), Int(-2)), lst())),
        ("Int_Map", mp((Str("k1"), Int(-1)))),
        ("int_map_array", lst(mp(), mp((Str("k1"), Int(1))), mp(), mp())),
        ("nested_Struct", grp(
            ("a", Int(-1)),
            ("B", lst(Int(-1))),
            ("c", grp(("D", lst(lst(grp(("e", Int(-1)), ("f", Str("nonnullable")))))))),
            ("G", mp()))))]
    assert rows_of(ctx, "nonnullable.impala.parquet") == exp


def _nullable_rows():
    """record/reader.rs:859-1141, one row at a time."""
    def E(e, f): return grp(("E", e), ("F", f))  # noqa: E704
    def H(i): return grp(("H", i))  # noqa: E704
    def I(v): return grp(("i", v))  # noqa: E704,E743
    r1 = row(("id", Long(1)),
             ("int_array", lst(Int(1), Int(2), Int(3))),
             ("int_array_Array", lst(lst(Int(1), Int(2)), lst(Int(3), Int(4)))),
             ("int_map", mp((Str("k1"), Int(1)), (Str("k2"), Int(100)))),
             ("int_Map_Array", lst(mp((Str("k1"), Int(1))))),
             ("nested_struct", grp(("A", Int(1)),
                                   ("b", lst(Int(1))),
                                   ("C", grp(("d", lst(lst(E(Int(10), Str("aaa")), E(Int(-10), Str("bbb"))),
                                                       lst(E(Int(11), Str("c"))))))),
                                   ("g", mp((Str("foo"), H(I(lst(Double(1.1))))))))))
    r2 = row(("id", Long(2)),
             ("int_array", lst(Null, Int(1), Int(2), Null, Int(3), Null)),
             ("int_array_Array", lst(lst(Null, Int(1), Int(2), Null), lst(Int(3), Null, Int(4)), lst(), Null)),
             ("int_map", mp((Str("k1"), Int(2)), (Str("k2"), Null))),
             ("int_Map_Array", lst(mp((Str("k3"), Null), (Str("k1"), Int(1))), Null, mp())),
             ("nested_struct", grp(("A", Null),
                                   ("b", lst(Null)),
                                   ("C", grp(("d", lst(lst(E(Null, Null), E(Int(10), Str("aaa")), E(Null, Null),
                                                           E(Int(-10), Str("bbb")), E(Null, Null)),
                                                       lst(E(Int(11), Str("c")), Null), lst(), Null)))),
                                   ("g", mp((Str("g1"), H(I(lst(Double(2.2), Null)))),
                                            (Str("g2"), H(I(lst()))),
                                            (Str("g3"), Null),
                                            (Str("g4"), H(I(Null))),
                                            (Str("g5"), grp(("H", Null))))))))
    r3 = row(("id", Long(3)), ("int_array", lst()), ("int_array_Array", lst(Null)), ("int_map", mp()),
             ("int_Map_Array", lst(Null, Null)),
             ("nested_struct", grp(("A", Null), ("b", Null), ("C", grp(("d", lst()))), ("g", mp()))))
    r4 = row(("id", Long(4)), ("int_array", Null), ("int_array_Array", lst()), ("int_map", mp()),
             ("int_Map_Array", lst()),
             ("nested_struct", grp(("A", Null), ("b", Null), ("C", grp(("d", Null))), ("g", Null))))
    r5 = row(("id", Long(5)), ("int_array", Null), ("int_array_Array", Null), ("int_map", mp()),
             ("int_Map_Array", Null),
             ("nested_struct", grp(("A", Null), ("b", Null), ("C", Null),
                                   ("g", mp((Str("foo"), H(I(lst(Double(2.2), Double(3.3))))))))))
    r6 = row(("id", Long(6)), ("int_array", Null), ("int_array_Array", Null), ("int_map", Null),
             ("int_Map_Array", Null), ("nested_struct", Null))
    r7 = row(("id", Long(7)), ("int_array", Null), ("int_array_Array", lst(Null, lst(Int(5), Int(6)))),
             ("int_map", mp((Str("k1"), Null), (Str("k3"), Null))), ("int_Map_Array", Null),
             ("nested_struct", grp(("A", Int(7)), ("b", lst(Int(2), Int(3), Null)),
                                   ("C", grp(("d", lst(lst(), lst(Null), Null)))), ("g", Null))))
    return [r1, r2, r3, r4, r5, r6, r7]


NULLABLE = _nullable_rows()


@pytest.mark.parametrize("batch_size", [1, 2, 3, 1024])
def test_rows_nullable(ctx, batch_size):  # reader.rs:859-1143
    assert rows_of(ctx, "nullable.impala.parquet", batch_size=batch_size) == NULLABLE


def test_rows_projection(ctx):  # reader.rs:1145-1182 (c, b of nested_maps, in that order)
    assert rows_of(ctx, "nested_maps.snappy.parquet", fields=["c", "b"]) == [row(("c", Double(1.0)), ("b", Int(1)))] * 6


def test_rows_projection_map(ctx):  # reader.rs:1184-1246
    exp = [row(("a", mp((Str("a"), mp((Int(1), Bool(True)), (Int(2), Bool(False))))))),
           row(("a", mp((Str("b"), mp((Int(1), Bool(True))))))),
           row(("a", mp((Str("c"), Null)))),
           row(("a", mp((Str("d"), mp())))),
           row(("a", mp((Str("e"), mp((Int(1), Bool(True))))))),
           row(("a", mp((Str("f"), mp((Int(3), Bool(True)), (Int(4), Bool(False)), (Int(5), Bool(True)))))))]
    assert rows_of(ctx, "nested_maps.snappy.parquet", fields=["a"]) == exp


def test_rows_projection_list(ctx):  # reader.rs:1248-1304
    a, b, c, d, e, f = (Str(x) for x in "abcdef")
    exp = [row(("a", lst(lst(lst(a, b), lst(c)), lst(Null, lst(d))))),
           row(("a", lst(lst(lst(a, b), lst(c, d)), lst(Null, lst(e))))),
           row(("a", lst(lst(lst(a, b), lst(c, d), lst(e)), lst(Null, lst(f)))))]
    assert rows_of(ctx, "nested_lists.snappy.parquet", fields=["a"]) == exp


def test_rows_invalid_projection(ctx):  # reader.rs:1306-1338
    import pqgpu
    with pytest.raises(pqgpu.PqgError, match="Root schema does not contain projection"):
        rows_of(ctx, "nested_maps.snappy.parquet", fields=["key", "value"])


def test_rows_repeated_no_annotation(ctx):  # reader.rs:1361-1434
    def ph(n, k): return grp(("number", Long(n)), ("kind", k))  # noqa: E704
    exp = [row(("id", Int(1)), ("phoneNumbers", Null)),
           row(("id", Int(2)), ("phoneNumbers", Null)),
           row(("id", Int(3)), ("phoneNumbers", grp(("phone", lst())))),
           row(("id", Int(4)), ("phoneNumbers", grp(("phone", lst(ph(5555555555, Null)))))),
           row(("id", Int(5)), ("phoneNumbers", grp(("phone", lst(ph(1111111111, Str("home"))))))),
           row(("id", Int(6)), ("phoneNumbers", grp(("phone", lst(ph(1111111111, Str("home")), ph(2222222222, Null),
                                                                  ph(3333333333, Str("mobile")))))))]
    assert rows_of(ctx, "repeated_no_annotation.parquet") == exp


def test_rows_row_group_and_file_agree(ctx):
    """RowIter::from_row_group over each row group, concatenated == RowIter::from_file."""
    import pqgpu
    for name in ("nullable.impala.parquet", "alltypes_plain.parquet", "nested_maps.snappy.parquet"):
        r = pqgpu.FileReader(os.path.join(DATA, name))
        n = r.num_row_groups
        r.close()
        per = sum((rows_of(ctx, name, row_group=g) for g in range(n)), [])
        assert per == rows_of(ctx, name), name


# ---- pyarrow's rows of every golden file
def _plain(v):
    """The iterator's JSON field as a plain Python value (pyarrow's to_pylist form)."""
    if v is None:
        return None
    (k, x), = v.items()
    if k in ("Group",):
        return {n: _plain(f) for n, f in x}
    if k == "List":
        return [_plain(e) for e in x]
    if k == "Map":
        return [(_plain(a), _plain(b)) for a, b in x]
    if k == "Bytes":
        return bytes(x)
    if k == "Float":  # (the f32's shortest text: back to the f32, then widened as pyarrow widens it)
        return float(np.float32(float(x)))
    if k == "Double":
        return float(x)
    return x


def _arrow(v, typ):
    import pyarrow as pa
    if v is None:
        return None
    if pa.types.is_timestamp(typ):
        epoch = datetime.datetime(1970, 1, 1, tzinfo=v.tzinfo)
        d = v - epoch
        return (d.days * 86400 + d.seconds) * 1000 + d.microseconds // 1000
    if pa.types.is_date32(typ):
        return (v - datetime.date(1970, 1, 1)).days
    if pa.types.is_struct(typ):
        return {typ.field(i).name: _arrow(v[typ.field(i).name], typ.field(i).type) for i in range(typ.num_fields)}
    if pa.types.is_map(typ):
        return [(_arrow(a, typ.key_type), _arrow(b, typ.item_type)) for a, b in v]
    if pa.types.is_list(typ) or pa.types.is_large_list(typ):
        return [_arrow(e, typ.value_type) for e in v]
    if pa.types.is_float32(typ):
        return float(np.float32(v))
    return v


@pytest.mark.parametrize("name", sorted(f for f in os.listdir(DATA) if f.endswith(".parquet")
                                        and f != "nation.dict-malformed.parquet"))
def test_rows_match_pyarrow(ctx, name):
    import pqgpu
    pq = pytest.importorskip("pyarrow.parquet")
    t = pq.read_table(os.path.join(DATA, name))
    if name == "10k-v2.parquet":
        # its INT96 column holds instants before 1970: Field::convert_int96 panics ("Expected
        # non-negative milliseconds", record/api.rs:505-510) on the first such row
        r = pqgpu.FileReader(os.path.join(DATA, name))
        it = pqgpu.RowIter(r, ctx)
        got = []
        with pytest.raises(pqgpu.PqgError, match="non-negative milliseconds") as ei:
            for row_ in it:
                got.append(row_)
        assert ei.value.status == pqgpu.PANIC
        it.close()
        r.close()
        raw = np.load(os.path.join(os.path.dirname(__file__), "golden", "vectors", "10k-v2.npz"))["7_0_val"]
        raw = raw.reshape(-1, 12)
        day = raw[:, 8:12].copy().view(np.uint32)[:, 0].astype(np.int64)
        nanos = raw[:, 0:8].copy().view(np.int64)[:, 0]
        millis = (day - 2440588) * 86400 * 1000 + nanos // 1000000
        first_neg = int(np.argmax(millis < 0)) if (millis < 0).any() else len(millis)
        assert len(got) == first_neg  # (all-zero INT96 values here: day 0, the very first row)
        t = t.slice(0, first_neg)
    else:
        got = rows_of(ctx, name)
    assert len(got) == t.num_rows
    cols = {f.name: (t.column(f.name).to_pylist(), f.type) for f in t.schema}
    for i, r in enumerate(got):
        assert [n for n, _ in r] == t.schema.names, name
        for n, v in r:
            exp = _arrow(cols[n][0][i], cols[n][1])
            g = _plain(v)
            if isinstance(exp, float) or isinstance(g, float):
                assert (exp != exp and g != g) or exp == g, (name, i, n, g, exp)
            else:
                assert g == exp, (name, i, n, g, exp)


def test_rows_display_text(ctx):
    """The Display rendering (record/api.rs:144-157, 557-616) of the reference's nonnullable row."""
    exp = ('{ID: 8, Int_Array: [-1], int_array_array: [[-1, -2], []], Int_Map: {"k1" -> -1}, '
           'int_map_array: [{}, {"k1" -> 1}, {}, {}], nested_Struct: {a: -1, B: [-1], c: {D: [[{e: -1, '
           'f: "nonnullable"}]]}, G: {}}}')
    import pqgpu
    r = pqgpu.FileReader(os.path.join(DATA, "nonnullable.impala.parquet"))
    it = pqgpu.RowIter(r, ctx, display=True)
    assert list(it) == [exp]
    it.close()
    r.close()


def test_rows_display_float_specials(ctx, tmp_path):
    """Display of FLOAT / DOUBLE fields outside the fixed-notation range (record/api.rs:570-583):
    {:E} above 1e19 and below 1e-15 (zero and negatives included), {:?} otherwise; a NaN fails
    both range tests and prints as Rust's {:?} does, "NaN"."""
    pa = pytest.importorskip("pyarrow")
    pq = pytest.importorskip("pyarrow.parquet")
    import pqgpu
    vals = [float("nan"), 1.5, 0.0, -2.0, float("inf"), 3e20]
    path = str(tmp_path / "floats.parquet")
    pq.write_table(pa.table({"f": pa.array(vals, pa.float32()), "d": pa.array(vals, pa.float64())}), path,
                   use_dictionary=False, compression="NONE")
    r = pqgpu.FileReader(path)
    it = pqgpu.RowIter(r, ctx, display=True)
    txt = ["NaN", "1.5", "0E0", "-2E0", "inf", "3E20"]
    assert list(it) == ["{f: %s, d: %s}" % (t, t) for t in txt]
    it.close()
    r.close()
