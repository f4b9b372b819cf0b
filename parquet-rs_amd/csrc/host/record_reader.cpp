// record_reader.cpp — pqg_row_iter_*: record assembly into rows (RowIter / ReaderIter /
// TreeBuilder / Reader, record/reader.rs:38-717) over the GPU column readers' triplet iterators
// (pqg_triplet_iter_*, TypedTripletIter, record/triplet.rs:168-330).
//
// The reader tree is built from the file schema exactly as TreeBuilder::reader_tree builds it
// (reader.rs:99-299): optional fields wrapped in an option reader, LIST groups (3-level and the
// legacy 2-level forms of Reader::is_element_type, :334-376) and MAP / MAP_KEY_VALUE groups as
// repeated / key-value readers, other repeated groups as required lists of required groups, plain
// groups as group readers, leaves as primitive readers over the leaf column's triplet iterator.
// Reading a row walks the tree with the reference's rules (Reader::read / read_field /
// advance_columns, :382-567), and leaf values convert by the column's physical and converted
// type (Field::convert_*, record/api.rs:449-555). Rows are rendered as the reference's Display
// text (api.rs:144-157, 557-666; dates and timestamps in UTC) or as typed JSON.
#include <stdio.h>
#include <string.h>
#include <time.h>

#include <charconv>
#include <memory>
#include <string>
#include <vector>

#include "file_reader.hpp"

using namespace pqg;

namespace {

// ConvertedType (parquet.thrift; basic.rs:49-129 LogicalType)
enum {
  CV_NONE = -1, CV_UTF8 = 0, CV_MAP = 1, CV_MAP_KEY_VALUE = 2, CV_LIST = 3, CV_ENUM = 4, CV_DECIMAL = 5,
  CV_DATE = 6, CV_TIMESTAMP_MILLIS = 9, CV_UINT_8 = 11, CV_UINT_16 = 12, CV_UINT_32 = 13, CV_UINT_64 = 14,
  CV_INT_8 = 15, CV_INT_16 = 16, CV_INT_32 = 17, CV_INT_64 = 18, CV_JSON = 19, CV_BSON = 20
};
enum { REP_REQUIRED = 0, REP_OPTIONAL = 1, REP_REPEATED = 2 };

// Field (record/api.rs:364-410)
struct Field {
  enum Kind {
    Null, Bool, Byte, Short, Int, Long, UByte, UShort, UInt, ULong, Float, Double, Decimal, Str, Bytes, Date,
    Timestamp, Group, List, Map
  } kind = Null;
  int64_t i = 0;     // signed integers, Bool
  uint64_t u = 0;    // unsigned integers, Date, Timestamp
  double d = 0;      // Float, Double
  std::string s;     // Str, Bytes, Decimal (its text)
  std::vector<std::pair<std::string, Field>> group;
  std::vector<Field> list;
  std::vector<std::pair<Field, Field>> map;
};

struct Leaf {  // a primitive reader's column
  pqg_column_reader* cr = nullptr;
  pqg_triplet_iter* it = nullptr;
  int ptype = 0, tl = 0, conv = CV_NONE, scale = 0, precision = 0;
  int16_t max_def = 0;
  std::vector<uint8_t> buf;
  ~Leaf() {
    pqg_triplet_iter_close(it);
    pqg_column_reader_close(cr);
  }
};

// Reader (reader.rs:303-317)
struct Node {
  enum Kind { Primitive, Option, Group, Repeated, KeyValue } kind;
  std::string name;        // field name (empty for the message)
  int repetition = REP_REQUIRED;
  int16_t def = 0, rep = 0;
  std::vector<std::unique_ptr<Node>> ch;  // Option/Repeated: [0]; Group: fields; KeyValue: keys, values
  std::unique_ptr<Leaf> leaf;
};

struct Err {
  int st;
  std::string msg;
};

bool is_element_type(const std::vector<SchemaNode>& sc, size_t i) {  // reader.rs:334-376
  const SchemaNode& n = sc[i];
  const bool prim = n.num_children <= 0 && n.type >= 0;
  const std::string& nm = n.name;
  return prim || (!prim && n.num_children > 1) || nm == "array" ||
         (nm.size() >= 6 && nm.compare(nm.size() - 6, 6, "_tuple") == 0);
}

// Children of schema node i (pre-order, num_children each).
std::vector<size_t> children(const std::vector<SchemaNode>& sc, size_t i) {
  std::vector<size_t> out;
  size_t j = i + 1;
  std::vector<size_t> stack;  // subtree sizes by walking
  for (int c = 0; c < sc[i].num_children; ++c) {
    out.push_back(j);
    // skip the subtree of j
    size_t need = 1;
    while (need) {
      need += (size_t)(sc[j].num_children > 0 ? sc[j].num_children : 0);
      --need;
      ++j;
    }
  }
  return out;
}

// Leaf column index of every schema node that is a leaf (pre-order).
std::vector<int> leaf_index(const std::vector<SchemaNode>& sc) {
  std::vector<int> idx(sc.size(), -1);
  int k = 0;
  for (size_t i = 1; i < sc.size(); ++i)
    if (sc[i].num_children <= 0 && sc[i].type >= 0) idx[i] = k++;
  return idx;
}

struct Builder {
  pqg_file_reader* r;
  int rg;
  pqg_ctx* ctx;
  size_t batch;
  const std::vector<SchemaNode>& sc;
  std::vector<int> lidx;

  std::unique_ptr<Node> leaf_reader(size_t i, const std::string& name, int repetition) {
    const SchemaNode& n = sc[i];
    auto node = std::make_unique<Node>();
    node->kind = Node::Primitive;
    node->name = name;
    node->repetition = repetition;
    auto lf = std::make_unique<Leaf>();
    const int col = lidx[i];
    if (col < 0) throw Err{PQG_ERR_GENERAL, "schema leaf without a column"};
    pqg_column c{};
    if (pqg_file_column(r, col, &c, nullptr, 0)) throw Err{PQG_ERR_GENERAL, "bad column"};
    lf->ptype = c.physical_type;
    lf->tl = c.type_length;
    lf->max_def = c.max_def;
    lf->conv = n.converted_type;
    lf->scale = n.scale;
    lf->precision = n.precision;
    int st = pqg_column_reader_open(r, rg, col, ctx, &lf->cr);
    if (st) throw Err{st, std::string("column ") + std::to_string(col) + ": " + pqg_file_error(r)};
    st = pqg_triplet_iter_open(lf->cr, batch, &lf->it);
    if (st) throw Err{st, "triplet iterator"};
    node->leaf = std::move(lf);
    return node;
  }

  // TreeBuilder::reader_tree (reader.rs:99-299); `as_required`: the node read as a REQUIRED group
  // (the required_field the reference builds for a repeated group outside LIST / MAP)
  std::unique_ptr<Node> tree(size_t i, int16_t def, int16_t rep, bool as_required = false) {
    const SchemaNode& f = sc[i];
    const int repetition = as_required ? REP_REQUIRED : f.repetition;
    if (repetition == REP_OPTIONAL) def += 1;
    else if (repetition == REP_REPEATED) {
      def += 1;
      rep += 1;
    }
    std::unique_ptr<Node> reader;
    const bool prim = f.num_children <= 0 && f.type >= 0;
    if (prim) {
      reader = leaf_reader(i, f.name, repetition);
    } else if (!as_required && f.converted_type == CV_LIST) {
      const std::vector<size_t> ch = children(sc, i);
      if (ch.size() != 1 || sc[ch[0]].repetition != REP_REPEATED)
        throw Err{PQG_ERR_PANIC, "Invalid list type " + f.name};
      reader = std::make_unique<Node>();
      reader->kind = Node::Repeated;
      reader->name = f.name;
      reader->repetition = repetition;
      reader->def = def;
      reader->rep = rep;
      if (is_element_type(sc, ch[0])) {
        reader->ch.push_back(tree(ch[0], def, rep));
      } else {
        const std::vector<size_t> gc = children(sc, ch[0]);
        if (gc.empty()) throw Err{PQG_ERR_PANIC, "Invalid list type " + f.name};
        reader->ch.push_back(tree(gc[0], def + 1, rep + 1));
      }
    } else if (!as_required && (f.converted_type == CV_MAP || f.converted_type == CV_MAP_KEY_VALUE)) {
      const std::vector<size_t> ch = children(sc, i);
      if (ch.size() != 1 || (sc[ch[0]].num_children <= 0 && sc[ch[0]].type >= 0))
        throw Err{PQG_ERR_PANIC, "Invalid map type: " + f.name};
      const size_t kv = ch[0];
      if (sc[kv].repetition != REP_REPEATED) throw Err{PQG_ERR_PANIC, "Invalid map type: " + f.name};
      const std::vector<size_t> kvc = children(sc, kv);
      if (kvc.size() != 2) throw Err{PQG_ERR_PANIC, "Invalid map type: " + f.name};
      if (!(sc[kvc[0]].num_children <= 0 && sc[kvc[0]].type >= 0))
        throw Err{PQG_ERR_PANIC, "Map key type is expected to be a primitive type"};
      reader = std::make_unique<Node>();
      reader->kind = Node::KeyValue;
      reader->name = f.name;
      reader->repetition = repetition;
      reader->def = def;
      reader->rep = rep;
      reader->ch.push_back(tree(kvc[0], def + 1, rep + 1));
      reader->ch.push_back(tree(kvc[1], def + 1, rep + 1));
    } else if (repetition == REP_REPEATED) {
      // a required list of required elements whose type is the field's (reader.rs:249-277)
      auto inner = tree(i, def, rep, true);
      reader = std::make_unique<Node>();
      reader->kind = Node::Repeated;
      reader->name = f.name;
      reader->repetition = repetition;
      reader->def = (int16_t)(def - 1);
      reader->rep = (int16_t)(rep - 1);
      reader->ch.push_back(std::move(inner));
    } else {
      reader = std::make_unique<Node>();
      reader->kind = Node::Group;
      reader->name = f.name;
      reader->repetition = repetition;
      reader->def = def;
      for (size_t c : children(sc, i)) reader->ch.push_back(tree(c, def, rep));
    }
    if (repetition == REP_OPTIONAL) {  // Reader::option (reader.rs:321-327)
      auto opt = std::make_unique<Node>();
      opt->kind = Node::Option;
      opt->name = reader->name;
      opt->repetition = repetition;
      opt->def = (int16_t)(def - 1);
      opt->ch.push_back(std::move(reader));
      return opt;
    }
    return reader;
  }
};

int16_t cur_def(const Node& n) {
  switch (n.kind) {
    case Node::Primitive: return pqg_triplet_iter_def_level(n.leaf->it);
    case Node::Group:
      if (n.ch.empty()) throw Err{PQG_ERR_PANIC, "Current definition level: empty group reader"};
      return cur_def(*n.ch[0]);
    default: return cur_def(*n.ch[0]);
  }
}

int16_t cur_rep(const Node& n) {
  switch (n.kind) {
    case Node::Primitive: return pqg_triplet_iter_rep_level(n.leaf->it);
    case Node::Group:
      if (n.ch.empty()) throw Err{PQG_ERR_PANIC, "Current repetition level: empty group reader"};
      return cur_rep(*n.ch[0]);
    default: return cur_rep(*n.ch[0]);
  }
}

bool has_next(const Node& n) {
  if (n.kind == Node::Primitive) return pqg_triplet_iter_has_next(n.leaf->it) != 0;
  return has_next(*n.ch[0]);
}

void advance(Node& n) {  // Reader::advance_columns (reader.rs:545-566)
  if (n.kind == Node::Primitive) {
    int hn = 0;
    const int st = pqg_triplet_iter_read_next(n.leaf->it, &hn);
    if (st) throw Err{st, "column read failed"};
    return;
  }
  for (auto& c : n.ch) advance(*c);
}

std::string decimal_text(const uint8_t* be, size_t n, int scale) {  // api.rs:641-666
  // two's complement big-endian -> sign + magnitude digits
  const bool neg = n && (be[0] & 0x80);
  std::vector<uint8_t> mag(be, be + n);
  if (neg) {  // negate
    for (auto& b : mag) b = (uint8_t)~b;
    for (size_t k = mag.size(); k-- > 0;)
      if (++mag[k] != 0) break;
  }
  std::string digits;
  bool zero = true;
  for (uint8_t b : mag) zero &= b == 0;
  if (zero) digits = "0";
  while (!zero) {  // repeated division by 10
    uint32_t rem = 0;
    zero = true;
    for (auto& b : mag) {
      const uint32_t cur = (rem << 8) | b;
      b = (uint8_t)(cur / 10);
      rem = cur % 10;
      zero &= b == 0;
    }
    digits.insert(digits.begin(), (char)('0' + rem));
  }
  std::string s = (neg ? "-" : "") + digits;
  const int negative = neg ? 1 : 0;
  int point = (int)s.size() - scale - negative;
  if (point <= 0) {
    while (point < 0) {
      s.insert((size_t)negative, "0");
      point += 1;
    }
    s.insert((size_t)negative, "0.");
  } else {
    s.insert((size_t)(point + negative), ".");
  }
  return s;
}

Field value(Leaf& lf) {  // TripletIter::current_value + Field::convert_* (api.rs:449-555)
  if (pqg_triplet_iter_is_null(lf.it)) throw Err{PQG_ERR_PANIC, "Value is null"};
  size_t len = 0;
  if (lf.buf.size() < 16) lf.buf.resize(16);
  int st = pqg_triplet_iter_value(lf.it, lf.buf.data(), lf.buf.size(), &len);
  if (st == PQG_ERR_CAPACITY) {
    lf.buf.resize(len);
    st = pqg_triplet_iter_value(lf.it, lf.buf.data(), lf.buf.size(), &len);
  }
  if (st) throw Err{st, "value"};
  const uint8_t* p = lf.buf.data();
  Field f;
  auto nyi = [&]() { throw Err{PQG_ERR_NYI, "conversion of this logical type is not implemented"}; };
  switch (lf.ptype) {
    case PQG_BOOLEAN:
      f.kind = Field::Bool;
      f.i = p[0] != 0;
      break;
    case PQG_INT32: {
      int32_t v;
      memcpy(&v, p, 4);
      switch (lf.conv) {
        case CV_INT_8: f.kind = Field::Byte; f.i = (int8_t)v; break;
        case CV_INT_16: f.kind = Field::Short; f.i = (int16_t)v; break;
        case CV_INT_32: case CV_NONE: f.kind = Field::Int; f.i = v; break;
        case CV_UINT_8: f.kind = Field::UByte; f.u = (uint8_t)v; break;
        case CV_UINT_16: f.kind = Field::UShort; f.u = (uint16_t)v; break;
        case CV_UINT_32: f.kind = Field::UInt; f.u = (uint32_t)v; break;
        case CV_DATE: f.kind = Field::Date; f.u = (uint32_t)v; break;
        case CV_DECIMAL: {
          const uint8_t be[4] = {(uint8_t)(v >> 24), (uint8_t)(v >> 16), (uint8_t)(v >> 8), (uint8_t)v};
          f.kind = Field::Decimal;
          f.s = decimal_text(be, 4, lf.scale);
          break;
        }
        default: nyi();
      }
      break;
    }
    case PQG_INT64: {
      int64_t v;
      memcpy(&v, p, 8);
      switch (lf.conv) {
        case CV_INT_64: case CV_NONE: f.kind = Field::Long; f.i = v; break;
        case CV_UINT_64: f.kind = Field::ULong; f.u = (uint64_t)v; break;
        case CV_TIMESTAMP_MILLIS: f.kind = Field::Timestamp; f.u = (uint64_t)v; break;
        case CV_DECIMAL: {
          uint8_t be[8];
          for (int k = 0; k < 8; ++k) be[k] = (uint8_t)((uint64_t)v >> (56 - 8 * k));
          f.kind = Field::Decimal;
          f.s = decimal_text(be, 8, lf.scale);
          break;
        }
        default: nyi();
      }
      break;
    }
    case PQG_INT96: {  // api.rs:492-513
      uint32_t w[3];
      memcpy(w, p, 12);
      const int64_t day = (int64_t)w[2];
      const int64_t nanos = ((int64_t)w[1] << 32) + (int64_t)w[0];
      const int64_t millis = (day - 2440588) * 86400 * 1000 + nanos / 1000000;
      if (millis < 0) throw Err{PQG_ERR_PANIC, "Expected non-negative milliseconds when converting Int96"};
      f.kind = Field::Timestamp;
      f.u = (uint64_t)millis;
      break;
    }
    case PQG_FLOAT: {
      float v;
      memcpy(&v, p, 4);
      f.kind = Field::Float;
      f.d = v;
      break;
    }
    case PQG_DOUBLE: {
      double v;
      memcpy(&v, p, 8);
      f.kind = Field::Double;
      f.d = v;
      break;
    }
    case PQG_BYTE_ARRAY:
      if (lf.conv == CV_UTF8 || lf.conv == CV_ENUM || lf.conv == CV_JSON) f.kind = Field::Str;
      else if (lf.conv == CV_BSON || lf.conv == CV_NONE) f.kind = Field::Bytes;
      else if (lf.conv == CV_DECIMAL) {
        f.kind = Field::Decimal;
        f.s = decimal_text(p, len, lf.scale);
        break;
      } else nyi();
      f.s.assign((const char*)p, len);
      break;
    case PQG_FIXED_LEN_BYTE_ARRAY:
      if (lf.conv == CV_DECIMAL) {
        f.kind = Field::Decimal;
        f.s = decimal_text(p, len, lf.scale);
      } else if (lf.conv == CV_NONE) {
        f.kind = Field::Bytes;
        f.s.assign((const char*)p, len);
      } else nyi();
      break;
    default: nyi();
  }
  return f;
}

Field read_field(Node& n) {  // Reader::read_field (reader.rs:397-472)
  switch (n.kind) {
    case Node::Primitive: {
      Field v = value(*n.leaf);
      advance(n);
      return v;
    }
    case Node::Option: {
      if (cur_def(*n.ch[0]) > n.def) return read_field(*n.ch[0]);
      advance(*n.ch[0]);
      return Field{};
    }
    case Node::Group: {
      Field g;
      g.kind = Field::Group;
      for (auto& c : n.ch) {
        if (c->repetition != REP_OPTIONAL || cur_def(*c) > n.def) {
          g.group.emplace_back(c->name, read_field(*c));
        } else {
          advance(*c);
          g.group.emplace_back(c->name, Field{});
        }
      }
      return g;
    }
    case Node::Repeated: {
      Field l;
      l.kind = Field::List;
      Node& r = *n.ch[0];
      for (;;) {
        if (cur_def(r) > n.def) {
          l.list.push_back(read_field(r));
        } else {
          advance(r);
          break;
        }
        if (!has_next(r) || cur_rep(r) <= n.rep) break;
      }
      return l;
    }
    case Node::KeyValue: {
      Field m;
      m.kind = Field::Map;
      Node& k = *n.ch[0];
      Node& v = *n.ch[1];
      for (;;) {
        if (cur_def(k) > n.def) {
          Field kf = read_field(k);
          Field vf = read_field(v);
          m.map.emplace_back(std::move(kf), std::move(vf));
        } else {
          advance(k);
          advance(v);
          break;
        }
        if (!has_next(k) || cur_rep(k) <= n.rep) break;
      }
      return m;
    }
  }
  return Field{};
}

// ---------------------------------------------------------------- rendering
std::string fmt_float(double v, bool is_f32) {  // api.rs:570-583: {:E} outside [1e-15, 1e19], else {:?}
  char b[64];
  if (v != v) return "NaN";  // both range tests fail: {:?} prints any NaN as "NaN"
  if (v > 1e19 || v < 1e-15) {
    auto res = is_f32 ? std::to_chars(b, b + sizeof(b), (float)v, std::chars_format::scientific)
                      : std::to_chars(b, b + sizeof(b), v, std::chars_format::scientific);
    std::string t(b, res.ptr);
    const size_t e = t.find('e');
    if (e == std::string::npos) return t;  // inf / nan
    std::string mant = t.substr(0, e), ex = t.substr(e + 1);
    const bool eneg = !ex.empty() && ex[0] == '-';
    size_t k = (!ex.empty() && (ex[0] == '-' || ex[0] == '+')) ? 1 : 0;
    while (k + 1 < ex.size() && ex[k] == '0') ++k;
    return mant + "E" + (eneg ? "-" : "") + ex.substr(k);
  }
  auto res = is_f32 ? std::to_chars(b, b + sizeof(b), (float)v, std::chars_format::fixed)
                    : std::to_chars(b, b + sizeof(b), v, std::chars_format::fixed);
  std::string t(b, res.ptr);
  if (t.find('.') == std::string::npos) t += ".0";
  return t;
}

std::string utc_date(uint64_t secs, bool with_time) {
  const time_t t = (time_t)secs;
  struct tm tmv;
  gmtime_r(&t, &tmv);
  char b[64];
  strftime(b, sizeof(b), with_time ? "%Y-%m-%d %H:%M:%S +00:00" : "%Y-%m-%d +00:00", &tmv);
  return b;
}

void display(const Field& f, std::string& o);

void display_row(const std::vector<std::pair<std::string, Field>>& fields, std::string& o) {
  o += "{";
  for (size_t k = 0; k < fields.size(); ++k) {
    o += fields[k].first;
    o += ": ";
    display(fields[k].second, o);
    if (k + 1 < fields.size()) o += ", ";
  }
  o += "}";
}

void display(const Field& f, std::string& o) {  // impl Display for Field (api.rs:557-616)
  switch (f.kind) {
    case Field::Null: o += "null"; break;
    case Field::Bool: o += f.i ? "true" : "false"; break;
    case Field::Byte: case Field::Short: case Field::Int: case Field::Long: o += std::to_string(f.i); break;
    case Field::UByte: case Field::UShort: case Field::UInt: case Field::ULong: o += std::to_string(f.u); break;
    case Field::Float: o += fmt_float(f.d, true); break;
    case Field::Double: o += fmt_float(f.d, false); break;
    case Field::Decimal: o += f.s; break;
    case Field::Str: o += "\"" + f.s + "\""; break;
    case Field::Bytes: {
      o += "[";
      for (size_t k = 0; k < f.s.size(); ++k) {
        o += std::to_string((uint8_t)f.s[k]);
        if (k + 1 < f.s.size()) o += ", ";
      }
      o += "]";
      break;
    }
    case Field::Date: o += utc_date((uint64_t)f.u * 86400ull, false); break;
    case Field::Timestamp: o += utc_date(f.u / 1000, true); break;
    case Field::Group: display_row(f.group, o); break;
    case Field::List:
      o += "[";
      for (size_t k = 0; k < f.list.size(); ++k) {
        display(f.list[k], o);
        if (k + 1 < f.list.size()) o += ", ";
      }
      o += "]";
      break;
    case Field::Map:
      o += "{";
      for (size_t k = 0; k < f.map.size(); ++k) {
        display(f.map[k].first, o);
        o += " -> ";
        display(f.map[k].second, o);
        if (k + 1 < f.map.size()) o += ", ";
      }
      o += "}";
      break;
  }
}

void json_str(const std::string& s, std::string& o) {
  o += '"';
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') {
      o += '\\';
      o += (char)c;
    } else if (c < 0x20 || c >= 0x7F) {
      char b[8];
      snprintf(b, sizeof(b), "\\u%04x", c);
      o += b;
    } else {
      o += (char)c;
    }
  }
  o += '"';
}

void json(const Field& f, std::string& o);

void json_fields(const std::vector<std::pair<std::string, Field>>& fields, std::string& o) {
  o += "[";
  for (size_t k = 0; k < fields.size(); ++k) {
    o += "[";
    json_str(fields[k].first, o);
    o += ", ";
    json(fields[k].second, o);
    o += "]";
    if (k + 1 < fields.size()) o += ", ";
  }
  o += "]";
}

void json(const Field& f, std::string& o) {  // {"Kind": value}, null for Field::Null
  static const char* names[] = {"Null", "Bool",   "Byte",  "Short",  "Int",     "Long", "UByte",
                                "UShort", "UInt", "ULong", "Float",  "Double",  "Decimal", "Str",
                                "Bytes",  "Date", "Timestamp", "Group", "List", "Map"};
  if (f.kind == Field::Null) {
    o += "null";
    return;
  }
  o += "{\"";
  o += names[f.kind];
  o += "\": ";
  switch (f.kind) {
    case Field::Bool: o += f.i ? "true" : "false"; break;
    case Field::Byte: case Field::Short: case Field::Int: case Field::Long: o += std::to_string(f.i); break;
    case Field::UByte: case Field::UShort: case Field::UInt: case Field::ULong: case Field::Date:
    case Field::Timestamp: o += std::to_string(f.u); break;
    case Field::Float: case Field::Double: {
      if (f.d != f.d || f.d == 1.0 / 0.0 || f.d == -1.0 / 0.0) {
        o += f.d != f.d ? "\"nan\"" : f.d > 0 ? "\"inf\"" : "\"-inf\"";
      } else {
        char b[64];
        auto res = f.kind == Field::Float ? std::to_chars(b, b + sizeof(b), (float)f.d)
                                          : std::to_chars(b, b + sizeof(b), f.d);
        o.append(b, res.ptr);
      }
      break;
    }
    case Field::Decimal: case Field::Str: json_str(f.s, o); break;
    case Field::Bytes: {
      o += "[";
      for (size_t k = 0; k < f.s.size(); ++k) {
        o += std::to_string((uint8_t)f.s[k]);
        if (k + 1 < f.s.size()) o += ", ";
      }
      o += "]";
      break;
    }
    case Field::Group: json_fields(f.group, o); break;
    case Field::List:
      o += "[";
      for (size_t k = 0; k < f.list.size(); ++k) {
        json(f.list[k], o);
        if (k + 1 < f.list.size()) o += ", ";
      }
      o += "]";
      break;
    case Field::Map:
      o += "[";
      for (size_t k = 0; k < f.map.size(); ++k) {
        o += "[";
        json(f.map[k].first, o);
        o += ", ";
        json(f.map[k].second, o);
        o += "]";
        if (k + 1 < f.map.size()) o += ", ";
      }
      o += "]";
      break;
    default: break;
  }
  o += "}";
}

}  // namespace

// RowIter (reader.rs:588-687): the row groups in turn (one, or all of the file), each a
// ReaderIter (:690-717) over a freshly built reader tree.
struct pqg_row_iter {
  pqg_file_reader* r = nullptr;
  pqg_ctx* ctx = nullptr;
  size_t batch = 1024;
  int rg_next = 0, rg_end = 0;  // row groups still to open
  std::vector<size_t> top;      // the message's fields read (schema nodes), in projection order
  std::unique_ptr<Node> root;   // the current row group's tree (message: a group reader)
  int64_t left = 0;             // records left in it
  std::string pending;          // a rendered row the caller's buffer was too small for
  bool has_pending = false;
  int pending_format = 0;
  std::string err;
};

static int rowit_open_group(pqg_row_iter* it) {
  pqg_file_reader* r = it->r;
  const std::vector<SchemaNode>& sc = r->meta.schema;
  if (sc.empty()) return PQG_ERR_GENERAL;
  const int rg = it->rg_next++;
  Builder b{r, rg, it->ctx, it->batch, sc, leaf_index(sc)};
  auto root = std::make_unique<Node>();  // TreeBuilder::build (reader.rs:58-85)
  root->kind = Node::Group;
  root->def = 0;
  for (size_t c : it->top) root->ch.push_back(b.tree(c, 0, 0));
  advance(*root);  // ReaderIter::new (reader.rs:696-703)
  it->root = std::move(root);
  it->left = r->meta.row_groups[rg].num_rows;
  return PQG_OK;
}

extern "C" {

int pqg_row_iter_open_fields(pqg_file_reader* r, int row_group, pqg_ctx* ctx, size_t batch_size,
                             const char* const* fields, uint32_t nfields, pqg_row_iter** out) {
  if (!r || !ctx || !out || batch_size == 0 || (nfields && !fields)) return PQG_ERR_INVALID;
  *out = nullptr;
  const int nrg = (int)r->meta.row_groups.size();
  if (row_group >= nrg || row_group < -1 || r->meta.schema.empty()) return PQG_ERR_INVALID;
  auto it = std::make_unique<pqg_row_iter>();
  const std::vector<size_t> all = children(r->meta.schema, 0);
  if (!fields) {
    it->top = all;
  } else {  // RowIter::get_proj_descr (reader.rs:640-656), by top-level field name
    for (uint32_t k = 0; k < nfields; ++k) {
      size_t hit = (size_t)-1;
      for (size_t c : all)
        if (fields[k] && r->meta.schema[c].name == fields[k]) hit = c;
      if (hit == (size_t)-1) {
        r->err = "Root schema does not contain projection";
        return PQG_ERR_GENERAL;
      }
      it->top.push_back(hit);
    }
  }
  it->r = r;
  it->ctx = ctx;
  it->batch = batch_size;
  it->rg_next = row_group < 0 ? 0 : row_group;
  it->rg_end = row_group < 0 ? nrg : row_group + 1;
  *out = it.release();
  return PQG_OK;
}

int pqg_row_iter_open(pqg_file_reader* r, int row_group, pqg_ctx* ctx, size_t batch_size, pqg_row_iter** out) {
  return pqg_row_iter_open_fields(r, row_group, ctx, batch_size, nullptr, 0, out);
}

void pqg_row_iter_close(pqg_row_iter* it) { delete it; }

const char* pqg_row_iter_error(pqg_row_iter* it) { return it ? it->err.c_str() : "null iterator"; }

int pqg_row_iter_next(pqg_row_iter* it, int format, char* buf, size_t cap, size_t* len, int* has_row) {
  if (!it || !len || !has_row || (format != 0 && format != 1)) return PQG_ERR_INVALID;
  *has_row = 0;
  *len = 0;
  if (!it->has_pending) {
    try {
      while (it->left == 0) {  // RowIter::next: the next row group with rows (reader.rs:662-686)
        it->root.reset();
        if (it->rg_next >= it->rg_end) return PQG_OK;
        const int st = rowit_open_group(it);
        if (st) return st;
      }
      it->left--;
      std::vector<std::pair<std::string, Field>> fields;  // Reader::read (reader.rs:382-393)
      for (auto& c : it->root->ch) fields.emplace_back(c->name, read_field(*c));
      it->pending.clear();
      if (format == 0) display_row(fields, it->pending);
      else json_fields(fields, it->pending);
      it->has_pending = true;
      it->pending_format = format;
    } catch (const Err& e) {
      it->err = e.msg;
      it->root.reset();
      it->left = 0;
      it->rg_next = it->rg_end;  // the reference panics / unwraps an Err here: the iteration ends
      return e.st;
    }
  }
  if (it->pending_format != format) return PQG_ERR_INVALID;
  *len = it->pending.size();
  if (!buf || cap < it->pending.size() + 1) return PQG_ERR_CAPACITY;  // kept for the next call
  memcpy(buf, it->pending.data(), it->pending.size());
  buf[it->pending.size()] = 0;
  it->has_pending = false;
  *has_row = 1;
  return PQG_OK;
}

}  // extern "C"
