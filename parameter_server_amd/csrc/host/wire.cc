// The Task frame of the reference's wire (van.cc:122-191: [Task][key][value...],
// the Task serialised by protobuf) restricted to the fields the filter path
// reads and writes, in protobuf's proto2 wire format with the reference's field
// numbers (src/system/proto/task.proto:10-57, src/filter/proto/filter.proto:3-35,
// src/util/proto/range.proto, src/parameter/proto/param.proto):
//
//   Task:         request 2, key_range 7 {begin 1, end 2}, key_channel 8,
//                 has_key 9, filter 12, key_type 13, value_type 14, param 20 {push 1}
//   FilterConfig: type 1, signature 2, uncompressed_size 3, fixed_point 4
//                 {min_value 1, max_value 2}, num_bytes 5, mean 6, std 7,
//                 clear_cache_if_done 20
//
// Serialisation follows protobuf's C++ serializer: set fields only, in field
// number order, repeated scalars unpacked (proto2).  Parsing follows protobuf:
// any field order, packed or unpacked repeated scalars, unknown fields and
// unknown enum values skipped, proto defaults for absent fields (ParamCall.push
// defaults to true).  Fields outside the filter path (time, wait_time, msg,
// ctrl, sgd, ...) belong to the executor / van and are skipped -- after the
// whole frame has been checked the way protobuf's C++ ParseFromArray checks
// it: against the schema of Task and every message it reaches
// (wire_schema.h, generated from the reference's .proto files), nested
// messages parsed, packed repeats well formed, required fields present.
#include "wire.h"

#include <string.h>

#include <utility>
#include <vector>

#include "wire_schema.h"

namespace psf {
namespace {

void put_varint(std::string* o, uint64_t v) {
  while (v >= 0x80) {
    o->push_back((char)(v | 0x80));
    v >>= 7;
  }
  o->push_back((char)v);
}
void put_tag(std::string* o, int field, int wt) { put_varint(o, ((uint64_t)field << 3) | (uint64_t)wt); }
void put_int32(std::string* o, int field, int32_t v) {  // int32 / enum: sign-extended to 64 bits
  put_tag(o, field, 0);
  put_varint(o, (uint64_t)(int64_t)v);
}
void put_uint(std::string* o, int field, uint64_t v) {
  put_tag(o, field, 0);
  put_varint(o, v);
}
void put_float(std::string* o, int field, float v) {
  put_tag(o, field, 5);
  char b[4];
  memcpy(b, &v, 4);  // little endian
  o->append(b, 4);
}
void put_bytes(std::string* o, int field, const std::string& b) {
  put_tag(o, field, 2);
  put_varint(o, b.size());
  o->append(b);
}

std::string serialize_filter(const FilterConfig& f) {
  std::string o;
  put_int32(&o, 1, (int32_t)f.type);
  if (f.has_signature) put_uint(&o, 2, f.signature);
  for (uint64_t u : f.uncompressed_size) put_uint(&o, 3, u);
  for (const auto& fp0 : f.fixed_point) {
    auto& fp = const_cast<FixedFloatConfig&>(fp0);
    fp.settle();  // computed min/max a batched encode left on the device
    std::string m;
    if (fp.has_min) put_float(&m, 1, fp.min_value);
    if (fp.has_max) put_float(&m, 2, fp.max_value);
    put_bytes(&o, 4, m);
  }
  if (f.has_num_bytes) put_int32(&o, 5, f.num_bytes);
  if (f.has_mean) put_float(&o, 6, f.mean);
  if (f.has_std) put_float(&o, 7, f.std);
  if (f.has_clear_cache_if_done) put_uint(&o, 20, f.clear_cache_if_done ? 1 : 0);
  return o;
}

// ------------------------------------------------------------- parsing ----
struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  [[noreturn]] static void fail(const char* what) {
    throw CheckError(kErrCheck, std::string("CHECK(task.ParseFromArray): ") + what);
  }
  bool done() const { return p >= end; }
  uint64_t varint() {
    uint64_t v = 0;
    for (int i = 0; i < 10; ++i) {
      if (p >= end) fail("truncated varint");
      const uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7f) << (7 * i);  // bits past 64 are dropped, as protobuf does
      if (b < 0x80) return v;
    }
    fail("varint too long");
  }
  uint32_t fixed32() {
    if (end - p < 4) fail("truncated fixed32");
    uint32_t v;
    memcpy(&v, p, 4);
    p += 4;
    return v;
  }
  Reader sub() {
    const uint64_t n = varint();
    if ((uint64_t)(end - p) < n) fail("truncated length-delimited field");
    Reader r{p, p + n};
    p += n;
    return r;
  }
  // (field, wire type) of the next tag
  void tag(int* field, int* wt) {
    const uint64_t t = varint();
    *field = (int)(t >> 3);
    *wt = (int)(t & 7);
    if (*field == 0 || (t >> 3) > 0x1fffffff) fail("invalid field number");
  }
  void skip(int wt, int field = 0) {
    switch (wt) {
      case 0: varint(); break;
      case 3: {  // group: skip to its END_GROUP
        for (;;) {
          if (done()) fail("unterminated group");
          int f, w;
          tag(&f, &w);
          if (w == 4) {
            if (f != field) fail("mismatched end group");
            return;
          }
          skip(w, f);
        }
      }
      case 1:
        if (end - p < 8) fail("truncated fixed64");
        p += 8;
        break;
      case 2: sub(); break;
      case 5: fixed32(); break;
      default: fail("unsupported wire type");
    }
  }
};

float as_float(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}

// repeated scalar: unpacked (wt 0) or packed (wt 2)
template <typename F> void repeated_varint(Reader& r, int wt, F&& add) {
  if (wt == 0) {
    add(r.varint());
  } else if (wt == 2) {
    Reader s = r.sub();
    while (!s.done()) add(s.varint());
  } else {
    r.skip(wt);
  }
}

bool known_data_type(uint64_t v) { return v <= 11; }  // task.proto DataType OTHER..CHAR

void parse_fixed_point(Reader r, FixedFloatConfig* fp) {
  while (!r.done()) {
    int field, wt;
    r.tag(&field, &wt);
    if (field == 1 && wt == 5) fp->set_min(as_float(r.fixed32()));
    else if (field == 2 && wt == 5) fp->set_max(as_float(r.fixed32()));
    else r.skip(wt, field);
  }
}

void parse_filter(Reader r, FilterConfig* f) {
  bool has_type = false;
  while (!r.done()) {
    int field, wt;
    r.tag(&field, &wt);
    if (field == 1 && wt == 0) {
      const uint64_t v = r.varint();
      if (v >= 1 && v <= 4) {  // unknown enum values go to the unknown fields
        f->type = (FilterConfig::Type)v;
        has_type = true;
      }
    } else if (field == 2 && wt == 0) {
      f->signature = (uint32_t)r.varint();
      f->has_signature = true;
    } else if (field == 3 && (wt == 0 || wt == 2)) {
      repeated_varint(r, wt, [&](uint64_t v) { f->uncompressed_size.push_back(v); });
    } else if (field == 4 && wt == 2) {
      f->fixed_point.emplace_back();
      parse_fixed_point(r.sub(), &f->fixed_point.back());
    } else if (field == 5 && wt == 0) {
      f->num_bytes = (int32_t)r.varint();
      f->has_num_bytes = true;
    } else if (field == 6 && wt == 5) {
      f->mean = as_float(r.fixed32());
      f->has_mean = true;
    } else if (field == 7 && wt == 5) {
      f->std = as_float(r.fixed32());
      f->has_std = true;
    } else if (field == 20 && wt == 0) {
      f->clear_cache_if_done = r.varint() != 0;
      f->has_clear_cache_if_done = true;
    } else {
      r.skip(wt, field);
    }
  }
  if (!has_type) Reader::fail("FilterConfig.type missing");
}

// ---------------------------------------- ParseFromArray's verdict ----
namespace ws = wire_schema;

const ws::Field* schema_field(const ws::Message& m, uint32_t number) {
  for (int i = 0; i < m.nfields; ++i)
    if (m.fields[i].number == number) return &m.fields[i];
  return nullptr;
}

bool enum_value_known(int e, uint64_t v) {
  const ws::Enum& E = ws::kEnums[e];
  const int64_t x = (int64_t)v;  // enums are int32 on the wire, sign-extended
  for (int i = 0; i < E.n; ++i)
    if (E.values[i] == x) return true;
  return false;
}

// a known field in the wire type protobuf parses it from (a repeated scalar
// also packed); any other wire type makes it an unknown field
bool wire_type_matches(const ws::Field& f, int wt) {
  const bool packed = f.label == ws::kRepeated && wt == 2;
  switch (f.kind) {
    case ws::kVarint:
    case ws::kEnum: return wt == 0 || packed;
    case ws::kFixed32: return wt == 5 || packed;
    case ws::kFixed64: return wt == 1 || packed;
    default: return wt == 2;
  }
}

typedef std::vector<std::pair<const uint8_t*, const uint8_t*>> Parts;

// One message given as the byte ranges of its occurrences (a singular
// sub-message that occurs several times is merged, i.e. parsed as the
// concatenation); throws where parse + IsInitialized fails.
void check_message(const Parts& parts, int mi, int depth) {
  if (depth > 100) Reader::fail("nesting deeper than protobuf's recursion limit");
  const ws::Message& M = ws::kMessages[mi];
  std::vector<char> seen(M.nfields, 0);
  std::vector<Parts> singular(M.nfields);
  for (const auto& part : parts) {
    Reader r{part.first, part.second};
    while (!r.done()) {
      int field, wt;
      r.tag(&field, &wt);
      const ws::Field* f = schema_field(M, (uint32_t)field);
      if (!f || !wire_type_matches(*f, wt)) {
        r.skip(wt, field);
        continue;
      }
      const int idx = (int)(f - M.fields);
      if (f->kind == ws::kMessage) {
        Reader s = r.sub();
        if (f->label == ws::kRepeated)
          check_message(Parts{{s.p, s.end}}, f->sub, depth + 1);
        else
          singular[idx].push_back({s.p, s.end});
        seen[idx] = 1;
      } else if (wt == 2 && f->kind != ws::kBytes) {  // packed repeated scalars
        Reader s = r.sub();
        const size_t len = (size_t)(s.end - s.p);
        if (f->kind == ws::kFixed32 ? len % 4 : f->kind == ws::kFixed64 ? len % 8 : 0)
          Reader::fail("packed fixed-width field of ragged length");
        if (f->kind == ws::kVarint || f->kind == ws::kEnum)
          while (!s.done()) s.varint();
        seen[idx] = 1;
      } else if (f->kind == ws::kEnum) {
        if (enum_value_known(f->sub, r.varint())) seen[idx] = 1;  // else an unknown field
      } else {
        r.skip(wt, field);
        seen[idx] = 1;
      }
    }
  }
  for (int i = 0; i < M.nfields; ++i) {
    if (!singular[i].empty()) check_message(singular[i], M.fields[i].sub, depth + 1);
    if (M.fields[i].label == ws::kRequired && !seen[i]) Reader::fail("required field missing");
  }
}

}  // namespace

std::string serialize_task(const Task& t) {
  std::string o;
  put_uint(&o, 2, t.request ? 1 : 0);
  if (t.has_key_range) {
    std::string r;
    put_uint(&r, 1, t.key_range.begin);
    put_uint(&r, 2, t.key_range.end);
    put_bytes(&o, 7, r);
  }
  put_int32(&o, 8, t.key_channel);
  if (t.has_key) put_uint(&o, 9, 1);
  for (const auto& f : t.filter) put_bytes(&o, 12, serialize_filter(f));
  if (t.has_key_type) put_int32(&o, 13, t.key_type);
  for (int v : t.value_type) put_int32(&o, 14, v);
  if (t.has_param) {
    std::string pc;
    put_uint(&pc, 1, t.push ? 1 : 0);
    put_bytes(&o, 20, pc);
  }
  return o;
}

void parse_task(const uint8_t* p, size_t n, Task* t) {
  *t = Task();
  check_message(Parts{{p, p + n}}, ws::kTask, 0);
  Reader r{p, p + n};
  bool hb = false, he = false;  // PbRange required fields (merged over repeats)
  while (!r.done()) {
    int field, wt;
    r.tag(&field, &wt);
    if (field == 2 && wt == 0) {
      t->request = r.varint() != 0;
    } else if (field == 7 && wt == 2) {
      Reader s = r.sub();
      while (!s.done()) {
        int f, w;
        s.tag(&f, &w);
        if (f == 1 && w == 0) { t->key_range.begin = s.varint(); hb = true; }
        else if (f == 2 && w == 0) { t->key_range.end = s.varint(); he = true; }
        else s.skip(w, f);
      }
      t->has_key_range = true;
    } else if (field == 8 && wt == 0) {
      t->key_channel = (int32_t)r.varint();
    } else if (field == 9 && wt == 0) {
      t->has_key = r.varint() != 0;
    } else if (field == 12 && wt == 2) {
      t->filter.emplace_back();
      parse_filter(r.sub(), &t->filter.back());
    } else if (field == 13 && wt == 0) {
      const uint64_t v = r.varint();
      if (known_data_type(v)) { t->key_type = (int)v; t->has_key_type = true; }
    } else if (field == 14 && (wt == 0 || wt == 2)) {
      repeated_varint(r, wt, [&](uint64_t v) { if (known_data_type(v)) t->value_type.push_back((int)v); });
    } else if (field == 20 && wt == 2) {
      Reader s = r.sub();
      if (!t->has_param) t->push = true;  // ParamCall.push [default = true]
      t->has_param = true;
      while (!s.done()) {
        int f, w;
        s.tag(&f, &w);
        if (f == 1 && w == 0) t->push = s.varint() != 0;
        else s.skip(w, f);
      }
    } else {
      r.skip(wt, field);
    }
  }
  if (t->has_key_range && (!hb || !he)) Reader::fail("PbRange.begin/end missing");
}

}  // namespace psf
