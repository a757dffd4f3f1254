// Minimal JSON DOM for the native apiserver: value-semantics tree, strict parser,
// compact serializer (shortest round-trip doubles), deep equality that ignores
// object key order.  Kubernetes objects are small (KiB), so objects are vectors of
// members with linear lookup — faster than hashing at these sizes and order-preserving.
#pragma once

#include <charconv>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

namespace kj {

enum class T : uint8_t { Null, Bool, Int, Double, String, Array, Object };

struct Member;

struct Value {
  T t = T::Null;
  bool b = false;
  int64_t i = 0;
  double d = 0;
  std::string s;
  std::vector<Value> arr;
  std::vector<Member> obj;

  Value() = default;
  static Value null() { return Value(); }
  static Value boolean(bool v) { Value x; x.t = T::Bool; x.b = v; return x; }
  static Value integer(int64_t v) { Value x; x.t = T::Int; x.i = v; return x; }
  static Value number(double v) { Value x; x.t = T::Double; x.d = v; return x; }
  static Value str(std::string v) { Value x; x.t = T::String; x.s = std::move(v); return x; }
  static Value array() { Value x; x.t = T::Array; return x; }
  static Value object() { Value x; x.t = T::Object; return x; }

  bool is_null() const { return t == T::Null; }
  bool is_obj() const { return t == T::Object; }
  bool is_arr() const { return t == T::Array; }
  bool is_str() const { return t == T::String; }

  // object access
  const Value* get(std::string_view k) const;
  Value* get(std::string_view k);
  Value& operator[](std::string_view k);  // insert null if absent (turns null into object)
  bool erase(std::string_view k);
  std::string str_or(std::string_view k, const std::string& dflt = "") const {
    const Value* v = get(k);
    return v && v->t == T::String ? v->s : dflt;
  }
  const Value* path(std::initializer_list<std::string_view> ks) const {
    const Value* cur = this;
    for (auto k : ks) {
      if (!cur || cur->t != T::Object) return nullptr;
      cur = cur->get(k);
    }
    return cur;
  }
};

struct Member {
  std::string k;
  Value v;
};

inline const Value* Value::get(std::string_view k) const {
  if (t != T::Object) return nullptr;
  for (auto& m : obj)
    if (m.k == k) return &m.v;
  return nullptr;
}
inline Value* Value::get(std::string_view k) {
  if (t != T::Object) return nullptr;
  for (auto& m : obj)
    if (m.k == k) return &m.v;
  return nullptr;
}
inline Value& Value::operator[](std::string_view k) {
  if (t != T::Object) {
    *this = Value::object();
  }
  for (auto& m : obj)
    if (m.k == k) return m.v;
  obj.push_back(Member{std::string(k), Value()});
  return obj.back().v;
}
inline bool Value::erase(std::string_view k) {
  if (t != T::Object) return false;
  for (size_t n = 0; n < obj.size(); ++n)
    if (obj[n].k == k) {
      obj.erase(obj.begin() + n);
      return true;
    }
  return false;
}

bool operator==(const Value& a, const Value& b);
inline bool operator!=(const Value& a, const Value& b) { return !(a == b); }

inline bool operator==(const Value& a, const Value& b) {
  if (a.t != b.t) {
    if ((a.t == T::Int && b.t == T::Double)) return (double)a.i == b.d;
    if ((a.t == T::Double && b.t == T::Int)) return a.d == (double)b.i;
    return false;
  }
  switch (a.t) {
    case T::Null: return true;
    case T::Bool: return a.b == b.b;
    case T::Int: return a.i == b.i;
    case T::Double: return a.d == b.d;
    case T::String: return a.s == b.s;
    case T::Array:
      if (a.arr.size() != b.arr.size()) return false;
      for (size_t n = 0; n < a.arr.size(); ++n)
        if (!(a.arr[n] == b.arr[n])) return false;
      return true;
    case T::Object: {
      if (a.obj.size() != b.obj.size()) return false;
      for (auto& m : a.obj) {
        const Value* o = b.get(m.k);
        if (!o || !(m.v == *o)) return false;
      }
      return true;
    }
  }
  return false;
}

// ------------------------------------------------------------------ parser

class ParseError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class Parser {
 public:
  Parser(const char* p, size_t n) : p_(p), end_(p + n) {}
  Value parse() {
    Value v = value(0);
    ws();
    if (p_ != end_) throw ParseError("trailing characters after JSON value");
    return v;
  }

 private:
  const char* p_;
  const char* end_;

  void ws() {
    while (p_ < end_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) ++p_;
  }
  [[noreturn]] void fail(const char* m) { throw ParseError(m); }

  Value value(int depth) {
    if (depth > 256) fail("JSON nesting too deep");
    ws();
    if (p_ >= end_) fail("unexpected end of JSON");
    char c = *p_;
    if (c == '{') return object(depth);
    if (c == '[') return array(depth);
    if (c == '"') return Value::str(string());
    if (c == 't') { lit("true"); return Value::boolean(true); }
    if (c == 'f') { lit("false"); return Value::boolean(false); }
    if (c == 'n') { lit("null"); return Value(); }
    if (c == '-' || (c >= '0' && c <= '9')) return number();
    fail("invalid JSON value");
  }
  void lit(const char* w) {
    size_t n = std::strlen(w);
    if ((size_t)(end_ - p_) < n || std::memcmp(p_, w, n) != 0) fail("invalid literal");
    p_ += n;
  }
  Value number() {
    const char* s = p_;
    bool fl = false;
    if (*p_ == '-') ++p_;
    while (p_ < end_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == 'e' || *p_ == 'E' || *p_ == '+' ||
                         *p_ == '-')) {
      if (*p_ == '.' || *p_ == 'e' || *p_ == 'E') fl = true;
      ++p_;
    }
    if (!fl) {
      int64_t v;
      auto r = std::from_chars(s, p_, v);
      if (r.ec == std::errc() && r.ptr == p_) return Value::integer(v);
    }
    double d;
    auto r = std::from_chars(s, p_, d);
    if (r.ec != std::errc() || r.ptr != p_) fail("invalid number");
    return Value::number(d);
  }
  static void utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) out += (char)cp;
    else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) {
      out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
    } else {
      out += (char)(0xF0 | (cp >> 18)); out += (char)(0x80 | ((cp >> 12) & 0x3F));
      out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
    }
  }
  uint32_t hex4() {
    if (end_ - p_ < 4) fail("bad \\u escape");
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = *p_++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex digit");
    }
    return v;
  }
  std::string string() {
    ++p_;  // opening quote
    std::string out;
    const char* run = p_;
    while (true) {
      if (p_ >= end_) fail("unterminated string");
      char c = *p_;
      if (c == '"') {
        out.append(run, p_ - run);
        ++p_;
        return out;
      }
      if (c == '\\') {
        out.append(run, p_ - run);
        ++p_;
        if (p_ >= end_) fail("bad escape");
        char e = *p_++;
        switch (e) {
          case '"': out += '"'; break;
          case '\\': out += '\\'; break;
          case '/': out += '/'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'n': out += '\n'; break;
          case 'r': out += '\r'; break;
          case 't': out += '\t'; break;
          case 'u': {
            uint32_t cp = hex4();
            if (cp >= 0xD800 && cp <= 0xDBFF && end_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
              p_ += 2;
              uint32_t lo = hex4();
              if (lo >= 0xDC00 && lo <= 0xDFFF) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
              else { utf8(out, cp); cp = lo; }
            }
            utf8(out, cp);
            break;
          }
          default: fail("bad escape");
        }
        run = p_;
        continue;
      }
      if ((unsigned char)c < 0x20) fail("control character in string");
      ++p_;
    }
  }
  Value array(int depth) {
    ++p_;
    Value v = Value::array();
    ws();
    if (p_ < end_ && *p_ == ']') { ++p_; return v; }
    while (true) {
      v.arr.push_back(value(depth + 1));
      ws();
      if (p_ >= end_) fail("unterminated array");
      if (*p_ == ',') { ++p_; continue; }
      if (*p_ == ']') { ++p_; return v; }
      fail("expected , or ]");
    }
  }
  Value object(int depth) {
    ++p_;
    Value v = Value::object();
    ws();
    if (p_ < end_ && *p_ == '}') { ++p_; return v; }
    while (true) {
      ws();
      if (p_ >= end_ || *p_ != '"') fail("expected object key");
      std::string k = string();
      ws();
      if (p_ >= end_ || *p_ != ':') fail("expected :");
      ++p_;
      Value val = value(depth + 1);
      // duplicate keys: last wins (encoding/json behaviour)
      Value* ex = v.get(k);
      if (ex) *ex = std::move(val);
      else v.obj.push_back(Member{std::move(k), std::move(val)});
      ws();
      if (p_ >= end_) fail("unterminated object");
      if (*p_ == ',') { ++p_; continue; }
      if (*p_ == '}') { ++p_; return v; }
      fail("expected , or }");
    }
  }
};

inline Value parse(std::string_view s) { return Parser(s.data(), s.size()).parse(); }

// ------------------------------------------------------------------ serializer

inline void escape(std::string& out, const std::string& s) {
  out += '"';
  size_t run = 0;
  for (size_t n = 0; n < s.size(); ++n) {
    unsigned char c = (unsigned char)s[n];
    const char* rep = nullptr;
    char buf[8];
    if (c == '"') rep = "\\\"";
    else if (c == '\\') rep = "\\\\";
    else if (c == '\n') rep = "\\n";
    else if (c == '\r') rep = "\\r";
    else if (c == '\t') rep = "\\t";
    else if (c < 0x20) {
      std::snprintf(buf, sizeof(buf), "\\u%04x", c);
      rep = buf;
    }
    if (rep) {
      out.append(s, run, n - run);
      out += rep;
      run = n + 1;
    }
  }
  out.append(s, run, std::string::npos);
  out += '"';
}

inline void dump(std::string& out, const Value& v) {
  switch (v.t) {
    case T::Null: out += "null"; break;
    case T::Bool: out += v.b ? "true" : "false"; break;
    case T::Int: {
      char buf[24];
      auto r = std::to_chars(buf, buf + sizeof(buf), v.i);
      out.append(buf, r.ptr);
      break;
    }
    case T::Double: {
      char buf[32];
      auto r = std::to_chars(buf, buf + sizeof(buf), v.d);
      out.append(buf, r.ptr);
      break;
    }
    case T::String: escape(out, v.s); break;
    case T::Array:
      out += '[';
      for (size_t n = 0; n < v.arr.size(); ++n) {
        if (n) out += ',';
        dump(out, v.arr[n]);
      }
      out += ']';
      break;
    case T::Object:
      out += '{';
      for (size_t n = 0; n < v.obj.size(); ++n) {
        if (n) out += ',';
        escape(out, v.obj[n].k);
        out += ':';
        dump(out, v.obj[n].v);
      }
      out += '}';
      break;
  }
}

inline std::string dump(const Value& v) {
  std::string s;
  s.reserve(512);
  dump(s, v);
  return s;
}

}  // namespace kj
