// Native JSON-tree core for the control plane (CPython C API).
//
// Kubernetes objects flow through the framework as dict/list trees in wire form.
// The Go reference gets typed DeepCopy() (generated, zz_generated.deepcopy.go) and
// equality.Semantic.DeepEqual for free; here they are the hot loops of the in-memory
// apiserver, the informer cache and every desired-vs-found comparison, so they are
// implemented natively:
//
//   deepcopy(o)            dict/list/tuple trees are copied (tuples become lists, as a
//                          JSON round trip would); str/int/float/bool/None are shared
//   semantic_equal(a, b)   structural equality where a missing key, None, {} and []
//                          are equivalent map values (apimachinery treats nil and empty
//                          maps/slices as equal, and omitempty drops them on the wire)
//   equal_except(a, b, keys)  equality of two objects ignoring the listed top-level
//                          metadata keys (the apiserver's no-op write detection)
//   loads_shared(data, old)   JSON -> dict/list tree (json.loads semantics) that reuses the
//                          subtrees of ``old`` the new document leaves unchanged
//   loads_event(line, lookup) one watch event line -> (type, object), the object decoded
//                          against lookup(namespace, name) — the informer's cached version
//
// Why share: a watch MODIFIED event carries the whole object again, while a status write
// changes a handful of fields.  Decoding against the cached version allocates only the
// changed subtrees (the rest is the cached objects, reference-counted), and the controllers'
// old-vs-new predicates over unchanged subtrees become identity comparisons.  Cached objects
// are never mutated in place (readers get deep copies), which is what makes sharing safe.
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <unordered_map>
#include <utility>
#include <vector>

namespace {

PyObject* copy_tree(PyObject* o, int depth) {
  if (depth > 512) {
    PyErr_SetString(PyExc_RecursionError, "object tree too deep");
    return nullptr;
  }
  if (PyDict_CheckExact(o)) {
    PyObject* out = _PyDict_NewPresized(PyDict_GET_SIZE(o));
    if (!out) return nullptr;
    Py_ssize_t pos = 0;
    PyObject *k, *v;
    while (PyDict_Next(o, &pos, &k, &v)) {
      PyObject* c = copy_tree(v, depth + 1);
      if (!c || PyDict_SetItem(out, k, c) < 0) {
        Py_XDECREF(c);
        Py_DECREF(out);
        return nullptr;
      }
      Py_DECREF(c);
    }
    return out;
  }
  if (PyList_CheckExact(o) || PyTuple_CheckExact(o)) {
    const bool is_list = PyList_CheckExact(o);
    const Py_ssize_t n = is_list ? PyList_GET_SIZE(o) : PyTuple_GET_SIZE(o);
    PyObject* out = PyList_New(n);
    if (!out) return nullptr;
    for (Py_ssize_t i = 0; i < n; ++i) {
      PyObject* c = copy_tree(is_list ? PyList_GET_ITEM(o, i) : PyTuple_GET_ITEM(o, i), depth + 1);
      if (!c) {
        Py_DECREF(out);
        return nullptr;
      }
      PyList_SET_ITEM(out, i, c);
    }
    return out;
  }
  if (PyDict_Check(o)) {  // dict subclasses: copy into a plain dict
    PyObject* plain = PyDict_Copy(o);
    if (!plain) return nullptr;
    PyObject* r = copy_tree(plain, depth);
    Py_DECREF(plain);
    return r;
  }
  Py_INCREF(o);
  return o;
}

// "empty" as a map value: None, a dict whose values are all empty, or an empty list
bool is_empty(PyObject* v) {
  if (v == Py_None) return true;
  if (PyDict_Check(v)) {
    Py_ssize_t pos = 0;
    PyObject *k, *x;
    while (PyDict_Next(v, &pos, &k, &x))
      if (!is_empty(x)) return false;
    return true;
  }
  if (PyList_Check(v)) return PyList_GET_SIZE(v) == 0;
  return false;
}

int sem_eq(PyObject* a, PyObject* b, int depth);

int dict_eq(PyObject* a, PyObject* b, int depth) {
  Py_ssize_t pos = 0;
  PyObject *k, *va;
  while (PyDict_Next(a, &pos, &k, &va)) {
    PyObject* vb = PyDict_GetItemWithError(b, k);
    if (!vb) {
      if (PyErr_Occurred()) return -1;
      if (!is_empty(va)) return 0;
      continue;
    }
    if (is_empty(va) && is_empty(vb)) continue;
    int r = sem_eq(va, vb, depth + 1);
    if (r <= 0) return r;
  }
  pos = 0;
  PyObject* vb;
  while (PyDict_Next(b, &pos, &k, &vb)) {
    PyObject* x = PyDict_GetItemWithError(a, k);
    if (!x) {
      if (PyErr_Occurred()) return -1;
      if (!is_empty(vb)) return 0;
    }
  }
  return 1;
}

int sem_eq(PyObject* a, PyObject* b, int depth) {
  if (depth > 512) {
    PyErr_SetString(PyExc_RecursionError, "object tree too deep");
    return -1;
  }
  if (a == b) return 1;
  if (PyDict_Check(a) && PyDict_Check(b)) return dict_eq(a, b, depth);
  const bool la = PyList_Check(a) || PyTuple_Check(a), lb = PyList_Check(b) || PyTuple_Check(b);
  if (la && lb) {
    PyObject* fa = PySequence_Fast(a, "");
    PyObject* fb = PySequence_Fast(b, "");
    if (!fa || !fb) {
      Py_XDECREF(fa);
      Py_XDECREF(fb);
      return -1;
    }
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(fa);
    int r = n == PySequence_Fast_GET_SIZE(fb) ? 1 : 0;
    for (Py_ssize_t i = 0; r == 1 && i < n; ++i) {
      PyObject* x = PySequence_Fast_GET_ITEM(fa, i);
      PyObject* y = PySequence_Fast_GET_ITEM(fb, i);
      // inside a list only dicts prune (a None element stays None)
      if (PyDict_Check(x) && PyDict_Check(y)) r = dict_eq(x, y, depth + 1);
      else r = sem_eq(x, y, depth + 1);
    }
    Py_DECREF(fa);
    Py_DECREF(fb);
    return r;
  }
  if (PyDict_Check(a) || PyDict_Check(b) || la || lb) return 0;
  return PyObject_RichCompareBool(a, b, Py_EQ);
}

PyObject* py_deepcopy(PyObject*, PyObject* o) { return copy_tree(o, 0); }

PyObject* py_semantic_equal(PyObject*, PyObject* args) {
  PyObject *a, *b;
  if (!PyArg_ParseTuple(args, "OO", &a, &b)) return nullptr;
  int r;
  if (is_empty(a) && is_empty(b)) r = 1;
  else r = sem_eq(a, b, 0);
  if (r < 0) return nullptr;
  return PyBool_FromLong(r);
}

// equal_except(a, b, meta_keys): a == b ignoring metadata[k] for k in meta_keys
PyObject* py_equal_except(PyObject*, PyObject* args) {
  PyObject *a, *b, *keys;
  if (!PyArg_ParseTuple(args, "O!O!O", &PyDict_Type, &a, &PyDict_Type, &b, &keys)) return nullptr;
  static PyObject* metadata_str = PyUnicode_InternFromString("metadata");
  if (PyDict_GET_SIZE(a) != PyDict_GET_SIZE(b)) Py_RETURN_FALSE;
  Py_ssize_t pos = 0;
  PyObject *k, *va;
  while (PyDict_Next(a, &pos, &k, &va)) {
    PyObject* vb = PyDict_GetItemWithError(b, k);
    if (!vb) {
      if (PyErr_Occurred()) return nullptr;
      Py_RETURN_FALSE;
    }
    int eq;
    if (PyUnicode_Check(k) && PyUnicode_Compare(k, metadata_str) == 0 && PyDict_Check(va) && PyDict_Check(vb)) {
      // compare metadata dicts skipping `keys`
      eq = 1;
      for (int pass = 0; pass < 2 && eq == 1; ++pass) {
        PyObject* x = pass ? vb : va;
        PyObject* y = pass ? va : vb;
        Py_ssize_t p2 = 0;
        PyObject *mk, *mv;
        while (PyDict_Next(x, &p2, &mk, &mv)) {
          int skip = PySequence_Contains(keys, mk);
          if (skip < 0) return nullptr;
          if (skip) continue;
          PyObject* other = PyDict_GetItemWithError(y, mk);
          if (!other) {
            if (PyErr_Occurred()) return nullptr;
            eq = 0;
            break;
          }
          if (pass == 0) {
            int r = PyObject_RichCompareBool(mv, other, Py_EQ);
            if (r < 0) return nullptr;
            if (!r) {
              eq = 0;
              break;
            }
          }
        }
      }
    } else {
      eq = PyObject_RichCompareBool(va, vb, Py_EQ);
      if (eq < 0) return nullptr;
    }
    if (!eq) Py_RETURN_FALSE;
  }
  Py_RETURN_TRUE;
}


// ------------------------------------------------------------------ shared-subtree JSON decoder

struct Parser {
  const char* p;
  const char* end;
  std::string buf;  // scratch for unescaped strings and number text
  // owned references of the objects and arrays being built, innermost last: a container's
  // members are collected here (one allocation for the whole document, not one per dict)
  std::vector<PyObject*> stack;
};

// a container's run of owned references on ps.stack, released (and popped) on every exit
struct Frame {
  Parser& ps;
  size_t base;
  explicit Frame(Parser& p) : ps(p), base(p.stack.size()) {}
  ~Frame() {
    for (size_t i = base; i < ps.stack.size(); ++i) Py_XDECREF(ps.stack[i]);
    ps.stack.resize(base);
  }
  size_t size() const { return ps.stack.size() - base; }
  PyObject*& at(size_t i) { return ps.stack[base + i]; }
};

// interned object keys: the small vocabulary of Kubernetes field names, decoded once; the
// map's string_views point into the (ASCII, immortal-while-cached) key objects themselves
std::unordered_map<std::string_view, PyObject*>* g_keys = nullptr;
constexpr size_t kMaxKeys = 1 << 15;

inline void ws(Parser& ps) {
  while (ps.p < ps.end && (*ps.p == ' ' || *ps.p == '\n' || *ps.p == '\r' || *ps.p == '\t')) ++ps.p;
}

PyObject* fail(Parser&, const char* what) {
  if (!PyErr_Occurred()) PyErr_Format(PyExc_ValueError, "invalid JSON: %s", what);
  return nullptr;
}

void put_utf8(std::string& out, uint32_t cp) {
  if (cp < 0x80) {
    out.push_back(static_cast<char>(cp));
  } else if (cp < 0x800) {
    out.push_back(static_cast<char>(0xC0 | (cp >> 6)));
    out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  } else if (cp < 0x10000) {  // lone surrogates too (decoded with surrogatepass, as json does)
    out.push_back(static_cast<char>(0xE0 | (cp >> 12)));
    out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  } else {
    out.push_back(static_cast<char>(0xF0 | (cp >> 18)));
    out.push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
    out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  }
}

int hex4(const char* s, uint32_t* out) {
  uint32_t v = 0;
  for (int i = 0; i < 4; ++i) {
    char c = s[i];
    v <<= 4;
    if (c >= '0' && c <= '9') v |= c - '0';
    else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
    else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
    else return -1;
  }
  *out = v;
  return 0;
}

// The string at ps.p (just past the opening quote) as UTF-8: a view into the input when it
// has no escapes, else unescaped into ps.buf.  *ascii: every byte < 0x80.
bool scan_string(Parser& ps, const char** s, Py_ssize_t* n, bool* ascii) {
  const char* start = ps.p;
  bool hi = false;
  while (ps.p < ps.end) {
    unsigned char c = static_cast<unsigned char>(*ps.p);
    if (c == '"') {
      *s = start;
      *n = ps.p - start;
      *ascii = !hi;
      ++ps.p;
      return true;
    }
    if (c == '\\') break;
    if (c >= 0x80) hi = true;
    ++ps.p;
  }
  if (ps.p >= ps.end) {
    PyErr_SetString(PyExc_ValueError, "invalid JSON: unterminated string");
    return false;
  }
  ps.buf.assign(start, ps.p - start);
  while (ps.p < ps.end) {
    unsigned char c = static_cast<unsigned char>(*ps.p);
    if (c == '"') {
      ++ps.p;
      *s = ps.buf.data();
      *n = static_cast<Py_ssize_t>(ps.buf.size());
      *ascii = !hi;
      return true;
    }
    if (c != '\\') {
      if (c >= 0x80) hi = true;
      ps.buf.push_back(static_cast<char>(c));
      ++ps.p;
      continue;
    }
    if (ps.p + 1 >= ps.end) break;
    char e = ps.p[1];
    ps.p += 2;
    switch (e) {
      case '"': ps.buf.push_back('"'); break;
      case '\\': ps.buf.push_back('\\'); break;
      case '/': ps.buf.push_back('/'); break;
      case 'b': ps.buf.push_back('\b'); break;
      case 'f': ps.buf.push_back('\f'); break;
      case 'n': ps.buf.push_back('\n'); break;
      case 'r': ps.buf.push_back('\r'); break;
      case 't': ps.buf.push_back('\t'); break;
      case 'u': {
        uint32_t cp;
        if (ps.end - ps.p < 4 || hex4(ps.p, &cp) < 0) {
          PyErr_SetString(PyExc_ValueError, "invalid JSON: bad \\u escape");
          return false;
        }
        ps.p += 4;
        if (cp >= 0xD800 && cp < 0xDC00 && ps.end - ps.p >= 6 && ps.p[0] == '\\' && ps.p[1] == 'u') {
          uint32_t lo;
          if (hex4(ps.p + 2, &lo) == 0 && lo >= 0xDC00 && lo < 0xE000) {
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            ps.p += 6;
          }
        }
        if (cp >= 0x80) hi = true;
        put_utf8(ps.buf, cp);
        break;
      }
      default:
        PyErr_SetString(PyExc_ValueError, "invalid JSON: bad escape");
        return false;
    }
  }
  PyErr_SetString(PyExc_ValueError, "invalid JSON: unterminated string");
  return false;
}

PyObject* make_str(const char* s, Py_ssize_t n, bool ascii) {
  if (ascii) {
    PyObject* u = PyUnicode_New(n, 127);
    if (!u) return nullptr;
    std::memcpy(PyUnicode_DATA(u), s, static_cast<size_t>(n));
    return u;
  }
  return PyUnicode_DecodeUTF8(s, n, "surrogatepass");
}

// ``old`` in place of the new scalar ``v`` when they are equal (the cases the fast paths do not
// decide: integers beyond 64 bits, strings whose UTF-8 form cannot be compared directly)
PyObject* same_or(PyObject* v, PyObject* old) {
  if (old && Py_TYPE(old) == Py_TYPE(v)) {
    int eq = PyObject_RichCompareBool(v, old, Py_EQ);
    if (eq < 0) {
      PyErr_Clear();
    } else if (eq) {
      Py_DECREF(v);
      Py_INCREF(old);
      return old;
    }
  }
  return v;
}

// ``old`` when it is the same string, else a new one
PyObject* string_value(const char* s, Py_ssize_t n, bool ascii, PyObject* old) {
  if (old && PyUnicode_CheckExact(old)) {
    if (ascii && PyUnicode_IS_ASCII(old)) {
      if (PyUnicode_GET_LENGTH(old) == n && std::memcmp(PyUnicode_DATA(old), s, static_cast<size_t>(n)) == 0) {
        Py_INCREF(old);
        return old;
      }
    } else if (!ascii && !PyUnicode_IS_ASCII(old)) {
      Py_ssize_t on;
      const char* os = PyUnicode_AsUTF8AndSize(old, &on);
      if (!os) {
        PyErr_Clear();
      } else if (on == n && std::memcmp(os, s, static_cast<size_t>(n)) == 0) {
        Py_INCREF(old);
        return old;
      }
    }
  }
  PyObject* u = make_str(s, n, ascii);
  return u ? same_or(u, old) : nullptr;
}

PyObject* key_object(const char* s, Py_ssize_t n, bool ascii) {
  if (!ascii) return make_str(s, n, false);
  auto it = g_keys->find(std::string_view(s, static_cast<size_t>(n)));
  if (it != g_keys->end()) {
    Py_INCREF(it->second);
    return it->second;
  }
  PyObject* u = make_str(s, n, true);
  if (!u) return nullptr;
  PyUnicode_InternInPlace(&u);
  if (g_keys->size() < kMaxKeys && PyUnicode_IS_ASCII(u)) {
    Py_INCREF(u);  // held for the process: the view below points into it
    g_keys->emplace(std::string_view(static_cast<const char*>(PyUnicode_DATA(u)), static_cast<size_t>(n)), u);
  }
  return u;
}

PyObject* number_value(Parser& ps, PyObject* old) {
  const char* start = ps.p;
  bool is_float = false;
  if (ps.p < ps.end && *ps.p == '-') ++ps.p;
  while (ps.p < ps.end) {
    char c = *ps.p;
    if (c >= '0' && c <= '9') {
      ++ps.p;
    } else if (c == '.' || c == 'e' || c == 'E' || c == '+' || c == '-') {
      is_float = true;
      ++ps.p;
    } else {
      break;
    }
  }
  if (ps.p == start || (ps.p - start == 1 && *start == '-')) return fail(ps, "bad number");
  if (!is_float) {  // the common case, at most 18 digits: no copy, no strtoll
    const char* q = start;
    const bool neg = *q == '-';
    if (neg) ++q;
    if (ps.p - q <= 18 && (ps.p - q == 1 || *q != '0')) {
      long long v = 0;
      for (; q < ps.p; ++q) v = v * 10 + (*q - '0');
      if (neg) v = -v;
      if (old && PyLong_CheckExact(old)) {
        int overflow = 0;
        long long ov = PyLong_AsLongLongAndOverflow(old, &overflow);
        if (!overflow && ov == v && !PyErr_Occurred()) {
          Py_INCREF(old);
          return old;
        }
        PyErr_Clear();
      }
      return PyLong_FromLongLong(v);
    }
  }
  ps.buf.assign(start, ps.p - start);
  if (!is_float) {
    errno = 0;
    char* e = nullptr;
    long long v = std::strtoll(ps.buf.c_str(), &e, 10);
    if (errno == 0 && e && *e == '\0') {
      if (old && PyLong_CheckExact(old)) {
        int overflow = 0;
        long long ov = PyLong_AsLongLongAndOverflow(old, &overflow);
        if (!overflow && ov == v && !PyErr_Occurred()) {
          Py_INCREF(old);
          return old;
        }
        PyErr_Clear();
      }
      return PyLong_FromLongLong(v);
    }
    PyObject* big = PyLong_FromString(ps.buf.c_str(), nullptr, 10);  // beyond 64 bits
    return big ? same_or(big, old) : nullptr;
  }
  char* e = nullptr;
  double d = std::strtod(ps.buf.c_str(), &e);
  if (!e || *e != '\0') return fail(ps, "bad number");
  if (old && PyFloat_CheckExact(old) && PyFloat_AS_DOUBLE(old) == d) {
    Py_INCREF(old);
    return old;
  }
  return PyFloat_FromDouble(d);
}

PyObject* value(Parser& ps, PyObject* old, int depth);

PyObject* object_value(Parser& ps, PyObject* old, int depth) {
  // ps.p just past '{'.  With an old dict the members are collected first: an unchanged
  // object is the old one, and no dict is built for it.
  PyObject* od = (old && PyDict_CheckExact(old)) ? old : nullptr;
  Frame f(ps);  // key, value, key, value, ...
  bool same = od != nullptr;
  // the old dict's members in order: a re-sent object lists its keys in the same order, so
  // the i-th key is usually the old i-th one (no hashing, no lookup)
  Py_ssize_t pos = 0;
  bool in_step = od != nullptr;
  ws(ps);
  if (ps.p < ps.end && *ps.p == '}') {
    ++ps.p;
  } else {
    while (true) {
      ws(ps);
      if (ps.p >= ps.end || *ps.p != '"') return fail(ps, "expected a key");
      ++ps.p;
      const char* ks;
      Py_ssize_t kn;
      bool kascii;
      if (!scan_string(ps, &ks, &kn, &kascii)) return nullptr;
      PyObject* key = nullptr;
      PyObject* ov = nullptr;
      if (in_step) {
        PyObject *k2, *v2;
        if (PyDict_Next(od, &pos, &k2, &v2) && PyUnicode_CheckExact(k2) && PyUnicode_IS_ASCII(k2) && kascii &&
            PyUnicode_GET_LENGTH(k2) == kn && std::memcmp(PyUnicode_DATA(k2), ks, static_cast<size_t>(kn)) == 0) {
          key = k2;
          Py_INCREF(key);
          ov = v2;
        } else {
          in_step = false;
        }
      }
      if (!key) {
        key = key_object(ks, kn, kascii);
        if (!key) return nullptr;
        ov = od ? PyDict_GetItemWithError(od, key) : nullptr;
        if (!ov && PyErr_Occurred()) PyErr_Clear();
      }
      ps.stack.push_back(key);
      ws(ps);
      if (ps.p >= ps.end || *ps.p != ':') return fail(ps, "expected ':'");
      ++ps.p;
      PyObject* v = value(ps, ov, depth + 1);
      if (!v) return nullptr;
      ps.stack.push_back(v);
      if (v != ov) same = false;
      ws(ps);
      if (ps.p < ps.end && *ps.p == ',') {
        ++ps.p;
        continue;
      }
      if (ps.p < ps.end && *ps.p == '}') {
        ++ps.p;
        break;
      }
      return fail(ps, "expected ',' or '}'");
    }
  }
  const Py_ssize_t n = static_cast<Py_ssize_t>(f.size() / 2);
  // every member is the old one's, in the old order, and there are as many: the keys matched
  // the old dict's one by one, so they are distinct and the object is the old one
  if (same && in_step && depth > 0 && n == PyDict_GET_SIZE(od)) {
    Py_INCREF(od);
    return od;
  }
  PyObject* out = _PyDict_NewPresized(n);
  if (!out) return nullptr;
  for (Py_ssize_t i = 0; i < n; ++i) {
    if (PyDict_SetItem(out, f.at(2 * i), f.at(2 * i + 1)) < 0) {
      Py_DECREF(out);
      return nullptr;
    }
  }
  // out of order, every value the old one's: the old dict iff as many DISTINCT keys — a
  // duplicated key ({"x":1,"x":1} against {"x":1,"y":2}) must not stand in for a missing one
  if (same && depth > 0 && PyDict_GET_SIZE(out) == PyDict_GET_SIZE(od)) {
    Py_DECREF(out);
    Py_INCREF(od);
    return od;
  }
  return out;
}

PyObject* array_value(Parser& ps, PyObject* old, int depth) {
  PyObject* ol = (old && PyList_CheckExact(old)) ? old : nullptr;
  Frame f(ps);
  bool same = ol != nullptr;
  ws(ps);
  if (ps.p < ps.end && *ps.p == ']') {
    ++ps.p;
  } else {
    while (true) {
      Py_ssize_t i = static_cast<Py_ssize_t>(f.size());
      PyObject* ov = (ol && i < PyList_GET_SIZE(ol)) ? PyList_GET_ITEM(ol, i) : nullptr;
      PyObject* v = value(ps, ov, depth + 1);
      if (!v) return nullptr;
      ps.stack.push_back(v);
      if (v != ov) same = false;
      ws(ps);
      if (ps.p < ps.end && *ps.p == ',') {
        ++ps.p;
        continue;
      }
      if (ps.p < ps.end && *ps.p == ']') {
        ++ps.p;
        break;
      }
      return fail(ps, "expected ',' or ']'");
    }
  }
  const size_t n = f.size();
  if (same && depth > 0 && static_cast<Py_ssize_t>(n) == PyList_GET_SIZE(ol)) {
    Py_INCREF(ol);
    return ol;
  }
  PyObject* out = PyList_New(static_cast<Py_ssize_t>(n));
  if (!out) return nullptr;
  for (size_t i = 0; i < n; ++i) {
    PyList_SET_ITEM(out, static_cast<Py_ssize_t>(i), f.at(i));  // the reference moves
    f.at(i) = nullptr;
  }
  return out;
}

bool literal(Parser& ps, const char* word, size_t n) {
  if (static_cast<size_t>(ps.end - ps.p) >= n && std::memcmp(ps.p, word, n) == 0) {
    ps.p += n;
    return true;
  }
  return false;
}

PyObject* value(Parser& ps, PyObject* old, int depth) {
  if (depth > 512) {
    PyErr_SetString(PyExc_RecursionError, "JSON too deep");
    return nullptr;
  }
  ws(ps);
  if (ps.p >= ps.end) return fail(ps, "unexpected end");
  char c = *ps.p;
  if (c == '{') {
    ++ps.p;
    return object_value(ps, old, depth);
  }
  if (c == '[') {
    ++ps.p;
    return array_value(ps, old, depth);
  }
  if (c == '"') {
    ++ps.p;
    if (old && PyUnicode_CheckExact(old) && PyUnicode_IS_ASCII(old)) {
      // the old string verbatim, closing quote included, with no quote or backslash inside:
      // it is the old string (one memcmp, no scan, no allocation)
      const Py_ssize_t on = PyUnicode_GET_LENGTH(old);
      const char* od = static_cast<const char*>(PyUnicode_DATA(old));
      if (ps.end - ps.p > on && ps.p[on] == '"' && std::memcmp(ps.p, od, static_cast<size_t>(on)) == 0 &&
          !std::memchr(ps.p, '"', static_cast<size_t>(on)) && !std::memchr(ps.p, '\\', static_cast<size_t>(on))) {
        ps.p += on + 1;
        Py_INCREF(old);
        return old;
      }
    }
    const char* s;
    Py_ssize_t n;
    bool ascii;
    if (!scan_string(ps, &s, &n, &ascii)) return nullptr;
    return string_value(s, n, ascii, old);
  }
  if (c == '-' || (c >= '0' && c <= '9')) return number_value(ps, old);
  if (literal(ps, "true", 4)) Py_RETURN_TRUE;
  if (literal(ps, "false", 5)) Py_RETURN_FALSE;
  if (literal(ps, "null", 4)) Py_RETURN_NONE;
  return fail(ps, "unexpected character");
}

// skip one value without building it (the pre-scan for an event's metadata)
bool skip_value(Parser& ps, int depth) {
  if (depth > 512) return false;
  ws(ps);
  if (ps.p >= ps.end) return false;
  char c = *ps.p;
  if (c == '"') {
    ++ps.p;
    while (ps.p < ps.end && *ps.p != '"') ps.p += (*ps.p == '\\') ? 2 : 1;
    if (ps.p >= ps.end) return false;
    ++ps.p;
    return true;
  }
  if (c == '{' || c == '[') {
    char close = c == '{' ? '}' : ']';
    ++ps.p;
    ws(ps);
    if (ps.p < ps.end && *ps.p == close) {
      ++ps.p;
      return true;
    }
    while (true) {
      if (c == '{') {
        if (!skip_value(ps, depth + 1)) return false;  // the key
        ws(ps);
        if (ps.p >= ps.end || *ps.p != ':') return false;
        ++ps.p;
      }
      if (!skip_value(ps, depth + 1)) return false;
      ws(ps);
      if (ps.p < ps.end && *ps.p == ',') {
        ++ps.p;
        continue;
      }
      if (ps.p < ps.end && *ps.p == close) {
        ++ps.p;
        return true;
      }
      return false;
    }
  }
  while (ps.p < ps.end && *ps.p != ',' && *ps.p != '}' && *ps.p != ']' && *ps.p != ' ' && *ps.p != '\n') ++ps.p;
  return true;
}

// metadata.namespace / metadata.name of the object at ps.p (ps is a copy: not advanced)
void peek_key(Parser ps, std::string* ns, std::string* name) {
  ws(ps);
  if (ps.p >= ps.end || *ps.p != '{') return;
  ++ps.p;
  while (true) {
    ws(ps);
    if (ps.p >= ps.end || *ps.p != '"') return;
    ++ps.p;
    const char* ks;
    Py_ssize_t kn;
    bool ascii;
    if (!scan_string(ps, &ks, &kn, &ascii)) {
      PyErr_Clear();
      return;
    }
    bool is_meta = kn == 8 && std::memcmp(ks, "metadata", 8) == 0;
    ws(ps);
    if (ps.p >= ps.end || *ps.p != ':') return;
    ++ps.p;
    ws(ps);
    if (is_meta) {
      if (ps.p >= ps.end || *ps.p != '{') return;
      ++ps.p;
      while (true) {
        ws(ps);
        if (ps.p >= ps.end || *ps.p != '"') return;
        ++ps.p;
        if (!scan_string(ps, &ks, &kn, &ascii)) {
          PyErr_Clear();
          return;
        }
        std::string* dst = (kn == 4 && std::memcmp(ks, "name", 4) == 0)        ? name
                           : (kn == 9 && std::memcmp(ks, "namespace", 9) == 0) ? ns
                                                                                : nullptr;
        ws(ps);
        if (ps.p >= ps.end || *ps.p != ':') return;
        ++ps.p;
        ws(ps);
        if (dst && ps.p < ps.end && *ps.p == '"') {
          ++ps.p;
          const char* vs;
          Py_ssize_t vn;
          if (!scan_string(ps, &vs, &vn, &ascii)) {
            PyErr_Clear();
            return;
          }
          dst->assign(vs, static_cast<size_t>(vn));
        } else if (!skip_value(ps, 2)) {
          return;
        }
        ws(ps);
        if (ps.p < ps.end && *ps.p == ',') {
          ++ps.p;
          continue;
        }
        return;  // end of metadata
      }
    }
    if (!skip_value(ps, 1)) return;
    ws(ps);
    if (ps.p < ps.end && *ps.p == ',') {
      ++ps.p;
      continue;
    }
    return;
  }
}

bool init_parser(PyObject* data, Parser* ps) {
  char* buf;
  Py_ssize_t n;
  if (PyBytes_Check(data)) {
    if (PyBytes_AsStringAndSize(data, &buf, &n) < 0) return false;
  } else if (PyByteArray_Check(data)) {
    buf = PyByteArray_AS_STRING(data);
    n = PyByteArray_GET_SIZE(data);
  } else if (PyUnicode_Check(data)) {
    const char* s = PyUnicode_AsUTF8AndSize(data, &n);
    if (!s) return false;
    buf = const_cast<char*>(s);
  } else {
    PyErr_SetString(PyExc_TypeError, "expected bytes or str");
    return false;
  }
  ps->p = buf;
  ps->end = buf + n;
  return true;
}

PyObject* py_loads_shared(PyObject*, PyObject* args) {
  PyObject *data, *old = Py_None;
  if (!PyArg_ParseTuple(args, "O|O", &data, &old)) return nullptr;
  Parser ps;
  if (!init_parser(data, &ps)) return nullptr;
  PyObject* out = value(ps, old == Py_None ? nullptr : old, 0);
  if (!out) return nullptr;
  ws(ps);
  if (ps.p != ps.end) {
    Py_DECREF(out);
    return fail(ps, "extra data");
  }
  return out;
}

// loads_event(line, lookup) -> (type, object): lookup(namespace, name) gives the cached
// version of the event's object (or None) to share unchanged subtrees with
PyObject* py_loads_event(PyObject*, PyObject* args) {
  PyObject *data, *lookup = Py_None;
  if (!PyArg_ParseTuple(args, "O|O", &data, &lookup)) return nullptr;
  Parser ps;
  if (!init_parser(data, &ps)) return nullptr;
  ws(ps);
  if (ps.p >= ps.end || *ps.p != '{') return fail(ps, "an event is an object");
  ++ps.p;
  PyObject* type = nullptr;
  PyObject* obj = nullptr;
  PyObject* ret = nullptr;
  ws(ps);
  if (ps.p < ps.end && *ps.p == '}') {
    ++ps.p;
  } else {
    while (true) {
      ws(ps);
      if (ps.p >= ps.end || *ps.p != '"') {
        fail(ps, "expected a key");
        goto done;
      }
      ++ps.p;
      const char* ks;
      Py_ssize_t kn;
      bool ascii;
      if (!scan_string(ps, &ks, &kn, &ascii)) goto done;
      bool is_type = kn == 4 && std::memcmp(ks, "type", 4) == 0;
      bool is_obj = kn == 6 && std::memcmp(ks, "object", 6) == 0;
      ws(ps);
      if (ps.p >= ps.end || *ps.p != ':') {
        fail(ps, "expected ':'");
        goto done;
      }
      ++ps.p;
      if (is_obj) {
        PyObject* old = nullptr;
        if (lookup != Py_None) {
          std::string ns, name;
          peek_key(ps, &ns, &name);
          if (!name.empty()) {
            PyObject* r = PyObject_CallFunction(lookup, "s#s#", ns.data(), static_cast<Py_ssize_t>(ns.size()),
                                                name.data(), static_cast<Py_ssize_t>(name.size()));
            if (!r) goto done;
            if (r != Py_None) old = r;
            else Py_DECREF(r);
          }
        }
        Py_XDECREF(obj);
        obj = value(ps, old, 0);
        Py_XDECREF(old);
        if (!obj) goto done;
      } else {
        PyObject* v = value(ps, nullptr, 1);
        if (!v) goto done;
        if (is_type) {
          Py_XDECREF(type);
          type = v;
        } else {
          Py_DECREF(v);
        }
      }
      ws(ps);
      if (ps.p < ps.end && *ps.p == ',') {
        ++ps.p;
        continue;
      }
      if (ps.p < ps.end && *ps.p == '}') {
        ++ps.p;
        break;
      }
      fail(ps, "expected ',' or '}'");
      goto done;
    }
  }
  ws(ps);
  if (ps.p != ps.end) {
    fail(ps, "extra data");
    goto done;
  }
  if (!obj) obj = PyDict_New();
  if (!obj) goto done;
  ret = PyTuple_Pack(2, type ? type : Py_None, obj);
done:
  Py_XDECREF(type);
  Py_XDECREF(obj);
  return ret;
}

// ------------------------------------------------------------------ encoding
// dumps(obj) -> bytes: json.dumps(obj, separators=(",", ":")) for JSON trees (dict with str
// keys, list, tuple, str, int, float, bool, None), written as UTF-8 rather than \u escapes.
// Anything else raises TypeError, and the caller falls back to json.dumps (which also
// reports cycles, deeper than the 512 levels taken here).

bool enc_value(std::string& out, PyObject* o, int depth);

void enc_string(std::string& out, PyObject* u) {
  Py_ssize_t n;
  const char* s = PyUnicode_AsUTF8AndSize(u, &n);
  out.push_back('"');
  const char* run = s;
  for (Py_ssize_t i = 0; i < n; ++i) {
    unsigned char c = static_cast<unsigned char>(s[i]);
    if (c >= 0x20 && c != '"' && c != '\\') continue;
    out.append(run, static_cast<size_t>(s + i - run));
    run = s + i + 1;
    switch (c) {
      case '"': out.append("\\\""); break;
      case '\\': out.append("\\\\"); break;
      case '\n': out.append("\\n"); break;
      case '\r': out.append("\\r"); break;
      case '\t': out.append("\\t"); break;
      case '\b': out.append("\\b"); break;
      case '\f': out.append("\\f"); break;
      default: {
        char u4[8];
        std::snprintf(u4, sizeof u4, "\\u%04x", c);
        out.append(u4);
      }
    }
  }
  out.append(run, static_cast<size_t>(s + n - run));
  out.push_back('"');
}

bool enc_value(std::string& out, PyObject* o, int depth) {
  if (depth > 512) {
    PyErr_SetString(PyExc_ValueError, "too deep");
    return false;
  }
  if (PyUnicode_Check(o)) {
    if (PyUnicode_IS_ASCII(o) || PyUnicode_AsUTF8(o)) {
      enc_string(out, o);
      return true;
    }
    return false;  // unpaired surrogates: json.dumps escapes them
  }
  if (o == Py_None) {
    out.append("null");
    return true;
  }
  if (o == Py_True) {
    out.append("true");
    return true;
  }
  if (o == Py_False) {
    out.append("false");
    return true;
  }
  if (PyLong_CheckExact(o)) {
    int overflow = 0;
    long long v = PyLong_AsLongLongAndOverflow(o, &overflow);
    if (!overflow && !(v == -1 && PyErr_Occurred())) {
      char b[24];
      int k = std::snprintf(b, sizeof b, "%lld", v);
      out.append(b, static_cast<size_t>(k));
      return true;
    }
    PyErr_Clear();
    PyObject* t = PyObject_Str(o);
    if (!t) return false;
    Py_ssize_t n;
    const char* d = PyUnicode_AsUTF8AndSize(t, &n);
    if (d) out.append(d, static_cast<size_t>(n));
    Py_DECREF(t);
    return d != nullptr;
  }
  if (PyFloat_CheckExact(o)) {
    double d = PyFloat_AS_DOUBLE(o);
    if (!std::isfinite(d)) {
      out.append(std::isnan(d) ? "NaN" : (d > 0 ? "Infinity" : "-Infinity"));
      return true;
    }
    char* r = PyOS_double_to_string(d, 'r', 0, Py_DTSF_ADD_DOT_0, nullptr);
    if (!r) return false;
    out.append(r);
    PyMem_Free(r);
    return true;
  }
  if (PyDict_CheckExact(o)) {
    out.push_back('{');
    Py_ssize_t pos = 0;
    PyObject *k, *v;
    bool first = true;
    while (PyDict_Next(o, &pos, &k, &v)) {
      if (!PyUnicode_CheckExact(k)) {
        PyErr_SetString(PyExc_TypeError, "non-str key");
        return false;
      }
      if (!first) out.push_back(',');
      first = false;
      if (!enc_value(out, k, depth + 1)) return false;
      out.push_back(':');
      if (!enc_value(out, v, depth + 1)) return false;
    }
    out.push_back('}');
    return true;
  }
  if (PyList_CheckExact(o) || PyTuple_CheckExact(o)) {
    const bool list = PyList_CheckExact(o);
    const Py_ssize_t n = list ? PyList_GET_SIZE(o) : PyTuple_GET_SIZE(o);
    out.push_back('[');
    for (Py_ssize_t i = 0; i < n; ++i) {
      if (i) out.push_back(',');
      if (!enc_value(out, list ? PyList_GET_ITEM(o, i) : PyTuple_GET_ITEM(o, i), depth + 1)) return false;
    }
    out.push_back(']');
    return true;
  }
  PyErr_SetString(PyExc_TypeError, "not a JSON tree");
  return false;
}

PyObject* py_dumps(PyObject*, PyObject* o) {
  std::string out;
  out.reserve(1024);
  if (!enc_value(out, o, 0)) {
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_TypeError, "not a JSON tree");
    return nullptr;
  }
  return PyBytes_FromStringAndSize(out.data(), static_cast<Py_ssize_t>(out.size()));
}

PyMethodDef methods[] = {
    {"dumps", py_dumps, METH_O,
     "dumps(obj) -> bytes: compact JSON (json.dumps with separators=(',', ':'), UTF-8) of a JSON tree."},
    {"deepcopy", py_deepcopy, METH_O, "Deep copy of a JSON tree (dict/list; tuples become lists)."},
    {"semantic_equal", py_semantic_equal, METH_VARARGS,
     "Structural equality treating missing/None/{}/[] map values as equal."},
    {"equal_except", py_equal_except, METH_VARARGS, "a == b ignoring the given metadata keys."},
    {"loads_shared", py_loads_shared, METH_VARARGS,
     "loads_shared(data, old=None): json.loads, reusing the subtrees of old the document leaves unchanged."},
    {"loads_event", py_loads_event, METH_VARARGS,
     "loads_event(line, lookup=None) -> (type, object): a watch event, the object decoded against "
     "lookup(namespace, name)."},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_objcore", "Native JSON-tree core", -1, methods,
                      nullptr, nullptr, nullptr, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__objcore(void) {
  if (!g_keys) g_keys = new std::unordered_map<std::string_view, PyObject*>();
  return PyModule_Create(&module);
}
