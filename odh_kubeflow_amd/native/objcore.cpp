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
#define PY_SSIZE_T_CLEAN
#include <Python.h>

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

PyMethodDef methods[] = {
    {"deepcopy", py_deepcopy, METH_O, "Deep copy of a JSON tree (dict/list; tuples become lists)."},
    {"semantic_equal", py_semantic_equal, METH_VARARGS,
     "Structural equality treating missing/None/{}/[] map values as equal."},
    {"equal_except", py_equal_except, METH_VARARGS, "a == b ignoring the given metadata keys."},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_objcore", "Native JSON-tree core", -1, methods,
                      nullptr, nullptr, nullptr, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__objcore(void) { return PyModule_Create(&module); }
