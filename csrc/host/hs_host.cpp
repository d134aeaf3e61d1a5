// Host hot paths of the query front end as a CPython extension (``hyperspace_amd._native._hs_host``).
//
// resolve(): binding a fresh DataFrame expression's column names to a plan's attributes
// (hyperspace_amd/plan/dataframe.py ``_resolve_walk``).
//
// fingerprint(): the plan cache's structural key of an analyzed logical plan
// (hyperspace_amd/plan/plan_cache.py ``_fp``).  A serving loop builds a fresh DataFrame per
// query, so this walk over a few hundred Python objects runs once per query on the submitting
// thread; done here it costs a fraction of the interpreted walk.  The output is the same nested
// tuple ``_fp`` builds (tests/test_plan_cache.py compares them), so either implementation can
// serve the cache.
//
// Dispatch is per exact type through ``kinds`` (type -> (code, type name)), filled by the Python
// ``classify`` callback the first time a type is seen:
//   0 generic node   (type name, ((field, fp(value)) for sorted fields)), expr_id canonicalized
//   1 literal        ("L", str(dtype), value is None), appended to ``lits``
//   2 attribute      ("A", name, str(dtype), nullable, eid(expr_id), qualifier)
//   3 children-only  (type name, (("children", fp(children)),)) when __dict__ has one field
//   4 Python         ``slow(obj)`` (dicts, Arrow types, identity-keyed objects, uncacheable nodes)
//   5 base relation  ``leaf(obj)``'s memo re-mapped into this query's attribute numbering
// Field names of a generic node come from the Python ``fields(__dict__)`` memo.
#include <Python.h>

namespace {

struct Ctx {
  PyObject* ids;      // dict: expr_id -> first-appearance number
  PyObject* lits;     // list: literal objects in walk order
  PyObject* kinds;    // dict: type -> (code, name)
  PyObject* classify; // callable(type) -> (code, name), also stores it in kinds
  PyObject* fields;   // callable(dict) -> tuple of sorted field names
  PyObject* slow;     // callable(obj) -> fingerprint (Python path)
  PyObject* leaf;     // callable(relation) -> (fp, expr ids, refs) memo or None
  PyObject* refs;     // list: objects keyed by identity (kept alive by the cache entry)
};

PyObject* s_L;
PyObject* s_A;
PyObject* s_children;
PyObject* s_expr_id;
PyObject* s_dtype;
PyObject* s_value;
PyObject* s_name;
PyObject* s_nullable;
PyObject* s_qualifier;

PyObject* fp(Ctx& c, PyObject* v);

PyObject* eid(Ctx& c, PyObject* x) {
  PyObject* hit = PyDict_GetItemWithError(c.ids, x);
  if (hit) {
    Py_INCREF(hit);
    return hit;
  }
  if (PyErr_Occurred()) return nullptr;
  PyObject* n = PyLong_FromSsize_t(PyDict_Size(c.ids));
  if (!n || PyDict_SetItem(c.ids, x, n) < 0) {
    Py_XDECREF(n);
    return nullptr;
  }
  return n;
}

PyObject* seq(Ctx& c, PyObject* v) {
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(v);
  PyObject** items = PySequence_Fast_ITEMS(v);
  PyObject* out = PyTuple_New(n);
  if (!out) return nullptr;
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* x = fp(c, items[i]);
    if (!x) {
      Py_DECREF(out);
      return nullptr;
    }
    PyTuple_SET_ITEM(out, i, x);
  }
  return out;
}

PyObject* str_attr(PyObject* v, PyObject* name) {
  PyObject* a = PyObject_GetAttr(v, name);
  if (!a) return nullptr;
  PyObject* s = PyObject_Str(a);
  Py_DECREF(a);
  return s;
}

PyObject* lit(Ctx& c, PyObject* v) {
  if (PyList_Append(c.lits, v) < 0) return nullptr;
  PyObject* dt = str_attr(v, s_dtype);
  if (!dt) return nullptr;
  PyObject* val = PyObject_GetAttr(v, s_value);
  if (!val) {
    Py_DECREF(dt);
    return nullptr;
  }
  PyObject* isnone = val == Py_None ? Py_True : Py_False;
  Py_DECREF(val);
  Py_INCREF(s_L);
  Py_INCREF(isnone);
  PyObject* t = PyTuple_New(3);
  if (!t) return nullptr;
  PyTuple_SET_ITEM(t, 0, s_L);
  PyTuple_SET_ITEM(t, 1, dt);
  PyTuple_SET_ITEM(t, 2, isnone);
  return t;
}

PyObject* attr(Ctx& c, PyObject* v) {
  PyObject* name = PyObject_GetAttr(v, s_name);
  PyObject* dt = name ? str_attr(v, s_dtype) : nullptr;
  PyObject* nul = dt ? PyObject_GetAttr(v, s_nullable) : nullptr;
  PyObject* xid = nul ? PyObject_GetAttr(v, s_expr_id) : nullptr;
  PyObject* e = xid ? eid(c, xid) : nullptr;
  Py_XDECREF(xid);
  PyObject* q = e ? PyObject_GetAttr(v, s_qualifier) : nullptr;
  if (!q) {
    Py_XDECREF(name);
    Py_XDECREF(dt);
    Py_XDECREF(nul);
    Py_XDECREF(e);
    return nullptr;
  }
  PyObject* t = PyTuple_New(6);
  if (!t) return nullptr;
  Py_INCREF(s_A);
  PyTuple_SET_ITEM(t, 0, s_A);
  PyTuple_SET_ITEM(t, 1, name);
  PyTuple_SET_ITEM(t, 2, dt);
  PyTuple_SET_ITEM(t, 3, nul);
  PyTuple_SET_ITEM(t, 4, e);
  PyTuple_SET_ITEM(t, 5, q);
  return t;
}

PyObject* pair(PyObject* k, PyObject* x) {  // steals x
  PyObject* t = PyTuple_New(2);
  if (!t) {
    Py_DECREF(x);
    return nullptr;
  }
  Py_INCREF(k);
  PyTuple_SET_ITEM(t, 0, k);
  PyTuple_SET_ITEM(t, 1, x);
  return t;
}

PyObject* node(Ctx& c, PyObject* v, PyObject* tname) {
  PyObject** dp = _PyObject_GetDictPtr(v);
  if (!dp || !*dp) return PyObject_CallOneArg(c.slow, v);
  PyObject* d = *dp;
  PyObject* names = PyObject_CallOneArg(c.fields, d);
  if (!names) return nullptr;
  if (!PyTuple_Check(names)) {
    Py_DECREF(names);
    PyErr_SetString(PyExc_TypeError, "fields() must return a tuple");
    return nullptr;
  }
  const Py_ssize_t n = PyTuple_GET_SIZE(names);
  PyObject* items = PyTuple_New(n);
  if (!items) {
    Py_DECREF(names);
    return nullptr;
  }
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* k = PyTuple_GET_ITEM(names, i);
    PyObject* x = PyDict_GetItemWithError(d, k);
    if (!x) {
      if (!PyErr_Occurred()) PyErr_SetObject(PyExc_KeyError, k);
      Py_DECREF(items);
      Py_DECREF(names);
      return nullptr;
    }
    const int is_eid = PyUnicode_Compare(k, s_expr_id) == 0;
    PyObject* f = is_eid ? eid(c, x) : fp(c, x);
    PyObject* p = f ? pair(k, f) : nullptr;
    if (!p) {
      Py_DECREF(items);
      Py_DECREF(names);
      return nullptr;
    }
    PyTuple_SET_ITEM(items, i, p);
  }
  Py_DECREF(names);
  PyObject* t = PyTuple_New(2);
  if (!t) {
    Py_DECREF(items);
    return nullptr;
  }
  Py_INCREF(tname);
  PyTuple_SET_ITEM(t, 0, tname);
  PyTuple_SET_ITEM(t, 1, items);
  return t;
}

PyObject* children_node(Ctx& c, PyObject* v, PyObject* tname) {
  PyObject** dp = _PyObject_GetDictPtr(v);
  if (!dp || !*dp || PyDict_GET_SIZE(*dp) != 1) return node(c, v, tname);
  PyObject* ch = PyDict_GetItemWithError(*dp, s_children);
  if (!ch || !PyTuple_CheckExact(ch)) {
    if (PyErr_Occurred()) return nullptr;
    return node(c, v, tname);
  }
  PyObject* f = seq(c, ch);
  if (!f) return nullptr;
  PyObject* p = pair(s_children, f);
  if (!p) return nullptr;
  PyObject* items = PyTuple_New(1);
  if (!items) {
    Py_DECREF(p);
    return nullptr;
  }
  PyTuple_SET_ITEM(items, 0, p);
  PyObject* t = PyTuple_New(2);
  if (!t) {
    Py_DECREF(items);
    return nullptr;
  }
  Py_INCREF(tname);
  PyTuple_SET_ITEM(t, 0, tname);
  PyTuple_SET_ITEM(t, 1, items);
  return t;
}

// a base relation: its memoized fingerprint in local attribute numbering, re-mapped into
// this query's numbering ("LR", fp, eids)
PyObject* leaf(Ctx& c, PyObject* v) {
  PyObject* hit = PyObject_CallOneArg(c.leaf, v);
  if (!hit) return nullptr;
  if (hit == Py_None) {
    Py_DECREF(hit);
    return PyObject_CallOneArg(c.slow, v);
  }
  if (!PyTuple_Check(hit) || PyTuple_GET_SIZE(hit) != 3 ||
      !PyTuple_Check(PyTuple_GET_ITEM(hit, 1)) || !PyTuple_Check(PyTuple_GET_ITEM(hit, 2))) {
    Py_DECREF(hit);
    PyErr_SetString(PyExc_TypeError, "leaf() must return (fp, ids tuple, refs tuple) or None");
    return nullptr;
  }
  PyObject* ids = PyTuple_GET_ITEM(hit, 1);
  PyObject* refs = PyTuple_GET_ITEM(hit, 2);
  for (Py_ssize_t i = 0; i < PyTuple_GET_SIZE(refs); ++i)
    if (PyList_Append(c.refs, PyTuple_GET_ITEM(refs, i)) < 0) {
      Py_DECREF(hit);
      return nullptr;
    }
  const Py_ssize_t n = PyTuple_GET_SIZE(ids);
  PyObject* e = PyTuple_New(n);
  if (!e) {
    Py_DECREF(hit);
    return nullptr;
  }
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* x = eid(c, PyTuple_GET_ITEM(ids, i));
    if (!x) {
      Py_DECREF(e);
      Py_DECREF(hit);
      return nullptr;
    }
    PyTuple_SET_ITEM(e, i, x);
  }
  PyObject* t = PyTuple_New(3);
  if (!t) {
    Py_DECREF(e);
    Py_DECREF(hit);
    return nullptr;
  }
  PyObject* lr = PyUnicode_InternFromString("LR");
  PyObject* f = PyTuple_GET_ITEM(hit, 0);
  Py_INCREF(f);
  PyTuple_SET_ITEM(t, 0, lr);
  PyTuple_SET_ITEM(t, 1, f);
  PyTuple_SET_ITEM(t, 2, e);
  Py_DECREF(hit);
  return t;
}

PyObject* fp(Ctx& c, PyObject* v) {
  PyTypeObject* t = Py_TYPE(v);
  if (t == &PyUnicode_Type || t == &PyLong_Type || t == &PyFloat_Type || t == &PyBool_Type ||
      v == Py_None) {
    Py_INCREF(v);
    return v;
  }
  if (t == &PyTuple_Type || t == &PyList_Type) return seq(c, v);
  PyObject* k = PyDict_GetItemWithError(c.kinds, (PyObject*)t);
  PyObject* owned = nullptr;
  if (!k) {
    if (PyErr_Occurred()) return nullptr;
    owned = PyObject_CallOneArg(c.classify, (PyObject*)t);
    if (!owned) return nullptr;
    k = owned;
  }
  if (!PyTuple_Check(k) || PyTuple_GET_SIZE(k) != 2) {
    Py_XDECREF(owned);
    PyErr_SetString(PyExc_TypeError, "kinds values must be (code, name) tuples");
    return nullptr;
  }
  const long code = PyLong_AsLong(PyTuple_GET_ITEM(k, 0));
  PyObject* tname = PyTuple_GET_ITEM(k, 1);
  Py_INCREF(tname);
  Py_XDECREF(owned);
  PyObject* out;
  if (Py_EnterRecursiveCall(" in plan fingerprint")) {
    Py_DECREF(tname);
    return nullptr;
  }
  switch (code) {
    case 0: out = node(c, v, tname); break;
    case 1: out = lit(c, v); break;
    case 2: out = attr(c, v); break;
    case 3: out = children_node(c, v, tname); break;
    case 5: out = leaf(c, v); break;
    default: out = PyObject_CallOneArg(c.slow, v); break;
  }
  Py_LeaveRecursiveCall();
  Py_DECREF(tname);
  return out;
}

PyObject* py_fingerprint(PyObject*, PyObject* args) {
  Ctx c;
  PyObject* v;
  if (!PyArg_ParseTuple(args, "OO!O!O!O!OOOO", &v, &PyDict_Type, &c.ids, &PyList_Type, &c.lits,
                        &PyList_Type, &c.refs, &PyDict_Type, &c.kinds, &c.classify, &c.fields,
                        &c.slow, &c.leaf))
    return nullptr;
  return fp(c, v);
}

// resolve(expr, names, cs, UnresolvedAttribute, missing): ``expr`` with every
// UnresolvedAttribute replaced by names[name] (names[name.lower()] unless ``cs``), rebuilding
// only the nodes above a replacement through ``with_children``; ``missing(name)`` raises for an
// unknown name (hyperspace_amd/plan/dataframe.py ``_resolve_walk``).
struct Res {
  PyObject* names;
  int cs;
  PyTypeObject* unresolved;
  PyObject* missing;
};

PyObject* s_children_attr;
PyObject* s_with_children;
PyObject* s_lower;

PyObject* resolve(Res& r, PyObject* x) {
  if (PyObject_TypeCheck(x, r.unresolved)) {
    PyObject* name = PyObject_GetAttr(x, s_name);
    if (!name) return nullptr;
    PyObject* key = name;
    if (!r.cs) {
      key = PyObject_CallMethodNoArgs(name, s_lower);
      if (!key) {
        Py_DECREF(name);
        return nullptr;
      }
    }
    PyObject* a = PyDict_GetItemWithError(r.names, key);
    if (key != name) Py_DECREF(key);
    if (a) {
      Py_DECREF(name);
      Py_INCREF(a);
      return a;
    }
    if (!PyErr_Occurred()) {
      PyObject* res = PyObject_CallOneArg(r.missing, name);
      Py_XDECREF(res);
      if (!PyErr_Occurred()) PyErr_SetObject(PyExc_KeyError, name);
    }
    Py_DECREF(name);
    return nullptr;
  }
  PyObject* ch = PyObject_GetAttr(x, s_children_attr);
  if (!ch) return nullptr;
  PyObject* fast = PySequence_Fast(ch, "children must be a sequence");
  Py_DECREF(ch);
  if (!fast) return nullptr;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
  if (n == 0) {
    Py_DECREF(fast);
    Py_INCREF(x);
    return x;
  }
  if (Py_EnterRecursiveCall(" in expression resolution")) {
    Py_DECREF(fast);
    return nullptr;
  }
  PyObject* nt = PyTuple_New(n);
  bool changed = false;
  for (Py_ssize_t i = 0; nt && i < n; ++i) {
    PyObject* c = PySequence_Fast_GET_ITEM(fast, i);
    PyObject* y = resolve(r, c);
    if (!y) {
      Py_CLEAR(nt);
      break;
    }
    changed |= y != c;
    PyTuple_SET_ITEM(nt, i, y);
  }
  Py_LeaveRecursiveCall();
  Py_DECREF(fast);
  if (!nt) return nullptr;
  if (!changed) {
    Py_DECREF(nt);
    Py_INCREF(x);
    return x;
  }
  PyObject* out = PyObject_CallMethodOneArg(x, s_with_children, nt);
  Py_DECREF(nt);
  return out;
}

PyObject* py_resolve(PyObject*, PyObject* args) {
  Res r;
  PyObject* x;
  PyObject* unresolved;
  if (!PyArg_ParseTuple(args, "OO!pO!O", &x, &PyDict_Type, &r.names, &r.cs, &PyType_Type,
                        &unresolved, &r.missing))
    return nullptr;
  r.unresolved = (PyTypeObject*)unresolved;
  return resolve(r, x);
}

PyMethodDef methods[] = {
    {"fingerprint", py_fingerprint, METH_VARARGS,
     "fingerprint(obj, ids, lits, refs, kinds, classify, fields, slow, leaf) -> nested tuple"},
    {"resolve", py_resolve, METH_VARARGS,
     "resolve(expr, names, case_sensitive, UnresolvedAttribute, missing) -> expr"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_hs_host",
                      "Host hot paths of the query front end (plan fingerprint).", -1, methods};

}  // namespace

PyMODINIT_FUNC PyInit__hs_host(void) {
  s_L = PyUnicode_InternFromString("L");
  s_A = PyUnicode_InternFromString("A");
  s_children = PyUnicode_InternFromString("children");
  s_expr_id = PyUnicode_InternFromString("expr_id");
  s_dtype = PyUnicode_InternFromString("dtype");
  s_value = PyUnicode_InternFromString("value");
  s_name = PyUnicode_InternFromString("name");
  s_nullable = PyUnicode_InternFromString("nullable");
  s_qualifier = PyUnicode_InternFromString("qualifier");
  s_children_attr = PyUnicode_InternFromString("children");
  s_with_children = PyUnicode_InternFromString("with_children");
  s_lower = PyUnicode_InternFromString("lower");
  PyObject* m = PyModule_Create(&module);
  // bumped with every signature change: a stale build is ignored (plan_cache._native)
  if (m && PyModule_AddIntConstant(m, "ABI", 2) < 0) {
    Py_DECREF(m);
    return nullptr;
  }
  return m;
}
