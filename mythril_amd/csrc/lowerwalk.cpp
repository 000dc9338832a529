// lowerwalk.cpp — the drop-in lowering's term walk in C++ (CPython extension _lowerwalk).
//
// IncrementalLowering (lower.py) keeps one hash-consed DAG of every term a run has lowered (the
// counterpart of z3's AST table behind the reference's check_quick_sat, support_utils.py:60-67:
// model.eval walks the same terms).  A fresh path's new terms are ~99 % constants, equalities,
// orders, binary bit-vector ops and NOT; this module adds those to the DAG exactly as
// IncrementalLowering._lower does in Python (same postorder, so the same node numbering; the same
// sort checks, hash-consing keys and memo dicts) and calls back into lower.py's _lower_one for
// every other kind.  The Python objects stay the source of truth: the id(term) -> node dict, the
// tape's node / kind lists, its memo dicts and constant pool are the ones lower.py reads.
//
// Term (smt.py) is a __slots__ class: its kind / sort / width / args / params fields are read at
// their slot offsets (taken from the member descriptors once, at bind()).
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <structmember.h>

#include <cstdint>
#include <algorithm>
#include <thread>
#include <cstring>
#include <vector>

// Non-negative int that fits in w bits / its little-endian bytes.  CPython's private long API
// (_PyLong_Sign, _PyLong_NumBits, _PyLong_AsByteArray) changed in 3.13 (_PyLong_AsByteArray gained
// a with_exceptions argument): from 3.13 on the public PyLong_AsNativeBytes is used instead.
static bool long_fits_unsigned(PyObject* v, long w) {
#if PY_VERSION_HEX >= 0x030D0000
  const int neg = PyObject_RichCompareBool(v, Py_False, Py_LT);   // (False == 0)
  if (neg != 0) {
    if (neg < 0) PyErr_Clear();
    return false;
  }
  PyObject* wo = PyLong_FromLong(w);
  PyObject* hi = wo ? PyNumber_Rshift(v, wo) : nullptr;
  Py_XDECREF(wo);
  if (!hi) {
    PyErr_Clear();
    return false;
  }
  const int nz = PyObject_IsTrue(hi);
  Py_DECREF(hi);
  if (nz < 0) PyErr_Clear();
  return nz == 0;
#else
  return _PyLong_Sign(v) >= 0 && _PyLong_NumBits(v) <= (size_t)w;
#endif
}

// v >= 0 into n little-endian bytes (v fits: masked by the caller); 0 on success, -1 on error
static int long_le_bytes(PyObject* v, unsigned char* buf, size_t n) {
#if PY_VERSION_HEX >= 0x030D0000
  const Py_ssize_t need = PyLong_AsNativeBytes(v, buf, (Py_ssize_t)n,
                                               Py_ASNATIVEBYTES_LITTLE_ENDIAN | Py_ASNATIVEBYTES_UNSIGNED_BUFFER);
  if (need < 0) return -1;
  if ((size_t)need > n) {
    PyErr_SetString(PyExc_OverflowError, "lowerwalk: constant wider than its width");
    return -1;
  }
  return 0;
#else
  return _PyLong_AsByteArray((PyLongObject*)v, buf, n, 1, 0);
#endif
}

namespace {

struct State {
  PyObject* node;        // dict id(term) -> DAG node
  PyObject* keep;        // dict id(term) -> term
  PyObject* bad;         // dict id(root) -> (root, reason)
  PyObject* nodes;       // list of (op, width, a, b, c)
  PyObject* kinds;       // list of "bool" / "bv" / "array"
  PyObject* memo;        // dict key -> node
  PyObject* cmemo;       // dict (value, width) -> constant pool offset
  PyObject* consts;      // list of u32 words
  PyObject* kind_code;   // dict term kind -> 1 VAL, 2 NOT, 3 binary BV op, 4 predicate
  PyObject* fast_bin;    // dict term kind -> Op
  PyObject* fast_pred;   // dict term kind -> Op
  PyObject* lower_one;   // lower._lower_one(t, arg_nodes, tape, syms, node)
  PyObject* to_words;    // tape.to_words(value, width)
  PyObject* tape;
  PyObject* syms;
  PyObject* lowering_error;
  PyObject* sort_error;
  PyObject* k_and;       // smt.AND
  PyObject* k_eq;        // smt.EQ
  PyObject* s_bv;        // "bv"
  PyObject* s_bool;      // "bool"
  PyObject* op_const;
  PyObject* op_not;
  long max_width;
  PyObject* false_fn;    // tape.false: called at each failing root (the Python loop's node numbering)
};

Py_ssize_t off_kind = -1, off_sort, off_width, off_args, off_params;

inline PyObject* slot(PyObject* t, Py_ssize_t off) { return *(PyObject**)((char*)t + off); }

int slot_offset(PyObject* type, const char* name, Py_ssize_t* out) {
  PyObject* d = PyObject_GetAttrString(type, name);
  if (!d) return -1;
  if (Py_TYPE(d) != &PyMemberDescr_Type) {
    Py_DECREF(d);
    PyErr_Format(PyExc_TypeError, "Term.%s is not a slot", name);
    return -1;
  }
  *out = ((PyMemberDescrObject*)d)->d_member->offset;
  Py_DECREF(d);
  return 0;
}

inline bool str_eq(PyObject* a, PyObject* b) {
  return a == b || (PyUnicode_Check(a) && PyUnicode_Compare(a, b) == 0);
}

// *out = node[id(t)]: 1 found, 0 absent, -1 error (a node value may itself be negative)
inline int node_lookup(const State& s, PyObject* t, long* out) {
  PyObject* k = PyLong_FromVoidPtr(t);
  if (!k) return -1;
  PyObject* v = PyDict_GetItemWithError(s.node, k);
  Py_DECREF(k);
  if (!v) return PyErr_Occurred() ? -1 : 0;
  *out = PyLong_AsLong(v);
  return (*out == -1 && PyErr_Occurred()) ? -1 : 1;
}

PyObject* key5(PyObject* op, PyObject* w, long a, long b) {
  PyObject* t = PyTuple_New(5);
  if (!t) return nullptr;
  Py_INCREF(op);
  PyTuple_SET_ITEM(t, 0, op);
  Py_INCREF(w);
  PyTuple_SET_ITEM(t, 1, w);
  PyTuple_SET_ITEM(t, 2, PyLong_FromLong(a));
  PyTuple_SET_ITEM(t, 3, PyLong_FromLong(b));
  PyTuple_SET_ITEM(t, 4, PyLong_FromLong(0));
  for (int i = 2; i < 5; i++)
    if (!PyTuple_GET_ITEM(t, i)) { Py_DECREF(t); return nullptr; }
  return t;
}

// The DAG node of a fast-kind term whose arguments are lowered: a new reference to the node
// index, Py_None when the term needs _lower_one, nullptr on error.
PyObject* fast_node(const State& s, PyObject* t, long code, PyObject* k, const long* an, Py_ssize_t na) {
  PyObject* key = nullptr;
  PyObject* kind = nullptr;
  if (code == 1) {   // VAL
    PyObject* wo = slot(t, off_width);
    const long w = PyLong_AsLong(wo);
    if (w == -1 && PyErr_Occurred()) return nullptr;
    if (!(0 < w && w <= s.max_width)) Py_RETURN_NONE;
    PyObject* params = slot(t, off_params);
    if (!PyTuple_Check(params) || PyTuple_GET_SIZE(params) < 1) Py_RETURN_NONE;
    // v = params[0] & ((1 << w) - 1)
    PyObject* p0 = PyTuple_GET_ITEM(params, 0);
    PyObject* v;
    if (PyLong_CheckExact(p0) && long_fits_unsigned(p0, w)) {
      Py_INCREF(p0);
      v = p0;
    } else {
      PyObject* one = PyLong_FromLong(1);
      if (!one) return nullptr;
      PyObject* sh = PyNumber_Lshift(one, wo);
      PyObject* mask = sh ? PyNumber_Subtract(sh, one) : nullptr;
      Py_DECREF(one);
      Py_XDECREF(sh);
      if (!mask) return nullptr;
      v = PyNumber_And(p0, mask);
      Py_DECREF(mask);
      if (!v) return nullptr;
    }
    PyObject* ck = PyTuple_Pack(2, v, wo);
    if (!ck) { Py_DECREF(v); return nullptr; }
    PyObject* off = PyDict_GetItemWithError(s.cmemo, ck);
    if (off) {
      Py_INCREF(off);
    } else {
      if (PyErr_Occurred()) { Py_DECREF(ck); Py_DECREF(v); return nullptr; }
      // the constant's little-endian u32 words into the pool (tape.to_words; v is masked, >= 0)
      off = PyLong_FromSsize_t(PyList_GET_SIZE(s.consts));
      const size_t nw = (size_t)(w + 31) / 32;
      std::vector<unsigned char> buf(nw * 4);
      int rc = off ? long_le_bytes(v, buf.data(), buf.size()) : -1;
      for (size_t i = 0; rc == 0 && i < nw; i++) {
        const unsigned long x = (unsigned long)buf[4 * i] | ((unsigned long)buf[4 * i + 1] << 8) |
                                ((unsigned long)buf[4 * i + 2] << 16) | ((unsigned long)buf[4 * i + 3] << 24);
        PyObject* o = PyLong_FromUnsignedLong(x);
        rc = o ? PyList_Append(s.consts, o) : -1;
        Py_XDECREF(o);
      }
      if (rc < 0 || PyDict_SetItem(s.cmemo, ck, off) < 0) {
        Py_XDECREF(off); Py_DECREF(ck); Py_DECREF(v);
        return nullptr;
      }
    }
    Py_DECREF(ck);
    Py_DECREF(v);
    const long o = PyLong_AsLong(off);
    Py_DECREF(off);
    key = key5(s.op_const, wo, o, 0);
    kind = s.s_bv;
  } else if (code == 3 || code == 4) {   // binary BV op / predicate
    if (na < 2) Py_RETURN_NONE;
    const long a = an[0], b = an[1];
    if (a < 0 || b < 0 || a >= PyList_GET_SIZE(s.kinds) || b >= PyList_GET_SIZE(s.kinds)) Py_RETURN_NONE;
    if (!str_eq(PyList_GET_ITEM(s.kinds, a), s.s_bv) || !str_eq(PyList_GET_ITEM(s.kinds, b), s.s_bv)) Py_RETURN_NONE;
    PyObject* ta = PyList_GET_ITEM(s.nodes, a);
    PyObject* tb = PyList_GET_ITEM(s.nodes, b);
    if (!PyTuple_Check(ta) || !PyTuple_Check(tb) || PyTuple_GET_SIZE(ta) < 2 || PyTuple_GET_SIZE(tb) < 2) Py_RETURN_NONE;
    PyObject* wa = PyTuple_GET_ITEM(ta, 1);
    PyObject* wb = PyTuple_GET_ITEM(tb, 1);
    const int ne = PyObject_RichCompareBool(wb, wa, Py_NE);
    if (ne < 0) return nullptr;
    if (ne) {
      PyErr_Format(s.sort_error, "width mismatch %S vs %S", wa, wb);
      return nullptr;
    }
    if (code == 3) {
      PyObject* op = PyDict_GetItemWithError(s.fast_bin, k);
      if (!op) return PyErr_Occurred() ? nullptr : (Py_INCREF(Py_None), Py_None);
      key = key5(op, wa, a, b);
      kind = s.s_bv;
    } else {
      if (str_eq(k, s.k_eq) && PyLong_AsLong(wa) > 256) Py_RETURN_NONE;   // (wider equalities: _wide_eq)
      PyObject* op = PyDict_GetItemWithError(s.fast_pred, k);
      if (!op) return PyErr_Occurred() ? nullptr : (Py_INCREF(Py_None), Py_None);
      PyObject* zero = PyLong_FromLong(0);
      if (!zero) return nullptr;
      key = key5(op, zero, a, b);
      Py_DECREF(zero);
      kind = s.s_bool;
    }
  } else if (code == 2) {   // NOT
    if (na < 1) Py_RETURN_NONE;
    const long a = an[0];
    if (a < 0 || a >= PyList_GET_SIZE(s.kinds) || !str_eq(PyList_GET_ITEM(s.kinds, a), s.s_bool)) Py_RETURN_NONE;
    PyObject* zero = PyLong_FromLong(0);
    if (!zero) return nullptr;
    key = key5(s.op_not, zero, a, 0);
    Py_DECREF(zero);
    kind = s.s_bool;
  } else {
    Py_RETURN_NONE;
  }
  if (!key) return nullptr;
  PyObject* r = PyDict_GetItemWithError(s.memo, key);
  if (r) {
    Py_INCREF(r);
    Py_DECREF(key);
    return r;
  }
  if (PyErr_Occurred()) { Py_DECREF(key); return nullptr; }
  r = PyLong_FromSsize_t(PyList_GET_SIZE(s.nodes));
  if (!r || PyList_Append(s.nodes, key) < 0 || PyList_Append(s.kinds, kind) < 0 || PyDict_SetItem(s.memo, key, r) < 0) {
    Py_XDECREF(r);
    Py_DECREF(key);
    return nullptr;
  }
  Py_DECREF(key);
  return r;
}

// _lower_one(t, [node.get(id(x), -1) for x in args], tape, syms, node)
PyObject* slow_node(const State& s, PyObject* t) {
  PyObject* args = slot(t, off_args);
  const Py_ssize_t n = PyTuple_Check(args) ? PyTuple_GET_SIZE(args) : 0;
  PyObject* lst = PyList_New(n);
  if (!lst) return nullptr;
  for (Py_ssize_t i = 0; i < n; i++) {
    long v = -1;
    if (node_lookup(s, PyTuple_GET_ITEM(args, i), &v) < 0) { Py_DECREF(lst); return nullptr; }
    PyObject* o = PyLong_FromLong(v);
    if (!o) { Py_DECREF(lst); return nullptr; }
    PyList_SET_ITEM(lst, i, o);
  }
  PyObject* r = PyObject_CallFunctionObjArgs(s.lower_one, t, lst, s.tape, s.syms, s.node, nullptr);
  Py_DECREF(lst);
  return r;
}

// IncrementalLowering._lower(root) without its bad-root bookkeeping: *out = the DAG node of root
// (lowering the terms not seen before); returns -1 with a Python exception set on failure.  A term is
// lowered when it is on top of the stack with every argument lowered, else its unlowered
// arguments go on top (last argument pushed first): the Python loop's postorder.
int walk(const State& s, PyObject* root, std::vector<PyObject*>& stack, long* out) {
  stack.clear();
  stack.push_back(root);
  long an[3];
  while (!stack.empty()) {
    PyObject* t = stack.back();
    PyObject* tk = PyLong_FromVoidPtr(t);
    if (!tk) return -1;
    const int have = PyDict_Contains(s.node, tk);
    if (have) {
      Py_DECREF(tk);
      if (have < 0) return -1;
      stack.pop_back();
      continue;
    }
    PyObject* args = slot(t, off_args);
    const Py_ssize_t na = PyTuple_Check(args) ? PyTuple_GET_SIZE(args) : 0;
    bool pending = false;
    for (Py_ssize_t i = na - 1; i >= 0; i--) {
      PyObject* x = PyTuple_GET_ITEM(args, i);
      long v = 0;
      const int f = node_lookup(s, x, &v);
      if (f < 0) { Py_DECREF(tk); return -1; }
      if (!f) {
        stack.push_back(x);
        pending = true;
      } else if (i < 3) {
        an[i] = v;
      }
    }
    if (pending) { Py_DECREF(tk); continue; }
    stack.pop_back();
    PyObject* k = slot(t, off_kind);
    PyObject* c = PyDict_GetItemWithError(s.kind_code, k);
    if (!c && PyErr_Occurred()) { Py_DECREF(tk); return -1; }
    const long code = c ? PyLong_AsLong(c) : 0;
    PyObject* r = code ? fast_node(s, t, code, k, an, na) : (Py_INCREF(Py_None), Py_None);
    if (r == Py_None) {
      Py_DECREF(r);
      r = slow_node(s, t);
    }
    if (!r) { Py_DECREF(tk); return -1; }
    int rc = PyDict_SetItem(s.node, tk, r);
    if (rc == 0) rc = PyDict_SetItem(s.keep, tk, t);
    Py_DECREF(tk);
    Py_DECREF(r);
    if (rc < 0) return -1;
  }
  const int f = node_lookup(s, root, out);
  if (f < 0) return -1;
  if (!f) { PyErr_SetString(PyExc_RuntimeError, "lowerwalk: root not lowered"); return -1; }
  return 0;
}

bool parse_state(PyObject* st, State& s) {
  if (!PyTuple_Check(st) || PyTuple_GET_SIZE(st) != 25) {
    PyErr_SetString(PyExc_TypeError, "lowering state: a 25-tuple");
    return false;
  }
  PyObject** f = &PyTuple_GET_ITEM(st, 0);
  s.node = f[0]; s.keep = f[1]; s.bad = f[2]; s.nodes = f[3]; s.kinds = f[4]; s.memo = f[5];
  s.cmemo = f[6]; s.consts = f[7]; s.kind_code = f[8]; s.fast_bin = f[9]; s.fast_pred = f[10];
  s.lower_one = f[11]; s.to_words = f[12]; s.tape = f[13]; s.syms = f[14]; s.lowering_error = f[15];
  s.sort_error = f[16]; s.k_and = f[17]; s.k_eq = f[18]; s.s_bv = f[19]; s.s_bool = f[20];
  s.op_const = f[21]; s.op_not = f[22];
  s.max_width = PyLong_AsLong(f[23]);
  s.false_fn = f[24];
  if (!PyDict_Check(s.node) || !PyDict_Check(s.keep) || !PyDict_Check(s.bad) || !PyList_Check(s.nodes) ||
      !PyList_Check(s.kinds) || !PyDict_Check(s.memo) || !PyDict_Check(s.cmemo) || !PyList_Check(s.consts) ||
      !PyDict_Check(s.kind_code) || !PyDict_Check(s.fast_bin) || !PyDict_Check(s.fast_pred)) {
    PyErr_SetString(PyExc_TypeError, "lowering state: unexpected container types");
    return false;
  }
  return !PyErr_Occurred();
}

// bind(Term): slot offsets of the term class
PyObject* py_bind(PyObject*, PyObject* type) {
  if (slot_offset(type, "kind", &off_kind) || slot_offset(type, "sort", &off_sort) ||
      slot_offset(type, "width", &off_width) || slot_offset(type, "args", &off_args) ||
      slot_offset(type, "params", &off_params)) {
    off_kind = -1;
    return nullptr;
  }
  Py_RETURN_NONE;
}

// lower_roots(roots, state) -> list, per root: the list of its conjuncts' DAG nodes, or the
// exception (LoweringError / TypeError) its first failing conjunct raised (recorded in bad as
// IncrementalLowering._lower does).  Raises LoweringError for a non-Bool root.
PyObject* py_lower_roots(PyObject*, PyObject* a) {
  PyObject *roots, *st;
  if (!PyArg_ParseTuple(a, "OO", &roots, &st)) return nullptr;
  if (off_kind < 0) {
    PyErr_SetString(PyExc_RuntimeError, "_lowerwalk.bind(Term) was not called");
    return nullptr;
  }
  State s;
  if (!parse_state(st, s)) return nullptr;
  PyObject* seq = PySequence_Fast(roots, "roots: a sequence");
  if (!seq) return nullptr;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  PyObject* out = PyList_New(n);
  if (!out) { Py_DECREF(seq); return nullptr; }
  std::vector<PyObject*> stack;
  stack.reserve(256);
  // the walk allocates a burst of key tuples: no cyclic collection in the middle of it (a
  // full collection traverses every term of the run); the collector runs again afterwards
  struct GcPause {
    int was = PyGC_Disable();
    ~GcPause() { if (was) PyGC_Enable(); }
  } gc_pause;
  for (Py_ssize_t i = 0; i < n; i++) {
    PyObject* r = PySequence_Fast_GET_ITEM(seq, i);
    if (!str_eq(slot(r, off_sort), s.s_bool)) {
      PyErr_SetString(s.lowering_error, "quick-sat root must be Bool");
      Py_DECREF(out); Py_DECREF(seq);
      return nullptr;
    }
    PyObject* rargs = slot(r, off_args);
    const bool is_and = str_eq(slot(r, off_kind), s.k_and) && PyTuple_Check(rargs);
    const Py_ssize_t nc = is_and ? PyTuple_GET_SIZE(rargs) : 1;
    PyObject* ids = PyList_New(nc);
    if (!ids) { Py_DECREF(out); Py_DECREF(seq); return nullptr; }
    PyObject* fail = nullptr;
    for (Py_ssize_t j = 0; j < nc && !fail; j++) {
      PyObject* c = is_and ? PyTuple_GET_ITEM(rargs, j) : r;
      long v = 0;
      const int found = node_lookup(s, c, &v);
      if (found < 0) { Py_DECREF(ids); Py_DECREF(out); Py_DECREF(seq); return nullptr; }
      if (!found) {
        PyObject* key = PyLong_FromVoidPtr(c);
        PyObject* b = key ? PyDict_GetItemWithError(s.bad, key) : nullptr;
        Py_XDECREF(key);
        if (b) {
          fail = PyObject_CallFunctionObjArgs(s.lowering_error, PyTuple_GET_ITEM(b, 1), nullptr);
          if (!fail) { Py_DECREF(ids); Py_DECREF(out); Py_DECREF(seq); return nullptr; }
          break;
        }
        if (PyErr_Occurred()) { Py_DECREF(ids); Py_DECREF(out); Py_DECREF(seq); return nullptr; }
        if (walk(s, c, stack, &v) < 0) {
          // (LoweringError, TypeError): the conjunct fails closed; anything else propagates
          if (!PyErr_ExceptionMatches(PyExc_TypeError)) { Py_DECREF(ids); Py_DECREF(out); Py_DECREF(seq); return nullptr; }
          PyObject *et, *ev, *tb;
          PyErr_Fetch(&et, &ev, &tb);
          PyErr_NormalizeException(&et, &ev, &tb);
          PyObject* msg = ev ? PyObject_Str(ev) : nullptr;
          Py_XDECREF(et); Py_XDECREF(ev); Py_XDECREF(tb);
          if (msg && PyUnicode_GET_LENGTH(msg) == 0) {
            Py_DECREF(msg);
            msg = PyUnicode_FromString("conjunct not in the tape vocabulary");
          }
          PyObject* rec = msg ? PyTuple_Pack(2, c, msg) : nullptr;
          PyObject* key = rec ? PyLong_FromVoidPtr(c) : nullptr;
          const int rc = key ? PyDict_SetItem(s.bad, key, rec) : -1;
          Py_XDECREF(key); Py_XDECREF(rec);
          fail = rc == 0 ? PyObject_CallFunctionObjArgs(s.lowering_error, msg, nullptr) : nullptr;
          Py_XDECREF(msg);
          if (!fail) { Py_DECREF(ids); Py_DECREF(out); Py_DECREF(seq); return nullptr; }
          break;
        }
      }
      PyObject* o = PyLong_FromLong(v);
      if (!o) { Py_DECREF(ids); Py_DECREF(out); Py_DECREF(seq); return nullptr; }
      PyList_SET_ITEM(ids, j, o);
    }
    if (fail) {
      Py_DECREF(ids);
      PyList_SET_ITEM(out, i, fail);
      // the Python loop adds the FALSE placeholder when the root fails, before the next root
      PyObject* fn = PyObject_CallNoArgs(s.false_fn);
      if (!fn) { Py_DECREF(out); Py_DECREF(seq); return nullptr; }
      Py_DECREF(fn);
    } else {
      PyList_SET_ITEM(out, i, ids);
    }
  }
  Py_DECREF(seq);
  return out;
}

// pack_nodes(nodes, start, end, out): nodes[start:end] (5-tuples of ints) into the writable
// buffer out as tape.NODE_DTYPE records (u16 op, u16 width, u32 a, b, c; values wrap like
// numpy's casts) — IncrementalLowering._sync's numpy mirror of the node table.
PyObject* py_pack_nodes(PyObject*, PyObject* a) {
  PyObject* nodes;
  Py_ssize_t start, end;
  Py_buffer out;
  if (!PyArg_ParseTuple(a, "Onnw*", &nodes, &start, &end, &out)) return nullptr;
  if (!PyList_Check(nodes) || start < 0 || end > PyList_GET_SIZE(nodes) || start > end ||
      out.len < (end - start) * 16) {
    PyBuffer_Release(&out);
    PyErr_SetString(PyExc_ValueError, "pack_nodes: bad range or buffer");
    return nullptr;
  }
  unsigned char* p = (unsigned char*)out.buf;
  for (Py_ssize_t i = start; i < end; i++, p += 16) {
    PyObject* t = PyList_GET_ITEM(nodes, i);
    if (!PyTuple_Check(t) || PyTuple_GET_SIZE(t) != 5) {
      PyBuffer_Release(&out);
      PyErr_SetString(PyExc_TypeError, "pack_nodes: a node is not a 5-tuple");
      return nullptr;
    }
    unsigned long v[5];
    for (int j = 0; j < 5; j++) {
      v[j] = PyLong_AsUnsignedLongMask(PyTuple_GET_ITEM(t, j));
      if (v[j] == (unsigned long)-1 && PyErr_Occurred()) {
        PyBuffer_Release(&out);
        return nullptr;
      }
    }
    const uint16_t op = (uint16_t)v[0], w = (uint16_t)v[1];
    const uint32_t abc[3] = {(uint32_t)v[2], (uint32_t)v[3], (uint32_t)v[4]};
    std::memcpy(p, &op, 2);
    std::memcpy(p + 2, &w, 2);
    std::memcpy(p + 4, abc, 12);
  }
  PyBuffer_Release(&out);
  Py_RETURN_NONE;
}

// candidate_rows(gen, lru, src, starts, patches, var_off, var_limbs): the generated candidates'
// variable rows (candidates.py CandidateGenerator._serialize).  gen: writable u32 [R, K] (rows may
// be strided: the candidates' columns of the whole batch's rows); lru: u32
// [R, n_lru] (the LRU's rows); src: i64 [K] base model of each candidate; starts: i64 [B + 1]
// block column ranges; patches: B tuples of (var, lo, n_bits, bits) applied in order over their
// block (value assignments; lo < 0: a size floor "var >= bits when var < 2^32", applied after the
// block's values); var_off / var_limbs: i64 [V] first row and limb count of each variable.
struct Buf {
  Py_buffer b{};
  bool ok = false;
  ~Buf() { if (ok) PyBuffer_Release(&b); }
};

static bool get_buf(PyObject* o, Buf& out, bool writable, Py_ssize_t itemsize, const char* what, bool strided = false) {
  const int flags = (writable ? PyBUF_WRITABLE : 0) | (strided ? PyBUF_STRIDES : PyBUF_C_CONTIGUOUS) | PyBUF_FORMAT;
  if (PyObject_GetBuffer(o, &out.b, flags) < 0) return false;
  out.ok = true;
  if (out.b.itemsize != itemsize) {
    PyErr_Format(PyExc_TypeError, "candidate_rows: %s has item size %zd, not %zd", what, out.b.itemsize, itemsize);
    return false;
  }
  return true;
}

// bits [b0, b0 + n) (n <= 32) of the little-endian word array w
static inline uint32_t bits_at(const std::vector<uint32_t>& w, int64_t b0, int n) {
  const size_t i = (size_t)(b0 >> 5);
  const int sh = (int)(b0 & 31);
  uint64_t x = i < w.size() ? w[i] : 0;
  if (i + 1 < w.size()) x |= (uint64_t)w[i + 1] << 32;
  x >>= sh;
  return (uint32_t)(x & (n >= 32 ? 0xFFFFFFFFull : ((1ull << n) - 1)));
}

PyObject* py_candidate_rows(PyObject*, PyObject* a) {
  PyObject *o_gen, *o_lru, *o_src, *o_starts, *patches, *o_off, *o_nl;
  if (!PyArg_ParseTuple(a, "OOOOOOO", &o_gen, &o_lru, &o_src, &o_starts, &patches, &o_off, &o_nl)) return nullptr;
  Buf gen, lru, src, starts, off, nl;
  if (!get_buf(o_gen, gen, true, 4, "gen", true) || !get_buf(o_lru, lru, false, 4, "lru") ||
      !get_buf(o_src, src, false, 8, "src") || !get_buf(o_starts, starts, false, 8, "starts") ||
      !get_buf(o_off, off, false, 8, "var_off") || !get_buf(o_nl, nl, false, 8, "var_limbs"))
    return nullptr;
  if (gen.b.ndim != 2 || lru.b.ndim != 2 || gen.b.shape[0] != lru.b.shape[0] || !PyList_Check(patches) ||
      gen.b.strides[1] != 4 || gen.b.strides[0] % 4 != 0 || gen.b.strides[0] < 4 * gen.b.shape[1]) {
    PyErr_SetString(PyExc_ValueError, "candidate_rows: shapes");
    return nullptr;
  }
  uint32_t* G = (uint32_t*)gen.b.buf;
  const uint32_t* L = (const uint32_t*)lru.b.buf;
  const int64_t* S = (const int64_t*)src.b.buf;
  const int64_t* ST = (const int64_t*)starts.b.buf;
  const int64_t* VO = (const int64_t*)off.b.buf;
  const int64_t* VL = (const int64_t*)nl.b.buf;
  const Py_ssize_t R = gen.b.shape[0], K = gen.b.shape[1], NL = lru.b.shape[1], GS = gen.b.strides[0] / 4;
  const Py_ssize_t B = PyList_GET_SIZE(patches), V = off.b.len / 8;
  if (src.b.len / 8 != K || starts.b.len / 8 != B + 1 || nl.b.len / 8 != V || (NL == 0 && K > 0 && R > 0)) {
    PyErr_SetString(PyExc_ValueError, "candidate_rows: sizes");
    return nullptr;
  }
  for (Py_ssize_t k = 0; k < K; k++)
    if (S[k] < 0 || S[k] >= NL) {
      PyErr_SetString(PyExc_ValueError, "candidate_rows: base index out of range");
      return nullptr;
    }
  // pass 1 (holding the GIL): every block's updates as plain records — (row, keep mask, bits) for
  // the value assignments, (first row, limbs, minimum) for the floors
  struct Up { int64_t row; uint32_t mask, val; };
  struct Fl { int64_t r0, nl; uint32_t mn; };
  std::vector<int64_t> up_off(B + 1, 0), fl_off(B + 1, 0);
  std::vector<Up> ups;
  std::vector<Fl> fls;
  std::vector<uint32_t> words;
  for (Py_ssize_t j = 0; j < B; j++) {
    const int64_t c0 = ST[j], c1 = ST[j + 1];
    if (c0 < 0 || c1 > K || c0 > c1) {
      PyErr_SetString(PyExc_ValueError, "candidate_rows: block range");
      return nullptr;
    }
    PyObject* patch = PyList_GET_ITEM(patches, j);
    if (!PyTuple_Check(patch)) {
      PyErr_SetString(PyExc_TypeError, "candidate_rows: a patch is not a tuple");
      return nullptr;
    }
    for (Py_ssize_t e = 0; e < PyTuple_GET_SIZE(patch); e++) {
      PyObject* el = PyTuple_GET_ITEM(patch, e);
      if (!PyTuple_Check(el) || PyTuple_GET_SIZE(el) != 4) {
        PyErr_SetString(PyExc_TypeError, "candidate_rows: a patch element is not a 4-tuple");
        return nullptr;
      }
      const long v = PyLong_AsLong(PyTuple_GET_ITEM(el, 0));
      const long lo = PyLong_AsLong(PyTuple_GET_ITEM(el, 1));
      const long n = PyLong_AsLong(PyTuple_GET_ITEM(el, 2));
      if (PyErr_Occurred()) return nullptr;
      if (v < 0 || v >= V || VO[v] < 0 || VO[v] + VL[v] > R) {
        PyErr_SetString(PyExc_ValueError, "candidate_rows: variable out of range");
        return nullptr;
      }
      PyObject* bits = PyTuple_GET_ITEM(el, 3);
      if (lo < 0) {   // size >= minimum (values < 2^32 in their low limb)
        const unsigned long mn = PyLong_AsUnsignedLongMask(bits);
        if (PyErr_Occurred()) return nullptr;
        fls.push_back(Fl{VO[v], VL[v], (uint32_t)mn});
        continue;
      }
      if (n <= 0) continue;
      if (!PyLong_Check(bits) || !long_fits_unsigned(bits, n)) {
        PyErr_SetString(PyExc_ValueError, "candidate_rows: assignment bits wider than the field");
        return nullptr;
      }
      words.assign((size_t)(n + 31) / 32 + 1, 0u);
      if (long_le_bytes(bits, (unsigned char*)words.data(), words.size() * 4) < 0) return nullptr;
      for (long i = lo / 32; i <= (lo + n - 1) / 32 && i < VL[v]; i++) {
        const long blo = 32 * i, aa = std::max(lo, blo), bb = std::min(lo + n, blo + 32);
        if (aa >= bb) continue;
        const uint32_t mask = (uint32_t)((bb - aa >= 32 ? 0xFFFFFFFFull : ((1ull << (bb - aa)) - 1)) << (aa - blo));
        ups.push_back(Up{VO[v] + i, ~mask, (bits_at(words, aa - lo, (int)(bb - aa)) << (aa - blo)) & mask});
      }
    }
    up_off[j + 1] = (int64_t)ups.size();
    fl_off[j + 1] = (int64_t)fls.size();
  }
  // pass 2 (GIL released): blocks are disjoint column ranges, so threads take ranges of blocks;
  // each copies its candidates' base rows, then applies its blocks' values, then their floors
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const int64_t work = (int64_t)R * K;
  const int nt = (int)std::min<int64_t>({(int64_t)std::min(8u, hw), std::max<int64_t>(1, work / (1 << 20)), std::max<Py_ssize_t>(B, 1)});
  auto run = [&](int64_t b0, int64_t b1) {
    if (b0 >= b1) return;
    const int64_t k0 = ST[b0], k1 = ST[b1];
    for (Py_ssize_t r = 0; r < R; r++) {
      uint32_t* g = G + r * GS;
      const uint32_t* l = L + r * NL;
      for (int64_t k = k0; k < k1; k++) g[k] = l[S[k]];
    }
    for (int64_t j = b0; j < b1; j++) {
      const int64_t c0 = ST[j], c1 = ST[j + 1];
      for (int64_t u = up_off[j]; u < up_off[j + 1]; u++) {
        uint32_t* g = G + ups[u].row * GS;
        const uint32_t keep = ups[u].mask, val = ups[u].val;
        for (int64_t k = c0; k < c1; k++) g[k] = (g[k] & keep) | val;
      }
      for (int64_t f = fl_off[j]; f < fl_off[j + 1]; f++) {
        uint32_t* g0 = G + fls[f].r0 * GS;
        for (int64_t k = c0; k < c1; k++) {
          bool small = true;
          for (int64_t q = 1; q < fls[f].nl && small; q++) small = G[(fls[f].r0 + q) * GS + k] == 0;
          if (small && g0[k] < fls[f].mn) g0[k] = fls[f].mn;
        }
      }
    }
  };
  Py_BEGIN_ALLOW_THREADS
  if (nt <= 1) {
    run(0, B);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; t++) th.emplace_back(run, (int64_t)B * t / nt, (int64_t)B * (t + 1) / nt);
    for (auto& x : th) x.join();
  }
  Py_END_ALLOW_THREADS
  Py_RETURN_NONE;
}

// conj_rows(roots, row_of, n_rows, R, slots, rows_out) -> (n_rows, todo): ConjunctRows' bookkeeping
// for one query batch (support.py VerdictEngine._rows_incremental).  roots: u32 [n] conjunct DAG
// nodes of the batch's queries, back to back; row_of: i64 [> max node] node -> row (-1: none),
// new rows numbered in first-appearance order from n_rows; R: i8 [rows cap, slot cap] verdicts
// (-1 unknown); slots: i64 [s] the candidate models' slots.  rows_out: i64 [n] each root's row.
// todo: the distinct nodes (first-appearance order) with an unknown verdict under some slot.
PyObject* py_conj_rows(PyObject*, PyObject* a) {
  PyObject *o_roots, *o_row_of, *o_R, *o_slots, *o_out;
  long long n_rows;
  if (!PyArg_ParseTuple(a, "OOLOOO", &o_roots, &o_row_of, &n_rows, &o_R, &o_slots, &o_out)) return nullptr;
  Buf roots, row_of, R, slots, out;
  if (!get_buf(o_roots, roots, false, 4, "roots") || !get_buf(o_row_of, row_of, true, 8, "row_of") ||
      !get_buf(o_R, R, true, 1, "R") || !get_buf(o_slots, slots, false, 8, "slots") ||
      !get_buf(o_out, out, true, 8, "rows_out"))
    return nullptr;
  const Py_ssize_t n = roots.b.len / 4, nro = row_of.b.len / 8, ns = slots.b.len / 8;
  if (R.b.ndim != 2 || out.b.len / 8 != n) {
    PyErr_SetString(PyExc_ValueError, "conj_rows: shapes");
    return nullptr;
  }
  const Py_ssize_t rcap = R.b.shape[0], scap = R.b.shape[1];
  const uint32_t* rt = (const uint32_t*)roots.b.buf;
  int64_t* ro = (int64_t*)row_of.b.buf;
  int8_t* RR = (int8_t*)R.b.buf;
  const int64_t* sl = (const int64_t*)slots.b.buf;
  int64_t* rows = (int64_t*)out.b.buf;
  for (Py_ssize_t j = 0; j < ns; j++)
    if (sl[j] < 0 || sl[j] >= scap) {
      PyErr_SetString(PyExc_ValueError, "conj_rows: slot beyond R");
      return nullptr;
    }
  PyObject* todo = PyList_New(0);
  if (!todo) return nullptr;
  for (Py_ssize_t i = 0; i < n; i++) {
    const uint32_t node = rt[i];
    if ((Py_ssize_t)node >= nro) {
      Py_DECREF(todo);
      PyErr_SetString(PyExc_ValueError, "conj_rows: node beyond row_of");
      return nullptr;
    }
    int64_t r = ro[node];
    bool fresh = false;
    if (r < 0) {
      if (n_rows >= rcap) {
        Py_DECREF(todo);
        PyErr_SetString(PyExc_ValueError, "conj_rows: R has too few rows");
        return nullptr;
      }
      r = ro[node] = n_rows++;
      fresh = true;   // (a new row is all unknown; its node is listed once, here)
    }
    rows[i] = r;
    bool unknown = fresh;
    if (!fresh) {
      // listed already when a row seen earlier in this batch was unknown: mark with -2 below
      const int8_t* rr = RR + r * scap;
      for (Py_ssize_t j = 0; j < ns && !unknown; j++) unknown = rr[sl[j]] < 0;
      if (unknown && rr[sl[0]] == -2) unknown = false;
    }
    if (unknown) {
      PyObject* o = PyLong_FromUnsignedLong(node);
      if (!o || PyList_Append(todo, o) < 0) {
        Py_XDECREF(o);
        Py_DECREF(todo);
        return nullptr;
      }
      Py_DECREF(o);
      if (ns) RR[r * scap + sl[0]] = -2;   // (a transient "listed" mark: still unknown)
    }
  }
  // clear the transient marks (they stay unknown, -1, until the caller writes the verdicts)
  for (Py_ssize_t i = 0; i < n && ns; i++) {
    int8_t* v = RR + rows[i] * scap + sl[0];
    if (*v == -2) *v = -1;
  }
  return Py_BuildValue("(LN)", n_rows, todo);
}

// conj_answer(R, rows, offsets, slots, out): out[q, j] = AND over the conjuncts of query q
// (rows[offsets[q] .. offsets[q + 1]]) of R[row, slots[j]] > 0 (And() of nothing: true)
PyObject* py_conj_answer(PyObject*, PyObject* a) {
  PyObject *o_R, *o_rows, *o_off, *o_slots, *o_out;
  if (!PyArg_ParseTuple(a, "OOOOO", &o_R, &o_rows, &o_off, &o_slots, &o_out)) return nullptr;
  Buf R, rows, off, slots, out;
  if (!get_buf(o_R, R, false, 1, "R") || !get_buf(o_rows, rows, false, 8, "rows") ||
      !get_buf(o_off, off, false, 8, "offsets") || !get_buf(o_slots, slots, false, 8, "slots") ||
      !get_buf(o_out, out, true, 1, "out"))
    return nullptr;
  const Py_ssize_t nq = off.b.len / 8 - 1, ns = slots.b.len / 8, nr = rows.b.len / 8;
  if (R.b.ndim != 2 || nq < 0 || out.b.len != nq * ns) {
    PyErr_SetString(PyExc_ValueError, "conj_answer: shapes");
    return nullptr;
  }
  const Py_ssize_t rcap = R.b.shape[0], scap = R.b.shape[1];
  const int8_t* RR = (const int8_t*)R.b.buf;
  const int64_t* rw = (const int64_t*)rows.b.buf;
  const int64_t* of = (const int64_t*)off.b.buf;
  const int64_t* sl = (const int64_t*)slots.b.buf;
  uint8_t* o = (uint8_t*)out.b.buf;
  for (Py_ssize_t j = 0; j < ns; j++)
    if (sl[j] < 0 || sl[j] >= scap) {
      PyErr_SetString(PyExc_ValueError, "conj_answer: slot beyond R");
      return nullptr;
    }
  for (Py_ssize_t q = 0; q < nq; q++) {
    if (of[q] < 0 || of[q + 1] > nr || of[q] > of[q + 1]) {
      PyErr_SetString(PyExc_ValueError, "conj_answer: offsets");
      return nullptr;
    }
    uint8_t* oq = o + q * ns;
    for (Py_ssize_t j = 0; j < ns; j++) oq[j] = 1;
    for (int64_t k = of[q]; k < of[q + 1]; k++) {
      if (rw[k] < 0 || rw[k] >= rcap) {
        PyErr_SetString(PyExc_ValueError, "conj_answer: row beyond R");
        return nullptr;
      }
      const int8_t* rr = RR + rw[k] * scap;
      for (Py_ssize_t j = 0; j < ns; j++) oq[j] &= rr[sl[j]] > 0 ? 1 : 0;
    }
  }
  Py_RETURN_NONE;
}

PyMethodDef methods[] = {
    {"conj_rows", py_conj_rows, METH_VARARGS, "conj_rows(roots, row_of, n_rows, R, slots, rows_out) -> (n_rows, todo)"},
    {"conj_answer", py_conj_answer, METH_VARARGS, "conj_answer(R, rows, offsets, slots, out): per-query AND of conjunct rows"},
    {"candidate_rows", py_candidate_rows, METH_VARARGS,
     "candidate_rows(gen, lru, src, starts, patches, var_off, var_limbs): generated candidates' rows"},
    {"pack_nodes", py_pack_nodes, METH_VARARGS, "pack_nodes(nodes, start, end, out): node tuples -> NODE_DTYPE records"},
    {"bind", py_bind, METH_O, "bind(Term): read the term class's slot offsets"},
    {"lower_roots", py_lower_roots, METH_VARARGS, "lower_roots(roots, state) -> per root: node list or exception"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_lowerwalk", "IncrementalLowering's term walk (lower.py)", -1, methods};

}  // namespace

PyMODINIT_FUNC PyInit__lowerwalk(void) { return PyModule_Create(&module); }
