/* _hostaddr: data addresses of many numpy arrays in one call.
 *
 * The tree records (tpe._tree_labels) and level records (Engine._labels)
 * point the native runtime at per-label numpy columns; numpy's own accessors
 * (arr.ctypes.data, __array_interface__) cost a Python object per array, which
 * for a thousand labels is a millisecond of host time per suggest.  This reads
 * PyArray_DATA directly. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <structmember.h>
#define NPY_NO_DEPRECATED_API NPY_2_0_API_VERSION
#include <numpy/arrayobject.h>
#include <numpy/arrayscalars.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* addresses(seq[, typenum]) -> int64 array of the items' data addresses (each
 * item a C-contiguous numpy array — of dtype typenum when given; anything else
 * raises TypeError, which callers take as "convert first"). */
static PyObject *addresses(PyObject *self, PyObject *args) {
  (void)self;
  PyObject *arg;
  int typenum = -1;
  if (!PyArg_ParseTuple(args, "O|i", &arg, &typenum)) return NULL;
  PyObject *seq = PySequence_Fast(arg, "addresses() takes a sequence of numpy arrays");
  if (!seq) return NULL;
  Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  npy_intp dims[1] = {n};
  PyObject *out = PyArray_SimpleNew(1, dims, NPY_INT64);
  if (!out) { Py_DECREF(seq); return NULL; }
  npy_int64 *o = (npy_int64 *)PyArray_DATA((PyArrayObject *)out);
  PyObject **items = PySequence_Fast_ITEMS(seq);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject *a = items[i];
    if (!PyArray_Check(a) || !PyArray_IS_C_CONTIGUOUS((PyArrayObject *)a) ||
        (typenum >= 0 && !PyArray_EquivTypenums(PyArray_TYPE((PyArrayObject *)a), typenum))) {
      PyErr_Format(PyExc_TypeError, "item %zd is not a C-contiguous numpy array of the type asked", i);
      Py_DECREF(out);
      Py_DECREF(seq);
      return NULL;
    }
    o[i] = (npy_int64)(intptr_t)PyArray_DATA((PyArrayObject *)a);
  }
  Py_DECREF(seq);
  return out;
}

/* tails(seq, start, stop) -> float64 array: seq[i][start[i]:stop[i]] for every
 * i, concatenated (each item a 1-D C-contiguous float64 array of at least
 * stop[i] values; start, stop int64 arrays of len(seq)). */
static PyObject *tails(PyObject *self, PyObject *args) {
  (void)self;
  PyObject *arg, *a0, *a1;
  if (!PyArg_ParseTuple(args, "OOO", &arg, &a0, &a1)) return NULL;
  PyObject *seq = PySequence_Fast(arg, "tails() takes a sequence of numpy arrays");
  if (!seq) return NULL;
  PyArrayObject *st = (PyArrayObject *)PyArray_FROMANY(a0, NPY_INT64, 1, 1, NPY_ARRAY_IN_ARRAY);
  PyArrayObject *sp = st ? (PyArrayObject *)PyArray_FROMANY(a1, NPY_INT64, 1, 1, NPY_ARRAY_IN_ARRAY) : NULL;
  PyObject *out = NULL;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  if (!sp) goto done;
  if (PyArray_DIM(st, 0) != n || PyArray_DIM(sp, 0) != n) {
    PyErr_SetString(PyExc_ValueError, "tails(): start / stop length");
    goto done;
  }
  {
    const npy_int64 *b = (const npy_int64 *)PyArray_DATA(st), *e = (const npy_int64 *)PyArray_DATA(sp);
    PyObject **items = PySequence_Fast_ITEMS(seq);
    npy_intp tot = 0;
    for (Py_ssize_t i = 0; i < n; ++i) {
      PyObject *a = items[i];
      if (!PyArray_Check(a) || PyArray_NDIM((PyArrayObject *)a) != 1 ||
          !PyArray_IS_C_CONTIGUOUS((PyArrayObject *)a) || PyArray_TYPE((PyArrayObject *)a) != NPY_FLOAT64 ||
          b[i] < 0 || e[i] < b[i] || e[i] > PyArray_DIM((PyArrayObject *)a, 0)) {
        PyErr_Format(PyExc_ValueError, "tails(): item %zd is not a float64 column holding [start, stop)", i);
        goto done;
      }
      tot += (npy_intp)(e[i] - b[i]);
    }
    npy_intp dims[1] = {tot};
    out = PyArray_SimpleNew(1, dims, NPY_FLOAT64);
    if (!out) goto done;
    double *o = (double *)PyArray_DATA((PyArrayObject *)out);
    for (Py_ssize_t i = 0; i < n; ++i) {
      const npy_int64 k = e[i] - b[i];
      if (k == 1) *o = ((const double *)PyArray_DATA((PyArrayObject *)items[i]))[b[i]];
      else if (k > 1) memcpy(o, (const double *)PyArray_DATA((PyArrayObject *)items[i]) + b[i], (size_t)k * sizeof(double));
      o += k;
    }
  }
done:
  Py_XDECREF(st);
  Py_XDECREF(sp);
  Py_DECREF(seq);
  return out;
}

/* typed_dicts(keys, ix, cat, values, active) -> per row i of values / active
 * ([n x L] float64 / int8, C-contiguous) the dict {keys[j]: value} in the
 * order of `keys` (k labels; ix: their k table indices, int64; cat: k bytes, 1
 * for a categorical label): np.int64(values[i, ix[j]]) for a categorical,
 * np.float64 for any other, None where active[i, ix[j]] == 0 — the reference's
 * value types (its vals come out of numpy arrays), made without a Python call
 * per value (a suggest of a 1000-dim space: 1000 scalars). */
static PyObject *typed_dicts(PyObject *self, PyObject *args) {
  (void)self;
  PyObject *keys, *ao, *co, *vo, *acto;
  if (!PyArg_ParseTuple(args, "O!OOOO", &PyTuple_Type, &keys, &ao, &co, &vo, &acto)) return NULL;
  PyArrayObject *ix = (PyArrayObject *)PyArray_FROMANY(ao, NPY_INT64, 1, 1, NPY_ARRAY_IN_ARRAY);
  PyArrayObject *cat = ix ? (PyArrayObject *)PyArray_FROMANY(co, NPY_INT8, 1, 1, NPY_ARRAY_IN_ARRAY) : NULL;
  PyObject *out = NULL;
  if (!cat) goto done;
  if (!PyArray_Check(vo) || !PyArray_Check(acto)) {
    PyErr_SetString(PyExc_TypeError, "typed_dicts(): values / active must be numpy arrays");
    goto done;
  }
  {
    PyArrayObject *va = (PyArrayObject *)vo, *aa = (PyArrayObject *)acto;
    const Py_ssize_t k = PyTuple_GET_SIZE(keys);
    if (PyArray_NDIM(va) != 2 || PyArray_NDIM(aa) != 2 || PyArray_TYPE(va) != NPY_FLOAT64 ||
        (PyArray_TYPE(aa) != NPY_INT8 && PyArray_TYPE(aa) != NPY_BOOL) || !PyArray_IS_C_CONTIGUOUS(va) ||
        !PyArray_IS_C_CONTIGUOUS(aa) || PyArray_DIM(va, 0) != PyArray_DIM(aa, 0) ||
        PyArray_DIM(va, 1) != PyArray_DIM(aa, 1) || PyArray_DIM(ix, 0) != k || PyArray_DIM(cat, 0) != k) {
      PyErr_SetString(PyExc_ValueError, "typed_dicts(): values / active [n x L] float64 / int8, k keys");
      goto done;
    }
    const npy_intp n = PyArray_DIM(va, 0), L = PyArray_DIM(va, 1);
    const npy_int64 *ixp = (const npy_int64 *)PyArray_DATA(ix);
    const npy_int8 *cp = (const npy_int8 *)PyArray_DATA(cat);
    for (Py_ssize_t j = 0; j < k; ++j)
      if (ixp[j] < 0 || ixp[j] >= L) {
        PyErr_SetString(PyExc_ValueError, "typed_dicts(): index out of range");
        goto done;
      }
    out = PyList_New(n);
    if (!out) goto done;
    const double *v = (const double *)PyArray_DATA(va);
    const npy_int8 *a = (const npy_int8 *)PyArray_DATA(aa);
    for (npy_intp i = 0; i < n; ++i) {
      PyObject *d = _PyDict_NewPresized(k);
      if (!d) { Py_CLEAR(out); goto done; }
      PyList_SET_ITEM(out, i, d);
      for (Py_ssize_t j = 0; j < k; ++j) {
        const npy_intp t = (npy_intp)ixp[j];
        PyObject *o;
        if (!a[i * L + t]) {
          o = Py_None;
          Py_INCREF(o);
        } else if (cp[j]) {
          o = PyArrayScalar_New(Long);
          if (o) PyArrayScalar_ASSIGN(o, Long, (npy_long)v[i * L + t]);
        } else {
          o = PyArrayScalar_New(Double);
          if (o) PyArrayScalar_ASSIGN(o, Double, v[i * L + t]);
        }
        if (!o || PyDict_SetItem(d, PyTuple_GET_ITEM(keys, j), o) < 0) {
          Py_XDECREF(o);
          Py_CLEAR(out);
          goto done;
        }
        Py_DECREF(o);
      }
    }
  }
done:
  Py_XDECREF(ix);
  Py_XDECREF(cat);
  return out;
}

/* a fresh empty instance of a list subclass (zeroed by tp_alloc: an empty
 * list, its slots unset) — no __new__ / __init__ dispatch */
static PyObject *new_list_of(PyTypeObject *t) { return t->tp_alloc(t, 0); }

static int set_up(PyObject *o, PyObject *name, PyObject *v) { return PyObject_SetAttr(o, name, v); }

/* the byte offset of a type's __slots__ member `name` (its member
 * descriptor), or -1: written directly, as the descriptor's __set__ writes */
static Py_ssize_t slot_offset(PyTypeObject *t, const char *name) {
  PyObject *d = PyObject_GetAttrString((PyObject *)t, name);
  if (!d) { PyErr_Clear(); return -1; }
  Py_ssize_t off = -1;
  if (Py_IS_TYPE(d, &PyMemberDescr_Type)) {
    PyMemberDef *m = ((PyMemberDescrObject *)d)->d_member;
    if (m->type == T_OBJECT_EX && !(m->flags & READONLY)) off = m->offset;
  }
  Py_DECREF(d);
  return off;
}

static void put_slot(PyObject *o, Py_ssize_t off, PyObject *v) {
  PyObject **p = (PyObject **)((char *)o + off);
  PyObject *old = *p;
  Py_INCREF(v);
  *p = v;
  Py_XDECREF(old);
}

/* tracked_misc(tid, cmd, workdir, chosen, Part, PartList) -> the misc of one
 * suggested id (base.tracked_misc): idxs [tid] / vals [value] per active
 * label, [] per inactive one (value None), every list a PartList whose _up is
 * a weak reference to its dict, the dicts Parts whose _up is a weak reference
 * to the misc, misc._up None and misc._fx False (weak: no reference cycle, see
 * base.py).  The dict entries go in through the base dict (no tracked
 * __setitem__), as the Python version's dict.__setitem__. */
static PyObject *tracked_misc(PyObject *self, PyObject *args) {
  (void)self;
  PyObject *tid, *cmd, *workdir, *chosen, *part, *plist;
  if (!PyArg_ParseTuple(args, "OOOO!O!O!", &tid, &cmd, &workdir, &PyDict_Type, &chosen, &PyType_Type, &part,
                        &PyType_Type, &plist))
    return NULL;
  PyTypeObject *PT = (PyTypeObject *)plist;
  if (!PyType_IsSubtype(PT, &PyList_Type) || !PyType_IsSubtype((PyTypeObject *)part, &PyDict_Type)) {
    PyErr_SetString(PyExc_TypeError, "tracked_misc(): Part must subclass dict, PartList list");
    return NULL;
  }
  static PyObject *s_up = NULL, *s_fx = NULL;
  if (!s_up && !(s_up = PyUnicode_InternFromString("_up"))) return NULL;
  if (!s_fx && !(s_fx = PyUnicode_InternFromString("_fx"))) return NULL;
  /* the PartList type whose _up offset is cached: held (a strong reference),
   * so another type can never reuse its address while the offset is kept */
  static PyTypeObject *s_pt = NULL;
  static Py_ssize_t s_pt_up = -1;
  if (s_pt != PT) {
    Py_INCREF(PT);
    Py_XDECREF(s_pt);
    s_pt = PT;
    s_pt_up = slot_offset(PT, "_up");
  }
  PyObject *idxs = PyObject_CallNoArgs(part), *vals = idxs ? PyObject_CallNoArgs(part) : NULL;
  PyObject *misc = NULL, *kw = NULL, *wi = NULL, *wv = NULL, *wm = NULL;
  if (!vals) goto fail;
  /* (one weak reference per parent, shared by its lists) */
  if (!(wi = PyWeakref_NewRef(idxs, NULL)) || !(wv = PyWeakref_NewRef(vals, NULL))) goto fail;
  PyObject *k, *v;
  Py_ssize_t pos = 0;
  while (PyDict_Next(chosen, &pos, &k, &v)) {
    PyObject *a = new_list_of(PT), *b = a ? new_list_of(PT) : NULL;
    if (!b) { Py_XDECREF(a); goto fail; }
    int bad = v != Py_None && (PyList_Append(a, tid) < 0 || PyList_Append(b, v) < 0);
    if (!bad && s_pt_up >= 0) {
      put_slot(a, s_pt_up, wi);
      put_slot(b, s_pt_up, wv);
    } else {
      bad = bad || set_up(a, s_up, wi) < 0 || set_up(b, s_up, wv) < 0;
    }
    bad = bad || PyDict_SetItem(idxs, k, a) < 0 || PyDict_SetItem(vals, k, b) < 0;
    Py_DECREF(a);
    Py_DECREF(b);
    if (bad) goto fail;
  }
  kw = Py_BuildValue("{sOsOsOsOsO}", "tid", tid, "cmd", cmd, "workdir", workdir, "idxs", idxs, "vals", vals);
  if (!kw) goto fail;
  {
    PyObject *empty = PyTuple_New(0);
    misc = empty ? PyObject_Call(part, empty, kw) : NULL;
    Py_XDECREF(empty);
  }
  if (!misc || !(wm = PyWeakref_NewRef(misc, NULL)) || set_up(idxs, s_up, wm) < 0 || set_up(vals, s_up, wm) < 0 ||
      set_up(misc, s_up, Py_None) < 0 || set_up(misc, s_fx, Py_False) < 0)
    goto fail;
  Py_DECREF(kw);
  Py_DECREF(wi);
  Py_DECREF(wv);
  Py_DECREF(wm);
  Py_DECREF(idxs);
  Py_DECREF(vals);
  return misc;
fail:
  Py_XDECREF(wi);
  Py_XDECREF(wv);
  Py_XDECREF(wm);
  Py_XDECREF(kw);
  Py_XDECREF(misc);
  Py_XDECREF(idxs);
  Py_XDECREF(vals);
  return NULL;
}

/* call_tree(fn, ...): tpe_suggest_tree (include/tpe_hip.h) called through its
 * address with the engine's 23 arguments as Python ints / floats, the GIL
 * released — ctypes spent microseconds converting them per suggest.  The
 * TPE_DEBUG_FLAGS environment bits are OR-ed into `flags` here (read per call,
 * as Engine._flags reads them). */
typedef int (*tree_fn)(const void *, int32_t, const int64_t *, int64_t, double, int32_t, const int64_t *, int32_t,
                       int32_t, int64_t, int64_t, const void *, uint64_t, double, int64_t, int32_t, const void *, void *,
                       void *, double *, int8_t *, int32_t *, int8_t *);
static PyObject *call_tree(PyObject *self, PyObject *args) {
  (void)self;
  unsigned long long fn, labels, below, ids, ex, seed, ws, need, stream, values, active, path, need_fit;
  int n_labels, lf, n_ids, n_cand, flags;
  long long n_below, cand_base, n_cand_global, dev_fit_min;
  double prior_weight, min_draws;
  if (!PyArg_ParseTuple(args, "KKiKLdiKiiLLKKdLiKKKKKKK", &fn, &labels, &n_labels, &below, &n_below, &prior_weight,
                        &lf, &ids, &n_ids, &n_cand, &cand_base, &n_cand_global, &ex, &seed, &min_draws,
                        &dev_fit_min, &flags, &ws, &need, &stream, &values, &active, &path, &need_fit))
    return NULL;
  if (!fn) {
    PyErr_SetString(PyExc_ValueError, "call_tree(): null function");
    return NULL;
  }
  const char *e = getenv("TPE_DEBUG_FLAGS");
  if (e && *e) flags |= (int)strtol(e, NULL, 10);
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = ((tree_fn)(uintptr_t)fn)((const void *)(uintptr_t)labels, n_labels, (const int64_t *)(uintptr_t)below,
                                n_below, prior_weight, lf, (const int64_t *)(uintptr_t)ids, n_ids, n_cand, cand_base,
                                n_cand_global, (const void *)(uintptr_t)ex, (uint64_t)seed, min_draws, dev_fit_min,
                                flags, (const void *)(uintptr_t)ws, (void *)(uintptr_t)need, (void *)(uintptr_t)stream,
                                (double *)(uintptr_t)values, (int8_t *)(uintptr_t)active, (int32_t *)(uintptr_t)path,
                                (int8_t *)(uintptr_t)need_fit);
  Py_END_ALLOW_THREADS
  return PyLong_FromLong(rc);
}

/* insert_sorted(perm, sorted, m, value, index) -> at: one appended value into
 * a column's sorting permutation (int64) and its sorted values (float64), both
 * holding m entries and room for one more — at = np.searchsorted(sorted[:m],
 * value, side='right') (numpy's order: NaN after every number), then the tails
 * from `at` move up one slot and perm[at] = index, sorted[at] = value
 * (history.value_order's one-observation case, without the numpy and ctypes
 * calls per suggest). */
static int npy_lt(double a, double b) { return a < b || (b != b && a == a); }
static PyObject *insert_sorted(PyObject *self, PyObject *args) {
  (void)self;
  PyArrayObject *perm, *sorted;
  Py_ssize_t m;
  double v;
  long long index;
  if (!PyArg_ParseTuple(args, "O!O!ndL", &PyArray_Type, &perm, &PyArray_Type, &sorted, &m, &v, &index)) return NULL;
  if (PyArray_TYPE(perm) != NPY_INT64 || PyArray_TYPE(sorted) != NPY_FLOAT64 || !PyArray_IS_C_CONTIGUOUS(perm) ||
      !PyArray_IS_C_CONTIGUOUS(sorted) || !PyArray_ISWRITEABLE(perm) || !PyArray_ISWRITEABLE(sorted) || m < 0 ||
      PyArray_SIZE(perm) < m + 1 || PyArray_SIZE(sorted) < m + 1) {
    PyErr_SetString(PyExc_ValueError, "insert_sorted(): int64 / float64 contiguous arrays with room for m + 1");
    return NULL;
  }
  int64_t *p = (int64_t *)PyArray_DATA(perm);
  double *a = (double *)PyArray_DATA(sorted);
  Py_ssize_t lo = 0, hi = m;
  while (lo < hi) {                                   /* first i with value < a[i] */
    const Py_ssize_t mid = lo + ((hi - lo) >> 1);
    if (npy_lt(v, a[mid])) hi = mid; else lo = mid + 1;
  }
  memmove(p + lo + 1, p + lo, (size_t)(m - lo) * sizeof(int64_t));
  memmove(a + lo + 1, a + lo, (size_t)(m - lo) * sizeof(double));
  p[lo] = (int64_t)index;
  a[lo] = v;
  return PyLong_FromSsize_t(lo);
}

/* obs_append(labels, vals, tid, tcols, vcols, changed): History._Cache.extend's
   per-label loop for one document (history.py) — for each label k with a truthy
   vals[k] (a dict or dict subclass read without its methods: the caller passes
   plain dicts and the package's tracked ones only), tid and vals[k][0] appended to
   the label's _Grow columns (a[n] = value, n += 1, numpy's item assignment) and k
   added to `changed`.  Returns -1, or the position of the first label whose
   column is full (nothing of it written: the caller grows it and goes on). */
static PyObject *s_a, *s_n;

static int grow_put(PyObject *g, PyObject *value) {      /* g.a[g.n] = value; g.n += 1 (room checked) */
  PyObject *a = PyObject_GetAttr(g, s_a), *nobj = a ? PyObject_GetAttr(g, s_n) : NULL;
  int rc = -1;
  if (nobj) {
    const Py_ssize_t n = PyLong_AsSsize_t(nobj);
    if (!(n == -1 && PyErr_Occurred()) && PyObject_SetItem(a, nobj, value) == 0) {
      PyObject *n1 = PyLong_FromSsize_t(n + 1);
      rc = n1 ? PyObject_SetAttr(g, s_n, n1) : -1;
      Py_XDECREF(n1);
    }
  }
  Py_XDECREF(a);
  Py_XDECREF(nobj);
  return rc;
}

static PyObject *obs_append(PyObject *self, PyObject *args) {
  (void)self;
  PyObject *labels, *vals, *tid, *tcols, *vcols, *changed;
  if (!PyArg_ParseTuple(args, "OO!OO!O!O!", &labels, &PyDict_Type, &vals, &tid, &PyList_Type, &tcols, &PyList_Type,
                        &vcols, &PySet_Type, &changed))
    return NULL;
  PyObject *seq = PySequence_Fast(labels, "obs_append(): labels must be a sequence");
  if (!seq) return NULL;
  const Py_ssize_t L = PySequence_Fast_GET_SIZE(seq);
  if (PyList_GET_SIZE(tcols) != L || PyList_GET_SIZE(vcols) != L) {
    Py_DECREF(seq);
    PyErr_SetString(PyExc_ValueError, "obs_append(): one tid and one value column per label");
    return NULL;
  }
  for (Py_ssize_t i = 0; i < L; ++i) {
    PyObject *k = PySequence_Fast_GET_ITEM(seq, i);
    PyObject *v = PyDict_GetItemWithError(vals, k);           /* borrowed */
    if (!v) {
      if (PyErr_Occurred()) goto fail;
      continue;
    }
    const int t = PyObject_IsTrue(v);
    if (t < 0) goto fail;
    if (!t) continue;
    PyObject *tc = PyList_GET_ITEM(tcols, i), *vc = PyList_GET_ITEM(vcols, i);
    /* both columns have room, else the label is handed back */
    {
      PyObject *a = PyObject_GetAttr(tc, s_a), *nobj = a ? PyObject_GetAttr(tc, s_n) : NULL;
      Py_ssize_t n = nobj ? PyLong_AsSsize_t(nobj) : -1, cap = a ? PyObject_Size(a) : -1;
      Py_XDECREF(a);
      Py_XDECREF(nobj);
      if (PyErr_Occurred()) goto fail;
      PyObject *b = PyObject_GetAttr(vc, s_a), *mobj = b ? PyObject_GetAttr(vc, s_n) : NULL;
      Py_ssize_t m = mobj ? PyLong_AsSsize_t(mobj) : -1, capb = b ? PyObject_Size(b) : -1;
      Py_XDECREF(b);
      Py_XDECREF(mobj);
      if (PyErr_Occurred()) goto fail;
      if (n >= cap || m >= capb) {
        Py_DECREF(seq);
        return PyLong_FromSsize_t(i);
      }
    }
    PyObject *x = PySequence_GetItem(v, 0);
    if (!x) goto fail;
    if (grow_put(tc, tid) < 0 || grow_put(vc, x) < 0) {
      Py_DECREF(x);
      goto fail;
    }
    Py_DECREF(x);
    if (PySet_Add(changed, k) < 0) goto fail;
  }
  Py_DECREF(seq);
  return PyLong_FromLong(-1);
fail:
  Py_DECREF(seq);
  return NULL;
}

static PyMethodDef methods[] = {
    {"addresses", addresses, METH_VARARGS,
     "int64 array of the data addresses of a sequence of C-contiguous numpy arrays (of dtype typenum)"},
    {"tails", tails, METH_VARARGS, "float64 concatenation of seq[i][start[i]:stop[i]]"},
    {"typed_dicts", typed_dicts, METH_VARARGS, "per-row {label: np.int64 / np.float64 / None} dicts"},
    {"tracked_misc", tracked_misc, METH_VARARGS, "base.tracked_misc: the tracked misc of one suggested id"},
    {"call_tree", call_tree, METH_VARARGS, "tpe_suggest_tree through its address (Engine.suggest_tree)"},
    {"insert_sorted", insert_sorted, METH_VARARGS, "one value into a sorting permutation and its sorted values"},
    {"obs_append", obs_append, METH_VARARGS, "one document's observations appended to the label columns"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_hostaddr", NULL, -1, methods,
                                    NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__hostaddr(void) {
  import_array();
  s_a = PyUnicode_InternFromString("a");
  s_n = PyUnicode_InternFromString("n");
  if (!s_a || !s_n) return NULL;
  return PyModule_Create(&module);
}
