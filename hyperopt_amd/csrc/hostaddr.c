/* _hostaddr: data addresses of many numpy arrays in one call.
 *
 * The tree records (tpe._tree_labels) and level records (Engine._labels)
 * point the native runtime at per-label numpy columns; numpy's own accessors
 * (arr.ctypes.data, __array_interface__) cost a Python object per array, which
 * for a thousand labels is a millisecond of host time per suggest.  This reads
 * PyArray_DATA directly. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#define NPY_NO_DEPRECATED_API NPY_2_0_API_VERSION
#include <numpy/arrayobject.h>
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

/* row_dicts(keys, columns) -> [dict(zip(keys, row)) for row in zip(*columns)]:
 * the per-id result dicts of a batched suggest (tpe._choice_dicts), built
 * without a zip, a tuple or an iterator per id (keys: a tuple of k keys;
 * columns: k lists of equal length n). */
static PyObject *row_dicts(PyObject *self, PyObject *args) {
  (void)self;
  PyObject *keys, *cols;
  if (!PyArg_ParseTuple(args, "O!O!", &PyTuple_Type, &keys, &PyList_Type, &cols)) return NULL;
  const Py_ssize_t k = PyTuple_GET_SIZE(keys);
  if (PyList_GET_SIZE(cols) != k) {
    PyErr_SetString(PyExc_ValueError, "row_dicts(): one column per key");
    return NULL;
  }
  Py_ssize_t n = -1;
  for (Py_ssize_t j = 0; j < k; ++j) {
    PyObject *c = PyList_GET_ITEM(cols, j);
    if (!PyList_Check(c) || (n >= 0 && PyList_GET_SIZE(c) != n)) {
      PyErr_SetString(PyExc_ValueError, "row_dicts(): columns must be lists of one length");
      return NULL;
    }
    n = PyList_GET_SIZE(c);
  }
  if (n < 0) n = 0;
  PyObject *out = PyList_New(n);
  if (!out) return NULL;
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject *d = _PyDict_NewPresized(k);
    if (!d) { Py_DECREF(out); return NULL; }
    for (Py_ssize_t j = 0; j < k; ++j) {
      if (PyDict_SetItem(d, PyTuple_GET_ITEM(keys, j), PyList_GET_ITEM(PyList_GET_ITEM(cols, j), i)) < 0) {
        Py_DECREF(d);
        Py_DECREF(out);
        return NULL;
      }
    }
    PyList_SET_ITEM(out, i, d);
  }
  return out;
}

static PyMethodDef methods[] = {
    {"addresses", addresses, METH_VARARGS,
     "int64 array of the data addresses of a sequence of C-contiguous numpy arrays (of dtype typenum)"},
    {"tails", tails, METH_VARARGS, "float64 concatenation of seq[i][start[i]:stop[i]]"},
    {"row_dicts", row_dicts, METH_VARARGS, "[dict(zip(keys, row)) for row in zip(*columns)]"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_hostaddr", NULL, -1, methods,
                                    NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__hostaddr(void) {
  import_array();
  return PyModule_Create(&module);
}
