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

/* addresses(seq) -> int64 array of the items' data addresses (each item a
 * C-contiguous numpy array; anything else raises TypeError). */
static PyObject *addresses(PyObject *self, PyObject *arg) {
  (void)self;
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
    if (!PyArray_Check(a) || !PyArray_IS_C_CONTIGUOUS((PyArrayObject *)a)) {
      PyErr_Format(PyExc_TypeError, "item %zd is not a C-contiguous numpy array", i);
      Py_DECREF(out);
      Py_DECREF(seq);
      return NULL;
    }
    o[i] = (npy_int64)(intptr_t)PyArray_DATA((PyArrayObject *)a);
  }
  Py_DECREF(seq);
  return out;
}

static PyMethodDef methods[] = {
    {"addresses", addresses, METH_O, "int64 array of the data addresses of a sequence of C-contiguous numpy arrays"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_hostaddr", NULL, -1, methods,
                                    NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__hostaddr(void) {
  import_array();
  return PyModule_Create(&module);
}
