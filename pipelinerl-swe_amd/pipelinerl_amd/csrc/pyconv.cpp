// Python-object helpers of libprl_data.so (not part of the C ABI in include/prl_data.h; the
// binding calls them through ctypes.PyDLL, i.e. with the GIL held).  The preprocessor's rollouts
// arrive as Python lists (pipelinerl/finetune/rl/__init__.py:504-525 builds them), and converting
// a list element by element is what bounds collate_packed (data.py:215-279) in Python:
// numpy.asarray / array.array spend 20-45 ns per element, this loop 2-5 ns.
#include <Python.h>

#include <cstdint>

extern "C" {

// Concatenate the lists in `seqs` (a list of lists) into `out` (n elements): dtype 0 = int64
// from Python ints, 3 = float64 from Python floats or ints (float(int), as numpy does).
// Returns 0, 1 when an element has another type (the caller converts that batch in Python) or a
// count mismatch, -1 with a Python error set.
int prl_py_concat(PyObject* seqs, int dtype, void* out, int64_t n) {
  if (!PyList_Check(seqs)) return 1;
  const Py_ssize_t ns = PyList_GET_SIZE(seqs);
  int64_t k = 0;
  for (Py_ssize_t i = 0; i < ns; ++i) {
    PyObject* s = PyList_GET_ITEM(seqs, i);
    if (!PyList_Check(s)) return 1;
    const Py_ssize_t m = PyList_GET_SIZE(s);
    if (k + m > n) return 1;
    PyObject** items = reinterpret_cast<PyListObject*>(s)->ob_item;
    if (dtype == 0) {
      int64_t* o = static_cast<int64_t*>(out) + k;
      for (Py_ssize_t j = 0; j < m; ++j) {
        PyObject* x = items[j];
        if (!PyLong_CheckExact(x)) return 1;  // bools, floats, numpy scalars: Python path
        int overflow = 0;
        const long long v = PyLong_AsLongLongAndOverflow(x, &overflow);
        if (overflow) return 1;
        o[j] = v;
      }
    } else if (dtype == 3) {
      double* o = static_cast<double*>(out) + k;
      for (Py_ssize_t j = 0; j < m; ++j) {
        PyObject* x = items[j];
        if (PyFloat_CheckExact(x)) {
          o[j] = PyFloat_AS_DOUBLE(x);
        } else if (PyLong_CheckExact(x)) {
          const double v = PyLong_AsDouble(x);
          if (v == -1.0 && PyErr_Occurred()) {
            PyErr_Clear();
            return 1;
          }
          o[j] = v;
        } else {
          return 1;
        }
      }
    } else {
      return 1;
    }
    k += m;
  }
  return k == n ? 0 : 1;
}

}  // extern "C"
