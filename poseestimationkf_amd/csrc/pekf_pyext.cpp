// pekf_pyext.cpp -- CPython binding of the n = 1 entry points the drop-in modules call once per
// record (main_file.py:42-45: Prediction, the discarded getQuarternion, Correction).  It only
// converts arguments and results; the arithmetic is libpekf.so's (pekf_predict, pekf_correct,
// pekf_wahba_quaternion -> gfx950 kernels).  Compared with the ctypes path it saves the Python
// side of a call (array conversion, argument marshalling: ~9 us of an ~18 us call).
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#define NPY_NO_DEPRECATED_API NPY_1_7_API_VERSION
#include <numpy/arrayobject.h>

#include "../../include/pekf.h"

namespace {

PyObject *g_linalg_error = nullptr;  // numpy.linalg.LinAlgError

// A float64 C-contiguous view (or converted copy) of `obj` with exactly `n` elements.
struct In {
    PyArrayObject *arr = nullptr;
    const double *p = nullptr;
    double scalar = 0.0;
    ~In() { Py_XDECREF(arr); }
    bool get(PyObject *obj, npy_intp n, const char *name) {
        if (n == 1 && PyFloat_Check(obj)) {
            scalar = PyFloat_AS_DOUBLE(obj);
            p = &scalar;
            return true;
        }
        arr = reinterpret_cast<PyArrayObject *>(
            PyArray_FROMANY(obj, NPY_DOUBLE, 0, 0, NPY_ARRAY_C_CONTIGUOUS | NPY_ARRAY_ALIGNED));
        if (!arr) return false;
        if (PyArray_SIZE(arr) != n) {
            PyErr_Format(PyExc_ValueError, "%s: expected %zd values, got %zd", name, (Py_ssize_t)n,
                         (Py_ssize_t)PyArray_SIZE(arr));
            return false;
        }
        p = static_cast<const double *>(PyArray_DATA(arr));
        return true;
    }
};

PyObject *new_array(int nd, npy_intp d0, npy_intp d1 = 0) {
    npy_intp dims[2] = {d0, d1};
    return PyArray_SimpleNew(nd, dims, NPY_DOUBLE);
}

double *data(PyObject *a) { return static_cast<double *>(PyArray_DATA(reinterpret_cast<PyArrayObject *>(a))); }

// Same mapping as poseestimationkf_amd._lib.check: LinAlgError for singular S / non-finite Wahba
// input (what NumPy raises there), NoDeviceError / PekfError otherwise.
PyObject *fail(int status) {
    const char *msg = pekf_last_error();
    if (!msg) msg = "";
    if (status == PEKF_ERR_SINGULAR || status == PEKF_ERR_SVD) {
        PyErr_SetString(g_linalg_error, *msg ? msg : "linear algebra error");
        return nullptr;
    }
    PyObject *lib = PyImport_ImportModule("poseestimationkf_amd._lib");
    PyObject *cls = lib ? PyObject_GetAttrString(lib, status == PEKF_ERR_NODEVICE ? "NoDeviceError" : "PekfError")
                        : nullptr;
    Py_XDECREF(lib);
    if (!cls) return nullptr;
    PyObject *exc = PyObject_CallFunction(cls, "is", status, msg);
    Py_DECREF(cls);
    if (exc) {
        PyErr_SetObject(reinterpret_cast<PyObject *>(Py_TYPE(exc)), exc);
        Py_DECREF(exc);
    }
    return nullptr;
}

// predict(gyro[3], dt_ns, X[4], P[4x4], Q[3x3], R[4x4]) -> (z[4], P-[4x4], K[4x4])
PyObject *py_predict(PyObject *, PyObject *args) {
    PyObject *o[6];
    if (!PyArg_UnpackTuple(args, "predict", 6, 6, &o[0], &o[1], &o[2], &o[3], &o[4], &o[5])) return nullptr;
    In g, dt, X, P, Q, R;
    if (!g.get(o[0], 3, "gyro") || !dt.get(o[1], 1, "dt") || !X.get(o[2], 4, "X") || !P.get(o[3], 16, "P") ||
        !Q.get(o[4], 9, "Q") || !R.get(o[5], 16, "R"))
        return nullptr;
    PyObject *z = new_array(1, 4), *Pm = new_array(2, 4, 4), *K = new_array(2, 4, 4);
    if (!z || !Pm || !K) {
        Py_XDECREF(z); Py_XDECREF(Pm); Py_XDECREF(K);
        return nullptr;
    }
    int st;
    Py_BEGIN_ALLOW_THREADS
    st = pekf_predict(1, g.p, dt.p, X.p, P.p, Q.p, R.p, data(z), data(Pm), data(K));
    Py_END_ALLOW_THREADS
    if (st) {
        Py_DECREF(z); Py_DECREF(Pm); Py_DECREF(K);
        return fail(st);
    }
    return Py_BuildValue("(NNN)", z, Pm, K);
}

// correct(mag[3], acc[3], z[4], P[4x4], K[4x4], acc0[3], mag0[3]) -> (X[4], P[4x4])
PyObject *py_correct(PyObject *, PyObject *args) {
    PyObject *o[7];
    if (!PyArg_UnpackTuple(args, "correct", 7, 7, &o[0], &o[1], &o[2], &o[3], &o[4], &o[5], &o[6])) return nullptr;
    In mag, acc, z, P, K, a0, m0;
    if (!mag.get(o[0], 3, "mag") || !acc.get(o[1], 3, "acc") || !z.get(o[2], 4, "z") || !P.get(o[3], 16, "P") ||
        !K.get(o[4], 16, "K") || !a0.get(o[5], 3, "acc0") || !m0.get(o[6], 3, "mag0"))
        return nullptr;
    PyObject *X = new_array(1, 4), *Po = new_array(2, 4, 4);
    if (!X || !Po) {
        Py_XDECREF(X); Py_XDECREF(Po);
        return nullptr;
    }
    int st;
    Py_BEGIN_ALLOW_THREADS
    st = pekf_correct(1, mag.p, acc.p, z.p, P.p, K.p, a0.p, m0.p, data(X), data(Po));
    Py_END_ALLOW_THREADS
    if (st) {
        Py_DECREF(X); Py_DECREF(Po);
        return fail(st);
    }
    return Py_BuildValue("(NN)", X, Po);
}

// wahba_quaternion(acc0[3], mag0[3], acc[3], mag[3], k_acc, k_mag) -> q[4]
PyObject *py_wahba_quaternion(PyObject *, PyObject *args) {
    PyObject *o[6];
    if (!PyArg_UnpackTuple(args, "wahba_quaternion", 6, 6, &o[0], &o[1], &o[2], &o[3], &o[4], &o[5]))
        return nullptr;
    In a0, m0, acc, mag, ka, km;
    if (!a0.get(o[0], 3, "acc0") || !m0.get(o[1], 3, "mag0") || !acc.get(o[2], 3, "acc") ||
        !mag.get(o[3], 3, "mag") || !ka.get(o[4], 1, "k_acc") || !km.get(o[5], 1, "k_mag"))
        return nullptr;
    PyObject *q = new_array(1, 4);
    if (!q) return nullptr;
    int st;
    Py_BEGIN_ALLOW_THREADS
    st = pekf_wahba_quaternion(1, a0.p, m0.p, acc.p, mag.p, ka.p, km.p, data(q));
    Py_END_ALLOW_THREADS
    if (st) {
        Py_DECREF(q);
        return fail(st);
    }
    return q;
}

PyMethodDef methods[] = {
    {"predict", py_predict, METH_VARARGS, "KalmanFilter.Prediction arithmetic for one record (pekf_predict, n = 1)."},
    {"correct", py_correct, METH_VARARGS, "KalmanFilter.Correction arithmetic for one record (pekf_correct, n = 1)."},
    {"wahba_quaternion", py_wahba_quaternion, METH_VARARGS,
     "Wahba.getQuarternion for one sample pair (pekf_wahba_quaternion, n = 1)."},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_fastcall",
                      "CPython binding of libpekf's n = 1 entry points used by the drop-in modules.", -1, methods,
                      nullptr, nullptr, nullptr, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__fastcall(void) {
    import_array();
    PyObject *linalg = PyImport_ImportModule("numpy.linalg");
    if (!linalg) return nullptr;
    g_linalg_error = PyObject_GetAttrString(linalg, "LinAlgError");
    Py_DECREF(linalg);
    if (!g_linalg_error) return nullptr;
    if (pekf_abi_version() != 1) {
        PyErr_SetString(PyExc_ImportError, "libpekf ABI mismatch");
        return nullptr;
    }
    return PyModule_Create(&module);
}
