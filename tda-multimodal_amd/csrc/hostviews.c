// hostviews.c -- the host side of a batched call's result, in C.
//
// A batch of L layers comes back as one (T, 2) float64 pairs array; every
// layer's dgms is a list of maxdim + 1 views into it (ripser.py's result
// dict, debug_tda_pipeline.py:110 reads result['dgms'] per layer).  In
// Python that is L x (maxdim + 1) slices plus L LayerResult tuples, ~0.5 us
// a layer on the bench host -- a quarter of the host-input headline's time
// per layer, and all of it under the GIL that the pipeline's worker threads
// share.  The functions below make the same objects in one call each (and
// the result blob's arrays, and the input check).
//
//   segments(pairs, off, cnt, nd) -> [[pairs[o:o+c] for the nd dims] per layer]
//   layer_tuples(cls, batch, L)   -> [cls((batch, l)) for l in range(L)]
//   finite_ptrs(arrays)           -> the input parts' data pointers, after the
//                                    NaN / infinity check
//
// Host code only (CPython + numpy C API); no device calls.
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#define NPY_NO_DEPRECATED_API NPY_1_7_API_VERSION
#include <numpy/arrayobject.h>

static PyObject* segments(PyObject* self, PyObject* args) {
    (void)self;
    PyArrayObject *pairs, *off, *cnt;
    Py_ssize_t nd;
    if (!PyArg_ParseTuple(args, "O!O!O!n", &PyArray_Type, &pairs, &PyArray_Type, &off, &PyArray_Type, &cnt, &nd))
        return NULL;
    if (PyArray_NDIM(pairs) != 2 || PyArray_DIM(pairs, 1) != 2 || PyArray_TYPE(pairs) != NPY_FLOAT64) {
        PyErr_SetString(PyExc_ValueError, "pairs must be a (T, 2) float64 array");
        return NULL;
    }
    if (PyArray_NDIM(off) != 1 || PyArray_NDIM(cnt) != 1 || PyArray_TYPE(off) != NPY_INT64 || PyArray_TYPE(cnt) != NPY_INT64 ||
        PyArray_DIM(off, 0) != PyArray_DIM(cnt, 0) || !PyArray_IS_C_CONTIGUOUS(off) || !PyArray_IS_C_CONTIGUOUS(cnt)) {
        PyErr_SetString(PyExc_ValueError, "off / cnt must be contiguous int64 arrays of one length");
        return NULL;
    }
    const Py_ssize_t S = PyArray_DIM(off, 0);
    if (nd <= 0 || S % nd != 0) {
        PyErr_SetString(PyExc_ValueError, "the segment count must be a multiple of nd");
        return NULL;
    }
    const npy_int64* o = (const npy_int64*)PyArray_DATA(off);
    const npy_int64* c = (const npy_int64*)PyArray_DATA(cnt);
    const npy_intp T = PyArray_DIM(pairs, 0);
    for (Py_ssize_t s = 0; s < S; ++s)
        if (o[s] < 0 || c[s] < 0 || o[s] > T || c[s] > T - o[s]) {
            PyErr_SetString(PyExc_ValueError, "segment out of the pairs array");
            return NULL;
        }
    char* base = PyArray_BYTES(pairs);
    npy_intp strides[2] = {PyArray_STRIDE(pairs, 0), PyArray_STRIDE(pairs, 1)};
    const int flags = PyArray_FLAGS(pairs) & (NPY_ARRAY_WRITEABLE | NPY_ARRAY_ALIGNED);
    PyArray_Descr* descr = PyArray_DESCR(pairs);
    const Py_ssize_t L = S / nd;
    PyObject* out = PyList_New(L);
    if (!out) return NULL;
    for (Py_ssize_t l = 0; l < L; ++l) {
        PyObject* lst = PyList_New(nd);
        if (!lst) goto fail;
        PyList_SET_ITEM(out, l, lst);
        for (Py_ssize_t k = 0; k < nd; ++k) {
            const Py_ssize_t s = l * nd + k;
            npy_intp dims[2] = {(npy_intp)c[s], 2};
            Py_INCREF(descr);  // stolen by NewFromDescr
            PyObject* v = PyArray_NewFromDescr(&PyArray_Type, descr, 2, dims, strides, base + (npy_intp)o[s] * strides[0], flags, NULL);
            if (!v) goto fail;
            Py_INCREF(pairs);  // stolen by SetBaseObject (which walks to the owner of the data, as slicing does)
            if (PyArray_SetBaseObject((PyArrayObject*)v, (PyObject*)pairs) < 0) {
                Py_DECREF(v);
                goto fail;
            }
            PyList_SET_ITEM(lst, k, v);
        }
    }
    return out;
fail:
    Py_DECREF(out);
    return NULL;
}

static PyObject* layer_tuples(PyObject* self, PyObject* args) {
    (void)self;
    PyTypeObject* cls;
    PyObject* batch;
    Py_ssize_t L;
    if (!PyArg_ParseTuple(args, "O!On", &PyType_Type, &cls, &batch, &L)) return NULL;
    if (!PyType_IsSubtype(cls, &PyTuple_Type) || L < 0) {
        PyErr_SetString(PyExc_TypeError, "cls must be a tuple subclass and L >= 0");
        return NULL;
    }
    PyObject* out = PyList_New(L);
    if (!out) return NULL;
    for (Py_ssize_t l = 0; l < L; ++l) {
        // what tuple.__new__ does for a subclass: tp_alloc(cls, n), then the items
        PyObject* t = cls->tp_alloc(cls, 2);
        if (!t) goto fail;
        PyObject* li = PyLong_FromSsize_t(l);
        if (!li) {
            Py_DECREF(t);
            goto fail;
        }
        Py_INCREF(batch);
        PyTuple_SET_ITEM(t, 0, batch);
        PyTuple_SET_ITEM(t, 1, li);
        PyList_SET_ITEM(out, l, t);
    }
    return out;
fail:
    Py_DECREF(out);
    return NULL;
}

// every element finite: no exponent field of all ones (NaN and +-inf)
static int all_finite(const char* p, npy_intp n, int f64) {
    unsigned bad = 0;
    if (f64) {
        const npy_uint64* q = (const npy_uint64*)p;
        for (npy_intp i = 0; i < n; ++i) bad |= (unsigned)((q[i] & 0x7FF0000000000000ull) == 0x7FF0000000000000ull);
    } else {
        const npy_uint32* q = (const npy_uint32*)p;
        for (npy_intp i = 0; i < n; ++i) bad |= (unsigned)((q[i] & 0x7F800000u) == 0x7F800000u);
    }
    return !bad;
}

// finite_ptrs(arrays) -> [data pointer of each]: the host input parts of one
// call (contiguous float32 / float64 numpy arrays), after ripser.py's
// "Input contains NaN or infinity." check over all of them
static PyObject* finite_ptrs(PyObject* self, PyObject* arg) {
    (void)self;
    PyObject* seq = PySequence_Fast(arg, "finite_ptrs needs a sequence of arrays");
    if (!seq) return NULL;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
    PyObject** items = PySequence_Fast_ITEMS(seq);
    PyObject* out = PyList_New(n);
    if (!out) {
        Py_DECREF(seq);
        return NULL;
    }
    for (Py_ssize_t i = 0; i < n; ++i) {
        if (!PyArray_Check(items[i])) {
            PyErr_SetString(PyExc_TypeError, "finite_ptrs: not a numpy array");
            goto fail;
        }
        PyArrayObject* a = (PyArrayObject*)items[i];
        const int t = PyArray_TYPE(a);
        if ((t != NPY_FLOAT32 && t != NPY_FLOAT64) || !PyArray_IS_C_CONTIGUOUS(a)) {
            PyErr_SetString(PyExc_TypeError, "finite_ptrs: arrays must be contiguous float32 / float64");
            goto fail;
        }
        if (!all_finite(PyArray_BYTES(a), PyArray_SIZE(a), t == NPY_FLOAT64)) {
            PyErr_SetString(PyExc_ValueError, "Input contains NaN or infinity.");
            goto fail;
        }
        PyObject* p = PyLong_FromVoidPtr(PyArray_DATA(a));
        if (!p) goto fail;
        PyList_SET_ITEM(out, i, p);
    }
    Py_DECREF(seq);
    return out;
fail:
    Py_DECREF(seq);
    Py_DECREF(out);
    return NULL;
}

// a C-contiguous view of `base`'s data at byte offset `off` (read-only unless `writeable`)
static PyObject* view_of(PyArrayObject* base, int type, Py_ssize_t off, int nd, npy_intp* dims, int writeable) {
    PyArray_Descr* d = PyArray_DescrFromType(type);  // new reference, stolen below
    PyObject* v = PyArray_NewFromDescr(&PyArray_Type, d, nd, dims, NULL, PyArray_BYTES(base) + off,
                                       NPY_ARRAY_ALIGNED | (writeable ? NPY_ARRAY_WRITEABLE : 0), NULL);
    if (!v) return NULL;
    Py_INCREF(base);
    if (PyArray_SetBaseObject((PyArrayObject*)v, (PyObject*)base) < 0) {
        Py_DECREF(v);
        return NULL;
    }
    return v;
}

// blob_arrays(address, nbytes, L, nd, total) -> (cnt, off, cs, na, nc, nr, nadd, ne, bidx, didx,
// thr, pairs): one copy of a result blob (include/tda_rips.h: meta[7][L][nd] | num_edges[L] |
// birth_idx[T], death_idx[T] | thresh[L] f32 (padded to 8 B) | birth[T], death[T] f32) and the
// read-only views ripser.py's _unpack made of it with a dozen numpy calls, plus the (T, 2) float64
// pairs every dgms view points into
static PyObject* blob_arrays(PyObject* self, PyObject* args) {
    (void)self;
    unsigned long long addr;
    Py_ssize_t nbytes, L, nd, T;
    if (!PyArg_ParseTuple(args, "Knnnn", &addr, &nbytes, &L, &nd, &T)) return NULL;
    const Py_ssize_t S = L * nd, o_ne = 7 * S, o_idx = o_ne + L, o_thr = o_idx + 2 * T, o_bd = o_thr + (L + 1) / 2;
    if (L < 0 || nd <= 0 || T < 0 || nbytes != 8 * (o_bd + T) || (!addr && nbytes)) {
        PyErr_SetString(PyExc_ValueError, "blob_arrays: size does not match the blob layout");
        return NULL;
    }
    npy_intp wd[1] = {(npy_intp)(o_bd + T)};
    PyArrayObject* w = (PyArrayObject*)PyArray_SimpleNew(1, wd, NPY_INT64);
    if (!w) return NULL;
    if (nbytes) memcpy(PyArray_DATA(w), (const void*)(uintptr_t)addr, (size_t)nbytes);
    npy_intp pdim[2] = {(npy_intp)T, 2};
    PyArrayObject* pairs = (PyArrayObject*)PyArray_SimpleNew(2, pdim, NPY_FLOAT64);
    if (!pairs) {
        Py_DECREF(w);
        return NULL;
    }
    {
        const float* bd = (const float*)(PyArray_BYTES(w) + 8 * o_bd);
        double* P = (double*)PyArray_DATA(pairs);
        for (Py_ssize_t i = 0; i < T; ++i) {
            P[2 * i] = (double)bd[i];
            P[2 * i + 1] = (double)bd[T + i];
        }
    }
    npy_intp md[2] = {(npy_intp)L, (npy_intp)nd}, ld[1] = {(npy_intp)L}, td[1] = {(npy_intp)T};
    PyObject* t = PyTuple_New(12);
    if (!t) {
        Py_DECREF(pairs);
        Py_DECREF(w);
        return NULL;
    }
    PyTuple_SET_ITEM(t, 11, (PyObject*)pairs);
    // (type, byte offset, rank, dims) of the eleven views: meta[7] (checksums unsigned), num_edges,
    // birth_idx, death_idx, thresh
    const int types[11] = {NPY_INT64, NPY_INT64, NPY_UINT64, NPY_INT64, NPY_INT64, NPY_INT64, NPY_INT64,
                           NPY_INT64, NPY_INT64, NPY_INT64, NPY_FLOAT32};
    const Py_ssize_t offs[11] = {0, 8 * S, 16 * S, 24 * S, 32 * S, 40 * S, 48 * S, 8 * o_ne, 8 * o_idx, 8 * (o_idx + T), 8 * o_thr};
    for (int k = 0; k < 11; ++k) {
        PyObject* v = view_of(w, types[k], offs[k], k < 7 ? 2 : 1, k < 7 ? md : (k == 8 || k == 9) ? td : ld, 0);
        if (!v) {
            Py_DECREF(t);  // releases pairs and the views made so far
            Py_DECREF(w);
            return NULL;
        }
        PyTuple_SET_ITEM(t, k, v);
    }
    Py_DECREF(w);  // the views hold it
    return t;
}

static PyMethodDef kMethods[] = {
    {"blob_arrays", blob_arrays, METH_VARARGS, "blob_arrays(address, nbytes, L, nd, total): a result blob's arrays, one copy"},
    {"finite_ptrs", finite_ptrs, METH_O, "finite_ptrs(arrays): data pointers of contiguous float arrays, all elements finite"},
    {"segments", segments, METH_VARARGS, "segments(pairs, off, cnt, nd): per-layer lists of nd views pairs[o:o+c]"},
    {"layer_tuples", layer_tuples, METH_VARARGS, "layer_tuples(cls, batch, L): [cls((batch, l)) for l in range(L)]"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_hostviews", NULL, -1, kMethods};

PyMODINIT_FUNC PyInit__hostviews(void) {
    import_array();
    return PyModule_Create(&kModule);
}
