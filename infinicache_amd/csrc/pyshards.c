/* pyshards.c — the Python mirror's per-object call marshalling, in C.
 *
 * ec.py's per-object methods (Encode, Verify, EncodeVerify, Reconstruct,
 * ReconstructData, DecodeVerify: the calls Client.encode / Client.decode make,
 * client/ecRedis.go:382-432) pass a table of shard pointers and lengths to
 * the C ABI (include/rsgpu.h).  Building that table through ctypes costs
 * ~50 us per call on this image's CPUs (numpy's __array_interface__ alone
 * ~2.4 us per shard) — several times the resident worker's whole 1 KiB call.
 * Here the table is filled through the buffer protocol and the rsgpu entry
 * point (its address taken from the ctypes handle) is called directly, with
 * the GIL released.  No coding happens here: this is argument plumbing for
 * librsgpu.so, and a missing module only means ec.py marshals with ctypes.
 *
 *   call(fn, ctx, shards, wlo, whi, missing, kind, arg)
 *     fn       address of an rsgpu per-object entry point
 *     ctx      rsgpu_ctx* (int)
 *     shards   list / tuple of buffers or None (None, or an empty buffer: length 0)
 *     [wlo, whi)  indices whose buffers the call writes (must be writable)
 *     missing  sequence of indices passed with length 0 although they hold a
 *              buffer (reconstruct's outputs; writable), or None
 *     kind 0:  rc = fn(ctx, ptrs, lens, n, arg)             -> rc
 *     kind 1:  rc = fn(ctx, ptrs, lens, n, &ok)             -> (rc, ok)
 *     kind 2:  rc = fn(ctx, ptrs, lens, n)                  -> rc
 *   Returns None (nothing called) when a buffer cannot be taken as one
 *   contiguous byte range (non-contiguous, read-only output, ...): ec.py then
 *   takes its ctypes path, which copies or raises exactly as before. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <stdint.h>
#include <string.h>

typedef int (*fn_4_t)(void *, uint8_t *const *, const size_t *, int);
typedef int (*fn_arg_t)(void *, uint8_t *const *, const size_t *, int, int);
typedef int (*fn_out_t)(void *, uint8_t *const *, const size_t *, int, int *);

enum { kMaxShards = 256 };

static PyObject *call(PyObject *self, PyObject *args) {
    (void)self;
    unsigned long long fn_addr = 0, ctx_addr = 0;
    PyObject *shards = NULL, *missing = NULL;
    int wlo = 0, whi = 0, kind = 0, arg = 0;
    if (!PyArg_ParseTuple(args, "KKOiiOii", &fn_addr, &ctx_addr, &shards, &wlo, &whi, &missing, &kind, &arg))
        return NULL;
    if (!fn_addr || kind < 0 || kind > 2) {
        PyErr_SetString(PyExc_ValueError, "pyshards.call: bad function or kind");
        return NULL;
    }
    PyObject *seq = PySequence_Fast(shards, "shards must be a sequence");
    if (!seq) return NULL;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
    if (n < 0 || n > kMaxShards) {
        Py_DECREF(seq);
        Py_RETURN_NONE;  /* (the ctypes path reports the upstream error) */
    }
    unsigned char zero[kMaxShards], wr[kMaxShards];
    memset(zero, 0, sizeof zero);
    memset(wr, 0, sizeof wr);
    for (Py_ssize_t i = wlo; i < whi && i < n; ++i)
        if (i >= 0) wr[i] = 1;
    if (missing && missing != Py_None) {
        PyObject *ms = PySequence_Fast(missing, "missing must be a sequence");
        if (!ms) {
            Py_DECREF(seq);
            return NULL;
        }
        for (Py_ssize_t j = 0; j < PySequence_Fast_GET_SIZE(ms); ++j) {
            const long i = PyLong_AsLong(PySequence_Fast_GET_ITEM(ms, j));
            if (i == -1 && PyErr_Occurred()) {
                Py_DECREF(ms);
                Py_DECREF(seq);
                return NULL;
            }
            if (i >= 0 && i < n) zero[i] = wr[i] = 1;
        }
        Py_DECREF(ms);
    }
    Py_buffer views[kMaxShards];
    unsigned char held[kMaxShards];
    memset(held, 0, sizeof held);
    uint8_t *ptrs[kMaxShards];
    size_t lens[kMaxShards];
    int ok_all = 1;
    for (Py_ssize_t i = 0; i < n; ++i) {
        ptrs[i] = NULL;
        lens[i] = 0;
        PyObject *o = PySequence_Fast_GET_ITEM(seq, i);
        if (o == Py_None) continue;
        /* PyBUF_SIMPLE: one C-contiguous byte range or BufferError */
        if (PyObject_GetBuffer(o, &views[i], wr[i] ? PyBUF_WRITABLE : PyBUF_SIMPLE) != 0) {
            PyErr_Clear();
            ok_all = 0;
            break;
        }
        held[i] = 1;
        if (views[i].len > 0) {
            ptrs[i] = (uint8_t *)views[i].buf;
            lens[i] = zero[i] ? 0 : (size_t)views[i].len;
        }
    }
    PyObject *ret = NULL;
    if (ok_all) {
        int rc = 0, ok = 0;
        Py_BEGIN_ALLOW_THREADS
        void *const c = (void *)(uintptr_t)ctx_addr;
        if (kind == 0)
            rc = ((fn_arg_t)(uintptr_t)fn_addr)(c, ptrs, lens, (int)n, arg);
        else if (kind == 1)
            rc = ((fn_out_t)(uintptr_t)fn_addr)(c, ptrs, lens, (int)n, &ok);
        else
            rc = ((fn_4_t)(uintptr_t)fn_addr)(c, ptrs, lens, (int)n);
        Py_END_ALLOW_THREADS
        ret = kind == 1 ? Py_BuildValue("(ii)", rc, ok) : PyLong_FromLong(rc);
    } else {
        Py_INCREF(Py_None);
        ret = Py_None;
    }
    for (Py_ssize_t i = 0; i < n; ++i)
        if (held[i]) PyBuffer_Release(&views[i]);
    Py_DECREF(seq);
    return ret;
}

static PyMethodDef methods[] = {
    {"call", call, METH_VARARGS, "marshal a shard table and call an rsgpu per-object entry point"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_pyshards", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__pyshards(void) { return PyModule_Create(&module); }
