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

/* ---- batches: rsgpu_encode_batch / rsgpu_decode_batch (ec.py encode_batch,
 * decode_batch with `present`).  A 512-object batch took ~50-66 ms of ctypes
 * marshalling per call on this image's CPUs, inside config 5's timed step.
 * Any entry that is not plainly valid (wrong shard count, sizes that differ,
 * rows that are not one Split array, a read-only output, None) returns None
 * and ec.py's ctypes path raises the same error it always did. */
typedef int (*fn_enc_batch_t)(void *, uint8_t *const *, const size_t *, int);
typedef int (*fn_dec_batch_t)(void *, uint8_t *const *, const uint8_t *, const size_t *, int, int *);

struct Views {
    Py_buffer *v;
    Py_ssize_t n;
};
static void views_release(struct Views *vs) {
    for (Py_ssize_t i = 0; i < vs->n; ++i) PyBuffer_Release(&vs->v[i]);
    PyMem_Free(vs->v);
    vs->v = NULL;
    vs->n = 0;
}
/* one more writable (or read-only) contiguous view, or 0 */
static int views_take(struct Views *vs, PyObject *o, int writable) {
    if (o == Py_None) return 0;
    if (PyObject_GetBuffer(o, &vs->v[vs->n], writable ? PyBUF_WRITABLE : PyBUF_SIMPLE) != 0) {
        PyErr_Clear();
        return 0;
    }
    ++vs->n;
    return 1;
}

/* encode_batch(fn, ctx, objs, nshards) -> rc | None */
static PyObject *encode_batch(PyObject *self, PyObject *args) {
    (void)self;
    unsigned long long fn_addr = 0, ctx_addr = 0;
    PyObject *objs = NULL;
    int n = 0;
    if (!PyArg_ParseTuple(args, "KKOi", &fn_addr, &ctx_addr, &objs, &n)) return NULL;
    if (!fn_addr || n < 1 || n > kMaxShards) Py_RETURN_NONE;
    PyObject *seq = PySequence_Fast(objs, "objs must be a sequence");
    if (!seq) return NULL;
    const Py_ssize_t nobj = PySequence_Fast_GET_SIZE(seq);
    struct Views vs = {PyMem_Malloc(sizeof(Py_buffer) * (size_t)(nobj * n + 1)), 0};
    uint8_t **ptrs = PyMem_Malloc(sizeof(uint8_t *) * (size_t)(nobj + 1));
    size_t *lens = PyMem_Malloc(sizeof(size_t) * (size_t)(nobj + 1));
    int fine = vs.v && ptrs && lens;
    for (Py_ssize_t o = 0; o < nobj && fine; ++o) {
        PyObject *e = PySequence_Fast_GET_ITEM(seq, o);
        if (PyList_Check(e) || PyTuple_Check(e)) {
            PyObject *rows = PySequence_Fast(e, "");
            if (!rows) {
                PyErr_Clear();
                fine = 0;
                break;
            }
            if (PySequence_Fast_GET_SIZE(rows) != n) fine = 0;
            const Py_ssize_t first = vs.n;
            for (int i = 0; i < n && fine; ++i) {
                if (!views_take(&vs, PySequence_Fast_GET_ITEM(rows, i), 1)) {
                    fine = 0;
                    break;
                }
                const Py_buffer *r0 = &vs.v[first], *ri = &vs.v[vs.n - 1];
                if (ri->len != r0->len || (const char *)ri->buf != (const char *)r0->buf + (size_t)i * (size_t)r0->len)
                    fine = 0;
            }
            Py_DECREF(rows);
            if (!fine) break;
            ptrs[o] = (uint8_t *)vs.v[first].buf;
            lens[o] = (size_t)vs.v[first].len;
        } else {
            if (!views_take(&vs, e, 1)) {
                fine = 0;
                break;
            }
            const Py_buffer *b = &vs.v[vs.n - 1];
            if (b->len % n) {
                fine = 0;
                break;
            }
            ptrs[o] = (uint8_t *)b->buf;
            lens[o] = (size_t)(b->len / n);
        }
        if (lens[o] == 0) fine = 0;  /* (upstream ErrShardNoData: the ctypes path reports it) */
    }
    PyObject *ret;
    if (fine) {
        int rc;
        Py_BEGIN_ALLOW_THREADS
        rc = ((fn_enc_batch_t)(uintptr_t)fn_addr)((void *)(uintptr_t)ctx_addr, ptrs, lens, (int)nobj);
        Py_END_ALLOW_THREADS
        ret = PyLong_FromLong(rc);
    } else {
        Py_INCREF(Py_None);
        ret = Py_None;
    }
    views_release(&vs);
    PyMem_Free(ptrs);
    PyMem_Free(lens);
    Py_DECREF(seq);
    return ret;
}

/* decode_batch(fn, ctx, objs, present, nshards) -> (rc, [ok...]) | None */
static PyObject *decode_batch(PyObject *self, PyObject *args) {
    (void)self;
    unsigned long long fn_addr = 0, ctx_addr = 0;
    PyObject *objs = NULL, *present = NULL;
    int n = 0;
    if (!PyArg_ParseTuple(args, "KKOOi", &fn_addr, &ctx_addr, &objs, &present, &n)) return NULL;
    if (!fn_addr || n < 1 || n > kMaxShards) Py_RETURN_NONE;
    PyObject *seq = PySequence_Fast(objs, "objs must be a sequence");
    if (!seq) return NULL;
    PyObject *pseq = PySequence_Fast(present, "present must be a sequence");
    if (!pseq) {
        Py_DECREF(seq);
        return NULL;
    }
    const Py_ssize_t nobj = PySequence_Fast_GET_SIZE(seq);
    int fine = PySequence_Fast_GET_SIZE(pseq) >= nobj;
    struct Views vs = {PyMem_Malloc(sizeof(Py_buffer) * (size_t)(nobj * n + 1)), 0};
    uint8_t **ptrs = PyMem_Malloc(sizeof(uint8_t *) * (size_t)(nobj * n + 1));
    uint8_t *pres = PyMem_Malloc((size_t)(nobj * n + 1));
    size_t *lens = PyMem_Malloc(sizeof(size_t) * (size_t)(nobj + 1));
    int *ok = PyMem_Malloc(sizeof(int) * (size_t)(nobj + 1));
    fine = fine && vs.v && ptrs && pres && lens && ok;
    for (Py_ssize_t o = 0; o < nobj && fine; ++o) {
        PyObject *rows = PySequence_Fast(PySequence_Fast_GET_ITEM(seq, o), "");
        PyObject *prow = rows ? PySequence_Fast(PySequence_Fast_GET_ITEM(pseq, o), "") : NULL;
        if (!rows || !prow) {
            PyErr_Clear();
            Py_XDECREF(rows);
            fine = 0;
            break;
        }
        if (PySequence_Fast_GET_SIZE(rows) != n || PySequence_Fast_GET_SIZE(prow) < n) fine = 0;
        Py_ssize_t S = -1;
        for (int i = 0; i < n && fine; ++i) {
            const int t = PyObject_IsTrue(PySequence_Fast_GET_ITEM(prow, i));
            if (t < 0) {
                PyErr_Clear();
                fine = 0;
                break;
            }
            pres[o * n + i] = (uint8_t)t;
            if (!views_take(&vs, PySequence_Fast_GET_ITEM(rows, i), !t)) {  /* absent rows are outputs */
                fine = 0;
                break;
            }
            const Py_buffer *b = &vs.v[vs.n - 1];
            if (S < 0) S = b->len;
            if (b->len != S || S == 0) fine = 0;
            ptrs[o * n + i] = (uint8_t *)b->buf;
        }
        Py_DECREF(prow);
        Py_DECREF(rows);
        lens[o] = S > 0 ? (size_t)S : 0;
    }
    PyObject *ret;
    if (fine) {
        int rc;
        Py_BEGIN_ALLOW_THREADS
        rc = ((fn_dec_batch_t)(uintptr_t)fn_addr)((void *)(uintptr_t)ctx_addr, ptrs, pres, lens, (int)nobj, ok);
        Py_END_ALLOW_THREADS
        PyObject *oks = PyList_New(nobj);
        for (Py_ssize_t o = 0; oks && o < nobj; ++o) PyList_SET_ITEM(oks, o, PyBool_FromLong(rc == 0 && ok[o]));
        ret = oks ? Py_BuildValue("(iN)", rc, oks) : NULL;
    } else {
        Py_INCREF(Py_None);
        ret = Py_None;
    }
    views_release(&vs);
    PyMem_Free(ptrs);
    PyMem_Free(pres);
    PyMem_Free(lens);
    PyMem_Free(ok);
    Py_DECREF(pseq);
    Py_DECREF(seq);
    return ret;
}

static PyMethodDef methods[] = {
    {"call", call, METH_VARARGS, "marshal a shard table and call an rsgpu per-object entry point"},
    {"encode_batch", encode_batch, METH_VARARGS, "marshal a batch of Split images and call rsgpu_encode_batch"},
    {"decode_batch", decode_batch, METH_VARARGS, "marshal a batch of Gets (with present flags) and call rsgpu_decode_batch"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_pyshards", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__pyshards(void) { return PyModule_Create(&module); }
