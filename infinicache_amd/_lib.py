"""ctypes binding of librsgpu.so (the C ABI declared in include/rsgpu.h).

The shared library is built in-tree by infinicache_amd/csrc/Makefile (see
__graft_entry__.build()).  There is deliberately no fallback: if the library
is missing, importing the codec raises, and every compute call on a machine
without a gfx950 device returns RSGPU_ERR_NO_DEVICE.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "librsgpu.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "rsgpu.h")

# the exported entry points (kept in sync with include/rsgpu.h; tests check)
EXPORTS = (
    "rsgpu_create", "rsgpu_destroy", "rsgpu_data_shards", "rsgpu_parity_shards", "rsgpu_matrix",
    "rsgpu_strerror", "rsgpu_device_count", "rsgpu_device_ok", "rsgpu_encode", "rsgpu_verify",
    "rsgpu_reconstruct", "rsgpu_decode", "rsgpu_update", "rsgpu_encode_dev", "rsgpu_verify_dev",
    "rsgpu_reconstruct_dev", "rsgpu_decode_dev", "rsgpu_reconstruct_dev_multi",
    "rsgpu_decode_dev_multi", "rsgpu_encode_batch", "rsgpu_decode_batch",
    "rsgpu_host_register", "rsgpu_host_unregister", "rsgpu_host_alloc", "rsgpu_host_free",
    "rsgpu_encode_verify", "rsgpu_decode_dev_masks", "rsgpu_reconstruct_dev_masks",
    "rsgpu_create_multi", "rsgpu_devices", "rsgpu_encode_image", "rsgpu_encode_verify_image",
    "rsgpu_verify_image", "rsgpu_reconstruct_image", "rsgpu_decode_image", "rsgpu_device_calls",
    "rsgpu_encode_dev_objs", "rsgpu_verify_dev_objs", "rsgpu_reconstruct_dev_objs", "rsgpu_decode_dev_objs",
    "rsgpu_worker_start", "rsgpu_worker_stop", "rsgpu_worker_stats", "rsgpu_shardmajor_layout",
    "rsgpu_copy_pieces", "rsgpu_retired_stats", "rsgpu_set_slab_bytes",
)

u8p = ctypes.POINTER(ctypes.c_uint8)
u8pp = ctypes.POINTER(u8p)
szp = ctypes.POINTER(ctypes.c_size_t)
intp = ctypes.POINTER(ctypes.c_int)
vp = ctypes.c_void_p
sz = ctypes.c_size_t
ci = ctypes.c_int

_lib = None


class DevObj(ctypes.Structure):
    """rsgpu_dev_obj: one object of a variable-size device batch."""
    _fields_ = [("base", ctypes.c_void_p), ("shard_len", ctypes.c_size_t), ("pitch", ctypes.c_size_t)]


class LibraryMissing(RuntimeError):
    pass


def load():
    """Load librsgpu.so; raise LibraryMissing (loudly) if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise LibraryMissing(
            f"{LIB_PATH} not found: build it with `make -C infinicache_amd/csrc` "
            "(or python -c 'import __graft_entry__ as g; g.build()')")
    # One HIP runtime per process: PyTorch-ROCm wheels bundle their own
    # libamdhip64.so.7 (+ HSA runtime).  If torch is installed it is imported
    # first so librsgpu.so's NEEDED libamdhip64.so.7 binds to that already
    # loaded runtime (same SONAME); otherwise a second runtime initialised
    # before torch makes torch see no device.  Without torch (a C/Go host)
    # the library uses /opt/rocm's runtime via its RUNPATH.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    L.rsgpu_create.argtypes = [ci, ci, ci, ctypes.c_uint, ctypes.POINTER(vp)]
    L.rsgpu_create_multi.argtypes = [ci, ci, intp, ci, ctypes.c_uint, ctypes.POINTER(vp)]
    L.rsgpu_devices.argtypes = [vp, intp, ci]
    L.rsgpu_device_calls.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), ci]
    L.rsgpu_destroy.argtypes = [vp]
    L.rsgpu_destroy.restype = None
    L.rsgpu_data_shards.argtypes = [vp]
    L.rsgpu_parity_shards.argtypes = [vp]
    L.rsgpu_matrix.argtypes = [vp, u8p]
    L.rsgpu_strerror.argtypes = [ci]
    L.rsgpu_strerror.restype = ctypes.c_char_p
    L.rsgpu_device_count.argtypes = []
    L.rsgpu_device_ok.argtypes = [ci]
    L.rsgpu_encode.argtypes = [vp, u8pp, szp, ci]
    L.rsgpu_verify.argtypes = [vp, u8pp, szp, ci, intp]
    L.rsgpu_encode_verify.argtypes = [vp, u8pp, szp, ci, intp]
    L.rsgpu_reconstruct.argtypes = [vp, u8pp, szp, ci, ci]
    L.rsgpu_decode.argtypes = [vp, u8pp, szp, ci, intp]
    L.rsgpu_update.argtypes = [vp, u8pp, szp, ci, u8pp, szp, ci]
    L.rsgpu_encode_dev.argtypes = [vp, vp, sz, sz, sz, ci, vp]
    L.rsgpu_verify_dev.argtypes = [vp, vp, sz, sz, sz, ci, vp, vp]
    L.rsgpu_reconstruct_dev.argtypes = [vp, vp, u8p, sz, sz, sz, ci, ci, vp]
    L.rsgpu_decode_dev.argtypes = [vp, vp, u8p, sz, sz, sz, ci, vp, vp]
    L.rsgpu_reconstruct_dev_multi.argtypes = [vp, vp, u8p, sz, sz, sz, ci, ci, vp]
    L.rsgpu_decode_dev_multi.argtypes = [vp, vp, u8p, sz, sz, sz, ci, vp, vp]
    L.rsgpu_decode_dev_masks.argtypes = [vp, vp, vp, sz, sz, sz, ci, vp, vp]
    L.rsgpu_reconstruct_dev_masks.argtypes = [vp, vp, vp, sz, sz, sz, ci, ci, vp, vp]
    L.rsgpu_encode_image.argtypes = [vp, vp, sz, ci]
    L.rsgpu_encode_verify_image.argtypes = [vp, vp, sz, ci, intp]
    L.rsgpu_verify_image.argtypes = [vp, vp, sz, ci, intp]
    L.rsgpu_reconstruct_image.argtypes = [vp, vp, sz, ci, ctypes.c_uint64, ci]
    L.rsgpu_decode_image.argtypes = [vp, vp, sz, ci, ctypes.c_uint64, intp]
    L.rsgpu_encode_dev_objs.argtypes = [vp, vp, ci, vp]
    L.rsgpu_verify_dev_objs.argtypes = [vp, vp, ci, vp, vp]
    L.rsgpu_reconstruct_dev_objs.argtypes = [vp, vp, ci, u8p, ci, vp]
    L.rsgpu_decode_dev_objs.argtypes = [vp, vp, ci, u8p, vp, vp]
    L.rsgpu_worker_start.argtypes = [vp, ci, ctypes.c_uint, sz]
    L.rsgpu_worker_stop.argtypes = [vp]
    u64p = ctypes.POINTER(ctypes.c_uint64)
    L.rsgpu_worker_stats.argtypes = [vp, u64p, u64p, u64p]
    L.rsgpu_shardmajor_layout.argtypes = [sz, ci, szp, szp]
    L.rsgpu_copy_pieces.argtypes = [vp, vp, sz, sz, vp, sz, sz, sz, ci, ctypes.c_uint64, vp]
    L.rsgpu_encode_batch.argtypes = [vp, u8pp, szp, ci]
    L.rsgpu_decode_batch.argtypes = [vp, u8pp, u8p, szp, ci, intp]
    L.rsgpu_host_register.argtypes = [vp, sz]
    L.rsgpu_host_unregister.argtypes = [vp]
    L.rsgpu_host_alloc.argtypes = [sz, ctypes.POINTER(vp)]
    L.rsgpu_host_free.argtypes = [vp]
    L.rsgpu_retired_stats.argtypes = [szp, szp, u64p]
    L.rsgpu_set_slab_bytes.argtypes = [sz]
    _lib = L
    return L
