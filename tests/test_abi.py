"""C-ABI boundary checks that need no GPU: the library loads, exports every
entry point include/rsgpu.h declares, follows upstream error precedence
before touching a device, and builds the same coding matrices as the
oracle.  (No compute calls succeed without a device: they must fail loudly
with RSGPU_ERR_NO_DEVICE — there is no CPU fallback.)"""
import ctypes
import re

import numpy as np
import pytest

import infinicache_amd as ia
import oracle
from infinicache_amd import _lib


def declared_functions():
    src = open(_lib.HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rsgpu_[a-z_]+)\s*\(", src)))


def test_header_declares_exports():
    assert declared_functions() == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol():
    L = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared_functions():
        assert hasattr(L, name), name


def test_library_has_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_error_codes_match_oracle_and_header():
    src = open(_lib.HEADER).read()
    codes = dict((m[0], int(m[1])) for m in re.findall(r"#define (RSGPU_ERR_\w+) (-?\d+)", src))
    assert codes["RSGPU_ERR_TOO_FEW_SHARDS"] == oracle.ERR_TOO_FEW_SHARDS == ia.ErrTooFewShards.code
    assert codes["RSGPU_ERR_SHARD_SIZE"] == oracle.ERR_SHARD_SIZE == ia.ErrShardSize.code
    assert codes["RSGPU_ERR_SHARD_NO_DATA"] == oracle.ERR_SHARD_NO_DATA == ia.ErrShardNoData.code
    assert codes["RSGPU_ERR_SINGULAR"] == oracle.ERR_SINGULAR == ia.ErrSingular.code
    assert codes["RSGPU_ERR_INV_SHARD_NUM"] == oracle.ERR_INV_SHARD_NUM == ia.ErrInvShardNum.code
    assert codes["RSGPU_ERR_MAX_SHARD_NUM"] == oracle.ERR_MAX_SHARD_NUM == ia.ErrMaxShardNum.code
    assert codes["RSGPU_ERR_INVALID_INPUT"] == oracle.ERR_INVALID_INPUT == ia.ErrInvalidInput.code
    L = _lib.load()
    for name, code in codes.items():
        assert L.rsgpu_strerror(code)


@pytest.mark.parametrize("kind", ["vandermonde", "cauchy", "par1"])
@pytest.mark.parametrize("k,p", [(1, 1), (4, 2), (10, 2), (10, 4), (17, 3), (128, 128)])
def test_matrix_matches_oracle(k, p, kind):
    enc = ia.New(k, p, matrix=kind)
    e, want = oracle.build_matrix(k, p, kind)
    assert e == 0
    assert np.array_equal(enc.matrix(), want)


def test_new_errors():
    with pytest.raises(ia.ErrInvShardNum):
        ia.New(0, 2)
    with pytest.raises(ia.ErrInvShardNum):
        ia.New(3, 0)
    with pytest.raises(ia.ErrInvShardNum):
        ia.New(-1, 2)
    with pytest.raises(ia.ErrMaxShardNum):
        ia.New(250, 7)
    ia.New(250, 6)  # exactly 256 is allowed


def test_error_precedence_without_device():
    """Length and checkShards errors come before any device work."""
    enc = ia.New(4, 2)
    with pytest.raises(ia.ErrTooFewShards):
        enc.Encode([bytearray(8)] * 5)
    with pytest.raises(ia.ErrShardSize):
        enc.Encode([bytearray(8)] * 5 + [None])
    with pytest.raises(ia.ErrShardNoData):
        enc.Encode([None] * 6)
    with pytest.raises(ia.ErrShardSize):
        enc.Verify([bytearray(8)] * 5 + [bytearray(7)])
    # fused Client.encode (Encode then Verify): Encode's checks, same order
    with pytest.raises(ia.ErrTooFewShards):
        enc.EncodeVerify([bytearray(8)] * 5)
    with pytest.raises(ia.ErrShardSize):
        enc.EncodeVerify([bytearray(8)] * 5 + [None])
    with pytest.raises(ia.ErrShardNoData):
        enc.EncodeVerify([None] * 6)
    with pytest.raises(ia.ErrTooFewShards):
        enc.Reconstruct([bytearray(8)] * 3 + [None] * 3)
    with pytest.raises(ia.ErrTooFewShards):
        enc.Update([bytearray(8)] * 6, [None] * 3)
    with pytest.raises(ia.ErrInvalidInput):
        enc.Update([None] + [bytearray(8)] * 5, [bytearray(8)] + [None] * 3)
    with pytest.raises(ia.ErrInvalidInput):
        enc.Update([bytearray(8)] * 5 + [None], [bytearray(8)] + [None] * 3)
    # all present -> Reconstruct is a no-op (no device needed), as upstream
    enc.Reconstruct([bytearray(8)] * 6)


@pytest.mark.skipif(ia.device_ok(0), reason="only meaningful on a host without the GPU")
def test_compute_fails_loudly_without_device():
    enc = ia.New(4, 2)
    with pytest.raises(ia.NoDevice):
        enc.Encode([bytearray(8)] * 6)
    with pytest.raises(ia.NoDevice):
        enc.Verify([bytearray(8)] * 6)
    with pytest.raises(ia.NoDevice):
        enc.EncodeVerify([bytearray(8)] * 6)
    with pytest.raises(ia.NoDevice):
        enc.Reconstruct([None] + [bytearray(8)] * 5)
    with pytest.raises(ia.NoDevice):
        enc.encode_dev(16, 8, 16, 96, 1)


def test_device_layout_validation():
    enc = ia.New(10, 2)
    with pytest.raises(ia.InvalidArgument):
        enc.encode_dev(0, 100, 112, 12 * 112, 1)        # NULL base
    with pytest.raises(ia.InvalidArgument):
        enc.encode_dev(4096, 100, 96, 12 * 96, 1)        # pitch < shard length
    with pytest.raises(ia.InvalidArgument):
        enc.encode_dev(4096, 100, 112, 112, 2)           # objects overlap
    with pytest.raises(ia.ErrShardNoData):
        enc.encode_dev(4096, 0, 112, 12 * 112, 1)
    # any alignment is a valid layout (byte-packed rows, unaligned base): such
    # a call gets as far as the device (ErrNoDevice on a CPU box)
    if not ia.device_ok(0):
        for args in ((4096 + 8, 100, 112, 12 * 112, 1), (4096, 100, 100, 12 * 100, 3)):
            with pytest.raises(ia.NoDevice):
                enc.encode_dev(*args)
    # the device-resolved mixed-pattern calls need 16-B aligned rows
    with pytest.raises(ia.InvalidArgument):
        enc.decode_dev_masks(4096, 8192, 100, 100, 12 * 100, 1, 16384)
    # rows spanning 4 GiB or more: a valid layout for the uniform calls
    # (coded in column slabs, launch_huge), not for the mixed-pattern ones
    big = 400 << 20
    if not ia.device_ok(0):
        with pytest.raises(ia.NoDevice):
            enc.encode_dev(4096, big, big, 12 * big, 1)
    with pytest.raises(ia.InvalidArgument):
        enc.decode_dev_masks(4096, 8192, big, big, 12 * big, 1, 16384)


@pytest.mark.parametrize("k,p", [(10, 2), (10, 4), (6, 3), (40, 20), (200, 50)])
def test_mixed_pattern_planning_without_device(k, p):
    """rsgpu_decode_dev_multi plans every object's pattern on the host before
    touching a device (present mask built eight flags per word, direct table
    for n <= 16 shards, open addressing up to 64, byte strings beyond): an
    object with fewer than k present shards is ErrTooFewShards wherever it
    sits in the batch and whatever nonzero values mark present flags; a valid
    batch gets as far as the device (ErrNoDevice here, on a CPU box)."""
    L = _lib.load()
    n = k + p
    enc = ia.New(k, p)
    rng = np.random.default_rng(n)
    nobj = 3000 if n <= 16 else 1000 if n <= 64 else 40  # distinct patterns cost one inverse each
    pm = np.ones((nobj, n), dtype=np.uint8)
    for o in range(nobj):  # lose 0..p shards, present flags any nonzero byte
        pm[o, rng.choice(n, int(rng.integers(0, p + 1)), replace=False)] = 0
        pm[o] *= rng.integers(1, 256, n, dtype=np.uint8)
    base = ctypes.c_void_p(1 << 20)  # never dereferenced: planning fails first or no device
    bad = ctypes.c_void_p(1 << 21)

    def call(m):
        m = np.ascontiguousarray(m)
        return L.rsgpu_decode_dev_multi(enc._ctx, base, m.ctypes.data_as(_lib.u8p), 64, 64, n * 64,
                                        nobj, bad, None)

    if not ia.device_ok(0):
        no_device = int(re.search(r"#define RSGPU_ERR_NO_DEVICE (-?\d+)", open(_lib.HEADER).read()).group(1))
        assert call(pm) == no_device
    for where in sorted({0, 7, 8, nobj // 2, nobj - 1}):
        m = pm.copy()
        m[where, :] = 0
        m[where, rng.choice(n, k - 1, replace=False)] = 0x80  # k-1 present
        assert call(m) == oracle.ERR_TOO_FEW_SHARDS, where


def test_multi_device_context_host_side():
    """rsgpu_create_multi / RSGPU_ALL_DEVICES need no device to be created
    (the matrix is host work); a device listed twice gives two independent
    entries; compute calls without a device fail loudly with ErrNoDevice,
    never on a CPU fallback."""
    L = _lib.load()
    ctx = ctypes.c_void_p()
    devs = (ctypes.c_int * 2)(0, 0)
    assert L.rsgpu_create_multi(10, 2, devs, 0, 0, ctypes.byref(ctx)) == -20  # no devices
    assert not ctx.value
    assert L.rsgpu_create_multi(0, 2, devs, 1, 0, ctypes.byref(ctx)) == oracle.ERR_INV_SHARD_NUM
    dup = ia.New(10, 2, devices=[0, 0, 0])
    assert dup.devices() == [0, 0, 0]
    assert dup.device_calls() == [0, 0, 0]
    enc = ia.New(10, 2, devices=[0])
    assert enc.devices() == [0]
    assert np.array_equal(enc.matrix(), ia.New(10, 2).matrix())
    allenc = ia.New(10, 2, device=ia.ALL_DEVICES)
    assert len(allenc.devices()) >= 1
    if not ia.device_ok(0):
        sh = [np.zeros(8, np.uint8) for _ in range(12)]
        with pytest.raises(ia.NoDevice):
            enc.Encode(sh)
        with pytest.raises(ia.NoDevice):
            allenc.Encode(sh)


def test_noncontiguous_output_buffer_rejected():
    """An output shard that is a strided view would be copied by the host
    mirror, the device writing into the copy: refused before any device work."""
    enc = ia.New(4, 2)
    big = np.zeros((6, 32), np.uint8)
    sh = [big[i] for i in range(4)] + [big[4, ::2], big[5, ::2]]  # strided parity rows
    sh = [s if i >= 4 else s[:16] for i, s in enumerate(sh)]
    with pytest.raises(ia.InvalidArgument):
        enc.Encode(sh)


def test_dev_objs_argument_checks():
    """rsgpu_*_dev_objs validate the whole table before any device work (no
    device needed): NULL base, zero shard_len, a pitch below roundup16(S)."""
    enc = ia.New(10, 2)
    with pytest.raises(ia.InvalidArgument):
        enc.encode_dev_objs([(0x1000, 100, 112), (0, 100, 112)])
    with pytest.raises(ia.ErrShardNoData):
        enc.encode_dev_objs([(0x1000, 0, 112)])
    with pytest.raises(ia.InvalidArgument):
        enc.encode_dev_objs([(0x1000, 100, 104)])  # pitch < roundup16(100)
    with pytest.raises(ia.ErrTooFewShards):
        enc.decode_dev_objs([(0x1000, 100, 112)], [0, 0, 0] + [1] * 9, 0x2000)
    with pytest.raises(ia.InvalidArgument):
        enc.decode_dev_objs([(0x1000, 100, 112)], [1] * 12, 0)  # no flag array


@pytest.mark.parametrize("S,nobj,stride", [(103, 1 << 20, 128), (100, 10, 112), (1, 5, 16), (410, 3, 512),
                                            (4096, 7, 4096), (4099, 2, 4224), (128, 1, 128), (17, 9, 32)])
def test_shardmajor_layout(S, nobj, stride):
    """rsgpu_shardmajor_layout (no device): whole 128-B lines when the gap is
    at most S/4 (the encode still codes the batch as one object), else 16-B
    aligned pieces; the pitch holds every piece, rounded up to 256."""
    st, pitch = ia.shardmajor_layout(S, nobj)
    assert st == stride
    assert pitch % 256 == 0 and pitch >= nobj * st and pitch - nobj * st < 256
    with pytest.raises(ia.ErrShardNoData):
        ia.shardmajor_layout(0, 4)


def test_copy_pieces_argument_checks():
    """rsgpu_copy_pieces validates before any device work: rows beyond the
    code, overlapping pieces (a stride below shard_len), zero shard_len;
    then fails loudly without a device."""
    enc = ia.New(10, 2)
    with pytest.raises(ia.InvalidArgument):
        enc.copy_pieces(0x1000, 1200, 12 * 1200, 0x100000, 4096, 128, 100, 4, rows=[12])
    with pytest.raises(ia.InvalidArgument):
        enc.copy_pieces(0x1000, 1200, 12 * 1200, 0x100000, 4096, 64, 100, 4)
    with pytest.raises(ia.ErrShardNoData):
        enc.copy_pieces(0x1000, 1200, 12 * 1200, 0x100000, 4096, 128, 0, 4)
    # rows that overlap: a shard-major destination whose pitch
    # is shorter than its objects' span (4 x 128-B pieces in a 400-B row)
    with pytest.raises(ia.InvalidArgument):
        enc.copy_pieces(0x1000, 1200, 12 * 1200, 0x100000, 400, 128, 100, 4)
    # object-major destination whose objects' rows run into the next object
    with pytest.raises(ia.InvalidArgument):
        enc.copy_pieces(0x1000, 1200, 12 * 1200, 0x100000, 128, 11 * 128, 100, 4)
    # ... and the same geometry on the source side
    with pytest.raises(ia.InvalidArgument):
        enc.copy_pieces(0x1000, 128, 11 * 128, 0x100000, 4096, 128, 100, 4)
    # a pitch below shard_len with two rows moving
    with pytest.raises(ia.InvalidArgument):
        enc.copy_pieces(0x1000, 1200, 12 * 1200, 0x100000, 64, 128 * 12, 100, 1, rows=[0, 1])
    # the rows that move decide: only row 0 of an 11-row object stride is fine
    if not ia.device_ok(0):
        with pytest.raises(ia.NoDevice):
            enc.copy_pieces(0x1000, 1200, 12 * 1200, 0x100000, 128, 11 * 128, 100, 4, rows=[0, 10])
    if not ia.device_ok(0):
        with pytest.raises(ia.NoDevice):
            enc.copy_pieces(0x1000, 1200, 12 * 1200, 0x100000, 4096, 128, 100, 4)


def test_diagnostics_and_knobs_without_device():
    """rsgpu_retired_stats / rsgpu_set_slab_bytes need no device: nothing is
    held back in a process that never started a worker, and the slab size
    setter accepts any value (< 4096 restores the 1 GiB default)."""
    st = ia.retired_stats()
    assert st == {"count": 0, "bytes": 0, "deferred": 0}
    for v in (0, 1, 4095, 4096, 1 << 20, 0):
        ia.set_slab_bytes(v)
