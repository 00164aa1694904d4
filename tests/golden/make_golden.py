"""Generates the committed golden fixtures under tests/golden/.

    python tests/golden/make_golden.py

Sources (no reference code is copied or executed — the Go reference cannot be
built offline):
  * kat.json: the upstream klauspost/reedsolomon v1.9.3 known-answer vectors
    recalled in SURVEY.md §8c (galois_test.go, matrix_test.go,
    reedsolomon_test.go) plus the RS(10+2)/RS(10+4) parity rows.  These PIN
    the oracles.
  * vectors.npz: parity of seeded small objects (data = splitmix64 bytes,
    regenerated from the stored seed index by oracle.rs_numpy.splitmix64_bytes(
    SEED, idx, k*size)) coded by the C oracle, cross-checked here against the independent numpy oracle before
    being written.  GPU tests compare the HIP path against these bytes.
  * digests.json: SHA-256 of the parity of seeded 1 MiB RS(10+2) and 4 MiB
    RS(10+4) objects (BASELINE configs 2/3 object shapes).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from oracle import rs_numpy as rn  # noqa: E402

SEED = 0x1F1C

KAT = {
    "gal_multiply": [[3, 4, 12], [7, 7, 21], [23, 45, 41]],
    "gal_exp": [[2, 2, 4], [5, 20, 235], [13, 7, 43]],
    "invert": {"in": [[56, 23, 98], [3, 100, 200], [45, 201, 123]],
               "out": [[175, 133, 33], [130, 13, 245], [112, 35, 126]]},
    "encode_5_5": {"data": [[0, 1], [4, 5], [2, 3], [6, 7], [8, 9]],
                   "parity": [[12, 13], [10, 11], [14, 15], [90, 91], [94, 95]]},
    "gal_mul_slice_25": {
        "in": [0, 1, 2, 3, 4, 5, 6, 10, 50, 100, 150, 174, 201, 255, 99, 32, 67, 85, 200, 199, 198,
               197, 196, 195, 194, 193, 192, 191, 190, 189, 188, 187, 186, 185],
        "out_hex": "0019322b647d56fab86dc785c31f220725feda5d446f7639200b121108233a756c47"},
    "parity_rows_10_2": ["8196afb8d2c4fee80302", "9681b8afc4d2e8fe0203"],
    "parity_rows_10_4_extra": ["bfd6620a066fdfb70504", "d6bf0a626f06b7df0405"],
}

# (k, p, matrix kind) x sizes
CONFIGS = [(10, 2, "vandermonde"), (10, 4, "vandermonde"), (5, 5, "vandermonde"),
           (4, 2, "cauchy"), (6, 3, "par1"), (17, 3, "vandermonde"), (10, 6, "vandermonde"),
           (1, 1, "vandermonde"), (3, 13, "vandermonde")]
SIZES = [1, 9, 103, 1023, 4096]


def main():
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(KAT, f, indent=1)

    arrays = {}
    idx = 0
    for (k, p, kind) in CONFIGS:
        e, m = oracle.build_matrix(k, p, kind)
        assert e == 0 and np.array_equal(m, rn.build_matrix(k, p, kind)), (k, p, kind)
        arrays[f"matrix_{k}_{p}_{kind}"] = m
        for size in SIZES:
            data = rn.splitmix64_bytes(SEED, idx, k * size).reshape(k, size)
            idx += 1
            e, sh = oracle.encode(k, p, [data[i] for i in range(k)] + [bytes(size)] * p, kind)
            assert e == 0
            par = np.stack(sh[k:])
            assert np.array_equal(par, rn.encode([data[i] for i in range(k)], p, kind)), (k, p, size)
            arrays[f"seedidx_{k}_{p}_{kind}_{size}"] = np.array([idx - 1])
            arrays[f"parity_{k}_{p}_{kind}_{size}"] = par
    np.savez_compressed(os.path.join(HERE, "vectors.npz"), **arrays)

    digests = {}
    for (k, p, n_bytes, tag) in [(10, 2, 1 << 20, "rs10_2_1MiB"), (10, 4, 4 << 20, "rs10_4_4MiB")]:
        for o in range(2):
            obj = rn.splitmix64_bytes(SEED, o, n_bytes)
            shards = rn.split(obj.tobytes(), k, p)
            e, m = oracle.build_matrix(k, p)
            par = oracle.code_fast(m[k:], shards[:k], nthreads=8)
            digests[f"{tag}_obj{o}"] = hashlib.sha256(b"".join(x.tobytes() for x in par)).hexdigest()
    with open(os.path.join(HERE, "digests.json"), "w") as f:
        json.dump(digests, f, indent=1)
    print("wrote", len(arrays), "arrays,", len(digests), "digests")


if __name__ == "__main__":
    main()
