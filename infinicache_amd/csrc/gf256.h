// gf256.h — host-side GF(2^8) arithmetic and coding matrices for the product
// library (the oracle under oracle/ is a separate, independent restatement).
//
// Field and matrices follow klauspost/reedsolomon v1.9.3 (the codec behind
// /root/reference/client/ec.go:19): polynomial 0x11D, generator 2;
// galExp(a, n) with 0^0 = 1; default matrix = vandermonde(n, k) x top^-1
// (reedsolomon.go buildMatrix); Cauchy = identity over 1/(r ^ c)
// (buildMatrixCauchy); PAR1 = identity over (c+1)^(r-k) (buildMatrixPAR1).
#pragma once
#include <cstdint>
#include <cstring>
#include <vector>

namespace rsgpu {

struct GF {
    uint8_t exp[512];
    uint8_t log[256];
    GF() {
        unsigned x = 1;
        for (int i = 0; i < 255; ++i) {
            exp[i] = (uint8_t)x;
            log[x] = (uint8_t)i;
            x <<= 1;
            if (x & 0x100) x ^= 0x11D;
        }
        for (int i = 255; i < 512; ++i) exp[i] = exp[i - 255];
        log[0] = 0;
    }
    uint8_t mul(uint8_t a, uint8_t b) const {
        return (a == 0 || b == 0) ? 0 : exp[log[a] + log[b]];
    }
    uint8_t div(uint8_t a, uint8_t b) const {  // b != 0
        if (a == 0) return 0;
        int l = (int)log[a] - (int)log[b];
        return exp[l < 0 ? l + 255 : l];
    }
    uint8_t pow(uint8_t a, int n) const {
        if (n == 0) return 1;
        if (a == 0) return 0;
        return exp[(log[a] * n) % 255];
    }
};

const GF &gf();

// n x n inverse by Gauss-Jordan; returns false when singular.
bool gf_invert(const uint8_t *in, int n, uint8_t *out);

// (k+p) x k coding matrix for kind 0 (Vandermonde), 1 (Cauchy), 2 (PAR1).
// Returns false if the top square is singular (cannot happen for kind 0).
bool gf_build_matrix(int k, int p, unsigned kind, std::vector<uint8_t> &out);

}  // namespace rsgpu
