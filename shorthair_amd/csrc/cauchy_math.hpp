// Host-side GF(256)/0x187 arithmetic and generator-matrix construction.
//
// This is the per-batch SETUP of the codec (a few KB of tables per (k, m)); the bulk data path
// runs on the GPU. Field: GF(2^8) with polynomial 0x187 and generator 2, as the reference codec
// (catid/shorthair cauchy_256.cpp:271-413). Log/exp/inverse tables are computed from the
// polynomial here; only the searched generator tables (cauchy_tables_data.h) are data.
#pragma once

#include <array>
#include <cstdint>
#include <cstring>
#include <vector>

#include "cauchy_tables_data.h"

namespace sh {

struct GF256 {
    uint8_t exp[512];
    uint16_t log[256];
    uint8_t inv[256];
    // row_bytes[c][b] = c * 2^b: row b of the 8x8 GF(2) submatrix of element c
    // (reference expansion, cauchy_256.cpp:1553-1568: "slice = GFC256Multiply(slice, 2)").
    uint8_t row_bytes[256][8];

    GF256() {
        unsigned x = 1;
        for (int i = 0; i < 255; ++i) {
            exp[i] = exp[i + 255] = static_cast<uint8_t>(x);
            log[x] = static_cast<uint16_t>(i);
            x <<= 1;
            if (x & 0x100) x ^= 0x187;
        }
        exp[510] = exp[511] = 0;
        log[0] = 0;
        inv[0] = 0;
        for (int i = 1; i < 256; ++i) inv[i] = exp[(255 - log[i]) % 255];
        for (int c = 0; c < 256; ++c) {
            uint8_t s = static_cast<uint8_t>(c);
            for (int b = 0; b < 8; ++b) {
                row_bytes[c][b] = s;
                s = mul(s, 2);
            }
        }
    }
    uint8_t mul(uint8_t a, uint8_t b) const { return (a && b) ? exp[log[a] + log[b]] : 0; }
    // x / y, 0 when either is 0 (the reference's DIV table is zero for y == 0, :361-366)
    uint8_t div(uint8_t a, uint8_t b) const { return (a && b) ? exp[log[a] + 255 - log[b]] : 0; }
};

inline const GF256 &gf() {
    static const GF256 g;
    return g;
}

struct GeneratorTables {
    std::vector<uint8_t> m2, m3, m4, m5, m6, Y, X;

    static std::vector<uint8_t> unhex(const char *h, int n) {
        std::vector<uint8_t> v(static_cast<size_t>(n));
        auto nib = [](char c) { return c <= '9' ? c - '0' : c - 'a' + 10; };
        for (int i = 0; i < n; ++i) v[i] = static_cast<uint8_t>(nib(h[2 * i]) * 16 + nib(h[2 * i + 1]));
        return v;
    }
    GeneratorTables()
        : m2(unhex(SH_TABLE_2_HEX, SH_TABLE_2_LEN)), m3(unhex(SH_TABLE_3_HEX, SH_TABLE_3_LEN)),
          m4(unhex(SH_TABLE_4_HEX, SH_TABLE_4_LEN)), m5(unhex(SH_TABLE_5_HEX, SH_TABLE_5_LEN)),
          m6(unhex(SH_TABLE_6_HEX, SH_TABLE_6_LEN)), Y(unhex(SH_TABLE_Y_HEX, SH_TABLE_Y_LEN)),
          X(unhex(SH_TABLE_X_HEX, SH_TABLE_X_LEN)) {}
};

inline const GeneratorTables &gen_tables() {
    static const GeneratorTables t;
    return t;
}

// Full m x k generator over the recovery rows: row 0 is all ones (the parity row the reference
// writes by plain XOR, cauchy_256.cpp:1496-1500), rows 1..m-1 follow cauchy_matrix()
// (cauchy_256.cpp:423-481): static "improved" rows with stride 256-m for m = 2..6, otherwise
// row y, col 0 = 1/(1 ^ Y[y-1]) and col x = X[x-1] / (X[x-1] ^ Y[y-1]) with the X vector of m
// at offset n*249 - n(n+1)/2, n = m-7. Precondition: 1 <= m, 2 <= k, k + m <= 256.
inline std::vector<uint8_t> generator_matrix(int k, int m) {
    std::vector<uint8_t> G(static_cast<size_t>(m) * k, 1);
    if (m < 2) return G;
    const GeneratorTables &t = gen_tables();
    const std::vector<uint8_t> *stat = nullptr;
    switch (m) {
    case 2: stat = &t.m2; break;
    case 3: stat = &t.m3; break;
    case 4: stat = &t.m4; break;
    case 5: stat = &t.m5; break;
    case 6: stat = &t.m6; break;
    default: break;
    }
    if (stat) {
        const int stride = 256 - m;
        for (int y = 1; y < m; ++y)
            std::memcpy(&G[static_cast<size_t>(y) * k], stat->data() + (y - 1) * stride, k);
        return G;
    }
    const GF256 &f = gf();
    const int n = m - 7;
    const uint8_t *X = t.X.data() + n * 249 - n * (n + 1) / 2;
    for (int y = 1; y < m; ++y) {
        const uint8_t Yv = t.Y[y - 1];
        uint8_t *row = &G[static_cast<size_t>(y) * k];
        row[0] = f.inv[1 ^ Yv];
        for (int x = 1; x < k; ++x) row[x] = f.div(X[x - 1], static_cast<uint8_t>(X[x - 1] ^ Yv));
    }
    return G;
}

// Cauchy parameters of the m >= 7 generator: C[y][x] = X'_x / (X'_x + Y'_y) with X'_0 = 1,
// X'_x = X[x-1] and Y'_0 = 0, Y'_y = Y[y-1] (same tables as generator_matrix()). Empty for m < 7.
inline void cauchy_params(int k, int m, std::vector<uint8_t> &xp, std::vector<uint8_t> &yp) {
    xp.assign(static_cast<size_t>(k), 0);
    yp.assign(static_cast<size_t>(m), 0);
    if (m < 7) return;
    const GeneratorTables &t = gen_tables();
    const int n = m - 7;
    const uint8_t *X = t.X.data() + n * 249 - n * (n + 1) / 2;
    xp[0] = 1;
    for (int x = 1; x < k; ++x) xp[x] = X[x - 1];
    yp[0] = 0;
    for (int y = 1; y < m; ++y) yp[y] = t.Y[y - 1];
}

}  // namespace sh
