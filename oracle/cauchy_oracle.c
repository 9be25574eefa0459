/*
 * CPU ORACLE -- TEST INFRASTRUCTURE ONLY (see cauchy_oracle.h). Never linked into the product.
 *
 * Clean-room restatement of the reference Cauchy Reed-Solomon codec (catid/shorthair,
 * cauchy_256.cpp). Deliberately simple: the bitmatrix is applied bit by bit (no windows), and
 * decode solves the erased columns with a GF(2) Gauss-Jordan on the full (8e x 8e) bitmatrix,
 * i.e. a different method from both the reference's windowed elimination and the GPU path's
 * GF(256)-inverse formulation. All three must agree byte for byte because the solution is unique.
 */
#include "cauchy_oracle.h"

#include <stdlib.h>
#include <string.h>

#include "../shorthair_amd/csrc/cauchy_tables_data.h"

/* ---- GF(256) with polynomial 0x187, generator 2 (cauchy_256.cpp:271-413) ---- */

static uint8_t g_exp[512];
static uint16_t g_log[256];
static uint8_t g_inv[256];
static uint8_t g_mat2[SH_TABLE_2_LEN], g_mat3[SH_TABLE_3_LEN], g_mat4[SH_TABLE_4_LEN];
static uint8_t g_mat5[SH_TABLE_5_LEN], g_mat6[SH_TABLE_6_LEN];
static uint8_t g_Y[SH_TABLE_Y_LEN], g_X[SH_TABLE_X_LEN];
static int g_ready;

static void unhex(const char *h, uint8_t *out, int n)
{
    for (int i = 0; i < n; ++i) {
        int v = 0;
        for (int j = 0; j < 2; ++j) {
            char c = h[2 * i + j];
            v = v * 16 + (c <= '9' ? c - '0' : c - 'a' + 10);
        }
        out[i] = (uint8_t)v;
    }
}

void ora_init(void)
{
    if (g_ready) return;
    unsigned x = 1;
    for (int i = 0; i < 255; ++i) {
        g_exp[i] = (uint8_t)x;
        g_exp[i + 255] = (uint8_t)x;
        g_log[x] = (uint16_t)i;
        x <<= 1;
        if (x & 0x100) x ^= 0x187;
    }
    g_log[0] = 512;
    g_inv[0] = 0;
    for (int i = 1; i < 256; ++i) g_inv[i] = g_exp[(255 - g_log[i]) % 255];
    unhex(SH_TABLE_2_HEX, g_mat2, SH_TABLE_2_LEN);
    unhex(SH_TABLE_3_HEX, g_mat3, SH_TABLE_3_LEN);
    unhex(SH_TABLE_4_HEX, g_mat4, SH_TABLE_4_LEN);
    unhex(SH_TABLE_5_HEX, g_mat5, SH_TABLE_5_LEN);
    unhex(SH_TABLE_6_HEX, g_mat6, SH_TABLE_6_LEN);
    unhex(SH_TABLE_Y_HEX, g_Y, SH_TABLE_Y_LEN);
    unhex(SH_TABLE_X_HEX, g_X, SH_TABLE_X_LEN);
    g_ready = 1;
}

uint8_t ora_gf_mul(uint8_t a, uint8_t b)
{
    if (!a || !b) return 0;
    return g_exp[g_log[a] + g_log[b]];
}

uint8_t ora_gf_div(uint8_t a, uint8_t b)
{
    /* The reference's division table holds 0 for b == 0 (cauchy_256.cpp:361-366). */
    if (!a || !b) return 0;
    return g_exp[g_log[a] + 255 - g_log[b]];
}

uint8_t ora_gf_inv(uint8_t a) { return g_inv[a]; }

/* ---- generator matrix: cauchy_matrix(), cauchy_256.cpp:423-481 ---- */

void ora_cauchy_matrix(int k, int m, uint8_t *out)
{
    ora_init();
    const uint8_t *tab = 0;
    int stride = 0;
    switch (m) {  /* static "improved" rows, stride 256 - m (:428-444) */
    case 2: tab = g_mat2; stride = 254; break;
    case 3: tab = g_mat3; stride = 253; break;
    case 4: tab = g_mat4; stride = 252; break;
    case 5: tab = g_mat5; stride = 251; break;
    case 6: tab = g_mat6; stride = 250; break;
    default: break;
    }
    if (tab) {
        for (int y = 0; y < m - 1; ++y) memcpy(out + y * k, tab + y * stride, (size_t)k);
        return;
    }
    /* m >= 7: X at offset n*249 - n(n+1)/2, n = m - 7; X[0] = 1, Y[0] = 0 implicit (:453-477) */
    int n = m - 7;
    const uint8_t *X = g_X + n * 249 - n * (n + 1) / 2;
    for (int y = 1; y < m; ++y) {
        uint8_t G = g_Y[y - 1];
        uint8_t *row = out + (y - 1) * k;
        row[0] = g_inv[1 ^ G];
        for (int x = 1; x < k; ++x) {
            uint8_t B = X[x - 1];
            row[x] = ora_gf_div(B, (uint8_t)(B ^ G));
        }
    }
}

/* Generator element of (recovery row r, column x); row 0 is all ones. */
static uint8_t coef(const uint8_t *mat, int k, int r, int x)
{
    return r == 0 ? 1 : mat[(r - 1) * k + x];
}

/* out ^= M(s) * in on sub-blocks: output sub-block b collects input sub-block a whenever bit a of
 * s*2^b is set (cauchy_256.cpp:1553-1568, :609-628). */
static void bitmatrix_muladd(uint8_t *out, const uint8_t *in, uint8_t s, int sub)
{
    for (int b = 0; b < 8; ++b) {
        for (int a = 0; a < 8; ++a) {
            if (s & (1u << a)) {
                uint8_t *o = out + b * sub;
                const uint8_t *i = in + a * sub;
                for (int p = 0; p < sub; ++p) o[p] ^= i[p];
            }
        }
        s = ora_gf_mul(s, 2);
    }
}

/* ---- encode: cauchy_256_encode, cauchy_256.cpp:1479-1578 ---- */

int ora_encode(int k, int m, const uint8_t **data, uint8_t *rec, int B)
{
    ora_init();
    if (k <= 1) {  /* copy data[0] to every output (:1485-1493) */
        for (int i = 0; i < m; ++i) memcpy(rec + (size_t)i * B, data[0], (size_t)B);
        return 0;
    }
    /* row 0 = XOR of all inputs, written before validation (:1496-1500) */
    for (int p = 0; p < B; ++p) rec[p] = data[0][p] ^ data[1][p];
    for (int x = 2; x < k; ++x)
        for (int p = 0; p < B; ++p) rec[p] ^= data[x][p];
    if (m == 1) return 0;
    if (k + m > 256 || (B % 8) != 0) return -1;  /* (:1509-1511) */

    uint8_t *mat = (uint8_t *)malloc((size_t)k * (m - 1));
    ora_cauchy_matrix(k, m, mat);
    int sub = B / 8;
    memset(rec + B, 0, (size_t)B * (m - 1));
    for (int y = 1; y < m; ++y)
        for (int x = 0; x < k; ++x)
            bitmatrix_muladd(rec + (size_t)y * B, data[x], coef(mat, k, y, x), sub);
    free(mat);
    return 0;
}

/* ---- decode: cauchy_256_decode, cauchy_256.cpp:1233-1392 ---- */

/* m == 1: XOR every other block into the first block whose row >= k; that block's row is NOT
 * rewritten (cauchy_decode_m1, :487-519). The reference reads blocks[k] when no such block exists
 * (undefined); we return without touching anything instead. */
static void decode_m1(int k, ora_block *blocks, int B)
{
    int e = -1;
    for (int i = 0; i < k; ++i)
        if (blocks[i].row >= k) { e = i; break; }
    if (e < 0) return;
    uint8_t *out = blocks[e].data;
    for (int i = 0; i < k; ++i) {
        if (i == e) continue;
        for (int p = 0; p < B; ++p) out[p] ^= blocks[i].data[p];
    }
}

int ora_decode(int k, int m, ora_block *blocks, int B)
{
    ora_init();
    if (k <= 1) { blocks[0].row = 0; return 0; }  /* (:1236-1240) */
    if (m == 1) { decode_m1(k, blocks, B); return 0; }

    /* sort_blocks (:522-554): originals / recovery in array order; erasures ascending */
    int orig[256], rec[256], no = 0, nr = 0;
    uint8_t present[256], erasures[256];
    memset(present, 0, sizeof present);
    for (int i = 0; i < k; ++i) {
        if (blocks[i].row < k) { orig[no++] = i; present[blocks[i].row] = 1; }
        else rec[nr++] = i;
    }
    int ne = 0;
    for (int r = 0; r < 256 && ne < nr; ++r)
        if (r >= k || !present[r]) erasures[ne++] = (uint8_t)r;
    if (nr <= 0) return 0;                               /* nothing erased (:1266-1268) */
    if (k + m > 256 || (B % 8) != 0) return -1;          /* (:1271-1273) */

    int e = nr, sub = B / 8;
    uint8_t *mat = (uint8_t *)malloc((size_t)k * (m - 1));
    ora_cauchy_matrix(k, m, mat);

    /* residual_i = recovery_i + sum over received originals of M(c) * orig (:557-689) */
    for (int i = 0; i < e; ++i) {
        ora_block *rb = &blocks[rec[i]];
        int r = rb->row - k;
        for (int j = 0; j < no; ++j) {
            ora_block *ob = &blocks[orig[j]];
            bitmatrix_muladd(rb->data, ob->data, coef(mat, k, r, ob->row), sub);
        }
    }

    /* (8e x 8e) GF(2) system over the erased columns (generate_bitmatrix, :691-774); bit row
     * 8i+b, bit column 8l+a = bit a of C[r_i][erasure_l] * 2^b. Solved by Gauss-Jordan with the
     * same row operations applied to the residual sub-blocks. */
    int n = 8 * e, words = (n + 63) / 64;
    uint64_t *A = (uint64_t *)calloc((size_t)n * words, sizeof(uint64_t));
    uint8_t **rows = (uint8_t **)malloc(sizeof(uint8_t *) * n);
    uint8_t *rhs = (uint8_t *)malloc((size_t)n * sub);
    for (int i = 0; i < e; ++i) {
        int r = blocks[rec[i]].row - k;
        for (int l = 0; l < e; ++l) {
            uint8_t s = coef(mat, k, r, erasures[l]);
            for (int b = 0; b < 8; ++b) {
                for (int a = 0; a < 8; ++a)
                    if (s & (1u << a)) {
                        int col = 8 * l + a;
                        A[(size_t)(8 * i + b) * words + col / 64] |= 1ull << (col % 64);
                    }
                s = ora_gf_mul(s, 2);
            }
        }
        for (int b = 0; b < 8; ++b) {
            rows[8 * i + b] = rhs + (size_t)(8 * i + b) * sub;
            memcpy(rows[8 * i + b], blocks[rec[i]].data + b * sub, (size_t)sub);
        }
    }
    int ok = 1;
    for (int col = 0; col < n && ok; ++col) {
        int piv = -1;
        for (int r = col; r < n; ++r)
            if (A[(size_t)r * words + col / 64] >> (col % 64) & 1) { piv = r; break; }
        if (piv < 0) { ok = 0; break; }  /* singular: cannot happen for an MDS submatrix */
        if (piv != col) {
            for (int w = 0; w < words; ++w) {
                uint64_t t = A[(size_t)piv * words + w];
                A[(size_t)piv * words + w] = A[(size_t)col * words + w];
                A[(size_t)col * words + w] = t;
            }
            uint8_t *t = rows[piv]; rows[piv] = rows[col]; rows[col] = t;
        }
        for (int r = 0; r < n; ++r) {
            if (r == col || !(A[(size_t)r * words + col / 64] >> (col % 64) & 1)) continue;
            for (int w = 0; w < words; ++w) A[(size_t)r * words + w] ^= A[(size_t)col * words + w];
            for (int p = 0; p < sub; ++p) rows[r][p] ^= rows[col][p];
        }
    }
    if (ok) {
        /* bit row 8l+a now holds sub-block a of erased original erasures[l]; the i-th recovery
         * block in array order receives erasure i and its row (:548-553, :770) */
        for (int i = 0; i < e; ++i) {
            ora_block *rb = &blocks[rec[i]];
            for (int a = 0; a < 8; ++a) memcpy(rb->data + a * sub, rows[8 * i + a], (size_t)sub);
            rb->row = erasures[i];
        }
    }
    free(A); free(rows); free(rhs); free(mat);
    return ok ? 0 : -2;
}

/* ---- PCG32 (SiameseTools.h:80-102) and synthetic workload ---- */

void ora_pcg_seed(ora_pcg *r, uint64_t y, uint64_t x)
{
    r->state = 0;
    r->inc = (y << 1u) | 1u;
    ora_pcg_next(r);
    r->state += x;
    ora_pcg_next(r);
}

uint32_t ora_pcg_next(ora_pcg *r)
{
    uint64_t old = r->state;
    r->state = old * 6364136223846793005ull + r->inc;
    uint32_t xs = (uint32_t)(((old >> 18) ^ old) >> 27);
    uint32_t rot = (uint32_t)(old >> 59);
    return (xs >> rot) | (xs << ((-(int32_t)rot) & 31));
}

void ora_fill_block(uint64_t g, int x, uint64_t cfg, uint8_t *out, int B)
{
    ora_pcg r;
    ora_pcg_seed(&r, g * 256 + (uint64_t)x, cfg);
    for (int p = 0; p < B; p += 4) {
        uint32_t v = ora_pcg_next(&r);
        for (int j = 0; j < 4 && p + j < B; ++j) out[p + j] = (uint8_t)(v >> (8 * j));
    }
}

int ora_erasure_pattern(uint64_t g, int k, int m, uint64_t cfg, int e_fixed, uint8_t *rows_out)
{
    ora_pcg r;
    ora_pcg_seed(&r, g, cfg ^ 0xE7A5u);
    int emax = m < k ? m : k;
    int e = e_fixed > 0 ? (e_fixed < emax ? e_fixed : emax) : 1 + (int)(ora_pcg_next(&r) % (uint32_t)emax);
    uint8_t perm_k[256], perm_m[256], lost[256], used[256];
    for (int i = 0; i < k; ++i) perm_k[i] = (uint8_t)i;
    for (int i = 0; i < m; ++i) perm_m[i] = (uint8_t)i;
    for (int i = 0; i < e; ++i) {  /* partial Fisher-Yates: first e entries are the picks */
        int j = i + (int)(ora_pcg_next(&r) % (uint32_t)(k - i));
        uint8_t t = perm_k[i]; perm_k[i] = perm_k[j]; perm_k[j] = t;
        j = i + (int)(ora_pcg_next(&r) % (uint32_t)(m - i));
        t = perm_m[i]; perm_m[i] = perm_m[j]; perm_m[j] = t;
    }
    memset(lost, 0, sizeof lost);
    memset(used, 0, sizeof used);
    for (int i = 0; i < e; ++i) { lost[perm_k[i]] = 1; used[perm_m[i]] = 1; }
    int n = 0;
    for (int x = 0; x < k; ++x) if (!lost[x]) rows_out[n++] = (uint8_t)x;
    for (int y = 0; y < m; ++y) if (used[y]) rows_out[n++] = (uint8_t)(k + y);
    return e;
}

int ora_encode_batch(int k, int m, int B, int groups, const uint8_t *in, uint8_t *out)
{
    const uint8_t *ptrs[256];
    for (int g = 0; g < groups; ++g) {
        for (int x = 0; x < k; ++x) ptrs[x] = in + ((size_t)g * k + x) * B;
        int rc = ora_encode(k, m, ptrs, out + (size_t)g * m * B, B);
        if (rc) return rc;
    }
    return 0;
}
