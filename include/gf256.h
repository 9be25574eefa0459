/*
 * gf256.h -- host-side GF(256) helper ABI of libcauchy256.so.
 *
 * Replaces the reference's gf256.h / gf256.o (catid/shorthair gf256.h:121-276, gf256.cpp) symbol
 * for symbol, so a program that links the reference helpers links this library instead:
 * gf256_init_, gf256_add_mem, gf256_add2_mem, gf256_addset_mem, gf256_mul_mem, gf256_muladd_mem,
 * gf256_memswap and the table object GF256Ctx, plus the same inline scalar helpers.
 *
 * Field: GF(2^8) with the reference's default generator polynomial 0x14D (= 0xA6 << 1 | 1,
 * gf256.cpp:358-371) -- NOT the codec's 0x187. These helpers are host code on caller memory
 * (spans of a few hundred bytes, arbitrary alignment), as in the reference; the codec itself
 * does not use them. Semantics are the reference's, including its conventions:
 *   - nothing works before gf256_init() except the XOR/swap helpers (the tables are zero);
 *   - gf256_init_ returns 0 (also when already initialised), -1 on a version mismatch;
 *   - mul_mem with y == 0 zero-fills, with y == 1 copies; muladd_mem with y == 0 is a no-op;
 *   - the log table's own conventions (log[0] = 512, log[1] = 255, the extended exp table).
 * GF256Ctx has the reference's x86-64 AVX2 layout (the 32-byte MM256 tables included), 157,728
 * bytes, checked against the reference build in tests/test_gf256.py.
 */
#ifndef SH_AMD_GF256_H
#define SH_AMD_GF256_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Library header version (gf256.h:51). */
#define GF256_VERSION 2

#define GF256_ALIGN_BYTES 32
#define GF256_ALIGNED __attribute__((aligned(GF256_ALIGN_BYTES)))
#define GF256_RESTRICT __restrict
#define GF256_FORCE_INLINE inline __attribute__((always_inline))

/* Table object (gf256.h:141-170 with GF256_TRY_AVX2): split-nibble product tables for 16- and
 * 32-byte shuffles, then the scalar tables. TABLE_LO_Y[y][i] = y * i, TABLE_HI_Y[y][i] =
 * y * (i << 4) (i < 16; the 32-byte rows hold the 16 bytes twice). */
typedef struct gf256_ctx {
    struct {
        GF256_ALIGNED uint8_t TABLE_LO_Y[256][16];
        GF256_ALIGNED uint8_t TABLE_HI_Y[256][16];
    } MM128;
    struct {
        GF256_ALIGNED uint8_t TABLE_LO_Y[256][32];
        GF256_ALIGNED uint8_t TABLE_HI_Y[256][32];
    } MM256;
    uint8_t GF256_MUL_TABLE[256 * 256]; /* [y << 8 | x] = x * y */
    uint8_t GF256_DIV_TABLE[256 * 256]; /* [y << 8 | x] = x / y (0 when y == 0) */
    uint8_t GF256_INV_TABLE[256];
    uint8_t GF256_SQR_TABLE[256];
    uint16_t GF256_LOG_TABLE[256];
    uint8_t GF256_EXP_TABLE[512 * 2 + 1];
    unsigned Polynomial;
} GF256_ALIGNED gf256_ctx;

extern gf256_ctx GF256Ctx;

/* Fill the tables once (gf256.h:200-201): 0 ok, -1 version mismatch, -3 self-check failed. */
extern int gf256_init_(int version);
#define gf256_init() gf256_init_(GF256_VERSION)

/* Scalar helpers (gf256.h:208-237). */
static GF256_FORCE_INLINE uint8_t gf256_add(uint8_t x, uint8_t y) { return (uint8_t)(x ^ y); }
static GF256_FORCE_INLINE uint8_t gf256_mul(uint8_t x, uint8_t y)
{
    return GF256Ctx.GF256_MUL_TABLE[((unsigned)y << 8) + x];
}
static GF256_FORCE_INLINE uint8_t gf256_div(uint8_t x, uint8_t y)
{
    return GF256Ctx.GF256_DIV_TABLE[((unsigned)y << 8) + x];
}
static GF256_FORCE_INLINE uint8_t gf256_inv(uint8_t x) { return GF256Ctx.GF256_INV_TABLE[x]; }
static GF256_FORCE_INLINE uint8_t gf256_sqr(uint8_t x) { return GF256Ctx.GF256_SQR_TABLE[x]; }

/* Bulk helpers (gf256.h:244-276); spans may be unaligned, bytes <= 0 does nothing. */
extern void gf256_add_mem(void *GF256_RESTRICT vx, const void *GF256_RESTRICT vy, int bytes);      /* x ^= y */
extern void gf256_add2_mem(void *GF256_RESTRICT vz, const void *GF256_RESTRICT vx,
                           const void *GF256_RESTRICT vy, int bytes);                               /* z ^= x ^ y */
extern void gf256_addset_mem(void *GF256_RESTRICT vz, const void *GF256_RESTRICT vx,
                             const void *GF256_RESTRICT vy, int bytes);                             /* z = x ^ y */
extern void gf256_mul_mem(void *GF256_RESTRICT vz, const void *GF256_RESTRICT vx, uint8_t y, int bytes); /* z = x * y */
extern void gf256_muladd_mem(void *GF256_RESTRICT vz, uint8_t y, const void *GF256_RESTRICT vx,
                             int bytes);                                                            /* z ^= x * y */
static GF256_FORCE_INLINE void gf256_div_mem(void *GF256_RESTRICT vz, const void *GF256_RESTRICT vx, uint8_t y,
                                             int bytes)
{
    gf256_mul_mem(vz, vx, y == 1 ? (uint8_t)1 : GF256Ctx.GF256_INV_TABLE[y], bytes);
}
extern void gf256_memswap(void *GF256_RESTRICT vx, void *GF256_RESTRICT vy, int bytes);

#ifdef __cplusplus
}
#endif

#endif /* SH_AMD_GF256_H */
