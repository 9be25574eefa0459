// Host-side GF(256) helper ABI (include/gf256.h): the reference's gf256.o replaced symbol for
// symbol (catid/shorthair gf256.cpp). Plain host C++ (compiled with the host compiler, not
// hipcc): these helpers work on caller memory in spans of a few hundred bytes, where a GPU
// round trip would cost more than the work.
//
// Tables (reference gf256.cpp:354-600, restated): polynomial 0x14D; exp/log with the reference's
// conventions; MUL/DIV [y << 8 | x]; INV, SQR; split-nibble shuffle rows for y. Bulk ops: XOR
// loops the compiler vectorises, and the multiply as two nibble shuffles (pshufb) per 16 or 32
// bytes -- the reference's method (gf256.cpp:1104-1266), reimplemented with an AVX2 path chosen
// at run time like the reference's CpuHasAVX2 (cpuid leaf 7, EBX bit 5).
#include "../../include/gf256.h"

#include <cpuid.h>
#include <immintrin.h>

#include <cstddef>
#include <cstdint>
#include <cstring>

extern "C" {
gf256_ctx GF256Ctx;
}

static_assert(sizeof(gf256_ctx) == 157728, "GF256Ctx must keep the reference's AVX2 layout");
static_assert(offsetof(gf256_ctx, GF256_MUL_TABLE) == 24576, "reference layout");
static_assert(offsetof(gf256_ctx, GF256_LOG_TABLE) == 156160, "reference layout");

namespace {

bool g_ready = false;
bool g_avx2 = false;
constexpr unsigned kPoly = (0xA6u << 1) | 1u;  // reference default index 3 of its 16 polynomials

bool cpu_has_avx2() {
    unsigned a, b, c, d;
    if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return false;
    return (b & (1u << 5)) != 0;
}

void build_tables() {
    gf256_ctx &t = GF256Ctx;
    t.Polynomial = kPoly;
    // exp[i] = 2^i for i < 255; log of each; then the reference's extensions: exp[255] = 1 with
    // log[1] = 255 (not 0), exp repeated up to index 509, exp[510] = 1, zeros after; log[0] = 512
    // so that any product with 0 lands in the zero run.
    unsigned v = 1;
    for (int i = 0; i < 255; ++i) {
        t.GF256_EXP_TABLE[i] = static_cast<uint8_t>(v);
        if (i) t.GF256_LOG_TABLE[v] = static_cast<uint16_t>(i);
        v <<= 1;
        if (v & 0x100u) v ^= kPoly;
    }
    t.GF256_EXP_TABLE[255] = 1;
    t.GF256_LOG_TABLE[1] = 255;
    t.GF256_LOG_TABLE[0] = 512;
    for (int i = 256; i < 510; ++i) t.GF256_EXP_TABLE[i] = t.GF256_EXP_TABLE[i % 255];
    t.GF256_EXP_TABLE[510] = 1;
    for (int i = 511; i < 1020; ++i) t.GF256_EXP_TABLE[i] = 0;

    for (int x = 0; x < 256; ++x) t.GF256_MUL_TABLE[x] = t.GF256_DIV_TABLE[x] = 0;
    for (int y = 1; y < 256; ++y) {
        const uint8_t ly = static_cast<uint8_t>(t.GF256_LOG_TABLE[y]);
        const uint8_t lyn = static_cast<uint8_t>(255 - ly);
        uint8_t *mr = t.GF256_MUL_TABLE + (y << 8);
        uint8_t *dr = t.GF256_DIV_TABLE + (y << 8);
        mr[0] = dr[0] = 0;
        for (int x = 1; x < 256; ++x) {
            const unsigned lx = t.GF256_LOG_TABLE[x];
            mr[x] = t.GF256_EXP_TABLE[lx + ly];
            dr[x] = t.GF256_EXP_TABLE[lx + lyn];
        }
    }
    for (int x = 0; x < 256; ++x) {
        t.GF256_INV_TABLE[x] = t.GF256_DIV_TABLE[(x << 8) + 1];
        t.GF256_SQR_TABLE[x] = t.GF256_MUL_TABLE[(x << 8) + x];
    }
    for (int y = 0; y < 256; ++y) {
        for (int i = 0; i < 16; ++i) {
            const uint8_t lo = t.GF256_MUL_TABLE[(y << 8) + i];
            const uint8_t hi = t.GF256_MUL_TABLE[(y << 8) + (i << 4)];
            t.MM128.TABLE_LO_Y[y][i] = lo;
            t.MM128.TABLE_HI_Y[y][i] = hi;
            if (g_avx2) {  // the reference fills the 32-byte rows only on AVX2 CPUs
                t.MM256.TABLE_LO_Y[y][i] = t.MM256.TABLE_LO_Y[y][i + 16] = lo;
                t.MM256.TABLE_HI_Y[y][i] = t.MM256.TABLE_HI_Y[y][i + 16] = hi;
            }
        }
    }
}

// Field sanity: x * y / y == x, x * inv(x) == 1, and the shuffle rows agree with MUL.
bool self_check() {
    const gf256_ctx &t = GF256Ctx;
    for (int x = 0; x < 256; ++x)
        for (int y = 1; y < 256; ++y) {
            const uint8_t p = t.GF256_MUL_TABLE[(y << 8) + x];
            if (t.GF256_DIV_TABLE[(y << 8) + p] != x) return false;
        }
    for (int x = 1; x < 256; ++x)
        if (t.GF256_MUL_TABLE[(t.GF256_INV_TABLE[x] << 8) + x] != 1) return false;
    return true;
}

// ---- XOR family: byte loops over unaligned spans; -O3 vectorises them (and the AVX2 clones
// below run 32 bytes per instruction).
template <int OP>
inline void xor_span(uint8_t *GF256_RESTRICT z, const uint8_t *GF256_RESTRICT x,
                     const uint8_t *GF256_RESTRICT y, size_t n) {
    for (size_t i = 0; i < n; ++i) {
        if (OP == 0) z[i] ^= x[i];                // add:    z ^= x
        else if (OP == 1) z[i] ^= x[i] ^ y[i];    // add2:   z ^= x ^ y
        else z[i] = x[i] ^ y[i];                  // addset: z = x ^ y
    }
}

template <int OP>
__attribute__((target("avx2"))) void xor_span_avx2(uint8_t *GF256_RESTRICT z, const uint8_t *GF256_RESTRICT x,
                                                   const uint8_t *GF256_RESTRICT y, size_t n) {
    xor_span<OP>(z, x, y, n);
}

template <int OP>
inline void xor_dispatch(void *z, const void *x, const void *y, int bytes) {
    if (bytes <= 0) return;
    auto *zz = static_cast<uint8_t *>(z);
    auto *xx = static_cast<const uint8_t *>(x);
    auto *yy = static_cast<const uint8_t *>(y);
    if (g_avx2) xor_span_avx2<OP>(zz, xx, yy, static_cast<size_t>(bytes));
    else xor_span<OP>(zz, xx, yy, static_cast<size_t>(bytes));
}

// ---- multiply: z (^)= x * y by nibble shuffles; tails through the MUL row.
template <bool ADD>
__attribute__((target("avx2"))) size_t mul_avx2(uint8_t *z, const uint8_t *x, uint8_t y, size_t n) {
    const __m256i tlo = _mm256_load_si256(reinterpret_cast<const __m256i *>(GF256Ctx.MM256.TABLE_LO_Y[y]));
    const __m256i thi = _mm256_load_si256(reinterpret_cast<const __m256i *>(GF256Ctx.MM256.TABLE_HI_Y[y]));
    const __m256i m = _mm256_set1_epi8(0x0f);
    size_t i = 0;
    for (; i + 32 <= n; i += 32) {
        const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(x + i));
        __m256i p = _mm256_xor_si256(_mm256_shuffle_epi8(tlo, _mm256_and_si256(v, m)),
                                     _mm256_shuffle_epi8(thi, _mm256_and_si256(_mm256_srli_epi64(v, 4), m)));
        if (ADD) p = _mm256_xor_si256(p, _mm256_loadu_si256(reinterpret_cast<const __m256i *>(z + i)));
        _mm256_storeu_si256(reinterpret_cast<__m256i *>(z + i), p);
    }
    return i;
}

template <bool ADD>
__attribute__((target("ssse3"))) size_t mul_ssse3(uint8_t *z, const uint8_t *x, uint8_t y, size_t n) {
    const __m128i tlo = _mm_load_si128(reinterpret_cast<const __m128i *>(GF256Ctx.MM128.TABLE_LO_Y[y]));
    const __m128i thi = _mm_load_si128(reinterpret_cast<const __m128i *>(GF256Ctx.MM128.TABLE_HI_Y[y]));
    const __m128i m = _mm_set1_epi8(0x0f);
    size_t i = 0;
    for (; i + 16 <= n; i += 16) {
        const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i *>(x + i));
        __m128i p = _mm_xor_si128(_mm_shuffle_epi8(tlo, _mm_and_si128(v, m)),
                                  _mm_shuffle_epi8(thi, _mm_and_si128(_mm_srli_epi64(v, 4), m)));
        if (ADD) p = _mm_xor_si128(p, _mm_loadu_si128(reinterpret_cast<const __m128i *>(z + i)));
        _mm_storeu_si128(reinterpret_cast<__m128i *>(z + i), p);
    }
    return i;
}

template <bool ADD>
void mul_span(void *vz, const void *vx, uint8_t y, int bytes) {
    auto *z = static_cast<uint8_t *>(vz);
    auto *x = static_cast<const uint8_t *>(vx);
    const size_t n = static_cast<size_t>(bytes);
    size_t i = g_avx2 ? mul_avx2<ADD>(z, x, y, n) : 0;
    i += mul_ssse3<ADD>(z + i, x + i, y, n - i);
    const uint8_t *row = GF256Ctx.GF256_MUL_TABLE + (static_cast<unsigned>(y) << 8);
    for (; i < n; ++i) z[i] = ADD ? static_cast<uint8_t>(z[i] ^ row[x[i]]) : row[x[i]];
}

}  // namespace

extern "C" int gf256_init_(int version) {
    if (version != GF256_VERSION) return -1;
    if (g_ready) return 0;
    g_ready = true;
    g_avx2 = cpu_has_avx2();
    build_tables();
    return self_check() ? 0 : -3;
}

extern "C" void gf256_add_mem(void *GF256_RESTRICT vx, const void *GF256_RESTRICT vy, int bytes) {
    xor_dispatch<0>(vx, vy, nullptr, bytes);
}

extern "C" void gf256_add2_mem(void *GF256_RESTRICT vz, const void *GF256_RESTRICT vx,
                               const void *GF256_RESTRICT vy, int bytes) {
    xor_dispatch<1>(vz, vx, vy, bytes);
}

extern "C" void gf256_addset_mem(void *GF256_RESTRICT vz, const void *GF256_RESTRICT vx,
                                 const void *GF256_RESTRICT vy, int bytes) {
    xor_dispatch<2>(vz, vx, vy, bytes);
}

extern "C" void gf256_mul_mem(void *GF256_RESTRICT vz, const void *GF256_RESTRICT vx, uint8_t y, int bytes) {
    if (bytes <= 0) return;
    if (y <= 1) {  // reference gf256.cpp:1106-1114
        if (y == 0) std::memset(vz, 0, static_cast<size_t>(bytes));
        else if (vz != vx) std::memcpy(vz, vx, static_cast<size_t>(bytes));
        return;
    }
    mul_span<false>(vz, vx, y, bytes);
}

extern "C" void gf256_muladd_mem(void *GF256_RESTRICT vz, uint8_t y, const void *GF256_RESTRICT vx, int bytes) {
    if (bytes <= 0) return;
    if (y <= 1) {  // reference gf256.cpp:1270-1277
        if (y == 1) gf256_add_mem(vz, vx, bytes);
        return;
    }
    mul_span<true>(vz, vx, y, bytes);
}

extern "C" void gf256_memswap(void *GF256_RESTRICT vx, void *GF256_RESTRICT vy, int bytes) {
    if (bytes <= 0) return;
    auto *x = static_cast<uint8_t *>(vx);
    auto *y = static_cast<uint8_t *>(vy);
    for (size_t i = 0; i < static_cast<size_t>(bytes); ++i) {
        const uint8_t t = x[i];
        x[i] = y[i];
        y[i] = t;
    }
}
