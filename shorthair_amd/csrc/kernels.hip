// HIP kernels (gfx950 / CDNA4) for the batched Cauchy Reed-Solomon codec.
//
// Data model (bitmatrix CRS, reference catid/shorthair cauchy_256.cpp:1398-1578): a block of B bytes
// is 8 sub-blocks of sub = B/8 bytes. Generator element c acts as the 8x8 GF(2) matrix M(c) whose
// row b is the byte c*2^b in GF(256)/0x187: output sub-block b ^= input sub-block a for every bit
// a set in c*2^b. Every byte position p in [0, sub) -- and every bit of it -- is an independent
// "column", so a lane owns one 32-bit word of columns (bytes 4q..4q+3 of each sub-block) and runs
// the whole group's bitmatrix on it with word-wide XORs. M is a ring homomorphism
// (M(a)M(b) = M(ab)), which is what lets decode use a GF(256) inverse.
//
// Layout in HBM: a batch is `groups` code groups stored back to back; inside a group, blocks are
// contiguous B-byte rows ([G][n][B]). Sub-block starts are generally not 4-byte aligned
// (B = 1400 -> sub = 175); gfx950 global loads/stores accept unaligned dword addresses, so a lane
// reads its word directly. The last word of a sub-block holds `tail` = sub - 4*(nq-1) valid bytes:
// it is loaded right-aligned (never reading past the sub-block) and stored byte-exact.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.hpp"
#include "measure.hpp"

namespace sh {

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // a ^ b ^ c in one VALU op
}

__device__ __forceinline__ uint32_t ld32(const uint8_t *p) {
    uint32_t w;
    __builtin_memcpy(&w, p, 4);  // unaligned global_load_dword
    return w;
}

__device__ __forceinline__ void st32(uint8_t *p, uint32_t w) { __builtin_memcpy(p, &w, 4); }

// Column geometry of one lane: byte offset of its word inside a sub-block, how far the load is
// shifted back to stay inside the sub-block, and how many bytes it may store.
struct LaneCol {
    int off;    // byte offset of the (possibly shifted) load inside the sub-block
    int shr;    // right shift (bits) applied after the load
    int nbytes; // valid bytes (1..4)
};

__device__ __forceinline__ LaneCol lane_col(int q, const Geometry &geo) {
    LaneCol c;
    const bool last = (q == geo.nq - 1);
    const int valid = last ? geo.tail : 4;
    // A short last word is loaded from (4q - (4 - valid)) so the load ends at the sub-block end.
    // Only possible when sub >= 4; tiny sub-blocks (B < 32) take the byte path instead.
    const int back = (geo.sub >= 4) ? (4 - valid) : 0;
    c.off = 4 * q - back;
    c.shr = 8 * back;
    c.nbytes = valid;
    return c;
}

__device__ __forceinline__ uint32_t load_col(const uint8_t *sb, const LaneCol &c, bool bytewise) {
    if (!bytewise) return ld32(sb + c.off) >> c.shr;
    uint32_t w = 0;
    for (int i = 0; i < c.nbytes; ++i) w |= static_cast<uint32_t>(sb[c.off + i]) << (8 * i);
    return w;
}

__device__ __forceinline__ void store_col(uint8_t *sb, int q, const LaneCol &c, uint32_t w) {
    uint8_t *p = sb + 4 * q;
    if (c.nbytes == 4) {
        st32(p, w);
    } else {
        for (int i = 0; i < c.nbytes; ++i) p[i] = static_cast<uint8_t>(w >> (8 * i));
    }
}

// ---------------------------------------------------------------------------------------------
// Generic bitmatrix apply with RUNTIME coefficients:
//     out[g][o] = sum_j M(coef[g][o][j]) * in[g][j]        (o in [0, n_out_g), j in [0, n_in))
// Per input j a lane builds the two 4-bit window tables of its 8 sub-block words (reference
// win_encode, cauchy_256.cpp:1426-1445, 22 XORs) and then folds, for each output sub-block b,
// lo-table[nibble] ^ hi-table[nibble] into the accumulator with one 3-input XOR. The coefficient is
// wave-uniform, so the table index is an SGPR (hipcc lowers it to s_set_gpr_idx moves).
// R output rows per launch row-chunk (grid.y). PER_GROUP: coefficients differ per group and the
// wave must hold a single group (grid.z = group); otherwise lanes are flattened over (g, q).
// ---------------------------------------------------------------------------------------------
template <int R, bool PER_GROUP>
__global__ __launch_bounds__(256) void apply_generic(ApplyArgs a) {
    int g, q;
    if (PER_GROUP) {
        g = blockIdx.z;
        q = blockIdx.x * blockDim.x + threadIdx.x;
        if (q >= a.geo.nq) return;
    } else {
        const long long t = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
        g = static_cast<int>(t / a.geo.nq);
        q = static_cast<int>(t - static_cast<long long>(g) * a.geo.nq);
        if (g >= a.groups) return;
    }
    const int n_out = PER_GROUP && a.n_out_g ? a.n_out_g[g] : a.n_out;
    const int o0 = blockIdx.y * R;
    if (o0 >= n_out) return;
    const int nrows = min(R, n_out - o0);

    const Geometry geo = a.geo;
    const LaneCol col = lane_col(q, geo);
    const bool bytewise = geo.sub < 4;
    const uint8_t *in_g = a.in + static_cast<long long>(g) * a.in_gstride;
    const uint8_t *coef = a.coef + (PER_GROUP ? static_cast<long long>(g) * a.coef_gstride : 0) +
                          static_cast<long long>(o0) * a.coef_ld;

    uint32_t acc[R][8];
#pragma unroll
    for (int o = 0; o < R; ++o)
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[o][b] = 0;

    for (int j4 = 0; j4 < a.n_in; j4 += 4) {
        uint32_t cw[R];
#pragma unroll
        for (int o = 0; o < R; ++o)
            cw[o] = (o < nrows) ? *reinterpret_cast<const uint32_t *>(coef + o * a.coef_ld + j4) : 0u;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int j = j4 + jj;
            if (j >= a.n_in) break;
            uint32_t any = 0;
#pragma unroll
            for (int o = 0; o < R; ++o) any |= (cw[o] >> (8 * jj)) & 0xffu;
            if (!any) continue;
            const uint8_t *blk = in_g + static_cast<long long>(j) * a.in_bstride;
            uint32_t t0[16], t1[16];
            t0[0] = 0;
            t1[0] = 0;
            t0[1] = load_col(blk + 0 * geo.sub, col, bytewise);
            t0[2] = load_col(blk + 1 * geo.sub, col, bytewise);
            t0[4] = load_col(blk + 2 * geo.sub, col, bytewise);
            t0[8] = load_col(blk + 3 * geo.sub, col, bytewise);
            t1[1] = load_col(blk + 4 * geo.sub, col, bytewise);
            t1[2] = load_col(blk + 5 * geo.sub, col, bytewise);
            t1[4] = load_col(blk + 6 * geo.sub, col, bytewise);
            t1[8] = load_col(blk + 7 * geo.sub, col, bytewise);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                uint32_t *t = h ? t1 : t0;
                t[3] = t[1] ^ t[2];
                t[5] = t[1] ^ t[4];
                t[6] = t[2] ^ t[4];
                t[7] = t[3] ^ t[4];
                t[9] = t[1] ^ t[8];
                t[10] = t[2] ^ t[8];
                t[11] = t[3] ^ t[8];
                t[12] = t[4] ^ t[8];
                t[13] = t[5] ^ t[8];
                t[14] = t[6] ^ t[8];
                t[15] = t[7] ^ t[8];
            }
#pragma unroll
            for (int o = 0; o < R; ++o) {
                const uint32_t c = (cw[o] >> (8 * jj)) & 0xffu;
                if (c == 0) continue;
                const uint64_t rb = a.rowbytes[c];
#pragma unroll
                for (int b = 0; b < 8; ++b) {
                    const uint32_t s = static_cast<uint32_t>(rb >> (8 * b)) & 0xffu;
                    acc[o][b] = xor3(acc[o][b], t0[s & 15], t1[s >> 4]);
                }
            }
        }
    }

    uint8_t *out_g = a.out + static_cast<long long>(g) * a.out_gstride;
#pragma unroll
    for (int o = 0; o < R; ++o) {
        if (o >= nrows) break;
        uint8_t *blk = out_g + static_cast<long long>(o0 + o) * a.out_bstride;
#pragma unroll
        for (int b = 0; b < 8; ++b) store_col(blk + b * geo.sub, q, col, acc[o][b]);
    }
}

// ---------------------------------------------------------------------------------------------
// Plain XOR of n_in blocks (any byte count): the parity row 0 (reference cauchy_256.cpp:1496-1500,
// written before parameter validation) and m == 1 encode. One thread per 4-byte word.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void xor_rows(const uint8_t *in, long long in_gstride, int n_in,
                                                uint8_t *out, long long out_gstride, int B,
                                                int groups) {
    const int nw = (B + 3) / 4;
    const long long t = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
    const int g = static_cast<int>(t / nw);
    const int w = static_cast<int>(t - static_cast<long long>(g) * nw);
    if (g >= groups) return;
    const int nb = min(4, B - 4 * w);
    const uint8_t *src = in + g * in_gstride + 4 * w;
    uint8_t *dst = out + g * out_gstride + 4 * w;
    if (nb == 4) {
        uint32_t x = 0;
        for (int j = 0; j < n_in; ++j) x ^= ld32(src + static_cast<long long>(j) * B);
        st32(dst, x);
    } else {
        for (int i = 0; i < nb; ++i) {
            uint8_t x = 0;
            for (int j = 0; j < n_in; ++j) x ^= src[static_cast<long long>(j) * B + i];
            dst[i] = x;
        }
    }
}

// k <= 1 encode: every output row is a copy of data block 0 (cauchy_256.cpp:1485-1493).
__global__ __launch_bounds__(256) void copy_first(const uint8_t *in, long long in_gstride,
                                                  uint8_t *out, long long out_gstride, int m,
                                                  int B, int groups) {
    const long long t = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
    const long long per = static_cast<long long>(m) * B;
    const int g = static_cast<int>(t / per);
    if (g >= groups) return;
    const long long r = t - static_cast<long long>(g) * per;
    const int p = static_cast<int>(r % B);
    out[g * out_gstride + r] = in[g * in_gstride + p];
}

// ---------------------------------------------------------------------------------------------
// Decode setup, one 64-lane workgroup (one wave) per group. Restates the reference's
// sort_blocks + generate_bitmatrix (cauchy_256.cpp:522-554, :691-774) in GF(256):
//   * originals (row < k) / recovery blocks (row >= k) in array order; erasures = missing
//     original rows ascending; e = number of recovery blocks (0 -> nothing to do);
//   * S[i][j] = C[r_i][E_j] over received recovery rows r_i and erased columns E_j, and
//     x_{E_j} = S^-1 applied to the residuals. The recovered erasure j goes to the j-th recovery
//     block in array order, whose row becomes E_j (reference row contract, :548-553, :770).
// S^-1: for m >= 7 the generator is a scaled Cauchy matrix, C[y][x] = X'_x / (X'_x + Y'_y)
// (X'_0 = 1, Y'_0 = 0 gives the all-ones row 0; cauchy_256.cpp:453-477), so
//   S^-1[j][i] = a_j b_i / (x_j (x_j + y_i)),  a_j = prod_k (x_j+y_k) / prod_{k!=j} (x_j+x_k),
//                                              b_i = prod_k (x_k+y_i) / prod_{k!=i} (y_i+y_k)
// with x_j = X'_{E_j}, y_i = Y'_{r_i}: O(e^2) log-domain table lookups, no elimination. The
// static "improved" tables for m = 2..6 have no such structure; there e <= 5 and a small
// Gauss-Jordan in LDS does it.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int mod255(int v) {
    v %= 255;
    return v < 0 ? v + 255 : v;
}

// Per-wave scratch of decode_setup (one group per wave).
struct SetupScratch {
    uint8_t rows[256];
    uint32_t present[64];  // occurrences of each row value, 4 x 8-bit counts per word
    uint8_t rec[256];      // array index of the i-th recovery block
    uint8_t rrow[256];     // its generator row r_i = row - k
    uint8_t era[256];      // j-th erased original row E_j
    uint8_t x[256], y[256];
    uint8_t la[256], lb[256];  // log a_j - log x_j and log b_i, mod 255
};

// Every wave handles its own group and synchronises only with itself: its lanes run in lockstep,
// so its LDS writes are visible to all of its lanes once they completed (lgkmcnt(0)).
#define SH_WAVE_SYNC() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")

// W groups per workgroup (one wave each): the exp/log tables are staged once per workgroup
// ((28,4,256), 209,263 groups: one wave per workgroup spent 0.28 ms of a 0.81 ms decode).
template <int W>
__global__ __launch_bounds__(64 * W, 8) void decode_setup(DecodeSetupArgs a, int groups) {
    const int wave = threadIdx.x >> 6;
    const int g = blockIdx.x * W + wave;
    const int lane = threadIdx.x & 63;
    const int k = a.k, m = a.m;
    // exp over [0, 1024): every exponent sum of the closed form's coefficients, [1, 763], without a
    // mod-255 reduction (s_exp[i] = exp(i mod 255))
    __shared__ uint8_t s_exp[1024];
    __shared__ uint8_t s_log[256];
    // generator data the coefficients need, staged with the tables so the per-group chain has one
    // global round trip (the rows): m <= 6 the searched rows 1..m-1, m >= 7 the Cauchy X', Y'
    __shared__ uint8_t s_gen[5 * 256];
    __shared__ uint8_t s_xp[256], s_yp[256];
    __shared__ SetupScratch sw[W];
    SetupScratch &S = sw[wave];

    // Every global load of the staging is issued before any is waited for (one round trip): the
    // group's row bytes as dwords where aligned, four exp entries per thread.
    if (g < groups) {
        const uint8_t *rows = a.rows + static_cast<long long>(g) * a.rows_gstride;
        if ((k & 3) == 0 && (reinterpret_cast<uintptr_t>(rows) & 3) == 0) {
            if (4 * lane < k)
                *reinterpret_cast<uint32_t *>(S.rows + 4 * lane) = *reinterpret_cast<const uint32_t *>(rows + 4 * lane);
        } else {
            for (int j = lane; j < k; j += 64) S.rows[j] = rows[j];
        }
    }
    S.present[lane] = 0;
    static_assert(64 * W * 4 >= 1024, "four exp entries per thread");
    {
        uint8_t ev[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) ev[u] = a.gf_exp[(4 * threadIdx.x + u) % 255];
#pragma unroll
        for (int u = 0; u < 4; ++u) s_exp[4 * threadIdx.x + u] = ev[u];
    }
    for (int i = threadIdx.x; i < 256; i += 64 * W) s_log[i] = static_cast<uint8_t>(a.gf_log[i]);
    if (m <= 6) {
        for (int i = threadIdx.x; i < (m - 1) * k; i += 64 * W) s_gen[i] = a.gen[i];
    } else {
        for (int i = threadIdx.x; i < k; i += 64 * W) s_xp[i] = a.xp[i];
        for (int i = threadIdx.x; i < m; i += 64 * W) s_yp[i] = a.yp[i];
    }
    __syncthreads();  // the only workgroup barrier: waves below may return independently
    if (g >= groups) return;
    auto present = [&](int r) { return static_cast<int>((S.present[r >> 2] >> (8 * (r & 3))) & 0xFFu); };
    for (int j = lane; j < k; j += 64)  // a row occurs at most k <= 255 times: no carry between counts
        atomicAdd(&S.present[S.rows[j] >> 2], 1u << (8 * (S.rows[j] & 3)));
    SH_WAVE_SYNC();
    // A row listed twice, or a recovery row past the generator (row >= k + m), is outside the
    // reference's contract (it would decode garbage): the group is left untouched and reported.
    bool bad = false;
    for (int r = lane; r < 256; r += 64) bad |= present(r) > 1 || (r >= k + m && present(r) > 0);
    if (__ballot(bad) != 0ull) {
        if (lane == 0) {
            a.e_out[g] = -1;
            if (a.errors) atomicAdd(a.errors, 1);
        }
        return;
    }

    // Ordered compaction with wave ballots (the workgroup is one wave).
    int nrec = 0;
    for (int base = 0; base < k; base += 64) {
        const int j = base + lane;
        const bool isrec = (j < k) && (S.rows[j] >= k);
        const unsigned long long mask = __ballot(isrec);
        if (isrec) {
            const int pos = nrec + __popcll(mask & ((1ull << lane) - 1ull));
            S.rec[pos] = static_cast<uint8_t>(j);
            S.rrow[pos] = static_cast<uint8_t>(S.rows[j] - k);
        }
        nrec += __popcll(mask);
    }
    int nera = 0;
    for (int base = 0; base < k; base += 64) {
        const int x = base + lane;
        const bool miss = (x < k) && !present(x);
        const unsigned long long mask = __ballot(miss);
        if (miss) {
            const int pos = nera + __popcll(mask & ((1ull << lane) - 1ull));
            S.era[pos] = static_cast<uint8_t>(x);
        }
        nera += __popcll(mask);
    }
    SH_WAVE_SYNC();
    const int e = nrec;
    if (lane == 0) a.e_out[g] = e;
    const bool fixed_mode = (a.coefA == nullptr);
    if (fixed_mode) {
        const int KP = a.kp, MP = (m + 3) & ~3;
        uint8_t *pos = a.pos + static_cast<long long>(g) * KP;
        uint8_t *rpos = a.rpos + static_cast<long long>(g) * MP;
        for (int x = lane; x < KP; x += 64) pos[x] = 0xFF;
        for (int y = lane; y < MP; y += 64) rpos[y] = 0xFF;
        for (int j = lane; j < k; j += 64) {  // same wave, issued after the fills: ordered
            const int row = S.rows[j];
            if (row < k) pos[row] = static_cast<uint8_t>(j);
            else if (row - k < m) rpos[row - k] = static_cast<uint8_t>(j);
        }
    }
    if (e == 0) return;
    if (nera < e) {  // more recovery blocks than erasures: outside the reference's contract
        if (lane == 0) {
            a.e_out[g] = -1;
            if (a.errors) atomicAdd(a.errors, 1);
        }
        return;
    }
    const int emax = a.emax;
    uint8_t *rec_idx = a.rec_idx + static_cast<long long>(g) * emax;
    uint8_t *era = a.erasures + static_cast<long long>(g) * emax;
    for (int i = lane; i < e; i += 64) {
        rec_idx[i] = S.rec[i];
        era[i] = S.era[i];
    }
    auto C = [&](int r, int x) -> uint32_t {
        return r == 0 ? 1u : (m <= 6 ? s_gen[(r - 1) * k + x] : a.gen[static_cast<long long>(r - 1) * k + x]);
    };

    // Stage-A coefficients (generic path only), row-major [i][j], leading dimension ldA.
    if (!fixed_mode) {
        uint8_t *A = a.coefA + static_cast<long long>(g) * a.coefA_gstride;
        for (int i = 0; i < e; ++i) {
            const int r = S.rrow[i];
            for (int j = lane; j < a.ldA; j += 64) {
                uint32_t c = 0;
                if (j < k) {
                    const int row = S.rows[j];
                    c = row < k ? C(r, row) : (j == S.rec[i] ? 1u : 0u);
                }
                A[static_cast<long long>(i) * a.ldA + j] = static_cast<uint8_t>(c);
            }
        }
    }

    // Stage-B coefficients, transposed ([i][j] = S^-1[j][i]). Generic path: bytes for the
    // copy-and-XOR snippet kernel, zero elsewhere. Fixed path: the address of the accumulating
    // snippet of each coefficient (the null snippet for zeros and for outputs j >= e), plus the
    // residual row of each received recovery block.
    // Byte coefficients (generic path, and the small-block stage B after a compile-time stage A:
    // targets == nullptr) or snippet addresses (stageb_fixed).
    uint8_t *Bc = a.targets ? nullptr : a.coefB + static_cast<long long>(g) * a.coefB_gstride;
    // fixed layout [g][j / 8][i][j % 8]: one wave's 8 addresses of consecutive rows are contiguous
    uint64_t *Tg = a.targets ? a.targets + static_cast<long long>(g) * emax * a.ldB : nullptr;
    const uint64_t tnull = a.snip_base + static_cast<uint64_t>(SNIP_NULL) * SNIP_STRIDE;
    if (fixed_mode) {
        uint8_t *rr = a.rrow + static_cast<long long>(g) * a.ldR;
        for (int i = lane; i < e; i += 64) rr[i] = S.rrow[i];
    }
    // Every entry stage B reads is written exactly once: the coefficient of (i < e, j < e), the
    // null snippet / zero for the unused outputs j in [e, ldB), and zero rows i >= e (bytes only).
    auto fill_unused = [&]() {
        if (Tg) {
            const int pad = a.ldB - e;
            for (int t = lane; t < e * pad; t += 64) {
                const int i = t / pad, j = e + (t - i * pad);
                Tg[(static_cast<long long>(j >> 3) * emax + i) * 8 + (j & 7)] = tnull;
            }
        } else {
            for (int t = lane; t < emax * a.ldB; t += 64) Bc[t] = 0;
        }
    };
    auto put = [&](int j, int i, uint32_t v) {
        if (Tg)
            Tg[(static_cast<long long>(j >> 3) * emax + i) * 8 + (j & 7)] =
                v ? a.snip_base + static_cast<uint64_t>(v) * SNIP_STRIDE : tnull;
        else
            Bc[static_cast<long long>(i) * a.ldB + j] = static_cast<uint8_t>(v);
    };
    if (m >= 7) {
        for (int t = lane; t < e; t += 64) {
            S.x[t] = s_xp[S.era[t]];
            S.y[t] = s_yp[S.rrow[t]];
        }
        SH_WAVE_SYNC();
        // log a_j - log x_j (items w < e, into la) and log b_i (items e <= w < 2e, into lb) on all
        // 64 lanes: a_j's sum runs over the other set (y) and its product over its own (x), b_i's
        // the other way round; q-loop unrolled so the lookups of several terms are in flight.
        for (int w = lane; w < 2 * e; w += 64) {
            const bool isa = w < e;
            const int t = isa ? w : w - e;
            const uint8_t *other = isa ? S.y : S.x;
            const uint8_t *own = isa ? S.x : S.y;
            const int me = own[t];
            int acc = isa ? 255 * 130 - s_log[me] : 255 * 130;  // offset keeps the sum positive
#pragma unroll 4
            for (int q = 0; q < e; ++q) {
                acc += s_log[me ^ other[q]];
                acc -= q != t ? s_log[me ^ own[q]] : 0;
            }
            (isa ? S.la : S.lb)[t] = static_cast<uint8_t>(acc % 255);
        }
        SH_WAVE_SYNC();
        // S^-1[j][i] = exp(log a_j - log x_j + log b_i - log(x_j + y_i)); index in [1, 763]
        auto coef = [&](int j, int i) -> uint32_t {
            return s_exp[S.la[j] + S.lb[i] + 255 - s_log[S.x[j] ^ S.y[i]]];
        };
        // Walk the output in memory order so every store instruction writes contiguous bytes,
        // the unused entries included: addresses [j/8][i][j%8] (i < e), bytes [i][j] (i < emax).
        if (Tg) {
            const int nt = (a.ldB >> 3) * e * 8;
            for (int t = lane; t < nt; t += 64) {
                const int jb = t / (e * 8), r = t - jb * e * 8, i = r >> 3, j = jb * 8 + (r & 7);
                const uint32_t c = j < e ? coef(j, i) : 0u;
                Tg[(static_cast<long long>(jb) * emax + i) * 8 + (r & 7)] =
                    c ? a.snip_base + static_cast<uint64_t>(c) * SNIP_STRIDE : tnull;
            }
        } else {
            // t = i * ldB + j stepped by 64 without a division per entry
            const int ldB = a.ldB, iinc = 64 / ldB, jinc = 64 - iinc * ldB, n = emax * ldB;
            int i = lane / ldB, j = lane - i * ldB;
#pragma unroll 4
            for (int t = lane; t < n; t += 64) {
                Bc[t] = static_cast<uint8_t>(i < e && j < e ? coef(j, i) : 0u);
                j += jinc;
                i += iinc;
                if (j >= ldB) {
                    j -= ldB;
                    ++i;
                }
            }
        }
        return;
    }
    fill_unused();  // the Gauss-Jordan below writes the (i < e, j < e) entries with put()
    // m <= 6: Gauss-Jordan on [S | I] (e <= m <= 6), element t = row * 2e + column held by lane
    // t % 64 in half t / 64 (e * 2e <= 72, so two halves), rows exchanged by cross-lane reads: a
    // handful of dependent LDS trips per column instead of serial pivot scans and an LDS round
    // trip per row.
    const int w = 2 * e, nel = e * w;
    uint32_t v[2];
    int r[2], c[2];
    bool el[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int t = lane + 64 * h;
        r[h] = t / w;
        c[h] = t - r[h] * w;
        el[h] = t < nel;
        v[h] = !el[h] ? 0u : (c[h] < e ? C(S.rrow[r[h]], S.era[c[h]]) : (c[h] - e == r[h] ? 1u : 0u));
    }
    // value of element src (per lane; src < nel)
    auto fetch = [&](int src) -> uint32_t {
        const uint32_t lo = __shfl(v[0], src & 63), hi = __shfl(v[1], src & 63);
        return src >= 64 ? hi : lo;
    };
    auto gmul = [&](uint32_t x, uint32_t y) -> uint32_t {
        return (x && y) ? s_exp[s_log[x] + s_log[y]] : 0u;
    };
    for (int col = 0; col < e; ++col) {
        const unsigned long long c0 = __ballot(el[0] && c[0] == col && r[0] >= col && v[0] != 0);
        const unsigned long long c1 = __ballot(el[1] && c[1] == col && r[1] >= col && v[1] != 0);
        if ((c0 | c1) == 0ull) {  // singular: impossible for an MDS submatrix
            if (lane == 0) {
                a.e_out[g] = -1;
                if (a.errors) atomicAdd(a.errors, 1);
            }
            return;
        }
        // wave-uniform pivot row: the first candidate (elements are row-major)
        const int p = c0 ? (__ffsll(static_cast<long long>(c0)) - 1) / w
                         : (__ffsll(static_cast<long long>(c1)) - 1 + 64) / w;
        if (p != col) {
            uint32_t nv[2];
#pragma unroll
            for (int h = 0; h < 2; ++h)
                nv[h] = fetch(r[h] == col ? p * w + c[h] : (r[h] == p ? col * w + c[h] : lane + 64 * h));
            v[0] = nv[0];
            v[1] = nv[1];
        }
        const uint32_t piv = fetch(col * w + col);
        const uint32_t pinv = s_exp[255 - s_log[piv]];
#pragma unroll
        for (int h = 0; h < 2; ++h)
            if (r[h] == col) v[h] = gmul(v[h], pinv);
        uint32_t f[2], pc[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            f[h] = fetch(el[h] ? r[h] * w + col : 0);    // this row's entry in the pivot column
            pc[h] = fetch(el[h] ? col * w + c[h] : 0);   // the pivot row's entry in this column
        }
#pragma unroll
        for (int h = 0; h < 2; ++h)
            if (el[h] && r[h] != col) v[h] ^= gmul(f[h], pc[h]);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
        if (el[h] && c[h] >= e) put(r[h], c[h] - e, v[h]);
}

// ---------------------------------------------------------------------------------------------
// Multi-group decode setups (fixed-kernel mode): L lanes per group, 64 / L groups per wave. Same
// outputs as decode_setup above; there one wave carries one group through a chain of dependent
// LDS / global round trips, so a batch of many small groups runs many rounds of resident waves
// ((28,4,256), 209,263 groups: 0.215 ms of a 0.743 ms decode). Here a wave carries 64 / L groups
// through the same chain:
//   decode_setup_small   m <= 6, L = 8: the searched tables, Gauss-Jordan with a row per lane
//   decode_setup_cauchy  m >= 7, emax <= L = 16: the closed-form Cauchy inverse (L = 32 at e = 32
//                        lost to the one-wave kernel: 0.073 vs 0.063 ms at (224,32,256))
// ---------------------------------------------------------------------------------------------
// Per-group scratch: EC >= emax entries in the lists, RP >= round4(m) in the rpos image.
template <int EC, int RP>
struct GroupScratch {
    uint8_t rows[256];
    uint8_t pos[256];       // pos table image (round4(k) <= 256 entries)
    uint32_t present[8];    // bitmap of row values
    uint8_t rpos[RP];       // rpos table image
    uint8_t rec[EC], rrow[EC], era[EC];
};

__device__ __forceinline__ void group_fail(const DecodeSetupArgs &a, int g, int l) {
    if (l == 0) {
        a.e_out[g] = -1;
        if (a.errors) atomicAdd(a.errors, 1);
    }
}

// bit l of the result = predicate of lane l of the group whose first lane is gb
template <int L>
__device__ __forceinline__ unsigned group_ballot(bool p, int gb) {
    return static_cast<unsigned>((__ballot(p) >> gb) & ((1ull << L) - 1ull));
}

// Before the workgroup's staging barrier: the group's row bytes (all loads in flight together),
// present bitmap cleared.
template <int L, class GS>
__device__ __forceinline__ void group_load_rows(const DecodeSetupArgs &a, int g, int l, GS &S) {
    const uint8_t *rows = a.rows + static_cast<long long>(g) * a.rows_gstride;
    for (int j = l; j < a.k; j += L) S.rows[j] = rows[j];
    for (int t = l; t < 8; t += L) S.present[t] = 0;
}

// After the barrier: malformed check, ordered compaction, position tables, e and the per-group
// lists. Returns e when coefficients remain to be written, 0 when the group is done.
template <int L, int EC, class GS>
__device__ int group_prologue(const DecodeSetupArgs &a, int g, int l, int gb, GS &S) {
    const int k = a.k, m = a.m;
    // A row listed twice, or a recovery row past the generator, is outside the reference's
    // contract (decode_setup above): the group is left untouched and reported.
    bool bad = false;
    for (int j = l; j < k; j += L) {
        const int row = S.rows[j];
        const uint32_t bit = 1u << (row & 31);
        bad |= (atomicOr(&S.present[row >> 5], bit) & bit) != 0u || row >= k + m;
    }
    if (group_ballot<L>(bad, gb)) {
        group_fail(a, g, l);
        return 0;
    }
    SH_WAVE_SYNC();
    // L entries per step: recovery blocks in array order (unique rows in [k, k+m): at most
    // min(k, m) = emax <= EC of them), erased originals ascending (the first EC are kept).
    int nrec = 0, nera = 0;
    const unsigned below = (1u << l) - 1u;
    for (int base = 0; base < k; base += L) {
        const int j = base + l;
        const int row = j < k ? S.rows[j] : 0;
        const bool isrec = j < k && row >= k;
        const bool miss = j < k && ((S.present[j >> 5] >> (j & 31)) & 1u) == 0u;
        const unsigned mr = group_ballot<L>(isrec, gb), me = group_ballot<L>(miss, gb);
        if (isrec) {
            const int p = nrec + __popc(mr & below);
            if (p < EC) {
                S.rec[p] = static_cast<uint8_t>(j);
                S.rrow[p] = static_cast<uint8_t>(row - k);
            }
        }
        if (miss) {
            const int p = nera + __popc(me & below);
            if (p < EC) S.era[p] = static_cast<uint8_t>(j);
        }
        nrec += __popc(mr);
        nera += __popc(me);
    }
    // position tables, assembled in LDS and stored as dwords
    const int KP = a.kp, MP = (m + 3) & ~3;
    for (int x = l; x < KP; x += L) S.pos[x] = 0xFF;
    for (int y = l; y < MP; y += L) S.rpos[y] = 0xFF;
    SH_WAVE_SYNC();
    for (int j = l; j < k; j += L) {
        const int row = S.rows[j];
        if (row < k) S.pos[row] = static_cast<uint8_t>(j);
        else S.rpos[row - k] = static_cast<uint8_t>(j);
    }
    SH_WAVE_SYNC();
    uint32_t *pos = reinterpret_cast<uint32_t *>(a.pos + static_cast<long long>(g) * KP);
    for (int t = l; t < KP / 4; t += L) pos[t] = reinterpret_cast<const uint32_t *>(S.pos)[t];
    uint32_t *rpos = reinterpret_cast<uint32_t *>(a.rpos + static_cast<long long>(g) * MP);
    for (int t = l; t < MP / 4; t += L) rpos[t] = reinterpret_cast<const uint32_t *>(S.rpos)[t];
    const int e = nrec;
    if (l == 0) a.e_out[g] = e;
    if (e == 0) return 0;
    if (nera < e || e > EC) {  // unreachable with unique rows and emax <= EC
        group_fail(a, g, l);
        return 0;
    }
    const int emax = a.emax;
    for (int i = l; i < e; i += L) {
        a.rec_idx[static_cast<long long>(g) * emax + i] = S.rec[i];
        a.erasures[static_cast<long long>(g) * emax + i] = S.era[i];
        a.rrow[static_cast<long long>(g) * a.ldR + i] = S.rrow[i];
    }
    return e;
}

// One Gauss-Jordan row of up to 12 bytes in three registers (byte c at bits 8 (c & 3) of word
// c >> 2); every index goes through selects, so no array is ever placed in scratch.
struct Row12 {
    uint32_t w0 = 0u, w1 = 0u, w2 = 0u;
    __device__ uint32_t byte(int c) const {
        const uint32_t v = c < 4 ? w0 : (c < 8 ? w1 : w2);
        return (v >> (8 * (c & 3))) & 0xFFu;
    }
    __device__ void or_byte(int c, uint32_t v) {
        const uint32_t x = v << (8 * (c & 3));
        if (c < 4) w0 |= x;
        else if (c < 8) w1 |= x;
        else w2 |= x;
    }
    __device__ Row12 from_lane(int src) const {
        Row12 r;
        r.w0 = __shfl(w0, src);
        r.w1 = __shfl(w1, src);
        r.w2 = __shfl(w2, src);
        return r;
    }
    __device__ Row12 operator^(const Row12 &o) const {
        Row12 r;
        r.w0 = w0 ^ o.w0;
        r.w1 = w1 ^ o.w1;
        r.w2 = w2 ^ o.w2;
        return r;
    }
};

template <int W>
__global__ __launch_bounds__(64 * W, 8) void decode_setup_small(DecodeSetupArgs a, int groups) {
    constexpr int L = 8;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int sub = lane / L, l = lane % L, gb = L * sub;  // gb: first lane of this group
    const int g = (blockIdx.x * W + wave) * (64 / L) + sub;
    const int k = a.k, m = a.m;
    __shared__ uint8_t s_exp[512];
    __shared__ uint8_t s_log[256];
    __shared__ uint8_t s_gen[5 * 256];
    __shared__ GroupScratch<8, 8> sw[(64 / L) * W];
    GroupScratch<8, 8> &S = sw[(64 / L) * wave + sub];
    const bool live = g < groups;
    if (live) group_load_rows<L>(a, g, l, S);
    for (int i = threadIdx.x; i < 512; i += 64 * W) s_exp[i] = a.gf_exp[i];
    for (int i = threadIdx.x; i < 256; i += 64 * W) s_log[i] = static_cast<uint8_t>(a.gf_log[i]);
    for (int i = threadIdx.x; i < (m - 1) * k; i += 64 * W) s_gen[i] = a.gen[i];
    __syncthreads();  // the only workgroup barrier: groups below may finish independently
    if (!live) return;
    const int e = group_prologue<L, 8>(a, g, l, gb, S);
    if (e == 0) return;
    const int emax = a.emax;
    uint8_t *Bc = a.targets ? nullptr : a.coefB + static_cast<long long>(g) * a.coefB_gstride;
    uint64_t *Tg = a.targets ? a.targets + static_cast<long long>(g) * emax * a.ldB : nullptr;
    const uint64_t tnull = a.snip_base + static_cast<uint64_t>(SNIP_NULL) * SNIP_STRIDE;
    if (Tg) {  // null snippet for the unused outputs j in [e, ldB)
        const int pad = a.ldB - e;
        for (int t = l; t < e * pad; t += L) {
            const int i = t / pad, j = e + (t - i * pad);
            Tg[(static_cast<long long>(j >> 3) * emax + i) * 8 + (j & 7)] = tnull;
        }
    } else {
        for (int t = l; t < emax * a.ldB; t += L) Bc[t] = 0;
    }
    auto gballot = [&](bool p) { return group_ballot<L>(p, gb); };
    auto fail = [&]() { group_fail(a, g, l); };

    // Gauss-Jordan on [S | I], S[i][j] = C[r_i][E_j]: lane l < e holds row l (2e <= 12 bytes).
    Row12 u;
    if (l < e) {
        const int r = S.rrow[l];
#pragma unroll
        for (int c = 0; c < 12; ++c) {
            uint32_t v = 0u;
            if (c < e) v = r == 0 ? 1u : s_gen[(r - 1) * k + S.era[c]];
            else if (c < 2 * e) v = c - e == l ? 1u : 0u;
            u.or_byte(c, v);
        }
    }
    for (int col = 0; col < e; ++col) {
        const unsigned cand = gballot(l >= col && l < e && u.byte(col) != 0u);
        if (cand == 0u) {  // singular: impossible for an MDS submatrix
            fail();
            return;
        }
        const int p = __ffs(cand) - 1;  // first candidate row (group-uniform)
        if (p != col) u = u.from_lane(gb + (l == col ? p : (l == p ? col : l)));
        const Row12 pu = u.from_lane(gb + col);
        // row l <- row l + f * pinv * pivot row (f = its pivot-column entry); the pivot row itself
        // <- pinv * pivot row. Exponent sums below 2 * 255: no reduction for the exp lookup.
        const int lp = 255 - s_log[pu.byte(col)];  // log of the pivot's inverse
        const uint32_t f = u.byte(col);
        const bool me = l == col;
        int lf = me ? lp : lp + s_log[f];
        lf = lf >= 255 ? lf - 255 : lf;
        if (l < e && (me || f != 0u)) {
            Row12 nu;
#pragma unroll
            for (int c = 0; c < 12; ++c) {
                const uint32_t b = pu.byte(c);
                nu.or_byte(c, b ? s_exp[lf + s_log[b]] : 0u);
            }
            u = me ? nu : u ^ nu;
        }
    }
    // lane j holds row j of S^-1 in columns e .. 2e-1
    if (l < e) {
        for (int i = 0; i < e; ++i) {
            const uint32_t v = u.byte(e + i);
            if (Tg)
                Tg[static_cast<long long>(i) * 8 + l] = v ? a.snip_base + static_cast<uint64_t>(v) * SNIP_STRIDE : tnull;
            else
                Bc[static_cast<long long>(i) * a.ldB + l] = static_cast<uint8_t>(v);
        }
    }
}

// Closed-form S^-1 (m >= 7, decode_setup above) for emax <= L: x_j, y_i, the la / lb sums and
// the coefficient walk spread over the group's L lanes instead of a wave.
template <int EC>
struct CauchyLists {
    uint8_t x[EC], y[EC], la[EC], lb[EC];
};

template <int W, int L>
__global__ __launch_bounds__(64 * W, 8) void decode_setup_cauchy(DecodeSetupArgs a, int groups) {
    static_assert(L % 8 == 0 && L <= 32, "group lanes: a multiple of 8, at most 32");
    constexpr int GPW = 64 / L;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int sub = lane / L, l = lane % L, gb = L * sub;
    const int g = (blockIdx.x * W + wave) * GPW + sub;
    const int k = a.k, m = a.m;
    __shared__ uint8_t s_exp[1024];  // exp(i mod 255): exponent sums up to 763 unreduced
    __shared__ uint8_t s_log[256];
    __shared__ uint8_t s_xp[256], s_yp[256];
    __shared__ GroupScratch<L, 256> sw[GPW * W];
    __shared__ CauchyLists<L> cw[GPW * W];
    GroupScratch<L, 256> &S = sw[GPW * wave + sub];
    CauchyLists<L> &X = cw[GPW * wave + sub];
    const bool live = g < groups;
    if (live) group_load_rows<L>(a, g, l, S);
    static_assert(64 * W * 4 >= 1024, "four exp entries per thread");
    {
        uint8_t ev[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) ev[u] = a.gf_exp[(4 * threadIdx.x + u) % 255];
#pragma unroll
        for (int u = 0; u < 4; ++u) s_exp[4 * threadIdx.x + u] = ev[u];
    }
    for (int i = threadIdx.x; i < 256; i += 64 * W) s_log[i] = static_cast<uint8_t>(a.gf_log[i]);
    for (int i = threadIdx.x; i < k; i += 64 * W) s_xp[i] = a.xp[i];
    for (int i = threadIdx.x; i < m; i += 64 * W) s_yp[i] = a.yp[i];
    __syncthreads();  // the only workgroup barrier: groups below may finish independently
    if (!live) return;
    const int e = group_prologue<L, L>(a, g, l, gb, S);
    if (e == 0) return;
    for (int t = l; t < e; t += L) {
        X.x[t] = s_xp[S.era[t]];
        X.y[t] = s_yp[S.rrow[t]];
    }
    SH_WAVE_SYNC();
    // log a_j - log x_j (items w < e) and log b_i (items e <= w < 2e), as in decode_setup
    for (int w = l; w < 2 * e; w += L) {
        const bool isa = w < e;
        const int t = isa ? w : w - e;
        const uint8_t *other = isa ? X.y : X.x;
        const uint8_t *own = isa ? X.x : X.y;
        const int me = own[t];
        int acc = isa ? 255 * 130 - s_log[me] : 255 * 130;  // offset keeps the sum positive
#pragma unroll 4
        for (int q = 0; q < e; ++q) {
            acc += s_log[me ^ other[q]];
            acc -= q != t ? s_log[me ^ own[q]] : 0;
        }
        (isa ? X.la : X.lb)[t] = static_cast<uint8_t>(acc % 255);
    }
    SH_WAVE_SYNC();
    auto coef = [&](int j, int i) -> uint32_t {
        return s_exp[X.la[j] + X.lb[i] + 255 - s_log[X.x[j] ^ X.y[i]]];
    };
    const int emax = a.emax, ldB = a.ldB;
    if (a.targets) {
        // addresses [j/8][i][j%8] for i < e, in memory order: lane l keeps j%8 = l%8 (L is a
        // multiple of 8) and steps i by L/8, carrying into the next block of 8 outputs
        uint64_t *Tg = a.targets + static_cast<long long>(g) * emax * ldB;
        const uint64_t tnull = a.snip_base + static_cast<uint64_t>(SNIP_NULL) * SNIP_STRIDE;
        const int jj = l & 7, nb = ldB >> 3;
        int i = l >> 3, jb = 0;
        while (i >= e) {
            i -= e;
            ++jb;
        }
        while (jb < nb) {
            const int j = jb * 8 + jj;
            const uint32_t c = j < e ? coef(j, i) : 0u;
            Tg[(static_cast<long long>(jb) * emax + i) * 8 + jj] =
                c ? a.snip_base + static_cast<uint64_t>(c) * SNIP_STRIDE : tnull;
            i += L / 8;
            while (i >= e) {
                i -= e;
                ++jb;
            }
        }
    } else {
        // bytes [i][j], i < emax, j < ldB, zero outside (i < e, j < e)
        uint8_t *Bc = a.coefB + static_cast<long long>(g) * a.coefB_gstride;
        const int iinc = L / ldB, jinc = L - iinc * ldB, n = emax * ldB;
        int i = l / ldB, j = l - i * ldB;
        for (int t = l; t < n; t += L) {
            Bc[t] = static_cast<uint8_t>(i < e && j < e ? coef(j, i) : 0u);
            j += jinc;
            i += iinc;
            if (j >= ldB) {
                j -= ldB;
                ++i;
            }
        }
    }
}

// In-place finish of decode: recovered erasure l (dense scratch) goes to the l-th recovery block
// of the group, whose row becomes erasure l. One thread per 4-byte word of the recovered data.
__global__ __launch_bounds__(256) void scatter_recovered(ScatterArgs a) {
    const int g = blockIdx.y;
    const int e = a.e[g];
    const int nw = (a.B + 3) / 4;
    const long long t = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
    const int l = static_cast<int>(t / nw);
    const int w = static_cast<int>(t - static_cast<long long>(l) * nw);
    if (l >= e) return;
    const int j = a.rec_idx[static_cast<long long>(g) * a.emax + l];
    const uint8_t *src = a.src + static_cast<long long>(g) * a.src_gstride + static_cast<long long>(l) * a.B + 4 * w;
    uint8_t *dst = a.blocks + static_cast<long long>(g) * a.blocks_gstride + static_cast<long long>(j) * a.B + 4 * w;
    const int nb = min(4, a.B - 4 * w);
    if (nb == 4) st32(dst, ld32(src));
    else for (int i = 0; i < nb; ++i) dst[i] = src[i];
    if (w == 0) a.rows[static_cast<long long>(g) * a.rows_gstride + j] = a.erasures[static_cast<long long>(g) * a.emax + l];
}

// m == 1 decode (reference cauchy_decode_m1, cauchy_256.cpp:487-519): XOR every other block into
// the first block with row >= k; its row is NOT rewritten. No such block -> untouched (the
// reference reads past the array there). One thread per 4-byte word.
__global__ __launch_bounds__(256) void decode_m1(uint8_t *blocks, long long blocks_gstride,
                                                 const uint8_t *rows, long long rows_gstride, int k,
                                                 int B, int groups) {
    const int nw = (B + 3) / 4;
    const long long t = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
    const int g = static_cast<int>(t / nw);
    const int w = static_cast<int>(t - static_cast<long long>(g) * nw);
    if (g >= groups) return;
    const uint8_t *r = rows + g * rows_gstride;
    int er = -1;
    for (int i = 0; i < k; ++i)
        if (r[i] >= k) { er = i; break; }
    if (er < 0) return;
    uint8_t *base = blocks + g * blocks_gstride;
    const int nb = min(4, B - 4 * w);
    if (nb == 4) {
        uint32_t x = ld32(base + static_cast<long long>(er) * B + 4 * w);
        for (int i = 0; i < k; ++i)
            if (i != er) x ^= ld32(base + static_cast<long long>(i) * B + 4 * w);
        st32(base + static_cast<long long>(er) * B + 4 * w, x);
    } else {
        for (int bi = 0; bi < nb; ++bi) {
            uint8_t x = base[static_cast<long long>(er) * B + 4 * w + bi];
            for (int i = 0; i < k; ++i)
                if (i != er) x ^= base[static_cast<long long>(i) * B + 4 * w + bi];
            base[static_cast<long long>(er) * B + 4 * w + bi] = x;
        }
    }
}

// k <= 1 decode: blocks[0].row = 0 (cauchy_256.cpp:1236-1240).
__global__ void decode_k1(uint8_t *rows, long long rows_gstride, int groups) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g < groups) rows[g * rows_gstride] = 0;
}

// XOR of the step slices' partial outputs (single-group latency path): one thread per dword.
__global__ __launch_bounds__(256) void xor_reduce(const uint8_t *parts, long long part_bytes, int nparts,
                                                  uint8_t *out, long long nbytes) {
    const long long i = (static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x) * 4;
    if (i >= nbytes) return;
    if (i + 4 <= nbytes && (part_bytes & 3) == 0) {
        uint32_t x = ld32(parts + i);
        for (int p = 1; p < nparts; ++p) x ^= ld32(parts + p * part_bytes + i);
        st32(out + i, x);
    } else {
        for (long long b = i; b < nbytes && b < i + 4; ++b) {
            uint8_t x = parts[b];
            for (int p = 1; p < nparts; ++p) x ^= parts[p * part_bytes + b];
            out[b] = x;
        }
    }
}

hipError_t launch_xor_reduce(const uint8_t *parts, long long part_bytes, int nparts, uint8_t *out,
                             long long nbytes, hipStream_t stream) {
    if (nbytes <= 0) return hipSuccess;
    const long long threads = (nbytes + 3) / 4;
    hipLaunchKernelGGL(xor_reduce, dim3(static_cast<unsigned>((threads + 255) / 256)), dim3(256), 0, stream,
                       parts, part_bytes, nparts, out, nbytes);
    return hipGetLastError();
}

// Synthetic workload (same stream as oracle/cauchy_oracle.c ora_fill_block): block x of group g
// is PCG32 Seed(g*256 + x, cfg) output words, little-endian. One thread per block.
__device__ __forceinline__ uint32_t pcg_next(uint64_t &state, uint64_t inc) {
    const uint64_t old = state;
    state = old * 6364136223846793005ull + inc;
    const uint32_t xs = static_cast<uint32_t>(((old >> 18) ^ old) >> 27);
    const uint32_t rot = static_cast<uint32_t>(old >> 59);
    return (xs >> rot) | (xs << ((32u - rot) & 31u));
}

__global__ __launch_bounds__(256) void fill_pcg(uint8_t *out, long long gstride, int n, int B,
                                                int groups, unsigned long long g0,
                                                unsigned long long cfg) {
    const long long t = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
    const int g = static_cast<int>(t / n);
    const int x = static_cast<int>(t - static_cast<long long>(g) * n);
    if (g >= groups) return;
    const uint64_t inc = (((g0 + g) * 256ull + x) << 1) | 1ull;
    uint64_t state = 0;
    pcg_next(state, inc);
    state += cfg;
    pcg_next(state, inc);
    uint8_t *dst = out + g * gstride + static_cast<long long>(x) * B;
    for (int p = 0; p < B; p += 4) {
        const uint32_t v = pcg_next(state, inc);
        if (p + 4 <= B) st32(dst + p, v);
        else for (int i = 0; p + i < B; ++i) dst[p + i] = static_cast<uint8_t>(v >> (8 * i));
    }
}

// ---------------------------------------------------------------------------------------------
// Launch helpers (called from the host library; all asynchronous on `stream`).
// ---------------------------------------------------------------------------------------------
template <int R, bool PG>
static hipError_t launch_apply_t(const ApplyArgs &a, hipStream_t stream) {
    const int row_chunks = (a.n_out + R - 1) / R;
    if (PG) {
        dim3 grid((a.geo.nq + 63) / 64, row_chunks, a.groups);
        hipLaunchKernelGGL((apply_generic<R, true>), grid, dim3(64), 0, stream, a);
    } else {
        const long long cols = static_cast<long long>(a.groups) * a.geo.nq;
        dim3 grid(static_cast<unsigned>((cols + 255) / 256), row_chunks, 1);
        hipLaunchKernelGGL((apply_generic<R, false>), grid, dim3(256), 0, stream, a);
    }
    return hipGetLastError();
}

hipError_t launch_apply(const ApplyArgs &a, bool per_group, hipStream_t stream) {
    if (a.n_out <= 0 || a.groups <= 0) return hipSuccess;
    return per_group ? launch_apply_t<8, true>(a, stream) : launch_apply_t<8, false>(a, stream);
}

hipError_t launch_xor_rows(const uint8_t *in, long long in_gstride, int n_in, uint8_t *out,
                           long long out_gstride, int B, int groups, hipStream_t stream) {
    const long long n = static_cast<long long>(groups) * ((B + 3) / 4);
    hipLaunchKernelGGL(xor_rows, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, stream,
                       in, in_gstride, n_in, out, out_gstride, B, groups);
    return hipGetLastError();
}

hipError_t launch_copy_first(const uint8_t *in, long long in_gstride, uint8_t *out,
                             long long out_gstride, int m, int B, int groups, hipStream_t stream) {
    const long long n = static_cast<long long>(groups) * m * B;
    hipLaunchKernelGGL(copy_first, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, stream,
                       in, in_gstride, out, out_gstride, m, B, groups);
    return hipGetLastError();
}

hipError_t launch_decode_setup(const DecodeSetupArgs &a, int groups, hipStream_t stream) {
    constexpr int W = 4;
    // The multi-group setups pay a longer per-group chain for fewer rounds of waves: they win once
    // the one-wave kernel needs more than one round (256 CUs x 32 resident waves = 8192 groups);
    // below that the one-wave kernel is as fast or faster (profiles/r06/ab_runs.txt, block 8).
    // Measurement builds: SH_SETUP_WAVE=1 runs the one-wave kernel for every shape,
    // SH_SETUP_MIN_SMALL / SH_SETUP_MIN_CAUCHY move the thresholds.
    static const bool wave_only = measure_int(SH_MEASURE_ENV("SH_SETUP_WAVE"), 0) != 0;
    static const int min_small = measure_int(SH_MEASURE_ENV("SH_SETUP_MIN_SMALL"), 8192);
    static const int min_cauchy = measure_int(SH_MEASURE_ENV("SH_SETUP_MIN_CAUCHY"), 8192);
    if (a.coefA == nullptr && !wave_only) {
        if (a.m <= 6 && groups >= min_small) {
            hipLaunchKernelGGL(decode_setup_small<W>, dim3((groups + 8 * W - 1) / (8 * W)), dim3(64 * W), 0,
                               stream, a, groups);
            return hipGetLastError();
        }
        if (a.m >= 7 && a.emax <= 16 && groups >= min_cauchy) {
            hipLaunchKernelGGL((decode_setup_cauchy<W, 16>), dim3((groups + 4 * W - 1) / (4 * W)), dim3(64 * W), 0,
                               stream, a, groups);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL(decode_setup<W>, dim3((groups + W - 1) / W), dim3(64 * W), 0, stream, a, groups);
    return hipGetLastError();
}

hipError_t launch_scatter(const ScatterArgs &a, int groups, hipStream_t stream) {
    const long long n = static_cast<long long>(a.emax) * ((a.B + 3) / 4);
    hipLaunchKernelGGL(scatter_recovered, dim3(static_cast<unsigned>((n + 255) / 256), groups),
                       dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_decode_m1(uint8_t *blocks, long long blocks_gstride, const uint8_t *rows,
                            long long rows_gstride, int k, int B, int groups, hipStream_t stream) {
    const long long n = static_cast<long long>(groups) * ((B + 3) / 4);
    hipLaunchKernelGGL(decode_m1, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, stream,
                       blocks, blocks_gstride, rows, rows_gstride, k, B, groups);
    return hipGetLastError();
}

hipError_t launch_decode_k1(uint8_t *rows, long long rows_gstride, int groups, hipStream_t stream) {
    hipLaunchKernelGGL(decode_k1, dim3((groups + 255) / 256), dim3(256), 0, stream, rows,
                       rows_gstride, groups);
    return hipGetLastError();
}

hipError_t launch_fill(uint8_t *out, long long gstride, int n, int B, int groups,
                       unsigned long long g0, unsigned long long cfg, hipStream_t stream) {
    const long long t = static_cast<long long>(groups) * n;
    hipLaunchKernelGGL(fill_pcg, dim3(static_cast<unsigned>((t + 255) / 256)), dim3(256), 0, stream,
                       out, gstride, n, B, groups, g0, cfg);
    return hipGetLastError();
}

}  // namespace sh
