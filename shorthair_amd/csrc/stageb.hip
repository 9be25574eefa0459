// Decode stage B: runtime-coefficient bitmatrix products through tables of compile-time snippets.
//
//   out[g][j] = sum_i M(coef[g][i][j]) * in[g][i]        (j < e_g outputs, i < e_g inputs)
//
// The coefficients (S^-1 of a group's erasure pattern) are only known at run time, so the
// compile-time schedule of the encode kernels does not apply, and a register table indexed by a
// runtime (wave-uniform) value costs 8.7x (hipcc's s_set_gpr_idx lowering). Here the
// runtime choice is made ONCE per coefficient instead of once per table lookup: 256 snippets,
// one per coefficient value c, each applying M(c) to the current input row from its window
// tables (the reference's win_encode tables, cauchy_256.cpp:1426-1445) held in pinned VGPRs,
// are emitted as code (csrc/gen/snippets.h); the kernel reaches snippet c with one s_swappc_b64
// and the snippet returns with s_setpc_b64.
//
// Two kernels: stageb_snip (generic path, any geometry; copy-and-XOR snippets, coefficients as
// bytes) and stageb_fixed (after a compile-time stage A: accumulating snippets in VGPR-index
// mode, setup-computed snippet addresses, residual rows through a per-workgroup LDS-DMA ring). Group-uniform coefficients
// require a wave to stay inside one group: at B = 1400 a group has 44 word columns.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.hpp"
#include "snippets.h"
#include "measure.hpp"

#include <algorithm>
#include <cstdlib>

namespace sh {

typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t ldw_b(const uint8_t *p) {
    uint32_t w;
    __builtin_memcpy(&w, p, 4);
    return w;
}

// Call snippet at `target`: tmp = M(c) * (input whose window tables are t0/t1).
#define SH_SNIP_CALL(target, t0, t1, tmp)                                                         \
    asm volatile("s_swappc_b64 s[40:41], %[tg]"                                                  \
                 : "={v[132:139]}"(tmp)                                                          \
                 : [tg] "s"(target), "{v[100:115]}"(t0), "{v[116:131]}"(t1)                      \
                 : "s40", "s41")

static_assert(SH_SNIP_T0 == 100 && SH_SNIP_T1 == 116 && SH_SNIP_TMP == 132,
              "snippet registers must match the call constraints");

__global__ __launch_bounds__(256) void stageb_snip(StageBArgs a) {
    SH_SNIPPET_TABLE(B);
    const int ncc = (a.geo.nq + 63) / 64;  // 64-column chunks per group
    const int g = blockIdx.x / ncc;
    const int cc = blockIdx.x - g * ncc;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int j0 = (blockIdx.y * 4 + wave) * 8;
    const int e = a.e[g];
    if (j0 >= e) return;  // wave-uniform
    const int q = cc * 64 + lane;
    const Geometry geo = a.geo;
    if (q >= geo.nq) return;  // idle lanes (e.g. 20 of 64 at B = 1400)

    uint64_t base;
    asm volatile(
        "s_getpc_b64 s[42:43]\n"
        "s_add_u32 s42, s42, sh_snip_baseB@rel32@lo+4\n"
        "s_addc_u32 s43, s43, sh_snip_baseB@rel32@hi+12\n"
        "s_mov_b64 %0, s[42:43]"
        : "=s"(base)
        :
        : "s42", "s43", "scc");

    const uint8_t *in = a.in + static_cast<long long>(g) * a.in_gstride + 4 * q;
    const uint8_t *coef = a.coefT + static_cast<long long>(g) * a.coefT_gstride + j0;

    uint32_t acc[8][8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[j][b] = 0;

    for (int y = 0; y < a.n_in; ++y) {
        const uint64_t cw = *reinterpret_cast<const uint64_t *>(coef + static_cast<long long>(y) * a.ldT);
        if (cw == 0) continue;  // wave-uniform: no output of this wave uses input y
        const uint8_t *blk = in + static_cast<long long>(y) * geo.B;
        uint32_t d[8];
#pragma unroll
        for (int s = 0; s < 8; ++s) d[s] = ldw_b(blk + s * geo.sub);
        u32x16 t0, t1;
        t0[0] = 0;
        t1[0] = 0;
        t0[1] = d[0]; t0[2] = d[1]; t0[4] = d[2]; t0[8] = d[3];
        t1[1] = d[4]; t1[2] = d[5]; t1[4] = d[6]; t1[8] = d[7];
        t0[3] = t0[1] ^ t0[2]; t0[5] = t0[1] ^ t0[4]; t0[6] = t0[2] ^ t0[4]; t0[7] = t0[3] ^ t0[4];
        t0[9] = t0[1] ^ t0[8]; t0[10] = t0[2] ^ t0[8]; t0[11] = t0[3] ^ t0[8]; t0[12] = t0[4] ^ t0[8];
        t0[13] = t0[5] ^ t0[8]; t0[14] = t0[6] ^ t0[8]; t0[15] = t0[7] ^ t0[8];
        t1[3] = t1[1] ^ t1[2]; t1[5] = t1[1] ^ t1[4]; t1[6] = t1[2] ^ t1[4]; t1[7] = t1[3] ^ t1[4];
        t1[9] = t1[1] ^ t1[8]; t1[10] = t1[2] ^ t1[8]; t1[11] = t1[3] ^ t1[8]; t1[12] = t1[4] ^ t1[8];
        t1[13] = t1[5] ^ t1[8]; t1[14] = t1[6] ^ t1[8]; t1[15] = t1[7] ^ t1[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t c = static_cast<uint32_t>(cw >> (8 * j)) & 0xffu;
            if (c == 0) continue;  // wave-uniform
            u32x8 tmp;
            SH_SNIP_CALL(base + (static_cast<uint64_t>(c) << 6), t0, t1, tmp);
#pragma unroll
            for (int b = 0; b < 8; ++b) acc[j][b] ^= tmp[b];
        }
    }

    // Store the rows this wave owns; a sub-block's short last word is stored byte-exact.
    const bool last = (q == geo.nq - 1);
    const int nbytes = last ? geo.tail : 4;
    uint8_t *out = a.out + static_cast<long long>(g) * a.out_gstride + 4 * q;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (j0 + j >= e) break;
        uint8_t *row = out + static_cast<long long>(j0 + j) * geo.B;
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            uint8_t *p = row + b * geo.sub;
            const uint32_t w = acc[j][b];
            if (nbytes == 4) {
                __builtin_memcpy(p, &w, 4);
            } else {
                for (int i = 0; i < nbytes; ++i) p[i] = static_cast<uint8_t>(w >> (8 * i));
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Compile-time path (after a generated stage-A kernel, csrc/gen/): one workgroup = one group x
// one 64-column chunk x 32 outputs (4 waves x 8 outputs j0..j0+7).
//
//   out[j] = sum_{i < e} M(S^-1[j][i]) residual[rrow[i]]      (reference :1233-1392 semantics)
//
// The decode setup hands over, per group, the residual row r_i of each received recovery block
// (compacted: only the e rows that exist are staged and visited, so the work scales with e^2)
// and, for every (i, j), the ABSOLUTE address of the snippet that applies M(S^-1[j][i])
// (snippet 256 = return at once for zero / unused entries). The row loop therefore does no
// scalar address arithmetic: per input row it takes the 8 sub-block words (from the ring), builds the
// two 4-bit window tables (reference win_encode tables, cauchy_256.cpp:1426-1445, 22 XORs) into
// the pinned registers v[96:127], and makes 8 calls into the snippet table in VGPR-index mode
// (accumulator set j at v[32+8j..]).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t colx_off(int q, int nq, int sub) {
    return 4u * q - (q >= nq - 4 ? static_cast<uint32_t>(4 * nq - sub) : 0u);
}

// Holds the stage-B snippet table; its only launch reports where the table was loaded.
__global__ void stageb_snip_probe(uint64_t *out) {
    SH_SNIPA_TABLE(P);
    uint64_t base;
    asm volatile(
        "s_getpc_b64 s[42:43]\n"
        "s_add_u32 s42, s42, sh_snipa_baseP@rel32@lo+4\n"
        "s_addc_u32 s43, s43, sh_snipa_baseP@rel32@hi+12\n"
        "s_mov_b64 %0, s[42:43]"
        : "=s"(base)
        :
        : "s42", "s43", "scc");
    if (threadIdx.x == 0) *out = base;
}

static_assert(SH_SNIPA_ACC == 32 && SH_SNIPA_T0 == 96 && SH_SNIPA_T1 == 112,
              "accumulating-snippet registers must match the asm constraints");
static_assert(SH_SNIPA_STRIDE == SNIP_STRIDE && SH_SNIPA_NULL == SNIP_NULL, "snippet table layout");

#define SH_ROW_ASM_R                                                                              \
    "v_mov_b32 v97, %[d0]\n"                                                                      \
    "v_mov_b32 v98, %[d1]\n"                                                                      \
    "v_mov_b32 v100, %[d2]\n"                                                                     \
    "v_mov_b32 v104, %[d3]\n"                                                                     \
    "v_mov_b32 v113, %[d4]\n"                                                                     \
    "v_mov_b32 v114, %[d5]\n"                                                                     \
    "v_mov_b32 v116, %[d6]\n"                                                                     \
    "v_mov_b32 v120, %[d7]\n"                                                                     \
    "v_xor_b32 v99, %[d0], %[d1]\n"                                                               \
    "v_xor_b32 v115, %[d4], %[d5]\n"                                                              \
    "v_xor_b32 v101, %[d0], %[d2]\n"                                                              \
    "v_xor_b32 v117, %[d4], %[d6]\n"                                                              \
    "v_xor_b32 v102, %[d1], %[d2]\n"                                                              \
    "v_xor_b32 v118, %[d5], %[d6]\n"                                                              \
    "v_xor_b32 v105, %[d0], %[d3]\n"                                                              \
    "v_xor_b32 v121, %[d4], %[d7]\n"                                                              \
    "v_xor_b32 v106, %[d1], %[d3]\n"                                                              \
    "v_xor_b32 v122, %[d5], %[d7]\n"                                                              \
    "v_xor_b32 v108, %[d2], %[d3]\n"                                                              \
    "v_xor_b32 v124, %[d6], %[d7]\n"                                                              \
    "v_xor_b32 v103, v99, %[d2]\n"                                                                \
    "v_xor_b32 v119, v115, %[d6]\n"                                                               \
    "v_xor_b32 v107, v99, %[d3]\n"                                                                \
    "v_xor_b32 v123, v115, %[d7]\n"                                                               \
    "v_xor_b32 v109, v101, %[d3]\n"                                                               \
    "v_xor_b32 v125, v117, %[d7]\n"                                                               \
    "v_xor_b32 v110, v102, %[d3]\n"                                                               \
    "v_xor_b32 v126, v118, %[d7]\n"                                                               \
    "v_xor_b32 v111, v103, %[d3]\n"                                                               \
    "v_xor_b32 v127, v119, %[d7]\n"                                                               \
    "s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)\n"                                                     \
    "s_swappc_b64 s[40:41], %[g0]\n"                                                              \
    "s_set_gpr_idx_idx 8\n"                                                                       \
    "s_swappc_b64 s[40:41], %[g1]\n"                                                              \
    "s_set_gpr_idx_idx 16\n"                                                                      \
    "s_swappc_b64 s[40:41], %[g2]\n"                                                              \
    "s_set_gpr_idx_idx 24\n"                                                                      \
    "s_swappc_b64 s[40:41], %[g3]\n"                                                              \
    "s_set_gpr_idx_idx 32\n"                                                                      \
    "s_swappc_b64 s[40:41], %[g4]\n"                                                              \
    "s_set_gpr_idx_idx 40\n"                                                                      \
    "s_swappc_b64 s[40:41], %[g5]\n"                                                              \
    "s_set_gpr_idx_idx 48\n"                                                                      \
    "s_swappc_b64 s[40:41], %[g6]\n"                                                              \
    "s_set_gpr_idx_idx 56\n"                                                                      \
    "s_swappc_b64 s[40:41], %[g7]\n"                                                              \
    "s_set_gpr_idx_off"

struct Row8 {
    uint32_t w[8];
};

__device__ __forceinline__ void row_regs(const Row8 &d, const uint64_t (&tg)[8], u32x16 &a01, u32x16 &a23,
                                         u32x16 &a45, u32x16 &a67, uint32_t &z0, uint32_t &z1) {
    asm volatile(SH_ROW_ASM_R
                 : "+{v[32:47]}"(a01), "+{v[48:63]}"(a23), "+{v[64:79]}"(a45), "+{v[80:95]}"(a67),
                   "+{v96}"(z0), "+{v112}"(z1)
                 : [d0] "v"(d.w[0]), [d1] "v"(d.w[1]), [d2] "v"(d.w[2]), [d3] "v"(d.w[3]), [d4] "v"(d.w[4]),
                   [d5] "v"(d.w[5]), [d6] "v"(d.w[6]), [d7] "v"(d.w[7]), [g0] "s"(tg[0]), [g1] "s"(tg[1]),
                   [g2] "s"(tg[2]), [g3] "s"(tg[3]), [g4] "s"(tg[4]), [g5] "s"(tg[5]), [g6] "s"(tg[6]),
                   [g7] "s"(tg[7])
                 : "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107",
                   "v108", "v109", "v110", "v111", "v113", "v114", "v115", "v116", "v117", "v118", "v119",
                   "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "s40", "s41", "m0", "memory");
}

// Small e (emax <= 16): the waves load their own rows, two rows ahead into registers, with no
// barrier. A workgroup ring would keep four waves resident per group for e <= 8 and spend its
// 12-row prologue on rows that do not exist (C4 (28,4,1400) decode 0.66 vs 0.55 ms, C2 0.83 vs
// 0.76 ms), while with e = 32 the shared ring wins (below).
__global__ __launch_bounds__(256, 4) void stageb_regs(StageBFixedArgs a) {
    const Geometry geo = a.geo;
    const int ncc = (geo.nq + 63) / 64;
    const int g = blockIdx.x / ncc;
    const int cc = blockIdx.x - g * ncc;
    const int c0 = cc * 64;
    const int ncols = min(64, geo.nq - c0);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int e = a.e[g];
    const int j0 = (blockIdx.y * 4 + wave) * 8;
    if (j0 >= e) return;  // wave-uniform; e <= 0 included
    // idle lanes (lane >= ncols) load a valid column of the group and store nothing
    const uint32_t col = colx_off(c0 + min(lane, ncols - 1), geo.nq, geo.sub);
    uint32_t voff[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) voff[s] = col + static_cast<uint32_t>(s) * geo.sub;
    const long long gbase = static_cast<long long>(g) * a.in_gstride;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.in + gbase), static_cast<short>(0), static_cast<int>(a.in_gstride), 0x00020000);
    // scalar loads (gfx950 has no sub-dword s_load: read the row list as dwords)
    typedef const __attribute__((address_space(4))) uint32_t cu32_t;
    typedef const __attribute__((address_space(4))) uint64_t cu64_t;
    const cu32_t *rr = (const cu32_t *)(a.rrow + static_cast<long long>(g) * a.ldR);  // ldR % 4 == 0
    const cu64_t *tp = (const cu64_t *)(a.targets + (static_cast<long long>(g) * (a.ldT / 8) + (j0 >> 3)) * a.emax * 8);
    const int elast = e - 1;
    auto row_of = [&](int i) { return min(i, elast); };  // prefetches past the end re-read the last row
    auto row_soff = [&](int i) {
        i = row_of(i);
        return ((rr[i >> 2] >> (8 * (i & 3))) & 0xFFu) * static_cast<uint32_t>(geo.B);
    };
    auto load_row = [&](uint32_t soff, Row8 &d) {
#pragma unroll
        for (int s = 0; s < 8; ++s) d.w[s] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff[s], soff, 0);
    };

    u32x16 a01, a23, a45, a67;
#pragma unroll
    for (int t = 0; t < 16; ++t) a01[t] = a23[t] = a45[t] = a67[t] = 0;
    uint32_t z0 = 0, z1 = 0;
    Row8 r0, r1, r2;
    load_row(row_soff(0), r0);
    load_row(row_soff(1), r1);
    int i = 0;
    for (; i + 3 <= e; i += 3) {  // rows i, i+1, i+2 in r0, r1, r2 (rotating, two rows in flight)
        // the three rows' snippet addresses and the next three row offsets in one batch of scalar
        // loads: scalar loads return out of order, so any wait for one of them waits for all
        // (one exposed latency per 3 rows). The row loads are unconditional (indices clamped to
        // the last row, re-reads are L2 hits) so the counted vmcnt waits stay two rows deep.
        const int i2 = row_of(i + 2), i3 = row_of(i + 3), i4 = row_of(i + 4);
        const uint32_t w2 = rr[i2 >> 2], w3 = rr[i3 >> 2], w4 = rr[i4 >> 2];
        uint64_t tg[3][8];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const int x = row_of(i + r);
#pragma unroll
            for (int j = 0; j < 8; ++j) tg[r][j] = tp[x * 8 + j];
        }
        auto pick = [&](uint32_t w, int x) { return ((w >> (8 * (x & 3))) & 0xFFu) * static_cast<uint32_t>(geo.B); };
        const uint32_t s2 = pick(w2, i2), s3 = pick(w3, i3), s4 = pick(w4, i4);
        load_row(s2, r2);
        row_regs(r0, tg[0], a01, a23, a45, a67, z0, z1);
        load_row(s3, r0);
        row_regs(r1, tg[1], a01, a23, a45, a67, z0, z1);
        load_row(s4, r1);
        row_regs(r2, tg[2], a01, a23, a45, a67, z0, z1);
    }
    if (i < e) {  // one or two rows left, in r0 (and r1)
        uint64_t tg[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) tg[j] = tp[row_of(i) * 8 + j];
        row_regs(r0, tg, a01, a23, a45, a67, z0, z1);
        if (i + 1 < e) {
#pragma unroll
            for (int j = 0; j < 8; ++j) tg[j] = tp[row_of(i + 1) * 8 + j];
            row_regs(r1, tg, a01, a23, a45, a67, z0, z1);
        }
    }

    if (lane >= ncols) return;
    uint32_t acc[8][8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        acc[0][b] = a01[b]; acc[1][b] = a01[8 + b];
        acc[2][b] = a23[b]; acc[3][b] = a23[8 + b];
        acc[4][b] = a45[b]; acc[5][b] = a45[8 + b];
        acc[6][b] = a67[b]; acc[7][b] = a67[8 + b];
    }
    uint8_t *out = a.out + static_cast<long long>(g) * a.out_gstride + colx_off(c0 + lane, geo.nq, geo.sub);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (j0 + j >= e) break;
        uint8_t *row = out + static_cast<long long>(j0 + j) * geo.B;
#pragma unroll
        for (int b = 0; b < 8; ++b) __builtin_memcpy(row + b * geo.sub, &acc[j][b], 4);
    }
}

// The residual rows are staged in one LDS ring per workgroup (one group, 64-column
// chunk): each row is fetched ONCE per workgroup by LDS-DMA (2 KB: waves 0 and 1 issue one 1 KB
// piece each) instead of once per wave, with up to 12 rows in flight per workgroup. Rows in groups
// of RB_S: before a group every wave waits for its own DMAs of it (counted vmcnt, constant in the
// steady state) and joins the barrier, which also frees the slots of the previous group; they are
// refilled right there. Waves without outputs (8 * wave >= e) join the barriers and compute nothing.
// Measured at the headline (8192 groups, e = 32): 0.360 vs 0.377-0.384 ms for waves that each
// loaded their own rows two rows ahead into registers (round 2's form; an LDS tile of the whole
// residual loaded up front, 48 KB per workgroup, took 0.42 ms).
constexpr int RB_R = 16, RB_S = 4, RB_ROW = 8 * 64 * 4;
static_assert(RB_R == 4 * RB_S, "steady state: the slots of one group are refilled per group");

__global__ __launch_bounds__(256, 4) void stageb_fixed(StageBFixedArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[RB_R * RB_ROW];
    const Geometry geo = a.geo;
    const int ncc = (geo.nq + 63) / 64;
    const int g = blockIdx.x / ncc;
    const int cc = blockIdx.x - g * ncc;
    const int c0 = cc * 64;
    const int ncols = min(64, geo.nq - c0);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int e = a.e[g];
    if (e <= 0) return;  // uniform over the workgroup
    const int j0 = (blockIdx.y * 4 + wave) * 8;
    const bool active = j0 < e;
    const long long gbase = static_cast<long long>(g) * a.in_gstride;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.in + gbase), static_cast<short>(0), static_cast<int>(a.in_gstride), 0x00020000);
    // DMA piece of waves 0 and 1: slot bytes [wave*1024 + lane*16, +16) = sub-block sa, columns
    // c0 + cq .. + 3 (a whole 4-column chunk: nq % 4 == 0); chunks past the group read zeros
    const int off = wave * 1024 + lane * 16;
    const int sa = off / 256, cq = (off % 256) / 4;
    const uint32_t dsrc = (c0 + cq < geo.nq) ? colx_off(c0 + cq, geo.nq, geo.sub) + static_cast<uint32_t>(sa * geo.sub)
                                             : 0x80000000u;
    typedef const __attribute__((address_space(4))) uint32_t cu32_t;
    typedef const __attribute__((address_space(4))) uint64_t cu64_t;
    const cu32_t *rr = (const cu32_t *)(a.rrow + static_cast<long long>(g) * a.ldR);
    const cu64_t *tp = (const cu64_t *)(a.targets + (static_cast<long long>(g) * (a.ldT / 8) + (j0 >> 3)) * a.emax * 8);
    const int elast = e - 1;
    // Row i into slot i % RB_R. Rows past the end are issued too (the counted waits stay
    // constant) but out of range: no memory access, zeros into a slot nobody reads (it held a
    // row of the previous group, which every wave has finished).
    auto issue = [&](int i) {
        if (wave < 2) {
            const int x = min(i, elast);
            const uint32_t soff = ((rr[x >> 2] >> (8 * (x & 3))) & 0xFFu) * static_cast<uint32_t>(geo.B);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void *)(ring + (i % RB_R) * RB_ROW + wave * 1024),
                                                     16, i < e ? dsrc : 0x80000000u, soff, 0, 0);
        }
    };
    u32x16 a01, a23, a45, a67;
#pragma unroll
    for (int t = 0; t < 16; ++t) a01[t] = a23[t] = a45[t] = a67[t] = 0;
    uint32_t z0 = 0, z1 = 0;
    for (int i = 0; i < RB_R - RB_S; ++i) issue(i);
    const int ngroups = (e + RB_S - 1) / RB_S;
    for (int ig = 0; ig < ngroups; ++ig) {
        // own DMAs of rows 4ig..4ig+3 landed (RB_R - 2 * RB_S younger ones may be outstanding)
        if (wave < 2)
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(RB_R - 2 * RB_S) : "memory");
        else
            asm volatile("s_barrier" ::: "memory");
#pragma unroll
        for (int r = 0; r < RB_S; ++r) issue(ig * RB_S + RB_R - RB_S + r);
        if (!active) continue;
#pragma unroll
        for (int r = 0; r < RB_S; ++r) {
            const int i = ig * RB_S + r;
            if (i >= e) break;  // uniform
            uint64_t tg[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) tg[j] = tp[i * 8 + j];
            const uint8_t *slot = ring + (i % RB_R) * RB_ROW + lane * 4;
            Row8 d;
#pragma unroll
            for (int s = 0; s < 8; ++s) d.w[s] = *reinterpret_cast<const uint32_t *>(slot + s * 256);
            row_regs(d, tg, a01, a23, a45, a67, z0, z1);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no ring DMA may land after the workgroup ends
    if (!active || lane >= ncols) return;
    uint32_t acc[8][8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        acc[0][b] = a01[b]; acc[1][b] = a01[8 + b];
        acc[2][b] = a23[b]; acc[3][b] = a23[8 + b];
        acc[4][b] = a45[b]; acc[5][b] = a45[8 + b];
        acc[6][b] = a67[b]; acc[7][b] = a67[8 + b];
    }
    uint8_t *out = a.out + static_cast<long long>(g) * a.out_gstride + colx_off(c0 + lane, geo.nq, geo.sub);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (j0 + j >= e) break;
        uint8_t *row = out + static_cast<long long>(j0 + j) * geo.B;
#pragma unroll
        for (int b = 0; b < 8; ++b) __builtin_memcpy(row + b * geo.sub, &acc[j][b], 4);
    }
}

// ---------------------------------------------------------------------------------------------
// stageb_v2: one workgroup = one group x one 64-column chunk x up to 8*NW outputs (NW waves of 8),
// so for e <= 8*NW every residual row is fetched ONCE per (group, chunk) however large e is
// (stageb_fixed re-streamed all e rows per 32 outputs: e = 56..66 at the Tester's shapes).
// Per row a wave needs the snippet addresses of its 8 coefficients S^-1[j0..j0+7][i]; they come
// from the byte coefficients (setup's transposed [i][j] table), copied once per workgroup into
// LDS ([wave][row], 8 bytes each), read one row ahead with the row's words (one ds_read_b64 at a
// wave-uniform address, two v_readfirstlane) and turned into addresses base + 72*c by SALU. The
// rows' scalar loads of round 2 (one 64-byte s_load of addresses per row, first touch of
// 64 MB written by the setup) exposed a memory latency on every row.
// ---------------------------------------------------------------------------------------------
#define SH_V2_STEP_ASM                                                                            \
    "v_mov_b32 v97, %[d0]\n"                                                                      \
    "v_mov_b32 v98, %[d1]\n"                                                                      \
    "v_mov_b32 v100, %[d2]\n"                                                                     \
    "v_mov_b32 v104, %[d3]\n"                                                                     \
    "v_mov_b32 v113, %[d4]\n"                                                                     \
    "v_mov_b32 v114, %[d5]\n"                                                                     \
    "v_mov_b32 v116, %[d6]\n"                                                                     \
    "v_mov_b32 v120, %[d7]\n"                                                                     \
    "v_xor_b32 v99, %[d0], %[d1]\n"                                                               \
    "v_xor_b32 v115, %[d4], %[d5]\n"                                                              \
    "v_xor_b32 v101, %[d0], %[d2]\n"                                                              \
    "v_xor_b32 v117, %[d4], %[d6]\n"                                                              \
    "v_xor_b32 v102, %[d1], %[d2]\n"                                                              \
    "v_xor_b32 v118, %[d5], %[d6]\n"                                                              \
    "v_xor_b32 v105, %[d0], %[d3]\n"                                                              \
    "v_xor_b32 v121, %[d4], %[d7]\n"                                                              \
    "v_xor_b32 v106, %[d1], %[d3]\n"                                                              \
    "v_xor_b32 v122, %[d5], %[d7]\n"                                                              \
    "v_xor_b32 v108, %[d2], %[d3]\n"                                                              \
    "v_xor_b32 v124, %[d6], %[d7]\n"                                                              \
    "v_xor_b32 v103, v99, %[d2]\n"                                                                \
    "v_xor_b32 v119, v115, %[d6]\n"                                                               \
    "v_xor_b32 v107, v99, %[d3]\n"                                                                \
    "v_xor_b32 v123, v115, %[d7]\n"                                                               \
    "v_xor_b32 v109, v101, %[d3]\n"                                                               \
    "v_xor_b32 v125, v117, %[d7]\n"                                                               \
    "v_xor_b32 v110, v102, %[d3]\n"                                                               \
    "v_xor_b32 v126, v118, %[d7]\n"                                                               \
    "v_xor_b32 v111, v103, %[d3]\n"                                                               \
    "v_xor_b32 v127, v119, %[d7]\n"                                                               \
    "s_mov_b32 s43, %[hi]\n"                                                                      \
    "s_bfe_u32 s42, %[c0], 0x80000\n"                                                             \
    "s_lshl3_add_u32 s42, s42, s42\n"                                                             \
    "s_lshl3_add_u32 s42, s42, %[lo]\n"                                                           \
    "s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)\n"                                                     \
    "s_swappc_b64 s[40:41], s[42:43]\n"                                                           \
    "s_bfe_u32 s42, %[c0], 0x80008\n"                                                             \
    "s_lshl3_add_u32 s42, s42, s42\n"                                                             \
    "s_lshl3_add_u32 s42, s42, %[lo]\n"                                                           \
    "s_set_gpr_idx_idx 8\n"                                                                       \
    "s_swappc_b64 s[40:41], s[42:43]\n"                                                           \
    "s_bfe_u32 s42, %[c0], 0x80010\n"                                                             \
    "s_lshl3_add_u32 s42, s42, s42\n"                                                             \
    "s_lshl3_add_u32 s42, s42, %[lo]\n"                                                           \
    "s_set_gpr_idx_idx 16\n"                                                                      \
    "s_swappc_b64 s[40:41], s[42:43]\n"                                                           \
    "s_lshr_b32 s42, %[c0], 24\n"                                                                 \
    "s_lshl3_add_u32 s42, s42, s42\n"                                                             \
    "s_lshl3_add_u32 s42, s42, %[lo]\n"                                                           \
    "s_set_gpr_idx_idx 24\n"                                                                      \
    "s_swappc_b64 s[40:41], s[42:43]\n"                                                           \
    "s_bfe_u32 s42, %[c1], 0x80000\n"                                                             \
    "s_lshl3_add_u32 s42, s42, s42\n"                                                             \
    "s_lshl3_add_u32 s42, s42, %[lo]\n"                                                           \
    "s_set_gpr_idx_idx 32\n"                                                                      \
    "s_swappc_b64 s[40:41], s[42:43]\n"                                                           \
    "s_bfe_u32 s42, %[c1], 0x80008\n"                                                             \
    "s_lshl3_add_u32 s42, s42, s42\n"                                                             \
    "s_lshl3_add_u32 s42, s42, %[lo]\n"                                                           \
    "s_set_gpr_idx_idx 40\n"                                                                      \
    "s_swappc_b64 s[40:41], s[42:43]\n"                                                           \
    "s_bfe_u32 s42, %[c1], 0x80010\n"                                                             \
    "s_lshl3_add_u32 s42, s42, s42\n"                                                             \
    "s_lshl3_add_u32 s42, s42, %[lo]\n"                                                           \
    "s_set_gpr_idx_idx 48\n"                                                                      \
    "s_swappc_b64 s[40:41], s[42:43]\n"                                                           \
    "s_lshr_b32 s42, %[c1], 24\n"                                                                 \
    "s_lshl3_add_u32 s42, s42, s42\n"                                                             \
    "s_lshl3_add_u32 s42, s42, %[lo]\n"                                                           \
    "s_set_gpr_idx_idx 56\n"                                                                      \
    "s_swappc_b64 s[40:41], s[42:43]\n"                                                           \
    "s_set_gpr_idx_off"

// acc sets j += M(c_j) * d, c_j = byte j of (c0, c1) (a zero byte runs snippet 0: XORs of zeros)
__device__ __forceinline__ void v2_row(const Row8 &d, uint32_t c0, uint32_t c1, uint32_t lo, uint32_t hi,
                                       u32x16 &a01, u32x16 &a23, u32x16 &a45, u32x16 &a67, uint32_t &z0,
                                       uint32_t &z1) {
    asm volatile(SH_V2_STEP_ASM
                 : "+{v[32:47]}"(a01), "+{v[48:63]}"(a23), "+{v[64:79]}"(a45), "+{v[80:95]}"(a67),
                   "+{v96}"(z0), "+{v112}"(z1)
                 : [d0] "v"(d.w[0]), [d1] "v"(d.w[1]), [d2] "v"(d.w[2]), [d3] "v"(d.w[3]), [d4] "v"(d.w[4]),
                   [d5] "v"(d.w[5]), [d6] "v"(d.w[6]), [d7] "v"(d.w[7]), [c0] "s"(c0), [c1] "s"(c1),
                   [lo] "s"(lo), [hi] "s"(hi)
                 : "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107",
                   "v108", "v109", "v110", "v111", "v113", "v114", "v115", "v116", "v117", "v118", "v119",
                   "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "s40", "s41", "s42",
                   "s43", "m0", "scc", "memory");
}

constexpr int V2_MAXE = 128;  // emax = min(k, m) <= 128 whenever k + m <= 256

// Ring depth: 16 rows (4 per barrier group) for 4- and 8-wave workgroups; 8 rows (2 per group)
// for the 1- and 2-wave workgroups of emax <= 16, so their 16 KB rings let 9 of them share a CU.
// MAXE: the rows a wave's coefficient copy holds (16 for the 1-2-wave workgroups of emax <= 16;
// V2_MAXE for the others, and for the 1-2-wave tail launches of a larger emax).
template <int NW, int MAXE = (NW <= 2 ? 16 : V2_MAXE)>
__global__ __launch_bounds__(64 * NW) void stageb_v2(StageBV2Args a) {
    constexpr int RB_R = NW <= 2 ? 8 : 16, RB_S = RB_R / 4;
    __shared__ __attribute__((aligned(16))) uint8_t ring[RB_R * RB_ROW];
    __shared__ __attribute__((aligned(8))) uint32_t cf[NW][MAXE][2];  // [wave][row] coefficient bytes
    const Geometry geo = a.geo;
    const int ncc = (geo.nq + 63) / 64;
    const int g = blockIdx.x / ncc;
    const int cc = blockIdx.x - g * ncc;
    const int c0 = cc * 64;
    const int ncols = min(64, geo.nq - c0);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int j0 = a.j_base + (blockIdx.y * NW + wave) * 8;
    // The prologue's loads do not depend on e (a scalar load of its own): the row list and this
    // wave's coefficient bytes are loaded for emax rows at once (entries past e are in the
    // group's workspace, unused), so e, the rows and the coefficients take one memory latency
    // together, the ring DMAs the next; loaded one after the other (each waiting for the last)
    // they took four.
    // the group's compacted residual-row list, 4 rows per lane (readlane by the issuing waves)
    uint32_t rrv;
    __builtin_memcpy(&rrv, a.rrow + static_cast<long long>(g) * a.ldR + 4 * (4 * lane < a.ldR ? lane : 0), 4);
    // this wave's coefficient bytes S^-1[j0..j0+7][i], i < emax (transposed table [i][j]: 8
    // contiguous bytes per row); rows 2l and 2l+1 per lane, written to LDS after the DMA issue
    constexpr int CFL = (2 * MAXE + 63) / 64;  // loads per lane
    const uint8_t *cg = a.coefT + static_cast<long long>(g) * a.coefT_gstride + (j0 < a.ldT ? j0 : 0);
    uint32_t cfw[CFL];
#pragma unroll
    for (int u = 0; u < CFL; ++u) {
        const int i = lane + 64 * u < 2 * a.emax ? lane + 64 * u : 0;  // unconditional: a static vmcnt
        __builtin_memcpy(&cfw[u], cg + static_cast<long long>(i >> 1) * a.ldT + 4 * (i & 1), 4);
    }
    const int e = a.e[g];
    // uniform over the workgroup: no erasures, or no output of this chunk below e (a group with
    // fewer erasures than emax: its later chunks would stream every row for nothing)
    if (e <= 0 || a.j_base + static_cast<int>(blockIdx.y) * NW * 8 >= e) return;
    const bool active = j0 < e;
    // this workgroup's input rows [i0, i0 + nr) (row slices; otherwise all e)
    const int i0 = a.row_slice > 0 ? static_cast<int>(blockIdx.z) * a.row_slice : 0;
    const int nr = a.row_slice > 0 ? max(0, min(e - i0, a.row_slice)) : e;
    const long long gbase = static_cast<long long>(g) * a.in_gstride;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.in + gbase), static_cast<short>(0), static_cast<int>(a.in_gstride), 0x00020000);
    // DMA pieces of a ring row (1 KB each): piece p by wave p; a one-wave workgroup issues both
    auto piece_src = [&](int p) {
        const int off = p * 1024 + lane * 16;
        const int sa = off / 256, cq = (off % 256) / 4;
        return (c0 + cq < geo.nq) ? colx_off(c0 + cq, geo.nq, geo.sub) + static_cast<uint32_t>(sa * geo.sub)
                                  : 0x80000000u;
    };
    const uint32_t dsrc = piece_src(NW >= 2 ? wave : 0);
    const uint32_t dsrc1 = NW >= 2 ? 0u : piece_src(1);
    const int elast = i0 + max(nr, 1) - 1;
    auto issue = [&](int i) {
        if (wave < 2) {
            const int x = min(i0 + i, elast);
            const uint32_t w = __builtin_amdgcn_readlane(rrv, x >> 2);
            const uint32_t soff = ((w >> (8 * (x & 3))) & 0xFFu) * static_cast<uint32_t>(geo.B);
            uint8_t *dst = ring + (i % RB_R) * RB_ROW + wave * 1024;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void *)dst, 16,
                                                     i < nr ? dsrc : 0x80000000u, soff, 0, 0);
            if (NW == 1)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void *)(dst + 1024), 16,
                                                         i < nr ? dsrc1 : 0x80000000u, soff, 0, 0);
        }
    };
    u32x16 a01, a23, a45, a67;
#pragma unroll
    for (int t = 0; t < 16; ++t) a01[t] = a23[t] = a45[t] = a67[t] = 0;
    uint32_t z0 = 0, z1 = 0;
    const uint32_t lo = static_cast<uint32_t>(a.snip_base), hi = static_cast<uint32_t>(a.snip_base >> 32);
    for (int i = 0; i < RB_R - RB_S; ++i) issue(i);
#pragma unroll
    for (int u = 0; u < CFL; ++u) {
        const int i = lane + 64 * u;
        if (i < 2 * e && active) cf[wave][i >> 1][i & 1] = cfw[u];
    }
    const int ngroups = (nr + RB_S - 1) / RB_S;
    for (int ig = 0; ig < ngroups; ++ig) {
        // own DMAs of rows RB_S*ig.. landed (RB_R - 2 * RB_S younger ones may be outstanding);
        // the first barrier also publishes the coefficient copies
        if (wave < 2)
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"((RB_R - 2 * RB_S) * (NW == 1 ? 2 : 1)) : "memory");
        else
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
        for (int r = 0; r < RB_S; ++r) issue(ig * RB_S + RB_R - RB_S + r);
        if (!active) continue;
#pragma unroll
        for (int r = 0; r < RB_S; ++r) {
            const int i = ig * RB_S + r;
            if (i >= nr) break;  // uniform
            const uint8_t *slot = ring + (i % RB_R) * RB_ROW + lane * 4;
            Row8 d;
#pragma unroll
            for (int s = 0; s < 8; ++s) d.w[s] = *reinterpret_cast<const uint32_t *>(slot + s * 256);
            const uint32_t q0 = __builtin_amdgcn_readfirstlane(cf[wave][i0 + i][0]);
            const uint32_t q1 = __builtin_amdgcn_readfirstlane(cf[wave][i0 + i][1]);
            v2_row(d, q0, q1, lo, hi, a01, a23, a45, a67, z0, z1);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no ring DMA may land after the workgroup ends
    if (!active || lane >= ncols) return;
    uint32_t acc[8][8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        acc[0][b] = a01[b]; acc[1][b] = a01[8 + b];
        acc[2][b] = a23[b]; acc[3][b] = a23[8 + b];
        acc[4][b] = a45[b]; acc[5][b] = a45[8 + b];
        acc[6][b] = a67[b]; acc[7][b] = a67[8 + b];
    }
    uint8_t *out = a.out + static_cast<long long>(g) * a.out_gstride + colx_off(c0 + lane, geo.nq, geo.sub) +
                   (a.row_slice > 0 ? static_cast<long long>(blockIdx.z) * a.out_slice_bytes : 0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (j0 + j >= e) break;
        uint8_t *row = out + static_cast<long long>(j0 + j) * geo.B;
#pragma unroll
        for (int b = 0; b < 8; ++b) __builtin_memcpy(row + b * geo.sub, &acc[j][b], 4);
    }
}

bool stageb_v2_ok(const Geometry &geo, int emax) {
    return geo.nq % 4 == 0 && geo.sub >= 16 && emax >= 1 && emax <= V2_MAXE;
}

hipError_t launch_stageb_v2(const StageBV2Args &a, hipStream_t stream) {
    if (a.groups <= 0 || a.emax <= 0) return hipSuccess;
    if (!stageb_v2_ok(a.geo, a.emax)) return hipErrorNotSupported;
    const int ncc = (a.geo.nq + 63) / 64;
    const int octets = (a.emax + 7) / 8;
    // Output chunks of 4 or 8 waves (32 or 64 outputs) per workgroup: a wave count that is not a
    // multiple of the CU's 4 SIMDs leaves one SIMD with an extra wave of every workgroup (5-7 waves
    // measured 10 % slower at e = 56, 66). Each chunk streams all e rows, so 8-wave chunks unless
    // 4-wave chunks need fewer wave slots (e = 66: 3 x 4 waves, 9 active, vs 2 x 8 with 7 idle):
    // (200,56,1352) stage B 0.478 vs 0.532 ms (7 waves), (190,66,1336) 0.763 vs 0.838 ms
    // (stageb_fixed), (120,136,1400) 1.772 vs 2.070 ms (4096 groups).
    // One or two output octets (emax <= 16): one workgroup of as many waves, no idle waves.
    static const int force = sh::measure_int(SH_MEASURE_ENV("SH_V2_NW"), 0);  // measurement
    const int c4 = (octets + 3) / 4, c8 = (octets + 7) / 8;
    const int nw = (force == 1 || force == 2) && octets <= 2 ? force                       // 1-2 waves hold <= 16 rows
                   : (force == 4 || force == 8) ? force
                   : (octets <= 2 ? octets : (8 * c8 <= 4 * c4 ? 8 : 4));
    // A last chunk with fewer octets than waves (e = 66: 3 x 4 waves, the third with one active
    // wave) runs as its own launch of 1- or 2-wave workgroups instead: no idle waves holding
    // registers and barrier slots (SH_V2_NO_TAIL: measurement switch).
    static const bool no_tail = SH_MEASURE_ENV("SH_V2_NO_TAIL") != nullptr;
    // One 8-wave chunk with 5 or 6 octets (e = 33..48): a 4-wave chunk plus a 1-2-wave tail.
    const int nw1 = (!no_tail && force == 0 && nw == 8 && (octets == 5 || octets == 6)) ? 4 : nw;
    int chunks = (octets + nw1 - 1) / nw1;
    const int rem = octets - (chunks - 1) * nw1;  // octets of the last chunk
    const bool tail = !no_tail && chunks > 1 && rem <= 2 && nw1 >= 4;
    if (tail) --chunks;
    StageBV2Args m = a;
    m.j_base = 0;
    const unsigned zs = a.row_slice > 0 ? static_cast<unsigned>(a.row_slices) : 1u;
    dim3 grid(static_cast<unsigned>(ncc) * a.groups, chunks, zs);
    if (nw1 == 1)
        hipLaunchKernelGGL(stageb_v2<1>, grid, dim3(64), 0, stream, m);
    else if (nw1 == 2)
        hipLaunchKernelGGL(stageb_v2<2>, grid, dim3(128), 0, stream, m);
    else if (nw1 == 4)
        hipLaunchKernelGGL(stageb_v2<4>, grid, dim3(256), 0, stream, m);
    else
        hipLaunchKernelGGL(stageb_v2<8>, grid, dim3(512), 0, stream, m);
    if (tail) {
        m.j_base = chunks * nw1 * 8;
        dim3 tg(static_cast<unsigned>(ncc) * a.groups, 1, zs);
        if (rem == 1)
            hipLaunchKernelGGL((stageb_v2<1, V2_MAXE>), tg, dim3(64), 0, stream, m);
        else
            hipLaunchKernelGGL((stageb_v2<2, V2_MAXE>), tg, dim3(128), 0, stream, m);
    }
    return hipGetLastError();
}

// Decode stage B for small blocks (fixed geometry with nq <= 16 word columns, B <= 512). A
// group fills only nq lanes there, and a snippet's coefficient is wave-uniform, so stageb_fixed
// would leave 64 - nq lanes idle; here each lane applies its own group's coefficients instead and
// one wave serves 64 / nq groups. Per residual row every lane writes its 30 window-table entries
// (the reference's win_encode tables, cauchy_256.cpp:1426-1445, of its column's 8 words) to LDS
// laid out [entry][lane]; coefficient c is applied as 8 x (two table lookups + one XOR3) with the
// 16 entry indices of c (lo and 16 + hi of c * 2^b) read from a 256 x 16-byte table, each lookup
// address one v_perm_b32 (entry into byte 1, lane * 4 into byte 0) and one ds_read_b32. One wave
// per workgroup, so the table base is a compile-time offset.
bool stageb_small_ok(const Geometry &geo, int emax) {
    return geo.nq % 4 == 0 && geo.nq <= 16 && geo.sub >= 16 && emax >= 1 && emax <= 128;
}

__global__ __launch_bounds__(64) void stageb_small(StageBSmallArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t tab[32 * 64];  // 8 KB window tables [entry][lane]
    __shared__ __attribute__((aligned(16))) uint32_t rbt[256 * 4];  // entry bytes of c * 2^b, b = 0..7
    extern __shared__ uint8_t rrs[];  // row lists of the wave's groups, [gpw][emax] (launch-sized:
                                      // 2 KB fixed kept 11 workgroups per CU instead of 13)
    const Geometry geo = a.geo;
    const int lane = threadIdx.x;
    const int gpw = 64 / geo.nq;
    const int gs = lane / geo.nq, q = lane - gs * geo.nq;
    // Block order: every output chunk of a group block streams the same e residual rows, so the
    // chunks of one group block are dealt to one XCD back to back (block b -> XCD b % 8) and the
    // later ones read the rows from that XCD's L2; in chunk-major order ((224,32,256): 4 chunks)
    // each chunk fetched them from memory again (4.5x the rows' bytes, PMC).
    int gb = blockIdx.x, chunk = blockIdx.y;
    if (a.xcd_map) {
        const int nch = (a.emax + 7) / 8;
        const int i = static_cast<int>(blockIdx.x) >> 3;
        chunk = i % nch;
        gb = (i / nch) * 8 + (static_cast<int>(blockIdx.x) & 7);
        if (gb * gpw >= a.groups) return;  // padding blocks of the last XCD round
    }
    const int g0 = gb * gpw;
    const bool valid = gs < gpw && g0 + gs < a.groups;
    const int g = valid ? g0 + gs : g0;
    const int j0 = chunk * 8;
    for (int c = lane; c < 256; c += 64) {
        uint32_t w[4] = {0, 0, 0, 0};
        uint32_t v = static_cast<uint32_t>(c);
        for (int b = 0; b < 8; ++b) {
            w[b >> 1] |= ((v & 15u) | ((16u + (v >> 4)) << 8)) << (16 * (b & 1));
            v = (v << 1) ^ ((v & 0x80u) ? 0x187u : 0u);  // c * 2^b in GF(256)/0x187
        }
        for (int t = 0; t < 4; ++t) rbt[c * 4 + t] = w[t];
    }
    tab[lane] = 0;            // T0[0]
    tab[16 * 64 + lane] = 0;  // T1[0]
    for (int t = lane; t < gpw * a.emax; t += 64) {
        const int sl = t / a.emax, i = t - sl * a.emax;
        const int gg = g0 + sl;
        rrs[sl * a.emax + i] = (gg < a.groups && i < a.e[gg]) ? a.rrow[static_cast<long long>(gg) * a.ldR + i] : 0;
    }
    __syncthreads();
    const int el = valid ? max(a.e[g], 0) : 0;
    int emx = el;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) emx = max(emx, __shfl_xor(emx, o));
    emx = __builtin_amdgcn_readfirstlane(emx);
    if (emx <= j0) return;  // no lane has an output in this chunk

    const uint8_t *res = a.in + static_cast<long long>(g) * a.in_gstride + colx_off(q, geo.nq, geo.sub);
    const uint8_t *cp = a.coefT + static_cast<long long>(g) * a.coefT_gstride + j0;
    const uint32_t lane4 = static_cast<uint32_t>(lane) * 4u;
    auto load = [&](int i, uint32_t (&d)[8], uint64_t &cc) {
        // lanes past the wave's last group (gs >= gpw, or past the batch) read row 0 of group g0:
        // their rrs row was never written, and any other row could lie past the workspace
        const int r = valid ? rrs[gs * a.emax + min(i, max(el - 1, 0))] : 0;
        const uint8_t *p = res + static_cast<long long>(r) * geo.B;
#pragma unroll
        for (int s = 0; s < 8; ++s) __builtin_memcpy(&d[s], p + s * geo.sub, 4);
        cc = 0;
        if (i < el) __builtin_memcpy(&cc, cp + static_cast<long long>(i) * a.ldT, 8);
    };
    auto lk = [&](uint32_t addr) { return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(tab) + addr); };

    uint32_t acc[8][8];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj)
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[jj][b] = 0;
    uint32_t d[8], dn[8];
    uint64_t cc, ccn;
    load(0, d, cc);
    for (int i = 0; i < emx; ++i) {
        if (i + 1 < emx) load(i + 1, dn, ccn);  // next row in flight under this row's work
        // window tables of this row's words: T0 from d0..d3, T1 from d4..d7
        const uint32_t e3 = d[0] ^ d[1], e5 = d[0] ^ d[2], e6 = d[1] ^ d[2], e9 = d[0] ^ d[3];
        const uint32_t e10 = d[1] ^ d[3], e12 = d[2] ^ d[3], e7 = e3 ^ d[2];
        const uint32_t f3 = d[4] ^ d[5], f5 = d[4] ^ d[6], f6 = d[5] ^ d[6], f9 = d[4] ^ d[7];
        const uint32_t f10 = d[5] ^ d[7], f12 = d[6] ^ d[7], f7 = f3 ^ d[6];
        const uint32_t tv[32] = {0, d[0], d[1], e3, d[2], e5, e6, e7, d[3], e9, e10, e3 ^ d[3], e12, e5 ^ d[3], e6 ^ d[3], e7 ^ d[3],
                                 0, d[4], d[5], f3, d[6], f5, f6, f7, d[7], f9, f10, f3 ^ d[7], f12, f5 ^ d[7], f6 ^ d[7], f7 ^ d[7]};
#pragma unroll
        for (int t = 1; t < 32; ++t)
            if (t != 16) tab[t * 64 + lane] = tv[t];
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
            const uint32_t c = static_cast<uint32_t>(cc >> (8 * jj)) & 0xFFu;
            const u32x4 rb = *reinterpret_cast<const u32x4 *>(&rbt[c * 4]);
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                const uint32_t w = rb[b >> 1];
                const uint32_t k = 2u * (b & 1);  // byte k: T0 entry, byte k + 1: T1 entry
                const uint32_t a0 = __builtin_amdgcn_perm(w, lane4, 0x0C0C0000u | ((4u + k) << 8));
                const uint32_t a1 = __builtin_amdgcn_perm(w, lane4, 0x0C0C0000u | ((5u + k) << 8));
                acc[jj][b] = __builtin_amdgcn_bitop3_b32(acc[jj][b], lk(a0), lk(a1), 0x96);
            }
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int s = 0; s < 8; ++s) d[s] = dn[s];
        cc = ccn;
    }
    if (!valid) return;
    uint8_t *out = a.out + static_cast<long long>(g) * a.out_gstride + colx_off(q, geo.nq, geo.sub);
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
        if (j0 + jj >= el) break;
        uint8_t *row = out + static_cast<long long>(j0 + jj) * geo.B;
#pragma unroll
        for (int b = 0; b < 8; ++b) __builtin_memcpy(row + b * geo.sub, &acc[jj][b], 4);
    }
}

// Two word columns per lane (stageb_small2): the two columns of a lane belong to one group, so
// both take the same table entry for a coefficient and one ds_read_b64 fetches the pair — the
// LDS array serves 8-byte reads at twice the 4-byte rate (MI355X_MICROARCH.md §LDS: ~150 vs
// ~75 TB/s chip-wide), and the lookups are most of stageb_small's LDS time. Table layout
// [half][entry][lane & 31] of uint2 (half = lane >> 5, 8 KB each), so an address is still one
// v_perm_b32: entry + 32 * half in byte 1 (pre-added in the half's copy of the entry table) and
// (lane & 31) * 8 in byte 0. Per launch at (224,32,256) (PMC, ab_runs block 10): LDS instructions
// 6.4e7 -> 3.2e7, VALU 1.14e8 -> 7.8e7; with 24 KB of LDS and 212 VGPRs a CU holds 6 of these
// waves (11-13 of stageb_small's), so the stage gains 7 %, not the halved lookup time.
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(64) void stageb_small2(StageBSmallArgs a) {
    __shared__ __attribute__((aligned(16))) u32x2 tab[2 * 32 * 32];        // 16 KB window tables
    __shared__ __attribute__((aligned(16))) uint32_t rbt[2 * 256 * 4];     // entry bytes per half
    extern __shared__ uint8_t rrs[];
    const Geometry geo = a.geo;
    const int lane = threadIdx.x;
    const int lpg = geo.nq / 2;  // lanes per group
    const int gpw = 64 / lpg;
    const int gs = lane / lpg, ql = lane - gs * lpg;
    int gb = blockIdx.x, chunk = blockIdx.y;
    if (a.xcd_map) {  // as stageb_small: the chunks of one group block on one XCD, back to back
        const int nch = (a.emax + 7) / 8;
        const int i = static_cast<int>(blockIdx.x) >> 3;
        chunk = i % nch;
        gb = (i / nch) * 8 + (static_cast<int>(blockIdx.x) & 7);
        if (gb * gpw >= a.groups) return;
    }
    const int g0 = gb * gpw;
    const bool valid = gs < gpw && g0 + gs < a.groups;
    const int g = valid ? g0 + gs : g0;
    const int j0 = chunk * 8;
    for (int t = lane; t < 2 * 256; t += 64) {
        const int h = t >> 8, c = t & 255;
        uint32_t w[4] = {0, 0, 0, 0};
        uint32_t v = static_cast<uint32_t>(c);
        for (int b = 0; b < 8; ++b) {
            const uint32_t lo = (v & 15u) + 32u * h, hi = 16u + (v >> 4) + 32u * h;
            w[b >> 1] |= (lo | (hi << 8)) << (16 * (b & 1));
            v = (v << 1) ^ ((v & 0x80u) ? 0x187u : 0u);  // c * 2^b in GF(256)/0x187
        }
        for (int u = 0; u < 4; ++u) rbt[t * 4 + u] = w[u];
    }
    const int half = lane >> 5;
    const int lbase = half * 32 * 32 + (lane & 31);  // tab index of entry 0 for this lane
    tab[lbase] = u32x2{0u, 0u};             // T0[0]
    tab[lbase + 16 * 32] = u32x2{0u, 0u};   // T1[0]
    for (int t = lane; t < gpw * a.emax; t += 64) {
        const int sl = t / a.emax, i = t - sl * a.emax;
        const int gg = g0 + sl;
        rrs[sl * a.emax + i] = (gg < a.groups && i < a.e[gg]) ? a.rrow[static_cast<long long>(gg) * a.ldR + i] : 0;
    }
    __syncthreads();
    const int el = valid ? max(a.e[g], 0) : 0;
    int emx = el;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) emx = max(emx, __shfl_xor(emx, o));
    emx = __builtin_amdgcn_readfirstlane(emx);
    if (emx <= j0) return;

    // the lane's two words are adjacent (colx_off shifts the last four columns together)
    const uint32_t coff = colx_off(2 * ql, geo.nq, geo.sub);
    const uint8_t *res = a.in + static_cast<long long>(g) * a.in_gstride + coff;
    const uint8_t *cp = a.coefT + static_cast<long long>(g) * a.coefT_gstride + j0;
    const uint32_t lane8 = static_cast<uint32_t>(lane & 31) * 8u;
    const uint32_t *rbh = rbt + half * 256 * 4;
    auto load = [&](int i, u32x2 (&d)[8], uint64_t &cc) {
        const int r = valid ? rrs[gs * a.emax + min(i, max(el - 1, 0))] : 0;
        const uint8_t *p = res + static_cast<long long>(r) * geo.B;
#pragma unroll
        for (int s = 0; s < 8; ++s) __builtin_memcpy(&d[s], p + s * geo.sub, 8);
        cc = 0;
        if (i < el) __builtin_memcpy(&cc, cp + static_cast<long long>(i) * a.ldT, 8);
    };
    auto lk = [&](uint32_t addr) {
        return *reinterpret_cast<const u32x2 *>(reinterpret_cast<const uint8_t *>(tab) + addr);
    };

    u32x2 acc[8][8];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj)
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[jj][b] = u32x2{0u, 0u};
    u32x2 d[8];
    uint64_t cc, ccn = 0;
    load(0, d, cc);
    for (int i = 0; i < emx; ++i) {
        const u32x2 e3 = d[0] ^ d[1], e5 = d[0] ^ d[2], e6 = d[1] ^ d[2], e9 = d[0] ^ d[3];
        const u32x2 e10 = d[1] ^ d[3], e12 = d[2] ^ d[3], e7 = e3 ^ d[2];
        const u32x2 f3 = d[4] ^ d[5], f5 = d[4] ^ d[6], f6 = d[5] ^ d[6], f9 = d[4] ^ d[7];
        const u32x2 f10 = d[5] ^ d[7], f12 = d[6] ^ d[7], f7 = f3 ^ d[6];
        const u32x2 tv[32] = {{0u, 0u}, d[0], d[1], e3, d[2], e5, e6, e7, d[3], e9, e10, e3 ^ d[3], e12, e5 ^ d[3], e6 ^ d[3], e7 ^ d[3],
                              {0u, 0u}, d[4], d[5], f3, d[6], f5, f6, f7, d[7], f9, f10, f3 ^ d[7], f12, f5 ^ d[7], f6 ^ d[7], f7 ^ d[7]};
#pragma unroll
        for (int t = 1; t < 32; ++t)
            if (t != 16) tab[lbase + t * 32] = tv[t];
        // the row's words are in LDS now: the next row loads into the same registers
        if (i + 1 < emx) load(i + 1, d, ccn);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
            const uint32_t c = static_cast<uint32_t>(cc >> (8 * jj)) & 0xFFu;
            const u32x4 rb = *reinterpret_cast<const u32x4 *>(&rbh[c * 4]);
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                const uint32_t w = rb[b >> 1];
                const uint32_t k = 2u * (b & 1);  // byte k: T0 entry, byte k + 1: T1 entry
                const uint32_t a0 = __builtin_amdgcn_perm(w, lane8, 0x0C0C0000u | ((4u + k) << 8));
                const uint32_t a1 = __builtin_amdgcn_perm(w, lane8, 0x0C0C0000u | ((5u + k) << 8));
                const u32x2 x0 = lk(a0), x1 = lk(a1);
                acc[jj][b].x = __builtin_amdgcn_bitop3_b32(acc[jj][b].x, x0.x, x1.x, 0x96);
                acc[jj][b].y = __builtin_amdgcn_bitop3_b32(acc[jj][b].y, x0.y, x1.y, 0x96);
            }
        }
        __builtin_amdgcn_wave_barrier();
        cc = ccn;
    }
    if (!valid) return;
    uint8_t *out = a.out + static_cast<long long>(g) * a.out_gstride + coff;
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
        if (j0 + jj >= el) break;
        uint8_t *row = out + static_cast<long long>(j0 + jj) * geo.B;
#pragma unroll
        for (int b = 0; b < 8; ++b) __builtin_memcpy(row + b * geo.sub, &acc[jj][b], 8);
    }
}

hipError_t launch_stageb_small(const StageBSmallArgs &a, hipStream_t stream) {
    if (a.groups <= 0 || a.emax <= 0) return hipSuccess;
    if (!stageb_small_ok(a.geo, a.emax)) return hipErrorNotSupported;
    const int gpw = 64 / a.geo.nq;
    const int ngb = (a.groups + gpw - 1) / gpw, nch = (a.emax + 7) / 8;
    static const bool xcd = sh::measure_int(SH_MEASURE_ENV("SH_SMALL_XCD"), 1) != 0;  // measurement
    StageBSmallArgs m = a;
    m.xcd_map = xcd && nch > 1 ? 1 : 0;
    // Two word columns per lane (stageb_small2, ab_runs block 10: (224,32,256) 0.410 -> 0.380 ms,
    // (112,16,256) -2 %, (28,4,256) equal); measurement builds: SH_SMALL2=0 runs stageb_small.
    static const bool two = sh::measure_int(SH_MEASURE_ENV("SH_SMALL2"), 1) != 0;
    if (two) {
        const int gpw2 = 64 / (a.geo.nq / 2);
        const int ngb2 = (a.groups + gpw2 - 1) / gpw2;
        const dim3 grid2 = m.xcd_map ? dim3(static_cast<unsigned>(8 * nch * ((ngb2 + 7) / 8)), 1, 1)
                                     : dim3(static_cast<unsigned>(ngb2), static_cast<unsigned>(nch), 1);
        const size_t rrs2 = (static_cast<size_t>(gpw2) * a.emax + 15) & ~static_cast<size_t>(15);
        hipLaunchKernelGGL(stageb_small2, grid2, dim3(64), rrs2, stream, m);
        return hipGetLastError();
    }
    const dim3 grid = m.xcd_map ? dim3(static_cast<unsigned>(8 * nch * ((ngb + 7) / 8)), 1, 1)
                                : dim3(static_cast<unsigned>(ngb), static_cast<unsigned>(nch), 1);
    const size_t rrs_bytes = (static_cast<size_t>(gpw) * a.emax + 15) & ~static_cast<size_t>(15);
    hipLaunchKernelGGL(stageb_small, grid, dim3(64), rrs_bytes, stream, m);
    return hipGetLastError();
}

bool stageb_fixed_ok(const Geometry &geo, int emax) {
    // whole 4-column chunks (fixed_geometry) and one snippet accumulator set per output
    return geo.nq % 4 == 0 && geo.sub >= 16 && emax >= 1;
}

hipError_t launch_stageb_fixed(const StageBFixedArgs &a, hipStream_t stream) {
    if (a.groups <= 0 || a.emax <= 0) return hipSuccess;
    if (!stageb_fixed_ok(a.geo, a.emax)) return hipErrorNotSupported;
    const int ncc = (a.geo.nq + 63) / 64;
    dim3 grid(static_cast<unsigned>(ncc) * a.groups, (a.emax + 31) / 32, 1);
    if (a.emax <= 16)
        hipLaunchKernelGGL(stageb_regs, grid, dim3(256), 0, stream, a);
    else
        hipLaunchKernelGGL(stageb_fixed, grid, dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t stageb_snip_base(uint64_t *out_host, hipStream_t stream) {
    uint64_t *d = nullptr;
    hipError_t err = hipMalloc(&d, sizeof(uint64_t));
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(stageb_snip_probe, dim3(1), dim3(64), 0, stream, d);
    err = hipGetLastError();
    if (err == hipSuccess) err = hipMemcpyAsync(out_host, d, sizeof(uint64_t), hipMemcpyDeviceToHost, stream);
    if (err == hipSuccess) err = hipStreamSynchronize(stream);
    (void)hipFree(d);
    return err;
}

hipError_t launch_stageb(const StageBArgs &a, int emax, hipStream_t stream) {
    if (a.groups <= 0 || emax <= 0) return hipSuccess;
    dim3 grid(static_cast<unsigned>((a.geo.nq + 63) / 64) * a.groups, (emax + 31) / 32, 1);
    hipLaunchKernelGGL(stageb_snip, grid, dim3(256), 0, stream, a);
    return hipGetLastError();
}

}  // namespace sh
