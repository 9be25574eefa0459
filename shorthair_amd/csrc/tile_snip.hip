// Runtime-coefficient tile kernels: ONE code path for every (k, m) the compile-time kernels do
// not cover (reference cauchy_256_encode serves every k + m <= 256 with one loop,
// cauchy_256.cpp:1519-1536 -> win_encode :1398-1477; Shorthair picks k = packets queued in the
// interval and m from the loss estimate, Shorthair.cpp:1130-1174, so most real calls are
// off-grid shapes).
//
// Same tile as the generated kernels (fixed_common.hpp): a workgroup covers COLS = 64*CW word
// columns of consecutive groups with CW column-waves x P part-waves (8 output rows each), the
// input blocks stream through one LDS-DMA ring per workgroup, and the output rows leave through
// the row-assembled stores (RowSink). What differs is the step body: instead of straight-line
// code with the coefficients baked in, a step builds the input's two 4-bit window tables
// (reference win_encode tables, cauchy_256.cpp:1426-1445) into pinned VGPRs and reaches, for
// each of the part's 8 rows, the compile-time snippet that applies M(C[y][x]) (the stage-B
// snippet table, csrc/gen/snippets.h) with one s_swappc_b64 in VGPR-index mode. The snippet
// addresses of every (step, row) are a per-(k, m) table built once on the host; the kernels
// load their low dwords with scalar loads (the 18 KB snippet table lies in one 4 GB page).
//
// Decode stage A is the same kernel over the k received blocks (erased columns read as zeros
// through out-of-range DMA offsets, per-group position tables in LDS) followed by one step per
// received recovery row, which XORs R_y into residual row y (snippet of coefficient 1 on row y
// only), exactly as the generated stage A does.
//
// m > 128 (k < 128 then) runs as several launches of <= 128 rows (16 part-waves), each
// re-reading the k input blocks.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fixed_common.hpp"
#include "kernels.hpp"

namespace sh {
namespace tile {

using fixed::OOR;
using fixed::lds_void;
using fixed::WGInfo;
using fixed::RowSink;

typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));

template <int P_, int CW_>
struct TShape {
    static constexpr int P = P_, CW = CW_, W = 16, PW = P_;  // all parts in one workgroup
    static constexpr int NW = CW * P, NT = 64 * NW, COLS = CW * 64;
    static constexpr int ROWB = COLS * 4, SLOT = 8 * ROWB, IMG = SLOT;
    static constexpr int NDMA = SLOT / (64 * W);
    static constexpr int DPW = (NDMA + NW - 1) / NW;
    // ring: <= 64 KB (two workgroups per CU; ds_read offsets), at least 2P slots (the row images alias it)
    static constexpr int RCAP = (65536 / SLOT) > 16 ? 16 : (65536 / SLOT);
    static constexpr int R = (2 * P > RCAP) ? 2 * P : RCAP;
    static constexpr int S = R >= 16 ? 4 : 2;  // steps per barrier (even: static register parity)
    static constexpr int AHEAD = R - 2 * S - 1;  // steps of DMA still in flight past the waited group
    static_assert(R * SLOT <= 65536, "ring must fit ds_read's 16-bit offsets");
    static_assert(AHEAD >= 1 && AHEAD * DPW < 64, "ring schedule");
};

template <class S, bool DEC>
struct TSrc {
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t dbase[S::DPW];
    int dgl[S::DPW];
    uint32_t B;
    int wave, n, x0, k, kp, pstride, row0;
    uint32_t rd;
    uint8_t *lds;
    const uint8_t *pos;

    __device__ __forceinline__ void init(const TileArgs &t, const WGInfo &w, uint8_t *lds_ring,
                                         const uint8_t *lds_pos) {
        const FixedArgs &a = t.f;
        const Geometry &geo = a.geo;
        rsrc = fixed::wg_rsrc(a.in, a.in_bytes, a.in_gstride, w.g_first);
        B = geo.B;
        lds = lds_ring;
        pos = lds_pos;
        wave = w.wave;
        x0 = t.slice_steps > 0 ? static_cast<int>(blockIdx.y) * t.slice_steps : 0;
        n = t.slice_steps > 0 ? min(t.slice_steps, t.nsteps - x0) : t.nsteps;
        k = t.k;
        kp = (t.k + 3) & ~3;
        pstride = kp + ((t.m + 3) & ~3);
        row0 = t.row0;
        rd = static_cast<uint32_t>(w.c) * 4u;
        const uint32_t gstride = static_cast<uint32_t>(a.in_gstride);
#pragma unroll
        for (int j = 0; j < S::DPW; ++j) {
            const int off = (w.wave * S::DPW + j) * 64 * S::W + w.lane * S::W;
            const int aa = off / S::ROWB;
            const int cc = (off - aa * S::ROWB) / 4;
            const long long colx = w.col0 + cc;
            const int gx = colx >= 0 ? static_cast<int>(colx / geo.nq) : -1;
            const int qx = static_cast<int>(colx - static_cast<long long>(gx) * geo.nq);
            dgl[j] = gx - w.g_first;
            dbase[j] = (colx >= w.lo && colx < w.hi)
                           ? static_cast<uint32_t>(gx - w.g_first) * gstride + fixed::col_off(qx, geo) + aa * geo.sub
                           : OOR;
        }
    }

    // DMA of step x into slot x % R; steps past the last one are issued out of range (no memory
    // access) so the counted waits stay constant.
    __device__ __forceinline__ void issue(int x) const {
        uint8_t *slot = lds + (x % S::R) * S::SLOT;
#pragma unroll
        for (int j = 0; j < S::DPW; ++j) {
            if (S::NDMA % S::NW != 0 && wave * S::DPW + j >= S::NDMA) break;  // uniform
            lds_void *dst = (lds_void *)(slot + (wave * S::DPW + j) * 64 * S::W);
            uint32_t o = OOR, so = 0;
            if (x < n && dbase[j] != OOR) {
                const int gx = x0 + x;  // step of the whole range
                if (DEC) {
                    const int t = gx < k ? gx : kp + row0 + (gx - k);
                    const int p = pos[dgl[j] * pstride + t];
                    o = p == 0xFF ? OOR : dbase[j] + static_cast<uint32_t>(p) * B;
                } else {
                    o = dbase[j];
                    so = static_cast<uint32_t>(gx) * B;
                }
            }
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, dst, S::W, o, so, 0, 0);
        }
    }

    // Wait until this wave's DMAs of all but the youngest N steps are done, then join the barrier.
    template <int N>
    __device__ __forceinline__ void wait() const {
        if (S::NDMA % S::NW != 0 && wave * S::DPW >= S::NDMA)
            asm volatile("s_barrier" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N * S::DPW) : "memory");
    }

    __device__ __forceinline__ void read(int slot, uint32_t (&d)[8]) const {
        const uint8_t *p = lds + slot * S::SLOT + rd;
#pragma unroll
        for (int s = 0; s < 8; ++s) d[s] = *reinterpret_cast<const uint32_t *>(p + s * S::ROWB);
    }
};

// One step of a part-wave: window tables of the step's 8 words into v[96:127] (v96 = v112 = 0
// are the zero entries), then one snippet call per row of the part, call j in VGPR-index mode
// with M0 = 8j so the snippet's destination and first source are accumulator set j
// (v[32+8j .. 32+8j+7]). A zero address skips the call (two SALU): rows past the part's last,
// zero coefficients, and decode's recovery-row steps, which add the received block into one row
// of one part (the unit snippet) and call nothing elsewhere.
#define SH_TILE_STEP_ASM                                                                          \
    SH_TILE_TABLE_ASM                                                                             \
    SH_TILE_CALLS_ASM

#define SH_TILE_TABLE_ASM                                                                         \
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
    "v_xor_b32 v127, v119, %[d7]\n"

#define SH_TILE_CALLS_ASM                                                                         \
    "s_mov_b32 s43, %[hi]\n"                                                                      \
    "s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)\n"                                                     \
    "s_cmp_eq_u32 %[g0], 0\n"                                                                     \
    "s_cbranch_scc1 1f\n"                                                                         \
    "s_mov_b32 s42, %[g0]\n"                                                                      \
    "s_swappc_b64 s[40:41], s[42:43]\n"                                                           \
    "1:\n"                                                                                        \
    "s_set_gpr_idx_idx 8\n"                                                                       \
    "s_cmp_eq_u32 %[g1], 0\n"                                                                     \
    "s_cbranch_scc1 2f\n"                                                                         \
    "s_mov_b32 s42, %[g1]\n"                                                                      \
    "s_swappc_b64 s[40:41], s[42:43]\n"                                                           \
    "2:\n"                                                                                        \
    "s_set_gpr_idx_idx 16\n"                                                                      \
    "s_cmp_eq_u32 %[g2], 0\n"                                                                     \
    "s_cbranch_scc1 3f\n"                                                                         \
    "s_mov_b32 s42, %[g2]\n"                                                                      \
    "s_swappc_b64 s[40:41], s[42:43]\n"                                                           \
    "3:\n"                                                                                        \
    "s_set_gpr_idx_idx 24\n"                                                                      \
    "s_cmp_eq_u32 %[g3], 0\n"                                                                     \
    "s_cbranch_scc1 4f\n"                                                                         \
    "s_mov_b32 s42, %[g3]\n"                                                                      \
    "s_swappc_b64 s[40:41], s[42:43]\n"                                                           \
    "4:\n"                                                                                        \
    "s_set_gpr_idx_idx 32\n"                                                                      \
    "s_cmp_eq_u32 %[g4], 0\n"                                                                     \
    "s_cbranch_scc1 5f\n"                                                                         \
    "s_mov_b32 s42, %[g4]\n"                                                                      \
    "s_swappc_b64 s[40:41], s[42:43]\n"                                                           \
    "5:\n"                                                                                        \
    "s_set_gpr_idx_idx 40\n"                                                                      \
    "s_cmp_eq_u32 %[g5], 0\n"                                                                     \
    "s_cbranch_scc1 6f\n"                                                                         \
    "s_mov_b32 s42, %[g5]\n"                                                                      \
    "s_swappc_b64 s[40:41], s[42:43]\n"                                                           \
    "6:\n"                                                                                        \
    "s_set_gpr_idx_idx 48\n"                                                                      \
    "s_cmp_eq_u32 %[g6], 0\n"                                                                     \
    "s_cbranch_scc1 7f\n"                                                                         \
    "s_mov_b32 s42, %[g6]\n"                                                                      \
    "s_swappc_b64 s[40:41], s[42:43]\n"                                                           \
    "7:\n"                                                                                        \
    "s_set_gpr_idx_idx 56\n"                                                                      \
    "s_cmp_eq_u32 %[g7], 0\n"                                                                     \
    "s_cbranch_scc1 8f\n"                                                                         \
    "s_mov_b32 s42, %[g7]\n"                                                                      \
    "s_swappc_b64 s[40:41], s[42:43]\n"                                                           \
    "8:\n"                                                                                        \
    "s_set_gpr_idx_off"

struct Acc {
    u32x16 a01, a23, a45, a67;
    uint32_t z0, z1;
};

__device__ __forceinline__ void step(const uint32_t (&d)[8], const uint32_t *g, uint32_t hi, Acc &A) {
    asm volatile(SH_TILE_STEP_ASM
                 : "+{v[32:47]}"(A.a01), "+{v[48:63]}"(A.a23), "+{v[64:79]}"(A.a45), "+{v[80:95]}"(A.a67),
                   "+{v96}"(A.z0), "+{v112}"(A.z1)
                 : [d0] "v"(d[0]), [d1] "v"(d[1]), [d2] "v"(d[2]), [d3] "v"(d[3]), [d4] "v"(d[4]),
                   [d5] "v"(d[5]), [d6] "v"(d[6]), [d7] "v"(d[7]), [g0] "s"(g[0]), [g1] "s"(g[1]),
                   [g2] "s"(g[2]), [g3] "s"(g[3]), [g4] "s"(g[4]), [g5] "s"(g[5]), [g6] "s"(g[6]),
                   [g7] "s"(g[7]), [hi] "s"(hi)
                 : "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107",
                   "v108", "v109", "v110", "v111", "v113", "v114", "v115", "v116", "v117", "v118", "v119",
                   "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "s40", "s41", "s42",
                   "s43", "m0", "scc", "memory");
}

// Column-snippet step (m >= 7, csrc/gen/colsnip_*.hip): the same window tables, then one call per
// 4-row block of the part (g0, g1: snippet-address low dwords; 0 = no call). A column snippet
// applies all 4 rows' coefficients of the input to its accumulator half with absolute register
// numbers, so no VGPR-index mode and 1/4 of the calls.
#define SH_COL_STEP_ASM                                                                           \
    SH_TILE_TABLE_ASM                                                                             \
    "s_cmp_eq_u32 %[g0], 0\n"                                                                     \
    "s_cbranch_scc1 9f\n"                                                                         \
    "s_mov_b32 s43, %[hi]\n"                                                                      \
    "s_mov_b32 s42, %[g0]\n"                                                                      \
    "s_swappc_b64 s[40:41], s[42:43]\n"                                                           \
    "s_cmp_eq_u32 %[g1], 0\n"                                                                     \
    "s_cbranch_scc1 9f\n"                                                                         \
    "s_mov_b32 s42, %[g1]\n"                                                                      \
    "s_swappc_b64 s[40:41], s[42:43]\n"                                                           \
    "9:\n"

__device__ __forceinline__ void step_col(const uint32_t (&d)[8], uint32_t g0, uint32_t g1, uint32_t hi, Acc &A) {
    asm volatile(SH_COL_STEP_ASM
                 : "+{v[32:47]}"(A.a01), "+{v[48:63]}"(A.a23), "+{v[64:79]}"(A.a45), "+{v[80:95]}"(A.a67),
                   "+{v96}"(A.z0), "+{v112}"(A.z1)
                 : [d0] "v"(d[0]), [d1] "v"(d[1]), [d2] "v"(d[2]), [d3] "v"(d[3]), [d4] "v"(d[4]),
                   [d5] "v"(d[5]), [d6] "v"(d[6]), [d7] "v"(d[7]), [g0] "s"(g0), [g1] "s"(g1), [hi] "s"(hi)
                 : "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107",
                   "v108", "v109", "v110", "v111", "v113", "v114", "v115", "v116", "v117", "v118", "v119",
                   "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "s40", "s41", "s42",
                   "s43", "scc", "memory");
}

// Every wave joins one barrier per row of a part (8), storing its part's rows < nr.
template <int YI, class Snk>
__device__ __forceinline__ void store_rows(const Snk &sink, int nr, int y0, const uint32_t (&acc)[8][8]) {
    if constexpr (YI == 0) sink.prepare();  // per-lane piece offsets, derived at the epilogue
    if constexpr (YI < 8) {
        if (YI < nr)
            sink.template row<YI>(y0 + YI, acc[YI]);
        else
            sink.template pad<YI>();
        store_rows<YI + 1>(sink, nr, y0, acc);
    }
}

// Column mode: rows of a part are 4-row blocks b0, b0+1 whose accumulator halves follow the
// block's parity (the column snippets of block r write half r % 2), so row y0 + i lives in
// accumulator set (i + 4 * (b0 & 1)) % 8.
template <int ROT, class Snk>
__device__ __forceinline__ void store_rows_rot(const Snk &sink, int nr, int y0, const uint32_t (&acc)[8][8]) {
    if constexpr (ROT == 0) {
        store_rows<0>(sink, nr, y0, acc);
    } else {
        uint32_t r[8][8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int b = 0; b < 8; ++b) r[i][b] = acc[(i + ROT) & 7][b];
        store_rows<0>(sink, nr, y0, r);
    }
}

template <class S, bool DEC, bool COL>
__device__ __forceinline__ void tile_body(const TileArgs &t) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const FixedArgs &a = t.f;
    const Geometry &geo = a.geo;
    WGInfo w;
    w.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    w.lane = threadIdx.x & 63;
    const int part = w.wave % S::P;
    const int cw = w.wave / S::P;
    w.c = cw * 64 + w.lane;
    const long long col0 = static_cast<long long>(fixed::xcd_tile(blockIdx.x, gridDim.x)) * S::COLS;
    w.col0 = col0;
    w.lo = 0;
    w.hi = static_cast<long long>(a.groups) * geo.nq;
    const int nq = geo.nq;
    w.g_first = static_cast<int>(col0 / nq);
    const long long col = col0 + w.c;
    w.valid = col < w.hi;
    const int g = w.valid ? static_cast<int>(col / nq) : w.g_first;
    w.q = static_cast<int>(col - static_cast<long long>(g) * nq);
    w.gl = g - w.g_first;
    uint8_t *lds_pos = lds + S::R * S::SLOT;
    if (DEC) {  // stage the position tables of the tile's groups: [gpw][KP + MP]
        const int ng = a.groups_per_wg;
        const int ghi = a.groups;
        const int kp = (t.k + 3) & ~3, mp = (t.m + 3) & ~3;
        const int tw = (kp + mp) / 4;
        for (int i = threadIdx.x; i < ng * tw; i += S::NT) {
            const int lg = i / tw, u = i - lg * tw;
            const int gg = w.g_first + lg;
            uint32_t v = 0xFFFFFFFFu;
            if (gg < ghi)
                v = (u < kp / 4) ? reinterpret_cast<const uint32_t *>(a.pos + gg * static_cast<long long>(kp))[u]
                                 : reinterpret_cast<const uint32_t *>(a.rpos + gg * static_cast<long long>(mp))[u - kp / 4];
            reinterpret_cast<uint32_t *>(lds_pos)[i] = v;
        }
        __syncthreads();
    }
    TSrc<S, DEC> src;
    src.init(t, w, lds, lds_pos);
    RowSink<S> sink;
    FixedArgs so = a;  // this slice's partial output
    if (t.slice_steps > 0) {
        so.out += static_cast<long long>(blockIdx.y) * t.out_slice_bytes;
        so.out_bytes = t.out_slice_bytes;
    }
    sink.init(so, w, part, lds);

    // snippet-address low dwords of this part: [ngroups * S steps][8], scalar loads
    typedef const __attribute__((address_space(4))) uint32_t cu32_t;
    constexpr int PER = COL ? 2 : 8;  // snippet-address dwords per step
    const cu32_t *tp = (const cu32_t *)(t.targets + static_cast<long long>(part) * t.tstride + PER * static_cast<long long>(src.x0));
    const uint32_t hi = t.snip_hi;
    // this part's rows [y0, y0 + nr): the launch's rows split evenly over the P parts (4..8 each);
    // column mode: whole 4-row blocks [b0, b1) (one or two), tile_plan agrees
    const int nb4 = (t.nrows + 3) / 4;
    const int b0 = part * nb4 / S::P, b1 = (part + 1) * nb4 / S::P;
    const int y0 = COL ? 4 * b0 : part * t.nrows / S::P;
    const int nr = COL ? min(4 * b1, t.nrows) - y0 : (part + 1) * t.nrows / S::P - y0;

    Acc A;
#pragma unroll
    for (int i = 0; i < 16; ++i) A.a01[i] = A.a23[i] = A.a45[i] = A.a67[i] = 0;
    A.z0 = A.z1 = 0;

    const int n = src.n;
    const int ngroups = (n + S::S - 1) / S::S;
    for (int x = 0; x < S::R - 1; ++x) src.issue(x);
    src.template wait<S::R - S::S - 1>();
    uint32_t dA[8], dB[8];
    src.read(0, dA);
    for (int ig = 0; ig < ngroups; ++ig) {
        uint32_t gl[S::S * PER];
#pragma unroll
        for (int j = 0; j < S::S * PER; ++j) gl[j] = tp[ig * S::S * PER + j];
#pragma unroll
        for (int r = 0; r < S::S; ++r) {
            const int i = ig * S::S + r;
            uint32_t(&cur)[8] = (r & 1) ? dB : dA;
            uint32_t(&nxt)[8] = (r & 1) ? dA : dB;
            if (r == S::S - 1) {  // group boundary: steps <= i + S landed, every wave past step i - 1
                src.template wait<S::AHEAD>();
#pragma unroll
                for (int u = 0; u < S::S; ++u) src.issue(i + S::R - S::S + u);
            }
            if (i + 1 < n) src.read((i + 1) % S::R, nxt);
            if (i < n) {
                if (COL)
                    step_col(cur, gl[r * PER], gl[r * PER + 1], hi, A);
                else
                    step(cur, &gl[r * PER], hi, A);
            }
        }
    }
    // no ring DMA may land in the row images (they alias the ring)
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    uint32_t acc[8][8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        acc[0][b] = A.a01[b]; acc[1][b] = A.a01[8 + b];
        acc[2][b] = A.a23[b]; acc[3][b] = A.a23[8 + b];
        acc[4][b] = A.a45[b]; acc[5][b] = A.a45[8 + b];
        acc[6][b] = A.a67[b]; acc[7][b] = A.a67[8 + b];
    }
    if (COL && (b0 & 1))
        store_rows_rot<4>(sink, nr, y0, acc);
    else
        store_rows_rot<0>(sink, nr, y0, acc);
}

#define SH_TILE_KERNEL(P, CW)                                                                      \
    __global__ __launch_bounds__(64 * CW * P) void tile_enc_p##P(TileArgs t) {                    \
        tile_body<TShape<P, CW>, false, false>(t);                                                \
    }                                                                                             \
    __global__ __launch_bounds__(64 * CW * P) void tile_dec_p##P(TileArgs t) {                    \
        tile_body<TShape<P, CW>, true, false>(t);                                                 \
    }                                                                                             \
    __global__ __launch_bounds__(64 * CW * P) void tile_col_enc_p##P(TileArgs t) {                \
        tile_body<TShape<P, CW>, false, true>(t);                                                 \
    }                                                                                             \
    __global__ __launch_bounds__(64 * CW * P) void tile_col_dec_p##P(TileArgs t) {                \
        tile_body<TShape<P, CW>, true, true>(t);                                                  \
    }
// Part counts whose workgroups fill the CU's 4 SIMDs evenly (P * CW a multiple of 4; tile_parts)
SH_TILE_KERNEL(1, 4)
SH_TILE_KERNEL(2, 4)
SH_TILE_KERNEL(4, 2)
SH_TILE_KERNEL(6, 2)
SH_TILE_KERNEL(8, 2)
SH_TILE_KERNEL(12, 1)
SH_TILE_KERNEL(16, 1)

template <int P, int CW>
hipError_t launch_p(const TileArgs &t0, bool dec, hipStream_t s, void (*ke)(TileArgs), void (*kd)(TileArgs)) {
    using S = TShape<P, CW>;
    TileArgs t = t0;
    t.f.groups_per_wg = (S::COLS - 1) / t.f.geo.nq + 2;
    const int kp = (t.k + 3) & ~3, mp = (t.m + 3) & ~3;
    const size_t lds = static_cast<size_t>(S::R) * S::SLOT + (dec ? static_cast<size_t>(t.f.groups_per_wg) * (kp + mp) : 0);
    const long long cols = static_cast<long long>(t.f.groups) * t.f.geo.nq;
    const unsigned blocks = static_cast<unsigned>((cols + S::COLS - 1) / S::COLS);
    const unsigned slices = t.slice_steps > 0 ? static_cast<unsigned>(t.slices) : 1u;
    hipLaunchKernelGGL(dec ? kd : ke, dim3(blocks, slices), dim3(S::NT), lds, s, t);
    return hipGetLastError();
}

}  // namespace tile

// Parts (part-waves per column-wave) for a launch of nrows <= 128 output rows: the smallest
// balanced count with <= 8 rows per part. A workgroup whose wave count is not a multiple of the
// CU's 4 SIMDs leaves one SIMD with an extra wave of every workgroup (10 waves at (150,40):
// 3, 3, 2, 2); parts then hold 4..8 rows and skip their unused snippet calls.
int tile_parts(int nrows) {
    const int p0 = (nrows + 7) / 8;
    for (int p : {1, 2, 4, 6, 8, 12, 16})
        if (p >= p0) return p;
    return 0;
}

// The column-snippet tables live in the generated translation units (csrc/gen/colsnip_<t>.hip);
// each holds its table inside a probe kernel whose only launch reports the table's address.
__global__ void colsnip_probe_0(uint64_t *out);
__global__ void colsnip_probe_1(uint64_t *out);
__global__ void colsnip_probe_2(uint64_t *out);
__global__ void colsnip_probe_3(uint64_t *out);

hipError_t colsnip_bases(uint64_t *out_host, int n, hipStream_t stream) {
    if (n != 4) return hipErrorInvalidValue;
    uint64_t *d = nullptr;
    hipError_t err = hipMalloc(&d, 4 * sizeof(uint64_t));
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(colsnip_probe_0, dim3(1), dim3(64), 0, stream, d + 0);
    hipLaunchKernelGGL(colsnip_probe_1, dim3(1), dim3(64), 0, stream, d + 1);
    hipLaunchKernelGGL(colsnip_probe_2, dim3(1), dim3(64), 0, stream, d + 2);
    hipLaunchKernelGGL(colsnip_probe_3, dim3(1), dim3(64), 0, stream, d + 3);
    err = hipGetLastError();
    if (err == hipSuccess) err = hipMemcpyAsync(out_host, d, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, stream);
    if (err == hipSuccess) err = hipStreamSynchronize(stream);
    (void)hipFree(d);
    return err;
}

int tile_steps_per_group(int parts) {
    switch (parts) {
#define SH_S(P, CW) case P: return tile::TShape<P, CW>::S;
        SH_S(1, 4) SH_S(2, 4) SH_S(4, 2) SH_S(6, 2) SH_S(8, 2) SH_S(12, 1) SH_S(16, 1)
#undef SH_S
    }
    return 0;
}

bool tile_ok(int B) { return B % 8 == 0 && B / 8 >= 16; }

hipError_t launch_tile(const TileArgs &t, bool dec, hipStream_t s) {
    if (t.f.groups <= 0 || t.nrows <= 0) return hipSuccess;
    if (!tile_ok(t.f.geo.B)) return hipErrorNotSupported;
    switch (tile_parts(t.nrows)) {
#define SH_L(P, CW)                                                                              \
    case P:                                                                                      \
        return t.col ? tile::launch_p<P, CW>(t, dec, s, tile::tile_col_enc_p##P, tile::tile_col_dec_p##P) \
                     : tile::launch_p<P, CW>(t, dec, s, tile::tile_enc_p##P, tile::tile_dec_p##P);
        SH_L(1, 4) SH_L(2, 4) SH_L(4, 2) SH_L(6, 2) SH_L(8, 2) SH_L(12, 1) SH_L(16, 1)
#undef SH_L
    }
    return hipErrorNotSupported;
}

}  // namespace sh
