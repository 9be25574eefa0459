// Runtime-coefficient bitmatrix product through a table of compile-time snippets (decode stage B).
//
//   out[g][j] = sum_y M(coef[g][y][j]) * in[g][y]        (j < e_g outputs, y < n_in inputs)
//
// The coefficients (S^-1 of a group's erasure pattern) are only known at run time, so the
// compile-time schedule of the encode kernels does not apply, and a register table indexed by a
// runtime (wave-uniform) value costs 8.7x (hipcc's s_set_gpr_idx lowering). Here the
// runtime choice is made ONCE per coefficient instead of once per table lookup: 256 snippets,
// one per coefficient value c, each computing tmp[b] = T0[lo(c*2^b)] ^ T1[hi(c*2^b)] for b = 0..7
// with compile-time register operands, are emitted inside the kernel (csrc/gen/snippets.h); the
// kernel reaches snippet c with one s_swappc_b64 and returns with s_setpc_b64. The window tables
// T0/T1 of the current input (the reference's win_encode tables, cauchy_256.cpp:1426-1445) and
// tmp live in VGPRs pinned through explicit-register asm operands, so hipcc keeps its own values
// out of them.
//
// One workgroup = one group x 64 word columns x 32 outputs (4 waves x 8 outputs). Group-uniform
// coefficients require a wave to stay inside one group: at B = 1400 a group has 44 word columns.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.hpp"
#include "snippets.h"

#include <algorithm>
#include <cstdlib>

namespace sh {

typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));

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

static_assert(SH_SNIPA_ACC == 32 && SH_SNIPA_T0 == 96 && SH_SNIPA_T1 == 112,
              "accumulating-snippet registers must match the asm constraints");
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

// LDS-staged variant (the fixed-generator decode path: n_in <= 32, nq % 4 == 0, sub >= 16). One
// workgroup = one group x one 64-column chunk x 32 outputs (4 waves x 8). The group's residual
// rows for the chunk (n_in x 8 sub-blocks x ncols words, <= 64 KB) are gathered into LDS by
// LDS-DMA up front, so the loop over input rows reads LDS (the next row prefetched into
// registers under the current row's snippet calls) instead of waiting on HBM once per row.
// Columns follow the fixed kernels' layout: the last 4-column chunk of each sub-block is
// shifted back to end at the sub-block's end (fixed_common.hpp), so loads and stores are whole
// dwords with no tail handling.
__device__ __forceinline__ uint32_t colx_off(int q, int nq, int sub) {
    return 4u * q - (q >= nq - 4 ? static_cast<uint32_t>(4 * nq - sub) : 0u);
}

typedef __attribute__((address_space(3))) void lds_void_t;

__global__ __launch_bounds__(256, 3) void stageb_lds(StageBArgs a) {
    SH_SNIPPET_TABLE(L);
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const Geometry geo = a.geo;
    const int ncc = (geo.nq + 63) / 64;
    const int g = blockIdx.x / ncc;
    const int cc = blockIdx.x - g * ncc;
    const int c0 = cc * 64;
    const int ncols = min(64, geo.nq - c0);
    const int nch = ncols / 4;        // 16-byte chunks per (row, sub-block)
    const int cpb = nch * 16;         // LDS bytes per (row, sub-block)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int e = a.e[g];
    const int j0 = (blockIdx.y * 4 + wave) * 8;

    // ---- gather the residual tile into LDS: chunk ch = (y*8 + a)*nch + t; then the group's
    // stage-B coefficients (n_in x ldT bytes) behind it
    const int total = a.n_in * 8 * nch;
    const int tile = ((total + 255) / 256) * 256 * 16;
    uint8_t *lcoef = lds + tile;
    {
        const long long gbase = static_cast<long long>(g) * a.in_gstride;
        long long avail = static_cast<long long>(a.groups) * a.in_gstride + a.in_slack - gbase;
        if (avail > 0x7FFFFFFFll) avail = 0x7FFFFFFFll;
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t *>(a.in + gbase), static_cast<short>(0), static_cast<int>(avail), 0x00020000);
        for (int base = wave * 64; base < total; base += 256) {  // uniform
            const int ch = base + lane;
            uint32_t off = 0x80000000u;
            if (ch < total) {
                const int ya = ch / nch, t = ch - ya * nch;
                const int y = ya >> 3, sa = ya & 7;
                off = static_cast<uint32_t>(y) * geo.B + static_cast<uint32_t>(sa) * geo.sub +
                      colx_off(c0 + 4 * t, geo.nq, geo.sub);
            }
            __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t *)(lds + base * 16), 16, off, 0, 0, 0);
        }
        const int cbytes = a.n_in * a.ldT;  // multiple of 8; <= 32 * 32
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t *>(a.coefT + static_cast<long long>(g) * a.coefT_gstride), static_cast<short>(0),
            cbytes, 0x00020000);
        for (int base = wave * 64; base * 16 < cbytes; base += 256)  // uniform
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rc, (lds_void_t *)(lcoef + base * 16), 16, (base + lane) * 16, 0, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    if (j0 >= e) return;  // wave-uniform (after the barrier)

    uint64_t snip;
    asm volatile(
        "s_getpc_b64 s[42:43]\n"
        "s_add_u32 s42, s42, sh_snip_baseL@rel32@lo+4\n"
        "s_addc_u32 s43, s43, sh_snip_baseL@rel32@hi+12\n"
        "s_mov_b64 %0, s[42:43]"
        : "=s"(snip)
        :
        : "s42", "s43", "scc");

    const uint8_t *rd = lds + 4 * lane;
    const uint8_t *cf = lcoef + j0;

    uint32_t acc[8][8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[j][b] = 0;

    // rows and coefficients are prefetched one input row ahead (LDS latency under the calls)
    uint32_t d[8], dn[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) d[s] = *reinterpret_cast<const uint32_t *>(rd + s * cpb);
    uint2 cv = *reinterpret_cast<const uint2 *>(cf);
    for (int y = 0; y < a.n_in; ++y) {
        const int yn = y + 1 < a.n_in ? y + 1 : y;
#pragma unroll
        for (int s = 0; s < 8; ++s) dn[s] = *reinterpret_cast<const uint32_t *>(rd + (yn * 8 + s) * cpb);
        const uint2 cvn = *reinterpret_cast<const uint2 *>(cf + yn * a.ldT);
        const uint32_t clo = __builtin_amdgcn_readfirstlane(cv.x), chi = __builtin_amdgcn_readfirstlane(cv.y);
        if ((clo | chi) != 0) {  // wave-uniform: no output of this wave uses input y otherwise
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
                // dense S^-1 (every coefficient of a received row is nonzero for e = m): no per-j
                // skip; a zero coefficient simply runs snippet 0 (adds nothing)
                const uint32_t c = ((j < 4 ? clo : chi) >> (8 * (j & 3))) & 0xffu;
                u32x8 tmp;
#ifndef SH_EXPERIMENT_NO_CALL
                SH_SNIP_CALL(snip + (static_cast<uint64_t>(c) << 6), t0, t1, tmp);
#else  // timing experiment only: the table work and accumulation without the call
                for (int b = 0; b < 8; ++b) tmp[b] = t0[(c + b) & 15] ^ t1[(c >> 4 + b) & 15];
#endif
#ifndef SH_EXPERIMENT_NO_ACC
#pragma unroll
                for (int b = 0; b < 8; ++b) acc[j][b] ^= tmp[b];
#else
                if (j == 0)
                    for (int b = 0; b < 8; ++b) acc[0][b] ^= tmp[b];
#endif
            }
        }
#pragma unroll
        for (int s = 0; s < 8; ++s) d[s] = dn[s];
        cv = cvn;
    }

    if (lane >= ncols) return;
    const uint32_t col = colx_off(c0 + lane, geo.nq, geo.sub);
    uint8_t *out = a.out + static_cast<long long>(g) * a.out_gstride + col;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (j0 + j >= e) break;
        uint8_t *row = out + static_cast<long long>(j0 + j) * geo.B;
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const uint32_t w = acc[j][b];
            __builtin_memcpy(row + b * geo.sub, &w, 4);
        }
    }
}

#ifdef SH_EXPERIMENT_INLINE_SNIP  // timing experiment: fixed inline snippet, no branches
#define SH_CALLX(G) "v_bitop3_b32 v64, v64, v129, v146 bitop3:0x96\n""v_bitop3_b32 v65, v65, v132, v151 bitop3:0x96\n""v_bitop3_b32 v66, v66, v135, v156 bitop3:0x96\n""v_bitop3_b32 v67, v67, v138, v145 bitop3:0x96\n""v_bitop3_b32 v68, v68, v141, v150 bitop3:0x96\n""v_bitop3_b32 v69, v69, v128, v155 bitop3:0x96\n""v_bitop3_b32 v70, v70, v131, v144 bitop3:0x96\n""v_bitop3_b32 v71, v71, v134, v149 bitop3:0x96\n"
#else
#define SH_CALLX(G) "s_swappc_b64 s[40:41], %[" #G "]\n"
#endif
#ifdef SH_EXPERIMENT_NO_ROWS  // timing experiment: wrong results, no per-row compute
#define SH_ROWS_ON false
#else
#define SH_ROWS_ON true
#endif
#ifdef SH_EXPERIMENT_NO_GPRIDX  // timing experiment: wrong results, no VGPR-index mode
#define SH_GI_ON ""
#define SH_GI_IDX(n) ""
#define SH_GI_OFF ""
#else
#define SH_GI_ON "s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)\n"
#define SH_GI_IDX(n) "s_set_gpr_idx_idx " n "\n"
#define SH_GI_OFF "s_set_gpr_idx_off"
#endif
#ifdef SH_EXPERIMENT_STAMPS
#define SH_BSTAMP(i)                                                                               \
    do {                                                                                           \
        unsigned long long t_;                                                                     \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");               \
        st_[i] = t_;                                                                               \
    } while (0)
#else
#define SH_BSTAMP(i)
#endif

__global__ __launch_bounds__(256, 3) void stageb_acc(StageBArgs a) {
    SH_SNIPA_TABLE(A);
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const Geometry geo = a.geo;
    const int ncc = (geo.nq + 63) / 64;
    const int g = blockIdx.x / ncc;
    const int cc = blockIdx.x - g * ncc;
    const int c0 = cc * 64;
    const int ncols = min(64, geo.nq - c0);
    const int nch = ncols / 4;        // 16-byte chunks per (row, sub-block)
    const int cpb = nch * 16;         // LDS bytes per (row, sub-block)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
#ifdef SH_EXPERIMENT_STAMPS
    unsigned long long st_[6];
#endif
    SH_BSTAMP(0);
    const int e = a.e[g];
#ifdef SH_EXPERIMENT_STAMPS
    asm volatile("" ::"s"(e));
#endif
    SH_BSTAMP(1);
    const int j0 = (blockIdx.y * 4 + wave) * 8;

    // ---- gather the residual tile into LDS: chunk ch = (y*8 + a)*nch + t; then the group's
    // stage-B coefficients (n_in x ldT bytes) behind it
    const int total = a.n_in * 8 * nch;
    const int tile = ((total + 255) / 256) * 256 * 16;
    uint8_t *lcoef = lds + tile;
    {
        const long long gbase = static_cast<long long>(g) * a.in_gstride;
        long long avail = static_cast<long long>(a.groups) * a.in_gstride + a.in_slack - gbase;
        if (avail > 0x7FFFFFFFll) avail = 0x7FFFFFFFll;
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t *>(a.in + gbase), static_cast<short>(0), static_cast<int>(avail), 0x00020000);
        for (int base = wave * 64; base < total; base += 256) {  // uniform
            const int ch = base + lane;
            uint32_t off = 0x80000000u;
            if (ch < total) {
                const int ya = ch / nch, t = ch - ya * nch;
                const int y = ya >> 3, sa = ya & 7;
                off = static_cast<uint32_t>(y) * geo.B + static_cast<uint32_t>(sa) * geo.sub +
                      colx_off(c0 + 4 * t, geo.nq, geo.sub);
            }
            __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t *)(lds + base * 16), 16, off, 0, 0, 0);
        }
        const int cbytes = a.n_in * a.ldT;  // multiple of 8; <= 32 * 32
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t *>(a.coefT + static_cast<long long>(g) * a.coefT_gstride), static_cast<short>(0),
            cbytes, 0x00020000);
        for (int base = wave * 64; base * 16 < cbytes; base += 256)  // uniform
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rc, (lds_void_t *)(lcoef + base * 16), 16, (base + lane) * 16, 0, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    if (j0 >= e) return;  // wave-uniform (after the barrier)
    SH_BSTAMP(2);

    uint64_t snip;
    asm volatile(
        "s_getpc_b64 s[42:43]\n"
        "s_add_u32 s42, s42, sh_snipa_baseA@rel32@lo+4\n"
        "s_addc_u32 s43, s43, sh_snipa_baseA@rel32@hi+12\n"
        "s_mov_b64 %0, s[42:43]"
        : "=s"(snip)
        :
        : "s42", "s43", "scc");

    const uint8_t *rd = lds + 4 * lane;
    const uint8_t *cf = lcoef + j0;

    // accumulators pinned to v[32:95] (output j at v[32+8j..]), window tables to v[96:127]
    u32x16 a01, a23, a45, a67;
#pragma unroll
    for (int i = 0; i < 16; ++i) a01[i] = a23[i] = a45[i] = a67[i] = 0;

    // rows and coefficients are prefetched one input row ahead (LDS latency under the calls)
    uint32_t d[8], dn[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) d[s] = *reinterpret_cast<const uint32_t *>(rd + s * cpb);
    uint2 cv = *reinterpret_cast<const uint2 *>(cf);
    for (int y = 0; y < a.n_in; ++y) {
        const int yn = y + 1 < a.n_in ? y + 1 : y;
#pragma unroll
        for (int s = 0; s < 8; ++s) dn[s] = *reinterpret_cast<const uint32_t *>(rd + (yn * 8 + s) * cpb);
        const uint2 cvn = *reinterpret_cast<const uint2 *>(cf + yn * a.ldT);
        const uint32_t clo = __builtin_amdgcn_readfirstlane(cv.x), chi = __builtin_amdgcn_readfirstlane(cv.y);
        if (SH_ROWS_ON && (clo | chi) != 0) {  // wave-uniform: no output of this wave uses input y otherwise
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
            uint64_t tg[8];
#pragma unroll
            for (int j = 0; j < 8; ++j)
                tg[j] = snip + (static_cast<uint64_t>(((j < 4 ? clo : chi) >> (8 * (j & 3))) & 0xffu) << 7);
            // One asm block: VGPR-index mode must not see any compiler VALU between on and off.
            asm volatile(
                SH_GI_ON
                SH_CALLX(g0)
                SH_GI_IDX("8")
                SH_CALLX(g1)
                SH_GI_IDX("16")
                SH_CALLX(g2)
                SH_GI_IDX("24")
                SH_CALLX(g3)
                SH_GI_IDX("32")
                SH_CALLX(g4)
                SH_GI_IDX("40")
                SH_CALLX(g5)
                SH_GI_IDX("48")
                SH_CALLX(g6)
                SH_GI_IDX("56")
                SH_CALLX(g7)
                SH_GI_OFF
                : "+{v[32:47]}"(a01), "+{v[48:63]}"(a23), "+{v[64:79]}"(a45), "+{v[80:95]}"(a67)
                : "{v[96:111]}"(t0), "{v[112:127]}"(t1), [g0] "s"(tg[0]), [g1] "s"(tg[1]),
                  [g2] "s"(tg[2]), [g3] "s"(tg[3]), [g4] "s"(tg[4]), [g5] "s"(tg[5]), [g6] "s"(tg[6]),
                  [g7] "s"(tg[7])
                : "s40", "s41", "m0", "memory");
        }
#pragma unroll
        for (int s = 0; s < 8; ++s) d[s] = dn[s];
        cv = cvn;
    }
    SH_BSTAMP(3);
    uint32_t acc[8][8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        acc[0][b] = a01[b]; acc[1][b] = a01[8 + b];
        acc[2][b] = a23[b]; acc[3][b] = a23[8 + b];
        acc[4][b] = a45[b]; acc[5][b] = a45[8 + b];
        acc[6][b] = a67[b]; acc[7][b] = a67[8 + b];
    }

    if (lane < ncols) {
    const uint32_t col = colx_off(c0 + lane, geo.nq, geo.sub);
    uint8_t *out = a.out + static_cast<long long>(g) * a.out_gstride + col;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (j0 + j >= e) break;
        uint8_t *row = out + static_cast<long long>(j0 + j) * geo.B;
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const uint32_t w = acc[j][b];
            __builtin_memcpy(row + b * geo.sub, &w, 4);
        }
    }    }
#ifdef SH_EXPERIMENT_STAMPS
    SH_BSTAMP(4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    SH_BSTAMP(5);
    if (lane == 0 && a.dbg) {
        unsigned long long *d = a.dbg + ((static_cast<size_t>(blockIdx.y) * gridDim.x + blockIdx.x) * 4 + wave) * 8;
        for (int t = 0; t < 6; ++t) d[t] = st_[t];
    }
#endif
}

bool stageb_lds_ok(const StageBArgs &a) {
    return a.n_in <= 32 && a.ldT <= 32 && a.geo.nq % 4 == 0 && a.geo.sub >= 16;
}

hipError_t launch_stageb(const StageBArgs &a, int emax, hipStream_t stream) {
    if (a.groups <= 0 || emax <= 0) return hipSuccess;
    if (stageb_lds_ok(a)) {
        const int ncc = (a.geo.nq + 63) / 64;
        const int nch = std::min(64, a.geo.nq) / 4;
        // tile bytes rounded up to whole 4-wave DMA rounds (out-of-range lanes still write LDS)
        const size_t chunks = static_cast<size_t>(a.n_in) * 8 * nch;
        const size_t cbytes = static_cast<size_t>(a.n_in) * a.ldT;  // coefficients behind the tile
        const size_t lds = ((chunks + 255) / 256) * 256 * 16 + ((cbytes + 4095) / 4096) * 4096;
        dim3 grid(static_cast<unsigned>(ncc) * a.groups, (emax + 31) / 32, 1);
        if (std::getenv("SH_STAGEB_SNIP"))  // A/B switch: the copy-and-XOR snippet kernel
            hipLaunchKernelGGL(stageb_lds, grid, dim3(256), lds, stream, a);
        else
            hipLaunchKernelGGL(stageb_acc, grid, dim3(256), lds, stream, a);
        return hipGetLastError();
    }
    dim3 grid(static_cast<unsigned>((a.geo.nq + 63) / 64) * a.groups, (emax + 31) / 32, 1);
    hipLaunchKernelGGL(stageb_snip, grid, dim3(256), 0, stream, a);
    return hipGetLastError();
}

}  // namespace sh
