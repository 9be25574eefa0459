// Microbenchmark for decode stage B's runtime-coefficient products (not part of the product).
//
// Each wave runs ROWS input rows; per row it builds the two window tables (22 XORs) and applies
// 8 coefficients to 8 accumulator sets, in one of these forms:
//   call   s_swappc into the accumulating snippet of the coefficient (VGPR-index mode), as
//          stageb_fixed does (2 redirects per product)
//   inline the same 8 bitop3 per product inline for a fixed coefficient (no redirect): the floor
//   call4  as call, 4 outputs per wave (accumulators v[32:63], tables v[64:95]: 5 waves/SIMD,
//          twice the table builds per product); run with twice the workgroups for equal work
//   chain1 one redirect per product: each snippet advances the index (m0 += 8), shifts the queue of
//          snippet addresses s[44:61] down one pair and jumps to the next (SNIPC table)
//   index  no redirect: per output bit two v_xor_b32 whose SRC0 is VGPR-indexed into the tables
//          (s_set_gpr_idx_idx per lookup, indices packed 4 per SGPR as lo, 16+hi)
//   chain  threaded dispatch: the caller jumps into the first snippet; every snippet returns to a
//          per-position trampoline that selects the next accumulator set and jumps on
//          (still 2 redirects, measured against "call" for the trampoline cost)
// Launch: NWG workgroups of 256 threads, LDS bytes per workgroup as given (occupancy control).
//   snip_bench MODE NWG LDS ROWS
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "snippets.h"

typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));

#define TABLES                                                                                    \
    "v_xor_b32 v99, v97, v98\n"                                                                   \
    "v_xor_b32 v115, v113, v114\n"                                                                \
    "v_xor_b32 v101, v97, v100\n"                                                                 \
    "v_xor_b32 v117, v113, v116\n"                                                                \
    "v_xor_b32 v102, v98, v100\n"                                                                 \
    "v_xor_b32 v118, v114, v116\n"                                                                \
    "v_xor_b32 v105, v97, v104\n"                                                                 \
    "v_xor_b32 v121, v113, v120\n"                                                                \
    "v_xor_b32 v106, v98, v104\n"                                                                 \
    "v_xor_b32 v122, v114, v120\n"                                                                \
    "v_xor_b32 v108, v100, v104\n"                                                                \
    "v_xor_b32 v124, v116, v120\n"                                                                \
    "v_xor_b32 v103, v99, v100\n"                                                                 \
    "v_xor_b32 v119, v115, v116\n"                                                                \
    "v_xor_b32 v107, v99, v104\n"                                                                 \
    "v_xor_b32 v123, v115, v120\n"                                                                \
    "v_xor_b32 v109, v101, v104\n"                                                                \
    "v_xor_b32 v125, v117, v120\n"                                                                \
    "v_xor_b32 v110, v102, v104\n"                                                                \
    "v_xor_b32 v126, v118, v120\n"                                                                \
    "v_xor_b32 v111, v103, v104\n"                                                                \
    "v_xor_b32 v127, v119, v120\n"

#define CLOBBERS                                                                                  \
    "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108",  \
        "v109", "v110", "v111", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120",   \
        "v121", "v122", "v123", "v124", "v125", "v126", "v127", "s40", "s41", "m0", "memory"

__global__ void snip_table_holder_b(uint64_t *out) {
    SH_SNIPB_TABLE(U);
    uint64_t base;
    asm volatile(
        "s_getpc_b64 s[42:43]\n"
        "s_add_u32 s42, s42, sh_snipb_baseU@rel32@lo+4\n"
        "s_addc_u32 s43, s43, sh_snipb_baseU@rel32@hi+12\n"
        "s_mov_b64 %0, s[42:43]"
        : "=s"(base)
        :
        : "s42", "s43", "scc");
    if (threadIdx.x == 0) *out = base;
}

__global__ void snip_table_holder_c(uint64_t *out) {
    SH_SNIPC_TABLE(V);
    uint64_t base;
    asm volatile(
        "s_getpc_b64 s[42:43]\n"
        "s_add_u32 s42, s42, sh_snipc_baseV@rel32@lo+4\n"
        "s_addc_u32 s43, s43, sh_snipc_baseV@rel32@hi+12\n"
        "s_mov_b64 %0, s[42:43]"
        : "=s"(base)
        :
        : "s42", "s43", "scc");
    if (threadIdx.x == 0) *out = base;
}

__global__ void snip_table_holder(uint64_t *out) {
    SH_SNIPA_TABLE(T);
    uint64_t base;
    asm volatile(
        "s_getpc_b64 s[42:43]\n"
        "s_add_u32 s42, s42, sh_snipa_baseT@rel32@lo+4\n"
        "s_addc_u32 s43, s43, sh_snipa_baseT@rel32@hi+12\n"
        "s_mov_b64 %0, s[42:43]"
        : "=s"(base)
        :
        : "s42", "s43", "scc");
    if (threadIdx.x == 0) *out = base;
}

// MODE 2: one index dword D holds the 4 lookups of bits (b, b+1) as bytes lo, 16+hi, lo, 16+hi;
// each lookup is s_set_gpr_idx_idx + one v_xor_b32 whose SRC0 (v96 = table base) is indexed.
#define IX_DW(D, A, B)                                                                            \
    "s_set_gpr_idx_idx %[" D "]\n v_xor_b32 v" A ", v96, v" A "\n"                                \
    "s_lshr_b32 s90, %[" D "], 8\n s_set_gpr_idx_idx s90\n v_xor_b32 v" A ", v96, v" A "\n"      \
    "s_lshr_b32 s90, %[" D "], 16\n s_set_gpr_idx_idx s90\n v_xor_b32 v" B ", v96, v" B "\n"     \
    "s_lshr_b32 s90, %[" D "], 24\n s_set_gpr_idx_idx s90\n v_xor_b32 v" B ", v96, v" B "\n"
#define IX_OUT(J, A0, A1, A2, A3, A4, A5, A6, A7)                                                 \
    IX_DW("x" #J "a", A0, A1) IX_DW("x" #J "b", A2, A3) IX_DW("x" #J "c", A4, A5) IX_DW("x" #J "d", A6, A7)

// window tables for MODE 3 (SNIPB registers: T0 = v64.., T1 = v80..)
#define TABLES_B \
    "v_xor_b32 v67, v65, v66\n" \
    "v_xor_b32 v83, v81, v82\n" \
    "v_xor_b32 v69, v65, v68\n" \
    "v_xor_b32 v85, v81, v84\n" \
    "v_xor_b32 v70, v66, v68\n" \
    "v_xor_b32 v86, v82, v84\n" \
    "v_xor_b32 v73, v65, v72\n" \
    "v_xor_b32 v89, v81, v88\n" \
    "v_xor_b32 v74, v66, v72\n" \
    "v_xor_b32 v90, v82, v88\n" \
    "v_xor_b32 v76, v68, v72\n" \
    "v_xor_b32 v92, v84, v88\n" \
    "v_xor_b32 v71, v67, v68\n" \
    "v_xor_b32 v87, v83, v84\n" \
    "v_xor_b32 v75, v67, v72\n" \
    "v_xor_b32 v91, v83, v88\n" \
    "v_xor_b32 v77, v69, v72\n" \
    "v_xor_b32 v93, v85, v88\n" \
    "v_xor_b32 v78, v70, v72\n" \
    "v_xor_b32 v94, v86, v88\n" \
    "v_xor_b32 v79, v71, v72\n" \
    "v_xor_b32 v95, v87, v88\n"

template <int MODE>
__global__ __launch_bounds__(256, MODE == 3 ? 5 : 1) void bench(const uint64_t *targets, uint32_t *sink, int rows,
                                                               uint64_t tbase, uint64_t tbaseb, uint64_t tbasec) {
    extern __shared__ uint8_t lds[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (lane == 0) lds[wave] = 0;
    u32x16 a01, a23, a45, a67;
    for (int i = 0; i < 16; ++i) a01[i] = a23[i] = a45[i] = a67[i] = lane * 7 + i;
    uint32_t z0 = 0, z1 = 0;
    uint32_t d0 = lane, d1 = lane * 3, d2 = lane * 5, d3 = lane * 9, d4 = lane * 11, d5 = lane * 13,
             d6 = lane * 17, d7 = lane * 19;
    typedef const __attribute__((address_space(4))) uint64_t cu64_t;
    const cu64_t *tp = (const cu64_t *)targets;
    typedef const __attribute__((address_space(4))) uint32_t cu32_t;
    const cu32_t *ip = (const cu32_t *)(targets + 64 * 8);
    for (int r = 0; r < rows; ++r) {
        uint64_t tg[8];
        for (int j = 0; j < 8; ++j) tg[j] = tp[((r + blockIdx.x + wave) & 63) * 8 + j];
        uint64_t tgb[4], tgc[8];
        for (int j = 0; j < 4; ++j) tgb[j] = tg[j] - tbase + tbaseb;  // same snippet, SNIPB table
        for (int j = 0; j < 8; ++j) tgc[j] = tbasec + (tg[j] - tbase) / SH_SNIPA_STRIDE * SH_SNIPC_STRIDE;
        if (MODE == 0) {
            asm volatile(
                "v_mov_b32 v97, %[d0]\n v_mov_b32 v98, %[d1]\n v_mov_b32 v100, %[d2]\n v_mov_b32 v104, %[d3]\n"
                "v_mov_b32 v113, %[d4]\n v_mov_b32 v114, %[d5]\n v_mov_b32 v116, %[d6]\n v_mov_b32 v120, %[d7]\n"
                TABLES
                "s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)\n"
                "s_swappc_b64 s[40:41], %[g0]\n"
                "s_set_gpr_idx_idx 8\n"
                "s_swappc_b64 s[40:41], %[g1]\n"
                "s_set_gpr_idx_idx 16\n"
                "s_swappc_b64 s[40:41], %[g2]\n"
                "s_set_gpr_idx_idx 24\n"
                "s_swappc_b64 s[40:41], %[g3]\n"
                "s_set_gpr_idx_idx 32\n"
                "s_swappc_b64 s[40:41], %[g4]\n"
                "s_set_gpr_idx_idx 40\n"
                "s_swappc_b64 s[40:41], %[g5]\n"
                "s_set_gpr_idx_idx 48\n"
                "s_swappc_b64 s[40:41], %[g6]\n"
                "s_set_gpr_idx_idx 56\n"
                "s_swappc_b64 s[40:41], %[g7]\n"
                "s_set_gpr_idx_off"
                : "+{v[32:47]}"(a01), "+{v[48:63]}"(a23), "+{v[64:79]}"(a45), "+{v[80:95]}"(a67),
                  "+{v96}"(z0), "+{v112}"(z1)
                : [d0] "v"(d0), [d1] "v"(d1), [d2] "v"(d2), [d3] "v"(d3), [d4] "v"(d4), [d5] "v"(d5),
                  [d6] "v"(d6), [d7] "v"(d7), [g0] "s"(tg[0]), [g1] "s"(tg[1]), [g2] "s"(tg[2]),
                  [g3] "s"(tg[3]), [g4] "s"(tg[4]), [g5] "s"(tg[5]), [g6] "s"(tg[6]), [g7] "s"(tg[7])
                : CLOBBERS);
        } else if (MODE == 1) {
            asm volatile(
                "v_mov_b32 v97, %[d0]\n v_mov_b32 v98, %[d1]\n v_mov_b32 v100, %[d2]\n v_mov_b32 v104, %[d3]\n"
                "v_mov_b32 v113, %[d4]\n v_mov_b32 v114, %[d5]\n v_mov_b32 v116, %[d6]\n v_mov_b32 v120, %[d7]\n"
                TABLES
                "v_bitop3_b32 v32, v32, v101, v119 bitop3:0x96\n"
                "v_bitop3_b32 v33, v33, v103, v114 bitop3:0x96\n"
                "v_bitop3_b32 v34, v34, v107, v125 bitop3:0x96\n"
                "v_bitop3_b32 v35, v35, v109, v117 bitop3:0x96\n"
                "v_bitop3_b32 v36, v36, v98, v127 bitop3:0x96\n"
                "v_bitop3_b32 v37, v37, v111, v120 bitop3:0x96\n"
                "v_bitop3_b32 v38, v38, v102, v122 bitop3:0x96\n"
                "v_bitop3_b32 v39, v39, v105, v116 bitop3:0x96\n"
                "v_bitop3_b32 v40, v40, v103, v114 bitop3:0x96\n"
                "v_bitop3_b32 v41, v41, v107, v125 bitop3:0x96\n"
                "v_bitop3_b32 v42, v42, v109, v117 bitop3:0x96\n"
                "v_bitop3_b32 v43, v43, v98, v127 bitop3:0x96\n"
                "v_bitop3_b32 v44, v44, v111, v120 bitop3:0x96\n"
                "v_bitop3_b32 v45, v45, v102, v122 bitop3:0x96\n"
                "v_bitop3_b32 v46, v46, v105, v116 bitop3:0x96\n"
                "v_bitop3_b32 v47, v47, v101, v119 bitop3:0x96\n"
                "v_bitop3_b32 v48, v48, v107, v125 bitop3:0x96\n"
                "v_bitop3_b32 v49, v49, v109, v117 bitop3:0x96\n"
                "v_bitop3_b32 v50, v50, v98, v127 bitop3:0x96\n"
                "v_bitop3_b32 v51, v51, v111, v120 bitop3:0x96\n"
                "v_bitop3_b32 v52, v52, v102, v122 bitop3:0x96\n"
                "v_bitop3_b32 v53, v53, v105, v116 bitop3:0x96\n"
                "v_bitop3_b32 v54, v54, v101, v119 bitop3:0x96\n"
                "v_bitop3_b32 v55, v55, v103, v114 bitop3:0x96\n"
                "v_bitop3_b32 v56, v56, v109, v117 bitop3:0x96\n"
                "v_bitop3_b32 v57, v57, v98, v127 bitop3:0x96\n"
                "v_bitop3_b32 v58, v58, v111, v120 bitop3:0x96\n"
                "v_bitop3_b32 v59, v59, v102, v122 bitop3:0x96\n"
                "v_bitop3_b32 v60, v60, v105, v116 bitop3:0x96\n"
                "v_bitop3_b32 v61, v61, v101, v119 bitop3:0x96\n"
                "v_bitop3_b32 v62, v62, v103, v114 bitop3:0x96\n"
                "v_bitop3_b32 v63, v63, v107, v125 bitop3:0x96\n"
                "v_bitop3_b32 v64, v64, v98, v127 bitop3:0x96\n"
                "v_bitop3_b32 v65, v65, v111, v120 bitop3:0x96\n"
                "v_bitop3_b32 v66, v66, v102, v122 bitop3:0x96\n"
                "v_bitop3_b32 v67, v67, v105, v116 bitop3:0x96\n"
                "v_bitop3_b32 v68, v68, v101, v119 bitop3:0x96\n"
                "v_bitop3_b32 v69, v69, v103, v114 bitop3:0x96\n"
                "v_bitop3_b32 v70, v70, v107, v125 bitop3:0x96\n"
                "v_bitop3_b32 v71, v71, v109, v117 bitop3:0x96\n"
                "v_bitop3_b32 v72, v72, v111, v120 bitop3:0x96\n"
                "v_bitop3_b32 v73, v73, v102, v122 bitop3:0x96\n"
                "v_bitop3_b32 v74, v74, v105, v116 bitop3:0x96\n"
                "v_bitop3_b32 v75, v75, v101, v119 bitop3:0x96\n"
                "v_bitop3_b32 v76, v76, v103, v114 bitop3:0x96\n"
                "v_bitop3_b32 v77, v77, v107, v125 bitop3:0x96\n"
                "v_bitop3_b32 v78, v78, v109, v117 bitop3:0x96\n"
                "v_bitop3_b32 v79, v79, v98, v127 bitop3:0x96\n"
                "v_bitop3_b32 v80, v80, v102, v122 bitop3:0x96\n"
                "v_bitop3_b32 v81, v81, v105, v116 bitop3:0x96\n"
                "v_bitop3_b32 v82, v82, v101, v119 bitop3:0x96\n"
                "v_bitop3_b32 v83, v83, v103, v114 bitop3:0x96\n"
                "v_bitop3_b32 v84, v84, v107, v125 bitop3:0x96\n"
                "v_bitop3_b32 v85, v85, v109, v117 bitop3:0x96\n"
                "v_bitop3_b32 v86, v86, v98, v127 bitop3:0x96\n"
                "v_bitop3_b32 v87, v87, v111, v120 bitop3:0x96\n"
                "v_bitop3_b32 v88, v88, v105, v116 bitop3:0x96\n"
                "v_bitop3_b32 v89, v89, v101, v119 bitop3:0x96\n"
                "v_bitop3_b32 v90, v90, v103, v114 bitop3:0x96\n"
                "v_bitop3_b32 v91, v91, v107, v125 bitop3:0x96\n"
                "v_bitop3_b32 v92, v92, v109, v117 bitop3:0x96\n"
                "v_bitop3_b32 v93, v93, v98, v127 bitop3:0x96\n"
                "v_bitop3_b32 v94, v94, v111, v120 bitop3:0x96\n"
                "v_bitop3_b32 v95, v95, v102, v122 bitop3:0x96\n"
                : "+{v[32:47]}"(a01), "+{v[48:63]}"(a23), "+{v[64:79]}"(a45), "+{v[80:95]}"(a67),
                  "+{v96}"(z0), "+{v112}"(z1)
                : [d0] "v"(d0), [d1] "v"(d1), [d2] "v"(d2), [d3] "v"(d3), [d4] "v"(d4), [d5] "v"(d5),
                  [d6] "v"(d6), [d7] "v"(d7), "s"(tg[0]), "s"(tg[1]), "s"(tg[2]), "s"(tg[3]), "s"(tg[4]),
                  "s"(tg[5]), "s"(tg[6]), "s"(tg[7])
                : CLOBBERS);
        } else if (MODE == 4) {  // chained snippets (SNIPC): one redirect per product
            uint64_t c0 = tgc[0], c1 = tgc[1], c2 = tgc[2], c3 = tgc[3], c4 = tgc[4], c5 = tgc[5], c6 = tgc[6],
                     c7 = tgc[7], rr;
            asm volatile(
                "v_mov_b32 v97, %[d0]\n v_mov_b32 v98, %[d1]\n v_mov_b32 v100, %[d2]\n v_mov_b32 v104, %[d3]\n"
                "v_mov_b32 v113, %[d4]\n v_mov_b32 v114, %[d5]\n v_mov_b32 v116, %[d6]\n v_mov_b32 v120, %[d7]\n"
                TABLES
                "s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)\n"
                "s_swappc_b64 s[60:61], s[44:45]\n"
                "s_set_gpr_idx_off"
                : "+{v[32:47]}"(a01), "+{v[48:63]}"(a23), "+{v[64:79]}"(a45), "+{v[80:95]}"(a67),
                  "+{v96}"(z0), "+{v112}"(z1), "+{s[44:45]}"(c0), "+{s[46:47]}"(c1), "+{s[48:49]}"(c2),
                  "+{s[50:51]}"(c3), "+{s[52:53]}"(c4), "+{s[54:55]}"(c5), "+{s[56:57]}"(c6), "+{s[58:59]}"(c7),
                  "={s[60:61]}"(rr)
                : [d0] "v"(d0), [d1] "v"(d1), [d2] "v"(d2), [d3] "v"(d3), [d4] "v"(d4), [d5] "v"(d5),
                  [d6] "v"(d6), [d7] "v"(d7)
                : CLOBBERS, "scc");
        } else if (MODE == 3) {  // 4 outputs per wave, SNIPB registers (v[32:95]: 5 waves/SIMD)
            asm volatile(
                "v_mov_b32 v65, %[d0]\n v_mov_b32 v66, %[d1]\n v_mov_b32 v68, %[d2]\n v_mov_b32 v72, %[d3]\n"
                "v_mov_b32 v81, %[d4]\n v_mov_b32 v82, %[d5]\n v_mov_b32 v84, %[d6]\n v_mov_b32 v88, %[d7]\n"
                TABLES_B
                "s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)\n"
                "s_swappc_b64 s[40:41], %[g0]\n"
                "s_set_gpr_idx_idx 8\n"
                "s_swappc_b64 s[40:41], %[g1]\n"
                "s_set_gpr_idx_idx 16\n"
                "s_swappc_b64 s[40:41], %[g2]\n"
                "s_set_gpr_idx_idx 24\n"
                "s_swappc_b64 s[40:41], %[g3]\n"
                "s_set_gpr_idx_off"
                : "+{v[32:47]}"(a01), "+{v[48:63]}"(a23), "+{v64}"(z0), "+{v80}"(z1)
                : [d0] "v"(d0), [d1] "v"(d1), [d2] "v"(d2), [d3] "v"(d3), [d4] "v"(d4), [d5] "v"(d5),
                  [d6] "v"(d6), [d7] "v"(d7), [g0] "s"(tgb[0]), [g1] "s"(tgb[1]), [g2] "s"(tgb[2]), [g3] "s"(tgb[3])
                : "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77",
                  "v78", "v79", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91",
                  "v92", "v93", "v94", "v95", "s40", "s41", "m0", "memory");
        } else if (MODE == 2) {
            uint32_t ix[32];
            for (int j = 0; j < 32; ++j) ix[j] = ip[((r + blockIdx.x + wave) & 63) * 32 + j];
            asm volatile(
                "v_mov_b32 v97, %[d0]\n v_mov_b32 v98, %[d1]\n v_mov_b32 v100, %[d2]\n v_mov_b32 v104, %[d3]\n"
                "v_mov_b32 v113, %[d4]\n v_mov_b32 v114, %[d5]\n v_mov_b32 v116, %[d6]\n v_mov_b32 v120, %[d7]\n"
                TABLES
                "s_set_gpr_idx_on 0, gpr_idx(SRC0)\n"
                IX_OUT(0, "32", "33", "34", "35", "36", "37", "38", "39")
                IX_OUT(1, "40", "41", "42", "43", "44", "45", "46", "47")
                IX_OUT(2, "48", "49", "50", "51", "52", "53", "54", "55")
                IX_OUT(3, "56", "57", "58", "59", "60", "61", "62", "63")
                IX_OUT(4, "64", "65", "66", "67", "68", "69", "70", "71")
                IX_OUT(5, "72", "73", "74", "75", "76", "77", "78", "79")
                IX_OUT(6, "80", "81", "82", "83", "84", "85", "86", "87")
                IX_OUT(7, "88", "89", "90", "91", "92", "93", "94", "95")
                "s_set_gpr_idx_off"
                : "+{v[32:47]}"(a01), "+{v[48:63]}"(a23), "+{v[64:79]}"(a45), "+{v[80:95]}"(a67),
                  "+{v96}"(z0), "+{v112}"(z1)
                : [d0] "v"(d0), [d1] "v"(d1), [d2] "v"(d2), [d3] "v"(d3), [d4] "v"(d4), [d5] "v"(d5),
                  [d6] "v"(d6), [d7] "v"(d7), [x0a] "s"(ix[0]), [x0b] "s"(ix[1]), [x0c] "s"(ix[2]), [x0d] "s"(ix[3]), [x1a] "s"(ix[4]), [x1b] "s"(ix[5]), [x1c] "s"(ix[6]), [x1d] "s"(ix[7]), [x2a] "s"(ix[8]), [x2b] "s"(ix[9]), [x2c] "s"(ix[10]), [x2d] "s"(ix[11]), [x3a] "s"(ix[12]), [x3b] "s"(ix[13]), [x3c] "s"(ix[14]), [x3d] "s"(ix[15]), [x4a] "s"(ix[16]), [x4b] "s"(ix[17]), [x4c] "s"(ix[18]), [x4d] "s"(ix[19]), [x5a] "s"(ix[20]), [x5b] "s"(ix[21]), [x5c] "s"(ix[22]), [x5d] "s"(ix[23]), [x6a] "s"(ix[24]), [x6b] "s"(ix[25]), [x6c] "s"(ix[26]), [x6d] "s"(ix[27]), [x7a] "s"(ix[28]), [x7b] "s"(ix[29]), [x7c] "s"(ix[30]), [x7d] "s"(ix[31])
                : CLOBBERS, "s90", "scc");
        }
        d0 += a01[r & 15];
    }
    uint32_t x = d0;
    for (int i = 0; i < 16; ++i) x ^= a01[i] ^ a23[i] ^ a45[i] ^ a67[i];
    if (x == 0x12345678u) sink[blockIdx.x * 256 + threadIdx.x] = x;
}

int main(int argc, char **argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    const int nwg = argc > 2 ? atoi(argv[2]) : 8192;
    const int ldsb = argc > 3 ? atoi(argv[3]) : 0;
    const int rows = argc > 4 ? atoi(argv[4]) : 32;
    uint64_t *d_base, base;
    hipMalloc(&d_base, 8);
    hipLaunchKernelGGL(snip_table_holder, dim3(1), dim3(64), 0, 0, d_base);
    hipMemcpy(&base, d_base, 8, hipMemcpyDeviceToHost);
    uint64_t baseb;
    hipLaunchKernelGGL(snip_table_holder_b, dim3(1), dim3(64), 0, 0, d_base);
    hipMemcpy(&baseb, d_base, 8, hipMemcpyDeviceToHost);
    uint64_t basec;
    hipLaunchKernelGGL(snip_table_holder_c, dim3(1), dim3(64), 0, 0, d_base);
    hipMemcpy(&basec, d_base, 8, hipMemcpyDeviceToHost);
    uint64_t h[64 * 8 + 64 * 16];  // snippet targets, then MODE 2 index dwords (64 rows x 32)
    srand(7);
    for (int i = 0; i < 64 * 8; ++i) h[i] = base + (uint64_t)(1 + rand() % 255) * SH_SNIPA_STRIDE;
    uint32_t *ixs = (uint32_t *)(h + 64 * 8);
    for (int i = 0; i < 64 * 32; ++i)  // bytes: lo, 16 + hi, lo, 16 + hi
        ixs[i] = (rand() & 15) | ((16 + (rand() & 15)) << 8) | ((rand() & 15) << 16) | ((16 + (rand() & 15)) << 24);
    uint64_t *d_t;
    uint32_t *d_sink;
    hipMalloc(&d_t, sizeof h);
    hipMemcpy(d_t, h, sizeof h, hipMemcpyHostToDevice);
    hipMalloc(&d_sink, (size_t)nwg * 256 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto go = [&]() {
        if (mode == 0) hipLaunchKernelGGL(bench<0>, dim3(nwg), dim3(256), ldsb, 0, d_t, d_sink, rows, base, baseb, basec);
        else if (mode == 1) hipLaunchKernelGGL(bench<1>, dim3(nwg), dim3(256), ldsb, 0, d_t, d_sink, rows, base, baseb, basec);
        else if (mode == 2) hipLaunchKernelGGL(bench<2>, dim3(nwg), dim3(256), ldsb, 0, d_t, d_sink, rows, base, baseb, basec);
        else if (mode == 3) hipLaunchKernelGGL(bench<3>, dim3(nwg), dim3(256), ldsb, 0, d_t, d_sink, rows, base, baseb, basec);
        else hipLaunchKernelGGL(bench<4>, dim3(nwg), dim3(256), ldsb, 0, d_t, d_sink, rows, base, baseb, basec);
    };
    go();
    hipDeviceSynchronize();
    hipEventRecord(e0, 0);
    const int it = 10;
    for (int i = 0; i < it; ++i) go();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= it;
    const double products = (double)nwg * 4 * rows * (mode == 3 ? 4 : 8);  // per-wave outputs
    printf("mode=%s nwg=%d lds=%d rows=%d: %.4f ms, %.2f G wave-products/s, %.1f ns per wave-product per CU\n",
           mode == 0 ? "call" : mode == 1 ? "inline" : mode == 2 ? "index" : mode == 3 ? "call4" : "chain1", nwg, ldsb, rows, ms, products / ms / 1e6, ms * 1e6 * 256 / products);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) printf("error %s\n", hipGetErrorString(err));
    return 0;
}
