// Device-side argument blocks and launch entry points (kernels.hip). Host code only sees plain
// pointers and sizes; no torch types anywhere in the library.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "geometry.hpp"

namespace sh {

struct ApplyArgs {
    const uint8_t *in;
    long long in_gstride;   // bytes between groups
    long long in_bstride;   // bytes between input blocks of a group
    int n_in;
    uint8_t *out;
    long long out_gstride;
    long long out_bstride;
    int n_out;              // rows covered by the grid (max over groups)
    const int *n_out_g;     // optional per-group row count (per-group mode)
    const uint8_t *coef;    // coef[g*coef_gstride + o*coef_ld + j]; coef_ld % 4 == 0
    long long coef_gstride; // 0 when shared by all groups
    int coef_ld;
    const uint64_t *rowbytes;  // 256 entries: byte b = c * 2^b in GF(256)/0x187
    int groups;
    Geometry geo;
};

struct DecodeSetupArgs {
    int k, m;
    const uint8_t *rows;    // [G][rows_gstride] block rows as handed in
    long long rows_gstride;
    const uint8_t *gen;     // (m-1) x k generator rows 1..m-1
    const uint8_t *xp;      // m >= 7: X'[x], x < k  (generator column parameters, X'_0 = 1)
    const uint8_t *yp;      // m >= 7: Y'[y], y < m  (generator row parameters, Y'_0 = 0)
    const uint8_t *gf_exp;  // 512
    const uint16_t *gf_log; // 256
    int emax;
    int *e_out;             // [G] erasure count (-1: singular)
    uint8_t *rec_idx;       // [G][emax] array index of the i-th recovery block
    uint8_t *erasures;      // [G][emax] i-th erased original row
    uint8_t *coefA;         // [G][emax][ldA]
    long long coefA_gstride;
    int ldA;
    uint8_t *coefB;         // generic mode: stage-B coefficients, TRANSPOSED [G][emax][ldB], entry [i][j]
    long long coefB_gstride;
    int ldB;                // >= emax, multiple of 8
    // Fixed-kernel mode (coefA == nullptr): stage A runs the compile-time generator over all m
    // rows, so the setup emits position tables instead of stage-A coefficients, and stage B gets
    // the residual row of each received recovery block plus ready-made snippet addresses.
    uint8_t *pos;           // [G][kp] array index of original row x (0xFF = erased, and x >= k)
    int kp;                 // position-table stride: round4 of the stage-A kernel's K (>= k)
    uint8_t *rpos;          // [G][round4(m)] array index of recovery row y (0xFF = absent)
    uint8_t *rrow;          // [G][ldR] generator row r_i of the i-th received recovery block
    int ldR;                // round4(emax)
    uint64_t *targets;      // [G][ldB/8][emax][8]: address of the stage-B snippet of S^-1[j][i] at [j/8][i][j%8]
    uint64_t snip_base;     // address of snippet 0 (stage-B snippet table, stride SNIP_STRIDE)
    int *errors;            // device counter: groups with more recovery blocks than erasures
};

struct ScatterArgs {
    const uint8_t *src;     // [G][emax][B] recovered, dense
    long long src_gstride;
    uint8_t *blocks;        // [G][k][B] decode blocks, in place
    long long blocks_gstride;
    uint8_t *rows;          // [G][k]
    long long rows_gstride;
    const int *e;
    const uint8_t *rec_idx;
    const uint8_t *erasures;
    int emax;
    int B;
};

// Decode stage B, generic path (csrc/stageb.hip): out[g][j] = sum_i M(coefT[g][i][j]) in[g][i], j < e[g].
struct StageBArgs {
    const uint8_t *in;        // [G][n_in][B] residual rows (>= 4 readable slack bytes at the end)
    long long in_gstride;
    int n_in;
    uint8_t *out;             // [G][emax][B]
    long long out_gstride;
    const int *e;             // [G] outputs per group
    const uint8_t *coefT;     // [G][n_in][ldT], ldT % 8 == 0
    long long coefT_gstride;
    int ldT;
    int groups;
    Geometry geo;
};
hipError_t launch_stageb(const StageBArgs &a, int emax, hipStream_t stream);

// Decode stage B, compile-time path: out[g][j] = sum_{i < e} M(S^-1[j][i]) in[g][rrow[g][i]]
// with the coefficients given as snippet addresses (DecodeSetupArgs::targets).
struct StageBFixedArgs {
    const uint8_t *in;        // [G][n_in][B] residual rows (all m generator rows)
    long long in_gstride;
    uint8_t *out;             // [G][emax][B]
    long long out_gstride;
    const int *e;             // [G] received recovery blocks = outputs (<= 0: nothing to do)
    const uint8_t *rrow;      // [G][ldR]
    const uint64_t *targets;  // [G][ldT/8][emax][8], entry [j/8][i][j%8]
    int emax;
    int ldR;                  // round4(emax): row lists are read as dwords
    int ldT;                  // multiple of 8
    int groups;
    Geometry geo;
};
bool stageb_fixed_ok(const Geometry &geo, int emax);
hipError_t launch_stageb_fixed(const StageBFixedArgs &a, hipStream_t stream);
// Decode stage B after a full-residual stage A (compile-time or tile kernels), byte coefficients:
// out[g][j] = sum_{i < e} M(coefT[g][i][j]) in[g][rrow[g][i]] (csrc/stageb.hip, stageb_v2).
struct StageBV2Args {
    const uint8_t *in;        // [G][n_in][B] residual rows (all m generator rows)
    long long in_gstride;
    uint8_t *out;             // [G][emax][B]
    long long out_gstride;
    const int *e;             // [G] received recovery blocks = outputs (<= 0: nothing to do)
    const uint8_t *rrow;      // [G][ldR] residual row of the i-th received recovery block
    int ldR;                  // round4(emax)
    const uint8_t *coefT;     // [G][emax][ldT]: entry [i][j] = S^-1[j][i] (0 past e)
    long long coefT_gstride;
    int ldT;                  // multiple of 8
    int emax;
    int groups;
    Geometry geo;
    uint64_t snip_base;       // address of snippet 0 of the accumulating table (stride SNIP_STRIDE)
    int j_base;               // set by the launcher: first output of the launch (a tail launch)
    // Row slices (single-group latency path; 0 = off): workgroup z applies input rows
    // [z * row_slice, min(e, (z + 1) * row_slice)) and writes its partial output at
    // out + z * out_slice_bytes; the caller XOR-reduces the partials.
    int row_slice;
    int row_slices;
    long long out_slice_bytes;
};
bool stageb_v2_ok(const Geometry &geo, int emax);
hipError_t launch_stageb_v2(const StageBV2Args &a, hipStream_t stream);
// Decode stage B for small blocks after a compile-time stage A (csrc/stageb.hip, stageb_small):
// per-lane coefficients, so one wave serves 64 / nq groups.
struct StageBSmallArgs {
    const uint8_t *in;        // [G][in_gstride] residual rows (all m generator rows)
    long long in_gstride;
    uint8_t *out;             // [G][out_gstride]
    long long out_gstride;
    const int *e;             // [G] received recovery blocks = outputs (<= 0: nothing to do)
    const uint8_t *rrow;      // [G][ldR] residual row of the i-th received recovery block
    int ldR;
    const uint8_t *coefT;     // [G][emax][ldT]: entry [i][j] = S^-1[j][i] (0 past e)
    long long coefT_gstride;
    int ldT;                  // multiple of 8
    int emax;
    int groups;
    Geometry geo;
    int xcd_map;              // set by the launcher: 1 = XCD-aware block order (see stageb_small)
};
bool stageb_small_ok(const Geometry &geo, int emax);
hipError_t launch_stageb_small(const StageBSmallArgs &a, hipStream_t stream);
// Address of stage-B snippet 0 in the loaded code object (one tiny kernel launch + copy).
hipError_t stageb_snip_base(uint64_t *out_host, hipStream_t stream);
constexpr int SNIP_STRIDE = 72;   // bytes per stage-B snippet (gen_fixed_kernels.py)
constexpr int SNIP_NULL = 256;    // index of the null snippet

// Runtime-coefficient tile kernels (csrc/tile_snip.hip): every (k, m) with B % 8 == 0, B/8 >= 16.
// One launch codes output rows [row0, row0 + nrows) (nrows <= 128) of every group: f.out points at
// row row0 of group 0 (f.out_gstride = m * B). targets = per-part tables of snippet-address low
// dwords, [parts][tstride] with tstride = ceil(nsteps / S) * S * 8 (S = tile_steps_per_group),
// entry [p][x][j] for row 8p + j of the launch and step x (decode: x < k input column x,
// x >= k recovery row row0 + x - k).
struct TileArgs {
    FixedArgs f;
    const uint32_t *targets;
    long long tstride;
    uint32_t snip_hi;         // high dword of every snippet address
    int k, m, row0, nrows, nsteps;
    // Step slices (single-group latency): slice s = blockIdx.y codes steps [s*slice_steps, ...)
    // into its own partial output at f.out + s * out_slice_bytes (XOR-reduced afterwards).
    // slice_steps = 0: one slice over every step.
    int slice_steps, slices;
    long long out_slice_bytes;
    // Column mode (m >= 7): targets hold 2 dwords per (part, step) -- the column snippets of the
    // part's one or two 4-row blocks (0 = no call) -- instead of 8 per-row snippet addresses.
    int col;
};
// Base addresses of the column-snippet tables (csrc/gen/colsnip_<t>.hip), one per translation unit.
hipError_t colsnip_bases(uint64_t *out_host, int n, hipStream_t stream);
bool tile_ok(int B);
int tile_parts(int nrows);
int tile_steps_per_group(int parts);
hipError_t launch_tile(const TileArgs &t, bool dec, hipStream_t stream);

// Returns hipErrorNotSupported (and launches nothing) when (k, m) has no generated kernel or the
// block is too short (sub < 4).
hipError_t launch_fixed(int k, int m, FixedArgs a, bool dec, hipStream_t stream);
bool has_fixed(int k, int m, int B);
// K of the compile-time kernel that codes (k, m, B): k itself, or the smallest compiled K > k for
// the same m with k >= 0.6 K (its steps past k read zeros, FixedArgs::k_rt); 0 = none.
int fixed_kernel_k(int k, int m, int B);

hipError_t launch_apply(const ApplyArgs &a, bool per_group, hipStream_t stream);
hipError_t launch_xor_rows(const uint8_t *in, long long in_gstride, int n_in, uint8_t *out,
                           long long out_gstride, int B, int groups, hipStream_t stream);
hipError_t launch_copy_first(const uint8_t *in, long long in_gstride, uint8_t *out,
                             long long out_gstride, int m, int B, int groups, hipStream_t stream);
hipError_t launch_decode_setup(const DecodeSetupArgs &a, int groups, hipStream_t stream);
hipError_t launch_scatter(const ScatterArgs &a, int groups, hipStream_t stream);
hipError_t launch_decode_m1(uint8_t *blocks, long long blocks_gstride, const uint8_t *rows,
                            long long rows_gstride, int k, int B, int groups, hipStream_t stream);
hipError_t launch_decode_k1(uint8_t *rows, long long rows_gstride, int groups, hipStream_t stream);
// out[i] = XOR over p < nparts of parts[p * part_bytes + i], i < nbytes (the slices' partials).
hipError_t launch_xor_reduce(const uint8_t *parts, long long part_bytes, int nparts, uint8_t *out,
                             long long nbytes, hipStream_t stream);
hipError_t launch_fill(uint8_t *out, long long gstride, int n, int B, int groups,
                       unsigned long long g0, unsigned long long cfg, hipStream_t stream);

}  // namespace sh
