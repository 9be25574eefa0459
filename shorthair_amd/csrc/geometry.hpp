// Block geometry and the argument block of the compile-time-scheduled kernels: the only part of
// the device ABI the generated kernels (csrc/gen/, via fixed_common.hpp) depend on, kept apart
// from kernels.hpp so that changes to other kernels' arguments do not recompile them.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sh {

// Column geometry of a block size B (multiple of 8): sub = B/8 bytes per sub-block, nq 32-bit
// word columns per sub-block, the last one holding `tail` (1..4) valid bytes.
struct Geometry {
    int B;
    int sub;
    int nq;
    int tail;
};

inline Geometry make_geometry(int B) {
    Geometry g;
    g.B = B;
    g.sub = B / 8;
    g.nq = (g.sub + 3) / 4;
    g.tail = g.sub - 4 * (g.nq - 1);
    return g;
}

// Geometry of the compile-time path: the word columns per sub-block are rounded up to a multiple
// of 4 so 16-byte (4-column) chunks never straddle two groups; the last chunk of a sub-block is
// shifted back by 4 * nq - sub (< 16) bytes so it ends at the sub-block's end (its first bytes
// are computed twice, identically). Needs sub >= 16.
inline Geometry fixed_geometry(int B) {
    Geometry g = make_geometry(B);
    g.nq = (g.nq + 3) & ~3;
    g.tail = 4;
    return g;
}

// Compile-time-scheduled kernels (csrc/gen/, tools/gen_fixed_kernels.py).
struct FixedArgs {
    const uint8_t *in;        // encode: data [G][k][B]; decode A: received blocks [G][k][B]
    long long in_gstride;
    long long in_bytes;       // groups * in_gstride
    uint8_t *out;             // encode: recovery [G][m][B]; decode A: residual [G][m][B]
    long long out_gstride;
    long long out_bytes;      // groups * out_gstride
    int groups;
    Geometry geo;
    const uint8_t *pos;       // decode: [G][round4(k)] array index of original row x, 0xFF = erased
    const uint8_t *rpos;      // decode: [G][round4(m)] array index of recovery row y, 0xFF = absent
    int groups_per_wg;        // set by the launcher
    // Tail split (fixed_common.hpp, "Split tiles"): the launch's last `nsplit` tiles run as two
    // half-step workgroups each, combined in-launch. Host-provided scratch (per stream):
    // split_part holds the halves' partial rows, split_cnt one arrival counter per split tile
    // (zero between launches); split_cap = bytes of split_part. nsplit is set by the launcher.
    uint8_t *split_part;
    uint32_t *split_cnt;
    long long split_cap;
    int split_max;            // counters available (split tiles at most)
    int nsplit;
    int pf_stride;            // workgroup slots of the launch (L2 prefetch of a later tile, A/B)
    // Runtime k (0 = the kernel's compile-time K). For m >= 7 and for the searched m <= 6 tables the
    // generator's column x does not depend on k (cauchy_256.cpp:423-481), so a kernel compiled for
    // (K, m) codes any k <= K: its steps x >= k read zeros (encode: out-of-range DMA; decode: the
    // position tables, K wide, mark them erased).
    int k_rt;
};

}  // namespace sh
