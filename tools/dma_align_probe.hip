// Measurement only (never part of the product): read-side cost of the compile-time kernels' input
// DMA pattern against reading the same blocks as aligned contiguous runs.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/dma_align_probe tools/dma_align_probe.hip
//   dma_align_probe [groups]
//
// Shape: encode k=200, B=1400 (sub-block 175 bytes, nq = 44 word columns per group), ring of 16
// LDS slots, a workgroup barrier every 4 steps, no compute, no stores. Per step a workgroup reads
// one input block of its columns into one slot:
//   gather   the product's pattern: 128 columns per tile (2.9 groups), each 16-byte DMA lane reads
//            4 columns of one sub-block (175-byte runs at arbitrary alignment)
//   raw      3 whole groups per tile (132 columns): the 3 blocks as contiguous 1400-byte runs, read
//            in 16-byte chunks aligned down to 16 (1408 bytes each)
//   aligned  as gather with the sub-block size padded to 176 (what the lab's "algn" variant did)
//   gorder   as gather, DMA lanes ordered (group, sub-block, chunk) instead of (sub-block, column)
//   a16      as gather, each lane's offset rounded down to 16 (same lines, wrong bytes)
//   xcd      as gather, tiles in XCD-aware order (neighbouring tiles share one L2)
//   gord16   gorder with each lane's offset rounded down to 16 (contiguous and aligned, wrong bytes)
//   gath3    gather over tiles of 3 whole groups (132 columns, the last 4 unread: timing only)
// Every variant moves within 3 % of the same bytes; the time per byte is what differs.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

typedef __attribute__((address_space(3))) void lds_void;
constexpr int K = 200, B = 1400, NQ = 44, R = 16, S = 4, NT = 256, W = 16;
constexpr long long GSTRIDE = (long long)K * B;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const uint8_t *p, long long bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(p), (short)0,
                                             (int)(bytes > 0x7FFFFFFFll ? 0x7FFFFFFFll : bytes), 0x00020000);
}

// MODE 0 gather (sub 175), 2 aligned (sub 176): lane's 16 bytes = 4 columns of one sub-block.
// MODE 1 raw: lane's 16 bytes = one aligned chunk of one of the tile's 3 blocks.
template <int MODE>
__global__ __launch_bounds__(NT) void probe(const uint8_t *in, long long in_bytes, int groups, uint32_t *sink) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[R * 4096 + 256];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // MODE 5: gather with an XCD-aware order (workgroup i runs on XCD i % 8: consecutive tiles
    // on one XCD, so a group split between two tiles is read through one L2)
    int tile = blockIdx.x;
    if (MODE == 5) {
        const int per = (gridDim.x + 7) / 8, xcd = blockIdx.x % 8, i = blockIdx.x / 8;
        tile = xcd * per + i;
        if (tile >= (int)gridDim.x) return;  // (the few extra slots of the last XCD)
    }
    uint32_t voff;
    long long base;
    if (MODE == 1) {
        const int g0 = tile * 3;
        base = (long long)g0 * GSTRIDE;
        const int i = threadIdx.x;                  // chunk 0..255 of 3 x 88 (the last 8 unread)
        const int r = i / 88, j = i - r * 88;
        voff = (g0 + r < groups) ? (uint32_t)(r * GSTRIDE + 16 * j) : 0x80000000u;
    } else if (MODE == 3 || MODE == 6) {
        // gorder: the product's 128-column tiles, DMA lanes ordered (group, sub-block, 4-column
        // chunk) -- consecutive lanes walk a group's block nearly contiguously (the LDS image
        // becomes [group segment][sub-block][columns], still 16-byte aligned per sub-block)
        const long long col0 = (long long)tile * 128;
        const int gf = (int)(col0 / NQ);
        base = (long long)gf * GSTRIDE;
        int i = threadIdx.x;  // chunk index 0..255
        voff = 0x80000000u;
        for (int g = gf; g * (long long)NQ < col0 + 128; ++g) {
            const long long lo = g * (long long)NQ > col0 ? g * (long long)NQ : col0;
            const long long hi = (g + 1) * (long long)NQ < col0 + 128 ? (g + 1) * (long long)NQ : col0 + 128;
            const int nch = (int)((hi - lo) / 4), q0 = (int)(lo - g * (long long)NQ);
            if (i < 8 * nch) {
                const int a = i / nch, q = q0 + 4 * (i - a * nch);
                const int co = 4 * q - (q >= NQ - 4 ? 4 * NQ - 175 : 0);
                if (g < groups) voff = (uint32_t)((g - gf) * GSTRIDE + a * 175 + co);
                if (MODE == 6 && voff != 0x80000000u) voff &= ~15u;  // contiguous AND aligned
                break;
            }
            i -= 8 * nch;
        }
    } else {
        const int sub = MODE == 2 ? 176 : 175;
        // MODE 7: tiles of 3 whole groups (132 columns; the 128 lanes leave the last 4 unread)
        const long long col0 = MODE == 7 ? (long long)tile * 132 : (long long)tile * 128;
        const int gf = (int)(col0 / NQ);
        base = (long long)gf * GSTRIDE;
        const int off = wave * 1024 + lane * W;
        const int a = off / 512, cc = (off % 512) / 4;
        const long long colx = col0 + cc;
        const int g = (int)(colx / NQ), q = (int)(colx - (long long)g * NQ);
        const int co = 4 * q - (q >= NQ - 4 ? 4 * NQ - sub : 0);
        voff = (g < groups) ? (uint32_t)((g - gf) * GSTRIDE + a * sub + co) : 0x80000000u;
        if (MODE == 4 && voff != 0x80000000u) voff &= ~15u;  // (MODE 5: as 0)  // same lines, 16-byte aligned lanes
    }
    const __amdgpu_buffer_rsrc_t rs = rsrc_of(in + base, in_bytes - base);
    uint8_t *slot0 = ring + wave * 1024;
    auto issue = [&](int x) {
        uint32_t so = (uint32_t)x * B;
        if (MODE == 1) so -= (x & 1) * 8;  // block x starts at 8 mod 16 for odd x
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void *)(slot0 + (x % R) * 4096), W, voff, so, 0, 0);
    };
#pragma unroll
    for (int x = 0; x < R - 1; ++x) issue(x);
    int nxt = R - 1;
    uint32_t acc = 0;
    for (int x0 = 0; x0 < K; x0 += S) {
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(R - 1 - S) : "memory");
        acc ^= *reinterpret_cast<const uint32_t *>(ring + (x0 % R) * 4096 + threadIdx.x * 16);
        for (int t = 0; t < S && nxt < K; ++t, ++nxt) issue(nxt);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}


// MODE blk (round 5): the product's 128-column tiles in XCD-aware order, but each step reads the
// WHOLE block of every group the tile touches (3-4 groups) as one contiguous 16-byte-aligned run of
// 88 chunks (1408 bytes; odd blocks start 8 bytes early): a lane would then read its words with
// unaligned ds_read_b32 from the raw block image. Edge groups are read by both neighbouring tiles
// (same XCD, same time: the second read hits L2). RB slots of 6 KB, SB steps per barrier, 2 DMA
// issues per wave and step (the 6th..8th 1 KB pieces only where the tile touches groups).
template <int RB, int SB, bool XCD, int SHIFT = 1>
__global__ __launch_bounds__(NT) void probe_blk(const uint8_t *in, long long in_bytes, int groups, int ntiles, uint32_t *sink) {
    constexpr int SLOTB = 6144;
    __shared__ __attribute__((aligned(16))) uint8_t ring[RB * SLOTB + 256];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int tile = blockIdx.x;
    if (XCD) {
        const int q = ntiles >> 3, r = ntiles & 7, x = blockIdx.x & 7, i = blockIdx.x >> 3;
        tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
    }
    const long long col0 = (long long)tile * 128;
    const int gf = (int)(col0 / NQ);
    long long cl = col0 + 127;
    if (cl > (long long)groups * NQ - 1) cl = (long long)groups * NQ - 1;
    const int ng = (int)(cl / NQ) - gf + 1;
    const long long base = (long long)gf * GSTRIDE;
    const __amdgpu_buffer_rsrc_t rs = rsrc_of(in + base, in_bytes - base);
    uint32_t voff[2];
    bool act[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int i = (wave * 2 + h) * 64 + lane;
        const int r = i / 88, j = i - r * 88;
        voff[h] = r < ng ? (uint32_t)(r * GSTRIDE + 16 * j) : 0x80000000u;
        act[h] = (wave * 2 + h) * 64 < ng * 88;  // uniform: a piece with any lane inside
    }
    auto issue = [&](int x) {
        // SHIFT 1: chunks 16-byte aligned (odd blocks start 8 bytes early); 0: from the block start
        // (odd blocks 8-misaligned); 2: every block 4 bytes past its start (all misaligned)
        const uint32_t so = SHIFT == 1 ? (uint32_t)x * B - (uint32_t)(x & 1) * 8 : (uint32_t)x * B + (SHIFT == 2 ? 4u : 0u);
#pragma unroll
        for (int h = 0; h < 2; ++h)
            if (act[h])
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void *)(ring + (x % RB) * SLOTB + (wave * 2 + h) * 1024), W,
                                                         voff[h], so, 0, 0);
    };
    const int nis = (int)act[0] + (int)act[1];  // this wave's DMAs per step
#pragma unroll
    for (int x = 0; x < RB - 1; ++x) issue(x);
    int nxt = RB - 1;
    uint32_t acc = 0;
    for (int x0 = 0; x0 < K; x0 += SB) {
        if (nis == 2)
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * (RB - 1 - SB)) : "memory");
        else if (nis == 1)
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(RB - 1 - SB) : "memory");
        else
            asm volatile("s_barrier" ::: "memory");
        acc ^= *reinterpret_cast<const uint32_t *>(ring + (x0 % RB) * SLOTB + threadIdx.x * 20 + 3);
        for (int t = 0; t < SB && nxt < K; ++t, ++nxt) issue(nxt);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

// Round 5: what makes `blk` fast? Gather pieces (16 bytes = 4 columns of one sub-block, the last
// chunk of a sub-block shifted back) over the tile's EXTENDED column range (every group the tile
// touches, whole), XCD-aware tile order, 6 pieces per step:
//   ORD 0: lanes over [sub-block][extended column] (the product's slot layout, 192 columns)
//   ORD 1: lanes over (group, sub-block, chunk): each 1 KB piece walks a group's block nearly
//          contiguously (like blk, but runs end at sub-block boundaries)
// XCD false: plain tile order.
template <int ORD, bool XCD>
__global__ __launch_bounds__(NT) void probe_ext(const uint8_t *in, long long in_bytes, int groups, int ntiles, uint32_t *sink) {
    constexpr int RB = 13, SB = 4, SLOTB = 6144;
    __shared__ __attribute__((aligned(16))) uint8_t ring[RB * SLOTB + 256];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int tile = blockIdx.x;
    if (XCD) {
        const int q = ntiles >> 3, r = ntiles & 7, x = blockIdx.x & 7, i = blockIdx.x >> 3;
        tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
    }
    const long long col0 = (long long)tile * 128;
    const int gf = (int)(col0 / NQ);
    long long cl = col0 + 127;
    if (cl > (long long)groups * NQ - 1) cl = (long long)groups * NQ - 1;
    const int ng = (int)(cl / NQ) - gf + 1;
    const long long base = (long long)gf * GSTRIDE;
    const __amdgpu_buffer_rsrc_t rs = rsrc_of(in + base, in_bytes - base);
    uint32_t voff[2];
    bool act[2];
    constexpr int CPS = NQ / 4;  // chunks per sub-block (11)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int i = (wave * 2 + h) * 64 + lane;  // piece lane index 0..511
        int r, a, c;
        if (ORD == 0) {  // [a][ext column]: 48 chunks per sub-block row (192 columns)
            a = i / 48;
            const int cc = i - a * 48;  // chunk within the extended row
            r = cc / CPS;
            c = cc - r * CPS;
        } else {  // (group, sub-block, chunk)
            r = i / (8 * CPS);
            const int t = i - r * 8 * CPS;
            a = t / CPS;
            c = t - a * CPS;
        }
        const int q = 4 * c;
        const int co = 4 * q - (q >= NQ - 4 ? 4 * NQ - 175 : 0);
        voff[h] = (r < ng && a < 8) ? (uint32_t)(r * GSTRIDE + a * 175 + co) : 0x80000000u;
        act[h] = (wave * 2 + h) < 6;
    }
    auto issue = [&](int x) {
        const uint32_t so = (uint32_t)x * B;
#pragma unroll
        for (int h = 0; h < 2; ++h)
            if (act[h])
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void *)(ring + (x % RB) * SLOTB + (wave * 2 + h) * 1024), W,
                                                         voff[h], so, 0, 0);
    };
    const int nis = (int)act[0] + (int)act[1];
#pragma unroll
    for (int x = 0; x < RB - 1; ++x) issue(x);
    int nxt = RB - 1;
    uint32_t acc = 0;
    for (int x0 = 0; x0 < K; x0 += SB) {
        if (nis == 2)
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * (RB - 1 - SB)) : "memory");
        else if (nis == 1)
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(RB - 1 - SB) : "memory");
        else
            asm volatile("s_barrier" ::: "memory");
        acc ^= *reinterpret_cast<const uint32_t *>(ring + (x0 % RB) * SLOTB + threadIdx.x * 20 + 3);
        for (int t = 0; t < SB && nxt < K; ++t, ++nxt) issue(nxt);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

int main(int argc, char **argv) {
    const int groups = argc > 1 ? atoi(argv[1]) : 8192;
    const long long bytes = (long long)groups * GSTRIDE;
    uint8_t *in;
    uint32_t *sink;
    CK(hipMalloc(&in, bytes));
    CK(hipMalloc(&sink, 4096));
    CK(hipMemset(in, 0x5A, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int tiles_g = (int)((groups * (long long)NQ + 127) / 128), tiles_r = (groups + 2) / 3;
    const char *names[8] = {"gather", "raw", "aligned", "gorder", "a16", "xcd", "gord16", "gath3"};
    for (int rep = 0; rep < 2; ++rep)
        for (int mode = 0; mode < 8; ++mode) {
            float best = 1e9f;
            for (int it = 0; it < 10; ++it) {
                CK(hipEventRecord(e0));
                if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(tiles_g), dim3(NT), 0, 0, in, bytes, groups, sink);
                if (mode == 1) hipLaunchKernelGGL(probe<1>, dim3(tiles_r), dim3(NT), 0, 0, in, bytes, groups, sink);
                if (mode == 2) hipLaunchKernelGGL(probe<2>, dim3(tiles_g), dim3(NT), 0, 0, in, bytes, groups, sink);
                if (mode == 3) hipLaunchKernelGGL(probe<3>, dim3(tiles_g), dim3(NT), 0, 0, in, bytes, groups, sink);
                if (mode == 4) hipLaunchKernelGGL(probe<4>, dim3(tiles_g), dim3(NT), 0, 0, in, bytes, groups, sink);
                if (mode == 5) hipLaunchKernelGGL(probe<5>, dim3(tiles_g), dim3(NT), 0, 0, in, bytes, groups, sink);
                if (mode == 6) hipLaunchKernelGGL(probe<6>, dim3(tiles_g), dim3(NT), 0, 0, in, bytes, groups, sink);
                if (mode == 7) hipLaunchKernelGGL(probe<7>, dim3(tiles_r), dim3(NT), 0, 0, in, bytes, groups, sink);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) best = ms;
            }
            const double moved = (double)(mode == 1 || mode == 7 ? tiles_r : tiles_g) * K * 4096.0;  // DMA'd bytes
            printf("%-8s groups %d  best %.4f ms  %.0f GB/s DMA'd  %.0f GB/s of block bytes\n", names[mode], groups,
                   best, moved / best / 1e6, (double)groups * K * B / best / 1e6);
        }
    const char *en[4] = {"ext_ax", "ext_gx", "ext_a", "ext_g"};
    for (int rep = 0; rep < 2; ++rep)
        for (int mode = 0; mode < 4; ++mode) {
            float best = 1e9f;
            for (int it = 0; it < 10; ++it) {
                CK(hipEventRecord(e0));
                if (mode == 0) hipLaunchKernelGGL((probe_ext<0, true>), dim3(tiles_g), dim3(NT), 0, 0, in, bytes, groups, tiles_g, sink);
                if (mode == 1) hipLaunchKernelGGL((probe_ext<1, true>), dim3(tiles_g), dim3(NT), 0, 0, in, bytes, groups, tiles_g, sink);
                if (mode == 2) hipLaunchKernelGGL((probe_ext<0, false>), dim3(tiles_g), dim3(NT), 0, 0, in, bytes, groups, tiles_g, sink);
                if (mode == 3) hipLaunchKernelGGL((probe_ext<1, false>), dim3(tiles_g), dim3(NT), 0, 0, in, bytes, groups, tiles_g, sink);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) best = ms;
            }
            printf("%-8s groups %d  best %.4f ms  %.0f GB/s of block bytes\n", en[mode], groups, best,
                   (double)groups * K * B / best / 1e6);
        }
    const char *bn[6] = {"blk13s4x", "blk_nosh", "blk_mis4", "blk13s4", "blk8s2x", "blk16s4x"};
    for (int rep = 0; rep < 2; ++rep)
        for (int mode = 0; mode < 6; ++mode) {
            float best = 1e9f;
            for (int it = 0; it < 10; ++it) {
                CK(hipEventRecord(e0));
                if (mode == 0) hipLaunchKernelGGL((probe_blk<13, 4, true>), dim3(tiles_g), dim3(NT), 0, 0, in, bytes, groups, tiles_g, sink);
                if (mode == 1) hipLaunchKernelGGL((probe_blk<13, 4, true, 0>), dim3(tiles_g), dim3(NT), 0, 0, in, bytes, groups, tiles_g, sink);
                if (mode == 2) hipLaunchKernelGGL((probe_blk<13, 4, true, 2>), dim3(tiles_g), dim3(NT), 0, 0, in, bytes, groups, tiles_g, sink);
                if (mode == 3) hipLaunchKernelGGL((probe_blk<13, 4, false>), dim3(tiles_g), dim3(NT), 0, 0, in, bytes, groups, tiles_g, sink);
                if (mode == 4) hipLaunchKernelGGL((probe_blk<8, 2, true>), dim3(tiles_g), dim3(NT), 0, 0, in, bytes, groups, tiles_g, sink);
                if (mode == 5) hipLaunchKernelGGL((probe_blk<16, 4, true>), dim3(tiles_g), dim3(NT), 0, 0, in, bytes, groups, tiles_g, sink);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) best = ms;
            }
            printf("%-8s groups %d  best %.4f ms  %.0f GB/s of block bytes\n", bn[mode], groups, best,
                   (double)groups * K * B / best / 1e6);
        }
    return 0;
}
