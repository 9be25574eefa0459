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
    return 0;
}
