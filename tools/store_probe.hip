// Measurement only (never part of the product): cost of the compile-time kernels' output store
// pattern (RowSink: 16-byte pieces in memory order, a sub-block run of 11 pieces at B = 1400 with
// the last piece shifted back one byte) against the same bytes stored as contiguous 16-byte
// chunks (one run per group row).
//   hipcc --offload-arch=gfx950 -O3 -o tools/store_probe tools/store_probe.hip
// Shape: k=200 m=32 B=1400, 8192 groups: 32 rows of 1400 bytes per group (0.367 GB), one
// workgroup of 256 threads per 128-column tile (2816 tiles); each writes its tile's pieces of
// every row (the product's piece assignment: group by group, sub-block by sub-block).
//   MODE 0 rowsink : pieces = 4 columns of one sub-block (byte offset a*175 + 16c, last c shifted)
//   MODE 1 contig  : pieces = aligned 16-byte chunks of each whole group row the tile starts
//                    (whole groups: tile t writes the groups whose first column lies in it)
//   MODE 2 rowsink, stores issued in one burst per row for all 32 rows (no waits)
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

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int M = 32, B = 1400, NQ = 44, NT = 256;
constexpr long long OSTRIDE = (long long)M * B;

template <int MODE>
__global__ __launch_bounds__(NT) void probe(uint8_t *out, long long out_bytes, int groups) {
    const int tile = blockIdx.x;
    const long long col0 = (long long)tile * 128;
    long long ce = col0 + 128;
    if (ce > (long long)groups * NQ) ce = (long long)groups * NQ;
    const int gf = (int)(col0 / NQ);
    const long long base = (long long)gf * OSTRIDE;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        out + base, (short)0, (int)((out_bytes - base) > 0x7FFFFFFFll ? 0x7FFFFFFFll : (out_bytes - base)), 0x00020000);
    uint32_t off[2];
    const u32x4 v = {threadIdx.x, 1u, 2u, 3u};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        int rem = h * 256 + threadIdx.x;  // piece index (512 per row: 128 columns x 8 sub-blocks / 4 ... x2)
        off[h] = 0x80000000u;
        if (MODE == 1) {
            // groups whose first column lies in [col0, col0 + 128): 88 chunks per group row
            const int g0 = (int)((col0 + NQ - 1) / NQ);
            const int g = g0 + rem / 88, j = rem % 88;
            if ((long long)g * NQ < ce && g < groups && j < 88) off[h] = (uint32_t)((g - gf) * OSTRIDE + 16 * j - (j == 87 ? 8 : 0));
        } else {
            // RowSink order over the tile's columns [col0, ce): group, sub-block, 4-column chunk
            for (long long g = col0 / NQ; g * NQ < ce; ++g) {
                const int qa = (int)((col0 > g * NQ ? col0 : g * NQ) - g * NQ);
                const int qb = (int)((ce < (g + 1) * NQ ? ce : (g + 1) * NQ) - g * NQ);
                const int nch = (qb - qa) >> 2;
                if (rem < 8 * nch) {
                    const int a = rem / nch, q = qa + 4 * (rem - a * nch);
                    off[h] = (uint32_t)((g - gf) * OSTRIDE + a * 175 + 4 * q - (q >= NQ - 4 ? 1 : 0));
                    break;
                }
                rem -= 8 * nch;
            }
        }
    }
    for (int y = 0; y < M; ++y) {
#pragma unroll
        for (int h = 0; h < 2; ++h) __builtin_amdgcn_raw_buffer_store_b128(v, rs, off[h], y * B, 0);
        if (MODE != 2) __syncthreads();
    }
}

int main(int argc, char **argv) {
    const int groups = argc > 1 ? atoi(argv[1]) : 8192;
    const long long bytes = (long long)groups * OSTRIDE;
    uint8_t *out;
    CK(hipMalloc(&out, bytes + 4096));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int tiles = (int)((groups * (long long)NQ + 127) / 128);
    const char *names[3] = {"rowsink", "contig", "rs_burst"};
    for (int rep = 0; rep < 2; ++rep)
        for (int mode = 0; mode < 3; ++mode) {
            float best = 1e9f;
            for (int it = 0; it < 10; ++it) {
                CK(hipEventRecord(e0));
                if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(tiles), dim3(NT), 0, 0, out, bytes, groups);
                if (mode == 1) hipLaunchKernelGGL(probe<1>, dim3(tiles), dim3(NT), 0, 0, out, bytes, groups);
                if (mode == 2) hipLaunchKernelGGL(probe<2>, dim3(tiles), dim3(NT), 0, 0, out, bytes, groups);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) best = ms;
            }
            printf("%-9s groups %d  best %.4f ms  %.0f GB/s of row bytes\n", names[mode], groups, best,
                   (double)bytes / best / 1e6);
        }
    return 0;
}
