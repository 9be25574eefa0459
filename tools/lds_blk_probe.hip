// Measurement only (never part of the product): cost of the whole-block ring's LDS reads
// (BlkSrc, fixed_common.hpp) -- ds_read_b32 at a * SUB + per-lane column bytes -- against the
// sub-block-row layout's aligned reads. Modes (lane L of a wave, read a = 0..7):
//   0 aligned, one run:            4L + 256a
//   1 one run, misaligned uniform: 4L + 175a
//   2 two runs (groups of 44 columns from column 20, slots 1456 B apart), misaligned: r*1456 + 4q + 175a
//   3 two runs, aligned pitch:     r*1456 + 4q + 176a
//   4 one run, misaligned, via the address VGPR (offset 0): (4L + 175a) in the VGPR
//   5 two runs, misaligned, via the address VGPR
//   hipcc --offload-arch=gfx950 -O3 -o tools/lds_blk_probe tools/lds_blk_probe.hip
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

typedef uint32_t u32_ua __attribute__((aligned(1)));

template <int MODE>
__global__ __launch_bounds__(256) void k(uint32_t *out, int iters) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 6144 + 64];
    for (int i = threadIdx.x; i < (4 * 6144 + 64) / 4; i += 256) reinterpret_cast<uint32_t *>(lds)[i] = i * 2654435761u;
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c = 20 + lane, r = c / 44, q = c - r * 44;
    uint32_t rd = (MODE == 0 || MODE == 1 || MODE == 4) ? 4 * lane : r * 1456 + 4 * q;
    rd += wave * 6144;
    uint32_t acc = 0;
    for (int it = 0; it < iters; ++it) {
        const uint32_t o = (it & 3) * 4;  // keep the compiler from hoisting
        uint32_t v[8];
        if (MODE == 4 || MODE == 5) {
#pragma unroll
            for (int a = 0; a < 8; ++a) {
                uint32_t addr = rd + o + 175 * a;
                asm volatile("" : "+v"(addr));  // force the offset into the VGPR
                v[a] = *reinterpret_cast<const u32_ua *>(lds + addr);
            }
        } else {
            const uint8_t *p = lds + rd + o;
#pragma unroll
            for (int a = 0; a < 8; ++a) {
                const int off = MODE == 0 ? 256 * a : (MODE == 3 ? 176 * a : 175 * a);
                v[a] = *reinterpret_cast<const u32_ua *>(p + off);
            }
        }
#pragma unroll
        for (int a = 0; a < 8; a += 2) acc = __builtin_amdgcn_bitop3_b32(acc, v[a], v[a + 1], 0x96);
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
    uint32_t *out;
    CK(hipMalloc(&out, 1 << 24));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int blocks = 256 * 6, iters = 2048;
    const char *names[6] = {"aligned_1run", "mis_1run", "mis_2runs", "al176_2runs", "mis_1run_vgpr", "mis_2runs_vgpr"};
    for (int rep = 0; rep < 2; ++rep)
        for (int mode = 0; mode < 6; ++mode) {
            float best = 1e9f;
            for (int t = 0; t < 5; ++t) {
                CK(hipEventRecord(e0));
                switch (mode) {
                    case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 3: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 4: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 5: hipLaunchKernelGGL(k<5>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                }
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) best = ms;
            }
            const double reads = (double)blocks * 4 * iters * 8;  // wave-instructions
            printf("%-15s %.3f ms  %.2f CU-cycles per wave-read at 2.4 GHz\n", names[mode], best,
                   256 * 2.4e9 / (reads / best * 1e3));
        }
    return 0;
}
