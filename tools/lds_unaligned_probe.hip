// Measurement only (never part of the product): cost of ds_read_b32 at byte-unaligned LDS
// addresses (gfx950 unaligned access mode) against aligned ones, and that the bytes are right.
//   hipcc --offload-arch=gfx950 -O3 -o tools/lds_unaligned_probe tools/lds_unaligned_probe.hip
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

// 8 reads per iteration at 8 row offsets (like a step's 8 sub-block words), row stride 176 bytes
// + shift so that rows have different alignments when shift != 0 (MODE 1), all aligned (MODE 0).
template <int MODE>
__global__ __launch_bounds__(256) void k(uint32_t *out, int iters) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[16384 + 64];
    for (int i = threadIdx.x; i < (16384 + 64) / 4; i += 256) reinterpret_cast<uint32_t *>(lds)[i] = i * 2654435761u;
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t acc = 0;
    const uint8_t *base = lds + wave * 4096 + lane * 4;
    for (int it = 0; it < iters; ++it) {
        const int o = (it & 3) * 8;  // keep the compiler from hoisting
#pragma unroll
        for (int a = 0; a < 8; ++a) {
            const int off = MODE == 0 ? a * 256 + o : a * 256 + o + ((a * 3) & 3);  // 0,3,2,1,...
            uint32_t v;
            __builtin_memcpy(&v, base + off, 4);
            acc = __builtin_amdgcn_bitop3_b32(acc, v, acc << 1, 0x96);
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

__global__ void check(uint32_t *out) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) lds[i] = static_cast<uint8_t>(i * 7 + 3);
    __syncthreads();
    uint32_t bad = 0;
    for (int s = 0; s < 4; ++s) {
        uint32_t v;
        __builtin_memcpy(&v, lds + threadIdx.x * 4 + s, 4);
        for (int b = 0; b < 4; ++b) {
            const int i = threadIdx.x * 4 + s + b;
            if (((v >> (8 * b)) & 0xFF) != static_cast<uint8_t>(i * 7 + 3)) ++bad;
        }
    }
    out[threadIdx.x] = bad;
}

int main() {
    uint32_t *out;
    CK(hipMalloc(&out, 1 << 24));
    hipLaunchKernelGGL(check, dim3(1), dim3(64), 0, 0, out);
    uint32_t h[64];
    CK(hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost));
    uint32_t bad = 0;
    for (int i = 0; i < 64; ++i) bad += h[i];
    printf("unaligned ds_read_b32 byte errors: %u\n", bad);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int blocks = 256 * 8, iters = 4096;
    for (int rep = 0; rep < 2; ++rep)
        for (int mode = 0; mode < 2; ++mode) {
            float best = 1e9f;
            for (int t = 0; t < 5; ++t) {
                CK(hipEventRecord(e0));
                if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters);
                else hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) best = ms;
            }
            const double reads = (double)blocks * 4 * iters * 8;  // wave-instructions
            printf("%-9s %.3f ms  %.1f G wave-reads/s  (%.2f CU-cycles per wave-read at 2.4 GHz)\n",
                   mode ? "unaligned" : "aligned", best, reads / best / 1e6, 256 * 2.4e9 / (reads / best * 1e3));
        }
    return 0;
}
