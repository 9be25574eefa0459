// Measurement only: does a v_bitop3_b32 whose three VGPR operands sit in the same register bank
// (register number mod 4) issue slower than one with operands in different banks?
//   hipcc --offload-arch=gfx950 -O3 tools/bank_probe.hip -o tools/lab_bin/bank_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP8(x) x x x x x x x x
// same bank: v8 ^= v12 ^ v16 (8, 12, 16: bank 0)
#define SAME "v_bitop3_b32 v8, v8, v12, v16 bitop3:0x96\n v_bitop3_b32 v20, v20, v24, v28 bitop3:0x96\n" \
             "v_bitop3_b32 v32, v32, v36, v40 bitop3:0x96\n v_bitop3_b32 v44, v44, v48, v52 bitop3:0x96\n"
// different banks: v8 ^= v13 ^ v18 (banks 0, 1, 2)
#define DIFF "v_bitop3_b32 v8, v8, v13, v18 bitop3:0x96\n v_bitop3_b32 v20, v20, v25, v30 bitop3:0x96\n" \
             "v_bitop3_b32 v32, v32, v37, v42 bitop3:0x96\n v_bitop3_b32 v44, v44, v49, v54 bitop3:0x96\n"
// two same-bank sources, accumulator elsewhere: v9 ^= v12 ^ v16
#define TWO "v_bitop3_b32 v9, v9, v12, v16 bitop3:0x96\n v_bitop3_b32 v21, v21, v24, v28 bitop3:0x96\n" \
            "v_bitop3_b32 v33, v33, v36, v40 bitop3:0x96\n v_bitop3_b32 v45, v45, v48, v52 bitop3:0x96\n"

// accumulator and first source in one bank: v8 ^= v12 ^ v17
#define AS1 "v_bitop3_b32 v8, v8, v12, v17 bitop3:0x96\n v_bitop3_b32 v20, v20, v24, v29 bitop3:0x96\n" \
            "v_bitop3_b32 v32, v32, v36, v41 bitop3:0x96\n v_bitop3_b32 v44, v44, v48, v53 bitop3:0x96\n"
// accumulator and second source in one bank: v8 ^= v13 ^ v16
#define AS2 "v_bitop3_b32 v8, v8, v13, v16 bitop3:0x96\n v_bitop3_b32 v20, v20, v25, v28 bitop3:0x96\n" \
            "v_bitop3_b32 v32, v32, v37, v40 bitop3:0x96\n v_bitop3_b32 v44, v44, v49, v52 bitop3:0x96\n"
// 2-input v_xor_b32 with both sources in one bank: v8 = v12 ^ v8
#define XS "v_xor_b32 v8, v12, v8\n v_xor_b32 v20, v24, v20\n v_xor_b32 v32, v36, v32\n v_xor_b32 v44, v48, v44\n"
#define XD "v_xor_b32 v8, v13, v8\n v_xor_b32 v20, v25, v20\n v_xor_b32 v32, v37, v32\n v_xor_b32 v44, v49, v44\n"

template <int MODE>
__global__ __launch_bounds__(256) void k(unsigned *out, int iters) {
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0) asm volatile(REP8(SAME) ::: "v8", "v20", "v32", "v44");
        if (MODE == 1) asm volatile(REP8(DIFF) ::: "v8", "v20", "v32", "v44");
        if (MODE == 2) asm volatile(REP8(TWO) ::: "v9", "v21", "v33", "v45");
        if (MODE == 3) asm volatile(REP8(AS1) ::: "v8", "v20", "v32", "v44");
        if (MODE == 4) asm volatile(REP8(AS2) ::: "v8", "v20", "v32", "v44");
        if (MODE == 5) asm volatile(REP8(XS) ::: "v8", "v20", "v32", "v44");
        if (MODE == 6) asm volatile(REP8(XD) ::: "v8", "v20", "v32", "v44");
    }
    unsigned r;
    asm volatile("v_mov_b32 %0, v8" : "=v"(r));
    if (r == 0x12345678u) out[threadIdx.x] = r;
}

int main() {
    unsigned *out;
    hipMalloc(&out, 4096);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int iters = 20000, blocks = 256 * 4;  // 4 workgroups of 4 waves per CU = 4 waves/SIMD
    const char *names[] = {"same bank (acc,src,src)", "different banks", "acc apart, 2 srcs same bank",
                           "acc + src1 same bank", "acc + src2 same bank", "v_xor 2 srcs same bank",
                           "v_xor 2 srcs different banks"};
    void (*ks[])(unsigned *, int) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>};
    for (int rep = 0; rep < 2; ++rep)
        for (int m = 0; m < 7; ++m) {
            hipLaunchKernelGGL(ks[m], dim3(blocks), dim3(256), 0, 0, out, iters);
            hipEventRecord(a);
            hipLaunchKernelGGL(ks[m], dim3(blocks), dim3(256), 0, 0, out, iters);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            const double wi = (double)blocks * 4 * iters * 32;  // wave-instructions
            printf("%-30s %.3f ms  %.3f wave-instr/ns\n", names[m], ms, wi / (ms * 1e6));
        }
    return 0;
}
