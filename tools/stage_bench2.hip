// Staging-ring microbenchmark, v2: models the generated kernels' register pressure and VALU mix.
// Per step and wave: 8 ds_read_b32, 22 "window table" bitop3 ops, then ACC accumulator updates
// (acc ^= T[i] ^ T[j]); P part-waves share each column set's ring slot. Reports input GB/s.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef __attribute__((address_space(3))) void lds_void;

struct Args {
    const uint8_t *in;
    uint32_t in_bytes, gstride, B, sub;
    int nq, groups;
    uint32_t *out;
};

#define X3(a, b, c) __builtin_amdgcn_bitop3_b32((a), (b), (c), 0x96)

template <int K, int R, int CW, int P, int ACC, int AUX, bool UNROLL = false, int SALT = 0>
__device__ __forceinline__ void body(Args a) {
    constexpr int NW = CW * P, COLS = CW * 64, ROWB = COLS * 4, SLOT = 8 * ROWB;
    constexpr int NDMA = SLOT / 1024, DPW = (NDMA + NW - 1) / NW;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int c = (wave / P) * 64 + lane;
    const long long col0 = (long long)blockIdx.x * COLS;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.in), (short)0, (int)a.in_bytes, 0x00020000);
    uint32_t db[DPW];
#pragma unroll
    for (int j = 0; j < DPW; ++j) {
        const int off = (wave * DPW + j) * 1024 + lane * 16;
        const int aa = off / ROWB, cc = (off - aa * ROWB) / 4;
        const long long colx = col0 + cc;
        const int gx = (int)(colx / a.nq), qx = (int)(colx - (long long)gx * a.nq);
        db[j] = gx < a.groups ? (uint32_t)gx * a.gstride + 4u * qx + aa * a.sub : 0x80000000u;
    }
    auto issue = [&](int x) {
        uint8_t *slot = lds + (x % R) * SLOT;
#pragma unroll
        for (int j = 0; j < DPW; ++j)
            if (wave * DPW + j < NDMA)  // uniform
                __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void *)(slot + (wave * DPW + j) * 1024), 16, db[j], (uint32_t)x * a.B, 0, AUX);
    };
#pragma unroll
    for (int x = 0; x < R - 1; ++x) issue(x);
    uint32_t acc[ACC];
#pragma unroll
    for (int i = 0; i < ACC; ++i) asm volatile("v_mov_b32 %0, 0" : "=v"(acc[i]));
#pragma unroll (UNROLL ? K : 1)
    for (int X = 0; X < K; ++X) {
        __builtin_amdgcn_sched_barrier(0);
        const bool steady = X + R - 1 < K;
        if (steady)
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((R - 2) * DPW) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        const uint8_t *p = lds + (X % R) * SLOT + c * 4;
        uint32_t d[8];
#pragma unroll
        for (int aa = 0; aa < 8; ++aa) d[aa] = *(const uint32_t *)(p + aa * ROWB);
        if (steady) issue(X + R - 1);
        uint32_t t[24];
#pragma unroll
        for (int i = 0; i < 8; ++i) t[i] = d[i];
#pragma unroll
        for (int i = 8; i < 24; ++i) t[i] = X3(t[i - 8], t[i - 7], t[(i * 5) % 8]);
#pragma unroll
        for (int i = 0; i < ACC; ++i) acc[i] = X3(acc[i], t[(i * 7 + 3 + SALT) % 24], t[(i * 11 + 5 + 3 * SALT) % 24]);
#pragma unroll
        for (int i = 0; i < ACC; i += 8)
            asm volatile("" : "+v"(acc[i]), "+v"(acc[i + 1]), "+v"(acc[i + 2]), "+v"(acc[i + 3]), "+v"(acc[i + 4]), "+v"(acc[i + 5]), "+v"(acc[i + 6]), "+v"(acc[i + 7]));
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < ACC; ++i) s ^= acc[i];
    a.out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// Per-wave independent ring: every wave DMAs its own copy of its 64 columns (2 KB per step), waits
// only on its own vmcnt, no workgroup barrier. P waves of a column set read the same HBM lines
// (L2 hits after the first).
template <int K, int R, int P, int ACC, bool DISTINCT>
__device__ __forceinline__ void body_indep(Args a, int salt) {
    constexpr int SLOT = 2048, NDMA = 2;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int cw = wave / P;
    uint8_t *ring = lds + wave * R * SLOT;
    const long long col0 = (long long)blockIdx.x * (blockDim.x / 64 / P) * 64 + cw * 64;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.in), (short)0, (int)a.in_bytes, 0x00020000);
    uint32_t db[NDMA];
#pragma unroll
    for (int j = 0; j < NDMA; ++j) {
        const int off = j * 1024 + lane * 16;
        const int aa = off / 256, cc = (off - aa * 256) / 4;
        const long long colx = col0 + cc;
        const int gx = (int)(colx / a.nq), qx = (int)(colx - (long long)gx * a.nq);
        db[j] = gx < a.groups ? (uint32_t)gx * a.gstride + 4u * qx + aa * a.sub : 0x80000000u;
    }
    auto issue = [&](int x) {
        uint8_t *slot = ring + (x % R) * SLOT;
#pragma unroll
        for (int j = 0; j < NDMA; ++j)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void *)(slot + j * 1024), 16, db[j], (uint32_t)x * a.B, 0, 0);
    };
#pragma unroll
    for (int x = 0; x < R - 1; ++x) issue(x);
    uint32_t acc[ACC];
#pragma unroll
    for (int i = 0; i < ACC; ++i) asm volatile("v_mov_b32 %0, 0" : "=v"(acc[i]));
    for (int X = 0; X < K; ++X) {
        __builtin_amdgcn_sched_barrier(0);
        const bool steady = X + R - 1 < K;
        if (steady)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"((R - 2) * NDMA) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint8_t *p = ring + (X % R) * SLOT + lane * 4;
        uint32_t d[8];
#pragma unroll
        for (int aa = 0; aa < 8; ++aa) d[aa] = *(const uint32_t *)(p + aa * 256);
        if (steady) issue(X + R - 1);
        uint32_t t[24];
#pragma unroll
        for (int i = 0; i < 8; ++i) t[i] = d[i];
#pragma unroll
        for (int i = 8; i < 24; ++i) t[i] = X3(t[i - 8], t[i - 7], t[(i * 5) % 8]);
#pragma unroll
        for (int i = 0; i < ACC; ++i) acc[i] = X3(acc[i], t[(i * 7 + 3 + salt) % 24], t[(i * 11 + 5) % 24]);
#pragma unroll
        for (int i = 0; i < ACC; i += 8)
            asm volatile("" : "+v"(acc[i]), "+v"(acc[i + 1]), "+v"(acc[i + 2]), "+v"(acc[i + 3]), "+v"(acc[i + 4]), "+v"(acc[i + 5]), "+v"(acc[i + 6]), "+v"(acc[i + 7]));
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < ACC; ++i) s ^= acc[i];
    a.out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ __launch_bounds__(256, 4) void k_ind_c1_p4_r4(Args a) { body_indep<200, 4, 4, 64, false>(a, 0); }
__global__ __launch_bounds__(256, 4) void k_ind_c1_p4_r3(Args a) { body_indep<200, 3, 4, 64, false>(a, 0); }
__global__ __launch_bounds__(512, 4) void k_ind_c2_p4_r4(Args a) { body_indep<200, 4, 4, 64, false>(a, 0); }

#define KERN(NAME, R, CW, P, ACC, AUX, MINW) \
    __global__ __launch_bounds__(64 * CW * P, MINW) void NAME(Args a) { body<200, R, CW, P, ACC, AUX>(a); }
KERN(k_r8_c2_p2_a128, 8, 2, 2, 128, 0, 2)
KERN(k_r8_c2_p2_a128_nt, 8, 2, 2, 128, 2, 2)
KERN(k_r8_c1_p2_a128, 8, 1, 2, 128, 0, 2)
KERN(k_r16_c1_p2_a128, 16, 1, 2, 128, 0, 2)
KERN(k_r8_c2_p3_a88, 8, 2, 3, 88, 0, 3)
KERN(k_r8_c1_p3_a88, 8, 1, 3, 88, 0, 3)
KERN(k_r8_c1_p4_a64, 8, 1, 4, 64, 0, 4)
KERN(k_r8_c2_p4_a64, 8, 2, 4, 64, 0, 4)
KERN(k_r8_c4_p1_a128, 8, 4, 1, 128, 0, 2)
__global__ __launch_bounds__(256, 4) void k_unr_c1_p4_a64(Args a) { body<200, 8, 1, 4, 64, 0, true>(a); }
__global__ __launch_bounds__(256, 4) void k_unr4_c1_p4_a64(Args a) {
    const int part = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) % 4;
    if (part == 0) body<200, 8, 1, 4, 64, 0, true, 0>(a);
    else if (part == 1) body<200, 8, 1, 4, 64, 0, true, 1>(a);
    else if (part == 2) body<200, 8, 1, 4, 64, 0, true, 2>(a);
    else body<200, 8, 1, 4, 64, 0, true, 3>(a);
}
__global__ __launch_bounds__(1024, 4) void k_unr_c4_p4_a64(Args a) { body<200, 8, 4, 4, 64, 0, true>(a); }
__global__ __launch_bounds__(1024, 4) void k_c4_p4_a64(Args a) { body<200, 8, 4, 4, 64, 0, false>(a); }

template <class F>
static float timeit(F f, int iters) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / iters;
}

static void run(const char *name, int R, int CW, int P, int ACC, Args a, double bytes, void (*kern)(Args),
                size_t lds_pad = 0) {
    const int COLS = CW * 64;
    const long long cols = (long long)a.groups * a.nq;
    const unsigned blocks = (unsigned)((cols + COLS - 1) / COLS);
    const size_t lds = std::max((size_t)R * 8 * COLS * 4, lds_pad);
    float ms = timeit([&] { hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * CW * P), lds, 0, a); }, 5);
    CK(hipGetLastError());
    const double valu = (double)blocks * CW * 200 * P * (16 + ACC) ;  // wave-instr
    printf("%-24s R=%2d CW=%d P=%d ACC=%3d: %8.1f us %7.1f GB/s in; VALU %.1f G wave-inst/s\n", name, R, CW, P, ACC,
           ms * 1e3, bytes / ms / 1e6, valu / ms / 1e6);
}

int main() {
    const int G = 7600, K = 200;
    const int B = 1400;
    Args a;
    a.B = B;
    a.sub = B / 8;
    a.nq = (a.sub + 3) / 4;
    a.groups = G;
    a.gstride = K * B;
    const size_t n = (size_t)G * K * B;
    a.in_bytes = (uint32_t)n;
    uint8_t *d;
    CK(hipMalloc(&d, n));
    CK(hipMemset(d, 0x5a, n));
    a.in = d;
    CK(hipMalloc(&a.out, (size_t)G * 64 * 4 * 16));
    const double bytes = (double)n;
    printf("== B=%d, %d groups x k=%d: %.2f GB input\n", B, G, K, bytes / 1e9);
    run("c2 p2 a128", 8, 2, 2, 128, a, bytes, k_r8_c2_p2_a128);
    run("c2 p2 a128 nt", 8, 2, 2, 128, a, bytes, k_r8_c2_p2_a128_nt);
    run("c1 p2 a128", 8, 1, 2, 128, a, bytes, k_r8_c1_p2_a128);
    run("c1 p2 a128 R16", 16, 1, 2, 128, a, bytes, k_r16_c1_p2_a128);
    run("c2 p3 a88", 8, 2, 3, 88, a, bytes, k_r8_c2_p3_a88);
    run("c1 p3 a88", 8, 1, 3, 88, a, bytes, k_r8_c1_p3_a88);
    run("c1 p4 a64", 8, 1, 4, 64, a, bytes, k_r8_c1_p4_a64);
    run("c1 p4 a64 occ4 (LDS pad)", 8, 1, 4, 64, a, bytes, k_r8_c1_p4_a64, 40 * 1024);
    run("c1 p4 a64 occ3 (LDS pad)", 8, 1, 4, 64, a, bytes, k_r8_c1_p4_a64, 53 * 1024);
    run("c2 p4 a64", 8, 2, 4, 64, a, bytes, k_r8_c2_p4_a64);
    run("c4 p1 a128 (half rows)", 8, 4, 1, 128, a, bytes, k_r8_c4_p1_a128);
    run("c1 p4 a64 UNROLLED", 8, 1, 4, 64, a, bytes, k_unr_c1_p4_a64);
    run("c4 p4 a64 UNROLLED", 8, 4, 4, 64, a, bytes, k_unr_c4_p4_a64);
    run("c1 p4 a64 UNROLLED distinct", 8, 1, 4, 64, a, bytes, k_unr4_c1_p4_a64);
    run("c4 p4 a64 loop", 8, 4, 4, 64, a, bytes, k_c4_p4_a64);
    {
        auto run_ind = [&](const char *name, int R, int CW, void (*kern)(Args)) {
            const int COLS = CW * 64;
            const long long cols = (long long)a.groups * a.nq;
            const unsigned blocks = (unsigned)((cols + COLS - 1) / COLS);
            const size_t lds = (size_t)CW * 4 * R * 2048;
            float ms = timeit([&] { hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * CW * 4), lds, 0, a); }, 5);
            CK(hipGetLastError());
            printf("%-24s R=%2d CW=%d P=4 ACC= 64 indep: %8.1f us %7.1f GB/s in\n", name, R, CW, ms * 1e3, bytes / ms / 1e6);
        };
        run_ind("indep c1 p4 r4", 4, 1, k_ind_c1_p4_r4);
        run_ind("indep c1 p4 r3", 3, 1, k_ind_c1_p4_r3);
        run_ind("indep c2 p4 r4", 4, 2, k_ind_c2_p4_r4);
    }
    return 0;
}
