// Microbenchmark of the LDS-DMA staging ring used by the compile-time kernels (fixed_common.hpp):
// same geometry (groups x nq word columns, 8 sub-blocks, K input blocks per group), same per-step
// protocol (counted vmcnt + s_barrier, ds_read x8, DMA of step x+R-1), with a synthetic VALU load
// of V bitop3 per step instead of the generated schedule. Reports input GB/s.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef __attribute__((address_space(3))) void lds_void;

struct Args {
    const uint8_t *in;
    uint32_t in_bytes, gstride, B, sub;
    int nq, groups;
    uint32_t *out;
};

template <int K, int R, int CW, int P, int V, int W>
__device__ __forceinline__ void stage_body(Args a) {
    constexpr int NW = CW * P, COLS = CW * 64, ROWB = COLS * 4, SLOT = 8 * ROWB;
    constexpr int NDMA = SLOT / (64 * W), DPW = NDMA / NW;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int c = (wave / P) * 64 + lane;
    const long long col0 = (long long)blockIdx.x * COLS;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.in), (short)0, (int)a.in_bytes, 0x00020000);
    uint32_t db[DPW];
#pragma unroll
    for (int j = 0; j < DPW; ++j) {
        const int off = (wave * DPW + j) * 64 * W + lane * W;
        const int aa = off / ROWB, cc = (off - aa * ROWB) / 4;
        const long long colx = col0 + cc;
        const int gx = (int)(colx / a.nq), qx = (int)(colx - (long long)gx * a.nq);
        db[j] = gx < a.groups ? (uint32_t)gx * a.gstride + 4u * qx + aa * a.sub : 0x80000000u;
    }
    auto issue = [&](int x) {
        uint8_t *slot = lds + (x % R) * SLOT;
#pragma unroll
        for (int j = 0; j < DPW; ++j)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void *)(slot + (wave * DPW + j) * 64 * W), W, db[j], (uint32_t)x * a.B, 0, 0);
    };
#pragma unroll
    for (int x = 0; x < R - 1; ++x) issue(x);
    uint32_t acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) asm volatile("v_mov_b32 %0, 0" : "=v"(acc[i]));
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
#pragma unroll
        for (int v = 0; v < V; ++v)
            acc[v & 15] = __builtin_amdgcn_bitop3_b32(acc[v & 15], d[v & 7], d[(v + 3) & 7], 0x96);
        asm volatile("" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]), "+v"(acc[6]), "+v"(acc[7]));
        asm volatile("" : "+v"(acc[8]), "+v"(acc[9]), "+v"(acc[10]), "+v"(acc[11]), "+v"(acc[12]), "+v"(acc[13]), "+v"(acc[14]), "+v"(acc[15]));
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s ^= acc[i];
    a.out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

#define STAGE_KERNEL(NAME, R, CW, P, V) \
    __global__ __launch_bounds__(64 * CW * P, 2) void NAME(Args a) { stage_body<200, R, CW, P, V, 16>(a); }
STAGE_KERNEL(k_s8_2_2_0, 8, 2, 2, 0)
STAGE_KERNEL(k_s8_2_2_150, 8, 2, 2, 150)
STAGE_KERNEL(k_s4_2_2_150, 4, 2, 2, 150)
STAGE_KERNEL(k_s12_2_2_150, 12, 2, 2, 150)
STAGE_KERNEL(k_s8_4_1_150, 8, 4, 1, 150)
STAGE_KERNEL(k_s8_2_2_75, 8, 2, 2, 75)

// Same work with direct dword loads (no LDS), prefetch 2 steps: the previous kernel design.
template <int K, int V>
__device__ __forceinline__ void direct_body(Args a) {
    const long long col = (long long)blockIdx.x * 128 + ((threadIdx.x >> 6) / 2) * 64 + (threadIdx.x & 63);
    const int g = (int)(col / a.nq), q = (int)(col - (long long)g * a.nq);
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.in), (short)0, (int)a.in_bytes, 0x00020000);
    const uint32_t base = g < a.groups ? (uint32_t)g * a.gstride + 4u * q : 0x80000000u;
    uint32_t acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) asm volatile("v_mov_b32 %0, 0" : "=v"(acc[i]));
    uint32_t d[8];
    for (int x = 0; x < K; ++x) {
#pragma unroll
        for (int aa = 0; aa < 8; ++aa) d[aa] = __builtin_amdgcn_raw_buffer_load_b32(r, base + aa * a.sub, (uint32_t)x * a.B, 0);
#pragma unroll
        for (int v = 0; v < V; ++v)
            acc[v & 15] = __builtin_amdgcn_bitop3_b32(acc[v & 15], d[v & 7], d[(v + 3) & 7], 0x96);
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s ^= acc[i];
    a.out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256, 2) void k_direct150(Args a) { direct_body<200, 150>(a); }
__global__ __launch_bounds__(256, 2) void k_direct0(Args a) { direct_body<200, 0>(a); }

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

template <int R, int CW, int P, int V>
static void run_stage(const char *name, Args a, double bytes, void (*kern)(Args)) {
    constexpr int COLS = CW * 64;
    const long long cols = (long long)a.groups * a.nq;
    const unsigned blocks = (unsigned)((cols + COLS - 1) / COLS);
    const size_t lds = (size_t)R * 8 * COLS * 4;
    float ms = timeit([&] { hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * CW * P), lds, 0, a); }, 5);
    CK(hipGetLastError());
    printf("%-40s R=%2d CW=%d P=%d V=%3d: %8.1f us  %7.1f GB/s input\n", name, R, CW, P, V, ms * 1e3, bytes / ms / 1e6);
}

int main() {
    const int G = 7600, K = 200;
    for (int B : {1400, 1408}) {
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
        CK(hipMalloc(&a.out, (size_t)G * 64 * 4 * 4));
        const double bytes = (double)n;
        printf("== B=%d (sub %d, nq %d), %d groups x k=%d: %.2f GB input\n", B, a.sub, a.nq, G, K, bytes / 1e9);
        run_stage<8, 2, 2, 0>("stage ring, no VALU", a, bytes, k_s8_2_2_0);
        run_stage<8, 2, 2, 150>("stage ring, 150 VALU/step", a, bytes, k_s8_2_2_150);
        run_stage<4, 2, 2, 150>("stage ring, 150 VALU/step", a, bytes, k_s4_2_2_150);
        run_stage<12, 2, 2, 150>("stage ring, 150 VALU/step", a, bytes, k_s12_2_2_150);
        run_stage<8, 4, 1, 150>("stage ring CW4 P1 (4 col waves)", a, bytes, k_s8_4_1_150);
        run_stage<8, 2, 2, 75>("stage ring, 75 VALU/step", a, bytes, k_s8_2_2_75);
        {
            const long long cols = (long long)a.groups * a.nq;
            const unsigned blocks = (unsigned)((cols + 127) / 128);
            float ms = timeit([&] { hipLaunchKernelGGL(k_direct150, dim3(blocks), dim3(256), 0, 0, a); }, 5);
            printf("%-40s %8.1f us  %7.1f GB/s input (x2 parts read)\n", "direct dword loads, 150 VALU", ms * 1e3, bytes / ms / 1e6);
            ms = timeit([&] { hipLaunchKernelGGL(k_direct0, dim3(blocks), dim3(256), 0, 0, a); }, 5);
            printf("%-40s %8.1f us  %7.1f GB/s input (x2 parts read)\n", "direct dword loads, no VALU", ms * 1e3, bytes / ms / 1e6);
        }
        CK(hipFree(d));
        CK(hipFree(a.out));
    }
    return 0;
}
