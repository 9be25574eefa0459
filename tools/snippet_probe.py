#!/usr/bin/env python3
"""Generate tools/snippet_probe.hip: throughput probe for runtime-coefficient bitmatrix products via
a table of 256 compile-time snippets reached with s_swappc_b64 (one call per coefficient).

Each snippet c computes tmp[b] = T0[lo(c*2^b)] ^ T1[hi(c*2^b)] for b = 0..7 from window tables
held in fixed VGPRs, then returns with s_setpc_b64. The kernel loops over (output j, input i)
coefficient pairs with uniform c (from memory), calls the snippet and folds tmp into acc[j].
Compared against the same loop with a compile-time coefficient (the lower bound).
"""
import os

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "snippet_probe.hip")
T0, T1, TMP = 100, 116, 132   # VGPR bases used by the snippets


def gmul2(x):
    x <<= 1
    return x ^ 0x187 if x & 0x100 else x


def snippets():
    # Emitted INSIDE a kernel (file-scope asm is dropped by HIP device compilation): the caller
    # branches over the table once; labels are made unique per kernel with a suffix.
    lines = ['#define SNIPPET_TABLE(SFX) asm volatile("s_branch sh_snip_end" #SFX "\\n"',
             '    ".p2align 6\\n"',
             '    "sh_snip_base" #SFX ":\\n"']
    for c in range(256):
        s = c
        body = []
        for b in range(8):
            lo, hi = s & 15, s >> 4
            body.append(f"v_xor_b32 v{TMP + b}, v{T0 + lo}, v{T1 + hi}")
            s = gmul2(s)
        body.append("s_setpc_b64 s[40:41]")
        # 8 x 4 B + 4 B = 36 B; pad to 64 B
        lines.append(f'    ".p2align 6\\n"')
        for ins in body:
            lines.append(f'    "{ins}\\n"')
    lines.append('    "sh_snip_end" #SFX ":\\n" ::: "memory")')
    return " \\\n".join(lines)


KERNEL = r'''
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
#define X3(a, b, c) __builtin_amdgcn_bitop3_b32((a), (b), (c), 0x96)

#define SNIP(SFX, c, t0, t1, tmp) \
    asm volatile( \
        "s_getpc_b64 s[42:43]\n" \
        "s_add_u32 s42, s42, sh_snip_base" #SFX "@rel32@lo+4\n" \
        "s_addc_u32 s43, s43, sh_snip_base" #SFX "@rel32@hi+12\n" \
        "s_lshl_b32 s44, %[cc], 6\n" \
        "s_add_u32 s42, s42, s44\n" \
        "s_addc_u32 s43, s43, 0\n" \
        "s_swappc_b64 s[40:41], s[42:43]\n" \
        : "={v[132:139]}"(tmp) \
        : [cc] "s"(c), "{v[100:115]}"(t0), "{v[116:131]}"(t1) \
        : "s40", "s41", "s42", "s43", "s44", "scc")

__device__ __forceinline__ u32x8 snip_unused(uint32_t c, const u32x16 &t0, const u32x16 &t1) {
    u32x8 tmp;
    asm volatile(
        "s_getpc_b64 s[42:43]\n"
        "s_lshl_b32 s44, %[c], 6\n"
        "s_add_u32 s42, s42, s44\n"
        "s_addc_u32 s43, s43, 0\n"
        "s_swappc_b64 s[40:41], s[42:43]\n"
        : "={v[132:139]}"(tmp)
        : [c] "s"(c), "{v[100:115]}"(t0), "{v[116:131]}"(t1)
        : "s40", "s41", "s42", "s43", "s44", "scc");
    return tmp;
}

template <bool SNIP>
__global__ __launch_bounds__(256) void k_pairs(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                               const uint32_t* __restrict__ coef, int n_in) {
    if (SNIP) SNIPPET_TABLE(P);
    u32x16 t0, t1;
    uint32_t acc[8][8];
    #pragma unroll
    for (int j = 0; j < 8; ++j)
        #pragma unroll
        for (int b = 0; b < 8; ++b) acc[j][b] = 0;
    const int lane = blockIdx.x * 256 + threadIdx.x;
    for (int i = 0; i < n_in; ++i) {
        uint32_t d[8];
        #pragma unroll
        for (int a = 0; a < 8; ++a) d[a] = in[(i & 7) * 8 * 4096 + a * 4096 + (lane & 4095)];
        t0[0] = 0; t1[0] = 0;
        t0[1] = d[0]; t0[2] = d[1]; t0[4] = d[2]; t0[8] = d[3];
        t1[1] = d[4]; t1[2] = d[5]; t1[4] = d[6]; t1[8] = d[7];
        t0[3] = t0[1] ^ t0[2]; t0[5] = t0[1] ^ t0[4]; t0[6] = t0[2] ^ t0[4]; t0[7] = t0[3] ^ t0[4];
        t0[9] = t0[1] ^ t0[8]; t0[10] = t0[2] ^ t0[8]; t0[11] = t0[3] ^ t0[8]; t0[12] = t0[4] ^ t0[8];
        t0[13] = t0[5] ^ t0[8]; t0[14] = t0[6] ^ t0[8]; t0[15] = t0[7] ^ t0[8];
        t1[3] = t1[1] ^ t1[2]; t1[5] = t1[1] ^ t1[4]; t1[6] = t1[2] ^ t1[4]; t1[7] = t1[3] ^ t1[4];
        t1[9] = t1[1] ^ t1[8]; t1[10] = t1[2] ^ t1[8]; t1[11] = t1[3] ^ t1[8]; t1[12] = t1[4] ^ t1[8];
        t1[13] = t1[5] ^ t1[8]; t1[14] = t1[6] ^ t1[8]; t1[15] = t1[7] ^ t1[8];
        #pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t c = __builtin_amdgcn_readfirstlane(coef[(i * 8 + j) & 1023]);
            if (SNIP) {
                u32x8 tmp;
                SNIP(P, c, t0, t1, tmp);
                #pragma unroll
                for (int b = 0; b < 8; ++b) acc[j][b] ^= tmp[b];
            } else {
                // compile-time coefficient stand-in: fixed nibbles (lower bound, 8 bitop3)
                #pragma unroll
                for (int b = 0; b < 8; ++b) acc[j][b] = X3(acc[j][b], t0[(b * 5 + j) & 15], t1[(b * 3 + j + 1) & 15]);
            }
        }
    }
    uint32_t r = 0;
    #pragma unroll
    for (int j = 0; j < 8; ++j)
        #pragma unroll
        for (int b = 0; b < 8; ++b) r ^= acc[j][b] * (j * 8 + b + 1);
    out[lane] = r;
}

// host reference of the snippet semantics on one lane's data
static uint8_t gm(uint8_t a, uint8_t b) { uint8_t r = 0; for (int i = 0; i < 8; ++i) { if (b & 1) r ^= a; b >>= 1; a = (a & 0x80) ? (uint8_t)((a << 1) ^ 0x87) : (uint8_t)(a << 1); } return r; }

template <class F> static float timeit(F f, int reps) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(a)); for (int i = 0; i < reps; ++i) f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms / reps;
}

__global__ void k_check(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint32_t c) {
    SNIPPET_TABLE(C);
    u32x16 t0, t1;
    uint32_t d[8];
    for (int a = 0; a < 8; ++a) d[a] = in[a * 64 + threadIdx.x];
    t0[0] = 0; t1[0] = 0;
    t0[1] = d[0]; t0[2] = d[1]; t0[4] = d[2]; t0[8] = d[3];
    t1[1] = d[4]; t1[2] = d[5]; t1[4] = d[6]; t1[8] = d[7];
    for (int h = 0; h < 2; ++h) {
        u32x16 &t = h ? t1 : t0;
        t[3] = t[1] ^ t[2]; t[5] = t[1] ^ t[4]; t[6] = t[2] ^ t[4]; t[7] = t[3] ^ t[4];
        t[9] = t[1] ^ t[8]; t[10] = t[2] ^ t[8]; t[11] = t[3] ^ t[8]; t[12] = t[4] ^ t[8];
        t[13] = t[5] ^ t[8]; t[14] = t[6] ^ t[8]; t[15] = t[7] ^ t[8];
    }
    u32x8 tmp;
    SNIP(C, __builtin_amdgcn_readfirstlane(c), t0, t1, tmp);
    for (int b = 0; b < 8; ++b) out[b * 64 + threadIdx.x] = tmp[b];
}

int main() {
    uint32_t *in, *out, *coef;
    CK(hipMalloc(&in, 8 * 8 * 4096 * 4)); CK(hipMalloc(&out, 256 * 64 * 1024 * 4)); CK(hipMalloc(&coef, 1024 * 4));
    uint32_t h[8 * 8 * 4096]; for (int i = 0; i < 8 * 8 * 4096; ++i) h[i] = (uint32_t)(i * 2654435761u);
    CK(hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice));
    uint32_t hc[1024]; for (int i = 0; i < 1024; ++i) hc[i] = (uint32_t)((i * 37 + 11) & 255) | 1;
    CK(hipMemcpy(coef, hc, sizeof hc, hipMemcpyHostToDevice));
    // correctness of the snippet semantics: bit columns against a host bitmatrix product
    int bad = 0;
    for (uint32_t c : {1u, 2u, 3u, 0x87u, 0xC3u, 0xFFu, 0x5Au}) {
        hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, in, out, c);
        uint32_t o[8 * 64]; CK(hipMemcpy(o, out, sizeof o, hipMemcpyDeviceToHost));
        for (int l = 0; l < 64; ++l) {
            uint32_t s = c;
            for (int b = 0; b < 8; ++b) {
                uint32_t e = 0;
                for (int a = 0; a < 8; ++a) if (s & (1u << a)) e ^= h[a * 64 + l];
                if (o[b * 64 + l] != e) ++bad;
                s = gm((uint8_t)s, 2);
            }
        }
    }
    printf("snippet correctness: %s (%d bad words)\n", bad ? "FAIL" : "ok", bad);
    const int blocks = 256 * 8, n_in = 256;
    const double pairs = (double)blocks * 256 * n_in * 8;  // lane-pairs
    float ms = timeit([&] { hipLaunchKernelGGL(k_pairs<false>, dim3(blocks), dim3(256), 0, 0, in, out, coef, n_in); }, 5);
    printf("compile-time pairs: %.2f G lane-pairs/s (%.3f ms)\n", pairs / ms / 1e6, ms);
    float ms2 = timeit([&] { hipLaunchKernelGGL(k_pairs<true>, dim3(blocks), dim3(256), 0, 0, in, out, coef, n_in); }, 5);
    printf("snippet pairs:      %.2f G lane-pairs/s (%.3f ms) -> %.2fx the compile-time cost\n", pairs / ms2 / 1e6, ms2, ms2 / ms);
    return bad ? 1 : 0;
}
'''

with open(OUT, "w") as f:
    f.write(snippets() + "\n" + KERNEL)
print("wrote", OUT)
