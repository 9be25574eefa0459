// Common scaffolding for the compile-time-scheduled kernels generated into csrc/gen/.
//
// A generated file defines `body_<name>(part, src, acc)` -- straight-line window-table XORs with
// the generator coefficients baked in -- and ends with FIXED_KERNELS(name, K, M, P), which
// instantiates the encode and decode-stage-A kernels and their launcher here.
//
// Work decomposition: lanes are flattened over (group g, word column q) exactly like the generic
// kernel (each lane runs the whole group's bitmatrix on its 32 bit-columns). A workgroup of 256
// threads holds CS = 4/P column sets of 64 lanes; its P waves per column set each produce one
// part (<= 16 rows) of the output, so the part waves read the same input words back to back
// (L1/L2 hits) instead of re-streaming them from HBM.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.hpp"

namespace sh {
namespace fixed {

#define X3(a, b, c) __builtin_amdgcn_bitop3_b32((a), (b), (c), 0x96)
// Zero-instruction pin of 8 accumulators to the current program point (see the generator).
#define PIN8(r)                                                                                    \
    asm volatile("" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]),      \
                 "+v"(r[6]), "+v"(r[7]))
#define ZERO(r) asm volatile("v_mov_b32 %0, 0" : "=v"(r))
// 2-input XOR as a bitop3 (third operand ignored): opaque to LLVM's reassociation.
#define X2(a, b) __builtin_amdgcn_bitop3_b32((a), (b), (a), 0x3C)

// What the sources need from FixedArgs, in 32-bit units (one launch's input spans < 2 GiB; the
// host splits larger batches into several launches).
struct FixedArgsView {
    const uint8_t *in;
    uint32_t in_bytes;
    uint32_t in_gstride;
    uint32_t B;
    uint32_t sub;
};

__device__ __forceinline__ uint32_t ldw(const uint8_t *p) {
    uint32_t w;
    __builtin_memcpy(&w, p, 4);
    return w;
}

__device__ __forceinline__ void stw(uint8_t *p, uint32_t w) { __builtin_memcpy(p, &w, 4); }

// Per-lane column geometry. A lane owns bytes 4q..4q+3 of every sub-block. The last word of a
// sub-block holds `tail` < 4 valid bytes when sub % 4 != 0; loading it whole over-reads into the
// next sub-block, which only pollutes bit-columns that are never stored -- harmless, except past
// the end of the whole input buffer. So only the LAST group's tail lane loads sub-block 7
// shifted back by (4 - tail) bytes and shifts the word into place (shr7).
struct Col {
    int q;
    int nbytes;     // bytes this lane stores per sub-block (1..4)
    int back7;      // bytes the sub-block-7 load is shifted back (last group's tail lane only)
};

__device__ __forceinline__ Col make_col(int g, int q, int groups, const Geometry &geo) {
    Col c;
    c.q = q;
    const bool tail = (q == geo.nq - 1) && geo.tail < 4;
    c.nbytes = tail ? geo.tail : 4;
    c.back7 = (tail && g == groups - 1) ? 4 - geo.tail : 0;
    return c;
}

// Buffer descriptor over one launch's input: raw (stride 0) buffer, `bytes` records.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const uint8_t *p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(p), static_cast<short>(0),
                                             static_cast<int>(bytes), 0x00020000);
}

__device__ __forceinline__ uint32_t bload(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0);
}

// Encode source: block x of group g = in + g*gstride + x*B. Per-lane offsets of the 8 sub-block
// words are computed once (voff[a]); the per-step block offset x*B is a scalar (soffset), so a
// step's 8 loads cost no vector ALU at all.
template <int K>
struct EncSrc {
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t voff[8];
    uint32_t voff7_last;  // sub-block 7 of the LAST block, shifted back on the buffer-end lane
    uint32_t B;
    uint32_t shr7;
    __device__ __forceinline__ void init(const FixedArgsView &v, int g, const Col &c) {
        rsrc = make_rsrc(v.in, v.in_bytes);
        B = v.B;
        const uint32_t base = static_cast<uint32_t>(g) * v.in_gstride + 4u * c.q;
#pragma unroll
        for (int a = 0; a < 8; ++a) voff[a] = base + a * v.sub;
        voff7_last = voff[7] - c.back7;
        shr7 = 8u * c.back7;
    }
    __device__ __forceinline__ void load(int x, uint32_t &d0, uint32_t &d1, uint32_t &d2,
                                         uint32_t &d3, uint32_t &d4, uint32_t &d5, uint32_t &d6,
                                         uint32_t &d7) const {
        const uint32_t s = static_cast<uint32_t>(x) * B;
        d0 = bload(rsrc, voff[0], s);
        d1 = bload(rsrc, voff[1], s);
        d2 = bload(rsrc, voff[2], s);
        d3 = bload(rsrc, voff[3], s);
        d4 = bload(rsrc, voff[4], s);
        d5 = bload(rsrc, voff[5], s);
        d6 = bload(rsrc, voff[6], s);
        d7 = bload(rsrc, x == K - 1 ? voff7_last : voff[7], s);
    }
    // Only the last block of the buffer can be over-read past its end (x == K-1).
    __device__ __forceinline__ uint32_t fix7(int x, uint32_t d7) const {
        return x == K - 1 ? d7 >> shr7 : d7;
    }
    __device__ __forceinline__ void add_row(int, uint32_t (&)[8]) const {}
};

// Decode stage-A source: original row x sits at array index pos[x] of the group's received
// blocks (pos in LDS), or is erased (0xFF): then the offset is pushed out of the buffer's range
// and the buffer load returns zeros. Per step: one LDS byte read + one multiply-add per lane;
// the sub-block offset a*sub is the scalar operand.
template <int K>
struct DecSrc {
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t base;      // g*gstride + 4q
    uint32_t soff[8];   // a*sub (uniform)
    uint32_t B;
    uint32_t shr7;
    int back7;
    const uint8_t *pos;
    __device__ __forceinline__ void init(const FixedArgsView &v, int g, const Col &c,
                                         const uint8_t *lds_pos, int kp) {
        KP_OFF = kp;
        rsrc = make_rsrc(v.in, v.in_bytes);
        B = v.B;
        base = static_cast<uint32_t>(g) * v.in_gstride + 4u * c.q;
#pragma unroll
        for (int a = 0; a < 8; ++a) soff[a] = a * v.sub;
        back7 = c.back7;
        shr7 = 8u * c.back7;
        pos = lds_pos;
    }
    __device__ __forceinline__ uint32_t block_off(int p) const {
        return p == 0xFF ? 0x80000000u : base + static_cast<uint32_t>(p) * B;
    }
    __device__ __forceinline__ void load(int x, uint32_t &d0, uint32_t &d1, uint32_t &d2,
                                         uint32_t &d3, uint32_t &d4, uint32_t &d5, uint32_t &d6,
                                         uint32_t &d7) const {
        const uint32_t o = block_off(pos[x]);
        d0 = bload(rsrc, o, soff[0]);
        d1 = bload(rsrc, o, soff[1]);
        d2 = bload(rsrc, o, soff[2]);
        d3 = bload(rsrc, o, soff[3]);
        d4 = bload(rsrc, o, soff[4]);
        d5 = bload(rsrc, o, soff[5]);
        d6 = bload(rsrc, o, soff[6]);
        d7 = bload(rsrc, o - back7, soff[7]);
    }
    __device__ __forceinline__ uint32_t fix7(int, uint32_t d7) const { return d7 >> shr7; }
    // acc ^= the received recovery block of generator row y (zeros when row y is absent).
    __device__ __forceinline__ void add_row(int y, uint32_t (&acc)[8]) const {
        const uint32_t o = block_off(pos[KP_OFF + y]);
#pragma unroll
        for (int a = 0; a < 7; ++a) acc[a] = X2(acc[a], bload(rsrc, o, soff[a]));
        acc[7] = X2(acc[7], bload(rsrc, o - back7, soff[7]) >> shr7);
    }
    int KP_OFF;
};

// Branch-free output: every lane issues a dword store, a short store and a byte store per output
// word; the ones a lane must not perform get an out-of-range offset and are dropped by the
// buffer unit. Normal lanes store the dword; a sub-block's short last word (tail = 1..3 valid
// bytes) is stored as short and/or byte. No branches -> the whole part stays one basic block,
// which keeps LLVM from sinking the accumulator updates into the epilogue.
struct Sink {
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t v_dw, v_sh, v_b8;  // per-lane offsets (or out of range)
    uint32_t b8_shr;            // byte store takes bits [b8_shr, b8_shr+8)
    uint32_t B, sub;
    bool has_tail;
    __device__ __forceinline__ void init(uint8_t *out, uint32_t out_bytes, uint32_t gstride,
                                         int g, const Col &c, const Geometry &geo) {
        rsrc = make_rsrc(out, out_bytes);
        B = geo.B;
        sub = geo.sub;
        has_tail = geo.tail < 4;
        const uint32_t base = static_cast<uint32_t>(g) * gstride + 4u * c.q;
        const uint32_t OOR = 0x80000000u;
        const bool t = c.nbytes < 4;
        v_dw = t ? OOR : base;
        v_sh = (t && c.nbytes >= 2) ? base : OOR;
        v_b8 = (t && (c.nbytes & 1)) ? base + (c.nbytes == 3 ? 2u : 0u) : OOR;
        b8_shr = c.nbytes == 3 ? 16u : 0u;
    }
    __device__ __forceinline__ void store(int y, int b, uint32_t w) const {
        const uint32_t so = static_cast<uint32_t>(y) * B + static_cast<uint32_t>(b) * sub;
        __builtin_amdgcn_raw_buffer_store_b32(w, rsrc, v_dw, so, 0);
        if (has_tail) {  // uniform
            __builtin_amdgcn_raw_buffer_store_b16(static_cast<uint16_t>(w), rsrc, v_sh, so, 0);
            __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(w >> b8_shr), rsrc, v_b8, so, 0);
        }
    }
};

}  // namespace fixed
}  // namespace sh

// Kernel + launcher for one generated (k, m). LDS: decode position tables of the groups a
// workgroup touches ([groups_per_wg][round4(K) + round4(M)] bytes).
#define FIXED_KERNELS(NAME, K, M, P, RPP)                                                            \
    namespace sh {                                                                                \
    namespace fixed {                                                                             \
    template <bool DEC>                                                                           \
    __global__ __launch_bounds__(256) void kern_##NAME(FixedArgs a) {                             \
        constexpr int CS = (P >= 4) ? 1 : 4 / P;                                                  \
        constexpr int KP = (K + 3) & ~3, MP = (M + 3) & ~3;                                       \
        extern __shared__ __attribute__((aligned(16))) uint8_t lds[];                             \
        const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);                        \
        const int lane = threadIdx.x & 63;                                                        \
        const int part = wave % P;                                                                \
        const long long col0 = static_cast<long long>(blockIdx.x) * CS * 64;                      \
        const long long col = col0 + (wave / P) * 64 + lane;                                      \
        const int g = static_cast<int>(col / a.geo.nq);                                           \
        const int q = static_cast<int>(col - static_cast<long long>(g) * a.geo.nq);               \
        const int g_first = static_cast<int>(col0 / a.geo.nq);                                    \
        if (DEC) {                                                                                \
            const int ng = a.groups_per_wg;                                                       \
            for (int i = threadIdx.x; i < ng * (KP + MP) / 4; i += blockDim.x) {                  \
                const int lg = i / ((KP + MP) / 4), w = i - lg * ((KP + MP) / 4);                 \
                const int gg = g_first + lg;                                                      \
                uint32_t v = 0xFFFFFFFFu;                                                         \
                if (gg < a.groups) {                                                              \
                    v = (w < KP / 4) ? reinterpret_cast<const uint32_t *>(a.pos + gg * (long long)KP)[w] \
                                     : reinterpret_cast<const uint32_t *>(a.rpos + gg * (long long)MP)[w - KP / 4]; \
                }                                                                                 \
                reinterpret_cast<uint32_t *>(lds)[i] = v;                                         \
            }                                                                                     \
            __syncthreads();                                                                      \
        }                                                                                         \
        if (g >= a.groups) return;                                                                \
        const Geometry geo = a.geo;                                                               \
        const Col c = make_col(g, q, a.groups, geo);                                              \
        const FixedArgsView v{a.in, static_cast<uint32_t>(a.in_bytes),                            \
                              static_cast<uint32_t>(a.in_gstride), static_cast<uint32_t>(geo.B),  \
                              static_cast<uint32_t>(geo.sub)};                                    \
        Sink sink;                                                                                \
        sink.init(a.out, static_cast<uint32_t>(a.out_bytes), static_cast<uint32_t>(a.out_gstride), \
                  g, c, geo);                                                                     \
        if (DEC) {                                                                                \
            DecSrc<K> src;                                                                        \
            src.init(v, g, c, lds + (g - g_first) * (KP + MP), KP);                               \
            run_##NAME(part, src, sink);                                                          \
        } else {                                                                                  \
            EncSrc<K> src;                                                                        \
            src.init(v, g, c);                                                                    \
            run_##NAME(part, src, sink);                                                          \
        }                                                                                         \
    }                                                                                             \
    hipError_t launch_##NAME(FixedArgs a, bool dec, hipStream_t s) {                              \
        constexpr int CS = (P >= 4) ? 1 : 4 / P;                                                  \
        a.groups_per_wg = (CS * 64 - 1) / a.geo.nq + 2;                                           \
        const long long cols = static_cast<long long>(a.groups) * a.geo.nq;                       \
        const unsigned blocks = static_cast<unsigned>((cols + CS * 64 - 1) / (CS * 64));           \
        const size_t lds = dec ? static_cast<size_t>(a.groups_per_wg) * (((K + 3) & ~3) + ((M + 3) & ~3)) : 0; \
        if (dec)                                                                                  \
            hipLaunchKernelGGL(kern_##NAME<true>, dim3(blocks), dim3(CS * P * 64), lds, s, a);    \
        else                                                                                      \
            hipLaunchKernelGGL(kern_##NAME<false>, dim3(blocks), dim3(CS * P * 64), lds, s, a);   \
        return hipGetLastError();                                                                 \
    }                                                                                             \
    }                                                                                             \
    }
