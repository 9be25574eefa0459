// Common scaffolding for the compile-time-scheduled kernels generated into csrc/gen/.
//
// A generated file (fixed_<name>.inc) defines `run_<name>_p<p>(src, sink)` -- straight-line
// window-table XORs with the generator coefficients baked in, one step per input block -- and
// fixed_<name>_{enc,dec}.hip instantiate one kernel each through FIXED_KERNEL below.
//
// Work decomposition. Lanes are flattened over (group g, word column q): a lane owns bytes
// 4q..4q+3 of all 8 sub-blocks of a group ("bitsliced": each bit position is an independent
// column of the bitmatrix product). A workgroup covers COLS = CW*64 consecutive columns with
// CW column-waves x P part-waves; part p produces output rows [p*rows, (p+1)*rows). The CW waves
// of one part execute the same straight-line code in lockstep, sharing instruction fetch.
//
// Input staging (LDS ring, filled by LDS-DMA). Input block x of all the workgroup's columns is
// one ring slot laid out [sub-block a][column c] (words), so a lane's 8 words of step x are 8
// conflict-free ds_read_b32 at compile-time offsets. The slot is filled by `buffer_load_dwordx4
// ... lds`: per-lane global source addresses gather each sub-block's (at B=1400: 175-byte) span
// into the aligned LDS image, so misalignment costs nothing in the compute loop. Measured on
// gfx950 (tools/dma_probe.hip): misaligned LDS-DMA sources are exact; a dword straddling the
// buffer's num_records reads as 0.
//
// Pipeline (R slots, a workgroup barrier every S blocks). Iteration x issues the ds_reads of
// block x+1 into the second register set and computes block x from the registers read one
// iteration earlier (LDS latency under the compute). Before reading the first block of each
// group of S, a wave waits (counted vmcnt) for its DMAs of the whole group and joins the barrier
// -- every wave's share of those slots has landed, and every wave is past block x-1, so the
// slots of blocks <= x-1 are free and their DMAs (blocks up to x+R-1) are issued right there.
// R >= 2S+1 keeps R-2S-1 blocks of DMA in flight beyond the group being waited for. Fewer
// barriers matter: measured per-wave stamps (round 1) showed 41 % of a wave's life at the barrier
// with S = 1; S = 4 is 6-8 % faster. All P part-waves read the same slots:
// HBM sees each input byte once.
//
// Sub-block tails. When sub = B/8 is not a multiple of 4 (175 at B = 1400) the last 4-column
// chunk of every sub-block is shifted back by shift = 4*nq - sub bytes, on input (DMA source)
// and output (store offset) alike: its 4 lanes compute bytes [sub-16, sub) instead of
// [4nq-16, 4nq). Every word a lane computes is then a real column, every store is a plain dword
// store, nothing reads or writes past a sub-block, and the first shift bytes of the chunk are
// written twice with identical values (also by the column before it).
//
// Addressing. Buffer descriptors are built per workgroup with the base at the workgroup's first
// group, so 32-bit offsets cover any batch (no 2 GiB launch split); num_records stops at the end
// of the batch.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "geometry.hpp"
#include "measure.hpp"

#include <algorithm>
#include <type_traits>

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
// acc ^= t as a 4-byte VOP2 v_xor_b32 (half the bytes of a bitop3: the straight-line schedules
// are instruction-fetch heavy); a non-volatile asm is opaque to reassociation yet schedulable.
#define XV(acc, t) asm("v_xor_b32 %0, %1, %2" : "=v"(acc) : "v"(t), "v"(acc))

// Cache policy of the output stores and of the input DMA (aux operand of the buffer op).
#ifndef SH_STORE_AUX
#define SH_STORE_AUX 0
#endif
#ifndef SH_LOAD_AUX
#define SH_LOAD_AUX 0
#endif

typedef __attribute__((address_space(3))) void lds_void;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32_ua __attribute__((aligned(1)));  // byte-aligned dword (LDS reads it unaligned)
constexpr uint32_t OOR = 0x80000000u;  // buffer offset past every descriptor's range (< 2 GiB)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const uint8_t *p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(p), static_cast<short>(0),
                                             static_cast<int>(bytes), 0x00020000);
}

__device__ __forceinline__ uint32_t bload(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0);
}

// Descriptor over [base + first*gstride, base + total) capped below 2 GiB.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wg_rsrc(const uint8_t *base, long long total,
                                                          long long gstride, int first) {
    const long long start = static_cast<long long>(first) * gstride;
    long long n = total - start;
    n = n < 0 ? 0 : (n > 0x7FFFFFFFll ? 0x7FFFFFFFll : n);
    return make_rsrc(base + start, static_cast<uint32_t>(n));
}

// XCD-aware tile order. Workgroups are dealt round-robin over the 8 XCDs (block b -> XCD b % 8;
// a speed assumption, never a correctness one). Adjacent column tiles usually split a group, so
// both read the same 128-byte lines at their shared edge; giving them blocks b and b + 8 puts
// them on one XCD at about the same time, and the second read hits that XCD's L2 instead of
// going to HBM again (measured: 29% over-fetch on the staging microbenchmark without it; a
// persistent variant that walked each workgroup's own group range tile by tile re-read those
// lines from memory: +30% FETCH_SIZE, 0.94 vs 0.75 ms, round 2). Bijective map of block b in
// [0, n) to a tile: XCD i gets the contiguous tile range [start_i, start_i + count_i),
// count_i = n/8 (+1 for the first n%8 XCDs).
__device__ __forceinline__ int xcd_tile(int b, int n) {
    const int q = n >> 3, r = n & 7;
    const int x = b & 7, i = b >> 3;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// Compile-time shape of one kernel instance.
// DMA_ = false only in measurement builds (tools/gen_fixed_kernels.py SH_GEN_ABLATE=nodma).
// PW_ = parts per workgroup (default all P): with PW < P the P parts of a tile run in H = P / PW
// workgroups, each reading the whole tile through its own ring (generator switch SH_PW, A/B
// builds: fewer code streams per workgroup for H times the input reads).
// SLOTB_ > 0: ring slots of that many bytes instead of one row image (BlkSrc's whole-block slots).
template <int K_, int M_, int P_, int CW_, int R_, bool DMA_ = true, int PW_ = P_, int SLOTB_ = 0>
struct Shape {
    static constexpr int K = K_, M = M_, P = P_, CW = CW_, R = R_, W = 16;
    static constexpr int PW = PW_, H = P_ / PW_;
    static_assert(PW_ >= 1 && P_ % PW_ == 0, "parts per workgroup");
    static constexpr bool DMA = DMA_;
    static constexpr int NW = CW * PW, NT = 64 * NW, COLS = CW * 64;
    static constexpr int ROWB = COLS * 4;               // bytes of one sub-block row of a slot
    static constexpr int IMG = 8 * ROWB;                // bytes of one epilogue row image
    static constexpr int SLOT = SLOTB_ > 0 ? SLOTB_ : IMG;  // bytes per ring slot (one input block)
    static constexpr int NDMA = SLOT / (64 * W);        // DMA wave-instructions per step
    static constexpr int DPW = (NDMA + NW - 1) / NW;    // ... issued by each wave (at most)
    static constexpr int KP = (K + 3) & ~3, MP = (M + 3) & ~3;
    // <= 64 KB: two workgroups per CU, and ds_read's 16-bit offsets reach every slot; the 16-wave
    // shapes (one workgroup per CU) take 128 KB (slot offsets past 64 KB cost an address add)
    static_assert(R >= 3 && R * SLOT <= 131072, "ring size");
};

// Per-lane geometry shared by the source and the sink.
struct WGInfo {
    long long col0;  // first column of the tile (may precede lo: the first tile of odd workgroups)
    long long lo, hi;  // this workgroup's columns [lo, hi): whole groups
    int g_first;     // group of max(col0, lo) (descriptor base)
    int wave, lane, c;
    int gl, q;       // this lane's group (relative to g_first) and word column
    bool valid;      // g < groups
};

// Input side. DMA instruction i = wave*DPW + j covers slot bytes [i*1024, (i+1)*1024): lane byte
// `off` -> sub-block a = off / ROWB, first column cc = (off % ROWB) / 4, a 4-column chunk that
// lies in one group because nq % 4 == 0 (has_fixed).
// Byte offset of word column q inside a sub-block (the last chunk shifted back, see above).
__device__ __forceinline__ uint32_t col_off(int q, const Geometry &geo) {
    return 4u * q - (q >= geo.nq - 4 ? static_cast<uint32_t>(4 * geo.nq - geo.sub) : 0u);
}

// Per-lane geometry of the tile starting at column col0.
template <class S>
__device__ __forceinline__ WGInfo tile_info(int nq, long long col0, long long lo, long long hi) {
    WGInfo w;
    w.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    w.lane = threadIdx.x & 63;
    const int cw = w.wave / S::PW;
    w.c = cw * 64 + w.lane;
    w.col0 = col0;
    w.lo = lo;
    w.hi = hi;
    w.g_first = static_cast<int>((col0 > lo ? col0 : lo) / nq);
    const long long col = w.col0 + w.c;
    w.valid = col >= lo && col < hi;
    const int g = w.valid ? static_cast<int>(col / nq) : w.g_first;
    w.q = static_cast<int>(col - static_cast<long long>(g) * nq);
    w.gl = g - w.g_first;
    return w;
}

template <class S, bool DEC>
struct Src {
    static constexpr bool kStream = false, kBlk = false;
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t dbase[S::DPW];   // chunk source offset, block 0 / array slot 0 (OOR past the batch)
    int dgl[S::DPW];          // decode: the chunk's group (position-table index)
    uint32_t B, sub;
    int wave;
    uint32_t rd;              // this lane's read offset in a slot (c * 4)
    const uint8_t *lds;       // ring base
    const uint8_t *pos;       // decode: [groups_per_wg][KP + MP] position tables (LDS)
    // Persistent workgroups (encode): the next tile's source, whether there is one, and whether
    // this tile's first NPF steps were already issued by the previous tile (`pref`).
    __amdgpu_buffer_rsrc_t nrsrc;
    uint32_t ndbase[S::DPW];
    bool has_next = false, pref = false;
    // uniform state (few SGPRs: the rest derives from k, B and the group count) to set up the
    // next tile at the end of this one, so no per-lane state of the next tile is live across the
    // body
    const uint8_t *in_ptr;
    long long next_col0;
    int nq, groups;
    const uint8_t *pos_g, *rpos_g;  // decode: the position tables in HBM (the next tile's are
                                    // staged into the LDS copy at this tile's end)
    uint32_t lbase;           // decode: this lane's column in its group (OOR: past the batch)
    int lgl;                  // ... and its group (position-table index)
    // encode: byte offset of step 0's block (the second half of a split tile starts at block x0)
    mutable uint32_t boff = 0;
    mutable int x0s = 0;
    __device__ __forceinline__ void set_step0(int x0) const {
        boff = static_cast<uint32_t>(x0) * B;
        x0s = x0;
    }
    int pf_stride = 0;        // FixedArgs::pf_stride (l2_prefetch)
    int krt = S::K;           // encode: steps x >= krt (FixedArgs::k_rt) read zeros

    __device__ __forceinline__ static void chunk_src(const Geometry &geo, long long in_gstride_, const WGInfo &w,
                                                     uint32_t (&db)[S::DPW], int (&gl)[S::DPW]) {
        const uint32_t gstride = static_cast<uint32_t>(in_gstride_);
#pragma unroll
        for (int j = 0; j < S::DPW; ++j) {
            const int off = (w.wave * S::DPW + j) * 64 * S::W + w.lane * S::W;
            const int aa = off / S::ROWB;
            const int cc = (off - aa * S::ROWB) / 4;
            const long long colx = w.col0 + cc;
            const int gx = colx >= 0 ? static_cast<int>(colx / geo.nq) : -1;
            const int qx = static_cast<int>(colx - static_cast<long long>(gx) * geo.nq);
            gl[j] = gx - w.g_first;
            db[j] = (colx >= w.lo && colx < w.hi)
                        ? static_cast<uint32_t>(gx - w.g_first) * gstride + col_off(qx, geo) + aa * geo.sub
                        : OOR;
        }
    }

    __device__ __forceinline__ void init(const FixedArgs &a, const WGInfo &w, const uint8_t *lds_ring,
                                         const uint8_t *lds_pos) {
        const Geometry &geo = a.geo;
        rsrc = wg_rsrc(a.in, a.in_bytes, a.in_gstride, w.g_first);
        B = geo.B;
        sub = geo.sub;
        lds = lds_ring;
        pos = lds_pos;
        wave = w.wave;
        rd = static_cast<uint32_t>(w.c) * 4u;
        chunk_src(a.geo, a.in_gstride, w, dbase, dgl);
        in_ptr = a.in;
        nq = geo.nq;
        groups = a.groups;
        pos_g = a.pos;
        rpos_g = a.rpos;
        lgl = w.gl;
        pf_stride = a.pf_stride;
        krt = a.k_rt > 0 ? a.k_rt : S::K;
        lbase = w.valid ? static_cast<uint32_t>(w.gl) * static_cast<uint32_t>(a.in_gstride) + col_off(w.q, geo) : OOR;
    }

    // Decode, generator switch SH_RINIT=1 (not the default: same time, more fetched bytes):
    // residual row y starts as the received recovery block R_y (position entry KP + y; absent:
    // zeros), loaded straight into the lane's 8 accumulators before the ring's first DMA, so
    // stage A runs the k input steps only. Older than every DMA, these loads are covered by the
    // ring's counted waits; the compiler's own wait guards the use.
    __device__ __forceinline__ void rrow(int y, uint32_t (&r)[8]) const {
        const int p = pos[lgl * (S::KP + S::MP) + S::KP + y];
        const uint32_t o = (p == 0xFF || lbase == OOR) ? OOR : lbase + static_cast<uint32_t>(p) * B;
#pragma unroll
        for (int s = 0; s < 8; ++s) r[s] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, o + s * sub, 0, SH_LOAD_AUX);
    }

    __device__ __forceinline__ void advance() {
        rsrc = nrsrc;
#pragma unroll
        for (int j = 0; j < S::DPW; ++j) dbase[j] = ndbase[j];
        pref = true;
    }

    // Wait until this wave's DMAs of steps <= T are done (I = steps issued so far), then join the
    // workgroup barrier. One asm statement: nothing is scheduled between the two. Waves that
    // issue no DMA (NDMA < NW) only join the barrier: their vmcnt holds nothing but output
    // stores, which nothing here needs to wait for. EX: vector-memory ops issued between the DMA
    // of step T and the later ones when this tile's first steps were prefetched (the previous
    // tile's epilogue stores, issued after its prefetch of steps < NPF): vmcnt counts them too.
    template <int T, int I, int EX = 0>
    __device__ __forceinline__ void wait() const {
        constexpr int N = (I - T - 1) * S::DPW;
        static_assert(N >= 0 && N + EX < 64, "vmcnt is 6 bits");
        if (S::NDMA % S::NW != 0 && wave * S::DPW >= S::NDMA)
            asm volatile("s_barrier" ::: "memory");
        else if (EX != 0 && pref)
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N + EX) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
    }

    // Persistent encode, right after the last step's ring reads (release()): the next tile's
    // steps 0..NP-1 into slots 0..NP-1 (free: every wave is past this tile's steps; the row
    // images of the epilogue use the ring's top 2P slots), so their HBM latency runs under this
    // tile's epilogue stores.
    // Decode: the next tile's steps read their DMA sources through its position tables, staged
    // into the LDS copy first (the current tile's are dead once its last step is read). Nothing
    // else is outstanding in vmcnt here (the last ring wait was vmcnt(0), the stores come later),
    // so waiting for these loads costs one load latency, still under the epilogue.
    __device__ __forceinline__ void stage_pos(int g_first) const {
        const int ghi = groups;
        const int ngwg = (S::COLS - 1) / nq + 2;  // FixedArgs::groups_per_wg (launch_shape)
        constexpr int TW = (S::KP + S::MP) / 4;
        for (int i = threadIdx.x; i < ngwg * TW; i += S::NT) {  // one or two dwords per thread
            const int lg = i / TW, t = i - lg * TW;
            const int gg = g_first + lg;
            uint32_t v = 0xFFFFFFFFu;
            if (gg < ghi)
                v = (t < S::KP / 4)
                        ? reinterpret_cast<const uint32_t *>(pos_g + gg * static_cast<long long>(S::KP))[t]
                        : reinterpret_cast<const uint32_t *>(rpos_g + gg * static_cast<long long>(S::MP))[t - S::KP / 4];
            reinterpret_cast<uint32_t *>(const_cast<uint8_t *>(pos))[i] = v;
        }
        __syncthreads();
    }

    __device__ __forceinline__ void prefetch_next(int np) const {
        if (!has_next) return;
        auto *self = const_cast<Src *>(this);
        {  // the next tile's source, computed here: nothing of it is live across the body
            const long long gstride = static_cast<long long>(S::K) * B;
            const WGInfo w = tile_info<S>(nq, next_col0, 0, static_cast<long long>(groups) * nq);
            self->nrsrc = wg_rsrc(in_ptr, gstride * groups, gstride, w.g_first);
            Geometry g;
            g.B = static_cast<int>(B);
            g.sub = static_cast<int>(sub);
            g.nq = nq;
            g.tail = 4;
            chunk_src(g, gstride, w, self->ndbase, self->dgl);
            if (DEC) stage_pos(w.g_first);
        }
#pragma unroll
        for (int t = 0; t < np; ++t) {
            uint8_t *slot = const_cast<uint8_t *>(lds) + (t % S::R) * S::SLOT;
            const Pre pr = pre(t);
#pragma unroll
            for (int j = 0; j < S::DPW; ++j) {
                if (S::NDMA % S::NW != 0 && wave * S::DPW + j >= S::NDMA) break;  // uniform
                lds_void *dst = (lds_void *)(slot + (wave * S::DPW + j) * 64 * S::W);
                if (DEC) {
                    const int p = pr.p[j];
                    const uint32_t o = (p == 0xFF || ndbase[j] == OOR) ? OOR : ndbase[j] + static_cast<uint32_t>(p) * B;
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(nrsrc, dst, S::W, o, 0, 0, SH_LOAD_AUX);
                } else {
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(nrsrc, dst, S::W, t < krt ? ndbase[j] : OOR,
                                                             static_cast<uint32_t>(t) * B, 0, SH_LOAD_AUX);
                }
            }
        }
    }

    // Encode, generator switch SH_L2PF=N (A/B): at the start of the epilogue, touch the first N
    // steps of the tile that workgroup blockIdx.x + pf_stride codes (the one about to take a slot
    // on this XCD when every workgroup takes as long: pf_stride = the launch's slots) with plain
    // dword loads, so its ring fill hits this XCD's L2 instead of waiting on HBM (the lab's first
    // ring wait: 9.2 us of a 109 us tile). The loads' results are never used; the generated
    // epilogue ends with a vmcnt wait that leaves only its own stores outstanding.
    // The loads' values are kept live until l2_done (an empty asm using them), so the compiler
    // places its own counted wait for them there, after the epilogue's stores are issued.
    template <int N>
    struct L2Pf {
        uint32_t v[N * S::DPW];
    };
    template <int N>
    __device__ __forceinline__ L2Pf<N> l2_prefetch() const {
        L2Pf<N> pf;
#pragma unroll
        for (int i = 0; i < N * S::DPW; ++i) pf.v[i] = 0;
        if (DEC || pf_stride <= 0) return pf;
        const int nb = static_cast<int>(blockIdx.x) + pf_stride;
        if (nb >= static_cast<int>(gridDim.x)) return pf;
        const long long gstride = static_cast<long long>(S::K) * B;
        const long long cols = static_cast<long long>(groups) * nq;
        const WGInfo w = tile_info<S>(nq, static_cast<long long>(xcd_tile(nb, gridDim.x)) * S::COLS, 0, cols);
        const __amdgpu_buffer_rsrc_t r = wg_rsrc(in_ptr, gstride * groups, gstride, w.g_first);
        Geometry g;
        g.B = static_cast<int>(B);
        g.sub = static_cast<int>(sub);
        g.nq = nq;
        g.tail = 4;
        uint32_t db[S::DPW];
        int gl[S::DPW];
        chunk_src(g, gstride, w, db, gl);
#pragma unroll
        for (int t = 0; t < N; ++t) {
#pragma unroll
            for (int j = 0; j < S::DPW; ++j) {
                if (S::NDMA % S::NW != 0 && wave * S::DPW + j >= S::NDMA) break;  // uniform
                pf.v[t * S::DPW + j] = __builtin_amdgcn_raw_buffer_load_b32(r, db[j], static_cast<uint32_t>(t) * B, 0);
            }
        }
        return pf;
    }
    template <int N>
    __device__ __forceinline__ static void l2_done(const L2Pf<N> &pf) {
#pragma unroll
        for (int i = 0; i < N * S::DPW; ++i) asm volatile("" ::"v"(pf.v[i]));
    }

    // Persistent encode, a prefetched tile: every wave has finished reading the previous tile's
    // row images (ring's top slots) before this tile's DMAs refill them.
    __device__ __forceinline__ void images_done() const {
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }

    // After the last step: every wave's reads of the ring are done before any wave writes its
    // store scratch (which aliases the ring).
    __device__ __forceinline__ static void release() {
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }

    // Decode: the DMA source of a step depends on the group's position table (LDS): entry t < KP
    // is the array index of original column t, entry KP + y that of recovery row y (0xFF =
    // absent). pre(t) reads it one iteration before issue(x, .) needs it, so the DMA issue never
    // waits on LDS latency.
    struct Pre {
        int p[S::DPW];
    };
    __device__ __forceinline__ Pre pre(int t) const {
        Pre r;
#pragma unroll
        for (int j = 0; j < S::DPW; ++j) r.p[j] = DEC ? pos[dgl[j] * (S::KP + S::MP) + t] : 0;
        return r;
    }

    // The position entries of up to 4 consecutive steps t..t+3 in one (byte-unaligned) LDS read,
    // taken one burst of DMA issues ahead: the issues of a burst then never wait on LDS (one
    // ds_read_u8 per step, each consumed by the next issue, put an LDS latency between every two
    // DMAs of a burst). The table has 4 bytes of padding past its last group.
    struct Pre4 {
        uint32_t w[S::DPW];
    };
    __device__ __forceinline__ Pre4 pre4(int t) const {
        Pre4 r;
#pragma unroll
        for (int j = 0; j < S::DPW; ++j) {
            r.w[j] = 0;
            if (DEC) r.w[j] = *reinterpret_cast<const u32_ua *>(pos + dgl[j] * (S::KP + S::MP) + t);
        }
        return r;
    }
    __device__ __forceinline__ void issue4(int x, const Pre4 &p4, int i) const {
        Pre r;
#pragma unroll
        for (int j = 0; j < S::DPW; ++j) r.p[j] = static_cast<int>((p4.w[j] >> (8 * i)) & 0xFFu);
        issue(x, r);
    }

    // DMA of step x into its ring slot (encode: input block x).
    __device__ __forceinline__ void issue(int x, const Pre &pr) const {
        uint8_t *slot = const_cast<uint8_t *>(lds) + (x % S::R) * S::SLOT;
#pragma unroll
        for (int j = 0; j < S::DPW; ++j) {
            if (S::NDMA % S::NW != 0 && wave * S::DPW + j >= S::NDMA) break;  // uniform
            lds_void *dst = (lds_void *)(slot + (wave * S::DPW + j) * 64 * S::W);
            if (DEC) {
                const int p = pr.p[j];
                const uint32_t o = (p == 0xFF || dbase[j] == OOR) ? OOR : dbase[j] + static_cast<uint32_t>(p) * B;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, dst, S::W, o, 0, 0, SH_LOAD_AUX);
            } else {
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, dst, S::W, x + x0s < krt ? dbase[j] : OOR,
                                                         static_cast<uint32_t>(x) * B + boff, 0, SH_LOAD_AUX);
            }
        }
    }

    __device__ __forceinline__ void read(int slot, uint32_t &d0, uint32_t &d1, uint32_t &d2,
                                         uint32_t &d3, uint32_t &d4, uint32_t &d5, uint32_t &d6,
                                         uint32_t &d7) const {
        const uint8_t *p = lds + slot * S::SLOT + rd;
        d0 = *reinterpret_cast<const uint32_t *>(p + 0 * S::ROWB);
        d1 = *reinterpret_cast<const uint32_t *>(p + 1 * S::ROWB);
        d2 = *reinterpret_cast<const uint32_t *>(p + 2 * S::ROWB);
        d3 = *reinterpret_cast<const uint32_t *>(p + 3 * S::ROWB);
        d4 = *reinterpret_cast<const uint32_t *>(p + 4 * S::ROWB);
        d5 = *reinterpret_cast<const uint32_t *>(p + 5 * S::ROWB);
        d6 = *reinterpret_cast<const uint32_t *>(p + 6 * S::ROWB);
        d7 = *reinterpret_cast<const uint32_t *>(p + 7 * S::ROWB);
    }

};

// Whole-block input (generator switch SH_BLK=<sub>, a kernel for one block size B = 8 * SUB;
// VERDICT r5 #2). The DMA reads each group the tile touches as ONE run of consecutive 16-byte
// chunks -- the group's whole block, 16-byte aligned in LDS at a stride GS -- instead of 175-byte
// sub-block rows realigned per lane (Src): the DMA's cost follows its runs of strictly
// consecutive chunks (reads alone 0.37 vs 0.42 ms, profiles/r05/ab_runs.txt block 2). A slot is
// then the raw image of up to NG blocks, and a lane's word of sub-block a sits at byte
// gl * GS + a * SUB + 4q: for a * SUB % 4 != 0 it is read as the two covering dwords and
// realigned with one v_alignbyte_b32 whose shift (a * SUB % 4) is a compile-time constant --
// round 5's version read it with byte-unaligned ds_read_b32 (~48 LDS cycles each, 5.3x slower).
// Column q = nq - 1 is read unshifted (bytes 4q..4q+3 of the sub-block, the last of them the
// next sub-block's first byte): the garbage byte lands in output byte SUB of each sub-block,
// which RowSink never stores (its last piece is realigned instead, RowSink::kBlk).
// GS: 16-byte multiple with GS/4 = nq (mod 32), so 32 consecutive tile columns hit 32 banks.
template <int SUB>
struct BlkGeo {
    static constexpr int NQ = ((SUB + 3) / 4 + 3) & ~3;
    static constexpr int B = 8 * SUB;
    static constexpr int CH = (B + 15) / 16;  // DMA chunks per block
    static constexpr int gs_of(int g) { return ((g / 4) % 32 == NQ % 32) ? g : gs_of(g + 16); }
    static constexpr int GS = gs_of((B + 15) & ~15);
    static constexpr int CPG = GS / 16;       // chunk slots per group image
    static constexpr int NG = (127 + NQ - 1) / NQ + 1;  // groups a 128-column tile can touch
    static constexpr int SLOT = ((NG * GS + 1023) / 1024) * 1024;
    static_assert(SUB >= 16 && NQ >= 8, "block size");
    // Tile starts. RowSink's last piece of a sub-block needs the byte before it from column
    // nq - 5 (BlkSrc reads the last chunk unshifted), so no tile may start at column nq - 4 of a
    // group: such a tile starts 4 columns earlier instead (those 4 columns are computed and
    // stored by both neighbours, with equal values). With 128 = -4 (mod 44) that happens once
    // per 10 tiles at B = 1400. The starts repeat with a period of PT tiles spanning D columns.
    static constexpr int next_start(int c) { return (c + 128) % NQ == NQ - 4 ? c + 124 : c + 128; }
    static constexpr int period() {
        int c = next_start(0), t = 1;
        while (c % NQ != 0) c = next_start(c), ++t;
        return t;
    }
    static constexpr int PT = period();
    struct Starts {
        int off[PT];
        int span;
    };
    static constexpr Starts starts() {
        Starts r{};
        int c = 0;
        for (int t = 0; t < PT; ++t) r.off[t] = c, c = next_start(c);
        r.span = c;
        return r;
    }
    __host__ __device__ static long long tile_start(int t) {
        constexpr Starts st = starts();
        return static_cast<long long>(st.span) * (t / PT) + st.off[t % PT];
    }
    __host__ __device__ static int tiles(long long cols) {
        constexpr Starts st = starts();
        const long long full = cols / st.span, rem = cols - full * st.span;
        int n = static_cast<int>(full) * PT;
        for (int t = 0; t < PT; ++t) n += st.off[t] < rem;
        return n;
    }
};

template <class S, bool DEC, int SUB>
struct BlkSrc {
    using G = BlkGeo<SUB>;
    static constexpr bool kStream = false, kBlk = true;
    static_assert(S::SLOT == G::SLOT && S::COLS == 128, "whole-block slots (generator SH_BLK)");
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t dbase[S::DPW];   // chunk source offset, block 0 / array slot 0 (OOR: none)
    int dgl[S::DPW];          // decode: the chunk's group (position-table index)
    int wave;
    uint32_t rd;              // this lane's word of sub-block 0 in a slot: gl * GS + 4q
    const uint8_t *lds;
    const uint8_t *pos;
    mutable uint32_t boff = 0;  // as Src::boff
    __device__ __forceinline__ void set_step0(int x0) const { boff = static_cast<uint32_t>(x0) * G::B; }

    __device__ __forceinline__ void init(const FixedArgs &a, const WGInfo &w, const uint8_t *lds_ring,
                                         const uint8_t *lds_pos) {
        rsrc = wg_rsrc(a.in, a.in_bytes, a.in_gstride, w.g_first);
        lds = lds_ring;
        pos = lds_pos;
        wave = w.wave;
        rd = w.valid ? static_cast<uint32_t>(w.gl * G::GS + 4 * w.q) : 0u;
        const long long tlo = w.col0 > w.lo ? w.col0 : w.lo;
        const long long thi = w.col0 + S::COLS < w.hi ? w.col0 + S::COLS : w.hi;
        const int ng = thi > tlo ? static_cast<int>((thi - 1) / G::NQ) - w.g_first + 1 : 0;
        const uint32_t gstride = static_cast<uint32_t>(a.in_gstride);
#pragma unroll
        for (int j = 0; j < S::DPW; ++j) {
            const int ci = (w.wave * S::DPW + j) * 64 + w.lane;  // chunk slot in the image
            const int gl = ci / G::CPG, ch = ci - gl * G::CPG;
            dgl[j] = gl < ng ? gl : 0;
            dbase[j] = (gl < ng && ch < G::CH) ? static_cast<uint32_t>(gl) * gstride + 16u * ch : OOR;
        }
    }
    template <int T, int I, int EX = 0>
    __device__ __forceinline__ void wait() const {
        constexpr int N = (I - T - 1) * S::DPW;
        static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
        if (S::NDMA % S::NW != 0 && wave * S::DPW >= S::NDMA)
            asm volatile("s_barrier" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
    }
    __device__ __forceinline__ static void release() {
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    struct Pre {
        int p[S::DPW];
    };
    __device__ __forceinline__ Pre pre(int t) const {
        Pre r;
#pragma unroll
        for (int j = 0; j < S::DPW; ++j) r.p[j] = DEC ? pos[dgl[j] * (S::KP + S::MP) + t] : 0;
        return r;
    }
    struct Pre4 {
        uint32_t w[S::DPW];
    };
    __device__ __forceinline__ Pre4 pre4(int t) const {
        Pre4 r;
#pragma unroll
        for (int j = 0; j < S::DPW; ++j) {
            r.w[j] = 0;
            if (DEC) r.w[j] = *reinterpret_cast<const u32_ua *>(pos + dgl[j] * (S::KP + S::MP) + t);
        }
        return r;
    }
    __device__ __forceinline__ void issue4(int x, const Pre4 &p4, int i) const {
        Pre r;
#pragma unroll
        for (int j = 0; j < S::DPW; ++j) r.p[j] = static_cast<int>((p4.w[j] >> (8 * i)) & 0xFFu);
        issue(x, r);
    }
    __device__ __forceinline__ void issue(int x, const Pre &pr) const {
        uint8_t *slot = const_cast<uint8_t *>(lds) + (x % S::R) * S::SLOT;
#pragma unroll
        for (int j = 0; j < S::DPW; ++j) {
            if (S::NDMA % S::NW != 0 && wave * S::DPW + j >= S::NDMA) break;  // uniform
            lds_void *dst = (lds_void *)(slot + (wave * S::DPW + j) * 64 * S::W);
            if (DEC) {
                const int p = pr.p[j];
                const uint32_t o = (p == 0xFF || dbase[j] == OOR) ? OOR : dbase[j] + static_cast<uint32_t>(p) * G::B;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, dst, S::W, o, 0, 0, SH_LOAD_AUX);
            } else {
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, dst, S::W, dbase[j],
                                                         static_cast<uint32_t>(x) * G::B + boff, 0, SH_LOAD_AUX);
            }
        }
    }
    template <int A>
    __device__ __forceinline__ static uint32_t word(const uint8_t *p) {
        constexpr int off = A * SUB, al = off & ~3, sh = off & 3;
        const uint32_t lo = *reinterpret_cast<const uint32_t *>(p + al);
        if constexpr (sh == 0) {
            return lo;
        } else {
            const uint32_t hi = *reinterpret_cast<const uint32_t *>(p + al + 4);
            return __builtin_amdgcn_alignbyte(hi, lo, sh);
        }
    }
    __device__ __forceinline__ void read(int slot, uint32_t &d0, uint32_t &d1, uint32_t &d2,
                                         uint32_t &d3, uint32_t &d4, uint32_t &d5, uint32_t &d6,
                                         uint32_t &d7) const {
        const uint8_t *p = lds + slot * S::SLOT + rd;
        d0 = word<0>(p);
        d1 = word<1>(p);
        d2 = word<2>(p);
        d3 = word<3>(p);
        d4 = word<4>(p);
        d5 = word<5>(p);
        d6 = word<6>(p);
        d7 = word<7>(p);
    }
};

// One-part shapes (P = 1): nothing is shared between the waves of a workgroup -- each column-wave
// alone consumes its columns -- so the LDS ring is pure overhead there: its DMA, the round trip
// through LDS and a workgroup barrier every step (the (28,4) ring holds only 4 slots of 16 KB).
// StreamSrc keeps the generated schedule but loads each lane's 8 words of a step straight into
// registers (8 coalesced buffer_load_dword: 64 consecutive columns of one sub-block per
// instruction, any byte alignment), R steps ahead; the compiler's own vmcnt waits guard each use,
// and no wave waits for another until the epilogue's row images.
template <class S, bool DEC>
struct StreamSrc {
    static constexpr bool kStream = true, kBlk = false;
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t lane_base;       // this lane's column in its group (OOR: past the batch)
    int gl;                   // decode: the lane's group (position-table index)
    uint32_t B, sub;
    const uint8_t *pos;
    mutable uint32_t buf[S::R][8];  // step x in buf[x % R] (compile-time indices after inlining)
    mutable uint32_t boff = 0;      // as Src::boff
    __device__ __forceinline__ void set_step0(int x0) const { boff = static_cast<uint32_t>(x0) * B; }

    __device__ __forceinline__ void init(const FixedArgs &a, const WGInfo &w, const uint8_t *, const uint8_t *lds_pos) {
        const Geometry &geo = a.geo;
        rsrc = wg_rsrc(a.in, a.in_bytes, a.in_gstride, w.g_first);
        B = geo.B;
        sub = geo.sub;
        pos = lds_pos;
        gl = w.gl;
        lane_base = w.valid ? static_cast<uint32_t>(w.gl) * static_cast<uint32_t>(a.in_gstride) + col_off(w.q, geo) : OOR;
    }
    template <int T, int I>
    __device__ __forceinline__ void wait() const {}
    __device__ __forceinline__ void rrow(int y, uint32_t (&r)[8]) const {  // as Src::rrow
        const int p = pos[gl * (S::KP + S::MP) + S::KP + y];
        const uint32_t o = (p == 0xFF || lane_base == OOR) ? OOR : lane_base + static_cast<uint32_t>(p) * B;
#pragma unroll
        for (int s = 0; s < 8; ++s) r[s] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, o + s * sub, 0, SH_LOAD_AUX);
    }
    __device__ __forceinline__ static void release() {
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    struct Pre {
        int p;
    };
    __device__ __forceinline__ Pre pre(int t) const {
        Pre r;
        r.p = DEC ? pos[gl * (S::KP + S::MP) + t] : 0;
        return r;
    }
    struct Pre4 {
        uint32_t w;
    };
    __device__ __forceinline__ Pre4 pre4(int t) const {  // as Src::pre4
        Pre4 r{0};
        if (DEC) r.w = *reinterpret_cast<const u32_ua *>(pos + gl * (S::KP + S::MP) + t);
        return r;
    }
    __device__ __forceinline__ void issue4(int x, const Pre4 &p4, int i) const {
        Pre r;
        r.p = static_cast<int>((p4.w >> (8 * i)) & 0xFFu);
        issue(x, r);
    }
    __device__ __forceinline__ void issue(int x, const Pre &pr) const {
        uint32_t o = lane_base, so = 0;
        if (DEC)
            o = (pr.p == 0xFF || lane_base == OOR) ? OOR : lane_base + static_cast<uint32_t>(pr.p) * B;
        else
            so = static_cast<uint32_t>(x) * B + boff;
#pragma unroll
        for (int s = 0; s < 8; ++s)
            buf[x % S::R][s] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, o == OOR ? OOR : o + s * sub, so, SH_LOAD_AUX);
    }
    __device__ __forceinline__ void read(int slot, uint32_t &d0, uint32_t &d1, uint32_t &d2, uint32_t &d3,
                                         uint32_t &d4, uint32_t &d5, uint32_t &d6, uint32_t &d7) const {
        d0 = buf[slot][0];
        d1 = buf[slot][1];
        d2 = buf[slot][2];
        d3 = buf[slot][3];
        d4 = buf[slot][4];
        d5 = buf[slot][5];
        d6 = buf[slot][6];
        d7 = buf[slot][7];
    }
};

// Output assembled per row across the part's CW column-waves, so every store instruction writes
// 64 consecutive 16-byte pieces of the output in MEMORY order (about 1 KB contiguous): the
// CW waves of a part write their words of row y into a shared LDS row image laid out like a ring
// slot ([sub-block][tile column]), meet at a workgroup barrier, and each then stores 128 pieces
// taken from the image in memory order -- group by group over the tile, sub-block by sub-block,
// 4-column chunk by chunk. A group whose columns all lie in the tile is written as one
// contiguous m*B span by one workgroup within a few microseconds; only the groups split between
// two tiles are written as per-sub-block runs. (A per-wave transposition, round 2's store path,
// stored 8 runs of <= 176 bytes per instruction: the encode kernel was 3 % slower with it.) Row images are double-buffered by row parity: a wave
// reads row y's image before it joins row y+1's barrier, so row y+2 may overwrite it.
// Every wave of the workgroup joins one barrier per row of the largest part (pad() for the
// shorter parts). The images ([2][PW][SLOT] bytes) alias the ring (after Src::release()).
// BLK (BlkSrc inputs): the words of a sub-block's last chunk were computed unshifted (bytes
// 4q..4q+3), so that piece (stored at sub - 16, as always) is taken from the image one byte
// earlier: five aligned dwords from lsrc - 4, realigned by v_alignbyte_b32 with shift 3 (shift 0,
// read from lsrc, for every other piece: one code path for all lanes).
template <class S, bool BLK = false>
struct RowSink {
    __amdgpu_buffer_rsrc_t rsrc;
    mutable uint32_t gdst[2];  // per piece: destination offset without the row term (OOR: none)
    mutable uint32_t lsrc[2];  // per piece: byte offset inside a row image
    mutable uint32_t lsh[2];   // BLK: per piece byte shift (3: last chunk of its sub-block)
    mutable uint32_t poff[2];  // split tiles: per piece offset in a partial row (piece index * 16)
    // Split tiles (see "Split tiles" below): this workgroup computes half `half` of the steps of
    // split tile `sidx`; its rows go to the partial scratch, the second arriver combines.
    __amdgpu_buffer_rsrc_t prsrc;
    uint32_t pbase;            // this split tile's partials: [half][M rows][2 * COLS pieces][16 B]
    uint32_t *cnt;             // its arrival counter (zero between launches)
    int half;
    uint8_t *lds0;             // workgroup LDS base (the combine's "last arriver" word)
    static constexpr uint32_t PR = 32u * S::COLS;  // bytes of one partial row (2 * COLS pieces)
    mutable uint32_t wofs;     // this lane's word in a row image (tile column * 4)
    uint32_t B;
    uint8_t *img;              // this part's row image, even rows (odd rows: + P * SLOT)
    // uniform state (SGPRs): prepare() derives the per-lane offsets at the epilogue, so they
    // are not live across the body
    long long col0, lo, hi;
    uint32_t out_gstride;
    int g_first, nq, sub;

    // img_slot: first ring slot of the images (persistent encode: the ring's top 2P slots, so the
    // next tile's prefetched steps 0..R-2P-1 stay intact)
    __device__ __forceinline__ void init(const FixedArgs &a, const WGInfo &w, int part, uint8_t *lds,
                                         int img_slot = 0) {
        rsrc = wg_rsrc(a.out, a.out_bytes, a.out_gstride, w.g_first);
        B = a.geo.B;
        img = lds + img_slot * S::SLOT + (part % S::PW) * S::IMG;
        col0 = w.col0;
        lo = w.lo;
        hi = w.hi;
        out_gstride = static_cast<uint32_t>(a.out_gstride);
        g_first = w.g_first;
        nq = a.geo.nq;
        sub = a.geo.sub;
    }
    // Per-lane piece offsets of the tile (called right before the first row).
    __device__ __forceinline__ void prepare() const {
        const int lane = threadIdx.x & 63;
        const int cw = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) / S::PW;
        wofs = static_cast<uint32_t>(cw * 64 + lane) * 4u;
        const long long cs = col0 > lo ? col0 : lo;
        const long long ce = col0 + S::COLS < hi ? col0 + S::COLS : hi;
        Geometry geo;
        geo.B = static_cast<int>(B);
        geo.sub = sub;
        geo.nq = nq;
        geo.tail = 4;
        // Groups overlapping the tile: the first (from column cs) and the last may be partial, every
        // one between is whole (8 * nq / 4 = 2 * nq pieces). O(1) per piece: the round-4 walk over
        // the tile's groups cost up to 64 iterations of 64-bit arithmetic per piece at nq = 8
        // (B = 256: a 512-column tile spans 64 groups), a regression of (28,4,256).
        const long long g0 = cs / nq;
        const int qa0 = static_cast<int>(cs - g0 * nq);
        const int n0 = static_cast<int>(((ce < (g0 + 1) * nq ? ce : (g0 + 1) * nq) - cs) >> 2);  // chunks
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            int rem = (cw * 2 + h) * 64 + lane;  // piece index in memory order
            poff[h] = static_cast<uint32_t>(rem) * 16u;
            gdst[h] = OOR;
            lsrc[h] = 0;
            lsh[h] = 0;
            long long g;
            int b, q;
            bool ok;
            if (rem < 8 * n0) {
                g = g0;
                b = rem / n0;
                q = qa0 + 4 * (rem - b * n0);
                ok = true;
            } else {
                rem -= 8 * n0;
                const int gi = rem / (2 * nq);
                g = g0 + 1 + gi;
                rem -= gi * 2 * nq;
                const long long gend = (ce < (g + 1) * nq ? ce : (g + 1) * nq);
                const int ng = g * nq < ce ? static_cast<int>((gend - g * nq) >> 2) : 0;
                ok = rem < 8 * ng;
                b = ok ? rem / ng : 0;
                q = ok ? 4 * (rem - b * ng) : 0;
            }
            if (ok) {
                gdst[h] = static_cast<uint32_t>(g - g_first) * out_gstride +
                          col_off(q, geo) + static_cast<uint32_t>(b * geo.sub);
                lsrc[h] = static_cast<uint32_t>(b * S::ROWB) + static_cast<uint32_t>(g * nq + q - col0) * 4u;
                if (BLK && q == nq - 4 && 4 * nq != sub) {
                    lsh[h] = 3;
                    lsrc[h] -= 4;  // column nq - 5 is in the tile (BlkGeo::tile_start)
                }
            }
        }
    }
    // Row y's words into the row image (parity YI), barrier; then piece h of the image.
    template <int YI>
    __device__ __forceinline__ uint8_t *image(const uint32_t (&w)[8]) const {
        uint8_t *im = img + (YI & 1) * S::PW * S::IMG;
#pragma unroll
        for (int b = 0; b < 8; ++b) *reinterpret_cast<uint32_t *>(im + b * S::ROWB + wofs) = w[b];
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        return im;
    }
    __device__ __forceinline__ u32x4 piece(const uint8_t *im, int h) const {
        u32x4 v;
        if constexpr (BLK) {
            const uint32_t *p = reinterpret_cast<const uint32_t *>(im + lsrc[h]);
            const uint32_t u0 = p[0], u1 = p[1], u2 = p[2], u3 = p[3], u4 = p[4];
            v.x = __builtin_amdgcn_alignbyte(u1, u0, lsh[h]);
            v.y = __builtin_amdgcn_alignbyte(u2, u1, lsh[h]);
            v.z = __builtin_amdgcn_alignbyte(u3, u2, lsh[h]);
            v.w = __builtin_amdgcn_alignbyte(u4, u3, lsh[h]);
        } else {
            v = *reinterpret_cast<const u32x4 *>(im + lsrc[h]);
        }
        return v;
    }
    template <int YI>
    __device__ __forceinline__ void row(int y, const uint32_t (&w)[8]) const {
        const uint8_t *im = image<YI>(w);
#pragma unroll
        for (int h = 0; h < 2; ++h)
            __builtin_amdgcn_raw_buffer_store_b128(piece(im, h), rsrc, gdst[h], static_cast<uint32_t>(y) * B, SH_STORE_AUX);
    }

    // ---- Split tiles. The launch's last tiles run as two workgroups each, one per half of the
    // steps (blocks 0..n0-1 and n0..), so the grid's tail drains in half-tile tasks. Each half
    // stores its rows' pieces as a partial (write-through sc1 stores, the whole tile's pieces in
    // memory order, offset poff), drains them (every wave vmcnt(0)), meets the workgroup barrier,
    // and one lane adds 1 to the tile's counter (relaxed, agent scope). The workgroup that draws 1
    // is the second: it reads both partials with sc1 loads, XORs them (the bitmatrix product is
    // linear in the steps) and stores the tile's rows; it then resets the counter. No workgroup
    // waits for another, and the protocol holds for any placement of the two halves (the
    // write-through hand-off of MI355X_MICROARCH.md "inter-workgroup visibility", first row);
    // placing both on one XCD back to back (FIXED_KERNEL) only makes the second's reads cheaper.
    __device__ __forceinline__ void split_init(const FixedArgs &a, int sidx, int h, uint8_t *lds) {
        prsrc = make_rsrc(a.split_part, static_cast<uint32_t>(a.split_cap));
        pbase = static_cast<uint32_t>(sidx) * 2u * S::M * PR;
        cnt = a.split_cnt + sidx;
        half = h;
        lds0 = lds;
    }
    template <int YI>
    __device__ __forceinline__ void part_row(int y, const uint32_t (&w)[8]) const {
        const uint8_t *im = image<YI>(w);
        const uint32_t so = pbase + static_cast<uint32_t>(half * S::M + y) * PR;
#pragma unroll
        for (int h = 0; h < 2; ++h) __builtin_amdgcn_raw_buffer_store_b128(piece(im, h), prsrc, poff[h], so, 16 /* sc1 */);
    }
    // After every row of every part (part_row / pad): rows y0 .. y0 + nr - 1 are this wave's.
    __device__ __forceinline__ void combine(int y0, int nr) const {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its partial
        __syncthreads();
        uint32_t *flag = reinterpret_cast<uint32_t *>(lds0);
        if (threadIdx.x == 0) *flag = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        if (*flag == 0) return;  // first arriver: the other half combines
        for (int yi = 0; yi < nr; ++yi) {
            const uint32_t y = static_cast<uint32_t>(y0 + yi);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const u32x4 p0 = __builtin_amdgcn_raw_buffer_load_b128(prsrc, poff[h], pbase + y * PR, 16);
                const u32x4 p1 = __builtin_amdgcn_raw_buffer_load_b128(prsrc, poff[h], pbase + (S::M + y) * PR, 16);
                __builtin_amdgcn_raw_buffer_store_b128(p0 ^ p1, rsrc, gdst[h], y * B, SH_STORE_AUX);
            }
        }
        if (threadIdx.x == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    template <int YI>
    __device__ __forceinline__ void pad() const {
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }

    // Row pairs (generator switch SH_ROW_PAIRS=1, A/B): rows 2i and 2i+1 share one barrier --
    // both images written, one barrier, then the four pieces read and stored -- so a part's 8
    // rows take 4 epilogue barriers instead of 8. Images [pair parity][row of the pair][PW][IMG]
    // (4 * PW * IMG bytes: the whole 64 KB ring at P = 4). LAST: the part's largest row count
    // ends on this row (an even row then stores alone).
    template <int YI, bool LAST>
    __device__ __forceinline__ void row2(int y, const uint32_t (&w)[8]) const {
        static_assert(4 * S::PW * S::IMG <= S::R * S::SLOT, "row-pair images must fit inside the ring");
        uint8_t *im = img + (((YI >> 1) & 1) * 2 + (YI & 1)) * S::PW * S::IMG;
#pragma unroll
        for (int b = 0; b < 8; ++b) *reinterpret_cast<uint32_t *>(im + b * S::ROWB + wofs) = w[b];
        if ((YI & 1) == 0 && !LAST) return;  // the pair's second row brings the barrier
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if ((YI & 1) == 1) {
            const uint8_t *im0 = im - S::PW * S::IMG;
#pragma unroll
            for (int h = 0; h < 2; ++h)
                __builtin_amdgcn_raw_buffer_store_b128(piece(im0, h), rsrc, gdst[h], static_cast<uint32_t>(y - 1) * B, SH_STORE_AUX);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h)
            __builtin_amdgcn_raw_buffer_store_b128(piece(im, h), rsrc, gdst[h], static_cast<uint32_t>(y) * B, SH_STORE_AUX);
    }
    template <int YI, bool LAST>
    __device__ __forceinline__ void pad2() const {
        if ((YI & 1) == 0 && !LAST) return;
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
};

// Sets up src/sink for the tile starting at column col0 (columns outside [lo, hi) are idle
// lanes) and returns this wave's part. The caller (the FIXED_KERNEL macro)
// then calls the generated run_<name> directly, so everything inlines into one function: a
// non-inlined body took `src` by reference through scratch and read the LDS ring with flat loads.
template <class S, bool DEC, class SrcT, class SinkT>
__device__ __forceinline__ int kernel_prologue(const FixedArgs &a, uint8_t *lds, SrcT &src,
                                               SinkT &sink, long long col0, long long lo, long long hi,
                                               int img_slot = 0, int hgrp = 0) {
    const WGInfo w = tile_info<S>(a.geo.nq, col0, lo, hi);
    const int part = hgrp * S::PW + w.wave % S::PW;
    const int nq = a.geo.nq;
    // The row images of the epilogue alias the start of the ring: they are used only after the
    // last step, behind Src::release()'s barrier, so the ring gets that LDS as extra slots.
    uint8_t *lds_pos = lds + (SrcT::kStream ? 2 * S::PW * S::SLOT : S::R * S::SLOT);
    if (DEC) {
        const int ng = a.groups_per_wg;
        const int ghi = static_cast<int>(hi / nq);
        constexpr int TW = (S::KP + S::MP) / 4;
        for (int i = threadIdx.x; i < ng * TW; i += S::NT) {
            const int lg = i / TW, t = i - lg * TW;
            const int gg = w.g_first + lg;
            uint32_t v = 0xFFFFFFFFu;
            if (gg < ghi) {
                v = (t < S::KP / 4)
                        ? reinterpret_cast<const uint32_t *>(a.pos + gg * static_cast<long long>(S::KP))[t]
                        : reinterpret_cast<const uint32_t *>(a.rpos + gg * static_cast<long long>(S::MP))[t - S::KP / 4];
            }
            reinterpret_cast<uint32_t *>(lds_pos)[i] = v;
        }
        __syncthreads();
    }
    src.init(a, w, lds, lds_pos);
    sink.init(a, w, part, lds, img_slot);
    return part;  // the generated body issues the ring's first DMAs
}


// Persistent encode workgroups: two per CU (the LDS ring and the registers allow two), each
// walking tiles v = blockIdx.x + i * grid in xcd_tile order (grid % 8 == 0, so every tile of a
// workgroup lies on its XCD and the 64 workgroups of an XCD code 64 neighbouring tiles at a time,
// as the one-tile grid does). A tile prefetches its successor's first NPF steps right after its
// last step, so their HBM latency runs under its epilogue stores instead of opening the next
// tile with an empty ring (round-4 lab: the first ring wait of a fresh tile took 9.2 us of a
// 109 us tile).
// Tile loop of a persistent workgroup; RUN(part, src, sink) is the generated body (a macro, so
// the ~15K-instruction body is inlined: called as a function it would take `src` through
// scratch, and a scratch load's vmcnt wait drains the ring).
#define SH_PERSISTENT_TILES(S, DEC, RUN)                                                          \
    do {                                                                                          \
        const long long hi_ = static_cast<long long>(a.groups) * a.geo.nq;                        \
        const int ntiles_ = static_cast<int>((hi_ + S::COLS - 1) / S::COLS);                      \
        int v_ = blockIdx.x;                                                                      \
        if (v_ >= ntiles_) break;                                                                 \
        Src<S, DEC> src;                                                                          \
        RowSink<S> sink;                                                                          \
        const int part = kernel_prologue<S, DEC>(a, lds, src, sink,                               \
                                                 static_cast<long long>(xcd_tile(v_, ntiles_)) * S::COLS, 0, \
                                                 hi_, S::R - 2 * S::P);                           \
        for (;;) {                                                                                \
            const int vn_ = v_ + static_cast<int>(gridDim.x);                                     \
            src.has_next = vn_ < ntiles_;                                                         \
            src.next_col0 = static_cast<long long>(xcd_tile(src.has_next ? vn_ : v_, ntiles_)) * S::COLS; \
            RUN(part, src, sink);                                                                 \
            if (!src.has_next) break;                                                             \
            v_ = vn_;                                                                             \
            const WGInfo w_ = tile_info<S>(a.geo.nq, src.next_col0, 0, hi_);                      \
            src.advance();                                                                        \
            sink.init(a, w_, part, lds, S::R - 2 * S::P);                                         \
        }                                                                                         \
    } while (0)

// Tile and part-group of a workgroup when a tile's parts run in H > 1 workgroups (Shape::PW < P):
// the H workgroups of a tile get blocks 8 * (H * j + h) + x, i.e. the same XCD x and consecutive
// dispatch slots there, so the second to H-th reads of the tile's input hit that XCD's L2. The
// grid is rounded up to a multiple of 8 * H; a block past the last tile returns -1.
template <class S>
__device__ __forceinline__ int tile_of(const FixedArgs &a, int &hgrp, int ntiles) {
    if (S::H == 1) {
        hgrp = 0;
        return xcd_tile(blockIdx.x, gridDim.x);
    }
    const int x = blockIdx.x & 7, i = blockIdx.x >> 3;
    hgrp = i % S::H;
    const int vb = (i / S::H) * 8 + x;
    return vb < ntiles ? xcd_tile(vb, ntiles) : -1;
}

inline int persistent_slots() {
    static const int cus = [] {
        int d = 0, n = 0;
        if (hipGetDevice(&d) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess)
            n = 256;
        return n > 0 ? n : 256;
    }();
    return 2 * cus;  // a multiple of 8 on MI355X (256 CUs)
}

// Measurement builds only (SH_HSACO_DIR, fixed_dispatch.cpp): launch the kernel `tag` from a
// code object of that directory instead (tools/il_reorder.py layouts); *used = false: none.
hipError_t module_launch(const char *tag, const FixedArgs &a, unsigned blocks, unsigned threads, size_t lds,
                         hipStream_t s, bool *used);
// Whether a measurement build launches `tag` from an external code object (no split tiles then).
bool tag_is_module(const char *tag);

// Split tiles of a launch (RowSink "Split tiles"): about half a round of workgroup slots' worth
// of the last tiles, so the grid drains in half-tile tasks; every tile when all halves fit one
// round. A multiple of 8 (split_tile_of), at most what the caller's scratch holds, 0 below 8.
// SH_SPLIT (measurement builds only) forces the count (0: no split).
// Workgroups of this kernel resident at once on the device (occupancy x CUs), cached.
template <class S, bool DEC>
inline int launch_slots(void (*kern)(FixedArgs), size_t lds) {
    static const int slots = [&] {
        int per_cu = 0, d = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, S::NT, lds) != hipSuccess || per_cu < 1) per_cu = 1;
        if (hipGetDevice(&d) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess)
            cus = 256;
        return per_cu * (cus > 0 ? cus : 256);
    }();
    return slots;
}

template <class S, bool DEC>
inline int split_count(const FixedArgs &a, int ntiles, void (*kern)(FixedArgs), size_t lds) {
    if (!a.split_part || !a.split_cnt || S::H != 1) return 0;
    const int slots = launch_slots<S, DEC>(kern, lds);
    long long n = std::min<long long>(ntiles, slots / 2);
    if (const char *e = SH_MEASURE_ENV("SH_SPLIT")) n = std::min<long long>(ntiles, std::atoi(e));
    const long long per = 2ll * S::M * 32 * S::COLS;  // partial bytes per split tile
    n = std::min<long long>(n, a.split_cap / per);
    n = std::min<long long>(n, a.split_max);
    n &= ~7ll;
    return n >= 8 ? static_cast<int>(n) : 0;
}

template <class S, bool DEC, bool STREAM = false, bool PERS = false, bool SPLIT = false>
inline hipError_t launch_shape(FixedArgs a, hipStream_t s, void (*kern)(FixedArgs), const char *tag = nullptr,
                               int ntiles = -1) {
    constexpr bool dec = DEC;
    // a runtime k below K: only the product source (Src) reads zeros past k
    if (a.k_rt > 0 && a.k_rt != S::K && (STREAM || S::SLOT != S::IMG)) return hipErrorNotSupported;
    a.groups_per_wg = (S::COLS - 1) / a.geo.nq + 2;
    // ring (the row images of the epilogue alias it); a streaming source needs only the images
    constexpr size_t front = STREAM ? 2ull * S::PW * S::SLOT : static_cast<size_t>(S::R) * S::SLOT;
    static_assert(STREAM || 2 * S::PW * S::IMG <= S::R * S::SLOT, "row images must fit inside the ring");
    // (+4: Src::pre4 reads up to 3 bytes past the last group's table)
    const size_t lds = front + (dec ? static_cast<size_t>(a.groups_per_wg) * (S::KP + S::MP) + 4 : 0);
    const long long cols = static_cast<long long>(a.groups) * a.geo.nq;
    unsigned blocks = static_cast<unsigned>(ntiles >= 0 ? ntiles : (cols + S::COLS - 1) / S::COLS);  // one tile each
    if (S::H > 1) blocks = (blocks + 7) / 8 * 8 * S::H;  // tile_of(): H part-groups per tile
    a.nsplit = (SPLIT && !PERS && !tag_is_module(tag)) ? split_count<S, DEC>(a, static_cast<int>(blocks), kern, lds) : 0;
    a.pf_stride = launch_slots<S, DEC>(kern, lds);
    blocks += static_cast<unsigned>(a.nsplit);  // split tiles: two workgroups each
    if (PERS) blocks = std::min<unsigned>(blocks, static_cast<unsigned>(persistent_slots()));
    if (tag) {
        bool used = false;
        const hipError_t e = module_launch(tag, a, blocks, S::NT, lds, s, &used);
        if (used) return e;
    }
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(S::NT), lds, s, a);
    return hipGetLastError();
}

// Tile of a workgroup when the launch's last `nsplit` tiles are split (a multiple of 8): blocks
// [0, T - nsplit) are the whole tiles in xcd_tile order; block T - nsplit + j is half (j >> 3) & 1
// of split tile xcd_tile(((j >> 4) << 3) | (j & 7), nsplit), so a tile's two halves get blocks 8
// apart (one XCD, dispatched back to back) and run after every whole tile has been dispatched.
__device__ __forceinline__ int split_tile_of(int ntiles, int nsplit, int &half, int &sidx) {
    const int nfull = ntiles - nsplit;
    if (static_cast<int>(blockIdx.x) < nfull) {
        half = -1;
        sidx = 0;
        return xcd_tile(blockIdx.x, nfull);
    }
    const int j = static_cast<int>(blockIdx.x) - nfull, i = j >> 3;
    half = i & 1;
    sidx = xcd_tile(((i >> 1) << 3) | (j & 7), nsplit);
    return nfull + sidx;
}

// Source of a kernel instance: StreamSrc (STREAM), BlkSrc (BLKSUB > 0: whole-block slots for
// B = 8 * BLKSUB) or the sub-block-row gather Src.
template <class S, bool DEC, bool STREAM, int BLKSUB>
using SrcOf = typename std::conditional<
    STREAM, StreamSrc<S, DEC>,
    typename std::conditional<(BLKSUB > 0), BlkSrc<S, DEC, (BLKSUB > 0 ? BLKSUB : 64)>, Src<S, DEC>>::type>::type;

// Tiles of a launch: COLS-column tiles, or BlkGeo's tile starts.
template <class S, int BLKSUB>
__host__ __device__ inline int tiles_of(long long cols) {
    if constexpr (BLKSUB > 0)
        return BlkGeo<BLKSUB>::tiles(cols);
    else
        return static_cast<int>((cols + S::COLS - 1) / S::COLS);
}
template <int BLKSUB>
__device__ __forceinline__ long long tile_col0(int tile, int cols_per_tile) {
    if constexpr (BLKSUB > 0)
        return BlkGeo<BLKSUB>::tile_start(tile);
    else
        return static_cast<long long>(tile) * cols_per_tile;
}

}  // namespace fixed
}  // namespace sh

// One kernel + launcher of a generated (k, m): MODE enc (DEC = false) or dec (DEC = true);
// MINW = waves per SIMD the registers are allocated for. The host routes shapes with
// nq % 4 != 0 (a 16-byte chunk could straddle two groups) or sub < 16 to the generic kernel.
#define FIXED_KERNEL(NAME, K, M, P, CW, R, MINW, MODE, DEC, DMA, STREAM, PW, BLKSUB, SPLIT)       \
    namespace sh {                                                                                \
    namespace fixed {                                                                             \
    using Shape_##NAME##_##MODE =                                                                 \
        Shape<K, M, P, CW, R, DMA, PW, ((BLKSUB) > 0 ? BlkGeo<((BLKSUB) > 0 ? (BLKSUB) : 64)>::SLOT : 0)>; \
    __global__ __launch_bounds__(64 * CW * PW, MINW) void kern_##NAME##_##MODE(FixedArgs a) {     \
        extern __shared__ __attribute__((aligned(16))) uint8_t lds[];                             \
        using S = Shape_##NAME##_##MODE;                                                          \
        using SrcT = SrcOf<S, DEC, STREAM, BLKSUB>;                                               \
        SrcT src;                                                                                 \
        RowSink<S, SrcT::kBlk> sink;                                                              \
        const long long cols_ = static_cast<long long>(a.groups) * a.geo.nq;                      \
        const int ntiles_ = tiles_of<S, BLKSUB>(cols_);                                           \
        int hgrp = 0, half = -1, sidx = 0, tile;                                                  \
        if ((SPLIT) && a.nsplit > 0) {                                                            \
            tile = split_tile_of(ntiles_, a.nsplit, half, sidx);                                  \
        } else {                                                                                  \
            tile = tile_of<S>(a, hgrp, ntiles_);                                                  \
            if (tile < 0) return;                                                                 \
        }                                                                                         \
        const long long c0 = tile_col0<BLKSUB>(tile, S::COLS);                                    \
        const int part = kernel_prologue<S, DEC>(a, lds, src, sink, c0, 0, cols_, 0, hgrp);        \
        if ((SPLIT) && half >= 0) {                                                               \
            sink.split_init(a, sidx, half, lds);                                                  \
            run_##NAME##_##MODE##_half(half, part, src, sink);                                    \
        } else {                                                                                  \
            run_##NAME##_##MODE(part, src, sink);                                                 \
        }                                                                                         \
    }                                                                                             \
    hipError_t launch_##NAME##_##MODE(FixedArgs a, hipStream_t s) {                               \
        if ((BLKSUB) > 0 && a.geo.B != 8 * (BLKSUB)) return hipErrorNotSupported;                 \
        const long long cols_ = static_cast<long long>(a.groups) * a.geo.nq;                      \
        return launch_shape<Shape_##NAME##_##MODE, DEC, STREAM, false, (SPLIT) != 0>(             \
            a, s, kern_##NAME##_##MODE, #NAME "_" #MODE, tiles_of<Shape_##NAME##_##MODE, BLKSUB>(cols_)); \
    }                                                                                             \
    }                                                                                             \
    }

// The persistent form (SH_PERSISTENT_TILES above): two workgroups per CU walk the
// tiles, each tile prefetching its successor's first steps.
#define FIXED_KERNEL_PERSISTENT(NAME, K, M, P, CW, R, MINW, MODE, DEC)                            \
    namespace sh {                                                                                \
    namespace fixed {                                                                             \
    __global__ __launch_bounds__(64 * CW * P, MINW) void kern_##NAME##_##MODE(FixedArgs a) {      \
        extern __shared__ __attribute__((aligned(16))) uint8_t lds[];                             \
        using S = Shape<K, M, P, CW, R, true>;                                                    \
        SH_PERSISTENT_TILES(S, DEC, run_##NAME##_##MODE);                                         \
    }                                                                                             \
    hipError_t launch_##NAME##_##MODE(FixedArgs a, hipStream_t s) {                               \
        return launch_shape<Shape<K, M, P, CW, R, true>, DEC, false, true>(a, s, kern_##NAME##_##MODE); \
    }                                                                                             \
    }                                                                                             \
    }
