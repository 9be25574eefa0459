// Measurement lab for the compile-time encode kernel (never part of the product): times the
// product kernel structure against experimental launch structures built from the SAME generated
// body, and records per-workgroup timestamps.
//
//   tools/enc_lab.sh  (generates the bodies, builds, runs; see there)
//
// Variants (all encode k=200 m=32 B=1400, 8192 groups unless --groups):
//   base   the product kernel (scratch aliases the ring), one tile per workgroup
//   sep    one tile per workgroup, store scratch in its own LDS (control for `pers`)
//   pers   persistent workgroups (2 per CU), tile v = xcd_tile(blockIdx + i * grid): the next
//          tile's first ring DMAs are issued right after the last compute step, before the
//          current tile's epilogue stores (scratch separate from the ring)
// Stamps (s_memrealtime, 100 MHz) per tile: start, first ring wait passed, last step done, end,
// plus the XCC / CU of the workgroup -> lab_stamps_<variant>.csv.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>

#include "fixed_k200_m32.inc"

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

namespace lab {
using namespace sh;
using namespace sh::fixed;

// Output, transposed through a per-wave 2 KB LDS scratch so every store is 16 contiguous bytes:
// a lane holds word q of the 8 sub-blocks of a row; it writes them to scratch[b][lane], then
// reads back two 16-byte items (sub-block b, 4-column chunk t) and stores each with one
// buffer_store_dwordx4 -- 2 store instructions per row instead of 8 dword stores. A chunk lies
// in one group (nq % 4 == 0) and is contiguous in memory (the shifted last chunk included).
// Item i = lane + 64h (h = 0, 1): b = i / 16, t = i % 16. Chunks past the last group get an
// out-of-range offset, dropped by the buffer unit.
struct PieceSink {
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t voff[2];         // per item: chunk base + b * sub (or OOR)
    uint32_t B;
    uint8_t *scr;             // this wave's scratch [8][64] words
    int lane;
    __device__ __forceinline__ void init(const FixedArgs &a, const WGInfo &w, uint8_t *scratch) {
        const Geometry &geo = a.geo;
        rsrc = wg_rsrc(a.out, a.out_bytes, a.out_gstride, w.g_first);
        B = geo.B;
        lane = w.lane;
        scr = scratch;
        const int t = w.lane & 15;
        const long long colx = w.col0 + (w.c - w.lane) + 4 * t;  // first column of chunk t
        const int gx = colx >= 0 ? static_cast<int>(colx / geo.nq) : -1;
        const int qx = static_cast<int>(colx - static_cast<long long>(gx) * geo.nq);
        const uint32_t base = static_cast<uint32_t>(gx - w.g_first) * static_cast<uint32_t>(a.out_gstride) +
                              col_off(qx, geo);
        const bool ok = colx >= w.lo && colx < w.hi;
#ifdef SH_GEN_STORE_ALIGNED  // measurement build only (see store_row_dw)
        const uint32_t sstride = 176, abase = (static_cast<uint32_t>(gx - w.g_first) * static_cast<uint32_t>(a.out_gstride) + 4u * qx) & ~15u;
#else
        const uint32_t sstride = static_cast<uint32_t>(geo.sub), abase = base;
#endif
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int b = (w.lane >> 4) + 4 * h;
            voff[h] = ok ? abase + static_cast<uint32_t>(b) * sstride : OOR;
        }
        sub = static_cast<uint32_t>(geo.sub);
        {
            const long long colc = w.col0 + w.c;
            const int gc = colc >= 0 ? static_cast<int>(colc / geo.nq) : -1;
            const int qc = static_cast<int>(colc - static_cast<long long>(gc) * geo.nq);
            dw_off = (colc >= w.lo && colc < w.hi)
                         ? static_cast<uint32_t>(gc - w.g_first) * static_cast<uint32_t>(a.out_gstride) + col_off(qc, geo)
                         : OOR;
        }
    }
    // Measurement-only store forms (tools/gen_fixed_kernels.py SH_GEN_STORE): 1 = one dword
    // store per sub-block straight from the registers; 2 = the transposed dwordx4 form at
    // 16-byte-aligned offsets (sub-block stride rounded up to 176: wrong bytes, alignment cost).
    uint32_t dw_off;          // this lane's column offset (dword form)
    __device__ __forceinline__ void store_row_dw(int y, const uint32_t (&w)[8]) const {
#pragma unroll
        for (int b = 0; b < 8; ++b)
            __builtin_amdgcn_raw_buffer_store_b32(w[b], rsrc, dw_off + static_cast<uint32_t>(b) * sub,
                                                  static_cast<uint32_t>(y) * B, SH_STORE_AUX);
    }
    uint32_t sub;
    __device__ __forceinline__ void store_row(int y, const uint32_t (&w)[8]) const {
#pragma unroll
        for (int b = 0; b < 8; ++b) reinterpret_cast<uint32_t *>(scr)[b * 64 + lane] = w[b];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int i = lane + 64 * h;
            const u32x4 v = *reinterpret_cast<const u32x4 *>(scr + (i >> 4) * 256 + (i & 15) * 16);
            __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, voff[h], static_cast<uint32_t>(y) * B, SH_STORE_AUX);
        }
    }
    // the generated epilogue's interface (YI = the part's row index; pad = a part with fewer rows)
    template <int YI>
    __device__ __forceinline__ void row(int y, const uint32_t (&w)[8]) const { store_row(y, w); }
    template <int YI>
    __device__ __forceinline__ void pad() const {}
};


using Sink = PieceSink;

#ifndef LAB_R
#define LAB_R 16
#endif
using S = Shape<200, 32, 4, 2, LAB_R, true>;
constexpr int NSTAMP = 96;  // + per wave (64 + 3*wave): s_memtime cycles computing, in vmcnt waits, in barrier waits  // start, first, last, end, hwid, -, then one per ring wait (after its barrier)

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

template <bool ON>
struct Stamp {
    uint64_t *p;  // this tile's record
    __device__ __forceinline__ void put(int i) const {
        if (ON && threadIdx.x == 0) p[i] = now();
    }
};

// Product Src plus hooks: stamps, and (persistent) skipping the DMAs already issued for this
// tile by the previous tile's epilogue / issuing the next tile's.
template <bool PERS, bool ST, bool ALN = false>
struct LabSrc : Src<S, false> {
    using Base = Src<S, false>;
    Stamp<ST> st;
    bool prefetched;          // this tile's first R-1 DMAs were issued by the previous tile
    bool has_next;            // persistent: nx is the tile after this one
    Base nx;

    __device__ __forceinline__ void issue(int x, const typename Base::Pre &pr) const {
        if (PERS && prefetched && x < S::R - 1) return;
        Base::issue(x, pr);
    }
    mutable uint64_t c_cmp = 0, c_dma = 0, c_bar = 0, c_last = 0;
    template <int T, int I>
    __device__ __forceinline__ void wait() const {
        if (ST && !PERS) {  // split the wait: own DMAs (vmcnt), then the barrier
            constexpr int N = (I - T - 1) * S::DPW;
            uint64_t t0, t1, t2;
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
            if (S::NDMA % S::NW != 0 && this->wave * S::DPW >= S::NDMA)
                asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
            else
                asm volatile("s_waitcnt vmcnt(%1)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1) : "n"(N) : "memory");
            asm volatile("s_barrier\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t2)::"memory");
            if (T != 3) c_cmp += t0 - c_last;
            c_dma += t1 - t0;
            c_bar += t2 - t1;
            c_last = t2;
            if (T == 3) st.put(1);
            st.put(6 + T / 4);
            return;
        }
        // persistent: the previous tile's 16 epilogue stores were issued after this tile's first
        // R-1 DMAs, so a wait for one of those DMAs leaves the stores outstanding
        if (PERS && prefetched && T < S::R - 1) {
            constexpr int N = (I - T - 1) * S::DPW + 16;
            static_assert(N < 64, "vmcnt");
            if (S::NDMA % S::NW != 0 && this->wave * S::DPW >= S::NDMA)
                asm volatile("s_barrier" ::: "memory");
            else
                asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
        } else {
            Base::template wait<T, I>();
        }
        if (T == 3) st.put(1);  // the first wait of the schedule (S = 4)
        st.put(6 + T / 4);
    }
    __device__ __forceinline__ void release() const {
        st.put(2);
        if (ST && !PERS && (threadIdx.x & 63) == 0) {
            uint64_t *q = st.p + 64 + 3 * this->wave;
            q[0] = c_cmp;
            q[1] = c_dma;
            q[2] = c_bar;
        }
        Base::release();  // every wave is past its last ring read
        if (PERS && has_next) {
            typename Base::Pre pr;
#pragma unroll
            for (int t = 0; t < S::R - 1; ++t) nx.issue(t, pr);
        }
    }
};

__device__ __forceinline__ int prologue(const FixedArgs &a, uint8_t *lds, uint8_t *scratch, Src<S, false> &src,
                                        Sink &sink, long long col0) {
    WGInfo w;
    w.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    w.lane = threadIdx.x & 63;
    const int part = w.wave % S::P;
    const int cw = w.wave / S::P;
    w.c = cw * 64 + w.lane;
    w.col0 = col0;
    w.lo = 0;
    w.hi = static_cast<long long>(a.groups) * a.geo.nq;
    const int nq = a.geo.nq;
    w.g_first = static_cast<int>((col0 > 0 ? col0 : 0) / nq);
    const long long col = w.col0 + w.c;
    w.valid = col >= w.lo && col < w.hi;
    const int g = w.valid ? static_cast<int>(col / nq) : w.g_first;
    w.q = static_cast<int>(col - static_cast<long long>(g) * nq);
    w.gl = g - w.g_first;
    src.init(a, w, lds, lds);
    sink.init(a, w, scratch + w.wave * 2048);
    return part;
}

__device__ __forceinline__ uint32_t hwid() {
    const uint32_t hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));    // HW_REG_HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11));  // HW_REG_XCC_ID
    return (xcc & 0xF) << 16 | (hw >> 8 & 0xFFFF);
}

// Timing-only (wrong results): each wave stores its rows as whole aligned 2 KB runs (the same
// number of bytes as the product's output, in full 128-byte lines).
struct ContigSink : Sink {
    uint32_t cbase;
    __device__ __forceinline__ void store_row(int y, const uint32_t (&w)[8]) const {
#pragma unroll
        for (int b = 0; b < 8; ++b) reinterpret_cast<uint32_t *>(scr)[b * 64 + lane] = w[b];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int i = lane + 64 * h;
            const u32x4 v = *reinterpret_cast<const u32x4 *>(scr + (i >> 4) * 256 + (i & 15) * 16);
            __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, cbase + h * 1024 + lane * 16, static_cast<uint32_t>(y & 7) * 2048u, 0);
        }
    }
};

// Timing-only (wrong results): every DMA source rounded down to 16 bytes.
template <class L>
__device__ __forceinline__ void align_src(L &src) {
#pragma unroll
    for (int j = 0; j < S::DPW; ++j)
        if (src.dbase[j] != OOR) src.dbase[j] &= ~15u;
}

// MODE 0: base (scratch aliases ring); 1: sep; 2: pers; 3: base with 16-byte-aligned DMA sources;
// 7: RowSink (row-assembled stores, correct results);
// 4: base with ContigSink stores; 5: aligned DMA + ContigSink; 6: pers + aligned DMA + ContigSink
template <int MODE, bool ST>
__global__ __launch_bounds__(S::NT, 4) void kern(FixedArgs a, uint64_t *stamps, int ntiles) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint8_t *scratch = (MODE == 0 || MODE == 3) ? lds : lds + S::R * S::SLOT;
    if (MODE != 2 && MODE != 6) {
        const int tile = xcd_tile(blockIdx.x, gridDim.x);
        LabSrc<false, ST> src;
        src.st.p = stamps + static_cast<size_t>(tile) * NSTAMP;
        src.st.put(0);
        src.prefetched = false;
        src.has_next = false;
        Sink sink;
        const int part = prologue(a, lds, scratch, src, sink, static_cast<long long>(tile) * S::COLS);
        if (MODE == 3 || MODE == 5) align_src(src);
        if (MODE == 7) {
            RowSink<S> rs;
            WGInfo w;
            w.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
            w.lane = threadIdx.x & 63;
            w.c = (w.wave / S::P) * 64 + w.lane;
            w.col0 = static_cast<long long>(tile) * S::COLS;
            w.lo = 0;
            w.hi = static_cast<long long>(a.groups) * a.geo.nq;
            w.g_first = static_cast<int>(w.col0 / a.geo.nq);
            rs.init(a, w, part, lds);
            run_k200_m32_enc(part, src, rs);
        } else if (MODE >= 4) {
            ContigSink cs;
            static_cast<Sink &>(cs) = sink;
            cs.rsrc = make_rsrc(a.out, static_cast<uint32_t>(a.out_bytes < 0x7FFFFFFFll ? a.out_bytes : 0x7FFFFFFFll));
            cs.cbase = (static_cast<uint32_t>(tile) * S::NW + static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(threadIdx.x >> 6))) * 16384u;
            run_k200_m32_enc(part, src, cs);
        } else {
            run_k200_m32_enc(part, src, sink);
        }
        src.st.put(3);
        if (ST && threadIdx.x == 0) stamps[static_cast<size_t>(tile) * NSTAMP + 4] = hwid() | (uint64_t)blockIdx.x << 32;
        return;
    }
    LabSrc<true, ST> cur;
    Sink sink, nsink;
    int v = blockIdx.x;
    if (v >= ntiles) return;
    int tile = xcd_tile(v, ntiles);
    int part = prologue(a, lds, scratch, cur, sink, static_cast<long long>(tile) * S::COLS);
    if (MODE == 6) align_src(cur);
    cur.prefetched = false;
    for (;;) {
        cur.st.p = stamps + static_cast<size_t>(tile) * NSTAMP;
        cur.st.put(0);
        const int vn = v + gridDim.x;
        const int tn = vn < ntiles ? xcd_tile(vn, ntiles) : -1;
        cur.has_next = tn >= 0;
        if (tn >= 0) prologue(a, lds, scratch, cur.nx, nsink, static_cast<long long>(tn) * S::COLS);
        if (MODE == 6) {
            if (tn >= 0) align_src(cur.nx);
            ContigSink cs;
            static_cast<Sink &>(cs) = sink;
            cs.rsrc = make_rsrc(a.out, static_cast<uint32_t>(a.out_bytes < 0x7FFFFFFFll ? a.out_bytes : 0x7FFFFFFFll));
            cs.cbase = (static_cast<uint32_t>(tile) * S::NW + static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(threadIdx.x >> 6))) * 16384u;
            run_k200_m32_enc(part, cur, cs);
        } else {
            run_k200_m32_enc(part, cur, sink);
        }
        cur.st.put(3);
        if (ST && threadIdx.x == 0) stamps[static_cast<size_t>(tile) * NSTAMP + 4] = hwid() | (uint64_t)blockIdx.x << 32;
        if (tn < 0) break;
        static_cast<Src<S, false> &>(cur) = cur.nx;
        cur.prefetched = true;
        sink = nsink;
        v = vn;
        tile = tn;
    }
}

__global__ void fill(uint32_t *p, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t x = static_cast<uint32_t>(i) * 0x9E3779B9u ^ seed;
        x ^= x >> 16; x *= 0x85EBCA6Bu; x ^= x >> 13; x *= 0xC2B2AE35u; x ^= x >> 16;
        p[i] = x;
    }
}

__global__ void diff(const uint32_t *a, const uint32_t *b, size_t n, unsigned long long *cnt) {
    unsigned long long c = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        c += a[i] != b[i];
    if (c) atomicAdd(cnt, c);
}
}  // namespace lab

int main(int argc, char **argv) {
    using namespace lab;
    int groups = 8192, iters = 30;
    const char *only = nullptr;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--groups")) groups = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--iters")) iters = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--only")) only = argv[++i];
    }
    const int k = 200, m = 32, B = 1400;
    FixedArgs a{};
    a.geo = make_geometry(B);
    a.geo = fixed_geometry(B);
    a.groups = groups;
    a.in_gstride = (long long)k * B;
    a.in_bytes = a.in_gstride * groups;
    a.out_gstride = (long long)m * B;
    a.out_bytes = a.out_gstride * groups;
    uint8_t *in, *out, *ref;
    CK(hipMalloc(&in, a.in_bytes));
    CK(hipMalloc(&out, a.out_bytes));
    CK(hipMalloc(&ref, a.out_bytes));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint32_t *)in, (size_t)a.in_bytes / 4, 0x1234u);
    a.in = in;
    a.groups_per_wg = (S::COLS - 1) / a.geo.nq + 2;
    const long long cols = (long long)groups * a.geo.nq;
    const int ntiles = (int)((cols + S::COLS - 1) / S::COLS);
    uint64_t *stamps;
    CK(hipMalloc(&stamps, (size_t)ntiles * NSTAMP * 8));
    unsigned long long *cnt;
    CK(hipMalloc(&cnt, 8));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;

    struct V { const char *name; void (*k)(FixedArgs, uint64_t *, int); void (*ks)(FixedArgs, uint64_t *, int); size_t lds; int grid; };
    const size_t ring = (size_t)S::R * S::SLOT, scr = (size_t)S::NW * 2048;
    std::vector<V> vs = {
        {"base", kern<0, false>, kern<0, true>, ring, ntiles},
#ifdef LAB_MORE
        {"pers", kern<2, false>, kern<2, true>, ring + scr, 2 * cus},
#endif
#ifndef LAB_ONLY_PERS
        {"sep", kern<1, false>, nullptr, ring + scr, ntiles},
        {"algn", kern<3, false>, kern<3, true>, ring, ntiles},
#endif
#ifndef LAB_ONLY_PERS
        {"cstore", kern<4, false>, nullptr, ring, ntiles},
        {"alcst", kern<5, false>, nullptr, ring, ntiles},
#endif
#ifdef LAB_MORE
        {"palcst", kern<6, false>, nullptr, ring + scr, 2 * cus},
#endif
        {"rows", kern<7, false>, kern<7, true>, ring, ntiles},
    };
    printf("tiles %d, R %d, lds base %zu sep %zu, CUs %d\n", ntiles, S::R, ring, ring + scr, cus);
    for (auto &v : vs) {
        CK(hipFuncSetAttribute((const void *)v.k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)v.lds));
        if (v.ks) CK(hipFuncSetAttribute((const void *)v.ks, hipFuncAttributeMaxDynamicSharedMemorySize, (int)v.lds));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    bool have_ref = false;
    for (auto &v : vs) {
        if (only && !strstr(only, v.name)) continue;
        a.out = out;
        CK(hipMemset(out, 0, a.out_bytes));
        hipLaunchKernelGGL(v.k, dim3(v.grid), dim3(S::NT), v.lds, 0, a, nullptr, ntiles);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        if (!have_ref) {
            CK(hipMemcpy(ref, out, a.out_bytes, hipMemcpyDeviceToDevice));
            have_ref = true;
        } else {
            CK(hipMemset(cnt, 0, 8));
            hipLaunchKernelGGL(diff, dim3(2048), dim3(256), 0, 0, (const uint32_t *)out, (const uint32_t *)ref,
                               (size_t)a.out_bytes / 4, cnt);
            unsigned long long c;
            CK(hipMemcpy(&c, cnt, 8, hipMemcpyDeviceToHost));
            printf("%-6s mismatching dwords vs first variant: %llu\n", v.name, c);
        }
        std::vector<float> ms;
        for (int it = 0; it < 5; ++it) hipLaunchKernelGGL(v.k, dim3(v.grid), dim3(S::NT), v.lds, 0, a, nullptr, ntiles);
        for (int it = 0; it < iters; ++it) {
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(v.k, dim3(v.grid), dim3(S::NT), v.lds, 0, a, nullptr, ntiles);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        const double alg = (double)groups * (k + m) * B;
        printf("%-6s min %.4f med %.4f ms  (%.0f GB/s at median)\n", v.name, ms[0], ms[ms.size() / 2],
               alg / ms[ms.size() / 2] / 1e6);
        if (!v.ks) continue;
        // stamped run
        CK(hipMemset(stamps, 0, (size_t)ntiles * NSTAMP * 8));
        hipLaunchKernelGGL(v.ks, dim3(v.grid), dim3(S::NT), v.lds, 0, a, stamps, ntiles);
        CK(hipDeviceSynchronize());
        std::vector<uint64_t> h((size_t)ntiles * NSTAMP);
        CK(hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost));
        char fn[256];
        snprintf(fn, sizeof fn, "gpurun_out/lab_stamps_%s.csv", v.name);
        FILE *f = fopen(fn, "w");
        if (f) {
            fprintf(f, "tile,start,first,last,end,xcc,hwid,block,waits,wavecyc\n");
            for (int t = 0; t < ntiles; ++t) {
                const uint64_t *r = &h[(size_t)t * NSTAMP];
                fprintf(f, "%d,%llu,%llu,%llu,%llu,%u,%u,%u,", t, (unsigned long long)r[0], (unsigned long long)r[1],
                        (unsigned long long)r[2], (unsigned long long)r[3], (unsigned)(r[4] >> 16 & 0xF),
                        (unsigned)(r[4] & 0xFFFF), (unsigned)(r[4] >> 32));
                for (int j = 6; j < 56; ++j) fprintf(f, "%lld ", r[j] ? (long long)(r[j] - r[0]) : -1ll);
                fprintf(f, ",");
                for (int j = 64; j < 88; ++j) fprintf(f, "%llu ", (unsigned long long)r[j]);
                fprintf(f, "\n");
            }
            fclose(f);
        }
    }
    return 0;
}
