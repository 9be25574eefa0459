// Host side of libcauchy256.so: the drop-in cauchy_256.h ABI and the batched device ABI.
//
// Every coding call runs on the GPU. The single-group reference entry points
// (cauchy_256_encode / cauchy_256_decode, reference cauchy_256.cpp:1479 / :1233) gather the
// caller's host blocks into pinned staging, run the batched kernels with groups = 1 and scatter
// the result back; there is deliberately no CPU implementation of the codec in this library.
// Without a usable GPU every call prints an error and returns -2.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <array>
#include <atomic>
#include <condition_variable>
#include <memory>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "../../include/cauchy_256.h"
#include "../../include/cauchy_256_batch.h"
#include "cauchy_math.hpp"
#include "colsnip.h"
#include "kernels.hpp"
#include "measure.hpp"

namespace {

using sh::Geometry;

#define SH_CHECK(expr)                                                                        \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess) {                                                               \
            std::fprintf(stderr, "libcauchy256: %s failed: %s (%s:%d)\n", #expr,             \
                         hipGetErrorString(_e), __FILE__, __LINE__);                          \
            return -2;                                                                        \
        }                                                                                     \
    } while (0)

inline int round4(int x) { return (x + 3) & ~3; }

// Grow-only device buffer. `owner` (if any) is the only stream that uses it: growing waits for
// that stream before freeing the old allocation.
struct DevBuf {
    void *p = nullptr;
    size_t n = 0;
    int ensure(size_t bytes, hipStream_t owner = nullptr) {
        if (bytes <= n) return 0;
        if (p) {
            (void)hipStreamSynchronize(owner);
            (void)hipFree(p);
        }
        p = nullptr;
        n = 0;
        if (hipMalloc(&p, bytes) != hipSuccess) {
            std::fprintf(stderr, "libcauchy256: hipMalloc(%zu) failed\n", bytes);
            return -2;
        }
        n = bytes;
        return 0;
    }
};

struct PinnedBuf {
    void *p = nullptr;
    size_t n = 0;
    int ensure(size_t bytes) {
        if (bytes <= n) return 0;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
            std::fprintf(stderr, "libcauchy256: hipHostMalloc(%zu) failed\n", bytes);
            return -2;
        }
        n = bytes;
        return 0;
    }
};

// Per-stream decode state: the workspace and the malformed-group counter of the decodes enqueued
// on that stream. `mu` is held from the workspace lookup until the call's kernels are enqueued, so a
// concurrent grow (another thread on the same stream, or cauchy_256_batch_reserve_stream) can never
// free a buffer that a call is about to use; calls on one stream are then ordered by the stream.
struct StreamState {
    std::mutex mu;
    DevBuf ws;
    int *d_errors = nullptr;
    // split-tile scratch of the compile-time kernels (lease_split), its own lock: a decode holds
    // `mu` while it launches stage A, which takes this one too
    std::mutex split_mu;
    DevBuf split;
};

// One launch of the tile kernels: output rows [row0, row0 + nrows) with its snippet-address table.
struct TileLaunch {
    int row0, nrows, nsteps;
    long long tstride;
    uint32_t *targets;  // device [parts][tstride]
    bool col;           // column snippets (2 dwords per step) instead of per-row snippets (8)
    uint32_t hi;        // high dword of every snippet address of the launch
};

// Staging of one single-group call (cauchy_256_encode / cauchy_256_decode): pinned host and
// device buffers and its own stream, so calls from different threads -- e.g. two Shorthair codec
// objects -- copy and compute concurrently instead of queueing on one buffer and one stream. The
// reference codec is reentrant per call (cauchy_256.cpp keeps no state beyond its init tables).
struct StageSlot {
    hipStream_t stream = nullptr;
    PinnedBuf h;
    DevBuf d;
};
constexpr size_t kMaxStageSlots = 8;  // concurrent single-group calls; more threads wait for a slot

struct Context {
    std::mutex mu;          // guards lazy state (tables, caches, the stream map, profiling events)
    bool ready = false;
    int device = 0;
    hipStream_t stream = nullptr;
    uint64_t snip_base = 0;           // stage-B snippet table address (code object)
    uint64_t col_base[SH_COL_TUS] = {};  // column-snippet tables (csrc/gen/colsnip_<t>.hip)
    bool col_ok = false;              // ... all inside one 4 GB page (the kernels take low dwords)
    uint64_t *d_rowbytes = nullptr;   // 256 x 8 bytes
    uint8_t *d_exp = nullptr;         // 512
    uint16_t *d_log = nullptr;        // 256
    // (k, m) -> device generator: [m][round4(k)] coefficients (row 0 = ones) for encode,
    // followed by the raw (m-1) x k rows 1..m-1 and the Cauchy parameters X'[k], Y'[m] for
    // decode setup.
    std::map<std::pair<int, int>, uint8_t *> gens;
    // (k, m, dec) -> launches of the runtime-coefficient tile kernels (csrc/tile_snip.hip)
    std::map<std::array<int, 3>, std::vector<TileLaunch>> tiles;
    // Decode state per stream: two decodes in flight on different streams never share scratch.
    std::map<hipStream_t, std::unique_ptr<StreamState>> streams;
    std::atomic<size_t> ws_reserve{0};  // cauchy_256_batch_reserve: minimum size of a workspace
    // stage timing (cauchy_256_profile): per profiled decode, events around setup / stage A /
    // stage B, in a ring of `evq.size()` quadruples (no host synchronisation while recording)
    std::vector<std::array<hipEvent_t, 4>> evq;
    int ev_next = 0, ev_count = 0;
    bool ev_stage_a_only = false;  // cauchy_256_profile(-n): two events per decode, around stage A
    // single-group staging slots (SlotLease): a call holds one for its whole duration
    std::mutex stage_mu;
    std::condition_variable stage_cv;
    std::vector<std::unique_ptr<StageSlot>> stage_all;
    std::vector<StageSlot *> stage_free;
};

Context &ctx() {
    static Context c;
    return c;
}

int init_locked(Context &c, int device) {
    if (c.ready) return 0;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        std::fprintf(stderr, "libcauchy256: no HIP device available; the codec runs only on the GPU\n");
        return -2;
    }
    if (device < 0 || device >= n) device = 0;
    SH_CHECK(hipSetDevice(device));
    SH_CHECK(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
    const sh::GF256 &f = sh::gf();
    uint64_t rb[256];
    for (int v = 0; v < 256; ++v) {
        uint64_t w = 0;
        for (int b = 0; b < 8; ++b) w |= static_cast<uint64_t>(f.row_bytes[v][b]) << (8 * b);
        rb[v] = w;
    }
    SH_CHECK(hipMalloc(&c.d_rowbytes, sizeof rb));
    SH_CHECK(hipMemcpy(c.d_rowbytes, rb, sizeof rb, hipMemcpyHostToDevice));
    SH_CHECK(hipMalloc(&c.d_exp, 512));
    SH_CHECK(hipMemcpy(c.d_exp, f.exp, 512, hipMemcpyHostToDevice));
    SH_CHECK(hipMalloc(&c.d_log, 512));
    SH_CHECK(hipMemcpy(c.d_log, f.log, 512, hipMemcpyHostToDevice));
    SH_CHECK(sh::stageb_snip_base(&c.snip_base, c.stream));
    SH_CHECK(sh::colsnip_bases(c.col_base, SH_COL_TUS, c.stream));
    {
        // every column-snippet address must share one high dword and have a non-zero low dword
        // (0 means "no call" to the kernels)
        const uint64_t hi0 = c.col_base[0] >> 32;
        bool ok = true;
        for (int t = 0; t < SH_COL_TUS; ++t) {
            const uint64_t n = static_cast<uint64_t>(SH_COL_BLOCKS_PER_TU) * 256 + (t == 0 ? 9 : 0);
            const uint64_t lo = c.col_base[t], hi = lo + n * SH_COL_STRIDE;
            ok = ok && (lo >> 32) == hi0 && (hi >> 32) == hi0 && static_cast<uint32_t>(lo) != 0;
        }
        c.col_ok = ok;
    }
    c.device = device;
    c.ready = true;
    return 0;
}

// Every entry point runs on the library's device, whatever the calling thread had current (HIP's
// current device is per thread; allocations and launches follow it), and gives the thread its
// previous device back when it returns: construct one at the top of each entry point.
struct DeviceScope {
    int rc = 0, prev = -1, dev = -1;
    explicit DeviceScope(Context &c) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        {
            std::lock_guard<std::mutex> g(c.mu);
            rc = init_locked(c, c.device);
        }
        if (rc) return;
        dev = c.device;
        if (prev != dev && hipSetDevice(dev) != hipSuccess) {
            std::fprintf(stderr, "libcauchy256: hipSetDevice(%d) failed\n", dev);
            rc = -2;
        }
    }
    ~DeviceScope() {
        if (prev >= 0 && dev >= 0 && prev != dev) (void)hipSetDevice(prev);
    }
    DeviceScope(const DeviceScope &) = delete;
    DeviceScope &operator=(const DeviceScope &) = delete;
};

// The decode state of `stream` (created on first use, never destroyed: the map owns it).
StreamState *stream_state(Context &c, hipStream_t stream) {
    std::lock_guard<std::mutex> g(c.mu);
    auto &slot = c.streams[stream];
    if (!slot) {
        auto st = std::make_unique<StreamState>();
        if (hipMalloc(&st->d_errors, sizeof(int)) != hipSuccess) return nullptr;
        if (hipMemset(st->d_errors, 0, sizeof(int)) != hipSuccess) {
            (void)hipFree(st->d_errors);
            return nullptr;
        }
        slot = std::move(st);
    }
    return slot.get();
}

// A stream's workspace, locked for one call: at least `bytes` (and the reserve), valid while the
// lease lives. Kernels enqueued under the lease are ordered before any later grow's free by the
// grow's stream synchronisation.
struct WsLease {
    std::unique_lock<std::mutex> lk;
    uint8_t *p = nullptr;
    int *errors = nullptr;
};

// reserve = false: the single-group calls' staging streams, sized by their own need only (up to
// 8 of them; cauchy_256_batch_reserve is for the batched calls' streams).
int lease_workspace(Context &c, hipStream_t stream, size_t bytes, WsLease &out, bool reserve = true) {
    StreamState *st = stream_state(c, stream);
    if (!st) return -2;
    out.lk = std::unique_lock<std::mutex>(st->mu);
    if (st->ws.ensure(reserve ? std::max(bytes, c.ws_reserve.load()) : bytes, stream)) return -2;
    out.p = static_cast<uint8_t *>(st->ws.p);
    out.errors = st->d_errors;
    return 0;
}

// Split-tile scratch of a stream (fixed_common.hpp RowSink "Split tiles": the last tiles of a
// compile-time launch run as two half-step workgroups whose partial rows meet here): 64 MB of
// partials and one arrival counter per split tile, zeroed once when allocated (every launch
// leaves them zero: the second arriver resets its tile's). Locked for one launch; launches on one
// stream are ordered by the stream.
constexpr size_t kSplitPartBytes = 64ull << 20;
constexpr int kSplitMinGroups = 16;  // smaller batches: whole tiles (no scratch for the stream)
// Only the A/B builds generate split-tile programs (tools/gen_fixed_kernels.py SH_SPLIT_GEN=1,
// measured no faster: profiles/r06/ab_runs.txt block 2); the product never leases the scratch.
#ifdef SH_MEASUREMENT_BUILD
constexpr bool kSplitLaunch = true;
#else
constexpr bool kSplitLaunch = false;
#endif
constexpr int kSplitCounters = 4096;
struct SplitLease {
    std::unique_lock<std::mutex> lk;
    uint8_t *part = nullptr;
    uint32_t *cnt = nullptr;
};
int lease_split(Context &c, hipStream_t stream, SplitLease &out) {
    StreamState *st = stream_state(c, stream);
    if (!st) return -2;
    out.lk = std::unique_lock<std::mutex>(st->split_mu);
    if (!st->split.p) {
        if (st->split.ensure(kSplitPartBytes + kSplitCounters * sizeof(uint32_t), stream)) return -2;
        if (hipMemsetAsync(static_cast<uint8_t *>(st->split.p) + kSplitPartBytes, 0,
                           kSplitCounters * sizeof(uint32_t), stream) != hipSuccess)
            return -2;
    }
    out.part = static_cast<uint8_t *>(st->split.p);
    out.cnt = reinterpret_cast<uint32_t *>(out.part + kSplitPartBytes);
    return 0;
}

// Device generator for (k, m), m >= 2, k + m <= 256. Cached; created once per shape.
uint8_t *generator(Context &c, int k, int m) {
    std::lock_guard<std::mutex> g(c.mu);
    auto it = c.gens.find({k, m});
    if (it != c.gens.end()) return it->second;
    const std::vector<uint8_t> G = sh::generator_matrix(k, m);
    std::vector<uint8_t> xp, yp;
    sh::cauchy_params(k, m, xp, yp);
    const int ld = round4(k);
    const size_t raw = static_cast<size_t>(m) * ld;
    const size_t par = raw + static_cast<size_t>(m - 1) * k;
    std::vector<uint8_t> host(par + k + m, 0);
    for (int y = 0; y < m; ++y) std::memcpy(&host[static_cast<size_t>(y) * ld], &G[static_cast<size_t>(y) * k], k);
    std::memcpy(&host[raw], &G[k], static_cast<size_t>(m - 1) * k);
    std::memcpy(&host[par], xp.data(), k);
    std::memcpy(&host[par + k], yp.data(), m);
    uint8_t *d = nullptr;
    if (hipMalloc(&d, host.size()) != hipSuccess) return nullptr;
    if (hipMemcpy(d, host.data(), host.size(), hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    c.gens[{k, m}] = d;
    return d;
}

// Whether (k, m, B) can run on the runtime-coefficient tile kernels: fixed_geometry's 16-byte
// chunks (B/8 >= 16) and a snippet table inside one 4 GB page (the kernels form the snippet
// addresses from their low dwords).
bool tile_usable(Context &c, int k, int m, int B) {
    if (k < 2 || m < 2 || k + m > 256 || !sh::tile_ok(B)) return false;
    if (SH_MEASURE_ENV("SH_NO_TILE")) return false;  // measurement switch: the older generic kernels
    const uint64_t lo = c.snip_base, hi = c.snip_base + static_cast<uint64_t>(sh::SNIP_NULL + 1) * sh::SNIP_STRIDE;
    return (lo >> 32) == (hi >> 32);
}

// Measurement switch (never the default): SH_FORCE_TILE=1 routes shapes that have compile-time
// kernels through the tile kernels too, to compare the two on the same shape.
bool force_tile() {
    static const bool f = SH_MEASURE_ENV("SH_FORCE_TILE") != nullptr;
    return f;
}

// Launch plan of the tile kernels for (k, m): <= 128 rows per launch; per launch and part-wave a
// table of snippet-address low dwords, [step][8] per part (reference generator cauchy_matrix(),
// cauchy_256.cpp:423-481, row 0 = ones). Decode (stage A): steps 0..k-1 are the received columns,
// step k + i adds recovery row row0 + i into its residual row (coefficient 1 on that row only).
const std::vector<TileLaunch> *tile_plan(Context &c, int k, int m, bool dec) {
    std::lock_guard<std::mutex> g(c.mu);
    auto it = c.tiles.find({k, m, dec ? 1 : 0});
    if (it != c.tiles.end()) return &it->second;
    const std::vector<uint8_t> G = sh::generator_matrix(k, m);  // [m][k], row 0 = ones
    const uint32_t base = static_cast<uint32_t>(c.snip_base);
    auto addr = [&](int cf) { return base + static_cast<uint32_t>(cf ? cf : sh::SNIP_NULL) * sh::SNIP_STRIDE; };
    // Decode stage A at m >= 7 runs column snippets (csrc/gen/colsnip_<t>.hip: one call per 4
    // rows, addressed by the input's Cauchy parameter X'_x, as the rows' Y' are the same for every
    // m; no VGPR-index mode): (150,40) 1.231 vs 1.317 ms, (180,76) 2.72 vs 2.82, (120,136) 3.83 vs
    // 4.37, (90,49) 0.98 vs 1.12 against the per-row snippets. Encode keeps the per-row snippets
    // ((180,76) 2.30 vs 2.43 ms; the others within 5 %): a column snippet's table (16 KB per
    // generator row) misses the instruction cache where the 18 KB per-row table stays resident.
    // SH_NO_COL / SH_COL_ENC: measurement switches.
    static const bool no_col = SH_MEASURE_ENV("SH_NO_COL") != nullptr;
    static const bool col_enc = SH_MEASURE_ENV("SH_COL_ENC") != nullptr;
    const bool col = m >= 7 && c.col_ok && !no_col && (dec || col_enc);
    std::vector<uint8_t> xp, yp;
    if (col) sh::cauchy_params(k, m, xp, yp);
    auto col_addr = [&](int blk, int v) {  // block = 4 generator rows
        const int tu = blk / SH_COL_BLOCKS_PER_TU, loc = blk - tu * SH_COL_BLOCKS_PER_TU;
        return static_cast<uint32_t>(c.col_base[tu] + (static_cast<uint64_t>(loc) * 256 + v) * SH_COL_STRIDE);
    };
    std::vector<TileLaunch> plan;
    for (int row0 = 0; row0 < m; row0 += 128) {
        TileLaunch L{};
        L.row0 = row0;
        L.nrows = std::min(128, m - row0);
        L.nsteps = k + (dec ? L.nrows : 0);
        L.col = col;
        L.hi = static_cast<uint32_t>((col ? c.col_base[0] : c.snip_base) >> 32);
        const int parts = sh::tile_parts(L.nrows);
        const int S = sh::tile_steps_per_group(parts);
        const int per = col ? 2 : 8;
        L.tstride = static_cast<long long>((L.nsteps + S - 1) / S) * S * per;
        // + 128 dwords of slack: a step slice's last scalar loads may run up to S - 1 steps past
        // the part's table (into the next part's, or this slack after the last)
        std::vector<uint32_t> t(static_cast<size_t>(parts) * L.tstride + 128, 0u);  // 0: no call
        const int nb4 = (L.nrows + 3) / 4;
        for (int p = 0; p < parts; ++p) {
            if (col) {
                // part p: 4-row blocks [b0, b1) (one or two; tile_snip.hip computes the same)
                const int b0 = p * nb4 / parts, b1 = (p + 1) * nb4 / parts;
                const int yend = std::min(4 * b1, L.nrows);
                for (int x = 0; x < L.nsteps; ++x) {
                    uint32_t *e = &t[static_cast<size_t>(p) * L.tstride + static_cast<size_t>(x) * 2];
                    if (x < k) {
                        for (int i = 0; i < b1 - b0; ++i) e[i] = col_addr(row0 / 4 + b0 + i, xp[x]);
                    } else {
                        const int yy = x - k;  // decode: recovery row yy into its residual row
                        if (yy >= 4 * b0 && yy < yend)
                            e[0] = static_cast<uint32_t>(c.col_base[0] + SH_COL_UNIT((yy - 4 * b0 + 4 * (b0 & 1)) & 7));
                    }
                }
                continue;
            }
            // part p: rows [p * nrows / parts, (p + 1) * nrows / parts) (tile_snip.hip)
            const int y0 = p * L.nrows / parts, y1 = (p + 1) * L.nrows / parts;
            for (int x = 0; x < L.nsteps; ++x) {
                uint32_t *e = &t[static_cast<size_t>(p) * L.tstride + static_cast<size_t>(x) * 8];
                if (x >= k) {  // decode recovery-row step: the unit snippet on its row, no other call
                    const int yy = x - k;
                    if (yy >= y0 && yy < y1) e[yy - y0] = addr(1);
                    continue;
                }
                for (int j = 0; j < y1 - y0; ++j) {  // zero coefficient: no call
                    const int cf = G[static_cast<size_t>(row0 + y0 + j) * k + x];
                    e[j] = cf ? addr(cf) : 0u;
                }
            }
        }
        if (hipMalloc(&L.targets, t.size() * sizeof(uint32_t)) != hipSuccess) return nullptr;
        if (hipMemcpy(L.targets, t.data(), t.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess)
            return nullptr;
        plan.push_back(L);
    }
    return &(c.tiles[{k, m, dec ? 1 : 0}] = std::move(plan));
}

// Batched calls take the caller's stream verbatim (NULL = the null stream, as in HIP itself).
hipStream_t pick(void *stream) { return static_cast<hipStream_t>(stream); }

// One launch of a compile-time-scheduled kernel over the whole batch (the kernels build their
// buffer descriptors per workgroup, so 32-bit offsets never limit the batch size).
// split: the stream's split-tile scratch (nullptr: whole tiles only).
hipError_t launch_fixed_batch(int k, int m, int B, int groups, const uint8_t *in, long long in_gs,
                              uint8_t *out, long long out_gs, const uint8_t *pos,
                              const uint8_t *rpos, bool dec, hipStream_t s, const SplitLease *split = nullptr) {
    sh::FixedArgs a{};
    if (split) {
        a.split_part = split->part;
        a.split_cnt = split->cnt;
        a.split_cap = static_cast<long long>(kSplitPartBytes);
        a.split_max = kSplitCounters;
    }
    a.in = in;
    a.in_gstride = in_gs;
    a.in_bytes = static_cast<long long>(groups) * in_gs;
    a.out = out;
    a.out_gstride = out_gs;
    a.out_bytes = static_cast<long long>(groups) * out_gs;
    a.groups = groups;
    a.geo = sh::fixed_geometry(B);
    a.pos = pos;
    a.rpos = rpos;
    return sh::launch_fixed(k, m, a, dec, s);
}

// Step slices of the single-group latency path: the k (+ m) serial ring steps of one group are
// split over up to 32 workgroups, each XOR-ing its steps' products into a partial output, and the
// partials are XOR-reduced (the products are linear). >= 6 steps per slice.
constexpr int kSliceCap = 32;  // slice_scratch holds this many partial outputs
int latency_slices(int nsteps) {
    // SH_SLICE_MAX / SH_SLICE_STEPS: measurement switches (slices at most, steps per slice at least)
    // (200,32,1400) single-group calls: 8 x 25 steps 80 / 112 us (encode / decode), 16 x 12 74 / 104,
    // 32 x 6 70 / 104 (profiles/r05/ab_runs.txt block 13)
    static const int mx = sh::measure_int(SH_MEASURE_ENV("SH_SLICE_MAX"), 32);
    static const int st = sh::measure_int(SH_MEASURE_ENV("SH_SLICE_STEPS"), 6);
    return std::max(1, std::min(std::min(mx, kSliceCap), nsteps / std::max(st, 1)));
}

// One pass of the tile kernels over the batch (encode, or decode stage A with position tables).
// slice_scratch (groups == 1 only): room for latency_slices() partial outputs of m * B bytes;
// the steps are then sliced and the partials XOR-reduced into `out`.
int launch_tile_batch(Context &c, int k, int m, int B, int groups, const uint8_t *in, long long in_gs,
                      uint8_t *out, long long out_gs, const uint8_t *pos, const uint8_t *rpos, bool dec,
                      hipStream_t s, uint8_t *slice_scratch = nullptr) {
    const std::vector<TileLaunch> *plan = tile_plan(c, k, m, dec);
    if (!plan) return -2;
    for (const TileLaunch &L : *plan) {
        const int parts = sh::tile_parts(L.nrows);
        const int S = sh::tile_steps_per_group(parts);
        const int ns = (slice_scratch && groups == 1) ? latency_slices(L.nsteps) : 1;
        sh::TileArgs t{};
        t.f.in = in;
        t.f.in_gstride = in_gs;
        t.f.in_bytes = static_cast<long long>(groups) * in_gs;
        t.f.out = out + static_cast<long long>(L.row0) * B;
        t.f.out_gstride = out_gs;
        t.f.out_bytes = static_cast<long long>(groups) * out_gs - static_cast<long long>(L.row0) * B;
        t.f.groups = groups;
        t.f.geo = sh::fixed_geometry(B);
        t.f.pos = pos;
        t.f.rpos = rpos;
        t.targets = L.targets;
        t.tstride = L.tstride;
        t.snip_hi = L.hi;
        t.col = L.col ? 1 : 0;
        t.k = k;
        t.m = m;
        t.row0 = L.row0;
        t.nrows = L.nrows;
        t.nsteps = L.nsteps;
        if (ns > 1) {
            // slices of a multiple of S steps; partial p at slice_scratch + p * m * B (row r of the
            // launch at + (row0 + r) * B, like the final output)
            const int per = ((L.nsteps + ns - 1) / ns + S - 1) / S * S;
            t.slice_steps = per;
            t.slices = (L.nsteps + per - 1) / per;
            t.out_slice_bytes = out_gs;
            t.f.out = slice_scratch + static_cast<long long>(L.row0) * B;
            t.f.out_bytes = out_gs - static_cast<long long>(L.row0) * B;
            SH_CHECK(sh::launch_tile(t, dec, s));
            SH_CHECK(sh::launch_xor_reduce(slice_scratch + static_cast<long long>(L.row0) * B, out_gs, t.slices,
                                           out + static_cast<long long>(L.row0) * B,
                                           static_cast<long long>(L.nrows) * B, s));
        } else {
            SH_CHECK(sh::launch_tile(t, dec, s));
        }
    }
    return 0;
}

// ---- batched encode ----
// slice_scratch (single-group ABI): kSliceCap * m * B device bytes that let one group's steps run as
// parallel slices on the tile kernels (latency); nullptr = the throughput kernels.
int encode_batch(int k, int m, int B, int groups, const uint8_t *d_in, uint8_t *d_out,
                 hipStream_t s, uint8_t *slice_scratch = nullptr) {
    Context &c = ctx();
    DeviceScope ds(c);
    if (ds.rc) return ds.rc;
    if (groups <= 0 || m <= 0 || k <= 0 || B <= 0) return 0;
    const long long in_gs = static_cast<long long>(k) * B, out_gs = static_cast<long long>(m) * B;
    if (k <= 1) {  // reference cauchy_256.cpp:1485-1493
        SH_CHECK(sh::launch_copy_first(d_in, in_gs, d_out, out_gs, m, B, groups, s));
        return 0;
    }
    const bool valid = (k + m <= 256) && (B % 8 == 0);
    if (m == 1 || !valid) {
        // Row 0 (plain XOR, any B) is written even when the parameters are then rejected
        // (reference cauchy_256.cpp:1496-1511).
        SH_CHECK(sh::launch_xor_rows(d_in, in_gs, k, d_out, out_gs, B, groups, s));
        return (m == 1 || valid) ? 0 : -1;  // m == 1 returns before validation (:1503-1506)
    }
    const bool sliced = slice_scratch && groups == 1 && tile_usable(c, k, m, B) && latency_slices(k) > 1;
    if (sh::has_fixed(k, m, B) && !force_tile() && !sliced) {
        SplitLease sp;
        const bool split = kSplitLaunch && groups >= kSplitMinGroups;
        if (split)
            if (int rc = lease_split(c, s, sp)) return rc;
        SH_CHECK(launch_fixed_batch(k, m, B, groups, d_in, in_gs, d_out, out_gs, nullptr, nullptr,
                                    false, s, split ? &sp : nullptr));
        return 0;
    }
    if (tile_usable(c, k, m, B))
        return launch_tile_batch(c, k, m, B, groups, d_in, in_gs, d_out, out_gs, nullptr, nullptr, false, s,
                                 sliced ? slice_scratch : nullptr);
    uint8_t *gen = generator(c, k, m);
    if (!gen) return -2;
    sh::ApplyArgs a{};
    a.in = d_in;
    a.in_gstride = in_gs;
    a.in_bstride = B;
    a.n_in = k;
    a.out = d_out;
    a.out_gstride = out_gs;
    a.out_bstride = B;
    a.n_out = m;  // row 0 = coefficient 1 everywhere: M(1) is the identity, i.e. plain XOR
    a.n_out_g = nullptr;
    a.coef = gen;
    a.coef_gstride = 0;
    a.coef_ld = round4(k);
    a.rowbytes = c.d_rowbytes;
    a.groups = groups;
    a.geo = sh::make_geometry(B);
    SH_CHECK(sh::launch_apply(a, false, s));
    return 0;
}

// Workspace carve for decode of `groups` groups.
struct DecodeWS {
    bool fixed;       // stage A by a compile-time-scheduled kernel, stage B by stageb_fixed
    bool small;       // ... and stage B by stageb_small (nq <= 16 word columns: byte coefficients)
    bool v2;          // ... or by stageb_v2 (byte coefficients, one workgroup per group chunk)
    int emax, ldA, ldB, nres;  // nres: residual rows per group (m when fixed, else emax)
    int kp;           // position-table stride: round4 of the stage-A kernel's K (a compiled K > k
                      // codes k, sh::fixed_kernel_k; the entries past k stay 0xFF)
    int *e;
    uint8_t *rec_idx, *erasures, *coefA, *coefB, *residual, *recovered, *pos, *rpos, *rrow;
    uint64_t *targets;
    long long coefA_gs, coefB_gs;
};

// Stage B after a full-residual stage A: stageb_v2 for emax > 8, where it measured faster
// ((200,32) e = 32: 0.34 vs 0.39 ms; (200,56) e = 56: 0.478 vs 0.532 ms; (190,66) e = 66: 0.763 vs
// 0.838 ms and (120,136) e = 120: 1.77 vs 2.07 ms against stageb_fixed, with 4- or 8-wave chunks;
// C2 (64,16) e = 16: 0.229 vs 0.280 ms and (112,16) 0.142 vs 0.177 ms against stageb_regs, with
// 2-wave workgroups and an 8-row ring, stageb.hip); round 2's stageb_regs with setup-written
// snippet addresses for emax <= 8 ((28,4,1400) 0.114 vs 0.132 ms for a one-wave v2).
// SH_STAGEB_OLD=1 (measurement switch) selects round 2's kernels everywhere; SH_V2_MIN / SH_V2_MAX
// bound the emax served by stageb_v2.
bool stageb_v2_on(const sh::Geometry &geo, int emax) {
    static const bool old = SH_MEASURE_ENV("SH_STAGEB_OLD") != nullptr;
    static const int vmax = sh::measure_int(SH_MEASURE_ENV("SH_V2_MAX"), 128);  // measurement
    static const int vmin = sh::measure_int(SH_MEASURE_ENV("SH_V2_MIN"), 8);    // measurement
    return !old && emax > vmin && emax <= vmax && sh::stageb_v2_ok(geo, emax);
}

size_t carve(DecodeWS &w, uint8_t *base, int k, int m, int B, int groups, bool need_recovered) {
    const sh::Geometry geo = sh::fixed_geometry(B);
    w.emax = std::min(k, m);
    // stage A over all m rows (compile-time or tile kernels), position tables, snippet stage B
    w.fixed = (sh::has_fixed(k, m, B) || tile_usable(ctx(), k, m, B)) && sh::stageb_fixed_ok(geo, w.emax);
    const int kfix = force_tile() ? 0 : sh::fixed_kernel_k(k, m, B);
    w.kp = round4(std::max(k, kfix));
    w.small = w.fixed && sh::stageb_small_ok(geo, w.emax);
    w.ldA = w.fixed ? 0 : round4(k);
    w.ldB = (w.emax + 7) & ~7;  // stage-B coefficients [i][ldB] (transposed, 8-entry rows)
    w.nres = w.fixed ? m : w.emax;
    w.coefA_gs = static_cast<long long>(w.emax) * w.ldA;
    w.coefB_gs = static_cast<long long>(w.emax) * w.ldB;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        uint8_t *p = base ? base + off : nullptr;
        off += (bytes + 255) & ~static_cast<size_t>(255);
        return p;
    };
    const size_t G = static_cast<size_t>(groups);
    w.e = reinterpret_cast<int *>(take(G * sizeof(int)));
    w.rec_idx = take(G * w.emax);
    w.erasures = take(G * w.emax);
    w.coefA = w.fixed ? nullptr : take(G * w.coefA_gs);
    w.coefB = (w.fixed && !w.small && !stageb_v2_on(geo, w.emax)) ? nullptr : take(G * w.coefB_gs);
    w.v2 = w.fixed && !w.small && stageb_v2_on(geo, w.emax);
    w.targets = (w.fixed && !w.small && !w.v2)
                    ? reinterpret_cast<uint64_t *>(take(G * w.emax * w.ldB * sizeof(uint64_t)))
                    : nullptr;
    w.rrow = w.fixed ? take(G * round4(w.emax)) : nullptr;
    w.pos = w.fixed ? take(G * w.kp) : nullptr;
    w.rpos = w.fixed ? take(G * round4(m)) : nullptr;
    w.residual = take(G * w.nres * static_cast<size_t>(B) + 256);  // + slack: word over-read
    w.recovered = need_recovered ? take(G * w.emax * static_cast<size_t>(B)) : nullptr;
    return off;
}

// Rows per stage-B slice on the single-group latency path (SH_SB_SLICE, measurement switch; 0 = one
// workgroup streams all e rows).
int stageb_row_slice() {
    static const int n = sh::measure_int(SH_MEASURE_ENV("SH_SB_SLICE"), 8);
    return std::max(0, n);
}

// slice_scratch (groups == 1, stageb_v2 only): the e input rows are split into slices of
// stageb_row_slice() rows, one workgroup each, whose partial outputs are XOR-reduced into dst.
hipError_t launch_stage_b(const DecodeWS &w, int n_in, int B, int groups, uint8_t *dst, hipStream_t s,
                          uint8_t *slice_scratch = nullptr) {
    if (w.small) {
        sh::StageBSmallArgs f{};
        f.in = w.residual;
        f.in_gstride = static_cast<long long>(n_in) * B;
        f.out = dst;
        f.out_gstride = static_cast<long long>(w.emax) * B;
        f.e = w.e;
        f.rrow = w.rrow;
        f.ldR = round4(w.emax);
        f.coefT = w.coefB;
        f.coefT_gstride = w.coefB_gs;
        f.ldT = w.ldB;
        f.emax = w.emax;
        f.groups = groups;
        f.geo = sh::fixed_geometry(B);
        return sh::launch_stageb_small(f, s);
    }
    if (w.v2) {
        sh::StageBV2Args f{};
        f.in = w.residual;
        f.in_gstride = static_cast<long long>(n_in) * B;
        f.out = dst;
        f.out_gstride = static_cast<long long>(w.emax) * B;
        f.e = w.e;
        f.rrow = w.rrow;
        f.ldR = round4(w.emax);
        f.coefT = w.coefB;
        f.coefT_gstride = w.coefB_gs;
        f.ldT = w.ldB;
        f.emax = w.emax;
        f.groups = groups;
        f.geo = sh::fixed_geometry(B);
        f.snip_base = ctx().snip_base;
        // at most kSliceCap partial outputs fit slice_scratch (a small measurement
        // setting of SH_SB_SLICE must not write past it)
        const int rs0 = stageb_row_slice();
        const int rs = rs0 > 0 ? std::max(rs0, (w.emax + kSliceCap - 1) / kSliceCap) : 0;
        if (slice_scratch && groups == 1 && rs > 0 && w.emax > rs) {
            f.row_slice = rs;
            f.row_slices = (w.emax + rs - 1) / rs;
            f.out_slice_bytes = f.out_gstride;
            f.out = slice_scratch;
            if (hipError_t r = sh::launch_stageb_v2(f, s)) return r;
            return sh::launch_xor_reduce(slice_scratch, f.out_gstride, f.row_slices, dst, f.out_gstride, s);
        }
        return sh::launch_stageb_v2(f, s);
    }
    if (w.fixed) {
        sh::StageBFixedArgs f{};
        f.in = w.residual;
        f.in_gstride = static_cast<long long>(n_in) * B;
        f.out = dst;
        f.out_gstride = static_cast<long long>(w.emax) * B;
        f.e = w.e;
        f.rrow = w.rrow;
        f.targets = w.targets;
        f.emax = w.emax;
        f.ldR = round4(w.emax);
        f.ldT = w.ldB;
        f.groups = groups;
        f.geo = sh::fixed_geometry(B);
        return sh::launch_stageb_fixed(f, s);
    }
    sh::StageBArgs b{};
    b.in = w.residual;
    b.in_gstride = static_cast<long long>(n_in) * B;
    b.n_in = n_in;
    b.out = dst;
    b.out_gstride = static_cast<long long>(w.emax) * B;
    b.e = w.e;
    b.coefT = w.coefB;
    b.coefT_gstride = w.coefB_gs;
    b.ldT = w.ldB;
    b.groups = groups;
    b.geo = sh::make_geometry(B);
    return sh::launch_stageb(b, w.emax, s);
}

// Common decode core (m >= 2, valid params): writes recovered blocks densely into `dst`
// ([G][emax][B]) and leaves per-group e / rec_idx / erasures in the workspace.
// host_setup: the workspace's setup fields were written by the host (single-group ABI,
// host_decode_setup below) and arrive with the blocks: no setup kernel.
int decode_core(Context &c, int k, int m, int B, int groups, const uint8_t *d_blocks,
                const uint8_t *d_rows, DecodeWS &w, int *errors, uint8_t *dst, hipStream_t s,
                uint8_t *slice_scratch = nullptr, bool host_setup = false) {
    uint8_t *gen = generator(c, k, m);
    if (!gen) return -2;
    sh::DecodeSetupArgs sa{};
    sa.k = k;
    sa.m = m;
    sa.rows = d_rows;
    sa.rows_gstride = k;
    sa.gen = gen + static_cast<size_t>(m) * round4(k);
    sa.xp = sa.gen + static_cast<size_t>(m - 1) * k;
    sa.yp = sa.xp + k;
    sa.gf_exp = c.d_exp;
    sa.gf_log = c.d_log;
    sa.emax = w.emax;
    sa.e_out = w.e;
    sa.rec_idx = w.rec_idx;
    sa.erasures = w.erasures;
    sa.coefA = w.coefA;
    sa.coefA_gstride = w.coefA_gs;
    sa.ldA = w.ldA;
    sa.coefB = w.coefB;
    sa.coefB_gstride = w.coefB_gs;
    sa.ldB = w.ldB;
    sa.pos = w.pos;
    sa.kp = w.kp;
    sa.rpos = w.rpos;
    sa.rrow = w.rrow;
    sa.ldR = round4(w.emax);
    sa.targets = w.targets;
    sa.snip_base = c.snip_base;
    sa.errors = errors;
    hipEvent_t *ev = nullptr;
    {  // check and claim the slot in one critical section (profile() may resize the ring)
        std::lock_guard<std::mutex> g(c.mu);
        if (!c.evq.empty()) {
            ev = c.evq[c.ev_next].data();
            c.ev_next = (c.ev_next + 1) % static_cast<int>(c.evq.size());
            c.ev_count = std::min(c.ev_count + 1, static_cast<int>(c.evq.size()));
        }
    }
    // stage-A-only profiling records ev[1] and ev[2] alone (fewer event packets in a timed loop)
    bool ev_all = false;
    if (ev) {
        std::lock_guard<std::mutex> g(c.mu);
        ev_all = !c.ev_stage_a_only;
    }
    if (ev && ev_all) SH_CHECK(hipEventRecord(ev[0], s));
    if (!host_setup) SH_CHECK(sh::launch_decode_setup(sa, groups, s));
    if (ev) SH_CHECK(hipEventRecord(ev[1], s));

    const Geometry geo = sh::make_geometry(B);
    if (w.fixed) {
        // Stage A (compile-time generator, all m rows, erased columns read as zeros):
        //   residual_y = R_y + sum_{received x} M(C[y][x]) d_x
        // (the tile kernels read position tables round4(k) wide: not after a wider compiled K)
        const bool sliced = slice_scratch && groups == 1 && tile_usable(c, k, m, B) && latency_slices(k + m) > 1 &&
                            w.kp == round4(k);
        if (sh::has_fixed(k, m, B) && !force_tile() && !sliced) {
            SplitLease sp;
            const bool split = kSplitLaunch && groups >= kSplitMinGroups;
            if (split)
                if (int rc = lease_split(c, s, sp)) return rc;
            SH_CHECK(launch_fixed_batch(k, m, B, groups, d_blocks, static_cast<long long>(k) * B,
                                        w.residual, static_cast<long long>(m) * B, w.pos, w.rpos, true, s,
                                        split ? &sp : nullptr));
        } else if (int rc = launch_tile_batch(c, k, m, B, groups, d_blocks, static_cast<long long>(k) * B,
                                              w.residual, static_cast<long long>(m) * B, w.pos, w.rpos, true, s,
                                              sliced ? slice_scratch : nullptr)) {
            return rc;
        }
        if (ev) SH_CHECK(hipEventRecord(ev[2], s));
        // Stage B: recovered_j = sum_y M(S^-1[j][i(y)]) residual_y over the received rows y
        SH_CHECK(launch_stage_b(w, m, B, groups, dst, s, groups == 1 ? slice_scratch : nullptr));
        if (ev && ev_all) SH_CHECK(hipEventRecord(ev[3], s));
        return 0;
    }
    // Stage A: residual_i = R_i + sum_{orig j} M(C[r_i][row_j]) d_j  (per-group coefficients)
    sh::ApplyArgs a{};
    a.in = d_blocks;
    a.in_gstride = static_cast<long long>(k) * B;
    a.in_bstride = B;
    a.n_in = k;
    a.out = w.residual;
    a.out_gstride = static_cast<long long>(w.emax) * B;
    a.out_bstride = B;
    a.n_out = w.emax;
    a.n_out_g = w.e;
    a.coef = w.coefA;
    a.coef_gstride = w.coefA_gs;
    a.coef_ld = w.ldA;
    a.rowbytes = c.d_rowbytes;
    a.groups = groups;
    a.geo = geo;
    SH_CHECK(sh::launch_apply(a, true, s));
    // Stage B: recovered_j = sum_i M(S^-1[j][i]) residual_i
    SH_CHECK(launch_stage_b(w, w.emax, B, groups, dst, s));
    return 0;
}

int invalid_decode_status(int k, int groups, const uint8_t *d_rows, hipStream_t s) {
    std::vector<uint8_t> rows(static_cast<size_t>(groups) * k);
    SH_CHECK(hipMemcpyAsync(rows.data(), d_rows, rows.size(), hipMemcpyDeviceToHost, s));
    SH_CHECK(hipStreamSynchronize(s));
    for (uint8_t r : rows)
        if (r >= k) return -1;
    return 0;
}

// Host restatement of decode_setup (kernels.hip) for one group, written into a host image of the
// workspace carved exactly as the device's (carve()): the single-group ABI uploads it with the
// blocks, so its decode runs no setup kernel. Covers the modes whose stage B takes byte
// coefficients (stageb_v2, stageb_small) after a full-residual stage A, for m >= 7 (closed-form
// Cauchy inverse, kernels.hip decode_setup: S^-1[j][i] = a_j b_i / (x_j (x_j + y_i))); returns
// false (device setup) otherwise. rec[i]: array index of the i-th recovery block, era[j]: j-th
// erased original row (sort_blocks order, cauchy_256.cpp:522-554), 0 < e <= number of erasures.
bool host_decode_setup(const DecodeWS &w, int k, int m, const uint8_t *rows, int e, const int *rec,
                       const int *era) {
    if (!w.fixed || !(w.v2 || w.small) || m < 7 || !w.coefB || !w.rrow || !w.pos || !w.rpos) return false;
    const sh::GF256 &f = sh::gf();
    std::vector<uint8_t> xp, yp;
    sh::cauchy_params(k, m, xp, yp);
    *w.e = e;
    std::memset(w.rrow, 0, round4(w.emax));
    std::memset(w.pos, 0xFF, w.kp);
    std::memset(w.rpos, 0xFF, round4(m));
    for (int j = 0; j < k; ++j) {
        if (rows[j] < k) w.pos[rows[j]] = static_cast<uint8_t>(j);
        else w.rpos[rows[j] - k] = static_cast<uint8_t>(j);
    }
    int x[256], y[256], la[256], lb[256];
    for (int t = 0; t < e; ++t) {
        w.rec_idx[t] = static_cast<uint8_t>(rec[t]);
        w.erasures[t] = static_cast<uint8_t>(era[t]);
        w.rrow[t] = static_cast<uint8_t>(rows[rec[t]] - k);
        x[t] = xp[era[t]];
        y[t] = yp[rows[rec[t]] - k];
    }
    auto mod255 = [](int v) { v %= 255; return v < 0 ? v + 255 : v; };
    for (int t = 0; t < e; ++t) {
        int a = 0, b = 0;
        for (int q = 0; q < e; ++q) {
            a += f.log[x[t] ^ y[q]];
            b += f.log[x[q] ^ y[t]];
            if (q != t) {
                a -= f.log[x[t] ^ x[q]];
                b -= f.log[y[t] ^ y[q]];
            }
        }
        la[t] = mod255(a - f.log[x[t]]);
        lb[t] = mod255(b);
    }
    std::memset(w.coefB, 0, static_cast<size_t>(w.emax) * w.ldB);  // [i][j] = S^-1[j][i], zero past e
    for (int i = 0; i < e; ++i)
        for (int j = 0; j < e; ++j)
            w.coefB[static_cast<size_t>(i) * w.ldB + j] = f.exp[mod255(la[j] + lb[i] - f.log[x[j] ^ y[i]])];
    return true;
}

// e_host (optional, pinned host memory): receives group 0's e, copied on `s` while the workspace
// is still leased to this call (the single-group ABI reads it after synchronising).
// h_dense (single-group ABI, optional): the e_dense recovered rows of group 0 are copied densely
// into this pinned buffer instead of being scattered on the device (the caller knows the
// recovery positions and places them itself).
// ws_ext (single-group ABI, optional): the workspace, carved by the caller in its staging
// buffer (no lease); host_setup: its setup fields are already there (decode_core).
int decode_batch(int k, int m, int B, int groups, uint8_t *d_blocks, uint8_t *d_rows,
                 hipStream_t s, int *e_host = nullptr, uint8_t *slice_scratch = nullptr,
                 uint8_t *h_dense = nullptr, int e_dense = 0, uint8_t *ws_ext = nullptr,
                 bool host_setup = false) {
    Context &c = ctx();
    DeviceScope ds(c);
    if (ds.rc) return ds.rc;
    if (groups <= 0 || k <= 0) return 0;
    if (k <= 1) {  // cauchy_256.cpp:1236-1240
        SH_CHECK(sh::launch_decode_k1(d_rows, k, groups, s));
        return 0;
    }
    if (m == 1) {  // cauchy_256.cpp:1243-1246 (no parameter check on this path)
        SH_CHECK(sh::launch_decode_m1(d_blocks, static_cast<long long>(k) * B, d_rows, k, k, B, groups, s));
        return 0;
    }
    if (k + m > 256 || B % 8 != 0) return invalid_decode_status(k, groups, d_rows, s);
    DecodeWS w{};
    WsLease ls;
    if (ws_ext) {
        carve(w, ws_ext, k, m, B, groups, true);
    } else {
        // slice_scratch: the single-group ABI (a staging stream, no batch reserve)
        if (int rc = lease_workspace(c, s, carve(w, nullptr, k, m, B, groups, true), ls, slice_scratch == nullptr)) return rc;
        carve(w, ls.p, k, m, B, groups, true);
    }
    if (int rc = decode_core(c, k, m, B, groups, d_blocks, d_rows, w, ws_ext ? nullptr : ls.errors, w.recovered, s,
                             slice_scratch, host_setup))
        return rc;
    if (h_dense) {  // still under the workspace lease: the copy is ordered before any regrowth
        SH_CHECK(hipMemcpyAsync(h_dense, w.recovered, static_cast<size_t>(e_dense) * B, hipMemcpyDeviceToHost, s));
        return 0;
    }
    sh::ScatterArgs sc{};
    sc.src = w.recovered;
    sc.src_gstride = static_cast<long long>(w.emax) * B;
    sc.blocks = d_blocks;
    sc.blocks_gstride = static_cast<long long>(k) * B;
    sc.rows = d_rows;
    sc.rows_gstride = k;
    sc.e = w.e;
    sc.rec_idx = w.rec_idx;
    sc.erasures = w.erasures;
    sc.emax = w.emax;
    sc.B = B;
    SH_CHECK(sh::launch_scatter(sc, groups, s));
    if (e_host) SH_CHECK(hipMemcpyAsync(e_host, w.e, sizeof(int), hipMemcpyDeviceToHost, s));
    return 0;
}

}  // namespace

// =============================================================================================
// Batched device ABI (cauchy_256_batch.h)
// =============================================================================================
extern "C" int cauchy_256_batch_init(int device) {
    Context &c = ctx();
    std::lock_guard<std::mutex> g(c.mu);
    return init_locked(c, device);
}

extern "C" int cauchy_256_encode_batch(int k, int m, int block_bytes, int groups,
                                       const void *d_data, void *d_recovery, void *stream) {
    return encode_batch(k, m, block_bytes, groups, static_cast<const uint8_t *>(d_data),
                        static_cast<uint8_t *>(d_recovery), pick(stream));
}

extern "C" int cauchy_256_decode_batch(int k, int m, int block_bytes, int groups, void *d_blocks,
                                       unsigned char *d_rows, void *stream) {
    return decode_batch(k, m, block_bytes, groups, static_cast<uint8_t *>(d_blocks), d_rows,
                        pick(stream));
}

extern "C" int cauchy_256_decode_batch_out(int k, int m, int block_bytes, int groups,
                                           const void *d_blocks, const unsigned char *d_rows,
                                           void *d_out, unsigned char *d_out_rows,
                                           int *d_out_count, void *stream) {
    Context &c = ctx();
    DeviceScope ds(c);
    if (ds.rc) return ds.rc;
    if (groups <= 0) return 0;
    if (k < 2 || m < 2) return -1;
    hipStream_t s = pick(stream);
    if (k + m > 256 || block_bytes % 8 != 0) return invalid_decode_status(k, groups, d_rows, s);
    DecodeWS w{};
    WsLease ls;
    if (int rc = lease_workspace(c, s, carve(w, nullptr, k, m, block_bytes, groups, false), ls)) return rc;
    carve(w, ls.p, k, m, block_bytes, groups, false);
    // the setup writes the erasure list ([G][emax]) and the counts ([G]) straight into the
    // caller's outputs (same layouts as the workspace's): no copies after the decode
    w.erasures = d_out_rows;
    w.e = d_out_count;
    return decode_core(c, k, m, block_bytes, groups, static_cast<const uint8_t *>(d_blocks), d_rows, w,
                       ls.errors, static_cast<uint8_t *>(d_out), s);
}

extern "C" int cauchy_256_batch_reserve(int k, int m, int block_bytes, int groups) {
    return cauchy_256_batch_reserve_stream(k, m, block_bytes, groups, nullptr);
}

extern "C" int cauchy_256_batch_reserve_stream(int k, int m, int block_bytes, int groups, void *stream) {
    Context &c = ctx();
    DeviceScope ds(c);
    if (ds.rc) return ds.rc;
    if (k < 2 || m < 2 || k + m > 256 || block_bytes <= 0 || groups <= 0) return 0;
    DecodeWS w{};
    const size_t need = carve(w, nullptr, k, m, block_bytes, groups, true);
    if (!generator(c, k, m)) return -2;
    size_t cur = c.ws_reserve.load();
    while (cur < need && !c.ws_reserve.compare_exchange_weak(cur, need)) {
    }
    WsLease ls;
    return lease_workspace(c, pick(stream), need, ls);
}

extern "C" int cauchy_256_batch_errors(void *stream) {
    Context &c = ctx();
    DeviceScope ds(c);
    if (ds.rc) return ds.rc;
    hipStream_t s = pick(stream);
    StreamState *st = stream_state(c, s);
    if (!st) return -2;
    // Read and clear in stream order, under the stream's lock: a decode enqueued on this stream
    // (by any thread) lands either before the read or after the clear, never in between.
    std::lock_guard<std::mutex> g(st->mu);
    int *n = nullptr;
    SH_CHECK(hipHostMalloc(reinterpret_cast<void **>(&n), sizeof(int), hipHostMallocDefault));
    *n = 0;
    hipError_t e = hipMemcpyAsync(n, st->d_errors, sizeof(int), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipMemsetAsync(st->d_errors, 0, sizeof(int), s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    const int r = *n;
    (void)hipHostFree(n);
    if (e != hipSuccess) {
        std::fprintf(stderr, "libcauchy256: batch_errors failed: %s\n", hipGetErrorString(e));
        return -2;
    }
    return r;
}

extern "C" int cauchy_256_fill_synthetic(void *d_out, int n, int block_bytes, int groups,
                                         unsigned long long g0, unsigned long long cfg,
                                         void *stream) {
    Context &c = ctx();
    DeviceScope ds(c);
    if (ds.rc) return ds.rc;
    SH_CHECK(sh::launch_fill(static_cast<uint8_t *>(d_out), static_cast<long long>(n) * block_bytes,
                             n, block_bytes, groups, g0, cfg, pick(stream)));
    return 0;
}

// Synthetic erasure pattern of group g (host integers, no GPU): the same PCG32 stream and
// partial Fisher-Yates picks as the test oracle's generator (oracle/cauchy_oracle.c), so the
// benchmark's decode inputs match the parity tests'. Survivors ascending, then the chosen
// recovery rows (k + y) ascending; returns the erasure count e.
extern "C" int cauchy_256_erasure_pattern(unsigned long long g, int k, int m, unsigned long long cfg,
                                          int e_fixed, unsigned char *rows_out) {
    if (k <= 0 || m <= 0 || k + m > 256 || !rows_out) return -1;
    const uint64_t inc = (static_cast<uint64_t>(g) << 1) | 1ull;
    uint64_t state = 0;
    auto next = [&]() {
        const uint64_t old = state;
        state = old * 6364136223846793005ull + inc;
        const uint32_t xs = static_cast<uint32_t>(((old >> 18) ^ old) >> 27);
        const uint32_t rot = static_cast<uint32_t>(old >> 59);
        return (xs >> rot) | (xs << ((32u - rot) & 31u));
    };
    next();
    state += cfg ^ 0xE7A5ull;
    next();
    const int emax = std::min(k, m);
    const int e = e_fixed > 0 ? std::min(e_fixed, emax) : 1 + static_cast<int>(next() % static_cast<uint32_t>(emax));
    uint8_t pk[256], pm[256];
    bool lost[256] = {}, used[256] = {};
    for (int i = 0; i < k; ++i) pk[i] = static_cast<uint8_t>(i);
    for (int i = 0; i < m; ++i) pm[i] = static_cast<uint8_t>(i);
    for (int i = 0; i < e; ++i) {
        std::swap(pk[i], pk[i + static_cast<int>(next() % static_cast<uint32_t>(k - i))]);
        std::swap(pm[i], pm[i + static_cast<int>(next() % static_cast<uint32_t>(m - i))]);
        lost[pk[i]] = true;
        used[pm[i]] = true;
    }
    int n = 0;
    for (int x = 0; x < k; ++x)
        if (!lost[x]) rows_out[n++] = static_cast<uint8_t>(x);
    for (int y = 0; y < m; ++y)
        if (used[y]) rows_out[n++] = static_cast<uint8_t>(k + y);
    return e;
}

extern "C" int cauchy_256_batch_path(int k, int m, int block_bytes) {
    if (k < 1 || m < 1 || k + m > 256 || block_bytes <= 0 || block_bytes % 8 != 0) return -1;
    if (sh::has_fixed(k, m, block_bytes) && !force_tile()) return 1;
    // Host-only answer (a launcher may ask before it spawns rank processes, so this never
    // initialises the GPU): the snippet table's one-4-GB-page condition needs the loaded code
    // object and is checked at launch (generic kernels otherwise); once the library is
    // initialised the answer includes it.
    if (k < 2 || m < 2 || !sh::tile_ok(block_bytes) || SH_MEASURE_ENV("SH_NO_TILE")) return 0;
    Context &c = ctx();
    std::lock_guard<std::mutex> g(c.mu);
    return !c.ready || tile_usable(c, k, m, block_bytes) ? 2 : 0;
}

extern "C" void *cauchy_256_default_stream(void) {
    Context &c = ctx();
    DeviceScope ds(c);
    if (ds.rc) return nullptr;
    return c.stream;
}

extern "C" int cauchy_256_profile(int capacity) {
    Context &c = ctx();
    DeviceScope ds(c);
    if (ds.rc) return ds.rc;
    std::lock_guard<std::mutex> g(c.mu);
    for (auto &q : c.evq)
        for (hipEvent_t e : q) (void)hipEventDestroy(e);
    c.ev_stage_a_only = capacity < 0;
    if (capacity < 0) capacity = -capacity;
    c.evq.assign(std::max(0, capacity), {});
    for (auto &q : c.evq)
        for (hipEvent_t &e : q) SH_CHECK(hipEventCreate(&e));
    c.ev_next = c.ev_count = 0;
    return 0;
}

extern "C" int cauchy_256_profile_read(float *ms) {
    Context &c = ctx();
    std::lock_guard<std::mutex> g(c.mu);
    if (c.ev_count == 0) return -1;
    double sum[3] = {0, 0, 0};
    const bool a_only = c.ev_stage_a_only;
    for (int i = 0; i < c.ev_count; ++i) {
        const auto &q = c.evq[i];
        SH_CHECK(hipEventSynchronize(q[a_only ? 2 : 3]));
        for (int t = a_only ? 1 : 0; t < (a_only ? 2 : 3); ++t) {
            float x = 0;
            SH_CHECK(hipEventElapsedTime(&x, q[t], q[t + 1]));
            sum[t] += x;
        }
    }
    for (int t = 0; t < 3; ++t) ms[t] = (a_only && t != 1) ? -1.0f : static_cast<float>(sum[t] / c.ev_count);
    return c.ev_count;
}

extern "C" int cauchy_256_sync(void *stream) {
    Context &c = ctx();
    DeviceScope ds(c);
    if (ds.rc) return ds.rc;
    SH_CHECK(hipStreamSynchronize(pick(stream)));
    return 0;
}

// =============================================================================================
// Drop-in single-group ABI (cauchy_256.h). One group per call through a pinned staging slot with
// its own stream (SlotLease): concurrent calls from different threads overlap on the GPU.
// =============================================================================================
// The reference's exported product/quotient tables (cauchy_256.cpp:346-347, built by GFC256Init
// :349-386 on the first _cauchy_256_init): 256 x 256 bytes each, entry (y << 8) + x = x * y and
// x / y in GF(256)/0x187, zero rows and columns for 0. Exported for symbol parity with
// cauchy_256.o; the codec itself does not read them. Null until the first successful version check.
extern "C" {
__attribute__((visibility("default"))) uint8_t *GFC256_MUL_TABLE = nullptr;
__attribute__((visibility("default"))) uint8_t *GFC256_DIV_TABLE = nullptr;
}

namespace {
void export_field_tables() {
    static std::once_flag once;
    std::call_once(once, [] {
        static uint8_t tab[2][256 * 256];
        const sh::GF256 &f = sh::gf();
        for (int y = 0; y < 256; ++y)
            for (int x = 0; x < 256; ++x) {
                tab[0][(y << 8) + x] = f.mul(static_cast<uint8_t>(x), static_cast<uint8_t>(y));
                tab[1][(y << 8) + x] = f.div(static_cast<uint8_t>(x), static_cast<uint8_t>(y));
            }
        GFC256_DIV_TABLE = tab[1];
        GFC256_MUL_TABLE = tab[0];
    });
}
}  // namespace

namespace {
// A staging slot for the duration of one call: a free one, a new one while fewer than
// kMaxStageSlots exist, else the next one released. `rc` != 0: no slot (stream creation failed).
struct SlotLease {
    Context &c;
    StageSlot *s = nullptr;
    int rc = 0;
    explicit SlotLease(Context &cx) : c(cx) {
        std::unique_lock<std::mutex> lk(c.stage_mu);
        for (;;) {
            if (!c.stage_free.empty()) {
                s = c.stage_free.back();
                c.stage_free.pop_back();
                return;
            }
            if (c.stage_all.size() < kMaxStageSlots) break;
            c.stage_cv.wait(lk);
        }
        auto slot = std::make_unique<StageSlot>();
        if (hipStreamCreateWithFlags(&slot->stream, hipStreamNonBlocking) != hipSuccess) {
            std::fprintf(stderr, "libcauchy256: hipStreamCreateWithFlags failed\n");
            rc = -2;
            return;
        }
        s = slot.get();
        c.stage_all.push_back(std::move(slot));
    }
    ~SlotLease() {
        if (!s) return;
        {
            std::lock_guard<std::mutex> g(c.stage_mu);
            c.stage_free.push_back(s);
        }
        c.stage_cv.notify_one();
    }
    SlotLease(const SlotLease &) = delete;
    SlotLease &operator=(const SlotLease &) = delete;
};
}  // namespace

extern "C" int _cauchy_256_init(int expected_version) {
    if (expected_version != CAUCHY_256_VERSION) return -1;  // reference cauchy_256.cpp:392-394
    export_field_tables();
    Context &c = ctx();
    std::lock_guard<std::mutex> g(c.mu);
    return init_locked(c, c.device);
}

extern "C" int cauchy_256_encode(int k, int m, const unsigned char *data_ptrs[],
                                 void *recovery_blocks, int block_bytes) {
    Context &c = ctx();
    DeviceScope ds(c);
    if (ds.rc) return ds.rc;
    if (k <= 0 || m <= 0 || block_bytes <= 0) return 0;
    const int kin = k <= 1 ? 1 : k;
    const size_t in_bytes = static_cast<size_t>(kin) * block_bytes;
    const size_t out_bytes = static_cast<size_t>(m) * block_bytes;
    SlotLease sl(c);
    if (sl.rc) return sl.rc;
    StageSlot &st = *sl.s;
    const size_t scratch = kSliceCap * out_bytes;  // step-slice partials (latency path)
    if (int rc = st.h.ensure(in_bytes + out_bytes)) return rc;
    if (int rc = st.d.ensure(in_bytes + out_bytes + scratch, st.stream)) return rc;
    uint8_t *h = static_cast<uint8_t *>(st.h.p);
    uint8_t *d = static_cast<uint8_t *>(st.d.p);
    for (int x = 0; x < kin; ++x) std::memcpy(h + static_cast<size_t>(x) * block_bytes, data_ptrs[x], block_bytes);
    SH_CHECK(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, st.stream));
    const int rc = encode_batch(k, m, block_bytes, 1, d, d + in_bytes, st.stream, d + in_bytes + out_bytes);
    if (rc == -2) {
        (void)hipStreamSynchronize(st.stream);  // the slot is released on return
        return rc;
    }
    // Like the reference, a rejected call has still written recovery row 0.
    const size_t copy = (rc == 0) ? out_bytes : static_cast<size_t>(block_bytes);
    SH_CHECK(hipMemcpyAsync(h + in_bytes, d + in_bytes, copy, hipMemcpyDeviceToHost, st.stream));
    SH_CHECK(hipStreamSynchronize(st.stream));
    std::memcpy(recovery_blocks, h + in_bytes, copy);
    return rc;
}

extern "C" int cauchy_256_decode(int k, int m, Block *blocks, int block_bytes) {
    Context &c = ctx();
    DeviceScope ds(c);
    if (ds.rc) return ds.rc;
    if (k <= 1) {  // cauchy_256.cpp:1236-1240: no data touched
        if (k == 1) blocks[0].row = 0;
        return 0;
    }
    if (block_bytes <= 0) return 0;
    // The reference's sort_blocks (cauchy_256.cpp:522-554) on the host: the recovery blocks in
    // array order receive the erased originals in increasing order. A row listed twice, a row
    // past the generator or more recovery blocks than erasures is outside the reference's
    // contract: rejected (-1) before any GPU work, as the device setup would report it.
    const bool general = m >= 2 && k + m <= 256 && block_bytes % 8 == 0;
    int rec[256], era[256], e = 0, nera = 0;
    if (general) {
        uint8_t seen[256] = {};
        for (int i = 0; i < k; ++i) {
            const int r = blocks[i].row;
            if (r >= k + m || seen[r]++) return -1;
            if (r >= k) rec[e++] = i;
        }
        for (int x = 0; x < k; ++x)
            if (!seen[x]) era[nera++] = x;
        if (e > nera) return -1;
        if (e == 0) return 0;
    }
    const size_t data_bytes = static_cast<size_t>(k) * block_bytes;
    SlotLease sl(c);
    if (sl.rc) return sl.rc;
    StageSlot &st = *sl.s;
    const size_t scratch = kSliceCap * static_cast<size_t>(std::max(m, 1)) * block_bytes;  // step-slice partials
    // staging: [blocks][rows (256)][workspace (general path)][slice partials]
    const size_t ws_off = (data_bytes + 256 + 255) & ~static_cast<size_t>(255);
    DecodeWS probe{};
    const size_t ws_bytes = general ? carve(probe, nullptr, k, m, block_bytes, 1, true) : 0;
    if (int rc = st.h.ensure(ws_off + ws_bytes + 8)) return rc;
    if (int rc = st.d.ensure(ws_off + ws_bytes + scratch, st.stream)) return rc;
    uint8_t *h = static_cast<uint8_t *>(st.h.p);
    uint8_t *d = static_cast<uint8_t *>(st.d.p);
    for (int i = 0; i < k; ++i) {
        std::memcpy(h + static_cast<size_t>(i) * block_bytes, blocks[i].data, block_bytes);
        h[data_bytes + i] = blocks[i].row;
    }
    if (general) {
        // The decode setup runs here (host_decode_setup) where it applies: its workspace fields
        // go up with the blocks in one copy, and the recovered rows come back densely (e blocks,
        // no device scatter kernel) to be placed here.
        DecodeWS wh{};
        carve(wh, h + ws_off, k, m, block_bytes, 1, true);
        const bool hs = host_decode_setup(wh, k, m, h + data_bytes, e, rec, era);
        const size_t up = hs ? ws_off + static_cast<size_t>(wh.residual - (h + ws_off)) : data_bytes + k;
        SH_CHECK(hipMemcpyAsync(d, h, up, hipMemcpyHostToDevice, st.stream));
        const int rc = decode_batch(k, m, block_bytes, 1, d, d + data_bytes, st.stream, nullptr,
                                    d + ws_off + ws_bytes, h, e, d + ws_off, hs);
        if (rc != 0) {
            // the staging slot is released on return: nothing queued may still read it
            (void)hipStreamSynchronize(st.stream);
            return rc;
        }
        SH_CHECK(hipStreamSynchronize(st.stream));
        for (int l = 0; l < e; ++l) {
            std::memcpy(blocks[rec[l]].data, h + static_cast<size_t>(l) * block_bytes, block_bytes);
            blocks[rec[l]].row = static_cast<uint8_t>(era[l]);
        }
        return 0;
    }
    SH_CHECK(hipMemcpyAsync(d, h, data_bytes + k, hipMemcpyHostToDevice, st.stream));
    // m == 1 (cauchy_decode_m1) and the parameter-error paths: the batch decode in place
    int *e_host = reinterpret_cast<int *>(h + ((data_bytes + k + 3) & ~static_cast<size_t>(3)));
    *e_host = 0;
    const int rc = decode_batch(k, m, block_bytes, 1, d, d + data_bytes, st.stream, e_host, d + data_bytes + 256);
    if (rc != 0) {
        (void)hipStreamSynchronize(st.stream);
        return rc;
    }
    SH_CHECK(hipMemcpyAsync(h, d, data_bytes + k, hipMemcpyDeviceToHost, st.stream));
    SH_CHECK(hipStreamSynchronize(st.stream));
    if (*e_host < 0) return -1;
    for (int i = 0; i < k; ++i) {
        if (blocks[i].row >= k) {
            std::memcpy(blocks[i].data, h + static_cast<size_t>(i) * block_bytes, block_bytes);
            blocks[i].row = h[data_bytes + i];
        }
    }
    return 0;
}
