// Batched packet-group framing around the codec (include/shorthair_groups.h).
//
// Sender: the reference's Encoder::EncodeQueued (Shorthair.cpp:480-576) and GenerateRecoveryBlock
// (:580-609) for many groups per call. Receiver: RecoverGroup (:704-761) over the packets OnData
// (:764-902) keeps, for many groups per call.
//
// Layer above the public batch ABI (cauchy_256_batch.h): groups are bucketed by (k, m, B), a
// bucket is cut into chunks of ~chunk_bytes() of blocks, and chunks alternate between two pinned
// staging slots. For chunk i the host threads frame the blocks into slot i%2 while the GPU runs
// chunk i-1 (H2D, kernel, D2H on one stream); once slot i%2's previous chunk has completed its
// outputs are unframed on the host threads. So host framing, PCIe and kernels overlap, and the
// only host work per byte is the framing copy the reference also does (its memset/memcpy).
#include <hip/hip_runtime.h>
#include <sched.h>
#include <emmintrin.h>

#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/cauchy_256_batch.h"
#include "measure.hpp"
#include "../../include/shorthair_groups.h"

namespace {

// device bytes per chunk (inputs + outputs); SH_PKT_CHUNK_MB: measurement switch
size_t chunk_bytes() {
    static const size_t b = [] {
        const char *e = SH_MEASURE_ENV("SH_PKT_CHUNK_MB");
        const int mb = e ? std::atoi(e) : 48;
        return static_cast<size_t>(std::max(1, mb)) << 20;
    }();
    return b;
}

#define SG_CHECK(expr)                                                                        \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess) {                                                               \
            std::fprintf(stderr, "libcauchy256: %s failed: %s (%s:%d)\n", #expr,             \
                         hipGetErrorString(_e), __FILE__, __LINE__);                          \
            return -2;                                                                        \
        }                                                                                     \
    } while (0)

inline int roundup8(int x) { return (x + 7) & ~7; }
inline void put_u16(uint8_t *p, unsigned v) {  // WriteU16_LE (ShorthairDetails.hpp)
    p[0] = static_cast<uint8_t>(v);
    p[1] = static_cast<uint8_t>(v >> 8);
}
inline unsigned get_u16(const uint8_t *p) { return p[0] | (static_cast<unsigned>(p[1]) << 8); }

// Framing copy into the pinned staging buffer: 16-byte non-temporal stores for the aligned body
// (the staging bytes are read next by the H2D DMA, not by this core, so a cached store's
// read-for-ownership of every line is wasted memory traffic), plain copies for the ragged ends.
// Callers fence (framing_fence) before the buffer is handed to the DMA.
inline void framing_copy(uint8_t *dst, const uint8_t *src, size_t n) {
    if (n < 64) {
        std::memcpy(dst, src, n);
        return;
    }
    const size_t head = (16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15;
    std::memcpy(dst, src, head);
    dst += head;
    src += head;
    n -= head;
    const size_t body = n & ~static_cast<size_t>(15);
    for (size_t i = 0; i < body; i += 16)
        _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i),
                         _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + i)));
    std::memcpy(dst + body, src + body, n - body);
}
inline void framing_fence() { _mm_sfence(); }

int host_threads() {
    static const int n = [] {
        // the cores this process may run on (its affinity mask: a job's share of a large host),
        // at most 16; SH_HOST_THREADS overrides it in measurement builds only
        cpu_set_t set;
        CPU_ZERO(&set);
        int v = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set)
                                                            : static_cast<int>(std::thread::hardware_concurrency());
        if (const char *e = SH_MEASURE_ENV("SH_HOST_THREADS")) v = std::atoi(e);
        return std::max(1, std::min(v > 0 ? v : 1, 16));
    }();
    return n;
}

// Persistent host workers for the framing copies: host_threads() - 1 threads started on first use
// and parked on a condition variable between calls (spawning and joining 15 threads per framing
// pass cost ~0.3 ms each time, two passes per chunk). Never destroyed: parked threads are fine at
// process exit.
class Workers {
  public:
    explicit Workers(int n) : nthreads_(n) {
        for (int w = 1; w < n; ++w) th_.emplace_back([this, w] { loop(w); });
        for (auto &t : th_) t.detach();
    }
    int size() const { return nthreads_; }
    // fn(i) for i in [0, n) split into t <= size() contiguous ranges; the caller runs range 0.
    // One pass owns the pool at a time; a pass from another thread that finds it busy runs its
    // whole range on its own thread instead of queueing behind the owner, so
    // concurrent shorthair_*_groups calls still overlap.
    void run(int n, int t, const std::function<void(int)> &fn) {
        std::unique_lock<std::mutex> one(run_mu_, std::try_to_lock);
        if (!one.owns_lock() || t <= 1) {
            for (int i = 0; i < n; ++i) fn(i);
            return;
        }
        {
            std::lock_guard<std::mutex> g(mu_);
            fn_ = &fn;
            n_ = n;
            t_ = t;
            pending_ = nthreads_ - 1;
            ++gen_;
        }
        cv_.notify_all();
        range(0, n, t, fn);
        std::unique_lock<std::mutex> g(mu_);
        done_.wait(g, [this] { return pending_ == 0; });
    }

  private:
    static void range(int w, int n, int t, const std::function<void(int)> &fn) {
        if (w >= t) return;
        const int a = static_cast<int>(static_cast<long long>(n) * w / t);
        const int b = static_cast<int>(static_cast<long long>(n) * (w + 1) / t);
        for (int i = a; i < b; ++i) fn(i);
    }
    void loop(int w) {
        unsigned long long seen = 0;
        for (;;) {
            const std::function<void(int)> *fn;
            int n, t;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return gen_ != seen; });
                seen = gen_;
                fn = fn_;
                n = n_;
                t = t_;
            }
            range(w, n, t, *fn);
            std::lock_guard<std::mutex> g(mu_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    const int nthreads_;
    std::vector<std::thread> th_;
    std::mutex run_mu_, mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)> *fn_ = nullptr;
    int n_ = 0, t_ = 0, pending_ = 0;
    unsigned long long gen_ = 0;
};

Workers &workers() {
    static Workers *w = new Workers(host_threads());
    return *w;
}

// fn(i) for i in [0, n) on up to host_threads() threads (contiguous ranges).
void parallel_for(int n, const std::function<void(int)> &fn) {
    const int t = std::min(host_threads(), std::max(1, n / 4));
    if (t <= 1) {
        for (int i = 0; i < n; ++i) fn(i);
        return;
    }
    workers().run(n, t, fn);
}

// Two pinned + device staging slots on one stream; each slot remembers how to finish the chunk
// it carries (unframe outputs once its event has fired).
struct Slot {
    void *h = nullptr, *d = nullptr;
    size_t nh = 0, nd = 0;
    hipEvent_t ev = nullptr;
    std::function<void()> finish;  // empty: nothing pending
};

struct Staging {
    std::mutex mu;  // one packet-group call at a time (shared slots)
    bool ready = false;
    hipStream_t stream = nullptr;
    Slot slot[2];
};

Staging &staging() {
    static Staging s;
    return s;
}

int ensure_slot(Slot &s, size_t bytes) {
    if (!s.ev) SG_CHECK(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming));
    if (bytes > s.nh) {
        if (s.h) (void)hipHostFree(s.h);
        s.h = nullptr;
        s.nh = 0;
        SG_CHECK(hipHostMalloc(&s.h, bytes, hipHostMallocDefault));
        s.nh = bytes;
    }
    if (bytes > s.nd) {
        if (s.d) (void)hipFree(s.d);
        s.d = nullptr;
        s.nd = 0;
        SG_CHECK(hipMalloc(&s.d, bytes));
        s.nd = bytes;
    }
    return 0;
}

int ensure_staging(Staging &st) {
    if (st.ready) return 0;
    if (cauchy_256_batch_init(-1) != 0) return -2;
    SG_CHECK(hipStreamCreateWithFlags(&st.stream, hipStreamNonBlocking));
    st.ready = true;
    return 0;
}

// Wait for the slot's previous chunk and unframe its outputs.
int drain(Slot &s) {
    if (!s.finish) return 0;
    SG_CHECK(hipEventSynchronize(s.ev));
    auto f = std::move(s.finish);
    s.finish = nullptr;
    f();
    return 0;
}

// Run `chunks` chunks through the two slots: prepare(i, slot) frames chunk i into the slot's
// pinned buffer, submit(i, slot) enqueues its copies and kernels and returns the finisher.
template <class Prep, class Submit>
int pipeline(Staging &st, int chunks, size_t slot_bytes, Prep prepare, Submit submit) {
    int err = 0;
    for (int i = 0; i < chunks && !err; ++i) {
        Slot &s = st.slot[i & 1];
        if ((err = drain(s))) break;
        if ((err = ensure_slot(s, slot_bytes))) break;
        prepare(i, s);
        std::function<void()> fin;
        if ((err = submit(i, s, fin))) break;
        if (hipEventRecord(s.ev, st.stream) != hipSuccess) {
            err = -2;
            break;
        }
        s.finish = std::move(fin);
    }
    for (Slot &s : st.slot) {
        if (err) {
            (void)hipStreamSynchronize(st.stream);
            s.finish = nullptr;
        } else if (int e = drain(s)) {
            err = e;
        }
    }
    return err;
}

// ---------------------------------------------------------------------------------------------
// Sender
// ---------------------------------------------------------------------------------------------
struct TxInfo {
    int k, m, B;  // m after truncation to 256 - k; B = block bytes (k >= 2)
};

bool tx_info(const ShorthairTxGroup &g, TxInfo &t) {
    if (g.k < 1 || g.k > 255 || g.m < 1 || !g.lens || !g.packets || !g.out) return false;
    int largest = 0;
    for (int x = 0; x < g.k; ++x) {
        if (!g.packets[x]) return false;
        largest = std::max(largest, static_cast<int>(g.lens[x]));
    }
    t.k = g.k;
    t.m = std::min(g.m, 256 - g.k);                   // Shorthair.cpp:501-504
    t.B = g.k == 1 ? largest : roundup8(2 + largest);  // :531-537 (k == 1: the payload itself)
    return true;
}

}  // namespace

extern "C" int shorthair_recovery_packet_bytes(int k, const unsigned short *lens) {
    if (k < 1 || k > 255 || !lens) return -1;
    int largest = 0;
    for (int x = 0; x < k; ++x) largest = std::max(largest, static_cast<int>(lens[x]));
    return k == 1 ? 2 + largest : 3 + roundup8(2 + largest);
}

extern "C" int shorthair_encode_groups(ShorthairTxGroup *groups, int count) {
    if (count < 0 || (count > 0 && !groups)) return -1;
    std::vector<TxInfo> info(count);
    for (int i = 0; i < count; ++i) {
        if (!tx_info(groups[i], info[i])) return -1;
        const TxInfo &t = info[i];
        const long long stride = t.k == 1 ? 2 + t.B : 3 + t.B;
        if (static_cast<long long>(groups[i].out_capacity) < stride * t.m) return -1;
    }
    // k == 1: "[1][0][payload]" for every request (GenerateRecoveryBlock :587-596), no codec
    std::map<std::tuple<int, int, int>, std::vector<int>> buckets;
    for (int i = 0; i < count; ++i) {
        ShorthairTxGroup &g = groups[i];
        const TxInfo &t = info[i];
        g.m_out = t.m;
        if (t.k == 1) {
            g.out_stride = 2 + t.B;
            for (int y = 0; y < t.m; ++y) {
                uint8_t *p = g.out + static_cast<size_t>(y) * g.out_stride;
                p[0] = 1;
                p[1] = 0;
                std::memcpy(p + 2, g.packets[0], g.lens[0]);
            }
        } else {
            g.out_stride = 3 + t.B;
            buckets[std::make_tuple(t.k, t.m, t.B)].push_back(i);
        }
    }
    if (buckets.empty()) return 0;
    Staging &st = staging();
    std::lock_guard<std::mutex> lock(st.mu);
    if (int rc = ensure_staging(st)) return rc;
    for (auto &kv : buckets) {
        const int k = std::get<0>(kv.first), m = std::get<1>(kv.first), B = std::get<2>(kv.first);
        const std::vector<int> &ids = kv.second;
        const size_t in_g = static_cast<size_t>(k) * B, out_g = static_cast<size_t>(m) * B;
        const int per = static_cast<int>(std::max<size_t>(1, chunk_bytes() / (in_g + out_g)));
        const int n = static_cast<int>(ids.size());
        const int chunks = (n + per - 1) / per;
        const size_t slot_bytes = static_cast<size_t>(std::min(per, n)) * (in_g + out_g);
        auto prepare = [&](int c, Slot &s) {
            const int g0 = c * per, gn = std::min(per, n - g0);
            uint8_t *h = static_cast<uint8_t *>(s.h);
            // EncodeQueued :540-557: "[len u16 LE][payload][zeros up to B]" per original
            parallel_for(gn, [&](int j) {
                const ShorthairTxGroup &g = groups[ids[g0 + j]];
                uint8_t *blk = h + static_cast<size_t>(j) * in_g;
                for (int x = 0; x < k; ++x, blk += B) {
                    const int len = g.lens[x];
                    put_u16(blk, len);
                    framing_copy(blk + 2, static_cast<const uint8_t *>(g.packets[x]), len);
                    std::memset(blk + 2 + len, 0, B - 2 - len);
                }
                framing_fence();
            });
        };
        auto submit = [&](int c, Slot &s, std::function<void()> &fin) -> int {
            const int g0 = c * per, gn = std::min(per, n - g0);
            uint8_t *h = static_cast<uint8_t *>(s.h), *d = static_cast<uint8_t *>(s.d);
            const size_t in_bytes = gn * in_g, out_bytes = gn * out_g;
            SG_CHECK(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, st.stream));
            const int rc = cauchy_256_encode_batch(k, m, B, gn, d, d + in_bytes, st.stream);
            if (rc != 0) return rc;
            SG_CHECK(hipMemcpyAsync(h + in_bytes, d + in_bytes, out_bytes, hipMemcpyDeviceToHost, st.stream));
            fin = [&, g0, gn, h, in_bytes]() {
                // GenerateRecoveryBlock :598-608: "[k+i][k-1][m-1][block i]"
                parallel_for(gn, [&](int j) {
                    ShorthairTxGroup &g = groups[ids[g0 + j]];
                    const uint8_t *rec = h + in_bytes + static_cast<size_t>(j) * out_g;
                    for (int y = 0; y < m; ++y) {
                        uint8_t *p = g.out + static_cast<size_t>(y) * g.out_stride;
                        p[0] = static_cast<uint8_t>(k + y);
                        p[1] = static_cast<uint8_t>(k - 1);
                        p[2] = static_cast<uint8_t>(m - 1);
                        std::memcpy(p + 3, rec + static_cast<size_t>(y) * B, B);
                    }
                });
            };
            return 0;
        };
        if (int rc = pipeline(st, chunks, slot_bytes, prepare, submit)) return rc;
    }
    return 0;
}

// ---------------------------------------------------------------------------------------------
// Receiver
// ---------------------------------------------------------------------------------------------
namespace {

struct RxInfo {
    int k = 0, m = 0, B = 0, use = 0;  // use: recovery packets listed (k - n_orig); 0 = skip
};

// -1 malformed, 0 skip, 1 decode (k >= 2), 2 k == 1 special form
int rx_info(const ShorthairRxGroup &g, RxInfo &r) {
    if (g.n_orig < 0 || g.n_rec < 0 || (g.n_orig && (!g.orig_ids || !g.orig_data || !g.orig_lens)) ||
        (g.n_rec && (!g.rec_packets || !g.rec_lens)))
        return -1;
    if (g.n_rec == 0) return 0;  // nothing to decode from
    for (int j = 0; j < g.n_rec; ++j)
        if (!g.rec_packets[j] || g.rec_lens[j] < 2) return -1;
    const int k = g.rec_packets[0][1] + 1;  // "[id][k-1]..." (OnData :785-786)
    for (int j = 1; j < g.n_rec; ++j)
        if (g.rec_packets[j][1] + 1 != k) return -1;
    r.k = k;
    if (k == 1) return g.n_orig == 0 ? 2 : 0;  // :858-866 ("a redundant packet won")
    if (g.n_orig >= k || g.n_orig + g.n_rec < k) return 0;  // CanRecover() (ShorthairDetails.hpp:328)
    const uint8_t *last = g.rec_packets[g.n_rec - 1];
    r.m = last[2] + 1;                       // :878 recovery_count = data[0] + 1
    r.B = g.rec_lens[g.n_rec - 1] - 3;       // :877 largest_len = data_len - 1
    if (r.B < 8 || r.B % 8 != 0 || k + r.m > 256) return -1;
    bool seen[256] = {false};
    for (int i = 0; i < g.n_orig; ++i) {
        const int id = g.orig_ids[i];
        if (id >= k || seen[id] || g.orig_lens[i] > r.B - 2 || !g.orig_data[i]) return -1;
        seen[id] = true;
    }
    r.use = k - g.n_orig;  // RecoverGroup :727-735: recovery packets until k blocks
    for (int j = 0; j < r.use; ++j) {
        const int id = g.rec_packets[j][0];
        if (id < k || id >= k + r.m || seen[id] || g.rec_lens[j] != r.B + 3) return -1;
        seen[id] = true;
    }
    return 1;
}

}  // namespace

extern "C" int shorthair_recover_groups(const ShorthairRxGroup *groups, int count,
                                        shorthair_on_packet_fn on_packet, void *cb_ctx) {
    if (count < 0 || (count > 0 && !groups)) return -1;
    std::vector<RxInfo> info(count);
    std::vector<int> kind(count);
    for (int i = 0; i < count; ++i)
        if ((kind[i] = rx_info(groups[i], info[i])) < 0) return -1;
    int decoded = 0;
    std::map<std::tuple<int, int, int>, std::vector<int>> buckets;
    for (int i = 0; i < count; ++i) {
        if (kind[i] == 2) {
            const ShorthairRxGroup &g = groups[i];
            if (on_packet) on_packet(cb_ctx, i, 0, g.rec_packets[0] + 2, g.rec_lens[0] - 2);
            ++decoded;
        } else if (kind[i] == 1) {
            buckets[std::make_tuple(info[i].k, info[i].m, info[i].B)].push_back(i);
        }
    }
    if (buckets.empty()) return decoded;
    Staging &st = staging();
    std::lock_guard<std::mutex> lock(st.mu);
    if (int rc = ensure_staging(st)) return rc;
    for (auto &kv : buckets) {
        const int k = std::get<0>(kv.first), m = std::get<1>(kv.first), B = std::get<2>(kv.first);
        const std::vector<int> &ids = kv.second;
        const int emax = std::min(k, m);
        // per group: blocks k*B, rows k; out emax*B; out rows emax; count 4 (m >= 2 only)
        const size_t in_g = static_cast<size_t>(k) * B;
        const size_t out_g = m >= 2 ? static_cast<size_t>(emax) * B : static_cast<size_t>(B);
        const size_t per_g = in_g + k + out_g + emax + 4;
        const int per = static_cast<int>(std::max<size_t>(1, chunk_bytes() / per_g));
        const int n = static_cast<int>(ids.size());
        const int chunks = (n + per - 1) / per;
        const int cap = std::min(per, n);
        const size_t slot_bytes = static_cast<size_t>(cap) * per_g + 64;
        // slot layout (chunk of gn groups, offsets for cap groups): blocks | rows | out | out rows | count
        const size_t o_rows = cap * in_g, o_out = o_rows + cap * static_cast<size_t>(k);
        const size_t o_orow = o_out + cap * out_g, o_cnt = (o_orow + cap * static_cast<size_t>(emax) + 3) & ~size_t(3);
        auto prepare = [&](int c, Slot &s) {
            const int g0 = c * per, gn = std::min(per, n - g0);
            uint8_t *h = static_cast<uint8_t *>(s.h);
            parallel_for(gn, [&](int j) {
                const ShorthairRxGroup &g = groups[ids[g0 + j]];
                const RxInfo &r = info[ids[g0 + j]];
                uint8_t *blk = h + static_cast<size_t>(j) * in_g;
                uint8_t *rows = h + o_rows + static_cast<size_t>(j) * k;
                int x = 0;
                // RecoverGroup :710-725: originals "[len][payload]" zero-padded to B
                for (int i = 0; i < g.n_orig; ++i, ++x, blk += B) {
                    const int len = g.orig_lens[i];
                    put_u16(blk, len);
                    framing_copy(blk + 2, static_cast<const uint8_t *>(g.orig_data[i]), len);
                    std::memset(blk + 2 + len, 0, B - 2 - len);
                    rows[x] = g.orig_ids[i];
                }
                for (int i = 0; i < r.use; ++i, ++x, blk += B) {  // :727-735
                    framing_copy(blk, g.rec_packets[i] + 3, B);
                    rows[x] = g.rec_packets[i][0];
                }
                framing_fence();
            });
        };
        auto submit = [&](int c, Slot &s, std::function<void()> &fin) -> int {
            const int g0 = c * per, gn = std::min(per, n - g0);
            uint8_t *h = static_cast<uint8_t *>(s.h), *d = static_cast<uint8_t *>(s.d);
            SG_CHECK(hipMemcpyAsync(d, h, gn * in_g, hipMemcpyHostToDevice, st.stream));
            SG_CHECK(hipMemcpyAsync(d + o_rows, h + o_rows, gn * static_cast<size_t>(k), hipMemcpyHostToDevice,
                                    st.stream));
            if (m >= 2) {
                const int rc = cauchy_256_decode_batch_out(k, m, B, gn, d, d + o_rows, d + o_out, d + o_orow,
                                                           reinterpret_cast<int *>(d + o_cnt), st.stream);
                if (rc != 0) return rc;
                SG_CHECK(hipMemcpyAsync(h + o_out, d + o_out, gn * out_g, hipMemcpyDeviceToHost, st.stream));
                SG_CHECK(hipMemcpyAsync(h + o_orow, d + o_orow, gn * static_cast<size_t>(emax),
                                        hipMemcpyDeviceToHost, st.stream));
            } else {
                // m == 1 (cauchy_decode_m1): the one erasure lands in place in block k-1, the
                // single recovery block (n_orig = k-1 originals precede it)
                const int rc = cauchy_256_decode_batch(k, m, B, gn, d, d + o_rows, st.stream);
                if (rc != 0) return rc;
                SG_CHECK(hipMemcpy2DAsync(h + o_out, B, d + static_cast<size_t>(k - 1) * B, in_g, B, gn,
                                          hipMemcpyDeviceToHost, st.stream));
            }
            if (!on_packet) {  // decode only (no delivery): still wait for the chunk before the
                fin = [] {};   // slot is reused and before the call returns
                return 0;
            }
            fin = [&, g0, gn, h]() {
                // RecoverGroup :741-756: deliver recovered blocks whose length prefix fits
                for (int j = 0; j < gn; ++j) {
                    const int gi = ids[g0 + j];
                    const ShorthairRxGroup &g = groups[gi];
                    const int e = k - g.n_orig;
                    const uint8_t *out = h + o_out + static_cast<size_t>(j) * out_g;
                    int missing = -1;
                    if (m < 2) {
                        bool seen[256] = {false};
                        for (int i = 0; i < g.n_orig; ++i) seen[g.orig_ids[i]] = true;
                        for (int x = 0; x < k && missing < 0; ++x)
                            if (!seen[x]) missing = x;
                    }
                    for (int i = 0; i < e; ++i) {
                        const uint8_t *blk = out + static_cast<size_t>(i) * B;
                        const int id = m >= 2 ? h[o_orow + static_cast<size_t>(j) * emax + i] : missing;
                        const int len = static_cast<int>(get_u16(blk));
                        if (len <= B - 2) on_packet(cb_ctx, gi, id, blk + 2, len);
                    }
                }
            };
            return 0;
        };
        if (int rc = pipeline(st, chunks, slot_bytes, prepare, submit)) return rc;
        decoded += n;
    }
    return decoded;
}
