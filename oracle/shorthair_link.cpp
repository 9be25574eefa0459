// Test infrastructure only: the reference's unchanged protocol layer (catid/shorthair
// Shorthair.cpp, PacketAllocator.cpp, SiameseTools.cpp, compiled in place from /root/reference by
// oracle/Makefile) linked against OUR libcauchy256.so -- the drop-in claim of include/cauchy_256.h
// exercised by the reference's own caller (Shorthair.cpp:566 encode, :747 decode, :912 init).
//
// A two-endpoint loopback in the shape of the reference's tests/Tester.cpp ZeroLossTest
// (Tester.cpp:224-240): every 5 ms the server sends 10 packets of 8..1350 bytes, [u32 id][PCG32
// stream seeded by id], through ShorthairCodec::Send; its SendData drops 10 % of the wire packets
// (deterministic LCG) and hands the rest to the client's Recv; the client's OnPacket checks every
// delivered payload byte for byte; the client's own traffic (loss statistics) goes back without
// loss. Unlike Tester, the run ends after --seconds and prints one JSON line with the counts.
// Shorthair ticks on the wall clock (Shorthair.cpp:1063), so the counts vary slightly run to run.
#include "Shorthair.hpp"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

using namespace cat::shorthair;

namespace {

struct Pcg32 {  // PCG-XSH-RR, as the reference's siamese::PCGRandom (SiameseTools.h:80-102)
    uint64_t state = 0, inc = 0;
    void seed(uint64_t y, uint64_t x = 0) {
        state = 0;
        inc = (y << 1u) | 1u;
        next();
        state += x;
        next();
    }
    uint32_t next() {
        const uint64_t old = state;
        state = old * 6364136223846793005ULL + inc;
        const uint32_t xs = static_cast<uint32_t>(((old >> 18) ^ old) >> 27);
        const uint32_t rot = static_cast<uint32_t>(old >> 59);
        return (xs >> rot) | (xs << ((0u - rot) & 31u));
    }
};

void payload(uint32_t id, uint8_t *out, int len) {
    std::memcpy(out, &id, 4);
    Pcg32 p;
    p.seed(id, 0x5A17);
    for (int i = 4; i < len; ++i) out[i] = static_cast<uint8_t>(p.next());
}

struct Endpoint : IShorthair {
    ShorthairCodec codec;
    Endpoint *peer = nullptr;
    bool lossy = false;
    uint64_t lcg = 0x9E3779B97F4A7C15ULL;
    long wire_sent = 0, wire_dropped = 0;
    long delivered = 0, corrupt = 0, duplicate = 0;
    std::vector<uint8_t> seen;
    std::vector<uint8_t> scratch = std::vector<uint8_t>(4096);

    void OnPacket(uint8_t *packet, int bytes) override {
        if (bytes < 4) {
            ++corrupt;
            return;
        }
        uint32_t id;
        std::memcpy(&id, packet, 4);
        std::vector<uint8_t> want(static_cast<size_t>(bytes));
        payload(id, want.data(), bytes);
        if (id >= seen.size() || std::memcmp(want.data(), packet, static_cast<size_t>(bytes)) != 0) {
            ++corrupt;
            return;
        }
        if (seen[id]) ++duplicate;
        seen[id] = 1;
        ++delivered;
    }
    void OnOOB(uint8_t *, int) override {}
    void SendData(uint8_t *buffer, int bytes) override {
        ++wire_sent;
        if (lossy) {
            lcg = lcg * 6364136223846793005ULL + 1442695040888963407ULL;
            if ((lcg >> 33) % 10 == 0) {  // 10 % loss, as Tester's ENABLE_PACKETLOSS 0.1f
                ++wire_dropped;
                return;
            }
        }
        std::memcpy(scratch.data(), buffer, static_cast<size_t>(bytes));  // Recv modifies its buffer
        peer->codec.Recv(scratch.data(), bytes);
    }
};

}  // namespace

int main(int argc, char **argv) {
    double seconds = 3.0;
    for (int i = 1; i + 1 < argc; ++i)
        if (std::strcmp(argv[i], "--seconds") == 0) seconds = std::atof(argv[i + 1]);

    Endpoint server, client;
    server.peer = &client;
    client.peer = &server;
    server.lossy = true;
    Settings ss, cs;  // the Tester's settings (Tester.cpp: Accept / Connect)
    ss.min_fec_overhead = cs.min_fec_overhead = 0.2f;
    ss.max_delay = cs.max_delay = 100;
    ss.max_data_size = 1350;
    cs.max_data_size = 1400;
    ss.interface_ptr = &server;
    cs.interface_ptr = &client;
    if (!server.codec.Initialize(ss) || !client.codec.Initialize(cs)) {
        std::printf("{\"error\": \"Initialize failed\"}\n");
        return 2;
    }
    const long max_packets = static_cast<long>(seconds / 0.005 * 10) + 100;
    client.seen.assign(static_cast<size_t>(max_packets), 0);
    Pcg32 lens;
    lens.seed(1234);
    uint32_t next_id = 0;
    std::vector<uint8_t> buf(1400);
    const auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < seconds) {
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
        client.codec.Tick();
        server.codec.Tick();
        for (int i = 0; i < 10 && next_id < static_cast<uint32_t>(max_packets); ++i) {
            const int len = 8 + static_cast<int>(lens.next() % (1350 - 8 + 1));
            payload(next_id++, buf.data(), len);
            server.codec.Send(buf.data(), static_cast<size_t>(len));
        }
    }
    // drain: let the last code group's recovery packets go out and be decoded
    for (int i = 0; i < 60; ++i) {
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
        client.codec.Tick();
        server.codec.Tick();
    }
    const long dropped_ids = static_cast<long>(next_id) - client.delivered;
    std::printf("{\"sent\": %u, \"delivered\": %ld, \"undelivered\": %ld, \"corrupt\": %ld, \"duplicate\": %ld, "
                "\"wire_packets\": %ld, \"wire_dropped\": %ld, \"delivery_ratio\": %.5f}\n",
                next_id, client.delivered, dropped_ids, client.corrupt, client.duplicate, server.wire_sent,
                server.wire_dropped, next_id ? static_cast<double>(client.delivered) / next_id : 0.0);
    server.codec.Finalize();
    client.codec.Finalize();
    return client.corrupt == 0 ? 0 : 1;
}
