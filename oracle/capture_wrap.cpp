// Test infrastructure only: BASELINE config C1's capture. Linked (-Wl,--wrap=...) between the
// reference's unchanged Shorthair.cpp and the REFERENCE codec (_ref/libref_cauchy.so, compiled in
// place from /root/reference), it records the codec calls the protocol layer really makes --
// misaligned packet pointers, Tester-shaped variable-length payloads framed by
// Encoder::EncodeQueued / RecoverGroup (Shorthair.cpp:529-566, :704-747) -- and passes every call
// through unchanged. tools/capture_c1.py turns the dumps into tests/golden/c1_*.npz.
//
// Dump format (CAPTURE_DIR/<n>_enc.bin, <n>_dec.bin), little-endian int32 header then bytes:
//   encode: [k, m, B, rc, align[k]] data[k][B] recovery[m][B]
//   decode: [k, m, B, rc, align[k]] rows_before[k] data_before[k][B] rows_after[k] data_after[k][B]
// align[i] = data pointer address mod 16. CAPTURE_MAX bounds the number of dumps per kind.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "cauchy_256.h"

extern "C" {
int __real_cauchy_256_encode(int k, int m, const unsigned char *data_ptrs[], void *recovery_blocks, int block_bytes);
int __real_cauchy_256_decode(int k, int m, Block *blocks, int block_bytes);
}

namespace {

int counter(const char *kind) {
    static int enc = 0, dec = 0;
    return kind[0] == 'e' ? enc++ : dec++;
}

FILE *open_dump(const char *kind, int n) {
    const char *dir = std::getenv("CAPTURE_DIR");
    const int max = std::getenv("CAPTURE_MAX") ? std::atoi(std::getenv("CAPTURE_MAX")) : 4;
    if (!dir || n >= max) return nullptr;
    const std::string path = std::string(dir) + "/" + std::to_string(n) + "_" + kind + ".bin";
    return std::fopen(path.c_str(), "wb");
}

void put_header(FILE *f, int k, int m, int B, int rc, const std::vector<int32_t> &align) {
    const int32_t h[4] = {k, m, B, rc};
    std::fwrite(h, sizeof h, 1, f);
    std::fwrite(align.data(), sizeof(int32_t), align.size(), f);
}

// Calls worth keeping: the protocol's real groups (k > 1, m > 1; decode with an erasure), which
// exercise the bitmatrix paths rather than the k <= 1 / m == 1 shortcuts.
bool interesting_encode(int k, int m) { return k > 1 && m > 1; }

}  // namespace

extern "C" int __wrap_cauchy_256_encode(int k, int m, const unsigned char *data_ptrs[], void *recovery_blocks,
                                        int block_bytes) {
    const int rc = __real_cauchy_256_encode(k, m, data_ptrs, recovery_blocks, block_bytes);
    if (!interesting_encode(k, m)) return rc;
    FILE *f = open_dump("enc", counter("enc"));
    if (!f) return rc;
    std::vector<int32_t> align(static_cast<size_t>(k));
    for (int i = 0; i < k; ++i) align[static_cast<size_t>(i)] = static_cast<int32_t>(reinterpret_cast<uintptr_t>(data_ptrs[i]) % 16);
    put_header(f, k, m, block_bytes, rc, align);
    for (int i = 0; i < k; ++i) std::fwrite(data_ptrs[i], 1, static_cast<size_t>(block_bytes), f);
    std::fwrite(recovery_blocks, 1, static_cast<size_t>(m) * block_bytes, f);
    std::fclose(f);
    return rc;
}

extern "C" int __wrap_cauchy_256_decode(int k, int m, Block *blocks, int block_bytes) {
    // snapshot before: decode works in place
    std::vector<uint8_t> rows0(static_cast<size_t>(k)), data0(static_cast<size_t>(k) * block_bytes);
    bool lost = false;
    for (int i = 0; i < k; ++i) {
        rows0[static_cast<size_t>(i)] = blocks[i].row;
        lost = lost || blocks[i].row >= k;
        std::memcpy(&data0[static_cast<size_t>(i) * block_bytes], blocks[i].data, static_cast<size_t>(block_bytes));
    }
    const int rc = __real_cauchy_256_decode(k, m, blocks, block_bytes);
    if (!(k > 1 && m > 1 && lost)) return rc;
    FILE *f = open_dump("dec", counter("dec"));
    if (!f) return rc;
    std::vector<int32_t> align(static_cast<size_t>(k));
    for (int i = 0; i < k; ++i) align[static_cast<size_t>(i)] = static_cast<int32_t>(reinterpret_cast<uintptr_t>(blocks[i].data) % 16);
    put_header(f, k, m, block_bytes, rc, align);
    std::fwrite(rows0.data(), 1, rows0.size(), f);
    std::fwrite(data0.data(), 1, data0.size(), f);
    for (int i = 0; i < k; ++i) std::fwrite(&blocks[i].row, 1, 1, f);
    for (int i = 0; i < k; ++i) std::fwrite(blocks[i].data, 1, static_cast<size_t>(block_bytes), f);
    std::fclose(f);
    return rc;
}
