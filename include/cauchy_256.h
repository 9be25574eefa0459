/*
 * cauchy_256.h -- drop-in C ABI of the MI355X-native Cauchy Reed-Solomon codec.
 *
 * Replaces the reference interface catid/shorthair cauchy_256.h:32-109 symbol for symbol, so the
 * unchanged caller (Shorthair.cpp:566 encode, :747 decode, :912 init) links against
 * libcauchy256.so instead of cauchy_256.o. Behind these entry points every call runs on the GPU
 * (gfx950) as a one-group batch; see cauchy_256_batch.h for the device-resident batched API
 * where throughput lives.
 *
 * Semantics are the reference's, bit for bit:
 *   - bitmatrix CRS over GF(256) with polynomial 0x187, k + m <= 256, block_bytes % 8 == 0;
 *   - return 0 on success, -1 on invalid parameters (checked only where the reference checks);
 *   - this library adds -2 for a GPU/runtime failure (message on stderr).
 */
#ifndef SH_AMD_CAUCHY_256_H
#define SH_AMD_CAUCHY_256_H

#ifdef __cplusplus
extern "C" {
#endif

/* API level; must equal the reference's (cauchy_256.h:36). */
#define CAUCHY_256_VERSION 2

/*
 * Version check + one-time initialisation (GPU context, field tables).
 * Replaces cauchy_256.h:47 / cauchy_256.cpp:390-399. Like the reference implementation it
 * returns 0 when expected_version matches and -1 when it does not (the reference header's
 * comment says the opposite; its code returns 0). Returns -2 if no usable GPU is found.
 */
extern int _cauchy_256_init(int expected_version);
#define cauchy_256_init() _cauchy_256_init(CAUCHY_256_VERSION)

/* Received-block descriptor, same layout as the reference (cauchy_256.h:52-55):
 * data pointer at offset 0, row at offset 8 (sizeof == 16 on LP64). */
typedef struct _Block {
    unsigned char *data;
    unsigned char row;
} Block;

/*
 * Encode k data blocks (pointers, any alignment) into m recovery blocks written back to back
 * into recovery_blocks (m * block_bytes bytes). Replaces cauchy_256.h:78 /
 * cauchy_256.cpp:1479-1578: k <= 1 copies data[0] to every output; otherwise recovery row 0 is
 * the XOR of all inputs; m == 1 stops there; k + m > 256 or block_bytes % 8 != 0 then returns -1
 * with row 0 already written.
 */
extern int cauchy_256_encode(int k, int m, const unsigned char *data_ptrs[], void *recovery_blocks,
                             int block_bytes);

/*
 * Recover erased originals in place. blocks[0..k-1] hold the k received blocks: originals with
 * row = their index (< k), recovery block i with row = k + i. Replaces cauchy_256.h:103 /
 * cauchy_256.cpp:1233-1392: on return the i-th recovery block in array order holds the i-th
 * smallest missing original and its row is set to that index (m == 1: the recovery block gets
 * the data but keeps its row; k <= 1: blocks[0].row = 0). Returns -1 for k + m > 256 or
 * block_bytes % 8 != 0 when there is something to recover.
 */
extern int cauchy_256_decode(int k, int m, Block *blocks, int block_bytes);

#ifdef __cplusplus
}
#endif

#endif /* SH_AMD_CAUCHY_256_H */
