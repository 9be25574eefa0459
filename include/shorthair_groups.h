/*
 * shorthair_groups.h -- batched packet-group framing around the codec.
 *
 * The reference protocol layer turns a queue of variable-length UDP payloads into one code group
 * and back, one group per call on one CPU thread:
 *
 *   sender    Encoder::EncodeQueued (Shorthair.cpp:480-576): block_bytes = roundup8(2 + largest
 *             payload); each original becomes a block "[len u16 LE][payload][zeros]"; k+m is
 *             truncated to 256; k == 1 sends the payload itself. Encoder::GenerateRecoveryBlock
 *             (:580-609) frames recovery block i as "[k+i][k-1][m-1][block]" (k == 1: "[1][0]
 *             [payload]", repeated for every request).
 *   receiver  ShorthairCodec::OnData (:764-902) keeps each original as "[len u16 LE][payload]"
 *             and each recovery packet's block; RecoverGroup (:704-761) zero-pads the originals
 *             to block_bytes, lists them (arrival order) followed by recovery packets (arrival
 *             order, up to k), decodes in place, and hands every recovered block whose length
 *             prefix is <= block_bytes - 2 to IShorthair::OnPacket(data + 2, len).
 *
 * These entry points do the same for many groups per call: framing on host threads into pinned
 * staging, groups bucketed by (k, m, block_bytes), one batched GPU launch per bucket chunk
 * (cauchy_256_encode_batch / cauchy_256_decode_batch_out), chunks double-buffered so host
 * framing overlaps the PCIe copies and the kernels. The bytes on the wire are exactly the
 * reference's. Host buffers only; any alignment.
 *
 * Return codes: >= 0 ok (see each call), -1 invalid arguments, -2 GPU/runtime error.
 */
#ifndef SH_AMD_SHORTHAIR_GROUPS_H
#define SH_AMD_SHORTHAIR_GROUPS_H

#ifdef __cplusplus
extern "C" {
#endif

/* One sender-side code group. */
typedef struct ShorthairTxGroup {
    int k;                                /* originals in the group, 1..255 */
    int m;                                /* recovery packets wanted, >= 1 (truncated to 256 - k) */
    const unsigned char *const *packets;  /* k payload pointers */
    const unsigned short *lens;           /* k payload lengths (0..65535) */
    unsigned char *out;                   /* recovery packets: m_out records of out_stride bytes */
    int out_capacity;                     /* bytes available at out */
    int m_out;                            /* [out] recovery packets written */
    int out_stride;                       /* [out] bytes per recovery packet */
} ShorthairTxGroup;

/* Bytes of one recovery packet for a group: 3 + roundup8(2 + largest) (k >= 2) or 2 + lens[0]
 * (k == 1); -1 on invalid arguments. */
int shorthair_recovery_packet_bytes(int k, const unsigned short *lens);

/* Encode every group (EncodeQueued + GenerateRecoveryBlock x m). Returns 0, -1 (nothing written
 * for any group: a group with k outside 1..255, m < 1, a null pointer or out_capacity too small)
 * or -2. */
int shorthair_encode_groups(ShorthairTxGroup *groups, int count);

/* One receiver-side code group, as OnData would hold it when CanRecover() turns true. */
typedef struct ShorthairRxGroup {
    int n_orig;                               /* originals received (arrival order) */
    const unsigned char *orig_ids;            /* their ids (0..k-1, distinct) */
    const unsigned char *const *orig_data;    /* their payloads */
    const unsigned short *orig_lens;          /* their payload lengths */
    int n_rec;                                /* recovery packets received (arrival order) */
    const unsigned char *const *rec_packets;  /* as produced by the sender: [id][k-1][m-1][block] */
    const int *rec_lens;                      /* their byte counts (3 + block_bytes) */
} ShorthairRxGroup;

/* Called once per recovered original, in RecoverGroup's delivery order (the i-th recovery
 * block in list order carries the i-th smallest missing id); `id` is that original's id. */
typedef void (*shorthair_on_packet_fn)(void *ctx, int group, int id, const unsigned char *data,
                                       int len);

/* Recover every group that can be (n_orig + n_rec >= k, k from the recovery headers, m and
 * block_bytes from the last recovery packet, as OnData keeps them). Returns the number of
 * groups decoded, -1 on malformed input (nothing delivered) or -2. Groups with every original
 * present or too few packets are skipped (no callback). on_packet may be NULL: decode only
 * (measurement), nothing delivered. */
int shorthair_recover_groups(const ShorthairRxGroup *groups, int count, shorthair_on_packet_fn on_packet,
                             void *ctx);

#ifdef __cplusplus
}
#endif

#endif /* SH_AMD_SHORTHAIR_GROUPS_H */
