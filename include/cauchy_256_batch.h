/*
 * cauchy_256_batch.h -- batched, device-resident C ABI (new; no counterpart in the reference).
 *
 * The reference codes one group per call on one CPU thread (cauchy_256.cpp:1479, :1233). Here a
 * call codes `groups` independent code groups that already sit in GPU memory (HBM), with the same
 * per-group semantics and bytes as cauchy_256_encode / cauchy_256_decode. All calls are
 * asynchronous on `stream` (a hipStream_t passed through verbatim: NULL = the null stream) and
 * enqueue no host
 * synchronisation, except where noted for invalid parameters.
 *
 * Layouts (byte offsets inside one device allocation, no alignment required):
 *   data      [groups][k][block_bytes]      encode input
 *   recovery  [groups][m][block_bytes]      encode output
 *   blocks    [groups][k][block_bytes]      decode blocks (received, in array order)
 *   rows      [groups][k]                   decode rows (the Block.row fields)
 *
 * Return codes: 0 ok, -1 invalid parameters (as the reference), -2 GPU/runtime error.
 */
#ifndef SH_AMD_CAUCHY_256_BATCH_H
#define SH_AMD_CAUCHY_256_BATCH_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Select the device for this process (default 0) and initialise; 0 ok, -2 no GPU. */
int cauchy_256_batch_init(int device);

/* Encode every group: recovery[g] = cauchy_256_encode(k, m, data[g]). */
int cauchy_256_encode_batch(int k, int m, int block_bytes, int groups, const void *d_data,
                            void *d_recovery, void *stream);

/* Decode every group in place, exactly like cauchy_256_decode on (blocks[g], rows[g]). */
int cauchy_256_decode_batch(int k, int m, int block_bytes, int groups, void *d_blocks,
                            unsigned char *d_rows, void *stream);

/*
 * Out-of-place decode: blocks and rows are read only. Group g's recovered originals go to
 * d_out[g][0 .. e_g-1][block_bytes] (dense, emax = min(k, m) slots per group) in the order the
 * in-place call would write them (i-th recovery block in array order <- i-th smallest erasure);
 * d_out_rows[g][i] receives that erasure index and d_out_count[g] = e_g. m >= 2 only.
 */
int cauchy_256_decode_batch_out(int k, int m, int block_bytes, int groups, const void *d_blocks,
                                const unsigned char *d_rows, void *d_out, unsigned char *d_out_rows,
                                int *d_out_count, void *stream);

/* Pre-allocate the internal decode workspace so later calls allocate nothing (graph capture).
 * Workspaces are per stream (decodes in flight on different streams never share scratch):
 * cauchy_256_batch_reserve sizes the null stream's workspace and the minimum size of every
 * workspace created later; cauchy_256_batch_reserve_stream does the same for `stream`. */
int cauchy_256_batch_reserve(int k, int m, int block_bytes, int groups);
int cauchy_256_batch_reserve_stream(int k, int m, int block_bytes, int groups, void *stream);

/* Malformed decode groups (more recovery blocks than erased originals: duplicate rows, outside
 * the reference's contract) are left untouched, counted, and flagged with d_out_count[g] = -1 by
 * cauchy_256_decode_batch_out. Counts are kept per stream: this waits for `stream` and returns the
 * number of such groups among the decodes enqueued on `stream` since the previous call for that
 * stream (read and reset in stream order), or -2 on a GPU error. The single-group
 * cauchy_256_decode returns -1 for such a group and counts it nowhere (it decodes on a private
 * staging stream).
 * Every entry point runs on the library's device and restores the calling thread's current HIP
 * device before it returns. */
int cauchy_256_batch_errors(void *stream);

/* Synthetic workload: block x of group g0+g = PCG32 Seed((g0+g)*256 + x, cfg) words (the same
 * stream as the test oracle), written to d_out[groups][n][block_bytes]. */
int cauchy_256_fill_synthetic(void *d_out, int n, int block_bytes, int groups,
                              unsigned long long g0, unsigned long long cfg, void *stream);

/* Synthetic erasure pattern of group g (host only, no GPU): rows_out[0..k-1] = the decoder's
 * input rows (survivors ascending, then e chosen recovery rows k+y ascending), same stream as the
 * test oracle; e = e_fixed (clamped to min(k, m)) or PCG-random in [1, min(k, m)] when 0.
 * Returns e, or -1 on bad arguments. */
int cauchy_256_erasure_pattern(unsigned long long g, int k, int m, unsigned long long cfg, int e_fixed,
                               unsigned char *rows_out);

/* Which kernels code (k, m, block_bytes): 1 = compile-time-scheduled (generated for this (k, m), or
 * for a larger K of the same m with k >= 0.6 K, whose steps past k then read zeros),
 * 2 = the runtime-coefficient tile kernels (any other (k, m) with block_bytes/8 >= 16),
 * 0 = the generic per-column kernels (shorter blocks), -1 = invalid parameters. Host-only: never
 * initialises the GPU. Before the library is initialised, 2 assumes the snippet table loaded
 * inside one 4 GB page (checked at launch, generic kernels otherwise); afterwards it includes it. */
int cauchy_256_batch_path(int k, int m, int block_bytes);

/* The library's stream (the batched calls' stream when they are passed a null stream) and a
 * synchronize helper for callers without HIP. The single-group calls use their own staging
 * streams (up to 8, one per concurrent call), so calls from different threads overlap. */
void *cauchy_256_default_stream(void);
int cauchy_256_sync(void *stream);

/* Measurement hooks (bench.py's roofline): after cauchy_256_profile(n), each batched decode on
 * the compile-time path records HIP events on its stream around its three kernels (the last n
 * decodes are kept; nothing synchronises while recording; n = 0 turns it off).
 * profile_read waits for them and returns ms[0..2] = mean setup, stage A and stage B times and
 * the number of decodes averaged (-1: none recorded). cauchy_256_profile(-n) records only the two
 * events around stage A (the headline's dominant kernel) of the last n decodes: ms[1] is then its
 * mean time and ms[0], ms[2] are -1. */
int cauchy_256_profile(int capacity);
int cauchy_256_profile_read(float *ms);

#ifdef __cplusplus
}
#endif

#endif /* SH_AMD_CAUCHY_256_BATCH_H */
