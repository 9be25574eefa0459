/*
 * CPU baseline timer -- TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).
 *
 * Times the REFERENCE codec (oracle/_ref/libref_cauchy.so: catid/shorthair cauchy_256.cpp +
 * gf256.cpp compiled by oracle/Makefile) on host threads, on the same synthetic inputs as the GPU
 * run (oracle/_ref/liboracle.so: PCG32 blocks and erasure patterns). Each thread codes its own
 * stream of groups: encode k data blocks -> m recovery blocks, then decode the group with e
 * erased originals (in place, reference semantics). Only the codec calls are timed; restoring
 * the decode buffers between calls is not.
 *
 *   cpu_bench K M B E THREADS SECONDS MODE      MODE: shipped | init
 *
 * "shipped" leaves gf256_init() uncalled, as Shorthair does (its XOR helpers then take the SSE2
 * path); "init" calls gf256_init() first (AVX2 helpers, gf256.cpp:622).
 * Prints one line: key=value pairs (groups, seconds, GiBps, us_per_encode, us_per_decode).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "cauchy_oracle.h"

typedef struct {
    unsigned char *data;
    unsigned char row;
} Block;

/* reference ABI (cauchy_256.h:47-103, gf256.h:200) */
extern int _cauchy_256_init(int expected_version);
extern int cauchy_256_encode(int k, int m, const unsigned char *data_ptrs[], void *recovery_blocks,
                             int block_bytes);
extern int cauchy_256_decode(int k, int m, Block *blocks, int block_bytes);
extern int gf256_init_(int version);

static int K, M, BB, E;
static double SECONDS;

typedef struct {
    int id;
    long groups;
    double t_enc, t_dec;
    long bytes;
} Work;

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

#define NS 4 /* distinct groups per thread, cycled */

static void *run(void *arg) {
    Work *w = (Work *)arg;
    const size_t blk = (size_t)BB;
    unsigned char *data[NS], *rec[NS], *whole[NS], *work, rows[NS][256];
    int es[NS];
    for (int s = 0; s < NS; ++s) {
        const uint64_t g = (uint64_t)w->id * NS + s;
        data[s] = malloc((size_t)K * blk);
        rec[s] = malloc((size_t)M * blk);
        whole[s] = malloc((size_t)(K + M) * blk);
        for (int x = 0; x < K; ++x) ora_fill_block(g, x, 0xBE, data[s] + x * blk, BB);
        es[s] = ora_erasure_pattern(g, K, M, 0xBE, E, rows[s]);
    }
    work = malloc((size_t)K * blk);
    const unsigned char *ptrs[256];
    Block blocks[256];
    /* recovery blocks for the decode inputs (one encode per distinct group, untimed) */
    for (int s = 0; s < NS; ++s) {
        for (int x = 0; x < K; ++x) ptrs[x] = data[s] + x * blk;
        cauchy_256_encode(K, M, ptrs, rec[s], BB);
        memcpy(whole[s], data[s], (size_t)K * blk);
        memcpy(whole[s] + (size_t)K * blk, rec[s], (size_t)M * blk);
    }
    const double stop = now() + SECONDS;
    long i = 0;
    while (now() < stop) {
        const int s = (int)(i % NS);
        for (int x = 0; x < K; ++x) ptrs[x] = data[s] + x * blk;
        double t0 = now();
        cauchy_256_encode(K, M, ptrs, rec[s], BB);
        double t1 = now();
        for (int x = 0; x < K; ++x) {
            memcpy(work + x * blk, whole[s] + (size_t)rows[s][x] * blk, blk);
            blocks[x].data = work + x * blk;
            blocks[x].row = rows[s][x];
        }
        double t2 = now();
        cauchy_256_decode(K, M, blocks, BB);
        double t3 = now();
        w->t_enc += t1 - t0;
        w->t_dec += t3 - t2;
        w->bytes += (long)(K + M) * BB + (long)(K + es[s]) * BB;
        ++w->groups;
        ++i;
    }
    for (int s = 0; s < NS; ++s) {
        free(data[s]);
        free(rec[s]);
        free(whole[s]);
    }
    free(work);
    return NULL;
}

int main(int argc, char **argv) {
    if (argc != 8) {
        fprintf(stderr, "usage: %s K M B E THREADS SECONDS shipped|init\n", argv[0]);
        return 2;
    }
    K = atoi(argv[1]);
    M = atoi(argv[2]);
    BB = atoi(argv[3]);
    E = atoi(argv[4]);
    const int T = atoi(argv[5]);
    SECONDS = atof(argv[6]);
    const int init = strcmp(argv[7], "init") == 0;
    if (K < 2 || M < 2 || K + M > 256 || BB % 8 || T < 1 || T > 1024) return 2;
    ora_init();
    if (_cauchy_256_init(2) != 0) return 1;
    if (init && gf256_init_(2) != 0) return 1;
    Work *w = calloc((size_t)T, sizeof(Work));
    pthread_t *th = malloc(sizeof(pthread_t) * (size_t)T);
    const double t0 = now();
    for (int t = 0; t < T; ++t) {
        w[t].id = t;
        pthread_create(&th[t], NULL, run, &w[t]);
    }
    long groups = 0, bytes = 0;
    double te = 0, td = 0;
    for (int t = 0; t < T; ++t) {
        pthread_join(th[t], NULL);
        groups += w[t].groups;
        bytes += w[t].bytes;
        te += w[t].t_enc;
        td += w[t].t_dec;
    }
    const double wall = now() - t0;
    /* throughput over the codec-call time of the threads (buffer restores excluded) */
    const double codec = (te + td) / T;
    printf("groups=%ld seconds=%.3f codec_seconds=%.3f GiBps=%.4f us_per_encode=%.1f us_per_decode=%.1f\n",
           groups, wall, codec, bytes / codec / 1073741824.0, 1e6 * te / groups, 1e6 * td / groups);
    free(w);
    free(th);
    return 0;
}
