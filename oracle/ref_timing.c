/*
 * ref_timing.c -- TEST/BENCH INFRASTRUCTURE ONLY. CPU baseline for bench.py.
 *
 * Built by oracle/Makefile into oracle/_ref/libccref_{awgn,bsc}[_stack].so together with an UNMODIFIED
 * reference decoder (AWGN-channel/viterbi-decoder.c or binary-symmetric-channel/viterbi-decoder.c, or
 * the stack-decoder.c of either channel).
 * It feeds pre-generated decoder input to the reference decoder one trellis step per decoder_input()
 * call, as the reference drivers do (AWGN-channel/main.c:108-116, binary-symmetric-channel/main.c:70),
 * on NTHREADS threads, one decoder handle per thread (the decoder keeps no globals), and returns the
 * wall time of the decode alone.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "code.h"
#include "decoder.h"

typedef struct {
    struct code_param param;
    uint64_t polys[8];
    const void* in;
    uint8_t* out;
    int32_t* pm;
    size_t first, count, done;
    size_t steps, out_bytes, in_step_bytes;
    int rc;
} job_t;

/* Stack / Fano builds (libccref_*_{stack,fano}.so): the sequential decoders' metrics (code.h:14-17). */
static float g_metric_weight = -15.0f;
static int32_t g_bit_metrics[2] = {1, -15};
void ccref_set_stack_metrics(float metric_weight, int32_t bm0, int32_t bm1) {
    g_metric_weight = metric_weight;
    g_bit_metrics[0] = bm0;
    g_bit_metrics[1] = bm1;
}

#ifdef TIMING_AWGN
static int on_decoded(uint8_t* data, uint8_t len, void* ud) {
    (void)len;
    job_t* j = (job_t*)ud;
    memcpy(j->out + (j->first + j->done) * j->out_bytes, data, j->out_bytes);
    j->done++;
    return -1;
}
#else
static int on_decoded(uint8_t* data, uint8_t len, int32_t path_metric, void* ud) {
    (void)len;
    job_t* j = (job_t*)ud;
    memcpy(j->out + (j->first + j->done) * j->out_bytes, data, j->out_bytes);
    if (j->pm) j->pm[j->first + j->done] = path_metric;
    j->done++;
    return -1;
}
#endif

static void* run_job(void* arg) {
    job_t* j = (job_t*)arg;
    struct decoder* d = decoder_create();
    j->param.userdata = j;
    j->param.polynomials = j->polys;
    j->param.metric_weight = j->param.fano_metric_weight = g_metric_weight;
    j->param.bit_metrics = j->param.fano_bit_metrics = g_bit_metrics;
    if (!d || decoder_init(d, &j->param) != 0) { j->rc = -1; return NULL; }
    decoder_register_callback(d, on_decoded);
    const uint8_t* base = (const uint8_t*)j->in + j->first * j->steps * j->in_step_bytes;
#ifdef TIMING_AWGN
    uint8_t per_call = (uint8_t)(j->in_step_bytes / sizeof(float));
    for (size_t s = 0; s < j->count * j->steps; ++s)
        (void)decoder_input(d, (float*)(base + s * j->in_step_bytes), per_call);
#else
    for (size_t s = 0; s < j->count * j->steps; ++s)
        (void)decoder_input(d, (uint8_t*)(base + s), 1);
#endif
    decoder_destroy(&d);
    j->rc = j->done == j->count ? 0 : -1;
    return NULL;
}

/* Decode nblocks blocks of pre-generated decoder input with the reference decoder on nthreads
 * threads. Returns wall seconds, or a negative value on failure. */
double ccref_decode(int n, int K, int blen, const uint64_t* polys, const void* in, size_t nblocks,
                    uint8_t* out, int32_t* path_metric, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    job_t* jobs = (job_t*)calloc((size_t)nthreads, sizeof(job_t));
    pthread_t* tids = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    size_t steps = (size_t)blen + K - 1;
    size_t per = nblocks / (size_t)nthreads, extra = nblocks % (size_t)nthreads, first = 0;
    for (int t = 0; t < nthreads; ++t) {
        job_t* j = &jobs[t];
        j->param.symlen_out = (uint8_t)n;
        j->param.constr_len = (uint8_t)K;
        j->param.block_len = (uint8_t)blen;
        memcpy(j->polys, polys, sizeof(uint64_t) * (size_t)n);
        j->in = in;
        j->out = out;
        j->pm = path_metric;
        j->first = first;
        j->count = per + ((size_t)t < extra ? 1 : 0);
        j->steps = steps;
        j->out_bytes = (steps + 7) / 8;
#ifdef TIMING_AWGN
        j->in_step_bytes = sizeof(float) << n;
#else
        j->in_step_bytes = 1;
#endif
        first += j->count;
    }
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < nthreads; ++t) pthread_create(&tids[t], NULL, run_job, &jobs[t]);
    for (int t = 0; t < nthreads; ++t) pthread_join(tids[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    int rc = 0;
    for (int t = 0; t < nthreads; ++t) rc |= jobs[t].rc;
    free(jobs);
    free(tids);
    if (rc) return -1.0;
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
