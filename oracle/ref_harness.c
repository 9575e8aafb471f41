/*
 * ref_harness.c -- TEST INFRASTRUCTURE ONLY. Golden-vector generator.
 *
 * Linked (by oracle/Makefile) against the UNMODIFIED reference sources under /root/reference; it
 * drives them exactly as the reference drivers do (AWGN-channel/main.c:80-144,212-229 and
 * binary-symmetric-channel/main.c:57-98,159-172) but seeds rand() with a fixed seed and records the
 * data crossing the decoder boundary: info bytes, the decoder's input stream, the decoder's output
 * buffer (all ceil(T/8) bytes, tail bits included), the BSC path metric and the bit-error count.
 *
 * usage: ref_harness_{awgn,bsc}[_stack] OUTPREFIX SEED NBLOCKS CHANNELPARAM CODESPEC [METRICS]
 *   CHANNELPARAM: AWGN noise scaling factor (float) | BSC crossover probability in ppm (int)
 *   CODESPEC:     cb:<codebook index>  |  n:K:blen:poly0hex:poly1hex[:poly2hex]
 *   METRICS:      stack decoder metrics overriding the codebook's (code.h:14-16):
 *                 AWGN metric_weight (float) | BSC bit_metrics "m0,m1"
 * The same harness is linked against viterbi-decoder.c, stack-decoder.c or fano-decoder.c
 * (oracle/Makefile).
 * writes OUTPREFIX.info .rx .out [.pm] .meta
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "code.h"
#include "codebook.h"
#include "decoder.h"
#include "encoder.h"
#ifdef HARNESS_AWGN
#include "demapper.h"
#include "gaussian.h"
#include "mapper.h"
#endif

typedef struct {
    struct code_param param;
    struct encoder* encoder;
    struct decoder* decoder;
#ifdef HARNESS_AWGN
    struct mapper* mapper;
    struct demapper* demapper;
    float scaling;
#else
    int32_t p_ppm;
#endif
    uint8_t info[40];
    size_t block;
    uint64_t errors;
    FILE *f_rx, *f_out, *f_pm;
} harness_t;

/* wall time spent inside decoder_input() (the decoder, and the output callback it calls) */
static double g_decoder_seconds = 0.0;
static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}
static void timed_decoder_input(struct decoder* d, void* data, uint8_t len) {
    double t0 = now_s();
#ifdef HARNESS_AWGN
    (void)decoder_input(d, (float*)data, len);
#else
    (void)decoder_input(d, (uint8_t*)data, len);
#endif
    g_decoder_seconds += now_s() - t0;
}

static size_t steps_of(const struct code_param* p) { return (size_t)p->block_len + p->constr_len - 1; }

static void count_errors(harness_t* h, const uint8_t* data, uint8_t len) {
    for (int i = 0; i < len; ++i) {
        uint8_t a = (uint8_t)((h->info[i / 8] << (i % 8)) & 0x80);
        uint8_t d = (uint8_t)((data[i / 8] << (i % 8)) & 0x80);
        h->errors += (a != d);
    }
}

#ifdef HARNESS_AWGN
static int on_encoded(uint8_t* data, uint8_t len, void* ud) {
    harness_t* h = (harness_t*)ud;
    (void)mapper_input(h->mapper, data, len);
    return -1;
}
static int on_mapped(float* data, uint8_t len, void* ud) {
    harness_t* h = (harness_t*)ud;
    for (uint8_t i = 0; i < len; ++i) data[i] += h->scaling * gengauss();
    (void)demapper_input(h->demapper, data, len);
    return -1;
}
static int on_demapped(float* data, uint8_t len, void* ud) {
    harness_t* h = (harness_t*)ud;
    fwrite(data, sizeof(float), len, h->f_rx);
    timed_decoder_input(h->decoder, data, len);
    return -1;
}
static int on_decoded(uint8_t* data, uint8_t len, void* ud) {
    harness_t* h = (harness_t*)ud;
    fwrite(data, 1, (steps_of(&h->param) + 7) / 8, h->f_out);
    count_errors(h, data, len);
    h->block++;
    return -1;
}
#else
static int on_encoded(uint8_t* data, uint8_t len, void* ud) {
    harness_t* h = (harness_t*)ud;
    for (uint8_t i = 0; i < len; ++i)
        for (uint8_t k = 0; k < h->param.symlen_out; ++k)
            if ((rand() % 1000000) < h->p_ppm) data[i] ^= (uint8_t)(1 << k);
    fwrite(data, 1, len, h->f_rx);
    timed_decoder_input(h->decoder, data, len);
    return -1;
}
static int on_decoded(uint8_t* data, uint8_t len, int32_t path_metric, void* ud) {
    harness_t* h = (harness_t*)ud;
    fwrite(data, 1, (steps_of(&h->param) + 7) / 8, h->f_out);
    fwrite(&path_metric, sizeof(int32_t), 1, h->f_pm);
    count_errors(h, data, len);
    h->block++;
    return -1;
}
#endif

static uint64_t custom_polys[8];
static int32_t custom_bit_metrics[2];

static int parse_code(const char* spec, struct code_param* p) {
    if (strncmp(spec, "cb:", 3) == 0) {
        get_code((uint8_t)atoi(spec + 3), p);
        return 0;
    }
    char buf[256];
    snprintf(buf, sizeof buf, "%s", spec);
    char* tok = strtok(buf, ":");
    int field = 0, npoly = 0;
    memset(p, 0, sizeof *p);
    while (tok) {
        if (field == 0) p->symlen_out = (uint8_t)atoi(tok);
        else if (field == 1) p->constr_len = (uint8_t)atoi(tok);
        else if (field == 2) p->block_len = (uint8_t)atoi(tok);
        else if (npoly < 8) custom_polys[npoly++] = strtoull(tok, NULL, 16);
        ++field;
        tok = strtok(NULL, ":");
    }
    if (npoly != p->symlen_out) return -1;
    p->polynomials = custom_polys;
    return 0;
}

static FILE* open_out(const char* prefix, const char* ext) {
    char path[512];
    snprintf(path, sizeof path, "%s.%s", prefix, ext);
    FILE* f = fopen(path, "wb");
    if (!f) { perror(path); exit(2); }
    return f;
}

int main(int argc, char** argv) {
    if (argc != 6 && argc != 7) {
        fprintf(stderr, "usage: %s OUTPREFIX SEED NBLOCKS CHANNELPARAM CODESPEC [METRICS]\n", argv[0]);
        return 2;
    }
    const char* prefix = argv[1];
    unsigned seed = (unsigned)strtoul(argv[2], NULL, 10);
    long nblocks = atol(argv[3]);
    harness_t h;
    memset(&h, 0, sizeof h);
    if (parse_code(argv[5], &h.param) != 0) { fprintf(stderr, "bad code spec\n"); return 2; }
    /* METRICS overrides both the stack and the Fano fields (only one decoder is linked) */
#ifdef HARNESS_AWGN
    h.scaling = (float)atof(argv[4]);
    if (argc == 7) h.param.metric_weight = h.param.fano_metric_weight = (float)atof(argv[6]);
#else
    h.p_ppm = (int32_t)atol(argv[4]);
    if (argc == 7) {
        if (sscanf(argv[6], "%d,%d", &custom_bit_metrics[0], &custom_bit_metrics[1]) != 2) return 2;
        h.param.bit_metrics = h.param.fano_bit_metrics = custom_bit_metrics;
    }
#endif
    h.param.userdata = &h;
    h.encoder = encoder_create();
    h.decoder = decoder_create();
    (void)encoder_init(h.encoder, &h.param);
    encoder_register_callback(h.encoder, on_encoded);
    (void)decoder_init(h.decoder, &h.param);
    decoder_register_callback(h.decoder, on_decoded);
#ifdef HARNESS_AWGN
    h.mapper = mapper_create();
    h.demapper = demapper_create();
    (void)mapper_init(h.mapper, &h.param);
    mapper_register_callback(h.mapper, on_mapped);
    (void)demapper_init(h.demapper, &h.param);
    demapper_register_callback(h.demapper, on_demapped);
#endif
    FILE* f_info = open_out(prefix, "info");
    h.f_rx = open_out(prefix, "rx");
    h.f_out = open_out(prefix, "out");
#ifndef HARNESS_AWGN
    h.f_pm = open_out(prefix, "pm");
#endif
    double t_start = now_s();
    srand(seed);
    size_t ib = ((size_t)h.param.block_len + 7) / 8;
    for (long k = 0; k < nblocks; ++k) {
        for (size_t j = 0; j < ib; ++j) h.info[j] = (uint8_t)(rand() % 256);
        fwrite(h.info, 1, ib, f_info);
        (void)encoder_input(h.encoder, h.info, h.param.block_len);
    }
    double wall = now_s() - t_start;
    fclose(f_info);
    fclose(h.f_rx);
    fclose(h.f_out);
    if (h.f_pm) fclose(h.f_pm);
    FILE* meta = open_out(prefix, "meta");
    fprintf(meta, "blocks_decoded %zu\nerrors %llu\nn %d\nK %d\nblen %d\n", h.block,
            (unsigned long long)h.errors, h.param.symlen_out, h.param.constr_len, h.param.block_len);
    for (int k = 0; k < h.param.symlen_out; ++k)
        fprintf(meta, "poly%d %016llx\n", k, (unsigned long long)h.param.polynomials[k]);
    fprintf(meta, "metric_weight %.9g\n", (double)h.param.metric_weight);
    fprintf(meta, "fano_metric_weight %.9g\n", (double)h.param.fano_metric_weight);
    fprintf(meta, "fano_bit_metric0 %d\nfano_bit_metric1 %d\n",
            h.param.fano_bit_metrics ? h.param.fano_bit_metrics[0] : 0,
            h.param.fano_bit_metrics ? h.param.fano_bit_metrics[1] : 0);
    fprintf(meta, "bit_metric0 %d\nbit_metric1 %d\n", h.param.bit_metrics ? h.param.bit_metrics[0] : 0,
            h.param.bit_metrics ? h.param.bit_metrics[1] : 0);
    fprintf(meta, "decoder_seconds %.6f\nwall_seconds %.6f\n", g_decoder_seconds, wall);
    fclose(meta);
    return h.block == (size_t)nblocks ? 0 : 1;
}
