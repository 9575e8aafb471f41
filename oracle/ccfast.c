/*
 * ccfast.c -- BENCH INFRASTRUCTURE ONLY. An optimised CPU Viterbi decoder for bench.py's second CPU
 * baseline ("optimized table-driven CPU decoder"), next to the reference
 * decoder itself (oracle/_ref). Only bench.py's cpu_baseline leg and tests/ load it; the product path
 * never does.
 *
 * Same arithmetic and tie rules as the reference (AWGN-channel/viterbi-decoder.c:71-141,
 * binary-symmetric-channel/viterbi-decoder.c:75-150), restated as the closed form of SURVEY.md
 * Appendix A: for new state ns, i = ns >> (K-2), s0 = 2 (ns mod S/2): m0 = M[s0] + bm(exp[s0][i]),
 * m1 = M[s0|1] + bm(exp[s0|1][i]), d = m1 < m0, M' = d ? m1 : m0; lowest-index argmin; traceback
 * through the decisions, tail bits included. Expected symbols come from a table (cco_trellis) instead
 * of the reference's per-branch parities, and the ACS runs on 8 blocks at once in AVX2 lanes (fp32 adds
 * and compares: bit-identical to the scalar reference; no FMA, -ffp-contract=off) -- soft metrics one
 * __m256 per state, hard metrics 16-bit with the reference's 0xFF00 saturation. Blocks are split over
 * pthreads. Output bytes and BSC path metrics equal the reference's.
 */
#include <immintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ccoracle.h"

#define VB 8            /* blocks per vector group */
#define MAXS 256        /* K <= 9 */
#define MAXT 264

typedef struct {
    const cco_code* c;
    const uint8_t* exp;     /* [S][2] */
    const void* in;         /* soft float [nb][T][2^n] / hard uint8 [nb][T] */
    uint8_t* out;           /* [nb][OB] */
    int32_t* pm;            /* hard: [nb] */
    size_t first, count;
    int hard;
} job_t;

static void traceback_out(const cco_code* c, const uint8_t* dec /* [T][S] bytes: bit b = block b */, int b,
                          uint32_t st, uint8_t* out) {
    const int K = c->K, T = c->blen + K - 1, S = 1 << (K - 1), OB = (T + 7) / 8;
    memset(out, 0, (size_t)OB);
    for (int t = T - 1; t >= 0; --t) {
        const uint32_t bit = (dec[(size_t)t * S + st] >> b) & 1u;
        out[t / 8] |= (uint8_t)((st >> (K - 2)) << (7 - t % 8));
        st = ((st << 1) & (uint32_t)(S - 1)) | bit;
    }
}

static void soft_group(const job_t* j, size_t g0, int nb, uint8_t* dec) {
    const cco_code* c = j->c;
    const int K = c->K, T = c->blen + K - 1, S = 1 << (K - 1), H = S / 2, NS = 1 << c->n;
    const int OB = (T + 7) / 8;
    const float* rx = (const float*)j->in;
    __m256 Ma[MAXS], Mb[MAXS], bm[8];
    __m256 *M = Ma, *N = Mb;
    const __m256 inf = _mm256_set1_ps(__builtin_inff());
    for (int s = 0; s < S; ++s) M[s] = s ? inf : _mm256_setzero_ps();
    for (int t = 0; t < T; ++t) {
        float tmp[8][VB];
        for (int b = 0; b < VB; ++b) {
            const int bb = b < nb ? b : nb - 1;
            const float* p = rx + ((g0 + (size_t)bb) * (size_t)T + (size_t)t) * (size_t)NS;
            for (int k = 0; k < NS; ++k) tmp[k][b] = p[k];
        }
        for (int k = 0; k < NS; ++k) bm[k] = _mm256_loadu_ps(tmp[k]);
        uint8_t* d = dec + (size_t)t * S;
        for (int ns = 0; ns < S; ++ns) {
            const int i = ns >> (K - 2), s0 = (ns & (H - 1)) << 1;
            const __m256 m0 = _mm256_add_ps(M[s0], bm[j->exp[2 * s0 + i]]);
            const __m256 m1 = _mm256_add_ps(M[s0 | 1], bm[j->exp[2 * (s0 | 1) + i]]);
            const __m256 lt = _mm256_cmp_ps(m1, m0, _CMP_LT_OQ);     /* strict <: ties keep s0 */
            N[ns] = _mm256_blendv_ps(m0, m1, lt);
            d[ns] = (uint8_t)_mm256_movemask_ps(lt);
        }
        __m256* x = M; M = N; N = x;
    }
    float Mf[MAXS][VB];
    for (int s = 0; s < S; ++s) _mm256_storeu_ps(Mf[s], M[s]);
    for (int b = 0; b < nb; ++b) {
        float best = __builtin_inff();
        uint32_t st = 0;
        for (int s = 0; s < S; ++s)
            if (Mf[s][b] < best) { best = Mf[s][b]; st = (uint32_t)s; }   /* lowest index wins */
        traceback_out(c, dec, b, st, j->out + (g0 + (size_t)b) * (size_t)OB);
    }
}

/* 16 blocks per group in 16-bit lanes; decisions as 16-bit masks (two bytes per state and step). */
static void hard_group(const job_t* j, size_t g0, int nb, uint16_t* dec) {
    const cco_code* c = j->c;
    const int K = c->K, T = c->blen + K - 1, S = 1 << (K - 1), H = S / 2, NS = 1 << c->n;
    const int OB = (T + 7) / 8;
    const uint8_t* syms = (const uint8_t*)j->in;
    __m256i Ma[MAXS], Mb[MAXS], bm[8];
    __m256i *M = Ma, *N = Mb;
    const __m256i sat = _mm256_set1_epi16((short)0xFF00), flip = _mm256_set1_epi16((short)0x8000);
    for (int s = 0; s < S; ++s) M[s] = s ? sat : _mm256_setzero_si256();
    for (int t = 0; t < T; ++t) {
        uint16_t tmp[8][16];
        for (int b = 0; b < 16; ++b) {
            const int bb = b < nb ? b : nb - 1;
            const uint32_t r = syms[(g0 + (size_t)bb) * (size_t)T + (size_t)t] & (uint32_t)(NS - 1);
            for (int k = 0; k < NS; ++k) tmp[k][b] = (uint16_t)__builtin_popcount((uint32_t)k ^ r);
        }
        for (int k = 0; k < NS; ++k) bm[k] = _mm256_loadu_si256((const __m256i*)tmp[k]);
        uint16_t* d = dec + (size_t)t * S;
        for (int ns = 0; ns < S; ++ns) {
            const int i = ns >> (K - 2), s0 = (ns & (H - 1)) << 1;
            /* binary-symmetric-channel/viterbi-decoder.c:127-131: saturate at 0xFF00, strict < */
            const __m256i m0 = _mm256_min_epu16(_mm256_add_epi16(M[s0], bm[j->exp[2 * s0 + i]]), sat);
            const __m256i m1 = _mm256_min_epu16(_mm256_add_epi16(M[s0 | 1], bm[j->exp[2 * (s0 | 1) + i]]), sat);
            const __m256i lt = _mm256_cmpgt_epi16(_mm256_xor_si256(m0, flip), _mm256_xor_si256(m1, flip));
            N[ns] = _mm256_blendv_epi8(m0, m1, lt);
            const uint32_t mm = (uint32_t)_mm256_movemask_epi8(lt);
            d[ns] = (uint16_t)_pext_u32(mm, 0x55555555u);
        }
        __m256i* x = M; M = N; N = x;
    }
    uint16_t Mh[MAXS][16];
    for (int s = 0; s < S; ++s) _mm256_storeu_si256((__m256i*)Mh[s], M[s]);
    for (int b = 0; b < nb; ++b) {
        uint32_t best = 0xFF00u, st = 0;
        for (int s = 0; s < S; ++s)
            if (Mh[s][b] < best) { best = Mh[s][b]; st = (uint32_t)s; }
        if (j->pm) j->pm[g0 + (size_t)b] = (int32_t)best;
        /* traceback over 16-bit masks */
        const int Kc = c->K;
        uint8_t* o = j->out + (g0 + (size_t)b) * (size_t)OB;
        memset(o, 0, (size_t)OB);
        for (int t = T - 1; t >= 0; --t) {
            const uint32_t bit = (dec[(size_t)t * S + st] >> b) & 1u;
            o[t / 8] |= (uint8_t)((st >> (Kc - 2)) << (7 - t % 8));
            st = ((st << 1) & (uint32_t)(S - 1)) | bit;
        }
    }
}

static void* run_job(void* arg) {
    job_t* j = (job_t*)arg;
    const int T = j->c->blen + j->c->K - 1, S = 1 << (j->c->K - 1);
    void* dec = malloc((size_t)T * (size_t)S * 2);
    const int G = j->hard ? 16 : VB;
    for (size_t g = 0; g < j->count; g += (size_t)G) {
        const int nb = (int)(j->count - g < (size_t)G ? j->count - g : (size_t)G);
        if (j->hard) hard_group(j, j->first + g, nb, (uint16_t*)dec);
        else soft_group(j, j->first + g, nb, (uint8_t*)dec);
    }
    free(dec);
    return NULL;
}

/* Decodes nblocks blocks on `threads` threads; returns the wall seconds of the decode, or -1. */
double ccfast_viterbi(const cco_code* c, int hard, const void* in, size_t nblocks, uint8_t* out, int32_t* pm,
                      int threads) {
    if (c->K < 2 || c->K > 9 || c->n < 1 || c->n > 3 || c->blen + c->K - 1 > MAXT) return -1.0;
    const int S = 1 << (c->K - 1);
    uint8_t exp[2 * MAXS];
    cco_trellis(c, exp);
    (void)S;
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    job_t* jobs = (job_t*)calloc((size_t)threads, sizeof(job_t));
    const size_t G = hard ? 16 : VB;
    const size_t groups = (nblocks + G - 1) / G, per = groups / (size_t)threads, extra = groups % (size_t)threads;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    size_t first = 0;
    for (int k = 0; k < threads; ++k) {
        size_t cnt = (per + ((size_t)k < extra ? 1 : 0)) * G;
        if (first + cnt > nblocks) cnt = nblocks > first ? nblocks - first : 0;
        jobs[k] = (job_t){c, exp, in, out, pm, first, cnt, hard};
        first += cnt;
        pthread_create(&th[k], NULL, run_job, &jobs[k]);
    }
    for (int k = 0; k < threads; ++k) pthread_join(th[k], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(th);
    free(jobs);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
