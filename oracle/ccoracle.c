/*
 * ccoracle.c -- TEST INFRASTRUCTURE ONLY (see ccoracle.h).
 *
 * CPU restatement of the reference's Viterbi hot path and its producers/consumer. Each function
 * cites the reference file:line it restates (paths relative to the reference repository root).
 * Compiled with gcc -O2 and no -march flags so, like the reference build (CMakeLists.txt:5), no
 * FMA contraction can change the fp32/fp64 channel arithmetic.
 */
#include "ccoracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- rand() / gengauss() */

/* glibc srandom_r/random_r, TYPE_3 (degree 31, separation 3). The reference seeds with
 * srand(time(NULL)) (AWGN-channel/main.c:147) and draws with rand(); golden harnesses use srand(seed). */
void cco_srand(cco_rng* g, uint32_t seed) {
    int32_t word = (int32_t)(seed == 0 ? 1u : seed);
    g->s[0] = (uint32_t)word;
    for (int i = 1; i < 31; ++i) {
        /* 16807 * word mod (2^31 - 1), Schrage's method exactly as glibc evaluates it */
        int32_t hi = word / 127773;
        int32_t lo = word % 127773;
        word = 16807 * lo - 2836 * hi;
        if (word < 0) word += 2147483647;
        g->s[i] = (uint32_t)word;
    }
    g->f = 3;
    g->r = 0;
    for (int i = 0; i < 310; ++i) (void)cco_rand(g);
    g->R = 0.0;
    g->T = 0.0;
    g->phase = 0;
}

int32_t cco_rand(cco_rng* g) {
    g->s[g->f] += g->s[g->r];
    int32_t out = (int32_t)(g->s[g->f] >> 1);
    g->f = (g->f + 1) % 31;
    g->r = (g->r + 1) % 31;
    return out;
}

/* common/gaussian.c:18-38: Box-Muller, cos half first, sin half cached for the next call. */
double cco_gengauss(cco_rng* g) {
    const double two_pi = 2.0 * 3.14159265358979323846;
    if (g->phase == 0) {
        double u1, u2;
        do {
            u1 = (double)cco_rand(g) / 2147483647.0;
            u2 = (double)cco_rand(g) / 2147483647.0;
        } while (u1 == 0.0);
        g->R = sqrt(-2.0 * log(u1));
        g->T = two_pi * u2;
        g->phase = 1;
        return g->R * cos(g->T);
    }
    g->phase = 0;
    return g->R * sin(g->T);
}

/* ---------------------------------------------------------------- trellis */

static int parity64(uint64_t v) {
    return __builtin_popcountll(v) & 1;
}

/* AWGN-channel/viterbi-decoder.c:50-57 (and encoder.c:93-100): generator bit of (sr & poly). */
int cco_gen_bit(uint64_t v, int gen_mode) {
    int p = parity64(v);
    if (gen_mode == CCO_GEN_REF_X86) {
        /* after the xor-fold, bit 4 of the shift count is the parity of v's bits 4,12,...,60;
         * when it is set the 5-bit-masked shift exceeds 15 and the result is 0. */
        p &= !parity64(v & 0x1010101010101010ull);
    }
    return p;
}

/* AWGN-channel/viterbi-decoder.c:45-63: shift register = state << (64-K) | input << 63; the
 * expected symbol packs polynomial 0 into its most significant bit. */
int cco_expected_symbol(const cco_code* c, uint32_t state, int input) {
    uint64_t sr = ((uint64_t)state << (64 - c->K)) | ((uint64_t)(input & 1) << 63);
    int e = 0;
    for (int k = 0; k < c->n; ++k) e = (e << 1) | cco_gen_bit(sr & c->poly[k], c->gen_mode);
    return e;
}

void cco_trellis(const cco_code* c, uint8_t* exp_sym) {
    uint32_t S = 1u << (c->K - 1);
    for (uint32_t s = 0; s < S; ++s)
        for (int i = 0; i < 2; ++i) exp_sym[2 * s + i] = (uint8_t)cco_expected_symbol(c, s, i);
}

size_t cco_steps(const cco_code* c) { return (size_t)c->blen + (size_t)c->K - 1; }
size_t cco_info_bytes(const cco_code* c) { return ((size_t)c->blen + 7) / 8; }
size_t cco_out_bytes(const cco_code* c) { return (cco_steps(c) + 7) / 8; }

/* ---------------------------------------------------------------- producers */

/* common/encoder.c:84-119: info bits MSB-first into bit 63 of a right-shifting register; K-1 zero
 * tail bits appended (encoder.c:112-115); one n-bit symbol per step, P0 in the MSB. */
void cco_encode_block(const cco_code* c, const uint8_t* info, uint8_t* syms) {
    size_t T = cco_steps(c);
    uint64_t sr = 0;
    for (size_t t = 0; t < T; ++t) {
        uint64_t bit = 0;
        if (t < (size_t)c->blen) bit = (info[t / 8] >> (7 - t % 8)) & 1u;
        sr = (sr >> 1) | (bit << 63);
        int e = 0;
        for (int k = 0; k < c->n; ++k) e = (e << 1) | cco_gen_bit(sr & c->poly[k], c->gen_mode);
        syms[t] = (uint8_t)e;
    }
}

/* common/constellations.c:6-28: unit-power Gray constellations (values as stored there). */
void cco_constellation(int n, float* pts) {
    static const float c1[] = {0.707107f, 0.707107f, -0.707107f, -0.707107f};
    static const float c2[] = {0.707107f, 0.707107f, 0.707107f, -0.707107f,
                               -0.707107f, 0.707107f, -0.707107f, -0.707107f};
    static const float c3[] = {0.408248f, 0.408248f, 0.408248f, 1.224745f,
                               -0.408248f, 0.408248f, -1.224745f, 0.408248f,
                               0.408248f, -0.408248f, 1.224745f, -0.408248f,
                               -0.408248f, -0.408248f, -0.408248f, -1.224745f};
    const float* src = n == 1 ? c1 : n == 2 ? c2 : c3;
    memcpy(pts, src, sizeof(float) * 2u * (1u << n));
}

/* common/demapper.c:43-45 (ndist) and :61-70 (normalised squared distances, fp32). */
void cco_demap(int n, float x, float y, float* out) {
    float pts[16];
    cco_constellation(n, pts);
    float ddx = pts[0] - pts[2];
    float ddy = pts[1] - pts[3];
    float ndist = (ddx * ddx) + (ddy * ddy);
    for (int k = 0; k < (1 << n); ++k) {
        float dx = x - pts[2 * k];
        float dy = y - pts[2 * k + 1];
        out[k] = ((dx * dx) + (dy * dy)) / ndist;
    }
}

/* common/hard-demapper.c:62-88: snap to the nearest constellation point (strict <, first minimum),
 * then the normalised squared distances from that point. */
void cco_demap_hard(int n, float x, float y, float* out) {
    float pts[16];
    cco_constellation(n, pts);
    float min_val = INFINITY;
    int min_idx = 0;
    for (int k = 0; k < (1 << n); ++k) {
        float dx = x - pts[2 * k];
        float dy = y - pts[2 * k + 1];
        float d = (dx * dx) + (dy * dy);
        if (d < min_val) { min_val = d; min_idx = k; }
    }
    cco_demap(n, pts[2 * min_idx], pts[2 * min_idx + 1], out);
}

/* AWGN-channel/main.c:212-229 (info bytes by rand()%256), :93-106 (noise added per I/Q sample in
 * double, stored back to float), common/mapper.c:54-71, common/demapper.c:61-85 or, hard != 0,
 * common/hard-demapper.c:62-102. */
void cco_awgn_blocks_demap(const cco_code* c, uint32_t seed, float scaling, size_t nblocks, int hard,
                           uint8_t* info, float* rx) {
    cco_rng g;
    cco_srand(&g, seed);
    size_t T = cco_steps(c), IB = cco_info_bytes(c), NS = (size_t)1 << c->n;
    float pts[16];
    cco_constellation(c->n, pts);
    uint8_t syms[520];
    for (size_t b = 0; b < nblocks; ++b) {
        uint8_t* ib = info + b * IB;
        for (size_t j = 0; j < IB; ++j) ib[j] = (uint8_t)(cco_rand(&g) % 256);
        cco_encode_block(c, ib, syms);
        for (size_t t = 0; t < T; ++t) {
            float x = pts[2 * syms[t]], y = pts[2 * syms[t] + 1];
            x = (float)((double)x + (double)scaling * cco_gengauss(&g));
            y = (float)((double)y + (double)scaling * cco_gengauss(&g));
            if (hard) cco_demap_hard(c->n, x, y, rx + (b * T + t) * NS);
            else cco_demap(c->n, x, y, rx + (b * T + t) * NS);
        }
    }
}

void cco_awgn_blocks(const cco_code* c, uint32_t seed, float scaling, size_t nblocks, uint8_t* info,
                     float* rx) {
    cco_awgn_blocks_demap(c, seed, scaling, nblocks, 0, info, rx);
}

/* binary-symmetric-channel/main.c:57-72 (per-bit flips with rand()%1000000 < p) and :159-172. */
void cco_bsc_blocks(const cco_code* c, uint32_t seed, int32_t p_ppm, size_t nblocks, uint8_t* info,
                    uint8_t* syms) {
    cco_rng g;
    cco_srand(&g, seed);
    size_t T = cco_steps(c), IB = cco_info_bytes(c);
    for (size_t b = 0; b < nblocks; ++b) {
        uint8_t* ib = info + b * IB;
        for (size_t j = 0; j < IB; ++j) ib[j] = (uint8_t)(cco_rand(&g) % 256);
        uint8_t* sb = syms + b * T;
        cco_encode_block(c, ib, sb);
        for (size_t t = 0; t < T; ++t)
            for (int k = 0; k < c->n; ++k)
                if ((cco_rand(&g) % 1000000) < p_ppm) sb[t] ^= (uint8_t)(1u << k);
    }
}

/* ---------------------------------------------------------------- decoders */

/* AWGN-channel/viterbi-decoder.c:108-141 (ACS: ascending s, inputs 0 then 1, strict <, +inf init
 * :109-112, :212-218) and :71-90 (traceback from the lowest-index argmin, tail bits included,
 * MSB-first). The uint8_t argmin counter (:74) is widened so K >= 9 terminates. */
void cco_viterbi_soft(const cco_code* c, const float* rx, size_t nblocks, uint8_t* out) {
    uint32_t S = 1u << (c->K - 1);
    size_t T = cco_steps(c), OB = cco_out_bytes(c), NS = (size_t)1 << c->n;
    uint8_t* exp_sym = (uint8_t*)malloc(2 * S);
    float* M = (float*)malloc(sizeof(float) * S);
    float* N = (float*)malloc(sizeof(float) * S);
    uint16_t* prev = (uint16_t*)malloc(sizeof(uint16_t) * S * T);
    uint8_t* inp = (uint8_t*)malloc(S * T);
    cco_trellis(c, exp_sym);
    memset(prev, 0, sizeof(uint16_t) * S * T);
    memset(inp, 0, S * T);
    for (size_t b = 0; b < nblocks; ++b) {
        for (uint32_t s = 0; s < S; ++s) M[s] = s ? INFINITY : 0.0f;
        for (size_t t = 0; t < T; ++t) {
            const float* r = rx + (b * T + t) * NS;
            for (uint32_t s = 0; s < S; ++s) N[s] = INFINITY;
            for (uint32_t s = 0; s < S; ++s) {
                for (int i = 0; i < 2; ++i) {
                    uint32_t ns = (s >> 1) | ((uint32_t)i << (c->K - 2));
                    float m = M[s] + r[exp_sym[2 * s + i]];
                    if (m < N[ns]) {
                        N[ns] = m;
                        prev[t * S + ns] = (uint16_t)s;
                        inp[t * S + ns] = (uint8_t)i;
                    }
                }
            }
            memcpy(M, N, sizeof(float) * S);
        }
        uint32_t st = 0;
        float best = INFINITY;
        for (uint32_t s = 0; s < S; ++s)
            if (M[s] < best) { best = M[s]; st = s; }
        uint8_t* ob = out + b * OB;
        memset(ob, 0, OB);
        for (size_t t = T; t-- > 0;) {
            ob[t / 8] |= (uint8_t)(inp[t * S + st] << (7 - t % 8));
            st = prev[t * S + st];
        }
    }
    free(exp_sym); free(M); free(N); free(prev); free(inp);
}

/* binary-symmetric-channel/viterbi-decoder.c:114-150 (uint16 metrics saturated at 0xFF00,
 * Hamming branch metric :68-72) and :75-96 (traceback; returns the minimum as the path metric). */
void cco_viterbi_hard(const cco_code* c, const uint8_t* syms, size_t nblocks, uint8_t* out,
                      int32_t* path_metric) {
    uint32_t S = 1u << (c->K - 1);
    size_t T = cco_steps(c), OB = cco_out_bytes(c);
    uint8_t mask = (uint8_t)((1u << c->n) - 1u);
    uint8_t* exp_sym = (uint8_t*)malloc(2 * S);
    uint16_t* M = (uint16_t*)malloc(sizeof(uint16_t) * S);
    uint16_t* N = (uint16_t*)malloc(sizeof(uint16_t) * S);
    uint16_t* prev = (uint16_t*)malloc(sizeof(uint16_t) * S * T);
    uint8_t* inp = (uint8_t*)malloc(S * T);
    cco_trellis(c, exp_sym);
    memset(prev, 0, sizeof(uint16_t) * S * T);
    memset(inp, 0, S * T);
    for (size_t b = 0; b < nblocks; ++b) {
        for (uint32_t s = 0; s < S; ++s) M[s] = s ? 0xFF00 : 0;
        for (size_t t = 0; t < T; ++t) {
            uint8_t rs = syms[b * T + t] & mask;   /* decoder_input masks (viterbi-decoder.c:235-237) */
            for (uint32_t s = 0; s < S; ++s) N[s] = 0xFF00;
            for (uint32_t s = 0; s < S; ++s) {
                for (int i = 0; i < 2; ++i) {
                    uint32_t ns = (s >> 1) | ((uint32_t)i << (c->K - 2));
                    uint32_t m = (uint32_t)M[s] + (uint32_t)__builtin_popcount(exp_sym[2 * s + i] ^ rs);
                    if (m > 0xFF00) m = 0xFF00;
                    if (m < N[ns]) {
                        N[ns] = (uint16_t)m;
                        prev[t * S + ns] = (uint16_t)s;
                        inp[t * S + ns] = (uint8_t)i;
                    }
                }
            }
            memcpy(M, N, sizeof(uint16_t) * S);
        }
        uint32_t st = 0;
        uint16_t best = 0xFF00;
        for (uint32_t s = 0; s < S; ++s)
            if (M[s] < best) { best = M[s]; st = s; }
        uint8_t* ob = out + b * OB;
        memset(ob, 0, OB);
        for (size_t t = T; t-- > 0;) {
            ob[t / 8] |= (uint8_t)(inp[t * S + st] << (7 - t % 8));
            st = prev[t * S + st];
        }
        if (path_metric) path_metric[b] = (int32_t)best;
    }
    free(exp_sym); free(M); free(N); free(prev); free(inp);
}

/* ---------------------------------------------------------------- stack decoders */

/* AWGN-channel/stack-decoder.c:243-276 / binary-symmetric-channel/stack-decoder.c:235-273: the
 * generator register is (state << (64-K)) | (input << 63) with a 64-bit state (K <= 64). */
static int stack_symbol(const cco_code* c, uint64_t state, int input, uint64_t* new_state) {
    uint64_t sr = (state << (64 - c->K)) | ((uint64_t)input << 63);
    int e = 0;
    for (int k = 0; k < c->n; ++k) e = (e << 1) | cco_gen_bit(sr & c->poly[k], c->gen_mode);
    *new_state = sr >> (64 + 1 - c->K);
    return e;
}

#define CCO_STACK_DEPTH 64   /* stack-decoder.c:12 */

typedef struct {
    uint16_t next;        /* next_input_index: floats (AWGN) or symbols (BSC, uint8 there) */
    uint64_t state;
    float fmetric;
    int32_t imetric;
    uint8_t path[40];
} cco_path;

/* One block with the reference's data structure and streaming loop (stack-decoder.c:105-115 reset,
 * :132-197 receive_symbol, :199-241 most/least probable and duplicate). The loop is the streaming
 * one: after step t arrives, extend the most probable path until it ends exactly at the received
 * frontier. This matters when the stack is full of equal metrics (idiom codes emit the same symbol
 * for both inputs, so twin paths accumulate): then the most and least probable path are the same
 * entry, duplicate_path copies it onto itself and the two extensions land on one path, which skips a
 * symbol and runs ahead of the frontier, reading whatever the input buffer holds there -- the
 * previous block's symbols (`buf` persists across blocks like the reference's input_symbols, zeroed
 * at creation). Returns -1 if the reference would read past its input buffer (not reproducible). */
static int stack_block(const cco_code* c, int soft, float weight, const int32_t* bm,
                       const float* rx, const uint8_t* syms, float* fbuf, uint8_t* hbuf,
                       uint8_t* out, int32_t* pm) {
    const size_t T = cco_steps(c), OB = cco_out_bytes(c);
    const unsigned NS = soft ? (1u << c->n) : 1u;
    const uint8_t mask = (uint8_t)((1u << c->n) - 1u);
    static cco_path st[CCO_STACK_DEPTH];
    unsigned size = 1, cur = 0;
    int status = 0;
    memset(st, 0, sizeof st);
    for (size_t t = 1; t <= T; ++t) {
        if (soft) memcpy(fbuf + (t - 1) * NS, rx + (t - 1) * NS, NS * sizeof(float));
        else hbuf[t - 1] = syms[t - 1] & mask;
        const uint16_t W = soft ? (uint16_t)(t * NS) : (uint16_t)(uint8_t)t;
        for (;;) {
            /* get_most_probable_path: strict >, first index wins */
            cur = size;
            float fmax = -INFINITY;
            int32_t imax = (int32_t)0x80000000;
            for (unsigned i = 0; i < size; ++i)
                if (soft ? (st[i].fmetric > fmax) : (st[i].imetric > imax)) {
                    fmax = st[i].fmetric; imax = st[i].imetric; cur = i;
                }
            if (cur == size) return -1;   /* no finite metric: the reference reads past its stack */
            if (st[cur].next == W) break;
            const unsigned idx = st[cur].next;
            if (idx + NS > T * NS) return -1;   /* past the input buffer */
            uint64_t ns[2];
            float ftm[2] = {0, 0};
            int32_t itm[2] = {0, 0};
            for (int in = 0; in < 2; ++in) {
                int e = stack_symbol(c, st[cur].state, in, &ns[in]);
                if (soft) {
                    ftm[in] = (float)(1.0 + (double)(weight * fbuf[idx + (unsigned)e]));
                } else {
                    int32_t d = __builtin_popcount((unsigned)(e ^ hbuf[idx]));
                    itm[in] = d * bm[1] + (c->n - d) * bm[0];
                }
            }
            /* duplicate_path */
            unsigned lhs;
            if (size == CCO_STACK_DEPTH) {
                lhs = size;
                float fmin = INFINITY;
                int32_t imin = 0x7FFFFFFF;
                for (unsigned i = 0; i < size; ++i)
                    if (soft ? (st[i].fmetric < fmin) : (st[i].imetric < imin)) {
                        fmin = st[i].fmetric; imin = st[i].imetric; lhs = i;
                    }
                if (lhs == size) return -1;
            } else {
                lhs = size++;
            }
            if (lhs != cur) st[lhs] = st[cur];
            for (int in = 0; in < 2; ++in) {
                cco_path* p = &st[in ? lhs : cur];
                unsigned w = (uint8_t)(p->next / NS);
                p->next = (uint16_t)(p->next + NS);
                if (!soft) p->next &= 0xFF;
                p->state = ns[in];
                if (soft) p->fmetric += ftm[in];
                else p->imetric += itm[in];
                if (w / 8 < sizeof p->path) p->path[w / 8] |= (uint8_t)(in << (7 - w % 8));
            }
        }
    }
    memcpy(out, st[cur].path, OB);
    if (pm) *pm = st[cur].imetric;
    return status;
}

int cco_stack_soft(const cco_code* c, float metric_weight, const float* rx, size_t nblocks,
                   uint8_t* out) {
    size_t T = cco_steps(c), NS = (size_t)1 << c->n, OB = cco_out_bytes(c);
    float* buf = (float*)calloc(T * NS, sizeof(float));
    int rc = 0;
    for (size_t b = 0; b < nblocks; ++b)
        if (stack_block(c, 1, metric_weight, NULL, rx + b * T * NS, NULL, buf, NULL, out + b * OB, NULL))
            rc = -1;
    free(buf);
    return rc;
}

int cco_stack_hard(const cco_code* c, const int32_t* bit_metrics, const uint8_t* syms, size_t nblocks,
                   uint8_t* out, int32_t* path_metric) {
    size_t T = cco_steps(c), OB = cco_out_bytes(c);
    uint8_t* buf = (uint8_t*)calloc(T, 1);
    int rc = 0;
    for (size_t b = 0; b < nblocks; ++b)
        if (stack_block(c, 0, 0.0f, bit_metrics, NULL, syms + b * T, NULL, buf, out + b * OB,
                        path_metric ? path_metric + b : NULL))
            rc = -1;
    free(buf);
    return rc;
}

/* ---------------------------------------------------------------- Fano decoders */

#define CCO_FANO_TIMEOUT 10000   /* fano-decoder.c:14, cycles per decoded bit */

typedef struct {
    uint64_t state;
    float fmetric;
    int32_t imetric;
    uint8_t sel;                 /* selected_path */
    float ftm[2];
    int32_t itm[2];
    uint64_t succ[2];
    uint8_t decoded;             /* decoded_input */
} cco_fano_node;

/* get_transition_metric (AWGN-channel/fano-decoder.c:282-313 / BSC :284-320) and the sort that
 * follows it (:169-181 / :224-236): best transition first, decoded_input = 1 if input 1 is best. */
static void fano_node_metrics(const cco_code* c, int soft, float fw, const int32_t* fbm, const float* r,
                              uint8_t rsym, cco_fano_node* nd) {
    for (int in = 0; in < 2; ++in) {
        int e = stack_symbol(c, nd->state, in, &nd->succ[in]);
        if (soft) {
            nd->ftm[in] = (float)(1.0 + (double)(fw * r[e]));
        } else {
            int32_t d = __builtin_popcount((unsigned)(e ^ rsym));
            nd->itm[in] = d * fbm[1] + (c->n - d) * fbm[0];
        }
    }
    if (soft ? (nd->ftm[0] < nd->ftm[1]) : (nd->itm[0] < nd->itm[1])) {
        uint64_t st = nd->succ[0]; nd->succ[0] = nd->succ[1]; nd->succ[1] = st;
        float ft = nd->ftm[0]; nd->ftm[0] = nd->ftm[1]; nd->ftm[1] = ft;
        int32_t it = nd->itm[0]; nd->itm[0] = nd->itm[1]; nd->itm[1] = it;
        nd->decoded = 1;
    }
}

/* One block of the Fano search (fano-decoder.c:108-124 reset, :140-273 receive_symbol, :315-325
 * output), written for a fully received block: the streaming loop returns whenever the search first
 * reaches the newest node and resumes there when its symbol arrives, where it computes exactly what
 * the forward move would (the node is fresh), so the operation sequence and the per-block timeout
 * count are the same. BSC path metric: the metric of the newest received node when the search ends
 * (:195, :269). */
static void fano_block(const cco_code* c, int soft, float fw, const int32_t* fbm, const float* rx,
                       const uint8_t* syms, cco_fano_node* nodes, uint8_t* out, int32_t* pm) {
    const size_t T = cco_steps(c), OB = cco_out_bytes(c), NS = (size_t)1 << c->n;
    const uint8_t mask = (uint8_t)((1u << c->n) - 1u);
    const float fdelta = 17.0f;
    const int32_t idelta = 17;
    memset(nodes, 0, T * sizeof *nodes);
    float fthr = 0.0f;
    int32_t ithr = 0;
    uint32_t timeout = CCO_FANO_TIMEOUT * (uint32_t)T;
    size_t cur = 0, frontier = 0;
#define RX(i) (soft ? rx + (i) * NS : NULL)
#define SY(i) (soft ? 0 : (uint8_t)(syms[i] & mask))
    fano_node_metrics(c, soft, fw, fbm, RX(0), SY(0), &nodes[0]);
    int done = 0;
    while (timeout != 0) {
        timeout--;
        cco_fano_node* cn = &nodes[cur];
        float fms = cn->fmetric + cn->ftm[cn->sel];
        int32_t ims = cn->imetric + cn->itm[cn->sel];
        if (soft ? (fms >= fthr) : (ims >= ithr)) {
            if (soft) {   /* tightening (:190-195) */
                if (cn->fmetric < (fthr + fdelta))
                    while (fms >= fthr + fdelta) fthr += fdelta;
            } else {
                if (cn->imetric < (ithr + idelta))
                    while (ims >= ithr + idelta) ithr += idelta;
            }
            ++cur;
            if (cur == T) { done = 1; break; }
            cco_fano_node* nn = &nodes[cur];
            nn->state = cn->succ[cn->sel];
            nn->fmetric = fms;
            nn->imetric = ims;
            nn->decoded = 0;
            nn->sel = 0;
            fano_node_metrics(c, soft, fw, fbm, RX(cur), SY(cur), nn);
            if (cur > frontier) frontier = cur;
        } else {
            for (;;) {
                int cant = cur == 0;
                if (!cant) {
                    cco_fano_node* pn = &nodes[cur - 1];
                    cant = soft ? (pn->fmetric < fthr) : (pn->imetric < ithr);
                }
                if (cant) {   /* relax the threshold, restart from the best branch (:241-250) */
                    if (soft) fthr -= fdelta; else ithr -= idelta;
                    if (nodes[cur].sel != 0) {
                        nodes[cur].sel = 0;
                        nodes[cur].decoded ^= 1;
                    }
                    break;
                }
                --cur;   /* move back (:251-261) */
                if (nodes[cur].sel == 0) {
                    nodes[cur].sel = 1;
                    nodes[cur].decoded ^= 1;
                    break;
                }
            }
        }
    }
#undef RX
#undef SY
    if (pm) *pm = done ? nodes[T - 1].imetric : nodes[frontier].imetric;
    memset(out, 0, OB);
    for (size_t i = 0; i < T; ++i)
        if (nodes[i].decoded == 1) out[i / 8] |= (uint8_t)(1u << (7 - i % 8));
}

void cco_fano_soft(const cco_code* c, float fano_metric_weight, const float* rx, size_t nblocks,
                   uint8_t* out) {
    size_t T = cco_steps(c), NS = (size_t)1 << c->n, OB = cco_out_bytes(c);
    cco_fano_node* nodes = (cco_fano_node*)calloc(T, sizeof *nodes);
    for (size_t b = 0; b < nblocks; ++b)
        fano_block(c, 1, fano_metric_weight, NULL, rx + b * T * NS, NULL, nodes, out + b * OB, NULL);
    free(nodes);
}

void cco_fano_hard(const cco_code* c, const int32_t* fano_bit_metrics, const uint8_t* syms,
                   size_t nblocks, uint8_t* out, int32_t* path_metric) {
    size_t T = cco_steps(c), OB = cco_out_bytes(c);
    cco_fano_node* nodes = (cco_fano_node*)calloc(T, sizeof *nodes);
    for (size_t b = 0; b < nblocks; ++b)
        fano_block(c, 0, 0.0f, fano_bit_metrics, NULL, syms + b * T, nodes, out + b * OB,
                   path_metric ? path_metric + b : NULL);
    free(nodes);
}

/* AWGN-channel/main.c:129-141: compare the first blen bits, MSB-first. */
uint64_t cco_count_errors(const cco_code* c, const uint8_t* info, const uint8_t* out, size_t nblocks) {
    size_t IB = cco_info_bytes(c), OB = cco_out_bytes(c);
    uint64_t errors = 0;
    for (size_t b = 0; b < nblocks; ++b)
        for (int i = 0; i < c->blen; ++i) {
            int a = (info[b * IB + i / 8] >> (7 - i % 8)) & 1;
            int d = (out[b * OB + i / 8] >> (7 - i % 8)) & 1;
            errors += (uint64_t)(a != d);
        }
    return errors;
}
