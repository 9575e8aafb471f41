/*
 * code1_table_probe.c -- CPU probe (test infrastructure, never shipped): variants of the reference hard
 * Viterbi (binary-symmetric-channel/viterbi-decoder.c:75-150, as restated in oracle/ccoracle.c
 * cco_viterbi_hard) to find which decoder produced the published code-1 BSC curve
 * (results/binary_symmetric_channel.m:7). tie = 0: strict < (reference), 1: <=;
 * zero = 0: traceback from the lowest-index argmin (reference :75-83), 1: from state 0 (the zero tail).
 * Returns the bit errors of the first blen bits of every block. Driven by tools/code1_table_probe.py.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "ccoracle.h"
/* variants of the reference hard Viterbi: tie = 0 strict <, 1 <=; zero = 0 argmin, 1 state 0 */
uint64_t var_hard(const cco_code* c, const uint8_t* syms, const uint8_t* info, size_t nblocks, int tie, int zero) {
    uint32_t S = 1u << (c->K - 1);
    size_t T = c->blen + c->K - 1;
    uint8_t mask = (uint8_t)((1u << c->n) - 1u);
    uint8_t exp_sym[2*512]; uint16_t M[512], N[512]; static uint16_t prev[512*300]; static uint8_t inp[512*300];
    cco_trellis(c, exp_sym);
    uint64_t errs = 0;
    for (size_t b = 0; b < nblocks; ++b) {
        for (uint32_t s = 0; s < S; ++s) M[s] = s ? 0xFF00 : 0;
        for (size_t t = 0; t < T; ++t) {
            uint8_t rs = syms[b * T + t] & mask;
            for (uint32_t s = 0; s < S; ++s) N[s] = 0xFF00;
            for (uint32_t s = 0; s < S; ++s) for (int i = 0; i < 2; ++i) {
                uint32_t ns = (s >> 1) | ((uint32_t)i << (c->K - 2));
                uint32_t m = (uint32_t)M[s] + (uint32_t)__builtin_popcount(exp_sym[2 * s + i] ^ rs);
                if (m > 0xFF00) m = 0xFF00;
                if (tie ? (m <= N[ns]) : (m < N[ns])) { N[ns] = m; prev[t * S + ns] = s; inp[t * S + ns] = i; }
            }
            memcpy(M, N, sizeof(uint16_t) * S);
        }
        uint32_t st = 0; uint16_t best = 0xFF00;
        if (!zero) for (uint32_t s = 0; s < S; ++s) if (M[s] < best) { best = M[s]; st = s; }
        uint8_t ob[64]; memset(ob, 0, sizeof ob);
        for (size_t t = T; t-- > 0;) { ob[t / 8] |= (uint8_t)(inp[t * S + st] << (7 - t % 8)); st = prev[t * S + st]; }
        size_t IB = (c->blen + 7) / 8;
        for (size_t k = 0; k < IB; ++k) {
            int valid = c->blen - 8 * (int)k; if (valid > 8) valid = 8;
            uint8_t m8 = (uint8_t)(0xFF << (8 - valid));
            errs += __builtin_popcount((ob[k] ^ info[b * IB + k]) & m8);
        }
    }
    return errs;
}
