/*
 * ccoracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference (thomas-emig/convolutional-codes) Viterbi hot path and of the
 * CPU-side producers that feed it. It exists to CHECK the MI355X decoder: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The product path
 * (convolutional-codes_amd/) never links or calls it.
 *
 * Parity status: PINNED. tests/test_oracle.py checks every function here against golden vectors
 * produced by the unmodified reference sources (oracle/ref_harness.c compiled against
 * /root/reference by oracle/Makefile, fixtures in tests/golden/, generator tests/golden/make_golden.py).
 */
#ifndef CCORACLE_H
#define CCORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Generator-bit semantics.  The reference computes the parity of (shift_register & poly) with
 * `(0x6996 >> val) & 1` on an unreduced 64-bit `val` (AWGN-channel/viterbi-decoder.c:53-57,
 * binary-symmetric-channel/viterbi-decoder.c:53-57, common/encoder.c:95-100).  On x86-64 the shift
 * count is masked to 5 bits, which makes the effective bit parity(v) & !parity(v & 0x1010..10).
 * CCO_GEN_REF_X86 restates that; CCO_GEN_TRUE_PARITY is the textbook generator. */
enum { CCO_GEN_REF_X86 = 0, CCO_GEN_TRUE_PARITY = 1 };

typedef struct {
    int n;              /* symlen_out: output bits per trellis step   (code.h:10) */
    int K;              /* constr_len                                  (code.h:11) */
    int blen;           /* block_len: info bits per block              (code.h:12) */
    uint64_t poly[8];   /* MSB-aligned generator polynomials           (code.h:13) */
    int gen_mode;       /* CCO_GEN_*                                               */
} cco_code;

/* glibc random()/rand() TYPE_3 additive-feedback generator + gaussian.c's Box-Muller cache. */
typedef struct {
    uint32_t s[31];     /* additive-feedback table */
    int f, r;           /* front / rear taps, 3 apart */
    double R, T;        /* gaussian.c:14-16 statics */
    int phase;
} cco_rng;

void     cco_srand(cco_rng* g, uint32_t seed);
int32_t  cco_rand(cco_rng* g);
double   cco_gengauss(cco_rng* g);

int      cco_gen_bit(uint64_t v, int gen_mode);
int      cco_expected_symbol(const cco_code* c, uint32_t state, int input);
void     cco_trellis(const cco_code* c, uint8_t* exp_sym /* [S][2] */);

size_t   cco_steps(const cco_code* c);          /* T = blen + K - 1 */
size_t   cco_info_bytes(const cco_code* c);     /* ceil(blen/8) */
size_t   cco_out_bytes(const cco_code* c);      /* ceil(T/8) */

void     cco_encode_block(const cco_code* c, const uint8_t* info, uint8_t* syms /* [T] */);
void     cco_constellation(int n, float* pts /* [2 * 2^n] */);
void     cco_demap(int n, float x, float y, float* out /* [2^n] */);
void     cco_demap_hard(int n, float x, float y, float* out /* [2^n] */);

/* Driver-order channels (AWGN-channel/main.c:80-116,212-229; binary-symmetric-channel/main.c:57-72,
 * 159-172) starting from srand(seed). */
void     cco_awgn_blocks(const cco_code* c, uint32_t seed, float scaling, size_t nblocks,
                         uint8_t* info /* [nb][IB] */, float* rx /* [nb][T][2^n] */);
void     cco_awgn_blocks_demap(const cco_code* c, uint32_t seed, float scaling, size_t nblocks, int hard,
                               uint8_t* info, float* rx);   /* hard: common/hard-demapper.c */
void     cco_bsc_blocks(const cco_code* c, uint32_t seed, int32_t p_ppm, size_t nblocks,
                        uint8_t* info /* [nb][IB] */, uint8_t* syms /* [nb][T] */);

/* Viterbi decoders with the reference's loop shape and tie rules; loop counters widened so K=9 runs. */
void     cco_viterbi_soft(const cco_code* c, const float* rx, size_t nblocks, uint8_t* out /* [nb][OB] */);
void     cco_viterbi_hard(const cco_code* c, const uint8_t* syms, size_t nblocks, uint8_t* out,
                          int32_t* path_metric /* [nb] */);

/* Stack (sequential) decoders, AWGN-channel/stack-decoder.c and binary-symmetric-channel/
 * stack-decoder.c: 64-entry path stack, extend the most probable path until it spans the block.
 * Soft branch metric (float)(1.0 + weight * d[sym]); hard: d * bit_metrics[1] + (n - d) *
 * bit_metrics[0] with d the Hamming distance. Blocks run through one decoder in order (a path that
 * overtakes the received frontier reads the previous block's symbols, as in the reference). Returns
 * -1 if some block made the reference read past its buffers. Requires T <= 255 and K <= 64. */
int      cco_stack_soft(const cco_code* c, float metric_weight, const float* rx, size_t nblocks,
                        uint8_t* out /* [nb][OB] */);
int      cco_stack_hard(const cco_code* c, const int32_t* bit_metrics /* [2] */, const uint8_t* syms,
                        size_t nblocks, uint8_t* out, int32_t* path_metric /* [nb] */);

/* Fano decoders, AWGN-channel/fano-decoder.c and binary-symmetric-channel/fano-decoder.c (KA9Q-
 * derived threshold search, DELTA 17, timeout 10000 iterations per block bit). Soft branch metric
 * (float)(1.0 + fano_metric_weight * d[sym]); hard: d * fano_bit_metrics[1] + (n - d) *
 * fano_bit_metrics[0]. path_metric: the BSC decoder's callback metric. */
void     cco_fano_soft(const cco_code* c, float fano_metric_weight, const float* rx, size_t nblocks,
                       uint8_t* out);
void     cco_fano_hard(const cco_code* c, const int32_t* fano_bit_metrics /* [2] */, const uint8_t* syms,
                       size_t nblocks, uint8_t* out, int32_t* path_metric);

/* Consumer: bit errors over the first blen bits of each block (AWGN-channel/main.c:118-144). */
uint64_t cco_count_errors(const cco_code* c, const uint8_t* info, const uint8_t* out, size_t nblocks);

#ifdef __cplusplus
}
#endif
#endif
