/*
 * ccv.h -- C ABI of the MI355X (gfx950) Viterbi decoder core, libccv_core.so.
 *
 * This is the batched, device-level API underneath the reference-compatible decoder_* shims
 * (include/decoder_awgn.h, include/decoder_bsc.h). It replaces, for whole batches of independent
 * zero-tail-terminated trellis blocks, the per-step work the reference does in
 *   receive_symbol()/get_transition_metric()  AWGN-channel/viterbi-decoder.c:38-69,108-141
 *                                             binary-symmetric-channel/viterbi-decoder.c:38-73,114-150
 *   traceback()                               AWGN-channel/viterbi-decoder.c:71-90
 *                                             binary-symmetric-channel/viterbi-decoder.c:75-96
 * and the bit-error count of the drivers' decoded callbacks (AWGN-channel/main.c:118-144,
 * binary-symmetric-channel/main.c:74-98).
 *
 * Data layouts (identical to what the reference decoder consumes and emits, block after block):
 *   soft input  float   [nblocks][T][2^n]   demapper output per trellis step (common/demapper.c:66-70)
 *   hard input  uint8_t [nblocks][T]        received symbol per step, low n bits used
 *   output      uint8_t [nblocks][OB]       MSB-first decoded bits, OB = ceil(T/8), tail bits included
 *   info        uint8_t [nblocks][IB]       transmitted info bits (optional), IB = ceil(blen/8)
 * with T = blen + K - 1.  All functions return 0 on success and -1 on failure (ccv_last_error()).
 * Not thread-safe per plan: use one plan per thread (as the reference decoder handle). A plan owns
 * device scratch (decision arrays, the Fano work counter) that every decode reuses, so the decodes of
 * one plan must also be serialised on ONE stream; decodes on several streams need one plan each.
 * After ccv_plan_reserve(max_blocks), ccv_decode_device of up to max_blocks blocks allocates and
 * synchronises nothing (ccv_simulate_device: after one call of at least as many blocks), so either can
 * be captured into a HIP graph and replayed -- the persistent kernels' group queue resets itself at
 * the end of every launch (tests/test_gpu_graph.py).
 */
#ifndef CCV_H
#define CCV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CCV_SOFT 0            /* AWGN soft decision: float branch metrics per expected symbol   */
#define CCV_HARD 1            /* BSC hard decision: Hamming branch metric, uint16-saturating    */

#define CCV_GEN_REF_X86 0     /* generator bit as the reference computes it on x86 (default)    */
#define CCV_GEN_TRUE_PARITY 1 /* textbook parity generator                                      */

#define CCV_FLAG_GENERIC 1u   /* force the table-driven kernel even if a specialised one exists */
#define CCV_FLAG_STEP_MAJOR 2u /* soft input is step-major float [T][nblocks][2^n] (coalesced;
                                  register-trellis codes only; ccv_decode_device only)            */
#define CCV_FLAG_GLOBAL_DECISIONS 4u /* keep survivor decisions in an HBM scratch array even where the
                                  register-resident-decision kernel applies (A/B measurements)    */
#define CCV_FLAG_NO_PERSISTENT 8u /* do not use the persistent K <= 7 kernels (A/B measurements)    */

#define CCV_KERNEL_REGISTER 1 /* code-specialised register-trellis kernel                       */
#define CCV_KERNEL_GENERIC 2  /* table-driven LDS kernel                                        */
#define CCV_KERNEL_MULTILANE 3 /* K = 8, 9: register-trellis kernel, 2^(K-7) lanes per block      */
#define CCV_KERNEL_STACK 4    /* stack (sequential) decoder, one wave per block                  */
#define CCV_KERNEL_FANO 5     /* Fano decoder, one persistent lane per block                     */

typedef struct ccv_plan ccv_plan;

typedef struct {
    int channel, n, K, blen, gen_mode;
    int steps;           /* T  */
    int states;          /* S = 2^(K-1) */
    int info_bytes;      /* IB */
    int out_bytes;       /* OB */
    int in_step_bytes;   /* 4 * 2^n (soft) or 1 (hard) */
    int kernel;          /* CCV_KERNEL_* */
    int decision_word_bytes; /* register kernels: bytes of one decision word */
    int device;
    int lanes;           /* wave lanes (decision words per step) per block: 1, or 2^(K-7) multilane */
} ccv_plan_desc;

/* A plan binds a code to the device that is current on the calling thread.
 * n in [1,8], K in [2,12], blen in [1,255]; polys[0..n-1] MSB-aligned (code.h:13). */
int ccv_plan_create(ccv_plan** plan, int channel, int n, int K, int blen, const uint64_t* polys,
                    int gen_mode, unsigned flags);
void ccv_plan_destroy(ccv_plan* plan);
int ccv_plan_describe(const ccv_plan* plan, ccv_plan_desc* desc);

/* Expected-symbol table of the plan's trellis: exp[2*s + i], S*2 bytes. */
int ccv_plan_trellis(const ccv_plan* plan, uint8_t* exp);

/* Where a ccv_decode_device call without decision export keeps the survivor decisions:
 * CCV_DECISIONS_NONE (stack / Fano decoders: no trellis), CCV_DECISIONS_HBM (scratch array in device
 * memory, read back by the traceback), CCV_DECISIONS_REGISTERS (VGPR-resident for the whole block:
 * the persistent K <= 7 kernels at blen 40, soft r = 1/2 codes with K <= 7 and blen + K - 1 <= 48,
 * K = 8, 9 with short blocks), CCV_DECISIONS_LDS (the generic kernel keeps a block's decisions in
 * LDS) or CCV_DECISIONS_SLOT (the K = 9 one-lane-per-block kernel: a scratch slot per resident wave,
 * rewritten by every group the wave decodes, so it stays in the L2 / Infinity Cache working set). */
#define CCV_DECISIONS_NONE 0
#define CCV_DECISIONS_HBM 1
#define CCV_DECISIONS_REGISTERS 2
#define CCV_DECISIONS_LDS 3
#define CCV_DECISIONS_SLOT 4
int ccv_plan_decision_storage(const ccv_plan* plan);

/* Name of the kernel a ccv_decode_device call without decision export runs: "persistent",
 * "persistent-wide" (K = 9, one lane per block), "persistent-slot2" (K = 9 true parity, two lanes
 * per block), "register-regdec", "register", "multilane-regdec", "multilane",
 * "generic", "stack" or "fano". */
const char* ccv_plan_kernel_variant(const ccv_plan* plan);

/* Grid (resident waves = occupancy x CUs, whole SIMDs) of the plan's persistent kernel: the value
 * cached per (kernel, device) that its launches use, or with fresh != 0 a new occupancy query that
 * bypasses the cache. 0 when the plan runs no persistent kernel, -1 on error. */
int ccv_plan_persistent_waves(const ccv_plan* plan, int fresh);

/* Grow the plan's device scratch so decodes of up to max_blocks blocks allocate nothing. */
int ccv_plan_reserve(ccv_plan* plan, size_t max_blocks);

/* Asynchronous decode of nblocks device-resident blocks on `stream` (a hipStream_t; NULL = the
 * legacy default stream).  d_path_metric (hard only), d_info + d_errors (error counting: adds the
 * batch's bit errors over the first blen bits to *d_errors) and d_decisions (register kernel only:
 * [T][P] words of ccv_plan_desc.decision_word_bytes, P = nblocks rounded up to a multiple of 64,
 * block b in column b; bit s set = the survivor into state s came from the odd predecessor; not
 * available for the multilane kernel, whose words are in its physical state order) may be NULL. */
int ccv_decode_device(ccv_plan* plan, const void* d_in, size_t nblocks, uint8_t* d_out,
                      int32_t* d_path_metric, const uint8_t* d_info, unsigned long long* d_errors,
                      void* d_decisions, void* stream);

/* On-device channel fused with the decode (register-trellis and multilane
 * codes): blocks first_block .. first_block + nblocks - 1 of the Philox stream `seed` are generated in
 * registers -- info bytes, encoder (common/encoder.c:84-119), then per step QPSK/8-PSK mapping, AWGN
 * with noise scaling `channel_param` and the demapper (AWGN-channel/main.c:93-106, demapper.c:61-70)
 * for a soft plan, or bit flips with probability channel_param ppm (binary-symmetric-channel/
 * main.c:57-72) for a hard plan -- in the draw order of ccv_sim_awgn / ccv_sim_bsc(CCV_RNG_PHILOX),
 * decoded, and the bit errors over the first blen bits of each block added to *d_errors.
 * d_info ([nb][IB] transmitted bytes), d_out ([nb][OB] decoded bytes), d_path_metric (hard),
 * d_errors and d_channel (export of the decoder input: float [nb][T][2^n] or uint8 [nb][T]) may be
 * NULL; info and output then go to plan-owned scratch. Info bits and BSC symbols are bit-identical
 * to ccv_sim_*; AWGN samples use the device's double log/sin/cos. AWGN scalings must lie in
 * [0, 2^28) (Eb/N0 above -160 dB), else -1. Asynchronous on `stream`. K = 8 / 9 plans -- soft at
 * blen 40 and every BSC one -- run as two kernels instead: the frames into d_channel (or plan
 * scratch), then the decode (the persistent kernels for soft, and for BSC through Hamming-distance
 * rows; same draws, same results); ccv_plan_set_option(plan, "channel_fused", 1) keeps the fused
 * kernel, and step-major plans always use it. */
#define CCV_CHANNEL_HARD_DEMAP 1u   /* AWGN: common/hard-demapper.c instead of common/demapper.c */
/* Frames only, no decode: info bytes into d_info (or plan scratch) and the decoder input into d_channel
 * (required), same draws as above, for ANY plan -- Viterbi, stack or Fano, n <= 3, K <= 64. d_out,
 * d_path_metric and d_errors are ignored. The frames are block-major ([nb][T][2^n] / [nb][T]): a
 * CCV_FLAG_STEP_MAJOR plan is rejected (-1). The device sweeps of the sequential decoders use it. */
#define CCV_CHANNEL_FRAMES_ONLY 2u
/* AWGN, opt-in: the Box-Muller in fp32 from the hardware log2 / sqrt / sin / cos (same uniforms and
 * draw order) instead of double precision. Faster; the samples are NOT bit-identical to the double
 * path or glibc (a few fp32 ulp, tools/chanmath_f32_check.hip), so only the BER statistics match. */
#define CCV_CHANNEL_NOISE_F32 4u
/* Frames only, AWGN (round 6): d_channel gets the demapper's INPUT -- the received point (x, y), float
 * [nb][T][2], after the hard demapper's snap with CCV_CHANNEL_HARD_DEMAP -- instead of its 2^n
 * distances. A Fano plan with option "fano_input" 1 decodes such frames, recomputing the distances with
 * the demapper's exact fp32 operations (common/demapper.c:66-70): the same decoder input bit for bit,
 * in half the bytes per node (n = 2). */
#define CCV_CHANNEL_IQ 8u
int ccv_simulate_device(ccv_plan* plan, uint64_t seed, uint64_t first_block, size_t nblocks,
                        double channel_param, unsigned channel_flags, uint8_t* d_info, uint8_t* d_out,
                        int32_t* d_path_metric, unsigned long long* d_errors, void* d_channel,
                        void* stream);

/* Stack (sequential) decoder plan (AWGN-channel/stack-decoder.c, binary-symmetric-channel/
 * stack-decoder.c): 64-entry path stack, K <= 64. metric_weight = code_param.metric_weight (soft),
 * bit_metrics = code_param.bit_metrics[2] (hard; code.h:14-16). ccv_decode_device / ccv_decode_host
 * accept the plan (a batch is decoded as if its blocks went through one fresh decoder in order). */
int ccv_stack_plan_create(ccv_plan** plan, int channel, int n, int K, int blen, const uint64_t* polys,
                          int gen_mode, float metric_weight, const int32_t* bit_metrics);

/* Stack decode with the streaming context made explicit: d_prev = the block the same decoder
 * received before block 0 (its input buffer still holds it; NULL = a fresh, zeroed decoder); blocks
 * b > 0 follow block b-1. d_status[nb] (optional): 1 where the reference would have read past its
 * buffers (a degenerate search; the output of that block is then not the reference's). For K <= 32,
 * n in {2, 3} and T <= 64 the call resets the plan's block counter on `stream` and, on the plan's
 * first such call with K <= 16, builds its expected-symbol table there, before the decode kernel. */
int ccv_stack_decode_device(ccv_plan* plan, const void* d_in, size_t nblocks, const void* d_prev,
                            uint8_t* d_out, int32_t* d_path_metric, const uint8_t* d_info,
                            unsigned long long* d_errors, int32_t* d_status, void* stream);

/* Fano decoder plan (AWGN-channel/fano-decoder.c, binary-symmetric-channel/fano-decoder.c): threshold
 * search with DELTA 17 and a timeout of 10000 iterations per block bit, K <= 64, T <= 255.
 * fano_metric_weight = code_param.fano_metric_weight (soft), fano_bit_metrics = code_param.
 * fano_bit_metrics[2] (hard; code.h:15-17). ccv_decode_device / ccv_decode_host accept the plan
 * (hard: d_path_metric = the reference callback's path metric). */
int ccv_fano_plan_create(ccv_plan** plan, int channel, int n, int K, int blen, const uint64_t* polys,
                         int gen_mode, float fano_metric_weight, const int32_t* fano_bit_metrics);

/* Fano decode with the per-block search length exported: d_iterations[nb] (optional) = iterations
 * used; 10000 * T means the block hit the reference's timeout. Soft input with n in {2, 3} and more
 * than 64 blocks first scores and sorts the blocks (noisiest first) on `stream`, into plan scratch;
 * outputs are per block index whatever the order. */
int ccv_fano_decode_device(ccv_plan* plan, const void* d_in, size_t nblocks, uint8_t* d_out,
                           int32_t* d_path_metric, const uint8_t* d_info, unsigned long long* d_errors,
                           uint32_t* d_iterations, void* stream);

/* Host-buffer form of ccv_stack_decode_device (prev, path_metric, status may be NULL). */
int ccv_stack_decode_host(ccv_plan* plan, const void* in, size_t nblocks, const void* prev,
                          uint8_t* out, int32_t* path_metric, int32_t* status);

/* Synchronous convenience: host buffers in and out (staged through plan-owned device buffers).
 * Batches of <= 4 blocks (the streaming decoder_input path) go to a resident service kernel of the
 * plan that polls a host mailbox and stays on the GPU for CCV_SERVICE_IDLE_MS (default 20 ms) after
 * the last request, holding one workgroup: a device-wide synchronise in the process waits for it
 * meanwhile. CCV_HOST_LATENCY=1 launches one kernel per call instead; ccv_plan_destroy stops it. */
int ccv_decode_host(ccv_plan* plan, const void* in, size_t nblocks, uint8_t* out,
                    int32_t* path_metric);

/* Per-plan kernel options: A/B switches for measurements and tests; the defaults are the measured-
 * best paths. Takes effect from the plan's next decode. Returns 0, or -1 for an unknown
 * name, a value out of range or an option of another decoder.
 *   stack plans:  "stack_kernel"     0 persistent rows (default), 1 one search per wave
 *                 "stack_row_lanes"  0 auto (16; 8 for hard input without keys), 8, 16
 *                 "stack_keys"       1 packed metric / index keys for hard input where they fit (default), 0
 *                 "stack_symtab"     1 expected-symbol table (default), 0 parities per iteration
 *   Fano plans:   "fano_rows"        -1 auto (default: 1 hard, 2 soft r = 1/2), 0 read after the move,
 *                                    1 LDS, 2 both candidates prefetched
 *                 "fano_symtab"      -1 auto (table for hard input), 0, 1
 *                 "fano_order"       1 noisiest blocks first for soft input (default), 0 natural order
 *                 "fano_cap"         -1 default (6000 x T moves soft, 1000 x T hard), 0 one pass, else moves
 *                                    before parking
 *                 "fano_count_moves" 1: d_iterations gets moves instead of timeout ticks (diagnostics)
 *                 "fano_input"       0 the demapper's distances (default: the reference decoder's input),
 *                                    1 received points float [nb][T][2] (CCV_CHANNEL_IQ frames; soft,
 *                                    n = 2, K <= 32); "fano_rows" 1 then keeps the points in LDS
 *   Viterbi plans (on-device channel):
 *                 "channel_fused"    1: K = 8 / 9 codes use the fused multilane channel kernel
 *                 "channel_lds_decisions"  -1 auto (LDS unless it costs occupancy), 0 HBM, 1 LDS (K <= 7) */
int ccv_plan_set_option(ccv_plan* plan, const char* name, long long value);

/* Achievable-HBM probe for the roofline (bench.py): one streaming pass over `bytes` (a multiple of
 * 16, 16-byte aligned buffers) with global_load_dwordx4 -- mode 0 copies src to dst
 * (global_store_dwordx4; read + write bytes move), mode 1 only reads src (sink: a 4-byte device
 * word the kernel never writes in practice, or NULL). Launched on `stream`; time it with events. */
int ccv_hbm_probe(int mode, void* dst, const void* src, size_t bytes, uint32_t* sink, void* stream);

/* Number of visible HIP devices (0 without a GPU; never fails). */
int ccv_device_count(void);

const char* ccv_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
