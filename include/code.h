/*
 * code.h -- code parameters, ABI-identical to the reference's common/include/code.h:9-19 so that a
 * caller built against the reference passes the same struct to this library unchanged.
 */
#pragma once

#include <stdint.h>

struct code_param {
    uint8_t symlen_out;        /* n: output bits per trellis step                              */
    uint8_t constr_len;        /* K: constraint length                                         */
    uint8_t block_len;         /* info bits per zero-tail-terminated block                     */
    uint64_t* polynomials;     /* n MSB-aligned generators (tap 0 = bit 63); borrowed, not copied */
    int32_t* bit_metrics;      /* stack-decoder metrics (unused by the Viterbi decoder)        */
    int32_t* fano_bit_metrics; /* Fano-decoder metrics (unused by the Viterbi decoder)         */
    float metric_weight;       /* soft stack-decoder weight (unused by the Viterbi decoder)    */
    float fano_metric_weight;  /* soft Fano-decoder weight (unused by the Viterbi decoder)     */
    void* userdata;            /* handed back to the output callback                           */
};
