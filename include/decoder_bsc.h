/*
 * decoder_bsc.h -- hard-decision (binary symmetric channel) Viterbi decoder, libccv_bsc.so.
 *
 * Drop-in for the reference's binary-symmetric-channel/include/decoder.h:9-26: same six symbols,
 * same callback type (with the path metric), same argument meaning, ownership and error behaviour;
 * the trellis work runs on the MI355X (libccv_core.so, include/ccv.h). Link either this library or
 * libccv_awgn.so, never both (the reference's symbol names collide by design).
 */
#pragma once

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* binary-symmetric-channel/include/decoder.h:9. path_metric = Hamming distance of the survivor
 * (viterbi-decoder.c:95). Return 0 to take ownership of `data`. */
typedef int (*callback_t)(uint8_t* data, uint8_t len, int32_t path_metric, void* userdata);

struct code_param;
struct decoder;

struct decoder* decoder_create(void);
void decoder_destroy(struct decoder** obj);

int decoder_init(struct decoder* obj, struct code_param* param);
void decoder_register_callback(struct decoder* obj, callback_t output_callback);
void decoder_reset(struct decoder* obj);

/* binary-symmetric-channel/include/decoder.h:26. len counts received symbols (one per trellis
 * step, low n bits used: viterbi-decoder.c:235-237). */
int decoder_input(struct decoder* obj, uint8_t* data, uint8_t len);

/* ---- batch extension (new; not in the reference) ---------------------------------------------- */
int decoder_set_generator_mode(struct decoder* obj, int mode);
int decoder_input_blocks(struct decoder* obj, const uint8_t* data, size_t n_blocks);
/* path_metrics may be NULL */
int decoder_decode_blocks(struct decoder* obj, const uint8_t* data, size_t n_blocks, uint8_t* out,
                          int32_t* path_metrics);
int decoder_decode_device(struct decoder* obj, const uint8_t* d_data, size_t n_blocks,
                          uint8_t* d_out, int32_t* d_path_metrics, void* stream);
const char* decoder_last_error(void);

#ifdef __cplusplus
}
#endif
