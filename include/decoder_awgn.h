/*
 * decoder_awgn.h -- soft-decision (AWGN) Viterbi decoder, libccv_awgn.so.
 *
 * Drop-in for the reference's AWGN-channel/include/decoder.h:9-26: same six symbols, same callback
 * type, same argument meaning, ownership and error behaviour; the trellis work runs on the MI355X
 * (libccv_core.so, include/ccv.h). The BSC variant (decoder_bsc.h / libccv_bsc.so) exports the same
 * symbol names with different signatures, so a program links exactly one of the two, as the
 * reference's CMakeLists.txt:21-23,41-45 links exactly one decoder per executable.
 */
#pragma once

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* AWGN-channel/include/decoder.h:9. Called once per decoded block, synchronously, from inside
 * decoder_input(); len = block_len in bits. Returning 0 hands ownership of `data` to the callee
 * (free() it); any other value lets the decoder reuse the buffer (viterbi-decoder.c:92-106). */
typedef int (*callback_t)(uint8_t* data, uint8_t len, void* userdata);

struct code_param;
struct decoder;

/* AWGN-channel/include/decoder.h:17-18 */
struct decoder* decoder_create(void);
void decoder_destroy(struct decoder** obj);

/* AWGN-channel/include/decoder.h:21-23. decoder_init binds the code to the current HIP device
 * and returns -1 if the code is unsupported (n > 8, K > 12) or no GPU is usable. */
int decoder_init(struct decoder* obj, struct code_param* param);
void decoder_register_callback(struct decoder* obj, callback_t output_callback);
void decoder_reset(struct decoder* obj);

/* AWGN-channel/include/decoder.h:26. len counts floats, a multiple of 2^n (else -1); each group of
 * 2^n floats is one trellis step's demapper output. Blocks end after block_len + K - 1 steps. */
int decoder_input(struct decoder* obj, float* data, uint8_t len);

/* ---- batch extension (new; not in the reference) ---------------------------------------------- */

/* Generator-bit semantics for the next decoder_init: 0 = as the reference computes it on x86
 * (default; overridable with environment CCV_GENERATOR_MODE=true_parity), 1 = true parity. */
int decoder_set_generator_mode(struct decoder* obj, int mode);

/* n_blocks whole blocks, float [n_blocks][T][2^n], decoded in one GPU pass; the callback then fires
 * once per block, in order, exactly as if the blocks had been streamed. The decoder must be at a
 * block boundary (-1 otherwise). */
int decoder_input_blocks(struct decoder* obj, const float* data, size_t n_blocks);

/* Host in/out, no callbacks: out = uint8 [n_blocks][ceil(T/8)] (the reference output buffers). */
int decoder_decode_blocks(struct decoder* obj, const float* data, size_t n_blocks, uint8_t* out);

/* Device-resident in/out, asynchronous on `stream` (a hipStream_t, NULL = default stream). */
int decoder_decode_device(struct decoder* obj, const float* d_data, size_t n_blocks, uint8_t* d_out,
                          void* stream);

/* Description of the last failure on this thread. */
const char* decoder_last_error(void);

#ifdef __cplusplus
}
#endif
