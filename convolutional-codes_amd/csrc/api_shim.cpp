// api_shim.cpp -- reference-compatible decoder_* API over libccv_core.
//
// Compiled six times: -DCCV_SHIM_AWGN -> libccv_awgn.so (include/decoder_awgn.h) and
// -DCCV_SHIM_BSC -> libccv_bsc.so (include/decoder_bsc.h) replace the Viterbi decoders; with
// -DCCV_SHIM_STACK added -> libccv_stack_{awgn,bsc}.so replace the stack decoders
// (AWGN-channel/stack-decoder.c, binary-symmetric-channel/stack-decoder.c; same decoder.h); with
// -DCCV_SHIM_FANO -> libccv_fano_{awgn,bsc}.so replace the Fano decoders (fano-decoder.c). Life
// cycle and semantics follow AWGN-channel/viterbi-decoder.c:143-236 and
// binary-symmetric-channel/viterbi-decoder.c:152-243 (stack-decoder.c:45-197 alike): streaming
// input, a block completes after block_len + K - 1 steps, the output callback fires synchronously
// inside decoder_input(), a callback returning 0 takes ownership of the output buffer, and the
// decoder resets itself after every block. Each completed block is decoded on the GPU. The stack
// decoder's input buffer outlives a block (stack-decoder.c:105-115 does not clear it), so the
// previous block is passed along as its streaming context (ccv_stack_decode_host).
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "ccv.h"
#include "code.h"
#if defined(CCV_SHIM_AWGN)
#include "decoder_awgn.h"
typedef float in_t;
#define CCV_CHANNEL CCV_SOFT
#elif defined(CCV_SHIM_BSC)
#include "decoder_bsc.h"
typedef uint8_t in_t;
#define CCV_CHANNEL CCV_HARD
#else
#error "define CCV_SHIM_AWGN or CCV_SHIM_BSC"
#endif

#define CCV_EXPORT extern "C" __attribute__((visibility("default")))

struct decoder {
  code_param parameter{};
  ccv_plan* plan = nullptr;
  callback_t output_callback = nullptr;
  int gen_mode = CCV_GEN_REF_X86;
  size_t steps = 0;            // T
  size_t step_elems = 0;       // input elements per step: 2^n floats or 1 symbol
  size_t out_bytes = 0;        // ceil(T/8)
  size_t symbol_counter = 0;   // steps received of the current block
  std::vector<in_t> block;     // the current block's input
  uint8_t* output_data = nullptr;
  std::vector<uint8_t> batch_out;
  std::vector<int32_t> batch_pm;
  std::vector<in_t> prev;      // stack: the last completed block (the input buffer's contents)
  bool prev_valid = false;
};

namespace {

constexpr size_t kBatchChunk = 1u << 16;   // blocks per GPU pass in decoder_input_blocks

thread_local const char* g_shim_error = "";

int shim_fail(const char* msg) {
  g_shim_error = msg;
  return -1;
}

int default_gen_mode() {
  const char* env = std::getenv("CCV_GENERATOR_MODE");
  if (env && (std::strcmp(env, "true_parity") == 0 || std::strcmp(env, "1") == 0))
    return CCV_GEN_TRUE_PARITY;
  return CCV_GEN_REF_X86;
}

// viterbi-decoder.c:92-106 (AWGN) / :98-112 (BSC)
int emit_output_buffer(decoder* obj, int32_t path_metric) {
  int res = -1;
  if (obj->output_callback != nullptr) {
#if defined(CCV_SHIM_AWGN)
    (void)path_metric;
    res = obj->output_callback(obj->output_data, obj->parameter.block_len, obj->parameter.userdata);
#else
    res = obj->output_callback(obj->output_data, obj->parameter.block_len, path_metric,
                               obj->parameter.userdata);
#endif
  }
  if (res == 0) {
    obj->output_data = static_cast<uint8_t*>(std::malloc(obj->out_bytes));
    if (obj->output_data == nullptr) return shim_fail("out of memory");
  }
  return 0;
}

int decode_host(decoder* obj, const in_t* data, size_t n_blocks, uint8_t* out, int32_t* pm) {
  if (ccv_decode_host(obj->plan, data, n_blocks, out, pm) != 0) return shim_fail(ccv_last_error());
  return 0;
}

// Blocks arriving through the streaming API: the stack decoder continues from the previous block.
int decode_stream(decoder* obj, const in_t* data, size_t n_blocks, uint8_t* out, int32_t* pm) {
#if defined(CCV_SHIM_STACK)
  if (ccv_stack_decode_host(obj->plan, data, n_blocks, obj->prev_valid ? obj->prev.data() : nullptr,
                            out, pm, nullptr) != 0)
    return shim_fail(ccv_last_error());
  const size_t per_block = obj->steps * obj->step_elems;
  obj->prev.assign(data + (n_blocks - 1) * per_block, data + n_blocks * per_block);
  obj->prev_valid = true;
  return 0;
#else
  return decode_host(obj, data, n_blocks, out, pm);
#endif
}

}  // namespace

CCV_EXPORT struct decoder* decoder_create(void) {
  decoder* obj = new (std::nothrow) decoder();
  if (obj != nullptr) obj->gen_mode = default_gen_mode();
  return obj;
}

CCV_EXPORT void decoder_destroy(struct decoder** obj) {
  if (obj == nullptr || *obj == nullptr) return;
  ccv_plan_destroy((*obj)->plan);
  std::free((*obj)->output_data);
  delete *obj;
  *obj = nullptr;
}

CCV_EXPORT void decoder_reset(struct decoder* obj) {
  obj->symbol_counter = 0;
  if (obj->output_data) std::memset(obj->output_data, 0, obj->out_bytes);
}

CCV_EXPORT int decoder_init(struct decoder* obj, struct code_param* param) {
  if (obj == nullptr || param == nullptr || param->polynomials == nullptr)
    return shim_fail("null argument");
  obj->parameter = *param;   // by value; the polynomial array stays borrowed (reference :169)
  ccv_plan_destroy(obj->plan);
  obj->plan = nullptr;
#if defined(CCV_SHIM_FANO)
  if (CCV_CHANNEL == CCV_HARD && param->fano_bit_metrics == nullptr)
    return shim_fail("null fano_bit_metrics");
  if (ccv_fano_plan_create(&obj->plan, CCV_CHANNEL, param->symlen_out, param->constr_len,
                           param->block_len, param->polynomials, obj->gen_mode,
                           param->fano_metric_weight, param->fano_bit_metrics) != 0)
    return shim_fail(ccv_last_error());
#elif defined(CCV_SHIM_STACK)
  // stack-decoder.c:74-103 reallocates its input buffer: no streaming context survives init
  obj->prev_valid = false;
  if (CCV_CHANNEL == CCV_HARD && param->bit_metrics == nullptr) return shim_fail("null bit_metrics");
  if (ccv_stack_plan_create(&obj->plan, CCV_CHANNEL, param->symlen_out, param->constr_len,
                            param->block_len, param->polynomials, obj->gen_mode, param->metric_weight,
                            param->bit_metrics) != 0)
    return shim_fail(ccv_last_error());
#else
  if (ccv_plan_create(&obj->plan, CCV_CHANNEL, param->symlen_out, param->constr_len,
                      param->block_len, param->polynomials, obj->gen_mode, 0) != 0)
    return shim_fail(ccv_last_error());
#endif
  ccv_plan_desc d;
  ccv_plan_describe(obj->plan, &d);
  obj->steps = (size_t)d.steps;
  obj->step_elems = CCV_CHANNEL == CCV_SOFT ? (size_t)1 << d.n : 1;
  obj->out_bytes = (size_t)d.out_bytes;
  obj->block.assign(obj->steps * obj->step_elems, in_t());
  std::free(obj->output_data);
  obj->output_data = static_cast<uint8_t*>(std::malloc(obj->out_bytes));
  if (obj->output_data == nullptr) return shim_fail("out of memory");
  decoder_reset(obj);
  return 0;
}

CCV_EXPORT void decoder_register_callback(struct decoder* obj, callback_t output_callback) {
  obj->output_callback = output_callback;
}

// One trellis step arrived; decode when the block is complete (viterbi-decoder.c:132-139).
static int receive_step(decoder* obj, const in_t* step) {
  std::memcpy(&obj->block[obj->symbol_counter * obj->step_elems], step,
              obj->step_elems * sizeof(in_t));
  if (++obj->symbol_counter < obj->steps) return 0;
  int32_t pm = 0;
  if (decode_stream(obj, obj->block.data(), 1, obj->output_data,
                    CCV_CHANNEL == CCV_HARD ? &pm : nullptr) != 0)
    return -1;
  if (emit_output_buffer(obj, pm) != 0) return -1;
  decoder_reset(obj);
  return 0;
}

#if defined(CCV_SHIM_AWGN)
// AWGN-channel/viterbi-decoder.c:224-236: len counts floats and must be a multiple of 2^n.
CCV_EXPORT int decoder_input(struct decoder* obj, float* data, uint8_t len) {
  if (obj->plan == nullptr) return shim_fail("decoder not initialised");
  if (len % obj->step_elems != 0) return shim_fail("len is not a multiple of 2^n");
  for (size_t k = 0; k < len; k += obj->step_elems)
    if (receive_step(obj, data + k) != 0) return -1;
  return 0;
}
#else
// binary-symmetric-channel/viterbi-decoder.c:234-243: one symbol per step, masked to n bits.
CCV_EXPORT int decoder_input(struct decoder* obj, uint8_t* data, uint8_t len) {
  if (obj->plan == nullptr) return shim_fail("decoder not initialised");
  const uint8_t mask = (uint8_t)((1u << obj->parameter.symlen_out) - 1u);
  for (size_t k = 0; k < len; ++k) {
    const uint8_t sym = data[k] & mask;
    if (receive_step(obj, &sym) != 0) return -1;
  }
  return 0;
}
#endif

CCV_EXPORT int decoder_set_generator_mode(struct decoder* obj, int mode) {
  if (obj == nullptr) return shim_fail("null decoder");
  if (mode != CCV_GEN_REF_X86 && mode != CCV_GEN_TRUE_PARITY) return shim_fail("bad mode");
  obj->gen_mode = mode;
  return 0;
}

CCV_EXPORT int decoder_input_blocks(struct decoder* obj, const in_t* data, size_t n_blocks) {
  if (obj->plan == nullptr) return shim_fail("decoder not initialised");
  if (obj->symbol_counter != 0) return shim_fail("decoder is inside a block");
  const size_t per_block = obj->steps * obj->step_elems;
  for (size_t first = 0; first < n_blocks; first += kBatchChunk) {
    const size_t nb = n_blocks - first < kBatchChunk ? n_blocks - first : kBatchChunk;
    obj->batch_out.resize(nb * obj->out_bytes);
    obj->batch_pm.resize(nb);
    if (decode_stream(obj, data + first * per_block, nb, obj->batch_out.data(),
                      CCV_CHANNEL == CCV_HARD ? obj->batch_pm.data() : nullptr) != 0)
      return -1;
    for (size_t b = 0; b < nb; ++b) {
      std::memcpy(obj->output_data, &obj->batch_out[b * obj->out_bytes], obj->out_bytes);
      if (emit_output_buffer(obj, obj->batch_pm[b]) != 0) return -1;
      decoder_reset(obj);
    }
  }
  return 0;
}

#if defined(CCV_SHIM_AWGN)
CCV_EXPORT int decoder_decode_blocks(struct decoder* obj, const float* data, size_t n_blocks,
                                     uint8_t* out) {
  if (obj->plan == nullptr) return shim_fail("decoder not initialised");
  return decode_host(obj, data, n_blocks, out, nullptr);
}
CCV_EXPORT int decoder_decode_device(struct decoder* obj, const float* d_data, size_t n_blocks,
                                     uint8_t* d_out, void* stream) {
  if (obj->plan == nullptr) return shim_fail("decoder not initialised");
  if (ccv_decode_device(obj->plan, d_data, n_blocks, d_out, nullptr, nullptr, nullptr, nullptr,
                        stream) != 0)
    return shim_fail(ccv_last_error());
  return 0;
}
#else
CCV_EXPORT int decoder_decode_blocks(struct decoder* obj, const uint8_t* data, size_t n_blocks,
                                     uint8_t* out, int32_t* path_metrics) {
  if (obj->plan == nullptr) return shim_fail("decoder not initialised");
  return decode_host(obj, data, n_blocks, out, path_metrics);
}
CCV_EXPORT int decoder_decode_device(struct decoder* obj, const uint8_t* d_data, size_t n_blocks,
                                     uint8_t* d_out, int32_t* d_path_metrics, void* stream) {
  if (obj->plan == nullptr) return shim_fail("decoder not initialised");
  if (ccv_decode_device(obj->plan, d_data, n_blocks, d_out, d_path_metrics, nullptr, nullptr,
                        nullptr, stream) != 0)
    return shim_fail(ccv_last_error());
  return 0;
}
#endif

CCV_EXPORT const char* decoder_last_error(void) { return g_shim_error; }
