// trellis.hpp -- code description and trellis tables, usable in constexpr (kernel specialisation)
// and at run time (plans for codes without a specialised kernel).
//
// Trellis convention of the reference (AWGN-channel/viterbi-decoder.c:38-69):
//   state s in [0, 2^(K-1)) holds the last K-1 inputs, newest in bit K-2;
//   successor under input i: (s >> 1) | (i << (K-2));
//   generator register: (s << (64-K)) | (i << 63), polynomials MSB-aligned (tap 0 = bit 63);
//   expected symbol: polynomial 0's generator bit is the most significant bit.
#pragma once
#include <stdint.h>

namespace ccv {

// Generator-bit semantics (see include/ccv.h, CCV_GEN_*).
enum : int { GEN_REF_X86 = 0, GEN_TRUE_PARITY = 1 };

constexpr int kMaxN = 8;    // output bits per step (symlen_out is uint8_t; symbols must fit a byte)
constexpr int kMaxK = 12;   // 2048 states: the generic kernel keeps all decisions of a block in LDS

struct CodeSpec {
  int n;
  int K;
  uint64_t poly[kMaxN];
  int gen;
};

constexpr int parity64(uint64_t v) {
  v ^= v >> 32;
  v ^= v >> 16;
  v ^= v >> 8;
  v ^= v >> 4;
  v ^= v >> 2;
  v ^= v >> 1;
  return (int)(v & 1u);
}

// The reference evaluates `(0x6996 >> val) & 1` with a 64-bit, un-reduced `val`
// (viterbi-decoder.c:53-57, encoder.c:95-100). x86 masks the shift count to 5 bits, so the bit is
// cleared whenever the fold leaves bit 4 set, i.e. when parity(v & 0x1010...10) is odd.
constexpr int gen_bit(uint64_t v, int gen) {
  int p = parity64(v);
  if (gen == GEN_REF_X86) p &= parity64(v & 0x1010101010101010ull) ^ 1;
  return p;
}

constexpr int expected_symbol(int n, int K, const uint64_t* poly, int gen, uint32_t s, int i) {
  const uint64_t sr = ((uint64_t)s << (64 - K)) | ((uint64_t)(i & 1) << 63);
  int e = 0;
  for (int k = 0; k < n; ++k) e = (e << 1) | gen_bit(sr & poly[k], gen);
  return e;
}

constexpr int expected_symbol(const CodeSpec& c, uint32_t s, int i) {
  return expected_symbol(c.n, c.K, c.poly, c.gen, s, i);
}

// exp[2*s + i] for all states.
inline void build_trellis(int n, int K, const uint64_t* poly, int gen, uint8_t* exp) {
  const uint32_t S = 1u << (K - 1);
  for (uint32_t s = 0; s < S; ++s)
    for (int i = 0; i < 2; ++i) exp[2 * s + i] = (uint8_t)expected_symbol(n, K, poly, gen, s, i);
}

}  // namespace ccv
