// sim.cpp -- libccv_sim.so: CPU producers of the decoder input (include/ccv_sim.h).
//
// Built with -ffp-contract=off and no -march flags: the channel's double/float arithmetic must
// round exactly like the reference build (gcc -O3, x86-64 baseline, no FMA) for the GLIBC source to
// reproduce the reference's decoder input bit for bit.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "ccv.h"
#include "ccv_sim.h"
#include "trellis.hpp"

namespace {

// common/constellations.c:6-28 (unit power, Gray mapped; index = symbol value, P0 = MSB).
const float kConst1[] = {0.707107f, 0.707107f, -0.707107f, -0.707107f};
const float kConst2[] = {0.707107f, 0.707107f, 0.707107f, -0.707107f,
                         -0.707107f, 0.707107f, -0.707107f, -0.707107f};
const float kConst3[] = {0.408248f, 0.408248f, 0.408248f, 1.224745f,
                         -0.408248f, 0.408248f, -1.224745f, 0.408248f,
                         0.408248f, -0.408248f, 1.224745f, -0.408248f,
                         -0.408248f, -0.408248f, -0.408248f, -1.224745f};

const float* constellation(int n) { return n == 1 ? kConst1 : n == 2 ? kConst2 : n == 3 ? kConst3 : nullptr; }

struct Code {
  int n, K, blen, T, IB, gen;
  uint64_t poly[ccv::kMaxN];
  std::vector<uint8_t> exp;   // trellis table for K <= kMaxK; longer codes (stack decoder) compute
  bool init(int n_, int K_, int blen_, const uint64_t* polys, int gen_) {
    if (n_ < 1 || n_ > ccv::kMaxN || K_ < 2 || K_ > 64 || blen_ < 1 || blen_ > 255 || !polys)
      return false;
    n = n_; K = K_; blen = blen_; gen = gen_;
    T = blen + K - 1;
    IB = (blen + 7) / 8;
    std::memcpy(poly, polys, sizeof(uint64_t) * (size_t)n);
    if (K <= ccv::kMaxK) {
      exp.resize(size_t{2} << (K - 1));
      ccv::build_trellis(n, K, polys, gen, exp.data());
    }
    return true;
  }
  // common/encoder.c:84-119: the encoder's shift register after shifting in bit i is exactly the
  // decoder's (state << (64-K)) | (i << 63) with state = the previous K-1 inputs.
  void encode(const uint8_t* info, uint8_t* syms) const {
    uint64_t s = 0;
    for (int t = 0; t < T; ++t) {
      uint64_t i = t < blen ? (info[t / 8] >> (7 - t % 8)) & 1u : 0u;
      if (!exp.empty()) {
        syms[t] = exp[2 * s + i];
      } else {
        const uint64_t sr = (s << (64 - K)) | (i << 63);
        int e = 0;
        for (int k = 0; k < n; ++k) e = (e << 1) | ccv::gen_bit(sr & poly[k], gen);
        syms[t] = (uint8_t)e;
      }
      s = (s >> 1) | (i << (K - 2));
    }
  }
};

// common/demapper.c:43-45,61-70
inline void demap(int n, const float* pts, float ndist, float x, float y, float* out) {
  for (int k = 0; k < (1 << n); ++k) {
    float dx = x - pts[2 * k];
    float dy = y - pts[2 * k + 1];
    out[k] = ((dx * dx) + (dy * dy)) / ndist;
  }
}

// common/hard-demapper.c:62-88: snap to the nearest point (strict <, first minimum), then the
// normalised squared distances from that point.
inline void demap_hard(int n, const float* pts, float ndist, float x, float y, float* out) {
  float min_val = INFINITY;
  int min_idx = 0;
  for (int k = 0; k < (1 << n); ++k) {
    float dx = x - pts[2 * k];
    float dy = y - pts[2 * k + 1];
    float d = (dx * dx) + (dy * dy);
    if (d < min_val) {
      min_val = d;
      min_idx = k;
    }
  }
  demap(n, pts, ndist, pts[2 * min_idx], pts[2 * min_idx + 1], out);
}

float ndist_of(const float* pts) {
  float dx = pts[0] - pts[2];
  float dy = pts[1] - pts[3];
  return (dx * dx) + (dy * dy);
}

// glibc random_r on a private TYPE_3 state: the same sequence srand(seed); rand() produces.
struct GlibcSource {
  random_data rd;
  char state[128];
  explicit GlibcSource(uint64_t seed) {
    std::memset(&rd, 0, sizeof rd);
    std::memset(state, 0, sizeof state);
    initstate_r((unsigned)seed, state, sizeof state, &rd);
  }
  uint32_t next() {
    int32_t r;
    random_r(&rd, &r);
    return (uint32_t)r;
  }
};

// Philox4x32-10, one counter stream per block; next() returns 31-bit values like rand().
struct PhiloxSource {
  uint32_t key[2];
  uint32_t ctr[4];
  uint32_t buf[4];
  int used = 4;
  PhiloxSource(uint64_t seed, uint64_t block) {
    key[0] = (uint32_t)seed;
    key[1] = (uint32_t)(seed >> 32);
    ctr[0] = (uint32_t)block;
    ctr[1] = (uint32_t)(block >> 32);
    ctr[2] = 0;
    ctr[3] = 0x43435631u;   // stream tag
  }
  void refill() {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3], k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
      uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
      uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n1 = (uint32_t)p1;
      uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1, n3 = (uint32_t)p0;
      c0 = n0; c1 = n1; c2 = n2; c3 = n3;
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    buf[0] = c0; buf[1] = c1; buf[2] = c2; buf[3] = c3;
    ++ctr[2];
    used = 0;
  }
  uint32_t next() {
    if (used == 4) refill();
    return buf[used++] >> 1;
  }
};

// common/gaussian.c:18-38: Box-Muller on rand()/RAND_MAX, cosine half first, sine half cached.
template <class Src>
struct Gauss {
  Src& src;
  double R = 0.0, Tt = 0.0;
  int phase = 0;
  explicit Gauss(Src& s) : src(s) {}
  double next() {
    if (phase == 0) {
      double u1, u2;
      do {
        u1 = (double)src.next() / 2147483647.0;
        u2 = (double)src.next() / 2147483647.0;
      } while (u1 == 0.0);
      R = std::sqrt(-2.0 * std::log(u1));
      Tt = 2.0 * M_PI * u2;
      phase = 1;
      return R * std::cos(Tt);
    }
    phase = 0;
    return R * std::sin(Tt);
  }
};

// One AWGN block in driver order (AWGN-channel/main.c:217-223 then :93-106 per symbol).
template <class Src>
void awgn_block(const Code& c, Src& src, Gauss<Src>& g, float scaling, const float* pts, float nd,
                bool hard, uint8_t* info, float* rx) {
  uint8_t syms[512];
  for (int j = 0; j < c.IB; ++j) info[j] = (uint8_t)(src.next() % 256);
  c.encode(info, syms);
  const int NS = 1 << c.n;
  for (int t = 0; t < c.T; ++t) {
    float x = pts[2 * syms[t]], y = pts[2 * syms[t] + 1];
    x = (float)((double)x + (double)scaling * g.next());
    y = (float)((double)y + (double)scaling * g.next());
    if (hard) demap_hard(c.n, pts, nd, x, y, rx + (size_t)t * NS);
    else demap(c.n, pts, nd, x, y, rx + (size_t)t * NS);
  }
}

// One BSC block in driver order (binary-symmetric-channel/main.c:162-164 then :62-68).
template <class Src>
void bsc_block(const Code& c, Src& src, int32_t p_ppm, uint8_t* info, uint8_t* syms) {
  for (int j = 0; j < c.IB; ++j) info[j] = (uint8_t)(src.next() % 256);
  c.encode(info, syms);
  for (int t = 0; t < c.T; ++t)
    for (int k = 0; k < c.n; ++k)
      if ((int32_t)(src.next() % 1000000u) < p_ppm) syms[t] ^= (uint8_t)(1u << k);
}

template <class F>
void parallel_blocks(size_t nblocks, int nthreads, F&& body) {
  if (nthreads < 1) nthreads = 1;
  if ((size_t)nthreads > nblocks) nthreads = (int)(nblocks ? nblocks : 1);
  if (nthreads == 1) {
    body(0, nblocks);
    return;
  }
  std::vector<std::thread> pool;
  const size_t per = nblocks / nthreads, extra = nblocks % nthreads;
  size_t first = 0;
  for (int t = 0; t < nthreads; ++t) {
    size_t cnt = per + ((size_t)t < extra ? 1 : 0);
    pool.emplace_back(body, first, first + cnt);
    first += cnt;
  }
  for (auto& th : pool) th.join();
}

}  // namespace

extern "C" {

int ccv_sim_encode(int n, int K, int blen, const uint64_t* polys, int gen_mode, const uint8_t* info,
                   size_t nblocks, uint8_t* syms) {
  Code c;
  if (!c.init(n, K, blen, polys, gen_mode) || !info || !syms) return -1;
  for (size_t b = 0; b < nblocks; ++b) c.encode(info + b * c.IB, syms + b * c.T);
  return 0;
}

int ccv_sim_demap(int n, const float* iq, size_t nsym, float* rx) {
  const float* pts = constellation(n);
  if (!pts || !iq || !rx) return -1;
  const float nd = ndist_of(pts);
  for (size_t k = 0; k < nsym; ++k) demap(n, pts, nd, iq[2 * k], iq[2 * k + 1], rx + (k << n));
  return 0;
}

double ccv_sim_noise_scaling(double ebn0_db) { return std::sqrt(0.5) * std::pow(10.0, -ebn0_db / 20.0); }

int ccv_sim_awgn(int n, int K, int blen, const uint64_t* polys, int gen_mode, int rng, uint64_t seed,
                 float scaling, size_t first_block, size_t nblocks, uint8_t* info, float* rx,
                 int nthreads) {
  Code c;
  const float* pts = constellation(n);
  if (!c.init(n, K, blen, polys, gen_mode) || !pts || !info || !rx) return -1;
  const float nd = ndist_of(pts);
  const size_t rx_per_block = (size_t)c.T << n;
  const bool hard = (rng & CCV_DEMAP_HARD) != 0;
  rng &= ~CCV_DEMAP_HARD;
  if (rng == CCV_RNG_GLIBC) {
    if (first_block != 0) return -1;
    GlibcSource src(seed);
    Gauss<GlibcSource> g(src);
    for (size_t b = 0; b < nblocks; ++b)
      awgn_block(c, src, g, scaling, pts, nd, hard, info + b * c.IB, rx + b * rx_per_block);
    return 0;
  }
  if (rng != CCV_RNG_PHILOX) return -1;
  parallel_blocks(nblocks, nthreads, [&](size_t lo, size_t hi) {
    for (size_t b = lo; b < hi; ++b) {
      PhiloxSource src(seed, first_block + b);
      Gauss<PhiloxSource> g(src);
      awgn_block(c, src, g, scaling, pts, nd, hard, info + b * c.IB, rx + b * rx_per_block);
    }
  });
  return 0;
}

int ccv_sim_bsc(int n, int K, int blen, const uint64_t* polys, int gen_mode, int rng, uint64_t seed,
                int32_t p_ppm, size_t first_block, size_t nblocks, uint8_t* info, uint8_t* syms,
                int nthreads) {
  Code c;
  if (!c.init(n, K, blen, polys, gen_mode) || !info || !syms) return -1;
  if (rng == CCV_RNG_GLIBC) {
    if (first_block != 0) return -1;
    GlibcSource src(seed);
    for (size_t b = 0; b < nblocks; ++b) bsc_block(c, src, p_ppm, info + b * c.IB, syms + b * c.T);
    return 0;
  }
  if (rng != CCV_RNG_PHILOX) return -1;
  parallel_blocks(nblocks, nthreads, [&](size_t lo, size_t hi) {
    for (size_t b = lo; b < hi; ++b) {
      PhiloxSource src(seed, first_block + b);
      bsc_block(c, src, p_ppm, info + b * c.IB, syms + b * c.T);
    }
  });
  return 0;
}

}  // extern "C"
