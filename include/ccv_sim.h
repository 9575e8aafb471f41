/*
 * ccv_sim.h -- CPU-side producers of the decoder's input, libccv_sim.so.
 *
 * The encoder -> mapper -> channel -> demapper chain the reference drivers run before the decoder
 * (common/encoder.c:84-119, common/mapper.c:54-71, AWGN-channel/main.c:93-106 with
 * common/gaussian.c:18-38, common/demapper.c:61-85; BSC: binary-symmetric-channel/main.c:57-72),
 * batched over independent blocks. Outputs use the layouts of include/ccv.h.
 *
 * Two random sources:
 *   CCV_RNG_GLIBC   glibc's own random_r() on a private state seeded like srand(seed), consumed in the
 *                   drivers' order (info bytes of a block, then its noise / flips); reproduces the
 *                   reference's inputs bit for bit, sequential (nthreads ignored).
 *   CCV_RNG_PHILOX  Philox4x32-10 keyed by seed, one counter stream per block index, same draw
 *                   formulas; block b's inputs depend only on (seed, b), so any thread count and any
 *                   sharding across GPUs give the same frames. Statistically identical channel.
 */
#ifndef CCV_SIM_H
#define CCV_SIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CCV_RNG_GLIBC 0
#define CCV_RNG_PHILOX 1
/* OR into ccv_sim_awgn's rng argument: demap with common/hard-demapper.c (snap to the nearest point,
 * then distances from it) instead of common/demapper.c. */
#define CCV_DEMAP_HARD 0x100

/* Encoder only: syms = uint8 [nblocks][T] from info = uint8 [nblocks][ceil(blen/8)]. */
int ccv_sim_encode(int n, int K, int blen, const uint64_t* polys, int gen_mode, const uint8_t* info,
                   size_t nblocks, uint8_t* syms);

/* Soft demapper only: iq = float [nsym][2] received samples -> rx = float [nsym][2^n]. */
int ccv_sim_demap(int n, const float* iq, size_t nsym, float* rx);

/* Noise scaling 1/sqrt(2) * 10^(-EbN0/20) (AWGN-channel/main.c:153-161), in double. */
double ccv_sim_noise_scaling(double ebn0_db);

/* AWGN: random info bytes, encode, map, add scaling * N(0,1) per I/Q sample, demap.
 * Blocks [first_block, first_block + nblocks) of the stream (PHILOX; GLIBC requires first_block = 0). */
int ccv_sim_awgn(int n, int K, int blen, const uint64_t* polys, int gen_mode, int rng, uint64_t seed,
                 float scaling, size_t first_block, size_t nblocks, uint8_t* info, float* rx,
                 int nthreads);

/* BSC: random info bytes, encode, flip each symbol bit with probability p_ppm / 1e6. */
int ccv_sim_bsc(int n, int K, int blen, const uint64_t* polys, int gen_mode, int rng, uint64_t seed,
                int32_t p_ppm, size_t first_block, size_t nblocks, uint8_t* info, uint8_t* syms,
                int nthreads);

#ifdef __cplusplus
}
#endif
#endif
