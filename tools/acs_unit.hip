// acs_unit.hip -- device unit check of acs_step (acs_reg.hpp) for one trellis step: the H16 (BSC),
// uint32 and float instantiations against a plain per-state loop of the reference's ACS rule.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "acs_reg.hpp"

using namespace ccv;
constexpr CodeSpec kK7Ref{2, 7, {0xF200000000000000ull, 0xB600000000000000ull, 0, 0, 0, 0, 0, 0}, GEN_REF_X86};

template <CodeSpec C>
__global__ void unit(const uint32_t* m_in, const uint32_t* bm_in, uint64_t* out) {
  constexpr int S = 1 << (C.K - 1), H = S / 2;
  const int l = threadIdx.x;
  uint32_t Mu[S];
  H16 Mh[S];
  float Mf[S];
  for (int s = 0; s < S; ++s) {
    Mu[s] = m_in[l * S + s];
    Mh[s].v = Mu[s];
    Mf[s] = (float)Mu[s];
  }
  uint32_t Bu[4];
  H16 Bh[4];
  float Bf[4];
  for (int k = 0; k < 4; ++k) {
    Bu[k] = bm_in[l * 4 + k];
    Bh[k].v = Bu[k];
    Bf[k] = (float)Bu[k];
  }
  uint64_t ref = 0;
  for (int ns = 0; ns < S; ++ns) {
    const int i = ns / H, s0 = 2 * (ns % H), s1 = s0 + 1;
    const uint32_t m0 = Mu[s0] + Bu[expected_symbol(C, s0, i)];
    const uint32_t m1 = Mu[s1] + Bu[expected_symbol(C, s1, i)];
    if (m1 < m0) ref |= 1ull << ns;
  }
  out[l * 4 + 0] = ref;
  out[l * 4 + 1] = acs_step<C, false, H16>(Mh, Bh);
  out[l * 4 + 2] = acs_step<C, false, uint32_t>(Mu, Bu);
  out[l * 4 + 3] = acs_step<C, false, float>(Mf, Bf);
}

int main() {
  const int L = 64, S = 64;
  uint32_t hm[L * S], hb[L * 4];
  uint32_t x = 99;
  for (auto& v : hm) { x = x * 1664525u + 1013904223u; v = (x >> 20) & 63; }
  for (auto& v : hb) { x = x * 1664525u + 1013904223u; v = (x >> 20) % 3; }
  uint32_t *dm, *db;
  uint64_t* dout;
  hipMalloc(&dm, sizeof hm);
  hipMalloc(&db, sizeof hb);
  hipMalloc(&dout, L * 4 * 8);
  hipMemcpy(dm, hm, sizeof hm, hipMemcpyHostToDevice);
  hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(unit<kK7Ref>, dim3(1), dim3(L), 0, 0, dm, db, dout);
  uint64_t ho[L * 4];
  hipMemcpy(ho, dout, sizeof ho, hipMemcpyDeviceToHost);
  int bad[4] = {0, 0, 0, 0};
  for (int l = 0; l < L; ++l)
    for (int v = 1; v < 4; ++v)
      if (ho[l * 4 + v] != ho[l * 4]) {
        if (bad[v]++ < 3)
          printf("lane %d variant %d: %016llx vs ref %016llx (xor %016llx)\n", l, v,
                 (unsigned long long)ho[l * 4 + v], (unsigned long long)ho[l * 4],
                 (unsigned long long)(ho[l * 4 + v] ^ ho[l * 4]));
      }
  printf("mismatching lanes: H16 %d, u32 %d, f32 %d of %d\n", bad[1], bad[2], bad[3], L);
  return 0;
}
