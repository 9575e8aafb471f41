// bitop3_probe.hip -- truth-table operand order of v_bitop3_b32 on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* o) {
  unsigned a = 0xF0F0F0F0u, b = 0xCCCCCCCCu, c = 0xAAAAAAAAu, r1, r2;
  asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(r1) : "v"(a), "v"(b), "v"(c));
  asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xf8" : "=v"(r2) : "v"(a), "v"(b), "v"(c));
  o[0] = r1; o[1] = r2;
}
int main() {
  unsigned* d; hipMalloc(&d, 8);
  hipLaunchKernelGGL(k, dim3(1), dim3(1), 0, 0, d);
  unsigned h[2]; hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
  // if TT index = (S0<<2)|(S1<<1)|S2: 0xca -> S0 ? S1 : S2 = 0xCCAACCAA... ; 0xf8 -> S0 | (S1 & S2)
  unsigned a = 0xF0F0F0F0u, b = 0xCCCCCCCCu, c = 0xAAAAAAAAu;
  printf("0xca: %08x (S0?S1:S2 = %08x)  0xf8: %08x (S0|(S1&S2) = %08x)\n", h[0], (a & b) | (~a & c), h[1],
         a | (b & c));
}
