#include <hip/hip_runtime.h>
__global__ void k(unsigned* o, unsigned a, unsigned b) {
  unsigned r = 0xFFFF0000u, r2 = 0xFFFF0000u, r3, r4 = 0xAAAA5555u;
  asm volatile("v_add_u16_e32 %0, %1, %2" : "+v"(r) : "v"(a), "v"(b));
  asm volatile("v_min_u16_e32 %0, %1, %2" : "+v"(r2) : "v"(a), "v"(b));
  asm volatile("v_sub_u16_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0" : "=v"(r3) : "v"(a), "v"(b));
  asm volatile("v_sub_u16_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0" : "+v"(r4) : "v"(a), "v"(b));
  o[0] = r; o[1] = r2; o[2] = r3; o[3] = r4;
}
int main() {
  unsigned* d; hipMalloc(&d, 16);
  hipLaunchKernelGGL(k, dim3(1), dim3(1), 0, 0, d, 0x12340005u, 0x56780009u);
  unsigned h[4]; hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
  printf("add16 %08x min16 %08x sub_sdwa_pad %08x sub_sdwa_preserve %08x\n", h[0], h[1], h[2], h[3]);
}
