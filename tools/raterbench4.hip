// raterbench4.hip -- issue rate of the 16-bit ACS candidates (SDWA forms) on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#define R8(x) x x x x x x x x
#define CLOB "v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","vcc"
#define K(name, ins) __global__ __launch_bounds__(256) void name(float* o, int it) { \
  for (int i = 0; i < it; ++i) asm volatile(R8(R8(ins)) ::: CLOB); if (it < 0) o[0] = 0; }
#define Q4(op, tail) op " v4, v8, v12" tail "\n" op " v5, v9, v13" tail "\n" op " v6, v10, v14" tail "\n" op " v7, v11, v15" tail "\n"
K(k_sub16_sdwa, Q4("v_sub_u16_sdwa", " dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0"))
K(k_sub32, Q4("v_sub_u32", ""))
K(k_add16, Q4("v_add_u16", ""))
K(k_sub16, Q4("v_sub_u16", ""))
K(k_min16, Q4("v_min_u16", ""))
int main() {
  float* d; hipMalloc(&d, 4096);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  struct { const char* n; void (*k)(float*, int); } ks[] = {
    {"v_sub_u16_sdwa WORD_1", k_sub16_sdwa}, {"v_sub_u32", k_sub32}, {"v_add_u16", k_add16},
    {"v_sub_u16", k_sub16}, {"v_min_u16", k_min16}};
  const int it = 200, blocks = 256 * 4;
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d, it);
    hipEventRecord(a); hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d, it); hipEventRecord(b);
    hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms, a, b);
    printf("%-24s %.2f ns/instr/SIMD\n", k.n, ms * 1e6 / (4.0 * it * 256));
  }
}
