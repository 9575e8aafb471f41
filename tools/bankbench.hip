// bankbench.hip -- VALU issue rate vs VGPR source-operand banks (index mod 4) on gfx950.
// Each kernel runs a long unrolled chain of independent v_add_f32 in inline asm with explicit
// registers: "same" reads two operands from the same bank, "diff" from different banks.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

#define BODY_SAME \
  "v_add_f32 v4, v8, v12\n v_add_f32 v5, v9, v13\n v_add_f32 v6, v10, v14\n v_add_f32 v7, v11, v15\n" \
  "v_add_f32 v16, v20, v24\n v_add_f32 v17, v21, v25\n v_add_f32 v18, v22, v26\n v_add_f32 v19, v23, v27\n"
#define BODY_DIFF \
  "v_add_f32 v4, v8, v13\n v_add_f32 v5, v9, v14\n v_add_f32 v6, v10, v15\n v_add_f32 v7, v11, v12\n" \
  "v_add_f32 v16, v20, v25\n v_add_f32 v17, v21, v26\n v_add_f32 v18, v22, v27\n v_add_f32 v19, v23, v24\n"
#define BODY_DEP \
  "v_add_f32 v4, v4, v13\n v_min_f32 v5, v4, v14\n v_add_f32 v6, v5, v15\n v_min_f32 v7, v6, v12\n" \
  "v_add_f32 v16, v7, v25\n v_min_f32 v17, v16, v26\n v_add_f32 v18, v17, v27\n v_min_f32 v19, v18, v24\n"
#define BODY_ALIGN \
  "v_alignbit_b32 v4, v8, v13, 31\n v_alignbit_b32 v5, v9, v14, 31\n v_alignbit_b32 v6, v10, v15, 31\n v_alignbit_b32 v7, v11, v12, 31\n" \
  "v_alignbit_b32 v16, v20, v25, 31\n v_alignbit_b32 v17, v21, v26, 31\n v_alignbit_b32 v18, v22, v27, 31\n v_alignbit_b32 v19, v23, v24, 31\n"
#define R8(x) x x x x x x x x
#define KERNEL(name, body) \
  __global__ __launch_bounds__(256) void name(float* out, int iters) { \
    for (int i = 0; i < iters; ++i) asm volatile(R8(R8(body)) ::: "v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27"); \
    if (iters < 0) out[threadIdx.x] = 0; }
KERNEL(k_same, BODY_SAME)
KERNEL(k_diff, BODY_DIFF)
KERNEL(k_dep, BODY_DEP)
KERNEL(k_align, BODY_ALIGN)

int main() {
  float* d; CK(hipMalloc(&d, 4096));
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const int iters = 200;                      // 200 * 512 instructions per wave
  void (*ks[])(float*, int) = {k_same, k_diff, k_dep, k_align};
  const char* names[] = {"same-bank add", "diff-bank add", "dependent add/min", "alignbit"};
  for (int wps : {1, 2, 4, 8}) {               // waves per SIMD
    int blocks = 256 * wps;                    // 256-thread blocks = 4 waves = 1 per SIMD
    for (int k = 0; k < 4; ++k) {
      hipLaunchKernelGGL(ks[k], dim3(blocks), dim3(256), 0, 0, d, iters);
      hipEventRecord(a); hipLaunchKernelGGL(ks[k], dim3(blocks), dim3(256), 0, 0, d, iters); hipEventRecord(b);
      hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms, a, b);
      double instr_per_simd = (double)wps * iters * 512;
      printf("waves/SIMD %d %-18s %.3f ms  %.2f ns/instr/SIMD\n", wps, names[k], ms, ms * 1e6 / instr_per_simd);
    }
  }
  return 0;
}
