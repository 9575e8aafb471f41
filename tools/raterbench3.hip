// raterbench3.hip -- issue rate of packed 16-bit and bit-manipulation VALU instructions on gfx950
// (candidates for the BSC packed-u16 ACS and cheaper decision packing); 4 waves/SIMD, independent ops.
#include <hip/hip_runtime.h>
#include <cstdio>
#define R8(x) x x x x x x x x
#define CLOB "v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","vcc"
#define K(name, ins) __global__ __launch_bounds__(256) void name(float* o, int it) { \
  for (int i = 0; i < it; ++i) asm volatile(R8(R8(ins)) ::: CLOB); if (it < 0) o[0] = 0; }
#define Q4(op, tail) op " v4, v8, v12" tail "\n" op " v5, v9, v13" tail "\n" op " v6, v10, v14" tail "\n" op " v7, v11, v15" tail "\n"
#define Q3(op) op " v4, v8, v12, v9\n" op " v5, v9, v13, v10\n" op " v6, v10, v14, v11\n" op " v7, v11, v15, v8\n"
K(k_add_f32, Q4("v_add_f32", ""))
K(k_min_f32, Q4("v_min_f32", ""))
K(k_pk_add_u16, Q4("v_pk_add_u16", ""))
K(k_pk_sub_u16, Q4("v_pk_sub_u16", ""))
K(k_pk_sub_i16, Q4("v_pk_sub_i16", ""))
K(k_pk_min_u16, Q4("v_pk_min_u16", ""))
K(k_pk_max_i16, Q4("v_pk_max_i16", ""))
K(k_pk_lshr_b16, Q4("v_pk_lshrrev_b16", ""))
K(k_add_u16, Q4("v_add_u16", ""))
K(k_min_u16, Q4("v_min_u16", ""))
K(k_pk_add_f16, Q4("v_pk_add_f16", ""))
K(k_pk_min_f16, Q4("v_pk_min_f16", ""))
K(k_min_u32, Q4("v_min_u32", ""))
K(k_sub_u32, Q4("v_sub_u32", ""))
K(k_lshr, Q4("v_lshrrev_b32", ""))
K(k_bitop3, Q3("v_bitop3_b32") )
K(k_mad_u24, Q3("v_mad_u32_u24"))
K(k_and_or, Q3("v_and_or_b32"))
K(k_alignbit, Q3("v_alignbit_b32"))
K(k_bcnt, Q4("v_bcnt_u32_b32", ""))
K(k_perm, Q3("v_perm_b32"))
K(k_sad_u16, Q3("v_sad_u16"))
int main() {
  float* d; hipMalloc(&d, 4096);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  struct { const char* n; void (*k)(float*, int); } ks[] = {
    {"v_add_f32", k_add_f32}, {"v_min_f32", k_min_f32}, {"v_pk_add_u16", k_pk_add_u16},
    {"v_pk_sub_u16", k_pk_sub_u16}, {"v_pk_sub_i16", k_pk_sub_i16}, {"v_pk_min_u16", k_pk_min_u16},
    {"v_pk_max_i16", k_pk_max_i16}, {"v_pk_lshrrev_b16", k_pk_lshr_b16}, {"v_add_u16", k_add_u16},
    {"v_min_u16", k_min_u16}, {"v_pk_add_f16", k_pk_add_f16}, {"v_pk_min_f16", k_pk_min_f16},
    {"v_min_u32", k_min_u32}, {"v_sub_u32", k_sub_u32}, {"v_lshrrev_b32", k_lshr},
    {"v_bitop3_b32", k_bitop3}, {"v_mad_u32_u24", k_mad_u24}, {"v_and_or_b32", k_and_or},
    {"v_alignbit_b32", k_alignbit}, {"v_bcnt_u32_b32", k_bcnt}, {"v_perm_b32", k_perm},
    {"v_sad_u16", k_sad_u16}};
  const int it = 200, blocks = 256 * 4;   // 4 waves per SIMD
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d, it);
    hipEventRecord(a); hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d, it); hipEventRecord(b);
    hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms, a, b);
    printf("%-20s %.2f ns/instr/SIMD\n", k.n, ms * 1e6 / (4.0 * it * 256));
  }
}
