// raterbench.hip -- issue rate of candidate VALU instructions on gfx950 (4 waves/SIMD, independent ops).
#include <hip/hip_runtime.h>
#include <cstdio>
#define R8(x) x x x x x x x x
#define CLOB "v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","s20","s21","s22","s23","vcc"
#define K(name, ins) __global__ __launch_bounds__(256) void name(float* o, int it) { \
  for (int i = 0; i < it; ++i) asm volatile(R8(R8(ins)) ::: CLOB); if (it < 0) o[0] = 0; }
#define Q4(a,b,c,d) a "\n" b "\n" c "\n" d "\n"
K(k_cmp32, Q4("v_cmp_lt_f32_e32 vcc, v8, v12","v_cmp_lt_f32_e32 vcc, v9, v13","v_cmp_lt_f32_e32 vcc, v10, v14","v_cmp_lt_f32_e32 vcc, v11, v15"))
K(k_cnd32, Q4("v_cndmask_b32_e32 v4, v8, v12, vcc","v_cndmask_b32_e32 v5, v9, v13, vcc","v_cndmask_b32_e32 v6, v10, v14, vcc","v_cndmask_b32_e32 v7, v11, v15, vcc"))
K(k_addc32, Q4("v_addc_co_u32_e32 v4, vcc, v8, v8, vcc","v_addc_co_u32_e32 v5, vcc, v9, v9, vcc","v_addc_co_u32_e32 v6, vcc, v10, v10, vcc","v_addc_co_u32_e32 v7, vcc, v11, v11, vcc"))
K(k_seq, Q4("v_cmp_lt_f32_e32 vcc, v8, v12","v_cndmask_b32_e32 v4, v12, v8, vcc","v_addc_co_u32_e32 v5, vcc, v5, v5, vcc","v_add_f32 v6, v10, v14"))
K(k_max, Q4("v_max_f32 v4, v8, v12","v_max_f32 v5, v9, v13","v_max_f32 v6, v10, v14","v_max_f32 v7, v11, v15"))
K(k_min_i32, Q4("v_min_i32 v4, v8, v12","v_min_i32 v5, v9, v13","v_min_i32 v6, v10, v14","v_min_i32 v7, v11, v15"))
K(k_and, Q4("v_and_b32 v4, v8, v12","v_and_b32 v5, v9, v13","v_and_b32 v6, v10, v14","v_and_b32 v7, v11, v15"))
K(k_or, Q4("v_or_b32 v4, v8, v12","v_or_b32 v5, v9, v13","v_or_b32 v6, v10, v14","v_or_b32 v7, v11, v15"))
K(k_lshl, Q4("v_lshlrev_b32 v4, 1, v8","v_lshlrev_b32 v5, 1, v9","v_lshlrev_b32 v6, 1, v10","v_lshlrev_b32 v7, 1, v11"))
K(k_mul, Q4("v_mul_f32 v4, v8, v12","v_mul_f32 v5, v9, v13","v_mul_f32 v6, v10, v14","v_mul_f32 v7, v11, v15"))
K(k_fma, Q4("v_fma_f32 v4, v8, v12, v9","v_fma_f32 v5, v9, v13, v10","v_fma_f32 v6, v10, v14, v11","v_fma_f32 v7, v11, v15, v8"))
K(k_mov, Q4("v_mov_b32 v4, v8","v_mov_b32 v5, v9","v_mov_b32 v6, v10","v_mov_b32 v7, v11"))
K(k_xor, Q4("v_xor_b32 v4, v8, v12","v_xor_b32 v5, v9, v13","v_xor_b32 v6, v10, v14","v_xor_b32 v7, v11, v15"))
K(k_subrev, Q4("v_subrev_f32 v4, v8, v12","v_subrev_f32 v5, v9, v13","v_subrev_f32 v6, v10, v14","v_subrev_f32 v7, v11, v15"))
K(k_add_e64, Q4("v_add_f32_e64 v4, v8, v12","v_add_f32_e64 v5, v9, v13","v_add_f32_e64 v6, v10, v14","v_add_f32_e64 v7, v11, v15"))
K(k_min_dpp, Q4("v_min_f32_dpp v4, v8, v12 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf","v_min_f32_dpp v5, v9, v13 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf","v_min_f32_dpp v6, v10, v14 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf","v_min_f32_dpp v7, v11, v15 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"))
K(k_add_dpp, Q4("v_add_f32_dpp v4, v8, v12 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf","v_add_f32_dpp v5, v9, v13 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf","v_add_f32_dpp v6, v10, v14 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf","v_add_f32_dpp v7, v11, v15 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"))
int main() {
  float* d; hipMalloc(&d, 4096);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  struct { const char* n; void (*k)(float*, int); } ks[] = {
    {"v_cmp_lt_f32_e32", k_cmp32}, {"v_cndmask_b32_e32", k_cnd32}, {"v_addc_co_u32_e32", k_addc32},
    {"cmp/cnd/addc/add mix", k_seq}, {"v_max_f32", k_max}, {"v_min_i32", k_min_i32}, {"v_and_b32", k_and},
    {"v_or_b32", k_or}, {"v_lshlrev_b32", k_lshl}, {"v_mul_f32", k_mul}, {"v_fma_f32", k_fma},
    {"v_mov_b32", k_mov}, {"v_xor_b32", k_xor}, {"v_subrev_f32", k_subrev}, {"v_add_f32_e64", k_add_e64},
    {"v_min_f32_dpp", k_min_dpp}, {"v_add_f32_dpp", k_add_dpp}};
  const int it = 200, blocks = 256 * 4;   // 4 waves per SIMD
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d, it);
    hipEventRecord(a); hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d, it); hipEventRecord(b);
    hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms, a, b);
    printf("%-20s %.2f ns/instr/SIMD\n", k.n, ms * 1e6 / (4.0 * it * 256));
  }
}
