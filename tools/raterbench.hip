// raterbench.hip -- issue rate of candidate VALU instructions on gfx950 (4 waves/SIMD, independent ops).
#include <hip/hip_runtime.h>
#include <cstdio>
#define R8(x) x x x x x x x x
#define CLOB "v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","s20","s21","s22","s23","vcc"
#define K(name, ins) __global__ __launch_bounds__(256) void name(float* o, int it) { \
  for (int i = 0; i < it; ++i) asm volatile(R8(R8(ins)) ::: CLOB); if (it < 0) o[0] = 0; }
#define Q4(a,b,c,d) a "\n" b "\n" c "\n" d "\n"
K(k_add, Q4("v_add_f32 v4, v8, v12","v_add_f32 v5, v9, v13","v_add_f32 v6, v10, v14","v_add_f32 v7, v11, v15"))
K(k_min, Q4("v_min_f32 v4, v8, v12","v_min_f32 v5, v9, v13","v_min_f32 v6, v10, v14","v_min_f32 v7, v11, v15"))
K(k_sub, Q4("v_sub_f32 v4, v8, v12","v_sub_f32 v5, v9, v13","v_sub_f32 v6, v10, v14","v_sub_f32 v7, v11, v15"))
K(k_alignbit, Q4("v_alignbit_b32 v4, v8, v12, 31","v_alignbit_b32 v5, v9, v13, 31","v_alignbit_b32 v6, v10, v14, 31","v_alignbit_b32 v7, v11, v15, 31"))
K(k_lshl_or, Q4("v_lshl_or_b32 v4, v8, 1, v12","v_lshl_or_b32 v5, v9, 1, v13","v_lshl_or_b32 v6, v10, 1, v14","v_lshl_or_b32 v7, v11, 1, v15"))
K(k_or3, Q4("v_or3_b32 v4, v8, v12, v9","v_or3_b32 v5, v9, v13, v10","v_or3_b32 v6, v10, v14, v11","v_or3_b32 v7, v11, v15, v8"))
K(k_lshr, Q4("v_lshrrev_b32 v4, 31, v8","v_lshrrev_b32 v5, 31, v9","v_lshrrev_b32 v6, 31, v10","v_lshrrev_b32 v7, 31, v11"))
K(k_lshl_add, Q4("v_lshl_add_u32 v4, v8, 1, v12","v_lshl_add_u32 v5, v9, 1, v13","v_lshl_add_u32 v6, v10, 1, v14","v_lshl_add_u32 v7, v11, 1, v15"))
K(k_bfi, Q4("v_bfi_b32 v4, v8, v12, v9","v_bfi_b32 v5, v9, v13, v10","v_bfi_b32 v6, v10, v14, v11","v_bfi_b32 v7, v11, v15, v8"))
K(k_and_or, Q4("v_and_or_b32 v4, v8, v12, v9","v_and_or_b32 v5, v9, v13, v10","v_and_or_b32 v6, v10, v14, v11","v_and_or_b32 v7, v11, v15, v8"))
K(k_perm, Q4("v_perm_b32 v4, v8, v12, v9","v_perm_b32 v5, v9, v13, v10","v_perm_b32 v6, v10, v14, v11","v_perm_b32 v7, v11, v15, v8"))
K(k_cmp_e64, Q4("v_cmp_lt_f32_e64 s[20:21], v8, v12","v_cmp_lt_f32_e64 s[22:23], v9, v13","v_cmp_lt_f32_e64 s[20:21], v10, v14","v_cmp_lt_f32_e64 s[22:23], v11, v15"))
K(k_cndmask, Q4("v_cndmask_b32_e64 v4, v8, v12, s[20:21]","v_cndmask_b32_e64 v5, v9, v13, s[22:23]","v_cndmask_b32_e64 v6, v10, v14, s[20:21]","v_cndmask_b32_e64 v7, v11, v15, s[22:23]"))
K(k_addc, Q4("v_addc_co_u32_e64 v4, s[20:21], v8, v8, s[22:23]","v_addc_co_u32_e64 v5, s[20:21], v9, v9, s[22:23]","v_addc_co_u32_e64 v6, s[20:21], v10, v10, s[22:23]","v_addc_co_u32_e64 v7, s[20:21], v11, v11, s[22:23]"))
K(k_add_u32, Q4("v_add_u32 v4, v8, v12","v_add_u32 v5, v9, v13","v_add_u32 v6, v10, v14","v_add_u32 v7, v11, v15"))
K(k_min_u32, Q4("v_min_u32 v4, v8, v12","v_min_u32 v5, v9, v13","v_min_u32 v6, v10, v14","v_min_u32 v7, v11, v15"))
K(k_pk_add, Q4("v_pk_add_f32 v[4:5], v[8:9], v[12:13]","v_pk_add_f32 v[6:7], v[10:11], v[14:15]","v_pk_add_f32 v[4:5], v[10:11], v[12:13]","v_pk_add_f32 v[6:7], v[8:9], v[14:15]"))
K(k_sub_u32, Q4("v_sub_u32 v4, v8, v12","v_sub_u32 v5, v9, v13","v_sub_u32 v6, v10, v14","v_sub_u32 v7, v11, v15"))
K(k_med3, Q4("v_med3_f32 v4, v8, v12, v9","v_med3_f32 v5, v9, v13, v10","v_med3_f32 v6, v10, v14, v11","v_med3_f32 v7, v11, v15, v8"))
K(k_ashr, Q4("v_ashrrev_i32 v4, 31, v8","v_ashrrev_i32 v5, 31, v9","v_ashrrev_i32 v6, 31, v10","v_ashrrev_i32 v7, 31, v11"))
K(k_bfe, Q4("v_bfe_u32 v4, v8, 31, 1","v_bfe_u32 v5, v9, 31, 1","v_bfe_u32 v6, v10, 31, 1","v_bfe_u32 v7, v11, 31, 1"))
int main() {
  float* d; hipMalloc(&d, 4096);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  struct { const char* n; void (*k)(float*, int); } ks[] = {
    {"v_add_f32", k_add}, {"v_min_f32", k_min}, {"v_sub_f32", k_sub}, {"v_alignbit_b32", k_alignbit},
    {"v_lshl_or_b32", k_lshl_or}, {"v_or3_b32", k_or3}, {"v_lshrrev_b32", k_lshr}, {"v_lshl_add_u32", k_lshl_add},
    {"v_bfi_b32", k_bfi}, {"v_and_or_b32", k_and_or}, {"v_perm_b32", k_perm}, {"v_cmp_lt_f32_e64", k_cmp_e64},
    {"v_cndmask_b32_e64", k_cndmask}, {"v_addc_co_u32_e64", k_addc}, {"v_add_u32", k_add_u32},
    {"v_min_u32", k_min_u32}, {"v_pk_add_f32", k_pk_add}, {"v_sub_u32", k_sub_u32}, {"v_med3_f32", k_med3},
    {"v_ashrrev_i32", k_ashr}, {"v_bfe_u32", k_bfe}};
  const int it = 200, blocks = 256 * 4;   // 4 waves per SIMD
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d, it);
    hipEventRecord(a); hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d, it); hipEventRecord(b);
    hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms, a, b);
    printf("%-20s %.2f ns/instr/SIMD\n", k.n, ms * 1e6 / (4.0 * it * 256));
  }
}
