// raterbench5.hip -- issue rate on gfx950 of the candidates for a compare-select ACS without
// v_min_f32 / v_alignbit: v_ashrrev_i32 (sign mask), v_bitop3 with an SGPR operand (decision insert),
// v_bfe_i32, v_cndmask_b32_e32, v_max/min_i32, v_sub_f32 and a mixed 6-instruction ACS state.
#include <hip/hip_runtime.h>
#include <cstdio>
#define R8(x) x x x x x x x x
#define CLOB "v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","s4","s5","vcc"
#define K(name, ins) __global__ __launch_bounds__(256) void name(float* o, int it) { \
  for (int i = 0; i < it; ++i) asm volatile(R8(R8(ins)) ::: CLOB); if (it < 0) o[0] = 0; }
#define Q4(op, tail) op " v4, v8, v12" tail "\n" op " v5, v9, v13" tail "\n" op " v6, v10, v14" tail "\n" op " v7, v11, v15" tail "\n"
#define Q4A(op, a) op " v4, " a ", v8\n" op " v5, " a ", v9\n" op " v6, " a ", v10\n" op " v7, " a ", v11\n"
#define Q4B(op, tail) op " v4, s4, v8, v12" tail "\n" op " v5, s4, v9, v13" tail "\n" op " v6, s5, v10, v14" tail "\n" op " v7, s5, v11, v15" tail "\n"
#define Q4V(op, tail) op " v4, v16, v8, v12" tail "\n" op " v5, v17, v9, v13" tail "\n" op " v6, v18, v10, v14" tail "\n" op " v7, v19, v11, v15" tail "\n"
// one ACS state: a0 = m0 + b0, a1 = m1 + b1, diff = a1 - a0, mask = diff >> 31 (arith),
// n = mask ? a1 : a0, d = s ? mask : d   (4 independent chains)
#define ACS1(x, m0, m1, b0, b1, a0, a1, d) \
  "v_add_f32 " a0 ", " m0 ", " b0 "\n" "v_add_f32 " a1 ", " m1 ", " b1 "\n" \
  "v_sub_f32 " x ", " a1 ", " a0 "\n" "v_ashrrev_i32 " x ", 31, " x "\n" \
  "v_bitop3_b32 " m0 ", " x ", " a1 ", " a0 " bitop3:0xca\n" "v_bitop3_b32 " d ", s4, " x ", " d " bitop3:0xca\n"
#define ACS4 ACS1("v4","v8","v9","v16","v17","v12","v13","v18") ACS1("v5","v10","v11","v16","v17","v14","v15","v19") \
             ACS1("v6","v8","v9","v16","v17","v12","v13","v18") ACS1("v7","v10","v11","v16","v17","v14","v15","v19")
#define ACSOLD1(x, m0, m1, b0, b1, a0, a1, d) \
  "v_add_f32 " a0 ", " m0 ", " b0 "\n" "v_add_f32 " a1 ", " m1 ", " b1 "\n" \
  "v_min_f32 " m0 ", " a0 ", " a1 "\n" "v_sub_f32 " x ", " a1 ", " a0 "\n" "v_alignbit_b32 " d ", " d ", " x ", 31\n"
#define ACSOLD4 ACSOLD1("v4","v8","v9","v16","v17","v12","v13","v18") ACSOLD1("v5","v10","v11","v16","v17","v14","v15","v19") \
             ACSOLD1("v6","v8","v9","v16","v17","v12","v13","v18") ACSOLD1("v7","v10","v11","v16","v17","v14","v15","v19")
K(k_ashr, Q4A("v_ashrrev_i32", "31"))
K(k_lshr, Q4A("v_lshrrev_b32", "31"))
K(k_bitop3_s, Q4B("v_bitop3_b32", " bitop3:0xca"))
K(k_bitop3_v, Q4V("v_bitop3_b32", " bitop3:0xca"))
K(k_bfe, Q4V("v_bfe_i32", ""))
K(k_cnd, Q4("v_cndmask_b32_e32", ""))
K(k_maxi, Q4("v_max_i32", ""))
K(k_subf, Q4("v_sub_f32", ""))
K(k_minf, Q4("v_min_f32", ""))
K(k_align, Q4V("v_alignbit_b32", ""))
K(k_acs_new, ACS4)
K(k_acs_old, ACSOLD4)
int main() {
  float* d; hipMalloc(&d, 4096);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  struct { const char* n; void (*k)(float*, int); double per; } ks[] = {
    {"v_ashrrev_i32", k_ashr, 4}, {"v_lshrrev_b32", k_lshr, 4}, {"v_bitop3 sgpr", k_bitop3_s, 4},
    {"v_bitop3 vgpr", k_bitop3_v, 4}, {"v_bfe_i32", k_bfe, 4}, {"v_cndmask_b32_e32", k_cnd, 4},
    {"v_max_i32", k_maxi, 4}, {"v_sub_f32", k_subf, 4}, {"v_min_f32", k_minf, 4},
    {"v_alignbit_b32", k_align, 4},
    {"ACS state new (6 instr)", k_acs_new, 24}, {"ACS state old (5 instr)", k_acs_old, 20}};
  const int it = 200, blocks = 256 * 4;
  for (int rep = 0; rep < 2; ++rep)
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d, it);
    hipEventRecord(a); hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d, it); hipEventRecord(b);
    hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms, a, b);
    const double per_instr = ms * 1e6 / (k.per * it * 256);
    printf("%-26s %.2f ns/instr/SIMD  %.2f ns/ACS-state\n", k.n, per_instr, per_instr * k.per / 4);
  }
}
