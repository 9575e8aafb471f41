// raterbench6.hip -- gfx950 issue cost of the argmin / traceback candidates (v_cmp + v_cndmask
// chains, v_min3_f32, v_ffbl) and of packed-f32 ACS butterflies (v_pk_add_f32 with op_sel / neg).
#include <hip/hip_runtime.h>
#include <cstdio>
#define R8(x) x x x x x x x x
#define CLOB "v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v20","v21","v22","v23","s4","s5","s6","s7","vcc"
#define K(name, ins) __global__ __launch_bounds__(256) void name(float* o, int it) { \
  for (int i = 0; i < it; ++i) asm volatile(R8(R8(ins)) ::: CLOB); if (it < 0) o[0] = 0; }
#define Q4(op, tail) op " v4, v8, v12" tail "\n" op " v5, v9, v13" tail "\n" op " v6, v10, v14" tail "\n" op " v7, v11, v15" tail "\n"
#define Q4M3(op) op " v4, v8, v12, v16\n" op " v5, v9, v13, v17\n" op " v6, v10, v14, v18\n" op " v7, v11, v15, v19\n"
#define Q4U(op) op " v4, v8\n" op " v5, v9\n" op " v6, v10\n" op " v7, v11\n"
// argmin node as the compiler emits it: lt = m < best; best = lt ? m : best; idx = lt ? s : idx
#define AM1(m, best, idx, s) "v_cmp_lt_f32_e32 vcc, " m ", " best "\n" "v_cndmask_b32_e32 " best ", " best ", " m ", vcc\n" \
  "v_cndmask_b32_e32 " idx ", " idx ", " s ", vcc\n"
#define AM4 AM1("v8", "v4", "v12", "v16") AM1("v9", "v5", "v13", "v16") AM1("v10", "v6", "v14", "v16") AM1("v11", "v7", "v15", "v16")
#define AM1S(m, best, idx, s, sm) "v_cmp_lt_f32_e64 " sm ", " m ", " best "\n" "v_cndmask_b32_e64 " best ", " best ", " m ", " sm "\n" \
  "v_cndmask_b32_e64 " idx ", " idx ", " s ", " sm "\n"
#define AM4S AM1S("v8", "v4", "v12", "v16", "s[4:5]") AM1S("v9", "v5", "v13", "v16", "s[6:7]") AM1S("v10", "v6", "v14", "v16", "s[4:5]") AM1S("v11", "v7", "v15", "v16", "s[6:7]")
// butterfly, scalar: 4 add, 2 sub, 2 min, 2 alignbit
#define BF_OLD(m0, m1, a0, b0, a1, b1, x, y, d, e) \
  "v_add_f32 " a0 ", " m0 ", v20\n" "v_add_f32 " b0 ", " m0 ", v21\n" "v_add_f32 " a1 ", " m1 ", v21\n" "v_add_f32 " b1 ", " m1 ", v20\n" \
  "v_sub_f32 " x ", " a1 ", " a0 "\n" "v_sub_f32 " y ", " b1 ", " b0 "\n" "v_min_f32 " m0 ", " a0 ", " a1 "\n" "v_min_f32 " m1 ", " b0 ", " b1 "\n" \
  "v_alignbit_b32 " d ", " d ", " x ", 31\n" "v_alignbit_b32 " e ", " e ", " y ", 31\n"
// butterfly with one packed difference: (a0,b0) and (a1,b1) register pairs, diff pair = (a1,b1) - (a0,b0)
#define BF_PKD(m0, m1, a0, b0, a1, b1, xy, x, y, d, e) \
  "v_add_f32 v" a0 ", " m0 ", v20\n" "v_add_f32 v" b0 ", " m0 ", v21\n" "v_add_f32 v" a1 ", " m1 ", v21\n" "v_add_f32 v" b1 ", " m1 ", v20\n" \
  "v_pk_add_f32 " xy ", v[" a1 ":" b1 "], v[" a0 ":" b0 "] neg_lo:[0,1] neg_hi:[0,1]\n" "v_min_f32 " m0 ", v" a0 ", v" a1 "\n" "v_min_f32 " m1 ", v" b0 ", v" b1 "\n" \
  "v_alignbit_b32 " d ", " d ", " x ", 31\n" "v_alignbit_b32 " e ", " e ", " y ", 31\n"
// fully packed: (a0,b0) = m0 + (B0,B1), (a1,b1) = m1 + (B1,B0), diff packed
#define BF_PK(mm, ab0, ab1, xy, x, y, d, e, a0, b0, a1, b1, m0, m1) \
  "v_pk_add_f32 " ab0 ", " mm ", v[20:21] op_sel:[0,0] op_sel_hi:[0,1]\n" "v_pk_add_f32 " ab1 ", " mm ", v[20:21] op_sel:[1,1] op_sel_hi:[1,0]\n" \
  "v_pk_add_f32 " xy ", " ab1 ", " ab0 " neg_lo:[0,1] neg_hi:[0,1]\n" "v_min_f32 " m0 ", " a0 ", " a1 "\n" "v_min_f32 " m1 ", " b0 ", " b1 "\n" \
  "v_alignbit_b32 " d ", " d ", " x ", 31\n" "v_alignbit_b32 " e ", " e ", " y ", 31\n"
K(k_argmin_vcc, AM4)
K(k_argmin_sgpr, AM4S)
K(k_cnd_e64, "v_cndmask_b32_e64 v4, v8, v12, s[4:5]\nv_cndmask_b32_e64 v5, v9, v13, s[4:5]\nv_cndmask_b32_e64 v6, v10, v14, s[6:7]\nv_cndmask_b32_e64 v7, v11, v15, s[6:7]\n")
K(k_cmp_e64, "v_cmp_lt_f32_e64 s[4:5], v8, v12\nv_cmp_lt_f32_e64 s[6:7], v9, v13\nv_cmp_lt_f32_e64 s[4:5], v10, v14\nv_cmp_lt_f32_e64 s[6:7], v11, v15\n")
K(k_min3, Q4M3("v_min3_f32"))
K(k_ffbl, Q4U("v_ffbl_b32"))
K(k_addu, Q4("v_add_u32", ""))
K(k_pkadd, "v_pk_add_f32 v[4:5], v[8:9], v[12:13]\nv_pk_add_f32 v[6:7], v[10:11], v[14:15]\nv_pk_add_f32 v[16:17], v[8:9], v[12:13]\nv_pk_add_f32 v[18:19], v[10:11], v[14:15]\n")
K(k_bf_old, BF_OLD("v4", "v5", "v8", "v9", "v10", "v11", "v12", "v13", "v16", "v17") BF_OLD("v6", "v7", "v18", "v19", "v14", "v15", "v22", "v23", "v16", "v17"))
K(k_bf_pkd, BF_PKD("v4", "v5", "8", "9", "10", "11", "v[12:13]", "v12", "v13", "v16", "v17") BF_PKD("v6", "v7", "18", "19", "14", "15", "v[22:23]", "v22", "v23", "v16", "v17"))
K(k_bf_pk, BF_PK("v[4:5]", "v[8:9]", "v[10:11]", "v[12:13]", "v12", "v13", "v16", "v17", "v8", "v9", "v10", "v11", "v4", "v5") BF_PK("v[6:7]", "v[18:19]", "v[14:15]", "v[22:23]", "v22", "v23", "v16", "v17", "v18", "v19", "v14", "v15", "v6", "v7"))
int main() {
  float* d; (void)hipMalloc(&d, 4096);
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  struct { const char* n; void (*k)(float*, int); double per; const char* unit; } ks[] = {
    {"argmin node (cmp vcc + 2 cndmask)", k_argmin_vcc, 12, "node"}, {"argmin node (cmp sgpr + 2 cndmask e64)", k_argmin_sgpr, 12, "node"},
    {"v_cndmask_b32_e64 sgpr", k_cnd_e64, 4, "instr"}, {"v_cmp_lt_f32_e64 sgpr", k_cmp_e64, 4, "instr"},
    {"v_min3_f32", k_min3, 4, "instr"}, {"v_ffbl_b32", k_ffbl, 4, "instr"}, {"v_add_u32", k_addu, 4, "instr"},
    {"v_pk_add_f32", k_pkadd, 4, "instr"},
    {"butterfly scalar (10 instr)", k_bf_old, 20, "butterfly"}, {"butterfly packed diff (9 instr)", k_bf_pkd, 18, "butterfly"},
    {"butterfly all packed (7 instr)", k_bf_pk, 14, "butterfly"}};
  const int it = 200, blocks = 256 * 4;
  for (int rep = 0; rep < 2; ++rep)
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d, it);
    (void)hipEventRecord(a); hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d, it); (void)hipEventRecord(b);
    (void)hipEventSynchronize(b); float ms; (void)hipEventElapsedTime(&ms, a, b);
    const double per_instr = ms * 1e6 / (k.per * it * 256);
    // k.per instructions per 4 (or 2 for butterflies) independent chains
    printf("%-42s %.2f ns/instr/SIMD\n", k.n, per_instr);
  }
}
