// raterbench8.hip -- gfx950 issue cost of packed 16-bit integer ops (v_pk_add_u16, v_pk_min_u16,
// v_pk_sub_i16) against v_add_f32 / v_add_u16 / v_min_f32, alone and in a packed-ACS butterfly mix:
// a candidate for the BSC ACS, whose path metrics are small integers (round 6 probe).
// Build: hipcc -O3 --offload-arch=gfx950 raterbench8.hip -o raterbench8
#include <hip/hip_runtime.h>
#include <cstdio>
#define R8(x) x x x x x x x x
#define CLOB "v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v20","v21","v22","v23"
#define K(name, ins) __global__ __launch_bounds__(256) void name(float* o, int it) { \
  for (int i = 0; i < it; ++i) asm volatile(R8(R8(ins)) ::: CLOB); if (it < 0) o[0] = 0; }
#define Q4(op) op " v4, v8, v12\n" op " v5, v9, v13\n" op " v6, v10, v14\n" op " v7, v11, v15\n"
K(k_add_f32, Q4("v_add_f32"))
K(k_min_f32, Q4("v_min_f32"))
K(k_add_u16, Q4("v_add_u16"))
K(k_pk_add_u16, Q4("v_pk_add_u16"))
K(k_pk_min_u16, Q4("v_pk_min_u16"))
K(k_pk_sub_i16, Q4("v_pk_sub_i16"))
K(k_pk_max_i16, Q4("v_pk_max_i16"))
// packed butterfly pair (new states j and j+32 in one register's halves): 2 pk_add (candidates with
// the old metric broadcast by op_sel), pk_min, pk_sub (both decisions' signs), alignbit (hi decision),
// bfe + lshl_or (lo decision) -- 7 instructions for 2 new states
#define PBF(m, a, b, n, d, dl, dh, t) \
  "v_pk_add_u16 " a ", " m ", v20 op_sel:[0,0] op_sel_hi:[0,1]\n" \
  "v_pk_add_u16 " b ", " m ", v21 op_sel:[1,0] op_sel_hi:[1,1]\n" \
  "v_pk_min_u16 " n ", " a ", " b "\n" \
  "v_pk_sub_i16 " d ", " b ", " a "\n" \
  "v_alignbit_b32 " dh ", " dh ", " d ", 31\n" \
  "v_bfe_u32 " t ", " d ", 15, 1\n" \
  "v_lshl_or_b32 " dl ", " dl ", 1, " t "\n"
K(k_pbf, PBF("v4", "v8", "v9", "v12", "v13", "v16", "v17", "v18") PBF("v5", "v10", "v11", "v14", "v15", "v19", "v22", "v23"))
// the scalar fp32 butterfly of the production kernels: 4 add, 2 sub, 2 min, 2 alignbit (2 new states)
#define BF(m0, m1, a0, b0, a1, b1, x, y, d, e) \
  "v_add_f32 " a0 ", " m0 ", v20\n" "v_add_f32 " b0 ", " m0 ", v21\n" "v_add_f32 " a1 ", " m1 ", v21\n" "v_add_f32 " b1 ", " m1 ", v20\n" \
  "v_sub_f32 " x ", " a1 ", " a0 "\n" "v_sub_f32 " y ", " b1 ", " b0 "\n" "v_min_f32 " m0 ", " a0 ", " a1 "\n" "v_min_f32 " m1 ", " b0 ", " b1 "\n" \
  "v_alignbit_b32 " d ", " d ", " x ", 31\n" "v_alignbit_b32 " e ", " e ", " y ", 31\n"
K(k_bf, BF("v4", "v5", "v8", "v9", "v10", "v11", "v12", "v13", "v16", "v17") BF("v6", "v7", "v18", "v19", "v14", "v15", "v22", "v23", "v16", "v17"))
int main() {
  float* d; (void)hipMalloc(&d, 4096);
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  struct { const char* n; void (*k)(float*, int); double per; double states; } ks[] = {
    {"v_add_f32", k_add_f32, 4, 0}, {"v_min_f32", k_min_f32, 4, 0}, {"v_add_u16", k_add_u16, 4, 0},
    {"v_pk_add_u16", k_pk_add_u16, 4, 0}, {"v_pk_min_u16", k_pk_min_u16, 4, 0}, {"v_pk_sub_i16", k_pk_sub_i16, 4, 0},
    {"v_pk_max_i16", k_pk_max_i16, 4, 0},
    {"packed u16 butterfly pair (7 instr, 2 states)", k_pbf, 14, 4},
    {"fp32 scalar butterfly (10 instr, 2 states)", k_bf, 20, 4}};
  const int it = 200, blocks = 256 * 4;
  for (int rep = 0; rep < 2; ++rep)
    for (auto& k : ks) {
      hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d, it);
      (void)hipEventRecord(a);
      hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d, it);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms; (void)hipEventElapsedTime(&ms, a, b);
      const double per_instr = ms * 1e6 / (k.per * it * 256);
      if (rep == 1) {
        if (k.states > 0)
          printf("%-46s %.2f ns/instr/SIMD  %.2f ns/state/SIMD\n", k.n, per_instr, ms * 1e6 / (k.states * it * 256));
        else
          printf("%-46s %.2f ns/instr/SIMD\n", k.n, per_instr);
      }
    }
}
