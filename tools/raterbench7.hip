// raterbench7.hip -- which part of a compiler-style select costs on gfx950: the VOP2 (e32) encoding
// of v_cndmask, the VCC register as its mask, or the v_cmp -> mask dependency.
#include <hip/hip_runtime.h>
#include <cstdio>
#define R8(x) x x x x x x x x
#define CLOB "v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","s4","s5","s6","s7","vcc"
#define K(name, pre, ins) __global__ __launch_bounds__(256) void name(float* o, int it) { \
  asm volatile(pre ::: CLOB); \
  for (int i = 0; i < it; ++i) asm volatile(R8(R8(ins)) ::: CLOB); if (it < 0) o[0] = 0; }
#define SETM "s_mov_b64 vcc, exec\ns_mov_b64 s[4:5], exec\ns_mov_b64 s[6:7], 0\n"
K(k_e32_vcc, SETM, "v_cndmask_b32_e32 v4, v8, v12, vcc\nv_cndmask_b32_e32 v5, v9, v13, vcc\nv_cndmask_b32_e32 v6, v10, v14, vcc\nv_cndmask_b32_e32 v7, v11, v15, vcc\n")
K(k_e64_vcc, SETM, "v_cndmask_b32_e64 v4, v8, v12, vcc\nv_cndmask_b32_e64 v5, v9, v13, vcc\nv_cndmask_b32_e64 v6, v10, v14, vcc\nv_cndmask_b32_e64 v7, v11, v15, vcc\n")
K(k_e64_sgpr, SETM, "v_cndmask_b32_e64 v4, v8, v12, s[4:5]\nv_cndmask_b32_e64 v5, v9, v13, s[4:5]\nv_cndmask_b32_e64 v6, v10, v14, s[6:7]\nv_cndmask_b32_e64 v7, v11, v15, s[6:7]\n")
K(k_cmp32_cnd32, SETM, "v_cmp_lt_f32_e32 vcc, v8, v12\nv_cndmask_b32_e32 v4, v8, v12, vcc\nv_cmp_lt_f32_e32 vcc, v9, v13\nv_cndmask_b32_e32 v5, v9, v13, vcc\n")
K(k_cmp64_cnd64, SETM, "v_cmp_lt_f32_e64 s[4:5], v8, v12\nv_cndmask_b32_e64 v4, v8, v12, s[4:5]\nv_cmp_lt_f32_e64 s[6:7], v9, v13\nv_cndmask_b32_e64 v5, v9, v13, s[6:7]\n")
K(k_cmp64_cnd64_same, SETM, "v_cmp_lt_f32_e64 s[4:5], v8, v12\nv_cndmask_b32_e64 v4, v8, v12, s[4:5]\nv_cmp_lt_f32_e64 s[4:5], v9, v13\nv_cndmask_b32_e64 v5, v9, v13, s[4:5]\n")
K(k_add_ref, SETM, "v_add_f32 v4, v8, v12\nv_add_f32 v5, v9, v13\nv_add_f32 v6, v10, v14\nv_add_f32 v7, v11, v15\n")
int main() {
  float* d; (void)hipMalloc(&d, 4096);
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  struct { const char* n; void (*k)(float*, int); } ks[] = {
    {"v_cndmask e32, vcc (constant)", k_e32_vcc}, {"v_cndmask e64, vcc (constant)", k_e64_vcc},
    {"v_cndmask e64, sgpr (constant)", k_e64_sgpr}, {"v_cmp e32 -> vcc -> v_cndmask e32", k_cmp32_cnd32},
    {"v_cmp e64 -> s[4:5]/s[6:7] -> v_cndmask e64", k_cmp64_cnd64}, {"v_cmp e64 -> s[4:5] -> cndmask e64 (same pair)", k_cmp64_cnd64_same},
    {"v_add_f32 (reference)", k_add_ref}};
  const int it = 200, blocks = 256 * 4;
  for (int rep = 0; rep < 2; ++rep)
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d, it);
    (void)hipEventRecord(a); hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d, it); (void)hipEventRecord(b);
    (void)hipEventSynchronize(b); float ms; (void)hipEventElapsedTime(&ms, a, b);
    printf("%-48s %.2f ns/instr/SIMD\n", k.n, ms * 1e6 / (4.0 * it * 256));
  }
}
