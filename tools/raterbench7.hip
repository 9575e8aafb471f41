// raterbench7.hip -- gfx950 issue cost of the cross-lane ACS forms of the multilane K = 9 kernels
// (acs_multi.hpp, acs_multi2.hpp): v_add_f32 with a quad_perm DPP source, in a butterfly stream, and
// mixed with plain butterflies at the kernels' ratios. ns per instruction per SIMD, 4 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#define R8(x) x x x x x x x x
#define CLOB "v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31","s4","s5","s6","s7","vcc"
#define K(name, ins) __global__ __launch_bounds__(256) void name(float* o, int it) { \
  for (int i = 0; i < it; ++i) asm volatile(R8(ins) ::: CLOB); if (it < 0) o[0] = 0; }
// in-lane butterfly: 4 add, 2 sub, 2 min, 2 alignbit
#define BF(m0, m1, a0, b0, a1, b1, x, y, d, e) \
  "v_add_f32 " a0 ", " m0 ", v20\n" "v_add_f32 " b0 ", " m0 ", v21\n" "v_add_f32 " a1 ", " m1 ", v21\n" "v_add_f32 " b1 ", " m1 ", v20\n" \
  "v_sub_f32 " x ", " a1 ", " a0 "\n" "v_sub_f32 " y ", " b1 ", " b0 "\n" "v_min_f32 " m0 ", " a0 ", " a1 "\n" "v_min_f32 " m1 ", " b0 ", " b1 "\n" \
  "v_alignbit_b32 " d ", " d ", " x ", 31\n" "v_alignbit_b32 " e ", " e ", " y ", 31\n"
// cross-lane state: 2 DPP adds (even / odd predecessor of the lane pair), min, sub, alignbit
#define XS(m, a0, a1, x, d) \
  "v_add_f32_dpp " a0 ", " m ", v20 quad_perm:[0,0,2,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n" \
  "v_add_f32_dpp " a1 ", " m ", v21 quad_perm:[1,1,3,3] row_mask:0xf bank_mask:0xf bound_ctrl:1\n" \
  "v_sub_f32 " x ", " a1 ", " a0 "\n" "v_min_f32 " m ", " a0 ", " a1 "\n" "v_alignbit_b32 " d ", " d ", " x ", 31\n"
// cross-lane state with ONE DPP move of the partner's metric and plain adds
#define XM(m, p, a0, a1, x, d) \
  "v_mov_b32_dpp " p ", " m " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n" \
  "v_add_f32 " a0 ", " m ", v20\n" "v_add_f32 " a1 ", " p ", v21\n" \
  "v_sub_f32 " x ", " a1 ", " a0 "\n" "v_min_f32 " m ", " a0 ", " a1 "\n" "v_alignbit_b32 " d ", " d ", " x ", 31\n"
// cross-lane state with the pair in lanes l and l + 32: one v_permlane32_swap of the metric and a
// copy gives the even (lower-half) and odd (upper-half) predecessor in every lane, then plain adds
#define XPMOV(m, t) "v_mov_b32 " t ", " m "\n"
#define XPST(m, t, a0, a1, x, d) \
  "v_permlane32_swap_b32 " m ", " t "\n" "v_add_f32 " a0 ", " m ", v20\n" "v_add_f32 " a1 ", " t ", v21\n" \
  "v_sub_f32 " x ", " a1 ", " a0 "\n" "v_min_f32 " m ", " a0 ", " a1 "\n" "v_alignbit_b32 " d ", " d ", " x ", 31\n"
#define XP4 XPMOV("v4", "v26") XPMOV("v5", "v27") XPMOV("v6", "v28") XPMOV("v7", "v29") \
  XPST("v4", "v26", "v8", "v9", "v12", "v16") XPST("v5", "v27", "v10", "v11", "v13", "v17") \
  XPST("v6", "v28", "v18", "v19", "v22", "v24") XPST("v7", "v29", "v14", "v15", "v23", "v25")
#define BF2 BF("v4", "v5", "v8", "v9", "v10", "v11", "v12", "v13", "v16", "v17") BF("v6", "v7", "v18", "v19", "v14", "v15", "v22", "v23", "v24", "v25")
#define XS4 XS("v4", "v8", "v9", "v12", "v16") XS("v5", "v10", "v11", "v13", "v17") XS("v6", "v18", "v19", "v22", "v24") XS("v7", "v14", "v15", "v23", "v25")
#define XM4 XM("v4", "v26", "v8", "v9", "v12", "v16") XM("v5", "v27", "v10", "v11", "v13", "v17") XM("v6", "v28", "v18", "v19", "v22", "v24") XM("v7", "v29", "v14", "v15", "v23", "v25")
#define SEL4 "v_cndmask_b32_e64 v20, v30, v31, s[4:5]\n" "v_cndmask_b32_e64 v21, v31, v30, s[4:5]\n" "v_cndmask_b32_e64 v20, v30, v31, s[4:5]\n" "v_cndmask_b32_e64 v21, v31, v30, s[4:5]\n"
K(k_bf, BF2 BF2)                        // 40 instructions
K(k_xs, XS4)                            // 20
K(k_xm, XM4)                            // 24
K(k_mix1of8, BF2 BF2 BF2 BF2 BF2 BF2 BF2 XS4 XS4)   // 7 in-lane : 1 cross (two-lane kernel): 140 + 40
K(k_mix2of8, BF2 BF2 BF2 XS4 XS4)       // 6 : 2 (four-lane kernel): 60 + 40
K(k_bfsel, BF2 BF2 SEL4)                // butterflies with per-lane selects: 44
K(k_xp, XP4)                            // 28
#define BF8 BF2 BF2 BF2 BF2
K(k_sparse, BF8 BF8 BF8 BF8 BF8 XS("v4", "v8", "v9", "v12", "v16"))   // 400 + 5: 2 DPP per 405
#define BF40 BF8 BF8 BF8 BF8 BF8
K(k_sparse1600, BF40 BF40 BF40 BF40 XS("v4", "v8", "v9", "v12", "v16"))   // 1600 + 5
// the same density with cross-lane moves through the LDS unit or the scalar unit instead of DPP
#define SWZ(m) "ds_swizzle_b32 v26, " m " offset:swizzle(QUAD_PERM,1,0,3,2)\n"
#define BPM(m) "ds_bpermute_b32 v27, v30, " m "\n"
#define RDL(m) "v_readlane_b32 s4, " m ", 5\n"
K(k_swz, BF40 SWZ("v4") "s_waitcnt lgkmcnt(0)\n")    // 400 + 2
K(k_bpm, BF40 BPM("v4") "s_waitcnt lgkmcnt(0)\n")    // 400 + 2
K(k_rdl, BF40 RDL("v4"))                             // 400 + 1
K(k_swz8, BF2 BF2 SWZ("v4") SWZ("v5") SWZ("v6") SWZ("v7") "s_waitcnt lgkmcnt(0)\n")   // 40 + 5
// one cross-lane instruction at the START of the kernel only, then the plain butterfly stream
__global__ __launch_bounds__(256) void k_rfl_start(float* o, int it) {
  asm volatile("v_readfirstlane_b32 s4, v4" ::: "s4");
  for (int i = 0; i < it; ++i) asm volatile(R8(BF2 BF2) ::: CLOB);
  if (it < 0) o[0] = 0;
}
__global__ __launch_bounds__(256) void k_dpp_start(float* o, int it) {
  asm volatile("v_add_f32_dpp v8, v4, v20 quad_perm:[0,0,2,2] row_mask:0xf bank_mask:0xf bound_ctrl:1" ::: "v8");
  for (int i = 0; i < it; ++i) asm volatile(R8(BF2 BF2) ::: CLOB);
  if (it < 0) o[0] = 0;
}
// the K = 7 persistent kernel's other instructions at its density (one 8-step chunk = ~1,600 VALU):
// 8 ds_read_b128 of the chunk rows and 8 LDS-DMA loads of the next chunk, per 1,600 VALU
__global__ __launch_bounds__(256) void k_bf_lds(float* o, int it) {
  __shared__ float4 buf[2048];
  const unsigned addr = (unsigned)(uintptr_t)buf + (threadIdx.x & 63) * 16;
  for (int i = 0; i < it; ++i) {
    asm volatile(R8(BF40 "ds_read_b128 v[26:29], %0\n") "s_waitcnt lgkmcnt(0)\n" :: "v"(addr) : CLOB);
  }
  if (it < 0) o[0] = buf[threadIdx.x].x;
}
__global__ __launch_bounds__(256) void k_bf_dma(float* o, int it) {
  __shared__ float4 buf[4096];
  const float* src = o + (threadIdx.x & 63) * 4;
  for (int i = 0; i < it; ++i) {
    for (int k = 0; k < 8; ++k)
      __builtin_amdgcn_global_load_lds(src + k * 256, (__attribute__((address_space(3))) void*)(buf + (threadIdx.x / 64) * 512 + k * 64), 16, 0, 0);
    asm volatile(R8(BF40) ::: CLOB);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (it < 0) o[0] = buf[threadIdx.x].x;
}
template <int NDMA, bool WAIT>
__global__ __launch_bounds__(256) void k_bf_dma_v(float* o, int it) {
  __shared__ float4 buf[4096];
  const float* src = o + (threadIdx.x & 63) * 4;
  for (int i = 0; i < it; ++i) {
    for (int k = 0; k < NDMA; ++k)
      __builtin_amdgcn_global_load_lds(src + k * 256, (__attribute__((address_space(3))) void*)(buf + (threadIdx.x / 64) * 512 + k * 64), 16, 0, 0);
    asm volatile(R8(BF40) ::: CLOB);
    if (WAIT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (it < 0) o[0] = buf[threadIdx.x].x;
}
// plain global loads into VGPRs at the same density (the data is consumed by an empty asm)
template <int NL>
__global__ __launch_bounds__(256) void k_bf_gload(float* o, int it) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const f4* src = reinterpret_cast<const f4*>(o) + (threadIdx.x & 63);
  f4 acc = {0, 0, 0, 0};
  for (int i = 0; i < it; ++i) {
    f4 v[NL];
#pragma unroll
    for (int k = 0; k < NL; ++k) v[k] = src[k * 64 + (i & 1)];
    asm volatile(R8(BF40) ::: CLOB);
#pragma unroll
    for (int k = 0; k < NL; ++k) asm volatile("" :: "v"(v[k]));
  }
  if (it < 0) o[0] = acc.x;
}
// a DPP add in a branch that never executes at run time (it < 0): a kernel that CONTAINS DPP
__global__ __launch_bounds__(256) void k_dead_dpp(float* o, int it) {
  for (int i = 0; i < it; ++i) {
    asm volatile(R8(BF2 BF2) ::: CLOB);
    if (it < 0) asm volatile(XS4 ::: CLOB);
  }
  if (it < 0) o[0] = 0;
}
K(k_mix1of8p, BF2 BF2 BF2 BF2 BF2 BF2 BF2 XP4 XP4)   // 140 + 56
int main() {
  float* d; (void)hipMalloc(&d, 1 << 20);
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  struct { const char* n; void (*k)(float*, int); double per; } ks[] = {
    {"butterflies (4 add 2 sub 2 min 2 alignbit)", k_bf, 40}, {"cross states, 2 DPP adds", k_xs, 20},
    {"cross states, DPP mov + 2 adds", k_xm, 24}, {"mix 7 in-lane : 1 cross (DPP adds)", k_mix1of8, 180},
    {"mix 6 in-lane : 2 cross (DPP adds)", k_mix2of8, 100}, {"butterflies + 10% cndmask_e64", k_bfsel, 44},
    {"cross states, mov + permlane32_swap + 2 adds", k_xp, 28}, {"mix 7 in-lane : 1 cross (permlane32)", k_mix1of8p, 196},
    {"butterflies + 2 DPP adds per 405 instructions", k_sparse, 405}, {"butterflies, DPP code never executed", k_dead_dpp, 40},
    {"butterflies + 2 DPP adds per 1605 instructions", k_sparse1600, 1605}, {"butterflies + 1 ds_swizzle per 402", k_swz, 402},
    {"butterflies + 1 ds_bpermute per 402", k_bpm, 402}, {"butterflies + 1 v_readlane per 401", k_rdl, 401},
    {"butterflies + 4 ds_swizzle per 45", k_swz8, 45}, {"butterflies, one v_readfirstlane at kernel start", k_rfl_start, 40},
    {"butterflies, one DPP add at kernel start", k_dpp_start, 40},
    {"butterflies + 1 ds_read_b128 per 400", k_bf_lds, 401}, {"butterflies + 8 LDS-DMA per 3,200", k_bf_dma, 400},
    {"butterflies + 8 LDS-DMA per 3,200, no wait", k_bf_dma_v<8, false>, 400},
    {"butterflies + 1 LDS-DMA per 3,200", k_bf_dma_v<1, true>, 400},
    {"butterflies + 16 LDS-DMA per 3,200", k_bf_dma_v<16, true>, 400},
    {"butterflies + 8 global_load_dwordx4 per 3,200", k_bf_gload<8>, 400}};
  const int it = 200, blocks = 256 * 4;
  for (int rep = 0; rep < 2; ++rep)
    for (auto& k : ks) {
      hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d, it);
      (void)hipEventRecord(a);
      hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d, it);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      const double per_instr = ms * 1e6 / (k.per * 8 * it * 4);   // 4 waves per SIMD
      printf("%-46s %.3f ns/instr/SIMD\n", k.n, per_instr);
    }
}
