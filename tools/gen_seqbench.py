"""Generate tools/seqbench.hip: issue throughput of candidate ACS instruction sequences on gfx950.

Each kernel runs `it` iterations of 16 x 4 independent copies of one per-state ACS sequence (inline
asm, registers disjoint between the 4 copies); reported as ns per state per SIMD at W waves/SIMD.
"""
SEQS = {
    # current production: 2 adds + v_min_f32 + v_sub_f32 + v_alignbit
    "cur_min_sub_alignbit": ["v_add_f32 {a0}, {M0}, {B0}", "v_add_f32 {a1}, {M1}, {B1}",
                             "v_min_f32 {N}, {a0}, {a1}", "v_sub_f32 {t}, {a1}, {a0}",
                             "v_alignbit_b32 {D}, {D}, {t}, 31"],
    # unsigned order of non-negative floats: borrow -> vcc, select, add-with-carry shift-in
    "co_cnd_addc": ["v_add_f32 {a0}, {M0}, {B0}", "v_add_f32 {a1}, {M1}, {B1}",
                    "v_sub_co_u32 {t}, vcc, {a1}, {a0}", "v_cndmask_b32 {N}, {a0}, {a1}, vcc",
                    "v_addc_co_u32 {D}, vcc, {D}, {D}, vcc"],
    "min_co_addc": ["v_add_f32 {a0}, {M0}, {B0}", "v_add_f32 {a1}, {M1}, {B1}",
                    "v_min_f32 {N}, {a0}, {a1}", "v_sub_co_u32 {t}, vcc, {a1}, {a0}",
                    "v_addc_co_u32 {D}, vcc, {D}, {D}, vcc"],
    # float compare (exact for any input) -> vcc, select, add-with-carry
    "cmpf_cnd_addc": ["v_add_f32 {a0}, {M0}, {B0}", "v_add_f32 {a1}, {M1}, {B1}",
                      "v_cmp_lt_f32 vcc, {a1}, {a0}", "v_cndmask_b32 {N}, {a0}, {a1}, vcc",
                      "v_addc_co_u32 {D}, vcc, {D}, {D}, vcc"],
    "sub_ashr_bitop3x2": ["v_add_f32 {a0}, {M0}, {B0}", "v_add_f32 {a1}, {M1}, {B1}",
                          "v_sub_f32 {t}, {a1}, {a0}", "v_ashrrev_i32 {t}, 31, {t}",
                          "v_bitop3_b32 {N}, {t}, {a1}, {a0} bitop3:0xd8",
                          "v_bitop3_b32 {D}, {D}, {t}, 4 bitop3:0xf8"],
    "min_sub_lshr_add3": ["v_add_f32 {a0}, {M0}, {B0}", "v_add_f32 {a1}, {M1}, {B1}",
                          "v_min_f32 {N}, {a0}, {a1}", "v_sub_f32 {t}, {a1}, {a0}",
                          "v_lshrrev_b32 {t}, 31, {t}", "v_add3_u32 {D}, {D}, {D}, {t}"],
    "min_sub_lshr_lshladd": ["v_add_f32 {a0}, {M0}, {B0}", "v_add_f32 {a1}, {M1}, {B1}",
                             "v_min_f32 {N}, {a0}, {a1}", "v_sub_f32 {t}, {a1}, {a0}",
                             "v_lshrrev_b32 {t}, 31, {t}", "v_lshl_add_u32 {D}, {D}, 1, {t}"],
    # min + sub only (no packing): lower bound of the decision-free part
    "adds_min_sub": ["v_add_f32 {a0}, {M0}, {B0}", "v_add_f32 {a1}, {M1}, {B1}",
                     "v_min_f32 {N}, {a0}, {a1}", "v_sub_f32 {t}, {a1}, {a0}"],
    "adds_only": ["v_add_f32 {a0}, {M0}, {B0}", "v_add_f32 {a1}, {M1}, {B1}"],
    # single instructions (4 independent copies)
    "i_cndmask_e32": ["v_cndmask_b32 {N}, {a0}, {a1}, vcc"],
    "i_sub_co_e32": ["v_sub_co_u32 {t}, vcc, {a1}, {a0}"],
    "i_addc_e32": ["v_addc_co_u32 {D}, vcc, {M0}, {M1}, vcc"],
    "i_add3": ["v_add3_u32 {D}, {M0}, {M1}, {t}"],
    "i_min3_f32": ["v_min3_f32 {N}, {a0}, {a1}, {t}"],
    "i_minimum3_f32": ["v_minimum3_f32 {N}, {a0}, {a1}, {t}"],
    "i_cmp_lt_f32": ["v_cmp_lt_f32 vcc, {a1}, {a0}"],
    "i_cmp_lt_u32": ["v_cmp_lt_u32 vcc, {a1}, {a0}"],
    "i_bitop3_vvv": ["v_bitop3_b32 {N}, {t}, {a1}, {a0} bitop3:0xd8"],
    "i_ashr": ["v_ashrrev_i32 {t}, 31, {a0}"],
    "i_min_f16": ["v_min_f16 {N}, {a0}, {a1}"],
    "i_pk_add_f32": ["v_pk_add_f32 {P0}, {P1}, {P2}"],
    "i_add_u32_e64": ["v_add_u32_e64 {N}, {a0}, {a1}"],
    "i_mov": ["v_mov_b32 {N}, {a0}"],
    "i_min_u16": ["v_min_u16 {N}, {a0}, {a1}"],
    "i_max_i16": ["v_max_i16 {N}, {a0}, {a1}"],
    # pipe-mix probes: is a "half-rate" op hidden behind full-rate ones?
    "mix_add_min": ["v_add_f32 {a0}, {M0}, {B0}", "v_min_f32 {N}, {a1}, {t}"],
    "mix_min_min_add": ["v_min_f32 {N}, {a1}, {t}", "v_min_f32 {D}, {M1}, {B1}", "v_add_f32 {a0}, {M0}, {B0}"],
    "mix_pk_min": ["v_pk_add_f32 {P0}, {P1}, {P2}", "v_min_f32 {N}, {a1}, {t}"],
    "mix_pk_add": ["v_pk_add_f32 {P0}, {P1}, {P2}", "v_add_f32 {N}, {a1}, {t}"],
    "mix_pk_pk_min": ["v_pk_add_f32 {P0}, {P1}, {P2}", "v_pk_add_f32 {P3}, {P1}, {P2}", "v_min_f32 {N}, {a1}, {t}"],
    "mix_min_align_add": ["v_min_f32 {N}, {a1}, {t}", "v_alignbit_b32 {D}, {D}, {t}, 31", "v_add_f32 {a0}, {M0}, {B0}"],
    "mix_pk16_add": ["v_pk_add_u16 {N}, {a1}, {t}", "v_add_f32 {a0}, {M0}, {B0}"],
    "mix_pk16_min": ["v_pk_add_u16 {N}, {a1}, {t}", "v_min_f32 {a0}, {M0}, {B0}"],
    # butterfly (2 states) on packed f32 adds: P=(a0,b0), Q=(a1,b1), R=Q-P; 7 instrs / 2 states
    "bfly_pk_f32": ["v_pk_add_f32 {P3}, {PM}, {PB0} op_sel:[0,0] op_sel_hi:[0,1]",
                    "v_pk_add_f32 {P4}, {PM}, {PB1} op_sel:[1,0] op_sel_hi:[1,1]",
                    "v_pk_add_f32 {P5}, {P4}, {P3} neg_lo:[0,1] neg_hi:[0,1]",
                    "v_min_f32 {N}, {P3l}, {P4l}", "v_min_f32 {N2}, {P3h}, {P4h}",
                    "v_alignbit_b32 {D}, {D}, {P5l}, 31", "v_alignbit_b32 {D2}, {D2}, {P5h}, 31"],
    # same butterfly in scalar form (10 instrs / 2 states) for reference
    "bfly_scalar": ["v_add_f32 {a0}, {M0}, {B0}", "v_add_f32 {a1}, {M1}, {B1}",
                    "v_add_f32 {P3l}, {M0}, {B1}", "v_add_f32 {P3h}, {M1}, {B0}",
                    "v_min_f32 {N}, {a0}, {a1}", "v_sub_f32 {t}, {a1}, {a0}",
                    "v_min_f32 {N2}, {P3l}, {P3h}", "v_sub_f32 {P4l}, {P3h}, {P3l}",
                    "v_alignbit_b32 {D}, {D}, {t}, 31", "v_alignbit_b32 {D2}, {D2}, {P4l}, 31"],
    # 16-bit BSC butterfly, 2 metrics per VGPR: 4 packed + lshr + bitop3 = 6 instrs / 2 states
    "bfly_pk_u16": ["v_pk_add_u16 {a0}, {M0}, {B0} op_sel:[0,0] op_sel_hi:[0,1]",
                    "v_pk_add_u16 {a1}, {M0}, {B1} op_sel:[1,0] op_sel_hi:[1,1]",
                    "v_pk_min_u16 {N}, {a0}, {a1}", "v_pk_sub_i16 {t}, {a1}, {a0}",
                    "v_lshrrev_b32 {D}, 1, {D}", "v_bitop3_b32 {D}, {D}, {t}, s8 bitop3:0xf8"],
    # current 16-bit BSC state: add_u16 x2, min_u16, sub_u32, alignbit
    "cur_u16": ["v_add_u16 {a0}, {M0}, {B0}", "v_add_u16 {a1}, {M1}, {B1}", "v_min_u16 {N}, {a0}, {a1}",
                "v_sub_u32 {t}, {a1}, {a0}", "v_alignbit_b32 {D}, {D}, {t}, 31"],
}


NREG = 24


def regs(k):
    b = 8 + NREG * k
    names = ["M0", "M1", "B0", "B1", "a0", "a1", "N", "t", "D", "N2", "D2", "x"]
    r = {n: f"v{b + i}" for i, n in enumerate(names)}
    for i in range(6):
        r[f"P{i}"] = f"v[{b + 12 + 2 * i}:{b + 13 + 2 * i}]"
        r[f"P{i}l"] = f"v{b + 12 + 2 * i}"
        r[f"P{i}h"] = f"v{b + 13 + 2 * i}"
    r["PM"] = f"v[{b}:{b + 1}]"
    r["PB0"] = f"v[{b + 2}:{b + 3}]"
    r["PB1"] = f"v[{b + 4}:{b + 5}]"
    return r


def kernel(name, seq):
    lines = []
    for _ in range(16):
        for k in range(4):
            for ins in seq:
                lines.append(ins.format(**regs(k)))
    body = "\\n".join(lines)
    clob = ",".join(f'"v{i}"' for i in range(8, 8 + 4 * NREG)) + ',"vcc","s8"'
    return (f"__global__ __launch_bounds__(64) void k_{name}(float* o, int it) {{\n"
            f"  for (int i = 0; i < it; ++i) asm volatile(\"{body}\" ::: {clob});\n"
            f"  if (it < 0) o[0] = 0;\n}}\n")


def real_kernel(path):
    """The VALU stream of one compiled 8-step chunk of the production K=7 kernel (no memory ops)."""
    body = [l for l in open(path).read().split("\n") if l.strip()]
    asm = "\\n".join(body)
    clob = ",".join(f'"v{i}"' for i in range(0, 141))
    return (f"__global__ __launch_bounds__(64) void k_real_k7_chunk(float* o, int it) {{\n"
            f"  for (int i = 0; i < it; ++i) asm volatile(\"{asm}\" ::: {clob});\n"
            f"  if (it < 0) o[0] = 0;\n}}\n"), len(body)


def main():
    out = ["// generated by tools/gen_seqbench.py -- do not edit",
           "#include <hip/hip_runtime.h>", "#include <cstdio>", "#include <cstring>", "#include <cstdlib>", ""]
    for n, s in SEQS.items():
        out.append(kernel(n, s))
    import os
    extra = []
    if os.path.exists("/tmp/k7body.txt"):
        src, n = real_kernel("/tmp/k7body.txt")
        out.append(src)
        extra.append(f'{{"real_k7_chunk", {n}, k_real_k7_chunk}}')
    out.append("struct KB { const char* n; int len; void (*k)(float*, int); };")
    out.append("KB ks[] = {" + ",".join(f'{{"{n}", {len(s)}, k_{n}}}' for n, s in SEQS.items()) + "".join("," + e for e in extra) + "};")
    out.append(r'''
int main(int argc, char** argv) {
  const char* filt = argc > 1 ? argv[1] : "";
  float* d; hipMalloc(&d, 4096);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const int it = argc > 2 ? atoi(argv[2]) : 2000;
  for (int w : {1, 2, 3, 4}) {
    for (auto& k : ks) {
      if (!strstr(k.n, filt)) continue;
      const int grid = 1024 * w;
      float best = 1e9f;
      for (int r = 0; r < 4; ++r) {
        hipEventRecord(a); hipLaunchKernelGGL(k.k, dim3(grid), dim3(64), 0, 0, d, it); hipEventRecord(b);
        hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms, a, b);
        if (r > 0 && ms < best) best = ms;
      }
      // per SIMD: w waves x it x 64 states; ns per state and per instruction
      const double states = (double)w * it * 64;
      printf("W=%d %-24s %6.3f ns/state/SIMD  %5.2f ns/instr\n", w, k.n, best * 1e6 / states,
             best * 1e6 / states / k.len);
    }
  }
}
''')
    open("tools/seqbench.hip", "w").write("\n".join(out))


if __name__ == "__main__":
    main()
