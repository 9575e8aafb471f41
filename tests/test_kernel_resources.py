"""Register budgets of the production kernels, read from the built gfx950 code objects (CPU only).

The persistent kernels are tuned to the register file: the K = 9 one-lane-per-block kernel
(acs_wide.hpp) holds ~156 value-numbered metrics in 252 of 256 VGPRs, the K <= 7 kernels keep 40
steps of decisions in VGPRs. A compiler change that spills them would keep every result bit-exact
and only show up as a slower bench -- this test catches it at build time instead: every persistent
kernel in lib/libccv_core.so must run without VGPR spills and without scratch memory.
"""
import os
import re
import shutil
import subprocess

import pytest

LLVM = "/opt/rocm/lib/llvm/bin"
LIB = os.path.join(os.path.dirname(__file__), "..", "convolutional-codes_amd", "lib", "libccv_core.so")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _kernel_metadata(tmp_path):
    """{kernel symbol: (vgpr_count, vgpr_spill_count, private_segment_fixed_size)} over every
    translation unit's gfx950 code object in the library's .hip_fatbin section."""
    fatbin = tmp_path / "fatbin.bin"
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fatbin}", LIB, str(tmp_path / "x.so")],
                   check=True, capture_output=True)
    data = fatbin.read_bytes()
    offs = [m.start() for m in re.finditer(re.escape(MAGIC), data)] + [len(data)]
    meta = {}
    for i in range(len(offs) - 1):
        bundle, co = tmp_path / f"b{i}.bin", tmp_path / f"c{i}.co"
        bundle.write_bytes(data[offs[i]:offs[i + 1]])
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={bundle}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
        if r.returncode:
            continue
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", str(co)], check=True, capture_output=True,
                               text=True).stdout
        for blk in notes.split("  - .agpr_count")[1:]:
            get = lambda k: int(re.search(rf"\.{k}:\s+(\d+)", blk).group(1))
            meta[re.search(r"\.name:\s+(\S+)", blk).group(1)] = (
                get("vgpr_count"), get("vgpr_spill_count"), get("private_segment_fixed_size"))
    return meta


@pytest.mark.skipif(not (os.path.exists(LIB) and shutil.which(f"{LLVM}/llvm-readelf")),
                    reason="needs the built library and the ROCm LLVM tools")
def test_persistent_kernels_do_not_spill(tmp_path):
    meta = _kernel_metadata(tmp_path)
    persistent = {k: v for k, v in meta.items() if "_persist" in k or "multi2_slot" in k}
    families = {f: [k for k in persistent if f in k] for f in
                ("viterbi_soft_persist", "viterbi_hard_persist", "viterbi_multi2_slot", "viterbi_wide_persist")}
    assert all(families.values()), {f: len(v) for f, v in families.items()}
    # the two-lane true-parity K = 9 kernel holds 256 VGPRs and spills one register outside its main
    # loop; every other persistent kernel spills nothing
    bad = {k: v for k, v in persistent.items()
           if ((v[1] > 1 or v[2] > 8) if "multi2_slot" in k else (v[1] or v[2]))}
    assert not bad, bad
    # the K = 9 one-lane kernel: two waves per SIMD (the launch bounds' waves_per_eu(2))
    assert all(v[0] <= 256 for k, v in persistent.items() if "wide_persist" in k)


def _code_objects(tmp_path):
    fatbin = tmp_path / "fatbin2.bin"
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fatbin}", LIB, str(tmp_path / "y.so")],
                   check=True, capture_output=True)
    data = fatbin.read_bytes()
    offs = [m.start() for m in re.finditer(re.escape(MAGIC), data)] + [len(data)]
    out = []
    for i in range(len(offs) - 1):
        bundle, co = tmp_path / f"d{i}.bin", tmp_path / f"e{i}.co"
        bundle.write_bytes(data[offs[i]:offs[i + 1]])
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={bundle}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
        if r.returncode == 0:
            out.append(co)
    return out


@pytest.mark.skipif(not (os.path.exists(LIB) and shutil.which(f"{LLVM}/llvm-objdump")),
                    reason="needs the built library and the ROCm LLVM tools")
def test_true_parity_k9_slot_kernels_have_no_cross_lane_valu(tmp_path):
    """On gfx950 one DPP / permlane VALU instruction halves a wave's VALU rate for hundreds of
    instructions; the production true-parity K = 9 kernel (two lanes per block) moves
    data between lanes only through ds_swizzle. A DPP or
    permlane instruction creeping back in (a compiler choice or an edit) keeps every result bit-exact
    and costs ~8 %: caught here."""
    found = {}
    for co in _code_objects(tmp_path):
        dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", str(co)], check=True, capture_output=True,
                             text=True).stdout
        for m in re.finditer(r"^[0-9a-f]+ <(\S+)>:\n(.*?)(?=^[0-9a-f]+ <|\Z)", dis, re.S | re.M):
            name, body = m.group(1), m.group(2)
            # viterbi_multi2_slot<C, 40, 7>
            if "viterbi_multi2_slot" in name:
                found[name] = len(re.findall(r"_dpp|\bdpp|permlane", body)), body.count("ds_swizzle")
    assert len(found) == 1, list(found)
    for name, (xlane, swz) in found.items():
        assert xlane == 0 and swz > 0, (name, xlane, swz)
