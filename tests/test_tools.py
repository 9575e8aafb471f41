"""CPU tests of the measurement tools' host logic: the paired f64 / f32 sweep comparison
(tools/noise_compare.py) and the bench line's HBM-ceiling and bound fields (bench.py)."""
import json
import os
import sys

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, REPO)

import noise_compare  # noqa: E402


def _rec(ebn0, errors, bits, mbit_s, blen=40):
    return {"code": "k7", "ebn0_db": ebn0, "blen": blen, "errors": errors, "bits": bits,
            "ber": errors / bits, "ber_99.9_binomial": [errors / bits * 0.99, errors / bits * 1.01],
            "mbit_s": mbit_s}


def test_noise_compare_paired_counts_pass_and_a_shift_fails(tmp_path):
    f64 = [_rec(10.0, 1000, 10**7, 100.0), _rec(12.0, 500, 10**7, 100.0)]
    same = [_rec(10.0, 1000, 10**7, 130.0), _rec(12.0, 500, 10**7, 131.0)]
    rows, ok = noise_compare.compare(f64, same)
    assert ok and all(r["inside_f64_binomial"] for r in rows)
    assert rows[0]["speedup"] == 1.3
    # a doubled error rate over 10^8 bits lies outside the burst-aware two-sample band
    f64 = [_rec(10.0, 10000, 10**8, 100.0), _rec(12.0, 5000, 10**8, 100.0)]
    shifted = [_rec(10.0, 20000, 10**8, 130.0), _rec(12.0, 5000, 10**8, 131.0)]
    rows, ok = noise_compare.compare(f64, shifted)
    assert not ok and not rows[0]["two_sample_ok"] and rows[1]["two_sample_ok"]
    a, b = tmp_path / "a.log", tmp_path / "b.log"
    a.write_text("noise line\n" + "\n".join(json.dumps(r) for r in f64) + "\n")
    b.write_text("\n".join(json.dumps(r) for r in same) + "\n")
    assert noise_compare.main(["x", str(a), str(b), str(tmp_path / "o.json")]) == 0
    assert json.load(open(tmp_path / "o.json"))["all_two_sample_ok"] is True


def test_hbm_ceiling_fields():
    import bench
    assert bench.hbm_ceiling_fields(None, 1e9, 0.5)["achievable_gbs"] is None
    f = bench.hbm_ceiling_fields({"copy": 5500.0, "read": 7000.0}, 2.625e9, 0.5)
    assert f["achievable_gbs"] == 7000.0
    assert abs(f["traffic_frac_of_achievable"] - 2.625e9 / 0.5e-3 / 1e9 / 7000.0) < 1e-4
    assert bench.HBM_PROBE_MIN_BYTES == 104 * 25000 * 46 * 16
    assert 0 < bench.LATENCY_BOUND_BELOW < 0.5


def test_pmc_calibration_uses_the_largest_copy_only(tmp_path):
    """The calibration copy's FETCH_SIZE / WRITE_SIZE scales come from the copy kernel's largest-grid
    dispatches only: a run also holds a 512-thread 1.6 KiB copy of the same kernel, and averaging it in
    read 2.67 / 1.33 instead of 2.00 / 1.00. Rows as rocprofv3 writes them."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import pmc_workload as P
    head = ('"Correlation_Id","Dispatch_Id","Agent_Id","Queue_Id","Process_Id","Thread_Id","Grid_Size",'
            '"Kernel_Id","Kernel_Name","Workgroup_Size","LDS_Block_Size","Scratch_Size","VGPR_Count",'
            '"Accum_VGPR_Count","SGPR_Count","Counter_Name","Counter_Value","Start_Timestamp","End_Timestamp"\n')
    copy_bytes = 1913600000

    def row(d, grid, kernel, counter, value):
        return f'{d},{d},"Agent 2",1,7,7,{grid},7,"{kernel}",512,0,0,8,0,32,"{counter}",{value},1,2\n'
    fetch = tmp_path / "f.csv"
    write = tmp_path / "w.csv"
    big_f = copy_bytes / 2 / 1024   # FETCH_SIZE counts half the bytes of a wide streaming read
    fetch.write_text(head + "".join(row(d, 131072, "__amd_rocclr_copyBuffer", "FETCH_SIZE", big_f) for d in (1, 2, 3))
                     + row(5, 512, "__amd_rocclr_copyBuffer", "FETCH_SIZE", 1.625)
                     + row(6, 2048, "ccv::viterbi_soft_persist", "FETCH_SIZE", 1.0e6))
    write.write_text(head + "".join(row(d, 131072, "__amd_rocclr_copyBuffer", "WRITE_SIZE", copy_bytes / 1024)
                                    for d in (1, 2, 3))
                     + row(5, 512, "__amd_rocclr_copyBuffer", "WRITE_SIZE", 1.625))
    cal = P.calibration(P.counter_rows([str(fetch)]), P.counter_rows([str(write)]), copy_bytes)
    assert abs(cal["read_scale"] - 2.0) < 1e-9 and abs(cal["write_scale"] - 1.0) < 1e-9
    assert cal["copies_averaged"] == [3, 3]
    # the committed records carry the rule's figures
    doc = json.load(open(os.path.join(REPO, "profiles", "pmc_workloads.json")))
    for key, rec in doc.items():
        c = rec.get("calibration") or {}
        if "copies_averaged" in c:
            assert abs(c["read_scale"] - 2.0) < 0.01 and abs(c["write_scale"] - 1.0) < 0.001, key
