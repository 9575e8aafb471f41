"""The bench.py line the driver parses (needs an MI355X): one JSON line on stdout with the contract's
fields and types -- metric / unit from BASELINE.json, value = whole-job decoded bits over the timed
steps, ms_per_step, the roofline object (bound, achieved, peak, unit, frac = achieved / peak, PMC
traffic) and the cpu_baseline object (value, unit, cores, kind, sample) -- on a small batch."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_line_contract():
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for k in ("MASTER_ADDR", "MASTER_PORT", "RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    frames, steps, warmup = 8, 3, 1
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", str(steps), "--warmup",
                        str(warmup), "--frames", str(frames), "--clock-warmup", "0.05", "--no-hbm-probe",
                        "--no-fused-channel", "--curve-frames", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = [ln for ln in r.stdout.strip().splitlines() if ln.strip()]
    assert len(out) == 1, "rank 0 prints exactly one line"
    line = json.loads(out[0])
    with open(os.path.join(REPO, "BASELINE.json")) as f:
        baseline = json.load(f)
    assert line["metric"] == baseline["metric"]
    assert line["unit"] == "Mbit/s"
    for key, typ in (("value", float), ("n_gpus", int), ("steps", int), ("warmup", int),
                     ("ms_per_step", float), ("higher_is_better", bool), ("scaling", str), ("dtype", str),
                     ("data", str), ("config", dict), ("roofline", dict), ("cpu_baseline", dict)):
        assert isinstance(line[key], typ), key
    assert "vs_baseline" in line
    assert line["n_gpus"] == 1 and line["steps"] == steps and line["warmup"] == warmup
    assert line["higher_is_better"] is True and line["scaling"] == "weak"
    assert "workload" in line["config"]
    bits = frames * 25000 * 40
    assert line["value"] == pytest.approx(bits / (line["ms_per_step"] * 1e-3) / 1e6, rel=0.01)
    roof = line["roofline"]
    for key in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert key in roof, key
    # derived from the committed PMC passes of the workload; none for this small batch
    assert roof["unit"] in ("GB/s", "TFLOP/s") and roof["bound"] in ("hbm", "mfma", "valu", "latency", None)
    assert roof["frac"] == pytest.approx(roof["achieved"] / roof["peak"], rel=1e-3)
    assert 0 < roof["frac"] < 1
    cpu = line["cpu_baseline"]
    for key in ("value", "unit", "cores", "kind", "sample"):
        assert key in cpu, key
    assert cpu["kind"] in ("reference", "port") and cpu["cores"] >= 1 and cpu["value"] > 0
