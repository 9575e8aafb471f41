"""Compare two on-device AWGN sweeps of the same points: the double-precision Box-Muller (default) and
the opt-in fp32 one (--noise f32). Usage: noise_compare.py F64_LOG F32_LOG [OUT_JSON]

Both logs hold the JSON lines of `python -m ccviterbi.sim ... --device-channel [--noise f32]`. Per
point: the fp32 BER, whether it lies inside the f64 run's 99.9 % binomial interval, and the
two-sample rule of tests/test_gpu_ber.py (burst factor B = blen: |p32 - p64| <= 3.29 sqrt(B q (1-q)
(1/N32 + 1/N64))), plus the throughput ratio. With the same --seed both runs draw the same uniforms,
so their error counts are paired (they differ only where an fp32 sample crossed a decision the
double sample did not); the interval check is then the conservative reading.
"""
import json
import math
import sys


def _points(path):
    with open(path) as f:
        return [json.loads(line) for line in f if line.startswith("{")]


def compare(f64, f32):
    rows, ok = [], True
    for a, b in zip(f64, f32):
        assert a["ebn0_db"] == b["ebn0_db"] and a["code"] == b["code"], (a, b)
        q = (a["errors"] + b["errors"]) / (a["bits"] + b["bits"])
        tol = 3.29 * math.sqrt(a["blen"] * q * (1 - q) * (1 / a["bits"] + 1 / b["bits"]))
        lo, hi = a["ber_99.9_binomial"]
        row = {"code": a["code"], "ebn0_db": a["ebn0_db"], "bits": b["bits"], "errors_f64": a["errors"],
               "errors_f32": b["errors"], "ber_f64": a["ber"], "ber_f32": b["ber"],
               "inside_f64_binomial": lo <= b["ber"] <= hi, "two_sample_tol": tol,
               "two_sample_ok": abs(a["ber"] - b["ber"]) <= tol,
               "mbit_s_f64": a["mbit_s"], "mbit_s_f32": b["mbit_s"],
               "speedup": round(b["mbit_s"] / a["mbit_s"], 3) if a["mbit_s"] else None}
        ok &= row["two_sample_ok"]
        rows.append(row)
    return rows, ok


def main(argv):
    rows, ok = compare(_points(argv[1]), _points(argv[2]))
    for r in rows:
        print(f"{r['code']} {r['ebn0_db']:5.1f} dB  f64 {r['ber_f64']:.6g} ({r['errors_f64']})  "
              f"f32 {r['ber_f32']:.6g} ({r['errors_f32']})  in-binomial {r['inside_f64_binomial']}  "
              f"two-sample {r['two_sample_ok']}  {r['mbit_s_f64']:.0f} -> {r['mbit_s_f32']:.0f} Mbit/s "
              f"(x{r['speedup']})")
    if len(argv) > 3:
        with open(argv[3], "w") as f:
            json.dump({"points": rows, "all_two_sample_ok": ok}, f, indent=1)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv))
