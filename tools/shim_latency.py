#!/usr/bin/env python3
"""Per-block latency of the streaming decoder_input() path (the reference drivers' call pattern,
AWGN-channel/main.c:114, binary-symmetric-channel/main.c:70: one trellis step per call, the block
decoded and the callback fired inside the call that completes it).
MI355X rows: CCV_HOST_LATENCY=2 (default: the resident service kernel polling a host mailbox), 1 (a
generic-kernel launch per block on zero-copy staging), 0 (device staging + the register kernel).

Runs oracle/ref_harness_*_ccv (the reference drivers' producer chain linked to the MI355X shims) and
oracle/ref_harness_* (the same chain linked to the reference decoder) and reads `decoder_seconds`
(wall time inside decoder_input) from their .meta files.
usage: shim_latency.py [NBLOCKS] > table"""
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(REPO, "oracle", "_ref")
CASES = [("bsc", "cb:0", "25000", "config 1: BSC K=3 code 0"),
         ("awgn", "cb:0", "0.446154216921401", "AWGN K=3 code 0, 4 dB"),
         ("awgn", "2:7:40:f200000000000000:b600000000000000", "0.446154216921401", "AWGN K=7 (171,133), 4 dB"),
         ("bsc", "2:7:40:f200000000000000:b600000000000000", "50000", "BSC K=7 (171,133)")]


def run(exe, nblocks, param, spec, env=None):
    with tempfile.TemporaryDirectory() as tmp:
        prefix = os.path.join(tmp, "x")
        subprocess.run([exe, prefix, "7", str(nblocks), param, spec], check=True, env=env,
                       stdout=subprocess.DEVNULL, timeout=600)
        meta = dict(line.split() for line in open(prefix + ".meta"))
        out = open(prefix + ".out", "rb").read()
    return float(meta["decoder_seconds"]), int(meta["blocks_decoded"]), int(meta["blen"]), out


def main():
    nblocks = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    print(f"{'case':34s} {'decoder':34s} {'us/block':>9s} {'Mbit/s':>8s} identical")
    for chan, spec, param, name in CASES:
        t_ref, nb, blen, ref_out = run(os.path.join(REF, f"ref_harness_{chan}"), nblocks, param, spec)
        print(f"{name:34s} {'reference decoder (CPU, 1 thread)':34s} {t_ref / nb * 1e6:9.2f} "
              f"{nb * blen / t_ref / 1e6:8.2f} -")
        for mode, label in (("2", "MI355X shim, resident service"), ("1", "MI355X shim, launch per block"),
                            ("0", "MI355X shim, staged register")):
            env = dict(os.environ, CCV_HOST_LATENCY=mode)
            t, nb, blen, out = run(os.path.join(REF, f"ref_harness_{chan}_ccv"), nblocks, param, spec, env)
            print(f"{name:34s} {label:34s} {t / nb * 1e6:9.2f} {nb * blen / t / 1e6:8.2f} {out == ref_out}")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
