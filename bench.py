#!/usr/bin/env python3
"""Benchmark of the MI355X Viterbi decoder on BASELINE.json's headline workload.

Metric (BASELINE.json): decoded Mbit/s (+ BER at the simulated Eb/N0) of K=7 r=1/2 soft-decision
Viterbi on 1/2/4/8 MI355X. One "step" = one pass of the decoder (branch metrics + ACS + traceback
+ fused bit-error count) over one batch of FRAMES_PER_STEP synthetic 1 M-bit frames (25,000
zero-tail blocks of 40 info bits each, the demapped AWGN channel output at 4 dB, generated once on
the host with the reference's channel arithmetic and then resident in HBM). One process per GPU;
frames are sharded across ranks (weak scaling), no collective on the data path.

    python bench.py [--gpus N --steps K --warmup W]

N > 1: one process per GPU. Started as `python bench.py --gpus N` the script re-launches itself under
torch.distributed.run (ccviterbi/launch.py: a child process, before anything touches the GPU); started
by torch.distributed.run it reads RANK / LOCAL_RANK / WORLD_SIZE. Prints ONE JSON line on rank 0.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "convolutional-codes_amd"))

FRAME_BLOCKS = 25000          # 25,000 x 40 bits = 1 M-bit frame
HBM_PEAK_GBS = 8000.0         # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "decoded Mbit/s + BER vs Eb/N0, K=7 r=1/2 soft Viterbi @1/2/4/8 MI355X"


def algorithmic_bytes_per_bit(code, soft=True, decisions=True):
    """B = [T*(in_step_bytes + S/8) + ceil(blen/8)] / blen bytes per info bit
    (input stream + packed survivor decisions + decoded output). The stack decoder keeps no
    decisions: B = [T*in_step_bytes + ceil(blen/8)] / blen."""
    step_in = (4 << code.n) if soft else 1
    dec = code.states / 8.0 if decisions else 0.0
    return (code.steps * (step_in + dec) + code.info_bytes) / code.blen


def _cgroup_cpu_quota():
    """CPUs granted by the cgroup v2 quota (cpu.max), or None when unlimited / unreadable."""
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            return max(1, int(int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    return None


def host_cpu_info():
    """What the host offers this process: nproc, the affinity mask, the cgroup quota, the CPU model
    and the CPU share the pool grants (OMP_NUM_THREADS: 16 per GPU on the MI355X boxes)."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    return {"nproc": os.cpu_count() or 1, "affinity": affinity, "cgroup_quota": _cgroup_cpu_quota(),
            "omp_num_threads": int(env) if env and env.isdigit() else None, "model": model}


def cpu_threads(info=None):
    """Every host core this process may use: the affinity mask, capped by the cgroup quota and by the
    pool's per-GPU CPU share (OMP_NUM_THREADS) where set."""
    info = info or host_cpu_info()
    n = info["affinity"]
    for cap in (info["cgroup_quota"], info["omp_num_threads"]):
        if cap:
            n = min(n, cap)
    return max(1, n)


def reference_cannot_decode(code, decoder="viterbi"):
    """Why the reference decoder cannot run this code, or None. Its Viterbi argmin counts states in a
    uint8_t (`for (uint8_t i = 0; i < obj->num_states; ++i)`, AWGN-channel/viterbi-decoder.c:74,
    binary-symmetric-channel/viterbi-decoder.c:78), so at 2^(K-1) >= 256 states (K >= 9) the loop never
    ends: calling it would hang bench.py."""
    if decoder == "viterbi" and code.K >= 9:
        return (f"reference Viterbi not run: K={code.K} has {code.states} states and its uint8_t argmin "
                "counter never reaches them (AWGN-channel/viterbi-decoder.c:74 loops forever)")
    if code.gen_mode != 0:
        return ("reference not run: compiled here it decodes the x86-idiom code of its generator-bit "
                "expression (common/encoder.c:95-100, SURVEY.md 0.4), not the textbook true-parity code")
    return None


def cpu_baseline(code, rx, gpu_out, target_cpu_seconds, decoder="viterbi", hard=False):
    """Reference decoder (oracle/_ref, compiled from the reference's own sources) on host cores,
    over a bounded sample of the SAME frames the GPU decodes; its output is checked against the GPU's.
    Falls back to the oracle restatement ("port", one thread) where oracle/_ref was not built or the
    reference cannot decode the code (K >= 9, reference_cannot_decode)."""
    stack = decoder == "stack"
    suffix = "" if decoder == "viterbi" else "_" + decoder
    ref_so = os.path.join(REPO, "oracle", "_ref", f"libccref_{'bsc' if hard else 'awgn'}{suffix}.so")
    polys = (ctypes.c_uint64 * code.n)(*code.polys)
    skipped = reference_cannot_decode(code, decoder)
    if not os.path.exists(ref_so) and skipped is None:
        skipped = f"{os.path.relpath(ref_so, REPO)} not built"
    if skipped is None:
        lib = ctypes.CDLL(ref_so)
        if decoder != "viterbi":
            lib.ccref_set_stack_metrics.argtypes = [ctypes.c_float, ctypes.c_int32, ctypes.c_int32]
            if stack:
                lib.ccref_set_stack_metrics(code.metric_weight, *code.bit_metrics)
            else:
                lib.ccref_set_stack_metrics(code.fano_metric_weight, *code.fano_bit_metrics)
        lib.ccref_decode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        lib.ccref_decode.restype = ctypes.c_double
        threads = cpu_threads()

        def run(nb, nthr):
            sample = np.ascontiguousarray(rx[:nb])
            out = np.zeros((nb, code.out_bytes), np.uint8)
            t = lib.ccref_decode(code.n, code.K, code.blen, polys, sample.ctypes.data, nb,
                                 out.ctypes.data, None, nthr)
            if t < 0:
                raise RuntimeError("reference decode failed")
            return t, out
        kind = "reference"
    else:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_ctypes as O
        oc = O.code(code.n, code.K, code.blen, code.polys, code.gen_mode)
        threads = 1

        def run(nb, nthr):
            t0 = time.perf_counter()
            if hard:
                fn = {"stack": lambda: O.stack_hard(oc, code.bit_metrics, rx[:nb]),
                      "fano": lambda: O.fano_hard(oc, code.fano_bit_metrics, rx[:nb])}.get(
                          decoder, lambda: O.viterbi_hard(oc, rx[:nb]))
                out = fn()[0]
            elif decoder == "stack":
                out = O.stack_soft(oc, code.metric_weight, rx[:nb])
            elif decoder == "fano":
                out = O.fano_soft(oc, code.fano_metric_weight, rx[:nb])
            else:
                out = O.viterbi_soft(oc, rx[:nb])
            return time.perf_counter() - t0, out
        kind = "port"
    t_cal, _ = run(200, 1)                      # calibrate: seconds per block on one core
    per_block = max(t_cal / 200, 1e-7)
    nb = int(min(len(rx), max(threads * 200, target_cpu_seconds / per_block)))
    nb -= nb % threads
    secs, out = run(nb, threads)
    parity = bool(np.array_equal(out, gpu_out[:nb]))
    if stack and not parity and kind == "reference":
        # each reference thread is a fresh decoder, while the GPU batch continues one decoder's
        # streaming context; a stack search that overtakes the frontier reads that context, so the
        # first block of each thread's share may legitimately differ -- compare the rest
        per, extra = nb // threads, nb % threads
        starts, first = set(), 0
        for t in range(threads):
            starts.add(first)
            first += per + (1 if t < extra else 0)
        diff = set(np.nonzero((out != gpu_out[:nb]).any(axis=1))[0].tolist())
        parity = diff <= starts
    bits = nb * code.blen
    host = host_cpu_info()
    how = ("one decoder_input() per trellis step as the reference driver feeds it" if kind == "reference"
           else "oracle/ccoracle.c, the cited restatement of the reference decoder (same loop shape and "
                "tie rules)")
    res = {"value": round(bits / secs / 1e6, 4), "unit": "Mbit/s", "cores": threads, "kind": kind,
           "sample": f"{nb} blocks ({bits} info bits) of the benchmark frames, {secs:.2f} s wall on "
                     f"{threads} thread(s), {how}; output bit-identical to the GPU's: {parity}",
           "bit_identical": parity, "host": host}
    if skipped:
        res["reference_skipped"] = skipped
    return res, parity


def cpu_optimized_baseline(code, rx, gpu_out, target_cpu_seconds, hard=False):
    """oracle/ccfast.c -- a table-driven Viterbi vectorised over 8 (soft) / 16 (hard) blocks in AVX2
    lanes, one pthread per host core, bit-identical to the reference -- over a bounded sample of the
    same frames: the CPU baseline a tuned CPU implementation would give."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ctypes as O
    oc = O.code(code.n, code.K, code.blen, code.polys, code.gen_mode)
    threads = cpu_threads()
    res = O.fast_viterbi(oc, rx[:2000], hard=hard, threads=1)
    per_block = max(res[0] / 2000, 1e-8)
    nb = int(min(len(rx), max(threads * 2000, target_cpu_seconds * threads / per_block)))
    # one pass over the sample can be a fraction of a second at K <= 7 (2.6 M blocks ~ 0.1-0.2 s), so
    # repeat passes until at least min_seconds of wall time and report the MEDIAN pass (a single short
    # pass swung 2x between runs)
    min_seconds, times, out = 2.0, [], None
    while sum(times) < min_seconds or len(times) < 5:
        res = O.fast_viterbi(oc, rx[:nb], hard=hard, threads=threads)
        times.append(res[0])
        if out is None:
            out = res[1]
        if len(times) >= 200:
            break
    secs = sorted(times)[len(times) // 2]
    parity = bool(np.array_equal(out, gpu_out[:nb]))
    bits = nb * code.blen
    return {"value": round(bits / secs / 1e6, 2), "unit": "Mbit/s", "cores": threads, "kind": "port",
            "sample": f"{nb} blocks ({bits} info bits) of the benchmark frames per pass, median of "
                      f"{len(times)} passes ({sum(times):.2f} s wall in total; passes "
                      f"{min(times):.3f}-{max(times):.3f} s) on {threads} thread(s): oracle/ccfast.c, "
                      f"table-driven ACS on 8/16 blocks per AVX2 vector; output bit-identical to the GPU's: "
                      f"{parity}",
            "passes": len(times), "pass_seconds_median": round(secs, 4),
            "bit_identical": parity}


def load_pmc(workload_key):
    """Per-launch PMC figures of this workload's dominant kernel from the committed rocprofv3 passes
    (profiles/pmc_workloads.json, written by tools/pmc_workload.py): HBM bytes (FETCH_SIZE and
    WRITE_SIZE passes, FETCH_SIZE x 2 and WRITE_SIZE x 1 as MI355X_MICROARCH.md prescribes for gfx950;
    a device copy in the same run is recorded as a cross-check), SQ_INSTS_VALU and GRBM_GUI_ACTIVE.
    {} if absent."""
    path = os.path.join(REPO, "profiles", "pmc_workloads.json")
    try:
        with open(path) as f:
            return json.load(f).get(workload_key, {})
    except (OSError, ValueError):
        return {}


def pmc_for_variant(pmc, variant):
    """The PMC record only if it was taken on the kernel this plan runs (a record of another kernel
    for the same workload key -- e.g. the K = 9 four-lane kernel before the one-lane-per-block one --
    is stale and reported as unmeasured)."""
    kernel = pmc.get("kernel", "")
    if not kernel:
        return pmc
    if variant == "persistent-wide":
        return pmc if "viterbi_wide_persist" in kernel else {}
    if variant == "persistent-slot2":
        return pmc if "viterbi_multi2_slot" in kernel else {}
    if variant == "persistent":
        return pmc if "_persist<" in kernel and "wide" not in kernel else {}
    return pmc


def valu_fraction(pmc):
    """Issued VALU wave-instructions over the chip's issue capacity in the same cycles: a wave64 VALU
    instruction issues over 2 cycles on a 32-lane CDNA4 SIMD (MI355X_MICROARCH.md), so 1,024 SIMDs
    issue at most 512 per cycle; GRBM_GUI_ACTIVE is the busy cycles summed over the 8 XCDs."""
    valu, grbm = pmc.get("sq_insts_valu"), pmc.get("grbm_gui_active")
    if not valu or not grbm:
        return None
    return valu / (512.0 * grbm / 8.0)


# PMC byte scales (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of a wide
# coalesced read on gfx950, WRITE_SIZE the exact bytes of 16-byte-per-lane stores.
PMC_FETCH_SCALE, PMC_WRITE_SCALE = 2.0, 1.0
def pmc_scale_note(cal):
    """How the PMC byte scales were chosen, with the in-run calibration they are checked against."""
    if not cal or "read_scale" not in cal:
        return "FETCH_SIZE x 2, WRITE_SIZE x 1 as the guide prescribes for gfx950 (no in-run calibration copy)"
    return (f"FETCH_SIZE x 2, WRITE_SIZE x 1 as the guide prescribes for gfx950; the PMC run's own device copy "
            f"of {cal['copy_bytes']} B (largest-grid copy dispatches, tools/pmc_workload.py calibration) reads "
            f"{cal['read_scale']:.3f} / {cal['write_scale']:.3f}")


HBM_PROBE_MIN_BYTES = 104 * 25000 * 46 * 16   # the headline's input batch, 1.91 GB
LATENCY_BOUND_BELOW = 0.35   # roofline.bound "latency" when both measured fractions are below this


def measure_hbm_ceiling(d_buf, stream, reps=5):
    """Achievable HBM rates on this box: ccv_hbm_probe's streaming copy of d_buf (read + write bytes)
    and its read-only stream of d_buf, each the best of `reps` HIP-event-timed launches on `stream`
    after one untimed launch. GB/s. A batch smaller than the headline's (hard input, few frames) is
    replaced by a random buffer of the headline's 1.91 GB: on a small buffer the launch overhead and
    ramp, not the HBM, set the rate (a 18 MB batch streams at ~4.3 TB/s)."""
    import torch
    from ccviterbi import _native
    L = _native.core()
    nbytes = d_buf.numel() * d_buf.element_size() // 16 * 16
    if nbytes < HBM_PROBE_MIN_BYTES:
        d_buf = torch.randint(0, 256, (HBM_PROBE_MIN_BYTES,), dtype=torch.uint8, device=d_buf.device)
        nbytes = HBM_PROBE_MIN_BYTES
    dst = torch.empty(nbytes, dtype=torch.uint8, device=d_buf.device)
    sink = torch.zeros(1, dtype=torch.int32, device=d_buf.device)
    out = {}
    for mode, name, moved in ((0, "copy", 2 * nbytes), (1, "read", nbytes)):
        def launch():
            if L.ccv_hbm_probe(mode, dst.data_ptr(), d_buf.data_ptr(), nbytes, sink.data_ptr(),
                               stream.cuda_stream) != 0:
                raise RuntimeError(_native.last_error())
        launch()
        best = None
        for _ in range(reps):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record(stream)
            launch()
            ev[1].record(stream)
            torch.cuda.synchronize()
            ms = ev[0].elapsed_time(ev[1])
            best = ms if best is None else min(best, ms)
        out[name] = moved / (best * 1e-3) / 1e9
    del dst
    return out


def hbm_ceiling_fields(probe, traffic, kernel_ms):
    """Roofline fields from the measured ceiling: the achievable rate is the faster of the probe's
    copy and read streams; traffic_frac_of_achievable = the kernel's PMC traffic rate over it."""
    if not probe:
        return {"hbm_copy_gbs": None, "hbm_read_gbs": None, "achievable_gbs": None,
                "traffic_frac_of_achievable": None}
    ach = max(probe["copy"], probe["read"])
    return {"hbm_copy_gbs": round(probe["copy"], 1), "hbm_read_gbs": round(probe["read"], 1),
            "achievable_gbs": round(ach, 1),
            "achievable_basis": "max of ccv_hbm_probe copy (read+write bytes) and read-only stream over "
                                "the input batch (at least 1.91 GB), best of 5, this run",
            "traffic_frac_of_achievable": (round(traffic / (kernel_ms * 1e-3) / 1e9 / ach, 4)
                                           if traffic else None)}


def reduce_over_ranks(dist, wall, kernel_ms, errors, device):
    """The only exchange of the sharded bench: MAX of the wall and kernel times, SUM of the bit-error
    counters (one RCCL all-reduce each over xGMI, or gloo on CPU) and an all-gather of every rank's
    kernel time. Returns (wall, kernel_ms, per_rank_kernel_ms, errors)."""
    import torch
    world = dist.get_world_size()
    t = torch.tensor([wall, kernel_ms], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    e = torch.tensor([int(errors)], dtype=torch.int64, device=device)
    dist.all_reduce(e, op=dist.ReduceOp.SUM)
    per = [torch.zeros(1, dtype=torch.float64, device=device) for _ in range(world)]
    dist.all_gather(per, torch.tensor([kernel_ms], dtype=torch.float64, device=device))
    return float(t[0]), float(t[1]), [round(float(x.item()), 4) for x in per], int(e.item())


def init_group(dist, torch, backend, world, device_index):
    """The process group of this run. N > 1: the ranks torch.distributed.run started. N = 1 with an
    explicit --backend: a world-size-1 group (127.0.0.1, a free port), so the exact collectives of an
    N-GPU run -- the MAX / SUM all-reduces, the all-gather and the barriers, over RCCL on cuda with
    nccl -- execute on a one-GPU box too. Returns the RCCL version string (nccl) or None."""
    from ccviterbi import launch
    if world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(launch.free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", device_index))
        v = torch.cuda.nccl.version()
        return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    dist.init_process_group("gloo")
    return None


def ber_curve(code, hard, frames, seed, rank, world, dist=None, device="cuda", noise=("f64",),
              decode=None, frame_blocks=FRAME_BLOCKS, threads=None):
    """The BER-vs-Eb/N0 half of the metric: the reference's sweep points (AWGN-channel/main.c:150-161:
    Eb/N0 0..14 dB; BSC: binary-symmetric-channel/main.c:103-109), `frames` 1 M-bit frames per rank
    per point, sharded as the sweep CLI shards them (contiguous frame ranges of each point's Philox
    stream, sim.shard) and generated on the GPU (the on-device channel, sim.DeviceChannelDecoder) --
    or decoded by `decode(info, data)` (tests: the oracle under gloo). One SUM all-reduce of the
    [point][errors, bits] table and one MAX of the sweep time per noise mode. Returns
    {mode: {"points": [...], "seconds", "gbit_s"}}."""
    import torch
    from ccviterbi import HARD, SOFT, channel as ch, sim
    chan = HARD if hard else SOFT
    points = list(ch.REFERENCE_P_PPM if hard else ch.REFERENCE_EBN0_DB)
    bits_per_point = world * frames * frame_blocks * code.blen
    curves = {}
    for nz in (("bsc",) if hard else noise):
        dev = None
        if decode is None:
            dev = sim.DeviceChannelDecoder(code, chan, frame_blocks, seed, noise_f32=nz == "f32",
                                           chunk_blocks=frames * frame_blocks)
            dev.warm_up(0.05, points[0])
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        pts = sim.ber_sweep(code, points, chan, bits_per_point=lambda p: bits_per_point,
                            frame_blocks=frame_blocks, seed=seed, rank=rank, world=world, decode=decode,
                            reduce=False, device_decoder=dev, threads=threads)
        secs = time.perf_counter() - t0
        counters = np.array([[pt.errors, pt.bits] for pt in pts], np.int64)
        if dist is not None:
            counters = sim.all_reduce_counters(counters)
            t = torch.tensor([secs], dtype=torch.float64, device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            secs = float(t.item())
        key = "p_ppm" if hard else "ebn0_db"
        curves[nz] = {
            "points": [{key: p, "errors": int(e), "bits": int(b), "ber": (int(e) / int(b)) if b else None}
                       for p, (e, b) in zip(points, counters)],
            "seconds": round(secs, 4),
            "gbit_s": round(int(counters[:, 1].sum()) / secs / 1e9, 2) if secs > 0 else None,
        }
    return curves


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--code", default=None,
                    help="k7 (default), k9, k15 (stack default), code0..code5; suffix :true = true parity")
    ap.add_argument("--decoder", choices=("viterbi", "stack", "fano"), default="viterbi",
                    help="viterbi (BASELINE configs 1-4), the stack decoder (config 5, K=15) or Fano")
    ap.add_argument("--frames", type=int, default=104,
                    help="1 M-bit frames per GPU per step. 104 = 2.6 M blocks = 40,625 groups of 64 "
                         "blocks for the 2,048 resident waves of the persistent K=7 kernel: 19.8 groups "
                         "each, so the last, partial round of groups idles <1%% of the waves (64 frames: "
                         "12.2 groups each, 6%%)")
    ap.add_argument("--ebn0", type=float, default=4.0)
    ap.add_argument("--channel", choices=("awgn", "bsc"), default="awgn",
                    help="awgn: soft decision (configs 2, 3, 5); bsc: hard decision (configs 1, 4)")
    ap.add_argument("--p-ppm", type=int, default=50000, help="BSC crossover probability in ppm")
    ap.add_argument("--layout", choices=("block", "step"), default="block",
                    help="input layout in HBM: block-major [nb][T][4] as the reference decoder consumes "
                         "it, or step-major [T][nb][4] (CCV_FLAG_STEP_MAJOR)")
    ap.add_argument("--decisions", choices=("register", "hbm"), default="register",
                    help="register: survivor decisions stay in VGPRs where the kernel allows it (K <= 7, "
                         "r = 1/2, T <= 48); hbm: force the decision scratch array in HBM (A/B)")
    ap.add_argument("--persistent", choices=("on", "off"), default="on",
                    help="on: the persistent K <= 7 kernels where they apply (blen 40); off: the "
                         "one-wave-per-64-blocks kernels (A/B, CCV_FLAG_NO_PERSISTENT)")
    ap.add_argument("--clock-warmup", type=float, default=0.3,
                    help="seconds of untimed decode launches before the W warmup steps: a cold MI355X "
                         "needs ~40 ms of continuous load to reach its sustained clock (per-launch times "
                         "fall from 0.51 to 0.33 ms over the first ~80 launches, profiles/r02_clock_ramp.txt)")
    ap.add_argument("--no-error-count", action="store_true",
                    help="decode without the fused bit-error count (A/B of its cost; no BER reported)")
    ap.add_argument("--seed", type=int, default=0xC0DE)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU-baseline work budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="plan option (ccv_plan_set_option, include/ccv.h) for A/B runs; repeatable")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default=None,
                    help="process-group backend for N > 1 (default nccl = RCCL over xGMI); given at N = 1 "
                         "it forces a world-size-1 group, so the N-GPU collectives run on one GPU")
    ap.add_argument("--step-events", choices=("on", "off"), default="off",
                    help="off (default): one HIP event pair around the K timed steps on the decode stream "
                         "(kernel_ms = its time / K, the ~1 us launch gaps included); on: a pair around "
                         "every step as in rounds 1-5 -- the event records cost ~5 us per step "
                         "(profiles/r06_events: 208.6 vs 210.3 Gbit/s)")
    ap.add_argument("--curve-frames", type=int, default=None,
                    help="1 M-bit frames per rank per point of the BER-vs-Eb/N0 curve run after the timed "
                         "region (default: --frames, one launch per point); 0 = no curve")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal on a one-GPU box: every rank on cuda:0, reductions over gloo")
    ap.add_argument("--no-hbm-probe", action="store_true",
                    help="skip the achievable-HBM probe (A/B runs of builds that predate it)")
    ap.add_argument("--no-fused-channel", action="store_true",
                    help="skip the informational on-device channel + decode measurement")
    args = ap.parse_args(argv)

    # --gpus N > 1 without a launcher: start N ranks under torch.distributed.run as a child process,
    # before torch (let alone HIP) is touched here
    from ccviterbi import launch
    if launch.needs_launch(args.gpus):
        return launch.relaunch(args.gpus, os.path.abspath(__file__),
                               sys.argv[1:] if argv is None else list(argv))
    rank, local_rank, world = launch.world_from_env()
    launch.check_world(args.gpus, world)

    import torch
    import torch.distributed as dist

    from ccviterbi import HARD, SOFT, FanoPlan, Plan, StackPlan, channel as ch, named_code
    from ccviterbi.decoder import FLAG_GLOBAL_DECISIONS, FLAG_NO_PERSISTENT, FLAG_STEP_MAJOR

    # --same-device (a multi-process rehearsal on a one-GPU box): every rank on cuda:0, the
    # reductions over gloo (RCCL refuses two ranks on one device); the production form is one rank
    # per GPU over RCCL
    device_index = 0 if args.same_device else local_rank
    backend = args.backend or ("gloo" if args.same_device else "nccl")
    torch.cuda.set_device(device_index)
    use_pg = world > 1 or args.backend is not None
    rccl_version = init_group(dist, torch, backend, world, device_index) if use_pg else None

    stack = args.decoder == "stack"
    sequential = args.decoder != "viterbi"
    if args.code is None:
        args.code = "k15" if sequential else "k7"
    if sequential and args.layout != "block":
        raise SystemExit("the sequential decoders read block-major input")
    code = named_code(args.code)
    nb = args.frames * FRAME_BLOCKS
    # this rank's frames: blocks [rank*nb, (rank+1)*nb) of the Philox stream
    hard = args.channel == "bsc"
    if hard and args.layout != "block":
        raise SystemExit("hard-decision input is one byte per step, block-major")
    chan = HARD if hard else SOFT
    t_prod = time.perf_counter()
    if hard:
        info, rx = ch.bsc_blocks(code, nb, args.p_ppm, args.seed, first_block=rank * nb,
                                 threads=cpu_threads())
    else:
        info, rx = ch.awgn_blocks(code, nb, ch.noise_scaling(args.ebn0), args.seed, first_block=rank * nb,
                                  threads=cpu_threads())
    t_prod = time.perf_counter() - t_prod
    host_in = rx if args.layout == "block" else np.ascontiguousarray(rx.transpose(1, 0, 2))
    d_rx = torch.from_numpy(host_in).to("cuda")
    d_info = torch.from_numpy(info).to("cuda")
    d_out = torch.empty((nb, code.out_bytes), dtype=torch.uint8, device="cuda")
    d_err = torch.zeros(1, dtype=torch.int64, device="cuda")
    if args.decoder == "stack":
        plan = StackPlan(code, chan)
    elif args.decoder == "fano":
        plan = FanoPlan(code, chan)
    else:
        plan = Plan(code, chan, (FLAG_STEP_MAJOR if args.layout == "step" else 0) |
                    (FLAG_GLOBAL_DECISIONS if args.decisions == "hbm" else 0) |
                    (FLAG_NO_PERSISTENT if args.persistent == "off" else 0))
    for opt in args.option:
        name, value = opt.split("=", 1)
        plan.set_option(name, int(value))
    plan.reserve(nb)
    stream = torch.cuda.current_stream()

    def step():
        if args.no_error_count:
            plan.decode_device(d_rx, nb, d_out, stream=stream)
        else:
            plan.decode_device(d_rx, nb, d_out, d_info=d_info, d_errors=d_err, stream=stream)

    # bring the GPU to its sustained clock (untimed), then the W warmup steps
    t_warm = time.perf_counter()
    while time.perf_counter() - t_warm < args.clock_warmup:
        for _ in range(10):
            step()
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    d_err.zero_()
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ev_all = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    if use_pg:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev_all[0].record(stream)
    for k in range(args.steps):
        if args.step_events == "on":
            starts[k].record(stream)
        step()
        if args.step_events == "on":
            ends[k].record(stream)
    ev_all[1].record(stream)
    torch.cuda.synchronize()
    if use_pg:
        dist.barrier()
    wall = time.perf_counter() - t0
    steps_ms = ev_all[0].elapsed_time(ev_all[1])   # device time of the K timed steps, gaps included
    if args.step_events == "on":
        step_ms = sorted(s.elapsed_time(e) for s, e in zip(starts, ends))
        kernel_ms = sum(step_ms) / args.steps
        kernel_ms_median = step_ms[len(step_ms) // 2]
    else:
        kernel_ms = steps_ms / args.steps
        kernel_ms_median = None

    errs = d_err.clone()   # the timed steps' error count (the informational runs below add more)

    # informational, outside the timed region: the same batch staged from pinned host memory
    # (H2D + decode + D2H of the decoded bits), i.e. the PCIe-inclusive rate
    pcie_s = None
    if rank == 0:
        h_in = torch.from_numpy(host_in).pin_memory()
        h_out = torch.empty((nb, code.out_bytes), dtype=torch.uint8).pin_memory()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            d_rx.copy_(h_in, non_blocking=True)
            step()
            h_out.copy_(d_out, non_blocking=True)
        torch.cuda.synchronize()
        pcie_s = (time.perf_counter() - t1) / reps

    # informational: the measured achievable-HBM ceiling: a hand-written streaming
    # pass over the input batch (ccv_hbm_probe: global_load_dwordx4, four in flight per lane), as a copy
    # (read + write bytes) and as a read-only stream (the decode kernels' access), best of 5 each
    hbm_probe = None
    if rank == 0 and not args.no_hbm_probe:
        hbm_probe = measure_hbm_ceiling(d_rx, stream)

    # informational: the same frames generated AND decoded on the GPU (ccv_simulate_device, the
    # on-device channel of SURVEY.md 8(f) #1) -- no host producer, no input in HBM
    fused = None
    if rank == 0 and not args.no_fused_channel and not sequential:
        d_ferr = torch.zeros(1, dtype=torch.int64, device="cuda")
        scaling = args.p_ppm if hard else ch.noise_scaling(args.ebn0)
        plan.simulate_device(args.seed, 0, nb, scaling, d_errors=d_ferr, stream=stream)   # warm-up
        d_ferr.zero_()
        reps = 5
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(stream)
        for _ in range(reps):
            plan.simulate_device(args.seed, 0, nb, scaling, d_errors=d_ferr, stream=stream)
        ev[1].record(stream)
        torch.cuda.synchronize()
        f_ms = ev[0].elapsed_time(ev[1]) / reps
        f_err = int(d_ferr.item()) // reps
        fused = {"mbit_s": round(nb * code.blen / (f_ms * 1e-3) / 1e6, 1), "kernel_ms": round(f_ms, 4),
                 "ber": f_err / (nb * code.blen),
                 "note": "same Philox frames generated on the GPU (encoder, mapper, Box-Muller AWGN, "
                         "demapper fused ahead of the ACS)"}

    # informational, Fano soft rate 1/2: the same frames as received points (x, y) from the on-device
    # channel (CCV_CHANNEL_IQ: 8 instead of 16 bytes per node) decoded with the distances recomputed in
    # the kernel (option fano_input 1) -- the device sweep's path; same Philox frames, so the same errors
    fano_iq = None
    if (rank == 0 and args.decoder == "fano" and not hard and code.n == 2 and code.K <= 32
            and not args.no_fused_channel):
        iq_plan = FanoPlan(code, chan).set_option("fano_input", 1)
        for opt in args.option:
            name, value = opt.split("=", 1)
            if name != "fano_input":
                iq_plan.set_option(name, int(value))
        iq_plan.reserve(nb)
        d_iq = torch.empty((nb, code.steps, 2), dtype=torch.float32, device="cuda")
        d_iinfo = torch.empty_like(d_info)
        iq_plan.simulate_frames(args.seed, 0, nb, ch.noise_scaling(args.ebn0), d_iq, d_info=d_iinfo,
                                stream=stream, iq=True)
        d_ierr = torch.zeros(1, dtype=torch.int64, device="cuda")
        reps = max(1, args.steps)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        torch.cuda.synchronize()
        ev[0].record(stream)
        for _ in range(reps):
            iq_plan.decode_device(d_iq, nb, d_out, d_info=d_iinfo, d_errors=d_ierr, stream=stream)
        ev[1].record(stream)
        torch.cuda.synchronize()
        i_ms = ev[0].elapsed_time(ev[1]) / reps
        i_err = int(d_ierr.item()) // reps
        fano_iq = {"mbit_s": round(nb * code.blen / (i_ms * 1e-3) / 1e6, 2), "kernel_ms": round(i_ms, 3),
                   "errors_per_step": i_err, "same_info_as_host_frames": bool(torch.equal(d_iinfo, d_info)),
                   "note": "the step's frames as received points from the on-device channel (8 B per node), "
                           "demapped in the Fano kernel (fano_input 1)"}
        del d_iq

    # the BER-vs-Eb/N0 half of the metric, after the timed region: every rank decodes its shard of
    # each point's frames on the on-device channel, one all-reduce of the counters (RCCL over xGMI)
    curve = None
    curve_frames = args.frames if args.curve_frames is None else args.curve_frames
    if curve_frames > 0 and not sequential:
        curve = ber_curve(code, hard, curve_frames, args.seed, rank, world, dist if use_pg else None,
                          "cuda" if backend == "nccl" else "cpu", noise=("f64", "f32"))

    errors = int(errs.item())
    per_rank_kernel_ms = [round(kernel_ms, 4)]
    if use_pg:   # MAX of the timings, SUM of the error counters (RCCL over xGMI)
        wall, kernel_ms, per_rank_kernel_ms, errors = reduce_over_ranks(
            dist, wall, kernel_ms, errors, "cuda" if backend == "nccl" else "cpu")
    bits_per_step = world * nb * code.blen

    if rank == 0:
        # SURVEY.md 8(d) prices every decoded bit with its survivor decisions (S/8 bytes per step)
        # whether or not they reach HBM ("the formula is unchanged, so the fraction stays
        # comparable"); hbm_bytes_per_bit counts only what must cross HBM for this kernel (decisions
        # excluded where they stay in VGPRs / LDS), and the PMC traffic what did cross it.
        bpb = algorithmic_bytes_per_bit(code, soft=not hard, decisions=not sequential)
        # ("slot": the K = 9 one-lane kernel's per-wave scratch, L2 / Infinity-Cache resident, counted
        # as HBM bytes here; the PMC traffic says what actually crossed)
        on_chip = sequential or getattr(plan, "decisions", "hbm") in ("registers", "lds")
        hbm_bpb = algorithmic_bytes_per_bit(code, soft=not hard, decisions=not on_chip)
        # K = 8 / 9 BSC on the soft persistent kernels: ccv_decode_device first turns each 1-byte symbol
        # into a 16-byte Hamming-distance row (core.hip hard_rows, inside the timed step), which the
        # decode then reads instead of the byte: +16 B written and +16 B read per step cross HBM
        conv_bpb = 0.0
        if hard and not sequential and getattr(plan, "variant", "") in ("persistent-wide", "persistent-slot2"):
            conv_bpb = code.steps * 32.0 / code.blen
            hbm_bpb += conv_bpb
        bytes_per_launch = bpb * nb * code.blen
        achieved = bytes_per_launch / (kernel_ms * 1e-3) / 1e9
        hbm_achieved = hbm_bpb * nb * code.blen / (kernel_ms * 1e-3) / 1e9
        workload_key = workload_key_of(args)
        pmc = pmc_for_variant(load_pmc(workload_key), getattr(plan, "variant", ""))
        traffic = pmc.get("hbm_bytes_per_launch")
        traffic_frac = traffic / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if traffic else None
        valu_frac = valu_fraction(pmc)
        # the binding resource, from the measured fractions: HBM traffic vs VALU issue
        if traffic_frac is not None and valu_frac is not None:
            bound = "valu" if valu_frac > traffic_frac else "hbm"
            bound_basis = ("the larger of traffic_frac (PMC HBM bytes / kernel time / 8 TB/s) and "
                           "valu_frac (SQ_INSTS_VALU / (512 per cycle x GRBM_GUI_ACTIVE / 8)); "
                           "frac / achieved / peak stay the SURVEY 8(d) HBM figure")
            if conv_bpb:
                bound_basis += ("; kernel_ms spans the Hamming-row conversion AND the decode, while the PMC "
                                "record (traffic, valu_frac) is the decode kernel's alone: both fractions "
                                "are lower bounds here, the conversion's 32 B per step are in hbm_bytes_per_bit")
            if max(valu_frac, traffic_frac) < LATENCY_BOUND_BELOW:
                # neither pipe is near busy: the waves' dependent chains (and, for the sequential
                # decoders, lanes idle behind the longest searches) set the time
                stall = pmc.get("stall") or {}
                bound = "latency"
                bound_basis = (f"traffic_frac {traffic_frac:.3f} and valu_frac {valu_frac:.3f} both below "
                               f"{LATENCY_BOUND_BELOW}: neither HBM nor VALU issue binds; waves waiting "
                               f"{stall.get('sq_wait_any_frac', float('nan')):.2f} / issue-stalled "
                               f"{stall.get('sq_wait_inst_any_frac', float('nan')):.2f} of their lifetime "
                               "(PMC stall pass)")
        else:
            bound = None   # not derived: no committed PMC pass for this workload
            bound_basis = (f"unmeasured: no PMC pass committed for workload key {workload_key!r} "
                           "(profiles/pmc_workloads.json; tools/pmc_workload.sh adds one)")
        cpu = cpu_opt = None
        if world == 1 and not args.no_cpu_baseline:
            gpu_out = d_out.cpu().numpy()
            cpu, _ = cpu_baseline(code, rx, gpu_out, args.cpu_seconds, decoder=args.decoder, hard=hard)
            if args.decoder == "viterbi" and code.K <= 9 and code.n <= 3:
                cpu_opt = cpu_optimized_baseline(code, rx, gpu_out, min(5.0, args.cpu_seconds), hard=hard)
        line = {
            "metric": METRIC,
            "value": round(bits_per_step * args.steps / wall / 1e6, 2),
            "unit": "Mbit/s",
            "n_gpus": world,
            "world_size": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u16" if hard else "f32",
            "data": ("synthetic: Philox BSC channel (per-bit flips at p_ppm), resident in HBM before timing"
                     if hard else
                     "synthetic: Philox AWGN channel at the reference's noise scaling, host-demapped, "
                     "resident in HBM before timing"),
            "config": {
                "workload": f"{'binary-symmetric' if hard else 'awgn'}-simulation {code.name or args.code} "
                            f"r=1/{code.n} K={code.K} {'hard' if hard else 'soft'} "
                            f"{ {'stack': 'stack decoder', 'fano': 'Fano decoder'}.get(args.decoder, 'Viterbi')}, "
                            f"blen {code.blen}, "
                            f"{args.frames} x 1M-bit frames per GPU per step",
                "code": args.code,
                "generator": "ref-x86" if code.gen_mode == 0 else "true-parity",
                "frames_per_gpu_per_step": args.frames,
                "blocks_per_gpu_per_step": nb,
                "channel": args.channel,
                **({"p_ppm": args.p_ppm} if hard else {"ebn0_db": args.ebn0}),
                "parallelism": f"dp{world} (frames sharded, counters all-reduced once)",
                "backend": backend if use_pg else None,
                "rccl_version": rccl_version,
                "same_device_rehearsal": bool(args.same_device),
                "kernel": plan.kernel,
                "variant": getattr(plan, "variant", plan.kernel),
                **({"options": dict(o.split("=", 1) for o in args.option)} if args.option else {}),
                "decisions": plan.decisions,
                "input_layout": ("block-major [nb][T] symbols (reference)" if hard else
                                 "block-major [nb][T][2^n] (reference)" if args.layout == "block"
                                 else "step-major [T][nb][2^n]"),
            },
            "ber": {**({"p_ppm": args.p_ppm} if hard else {"ebn0_db": args.ebn0}),
                    "errors": errors, "bits": bits_per_step * args.steps,
                    "ber": errors / (bits_per_step * args.steps)},
            "kernel_ms": round(kernel_ms, 4),
            "kernel_ms_median": round(kernel_ms_median, 4) if kernel_ms_median is not None else None,
            "timed_steps_device_ms": round(steps_ms, 4),
            "per_rank_kernel_ms": per_rank_kernel_ms,
            "clock_warmup_s": args.clock_warmup,
            # per rank, before the timed region: the host producer (Philox channel on cpu_threads()
            # threads) and the host bytes it holds (frames + info; rank 0 adds a pinned copy of the
            # frames for the PCIe-inclusive rate)
            "host_producer_s": round(t_prod, 3),
            "host_producer_threads": cpu_threads(),
            "host_bytes_per_rank": int(rx.nbytes + info.nbytes),
            "pcie_inclusive_mbit_s": round(nb * code.blen / pcie_s / 1e6, 1) if pcie_s else None,
            "roofline": {
                "bound": bound,
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "algorithmic_bytes_per_bit": round(bpb, 4),
                "bytes_per_launch": int(bytes_per_launch),
                "hbm_bytes_per_bit": round(hbm_bpb, 4),
                "conversion_bytes_per_bit": round(conv_bpb, 4) if conv_bpb else None,
                "hbm_achieved": round(hbm_achieved, 1),
                "hbm_frac": round(hbm_achieved / HBM_PEAK_GBS, 4),
                "traffic_frac": round(traffic_frac, 4) if traffic_frac is not None else None,
                "valu_frac": round(valu_frac, 4) if valu_frac is not None else None,
                "clock_ghz": (round(pmc["grbm_gui_active"] / 8 / (pmc["kernel_ns"] * 1e-9) / 1e9, 3)
                              if pmc.get("grbm_gui_active") and pmc.get("kernel_ns") else None),
                "pmc_source": pmc.get("source"),
                "traffic_gbs": round(traffic / (kernel_ms * 1e-3) / 1e9, 1) if traffic else None,
                **hbm_ceiling_fields(hbm_probe, traffic, kernel_ms),
                "pmc_scale_used": {"fetch": PMC_FETCH_SCALE, "write": PMC_WRITE_SCALE} if traffic else None,
                "pmc_calibration": pmc.get("calibration") if traffic else None,
                "pmc_scale_note": pmc_scale_note(pmc.get("calibration")) if traffic else None,
                "bound_basis": bound_basis,
            },
            "cpu_baseline": cpu,
            "cpu_baseline_optimized": cpu_opt,
            "fused_channel": fused,
            **({"fano_received_points": fano_iq} if fano_iq else {}),
            "ber_curve": ({"frames_per_gpu_per_point": curve_frames, "data": "on-device channel "
                           "(Philox, the reference's noise scaling), stream of point k = (seed, k << 40 | block)",
                           **curve} if curve else None),
        }
        print(json.dumps(line), flush=True)
    if use_pg:
        dist.destroy_process_group()


def workload_key_of(args):
    """Key of this workload in profiles/pmc_workloads.json."""
    key = f"{args.code}:frames{args.frames}:{args.layout}"
    if args.decoder != "viterbi":
        key += ":" + args.decoder
    if args.channel == "bsc":
        key += ":bsc"
    return key


if __name__ == "__main__":
    sys.exit(main())
