"""The collectives of the sharded sweep and bench (independent Monte-Carlo frames per
Eb/N0 point sharded over the GPUs, AWGN-channel/main.c:193-235, with one all-reduce of the bit-error
counters).

CPU (gloo): bench.ber_curve's sharded curve equals the one-process curve at world sizes 2 and 3, and
bench.init_group forms a world-size-1 group. GPU: the same calls over RCCL (the nccl backend on
cuda) in a world-size-1 group on the box's one MI355X -- sim.all_reduce_counters,
bench.reduce_over_ranks (MAX / SUM all-reduces, all-gather) and a barrier -- in a child process,
and `bench.py --gpus 1 --backend nccl`, whose line carries the RCCL version and the curve."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG_ROOT, REPO
from ccviterbi import launch

CURVE_FRAME_BLOCKS = 300   # small frames: the oracle decodes them on the CPU


def _oracle_decode():
    import oracle_ctypes as O
    from ccviterbi import named_code
    c = named_code("code0")
    oc = O.code(c.n, c.K, c.blen, c.polys, c.gen_mode)
    return lambda info, data: O.count_errors(oc, info, O.viterbi_soft(oc, data))


def _curve(rank, world, use_dist):
    import bench
    from ccviterbi import named_code
    return bench.ber_curve(named_code("code0"), False, 2, 77, rank, world, dist if use_dist else None,
                           "cpu", decode=_oracle_decode(), frame_blocks=CURVE_FRAME_BLOCKS, threads=1)


def _curve_worker(rank, world, port, outdir, paths):
    sys.path[:0] = paths
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    dist.init_process_group("gloo")
    res = _curve(rank, world, True)
    with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_bench_ber_curve_sharded_equals_one_process(tmp_path, world):
    """Every rank reports the all-reduced curve, equal to one process decoding all world x 2 frames of
    each point (the per-block Philox stream: the totals do not depend on the sharding)."""
    mp.spawn(_curve_worker, args=(world, launch.free_port(), str(tmp_path), [REPO, PKG_ROOT]),
             nprocs=world, join=True)
    import bench
    from ccviterbi import named_code
    one = bench.ber_curve(named_code("code0"), False, 2 * world, 77, 0, 1, None, "cpu",
                          decode=_oracle_decode(), frame_blocks=CURVE_FRAME_BLOCKS, threads=1)
    for r in range(world):
        got = json.load(open(tmp_path / f"r{r}.json"))
        assert got["f64"]["points"] == one["f64"]["points"]
    pts = one["f64"]["points"]
    assert [p["ebn0_db"] for p in pts] == [0.0, 2.0, 4.0, 6.0, 8.0, 10.0, 12.0, 14.0]
    assert all(p["bits"] == 2 * world * CURVE_FRAME_BLOCKS * 40 for p in pts)
    assert pts[0]["errors"] > pts[3]["errors"]   # the curve falls with Eb/N0


def test_init_group_world_one_gloo(monkeypatch):
    """--backend at N = 1 forms a world-size-1 group on 127.0.0.1 (gloo here; nccl on the box)."""
    import torch
    import bench
    for k in ("MASTER_ADDR", "MASTER_PORT", "RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    assert bench.init_group(dist, torch, "gloo", 1, 0) is None
    try:
        assert dist.get_world_size() == 1 and os.environ["MASTER_ADDR"] == "127.0.0.1"
        wall, kms, per, err = bench.reduce_over_ranks(dist, 2.0, 0.5, 17, "cpu")
        assert (wall, kms, per, err) == (2.0, 0.5, [0.5], 17)
    finally:
        dist.destroy_process_group()


RCCL_CHILD = r"""
import json, os, sys
sys.path[:0] = [%r, %r]
os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": %r, "RANK": "0", "WORLD_SIZE": "1"})
import numpy as np, torch, torch.distributed as dist
import bench
from ccviterbi import sim
torch.cuda.set_device(0)
ver = bench.init_group(dist, torch, "nccl", 1, 0)
assert dist.get_backend() == "nccl"
table = np.array([[5, 1000], [7, 2000], [1 << 40, 3]], np.int64)
red = sim.all_reduce_counters(table)
wall, kms, per, err = bench.reduce_over_ranks(dist, 1.5, 0.25, 123456789012, "cuda")
dist.barrier()
dist.destroy_process_group()
print(json.dumps({"version": ver, "table": red.tolist(), "reduce": [wall, kms, per, err]}))
"""


@pytest.mark.gpu
def test_rccl_world_one_collectives():
    """The RCCL calls an N-GPU run makes, executed on the MI355X in a world-size-1 nccl group: the
    counter table's SUM all-reduce (int64, on cuda), the bench's MAX / SUM all-reduces and all-gather,
    a barrier. A child process, so this test's own process state does not matter."""
    code = RCCL_CHILD % (REPO, PKG_ROOT, str(launch.free_port()))
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    got = json.loads(r.stdout.strip().splitlines()[-1])
    print("RCCL version", got["version"])
    assert got["version"]
    assert got["table"] == [[5, 1000], [7, 2000], [1 << 40, 3]]
    assert got["reduce"] == [1.5, 0.25, [0.25], 123456789012]


@pytest.mark.gpu
def test_bench_world_one_rccl_line_with_curve(tmp_path):
    """`bench.py --gpus 1 --backend nccl`: the timed steps inside RCCL barriers, the reductions and the
    BER curve's all-reduce over RCCL; the line names the backend and the RCCL version, and the curve
    holds the reference's eight points for both noise modes, falling with Eb/N0."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for k in ("MASTER_ADDR", "MASTER_PORT", "RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1", "--backend", "nccl",
                        "--steps", "3", "--warmup", "1", "--frames", "8", "--clock-warmup", "0.05",
                        "--no-cpu-baseline", "--no-hbm-probe", "--no-fused-channel"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["config"]["backend"] == "nccl" and line["config"]["rccl_version"]
    curve = line["ber_curve"]
    for mode in ("f64", "f32"):
        pts = curve[mode]["points"]
        assert [p["ebn0_db"] for p in pts] == [0.0, 2.0, 4.0, 6.0, 8.0, 10.0, 12.0, 14.0]
        assert all(p["bits"] == 8 * 25000 * 40 for p in pts)
        assert pts[0]["ber"] > pts[2]["ber"] > 0
    # 4 dB, the x86-idiom K = 7 code's floor: ~3.55e-2 in both noise modes
    assert abs(curve["f64"]["points"][2]["ber"] - 0.0355) < 0.003
    assert abs(curve["f32"]["points"][2]["ber"] - 0.0355) < 0.003
