"""One process per GPU as the driver starts it (`python bench.py --gpus N`): the self-launch under
torch.distributed.run, the cross-rank reductions of bench.py and the sharded sweep CLI
(`python -m ccviterbi.sim`), all on CPU (no GPU is touched: gloo, an injected oracle decode)."""
import json
import os
import subprocess
import sys

import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist          # noqa: E402
import torch.multiprocessing as mp        # noqa: E402

from conftest import PKG_ROOT, REPO       # noqa: E402
from ccviterbi import launch              # noqa: E402


def test_launcher_argv():
    cmd = launch.launcher_argv(8, "/x/bench.py", ["--gpus", "8", "--steps", "5"], 29511, python="py")
    assert cmd == ["py", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
                   "--master-addr=127.0.0.1", "--master-port=29511", "/x/bench.py", "--gpus", "8",
                   "--steps", "5"]
    cmd = launch.launcher_argv(2, "ccviterbi.sim", ["--gpus", "2"], 1234, module=True, python="py")
    assert cmd[-4:] == ["-m", "ccviterbi.sim", "--gpus", "2"]


def test_needs_launch_rules():
    assert not launch.needs_launch(1, {})
    assert launch.needs_launch(2, {})
    assert not launch.needs_launch(8, {"WORLD_SIZE": "8"})          # started by torchrun (the driver's form)
    with pytest.raises(SystemExit):                                   # a relaunch that lost WORLD_SIZE
        launch.needs_launch(2, {launch.LAUNCHED_ENV: "bench.py"})
    launch.check_world(4, 4)
    with pytest.raises(SystemExit):
        launch.check_world(8, 1)
    assert launch.world_from_env({"RANK": "3", "LOCAL_RANK": "3", "WORLD_SIZE": "8"}) == (3, 3, 8)
    assert launch.world_from_env({}) == (0, 0, 1)


def test_bench_relaunches_before_touching_torch(monkeypatch):
    """`bench.py --gpus 4` without WORLD_SIZE hands its argv to torch.distributed.run unchanged and
    returns the child's exit code; `--gpus 1` output is unaffected (no launch)."""
    sys.path.insert(0, REPO)
    import bench
    calls = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv(launch.LAUNCHED_ENV, raising=False)
    monkeypatch.setattr(launch, "relaunch", lambda n, target, argv, module=False: calls.append(
        (n, target, list(argv), module)) or 7)
    assert bench.main(["--gpus", "4", "--steps", "3", "--warmup", "1"]) == 7
    assert calls == [(4, os.path.abspath(bench.__file__), ["--gpus", "4", "--steps", "3", "--warmup", "1"],
                      False)]


def test_relaunch_runs_ranks_under_torchrun(tmp_path):
    """The real torch.distributed.run command line: 2 ranks of a probe script each see their RANK and
    WORLD_SIZE=2, and the parent returns the launcher's exit code."""
    probe = tmp_path / "probe.py"
    probe.write_text("import os, json, sys\n"
                     f"open(os.path.join({str(tmp_path)!r}, 'r' + os.environ['RANK']), 'w').write(json.dumps("
                     "[os.environ['RANK'], os.environ['LOCAL_RANK'], os.environ['WORLD_SIZE'], sys.argv[1:]]))\n")
    code = ("import sys; sys.path.insert(0, %r); from ccviterbi import launch; "
            "sys.exit(launch.relaunch(2, %r, ['--gpus', '2']))" % (PKG_ROOT, str(probe)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", launch.LAUNCHED_ENV)}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    got = sorted(json.loads((tmp_path / f"r{k}").read_text()) for k in range(2))
    assert got == [["0", "0", "2", ["--gpus", "2"]], ["1", "1", "2", ["--gpus", "2"]]]


def _env(rank, world, port):
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})


def _reduce_worker(rank, world, port, outdir, paths):
    sys.path[:0] = paths
    _env(rank, world, port)
    import bench
    dist.init_process_group("gloo")
    res = bench.reduce_over_ranks(dist, 1.0 + rank, 0.25 * (rank + 1), 10 * (rank + 1), "cpu")
    with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_bench_rank_reductions_gloo(tmp_path, world):
    """bench.py's only exchange: MAX of wall and kernel time, SUM of the error counters, all-gather
    of the per-rank kernel times (the same calls run over RCCL on the GPUs), at world sizes 2, 3, 8."""
    mp.spawn(_reduce_worker, args=(world, launch.free_port(), str(tmp_path), [REPO, PKG_ROOT]),
             nprocs=world, join=True)
    for r in range(world):
        wall, kms, per_rank, errors = json.load(open(tmp_path / f"r{r}.json"))
        assert wall == float(world) and kms == 0.25 * world
        assert per_rank == [0.25 * (k + 1) for k in range(world)]
        assert errors == 10 * world * (world + 1) // 2


def _oracle_decode():
    import oracle_ctypes as O
    from ccviterbi import named_code
    c = named_code("code0")
    oc = O.code(c.n, c.K, c.blen, c.polys, c.gen_mode)
    return lambda info, data: O.count_errors(oc, info, O.viterbi_soft(oc, data))


SWEEP_ARGS = ["--code", "code0", "--points", "1,3,5", "--bits", str(6 * 400 * 40), "--frame-blocks", "400",
              "--seed", "91", "--threads", "2"]


def _cli_worker(rank, world, port, outdir, paths):
    sys.path[:0] = paths
    _env(rank, world, port)
    from ccviterbi import sim
    assert sim.main(SWEEP_ARGS + ["--gpus", str(world), "--backend", "gloo",
                                  "--out", os.path.join(outdir, "sweep.json")], decode=_oracle_decode()) == 0


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sweep_cli_gloo_matches_one_process(tmp_path, monkeypatch, capsys, world):
    """`python -m ccviterbi.sim --gpus N`: a contiguous frame range per rank, one all-reduce of the
    [points][errors, bits] table; the counts equal one process decoding every frame. 6 frames per
    point over 2, 3 and 8 ranks: even, uneven, and two ranks without a frame."""
    mp.spawn(_cli_worker, args=(world, launch.free_port(), str(tmp_path),
                                [REPO, PKG_ROOT, os.path.join(REPO, "tests")]),
             nprocs=world, join=True)
    two = json.load(open(tmp_path / "sweep.json"))
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    from ccviterbi import sim
    assert sim.main(SWEEP_ARGS + ["--out", str(tmp_path / "one.json")], decode=_oracle_decode()) == 0
    lines = [json.loads(x) for x in capsys.readouterr().out.splitlines() if x.startswith("{")]
    one = json.load(open(tmp_path / "one.json"))
    assert lines == one
    assert [(r["errors"], r["bits"]) for r in two] == [(r["errors"], r["bits"]) for r in one]
    assert [r["world_size"] for r in two] == [world] * 3 and one[0]["world_size"] == 1
    assert all(r["bits"] == 6 * 400 * 40 for r in one)
    assert one[0]["errors"] > one[1]["errors"] > one[2]["errors"]      # BER falls with Eb/N0
    for r in one:
        lo, hi = r["ber_99.9_binomial"]
        assert lo <= r["ber"] <= hi


def test_sweep_cli_split_with_first_point_index_matches_one_call(tmp_path, monkeypatch):
    """Point k of --points draws Philox stream --first-point-index + k: a sweep split over two
    invocations (the second passing the index its first point had in the whole sweep) gives the same
    counts as one call, and each record names its stream."""
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    from ccviterbi import sim
    base = [a for a in SWEEP_ARGS]
    i = base.index("--points")
    whole = base[:i] + ["--points", "1,3,5"] + base[i + 2:]
    part1 = base[:i] + ["--points", "1"] + base[i + 2:]
    part2 = base[:i] + ["--points", "3,5", "--first-point-index", "1"] + base[i + 2:]
    assert sim.main(whole + ["--out", str(tmp_path / "w.json")], decode=_oracle_decode()) == 0
    assert sim.main(part1 + ["--out", str(tmp_path / "a.json")], decode=_oracle_decode()) == 0
    assert sim.main(part2 + ["--out", str(tmp_path / "b.json")], decode=_oracle_decode()) == 0
    w = json.load(open(tmp_path / "w.json"))
    ab = json.load(open(tmp_path / "a.json")) + json.load(open(tmp_path / "b.json"))
    assert [(r["errors"], r["bits"], r["point_index"]) for r in w] == \
        [(r["errors"], r["bits"], r["point_index"]) for r in ab]
    assert [r["point_index"] for r in w] == [0, 1, 2]


def test_ber_interval():
    from ccviterbi.sim import ber_interval
    lo, hi = ber_interval(100, 10 ** 6)
    assert lo < 1e-4 < hi and hi - lo < 1e-4
    lo2, hi2 = ber_interval(100, 10 ** 6, burst=4.0)
    assert lo2 < lo and hi2 > hi
    assert ber_interval(0, 10 ** 6)[0] == 0.0


def test_point_ranges():
    """--points takes a comma list or an inclusive start:stop[:step] range (step 2 dB by default,
    the reference's spacing)."""
    from ccviterbi.sim import _parse_points
    assert _parse_points("0:14", 0) == [0.0, 2.0, 4.0, 6.0, 8.0, 10.0, 12.0, 14.0]
    assert _parse_points("10:14:1", 0) == [10.0, 11.0, 12.0, 13.0, 14.0]
    assert _parse_points("3,5", 0) == [3.0, 5.0]
