"""Multi-process path on CPU: gloo runs of the sharded BER sweep at world sizes 2, 3 and 8 (one
process per GPU on the box; here the decode step is the oracle) ending in the single counter
all-reduce. 5 frames per point do not divide by 2, 3 or 8: uneven shards, and at world 8 ranks with no
frame at all (AWGN-channel/main.c:193-235 is the sweep being sharded)."""
import json
import os
import socket
import sys

import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist          # noqa: E402
import torch.multiprocessing as mp        # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, outdir, paths):
    sys.path[:0] = paths
    import oracle_ctypes as O
    from ccviterbi import CODEBOOK, sim
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    c = CODEBOOK[0]
    oc = O.code(c.n, c.K, c.blen, c.polys, c.gen_mode)

    def decode(info, data):
        return O.count_errors(oc, info, O.viterbi_soft(oc, data))

    res = sim.ber_sweep(c, [1.0, 3.0], bits_per_point=lambda p: 5 * 400 * c.blen, frame_blocks=400,
                        decode=decode, seed=77, rank=rank, world=world)
    with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
        json.dump([[p.errors, p.bits] for p in res], f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_gloo_ber_sweep_matches_single_process(tmp_path, world):
    from conftest import PKG_ROOT, REPO
    paths = [PKG_ROOT, os.path.join(REPO, "tests")]
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), paths), nprocs=world, join=True)
    r0 = json.load(open(tmp_path / "r0.json"))
    for r in range(1, world):                        # every rank holds the reduced counters
        assert json.load(open(tmp_path / f"r{r}.json")) == r0

    import oracle_ctypes as O
    from ccviterbi import CODEBOOK, sim
    c = CODEBOOK[0]
    oc = O.code(c.n, c.K, c.blen, c.polys, c.gen_mode)
    single = sim.ber_sweep(c, [1.0, 3.0], bits_per_point=lambda p: 5 * 400 * c.blen, frame_blocks=400,
                           decode=lambda i, d: O.count_errors(oc, i, O.viterbi_soft(oc, d)), seed=77)
    assert r0 == [[p.errors, p.bits] for p in single]
    assert r0[0][1] == 5 * 400 * c.blen


@pytest.mark.parametrize("nframes", [0, 1, 5, 7, 104, 1000])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_covers_every_frame_once(nframes, world):
    """sim.shard: contiguous, disjoint ranges whose union is every frame, sizes differing by at most
    one (ranks past the frame count get an empty range)."""
    from ccviterbi.sim import shard
    parts = [shard(nframes, r, world) for r in range(world)]
    assert [f for p in parts for f in p] == list(range(nframes))
    sizes = [len(p) for p in parts]
    assert max(sizes) - min(sizes) <= 1
