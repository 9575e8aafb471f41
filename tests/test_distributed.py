"""Multi-process path on CPU: world_size-2 gloo run of the sharded BER sweep (one process per GPU on
the box; here the decode step is the oracle) ending in the single counter all-reduce."""
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


def test_gloo_world2_ber_sweep_matches_single_process(tmp_path):
    from conftest import PKG_ROOT, REPO
    paths = [PKG_ROOT, os.path.join(REPO, "tests")]
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), paths), nprocs=2, join=True)
    r0 = json.load(open(tmp_path / "r0.json"))
    r1 = json.load(open(tmp_path / "r1.json"))
    assert r0 == r1                                  # every rank holds the reduced counters

    import oracle_ctypes as O
    from ccviterbi import CODEBOOK, sim
    c = CODEBOOK[0]
    oc = O.code(c.n, c.K, c.blen, c.polys, c.gen_mode)
    single = sim.ber_sweep(c, [1.0, 3.0], bits_per_point=lambda p: 5 * 400 * c.blen, frame_blocks=400,
                           decode=lambda i, d: O.count_errors(oc, i, O.viterbi_soft(oc, d)), seed=77)
    assert r0 == [[p.errors, p.bits] for p in single]
    assert r0[0][1] == 5 * 400 * c.blen
