"""One process per GPU: self-launch under torch.distributed.run for bench.py and the sweep CLI.

The driver runs `python bench.py --gpus N` (and may equally run it under torchrun itself). When
N > 1 and no launcher has set WORLD_SIZE, the entry point calls `relaunch()` BEFORE anything touches
the GPU (torch is not even imported): it starts

    python -m torch.distributed.run --nnodes=1 --nproc-per-node=N --master-addr=127.0.0.1
           --master-port=P <script | -m module> <the same arguments>

as a CHILD process and exits with its return code (never exec: a process that initialised HIP must
not replace itself, and a child keeps the parent's exit status meaningful). Each rank then reads
RANK / LOCAL_RANK / WORLD_SIZE from its environment.
"""
import os
import socket
import subprocess
import sys
from typing import List, Mapping, Optional, Sequence

LAUNCHED_ENV = "CCV_LAUNCHED_BY"   # set in the children's environment, guards against a relaunch loop


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launcher_argv(nproc: int, target: str, argv: Sequence[str], port: int,
                  module: bool = False, python: Optional[str] = None) -> List[str]:
    """The torch.distributed.run command line that starts `nproc` ranks of `target`."""
    cmd = [python or sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={int(nproc)}", "--master-addr=127.0.0.1", f"--master-port={int(port)}"]
    if module:
        cmd.append("-m")
    cmd.append(target)
    cmd.extend(argv)
    return cmd


def world_from_env(env: Mapping[str, str] = os.environ):
    """(rank, local_rank, world_size) as torch.distributed.run exports them; (0, 0, 1) standalone."""
    return (int(env.get("RANK", "0")), int(env.get("LOCAL_RANK", "0")), int(env.get("WORLD_SIZE", "1")))


def needs_launch(gpus: int, env: Mapping[str, str] = os.environ) -> bool:
    """True when `--gpus N` (N > 1) asks for ranks that no launcher has started yet."""
    if gpus <= 1 or "WORLD_SIZE" in env:
        return False
    if env.get(LAUNCHED_ENV):
        raise SystemExit(f"--gpus {gpus}: relaunched under torch.distributed.run but WORLD_SIZE is unset")
    return True


def check_world(gpus: int, world: int):
    if world != gpus:
        raise SystemExit(f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks")


def relaunch(nproc: int, target: str, argv: Sequence[str], module: bool = False) -> int:
    """Run `nproc` ranks of `target` under torch.distributed.run as a child; its return code."""
    env = dict(os.environ)
    env[LAUNCHED_ENV] = target
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # RCCL peer memory over dmabuf on this host
    if module:   # `-m ccviterbi.sim` in the children: the package root on their path
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    cmd = launcher_argv(nproc, target, argv, free_port(), module=module)
    print("launching: " + " ".join(cmd), file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode
