"""One process per GPU: rank spawning and process-group bring-up.

The reference runs one process on one device (main.py:92); the multi-GPU
split is build-only scope. Two launch forms are supported:

  * under ``torch.distributed.run`` (RANK / WORLD_SIZE / LOCAL_RANK set by it);
  * ``python bench.py --gpus N`` with no launcher: :func:`spawn_ranks` starts N
    child processes of the same script with the torchrun environment, BEFORE
    the parent touches the GPU (a process that has initialised HIP must never
    exec another program, and the children each own one device).

:func:`init_distributed` then brings up the group (RCCL = backend ``nccl`` on
ROCm, or gloo on the CPU) and fails loudly when the group's size is not the
requested one.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional, Sequence, Tuple

ENV_KEYS = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


class LaunchError(RuntimeError):
    """The rank set could not be started or did not match the requested size."""


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def under_launcher() -> bool:
    """True when this process is one rank of an already-launched group."""
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def rank_env(rank: int, world: int, port: int, base: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # dmabuf IPC is the only mode the host driver supports (RCCL / tensor sharing)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def spawn_ranks(nprocs: int, argv: Sequence[str], poll_s: float = 0.2, timeout_s: Optional[float] = None) -> int:
    """Run ``python argv…`` as ranks 0..nprocs-1 on this node and wait for all of them.

    Children inherit stdout / stderr (rank 0 prints the result line). When a
    rank fails, the remaining ranks are terminated (their exact PIDs) and the
    first non-zero exit code is returned; 0 when every rank succeeded. A SIGTERM /
    SIGHUP / SIGINT to this parent (e.g. a job timeout) terminates the ranks before the
    parent exits (status 128 + signal), so no rank is orphaned holding its GPU and the
    rendezvous port."""
    if nprocs < 1:
        raise LaunchError(f"nprocs must be >= 1, got {nprocs}")
    port = free_port()
    procs: List[subprocess.Popen] = []

    class _Signalled(Exception):
        def __init__(self, signum):
            super().__init__(signum)
            self.signum = signum

    def _on_signal(signum, _frame):
        raise _Signalled(signum)

    old = {}
    for sig in (signal.SIGTERM, signal.SIGHUP, signal.SIGINT):
        try:
            old[sig] = signal.signal(sig, _on_signal)
        except ValueError:  # not the main thread: keep the default handlers
            break
    try:
        for r in range(nprocs):
            procs.append(subprocess.Popen([sys.executable, *argv], env=rank_env(r, nprocs, port)))
        t0 = time.time()
        rc = 0
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            if timeout_s is not None and time.time() - t0 > timeout_s:
                rc = 124
                break
            time.sleep(poll_s)
        return rc
    except _Signalled as e:
        return 128 + int(e.signum)
    finally:
        # a second signal during cleanup (a scheduler re-sending SIGTERM) must not kill this parent
        # before every rank is terminated and reaped: ignore them until then, restore the old
        # handlers last
        for sig in old:
            signal.signal(sig, signal.SIG_IGN)
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        for sig, h in old.items():
            signal.signal(sig, h)


def env_rank_world() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the launcher's environment (defaults 0/1/0)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def init_distributed(expected_world: Optional[int], backend: str = "nccl", device=None,
                     same_device: bool = False) -> Tuple[int, int, int]:
    """Bring up the process group and check its size against the requested rank count.

    Returns (rank, world, local_rank). world == 1 creates no group. ``expected_world``
    None (no explicit ``--gpus``) takes the launcher's WORLD_SIZE, so
    ``torchrun --nproc-per-node 8 bench.py`` works as before. Raises LaunchError if an
    explicit ``expected_world`` differs from the environment's or the group's size
    (e.g. ``--gpus 8`` started as a single process), or if ``same_device`` (every rank
    on one GPU) is asked of a backend other than gloo (RCCL refuses duplicate GPUs)."""
    import torch.distributed as dist
    rank, world, local = env_rank_world()
    if expected_world is None:
        expected_world = world
    if same_device and world > 1 and backend != "gloo":
        raise LaunchError(f"--same-device puts every rank on one GPU and needs --backend gloo, got {backend!r}")
    if world != expected_world:
        raise LaunchError(f"requested {expected_world} ranks but WORLD_SIZE={world} (rank {rank})")
    if world == 1:
        return rank, world, local
    kw = {"device_id": device} if (device is not None and backend == "nccl") else {}
    dist.init_process_group(backend, **kw)
    got = dist.get_world_size()
    if got != expected_world or dist.get_rank() != rank:
        raise LaunchError(f"process group has {got} ranks (rank {dist.get_rank()}), expected {expected_world} "
                          f"(rank {rank})")
    return rank, world, local
