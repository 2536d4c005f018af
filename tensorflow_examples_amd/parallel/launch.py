"""Process-group bring-up and the framework's own local launcher: one process per GPU.

The reference runs "one process per task, launched per role" by hand
(R/distributed/distributed.py:7-14,37-43); the synchronous data-parallel path does the same on
one MI355X node without an external launcher:

* :func:`spawn_local` starts N fresh ranks of a script with RANK / LOCAL_RANK / WORLD_SIZE /
  LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT set (rendezvous on 127.0.0.1, a free port), relays
  rank 0's stdout, sends every other rank's stdout to stderr, and tears the whole job down as soon
  as one rank fails or the job times out.  The launching process never touches the GPU (it only
  execs ``sys.executable``), so the children initialise HIP from scratch -- never fork/exec a
  process that has initialised the GPU.
* :func:`init_distributed` (called by every rank) reads that torchrun-compatible contract, so a
  script runs unchanged under this launcher, under ``python -m torch.distributed.run`` or alone.
  Backend ``nccl`` (= RCCL over xGMI) for GPU runs, ``gloo`` for CPU runs and CPU tests.

CLI: ``python -m tensorflow_examples_amd.parallel.launch --nproc N [--timeout S] script.py args...``
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time
from datetime import timedelta
from typing import Dict, List, Optional, Sequence

LAUNCH_ENV = "TFX_LAUNCHED"  # set in every child: a child never re-spawns


def world_size() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def rank() -> int:
    return int(os.environ.get("RANK", "0"))


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def under_launcher() -> bool:
    """True when a launcher (ours or torchrun) has already assigned this process a rank."""
    return "RANK" in os.environ and "WORLD_SIZE" in os.environ


def free_port(host: str = "127.0.0.1") -> int:
    s = socket.socket()
    s.bind((host, 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _terminate(procs: Sequence[subprocess.Popen], grace_s: float = 10.0) -> None:
    """SIGTERM every live rank (its whole process group), SIGKILL what is left after ``grace_s``."""
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except (ProcessLookupError, PermissionError):
                pass
    deadline = time.monotonic() + grace_s
    for p in procs:
        while p.poll() is None and time.monotonic() < deadline:
            time.sleep(0.05)
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass
            p.wait()


def spawn_local(nprocs: int, argv: Sequence[str], timeout_s: Optional[float] = None,
                env: Optional[Dict[str, str]] = None, master_addr: str = "127.0.0.1",
                master_port: Optional[int] = None) -> int:
    """Run ``sys.executable *argv`` as ``nprocs`` local ranks and wait for all of them.

    Returns 0 when every rank exits 0; otherwise the first failing rank's exit code (the other
    ranks are terminated at once -- a rank stuck in a collective with a dead peer would otherwise
    wait out the process-group timeout), or 124 on ``timeout_s``."""
    if nprocs < 1:
        raise ValueError("nprocs must be >= 1")
    port = master_port or free_port(master_addr)
    base = dict(os.environ if env is None else env)
    procs: List[subprocess.Popen] = []
    for r in range(nprocs):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs), LOCAL_WORLD_SIZE=str(nprocs),
                 MASTER_ADDR=master_addr, MASTER_PORT=str(port), GROUP_RANK="0")
        e[LAUNCH_ENV] = "1"
        # rank 0 owns stdout (the one result line); every other rank's stdout goes to stderr
        out = None if r == 0 else sys.stderr
        procs.append(subprocess.Popen([sys.executable, *argv], env=e, stdout=out, start_new_session=True))
    t0 = time.monotonic()
    code = 0
    try:
        while True:
            states = [p.poll() for p in procs]
            bad = [(i, c) for i, c in enumerate(states) if c not in (None, 0)]
            if bad:
                i, code = bad[0]
                print(f"launch: rank {i} exited with {code}; terminating the job", file=sys.stderr, flush=True)
                break
            if all(c == 0 for c in states):
                return 0
            if timeout_s is not None and time.monotonic() - t0 > timeout_s:
                print(f"launch: job exceeded {timeout_s:.0f}s; terminating", file=sys.stderr, flush=True)
                code = 124
                break
            time.sleep(0.1)
    except KeyboardInterrupt:
        code = 130
    _terminate(procs)
    return code if code > 0 else 1


def init_distributed(backend: Optional[str] = None, device: str = "cuda", timeout_s: int = 600):
    """Initialise the default process group if WORLD_SIZE > 1. Returns the device to use."""
    import torch
    import torch.distributed as dist

    ws = world_size()
    if device == "cuda":
        dev = torch.device("cuda", local_rank())
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    # TFX_DP_FORCE_COLLECTIVE=1 under a launcher: a 1-rank process group, so a one-GPU box runs the
    # real RCCL path of the DP step (GradAllReduce issues its collectives at world size 1 too)
    force = os.environ.get("TFX_DP_FORCE_COLLECTIVE", "0") == "1" and "RANK" in os.environ
    if (ws > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        backend = backend or ("nccl" if dev.type == "cuda" else "gloo")
        kw = {}
        if backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(backend=backend, rank=rank(), world_size=ws, timeout=timedelta(seconds=timeout_s), **kw)
    return dev


def control_group():
    """A gloo process group for host-side control collectives (agreement flags, barriers, timing
    reductions), so the RCCL communicator carries only the (possibly graph-captured) gradient
    collectives.  Falls back to the default group if gloo cannot be brought up on this host."""
    import torch.distributed as dist

    if not dist.is_initialized():
        return None
    if dist.get_backend() == "gloo":
        return None  # the default group already is gloo
    try:
        return dist.new_group(backend="gloo")
    except Exception as e:  # pragma: no cover - host networking dependent
        print(f"control group: gloo unavailable ({e}); using the default group", file=sys.stderr)
        return None


def control_device(group, device):
    """Where a control collective's tensor lives: the host for a gloo group, else ``device``."""
    import torch
    import torch.distributed as dist

    if group is not None or (dist.is_initialized() and dist.get_backend() == "gloo"):
        return torch.device("cpu")
    return device


def verify_world(expected: int, device) -> int:
    """Check the process group really spans ``expected`` ranks: the group size must match and an
    all-reduce of ones must sum to it (a collective that every rank completes).  Returns the size."""
    import torch
    import torch.distributed as dist

    ws = dist.get_world_size() if dist.is_initialized() else 1
    if ws != expected:
        raise RuntimeError(f"process group has {ws} ranks, expected {expected}")
    if dist.is_initialized():
        one = torch.ones(1, dtype=torch.float32, device=device)
        dist.all_reduce(one)
        if int(round(float(one.item()))) != expected:
            raise RuntimeError(f"all-reduce of ones returned {float(one.item())}, expected {expected}")
    return ws


def main(argv: Optional[Sequence[str]] = None) -> int:
    ap = argparse.ArgumentParser(description="spawn N local ranks of a script (one process per GPU)")
    ap.add_argument("--nproc", "--nproc-per-node", dest="nproc", type=int, required=True)
    ap.add_argument("--timeout", type=float, default=None, help="seconds before the whole job is killed")
    ap.add_argument("--master-port", type=int, default=None)
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    return spawn_local(a.nproc, [a.script, *a.args], timeout_s=a.timeout, master_port=a.master_port)


if __name__ == "__main__":
    sys.exit(main())
