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

* :func:`launch_with_fallback` / :func:`supervise_rank`: a job that must END WITH A RESULT (the
  driver's scaling bench runs under a fixed lease).  Attempt 1 runs the ranks as configured under a
  deadline; if any rank fails or the deadline passes (a hung collective, a graph replay that never
  returns) every rank is killed and the job runs once more as fresh child processes with the
  fallback environment (e.g. ``TFX_DP_GRAPH=0``: eager collectives) on a fresh rendezvous, within
  what is left of the overall deadline.  Rank 0's stdout is buffered and relayed only for the
  attempt that succeeded on every rank, so the job prints exactly one result.  Under
  ``torch.distributed.run`` each rank process supervises its own child (the ranks agree on the
  outcome and the retry port through the agent's store); under our own launcher the launcher does.

CLI: ``python -m tensorflow_examples_amd.parallel.launch --nproc N [--timeout S] script.py args...``
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import threading
import time
from datetime import timedelta
from typing import Dict, List, Optional, Sequence, Tuple

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


class _Capture:
    """Drains a child's stdout pipe on a thread (a full pipe would block the child)."""

    def __init__(self, pipe):
        self.chunks: List[str] = []
        self._t = threading.Thread(target=self._run, args=(pipe,), daemon=True)
        self._t.start()

    def _run(self, pipe):
        for line in iter(pipe.readline, ""):
            self.chunks.append(line)
        pipe.close()

    def text(self, wait_s: float = 5.0) -> str:
        self._t.join(wait_s)
        return "".join(self.chunks)


def spawn_local(nprocs: int, argv: Sequence[str], timeout_s: Optional[float] = None,
                env: Optional[Dict[str, str]] = None, master_addr: str = "127.0.0.1",
                master_port: Optional[int] = None, capture_rank0: bool = False):
    """Run ``sys.executable *argv`` as ``nprocs`` local ranks and wait for all of them.

    Returns 0 when every rank exits 0; otherwise the first failing rank's exit code (the other
    ranks are terminated at once -- a rank stuck in a collective with a dead peer would otherwise
    wait out the process-group timeout), or 124 on ``timeout_s``.  ``capture_rank0``: rank 0's
    stdout is buffered instead of relayed and the call returns ``(code, stdout)``."""
    if nprocs < 1:
        raise ValueError("nprocs must be >= 1")
    port = master_port or free_port(master_addr)
    base = dict(os.environ if env is None else env)
    procs: List[subprocess.Popen] = []
    cap = None
    for r in range(nprocs):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs), LOCAL_WORLD_SIZE=str(nprocs),
                 MASTER_ADDR=master_addr, MASTER_PORT=str(port), GROUP_RANK="0")
        e[LAUNCH_ENV] = "1"
        # rank 0 owns stdout (the one result line); every other rank's stdout goes to stderr
        out = (subprocess.PIPE if capture_rank0 else None) if r == 0 else sys.stderr
        procs.append(subprocess.Popen([sys.executable, *argv], env=e, stdout=out, start_new_session=True,
                                      text=True if (r == 0 and capture_rank0) else None))
        if r == 0 and capture_rank0:
            cap = _Capture(procs[0].stdout)
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
                return (0, cap.text()) if capture_rank0 else 0
            if timeout_s is not None and time.monotonic() - t0 > timeout_s:
                print(f"launch: job exceeded {timeout_s:.0f}s; terminating", file=sys.stderr, flush=True)
                code = 124
                break
            time.sleep(0.1)
    except KeyboardInterrupt:
        code = 130
    _terminate(procs)
    code = code if code > 0 else 1
    return (code, cap.text(0.5) if cap is not None else "") if capture_rank0 else code


def _attempt_budget(deadline_s: float, first_s: Optional[float]) -> float:
    return first_s if first_s is not None else deadline_s / 2


def launch_with_fallback(nprocs: int, argv: Sequence[str], deadline_s: float, fallback_env: Dict[str, str],
                         first_s: Optional[float] = None) -> int:
    """spawn_local with one retry: attempt 1 gets ``first_s`` (default half the deadline); on any
    failure or time-out the whole job is relaunched as fresh processes with ``fallback_env`` on a new
    port, within the rest of ``deadline_s``.  Rank 0's stdout of the successful attempt only is
    written to stdout.  Returns the exit code of the last attempt."""
    t0 = time.monotonic()
    code, out = spawn_local(nprocs, argv, timeout_s=_attempt_budget(deadline_s, first_s),
                            env=dict(os.environ, TFX_BENCH_ATTEMPT="1"), capture_rank0=True)
    if code == 0:
        sys.stdout.write(out)
        sys.stdout.flush()
        return 0
    left = deadline_s - (time.monotonic() - t0)
    print(f"launch: attempt 1 failed ({code}); relaunching {nprocs} fresh ranks with "
          f"{fallback_env} ({left:.0f}s left)", file=sys.stderr, flush=True)
    if left <= 5:
        return code
    code, out = spawn_local(nprocs, argv, timeout_s=left, env=dict(os.environ, TFX_BENCH_ATTEMPT="2", **fallback_env),
                            capture_rank0=True)
    if code == 0:
        sys.stdout.write(out)
        sys.stdout.flush()
    return code


SUPERVISED_ENV = "TFX_SUPERVISED"


def can_supervise() -> bool:
    """Under torch.distributed.run (the agent hosts a store at MASTER_ADDR:MASTER_PORT) and not
    already a supervised child or a child of our own launcher."""
    return (os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "") == "True" and "RANK" in os.environ and
            "MASTER_PORT" in os.environ and os.environ.get(SUPERVISED_ENV) != "1" and
            os.environ.get(LAUNCH_ENV) != "1")


def _run_child(cmd, env, budget_s: float, capture: bool, store=None, fail_key: Optional[str] = None
               ) -> Tuple[int, str]:
    """Run one child under a deadline; stop early when a peer has posted ``fail_key`` (its collectives
    can never complete then).  Returns (exit code or 124, captured stdout)."""
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE if capture else None, text=capture or None,
                         start_new_session=True)
    cap = _Capture(p.stdout) if capture else None
    t0 = time.monotonic()
    last_check = 0.0
    code = None
    while True:
        c = p.poll()
        if c is not None:
            code = c
            break
        now = time.monotonic()
        if now - t0 > budget_s:
            print(f"supervise: rank {rank()} attempt exceeded {budget_s:.0f}s; killing it", file=sys.stderr, flush=True)
            code = 124
            break
        if store is not None and fail_key is not None and now - last_check > 1.0:
            last_check = now
            try:
                if store.check([fail_key]):
                    print(f"supervise: rank {rank()}: a peer failed; stopping this attempt", file=sys.stderr,
                          flush=True)
                    code = 125
                    break
            except Exception:  # pragma: no cover - the store went away: keep waiting on the child
                pass
        time.sleep(0.1)
    if p.poll() is None:
        _terminate([p])
    return code, (cap.text(0.5 if code else 5.0) if cap is not None else "")


def supervise_rank(argv: Sequence[str], deadline_s: float, fallback_env: Dict[str, str],
                   first_s: Optional[float] = None) -> int:
    """This process (one torch.distributed.run rank) never touches the GPU: it runs the real rank as a
    child process, at most twice (see the module docstring).  The ranks agree through the agent's
    store: each posts its attempt's outcome, a failing rank also posts a shared fail key (the peers
    then stop waiting at once), and rank 0 publishes a fresh rendezvous port for attempt 2."""
    import torch.distributed as dist

    r, ws = rank(), world_size()
    addr, port = os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ["MASTER_PORT"])
    store = dist.TCPStore(addr, port, is_master=False, timeout=timedelta(seconds=max(30.0, deadline_s)))
    run_id = os.environ.get("TORCHELASTIC_RUN_ID", "none") + "/" + os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
    t0 = time.monotonic()
    code = 1
    for k in (1, 2):
        left = deadline_s - (time.monotonic() - t0)
        budget = min(_attempt_budget(deadline_s, first_s), left) if k == 1 else left
        if budget <= 5:
            break
        env = dict(os.environ, TFX_BENCH_ATTEMPT=str(k))
        env[SUPERVISED_ENV] = "1"
        if k == 2:
            env.update(fallback_env)
            key = f"tfx/{run_id}/port{k}"
            if r == 0:
                store.set(key, str(free_port(addr)))
            env["MASTER_PORT"] = store.get(key).decode()
            env.pop("TORCHELASTIC_USE_AGENT_STORE", None)  # rank 0's child hosts the new rendezvous
            print(f"supervise: rank {r}: attempt 2 with {fallback_env} on port {env['MASTER_PORT']} "
                  f"({budget:.0f}s left)", file=sys.stderr, flush=True)
        fail_key = f"tfx/{run_id}/a{k}/fail"
        code, out = _run_child([sys.executable, *argv], env, budget, capture=(r == 0), store=store,
                               fail_key=fail_key)
        if code != 0:
            store.set(fail_key, str(r))
        store.set(f"tfx/{run_id}/a{k}/r{r}", "0" if code == 0 else "1")
        keys = [f"tfx/{run_id}/a{k}/r{q}" for q in range(ws)]
        try:
            store.wait(keys, timedelta(seconds=max(10.0, deadline_s - (time.monotonic() - t0))))
            ok = all(store.get(kk) == b"0" for kk in keys)
        except Exception as e:  # pragma: no cover - a peer vanished without posting
            print(f"supervise: rank {r}: no outcome from every rank ({e})", file=sys.stderr, flush=True)
            ok = False
        if ok:
            if r == 0:
                sys.stdout.write(out)
                sys.stdout.flush()
            return 0
        code = code or 1
    return code


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
