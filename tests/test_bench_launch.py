"""bench.py's own N-rank launch (parallel/launch.py spawn_local) on the CPU over gloo.

The driver's scaling run is ``bench.py --gpus N`` (under torchrun, or alone): the job must really
span N ranks and report the verified world size -- the process-per-task model of
R/distributed/distributed.py:7-14,37-43.
"""
import json
import math
import os
import subprocess
import sys
import textwrap
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    return dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=ROOT)


def test_bench_spawns_two_ranks_on_cpu():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu", "--depth", "18",
           "--batch", "4", "--steps", "2", "--warmup", "1", "--nbatches", "2", "--launch-timeout", "600"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=_env(), cwd=ROOT)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2
    assert rec["config"]["parallelism"] == "dp2"
    assert rec["config"]["global_batch"] == 8
    assert rec["config"]["backend"] == "gloo"
    assert math.isfinite(rec["config"]["final_loss"])
    assert rec["value"] > 0 and rec["steps"] == 2 and rec["warmup"] == 1


def test_launcher_fails_fast_when_a_rank_dies(tmp_path):
    """Rank 1 exits with an error while rank 0 waits in a collective: the launcher must tear the job
    down and return the failing code, not hang until the process-group timeout."""
    script = tmp_path / "w.py"
    script.write_text(textwrap.dedent("""
        import os, sys, time
        import torch, torch.distributed as dist
        sys.path.insert(0, os.environ["ROOT"])
        from tensorflow_examples_amd.parallel.launch import init_distributed, verify_world
        dev = init_distributed(device="cpu")
        verify_world(2, dev)
        if dist.get_rank() == 1:
            sys.exit(7)
        dist.barrier()          # never completes: rank 1 is gone
        time.sleep(600)
    """))
    cmd = [sys.executable, "-m", "tensorflow_examples_amd.parallel.launch", "--nproc", "2", "--timeout", "120",
           str(script)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=200, env=dict(_env(), ROOT=ROOT), cwd=ROOT)
    assert p.returncode == 7, (p.returncode, p.stderr[-3000:])
    assert "rank 1 exited with 7" in p.stderr


def test_verify_world_rejects_wrong_size(tmp_path):
    """A rank launched into a 1-rank job but asked for --gpus 2 refuses to time anything."""
    env = dict(_env(), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29999")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu", "--depth", "18",
           "--batch", "2", "--steps", "1", "--warmup", "0"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode != 0
    assert "expected 2" in p.stderr


def _one_json(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


_BENCH_SMALL = ["--gpus", "2", "--device", "cpu", "--depth", "18", "--batch", "4", "--steps", "2", "--warmup", "1",
                "--nbatches", "2", "--launch-timeout", "240", "--attempt-timeout", "45"]


def test_bench_hang_falls_back_in_launcher_mode():
    """Rank 1 hangs before its first step (TFX_BENCH_HANG, attempt 1 only): the launcher kills the job
    at the attempt deadline and reruns fresh ranks with the eager fallback -- exactly one JSON line,
    from attempt 2, spanning both ranks, well inside the overall deadline."""
    env = dict(_env(), TFX_BENCH_HANG="1:1")
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *_BENCH_SMALL], capture_output=True,
                       text=True, timeout=400, env=env, cwd=ROOT)
    took = time.monotonic() - t0
    assert p.returncode == 0, p.stderr[-4000:]
    rec = _one_json(p.stdout)
    assert rec["n_gpus"] == 2 and rec["config"]["verified_ranks"] == 2
    assert rec["config"]["attempt"] == 2 and rec["config"]["hip_graph"] is False
    assert "attempt 1 failed" in p.stderr
    assert took < 240, took


def test_bench_hang_falls_back_under_torchrun():
    """The driver's form of the scaling run: ``python -m torch.distributed.run ... bench.py --gpus 2``.
    Each torchrun rank supervises its real rank as a child; rank 1's child hangs in attempt 1, the
    supervisors agree on the failure through the agent store and rerun on a fresh rendezvous: one JSON
    line, from attempt 2, with n_gpus == 2."""
    env = dict(_env(), TFX_BENCH_HANG="1:1")
    t0 = time.monotonic()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), *_BENCH_SMALL]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    took = time.monotonic() - t0
    assert p.returncode == 0, p.stderr[-4000:]
    rec = _one_json(p.stdout)
    assert rec["n_gpus"] == 2 and rec["config"]["attempt"] == 2
    assert "attempt 2" in p.stderr
    assert took < 240, took


def test_bench_under_torchrun_no_fault_runs_once():
    """Without a fault the supervised job runs attempt 1 only and prints its one JSON line."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), *_BENCH_SMALL]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=_env(), cwd=ROOT)
    assert p.returncode == 0, p.stderr[-4000:]
    rec = _one_json(p.stdout)
    assert rec["n_gpus"] == 2 and rec["config"]["attempt"] == 1


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port
