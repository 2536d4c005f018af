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
