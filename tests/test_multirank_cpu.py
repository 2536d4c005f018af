"""The multi-GPU configurations rehearsed at their REAL rank counts on the CPU over gloo.

BASELINE.json config 3 (ResNet-50 DP on 8 GPUs) and config 5 (char-LSTM DP on 4 GPUs) run as one
process per rank -- the process-per-task model of R/distributed/distributed.py:7-14,37-43.  The other
multi-process tests stop at 2 ranks; these run the same code paths at 4 and 8:

* ``bench.py --gpus 8`` in launcher mode and under ``torch.distributed.run``, with and without a hung
  rank (attempt-1 hang -> fresh ranks, eager fallback): one JSON line spanning all 8 verified ranks;
* ``GradAllReduce`` at world 4 and 8 against one process on the full batch: the replicas stay
  bit-identical and match the single-process update;
* ``examples/char_lstm.py`` at 4 ranks (config 5's rank count), with a checkpoint resume.
"""
import json
import os
import socket
import subprocess
import sys
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tensorflow_examples_amd import ops
from tensorflow_examples_amd.models.mnist_mlp import MnistMLP
from tensorflow_examples_amd.optim import MomentumOptimizer
from tensorflow_examples_amd.parallel import GradAllReduce, broadcast_variables
from tensorflow_examples_amd.variables import VariableStore

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _env():
    # 8 ranks on the 8-CPU container: one thread each
    return dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=ROOT)


def _one_json(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


_BENCH8 = ["--gpus", "8", "--device", "cpu", "--depth", "18", "--batch", "2", "--steps", "2", "--warmup", "1",
           "--nbatches", "2", "--launch-timeout", "420"]


@pytest.mark.parametrize("form", ["launcher", "torchrun"])
def test_bench_eight_ranks(form):
    """The driver's N = 8 scaling command shape, on gloo: 8 verified ranks, dp8, global batch 8 x 2."""
    bench = os.path.join(ROOT, "bench.py")
    if form == "launcher":
        cmd = [sys.executable, bench, *_BENCH8]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8", "--master-addr",
               "127.0.0.1", "--master-port", str(_free_port()), bench, *_BENCH8]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=_env(), cwd=ROOT)
    assert p.returncode == 0, p.stderr[-4000:]
    rec = _one_json(p.stdout)
    assert rec["n_gpus"] == 8 and rec["config"]["verified_ranks"] == 8
    assert rec["config"]["parallelism"] == "dp8" and rec["config"]["global_batch"] == 16
    assert rec["config"]["attempt"] == 1 and rec["value"] > 0


def test_bench_eight_ranks_hang_falls_back():
    """Rank 5 of 8 hangs before its first step in attempt 1: the launcher kills all 8 at the attempt
    deadline and reruns 8 fresh ranks with the eager fallback -- one JSON line, from attempt 2."""
    env = dict(_env(), TFX_BENCH_HANG="5:1")
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *_BENCH8[:-2], "--launch-timeout", "420",
                        "--attempt-timeout", "90"], capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    took = time.monotonic() - t0
    assert p.returncode == 0, p.stderr[-4000:]
    rec = _one_json(p.stdout)
    assert rec["n_gpus"] == 8 and rec["config"]["attempt"] == 2 and rec["config"]["hip_graph"] is False
    assert "attempt 1 failed" in p.stderr
    assert took < 420, took


def _data(seed=0, n=64):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(n, 784, generator=g), torch.randint(0, 10, (n,), generator=g)


def _model(seed):
    st = VariableStore("cpu", seed=seed)
    m = MnistMLP(st)
    st.finalize()
    return st, m


def _dp_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    st, m = _model(seed=10 + rank)  # a different init per rank: the broadcast must make them equal
    broadcast_variables(st)
    dp = GradAllReduce(st, bucket_bytes=2048)  # several buckets
    opt = MomentumOptimizer(st, 0.1, momentum=0.9)
    x, y = _data()
    per = x.shape[0] // world
    xs, ys = x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per]
    for _ in range(3):
        st.zero_grad()
        ops.softmax_cross_entropy(m.logits(xs), ys, naive=False).backward()
        dp.finish()
        opt.apply_gradients(grad_scale=dp.grad_scale, grad=dp.reduced_grad)
    out[rank] = st.master.clone()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [4, 8])
def test_grad_allreduce_matches_single_process(world):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_dp_worker, args=(world, _free_port(), out), nprocs=world, join=True, start_method="spawn")
    p0 = out[0]
    for r in range(1, world):
        assert torch.equal(out[r], p0), r  # replicas bit-identical
    # one process, the full batch: mean loss = the average of the ranks' shard means (equal shards)
    st, m = _model(seed=10)
    opt = MomentumOptimizer(st, 0.1, momentum=0.9)
    x, y = _data()
    per = x.shape[0] // world
    for _ in range(3):
        st.zero_grad()
        losses = [ops.softmax_cross_entropy(m.logits(x[r * per:(r + 1) * per]), y[r * per:(r + 1) * per])
                  for r in range(world)]
        (sum(losses) / world).backward()
        opt.apply_gradients()
    assert torch.allclose(st.master, p0, atol=1e-5, rtol=1e-5)


def test_char_lstm_example_four_ranks(tmp_path):
    """Config 5's rank count: examples/char_lstm.py under torchrun with 4 ranks, checkpoints and a resume."""
    cp = tmp_path / "ck"
    args = ("--hidden_size=32", "--embed_size=16", "--batch_size=4", "--num_steps=10", "--synthetic_chars=20000",
            "--log_every=10", f"--logdir={cp}", "--save_checkpoint_steps=20")

    def run(steps):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4", "--master-addr",
               "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "examples", "char_lstm.py"),
               f"--max_steps={steps}", *args]
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=_env(), cwd=ROOT)
        assert p.returncode == 0, p.stderr[-4000:]
        return p.stdout

    out = run(20)
    assert "tokens/sec (all GPUs)" in out and "valid perplexity" in out
    from tensorflow_examples_amd import ckpt
    assert ckpt.latest_checkpoint(str(cp)).endswith("-20")
    run(40)
    assert ckpt.latest_checkpoint(str(cp)).endswith("-40")
