"""Reference MLP on the GPU (exact-f32 MFMA GEMMs, fused naive xent) vs the CPU reference path."""
import os
import subprocess
import sys

import pytest
import torch

from tensorflow_examples_amd import ops
from tensorflow_examples_amd.models.mnist_mlp import MnistMLP
from tensorflow_examples_amd.variables import VariableStore

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_mlp_grads_match_cpu(gpu):
    stores = []
    for dev in (gpu, torch.device("cpu")):
        st = VariableStore(dev, seed=2)
        m = MnistMLP(st)
        st.finalize()
        g = torch.Generator().manual_seed(0)
        x = torch.rand(100, 784, generator=g)
        y = torch.nn.functional.one_hot(torch.randint(0, 10, (100,), generator=g), 10).float()
        st.zero_grad()
        loss = m.loss(x.to(dev), y.to(dev), naive=True)
        loss.backward()
        acc = ops.accuracy(m.logits(x.to(dev)), y.to(dev))
        stores.append((st, float(loss), float(acc)))
    (sg, lg, ag), (sc, lc, ac) = stores
    assert abs(lg - lc) < 1e-4 * abs(lc) and abs(ag - ac) < 1e-6
    assert torch.allclose(sg.grad.cpu(), sc.grad, atol=1e-5, rtol=1e-4)


def test_distributed_script_on_gpu(tmp_path):
    import socket
    s = [socket.socket() for _ in range(3)]
    for x in s:
        x.bind(("127.0.0.1", 0))
    ps, w1, w2 = [x.getsockname()[1] for x in s]
    for x in s:
        x.close()
    script = os.path.join(ROOT, "distributed", "distributed.py")
    args = [f"--ps_hosts=127.0.0.1:{ps}", f"--worker_hosts=127.0.0.1:{w1},127.0.0.1:{w2}", "--device=cuda",
            f"--logs_path={tmp_path}", "--recovery_wait_secs=0.2", "--training_epochs=2",
            "--max_batches_per_epoch=200", "--ps_exit_after_workers"]
    p = subprocess.Popen([sys.executable, script, *args, "--job_name=ps", "--task_index=0"])
    w = [subprocess.Popen([sys.executable, script, *args, "--job_name=worker", f"--task_index={i}"],
                          stdout=subprocess.PIPE, text=True) for i in (0, 1)]
    try:
        outs = [x.communicate(timeout=300)[0] for x in w]
        assert all(x.returncode == 0 for x in w), outs
        assert p.wait(timeout=60) == 0
    finally:
        for x in [p] + w:
            if x.poll() is None:
                x.kill()
    for o in outs:
        print(o)
        assert o.strip().splitlines()[-1] == "done with training"
