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


@pytest.mark.parametrize("transport,num_ps", [("tcp", 1), ("xgmi", 1), ("xgmi", 2)])
def test_distributed_script_on_gpu(tmp_path, transport, num_ps):
    """ps + 2 workers on the GPU (the reference's 3-process recipe, R/distributed/distributed.py:7-14).
    xgmi: the ps arena is mapped into both workers; every push lands and bumps global_step exactly once,
    so the last progress line printed by the later worker shows the total worker step count.  With
    two ps tasks the variables are placed round-robin (global_step, W2, b2 on ps0; W1, b1 on ps1) and
    the step bump is issued behind BOTH tasks' SGD runs (cluster/xgmi.py push_async)."""
    import re
    import socket
    s = [socket.socket() for _ in range(2 + num_ps)]
    for x in s:
        x.bind(("127.0.0.1", 0))
    ports = [x.getsockname()[1] for x in s]
    for x in s:
        x.close()
    pss, (w1, w2) = ports[:num_ps], ports[num_ps:]
    script = os.path.join(ROOT, "distributed", "distributed.py")
    epochs, batches = 2, 200
    args = ["--ps_hosts=" + ",".join(f"127.0.0.1:{q}" for q in pss), f"--worker_hosts=127.0.0.1:{w1},127.0.0.1:{w2}",
            "--device=cuda", f"--logs_path={tmp_path}", "--recovery_wait_secs=0.2", f"--training_epochs={epochs}",
            f"--max_batches_per_epoch={batches}", "--ps_exit_after_workers", f"--transport={transport}",
            "--xgmi_arena_mb=4"]
    p = [subprocess.Popen([sys.executable, script, *args, "--job_name=ps", f"--task_index={k}"])
         for k in range(num_ps)]
    w = [subprocess.Popen([sys.executable, script, *args, "--job_name=worker", f"--task_index={i}"],
                          stdout=subprocess.PIPE, text=True) for i in (0, 1)]
    try:
        outs = [x.communicate(timeout=300)[0] for x in w]
        assert all(x.returncode == 0 for x in w), outs
        for q in p:
            assert q.wait(timeout=60) == 0
    finally:
        for x in p + w:
            if x.poll() is None:
                x.kill()
    finals = []
    for o in outs:
        print(o)
        lines = o.strip().splitlines()
        assert lines[-1] == "done with training"
        assert any(ln.startswith("Acc: ") for ln in lines)
        steps = [int(m.group(1)) for m in re.finditer(r"Step so far: (\d+),", o)]
        finals.append(steps[-1])
    assert max(finals) == 2 * epochs * batches, finals


def test_xgmi_graph_loop_matches_eager(tmp_path):
    """One ps + one worker over xGMI: the graphed step (device-resident feed in TF1 next_batch order,
    pull/fwd/bwd/peer-SGD/step-bump in one HIP graph, cost read back at the log cadence) prints the
    same progress lines as the eager per-step loop (parallel/ps_worker.py GraphedPSLoop)."""
    import re
    import socket

    def run(graph):
        s = [socket.socket() for _ in range(2)]
        for x in s:
            x.bind(("127.0.0.1", 0))
        ps, wk = [x.getsockname()[1] for x in s]
        for x in s:
            x.close()
        script = os.path.join(ROOT, "distributed", "distributed.py")
        args = [f"--ps_hosts=127.0.0.1:{ps}", f"--worker_hosts=127.0.0.1:{wk}", "--device=cuda",
                f"--logs_path={tmp_path / str(graph)}", "--training_epochs=2", "--max_batches_per_epoch=300",
                "--ps_exit_after_workers", "--transport=xgmi", "--xgmi_arena_mb=4", f"--graph={graph}"]
        p = subprocess.Popen([sys.executable, script, *args, "--job_name=ps", "--task_index=0"])
        w = subprocess.Popen([sys.executable, script, *args, "--job_name=worker", "--task_index=0"],
                             stdout=subprocess.PIPE, text=True)
        try:
            out = w.communicate(timeout=300)[0]
            assert w.returncode == 0, out
            assert p.wait(timeout=60) == 0
        finally:
            for x in (p, w):
                if x.poll() is None:
                    x.kill()
        steps = [int(m.group(1)) for m in re.finditer(r"Step so far: (\d+),", out)]
        costs = [float(m.group(1)) for m in re.finditer(r"Cost now: ([0-9.]+),", out)]
        acc = float(re.search(r"Acc: ([0-9.]+)", out).group(1))
        return steps, costs, acc

    s_e, c_e, a_e = run(False)
    s_g, c_g, a_g = run(True)
    assert s_e == s_g and s_g[-1] == 600, (s_e, s_g)
    assert len(c_e) == len(c_g) and all(abs(x - y) <= 2e-4 for x, y in zip(c_e, c_g)), (c_e, c_g)
    assert abs(a_e - a_g) <= 0.01, (a_e, a_g)


def test_simple_script_on_gpu():
    """simple.py on the HIP kernels (affine / SSE / fused SGD) reaches the reference's golden values."""
    import numpy as np
    p = subprocess.run([sys.executable, os.path.join(ROOT, "simple", "simple.py"), "--device", "cuda"],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    import re
    m = re.search(r"W: \[(\S+)\] b: \[(\S+)\] loss (\S+)", p.stdout)
    W, b, loss = float(m.group(1)), float(m.group(2)), float(m.group(3))
    assert abs(W - (-0.9999971)) < 1e-6 and abs(b - 0.9999914) < 1e-6 and loss < 1e-9, p.stdout


def test_elementwise_kernels(gpu):
    """affine / SSE / fused activation-backward + bias colsum / scalar scale vs PyTorch fp32."""
    torch.manual_seed(9)
    for C in (1, 7, 64):
        x = torch.randn(300, C, device=gpu)
        w, b = torch.randn(C, device=gpu), torch.randn(C, device=gpu)
        y = torch.ops.tfx.affine_fwd(x, w, b)
        assert torch.allclose(y, w * x + b, atol=1e-6)
        g = torch.randn_like(x)
        dw, db = torch.zeros(C, device=gpu), torch.zeros(C, device=gpu)
        dx = torch.ops.tfx.affine_bwd(g, x, w, dw, db, True)
        assert torch.allclose(dx, g * w, atol=1e-6)
        assert torch.allclose(dw, (g * x).sum(0), atol=1e-4, rtol=1e-5)
        assert torch.allclose(db, g.sum(0), atol=1e-4, rtol=1e-5)
    p, t = torch.randn(5000, device=gpu), torch.randn(5000, device=gpu)
    loss = torch.ops.tfx.sse_fwd(p, t)
    assert abs(loss.item() - ((p - t) ** 2).sum().item()) < 1e-3 * loss.item()
    gs = torch.tensor([0.5], device=gpu)
    assert torch.allclose(torch.ops.tfx.sse_bwd(p, t, gs), 2 * (p - t) * 0.5, atol=1e-6)
    for act in (0, 1, 2):
        gy = torch.randn(100, 100, device=gpu)
        ya = torch.rand(100, 100, device=gpu) if act == 2 else torch.relu(torch.randn(100, 100, device=gpu))
        dbias = torch.ones(100, device=gpu)
        dz = torch.ops.tfx.act_bwd_colsum(gy, ya, act, dbias)
        ref = gy if act == 0 else (gy * (ya > 0) if act == 1 else gy * ya * (1 - ya))
        assert torch.allclose(dz, ref, atol=1e-6)
        assert torch.allclose(dbias - 1, ref.sum(0), atol=1e-4, rtol=1e-5)
    # bf16 dense-layer backward: ReLU mask + bias column sums in one pass (M large: atomic partials)
    for act in (0, 1):
        gy = torch.randn(6400, 65, device=gpu).to(torch.bfloat16)
        ya = torch.relu(torch.randn(6400, 65, device=gpu)).to(torch.bfloat16) if act else gy
        dbias = torch.zeros(65, device=gpu)
        dz = torch.ops.tfx.act_bwd_colsum(gy, ya, act, dbias)
        ref = gy.float() * (ya.float() > 0) if act else gy.float()
        if act:
            assert dz.dtype == torch.bfloat16 and torch.equal(dz.float(), ref)
        assert torch.allclose(dbias, ref.sum(0), atol=1e-2, rtol=1e-4)
    z = torch.randn(64, 10, device=gpu)
    s16 = torch.ops.tfx.scale_by_scalar(z, torch.tensor([2.0], device=gpu), True)
    assert s16.dtype == torch.bfloat16 and torch.allclose(s16.float(), 2 * z, rtol=1e-2)
