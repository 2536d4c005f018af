"""Data-parallel ResNet training through the HIP kernels with 2 ranks on one GPU.

RCCL refuses two ranks on one device, so this uses the gloo backend (GPU tensors) to exercise the
same GradAllReduce hooks / bucket launches / stream ordering as the RCCL path; the 8-GPU RCCL
run is the driver's scaling bench."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.environ["ROOT"])
from tensorflow_examples_amd.models.resnet import build_resnet_cifar, to_model_input
from tensorflow_examples_amd.optim import MomentumOptimizer
from tensorflow_examples_amd.parallel import GradAllReduce, broadcast_variables, init_distributed
from tensorflow_examples_amd.train import ClassifierTrainer
dev = init_distributed(backend="gloo", device="cuda")
rank = dist.get_rank()
store, model = build_resnet_cifar(device=dev, depth=int(os.environ["DEPTH"]), dtype=torch.bfloat16, seed=rank)
broadcast_variables(store)
dp = GradAllReduce(store, bucket_bytes=4 << 20)
tr = ClassifierTrainer(store, model, MomentumOptimizer(store, 0.01, momentum=0.9), dp)
g = torch.Generator().manual_seed(rank)
img = torch.randint(0, 256, (16, 32, 32, 3), dtype=torch.uint8, generator=g).to(dev)
lab = torch.randint(0, 10, (16,), generator=g).to(dev)
losses = [tr.step(to_model_input(img), lab).item() for _ in range(3)]
w = store.master.clone()
dist.broadcast(w, 0)
diff = (w - store.master).abs().max().item()
print(f"RANK{rank} buckets={len(dp.buckets)} diff={diff} losses={losses}", flush=True)
assert diff == 0.0, diff
dist.destroy_process_group()
'''


@pytest.mark.parametrize("depth", [18, 50])
def test_dp_two_ranks_one_gpu(gpu, tmp_path, depth):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    script = tmp_path / "w.py"
    script.write_text(WORKER)
    procs = []
    for r in range(2):
        env = dict(os.environ, ROOT=ROOT, DEPTH=str(depth), RANK=str(r), LOCAL_RANK="0", WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=300)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    print("\n".join(outs))
    assert all(p.returncode == 0 for p in procs), outs
    assert all("diff=0.0" in o for o in outs)


GRAPH_WORKER = r'''
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.environ["ROOT"])
from tensorflow_examples_amd.models.resnet import build_resnet_cifar, to_model_input
from tensorflow_examples_amd.optim import MomentumOptimizer
from tensorflow_examples_amd.parallel import GradAllReduce, init_distributed
from tensorflow_examples_amd.train import ClassifierTrainer
dev = init_distributed(device="cuda")  # TFX_DP_FORCE_COLLECTIVE=1: 1-rank RCCL process group
assert dist.is_initialized() and dist.get_backend() == "nccl", dist.get_backend()
g = torch.Generator().manual_seed(0)
img = torch.randint(0, 256, (16, 32, 32, 3), dtype=torch.uint8, generator=g).to(dev)
lab = torch.randint(0, 10, (16,), generator=g).to(dev)
x = to_model_input(img)
masters = []
for graphed in (False, True):
    store, model = build_resnet_cifar(device=dev, depth=18, dtype=torch.bfloat16, seed=0)
    dp = GradAllReduce(store, bucket_bytes=2 << 20)
    assert dp.force and len(dp.buckets) > 2
    tr = ClassifierTrainer(store, model, MomentumOptimizer(store, 0.01, momentum=0.9), dp)
    if graphed:
        tr.capture(x, lab, warmup=3)  # 3 eager steps, then the captured step (recorded only)
        losses = [tr.step(x, lab).item() for _ in range(2)]
    else:
        losses = [tr.step(x, lab).item() for _ in range(5)]
    torch.cuda.synchronize()
    masters.append(store.master.clone())
    print("graphed" if graphed else "eager", losses, flush=True)
    assert all(l == l for l in losses)
a, b = masters
rel = ((a - b).norm() / a.norm()).item()
print("REL", rel, flush=True)
assert rel < 1e-2, rel
dist.destroy_process_group()
'''


def test_dp_graph_capture_rccl_one_rank(gpu, tmp_path):
    """The DP step (bucketed RCCL all-reduces launched from grad-ready hooks) captured in a HIP graph
    and replayed, on a 1-rank RCCL process group: after 3 eager + 2 replayed steps the weights match
    5 eager steps (split-K atomics make the two runs differ in rounding only)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    script = tmp_path / "g.py"
    script.write_text(GRAPH_WORKER)
    env = dict(os.environ, ROOT=ROOT, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port), TFX_DP_FORCE_COLLECTIVE="1")
    p = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=300)
    print(p.stdout, p.stderr[-3000:])
    assert p.returncode == 0, p.stderr[-3000:]
    assert "REL" in p.stdout
