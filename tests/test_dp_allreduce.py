"""Synchronous data parallel (GradAllReduce) over gloo, world_size 2, on CPU."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tensorflow_examples_amd import ops
from tensorflow_examples_amd.models.mnist_mlp import MnistMLP
from tensorflow_examples_amd.optim import MomentumOptimizer
from tensorflow_examples_amd.parallel import GradAllReduce, broadcast_variables
from tensorflow_examples_amd.variables import VariableStore


def _data(seed=0, n=64):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(n, 784, generator=g), torch.randint(0, 10, (n,), generator=g)


def _model(seed):
    st = VariableStore("cpu", seed=seed)
    m = MnistMLP(st)
    st.finalize()
    return st, m


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    st, m = _model(seed=10 + rank)  # different init per rank: broadcast must fix it
    broadcast_variables(st)
    dp = GradAllReduce(st, bucket_bytes=2048)  # several buckets
    opt = MomentumOptimizer(st, 0.1, momentum=0.9)
    x, y = _data()
    per = x.shape[0] // world
    xs, ys = x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per]
    for _ in range(3):
        st.zero_grad()
        loss = ops.softmax_cross_entropy(m.logits(xs), ys, naive=False)
        loss.backward()
        dp.finish()
        opt.apply_gradients(grad_scale=dp.grad_scale)
    out[rank] = (st.master.clone(), len(dp.buckets))
    dist.destroy_process_group()


def test_dp_matches_single_process_full_batch():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(2, port, out), nprocs=2, join=True, start_method="spawn")
    (p0, nb0), (p1, nb1) = out[0], out[1]
    assert nb0 >= 2
    assert torch.equal(p0, p1)  # replicas stay bit-identical
    # single process, full batch, rank-0 initial weights
    st, m = _model(seed=10)
    opt = MomentumOptimizer(st, 0.1, momentum=0.9)
    x, y = _data()
    for _ in range(3):
        st.zero_grad()
        # mean over the full batch == average of the two half-batch means
        l0 = ops.softmax_cross_entropy(m.logits(x[:32]), y[:32])
        l1 = ops.softmax_cross_entropy(m.logits(x[32:]), y[32:])
        ((l0 + l1) / 2).backward()
        opt.apply_gradients()
    assert torch.allclose(st.master, p0, atol=1e-5, rtol=1e-5)


def test_force_collective_flag_without_process_group():
    """TFX_DP_FORCE_COLLECTIVE only takes effect with an initialised process group."""
    import torch
    from tensorflow_examples_amd.parallel import GradAllReduce
    from tensorflow_examples_amd.variables import VariableStore, Zeros
    store = VariableStore(device="cpu", compute_dtype=torch.float32, seed=0)
    store.variable([4], Zeros(), name="a")
    store.finalize()
    dp = GradAllReduce(store, force_collective=True)
    assert not dp.force and dp.world == 1
    dp.finish()  # no collectives issued, no error
