#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 / CIFAR-10 bf16 training throughput (images/sec, whole job).

BASELINE.json metric: "images/sec (whole node) ResNet-50/CIFAR-10 bf16 at 1/2/4/8 MI355X".
One process per GPU, RCCL bucketed all-reduce overlapped with backward, fused momentum-SGD on the
flat master buffer.  Weak scaling: ``--batch`` images per GPU, global batch = batch * N.
Synthetic CIFAR-shaped data (uint8 32x32x3 images + int64 labels), random-init weights: there is
no dataset or network on the box.

Launch modes (the process-per-task model of R/distributed/distributed.py:7-14,37-43):
* ``python bench.py --gpus N`` with no RANK in the environment: this process is only a launcher --
  it never touches the GPU, spawns N fresh ranks of itself (parallel/launch.py ``spawn_local``,
  rendezvous on 127.0.0.1), relays rank 0's JSON line and exits non-zero if any rank fails;
* under ``torch.distributed.run`` each rank process is a supervisor that never touches the GPU and
  runs the real rank as a child (parallel/launch.py ``supervise_rank``);
* either way the job cannot end without a result line inside ``--launch-timeout`` (default 480 s,
  below the driver's 600 s lease): attempt 1 (HIP-graph-replayed DP step) gets half of it; if any
  rank fails or hangs, every rank is killed and the job reruns ONCE as fresh processes with
  ``TFX_DP_GRAPH=0`` (eager RCCL collectives) on a new rendezvous.  The JSON says which attempt
  produced it (``config.attempt``, ``config.hip_graph``).  ``TFX_BENCH_HANG=<rank>:<attempt>`` makes
  that rank hang before its first step (test hook);
* every rank checks that the process group spans exactly ``--gpus`` ranks (size + an all-reduce of
  ones) before timing; ``n_gpus`` / ``config.rccl_ranks`` in the JSON are that verified size.

Timing: W untimed warmup steps; barrier + synchronize; K timed steps; barrier + synchronize; the
MAX elapsed over ranks is reported.  Rank 0 prints ONE JSON line.

``--host-input [zerocopy|copy|none]``: by default (``zerocopy``) the batches live in pinned host memory
(the tf.data/feed_dict path) and go through the framework's pinned ring (data/pipeline.py): the fused
input kernel reads the pinned slot over the host link every step; ``copy`` -- an async H2D copy per
step on a side stream into device slots; ``none`` -- batches resident on the device.
``--impl torch`` runs a stock PyTorch-ROCm eager ResNet-50 (torch.nn + MIOpen, channels_last, bf16
autocast) for a labelled comparison; the headline is ``--impl native``.
``--device cpu`` runs the same step on the CPU reference ops over gloo (tests of the launch path).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec (whole node) ResNet-50/CIFAR-10 bf16 at 1/2/4/8 MI355X"
BASELINE_VALUE = None  # the reference publishes no number for this metric


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU) of the job")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="images per GPU")
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--impl", choices=["native", "torch"], default="native")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda")
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--allreduce-dtype", choices=["f32", "bf16"], default="bf16",
                    help="gradient wire format of the bucketed all-reduce (N > 1): bf16 (default: cast per bucket "
                         "into a persistent bf16 twin, reduced in place, read by the optimizer directly -- half the "
                         "ring bytes; 300-step convergence within 0.45 %% of the f32 wire, profiles/r06_dp_wire, "
                         "tests/test_convergence_gpu.py) or f32")
    ap.add_argument("--graph", dest="graph", action="store_true", default=True,
                    help="capture the whole step in a HIP graph and replay it (default on; for N>1 the bucketed "
                         "RCCL all-reduces are captured too -- measured on a 1-rank RCCL group: 8.09-8.16 ms graph vs "
                         "8.27-9.03 ms eager, profiles/r02_final/dp_graph_ab.txt; TFX_DP_GRAPH=0 keeps N>1 eager)")
    ap.add_argument("--no-graph", dest="graph", action="store_false", help="eager step launches")
    ap.add_argument("--host-input", nargs="?", const="zerocopy", default="zerocopy", choices=["copy", "zerocopy", "none"],
                    help="where the batches live: 'zerocopy' (default) = pinned host memory, the input kernel reads "
                         "the pinned slot over the host link (the north star's pinned-host input pipeline); 'copy' = "
                         "pinned host memory, async H2D into device slots on a side stream (data/pipeline.py "
                         "PinnedRing); 'none' = batches resident on the device")
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--nbatches", type=int, default=4, help="distinct synthetic batches cycled")
    ap.add_argument("--backend", default=None, help="process-group backend (default nccl = RCCL, gloo on cpu)")
    ap.add_argument("--launch-timeout", type=float, default=480.0,
                    help="N>1: seconds by which the job must have produced its result line (both attempts)")
    ap.add_argument("--attempt-timeout", type=float, default=None,
                    help="N>1: seconds for attempt 1 before the eager fallback (default: half of --launch-timeout)")
    return ap.parse_args(argv)


def synthetic_batches(n, batch, seed):
    import torch
    g = torch.Generator(device="cpu").manual_seed(seed)
    out = []
    for _ in range(n):
        img = torch.randint(0, 256, (batch, 32, 32, 3), dtype=torch.uint8, generator=g)
        lab = torch.randint(0, 10, (batch,), dtype=torch.long, generator=g)
        out.append((img, lab))
    return out


def run(a):
    import torch
    import torch.distributed as dist

    from tensorflow_examples_amd.data.pipeline import PinnedRing
    from tensorflow_examples_amd.models.resnet import build_resnet_cifar, to_model_batch, to_model_input
    from tensorflow_examples_amd.optim import MomentumOptimizer
    from tensorflow_examples_amd.parallel import GradAllReduce, broadcast_variables, init_distributed
    from tensorflow_examples_amd.parallel.launch import control_device, control_group as _control_group, verify_world
    from tensorflow_examples_amd.train import ClassifierTrainer

    cuda = a.device == "cuda"
    dev = init_distributed(backend=a.backend, device=a.device)
    world = dist.get_world_size() if dist.is_initialized() else 1
    forced = dist.is_initialized() and world == 1  # TFX_DP_FORCE_COLLECTIVE rehearsal of the RCCL path
    ranks = 1
    if "RANK" in os.environ or a.gpus > 1:
        ranks = verify_world(a.gpus if not forced else 1, dev)
    rank = dist.get_rank() if dist.is_initialized() else 0
    # host-side control collectives (capture agreement, timing barriers, elapsed-time MAX) run on a
    # gloo group: the RCCL communicator then carries only the gradient all-reduces, and no eager RCCL
    # call is ever interleaved with replays of a graph that holds captured RCCL collectives
    ctl = _control_group() if dist.is_initialized() else None
    cdev = control_device(ctl, dev)
    torch.manual_seed(1234 + rank)
    host = synthetic_batches(a.nbatches, a.batch, seed=1000 + rank)
    dtype = torch.bfloat16 if cuda else torch.float32

    def sync():
        if cuda:
            torch.cuda.synchronize()

    ring = None
    if a.host_input != "none" and cuda:
        ring = PinnedRing.for_batches(host, dev, depth=2, zero_copy=a.host_input == "zerocopy")
        data = None
    else:
        data = [(img.to(dev), lab.to(dev)) for img, lab in host]

    def batch(i):
        if ring is not None:
            return ring.next()
        return data[i % len(data)]

    graphed = False
    if a.impl == "native":
        store, model = build_resnet_cifar(device=dev, depth=a.depth, dtype=dtype, seed=0)
        broadcast_variables(store)
        opt = MomentumOptimizer(store, a.lr, momentum=0.9, weight_decay=5e-4)
        dp = GradAllReduce(store, bucket_bytes=int(a.bucket_mb * (1 << 20)),
                           compress_bf16=a.allreduce_dtype == "bf16") if dist.is_initialized() else None
        # the optimizer kernel clears the gradients in its pass: no gradient fill launch in the step
        trainer = ClassifierTrainer(store, model, opt, dp, fuse_zero_grad=True)

        label_fuse = os.environ.get("TFX_LABEL_FUSE", "1") == "1"  # 0: separate label copy (A/B)

        def step(i):
            img, lab = batch(i)
            # graphed: the input kernel writes straight into the graph's static input and label
            # buffers (zero-copy ring: reading the pinned host slot over the host link)
            x, y = to_model_batch(img, lab, dtype=dtype, device=dev, out=trainer.input_buffer(),
                                  labels_out=trainer.label_buffer() if label_fuse else None)
            return trainer.step(x, y)

        if cuda and a.graph and ((world == 1 and not forced) or os.environ.get("TFX_DP_GRAPH", "1") == "1"):
            # the captured step is the same work (forward, backward with the bucketed RCCL
            # all-reduces, fused optimizer) replayed with one launch; the per-step input batch is
            # copied into the graph's static input
            img, lab = batch(0)
            try:
                trainer.capture(to_model_input(img, device=dev), lab.to(dev))
                graphed = True
            except Exception as e:  # pragma: no cover - capture is best effort, eager is the fallback
                print("rank %d: hip graph capture failed (%s)" % (rank, e), file=sys.stderr)
            if world > 1 or forced:
                # every rank replays its graph or none does: a rank left eager would issue its
                # collectives in a different order from the graph replays of the others
                agree = torch.tensor([1 if graphed else 0], dtype=torch.int32, device=cdev)
                dist.all_reduce(agree, op=dist.ReduceOp.MIN, group=ctl)
                graphed = bool(agree.item())
            if not graphed:
                if rank == 0:
                    print("hip graph capture not used on every rank; running eager", file=sys.stderr)
                trainer.graph = None
        nparams = store.num_params()
    else:
        from tensorflow_examples_amd.models.torch_baseline import TorchResNet50Cifar
        net = TorchResNet50Cifar().to(dev).to(memory_format=torch.channels_last)
        if world > 1:
            net = torch.nn.parallel.DistributedDataParallel(net, device_ids=[dev.index] if cuda else None,
                                                            bucket_cap_mb=a.bucket_mb)
        topt = torch.optim.SGD(net.parameters(), lr=a.lr, momentum=0.9, weight_decay=5e-4, foreach=True)
        mean = torch.tensor([0.4914, 0.4822, 0.4465], device=dev).view(1, 3, 1, 1)
        std = torch.tensor([0.2470, 0.2435, 0.2616], device=dev).view(1, 3, 1, 1)
        nparams = sum(p.numel() for p in net.parameters())

        def step(i):
            img, lab = batch(i)
            if img.device != dev:  # zero-copy ring: stock torch has no zero-copy kernel, copy H2D
                img, lab = img.to(dev, non_blocking=True), lab.to(dev, non_blocking=True)
            x = ((img.permute(0, 3, 1, 2).float() / 255.0 - mean) / std).contiguous(memory_format=torch.channels_last)
            topt.zero_grad(set_to_none=True)
            with torch.autocast(dev.type, dtype=torch.bfloat16):
                loss = torch.nn.functional.cross_entropy(net(x), lab)
            loss.backward()
            topt.step()
            return loss.detach()

    hang = os.environ.get("TFX_BENCH_HANG", "")
    if hang and hang == "%d:%s" % (rank, os.environ.get("TFX_BENCH_ATTEMPT", "1")):
        print("rank %d: TFX_BENCH_HANG -- hanging before the first step" % rank, file=sys.stderr, flush=True)
        time.sleep(1e6)
    for i in range(a.warmup):
        loss = step(i)
    if rank == 0 and a.impl == "native" and getattr(trainer, "plan", None) is not None:
        print(trainer.plan.table(), file=sys.stderr, flush=True)  # the fusion plan the step runs (stderr)
    sync()
    if world > 1:
        dist.barrier(group=ctl)
    sync()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = step(i)
    sync()
    if world > 1:
        dist.barrier(group=ctl)
    sync()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX, group=ctl)
    elapsed = float(el.item())
    final_loss = float(loss.float().item())
    images = a.batch * world * a.steps
    value = images / elapsed
    if rank == 0:
        rec = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed * 1000 / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(value / BASELINE_VALUE, 4) if BASELINE_VALUE else None),
            "dtype": "bf16" if dtype == torch.bfloat16 else "fp32",
            "data": "synthetic (CIFAR-10-shaped uint8 32x32x3 images, random labels, random-init weights)"
                    + ({"copy": "; pinned-host batches copied H2D every step",
                        "zerocopy": "; pinned-host batches read by the input kernel every step (zero-copy)"}
                       [a.host_input] if ring is not None else "; batches resident on the device"),
            "config": {
                "model": "ResNet-%d (CIFAR-10 adaptation: 3x3 stem, bottleneck [3,4,6,3])" % a.depth,
                "global_batch": a.batch * world,
                "per_gpu_batch": a.batch,
                "seq_len": None,
                "image_hw": [32, 32],
                "parallelism": "dp%d" % world,
                "device": a.device,
                "backend": dist.get_backend() if dist.is_initialized() else None,
                "rccl_ranks": ranks if (dist.is_initialized() and dist.get_backend() == "nccl") else None,
                "verified_ranks": ranks,
                "attempt": int(os.environ.get("TFX_BENCH_ATTEMPT", "1")),
                "impl": a.impl,
                "optimizer": "momentum-SGD 0.9, wd 5e-4 (fused flat-buffer kernel)" if a.impl == "native" else "torch.optim.SGD foreach",
                "allreduce_bucket_mb": a.bucket_mb,
                "allreduce_dtype": a.allreduce_dtype,
                "hip_graph": bool(a.impl == "native" and graphed),
                "host_input": a.host_input if ring is not None else False,
                "params": nparams,
                "final_loss": round(final_loss, 4),
            },
        }
        print(json.dumps(rec), flush=True)
    if ring is not None:
        ring.close()
    if dist.is_initialized():
        dist.destroy_process_group()


FALLBACK_ENV = {"TFX_DP_GRAPH": "0"}  # attempt 2: eager RCCL collectives instead of graph replay


def main(argv=None):
    a = parse(argv)
    from tensorflow_examples_amd.parallel.launch import (can_supervise, launch_with_fallback, supervise_rank,
                                                         under_launcher)
    args = [os.path.abspath(__file__), *list(sys.argv[1:] if argv is None else argv)]
    if a.gpus > 1 and not under_launcher():
        # launcher mode: this process never initialises the GPU; the ranks are fresh processes
        return launch_with_fallback(a.gpus, args, a.launch_timeout, FALLBACK_ENV, a.attempt_timeout)
    if a.gpus > 1 and can_supervise():
        # one torch.distributed.run rank: supervise the real rank as a child (never touch the GPU here)
        return supervise_rank(args, a.launch_timeout, FALLBACK_ENV, a.attempt_timeout)
    run(a)
    return 0


if __name__ == "__main__":
    sys.exit(main())
