"""ResNet on CIFAR-10 (BASELINE.json config 3: "CIFAR-10 ResNet-50 bf16 DP on 8xMI355X").

One process per GPU (launch with torchrun), RCCL bucketed all-reduce overlapped with backward,
fused momentum SGD with weight decay and a step-wise LR schedule, on-device augmentation
(pad-4 random crop + flip, written straight into the captured graph's static input), host->HBM
double-buffered prefetch, per-epoch test accuracy, TensorBoard scalars (``--logs_path``: cost,
accuracy, learning rate, test accuracy) and periodic checkpoints with resume (``--logdir``,
``--save_checkpoint_steps``; rank 0 writes) -- the reference's conventions
(R/distributed/distributed.py:120-138, Supervisor :129-131; utils/runlog.py).  CIFAR-10 binary files
from ``--data_dir`` when present, else synthetic.  The reported images/sec is the steady state: the
graph-capture step (with its warm-up) and the evaluations are timed apart.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/resnet_cifar.py --depth=50 --batch_size=256
"""
import itertools
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from tensorflow_examples_amd import app, ops  # noqa: E402
from tensorflow_examples_amd.ckpt import export_saved_model  # noqa: E402
from tensorflow_examples_amd.data.cifar import augment_model_input, hard_synthetic_cifar, load_cifar10  # noqa: E402
from tensorflow_examples_amd.data.pipeline import DevicePrefetcher, batches  # noqa: E402
from tensorflow_examples_amd.models.resnet import build_resnet_cifar, to_model_input  # noqa: E402
from tensorflow_examples_amd.optim import MomentumOptimizer  # noqa: E402
from tensorflow_examples_amd.parallel import GradAllReduce, broadcast_variables, init_distributed  # noqa: E402
from tensorflow_examples_amd.parallel.launch import control_device, control_group as _control_group  # noqa: E402
from tensorflow_examples_amd.train import ClassifierTrainer  # noqa: E402
from tensorflow_examples_amd.utils import runlog  # noqa: E402

flags = app.flags
flags.DEFINE_string("data_dir", "", "directory with the CIFAR-10 binary batches (synthetic if absent)")
flags.DEFINE_integer("depth", 50, "ResNet depth: 18, 34, 50, 101, 152")
flags.DEFINE_integer("batch_size", 256, "images per GPU")
flags.DEFINE_integer("epochs", 1, "training epochs")
flags.DEFINE_integer("max_steps", 0, "stop after N steps (0 = full epochs)")
flags.DEFINE_float("learning_rate", 0.1, "base LR (scaled by the number of GPUs)")
flags.DEFINE_float("weight_decay", 5e-4, "L2 weight decay")
flags.DEFINE_string("lr_boundaries", "0.5,0.75", "fractions of training where the LR drops 10x")
flags.DEFINE_float("bucket_mb", 32.0, "all-reduce bucket size (MB)")
flags.DEFINE_string("export_dir", "", "after training, export a SavedModel (saved_model.pb + variables/) here")
flags.DEFINE_integer("synthetic_train", 50000, "synthetic training-set size when no data is found")
flags.DEFINE_integer("eval_examples", 0, "evaluate on the first N test images (0 = all)")
flags.DEFINE_integer("seed", 0, "weight-initialisation seed (also offsets the data shuffle)")
flags.DEFINE_boolean("zero_init_residual", True, "start every residual branch's last BN at gamma = 0 (identity blocks "
                     "at init; --nozero_init_residual for the plain random init)")
flags.DEFINE_integer("warmup_steps", 50, "linear learning-rate warm-up over the first N steps (0 = none)")
flags.DEFINE_boolean("graph", True, "GPU: capture the training step (forward, backward with the bucketed RCCL "
                     "all-reduces, optimizer) in a HIP graph on the first batch and replay it (the capture's "
                     "warm-up trains on that batch 3 extra times); --nograph runs eager launches")
flags.DEFINE_integer("log_every", 50, "print / log scalars every N steps")
flags.DEFINE_string("data", "auto", "auto (CIFAR-10 files, else synthetic) | synthetic | hard: the overlapping "
                    "class-conditional texture task of data/cifar.py (not solved perfectly)")
runlog.define_flags(flags)
FLAGS = flags.FLAGS


def evaluate(model, xte, yte, dev, dtype):
    correct = 0.0
    with torch.no_grad():
        for i in range(0, len(xte), 500):
            x = to_model_input(torch.as_tensor(xte[i:i + 500], device=dev), dtype)
            y = torch.as_tensor(yte[i:i + 500], device=dev)
            correct += float(ops.accuracy(model(x, training=False), y)) * len(y)
    return correct / len(xte)


def main(_):
    dev = init_distributed(device="cuda" if torch.cuda.is_available() else "cpu")
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    # host-side control collectives on gloo: after the graph is captured, the RCCL communicator only
    # ever runs the captured gradient all-reduces (no eager RCCL call between replays)
    ctl = _control_group() if dist.is_initialized() else None
    cdev = control_device(ctl, dev)
    dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
    if FLAGS.data == "hard":
        xtr, ytr = hard_synthetic_cifar(FLAGS.synthetic_train, 0)
        xte, yte = hard_synthetic_cifar(10000, 1)
        synth = "hard synthetic"
    else:
        xtr, ytr, xte, yte, synth = load_cifar10(None if FLAGS.data == "synthetic" else (FLAGS.data_dir or None),
                                                 synthetic_train=FLAGS.synthetic_train)
        synth = "synthetic" if synth else "binary"
    if FLAGS.eval_examples:
        xte, yte = xte[:FLAGS.eval_examples], yte[:FLAGS.eval_examples]
    if rank == 0:
        print("CIFAR-10 %s: %d train / %d test" % (synth, len(xtr), len(xte)))
    store, model = build_resnet_cifar(device=dev, depth=FLAGS.depth, dtype=dtype, seed=FLAGS.seed,
                                      zero_init_residual=FLAGS.zero_init_residual)
    opt = MomentumOptimizer(store, FLAGS.learning_rate * world, momentum=0.9, weight_decay=FLAGS.weight_decay)
    log = runlog.RunLog(store, opt, FLAGS.logs_path, FLAGS.logdir, FLAGS.save_checkpoint_steps, rank=rank)
    start_step = log.restore()  # every rank restores the same checkpoint (then broadcast keeps them equal)
    broadcast_variables(store)
    dp = GradAllReduce(store, bucket_bytes=int(FLAGS.bucket_mb * (1 << 20))) if world > 1 else None
    trainer = ClassifierTrainer(store, model, opt, dp, fuse_zero_grad=True)  # optimizer clears the grads
    shard = np.arange(rank, len(xtr), world)
    # this rank's shard, gathered once (not a 150 MB copy at every epoch start)
    xs, ys = (xtr, ytr) if world == 1 else (xtr[shard], ytr[shard])
    steps_per_epoch = len(shard) // FLAGS.batch_size
    # an ABSOLUTE step budget (like the other examples): a resumed run trains up to `total`, not `total` more;
    # the LR boundaries / warm-up use the absolute step, and the epochs the checkpoint covers are skipped
    total = FLAGS.max_steps or steps_per_epoch * FLAGS.epochs
    bounds = [int(float(f) * total) for f in FLAGS.lr_boundaries.split(",") if f]
    step, seen = start_step, 0
    want_graph = FLAGS.graph and dev.type == "cuda"
    sync = (lambda: torch.cuda.synchronize()) if dev.type == "cuda" else (lambda: None)
    t_start = time.time()
    t0, t_eval, t_capture, t_save = None, 0.0, 0.0, 0.0  # steady state starts after the first (capture) step
    test_acc = None
    ep0 = min(start_step // max(steps_per_epoch, 1), FLAGS.epochs)
    skip = start_step - ep0 * steps_per_epoch  # batches of the resumed epoch the checkpoint already covers
    for ep in range(ep0, FLAGS.epochs):
        if step >= total:
            break
        src = batches([xs, ys], FLAGS.batch_size, seed=ep * 1000 + rank + 7919 * FLAGS.seed)
        if skip > 0:
            src, skip = itertools.islice(src, skip, None), 0
        for img, lab in DevicePrefetcher(src, dev):
            lr = FLAGS.learning_rate * world * (0.1 ** sum(step >= b for b in bounds))
            if FLAGS.warmup_steps and step < FLAGS.warmup_steps:
                lr *= (step + 1) / FLAGS.warmup_steps
            opt.set_learning_rate(lr)  # a device scalar: a replayed graph reads the new value
            if want_graph:
                want_graph = False
                tc = time.time()
                x = augment_model_input(img, dtype)
                ok = True
                try:
                    trainer.capture(x, lab)
                except Exception as e:  # eager fallback
                    print("rank %d: hip graph capture failed (%s)" % (rank, e), file=sys.stderr)
                    ok = False
                if world > 1:  # every rank replays or none does (collective order must match)
                    agree = torch.tensor([1 if ok else 0], dtype=torch.int32, device=cdev)
                    dist.all_reduce(agree, op=dist.ReduceOp.MIN, group=ctl)
                    ok = bool(agree.item())
                if not ok:
                    trainer.graph = None
                sync()
                t_capture = time.time() - tc
                if rank == 0:
                    print("hip graph: %s (capture + warm-up %.2f s, timed apart)" %
                          ("replaying the captured step" if ok else "eager launches", t_capture), flush=True)
            # graphed: crop + flip + normalise written straight into the graph's static input (one fused
            # kernel, no copy), the labels into its static label buffer
            xbuf, ybuf = trainer.input_buffer(), trainer.label_buffer()
            x = augment_model_input(img, dtype, out=xbuf)
            if ybuf is not None:
                ybuf.copy_(lab, non_blocking=True)
                lab = ybuf
            loss = trainer.step(x, lab)
            if rank == 0 and step == start_step and trainer.plan is not None:
                print(trainer.plan.table(), flush=True)  # which fusion group ran which layer (ops/fusion.py)
            step += 1
            if t0 is None:  # the first step (graph capture + its warm-up + first replay) is not steady state
                sync()
                t0 = time.time()
            else:
                seen += img.shape[0]
            if step % FLAGS.log_every == 0:
                if rank == 0:
                    with torch.no_grad():  # training-batch accuracy (the reference's summary op), eval-mode forward
                        acc = float(ops.accuracy(model(x, training=False), lab))
                    print("epoch %d step %d lr %.4f loss %.4f" % (ep + 1, step, lr, float(loss)), flush=True)
                    log.scalars(step, cost=float(loss), accuracy=acc, learning_rate=lr)
            if log.save_steps > 0 and step % log.save_steps == 0 and FLAGS.logdir:
                sync()
                ts = time.time()
                log.maybe_save(step)  # device -> host copy + file write, timed apart like the evaluations
                if world > 1:  # every rank waits here, so every rank subtracts the same interval
                    dist.barrier(group=ctl)
                t_save += time.time() - ts
            if step >= total:
                break
        # per-epoch test accuracy (rank 0), timed apart: the other ranks wait at a control-group barrier
        # inside the same interval (not in the next collective, which would count as training time)
        sync()
        te = time.time()
        if rank == 0:
            test_acc = evaluate(model, xte, yte, dev, dtype)
            print("epoch %d test accuracy %.4f" % (ep + 1, test_acc), flush=True)
            log.scalars(step, test_accuracy=test_acc)
        if world > 1:
            dist.barrier(group=ctl)
        t_eval += time.time() - te
    sync()
    t_end = time.time()
    dt = max((t_end - t0) - t_eval - t_save, 1e-9) if t0 is not None else 1e-9
    ips = torch.tensor([seen / dt], dtype=torch.float64, device=cdev)
    if world > 1:
        dist.all_reduce(ips, group=ctl)
    if test_acc is None and rank == 0:
        test_acc = evaluate(model, xte, yte, dev, dtype)
    if rank == 0:
        print("test accuracy %.4f" % test_acc)
        print("images/sec (all GPUs) %.1f" % float(ips))
        print("end-to-end %.1f s: steady-state training %.1f s, graph capture %.1f s, evaluation %.1f s, "
              "checkpoints %.1f s" % (t_end - t_start, dt, t_capture, t_eval, t_save))
    saved = log.close(step)
    if rank == 0:
        if saved:
            print("saved", saved)
        if FLAGS.export_dir:
            sig = {"serving_default": {"inputs": {"images": ("images:0", "uint8", [-1, 32, 32, 3])},
                                       "outputs": {"logits": ("logits:0", "float32", [-1, 10])}}}
            print("exported", export_saved_model(store, FLAGS.export_dir, {"model": "resnet%d" % FLAGS.depth},
                                                 signature_defs=sig))
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    app.run(main)
