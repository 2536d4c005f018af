'''

This trains a very simple SNN on mnist data with asynchronous parameter-server data parallelism,
on tensorflow_examples_amd (MI355X-native re-implementation of R/distributed/distributed.py:
same flags, roles, placement, async semantics, console output and TensorBoard event files).

To run (simulated on one host on independent ports, as the reference does):

python distributed.py  --ps_hosts=127.0.0.1:2222  --worker_hosts=127.0.0.1:2223,127.0.0.1:2224  --job_name=ps --task_index=0
python distributed.py  --ps_hosts=127.0.0.1:2222  --worker_hosts=127.0.0.1:2223,127.0.0.1:2224  --job_name=worker --task_index=0
python distributed.py  --ps_hosts=127.0.0.1:2222  --worker_hosts=127.0.0.1:2223,127.0.0.1:2224  --job_name=worker --task_index=1

Workers use the GPU (one per worker, cuda:<task_index % n_gpus>) when present, else the CPU.
Documented deviations: "Time Taken" is printed with "%.2fs" (the reference's "2fs" format raises
TypeError at :165); the ps does not load MNIST (Q5); missing --ps_hosts/--worker_hosts
give a usage error instead of AttributeError (Q12).

'''
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tensorflow_examples_amd import app  # noqa: E402

# flags for input defined here
flags = app.flags
app.flags.DEFINE_string("job_name", "", "Either 'ps' or 'worker'")
app.flags.DEFINE_integer("task_index", 0, "Index of task within the job")
flags.DEFINE_string("worker_hosts", None,
                    "The worker url list, separated by comma (e.g. tf-worker1:2222,1.2.3.4:2222)")
flags.DEFINE_string("ps_hosts", None,
                    "The ps url list, separated by comma (e.g. tf-ps2:2222,1.2.3.5:2222)")
# opt-in flags of this framework (defaults reproduce the reference)
flags.DEFINE_string("device", "auto", "auto | cuda | cpu")
flags.DEFINE_string("data_dir", "MNIST_data", "MNIST IDX directory (synthetic MNIST if absent)")
flags.DEFINE_integer("training_epochs", 50, "epochs per worker")
flags.DEFINE_integer("batch_size", 100, "batch size")
flags.DEFINE_float("learning_rate", 0.001, "SGD learning rate")
flags.DEFINE_string("logs_path", "/tmp/mnist/", "TensorBoard event directory")
flags.DEFINE_string("logdir", "", "checkpoint directory: enables Supervisor save/restore")
flags.DEFINE_float("recovery_wait_secs", 30.0, "non-chief readiness poll interval (TF1 default 30 s)")
flags.DEFINE_integer("max_batches_per_epoch", 0, "cap batches per epoch (0 = num_examples / batch_size)")
flags.DEFINE_boolean("stable_xent", False, "log-softmax cross entropy instead of the reference's log(softmax)")
flags.DEFINE_boolean("ps_exit_after_workers", False, "ps exits once every worker has finished")
flags.DEFINE_boolean("sync_replicas", False, "aggregate all workers' gradients per global step "
                     "(SyncReplicasOptimizer semantics, R/distributed/distributed.py:109-112)")
flags.DEFINE_integer("sync_port_offset", 1000, "worker-group rendezvous port = worker 0 port + offset")
flags.DEFINE_string("transport", "tcp", "ps data path: tcp (portable) | xgmi (same-node GPUs: the ps arena "
                    "is mapped into every worker over xGMI peer memory, SURVEY.md §5.8)")
flags.DEFINE_integer("xgmi_arena_mb", 64, "size of each ps task's xGMI arena")
flags.DEFINE_boolean("graph", True, "xGMI async workers: run the step as one HIP graph (feed, pull, fwd, bwd, "
                     "peer SGD, step bump) and read cost / accuracy back at the log cadence")
flags.DEFINE_integer("ps_device", -1, "GPU of the ps arena with --transport=xgmi (-1: task_index % n_gpus)")
flags.DEFINE_integer("save_checkpoint_steps", 0, "chief saves a checkpoint into --logdir every N local steps "
                     "(0 = only at the end; TF1 Supervisor saves on a timer when logdir is set)")
FLAGS = app.flags.FLAGS

if not FLAGS.ps_hosts or not FLAGS.worker_hosts:
    sys.stderr.write("usage: distributed.py --ps_hosts=h:p[,h:p] --worker_hosts=h:p[,h:p] "
                     "--job_name=ps|worker --task_index=N\n")
    sys.exit(2)

from tensorflow_examples_amd.cluster import ClusterSpec, Server  # noqa: E402

# creating a cluster using the flags defined above
cluster = ClusterSpec({"ps": FLAGS.ps_hosts.split(","), "worker": FLAGS.worker_hosts.split(",")})

# start a server for a specific task
server = Server(cluster, job_name=FLAGS.job_name, task_index=FLAGS.task_index)

# training configurations
batch_size = FLAGS.batch_size
learning_rate = FLAGS.learning_rate
training_epochs = FLAGS.training_epochs
logs_path = FLAGS.logs_path
DONE = "__workers_done__"

if FLAGS.job_name == "ps":
    if FLAGS.transport == "xgmi":
        # the ps owns its variables in one GPU arena that every worker maps over xGMI
        import torch
        from tensorflow_examples_amd.cluster.xgmi import XgmiArena
        ps_dev = FLAGS.ps_device if FLAGS.ps_device >= 0 else FLAGS.task_index % max(1, torch.cuda.device_count())
        torch.cuda.set_device(ps_dev)
        arena = XgmiArena(server, FLAGS.xgmi_arena_mb << 20, ps_dev)
    if FLAGS.ps_exit_after_workers:
        n_workers = cluster.num_tasks("worker")
        while True:
            v = server.read(DONE, 1)
            if v is not None and v[0] >= n_workers:
                break
            time.sleep(0.5)
        server.stop()
    else:
        server.join()
elif FLAGS.job_name == "worker":
    import torch

    from tensorflow_examples_amd import summary
    from tensorflow_examples_amd.cluster.ps import PSClient
    from tensorflow_examples_amd.cluster.supervisor import Supervisor
    from tensorflow_examples_amd.data.mnist import read_data_sets
    from tensorflow_examples_amd.models.mnist_mlp import MnistMLP
    from tensorflow_examples_amd.parallel.ps_worker import (AsyncPSWorker, GraphedPSLoop, SyncReplicasPSWorker,
                                                            init_worker_group)
    from tensorflow_examples_amd.utils import fault
    from tensorflow_examples_amd.variables import VariableStore

    # load training examples, read with one_hot set to true
    mnist = read_data_sets(FLAGS.data_dir, one_hot=True, seed=FLAGS.task_index)

    if FLAGS.device == "cpu" or not torch.cuda.is_available():
        torch.set_num_threads(max(1, (os.cpu_count() or 2) // (cluster.num_tasks("worker") + 1)))
    use_cuda = FLAGS.device == "cuda" or (FLAGS.device == "auto" and torch.cuda.is_available())
    device = torch.device("cuda", FLAGS.task_index % max(1, torch.cuda.device_count())) if use_cuda else \
        torch.device("cpu")
    if use_cuda:
        torch.cuda.set_device(device)

    # <--- Between-graph replication: every worker builds its own replica of the model --->
    store = VariableStore(device=device, compute_dtype=torch.float32, seed=2)  # tf.set_random_seed(2)
    model = MnistMLP(store)
    store.finalize()
    if FLAGS.transport == "xgmi":
        from tensorflow_examples_amd.cluster.xgmi import XgmiPSClient
        client = XgmiPSClient(cluster, store)
    else:
        client = PSClient(cluster, store)
    # done-counter for --ps_exit_after_workers lives on every ps task
    if FLAGS.sync_replicas:
        group = init_worker_group(FLAGS.worker_hosts.split(","), FLAGS.task_index, FLAGS.sync_port_offset)
        worker = SyncReplicasPSWorker(model, client, learning_rate, group, is_chief=(FLAGS.task_index == 0),
                                      naive_xent=not FLAGS.stable_xent)
    else:
        worker = AsyncPSWorker(model, client, learning_rate, naive_xent=not FLAGS.stable_xent)

    cost_v, acc_v = [0.0], [0.0]
    summary.scalar("cost", lambda: cost_v[0])
    summary.scalar("accuracy", lambda: acc_v[0])
    summary_op = summary.merge_all()
    print("Variables initialized ...")

    sv = Supervisor(is_chief=(FLAGS.task_index == 0), client=client, logdir=FLAGS.logdir or None,
                    recovery_wait_secs=FLAGS.recovery_wait_secs,
                    graph_nodes=lambda: model.graph_nodes(lambda n: client.shard_map().get(n, "")))

    begin_time = time.time()
    frequency = 100
    fault.before_init()  # TFX_FAULT hooks: recovery tests
    with sv.prepare_or_wait_for_session() as sess:
        if FLAGS.task_index == 0 and FLAGS.ps_exit_after_workers:
            import ctypes
            from tensorflow_examples_amd import runtime
            import numpy as np
            z = np.zeros(1, np.float32)
            for h in client.handles:  # every ps task counts finished workers (each exits on its own count)
                runtime.lib().tfx_ps_create(h, 1, (ctypes.c_char_p * 1)(DONE.encode()),
                                            (ctypes.c_void_p * 1)(z.ctypes.data), (ctypes.c_uint64 * 1)(4), 0)

        # this will log on every node of our cluster
        placement = client.shard_map()
        writer = summary.FileWriter(logs_path, graph=model.graph_nodes(lambda n: placement.get(n, "")))

        # xGMI async worker: the whole step is one HIP graph; cost / accuracy / global step land in a
        # device ring read back at the log cadence, where that interval's per-step summaries are written
        runner = None
        if FLAGS.graph and FLAGS.transport == "xgmi" and not FLAGS.sync_replicas and use_cuda and \
                mnist.train.num_examples % batch_size == 0:
            runner = GraphedPSLoop(worker, mnist.train, batch_size, ring=frequency + 1)

        def flush():
            rows = runner.read()
            for c, a, st in rows:
                cost_v[0], acc_v[0] = c, a
                writer.add_summary(summary_op(), st)
            return rows[-1] if rows else (cost_v[0], acc_v[0], step)

        start_time = time.time()
        cost = 0.0
        step = 0
        local_steps = 0
        for epoch in range(training_epochs):
            batch_count = int(mnist.train.num_examples / batch_size)
            if FLAGS.max_batches_per_epoch:
                batch_count = min(batch_count, FLAGS.max_batches_per_epoch)

            count = 0
            for i in range(batch_count):
                if runner is not None:
                    runner.step()
                    local_steps += 1
                    if FLAGS.logdir and FLAGS.save_checkpoint_steps and local_steps % FLAGS.save_checkpoint_steps == 0:
                        cost, _, step = flush()
                        sv.save(step + 1)
                    if fault.armed():
                        # runner.step() only enqueued the replay: complete its pushes to the ps first
                        torch.cuda.synchronize()
                    fault.after_step(local_steps)
                    if (count + 1) % frequency == 0 or i + 1 == batch_count:
                        cost, _, step = flush()
                else:
                    batch_x, batch_y = mnist.train.next_batch(batch_size)

                    cost, acc, step = worker.step(batch_x, batch_y)
                    cost_v[0], acc_v[0] = cost, acc
                    writer.add_summary(summary_op(), step)
                    local_steps += 1
                    if FLAGS.logdir and FLAGS.save_checkpoint_steps and local_steps % FLAGS.save_checkpoint_steps == 0:
                        sv.save(step + 1)
                    fault.after_step(local_steps)

                count += 1
                if count % frequency == 0 or i + 1 == batch_count:
                    elapsed_time = time.time() - start_time
                    start_time = time.time()
                    print("Step so far: %d," % (step + 1),
                          " Epoch so far: %2d," % (epoch + 1),
                          " Batch used: %3d of %3d," % (i + 1, batch_count),
                          " Cost now: %.4f," % cost,
                          " Time spent (delta): %3.1fms" % float(elapsed_time * 1000 / frequency), flush=True)
                    count = 0

        print("Acc: %2.2f" % worker.evaluate(mnist.test.images, mnist.test.labels))
        print("Time Taken: %.2fs" % float(time.time() - begin_time))
        print("Final Computed Cost: %.2f" % cost)
        if FLAGS.logdir:
            sv.save(step + 1)
        writer.close()
        if FLAGS.ps_exit_after_workers:
            from tensorflow_examples_amd import runtime
            import ctypes
            for h in client.handles:
                runtime.lib().tfx_ps_inc(h, DONE.encode(), 1.0, ctypes.byref(ctypes.c_double()))

    sv.stop()
    print("done with training")
