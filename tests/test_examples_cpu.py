"""The examples/ scripts (BASELINE.json configs 1-5) run end to end on the CPU path with tiny settings,
as subprocesses exactly as a user would run them; the DP examples also run as 2 gloo ranks."""
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")


def _run(script, *args, timeout=600):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "examples", script), *args], capture_output=True,
                       text=True, timeout=timeout, env=ENV, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    return p.stdout


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(script, n, *args, timeout=900):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "examples", script), *args]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=ENV, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    return p.stdout


def _scalars(path):
    from tensorflow_examples_amd.utils.runlog import read_scalars
    return read_scalars(str(path))


def _ckpt_step(d):
    from tensorflow_examples_amd import ckpt
    p = ckpt.latest_checkpoint(str(d))
    return int(p.rsplit("-", 1)[1]) if p else None


def _graph_events(path):
    from tensorflow_examples_amd import summary
    n = 0
    for f in os.listdir(path):
        if f.startswith("events.out.tfevents."):
            n += sum(1 for ev in summary.summary_iterator(os.path.join(path, f)) if "graph_def" in ev)
    return n


def test_mnist_softmax_example(tmp_path):
    """--logs_path: cost / accuracy scalars at the log cadence + the graph (tfevents, read back); --logdir:
    periodic checkpoints, and a second run resumes from the latest one (reference conventions,
    R/distributed/distributed.py:120-138)."""
    ev, cp = tmp_path / "ev", tmp_path / "ck"
    out = _run("mnist_softmax.py", "--train_steps=200", "--log_every=100", "--data_dir=/nonexistent",
               f"--logs_path={ev}", f"--logdir={cp}", "--save_checkpoint_steps=100")
    acc = float([l for l in out.splitlines() if l.startswith("accuracy")][0].split()[1])
    assert acc > 0.8
    sc = _scalars(ev)
    assert [s for s, _ in sc["cost"]] == [100, 200] and len(sc["accuracy"]) == 2 and "test_accuracy" in sc
    assert _graph_events(ev) == 1 and os.path.exists(cp / "graph.pbtxt")
    assert _ckpt_step(cp) == 200 and os.path.exists(cp / "model.ckpt-100.index")
    out2 = _run("mnist_softmax.py", "--train_steps=300", "--log_every=100", "--data_dir=/nonexistent",
                f"--logs_path={ev}", f"--logdir={cp}")
    assert _ckpt_step(cp) == 300
    assert [s for s, _ in _scalars(ev)["cost"]] == [100, 200, 300]  # the resumed run logged step 300 only
    assert float([l for l in out2.splitlines() if l.startswith("accuracy")][0].split()[1]) > 0.8


def test_lenet5_example(tmp_path):
    ev, cp = tmp_path / "ev", tmp_path / "ck"
    out = _run("lenet5.py", "--max_steps=40", "--batch_size=64", "--data_dir=/nonexistent", f"--logdir={cp}",
               f"--logs_path={ev}", "--log_every=20", "--save_checkpoint_steps=20")
    acc = float([l for l in out.splitlines() if l.startswith("test accuracy")][0].split()[2])
    assert acc > 0.5
    assert os.path.exists(cp / "checkpoint") and _ckpt_step(cp) == 40 and os.path.exists(cp / "model.ckpt-20.index")
    sc = _scalars(ev)
    assert [s for s, _ in sc["cost"]] == [20, 40] and len(sc["accuracy"]) == 2 and _graph_events(ev) == 1
    # resume: momentum slots restored with the weights, training continues from step 40
    from tensorflow_examples_amd import ckpt
    t = ckpt.read_checkpoint(ckpt.latest_checkpoint(str(cp)))
    assert "optimizer/m" in t and float(t["optimizer/m"].abs().sum()) > 0
    _run("lenet5.py", "--max_steps=60", "--batch_size=64", "--data_dir=/nonexistent", f"--logdir={cp}",
         f"--logs_path={ev}", "--log_every=20")
    assert _ckpt_step(cp) == 60 and [s for s, _ in _scalars(ev)["cost"]] == [20, 40, 60]


def test_resnet_cifar_example_dp2(tmp_path):
    ev = tmp_path / "events"
    out = _torchrun("resnet_cifar.py", 2, "--depth=18", "--batch_size=8", "--max_steps=2", "--synthetic_train=256",
                    "--eval_examples=100", f"--logdir={tmp_path}", f"--logs_path={ev}", "--log_every=1")
    assert "test accuracy" in out and "images/sec (all GPUs)" in out and "epoch 1 test accuracy" in out
    sc = _scalars(ev)  # rank 0 only: one event file
    assert [s for s, _ in sc["cost"]] == [1, 2] and "accuracy" in sc and "learning_rate" in sc
    assert "test_accuracy" in sc and _graph_events(ev) == 1
    assert os.path.exists(tmp_path / "checkpoint")
    # TF1 Supervisor layout: graph.pbtxt + a MetaGraphDef .meta, parsed by the repo's readers
    from tensorflow_examples_amd import ckpt
    nodes = ckpt.read_graph(str(tmp_path / "graph.pbtxt"))
    assert len(nodes) > 50 and all(n["op"] == "VariableV2" for n in nodes)
    first = ckpt.latest_checkpoint(str(tmp_path))
    mg = ckpt.read_meta_graph(first)
    assert len(mg["trainable_variables"]) > 50 and mg["saver"]["version"] == 2
    # resume: the second run restores the checkpoint and trains up to the ABSOLUTE --max_steps
    out2 = _torchrun("resnet_cifar.py", 2, "--depth=18", "--batch_size=8", "--max_steps=4", "--synthetic_train=256",
                     "--eval_examples=100", f"--logdir={tmp_path}", f"--export_dir={tmp_path / 'export'}")
    second = ckpt.latest_checkpoint(str(tmp_path))
    assert int(first.rsplit("-", 1)[1]) == 2 and int(second.rsplit("-", 1)[1]) == 4, (first, second, out2[-500:])
    # SavedModel export: a SavedModel protobuf with the serving signature + the variables directory
    sm = ckpt.read_saved_model(str(tmp_path / "export"))
    assert sm["tags"] == ["serve"] and sm["schema_version"] == 1
    assert sm["signature_defs"]["serving_default"]["inputs"]["images"]["shape"] == [-1, 32, 32, 3]
    assert os.path.exists(tmp_path / "export" / "variables" / "variables.data-00000-of-00001")


def test_word2vec_example(tmp_path):
    ev, cp = tmp_path / "ev", tmp_path / "ck"
    common = ("--vocabulary_size=2000", "--log_every=100", "--corpus_words=50000", "--embedding_size=32",
              "--num_sampled=16", f"--logs_path={ev}", f"--logdir={cp}", "--save_checkpoint_steps=100")
    out = _run("word2vec.py", "--num_steps=200", *common)
    assert "Nearest to" in out and "examples/sec" in out
    losses = [float(l.split(":")[1].split()[0]) for l in out.splitlines() if l.startswith("Average loss")]
    assert losses[-1] < losses[0]
    assert [s for s, _ in _scalars(ev)["loss"]] == [100, 200] and _ckpt_step(cp) == 200
    from tensorflow_examples_amd import ckpt
    t = ckpt.read_checkpoint(ckpt.latest_checkpoint(str(cp)))
    assert int(t["skipgram/step_counter"].item()) == 200  # the batch generator's counter resumes too
    _run("word2vec.py", "--num_steps=300", *common)
    assert _ckpt_step(cp) == 300 and [s for s, _ in _scalars(ev)["loss"]] == [100, 200, 300]


def test_char_lstm_example_dp2(tmp_path):
    ev, cp = tmp_path / "ev", tmp_path / "ck"
    args = ("--hidden_size=32", "--embed_size=16", "--batch_size=4", "--num_steps=10", "--synthetic_chars=20000",
            "--log_every=20", f"--logs_path={ev}", f"--logdir={cp}", "--save_checkpoint_steps=30")
    out = _torchrun("char_lstm.py", 2, "--max_steps=60", *args)
    assert "valid perplexity" in out and "tokens/sec (all GPUs)" in out
    sc = _scalars(ev)
    assert [s for s, _ in sc["perplexity"]] == [20, 40, 60] and "valid_perplexity" in sc
    assert _ckpt_step(cp) == 60 and os.path.exists(cp / "model.ckpt-30.index")
    _torchrun("char_lstm.py", 2, "--max_steps=80", *args)
    assert _ckpt_step(cp) == 80 and [s for s, _ in _scalars(ev)["perplexity"]][-1] == 80
