"""bench.py with N>1 ranks captures the DP step (bucketed all-reduces included) in a HIP graph by
default; when any rank cannot capture, every rank must fall back to eager together (a rank left
replaying would issue its collectives in a different order).  Exercised here with 2 ranks on the one
GPU over gloo, whose host-staged collectives cannot be captured: the capture fails on both ranks,
the bucket bookkeeping is reset, the agreement all-reduce runs, and the eager steps must still
reduce every bucket (the JSON reports 2 ranks, no graph, a finite loss)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_dp_capture_failure_falls_back_to_eager_on_every_rank():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--depth", "18",
               "--batch", "16", "--steps", "3", "--warmup", "2"]
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                      cwd=ROOT))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=300))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    if any(p.returncode != 0 for p in procs):
        log = os.path.join(ROOT, "gpurun_out", "dp_fallback_stderr.log")
        if os.path.isdir(os.path.dirname(log)):
            with open(log, "w") as f:
                for r, o in enumerate(outs):
                    f.write("==== rank %d rc=%s\n%s\n%s\n" % (r, procs[r].returncode, o[0], o[1]))
    assert all(p.returncode == 0 for p in procs), [o[1][-6000:] for o in outs]
    rec = json.loads([ln for ln in outs[0][0].splitlines() if ln.startswith("{")][0])
    assert rec["n_gpus"] == 2 and rec["config"]["backend"] == "gloo"
    assert rec["config"]["hip_graph"] is False
    assert rec["config"]["final_loss"] == rec["config"]["final_loss"]  # not NaN
    assert "running eager" in outs[0][1]
