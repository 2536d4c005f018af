"""Parameter-server client + asynchronous between-graph data parallelism.

Replaces the per-step traffic of the reference worker's ``sess.run([train_op, cross_entropy,
summary_op, global_step])`` (R/distributed/distributed.py:148-150):

* PULL: one request per ps task returns all of that task's variables (X1-X4) straight into a
  pinned host staging buffer laid out like the flat variable store, then ONE host->device copy;
* PUSH: one device->host copy of the flat grad buffer, then one request per ps task carrying
  that task's gradients; the ps applies ``p -= lr * g`` (ApplyGradientDescent, lock-free like
  TF's use_locking=False) and the task holding ``global_step`` increments it (AssignAdd) and
  returns the new value (X9).
Workers never synchronise with each other: updates interleave Hogwild-style, exactly the
reference's asynchronous semantics.  The transport is the native TCP service
(csrc/runtime/ps_service.cpp); all socket work runs in C++ (ctypes calls release the GIL).
"""
from __future__ import annotations

import ctypes as C
import time
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .. import runtime
from ..variables import VariableStore
from . import ClusterSpec, parse_address, replica_device_setter

GLOBAL_STEP = "global_step"


class PSError(RuntimeError):
    pass


class _Shard:
    """The variables of one ps task, with ctypes arrays prepared once."""

    def __init__(self, handle, names: List[str], host_views: List[np.ndarray]):
        self.h = handle
        self.names = names
        n = len(names)
        self.c_names = (C.c_char_p * n)(*[s.encode() for s in names])
        self.c_ptrs = (C.c_void_p * n)(*[v.ctypes.data for v in host_views])
        self.c_sizes = (C.c_uint64 * n)(*[v.nbytes for v in host_views])
        self.n = n


class PSClient:
    def __init__(self, cluster: ClusterSpec, store: VariableStore, connect_timeout_s: float = 60.0,
                 ps_job: str = "ps"):
        self.cluster = ClusterSpec(cluster)
        self.store = store
        self.num_ps = self.cluster.num_tasks(ps_job)
        names = [GLOBAL_STEP] + [v.name for v in store.vars]  # global_step is created first (:68)
        self.placement: Dict[str, int] = replica_device_setter(self.cluster, ps_job)(names)
        # pinned host staging buffers, same flat layout as the store (+1 slot for global_step)
        pin = store.device.type == "cuda"
        self.host_vals = torch.zeros(store.total, dtype=torch.float32, pin_memory=pin)
        self.host_grads = torch.zeros(store.total, dtype=torch.float32, pin_memory=pin)
        self.step_val = np.zeros(1, np.float32)
        hv, hg = self.host_vals.numpy(), self.host_grads.numpy()
        self.handles = []
        for t in range(self.num_ps):
            host, port = parse_address(self.cluster.task_address(ps_job, t))
            h = runtime.lib().tfx_ps_connect(host.encode(), port, int(connect_timeout_s * 1000))
            if not h:
                raise PSError(f"cannot reach ps task {t} at {host}:{port} within {connect_timeout_s}s")
            self.handles.append(h)
        self.pull_shards: List[_Shard] = []
        self.push_shards: List[_Shard] = []
        for t in range(self.num_ps):
            vs = [v for v in store.vars if self.placement[v.name] == t]
            nm = ([GLOBAL_STEP] if self.placement[GLOBAL_STEP] == t else []) + [v.name for v in vs]
            pv = ([self.step_val] if self.placement[GLOBAL_STEP] == t else []) + \
                 [hv[v.offset:v.offset + v.numel] for v in vs]
            self.pull_shards.append(_Shard(self.handles[t], nm, pv))
            tv = [v for v in vs if v.trainable]
            self.push_shards.append(_Shard(self.handles[t], [v.name for v in tv],
                                           [hg[v.offset:v.offset + v.numel] for v in tv]))
        self.step_task = self.placement[GLOBAL_STEP]

    def shard_map(self) -> Dict[str, str]:
        return {n: f"/job:ps/task:{t}" for n, t in self.placement.items()}

    # ---------------------------------------------------------------- init / readiness
    def initialize(self, force: bool = True, global_step: float = 0.0) -> int:
        """Chief: write the store's current values (+global_step) to the ps tasks.
        force=True re-initialises (TF1 chief without a checkpoint re-runs init_op)."""
        self.host_vals.copy_(self.store.master.detach().cpu())
        self.step_val[0] = global_step
        done = 0
        for sh in self.pull_shards:
            r = runtime.lib().tfx_ps_create(sh.h, sh.n, sh.c_names, sh.c_ptrs, sh.c_sizes, int(force))
            if r == -2:
                raise PSError("a variable already exists on the ps with a different shape (model mismatch)")
            if r < 0:
                raise PSError("ps connection lost during initialisation")
            done += r
        return done

    def num_uninitialized(self) -> int:
        tot = 0
        for sh in self.pull_shards:
            r = runtime.lib().tfx_ps_uninitialized(sh.h, sh.n, sh.c_names)
            if r < 0:
                raise PSError("ps connection lost")
            tot += r
        return tot

    # ---------------------------------------------------------------- per-step traffic
    def pull(self) -> int:
        """Fetch every variable into the store (one request per ps task + one H2D copy)."""
        for sh in self.pull_shards:
            r = runtime.lib().tfx_ps_pull(sh.h, sh.n, sh.c_names, sh.c_ptrs, sh.c_sizes)
            if r != 0:
                raise PSError("ps unavailable" if r < 0 else "variables not initialised on the ps")
        self.store.master.copy_(self.host_vals, non_blocking=True)
        self.store.refresh_shadow()
        return int(self.step_val[0])

    def push(self, lr: float) -> int:
        """Send the store's gradients; the ps applies SGD and bumps global_step. Returns new step."""
        self.host_grads.copy_(self.store.grad)  # synchronous D2H
        new_step = C.c_double(-1.0)
        step = -1
        for t, sh in enumerate(self.push_shards):
            inc = int(t == self.step_task)
            r = runtime.lib().tfx_ps_push(sh.h, sh.n, sh.c_names, sh.c_ptrs, sh.c_sizes, C.c_float(lr), inc,
                                          C.byref(new_step))
            if r != 0:
                raise PSError("ps unavailable during push" if r < 0 else f"push rejected ({r})")
            if inc:
                step = int(new_step.value)
        return step

    def shutdown_servers(self) -> None:
        for h in self.handles:
            runtime.lib().tfx_ps_shutdown(h)

    def close(self) -> None:
        for h in self.handles:
            runtime.lib().tfx_ps_close(h)
        self.handles = []


def wait_for_initialization(client: PSClient, recovery_wait_secs: float = 30.0, max_wait_secs: float = 7200.0,
                            log=None) -> None:
    """Non-chief readiness loop (TF1 SessionManager.wait_for_session): poll every
    ``recovery_wait_secs`` until the chief has initialised every variable."""
    t0 = time.time()
    while True:
        n = client.num_uninitialized()
        if n == 0:
            return
        if time.time() - t0 > max_wait_secs:
            raise PSError(f"timed out after {max_wait_secs}s waiting for the chief to initialise variables")
        if log:
            log(f"Waiting for model to be ready. Ready_for_local_init_op: None, ready: {n} variables uninitialized")
        time.sleep(recovery_wait_secs)
