"""Parameter-server transport over xGMI peer memory (``distributed.py --transport=xgmi``).

The reference moves every variable between worker and ps over gRPC each step -- RecvTensor for
the pulls, RunGraph for the ps-side ApplyGradientDescent + AssignAdd(global_step)
(R/distributed/distributed.py:63-65,107-108,148-150).  On one
MI355X node the ps task instead owns one device arena on its GPU and exports it with
hipIpcGetMemHandle; every worker maps it (hipIpcOpenMemHandle) and

* PULL  = one copy kernel per contiguous run of that task's variables, arena -> worker store
          (xGMI reads, no host hop);
* PUSH  = ``ps_peer_sgd``: the worker's own kernel applies ``p -= lr * g`` straight into the peer
          arena (lock-free like TF's use_locking=False) and clears its local gradient; the task
          that owns ``global_step`` then gets a one-thread SYSTEM-scope atomic increment, ordered
          behind the whole update, whose new value comes back to the worker.

Control stays on the TCP service (csrc/runtime/ps_service.cpp): the ps publishes the arena's
64-byte IPC handle and size there as two tiny variables, readiness / the done counter / shutdown
are unchanged.

Arena layout (per ps task): 256-byte header of int64 words -- [0] global step, [1] ready flag
(the chief sets it after writing the initial values), [2] layout fingerprint -- then the store's
flat f32 layout (every worker replica builds the identical layout; only the variables placed on
this task are authoritative there).
"""
from __future__ import annotations

import ctypes as C
import time
import zlib
from typing import Dict, List, Tuple

import numpy as np
import torch

from .. import runtime
from ..variables import VariableStore
from . import ClusterSpec, parse_address, replica_device_setter
from .ps import GLOBAL_STEP, PSError

HANDLE_VAR = "__xgmi_handle__"   # 64-byte hipIpcMemHandle_t as 16 float32 words
INFO_VAR = "__xgmi_info__"       # [arena bytes, device index] as float32 (exact below 2^24 MiB units)
HEADER = 256


def _ops():
    from ..ops import _native
    return _native.ops()


class XgmiArena:
    """ps side: allocate the arena on this process's GPU and publish its handle on the task's own
    TCP service (``server``: a started :class:`~tensorflow_examples_amd.cluster.Server`)."""

    def __init__(self, server, nbytes: int, device: int = 0):
        nbytes = (int(nbytes) + 255) // 256 * 256
        self.device = device
        self.arena = _ops().ipc_arena_alloc(nbytes, device)  # zero-filled: ready flag 0
        handle = _ops().ipc_handle(self.arena).numpy()
        words = np.frombuffer(handle.tobytes(), dtype=np.float32).copy()
        info = np.array([nbytes / (1 << 20), float(device)], dtype=np.float32)
        h = runtime.lib().tfx_ps_connect(b"127.0.0.1", server.port, 10000)
        if not h:
            raise PSError("xgmi: cannot reach the local ps service to publish the arena")
        names = (C.c_char_p * 2)(HANDLE_VAR.encode(), INFO_VAR.encode())
        ptrs = (C.c_void_p * 2)(words.ctypes.data, info.ctypes.data)
        sizes = (C.c_uint64 * 2)(words.nbytes, info.nbytes)
        if runtime.lib().tfx_ps_create(h, 2, names, ptrs, sizes, 1) < 0:
            raise PSError("xgmi: publishing the arena handle failed")
        runtime.lib().tfx_ps_close(h)
        self.nbytes = nbytes


def _fingerprint(store: VariableStore) -> int:
    sig = ";".join(f"{v.name}:{v.offset}:{v.numel}" for v in store.vars).encode()
    return zlib.crc32(sig) & 0x7FFFFFFF


def _runs(store: VariableStore, names) -> List[Tuple[int, int]]:
    """Contiguous [lo, hi) element runs of the store covering the given variables (gaps of alignment
    padding between adjacent variables are included)."""
    vs = sorted((v for v in store.vars if v.name in names), key=lambda v: v.offset)
    runs: List[List[int]] = []
    for v in vs:
        lo, hi = v.offset, v.offset + v.numel
        if runs and lo - runs[-1][1] < 64:  # ALIGN padding only: merge
            runs[-1][1] = hi
        else:
            runs.append([lo, hi])
    return [(a, b) for a, b in runs]


class XgmiPSClient:
    """Worker side, the same interface as :class:`~.ps.PSClient` (initialize / num_uninitialized /
    pull / push / shard_map / handles / close), with the data path on xGMI peer memory."""

    push_zeroes_grad = True

    def __init__(self, cluster: ClusterSpec, store: VariableStore, connect_timeout_s: float = 60.0,
                 ps_job: str = "ps"):
        if store.device.type != "cuda":
            raise PSError("--transport=xgmi needs GPU workers")
        self.cluster = ClusterSpec(cluster)
        self.store = store
        self.num_ps = self.cluster.num_tasks(ps_job)
        names = [GLOBAL_STEP] + [v.name for v in store.vars]
        self.placement: Dict[str, int] = replica_device_setter(self.cluster, ps_job)(names)
        self.step_task = self.placement[GLOBAL_STEP]
        self.fp = _fingerprint(store)
        need = HEADER + store.total * 4
        dev = store.device.index or 0
        self.handles, self.arenas, self.params, self.headers, self.runs = [], [], [], [], []
        hbuf = np.zeros(16, np.float32)
        ibuf = np.zeros(2, np.float32)
        for t in range(self.num_ps):
            host, port = parse_address(self.cluster.task_address(ps_job, t))
            h = runtime.lib().tfx_ps_connect(host.encode(), port, int(connect_timeout_s * 1000))
            if not h:
                raise PSError(f"cannot reach ps task {t} at {host}:{port} within {connect_timeout_s}s")
            self.handles.append(h)
            # the ps publishes its arena right after it starts; wait for it like a readiness poll
            nm = (C.c_char_p * 2)(HANDLE_VAR.encode(), INFO_VAR.encode())
            ptrs = (C.c_void_p * 2)(hbuf.ctypes.data, ibuf.ctypes.data)
            sizes = (C.c_uint64 * 2)(hbuf.nbytes, ibuf.nbytes)
            t0 = time.time()
            while True:
                r = runtime.lib().tfx_ps_pull(h, 2, nm, ptrs, sizes)
                if r == 0:
                    break
                if r < 0 or time.time() - t0 > connect_timeout_s:
                    raise PSError(f"ps task {t} did not publish an xGMI arena (start it with --transport=xgmi)")
                time.sleep(0.05)
            nbytes = int(round(float(ibuf[0]) * (1 << 20)))
            if nbytes < need:
                raise PSError(f"ps task {t} arena is {nbytes} B, the model needs {need} B (raise --xgmi_arena_mb)")
            handle = torch.from_numpy(np.frombuffer(hbuf.tobytes(), dtype=np.uint8).copy())
            arena = _ops().ipc_open(handle, nbytes, dev)
            self.arenas.append(arena)
            self.headers.append(arena[:HEADER].view(torch.int64))
            self.params.append(arena[HEADER:HEADER + store.total * 4].view(torch.float32))
            self.runs.append(_runs(store, {n for n, tt in self.placement.items() if tt == t and n != GLOBAL_STEP}))
        self.step_out = torch.zeros(1, dtype=torch.int64, device=store.device)
        self._step_host = torch.zeros(1, dtype=torch.int64, pin_memory=True)

    def shard_map(self) -> Dict[str, str]:
        return {n: f"/job:ps/task:{t}" for n, t in self.placement.items()}

    # ---------------------------------------------------------------- init / readiness
    def initialize(self, force: bool = True, global_step: float = 0.0) -> int:
        done = 0
        hdr = torch.tensor([int(global_step), 1, self.fp, 0], dtype=torch.int64)
        for t in range(self.num_ps):
            cur = self.headers[t][:3].cpu()
            if int(cur[1]) == 1 and not force:
                if int(cur[2]) != self.fp:
                    raise PSError("a different model layout is already initialised on the ps")
                continue
            for lo, hi in self.runs[t]:
                _ops().ps_peer_copy(self.params[t][lo:hi], self.store.master[lo:hi])
            torch.cuda.synchronize(self.store.device)
            h = hdr.clone()
            if t != self.step_task:
                h[0] = 0
            self.headers[t][:4].copy_(h.to(self.store.device))
            torch.cuda.synchronize(self.store.device)
            done += len(self.runs[t])
        return done

    def num_uninitialized(self) -> int:
        n = 0
        for t in range(self.num_ps):
            cur = self.headers[t][:3].cpu()
            if int(cur[1]) != 1:
                n += len(self.runs[t]) + (1 if t == self.step_task else 0)
            elif int(cur[2]) != self.fp:
                raise PSError("the ps holds a different model layout")
        return n

    # ---------------------------------------------------------------- per-step traffic
    def pull(self) -> int:
        for t in range(self.num_ps):
            for lo, hi in self.runs[t]:
                _ops().ps_peer_copy(self.store.master[lo:hi], self.params[t][lo:hi])
        self.store.refresh_shadow()
        return -1  # the step value arrives with the next push

    def push_async(self, lr: float, zero_grad: bool = True) -> torch.Tensor:
        """Apply SGD into the peer arenas and bump global_step behind the WHOLE update: every ps
        task's runs are issued first and the step task's counter is bumped by the last launch of all
        (stream order puts it after every earlier SGD kernel's peer writes) -- TF orders
        AssignAdd(global_step) after all ApplyGradientDescent ops (R/distributed/distributed.py:108).
        No host sync: returns the device tensor the new step value lands in (``step_out``)."""
        launches = [(t, lo, hi) for t in range(self.num_ps) for lo, hi in self.runs[t]]
        step_hdr = self.headers[self.step_task][:1]
        if not launches:
            _ops().ps_peer_sgd(self.params[self.step_task][:0], self.store.grad[:0], float(lr), step_hdr,
                               self.step_out, zero_grad)
        for n, (t, lo, hi) in enumerate(launches):
            last = n == len(launches) - 1
            _ops().ps_peer_sgd(self.params[t][lo:hi], self.store.grad[lo:hi], float(lr), step_hdr if last else None,
                               self.step_out, zero_grad)
        return self.step_out

    def push(self, lr: float, zero_grad: bool = True) -> int:
        """:meth:`push_async` + wait: returns the new global step."""
        self.push_async(lr, zero_grad)
        self._step_host.copy_(self.step_out, non_blocking=True)
        torch.cuda.current_stream(self.store.device).synchronize()
        return int(self._step_host[0])

    def shutdown_servers(self) -> None:
        for h in self.handles:
            runtime.lib().tfx_ps_shutdown(h)

    def close(self) -> None:
        torch.cuda.synchronize(self.store.device)
        self.params, self.headers, self.arenas = [], [], []
        for h in self.handles:
            runtime.lib().tfx_ps_close(h)
        self.handles = []
