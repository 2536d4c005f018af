"""Cluster runtime of the async parameter-server path (reference: R/distributed/distributed.py:37-43
ClusterSpec + Server, :57-59 role dispatch, :63-65 replica_device_setter, :129-135 Supervisor).

* :class:`ClusterSpec` -- ``{"ps": [...], "worker": [...]}``; a task's index is its list position.
* :class:`Server` -- ``job_name="ps"`` starts the native PS service (csrc/runtime/ps_service.cpp)
  on the task's port; ``join()`` blocks like ``server.join()`` (the ps never exits on its own,
  SURVEY Q10; a client ``shutdown()`` or ``--ps_exit_after_workers`` ends it).  Workers get a
  ``target`` string; they talk to the ps tasks through :class:`~.ps.PSClient`.
* :func:`replica_device_setter` -- round-robin placement of variables over ps tasks in creation
  order (global_step -> ps0, W1 -> ps1, ...), whole-variable granularity like TF1.
"""
from __future__ import annotations

import time
from typing import Dict, List, Sequence, Union

from .. import runtime


def parse_address(addr: str):
    host, _, port = addr.rpartition(":")
    if not host or not port.isdigit():
        raise ValueError(f"bad task address {addr!r} (want host:port)")
    return host, int(port)


class ClusterSpec:
    def __init__(self, cluster: Union[Dict[str, Union[Sequence[str], Dict[int, str]]], "ClusterSpec"]):
        if isinstance(cluster, ClusterSpec):
            cluster = cluster.as_dict()
        self._jobs: Dict[str, List[str]] = {}
        for job, tasks in cluster.items():
            if isinstance(tasks, dict):
                n = max(tasks) + 1 if tasks else 0
                self._jobs[job] = [tasks.get(i, "") for i in range(n)]
            else:
                self._jobs[job] = [str(t) for t in tasks]

    @property
    def jobs(self) -> List[str]:
        return list(self._jobs)

    def num_tasks(self, job: str) -> int:
        return len(self._jobs[job])

    def job_tasks(self, job: str) -> List[str]:
        return list(self._jobs[job])

    def task_address(self, job: str, index: int) -> str:
        try:
            return self._jobs[job][index]
        except (KeyError, IndexError):
            raise ValueError(f"no task {index} in job {job!r}") from None

    def as_dict(self) -> Dict[str, List[str]]:
        return {k: list(v) for k, v in self._jobs.items()}

    def __repr__(self):
        return f"ClusterSpec({self._jobs})"


class Server:
    def __init__(self, cluster: ClusterSpec, job_name: str, task_index: int = 0, start: bool = True,
                 use_locking: bool = False):
        cluster = ClusterSpec(cluster)
        if job_name not in cluster.jobs:
            raise ValueError(f"job_name {job_name!r} is not in the cluster spec {cluster.jobs} "
                             "(expected 'ps' or 'worker')")
        self.cluster, self.job_name, self.task_index = cluster, job_name, task_index
        host, port = parse_address(cluster.task_address(job_name, task_index))
        self.host, self.port = host, port
        self.target = f"tfx://{host}:{port}"
        self._h = None
        self.use_locking = use_locking
        if start and job_name == "ps":
            self.start()

    def start(self):
        bind = "0.0.0.0" if self.host not in ("127.0.0.1", "localhost") else "127.0.0.1"
        self._h = runtime.lib().tfx_ps_server_start(bind.encode(), self.port, int(self.use_locking))
        if not self._h:
            raise OSError(f"cannot start parameter server on {self.host}:{self.port} (port in use?)")
        self.port = runtime.lib().tfx_ps_server_port(self._h)
        self.target = f"tfx://{self.host}:{self.port}"

    def join(self, poll_secs: float = 0.2):
        """Block while the service runs (forever unless a client sends shutdown)."""
        if self._h is None:
            return
        while not runtime.lib().tfx_ps_server_stopped(self._h):
            time.sleep(poll_secs)
        self.stop()

    def read(self, name: str, n: int):
        import ctypes as C
        buf = (C.c_float * n)()
        got = runtime.lib().tfx_ps_server_read(self._h, name.encode(), buf, n)
        return None if got < 0 else list(buf)[:min(n, got)]

    @property
    def pushes(self) -> int:
        return int(runtime.lib().tfx_ps_server_pushes(self._h)) if self._h else 0

    def stop(self):
        if self._h is not None:
            runtime.lib().tfx_ps_server_stop(self._h)
            self._h = None


def replica_device_setter(cluster: ClusterSpec, ps_job: str = "ps"):
    """Returns ``assign(names) -> {name: ps_task}``: round-robin over ps tasks in creation order."""
    n = ClusterSpec(cluster).num_tasks(ps_job)

    def assign(names: Sequence[str]) -> Dict[str, int]:
        return {name: i % n for i, name in enumerate(names)}

    return assign


__all__ = ["ClusterSpec", "Server", "replica_device_setter", "parse_address"]
