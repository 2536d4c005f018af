"""Supervisor: chief / non-chief session bring-up of the async-PS worker
(reference: ``tf.train.Supervisor(is_chief=(task_index == 0), global_step, init_op)`` and
``sv.prepare_or_wait_for_session(server.target)``, R/distributed/distributed.py:129-135).

TF1 semantics kept:
* chief without ``logdir``: runs init every time it starts -> a restarted chief RE-INITIALISES
  the ps variables (wipes training state), exactly like TF1;
* chief with ``logdir`` and a checkpoint there: restores it into the ps instead (TF1 behaviour
  when logdir is set), and ``save()`` writes checkpoints (MetaGraphDef ``.meta`` with the model's
  graph); at bring-up the chief writes ``<logdir>/graph.pbtxt`` like TF1's Supervisor;
* non-chief: polls the ps every ``recovery_wait_secs`` (default 30 s) until every variable is
  initialised (``report_uninitialized_variables``), up to ``max_wait_secs`` (7200 s);
* ps death surfaces as :class:`~.ps.PSError` at the next pull/push (uncaught -> worker exits
  non-zero, like the reference's unguarded sess.run).
"""
from __future__ import annotations

import os
from typing import Callable, Dict, List, Optional, Union

from .. import ckpt
from .ps import GLOBAL_STEP, PSClient, wait_for_initialization


class Supervisor:
    def __init__(self, is_chief: bool, client: PSClient, logdir: Optional[str] = None,
                 recovery_wait_secs: float = 30.0, max_wait_secs: float = 7200.0, log=print,
                 save_model_secs: float = 600.0,
                 graph_nodes: Optional[Union[List[Dict], Callable[[], List[Dict]]]] = None):
        self.is_chief, self.client, self.logdir = is_chief, client, logdir
        self.recovery_wait_secs, self.max_wait_secs = recovery_wait_secs, max_wait_secs
        self.log = log
        self.saver = ckpt.Saver() if logdir else None
        self.restored_from: Optional[str] = None
        self.save_model_secs = save_model_secs
        self._graph_nodes = graph_nodes
        self.graph_path: Optional[str] = None

    def graph_nodes(self) -> Optional[List[Dict]]:
        g = self._graph_nodes
        return g() if callable(g) else g

    def prepare_or_wait_for_session(self):
        if self.is_chief:
            path = ckpt.latest_checkpoint(self.logdir) if self.logdir else None
            if path:
                tensors = self.saver.restore(self.client.store, path)
                step = float(tensors[GLOBAL_STEP]) if GLOBAL_STEP in tensors else 0.0
                self.client.initialize(force=True, global_step=step)
                self.restored_from = path
            else:
                self.client.initialize(force=True, global_step=0.0)
            if self.logdir:
                nodes = self.graph_nodes() or ckpt.store_graph_nodes(self.client.store)
                self.graph_path = ckpt.write_graph(self.logdir, nodes)
        else:
            wait_for_initialization(self.client, self.recovery_wait_secs, self.max_wait_secs)
        return self

    def save(self, global_step: int) -> Optional[str]:
        if not (self.is_chief and self.saver):
            return None
        self.client.pull()
        return self.saver.save(self.client.store, os.path.join(self.logdir, "model.ckpt"), global_step=global_step,
                               graph_nodes=self.graph_nodes())

    def stop(self):
        self.client.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False
