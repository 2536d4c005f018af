"""The reference's observability and checkpoint conventions for every example script.

The reference worker writes ``cost`` / ``accuracy`` scalars and the graph to a TensorBoard event
file (``tf.summary.FileWriter(logs_path, graph=...)`` + ``writer.add_summary(summary, step)``,
R/distributed/distributed.py:120-125,138,151), and TF1's ``Supervisor`` with a ``logdir``
(:129-131) restores the latest checkpoint on start, saves periodically and writes
``graph.pbtxt``.  :class:`RunLog` gives the north-star examples the same conventions:

* ``--logs_path``: an event file (graph + MetaGraphDef at start, scalars at the log cadence --
  the examples log every N steps instead of every step so a HIP-graph-replayed step is not
  synchronised with the host each iteration);
* ``--logdir``: restore on start (model, optimizer slots, global step and any extra run state such
  as an RNG counter), ``graph.pbtxt``, a checkpoint every ``--save_checkpoint_steps`` steps and at
  the end (``model.ckpt-<step>`` + ``checkpoint`` state file, TF names).

Only rank 0 writes; every rank restores (all ranks hold the same weights)."""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import torch

from .. import summary
from ..ckpt import Saver, latest_checkpoint, read_checkpoint, store_graph_nodes, write_graph

_OPT_SLOTS = ("m", "v", "step_t")


class RunLog:
    def __init__(self, store, optimizer=None, logs_path: str = "", logdir: str = "", save_checkpoint_steps: int = 0,
                 rank: int = 0, graph_nodes: Optional[List[Dict]] = None, extra_state: Optional[Dict] = None):
        self.store, self.opt, self.rank = store, optimizer, rank
        self.logdir, self.save_steps = logdir, int(save_checkpoint_steps)
        self.extra = dict(extra_state or {})  # name -> tensor saved with the checkpoint, restored in place
        self.nodes = graph_nodes if graph_nodes is not None else store_graph_nodes(store)
        self.writer = summary.FileWriter(logs_path, graph=self.nodes) if (logs_path and rank == 0) else None
        self.saver = Saver()
        self.last_saved = -1
        if logdir and rank == 0:
            write_graph(logdir, self.nodes)  # graph.pbtxt, as TF1's Supervisor writes it

    # ------------------------------------------------------------------ checkpoints
    def restore(self) -> int:
        """Restore the latest checkpoint of ``logdir`` (model, optimizer slots, extra state); returns its
        global step (0 when there is none)."""
        if not self.logdir:
            return 0
        prefix = latest_checkpoint(self.logdir)
        if not prefix:
            return 0
        tensors = self.saver.restore(self.store, prefix)
        if self.opt is not None:
            for slot in _OPT_SLOTS:
                t, v = getattr(self.opt, slot, None), tensors.get("optimizer/" + slot)
                if t is not None and v is not None:
                    t.copy_(v.to(t.device, t.dtype).view(t.shape))
        for k, t in self.extra.items():
            v = tensors.get(k)
            if v is not None:
                t.copy_(v.to(t.device, t.dtype).view(t.shape))
        step = int(float(tensors["global_step"])) if "global_step" in tensors else 0
        self.last_saved = step
        return step

    def save(self, step: int) -> Optional[str]:
        if not self.logdir or self.rank != 0 or step == self.last_saved:
            return None
        extra = {k: t.detach().cpu() for k, t in self.extra.items()}
        if self.opt is not None:
            for slot in _OPT_SLOTS:
                t = getattr(self.opt, slot, None)
                if t is not None:
                    extra["optimizer/" + slot] = t.detach().cpu()
        self.last_saved = step
        return self.saver.save(self.store, os.path.join(self.logdir, "model.ckpt"), global_step=step, extra=extra,
                               graph_nodes=self.nodes)

    def maybe_save(self, step: int) -> Optional[str]:
        if self.save_steps > 0 and step % self.save_steps == 0:
            return self.save(step)
        return None

    # ------------------------------------------------------------------ scalars
    def scalars(self, step: int, **values: float) -> None:
        if self.writer is not None:
            self.writer.add_scalars(int(step), **{k: float(v) for k, v in values.items()})

    def close(self, step: Optional[int] = None) -> Optional[str]:
        path = self.save(step) if step is not None else None
        if self.writer is not None:
            self.writer.flush()
            self.writer.close()
            self.writer = None
        return path


def define_flags(flags, save_steps_default: int = 500) -> None:
    """The three flags every example takes (reference: ``logs_path`` R/distributed/distributed.py:49;
    the Supervisor ``logdir`` SURVEY §5.4)."""
    flags.DEFINE_string("logs_path", "", "TensorBoard event-file directory (cost / accuracy scalars + the graph)")
    flags.DEFINE_string("logdir", "", "checkpoint directory: restore the latest checkpoint on start, save every "
                        "--save_checkpoint_steps steps and at the end")
    flags.DEFINE_integer("save_checkpoint_steps", save_steps_default, "checkpoint period in steps (0 = only at the end)")


def read_scalars(logs_path: str) -> Dict[str, List]:
    """{tag: [(step, value), ...]} over every event file in ``logs_path`` (tests / tools)."""
    out: Dict[str, List] = {}
    for f in sorted(os.listdir(logs_path)):
        if not f.startswith("events.out.tfevents."):
            continue
        for ev in summary.summary_iterator(os.path.join(logs_path, f)):
            for tag, val in ev.get("summary", []):
                out.setdefault(tag, []).append((ev["step"], val))
    return out


__all__ = ["RunLog", "define_flags", "read_scalars", "read_checkpoint"]
