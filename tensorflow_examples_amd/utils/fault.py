"""Fault injection for the failure / recovery tests (test tier T-fault).

The reference has no fault injection; its recovery behaviour is implicit in TF1's Supervisor
(R/distributed/distributed.py:129-135): a restarted non-chief waits for the initialised ps and
rejoins, a restarted chief re-runs init (or restores ``logdir``'s checkpoint), and a dead ps makes
the next ``sess.run`` raise.  These hooks let the tests kill a process at a precise point:

``TFX_FAULT=after_step:N``  the process dies right after its N-th local training step;
``TFX_FAULT=before_init``   it dies before session bring-up.

A fault is an abrupt ``os._exit(FAULT_EXIT_CODE)``: no ``finally`` blocks, no flush, no ps
notification -- what a killed worker looks like to the rest of the cluster.  With the variable
unset every hook is a no-op (one int compare per step).
"""
from __future__ import annotations

import os
import sys

FAULT_EXIT_CODE = 43


def _parse(spec: str):
    if not spec:
        return None, -1
    kind, _, arg = spec.partition(":")
    if kind == "after_step":
        return kind, int(arg)
    if kind == "before_init":
        return kind, 0
    raise ValueError("TFX_FAULT: unknown fault %r (after_step:N | before_init)" % spec)


_KIND, _N = _parse(os.environ.get("TFX_FAULT", ""))


def _die(what: str) -> None:
    sys.stderr.write("TFX_FAULT: injected fault %s\n" % what)
    sys.stderr.flush()
    os._exit(FAULT_EXIT_CODE)


def armed() -> bool:
    """True when a fault is configured (callers that enqueue work asynchronously -- a replayed HIP
    graph -- must complete it before :func:`after_step`, whose contract is steps *completed*)."""
    return _KIND is not None


def before_init() -> None:
    if _KIND == "before_init":
        _die("before_init")


def after_step(local_step: int) -> None:
    """Call with the 1-based count of training steps this process has completed."""
    if _KIND == "after_step" and local_step >= _N:
        _die("after_step:%d" % local_step)
