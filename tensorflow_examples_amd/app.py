"""``tf.app``-shaped entry point: ``app.flags`` (lazy-parsed absl-compatible flags) and ``app.run``.

The reference uses ``tf.app.flags`` / ``flags.FLAGS`` interchangeably
(R/distributed/distributed.py:24-32); scripts of this framework do the same through
``from tensorflow_examples_amd import app; flags = app.flags``.
"""
from __future__ import annotations

import sys

from .utils import flags  # noqa: F401  (re-exported as app.flags)


def run(main=None, argv=None):
    """Parse flags (all of them: unknown flags are an error, as absl.app.run) and call main(argv)."""
    args = flags.FLAGS(sys.argv if argv is None else argv, known_only=False)
    main = main or sys.modules["__main__"].main
    sys.exit(main(args))
