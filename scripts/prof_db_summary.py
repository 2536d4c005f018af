#!/usr/bin/env python3
"""Per-kernel summary (calls, total us, avg us, %) of a rocprofv3 SQLite output (``*_results.db``; durations there are already in microseconds),
for runs that did not pass ``--output-format csv``.  Usage: prof_db_summary.py DB [TOP] [STEPS]"""
import sqlite3
import sys

db = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 0
c = sqlite3.connect(db)
rows = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
tot = sum(r[2] for r in rows)
print(f"{'calls':>7} {'total_us':>10} {'avg_us':>8} {'pct':>6}" + (f" {'us/step':>8}" if steps else "") + "  kernel")
for name, calls, dur, avg, pct in rows[:top]:
    short = name if len(name) < 110 else name[:107] + "..."
    extra = f" {dur / steps:8.1f}" if steps else ""
    print(f"{calls:7d} {dur:10.1f} {avg:8.2f} {pct:6.2f}{extra}  {short}")
print(f"total kernel time {tot:.1f} us over {sum(r[1] for r in rows)} dispatches"
      + (f" = {tot / steps:.1f} us/step" if steps else ""))
