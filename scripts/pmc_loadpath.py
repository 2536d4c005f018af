#!/usr/bin/env python3
"""Load-path counters per kernel from one rocprofv3 ``--pmc`` pass: is an implicit GEMM bound by the
texture-address unit (TA busy), the data return path (TD busy), or by L2 latency with too few bytes in
flight (long TCP->TCC read latency, TA/TD mostly idle)?

usage: python scripts/pmc_loadpath.py <dir with *counter_collection.csv> [--steps N]

Per kernel (counters summed over its dispatches; ``*_sum`` counters are already summed over the 256
CUs, GRBM_GUI_ACTIVE over the 8 XCDs):

* TA busy %  = TA_TA_BUSY / (GRBM_GUI_ACTIVE / 8 * 256)
* TA stalled-by-TCP % = TA_ADDR_STALLED_BY_TC_CYCLES / (same)
* TD busy %  = TD_TD_BUSY / (same)
* TCP pending-stall % = TCP_PENDING_STALL_CYCLES / (same)
* L2 read latency (cycles per request) = TCP_TCC_READ_REQ_LATENCY / TCP_TCC_READ_REQ
* L2 read MB = TCP_TCC_READ_REQ x 128 B (gfx950 line size; on the 1x1 weight gradient this matches the
  tile bytes its loaders request, 5.1 GB/step by the tiling arithmetic vs 5.9 GB counted)
"""
import argparse

from pmc_summary import load  # same CSV aggregation as the main PMC table


def pick(c, base):
    for k in (base + "_sum", base):
        if k in c:
            return c[k]
    return float("nan")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--steps", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    per, dur, calls = load(a.root)
    rows = []
    for k, c in per.items():
        cu_cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8 * 256
        pct = (lambda v: 100.0 * v / cu_cyc) if cu_cyc else (lambda v: float("nan"))
        req = pick(c, "TCP_TCC_READ_REQ")
        lat = pick(c, "TCP_TCC_READ_REQ_LATENCY") / req if req == req and req else float("nan")
        rows.append((dur.get(k, 0.0), k, calls.get(k, 0), pct(pick(c, "TA_TA_BUSY")),
                     pct(pick(c, "TA_ADDR_STALLED_BY_TC_CYCLES")), pct(pick(c, "TD_TD_BUSY")),
                     pct(pick(c, "TCP_PENDING_STALL_CYCLES")), lat, req * 128 / 1e6 / a.steps))
    rows.sort(reverse=True)
    print("%9s %6s %7s %8s %7s %8s %9s %9s  %s" % ("us/step", "calls", "TA%", "TAstl%", "TD%", "TCPstl%",
                                                  "L2lat", "L2rdMB", "kernel"))
    for us, k, n, ta, tas, td, tcs, lat, mb in rows[:a.top]:
        print("%9.1f %6d %7.1f %8.1f %7.1f %8.1f %9.0f %9.0f  %s" % (us / a.steps, n, ta, tas, td, tcs, lat, mb, k))


if __name__ == "__main__":
    main()
