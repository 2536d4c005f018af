"""The PMC summarisers (scripts/pmc_summary.py, scripts/pmc_loadpath.py) on a synthetic rocprofv3
counter_collection.csv: per-kernel sums over dispatches, the derived percentages and the
rate x latency columns the profiles/r04_* READMEs quote."""
import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPTS = os.path.join(ROOT, "scripts")


def _write(path, rows):
    cols = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"]
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=cols)
        w.writeheader()
        for r in rows:
            w.writerow(dict(zip(cols, r)))


def test_loadpath_summary(tmp_path):
    d = tmp_path / "pmc" / "p1"
    d.mkdir(parents=True)
    # two dispatches of one kernel, 10 us each; GUI = 8 XCDs x 24,000 cycles per dispatch
    rows = []
    for disp, t0 in ((1, 0), (2, 50_000)):
        base = (disp, "void tfx::(anonymous namespace)::igemm_kernel<10, 10>(tfx::IgemmArgs)")
        for name, val in (("GRBM_GUI_ACTIVE", 8 * 24_000), ("TA_TA_BUSY", 0.5 * 24_000 * 256),
                          ("TD_TD_BUSY", 0.25 * 24_000 * 256), ("TCP_TCC_READ_REQ", 1_000_000),
                          ("TCP_TCC_READ_REQ_LATENCY", 500 * 1_000_000)):
            rows.append(base + (name, val, t0, t0 + 10_000))
    _write(d / "p_counter_collection.csv", rows)
    out = subprocess.run([sys.executable, os.path.join(SCRIPTS, "pmc_loadpath.py"), str(tmp_path / "pmc")],
                         capture_output=True, text=True, check=True).stdout
    line = [ln for ln in out.splitlines() if "igemm_kernel" in ln]
    assert len(line) == 1, out
    f = line[0].split()
    us, calls, ta, tas, td = float(f[0]), int(f[1]), float(f[2]), f[3], float(f[4])
    lat, mb = float(f[6]), float(f[7])
    assert abs(us - 20.0) < 1e-6 and calls == 2
    assert abs(ta - 50.0) < 0.1 and abs(td - 25.0) < 0.1 and tas == "nan"
    assert abs(lat - 500) < 1 and mb == 256  # 2e6 requests x 128 B


def test_pmc_summary_load_sums_dispatches(tmp_path):
    sys.path.insert(0, SCRIPTS)
    try:
        import pmc_summary
    finally:
        sys.path.remove(SCRIPTS)
    d = tmp_path / "p2"
    d.mkdir()
    _write(d / "x_counter_collection.csv", [
        (1, "void tfx::bn_apply_vec_kernel<false, true, false>(tfx::Args)", "FETCH_SIZE", 100, 0, 2000),
        (2, "void tfx::bn_apply_vec_kernel<false, true, false>(tfx::Args)", "FETCH_SIZE", 50, 5000, 9000),
    ])
    per, dur, calls = pmc_summary.load(str(tmp_path))
    (k,) = per.keys()
    assert k == "tfx::bn_apply_vec_kernel<false, true, false>"
    assert per[k]["FETCH_SIZE"] == 150 and calls[k] == 2 and abs(dur[k] - 6.0) < 1e-9
