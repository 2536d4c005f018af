"""Race detection / memory checking of the native host runtime (tier T-sanitize).

csrc/tests/rt_stress.cpp drives the parameter-server service (concurrent Hogwild clients, shutdown
with open connections) and the tfevents writer (producer vs background flush thread) and is built
straight from csrc/runtime/*.cpp with ThreadSanitizer and with AddressSanitizer +
UndefinedBehaviorSanitizer (host code only; GPU sanitizers are not used on this pool)."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CXX = shutil.which("g++") or shutil.which("c++")


def _build(tmp_path, flags, name):
    srcs = sorted(glob.glob(os.path.join(ROOT, "csrc", "runtime", "*.cpp"))) + \
        [os.path.join(ROOT, "csrc", "tests", "rt_stress.cpp")]
    exe = str(tmp_path / name)
    cmd = [CXX, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread",
           f"-I{os.path.join(ROOT, 'csrc', 'include')}", *flags, *srcs, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if r.returncode != 0 and ("sanitizer" in r.stderr.lower() or "cannot find" in r.stderr):
        pytest.skip("sanitizer runtime unavailable: " + r.stderr[-300:])
    assert r.returncode == 0, r.stderr
    return exe


@pytest.mark.skipif(CXX is None, reason="no host C++ compiler")
@pytest.mark.parametrize("kind,flags,env", [
    ("tsan", ["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1 second_deadlock_stack=1"}),
    ("asan", ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
     {"ASAN_OPTIONS": "detect_leaks=1 abort_on_error=1", "UBSAN_OPTIONS": "print_stacktrace=1"}),
])
def test_runtime_under_sanitizer(tmp_path, kind, flags, env):
    exe = _build(tmp_path, flags, "rt_stress_" + kind)
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, **env))
    assert r.returncode == 0 and "RT_STRESS_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-6000:])
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr, r.stderr[-6000:]
