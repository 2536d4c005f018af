"""Tracing utilities: roctx ranges and the step timer."""
import pytest
import torch

from tensorflow_examples_amd.utils import fault, trace


def test_ranges_are_noops_when_disabled():
    was = trace.enabled()
    trace.enable(False)
    with trace.range("forward"):
        x = 1
    trace.mark("m")
    assert x == 1 and not trace.enabled()
    trace.enable(was)


def test_roctx_ranges_nest_when_library_present():
    if not trace._R.load():
        pytest.skip("no roctx library in this image")
    assert trace.enable(True)
    try:
        with trace.range("step"):
            with trace.range("forward"):
                trace.mark("inside")
    finally:
        trace.enable(False)


def test_step_timer_cpu():
    t = trace.StepTimer(device="cpu")
    for _ in range(3):
        t.start()
        torch.ones(100).sum()
        t.stop()
    s = t.summary()
    assert s["steps"] == 3 and s["min_ms"] >= 0 and s["max_ms"] >= s["p50_ms"] >= s["min_ms"]


def test_fault_spec_parsing():
    assert fault._parse("") == (None, -1)
    assert fault._parse("after_step:7") == ("after_step", 7)
    assert fault._parse("before_init") == ("before_init", 0)
    with pytest.raises(ValueError):
        fault._parse("explode")


@pytest.mark.gpu
def test_step_timer_gpu(gpu):
    t = trace.StepTimer(device=gpu)
    a = torch.randn(1024, 1024, device=gpu)
    for _ in range(3):
        t.start()
        a = a @ a
        t.stop()
    s = t.summary()
    assert s["steps"] == 3 and s["mean_ms"] > 0
