"""The fusion-plan module (ops/fusion.py) and the gradient-zeroed store scratch, on the CPU: profile
parsing, switching groups on and off (and restoring them), the opt-in group staying out of the default
profile, the plan recorder's table, and VariableStore.reserve_scratch / zero_grad / grad_epoch."""
import pytest
import torch

from tensorflow_examples_amd.ops import fusion
from tensorflow_examples_amd.ops import nn as tnn
from tensorflow_examples_amd.variables import VariableStore, Zeros


def test_profiles_parse():
    assert fusion.parse_profile("all") == fusion.PROFILES["all"]
    assert fusion.parse_profile("") == fusion.PROFILES["all"]
    assert fusion.parse_profile("none") == set()
    assert "bn_finalize_fold" not in fusion.PROFILES["all"]  # opt-in (profiles/r04_fold)
    assert fusion.parse_profile("+bn_finalize_fold") == fusion.PROFILES["all"] | {"bn_finalize_fold"}
    assert fusion.parse_profile("-head_tail,-bn_on_load") == fusion.PROFILES["all"] - {"head_tail", "bn_on_load"}
    assert fusion.PROFILES["r2"] <= fusion.PROFILES["all"]
    with pytest.raises(ValueError):
        fusion.parse_profile("-no_such_group")


def test_set_groups_and_restore():
    prev = fusion.enabled()
    try:
        fusion.set_groups(fusion.PROFILES["r2"])
        on = fusion.enabled()
        assert {g for g, v in on.items() if v} == fusion.PROFILES["r2"]
        assert tnn._DEFER_TAIL is False and tnn._FUSE_HEAD is True and tnn._FOLD_FIN is False
        fusion.set_groups(set(fusion.GROUPS))
        assert all(fusion.enabled().values()) and tnn._FOLD_FIN is True
    finally:
        fusion.restore(prev)
    assert fusion.enabled() == prev


def test_recorder_table():
    with fusion.record() as r:
        fusion.note("bn_epilogue", "stage1/conv1", "igemm_fwd_stats")
        fusion.note("bn_epilogue", "stage1/conv2", "igemm_fwd_stats")
        fusion.note("fused_head", "fc", "head_xent")
        fusion.note("layerwise", "stage3/conv2", "bn_apply_into")
    fusion.note("fused_head", "ignored", "outside the recorder")
    assert len(r.events) == 4
    assert r.counts()[("bn_epilogue", "igemm_fwd_stats")] == 2
    t = r.table()
    assert "fusion plan (4 decisions)" in t and "igemm_fwd_stats x2" in t and "layerwise" in t
    plan = r.plan()
    assert plan["fused_head"] == [("fc", "head_xent")]


def test_store_scratch_zeroed_with_grads():
    st = VariableStore(device="cpu", seed=0)
    st.variable([10], Zeros(), name="w")
    off = st.reserve_scratch(100)
    off2 = st.reserve_scratch(7)
    assert off == 0 and off2 >= 100
    st.finalize()
    assert st.scratch is not None and st.scratch.numel() >= off2 + 7
    assert st.grad.numel() == st.total and st.grad.data_ptr() == st._grad_ext.data_ptr()
    st.scratch.fill_(3.0)
    st.grad.fill_(2.0)
    e0 = st.grad_epoch
    st.zero_grad()
    assert st.grad_epoch == e0 + 1
    assert float(st.scratch.abs().max()) == 0.0 and float(st.grad.abs().max()) == 0.0
    with pytest.raises(RuntimeError):
        st.reserve_scratch(4)  # after finalize


def test_bn_workspace_rows_once_per_step():
    st = VariableStore(device="cpu", seed=0)
    ws = tnn.BNWorkspace(8, st)
    st.variable([4], Zeros(), name="w")
    st.finalize()
    st.zero_grad()
    r1 = ws.fin_rows()
    assert r1 is not None and r1.numel() == tnn.BNWorkspace.FIN_ROWS * 2 * 8
    assert ws.fin_rows() is None  # used already this step: the caller falls back to the finalize launch
    st.zero_grad()
    assert ws.fin_rows() is not None
    assert tnn.BNWorkspace(8).fin_rows() is None  # no store: no scratch
