import pytest

from tensorflow_examples_amd.utils.flags import FlagValues, FlagsError, DEFINE_boolean, DEFINE_float, \
    DEFINE_integer, DEFINE_list, DEFINE_string


def mk():
    fv = FlagValues()
    DEFINE_string("job_name", "", "Either 'ps' or 'worker'", fv)
    DEFINE_integer("task_index", 0, "Index of task within the job", fv)
    DEFINE_string("worker_hosts", None, "workers", fv)
    DEFINE_string("ps_hosts", None, "ps", fv)
    DEFINE_float("lr", 0.001, "lr", fv)
    DEFINE_boolean("stable", False, "b", fv)
    DEFINE_list("ids", [], "l", fv)
    return fv


def test_reference_cli_forms():
    fv = mk()
    fv(["prog", "--ps_hosts=127.0.0.1:2222", "--worker_hosts", "127.0.0.1:2223,127.0.0.1:2224",
        "--job_name=worker", "--task_index=1", "--stable", "--ids=a,b"])
    assert fv.ps_hosts == "127.0.0.1:2222"
    assert fv.worker_hosts.split(",") == ["127.0.0.1:2223", "127.0.0.1:2224"]
    assert fv.job_name == "worker" and fv.task_index == 1 and fv.stable is True and fv.ids == ["a", "b"]


def test_defaults_and_lazy_parse(monkeypatch):
    fv = mk()
    monkeypatch.setattr("sys.argv", ["prog", "--task_index=3", "--unknown_flag=1"])
    # first attribute access parses sys.argv with known_only (TF1 lazy parse)
    assert fv.task_index == 3
    assert fv.ps_hosts is None and fv.lr == 0.001
    assert "--unknown_flag=1" in fv.unparsed_args


def test_errors():
    fv = mk()
    with pytest.raises(FlagsError):
        fv(["prog", "--task_index=abc"])
    with pytest.raises(FlagsError):
        mk()(["prog", "--nope=1"])
    fv = mk()
    fv(["prog", "--nostable"])
    assert fv.stable is False
