import glob
import os

from tensorflow_examples_amd import summary
from tensorflow_examples_amd.runtime import crc32c, masked_crc32c


def test_crc32c_vectors():
    # RFC 3720 B.4 test vectors, hardware (SSE4.2) and table paths
    for sw in (False, True):
        assert crc32c(b"123456789", sw) == 0xE3069283
        assert crc32c(bytes(32), sw) == 0x8A9136AA
        assert crc32c(b"\xff" * 32, sw) == 0x62A8AB43
        assert crc32c(bytes(range(32)), sw) == 0x46DD794E
        assert crc32c(bytes(range(31, -1, -1)), sw) == 0x113FDB5C
    c = crc32c(b"abc")
    assert masked_crc32c(b"abc") == (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def test_event_file_roundtrip(tmp_path):
    summary.reset_registry()
    vals = {"cost": 2.5, "accuracy": 0.25}
    summary.scalar("cost", lambda: vals["cost"])
    summary.scalar("accuracy", lambda: vals["accuracy"])
    op = summary.merge_all()
    w = summary.FileWriter(str(tmp_path), graph=[{"name": "x", "op": "Placeholder"}])
    for step in range(5):
        vals["cost"] = 2.5 - step
        w.add_summary(op(), step)
    w.close()
    files = glob.glob(os.path.join(str(tmp_path), "events.out.tfevents.*"))
    assert len(files) == 1
    evs = list(summary.summary_iterator(files[0]))
    assert evs[0]["file_version"] == "brain.Event:2"
    assert b"Placeholder" in evs[1]["graph_def"]
    # TF1 FileWriter(graph=...) also writes the MetaGraphDef (Event field 9) wrapping the same GraphDef
    meta = summary._parse(evs[2]["meta_graph_def"])
    assert meta[2][0] == evs[1]["graph_def"]
    assert summary._parse(meta[1][0])[1][0] == b"v1"
    scal = [e for e in evs if "summary" in e]
    assert [e["step"] for e in scal] == list(range(5))
    assert scal[3]["summary"] == [("cost", -0.5), ("accuracy", 0.25)]


def test_two_writers_same_dir(tmp_path):
    a = summary.FileWriter(str(tmp_path))
    b = summary.FileWriter(str(tmp_path))
    assert a.path != b.path  # two workers on one host share /tmp/mnist/
    a.close(), b.close()
