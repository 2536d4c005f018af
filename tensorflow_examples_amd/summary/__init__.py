"""TensorBoard summaries: ``scalar`` / ``merge_all`` / ``FileWriter`` with byte-compatible
tfevents files (reference: R/distributed/distributed.py:120-125 register ``cost`` and
``accuracy`` scalars, :138 opens ``FileWriter(logs_path, graph=...)`` on every worker, :151 calls
``writer.add_summary(summary, step)`` every step).

Encoding/IO is native (csrc/runtime/events.cpp: CRC32C with SSE4.2, TFRecord framing, hand-encoded
Event protos, background flush thread).  Decoding (``summary_iterator``) is Python, for tests
and tools.  File name: ``events.out.tfevents.<unix_ts>.<hostname>`` like TF1; when two writers
on one host open in the same second (two workers) a ``.<pid>`` suffix keeps them apart.
"""
from __future__ import annotations

import ctypes as C
import os
import socket
import struct
import time
from typing import Callable, Dict, Iterator, List, Optional, Sequence, Tuple, Union

from .. import runtime

# ---------------------------------------------------------------- registry (tf.summary.scalar)
_REGISTRY: List[Tuple[str, Callable[[], float]]] = []


class Summary:
    """A Summary proto with scalar values: value { tag, simple_value }."""

    def __init__(self, values: Optional[Sequence[Tuple[str, float]]] = None):
        self.values: List[Tuple[str, float]] = list(values or [])

    def SerializeToString(self) -> bytes:
        out = bytearray()
        for tag, v in self.values:
            val = _bytes_field(1, tag.encode()) + b"\x15" + struct.pack("<f", float(v))
            out += _bytes_field(1, val)
        return bytes(out)

    def __repr__(self):
        return f"Summary({self.values})"


def scalar(name: str, value_fn: Union[Callable[[], float], float]) -> Callable[[], Summary]:
    """Register a scalar summary. ``value_fn`` is evaluated when the merged op runs."""
    fn = value_fn if callable(value_fn) else (lambda v=value_fn: v)
    _REGISTRY.append((name, fn))
    return lambda: Summary([(name, float(fn()))])


def merge_all() -> Callable[[], Summary]:
    """Returns the merged summary op: calling it evaluates every registered scalar."""
    items = list(_REGISTRY)
    return lambda: Summary([(n, float(f())) for n, f in items])


def reset_registry() -> None:
    _REGISTRY.clear()


# ---------------------------------------------------------------- protobuf helpers
def _varint(v: int) -> bytes:
    out = bytearray()
    v &= (1 << 64) - 1
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _bytes_field(field: int, data: bytes) -> bytes:
    return _varint((field << 3) | 2) + _varint(len(data)) + data


def graph_def(nodes: Sequence[Dict]) -> bytes:
    """GraphDef: node { name op input* device attr* } + versions { producer }.
    ``nodes`` = [{"name", "op", "inputs": [...], "device": "...", "attrs": {name: AttrValue bytes}}]
    (``attrs`` optional: the ``attr_*`` helpers below encode the values)."""
    out = bytearray()
    for n in nodes:
        nd = _bytes_field(1, n["name"].encode()) + _bytes_field(2, n["op"].encode())
        for i in n.get("inputs", []):
            nd += _bytes_field(3, i.encode())
        if n.get("device"):
            nd += _bytes_field(4, n["device"].encode())
        for k in sorted(n.get("attrs", {})):  # map<string, AttrValue> attr = 5
            nd += _bytes_field(5, _bytes_field(1, k.encode()) + _bytes_field(2, n["attrs"][k]))
        out += _bytes_field(1, nd)
    out += _bytes_field(4, b"\x08\x1a")  # versions { producer: 26 }
    return bytes(out)


def _varint_field(field: int, v: int) -> bytes:
    return _varint(field << 3) + _varint(int(v))


# AttrValue encoders (oneof: list 1, s 2, i 3, f 4, b 5, type 6, shape 7, tensor 8)
def attr_type(dtype: int) -> bytes:
    return _varint_field(6, dtype)


def attr_bool(v: bool) -> bytes:
    return _varint_field(5, 1 if v else 0)


def attr_str(v: str) -> bytes:
    return _bytes_field(2, v.encode())


def attr_shape(shape: Sequence[int]) -> bytes:
    return _bytes_field(7, b"".join(_bytes_field(2, _varint_field(1, int(d))) for d in shape))


def attr_type_list(dtypes: Sequence[int]) -> bytes:
    return _bytes_field(1, b"".join(_varint_field(6, d) for d in dtypes))


def attr_str_list(values: Sequence[str]) -> bytes:
    return _bytes_field(1, b"".join(_bytes_field(2, v.encode()) for v in values))


def attr_string_tensor(values: Sequence[str], shape: Optional[Sequence[int]] = None) -> bytes:
    """A DT_STRING TensorProto {dtype 7, tensor_shape, string_val*} as an AttrValue (a Const's value)."""
    shp = b"".join(_bytes_field(2, _varint_field(1, int(d))) for d in (shape if shape is not None else []))
    t = _varint_field(1, 7) + _bytes_field(2, shp) + b"".join(_bytes_field(8, v.encode()) for v in values)
    return _bytes_field(8, t)


def parse_node_attrs(node_bytes: bytes) -> Dict[str, Dict[int, list]]:
    """A NodeDef's attr map as {name: parsed AttrValue fields}."""
    out = {}
    for eb in _parse(bytes(node_bytes)).get(5, []):
        e = _parse(eb)
        out[e[1][0].decode()] = _parse(e.get(2, [b""])[0])
    return out


def saver_def(max_to_keep: int = 5, sharded: bool = False) -> bytes:
    """SaverDef { filename_tensor_name, save_tensor_name, restore_op_name, max_to_keep, [sharded],
    keep_checkpoint_every_n_hours, version: V2 } with the names TF1's default (non-sharded) Saver uses --
    the one the Supervisor builds; ``sharded`` is written only when set (proto3 default false).

    The checkpoint ``.meta`` graph carries the ops this SaverDef names (``ckpt.saver_graph_nodes``:
    ``save/Const``, ``save/SaveV2``, ``save/control_dependency``, ``save/RestoreV2``, one ``save/Assign*`` per
    variable, ``save/restore_all``) and its VariableV2 nodes their dtype / shape attrs.  Whether TensorFlow
    imports these bytes is unpinned here (TF is not importable); this package's parsers read them back."""
    return (_bytes_field(1, b"save/Const:0") + _bytes_field(2, b"save/control_dependency:0") +
            _bytes_field(3, b"save/restore_all") + _varint_field(4, max_to_keep) +
            (_varint_field(5, 1) if sharded else b"") + b"\x35" + struct.pack("<f", 10000.0) + _varint_field(7, 2))


def variable_def(name: str, trainable: bool = True) -> bytes:
    """VariableDef { variable_name, initializer_name, snapshot_name, trainable } (TF1 names)."""
    return (_bytes_field(1, f"{name}:0".encode()) + _bytes_field(2, f"{name}/Assign".encode()) +
            _bytes_field(3, f"{name}/read:0".encode()) + _varint_field(7, 1 if trainable else 0))


# tensorflow DataType enum values of the dtypes a signature names
_DT = {"float32": 1, "float64": 2, "int32": 3, "uint8": 4, "int64": 9, "bool": 10, "float16": 19, "bfloat16": 14}
_DT_NAME = {v: k for k, v in _DT.items()}


def tensor_info(name: str, dtype: str = "float32", shape: Optional[Sequence[int]] = None) -> bytes:
    """TensorInfo { name, dtype, tensor_shape { dim { size }* } } (-1 = unknown dimension)."""
    out = _bytes_field(1, name.encode()) + _varint_field(2, _DT[dtype])
    if shape is not None:
        dims = b"".join(_bytes_field(2, _varint_field(1, int(d) & 0xFFFFFFFFFFFFFFFF)) for d in shape)
        out += _bytes_field(3, dims)
    return out


def signature_def(inputs: Dict[str, bytes], outputs: Dict[str, bytes],
                  method_name: str = "tensorflow/serving/predict") -> bytes:
    """SignatureDef { inputs map, outputs map, method_name } from TensorInfo bytes (tensor_info)."""
    out = b""
    for field, m in ((1, inputs), (2, outputs)):
        for k, ti in m.items():
            out += _bytes_field(field, _bytes_field(1, k.encode()) + _bytes_field(2, ti))
    return out + _bytes_field(3, method_name.encode())


def saved_model(meta_graphs: Sequence[bytes]) -> bytes:
    """SavedModel { saved_model_schema_version = 1, meta_graphs* } (the saved_model.pb message)."""
    return _varint_field(1, 1) + b"".join(_bytes_field(2, bytes(m)) for m in meta_graphs)


def meta_graph_def(graph: bytes, tags: Sequence[str] = (), saver: Optional[bytes] = None,
                   collections: Optional[Dict[str, Sequence[bytes]]] = None,
                   signatures: Optional[Dict[str, bytes]] = None) -> bytes:
    """MetaGraphDef: meta_info_def { meta_graph_version, tags*, tensorflow_version,
    tensorflow_git_version } + graph_def (what TF1's FileWriter(graph=...) writes after the GraphDef
    event, R/distributed/distributed.py:138), plus -- for a checkpoint's ``.meta`` (what TF1's
    Saver.save writes next to the data) -- saver_def and collection_def entries
    ``name -> CollectionDef { bytes_list { value* } }`` (e.g. "variables" = serialized VariableDefs)."""
    info = _bytes_field(1, b"v1")
    for t in tags:
        info += _bytes_field(4, t.encode())
    info += _bytes_field(5, b"tensorflow_examples_amd") + _bytes_field(6, b"mi355x-native")
    out = _bytes_field(1, info) + _bytes_field(2, bytes(graph))
    if saver is not None:
        out += _bytes_field(3, saver)
    for key, values in (collections or {}).items():
        blist = b"".join(_bytes_field(1, bytes(v)) for v in values)
        entry = _bytes_field(1, key.encode()) + _bytes_field(2, _bytes_field(2, blist))
        out += _bytes_field(4, entry)
    for key, sig in (signatures or {}).items():  # signature_def map (a SavedModel's serving signatures)
        out += _bytes_field(5, _bytes_field(1, key.encode()) + _bytes_field(2, bytes(sig)))
    return out


def parse_tensor_info(b: bytes) -> Dict:
    f = _parse(bytes(b))
    shape = None
    if 3 in f:
        shape = []
        for db in _parse(f[3][0]).get(2, []):
            v = _parse(db).get(1, [0])[0]
            shape.append(v - (1 << 64) if v >= (1 << 63) else v)
    return {"name": f[1][0].decode(), "dtype": _DT_NAME.get(f.get(2, [0])[0], "invalid"), "shape": shape}


def parse_signature_def(b: bytes) -> Dict:
    f = _parse(bytes(b))
    out = {"inputs": {}, "outputs": {}, "method_name": f.get(3, [b""])[0].decode()}
    for field, key in ((1, "inputs"), (2, "outputs")):
        for eb in f.get(field, []):
            e = _parse(eb)
            out[key][e[1][0].decode()] = parse_tensor_info(e[2][0])
    return out


def parse_saved_model(b: bytes) -> Dict:
    """A SavedModel as {"schema_version", "meta_graphs": [parse_meta_graph_def(...)]}."""
    f = _parse(bytes(b))
    return {"schema_version": f.get(1, [0])[0], "meta_graphs": [parse_meta_graph_def(m) for m in f.get(2, [])]}


def parse_graph_def(b: bytes) -> List[Dict]:
    """Nodes of a binary GraphDef as {"name", "op", "inputs", "device"} dicts (inverse of graph_def)."""
    nodes = []
    for nb in _parse(bytes(b)).get(1, []):
        f = _parse(nb)
        nodes.append({"name": f[1][0].decode(), "op": f.get(2, [b""])[0].decode(),
                      "inputs": [i.decode() for i in f.get(3, [])],
                      "device": f.get(4, [b""])[0].decode(), "attrs": parse_node_attrs(nb)})
    return nodes


def parse_meta_graph_def(b: bytes) -> Dict:
    """A MetaGraphDef as {"meta_info": {...}, "nodes": [...], "saver": {...}, "collections": {...}}."""
    f = _parse(bytes(b))
    info = _parse(f[1][0]) if 1 in f else {}
    out = {"meta_info": {"meta_graph_version": info.get(1, [b""])[0].decode(),
                         "tags": [t.decode() for t in info.get(4, [])],
                         "tensorflow_version": info.get(5, [b""])[0].decode()},
           "nodes": parse_graph_def(f[2][0]) if 2 in f else [], "saver": None, "collections": {}}
    if 3 in f:
        s = _parse(f[3][0])
        out["saver"] = {"filename_tensor_name": s[1][0].decode(), "save_tensor_name": s[2][0].decode(),
                        "restore_op_name": s[3][0].decode(), "max_to_keep": s.get(4, [0])[0],
                        "version": s.get(7, [0])[0]}
    for eb in f.get(4, []):
        e = _parse(eb)
        coll = _parse(e[2][0])
        vals = _parse(coll[2][0]).get(1, []) if 2 in coll else []
        out["collections"][e[1][0].decode()] = [bytes(v) for v in vals]
    out["signature_defs"] = {}
    for eb in f.get(5, []):
        e = _parse(eb)
        out["signature_defs"][e[1][0].decode()] = parse_signature_def(e[2][0])
    return out


def parse_variable_def(b: bytes) -> Dict:
    f = _parse(bytes(b))
    return {"variable_name": f[1][0].decode(), "initializer_name": f.get(2, [b""])[0].decode(),
            "snapshot_name": f.get(3, [b""])[0].decode(), "trainable": bool(f.get(7, [0])[0])}


def _pbtxt_str(s: str) -> str:
    return '"' + s.replace("\\", "\\\\").replace('"', '\\"') + '"'


def graph_def_pbtxt(nodes: Sequence[Dict]) -> str:
    """The text-format GraphDef TF1's Supervisor writes as ``<logdir>/graph.pbtxt``."""
    lines = []
    for n in nodes:
        lines.append("node {")
        lines.append(f"  name: {_pbtxt_str(n['name'])}")
        lines.append(f"  op: {_pbtxt_str(n['op'])}")
        for i in n.get("inputs", []):
            lines.append(f"  input: {_pbtxt_str(i)}")
        if n.get("device"):
            lines.append(f"  device: {_pbtxt_str(n['device'])}")
        lines.append("}")
    lines += ["versions {", "  producer: 26", "}"]
    return "\n".join(lines) + "\n"


def parse_graph_pbtxt(text: str) -> List[Dict]:
    """Reader for :func:`graph_def_pbtxt`'s output (node blocks of name / op / input / device)."""
    import re
    nodes, cur, depth = [], None, 0
    for raw in text.splitlines():
        line = raw.strip()
        if not line:
            continue
        if line.endswith("{"):
            depth += 1
            if depth == 1 and line.startswith("node"):
                cur = {"name": "", "op": "", "inputs": [], "device": ""}
            continue
        if line == "}":
            depth -= 1
            if depth == 0 and cur is not None:
                nodes.append(cur)
                cur = None
            continue
        m = re.match(r'(\w+):\s*"((?:[^"\\]|\\.)*)"$', line)
        if cur is not None and m:
            k, v = m.group(1), m.group(2).replace('\\"', '"').replace("\\\\", "\\")
            if k == "input":
                cur["inputs"].append(v)
            elif k in ("name", "op", "device"):
                cur[k] = v
    return nodes


# ---------------------------------------------------------------- writer
class FileWriter:
    def __init__(self, logdir: str, graph: Optional[Union[bytes, Sequence[Dict]]] = None, filename_suffix: str = ""):
        os.makedirs(logdir, exist_ok=True)
        now = time.time()
        base = os.path.join(logdir, "events.out.tfevents.%010d.%s%s" % (int(now), socket.gethostname(), filename_suffix))
        path = base
        if os.path.exists(path):
            path = f"{base}.{os.getpid()}"
        self.path = path
        self._h = runtime.lib().tfx_events_open(path.encode(), now)
        if not self._h:
            raise OSError(f"cannot open event file {path}")
        if graph is not None:
            self.add_graph(graph)
            self.add_meta_graph(graph)

    def add_graph(self, graph: Union[bytes, Sequence[Dict]], step: int = 0) -> None:
        data = graph if isinstance(graph, (bytes, bytearray)) else graph_def(graph)
        runtime.lib().tfx_events_add_bytes(self._h, int(step), time.time(), 4, bytes(data), len(data))

    def add_meta_graph(self, graph: Union[bytes, Sequence[Dict]], step: int = 0) -> None:
        """Event.meta_graph_def (field 9), as TF1's FileWriter writes it next to the GraphDef."""
        g = graph if isinstance(graph, (bytes, bytearray)) else graph_def(graph)
        data = meta_graph_def(g)
        runtime.lib().tfx_events_add_bytes(self._h, int(step), time.time(), 9, bytes(data), len(data))

    def add_summary(self, summary: Union[Summary, bytes], global_step: Optional[int] = None) -> None:
        step = int(global_step or 0)
        if isinstance(summary, Summary) and summary.values:
            n = len(summary.values)
            tags = (C.c_char_p * n)(*[t.encode() for t, _ in summary.values])
            vals = (C.c_float * n)(*[float(v) for _, v in summary.values])
            runtime.lib().tfx_events_add_scalars(self._h, step, time.time(), n, tags, vals)
        elif isinstance(summary, (bytes, bytearray)):
            runtime.lib().tfx_events_add_bytes(self._h, step, time.time(), 5, bytes(summary), len(summary))

    def add_scalars(self, step: int, **values: float) -> None:
        self.add_summary(Summary(list(values.items())), step)

    def flush(self) -> None:
        if self._h:
            runtime.lib().tfx_events_flush(self._h)

    def close(self) -> None:
        if self._h:
            runtime.lib().tfx_events_close(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


# ---------------------------------------------------------------- reader (tests / tools)
def _read_varint(b: bytes, i: int) -> Tuple[int, int]:
    shift = v = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << shift
        if c < 0x80:
            return v, i
        shift += 7


def _parse(b: bytes) -> Dict[int, list]:
    out: Dict[int, list] = {}
    i = 0
    while i < len(b):
        key, i = _read_varint(b, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(b, i)
        elif wt == 1:
            v = struct.unpack_from("<d", b, i)[0]
            i += 8
        elif wt == 5:
            v = struct.unpack_from("<f", b, i)[0]
            i += 4
        elif wt == 2:
            n, i = _read_varint(b, i)
            v = b[i:i + n]
            i += n
        else:
            raise ValueError(f"unsupported wire type {wt}")
        out.setdefault(f, []).append(v)
    return out


def read_records(path: str, verify: bool = True) -> Iterator[bytes]:
    with open(path, "rb") as fh:
        data = fh.read()
    i = 0
    while i < len(data):
        (n,) = struct.unpack_from("<Q", data, i)
        (lc,) = struct.unpack_from("<I", data, i + 8)
        if verify and runtime.masked_crc32c(data[i:i + 8]) != lc:
            raise ValueError("corrupt record length crc")
        rec = data[i + 12:i + 12 + n]
        (dc,) = struct.unpack_from("<I", data, i + 12 + n)
        if verify and runtime.masked_crc32c(rec) != dc:
            raise ValueError("corrupt record data crc")
        yield rec
        i += 16 + n


def summary_iterator(path: str) -> Iterator[Dict]:
    """Yields dicts: wall_time, step, file_version, graph_def, summary=[(tag, value)]."""
    for rec in read_records(path):
        f = _parse(rec)
        ev = {"wall_time": f.get(1, [0.0])[0], "step": f.get(2, [0])[0]}
        if 3 in f:
            ev["file_version"] = f[3][0].decode()
        if 4 in f:
            ev["graph_def"] = f[4][0]
        if 9 in f:
            ev["meta_graph_def"] = f[9][0]
        if 5 in f:
            vals = []
            for vb in _parse(f[5][0]).get(1, []):
                vf = _parse(vb)
                vals.append((vf[1][0].decode(), vf.get(2, [float("nan")])[0]))
            ev["summary"] = vals
        yield ev


__all__ = ["Summary", "scalar", "merge_all", "FileWriter", "summary_iterator", "read_records", "graph_def",
           "meta_graph_def", "reset_registry", "saver_def", "variable_def", "parse_graph_def",
           "parse_meta_graph_def", "parse_variable_def", "graph_def_pbtxt", "parse_graph_pbtxt"]
