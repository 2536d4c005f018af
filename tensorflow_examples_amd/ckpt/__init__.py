"""Checkpoints in TF1's on-disk layout AND TF's V2 tensor-bundle format.

``Saver.save(store, "<dir>/model.ckpt", global_step=N)`` writes::

    <dir>/checkpoint                          text: model_checkpoint_path / all_model_checkpoint_paths
    <dir>/model.ckpt-N.index                  SSTable of BundleEntryProto (dtype, shape, offset, size, crc32c)
    <dir>/model.ckpt-N.data-00000-of-00001    the raw little-endian tensor bytes
    <dir>/model.ckpt-N.meta                   MetaGraphDef protobuf (graph_def, saver_def, collections)
    <dir>/graph.pbtxt                         text GraphDef (write_graph; TF1's Supervisor writes it)

The ``.index`` / ``.data`` pair is TensorFlow's tensor bundle (``ckpt/bundle.py``: LevelDB-format table,
BundleHeaderProto under the empty key, masked CRC32C per tensor and per table block).  The round-1..5
container (JSON index + safetensors data) is still written with ``TFX_CKPT_FORMAT=safetensors`` (or
``Saver(fmt="safetensors")``) and read either way: the reader tells them apart by the index's bytes.
Variables keep their TF names (``global_step``, ``weights/Variable``, ``biases/Variable_1``, ...);
CRC32C of every tensor is verified on restore.  ``.meta`` is a binary MetaGraphDef encoded by
``summary.meta_graph_def``: the graph -- one ``VariableV2`` node per variable with its ``dtype`` /
``shape`` attrs, its ``/read`` and ``/Assign`` nodes, and the ``save/*`` ops the SaverDef names
(:func:`saver_graph_nodes`) -- TF1's default SaverDef, the ``variables`` / ``trainable_variables``
collections (serialized VariableDefs) and a ``tfx_meta`` collection holding the caller's metadata as
JSON; ``read_meta_graph`` parses it.  ``export_saved_model`` writes the SavedModel-shaped directory
``saved_model.pb`` + ``variables/variables.{index,data-00000-of-00001}``; ``saved_model.pb`` is a SavedModel
protobuf (one MetaGraphDef tagged ``serve`` with the graph, SaverDef, variable collections and the serving
SignatureDefs; ``read_saved_model`` parses it).
The reference's Supervisor builds a default Saver but never saves without ``logdir``
(R/distributed/distributed.py:129-131); ``--logdir`` turns it on in this framework.
"""
from __future__ import annotations

import json
import os
import re
import time
from typing import Dict, List, Optional

import torch
from safetensors.torch import load_file, save_file

from .. import runtime, summary
from . import bundle

FORMAT = "tfx-ckpt-v1"  # the JSON + safetensors container (opt-in)
DEFAULT_FORMAT = os.environ.get("TFX_CKPT_FORMAT", "tf")  # "tf" = tensor bundle, "safetensors"
SM_MAGIC = b"TFXSM001"


def _crc(t: torch.Tensor) -> int:
    return runtime.crc32c(t.detach().cpu().contiguous().numpy().tobytes())


def _default_nodes(names: List[str]) -> List[Dict]:
    return [{"name": n, "op": "VariableV2", "inputs": [], "device": ""} for n in names]


def saver_graph_nodes(tensors: Dict[str, torch.Tensor], var_nodes: Optional[List[Dict]] = None) -> List[Dict]:
    """The GraphDef nodes of TF1's default (V2, non-sharded) Saver over ``tensors`` -- what the SaverDef's
    ``save/Const:0`` / ``save/control_dependency:0`` / ``save/restore_all`` name -- plus each variable's
    ``VariableV2`` (dtype / shape attrs), ``<v>/read`` (Identity) and ``<v>/Assign`` nodes (the names its
    VariableDef refers to).  ``var_nodes``: the caller's variable nodes (device placement kept)."""
    names = sorted(tensors)
    dev = {n["name"]: n.get("device", "") for n in (var_nodes or [])}
    dts = {k: bundle._TORCH_DT[v.dtype] for k, v in tensors.items()}
    nodes = []
    for n in names:
        d = dev.get(n, "")
        t = dts[n]
        nodes.append({"name": n, "op": "VariableV2", "inputs": [], "device": d,
                      "attrs": {"dtype": summary.attr_type(t), "shape": summary.attr_shape(tensors[n].shape),
                                "container": summary.attr_str(""), "shared_name": summary.attr_str("")}})
        nodes.append({"name": n + "/read", "op": "Identity", "inputs": [n], "device": d,
                      "attrs": {"T": summary.attr_type(t), "_class": summary.attr_str_list(["loc:@" + n])}})
        nodes.append({"name": n + "/Assign", "op": "Assign", "inputs": [n, n + "/initial_value"], "device": d,
                      "attrs": {"T": summary.attr_type(t), "use_locking": summary.attr_bool(True),
                                "validate_shape": summary.attr_bool(True),
                                "_class": summary.attr_str_list(["loc:@" + n])}})
    str_attr = {"dtype": summary.attr_type(7)}
    nodes.append({"name": "save/Const", "op": "Const", "inputs": [],
                  "attrs": dict(str_attr, value=summary.attr_string_tensor(["model"]))})
    for op in ("SaveV2", "RestoreV2"):
        nodes.append({"name": "save/%s/tensor_names" % op, "op": "Const", "inputs": [],
                      "attrs": dict(str_attr, value=summary.attr_string_tensor(names, [len(names)]))})
        nodes.append({"name": "save/%s/shape_and_slices" % op, "op": "Const", "inputs": [],
                      "attrs": dict(str_attr, value=summary.attr_string_tensor([""] * len(names), [len(names)]))})
    types = summary.attr_type_list([dts[n] for n in names])
    nodes.append({"name": "save/SaveV2", "op": "SaveV2",
                  "inputs": ["save/Const", "save/SaveV2/tensor_names", "save/SaveV2/shape_and_slices", *names],
                  "attrs": {"dtypes": types}})
    nodes.append({"name": "save/control_dependency", "op": "Identity", "inputs": ["save/Const", "^save/SaveV2"],
                  "attrs": {"T": summary.attr_type(7), "_class": summary.attr_str_list(["loc:@save/Const"])}})
    nodes.append({"name": "save/RestoreV2", "op": "RestoreV2",
                  "inputs": ["save/Const", "save/RestoreV2/tensor_names", "save/RestoreV2/shape_and_slices"],
                  "attrs": {"dtypes": types}})
    assigns = []
    for i, n in enumerate(names):
        an = "save/Assign" if i == 0 else "save/Assign_%d" % i
        assigns.append(an)
        nodes.append({"name": an, "op": "Assign", "inputs": [n, "save/RestoreV2:%d" % i if i else "save/RestoreV2"],
                      "attrs": {"T": summary.attr_type(dts[n]), "use_locking": summary.attr_bool(True),
                                "validate_shape": summary.attr_bool(True),
                                "_class": summary.attr_str_list(["loc:@" + n])}})
    nodes.append({"name": "save/restore_all", "op": "NoOp", "inputs": ["^" + a for a in assigns]})
    return nodes


def _write_tensors(prefix: str, tensors: Dict[str, torch.Tensor], meta: Optional[dict],
                   graph_nodes: Optional[List[Dict]] = None, trainable: Optional[Dict[str, bool]] = None,
                   max_to_keep: int = 5, fmt: Optional[str] = None) -> None:
    cpu = {k: v.detach().cpu().contiguous() for k, v in tensors.items()}
    fmt = fmt or DEFAULT_FORMAT
    if fmt == "safetensors":
        save_file(cpu, prefix + ".data-00000-of-00001", metadata={"format": FORMAT})
        index = {"format": FORMAT, "num_shards": 1,
                 "tensors": {k: {"dtype": str(v.dtype).replace("torch.", ""), "shape": list(v.shape), "crc32c": _crc(v)}
                             for k, v in cpu.items()}}
        with open(prefix + ".index", "w") as f:
            json.dump(index, f, indent=1, sort_keys=True)
    elif fmt == "tf":
        bundle.write_bundle(prefix, cpu)
    else:
        raise ValueError("checkpoint format %r (tf | safetensors)" % fmt)
    names = sorted(cpu)
    trainable = trainable or {}
    nodes = saver_graph_nodes(cpu, graph_nodes)
    if graph_nodes is not None:  # the caller's non-variable nodes too (the model graph)
        have = {n["name"] for n in nodes}
        nodes = [n for n in graph_nodes if n["name"] not in have] + nodes
    tr = [n for n in names if trainable.get(n, False)]
    body = summary.meta_graph_def(
        summary.graph_def(nodes), saver=summary.saver_def(max_to_keep),
        collections={"variables": [summary.variable_def(n, trainable.get(n, False)) for n in names],
                     "trainable_variables": [summary.variable_def(n, True) for n in tr],
                     "tfx_meta": [json.dumps({"format": FORMAT if fmt == "safetensors" else "tf-tensor-bundle",
                                              "meta": meta or {}, "time": time.time()}).encode()]})
    with open(prefix + ".meta", "wb") as f:
        f.write(body)


def read_meta_graph(prefix_or_path: str) -> dict:
    """Parse a checkpoint's ``.meta`` (MetaGraphDef): nodes, saver, variable names, user metadata."""
    path = prefix_or_path if prefix_or_path.endswith(".meta") else prefix_or_path + ".meta"
    with open(path, "rb") as f:
        mg = summary.parse_meta_graph_def(f.read())
    colls = mg["collections"]
    mg["variables"] = [summary.parse_variable_def(b)["variable_name"].rsplit(":", 1)[0]
                       for b in colls.get("variables", [])]
    mg["trainable_variables"] = [summary.parse_variable_def(b)["variable_name"].rsplit(":", 1)[0]
                                 for b in colls.get("trainable_variables", [])]
    tm = colls.get("tfx_meta")
    mg["meta"] = json.loads(tm[0])["meta"] if tm else {}
    return mg


def write_graph(logdir: str, nodes: List[Dict], name: str = "graph.pbtxt") -> str:
    """``<logdir>/graph.pbtxt``: the text GraphDef TF1's Supervisor writes when logdir is set
    (R/distributed/distributed.py:129-131)."""
    os.makedirs(logdir, exist_ok=True)
    path = os.path.join(logdir, name)
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        f.write(summary.graph_def_pbtxt(nodes))
    os.replace(tmp, path)
    return path


def read_graph(path: str) -> List[Dict]:
    with open(path) as f:
        return summary.parse_graph_pbtxt(f.read())


def store_graph_nodes(store, device_of=lambda name: "") -> List[Dict]:
    """GraphDef nodes of a VariableStore's variables (VariableV2 each, creation order)."""
    out = [{"name": v.name, "op": "VariableV2", "inputs": [], "device": device_of(v.name)} for v in store.vars]
    out += [{"name": n, "op": "VariableV2", "inputs": [], "device": device_of(n)} for n in store.state]
    return out


def read_checkpoint(prefix: str, verify: bool = True) -> Dict[str, torch.Tensor]:
    """Every tensor of a checkpoint, CRC-checked: TF's tensor bundle or the JSON + safetensors container."""
    if bundle.is_bundle_index(prefix + ".index"):
        return bundle.read_bundle(prefix, verify)
    with open(prefix + ".index") as f:
        index = json.load(f)
    if index.get("format") != FORMAT:
        raise ValueError(f"{prefix}.index: unknown checkpoint format {index.get('format')!r}")
    tensors = load_file(prefix + ".data-00000-of-00001")
    if verify:
        for k, info in index["tensors"].items():
            if _crc(tensors[k]) != info["crc32c"]:
                raise ValueError(f"checkpoint tensor {k!r} fails its CRC32C check")
    return tensors


class Saver:
    def __init__(self, max_to_keep: int = 5, fmt: Optional[str] = None):
        self.max_to_keep = max_to_keep
        self.fmt = fmt  # None = DEFAULT_FORMAT ("tf" tensor bundle unless TFX_CKPT_FORMAT says otherwise)
        self._kept: List[str] = []

    def save(self, store, save_path: str, global_step: Optional[int] = None, extra: Optional[Dict] = None,
             meta: Optional[dict] = None, graph_nodes: Optional[List[Dict]] = None) -> str:
        prefix = f"{save_path}-{int(global_step)}" if global_step is not None else save_path
        d = os.path.dirname(os.path.abspath(prefix))
        os.makedirs(d, exist_ok=True)
        tensors = dict(store.named_values())
        if global_step is not None:
            tensors.setdefault("global_step", torch.tensor(float(global_step)))
        for k, v in (extra or {}).items():
            tensors[k] = torch.as_tensor(v)
        trainable = {v.name: bool(v.trainable) for v in getattr(store, "vars", [])}
        _write_tensors(prefix, tensors, meta, graph_nodes, trainable, self.max_to_keep, self.fmt)
        self._kept = [p for p in _read_state(d) if p != prefix] + [prefix]
        while self.max_to_keep and len(self._kept) > self.max_to_keep:
            old = self._kept.pop(0)
            for suf in (".index", ".data-00000-of-00001", ".meta"):
                try:
                    os.remove(old + suf)
                except FileNotFoundError:
                    pass
        _write_state(d, prefix, self._kept)
        return prefix

    def restore(self, store, prefix: str, strict: bool = True) -> Dict[str, torch.Tensor]:
        tensors = read_checkpoint(prefix)
        store.load_named({k: v for k, v in tensors.items() if k != "global_step"}, strict=strict)
        return tensors


def _state_path(d: str) -> str:
    return os.path.join(d, "checkpoint")


def _read_state(d: str) -> List[str]:
    p = _state_path(d)
    if not os.path.exists(p):
        return []
    out = []
    for line in open(p):
        m = re.match(r'\s*all_model_checkpoint_paths:\s*"(.*)"', line)
        if m:
            q = m.group(1)
            out.append(q if os.path.isabs(q) else os.path.join(d, q))
    return out


def _write_state(d: str, latest: str, all_paths: List[str]) -> None:
    rel = lambda p: os.path.relpath(p, d)  # noqa: E731
    lines = [f'model_checkpoint_path: "{rel(latest)}"'] + [f'all_model_checkpoint_paths: "{rel(p)}"' for p in all_paths]
    tmp = _state_path(d) + ".tmp"
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, _state_path(d))


def latest_checkpoint(checkpoint_dir: str) -> Optional[str]:
    p = _state_path(checkpoint_dir)
    if not os.path.exists(p):
        return None
    for line in open(p):
        m = re.match(r'\s*model_checkpoint_path:\s*"(.*)"', line)
        if m:
            q = m.group(1)
            q = q if os.path.isabs(q) else os.path.join(checkpoint_dir, q)
            return q if os.path.exists(q + ".index") else None
    return None


def export_saved_model(store, export_dir: str, signature: Optional[dict] = None,
                       signature_defs: Optional[Dict[str, dict]] = None, graph_nodes: Optional[List[Dict]] = None,
                       tags=("serve",)) -> str:
    """The SavedModel directory layout: ``saved_model.pb`` -- a SavedModel protobuf (schema version 1, one
    MetaGraphDef tagged ``tags`` with the graph, TF1's default SaverDef, the variable collections and the
    serving ``signature_defs``) -- and ``variables/variables.{index,data-00000-of-00001}`` (the tensor bundle).
    ``signature_defs``: {key: {"inputs": {name: (tensor, dtype, shape)}, "outputs": {...},
    "method_name": ...}}; ``signature`` is free-form caller metadata kept in the ``tfx_meta`` collection."""
    os.makedirs(os.path.join(export_dir, "variables"), exist_ok=True)
    values = store.named_values()
    _write_tensors(os.path.join(export_dir, "variables", "variables"), values, {"saved_model": True})
    trainable = {v.name: bool(v.trainable) for v in store.vars}
    names = sorted(values)
    nodes = graph_nodes if graph_nodes is not None else store_graph_nodes(store)
    sigs = {}
    for key, d in (signature_defs or {}).items():
        ins = {k: summary.tensor_info(*spec) for k, spec in d.get("inputs", {}).items()}
        outs = {k: summary.tensor_info(*spec) for k, spec in d.get("outputs", {}).items()}
        sigs[key] = summary.signature_def(ins, outs, d.get("method_name", "tensorflow/serving/predict"))
    meta = {"format": FORMAT, "signature": signature or {},
            "variables": [{"name": v.name, "shape": list(v.shape)} for v in store.vars]}
    cpu = {k: v.detach().cpu() for k, v in values.items()}
    sv = saver_graph_nodes(cpu, nodes)
    have = {n["name"] for n in sv}
    mg = summary.meta_graph_def(
        summary.graph_def([n for n in nodes if n["name"] not in have] + sv), tags=tags, saver=summary.saver_def(),
        collections={"variables": [summary.variable_def(n, trainable.get(n, False)) for n in names],
                     "trainable_variables": [summary.variable_def(n, True) for n in names if trainable.get(n)],
                     "tfx_meta": [json.dumps(meta).encode()]},
        signatures=sigs)
    tmp = os.path.join(export_dir, "saved_model.pb.tmp")
    with open(tmp, "wb") as f:
        f.write(summary.saved_model([mg]))
    os.replace(tmp, os.path.join(export_dir, "saved_model.pb"))
    return export_dir


def read_saved_model(export_dir: str) -> dict:
    """Parse ``saved_model.pb``: schema version, tags, graph nodes, saver, signature_defs, variables and the
    caller metadata (``meta``).  Round-1..3 exports (magic ``TFXSM001`` + JSON) read too."""
    with open(os.path.join(export_dir, "saved_model.pb"), "rb") as f:
        raw = f.read()
    if raw.startswith(SM_MAGIC):  # the pre-protobuf container
        meta = json.loads(raw[len(SM_MAGIC):])
        return {"schema_version": 0, "tags": [], "nodes": [], "saver": None, "signature_defs": {}, "meta": meta,
                "variables": [v["name"] for v in meta.get("variables", [])]}
    sm = summary.parse_saved_model(raw)
    if not sm["meta_graphs"]:
        raise ValueError(f"{export_dir}/saved_model.pb: no MetaGraphDef")
    mg = sm["meta_graphs"][0]
    colls = mg["collections"]
    tm = colls.get("tfx_meta")
    return {"schema_version": sm["schema_version"], "tags": mg["meta_info"]["tags"], "nodes": mg["nodes"],
            "saver": mg["saver"], "signature_defs": mg["signature_defs"],
            "meta": json.loads(tm[0]) if tm else {},
            "variables": [summary.parse_variable_def(b)["variable_name"].rsplit(":", 1)[0]
                          for b in colls.get("variables", [])]}


def load_saved_model(store, export_dir: str) -> dict:
    """Restore a SavedModel export into ``store``; returns its caller metadata (format, signature,
    variables) plus the parsed ``tags`` and ``signature_defs``."""
    sm = read_saved_model(export_dir)
    tensors = read_checkpoint(os.path.join(export_dir, "variables", "variables"))
    store.load_named(tensors, strict=False)
    meta = dict(sm["meta"])
    meta["tags"], meta["signature_defs"] = sm["tags"], sm["signature_defs"]
    return meta


__all__ = ["Saver", "latest_checkpoint", "read_checkpoint", "export_saved_model", "load_saved_model", "read_saved_model",
           "read_meta_graph", "write_graph", "read_graph", "store_graph_nodes"]
