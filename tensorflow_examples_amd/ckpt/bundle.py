"""TensorFlow's tensor-bundle checkpoint format (the V2 checkpoint TF1's ``tf.train.Saver`` writes).

The reference's Supervisor builds TF1's default Saver (R/distributed/distributed.py:129-131), whose V2
checkpoint is two files per prefix:

* ``<prefix>.data-00000-of-00001`` -- the raw little-endian bytes of every tensor, back to back;
* ``<prefix>.index`` -- an SSTable (LevelDB table format: prefix-compressed data blocks with restart
  points, a metaindex block, an index block of BlockHandles and the 48-byte footer with the table
  magic) mapping each tensor name to a serialized ``BundleEntryProto`` {dtype, shape, shard_id,
  offset, size, crc32c (masked CRC32C of the bytes)}; the first key, the empty string, holds the
  ``BundleHeaderProto`` {num_shards, endianness LITTLE, version {producer 1}}.

Every block carries TF's 5-byte trailer (compression type 0 + masked CRC32C of contents + type byte).
The CRC32C is the native runtime's (csrc/runtime/events.cpp, SSE4.2).  This module writes and reads
that format itself (TensorFlow is not importable here, so byte-level importability by TF is "parity
unpinned": the tests check the structure with this reader and the CRCs).
"""
from __future__ import annotations

import struct
from typing import Dict, List, Tuple

import numpy as np
import torch

from .. import runtime

TABLE_MAGIC = 0xDB4775248B80FB57
BLOCK_SIZE = 4096          # TF's table::Options default
RESTART_INTERVAL = 16      # TF's table::Options default
FOOTER_LEN = 48            # 2 x BlockHandle::kMaxEncodedLength (20) + 8-byte magic

# tensorflow DataType enum
_TORCH_DT = {torch.float32: 1, torch.float64: 2, torch.int32: 3, torch.uint8: 4, torch.int16: 5, torch.int8: 6,
             torch.int64: 9, torch.bool: 10, torch.bfloat16: 14, torch.float16: 19}
_DT_TORCH = {v: k for k, v in _TORCH_DT.items()}


# ------------------------------------------------------------------ protobuf wire helpers
def _varint(v: int) -> bytes:
    out = bytearray()
    v &= (1 << 64) - 1
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _read_varint(b: bytes, i: int) -> Tuple[int, int]:
    v, shift = 0, 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << shift
        if c < 0x80:
            return v, i
        shift += 7


def _fld_varint(f: int, v: int) -> bytes:
    return _varint(f << 3) + _varint(int(v))


def _fld_bytes(f: int, data: bytes) -> bytes:
    return _varint((f << 3) | 2) + _varint(len(data)) + data


def _fld_fixed32(f: int, v: int) -> bytes:
    return _varint((f << 3) | 5) + struct.pack("<I", v & 0xFFFFFFFF)


def _parse(b: bytes) -> Dict[int, list]:
    out: Dict[int, list] = {}
    i = 0
    while i < len(b):
        key, i = _read_varint(b, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(b, i)
        elif wt == 1:
            v = struct.unpack_from("<Q", b, i)[0]
            i += 8
        elif wt == 2:
            n, i = _read_varint(b, i)
            v = bytes(b[i:i + n])
            i += n
        elif wt == 5:
            v = struct.unpack_from("<I", b, i)[0]
            i += 4
        else:
            raise ValueError("unsupported protobuf wire type %d" % wt)
        out.setdefault(f, []).append(v)
    return out


def shape_proto(shape) -> bytes:
    """TensorShapeProto { dim { size }* }."""
    return b"".join(_fld_bytes(2, _fld_varint(1, int(d))) for d in shape)


def parse_shape_proto(b: bytes) -> List[int]:
    return [_parse(d).get(1, [0])[0] for d in _parse(b).get(2, [])]


def header_proto(num_shards: int = 1) -> bytes:
    """BundleHeaderProto { num_shards, endianness LITTLE (0, the proto3 default: omitted), version {producer 1} }."""
    return _fld_varint(1, num_shards) + _fld_bytes(3, _fld_varint(1, 1))


def entry_proto(dtype: int, shape, offset: int, size: int, crc: int) -> bytes:
    """BundleEntryProto { dtype, shape, shard_id 0 (omitted), offset, size, crc32c (fixed32, masked) }."""
    out = _fld_varint(1, dtype) + _fld_bytes(2, shape_proto(shape))
    if offset:
        out += _fld_varint(4, offset)
    if size:
        out += _fld_varint(5, size)
    return out + _fld_fixed32(6, crc)


def parse_entry_proto(b: bytes) -> dict:
    f = _parse(b)
    return {"dtype": f.get(1, [0])[0], "shape": parse_shape_proto(f[2][0]) if 2 in f else [],
            "shard_id": f.get(3, [0])[0], "offset": f.get(4, [0])[0], "size": f.get(5, [0])[0],
            "crc32c": f.get(6, [0])[0]}


# ------------------------------------------------------------------ SSTable (LevelDB table format)
class _BlockBuilder:
    def __init__(self):
        self.buf = bytearray()
        self.restarts = [0]
        self.counter = 0
        self.last = b""

    def add(self, key: bytes, value: bytes) -> None:
        shared = 0
        if self.counter < RESTART_INTERVAL:
            n = min(len(self.last), len(key))
            while shared < n and self.last[shared] == key[shared]:
                shared += 1
        else:
            self.restarts.append(len(self.buf))
            self.counter = 0
        self.buf += _varint(shared) + _varint(len(key) - shared) + _varint(len(value))
        self.buf += key[shared:] + value
        self.last = key
        self.counter += 1

    def size(self) -> int:
        return len(self.buf) + 4 * len(self.restarts) + 4

    def finish(self) -> bytes:
        return bytes(self.buf) + b"".join(struct.pack("<I", r) for r in self.restarts) + \
            struct.pack("<I", len(self.restarts))


def _handle(offset: int, size: int) -> bytes:
    return _varint(offset) + _varint(size)


def _write_block(out: bytearray, contents: bytes) -> bytes:
    """Append a block + its trailer (type 0 = uncompressed, masked CRC32C of contents + type); return the
    block's handle."""
    off = len(out)
    out += contents
    trailer_type = b"\x00"
    out += trailer_type + struct.pack("<I", runtime.masked_crc32c(contents + trailer_type))
    return _handle(off, len(contents))


def sstable(items: List[Tuple[bytes, bytes]]) -> bytes:
    """A LevelDB-format table of ``items`` (keys strictly increasing, bytewise)."""
    out = bytearray()
    index = _BlockBuilder()
    blk = _BlockBuilder()
    last_key = None
    for k, v in items:
        if last_key is not None and not k > last_key:
            raise ValueError("sstable keys must be strictly increasing")
        blk.add(k, v)
        last_key = k
        if blk.size() >= BLOCK_SIZE:
            # index entry: any separator >= the block's last key and < the next block's first key works;
            # the last key itself is one
            index.add(last_key, _write_block(out, blk.finish()))
            blk = _BlockBuilder()
    if blk.counter or not items:
        index.add(last_key if last_key is not None else b"", _write_block(out, blk.finish()))
    meta = _write_block(out, _BlockBuilder().finish())  # empty metaindex block
    idx = _write_block(out, index.finish())
    footer = (meta + idx).ljust(FOOTER_LEN - 8, b"\x00") + struct.pack("<Q", TABLE_MAGIC)
    return bytes(out + footer)


def _read_block(data: bytes, handle: bytes, verify: bool) -> List[Tuple[bytes, bytes]]:
    off, i = _read_varint(handle, 0)
    size, _ = _read_varint(handle, i)
    contents = data[off:off + size]
    if verify:
        typ = data[off + size:off + size + 1]
        want = struct.unpack_from("<I", data, off + size + 1)[0]
        if typ != b"\x00":
            raise ValueError("sstable: compressed blocks are not supported")
        if runtime.masked_crc32c(contents + typ) != want:
            raise ValueError("sstable: block CRC32C mismatch at offset %d" % off)
    nrest = struct.unpack_from("<I", contents, len(contents) - 4)[0]
    end = len(contents) - 4 - 4 * nrest
    items, i, last = [], 0, b""
    while i < end:
        shared, i = _read_varint(contents, i)
        nonshared, i = _read_varint(contents, i)
        vlen, i = _read_varint(contents, i)
        key = last[:shared] + contents[i:i + nonshared]
        i += nonshared
        items.append((key, bytes(contents[i:i + vlen])))
        i += vlen
        last = key
    return items


def read_sstable(data: bytes, verify: bool = True) -> List[Tuple[bytes, bytes]]:
    if len(data) < FOOTER_LEN or struct.unpack_from("<Q", data, len(data) - 8)[0] != TABLE_MAGIC:
        raise ValueError("not an SSTable (bad footer magic)")
    footer = data[len(data) - FOOTER_LEN:]
    _, j = _read_varint(footer, 0)   # metaindex handle (an empty block): skipped
    _, j = _read_varint(footer, j)
    io, j = _read_varint(footer, j)  # index handle
    isz, _ = _read_varint(footer, j)
    items = []
    for _, h in _read_block(data, _handle(io, isz), verify):
        items.extend(_read_block(data, h, verify))
    return items


# ------------------------------------------------------------------ the bundle
def is_bundle_index(path: str) -> bool:
    try:
        with open(path, "rb") as f:
            f.seek(-8, 2)
            return struct.unpack("<Q", f.read(8))[0] == TABLE_MAGIC
    except (OSError, struct.error):
        return False


def _tensor_bytes(t: torch.Tensor) -> bytes:
    t = t.detach().cpu().contiguous()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().tobytes()
    return t.numpy().tobytes()


def write_bundle(prefix: str, tensors: Dict[str, torch.Tensor]) -> None:
    """``<prefix>.index`` (SSTable) + ``<prefix>.data-00000-of-00001`` (raw bytes), keys sorted."""
    data = bytearray()
    entries = []
    for name in sorted(tensors):
        t = tensors[name]
        if t.dtype not in _TORCH_DT:
            raise TypeError("tensor %r: dtype %s has no TF DataType here" % (name, t.dtype))
        raw = _tensor_bytes(t)
        entries.append((name.encode(), entry_proto(_TORCH_DT[t.dtype], list(t.shape), len(data), len(raw),
                                                   runtime.masked_crc32c(raw))))
        data += raw
    with open(prefix + ".data-00000-of-00001", "wb") as f:
        f.write(bytes(data))
    with open(prefix + ".index", "wb") as f:
        f.write(sstable([(b"", header_proto(1))] + entries))


def read_bundle_index(prefix: str, verify: bool = True) -> Tuple[dict, Dict[str, dict]]:
    with open(prefix + ".index", "rb") as f:
        items = read_sstable(f.read(), verify)
    if not items or items[0][0] != b"":
        raise ValueError("%s.index: no BundleHeaderProto entry" % prefix)
    h = _parse(items[0][1])
    header = {"num_shards": h.get(1, [0])[0], "endianness": h.get(2, [0])[0],
              "version": _parse(h[3][0]).get(1, [0])[0] if 3 in h else 0}
    return header, {k.decode(): parse_entry_proto(v) for k, v in items[1:]}


def read_bundle(prefix: str, verify: bool = True) -> Dict[str, torch.Tensor]:
    header, entries = read_bundle_index(prefix, verify)
    if header["num_shards"] != 1 or header["endianness"] != 0:
        raise ValueError("%s: only single-shard little-endian bundles are supported" % prefix)
    with open(prefix + ".data-00000-of-00001", "rb") as f:
        data = f.read()
    out = {}
    for name, e in entries.items():
        raw = data[e["offset"]:e["offset"] + e["size"]]
        if verify and runtime.masked_crc32c(raw) != e["crc32c"]:
            raise ValueError("checkpoint tensor %r fails its CRC32C check" % name)
        dt = _DT_TORCH[e["dtype"]]
        if dt == torch.bfloat16:
            t = torch.from_numpy(np.frombuffer(raw, dtype=np.int16).copy()).view(torch.bfloat16)
        else:
            t = torch.from_numpy(np.frombuffer(raw, dtype=torch.empty(0, dtype=dt).numpy().dtype).copy())
        out[name] = t.reshape(e["shape"])
    return out
