"""ctypes bindings of the host runtime library ``_lib/libtfx_rt.so`` (csrc/runtime): the
parameter-server service/client (ps_service.cpp) and the CRC32C/TFRecord/tfevents writer
(events.cpp).  Plain C ABI, no torch dependency."""
from __future__ import annotations

import ctypes as C
import os
import threading

from ..ops._native import RT_LIB

_lib = None
_lock = threading.Lock()


def lib() -> C.CDLL:
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(RT_LIB):
                raise RuntimeError(f"{RT_LIB} not built (run `python build.py`)")
            L = C.CDLL(RT_LIB)
            vp, cp, u64p = C.c_void_p, C.c_char_p, C.POINTER(C.c_uint64)
            sigs = {
                "tfx_crc32c": (C.c_uint32, [cp, C.c_size_t]),
                "tfx_crc32c_sw": (C.c_uint32, [cp, C.c_size_t]),
                "tfx_masked_crc32c": (C.c_uint32, [cp, C.c_size_t]),
                "tfx_events_open": (vp, [cp, C.c_double]),
                "tfx_events_add_scalars": (None, [vp, C.c_int64, C.c_double, C.c_int, C.POINTER(cp),
                                                  C.POINTER(C.c_float)]),
                "tfx_events_add_bytes": (None, [vp, C.c_int64, C.c_double, C.c_int, cp, C.c_size_t]),
                "tfx_events_add_record": (None, [vp, cp, C.c_size_t]),
                "tfx_events_flush": (None, [vp]),
                "tfx_events_written": (C.c_uint64, [vp]),
                "tfx_events_close": (None, [vp]),
                "tfx_tfrecord_append": (C.c_int, [cp, cp, C.c_size_t]),
                "tfx_ps_server_start": (vp, [cp, C.c_int, C.c_int]),
                "tfx_ps_server_port": (C.c_int, [vp]),
                "tfx_ps_server_stopped": (C.c_int, [vp]),
                "tfx_ps_server_pushes": (C.c_uint64, [vp]),
                "tfx_ps_server_stop": (None, [vp]),
                "tfx_ps_server_read": (C.c_int64, [vp, cp, C.POINTER(C.c_float), C.c_int64]),
                "tfx_ps_connect": (vp, [cp, C.c_int, C.c_int]),
                "tfx_ps_close": (None, [vp]),
                "tfx_ps_create": (C.c_int, [vp, C.c_int, C.POINTER(cp), C.POINTER(vp), u64p, C.c_int]),
                "tfx_ps_uninitialized": (C.c_int, [vp, C.c_int, C.POINTER(cp)]),
                "tfx_ps_pull": (C.c_int, [vp, C.c_int, C.POINTER(cp), C.POINTER(vp), u64p]),
                "tfx_ps_push": (C.c_int, [vp, C.c_int, C.POINTER(cp), C.POINTER(vp), u64p, C.c_float, C.c_int,
                                          C.POINTER(C.c_double)]),
                "tfx_ps_inc": (C.c_int, [vp, cp, C.c_float, C.POINTER(C.c_double)]),
                "tfx_ps_ping": (C.c_int, [vp]),
                "tfx_ps_shutdown": (C.c_int, [vp]),
                "tfx_rt_version": (C.c_int, []),
            }
            for name, (res, args) in sigs.items():
                f = getattr(L, name)
                f.restype = res
                f.argtypes = args
            _lib = L
    return _lib


def crc32c(data: bytes, software: bool = False) -> int:
    f = lib().tfx_crc32c_sw if software else lib().tfx_crc32c
    return int(f(data, len(data)))


def masked_crc32c(data: bytes) -> int:
    return int(lib().tfx_masked_crc32c(data, len(data)))
