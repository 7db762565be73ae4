"""ctypes binding of the native host runtime ``wellflow/_runtime.so`` (csrc/runtime/).

The reference's data path runs in Spark's JVM (cnn.py:49, 65-103); this framework's host
data path is native C++: multithreaded CSV ingest against the submission schema, window
enumeration / batch gathering for the sequence models, and a background prefetcher that
fills pinned host buffers for the host->HBM streamer. Built in-tree by
``python -m wellflow._build`` (g++, no GPU code). ``available()`` tells whether the library
is present; callers fall back to the numpy / pyarrow paths when it is not (CPU-only
checkouts) unless ``WELLFLOW_NATIVE_IO=1`` demands it.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from .schema import FLOAT, INT, Schema

_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_runtime.so")
_LIB = None
_KIND = {INT: 0, FLOAT: 1}

_i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")


def _load():
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(_PATH):
        raise ImportError(f"native runtime not built ({_PATH}); run python -m wellflow._build")
    lib = C.CDLL(_PATH)
    vp = C.c_void_p
    lib.wf_csv_read.restype = vp
    lib.wf_csv_read.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_int), C.c_char, C.c_int, C.c_int,
                                C.c_char_p, C.c_int]
    for name, rt in (("wf_table_rows", C.c_int64), ("wf_table_dropped", C.c_int64)):
        getattr(lib, name).restype = rt
        getattr(lib, name).argtypes = [vp]
    for name in ("wf_table_int", "wf_table_float", "wf_table_codes"):
        getattr(lib, name).restype = vp
        getattr(lib, name).argtypes = [vp, C.c_int]
    lib.wf_table_vocab_size.restype = C.c_int32
    lib.wf_table_vocab_size.argtypes = [vp, C.c_int]
    lib.wf_table_vocab_bytes.restype = C.c_int64
    lib.wf_table_vocab_bytes.argtypes = [vp, C.c_int]
    lib.wf_table_vocab.restype = None
    lib.wf_table_vocab.argtypes = [vp, C.c_int, C.c_char_p, _i64p]
    lib.wf_table_free.restype = None
    lib.wf_table_free.argtypes = [vp]
    lib.wf_window_starts.restype = C.c_int64
    lib.wf_window_starts.argtypes = [vp, C.c_int64, C.c_int, C.c_int, vp, C.c_int64]
    lib.wf_gather_windows.restype = None
    lib.wf_gather_windows.argtypes = [vp, C.c_int, vp, vp, C.c_int64, C.c_int, vp, vp, vp, C.c_int]
    lib.wf_prefetch_create.restype = vp
    lib.wf_prefetch_create.argtypes = [vp, C.c_int, vp, vp, C.c_int, C.c_int, C.c_int,
                                       C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.c_int]
    lib.wf_prefetch_submit.restype = C.c_int
    lib.wf_prefetch_submit.argtypes = [vp, C.c_int, _i64p, C.c_int64]
    lib.wf_prefetch_wait.restype = C.c_int64
    lib.wf_prefetch_wait.argtypes = [vp, C.c_int]
    lib.wf_prefetch_destroy.restype = None
    lib.wf_prefetch_destroy.argtypes = [vp]
    _LIB = lib
    return lib


def available() -> bool:
    try:
        _load()
        return True
    except (ImportError, OSError):
        return False


def wanted() -> bool:
    """Use the native path? ``WELLFLOW_NATIVE_IO``: 0 = never, 1 = always (error if missing),
    unset = when built."""
    v = os.environ.get("WELLFLOW_NATIVE_IO")
    if v == "0":
        return False
    if v == "1":
        _load()
        return True
    return available()


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def read_csv(path: str, schema: Schema, header: bool = False, delimiter: str = ",", threads: int = 0) -> dict:
    """Schema-typed table {name: array} (int -> int64, float -> float32, string -> object),
    rows with unparsable / missing cells dropped; same contract as io.read_csv."""
    lib = _load()
    kinds = (C.c_int * len(schema.fields))(*[_KIND.get(f.kind, 2) for f in schema.fields])
    err = C.create_string_buffer(512)
    t = lib.wf_csv_read(os.fsencode(path), len(schema.fields), kinds, delimiter.encode(), int(header),
                        int(threads), err, 512)
    if not t:
        raise OSError(err.value.decode(errors="replace"))
    try:
        n = lib.wf_table_rows(t)
        out = {}
        for c, f in enumerate(schema.fields):
            if f.kind == INT:
                out[f.name] = np.ctypeslib.as_array(C.cast(lib.wf_table_int(t, c), C.POINTER(C.c_int64)),
                                                    (n,)).copy() if n else np.zeros(0, np.int64)
            elif f.kind == FLOAT:
                out[f.name] = np.ctypeslib.as_array(C.cast(lib.wf_table_float(t, c), C.POINTER(C.c_float)),
                                                    (n,)).copy() if n else np.zeros(0, np.float32)
            else:
                nv = lib.wf_table_vocab_size(t, c)
                buf = C.create_string_buffer(max(1, lib.wf_table_vocab_bytes(t, c)))
                offs = np.zeros(nv + 1, np.int64)
                lib.wf_table_vocab(t, c, buf, offs)
                raw = buf.raw
                vocab = np.empty(nv, dtype=object)
                for k in range(nv):
                    vocab[k] = raw[offs[k]:offs[k + 1]].decode("utf-8", errors="replace")
                codes = (np.ctypeslib.as_array(C.cast(lib.wf_table_codes(t, c), C.POINTER(C.c_int32)), (n,))
                         if n else np.zeros(0, np.int32))
                out[f.name] = vocab[codes] if n else np.zeros(0, dtype=object)
        out_dropped = int(lib.wf_table_dropped(t))
    finally:
        lib.wf_table_free(t)
    read_csv.last_dropped = out_dropped
    return out


read_csv.last_dropped = 0


def window_starts(n: int, T: int, groups=None, stride: int = 1) -> np.ndarray:
    lib = _load()
    g = None if groups is None else np.ascontiguousarray(groups, dtype=np.int64)
    gp = None if g is None else _ptr(g)
    cnt = lib.wf_window_starts(gp, int(n), int(T), int(stride), None, 0)
    out = np.empty(cnt, np.int64)
    if cnt:
        lib.wf_window_starts(gp, int(n), int(T), int(stride), _ptr(out), cnt)
    return out


def gather_windows(rows: np.ndarray, starts: np.ndarray, T: int, idx=None, y=None, out=None, threads: int = 0):
    """[len(idx), T, F] fp32 windows rows[starts[idx[b]] : +T] (and y at each window's last row)."""
    lib = _load()
    rows = np.ascontiguousarray(rows, dtype=np.float32)
    starts = np.ascontiguousarray(starts, dtype=np.int64)
    ix = None if idx is None else np.ascontiguousarray(idx, dtype=np.int64).reshape(-1)
    B = len(starts) if ix is None else len(ix)
    F = rows.shape[1]
    if out is None:
        out = np.empty((B, T, F), np.float32)
    yo = None
    if y is not None:
        y = np.ascontiguousarray(y, dtype=np.float32)
        yo = np.empty(B, np.float32)
    if B:
        lib.wf_gather_windows(_ptr(rows), F, _ptr(starts), None if ix is None else _ptr(ix), B, int(T), _ptr(out),
                              None if y is None else _ptr(y), None if yo is None else _ptr(yo), int(threads))
    return (out, yo) if y is not None else out


class Prefetcher:
    """Background gathers of window batches into ``nslots`` caller-visible host buffers
    (pinned torch tensors when ``pin``), so the host side of batch k+1 overlaps batch k."""

    def __init__(self, rows: np.ndarray, starts: np.ndarray, y: np.ndarray, T: int, batch: int,
                 nslots: int = 3, threads: int = 2, pin: bool = False):
        import torch

        lib = _load()
        self._lib = lib
        self.rows = np.ascontiguousarray(rows, dtype=np.float32)
        self.starts = np.ascontiguousarray(starts, dtype=np.int64)
        self.y = np.ascontiguousarray(y, dtype=np.float32)
        self.T, self.B, self.F = int(T), int(batch), self.rows.shape[1]
        mk = (lambda *s: torch.empty(*s, dtype=torch.float32).pin_memory()) if pin else \
            (lambda *s: torch.empty(*s, dtype=torch.float32))
        self.x_slots = [mk(self.B, self.T, self.F) for _ in range(nslots)]
        self.y_slots = [mk(self.B) for _ in range(nslots)]
        xs = (C.c_void_p * nslots)(*[t.data_ptr() for t in self.x_slots])
        ys = (C.c_void_p * nslots)(*[t.data_ptr() for t in self.y_slots])
        self._h = lib.wf_prefetch_create(_ptr(self.rows), self.F, _ptr(self.starts), _ptr(self.y), self.T, self.B,
                                         nslots, xs, ys, int(threads))
        if not self._h:
            raise ValueError("wf_prefetch_create failed")
        self._pending = {}

    def submit(self, slot: int, idx) -> None:
        ix = np.ascontiguousarray(idx, dtype=np.int64).reshape(-1)
        if len(ix) > self.B:
            raise ValueError("batch larger than the prefetcher's slots")
        self._pending[slot] = ix  # keep alive until waited (the C side copies it anyway)
        if self._lib.wf_prefetch_submit(self._h, int(slot), ix, len(ix)) != 0:
            raise ValueError("bad prefetch slot")

    def wait(self, slot: int):
        n = self._lib.wf_prefetch_wait(self._h, int(slot))
        self._pending.pop(slot, None)
        return self.x_slots[slot][:n], self.y_slots[slot][:n]

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.wf_prefetch_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()
