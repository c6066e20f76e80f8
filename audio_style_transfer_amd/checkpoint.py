"""TensorFlow checkpoint-V2 reading for the encoder weights (the reference's Saver.restore,
methods.py:79-84), through libastyle's native reader (csrc/ckpt.cpp: the .index SSTable of
BundleEntryProtos + the .data shards, CRC-checked).  Host only: no GPU is touched.

    list_variables(prefix)      -> [(name, shape)]          (tf.train.list_variables)
    read_variables(prefix, names=None) -> {name: float32 ndarray}
    encoder_weights(prefix)     -> the 124 encoder variables StyleEngine.set_weights takes
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib
from .weights import weight_shapes


def is_checkpoint(prefix) -> bool:
    return bool(prefix) and os.path.isfile(str(prefix) + '.index')


class _Reader(object):
    def __init__(self, prefix):
        self.lib = _lib.load()
        self.h = ctypes.c_void_p()
        _lib.check(self.lib.ast_ckpt_open(str(prefix).encode(), ctypes.byref(self.h)))

    def close(self):
        if self.h:
            self.lib.ast_ckpt_close(self.h)
            self.h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def entries(self):
        out = []
        name = ctypes.create_string_buffer(4096)
        dt, nd = ctypes.c_int(), ctypes.c_int()
        dims = (ctypes.c_int64 * 16)()
        for i in range(self.lib.ast_ckpt_num_entries(self.h)):
            _lib.check(self.lib.ast_ckpt_entry(self.h, i, name, len(name), ctypes.byref(dt),
                                               ctypes.byref(nd), dims, 16))
            out.append((name.value.decode(), tuple(int(dims[k]) for k in range(nd.value)), dt.value))
        return out

    def read(self, name, shape):
        a = np.empty(shape, dtype=np.float32)
        _lib.check(self.lib.ast_ckpt_read_f32(self.h, name.encode(),
                                              a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                              a.size))
        return a


def list_variables(prefix):
    with _Reader(prefix) as r:
        return [(n, list(s)) for n, s, _ in r.entries()]


def read_variables(prefix, names=None):
    with _Reader(prefix) as r:
        ents = {n: s for n, s, _ in r.entries()}
        names = list(ents) if names is None else list(names)
        missing = [n for n in names if n not in ents]
        if missing:
            raise _lib.AstError('%s: no variable %s' % (prefix, ', '.join(missing[:4])))
        return {n: r.read(n, ents[n]) for n in names}


def encoder_weights(prefix):
    """Every encoder variable (weights.weight_shapes names), shape-checked."""
    shapes = weight_shapes()
    w = read_variables(prefix, list(shapes))
    for n, s in shapes.items():
        if tuple(w[n].shape) != tuple(s):
            raise _lib.AstError('%s: %s has shape %s, the encoder needs %s'
                                % (prefix, n, w[n].shape, tuple(s)))
    return w
