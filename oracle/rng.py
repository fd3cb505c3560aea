"""ORACLE (test infrastructure only): ctypes binding of oracle/mt19937.c.

``np.random.randint(0, high, n)`` under ``np.random.seed(s)`` — the index draw
of rltoolkit/buffer/replay_buffer.py:234 and :418.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "mt19937.c")
LIB = os.path.join(HERE, "_build", "liboracle_mt.so")


def build(force=False):
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", "-o", LIB, SRC])
    return LIB


_lib = None


def _load():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(build())
        _lib.oracle_mt_state_size.restype = ctypes.c_int
        _lib.oracle_mt_seed.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        _lib.oracle_mt_randint.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                           ctypes.c_void_p]
    return _lib


class OracleMT:
    """Host MT19937 stream equivalent to ``np.random.RandomState(seed)``."""

    def __init__(self, seed):
        lib = _load()
        self._buf = ctypes.create_string_buffer(lib.oracle_mt_state_size())
        lib.oracle_mt_seed(self._buf, ctypes.c_uint32(int(seed)))

    def randint(self, high, n):
        out = np.empty(int(n), np.int64)
        _load().oracle_mt_randint(self._buf, int(high), int(n), out.ctypes.data)
        return out
