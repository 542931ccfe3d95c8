"""Shared ctypes plumbing of the per-module drop-ins (pyencode, pygpuhash, pydebruijn,
pycomponent, pyeulertour): symbol registration and numpy <-> pointer helpers."""
import ctypes

import numpy as np

import eulerhip

P = ctypes.c_void_p
U64 = ctypes.c_uint64
U32 = ctypes.c_uint32
INT = ctypes.c_int
UINT = ctypes.c_uint

for name, res, args in [
    ("ec_encode_lmers", INT, [P, U64, U32, P]),
    ("ec_encode_lmers_rc", INT, [P, U64, U32, P]),
    ("ec_split_kmers", INT, [P, U64, U64, P, P]),
    ("ec_hash_bucket_count", U32, [U64]),
    ("ec_hash_build", INT, [P, P, U64, U32, UINT, P, P, P]),
    ("ec_hash_lookup", INT, [P, P, P, U32, P, U64, P]),
    ("ec_hash_phase1", INT, [P, U64, U32, UINT, P, P]),
    ("ec_hash_copy_to_bucket", INT, [P, P, P, U64, P, U32, P, P, U64]),
    ("ec_hash_bucket_sort", INT, [P, P, U64, P, P, U32, P, P]),
    ("ec_debruijn_build", INT, [P, P, U64, P, U64, U32, P, P, P, U32, UINT, P, P, P, P, ctypes.POINTER(U64)]),
    ("ec_components", INT, [P, U64, P]),
    ("ec_find_euler", INT, [P, U64, P, P, P, U64, P, ctypes.POINTER(U64), ctypes.POINTER(U32)]),
    ("ec_execute_swipe", INT, [P, U64, P, P, U64, P, U64, P, U64, UINT, P]),
    ("ec_identify_contig_start", INT, [P, U64, P]),
    ("ec_spanning_forest", INT, [P, U64, U64, P, ctypes.POINTER(U64)]),
    ("ec_assign_successor", INT, [P, U64, P, P, P, U64]),
    ("ec_db_counts", INT, [P, P, U64, U32, P, P, P, U32, U64, P, P]),
    ("ec_db_vertices", INT, [P, U64, P, P, P, U32, P, P, P, P, P]),
    ("ec_db_edges", INT, [P, P, P, U64, U32, P, P, P, U32, U64, P, P, UINT, P, P, P, U64]),
    ("ec_successor_graph", INT, [P, U64, P]),
    ("ec_read_lmers_kmers", INT, [P, U64, U32, P, P, ctypes.POINTER(U64), ctypes.POINTER(U64), P,
                                  ctypes.POINTER(U64)]),
    ("ec_partial_contigs", INT, [P, U64, P, U64, U32, P, P, ctypes.POINTER(U64), ctypes.POINTER(U64)]),
    ("ec_component_step", INT, [INT, P, P, P, P, P, P, P, P, P, U64, U32]),
    ("ec_cg_vertex_data", INT, [P, U64, P, U64]),
    ("ec_cg_vertices", INT, [P, P, U64, P, U64]),
    ("ec_cg_edges_step", INT, [P, U64, P, P, P, U64, U64, P, P, U64, P, U64]),
]:
    eulerhip.register(name, res, args)

EC_MOD_TAIL_DROP = 1
EC_MOD_REF_BOUNDS = 2
EC_MOD_SWIPE = 4
EC_MOD_TREE_MARKS = 8
BUCKET_ITEMS = 520

# the reference's structured dtypes (src/pydebruijn.py:604-606, src/pyeulertour.py:734,785)
EV = np.dtype([("vid", "<u8"), ("ep", "<u4"), ("ecount", "<u4"), ("lp", "<u4"), ("lcount", "<u4")])
EE = np.dtype([("eid", "<u8"), ("v1", "<u4"), ("v2", "<u4"), ("s", "<u4"), ("pad", "<u4")])
VTX = np.dtype([("vid", "<u4"), ("n1", "<u4"), ("n2", "<u4")])
CE = np.dtype([("ceid", "<u4"), ("e1", "<u4"), ("e2", "<u4"), ("c1", "<u4"), ("c2", "<u4")])


def lib():
    return eulerhip.lib()


def call(name, *args):
    return eulerhip.check(getattr(lib(), name)(*args))


def ptr(a):
    """pointer of a C-contiguous numpy array (None for an empty one)"""
    return a.ctypes.data if a is not None and a.size else None


def arr(x, dtype):
    return np.ascontiguousarray(np.asarray(x, dtype=dtype))


def as_struct(x, dtype):
    """a C-contiguous structured array of exactly `dtype` (the reference passes its own)"""
    a = np.ascontiguousarray(x)
    if a.dtype != dtype:
        b = np.zeros(a.shape, dtype)
        for f in dtype.names:
            b[f] = a[f]
        a = b
    return a


def raw_bytes(buffer):
    """the bytes the reference hands to the kernel via drv.In(buffer): a numpy 'S' array
    (possibly 0-d), bytes or str"""
    if isinstance(buffer, np.ndarray):
        return buffer.tobytes()
    if isinstance(buffer, str):
        return buffer.encode("ascii")
    return bytes(buffer)
