"""pydebruijn -- drop-in for the reference module src/pydebruijn.py (rows G1-G5).

Edge-centric de Bruijn graph over l-mers (edges) and (l-1)-mers (vertices, looked up in the
pygpuhash table): per-vertex x4 leaving / entering counts, three exclusive scans, EulerVertex
and EulerEdge arrays, leaving list l[] and entering list e[].  Fixed: the vertex-slot bound
(the reference compares with lmerCount, :449, dropping most edges; ref_bounds=True
reproduces it) and the edge arrays are sized E = sum(lmerValues) (the reference allocates
2*len(lmers) and writes up to E, :574-576).
"""
import ctypes
import logging

import numpy as np

import _modlib as M

module_logger = logging.getLogger("eulercuda.pydebruijn")


def _build(d_lmerKeys, d_lmerValues, lmerCount, d_kmerKeys, kmerCount, l, d_TK, d_TV, d_bucketSize, bucketCount,
           ref_bounds=False):
    lk = M.arr(d_lmerKeys, np.uint64)[: int(lmerCount)]
    lv = M.arr(d_lmerValues, np.uint32)[: int(lmerCount)]
    kk = M.arr(d_kmerKeys, np.uint64)[: int(kmerCount)]
    TK, TV, bs = M.arr(d_TK, np.uint64), M.arr(d_TV, np.uint32), M.arr(d_bucketSize, np.uint32)
    E = int(lv.astype(np.uint64).sum())
    ev = np.zeros(len(kk), M.EV)
    ee = np.zeros(E, M.EE)
    lo = np.zeros(max(E, 1), np.uint32)
    eo = np.zeros(max(E, 1), np.uint32)
    ec = ctypes.c_uint64(0)
    M.call("ec_debruijn_build", M.ptr(lk), M.ptr(lv), len(lk), M.ptr(kk), len(kk), int(l), M.ptr(TK), M.ptr(TV),
           M.ptr(bs), int(bucketCount), M.EC_MOD_REF_BOUNDS if ref_bounds else 0, M.ptr(ev) if len(kk) else None,
           M.ptr(ee) if E else None, M.ptr(lo), M.ptr(eo), ctypes.byref(ec))
    return ev, ee, lo[:E], eo[:E], E


def construct_debruijn_graph_device(d_lmerKeys, d_lmerValues, lmerCount, d_kmerKeys, kmerCount, l, d_TK, d_TV,
                                    d_bucketSize, bucketCount, d_ev, d_l, d_e, d_ee, readLength, ref_bounds=False):
    """src/pydebruijn.py:515-619: returns (ee, ev, l, e, kmerCount, edgeCount)."""
    module_logger.info("started construct_debruijn_graph_device.")
    ev, ee, lo, eo, E = _build(d_lmerKeys, d_lmerValues, lmerCount, d_kmerKeys, kmerCount, l, d_TK, d_TV,
                               d_bucketSize, bucketCount, ref_bounds)
    module_logger.info("Finished construct_debruijn_graph_device.")
    return ee, ev, lo, eo, kmerCount, E


def _l_from_mask(valid_bitmask):
    return bin(int(valid_bitmask)).count("1") // 2 + 1


def debruijn_count_device(d_lmerKeys, d_lmerValues, lmerCount, d_TK, d_TV, d_bucketSize, bucketCount, d_lcount,
                          d_ecount, valid_bitmask, readLength):
    """src/pydebruijn.py:15-178: lcount[4*H(prefix)+last] = ecount[4*H(suffix)+first] = count;
    updates d_lcount / d_ecount in place and returns them."""
    lk = M.arr(d_lmerKeys, np.uint64)[: int(lmerCount)]
    lv = M.arr(d_lmerValues, np.uint32)[: int(lmerCount)]
    lc = M.arr(d_lcount, np.uint32)
    ec = M.arr(d_ecount, np.uint32)
    M.call("ec_db_counts", M.ptr(lk), M.ptr(lv), len(lk), _l_from_mask(valid_bitmask), M.ptr(M.arr(d_TK, np.uint64)),
           M.ptr(M.arr(d_TV, np.uint32)), M.ptr(M.arr(d_bucketSize, np.uint32)), int(bucketCount), len(lc),
           M.ptr(lc), M.ptr(ec))
    d_lcount[:] = lc
    d_ecount[:] = ec
    return d_lcount, d_ecount


def setup_vertices_device(d_kmerKeys, kmerCount, d_TK, d_TV, d_bucketSeed, bucketCount, d_ev, d_lcount, d_lstart,
                          d_ecount, d_estart):
    """src/pydebruijn.py:181-324: ev[H(k)] = {vid, ep, ecount, lp, lcount}; returns ev."""
    kk = M.arr(d_kmerKeys, np.uint64)[: int(kmerCount)]
    ev = M.as_struct(d_ev, M.EV)
    M.call("ec_db_vertices", M.ptr(kk), len(kk), M.ptr(M.arr(d_TK, np.uint64)), M.ptr(M.arr(d_TV, np.uint32)),
           M.ptr(M.arr(d_bucketSeed, np.uint32)), int(bucketCount), M.ptr(M.arr(d_lcount, np.uint32)),
           M.ptr(M.arr(d_lstart, np.uint32)), M.ptr(M.arr(d_ecount, np.uint32)), M.ptr(M.arr(d_estart, np.uint32)),
           M.ptr(ev))
    return ev


def setup_edges_device(d_lmerKeys, d_lmerValues, d_lmerOffsets, lmerCount, d_TK, d_TV, d_bucketSeed, bucketCount,
                       d_l, d_e, d_ee, d_lstart, d_estart, validBitMask, ref_bounds=False):
    """src/pydebruijn.py:326-512: for every copy j of an l-mer: ee[off+j] = {eid, v1, v2, s=E},
    l[lstart+j] = e[estart+j] = off+j; returns (ee, l, e)."""
    lk = M.arr(d_lmerKeys, np.uint64)[: int(lmerCount)]
    lv = M.arr(d_lmerValues, np.uint32)[: int(lmerCount)]
    lo = M.arr(d_lmerOffsets, np.uint32)[: int(lmerCount)]
    ee = M.as_struct(d_ee, M.EE)
    L = M.arr(d_l, np.uint32).copy()
    Ee = M.arr(d_e, np.uint32).copy()
    ls, es = M.arr(d_lstart, np.uint32), M.arr(d_estart, np.uint32)
    M.call("ec_db_edges", M.ptr(lk), M.ptr(lv), M.ptr(lo), len(lk), _l_from_mask(validBitMask),
           M.ptr(M.arr(d_TK, np.uint64)), M.ptr(M.arr(d_TV, np.uint32)), M.ptr(M.arr(d_bucketSeed, np.uint32)),
           int(bucketCount), len(ls) // 4, M.ptr(ls), M.ptr(es), M.EC_MOD_REF_BOUNDS if ref_bounds else 0, M.ptr(ee),
           M.ptr(L), M.ptr(Ee), len(ee))
    return ee, L, Ee


def getOptimalLaunchConfiguration(threadCount, threadPerBlock=32):
    """src/pydebruijn.py:622-640 (API parity)."""
    import pyencode

    return pyencode.getOptimalLaunchConfiguration(threadCount, threadPerBlock)
