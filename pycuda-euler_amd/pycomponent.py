"""pycomponent -- drop-in for the reference module src/pycomponent.py (row C1).

find_component_device labels the connected components of the successor graph, whose vertices
are Vertex{vid, n1, n2} (<= 2 neighbours; a neighbour >= length means none).  The reference
intends a Shiloach-Vishkin fixpoint but stops after one iteration (:716); here the
fixpoint is computed on the GPU (lock-free union by smaller root + pointer jumping) and every
vertex gets the smallest vertex index of its component.
"""
import logging

import numpy as np

import _modlib as M

module_logger = logging.getLogger("eulercuda.pycomponent")


def find_component_device(d_v, d_D, length):
    """src/pycomponent.py:668-723: returns D (filled in place) with D[i] = min vertex of i's
    component."""
    logger = logging.getLogger("eulercuda.pycomponent.find_component_device")
    logger.info("started.")
    n = int(length)
    v = M.as_struct(np.asarray(d_v)[:n], M.VTX)
    D = np.zeros(max(n, 1), np.uint32)
    M.call("ec_components", M.ptr(v), n, M.ptr(D))
    d_D[:n] = D[:n]
    logger.info("Finished. Leaving.")
    return d_D


# ---- the ten Shiloach-Vishkin step kernels (src/pycomponent.py:16-665), one device launch each
# (libeulerhip.so ec_component_step).  Arguments, in-place updates and return values are the
# reference's: every array the reference copies back is updated in place, the listed ones
# returned.  find_component_device's own fixpoint does not go through them (one fused loop).
SV_INIT, SV_S1P1, SV_S1P2, SV_S2P1, SV_S2P2, SV_S3P1, SV_S3P2, SV_S4P1, SV_S4P2, SV_S5 = range(10)


def _u32(x, n):
    """the caller's array as a contiguous uint32 buffer of >= n entries (None passes through)"""
    if x is None:
        return None
    a = np.ascontiguousarray(np.asarray(x).reshape(-1), dtype=np.uint32)
    if a.size < n:
        raise ValueError("array of %d entries, %d needed" % (a.size, n))
    return a


def _back(dst, src):
    """in place into the caller's array (the reference's np_x.get(d_x))"""
    if dst is not None and src is not None and dst is not src:
        np.asarray(dst).reshape(-1)[: src.size] = src
    return dst


def _step(step, d_v, d_prevD, d_D, d_Q, d_t1, d_val1, d_t2, d_val2, d_sptemp, length, s):
    n = int(length)
    v = M.as_struct(np.asarray(d_v)[:n], M.VTX) if d_v is not None else None
    arrs = [_u32(x, n if x is not d_sptemp else 1) for x in (d_prevD, d_D, d_Q, d_t1, d_val1, d_t2, d_val2, d_sptemp)]
    M.call("ec_component_step", int(step), M.ptr(v), *[M.ptr(a) for a in arrs], n, int(s) & 0xFFFFFFFF)
    for dst, a in zip((d_prevD, d_D, d_Q, d_t1, d_val1, d_t2, d_val2, d_sptemp), arrs):
        _back(dst, a)


def component_step_init(d_v, d_D, d_Q, length):
    """src/pycomponent.py:16-64 (componentStepInit :34-43): D[i] = i, Q[i] = 0; returns (D, Q)"""
    _step(SV_INIT, d_v, None, d_D, d_Q, None, None, None, None, None, length, 0)
    return d_D, d_Q


def component_step1_shortcutting_p1(d_v, d_prevD, d_D, d_Q, length, s):
    """src/pycomponent.py:66-123 (:87-94): D[i] = prevD[prevD[i]]; returns D"""
    _step(SV_S1P1, d_v, d_prevD, d_D, d_Q, None, None, None, None, None, length, s)
    return d_D


def component_step1_shortcutting_p2(d_v, d_prevD, d_D, d_Q, length, s):
    """src/pycomponent.py:126-185 (:148-158): Q[D[i]] = s where D[i] != prevD[i]; returns Q"""
    _step(SV_S1P2, d_v, d_prevD, d_D, d_Q, None, None, None, None, None, length, s)
    return d_Q


def component_Step2_P1(d_v, d_prevD, d_D, d_Q, d_t1, d_val1, d_t2, d_val2, length, s):
    """src/pycomponent.py:187-274 (:212-242): hook candidates of unchanged roots (t = length:
    none); returns (t1, t2, val1, val2)"""
    _step(SV_S2P1, d_v, d_prevD, d_D, d_Q, d_t1, d_val1, d_t2, d_val2, None, length, s)
    return d_t1, d_t2, d_val1, d_val2


def component_Step2_P2(d_v, d_prevD, d_D, d_Q, d_t1, d_val1, d_t2, d_val2, length, s):
    """src/pycomponent.py:277-366 (:301-330): D[t] = min(D[t], val), Q[val] = s; returns (D, Q)"""
    _step(SV_S2P2, d_v, d_prevD, d_D, d_Q, d_t1, d_val1, d_t2, d_val2, None, length, s)
    return d_D, d_Q


def component_Step3_P1(d_v, d_prevD, d_D, d_Q, d_t1, d_val1, d_t2, d_val2, length, s):
    """src/pycomponent.py:369-447 (:394-414): hook candidates of stagnant stars; returns
    (t1, t2, val1, val2)"""
    _step(SV_S3P1, d_v, d_prevD, d_D, d_Q, d_t1, d_val1, d_t2, d_val2, None, length, s)
    return d_t1, d_t2, d_val1, d_val2


def component_Step3_P2(d_v, d_prevD, d_D, d_Q, d_t1, d_val1, d_t2, d_val2, length, s):
    """src/pycomponent.py:450-527 (:474-494): D[t] = min(D[t], val); returns D"""
    _step(SV_S3P2, d_v, d_prevD, d_D, d_Q, d_t1, d_val1, d_t2, d_val2, None, length, s)
    return d_D


def component_step4_P1(d_v, d_D, d_val1, length):
    """src/pycomponent.py:529-573 (:548-553): val1[i] = D[D[i]]; returns val1"""
    _step(SV_S4P1, d_v, None, d_D, None, None, d_val1, None, None, None, length, 0)
    return d_val1


def component_step4_P2(d_v, d_D, d_val1, length):
    """src/pycomponent.py:576-622 (:595-601): D[i] = val1[i]; returns D"""
    _step(SV_S4P2, d_v, None, d_D, None, None, d_val1, None, None, None, length, 0)
    return d_D


def component_step5(d_Q, length, d_sptemp, s):
    """src/pycomponent.py:625-665 (:638-646): sptemp[0] = 1 if any Q[i] == s; returns sptemp"""
    _step(SV_S5, None, None, None, d_Q, None, None, None, None, d_sptemp, length, s)
    return d_sptemp
