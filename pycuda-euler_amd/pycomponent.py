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


def component_step_init(d_v, d_D, d_Q, length):
    """src/pycomponent.py:16-62: D[i] = i, Q[i] = 0 (the first of the ten SV step kernels; the
    remaining steps are internal to find_component_device's fixpoint)."""
    n = int(length)
    d_D[:n] = np.arange(n, dtype=np.asarray(d_D).dtype)
    d_Q[:n] = 0
    return d_D, d_Q
