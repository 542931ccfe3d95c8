"""pyeulertour -- drop-in for the reference module src/pyeulertour.py (rows T1-T3, T5, T6).

Euler-tour machinery on the de Bruijn graph of pydebruijn: pair the i-th entering edge of a
vertex with its i-th leaving edge (successor), build the successor graph, its components
(= circuits), the circuit graph and the contig starts.  All device work runs in
libeulerhip.so; the final (c1, c2) sort of the circuit-graph edges stays on the host as in
the reference (:791).  Fixed defects: no unbound circuitGraphEdgeCount when
there is <= 1 circuit, the tree is a list of circuit-graph EDGE indices, contigStart is u32.
"""
import ctypes
import logging

import numpy as np

import _modlib as M

module_logger = logging.getLogger("eulercuda.pyeulertour")


def _ev(x):
    return M.as_struct(x, M.EV)


def _ee(x):
    return M.as_struct(x, M.EE)


def _copy_fields(dst, src):
    if dst is src:
        return dst
    for f in dst.dtype.names:
        dst[f] = src[f]
    return dst


def assign_successor_device(d_ev, d_l, d_e, vcount, d_ee, ecount):
    """src/pyeulertour.py:17-107: ee[e[ep+i]].s = l[lp+i] for i < min(ecount, lcount); returns (ev, ee)."""
    ev, ee = _ev(d_ev), _ee(d_ee)
    M.call("ec_assign_successor", M.ptr(ev), int(vcount), M.ptr(M.arr(d_l, np.uint32)), M.ptr(M.arr(d_e, np.uint32)),
           M.ptr(ee), int(ecount))
    return d_ev, _copy_fields(d_ee, ee)


def construct_successor_graph_device(d_ee, d_v, ecount):
    """src/pyeulertour.py:109-216 (P1 + P2): v[i] = {eid, n1 = s, n2 = predecessor or E}."""
    ee = _ee(d_ee)
    v = np.zeros(int(ecount), M.VTX)
    M.call("ec_successor_graph", M.ptr(ee), int(ecount), M.ptr(v))
    return _copy_fields(d_v, v) if d_v is not None and len(d_v) == len(v) else v


def construct_successor_graphP1_device(d_ee, d_v, ecount):
    """src/pyeulertour.py:109-161 -- computed together with P2 (the n2 links are P2's output)."""
    return construct_successor_graph_device(d_ee, d_v, ecount)


def construct_successor_graphP2_device(d_ee, d_v, ecount):
    """src/pyeulertour.py:164-216"""
    return construct_successor_graph_device(d_ee, d_v, ecount)


# ---- circuit-graph step kernels (src/pyeulertour.py:219-493), one device launch each; the
# reference's arguments, in-place updates and return values.  findEulerDevice runs them fused.
def _u32v(x):
    return np.ascontiguousarray(np.asarray(x).reshape(-1), dtype=np.uint32)


def _into(dst, src):
    if dst is not src:
        np.asarray(dst).reshape(-1)[: src.size] = src
    return dst


def calculate_circuit_graph_vertex_data_device(d_D, d_C, length):
    """src/pyeulertour.py:219-250 (:223-231): C[D[i]] = 1 for i < length; returns (D, C)"""
    D, C = _u32v(d_D)[: int(length)], _u32v(d_C)
    M.call("ec_cg_vertex_data", M.ptr(D), int(length), M.ptr(C), C.size)
    return d_D, _into(d_C, C)


def construct_circuit_Graph_vertex(d_C, d_cg_offset, ecount, d_cv):
    """src/pyeulertour.py:268-304 (:280-288): cv[offset[i]] = i where C[i] != 0; returns cv"""
    C, off, cv = _u32v(d_C)[: int(ecount)], _u32v(d_cg_offset)[: int(ecount)], _u32v(d_cv)
    M.call("ec_cg_vertices", M.ptr(C), M.ptr(off), int(ecount), M.ptr(cv), cv.size)
    return _into(d_cv, cv)


def calculate_circuit_graph_edge_data(d_ev, d_e, vcount, d_D, d_cg_offset, ecount, d_cedgeCount):
    """src/pyeulertour.py:307-390 (:331-371): per circuit c, the circuit-graph edges whose
    smaller end is c (consecutive entering edges on different circuits) added to cedgeCount[c];
    returns cedgeCount"""
    ev, e, D, mp = _ev(np.asarray(d_ev)[: int(vcount)]), _u32v(d_e), _u32v(d_D), _u32v(d_cg_offset)
    cnt = _u32v(d_cedgeCount)
    M.call("ec_cg_edges_step", M.ptr(ev), int(vcount), M.ptr(e), M.ptr(D), M.ptr(mp), mp.size, int(ecount), None,
           M.ptr(cnt), cnt.size, None, 0)
    return _into(d_cedgeCount, cnt)


def assign_circuit_graph_edge_data(d_ev, d_e, vcount, d_D, d_cg_offset, ecount, d_cg_edge_start, d_cedgeCount,
                                   circuitVertexSize, d_cg_edge, circuitGraphEdgeCount):
    """src/pyeulertour.py:393-493 (:428-469): every circuit-graph edge written at
    cg_edge[cg_edge_start[c] + i] with i = atomicDec's return - 1 on cedgeCount[c] (c = min(c1,
    c2)); ceid untouched; cedgeCount is an input only (the reference passes it drv.In).  The
    reference's slot order inside a group is a race; here it is that of a sequential run of its
    threads (vertex, then entry order).  Returns cg_edge."""
    ev, e, D, mp = _ev(np.asarray(d_ev)[: int(vcount)]), _u32v(d_e), _u32v(d_D), _u32v(d_cg_offset)
    start, cnt = _u32v(d_cg_edge_start), _u32v(d_cedgeCount).copy()
    cg = M.as_struct(np.asarray(d_cg_edge).reshape(-1), M.CE)
    ng = min(start.size, cnt.size)
    M.call("ec_cg_edges_step", M.ptr(ev), int(vcount), M.ptr(e), M.ptr(D), M.ptr(mp), mp.size, int(ecount),
           M.ptr(start), M.ptr(cnt), ng, M.ptr(cg), cg.size)  # (slots bounded by the array)
    return _copy_fields(d_cg_edge, cg) if isinstance(d_cg_edge, np.ndarray) and d_cg_edge.dtype.names else cg


def findEulerDevice(d_ev, d_l, d_e, vcount, d_ee, ecount, d_cg_edge, cg_edgeCount, cg_vertexCount):
    """src/pyeulertour.py:714-792: successors (written into d_ee in place), circuits and the
    circuit graph; returns (cg_edge sorted by (c1, c2), cg_edgeCount, cg_vertexCount)."""
    ev, ee = _ev(d_ev), _ee(d_ee)
    E = int(ecount)
    cg = np.zeros(max(E, 1), M.CE)
    ne = ctypes.c_uint64(0)
    nv = ctypes.c_uint32(0)
    M.call("ec_find_euler", M.ptr(ev), int(vcount), M.ptr(M.arr(d_l, np.uint32)), M.ptr(M.arr(d_e, np.uint32)),
           M.ptr(ee), E, M.ptr(cg), ctypes.byref(ne), ctypes.byref(nv))
    _copy_fields(d_ee, ee)
    cg = cg[: ne.value].copy()
    cg.sort(order=["c1", "c2"])  # host sort, as the reference (:791)
    return cg, int(ne.value), int(nv.value)


def mark_spanning_euler_edges(d_ee, d_mark, ecount, d_cg_edge, cg_edgeCount, d_tree, treeCount):
    """src/pyeulertour.py:586-653: mark[min(cg_edge[tree[t]].e1, .e2)] = 1 (mark starts all ones)."""
    return _swipe(None, 0, None, d_ee, ecount, d_cg_edge, cg_edgeCount, d_tree, treeCount, False)[1]


def _swipe(d_ev, vcount, d_e, d_ee, ecount, d_cg_edge, cg_edgeCount, d_tree, treeCount, swipe, merge=False):
    E = int(ecount)
    ee = _ee(d_ee)
    ev = _ev(d_ev) if d_ev is not None else np.zeros(0, M.EV)
    e = M.arr(d_e, np.uint32) if d_e is not None else np.zeros(max(E, 1), np.uint32)
    cg = M.as_struct(d_cg_edge, M.CE) if cg_edgeCount else np.zeros(0, M.CE)
    tree = M.arr(d_tree, np.uint32).reshape(-1)[: int(treeCount)] if treeCount else np.zeros(0, np.uint32)
    mark = np.zeros(max(E, 1), np.uint32)
    M.call("ec_execute_swipe", M.ptr(ev), int(vcount), M.ptr(e), M.ptr(ee), E, M.ptr(cg), int(cg_edgeCount),
           M.ptr(tree), len(tree), (M.EC_MOD_SWIPE if swipe else 0) | (M.EC_MOD_TREE_MARKS if merge else 0),
           M.ptr(mark))
    return _copy_fields(d_ee, ee), mark[:E]


def execute_swipe(d_ev, d_e, vcount, d_ee, d_mark, ecount, swipe=False):
    """src/pyeulertour.py:495-583: the swipe body is commented out in the reference (a no-op);
    swipe=True runs it."""
    return _swipe(d_ev, vcount, d_e, d_ee, ecount, None, 0, None, 0, swipe)


def executeSwipeDevice(d_ev, d_e, vcount, d_ee, ecount, d_cg_edge, cg_edgeCount, d_tree, treeCount, swipe=False,
                       merge=False):
    """src/pyeulertour.py:656-664: mark spanning-tree edges, swipe; returns ee.  d_tree holds
    circuit-graph edge indices (the reference passed vertex pairs).  merge=True
    (with swipe=True): marks start at zero and only the tree's edges rotate, so every connected
    component's circuits merge into one Euler tour (the reference's intent; its merge is a no-op)."""
    return _swipe(d_ev, vcount, d_e, d_ee, ecount, d_cg_edge, cg_edgeCount, d_tree, treeCount, swipe, merge)[0]


def identify_contig_start(d_ee, d_contigStart, ecount):
    """src/pyeulertour.py:667-706: contigStart[ee[i].s] = 0 for s < E (contigStart starts as ones)."""
    ee = _ee(d_ee)
    cs = M.arr(d_contigStart, np.uint32).copy()
    M.call("ec_identify_contig_start", M.ptr(ee), int(ecount), M.ptr(cs))
    d_contigStart[: len(cs)] = cs
    return d_contigStart
