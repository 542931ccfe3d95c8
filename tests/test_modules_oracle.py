"""CPU checks of the per-module oracle (oracle/modules_ref.py) against the known answers in
tests/golden/kat.json: encode values, hash_h values, and the bucket layout of
the reference's own TK dump src/hash_tk.txt (src/pygpuhash.py:309-311)."""
import json
import os

import numpy as np
import pytest

import modules_ref as R  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def kat():
    with open(os.path.join(HERE, "golden", "kat.json")) as f:
        return json.load(f)


def test_encode_kat(kat):
    for s, L, v in kat["encode"]:
        assert int(R.encode_lmers(s.encode(), L)[0]) == v


def test_encode_tail_and_codes():
    out = R.encode_lmers(b"ACGTN\nacgt", 3)
    # codeF[c & 7]: lowercase maps like uppercase, N / newline -> 0, past the end -> 0
    assert int(out[0]) == 0b000110
    assert int(out[-1]) == (3 << 4)
    assert int(R.encode_lmers(b"acg", 3)[0]) == int(R.encode_lmers(b"ACG", 3)[0])


def test_rc_is_reverse_complement():
    s = b"ACGTTGCAAGGCTA"
    L = 6
    rc = R.encode_lmers_rc(s, L)
    comp = {65: 84, 67: 71, 71: 67, 84: 65}
    for p in range(len(s) - L + 1):
        w = bytes(comp[c] for c in reversed(s[p:p + L]))
        assert int(rc[p]) == int(R.encode_lmers(w, L)[0])


def test_split(kat):
    L = 11
    lm = R.encode_lmers(kat["g200_reads"][0].encode(), L)
    mask = (1 << (2 * (L - 1))) - 1
    pre, suf = R.split_kmers(lm, mask)
    for x, p, q in zip(lm[:50], pre[:50], suf[:50]):
        assert int(p) == int(x) >> 2 and int(q) == int(x) & mask


def test_hash_h_kat(kat):
    for key, nb, v in kat["hash_h"]:
        assert R.hash_h(key, nb) == v


def _dump_keys(kat):
    nb = kat["hash_tk_bucket_count"]
    buckets = [list(b) for b in kat["hash_tk_buckets"]]
    z = R.hash_h(0, nb)
    # the dump is zero-initialised: a literal zero key sits at rank 0 of its bucket
    n_stored = sum(len(b) for b in buckets)
    if n_stored % 1024:
        buckets[z] = [0] + buckets[z]
    return nb, buckets


def test_hash_tk_dump_invariants(kat):
    nb, buckets = _dump_keys(kat)
    assert nb == 77
    assert sum(len(b) for b in buckets) == 30 * 1024
    for b, row in enumerate(buckets):
        assert row == sorted(row)
        assert all(R.hash_h(x, nb) == b for x in row)


def test_hash_build_reproduces_dump(kat):
    """Rebuild from the dump's keys in shuffled order plus a tail that the reference's
    floor(n/1024) grid drops: the layout equals the dump's (implied n in [31084, 31492])."""
    nb, buckets = _dump_keys(kat)
    keys = np.array([x for row in buckets for x in row], np.uint64)
    rng = np.random.default_rng(7)
    rng.shuffle(keys)
    tail = rng.integers(1, 1 << 62, 400, dtype=np.uint64)
    allk = np.concatenate([keys, tail])
    assert R.bucket_count(len(allk)) == nb
    TK, TV, size, nb2 = R.hash_build(allk, np.arange(len(allk), dtype=np.uint32), tail_drop=True)
    assert nb2 == nb
    for b, row in enumerate(buckets):
        assert int(size[b]) == len(row)
        assert [int(x) for x in TK[b * 520:b * 520 + len(row)]] == row
    # every stored key is found, its value is its input index
    for i in range(0, len(keys), 97):
        assert R.hash_lookup(TK, TV, size, nb, int(keys[i])) == i
    assert R.hash_lookup(TK, TV, size, nb, int(tail[0])) == 0xFFFFFFFF


def _pipeline(buf, l):
    keys, counts, kmers = R.lmer_table(buf, l)
    table = R.hash_build(kmers, np.arange(len(kmers), dtype=np.uint32))
    ev, ee, L, Ee, E = R.debruijn(keys, counts, kmers, l, table)
    return keys, counts, kmers, table, ev, ee, L, Ee, E


def test_debruijn_is_an_euler_graph(kat):
    """De Bruijn graph invariants: every edge leaves its prefix vertex and enters its suffix
    vertex; a vertex's entering / leaving lists hold exactly its edges."""
    buf = "".join(kat["g200_reads"][:20]).encode()
    l = 10
    keys, counts, kmers, table, ev, ee, L, Ee, E = _pipeline(buf, l)
    assert E == int(counts.sum())
    assert sorted(L.tolist()) == list(range(E)) and sorted(Ee.tolist()) == list(range(E))
    for v, x in enumerate(ev):
        assert int(x["vid"]) == int(kmers[v])
        for j in range(int(x["lcount"])):
            assert ee[int(L[int(x["lp"]) + j])]["v1"] == v
        for j in range(int(x["ecount"])):
            assert ee[int(Ee[int(x["ep"]) + j])]["v2"] == v


def test_find_euler_circuits(kat):
    buf = "".join(kat["g200_reads"][:20]).encode()
    l = 10
    keys, counts, kmers, table, ev, ee, L, Ee, E = _pipeline(buf, l)
    ee2, cg, cgV = R.find_euler(ev, L, Ee, ee)
    # the successor of an edge leaves the vertex the edge enters, and successors are a permutation
    # of the edges whose source vertex has entering edges
    s = ee2["s"]
    for i in range(E):
        if s[i] < E:
            assert ee2[int(s[i])]["v1"] == ee2[i]["v2"]
    used = s[s < E]
    assert len(np.unique(used)) == len(used)
    assert cgV >= 1
    assert all(c["c1"] < c["c2"] < cgV for c in cg)
    cs = R.contig_start(ee2)
    assert cs.sum() == E - len(used)


def test_components_and_swipe():
    vtx = np.zeros(7, R.VTX)
    vtx["vid"] = np.arange(7)
    vtx["n1"] = [1, 2, 7, 4, 3, 7, 7]
    vtx["n2"] = [7, 0, 1, 4, 3, 7, 5]
    assert R.components(vtx).tolist() == [0, 0, 0, 3, 3, 5, 5]
    mark = R.mark_spanning(np.array([(0, 5, 2, 0, 1)], R.CE), [0], 6)
    assert mark.tolist() == [1] * 6


def _succ_vertices(n, seed, cut=0.05):
    rng = np.random.default_rng(seed)
    s = rng.permutation(n).astype(np.uint32)
    s[rng.random(n) < cut] = n
    v = np.zeros(n, R.VTX)
    v["vid"] = np.arange(n)
    v["n1"] = s
    v["n2"] = n
    for i in range(n):
        if s[i] < n:
            v[s[i]]["n2"] = i
    return v


def _partition(D):
    """component labels -> canonical form (first index of each label)"""
    first = {}
    return [first.setdefault(int(d), i) for i, d in enumerate(D)]


def test_sv_step_loop_is_components():
    """find_component_device's intended loop (src/pycomponent.py:689-720, step 5 called as
    intended) over the restated step kernels labels the same components as the fixpoint"""
    for n, seed in ((1, 0), (7, 1), (200, 2), (1500, 3)):
        v = _succ_vertices(n, seed)
        assert _partition(R.sv_components(v)) == _partition(R.components(v))


def test_cg_step_restatements_compose_to_find_euler(kat):
    """the circuit-graph step kernels restated one by one (src/pyeulertour.py:219-493) give the
    circuit graph find_euler builds in one piece"""
    buf = "".join(kat["g200_reads"][:60]).encode()
    keys, counts, kmers, table, ev, ee, L, Ee, E = _pipeline(buf, 12)
    ree, rcg, cgV = R.find_euler(ev, L, Ee, ee)
    vtx = np.zeros(E, R.VTX)
    vtx["vid"] = ree["eid"].astype(np.uint32)
    vtx["n1"] = ree["s"]
    vtx["n2"] = E
    for i in range(E):
        if vtx[i]["n1"] < E:
            vtx[int(vtx[i]["n1"])]["n2"] = vtx[i]["vid"]
    D = R.components(vtx)
    C = R.cg_vertex_data(D, np.zeros(E, np.uint32))
    mp = np.concatenate([[0], np.cumsum(C)[:-1]]).astype(np.uint32)
    assert int(mp[-1] + C[-1]) == cgV
    cv = R.cg_vertices(C, mp, np.zeros(cgV, np.uint32))
    assert list(cv) == [i for i in range(E) if C[i]]
    cnt = R.cg_edge_count(ev, Ee, D, mp, E, np.zeros(cgV, np.uint32))
    start = np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.uint32)
    cg = R.cg_edge_assign(ev, Ee, D, mp, E, start, cnt, np.zeros(int(cnt.sum()), R.CE))
    assert len(cg) == len(rcg)
    key = lambda a: np.sort(a, order=["c1", "c2", "e1", "e2"])  # noqa: E731
    assert np.array_equal(key(cg), key(rcg))
