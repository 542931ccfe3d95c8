"""GPU parity of the per-module drop-ins (pyencode, pygpuhash, pydebruijn, pycomponent,
pyeulertour -> libeulerhip.so) against oracle/modules_ref.py on the same inputs (bit-exact)."""
import json
import os

import numpy as np
import pytest

import modules_ref as R  # noqa: E402

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def kat():
    with open(os.path.join(HERE, "golden", "kat.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def mods():
    import pycomponent
    import pydebruijn
    import pyencode
    import pyeulertour
    import pygpuhash

    return pyencode, pygpuhash, pydebruijn, pycomponent, pyeulertour


def _buffers(kat):
    rng = np.random.default_rng(11)
    g200 = "".join(kat["g200_reads"]).encode()
    rnd = bytes(rng.choice(list(b"ACGTNacgt\n"), 3000).tolist())
    return [g200, rnd, b"ACGT", b"A"]


@pytest.mark.parametrize("L", [1, 3, 11, 21, 31, 32])
def test_encode(kat, mods, L):
    enc = mods[0]
    for buf in _buffers(kat):
        b = np.array(buf.decode()).astype("S")
        d = np.zeros(len(buf), np.uint64)
        out = enc.encode_lmer_device(b, len(buf), d, 0, L)
        assert out is d
        assert np.array_equal(out, R.encode_lmers(buf, L))
        d2 = np.zeros(len(buf), np.uint64)
        assert np.array_equal(enc.compute_lmer_complement_device(b, len(buf), d2, 0, L), R.encode_lmers_rc(buf, L))


def test_encode_kat(kat, mods):
    enc = mods[0]
    for s, L, v in kat["encode"]:
        d = np.zeros(len(s), np.uint64)
        assert int(enc.encode_lmer_device(np.array(s).astype("S"), len(s), d, 0, L)[0]) == v


def test_encode_reference_error_behaviour(mods):
    enc = mods[0]
    d = [0, 0]
    assert enc.encode_lmer_device("AC", 2, d, 0, 2) is d  # non-ndarray input: returned unchanged


def test_split(kat, mods):
    enc = mods[0]
    buf = "".join(kat["g200_reads"]).encode()
    for l in (5, 12, 32):
        lm = R.encode_lmers(buf, l)
        mask = (1 << (2 * (l - 1))) - 1
        pk, sk = np.zeros_like(lm), np.zeros_like(lm)
        enc.compute_kmer_device(lm, pk, sk, mask, 0, len(lm))
        p2, s2 = R.split_kmers(lm, mask)
        assert np.array_equal(pk, p2) and np.array_equal(sk, s2)


def test_hash_reproduces_reference_dump(kat, mods):
    gh = mods[1]
    nb = kat["hash_tk_bucket_count"]
    buckets = [list(b) for b in kat["hash_tk_buckets"]]
    if sum(len(b) for b in buckets) % 1024:
        buckets[R.hash_h(0, nb)] = [0] + buckets[R.hash_h(0, nb)]
    keys = np.array([x for row in buckets for x in row], np.uint64)
    rng = np.random.default_rng(7)
    rng.shuffle(keys)
    tail = rng.integers(1, 1 << 62, 400, dtype=np.uint64)
    allk = np.concatenate([keys, tail])
    vals = np.arange(len(allk), dtype=np.uint32)
    tl, size, nb2, TK, TV = gh.create_hash_table_device(allk, vals, len(allk), None, None, 0, None, 0, tail_drop=True)
    assert nb2 == nb and tl == nb * 520
    for b, row in enumerate(buckets):
        assert int(size[b]) == len(row)
        assert [int(x) for x in TK[b * 520:b * 520 + len(row)]] == row
    rTK, rTV, rsize, _ = R.hash_build(allk, vals, tail_drop=True)
    assert np.array_equal(TK, rTK) and np.array_equal(TV, rTV) and np.array_equal(size, rsize)
    # lookups: hits give the input index, misses 0xFFFFFFFF
    got = gh.hash_lookup(np.concatenate([keys[:500], tail[:50]]), TK, TV, size, nb)
    assert got[:500].tolist() == list(range(500))
    assert (got[500:] == 0xFFFFFFFF).all()
    # fixed default: nothing dropped
    tl, size, nb3, TK, TV = gh.create_hash_table_device(allk, vals, len(allk), None, None, 0, None, 0)
    assert int(size.sum()) == len(allk)
    assert (gh.hash_lookup(tail, TK, TV, size, nb3) == vals[len(keys):]).all()


def test_hash_steps(mods):
    gh = mods[1]
    rng = np.random.default_rng(3)
    keys = rng.integers(0, 1 << 40, 5000, dtype=np.uint64)
    keys[100:110] = keys[0]  # duplicates: the later index wins the shared rank
    vals = np.arange(len(keys), dtype=np.uint32)
    nb = R.bucket_count(len(keys))
    off, cnt = gh.phase1_device(keys, None, len(keys), None, nb)
    hb = np.array([R.hash_h(int(x), nb) for x in keys])
    assert np.array_equal(cnt, np.bincount(hb, minlength=nb))
    for b in range(nb):  # offsets: a permutation of 0..size-1 inside each bucket
        assert sorted(off[hb == b].tolist()) == list(range(int(cnt[b])))
    start = np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.uint32)
    bk, bv = gh.copy_to_bucket_device(keys, vals, off, len(keys), start, nb, np.zeros(len(keys), np.uint64),
                                      np.zeros(len(keys), np.uint32))
    assert np.array_equal(bk[start[hb] + off], keys)
    TK, TV = gh.bucket_sort_device(bk, bv, start, cnt, nb, np.zeros(0), np.zeros(0))
    rTK, rTV, rsize, _ = R.hash_build(keys, vals, nb)
    assert np.array_equal(TK, rTK) and np.array_equal(TV, rTV)


def _ref_pipeline(buf, l, ref_bounds=False):
    keys, counts, kmers = R.lmer_table(buf, l)
    table = R.hash_build(kmers, np.arange(len(kmers), dtype=np.uint32))
    ev, ee, L, Ee, E = R.debruijn(keys, counts, kmers, l, table, ref_bounds)
    return keys, counts, kmers, table, ev, ee, L, Ee, E


@pytest.mark.parametrize("l,nreads,ref_bounds", [(10, 20, False), (12, 200, False), (8, 50, True), (21, 200, False)])
def test_debruijn_and_euler(kat, mods, l, nreads, ref_bounds):
    enc, gh, db, cc, et = mods
    buf = "".join(kat["g200_reads"][:nreads]).encode()
    keys, counts, kmers, (TK, TV, size, nb), ev, ee, L, Ee, E = _ref_pipeline(buf, l, ref_bounds)
    mask = (1 << (2 * (l - 1))) - 1
    tl, gsize, gnb, gTK, gTV = gh.create_hash_table_device(kmers, np.arange(len(kmers), dtype=np.uint32), len(kmers),
                                                           None, None, 0, None, 0)
    assert np.array_equal(gTK, TK) and np.array_equal(gTV, TV)
    gee, gev, gl, ge, kc, gE = db.construct_debruijn_graph_device(keys, counts, len(keys), kmers, len(kmers), l, gTK,
                                                                  gTV, gsize, gnb, None, None, None, None, 0,
                                                                  ref_bounds=ref_bounds)
    assert gE == E
    assert np.array_equal(gev, ev) and np.array_equal(gee, ee)
    assert np.array_equal(gl, L) and np.array_equal(ge, Ee)
    # step-level G1 / G3 / G4
    V4 = 4 * len(kmers)
    lc, ec = np.zeros(V4, np.uint32), np.zeros(V4, np.uint32)
    db.debruijn_count_device(keys, counts, len(keys), gTK, gTV, gsize, gnb, lc, ec, mask, 0)
    ls = np.concatenate([[0], np.cumsum(lc)[:-1]]).astype(np.uint32)
    es = np.concatenate([[0], np.cumsum(ec)[:-1]]).astype(np.uint32)
    ev3 = db.setup_vertices_device(kmers, len(kmers), gTK, gTV, gsize, gnb, np.zeros(len(kmers), R.EV), lc, ls, ec, es)
    assert np.array_equal(ev3, ev)
    lo = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.uint32)
    ee3, l3, e3 = db.setup_edges_device(keys, counts, lo, len(keys), gTK, gTV, gsize, gnb, np.zeros(E, np.uint32),
                                        np.zeros(E, np.uint32), np.zeros(E, R.EE), ls, es, mask, ref_bounds=ref_bounds)
    assert np.array_equal(ee3, ee) and np.array_equal(l3, L) and np.array_equal(e3, Ee)
    # Euler tour: successors, circuits, circuit graph
    ree, rcg, rcgV = R.find_euler(ev, L, Ee, ee)
    work = ee.copy()
    cg, ncg, cgV = et.findEulerDevice(ev, L, Ee, len(ev), work, E, None, 0, 0)
    assert np.array_equal(work, ree)
    assert cgV == rcgV and ncg == len(rcg)
    key = lambda a: np.sort(a, order=["c1", "c2", "e1", "e2"])  # noqa: E731 -- ties in (c1, c2) are unordered
    assert np.array_equal(key(cg), key(rcg))
    assert np.array_equal(cg[["c1", "c2"]], rcg[["c1", "c2"]])
    # step-level successor + successor graph + components
    ev2, ee2 = et.assign_successor_device(ev, L, Ee, len(ev), ee.copy(), E)
    assert np.array_equal(ee2, ree)
    v = et.construct_successor_graph_device(ee2, None, E)
    D = cc.find_component_device(v, np.zeros(E, np.uint32), E)
    assert np.array_equal(D, R.components(v))
    cs = et.identify_contig_start(ree, np.ones(E, np.uint32), E)
    assert np.array_equal(cs, R.contig_start(ree))
    # spanning marks + the swipe the reference leaves commented out
    tree = np.arange(0, ncg, 2, dtype=np.uint32)
    mk = et.mark_spanning_euler_edges(ree, None, E, cg, ncg, tree, len(tree))
    assert np.array_equal(mk, R.mark_spanning(cg, tree, E))
    if ref_bounds:  # the reference's bounds leave e with repeated slots: no well-defined swipe
        import eulerhip

        with pytest.raises(eulerhip.EulerHipError):
            et.executeSwipeDevice(ev, Ee, len(ev), ree.copy(), E, cg, ncg, tree, len(tree), swipe=True)
    else:
        sw = et.executeSwipeDevice(ev, Ee, len(ev), ree.copy(), E, cg, ncg, tree, len(tree), swipe=True)
        assert np.array_equal(sw, R.swipe(ev, Ee, ree, R.mark_spanning(cg, tree, E)))
    nosw = et.executeSwipeDevice(ev, Ee, len(ev), ree.copy(), E, cg, ncg, tree, len(tree))
    assert np.array_equal(nosw, ree)  # reference: the swipe body is commented out


def test_components_random(mods):
    cc = mods[3]
    rng = np.random.default_rng(5)
    for n in (1, 2, 17, 5000, 100000):
        # random successor permutation -> cycles; break some links -> paths
        s = rng.permutation(n).astype(np.uint32)
        s[rng.random(n) < 0.01] = n
        v = np.zeros(n, R.VTX)
        v["vid"] = np.arange(n)
        v["n1"] = s
        v["n2"] = n
        for i in range(n):
            if s[i] < n:
                v[s[i]]["n2"] = i
        D = cc.find_component_device(v, np.zeros(n, np.uint32), n)
        assert np.array_equal(D, R.components(v))


def test_spanning_forest_vs_kruskal():
    """T4 on the device (ec_spanning_forest, Boruvka) = Kruskal in edge-index order (the
    restatement of src/eulercuda.py:266-305): the KAT forest, random multigraphs with self-loops
    and isolated circuits, a long path (many rounds), empty input"""
    import eulercuda

    cg = np.zeros(6, R.CE)
    cg["c1"] = [0, 0, 1, 2, 3, 3]
    cg["c2"] = [1, 2, 2, 3, 4, 4]
    assert eulercuda.findSpanningTree(cg, 6, 6).tolist() == [0, 1, 3, 4]
    rng = np.random.default_rng(4)
    for V, E in [(10, 30), (1000, 800), (1000, 5000), (50_000, 120_000), (3, 0)]:
        cg = np.zeros(E, R.CE)
        cg["c1"] = rng.integers(0, V, E)
        cg["c2"] = rng.integers(0, V, E)
        cg["ceid"] = np.arange(E)
        assert eulercuda.findSpanningTree(cg, E, V).tolist() == R.spanning_forest(cg, E, V), (V, E)
    V = 20_000  # a path given in reverse: every vertex hooks to v + 1, one chain of length V
    cg = np.zeros(V - 1, R.CE)
    cg["c1"] = np.arange(V - 1)[::-1]
    cg["c2"] = np.arange(1, V)[::-1]
    assert eulercuda.findSpanningTree(cg, V - 1, V).tolist() == list(range(V - 1))


def test_spanning_forest_long_chain_time():
    """10^6 circuits on a forward-sorted path: round 1 hooks every vertex to v - 1, a single
    chain of length 10^6; the roots are found by pointer jumping (log2 launches), not by a serial
    chase per vertex (O(n^2))"""
    import time

    import eulercuda

    for V in (1_000_000, 300_001):
        cg = np.zeros(V - 1, R.CE)
        cg["c1"] = np.arange(V - 1)
        cg["c2"] = np.arange(1, V)
        cg["ceid"] = np.arange(V - 1)
        t = time.perf_counter()
        tree = eulercuda.findSpanningTree(cg, V - 1, V)
        dt = time.perf_counter() - t
        assert np.array_equal(tree, np.arange(V - 1)), V
        assert dt < 10.0, (V, dt)
    # two interleaved chains joined at the end, plus isolated circuits
    rng = np.random.default_rng(9)
    V = 200_000
    perm = rng.permutation(V)
    cg = np.zeros(V - 2, R.CE)
    cg["c1"] = perm[:-2]
    cg["c2"] = perm[1:-1]
    cg["ceid"] = np.arange(V - 2)
    assert eulercuda.findSpanningTree(cg, V - 2, V).tolist() == R.spanning_forest(cg, V - 2, V)


def _euler_graph(seqs, l):
    """de Bruijn multigraph of circular sequences (every vertex balanced: an Euler graph), laid
    out by the pydebruijn restatement: l-mer keys / multiplicities / (l-1)-mer vertex keys"""
    code = {"A": 0, "C": 1, "G": 2, "T": 3}
    cnt = {}
    for s in seqs:
        t = s + s[: l - 1]
        for i in range(len(s)):
            x = 0
            for c in t[i:i + l]:
                x = (x << 2) | code[c]
            cnt[x] = cnt.get(x, 0) + 1
    keys = np.array(sorted(cnt), dtype=np.uint64)
    counts = np.array([cnt[int(x)] for x in keys], dtype=np.uint32)
    mask = (1 << (2 * (l - 1))) - 1
    kmers = np.unique(np.concatenate([(keys >> np.uint64(2)) & np.uint64(mask), keys & np.uint64(mask)]))
    table = R.hash_build(kmers, np.arange(len(kmers), dtype=np.uint32))
    ev, ee, L, Ee, E = R.debruijn(keys, counts, kmers, l, table)
    return ev, ee, L, Ee, E


@pytest.mark.parametrize("seed,nseq,n,l", [(1, 1, 400, 8), (2, 5, 300, 7), (3, 20, 200, 6), (4, 3, 3000, 10),
                                           (5, 40, 60, 5)])
def test_euler_circuit_merge(mods, seed, nseq, n, l):
    """SURVEY §8f row 4, the merge the reference leaves as a no-op: successor pairing, circuits,
    spanning forest of the circuit graph, then the swipe with only the forest's edges marked
    (EC_MOD_TREE_MARKS).  Every connected component of the Euler graph becomes ONE tour whose
    consecutive edges meet (v2(e) = v1(s(e))); the swipe equals its restatement on the same tree"""
    import eulercuda

    enc, gh, db, cc, et = mods
    rng = np.random.default_rng(60 + seed)
    seqs = []
    while len(seqs) < nseq:
        s = "".join(rng.choice(list("ACGT"), n))
        if "A" * l not in s + s[: l]:  # (the all-A l-mer is the reference's empty key)
            seqs.append(s)
    ev, ee, L, Ee, E = _euler_graph(seqs, l)
    merged = eulercuda.mergeEulerCircuits(ev, ee, L, Ee, E, len(ev))
    # components of the graph (edges' vertices united)
    par = list(range(len(ev)))

    def find(x):
        while par[x] != x:
            par[x] = par[par[x]]
            x = par[x]
        return x

    for x in ee:
        a, b = find(int(x["v1"])), find(int(x["v2"]))
        if a != b:
            par[max(a, b)] = min(a, b)
    ncomp = len({find(int(x["v1"])) for x in ee})
    tours = R.successor_cycles(merged)
    assert sorted(i for t in tours for i in t) == list(range(E))
    assert len(tours) == ncomp, (len(tours), ncomp)
    for t in tours:
        assert int(merged[t[-1]]["s"]) == t[0]  # closed: a circuit
        for a, b in zip(t, t[1:] + t[:1]):
            assert int(merged[a]["v2"]) == int(merged[b]["v1"])
    # the swipe itself against its restatement, on the device's circuit graph and forest
    ree, _, _ = R.find_euler(ev, L, Ee, ee)
    work = ee.copy()
    cg, ncg, cgV = et.findEulerDevice(ev, L, Ee, len(ev), work, E, None, 0, 0)
    if ncg:
        tree = eulercuda.findSpanningTree(cg, ncg, cgV)
        sw = et.executeSwipeDevice(ev, Ee, len(ev), work.copy(), E, cg, ncg, tree, len(tree), swipe=True, merge=True)
        assert np.array_equal(sw, R.swipe(ev, Ee, work, R.mark_spanning(cg, tree, E, tree_marks=True)))
        assert len(R.successor_cycles(sw)) == ncomp


# ---- step-level drop-ins of C1 / T3 (round 5): pycomponent.component_* and the circuit-graph
# steps of pyeulertour, each against its restatement in oracle/modules_ref.py
def _sv_vertices(n, seed, cut=0.03):
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


@pytest.mark.parametrize("n,seed", [(1, 1), (9, 2), (300, 3), (4000, 4)])
def test_component_steps_vs_restatement(mods, n, seed):
    """every SV step kernel (src/pycomponent.py:16-665) on the states the intended loop
    (:689-720) passes through, in place, against modules_ref.sv_step"""
    cc = mods[3]
    v = _sv_vertices(n, seed)
    rng = np.random.default_rng(seed)
    # device and reference states side by side
    st = {k: np.zeros(n, np.uint32) for k in ("D", "Q", "prevD", "t1", "t2", "val1", "val2")}
    ref = {k: a.copy() for k, a in st.items()}
    # garbage in val1 / val2: P1 must leave them where it writes no candidate
    for d in (st, ref):
        d["val1"][:] = d["val2"][:] = 0
    junk = rng.integers(0, max(n, 1), n).astype(np.uint32)
    st["val1"][:] = junk
    ref["val1"][:] = junk
    out = cc.component_step_init(v, st["D"], st["Q"], n)
    assert out[0] is st["D"] and out[1] is st["Q"]
    R.sv_step(R.SV_INIT, v, ref["prevD"], ref["D"], ref["Q"], ref["t1"], ref["val1"], ref["t2"], ref["val2"], None, n, 0)
    s, sp = 1, 1
    calls = [
        (R.SV_S1P1, lambda: cc.component_step1_shortcutting_p1(v, st["prevD"], st["D"], st["Q"], n, s)),
        (R.SV_S1P2, lambda: cc.component_step1_shortcutting_p2(v, st["prevD"], st["D"], st["Q"], n, s)),
        (R.SV_S2P1, lambda: cc.component_Step2_P1(v, st["prevD"], st["D"], st["Q"], st["t1"], st["val1"], st["t2"],
                                                  st["val2"], n, s)),
        (R.SV_S2P2, lambda: cc.component_Step2_P2(v, st["prevD"], st["D"], st["Q"], st["t1"], st["val1"], st["t2"],
                                                  st["val2"], n, s)),
        (R.SV_S3P1, lambda: cc.component_Step3_P1(v, st["prevD"], st["D"], st["Q"], st["t1"], st["val1"], st["t2"],
                                                  st["val2"], n, s)),
        (R.SV_S3P2, lambda: cc.component_Step3_P2(v, st["prevD"], st["D"], st["Q"], st["t1"], st["val1"], st["t2"],
                                                  st["val2"], n, s)),
        (R.SV_S4P1, lambda: cc.component_step4_P1(v, st["D"], st["val1"], n)),
        (R.SV_S4P2, lambda: cc.component_step4_P2(v, st["D"], st["val1"], n)),
    ]
    rounds = 0
    while s == sp:
        st["D"], st["prevD"] = st["prevD"], st["D"]
        ref["D"], ref["prevD"] = ref["prevD"], ref["D"]
        for step, call in calls:
            call()
            R.sv_step(step, v, ref["prevD"], ref["D"], ref["Q"], ref["t1"], ref["val1"], ref["t2"], ref["val2"], None,
                      n, s)
            for k in st:
                assert np.array_equal(st[k], ref[k]), (step, k, s)
        sptemp = np.zeros(1, np.uint32)
        assert cc.component_step5(st["Q"], n, sptemp, s) is sptemp
        rsp = np.zeros(1, np.uint32)
        R.sv_step(R.SV_S5, v, ref["prevD"], ref["D"], ref["Q"], ref["t1"], ref["val1"], ref["t2"], ref["val2"], rsp, n, s)
        assert sptemp[0] == rsp[0]
        sp += int(sptemp[0])
        s += 1
        rounds += 1
        assert rounds < 64
    # the loop run as intended labels the components
    first = {}
    want = [first.setdefault(int(d), i) for i, d in enumerate(R.components(v))]
    first = {}
    assert [first.setdefault(int(d), i) for i, d in enumerate(st["D"])] == want


@pytest.mark.parametrize("l,nreads", [(10, 40), (12, 200), (21, 200)])
def test_circuit_graph_steps_vs_restatement(kat, mods, l, nreads):
    """calculate_circuit_graph_vertex_data_device / construct_circuit_Graph_vertex /
    calculate_circuit_graph_edge_data / assign_circuit_graph_edge_data (src/pyeulertour.py:219-493)
    one launch each against their restatements, and composed into findEulerDevice's circuit
    graph"""
    enc, gh, db, cc, et = mods
    buf = "".join(kat["g200_reads"][:nreads]).encode()
    keys, counts, kmers, table, ev, ee, L, Ee, E = _ref_pipeline(buf, l, False)
    ree, rcg, rcgV = R.find_euler(ev, L, Ee, ee)
    v = et.construct_successor_graph_device(ree, None, E)
    D = cc.find_component_device(v, np.zeros(E, np.uint32), E)
    C = np.zeros(E, np.uint32)
    D2, C2 = et.calculate_circuit_graph_vertex_data_device(D, C, E)
    assert C2 is C and np.array_equal(C, R.cg_vertex_data(D, np.zeros(E, np.uint32)))
    mp = np.concatenate([[0], np.cumsum(C)[:-1]]).astype(np.uint32)
    cgV = int(mp[-1] + C[-1]) if E else 0
    assert cgV == rcgV
    cv = np.zeros(max(cgV, 1), np.uint32)
    assert et.construct_circuit_Graph_vertex(C, mp, E, cv) is cv
    assert np.array_equal(cv, R.cg_vertices(C, mp, np.zeros(max(cgV, 1), np.uint32)))
    cnt = np.zeros(max(cgV, 1), np.uint32)
    assert et.calculate_circuit_graph_edge_data(ev, Ee, len(ev), D, mp, E, cnt) is cnt
    assert np.array_equal(cnt, R.cg_edge_count(ev, Ee, D, mp, E, np.zeros(max(cgV, 1), np.uint32)))
    start = np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.uint32)
    ncg = int(cnt.sum())
    cg = np.zeros(max(ncg, 1), R.CE)
    cg["ceid"] = 7  # the kernel leaves ceid alone
    cnt_in = cnt.copy()
    got = et.assign_circuit_graph_edge_data(ev, Ee, len(ev), D, mp, E, start, cnt, cgV, cg, ncg)
    assert got is cg and np.array_equal(cnt, cnt_in)  # cedgeCount is an input (drv.In)
    want = R.cg_edge_assign(ev, Ee, D, mp, E, start, cnt, np.array([(7, 0, 0, 0, 0)] * max(ncg, 1), R.CE))
    assert np.array_equal(cg, want)
    key = lambda a: np.sort(a[:ncg], order=["c1", "c2", "e1", "e2"])[["e1", "e2", "c1", "c2"]]  # noqa: E731
    assert ncg == len(rcg) and np.array_equal(key(cg), key(rcg))
