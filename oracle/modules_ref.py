"""oracle/modules_ref.py -- TEST INFRASTRUCTURE ONLY.

numpy / pure-Python restatement of the INTENDED semantics of the reference's per-module PyCUDA
kernels (the rows E1-E3, H1-H6, G1-G4, C1, T1-T3, T5, T6 of SURVEY §8a), written from the
kernel sources' behaviour.  Each function cites the reference lines it restates.  Pinned by
the known answers in tests/golden/kat.json (SURVEY §8a E1 values; hash_h values; the bucket
layout of the reference's own dump src/hash_tk.txt) -- see tests/test_modules_oracle.py.
The product (pycuda-euler_amd/) never imports this module.
"""
import numpy as np

CODE_F = [0, 0, 0, 1, 3, 0, 0, 2]  # src/pyencode.py:40 codeF
CODE_R = [0, 3, 0, 2, 0, 0, 0, 1]  # src/pyencode.py:41 codeR
M64 = (1 << 64) - 1
BUCKET_ITEMS = 520                 # src/pygpuhash.py:14


def encode_lmers(buf, L):
    """E1 encodeLmerDevice (src/pyencode.py:43-74): MSB-first codeF of buf[p..p+L-1]; 0 past end."""
    b = bytes(buf)
    n = len(b)
    out = np.zeros(n, np.uint64)
    for p in range(n):
        v = 0
        for i in range(L):
            c = b[p + i] if p + i < n else 0
            v = (v << 2) | CODE_F[c & 7]
        out[p] = v
    return out


def encode_lmers_rc(buf, L):
    """E3 encodeLmerComplementDevice, intended (src/pyencode.py:199-203): sum codeR(c[p+i]) << 2i."""
    b = bytes(buf)
    n = len(b)
    out = np.zeros(n, np.uint64)
    for p in range(n):
        v = 0
        for i in range(L):
            c = b[p + i] if p + i < n else 0
            v |= CODE_R[c & 7] << (2 * i)
        out[p] = v
    return out


def split_kmers(lmers, mask):
    """E2 computeKmerDevice (src/pyencode.py:107-130)."""
    lm = np.asarray(lmers, np.uint64)
    m = np.uint64(mask)
    return (lm & (m << np.uint64(2))) >> np.uint64(2), lm & m


def hash_h(key, nb):
    """src/pygpuhash.py:32-35"""
    return (((0x01010101 + 0x12345678 * int(key)) & M64) % 1900813) % nb


def bucket_count(n):
    return n // 409 + 1  # src/pygpuhash.py:273


def hash_build(keys, vals, nb=0, tail_drop=False):
    """H1-H5 phase1 / scan / copyToBucket / bucketSort (src/pygpuhash.py:36-231, 261-314)."""
    keys = [int(k) for k in keys]
    n = len(keys)
    nb = nb or bucket_count(n)
    used = (n // 1024) * 1024 if tail_drop and n >= 1024 else n
    TK = np.zeros(nb * BUCKET_ITEMS, np.uint64)
    TV = np.zeros(nb * BUCKET_ITEMS, np.uint32)
    size = np.zeros(nb, np.uint32)
    kk = np.array(keys[:used], dtype=np.uint64)
    hb = np.array([hash_h(x, nb) for x in keys[:used]], dtype=np.int64)
    for b in range(nb):
        idx = np.nonzero(hb == b)[0]  # input order
        size[b] = len(idx)
        ks = np.sort(kk[idx])
        rank = np.searchsorted(ks, kk[idx], side="left")  # #{bucket keys < key}
        for i, r in zip(idx, rank):  # a later input index wins a tie
            TK[b * BUCKET_ITEMS + r] = kk[i]
            TV[b * BUCKET_ITEMS + r] = vals[i]
    return TK, TV, size, nb


def hash_lookup(TK, TV, size, nb, key):
    """H6 getHashValue (src/pydebruijn.py:56-87)."""
    b = hash_h(key, nb)
    row = TK[b * BUCKET_ITEMS:b * BUCKET_ITEMS + int(size[b])]
    i = int(np.searchsorted(row, np.uint64(key)))
    if i < len(row) and int(row[i]) == int(key):
        return int(TV[b * BUCKET_ITEMS + i])
    return 0xFFFFFFFF


EV = np.dtype([("vid", "<u8"), ("ep", "<u4"), ("ecount", "<u4"), ("lp", "<u4"), ("lcount", "<u4")])
EE = np.dtype([("eid", "<u8"), ("v1", "<u4"), ("v2", "<u4"), ("s", "<u4"), ("pad", "<u4")])
VTX = np.dtype([("vid", "<u4"), ("n1", "<u4"), ("n2", "<u4")])
CE = np.dtype([("ceid", "<u4"), ("e1", "<u4"), ("e2", "<u4"), ("c1", "<u4"), ("c2", "<u4")])


def debruijn(lmer_keys, lmer_values, kmer_keys, l, table, ref_bounds=False):
    """G1-G4 debruijnCount / scans / setupVertices / setupEdges (src/pydebruijn.py:89-145,
    259-295, 403-477, 515-619) with fixed bounds (4V) unless ref_bounds."""
    TK, TV, size, nb = table
    mask = (1 << (2 * (l - 1))) - 1
    nl, nk = len(lmer_keys), len(kmer_keys)
    V4 = 4 * nk
    lc = np.zeros(V4, np.int64)
    ec = np.zeros(V4, np.int64)
    geo = []
    for i in range(nl):
        x = int(lmer_keys[i])
        pre, suf = (x & (mask << 2)) >> 2, x & mask
        pi, si = hash_lookup(TK, TV, size, nb, pre), hash_lookup(TK, TV, size, nb, suf)
        to = ((pi << 2) & 0xFFFFFFFF) + (x & 3)
        fr = ((si << 2) & 0xFFFFFFFF) + ((x >> (2 * (l - 1))) & 3)
        geo.append((pi, si, to, fr))
        if to < V4:
            lc[to] = lmer_values[i]
        if fr < V4:
            ec[fr] = lmer_values[i]
    ls = np.concatenate([[0], np.cumsum(lc)[:-1]]) if V4 else lc
    es = np.concatenate([[0], np.cumsum(ec)[:-1]]) if V4 else ec
    lv = np.asarray(lmer_values, np.int64)
    lo = np.concatenate([[0], np.cumsum(lv)[:-1]]) if nl else lv
    E = int(lv.sum()) if nl else 0
    ev = np.zeros(nk, EV)
    for key in kmer_keys:
        i = hash_lookup(TK, TV, size, nb, int(key))
        if i < nk:
            q = 4 * i
            ev[i] = (int(key), es[q], ec[q:q + 4].sum(), ls[q], lc[q:q + 4].sum())
    ee = np.zeros(E, EE)
    L = np.zeros(E, np.uint32)
    Ee = np.zeros(E, np.uint32)
    bound = min(nl, V4) if ref_bounds else V4
    for i in range(nl):
        pi, si, to, fr = geo[i]
        if not (to < bound and fr < bound):
            continue
        lo_, eo, off = int(ls[to]), int(es[fr]), int(lo[i])
        if ref_bounds and off >= nl:
            continue
        for _ in range(int(lmer_values[i])):
            if off >= E:
                break
            ee[off] = (off, pi, si, E, 0)
            if lo_ < E:
                L[lo_] = off
            if eo < E:
                Ee[eo] = off
            lo_ += 1
            eo += 1
            off += 1
    return ev, ee, L, Ee, E


def components(vtx):
    """C1 intended fixpoint (src/pycomponent.py:668-723): smallest vertex of the component."""
    n = len(vtx)
    parent = list(range(n))

    def find(x):
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x

    for i in range(n):
        for nb in (int(vtx[i]["n1"]), int(vtx[i]["n2"])):
            if nb < n:
                a, b = find(i), find(nb)
                if a != b:
                    parent[max(a, b)] = min(a, b)
    return np.array([find(i) for i in range(n)], np.uint32)


def find_euler(ev, l, e, ee):
    """T1-T3 findEulerDevice (src/pyeulertour.py:53-83, 133-199, 223-469, 714-792)."""
    ee = ee.copy()
    E = len(ee)
    for v in ev:
        for i in range(min(int(v["ecount"]), int(v["lcount"]))):
            ei, li = int(v["ep"]) + i, int(v["lp"]) + i
            if ei < E:
                x = int(e[ei])
                if li < E and x < E:
                    ee[x]["s"] = l[li]
    vtx = np.zeros(E, VTX)
    vtx["vid"] = ee["eid"].astype(np.uint32)
    vtx["n1"] = ee["s"]
    vtx["n2"] = E
    for i in range(E):
        if vtx[i]["n1"] < E:
            vtx[int(vtx[i]["n1"])]["n2"] = vtx[i]["vid"]
    D = components(vtx) if E else np.zeros(0, np.uint32)
    C = np.zeros(E, np.uint32)
    C[D] = 1
    mp = np.concatenate([[0], np.cumsum(C)[:-1]]).astype(np.uint32) if E else C
    cgV = int(mp[-1] + C[-1]) if E else 0
    edges = []
    if cgV > 1:
        for v in ev:
            if int(v["ecount"]) == 0:
                continue
            mx = int(v["ep"]) + int(v["ecount"]) - 1
            idx = int(v["ep"])
            while idx < mx and idx + 1 < E:
                if int(e[idx]) < E and int(e[idx + 1]) < E:
                    c1, c2 = int(mp[D[e[idx]]]), int(mp[D[e[idx + 1]]])
                    if c1 != c2:
                        edges.append((0, int(e[idx]), int(e[idx + 1]), min(c1, c2), max(c1, c2)))
                idx += 1
    cg = np.array(edges, CE) if edges else np.zeros(0, CE)
    cg.sort(order=["c1", "c2"])
    return ee, cg, cgV


def contig_start(ee):
    """T6 identifyContigStart (src/pyeulertour.py:680-688)."""
    E = len(ee)
    cs = np.ones(E, np.uint32)
    for s in ee["s"]:
        if s < E:
            cs[s] = 0
    return cs


def mark_spanning(cg, tree, E, tree_marks=False):
    """T5 markSpanningEulerEdges (src/pyeulertour.py:613-632): mark starts all ones (:659);
    tree holds circuit-graph EDGE indices.  tree_marks (EC_MOD_TREE_MARKS, the
    intended merge): mark starts at zero and each tree edge marks e1, the first of the two
    consecutive entering edges it joins (assignCircuitGraphEdgeData :458-463)."""
    mark = np.zeros(E, np.uint32) if tree_marks else np.ones(E, np.uint32)
    for t in tree:
        c = cg[int(t)]
        m = int(c["e1"]) if tree_marks else min(int(c["e1"]), int(c["e2"]))
        if m < E:
            mark[m] = 1
    return mark


def swipe(ev, e, ee, mark):
    """T5 executeSwipe, the body the reference comments out (src/pyeulertour.py:534-555): every
    run of marked entering edges of a vertex rotates its successors."""
    ee = ee.copy()
    E = len(ee)
    for v in ev:
        if int(v["ecount"]) == 0:
            continue
        index = int(v["ep"])
        mx = index + int(v["ecount"]) - 1
        if mx >= E:
            continue
        while index < mx and int(ee[int(e[index])]["eid"]) < E:
            if mark[int(ee[int(e[index])]["eid"])] == 1:
                t0, s = index, int(ee[int(e[index])]["s"])
                while mark[int(ee[int(e[index])]["eid"])] == 1 and index < mx:
                    ee[int(e[index])]["s"] = ee[int(e[index + 1])]["s"]
                    index += 1
                if t0 != index:
                    ee[int(e[index])]["s"] = s
            index += 1
    return ee


def successor_cycles(ee):
    """The successor structure of the edges as cycles / paths of edge indices (each edge once):
    paths from the edges no edge points to, then cycles from their smallest edge.  After the
    merge (EC_MOD_TREE_MARKS + swipe) every connected component is one of them."""
    E = len(ee)
    s = [int(x) for x in ee["s"]]
    has_pred = [False] * E
    for x in s:
        if x < E:
            has_pred[x] = True
    seen = [False] * E
    out = []
    for start in [i for i in range(E) if not has_pred[i]] + list(range(E)):
        if seen[start]:
            continue
        walk, x = [], start
        while x < E and not seen[x]:
            seen[x] = True
            walk.append(x)
            x = s[x]
        out.append(walk)
    return out


def lmer_table(buf, l):
    """H0 host dedup of readLmersKmersCuda (src/eulercuda.py:73-179) as the modular pipeline
    feeds it: distinct l-mer codes of the whole buffer with their counts (ascending), the
    distinct (l-1)-mer prefix/suffix codes (ascending)."""
    lm = encode_lmers(buf, l)
    keys, counts = np.unique(lm, return_counts=True)
    mask = (1 << (2 * (l - 1))) - 1
    pre, suf = split_kmers(keys, mask)
    kmers = np.unique(np.concatenate([pre, suf]))
    return keys, counts.astype(np.uint32), kmers


def read_lmers_kmers(buf, L):
    """H0 readLmersKmersCuda (src/eulercuda.py:73-179), dict-for-dict: returns
    [lmerCount, kmerCount, lmerKeys, lmerValues, kmerKeys, kmerValues]."""
    F = encode_lmers(buf, L)
    R = encode_lmers_rc(buf, L)
    mask = (1 << (2 * (L - 1))) - 1
    pF, sF = split_kmers(F, mask)
    pR, sR = split_kmers(R, mask)
    kmerMap, lmerMap = {}, {}
    lmerEmpty = 0
    for i in range(len(F)):
        for x in (pF[i], sF[i], pR[i], sR[i]):
            kmerMap[int(x)] = 1
        for x in (int(F[i]), int(R[i])):
            if x == 0:
                lmerEmpty += 1
            else:
                lmerMap[x] = lmerMap.get(x, 0) + 1
    kmerKeys = list(kmerMap)
    lmerKeys = list(lmerMap)
    lmerValues = list(lmerMap.values())
    if lmerEmpty > 0:  # :175-177 -- overwrites the last real l-mer
        lmerKeys[len(lmerMap) - 1] = 0
        lmerValues[len(lmerMap) - 1] = lmerEmpty
    return [len(lmerMap) + lmerEmpty, len(kmerMap), lmerKeys, lmerValues, kmerKeys, list(range(len(kmerKeys)))]


def get_string(length, value):
    """T7 getString / dna_translate (src/eulercuda.py:307-320)."""
    out = [""] * length
    v = int(value)
    for i in range(1, length + 1):
        out[length - i] = "ACGT"[v % 4]
        v //= 4
    return "".join(out)


def partial_contigs(ev, ee, l):
    """T6 generatePartialContig (src/eulercuda.py:328-402), loop for loop; returns the list of
    buffers (each a list of (l-1)-mer strings)."""
    E = len(ee)
    cs = contig_start(ee)
    visited = np.zeros(E, np.uint32)
    output = []

    def walk(i):
        buf = [get_string(l - 1, ev[int(ee[i]["v1"])]["vid"])]
        nxt = i
        while int(ee[nxt]["s"]) < E and visited[int(ee[nxt]["s"])] == 0:
            visited[nxt] = 1
            nxt = int(ee[nxt]["s"])
            buf.append(get_string(l - 1, ev[int(ee[nxt]["v1"])]["vid"]))
        if visited[nxt] == 0:
            buf.append(get_string(l - 1, ev[int(ee[nxt]["v2"])]["vid"]))
            visited[nxt] = 1
        output.append(buf)

    for i in range(E):
        if cs[i] != 0 and visited[i] == 0:
            walk(i)
    for i in range(E):
        if visited[i] == 0:
            walk(i)
    return output


def spanning_forest(cg, E, V):
    """T4 findSpanningTree (src/eulercuda.py:266-305, graph_tool Kruskal with unit weights):
    restated as Kruskal over the circuit edges in index order -- circuit-edge indices of the
    forest, ascending (the module returns edge indices; parity unpinned: graph_tool's
    tie-breaking among equal weights is unversioned)."""
    parent = list(range(int(V)))

    def find(x):
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x

    tree = []
    for j in range(int(E)):
        a, b = find(int(cg[j]["c1"])), find(int(cg[j]["c2"]))
        if a != b:
            parent[max(a, b)] = min(a, b)
            tree.append(j)
    return tree


# ---- C1 step kernels (src/pycomponent.py:16-665), restated one by one ----------------------
SV_INIT, SV_S1P1, SV_S1P2, SV_S2P1, SV_S2P2, SV_S3P1, SV_S3P2, SV_S4P1, SV_S4P2, SV_S5 = range(10)


def sv_step(step, v, prevD, D, Q, t1, val1, t2, val2, sptemp, n, s):
    """One Shiloach-Vishkin step kernel of the reference over tid < n, in place on the given
    uint32 arrays (elementwise; the P2 atomics are minima / one-value stores, so a sequential
    pass equals the parallel kernel).  Indices past n, which the reference would read out of
    bounds, are skipped (the device restatement does the same)."""
    for t in range(n):
        if step == SV_INIT:  # componentStepInit (:34-43)
            D[t] = t
            Q[t] = 0
        elif step == SV_S1P1:  # componentStepOne_ShortCuttingP1 (:87-94)
            if prevD[t] < n:
                D[t] = prevD[prevD[t]]
        elif step == SV_S1P2:  # componentStepOne_ShortCuttingP2 (:148-158)
            if D[t] != prevD[t] and D[t] < n:
                Q[D[t]] = s
        elif step in (SV_S2P1, SV_S3P1):  # componentStepTwoP1 (:212-242) / ThreeP1 (:394-414)
            d = int(D[t])
            t1[t] = n
            t2[t] = n
            live = d == prevD[t] if step == SV_S2P1 else (d < n and d == D[d] and Q[d] < s)
            if not live:
                continue
            for q, nb in enumerate((int(v[t]["n1"]), int(v[t]["n2"]))):
                if nb >= n:
                    continue
                dn = int(D[nb])
                if (dn < d) if step == SV_S2P1 else (dn != d):
                    (t2 if q else t1)[t] = d
                    (val2 if q else val1)[t] = dn
        elif step in (SV_S2P2, SV_S3P2):  # componentStepTwoP2 (:301-330) / ThreeP2 (:474-494)
            for a, val in ((int(t1[t]), int(val1[t])), (int(t2[t]), int(val2[t]))):
                if a >= n:
                    continue
                D[a] = min(int(D[a]), val)
                if step == SV_S2P2 and val < n:
                    Q[val] = s
        elif step == SV_S4P1:  # componentStepFourP1 (:548-553)
            if D[t] < n:
                val1[t] = D[D[t]]
        elif step == SV_S4P2:  # componentStepFourP2 (:595-601)
            D[t] = val1[t]
        elif step == SV_S5:  # componentStepFive (:638-646)
            if Q[t] == s:
                sptemp[0] = 1


def sv_components(v):
    """find_component_device's intended loop (:689-720, with step 5 called as intended, §A6)
    driven through sv_step; returns D"""
    n = len(v)
    D = np.zeros(n, np.uint32)
    Q = np.zeros(n, np.uint32)
    prevD = np.zeros(n, np.uint32)
    t1, t2, val1, val2 = (np.zeros(n, np.uint32) for _ in range(4))
    sv_step(SV_INIT, v, prevD, D, Q, t1, val1, t2, val2, None, n, 0)
    s, sp = 1, 1
    while s == sp:
        D, prevD = prevD, D
        for st in (SV_S1P1, SV_S1P2, SV_S2P1, SV_S2P2, SV_S3P1, SV_S3P2, SV_S4P1, SV_S4P2):
            sv_step(st, v, prevD, D, Q, t1, val1, t2, val2, None, n, s)
        sp_t = np.zeros(1, np.uint32)
        sv_step(SV_S5, v, prevD, D, Q, t1, val1, t2, val2, sp_t, n, s)
        sp += int(sp_t[0])
        s += 1
    return D


# ---- T3 circuit-graph step kernels (src/pyeulertour.py:219-493) ----------------------------
def cg_vertex_data(D, C):
    """calculateCircuitGraphVertexData (:223-231): C[D[tid]] = 1"""
    C = C.copy()
    for d in D:
        C[d] = 1
    return C


def cg_vertices(C, offset, cv):
    """constructCircuitGraphVertex (:280-288): cv[offset[tid]] = tid where C[tid] != 0"""
    cv = cv.copy()
    for t in range(len(C)):
        if C[t] != 0 and offset[t] < len(cv):
            cv[offset[t]] = t
    return cv


def _cg_pairs(ev, e, D, mp, E):
    """the candidate circuit-graph edges in the order a sequential run of the kernel's threads
    meets them: (c = min, t = max, e1, e2)"""
    out = []
    for v in ev:
        if int(v["ecount"]) == 0:
            continue
        idx, mx = int(v["ep"]), int(v["ep"]) + int(v["ecount"]) - 1
        while idx < mx and idx < E:
            if idx + 1 < E and int(e[idx]) < E and int(e[idx + 1]) < E:
                d1, d2 = int(D[e[idx]]), int(D[e[idx + 1]])
                if d1 < len(mp) and d2 < len(mp):
                    c1, c2 = int(mp[d1]), int(mp[d2])
                    if c1 != c2:
                        out.append((min(c1, c2), max(c1, c2), int(e[idx]), int(e[idx + 1])))
            idx += 1
    return out


def cg_edge_count(ev, e, D, mp, E, cedge_count):
    """calculateCircuitGraphEdgeData (:331-371): atomicInc(cedgeCount + min(c1, c2))"""
    cnt = cedge_count.copy()
    for c, _, _, _ in _cg_pairs(ev, e, D, mp, E):
        cnt[c] += 1
    return cnt


def cg_edge_assign(ev, e, D, mp, E, cedge_offset, cedge_count, cg_edge):
    """assignCircuitGraphEdgeData (:428-469): the r-th candidate of group c (sequential order)
    takes atomicDec's r-th return, slot offset[c] + count[c] - 1 - r; ceid untouched"""
    cg = cg_edge.copy()
    seen = {}
    for c, t, e1, e2 in _cg_pairs(ev, e, D, mp, E):
        r = seen.get(c, 0)
        seen[c] = r + 1
        if r >= int(cedge_count[c]):
            continue
        slot = int(cedge_offset[c]) + int(cedge_count[c]) - 1 - r
        if slot < len(cg):
            cg[slot]["c1"], cg[slot]["c2"], cg[slot]["e1"], cg[slot]["e2"] = c, t, e1, e2
    return cg
