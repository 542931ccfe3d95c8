"""GPU parity of the reference-interface host modules: assembler.build / all_contigs /
assemble against the golden vectors of the reference CPU assembler, eulercuda.assemble2 in
both modes, and the device H0 / T6 steps against their oracle restatements."""
import collections
import json
import os

import numpy as np
import pytest

import modules_ref as R
import model_parallel
from conftest import GOLDEN, golden_cases

pytestmark = pytest.mark.gpu

CASES = golden_cases("g200.json", "synthetic.json")


@pytest.fixture(scope="module")
def asm():
    import assembler

    return assembler


@pytest.fixture(scope="module")
def ec():
    import eulercuda

    return eulercuda


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_build_and_all_contigs(asm, case):
    k, limit = case["k"], case["limit"]
    d = asm.build(case["reads"], k, limit)
    assert [[x, v] for x, v in d.items()] == case["d"]
    G, r = asm.all_contigs(d, k)
    assert r == case["contigs"]
    assert [[[list(x) for x in G[i][0]], [list(x) for x in G[i][1]]] for i in range(len(r))] == case["links"]
    d2, G2, r2 = asm.assemble(case["reads"], k, limit)
    assert d2 == d and r2 == r and G2 == G


@pytest.mark.parametrize("seed", range(6))
def test_all_contigs_any_dict_order(asm, seed):
    """all_contigs follows the caller's dict order (contig starts = first entry of each
    component): shuffled dicts against the design model, which is pinned to the reference."""
    c = [x for x in CASES if x["name"] == "g200_k11"][0]
    k = c["k"]
    rng = np.random.default_rng(seed)
    items = list(c["d"])
    rng.shuffle(items)
    d = collections.OrderedDict((x, v) for x, v in items)
    G, r = asm.all_contigs(d, k)
    first = {x: i for i, (x, _) in enumerate(items)}
    cnt = {min(x, model_parallel.twin(x)): v for x, v in items}
    _, mr, ml = model_parallel.model_graph(cnt, first, k)
    assert r == mr
    assert [[[list(x) for x in G[i][0]], [list(x) for x in G[i][1]]] for i in range(len(r))] == ml


EXT = golden_cases("synthetic.json", alphabet="extended") + golden_cases("extended.json", alphabet="all")[::4]


@pytest.mark.parametrize("case", EXT, ids=[c["name"] for c in EXT])
def test_all_contigs_extended_dict(asm, case):
    """all_contigs on build()'s dict of reads with opaque bytes (a caller's dict of arbitrary
    strings: ec_assemble_from_kmers on the extended alphabet) gives the reference's contigs and G"""
    k = case["k"]
    d = collections.OrderedDict((x, v) for x, v in case["d"])
    G, r = asm.all_contigs(d, k)
    assert r == case["contigs"]
    assert [[[list(x) for x in G[i][0]], [list(x) for x in G[i][1]]] for i in range(len(r))] == case["links"]


def test_all_contigs_rejects_bad_input(asm):
    import eulerhip

    # opaque R is its own complement, so RCGT is ACGR's twin: all_contigs marks the twin of every
    # contig k-mer done (tests/referenceAssembler.py all_contigs), one contig, no links
    G, r = asm.all_contigs({"ACGR": 2, "RCGT": 2}, 4)
    assert r == ["ACGR"] and G == {0: ([], [])}
    with pytest.raises(eulerhip.EulerHipError):
        asm.all_contigs({"ACG": 2}, 4)
    assert asm.all_contigs({}, 5) == ({}, [])


def test_assemble2_fused(ec, tmp_path):
    c = [x for x in CASES if x["name"] == "g200_k15"][0]
    out = tmp_path / "contigs.fa"
    contigs = ec.assemble2(c["k"] + 1, buffer=c["reads"], outfile=str(out))
    assert contigs == c["contigs"]
    lines = out.read_text().splitlines()
    assert lines[0::2] == [">%u" % i for i in range(len(contigs))] and lines[1::2] == contigs
    contigs2 = ec.assemble2(c["k"] + 1, infile=os.path.join(GOLDEN, "g200reads.fa"))
    assert contigs2 == c["contigs"]


@pytest.mark.parametrize("L,nreads", [(4, 30), (8, 100), (12, 200), (21, 200), (32, 200)])
def test_read_lmers_kmers(ec, L, nreads):
    kat = json.load(open(os.path.join(GOLDEN, "kat.json")))
    buf = "".join(kat["g200_reads"][:nreads]).encode()
    got = ec.readLmersKmersCuda(buf, 20, len(buf), L, [], [], 0, [], [], 0, nreads)
    assert got == R.read_lmers_kmers(buf, L)


def _oracle_modular(buf, l):
    lc, kc, lk, lv, kk, kv = R.read_lmers_kmers(buf, l)
    table = R.hash_build(np.array(kk, np.uint64), np.array(kv, np.uint32))
    ev, ee, L, Ee, E = R.debruijn(np.array(lk, np.uint64), np.array(lv, np.uint32), np.array(kk, np.uint64), l, table)
    ee2, cg, cgV = R.find_euler(ev, L, Ee, ee)
    return R.partial_contigs(ev, ee2, l)


@pytest.mark.parametrize("l,nreads", [(6, 40), (10, 200), (16, 200), (21, 120)])
def test_assemble2_modular(ec, tmp_path, l, nreads):
    kat = json.load(open(os.path.join(GOLDEN, "kat.json")))
    reads = kat["g200_reads"][:nreads]
    out = tmp_path / "m.fa"
    got = ec.assemble2(l, buffer=reads, outfile=str(out), mode="modular")
    assert got == _oracle_modular("".join(reads).encode(), l)
    lines = out.read_text().splitlines()
    assert lines[1::2] == ["".join(b) for b in got]


@pytest.mark.parametrize("n", [1, 2, 7, 1000, 100000])
def test_partial_contigs_random(ec, n):
    """random injective successor maps (paths + cycles + self loops)"""
    rng = np.random.default_rng(n)
    perm = rng.permutation(n)
    s = np.full(n, n, np.uint32)
    cut = rng.random(n) < 0.05
    for i in range(n):
        if not cut[i]:
            s[perm[i]] = perm[(i + 1) % n]
    nv = max(1, n // 3)
    ev = np.zeros(nv, R.EV)
    ev["vid"] = rng.integers(0, 1 << 40, nv, dtype=np.uint64)
    ee = np.zeros(n, R.EE)
    ee["eid"] = np.arange(n)
    ee["v1"] = rng.integers(0, nv, n)
    ee["s"] = s
    # make the walk consistent: v2(e) = v1(s(e))
    ee["v2"] = np.where(s < n, ee["v1"][np.minimum(s, n - 1)], rng.integers(0, nv, n))
    got = ec.partial_contigs_device(ev, nv, ee, n, 21)
    assert got == R.partial_contigs(ev, ee, 21)


def test_partial_contigs_rejects_non_injective(ec):
    import eulerhip

    ee = np.zeros(3, R.EE)
    ee["s"] = [2, 2, 3]
    with pytest.raises(eulerhip.EulerHipError):
        ec.partial_contigs_device(np.zeros(1, R.EV), 1, ee, 3, 5)
