"""The CPU oracle (oracle/refasm.c) and the parallel design model (tests/model_parallel.py)
pinned against every golden vector generated from the real reference
(tests/golden/make_golden.py -> referenceAssembler.build/all_contigs)."""
import pytest

import oracle
from conftest import golden_cases
from model_parallel import model_assemble

CASES = golden_cases("g200.json", "synthetic.json", "fuzz.json")
ALL = golden_cases("g200.json", "synthetic.json", "fuzz.json", alphabet="all")


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_matches_reference(case):
    d, r, g = oracle.assemble(case["reads"], case["k"], case["limit"])
    assert d == case["d"]
    assert r == case["contigs"]
    assert g == case["links"]


@pytest.mark.parametrize("case", CASES[::3], ids=[c["name"] for c in CASES[::3]])
def test_parallel_model_matches_reference(case):
    d, r, g = model_assemble(case["reads"], case["k"], case["limit"])
    assert d == case["d"]
    assert r == case["contigs"]
    assert g == case["links"]


def test_oracle_extended_alphabet_matches_reference():
    """lowercase and IUPAC bytes are opaque symbols, their own complement (twin:7-10): the
    oracle takes its string-keyed restatement (refasm_str.c) for such reads"""
    cases = golden_cases("synthetic.json", alphabet="extended")
    assert cases
    for case in cases:
        for th in (None, 4):
            d, r, g = oracle.assemble(case["reads"], case["k"], case["limit"], threads=th)
            assert d == case["d"] and r == case["contigs"] and g == case["links"], case["name"]


@pytest.mark.parametrize("case", ALL, ids=[c["name"] for c in ALL])
def test_string_oracle_matches_reference(case):
    """the string-keyed restatement on every golden case (forced: string=True)"""
    d, r, g = oracle.assemble(case["reads"], case["k"], case["limit"], string=True)
    assert d == case["d"]
    assert r == case["contigs"]
    assert g == case["links"]


def test_g200_config1_is_empty_at_k21():
    (case,) = [c for c in golden_cases("g200.json") if c["k"] == 21]
    d, r, g = oracle.assemble(case["reads"], 21)
    assert d == [] and r == [] and g == []


@pytest.mark.parametrize("threads", [1, 3, 8])
@pytest.mark.parametrize("case", CASES[::5], ids=[c["name"] for c in CASES[::5]])
def test_oracle_ncore_matches_reference(case, threads):
    """the N-core map -> reduceByKey variant (bench.py's N-core CPU baseline) gives build()'s
    dict order and all_contigs' results"""
    d, r, g = oracle.assemble(case["reads"], case["k"], case["limit"], threads=threads)
    assert d == case["d"]
    assert r == case["contigs"]
    assert g == case["links"]


@pytest.mark.parametrize("k", [21, 31, 51])
def test_oracle_ncore_synthetic(k):
    import numpy as np
    from synth import make_reads

    buf, off = make_reads(60_000, 30_000, 100, 77 + k, err=0.003, n_rate=0.001)
    a = oracle.assemble_packed(buf, off, k, 1, True)
    b = oracle.assemble_packed(buf, off, k, 1, True, threads=6)
    assert a["n_positions"] == b["n_positions"] and a["d"] == b["d"]
    assert a["contig_chars"] == b["contig_chars"]
    assert np.array_equal(a["links"], b["links"]) and np.array_equal(a["link_offsets"], b["link_offsets"])


def test_solid_run_property_matches_oracle():
    """The size-independent property test_configs_gpu.py checks config 5's per-rank shape with
    (solid k-mers = positions covered by > limit read windows; contigs = maximal solid runs as
    genome substrings) agrees with the oracle on a small error-free set of the same shape"""
    import numpy as np

    from synth import make_genome, make_reads, read_starts
    from test_configs_gpu import _canon, _solid_runs

    G, n, L, k, seed = 300_000, 20_000, 150, 51, 99
    buf, off = make_reads(G, n, L, seed)
    ref = oracle.assemble_packed(buf, off, k, 1)
    n_solid, a, b = _solid_runs(G, read_starts(G, n, L, seed), L, k)
    assert ref["n_dict"] == 2 * n_solid
    genome = make_genome(G, seed)
    ch, co = ref["contig_chars"], ref["contig_offsets"]
    got = sorted(_canon(ch[int(co[i]):int(co[i + 1])]) for i in range(len(co) - 1))
    assert got == sorted(_canon(genome[int(x):int(y) - 1 + k]) for x, y in zip(a, b))
    assert len(got) > 10
