"""BASELINE.json configurations at full size on the HIP path (libeulerhip.so).

* config 2 (4.6 Mbp, 1 M x 100 bp, k = 31) and config 3 (12 Mbp, 5 M x 100 bp, k = 31):
  contigs, their offsets and the GFA link table bit-exact against the C oracle
  (oracle/refasm.c, the restatement of referenceAssembler.py:25-111 pinned in test_oracle.py);
* the headline read set (4.6 Mbp, 10 M x 100 bp, k = 31; config 4's data): size-independent
  properties -- every k-mer of the error-free genome is solid (n_solid = G - k + 1) and the one
  contig is the genome itself or its reverse complement (all_contigs:79-111 walks the unique
  path of a repeat-free genome end to end);
* config 5's read shape (150 bp reads, k = 51, 128-bit keys, 75-fold coverage) at 10^8
  positions: bit-exact against the oracle.

Inputs are synth.make_reads with the bench's seeds (20261015 + config#).
"""
import numpy as np
import pytest

import eulerhip
import oracle
from synth import make_genome, make_reads, read_starts

pytestmark = pytest.mark.gpu

COMP = bytes.maketrans(b"ACGT", b"TGCA")


def _check_vs_oracle(sess, buf, off, k, limit=1):
    ref = oracle.assemble_packed(buf, off, k, limit)
    sess.run_host(buf, off, k, limit)
    res = sess.fetch(k)
    assert res.stats.n_positions == ref["n_positions"]
    assert res.stats.n_dict == ref["n_dict"]
    assert res.stats.n_contigs == len(ref["contig_offsets"]) - 1
    assert res.contig_bytes == ref["contig_chars"]
    assert np.array_equal(res.contig_offsets, ref["contig_offsets"])
    assert np.array_equal(res.link_offsets, ref["link_offsets"])
    assert np.array_equal(res.link_codes, ref["links"])
    return res


def test_config2_ecoli_1m_vs_oracle(gpu_session):
    """BASELINE configs[1]: E. coli size, 1 M x 100 bp, k = 31"""
    buf, off = make_reads(4_600_000, 1_000_000, 100, 20261015 + 2)
    res = _check_vs_oracle(gpu_session, buf, off, 31)
    assert res.stats.n_positions == 70_000_000


def test_config3_yeast_5m_vs_oracle(gpu_session):
    """BASELINE configs[2]: S. cerevisiae size, 5 M x 100 bp, k = 31"""
    buf, off = make_reads(12_000_000, 5_000_000, 100, 20261015 + 3)
    res = _check_vs_oracle(gpu_session, buf, off, 31)
    assert res.stats.n_positions == 350_000_000


def test_headline_10m_contig_is_the_genome(gpu_session):
    """the metric's workload: 10 M x 100 bp of a 4.6 Mbp genome; the single contig is the
    genome (or its reverse complement) and every genome k-mer is solid"""
    G, k, seed = 4_600_000, 31, 20261015 + 4
    buf, off = make_reads(G, 10_000_000, 100, seed)
    genome = make_genome(G, seed)
    gpu_session.run_host(buf, off, k, 1)
    res = gpu_session.fetch(k)
    st = res.stats
    assert st.n_positions == 700_000_000
    assert st.n_solid == G - k + 1
    assert st.n_dict == 2 * (G - k + 1)
    assert st.n_contigs == 1
    c = res.contig_bytes
    assert c == genome or c == genome.translate(COMP)[::-1]
    # a linear contig has no GFA links (all_contigs:90-109: its ends extend nowhere)
    assert st.n_links == 0


def test_config5_shape_k51_vs_oracle(gpu_session):
    """BASELINE configs[4]'s read shape: 150 bp reads, k = 51 (128-bit keys), 75-fold coverage
    as 100 M reads of 200 Mbp give; 10^8 positions (1 M reads of a 2 Mbp genome)"""
    buf, off = make_reads(2_000_000, 1_000_000, 150, 20261015 + 5)
    res = _check_vs_oracle(gpu_session, buf, off, 51)
    assert res.stats.n_positions == 100_000_000


def _solid_runs(G, starts, L, k, limit=1):
    """For error-free reads of a repeat-free genome, the count of a canonical k-mer is the number
    of read windows covering its genome position (a read and its reverse complement insert the
    same canonical k-mers, build:25-42), so the solid k-mers are the positions covered by more
    than `limit` windows; all_contigs:79-111 walks each maximal run of consecutive solid positions
    as one contig (no branches: every (k - 1)-mer is unique).  Returns (n_solid, run starts,
    run ends) with runs [a, b) of k-mer positions."""
    W = L - k + 1
    C = np.cumsum(np.bincount(starts, minlength=G - k + 1), dtype=np.int64)
    cov = C.copy()
    cov[W:] -= C[:-W]
    solid = cov > limit
    e = np.diff(np.concatenate([[0], solid.view(np.int8), [0]]).astype(np.int8))
    return int(solid.sum()), np.flatnonzero(e == 1), np.flatnonzero(e == -1)


def _canon(s):
    t = s.translate(COMP)[::-1]
    return s if s <= t else t


def test_config5_rank_shape_solid_runs(gpu_session):
    """BASELINE configs[4] at its per-rank shape (8 ranks: 12.5 M x 150 bp of the 200 Mbp genome,
    k = 51, 128-bit keys, third partition level, 1.9 * 10^9 positions): n_solid equals the
    solid positions computed from the read starts, and the contigs, each in canonical
    orientation, are exactly the genome substrings of the maximal solid runs (a size-independent
    property; the oracle is bit-exact on the same path below at 10^9 positions)"""
    import torch

    G, n, L, k, seed = 200_000_000, 12_500_000, 150, 51, 20261015 + 5
    buf, off = make_reads(G, n, L, seed)
    gpu_session.trim()
    torch.cuda.empty_cache()
    s = eulerhip.Session(0)
    try:
        free0, total = torch.cuda.mem_get_info()
        s.run_host(buf, off, k, 1)
        res = s.fetch(k)
        free1, _ = torch.cuda.mem_get_info()
        print("config-5 rank shape: session HBM %.1f GB of %.1f GB" % ((free0 - free1) / 1e9, total / 1e9))
    finally:
        s.close()
    del buf, off
    st = res.stats
    assert st.n_positions == n * (L - k + 1)
    n_solid, a, b = _solid_runs(G, read_starts(G, n, L, seed), L, k)
    assert st.n_solid == n_solid and st.n_dict == 2 * n_solid
    assert st.n_contigs == len(a)
    assert st.n_links == 0  # a run's ends extend nowhere
    genome = make_genome(G, seed)
    ch, co = res.contig_bytes, res.contig_offsets
    got = sorted(_canon(ch[int(co[i]):int(co[i + 1])]) for i in range(len(co) - 1))
    want = sorted(_canon(genome[int(x):int(y) - 1 + k]) for x, y in zip(a, b))
    assert got == want


def test_config5_rank_sharded_junction_flow(gpu_session):
    """One rank of BASELINE configs[4] through the whole sharded step of the multi-GPU design
    (rank 3 of 8: its 12.5 M x 150 bp reads of the 200 Mbp genome at global read ids 37.5 M..,
    k = 51): shard count, compact export, owner merge, placement at global ids, the junction join,
    the partitioned finish -- distributed.local_sharded_assemble_shards at world 1, so this rank
    owns every key (its merge and graph hold the whole genome's 2 * 10^8 keys, 8x the 8-rank
    share: an upper bound of a real rank's memory).  Checks the size-independent properties of
    test_config5_rank_shape_solid_runs and reports the peak HBM of the session buffers and of
    torch's (reads, exchange records) -- src/cli_spark_gpu.py:37"""
    import torch

    import distributed

    G, n, L, k, seed = 200_000_000, 12_500_000, 150, 51, 20261015 + 5
    buf, off = make_reads(G, n, L, seed)
    gpu_session.trim()  # (the suite's shared session and torch's cache give their memory back first)
    torch.cuda.empty_cache()
    eng = distributed.HipEngine(0)
    try:
        torch.cuda.reset_peak_memory_stats()
        eulerhip.mem_stats(reset=True)
        res, P = distributed.local_sharded_assemble_shards([eng], [(buf, off, 37_500_000)], k, 1, finish="partitioned")
        held, peak = eulerhip.mem_stats()
        print("config-5 rank, sharded step: session buffers peak %.1f GB, torch peak %.1f GB, device %.1f GB"
              % (peak / 1e9, torch.cuda.max_memory_allocated() / 1e9, torch.cuda.mem_get_info()[1] / 1e9))
    finally:
        eng.sess.close()
    del buf, off
    st = res.stats
    assert P == n * (L - k + 1)
    n_solid, a, b = _solid_runs(G, read_starts(G, n, L, seed), L, k)
    assert st.n_dict == 2 * n_solid
    assert st.n_contigs == len(a)
    assert st.n_links == 0
    genome = make_genome(G, seed)
    ch, co = res.contig_bytes, res.contig_offsets
    got = sorted(_canon(ch[int(co[i]):int(co[i + 1])]) for i in range(len(co) - 1))
    want = sorted(_canon(genome[int(x):int(y) - 1 + k]) for x, y in zip(a, b))
    assert got == want


def test_genome20m_k51_third_level_vs_oracle(gpu_session, monkeypatch):
    """config 5's read shape at a tenth of its genome (20 Mbp, 10 M x 150 bp, k = 51: 10^9
    positions, 2 * 10^7 solid 51-mers) through the wide path's third partition level (forced:
    2^2 sub-buckets per fine bucket), bit-exact against the oracle (N-core count)"""
    import os

    monkeypatch.setenv("EULERHIP_WIDE_L3", "2")
    buf, off = make_reads(20_000_000, 10_000_000, 150, 20261015 + 5)
    th = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    ref = oracle.assemble_packed(buf, off, 51, 1, threads=th)
    gpu_session.run_host(buf, off, 51, 1)
    res = gpu_session.fetch(51)
    assert res.stats.n_buckets == (1 << 14) << 2
    assert res.stats.n_positions == ref["n_positions"] == 10 ** 9
    assert res.stats.n_dict == ref["n_dict"]
    assert res.contig_bytes == ref["contig_chars"]
    assert np.array_equal(res.contig_offsets, ref["contig_offsets"])
    assert np.array_equal(res.link_offsets, ref["link_offsets"])
    assert np.array_equal(res.link_codes, ref["links"])


def test_ecoli10m_err_vs_oracle(gpu_session):
    """the headline read set with 0.5 % substitution errors (SURVEY §8d's error variant: 1.6·10^8
    distinct k-mers, mostly singletons) at full size, bit-exact against the oracle (N-core
    count): the super-k-mer count behind the seen-twice filter (k_skbucket_filt)"""
    import os

    buf, off = make_reads(4_600_000, 10_000_000, 100, 20261015 + 4, err=0.005)
    th = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    ref = oracle.assemble_packed(buf, off, 31, 1, threads=th)
    gpu_session.run_host(buf, off, 31, 1)
    res = gpu_session.fetch(31)
    assert res.stats.count_variant == 3
    assert res.stats.n_positions == ref["n_positions"] == 700_000_000
    assert res.stats.n_dict == ref["n_dict"]
    assert res.contig_bytes == ref["contig_chars"]
    assert np.array_equal(res.contig_offsets, ref["contig_offsets"])
    assert np.array_equal(res.link_offsets, ref["link_offsets"])
    assert np.array_equal(res.link_codes, ref["links"])


# ---- BASELINE config 4: the headline read set read-sharded over 8 ranks ----------------------
@pytest.fixture(scope="module")
def engines8():
    import distributed

    es = [distributed.HipEngine(0) for _ in range(8)]
    yield es
    for e in es:
        e.sess.close()


@pytest.mark.parametrize("finish", ["partitioned", "replicated"])
def test_config4_sharded_8_ranks_contig_is_the_genome(engines8, finish):
    """BASELINE configs[3]: E. coli 10 M x 100 bp, k = 31, read-sharded over 8 ranks (8 simulated
    HipEngines on one GPU: every rank's count / export / owner merge / load / partitioned links
    and finish, the collectives by concatenation -- distributed.local_sharded_assemble, the same
    engine calls sharded_assemble makes over RCCL).  Size-independent properties of the
    error-free repeat-free genome: every genome k-mer is solid, the one contig is the genome or
    its reverse complement, no GFA links (src/cli_spark_gpu.py:37, src/ref_spark.py:76-88)"""
    import distributed

    G, k, seed = 4_600_000, 31, 20261015 + 4
    buf, off = make_reads(G, 10_000_000, 100, seed)
    res, P = distributed.local_sharded_assemble(engines8, buf, off, k, 1, finish=finish)
    del buf, off
    assert distributed.local_sharded_assemble_shards.last_rule == distributed.OWNER_MINIMIZER
    st = res.stats
    assert P == 700_000_000
    assert st.n_solid == G - k + 1
    assert st.n_dict == 2 * (G - k + 1)
    assert st.n_contigs == 1
    genome = make_genome(G, seed)
    c = res.contig_bytes
    assert c == genome or c == genome.translate(COMP)[::-1]
    assert st.n_links == 0


@pytest.mark.parametrize("finish", ["partitioned", "replicated"])
def test_config2_sharded_8_ranks_vs_oracle(engines8, finish):
    """BASELINE configs[1] (4.6 Mbp, 1 M x 100 bp, k = 31) read-sharded over 8 simulated ranks,
    bit-exact against the oracle: contigs, offsets, GFA links and dict size"""
    import distributed

    buf, off = make_reads(4_600_000, 1_000_000, 100, 20261015 + 2)
    ref = oracle.assemble_packed(buf, off, 31, 1)
    res, P = distributed.local_sharded_assemble(engines8, buf, off, 31, 1, finish=finish)
    assert P == ref["n_positions"] == 70_000_000
    assert res.stats.n_dict == ref["n_dict"]
    assert res.contig_bytes == ref["contig_chars"]
    assert np.array_equal(res.contig_offsets, ref["contig_offsets"])
    assert np.array_equal(res.link_offsets, ref["link_offsets"])
    assert np.array_equal(res.link_codes, ref["links"])


def test_config4_err_sharded_8_ranks_vs_oracle(engines8):
    """the headline read set with 0.5 % substitutions (1.3 * 10^7 solid k-mers in ~10^6 contigs,
    so GFA links everywhere) read-sharded over 8 simulated ranks, bit-exact vs the oracle"""
    import os

    import distributed

    buf, off = make_reads(4_600_000, 10_000_000, 100, 20261015 + 4, err=0.005)
    th = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    ref = oracle.assemble_packed(buf, off, 31, 1, threads=th)
    res, P = distributed.local_sharded_assemble(engines8, buf, off, 31, 1)
    assert P == ref["n_positions"] == 700_000_000
    assert res.stats.n_dict == ref["n_dict"]
    assert res.contig_bytes == ref["contig_chars"]
    assert np.array_equal(res.contig_offsets, ref["contig_offsets"])
    assert np.array_equal(res.link_offsets, ref["link_offsets"])
    assert np.array_equal(res.link_codes, ref["links"])
