"""Device side of the read-sharded path (ec_count_shard / ec_export_by_owner / ec_merge_owned /
ec_export_dense / ec_assemble_from_solid) on one MI355X: N simulated ranks (N sessions on the
same GPU, collectives by concatenation) and a real 1-rank RCCL group must reproduce the
single-GPU / oracle result exactly."""
import os
import socket

import numpy as np
import pytest

import eulerhip
import oracle
from synth import make_reads

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engines():
    import distributed

    es = [distributed.HipEngine(0) for _ in range(4)]
    yield es
    for e in es:
        e.sess.close()


@pytest.mark.parametrize("world", [1, 2, 3, 4])
@pytest.mark.parametrize("seed,g,n,L,err,k", [(1, 20_000, 6_000, 100, 0.002, 31), (2, 3_000, 2_000, 50, 0.01, 15),
                                              (3, 200_000, 60_000, 100, 0.0, 25),
                                              (4, 30_000, 8_000, 150, 0.002, 51)])
def test_local_sharded_equals_oracle(engines, world, seed, g, n, L, err, k):
    import distributed

    buf, off = make_reads(g, n, L, 7000 + seed, err=err, n_rate=0.001)
    ref = oracle.assemble_packed(buf, off, k, 1)
    res, P = distributed.local_sharded_assemble(engines[:world], buf, off, k, 1)
    assert P == ref["n_positions"]
    assert res.contig_bytes == ref["contig_chars"]
    assert res.links == oracle.unpack_links(ref)


def test_owner_partition_is_disjoint(engines):
    """Every canonical k-mer is merged by exactly one owner: the owners' solid sets add up to the
    single-GPU solid set (engines run on torch's stream, ordered after the torch ops that build
    their inputs -- a session on a private stream raced with them)"""
    import torch

    import distributed

    buf, off = make_reads(300_000, 400_000, 100, 4545)
    s = eulerhip.Session(0)
    s.run_host(buf, off, 31, 1, 0)
    U = s.stats().n_solid
    s.close()
    world = len(engines)
    sends = []
    for r, eng in enumerate(engines):
        lo, hi = distributed.shard_range(len(off) - 1, r, world)
        d_reads = torch.from_numpy(np.ascontiguousarray(buf[int(off[lo]):int(off[hi])])).cuda()
        d_off = torch.from_numpy((off[lo:hi + 1] - off[lo]).astype(np.int64)).cuda()
        eng.count_shard(d_reads, d_off, hi - lo, lo, 31, 0)
        sends.append(eng.export_by_owner(world))
    total = 0
    rb = distributed.rec_bytes(31)
    for dst, eng in enumerate(engines):
        parts = []
        for src in range(world):
            recs, counts = sends[src]
            o = sum(counts[:dst]) * rb
            parts.append(recs[o:o + counts[dst] * rb])
        solid = eng.merge_owned(torch.cat(parts), 31, 1, 0)
        total += solid.numel() // rb
    assert total == U


@pytest.mark.parametrize("world", [1, 3])
def test_local_sharded_general_tables(engines, world):
    """EC_FLAG_GENERAL: HBM-table counting and HBM-table merges instead of the LDS buckets"""
    import distributed

    buf, off = make_reads(20_000, 6_000, 100, 7100, err=0.002, n_rate=0.001)
    ref = oracle.assemble_packed(buf, off, 27, 1)
    res, P = distributed.local_sharded_assemble(engines[:world], buf, off, 27, 1, eulerhip.EC_FLAG_GENERAL)
    assert P == ref["n_positions"]
    assert res.contig_bytes == ref["contig_chars"]
    assert res.links == oracle.unpack_links(ref)
    assert res.stats.count_path == eulerhip.EC_PATH_GENERAL


def test_rccl_world1_sharded(engines):
    import torch
    import torch.distributed as dist

    import distributed

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        buf, off = make_reads(30_000, 9_000, 100, 99, err=0.002)
        ref = oracle.assemble_packed(buf, off, 31, 1)
        sa = distributed.ShardedAssembler(buf, off, 31, 1, 0, 1, 0)
        res = sa.run()
        assert sa.total_positions == ref["n_positions"]
        assert res.contig_bytes == ref["contig_chars"] and res.links == oracle.unpack_links(ref)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("seed,g,n,L,err,k", [(5, 50_000, 20_000, 100, 0.003, 31), (6, 4_000, 3_000, 60, 0.01, 20),
                                              (7, 2_000, 800, 40, 0.0, 32),
                                              # 128-bit keys: HBM lookup table with gathered-order ids
                                              (8, 40_000, 12_000, 150, 0.002, 51), (9, 3_000, 2_000, 90, 0.0, 36)])
def test_partitioned_links_equal_replicated(engines, world, seed, g, n, L, err, k):
    """ec_graph_load / ec_graph_links_part / ec_graph_finish (each simulated rank computes the
    links of its own owner segment, parts concatenated) == ec_assemble_from_solid == oracle"""
    import distributed

    buf, off = make_reads(g, n, L, 7300 + seed, err=err, n_rate=0.001, circular=(seed == 7))
    ref = oracle.assemble_packed(buf, off, k, 1)
    for partitioned in (True, False):
        res, P = distributed.local_sharded_assemble(engines[:world], buf, off, k, 1, partitioned=partitioned)
        assert P == ref["n_positions"]
        assert res.contig_bytes == ref["contig_chars"], partitioned
        assert res.links == oracle.unpack_links(ref), partitioned
        assert res.stats.n_dict == ref["n_dict"], partitioned


@pytest.mark.parametrize("k", [31, 47])
def test_partitioned_links_part_ranges(engines, k):
    """the per-rank successor parts are independent of how the canonical ids are split"""
    import torch

    import distributed

    buf, off = make_reads(30_000, 10_000, 100, 7401, err=0.002)
    eng = engines[0]
    d_reads = torch.from_numpy(buf).cuda()
    d_off = torch.from_numpy(off.astype(np.int64)).cuda()
    eng.count_shard(d_reads, d_off, len(off) - 1, 0, k, 0)
    recs, counts = eng.export_by_owner(1)
    solid = eng.merge_owned(recs, k, 1, 0)
    U = eng.graph_load(solid, k)
    whole = eng.empty(8 * U)
    eng.graph_links_part(0, U, whole)
    cuts = [0, 1, U // 3, U // 2 + 7, U - 1, U]
    parts = []
    for a, b in zip(cuts, cuts[1:]):
        p = eng.empty(8 * (b - a))
        eng.graph_links_part(a, b, p)
        parts.append(p[: 8 * (b - a)])
    assert torch.equal(torch.cat(parts), whole[: 8 * U])
    ref = oracle.assemble_packed(buf, off, k, 1)
    res = eng.graph_finish(whole[: 8 * U], k)
    assert res.contig_bytes == ref["contig_chars"] and res.links == oracle.unpack_links(ref)


@pytest.mark.parametrize("world", [1, 3])
def test_local_sharded_split_tables(engines, monkeypatch, world):
    """shard counts (no solid filter) on the half-table buckets of k_bucket_filt, as taken when
    a rank's distinct keys outgrow one LDS table per bucket (error-rich input)"""
    import distributed

    monkeypatch.setenv("EULERHIP_FORCE_FILTER", "1")
    buf, off = make_reads(40_000, 15_000, 100, 7600 + world, err=0.01, n_rate=0.001)
    ref = oracle.assemble_packed(buf, off, 31, 1)
    res, P = distributed.local_sharded_assemble(engines[:world], buf, off, 31, 1)
    assert P == ref["n_positions"]
    assert res.contig_bytes == ref["contig_chars"] and res.links == oracle.unpack_links(ref)


@pytest.mark.parametrize("k", [31, 25])
def test_weak_shards_large_read_base(engines, k):
    """bench.py's weak-scaled shards: every rank its own read set of one genome, global read ids
    starting at rank * 40 M.  The shard count runs on shard-relative ids, so every rank takes the
    super-k-mer count (its 32-bit positions read * M + window would overflow at a global
    id of 80 M), and the export's global first events give the oracle's order of the
    concatenated reads"""
    import distributed

    world = 3
    sets = [make_reads(60_000, 20_000, 100, 7700, part=r) for r in range(world)]
    buf = np.concatenate([b for b, _ in sets])
    off = np.arange(world * 20_000 + 1, dtype=np.uint64) * np.uint64(100)
    ref = oracle.assemble_packed(buf, off, k, 1)
    res, P = distributed.local_sharded_assemble_shards(
        engines[:world], [(b, o, r * 40_000_000) for r, (b, o) in enumerate(sets)], k, 1)
    assert [e.count_variant for e in engines[:world]] == [3] * world
    assert P == ref["n_positions"]
    assert res.contig_bytes == ref["contig_chars"] and res.links == oracle.unpack_links(ref)
    assert res.stats.n_dict == ref["n_dict"]


@pytest.mark.parametrize("k", [31, 21, 19, 41, 51])
def test_owner_rule_matches_fake_engine(engines, k):
    """ec_export_by_owner puts every record in the segment of shard.h OwnerFn's owner -- the
    minimizer's range for 21 <= k <= 52 (128-bit keys: minimizer_of_w), a key hash otherwise --
    as tests/fake_engine.py restates it for the gloo tests"""
    import torch

    import distributed
    from fake_engine import owner_fn

    buf, off = make_reads(5_000, 1_500, 100, 7801)
    eng = engines[0]
    eng.count_shard(torch.from_numpy(buf).cuda(), torch.from_numpy(off.astype(np.int64)).cuda(), len(off) - 1, 0, k, 0)
    for rule in (0, 1, 0):
        eng.set_owner_rule(rule)
        pre = eng.owner_counts(5)
        recs, counts = eng.export_by_owner(5)
        assert counts == pre
        rb = distributed.rec_bytes(k)
        raw = recs.cpu().numpy()
        o = 0
        for dst, c in enumerate(counts):
            for i in range(o, o + c):
                if k <= 32:
                    key = int(raw[i * rb: i * rb + 8].view(np.uint64)[0])
                    assert owner_fn(key, 5, k, rule) == dst
                elif rule == 0:  # 128-bit key: lo, hi words
                    lo, hi = (int(x) for x in raw[i * rb: i * rb + 16].view(np.uint64))
                    assert owner_fn((hi << 64) | lo, 5, k, rule) == dst
            o += c
        assert o * rb == raw.size
    eng.set_owner_rule(0)


def test_sharded_minimizer_skew_falls_back(engines):
    """~25 K distinct 31-mers share one minimizer (poly-A 15-mers, whose hash is the smallest
    possible): the minimizer-bucketed merge / load overflow that bucket's table and redo the
    call on key-hash buckets; the result still equals the oracle"""
    import distributed

    rng = np.random.Generator(np.random.PCG64(7901))
    parts = []
    for _ in range(1_500):
        parts.append(rng.integers(0, 4, 35, dtype=np.uint8))
        parts.append(np.zeros(15, np.uint8))
    g = np.concatenate(parts)
    L, n = 100, 30_000
    starts = rng.integers(0, len(g) - L + 1, n)
    reads = np.frombuffer(b"ACGT", np.uint8)[g[starts[:, None] + np.arange(L)[None, :]]]
    buf = reads.reshape(-1).copy()
    off = np.arange(n + 1, dtype=np.uint64) * np.uint64(L)
    ref = oracle.assemble_packed(buf, off, 31, 1)
    for world in (1, 2):
        res, P = distributed.local_sharded_assemble(engines[:world], buf, off, 31, 1)
        assert P == ref["n_positions"]
        assert res.contig_bytes == ref["contig_chars"] and res.links == oracle.unpack_links(ref)


def test_sharded_owner_rule_switches_on_skew(engines):
    """every 31-mer of this genome holds 15 A's, so they all share one minimizer and minimizer-range
    owners would send every record to one rank; the summed owner counts switch all ranks to key-hash
    owners, whose parts are balanced, and the result still equals the oracle"""
    import distributed

    rng = np.random.Generator(np.random.PCG64(7902))
    parts = []
    for _ in range(3_000):
        parts.append(np.zeros(15, np.uint8))
        parts.append(rng.integers(0, 4, 2, dtype=np.uint8))
    g = np.concatenate(parts)
    L, n = 100, 20_000
    starts = rng.integers(0, len(g) - L + 1, n)
    reads = np.frombuffer(b"ACGT", np.uint8)[g[starts[:, None] + np.arange(L)[None, :]]]
    buf = reads.reshape(-1).copy()
    off = np.arange(n + 1, dtype=np.uint64) * np.uint64(L)
    ref = oracle.assemble_packed(buf, off, 31, 1)
    world = 3
    res, P = distributed.local_sharded_assemble(engines[:world], buf, off, 31, 1)
    assert distributed.local_sharded_assemble_shards.last_rule == distributed.OWNER_HASH
    totals = [sum(c[d] for c in distributed.local_sharded_assemble_shards.last_counts) for d in range(world)]
    assert max(totals) <= 1.25 * sum(totals) / world, totals
    assert P == ref["n_positions"]
    assert res.contig_bytes == ref["contig_chars"] and res.links == oracle.unpack_links(ref)
    for e in engines:
        e.set_owner_rule(distributed.OWNER_MINIMIZER)


@pytest.mark.parametrize("partitioned", [True, False])
def test_local_sharded_8_ranks_k51_vs_oracle(partitioned):
    """BASELINE config 5's path (128-bit keys, "8xMI355X partitioned graph") at 8 simulated ranks
    on a k = 51 slice of 1.0 * 10^7 positions: the owners' merges, the gathered set's HBM lookup
    table and the partitioned links equal the oracle (contigs, links, dict size)"""
    import distributed

    es = [distributed.HipEngine(0) for _ in range(8)]
    try:
        buf, off = make_reads(200_000, 100_000, 150, 20261015 + 5, err=0.001)
        ref = oracle.assemble_packed(buf, off, 51, 1)
        assert ref["n_positions"] >= 10 ** 7 - 10 ** 5
        res, P = distributed.local_sharded_assemble(es, buf, off, 51, 1, partitioned=partitioned)
        assert P == ref["n_positions"]
        assert res.stats.n_dict == ref["n_dict"]
        assert res.contig_bytes == ref["contig_chars"]
        assert res.links == oracle.unpack_links(ref)
    finally:
        for e in es:
            e.sess.close()


@pytest.mark.parametrize("world", [1, 2, 5])
@pytest.mark.parametrize("seed,g,n,L,err,k,circ", [(11, 20_000, 6_000, 100, 0.002, 31, False),
                                                   (12, 3_000, 1_500, 60, 0.0, 25, True),
                                                   (13, 30_000, 8_000, 150, 0.002, 51, False),
                                                   (14, 2_000, 800, 40, 0.01, 16, False)])
def test_partitioned_finish_equals_replicated(world, seed, g, n, L, err, k, circ):
    """distributed.partitioned_finish (each rank ranks its own segment's chains, the chains and
    contig starts all-gathered, every rank emits its own nodes, rank 0 collects) against the
    replicated finish and the oracle: cycles (circular genomes) across the segments, k <= 32
    and k > 32, error-rich reads"""
    import distributed

    es = [distributed.HipEngine(0) for _ in range(world)]
    try:
        buf, off = make_reads(g, n, L, 7900 + seed, err=err, n_rate=0.001, circular=circ)
        ref = oracle.assemble_packed(buf, off, k, 1)
        for finish in ("partitioned", "replicated"):
            res, P = distributed.local_sharded_assemble(es, buf, off, k, 1, finish=finish)
            assert P == ref["n_positions"], finish
            assert res.contig_bytes == ref["contig_chars"], finish
            assert np.array_equal(res.contig_offsets, ref["contig_offsets"]), finish
            assert res.links == oracle.unpack_links(ref), finish
            assert res.stats.n_dict == ref["n_dict"], finish
    finally:
        for e in es:
            e.sess.close()


@pytest.mark.parametrize("compact", [True, False, [True, False, True]])
@pytest.mark.parametrize("k", [31, 51])
def test_exchange_record_formats(engines, compact, k):
    """the all-to-all's records: compact (shard-relative events in 32 bits, 20 / 28 B), full
    (global events, 32 / 48 B) and both at once (ec_merge_owned_from decodes per source), at
    read bases 0 / 40 M / 80 M, equal to the oracle on the concatenated reads"""
    import distributed

    world = 3
    sets = [make_reads(60_000, 20_000, 150 if k > 32 else 100, 8100 + k, part=r, err=0.002) for r in range(world)]
    buf = np.concatenate([b for b, _ in sets])
    L = 150 if k > 32 else 100
    off = np.arange(world * 20_000 + 1, dtype=np.uint64) * np.uint64(L)
    ref = oracle.assemble_packed(buf, off, k, 1)
    for finish in ("partitioned", "replicated"):
        res, P = distributed.local_sharded_assemble_shards(
            engines[:world], [(b, o, r * 40_000_000) for r, (b, o) in enumerate(sets)], k, 1, finish=finish,
            compact=compact)
        want = [compact] * world if isinstance(compact, bool) else compact
        assert [b >= 0 for b in distributed.local_sharded_assemble_shards.last_lf_bits] == want
        assert P == ref["n_positions"]
        assert res.contig_bytes == ref["contig_chars"] and res.links == oracle.unpack_links(ref), finish
        assert res.stats.n_dict == ref["n_dict"]


@pytest.mark.parametrize("knobs", [{"EULERHIP_JUNCTION_BT": "2", "EULERHIP_JUNCTION_SB": "3"},
                                   # (a claim cap of 96: the 2^9 sub-buckets of ~39 junctions the retries end
                                   # at stay under it; at 64 the transient claims of racing lanes could pass it)
                                   {"EULERHIP_JUNCTION_BT": "1", "EULERHIP_JUNCTION_CLAIM": "96"},
                                   {"EULERHIP_JUNCTION_CLAIM": "24"},
                                   {"EULERHIP_JUNCTION_RADIX": "1"},
                                   {"EULERHIP_JUNCTION_RADIX": "1", "EULERHIP_JUNCTION_CLAIM": "64"}])
@pytest.mark.parametrize("k", [31, 51])
def test_junction_join_split_and_retries(engines, monkeypatch, knobs, k):
    """the junction join past 2^14 buckets' worth of junctions (a rank of > ~4.7 * 10^7 keys):
    every bucket split into sub-buckets joined one after the other in one table, forced here on a
    small set by capping the bucket bits; and a table that overflows (claim cap forced small)
    retried with 4096-slot tables, finer buckets, then more sub-buckets -- the same contigs, links
    and dict size as the oracle (a rank used to fail with EC_ERR_CAPACITY at 2^14 buckets); and the
    buckets ordered by the radix sort (past 2^14 buckets, EULERHIP_JUNCTION_RADIX forces it)"""
    import distributed

    for n, v in knobs.items():
        monkeypatch.setenv(n, v)
    buf, off = make_reads(40_000, 12_000, 150 if k > 32 else 100, 9300 + k, err=0.002)
    ref = oracle.assemble_packed(buf, off, k, 1)
    world = 2
    res, P = distributed.local_sharded_assemble(engines[:world], buf, off, k, 1, finish="partitioned")
    assert P == ref["n_positions"]
    assert res.stats.n_dict == ref["n_dict"]
    assert res.contig_bytes == ref["contig_chars"]
    assert res.links == oracle.unpack_links(ref)


@pytest.mark.parametrize("k,L,g,n,chunk,fold,err,base", [(51, 150, 2_000_000, 1_000_000, 150_000, 3, 0.0, 0),
                                                         (31, 100, 300_000, 200_000, 37_000, 2, 0.003, 5_000_000),
                                                         (25, 100, 50_000, 30_000, 7_000, 10, 0.01, 0),
                                                         (45, 120, 60_000, 20_000, 20_000, 4, 0.002, 0)])
def test_streaming_count_vs_oracle(k, L, g, n, chunk, fold, err, base):
    """out-of-core count (distributed.streaming_assemble): the reads counted chunk by chunk (the
    count's buffers released after each chunk's export), the chunks' records folded into a
    running merged set, the final merge filtered, then the junction graph and partitioned
    finish of one rank -- forced small chunks, bit-exact against the oracle (contigs, offsets,
    GFA links, dict size); BASELINE config 5's read shape at 10^8 positions among them"""
    import distributed

    buf, off = make_reads(g, n, L, 9500 + k, err=err)
    ref = oracle.assemble_packed(buf, off, k, 1)
    eng = distributed.HipEngine(0)
    try:
        stats = {}
        res, P = distributed.streaming_assemble(eng, buf, off, k, 1, chunk_reads=chunk, fold=fold, read_base=base,
                                                stats=stats)
    finally:
        eng.sess.close()
    assert stats["chunks"] == (n + chunk - 1) // chunk
    assert stats["folds"] == (stats["chunks"] - 1) // fold
    assert P == ref["n_positions"]
    assert res.stats.n_dict == ref["n_dict"]
    assert res.contig_bytes == ref["contig_chars"]
    assert np.array_equal(res.contig_offsets, ref["contig_offsets"])
    assert res.links == oracle.unpack_links(ref)


def test_chains_drop_held_place_records():
    """ec_graph_chains_part keeps its tile records in the junction-record buffer ec_graph_place
    filled (round 6: no 64-B-a-key buffer of its own), so place records still held then are
    refused by ec_graph_place_copy (EC_ERR_STATE) instead of copied overwritten; copied first,
    they are taken as before"""
    import ctypes

    import distributed

    buf, off = make_reads(20_000, 6_000, 100, 7105, err=0.002)
    k = 31
    ref = oracle.assemble_packed(buf, off, k, 1)
    e = distributed.HipEngine(0)
    try:
        st = {}
        res, _ = distributed.streaming_assemble(e, buf, off, k, 1, chunk_reads=2_500, fold=2, stats=st)
        assert res.contig_bytes == ref["contig_chars"]
        ur = int(st["solid"])
        L, h = e.L, e._h()
        counts = (ctypes.c_uint64 * 1)()
        npal = ctypes.c_uint64(0)
        out = e.empty(4 * ur * distributed.junction_bytes(k))
        # in order: counted, then copied
        eulerhip.check(L.ec_graph_place(h, 0, ur, 1, None, counts, ctypes.byref(npal)))
        assert 0 < counts[0] <= 4 * ur
        assert L.ec_graph_place_copy(h, ctypes.c_void_p(out.data_ptr())) == 0
        # counted, then the chains step reuses the buffer: the held records are gone
        eulerhip.check(L.ec_graph_place(h, 0, ur, 1, None, counts, ctypes.byref(npal)))
        n = ctypes.c_uint64(0)
        eulerhip.check(L.ec_graph_chains_part(h, 0, ur, None, None, ctypes.byref(n)))
        assert n.value > 0
        assert L.ec_graph_place_copy(h, ctypes.c_void_p(out.data_ptr())) == eulerhip.EC_ERR_STATE
    finally:
        e.sess.close()
