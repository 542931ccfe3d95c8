"""The N > 1 path (pycuda-euler_amd/distributed.py) on CPU: world_size 2 and 3 over gloo, the
real orchestration and collectives (TorchComm: all-to-all-v, all-gather-v, all-reduce), the
compute from tests/fake_engine.py.  Rank 0 (every rank under the replicated finish) must hold
the reference's result for the whole read set (checked against the oracle, itself pinned to the
golden vectors); the partitioned finish leaves the other ranks without a result.  Owner-rule
and exchange checks read every rank's values, whatever its result."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle
from conftest import PKG, ROOT, golden_cases
from synth import make_reads


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, reads, k, limit, q, partitioned=None, gap=None, want_counts=False,
            finish="partitioned"):
    import torch
    import torch.distributed as dist

    for p in (PKG, os.path.join(ROOT, "oracle"), os.path.dirname(os.path.abspath(__file__))):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import distributed
        from fake_engine import FakeEngine

        lo, hi = distributed.shard_range(len(reads), rank, world)
        mine = reads[lo:hi]
        buf = "".join(mine).encode()
        off = np.zeros(len(mine) + 1, np.int64)
        off[1:] = np.cumsum([len(r) for r in mine])
        eng = FakeEngine(k)
        res, P = distributed.sharded_assemble(eng, distributed.TorchComm(),
                                              torch.frombuffer(bytearray(buf or b"\0"), dtype=torch.uint8),
                                              torch.from_numpy(off), len(mine), lo if gap is None else rank * gap,
                                              k, limit,
                                              partitioned=partitioned, finish=finish)
        # the partitioned finish leaves the result on rank 0 only
        q.put((rank, P, res.contigs if res else None, res.links if res else None)
              + ((eng.rule, eng.last_counts) if want_counts else ()))
    finally:
        dist.destroy_process_group()


def _run(reads, k, limit, world, partitioned=None, gap=None, want_counts=False, finish="partitioned",
         all_ranks=False):
    """(rank, P, contigs, links[, rule, counts]) of the ranks holding a result; all_ranks: of
    every rank (with the partitioned finish -- the default, partitioned links -- only rank 0
    holds contigs / links, None elsewhere)"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, reads, k, limit, q, partitioned, gap, want_counts,
                                               finish))
             for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    out = sorted(out, key=lambda o: o[0])
    assert out[0][2] is not None, "rank 0 holds no result"
    part_finish = finish == "partitioned" and partitioned is not False
    if all_ranks:
        return out
    return [o for o in out if not (part_finish and o[0] != 0 and o[2] is None)]


# partitioned: each rank computes the links of its own owner segment (ec_graph_links_part's
# rule restated in fake_engine) and the parts are all-gathered; replicated: one rank-local
# graph phase on the gathered set (ec_assemble_from_solid)
@pytest.mark.parametrize("world,partitioned,finish", [(2, True, "partitioned"), (3, True, "partitioned"),
                                                     (3, True, "replicated"), (2, False, "replicated")])
def test_sharded_matches_reference_g200(world, partitioned, finish):
    """partitioned finish: every rank ranks / emits its own segment, the chains, the contig
    starts and the characters travel (distributed.partitioned_finish); replicated: the successor
    parts are all-gathered and every rank finishes the whole set"""
    (case,) = [c for c in golden_cases("g200.json") if c["k"] == 15]
    out = _run(case["reads"], 15, 1, world, partitioned, finish=finish)
    assert len(out) == (1 if finish == "partitioned" else world)
    for rank, P, contigs, links in out:
        assert contigs == case["contigs"] and links == case["links"]


def test_sharded_matches_oracle_synthetic():
    buf, off = make_reads(3_000, 600, 60, 5151, err=0.003, circular=True)
    reads = [buf[int(off[i]):int(off[i + 1])].tobytes().decode() for i in range(len(off) - 1)]
    _, rc, rl = oracle.assemble(reads, 17, 1, want_dict=False)
    out = _run(reads, 17, 1, 2)
    P_ref = sum(len(r) - 16 for r in reads)
    for rank, P, contigs, links in out:
        assert P == P_ref
        assert contigs == rc and links == rl


def test_sharded_weak_read_bases():
    """bench.py's weak scaling: rank r's reads start at global read id r * gap (its own read
    set, ids with gaps between the ranks); the dict order -- and so the contigs -- is that of
    the ranks' reads concatenated in rank order"""
    sets = [make_reads(2_500, 300, 60, 5252, err=0.003, part=r) for r in range(3)]
    reads = [b[int(o[i]):int(o[i + 1])].tobytes().decode() for b, o in sets for i in range(len(o) - 1)]
    _, rc, rl = oracle.assemble(reads, 19, 1, want_dict=False)
    for rank, P, contigs, links in _run(reads, 19, 1, 3, gap=40_000_000):
        assert P == sum(len(r) - 18 for r in reads)
        assert contigs == rc and links == rl


def test_shard_range_partitions_reads():
    import distributed

    for n in (0, 1, 7, 100):
        for w in (1, 2, 3, 8):
            spans = [distributed.shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))


def test_sharded_skewed_minimizers_take_hash_owners():
    """low-complexity reads: most k-mers share a few minimizers, so minimizer-range owners would
    put most records on one rank; the all-reduced owner counts switch every rank to key-hash
    owners (ec_session_set_owner_rule), and the exchange is balanced"""
    rng = np.random.default_rng(61)
    # 15 A's (mmer_hash 0, the global minimum m-mer) every 17 bases: every 31-mer holds one, so
    # every k-mer of g1 has the same minimizer; g2 is ordinary random sequence
    g1 = "".join("A" * 15 + "".join("ACGT"[x] for x in rng.integers(0, 4, 2)) for _ in range(180))
    g2 = "".join("ACGT"[x] for x in rng.integers(0, 4, 1500))
    reads = []
    for g, n in ((g1, 200), (g2, 80)):
        for _ in range(n):
            p = int(rng.integers(0, len(g) - 70))
            reads.append(g[p:p + 70])
    _, rc, rl = oracle.assemble(reads, 31, 1, want_dict=False)
    world = 3
    out = _run(reads, 31, 1, world, want_counts=True, all_ranks=True)
    assert len(out) == world
    rules = {o[4] for o in out}
    assert rules == {1}, rules  # every rank switched
    totals = [sum(o[5][d] for o in out) for d in range(world)]  # the job's records per owner
    assert max(totals) <= 2.0 * (sum(totals) / world), totals
    assert out[0][2] is not None
    for rank, P, contigs, links, _, _ in out:
        if contigs is not None:
            assert contigs == rc and links == rl


def test_owner_rule_balanced_input_keeps_minimizers():
    import distributed

    assert distributed.owner_rule_for([100, 110, 95], 31) == distributed.OWNER_MINIMIZER
    assert distributed.owner_rule_for([300, 10, 5], 31) == distributed.OWNER_HASH
    assert distributed.owner_rule_for([300, 10, 5], 45) == distributed.OWNER_HASH  # 128-bit minimizers
    assert distributed.owner_rule_for([300, 10, 5], 55) == distributed.OWNER_MINIMIZER  # key hash already
    assert distributed.owner_rule_for([300], 31) == distributed.OWNER_MINIMIZER
