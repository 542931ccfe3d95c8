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
