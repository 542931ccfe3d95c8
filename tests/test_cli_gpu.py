"""End-to-end command line (pycuda-euler_amd/euler_run.py): read file -> native ingest ->
GPU assembly (fused with one process, RCCL-sharded under torch.distributed.run) -> FASTA /
GFA files, checked against the oracle on the same reads."""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle
from synth import make_reads

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUN = os.path.join(ROOT, "pycuda-euler_amd", "euler_run.py")


def _expected(reads, k, limit):
    _, contigs, links = oracle.assemble(reads, k, limit, want_dict=False)
    fa = "".join(">contig%d\n%s\n" % (i, c) for i, c in enumerate(contigs))
    gfa = ["H  VN:Z:1.0"] + ["S\t%d\t%s\t*" % (i, c) for i, c in enumerate(contigs)]
    for i, (f, b) in enumerate(links):
        gfa += ["L\t%d\t+\t%d\t%s\t%dM" % (i, j, o, k - 1) for j, o in f]
        gfa += ["L\t%d\t-\t%d\t%s\t%dM" % (i, j, o, k - 1) for j, o in b]
    return fa, "\n".join(gfa) + "\n"


@pytest.fixture(scope="module")
def readfile(tmp_path_factory):
    buf, off = make_reads(30000, 4000, 90, 99, err=0.003)
    s = buf.tobytes().decode()
    reads = [s[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]
    p = tmp_path_factory.mktemp("cli") / "reads.fa"
    with open(p, "w") as f:
        for i, r in enumerate(reads):
            f.write(">r%d\n%s\n%s\n" % (i, r[:45], r[45:]))  # two-line records
    return str(p), reads


def _run(cmd, tmp_path):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return r


@pytest.mark.parametrize("k,limit", [(21, 1), (31, 2)])
def test_single_gpu(readfile, tmp_path, k, limit):
    path, reads = readfile
    _run([sys.executable, RUN, "-i", path, "-k", str(k), "--limit", str(limit), "-o", "c.fa", "--gfa", "g.gfa"],
         tmp_path)
    fa, gfa = _expected(reads, k, limit)
    assert (tmp_path / "c.fa").read_text() == fa
    assert (tmp_path / "g.gfa").read_text() == gfa


def test_torchrun_rccl_one_rank(readfile, tmp_path):
    path, reads = readfile
    port = str(29600 + os.getpid() % 300)
    _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
          "127.0.0.1", "--master-port", port, RUN, "-i", path, "-k", "25", "-o", "c.fa"], tmp_path)
    fa, _ = _expected(reads, 25, 1)
    assert (tmp_path / "c.fa").read_text() == fa


def test_torchrun_rccl_one_rank_sharded(readfile, tmp_path):
    """the sharded step itself over a real RCCL group (world 1): TorchComm's all-to-all-v,
    all-gathers and the run gather to rank 0 on device tensors, HipEngine's calls in between"""
    path, reads = readfile
    port = str(29300 + os.getpid() % 300)
    _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
          "127.0.0.1", "--master-port", port, RUN, "-i", path, "-k", "31", "--sharded", "-o", "c.fa", "--gfa",
          "g.gfa"], tmp_path)
    fa, gfa = _expected(reads, 31, 1)
    assert (tmp_path / "c.fa").read_text() == fa
    assert (tmp_path / "g.gfa").read_text() == gfa


@pytest.mark.parametrize("world,k", [(2, 31), (3, 25), (2, 51)])
def test_torchrun_gloo_ranks_share_one_gpu(readfile, tmp_path, world, k):
    """N > 1 processes of the product engine (HipEngine on one MI355X) driven by TorchComm over
    gloo, device tensors staged through host memory: the multi-GPU orchestration with real
    collectives between real engines (the 8-GPU RCCL run is the driver's), bit-exact against the
    oracle (contigs, GFA)"""
    path, reads = readfile
    port = str(29000 + os.getpid() % 300 + 7 * world + k)
    _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
          "--master-addr", "127.0.0.1", "--master-port", port, RUN, "-i", path, "-k", str(k), "--backend", "gloo",
          "--device", "0", "-o", "c.fa", "--gfa", "g.gfa"], tmp_path)
    fa, gfa = _expected(reads, k, 1)
    assert (tmp_path / "c.fa").read_text() == fa
    assert (tmp_path / "g.gfa").read_text() == gfa
