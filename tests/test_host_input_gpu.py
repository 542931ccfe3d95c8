"""The host-input entry points on the HIP path: ec_assemble_host (ASCII, chunked copies
overlapped with the partition) and ec_assemble_packed_host (2 bits per base + exception bytes),
against the oracle -- the reference's GPU path starts from host reads (src/eulercuda.py:484-497).
EULERHIP_HOST_CHUNKS forces many chunks on small inputs so the per-chunk partition launches,
offsets slices and exception ranges are all exercised."""
import numpy as np
import pytest

import eulerhip
import oracle
from synth import make_reads

pytestmark = pytest.mark.gpu


def _ref(buf, off, k, limit=1):
    out = oracle.assemble_packed(buf, off, k, limit)
    return out, oracle.unpack_links(out)


def _same(res, ref, rl):
    assert res.stats.n_positions == ref["n_positions"] and res.stats.n_dict == ref["n_dict"]
    assert res.contig_bytes == ref["contig_chars"]
    assert np.array_equal(res.contig_offsets, ref["contig_offsets"])
    assert res.links == rl


CASES = [  # genome, reads, len, seed, err, n_rate, k
    (40_000, 20_000, 100, 1, 0.0, 0.0, 31),     # super-k-mer path, chunked partition launches
    (50_000, 20_000, 100, 2, 0.004, 0.0, 31),   # error-rich: window records after the pipeline drains
    (30_000, 10_000, 90, 3, 0.002, 0.003, 25),  # N bytes: exceptions, exact path
    (20_000, 6_000, 150, 4, 0.002, 0.0, 51),    # 128-bit keys
    (10_000, 8_000, 60, 5, 0.01, 0.0, 17),      # k < 21: window records
]


@pytest.mark.parametrize("chunks", ["1", "7", "64"])
@pytest.mark.parametrize("g,n,L,seed,err,nr,k", CASES)
def test_host_paths_vs_oracle(gpu_session, monkeypatch, g, n, L, seed, err, nr, k, chunks):
    monkeypatch.setenv("EULERHIP_HOST_CHUNKS", chunks)
    buf, off = make_reads(g, n, L, 7000 + seed, err=err, n_rate=nr)
    ref, rl = _ref(buf, off, k)
    gpu_session.run_host(buf, off, k, 1)
    _same(gpu_session.fetch(k), ref, rl)
    pr = eulerhip.pack_2bit(buf, off)
    assert pr.read_len == L and pr.offsets is None
    assert len(pr.exc_pos) == int((buf == ord("N")).sum())
    gpu_session.run_packed_host(pr, k, 1)
    _same(gpu_session.fetch(k), ref, rl)


@pytest.mark.parametrize("chunks", ["1", "5"])
def test_packed_ragged_reads_vs_oracle(gpu_session, monkeypatch, chunks):
    """reads of many lengths: offsets travel with the codes, chunk by chunk"""
    monkeypatch.setenv("EULERHIP_HOST_CHUNKS", chunks)
    rng = np.random.default_rng(9)
    g = rng.integers(0, 4, 30_000)
    reads = []
    for _ in range(6_000):
        L = int(rng.choice([0, 3, 30, 31, 32, 77, 100, 151, 400]))
        p = int(rng.integers(0, len(g) - L))
        reads.append("".join("ACGT"[x] for x in g[p:p + L]))
    buf, off = eulerhip.pack_reads(reads)
    for k in (21, 31, 45):
        ref, rl = _ref(buf, off, k)
        pr = eulerhip.pack_2bit(buf, off)
        assert pr.read_len == 0 and pr.offsets is not None
        gpu_session.run_packed_host(pr, k, 1)
        _same(gpu_session.fetch(k), ref, rl)
        gpu_session.run_host(buf, off, k, 1)
        _same(gpu_session.fetch(k), ref, rl)


def test_packed_extended_alphabet(gpu_session, monkeypatch):
    """a byte outside {A,C,G,T,N} travels as an exception and, as in ASCII input, is an opaque
    symbol (extended.h): both host-input paths equal the oracle's string-keyed restatement"""
    monkeypatch.setenv("EULERHIP_HOST_CHUNKS", "3")
    buf, off = make_reads(20_000, 4_000, 100, 7100)
    buf = buf.copy()
    buf[250_123] = ord("a")
    buf[[5, 300_001, 399_999]] = [ord("R"), ord("n"), ord("y")]
    pr = eulerhip.pack_2bit(buf, off)
    assert list(pr.exc_pos) == [5, 250_123, 300_001, 399_999]
    ref, rl = _ref(buf, off, 31)
    gpu_session.run_packed_host(pr, 31, 1)
    _same(gpu_session.fetch(31), ref, rl)
    gpu_session.run_host(buf, off, 31, 1)
    _same(gpu_session.fetch(31), ref, rl)
    # the session still works afterwards on ordinary input (the pipeline was drained)
    buf2, off2 = make_reads(20_000, 4_000, 100, 7101)
    ref, rl = _ref(buf2, off2, 31)
    gpu_session.run_packed_host(eulerhip.pack_2bit(buf2, off2), 31, 1)
    _same(gpu_session.fetch(31), ref, rl)


def test_packed_empty_and_tiny(gpu_session):
    for reads in ([], [""], ["ACG"], ["ACGTTGCAACGTAGGCT" * 3, "NNACGTTGCAAC"]):
        buf, off = eulerhip.pack_reads(reads)
        pr = eulerhip.pack_2bit(buf, off)
        for k in (3, 5):
            d, r, g = oracle.assemble(reads, k, 1)
            gpu_session.run_packed_host(pr, k, 1)
            res = gpu_session.fetch(k)
            assert res.contigs == r and res.links == g


def test_packed_headline_shape_pinned(gpu_session):
    """the bench's host-input leg: page-locked codes, 1 M reads of 100 bp (super-k-mer path)"""
    torch = pytest.importorskip("torch")
    buf, off = make_reads(460_000, 1_000_000, 100, 7200)
    ref, rl = _ref(buf, off, 31)
    pr = eulerhip.pack_2bit(buf, off, alloc=lambda n: torch.empty(n, dtype=torch.uint8, pin_memory=True).numpy())
    gpu_session.run_packed_host(pr, 31, 1)
    res = gpu_session.fetch(31)
    assert res.stats.count_variant == 3
    _same(res, ref, rl)


@pytest.mark.parametrize("chunks", ["1", "6"])
def test_staged_batches_vs_oracle(gpu_session, monkeypatch, chunks):
    """ec_stage_packed_host / ec_assemble_staged: a pipeline of batches of different shapes (one
    length, ragged with offsets, N exceptions, k = 31 / 25 / 51), batch i + 1 staged before batch
    i is assembled, each result equal to the oracle; misuse is refused (EC_ERR_STATE)"""
    monkeypatch.setenv("EULERHIP_HOST_CHUNKS", chunks)
    batches = []
    for i, (g, n, L, err, nr, k) in enumerate([(40_000, 20_000, 100, 0.0, 0.0, 31), (30_000, 10_000, 90, 0.002, 0.003, 25),
                                                (20_000, 6_000, 150, 0.002, 0.0, 51), (40_000, 12_000, 100, 0.0, 0.0, 31)]):
        buf, off = make_reads(g, n, L, 7300 + i, err=err, n_rate=nr)
        if i == 3:  # ragged: drop the tail of every 7th read
            reads = [buf[int(off[j]):int(off[j + 1])].tobytes().decode()[: (60 if j % 7 == 0 else L)] for j in range(n)]
            buf, off = eulerhip.pack_reads(reads)
        pr = eulerhip.pack_2bit(buf, off)
        batches.append((pr, k, _ref(buf, off, k)))
    with pytest.raises(eulerhip.EulerHipError):
        gpu_session.assemble_staged(31)  # nothing staged
    gpu_session.stage_packed(batches[0][0])
    gpu_session.stage_packed(batches[1][0])
    with pytest.raises(eulerhip.EulerHipError):
        gpu_session.stage_packed(batches[2][0])  # both slots taken
    with pytest.raises(eulerhip.EulerHipError):
        gpu_session.run_packed_host(batches[2][0], 31, 1)  # batches pending
    for i in range(len(batches)):
        pr, k, (ref, rl) = batches[i]
        gpu_session.assemble_staged(k, 1)
        if i + 2 < len(batches):
            gpu_session.stage_packed(batches[i + 2][0])
        _same(gpu_session.fetch(k), ref, rl)
    # the immediate entry works again once the pipeline is empty
    pr, k, (ref, rl) = batches[0]
    gpu_session.run_packed_host(pr, k, 1)
    _same(gpu_session.fetch(k), ref, rl)


def test_staged_read_set_from_file(gpu_session, tmp_path):
    """FASTA file -> page-locked 2-bit codes (EC_READS_PACKED) -> staged batches -> contigs"""
    import ingest

    paths = []
    for i in range(3):
        buf, off = make_reads(30_000, 8_000, 100, 7400 + i, err=0.001)
        p = tmp_path / ("r%d.fa" % i)
        with open(p, "wb") as f:
            for j in range(len(off) - 1):
                f.write(b">r\n" + buf[int(off[j]):int(off[j + 1])].tobytes() + b"\n")
        paths.append((str(p), _ref(buf, off, 31)))
    sets = [ingest.ReadSet(p, packed=True) for p, _ in paths]
    sets[0].stage(gpu_session)
    sets[1].stage(gpu_session)
    for i in range(3):
        gpu_session.assemble_staged(31, 1)
        if i + 2 < 3:
            sets[i + 2].stage(gpu_session)
        ref, rl = paths[i][1]
        _same(gpu_session.fetch(31), ref, rl)
    # and the one-call form
    sets[2].assemble(gpu_session, 31, 1)
    _same(gpu_session.fetch(31), *paths[2][1])
    for rs in sets:
        rs.close()
