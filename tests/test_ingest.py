"""Native ingest (csrc/ingest.cpp, host code: runs without a GPU) against the reference's
Python readers restated in eulercuda.py / assembler.py, incl. multi-threaded chunking."""
import os

import numpy as np
import pytest

import assembler
import eulercuda
import ingest
from conftest import GOLDEN


def _reads(path, fmt, threads=0):
    with ingest.ReadSet(str(path), fmt, threads) as rs:
        out = rs.reads()
        assert rs.n_bases == sum(len(r) for r in out)
        return out


def test_g200():
    p = os.path.join(GOLDEN, "g200reads.fa")
    assert _reads(p, ingest.FASTA_RECORDS) == assembler.read_fasta_records(p)
    assert _reads(p, ingest.FASTA_LINES) == eulercuda.read_fasta(p)


EDGE = [
    "",
    "\n",
    ">only\n",
    ">a\nACGT\n>b\n\n>c\nAC\nGT\n  TT  \n",
    "junk before\n>a\nAC\r\nGT\r\n>b\nNNNN",
    ">a\n\n\nACG\n>b\n>c\nT\n",
    "ACGT\nGGCC\n",
]


@pytest.mark.parametrize("text", EDGE)
def test_fasta_edge_cases(tmp_path, text):
    p = tmp_path / "x.fa"
    p.write_text(text)
    assert _reads(p, ingest.FASTA_RECORDS) == assembler.read_fasta_records(str(p))
    assert _reads(p, ingest.FASTA_LINES) == eulercuda.read_fasta(str(p))


def test_fastq(tmp_path):
    p = tmp_path / "r.fastq"
    p.write_text("@r1\nACGT\n+\n@@@@\n@r2\nGGCN\n+\nIIII\n@r3\nTT")
    assert _reads(p, ingest.FASTQ) == eulercuda.read_fastq(str(p)) == ["ACGT", "GGCN", "TT"]


@pytest.mark.parametrize("threads", [1, 3, 7, 16])
def test_large_multithreaded(tmp_path, threads):
    """~3 MB files split into many chunks: records spanning chunk boundaries, FASTQ line
    numbering across chunks, quality lines starting with '@' or '>'."""
    rng = np.random.default_rng(threads)
    recs = []
    for i in range(6000):
        n = int(rng.integers(0, 700))
        recs.append("".join(rng.choice(list("ACGTN"), n)))
    fa = tmp_path / "big.fa"
    with open(fa, "w") as f:
        for i, r in enumerate(recs):
            f.write(">r%d\n" % i)
            for j in range(0, len(r), 61):
                f.write(r[j:j + 61] + ("\n" if i % 5 else "\r\n"))
    assert _reads(fa, ingest.FASTA_RECORDS, threads) == assembler.read_fasta_records(str(fa))
    assert _reads(fa, ingest.FASTA_LINES, threads) == eulercuda.read_fasta(str(fa))
    fq = tmp_path / "big.fastq"
    with open(fq, "w") as f:
        for i, r in enumerate(recs):
            f.write("@r%d\n%s\n+\n%s\n" % (i, r, ("@>" * len(r))[:len(r)]))
    assert _reads(fq, ingest.FASTQ, threads) == eulercuda.read_fastq(str(fq)) == recs


def test_shards(tmp_path):
    p = os.path.join(GOLDEN, "g200reads.fa")
    with ingest.ReadSet(p) as rs:
        allr = rs.reads()
        buf, off = rs.packed()
        assert off[0] == 0 and int(off[-1]) == len(buf) == rs.n_bases
        got = []
        for first, count in [(0, 30), (30, 0), (30, 41), (71, len(rs) - 71)]:
            b, o = rs.packed(first, count)
            s = b.tobytes().decode()
            got += [s[int(o[i]):int(o[i + 1])] for i in range(count)]
        assert got == allr
        import eulerhip

        with pytest.raises(eulerhip.EulerHipError):
            rs.packed(50, len(rs))


def test_missing_file(tmp_path):
    import eulerhip

    with pytest.raises(eulerhip.EulerHipError):
        ingest.ReadSet(str(tmp_path / "nope.fa"))


def test_detect_format(tmp_path):
    a = tmp_path / "reads.txt"
    a.write_text("@r\nAC\n+\nII\n")
    assert ingest.detect_format(str(a)) == ingest.FASTQ
    assert ingest.detect_format("x.fna") == ingest.FASTA_RECORDS
    assert ingest.detect_format("x.fa", "lines") == ingest.FASTA_LINES


def test_pack_2bit_roundtrip():
    """ec_pack_reads (host): codes + exception bytes give the reads back; one-length detection"""
    import eulerhip
    from synth import make_reads

    for L, nr in ((100, 0.0), (150, 0.01)):
        buf, off = make_reads(50_000, 40_000, L, 11 + L, n_rate=nr)
        buf = buf.copy()
        buf[[5, 77, 4000]] = [ord("a"), ord("x"), ord("\n")]
        pr = eulerhip.pack_2bit(buf, off, threads=4)
        assert pr.read_len == L and pr.offsets is None and pr.nbases == buf.size
        b = np.arange(pr.nbases)
        asc = np.frombuffer(b"ACGT", np.uint8)[(pr.codes[b >> 2] >> (2 * (b & 3))) & 3].copy()
        asc[pr.exc_pos] = pr.exc_byte
        assert np.array_equal(asc, buf)
        assert np.all(np.diff(pr.exc_pos.astype(np.int64)) > 0)
    off2 = off.copy()
    off2[1] += 1  # ragged
    assert eulerhip.pack_2bit(buf, off2).read_len == 0


def test_pack_2bit_rejects_bad_offsets():
    """empty offsets (no nreads + 1 entries), offsets not starting at 0 or not monotone are
    rejected before any read is touched"""
    import pytest

    import eulerhip

    buf = np.frombuffer(b"ACGTACGT", np.uint8)
    with pytest.raises(ValueError):
        eulerhip.pack_2bit(buf, np.zeros(0, np.uint64))
    for bad in ([0, 5, 3, 8], [1, 4, 8]):
        with pytest.raises(eulerhip.EulerHipError):
            eulerhip.pack_2bit(buf, np.array(bad, np.uint64))
    pr = eulerhip.pack_2bit(buf[:0], np.zeros(1, np.uint64))
    assert pr.nreads == 0 and pr.nbases == 0


def _same_packed(pr, ref):
    nc = (ref.nbases + 3) // 4
    assert pr.nbases == ref.nbases and pr.nreads == ref.nreads and pr.read_len == ref.read_len
    assert np.array_equal(pr.codes[:nc], ref.codes[:nc])
    assert np.array_equal(pr.exc_pos, ref.exc_pos) and np.array_equal(pr.exc_byte, ref.exc_byte)
    assert (pr.offsets is None) == (ref.offsets is None)
    if pr.offsets is not None:
        assert np.array_equal(pr.offsets, ref.offsets)


@pytest.mark.parametrize("threads", [1, 5, 16])
def test_packed_load_equals_pack_2bit(tmp_path, threads):
    """EC_READS_PACKED (2-bit codes written by the parser itself, chunk-boundary code bytes by
    atomic OR) == ec_pack_reads of the ASCII load, for every format; one read length -> no offsets"""
    rng = np.random.default_rng(40 + threads)
    for uniform in (False, True):
        recs = []
        for i in range(9000):
            n = 150 if uniform else int(rng.integers(0, 400))
            recs.append("".join(rng.choice(list("ACGTACGTACGTNacgx"), n)))
        fa = tmp_path / "p.fa"
        with open(fa, "w") as f:
            f.write("ACGTjunk before\n")
            for i, r in enumerate(recs):
                f.write(">r%d\n" % i)
                for j in range(0, len(r), 61):
                    f.write(r[j:j + 61] + ("\n" if i % 7 else "\r\n"))
        fq = tmp_path / "p.fastq"
        with open(fq, "w") as f:
            for i, r in enumerate(recs):
                f.write("@r%d\n%s\n+\n%s\n" % (i, r, ("@>" * len(r))[:len(r)]))
        for path, fmt in ((fa, ingest.FASTA_RECORDS), (fa, ingest.FASTA_LINES), (fq, ingest.FASTQ)):
            with ingest.ReadSet(str(path), fmt, threads) as rs:
                buf, off = rs.packed()
            import eulerhip

            ref = eulerhip.pack_2bit(buf, off)
            with ingest.ReadSet(str(path), fmt, threads, packed=True) as rs:
                assert len(rs) == len(off) - 1 and rs.n_bases == len(buf)
                _same_packed(rs.packed_reads(), ref)
                with pytest.raises(eulerhip.EulerHipError):
                    rs.packed(0, 1)  # no ASCII bases in a packed set
            if uniform and fmt != ingest.FASTA_LINES:
                assert ref.read_len == 150


def test_packed_load_empty(tmp_path):
    p = tmp_path / "e.fa"
    p.write_text(">a\n>b\n")
    with ingest.ReadSet(str(p), packed=True) as rs:
        pr = rs.packed_reads()
        assert len(rs) == 2 and pr.nbases == 0 and len(pr.exc_pos) == 0
