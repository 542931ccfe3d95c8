"""CPU tests of the reference-interface host modules (eulercuda.py, assembler.py): ingest,
string helpers, output formats, spanning forest -- and of the oracle restatements the GPU
module tests check against (readLmersKmersCuda, generatePartialContig)."""
import io
import json
import os

import numpy as np

import modules_ref as R
from conftest import GOLDEN, golden_cases

import assembler  # noqa: E402
import eulercuda  # noqa: E402


def test_read_fasta_matches_reference_test():
    """tests/test_fasta_reader.py:3 holds the expected read list of g200reads.fa"""
    kat = json.load(open(os.path.join(GOLDEN, "kat.json")))
    assert eulercuda.read_fasta(os.path.join(GOLDEN, "g200reads.fa")) == kat["g200_reads"]
    assert assembler.read_fasta_records(os.path.join(GOLDEN, "g200reads.fa")) == kat["g200_reads"]


def test_fasta_records_join_lines(tmp_path):
    p = tmp_path / "x.fa"
    p.write_text(">a\nACG\nTT\n>b\nGG\n")
    assert assembler.read_fasta_records(str(p)) == ["ACGTT", "GG"]
    assert eulercuda.read_fasta(str(p)) == ["ACG", "TT", "GG"]  # per line, as src/eulercuda.py:443


def test_fastq(tmp_path, capsys):
    p = tmp_path / "r.fastq"
    p.write_text("@r1\nACGT\n+\nIIII\n@r2\nGGCN\n+\nIIII\n")
    assert eulercuda.read_fastq(str(p)) == ["ACGT", "GGCN"]
    assert eulercuda.parse_fastq(str(p)) == {"@r1": "ACGT", "@r2": "GGCN"}
    assert "quality is IIII" in capsys.readouterr().out


def test_get_string():
    assert eulercuda.getString(4, 27) == "ACGT"
    assert eulercuda.getString(11, 3836979) == "TGGGATAATAT"
    assert eulercuda.dna_translate(7) == "."
    for v in (0, 1, 12345, (1 << 62) + 77):
        assert eulercuda.getString(31, v) == R.get_string(31, v)


def test_spanning_forest():
    cg = np.zeros(6, R.CE)
    cg["c1"] = [0, 0, 1, 2, 3, 3]
    cg["c2"] = [1, 2, 2, 3, 4, 4]
    assert R.spanning_forest(cg, 6, 6) == [0, 1, 3, 4]  # vertex 5 isolated: a forest with 4 edges


def test_string_helpers():
    assert assembler.twin("AACGN") == "NCGTT"
    assert list(assembler.fw("ACG")) == ["CGA", "CGC", "CGG", "CGT"]
    assert list(assembler.bw("ACG")) == ["AAC", "CAC", "GAC", "TAC"]
    assert list(assembler.kmers("ACGTA", 3)) == ["ACG", "CGT", "GTA"]
    assert assembler.contig_to_string(["ACG", "CGT", "GTA"]) == "ACGTA"


def test_output_formats():
    c = [x for x in golden_cases("g200.json") if x["name"] == "g200_k11"][0]
    G = {i: ([tuple(x) for x in s[0]], [tuple(x) for x in s[1]]) for i, s in enumerate(c["links"])}
    f = io.StringIO()
    assembler.print_GFA(G, c["contigs"], 11, file=f)
    lines = f.getvalue().splitlines()
    assert lines[0] == "H  VN:Z:1.0"
    assert lines[1] == "S\t0\t%s\t*" % c["contigs"][0]
    nl = sum(len(s[0]) + len(s[1]) for s in c["links"])
    assert len(lines) == 1 + len(c["contigs"]) + nl
    assert all(x.endswith("\t10M") for x in lines[1 + len(c["contigs"]):])
    f = io.StringIO()
    assembler.print_dbg(c["contigs"][:2], file=f)
    assert f.getvalue() == ">contig0\n%s\n\n>contig1\n%s\n\n" % tuple(c["contigs"][:2])


def test_oracle_read_lmers_kmers_semantics():
    buf = b"ACGTAAAACG"
    lc, kc, lk, lv, kk, kv = R.read_lmers_kmers(buf, 4)
    F = R.encode_lmers(buf, 4)
    Rr = R.encode_lmers_rc(buf, 4)
    zeros = int((F == 0).sum() + (Rr == 0).sum())
    assert zeros > 0 and lk[-1] == 0 and lv[-1] == zeros  # the empty l-mer overwrites the last one
    assert lc == len(lk) + zeros
    assert kv == list(range(kc)) and len(set(kk)) == kc


def test_oracle_partial_contigs_paths_and_cycles():
    # edges 0->1->2 (a path), 3->4->3 (a cycle), 5 alone
    ev = np.zeros(6, R.EV)
    ev["vid"] = [0, 1, 2, 3, 4, 5]
    ee = np.zeros(6, R.EE)
    ee["eid"] = np.arange(6)
    ee["v1"] = [0, 1, 2, 3, 4, 5]
    ee["v2"] = [1, 2, 3, 4, 3, 0]
    ee["s"] = [1, 2, 6, 4, 3, 6]
    out = R.partial_contigs(ev, ee, 3)
    g = [R.get_string(2, i) for i in range(6)]
    assert out == [[g[0], g[1], g[2], g[3]], [g[5], g[0]], [g[3], g[4], g[3]]]


def test_get_optimal_launch_configuration():
    """E4 (src/pyencode.py:237-255): block = (threadPerBlock, 1, 1); grid y = ceil(threads /
    threadPerBlock) capped at 65535, grid x = y_uncapped // 65535 + 1 -- values worked out by hand
    from the reference's arithmetic"""
    import pyencode

    cases = [
        ((10, 32), ((32, 1, 1), (1, 1, 1))),            # threadCount <= threadPerBlock
        ((32, 32), ((32, 1, 1), (1, 1, 1))),
        ((33, 32), ((32, 1, 1), (1, 2, 1))),
        ((100, 32), ((32, 1, 1), (1, 4, 1))),
        ((65535 * 32, 32), ((32, 1, 1), (2, 65535, 1))),  # y = 65535 exactly: x = 65535 // 65535 + 1
        ((65535 * 32 + 1, 32), ((32, 1, 1), (2, 65535, 1))),
        ((200_000_000, 100), ((100, 1, 1), (31, 65535, 1))),
    ]
    for args, want in cases:
        assert pyencode.getOptimalLaunchConfiguration(*args) == want, args
