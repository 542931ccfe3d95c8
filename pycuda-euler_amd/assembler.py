"""assembler -- the reference CPU assembler's interface, GPU-backed.

Mirrors src/referenceassembler/referenceAssembler.py (and its twin tests/referenceAssembler.py):
the same names, arguments and results, with build() and all_contigs() running on the MI355X
through libeulerhip.so:

* build(reads, k, limit)  (:25-42)  -> the insertion-ordered dict {k-mer: count} of solid k-mers,
  produced by the fused counting path with the dict rendered on the device;
* all_contigs(d, k)       (:79-111) -> (G, r): contigs in the reference's order and the GFA link
  table, computed by the device graph phase from the caller's dict (any dict closed under
  twin, as build returns, in any order -- the order decides the contig order as in the
  reference);
* assemble(reads, k, limit) -> (d, G, r) in one fused device pass (no dict round trip);
* print_GFA / print_dbg (:115-130, with the working formatting of tests/referenceAssembler.py:119-134);
* twin / kmers / fw / bw / contig_to_string: the reference's string helpers (host, not on
  the hot path).

Documented deviation: k-mers with bytes other than A/C/G/T (after N-splitting) raise
eulerhip.AlphabetError (the reference keeps them as opaque strings; a 2-bit code cannot).
get_contig / get_contig_forward, the reference's serial per-k-mer walkers inside all_contigs,
are subsumed by the device graph phase and are not exposed.
"""
import argparse
import collections
import sys

import eulerhip

_COMP = {"A": "T", "C": "G", "G": "C", "T": "A"}


def twin(km):
    """:7-10 reverse complement (other characters map to themselves)."""
    return "".join(_COMP.get(c, c) for c in reversed(km))


def kmers(seq, k):
    """:12-14"""
    for i in range(len(seq) - k + 1):
        yield seq[i:i + k]


def fw(km):
    """:16-18"""
    for x in "ACGT":
        yield km[1:] + x


def bw(km):
    """:20-22"""
    for x in "ACGT":
        yield x + km[:-1]


def contig_to_string(c):
    """:44-45"""
    return c[0] + "".join(x[-1] for x in c[1:])


def _session(session):
    return session or eulerhip.default_session()


def build(reads, k=31, limit=1, session=None):
    """:25-42 -- the solid-k-mer dict in the reference's insertion order."""
    res = _session(session).assemble(list(reads), int(k), limit=limit, want_dict=True)
    return collections.OrderedDict(res.dict_items)


def all_contigs(d, k, session=None):
    """:79-111 -- (G, r) for the dict d."""
    res = _session(session).assemble_dict(d, int(k))
    return res.G(), res.contigs


def assemble(reads, k=31, limit=1, session=None, want_dict=True):
    """build + all_contigs in one device pass: (d, G, r)."""
    res = _session(session).assemble(list(reads), int(k), limit=limit, want_dict=want_dict)
    d = collections.OrderedDict(res.dict_items) if want_dict else None
    return d, res.G(), res.contigs


def print_GFA(G, cs, k, file=None):
    """:115-124 (tests/referenceAssembler.py:119-128 formatting)."""
    out = file or sys.stdout
    print("H  VN:Z:1.0", file=out)
    for i, x in enumerate(cs):
        print("S\t%d\t%s\t*" % (i, x), file=out)
    for i in G:
        for j, o in G[i][0]:
            print("L\t%d\t+\t%d\t%s\t%dM" % (i, j, o, k - 1), file=out)
        for j, o in G[i][1]:
            print("L\t%d\t-\t%d\t%s\t%dM" % (i, j, o, k - 1), file=out)


def print_dbg(cs, file=None):
    """:127-130 FASTA (tests/referenceAssembler.py:131-134 formatting)."""
    out = file or sys.stdout
    for i, x in enumerate(cs):
        print(">contig%d\n%s\n" % (i, x), file=out)


def read_fasta_records(path):
    """FASTA records with multi-line sequences joined (the SeqIO parsing of
    tests/referenceAssembler.py:28)."""
    seqs, cur = [], None
    with open(path) as f:
        for line in f:
            line = line.strip()
            if line.startswith(">"):
                if cur is not None:
                    seqs.append("".join(cur))
                cur = []
            elif cur is not None:
                cur.append(line)
    if cur is not None:
        seqs.append("".join(cur))
    return seqs


def build_from_files(fns, k=31, limit=1, session=None):
    """tests/referenceAssembler.py:23-46 -- build over the records of FASTA files."""
    reads = []
    for fn in fns:
        reads.extend(read_fasta_records(fn))
    return build(reads, k, limit, session)


def runAssembler(k, src, session=None):
    """:135-140 -- build over a list of reads, print and return the dict."""
    d = build(src, k=int(k), session=session)
    print("done")
    print(d)
    return d


def main(argv=None):
    """A working CLI for src/assembler.py (whose own is non-functional):
    reads FASTA files, writes contigs as FASTA (print_dbg) or GFA (print_GFA)."""
    p = argparse.ArgumentParser(description="de Bruijn unitig assembler on MI355X")
    p.add_argument("inputs", nargs="+", help="FASTA files")
    p.add_argument("-k", type=int, default=31)
    p.add_argument("--limit", type=int, default=1, help="keep k-mers seen more than this many times")
    p.add_argument("--gfa", action="store_true", help="write GFA instead of FASTA")
    p.add_argument("-o", dest="output", default="", help="output file (default stdout)")
    a = p.parse_args(argv)
    reads = []
    for fn in a.inputs:
        reads.extend(read_fasta_records(fn))
    _, G, cs = assemble(reads, a.k, a.limit, want_dict=False)
    out = open(a.output, "w") if a.output else sys.stdout
    try:
        if a.gfa:
            print_GFA(G, cs, a.k, file=out)
        else:
            print_dbg(cs, file=out)
    finally:
        if a.output:
            out.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
