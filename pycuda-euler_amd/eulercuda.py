"""eulercuda -- drop-in for the reference driver src/eulercuda.py (assemble2 and its helpers).

Two pipelines sit behind the reference's entry point assemble2 (src/eulercuda.py:448-508,
reached from Spark as ec.assemble2, src/cli_spark_gpu.py:37):

* mode="fused" (default): the production path.  One libeulerhip.so call (ec_assemble_*) runs
  encode -> count -> solid filter -> de Bruijn links -> list ranking -> contigs on the GPU and
  returns exactly the contigs of the reference's CPU assembler (referenceAssembler.build +
  all_contigs) at node length k = lmerLength - 1 (the GPU path's -k is the EDGE
  length l, vertices are (l-1)-mers).  Windows are per read (SURVEY §A2 fixed).
* mode="modular": the reference's own module-by-module flow (readLmersKmersCuda ->
  create_hash_table_device -> construct_debruijn_graph_device -> findEulerDevice ->
  findSpanningTree -> executeSwipeDevice -> generatePartialContig), every device step in
  libeulerhip.so through the drop-in modules, with the defects of SURVEY §A fixed (racy RC
  encode, tail drop, edge bounds, circuit counts overwriting the graph counts, unbound
  outstrings).  It returns the reference's output format: per contig the list of (l-1)-mer
  strings of the Euler walk (§A9: not overlap-merged).

Both write the reference's FASTA ('>%u' headers, src/eulercuda.py:352) to outfile.
"""
import argparse
import ctypes
import logging

import numpy as np

import _modlib as M
import eulerhip

ULONGLONG = 8
UINTC = 4

module_logger = logging.getLogger("eulercuda")


# ---- ingest (src/eulercuda.py:22-56, 437-445) -----------------------------------------------
def parse_fastq(filename):
    """src/eulercuda.py:22-40: {read_name: read} of a 4-line FASTQ (prints each quality line)."""
    result = {}
    current_name = None
    with open(filename) as f:
        for i, line in enumerate(f):
            if i % 4 == 0:
                current_name = line.rstrip("\n")
            if i % 4 == 1:
                result[current_name] = line.rstrip("\n")
            if i % 4 == 3:
                print("quality is " + line.rstrip("\n"))
    return result


def read_fastq(filename):
    """src/eulercuda.py:43-55: the sequence line of every 4-line record."""
    with open(filename) as f:
        return [line.rstrip("\n") for i, line in enumerate(f) if i % 4 == 1]


def read_fasta(infilename):
    """src/eulercuda.py:437-445: every non-header line, stripped (one read per line)."""
    with open(infilename) as f:
        return [line.strip() for line in f if line[0] != ">"]


def doErrorCorrection(readBuffer, readCount, ec_tuple_size, max_ec_pos):
    """src/eulercuda.py:58-59 (a stub in the reference)."""
    return readCount


# ---- k-mer strings (src/eulercuda.py:307-325) ------------------------------------------------
def dna_translate(i):
    return "ACGT"[i] if i < 4 else "."


def getString(length, value):
    """MSB-first decode of a 2-bit code into `length` bases."""
    v = int(value)
    out = [""] * length
    for i in range(1, length + 1):
        out[length - i] = dna_translate(v % 4)
        v //= 4
    return "".join(out)


def check_kmers(outfile, length, kmers):
    with open(outfile, "w") as f:
        for kmer in kmers:
            f.write(getString(length, kmer) + "\t")


def verify_kmers(buffer, encoded_list, length):
    """src/eulercuda.py:61-70 (unused by the reference): (hits, misses) of decoded codes in buffer."""
    hits = misses = 0
    for x in encoded_list:
        if getString(length, x) in buffer:
            hits += 1
        else:
            misses += 1
    return hits, misses


# ---- the modular pipeline ---------------------------------------------------------------------
def readLmersKmersCuda(readBuffer, readLength, partitionReadCount, lmerLength, lmerKeys, lmerValues, lmerCount,
                       kmerKeys, kmerValues, kmerCount, numReads):
    """src/eulercuda.py:73-179 on the device (ec_read_lmers_kmers): l-mers of the concatenated
    buffer (partitionReadCount positions, zero past the end), F and RC streams deduplicated in
    dict insertion order.  kmerKeys / kmerValues are extended in place as in the reference;
    returns [lmerCount, kmerCount, lmerKeys, lmerValues, kmerKeys, kmerValues]."""
    raw = M.raw_bytes(readBuffer)
    B = int(partitionReadCount)
    raw = (raw + b"\0" * max(0, B - len(raw)))[:B]
    b = np.frombuffer(raw, np.uint8) if B else np.zeros(1, np.uint8)
    lk = np.zeros(max(2 * B, 1), np.uint64)
    lv = np.zeros(max(2 * B, 1), np.uint32)
    kk = np.zeros(max(4 * B, 1), np.uint64)
    nl, ne, nk = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
    M.call("ec_read_lmers_kmers", M.ptr(b), B, int(lmerLength), M.ptr(lk), M.ptr(lv), ctypes.byref(nl),
           ctypes.byref(ne), M.ptr(kk), ctypes.byref(nk))
    keys = [int(x) for x in lk[: nl.value]]
    vals = [int(x) for x in lv[: nl.value]]
    if ne.value > 0 and keys:  # the zero l-mer overwrites the last real one (:175-177)
        keys[-1] = 0
        vals[-1] = int(ne.value)
    kmerKeys.extend(int(x) for x in kk[: nk.value])
    kmerValues.extend(range(len(kmerValues), len(kmerValues) + nk.value))
    return [nl.value + ne.value, nk.value, keys, vals, kmerKeys, kmerValues]


def constructDebruijnGraph(readBuffer, partitionReadCount, readLength, lmerLength, evList, eeList, levEdgeList,
                           entEdgeList, numReads):
    """src/eulercuda.py:182-263.  Returns (ee, ev, levEdge, entEdge, kmerCount, edgeCount) -- the
    reference's two name swaps (:259, :497) cancel, so its caller receives ee first."""
    import pydebruijn as db
    import pygpuhash as gh

    lmerCount, kmerCount, lmerKeys, lmerValues, kmerKeys, kmerValues = readLmersKmersCuda(
        readBuffer, readLength, partitionReadCount, lmerLength, [], [], 0, [], [], 0, numReads)
    tableLength, bucketSize, bucketCount, TK, TV = gh.create_hash_table_device(kmerKeys, kmerValues, kmerCount, None,
                                                                               None, 0, None, 0)
    # the arrays hold len(lmerMap) entries; lmerCount adds the empties and is not
    # used to read past them
    ee, ev, lev, ent, kmerCount, edgeCount = db.construct_debruijn_graph_device(
        lmerKeys, lmerValues, len(lmerKeys), kmerKeys, kmerCount, lmerLength, TK, TV, bucketSize, bucketCount, None,
        None, None, None, readLength)
    return ee, ev, lev, ent, kmerCount, edgeCount


def findSpanningTree(cg_edge, cg_edgecount, cg_vertexcount):
    """src/eulercuda.py:266-305: a spanning forest of the circuit graph (unit weights, Kruskal in
    the (c1, c2)-sorted edge order), on the device (ec_spanning_forest: Boruvka rounds that find
    the forest Kruskal takes in edge-index order).  Returns circuit-graph EDGE indices -- what
    markSpanningEulerEdges indexes with (the reference returned vertex pairs).
    The reference's graph_tool tie-breaking is unversioned: parity unpinned."""
    E = int(cg_edgecount)
    cg = M.as_struct(np.asarray(cg_edge)[:E], M.CE) if E else np.zeros(0, M.CE)
    tree = np.zeros(max(E, 1), np.uint32)
    nt = ctypes.c_uint64(0)
    M.call("ec_spanning_forest", M.ptr(cg), E, int(cg_vertexcount), M.ptr(tree), ctypes.byref(nt))
    return tree[: nt.value].copy()


def partial_contigs_device(d_ev, vcount, d_ee, ecount, l):
    """The walk of generatePartialContig on the device (ec_partial_contigs): list of contigs,
    each the list of (l-1)-mer strings."""
    E = int(ecount)
    ev = M.as_struct(np.asarray(d_ev)[: int(vcount)], M.EV)
    ee = M.as_struct(np.asarray(d_ee)[:E], M.EE)
    km1 = int(l) - 1
    chars = np.zeros(max(2 * E * km1, 1), np.uint8)
    coff = np.zeros(E + 1, np.uint64)
    nc, nch = ctypes.c_uint64(0), ctypes.c_uint64(0)
    M.call("ec_partial_contigs", M.ptr(ev), len(ev), M.ptr(ee), E, int(l), M.ptr(chars), M.ptr(coff),
           ctypes.byref(nc), ctypes.byref(nch))
    text = chars[: nch.value].tobytes().decode("ascii")
    out = []
    for c in range(nc.value):
        s = text[int(coff[c]):int(coff[c + 1])]
        out.append([s[i:i + km1] for i in range(0, len(s), km1)])
    return out


def generatePartialContig(outfile, d_ev, vcount, d_ee, ecount, l):
    """src/eulercuda.py:328-402: contig starts, the Euler walk, FASTA output ('>%u' headers);
    returns the list of buffers.  (The reference's debug dump generatePartialContig.tsv is
    not written.)"""
    output = partial_contigs_device(d_ev, vcount, d_ee, ecount, l)
    if outfile:
        with open(outfile, "w") as f:
            for i, buf in enumerate(output):
                f.write(">%u\n" % i)
                f.write("".join(buf) + "\n")
    return output


def mergeEulerCircuits(d_ev, d_ee, d_levEdge, d_entEdge, edgeCountList, vertexCount):
    """The Euler-circuit merge the reference sets up and leaves as a no-op (src/eulercuda.py:
    425-431, src/pyeulertour.py:495-664), on the device: successor pairing
    and circuits (findEulerDevice), the spanning forest of the circuit graph (findSpanningTree,
    Boruvka on the device), then the swipe with only the forest's edges marked.  Returns the
    edges with merged successors: every connected component of the circuit graph is one tour."""
    import pyeulertour as et

    ee = np.array(d_ee, copy=True)
    cg_edge, cg_edgeCount, cg_vertexCount = et.findEulerDevice(d_ev, d_levEdge, d_entEdge, vertexCount, ee,
                                                               edgeCountList, None, 0, 0)
    if cg_edgeCount > 0:
        tree = findSpanningTree(cg_edge, cg_edgeCount, cg_vertexCount)
        ee = et.executeSwipeDevice(d_ev, d_entEdge, vertexCount, ee, edgeCountList, cg_edge, cg_edgeCount, tree,
                                   len(tree), swipe=True, merge=True)
    return ee


def findEulerTour(d_ev, d_ee, d_levEdge, d_entEdge, edgeCountList, vertexCount, lmerLength, outfile, swipe=False,
                  merge=False):
    """src/eulercuda.py:405-434, with the de Bruijn counts kept (the reference
    overwrote them with the circuit-graph counts and left outstrings unbound without circuit
    edges).  swipe=True runs the swipe body the reference leaves commented out; merge=True
    merges each component's circuits into one tour first (mergeEulerCircuits)."""
    import pyeulertour as et

    if merge:
        ee = mergeEulerCircuits(d_ev, d_ee, d_levEdge, d_entEdge, edgeCountList, vertexCount)
        return generatePartialContig(outfile, d_ev, vertexCount, ee, edgeCountList, lmerLength)
    ee = np.array(d_ee, copy=True)
    cg_edge, cg_edgeCount, cg_vertexCount = et.findEulerDevice(d_ev, d_levEdge, d_entEdge, vertexCount, ee,
                                                               edgeCountList, None, 0, 0)
    if cg_edgeCount > 0:
        tree = findSpanningTree(cg_edge, cg_edgeCount, cg_vertexCount)
        ee = et.executeSwipeDevice(d_ev, d_entEdge, vertexCount, ee, edgeCountList, cg_edge, cg_edgeCount, tree,
                                   len(tree), swipe=swipe)
    return generatePartialContig(outfile, d_ev, vertexCount, ee, edgeCountList, lmerLength)


# ---- assemble2 --------------------------------------------------------------------------------
def _load(buffer, infile):
    if infile:
        ext = infile.split(".")[-1]
        if ext in ("fa", "fasta", "fsa"):
            return read_fasta(infile)
        if ext in ("fq", "fastq"):
            return read_fastq(infile)
        raise ValueError("unknown read file extension %r" % ext)
    return list(buffer) if not isinstance(buffer, (str, bytes)) else [buffer]


def write_fasta(outfile, contigs):
    with open(outfile, "w") as f:
        for i, c in enumerate(contigs):
            f.write(">%u\n%s\n" % (i, c))


def assemble2(lmerLength, buffer="", readLength=0, readCount=0, infile="", outfile="", mode="fused", limit=1,
              session=None):
    """src/eulercuda.py:448-508.  buffer: list of reads (or read file via infile).  Returns
    the contigs (fused: strings; modular: lists of (l-1)-mer strings) and writes them to
    outfile as FASTA when given."""
    reads = [r.decode("ascii") if isinstance(r, bytes) else r for r in _load(buffer, infile)]
    module_logger.info("Got %d reads.", len(reads))
    if mode == "fused":
        sess = session or eulerhip.default_session()
        res = sess.assemble(reads, int(lmerLength) - 1, limit=limit)
        contigs = list(res.contigs)
        if outfile:
            write_fasta(outfile, contigs)
        return contigs
    if mode != "modular":
        raise ValueError("mode must be 'fused' or 'modular'")
    readBuffer = "".join(reads).encode("ascii")
    baseCount = len(readBuffer)
    if baseCount == 0:
        return []
    readLength = len(reads[0]) if reads else 0
    ee, ev, lev, ent, vertexCount, edgeCount = constructDebruijnGraph(readBuffer, baseCount, readLength, lmerLength,
                                                                      [], [], [], [], len(reads))
    return findEulerTour(ev, ee, lev, ent, edgeCount, vertexCount, lmerLength, outfile or "")


def main(argv=None):
    """src/eulercuda.py:510-530 CLI: -i reads -o contigs -k lmerLength (required here)."""
    p = argparse.ArgumentParser(description="MI355X de Bruijn / Euler-tour assembler")
    p.add_argument("-i", dest="input_filename", required=True, help="input FASTA / FASTQ")
    p.add_argument("-o", dest="output_filename", default="", help="output contig FASTA")
    p.add_argument("-k", dest="k", type=int, required=True, help="l-mer (edge) length; contigs use k-1 nodes")
    p.add_argument("-d", dest="debug", action="store_true", default=False)
    p.add_argument("--mode", default="fused", choices=["fused", "modular"])
    p.add_argument("--limit", type=int, default=1, help="solid filter: keep k-mers seen more than this")
    a = p.parse_args(argv)
    logging.basicConfig(level=logging.DEBUG if a.debug else logging.INFO)
    out = assemble2(a.k, infile=a.input_filename, outfile=a.output_filename or "", mode=a.mode, limit=a.limit)
    if not a.output_filename:
        for i, c in enumerate(out):
            print(">%u\n%s" % (i, c if isinstance(c, str) else "".join(c)))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
