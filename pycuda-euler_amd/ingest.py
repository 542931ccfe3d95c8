"""ingest -- native FASTA / FASTQ ingest and contig / GFA writers (row 2).

ReadSet parses a read file with the multi-threaded C++ reader of libeulerhip.so
(csrc/ingest.cpp: mmap + two-pass parallel parse) straight into the packed CSR layout the
device path consumes (uint8 bases + uint64 offsets); packed(first, count) hands out one
rank's shard.  The writers emit the reference's output formats from a Result.
"""
import ctypes
import os

import numpy as np

import eulerhip

FASTA_RECORDS, FASTA_LINES, FASTQ = 0, 1, 2
_P = ctypes.c_void_p
_U64 = ctypes.c_uint64
eulerhip.register("ec_reads_load", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_P)])
eulerhip.register("ec_reads_count", _U64, [_P])
eulerhip.register("ec_reads_bases", _U64, [_P])
eulerhip.register("ec_reads_span", _U64, [_P, _U64, _U64])
eulerhip.register("ec_reads_copy", ctypes.c_int, [_P, _U64, _U64, _P, _P])
eulerhip.register("ec_reads_free", None, [_P])
eulerhip.register("ec_reads_release_pool", None, [])
eulerhip.register("ec_reads_packed_info", ctypes.c_int, [_P, _P, _P, _P])
eulerhip.register("ec_reads_packed_copy", ctypes.c_int, [_P, _P, _P, _P])
eulerhip.register("ec_assemble_packed_reads", ctypes.c_int, [_P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_uint])
eulerhip.register("ec_stage_packed_reads", ctypes.c_int, [_P, _P])
READS_PACKED = 0x100  # EC_READS_PACKED


def detect_format(path, fasta_mode="records"):
    """FASTQ for .fq/.fastq (or a leading '@'), else FASTA as records or lines."""
    fasta = FASTA_LINES if fasta_mode == "lines" else FASTA_RECORDS
    ext = path.rsplit(".", 1)[-1].lower()
    if ext in ("fq", "fastq"):
        return FASTQ
    if ext in ("fa", "fasta", "fsa", "fna"):
        return fasta
    with open(path, "rb") as f:
        return FASTQ if f.read(1) == b"@" else fasta


class ReadSet:
    """A read file parsed by the native reader (host memory, freed on close).

    packed=True: the reader writes the bases straight as 2-bit codes into page-locked memory
    (EC_READS_PACKED) -- the input of assemble(); packed_reads() copies them out."""

    def __init__(self, path, fmt=None, threads=0, fasta_mode="records", packed=False):
        self.path = path
        self.format = detect_format(path, fasta_mode) if fmt is None else fmt
        self.is_packed = bool(packed)
        h = _P()
        f = int(self.format) | (READS_PACKED if packed else 0)
        eulerhip.check(eulerhip.lib().ec_reads_load(os.fsencode(path), f, int(threads), ctypes.byref(h)))
        self._h = h

    def __len__(self):
        return int(eulerhip.lib().ec_reads_count(self._h))

    @property
    def n_bases(self):
        return int(eulerhip.lib().ec_reads_bases(self._h))

    def packed(self, first=0, count=None):
        """(bases uint8[], offsets uint64[count + 1]) of reads [first, first + count)."""
        n = len(self)
        count = n - first if count is None else int(count)
        nb = int(eulerhip.lib().ec_reads_span(self._h, int(first), count))
        buf = np.zeros(max(nb, 1), np.uint8)
        off = np.zeros(count + 1, np.uint64)
        eulerhip.check(eulerhip.lib().ec_reads_copy(self._h, int(first), count, buf.ctypes.data, off.ctypes.data))
        return buf[:nb], off

    def packed_reads(self):
        """the packed set as an eulerhip.PackedReads (numpy copies; packed=True sets only)"""
        nb, rl, ne = ctypes.c_uint64(0), ctypes.c_uint32(0), ctypes.c_uint64(0)
        eulerhip.check(eulerhip.lib().ec_reads_packed_info(self._h, ctypes.byref(nb), ctypes.byref(rl),
                                                           ctypes.byref(ne)))
        nb, rl, ne = nb.value, rl.value, ne.value
        codes = np.zeros(max((nb + 3) // 4, 1), np.uint8)
        pos = np.zeros(max(ne, 1), np.uint64)
        byt = np.zeros(max(ne, 1), np.uint8)
        eulerhip.check(eulerhip.lib().ec_reads_packed_copy(self._h, codes.ctypes.data, pos.ctypes.data,
                                                           byt.ctypes.data))
        off = None
        if not rl:
            off = np.zeros(len(self) + 1, np.uint64)
            eulerhip.check(eulerhip.lib().ec_reads_copy(self._h, 0, len(self), None, off.ctypes.data))
        return eulerhip.PackedReads(codes, nb, len(self), off, rl, pos[:ne], byt[:ne])

    def assemble(self, session, k, limit=1, flags=0):
        """the fused assembly on session straight from the packed set (ec_assemble_packed_reads);
        session.fetch(k) then returns the Result"""
        eulerhip.check(eulerhip.lib().ec_assemble_packed_reads(session._h, self._h, int(k), int(limit), int(flags)))

    def stage(self, session):
        """queue this packed set as session's next staged batch (ec_stage_packed_reads); keep the
        ReadSet open until session.assemble_staged() has consumed it"""
        eulerhip.check(eulerhip.lib().ec_stage_packed_reads(session._h, self._h))

    def reads(self):
        """the reads as Python strings (small inputs / tests)"""
        buf, off = self.packed()
        s = buf.tobytes().decode("ascii", errors="replace")
        return [s[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]

    def close(self):
        if getattr(self, "_h", None):
            eulerhip.lib().ec_reads_free(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        self.close()


def release_pool():
    """free the page-locked code buffer ec_reads_free keeps for the next packed load (teardown)"""
    eulerhip.lib().ec_reads_release_pool()


def load_reads(path, fmt=None, threads=0, fasta_mode="records", first=0, count=None):
    """(bases, offsets) of a read file (or of reads [first, first + count))."""
    with ReadSet(path, fmt, threads, fasta_mode) as rs:
        return rs.packed(first, count)


# ---- writers ---------------------------------------------------------------
def write_contigs_fasta(path, result, header="contig%d", blank_line=False):
    """Contigs of a Result as FASTA: header 'contig%d' with a blank line = print_dbg
    (tests/referenceAssembler.py:131-134); header '%u' = generatePartialContig / assemble2
    (src/eulercuda.py:352)."""
    ch = result.contig_bytes
    o = result.contig_offsets
    with open(path, "wb") as f:
        for i in range(len(o) - 1):
            f.write(b">" + (header % i).encode() + b"\n")
            f.write(ch[int(o[i]):int(o[i + 1])])
            f.write(b"\n\n" if blank_line else b"\n")


def write_gfa(path, result, k):
    """GFA 1 of a Result: print_GFA (tests/referenceAssembler.py:119-129)."""
    ch = result.contig_bytes
    o = result.contig_offsets
    lo, lk = result.link_offsets, result.link_codes
    with open(path, "w") as f:
        f.write("H  VN:Z:1.0\n")
        for i in range(len(o) - 1):
            f.write("S\t%d\t%s\t*\n" % (i, ch[int(o[i]):int(o[i + 1])].decode("ascii")))
        for i in range(len(o) - 1):
            for side, sgn in ((0, "+"), (1, "-")):
                for v in lk[int(lo[2 * i + side]):int(lo[2 * i + side + 1])]:
                    f.write("L\t%d\t%s\t%d\t%s\t%dM\n" % (i, sgn, int(v) >> 1, "-" if v & 1 else "+", k - 1))
