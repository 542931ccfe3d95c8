"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes front-end of the plain-C restatement (oracle/refasm.c) of the reference CPU
assembler src/referenceassembler/referenceAssembler.py (build:25-42, all_contigs:79-111).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module;
the product path (pycuda-euler_amd/) never does.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")


class _Result(ctypes.Structure):
    _fields_ = [
        ("n_positions", ctypes.c_uint64),
        ("n_dict", ctypes.c_uint64),
        ("dict_kmers", ctypes.POINTER(ctypes.c_char)),
        ("dict_counts", ctypes.POINTER(ctypes.c_uint32)),
        ("n_contigs", ctypes.c_uint64),
        ("contig_chars", ctypes.POINTER(ctypes.c_char)),
        ("contig_offsets", ctypes.POINTER(ctypes.c_uint64)),
        ("link_offsets", ctypes.POINTER(ctypes.c_uint64)),
        ("links", ctypes.POINTER(ctypes.c_int64)),
    ]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        _lib.oracle_assemble.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_uint, ctypes.POINTER(_Result)]
        _lib.oracle_assemble.restype = ctypes.c_int
        _lib.oracle_assemble_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_uint, ctypes.c_int, ctypes.POINTER(_Result)]
        _lib.oracle_assemble_mt.restype = ctypes.c_int
        _lib.oracle_assemble_str.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_uint, ctypes.POINTER(_Result)]
        _lib.oracle_assemble_str.restype = ctypes.c_int
        _lib.oracle_free.argtypes = [ctypes.POINTER(_Result)]
        _lib.oracle_last_error.restype = ctypes.c_char_p
    return _lib


class OracleError(RuntimeError):
    pass


def pack_reads(reads):
    """list[str] -> (uint8 buffer, uint64 offsets[n+1])"""
    b = "".join(reads).encode("ascii")
    off = np.zeros(len(reads) + 1, dtype=np.uint64)
    if reads:
        off[1:] = np.cumsum([len(r) for r in reads], dtype=np.uint64)
    return np.frombuffer(b, dtype=np.uint8) if b else np.zeros(1, np.uint8), off


def assemble_packed(buf, offsets, k, limit=1, want_dict=False, threads=None, string=False):
    """Run the oracle on a packed read set. Returns dict with d (optional), contigs, links.
    threads = N: the N-core variant (map -> reduceByKey counting as src/ref_spark.py:76-84 on N
    host threads, all_contigs single-threaded); same results.  Reads with bytes outside
    {A,C,G,T,N} take the string-keyed restatement (refasm_str.c); string=True forces it."""
    L = lib()
    res = _Result()
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    nreads = len(offsets) - 1
    if string:
        rc = L.oracle_assemble_str(buf.ctypes.data, offsets.ctypes.data, nreads, k, limit,
                                   1 if want_dict else 0, ctypes.byref(res))
    elif threads:
        rc = L.oracle_assemble_mt(buf.ctypes.data, offsets.ctypes.data, nreads, k, limit,
                                  1 if want_dict else 0, int(threads), ctypes.byref(res))
    else:
        rc = L.oracle_assemble(buf.ctypes.data, offsets.ctypes.data, nreads, k, limit,
                               1 if want_dict else 0, ctypes.byref(res))
    if rc != 0:
        raise OracleError("oracle_assemble rc=%d: %s" % (rc, L.oracle_last_error().decode()))
    try:
        out = {"n_positions": res.n_positions, "n_dict": res.n_dict}
        nc = res.n_contigs
        coff = np.ctypeslib.as_array(res.contig_offsets, shape=(nc + 1,)).copy() if nc else np.zeros(1, np.uint64)
        total = int(coff[-1])
        chars = ctypes.string_at(res.contig_chars, total) if total else b""
        out["contig_chars"] = chars
        out["contig_offsets"] = coff
        loff = np.ctypeslib.as_array(res.link_offsets, shape=(2 * nc + 1,)).copy() if nc else np.zeros(1, np.uint64)
        nl = int(loff[-1])
        out["link_offsets"] = loff
        out["links"] = np.ctypeslib.as_array(res.links, shape=(nl,)).copy() if nl else np.zeros(0, np.int64)
        if want_dict:
            n = res.n_dict
            ks = ctypes.string_at(res.dict_kmers, n * k).decode() if n else ""
            cnt = np.ctypeslib.as_array(res.dict_counts, shape=(n,)).copy() if n else np.zeros(0, np.uint32)
            out["d"] = [[ks[i * k:(i + 1) * k], int(cnt[i])] for i in range(n)]
        return out
    finally:
        L.oracle_free(ctypes.byref(res))


def unpack_contigs(out):
    ch = out["contig_chars"].decode()
    off = out["contig_offsets"]
    return [ch[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]


def unpack_links(out):
    loff, lk = out["link_offsets"], out["links"]
    n = (len(loff) - 1) // 2
    res = []
    for i in range(n):
        sides = []
        for s in range(2):
            a, b = int(loff[2 * i + s]), int(loff[2 * i + s + 1])
            sides.append([[int(v) >> 1, "-" if v & 1 else "+"] for v in lk[a:b]])
        res.append(sides)
    return res


def assemble(reads, k, limit=1, want_dict=True, threads=None, string=False):
    buf, off = pack_reads(reads)
    out = assemble_packed(buf, off, k, limit, want_dict, threads, string)
    return out.get("d"), unpack_contigs(out), unpack_links(out)
