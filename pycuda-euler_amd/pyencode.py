"""pyencode -- drop-in for the reference module src/pyencode.py (rows E1-E4 of SURVEY §8a).

Same function names, arguments and in-place-fill-and-return behaviour as the PyCUDA module;
the work runs in libeulerhip.so (csrc/modules.hip) on the MI355X.  The reverse-complement
encoder implements the intended semantics (the reference kernel races).
"""
import logging

import numpy as np

import _modlib as M

module_logger = logging.getLogger("eulercuda.pyencode")


def _encode(name, buffer, readCount, d_lmers, lmerLength):
    raw = M.raw_bytes(buffer)
    n = len(d_lmers)
    if len(raw) < n:
        raw = raw + b"\0" * (n - len(raw))
    b = np.frombuffer(raw, dtype=np.uint8)
    out = np.zeros(max(len(b), 1), dtype=np.uint64)
    M.call(name, M.ptr(b), len(b), int(lmerLength), M.ptr(out))
    d_lmers[:] = out[:n]
    return d_lmers


def encode_lmer_device(buffer, readCount, d_lmers, readLength, lmerLength):
    """src/pyencode.py:14-98: d_lmers[p] = 2-bit MSB-first code of buffer[p : p+lmerLength]
    (codeF[c & 7]: A0 C1 G2 T3, N and newline -> 0); filled in place and returned."""
    module_logger.info("started encode_lmer_device.")
    if not (isinstance(buffer, np.ndarray) and isinstance(d_lmers, np.ndarray)):
        print(isinstance(buffer, np.ndarray), isinstance(d_lmers, np.ndarray))  # reference :91-92
        return d_lmers
    _encode("ec_encode_lmers", buffer, readCount, d_lmers, lmerLength)
    module_logger.info("finished encode_lmer_device.")
    return d_lmers


def compute_kmer_device(lmers, pkmers, skmers, kmerBitMask, readLength, readCount):
    """src/pyencode.py:101-159: prefix = (l & (mask<<2)) >> 2, suffix = l & mask for the first
    readCount l-mers (the rest of pkmers / skmers is left as is); returns (pkmers, skmers)."""
    module_logger.info("started compute_kmer_device.")
    if not (isinstance(lmers, np.ndarray) and isinstance(pkmers, np.ndarray) and isinstance(skmers, np.ndarray)):
        module_logger.warning("PROBLEM WITH GPU.")  # reference :152-153
        return pkmers, skmers
    n = min(int(readCount), len(lmers), len(pkmers), len(skmers))
    lm = M.arr(lmers[:n], np.uint64)
    pk = np.zeros(max(n, 1), np.uint64)
    sk = np.zeros(max(n, 1), np.uint64)
    M.call("ec_split_kmers", M.ptr(lm), n, int(kmerBitMask) & 0xFFFFFFFFFFFFFFFF, M.ptr(pk), M.ptr(sk))
    pkmers[:n] = pk[:n]
    skmers[:n] = sk[:n]
    module_logger.info("leaving compute_kmer_device.")
    return pkmers, skmers


def compute_lmer_complement_device(buffer, readCount, d_lmers, readLength, lmerLength):
    """src/pyencode.py:162-232, intended semantics: d_lmers[p] = sum_i codeR(buffer[p+i]) << 2i,
    i.e. the MSB-first code of the reverse complement of the l-mer at p."""
    module_logger.info("started compute_lmer_complement_device.")
    if not (isinstance(buffer, np.ndarray) and isinstance(d_lmers, np.ndarray)):
        print("Problem with data to GPU")  # reference :223-225
        return d_lmers
    _encode("ec_encode_lmers_rc", buffer, readCount, d_lmers, lmerLength)
    module_logger.info("Finished compute_lmer_complement_device.")
    return d_lmers


def getOptimalLaunchConfiguration(threadCount, threadPerBlock):
    """src/pyencode.py:237-255: the reference's 2-D launch helper (kept for API parity; the HIP
    kernels size their own grids)."""
    block = (threadPerBlock, 1, 1)
    gx, gy = 1, 1
    if threadCount > threadPerBlock:
        gy = -(-threadCount // threadPerBlock)
        gx = gy // 65535 + 1
        gy = min(gy, 65535)
    return block, (gx, gy, 1)
