"""pygpuhash -- drop-in for the reference module src/pygpuhash.py (rows H1-H6).

The reference's static bucketed hash (despite the "Cuckoo" comment at :299): keys binned by
hash_h(key, nb) = ((0x01010101 + 0x12345678*key) mod 2^64 mod 1900813) mod nb with
nb = n//409 + 1, then rank-sorted per bucket into TK/TV[nb*520] (MAX_BUCKET_ITEM = 520).
Layout identical to the reference (checked against its own dump src/hash_tk.txt).  The grid
of floor(n/1024) blocks that silently drops the last n mod 1024 keys (:57-61, :143-147,
SURVEY §A3) is fixed by default; tail_drop=True reproduces it.
"""
import logging

import numpy as np

import _modlib as M

module_logger = logging.getLogger("eulercuda.pygpuhash")

MAX_BUCKET_ITEM = M.BUCKET_ITEMS
ULONGLONG = 8
UINTC = 4


def _flags(tail_drop):
    return M.EC_MOD_TAIL_DROP if tail_drop else 0


def phase1_device(d_keys, d_offset, d_length, count, bucketCount, tail_drop=False):
    """src/pygpuhash.py:18-73: offset of every key inside its bucket and the bucket sizes;
    returns (d_offset, count).  Offsets follow input order (the reference's atomicInc order
    is arbitrary)."""
    keys = M.arr(d_keys, np.uint64)[: int(d_length)]
    n = len(keys)
    off = np.zeros(max(n, 1), np.uint32)
    cnt = np.zeros(int(bucketCount), np.uint32)
    M.call("ec_hash_phase1", M.ptr(keys), n, int(bucketCount), _flags(tail_drop), M.ptr(off), M.ptr(cnt))
    return off[:n], cnt


def copy_to_bucket_device(d_keys, d_values, d_offset, d_length, d_start, bucketCount, d_bufferK, d_bufferV,
                          tail_drop=False):
    """src/pygpuhash.py:76-170: bufferK/V[start[bucket] + offset[i]] = key/value[i]."""
    n = int(d_length)
    if tail_drop and n >= 1024:
        n = (n // 1024) * 1024
    keys = M.arr(d_keys, np.uint64)[:n]
    vals = M.arr(d_values, np.uint32)[:n]
    off = M.arr(d_offset, np.uint32)[:n]
    start = M.arr(d_start, np.uint32)
    bk = M.arr(d_bufferK, np.uint64).copy()
    bv = M.arr(d_bufferV, np.uint32).copy()
    M.call("ec_hash_copy_to_bucket", M.ptr(keys), M.ptr(vals), M.ptr(off), n, M.ptr(start), int(bucketCount),
           M.ptr(bk), M.ptr(bv), len(bk))
    return bk, bv


def bucket_sort_device(d_bufferK, d_bufferV, d_start, d_bucketSize, bucketCount, d_TK, d_TV):
    """src/pygpuhash.py:173-258: TK[b*520 + rank] = key (rank = #{bucket keys < key}), TV alike."""
    bk = M.arr(d_bufferK, np.uint64)
    bv = M.arr(d_bufferV, np.uint32)
    start = M.arr(d_start, np.uint32)
    size = M.arr(d_bucketSize, np.uint32)
    nb = int(bucketCount)
    TK = np.zeros(nb * MAX_BUCKET_ITEM, np.uint64)
    TV = np.zeros(nb * MAX_BUCKET_ITEM, np.uint32)
    TK[: min(len(d_TK), len(TK))] = np.asarray(d_TK, np.uint64)[: len(TK)]
    TV[: min(len(d_TV), len(TV))] = np.asarray(d_TV, np.uint32)[: len(TV)]
    M.call("ec_hash_bucket_sort", M.ptr(bk), M.ptr(bv), len(bk), M.ptr(start), M.ptr(size), nb, M.ptr(TK), M.ptr(TV))
    return TK, TV


def create_hash_table_device(d_keys, d_values, d_length, d_TK, d_TV, tableLength, d_bucketSize, bucketCount,
                             tail_drop=False, dump_path=None):
    """src/pygpuhash.py:261-314: returns [tableLength, bucketSize, bucketCount, TK, TV] with
    bucketCount = d_length//409 + 1 (the passed bucketCount is ignored, as in the reference).
    The reference always writes the TK dump 'hash_tk.txt' (:309-311); pass dump_path for it."""
    module_logger.info("started.")
    keys = M.arr(d_keys, np.uint64)[: int(d_length)]
    vals = M.arr(d_values, np.uint32)[: int(d_length)]
    n = len(keys)
    nb = int(M.lib().ec_hash_bucket_count(n))
    TK = np.zeros(nb * MAX_BUCKET_ITEM, np.uint64)
    TV = np.zeros(nb * MAX_BUCKET_ITEM, np.uint32)
    size = np.zeros(nb, np.uint32)
    M.call("ec_hash_build", M.ptr(keys), M.ptr(vals), n, nb, _flags(tail_drop), M.ptr(TK), M.ptr(TV), M.ptr(size))
    if dump_path:
        with open(dump_path, "w") as f:
            for x in TK:
                f.write(str(int(x)) + "\t")
    module_logger.info("Finished. Leaving.")
    return [nb * MAX_BUCKET_ITEM, size, nb, TK, TV]


def hash_lookup(keys, TK, TV, bucketSize, bucketCount):
    """getHashValue of src/pydebruijn.py:56-87 for a batch of keys: TV or 0xFFFFFFFF."""
    k = M.arr(keys, np.uint64)
    out = np.zeros(max(len(k), 1), np.uint32)
    M.call("ec_hash_lookup", M.ptr(M.arr(TK, np.uint64)), M.ptr(M.arr(TV, np.uint32)),
           M.ptr(M.arr(bucketSize, np.uint32)), int(bucketCount), M.ptr(k), len(k), M.ptr(out))
    return out[: len(k)]
