"""distributed -- read-sharded multi-GPU assembly, one process per GPU.

Replaces the reference's distribution layer -- Spark `mapPartitions(assemble2)` over read
partitions (src/cli_spark_gpu.py:37) and the CPU path's `reduceByKey` k-mer shuffle
(src/ref_spark.py:76-84) -- with one exchange step over RCCL / xGMI and a correct global
result (the reference's per-partition contigs were never merged):

  1. every rank counts its contiguous read shard on its GPU (ec_count_shard; global read ids
     keep the reference's dict insertion order across shards), keeping all distinct k-mers;
  2. records {key, count, first events} are packed owner-major (owner = hash of the canonical
     key) and exchanged with ONE all-to-all-v (torch.distributed, backend "nccl" = RCCL);
  3. each owner merges what it received (sum of counts, min of first events) and applies the
     solid filter count > limit (build:37-39) -- the reduceByKey of ref_spark.py:84;
  4. each rank places its merged segment at its global ids and emits the (k-1)-mer junction
     records of its keys to the junctions' owners (an all-to-all-v; with minimizer owners
     nearly all stay local); the owners join them into successor links (the links of other
     ranks' nodes travel back in a second, small all-to-all-v) -- no rank holds the job's solid
     set (junction.h);
  5. every rank ranks the chains of its segment in LDS tiles; only the chains (~1/9 of the
     nodes) and then the contig starts are all-gathered; each rank emits its own nodes'
     characters and contig ends and sends rank 0 just those (runs of the positions it wrote:
     ec_graph_emit_runs), and rank 0 collects them with the GFA links -- the complete,
     reference-identical result.  finish="replicated" (hash owners): the solid sets and the
     successor parts are all-gathered and every rank ranks / emits the whole set.

The compute steps go through an *engine* (HipEngine = libeulerhip.so on the rank's GPU) and
the collectives through a *comm* (TorchComm = torch.distributed).  Tests drive the same
orchestration with a CPU engine over gloo (tests/test_distributed.py) and with N simulated
ranks on one GPU (LocalComm), so the N > 1 path is covered without an 8-GPU node.
"""
import ctypes

import numpy as np

import eulerhip

REC_BYTES = 32  # ec_kmer_record (k <= 32)
REC_BYTES_WIDE = 48  # ec_kmer_record_wide (32 < k <= 63)


def rec_bytes(k):
    """exchange record size for node length k (ec_record_bytes)"""
    return REC_BYTES if k <= 32 else REC_BYTES_WIDE


REC_DTYPE = np.dtype([("key", "<u8"), ("count", "<u4"), ("pad", "<u4"), ("first_canon", "<u8"),
                      ("first_twin", "<u8")])

_P = ctypes.c_void_p
_U64 = ctypes.c_uint64
eulerhip.register("ec_count_shard", ctypes.c_int, [_P, _P, _P, _U64, _U64, ctypes.c_int, ctypes.c_uint])
eulerhip.register("ec_dense_count", ctypes.c_uint64, [_P])
eulerhip.register("ec_export_by_owner", ctypes.c_int, [_P, ctypes.c_int, _P, ctypes.POINTER(ctypes.c_uint64)])
eulerhip.register("ec_session_set_owner_rule", ctypes.c_int, [_P, ctypes.c_int])
# compact exchange records (round 5): 20 / 28 B, events shard-relative (the receiver adds bases)
eulerhip.register("ec_export_by_owner_ex", ctypes.c_int, [_P, ctypes.c_int, _P, ctypes.POINTER(ctypes.c_uint64),
                                                          ctypes.c_int, ctypes.POINTER(ctypes.c_int)])
eulerhip.register("ec_compact_record_bytes", ctypes.c_int, [ctypes.c_int])
eulerhip.register("ec_merge_owned_from", ctypes.c_int, [_P, _P, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                                                        ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int32),
                                                        ctypes.c_int, ctypes.c_int, ctypes.c_uint])


def compact_bytes(k):
    """ec_compact_record_bytes"""
    return 20 if k <= 32 else 28

# owner rules (ec_session_set_owner_rule): minimizer ranges (21 <= k <= 52), or a key hash when
# the job's minimizer-range counts are skewed past SKEW times the mean owner (low-complexity input:
# one minimizer can own most records; the merge then falls to the HBM table and every rank pays
# the all-gather padding of the largest part)
OWNER_MINIMIZER, OWNER_HASH = 0, 1
SKEW = 2.0


def minimizer_owners(k):
    """k with minimizer-range owners under OWNER_MINIMIZER (shard.h OwnerFn: 64-bit keys from
    k = 21, 128-bit keys up to count_wide.h's WMB_MAX_K = 52); other k use key-hash owners"""
    return 21 <= k <= 52


def owner_rule_for(totals, k):
    """the rule every rank takes, from the all-reduced per-owner record counts"""
    if not minimizer_owners(k) or len(totals) < 2:
        return OWNER_MINIMIZER
    mean = sum(totals) / len(totals)
    return OWNER_HASH if mean > 0 and max(totals) > SKEW * mean else OWNER_MINIMIZER
eulerhip.register("ec_merge_owned", ctypes.c_int, [_P, _P, _U64, ctypes.c_int, ctypes.c_int, ctypes.c_uint])
eulerhip.register("ec_export_dense", ctypes.c_int, [_P, _P])
eulerhip.register("ec_assemble_from_solid", ctypes.c_int, [_P, _P, _U64, ctypes.c_int, ctypes.c_uint])
eulerhip.register("ec_record_bytes", ctypes.c_int, [ctypes.c_int])
eulerhip.register("ec_graph_load", ctypes.c_int, [_P, _P, _U64, ctypes.c_int, ctypes.c_uint])
eulerhip.register("ec_graph_links_part", ctypes.c_int, [_P, _U64, _U64, _P])
eulerhip.register("ec_graph_finish", ctypes.c_int, [_P, _P, ctypes.c_uint])
eulerhip.register("ec_merge_owned_export", ctypes.c_int, [_P, _P, _U64, ctypes.c_int, ctypes.c_int, ctypes.c_uint, _P])
eulerhip.register("ec_graph_load_links", ctypes.c_int, [_P, _P, _U64, ctypes.c_int, ctypes.c_uint, _U64, _U64, _P])
# partitioned finish (each rank ranks / emits its own segment; include/eulerhip.h)
eulerhip.register("ec_graph_chains_part", ctypes.c_int, [_P, _U64, _U64, _P, _P, ctypes.POINTER(_U64)])
eulerhip.register("ec_graph_rank_supers", ctypes.c_int, [_P, _P, _U64])
eulerhip.register("ec_graph_starts_part", ctypes.c_int, [_P, ctypes.c_int, _P, ctypes.POINTER(_U64)])
eulerhip.register("ec_graph_layout", ctypes.c_int, [_P, _P, _U64, ctypes.POINTER(_U64)])
eulerhip.register("ec_graph_emit_part", ctypes.c_int, [_P, _P, _P])
eulerhip.register("ec_graph_collect", ctypes.c_int, [_P, _P, _P, _U64])
eulerhip.register("ec_graph_emit_runs", ctypes.c_int, [_P, ctypes.POINTER(_U64)])
eulerhip.register("ec_graph_copy_runs", ctypes.c_int, [_P, _P])
eulerhip.register("ec_graph_collect_runs", ctypes.c_int, [_P, _P, ctypes.c_int, ctypes.POINTER(_U64), _U64])
eulerhip.register("ec_end_record_bytes", ctypes.c_int, [ctypes.c_int])
# exact-size outputs: the steps called with a NULL output count, the copies write (round 6)
eulerhip.register("ec_graph_place_copy", ctypes.c_int, [_P, _P])
eulerhip.register("ec_graph_chains_copy", ctypes.c_int, [_P, _P])
eulerhip.register("ec_graph_starts_copy", ctypes.c_int, [_P, _P])
# junction-partitioned graph (round 5, csrc/junction.h): no rank holds the job's solid set
eulerhip.register("ec_graph_place", ctypes.c_int, [_P, _U64, _U64, ctypes.c_int, _P, ctypes.POINTER(_U64),
                                                   ctypes.POINTER(_U64)])
eulerhip.register("ec_graph_join", ctypes.c_int, [_P, _P, _U64, ctypes.c_int, ctypes.POINTER(_U64), _P,
                                                  ctypes.POINTER(_U64)])
eulerhip.register("ec_graph_links_apply", ctypes.c_int, [_P, _P, _U64])
eulerhip.register("ec_junction_record_bytes", ctypes.c_int, [ctypes.c_int])
eulerhip.register("ec_link_record_bytes", ctypes.c_int, [])
LINK_BYTES = 8  # ec_link_record_bytes()


def junction_bytes(k):
    """ec_junction_record_bytes: RecJ64 (k <= 32) / RecJ"""
    return 16 if k <= 32 else 24


def end_bytes(k):
    """ec_end_record_bytes: one contig-end k-mer code"""
    return 8 if k <= 32 else 16
eulerhip.register("ec_super_record_bytes", ctypes.c_int, [])
eulerhip.register("ec_start_record_bytes", ctypes.c_int, [])
SUPER_BYTES = 32  # ec_super_record_bytes()
START_BYTES = 48  # ec_start_record_bytes()


def shard_range(nreads, rank, world):
    """Contiguous read shard of `rank` (first nreads % world ranks get one extra read)."""
    q, r = divmod(nreads, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


# a shard count past this fraction of the device's memory is released after its export
TRIM_FRACTION = 0.1
TRIM_FREE_FRACTION = 0.15


# ---- engines -------------------------------------------------------------------------------
class HipEngine:
    """The product engine: libeulerhip.so on this rank's GPU, buffers are torch uint8 tensors."""

    def __init__(self, device, stream=None):
        import torch

        self.torch = torch
        self.device = torch.device("cuda", device)
        self._total = None  # device memory (trim_if_large)
        # default: torch's current stream, so the engine's kernels are ordered after the torch
        # ops that produce its inputs (slices, concatenations, RCCL outputs)
        if stream is None:
            stream = torch.cuda.current_stream(self.device).cuda_stream
        self.sess = eulerhip.Session(device, stream=stream)
        self.L = eulerhip.lib()

    def _h(self):
        return self.sess._h

    def empty(self, nbytes):
        return self.torch.empty(max(int(nbytes), 1), dtype=self.torch.uint8, device=self.device)

    def _retry_nomem(self, call):
        """a call that ran out of device memory runs once more after the session's and torch's
        cached buffers are released (the count and the merge start from scratch: re-runnable)"""
        try:
            eulerhip.check(call())
        except eulerhip.EulerHipError as e:
            if e.code != eulerhip.EC_ERR_NOMEM:
                raise
            self.sess.trim(0)
            self.torch.cuda.empty_cache()
            eulerhip.check(call())

    def count_shard(self, d_reads, d_off, nreads, read_base, k, flags=0):
        self.k = int(k)
        self._retry_nomem(lambda: self.L.ec_count_shard(self._h(), ctypes.c_void_p(d_reads.data_ptr()),
                                                        ctypes.c_void_p(d_off.data_ptr()), int(nreads),
                                                        int(read_base), int(k), flags))
        return self.sess.stats()

    def rec_bytes(self):
        return int(self.L.ec_record_bytes(self.k))

    def trim_if_large(self, frac=TRIM_FRACTION, free_frac=TRIM_FREE_FRACTION):
        """before the count and after the export: a session holding more than frac of the device's
        memory releases its buffers (ec_session_trim) when less than free_frac of the device is
        free (torch's cached blocks counted free), so the next phase gets them.  A session that
        fits is kept: its buffers are the next phase's / step's at their sizes already, and large
        buffers freed and allocated again are slow -- config 5's per-rank step freeing ~165 GB
        before its count measured 5.6 s of count against 67 ms without (r06_f)"""
        torch = self.torch
        held = self.sess.device_bytes()
        if self._total is None:
            self._total = torch.cuda.get_device_properties(self.device).total_memory
        if held <= frac * self._total:  # (the common case decided without a device query)
            return False
        free, total = torch.cuda.mem_get_info(self.device)
        free += torch.cuda.memory_reserved(self.device) - torch.cuda.memory_allocated(self.device)
        if free < free_frac * total:
            self.sess.trim(64 << 20)
            self.torch.cuda.empty_cache()  # (and torch's cached blocks: the next allocations are the session's)
            return True
        return False

    def owner_counts(self, nowners):
        """records per owner under the current rule (no export; the owner ids are kept for it)"""
        counts = (ctypes.c_uint64 * nowners)()
        eulerhip.check(self.L.ec_export_by_owner(self._h(), int(nowners), None, counts))
        return [int(c) for c in counts]

    def set_owner_rule(self, rule):
        eulerhip.check(self.L.ec_session_set_owner_rule(self._h(), int(rule)))

    def export_by_owner(self, nowners, compact=False):
        """records grouped by owner and the records per owner; compact=True: also the records'
        lf_bits (compact_bytes(k)-B records with shard-relative events, or -1: full records)"""
        n = int(self.L.ec_dense_count(self._h()))
        rb = self.rec_bytes()
        counts = (ctypes.c_uint64 * nowners)()
        out = self.empty(n * rb)
        if not compact:
            eulerhip.check(self.L.ec_export_by_owner(self._h(), int(nowners), ctypes.c_void_p(out.data_ptr()), counts))
            return out[: n * rb], [int(c) for c in counts]
        lfb = ctypes.c_int(-1)
        eulerhip.check(self.L.ec_export_by_owner_ex(self._h(), int(nowners), ctypes.c_void_p(out.data_ptr()), counts, 1,
                                                    ctypes.byref(lfb)))
        rb = compact_bytes(self.k) if lfb.value >= 0 else rb
        return out[: n * rb], [int(c) for c in counts], int(lfb.value)

    def merge_owned_from(self, recs, src_bytes, src_base, src_lfb, k, limit, flags=0, export=True):
        """ec_merge_owned_from on the records of every source (rank order); export as merge_owned"""
        self.k = int(k)
        ns = len(src_bytes)
        self._retry_nomem(lambda: self.L.ec_merge_owned_from(
            self._h(), ctypes.c_void_p(recs.data_ptr()), ns, (ctypes.c_uint64 * ns)(*[int(x) for x in src_bytes]),
            (ctypes.c_int64 * ns)(*[int(x) for x in src_base]), (ctypes.c_int32 * ns)(*[int(x) for x in src_lfb]),
            int(k), int(limit), flags))
        m = int(self.L.ec_dense_count(self._h()))
        if not export:
            return m
        rb = self.rec_bytes()
        out = self.empty(m * rb)
        eulerhip.check(self.L.ec_export_dense(self._h(), ctypes.c_void_p(out.data_ptr())))
        return out[: m * rb]

    def merge_owned(self, recs, k, limit, flags=0, export=True):
        """ec_merge_owned_export: merge + solid filter + export in one call into a buffer
        sized for every received record (an upper bound of the solid ones).  export=False
        (the junction-partitioned graph): ec_merge_owned only, returns the solid count"""
        self.k = int(k)
        rb = self.rec_bytes()
        n = recs.numel() // rb
        if not export:
            eulerhip.check(self.L.ec_merge_owned(self._h(), ctypes.c_void_p(recs.data_ptr()), n, int(k), int(limit),
                                                 flags))
            return int(self.L.ec_dense_count(self._h()))
        out = self.empty(n * rb)
        eulerhip.check(self.L.ec_merge_owned_export(self._h(), ctypes.c_void_p(recs.data_ptr()), n, int(k),
                                                    int(limit), flags, ctypes.c_void_p(out.data_ptr())))
        m = int(self.L.ec_dense_count(self._h()))
        return out[: m * rb]

    def assemble_from_solid(self, recs, k, flags=0, fetch=True):
        self.k = int(k)
        n = recs.numel() // self.rec_bytes()
        eulerhip.check(self.L.ec_assemble_from_solid(self._h(), ctypes.c_void_p(recs.data_ptr()), n, int(k), flags))
        return self.sess.fetch(k) if fetch else None

    # partitioned graph phase: ec_graph_load / ec_graph_links_part / ec_graph_finish
    def graph_load(self, recs, k, flags=0):
        self.k = int(k)
        n = recs.numel() // self.rec_bytes()
        eulerhip.check(self.L.ec_graph_load(self._h(), ctypes.c_void_p(recs.data_ptr()), n, int(k), flags))
        return int(self.L.ec_dense_count(self._h()))

    def graph_load_links(self, recs, k, lo, hi, out, flags=0):
        """graph_load + graph_links_part in one call (ec_graph_load_links)"""
        self.k = int(k)
        n = recs.numel() // self.rec_bytes()
        eulerhip.check(self.L.ec_graph_load_links(self._h(), ctypes.c_void_p(recs.data_ptr()), n, int(k), flags,
                                                  int(lo), int(hi), ctypes.c_void_p(out.data_ptr())))
        return int(self.L.ec_dense_count(self._h()))

    def graph_links_part(self, lo, hi, out):
        """successors (uint32) of the oriented nodes of canonical ids [lo, hi) into `out`"""
        eulerhip.check(self.L.ec_graph_links_part(self._h(), int(lo), int(hi), ctypes.c_void_p(out.data_ptr())))

    def graph_finish(self, succ, k, flags=0, fetch=True):
        """fetch = False: the results stay in the session's pinned host buffers (as after
        ec_assemble_device); engine.sess.fetch(k) copies them out later"""
        eulerhip.check(self.L.ec_graph_finish(self._h(), ctypes.c_void_p(succ.data_ptr()), flags))
        return self.sess.fetch(k) if fetch else None

    # partitioned finish: ec_graph_chains_part .. ec_graph_collect
    # junction-partitioned graph: ec_graph_place / ec_graph_join / ec_graph_links_apply
    def graph_place(self, lo, U, nowners):
        """this rank's merged segment at global ids [lo, lo + Ur); returns (junction records
        grouped by owner, records per owner, palindromic keys of the segment)"""
        jb = junction_bytes(self.k)
        counts = (_U64 * nowners)()
        npal = _U64(0)
        # counted first, then copied into a buffer of exactly that size (not the 4 Ur bound)
        eulerhip.check(self.L.ec_graph_place(self._h(), int(lo), int(U), int(nowners), None, counts,
                                             ctypes.byref(npal)))
        tot = sum(int(c) for c in counts)
        out = self.empty(tot * jb)
        eulerhip.check(self.L.ec_graph_place_copy(self._h(), ctypes.c_void_p(out.data_ptr())))
        return out[: tot * jb], [int(c) for c in counts], int(npal.value)

    def graph_join(self, recs, seg_lo):
        """the links of the junctions this rank owns (recs: every record it received); returns
        (link records of other ranks' nodes grouped by rank, records per rank)"""
        nowners = len(seg_lo) - 1
        n = recs.numel() // junction_bytes(self.k)
        out = self.empty(n * LINK_BYTES)
        counts = (_U64 * nowners)()
        bounds = (_U64 * len(seg_lo))(*[int(x) for x in seg_lo])
        eulerhip.check(self.L.ec_graph_join(self._h(), ctypes.c_void_p(recs.data_ptr()), n, int(nowners), bounds,
                                            ctypes.c_void_p(out.data_ptr()), counts))
        tot = sum(int(c) for c in counts)
        return out[: tot * LINK_BYTES], [int(c) for c in counts]

    def graph_links_apply(self, links):
        eulerhip.check(self.L.ec_graph_links_apply(self._h(), ctypes.c_void_p(links.data_ptr()),
                                                   links.numel() // LINK_BYTES))

    def graph_chains_part(self, lo, hi, succ_part=None):
        """this rank's chains as super records (uint8 tensor of n * SUPER_BYTES) and n
        (succ_part None: a placed segment, whose links the session holds)"""
        n = ctypes.c_uint64(0)
        sp = ctypes.c_void_p(succ_part.data_ptr()) if succ_part is not None else None
        eulerhip.check(self.L.ec_graph_chains_part(self._h(), int(lo), int(hi), sp, None, ctypes.byref(n)))
        out = self.empty(n.value * SUPER_BYTES)
        eulerhip.check(self.L.ec_graph_chains_copy(self._h(), ctypes.c_void_p(out.data_ptr())))
        return out[: n.value * SUPER_BYTES], int(n.value)

    def graph_rank_supers(self, supers, n):
        eulerhip.check(self.L.ec_graph_rank_supers(self._h(), ctypes.c_void_p(supers.data_ptr()), int(n)))

    def graph_starts_part(self, have_supers, lo, hi):
        n = ctypes.c_uint64(0)
        eulerhip.check(self.L.ec_graph_starts_part(self._h(), 1 if have_supers else 0, None, ctypes.byref(n)))
        out = self.empty(n.value * START_BYTES)
        eulerhip.check(self.L.ec_graph_starts_copy(self._h(), ctypes.c_void_p(out.data_ptr())))
        return out[: n.value * START_BYTES], int(n.value)

    def graph_layout(self, starts, n):
        nchars = ctypes.c_uint64(0)
        eulerhip.check(self.L.ec_graph_layout(self._h(), ctypes.c_void_p(starts.data_ptr()), int(n),
                                              ctypes.byref(nchars)))
        return int(nchars.value)

    def graph_emit_part(self, chars, ends):
        eulerhip.check(self.L.ec_graph_emit_part(self._h(), ctypes.c_void_p(chars.data_ptr()),
                                                 ctypes.c_void_p(ends.data_ptr())))

    def graph_collect(self, chars, ends, k, npal, fetch=True):
        """npal: the job's palindromic solid k-mers (n_dict = 2 U - npal)"""
        eulerhip.check(self.L.ec_graph_collect(self._h(), ctypes.c_void_p(chars.data_ptr()),
                                               ctypes.c_void_p(ends.data_ptr()), int(npal)))
        return self.sess.fetch(k) if fetch else None

    def graph_emit_runs(self):
        """this rank's emission as one transfer record (uint8 tensor): the runs of character
        positions it wrote, their characters and its contig ends (ec_graph_emit_runs / copy_runs)"""
        n = _U64(0)
        eulerhip.check(self.L.ec_graph_emit_runs(self._h(), ctypes.byref(n)))
        out = self.empty(n.value)
        eulerhip.check(self.L.ec_graph_copy_runs(self._h(), ctypes.c_void_p(out.data_ptr())))
        return out[: n.value]

    def graph_collect_runs(self, recs, src_bytes, k, npal, fetch=True):
        """the collecting rank: every rank's transfer record (rank order) -> the job's results"""
        ns = len(src_bytes)
        eulerhip.check(self.L.ec_graph_collect_runs(self._h(), ctypes.c_void_p(recs.data_ptr()), ns,
                                                    (_U64 * ns)(*[int(x) for x in src_bytes]), int(npal)))
        return self.sess.fetch(k) if fetch else None

    def zeros(self, nbytes):
        return self.torch.zeros(max(int(nbytes), 1), dtype=self.torch.uint8, device=self.device)

    def stats(self):
        return self.sess.stats()


# ---- communicators ---------------------------------------------------------------------------
class TorchComm:
    """torch.distributed collectives (backend "nccl" = RCCL over xGMI on MI355X, or gloo)."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist

        self.torch, self.dist, self.group = torch, dist, group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        # gloo moves host tensors only: device tensors are staged through host memory (a
        # multi-process test of HipEngines sharing one GPU; RCCL takes device tensors as they are)
        self.stage = dist.get_backend(group) == "gloo"

    def _h(self, t):
        return t.cpu() if self.stage and t.is_cuda else t

    def _d(self, t, dev):
        return t.to(dev) if self.stage and dev.type == "cuda" else t

    def alltoallv(self, send, counts_bytes, tag=0, meta=None):
        """send: uint8 tensor laid out destination-major with counts_bytes[d] bytes for rank d.
        Returns (received bytes, sum over ranks of `tag`): the per-rank integer rides along with
        the byte-count exchange, so no separate all-reduce (and host sync) is needed for it.
        meta (a list of ints): rides along too; then also returns every source's byte count
        and meta list (rank order)."""
        torch, dist = self.torch, self.dist
        dev = send.device
        cdev = "cpu" if self.stage else dev
        m = [int(x) for x in (meta or [])]
        sc = torch.tensor([[int(c), int(tag)] + m for c in counts_bytes], dtype=torch.int64, device=cdev)
        rc = torch.empty_like(sc)
        dist.all_to_all_single(rc, sc, group=self.group)
        rcv = rc.tolist()
        rcl = [int(x[0]) for x in rcv]
        total_tag = sum(int(x[1]) for x in rcv)
        recv = torch.empty(max(sum(rcl), 1), dtype=torch.uint8, device=cdev)
        if sum(rcl) or sum(counts_bytes):
            dist.all_to_all_single(recv[: sum(rcl)], self._h(send[: sum(counts_bytes)]), output_split_sizes=rcl,
                                   input_split_sizes=list(counts_bytes), group=self.group)
        recv = self._d(recv[: sum(rcl)], dev)
        if meta is not None:
            return recv, total_tag, rcl, [[int(v) for v in x[2:]] for x in rcv]
        return recv, total_tag

    def allgatherv(self, t, fill=0, with_sizes=False, sizes=None):
        """Concatenation of every rank's `t` in rank order, each part padded with `fill` bytes
        to the largest part (no compaction copy: the record consumers skip all-0xFF filler
        records, ec_assemble_from_solid).  with_sizes: also return every rank's byte count.
        sizes: every rank's byte count when the caller knows them already (no size exchange,
        no host round trip)."""
        torch, dist = self.torch, self.dist
        if self.world == 1:
            return (t, [t.numel()]) if with_sizes else t
        cdev = "cpu" if self.stage else t.device
        if sizes is not None:
            szl = [int(x) for x in sizes]
            assert szl[self.rank] == t.numel(), "allgatherv: this rank's size differs from sizes[rank]"
        else:
            n = torch.tensor([t.numel()], dtype=torch.int64, device=cdev)
            sz = torch.empty(self.world, dtype=torch.int64, device=cdev)
            dist.all_gather_into_tensor(sz, n, group=self.group)
            szl = [int(x) for x in sz.tolist()]
        mx = max(max(szl), 1)
        pad = torch.full((mx,), fill, dtype=torch.uint8, device=cdev)
        pad[: t.numel()] = self._h(t)
        out = torch.empty(self.world * mx, dtype=torch.uint8, device=cdev)
        dist.all_gather_into_tensor(out, pad, group=self.group)
        out = self._d(out, t.device)
        return (out, szl) if with_sizes else out

    def allgather_int(self, v):
        """every rank's integer v, in rank order (one small all-gather)"""
        if self.world == 1:
            return [int(v)]
        dev = "cuda" if self.dist.get_backend(self.group) == "nccl" else "cpu"
        t = self.torch.tensor([int(v)], dtype=self.torch.int64, device=dev)
        out = self.torch.empty(self.world, dtype=self.torch.int64, device=dev)
        self.dist.all_gather_into_tensor(out, t, group=self.group)
        return [int(x) for x in out.tolist()]

    def reduce_sum(self, t, dst=0):
        """element-wise sum of every rank's uint8 tensor `t` into rank dst's (in place); the
        partitioned finish's characters / contig ends, each byte set by exactly one rank"""
        if self.world > 1:
            h = self._h(t)
            self.dist.reduce(h, dst=dst, op=self.dist.ReduceOp.SUM, group=self.group)
            if h is not t:
                t.copy_(h)
        return t

    def allreduce_vec(self, vals):
        """element-wise sum over the ranks of a list of integers"""
        dev = "cuda" if self.dist.get_backend(self.group) == "nccl" else "cpu"
        t = self.torch.tensor([int(v) for v in vals], dtype=self.torch.int64, device=dev)
        self.dist.all_reduce(t, group=self.group)
        return [int(x) for x in t.tolist()]

    def allreduce_sum(self, v):
        dev = "cuda" if self.dist.get_backend(self.group) == "nccl" else "cpu"
        t = self.torch.tensor([int(v)], dtype=self.torch.int64, device=dev)
        self.dist.all_reduce(t, group=self.group)
        return int(t.item())

    def barrier(self):
        self.dist.barrier(group=self.group)


# ---- the orchestration -----------------------------------------------------------------------
def _gather_concat(comm, t, nbytes_each=None):
    """all-gather of variable-size uint8 parts, padding dropped (rank order); returns (tensor, sizes)"""
    g, sz = comm.allgatherv(t, fill=0, with_sizes=True)
    if comm.world == 1:
        return g, sz
    mx = max(max(sz), 1)
    return comm.torch.cat([g[r * mx: r * mx + sz[r]] for r in range(comm.world)]), sz


def junction_links(engine, comm, k, ur, tick=None):
    """The junction-partitioned graph (csrc/junction.h): this rank's merged segment (ur keys)
    placed at its global ids, the (k-1)-mer junction records exchanged by junction owner (one
    all-to-all-v; with minimizer owners nearly all stay local), the links of the owned
    junctions joined, the other ranks' link records exchanged (a second all-to-all-v) and
    applied.  No rank holds the job's solid set.  Returns (lo, hi, U, job palindromes)."""
    tick = tick or (lambda name: None)
    sizes = comm.allgather_int(ur)
    lo = sum(sizes[: comm.rank])
    U = sum(sizes)
    seg_lo = [sum(sizes[:r]) for r in range(comm.world + 1)]
    jrecs, jcounts, npal = engine.graph_place(lo, U, comm.world)
    jb = junction_bytes(k)
    recv, npal_job = comm.alltoallv(jrecs, [c * jb for c in jcounts], tag=npal)  # (the palindromes ride along)
    tick("place")
    links, lcounts = engine.graph_join(recv, seg_lo)
    lrecv, _ = comm.alltoallv(links, [c * LINK_BYTES for c in lcounts])
    engine.graph_links_apply(lrecv)
    tick("join")
    return lo, lo + ur, U, npal_job


def partitioned_finish(engine, comm, k, lo, hi, part, fetch=True, tick=None, npal=None):
    """The graph finish with every rank ranking / emitting its own segment (ec_graph_chains_part ..
    ec_graph_collect): all-gathers of the chains' super records (~1/9 of the nodes on the
    super-k-mer path) and of the contig starts, then each rank's transfer record -- the runs of
    character positions it wrote and the contig ends it holds -- gathered to rank 0 (round 5
    reduced job-sized character and end buffers there; engines without graph_emit_runs still
    do).  part None: a placed segment (junction_links), npal its job palindromes.  Returns rank
    0's result (None elsewhere)."""
    tick = tick or (lambda name: None)
    sup, _ = engine.graph_chains_part(lo, hi, part)
    tick("chains")
    supers, _ = _gather_concat(comm, sup)
    M = supers.numel() // SUPER_BYTES
    engine.graph_rank_supers(supers, M)
    tick("rank")
    st, _ = engine.graph_starts_part(M > 0, lo, hi)
    starts, _ = _gather_concat(comm, st)
    nc = starts.numel() // START_BYTES
    nchars = engine.graph_layout(starts, nc)
    tick("starts")
    if hasattr(engine, "graph_emit_runs"):
        # each rank's own characters (runs of positions it wrote) and contig ends, gathered to
        # rank 0 (an all-to-all-v with every other destination empty): no job-sized buffer
        rec = engine.graph_emit_runs()
        recv, _, rcl, _ = comm.alltoallv(rec, [rec.numel() if d == 0 else 0 for d in range(comm.world)], meta=[])
        tick("emit")
        res = engine.graph_collect_runs(recv, rcl, k, npal, fetch=fetch) if comm.rank == 0 else None
        tick("collect")
        return res
    # (engines without the transfer records: job-sized buffers reduced to rank 0)
    chars = engine.zeros(nchars)
    ends = engine.zeros(max(2 * nc * end_bytes(k), 8))
    engine.graph_emit_part(chars, ends)
    comm.reduce_sum(chars)
    comm.reduce_sum(ends)
    tick("emit")
    res = engine.graph_collect(chars, ends, k, npal, fetch=fetch) if comm.rank == 0 else None
    tick("collect")
    return res


def finish_mode(finish, k, rule):
    """"auto": the partitioned finish where the gathered ids have minimizer locality (21 <= k <=
    52 on minimizer owners: a segment's chains are a fraction of its nodes; 128-bit keys since
    round 5, the owner merge emitting its set in minimizer order), else the replicated one (on
    hash-ordered ids every node is its own chain and the all-gathered chain records would
    outweigh the successor array 8 : 1)"""
    if finish != "auto":
        return finish
    return "partitioned" if minimizer_owners(k) and rule == OWNER_MINIMIZER else "replicated"


def sharded_assemble(engine, comm, d_reads, d_off, nreads, read_base, k, limit=1, flags=0, on_count=None,
                     phase_ms=None, partitioned=None, fetch=True, finish="auto"):
    """Run steps 1-4 for this rank; returns (result, n_positions_total).  on_count(stats)
    receives the shard-count statistics (per-kernel times with EC_FLAG_TIMING); phase_ms, a
    dict, receives the wall time of every step (device-synchronised by the engine calls).
    fetch = False: the result stays in the engine's session (result None; bench.py, like the
    single-GPU step, which ends with the results in pinned host buffers).
    partitioned (default, unless EC_FLAG_GENERAL): each rank computes the successor links of its own owner
    segment of the gathered solid set only ("each GPU builds its local graph partition").
    finish "partitioned" (the "auto" choice where the ids have minimizer locality): every rank
    ranks / emits its own segment and ONLY RANK 0 returns the result (None on the others);
    "replicated": the successor parts are all-gathered and every rank returns the result.  An
    engine without graph_place runs the replicated finish for "partitioned" too (with a
    RuntimeWarning), and then every rank returns the result."""
    import time

    if partitioned is None:
        partitioned = hasattr(engine, "graph_load") and not (flags & eulerhip.EC_FLAG_GENERAL)
    marks = [("start", time.perf_counter())]

    def tick(name):
        marks.append((name, time.perf_counter()))

    if hasattr(engine, "trim_if_large"):  # (a large previous step's graph buffers: the count needs the memory)
        engine.trim_if_large()
    st = engine.count_shard(d_reads, d_off, nreads, read_base, k, flags)
    tick("count")
    if on_count:
        on_count(st)
    rule = OWNER_MINIMIZER
    if comm.world > 1 and minimizer_owners(k):  # one owner rule for every rank, from the job's counts
        engine.set_owner_rule(OWNER_MINIMIZER)
        rule = owner_rule_for(comm.allreduce_vec(engine.owner_counts(comm.world)), k)
        if rule != OWNER_MINIMIZER:
            engine.set_owner_rule(rule)
    finish = finish_mode(finish, k, rule)
    # compact records where the events fit (the receivers add this shard's read base)
    recs, counts, lfb = engine.export_by_owner(comm.world, compact=True)
    rb = compact_bytes(k) if lfb >= 0 else rec_bytes(k)
    if hasattr(engine, "trim_if_large"):
        engine.trim_if_large()
    tick("export")
    # the job's k-mer positions, this shard's read base and record format ride along with the
    # exchange's byte counts
    received, P, src_bytes, metas = comm.alltoallv(recs, [c * rb for c in counts], tag=st.n_positions,
                                                   meta=[read_base, lfb])
    src_base, src_lfb = [m[0] for m in metas], [m[1] for m in metas]
    del recs  # (the send buffer: its memory goes to the merge)
    tick("alltoall")
    junction = partitioned and finish == "partitioned" and hasattr(engine, "graph_place")
    if partitioned and finish == "partitioned" and not junction:
        # (an engine without the junction steps cannot keep only its segment: the replicated
        # finish below gives the same result, and every rank returns it)
        import warnings

        warnings.warn("sharded_assemble: the engine cannot place segments (no graph_place); "
                      "finish='partitioned' runs the replicated finish", RuntimeWarning, stacklevel=2)
    if junction:  # each rank keeps its own segment: the links come out of the junction join
        ur = engine.merge_owned_from(received, src_bytes, src_base, src_lfb, k, limit, flags, export=False)
        del received
        tick("merge")
        lo, hi, _, npal = junction_links(engine, comm, k, ur, tick=tick)
        res = partitioned_finish(engine, comm, k, lo, hi, None, fetch=fetch, tick=tick, npal=npal)
        if phase_ms is not None:
            for (_, a), (name, b) in zip(marks, marks[1:]):
                phase_ms[name] = phase_ms.get(name, 0.0) + (b - a) * 1e3
        return res, P
    solid = engine.merge_owned_from(received, src_bytes, src_base, src_lfb, k, limit, flags)
    tick("merge")
    if not partitioned:
        everything = comm.allgatherv(solid, fill=0xFF)  # filler records: all-ones keys, skipped
        tick("allgather")
        res = engine.assemble_from_solid(everything, k, flags, fetch=fetch)
        tick("graph")
    else:
        everything, sizes = comm.allgatherv(solid, fill=0xFF, with_sizes=True)
        tick("allgather")
        nrec = [sz // rec_bytes(k) for sz in sizes]
        lo = sum(nrec[: comm.rank])
        hi = lo + nrec[comm.rank]
        part = engine.empty(8 * (hi - lo))
        if hasattr(engine, "graph_load_links"):  # one call: no host round trip in between
            engine.graph_load_links(everything, k, lo, hi, part, flags)
            tick("load_links")
        else:
            engine.graph_load(everything, k, flags)
            tick("load")
            engine.graph_links_part(lo, hi, part)
            tick("links")
        # replicated finish: the successor parts all-gathered, every rank ranks / emits everything
        # (every rank's part size is known from the solid-set sizes: no size exchange)
        gathered, psz = comm.allgatherv(part[: 8 * (hi - lo)], fill=0xFF, with_sizes=True,
                                        sizes=[8 * x for x in nrec])
        if comm.world > 1:  # drop the padding: node order = rank order
            mx = max(max(psz), 1)
            succ = comm.torch.cat([gathered[r * mx: r * mx + psz[r]] for r in range(comm.world)])
        else:
            succ = gathered
        tick("gather_links")
        res = engine.graph_finish(succ, k, flags, fetch=fetch)
        tick("graph")
    if phase_ms is not None:
        for (_, a), (name, b) in zip(marks, marks[1:]):
            phase_ms[name] = phase_ms.get(name, 0.0) + (b - a) * 1e3
    return res, P


class ShardedAssembler:
    """bench.py / CLI front-end: this rank's shard of a read set already in host memory is
    moved to its GPU once; run() performs one full distributed assembly."""

    def __init__(self, buf, off, k, limit, rank, world, local_rank, comm=None, read_base=None):
        """read_base None: (buf, off) is the whole read set and this rank takes its contiguous
        shard; otherwise (buf, off) is this rank's shard already, its first read being global
        read read_base (the ranks' shards in rank order form the job's read set)."""
        import torch

        if read_base is None:
            lo, hi = shard_range(len(off) - 1, rank, world)
        else:
            lo, hi = 0, len(off) - 1
        b0, b1 = int(off[lo]), int(off[hi])
        self.nreads = hi - lo
        self.read_base = lo if read_base is None else int(read_base)
        self.k, self.limit = k, limit
        self.d_reads = torch.from_numpy(np.ascontiguousarray(buf[b0:b1])).to(f"cuda:{local_rank}")
        self.d_off = torch.from_numpy((off[lo:hi + 1] - off[lo]).astype(np.int64)).to(f"cuda:{local_rank}")
        torch.cuda.synchronize()
        self.engine = HipEngine(local_rank, stream=torch.cuda.current_stream().cuda_stream)
        self.comm = comm or TorchComm()
        self.total_positions = 0
        self.result = None
        self.phase_ms = {}

    def run(self, timing=False, fetch=True):
        """timing: True = EC_FLAG_TIMING, or the timing flag bits to pass (EC_FLAG_KERNEL_TIMING)"""
        flags = eulerhip.EC_FLAG_TIMING if timing is True else int(timing or 0)
        self.result, self.total_positions = sharded_assemble(self.engine, self.comm, self.d_reads, self.d_off,
                                                             self.nreads, self.read_base, self.k, self.limit, flags,
                                                             on_count=self._keep, phase_ms=self.phase_ms, fetch=fetch)
        return self.result

    def _keep(self, st):
        self.count_stats = st

    def stats(self):
        """counting-phase statistics of this rank's shard (kernel_ms / stage_ms)"""
        return self.count_stats


def streaming_assemble(engine, buf, off, k, limit=1, chunk_reads=4_000_000, fold=4, read_base=0, flags=0,
                       stats=None):
    """Out-of-core count on one GPU for read sets whose one-shot count does not fit its memory
    (BASELINE config 5 on fewer than 8 GPUs, larger genomes; the reference's chunk loop,
    src/eulercuda.py:99-119, never finished).  The reads (host arrays: buf, uint64 offsets) go
    through the shard count chunk_reads at a time -- each chunk's distinct k-mers exported with
    their counts and first events (compact records, events relative to the chunk), the count's
    buffers released -- and every `fold` chunks the pending records are merged into one running
    set (counts summed, first events min'd, no filter: limit -1).  The last merge applies the
    solid filter; the graph (junction join), ranking and emission then run on the merged set as
    the one rank of the partitioned flow.  Events are global read ids from read_base, so the
    dict order, contigs and links equal the one-shot assembly's (tests: bit-exact vs the oracle
    at forced small chunks).  stats (a dict): chunks, folds, device-buffer peak, positions.
    Returns (result, k-mer positions)."""
    import torch

    dev = engine.device
    nreads = len(off) - 1
    chunk_reads = max(1, int(chunk_reads))
    k = int(k)
    P = 0
    running = None  # (records, lf_bits, read base) of the merged chunks so far
    pending = []
    nfold = 0
    nchunks = 0

    def merge(srcs, lim, export):
        recs = torch.cat([r for r, _, _ in srcs]) if len(srcs) > 1 else srcs[0][0]
        return engine.merge_owned_from(recs, [r.numel() for r, _, _ in srcs], [b for _, _, b in srcs],
                                       [f for _, f, _ in srcs], k, lim, flags, export=export)

    engine.set_owner_rule(OWNER_MINIMIZER)
    for c0 in range(0, max(nreads, 1), chunk_reads):
        c1 = min(nreads, c0 + chunk_reads)
        b0, b1 = int(off[c0]), int(off[c1])
        d_reads = torch.from_numpy(np.ascontiguousarray(buf[b0:b1]) if b1 > b0 else np.zeros(1, np.uint8)).to(dev)
        d_off = torch.from_numpy((np.asarray(off[c0:c1 + 1]) - off[c0]).astype(np.int64)).to(dev)
        st = engine.count_shard(d_reads, d_off, c1 - c0, read_base + c0, k, flags)
        P += st.n_positions
        recs, _, lfb = engine.export_by_owner(1, compact=True)
        del d_reads, d_off
        engine.sess.trim(64 << 20)  # (the count's buffers: the next chunk or the merge reuses the memory)
        pending.append((recs, lfb, read_base + c0 if lfb >= 0 else 0))
        nchunks += 1
        if len(pending) >= fold and c1 < nreads:  # fold the pending chunks into the running set
            merged = merge(([running] if running else []) + pending, -1, True)
            running = (merged, -1, 0)  # (full records, global events)
            pending = []
            nfold += 1
            engine.sess.trim(64 << 20)
    ur = merge(([running] if running else []) + pending, limit, False)
    running = None
    pending = []
    jrecs, _, npal = engine.graph_place(0, ur, 1)
    links, _ = engine.graph_join(jrecs, [0, ur])
    del jrecs
    engine.graph_links_apply(links)
    del links
    res = local_partitioned_finish([engine], [(0, ur, None)], k, npal)
    if stats is not None:
        stats.update(chunks=nchunks, folds=nfold, positions=P, solid=ur)
    return res, P


def local_sharded_assemble(engines, buf, off, k, limit=1, flags=0, partitioned=None, finish="auto", compact=True):
    """Simulate the distributed algorithm with len(engines) ranks on the local device(s):
    same engine calls, the collectives done by concatenation.  Returns rank 0's result."""
    world = len(engines)
    nreads = len(off) - 1
    parts = []
    for r in range(world):
        lo, hi = shard_range(nreads, r, world)
        b0, b1 = int(off[lo]), int(off[hi])
        parts.append((buf[b0:b1], off[lo:hi + 1] - off[lo], lo))
    return local_sharded_assemble_shards(engines, parts, k, limit, flags, partitioned, finish, compact)


def local_sharded_assemble_shards(engines, parts, k, limit=1, flags=0, partitioned=None, finish="auto", compact=True):
    """local_sharded_assemble on given shards: parts[r] = (buf, off, read_base) of rank r (host
    arrays; global read ids read_base.., increasing with r, gaps allowed).  compact: the
    exchange's record format per rank (a bool for all; compact records where events fit)."""
    import torch

    world = len(engines)
    shards = []
    for eng, (b, o, base) in zip(engines, parts):
        d_reads = torch.from_numpy(np.ascontiguousarray(b) if len(b) else np.zeros(1, np.uint8)).to(eng.device)
        d_off = torch.from_numpy(np.asarray(o).astype(np.int64)).to(eng.device)
        shards.append((d_reads, d_off, len(o) - 1, int(base)))
    P = 0
    sends = []
    for eng, (d_reads, d_off, n, lo) in zip(engines, shards):
        if hasattr(eng, "trim_if_large"):
            eng.trim_if_large()
        st = eng.count_shard(d_reads, d_off, n, lo, k, flags)
        eng.count_variant = int(st.count_variant)
        P += st.n_positions
    rule = OWNER_MINIMIZER
    if world > 1 and minimizer_owners(k):  # as sharded_assemble: the summed owner counts decide the rule
        for eng in engines:
            eng.set_owner_rule(OWNER_MINIMIZER)
        rule = owner_rule_for([sum(c) for c in zip(*[eng.owner_counts(world) for eng in engines])], k)
    comp = compact if isinstance(compact, (list, tuple)) else [compact] * world
    for eng, c in zip(engines, comp):
        eng.set_owner_rule(rule)
        sends.append(eng.export_by_owner(world, compact=True) if c else eng.export_by_owner(world) + (-1,))
        if hasattr(eng, "trim_if_large"):
            eng.trim_if_large()
    local_sharded_assemble_shards.last_rule = rule
    finish = finish_mode(finish, k, rule)
    local_sharded_assemble_shards.last_counts = [c for _, c, _ in sends]
    local_sharded_assemble_shards.last_lf_bits = [b for _, _, b in sends]
    rbs = [compact_bytes(k) if b >= 0 else rec_bytes(k) for _, _, b in sends]
    bases = [int(base) for _, _, base in parts]

    def merge(dst, eng, export):
        got = []
        for src in range(world):
            recs, counts, _ = sends[src]
            o = sum(counts[:dst]) * rbs[src]
            got.append(recs[o:o + counts[dst] * rbs[src]].to(eng.device))
        return eng.merge_owned_from(torch.cat(got) if world > 1 else got[0], [g.numel() for g in got], bases,
                                    [b for _, _, b in sends], k, limit, flags, export=export)

    if partitioned is None:
        partitioned = not (flags & eulerhip.EC_FLAG_GENERAL)
    if partitioned and finish == "partitioned":  # the junction-partitioned graph (junction_links)
        urs = [merge(dst, eng, False) for dst, eng in enumerate(engines)]
        sends.clear()  # (each exchange buffer is dropped once consumed: config 5's rank holds ~10^11 B)
        seg_lo = [sum(urs[:r]) for r in range(world + 1)]
        U = seg_lo[-1]
        placed = [eng.graph_place(seg_lo[r], U, world) for r, eng in enumerate(engines)]
        npal = sum(p[2] for p in placed)
        jb = junction_bytes(k)
        links = []
        for dst, eng in enumerate(engines):
            got = [rec[sum(c[:dst]) * jb:sum(c[:dst + 1]) * jb].to(eng.device) for rec, c, _ in placed]
            links.append(eng.graph_join(torch.cat(got) if len(got) > 1 else got[0], seg_lo))
            del got
        placed.clear()
        for dst, eng in enumerate(engines):
            got = [rec[sum(c[:dst]) * LINK_BYTES:sum(c[:dst + 1]) * LINK_BYTES].to(eng.device) for rec, c in links]
            eng.graph_links_apply(torch.cat(got))
        links.clear()
        segs = [(seg_lo[r], seg_lo[r + 1], None) for r in range(world)]
        return local_partitioned_finish(engines, segs, k, npal), P
    solids = [merge(dst, eng, True) for dst, eng in enumerate(engines)]
    rb = rec_bytes(k)
    mx = max(max(x.numel() for x in solids), 1)  # padded like TorchComm.allgatherv (0xFF filler records)
    allsolid = torch.full((world * mx,), 0xFF, dtype=torch.uint8, device=engines[0].device)
    for i, x in enumerate(solids):
        allsolid[i * mx: i * mx + x.numel()] = x.to(engines[0].device)
    if not partitioned:
        res = engines[0].assemble_from_solid(allsolid, k, flags)
        return res, P
    # partitioned links, replicated finish: every simulated rank loads the gathered set and
    # computes the links of its own segment; the parts are concatenated in rank order
    nrec = [x.numel() // rb for x in solids]
    parts = []
    for r, eng in enumerate(engines):
        lo = sum(nrec[:r])
        eng.graph_load(allsolid.to(eng.device), k, flags)
        part = eng.empty(8 * nrec[r])
        eng.graph_links_part(lo, lo + nrec[r], part)
        parts.append(part[: 8 * nrec[r]].to(engines[0].device))
    succ = torch.cat(parts) if parts else torch.empty(0, dtype=torch.uint8, device=engines[0].device)
    res = engines[0].graph_finish(succ if succ.numel() else engines[0].empty(4), k, flags)
    return res, P


def local_partitioned_finish(engines, segs, k, npal):
    """partitioned_finish with the collectives done by concatenation / summation (simulated ranks)"""
    import torch

    dev = engines[0].device
    sups = [eng.graph_chains_part(lo, hi, part)[0] for eng, (lo, hi, part) in zip(engines, segs)]
    supers = torch.cat([x.to(dev) for x in sups]) if len(sups) > 1 else sups[0]
    del sups
    M = supers.numel() // SUPER_BYTES
    for eng in engines:
        eng.graph_rank_supers(supers.to(eng.device), M)
    del supers
    sts = [eng.graph_starts_part(M > 0, lo, hi)[0] for eng, (lo, hi, _) in zip(engines, segs)]
    starts = torch.cat([x.to(dev) for x in sts])
    nc = starts.numel() // START_BYTES
    if hasattr(engines[0], "graph_emit_runs"):  # as partitioned_finish: transfer records gathered
        recs = []
        for eng in engines:
            eng.graph_layout(starts.to(eng.device), nc)
            recs.append(eng.graph_emit_runs().to(dev))
        sizes = [r.numel() for r in recs]
        allr = torch.cat(recs) if len(recs) > 1 else recs[0]
        del recs
        return engines[0].graph_collect_runs(allr, sizes, k, npal)
    chars, ends = None, None
    for eng in engines:
        nchars = eng.graph_layout(starts.to(eng.device), nc)
        c, e = eng.zeros(nchars), eng.zeros(max(2 * nc * end_bytes(k), 8))
        eng.graph_emit_part(c, e)
        chars = c.to(dev) if chars is None else chars + c.to(dev)
        ends = e.view(torch.int32).to(dev) if ends is None else ends + e.view(torch.int32).to(dev)
    return engines[0].graph_collect(chars, ends.view(torch.uint8), k, npal)
