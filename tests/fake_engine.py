"""CPU stand-in for distributed.HipEngine -- TEST INFRASTRUCTURE ONLY.

Lets tests drive the real multi-rank orchestration (distributed.sharded_assemble, TorchComm)
over the gloo backend on CPU.  Its compute comes from the design model (model_parallel.py),
which is pinned to the reference's golden vectors; the record layout and the owner function
are the device ones (ec_kmer_record, shard.h OwnerFn), so the exchange is byte-identical.
"""
import numpy as np
import torch

import bisect

from distributed import REC_BYTES, REC_DTYPE
from model_parallel import model_count, model_graph, twin

M64 = (1 << 64) - 1
CODE = {"A": 0, "C": 1, "G": 2, "T": 3}


def mix64(x):
    """common.h mix64"""
    x &= M64
    x ^= x >> 29
    x = (x * 0xbf58476d1ce4e5b9) & M64
    x ^= x >> 32
    return x


def owner_of(key, n):
    return ((mix64(key ^ 0xD6E8FEB86659FD93) >> 32) * n) >> 32


M32 = (1 << 32) - 1


def _rev2_32(x):
    x = ((x >> 2) & 0x33333333) | ((x & 0x33333333) << 2)
    x = ((x >> 4) & 0x0F0F0F0F) | ((x & 0x0F0F0F0F) << 4)
    return ((x >> 24) | ((x >> 8) & 0xFF00) | ((x << 8) & 0xFF0000) | (x << 24)) & M32


def _mmer_hash(x):
    x = (x * 0x9E3779B1) & M32
    return x ^ (x >> 15)


def _min_remix(x):
    """superkmer.h min_remix: rotate right by 14 (the minimum's uniform low bits on top)"""
    return ((x >> 14) | (x << 18)) & M32


def minimizer_of(c, k, m=15):
    """superkmer.h minimizer_of: min over the k-m+1 canonical m-mers of mmer_hash, remixed"""
    mm = (1 << (2 * m)) - 1
    v = M32
    for p in range(k - m + 1):
        f = (c >> (2 * (k - m - p))) & mm
        r = _rev2_32(f ^ mm) >> (32 - 2 * m)
        v = min(v, _mmer_hash(min(f, r)))
    return _min_remix(v)


def minimizer_of_w(c, k, m=15):
    """graph.h minimizer_of_w: minimizer of a 128-bit code c (< 4^k), remixed by min_remix_w"""
    mm = (1 << (2 * m)) - 1
    v = M32
    for p in range(k - m + 1):
        f = (c >> (2 * (k - m - p))) & mm
        r = _rev2_32(f ^ mm) >> (32 - 2 * m)
        v = min(v, _mmer_hash(min(f, r)))
    return ((v >> 20) | (v << 12)) & M32


def owner_fn(key, n, k, rule=0):
    """shard.h OwnerFn: the minimizer's range for 21 <= k <= 52 (rule 0), else the key hash
    (64-bit keys; the 128-bit key hash is wide.h owner_of_w, not restated here)"""
    if 21 <= k <= 32 and rule == 0:
        return (minimizer_of(key, k) * n) >> 32
    if 32 < k <= 52 and rule == 0:
        return (minimizer_of_w(key, k) * n) >> 32
    return owner_of(key, n)


def encode(s):
    v = 0
    for c in s:
        v = (v << 2) | CODE[c]
    return v


def decode(v, k):
    return "".join("ACGT"[(v >> (2 * (k - 1 - i))) & 3] for i in range(k))


class _Stats:
    def __init__(self, P):
        self.n_positions = P


class _Result:
    def __init__(self, d, contigs, links):
        self.dict_items, self.contigs, self.links = d, contigs, links


class FakeEngine:
    def __init__(self, k):
        self.k = k
        self.recs = np.zeros(0, REC_DTYPE)

    def _bytes(self, recs):
        return torch.from_numpy(np.frombuffer(recs.tobytes(), dtype=np.uint8).copy())

    def _recs(self, t):
        return np.frombuffer(t.numpy().tobytes(), dtype=REC_DTYPE)

    def count_shard(self, d_reads, d_off, nreads, read_base, k, flags=0):
        buf = d_reads.numpy().tobytes()
        off = d_off.numpy()
        reads = [buf[int(off[i]):int(off[i + 1])].decode() for i in range(nreads)]
        cnt, first = model_count(reads, k, read_base)
        P = sum(max(0, len(seg) - k + 1) for r in reads for seg in r.split("N"))
        out = np.zeros(len(cnt), REC_DTYPE)
        for i, (c, v) in enumerate(cnt.items()):
            out[i] = (encode(c), v, 0, first[c], first[twin(c)])
        self.recs = out
        return _Stats(P)

    rule = 0
    last_counts = None

    def set_owner_rule(self, rule):
        self.rule = rule

    def owner_counts(self, nowners):
        own = [owner_fn(int(x), nowners, self.k, self.rule) for x in self.recs["key"]]
        return [own.count(o) for o in range(nowners)]

    def export_by_owner(self, nowners, compact=False):
        """(compact: the device's compact records carry shard-relative events; this engine always
        sends full records, lf_bits -1, with global events -- the exchange's mixed-format case)"""
        own = np.array([owner_fn(int(x), nowners, self.k, self.rule) for x in self.recs["key"]], dtype=np.int64)
        order = np.argsort(own, kind="stable")
        counts = [int((own == o).sum()) for o in range(nowners)]
        self.last_counts = counts
        out = self._bytes(self.recs[order])
        return (out, counts, -1) if compact else (out, counts)

    def merge_owned_from(self, recs, src_bytes, src_base, src_lfb, k, limit, flags=0, export=True):
        assert all(b == -1 for b in src_lfb) and sum(src_bytes) == recs.numel()
        return self.merge_owned(recs, k, limit, flags, export)

    def merge_owned(self, recs, k, limit, flags=0, export=True):
        agg = {}
        for r in self._recs(recs):
            key = int(r["key"])
            c, a, b = agg.get(key, (0, 1 << 63, 1 << 63))
            agg[key] = (c + int(r["count"]), min(a, int(r["first_canon"])), min(b, int(r["first_twin"])))
        keep = [(key, c, a, b) for key, (c, a, b) in agg.items() if c > limit]
        out = np.zeros(len(keep), REC_DTYPE)
        for i, (key, c, a, b) in enumerate(keep):
            out[i] = (key, c, 0, a, b)
        self.recs = out
        return self._bytes(out) if export else len(out)

    def assemble_from_solid(self, recs, k, flags=0, fetch=True):
        cnt, first = {}, {}
        for r in self._recs(recs):
            if int(r["key"]) == M64:  # all-gather filler record (ec_assemble_from_solid skips it)
                continue
            c = decode(int(r["key"]), k)
            cnt[c] = int(r["count"])
            first[c] = int(r["first_canon"])
            first[twin(c)] = int(r["first_twin"]) if twin(c) != c else int(r["first_canon"])
        d, contigs, links = model_graph(cnt, first, k)
        return _Result(d, contigs, links)

    # ---- partitioned graph phase (distributed.sharded_assemble, k <= 32) ----------------------
    # restates k_links_part on the oriented nodes 2u+o of the gathered order (ec_graph_load ids)
    def empty(self, nbytes):
        return torch.zeros(max(int(nbytes), 1), dtype=torch.uint8)

    def graph_load(self, recs, k, flags=0):
        self.grecs = np.array([r for r in self._recs(recs) if int(r["key"]) != M64], dtype=REC_DTYPE)
        self.gid = {int(x): i for i, x in enumerate(self.grecs["key"])}
        self.gk = k
        return len(self.grecs)

    def _tw(self, x):
        return encode(twin(decode(x, self.gk)))

    def _node_code(self, x):
        c = int(self.grecs["key"][x >> 1])
        return self._tw(c) if x & 1 else c

    def _fw_present(self, xs):
        mask = (1 << (2 * self.gk)) - 1
        out = []
        for b in range(4):
            y = ((xs << 2) | b) & mask
            ty = self._tw(y)
            cy = min(y, ty)
            if cy in self.gid:
                out.append(2 * self.gid[cy] + (1 if y != cy else 0))
        return out

    def _succ_of(self, x):
        c = int(self.grecs["key"][x >> 1])
        pal = self._tw(c) == c
        if (x & 1) and pal:
            return 0xFFFFFFFF
        fw = self._fw_present(self._node_code(x))
        tx = x if pal else x ^ 1
        if len(fw) != 1 or fw[0] == tx:
            return 0xFFFFFFFF
        y = fw[0]
        yc = int(self.grecs["key"][y >> 1])
        tyn = y if self._tw(yc) == yc else y ^ 1
        return y if len(self._fw_present(self._node_code(tyn))) == 1 else 0xFFFFFFFF

    def graph_links_part(self, lo, hi, out):
        part = np.array([self._succ_of(x) for x in range(2 * lo, 2 * hi)], dtype=np.uint32)
        if part.size:
            out[: part.nbytes] = torch.from_numpy(part.view(np.uint8).copy())

    def graph_finish(self, succ, k, flags=0, fetch=True):
        got = np.frombuffer(succ.numpy().tobytes(), dtype=np.uint32)[: 2 * len(self.grecs)]
        want = np.array([self._succ_of(x) for x in range(2 * len(self.grecs))], dtype=np.uint32)
        assert np.array_equal(got, want), "gathered successor parts differ from the whole-set links"
        return self.assemble_from_solid(self._bytes(self.grecs), k, flags)


    # ---- junction-partitioned graph (distributed.junction_links; csrc/junction.h) ----------
    # RecJ64 {key u64, tag u32 = oriented global node | side << 31, pad u32 = palindrome flag},
    # LinkRec {node u32, value u32}; junction owners as JOwnerFn (the keys' rule on k - 1 bases)
    JREC = np.dtype([("key", "<u8"), ("tag", "<u4"), ("pad", "<u4")])
    LINK = np.dtype([("node", "<u4"), ("value", "<u4")])

    def _jowner(self, o, n):
        if 21 <= self.k <= 32 and self.rule == 0:
            return (minimizer_of(o, self.k - 1) * n) >> 32
        return owner_of(o, n)

    def graph_place(self, lo, U, nowners):
        k = self.k
        self.lo, self.U = lo, U
        self.seg = self.recs.copy()  # the merge's segment, global ids lo..
        self.succ_seg = {}
        recs, npal = [], 0
        for i, r in enumerate(self.seg):
            c = decode(int(r["key"]), k)
            pal = twin(c) == c
            npal += pal
            g = lo + i
            ic, itc = 2 * g, (2 * g if pal else 2 * g + 1)
            s_, p_ = c[1:], c[:-1]  # suffix / prefix junctions (half_recs)
            for (j, side, node, tnode) in ((s_, 0, ic, itc), (p_, 1, ic, itc)):
                tj = twin(j)
                if j < tj:
                    recs.append((encode(j), node | (side << 31), int(pal)))
                elif j > tj:
                    recs.append((encode(tj), tnode | ((1 - side) << 31), int(pal)))
                else:  # palindromic junction: both records
                    recs.append((encode(j), tnode | ((1 - side) << 31), int(pal)))
                    recs.append((encode(j), node | (side << 31), int(pal)))
        own = [self._jowner(key, nowners) for key, _, _ in recs]
        order = sorted(range(len(recs)), key=lambda q: own[q])
        out = np.array([recs[q] for q in order], dtype=self.JREC) if recs else np.zeros(0, self.JREC)
        return self._bytes(out), [own.count(o) for o in range(nowners)], npal

    def graph_join(self, recs, seg_lo):
        groups = {}
        for r in np.frombuffer(recs.numpy().tobytes(), dtype=self.JREC):
            g = groups.setdefault(int(r["key"]), ([set(), set()], {}))
            tag = int(r["tag"])
            node = tag & 0x7FFFFFFF
            g[0][tag >> 31].add(node)
            g[1][node] = int(r["pad"])
        n0, n1 = 2 * self.lo, 2 * (self.lo + len(self.seg))
        out = []
        for a, pal in groups.values():
            if len(a[0]) != 1 or len(a[1]) != 1:
                continue
            (x,), (y,) = a[0], a[1]
            tx, ty = (x if pal[x] else x ^ 1), (y if pal[y] else y ^ 1)
            if y == tx:
                continue
            for t, v in ((x, y), (ty, tx)):
                if n0 <= t < n1:
                    self.succ_seg[t] = v
                else:
                    out.append((t, v))
        own = [bisect.bisect_right(seg_lo, t >> 1) - 1 for t, _ in out]
        order = sorted(range(len(out)), key=lambda q: own[q])
        arr = np.array([out[q] for q in order], dtype=self.LINK) if out else np.zeros(0, self.LINK)
        return self._bytes(arr), [own.count(o) for o in range(len(seg_lo) - 1)]

    def graph_links_apply(self, links):
        n0, n1 = 2 * self.lo, 2 * (self.lo + len(self.seg))
        for r in np.frombuffer(links.numpy().tobytes(), dtype=self.LINK):
            assert n0 <= int(r["node"]) < n1, "a link record for another rank's node"
            self.succ_seg[int(r["node"])] = int(r["value"])

    # ---- partitioned finish (distributed.partitioned_finish): the same records / collectives,
    # computed by the design model -- every node is its own chain; its super record carries its
    # key and count in the spare fields, so the all-gathered supers rebuild the job's solid set
    # and check the junction join's links against the direct rule; contig i is emitted by the
    # rank whose segment holds the canonical id of its first k-mer
    SUP = np.dtype([("head", "<u4"), ("succ", "<u4"), ("w", "<u4"), ("pad", "<u4"), ("fmin", "<u8"), ("pad2", "<u8")])
    ST = np.dtype([("ev", "<u8"), ("node", "<u4"), ("pk", "<u4"), ("walk", "<u4", 6), ("clen", "<u4"), ("pad", "<u4")])

    def zeros(self, nbytes):
        return torch.zeros(max(int(nbytes), 1), dtype=torch.uint8)

    def graph_chains_part(self, lo, hi, part=None):
        assert part is None and lo == self.lo and hi == lo + len(self.seg)
        out = np.zeros(2 * (hi - lo), self.SUP)
        out["head"] = np.arange(2 * lo, 2 * hi, dtype=np.uint32)
        out["succ"] = [self.succ_seg.get(x, 0xFFFFFFFF) for x in range(2 * lo, 2 * hi)]
        out["w"] = 1
        out["pad"] = np.repeat(self.seg["count"], 2)
        out["pad2"] = np.repeat(self.seg["key"], 2)
        fm = np.zeros(2 * (hi - lo), np.uint64)
        fm[0::2] = self.seg["first_canon"]
        fm[1::2] = self.seg["first_twin"]
        out["fmin"] = fm
        return self._bytes(out), len(out)

    def graph_rank_supers(self, supers, M):
        sup = np.frombuffer(supers.numpy().tobytes(), dtype=self.SUP)[:M]
        N = 2 * self.U
        assert M == N and np.array_equal(sup["head"], np.arange(N)), "super records out of rank order"
        g = np.zeros(self.U, REC_DTYPE)
        g["key"] = sup["pad2"][0::2]
        g["count"] = sup["pad"][0::2]
        g["first_canon"] = sup["fmin"][0::2]
        g["first_twin"] = sup["fmin"][1::2]
        self.grecs = g
        self.gid = {int(x): i for i, x in enumerate(g["key"])}
        self.gk = self.k
        want = np.array([self._succ_of(x) for x in range(N)], dtype=np.uint32)
        assert np.array_equal(sup["succ"], want), "junction-joined links differ from the whole-set rule"
        self.full = self.assemble_from_solid(self._bytes(g), self.k)
    def _first_id(self, c):
        x = encode(c[: self.gk])
        return self.gid[min(x, self._tw(x))]

    def graph_starts_part(self, have_supers, lo, hi):
        own = [i for i, c in enumerate(self.full.contigs) if lo <= self._first_id(c) < hi]
        out = np.zeros(len(own), self.ST)
        out["ev"] = own
        out["node"] = own
        out["pk"] = own
        out["clen"] = [len(self.full.contigs[i]) for i in own]
        self.own = own
        return self._bytes(out), len(out)

    def graph_layout(self, starts, n):
        st = np.frombuffer(starts.numpy().tobytes(), dtype=self.ST)[:n]
        st = st[np.argsort(st["ev"], kind="stable")]
        assert list(st["ev"]) == list(range(len(self.full.contigs))), "gathered starts miss contigs"
        self.coff = np.concatenate([[0], np.cumsum(st["clen"].astype(np.int64))])
        self.nc = n
        return int(self.coff[-1])

    def graph_emit_part(self, chars, ends):
        e = np.zeros(max(2 * self.nc, 2), np.uint64)  # (the device writes end codes; one set per end)
        c = chars.numpy()
        for i in self.own:
            s = self.full.contigs[i].encode()
            c[self.coff[i]:self.coff[i] + len(s)] = np.frombuffer(s, np.uint8)
            e[i] = e[self.nc + i] = i + 1
        ends[: 16 * self.nc] = torch.from_numpy(e[: 2 * self.nc].view(np.uint8).copy())

    def graph_collect(self, chars, ends, k, npal, fetch=True):
        assert npal == sum(decode(int(x), k) == twin(decode(int(x), k)) for x in self.grecs["key"])
        e = np.frombuffer(ends.numpy().tobytes(), dtype=np.uint64)[: 2 * self.nc]
        assert list(e) == list(range(1, self.nc + 1)) * 2, "contig ends not set exactly once"
        ch = chars.numpy().tobytes()
        contigs = [ch[self.coff[i]:self.coff[i + 1]].decode() for i in range(self.nc)]
        assert contigs == self.full.contigs
        return _Result(self.full.dict_items, contigs, self.full.links)
