"""eulerhip -- ctypes binding of libeulerhip.so (include/eulerhip.h), the MI355X HIP core.

The product path.  Every call goes to the gfx950 kernels in csrc/; there is no CPU
fallback: if the shared library (or a GPU) is missing, the calls raise EulerHipError.

Layer 1 (fused, device-resident) mirrors the reference CPU assembler
src/referenceassembler/referenceAssembler.py build:25-42 + all_contigs:79-111:

    with Session() as s:
        res = s.assemble(reads, k=31, limit=1, want_dict=True)
        res.contigs      # == all_contigs(d, k)[1]   (r, in order)
        res.links        # == all_contigs(d, k)[0]   (G as [[fw], [bw]] per contig)
        res.dict_items   # == list(build(reads, k, limit).items())
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("EULERHIP_LIB") or os.path.join(HERE, "libeulerhip.so")  # override: experiments

EC_OK = 0
EC_ERR_ARG = -1
EC_ERR_ALPHABET = -2
EC_ERR_NOMEM = -3
EC_ERR_HIP = -4
EC_ERR_CAPACITY = -5
EC_ERR_STATE = -6

EC_FLAG_WANT_DICT = 1
EC_FLAG_TIMING = 2
EC_FLAG_KERNEL_TIMING = 128  # kernel_ms only (fewer events: bench.py's timed steps)
EC_FLAG_GENERAL = 4
EC_FLAG_WIDE_RECORDS = 8
EC_FLAG_WINDOW_RECORDS = 16
EC_FLAG_SUPERKMER = 32
EC_FLAG_EXACT_COUNT = 64
EC_NSTAGES = 8
EC_NKERNELS = 5
KERNEL_NAMES = ("k_upsweep", "k_downsweep", "k_bucket", "k_count", "k_refine")
EC_PATH_PARTITIONED = 0
EC_PATH_GENERAL = 1
EC_PATH_SUPERKMER = 2
EC_MAX_K = 63


class EulerHipError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("eulerhip error %d: %s" % (code, msg))
        self.code = code


class AlphabetError(EulerHipError, ValueError):
    pass


class Stats(ctypes.Structure):
    _fields_ = [
        ("n_reads", ctypes.c_uint64),
        ("n_positions", ctypes.c_uint64),
        ("n_distinct_est", ctypes.c_uint64),
        ("n_distinct", ctypes.c_uint64),
        ("n_solid", ctypes.c_uint64),
        ("n_dict", ctypes.c_uint64),
        ("n_contigs", ctypes.c_uint64),
        ("n_contig_chars", ctypes.c_uint64),
        ("n_links", ctypes.c_uint64),
        ("table_capacity", ctypes.c_uint64),
        ("n_rulers", ctypes.c_uint64),
        ("n_records", ctypes.c_uint64),
        ("table_retries", ctypes.c_uint32),
        ("rank_rounds", ctypes.c_uint32),
        ("count_path", ctypes.c_uint32),
        ("n_buckets", ctypes.c_uint32),
        ("record_bytes", ctypes.c_uint32),
        ("count_variant", ctypes.c_uint32),
        ("stage_ms", ctypes.c_float * EC_NSTAGES),
        ("kernel_ms", ctypes.c_float * EC_NKERNELS),
    ]

    def as_dict(self):
        d = {f: getattr(self, f) for f, _ in self._fields_ if f not in ("stage_ms", "kernel_ms")}
        d["stage_ms"] = list(self.stage_ms)
        d["kernel_ms"] = list(self.kernel_ms)
        return d


_lib = None

# exported symbols and their signatures (tests check that every one declared in
# include/eulerhip.h is exported by the library)
_P = ctypes.c_void_p
_U64 = ctypes.c_uint64
_SIGS = {
    "ec_last_error": (ctypes.c_char_p, []),
    "ec_version": (ctypes.c_int, []),
    "ec_session_create": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int]),
    "ec_session_set_stream": (ctypes.c_int, [_P, _P]),
    "ec_session_destroy": (ctypes.c_int, [_P]),
    "ec_mem_stats": (ctypes.c_int, [ctypes.POINTER(_U64), ctypes.POINTER(_U64), ctypes.c_int]),
    "ec_session_trim": (ctypes.c_int, [_P, _U64]),
    "ec_session_bytes": (_U64, [_P]),
    "ec_assemble_device": (ctypes.c_int, [_P, _P, _P, _U64, ctypes.c_int, ctypes.c_int, ctypes.c_uint]),
    "ec_assemble_host": (ctypes.c_int, [_P, _P, _U64, _P, _U64, ctypes.c_int, ctypes.c_int, ctypes.c_uint]),
    "ec_assemble_packed_host": (ctypes.c_int, [_P, _P, _U64, _P, _U64, ctypes.c_uint32, _P, _P, _U64, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_uint]),
    "ec_stage_packed_host": (ctypes.c_int, [_P, _P, _U64, _P, _U64, ctypes.c_uint32, _P, _P, _U64]),
    "ec_assemble_staged": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_uint]),
    "ec_pack_reads": (ctypes.c_int, [_P, _P, _U64, ctypes.c_int, _P, _P, _P, _U64, ctypes.POINTER(_U64),
                                     ctypes.POINTER(ctypes.c_uint32)]),
    "ec_assemble_from_kmers": (ctypes.c_int, [_P, ctypes.c_char_p, _P, _U64, ctypes.c_int, ctypes.c_uint]),
    "ec_get_stats": (ctypes.c_int, [_P, ctypes.POINTER(Stats)]),
    "ec_stage_name": (ctypes.c_char_p, [ctypes.c_int]),
    "ec_copy_contigs": (ctypes.c_int, [_P, _P, _P]),
    "ec_copy_links": (ctypes.c_int, [_P, _P, _P]),
    "ec_copy_dict": (ctypes.c_int, [_P, _P, _P]),
}


def lib():
    """Load libeulerhip.so (in-tree).  Raises if it has not been built."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: PyTorch-ROCm bundles libamdhip64.so.7 /
        # libhsa-runtime64.so.1 with the same SONAMEs as /opt/rocm.  Loading torch first makes
        # the dynamic loader bind libeulerhip.so to torch's copy, so torch tensors, streams and
        # our kernels share one runtime (loading ours first would give torch a second HSA
        # runtime that sees no GPUs).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise EulerHipError(EC_ERR_STATE, "libeulerhip.so not built (run __graft_entry__.build() or make -C csrc)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def register(name, restype, argtypes):
    """Per-module wrappers declare their extra symbols here."""
    _SIGS[name] = (restype, argtypes)
    if _lib is not None:
        fn = getattr(_lib, name)
        fn.restype = restype
        fn.argtypes = argtypes


def check(rc):
    if rc != EC_OK:
        msg = lib().ec_last_error().decode(errors="replace")
        if rc == EC_ERR_ALPHABET:
            raise AlphabetError(rc, msg)
        raise EulerHipError(rc, msg)
    return rc


def mem_stats(reset=False):
    """(held, peak): device bytes this process's session buffers hold and their high-water mark
    (ec_mem_stats); reset restarts the mark at the current holding"""
    h, p = _U64(0), _U64(0)
    check(lib().ec_mem_stats(ctypes.byref(h), ctypes.byref(p), int(bool(reset))))
    return int(h.value), int(p.value)


def stage_names():
    L = lib()
    return [L.ec_stage_name(i).decode() for i in range(EC_NSTAGES)]


def pack_reads(reads):
    """list[str|bytes] -> (uint8 buffer, uint64 offsets[n+1]).  Host-side CSR packing."""
    bs = [r.encode("ascii") if isinstance(r, str) else bytes(r) for r in reads]
    off = np.zeros(len(bs) + 1, dtype=np.uint64)
    if bs:
        off[1:] = np.cumsum([len(b) for b in bs], dtype=np.uint64)
    buf = np.frombuffer(b"".join(bs), dtype=np.uint8)
    return buf, off


class PackedReads:
    """Reads 2 bits per base (include/eulerhip.h ec_assemble_packed_host): codes uint8[ceil(n/4)],
    offsets uint64[nreads + 1] or None with read_len = the common length, and the bytes other than
    A/C/G/T as (exc_pos uint64[], exc_byte uint8[])."""

    def __init__(self, codes, nbases, nreads, offsets=None, read_len=0, exc_pos=None, exc_byte=None):
        self.codes, self.nbases, self.nreads = codes, int(nbases), int(nreads)
        self.offsets, self.read_len = offsets, int(read_len)
        self.exc_pos = exc_pos if exc_pos is not None else np.zeros(0, np.uint64)
        self.exc_byte = exc_byte if exc_byte is not None else np.zeros(0, np.uint8)


def pack_2bit(buf, offsets, threads=0, alloc=None):
    """ASCII CSR reads -> PackedReads (ec_pack_reads, host threads).  alloc(n) -> a uint8 array of
    n bytes for the codes (e.g. page-locked memory); numpy by default."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    if offsets.size == 0:
        raise ValueError("offsets must hold nreads + 1 entries (at least [0])")
    n = len(offsets) - 1
    nb = int(offsets[-1])
    ncodes = (nb + 3) // 4
    codes = alloc(max(ncodes, 1)) if alloc else np.empty(max(ncodes, 1), np.uint8)
    nexc = ctypes.c_uint64(0)
    rl = ctypes.c_uint32(0)
    cap = 1 << 16
    while True:
        pos = np.empty(cap, np.uint64)
        byt = np.empty(cap, np.uint8)
        check(lib().ec_pack_reads(buf.ctypes.data if buf.size else None, offsets.ctypes.data, n, int(threads),
                                  codes.ctypes.data, pos.ctypes.data, byt.ctypes.data, cap, ctypes.byref(nexc),
                                  ctypes.byref(rl)))
        if nexc.value <= cap:
            break
        cap = int(nexc.value)
    ne = int(nexc.value)
    return PackedReads(codes, nb, n, None if rl.value else offsets, rl.value, pos[:ne].copy(), byt[:ne].copy())


class Result:
    """Outputs of one fused assembly (host copies)."""

    def __init__(self, k, stats, chars, coff, loff, links, dict_items=None):
        self.k = k
        self.stats = stats
        self._chars = chars
        self.contig_offsets = coff
        self.link_offsets = loff
        self.link_codes = links
        self.dict_items = dict_items

    @property
    def contig_bytes(self):
        """all contig characters concatenated (bytes; converted once, on first use)"""
        if not isinstance(self._chars, bytes):
            self._chars = self._chars.tobytes()
        return self._chars

    @property
    def contigs(self):
        ch = self.contig_bytes.decode("ascii")
        o = self.contig_offsets
        return [ch[int(o[i]):int(o[i + 1])] for i in range(len(o) - 1)]

    @property
    def links(self):
        """G of all_contigs as [[fw links], [bw links]] per contig, link = [j, '+'|'-']."""
        out = []
        lo, lk = self.link_offsets, self.link_codes
        for i in range((len(lo) - 1) // 2):
            sides = []
            for s in range(2):
                a, b = int(lo[2 * i + s]), int(lo[2 * i + s + 1])
                sides.append([[int(v) >> 1, "-" if v & 1 else "+"] for v in lk[a:b]])
            out.append(sides)
        return out

    def G(self):
        """all_contigs' G exactly: {i: ([(j, o), ...], [(j, o), ...])}"""
        return {i: ([tuple(x) for x in s[0]], [tuple(x) for x in s[1]]) for i, s in enumerate(self.links)}


class Session:
    """A device-resident assembly session on one GPU (ec_session)."""

    def __init__(self, device=0, stream=None):
        L = lib()
        h = ctypes.c_void_p()
        check(L.ec_session_create(ctypes.byref(h), int(device)))
        self._h = h
        self.device = device
        if stream is not None:
            check(L.ec_session_set_stream(self._h, ctypes.c_void_p(int(stream))))

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            lib().ec_session_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def trim(self, min_bytes=0):
        """release the device buffers of >= min_bytes and the device state they hold
        (ec_session_trim); host-side results stay fetchable"""
        check(lib().ec_session_trim(self._h, int(min_bytes)))

    def device_bytes(self):
        """device bytes the session's buffers hold (ec_session_bytes)"""
        return int(lib().ec_session_bytes(self._h))

    def set_stream(self, stream):
        """stream: a hipStream_t handle (0 = the null stream, torch's default) or None for the
        session's own non-blocking stream"""
        h = ctypes.c_void_p(-1 & 0xFFFFFFFFFFFFFFFF) if stream is None else ctypes.c_void_p(int(stream))
        check(lib().ec_session_set_stream(self._h, h))

    # -- run -------------------------------------------------------------------------------
    def run_host(self, buf, offsets, k, limit=1, flags=0):
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = len(offsets) - 1
        pbuf = buf.ctypes.data if buf.size else None
        check(lib().ec_assemble_host(self._h, pbuf, buf.size, offsets.ctypes.data, n, int(k), int(limit), flags))

    def run_packed_host(self, pr, k, limit=1, flags=0):
        """Reads 2 bits per base in host memory (PackedReads): a quarter of run_host's PCIe bytes."""
        off = None if pr.offsets is None else np.ascontiguousarray(pr.offsets, dtype=np.uint64)
        ne = len(pr.exc_pos)
        check(lib().ec_assemble_packed_host(
            self._h, pr.codes.ctypes.data if pr.nbases else None, pr.nbases, None if off is None else off.ctypes.data,
            pr.nreads, pr.read_len, pr.exc_pos.ctypes.data if ne else None, pr.exc_byte.ctypes.data if ne else None,
            ne, int(k), int(limit), flags))

    def stage_packed(self, pr):
        """Queue a PackedReads batch's H2D copies (ec_stage_packed_host; two slots).  pr must stay
        alive and unchanged until assemble_staged() has consumed it."""
        off = None if pr.offsets is None else np.ascontiguousarray(pr.offsets, dtype=np.uint64)
        if off is not None:
            pr.offsets = off  # (kept alive with pr)
        ne = len(pr.exc_pos)
        check(lib().ec_stage_packed_host(
            self._h, pr.codes.ctypes.data if pr.nbases else None, pr.nbases, None if off is None else off.ctypes.data,
            pr.nreads, pr.read_len, pr.exc_pos.ctypes.data if ne else None, pr.exc_byte.ctypes.data if ne else None,
            ne))

    def assemble_staged(self, k, limit=1, flags=0):
        """Assemble the oldest staged batch (ec_assemble_staged): staging batch i + 1 before this
        call overlaps its PCIe copy with batch i's kernels."""
        check(lib().ec_assemble_staged(self._h, int(k), int(limit), flags))

    def run_device(self, d_reads_ptr, d_offsets_ptr, nreads, k, limit=1, flags=0):
        """Reads already in HBM (e.g. torch uint8 / int64 tensors' data_ptr())."""
        check(lib().ec_assemble_device(self._h, ctypes.c_void_p(int(d_reads_ptr)), ctypes.c_void_p(int(d_offsets_ptr)),
                                       int(nreads), int(k), int(limit), flags))

    def stats(self):
        st = Stats()
        check(lib().ec_get_stats(self._h, ctypes.byref(st)))
        return st

    def fetch(self, k, want_dict=False):
        st = self.stats()
        L = lib()
        nc, nch, nl = st.n_contigs, st.n_contig_chars, st.n_links
        chars = np.empty(max(nch, 1), dtype=np.uint8)  # one copy out of the pinned result buffer
        coff = np.empty(nc + 1, dtype=np.uint64)
        check(L.ec_copy_contigs(self._h, chars.ctypes.data, coff.ctypes.data))
        loff = np.zeros(2 * nc + 1, dtype=np.uint64)
        links = np.zeros(max(nl, 1), dtype=np.int64)
        check(L.ec_copy_links(self._h, loff.ctypes.data, links.ctypes.data))
        items = None
        if want_dict:
            nd = st.n_dict
            km = ctypes.create_string_buffer(max(nd * k, 1))
            cnt = np.zeros(max(nd, 1), dtype=np.uint32)
            check(L.ec_copy_dict(self._h, km, cnt.ctypes.data))
            s = km.raw[: nd * k].decode("ascii")
            items = [(s[i * k:(i + 1) * k], int(cnt[i])) for i in range(nd)]
        return Result(k, st, chars[:nch], coff, loff, links[:nl], items)

    def assemble(self, reads, k, limit=1, want_dict=False, timing=False, general=False, wide_records=False,
                 window_records=False, superkmer=False, exact_count=False):
        buf, off = pack_reads(reads)
        flags = (EC_FLAG_WANT_DICT if want_dict else 0) | (EC_FLAG_TIMING if timing else 0)
        flags |= (EC_FLAG_GENERAL if general else 0) | (EC_FLAG_WIDE_RECORDS if wide_records else 0)
        flags |= (EC_FLAG_WINDOW_RECORDS if window_records else 0) | (EC_FLAG_SUPERKMER if superkmer else 0)
        flags |= EC_FLAG_EXACT_COUNT if exact_count else 0
        self.run_host(buf, off, k, limit, flags)
        return self.fetch(k, want_dict)

    def assemble_dict(self, d, k):
        """all_contigs on a caller's dict {k-mer: count} (dict order matters): the graph phase
        of the fused path, on the device (ec_assemble_from_kmers)."""
        items = list(d.items())
        n = len(items)
        for x, _ in items:
            if len(x) != k:
                raise EulerHipError(EC_ERR_ARG, "dict key %r is not a %d-mer" % (x, k))
        km = "".join(x for x, _ in items).encode("ascii")
        cnt = np.array([c for _, c in items], dtype=np.uint32) if n else np.zeros(1, np.uint32)
        check(lib().ec_assemble_from_kmers(self._h, km, cnt.ctypes.data, n, int(k), 0))
        return self.fetch(k)


_default = {}


def default_session(device=0):
    s = _default.get(device)
    if s is None:
        s = _default[device] = Session(device)
    return s


def assemble(reads, k, limit=1, want_dict=False, device=0):
    """One-shot fused assembly on `device`."""
    return default_session(device).assemble(reads, k, limit, want_dict)
