"""Parity of the fused HIP path (libeulerhip.so, ec_assemble_*) with the reference.

* every golden case generated from the real reference (tests/golden/): ordered dict,
  contigs and GFA links must be identical;
* larger seeded synthetic inputs against the C oracle (oracle/refasm.c, itself pinned to
  the golden vectors in test_oracle.py): bit-exact contigs + links (+ dict on some);
* error behaviour (alphabet, k range), determinism, device-pointer entry point.
"""
import numpy as np
import pytest

import eulerhip
import oracle
from conftest import golden_cases
from synth import make_reads

pytestmark = pytest.mark.gpu

CASES = golden_cases("g200.json", "synthetic.json", "fuzz.json")
CASES32 = [c for c in CASES if c["k"] <= eulerhip.EC_MAX_K]


@pytest.mark.parametrize("case", CASES32, ids=[c["name"] for c in CASES32])
def test_golden(gpu_session, case):
    res = gpu_session.assemble(case["reads"], case["k"], case["limit"], want_dict=True)
    assert [[x, c] for x, c in res.dict_items] == case["d"]
    assert res.contigs == case["contigs"]
    assert res.links == case["links"]
    if res.stats.n_positions > 0:
        assert res.stats.count_path in _want_paths(case["reads"], case["k"], False)


def _sk_applies(reads, k):
    return 21 <= k <= 32 and not any("N" in r for r in reads)


def _want_paths(reads, k, superkmer):
    """partitioned counting (super-k-mer or window records) for k <= 32; k > 32: 24-B records
    without N, else the general table.  EC_FLAG_SUPERKMER is accepted and changes nothing
    (super-k-mer records are the default where they apply)."""
    if k > 32:  # partitioned 24-B records for N-free reads (count_wide.h)
        return (eulerhip.EC_PATH_GENERAL,) if any("N" in r for r in reads) else (eulerhip.EC_PATH_PARTITIONED,)
    return (eulerhip.EC_PATH_PARTITIONED,)


@pytest.mark.parametrize("case", CASES32[1::3], ids=[c["name"] for c in CASES32[1::3]])
def test_golden_superkmer(gpu_session, case):
    """EC_FLAG_SUPERKMER (accepted, the default behaviour)"""
    res = gpu_session.assemble(case["reads"], case["k"], case["limit"], want_dict=True, superkmer=True)
    assert [[x, c] for x, c in res.dict_items] == case["d"]
    assert res.contigs == case["contigs"]
    assert res.links == case["links"]
    if res.stats.n_positions > 0:
        assert res.stats.count_path in _want_paths(case["reads"], case["k"], True)


@pytest.mark.parametrize("case", CASES32[::3], ids=[c["name"] for c in CASES32[::3]])
def test_golden_window_records(gpu_session, case):
    """one record per window forced (EC_FLAG_WINDOW_RECORDS) where super-k-mers would apply"""
    res = gpu_session.assemble(case["reads"], case["k"], case["limit"], want_dict=True, window_records=True)
    assert [[x, c] for x, c in res.dict_items] == case["d"]
    assert res.contigs == case["contigs"]
    assert res.links == case["links"]
    if res.stats.n_positions > 0 and case["k"] <= 32:
        assert res.stats.count_path == eulerhip.EC_PATH_PARTITIONED


@pytest.mark.parametrize("case", CASES32[1::2], ids=[c["name"] for c in CASES32[1::2]])
def test_golden_wide_records(gpu_session, case):
    """16-B records forced (EC_FLAG_WIDE_RECORDS; one-length N-free inputs default to 12-B records)"""
    res = gpu_session.assemble(case["reads"], case["k"], case["limit"], want_dict=True, wide_records=True)
    assert [[x, c] for x, c in res.dict_items] == case["d"]
    assert res.contigs == case["contigs"]
    assert res.links == case["links"]


@pytest.mark.parametrize("case", CASES32[::2], ids=[c["name"] for c in CASES32[::2]])
def test_golden_exact_count(gpu_session, case):
    """count_part.h's histogram-sized runs forced (EC_FLAG_EXACT_COUNT)"""
    res = gpu_session.assemble(case["reads"], case["k"], case["limit"], want_dict=True, exact_count=True)
    assert [[x, c] for x, c in res.dict_items] == case["d"]
    assert res.contigs == case["contigs"]
    assert res.links == case["links"]
    assert res.stats.count_variant == 0


@pytest.mark.parametrize("case", CASES32[::2], ids=[c["name"] for c in CASES32[::2]])
def test_golden_general_path(gpu_session, case):
    res = gpu_session.assemble(case["reads"], case["k"], case["limit"], want_dict=True, general=True)
    assert [[x, c] for x, c in res.dict_items] == case["d"]
    assert res.contigs == case["contigs"]
    assert res.links == case["links"]


def test_extended_alphabet_rejected(gpu_session):
    for case in golden_cases("synthetic.json", alphabet="extended"):
        with pytest.raises(eulerhip.AlphabetError):
            gpu_session.assemble(case["reads"], case["k"], case["limit"])


def test_k_out_of_range(gpu_session):
    with pytest.raises(eulerhip.EulerHipError):
        gpu_session.assemble(["ACGT" * 20], 0)
    with pytest.raises(eulerhip.EulerHipError):
        gpu_session.assemble(["ACGT" * 20], 64)
    with pytest.raises(eulerhip.EulerHipError):
        gpu_session.assemble(["ACGT" * 20], 65)


def _oracle_packed(buf, off, k, limit=1, want_dict=False):
    out = oracle.assemble_packed(buf, off, k, limit, want_dict)
    return out, oracle.unpack_contigs(out), oracle.unpack_links(out)


SYN = [
    # genome, reads, len, seed, err, n_rate, circular, k
    (20_000, 4_000, 100, 1, 0.0, 0.0, False, 31),
    (50_000, 20_000, 100, 2, 0.005, 0.0, False, 31),
    (30_000, 10_000, 80, 3, 0.002, 0.002, True, 25),
    (5_000, 5_000, 60, 4, 0.01, 0.0, False, 20),
    (2_000, 3_000, 50, 5, 0.0, 0.0, True, 16),
    (200_000, 60_000, 100, 6, 0.0, 0.0, False, 32),
    (1_000, 2_000, 40, 7, 0.02, 0.01, False, 11),
    # 128-bit keys (32 < k <= 63; BASELINE config 5 uses k = 51)
    (30_000, 12_000, 150, 8, 0.002, 0.0, False, 51),
    (20_000, 8_000, 100, 9, 0.003, 0.002, True, 33),
    (10_000, 6_000, 120, 10, 0.0, 0.0, False, 63),
    (3_000, 4_000, 90, 11, 0.01, 0.0, False, 40),
]


@pytest.mark.parametrize("mode", ["partitioned", "exact", "superkmer", "window_records", "wide_records", "general"])
@pytest.mark.parametrize("g,n,L,seed,err,nr,circ,k", SYN)
def test_synthetic_vs_oracle(gpu_session, g, n, L, seed, err, nr, circ, k, mode):
    buf, off = make_reads(g, n, L, 1000 + seed, err=err, n_rate=nr, circular=circ)
    want_dict = g <= 50_000
    ref, rc, rl = _oracle_packed(buf, off, k, 1, want_dict)
    flags = (eulerhip.EC_FLAG_WANT_DICT if want_dict else 0) | {
        "partitioned": 0, "exact": eulerhip.EC_FLAG_EXACT_COUNT,
        "general": eulerhip.EC_FLAG_GENERAL, "wide_records": eulerhip.EC_FLAG_WIDE_RECORDS,
        "window_records": eulerhip.EC_FLAG_WINDOW_RECORDS, "superkmer": eulerhip.EC_FLAG_SUPERKMER}[mode]
    gpu_session.run_host(buf, off, k, 1, flags)
    res = gpu_session.fetch(k, want_dict)
    assert res.stats.n_positions == ref["n_positions"]
    assert res.stats.n_dict == ref["n_dict"]
    assert res.contig_bytes == ref["contig_chars"]
    assert np.array_equal(res.contig_offsets, ref["contig_offsets"])
    assert res.links == rl
    if want_dict:
        assert [[x, c] for x, c in res.dict_items] == ref["d"]
    if mode in ("partitioned", "window_records") and k <= 32 and nr == 0 \
            and res.stats.count_path == eulerhip.EC_PATH_PARTITIONED and res.stats.count_variant != 3:
        assert res.stats.record_bytes == 12  # one read length, no N: 12-B window records
    if mode == "window_records" and k <= 32:
        assert res.stats.count_path in (eulerhip.EC_PATH_PARTITIONED, eulerhip.EC_PATH_GENERAL)
    if mode == "wide_records" and k <= 32:
        assert res.stats.record_bytes == 16
    # one read length, no N, k <= 32: the fixed-capacity runs of count_v2.h unless asked otherwise
    if mode in ("partitioned", "window_records", "superkmer") and k <= 32 and nr == 0:
        if mode != "window_records" and 21 <= k and err <= 0.01:  # 16-B super-k-mer records (count_sk2.h)
            assert res.stats.count_variant == 3 and res.stats.record_bytes == 16
            assert 0 < res.stats.n_records < res.stats.n_positions
        else:  # small inputs: 12-B window records
            assert res.stats.count_variant == 1 and res.stats.record_bytes == 12
    if mode == "exact":
        assert res.stats.count_variant == 0


def test_limits_vs_oracle(gpu_session):
    buf, off = make_reads(3_000, 1_500, 50, 99, err=0.01)
    for lim in (-1, 0, 2, 5):
        _, rc, rl = _oracle_packed(buf, off, 15, lim)
        gpu_session.run_host(buf, off, 15, lim)
        res = gpu_session.fetch(15)
        assert res.contigs == rc and res.links == rl, lim


def test_deterministic(gpu_session):
    buf, off = make_reads(100_000, 30_000, 100, 11, err=0.003)
    outs = []
    for _ in range(3):
        gpu_session.run_host(buf, off, 31, 1)
        r = gpu_session.fetch(31)
        outs.append((r.contig_bytes, r.contig_offsets.tobytes(), r.link_codes.tobytes()))
    assert outs[0] == outs[1] == outs[2]


def test_device_pointer_entry_point(gpu_session):
    torch = pytest.importorskip("torch")
    buf, off = make_reads(40_000, 12_000, 100, 12, err=0.002)
    gpu_session.run_host(buf, off, 31, 1)
    want = gpu_session.fetch(31)
    d_buf = torch.from_numpy(buf).cuda()
    d_off = torch.from_numpy(off.astype(np.int64)).cuda()
    torch.cuda.synchronize()
    gpu_session.run_device(d_buf.data_ptr(), d_off.data_ptr(), len(off) - 1, 31, 1)
    got = gpu_session.fetch(31)
    assert got.contig_bytes == want.contig_bytes and got.links == want.links


def test_empty_and_ragged(gpu_session):
    for reads in ([], [""], ["ACG"], ["N" * 50], ["ACGTTGCA" * 3, "", "A", "ACGTTGCAACG" * 2, "NNACGTTGCAAC"]):
        for k in (1, 3, 5):
            res = gpu_session.assemble(reads, k, 1, want_dict=True)
            d, r, g = oracle.assemble(reads, k, 1)
            assert [[x, c] for x, c in res.dict_items] == d and res.contigs == r and res.links == g


def test_long_reads_take_general_path(gpu_session):
    # > 32767 windows in one read: local events exceed 16 bits -> general counting path
    buf, off = make_reads(60_000, 4, 40_000, 31, err=0.0, circular=True)
    ref, rc, rl = _oracle_packed(buf, off, 21)
    gpu_session.run_host(buf, off, 21, 1)
    res = gpu_session.fetch(21)
    assert res.stats.count_path == eulerhip.EC_PATH_GENERAL
    assert res.contig_bytes == ref["contig_chars"] and res.links == rl


def test_many_buckets_vs_oracle(gpu_session):
    # enough distinct k-mers for B > 1 buckets with errors (singletons fill the LDS tables)
    buf, off = make_reads(300_000, 200_000, 100, 32, err=0.004)
    ref, rc, rl = _oracle_packed(buf, off, 31)
    gpu_session.run_host(buf, off, 31, 1)
    res = gpu_session.fetch(31)
    assert res.stats.count_path == eulerhip.EC_PATH_PARTITIONED
    assert res.stats.n_buckets > 64
    assert res.contig_bytes == ref["contig_chars"] and res.links == rl
    gpu_session.run_host(buf, off, 31, 1, eulerhip.EC_FLAG_SUPERKMER)
    res = gpu_session.fetch(31)
    assert res.stats.count_path == eulerhip.EC_PATH_PARTITIONED and res.stats.n_buckets > 64
    assert res.contig_bytes == ref["contig_chars"] and res.links == rl
    gpu_session.run_host(buf, off, 31, 1, eulerhip.EC_FLAG_WINDOW_RECORDS)
    res = gpu_session.fetch(31)
    assert res.stats.count_path == eulerhip.EC_PATH_PARTITIONED and res.stats.n_buckets > 64
    assert res.contig_bytes == ref["contig_chars"] and res.links == rl


def _low_complexity_reads(n, L, seed):
    """reads over short tandem repeats and homopolymers: minimizer runs reach the record cap,
    heavy minimizers, palindromic k-mers for even k"""
    rng = np.random.default_rng(seed)
    units = ["A", "AC", "ACGT", "AT", "CG", "AAC", "GATC", "ACGTTGCA", "TTAGGG"]
    out = []
    for i in range(n):
        u = units[rng.integers(len(units))]
        body = (u * (L // len(u) + 2))[: L]
        b = list(body)
        for _ in range(rng.integers(0, 3)):  # a few substitutions
            b[rng.integers(L)] = "ACGT"[rng.integers(4)]
        out.append("".join(b))
    rnd = "".join("ACGT"[x] for x in rng.integers(0, 4, 5000))
    for i in range(n):
        p = int(rng.integers(0, len(rnd) - L))
        out.append(rnd[p:p + L])
    return out


@pytest.mark.parametrize("k", [21, 22, 27, 31, 32])
def test_superkmer_low_complexity_vs_oracle(gpu_session, k):
    reads = _low_complexity_reads(400, 120, 40 + k)
    d, r, g = oracle.assemble(reads, k, 1)
    res = gpu_session.assemble(reads, k, 1, want_dict=True)
    assert res.stats.count_path == eulerhip.EC_PATH_PARTITIONED
    assert [[x, c] for x, c in res.dict_items] == d and res.contigs == r and res.links == g


@pytest.mark.parametrize("k", [21, 26, 31])
def test_superkmer_ragged_lengths_vs_oracle(gpu_session, k):
    # mixed read lengths (some shorter than k, some long): per-read window counts in the records
    rng = np.random.default_rng(k)
    g = "".join("ACGT"[x] for x in rng.integers(0, 4, 30_000))
    reads = []
    for i in range(6000):
        L = int(rng.choice([5, k - 1, k, k + 1, 60, 151, 300, 1000]))
        p = int(rng.integers(0, len(g) - L))
        x = g[p:p + L]
        reads.append(x if rng.random() < 0.5 else x[::-1].translate(str.maketrans("ACGT", "TGCA")))
    buf = np.frombuffer("".join(reads).encode(), np.uint8).copy()
    off = np.zeros(len(reads) + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in reads])
    ref, rc, rl = _oracle_packed(buf, off, k, 1, True)
    gpu_session.run_host(buf, off, k, 1, eulerhip.EC_FLAG_WANT_DICT)
    res = gpu_session.fetch(k, True)
    assert res.stats.count_path == eulerhip.EC_PATH_PARTITIONED
    assert [[x, c] for x, c in res.dict_items] == ref["d"]
    assert res.contig_bytes == ref["contig_chars"] and res.links == rl


# ---- seen-twice filter buckets (k_bucket_filt) -----------------------------------------------
# Taken automatically when the distinct k-mers (mostly error singletons) outgrow the LDS tables
# (> ~2·10^7 distinct); EULERHIP_FORCE_FILTER takes it at any size so the oracle can check it.
@pytest.mark.parametrize("fmt", ["compact", "wide_records"])
@pytest.mark.parametrize("g,n,L,seed,err,nr,circ,k", [c for c in SYN if c[-1] <= 32])
def test_filter_buckets_vs_oracle(gpu_session, monkeypatch, g, n, L, seed, err, nr, circ, k, fmt):
    monkeypatch.setenv("EULERHIP_FORCE_FILTER", "1")
    buf, off = make_reads(g, n, L, 1000 + seed, err=err, n_rate=nr, circular=circ)
    want_dict = g <= 50_000
    ref, rc, rl = _oracle_packed(buf, off, k, 1, want_dict)
    flags = (eulerhip.EC_FLAG_WANT_DICT if want_dict else 0) | \
        (eulerhip.EC_FLAG_WIDE_RECORDS if fmt == "wide_records" else 0)
    gpu_session.run_host(buf, off, k, 1, flags)
    res = gpu_session.fetch(k, want_dict)
    assert res.stats.count_path == eulerhip.EC_PATH_PARTITIONED
    assert res.stats.n_dict == ref["n_dict"]
    assert res.contig_bytes == ref["contig_chars"] and res.links == rl
    if want_dict:
        assert [[x, c] for x, c in res.dict_items] == ref["d"]


def test_filter_buckets_limits_vs_oracle(gpu_session, monkeypatch):
    """limit >= 1: seen-twice filter; limit < 1: no filter, the two half tables only; even k
    keeps palindromes, whose single insert adds 2"""
    monkeypatch.setenv("EULERHIP_FORCE_FILTER", "1")
    for k, lim in ((15, 1), (15, 2), (16, 1), (20, 3), (31, 5), (15, 0), (16, -1), (31, 0)):
        buf, off = make_reads(4_000, 3_000, 60, 500 + k + lim, err=0.01)
        ref, rc, rl = _oracle_packed(buf, off, k, lim)
        gpu_session.run_host(buf, off, k, lim)
        res = gpu_session.fetch(k)
        assert res.contig_bytes == ref["contig_chars"] and res.links == rl, (k, lim)


# ---- partitioned 128-bit counting (count_wide.h, 32 < k <= 63) -------------------------------
WIDE = [  # genome, reads, len, seed, err, circular, k
    (30_000, 12_000, 150, 21, 0.002, False, 51),
    (20_000, 8_000, 100, 22, 0.003, True, 33),
    (10_000, 6_000, 120, 23, 0.0, False, 63),
    (3_000, 4_000, 90, 24, 0.01, False, 40),
    (300_000, 60_000, 150, 25, 0.002, False, 51),  # 2^9 buckets: refine pass
    (200_000, 50_000, 150, 26, 0.0, True, 62),
]


@pytest.mark.parametrize("g,n,L,seed,err,circ,k", WIDE)
def test_wide_partitioned_vs_oracle(gpu_session, g, n, L, seed, err, circ, k):
    buf, off = make_reads(g, n, L, 2000 + seed, err=err, circular=circ)
    want_dict = g <= 50_000
    ref, rc, rl = _oracle_packed(buf, off, k, 1, want_dict)
    gpu_session.run_host(buf, off, k, 1, eulerhip.EC_FLAG_WANT_DICT if want_dict else 0)
    res = gpu_session.fetch(k, want_dict)
    assert res.stats.count_path == eulerhip.EC_PATH_PARTITIONED and res.stats.record_bytes == 24
    if g >= 200_000:
        assert res.stats.n_buckets >= 128
    assert res.stats.n_positions == ref["n_positions"] and res.stats.n_dict == ref["n_dict"]
    assert res.contig_bytes == ref["contig_chars"] and res.links == rl
    if want_dict:
        assert [[x, c] for x, c in res.dict_items] == ref["d"]


@pytest.mark.parametrize("k", [34, 40, 51, 62])
def test_wide_low_complexity_vs_oracle(gpu_session, k):
    """tandem repeats: heavy keys, long probe chains; even k: palindromic 128-bit keys"""
    reads = _low_complexity_reads(300, 140, 60 + k)
    d, r, g = oracle.assemble(reads, k, 1)
    res = gpu_session.assemble(reads, k, 1, want_dict=True)
    assert res.stats.count_path == eulerhip.EC_PATH_PARTITIONED
    assert [[x, c] for x, c in res.dict_items] == d and res.contigs == r and res.links == g


def test_wide_ragged_and_limits_vs_oracle(gpu_session):
    rng = np.random.default_rng(77)
    g = "".join("ACGT"[x] for x in rng.integers(0, 4, 20_000))
    reads = []
    for i in range(5000):
        L = int(rng.choice([10, 50, 51, 52, 90, 150, 155]))
        p = int(rng.integers(0, len(g) - L))
        reads.append(g[p:p + L])
    for lim in (-1, 0, 1, 3):
        d, r, gl = oracle.assemble(reads, 51, lim)
        res = gpu_session.assemble(reads, 51, lim, want_dict=True)
        assert res.stats.count_path == eulerhip.EC_PATH_PARTITIONED
        assert [[x, c] for x, c in res.dict_items] == d and res.contigs == r and res.links == gl, lim


def test_wide_fallbacks_vs_oracle(gpu_session, monkeypatch):
    """N in a read, tiles over the 40 KB stage, buckets past their table: the HBM table"""
    cases = [
        (make_reads(20_000, 6_000, 100, 31, err=0.002, n_rate=0.002), None),
        (make_reads(20_000, 3_000, 200, 32, err=0.002), None),   # 256 x 200 B > 40 KB
        (make_reads(100_000, 30_000, 120, 33, err=0.003), "2"),  # 4 buckets of ~5e4 keys
    ]
    for (buf, off), maxb in cases:
        if maxb:
            monkeypatch.setenv("EULERHIP_WIDE_MAX_BBITS", maxb)
        ref, rc, rl = _oracle_packed(buf, off, 45, 1)
        gpu_session.run_host(buf, off, 45, 1)
        res = gpu_session.fetch(45)
        assert res.stats.count_path == eulerhip.EC_PATH_GENERAL
        if maxb:
            assert res.stats.table_retries >= 1
        assert res.stats.n_positions == ref["n_positions"]
        assert res.contig_bytes == ref["contig_chars"] and res.links == rl


@pytest.mark.parametrize("k,sbits", [(51, 2), (45, 1), (63, 3)])
def test_wide_third_level_vs_oracle(gpu_session, monkeypatch, k, sbits):
    """k > 32 past 2^14 bucket tables (config 5: 2e8 keys): every fine bucket split again into
    2^sbits fixed-capacity sub-buckets (k_refine with fcap) counted in 1664-slot tables; forced
    here on small inputs"""
    monkeypatch.setenv("EULERHIP_WIDE_L3", str(sbits))
    buf, off = make_reads(60_000, 25_000, 150, 70 + k, err=0.003)
    ref, rc, rl = _oracle_packed(buf, off, k, 1, True)
    gpu_session.run_host(buf, off, k, 1, eulerhip.EC_FLAG_WANT_DICT)
    res = gpu_session.fetch(k, True)
    assert res.stats.count_path == eulerhip.EC_PATH_PARTITIONED
    assert res.stats.n_buckets == (1 << 14) << sbits
    assert res.contig_bytes == ref["contig_chars"] and res.links == rl
    assert [[x, c] for x, c in res.dict_items] == ref["d"]


@pytest.mark.parametrize("case", [c for c in CASES32 if c["k"] >= 8], ids=lambda c: c["name"])
def test_golden_join_links(gpu_session, monkeypatch, case):
    """links by the (k-1)-mer half-edge join (join_w.h; 64-bit records for k <= 32, 128-bit
    above), forced at any size: golden vectors of the imported reference"""
    monkeypatch.setenv("EULERHIP_JOIN_LINKS", "1")
    res = gpu_session.assemble(case["reads"], case["k"], case["limit"], want_dict=True)
    assert [[x, c] for x, c in res.dict_items] == case["d"]
    assert res.contigs == case["contigs"] and res.links == case["links"]


@pytest.mark.parametrize("k", [31, 51])
def test_join_links_overflow_falls_back(gpu_session, monkeypatch, k):
    """a join level region past its capacity: the probe kernels, gated on the device-side flag,
    rewrite every successor (no host round trip decides it)"""
    monkeypatch.setenv("EULERHIP_JOIN_LINKS", "1")
    monkeypatch.setenv("EULERHIP_JOIN_CAP", "64")
    buf, off = make_reads(30_000, 10_000, 120, 800 + k, err=0.003)
    ref, rc, rl = _oracle_packed(buf, off, k, 1, True)
    gpu_session.run_host(buf, off, k, 1, eulerhip.EC_FLAG_WANT_DICT)
    res = gpu_session.fetch(k, True)
    assert res.contig_bytes == ref["contig_chars"] and res.links == rl
    assert [[x, c] for x, c in res.dict_items] == ref["d"] and res.stats.n_dict == ref["n_dict"]


@pytest.mark.parametrize("k", [8, 15, 16, 21, 22, 31, 32])
def test_join_links_vs_oracle(gpu_session, monkeypatch, k):
    """64-bit half-edge join against the oracle on error-rich reads with N (the window-record
    count paths it serves by default from 4e6 keys), both parities of k; and the probe path"""
    buf, off = make_reads(60_000, 30_000, 100, 500 + k, err=0.006, n_rate=0.0005)
    ref, rc, rl = _oracle_packed(buf, off, k, 1)
    for mode in ("1", "0"):
        monkeypatch.setenv("EULERHIP_JOIN_LINKS", mode)
        gpu_session.run_host(buf, off, k, 1)
        res = gpu_session.fetch(k)
        assert res.contig_bytes == ref["contig_chars"] and res.links == rl, mode
    monkeypatch.setenv("EULERHIP_JOIN_LINKS", "1")
    reads = _low_complexity_reads(300, 140, 40 + k)
    d, r, g = oracle.assemble(reads, k, 1)
    res = gpu_session.assemble(reads, k, 1, want_dict=True)
    assert [[x, c] for x, c in res.dict_items] == d and res.contigs == r and res.links == g


@pytest.mark.parametrize("k", [33, 34, 40, 51, 62, 63])
def test_wide_join_links_vs_oracle(gpu_session, monkeypatch, k):
    """the half-edge join against the oracle: k = 33 (32-base junctions), even k (palindromic
    k-mers), odd k (palindromic (k-1)-mer junctions), random reads with errors and tandem
    repeats; and the probe path (EULERHIP_JOIN_LINKS=0) on the same input"""
    buf, off = make_reads(40_000, 15_000, 150, 300 + k, err=0.004)
    ref, rc, rl = _oracle_packed(buf, off, k, 1)
    for mode in ("1", "0"):
        monkeypatch.setenv("EULERHIP_JOIN_LINKS", mode)
        gpu_session.run_host(buf, off, k, 1)
        res = gpu_session.fetch(k)
        assert res.contig_bytes == ref["contig_chars"] and res.links == rl, mode
    monkeypatch.setenv("EULERHIP_JOIN_LINKS", "1")
    reads = _low_complexity_reads(300, 140, 90 + k)
    d, r, g = oracle.assemble(reads, k, 1)
    res = gpu_session.assemble(reads, k, 1, want_dict=True)
    assert [[x, c] for x, c in res.dict_items] == d and res.contigs == r and res.links == g


def test_wide_third_level_overflow_falls_back(gpu_session, monkeypatch):
    """a third-level sub-bucket past its capacity drops nothing silently: the call is redone on
    the HBM table"""
    monkeypatch.setenv("EULERHIP_WIDE_L3", "2")
    monkeypatch.setenv("EULERHIP_WIDE_L3_CAP", "8")
    buf, off = make_reads(40_000, 20_000, 150, 91, err=0.002)
    ref, rc, rl = _oracle_packed(buf, off, 51, 1)
    gpu_session.run_host(buf, off, 51, 1)
    res = gpu_session.fetch(51)
    assert res.stats.count_path == eulerhip.EC_PATH_GENERAL and res.stats.table_retries >= 1
    assert res.contig_bytes == ref["contig_chars"] and res.links == rl


@pytest.mark.parametrize("pmax,lim", [(2, 1), (3, 1), (3, 0), (2, -1)])
def test_filter_bucket_parts_vs_oracle(gpu_session, monkeypatch, pmax, lim):
    """buckets split into 2^pmax part tables (hash bits 11..; SolidIndex::npb), as for genomes
    past ~2·10^7 solid k-mers, forced here on small inputs"""
    monkeypatch.setenv("EULERHIP_FORCE_FILTER", "1")
    monkeypatch.setenv("EULERHIP_FILTER_PMAX", str(pmax))
    monkeypatch.setenv("EULERHIP_FILTER_PMIN", str(pmax))
    for k in (31, 22):
        buf, off = make_reads(60_000, 20_000, 100, 900 + pmax + k, err=0.004, n_rate=0.001)
        ref, rc, rl = _oracle_packed(buf, off, k, lim, True)
        gpu_session.run_host(buf, off, k, lim, eulerhip.EC_FLAG_WANT_DICT)
        res = gpu_session.fetch(k, True)
        assert res.stats.count_path == eulerhip.EC_PATH_PARTITIONED
        assert res.contig_bytes == ref["contig_chars"] and res.links == rl, (k, pmax, lim)
        assert [[x, c] for x, c in res.dict_items] == ref["d"]


# ---- fixed-capacity runs (count_v2.h) ----------------------------------------------------------
@pytest.mark.parametrize("k", [11, 16, 21, 31, 32])
def test_v2_skew_falls_back_vs_oracle(gpu_session, k):
    """tandem repeats and homopolymers of one length: heavy keys overfill a (bucket, group) run or
    a final bucket; the call is redone on the exact path with the same results"""
    reads = _low_complexity_reads(3000, 100, 70 + k)
    d, r, g = oracle.assemble(reads, k, 1)
    res = gpu_session.assemble(reads, k, 1, want_dict=True)
    assert res.stats.count_path in (eulerhip.EC_PATH_PARTITIONED, eulerhip.EC_PATH_GENERAL)
    assert [[x, c] for x, c in res.dict_items] == d and res.contigs == r and res.links == g


@pytest.mark.parametrize("L,k", [(40, 11), (63, 31), (100, 17), (111, 27), (150, 31), (159, 32), (200, 31)])
def test_v2_read_lengths_vs_oracle(gpu_session, monkeypatch, L, k):
    """wave tiles of 64 reads staged in 4, 7 or 10 KiB per wave; longer reads take the exact path"""
    monkeypatch.setenv("EULERHIP_NO_SK2", "1")
    buf, off = make_reads(40_000, 9_000 - 30 * L, L, 3000 + L + k, err=0.003)
    ref, rc, rl = _oracle_packed(buf, off, k, 1, True)
    gpu_session.run_host(buf, off, k, 1, eulerhip.EC_FLAG_WANT_DICT)
    res = gpu_session.fetch(k, True)
    assert res.stats.count_variant == (1 if L <= 159 else 0)
    assert res.stats.n_positions == ref["n_positions"]
    assert [[x, c] for x, c in res.dict_items] == ref["d"]
    assert res.contig_bytes == ref["contig_chars"] and res.links == rl


@pytest.mark.parametrize("pmax,lim", [(2, 1), (3, 0)])
def test_v2_filter_parts_vs_oracle(gpu_session, monkeypatch, pmax, lim):
    """seen-twice filter + part tables over the fixed-capacity final buckets (count_sk2.h
    declines inputs that need the filter)"""
    monkeypatch.setenv("EULERHIP_FORCE_FILTER", "1")
    monkeypatch.setenv("EULERHIP_FILTER_PMAX", str(pmax))
    monkeypatch.setenv("EULERHIP_FILTER_PMIN", str(pmax))
    buf, off = make_reads(60_000, 20_000, 100, 950 + pmax, err=0.004)
    ref, rc, rl = _oracle_packed(buf, off, 31, lim, True)
    gpu_session.run_host(buf, off, 31, lim, eulerhip.EC_FLAG_WANT_DICT)
    res = gpu_session.fetch(31, True)
    assert res.stats.count_variant == 1
    assert res.contig_bytes == ref["contig_chars"] and res.links == rl
    assert [[x, c] for x, c in res.dict_items] == ref["d"]


@pytest.mark.parametrize("sk2", [False, True])
def test_v2_read_base_and_short_reads_vs_oracle(gpu_session, monkeypatch, sk2):
    """reads shorter than k (any length) beside one windowed length; a non-multiple-of-64 count"""
    if not sk2:
        monkeypatch.setenv("EULERHIP_NO_SK2", "1")
    rng = np.random.default_rng(5)
    g = "".join("ACGT"[x] for x in rng.integers(0, 4, 20_000))
    reads = []
    for i in range(7_777):
        L = 90 if rng.random() < 0.8 else int(rng.integers(0, 31))
        p = int(rng.integers(0, len(g) - L))
        reads.append(g[p:p + L])
    d, r, gl = oracle.assemble(reads, 31, 1)
    res = gpu_session.assemble(reads, 31, 1, want_dict=True)
    assert res.stats.count_variant == (3 if sk2 else 1)
    assert [[x, c] for x, c in res.dict_items] == d and res.contigs == r and res.links == gl


# ---- 10-byte records (count_v2.h R10: hashed-key remnants, relative read ids) -------------------
@pytest.mark.parametrize("g,n,L,seed,err,k", [
    (20_000, 4_000, 100, 1, 0.0, 31), (50_000, 20_000, 100, 2, 0.005, 31), (30_000, 10_000, 80, 3, 0.002, 25),
    (5_000, 5_000, 60, 4, 0.01, 20), (200_000, 60_000, 100, 6, 0.0, 32), (40_000, 30_000, 150, 7, 0.003, 16),
    (30_000, 9_000, 120, 8, 0.002, 22), (10_000, 3_333, 64, 9, 0.0, 17)])
def test_r10_vs_oracle(gpu_session, monkeypatch, g, n, L, seed, err, k):
    monkeypatch.setenv("EULERHIP_V2_R10", "1")
    monkeypatch.setenv("EULERHIP_NO_SK2", "1")
    buf, off = make_reads(g, n, L, 4000 + seed, err=err)
    want_dict = g <= 50_000
    ref, rc, rl = _oracle_packed(buf, off, k, 1, want_dict)
    gpu_session.run_host(buf, off, k, 1, eulerhip.EC_FLAG_WANT_DICT if want_dict else 0)
    res = gpu_session.fetch(k, want_dict)
    assert res.stats.count_variant == 2 and res.stats.record_bytes == 10
    assert res.stats.n_positions == ref["n_positions"] and res.stats.n_dict == ref["n_dict"]
    assert res.contig_bytes == ref["contig_chars"] and res.links == rl
    if want_dict:
        assert [[x, c] for x, c in res.dict_items] == ref["d"]


@pytest.mark.parametrize("rs", ["8", "16", "32"])
def test_r10_slices_vs_oracle(gpu_session, monkeypatch, rs):
    """the refine over 8..32 group slices per coarse bucket"""
    monkeypatch.setenv("EULERHIP_V2_R10", "1")
    monkeypatch.setenv("EULERHIP_NO_SK2", "1")
    monkeypatch.setenv("EULERHIP_REFINE_RS", rs)
    buf, off = make_reads(60_000, 40_000, 100, 4100 + int(rs), err=0.003)
    ref, rc, rl = _oracle_packed(buf, off, 27, 1, True)
    gpu_session.run_host(buf, off, 27, 1, eulerhip.EC_FLAG_WANT_DICT)
    res = gpu_session.fetch(27, True)
    assert res.stats.count_variant == 2
    assert [[x, c] for x, c in res.dict_items] == ref["d"]
    assert res.contig_bytes == ref["contig_chars"] and res.links == rl


@pytest.mark.parametrize("lim,pmax", [(1, 0), (0, 0), (2, 0), (1, 2), (0, 3)])
def test_r10_filter_and_limits_vs_oracle(gpu_session, monkeypatch, lim, pmax):
    """seen-twice filter / part tables and other limits over 10-byte records"""
    monkeypatch.setenv("EULERHIP_V2_R10", "1")
    monkeypatch.setenv("EULERHIP_NO_SK2", "1")
    if pmax:
        monkeypatch.setenv("EULERHIP_FORCE_FILTER", "1")
        monkeypatch.setenv("EULERHIP_FILTER_PMAX", str(pmax))
        monkeypatch.setenv("EULERHIP_FILTER_PMIN", str(pmax))
    buf, off = make_reads(40_000, 15_000, 100, 4200 + lim + pmax, err=0.004)
    for k in (31, 24):
        ref, rc, rl = _oracle_packed(buf, off, k, lim, True)
        gpu_session.run_host(buf, off, k, lim, eulerhip.EC_FLAG_WANT_DICT)
        res = gpu_session.fetch(k, True)
        assert res.stats.count_variant == 2
        assert [[x, c] for x, c in res.dict_items] == ref["d"], (k, lim, pmax)
        assert res.contig_bytes == ref["contig_chars"] and res.links == rl, (k, lim, pmax)


def test_r10_palindromes_vs_oracle(gpu_session, monkeypatch):
    """even k: palindromic k-mers (inserted twice by build) recovered from the hashed keys"""
    monkeypatch.setenv("EULERHIP_V2_R10", "1")
    monkeypatch.setenv("EULERHIP_NO_SK2", "1")
    reads = _low_complexity_reads(1500, 100, 77)
    for k in (16, 20, 24, 32):
        d, r, g = oracle.assemble(reads, k, 1)
        res = gpu_session.assemble(reads, k, 1, want_dict=True)
        assert [[x, c] for x, c in res.dict_items] == d and res.contigs == r and res.links == g, k


# ---- super-k-mer records (count_sk2.h) -------------------------------------------------------
SK2 = [(20_000, 4_000, 100, 1, 0.0, 31), (50_000, 20_000, 100, 2, 0.002, 31), (30_000, 10_000, 80, 3, 0.001, 25),
       (200_000, 60_000, 100, 6, 0.0, 32), (30_000, 9_000, 120, 8, 0.0, 22), (10_000, 3_333, 64, 9, 0.0, 21),
       (40_000, 12_000, 150, 10, 0.001, 27), (5_000, 2_000, 40, 11, 0.0, 21), (8_000, 700, 31, 12, 0.0, 31)]


@pytest.mark.parametrize("g,n,L,seed,err,k", SK2)
def test_sk2_vs_oracle(gpu_session, g, n, L, seed, err, k):
    """16-byte super-k-mer records: partition by minimizer, refine, rolled-out bucket tables"""
    buf, off = make_reads(g, n, L, 5000 + seed, err=err)
    want_dict = g <= 50_000
    ref, rc, rl = _oracle_packed(buf, off, k, 1, want_dict)
    gpu_session.run_host(buf, off, k, 1, eulerhip.EC_FLAG_WANT_DICT if want_dict else 0)
    res = gpu_session.fetch(k, want_dict)
    assert res.stats.count_variant == 3 and res.stats.record_bytes == 16
    assert 0 < res.stats.n_records <= res.stats.n_positions
    assert res.stats.n_positions == ref["n_positions"] and res.stats.n_dict == ref["n_dict"]
    assert res.contig_bytes == ref["contig_chars"] and np.array_equal(res.contig_offsets, ref["contig_offsets"])
    assert res.links == rl
    if want_dict:
        assert [[x, c] for x, c in res.dict_items] == ref["d"]


@pytest.mark.parametrize("rs", ["1", "8", "32"])
def test_sk2_slices_and_limits_vs_oracle(gpu_session, monkeypatch, rs):
    """the super-k-mer refine over 1..32 group slices per coarse bucket; limits -1 .. 5"""
    monkeypatch.setenv("EULERHIP_REFINE_RS", rs)
    buf, off = make_reads(40_000, 15_000, 100, 5100 + int(rs), err=0.003)
    for k, lim in ((31, 1), (24, 0), (29, 2), (31, -1), (26, 5)):
        ref, rc, rl = _oracle_packed(buf, off, k, lim, True)
        gpu_session.run_host(buf, off, k, lim, eulerhip.EC_FLAG_WANT_DICT)
        res = gpu_session.fetch(k, True)
        assert res.stats.count_variant == 3, (k, lim)
        assert [[x, c] for x, c in res.dict_items] == ref["d"], (k, lim)
        assert res.contig_bytes == ref["contig_chars"] and res.links == rl, (k, lim)


@pytest.mark.parametrize("cap,variant", [("400", 3), ("8", None)])
def test_sk2_record_overflow_list_vs_oracle(gpu_session, monkeypatch, cap, variant):
    """k_skbucket3 with its record-table claims capped (EULERHIP_SK2_CLAIM): records past the cap
    go to the overflow list and are rolled out one by one (cap 400 of ~530 distinct records a
    bucket); a full list (cap 8) redoes the call on another path -- exact either way"""
    monkeypatch.setenv("EULERHIP_SK2_CLAIM", cap)
    buf, off = make_reads(20_000, 4_000, 100, 5300, err=0.0)
    ref, rc, rl = _oracle_packed(buf, off, 31, 1, True)
    gpu_session.run_host(buf, off, 31, 1, eulerhip.EC_FLAG_WANT_DICT)
    res = gpu_session.fetch(31, True)
    if variant is not None:
        assert res.stats.count_variant == variant
    assert [[x, c] for x, c in res.dict_items] == ref["d"]
    assert res.contig_bytes == ref["contig_chars"] and res.links == rl


@pytest.mark.parametrize("g,n,L,seed", [(22_000, 80_000, 60, 1), (23_000, 60_000, 50, 2), (21_000, 90_000, 70, 3)])
def test_sk2_record_table_full_default_cap_vs_oracle(gpu_session, monkeypatch, capfd, g, n, L, seed):
    """k_skbucket3 at its default claim cap with buckets of more than 832 distinct records (the
    compact arrays' size, RS / 2): short reads at high coverage, so nearly every start position
    adds two read-truncated records.  The cap must be a hard bound -- records past it go to the
    overflow list, never past the compact arrays (a racing wave used to overshoot)."""
    monkeypatch.setenv("EULERHIP_SK2_STATS", "1")
    buf, off = make_reads(g, n, L, 5400 + seed, err=0.0)
    ref, rc, rl = _oracle_packed(buf, off, 31, 1, True)
    capfd.readouterr()
    gpu_session.run_host(buf, off, 31, 1, eulerhip.EC_FLAG_WANT_DICT)
    res = gpu_session.fetch(31, True)
    err = capfd.readouterr().err
    assert [[x, c] for x, c in res.dict_items] == ref["d"]
    assert res.contig_bytes == ref["contig_chars"] and res.links == rl
    most = [int(l.rsplit(" ", 1)[1]) for l in err.splitlines() if l.startswith("k_skbucket3:")]
    assert res.stats.count_variant == 3 and most, err
    assert most[-1] > 832, err


@pytest.mark.parametrize("k", [31, 24])
def test_sk2_large_table_kernel_vs_oracle(gpu_session, monkeypatch, k):
    """EULERHIP_NO_SKB3: k_skbucket's 2048-slot tables (the plan for inputs past ~6 M keys)"""
    monkeypatch.setenv("EULERHIP_NO_SKB3", "1")
    buf, off = make_reads(50_000, 15_000, 100, 5310 + k, err=0.001)
    ref, rc, rl = _oracle_packed(buf, off, k, 1, True)
    gpu_session.run_host(buf, off, k, 1, eulerhip.EC_FLAG_WANT_DICT)
    res = gpu_session.fetch(k, True)
    assert res.stats.count_variant == 3
    assert [[x, c] for x, c in res.dict_items] == ref["d"]
    assert res.contig_bytes == ref["contig_chars"] and res.links == rl


def test_sk2_palindromes_vs_oracle(gpu_session):
    """even k: palindromic k-mers (inserted twice by build) inside super-k-mers"""
    rng = np.random.default_rng(17)
    comp = str.maketrans("ACGT", "TGCA")
    parts = []
    for _ in range(60):
        parts.append("".join("ACGT"[x] for x in rng.integers(0, 4, 300)))
        x = "".join("ACGT"[x] for x in rng.integers(0, 4, 16))
        parts.append(x + x.translate(comp)[::-1])  # a 32-base palindrome: its centred even k-mers are too
    g = "".join(parts)
    reads = []
    for _ in range(4000):
        p = int(rng.integers(0, len(g) - 100))
        r = g[p:p + 100]
        reads.append(r if rng.random() < 0.5 else r.translate(comp)[::-1])
    for k in (22, 24, 32):
        d, r, gl = oracle.assemble(reads, k, 1)
        res = gpu_session.assemble(reads, k, 1, want_dict=True)
        assert res.stats.count_variant == 3, k
        assert [[x, c] for x, c in res.dict_items] == d and res.contigs == r and res.links == gl, k


def test_sk2_declines_filter_and_window_records(gpu_session, monkeypatch):
    """inputs that need the seen-twice filter, and EC_FLAG_WINDOW_RECORDS, count window records"""
    buf, off = make_reads(30_000, 8_000, 100, 5200, err=0.004)
    ref, rc, rl = _oracle_packed(buf, off, 31, 1, True)
    gpu_session.run_host(buf, off, 31, 1, eulerhip.EC_FLAG_WANT_DICT | eulerhip.EC_FLAG_WINDOW_RECORDS)
    res = gpu_session.fetch(31, True)
    assert res.stats.count_variant == 1
    assert [[x, c] for x, c in res.dict_items] == ref["d"] and res.links == rl
    monkeypatch.setenv("EULERHIP_FORCE_FILTER", "1")
    gpu_session.run_host(buf, off, 31, 1, eulerhip.EC_FLAG_WANT_DICT)
    res = gpu_session.fetch(31, True)
    assert res.stats.count_variant == 1
    assert [[x, c] for x, c in res.dict_items] == ref["d"] and res.links == rl


def test_sk2_fast_path_fallbacks_vs_oracle(gpu_session):
    """the prescan-free super-k-mer partition takes its read length from the first read and
    hands anything else back to the prescan path: a longer read later on, an N in the last read,
    reads shorter than k beside the windowed ones"""
    rng = np.random.default_rng(77)
    g = "".join("ACGT"[x] for x in rng.integers(0, 4, 30_000))

    def sample(L):
        p = int(rng.integers(0, len(g) - L))
        return g[p:p + L]

    base = [sample(90) for _ in range(5_000)]
    cases = {
        "longer_later": base[:2_500] + [sample(140)] + base[2_500:],
        "n_last": base[:-1] + [base[-1][:40] + "N" + base[-1][41:]],
        "short_reads": base[:100] + [sample(int(rng.integers(1, 31))) for _ in range(300)] + base[100:],
    }
    for name, reads in cases.items():
        d, r, gl = oracle.assemble(reads, 31, 1)
        res = gpu_session.assemble(reads, 31, 1, want_dict=True)
        assert [[x, c] for x, c in res.dict_items] == d and res.contigs == r and res.links == gl, name
        if name == "short_reads":
            assert res.stats.count_variant == 3, name
        else:
            assert res.stats.count_variant != 3, name


def test_sk2_cached_read_length_same_buffers(gpu_session):
    """run_device reuses the read length of its last call on the same offsets pointer and read
    count (no host round trip); new reads of another length in the same device buffers fail the
    partition's own length check and are redone correctly, as are N-bearing reads"""
    import torch

    rng = np.random.default_rng(78)
    g = rng.integers(0, 4, 40_000, dtype=np.uint8)
    n = 4_000

    def reads_of(L, with_n=False):
        st = rng.integers(0, len(g) - 120, n)
        b = np.frombuffer(b"ACGT", np.uint8)[g[st[:, None] + np.arange(L)[None, :]]].reshape(-1).copy()
        if with_n:
            b[L * 17 + 5] = ord("N")
        return b, np.arange(n + 1, dtype=np.uint64) * np.uint64(L)

    d_buf = torch.zeros(n * 100, dtype=torch.uint8, device="cuda")
    d_off = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    for L, with_n in ((100, False), (100, False), (90, False), (90, False), (100, True), (100, False)):
        buf, off = reads_of(L, with_n)
        d_buf[: buf.size].copy_(torch.from_numpy(buf))
        d_off.copy_(torch.from_numpy(off.astype(np.int64)))
        torch.cuda.synchronize()
        gpu_session.run_device(d_buf.data_ptr(), d_off.data_ptr(), n, 31, 1, 0)
        res = gpu_session.fetch(31)
        ref = oracle.assemble_packed(buf, off, 31, 1)
        assert res.contig_bytes == ref["contig_chars"] and res.links == oracle.unpack_links(ref), (L, with_n)
        assert res.stats.n_positions == ref["n_positions"], (L, with_n)
