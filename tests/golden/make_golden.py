"""Generate the golden parity fixtures under tests/golden/ from the REAL reference.

This script is run once, in the build container only (it reads /root/reference,
which does not exist on the GPU box).  It imports the reference CPU assembler
`src/referenceassembler/referenceAssembler.py` (build:25, all_contigs:79) unchanged;
the module imports `dask.delayed` at :5 but never uses it (the decorator is
commented out at :134), so a one-line `sys.modules['dask']` stub stands in for
the missing dask package.  Nothing else from the reference is executed.

Fixtures written (all plain JSON, data only):
  g200.json      tests/g200reads.fa reads at k = 9, 11, 15, 20, 21 (BASELINE config 1)
  synthetic.json hand-shaped cases: linear, circular, repeats, tandem, N-containing,
                 even-k palindromes / hairpins, lowercase + IUPAC pass-through, limit variants
  fuzz.json      seeded random small cases (low-complexity alphabets force branching,
                 cycles, Moebius paths and palindromes)
  extended.json  reads with bytes outside {A,C,G,T,N} (soft-masked lowercase runs, IUPAC codes,
                 lowercase n): opaque symbols that are their own complement (twin:7-10), odd-k
                 palindromes, and k-mers with an opaque first symbol whose one fw neighbour has a
                 different single bw neighbour (one-way links, get_contig_forward:63-73);
                 cases where the reference's walk never returns are skipped (alarm)
  kat.json       known-answer values for the per-kernel rows (E1/E2/E3/H1) + the
                 pinned hash_tk.txt layout summary (src/hash_tk.txt)

Each assembler case stores: reads, k, limit, d (ordered [kmer, count] list = the
dict returned by build, in insertion order), contigs (all_contigs r) and links
(all_contigs G as [[fw links], [bw links]] per contig, each link [j, '+'|'-']).
"""
import json
import os
import sys
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def load_reference():
    sys.modules.setdefault("dask", types.SimpleNamespace(delayed=lambda f=None, **kw: f))
    sys.path.insert(0, os.path.join(REF, "src", "referenceassembler"))
    import referenceAssembler as ra  # noqa: E402
    return ra


def run_case(ra, reads, k, limit=1, name=""):
    d = ra.build(reads, k=k, limit=limit)
    G, r = ra.all_contigs(d, k)
    links = [[[list(x) for x in G[i][0]], [list(x) for x in G[i][1]]] for i in range(len(r))]
    return {"name": name, "k": k, "limit": limit, "reads": list(reads),
            "d": [[x, int(c)] for x, c in d.items()], "contigs": list(r), "links": links}


COMP = {"A": "T", "C": "G", "G": "C", "T": "A"}


def rc(s):
    return "".join(COMP.get(c, c) for c in reversed(s))


def sample_reads(rng, genome, n, L, circular=False, rc_frac=0.5):
    G = len(genome)
    out = []
    g2 = genome + genome if circular else genome
    for _ in range(n):
        if circular:
            s = int(rng.integers(0, G))
        else:
            s = int(rng.integers(0, max(1, G - L + 1)))
        r = g2[s:s + L]
        if rng.random() < rc_frac:
            r = rc(r)
        out.append(r)
    return out


def rand_seq(rng, n, alphabet="ACGT", p=None):
    return "".join(rng.choice(list(alphabet), size=n, p=p))


def synthetic_cases(ra):
    cases = []
    rng = np.random.default_rng(20261015)
    g = rand_seq(rng, 400)
    cases.append(run_case(ra, sample_reads(rng, g, 120, 40), 15, name="linear_k15"))
    cases.append(run_case(ra, sample_reads(rng, g, 120, 40), 21, name="linear_k21"))
    g = rand_seq(rng, 300)
    cases.append(run_case(ra, sample_reads(rng, g, 150, 35, circular=True), 13, name="circular_k13"))
    cases.append(run_case(ra, sample_reads(rng, g, 150, 35, circular=True), 12, name="circular_k12_even"))
    rep = rand_seq(rng, 40)
    g = rand_seq(rng, 100) + rep + rand_seq(rng, 120) + rep + rand_seq(rng, 80) + rc(rep) + rand_seq(rng, 60)
    cases.append(run_case(ra, sample_reads(rng, g, 200, 50), 17, name="repeats_k17"))
    unit = rand_seq(rng, 7)
    g = rand_seq(rng, 60) + unit * 12 + rand_seq(rng, 60)
    cases.append(run_case(ra, sample_reads(rng, g, 150, 30), 9, name="tandem_k9"))
    g = rand_seq(rng, 250)
    rs = sample_reads(rng, g, 120, 40)
    rs = ["".join("N" if rng.random() < 0.03 else c for c in r) for r in rs]
    rs += ["NNNN" + rs[0][4:], rs[1][:10] + "NN" + rs[1][12:], "N" * 30]
    cases.append(run_case(ra, rs, 11, name="with_N_k11"))
    # inverted repeat -> hairpins; even k -> palindromic k-mers
    arm = rand_seq(rng, 25)
    pal = rand_seq(rng, 5)
    pal = pal + rc(pal)  # 10-bp palindrome
    g = rand_seq(rng, 50) + arm + rand_seq(rng, 6) + rc(arm) + rand_seq(rng, 40) + pal + rand_seq(rng, 40)
    for k in (8, 10, 12, 9):
        cases.append(run_case(ra, sample_reads(rng, g, 120, 30), k, name=f"hairpin_pal_k{k}"))
    # lowercase + IUPAC pass through twin() unchanged (referenceAssembler.py:7-10)
    g = rand_seq(rng, 120)
    rs = sample_reads(rng, g, 60, 30, rc_frac=0.0)
    rs += ["acgtacgtacgtacgt", "ACGTRYACGTACGT", "acgtacgtacgtacgt"]
    cases.append(run_case(ra, rs, 7, name="extended_alphabet_k7"))
    g = rand_seq(rng, 200)
    rs = sample_reads(rng, g, 40, 30)
    for lim in (0, 2, 3):
        cases.append(run_case(ra, rs, 11, limit=lim, name=f"limit{lim}_k11"))
    # k = 32 (64-bit key boundary) and k = 31 (BASELINE k)
    g = rand_seq(rng, 500)
    cases.append(run_case(ra, sample_reads(rng, g, 200, 60), 31, name="linear_k31"))
    cases.append(run_case(ra, sample_reads(rng, g, 200, 60), 32, name="linear_k32"))
    # k > 32 (128-bit keys, BASELINE config 5 uses k = 51)
    g = rand_seq(rng, 600)
    cases.append(run_case(ra, sample_reads(rng, g, 200, 90), 51, name="linear_k51"))
    cases.append(run_case(ra, sample_reads(rng, g, 200, 90, circular=True), 40, name="circular_k40"))
    # degenerate inputs
    cases.append(run_case(ra, [], 5, name="empty"))
    cases.append(run_case(ra, ["ACG", "T", ""], 5, name="all_short"))
    cases.append(run_case(ra, ["AAAAAAAAAAAA", "TTTTTTTTTT"], 4, name="homopolymer_k4"))
    cases.append(run_case(ra, ["ACGTACGTACGT", "ACGTACGT"], 4, name="period2_pal_k4"))
    return cases


def fuzz_cases(ra, n=400):
    cases = []
    rng = np.random.default_rng(77)
    for i in range(n):
        k = int(rng.integers(2, 14))
        mode = i % 4
        if mode == 0:     # uniform
            g = rand_seq(rng, int(rng.integers(10, 120)))
        elif mode == 1:   # low complexity -> branching, cycles
            g = rand_seq(rng, int(rng.integers(10, 120)), "ACGT", p=[0.55, 0.15, 0.15, 0.15])
        elif mode == 2:   # two-letter alphabet -> palindromes / Moebius
            g = rand_seq(rng, int(rng.integers(10, 80)), "AT" if rng.random() < 0.5 else "CG")
        else:             # mixed with inverted repeats
            a = rand_seq(rng, int(rng.integers(3, 20)))
            g = rand_seq(rng, 5) + a + rand_seq(rng, int(rng.integers(0, 4))) + rc(a) + rand_seq(rng, 5)
        L = int(rng.integers(max(2, k - 1), k + 25))
        circ = bool(rng.random() < 0.3)
        rs = sample_reads(rng, g, int(rng.integers(1, 40)), L, circular=circ)
        if rng.random() < 0.15:
            rs = ["".join("N" if rng.random() < 0.05 else c for c in r) for r in rs]
        lim = 1 if rng.random() < 0.85 else int(rng.integers(0, 3))
        cases.append(run_case(ra, rs, k, limit=lim, name=f"fuzz{i}"))
    return cases


def extended_cases(ra, n=240):
    import signal

    def on_alarm(*a):
        raise TimeoutError

    signal.signal(signal.SIGALRM, on_alarm)
    cases = []
    rng = np.random.default_rng(4711)
    lower = str.maketrans("ACGT", "acgt")
    iupac = "RYKMSWBDHVrykmswbdhvn"
    i = 0
    skipped = 0
    while len(cases) < n:
        i += 1
        k = int(rng.integers(3, 14))
        mode = len(cases) % 5
        g = rand_seq(rng, int(rng.integers(20, 150)), "ACGT", p=[0.4, 0.2, 0.2, 0.2] if i % 3 == 0 else None)
        L = int(rng.integers(max(2, k), k + 25))
        circ = bool(rng.random() < 0.25)
        rs = sample_reads(rng, g, int(rng.integers(2, 40)), L, circular=circ)
        if mode == 0:    # soft-masked runs (lowercase), as in repeat-masked FASTA
            out = []
            for r in rs:
                if rng.random() < 0.6:
                    a = int(rng.integers(0, len(r) + 1))
                    b = int(rng.integers(a, len(r) + 1))
                    r = r[:a] + r[a:b].translate(lower) + r[b:]
                out.append(r)
            rs = out
        elif mode == 1:  # sparse IUPAC / lowercase n bytes
            rs = ["".join(iupac[int(rng.integers(0, len(iupac)))] if rng.random() < 0.04 else c for c in r)
                  for r in rs]
        elif mode == 2:  # one-way links: a read copy whose first base is lowercased
            out = list(rs)
            for r in rs[: max(1, len(rs) // 3)]:
                j = int(rng.integers(0, max(1, len(r) - k)))
                t = r[j:]
                if t:
                    out += [t[0].lower() + t[1:]] * int(rng.integers(1, 3))
            rs = out
        elif mode == 3:  # odd-k palindromes around an opaque middle symbol
            a = rand_seq(rng, int(rng.integers(1, 8)))
            mid = iupac[int(rng.integers(0, len(iupac)))]
            pal = a + mid + rc(a)
            rs = rs + [rand_seq(rng, 4) + pal + rand_seq(rng, 4) for _ in range(3)] + [pal] * 2
        else:            # everything at once, with N splits
            rs = ["".join("N" if rng.random() < 0.03 else
                          (c.lower() if rng.random() < 0.15 else
                           (iupac[int(rng.integers(0, len(iupac)))] if rng.random() < 0.03 else c)) for c in r)
                  for r in rs]
        rs = rs + rs[: len(rs) // 2]  # coverage: most k-mers seen twice
        lim = 1 if rng.random() < 0.85 else int(rng.integers(0, 3))
        signal.alarm(2)
        try:
            c = run_case(ra, rs, k, limit=lim, name=f"ext{len(cases)}")
        except TimeoutError:
            skipped += 1
            continue
        finally:
            signal.alarm(0)
        cases.append(c)
    return cases, skipped


def kat_values():
    """Known answers for the per-kernel rows, computed by the definitions in SURVEY §8a rows
    E1 (src/pyencode.py:43-74), E2 (:110-133), E3 intended (:171-207), H1 (src/pygpuhash.py:32-35),
    plus a compact summary of the reference's own TK dump src/hash_tk.txt (pygpuhash.py:309-311)."""
    reads = [l.strip() for l in open(os.path.join(REF, "tests", "g200reads.fa")) if not l.startswith(">")]
    buf = "".join(reads)
    tk = [int(x) for x in open(os.path.join(REF, "src", "hash_tk.txt")).read().split()]
    nb = len(tk) // 520
    buckets = []
    for b in range(nb):
        row = tk[b * 520:(b + 1) * 520]
        nz = [x for x in row if x != 0]
        # the dump is zero-initialised, so a bucket's used prefix is its sorted keys
        # (a literal zero key can only sit at rank 0)
        buckets.append(nz)
    return {
        "g200_reads": reads,
        "g200_buffer_len": len(buf),
        "encode": [["ACGT", 4, 27], [buf[0:11], 11, 3836979], [buf[0:21], 21, 4023364798006]],
        "hash_h": [[27, 10, 0], [2 ** 63 + 5, 1000, 333]],
        "hash_tk_bucket_count": nb,
        "hash_tk_buckets": buckets,
    }


def main():
    ra = load_reference()
    if len(sys.argv) > 1 and sys.argv[1] == "extended":  # (added in round 4: only this file)
        cases, skipped = extended_cases(ra)
        with open(os.path.join(HERE, "extended.json"), "w") as f:
            json.dump({"cases": cases, "skipped_nonterminating": skipped}, f, separators=(",", ":"))
        print("extended.json", len(cases), "cases;", skipped, "skipped (the reference's walk does not return)")
        return
    reads = [l.strip() for l in open(os.path.join(REF, "tests", "g200reads.fa")) if not l.startswith(">")]
    g200 = [run_case(ra, reads, k, name=f"g200_k{k}") for k in (9, 11, 15, 20, 21)]
    # also the even / small k on g200 (palindromes exist at even k)
    g200 += [run_case(ra, reads, k, name=f"g200_k{k}") for k in (4, 6, 7, 12, 16)]
    out = {
        "g200.json": {"source": "tests/g200reads.fa", "cases": g200},
        "synthetic.json": {"cases": synthetic_cases(ra)},
        "fuzz.json": {"cases": fuzz_cases(ra)},
        "kat.json": kat_values(),
    }
    for fn, obj in out.items():
        with open(os.path.join(HERE, fn), "w") as f:
            json.dump(obj, f, separators=(",", ":"))
        print(fn, os.path.getsize(os.path.join(HERE, fn)))


if __name__ == "__main__":
    main()
