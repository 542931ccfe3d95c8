"""Seeded synthetic read sets: iid uniform ACGT genome, read starts uniform,
50% reverse-complemented, optional substitution errors / N bases / circular genome.
Shared by tests and bench.py (numpy PCG64, seed = 20261015 + config#)."""
import numpy as np

LUT = np.frombuffer(b"ACGT", dtype=np.uint8)


def make_genome(genome_len, seed):
    """The genome make_reads(genome_len, ..., seed) samples from, as ASCII bytes."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return LUT[rng.integers(0, 4, genome_len, dtype=np.uint8)].tobytes()


def read_starts(genome_len, n_reads, read_len, seed):
    """Genome start of every read of make_reads(genome_len, n_reads, read_len, seed) (linear,
    part None): the same draws in the same order."""
    rng = np.random.Generator(np.random.PCG64(seed))
    rng.integers(0, 4, genome_len, dtype=np.uint8)
    return rng.integers(0, max(1, genome_len - read_len + 1), n_reads)


def make_reads(genome_len, n_reads, read_len, seed, err=0.0, n_rate=0.0, circular=False, rc_frac=0.5,
               part=None, rows=None):
    """Returns (buf uint8[n_reads*read_len], offsets uint64[n_reads+1]) of ASCII reads.
    part = i >= 1: the i-th further read set of the same genome (weak-scaled multi-GPU bench:
    rank i samples its own n_reads from the genome of `seed`; part None / 0 = the seed's reads).
    rows = (a, b): only reads a..b-1 of that set (offsets from 0): a strong-scaled shard built
    without the other ranks' reads (exact for error- and N-free sets, whose per-read random
    draws all precede the reads; otherwise the whole set is built and sliced)."""
    if rows is not None:
        a, b = int(rows[0]), int(rows[1])
        if err > 0 or n_rate > 0:
            buf, off = make_reads(genome_len, n_reads, read_len, seed, err, n_rate, circular, rc_frac, part)
            return (buf[a * read_len:b * read_len].copy(),
                    np.arange(b - a + 1, dtype=np.uint64) * np.uint64(read_len))
    rng = np.random.Generator(np.random.PCG64(seed))
    g = rng.integers(0, 4, genome_len, dtype=np.uint8)
    if part:
        rng = np.random.Generator(np.random.PCG64([seed, int(part)]))
    if circular:
        g2 = np.concatenate([g, g[:read_len]])
        starts = rng.integers(0, genome_len, n_reads)
    else:
        g2 = g
        starts = rng.integers(0, max(1, genome_len - read_len + 1), n_reads)
    flip = rng.random(n_reads) < rc_frac
    r0, r1 = (0, n_reads) if rows is None else (int(rows[0]), int(rows[1]))
    out = np.empty((r1 - r0, read_len), dtype=np.uint8)
    CH = 1 << 20
    for a in range(r0, r1, CH):
        b = min(r1, a + CH)
        idx = starts[a:b, None] + np.arange(read_len)[None, :]
        blk = g2[idx]
        f = flip[a:b]
        blk[f] = 3 - blk[f][:, ::-1]
        if err > 0:
            m = rng.random(blk.shape) < err
            blk[m] = (blk[m] + rng.integers(1, 4, int(m.sum()), dtype=np.uint8)) & 3
        chars = LUT[blk]
        if n_rate > 0:
            chars[rng.random(blk.shape) < n_rate] = ord("N")
        out[a - r0:b - r0] = chars
    offsets = np.arange(r1 - r0 + 1, dtype=np.uint64) * np.uint64(read_len)
    return out.reshape(-1), offsets
