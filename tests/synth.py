"""Seeded synthetic read sets: iid uniform ACGT genome, read starts uniform,
50% reverse-complemented, optional substitution errors / N bases / circular genome.
Shared by tests and bench.py (numpy PCG64, seed = 20261015 + config#)."""
import numpy as np

LUT = np.frombuffer(b"ACGT", dtype=np.uint8)


def make_genome(genome_len, seed):
    """The genome make_reads(genome_len, ..., seed) samples from, as ASCII bytes."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return LUT[rng.integers(0, 4, genome_len, dtype=np.uint8)].tobytes()


def make_reads(genome_len, n_reads, read_len, seed, err=0.0, n_rate=0.0, circular=False, rc_frac=0.5,
               part=None):
    """Returns (buf uint8[n_reads*read_len], offsets uint64[n_reads+1]) of ASCII reads.
    part = i >= 1: the i-th further read set of the same genome (weak-scaled multi-GPU bench:
    rank i samples its own n_reads from the genome of `seed`; part None / 0 = the seed's reads)."""
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
    out = np.empty((n_reads, read_len), dtype=np.uint8)
    CH = 1 << 20
    flip = rng.random(n_reads) < rc_frac
    for a in range(0, n_reads, CH):
        b = min(n_reads, a + CH)
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
        out[a:b] = chars
    offsets = np.arange(n_reads + 1, dtype=np.uint64) * np.uint64(read_len)
    return out.reshape(-1), offsets
