import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "pycuda-euler_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import torch
import distributed, oracle
from synth import make_reads
for world, nreads in ((8, 60000), (8, 1000000), (5, 60000)):
    buf, off = make_reads(200_000, nreads, 100, 77, err=0.001)
    engines = [distributed.HipEngine(0) for _ in range(world)]
    res, P = distributed.local_sharded_assemble(engines, buf, off, 31, 1)
    ref = oracle.assemble_packed(buf, off, 31, 1)
    print(world, nreads, "P", P, ref["n_positions"], "contigs", len(res.contig_offsets) - 1,
          len(ref["contig_offsets"]) - 1, "equal", res.contig_bytes == ref["contig_chars"], flush=True)
    for e in engines:
        st = e.stats()
        print("   solid", st.n_solid, "distinct", st.n_distinct, "path", st.count_path, "buckets", st.n_buckets, flush=True)
    for e in engines:
        e.sess.close()
