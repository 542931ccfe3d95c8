import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "pycuda-euler_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import torch
import distributed, eulerhip
from synth import make_reads
nreads = int(sys.argv[1]); world = int(sys.argv[2])
buf, off = make_reads(4_600_000, nreads, 100, 20261019)
s = eulerhip.Session(0)
s.run_host(buf, off, 31, 1, 0)
ref = s.fetch(31)
print("fused: contigs", len(ref.contig_offsets) - 1, "solid", ref.stats.n_solid, flush=True)
engines = [distributed.HipEngine(0) for _ in range(world)]
for rep in range(2):
    res, P = distributed.local_sharded_assemble(engines, buf, off, 31, 1)
    print(rep, "sharded", world, "contigs", len(res.contig_offsets) - 1, "equal", res.contig_bytes == ref.contig_bytes, flush=True)
    for e in engines:
        st = e.stats()
        print("   solid", st.n_solid, "distinct", st.n_distinct, "path", st.count_path, "buckets", st.n_buckets, "retries", st.table_retries, flush=True)
