"""The bench's pipelined host-input loop alone (packed reads staged from page-locked memory while
the previous batch assembles: ec_stage_packed_host / ec_assemble_staged), for a rocprofv3 trace of
its copies and kernels.  Prints the per-step time of the loop."""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pycuda-euler_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def main():
    import torch

    import bench
    import eulerhip
    import ingest
    from synth import make_reads

    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    c = bench.CONFIGS["ecoli10m"]
    buf, off = make_reads(c["genome"], c["reads"], c["read_len"], c["seed"])
    tmp = tempfile.mkdtemp(prefix="ec_pipe_")
    fa = os.path.join(tmp, "reads.fa")
    bench.write_fasta(fa, buf, off)
    rs = ingest.ReadSet(fa, ingest.FASTA_RECORDS, threads=bench.host_threads(), packed=True)
    sess = eulerhip.Session(0)
    k = c["k"]
    for _ in range(3):
        rs.assemble(sess, k, 1, 0)
    rs.stage(sess)
    rs.stage(sess)
    for _ in range(3):
        sess.assemble_staged(k, 1, 0)
        rs.stage(sess)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        sess.assemble_staged(k, 1, 0)
        rs.stage(sess)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / steps * 1e3
    sess.assemble_staged(k, 1, 0)
    sess.assemble_staged(k, 1, 0)
    print("pipelined packed host input: %.3f ms / step (%d steps)" % (ms, steps), flush=True)
    rs.close()
    sess.close()


if __name__ == "__main__":
    main()
