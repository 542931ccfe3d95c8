"""The streaming (out-of-core) count on config 5's per-rank shape or larger: reads of the 200 Mbp
genome (150 bp, k = 51) counted chunk by chunk on one GPU (distributed.streaming_assemble), with
the device-buffer peak, torch's peak and the wall time of the whole assembly printed, and the
one-shot assembly of the same reads beside it (--oneshot)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "pycuda-euler_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=12_500_000)
    ap.add_argument("--genome", type=int, default=200_000_000)
    ap.add_argument("--len", type=int, default=150)
    ap.add_argument("--k", type=int, default=51)
    ap.add_argument("--chunk", type=int, default=4_000_000)
    ap.add_argument("--fold", type=int, default=2)
    ap.add_argument("--seed", type=int, default=20261015 + 5)
    ap.add_argument("--oneshot", action="store_true", help="also the one-shot single-GPU assembly")
    a = ap.parse_args()
    import torch

    import distributed
    import eulerhip
    from synth import make_reads

    buf, off = make_reads(a.genome, a.reads, a.len, a.seed)
    print("reads %d x %d bp, genome %d, k %d, chunk %d, fold %d" % (a.reads, a.len, a.genome, a.k, a.chunk, a.fold),
          flush=True)
    total = torch.cuda.mem_get_info()[1]
    eng = distributed.HipEngine(0)
    torch.cuda.reset_peak_memory_stats()
    eulerhip.mem_stats(reset=True)
    st = {}
    t0 = time.time()
    res, P = distributed.streaming_assemble(eng, buf, off, a.k, 1, chunk_reads=a.chunk, fold=a.fold, stats=st)
    torch.cuda.synchronize()
    t = time.time() - t0
    held, peak = eulerhip.mem_stats()
    print("streaming: %.2f s  positions %d  solid %d  contigs %d  chunks %d folds %d  session buffers peak %.1f GB, "
          "torch peak %.1f GB, device %.1f GB" % (t, P, st["solid"], len(res.contig_offsets) - 1, st["chunks"],
                                                  st["folds"], peak / 1e9, torch.cuda.max_memory_allocated() / 1e9,
                                                  total / 1e9), flush=True)
    eng.sess.close()
    contigs = res.contig_bytes
    if a.oneshot:
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats()
        eulerhip.mem_stats(reset=True)
        s = eulerhip.Session(0)
        t0 = time.time()
        s.run_host(buf, off, a.k, 1)
        r2 = s.fetch(a.k)
        t = time.time() - t0
        held, peak = eulerhip.mem_stats()
        print("one-shot: %.2f s (incl. the H2D copy of the reads)  contigs %d  session buffers peak %.1f GB  same "
              "contigs: %s" % (t, len(r2.contig_offsets) - 1, peak / 1e9, r2.contig_bytes == contigs), flush=True)
        s.close()


if __name__ == "__main__":
    main()
