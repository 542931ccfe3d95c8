"""euler_run -- command-line assembler: read file -> contigs (FASTA) and GFA, on 1..8 GPUs.

Replaces the reference's distribution front-end, Spark mapPartitions(assemble2) over read
partitions (src/cli_spark_gpu.py:37), whose per-partition contigs were never merged (SURVEY
§8f row 3), with one process per GPU and a correct global result:

    python pycuda-euler_amd/euler_run.py -i reads.fa -k 31 -o contigs.fa --gfa graph.gfa
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 pycuda-euler_amd/euler_run.py -i reads.fq -k 31 ...

Every rank parses the file with the native reader (csrc/ingest.cpp) and moves only its
contiguous read shard to its GPU; the counts are exchanged by owner with one RCCL
all-to-all-v, owners merge and filter, and the graph is built, ranked and emitted in owner
segments (distributed.sharded_assemble: junction join, partitioned finish).  Rank 0 writes
the outputs.  With one process the fused single-GPU path runs instead (--sharded: the sharded
path at any world size).  --backend gloo with --device N puts every rank on GPU N, the
collectives staged through host memory (tests: several ranks of the real engine on one GPU).
Contigs equal referenceAssembler.all_contigs(build(reads, k, limit), k) with reads parsed as
--fasta-mode says.
"""
import argparse
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def main(argv=None):
    ap = argparse.ArgumentParser(description="MI355X de Bruijn unitig assembler")
    ap.add_argument("-i", "--input", required=True, help="FASTA / FASTQ read file")
    ap.add_argument("-k", type=int, default=31, help="k-mer (node) length, 1..63")
    ap.add_argument("--limit", type=int, default=1, help="keep k-mers seen more than this many times")
    ap.add_argument("-o", "--output", default="", help="contig FASTA ('>contig%%d' records)")
    ap.add_argument("--gfa", default="", help="GFA 1 output")
    ap.add_argument("--fasta-mode", choices=["records", "lines"], default="records",
                    help="records: SeqIO-style multi-line records; lines: one read per line (src/eulercuda.py)")
    ap.add_argument("--threads", type=int, default=0, help="ingest threads (0: up to 16)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="torch.distributed backend (nccl = RCCL over xGMI; gloo stages through host memory)")
    ap.add_argument("--device", type=int, default=-1, help="GPU of every rank (default: LOCAL_RANK)")
    ap.add_argument("--sharded", action="store_true", help="the sharded path even with one process")
    a = ap.parse_args(argv)

    import torch

    import distributed
    import eulerhip
    import ingest

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0")) if a.device < 0 else a.device
    torch.cuda.set_device(local)
    t0 = time.time()
    rs = ingest.ReadSet(a.input, None, a.threads, a.fasta_mode)
    nreads = len(rs)
    lo, hi = distributed.shard_range(nreads, rank, world)
    buf, off = rs.packed(lo, hi - lo)
    rs.close()
    t_ingest = time.time() - t0
    d_buf = torch.from_numpy(buf if len(buf) else np.zeros(1, np.uint8)).cuda()
    d_off = torch.from_numpy(off.astype(np.int64)).cuda()
    torch.cuda.synchronize()
    t1 = time.time()
    sharded = world > 1 or a.sharded
    if not sharded:
        sess = eulerhip.Session(local, stream=torch.cuda.current_stream().cuda_stream)
        sess.run_device(d_buf.data_ptr(), d_off.data_ptr(), hi - lo, a.k, a.limit, 0)
        res = sess.fetch(a.k)
        P = res.stats.n_positions
    else:
        import torch.distributed as dist

        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
        eng = distributed.HipEngine(local, stream=torch.cuda.current_stream().cuda_stream)
        res, P = distributed.sharded_assemble(eng, distributed.TorchComm(), d_buf, d_off, hi - lo, lo, a.k, a.limit)
    torch.cuda.synchronize()
    t_asm = time.time() - t1
    if rank == 0:
        if a.output:
            ingest.write_contigs_fasta(a.output, res, "contig%d", blank_line=False)
        if a.gfa:
            ingest.write_gfa(a.gfa, res, a.k)
        print("reads %d  k-mer positions %d  contigs %d  ingest %.2f s  assemble %.3f s  (%d GPU%s)"
              % (nreads, P, len(res.contig_offsets) - 1, t_ingest, t_asm, world, "s" if world > 1 else ""),
              file=sys.stderr)
        if not a.output and not a.gfa:
            sys.stdout.write("".join(">contig%d\n%s\n" % (i, c) for i, c in enumerate(res.contigs)))
    if sharded:
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
