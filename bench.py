"""bench.py -- headline benchmark of the MI355X de Bruijn + Euler-tour core.

Metric (BASELINE.json): k-mers/sec (encode+hash+deBruijn+Euler), 10Mx100bp k=31, 1/2/4/8 GPU.
One step = one full fused assembly (encode -> canonical count -> solid filter -> links ->
list ranking -> contig starts/order -> contig strings -> GFA links, i.e. the reference's
build() + all_contigs()) of the whole synthetic read set, reads already resident in HBM.
value = k-mer positions of the whole job / wall time of one step (max over ranks).
N > 1 is weak-scaled by default: every rank holds its own config-sized read set (10 M x 100 bp
on the headline) of the same genome, so the job is N x 10 M reads; --strong splits the
config's reads over the ranks instead.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (read-sharded, RCCL exchange)
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "pycuda-euler_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

METRIC = "k-mers/sec (encode+hash+deBruijn+Euler), 10Mx100bp k=31, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)

# SURVEY §8d synthetic inputs: seed = 20261015 + config#
CONFIGS = {
    # the metric's own workload (BASELINE configs[3] data: E. coli size, 10M x 100 bp, k = 31)
    "ecoli10m": dict(genome=4_600_000, reads=10_000_000, read_len=100, k=31, seed=20261015 + 4,
                     name="ecoli-4.6Mbp-10Mx100bp-k31"),
    # BASELINE configs[1]: 1M x 100 bp
    "ecoli1m": dict(genome=4_600_000, reads=1_000_000, read_len=100, k=31, seed=20261015 + 2,
                    name="ecoli-4.6Mbp-1Mx100bp-k31"),
    # BASELINE configs[2]: S. cerevisiae size, 5M x 100 bp
    "yeast5m": dict(genome=12_000_000, reads=5_000_000, read_len=100, k=31, seed=20261015 + 3,
                    name="yeast-12Mbp-5Mx100bp-k31"),
    # BASELINE configs[4]: synthetic 200 Mbp genome, 100M x 150 bp, k = 51 (128-bit keys)
    "genome200m_k51": dict(genome=200_000_000, reads=100_000_000, read_len=150, k=51, seed=20261015 + 5,
                           name="synthetic-200Mbp-100Mx150bp-k51"),
    # config 5's per-rank shape at 8 ranks: 1/8 of its reads (12.5 M x 150 bp) of the 200 Mbp genome
    "genome200m_k51_r8": dict(genome=200_000_000, reads=12_500_000, read_len=150, k=51, seed=20261015 + 5,
                              name="synthetic-200Mbp-12.5Mx150bp-k51"),
    # the same read length / k at a tenth of the size (20 Mbp genome, same 75x coverage)
    "genome20m_k51": dict(genome=20_000_000, reads=10_000_000, read_len=150, k=51, seed=20261015 + 5,
                          name="synthetic-20Mbp-10Mx150bp-k51"),
    # the metric's workload with 0.5 % substitution errors (SURVEY §8d optional variant: most
    # erroneous k-mers occur once and fail the count > 1 solid filter)
    "ecoli10m_err": dict(genome=4_600_000, reads=10_000_000, read_len=100, k=31, seed=20261015 + 4, err=0.005,
                         name="ecoli-4.6Mbp-10Mx100bp-k31-err0.5pct"),
    # a genome past one LDS table per bucket (5·10^7 solid 31-mers: buckets split into part tables)
    "genome50m": dict(genome=50_000_000, reads=10_000_000, read_len=100, k=31, seed=20261015 + 6,
                      name="synthetic-50Mbp-10Mx100bp-k31"),
    "tiny": dict(genome=50_000, reads=50_000, read_len=100, k=31, seed=7, name="tiny-50kbp-50kx100bp-k31"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def alg_bytes(P, R, L, U, K=8):
    """SURVEY §8d official algorithmic bytes: R*L + P*(K+8) + U*(10K+33)."""
    return R * L + P * (K + 8) + U * (10 * K + 33)


def kernel_alg_bytes(name, P, R, L, K=8, rec=16, NR=None, nsub=0, rec2=None):
    """HBM bytes per launch of the counting kernels, from the algorithm's data movement
    (DESIGN.md "Roofline accounting"; kernel names by slot, see kernel_names()).
    Window records (rec = 16, 12 or 10 bytes written by the partition pass, rec2 = bytes of the
    refine's output records, NR = P records, nsub = bucket sub-table bytes written):
    k_upsweep / k_prescan     reads the ASCII reads once                      R*L
    k_downsweep / k_partition reads them again + writes one record/position   R*L + rec*P
    k_refine / k_refine2      reads every record, writes it to its bucket     (rec + rec2)*P
    k_bucket                  reads every record, writes the sub-tables       rec2*P + nsub
    k_count     general path: read once + one insert per position R*L + P*(K+8)
    Super-k-mer records (rec = 32 or 16 bytes, NR records):
    k_downsweep / k_skpart R*L + rec*NR;  k_refine / k_skrefine 2*rec*NR
    k_bucket / k_skbucket rec*NR + nsub: the records read, the sub-tables written (SURVEY 8d's
                           per-position insert, P*(K+8), overstates it: the kernel inserts each
                           distinct super-k-mer's windows once, ~P/10 inserts, in LDS)"""
    if NR is not None and NR < P and rec in (16, 32):
        return {"k_upsweep": R * L, "k_downsweep": R * L + rec * NR,
                "k_bucket": rec * NR + nsub,
                "k_count": R * L + P * (K + 8), "k_refine": 2 * rec * NR}[name]
    rec2 = rec2 or rec
    return {"k_upsweep": R * L, "k_downsweep": R * L + rec * P, "k_bucket": rec2 * P + nsub,
            "k_count": R * L + P * (K + 8), "k_refine": (rec + rec2) * P}[name]


def kernel_names(variant):
    """kernel names of the ec_stats.kernel_ms slots: count_part.h's exact path (variant 0),
    count_v2.h's fixed-capacity runs (variants 1, 2) or count_sk2.h's super-k-mers (variant 3)"""
    if variant == 3:
        return ("k_prescan", "k_skpart", "k_skbucket", "k_count", "k_skrefine")
    if variant:
        return ("k_prescan", "k_partition", "k_bucket", "k_count", "k_refine2")
    return ("k_upsweep", "k_downsweep", "k_bucket", "k_count", "k_refine")


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def host_threads():
    """host cores this process may use: the box's CPU share (OMP_NUM_THREADS is set to it on
    the GPU boxes; os.cpu_count() there counts the whole machine), else the affinity mask"""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, n)


def cpu_baseline(buf, off, k, sample_reads):
    """The test-only C restatement (oracle/refasm.c) of the reference CPU assembler on the first
    `sample_reads` reads of the same workload, timed twice: 1 core (the
    reference's build + all_contigs are single-threaded) and N cores (oracle_assemble_mt:
    map -> reduceByKey counting as src/ref_spark.py:76-84 on N threads, all_contigs
    single-threaded).  value = the N-core rate."""
    import oracle

    n = min(sample_reads, len(off) - 1)
    sb = buf[: int(off[n])]
    so = off[: n + 1]
    t0 = time.perf_counter()
    out = oracle.assemble_packed(sb, so, k, 1)
    dt1 = time.perf_counter() - t0
    nth = host_threads()
    t0 = time.perf_counter()
    outn = oracle.assemble_packed(sb, so, k, 1, threads=nth)
    dtn = time.perf_counter() - t0
    assert outn["contig_chars"] == out["contig_chars"], "N-core oracle differs from the 1-core oracle"
    P = int(out["n_positions"])
    return {"value": P / dtn, "unit": "k-mers/s", "cores": nth, "kind": "port",
            "sample": "first %d of %d reads (%d k-mer positions): oracle/refasm.c map->reduceByKey count on %d "
                      "threads + single-threaded all_contigs %.1f s; single-threaded build+all_contigs %.1f s"
                      % (n, len(off) - 1, P, nth, dtn, dt1),
            "one_core": {"value": P / dt1, "unit": "k-mers/s", "cores": 1, "seconds": round(dt1, 2)},
            "cpu": cpu_model(), "node_cpus": os.cpu_count()}


def write_fasta(path, buf, off):
    """the synthetic reads as a FASTA file, one '>r' record a read (uniform length: numpy rows)"""
    R = len(off) - 1
    L = int(off[1] - off[0]) if R else 0
    assert int(off[-1]) == R * L, "uniform read length expected"
    rows = np.empty((R, L + 4), np.uint8)
    rows[:, :3] = np.frombuffer(b">r\n", np.uint8)
    rows[:, 3:3 + L] = buf[:R * L].reshape(R, L)
    rows[:, -1] = ord("\n")
    rows.tofile(path)
    return rows.size


def host_input_legs(sess, buf, off, k, P, steps, warmup):
    """The drop-in entry from host memory (the reference hands host reads to its GPU path,
    src/eulercuda.py:484-497; SURVEY 8d: "timer starts after reads are in pinned host memory; H2D
    is included"): one step = ec_assemble_packed_reads on the 2-bit codes the native FASTA reader
    wrote into page-locked memory (ec_reads_load with EC_READS_PACKED, timed as load_ms), and
    ec_assemble_host on the ASCII reads in page-locked memory.  Chunked copies on a second stream
    overlap the partition.  fasta_to_contigs: file (page cache) -> pinned codes -> contigs and
    links back in host memory, end to end.  h2d_gbs: one plain pinned -> HBM copy of the codes'
    size, the PCIe floor of the packed step."""
    import shutil
    import tempfile

    import torch
    import eulerhip
    import ingest

    def timed(fn, n=steps, w=warmup):
        for _ in range(w):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            fn()  # (each call ends with the results in the session's pinned host buffers)
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / n * 1e3

    tmp = tempfile.mkdtemp(prefix="ec_bench_")
    try:
        fa = os.path.join(tmp, "reads.fa")
        fbytes = write_fasta(fa, buf, off)
        loads = []
        for _ in range(3):  # the file is in the page cache after writing it
            t0 = time.perf_counter()
            rs = ingest.ReadSet(fa, ingest.FASTA_RECORDS, threads=host_threads(), packed=True)
            loads.append((time.perf_counter() - t0) * 1e3)
            if len(loads) < 3:
                rs.close()
        load_ms = float(np.median(loads))
        nb = rs.n_bases
        ms_packed = timed(lambda: rs.assemble(sess, k, 1, eulerhip.EC_FLAG_KERNEL_TIMING))
        # pipelined: batch i + 1 staged (its PCIe copy queued) before batch i is assembled --
        # the same read set each step, as every step of the bench; the copy left in flight by
        # the last stage is inside the timed region (synchronize)
        rs.stage(sess)
        rs.stage(sess)

        def piped():
            sess.assemble_staged(k, 1, eulerhip.EC_FLAG_KERNEL_TIMING)
            rs.stage(sess)

        ms_piped = timed(piped)
        sess.assemble_staged(k, 1, 0)
        sess.assemble_staged(k, 1, 0)  # (the pipeline drained)
        # FASTA file -> contigs + links in host memory (three times; median)
        e2e = []
        for _ in range(3):
            t0 = time.perf_counter()
            with ingest.ReadSet(fa, ingest.FASTA_RECORDS, threads=host_threads(), packed=True) as r2:
                t1 = time.perf_counter()
                r2.assemble(sess, k, 1, 0)
            t2 = time.perf_counter()
            res = sess.fetch(k)
            t3 = time.perf_counter()
            e2e.append(((t3 - t0) * 1e3, (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3))
        e2e.sort()
        tot, l_ms, a_ms, f_ms = e2e[1]
        ncodes = (nb + 3) // 4
        # PCIe floor: the codes' bytes pinned -> HBM in one copy
        hsrc = torch.empty(ncodes, dtype=torch.uint8, pin_memory=True)
        ddst = torch.empty(ncodes, dtype=torch.uint8, device="cuda")
        h2d_ms = timed(lambda: ddst.copy_(hsrc, non_blocking=True), n=5, w=2)
        del hsrc, ddst
        rs.close()
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    abuf = torch.empty(buf.size, dtype=torch.uint8, pin_memory=True).numpy()
    abuf[:] = buf
    aoff = torch.empty(len(off), dtype=torch.int64, pin_memory=True).numpy().view(np.uint64)
    aoff[:] = off
    ms_ascii = timed(lambda: sess.run_host(abuf, aoff, k, 1, eulerhip.EC_FLAG_KERNEL_TIMING))
    return {"value": round(P / (ms_packed / 1e3), 1), "unit": "k-mers/s", "ms_per_step": round(ms_packed, 3),
            "input": "2-bit codes in page-locked host memory written by the FASTA reader (%d bytes, one read "
                     "length: no offsets)" % ncodes,
            "load_ms": round(load_ms, 1),
            "pipelined": {"value": round(P / (ms_piped / 1e3), 1), "ms_per_step": round(ms_piped, 3),
                          "note": "ec_stage_packed_host / ec_assemble_staged: batch i + 1's H2D copy overlaps "
                                  "batch i's kernels (two device slots)"},
            "h2d_gbs": round(ncodes / (h2d_ms / 1e3) / 1e9, 2), "h2d_ms": round(h2d_ms, 3),
            "fasta_to_contigs": {"ms": round(tot, 1), "load_ms": round(l_ms, 1), "assemble_ms": round(a_ms, 1),
                                 "fetch_ms": round(f_ms, 1), "fasta_bytes": int(fbytes),
                                 "contigs": len(res.contig_offsets) - 1, "threads": host_threads(),
                                 "note": "FASTA in the page cache -> contigs + links in host memory (median of 3)"},
            "ascii": {"value": round(P / (ms_ascii / 1e3), 1), "ms_per_step": round(ms_ascii, 3),
                      "input": "ASCII reads + uint64 offsets in page-locked host memory (%d bytes)"
                               % (buf.size + 8 * len(off))}}


def load_traffic(workload, kernel):
    """HBM bytes per launch of `kernel` from rocprofv3 PMC passes (profiles/traffic_*.json,
    written by profiles/collect_traffic.py; FETCH_SIZE doubled per the gfx950 note)."""
    import glob

    best = None
    for fn in sorted(glob.glob(os.path.join(ROOT, "profiles", "traffic_*.json"))):
        try:
            d = json.load(open(fn))
        except (OSError, ValueError):
            continue
        kd = d.get("kernels", {}).get(kernel)
        if d.get("workload") == workload and kd and kd.get("kernel_bytes_per_launch"):
            best = dict(kd, file=os.path.basename(fn))
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="ecoli10m", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-sample-reads", type=int, default=1_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-input", action="store_true",
                    help="skip the host-input legs (reads in pinned host memory, PCIe copy inside the step)")
    ap.add_argument("--sharded", action="store_true", help="use the multi-GPU path even with one rank")
    ap.add_argument("--strong", action="store_true",
                    help="N > 1: split the config's reads over the ranks (fixed job) instead of the default "
                         "weak scaling (every rank samples its own config-sized read set of the same genome)")
    ap.add_argument("--strong-leg", action="store_true",
                    help="run the strong-scaled leg at any N (with --sharded at N = 1: rehearses its code path)")
    ap.add_argument("--no-strong-leg", action="store_true",
                    help="N > 1 weak-scaled runs: skip the strong-scaled leg (the config's read set split over "
                         "the ranks, reported under \"strong\")")
    ap.add_argument("--wide-records", action="store_true", help="16-B count records only (EC_FLAG_WIDE_RECORDS)")
    ap.add_argument("--window-records", action="store_true",
                    help="one record per k-mer window, no super-k-mers (EC_FLAG_WINDOW_RECORDS)")
    args = ap.parse_args()
    # stdout carries exactly one JSON line: libraries that print banners (RCCL prints its
    # version block on communicator init) are sent to stderr
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("note: --gpus %d but WORLD_SIZE=%d; using WORLD_SIZE" % (args.gpus, world))
    torch.cuda.set_device(local)
    dist = None
    use_dist = world > 1 or args.sharded
    if use_dist:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29541")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import eulerhip

    cfg = CONFIGS[args.config]
    t0 = time.time()
    from synth import make_reads

    # weak scaling (default): rank r holds reads r*R .. (r+1)*R - 1 of an N*R-read job on the
    # config's genome, sampled by rank (synth.make_reads part=r); --strong: the config's R reads
    # are split into contiguous shards (distributed.shard_range)
    weak = use_dist and not args.strong
    buf, off = make_reads(cfg["genome"], cfg["reads"], cfg["read_len"], cfg["seed"], err=cfg.get("err", 0.0),
                          part=(rank if weak else None))
    log("rank %d: generated %d reads in %.1f s" % (rank, cfg["reads"], time.time() - t0))
    k = cfg["k"]

    hbm_free0 = torch.cuda.mem_get_info()[0]  # device memory before the inputs and the session
    if not use_dist:
        d_buf = torch.from_numpy(buf).cuda()
        d_off = torch.from_numpy(off.astype(np.int64)).cuda()
        torch.cuda.synchronize()
        sess = eulerhip.Session(local, stream=torch.cuda.current_stream().cuda_stream)

        def step(timing=0):
            sess.run_device(d_buf.data_ptr(), d_off.data_ptr(), cfg["reads"], k, 1, timing
                            | (eulerhip.EC_FLAG_WIDE_RECORDS if args.wide_records else 0)
                            | (eulerhip.EC_FLAG_WINDOW_RECORDS if args.window_records else 0))
    else:
        import distributed

        runner = distributed.ShardedAssembler(buf, off, k, 1, rank, world, local,
                                              read_base=(rank * cfg["reads"] if weak else None))

        def step(timing=0):  # results left in the session's pinned buffers, as run_device leaves them
            runner.run(timing, fetch=False)

    # timed steps record the kernel events only (EC_FLAG_KERNEL_TIMING: the roofline's kernel
    # durations, live over the timed region); the stage breakdown (EC_FLAG_TIMING, ~26 events
    # a call, ~0.1 ms) comes from one untimed step after it
    for _ in range(args.warmup):
        step(eulerhip.EC_FLAG_TIMING)
    if use_dist:
        runner.phase_ms = {}  # per-phase times of the timed steps only
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    kern = np.zeros(eulerhip.EC_NKERNELS)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step(eulerhip.EC_FLAG_KERNEL_TIMING)
        st = sess.stats() if not use_dist else runner.stats()
        kern += np.array(list(st.kernel_ms))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if dist:
        t = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = elapsed / args.steps * 1e3
    # HBM held after the steps: inputs + the session's buffers (sized by their largest use and
    # kept between calls, so this is the run's peak allocation)
    hbm_used = hbm_free0 - torch.cuda.mem_get_info()[0]
    timed_phase_ms = dict(runner.phase_ms) if use_dist else None
    step(eulerhip.EC_FLAG_TIMING)  # untimed (every rank: it has collectives): the per-stage breakdown
    stage = np.array(list((sess.stats() if not use_dist else runner.stats()).stage_ms))
    st = sess.stats() if not use_dist else runner.stats()
    P = int(st.n_positions) if not use_dist else runner.total_positions
    U = int(st.n_solid) if not use_dist else int(runner.engine.stats().n_solid)
    R, L = cfg["reads"] * (world if weak else 1), cfg["read_len"]
    value = P / (ms / 1e3)

    # strong-scaled leg (N > 1, weak mode): the config's own read set (rank 0's) split into
    # contiguous shards over the ranks (BASELINE config 4: "10M x 100 bp reads, read-sharded"),
    # timed the same way; reported beside the weak-scaled value
    strong = None
    if weak and (world > 1 or args.strong_leg) and not args.no_strong_leg:
        import distributed

        lo, hi = distributed.shard_range(cfg["reads"], rank, world)
        sbuf, soff = make_reads(cfg["genome"], cfg["reads"], cfg["read_len"], cfg["seed"], err=cfg.get("err", 0.0),
                                rows=(lo, hi))
        srun = distributed.ShardedAssembler(sbuf, soff, k, 1, rank, world, local, comm=runner.comm, read_base=lo)
        for _ in range(max(1, args.warmup)):
            srun.run(eulerhip.EC_FLAG_KERNEL_TIMING, fetch=False)
        torch.cuda.synchronize()
        dist.barrier()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            srun.run(eulerhip.EC_FLAG_KERNEL_TIMING, fetch=False)
        torch.cuda.synchronize()
        dist.barrier()
        t = torch.tensor([time.perf_counter() - t1], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        sms = float(t.item()) / args.steps * 1e3
        strong = {"value": round(srun.total_positions / (sms / 1e3), 1), "unit": "k-mers/s",
                  "ms_per_step": round(sms, 3), "reads": cfg["reads"], "reads_per_gpu": hi - lo,
                  "positions": int(srun.total_positions), "scaling": "strong"}

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    kern /= args.steps
    sharded_ms = None
    if use_dist:
        sharded_ms = {kk: round(v / args.steps, 3) for kk, v in timed_phase_ms.items()}
    kid = int(np.argmax(kern))
    kname = eulerhip.KERNEL_NAMES[kid]  # slot name (kernel_alg_bytes); reported by its variant name
    variant = int(getattr(st, "count_variant", 0))
    names_v = kernel_names(variant)
    kms = float(kern[kid])
    K = 8 if k <= 32 else 16  # key bytes
    rec = int(st.record_bytes) or 16
    rec2 = 12 if variant == 2 else rec  # the 10-B partition records are refined to 12 B
    nsub = int(st.table_capacity) * 16  # bucket sub-tables written by k_bucket
    kb = kernel_alg_bytes(kname, int(st.n_positions), int(st.n_reads), L, K, rec, int(st.n_records), nsub, rec2)
    achieved = kb / (kms / 1e3) / 1e9
    tr = load_traffic(cfg["name"], names_v[kid])
    roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": (tr["kernel_bytes_per_launch"] if tr else None),
            "traffic_source": (tr["file"] if tr else None),
            "kernel": names_v[kid], "kernel_ms": round(kms, 4), "alg_bytes_per_launch": int(kb),
            "alg_basis": "bytes the kernel must move through HBM",
            "kernels_ms": {names_v[i]: round(float(kern[i]), 4) for i in range(len(kern)) if kern[i] > 0},
            # every counting kernel against the same roofline (k_downsweep and k_refine run within
            # a few % of each other on the headline, so the dominant one can change between runs)
            "kernels_frac": {names_v[i]: round(
                kernel_alg_bytes(eulerhip.KERNEL_NAMES[i], int(st.n_positions), int(st.n_reads), L, K, rec,
                                 int(st.n_records), nsub, rec2) / (float(kern[i]) / 1e3) / (HBM_PEAK_GBS * 1e9), 5)
                for i in range(len(kern)) if kern[i] > 0},
            # measured HBM bytes (PMC traffic) per launch / launch time / peak: the HBM roofline on
            # what the kernels really move (k_skbucket's §8d basis counts LDS insert work)
            "frac_hbm": (round(tr["kernel_bytes_per_launch"] / (kms / 1e3) / (HBM_PEAK_GBS * 1e9), 5) if tr else None),
            "kernels_frac_hbm": {names_v[i]: round(t["kernel_bytes_per_launch"] / (float(kern[i]) / 1e3)
                                                   / (HBM_PEAK_GBS * 1e9), 5)
                                 for i in range(len(kern)) if kern[i] > 0
                                 for t in [load_traffic(cfg["name"], names_v[i])] if t},
            "pipeline_alg_bytes": int(alg_bytes(P, R, L, U, K)),
            "pipeline_frac": round(alg_bytes(P, R, L, U, K) / (ms / 1e3) / (HBM_PEAK_GBS * 1e9), 5)}
    host = None
    if not use_dist and not args.no_host_input:
        host = host_input_legs(sess, buf, off, k, P, args.steps, max(2, args.warmup))
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(buf, off, k, args.cpu_sample_reads)
    names = eulerhip.stage_names()
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "k-mers/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
        "scaling": "none" if world == 1 and not use_dist else ("strong" if args.strong else "weak"),
        "vs_baseline": None, "dtype": "u64" if k <= 32 else "u128",
        "data": "synthetic (iid ACGT genome, uniform %s %d bp reads, 50%% reverse-complemented, numpy PCG64 seed %d)"
                % ("error-free" if not cfg.get("err") else "%.1f%%-substitution" % (100 * cfg["err"]), L, cfg["seed"]),
        "config": {"workload": cfg["name"] + ("" if world == 1 or not weak else " per GPU"), "genome_bp": cfg["genome"],
                   "reads": R, "reads_per_gpu": R // world, "read_len": L, "k": k,
                   "positions": P, "solid_kmers": U,
                   "contigs": int(st.n_contigs if not use_dist else runner.engine.stats().n_contigs),
                   "count_path": ["partitioned", "general", "superkmer"][int(st.count_path)],
                   "count_variant": ["histogram runs", "fixed-capacity runs", "fixed-capacity runs, 10-B records",
                                     "super-k-mer records, 16 B"][variant],
                   "buckets": int(st.n_buckets), "record_bytes": int(st.record_bytes), "records": int(st.n_records),
                   "parallelism": ("dp%d" % world) + ("-sharded" if use_dist else ""),
                   "hbm_used_gb": round(hbm_used / 1e9, 2)},
        # SURVEY 8d's host-input rate (reads in pinned host memory, PCIe copy inside the step)
        "host_input_value": host["value"] if host else None,
        "host_input_ms_per_step": host["ms_per_step"] if host else None,
        "roofline": roof,
        "cpu_baseline": cpu,
        "host_input": host,
        "stage_ms": {names[i]: round(stage[i], 3) for i in range(len(names))},
        "sharded_phase_ms": sharded_ms,
        "strong": strong,
    }
    print(json.dumps(out), file=json_out, flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
