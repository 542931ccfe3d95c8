"""Estimate per-rank step times of the read-sharded path at N ranks on ONE GPU: runs every
rank's engine calls back to back (collectives by concatenation) and reports each phase's
device time for rank 0 (counting its 1/N shard, exporting, merging its owned records,
loading the gathered solid set + graph phase).  Communication time is not included."""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "pycuda-euler_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--reads", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--err", type=float, default=0.0, help="substitution rate (bench ecoli10m_err: 0.005)")
    ap.add_argument("--genome", type=int, default=4_600_000, help="genome length (genome20m_k51 shape: 20000000)")
    ap.add_argument("--len", type=int, default=100, help="read length (config 5 shape: 150)")
    ap.add_argument("--k", type=int, default=31, help="node length (config 5: 51, 128-bit keys)")
    ap.add_argument("--seed", type=int, default=20261019)
    ap.add_argument("--finish", default="partitioned", choices=["partitioned", "replicated"],
                    help="partitioned: every rank ranks / emits its own segment (distributed.partitioned_finish)")
    ap.add_argument("--read-base", type=int, default=0,
                    help="global id of the first read (one rank of a larger job: config 5's rank 3 of 8 = 37500000)")
    ap.add_argument("--weak", action="store_true",
                    help="bench.py's default N > 1 mode: every rank its own --reads reads (synth part = rank)")
    a = ap.parse_args()
    import torch

    import distributed
    from synth import make_reads

    world = a.ranks
    engines = [distributed.HipEngine(0) for _ in range(world)]
    shards = []
    if a.weak:
        for r in range(world):
            buf, off = make_reads(a.genome, a.reads, a.len, a.seed, err=a.err, part=r)
            shards.append((torch.from_numpy(buf).cuda(), torch.from_numpy(off.astype(np.int64)).cuda(), a.reads,
                           r * a.reads))
    else:
        buf, off = make_reads(a.genome, a.reads, a.len, a.seed, err=a.err)
        for r in range(world):
            lo, hi = distributed.shard_range(a.reads, r, world)
            shards.append((torch.from_numpy(np.ascontiguousarray(buf[int(off[lo]):int(off[hi])])).cuda(),
                           torch.from_numpy((off[lo:hi + 1] - off[lo]).astype(np.int64)).cuda(), hi - lo,
                           a.read_base + lo))
        del buf, off
    torch.cuda.synchronize()
    import eulerhip
    eulerhip.mem_stats(reset=True)
    torch.cuda.reset_peak_memory_stats()
    for rep in range(a.reps):
        t = {}

        def t_start():  # the host-side copies between calls are not charged to the next call
            torch.cuda.synchronize()
            return time.perf_counter()

        def tick(name, t0):
            torch.cuda.synchronize()
            t[name] = t.get(name, []) + [(time.perf_counter() - t0) * 1e3]

        sends = []
        for eng, (d_reads, d_off, n, lo) in zip(engines, shards):
            eng.trim_if_large()  # (as sharded_assemble: a large previous step's buffers released first)
            t0 = t_start()
            eng.count_shard(d_reads, d_off, n, lo, a.k, 0)
            tick("count", t0)
            t0 = t_start()
            sends.append(eng.export_by_owner(world, compact=True))
            eng.trim_if_large()
            tick("export", t0)
        rb = distributed.rec_bytes(a.k)
        rbs = [distributed.compact_bytes(a.k) if b >= 0 else rb for _, _, b in sends]
        recvs = []
        for dst, eng in enumerate(engines):
            parts = []
            for src in range(world):
                recs, counts, _ = sends[src]
                o = sum(counts[:dst]) * rbs[src]
                parts.append(recs[o:o + counts[dst] * rbs[src]])
            recvs.append((parts[0] if world == 1 else torch.cat(parts), [x.numel() for x in parts]))
        bases = [sh[3] for sh in shards]
        lfbs = [b for _, _, b in sends]
        import ctypes
        import eulerhip
        extra = ""
        if a.finish == "replicated":  # the round-4 layout: gathered solid set, loaded on every rank
            solids = []
            for eng, (recv, sb) in zip(engines, recvs):
                t0 = t_start()
                solids.append(eng.merge_owned_from(recv, sb, bases, lfbs, a.k, 1, 0))
                tick("merge", t0)
            mx = max(x.numel() for x in solids)
            allsolid = torch.full((world * mx,), 0xFF, dtype=torch.uint8, device="cuda")
            for i, x in enumerate(solids):
                allsolid[i * mx: i * mx + x.numel()] = x
            nrec = [x.numel() // rb for x in solids]
            parts = []
            for r, eng in enumerate(engines):
                lo = sum(nrec[:r])
                t0 = t_start()
                eng.graph_load(allsolid, a.k)
                tick("load", t0)
                t0 = t_start()
                part = eng.empty(8 * nrec[r])
                eng.graph_links_part(lo, lo + nrec[r], part)
                tick("links", t0)
                parts.append(part[: 8 * nrec[r]])
            succ = torch.cat(parts)
            eng = engines[0]
            t0 = t_start()
            eulerhip.check(eng.L.ec_graph_finish(eng._h(), ctypes.c_void_p(succ.data_ptr()), eulerhip.EC_FLAG_TIMING))
            tick("finish", t0)
            t0 = t_start()
            res = eng.sess.fetch(a.k)
            tick("fetch", t0)
            st = eng.stats()
            print("finish stages ms:", {n: round(v, 3) for n, v in zip(eulerhip.stage_names(), st.stage_ms)})
            xb = allsolid.numel()
        else:  # the junction-partitioned graph and the partitioned finish, every rank's calls timed
            urs = []
            for eng, (recv, sb) in zip(engines, recvs):
                t0 = t_start()
                urs.append(eng.merge_owned_from(recv, sb, bases, lfbs, a.k, 1, 0, export=False))
                tick("merge", t0)
            seg_lo = [sum(urs[:r]) for r in range(world + 1)]
            U = seg_lo[-1]
            placed = []
            for r, eng in enumerate(engines):
                t0 = t_start()
                placed.append(eng.graph_place(seg_lo[r], U, world))
                tick("place", t0)
            npal = sum(p[2] for p in placed)
            jb = distributed.junction_bytes(a.k)
            links = []
            jx = 0
            for dst, eng in enumerate(engines):
                got = [rec[sum(c[:dst]) * jb:sum(c[:dst + 1]) * jb] for rec, c, _ in placed]
                jx = max(jx, sum(g.numel() for i, g in enumerate(got) if i != dst))
                recv = got[0] if len(got) == 1 else torch.cat(got)
                t0 = t_start()
                links.append(eng.graph_join(recv, seg_lo))
                tick("join", t0)
            lx = 0
            for dst, eng in enumerate(engines):
                got = [rec[sum(c[:dst]) * 8:sum(c[:dst + 1]) * 8] for rec, c in links]
                lx = max(lx, sum(g.numel() for g in got))
                t0 = t_start()
                eng.graph_links_apply(torch.cat(got))
                tick("apply", t0)
            segs = [(seg_lo[r], seg_lo[r + 1]) for r in range(world)]
            sups = []
            for eng, (lo, hi) in zip(engines, segs):
                t0 = t_start()
                sups.append(eng.graph_chains_part(lo, hi)[0])
                tick("chains", t0)
            supers = torch.cat(sups)
            M = supers.numel() // distributed.SUPER_BYTES
            for eng in engines:
                t0 = t_start()
                eng.graph_rank_supers(supers, M)
                tick("rank_supers", t0)
            sts = []
            for eng, (lo, hi) in zip(engines, segs):
                t0 = t_start()
                sts.append(eng.graph_starts_part(M > 0, lo, hi)[0])
                tick("starts", t0)
            starts = torch.cat(sts)
            nc = starts.numel() // distributed.START_BYTES
            runs = []
            for eng in engines:  # (as partitioned_finish: each rank's own runs gathered to rank 0)
                t0 = t_start()
                eng.graph_layout(starts, nc)
                tick("layout", t0)
                t0 = t_start()
                runs.append(eng.graph_emit_runs())
                tick("emit", t0)
            allruns = torch.cat(runs)
            t0 = t_start()
            engines[0].graph_collect_runs(allruns, [r.numel() for r in runs], a.k, npal, fetch=False)
            tick("collect", t0)  # (results left in the session's pinned buffers, as the bench step)
            res = engines[0].sess.fetch(a.k)
            extra = (", junction records off-rank %.2f MB, link records %.2f MB, chains gathered %.1f MB (%d), "
                     "starts %.2f MB, runs gathered %.1f MB" % (jx / 1e6, lx / 1e6, supers.numel() / 1e6, M,
                                                                starts.numel() / 1e6, allruns.numel() / 1e6))
            xb = 0
        print("export per rank:", [round(x, 2) for x in t["export"]], "count per rank:", [round(x, 2) for x in t["count"]])
        mx_ph = {k: round(max(v), 2) for k, v in t.items()}
        med = {k: round(float(np.median(v)), 2) for k, v in t.items()}
        print("rep %d  per-rank median ms: %s  sum %.2f" % (rep, med, sum(med.values())))
        print("rep %d  ranks %d  per-rank max ms: %s  sum %.2f  exchanged bytes/rank ~%.0f MB, gathered %.0f MB%s" % (
            rep, world, mx_ph, sum(mx_ph.values()),
            sum(c for c in sends[0][1]) * rbs[0] / 1e6, xb / 1e6, extra))
        held, peak = eulerhip.mem_stats()
        print("rep %d  HBM: session buffers of all %d simulated ranks held %.1f GB, peak %.1f GB; torch tensors "
              "(reads, exchange buffers) peak %.1f GB; device total %.1f GB" % (
                  rep, world, held / 1e9, peak / 1e9, torch.cuda.max_memory_allocated() / 1e9,
                  torch.cuda.mem_get_info()[1] / 1e9), flush=True)
    print("contigs", len(res.contig_offsets) - 1, "chars", len(res.contig_bytes))


if __name__ == "__main__":
    main()
