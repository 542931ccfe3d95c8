"""Turn rocprofv3 PMC passes (FETCH_SIZE pass, WRITE_SIZE pass; gfx950 cannot count both in one
pass) into per-kernel HBM bytes per launch: profiles/traffic_<tag>.json, read by bench.py.

FETCH_SIZE / WRITE_SIZE are in KiB.  Per MI355X_MICROARCH.md (HBM section) FETCH_SIZE reports
half the bytes of wide coalesced streaming reads on gfx950, so it is doubled; WRITE_SIZE is
taken as is.  The result is therefore an estimate of the kernel's HBM traffic.

    python profiles/collect_traffic.py FETCH_DIR WRITE_DIR WORKLOAD TAG
"""
import csv
import glob
import json
import os
import re
import sys

KERNELS = ("k_bucket_wr", "k_run_codes", "k_downsweep_wr", "k_wbv", "k_jl_scan", "k_jl_edges", "k_jl_scatter",
           "k_jl_join", "k_upsweep", "k_downsweep", "k_bucket", "k_count", "k_refine", "k_prescan", "k_partition", "k_refine2",
           "k_skpart", "k_skrefine", "k_skbucket", "k_neighbors", "k_walk", "k_half_join64", "k_half_join", "k_half_emit64", "k_half_emit", "k_pred_rc",
           "k_tile_chains", "k_tile_compact", "k_walk_s", "k_rjump", "k_expand", "k_super_link", "k_finalize_s",
           "k_starts_count", "k_emit", "k_gfa")


def short(name):
    for k in KERNELS:
        if re.search(r"\b%s(_sk|_w|3)?\b" % k, name):
            return k
    return None


def rows(d, counter):
    """(kernel name, dispatch id, value) of `counter`: rocprofv3 CSV output or its rocpd SQLite
    database (run_results.db, the default output format of newer rocprofv3)."""
    import sqlite3

    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row["Counter_Name"] == counter:
                    yield row["Kernel_Name"], row["Dispatch_Id"], float(row["Counter_Value"])
    for fn in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        con = sqlite3.connect(fn)
        for name, disp, val in con.execute(
                "select kernel_name, dispatch_id, value from counters_collection where counter_name = ?", (counter,)):
            yield name, str(disp), float(val)
        con.close()


def per_kernel(d, counter):
    vals = {}
    for name, disp, val in rows(d, counter):
        k = short(name)
        if k:
            vals.setdefault(k, {}).setdefault(disp, 0.0)
            vals[k][disp] += val
    return {k: sum(v.values()) / len(v) * 1024.0 for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    fdir, wdir, workload, tag = sys.argv[1:5]
    fetch, nf = per_kernel(fdir, "FETCH_SIZE")
    write, nw = per_kernel(wdir, "WRITE_SIZE")
    out = {"workload": workload, "tag": tag, "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, bench.py",
           "correction": "FETCH_SIZE x2 (gfx950 wide-read note), WRITE_SIZE x1, KiB -> bytes", "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f2 = 2.0 * fetch.get(k, 0.0)
        w = write.get(k, 0.0)
        out["kernels"][k] = {"fetch_bytes_per_launch": round(f2), "write_bytes_per_launch": round(w),
                             "kernel_bytes_per_launch": round(f2 + w), "launches": [nf.get(k, 0), nw.get(k, 0)]}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "traffic_%s.json" % tag)
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
