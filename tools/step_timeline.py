"""Per-step timeline of a rocprofv3 kernel trace (rocpd database): for the last bench step,
every dispatch with its start offset, duration and the idle gap before it; then per-step wall
(first start .. last end) against summed kernel time.

    python tools/step_timeline.py RUN_RESULTS.db [FIRST_KERNEL_SUBSTRING]"""
import re
import sqlite3
import sys


def main():
    db = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else "k_skpart_w"
    c = sqlite3.connect(db)
    ks = list(c.execute("select name, start, end from kernels order by start"))
    idx = [i for i, (n, _, _) in enumerate(ks) if first in n]
    steps = []
    for a, b in zip(idx, idx[1:] + [len(ks)]):
        steps.append(ks[a:b])
    for s in steps:
        wall = (s[-1][2] - s[0][1]) / 1e3
        busy = sum(e - st for _, st, e in s) / 1e3
        print("step: %d dispatches, wall %.1f us, busy %.1f us, idle %.1f us" % (len(s), wall, busy, wall - busy))
    s = steps[-2] if len(steps) > 1 else steps[-1]
    t0 = s[0][1]
    prev = t0
    for n, st, e in s:
        short = re.sub(r"\(.*", "", n)[:60]
        print("%9.1f %8.1f gap %7.1f  %s" % ((st - t0) / 1e3, (e - st) / 1e3, (st - prev) / 1e3, short))
        prev = e


main()
