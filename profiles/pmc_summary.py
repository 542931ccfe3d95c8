"""Per-kernel averages of every counter in rocprofv3 --pmc CSV outputs under the given dirs.

    python profiles/pmc_summary.py DIR [DIR ...]
"""
import csv
import glob
import os
import re
import sys


def short(name):
    m = re.search(r"ec::(k_\w+)", name)
    return m.group(1) if m else None


def main():
    vals = {}
    for d in sys.argv[1:]:
        for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(fn) as f:
                for row in csv.DictReader(f):
                    k = short(row["Kernel_Name"])
                    if not k:
                        continue
                    c = vals.setdefault(k, {}).setdefault(row["Counter_Name"], {})
                    c[(fn, row["Dispatch_Id"])] = c.get((fn, row["Dispatch_Id"]), 0.0) + float(row["Counter_Value"])
    for k in sorted(vals):
        print(k)
        for cn in sorted(vals[k]):
            v = vals[k][cn]
            print("  %-24s %14.4g  (%d launches)" % (cn, sum(v.values()) / len(v), len(v)))


if __name__ == "__main__":
    main()
