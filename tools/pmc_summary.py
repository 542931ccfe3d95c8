"""Per-kernel mean of each PMC counter in a rocprofv3 counter_collection.csv."""
import collections
import csv
import sys

KEYS = ('k_sk', 'k_partition', 'k_refine2', 'k_bucket', 'k_prescan', 'k_link', 'k_walk', 'k_rjump', 'k_final', 'k_starts', 'k_emit')
for path in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        agg[r['Kernel_Name'][:48]][r['Counter_Name']].append(float(r['Counter_Value']))
    for k, d in agg.items():
        if any(x in k for x in KEYS):
            print(k, {c: '%.3g' % (sum(v) / len(v)) for c, v in d.items()})
