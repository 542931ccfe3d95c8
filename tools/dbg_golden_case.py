"""Run one golden case through the GPU path and print where it differs from the golden result
(debug helper: python tools/dbg_golden_case.py NAME [wide_records])"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pycuda-euler_amd"))
os.environ.setdefault("EULERHIP_DEBUG", "1")
import eulerhip  # noqa: E402

name = sys.argv[1]
wr = len(sys.argv) > 2
case = None
for f in ("synthetic.json", "fuzz.json"):
    for c in json.load(open(os.path.join(ROOT, "tests", "golden", f))).get("cases", []):
        if c["name"] == name:
            case = c
s = eulerhip.Session(0)
for rep in range(3):
    res = s.assemble(case["reads"], case["k"], case["limit"], want_dict=True, wide_records=wr)
    d = [[x, c] for x, c in res.dict_items]
    ok_d, ok_c, ok_l = d == case["d"], res.contigs == case["contigs"], res.links == case["links"]
    print("rep", rep, "dict", ok_d, "contigs", ok_c, "links", ok_l, "stats", res.stats.count_path,
          res.stats.record_bytes, res.stats.n_records, res.stats.n_positions, res.stats.n_solid, flush=True)
    if not ok_d:
        i = next((j for j, (a, b) in enumerate(zip(d, case["d"])) if a != b), min(len(d), len(case["d"])))
        print("  dict len", len(d), len(case["d"]), "first diff", i, d[i:i + 2], case["d"][i:i + 2])
