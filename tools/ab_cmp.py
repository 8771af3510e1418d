"""Compare per-launch times of two breakdown JSONs (bench.py DMX_BENCH_BREAKDOWN) for kernels
matching a pattern:  python tools/ab_cmp.py A.json B.json [regex]"""
import json
import re
import sys

a = json.load(open(sys.argv[1]))["records"]
b = json.load(open(sys.argv[2]))["records"]
pat = sys.argv[3] if len(sys.argv) > 3 else "."
ta = tb = 0.0
for x, y in zip(a, b):
    if re.search(pat, x["kernel"]) or re.search(pat, y["kernel"]):
        print(f"{x['layer']:8s} {x['kernel'][:44]:44s} {x['ms'] * 1e3:7.1f} | {y['kernel'][:44]:44s} {y['ms'] * 1e3:7.1f}")
        ta += x["ms"]
        tb += y["ms"]
print(f"matched: {ta * 1e3:.1f} vs {tb * 1e3:.1f} us; step {sum(r['ms'] for r in a) * 1e3:.1f} vs "
      f"{sum(r['ms'] for r in b) * 1e3:.1f} us")
