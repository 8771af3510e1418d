"""Per-launch listing of a bench breakdown dump (DMX_BENCH_BREAKDOWN): layer, kernel, us, TF/s of
reference work — optionally filtered by a kernel-name substring.  python tools/bd_convs.py FILE [SUBSTR]"""
import json
import sys

d = json.load(open(sys.argv[1]))
sub = sys.argv[2] if len(sys.argv) > 2 else ""
tot = 0.0
for r in d["records"]:
    if sub and sub not in r["kernel"]:
        continue
    us = r["ms"] * 1e3
    tot += us
    tf = r["flops"] / (r["ms"] * 1e-3) / 1e12 if r.get("flops") else 0.0
    print(f"{r['layer']:28s} {r['kernel']:52s} {us:8.1f} us  {tf:6.1f} TF")
print(f"total {tot:.1f} us")
