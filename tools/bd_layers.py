"""Per-layer (stage) totals of several breakdown dumps side by side:
python tools/bd_layers.py A.json B.json ... [--kernel SUBSTR]"""
import collections
import json
import sys

files = [a for a in sys.argv[1:] if not a.startswith("--")]
sub = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else ""
if sub:
    files = [f for f in files if f != sub]
tabs = []
for f in files:
    t = collections.OrderedDict()
    for r in json.load(open(f))["records"]:
        if sub and sub not in r["kernel"]:
            continue
        s = t.setdefault(r["layer"].split(".")[0], [0.0, 0])
        s[0] += r["ms"] * 1e3
        s[1] += 1
    tabs.append(t)
keys = list(tabs[0])
for k in keys:
    print(f"{k:14s}" + "".join(f"{t.get(k, [0, 0])[0]:9.1f} ({t.get(k, [0, 0])[1]:2d})" for t in tabs))
print(f"{'total':14s}" + "".join(f"{sum(v[0] for v in t.values()):9.1f} ({sum(v[1] for v in t.values()):2d})" for t in tabs))
