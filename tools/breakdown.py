import json, sys
d = json.load(open(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/breakdown.json'))
agg = d['by_kernel']
tot = sum(v['ms'] for v in agg.values())
print(f"total {tot:.3f} ms")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1]['ms'])[:int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    tf = v['flops'] / (v['ms'] * 1e-3) / 1e12 if v['flops'] else 0
    gbs = v['bytes'] / (v['ms'] * 1e-3) / 1e9
    print(f"{k:40s} n={v['n']:3d} ms={v['ms']:7.3f} ({100 * v['ms'] / tot:4.1f}%) TF={tf:6.1f} GB/s={gbs:7.0f}")
by_layer = {}
for r in d['records']:
    by_layer[r['layer']] = by_layer.get(r['layer'], 0) + r['ms']
print(" | ".join(f"{k}:{v*1e3:.0f}us" for k, v in sorted(by_layer.items(), key=lambda kv: -kv[1])))
