"""Compare two bench breakdown dumps (DMX_BENCH_BREAKDOWN) per kernel name and per layer."""
import json
import sys
from collections import defaultdict


def agg(path, key):
    d = defaultdict(float)
    for r in json.load(open(path))["records"]:
        d[key(r)] += r["ms"] * 1e3
    return d


def main():
    a, b = sys.argv[1], sys.argv[2]
    for title, key in (("kernel", lambda r: r["kernel"]), ("layer", lambda r: r["layer"])):
        A, B = agg(a, key), agg(b, key)
        print(f"== by {title} (us)   {a}  ->  {b}")
        for k in sorted(set(A) | set(B), key=lambda k: -max(A.get(k, 0), B.get(k, 0))):
            x, y = A.get(k, 0.0), B.get(k, 0.0)
            if max(x, y) < 15:
                continue
            print(f"  {k:44s} {x:8.1f} {y:8.1f}  {y - x:+8.1f}")
        print(f"  {'TOTAL':44s} {sum(A.values()):8.1f} {sum(B.values()):8.1f}")


if __name__ == "__main__":
    main()
