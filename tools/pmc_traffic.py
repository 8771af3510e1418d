"""Per-kernel HBM traffic per launch from rocprofv3 --pmc passes (MI355X_MICROARCH.md §HBM):
bytes = 2 * FETCH_SIZE * 1024 (gfx950 reports half of a wide coalesced read) + WRITE_SIZE * 1024.
Usage: python tools/pmc_traffic.py gpurun_out/prof_fetch gpurun_out/prof_write profiles/pmc_traffic.json"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.match(r"^_ZN3dmx\d+(\w+?)ILi(\d+)EE", name)  # rocprofv3 leaves some templates mangled (_Float16 args)
    if m:
        return f"{m.group(1)}<{m.group(2)}>"
    name = re.sub(r"^void\s+", "", name)
    name = re.sub(r"^dmx::", "", name)
    return re.sub(r"\(.*\)$", "", name).strip()


def load(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] == counter:
                vals[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return vals


def lib_sha256():
    """Build identity of the profiled library (bench.py refuses PMC bytes of another build)."""
    import hashlib
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "diffusion-model_amd"))
    from dmx import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def main(fetch_dir, write_dir, out):
    fe, wr = load(fetch_dir, "FETCH_SIZE"), load(write_dir, "WRITE_SIZE")
    res = {}
    for k in fe:
        if k in wr and fe[k] and wr[k]:
            f = sum(fe[k]) / len(fe[k])
            w = sum(wr[k]) / len(wr[k])
            res[k] = {"fetch_kb_raw": f, "write_kb": w, "bytes": 2 * f * 1024 + w * 1024, "launches": len(fe[k])}
    doc = {"method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of `python3 bench.py "
                     "--steps 3 --warmup 1 --cpu-steps 0 --config4-steps 0 --config5-steps 0 --no-profile` (tools/prof.sh); bytes/launch = 2*FETCH_SIZE*1024 + "
                     "WRITE_SIZE*1024 (gfx950 FETCH_SIZE = half of wide coalesced reads); averages over all "
                     "launches of the kernel name",
           "lib_sha256": lib_sha256(),
           "traffic_bytes_per_launch": {k: round(v["bytes"]) for k, v in res.items()},
           "detail": res}
    json.dump(doc, open(out, "w"), indent=1)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["bytes"] * kv[1]["launches"])[:12]:
        print(f"{k:45s} {v['bytes'] / 1e6:9.2f} MB/launch  n={v['launches']}")


if __name__ == "__main__":
    main(*sys.argv[1:4])
