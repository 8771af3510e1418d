"""Per-kernel SQ counter summary from rocprofv3 --pmc passes (gpurun_out/pmc_sq*/).

Derived (MI355X_MICROARCH.md §rocprofv3 PMC slots, §Per-instruction constants):
  kernel cycles  = GRBM_GUI_ACTIVE / 8            (summed over the 8 XCDs)
  mfma_busy      = SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / kernel cycles   (counts cycles)
  wait_any / wait_inst / active = fractions of SQ_WAVE_CYCLES (quad-cycles, disjoint buckets)
  lds_busy       = SQ_LDS_IDX_ACTIVE / 256 CUs / kernel cycles
Usage: python tools/pmc_sq.py [regex]"""
import csv
import glob
import re
import sys
from collections import defaultdict


def short(name):
    m = re.match(r"^_ZN3dmx\d+(\w+?)ILi(\d+)EE", name)
    if m:
        return f"{m.group(1)}<{m.group(2)}>"
    name = re.sub(r"^void\s+", "", name)
    name = re.sub(r"^dmx::", "", name)
    return re.sub(r"\(.*\)$", "", name).strip()


acc = defaultdict(lambda: defaultdict(list))
for d in sorted(glob.glob("gpurun_out/pmc_sq*")):
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            acc[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
pat = sys.argv[1] if len(sys.argv) > 1 else "igemm|attention|norm"
print(f"{'kernel':58s} {'n':>4s} {'cyc(k)':>8s} {'mfma%':>6s} {'lds%':>5s} {'w_any':>6s} {'w_inst':>6s} "
      f"{'active':>6s} {'valu':>5s} {'ldsconf':>8s} {'L2hit':>6s}")
for k, c in sorted(acc.items()):
    if not re.search(pat, k):
        continue
    avg = {n: sum(v) / len(v) for n, v in c.items()}
    kc = avg.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    wc = avg.get("SQ_WAVE_CYCLES", 0.0) or 1.0
    mf = avg.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / 1024.0 / kc if kc else float("nan")
    lds = avg.get("SQ_LDS_IDX_ACTIVE", 0.0) / 256.0 / kc if kc else float("nan")
    n = len(next(iter(c.values())))
    print(f"{k[:58]:58s} {n:4d} {kc / 1e3:8.1f} {100 * mf:6.1f} {100 * lds:5.1f} "
          f"{avg.get('SQ_WAIT_ANY', 0) / wc:6.2f} {avg.get('SQ_WAIT_INST_ANY', 0) / wc:6.2f} "
          f"{avg.get('SQ_ACTIVE_INST_ANY', 0) / wc:6.2f} {avg.get('SQ_ACTIVE_INST_VALU', 0) / wc:5.2f} "
          f"{avg.get('SQ_LDS_BANK_CONFLICT', 0):8.3g} "
          f"{avg.get('TCC_HIT_sum', 0) / max(1.0, avg.get('TCC_HIT_sum', 0) + avg.get('TCC_MISS_sum', 0)):6.3f}")
