import csv, glob, re, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for d in sorted(glob.glob('gpurun_out/pmc_sq*')):
    for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
        for row in csv.DictReader(open(f)):
            k = re.sub(r'\(.*\)$', '', re.sub(r'^void\s+dmx::', '', row['Kernel_Name']))
            acc[k][row['Counter_Name']].append(float(row['Counter_Value']))
pat = sys.argv[1] if len(sys.argv) > 1 else 'igemm_x3|attention|norm'
for k, c in sorted(acc.items()):
    if not re.search(pat, k):
        continue
    avg = {n: sum(v) / len(v) for n, v in c.items()}
    wc = avg.get('SQ_WAVE_CYCLES', 0) or 1
    print(f"== {k}  (n={len(next(iter(c.values())))})")
    print("   " + "  ".join(f"{n.replace('SQ_','')}={v:.3g}" for n, v in sorted(avg.items())))
    if 'SQ_WAIT_ANY' in avg:
        print(f"   wait_any {avg['SQ_WAIT_ANY']/wc:.2f}  wait_inst {avg['SQ_WAIT_INST_ANY']/wc:.2f}  active {avg['SQ_ACTIVE_INST_ANY']/wc:.2f}"
              f"  valu {avg['SQ_ACTIVE_INST_VALU']/wc:.2f}  lds {avg['SQ_ACTIVE_INST_LDS']/wc:.2f}")
