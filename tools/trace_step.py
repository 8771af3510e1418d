"""One graph-replayed CFG step from a rocprofv3 --kernel-trace CSV: every dispatch's duration and the
gap before it, plus per-family sums (device timestamps, so this is the replay's real timeline).

  python tools/trace_step.py <dir with *kernel_trace.csv> [out.json]

Steps are delimited by step_tail4_kernel; the step whose span is the median of the timed steps is
printed."""
import csv
import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    with open(f) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if r[2].startswith("dmx::step_tail") or "step_tail" in r[2]]
    steps = []
    for a, b in zip(ends, ends[1:]):
        seg = rows[a + 1:b + 1]
        if 40 <= len(seg) <= 300:
            steps.append(seg)
    if not steps:
        print("no step found;", len(rows), "dispatches,", len(ends), "step tails; names:",
              sorted({r[2][:80] for r in rows})[:40])
        return
    spans = sorted((s[-1][1] - s[0][0], i) for i, s in enumerate(steps))
    span, idx = spans[len(spans) // 2]
    seg = steps[idx]
    prev_end = rows[ends[idx]][1] if idx < len(ends) else seg[0][0]
    out, fam = [], {}
    busy = 0
    for s, e, name in seg:
        short = name.replace("void ", "").replace("dmx::", "").split("(")[0]
        gap = (s - prev_end) / 1e3
        dur = (e - s) / 1e3
        busy += dur
        prev_end = e
        out.append({"kernel": short, "us": round(dur, 2), "gap_us": round(gap, 2)})
        k = short.split("<")[0]
        fam[k] = fam.get(k, 0.0) + dur
        print(f"{short[:60]:60s} {dur:8.2f} us  gap {gap:6.2f}")
    print(f"steps found {len(steps)}; median step span {span / 1e3:.1f} us, kernel busy {busy:.1f} us, "
          f"{len(seg)} dispatches")
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
        print(f"  {k:30s} {v:8.1f} us {100 * v / busy:5.1f} %")
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as fh:
            json.dump({"span_us": span / 1e3, "busy_us": busy, "dispatches": out, "by_family_us": fam}, fh, indent=1)


if __name__ == "__main__":
    main()
