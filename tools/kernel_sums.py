"""Per-kernel total time per step from a rocprofv3 kernel trace (steps delimited by the replay
index kernel).  usage: kernel_sums.py <kernel_trace.csv> [top N]"""
import collections
import csv
import sys

rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
              for r in csv.DictReader(open(sys.argv[1])))
starts = [s for s, e, n in rows if "replay_indices" in n]
a, b = starts[2], starts[-1]  # skip warm-up steps
nsteps = len(starts) - 3
tot = collections.Counter()
cnt = collections.Counter()
for s, e, n in rows:
    if a <= s < b:
        k = n.replace("mtsac::", "").replace("(anonymous namespace)::", "").replace("x3pk::", "").split("(")[0][:90]
        tot[k] += e - s
        cnt[k] += 1
print(f"{nsteps} steps, wall {(b - a) / nsteps / 1e3:.1f} us/step, kernel sum {sum(tot.values()) / nsteps / 1e3:.1f} us/step")
for k, v in tot.most_common(int(sys.argv[2]) if len(sys.argv) > 2 else 30):
    print(f"{v / nsteps / 1e3:9.1f} us/step {cnt[k] / nsteps:5.1f}x  {k}")
