"""Per-kernel time per step from a rocprofv3 --kernel-trace database (rocpd, the default output).
usage: rocpd_sums.py <run_results.db> <step-marker kernel substring> [top N]
Steps are counted by the marker kernel's dispatches; the first two steps are skipped as warm-up."""
import collections
import sqlite3
import sys

db, marker = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
rows = sorted(sqlite3.connect(db).execute("select start, end, name from kernels"))
starts = [s for s, e, n in rows if marker in n]
a, b = starts[2], starts[-1]
nsteps = len(starts) - 3
tot, cnt = collections.Counter(), collections.Counter()
for s, e, n in rows:
    if a <= s < b:
        k = n.replace("mtsac::", "").replace("drq::", "").replace("(anonymous namespace)::", "").split("(")[0][:88]
        tot[k] += e - s
        cnt[k] += 1
print(f"{nsteps} steps, wall {(b - a) / nsteps / 1e3:.1f} us/step, kernel sum {sum(tot.values()) / nsteps / 1e3:.1f} us/step")
for k, v in tot.most_common(top):
    print(f"{v / nsteps / 1e3:9.1f} us/step {cnt[k] / nsteps:5.1f}x  {k}")
