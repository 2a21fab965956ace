"""Per-step kernel timeline from a rocprofv3 kernel trace (eager bench run): busy union, GEMM vs
other kernel time, and the last full step's launches.  usage: step_timeline.py <kernel_trace.csv> [full]"""
import csv
import sys

rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"])
              for r in csv.DictReader(open(sys.argv[1])))
starts = [s for s, e, n, _ in rows if "replay_indices" in n]
print("steps", len(starts))
for k in range(max(0, len(starts) - 4), len(starts) - 1):
    a, b = starts[k], starts[k + 1]
    ks = [(s, e, n) for s, e, n, _ in rows if a <= s < b]
    iv = sorted((s, e) for s, e, n in ks)
    tot, (cs, ce) = 0, iv[0]
    for s, e in iv[1:]:
        if s > ce:
            tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    tot += ce - cs
    g = sum(e - s for s, e, n in ks if "gemm" in n)
    o = sum(e - s for s, e, n in ks if "gemm" not in n)
    print(f"step {k}: wall {(b - a) / 1e3:.0f} us, busy-union {tot / 1e3:.0f} us, gemm sum {g / 1e3:.0f}, other sum {o / 1e3:.0f}, n={len(ks)}")
if len(sys.argv) > 2:
    a, b = starts[-3], starts[-2]
    for s, e, n, st in rows:
        if a <= s < b:
            n = n.replace("mtsac::", "").replace("(anonymous namespace)::", "").replace("x3pk::", "")
            print(f"{(s - a) / 1e3:8.1f} {(e - a) / 1e3:8.1f} {(e - s) / 1e3:7.1f} st{st} {n[:100]}")
