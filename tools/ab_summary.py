"""ab_summary.py DIR -- steps/s of tools/ab.sh's alternating new / old bench lines, per workload."""
import glob
import json
import re
import sys

d = sys.argv[1]
rows = {}
for f in sorted(glob.glob(f"{d}/*_*_[0-9].json")):
    m = re.match(r".*/(new|old)_(.+)_(\d)\.json$", f)
    if not m:
        continue
    try:
        v = json.loads(open(f).read().strip().splitlines()[-1])["value"]
    except Exception:
        continue
    rows.setdefault(m.group(2), {}).setdefault(m.group(1), []).append(v)
for w, r in rows.items():
    new, old = r.get("new", []), r.get("old", [])
    gain = (sum(new) / len(new)) / (sum(old) / len(old)) - 1 if new and old else float("nan")
    print(f"{w}: new {' '.join(f'{x:.1f}' for x in new)} | old {' '.join(f'{x:.1f}' for x in old)} | {gain * 100:+.2f} %")
