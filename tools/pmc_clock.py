"""Effective shader clock per kernel family under load, from a rocprofv3 GRBM_GUI_ACTIVE pass
(MI355X_MICROARCH.md 'DVFS give-back': clock ~= GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time; reads high
on dispatches shorter than ~0.3 ms, and profiled passes run a few % below un-profiled ones).  For each
family: mean duration, mean clock, and the fraction of the split2h / bf16 peak AT THAT CLOCK that the
family's flops reach -- how much of the gap to the nominal peak is the clock rather than the issue
schedule.

usage: python tools/pmc_clock.py <counter_collection.csv> [out.txt]
With out.txt, also out.json ({precision: {family: {clock_ghz, frac_nominal, frac_at_clock, ...}}}, the
split2h families 0 = hidden forward, 1 = hidden data grad), which bench.py quotes in its roofline block.
"""
import json
import csv
import sys
from collections import defaultdict

PEAK_GHZ = 2.4
FAMILIES = [
    # (label, kernel-name prefix, flops per launch and ensemble member at S3 (MT50/W2048, B = 6400), peak TF,
    #  bench family id)
    ("hidden forward (split2h)", "gemm_x3f_kernel<208, 1, ", 2 * 6400 * 2048 * 2048, 2500.0 / 3, 0),
    ("hidden data grad (split2h)", "gemm_x3f_kernel<208, 2, ", 2 * 6400 * 2048 * 2048, 2500.0 / 3, 1),
]
TILES_PER_MEMBER = 31 * 8  # 208 x 256 tiles of a 6400 x 2048 output
WG_THREADS = 512


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    acc = defaultdict(lambda: [0, 0.0, 0.0, 0])  # launches, ns, GRBM_GUI_ACTIVE, ensemble members
    for r in rows:
        if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
            continue
        k = r["Kernel_Name"]
        a = acc[k + "|" + r["Grid_Size"]]
        a[3] = max(1, round(int(r["Grid_Size"]) / WG_THREADS / TILES_PER_MEMBER))
        a[0] += 1
        a[1] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        a[2] += float(r["Counter_Value"])
    out = []
    js = {}
    for label, pre, flops, peak, fam in FAMILIES:
        n = ns = cyc = fl = 0.0
        names = []
        for k, (c, t, g, e) in acc.items():
            if pre in k:
                # the hidden layers only: input-layer launches carry TAG (6th parameter) 8
                params = k[k.index(pre) + len("gemm_x3f_kernel<"):].split(">")[0].split(", ")
                if len(params) > 5 and params[5] != "0":
                    continue
                n += c
                ns += t
                cyc += g
                fl += c * e * flops
                names.append(k.split("(")[0] + f" (E = {e})")
        if not n:
            continue
        us = ns / n / 1e3
        ghz = cyc / 8 / ns
        tf = fl / (ns * 1e-9) / 1e12
        js[str(fam)] = {"label": label, "launches": int(n), "avg_launch_us": us, "clock_ghz": ghz, "tflops": tf,
                        "frac_nominal": tf / peak, "frac_at_clock": tf / (peak * ghz / PEAK_GHZ),
                        "source": "rocprofv3 --pmc GRBM_GUI_ACTIVE (eager pass): clock = GRBM_GUI_ACTIVE / 8 / duration"}
        out.append(f"{label}: {int(n)} launches, {us:.1f} us, clock {ghz:.3f} GHz, {tf:.0f} TF = "
                   f"{tf / peak:.3f} of the nominal peak, {tf / (peak * ghz / PEAK_GHZ):.3f} of the peak at that clock")
        out.extend("    " + s for s in sorted(set(names)))
    # every kernel above 50 us mean, for context
    out.append("kernels with mean duration > 50 us (profiled pass):")
    for k, (c, t, g, e) in sorted(acc.items(), key=lambda kv: -kv[1][1]):
        if t / c > 50e3:
            out.append(f"  {t / c / 1e3:8.1f} us  {g / 8 / t:.3f} GHz  x{c:<5d} grid {k.split('|')[1]:>7s} "
                       f"{k.split('(')[0][:140]}")
    text = "\n".join(out)
    print(text)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text + "\n")
        with open(sys.argv[2].rsplit(".", 1)[0] + ".json", "w") as f:
            json.dump({"split2h": js}, f, indent=1)


if __name__ == "__main__":
    main()
