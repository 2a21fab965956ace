"""HBM traffic per GEMM launch from rocprofv3 PMC passes (separate FETCH_SIZE and WRITE_SIZE
runs of bench.py, MI355X_MICROARCH.md 'HBM': FETCH_SIZE reports half the bytes of wide
coalesced reads on gfx950 -> doubled; WRITE_SIZE taken as is).  Both counters are in KiB.

usage: python tools/pmc_traffic.py <precision> <fetch_counter_collection.csv> <write_counter_collection.csv> <out.json>
Merges the per-family result into out.json ({precision: {family: {...}}}).
"""
import csv
import json
import os
import sys

FAMILY_KEYS = {
    "split3": {
        # gemm_x3f_kernel<BM, EPI, C_OUT, P_OUT, MASK16, TAG, NP>: TAG 8 = input-layer launches
        0: ("gemm_x3f_kernel<208, 1, false, true, false, 0,", "gemm_x3f_kernel<208, 1, true, false, false, 0,",
            "gemm_x3f_kernel<208, 1, true, true, false, 0,"),
        1: ("gemm_x3f_kernel<208, 2,",),
        2: ("gemm_x3p_kernel<mtsac::x3pk::Geo<256, 256, 2, 4, 3, 16, 0>, true, true, 0,",),
        3: ("gemm_x3f_kernel<208, 1, false, true, false, 8,",),
        4: ("gemm_x3_kernel<true, false, 0>",),
    },
    # split2h: the same forward / data-grad templates with NP = 2; since round 5 every S3 weight grad
    # (hidden and input layer) runs on the 256 x 128 k16 tiles: one symbol, and split-K gives the input
    # layers' launches the hidden layers' grids, so family 2 here is every weight grad (5 hidden-sized
    # 256-workgroup launches and one 128-workgroup launch per step) and family 4 has no launches
    "split2h": {
        0: ("gemm_x3f_kernel<208, 1, false, true, false, 0,", "gemm_x3f_kernel<208, 1, true, false, false, 0,",
            "gemm_x3f_kernel<208, 1, true, true, false, 0,"),
        1: ("gemm_x3f_kernel<208, 2,",),
        2: ("gemm_x3p_kernel<mtsac::x3pk::Geo<256, 128, 4, 2, 4, 16, 0>, true, true, 0,",),
        3: ("gemm_x3f_kernel<208, 1, false, true, false, 8,",),
    },
    "fp32": {
        0: ("gemm_f32_kernel<false, true, 1>",),
        1: ("gemm_f32_kernel<false, true, 2>",),
        2: ("gemm_f32_kernel<true, false, 0>",),
        3: ("gemm_f32_kernel<false, false, 1>",),
        4: ("gemm_f32_kernel<true, false, 0>",),
    },
}


def per_dispatch(path, counter):
    """{dispatch id: (kernel name, value, grid size in work-items)} for one counter."""
    out = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter:
                continue
            did = r.get("Dispatch_Id") or r.get("Correlation_Id")
            name = r.get("Kernel_Name", "")
            v = float(r.get("Counter_Value", 0.0))
            grid = int(r.get("Grid_Size", 0) or 0)
            if did in out:
                out[did] = (name, out[did][1] + v, grid)  # one row per XCD / instance: sum
            else:
                out[did] = (name, v, grid)
    return out


def _match(name, grid, k):
    """k: a kernel-name prefix, or (prefix, min grid, max grid or None)."""
    if isinstance(k, str):
        return k in name
    pre, lo, hi = k
    return pre in name and grid >= lo and (hi is None or grid <= hi)


def _label(k):
    return k if isinstance(k, str) else f"{k[0]} (grid {k[1]}..{k[2] if k[2] is not None else ''})"


def family_means(rows, keys, scale):
    res = {}
    for fam, key in keys.items():
        vals = [v for (name, v, grid) in rows.values() if any(_match(name, grid, k) for k in key)]
        if vals:
            res[fam] = (sum(vals) / len(vals) * scale, len(vals))
    return res


def main():
    prec, fetch_csv, write_csv, out_json = sys.argv[1:5]
    keys = FAMILY_KEYS[prec]
    fetch = family_means(per_dispatch(fetch_csv, "FETCH_SIZE"), keys, 2.0 * 1024.0)
    write = family_means(per_dispatch(write_csv, "WRITE_SIZE"), keys, 1024.0)
    d = {}
    if os.path.exists(out_json):
        with open(out_json) as f:
            d = json.load(f)
    fam_out = {}
    for fam in keys:
        if fam in fetch and fam in write:
            fam_out[str(fam)] = {"kernel": " | ".join(_label(k) for k in keys[fam]), "hbm_bytes_per_launch": fetch[fam][0] + write[fam][0],
                                 "fetch_bytes_per_launch": fetch[fam][0], "write_bytes_per_launch": write[fam][0],
                                 "dispatches": fetch[fam][1],
                                 "correction": "FETCH_SIZE (KiB) x 2 (gfx950 half-count) + WRITE_SIZE (KiB)"}
    d[prec] = fam_out
    with open(out_json, "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps(fam_out, indent=1))


if __name__ == "__main__":
    main()
