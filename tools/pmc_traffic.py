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
    # split2h: the same kernel templates with NP = 2 (the prefixes above match both)
    "split2h": {
        0: ("gemm_x3f_kernel<208, 1, false, true, false, 0,", "gemm_x3f_kernel<208, 1, true, false, false, 0,",
            "gemm_x3f_kernel<208, 1, true, true, false, 0,"),
        1: ("gemm_x3f_kernel<208, 2,",),
        2: ("gemm_x3p_kernel<mtsac::x3pk::Geo<256, 256, 2, 4, 3, 16, 0>, true, true, 0,",),
        3: ("gemm_x3f_kernel<208, 1, false, true, false, 8,",),
        4: ("gemm_x3_kernel<true, false, 0>",),
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
    """{dispatch id: (kernel name, value)} for one counter."""
    out = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter:
                continue
            did = r.get("Dispatch_Id") or r.get("Correlation_Id")
            name = r.get("Kernel_Name", "")
            v = float(r.get("Counter_Value", 0.0))
            if did in out:
                out[did] = (name, out[did][1] + v)  # one row per XCD / instance: sum
            else:
                out[did] = (name, v)
    return out


def family_means(rows, keys, scale):
    res = {}
    for fam, key in keys.items():
        vals = [v for (name, v) in rows.values() if any(k in name for k in key)]
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
            fam_out[str(fam)] = {"kernel": " | ".join(keys[fam]), "hbm_bytes_per_launch": fetch[fam][0] + write[fam][0],
                                 "fetch_bytes_per_launch": fetch[fam][0], "write_bytes_per_launch": write[fam][0],
                                 "dispatches": fetch[fam][1],
                                 "correction": "FETCH_SIZE (KiB) x 2 (gfx950 half-count) + WRITE_SIZE (KiB)"}
    d[prec] = fam_out
    with open(out_json, "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps(fam_out, indent=1))


if __name__ == "__main__":
    main()
