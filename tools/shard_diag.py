"""Diagnose the 8-way S3 shard step against the float64 oracle, leaf by leaf.

Runs the MT50 8-way task split (8 engines on one device, in-process all-reduce hook, exactly as
tests/test_gpu_fullbatch.py::test_full_batch_8way_shard_matches_oracle) REPEATS times from the same
inputs and prints:
  * the log errors against the oracle, and whether the repeats are bitwise equal;
  * per actor / critic leaf, the first Adam moment (mu = (1 - b1) g after one step) against the
    oracle's: max |d| / max |ref| and the relative L2 error -- which leaf carries an error.
Optionally the unsharded engine for contrast.

usage: python tools/shard_diag.py [--precision 3] [--repeats 3] [--single] [--name s3_mt50_w2048]
With MTSAC_GUARD_BYTES=n in the environment every engine allocation carries n-byte NaN guard zones,
checked after each sharded step (mtsac_debug_check_guards).
"""

from __future__ import annotations

import argparse
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import test_gpu_fullbatch as t  # noqa: E402
from mtrl_amd import _lib as L  # noqa: E402
from mtrl_amd.init import leaf_shapes, slice_heads  # noqa: E402
from mtrl_amd.shard import InProcessAllReduce, local_rows, shard_tasks  # noqa: E402


def leaf_errs(got, ref, shapes, tag):
    o = 0
    out = []
    for k, s in shapes:
        m = int(np.prod(s))
        g, r = got[o:o + m].astype(np.float64), ref[o:o + m]
        o += m
        d = np.abs(g - r)
        rmax = np.abs(r).max()
        l2 = np.linalg.norm(g - r) / max(np.linalg.norm(r), 1e-300)
        out.append((k, d.max() / max(rmax, 1e-300), l2, np.linalg.norm(r)))
    print(tag, " ".join(f"{k}:max{a:.1e}/l2{b:.1e}(|r|{c:.2e})" for k, a, b, c in out))
    return out


SNAP = False
CU_SLICE = False  # --cu-slice: engine r runs on CU slice r of 8 (MTSAC_CU_SLICE)
FULL_MASK = False  # --full-mask: every engine's streams CU-masked to ALL CUs (MTSAC_CU_SLICE=0:1): engines
#                   co-resident on every CU as unsliced, but each stream on a queue of its own
HEADG = {}  # (arm, rank) -> the actor gradient's head leaves of the arm's first repeat (--grad-diff)
GRAD_DIFF = False
ARM = ""
SNAP0 = {}  # rank -> the first repeat's h after the forward


def snap_count(e, i):
    """float count of debug buffer i (the engine names it in the error of a wrong count)"""
    rc = e.lib.mtsac_debug_read(e._h, i, 1, -1)
    msg = e.lib.mtsac_last_error().decode()
    assert rc != 0 and "count must be" in msg, msg
    return int(msg.rsplit(" ", 1)[1])


def run_sharded(name, precision, world=8):
    spec = t.SHARD_CASES[name]
    cfg, st, batch, en, ec, st1, want = t._problem(name)
    T, n = spec["T"], spec["n"]
    shards = []
    for r in range(world):
        b0, c0 = shard_tasks(T, world, r)
        if CU_SLICE:
            os.environ["MTSAC_CU_SLICE"] = f"{r}:{world}"
        elif FULL_MASK:
            os.environ["MTSAC_CU_SLICE"] = "0:1"
        e = t._engine(spec, precision, b0, c0)
        t._load(e, st, b0, c0)
        shards.append(e)
    os.environ.pop("MTSAC_CU_SLICE", None)
    if SNAP:
        for e in shards:
            L.check(e.lib.mtsac_debug_snapshot(e._h, 1))
    group = InProcessAllReduce(world)
    for r, e in enumerate(shards):
        e.set_allreduce_hook(group.hook(r))
    errs = []

    def run(r):
        try:
            b0, c0 = shard_tasks(T, world, r)
            rows = local_rows(T, n, b0, c0)
            shards[r].update(tuple(x[rows] for x in batch), en[rows], ec[rows])
        except Exception as ex:  # pragma: no cover
            errs.append(ex)

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    [x.start() for x in th]
    [x.join() for x in th]
    assert not errs, errs
    for r, e in enumerate(shards):
        if os.environ.get("MTSAC_GUARD_BYTES"):
            nb = e.lib.mtsac_debug_check_guards(e._h)
            print(f"  guards rank {r}: {nb} written", e.lib.mtsac_last_error().decode() if nb else "", flush=True)
    snaps = []
    if SNAP:
        W = spec["W"]
        for r, e in enumerate(shards):
            b0, c0 = shard_tasks(T, world, r)
            B = n * c0
            bufs = {}
            for i, cnt in ((0, None), (1, None), (2, None), (3, B * 8), (4, None)):
                if cnt is None:
                    cnt = snap_count(e, i)
                a = np.empty(cnt, np.float32)
                L.check(e.lib.mtsac_debug_read(e._h, i, a.ctypes.data, cnt))
                bufs[i] = a
            h = bufs[0].reshape(-1, W)[:B].astype(np.float64)
            d = bufs[3].reshape(B, 8).astype(np.float64)
            gW = np.zeros((c0, W, 8))
            for t_ in range(c0):
                rr = np.arange(n) * c0 + t_
                gW[t_] = h[rr].T @ d[rr]
            off = -(-8 * c0 // 64) * 64  # leaves are 64-float aligned
            eng = bufs[4][off:off + c0 * W * 8].reshape(c0, W, 8).astype(np.float64)
            rel = np.abs(eng - gW).max() / np.abs(gW).max()
            if rel > 1e-5 and os.environ.get("DIAG_DUMP"):  # the failing rank's operands, for offline analysis
                os.makedirs(os.environ["DIAG_DUMP"], exist_ok=True)
                np.savez_compressed(os.path.join(os.environ["DIAG_DUMP"], f"fail_r{r}_{len(SNAP0)}_{np.random.randint(1 << 30)}.npz"),
                                    h=bufs[0].reshape(-1, W)[:B], dout=bufs[3], eng=bufs[4], c0=c0, n=n)
            if rel > 1e-5:  # which contributions are wrong: fit D[t, w, :] = c * dout[row, :] per row
                D = eng - gW
                tt, ww = np.unravel_index(np.argmax(np.abs(D).max(axis=2)), D.shape[:2])
                rr = np.arange(n) * c0 + tt
                dv = D[tt, ww]
                best = []
                for row in rr:
                    dd = d[row]
                    c = float(dv @ dd) / max(float(dd @ dd), 1e-300)
                    best.append((float(np.linalg.norm(dv - c * dd)), int(row), c, float(h[row, ww])))
                best.sort()
                bad_w = np.flatnonzero(np.abs(D[tt]).max(axis=1) > 1e-5 * np.abs(gW).max())
                print(f"  rank {r}: worst (t {tt}, w {ww}) D {np.array2string(dv, precision=3)}; bad w of t: {bad_w}; "
                      f"best single-row fits (resid, row, coef, h[row,w]): {best[:3]} |dv| {np.linalg.norm(dv):.3e}",
                      flush=True)
            s01 = np.array_equal(bufs[1], bufs[2]) and np.array_equal(bufs[1], bufs[0])
            diffrows = np.unique(np.flatnonzero((bufs[1] != bufs[0]).reshape(-1, W).any(axis=1)))
            diffcols = np.unique(np.flatnonzero((bufs[1] != bufs[0]).reshape(-1, W).any(axis=0)))
            print(f"  rank {r}: h snapshots equal {s01}; head_W grad vs numpy(h_final, dout) max rel {rel:.2e}; "
                  f"h changed after fwd: rows {diffrows[:10]} ({diffrows.size}) cols {diffcols[:10]} ({diffcols.size}); "
                  f"changed after loss pass: {not np.array_equal(bufs[2], bufs[0])}", flush=True)
            if r in SNAP0:
                d0 = (bufs[1] != SNAP0[r]).reshape(-1, W)
                rr, cc = np.nonzero(d0)
                print(f"  rank {r}: h after fwd vs rep 0: {rr.size} entries differ, rows {np.unique(rr)[:12]}, "
                      f"cols {np.unique(cc)[:16]}", flush=True)
            else:
                SNAP0[r] = bufs[1].copy()
            snaps.append(bufs)
    if GRAD_DIFF:  # the actor gradient's head leaves against this arm's first repeat, per rank
        W = t.SHARD_CASES[name]["W"]
        for r, e in enumerate(shards):
            b0, c0 = shard_tasks(t.SHARD_CASES[name]["T"], world, r)
            g = np.empty(snap_count(e, 4), np.float32)
            L.check(e.lib.mtsac_debug_read(e._h, 4, g.ctypes.data, g.size))
            key = (ARM, r)
            if key not in HEADG:
                HEADG[key] = g.copy()
                continue
            off = -(-8 * c0 // 64) * 64  # head_b (T_l x 8, 64-float aligned), then head_W [T_l][W][8]
            dif = np.flatnonzero(g != HEADG[key])
            if dif.size == 0:
                print(f"  [{ARM}] rank {r}: actor head grads bitwise equal to the arm's first repeat", flush=True)
                continue
            ref = HEADG[key]
            rel = np.abs(g[dif] - ref[dif]) / np.abs(ref[off:off + c0 * W * 8]).max()
            desc = []
            for i in dif[:24]:
                if i >= off:
                    tt, rem = divmod(int(i - off), W * 8)
                    desc.append(f"W(t{tt},w{rem // 8},o{rem % 8})")
                else:
                    desc.append(f"b({int(i) // 8},{int(i) % 8})")
            print(f"  [{ARM}] rank {r}: {dif.size} head-grad entries differ (max {rel.max():.2e} of the leaf max): "
                  f"{' '.join(desc)}", flush=True)
    logs = [e.logs() for e in shards]
    mus = [(e.get_params(L.ACTOR_ADAM_MU), e.get_params(L.CRITIC_ADAM_MU)) for e in shards]
    for e in shards:
        e.close()
    return logs, mus


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", type=int, default=3)
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--single", action="store_true")
    ap.add_argument("--name", default="s3_mt50_w2048")
    ap.add_argument("--snap", action="store_true", help="snapshot the actor's top activations in the step")
    ap.add_argument("--cu-slice", action="store_true", help="engine r on CU slice r of 8: no two engines share a CU")
    ap.add_argument("--alternate", action="store_true", help="alternate --cu-slice on / off between repeats")
    ap.add_argument("--queue-ab", action="store_true",
                    help="alternate full-mask streams (own queues, all CUs) and plain streams between repeats")
    ap.add_argument("--grad-diff", action="store_true", help="compare the actor head grads with the arm's first repeat")
    a = ap.parse_args()
    global SNAP, CU_SLICE, FULL_MASK, GRAD_DIFF, ARM
    SNAP = a.snap
    CU_SLICE = a.cu_slice
    GRAD_DIFF = a.grad_diff
    spec = t.SHARD_CASES[a.name]
    cfg, st, batch, en, ec, st1, want = t._problem(a.name)
    T, W = spec["T"], spec["W"]
    D = 39 + T
    keys = t.LOSS_KEYS + t.NORM_KEYS
    print("oracle", {k: want[k] for k in keys}, flush=True)
    ref_a, ref_c = st1.actor_opt.mu, st1.critic_opt.mu
    first = None
    for rep in range(a.repeats):

        if a.alternate:  # even repeats on CU slices, odd ones unsliced (same box, interleaved)
            CU_SLICE = rep % 2 == 0
            print(f"rep {rep}: cu slices {CU_SLICE}", flush=True)
        if a.queue_ab:  # even repeats full-mask (each stream its own queue), odd ones plain streams
            FULL_MASK = rep % 2 == 0
            ARM = "fullmask" if FULL_MASK else "plain"
            print(f"rep {rep}: arm {ARM}", flush=True)
        logs, mus = run_sharded(a.name, a.precision)
        same_ranks = all(lg == logs[0] for lg in logs)
        errs = {k: abs(logs[0][k] - want[k]) / max(abs(want[k]), 1e-30) for k in keys}
        print(f"rep {rep}: ranks equal {same_ranks}", {k: f"{v:.2e}" for k, v in errs.items()}, flush=True)
        print(f"rep {rep}: actor_grad_magnitude {logs[0]['metrics/actor_grad_magnitude']!r}", flush=True)
        if first is None:
            first = (logs, mus)
        else:
            same_logs = logs[0] == first[0][0]
            same_mu = all(np.array_equal(x[0], y[0]) and np.array_equal(x[1], y[1]) for x, y in zip(mus, first[1]))
            print(f"rep {rep}: bitwise equal to rep 0: logs {same_logs} moments {same_mu}", flush=True)
            if not same_mu:
                for r, (x, y) in enumerate(zip(mus, first[1])):
                    da = np.flatnonzero(x[0] != y[0])
                    dc = np.flatnonzero(x[1] != y[1])
                    print(f"   rank {r}: actor mu differs at {da.size} ({da[:8]}), critic at {dc.size}")
        for r in range(8):
            b0, c0 = shard_tasks(T, 8, r)
            ref = slice_heads(ref_a, D, W, 3, T, 8, None, b0, c0)
            nh = 8 * c0 + 8 * W * c0  # head_b, head_W
            d = np.abs(mus[r][0][:nh].astype(np.float64) - ref[:nh])
            rel = d / np.abs(ref[:nh]).max()
            if rel.max() > 1e-4:
                bad = np.flatnonzero(rel > 1e-4)
                print(f"  rep {rep} rank {r}: actor head mu max rel {rel.max():.2e} at {bad.size} entries "
                      f"(first {bad[:6]}, tasks {np.unique(((bad - 8 * c0) // (8 * W))[bad >= 8 * c0])}, "
                      f"w {np.unique(((bad - 8 * c0) % (8 * W)) // 8)[:12]})", flush=True)
        if rep == 0:
            for r in range(8):
                b0, c0 = shard_tasks(T, 8, r)
                sa = leaf_shapes(D, W, 3, c0, 8, None)
                sc = leaf_shapes(D + 4, W, 3, c0, 1, 2)
                leaf_errs(mus[r][0], slice_heads(ref_a, D, W, 3, T, 8, None, b0, c0), sa, f"  r{r} actor mu")
                if r == 0:
                    leaf_errs(mus[r][1], slice_heads(ref_c, D + 4, W, 3, T, 1, 2, b0, c0), sc, f"  r{r} critic mu")
    if a.single:
        e = t._engine(spec, a.precision)
        t._load(e, st)
        e.update(batch, en, ec)
        lg = e.logs()
        errs = {k: abs(lg[k] - want[k]) / max(abs(want[k]), 1e-30) for k in keys}
        print("single", {k: f"{v:.2e}" for k, v in errs.items()}, flush=True)
        leaf_errs(e.get_params(L.ACTOR_ADAM_MU), ref_a, leaf_shapes(D, W, 3, T, 8, None), "  single actor mu")
        e.close()


if __name__ == "__main__":
    main()
