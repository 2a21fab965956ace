"""Exposed collective time per bucket of one rank of an N-GPU MT50/W2048 job, on ONE GPU (DESIGN.md
section 4).  Two modes:

  run  T_LOCAL GBPS PRECISION   eager pipelined steps of the rank's task shard with the modelled trunk
                                all-reduce (mtsac_debug_set_collective_model: at every RCCL point a delay of
                                2 (N - 1) / N x bucket bytes over GBPS, on the collective stream); run it
                                under rocprofv3 --kernel-trace
  classes TRACE.csv [N]         any bucketing (the sharded optimizer's too): modelled and exposed time per
                                step by op class (N = critic hidden-layer ops per step: 2, or 4 sharded)
  parse TRACE.csv               per bucket (cm_delay_kernel launch, in issue order) of the last full steps:
                                its modelled length, how much of it the compute streams cover, and the
                                exposed rest; plus the step wall time

usage: python tools/coll_exposure.py run 7 150 split2h
       python tools/coll_exposure.py parse kernel_trace.csv"""
import csv
import sys

# the modelled collective launches one delay per bucket whose modelled time rounds to >= one 10-ns
# tick (the scalar tails only at low bandwidths, the head |p|^2 pair never), in this order per step
BUCKETS = ["critic layer 2", "critic layer 1", "critic layer 0 + tail", "actor layer 2", "actor layer 1",
           "actor layer 0 + tail"]


def run(tl, gbps, prec):
    import os

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from mtrl_amd import _lib as L
    from mtrl_amd.engine import MTSACEngine, make_config
    from mtrl_amd.init import init_mtsac

    T, W = 50, 2048
    nr = {7: 8, 13: 4, 25: 2}.get(tl, 8)
    p = {"split3": 1, "bf16": 2, "split2h": 3}[prec]
    cfg = make_config(num_tasks=T, task_begin=0, task_count=tl, obs_dim=39 + T, actor_width=W, critic_width=W,
                      batch_per_task=128, capacity=20_000, clip=0, precision=p)
    eng = MTSACEngine(cfg, device=0)
    actor, critic = init_mtsac(T, 39 + T, 4, W, 3, W, 3, 2, seed=1, task_begin=0, task_count=tl)
    eng.set_params(L.ACTOR, actor)
    eng.set_params(L.CRITIC, critic)
    eng.set_params(L.CRITIC_TARGET, critic)
    eng.buffer_fill_synthetic(1234)
    eng.seed_rng(1)
    eng.enable_graph(False)
    L.check(eng.lib.mtsac_debug_set_collective_model(eng._h, nr, gbps, 0))
    eng.lib.mtsac_debug_set_pipeline(eng._h, 1)
    eng.update_many(4)
    eng.synchronize()
    eng.update_many(12)
    eng.synchronize()
    eng.close()
    print(f"ran T_local={tl} N={nr} bus {gbps} GB/s {prec}")


def union(iv):
    tot, cur = 0, None
    for s, e in sorted(iv):
        if cur is None or s > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [s, e]
        else:
            cur[1] = max(cur[1], e)
    return tot + (cur[1] - cur[0] if cur else 0)


def parse(path):
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in csv.DictReader(open(path)))
    delays = [(s, e) for s, e, n in rows if "cm_delay" in n]
    comp = [(s, e) for s, e, n in rows if "cm_" not in n]
    big = max(e - s for s, e in delays)
    # classify by modelled length: critic hidden layers ~big, actor hidden layers ~big / 2 (one member),
    # the rest small; a step starts at its first critic hidden-layer bucket
    steps, cur = [], None
    for s, e in delays:
        d = e - s
        kind = 0 if d > 0.75 * big else 1 if d > 0.35 * big else 2
        if kind == 0 and (cur is None or cur["phase"] > 0):
            cur = {"phase": 0, "b": [[] for _ in BUCKETS], "n0": 0, "n1": 0, "first": s}
            steps.append(cur)
        if cur is None:
            continue
        if kind == 0:
            j = min(cur["n0"], 1)
            cur["n0"] += 1
        elif kind == 1:
            cur["phase"] = 1
            j = 3 + min(cur["n1"], 1)
            cur["n1"] += 1
        else:
            j = 2 if cur["phase"] == 0 else 5
        cur["b"][j].append((s, e))
    steps = [st for st in steps[1:-1] if st["n0"] == 2 and st["n1"] == 2]  # whole steps, the first skipped
    per = [[] for _ in BUCKETS]
    for st in steps:
        for j, iv in enumerate(st["b"]):
            m = sum(e - s for s, e in iv)
            cov = sum(union([(max(s, cs), min(e, ce)) for cs, ce in comp if cs < e and ce > s]) for s, e in iv)
            per[j].append((m, cov))
    firsts = [st["first"] for st in steps]
    wall = (firsts[-1] - firsts[0]) / (len(firsts) - 1) / 1e3
    print(f"steps {len(steps)}: wall {wall:.1f} us per step (first bucket to first bucket)")
    print(f"{'bucket':22s} {'modelled us':>11s} {'covered us':>11s} {'exposed us':>11s}")
    tot = 0.0
    for name, v in zip(BUCKETS, per):
        m = sum(x for x, _ in v) / len(v) / 1e3
        c = sum(y for _, y in v) / len(v) / 1e3
        tot += m - c
        print(f"{name:22s} {m:11.1f} {c:11.1f} {m - c:11.1f}")
    print(f"{'sum':22s} {'':11s} {'':11s} {tot:11.1f}")


def parse_classes(path, per_step_big):
    """Any bucketing (the sharded optimizer's reduce-scatters and all-gathers too): the delays by
    modelled-length class -- critic hidden-layer ops (the longest), actor hidden-layer ops (about half),
    the rest -- their modelled and exposed time per step; per_step_big = critic hidden-layer ops per step
    (2 all-reduce, 4 reduce-scatter + all-gather)."""
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in csv.DictReader(open(path)))
    delays = [(s, e) for s, e, n in rows if "cm_delay" in n]
    comp = [(s, e) for s, e, n in rows if "cm_" not in n]
    big = max(e - s for s, e in delays)
    firsts = [s for s, e in delays if e - s > 0.75 * big]
    # skip the warm-up step and the last (partial) one
    t0, t1 = firsts[per_step_big], firsts[-per_step_big]
    out = {"critic hidden-layer ops": [0.0, 0.0], "actor hidden-layer ops": [0.0, 0.0], "other": [0.0, 0.0]}
    for s, e in delays:
        if not (t0 <= s < t1):
            continue
        d = e - s
        k = "critic hidden-layer ops" if d > 0.75 * big else "actor hidden-layer ops" if d > 0.35 * big else "other"
        cov = union([(max(s, cs), min(e, ce)) for cs, ce in comp if cs < e and ce > s])
        out[k][0] += d
        out[k][1] += d - cov
    steps = sum(1 for f in firsts if t0 <= f < t1) / per_step_big
    print(f"steps {steps:.0f}: wall {(t1 - t0) / steps / 1e3:.1f} us per step")
    print(f"{'class':26s} {'modelled us':>11s} {'exposed us':>11s}   (per step)")
    tot = 0.0
    for k, (m, x) in out.items():
        tot += x
        print(f"{k:26s} {m / steps / 1e3:11.1f} {x / steps / 1e3:11.1f}")
    print(f"{'sum':26s} {'':11s} {tot / steps / 1e3:11.1f}")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]), float(sys.argv[3]), sys.argv[4])
    elif sys.argv[1] == "classes":
        parse_classes(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 2)
    else:
        parse(sys.argv[2])
