#!/usr/bin/env python3
"""How the two chunk pipelines of the chain overlap in a rocprofv3 --kernel-trace of bench.py:
the device time spent in each concurrency state ({PC}, {PC, PC}, {PC, MTD}, {MTD, MTD}, ...)
over the timed steps (the last `steps` x launches-per-step chain launches).  In-phase lanes
(PC beside PC, MTD beside MTD) pair two kernels that want the same resource; PC beside MTD
pairs the compute-heavier one with the stream-heavier one.

Usage: lane_overlap.py <kernel_trace.csv> --steps K (--warmup W | --warmup-from bench.log) [--json out.json]
"""
import collections
import csv
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import short  # noqa: E402

OURS = {"pc_kernel": "PC", "mtd_kernel": "MTD", "cfar_r_kernel": "CFAR_R", "cfar_hits_kernel": "CFAR_R"}


def main():
    a = sys.argv[1:]
    steps = int(a[a.index("--steps") + 1])
    if "--warmup-from" in a:   # the warmup count bench.py chose (its JSON line's "warmup")
        line = [ln for ln in open(a[a.index("--warmup-from") + 1]) if ln.startswith("{")][-1]
        warmup = int(json.loads(line)["warmup"])
    else:
        warmup = int(a[a.index("--warmup") + 1])
    rows = []
    for r in csv.DictReader(open(a[0])):
        k = OURS.get(short(r["Kernel_Name"]))
        if k:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    rows.sort()
    per_step = len(rows) // (steps + warmup)
    tail = rows[-steps * per_step:]
    ev = []
    for s, e, k in tail:
        ev.append((s, 1, k))
        ev.append((e, -1, k))
    ev.sort(key=lambda x: (x[0], x[1]))
    running = collections.Counter()
    state_ns = collections.Counter()
    t_prev = ev[0][0]
    for t, d, k in ev:
        if t > t_prev:
            key = "+".join(sorted(running.elements())) or "idle"
            state_ns[key] += t - t_prev
        running[k] += d
        if running[k] == 0:
            del running[k]
        t_prev = t
    span = ev[-1][0] - ev[0][0]
    out = {"span_ms_per_step": round(span / 1e6 / steps, 4),
           "states_ms_per_step": {k: round(v / 1e6 / steps, 4) for k, v in state_ns.most_common()},
           "states_frac": {k: round(v / span, 4) for k, v in state_ns.most_common()}}
    print(json.dumps(out, indent=1))
    if "--json" in a:
        json.dump(out, open(a[a.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
