#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace of bench.py (run with --no-profile) for the chain's
kernels: per-kernel launches / mean / total duration, and the device span of the timed steps
(the last `steps` x launches-per-step chain launches), to set beside bench.py's own
ms_per_step and roofline.

Usage: trace_summary.py <run_kernel_trace.csv> --steps K (--warmup W | --warmup-from bench.log) [--json out.json]
"""
import collections
import csv
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import short  # noqa: E402

OURS = ("pc_kernel", "mtd_kernel", "cfar_r_kernel", "cfar_v_kernel", "chain_kernel")


def main():
    a = sys.argv[1:]
    path = a[0]
    steps = int(a[a.index("--steps") + 1])
    if "--warmup-from" in a:   # the warmup count bench.py chose (its JSON line's "warmup")
        line = [ln for ln in open(a[a.index("--warmup-from") + 1]) if ln.startswith("{")][-1]
        warmup = int(json.loads(line)["warmup"])
    else:
        warmup = int(a[a.index("--warmup") + 1])
    rows = []
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        if "chain_kernel" in r["Kernel_Name"]:
            k = "chain_kernel"
        if k in OURS:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    rows.sort()
    per_step = len(rows) // (steps + warmup)
    tail = rows[-steps * per_step:]
    span_ms = (max(e for _, e, _ in tail) - tail[0][0]) / 1e6
    busy = collections.defaultdict(list)
    for s, e, k in tail:
        busy[k].append((e - s) / 1e3)
    out = {"launches_per_step": per_step, "timed_steps": steps, "span_ms_per_step": round(span_ms / steps, 4),
           "kernels": {k: {"launches_per_step": len(v) // steps, "avg_us": round(sum(v) / len(v), 2),
                           "ms_per_step": round(sum(v) / 1e3 / steps, 4)} for k, v in busy.items()}}
    out["kernel_sum_ms_per_step"] = round(sum(v["ms_per_step"] for v in out["kernels"].values()), 4)
    print(json.dumps(out, indent=1))
    if "--json" in a:
        json.dump(out, open(a[a.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
