#!/usr/bin/env python3
"""Median phase times of the host-path trace lines (RSP_HOST_TRACE=1, rsp_capi.cpp HostTrace)
in a stderr capture:  python tools/parse_host_trace.py gpurun_out/mex_trace.err"""
import statistics as st
import sys

KEYS = ["setup", "stage_in", "enqueue", "stage_out", "sync", "total", "h2d", "chain", "d2h",
        "narrow", "wait", "widen"]


def main(path):
    rows = [ln.split() for ln in open(path) if ln.startswith("rsp_host_trace")]
    vals = {k: [] for k in KEYS}
    for f in rows:
        for k in KEYS:
            if k in f:
                vals[k].append(float(f[f.index(k) + 1]))
    print(len(rows), {k: round(st.median(v), 1) for k, v in vals.items() if v})


if __name__ == "__main__":
    main(sys.argv[1])
