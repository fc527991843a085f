#!/usr/bin/env python3
"""Why a caller's new output arrays are expensive to RELEASE after a host-API call (VERDICT r5
weak #6; tools/host_fresh_probe.py measured ~4.5 ms of `del` per 32-CPI call at c3): for three
ways of filling fresh numpy outputs -- rsp_pc_mtd_cfar (library copy threads, with and without
the output prefault), a numpy copy on one thread, and no fill -- the transparent-huge-page
share of the arrays' memory (/proc/self/smaps AnonHugePages) and the time of their release.

    python tools/host_thp_probe.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "radar-signal-process_amd"))


def thp_kib(arrs):
    """AnonHugePages / Rss (KiB) of the mappings holding the arrays' data."""
    spans = [(a.ctypes.data, a.ctypes.data + a.nbytes) for a in arrs]
    hp = rss = 0
    cur = None
    with open("/proc/self/smaps") as f:
        for line in f:
            p = line.split()
            if "-" in p[0] and len(p) >= 5 and all(c in "0123456789abcdef-" for c in p[0]):
                lo, hi = (int(x, 16) for x in p[0].split("-"))
                cur = any(lo < e and b < hi for b, e in spans)   # every mapping the data overlaps
            elif cur and p[0] == "AnonHugePages:":
                hp += int(p[1])
            elif cur and p[0] == "Rss:":
                rss += int(p[1])
    return hp, rss


def numa_kib(arrs):
    """KiB of the arrays' mappings per NUMA node (/proc/self/numa_maps N<k>= page counts)."""
    spans = [(a.ctypes.data, a.ctypes.data + a.nbytes) for a in arrs]
    starts = []
    with open("/proc/self/maps") as f:
        for line in f:
            lo, hi = (int(x, 16) for x in line.split()[0].split("-"))
            if any(lo < e and b < hi for b, e in spans):
                starts.append(lo)
    per = {}
    with open("/proc/self/numa_maps") as f:
        for line in f:
            p = line.split()
            if int(p[0], 16) not in starts:
                continue
            kps = 4
            for t in p:
                if t.startswith("kernelpagesize_kB="):
                    kps = int(t.split("=")[1])
            for t in p:
                if t.startswith("N") and "=" in t:
                    k, v = t.split("=")
                    per[k] = per.get(k, 0) + int(v) * kps
    return per


def main():
    from rsp import _capi as capi, presets, synth
    from rsp.engine import Engine
    spec = presets.v2(128, 4096)
    cf = presets.default_cfar(spec)
    eng = Engine(spec)
    n = 32
    h = np.ascontiguousarray(np.swapaxes(synth.echo_numpy(spec, n, seed=5).astype(np.complex128), 1, 2))
    V, Ro = eng.shape
    src = np.ones((n, Ro, V), np.float32)
    import ctypes
    cpu, node = ctypes.c_uint(), ctypes.c_uint()
    ctypes.CDLL(None).syscall(309, ctypes.byref(cpu), ctypes.byref(node), None)   # SYS_getcpu (x86-64)
    out = {"thp_enabled": open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip(),
           "prefault_numa": os.environ.get("RSP_PREFAULT_NUMA", "1"), "caller_cpu_node": [cpu.value, node.value]}
    for mode in ("library", "numpy_fill", "untouched"):
        rows = []
        for rep in range(4):
            o = (np.empty((n, Ro, V), np.float32), np.empty((n, Ro, V), np.uint8), np.empty((n, Ro, V), np.uint8))
            if mode == "library":
                eng.pc_mtd_cfar(h, cf, layout=capi.RSP_COLMAJOR, out_layout=capi.RSP_COLMAJOR, out=o)
            elif mode == "numpy_fill":
                o[0][...] = src
                o[1][...] = 1
                o[2][...] = 1
            hp, rss = thp_kib(o)
            nodes = numa_kib(o)
            t0 = time.perf_counter()
            del o
            rows.append({"anon_huge_kib": hp, "rss_kib": rss, "numa_kib": nodes,
                         "release_ms": round((time.perf_counter() - t0) * 1e3, 3)})
        out[mode] = rows
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
