#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/g*/run_counter_collection.csv) per kernel.

Prints the mean counter value per dispatch and derived figures.  gfx950 corrections
(MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of a wide coalesced read,
so read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is exact for 16-B stores (KiB units).
Usage: pmc_summary.py [pmc_dir] [--json out.json --cpis-per-dispatch N]
"""
import collections
import csv
import glob
import json
import os
import sys


# kernel-name fragment -> the bench's kernel label (rsp_profile ids)
LABELS = (("pc_persist_kernel", "pc_kernel"), ("pc_mf_kernel", "pc_kernel"), ("pc_kernel", "pc_kernel"),
          ("mtd_bluestein_kernel", "mtd_kernel"), ("mtd_kernel", "mtd_kernel"),
          ("cfar_hits_kernel", "cfar_r_kernel"), ("cfar_hits57_kernel", "cfar_r_kernel"), ("cfar_r16_kernel", "cfar_r_kernel"),
          ("cfar_r_kernel", "cfar_r_kernel"), ("cfar_r_generic_kernel", "cfar_r_kernel"),
          ("cfar_v_kernel", "cfar_v_kernel"), ("fillBuffer", "flag_memset"), ("hits_kernel", "hits_kernel"),
          ("measure_kernel", "measure_kernel"), ("prefilter_kernel", "prefilter_kernel"), ("mti_chain_kernel", "mti_chain_kernel"),
          ("ingest_ddc_kernel", "ingest_ddc_kernel"), ("ingest_check_kernel", "ingest_check_kernel"))


def short(name):
    for k, label in LABELS:
        if k in name:
            return label
    return name[:40]


def load(pmc_dir):
    """Per kernel: counter -> values, and the dispatch durations (us) of the FETCH_SIZE pass and
    of the pass that carried GRBM_GUI_ACTIVE (each counter is normalised by its own pass)."""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    dur_grbm = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(pmc_dir, "g*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            if r["Counter_Name"] in ("FETCH_SIZE",):
                dur[k].append(us)
            if r["Counter_Name"] in ("GRBM_GUI_ACTIVE",):
                dur_grbm[k].append(us)
    return acc, dur, dur_grbm


# GRBM_GUI_ACTIVE counts the busy cycles of a dispatch's sampling window, summed over the 8 XCDs;
# the window exceeds the kernel by a roughly fixed launch overhead, so GRBM/8/duration reads high
# on short dispatches (MI355X_MICROARCH.md, DVFS give-back: within 3 % only from ~10 ms, high
# below ~0.3 ms).  The clock is reported only for dispatches of at least this length.
MIN_CLOCK_US = 300.0


def main():
    args = sys.argv[1:]
    pmc_dir = args[0] if args and not args[0].startswith("--") else "gpurun_out/pmc"
    acc, dur, dur_grbm = load(pmc_dir)
    rows = {}
    for k, cs in acc.items():
        if not any(x in k for x in ("pc_", "mtd", "cfar", "memset", "hits_kernel", "measure_kernel", "prefilter_kernel", "mti_chain", "ingest")):
            continue
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = sum(dur[k]) / len(dur[k]) if dur[k] else float("nan")
        rd = 2 * m.get("FETCH_SIZE", 0) * 1024
        wr = m.get("WRITE_SIZE", 0) * 1024
        row = {"dispatches": len(cs.get("FETCH_SIZE", [])), "avg_us_profiled": round(d, 2),
               "read_MB": round(rd / 1e6, 3), "write_MB": round(wr / 1e6, 3),
               "GBps": round((rd + wr) / (d * 1e3), 1) if d == d and d > 0 else None}
        for c in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                  "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS",
                  "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                  "SQ_ACTIVE_INST_ANY", "TCC_HIT_sum", "TCC_MISS_sum", "GRBM_GUI_ACTIVE",
                  "SQ_LDS_IDX_ACTIVE", "SQ_LDS_DATA_FIFO_FULL", "SQ_LDS_CMD_FIFO_FULL", "SQ_INST_LEVEL_LDS",
                  "SQ_LEVEL_WAVES", "SQ_BUSY_CU_CYCLES", "SQ_INST_LEVEL_VMEM", "SQ_INST_CYCLES_VMEM_RD",
                  "SQ_INST_CYCLES_VMEM_WR", "SQ_VMEM_TA_ADDR_FIFO_FULL", "SQ_VMEM_WR_TA_DATA_FIFO_FULL",
                  "SQ_THREAD_CYCLES_VALU"):
            if c in m:
                row[c] = m[c]
        if "TCC_HIT_sum" in m:
            row["L2_hit"] = round(m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"]), 3)
        if "GRBM_GUI_ACTIVE" in m and dur_grbm[k]:
            dg = sum(dur_grbm[k]) / len(dur_grbm[k])   # the GRBM pass's own dispatch durations
            row["grbm_pass_avg_us"] = round(dg, 2)
            if dg >= MIN_CLOCK_US:
                row["eff_clock_GHz"] = round(m["GRBM_GUI_ACTIVE"] / 8 / (dg * 1e3), 3)
            else:
                row["eff_clock_GHz"] = None
                row["eff_clock_note"] = "dispatch < %.0f us: the GRBM sampling window exceeds the kernel" % MIN_CLOCK_US
        if "SQ_WAVE_CYCLES" in m and "SQ_WAIT_ANY" in m:
            wc = m["SQ_WAVE_CYCLES"]
            row["wait_frac"] = round(m["SQ_WAIT_ANY"] / wc, 3)
            row["valu_frac"] = round(m.get("SQ_ACTIVE_INST_VALU", 0) / wc, 3)
            row["lds_frac"] = round(m.get("SQ_ACTIVE_INST_LDS", 0) / wc, 3)
            if "SQ_WAIT_INST_ANY" in m:   # issue stalls (dependency / pipe busy), disjoint from WAIT_ANY
                row["issue_stall_frac"] = round(m["SQ_WAIT_INST_ANY"] / wc, 3)
            if "SQ_ACTIVE_INST_ANY" in m:
                row["active_frac"] = round(m["SQ_ACTIVE_INST_ANY"] / wc, 3)
            if "SQ_INSTS_VALU" in m and m.get("SQ_WAVES"):
                row["valu_insts_per_wave"] = round(m["SQ_INSTS_VALU"] / m["SQ_WAVES"], 1)
        rows[k] = row
    for k, r in rows.items():
        print(k)
        for c, v in r.items():
            print("   %-22s %s" % (c, v))
    if "--json" in args:
        # bench.py reads bytes_per_unit (roofline.traffic) and kernels[<name>].hbm_bytes_per_launch
        out = args[args.index("--json") + 1]
        units = float(args[args.index("--units-total") + 1]) if "--units-total" in args else None
        doc = {"note": "rocprofv3 --pmc, one counter group per pass; HBM-side bytes = 2*FETCH_SIZE*1024 "
                       "(gfx950 FETCH_SIZE halving, MI355X_MICROARCH.md HBM) + WRITE_SIZE*1024 per dispatch; "
                       "Infinity-Cache hits are counted by these counters. bytes_per_unit = the bytes of every "
                       "dispatch of the chain's kernels in the profiled run / the CPIs (windows) it processed",
               "units_total": units, "kernels": {}}
        total = 0.0
        for k, r in rows.items():
            r = dict(r)
            r["hbm_bytes_per_launch"] = int(round((r["read_MB"] + r["write_MB"]) * 1e6))
            total += r["hbm_bytes_per_launch"] * r["dispatches"]
            doc["kernels"][k] = r
        if units:
            doc["bytes_per_unit"] = round(total / units)
        json.dump(doc, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
