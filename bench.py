#!/usr/bin/env python3
"""Benchmark: CPIs/s through PC -> MTD -> 0-v -> 2-D CA-CFAR (BASELINE.json metric).

Default workload (config c3 of BASELINE.json, the metric's config): 128 pulses x 4096 range
bins, complex fp32 echo, batch 1024 CPIs per GPU, `v2` preset (fun_MTD_produce's 3-segment
pulse compression, kaiser-8 MTD with fftshift, 0-v /150) followed by main_cfar's /20 0-v and
executeCFAR per PC segment (ref 5, guard 7, T 5, GO, range CFAR on).  A step is one pass of
the chain over the batch, inputs resident in HBM.  Synthetic echoes (SURVEY.md §8d recipe,
noise drawn on the GPU).  --config c2 / c4 / c5 select the other BASELINE configs (c4: the
sliding-window stream, unit = window; c5: 512 x 16384 fp16 I/Q).

Multi-GPU: one process per GPU (torchrun); each rank owns a contiguous shard of the CPI
stream (weak scaling, no data-path collective: CPIs are independent); the only collectives
are the timing barrier and the max-over-ranks of the elapsed time.

Prints ONE JSON line (rank 0).  See DESIGN.md for the roofline accounting.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "radar-signal-process_amd"))

METRIC = "CPIs/sec (4096 range × 128 pulse) through PC→MTD→CFAR; achieved HBM GB/s"
HBM_PEAK_GBPS = 8000.0


# BASELINE.json configs.  mode "window": batch = frame pairs per GPU per step,
# each giving `win` windowed CPIs (MTD/main_produce_dataset_win_xzr_v2.m:94-144).
WARMUP_S = 0.3   # default warmup: seconds of device work before the timed region

CONFIGS = {
    "c2": dict(P=128, R=4096, batch=256, cfar=False, half=False, win=0),
    "c3": dict(P=128, R=4096, batch=1024, cfar=True, half=False, win=0),
    "c4": dict(P=256, R=8192, batch=32, cfar=True, half=False, win=4),
    "c5": dict(P=512, R=16384, batch=64, cfar=True, half=True, win=0),
    # SURVEY.md §8f-2 (not a BASELINE config): raw PRT records -> DBF beams, v2 capture frames
    "ingest": dict(P=332, R=3404, batch=8, cfar=False, half=False, win=0),
    # motionParaMeasure over DMX long-part planes (2048 Doppler x 512 range)
    "measure": dict(P=2048, R=512, batch=256, cfar=False, half=False, win=0),
    # iSTC gain + MTI (lag 30) on c3-shaped echoes ahead of the chain
    "prefilter": dict(P=128, R=4096, batch=1024, cfar=False, half=False, win=0),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed warmup steps, >= 1 (the first one counts launches); default: as many as "
                         "fill %.1f s of device work, at least 3 -- the GPU's clocks ramp up over its first "
                         "~50 ms of work (tools/warmup_probe.py: c3 4.1 -> 3.55 ms per step)" % WARMUP_S)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--preset", default="v2", choices=["v2", "dmx"])
    ap.add_argument("--P", type=int, default=None)
    ap.add_argument("--R", type=int, default=None)
    ap.add_argument("--batch", type=int, default=None, help="CPIs (window mode: frame pairs) per GPU per step")
    ap.add_argument("--no-cfar", action="store_true", help="PC + MTD only")
    ap.add_argument("--half", action="store_true", help="fp16 I/Q input")
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--host-path", action="store_true",
                    help="also time the PCIe-inclusive host entry point (rsp_pc_mtd_cfar, C128 column-major "
                         "host echo as MATLAB holds it, RDM + flags back to host)")
    ap.add_argument("--host-batch", type=int, default=1,
                    help="--host-path: CPIs per host call besides 32 (MATLAB calls one CPI per call)")
    ap.add_argument("--ingest-mix", action="store_true",
                    help="--config ingest: frames whose PRTs cycle through payload types 1 (DDC), 0 (ADC) and 3 "
                         "(FrameDataRead_xzr.m:57-198), 16 beams, instead of all-DDC capture frames")
    ap.add_argument("--prefilter", action="store_true",
                    help="fused iSTC (a synthetic stc curve) + MTI lag 30 in the chain (rsp_set_prefilter)")
    ap.add_argument("--streams", type=int, default=0, help="chunk pipelines (0 = library default)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 = skip)")
    ap.add_argument("--no-profile", action="store_true", help="no per-kernel HIP events in the timed region")
    ap.add_argument("--profile-every", type=int, default=7,
                    help="(unused; kept for old command lines)")
    ap.add_argument("--lane-steps", type=int, default=2,
                    help="steps of the single-lane per-kernel pass after the timed region (0 = skip)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: gloo collectives, a stub step; checks the rank launcher, shards and halo")
    ap.add_argument("--share-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank on device 0, gloo collectives (value not a result)")
    ap.add_argument("--dry-run-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)   # launcher test hook
    # test hook: every rank on this device WITHOUT --share-device (the duplicate-device guard must fire);
    # in --dry-run, a fake device identity shared by all ranks
    ap.add_argument("--force-device", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--launch-timeout", type=float, default=1800.0,
                    help="--gpus N launcher: seconds before the ranks are stopped")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    args.P = args.P or cfg["P"]
    args.R = args.R or cfg["R"]
    args.batch = args.batch or cfg["batch"]
    args.no_cfar = args.no_cfar or not cfg["cfar"]
    args.half = args.half or cfg["half"]
    args.win = cfg["win"]
    return args


def host_cpus():
    """The host's CPU facts for the baseline: nproc (os.cpu_count), the CPUs this process may
    run on (sched_getaffinity), the cgroup CPU quota (cpu.max), the CPU model (lscpu), and the
    thread count used = the smallest of affinity and quota (on the GPU box nproc shows the whole
    machine, many times this job's share)."""
    import math
    import subprocess
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        info["affinity"] = os.cpu_count()
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    info["cgroup_quota_cpus"] = quota
    try:
        lscpu = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in lscpu.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core", "CPU(s)"):
                info["lscpu_" + k.strip().lower().replace(" ", "_").replace("(s)", "s")] = v.strip()
    except (OSError, subprocess.SubprocessError):
        pass
    n = info["affinity"] or 1
    if quota:
        n = min(n, max(1, int(math.floor(quota))))
    info["threads_used"] = n
    return info


def host_path(eng, echo, cfar, args, seconds=1.5):
    """The MEX-style host entry point: rsp_pc_mtd_cfar on a host complex128 echo in MATLAB's
    column-major layout ([b][R][P] C order), RDM and flags returned to host column-major -- H2D
    of 16 B per sample, the chain, D2H of 6 B per cell (RDM f32 + flag + flagV), and the
    layout/precision conversions on the GPU -- at args.host_batch CPIs per call (MATLAB calls
    fun_MTD_produce once per CPI: MTD/main_produce_dataset_win_xzr_v2.m:136) and at 32.
    Secondary figure; never the headline value."""
    import numpy as np
    from rsp import _capi as capi
    if echo.dtype != __import__("torch").complex64:
        return None
    out = {"input": "host C128 column-major (MATLAB layout), pageable numpy buffers",
           "output": "host f32 RDM + u8 flag/flagV, column-major",
           "bytes_per_cpi_pcie": int(eng.spec.P * eng.spec.R * 8 + eng.spec.V * eng.spec.R_out * 6),
           "note": "PCIe-inclusive synchronous host API (rsp_pc_mtd_cfar): chunked H2D / chain / D2H "
                   "pipeline through pinned staging rings; the C128 echo is narrowed to C64 by the host "
                   "copy threads, so PCIe carries 8 B per sample"}
    sizes = sorted({min(32, echo.shape[0]), min(args.host_batch, echo.shape[0])}, reverse=True)
    V, Ro = eng.shape
    for n in sizes:
        h = np.ascontiguousarray(np.swapaxes(echo[:n].cpu().numpy().astype(np.complex128), 1, 2))
        # outputs: fresh arrays per call (first-touch page faults in the caller's memory, the
        # worst case) and arrays reused across calls
        reused = (np.empty((n, Ro, V), np.float32), np.empty((n, Ro, V), np.uint8), np.empty((n, Ro, V), np.uint8))
        for mode, o in (("fresh", None), ("reused", reused)):
            eng.pc_mtd_cfar(h, cfar, layout=capi.RSP_COLMAJOR, out_layout=capi.RSP_COLMAJOR, out=o)   # warm-up
            calls, t0 = 0, time.perf_counter()
            while calls < 3 or time.perf_counter() - t0 < seconds:
                eng.pc_mtd_cfar(h, cfar, layout=capi.RSP_COLMAJOR, out_layout=capi.RSP_COLMAJOR, out=o)
                calls += 1
            el = time.perf_counter() - t0
            rate = n * calls / el
            out["batch%d_%s" % (n, mode)] = {"value": round(rate, 1), "unit": "CPI/s", "cpis_per_call": n,
                                             "calls": calls, "ms_per_call": round(el / calls * 1e3, 3),
                                             "pcie_GBps": round(rate * out["bytes_per_cpi_pcie"] / 1e9, 2)}
    first = out["batch%d_reused" % sizes[0]]
    out["value"], out["unit"], out["cpis_per_call"] = first["value"], "CPI/s", first["cpis_per_call"]
    out["value_note"] = "value = %d CPIs per call with reused output arrays; *_fresh: new arrays every call" % sizes[0]
    return out


def cpu_baseline(spec, cfar, seconds, unit="CPI/s"):
    """The CPU path beside the GPU: the fp64 C restatement of the MATLAB chain
    (oracle/rsp_oracle.c, OpenMP over CPIs) timed on this host's CPU share and on one thread,
    on a bounded sample of the same workload, plus the loop-faithful numpy oracle at c1
    (64 x 1024, one CPI: the 'MATLAB-semantics' plumbing baseline)."""
    if seconds <= 0:
        return None
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import coracle
    import rsp_ref
    from rsp import presets, synth
    cpus = host_cpus()
    threads = cpus["threads_used"]
    pool_n = max(threads, 8)
    echo = synth.echo_numpy(spec, pool_n, seed=1003).astype(np.complex128)
    pre = coracle.preset(spec.name, spec.P, spec.R)
    c = cfar.as_dict() if cfar is not None else None
    if c is not None:
        c["zero_v_div"] = cfar.zero_v_div

    def run(nthreads, budget, n):
        done, t0 = 0, time.perf_counter()
        while True:
            rdm = coracle.pc_mtd(echo[:n], pre, nthreads=nthreads)
            if c is not None:
                coracle.cfar(rdm, c, cfar.segments, nthreads=nthreads)
            done += n
            el = time.perf_counter() - t0
            if el >= budget:
                return done, el

    done, el = run(threads, 0.6 * seconds, pool_n)
    done1, el1 = run(1, 0.3 * seconds, 1)
    # c1: the numpy loop-faithful oracle, one 64 x 1024 CPI, fun_MTD_produce + main_cfar chain
    s1 = presets.v2(64, 1024)
    e1 = synth.echo_numpy(s1, 1, seed=1001)[0].astype(np.complex128)
    c1 = presets.default_cfar(s1)
    cd = c1.as_dict()
    t1 = time.perf_counter()
    m1 = rsp_ref.fun_MTD_produce_v2(e1, rsp_ref.v2_params(64, 1024))
    rsp_ref.main_cfar_chain(m1, cd, [(a + 1, b) for a, b in c1.segments], c1.zero_v_div)
    c1_s = time.perf_counter() - t1
    return {"value": done / el, "unit": unit, "cores": threads, "kind": "port",
            "sample": "%d CPIs (%d x %d, %s preset%s) in %.1f s on %d threads: a pool of %d distinct synthetic "
                      "CPIs cycled; fp64 C restatement of the MATLAB chain with OpenMP over CPIs (MATLAB itself is "
                      "not available)" % (done, spec.P, spec.R, spec.name, " + CFAR" if c else "", el, threads, pool_n),
            "one_thread": {"value": done1 / el1, "unit": unit, "sample": "%d CPIs in %.1f s" % (done1, el1)},
            "c1_numpy_oracle_s_per_cpi": round(c1_s, 3),
            "host": cpus}


def hbm_ceiling():
    """The measured streaming ceiling of this part (profiles/hbm_ceiling.json, written from
    tools/micro/hbm_ceiling.hip): copy (equal read and write bytes, the chain's mix), read-only,
    write-only GB/s."""
    p = os.path.join(ROOT, "profiles", "hbm_ceiling.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)


def pmc_traffic(tag):
    """HBM bytes per launch from a committed rocprofv3 PMC summary, if one exists."""
    p = os.path.join(ROOT, "profiles", "pmc_%s.json" % tag)
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)


def bench_ingest(args, world, rank, local, dev, dist):
    """--config ingest: frames/s through rsp_ingest_frame_dev (record parse + DBF), v2 capture
    frames (332 PRTs x 3404 samples x 16 channels int16 I/Q -> 13 beams complex64), records
    resident in HBM; each rank decodes its own frames (no collective)."""
    import torch
    sys.path[:0] = [os.path.join(ROOT, "tests", "golden")]
    from make_golden_ingest import synth_frame, synth_mixed_frame   # synthetic record writers (test data only)
    from rsp import ingest, shard
    B = args.batch
    lo, _ = shard.weak_shard(B, rank)
    if args.ingest_mix:
        # PRT p carries payload type (1, 0, 3)[p % 3]: DDC, ADC (its matrix passes the :171 size
        # check only with channel_num == beam_num, hence 16 beams) and a type without a decode
        # case (a zero row).  Every PRT is valid, so the frame decodes to its last row.  (The
        # 24-bit DBF branch never passes the size check with 16 channels: the reference marks
        # it unfinished.)
        NB = 16
        dbf, cfg, rec = synth_mixed_frame([(1, 0, 3)[p % 3] for p in range(args.P)], args.R, 16, NB, seed=3000 + lo)
    else:
        NB = 13
        _, dbf, _, cfg, rec = synth_frame(args.P, args.R, 16, NB, seed=3000 + lo)
    ing = ingest.Ingest(local)
    d_rec = torch.frombuffer(bytearray(rec), dtype=torch.uint8).to(dev)
    frames = d_rec.repeat(B)                          # B distinct frame slots of identical records
    d_dbf = ing.dbf_device(dbf)
    out = torch.empty((B, NB, args.P, args.R), dtype=torch.complex64, device=dev)
    stream = torch.cuda.current_stream(dev)
    nb = len(rec)

    def step():
        for f in range(B):
            ing.decode_dev(frames[f * nb:(f + 1) * nb], nb, cfg, d_dbf, out=out[f], stream=stream)

    warm(step, args, dev)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1)
    if world > 1:
        elapsed = shard.max_over_ranks(elapsed, dist, device=dev)
    cpu = None
    if rank == 0 and args.cpu_seconds > 0:
        # the fp64 oracle restatement of FrameDataRead_xzr.m on one host thread
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import ingest_ref
        from threadpoolctl import threadpool_limits
        done, t1 = 0, time.perf_counter()
        with threadpool_limits(limits=1):
            while time.perf_counter() - t1 < args.cpu_seconds or done == 0:
                ingest_ref.FrameReader().read(ingest_ref.BytesStream(rec), dbf, cfg, 0)
                done += 1
        el = time.perf_counter() - t1
        cpu = {"value": done / el, "unit": "frame/s", "cores": 1, "kind": "port",
               "sample": "%d v2 capture frames in %.1f s: fp64 numpy restatement of FrameDataRead_xzr.m "
                         "(record parse + DDC decode + DBF), BLAS limited to 1 thread" % (done, el)}
    if rank == 0:
        unit_bytes = nb + NB * args.P * args.R * 8                 # records read + beams written
        per_frame_s = gpu_ms / 1e3 / (args.steps * B)
        ach = unit_bytes / per_frame_s / 1e9
        print(json.dumps({
            "metric": "frames/sec (v2 capture frame: 332 PRT x 3404 samples x 16 channels -> 13 DBF beams) "
                      "through the record codec + DBF",
            "value": round(world * B * args.steps / elapsed, 1), "unit": "frame/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int16 in, f32",
            "data": "synthetic PRT records (oracle/ingest_ref.prt_record format, seeded int16 I/Q)",
            "config": {"workload": "ingest: %d frames per GPU per step, records resident in HBM" % B,
                       "payload": "mixed PRTs: DDC / ADC / type 3 (no decode case)" if args.ingest_mix else "DDC (type 1)",
                       "prt": args.P, "samples": args.R, "channels": 16, "beams": NB,
                       "parallelism": "frame-sharded x%d, no collective" % world},
            "roofline": {"bound": "hbm", "kernel": "ingest_decode_kernel", "achieved": round(ach, 1),
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 4),
                         "traffic": None, "alg_bytes_per_unit": unit_bytes,
                         "avg_launch_us": round(per_frame_s * 1e6, 2),
                         "note": "per-frame device time from events around the frame launches "
                                 "(check + decode kernels)"},
            "cpu_baseline": cpu}), flush=True)
    ing.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _timed(args, world, dev, dist, stream, step):
    """W warmup steps, then K timed steps between barrier + synchronize; (wall s, event ms)."""
    import torch
    warm(step, args, dev)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    return time.perf_counter() - t0, ev0.elapsed_time(ev1)


def bench_prefilter(args, world, rank, local, dev, dist):
    """--config prefilter: CPIs/s through rsp_prefilter_dev (fun_iSTC.m gain + fun_Process_MTI.m
    lag-30 difference in one pass) on c3-shaped echoes (128 x 4096 complex64, 1024 CPIs per GPU),
    resident in HBM; each rank filters its own CPIs (no collective)."""
    import numpy as np
    import torch
    from rsp import prefilter, shard
    B, P, R = args.batch, args.P, args.R
    lo, _ = shard.weak_shard(B, rank)
    g = torch.Generator(device=dev)
    g.manual_seed(5000 + lo)
    x = torch.randn((B, P, R), dtype=torch.complex64, generator=g, device=dev)
    out = torch.empty_like(x)
    pf = prefilter.Prefilter(local)
    stc = np.linspace(-30.0, 0.0, 1025)
    _, gain = prefilter.istc_gain(stc, R)
    d_gain = torch.from_numpy(gain).to(dev)
    stream = torch.cuda.current_stream(dev)
    import ctypes as C

    def step():
        rc = pf.lib.rsp_prefilter_dev(pf.ctx, x.data_ptr(), out.data_ptr(), P, R, B, d_gain.data_ptr(), 30,
                                      C.c_void_p(stream.cuda_stream))
        assert rc == 0

    elapsed, gpu_ms = _timed(args, world, dev, dist, stream, step)
    if world > 1:
        elapsed = shard.max_over_ranks(elapsed, dist, device=dev)
    cpu = None
    if rank == 0 and args.cpu_seconds > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import prefilter_ref
        hx = x[:4].cpu().numpy().astype(np.complex128)
        done, t1 = 0, time.perf_counter()
        while time.perf_counter() - t1 < args.cpu_seconds or done == 0:
            prefilter_ref.fun_iSTC(prefilter_ref.fun_Process_MTI(hx[done % 4]), stc)
            done += 1
        el = time.perf_counter() - t1
        cpu = {"value": done / el, "unit": "CPI/s", "cores": 1, "kind": "port",
               "sample": "%d CPIs in %.1f s: fp64 numpy restatement (row loops as fun_Process_MTI.m / "
                         "fun_iSTC.m), one thread" % (done, el)}
    if rank == 0:
        unit_bytes = 2 * P * R * 8                                   # echo read once + written once
        pmc = pmc_traffic("prefilter")
        traffic = pmc["kernels"].get("mti_chain_kernel", {}).get("hbm_bytes_per_launch") if pmc else None
        per_launch_s = gpu_ms / 1e3 / args.steps
        ach = unit_bytes * B / per_launch_s / 1e9
        print(json.dumps({
            "metric": "CPIs/sec (4096 range x 128 pulse) through the echo pre-filters (iSTC gain + MTI lag 30)",
            "value": round(world * B * args.steps / elapsed, 1), "unit": "CPI/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "c64 (f32)",
            "data": "synthetic echo (torch.randn complex64, seeded), 1025-point stc ramp",
            "config": {"workload": "prefilter: %d CPIs per GPU per step, echo resident in HBM" % B,
                       "pulses": P, "range": R, "mti_lag": 30,
                       "parallelism": "CPI-sharded x%d, no collective" % world},
            "roofline": {"bound": "hbm", "kernel": "mti_chain_kernel<true>", "achieved": round(ach, 1),
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 4),
                         "traffic": traffic, "traffic_source": "profiles/pmc_prefilter.json (bytes per launch)", "alg_bytes_per_unit": unit_bytes,
                         "avg_launch_us": round(per_launch_s * 1e6, 2),
                         "note": "one launch per step over the whole batch; events around the launches"},
            "cpu_baseline": cpu}), flush=True)
    pf.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def bench_measure(args, world, rank, local, dev, dist):
    """--config measure: CPIs/s through rsp_motion_measure_dev (motionParaMeasure.m:1-88) on
    DMX long-part planes (V = 2048 Doppler rows x R = 512 range bins, the shape
    DMX_SignalProcessing_main_xzr.m:489-494 measures), sum / diff / flag planes resident in
    HBM; ~0.1 % of cells flagged (about 1000 hits per CPI), extraDots 2, interpolation 8 / 4
    (the reference's :256-258 values).  Each rank measures its own CPIs (no collective)."""
    import numpy as np
    import torch
    from rsp import measure, shard
    B, V, R = args.batch, args.P, args.R
    lo, _ = shard.weak_shard(B, rank)
    g = torch.Generator(device=dev)
    g.manual_seed(4000 + lo)
    s = torch.rand((B, V, R), generator=g, device=dev) * 2 + 0.1
    d = torch.randn((B, V, R), generator=g, device=dev) * 0.5
    M0 = 6
    f = (torch.rand((B, V, R), generator=g, device=dev) < 1e-3).to(torch.uint8)
    f[:, :M0 + 1, :] = 0                             # executeCFAR never flags the zeroed rows
    f[:, V - M0:, :] = 0
    meas = measure.Measure(local)
    kv = measure.angle_KvalueGen(1)
    p = meas.params(2, 5.996, 8, 0.2, 4, kv[4, 3], 3, 5.0, 0.0, 0.0, M0)
    r_scale = np.arange(R) * 5.996
    v_scale = -(np.arange(V) - V / 2) * 0.2
    max_hits = 4096
    stream = torch.cuda.current_stream(dev)
    est, cells, count = meas.measure_dev(s, d, f, p, r_scale, v_scale, max_hits=max_hits)
    torch.cuda.synchronize(dev)
    hits = count[:, 0].double().mean().item()
    assert int(count[:, 0].max()) <= max_hits and int(count[:, 1].sum()) == 0
    rs = torch.as_tensor(r_scale, device=dev)
    vs = torch.as_tensor(v_scale, device=dev)

    import ctypes as C

    def step():
        rc = meas.lib.rsp_motion_measure_dev(meas.ctx, s.data_ptr(), d.data_ptr(), f.data_ptr(), V, R, B,
                                             C.byref(p), rs.data_ptr(), vs.data_ptr(), max_hits, est.data_ptr(),
                                             cells.data_ptr(), count.data_ptr(), C.c_void_p(stream.cuda_stream))
        assert rc == 0

    warm(step, args, dev)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1)
    if world > 1:
        elapsed = shard.max_over_ranks(elapsed, dist, device=dev)
    cpu = None
    if rank == 0 and args.cpu_seconds > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import measure_ref
        hs, hd, hf = s[0].double().cpu().numpy(), d[0].double().cpu().numpy(), f[0].cpu().numpy()
        done, nh, t1 = 0, 0, time.perf_counter()
        while time.perf_counter() - t1 < args.cpu_seconds or done == 0:
            re, _, _, _ = measure_ref.motion_para_measure(hs, hd, hf, 2, r_scale, 5.996, 8, v_scale, 0.2, 4,
                                                          kv[4, 3], 3, 5.0, 0.0, 0.0, M0)
            done += 1
            nh += len(re)
        el = time.perf_counter() - t1
        cpu = {"value": done / el, "unit": "CPI/s", "cores": 1, "kind": "port",
               "sample": "%d CPI(s) (%d hits) in %.1f s: fp64 Python restatement of motionParaMeasure.m, "
                         "one thread" % (done, nh, el)}
    if rank == 0:
        # compulsory bytes per CPI: the flag plane, per hit 2 x (2e+1) sum cells + sum/diff at the
        # hit + rScale/vScale entries read, 3 estimates + 2 cells written
        unit_bytes = V * R + hits * (2 * 5 * 4 + 8 + 16 + 24 + 8)
        pmc = pmc_traffic("measure")
        traffic = sum(pmc["kernels"].get(k, {}).get("hbm_bytes_per_launch", 0)
                      for k in ("hits_kernel", "measure_kernel")) if pmc else None
        per_cpi_s = gpu_ms / 1e3 / (args.steps * B)
        ach = unit_bytes / per_cpi_s / 1e9
        print(json.dumps({
            "metric": "CPIs/sec (2048 Doppler x 512 range DMX long part, ~0.1% cells flagged) through "
                      "motionParaMeasure (range/velocity spline refinement + elevation per CFAR hit)",
            "value": round(world * B * args.steps / elapsed, 1), "unit": "CPI/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32 in, f64",
            "data": "synthetic planes (uniform sum, normal diff, Bernoulli(1e-3) flags, torch.Generator seeded)",
            "config": {"workload": "measure: %d CPIs per GPU per step, planes resident in HBM" % B,
                       "doppler": V, "range": R, "hits_per_cpi": round(hits, 1), "extra_dots": 2,
                       "parallelism": "CPI-sharded x%d, no collective" % world},
            "roofline": {"bound": "hbm", "kernel": "hits_kernel + measure_kernel", "achieved": round(ach, 1),
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 4),
                         "traffic": traffic, "traffic_source": "profiles/pmc_measure.json (both launches of a step)", "alg_bytes_per_unit": round(unit_bytes),
                         "avg_launch_us": round(gpu_ms * 1e3 / args.steps, 2),
                         "note": "one hits_kernel + one measure_kernel launch per step cover the whole batch; events around both"},
            "cpu_baseline": cpu}), flush=True)
    meas.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv):
    """`bench.py --gpus N` started without a launcher (no WORLD_SIZE in the environment): start
    N ranks of this script as child processes, one per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE =
    N, rendezvous on 127.0.0.1), before this process touches any GPU.  Rank 0's JSON line is
    checked (n_gpus == N) and printed as this process's one line; the exit status is non-zero
    when any rank fails, the ranks outlive --launch-timeout, or the line is missing or wrong.
    The stream each rank processes is its contiguous shard of the frame loop of
    MTD/main_produce_dataset_win_xzr_v2.m:70-166 (rank_plan); no data crosses ranks."""
    import subprocess
    import threading
    n = args.gpus
    port = _free_port()
    procs, lines = [], []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno(), text=True))

    def drain():
        for line in procs[0].stdout:
            lines.append(line)
    reader = threading.Thread(target=drain, daemon=True)
    reader.start()
    t0, failed = time.time(), None
    while any(p.poll() is None for p in procs):
        bad = [r for r, p in enumerate(procs) if p.poll() not in (None, 0)]
        if bad:
            failed = "rank %d exited with status %d" % (bad[0], procs[bad[0]].returncode)
            break
        if time.time() - t0 > args.launch_timeout:
            failed = "ranks still running after %.0f s" % args.launch_timeout
            break
        time.sleep(0.2)
    if failed:
        for p in procs:              # the exact child processes this launcher started
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
    reader.join(timeout=30)
    rcs = [p.wait() for p in procs]
    if failed is None and any(rcs):
        r = next(i for i, c in enumerate(rcs) if c)
        failed = "rank %d exited with status %d" % (r, rcs[r])
    out = None
    for line in reversed(lines):
        if line.lstrip().startswith("{"):
            out = json.loads(line)
            break
    if failed is None and out is None:
        failed = "rank 0 printed no JSON line"
    if failed is None and out.get("n_gpus") != n:
        failed = "rank 0 reported n_gpus=%s, expected %d" % (out.get("n_gpus"), n)
    if failed:
        print("bench.py --gpus %d: %s" % (n, failed), file=sys.stderr, flush=True)
        return 1
    out["launcher"] = "bench.py --gpus %d: %d child processes, one per GPU (RANK = LOCAL_RANK = r)" % (n, n)
    print(json.dumps(out), flush=True)
    return 0


def rank_plan(args, rank):
    """The contiguous shard of the unit stream one rank processes (weak scaling):
    CPIs [lo, hi), or in window mode frame pairs [lo, hi) plus the look-ahead (halo) frame hi,
    which the next rank owns; the synthetic echo seed follows the first frame or CPI, so the
    data of a shard does not depend on the number of ranks."""
    from rsp import shard
    cfg_id = int(args.config[1:]) if args.config[1:].isdigit() else 0
    lo, hi = shard.weak_shard(args.batch, rank)
    if args.win:
        flo, fhi = shard.window_frames(lo, hi)
        return {"rank": rank, "frame_pairs": [lo, hi], "frames": [flo, fhi], "halo_frame": fhi - 1,
                "windows": [lo * args.win, hi * args.win], "seed": 1000 + cfg_id + flo}
    return {"rank": rank, "cpis": [lo, hi], "seed": 1000 + cfg_id + lo}


def warm(step, args, dev):
    """The untimed warmup: args.warmup steps, or (None) steps until WARMUP_S seconds of device
    work have run (at least 3); args.warmup is set to the count used (the JSON reports it)."""
    import torch
    if args.warmup is not None:
        for _ in range(args.warmup):
            step()
        return
    n, t0 = 0, time.perf_counter()
    while n < 3 or time.perf_counter() - t0 < WARMUP_S:
        step()
        n += 1
        torch.cuda.synchronize(dev)
    args.warmup = n


def device_identity(local, dry=False, force=-1):
    """What identifies the GPU this rank drives: the local index, HIP/CUDA_VISIBLE_DEVICES, and
    from the device properties the UUID and the PCI domain/bus/device (the duplicate-device guard
    compares these).  --dry-run: a fake identity (all ranks alike under --force-device)."""
    vis = os.environ.get("HIP_VISIBLE_DEVICES", os.environ.get("CUDA_VISIBLE_DEVICES"))
    if dry:
        return {"local": local, "visible": vis, "uuid": "dry-run-%d" % (force if force >= 0 else local),
                "pci": None, "name": "none (dry run)"}
    import torch
    pr = torch.cuda.get_device_properties(local)
    pci = [getattr(pr, k, None) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id")]
    uuid = getattr(pr, "uuid", None)
    return {"local": local, "visible": vis, "uuid": str(uuid) if uuid is not None else None,
            "pci": ("%04x:%02x:%02x" % tuple(pci)) if all(v is not None for v in pci) else None,
            "name": getattr(pr, "gcnArchName", None) or pr.name}


def device_key(d):
    """One GPU's identity: its UUID, else its PCI address, else (visible devices, local index)."""
    if d.get("uuid") is not None:
        return "uuid:" + str(d["uuid"])
    if d.get("pci") is not None:
        return "pci:" + str(d["pci"])
    return "local:%s/%s" % (d.get("visible"), d.get("local"))


def duplicate_devices(idents):
    """Pairs of ranks whose identities name one physical GPU (same UUID, or same PCI address)."""
    dup = []
    for i in range(len(idents)):
        for j in range(i + 1, len(idents)):
            a, b = idents[i], idents[j]
            if any(a.get(k) is not None and a.get(k) == b.get(k) for k in ("uuid", "pci")) or \
                    device_key(a) == device_key(b):
                dup.append((i, j))
    return dup


def check_devices(args, world, rank, local, dist):
    """Gather every rank's device identity over gloo and refuse to run when two ranks drive
    one GPU without --share-device: n_gpus must count distinct GPUs.  Returns the identities."""
    ident = device_identity(local, dry=args.dry_run, force=args.force_device)
    idents = [ident]
    if world > 1:
        idents = [None] * world
        dist.all_gather_object(idents, ident)
    dup = duplicate_devices(idents)
    if dup and not args.share_device:
        i, j = dup[0]
        raise SystemExit("bench.py: ranks %d and %d drive the same GPU (%s); %d ranks would not be %d GPUs "
                         "(use --share-device for a one-GPU rehearsal)" % (
                             i, j, idents[i].get("uuid") or idents[i].get("pci"), world, world))
    return idents


def dry_run(args, world, rank, dist):
    """--dry-run: the multi-rank path without a GPU -- gloo rendezvous, each rank's shard plan,
    a stub step (sleep), barrier + max-over-ranks timing, the per-rank step times and the JSON
    line, so the launcher, sharding and halo are testable on CPU (tests/test_bench_launch.py)."""
    from rsp import shard
    plan = rank_plan(args, rank)
    if rank == args.dry_run_fail_rank:
        raise SystemExit("dry run: rank %d fails on request" % rank)
    plan["device"] = check_devices(args, world, rank, rank, dist)[rank]

    def barrier():
        if world > 1:
            dist.barrier()
    args.warmup = 3 if args.warmup is None else args.warmup
    for _ in range(args.warmup):
        time.sleep(0.001)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.001 * (1 + rank))
    barrier()
    elapsed = time.perf_counter() - t0
    per_rank = shard.gather_over_ranks(elapsed, dist if world > 1 else None)
    plans = [None] * world
    if world > 1:
        dist.all_gather_object(plans, plan)
    else:
        plans = [plan]
    if rank == 0:
        units = args.batch * (args.win or 1)
        print(json.dumps({
            "metric": "dry run (no GPU): launcher, shard plan and halo only", "value": round(world * units * args.steps / max(per_rank), 1),
            "unit": "window/s" if args.win else "CPI/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(max(per_rank) / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dry_run": True, "config": {"workload": args.config, "batch_per_gpu": args.batch},
            "per_rank_ms_per_step": [round(e / args.steps * 1e3, 4) for e in per_rank], "shards": plans,
            "collectives": dist.get_backend() if world > 1 else None,
            "distinct_devices": len({device_key(p["device"]) for p in plans})}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    args = parse()
    if args.warmup is not None:
        args.warmup = max(args.warmup, 1)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, args.gpus), file=sys.stderr, flush=True)
        sys.exit(2)
    import torch
    import torch.distributed as dist
    if world > 1:
        # gloo (host) for the timing barrier and the per-rank gathers: the data path exchanges
        # nothing between GPUs (north_star: frames are independent), so no RCCL communicator
        # is created at all
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend="gloo")
    if args.dry_run:
        return dry_run(args, world, rank, dist)
    from rsp import presets, shard, synth
    from rsp.engine import Engine
    if args.share_device:
        local = 0
    elif args.force_device >= 0:
        local = args.force_device
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    devices = check_devices(args, world, rank, local, dist)
    args.device_identity = devices[rank]
    if args.config == "ingest":
        return bench_ingest(args, world, rank, local, dev, dist)
    if args.config == "measure":
        return bench_measure(args, world, rank, local, dev, dist)
    if args.config == "prefilter":
        return bench_prefilter(args, world, rank, local, dev, dist)

    spec = presets.make(args.preset, args.P, args.R)
    cfar = None if args.no_cfar else presets.default_cfar(spec)
    eng = Engine(spec, device=local, chunk=args.chunk, streams=args.streams)
    if args.prefilter:
        import numpy as np
        from rsp.prefilter import istc_gain
        _, gain = istc_gain(np.linspace(-30.0, 0.0, 1025), spec.R)
        eng.set_prefilter(gain=gain, mti_lag=30)
    B, P, R, win = args.batch, spec.P, spec.R_out, args.win
    units = B * win if win else B                   # CPIs (windows) per GPU per step
    # contiguous shard of the stream per rank (weak scaling): seed = 1000 + config id + first
    # unit index; window mode also holds the look-ahead frame of its last pair (halo)
    plan = rank_plan(args, rank)
    plan["device"] = args.device_identity
    if win:
        flo, fhi = plan["frames"]
        echo = synth.echo_torch(spec, fhi - flo, seed=plan["seed"], device=dev, half=args.half)
        echo = echo.reshape((1, fhi - flo) + tuple(echo.shape[1:]))
        oshape = (1, B, win, P, R)
    else:
        echo = synth.echo_torch(spec, B, seed=plan["seed"], device=dev, half=args.half)
        oshape = (B, P, R)
    rdm = torch.empty(oshape, dtype=torch.float32, device=dev)
    flag = torch.empty(oshape, dtype=torch.uint8, device=dev) if cfar else None
    stream = torch.cuda.current_stream(dev)

    def step():
        if win:
            eng.window_dev(echo, win, rdm=rdm, flag=flag, cfar=cfar, stream=stream)
        else:
            eng.run_dev(echo, rdm=rdm, flag=flag, cfar=cfar, stream=stream)

    def barrier():
        if world > 1:
            dist.barrier()

    warm(step, args, dev)
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1)
    per_rank = shard.gather_over_ranks(elapsed, dist if world > 1 else None, device=dev)
    elapsed = max(per_rank)
    plans = [plan]
    if world > 1:
        plans = [None] * world
        dist.all_gather_object(plans, plan)

    # Per-kernel device times, measured separately from the throughput: a short pass on ONE
    # chunk pipeline (rsp_set_streams(1)) with every launch bracketed by HIP events on the
    # stream it runs on, so no two kernels overlap and each kernel's time per step is its own
    # (in the timed region the two pipelines overlap PC of one chunk with MTD of the other).
    kernels = launches = None
    if not args.no_profile and args.lane_steps > 0:
        eng.set_streams(1)
        eng.profile(True, every=1)
        for _ in range(args.lane_steps):
            step()
        torch.cuda.synchronize(dev)
        prof = eng.profile_read()
        eng.profile(False)
        eng.set_streams(args.streams)    # back to what the timed region used (0 = library default)
        kernels = {k: (ms / args.lane_steps, n // args.lane_steps) for k, (ms, n) in prof.items()}

    if rank == 0:
        esz = 4 if args.half else 8
        in_b = P * spec.R * esz / (win if win else 1)   # window mode: each frame feeds `win` windows
        rdm_b, flag_b = P * R * 4, (P * R if cfar else 0)
        cpi_bytes = int(in_b + rdm_b + flag_b)          # SURVEY.md §8d algorithmic bytes per CPI / window
        total_units = world * units * args.steps
        value = total_units / elapsed
        per_gpu_units_s = units * args.steps / (gpu_ms / 1e3)
        chain_gbps = per_gpu_units_s * cpi_bytes / 1e9
        tag = "%s_P%d_R%d%s%s%s" % (args.preset, args.P, args.R, "" if cfar else "_nocfar",
                                    "_f16" if args.half else "", "_win%d" % win if win else "")
        pmc = pmc_traffic(tag)
        # Headline: the whole chain (SURVEY.md §8d algorithmic bytes per CPI x CPIs/s over one
        # step, the dominant cost being two overlapping kernels); traffic = every kernel's
        # PMC HBM-side bytes of a profiled run / the CPIs it processed.
        pipes = args.streams or (1 if win else 2)      # the library default: rsp.h rsp_set_streams
        roof = {"bound": "hbm", "kernel": "chain (PC + MTD/Doppler-CFAR%s, %d pipeline%s)" % (
                    " + range CFAR" if cfar else "", pipes, "" if pipes == 1 else "s"),
                "achieved": round(chain_gbps, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(chain_gbps / HBM_PEAK_GBPS, 4), "traffic": None, "alg_bytes_per_unit": cpi_bytes,
                "units_per_launch": units, "avg_launch_us": round(gpu_ms * 1e3 / args.steps, 1),
                "note": "one step = one launch sequence over the batch; achieved = units/s (device events "
                        "around the timed steps) x alg bytes per unit"}
        ceil = hbm_ceiling()
        if ceil:
            roof["ceiling"] = {"copy_GBps": ceil["copy_GBps"], "read_GBps": ceil["read_GBps"],
                               "write_GBps": ceil["write_GBps"], "source": "profiles/hbm_ceiling.json"}
        if pmc and pmc.get("bytes_per_unit"):
            # per launch like `achieved` (one launch sequence = one step of `units` CPIs/windows)
            roof["traffic"] = int(pmc["bytes_per_unit"] * units)
            roof["traffic_per"] = "step (units_per_launch units), all kernels, from a profiled run's bytes per unit"
            roof["traffic_per_unit"] = int(pmc["bytes_per_unit"])
            roof["traffic_ratio"] = round(pmc["bytes_per_unit"] / cpi_bytes, 3)
            roof["traffic_source"] = "profiles/pmc_%s.json" % tag
            if ceil:
                # the counted L2<->fabric bytes per second of this run against the measured copy
                # ceiling (Infinity-Cache hits are counted too, so this can exceed 1 in principle)
                counted_gbps = pmc["bytes_per_unit"] * per_gpu_units_s / 1e9
                roof["counted_GBps"] = round(counted_gbps, 1)
                roof["ceiling_frac"] = round(counted_gbps / ceil["copy_GBps"], 4)
        if kernels:
            # each kernel's own compulsory bytes per launch: PC reads the echo and writes the
            # pulse-compressed rows; MTD reads them and writes the RDM and the flag plane
            npc = kernels.get("pc_kernel", (0, 0))[1]
            pc_rows = (B + npc) * P * spec.beams if win else B * P * spec.beams
            # window mode: the `win` windows of a frame pair read overlapping PC rows, and each
            # row is compulsory once -- P rows per frame pair, P*R*8/win bytes per window
            per_kernel_bytes = {
                "pc_kernel": (pc_rows / max(npc, 1)) * (spec.R * esz + R * 8),
                "mtd_kernel": units / max(kernels.get("mtd_kernel", (0, 1))[1], 1)
                * (P * R * 8 * spec.beams / (win or 1) + spec.V * R * 4 + (spec.V * R if cfar else 0)),
            }
            ks = {}
            for name, (ms, n) in kernels.items():
                avg_us = ms * 1e3 / max(n, 1)
                k = {"avg_us": round(avg_us, 2), "launches_per_step": n, "ms_per_step": round(ms, 3)}
                if name in per_kernel_bytes:
                    # `frac`: the kernel's own compulsory I/O (PC: echo in + scratch out; MTD:
                    # scratch in + RDM / flags out) per launch / its time / peak
                    ab = per_kernel_bytes[name]
                    k["io_bytes_per_launch"] = int(ab)
                    k["achieved"] = round(ab / (avg_us * 1e3), 1)
                    k["frac"] = round(ab / (avg_us * 1e3) / HBM_PEAK_GBPS, 4)
                    k["frac_basis"] = "own I/O (incl. the PC->MTD scratch)"
                    # `frac_alg` (the contract's definition): the chain's algorithmic
                    # bytes per unit x the units one launch processes / the launch's average time /
                    # peak -- for the two passes that carry the compulsory bytes (the range stage
                    # reads a few cells per Doppler hit and moves none of them)
                    upl = units / max(n, 1)
                    k["units_per_launch"] = round(upl, 3)
                    k["alg_bytes_per_launch"] = int(upl * cpi_bytes)
                    k["frac_alg"] = round(upl * cpi_bytes / (avg_us * 1e3) / HBM_PEAK_GBPS, 4)
                if pmc and name in pmc.get("kernels", {}):
                    pk = pmc["kernels"][name]
                    k["hbm_bytes_per_launch"] = pk.get("hbm_bytes_per_launch")
                    if pk.get("valu_frac") is not None:
                        # SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES of the profiled run (per-wave share of
                        # cycles issuing VALU; BASELINE.md's VALU fraction beside the HBM fraction)
                        k["valu_frac"] = pk["valu_frac"]
                        k["wait_frac"] = pk.get("wait_frac")
                ks[name] = k
            roof["kernels"] = ks
            roof["kernels_source"] = ("single-pipeline pass after the timed region (%d steps, every launch "
                                      "bracketed by HIP events on its stream)" % args.lane_steps)
            roof["kernel_sum_ms_per_step"] = round(sum(ms for ms, _ in kernels.values()), 3)
            dom = max(kernels, key=lambda q: kernels[q][0])
            roof["dominant_kernel"] = dom
            roof["dominant_ms_per_step"] = round(kernels[dom][0], 3)
            roof["dominant_frac_alg"] = ks[dom].get("frac_alg")
            if "valu_frac" in ks.get(dom, {}):
                roof["valu_frac"] = ks[dom]["valu_frac"]
                roof["valu_frac_source"] = "profiles/pmc_%s.json (dominant kernel, SQ counters)" % tag
        achieved = chain_gbps
        host = host_path(eng, echo, cfar, args) if (args.host_path and world == 1 and not win) else None
        # rank 0 only (the other ranks wait at the closing barrier); window mode: the reference
        # runs fun_MTD_produce per window, so its rate is CPIs/s
        cpu = cpu_baseline(spec, cfar, args.cpu_seconds, unit="window/s" if win else "CPI/s")
        mode = "%s: %d pulses x %d range bins, %s, preset %s, PC->MTD->0v%s" % (
            args.config, P, spec.R,
            ("%d frame pairs x %d windows per GPU per step (sliding window, PC shared by windows)" % (B, win))
            if win else "%d CPIs per GPU per step" % B, args.preset,
            "->2D CA-CFAR (executeCFAR per PC segment)" if cfar else "")
        if args.config == "c3" and not win and P == 128 and spec.R == 4096 and cfar:
            metric, unit = METRIC, "CPI/s"
        elif win:
            metric, unit = "windows/sec (%d range x %d pulse, %d windows per frame pair) through PC->MTD%s" % (
                spec.R, P, win, "->CFAR" if cfar else ""), "window/s"
        else:
            metric, unit = "CPIs/sec (%d range x %d pulse) through PC->MTD%s" % (
                spec.R, P, "->CFAR" if cfar else ""), "CPI/s"
        out = {
            "metric": metric,
            "value": round(value, 1),
            "unit": unit,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32" if not args.half else "f32 (fp16 I/Q storage)",
            "data": "synthetic (SURVEY.md §8d echo: 3 targets + zero-Doppler clutter + CN(0,1) noise, GPU-drawn)",
            "config": {"workload": mode, "pulses": P, "range_bins": spec.R, "batch_per_gpu": B,
                       "windows_per_pair": win or None, "preset": args.preset,
                       "input": "c32f16" if args.half else "c64",
                       "prefilter": "fused iSTC + MTI(30)" if args.prefilter else None,
                       "parallelism": ("%d ranks sharing device 0 (launcher rehearsal, not a scaling result)" % world
                                       if args.share_device else "frame-sharded x%d, no data-path collective "
                                       "(gloo host barrier/gathers only)" % world)},
            "distinct_devices": len({device_key(d["device"]) for d in plans}),
            "collectives": dist.get_backend() if world > 1 else None,
            "per_rank_ms_per_step": [round(e / args.steps * 1e3, 4) for e in per_rank],
            "shards": plans,
            "hbm_GBps_per_gpu": round(achieved, 1),
            "gpu_event_ms_per_step": round(gpu_ms / args.steps, 4),
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if host is not None:
            out["host_path"] = host
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
