#!/usr/bin/env python3
"""Benchmark: CPIs/s through PC -> MTD -> 0-v -> 2-D CA-CFAR (BASELINE.json metric).

Workload (config c3 of BASELINE.json): 128 pulses x 4096 range bins, complex fp32 echo,
batch 1024 CPIs per GPU, `v2` preset (fun_MTD_produce's 3-segment pulse compression,
kaiser-8 MTD with fftshift, 0-v /150) followed by main_cfar's /20 0-v and executeCFAR per
PC segment (ref 5, guard 7, T 5, GO, range CFAR on).  A step is one pass of the chain
over the batch, inputs resident in HBM.  Synthetic echoes (SURVEY.md §8d recipe, noise
drawn on the GPU).

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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3, help=">= 1 (the first warmup step counts launches)")
    ap.add_argument("--preset", default="v2", choices=["v2", "dmx"])
    ap.add_argument("--P", type=int, default=128)
    ap.add_argument("--R", type=int, default=4096)
    ap.add_argument("--batch", type=int, default=1024, help="CPIs per GPU per step")
    ap.add_argument("--no-cfar", action="store_true", help="PC + MTD only (config c2)")
    ap.add_argument("--half", action="store_true", help="fp16 I/Q input (config c5 style)")
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--streams", type=int, default=0, help="chunk pipelines (0 = library default)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 = skip)")
    ap.add_argument("--no-profile", action="store_true", help="no per-kernel HIP events in the timed region")
    ap.add_argument("--profile-every", type=int, default=8, help="bracket every N-th kernel launch with events")
    return ap.parse_args()


def cpu_baseline(spec, cfar, seconds):
    """fp64 C restatement (oracle/rsp_oracle.c, OpenMP over CPIs) on a bounded sample."""
    if seconds <= 0:
        return None
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import coracle
    from rsp import synth
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    threads = min(threads, 16)
    pool_n = max(threads, 16)
    echo = synth.echo_numpy(spec, pool_n, seed=1003).astype(np.complex128)
    pre = coracle.preset(spec.name, spec.P, spec.R)
    c = cfar.as_dict() if cfar is not None else None
    if c is not None:
        c["zero_v_div"] = cfar.zero_v_div
    done, t0 = 0, time.perf_counter()
    while True:
        rdm = coracle.pc_mtd(echo, pre, nthreads=threads)
        if c is not None:
            coracle.cfar(rdm, c, cfar.segments, nthreads=threads)
        done += pool_n
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": done / el, "unit": "CPI/s", "cores": threads, "kind": "port",
            "sample": "%d CPIs (%d x %d, %s preset%s) in %.1f s: a pool of %d distinct synthetic CPIs "
                      "cycled; fp64 C restatement of the MATLAB chain (MATLAB itself is not available)"
                      % (done, spec.P, spec.R, spec.name, " + CFAR" if c else "", el, pool_n)}


def pmc_traffic(tag):
    """HBM bytes per launch from a committed rocprofv3 PMC summary, if one exists."""
    p = os.path.join(ROOT, "profiles", "pmc_%s.json" % tag)
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)


def main():
    args = parse()
    args.warmup = max(args.warmup, 1)
    import torch
    import torch.distributed as dist
    from rsp import presets, shard, synth
    from rsp.engine import Engine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    spec = presets.make(args.preset, args.P, args.R)
    cfar = None if args.no_cfar else presets.default_cfar(spec)
    eng = Engine(spec, device=local, chunk=args.chunk, streams=args.streams)
    B, P, R = args.batch, spec.P, spec.R_out
    # contiguous shard of the CPI stream per rank: seed = 1000 + config id 3 + first CPI index
    lo, _ = shard.weak_shard(B, rank)
    echo = synth.echo_torch(spec, B, seed=1003 + lo, device=dev, half=args.half)
    rdm = torch.empty((B, P, R), dtype=torch.float32, device=dev)
    flag = torch.empty((B, P, R), dtype=torch.uint8, device=dev) if cfar else None
    stream = torch.cuda.current_stream(dev)

    def step():
        eng.run_dev(echo, rdm=rdm, flag=flag, cfar=cfar, stream=stream)

    def barrier():
        if world > 1:
            dist.barrier()

    launches_per_step = None
    for i in range(args.warmup):
        if i == 0 and not args.no_profile:
            eng.profile(True, every=1)      # count launches per step (chunks) once, untimed
        step()
        if i == 0 and not args.no_profile:
            launches_per_step = {k: n for k, (_, n) in eng.profile_read().items()}
            eng.profile(False)
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # per-kernel device time, live: the library brackets every --profile-every-th launch of the
    # timed steps with HIP events on the stream it is launched on (rsp_profile); read after
    # the timed region.  Sampling keeps the events' own cost out of the measured throughput.
    if not args.no_profile:
        eng.profile(True, every=args.profile_every)
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
    elapsed = shard.max_over_ranks(elapsed, dist if world > 1 else None, device=dev)

    kernels = None
    if not args.no_profile:
        kernels = eng.profile_read()
        eng.profile(False)

    if rank == 0:
        esz = 4 if args.half else 8
        in_b, rdm_b, flag_b = P * spec.R * esz, P * R * 4, (P * R if cfar else 0)
        cpi_bytes = in_b + rdm_b + flag_b              # SURVEY.md §8d algorithmic bytes per CPI
        total_cpis = world * B * args.steps
        value = total_cpis / elapsed
        per_gpu_cpis_s = B * args.steps / (gpu_ms / 1e3)
        chain_gbps = per_gpu_cpis_s * cpi_bytes / 1e9
        tag = "%s_P%d_R%d%s%s" % (args.preset, args.P, args.R, "" if cfar else "_nocfar", "_f16" if args.half else "")
        pmc = pmc_traffic(tag)
        # Dominant kernel (largest device time per step): achieved = §8d bytes per CPI x CPIs per
        # launch / its mean launch duration (HIP events on its launch stream); traffic = HBM-side
        # bytes per launch from the committed PMC summary.
        roof = {"bound": "hbm", "kernel": None, "achieved": None, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": None, "traffic": None, "alg_bytes_per_cpi": cpi_bytes,
                "chain": {"achieved": round(chain_gbps, 1), "frac": round(chain_gbps / HBM_PEAK_GBPS, 4),
                          "note": "whole step: CPIs/s x alg bytes per CPI"}}
        if kernels:
            ks = {}
            for name, (ms, n) in kernels.items():
                avg_us = ms * 1e3 / n
                ks[name] = {"avg_us": round(avg_us, 2), "sampled_launches": n,
                            "launches_per_step": launches_per_step.get(name)}
            dom = max(kernels, key=lambda k: kernels[k][0])
            cpl = B / launches_per_step[dom]           # CPIs per launch (chunk)
            avg_s = kernels[dom][0] / 1e3 / kernels[dom][1]
            ach = cpi_bytes * cpl / avg_s / 1e9
            roof.update({"kernel": dom, "achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBPS, 4),
                         "cpis_per_launch": cpl, "alg_bytes_per_launch": int(cpi_bytes * cpl),
                         "avg_launch_us": round(avg_s * 1e6, 2)})
            if pmc and dom in pmc.get("kernels", {}):
                kp = pmc["kernels"][dom]
                scale = cpl / pmc["cpis_per_launch"] if pmc.get("cpis_per_launch") else 1.0
                roof["traffic"] = int(kp["hbm_bytes_per_launch"] * scale)
                roof["traffic_source"] = "profiles/pmc_%s.json" % tag
            roof["kernels"] = ks
            roof["kernel_sum_ms_per_step"] = round(
                sum(kernels[k][0] / kernels[k][1] * launches_per_step[k] for k in kernels), 3)
        else:
            roof.update({"kernel": "chain", "achieved": round(chain_gbps, 1),
                         "frac": round(chain_gbps / HBM_PEAK_GBPS, 4)})
        achieved = chain_gbps
        cpu = None
        if world == 1:
            cpu = cpu_baseline(spec, cfar, args.cpu_seconds)
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "CPI/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32" if not args.half else "f32 (fp16 I/Q storage)",
            "data": "synthetic (SURVEY.md §8d echo: 3 targets + zero-Doppler clutter + CN(0,1) noise, GPU-drawn)",
            "config": {"workload": "c3: %d pulses x %d range bins, %d CPIs per GPU per step, preset %s, "
                                   "PC->MTD->0v%s" % (P, spec.R, B, args.preset,
                                                      "->2D CA-CFAR (executeCFAR per PC segment)" if cfar else ""),
                       "pulses": P, "range_bins": spec.R, "batch_per_gpu": B, "preset": args.preset,
                       "input": "c32f16" if args.half else "c64",
                       "parallelism": "frame-sharded x%d, no collective" % world},
            "hbm_GBps_per_gpu": round(achieved, 1),
            "gpu_event_ms_per_step": round(gpu_ms / args.steps, 4),
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
