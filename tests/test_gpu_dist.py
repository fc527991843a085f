"""Multi-rank product path on one GPU: the frame-sharded window stream run by
two ranks, each a separate process driving the HIP engine on cuda:0 over its own shard (its
frame pairs plus the look-ahead halo frame, MTD/main_produce_dataset_win_xzr_v2.m:70-166),
gathered over gloo, equals the single-process product run over the whole stream bit for bit;
and `bench.py --gpus 2` launches its own ranks end to end (--share-device: both ranks on
device 0, gloo collectives -- a rehearsal of the launcher, not a scaling result)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P, R, WIN, PER, WORLD = 64, 2048, 4, 3, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _frames(flo, fhi):
    from rsp import presets, synth
    return synth.echo_numpy(presets.v2(P, R), fhi - flo, seed=2000 + flo)


def _run_windows(frames):
    import torch
    from rsp import presets
    from rsp.engine import Engine
    spec = presets.v2(P, R)
    eng = Engine(spec, device=0)
    cf = presets.default_cfar(spec)
    nf = frames.shape[0] - 1
    d = torch.from_numpy(frames.reshape((1,) + frames.shape)).cuda()
    rdm = torch.empty((1, nf, WIN, P, spec.R_out), dtype=torch.float32, device="cuda")
    flag = torch.empty((1, nf, WIN, P, spec.R_out), dtype=torch.uint8, device="cuda")
    eng.window_dev(d, WIN, rdm=rdm, flag=flag, cfar=cf)
    torch.cuda.synchronize()
    out = rdm.cpu().numpy().reshape(nf * WIN, P, -1), flag.cpu().numpy().reshape(nf * WIN, P, -1)
    eng.close()
    return out


def _rank(rank, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path[:0] = [os.path.join(ROOT, "radar-signal-process_amd")]
    import torch
    import torch.distributed as dist
    from rsp import shard
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    lo, hi = shard.weak_shard(PER, rank)
    flo, fhi = shard.window_frames(lo, hi)
    rdm, flag = _run_windows(_frames(flo, fhi))
    g_rdm = [torch.empty(rdm.shape, dtype=torch.float32) for _ in range(WORLD)]
    g_flag = [torch.empty(flag.shape, dtype=torch.uint8) for _ in range(WORLD)]
    dist.all_gather(g_rdm, torch.from_numpy(rdm))
    dist.all_gather(g_flag, torch.from_numpy(flag))
    if rank == 0:
        q.put((np.concatenate([t.numpy() for t in g_rdm]), np.concatenate([t.numpy() for t in g_flag])))
    dist.barrier()
    dist.destroy_process_group()


def test_window_stream_two_ranks_bit_exact():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got_rdm, got_flag = q.get(timeout=150)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want_rdm, want_flag = _run_windows(_frames(0, WORLD * PER + 1))
    assert got_rdm.shape == (WORLD * PER * WIN, P, R)
    assert np.array_equal(got_rdm, want_rdm)
    assert np.array_equal(got_flag, want_flag)
    assert want_flag.any()


def test_bench_launcher_two_ranks_share_device():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-device",
                        "--config", "c4", "--batch", "2", "--steps", "2", "--warmup", "1", "--cpu-seconds", "0",
                        "--lane-steps", "0", "--launch-timeout", "100"],
                       capture_output=True, text=True, timeout=150, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert out["n_gpus"] == 2 and len(out["per_rank_ms_per_step"]) == 2
    assert [tuple(s["frames"]) for s in out["shards"]] == [(0, 3), (2, 5)]
    assert out["value"] > 0
    assert out["collectives"] == "gloo" and out["distinct_devices"] == 1
    dev = [s["device"] for s in out["shards"]]
    assert dev[0]["local"] == dev[1]["local"] == 0 and (dev[0]["uuid"] or dev[0]["pci"])


def test_bench_refuses_two_ranks_on_one_gpu():
    """Without --share-device, two ranks that land on one GPU (forced here) must not report
    n_gpus = 2: the launch fails, naming the shared device."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--force-device", "0",
                        "--config", "c2", "--batch", "2", "--steps", "1", "--warmup", "1", "--cpu-seconds", "0",
                        "--lane-steps", "0", "--launch-timeout", "100"],
                       capture_output=True, text=True, timeout=150, env=env)
    assert p.returncode != 0
    assert "drive the same GPU" in p.stderr
    assert not [l for l in p.stdout.splitlines() if l.startswith("{")]
