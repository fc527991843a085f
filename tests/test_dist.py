"""Multi-process path on CPU (gloo, world_size 2): shards are disjoint and cover the CPI
stream, each rank's synthetic CPIs equal the corresponding CPIs of a single-process run
(so results do not depend on the number of GPUs), and the timing reduction is a max."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rsp import presets, shard, synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    spec = presets.v2(16, 1024)
    per = 3
    lo, hi = shard.weak_shard(per, rank)
    echo = synth.echo_numpy(spec, hi - lo, seed=1003 + lo)
    # gather every rank's CPIs on every rank
    t = torch.from_numpy(np.ascontiguousarray(echo.view(np.float32)))
    gathered = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(gathered, t)
    elapsed = 1.0 + rank                       # pretend rank r took 1 + r seconds
    mx = shard.max_over_ranks(elapsed, dist)
    lohi = torch.tensor([lo, hi])
    all_lohi = [torch.empty_like(lohi) for _ in range(world)]
    dist.all_gather(all_lohi, lohi)
    if rank == 0:
        full = np.concatenate([g.numpy().view(np.complex64) for g in gathered])
        out.put((full, mx, [tuple(x.tolist()) for x in all_lohi]))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_sharding():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 2
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    full, mx, bounds = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert bounds == [(0, 3), (3, 6)]
    assert mx == 2.0
    single = synth.echo_numpy(presets.v2(16, 1024), 6, seed=1003)
    np.testing.assert_array_equal(full, single)


def test_shard_bounds():
    for total in (0, 1, 7, 1024):
        for world in (1, 2, 3, 8):
            spans = [shard.shard_bounds(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1
    assert shard.window_frames(4, 8) == (4, 9)


def _windows_of(frames, win):
    """Windows of consecutive frame pairs (main_produce_dataset_win_xzr_v2.m:94-139): window i
    of pair n = rows start_i .. start_i + P of [frame n; frame n+1], start_i = round(i*P/win)."""
    nf1, P, R = frames.shape
    starts = [int(np.floor(i * P / win + 0.5)) for i in range(win)]
    out = np.empty((nf1 - 1, win, P, R), frames.dtype)
    for n in range(nf1 - 1):
        pair = np.concatenate([frames[n], frames[n + 1]])
        for i, s in enumerate(starts):
            out[n, i] = pair[s:s + P]
    return out


def _win_worker(rank, world, port, out):
    """One rank of the sliding-window stream (config c4 layout): its frame pairs [lo, hi) and
    the look-ahead frame hi (shard.window_frames), windows sliced locally, fp64 oracle RDMs."""
    import coracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    spec = presets.v2(16, 1024)
    per, win = 2, 4
    lo, hi = shard.weak_shard(per, rank)
    flo, fhi = shard.window_frames(lo, hi)
    frames = synth.echo_numpy(spec, fhi - flo, seed=2000 + flo)
    wins = _windows_of(frames, win).reshape(-1, spec.P, spec.R)
    rdm = coracle.pc_mtd(wins.astype(np.complex128), coracle.preset(spec.name, spec.P, spec.R), nthreads=1)
    t = torch.from_numpy(np.ascontiguousarray(rdm))
    gathered = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(gathered, t)
    if rank == 0:
        out.put(np.concatenate([g.numpy() for g in gathered]))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_window_halo():
    """Window mode sharded over 2 ranks: each rank holds its frames plus the next rank's first
    frame (halo) and no data moves between ranks; the gathered RDMs of all windows equal a
    single-process run over the whole frame stream, bit for bit (fp64 oracle on both sides)."""
    import coracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, per, win = 2, 2, 4
    port = _free_port()
    procs = [ctx.Process(target=_win_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    spec = presets.v2(16, 1024)
    frames = synth.echo_numpy(spec, world * per + 1, seed=2000)
    wins = _windows_of(frames, win).reshape(-1, spec.P, spec.R)
    want = coracle.pc_mtd(wins.astype(np.complex128), coracle.preset(spec.name, spec.P, spec.R), nthreads=1)
    assert got.shape == (world * per * win, spec.V, spec.R_out)
    np.testing.assert_array_equal(got, want)
