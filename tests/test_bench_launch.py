"""bench.py's rank launcher on CPU (--dry-run: gloo rendezvous, stub steps, no GPU and no
oracle): `bench.py --gpus N` started without WORLD_SIZE spawns N ranks itself, each rank owns
a contiguous shard of the unit stream (window mode: its frame pairs plus the look-ahead halo
frame, MTD/main_produce_dataset_win_xzr_v2.m:70-166), and the launcher fails loudly when a
rank fails or the rank count disagrees."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=env)
    lines = [l for l in p.stdout.splitlines() if l.lstrip().startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


@pytest.mark.parametrize("world", [2, 3])
def test_launcher_cpi_shards(world):
    rc, out, err = _run(["--gpus", str(world), "--dry-run", "--steps", "2", "--warmup", "1", "--batch", "5"])
    assert rc == 0, err
    assert out["n_gpus"] == world and out["dry_run"] is True
    assert len(out["per_rank_ms_per_step"]) == world
    assert out["ms_per_step"] == max(out["per_rank_ms_per_step"])
    spans = [tuple(s["cpis"]) for s in out["shards"]]
    assert [s["rank"] for s in out["shards"]] == list(range(world))
    assert spans[0][0] == 0 and all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    assert all(hi - lo == 5 for lo, hi in spans)                     # weak scaling: 5 CPIs per rank
    assert [s["seed"] for s in out["shards"]] == [1003 + lo for lo, _ in spans]
    assert out["launcher"].startswith("bench.py --gpus %d" % world)
    # host-side gloo is the only process group (no RCCL communicator on the path), and every
    # rank records the device it drives
    assert out["collectives"] == "gloo"
    assert [s["device"]["local"] for s in out["shards"]] == list(range(world))
    assert out["distinct_devices"] == world


def test_launcher_window_halo():
    rc, out, err = _run(["--gpus", "2", "--dry-run", "--config", "c4", "--steps", "2", "--warmup", "1",
                         "--batch", "3"])
    assert rc == 0, err
    sh = out["shards"]
    assert [tuple(s["frame_pairs"]) for s in sh] == [(0, 3), (3, 6)]
    # each rank holds its own frames plus the next rank's first frame (the halo)
    assert [tuple(s["frames"]) for s in sh] == [(0, 4), (3, 7)]
    assert sh[0]["halo_frame"] == sh[1]["frame_pairs"][0]
    assert [tuple(s["windows"]) for s in sh] == [(0, 12), (12, 24)]
    assert out["unit"] == "window/s" and out["n_gpus"] == 2


def test_launcher_fails_when_a_rank_fails():
    rc, out, err = _run(["--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1", "--dry-run-fail-rank", "1",
                         "--launch-timeout", "120"])
    assert rc != 0
    assert out is None
    assert "rank 1 exited" in err


def test_world_size_must_match_gpus():
    rc, out, err = _run(["--gpus", "2", "--dry-run", "--steps", "1"], env_extra={"WORLD_SIZE": "1"})
    assert rc == 2 and out is None
    assert "WORLD_SIZE=1 but --gpus 2" in err


def test_duplicate_device_guard():
    """Two ranks that report one physical GPU (here: the dry run's fake identity, all ranks
    on device 0 without --share-device) make the launch fail instead of printing n_gpus = 2."""
    rc, out, err = _run(["--gpus", "2", "--dry-run", "--steps", "1", "--warmup", "1", "--force-device", "0",
                         "--launch-timeout", "120"])
    assert rc != 0 and out is None
    assert "drive the same GPU" in err


def test_duplicate_device_check_unit():
    sys.path.insert(0, ROOT)
    import bench
    a = {"local": 0, "uuid": "GPU-1", "pci": "0000:05:00"}
    b = {"local": 1, "uuid": "GPU-2", "pci": "0000:15:00"}
    assert bench.duplicate_devices([a, b]) == []
    assert bench.duplicate_devices([a, b, dict(a, local=2)]) == [(0, 2)]
    assert bench.duplicate_devices([a, dict(b, uuid=None, pci="0000:05:00")]) == [(0, 1)]
    # neither UUID nor PCI address: the local index (under the same device visibility) decides
    assert bench.duplicate_devices([dict(a, uuid=None, pci=None), dict(b, uuid=None, pci=None)]) == []
    assert bench.duplicate_devices([dict(a, uuid=None, pci=None), dict(a, uuid=None, pci=None)]) == [(0, 1)]
