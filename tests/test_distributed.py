"""bench.py's multi-GPU contract on CPU (gloo, world_size 2): images shard
across ranks with no data-path collective (disjoint, covering seed blocks),
and the timed region reduces with MAX over ranks."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, batch, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r, w, _ = bench.dist_env()
    seeds = torch.tensor(bench.shard_seeds(batch, r), dtype=torch.int64)
    gathered = [torch.zeros_like(seeds) for _ in range(w)]
    dist.all_gather(gathered, seeds)
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        out.put((torch.cat(gathered).tolist(), float(t.item())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_shards_disjoint_and_max_reduce(world):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    batch = 5
    mp.start_processes(_worker, args=(world, _free_port(), batch, q), nprocs=world, join=True, start_method="spawn")
    seeds, tmax = q.get()
    assert sorted(seeds) == list(range(world * batch))
    assert tmax == float(world)


def test_single_rank_defaults(monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    assert bench.dist_env() == (0, 1, 0)
    assert bench.shard_seeds(4, 0) == [0, 1, 2, 3]
    assert bench.shard_seeds(4, 3) == [12, 13, 14, 15]


def _split_worker(rank, world, port, exe, sample, out):
    """Rank `rank` decodes grid tiles k % world == rank of one image with the
    kernels emulated on the host (emu_check checks its windows against the
    oracle); the ranks' TB counts must add up to the whole image's."""
    import subprocess

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r = subprocess.run([exe, sample, "5", str(world), str(rank)], capture_output=True, text=True, timeout=600)
    ok = r.returncode == 0 and "EMU PARITY OK" in r.stdout
    line = next((l for l in r.stdout.splitlines() if l.startswith("parse: status")), "parse: status 0x0, 0 TBs")
    t = torch.tensor([int(line.split()[3]), 0 if ok else 1], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    if rank == 0:
        out.put(t.tolist())
    dist.barrier()
    dist.destroy_process_group()


def test_tile_split_ranks_compose_the_image():
    """Row e2 through the distributed runtime (gloo, world_size 2): each rank
    decodes its tile subset; no rank fails parity and together they decode
    every TB of the image exactly once (halfmoonbay: 207,654 TBs)."""
    import pathlib
    import subprocess

    root = pathlib.Path(__file__).resolve().parents[1]
    subprocess.run(["make", "-s", "-C", str(root / "heif_amd" / "csrc"), "emu-fast"], check=True, capture_output=True)
    exe = str(root / "heif_amd" / "csrc" / "build" / "emu_fast" / "emu_check")
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.start_processes(_split_worker, args=(2, _free_port(), exe, str(root / "tests/golden/halfmoonbay.heic"), q),
                       nprocs=2, join=True, start_method="spawn")
    tbs, failures = q.get()
    assert failures == 0
    assert tbs == 207654
