"""bench.py's multi-GPU contract on CPU (gloo, world_size 2): images shard
across ranks with no data-path collective (disjoint, covering seed blocks),
and the timed region reduces with MAX over ranks."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from conftest import make_emu


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
    make_emu("emu-fast")
    exe = str(root / "heif_amd" / "csrc" / "build" / "emu_fast" / "emu_check")
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.start_processes(_split_worker, args=(2, _free_port(), exe, str(root / "tests/golden/halfmoonbay.heic"), q),
                       nprocs=2, join=True, start_method="spawn")
    tbs, failures = q.get()
    assert failures == 0
    assert tbs == 207654


# ---------------------------------------------------------------- e2 gather
class _Info:
    width, height, tile_width, tile_height, grid_cols, num_tiles, chroma = 1000, 700, 256, 256, 4, 12, 1


def _windows(k, c, info=_Info):
    """Plane-c window of grid tile k (k_gather_tiles' geometry, gather.hip)."""
    sh = 1 if c else 0
    pw, ph = (info.width + sh) >> sh, (info.height + sh) >> sh
    x0, y0 = ((k % info.grid_cols) * info.tile_width) >> sh, ((k // info.grid_cols) * info.tile_height) >> sh
    if x0 >= pw or y0 >= ph:
        return None
    w, h = min(info.tile_width >> sh, pw - x0), min(info.tile_height >> sh, ph - y0)
    return slice(y0, y0 + h), slice(x0, x0 + w)


class _ShmBackend:
    """CPU stand-in for tile_split.DeviceBackend: "device memory" is shared
    memory, addresses are fake 64-bit integers (one region per mapping), so
    the handle exchange, the per-rank base + offset arithmetic and the open /
    close / barrier order run exactly as on the GPU; k_gather_tiles is the
    numpy window copy above."""

    def __init__(self, rank):
        self.regions = {}  # base -> (SharedMemory, ndarray)
        self.next = (rank + 1) << 40
        self.opened = 0

    def _map(self, shm):
        base = self.next
        self.next += 1 << 32
        self.regions[base] = (shm, np.ndarray((shm.size,), np.uint8, shm.buf))
        return base

    def alloc(self, info=_Info):
        from multiprocessing import shared_memory

        dims = [(info.height, info.width)] + [((info.height + 1) // 2, (info.width + 1) // 2)] * 2
        offs, total = [], 0
        for h, w in dims:
            offs.append((total, h, w))
            total += (h * w + 255) // 256 * 256
        shm = shared_memory.SharedMemory(create=True, size=total)
        base = self._map(shm)
        return [{"planes": [(base + o, w) for o, h, w in offs], "dims": dims}], (shm, base)

    def view(self, ptr, pitch, h, w):
        base = max(b for b in self.regions if b <= ptr)
        arr = self.regions[base][1]
        o = ptr - base
        return arr[o:o + h * pitch].reshape(h, pitch)[:, :w]

    def sync(self):
        pass

    def export(self, buf):
        return buf[0].name.encode()

    def open(self, blob):
        from multiprocessing import shared_memory

        self.opened += 1
        return self._map(shared_memory.SharedMemory(name=blob.decode()))

    def close(self, ptr):
        shm, _ = self.regions.pop(ptr)
        shm.close()

    @staticmethod
    def buffer_ptr(buf):
        return buf[1]

    @staticmethod
    def planes(out):
        return out["planes"]

    def _copy(self, dst, src_pl, stride, offset):
        for k in range(offset, _Info.num_tiles, stride):
            for c, ((dp, dpitch), (sp, spitch), (h, w)) in enumerate(zip(dst["planes"], src_pl, dst["dims"])):
                win = _windows(k, c)
                if win is not None:
                    self.view(dp, dpitch, h, w)[win] = self.view(sp, spitch, h, w)[win]

    def gather_own(self, dst, src, stride, offset):
        self._copy(dst, src["planes"], stride, offset)

    def gather_from(self, dst, src_ptrs, pitches, stride, offset):
        self._copy(dst, list(zip(src_ptrs, pitches)), stride, offset)


def _pattern(k, c):
    return (k * 7 + c * 3 + 1) & 0xFF


def _gather_worker(rank, world, port, out):
    from heif_amd.tile_split import gather_to_rank0

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    be = _ShmBackend(rank)
    outs, buf = be.alloc()
    # "decode" this rank's tiles k % world == rank; every other sample keeps a sentinel
    for c, ((p, pitch), (h, w)) in enumerate(zip(outs[0]["planes"], outs[0]["dims"])):
        v = be.view(p, pitch, h, w)
        v[:] = 0xA5
        for k in range(rank, _Info.num_tiles, world):
            win = _windows(k, c)
            if win is not None:
                v[win] = _pattern(k, c)
    full = None
    if rank == 0:
        full, fbuf = be.alloc()
    gather_to_rank0(be, dist, outs, buf, full, rank, world)
    if rank == 0:
        bad = 0
        for c, ((p, pitch), (h, w)) in enumerate(zip(full[0]["planes"], full[0]["dims"])):
            v = be.view(p, pitch, h, w)
            for k in range(_Info.num_tiles):
                win = _windows(k, c)
                if win is not None:
                    bad += int((v[win] != _pattern(k, c)).sum())
        out.put((bad, be.opened, len(be.regions)))
        fbuf[0].close()
        fbuf[0].unlink()
    dist.barrier()
    buf[0].close()
    buf[0].unlink()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_tile_split_gather_to_rank0_over_gloo(world):
    """Row e2's cross-process gather (heif_amd/tile_split.py, used by bench.py
    --split tiles and the multi-GPU bench check) on CPU: handles exchanged with
    all_gather_object, rank 0 maps world - 1 peer buffers, copies every peer's
    tile windows at the peer's own base + the shared plane offsets, unmaps them,
    and the assembled planes hold every tile exactly once."""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.start_processes(_gather_worker, args=(world, _free_port(), q), nprocs=world, join=True, start_method="spawn")
    bad, opened, live = q.get()
    assert bad == 0
    assert opened == world - 1
    assert live == 2  # rank 0's own two buffers; every peer mapping closed


class _FailingOpen(_ShmBackend):
    def open(self, blob):
        raise RuntimeError("ipc_open failed")


def _gather_fail_worker(rank, world, port, out):
    from heif_amd.tile_split import gather_to_rank0

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    be = _FailingOpen(rank)
    outs, buf = be.alloc()
    full, fbuf = be.alloc() if rank == 0 else (None, None)
    try:
        gather_to_rank0(be, dist, outs, buf, full, rank, world)
        res = "returned"
    except RuntimeError as e:
        res = str(e)
    out.put((rank, res))
    for b in (buf, fbuf):
        if b is not None:
            b[0].close()
            b[0].unlink()
    dist.destroy_process_group()


def test_tile_split_gather_failure_releases_peers():
    """A failure inside rank 0's gather (here ipc_open) is raised on rank 0
    after the closing barrier, so the peers return instead of blocking in it."""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.start_processes(_gather_fail_worker, args=(2, _free_port(), q), nprocs=2, join=True, start_method="spawn")
    res = dict(q.get() for _ in range(2))
    assert res == {0: "ipc_open failed", 1: "returned"}


def _run_bench(args, extra_env=None, timeout=180):
    import json
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(extra_env or {})
    p = subprocess.run([sys.executable, str(bench.ROOT / "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=timeout)
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    return p.returncode, lines, p.stderr


def test_bench_gpus_flag_launches_ranks():
    """`python bench.py --gpus 2` with no torchrun environment starts two
    ranks itself (gloo dry run: no GPU), and rank 0 alone prints one line
    with n_gpus 2 and both ranks' disjoint shards."""
    rc, lines, err = _run_bench(["--gpus", "2", "--dry-run", "--batch", "3", "--steps", "4", "--warmup", "1"])
    assert rc == 0, err
    assert len(lines) == 1, lines
    line = lines[0]
    assert line["n_gpus"] == 2 and line["steps"] == 4 and line["warmup"] == 1
    ranks = sorted(line["ranks"], key=lambda r: r["rank"])
    assert [r["rank"] for r in ranks] == [0, 1]
    assert len({r["pid"] for r in ranks}) == 2
    assert [r["seeds"] for r in ranks] == [[0, 3], [3, 6]]


def test_bench_gpus_flag_fails_when_a_rank_fails():
    """A failing rank makes the launcher exit non-zero (and ends the other
    rank instead of leaving it blocked at the rendezvous)."""
    rc, lines, err = _run_bench(["--gpus", "2", "--dry-run"], {"BENCH_DRY_FAIL_RANK": "1"}, timeout=120)
    assert rc != 0
    assert lines == []
    assert "rank 1" in err


def test_bench_torchrun_environment_is_used_as_is():
    """Under torchrun (WORLD_SIZE set) bench.py does not spawn: the one
    process is its rank."""
    rc, lines, err = _run_bench(["--gpus", "1", "--dry-run", "--batch", "2"],
                                {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc == 0, err
    assert lines[0]["n_gpus"] == 1 and len(lines[0]["ranks"]) == 1
