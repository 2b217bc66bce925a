"""Row e2 across processes on the GPU: two ranks (one process each, here on
the same device) decode the tile subsets k % 2 == rank of halfmoonbay into one
buffer each; rank 0 maps rank 1's buffer with heifgpu_ipc_open and gathers
both subsets with k_gather_tiles (heif_amd/tile_split.py, the same code
bench.py runs across GPUs).  The assembled planes must equal the oracle's."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _log(rank, msg):
    import sys
    import time

    print(f"[ipc rank {rank} {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _digest(a) -> str:
    import hashlib

    return hashlib.sha256(np.ascontiguousarray(a.astype(np.uint16)).tobytes()).hexdigest()


def _worker(rank, world, port, path, q):
    import torch.distributed as dist

    import heif_amd as H
    from heif_amd.tile_split import DeviceBackend, gather_to_rank0

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    _log(rank, "init")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    _log(rank, "decode")
    ctx = H.DecodeContext(0)
    img = H.HeifImage.parse(open(path, "rb").read())
    b = ctx.prepare([img], tile_stride=world, tile_offset=rank)
    outs, buf = ctx.alloc_outputs_contiguous([img])
    buf.fill_(0xA5)
    b.decode_async(outs)
    st = b.status()
    b.free()
    full = ctx.alloc_outputs([img]) if rank == 0 else None
    if full:
        for t in (full[0].y, full[0].cb, full[0].cr):
            t.fill_(0)
    _log(rank, f"status {st}; gather")
    gather_to_rank0(DeviceBackend(H, ctx), dist, outs, buf, full, rank, world)
    _log(rank, "gathered")
    if rank == 0:  # digests only: a large object would block in the pipe until the parent joins
        q.put((st, [_digest(t.cpu().numpy()) for t in (full[0].y, full[0].cb, full[0].cr)]))
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_ipc_tile_split_gather(world, oracle_halfmoonbay):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import pathlib

    import torch.multiprocessing as mp

    path = str(pathlib.Path(__file__).resolve().parent / "golden" / "halfmoonbay.heic")
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.start_processes(_worker, args=(world, _free_port(), path, q), nprocs=world, join=True, start_method="spawn")
    st, digests = q.get()
    assert st == [0]
    assert digests == [_digest(p) for p in (oracle_halfmoonbay.y, oracle_halfmoonbay.cb, oracle_halfmoonbay.cr)]
