"""Single-image tile split across GPUs, one process per GPU (SURVEY §8(e),
config 5 "1->8 GPUs").

Grid tiles are independent pictures (the reference decodes them one by one,
src/heic/decoder.rs:98-119), so rank r of `world` decodes the tiles
k % world == r of every image into its own full-size planes
(heifgpu_batch_opts tile_stride / tile_offset) with no data-path collective.
`gather_to_rank0` then assembles the images on rank 0: every rank exports the
one device buffer holding its planes (heifgpu_ipc_export), the 72-byte
handles travel over torch.distributed (all_gather_object), and rank 0 maps
each peer's buffer (heifgpu_ipc_open) and runs k_gather_tiles, which reads
the peer planes over xGMI.  The peers keep their buffers alive until rank 0
has finished (the closing barrier).

The device operations sit behind a small backend interface so the exchange
and the address arithmetic are also exercised on CPU (tests/test_distributed.py
runs them over gloo with shared-memory buffers).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple


class DeviceBackend:
    """heif_amd device operations for gather_to_rank0 (one DecodeContext)."""

    def __init__(self, H, ctx, stream=None):
        self.H, self.ctx, self.stream = H, ctx, stream

    def _s(self):
        return None if self.stream is None else self.stream.cuda_stream

    def sync(self):
        self.ctx._torch.cuda.synchronize(self.ctx.device)

    def export(self, buf) -> bytes:
        return self.H.ipc_export(buf)

    def open(self, blob: bytes) -> int:
        return self.H.ipc_open(self.ctx.device, blob)

    def close(self, ptr: int):
        self.H.ipc_close(ptr)

    @staticmethod
    def buffer_ptr(buf) -> int:
        return buf.data_ptr()

    @staticmethod
    def planes(out) -> List[Tuple[int, int]]:
        return [(t.data_ptr(), t.stride(0) * t.element_size()) for t in (out.y, out.cb, out.cr) if t is not None]

    def gather_own(self, dst, src, stride: int, offset: int):
        self.ctx.gather_tiles(dst, src, stride, offset, self._s())

    def gather_from(self, dst, src_ptrs: Sequence[int], pitches: Sequence[int], stride: int, offset: int):
        self.ctx.gather_tiles_from(dst, src_ptrs, pitches, stride, offset, self._s())


def gather_to_rank0(backend, dist, outs, buf, full: Optional[list], rank: int, world: int) -> None:
    """Assembles the tile-split images `outs` (this rank's planes, all inside
    `buf`, decoded with tile_stride = world, tile_offset = rank) into `full`
    (rank 0's full-size planes; None on other ranks).  Collective: every rank
    calls it."""
    backend.sync()  # this rank's decode has written its planes
    blob = backend.export(buf)
    blobs = [None] * world
    dist.all_gather_object(blobs, blob)
    # Every rank reaches the closing barrier, also when rank 0's gather fails
    # (the error is raised after it), so no peer is left blocked in it.
    try:
        if rank == 0:
            for dst, src in zip(full, outs):
                backend.gather_own(dst, src, world, 0)
            bases = []
            try:
                for r in range(1, world):
                    base = backend.open(blobs[r])
                    bases.append(base)
                    b0 = backend.buffer_ptr(buf)  # every rank carved the same layout from its buffer
                    for dst, src in zip(full, outs):
                        pl = backend.planes(src)
                        backend.gather_from(dst, [base + (p - b0) for p, _ in pl], [pitch for _, pitch in pl],
                                            world, r)
                backend.sync()  # the gather kernels have read the peer planes
            finally:
                for b in bases:
                    backend.close(b)
    finally:
        dist.barrier()  # peers keep their planes until rank 0 is done
