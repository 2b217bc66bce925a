"""heif_amd — MI355X-native HEIC (HEVC intra still) decode path.

Host-side mirror of the reference API (friendlymatthew/heif):

* ``HeicDecoder.decode(data)``  ↔ ``heif::HeicDecoder::decode(&[u8])``
  (src/heic/decoder.rs:12) — but returns the decoded planes instead of ``()``.
* ``HeifImage.parse(data)`` / ``.info`` ↔ the host half of that function
  (HeifReader::read, hvcC → VPS/SPS/PPS, grid tiles, slice headers).
* ``RbspReader.remove_emulation_prevention`` / ``read_ue`` / ``read_se``
  ↔ src/hevc/rbsp_reader.rs.

Everything runs through the C ABI in ``include/heifgpu.h`` (libheifgpu.so);
decoding runs in gfx950 HIP kernels.  PyTorch only supplies device memory,
streams and ``torch.distributed``.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence

from . import _lib
from ._lib import HeifGpuError, UnsupportedError, lib

__all__ = [
    "HeicDecoder", "HeifImage", "DecodeContext", "DeviceBatch", "DecodedImage", "RbspReader",
    "HeifGpuError", "UnsupportedError", "ipc_export", "ipc_open", "ipc_close", "chroma_dims",
]


class RbspReader:
    """rbsp_reader.rs surface used by the reference's unit tests."""

    @staticmethod
    def remove_emulation_prevention(data: bytes) -> bytes:
        src = _lib.u8buf(data)
        dst = (ctypes.c_uint8 * max(len(data), 1))()
        n = lib.heifgpu_remove_emulation_prevention(src, len(data), dst)
        return bytes(dst[:n])

    @staticmethod
    def read_ue(data: bytes) -> int:
        v = ctypes.c_uint32()
        _lib.check(lib.heifgpu_read_ue(_lib.u8buf(data), len(data), ctypes.byref(v)))
        return v.value

    @staticmethod
    def read_se(data: bytes) -> int:
        v = ctypes.c_int32()
        _lib.check(lib.heifgpu_read_se(_lib.u8buf(data), len(data), ctypes.byref(v)))
        return v.value


class HeifImage:
    """A host-parsed HEIC image (container + parameter sets + slice headers)."""

    def __init__(self, handle: int):
        self._h = ctypes.c_void_p(handle)

    @classmethod
    def parse(cls, data: bytes, item_id: int = 0) -> "HeifImage":
        """The primary image (item_id 0), or any coded image item, e.g. the
        auxiliary HDR gain map at `HeifImage.parse(d).info.aux_item_id`."""
        h = ctypes.c_void_p()
        _lib.check(lib.heifgpu_image_parse_item(_lib.u8buf(data), len(data), item_id, ctypes.byref(h)))
        return cls(h.value)

    @classmethod
    def parse_many(cls, files: Sequence[bytes], threads: int = 0) -> List["HeifImage"]:
        """Primary images of many files, parsed on `threads` native host threads
        (heifgpu_image_parse_many; 0 = every hardware thread)."""
        n = len(files)
        files = [bytes(f) for f in files]  # no copy for bytes; the library copies what it keeps
        # pointers straight into the bytes objects (no Python-side copy of the files)
        data = (ctypes.POINTER(ctypes.c_uint8) * max(n, 1))(
            *[ctypes.cast(ctypes.c_char_p(f), ctypes.POINTER(ctypes.c_uint8)) for f in files])
        lens = (ctypes.c_size_t * max(n, 1))(*[len(f) for f in files])
        hs = (ctypes.c_void_p * max(n, 1))()
        rc = lib.heifgpu_image_parse_many(data, lens, n, threads, hs, None)
        imgs = [cls(h) if h else None for h in hs[:n]]
        _lib.check(rc)
        return imgs

    @property
    def info(self) -> _lib.ImageInfo:
        info = _lib.ImageInfo()
        _lib.check(lib.heifgpu_image_get_info(self._h, ctypes.byref(info)))
        return info

    def tile_params(self, tile: int) -> dict:
        """Parsed SPS/PPS/slice-header fields of grid tile `tile` (row-major)."""
        tp = _lib.TileParams()
        _lib.check(lib.heifgpu_image_tile_params(self._h, tile, ctypes.byref(tp)))
        d = {n: getattr(tp, n) for n, _ in tp._fields_ if n != "entry_point_offset"}
        d["entry_point_offset"] = list(tp.entry_point_offset[: min(tp.num_entry_point_offsets, 64)])
        return d

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and lib is not None:  # lib is None during interpreter teardown
            lib.heifgpu_image_free(h)
            self._h = None


def chroma_dims(info):
    """(height, width) of an image's Cb / Cr planes: chroma_format_idc 1 (4:2:0)
    halves both axes, 2 (4:2:2) the width, 3 (4:4:4) neither (Table 6-1), odd
    sizes rounded up."""
    sx = 1 if info.chroma_format_idc in (1, 2) else 0
    sy = 1 if info.chroma_format_idc == 1 else 0
    return (info.height + sy) >> sy, (info.width + sx) >> sx


@dataclass
class DecodedImage:
    y: "object"            # torch tensor on the device, (H, W)
    cb: Optional["object"]  # (ceil(H/2), ceil(W/2)) for 4:2:0
    cr: Optional["object"]
    info: _lib.ImageInfo


class DecodeContext:
    """One heifgpu context per device (not shared across threads)."""

    def __init__(self, device: int = 0):
        import torch

        self.device = device
        self._torch = torch
        h = ctypes.c_void_p()
        _lib.check(lib.heifgpu_create(device, ctypes.byref(h)))
        self._h = h

    def close(self):
        if self._h is not None and self._h.value:
            lib.heifgpu_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def alloc_outputs_contiguous(self, images: Sequence[HeifImage]):
        """Output planes of `images` carved from ONE device buffer (256-byte
        aligned planes), so a single heifgpu_ipc_export handle covers all of
        them; returns (outputs, buffer)."""
        torch = self._torch
        dev = torch.device("cuda", self.device)
        shapes = []
        total = 0
        for im in images:
            inf = im.info
            dims = [(inf.height, inf.width)]
            if inf.chroma_format_idc:
                dims += [chroma_dims(inf)] * 2
            offs = []
            for h, w in dims:
                offs.append((total, h, w))
                total += (h * w * inf.bytes_per_sample + 255) // 256 * 256
            shapes.append((inf, offs))
        buf = torch.empty(max(total, 256), dtype=torch.uint8, device=dev)
        outs = []
        for inf, offs in shapes:
            dt = torch.uint8 if inf.bytes_per_sample == 1 else torch.int16
            pl = [buf[o:o + h * w * inf.bytes_per_sample].view(dt).view(h, w) for o, h, w in offs]
            outs.append(DecodedImage(pl[0], pl[1] if len(pl) > 1 else None, pl[2] if len(pl) > 1 else None, inf))
        return outs, buf

    def alloc_outputs(self, images: Sequence[HeifImage]) -> List[DecodedImage]:
        torch = self._torch
        outs = []
        for im in images:
            inf = im.info
            dt = torch.uint8 if inf.bytes_per_sample == 1 else torch.int16
            dev = torch.device("cuda", self.device)
            y = torch.empty((inf.height, inf.width), dtype=dt, device=dev)
            cb = cr = None
            if inf.chroma_format_idc:
                ch, cw = chroma_dims(inf)
                cb = torch.empty((ch, cw), dtype=dt, device=dev)
                cr = torch.empty((ch, cw), dtype=dt, device=dev)
            outs.append(DecodedImage(y, cb, cr, inf))
        return outs

    @staticmethod
    def planes_of(outs: Sequence[DecodedImage]):
        arr = (_lib.Planes * len(outs))()
        for i, o in enumerate(outs):
            for c, t in enumerate((o.y, o.cb, o.cr)):
                if t is not None:
                    arr[i].plane[c] = t.data_ptr()
                    arr[i].pitch[c] = t.stride(0) * t.element_size()
        return arr

    def prepare(self, images: Sequence[HeifImage], tile_stride: int = 1, tile_offset: int = 0,
                reuse: Optional["DeviceBatch"] = None, wait: bool = True, parse: str = "auto",
                pics_per_wave: int = 0, pipeline_sets: int = 0) -> "DeviceBatch":
        """Device batch of `images` (heifgpu_batch_prepare_ex).  tile_stride /
        tile_offset select the grid tiles k % tile_stride == tile_offset (the
        single-image tile split across GPUs); `reuse` reloads an existing batch
        in place; wait=False returns before the upload has finished (the next
        decode of the batch waits for it).  parse: "auto" (by batch size),
        "lanes" (one substream per lane, `pics_per_wave` pictures per wave, 0 =
        adaptive), "solo" (one substream per wave, a picture's rows in one
        workgroup) or "spread" (one substream per wave, one workgroup per row:
        small-batch latency).  pipeline_sets: parse-output sets of a new batch
        (0 = default 3; 1-3, include/heifgpu.h)."""
        arr = (ctypes.c_void_p * len(images))(*[im._h.value for im in images])
        opts = _lib.BatchOpts(tile_stride, tile_offset, _lib.PARSE_MODES[parse], pics_per_wave, pipeline_sets)
        if reuse is not None:
            _lib.check(lib.heifgpu_batch_prepare_ex(self._h, arr, len(images), ctypes.byref(opts),
                                                    ctypes.byref(reuse._h)))
            reuse.images = list(images)
            batch = reuse
        else:
            b = ctypes.c_void_p()
            _lib.check(lib.heifgpu_batch_prepare_ex(self._h, arr, len(images), ctypes.byref(opts), ctypes.byref(b)))
            batch = DeviceBatch(self, b, list(images))
        if wait:
            self._torch.cuda.synchronize(self.device)
        return batch

    def gather_tiles(self, dst: DecodedImage, src: DecodedImage, tile_stride: int, tile_offset: int,
                     stream: Optional[int] = None):
        """Copy the tiles k % tile_stride == tile_offset of `src` (decoded with
        those options, on any device) into `dst` on this context's device."""
        if stream is None:
            stream = self._torch.cuda.current_stream(self.device).cuda_stream
        _lib.check(lib.heifgpu_gather_tiles(ctypes.byref(dst.info), DecodeContext.planes_of([dst]),
                                            DecodeContext.planes_of([src]), tile_stride, tile_offset,
                                            ctypes.c_void_p(stream)))

    def gather_tiles_from(self, dst: DecodedImage, src_ptrs: Sequence[int], src_pitches: Sequence[int],
                          tile_stride: int, tile_offset: int, stream: Optional[int] = None):
        """gather_tiles from raw device pointers, e.g. another process's planes
        mapped with ipc_open."""
        if stream is None:
            stream = self._torch.cuda.current_stream(self.device).cuda_stream
        src = (_lib.Planes * 1)()
        for c in range(3):
            src[0].plane[c] = src_ptrs[c] if c < len(src_ptrs) else None
            src[0].pitch[c] = src_pitches[c] if c < len(src_pitches) else 0
        _lib.check(lib.heifgpu_gather_tiles(ctypes.byref(dst.info), DecodeContext.planes_of([dst]), src, tile_stride,
                                            tile_offset, ctypes.c_void_p(stream)))

    def set_timing(self, enable: bool):
        _lib.check(lib.heifgpu_set_timing(self._h, 1 if enable else 0))

    def stage_times(self) -> List[float]:
        """ms of the last timed decode: parse, transform, intra, deblock, sao_out, rbsp."""
        ms = (ctypes.c_float * 6)()
        _lib.check(lib.heifgpu_stage_times(self._h, ms))
        return list(ms)

    def to_rgb(self, img: DecodedImage, stream: Optional[int] = None):
        """Interleaved 8-bit RGB (H', W', 3) with the irot rotation applied
        (heifgpu_ycbcr_to_rgb), as a torch tensor on the device."""
        torch = self._torch
        inf = img.info
        rot = inf.rotation & 3
        ow, oh = (inf.height, inf.width) if rot & 1 else (inf.width, inf.height)
        rgb = torch.empty((oh, ow, 3), dtype=torch.uint8, device=torch.device("cuda", self.device))
        if stream is None:
            stream = torch.cuda.current_stream(self.device).cuda_stream
        planes = DecodeContext.planes_of([img])
        _lib.check(lib.heifgpu_ycbcr_to_rgb(self._h, ctypes.byref(inf), planes, ctypes.c_void_p(rgb.data_ptr()),
                                            rgb.stride(0), ctypes.c_void_p(stream)))
        return rgb


def ipc_export(tensor) -> bytes:
    """heifgpu_ipc_export of a device tensor's storage: 72 bytes another
    process passes to ipc_open (e.g. through torch.distributed)."""
    h = _lib.IpcHandle()
    _lib.check(lib.heifgpu_ipc_export(ctypes.c_void_p(tensor.data_ptr()), ctypes.byref(h)))
    return bytes(h)


def ipc_open(device: int, blob: bytes) -> int:
    """Maps another process's exported allocation on `device`; returns the
    device address of the exported byte (close with ipc_close)."""
    h = _lib.IpcHandle.from_buffer_copy(blob)
    p = ctypes.c_void_p()
    _lib.check(lib.heifgpu_ipc_open(device, ctypes.byref(h), ctypes.byref(p)))
    return p.value


def ipc_close(ptr: int) -> None:
    _lib.check(lib.heifgpu_ipc_close(ctypes.c_void_p(ptr)))


class DeviceBatch:
    """Device-resident batch: bitstreams uploaded once, decoded many times."""

    def __init__(self, ctx: DecodeContext, handle: ctypes.c_void_p, images: List[HeifImage]):
        self.ctx, self._h, self.images = ctx, handle, images

    def decode_async(self, outs: Sequence[DecodedImage], stream: Optional[int] = None):
        torch = self.ctx._torch
        if stream is None:
            stream = torch.cuda.current_stream(self.ctx.device).cuda_stream
        planes = DecodeContext.planes_of(outs)
        _lib.check(lib.heifgpu_batch_decode(self.ctx._h, self._h, planes, ctypes.c_void_p(stream)))

    def status(self, stream: Optional[int] = None) -> List[int]:
        torch = self.ctx._torch
        if stream is None:
            stream = torch.cuda.current_stream(self.ctx.device).cuda_stream
        st = (ctypes.c_uint32 * len(self.images))()
        rc = lib.heifgpu_batch_status(self.ctx._h, self._h, st, ctypes.c_void_p(stream))
        if rc not in (_lib.HEIFGPU_OK, _lib.HEIFGPU_E_DECODE):
            _lib.check(rc)
        return list(st)

    def status_previous(self, stream: Optional[int] = None) -> List[int]:
        """Per-image status of the load before the current one (its decodes
        that were in flight at the reload), read and cleared
        (heifgpu_batch_status_previous); [] if there was no previous load."""
        torch = self.ctx._torch
        if stream is None:
            stream = torch.cuda.current_stream(self.ctx.device).cuda_stream
        n = ctypes.c_size_t()
        rc = lib.heifgpu_batch_status_previous(self.ctx._h, self._h, None, 0, ctypes.byref(n),
                                               ctypes.c_void_p(stream))
        if n.value == 0:
            _lib.check(rc)
            return []
        st = (ctypes.c_uint32 * n.value)()
        rc = lib.heifgpu_batch_status_previous(self.ctx._h, self._h, st, n.value, ctypes.byref(n),
                                               ctypes.c_void_p(stream))
        if rc not in (_lib.HEIFGPU_OK, _lib.HEIFGPU_E_DECODE):
            _lib.check(rc)
        return list(st)

    def parse_geometry(self) -> dict:
        """The CABAC parse launch of this batch (heifgpu_batch_parse_geometry)."""
        v = [ctypes.c_uint32() for _ in range(4)]
        _lib.check(lib.heifgpu_batch_parse_geometry(self._h, *[ctypes.byref(x) for x in v]))
        mode = {_lib.PARSE_LANES: "lanes", _lib.PARSE_SOLO: "solo", _lib.PARSE_SPREAD: "spread"}[v[0].value]
        return {"mode": mode, "workgroups": v[1].value, "pics_per_wave": v[2].value,
                "waves_per_workgroup": v[3].value}

    def free(self):
        if self._h is not None and self._h.value:
            lib.heifgpu_batch_free(self._h)
        self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class HeicDecoder:
    """Mirror of heif::HeicDecoder (src/heic/decoder.rs:8-132)."""

    _ctx: dict = {}

    @classmethod
    def context(cls, device: int = 0) -> DecodeContext:
        ctx = cls._ctx.get(device)
        if ctx is None:
            ctx = cls._ctx[device] = DecodeContext(device)
        return ctx

    @classmethod
    def decode_rgb(cls, data: bytes, device: int = 0, item_id: int = 0):
        """decode() then YCbCr -> RGB8 with the irot rotation (libheif's default output)."""
        return cls.context(device).to_rgb(cls.decode(data, device, item_id))

    @classmethod
    def decode(cls, data: bytes, device: int = 0, item_id: int = 0) -> DecodedImage:
        ctx = cls.context(device)
        img = HeifImage.parse(data, item_id)
        outs = ctx.alloc_outputs([img])
        batch = ctx.prepare([img])
        try:
            batch.decode_async(outs)
            st = batch.status()
        finally:
            batch.free()
        if st[0]:
            bits = [n for b, n in _lib.STATUS_BITS.items() if st[0] & b]
            raise HeifGpuError(_lib.HEIFGPU_E_DECODE, f"bitstream check failed: {bits}")
        return outs[0]
