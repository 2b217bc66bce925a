"""ctypes binding of include/heifgpu.h (libheifgpu.so, built in-tree).

The product path has no CPU fallback: if the HIP library is missing this
module raises at import time.
"""
from __future__ import annotations

import ctypes
import os
import pathlib

_HERE = pathlib.Path(__file__).resolve().parent
# HEIFGPU_LIBRARY selects another in-tree build of the same ABI (e.g. the
# counter-instrumented heif_amd/libheifgpu_prof.so from `make prof`)
LIB_PATH = pathlib.Path(os.environ.get("HEIFGPU_LIBRARY", _HERE / "libheifgpu.so"))

HEIFGPU_OK = 0
HEIFGPU_E_INVALID = -1
HEIFGPU_E_PARSE = -2
HEIFGPU_E_UNSUPPORTED = -3
HEIFGPU_E_DEVICE = -4
HEIFGPU_E_DECODE = -5

STATUS_BITS = {
    1 << 0: "cabac_init",
    1 << 1: "substream_end",
    1 << 2: "overrun",
    1 << 3: "syntax",
    1 << 4: "unsupported",
    1 << 5: "capacity",
}


class ImageInfo(ctypes.Structure):
    _fields_ = [
        (name, ctypes.c_uint32)
        for name in (
            "width", "height", "chroma_format_idc", "bit_depth", "bytes_per_sample", "grid_rows",
            "grid_cols", "tile_width", "tile_height", "num_tiles", "rotation", "ispe_width",
            "ispe_height", "coded_bytes", "primary_item_id", "num_thumbnails", "matrix_coeffs",
            "full_range", "item_id", "aux_item_id",
        )
    ]


class TileParams(ctypes.Structure):
    """heifgpu_tile_params (parsed SPS/PPS/slice header of one tile)."""
    _fields_ = [(name, ctypes.c_int32) for name in (
            "nal_unit_type",
            "slice_type",
            "first_slice_segment_in_pic",
            "general_profile_idc",
            "general_level_idc",
            "pic_width",
            "pic_height",
            "chroma_format_idc",
            "bit_depth_luma",
            "bit_depth_chroma",
            "log2_max_poc_lsb",
            "log2_min_cb",
            "log2_ctb",
            "log2_min_tb",
            "log2_max_tb",
            "max_th_depth_inter",
            "max_th_depth_intra",
            "scaling_list_enabled",
            "amp",
            "sao",
            "pcm",
            "num_short_term_ref_pic_sets",
            "long_term_refs",
            "temporal_mvp",
            "strong_intra_smoothing",
            "video_full_range",
            "colour_primaries",
            "transfer_characteristics",
            "matrix_coeffs",
            "init_qp",
            "sign_data_hiding",
            "cabac_init_present",
            "constrained_intra_pred",
            "transform_skip",
            "cu_qp_delta_enabled",
            "diff_cu_qp_delta_depth",
            "cb_qp_offset",
            "cr_qp_offset",
            "slice_chroma_qp_offsets_present",
            "transquant_bypass",
            "tiles_enabled",
            "entropy_coding_sync",
            "loop_filter_across_slices",
            "deblocking_control_present",
            "deblocking_override_enabled",
            "deblocking_disabled",
            "beta_offset_div2",
            "tc_offset_div2",
            "log2_parallel_merge_level",
            "slice_sao_luma",
            "slice_sao_chroma",
            "slice_qp_y",
            "num_entry_point_offsets",
            "slice_data_raw_offset",
            "payload_bytes",
    )] + [("entry_point_offset", ctypes.c_uint32 * 64)]


class Planes(ctypes.Structure):
    _fields_ = [("plane", ctypes.c_void_p * 3), ("pitch", ctypes.c_int32 * 3)]


class BatchOpts(ctypes.Structure):
    """heifgpu_batch_opts: decode only grid tiles k with k % tile_stride == tile_offset;
    parse_mode (PARSE_*) and, in lanes mode, pictures per wave (0 = adaptive)."""
    _fields_ = [("tile_stride", ctypes.c_uint32), ("tile_offset", ctypes.c_uint32),
                ("parse_mode", ctypes.c_uint32), ("pics_per_wave", ctypes.c_uint32),
                ("pipeline_sets", ctypes.c_uint32)]


class IpcHandle(ctypes.Structure):
    """heifgpu_ipc_handle: a device allocation exported to another process."""
    _fields_ = [("handle", ctypes.c_uint8 * 64), ("offset", ctypes.c_uint64)]


PARSE_AUTO, PARSE_LANES, PARSE_SOLO, PARSE_SPREAD = 0, 1, 2, 3
PARSE_ROWS = 4  # ABI 5 only; removed in ABI 6 (prepare answers HEIFGPU_E_UNSUPPORTED)
PARSE_MODES = {"auto": PARSE_AUTO, "lanes": PARSE_LANES, "solo": PARSE_SOLO, "spread": PARSE_SPREAD}
ABI_VERSION = 6  # HEIFGPU_ABI_VERSION of include/heifgpu.h these declarations follow


# every symbol include/heifgpu.h declares (checked by tests/test_abi.py)
EXPORTS = (
    "heifgpu_image_parse", "heifgpu_image_get_info", "heifgpu_image_free", "heifgpu_create",
    "heifgpu_destroy", "heifgpu_last_error", "heifgpu_batch_prepare", "heifgpu_batch_decode",
    "heifgpu_batch_status", "heifgpu_batch_free", "heifgpu_set_timing", "heifgpu_stage_times",
    "heifgpu_decode_batch", "heifgpu_remove_emulation_prevention", "heifgpu_read_ue",
    "heifgpu_read_se", "heifgpu_bins_truncated_rice", "heifgpu_bins_chroma_pred_mode",
    "heifgpu_bins_coeff_abs_level_remaining", "heifgpu_bins_exp_golomb", "heifgpu_image_tile_params", "heifgpu_debug_counters",
    "heifgpu_image_parse_item", "heifgpu_ycbcr_to_rgb", "heifgpu_batch_prepare_ex", "heifgpu_gather_tiles",
    "heifgpu_image_parse_many", "heifgpu_batch_parse_geometry", "heifgpu_ipc_export", "heifgpu_ipc_open",
    "heifgpu_ipc_close", "heifgpu_batch_status_previous", "heifgpu_abi_version",
)


class HeifGpuError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"heifgpu error {code}: {msg}")
        self.code = code


class UnsupportedError(HeifGpuError):
    pass


def _bind_hip_runtime() -> None:
    """One HIP runtime per process.  PyTorch-ROCm ships its own libamdhip64;
    if libheifgpu.so were loaded first it would pull /opt/rocm's copy and the
    two runtimes cannot share the device (whichever initialises second sees
    no GPU).  Importing torch first makes the dynamic linker bind
    libheifgpu.so's libamdhip64.so.7 dependency to torch's already-loaded
    copy.  Without torch (e.g. a C/Rust host) nothing changes."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def _load() -> ctypes.CDLL:
    _bind_hip_runtime()
    if not LIB_PATH.exists():
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no CPU fallback on the product path)"
        )
    lib = ctypes.CDLL(str(LIB_PATH), mode=os.RTLD_LOCAL)
    P, VP, SZ, I32, U32 = ctypes.POINTER, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint32
    u8p = P(ctypes.c_uint8)
    sig = {
        "heifgpu_image_parse": (I32, [u8p, SZ, P(VP)]),
        "heifgpu_image_get_info": (I32, [VP, P(ImageInfo)]),
        "heifgpu_image_free": (None, [VP]),
        "heifgpu_create": (I32, [I32, P(VP)]),
        "heifgpu_destroy": (None, [VP]),
        "heifgpu_last_error": (ctypes.c_char_p, []),
        "heifgpu_batch_prepare": (I32, [VP, P(VP), SZ, P(VP)]),
        "heifgpu_batch_decode": (I32, [VP, VP, P(Planes), VP]),
        "heifgpu_batch_status": (I32, [VP, VP, P(U32), VP]),
        "heifgpu_batch_status_previous": (I32, [VP, VP, P(U32), SZ, P(SZ), VP]),
        "heifgpu_abi_version": (I32, []),
        "heifgpu_batch_free": (None, [VP]),
        "heifgpu_set_timing": (I32, [VP, I32]),
        "heifgpu_stage_times": (I32, [VP, P(ctypes.c_float)]),
        "heifgpu_decode_batch": (I32, [VP, P(VP), SZ, P(Planes), VP, P(U32)]),
        "heifgpu_remove_emulation_prevention": (SZ, [u8p, SZ, u8p]),
        "heifgpu_read_ue": (I32, [u8p, SZ, P(U32)]),
        "heifgpu_read_se": (I32, [u8p, SZ, P(ctypes.c_int32)]),
        "heifgpu_bins_truncated_rice": (I32, [u8p, I32, I32, I32, P(I32)]),
        "heifgpu_bins_chroma_pred_mode": (I32, [u8p, I32, P(I32)]),
        "heifgpu_bins_coeff_abs_level_remaining": (I32, [u8p, I32, I32, P(I32)]),
        "heifgpu_bins_exp_golomb": (I32, [u8p, I32, I32, P(I32)]),
        "heifgpu_image_tile_params": (I32, [VP, U32, P(TileParams)]),
        "heifgpu_debug_counters": (I32, [P(ctypes.c_uint64), I32]),
        "heifgpu_image_parse_item": (I32, [u8p, SZ, U32, P(VP)]),
        "heifgpu_ycbcr_to_rgb": (I32, [VP, P(ImageInfo), P(Planes), VP, I32, VP]),
        "heifgpu_batch_prepare_ex": (I32, [VP, P(VP), SZ, P(BatchOpts), P(VP)]),
        "heifgpu_gather_tiles": (I32, [P(ImageInfo), P(Planes), P(Planes), U32, U32, VP]),
        "heifgpu_image_parse_many": (I32, [P(P(ctypes.c_uint8)), P(SZ), SZ, I32, P(VP), P(I32)]),
        "heifgpu_batch_parse_geometry": (I32, [VP, P(U32), P(U32), P(U32), P(U32)]),
        "heifgpu_ipc_export": (I32, [VP, P(IpcHandle)]),
        "heifgpu_ipc_open": (I32, [I32, P(IpcHandle), P(VP)]),
        "heifgpu_ipc_close": (I32, [VP]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    # the structs above follow ABI_VERSION: a library of another version must not be called
    got = lib.heifgpu_abi_version()
    if got != ABI_VERSION:
        raise ImportError(f"{LIB_PATH}: library ABI {got}, these bindings expect {ABI_VERSION} (rebuild it)")
    return lib


lib = _load()


def last_error() -> str:
    return lib.heifgpu_last_error().decode(errors="replace")


def check(rc: int) -> None:
    if rc == HEIFGPU_OK:
        return
    if rc == HEIFGPU_E_UNSUPPORTED:
        raise UnsupportedError(rc, last_error())
    raise HeifGpuError(rc, last_error())


def u8buf(data: bytes):
    return (ctypes.c_uint8 * max(len(data), 1)).from_buffer_copy(data if data else b"\0")
