"""Container / parameter-set / slice-header values on halfmoonbay.heic.

The golden values are the ones tests/libheif_comparison.rs:102-111 asserts
(ispe 4032x3024, irot 3 -> 3024x4032, luma/chroma 8/8, primary, no
thumbnails) plus the parameter-set and slice-header dissection of SURVEY.md
Appendix A.  Both the product's host parser (C ABI) and the oracle's are
checked.  No GPU needed.
"""
import pytest

import heif_amd as H


@pytest.fixture(scope="module")
def img(halfmoonbay):
    return H.HeifImage.parse(halfmoonbay)


def test_libheif_comparison_values(img):
    i = img.info
    assert (i.ispe_width, i.ispe_height) == (4032, 3024)
    assert i.rotation == 3
    rot_w, rot_h = (i.height, i.width) if i.rotation % 2 else (i.width, i.height)
    assert (rot_w, rot_h) == (3024, 4032)
    assert i.bit_depth == 8 and i.chroma_format_idc == 1
    assert i.primary_item_id == 49
    assert i.num_thumbnails == 0


def test_grid_geometry(img):
    i = img.info
    assert (i.grid_rows, i.grid_cols, i.num_tiles) == (6, 8, 48)
    assert (i.tile_width, i.tile_height) == (512, 512)
    assert (i.width, i.height) == (4032, 3024)
    assert i.coded_bytes == 1_704_187
    assert (i.matrix_coeffs, i.full_range) == (6, 1)


def test_oracle_metadata_agrees(img, oracle_mod, halfmoonbay):
    m = oracle_mod.read_meta(halfmoonbay)
    i = img.info
    assert (m["ispe_width"], m["ispe_height"], m["rotation"]) == (4032, 3024, 3)
    assert (m["width"], m["height"]) == (3024, 4032)
    assert (m["luma_bits"], m["chroma_bits"], m["num_thumbnails"]) == (8, 8, 0)
    assert m["primary_item_id"] == i.primary_item_id
    assert (m["grid_rows"], m["grid_cols"], m["num_tiles"]) == (i.grid_rows, i.grid_cols, i.num_tiles)
    assert (m["out_width"], m["out_height"]) == (i.width, i.height)


def test_sps_pps_appendix_a(img):
    t = img.tile_params(0)
    want = dict(
        general_profile_idc=3, general_level_idc=90, pic_width=512, pic_height=512, chroma_format_idc=1,
        bit_depth_luma=8, bit_depth_chroma=8, log2_max_poc_lsb=11, log2_min_cb=3, log2_ctb=5, log2_min_tb=2,
        log2_max_tb=5, max_th_depth_inter=1, max_th_depth_intra=0, scaling_list_enabled=1, amp=0, sao=1,
        pcm=0, num_short_term_ref_pic_sets=0, long_term_refs=0, temporal_mvp=1, strong_intra_smoothing=0,
        video_full_range=1, colour_primaries=2, transfer_characteristics=2, matrix_coeffs=6,
        init_qp=15, sign_data_hiding=0, cabac_init_present=0, constrained_intra_pred=0, transform_skip=0,
        cu_qp_delta_enabled=1, diff_cu_qp_delta_depth=2, cb_qp_offset=2, cr_qp_offset=2,
        slice_chroma_qp_offsets_present=0, transquant_bypass=0, tiles_enabled=0, entropy_coding_sync=1,
        loop_filter_across_slices=0, deblocking_control_present=1, deblocking_override_enabled=0,
        deblocking_disabled=0, beta_offset_div2=0, tc_offset_div2=0, log2_parallel_merge_level=2,
    )
    assert {k: t[k] for k in want} == want


def test_slice_headers_all_tiles(img):
    for k in range(48):
        t = img.tile_params(k)
        assert t["nal_unit_type"] == 20 and t["slice_type"] == 2 and t["first_slice_segment_in_pic"] == 1
        assert (t["slice_sao_luma"], t["slice_sao_chroma"], t["slice_qp_y"]) == (1, 1, 15)
        assert t["num_entry_point_offsets"] == 15
        # the 16 substreams tile the slice data exactly
        assert t["slice_data_raw_offset"] + sum(t["entry_point_offset"]) < t["payload_bytes"]


def test_tile1_entry_points(img):
    t = img.tile_params(0)
    assert t["entry_point_offset"] == [136, 109, 118, 83, 80, 101, 92, 87, 79, 81, 81, 77, 74, 84, 78]
    last = t["payload_bytes"] - t["slice_data_raw_offset"] - sum(t["entry_point_offset"])
    assert last == 75


def test_tile_index_out_of_range(img):
    with pytest.raises(H.HeifGpuError):
        img.tile_params(48)


@pytest.mark.parametrize("cut", [0, 8, 100, 3626, 9000])
def test_truncated_file_is_a_parse_error(halfmoonbay, cut):
    with pytest.raises(H.HeifGpuError):
        H.HeifImage.parse(halfmoonbay[:cut])


def test_not_heif_is_a_parse_error():
    with pytest.raises(H.HeifGpuError):
        H.HeifImage.parse(b"\x89PNG\r\n\x1a\n" + bytes(64))
