"""The C ABI library: loads without a GPU, exports every symbol include/pcfm.h
declares, and validates arguments on the host before touching the device."""
import ctypes
import os
import re

import pytest

from pcfm import _lib

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                      "pcfm.h")


def header_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(pcfm_[a-z0-9_]+)\s*\(", text)))


def test_header_and_binding_agree():
    assert header_symbols() == sorted(_lib.SIGNATURES)


def test_library_exports_every_symbol():
    lib = _lib.load()
    for name in header_symbols():
        assert hasattr(lib, name), name
    assert lib.pcfm_abi_version() == _lib.ABI_VERSION


def test_built_for_gfx950():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_workspace_queries():
    q = _lib.query
    assert q("pcfm_avg_voxelize_fwd_workspace_bytes", 8, 128, 20000, 32) > 8 * 20000 * 128 * 4
    assert q("pcfm_trilinear_devoxelize_bwd_workspace_bytes", 8, 128, 20000, 32) > 0
    assert q("pcfm_grouping_bwd_workspace_bytes", 2, 16, 1000, 64, 16) > 0
    assert q("pcfm_emd_workspace_bytes", 2, 100, 100, 4) * 2 == \
        q("pcfm_emd_workspace_bytes", 2, 100, 100, 8)
    assert q("pcfm_emd_workspace_bytes", 2, 100, 100, 3) == 0
    assert q("pcfm_avg_voxelize_fwd_workspace_bytes", -1, 1, 1, 2) == 0
    # occupancy masks: tile / pair-chunk / 16-voxel words; voxel lists: counts,
    # per-tile offsets of the chunk and voxel lists, lists 0-3 and the voxel
    # lists' bitmaps (include/pcfm.h)
    b, r = 2, 32
    v = r ** 3
    assert q("pcfm_conv3d_occupancy_bytes", b, r) == 4 * b * (v // 256 + v // 64 + v // 16)
    tiles = b * v // 256
    assert q("pcfm_conv3d_vlist_bytes", b, r) == 4 * (64 + 4 * tiles + 4 * b * v // 32 + 2 * b * v)
    assert q("pcfm_conv3d_vlist_bytes", b, 6) == 0  # r^3 % 256 != 0


def test_invalid_arguments_rejected_on_host():
    lib = _lib.load()
    rc = lib.pcfm_avg_voxelize_fwd(None, None, -1, 4, 10, 2, None, None, None, None, 0, None)
    assert rc == -1
    assert b"negative size" in lib.pcfm_last_error()
    rc = lib.pcfm_trilinear_devoxelize_fwd(None, None, 1, 4, 10, 0, 1, None, None, None, None)
    assert rc == -1 and b"resolution" in lib.pcfm_last_error()
    with pytest.raises(_lib.PcfmError, match="workspace"):
        _lib.call("pcfm_chamfer_fwd", None, None, 8, 20000, 20000, None, None, None, None, None,
                  0, None)


def test_pointwise_bnstats_request_on_a_path_without_statistics_fails(monkeypatch):
    """The forward GEMM's shape -> kernel choice is one function (pointwise.hip
    pw_path); the 256-row tiles (64-point groups) and the 128-row streaming form
    (32-point groups) write BatchNorm statistics, the 128 / 64-row tiles do not.
    A statistics request for a shape that takes such a kernel is refused on the
    host (nothing launched), instead of returning with the stats buffer
    unwritten."""
    lib = _lib.load()
    assert lib.pcfm_pointwise_bnstats_groups(8, 256, 256, 20000) == 8 * 313
    assert lib.pcfm_pointwise_bnstats_groups(8, 128, 128, 20000) == 8 * 625
    monkeypatch.setenv("PCFM_PW_STREAM_STATS", "0")  # the streaming form without its epilogue
    assert lib.pcfm_pointwise_bnstats_groups(8, 128, 128, 20000) == 0
    monkeypatch.delenv("PCFM_PW_STREAM_STATS")
    for shape in ((8, 100, 128, 20000),   # ragged K: the 128-row tile
                  (1, 256, 256, 512)):    # too few tiles for the 256-row tile
        assert lib.pcfm_pointwise_bnstats_groups(*shape) == 0
        rc = lib.pcfm_pointwise_gemm_bnstats(None, None, None, *shape, None, None, None)
        assert rc == -1, shape
        assert b"unsupported shape" in lib.pcfm_last_error()
