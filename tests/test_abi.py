"""The C-ABI library loads and exports every symbol include/wx_align.h declares (CPU only:
no compute calls; argument validation paths return before any launch)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "wx_align.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(wx_[a-z_0-9]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    from whisperx_amd import _lib

    _lib.build()
    return _lib.load(require_device=False)


def test_header_lists_expected_entry_points():
    syms = declared_symbols()
    for s in ("wx_align_dp", "wx_trellis", "wx_backtrack", "wx_merge_repeats", "wx_binarize"):
        assert s in syms


def test_library_exports_every_declared_symbol(lib):
    from whisperx_amd import _lib

    for s in declared_symbols():
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, f"{s} not bound in _lib.SIGNATURES"


def test_version_and_errors(lib):
    assert b"gfx950" in lib.wx_version()
    assert lib.wx_strerror(0) == b"ok"
    assert b"workspace" in lib.wx_strerror(1004)


def test_workspace_queries_monotone(lib):
    a = lib.wx_align_dp_workspace_bytes(64, 64 * 1499, 500)
    b = lib.wx_align_dp_workspace_bytes(128, 128 * 1499, 500)
    assert 0 < a < b
    assert lib.wx_backtrack_workspace_bytes(4, 4000, 900) > 0


def test_argument_validation_without_device(lib):
    # S < 0 and oversized vocab/tokens are rejected before anything touches the device
    assert lib.wx_align_dp(None, None, 32, None, None, None, -1, 0, 0, 0, None, None, None, None, None,
                           None, 0, None) == 1001
    assert lib.wx_align_dp(None, None, 32, None, None, None, 0, 0, 0, 0, None, None, None, None, None,
                           None, 0, None) == 0
    dummy = ctypes.c_void_p(8)
    assert lib.wx_align_dp(dummy, dummy, 20000, dummy, dummy, dummy, 1, 1, 1, 10, dummy, dummy, dummy, dummy,
                           dummy, dummy, 1 << 30, None) == 1002
    assert lib.wx_align_dp(dummy, dummy, 32, dummy, dummy, dummy, 1, 1, 20000, 10, dummy, dummy, dummy, dummy,
                           dummy, dummy, 1 << 30, None) == 1003
    assert lib.wx_align_dp(dummy, dummy, 32, dummy, dummy, dummy, 1, 1, 10, 10, dummy, dummy, dummy, dummy,
                           dummy, dummy, 16, None) == 1004
    assert lib.wx_align_dp_mode(dummy, dummy, 32, dummy, dummy, dummy, 1, 1, 10, 10, dummy, dummy, dummy, dummy,
                                dummy, dummy, 1 << 30, 7, None) == 1001  # unknown launch shape
    assert lib.wx_binarize(None, None, -1, None, None, None, 0.5, 0.3, 1.0, 0.0, 0.0, None, None, None, None,
                           None) == 1001
    ws = lib.wx_binarize_workspace_bytes(3, 213334)
    assert ws >= 24 * (213334 // 64 + 4)
    assert lib.wx_binarize_ex(dummy, dummy, 3, 213334, dummy, dummy, dummy, 0.5, 0.3, 30.0, 0.0, 0.0, dummy, dummy,
                              dummy, dummy, dummy, ws - 1, None) == 1004
    assert lib.wx_binarize_ex(None, None, -1, 0, None, None, None, 0.5, 0.3, 1.0, 0.0, 0.0, None, None, None, None,
                              None, 0, None) == 1001


def test_launch_plan_bucket_selection(lib):
    """Host-side launch planning (wx_align_dp_plan, no device work): the kernels a batch maps
    to in each launch shape."""
    from whisperx_amd import _lib

    k = "void wx::align_dp_kernel<{}>(wx::AlignArgs)".format
    sk = "void wx::align_dp_split_kernel<{}>(wx::AlignArgs)".format
    # config 2 (64 x 30 s, N 300..500): one latency launch, each segment over 4 CUs (the
    # planner assumes 256 CUs without a device); 128 segments: one CU per segment
    assert _lib.align_dp_plan(64, 300, 500, 32) == [sk("1, 32, 4")]
    assert _lib.align_dp_plan(128, 300, 500, 32) == [k("2, 32, 7, 1")]
    assert _lib.align_dp_plan(64, 300, 500, 32, _lib.MODE_LATENCY) == [k("2, 32, 7, 1")]
    assert _lib.align_dp_plan(64, 300, 500, 32, _lib.MODE_LATENCY_1CU) == [k("2, 32, 7, 1")]
    # split over 4 CUs: one split kernel for the whole batch (the bucket of its longest segment)
    assert _lib.align_dp_plan(64, 300, 500, 32, _lib.MODE_SPLIT4) == [sk("1, 32, 4")]
    assert _lib.align_dp_plan(64, 300, 1100, 32, _lib.MODE_SPLIT4) == [sk("2, 32, 3")]
    # ... short segments a wide split bucket cannot lay out take throughput buckets beside it
    assert _lib.align_dp_plan(64, 1, 2000, 32, _lib.MODE_SPLIT4) == [sk("4, 32, 3"), k("1, 32, 1, 0")]
    # saturated batches: throughput buckets by N; V picks the LDS row width (32 / 64 / gather)
    assert _lib.align_dp_plan(4096, 300, 500, 32) == [k("6, 32, 1, 0"), k("8, 32, 1, 0")]
    assert _lib.align_dp_plan(2048, 850, 951, 40) == [k("8, 64, 2, 0")]
    assert _lib.align_dp_plan(2048, 850, 951, 1000) == [k("8, 256, 2, 0")]
    assert _lib.align_dp_plan(0, 1, 1, 32) == []


def test_product_refuses_without_device():
    import torch

    from whisperx_amd import _lib

    if torch.cuda.is_available():
        pytest.skip("a device is visible")
    with pytest.raises(_lib.WXError):
        _lib.load(require_device=True)


def test_binarize_plan_kernel_selection(lib):
    """wx_binarize_plan (no device work): offset <= onset takes the parallel scan, offset >
    onset (vad.py:146-175: a frame may both set and reset) the event-jumping state machine."""
    from whisperx_amd import _lib

    words = "void wx::binarize_words_kernel(wx::BinWordArgs)"
    scan = "void wx::binarize_scan_kernel(wx::BinScanArgs)"
    fsm = "void wx::binarize_fsm_kernel(wx::BinarizeArgs, wx::BinWords)"
    assert _lib.binarize_plan(0.5, 0.363, 1000) == [words, scan]
    assert _lib.binarize_plan(0.5, 0.5, 1000) == [words, scan]
    assert _lib.binarize_plan(0.4, 0.6, 1000) == [words, fsm]
    assert _lib.binarize_plan(0.5, 0.55, 0) == [fsm]
