"""The C-ABI library loads on a machine without a GPU, exports every entry point
include/dsp_audiorec.h declares, and rejects bad arguments on the host before any launch."""
import ctypes
import os
import re

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "dsp_audiorec.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:size_t|int)\s+(dsp_\w+)\s*\(", src, flags=re.M)))


@pytest.fixture(scope="module")
def lib():
    from src import _hip
    return _hip.load_library()


def test_header_declares_the_path():
    names = declared_functions()
    assert {"dsp_extract_features", "dsp_extract_lds_bytes", "dsp_knn_classify",
            "dsp_knn_workspace_bytes", "dsp_extract_general", "dsp_extract_general_workspace_bytes", "dsp_zscore_fit", "dsp_zscore_apply", "dsp_abi_version"} <= set(names)


def test_every_declared_symbol_is_exported(lib):
    from src import _hip
    for name in declared_functions():
        assert hasattr(lib, name), name
        assert name in _hip.EXPORTS, "binding does not type %s" % name


def test_abi_version(lib):
    m = re.search(r"#define DSP_ABI_VERSION (\d+)", open(HEADER).read())
    assert lib.dsp_abi_version() == int(m.group(1))


def test_lds_sizing(lib):
    assert lib.dsp_extract_lds_bytes(44100, 1102, 441) > 0
    assert lib.dsp_extract_lds_bytes(44100, 1024, 512) > 0
    assert lib.dsp_extract_lds_bytes(44100, 1102, 441) <= 80 * 1024  # two workgroups per CU
    assert 0 < lib.dsp_extract_lds_bytes(200000, 1102, 441) <= 160 * 1024  # 4.5 s: summaries only
    assert lib.dsp_extract_lds_bytes(400000, 1102, 441) == 0  # beyond one CU's LDS
    assert lib.dsp_extract_lds_bytes(0, 1102, 441) == 0
    assert lib.dsp_extract_lds_bytes(44100, 0, 441) == 0


def test_host_argument_checks(lib):
    """Argument errors are returned before anything touches the device."""
    from src import _hip
    f = lib.dsp_extract_features
    buf = ctypes.create_string_buffer(64)
    p = ctypes.cast(buf, ctypes.c_void_p)
    p2 = ctypes.c_void_p(p.value + 2)  # misaligned pcm
    args = lambda pcm, B, L=1102, S=441, feat=p, q=None, os_=0: (pcm, p, B, 44100, L, S, p, 1, 0.5, 0.1, 1.5,
                                                                 feat, p, p, p, os_, None, None, 0, None, 0, q, None)
    assert f(*args(p, -1)) == _hip.DSP_ERR_ARGS
    assert f(*args(p, 4, feat=None)) == _hip.DSP_ERR_ARGS
    assert f(*args(p2, 4)) == _hip.DSP_ERR_ARGS
    assert f(*args(p, 4, L=0)) == _hip.DSP_ERR_ARGS
    assert f(*args(p, 4, q=p2)) == _hip.DSP_ERR_ARGS  # misaligned clip-queue scratch
    assert f(*args(p, 4, os_=18)) == _hip.DSP_ERR_ARGS  # a result row needs DSP_OUT_ROW_WORDS words
    assert f(*args(p, 0, os_=19)) == _hip.DSP_OK
    assert f(*args(p, 0)) == _hip.DSP_OK  # empty batch: nothing to launch
    assert lib.dsp_knn_workspace_bytes(100, 100, 4097, 5) == 0
    assert lib.dsp_knn_workspace_bytes(100, 100, 33, 5) > 0  # high-dimensional screen
    assert lib.dsp_knn_workspace_bytes(100, 100, 15, 33) == 0
    assert lib.dsp_knn_workspace_bytes(100, 100, 15, 5) > 0
    k = lib.dsp_knn_classify
    assert k(p, p, 100, p, 10, 0, 3, -1, 0, p, p, p, p, 1 << 20, 0, None) == _hip.DSP_ERR_ARGS
    assert k(p, p, 100, p, 10, 15, 3, -1, 0, p, p, p, None, 0, 0, None) == _hip.DSP_ERR_WORKSPACE
    assert k(p, p, 100, p, 0, 15, 3, -1, 0, None, None, None, None, 0, 0, None) == _hip.DSP_OK
    assert lib.dsp_zscore_fit(None, 10, 15, p, p, None) == _hip.DSP_ERR_ARGS
    g = lib.dsp_extract_general
    gargs = lambda sb=2, ws=None, nws=0, n=4: (p, sb, p, None, n, 0, 44100, 1102, 441, p, 1, 0.5, 0.1, 1.5,
                                              p, p, p, p, 0, None, None, 0, None, 0, ws, nws, None)
    assert g(*gargs(sb=3)) == _hip.DSP_ERR_ARGS
    assert g(*gargs()) == _hip.DSP_ERR_WORKSPACE
    assert g(*gargs(n=0)) == _hip.DSP_OK
    one = lib.dsp_extract_general_workspace_bytes(1, 44100, 1102, 441)
    assert one > 0 and lib.dsp_extract_general_workspace_bytes(3, 44100, 1102, 441) == 3 * one
    assert lib.dsp_extract_general_workspace_bytes(1, 30 * 44100, 1102, 441) > 20 * one
    assert lib.dsp_zscore_apply(p, 0, 15, p, p, p, None) == _hip.DSP_OK


def test_no_cpu_fallback():
    """Without a HIP device the product path raises instead of computing on the host."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from src import _hip
    from src.pipeline import FeatureExtractor, knn_classify, zscore_fit
    with pytest.raises(_hip.HipError):
        FeatureExtractor(1102, 441)
    with pytest.raises(_hip.HipError):
        knn_classify([[0.0]], [0], [[0.0]], 1)
    with pytest.raises(_hip.HipError):
        zscore_fit([[0.0]])
