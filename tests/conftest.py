import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built librfhip.so")
    config.addinivalue_line("markers", "slow: long-running CPU case")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no HIP device visible")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


def needs_study(what: str) -> None:
    """Skip unless librfhip is the study build (rf_build_flags() & RF_BUILD_STUDY): the measured-slower kernels
    and ablation variants (4-wave GEMM / conv, one-wave-per-SIMD and legacy split-KV attention) are compiled only
    there (make -C renderformer_amd/csrc study; RF_LIB=renderformer_amd/lib/librfhip_study.so)."""
    from renderformer_amd import _lib
    if not _lib.study_build():
        pytest.skip(f"{what}: a study kernel, not in the production librfhip (RF_LIB=<librfhip_study.so> to test)")
