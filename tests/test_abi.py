"""The C-ABI library loads and exports every symbol include/rf.h declares (no GPU needed)."""
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    text = open(os.path.join(REPO, "include", "rf.h")).read()
    return sorted(set(re.findall(r"^(?:int|int64_t|const char\*)\s+(rf_\w+)\(", text, flags=re.M)))


def test_header_lists_entry_points():
    fns = header_functions()
    assert "rf_gemm_bf16" in fns and "rf_attn_fwd" in fns and len(fns) >= 14


def test_library_exports_every_header_symbol():
    import torch  # noqa: F401
    from renderformer_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("librfhip.so not built (run __graft_entry__.build())")
    lib = _lib.load(require_device=False)
    for fn in header_functions():
        assert hasattr(lib, fn), fn
    assert lib.rf_abi_version() == 8
    # every int-returning entry point has a ctypes signature in the binding
    assert set(_lib.SIGNATURES) == set(header_functions()) - {"rf_last_error", "rf_abi_version",
                                                               "rf_attn_workspace_bytes", "rf_gemm_workspace_bytes",
                                                               "rf_scene_pos_partials"}


def test_invalid_arguments_raise_value_error_without_device():
    """Argument validation happens before any launch, so it is testable on CPU."""
    import ctypes
    import torch  # noqa: F401
    from renderformer_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("librfhip.so not built")
    lib = _lib.load(require_device=False)
    rc = lib.rf_gemm_bf16(ctypes.c_void_p(16), 64, ctypes.c_void_p(16), 64, ctypes.c_void_p(16), 128, None,
                          10, 100, 64, 0, None, 0, None)  # N % 128 != 0
    assert rc == 1 and b"multiple of 128" in lib.rf_last_error()
    rc = lib.rf_attn_fwd(ctypes.c_void_p(16), 256, ctypes.c_void_p(16), 256, ctypes.c_void_p(16), 256,
                         ctypes.c_void_p(16), 256, ctypes.c_void_p(16), 1, 10, 2, 64, 1.0, 1, None, 0, None)
    assert rc == 1 and b"head_dim" in lib.rf_last_error()


@pytest.mark.gpu
def test_device_error_word_surfaces_on_next_call():
    """A device-side error (here raised on purpose by a debug kernel; in production a stream-K owner whose
    partner never published) makes the next entry point fail loudly, without a device sync, until cleared."""
    import torch
    from renderformer_amd import _lib, ops
    lib = _lib.load()
    assert lib.rf_device_error() == 0
    _lib.call("rf_debug_raise_device_error", 7, _lib.stream())
    torch.cuda.synchronize()
    assert lib.rf_device_error() == 7
    x = torch.randn(4, 256, device="cuda")
    out = torch.empty(4, 256, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(_lib.DeviceError, match="device error 7"):
        ops.rmsnorm(x, torch.ones(256, device="cuda"), 1e-6, out)
    lib.rf_clear_device_error()
    ops.rmsnorm(x, torch.ones(256, device="cuda"), 1e-6, out)  # clean again


@pytest.mark.gpu
def test_kernel_timer_times_the_tagged_launch():
    """rf_ktimer_arm + a tagged op: exactly the tagged launch is timed (dispatch-packet events), its duration is
    positive and no longer than a marker-event bracket around the same launch."""
    import torch
    from renderformer_amd import ops
    a = torch.randn(4096, 1024, device="cuda").bfloat16()
    w = torch.randn(8192, 1024, device="cuda").bfloat16()
    out = torch.empty(4096, 8192, device="cuda", dtype=torch.bfloat16)
    ops.gemm(a, w, out)  # warm
    t = ops.KernelTimer("timed")
    ops.TIMER = t
    try:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.gemm(a, w, out, tag="timed")
        e1.record()
        ops.gemm(a, w, out, tag="other")  # not timed
        ops.gemm(a, w, out, tag="timed")
    finally:
        ops.TIMER = None
    d = t.durations_ms()
    torch.cuda.synchronize()
    assert len(d) == 2 and all(x > 0 for x in d), d
    assert d[0] <= e0.elapsed_time(e1) + 1e-3
    assert t.durations_ms() == []  # pairs released
