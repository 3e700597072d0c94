"""Host C++ under AddressSanitizer + UBSan (SURVEY §5 "Race detection / sanitizers").

`make -C renderformer_amd/csrc asan` (run by __graft_entry__.build()) compiles the library's pointer-heavy host
code -- capi.cpp (error words, range words, stream-K epoch table), stage.cpp (stage descriptor walkers) and
attn_sched.cpp (rf_attn_schedule) -- with -fsanitize=address,undefined on the host side only, links it with the
other objects into tests/host/host_asan.cpp's driver, and this test runs it on the CPU (no GPU needed: the
walkers run up to their first launch, which fails cleanly without a device).  Any sanitizer report aborts the
driver with a non-zero status."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "renderformer_amd", "csrc")
BIN = os.path.join(REPO, "build", "rfhip", "asan", "host_asan")


def _build():
    if not os.path.exists(BIN):
        r = subprocess.run(["make", "-C", CSRC, f"-j{min(8, os.cpu_count() or 8)}", "asan"], capture_output=True,
                           text=True, timeout=1500)
        if r.returncode != 0:
            pytest.fail(f"make asan failed:\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}")


def test_host_code_clean_under_asan_ubsan():
    _build()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=600, env=env)
    out = r.stdout + r.stderr
    print(out[-2000:])
    assert r.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out
    assert "host_asan: all checks passed" in r.stdout
