"""Host sanitizer job (CPU only): the GPU-free host code — the
E-step store planning (hmc_amd/csrc/plan.hpp), the HaploFile readers and
writers (hmc_amd/csrc/haplofile.cpp), hmc_resolve's option parser
(tools/hmc_options.hpp) and the CPU restatement (oracle/hmc_oracle.cpp) — built
with -fsanitize=address,undefined and run over small seeded inputs and
malformed files (tests/sanitize/san_main.cpp).  Any AddressSanitizer or
UndefinedBehaviorSanitizer report ends the run with a non-zero status."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = ["tests/sanitize/san_main.cpp", "hmc_amd/csrc/haplofile.cpp", "oracle/hmc_oracle.cpp"]


@pytest.mark.timeout(900)
def test_host_code_under_asan_ubsan(tmp_path):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    exe = str(tmp_path / "san_main")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-ffp-contract=off", "-pthread", "-o", exe] + SRCS
    subprocess.run(cmd, cwd=ROOT, check=True, capture_output=True, text=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, str(tmp_path)], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "sanitized host checks ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
