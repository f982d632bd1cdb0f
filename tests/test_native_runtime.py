"""C++ unit tests of the runtime core (csrc/tests/test_runtime.cpp), built plain,
with AddressSanitizer + UBSan, and with ThreadSanitizer (race
detection on host code; GPU sanitizers are not used)."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SRCS = [ROOT / "csrc/tests/test_runtime.cpp"] + [ROOT / f"csrc/runtime/{n}.cpp" for n in
                                                  ("kv_blocks", "scheduler", "router", "validator", "shm_channel")]

VARIANTS = {
    "plain": ["-O2"],
    "asan_ubsan": ["-O1", "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"],
    "tsan": ["-O1", "-fsanitize=thread"],
}


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("variant", list(VARIANTS))
def test_runtime_unit_binary(tmp_path, variant):
    exe = tmp_path / f"t_{variant}"
    cmd = ["g++", "-std=c++17", "-g", *VARIANTS[variant], f"-I{ROOT / 'csrc/runtime'}", *map(str, SRCS),
           "-o", str(exe), "-lpthread", "-lrt"]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "checks passed" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
