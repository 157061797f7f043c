"""The host worker pool of the subscriber tables (emqx_amd/csrc/workpool.h), built and run on
the CPU (tests/c/test_workpool.cpp): every run executes its job on exactly t threads, with and
without the spin window, and concurrent callers are serialised; once more under ThreadSanitizer."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GXX = shutil.which("g++")


@pytest.mark.skipif(GXX is None, reason="no g++")
@pytest.mark.parametrize("sanitize", [False, True])
def test_workpool(tmp_path, sanitize):
    exe = tmp_path / "test_workpool"
    cmd = [GXX, "-std=c++17", "-O1" if sanitize else "-O2", "-Wall", "-Wextra", "-Werror", "-pthread", "-o", str(exe),
           os.path.join(ROOT, "tests/c/test_workpool.cpp")]
    if sanitize:
        cmd[4:4] = ["-fsanitize=thread", "-g"]
    subprocess.run(cmd, check=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "workpool ok" in out.stdout
