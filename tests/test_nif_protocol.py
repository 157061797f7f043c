"""The NIF boundary on the CPU (OTP is absent here):

* the output-capacity protocol the NIF uses for emqx_match_batch / emqx_publish_batch
  (emqx_amd/csrc/nif/grow_retry.h), driven by tests/c/test_grow_retry.c: a PUBLISH to a topic
  with 10K subscribers overflows the first guess and is retried at the reported size
  (emqx_broker.erl:500-524 delivers to every subscriber);
* a -fsyntax-only type check of emqx_amd/csrc/nif/emqx_match_nif.c against the erl_nif
  declarations it uses (tests/c/erl_nif_decls, written from the erl_nif reference)."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GCC = shutil.which("gcc")


@pytest.mark.skipif(GCC is None, reason="no gcc")
def test_grow_retry_protocol(tmp_path):
    exe = tmp_path / "test_grow_retry"
    subprocess.run([GCC, "-std=c99", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "emqx_amd/csrc/nif"),
                    "-o", str(exe), os.path.join(ROOT, "tests/c/test_grow_retry.c")], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "ok"


@pytest.mark.skipif(GCC is None, reason="no gcc")
def test_nif_type_checks():
    r = subprocess.run([GCC, "-std=c99", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter", "-fsyntax-only",
                        "-I", os.path.join(ROOT, "tests/c/erl_nif_decls"),
                        os.path.join(ROOT, "emqx_amd/csrc/nif/emqx_match_nif.c")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
