"""The NIF boundary on the CPU (OTP is absent here):

* the output-capacity protocol the NIF uses for emqx_match_batch / emqx_publish_batch
  (emqx_amd/csrc/nif/grow_retry.h), driven by tests/c/test_grow_retry.c: a PUBLISH to a topic
  with 10K subscribers overflows the first guess and is retried at the reported size
  (emqx_broker.erl:500-524 delivers to every subscriber);
* a -fsyntax-only type check of emqx_amd/csrc/nif/emqx_match_nif.c against the erl_nif
  declarations it uses (tests/c/erl_nif_decls, written from the erl_nif reference);
* the scheduler contract: every NIF that can wait on the device is registered DIRTY; the two
  per-PUBLISH NIFs on normal schedulers use only the batchers' try_submit and reschedule
  themselves onto a dirty scheduler when it says EMQX_EBUSY;
* every function INTEGRATION.md's emqx_match_nif module exports has a nif_funcs entry;
* the batchers themselves (emqx_amd/csrc/batcher.cpp) against a fake device
  (tests/c/test_batcher_busy.cpp): with every pinned buffer busy, try_submit returns
  EMQX_EBUSY without waiting, the blocking submit waits, and destroy never hangs."""

import os
import re
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


NIF_SRC = os.path.join(ROOT, "emqx_amd/csrc/nif/emqx_match_nif.c")


def nif_funcs():
    src = open(NIF_SRC).read()
    table = src[src.index("static ErlNifFunc nif_funcs[]"):]
    table = table[:table.index("};")]
    return {(m.group(1), int(m.group(2))): (m.group(3), m.group(4))
            for m in re.finditer(r'\{"(\w+)", (\d+), (\w+), ([\w]+)\}', table)}


def c_function_body(src, name):
    i = src.index("static ERL_NIF_TERM %s(" % name)
    j = src.index("{", i)
    depth = 0
    for k in range(j, len(src)):
        depth += {"{": 1, "}": -1}.get(src[k], 0)
        if depth == 0:
            return src[j:k + 1]
    raise AssertionError(name)


def test_nif_scheduler_contract():
    funcs = nif_funcs()
    normal = {name for (name, _), (_, flags) in funcs.items() if flags == "0"}
    assert normal == {"topic_match", "match_async", "publish_async"}, normal
    src = open(NIF_SRC).read()
    for name, helper, api in (("nif_match_async", "match_async_submit", "emqx_batcher"),
                              ("nif_publish_async", "publish_async_submit", "emqx_pub_batcher")):
        body = c_function_body(src, name)
        assert "%s(env, argv, 0, &busy)" % helper in body          # may_wait = 0 on the normal scheduler
        assert "enif_schedule_nif" in body and "ERL_NIF_DIRTY_JOB_CPU_BOUND" in body
        helper_body = c_function_body(src, helper)
        assert "%s_try_submit" % api in helper_body
        # the blocking submit only runs with may_wait set, i.e. in the dirty continuation
        assert re.search(r"may_wait \? %s_submit\(" % api, helper_body)
        dirty = c_function_body(src, name + "_dirty")
        assert "%s(env, argv, 1, &busy)" % helper in dirty
    # topic_match touches no device and takes no lock
    body = c_function_body(src, "nif_topic_match")
    assert "emqx_topic_match(" in body and "enif_get_resource" not in body


def test_integration_exports_are_bound():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"-export\(\[(.*?)\]\)\.", text, re.S)
    exports = {(n, int(a)) for n, a in re.findall(r"(\w+)/(\d+)", m.group(1))}
    # Erlang wrappers over the async NIFs
    wrappers = {("match", 2), ("publish", 3), ("subscribe", 3), ("route_add", 2), ("route_delete", 2)}
    funcs = set(nif_funcs())
    missing = sorted(exports - wrappers - funcs)
    assert not missing, missing
    # and every NIF has its Erlang stub in the module text
    for name, arity in funcs:
        args = ", ".join(["_"] * arity) if arity else ""
        assert re.search(r"\b%s\(%s\) -> erlang:nif_error\(not_loaded\)" % (name, r"[^)]*" if arity else ""), text), name


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_batcher_never_waits_when_busy(tmp_path):
    exe = tmp_path / "test_batcher_busy"
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror", "-pthread",
                    "-I", os.path.join(ROOT, "include"), "-o", str(exe),
                    os.path.join(ROOT, "tests/c/test_batcher_busy.cpp"),
                    os.path.join(ROOT, "emqx_amd/csrc/batcher.cpp")], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "ok"


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_commit_coalescer_group_commits(tmp_path):
    """emqx_amd/csrc/coalescer.cpp against a fake engine / subscription table: callbacks only after
    the commit that carries the change, group commit, routes before subscriptions, failures
    reported, destroy drains (tests/c/test_coalescer.cpp)."""
    exe = tmp_path / "test_coalescer"
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror", "-pthread",
                    "-I", os.path.join(ROOT, "include"), "-o", str(exe),
                    os.path.join(ROOT, "tests/c/test_coalescer.cpp"),
                    os.path.join(ROOT, "emqx_amd/csrc/coalescer.cpp")], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "ok"
