"""SURVEY.md §5 sanitizers: the CPU oracle (gcc) and librtamd's host code
(rt_abi.cpp + scene_io.cpp, clang with -Xarch_host) built with AddressSanitizer
+ UndefinedBehaviorSanitizer (`make -C tests/c sanitize`) and driven by two C
programs: tests/c/oracle_san.c (every oracle function over small and
degenerate scenes) and tests/c/rt_san.c (ingest, OBJ edge cases and malformed
files, RTSOUP1, camera, knobs, dumps, and -- without a GPU -- the RT_EDEVICE
refusal of every compute entry point).  Any sanitizer report aborts the
program, so exit status 0 means clean.  Host-only: no GPU needed."""
import os
import subprocess

import pytest

from conftest import ROOT

CDIR = os.path.join(ROOT, "tests", "c")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


@pytest.fixture(scope="module")
def built():
    r = subprocess.run(["make", "-C", CDIR, "sanitize"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return os.path.join(CDIR, "build", "asan")


def test_oracle_under_asan_ubsan(built):
    r = subprocess.run([os.path.join(built, "oracle_san")], capture_output=True, text=True, timeout=300, env=ENV)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "oracle_san OK" in r.stdout


def test_library_host_code_under_asan_ubsan(built, tmp_path):
    r = subprocess.run([os.path.join(built, "rt_san"), str(tmp_path)], capture_output=True, text=True,
                       timeout=300, env=ENV)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "rt_san OK" in r.stdout
