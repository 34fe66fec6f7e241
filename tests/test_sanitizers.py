"""Sanitizer runs of the CPU-side native code (SURVEY.md §5 "Race detection / sanitizers").

* The C restatement (oracle/) under UBSan (-fno-sanitize-recover: the first undefined
  operation aborts; signed overflow matters because the reference's Go int64
  arithmetic wraps and the C must do it unsigned) and under ASan (LD_PRELOAD of gcc's
  runtime), through the golden-vector, engine and cross-check suites.
* The library's host runtime (kubernetes_amd/csrc/ksg_runtime.cpp) built with
  `-Xarch_host -fsanitize=undefined` into libkschedgpu_ubsan.so (GPU code unchanged),
  loaded through KSG_LIB by the -m gpu run in tests/test_gpu_ubsan_runtime.py.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SUITES = ["tests/test_oracle_golden.py", "tests/test_golden_engines.py", "tests/test_oracle_crosscheck.py"]


def _run_suite(env_extra):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, "-m", "pytest", *SUITES, "-m", "not gpu", "-q", "-x", "-p",
                        "no:cacheprovider"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr, tail
    return tail


@pytest.fixture(scope="module")
def san_libs():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitizers"], check=True)
    return os.path.join(ROOT, "oracle", "_build")


def test_oracle_under_ubsan(san_libs):
    out = _run_suite({"KSG_ORACLE_LIB": os.path.join(san_libs, "liboracle_ubsan.so")})
    assert "passed" in out


def test_oracle_under_asan(san_libs):
    asan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.isabs(asan) or not os.path.exists(asan):
        pytest.skip("gcc's libasan.so is not installed")
    out = _run_suite({"KSG_ORACLE_LIB": os.path.join(san_libs, "liboracle_asan.so"), "LD_PRELOAD": asan,
                      "ASAN_OPTIONS": "detect_leaks=0"})
    assert "passed" in out
