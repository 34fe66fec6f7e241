"""The library's host runtime under UBSan on the MI355X: a child pytest process loads
kubernetes_amd/libkschedgpu_ubsan.so (KSG_LIB; the same gfx950 kernels, ksg_runtime.cpp
built with -Xarch_host -fsanitize=undefined -fno-sanitize-recover=all by build()) and runs
the GPU parity, begin/commit, add/remove, queued-update and reflector-thread tests. The
first undefined operation on the host side (signed overflow in the mirror's int64
totals, a bad shift, a misaligned access) aborts the child."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_runtime_under_ubsan():
    lib = os.path.join(ROOT, "kubernetes_amd", "libkschedgpu_ubsan.so")
    assert os.path.exists(lib), "build() makes libkschedgpu_ubsan.so"
    sel = ("test_batch_matches_oracle and (700 or 900) or test_begin_commit or test_existing_pods "
           "or test_no_nodes or test_rejects_duplicate or test_updates_during or test_duplicate_and_unknown "
           "or test_reflector_thread_stress or test_rccl_one_rank")
    env = dict(os.environ, KSG_LIB="libkschedgpu_ubsan.so", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-m", "gpu", "-x", "-q", "-p", "no:cacheprovider",
                        "tests/test_gpu_parity.py", "tests/test_gpu_threads.py", "tests/test_gpu_sharded.py",
                        "-k", sel], cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "runtime error" not in out, out[-4000:]
    assert " passed" in out
    probe = subprocess.run([sys.executable, "-c", "from kubernetes_amd import abi; abi.load_library(); "
                            "print(any('ubsan_standalone' in l for l in open('/proc/self/maps')))"],
                           cwd=ROOT, env=env, capture_output=True, text=True, timeout=60)
    assert probe.stdout.strip() == "True", probe.stdout + probe.stderr
