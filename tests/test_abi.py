"""The drop-in boundary without a GPU: libkschedgpu.so loads, exports every entry point
include/kschedgpu.h declares, and the ctypes/numpy mirrors match the C struct layouts
(checked by compiling the header with gcc). No compute call is made here."""
import ctypes as C
import os
import re
import subprocess

import pytest

from kubernetes_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "kschedgpu.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^[A-Za-z_][\w \*]*?\b(ksg_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_abi():
    d = _declared()
    assert "ksg_schedule_begin" in d and "ksg_schedule_batch" in d
    assert sorted(abi.EXPORTS) == d


def test_library_exports_every_declared_symbol():
    path = abi.lib_path()
    assert os.path.exists(path), "build() must produce the in-tree library"
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if l.strip()}
    missing = [s for s in _declared() if s not in exported]
    assert not missing, missing
    lib = abi.load_library()  # dlopen + signatures; no HIP call is made
    for s in _declared():
        assert getattr(lib, s) is not None


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(abi, "_lib", None)
    monkeypatch.setattr(abi, "lib_path", lambda: str(tmp_path / "nope.so"))
    with pytest.raises(RuntimeError, match="missing"):
        abi.load_library()


STRUCTS = (("ksg_config", abi.KsgConfig), ("ksg_node", abi.KsgNode), ("ksg_pod", abi.KsgPod),
           ("ksg_shard_record", abi.KsgShardRecord), ("ksg_admission_set", abi.KsgAdmissionSet))

_LAYOUT_C = r"""
#include <stdio.h>
#include <stddef.h>
#include "kschedgpu.h"
#define P(T, f) printf(#T "." #f " %zu\n", offsetof(T, f));
int main(void) {
  printf("ksg_config %zu\nksg_node %zu\nksg_pod %zu\nksg_shard_record %zu\nksg_admission_set %zu\n",
         sizeof(ksg_config), sizeof(ksg_node), sizeof(ksg_pod), sizeof(ksg_shard_record), sizeof(ksg_admission_set));
  %FIELDS%
  return 0;
}
"""


def test_struct_layouts_match_header(tmp_path):
    fields = []
    for T, cls in STRUCTS:
        for name, _ in cls._fields_:
            fields.append(f"P({T}, {name})")
    src = tmp_path / "layout.c"
    src.write_text(_LAYOUT_C.replace("%FIELDS%", "\n  ".join(fields)))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                          check=True).stdout.splitlines())
    assert int(got["ksg_config"]) == C.sizeof(abi.KsgConfig)
    assert int(got["ksg_node"]) == C.sizeof(abi.KsgNode) == abi.NODE_DTYPE.itemsize
    assert int(got["ksg_pod"]) == C.sizeof(abi.KsgPod) == abi.POD_DTYPE.itemsize
    for T, cls in STRUCTS:
        assert int(got[T]) == C.sizeof(cls), T
        for name, _ in cls._fields_:
            assert int(got[f"{T}.{name}"]) == getattr(cls, name).offset, (T, name)
    for name in abi.POD_DTYPE.names:
        assert abi.POD_DTYPE.fields[name][1] == getattr(abi.KsgPod, name).offset


def test_product_never_imports_the_oracle():
    """The oracle is test infrastructure: nothing under kubernetes_amd/ may reference it."""
    pkg = os.path.join(ROOT, "kubernetes_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                txt = open(os.path.join(dp, f), encoding="utf-8").read()
                assert not re.search(r"^\s*(from|import)\s+oracle\b", txt, flags=re.M), f
                assert "liboracle" not in txt and "ksg_oracle" not in txt, f


# entry points that fill a fixed number of caller-allocated words: the width is in the
# parameter's name (or, for the debug counters, an explicit length argument), and the
# Python wrapper allocates exactly that many (VERDICT round 4 "silent ABI widening")
_WIDTHS = {"ksg_last_batch_stats": ("stats4", 4), "ksg_last_batch_kernel_ms": ("out3", 3),
           "ksg_last_batch_host_us": ("out8", 8), "ksg_batch_totals": ("out24", 24), "ksg_serve_stats": ("out4", 4)}

_PROTO_C = r"""
#include <stdint.h>
#include "kschedgpu.h"
int (*p_dbg)(ksg_ctx*, int32_t*, uint32_t) = ksg_debug_counters;
int (*p_stats)(ksg_ctx*, uint32_t*) = ksg_last_batch_stats;
int (*p_kms)(ksg_ctx*, double*) = ksg_last_batch_kernel_ms;
int (*p_hus)(ksg_ctx*, double*) = ksg_last_batch_host_us;
int (*p_tot)(ksg_ctx*, double*) = ksg_batch_totals;
int (*p_srv)(ksg_ctx*, uint64_t*) = ksg_serve_stats;
_Static_assert(KSG_DEBUG_COUNTER_WORDS == %WORDS%, "debug counter width");
_Static_assert(KSG_ABI_VERSION == 3, "ABI version");
int main(void) { return 0; }
"""


def test_fixed_width_outputs_are_pinned(tmp_path):
    src = open(HEADER).read()
    for fn, (param, n) in _WIDTHS.items():
        m = re.search(r"\b%s\s*\(([^)]*)\)" % fn, src)
        assert m and re.search(r"\b%s\b" % param, m.group(1)), (fn, param)
    # the debug counters take their length: an old two-argument caller no longer compiles
    m = re.search(r"\bksg_debug_counters\s*\(([^)]*)\)", src)
    assert m and "n_words" in m.group(1)
    c = tmp_path / "proto.c"
    c.write_text(_PROTO_C.replace("%WORDS%", str(abi.KSG_DEBUG_COUNTER_WORDS)))
    subprocess.run(["gcc", "-std=c11", "-Werror", "-Wall", "-c", "-I", os.path.join(ROOT, "include"), str(c), "-o",
                    str(tmp_path / "proto.o")], check=True)
    old = tmp_path / "old.c"
    old.write_text('#include "kschedgpu.h"\nint f(ksg_ctx* c, int32_t* o) { return ksg_debug_counters(c, o); }\n')
    r = subprocess.run(["gcc", "-std=c11", "-c", "-I", os.path.join(ROOT, "include"), str(old), "-o",
                        str(tmp_path / "old.o")], capture_output=True, text=True)
    assert r.returncode != 0 and "few arguments" in r.stderr
    # the Python wrappers allocate the declared widths
    eng = open(os.path.join(ROOT, "kubernetes_amd", "engine.py")).read()
    for fn, (_, n) in _WIDTHS.items():
        body = eng[:eng.index("self._lib.%s(" % fn)]
        alloc = re.findall(r"np\.zeros\((\d+),", body[-400:])
        assert alloc and int(alloc[-1]) == n, (fn, alloc)
    assert list(abi.load_library().ksg_debug_counters.argtypes)[2] is abi.U32
