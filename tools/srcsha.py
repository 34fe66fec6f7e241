"""The sha256 (first 16 hex digits) of the sources the HIP library is built from
(kubernetes_amd/csrc/*.hip, *.h, *.cpp and include/kschedgpu.h, by name order): the
build tag that profiles/traffic.json entries carry, so bench.py uses counter-measured
bytes only for the build they were measured on."""
import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_src_sha(root: str = ROOT) -> str:
    files = sorted(glob.glob(os.path.join(root, "kubernetes_amd", "csrc", "*.hip")) +
                   glob.glob(os.path.join(root, "kubernetes_amd", "csrc", "*.h")) +
                   glob.glob(os.path.join(root, "kubernetes_amd", "csrc", "*.cpp")) +
                   [os.path.join(root, "include", "kschedgpu.h")])
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(kernel_src_sha())
