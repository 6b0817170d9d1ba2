"""Build libsndvae.so (all HIP kernels + the C ABI) for gfx950 with hipcc.

In-tree build: the .so lands next to this file so it travels with the repo
snapshot to the GPU box (git-ignored, not gpurun-ignored).  Incremental:
objects are rebuilt when the content hash of their source, the headers or the
flags changes; the link records the source digest (``lib_status``).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import json
import os
import platform
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
ROOT = os.path.dirname(HERE)
INCLUDE = os.path.join(ROOT, "include")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libsndvae.so")
BUILD_INFO = os.path.join(HERE, "libsndvae.build.json")
ARCH = os.environ.get("SND_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", INCLUDE, "-I", CSRC,
         "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]


def _headers():
    return glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(os.path.join(INCLUDE, "*.h"))


def _digest(paths, extra=()):
    h = hashlib.sha256()
    for e in extra:                      # flags; the include paths differ per checkout
        h.update((os.path.relpath(e, ROOT) if os.path.isabs(e) else e).encode())
    for p in sorted(paths):
        h.update(os.path.basename(p).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def source_digest() -> str:
    """Content hash of every source and header the library is built from, plus the
    flags: what a built libsndvae.so must match (build_info)."""
    srcs = glob.glob(os.path.join(CSRC, "*.hip"))
    return _digest(srcs + _headers(), FLAGS + [ARCH])


# the compiler's per-kernel resource remarks (no effect on code generation): every
# kernel's VGPRs, spills and scratch are recorded beside its object and in BUILD_INFO,
# so a register spill in a shipped kernel is visible without a GPU (tests/test_host.py;
# round 5: a 72-VGPR spill in dec_bwd_kernel cost 26 us per C2 step unnoticed)
REMARKS = ["-Rpass-analysis=kernel-resource-usage"]
_RES_KEYS = {"VGPRs": "vgprs", "AGPRs": "agprs", "VGPRs Spill": "vgpr_spill",
             "SGPRs Spill": "sgpr_spill", "ScratchSize [bytes/lane]": "scratch",
             "Occupancy [waves/SIMD]": "occupancy", "LDS Size [bytes/block]": "lds"}


def parse_resources(text: str) -> dict:
    """{mangled kernel name: {vgprs, vgpr_spill, scratch, ...}} from hipcc's
    kernel-resource-usage remarks."""
    import re
    out, name = {}, None
    for line in text.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            name = m.group(1)
            out[name] = {}
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+(?:\[[^\]]*\])?): (\d+)", line)
        if m and name and m.group(1).strip() in _RES_KEYS:
            out[name][_RES_KEYS[m.group(1).strip()]] = int(m.group(2))
    return out


def _compile(src):
    """Staleness by content: an object is rebuilt when the hash of its source, the
    headers and the flags differs from the one recorded beside it (mtimes do not
    survive a snapshot copy to the GPU box)."""
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    want = _digest([src] + _headers(), FLAGS + [ARCH])
    stamp, res = obj + ".sha256", obj + ".res.json"
    if (os.path.exists(obj) and os.path.exists(stamp) and os.path.exists(res)
            and open(stamp).read() == want):
        return obj, False
    cmd = [HIPCC] + FLAGS + REMARKS + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    with open(res, "w") as f:
        json.dump(parse_resources(r.stderr), f)
    with open(stamp, "w") as f:
        f.write(want)
    return obj, True


def kernel_resources() -> dict:
    """Every kernel's resource record of the current objects (see REMARKS)."""
    out = {}
    for p in sorted(glob.glob(os.path.join(BUILD, "*.res.json"))):
        with open(p) as f:
            out.update(json.load(f))
    return out


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile what changed and link; records the source digest in BUILD_INFO."""
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    if force:
        for o in glob.glob(os.path.join(BUILD, "*.o*")):
            os.remove(o)
    jobs = min(len(srcs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16)
    with cf.ThreadPoolExecutor(jobs) as ex:
        res = list(ex.map(_compile, srcs))
    objs = [o for o, _ in res]
    digest = source_digest()
    recompiled = sum(1 for _, c in res if c)
    info = build_info()
    if force or recompiled or not os.path.exists(LIB) or info.get("source_sha256") != digest:
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        with open(LIB, "rb") as f:
            lib_sha = hashlib.sha256(f.read()).hexdigest()
        spills = {k: {"vgpr_spill": v.get("vgpr_spill", 0), "scratch": v.get("scratch", 0)}
                  for k, v in kernel_resources().items()
                  if v.get("vgpr_spill", 0) or v.get("scratch", 0)}
        with open(BUILD_INFO, "w") as f:
            json.dump({"source_sha256": digest, "lib_sha256": lib_sha,
                       "objects_recompiled": recompiled, "host": platform.node(),
                       "time": time.strftime("%Y-%m-%dT%H:%M:%S"), "spills": spills}, f)
    if verbose:
        print(LIB)
    return LIB


def build_info() -> dict:
    """The record of the last link (empty when there is none)."""
    try:
        with open(BUILD_INFO) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def lib_status() -> dict:
    """Is the library on disk the build of the sources on disk?  (bench.py reports
    this: the GPU box runs the prebuilt .so of the snapshot without building.)"""
    info = build_info()
    out = {"lib": os.path.relpath(LIB, ROOT), "built_on": info.get("host"), "built_at": info.get("time")}
    if os.path.exists(LIB):
        with open(LIB, "rb") as f:
            out["lib_sha16"] = hashlib.sha256(f.read()).hexdigest()[:16]
    out["matches_sources"] = (info.get("source_sha256") == source_digest()
                              and out.get("lib_sha16") == info.get("lib_sha256", "")[:16])
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
