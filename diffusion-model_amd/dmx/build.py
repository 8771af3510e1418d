"""Build libdmx.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

engine.hip (host orchestration, C ABI, small kernels) and the k_*.hip translation units (one
per templated kernel family, see csrc/launch.h) compile in parallel to objects under
dmx/build/, then link into dmx/libdmx.so."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libdmx.so")
OBJ = os.path.join(HERE, "build")
SOURCES = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))
HEADERS = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")] + \
    [os.path.join(REPO, "include", "dmx.h")]
DEPS = SOURCES + HEADERS
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
         "-Wno-unused-variable", "-I" + os.path.join(REPO, "include"), "-I" + CSRC,
         # MFMA accumulators in ArchVGPRs (gfx950's unified register file): no v_accvgpr_read/write
         # round trips where VALU touches accumulators (softmax, epilogues); measured +2 % per step
         "-mllvm", "-amdgpu-mfma-vgpr-form=1"]


# Per-translation-unit flags.  The attention cores keep their softmax in scalar f32 VALU: the
# SLP vectoriser would pack it into v_pk_add / v_pk_mul_f32, whose issue cost beside MFMAs is
# far above that of the two scalar halves (MI355X_MICROARCH.md, constants table).
# No NaN semantics there either: fmaxf needs no canonicalising v_max x, x, x per operand (the
# scores are finite or the -inf of a masked key).
FILE_FLAGS = {"k_attn.hip": ["-fno-slp-vectorize", "-fno-honor-nans"]}


def _newest_header() -> float:
    return max(os.path.getmtime(h) for h in HEADERS)


def up_to_date() -> bool:
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def build(force: bool = False, verbose: bool = True, out: str = OUT, extra=(), jobs: int = 0) -> str:
    if not force and out == OUT and up_to_date():
        return OUT
    os.makedirs(OBJ, exist_ok=True)
    tag = "" if out == OUT else "." + os.path.basename(out).replace(".so", "")
    hdr = _newest_header()
    todo, objs = [], []
    for src in SOURCES:
        obj = os.path.join(OBJ, os.path.basename(src).replace(".hip", tag + ".o"))
        objs.append(obj)
        if force or extra or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), hdr):
            todo.append((src, obj))
    jobs = jobs or min(len(todo) or 1, max(1, int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    running = []
    for src, obj in todo:
        cmd = [HIPCC] + FLAGS + FILE_FLAGS.get(os.path.basename(src), []) + list(extra) + \
            ["-c", "-o", obj + ".tmp", src]
        if verbose:
            print("[dmx.build]", os.path.basename(src), flush=True)
        running.append((subprocess.Popen(cmd), obj))
        if len(running) >= jobs:
            _wait(running.pop(0))
    for r in running:
        _wait(r)
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out + ".tmp"] + objs
    if verbose:
        print("[dmx.build] link", os.path.basename(out), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def _wait(r):
    proc, obj = r
    if proc.wait() != 0:
        raise subprocess.CalledProcessError(proc.returncode, proc.args)
    os.replace(obj + ".tmp", obj)


if __name__ == "__main__":
    # python build.py [--force] [--out NAME.so] [-- extra hipcc flags]   (NAME.so lands next to libdmx.so)
    argv = sys.argv[1:]
    extra = argv[argv.index("--") + 1:] if "--" in argv else []
    argv = argv[:argv.index("--")] if "--" in argv else argv
    out = os.path.join(HERE, argv[argv.index("--out") + 1]) if "--out" in argv else OUT
    build(force="--force" in argv or out != OUT, out=out, extra=extra)
