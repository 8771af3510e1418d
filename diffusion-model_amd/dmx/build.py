"""Build libdmx.so in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libdmx.so")
SOURCES = [os.path.join(CSRC, "engine.hip")]
DEPS = SOURCES + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")] + \
    [os.path.join(REPO, "include", "dmx.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wno-unused-function",
         "-Wno-unused-variable", "-I" + os.path.join(REPO, "include"), "-I" + CSRC,
         # MFMA accumulators in ArchVGPRs (gfx950's unified register file): no v_accvgpr_read/write
         # round trips where VALU touches accumulators (softmax, epilogues); measured +2 % per step
         "-mllvm", "-amdgpu-mfma-vgpr-form=1"]


def up_to_date() -> bool:
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def build(force: bool = False, verbose: bool = True, out: str = OUT, extra=()) -> str:
    if not force and out == OUT and up_to_date():
        return OUT
    cmd = [HIPCC] + FLAGS + list(extra) + ["-o", out + ".tmp"] + SOURCES
    if verbose:
        print("[dmx.build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    # python build.py [--force] [--out NAME.so] [-- extra hipcc flags]   (NAME.so lands next to libdmx.so)
    argv = sys.argv[1:]
    extra = argv[argv.index("--") + 1:] if "--" in argv else []
    argv = argv[:argv.index("--")] if "--" in argv else argv
    out = os.path.join(HERE, argv[argv.index("--out") + 1]) if "--out" in argv else OUT
    build(force="--force" in argv or out != OUT, out=out, extra=extra)
