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
         "-Wno-unused-variable", "-I" + os.path.join(REPO, "include"), "-I" + CSRC]


def up_to_date() -> bool:
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and up_to_date():
        return OUT
    cmd = [HIPCC] + FLAGS + ["-o", OUT + ".tmp"] + SOURCES
    if verbose:
        print("[dmx.build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
