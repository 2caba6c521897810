"""Build libsentinel_amd.so for gfx950 in-tree with hipcc (no JIT cache, travels with the repo)."""
from __future__ import annotations

import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(_HERE)
SOURCES = [os.path.join(_HERE, "csrc", "engine.hip")]
DEPS = SOURCES + [os.path.join(_HERE, "csrc", f) for f in ("common.hpp", "scan_sort.hpp", "admission.hpp", "param_rules.hpp", "concurrent.hpp", "partition.hpp", "small.hpp", "param_part.hpp", "wire_server.hpp", "local_entry.hpp", "param_table.hpp")] + [
    os.path.join(ROOT, "include", "sentinel_amd.h")]
OUT = os.path.join(_HERE, "libsentinel_amd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", "-ffp-contract=off", "-Wall", "-Wno-pass-failed"]


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(d) > t for d in DEPS)


# name -> (source, links libsentinel_amd)
TOOLS = {"dropin_bench": (os.path.join(ROOT, "tools", "dropin_bench.cpp"), True),
         "wire_client": (os.path.join(ROOT, "tools", "wire_client.cpp"), False)}


def build(force: bool = False, out: str = OUT, defines=()) -> str:
    if force or needs_build() or out != OUT:
        cmd = [HIPCC, *FLAGS, *[f"-D{d}" for d in defines], "-o", out, *SOURCES]
        subprocess.run(cmd, check=True)
    return out


def build_tools() -> None:
    """Native benchmark / front-end tools linked against the library (tools/, binaries next to them)."""
    for name, (src, lib) in TOOLS.items():
        exe = os.path.join(os.path.dirname(src), name)
        deps = [src, OUT] if lib else [src]
        if os.path.exists(exe) and os.path.getmtime(exe) > max(os.path.getmtime(d) for d in deps):
            continue
        if lib:
            cmd = [HIPCC, "-O2", "-std=c++17", "-o", exe, src, "-L" + _HERE, "-lsentinel_amd",
                   "-Wl,-rpath,$ORIGIN/../sentinel_amd", "-lpthread"]
        else:
            cmd = ["g++", "-O2", "-std=c++17", "-Wall", "-o", exe, src, "-lpthread"]
        subprocess.run(cmd, check=True)
    if not os.path.exists(GLUE_OUT) or os.path.getmtime(GLUE_OUT) <= os.path.getmtime(GLUE_SRC):
        subprocess.run([HIPCC, *FLAGS, "-o", GLUE_OUT, GLUE_SRC], check=True)


# bench.py's client-traffic kernel for --config 5conc (not part of the engine)
GLUE_SRC = os.path.join(ROOT, "tools", "bench_glue.hip")
GLUE_OUT = os.path.join(ROOT, "tools", "libbench_glue.so")


if __name__ == "__main__":
    print(build(force=True))
