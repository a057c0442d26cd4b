"""Build libpacmann.so (hand-written HIP for gfx950) in-tree.

    python -m pacmann_amd.build

The .so lands next to this file (pacmann_amd/libpacmann.so) so that it travels
to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIB = PKG / "libpacmann.so"
SOURCES = [CSRC / "pm_kernels.hip", CSRC / "pm_query.hip", CSRC / "pm_graph.hip", CSRC / "pm_shard.hip",
           CSRC / "pm_drl.hip", CSRC / "pm_engine.cpp"]
HEADERS = [CSRC / "pm_internal.h", CSRC / "pm_aes.h", CSRC / "pm_aes_bs.h", ROOT / "include" / "pacmann.h"]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = [
    "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
    # bit-exact fp32 L2: no FMA contraction, IEEE denormals (l2_distance_amd64.s order)
    "-ffp-contract=off", "-fno-gpu-flush-denormals-to-zero",
    "-Wall", "-Werror=return-type",
]


def needs_build() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    return any(p.stat().st_mtime > t for p in SOURCES + HEADERS)


def _compile_link(out: Path, defines: list[str], verbose: bool) -> None:
    """Each translation unit compiled on its own core (pm_query.hip dominates),
    then one link; the objects go to build/obj_<name>/."""
    from concurrent.futures import ThreadPoolExecutor
    objdir = ROOT / "build" / f"obj_{out.stem}"
    objdir.mkdir(parents=True, exist_ok=True)
    cflags = [f for f in FLAGS if f != "-shared"]

    def cc(src: Path) -> Path:
        obj = objdir / (src.name + ".o")
        cmd = [HIPCC, *cflags, *defines, "-c", "-o", str(obj), str(src)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True, cwd=CSRC)
        return obj
    with ThreadPoolExecutor(max_workers=min(len(SOURCES), os.cpu_count() or 1)) as ex:
        objs = list(ex.map(cc, SOURCES))
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(out), *map(str, objs), "-ldl"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, cwd=CSRC)


def build(force: bool = False, verbose: bool = True) -> Path:
    if force or needs_build():
        _compile_link(LIB, [], verbose)
    return LIB


def build_variant(name: str, defines: list[str]) -> Path:
    """An experiment build (e.g. -DPM_PUBLISH=0) at build/libpacmann_<name>.so,
    loaded instead of the default with PM_LIB=<path>."""
    out = ROOT / "build" / f"libpacmann_{name}.so"
    out.parent.mkdir(exist_ok=True)
    _compile_link(out, defines, True)
    return out


if __name__ == "__main__":
    if "--variant" in sys.argv:
        i = sys.argv.index("--variant")
        build_variant(sys.argv[i + 1], sys.argv[i + 2:])
    else:
        build(force="--force" in sys.argv)
