"""Build libcauchy256.so in-tree: hand-written HIP kernels for gfx950 + the C-ABI host library.

    python shorthair_amd/build.py        (also run by __graft_entry__.build())

hipcc cross-compiles for gfx950 without a GPU. The .so lands next to this file so it travels
with the repository snapshot to the GPU box (it is git-ignored, not gpurun-ignored).
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, os.environ.get("SH_LIB_NAME", "libcauchy256.so"))
SOURCES = ["kernels.hip", "stageb.hip", "tile_snip.hip", "fixed_dispatch.cpp", "cauchy_256_host.cpp", "shorthair_groups.cpp"]
HOST_SOURCES = ["gf256_host.cpp"]  # plain host C++ (no HIP): compiled with the host compiler
CXX = os.environ.get("CXX", "g++")
GEN_DIR = os.path.join(CSRC, os.environ.get("SH_GEN_DIR", "gen"))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SH_OFFLOAD_ARCH", "gfx950")


def generate():
    """Emit csrc/gen/ (compile-time-scheduled kernels) from tools/gen_fixed_kernels.py."""
    import importlib.util
    path = os.path.join(HERE, "..", "tools", "gen_fixed_kernels.py")
    spec = importlib.util.spec_from_file_location("gen_fixed_kernels", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    os.makedirs(GEN_DIR, exist_ok=True)
    for f in os.listdir(GEN_DIR):  # drop outputs of earlier generator versions
        os.remove(os.path.join(GEN_DIR, f))
    mod.OUTDIR = GEN_DIR
    mod.main([])


def _gen_sources():
    return sorted(os.path.join(GEN_DIR, f) for f in os.listdir(GEN_DIR) if f.endswith(".hip"))


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if os.path.isfile(os.path.join(CSRC, f))]
    deps += [os.path.join(GEN_DIR, f) for f in os.listdir(GEN_DIR)]
    deps += [os.path.join(HERE, "..", "include", f) for f in os.listdir(os.path.join(HERE, "..", "include"))]
    return any(os.path.getmtime(d) > t for d in deps)


FLAGS = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-result"]
FLAGS += os.environ.get("SH_EXTRA_FLAGS", "").split()  # experiments only (tools/build_variant.sh)
# A/B variants only (tools/build_variant.sh): the environment switches of csrc/measure.hpp. The
# product library is never built with it.
if os.environ.get("SH_MEASUREMENT") == "1":
    FLAGS.append("-DSH_MEASUREMENT_BUILD")
OBJ_DIR = os.path.join(HERE, os.environ.get("SH_OBJ_DIR", "build_obj"))


def _includes(path, seen=None):
    """Files `path` pulls in through #include "..." (recursively; resolved against the including
    file's directory, csrc/ and the generated-kernel directory, as the -I flags do)."""
    import re
    seen = set() if seen is None else seen
    try:
        text = open(path, errors="replace").read()
    except OSError:
        return seen
    for name in re.findall(r'^\s*#\s*include\s+"([^"]+)"', text, re.M):
        for d in (os.path.dirname(path), CSRC, GEN_DIR):
            cand = os.path.normpath(os.path.join(d, name))
            if os.path.exists(cand):
                if cand not in seen:
                    seen.add(cand)
                    _includes(cand, seen)
                break
    return seen


def _compile(src, verbose):
    obj = os.path.join(OBJ_DIR, os.path.basename(src) + ".o")
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(
            os.path.getmtime(src), *[os.path.getmtime(h) for h in _includes(src)], 0):
        return obj, None
    if os.path.basename(src) in HOST_SOURCES:
        cmd = [CXX, "-O3", "-std=c++17", "-fPIC", "-Wall", "-c", src, "-o", obj]
    else:
        cmd = [HIPCC] + FLAGS + [f"-I{GEN_DIR}", "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    return obj, subprocess.Popen(cmd)


def build(force=False, verbose=True, jobs=None):
    """Compile every source to build_obj/ (generated kernels in parallel: each is a large
    straight-line function, ~1-2 min for k=200) and link libcauchy256.so."""
    gen_script = os.path.join(HERE, "..", "tools", "gen_fixed_kernels.py")
    gen_inputs = max(os.path.getmtime(gen_script),
                     os.path.getmtime(os.path.join(HERE, "..", "tools", "xor_sched.py")),
                     os.path.getmtime(os.path.join(CSRC, "cauchy_tables_data.h")))
    if (force or not os.path.isdir(GEN_DIR) or not _gen_sources()
            or min(os.path.getmtime(f) for f in _gen_sources()) < gen_inputs):
        generate()
    if not force and not _stale():
        return LIB
    os.makedirs(OBJ_DIR, exist_ok=True)
    if force:
        for f in os.listdir(OBJ_DIR):
            os.remove(os.path.join(OBJ_DIR, f))
    jobs = jobs or max(1, min(8, os.cpu_count() or 1))
    srcs = _gen_sources() + [os.path.join(CSRC, s) for s in SOURCES + HOST_SOURCES]
    objs, running = [], []
    for src in srcs:
        while len(running) >= jobs:
            p = running.pop(0)
            if p.wait() != 0:
                raise subprocess.CalledProcessError(p.returncode, p.args)
        obj, p = _compile(src, verbose)
        objs.append(obj)
        if p is not None:
            running.append(p)
    for p in running:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, p.args)
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC",
           f"-Wl,--version-script={os.path.join(CSRC, 'exports.map')}", "-o", LIB + ".tmp"] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
