"""CPU tests of the drop-in boundary: the C-ABI library builds, loads and exports exactly the
symbols include/*.h declares, with the reference's Block layout; a C caller compiles and links
against it the way Shorthair.cpp would. No codec call is made here (no GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
INCLUDE = os.path.join(ROOT, "include")


def _declared_functions():
    names = set()
    for h in os.listdir(INCLUDE):
        text = open(os.path.join(INCLUDE, h)).read()
        text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
        for m in re.finditer(r"^\s*(?!\s*typedef\b)(?:extern\s+)?[\w\s\*]+?\b(\w+)\s*\([^;{]*\)\s*;", text, re.M):
            names.add(m.group(1))
    return names


def _exported(lib_path):
    out = subprocess.run(["nm", "-D", "--defined-only", lib_path], capture_output=True, text=True,
                         check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_library_exports_every_declared_symbol():
    import shorthair_amd
    declared = _declared_functions()
    assert {"_cauchy_256_init", "cauchy_256_encode", "cauchy_256_decode"} <= declared
    exported = _exported(shorthair_amd.LIB_PATH)
    assert declared <= exported, f"missing: {declared - exported}"
    # nothing else leaks out of the library (version script)
    assert exported == declared
    assert set(shorthair_amd.EXPORTED_SYMBOLS) == declared


def test_block_layout_matches_reference():
    """Reference Block (cauchy_256.h:52-55): data @0, row @8, sizeof 16 on LP64."""
    import shorthair_amd
    B = shorthair_amd.Block
    assert ctypes.sizeof(B) == 16
    assert B.data.offset == 0 and B.row.offset == 8


def test_version_mismatch_is_rejected_without_gpu():
    """_cauchy_256_init returns -1 on a version mismatch before touching the GPU
    (reference cauchy_256.cpp:392-394)."""
    import shorthair_amd
    assert shorthair_amd.lib._cauchy_256_init(3) == -1


def test_field_table_pointers_exported():
    """cauchy_256.o's two data symbols (cauchy_256.cpp:346-347) are exported, null until a
    successful _cauchy_256_init (filled on the GPU box: test_gpu_parity)."""
    import shorthair_amd
    out = subprocess.run(["nm", "-D", "--defined-only", shorthair_amd.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    data = {line.split()[-1] for line in out.splitlines() if line.split()[1] in ("B", "D")}
    assert {"GFC256_MUL_TABLE", "GFC256_DIV_TABLE"} <= data
    # no GPU here, so no _cauchy_256_init has succeeded in this process
    assert ctypes.c_void_p.in_dll(shorthair_amd.lib, "GFC256_MUL_TABLE").value is None


# Environment switches that select other kernels or launch splits for same-box A/B runs. They
# exist only in measurement builds (tools/build_variant.sh, csrc/measure.hpp); the shipped drop-in
# library must not change its code path because of its caller's environment.
MEASUREMENT_SWITCHES = ("SH_HSACO_DIR", "SH_DEC_CHUNKS", "SH_STAGEB_OLD", "SH_FORCE_TILE", "SH_NO_TILE",
                        "SH_NO_COL", "SH_COL_ENC", "SH_SB_SLICE", "SH_SLICE_MAX", "SH_SLICE_STEPS",
                        "SH_SMALL_XCD", "SH_V2_NW", "SH_V2_NO_TAIL", "SH_V2_MIN", "SH_V2_MAX",
                        "SH_PKT_CHUNK_MB", "SH_HOST_THREADS", "SH_SETUP_WAVE", "SH_SETUP_MIN_SMALL", "SH_SETUP_MIN_CAUCHY", "SH_SMALL2")


def test_product_library_has_no_measurement_hooks():
    """The default libcauchy256.so names none of the A/B switches, imports no module loader and
    reads no environment variable at all."""
    import shorthair_amd
    blob = open(shorthair_amd.LIB_PATH, "rb").read()
    for name in MEASUREMENT_SWITCHES:
        assert name.encode() not in blob, name
    out = subprocess.run(["nm", "-D", "--undefined-only", shorthair_amd.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    undefined = {line.split()[-1].split("@")[0] for line in out.splitlines() if line.strip()}
    assert not any(u.startswith("hipModule") for u in undefined), sorted(u for u in undefined if "Module" in u)
    assert "getenv" not in undefined and "secure_getenv" not in undefined


def test_measurement_switches_only_behind_the_build_flag():
    """Every getenv in the library sources goes through csrc/measure.hpp's SH_MEASURE_ENV (a null
    pointer unless -DSH_MEASUREMENT_BUILD), and only variant builds set that flag."""
    csrc = os.path.join(ROOT, "shorthair_amd", "csrc")
    for f in os.listdir(csrc):
        if f.endswith((".cpp", ".hip", ".hpp", ".h")) and f != "measure.hpp":
            text = open(os.path.join(csrc, f)).read()
            assert "getenv" not in text, f
            assert "hipModuleLoad" not in text or "#ifdef SH_MEASUREMENT_BUILD" in text, f
    build = open(os.path.join(ROOT, "shorthair_amd", "build.py")).read()
    assert 'os.environ.get("SH_MEASUREMENT") == "1"' in build
    assert "SH_MEASUREMENT=1" in open(os.path.join(ROOT, "tools", "build_variant.sh")).read()


def test_headers_have_no_torch_or_cpp_types():
    for h in os.listdir(INCLUDE):
        text = re.sub(r"/\*.*?\*/", " ", open(os.path.join(INCLUDE, h)).read(), flags=re.S)
        assert "torch" not in text and "std::" not in text and "hipStream_t" not in text


def test_c_caller_compiles_and_links(tmp_path):
    """A plain-C translation unit written against include/cauchy_256.h links against the library
    exactly like the reference's caller (Shorthair.cpp:566, :747, :912) would."""
    import shorthair_amd
    src = tmp_path / "caller.c"
    src.write_text(r'''
#include "cauchy_256.h"
#include "cauchy_256_batch.h"
#include <stdio.h>
int main(void) {
    if (cauchy_256_init() != 0) { printf("init failed\n"); return 2; }
    unsigned char a[16] = {1}, b[16] = {2}, rec[32];
    const unsigned char *ptrs[2] = {a, b};
    int rc = cauchy_256_encode(2, 2, ptrs, rec, 16);
    Block blocks[2] = {{a, 0}, {rec + 16, 3}};
    rc |= cauchy_256_decode(2, 2, blocks, 16);
    printf("rc=%d row=%d\n", rc, blocks[1].row);
    return rc;
}
''')
    exe = tmp_path / "caller"
    libdir = os.path.dirname(shorthair_amd.LIB_PATH)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", f"-I{INCLUDE}", str(src), "-o", str(exe),
                    f"-L{libdir}", "-lcauchy256", f"-Wl,-rpath,{libdir}"], check=True)
    assert exe.exists()


@pytest.mark.gpu
def test_c_caller_runs_on_gpu(tmp_path):
    import shorthair_amd
    test_c_caller_compiles_and_links(tmp_path)
    res = subprocess.run([str(tmp_path / "caller")], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stdout + res.stderr
    # row 1 was recovery row k+1 = 3 -> receives the missing original row 1
    assert "rc=0 row=1" in res.stdout


@pytest.mark.parametrize("k,m,e_fixed", [(200, 32, 32), (200, 32, 0), (28, 4, 0), (3, 250, 0), (1, 1, 0),
                                         (64, 16, 7)])
def test_synthetic_erasure_pattern_matches_oracle(k, m, e_fixed):
    """The library's host-side pattern generator (bench.py's decode inputs) reproduces the test
    oracle's stream exactly, so the benchmark decodes what the parity tests check."""
    import shorthair_amd
    from oracle import pyoracle as po
    for g in (0, 1, 17, 8191, 123456789):
        e1, r1 = shorthair_amd.erasure_pattern(g, k, m, 0xBE, e_fixed)
        e2, r2 = po.erasure_pattern(g, k, m, 0xBE, e_fixed)
        assert e1 == e2 and (r1 == r2).all()
    assert shorthair_amd.lib.cauchy_256_erasure_pattern(0, 200, 57, 0, 0, None) == -1


@pytest.mark.gpu
def test_package_before_torch_shares_one_hip_runtime():
    """Importing shorthair_amd before torch must not load a second HIP/HSA runtime (torch ships
    its own libamdhip64 with the same SONAME): both the library and torch see the GPU."""
    import subprocess
    import sys
    code = ("import shorthair_amd as s; import torch; assert torch.cuda.is_available(); "
            "assert s.lib.cauchy_256_batch_init(0) == 0; x = torch.ones(4, device='cuda'); "
            "assert x.sum().item() == 4.0; print('ok')")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-500:]
