"""CPU checks of bench.py's host-side legs (no GPU): the CPU baseline runs the reference build
and reports the contract's fields; the PMC traffic lookup refuses a summary of another build."""
import os

import pytest

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def test_cpu_baseline_runs_reference():
    import bench
    if not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libref_cauchy.so")):
        pytest.skip("oracle/_ref not built")
    cpu = bench.cpu_baseline(28, 4, 1400, 0, 0.2, 2)
    assert cpu is not None and cpu["kind"] == "reference" and cpu["cores"] == 2
    assert cpu["value"] > 0 and cpu["unit"] == "GiB/s" and "group pairs" in cpu["sample"]


def test_traffic_lookup_requires_matching_build():
    import bench
    import shorthair_amd as sh

    class Fake:
        LIB_PATH = os.path.join(ROOT, "bench.py")  # any file whose hash no summary carries

    assert bench.pmc_traffic(Fake, 200, 32, 1400, 8192, 32) == (None, None)
    t, src = bench.pmc_traffic(sh, 200, 32, 1400, 8192, 32)
    assert (t is None) == (src is None)
    if t is not None:  # a summary of this very build: per-kernel read/write/total bytes
        for v in t.values():
            assert v["hbm_bytes"] > 0 and abs(v["hbm_bytes"] - v["read_bytes"] - v["write_bytes"]) <= 1  # rounding


@pytest.mark.parametrize("n", [1, 2, 3])
def test_launcher_spawns_ranks(n):
    """`bench.py --gpus N` outside a launcher starts N rank processes (before any GPU call) with
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set; --dry-run joins them in a gloo group (no GPU)
    and rank 0 reports what every rank saw."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1  # only rank 0 prints
    d = json.loads(line[0])
    assert d["dry_run"] and d["n_gpus"] == n and d["gpus_arg"] == n
    ranks = d["ranks"]
    assert [x["rank"] for x in ranks] == list(range(n))
    assert all(x["local_rank"] == x["rank"] and x["world_size"] == n for x in ranks)
    assert len({x["master_port"] for x in ranks}) == 1 and len({x["pid"] for x in ranks}) == n


def test_cpu_baseline_native_modes():
    import bench
    if not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "cpu_bench")):
        pytest.skip("oracle/_ref/cpu_bench not built")
    cpu = bench.cpu_baseline(28, 4, 1400, 4, 0.2, 2)
    assert set(cpu["modes"]) == {"shipped_t1", "init_t1", "shipped_t2", "init_t2"}
    assert cpu["value"] == max(cpu["modes"]["shipped_t2"]["GiBps"], cpu["modes"]["init_t2"]["GiBps"])
    assert cpu["cpu"]


@pytest.mark.gpu
def test_bench_two_ranks_on_one_gpu():
    """The whole N > 1 path of `bench.py --gpus 2` (spawn, process group, per-rank shards,
    barrier + max-over-ranks timing, root-resident scatter/encode/gather) with both ranks on the
    box's one GPU over gloo: the JSON line reports 2 GPUs and the root shards round-trip."""
    import json
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--steps", "2", "--warmup", "1", "--groups", "256", "--root-steps", "1", "--no-cpu",
                        "--host-calls", "0", "--no-sweep"], capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["value"] > 0 and line["config"]["parallelism"] == "groups sharded x2"
    rr = line["root_resident"]
    assert rr.get("roundtrip_ok") is True, rr
    assert rr["encode"]["GiBps"] > 0 and rr["decode"]["GiBps"] > 0


@pytest.mark.gpu
def test_bench_total_groups_chunked_root_two_ranks():
    """C5's form at small scale: `--total-groups` shards an odd number of groups unevenly over two
    ranks ("scaling": "strong"), and the root-resident leg streams them through a small root
    window in several chunks (partial last chunk on one rank) with the round trip checked."""
    import json
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--steps", "2", "--warmup", "1", "--total-groups", "301", "--root-chunk", "64",
                        "--root-steps", "1", "--no-cpu", "--host-calls", "0", "--no-sweep"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["config"]["total_groups"] == 301
    rr = line["root_resident"]
    assert rr.get("roundtrip_ok") is True, rr
    for op in ("encode", "decode"):
        assert rr[op]["chunks"] == 3 and rr[op]["chunk_groups_per_rank"] == 64


@pytest.mark.gpu
def test_bench_uneven_shards_default_chunk():
    """an odd --total-groups with the DEFAULT chunk (every rank derives it from the
    largest shard) and a root window small enough for several chunks, the last one partial on one
    rank only: both root-resident legs (encode, decode) round-trip."""
    import json
    import subprocess
    import sys
    env = dict(os.environ, SH_ROOT_WINDOW_BYTES=str(int(2 * 70 * (200 + 32) * 1400)))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--steps", "1", "--warmup", "1", "--total-groups", "281",
                        "--root-steps", "1", "--no-cpu", "--host-calls", "0", "--no-sweep"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    rr = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])["root_resident"]
    assert rr.get("roundtrip_ok") is True, rr
    assert rr["encode"]["chunk_groups_per_rank"] == 70 and rr["encode"]["chunks"] == 3


def test_sweep_regression_check(tmp_path):
    """tools/sweep_table.py --against flags a sweep row or headline op that got slower."""
    import importlib.util
    import json
    spec = importlib.util.spec_from_file_location("sweep_table", os.path.join(ROOT, "tools", "sweep_table.py"))
    st = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(st)
    row = {"config": "C4", "k": 28, "m": 4, "B": 256, "groups": 209263, "path": "fixed",
           "encode_ms": 0.35, "decode_ms": 0.705, "decode_frac": 0.1, "mean_e": 4.0}
    old = {"value": 1.0, "unit": "GiB/s", "ops": {"encode_ms": 0.68, "decode_ms": 1.08}, "sweep": [row]}
    new = json.loads(json.dumps(old))
    new["sweep"][0]["decode_ms"] = 0.765  # 8.5 % slower
    regs, n = st.compare(new, old, 0.05)
    assert n == 4 and [r[0] for r in regs] == ["C4 (28,4,256) G=209263 fixed decode"]
    assert st.compare(new, old, 0.10)[0] == []
    a, b = tmp_path / "old.json", tmp_path / "new.json"
    a.write_text(json.dumps(old) + "\n")
    b.write_text("log line\n" + json.dumps(new) + "\n")
    assert st.main([str(b), "--against", str(a)]) == 1
    assert st.main([str(a), "--against", str(a)]) == 0
