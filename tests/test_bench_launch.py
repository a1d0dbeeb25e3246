"""bench.py's N-rank launcher and CPU-baseline pool (CPU tests), plus the
launcher on one real GPU.

* `bench.py --gpus N` with no WORLD_SIZE starts N fresh ranks itself (the
  driver's scaling leg runs it that way); `--launch-selftest` makes the ranks
  join a gloo group and compute the same LPT chromosome shares as the GPU
  bench, so the launcher, its environment and the shard plan run on the CPU.
* `--gpus N` with fewer than N visible GPUs must fail, never run fewer ranks.
* oracle/cpu_pool.c (the cpu_baseline leg) must compute exactly the
  oracle's transform + bzip2 per piece.
"""
import json
import os
import subprocess
import sys

import pytest

from tests import corpus, oracle_lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


@pytest.mark.parametrize("n", [1, 2, 4])
def test_launcher_starts_n_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--launch-selftest", "--lines", "1000000"],
                       env=_env(), capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    lines = [ln for ln in r.stdout.decode().splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    res = json.loads(lines[0])
    assert res["n_gpus"] == n
    assert len(res["rank_bytes"]) == n and all(b > 0 for b in res["rank_bytes"])
    assert sum(res["rank_units"]) == 24


def test_launcher_refuses_missing_gpus():
    import torch
    have = torch.cuda.device_count()
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(max(2, have + 1)), "--steps", "1", "--warmup", "0"],
                       env=_env(), capture_output=True, timeout=300)
    assert r.returncode != 0
    assert b"refusing" in r.stderr


def test_kfd_gpu_count_from_sysfs(tmp_path):
    """The launcher counts GPUs from the KFD topology (no HIP call): nodes with
    SIMDs whose render node is accessible; CPU nodes (simd_count 0) and GPUs
    whose render node this process cannot open are not counted."""
    sys.path.insert(0, ROOT)
    import bench
    nodes, dri = tmp_path / "nodes", tmp_path / "dri"
    dri.mkdir()
    for i, (simd, minor, present) in enumerate([(0, 0, False), (1024, 128, True), (1024, 129, True),
                                                 (1024, 130, False)]):
        d = nodes / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text("cpu_cores_count 0\nsimd_count %d\ndrm_render_minor %d\n" % (simd, minor))
        if present:
            (dri / ("renderD%d" % minor)).write_text("")
    assert bench._kfd_gpus(str(nodes), str(dri)) == 2
    assert bench._kfd_gpus(str(tmp_path / "absent"), str(dri)) is None


def test_world_size_mismatch_fails():
    env = _env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--launch-selftest"], env=env, capture_output=True,
                       timeout=300)
    assert r.returncode != 0


def test_cpu_pool_matches_oracle():
    data = corpus.multi_chrom_bed(5, 3000, seed=5, kind="bed6") + corpus.multi_chrom_bed(3, 2000, seed=6)
    import starch_amd
    units = starch_amd.plan_units(data, 64)
    spans = [(u.offset, u.length) for u in units]
    secs, per, outb, kind = oracle_lib.cpu_pool(data, spans, 3)
    assert secs > 0 and len(per) == len(spans)
    for (o, l), got in zip(spans, outb):
        _, segs = oracle_lib.transform(data[o:o + l])
        want = sum(len(oracle_lib.ref_bz2(t, 9) if kind == "reference" else oracle_lib.bz2(t, 9))
                   for _, _, t in segs)
        assert got == want


@pytest.mark.gpu
def test_launcher_one_gpu_bench():
    """The launcher path on the GPU box: --gpus 1 --spawn: one launched
    rank (torch.distributed + the RCCL gather at world 1) on a small
    input; the line must say one GPU and carry the encode / gather split."""
    env = _env()
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--spawn", "--lines", "2000000", "--steps", "2",
                        "--warmup", "1", "--no-cpu-baseline", "--no-e2e"], env=env, capture_output=True, timeout=600)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    res = json.loads([ln for ln in r.stdout.decode().splitlines() if ln.startswith("{")][-1])
    assert res["n_gpus"] == 1
    assert res["dist"]["ms_encode_max"] > 0 and res["dist"]["ms_gather_max"] >= 0


@pytest.mark.gpu
def test_launcher_counts_gpus_without_hip():
    """bench.visible_gpus() in a fresh process equals torch's device count
    (taken in another process) and leaves no HIP runtime mapped: the launcher
    must not initialise the GPU before it starts its rank processes."""
    code = ("import sys; sys.path.insert(0, %r); import bench; n = bench.visible_gpus(); "
            "maps = open('/proc/self/maps').read(); print(n, int('libamdhip64' in maps))" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], env=_env(), capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    n, hip = map(int, r.stdout.split())
    r2 = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"], env=_env(),
                        capture_output=True, timeout=300)
    assert n == int(r2.stdout.split()[-1]) and n >= 1
    assert hip == 0
