"""bench.py's `--gpus N` contract: the line measures N GPUs or the run
refuses. CPU only: the layout planner with stand-in device counts, and the real script on this
GPU-less container, which must exit 2 with the reason rather than measure one GPU."""
import os
import pathlib
import subprocess
import sys

import pytest

REPO = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import bench  # noqa: E402


def devices(n):
    calls = []

    def count():
        calls.append(1)
        return n
    count.calls = calls
    return count


def test_single_gpu_needs_no_device_query():
    c = devices(0)
    assert bench.plan_layout(1, {}, c) == {"mode": "single", "world": 1}
    assert not c.calls


def test_in_process_handle_over_n_devices():
    lay = bench.plan_layout(4, {}, devices(8))
    assert lay == {"mode": "in-process", "world": 4, "devices": [0, 1, 2, 3]}


@pytest.mark.parametrize("n", [0, 1, 3])
def test_in_process_refuses_fewer_devices(n):
    with pytest.raises(bench.LayoutError, match=rf"needs 4 HIP devices; {n} visible"):
        bench.plan_layout(4, {"HIP_VISIBLE_DEVICES": "0"}, devices(n))


def test_launcher_world_must_equal_gpus():
    with pytest.raises(bench.LayoutError, match="WORLD_SIZE=2"):
        bench.plan_layout(8, {"WORLD_SIZE": "2", "LOCAL_WORLD_SIZE": "2"}, devices(8))
    with pytest.raises(bench.LayoutError, match="WORLD_SIZE=8"):
        bench.plan_layout(1, {"WORLD_SIZE": "8", "LOCAL_WORLD_SIZE": "8"}, devices(8))


def test_launcher_needs_a_device_per_local_rank():
    env = {"WORLD_SIZE": "8", "LOCAL_WORLD_SIZE": "8"}
    assert bench.plan_layout(8, env, devices(8)) == {"mode": "launcher", "world": 8}
    with pytest.raises(bench.LayoutError, match="8 ranks on this node need 8 HIP devices"):
        bench.plan_layout(8, env, devices(1))
    # the one-GPU test mode (two ranks sharing GPU 0 over the host exchange) asks no device count
    c = devices(1)
    assert bench.plan_layout(2, {"WORLD_SIZE": "2"}, c, same_device=True)["mode"] == "launcher"
    assert not c.calls


def test_multi_shards_diagnostic_is_one_gpu_only():
    with pytest.raises(bench.LayoutError, match="--multi-shards"):
        bench.plan_layout(2, {}, devices(8), multi_shards=2)
    assert bench.plan_layout(1, {}, devices(1), multi_shards=2)["mode"] == "single"


def run_bench(args, env_extra):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    env.update(env_extra)
    return subprocess.run([sys.executable, str(REPO / "bench.py"), *args], cwd=REPO, env=env,
                          capture_output=True, text=True, timeout=300)


def test_script_refuses_gpus_2_without_two_devices():
    """The real script on a host with no visible GPU: exit 2, reason on stderr, no JSON line."""
    r = run_bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"], {})
    assert r.returncode == 2, r.stderr[-2000:]
    assert "needs 2 HIP devices" in r.stderr
    assert r.stdout.strip() == ""


def test_script_refuses_launcher_mismatch():
    r = run_bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"],
                  {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2, r.stderr[-2000:]
    assert "WORLD_SIZE=1" in r.stderr
    assert r.stdout.strip() == ""


class _FakeCtx:
    """col_names / col_find / col_download / weights_download over numpy arrays (the calls
    bench.state_digests makes)."""
    def __init__(self, cols, w):
        self.cols, self.w = cols, w

    def col_names(self):
        return list(self.cols)

    def col_find(self, name):
        return name

    def col_download(self, c):
        return self.cols[c]

    def weights_download(self):
        return self.w


def _population(n=12, seed=0):
    import numpy as np
    r = np.random.default_rng(seed)
    return {"x_1": r.standard_normal((2, n)), "v": r.standard_normal((2, n)), "a": r.standard_normal(n)}, \
        r.standard_normal(n)


def test_self_check_digests_and_verdict():
    """a sharded line carries its own parity proof. The digests of a shard
    slice of one population equal those of the same slice held by a shard; the verdict passes
    only when every shard and the evidence agree."""
    cols, w = _population()
    full = _FakeCtx(cols, w)
    shard1 = _FakeCtx({k: v[..., 6:12] for k, v in cols.items()}, w[6:12])
    ref = [bench.state_digests(full, 0, 6), bench.state_digests(full, 6, 12)]
    assert bench.state_digests(shard1, 0, 6) == ref[1]
    assert bench.state_digests(full, 0, 12) != ref[0]
    ok = bench.check_verdict(ref, list(ref), -1.5, -1.5)
    assert ok["exact_vs_1gpu"] and ok["mismatched_shards"] == []
    bench.refuse_on_mismatch(ok)                       # passes silently


def test_self_check_mismatch_refuses_the_line():
    cols, w = _population()
    full = _FakeCtx(cols, w)
    ref = [bench.state_digests(full, 0, 6), bench.state_digests(full, 6, 12)]
    bad_w = w.copy()
    bad_w[8] = -bad_w[8]                               # one weight of shard 1 differs
    got = [ref[0], bench.state_digests(_FakeCtx(cols, bad_w), 6, 12)]
    v = bench.check_verdict(ref, got, -1.5, -1.5)
    assert not v["exact_vs_1gpu"] and v["mismatched_shards"] == [1]
    with pytest.raises(SystemExit) as e:
        bench.refuse_on_mismatch(v)
    assert e.value.code == 2
    v = bench.check_verdict(ref, list(ref), -1.5, -1.5000000000000002)   # the evidence alone
    assert not v["exact_vs_1gpu"] and not v["evidence_equal"]
    with pytest.raises(SystemExit):
        bench.refuse_on_mismatch(v)
