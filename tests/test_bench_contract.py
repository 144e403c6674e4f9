"""bench.py driver contract on CPU: one JSON line with the required keys, at world
size 1 and under torch.distributed.run at world size 2 (gloo), tiny shapes."""
import json
import os
import subprocess
import sys

import pytest


def _free_port() -> str:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return str(sk.getsockname()[1])

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}
TINY = ["--users", "3000", "--items", "700", "--batch", "4096", "--pool", "2", "--steps", "2", "--warmup", "1"]


def _env():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    env.pop("FPS_SHARE_GPU", None)
    return env


def _json_lines(out: str):
    return [json.loads(x) for x in out.splitlines() if x.startswith("{")]


def test_bench_single_rank_json_line():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + TINY, capture_output=True, text=True,
                       timeout=300, env=_env(), cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1
    d = lines[0]
    assert KEYS <= set(d)
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["value"] > 0
    assert d["config"]["global_batch"] == 4096


@pytest.mark.parametrize("exchange", ["rotate", "ps"])
def test_bench_two_ranks_gloo(exchange):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", _free_port(),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--exchange", exchange] + TINY
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=_env(), cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1  # rank 0 only
    d = lines[0]
    assert KEYS <= set(d) and d["n_gpus"] == 2 and d["config"]["global_batch"] == 2 * 4096
    assert d["config"]["exchange"] == exchange
    # --verify is on by default at N > 1: the job's exchange on its process group == the sequential replay
    assert d["verify_ok"] is True and d["verify"]["verify_exchange"] == exchange
    assert d["verify"]["verify_world"] == 2 and len(d["verify"]["devices"]) == 2


def test_bench_gpus_without_torchrun_launches_ranks():
    """``--gpus 2`` without torchrun must run 2 ranks (never silently 1)."""
    env = _env()
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + TINY, capture_output=True,
                       text=True, timeout=600, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1
    d = lines[0]
    assert d["n_gpus"] == 2 and d["world_size"] == 2 and d["backend"] == "gloo"
    assert len(d["config"]["bytes_sent_per_rank"]) == 2 and min(d["config"]["bytes_sent_per_rank"]) > 0


def test_bench_verify_failure_prints_no_value():
    """A broken exchange (FPS_VERIFY_MUTANT: the rotation sends the block it is about to
    update instead of the finished one) must end every rank non-zero with no JSON line."""
    env = dict(_env(), FPS_VERIFY_MUTANT="wrong_buffer")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", _free_port(), os.path.join(ROOT, "bench.py"), "--gpus", "2"] + TINY
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert p.returncode != 0
    assert _json_lines(p.stdout) == []
    assert "VERIFY FAILED" in p.stderr


def test_bench_world_size_mismatch_fails():
    env = dict(_env(), WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + TINY, capture_output=True,
                       text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode != 0
    assert _json_lines(p.stdout) == []


def test_bench_metrics_jsonl(tmp_path):
    path = tmp_path / "m.jsonl"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--metrics-jsonl", str(path)] + TINY,
                       capture_output=True, text=True, timeout=300, env=_env(), cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    recs = [json.loads(x) for x in path.read_text().splitlines()]
    steps = [r for r in recs if r["kind"] == "step"]
    assert len(steps) == 3  # 2 timed steps + the flush
    assert all("mf.sgd" in s["stage_ms"] for s in steps[:2])
    summ = [r for r in recs if r["kind"] == "summary"][0]
    assert summ["counters"]["ratings"] == 3 * 4096


@pytest.mark.parametrize("script,args,metric_key", [
    ("bench/bench_mf_topk.py", ["--users", "3000", "--items", "2000", "--batch", "64", "--bucket", "512", "--steps",
                                "2", "--warmup", "1"], "learning_updates_per_s"),
    ("bench/bench_w2v.py", ["--vocab", "5000", "--dim", "32", "--pairs", "4096", "--steps", "2", "--warmup", "1"],
     "loss_first_last"),
    ("bench/bench_pa.py", ["--features", "100000", "--batch", "512", "--nnz", "16", "--steps", "2", "--warmup", "1"],
     "feature_updates_per_s"),
])
def test_secondary_benches_two_ranks_gloo(script, args, metric_key):
    """The secondary benches run end to end at world size 2 (gloo) and report the
    whole job from rank 0 only."""
    for attempt in range(2):  # CPU only: a port taken between _free_port() and the bind (parallel test workers)
        port = _free_port()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
               "127.0.0.1", "--master-port", port, os.path.join(ROOT, script)] + args
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=_env(), cwd=ROOT)
        if p.returncode == 0 or not any(m in p.stderr for m in ("Address already in use", "EADDRINUSE",
                                                                 "DistNetworkError")):
            break
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1
    d = lines[0]
    assert d["n_gpus"] == 2 and d["value"] > 0 and metric_key in d
