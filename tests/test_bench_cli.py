"""bench.py contract under the driver's launcher, on CPU (gloo): two ranks via
torch.distributed.run, one JSON line from rank 0 with the whole-job value."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_json_contract():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--preset", "tiny",
           "--local-batch", "4", "--seq-len", "16"]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1
    assert d["scaling"] == "weak" and d["higher_is_better"] is True
    assert d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 8
    # whole-job tokens/s: global batch x (src + tgt) tokens per step / step time
    expect = 8 * (16 + 16) / (d["ms_per_step"] / 1000.0)
    assert abs(d["value"] - expect) / expect < 0.01


def test_bench_self_launches_ranks():
    """`python bench.py --gpus 2` with no launcher starts its own two ranks
    (here over gloo on CPU) and prints one dp2 line."""
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--preset", "tiny", "--local-batch", "4", "--seq-len", "16"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                            "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["config"]["global_batch"] == 8


def test_bench_rejects_world_mismatch():
    """A launcher world that differs from --gpus is an error, not a warning."""
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0",
           "--preset", "tiny", "--local-batch", "2", "--seq-len", "8"]
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_bench_self_launches_eight_ranks():
    """`python bench.py --gpus 8` -- the driver's largest case -- starting its
    own eight ranks (gloo on CPU, tiny preset), with the host comm-thread
    issue path forced and random per-rank issue jitter: one dp8 line from
    rank 0, global batch 8 x local."""
    cmd = [sys.executable, "bench.py", "--gpus", "8", "--steps", "2", "--warmup", "1",
           "--preset", "tiny", "--local-batch", "2", "--seq-len", "8"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                            "MASTER_ADDR", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="1", TDG_DP_COMM_THREAD="force", TDG_DP_ISSUE_JITTER_MS="10")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["config"]["parallelism"] == "dp8"
    assert d["config"]["global_batch"] == 16
    assert d["config"]["comm_issue"] == "thread"
    assert r.stderr.count("comm_issue=thread") == 8  # every rank on the thread path


def test_visible_gpus_does_not_initialise_hip(monkeypatch):
    """The self-launching parent counts GPUs from the visible-devices lists
    or the KFD topology, never through a HIP call."""
    import importlib.util

    import torch

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    for var in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2")
    assert bench.visible_gpus() == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert bench.visible_gpus() == 0
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    assert bench.visible_gpus() >= 0  # KFD topology (0 without a GPU)
    assert not torch.cuda.is_initialized()


def test_fp8_precision_record_lists_every_op():
    """bench.py's dtype field for --dtype fp8 says exactly what runs in which
    format: the output projection, the dgrads and the weight gradients are
    fp8, the attention backward is the fp8-MFMA kernel up to 512 keys (the
    bf16 backward with e5m2 outputs beyond), the vocabulary projection bf16."""
    from tensorflow_distributed_on_gke_amd.ops import fp8

    m = fp8.precision_map()
    s = fp8.precision_string()
    assert m["attention_output_projection_forward"].startswith("e4m3")
    assert m["ffn_weight_gradients"].startswith("e5m2")
    assert m["attention_projection_weight_gradients"].startswith("e5m2")
    assert m["attention_projection_dgrads"].startswith("e5m2")
    assert m["attention_backward"] == fp8.ATTN_BWD_PRECISION
    assert "512" in m["attention_backward"] and "e5m2" in m["attention_backward"]
    assert "attention_backward=" + fp8.ATTN_BWD_PRECISION in s
    assert m["vocab_projection"].startswith("bf16")
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert "_fp8_precision()" in src  # the record prints the map
