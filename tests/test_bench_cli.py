"""bench.py's --gpus contract on a host without enough GPUs (CPU test): the run must fail loudly,
never report fewer GPUs than asked for."""
import os
import subprocess
import sys
import types

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _args(gpus):
    return types.SimpleNamespace(gpus=gpus)


def test_gpus_2_on_a_host_with_fewer_devices_exits_nonzero():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""      # (this container has no GPU anyway)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0
    assert "--gpus 2 requested but only" in r.stderr
    assert '"n_gpus"' not in r.stdout


def test_launch_modes(monkeypatch):
    import torch
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    assert bench.launch_mode(_args(1)) == ("single", 1)
    assert bench.launch_mode(_args(8)) == ("context", 8)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 4)
    with pytest.raises(SystemExit, match="only 4 GPU"):
        bench.launch_mode(_args(8))
    # the driver's N > 1 launch (torchrun): one rank per GPU, --gpus agrees with WORLD_SIZE
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert bench.launch_mode(_args(4)) == ("torchrun", 4)
    assert bench.launch_mode(_args(1)) == ("torchrun", 4)
    with pytest.raises(SystemExit, match="disagrees"):
        bench.launch_mode(_args(2))


def test_calls_avoided_leg_counts_at_get_model(monkeypatch):
    """The bench's "z3 calls avoided" leg on the oracle engine (small): counted at get_model,
    off = quick-sat hits only (each fork's not-taken side hits the parent's model), on = at least
    as many, and calls = quick-sat + candidate answers + solver calls."""
    import test_support as ts
    from mythril_amd import support as sp
    monkeypatch.setattr(sp, "VerdictEngine", lambda ev: ts.OracleEngine())
    r = bench.calls_avoided_leg(None, n_forks=12, budget=2000)
    off, on = r["candidates_off"], r["candidates_on"]
    for d in (off, on):
        assert d["get_model_calls"] == 24
        assert d["quick_sat_answers"] + d["candidate_answers"] + d["solver_calls"] == d["get_model_calls"]
        assert d["solver_calls_avoided"] == d["get_model_calls"] - d["solver_calls"]
    assert off["candidate_answers"] == 0 and off["quick_sat_answers"] == 12
    assert on["solver_calls_avoided"] >= off["solver_calls_avoided"]


class _NoTimers:
    """The evaluator timing hooks the drop-in legs call (no device: nothing to time)."""

    def time_kernels(self, on=True):
        pass

    def kernel_times(self, reset=True):
        return []

    def host_times(self, reset=False):
        return {}


def test_dropin_legs_time_several_new_batches_and_report_the_median(monkeypatch):
    """bench.py's drop-in cells on the oracle engine (small): every timed batch is new paths (the
    stream's rounds new parents), answers equal the reference loop replayed on the oracle, and the
    cell is the median repetition with all samples beside it."""
    import test_support as ts
    from mythril_amd import support as sp
    monkeypatch.setattr(sp, "VerdictEngine", lambda ev: ts.OracleEngine())
    ev = _NoTimers()
    for cell in bench.dropin_leg(ev, grid=((2, 4),), reps=3) + bench.dropin_stream_leg(ev, grid=((2, 4),), reps=3):
        assert cell["timed_batches"] == 3 and len(cell["ms_samples"]) == 3
        assert sorted(cell["ms_samples"])[1] == round(cell["ms_per_batch"], 4)
        assert cell["answers_match_reference_loop"]
    stream = bench.dropin_stream_leg(ev, grid=((2, 4),), reps=2)[0]
    assert stream["n_queries"] == 4 and stream["conjuncts_cached"] > 0


def test_two_rank_line_under_gloo_with_the_oracle_engine():
    """bench.py's N > 1 protocol end to end on CPU: torchrun world 2, gloo, the oracle answering
    for the GPU (--engine oracle).  The line keeps the driver's keys, the per-rank split of
    kernel / all-reduce / barrier time, and the planted first hits of the global model order."""
    import json
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--engine", "oracle", "--config", "c2", "--tapes", "50", "--models", "64",
                        "--steps", "2", "--warmup", "1"], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "per_rank", "parity_ok"):
        assert k in line, k
    assert line["n_gpus"] == 2 and line["steps"] == 2 and line["parity_ok"] is True
    assert line["config"]["models_total"] == 128
    pr = line["per_rank"]
    for k in ("kernel_ms", "allreduce_ms", "barrier_wait_ms"):
        assert 0 <= pr[k]["min"] <= pr[k]["max"], (k, pr[k])
    assert line["engine"].startswith("oracle")


@pytest.mark.parametrize("gpus", [1, 2])
def test_context_mode_line_is_attributable_with_the_oracle_engine(gpus):
    """One process driving N devices (--context, the way single-process Mythril would,
    mythril_analyzer.py:136-185), rehearsed on CPU with the oracle answering per model shard:
    the line carries each device's kernel time, the reduce and the host issue time."""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--context",
                        "--engine", "oracle", "--config", "c2", "--tapes", "40", "--models", "64", "--steps", "2",
                        "--warmup", "1", "--no-dropin", "--no-cpu-baseline"],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == gpus and line["parity_ok"] is True
    assert line["config"]["models_total"] == 64 * gpus
    pr = line["per_rank"]
    assert len(pr["kernel_ms_per_device"]) == gpus
    assert 0 <= pr["kernel_ms"]["min"] <= pr["kernel_ms"]["max"]
    assert pr["kernel_ms"]["max"] == max(pr["kernel_ms_per_device"])
    assert pr["allreduce_ms"]["min"] >= 0 and pr["issue_ms"] >= pr["peer_issue_ms"] >= 0
    assert "oracle" in pr["allreduce_timer"]
