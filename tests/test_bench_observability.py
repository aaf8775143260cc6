"""bench.py's multi-rank contract on the CPU (gloo), the way the driver's
8-GPU run uses it: the JSON line carries per-rank step times, the operand
all-gather's time and bytes, and the process group's world size; and a rank
that stops answering makes the job exit non-zero within the collective
timeout instead of hanging (VERDICT r3 "next round" #5; the reference prints
its wall-clock on every rank, sparse_matrix_mult.cu:677-679, and has no
timeout on its blocking MPI calls)."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(extra_env, *args, timeout=240):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2", **extra_env)
    for v in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(v, None)
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--matrix-n", "8192", "--matrix-density", "0.002", *args],
                       capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    return r, time.time() - t0


def test_bench_two_gloo_ranks_reports_per_rank_fields():
    r, _ = _bench({}, "--steps", "3", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout   # rank 0 prints ONE line
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["torch_dist_world"] == 2
    pr = rec["per_rank"]
    for key in ("step_ms_mean", "step_ms_min", "step_ms_max", "wall_ms_per_step", "allgather_ms_per_step",
                "allgather_bytes_per_step"):
        assert len(pr[key]) == 2, key
    assert all(b > 0 for b in pr["allgather_bytes_per_step"])   # B's row panels crossed the wire every step
    assert rec["rank_step_ms"]["min"] <= rec["rank_step_ms"]["mean"] <= rec["rank_step_ms"]["max"]
    assert rec["ms_per_step"] > 0


def test_bench_stuck_rank_exits_nonzero_within_timeout():
    r, dt = _bench({"SPMM_COMM_TIMEOUT": "8", "SPMM_BENCH_STALL_RANK": "1", "SPMM_BENCH_STALL_S": "300"},
                   "--steps", "2", "--warmup", "1", timeout=200)
    assert r.returncode != 0
    assert dt < 120, f"stuck collective took {dt:.0f} s to surface"
    assert "exited with" in r.stderr   # the launcher names the failing rank and stops the others
