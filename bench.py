#!/usr/bin/env python
"""Headline benchmark (BASELINE.json metric): whole-node GFLOP/s + wall-clock of
an n x n CSR SpGEMM at fixed density, 1D row-block over N MI355X GPUs.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Config (BASELINE.json config 4): A, B = 1M x 1M (n = 2^20) uniform random CSR
at 0.01 % density (~105 nnz/row), fp32 values, synthetic data generated on the
device with a row-chunk-seeded RNG, so every N multiplies the SAME matrices
(strong scaling).  One step = all-gather of B's row panels over RCCL + local
symbolic + numeric SpGEMM of this rank's A row panel (C stays distributed).
FLOPs = 2 x intermediate products (BASELINE.md convention), summed over ranks;
value = total FLOPs / max-over-ranks step time.

Other workloads (--workload): ``spmm`` (65536^2 CSR x dense 128 cols, bf16,
config 3), ``spgemm64k`` (65536^2 @ 0.1 %, config 2), ``rmat`` (R-MAT scale-24
A.A^T, config 5; ``--scale 20`` keeps C resident on one GPU), ``chain`` (the
reference's block-sparse uint64 chain through the native ``a4`` executable,
end to end like report Table 1, Medium preset by default).  BASELINE.json
publishes no number for the CSR configs, so vs_baseline is null for them; for
``chain`` it is the report's optimized wall-clock over ours.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GFLOP/s (whole node) + wall-clock, NxN SpGEMM at fixed density, 1/2/4/8 GPU"


def _sync_barrier(comm):
    import torch

    if comm.device.type == "cuda":
        torch.cuda.synchronize(comm.device)
    comm.barrier()
    if comm.device.type == "cuda":
        torch.cuda.synchronize(comm.device)


def _allreduce_sum(comm, x: float) -> float:
    return comm.allreduce_sum(x)


def run_spgemm(comm, args, n: int, density: float, model: str):
    from spmm_amd.models import spgemm as MS
    from spmm_amd.ops.spgemm import SpgemmInfo

    prob = MS.UniformProblem.build(n, density, comm, seed=args.seed)
    info = SpgemmInfo()
    if args.decomp == "inner":
        # A's column panel x B's row panel per rank, sparse reduce-scatter of C
        from spmm_amd.parallel.partition import row_panels

        Ac = prob.inner_operand()
        counts = [b - a for a, b in row_panels(n, comm.world)]
        C = MS.innerdim_spgemm(Ac, prob.B, comm, counts, info)
        nnz_local = C.nnz
        step = lambda: MS.innerdim_spgemm(Ac, prob.B, comm, counts)  # noqa: E731
    else:
        C = MS.rowblock_spgemm(prob.A, prob.B, comm, info)   # first (untimed) run also counts FLOPs
        nnz_local = info.nnz
        step = lambda: MS.rowblock_spgemm(prob.A, prob.B, comm)  # noqa: E731
    eager_step = step
    flops_local = info.flops
    del C
    graph = None
    if comm.device.type == "cuda" and args.decomp != "inner" and args.graph == "on" and (
            not comm.is_dist or comm.device_collectives):
        # the product's kernels (splits, count, scan, numeric) replayed from
        # captured HIP graphs, no host synchronisation inside the step; on N
        # ranks (RowblockGraph) the two payload all-gathers run between the
        # graphs, every step
        import torch

        from spmm_amd.ops.spgemm import SpgemmGraph

        try:
            torch.cuda.empty_cache()
            graph = MS.RowblockGraph(prob.A, prob.B, comm) if comm.is_dist else SpgemmGraph(prob.A, prob.B)
            step = lambda: graph.run()  # noqa: E731
        except ValueError as e:   # (no graph for this product on some rank: every rank takes eager steps, said so)
            if comm.rank == 0:
                print(f"[bench] spgemm graph unavailable ({e}); eager steps", file=sys.stderr, flush=True)
            graph = None
            torch.cuda.empty_cache()

        def verify():
            """After the timed loop: (1) the last replay's C equals an eager
            product's (row pointer and column sum exactly, value sum to fp32
            accumulation-order tolerance); (2) the eager step -- row-plan
            inspector, host read-backs, exact C allocation (and on N ranks the
            size / row-count gathers): everything the graph does once at
            construction -- timed on its own and reported next to the
            replayed step as ``eager_ms_per_step`` (5 steps, not the timed
            loop: a sanity field, not a like-for-like number)."""
            if graph is None:
                return {}
            gi = SpgemmInfo()
            Cg = graph.result(gi)
            if Cg is None or gi.nnz != nnz_local:
                raise SystemExit(f"[bench] graph replay disagrees with the eager product: nnz {gi.nnz} vs {nnz_local}")
            dig = lambda C: (C.col.long().sum().item(), C.val.double().sum().item())  # noqa: E731
            g_col, g_val = dig(Cg)
            rp_g = Cg.rowptr.clone()
            del Cg
            ne = max(1, min(args.steps, 5))
            Ce = eager_step()   # (warm: allocator)
            del Ce
            _sync_barrier(comm)
            t = time.perf_counter()
            for _ in range(ne):
                Ce = None
                Ce = eager_step()
            torch.cuda.synchronize()
            eager_ms = (time.perf_counter() - t) / ne * 1e3
            e_col, e_val = dig(Ce)
            same_rp = bool(torch.equal(rp_g, Ce.rowptr))
            del Ce, rp_g
            ok = same_rp and g_col == e_col and abs(g_val - e_val) <= 1e-5 * max(1.0, abs(e_val))
            if not ok:
                raise SystemExit(f"[bench] graph replay C differs from the eager C: rowptr equal {same_rp}, "
                                 f"col sums {g_col} / {e_col}, value sums {g_val} / {e_val}")
            return dict(graph_replay_nnz=gi.nnz, bitmap_cfg=gi.rows_per_bin_num.get("bitmap_cfg"),
                        bitmap_deferred=gi.rows_per_bin_num.get("bitmap_deferred"),
                        eager_ms_per_step=round(comm.allreduce_max(eager_ms), 3),
                        graph_vs_eager_check=dict(rowptr_equal=same_rp, col_sum=e_col, val_sum=e_val))
        if graph is not None:
            step.verify = verify
    total_flops = int(_allreduce_sum(comm, flops_local))
    total_nnz = _allreduce_sum(comm, nnz_local)
    extra = dict(nnz_A=int(_allreduce_sum(comm, prob.A.nnz)), nnz_C=int(total_nnz), hip_graph=graph is not None)
    return step, total_flops, extra, dict(model=model, n=n, density=density, dtype_values="fp32",
                                          global_batch=1, seq_len=n, parallelism=f"{'innerdim' if args.decomp == 'inner' else 'rowblock'}{comm.world}")


def run_rmat(comm, args):
    """BASELINE config 5: R-MAT A.A^T as a distributed 1D row-block workload
    (``models.spgemm.RmatProblem``): every rank generates its share of the
    edge chunks, the edges are shuffled to product-balanced row panels and
    transposed with all-to-all-v exchanges, and each step all-gathers A^T and
    multiplies the local A panel by it.  C is kept resident when its
    product-count bound fits this GPU; otherwise (scale 24: ~10^12 products,
    C of several TB) it is produced in row panels that are consumed and freed
    one at a time (``streamed_spgemm``; every product is still computed)."""
    import torch

    from spmm_amd.models import spgemm as MS
    from spmm_amd.ops.spgemm import SpgemmInfo, row_nprod

    prob = MS.RmatProblem.build(args.scale, args.edge_factor, comm, seed=args.seed)
    local_products = int(row_nprod(prob.A, prob.right_operand(comm)).sum())
    if comm.device.type == "cuda":
        torch.cuda.empty_cache()
    stream = args.rmat_stream == "on" or (args.rmat_stream == "auto" and local_products > MS.stream_budget(comm.device))
    info = SpgemmInfo()
    check = dict(panels=0, sum_val=0.0, sum_col=0)
    if stream:
        nnz = [0]

        def consume(_lo, _hi, C):   # count C's row panel and let it go (its last copies may still be running:
            nnz[0] += C.nnz         # every write ends inside the step's closing synchronise)

        def consume_check(_lo, _hi, C):   # setup run only (untimed): observe every panel
            check["panels"] += 1
            check["sum_val"] += float(C.val.double().sum())
            check["sum_col"] += int(C.col.long().sum())
            consume(_lo, _hi, C)

        prob.step(comm, info, consume_check)
        step = lambda: prob.step(comm, None, consume, overlap=True)  # noqa: E731
    else:
        C = prob.step(comm, info)
        check.update(panels=1, sum_val=float(C.val.double().sum()), sum_col=int(C.col.long().sum()))
        del C
        step = lambda: prob.step(comm)  # noqa: E731
    if comm.device.type == "cuda":
        torch.cuda.empty_cache()
    par = f"rowblock{comm.world}-product-balanced" + ("-streamed-C" if stream else "")
    return step, int(_allreduce_sum(comm, info.flops)), dict(
        nnz_A=int(_allreduce_sum(comm, prob.A.nnz)), nnz_C=int(_allreduce_sum(comm, info.nnz)), c_streamed=stream,
        # C observed in the untimed setup product: sums over all ranks' panels (unit weights: exact integers)
        c_checksum=dict(panels=int(_allreduce_sum(comm, check["panels"])),
                        sum_val=_allreduce_sum(comm, check["sum_val"]),
                        sum_col=int(_allreduce_sum(comm, check["sum_col"])))), dict(
        model=f"R-MAT scale-{args.scale} A.A^T", scale=args.scale, edge_factor=args.edge_factor, global_batch=1,
        seq_len=1 << args.scale, parallelism=par)


def run_spmm(comm, args):
    from spmm_amd.models import spmm as MM

    step, flops, extra, cfg = MM.bench_setup(comm, n=args.spmm_n, density=args.spmm_density, cols=128,
                                             seed=args.seed, method=args.spmm_method)
    return step, flops, extra, cfg


def run_chain(comm, args):
    """The reference's own workload the way its users run it: the native
    ``a4`` executable (``mpiexec -n N a4 <folder>``: parse the text files,
    reduce the chain on the GPUs, prune, write ``./matrix``), i.e. the
    end-to-end program of report.pdf Table 1.  The input folder (report tile
    count of the preset; chain shapes are ours) is generated once, untimed;
    every step is one complete a4 run (rank 0 launches it over all N GPUs,
    the other bench ranks wait at the barrier).  value = integer GOP/s of the
    whole program (2 k^3 per tile pair over its wall-clock); vs_baseline =
    report's optimized time for the preset / our time (P100 x 8 ranks)."""
    import shutil
    import subprocess
    import tempfile

    sys.path.insert(0, os.path.join(ROOT, "benches"))
    from bench_a4_e2e import REPORT, generate

    from spmm_amd import _build

    a4 = _build.A4_BIN if os.path.exists(_build.A4_BIN) else _build.build_a4()
    if a4 is None:
        raise SystemExit("native a4 not built (no MPI headers)")
    mpiexec = os.path.join(_build.mpi_home(), "bin", "mpiexec")
    work = tempfile.mkdtemp(prefix="bench_a4_")
    folder, out, met = os.path.join(work, "in"), os.path.join(work, "matrix"), os.path.join(work, "m.json")
    info = {}
    if comm.rank == 0:
        info = generate(folder, args.chain_preset, args.seed)
    comm.barrier()
    last = {}

    def step():
        if comm.rank == 0:
            cmd = [mpiexec, "-n", str(comm.world), a4, folder, "--quiet", "--out", out, "--metrics-json", met,
                   "--device", "hip" if comm.device.type == "cuda" else "cpu"]
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=1800)
            if r.returncode != 0:
                sys.stderr.write(r.stdout[-4000:] + r.stderr[-4000:])
                raise SystemExit(f"a4 failed with {r.returncode}")
            last["taken"] = max(float(x) for x in re.findall(r"time taken ([0-9.eE+-]+) seconds", r.stdout))
            last["metrics"] = json.load(open(met))
        comm.barrier()

    step()   # setup run: the op count (tile pairs of the exact tree)
    ops = float(last.get("metrics", {}).get("int_ops", 0.0))
    tiles_ref, t_opt, t_cpu = REPORT[args.chain_preset]
    extra = dict(tile_pairs=last.get("metrics", {}).get("tile_pairs"), engine="native a4 (csrc/runtime)",
                 report_optimized_s=t_opt, report_cpu_only_s=t_cpu, a4_time_taken_s=last.get("taken"),
                 a4_phases=last.get("metrics"), **{k: v for k, v in info.items() if k != "density"})
    cfg = dict(model=f"block-sparse uint64 chain, report {args.chain_preset} preset (k=32), native a4 end to end",
               global_batch=1, seq_len=info.get("n"), parallelism=f"chain-split{comm.world}")

    def cleanup():
        shutil.rmtree(work, ignore_errors=True)
    step.cleanup = cleanup
    return step, _allreduce_sum(comm, ops), extra, cfg   # (only rank 0 ran a4: the others add 0)


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _self_launch(n: int, backend: str) -> int:
    """``--gpus N`` without a launcher: start N rank processes (torchrun-style
    environment, one per GPU, rendezvous on 127.0.0.1) BEFORE this process
    touches the GPU, let rank 0's JSON line through on the shared stdout, and
    return the first failing exit code (the other ranks are stopped then:
    they would otherwise wait in a collective until the timeout)."""
    import subprocess

    import torch

    ndev = torch.cuda.device_count()   # (does not initialise the GPU)
    if ndev and ndev < n and backend != "gloo":
        print(f"[bench] --gpus {n} but only {ndev} GPU(s) visible; RCCL needs one GPU per rank "
              f"(rehearse several ranks on one card with --backend gloo)", file=sys.stderr, flush=True)
        return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                print(f"[bench] rank {procs.index(p)} exited with {code}; stopping the others", file=sys.stderr,
                      flush=True)
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    return rc


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="spgemm", choices=["spgemm", "spgemm64k", "spmm", "rmat", "chain"])
    ap.add_argument("--matrix-n", dest="n", type=int, default=1 << 20)
    ap.add_argument("--matrix-density", dest="density", type=float, default=1e-4)
    ap.add_argument("--spmm-n", type=int, default=65536)
    ap.add_argument("--spmm-density", type=float, default=1e-3)
    ap.add_argument("--spmm-method", default="auto", choices=["auto", "mfma", "panel", "sweep", "rowwise"],
                    help="spmm workload: executor (auto: the fastest measured on the real operands)")
    ap.add_argument("--scale", type=int, default=24, help="R-MAT scale (BASELINE config 5: 24)")
    ap.add_argument("--rmat-stream", default="auto", choices=["auto", "on", "off"],
                    help="produce C in consumed row panels (auto: when its product bound does not fit)")
    ap.add_argument("--edge-factor", type=int, default=16)
    ap.add_argument("--decomp", default="rowblock", choices=["rowblock", "inner"],
                    help="spgemm / spgemm64k: 1D row-block with B all-gathered (default), or inner-dimension "
                         "split with a sparse reduce-scatter of C")
    ap.add_argument("--chain-preset", default="medium", choices=["small", "medium", "large"],
                    help="chain workload: report preset (one folder, any N: strong scaling)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--graph", default="on", choices=["on", "off"],
                    help="spgemm / spgemm64k on one GPU: replay the product from a captured HIP graph")
    ap.add_argument("--backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="process-group backend (gloo on GPUs: rehearse several ranks on one card)")
    args = ap.parse_args()

    from spmm_amd.parallel.comm import launcher_env

    _, env_world, _ = launcher_env()
    launched = any(os.environ.get(v) for v in ("WORLD_SIZE", "PMI_SIZE", "OMPI_COMM_WORLD_SIZE", "SLURM_NTASKS"))
    if not launched and args.gpus > 1:
        sys.exit(_self_launch(args.gpus, args.backend))
    if launched and env_world != args.gpus:
        print(f"[bench] launcher world size {env_world} != --gpus {args.gpus}", file=sys.stderr, flush=True)
        sys.exit(2)

    if os.environ.get("SPMM_BENCH_DUMP_S"):   # diagnostics: every thread's stack every N seconds (stderr)
        import faulthandler

        faulthandler.dump_traceback_later(float(os.environ["SPMM_BENCH_DUMP_S"]), repeat=True)

    import torch

    import spmm_amd  # noqa: F401
    from spmm_amd import _native
    from spmm_amd.parallel import comm as CM

    comm = CM.init(backend=args.backend, device="auto")
    if comm.device.type == "cuda" and args.workload == "rmat":
        # the pipelined one-pass's side stream, created before any other stream of this process
        # (HIP hands streams hardware queues round-robin: a late one can share the main queue)
        from spmm_amd.ops import spgemm as _SG

        _SG._side_stream(comm.device)
    if comm.world != args.gpus:
        print(f"[bench] process group has {comm.world} rank(s), --gpus {args.gpus}", file=sys.stderr, flush=True)
        sys.exit(2)
    if comm.device.type == "cuda":
        _native.hip()
    if comm.rank == 0:
        import torch.distributed as dist

        pg = dist.get_world_size() if dist.is_initialized() else 1
        print(f"[bench] {args.workload}: process group up ({comm.world} rank(s), backend {comm.backend}, "
              f"torch.distributed world {pg}, {comm.device})", file=sys.stderr, flush=True)
    if args.workload == "spgemm":
        label = "1M" if args.n == 1 << 20 else str(args.n)
        step, flops, extra, cfg = run_spgemm(comm, args, args.n, args.density,
                                             f"{label}x{label} CSR SpGEMM at {args.density * 100:g}% density, "
                                             f"1D row-block via RCCL/xGMI")
    elif args.workload == "spgemm64k":
        step, flops, extra, cfg = run_spgemm(comm, args, 65536, 1e-3, "65536x65536 CSR SpGEMM at 0.1% density")
    elif args.workload == "rmat":
        step, flops, extra, cfg = run_rmat(comm, args)
    elif args.workload == "spmm":
        step, flops, extra, cfg = run_spmm(comm, args)
    else:
        step, flops, extra, cfg = run_chain(comm, args)

    if comm.rank == 0:
        print(f"[bench] setup done: {args.workload}, {comm.world} rank(s)", file=sys.stderr, flush=True)
    last = [time.perf_counter()]

    def progress(what: str, i: int) -> None:   # long steps (R-MAT scale 24: ~25 s on one GPU) report liveness
        now = time.perf_counter()
        if now - last[0] > 20.0 and comm.rank == 0:
            print(f"[bench] {what} {i + 1} done", file=sys.stderr, flush=True)
            last[0] = now

    for i in range(args.warmup):
        out = step()
        del out
        progress("warm-up", i)
    from spmm_amd.models.spgemm import GATHER_STATS

    stall = os.environ.get("SPMM_BENCH_STALL_RANK")   # fault injection (tests): this rank stops answering
    if stall not in (None, "") and int(stall) == comm.rank:
        time.sleep(float(os.environ.get("SPMM_BENCH_STALL_S", "600")))
    GATHER_STATS.reset(enabled=True)
    marks = []   # per-step boundaries on this rank: device events (no host sync) or host clock

    def mark():
        if comm.device.type == "cuda":
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            marks.append(ev)
        else:
            marks.append(time.perf_counter())

    _sync_barrier(comm)
    t0 = time.perf_counter()
    mark()
    for i in range(args.steps):
        out = None
        out = step()
        mark()
        progress("step", i)
    del out
    _sync_barrier(comm)
    t_local = time.perf_counter() - t0
    dt = comm.allreduce_max(t_local)
    GATHER_STATS.enabled = False
    ms = dt / args.steps * 1e3
    value = flops * args.steps / dt / 1e9
    # per-rank observability (after the timed region): this rank's step times
    # (device timeline between step boundaries), wall time, and the operand
    # all-gather's bytes and issue-to-ready time per step
    if comm.device.type == "cuda":
        steps_ms = [marks[i].elapsed_time(marks[i + 1]) for i in range(args.steps)]
    else:
        steps_ms = [(marks[i + 1] - marks[i]) * 1e3 for i in range(args.steps)]
    if hasattr(step, "verify"):
        extra.update(step.verify())
    g_bytes, g_ms = GATHER_STATS.summary()
    mine = torch.tensor([sum(steps_ms) / len(steps_ms), min(steps_ms), max(steps_ms), t_local * 1e3 / args.steps,
                         g_ms / args.steps, g_bytes / args.steps], dtype=torch.float64)
    if comm.is_dist:
        wire = torch.device("cuda", comm.device.index) if comm.device_collectives else torch.device("cpu")
        per_rank = comm.all_gather(mine.to(wire)).view(comm.world, -1).cpu()
    else:
        per_rank = mine.view(1, -1)
    import torch.distributed as dist

    col = lambda j: [round(float(x), 3) for x in per_rank[:, j]]  # noqa: E731
    observ = dict(
        torch_dist_world=dist.get_world_size() if dist.is_initialized() else 1,
        rank_step_ms=dict(min=round(float(per_rank[:, 0].min()), 3), mean=round(float(per_rank[:, 0].mean()), 3),
                          max=round(float(per_rank[:, 0].max()), 3)),
        per_rank=dict(step_ms_mean=col(0), step_ms_min=col(1), step_ms_max=col(2), wall_ms_per_step=col(3),
                      allgather_ms_per_step=col(4), allgather_bytes_per_step=[int(x) for x in per_rank[:, 5]]))
    vs = None
    unit = "GFLOP/s"
    metric = METRIC
    if args.workload == "chain":
        unit = "GOP/s (integer, 2k^3 per tile pair, whole program)"
        metric = "block-sparse uint64 chain, native a4 end to end (report.pdf Table 1)"
        vs = extra["report_optimized_s"] / (ms / 1e3)   # report's optimized wall-clock / ours
        if hasattr(step, "cleanup"):
            step.cleanup()
    elif args.workload == "spmm":
        metric = f"GFLOP/s (whole node), CSR x dense 128-col SpMM, bf16, {extra['spmm_kernel']}"
    if comm.rank == 0:
        rec = {"metric": metric, "value": round(value, 3), "unit": unit, "n_gpus": comm.world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
               "scaling": "strong", "vs_baseline": vs,
               "dtype": "fp32" if args.workload in ("spgemm", "spgemm64k", "rmat") else (
                   "bf16" if args.workload == "spmm" else "uint64"),
               "data": "synthetic (device RNG, random values)", "config": cfg, "flops_per_step": flops,
               "backend": comm.backend or "single-process",
               "device": torch.cuda.get_device_name(0) if torch.cuda.is_available() else "cpu", **extra, **observ}
        print(json.dumps(rec), flush=True)
    comm.close()


if __name__ == "__main__":
    main()
