#!/usr/bin/env python3
"""Benchmark: batched SRBD OCP-QP solves/sec on MI355X (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME] [--batch B]

A "step" is one solve of the whole per-rank batch (one C-ABI call, inputs
already resident in HBM).  Every rank generates its own shard of synthetic
SRBD QPs from seed + global QP index, so the data path has no
collective; `value` = QPs solved by all ranks / max-over-ranks wall time
("scaling": "weak").  After the timed region the solutions are gathered to
rank 0 over RCCL (BASELINE config 4) and that rate is reported separately.

Rank 0 prints ONE JSON line on stdout; progress goes to stderr.
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent
PKG_DIR = REPO / "srbd-nmpc-solver_amd"

METRIC = "SRBD OCP-QP solves/sec (N=20, nx=12, nu=12, fp64) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0    # MI355X_MICROARCH.md chip table (spec)
FP64_PEAK_TFS = 78.6     # FP64 vector/matrix
FP32_PEAK_TFS = 157.3    # FP32 vector (MI355X spec sheet; 2x FP64)

# solver settings of the reference caller (NMPC_solver.cpp:70-82)
NMPC_SETTINGS = {"mode": "Speed", "iter_max": 30, "alpha_min": 1e-8, "mu0": 1e2,
                 "tol_stat": 1e-4, "tol_eq": 1e-4, "tol_ineq": 1e-4, "tol_comp": 1e-4,
                 "reg_prim": 1e-12, "warm_start": 0, "pred_corr": 1, "ric_alg": 0, "split_step": 1}
# fp32: the stationarity floor of an fp32 iterate on SRBD data is ~1e-2
F32_SETTINGS = dict(NMPC_SETTINGS, tol_stat=3e-2, tol_eq=1e-3, tol_ineq=1e-3, tol_comp=1e-3)

WORKLOADS = {
    # name: (N, constraints, default batch, description[, dtype])
    "unconstr_n20": (20, "none", 65536,
                     "SRBD NMPC QP as the reference builds it (friction cone as barrier in the cost, "
                     "no inequalities), batch 65536, N=20"),
    "unconstr_n10_b4096": (10, "none", 4096, "BASELINE config 2: batch 4096, N=10"),
    "box_u_n20": (20, "box_u", 65536,
                  "BASELINE config 3: batch 65536, N=20, box constraints on u (IPM)"),
    "cone_n40_f32": (40, "cone", 65536,
                     "BASELINE config 5: batch 65536, N=40, friction-cone rows (ng=24), fp32 IPM",
                     "f32"),
    "cone_n40_f64": (40, "cone", 65536,
                     "config 5's problem solved in fp64 (batch 65536, N=40, friction-cone rows)"),
}
DEFAULT_WORKLOAD = "unconstr_n20"
# settings.f64_rescue of the cone_n40_f32_f64_rescue line (fp32 iterations before the fp64 re-solve)
RESCUE_CAP = 12
# settings.f32_iters of the box_u_n20_mixed line (fp32 iterations before fp64 takes over)
MIXED_F32_ITERS = 6
# ... and of the cone_n40_f64_mixed line (config 5's problem solved to fp64 tolerances)
MIXED_F32_ITERS_CONE = 9


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def import_pkg():
    name = "srbd_nmpc_solver_amd"
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, PKG_DIR / "__init__.py",
                                                  submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def alg_bytes_per_qp(N, nx=12, nu=12, constraints="none", elem=8, ng=24):
    """dense interface read once + x, u, pi written once."""
    stage = nx * nx + nx * nu + nx + nx * nx + nu * nx + nu * nu + nx + nu  # A B b Q S R q r
    vals = N * stage + nx * nx + nx + nx  # + terminal Q, q + x0
    if constraints == "box_u":
        vals += N * 2 * nu
    if constraints == "cone":
        vals += N * (ng * nu + 2 * ng)  # D, lg, ug per stage (C = 0 is passed as NULL)
    out = (N + 1) * nx + N * nu + (N + 1) * nx
    return elem * (vals + out)


def alg_flops_per_qp(N, nx=12, nu=12):
    """SURVEY.md 8(d) flop count of one Riccati factor + solve sweep."""
    n = nx + nu
    back = 2 * (n + 1) * nx * nx + 2 * nx * (n * (n + 1) // 2 + n) + n ** 3 / 3 + n * n + 2 * nx * nx * (nx + 1) / 2
    fwd = nu * nu + 2 * nu * nx + 2 * (n + 1) * nx + 2 * nx * nx
    return N * (back + fwd)


def make_cpu_sample(pkg, N, constraints, n, rank, batch, seed):
    """Host copy (numpy) of the first `n` QPs of this rank's shard, for the CPU
    baseline: the same seed + global index as the device batch."""
    first, _ = pkg.dist.shard_range(rank, batch)
    return pkg.srbd_model.generate_batch(n, N=N, seed=seed, constraints=constraints, first=first)


def device_shard(pkg, h, N, constraints, batch, rank, seed, device, np_dtype=np.float64,
                 stage_major=False):
    """Every QP of this rank's shard distinct: linearisation points sampled from
    seed + global QP index, then linearised on the device by
    srbd_qp_srbd_linearize_f64 (= prepareQpStructures, NMPC_solver.cpp:276-314;
    parity with the numpy model at 1e-11, tests/test_gpu_linearize.py).
    Returns (dict of device tensors in the C-ABI layout incl. x0, xs, us, x0 numpy)."""
    import torch
    first, _ = pkg.dist.shard_range(rank, batch)
    xs, us, x0 = pkg.srbd_model.sample_trajectories(batch, N, seed, pkg.srbd_model.SrbdParams(), first)
    xs_t = torch.from_numpy(xs).to(device)
    us_t = torch.from_numpy(us).to(device)
    t, _ = pkg.capi.srbd_linearize(h, xs_t, us_t, constraints)
    h.synchronize()
    del xs_t, us_t
    t["x0"] = torch.from_numpy(np.ascontiguousarray(x0)).to(device)
    tdt = torch.float32 if np_dtype == np.float32 else torch.float64
    dt = {}
    for k, v in t.items():
        v = v.to(tdt)
        if stage_major and k != "x0":  # [batch][stage][...] -> [stage][batch][...]
            v = v.transpose(0, 1)
        dt[k] = v.contiguous()
    torch.cuda.synchronize()
    return dt, xs, us, x0


def shard_buffers(capi, dt, batch, N, dtype, device):
    """Zeroed solution tensors (x, u, pi, status, iter) for one rank's shard and the
    C-ABI structs pointing at the shard's device data / solution."""
    import torch
    f = dict(dtype=torch.float32 if dtype == "f32" else torch.float64, device=device)
    sol_t = {"x": torch.zeros(batch, N + 1, 12, **f), "u": torch.zeros(batch, N, 12, **f),
             "pi": torch.zeros(batch, N + 1, 12, **f),
             "status": torch.zeros(batch, dtype=torch.int32, device=device),
             "iter": torch.zeros(batch, dtype=torch.int32, device=device)}
    DataT, SolT = (capi.Data32, capi.Solution32) if dtype == "f32" else (capi.Data, capi.Solution)
    data = DataT(**{k: (None if dt.get(k) is None else dt[k].data_ptr()) for k in capi.DATA_FIELDS})
    sol = SolT(**{k: (sol_t[k].data_ptr() if k in sol_t else None) for k in capi.SOL_FIELDS})
    return sol_t, data, sol


def gather_solutions(pkg, sol_t, world, rank, cpu_staged=False):
    """The config-4 gather: every rank's (x, u, pi) to rank 0 in one message per rank
    (RCCL over xGMI; cpu_staged=True stages through host memory for a gloo group).
    Returns the list of payloads on rank 0, None elsewhere."""
    payload = pkg.dist.solution_payload(sol_t["x"], sol_t["u"], sol_t["pi"])
    if cpu_staged:
        payload = payload.cpu()
    return pkg.dist.gather_to_root(payload, world, rank)


def baseline_config_name(workload, global_batch, world):
    """Which BASELINE.json config a run measures (None if it is none of them)."""
    if workload == "unconstr_n20" and global_batch == 262144 and world == 8:
        return "config 4: batch 262144, N=20, sharded 8 x MI355X with RCCL gather"
    if workload == "unconstr_n10_b4096" and global_batch == 4096:
        return "config 2: batch 4096, N=10"
    if workload == "box_u_n20" and global_batch == 65536:
        return "config 3: batch 65536, N=20, box constraints on u"
    if workload == "cone_n40_f32" and global_batch == 65536:
        return "config 5: batch 65536, N=40, friction cone, fp32"
    return None


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """`bench.py --gpus N` without an external launcher: start N rank processes
    of this same script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their
    environment, rendezvous on 127.0.0.1), wait for all of them and return the
    worst exit code.  Called before this process touches the GPU; the ranks are
    children, this process is not replaced.  Only rank 0 prints the JSON line."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:],
                                      env=env))
    log(f"[launcher] {n} ranks started (pids {[p.pid for p in procs]}, port {port})")
    rc, kill_at = 0, None
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                # one rank failed: the others would wait in a collective forever
                for q in pending:
                    q.terminate()
                kill_at = time.monotonic() + 15.0
        if kill_at is not None and time.monotonic() > kill_at:
            for q in pending:
                q.kill()
            kill_at = None
        time.sleep(0.05)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default=DEFAULT_WORKLOAD, choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=0, help="QPs per rank (default: workload's)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="QPs over all ranks, split evenly (strong scaling; BASELINE config 4 is "
                         "--gpus 8 --global-batch 262144)")
    ap.add_argument("--cpu-pool", type=int, default=4096, help="QPs in the cpu_baseline sample")
    ap.add_argument("--seed", type=int, default=1003)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="cpu_baseline budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--layout", choices=("qp", "stage"), default="qp",
                    help="input layout handed to the solver (stage: [stage][batch][block], "
                         "unconstrained workloads only)")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the host-buffer (PCIe-inclusive) measurement")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the IPM workloads (configs 3 and 5) measured beside the default line")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="skip the on-device SQP-iteration measurement (linearise + solve + line search)")
    ap.add_argument("--f64-rescue", type=int, default=0,
                    help="fp32 workloads: settings.f64_rescue = n (the fp32 pass runs at most n "
                         "iterations, the QPs it leaves unsolved are solved again in fp64)")
    ap.add_argument("--f32-iters", type=int, default=0,
                    help="fp64 IPM workloads: settings.f32_iters = n (mixed precision: the first n "
                         "IPM iterations in fp32, then fp64 to the fp64 tolerances)")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="process-group backend for N > 1: nccl (= RCCL over xGMI, one GPU per "
                         "rank) or gloo (host-staged gather; ranks may share a GPU, for tests)")
    ap.add_argument("--print-ranks", action="store_true",
                    help="print each rank's RANK / WORLD_SIZE / MASTER_* and exit (launcher check)")
    ap.add_argument("--mode", choices=("SpeedAbs", "Speed", "Balance", "Robust"), default=None,
                    help="IPM workloads: settings.mode instead of the NMPC's Speed (Balance / Robust "
                         "add HPIPM's iterative refinement of the corrector, DESIGN.md 4.8)")
    args = ap.parse_args()
    if args.mode:
        NMPC_SETTINGS["mode"] = args.mode
        F32_SETTINGS["mode"] = args.mode
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: start the N ranks ourselves, before anything touches the GPU
        sys.exit(launch_ranks(args.gpus))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: refusing to report "
                         f"a {world}-rank measurement as {args.gpus} GPUs")
    if args.print_ranks:  # launcher check: report this rank's environment, touch nothing
        print(json.dumps({"rank": rank, "local_rank": local_rank, "world": world,
                          "master": [os.environ.get("MASTER_ADDR"), os.environ.get("MASTER_PORT")]}),
              flush=True)
        return

    import torch
    import torch.distributed as dist

    distributed = world > 1
    gloo = args.dist_backend == "gloo"
    ndev = torch.cuda.device_count()  # counting devices does not initialise the GPU
    if distributed and not gloo and ndev < world:
        raise SystemExit(f"bench.py: {world} nccl ranks need {world} GPUs, {ndev} visible")
    dev_index = local_rank % max(ndev, 1) if gloo else local_rank
    if distributed:
        torch.cuda.set_device(dev_index)
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
    device = torch.device("cuda", dev_index)
    # the time reduction runs on the backend's own device type
    red_device = torch.device("cpu") if gloo else device
    pkg = import_pkg()
    capi = pkg.capi

    wl = WORKLOADS[args.workload]
    N, constraints, default_batch, desc = wl[:4]
    dtype = wl[4] if len(wl) > 4 else "f64"
    np_dtype = np.float32 if dtype == "f32" else np.float64
    batch = args.batch or default_batch
    if args.global_batch:
        if args.global_batch % world:
            raise SystemExit(f"--global-batch {args.global_batch} is not divisible by {world} ranks")
        batch = args.global_batch // world
    log(f"[rank {rank}] workload={args.workload} batch/rank={batch} N={N} world={world}")
    t0 = time.perf_counter()
    stage_major = args.layout == "stage"
    if stage_major and constraints != "none":
        raise SystemExit("--layout stage: unconstrained workloads only")
    ng = 24 if constraints == "cone" else 0
    h = capi.Handle(N, 12, 12, ng, constraints == "box_u", False, capacity=batch, device=dev_index,
                    layout=1 if stage_major else 0)
    dt, xs_np, us_np, x0_np = device_shard(pkg, h, N, constraints, batch, rank, args.seed, device,
                                           np_dtype, stage_major)
    log(f"[rank {rank}] {batch} distinct QPs generated (linearised on device) in "
        f"{time.perf_counter() - t0:.1f}s")

    sol_t, data, sol = shard_buffers(capi, dt, batch, N, dtype, device)
    # solver settings of the reference caller (NMPC_solver.cpp:70-82)
    settings = capi.settings_struct(F32_SETTINGS if dtype == "f32" else NMPC_SETTINGS)
    settings.f64_rescue = int(args.f64_rescue)
    settings.f32_iters = int(args.f32_iters)
    stream_ptr = h.stream()
    ext = torch.cuda.ExternalStream(stream_ptr, device=device)

    for _ in range(args.warmup):
        h.solve_device(batch, settings, data, sol)
    h.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t_start = time.perf_counter()
    ev0.record(ext)
    for _ in range(args.steps):
        h.solve_device(batch, settings, data, sol)
    ev1.record(ext)
    h.synchronize()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    t_wall = time.perf_counter() - t_start
    kernel_ms = ev0.elapsed_time(ev1) / args.steps
    t_max = pkg.dist.max_over_ranks(t_wall, red_device)
    rank_walls = [t_wall]
    if distributed:
        rank_walls = [None] * world
        dist.all_gather_object(rank_walls, t_wall)
    status = sol_t["status"].cpu().numpy()
    iters = sol_t["iter"].cpu().numpy()
    n_ok = int((status == 0).sum())
    log(f"[rank {rank}] wall {t_wall * 1e3:.2f} ms for {args.steps} steps, kernel avg {kernel_ms:.3f} ms, "
        f"success {n_ok}/{batch}")

    # ---- the whole SQP iteration on the device (secondary; not `value`) ----
    pipeline = None
    if not args.no_pipeline and dtype == "f64" and not stage_major:
        pipeline = sqp_pipeline(pkg, h, N, constraints, batch, xs_np, us_np, x0_np, device, settings)

    # ---- host buffers in, host buffers out (secondary; PCIe-inclusive, not `value`) ----
    host = None
    if not args.no_host_path and not stage_major and rank == 0:
        host = host_path(capi, h, dt, batch, N, settings, dtype)

    # ---- the reference's construct-solve-destroy call pattern, batch 1 (secondary) ----
    pattern = None
    if not args.no_host_path and rank == 0 and world == 1 and args.workload == DEFAULT_WORKLOAD:
        pattern = call_pattern(pkg, args.seed)

    # ---- solution gather to rank 0 over RCCL (BASELINE config 4) ----
    gather_ms = None
    if distributed and not args.no_gather:
        dist.barrier()
        torch.cuda.synchronize()
        tg = time.perf_counter()
        reps = 5
        for _ in range(reps):
            gather_solutions(pkg, sol_t, world, rank, cpu_staged=gloo)
        torch.cuda.synchronize()
        gather_ms = pkg.dist.max_over_ranks((time.perf_counter() - tg) / reps, red_device) * 1e3

    if rank != 0:
        if distributed:
            dist.barrier()
            dist.destroy_process_group()
        return

    total_qps = batch * world
    value = total_qps * args.steps / t_max
    ms_per_step = t_max / args.steps * 1e3
    bytes_qp = alg_bytes_per_qp(N, constraints=constraints, elem=4 if dtype == "f32" else 8)
    achieved_gbs = bytes_qp * batch / (kernel_ms * 1e-3) / 1e9
    flops_qp = alg_flops_per_qp(N)

    cpu = None
    if not args.no_cpu_baseline and world == 1:  # rank 0 at N = 1 only
        qp, x0 = make_cpu_sample(pkg, N, constraints, min(batch, args.cpu_pool), rank, batch, args.seed)
        cpu = cpu_baseline(pkg, qp, x0, settings_dict(settings), args.cpu_seconds)
        if dtype == "f32":
            cpu["sample"] += " (the oracle computes in fp64)"

    # ---- the IPM configurations (BASELINE configs 3 and 5) beside the default line ----
    secondary = None
    if not args.no_secondary and world == 1 and args.workload == DEFAULT_WORKLOAD:
        del h, dt, data, sol, sol_t
        torch.cuda.empty_cache()
        secondary = {w: secondary_workload(pkg, capi, w, device, args.seed)
                     for w in ("box_u_n20", "cone_n40_f32")}
        secondary["box_u_n20_mixed"] = secondary_workload(pkg, capi, "box_u_n20", device, args.seed,
                                                          f32_iters=MIXED_F32_ITERS)
        secondary["cone_n40_f64_mixed"] = secondary_workload(pkg, capi, "cone_n40_f64", device, args.seed,
                                                             f32_iters=MIXED_F32_ITERS_CONE)
        secondary["box_u_n20_balance"] = secondary_workload(pkg, capi, "box_u_n20", device, args.seed,
                                                            mode="Balance")
        secondary["cone_n40_f32_f64_rescue"] = secondary_workload(pkg, capi, "cone_n40_f32", device,
                                                                  args.seed, rescue=RESCUE_CAP)
        secondary["nmpc_step_config1"] = nmpc_config1(pkg, capi, device, args.seed,
                                                      with_cpu=not args.no_cpu_baseline)
        secondary["unconstr_n20_full_outputs"] = full_outputs_line(pkg, capi, device, args.seed)
        secondary["ipm_small_batch"] = ipm_small_batch(pkg, capi, device, args.seed,
                                                       with_cpu=not args.no_cpu_baseline)

    traffic = pmc_traffic(args.workload, batch)
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "QP solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if args.global_batch else "weak",
        "vs_baseline": None,
        "dtype": dtype + (f" (first {args.f32_iters} IPM iterations f32)"
                          if args.f32_iters and dtype == "f64" and constraints != "none" else "")
                 + (f" + f64 rescue after {args.f64_rescue} it" if args.f64_rescue and dtype == "f32" else ""),
        "data": f"synthetic SRBD linearisations (seed {args.seed} + global QP index; every QP of "
                f"the batch distinct, linearised on the device), generated per rank",
        "config": {"workload": args.workload, "description": desc, "batch_per_gpu": batch,
                   "global_batch": total_qps, "N": N, "nx": 12, "nu": 12, "constraints": constraints,
                   "parallelism": f"dp{world} (independent QP shards)",
                   "baseline_config": baseline_config_name(args.workload, total_qps, world),
                   "dist_backend": (args.dist_backend if distributed else None),
                   "rank_ms_per_step": [w / args.steps * 1e3 for w in rank_walls],
                   "input_layout": "stage-major" if stage_major else "qp-major",
                   "settings": ("NMPC_solver.cpp:70-82 (Speed, iter_max 30, split_step) with fp32 "
                                "tolerances stat 3e-2 / 1e-3" if dtype == "f32" else
                                "NMPC_solver.cpp:70-82 (Speed, iter_max 30, tol 1e-4, split_step)")},
        "roofline": roofline(constraints, achieved_gbs, traffic, kernel_ms, bytes_qp, flops_qp, batch,
                             iters, dtype),
        "fp_vector_frac_one_sweep": flops_qp * batch / (kernel_ms * 1e-3) /
                                    ((FP32_PEAK_TFS if dtype == "f32" else FP64_PEAK_TFS) * 1e12),
        "success_rate": n_ok / batch,
        "iters_mean": float(iters.mean()), "iters_max": int(iters.max()),
        "cpu_baseline": cpu,
    }
    if secondary is not None:
        line["ipm_workloads"] = secondary
    if pipeline is not None:
        line["sqp_pipeline"] = pipeline
    if host is not None:
        line["host_buffers"] = host
    if pattern is not None:
        line["reference_call_pattern"] = pattern
    if gather_ms is not None:
        elem = 4 if dtype == "f32" else 8
        line["gather"] = {"what": "x, u, pi of every rank to rank 0 (dist.gather, one message per rank"
                                  + (", host-staged over gloo)" if gloo else ", RCCL over xGMI)"),
                          "ms": gather_ms, "bytes_per_rank": batch * (2 * (N + 1) * 12 + N * 12) * elem,
                          "value_kernel_only": value,
                          "value_with_gather": total_qps / (t_max / args.steps + gather_ms * 1e-3)}
    print(json.dumps(line), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


def secondary_workload(pkg, capi, name, device, seed, steps=3, warmup=1, rescue=0, f32_iters=0,
                       mode=None):
    """One IPM workload (its own handle and synthetic shard) timed the same way as
    the main line: kernel time from HIP events on the handle's stream, wall time
    around `steps` solves.  Reported beside `value`, never as it.  rescue = n > 0 runs
    an fp32 workload with settings.f64_rescue = n (the fp32 pass capped at n
    iterations, the QPs it leaves unsolved solved again in fp64).  f32_iters = n > 0
    runs an fp64 workload as the mixed-precision IPM (settings.f32_iters: n fp32
    iterations, then fp64 to the fp64 tolerances) and reports its distance to the
    plain fp64 solve of the same shard.  mode = "Balance" / "Robust" runs it with
    HPIPM's iterative refinement of the corrector."""
    import torch
    N, constraints, batch, desc = WORKLOADS[name][:4]
    dtype = WORKLOADS[name][4] if len(WORKLOADS[name]) > 4 else "f64"
    ng = 24 if constraints == "cone" else 0
    h = capi.Handle(N, 12, 12, ng, constraints == "box_u", False, capacity=batch,
                    device=device.index or 0)
    dt, _, _, _ = device_shard(pkg, h, N, constraints, batch, 0, seed, device,
                               np.float32 if dtype == "f32" else np.float64)
    tt = dict(dtype=torch.float32 if dtype == "f32" else torch.float64, device=device)
    sol_t = {"x": torch.zeros(batch, N + 1, 12, **tt), "u": torch.zeros(batch, N, 12, **tt),
             "pi": torch.zeros(batch, N + 1, 12, **tt),
             "status": torch.zeros(batch, dtype=torch.int32, device=device),
             "iter": torch.zeros(batch, dtype=torch.int32, device=device)}
    DataT, SolT = (capi.Data32, capi.Solution32) if dtype == "f32" else (capi.Data, capi.Solution)
    data = DataT(**{k: (None if dt.get(k) is None else dt[k].data_ptr()) for k in capi.DATA_FIELDS})
    sol = SolT(**{k: (sol_t[k].data_ptr() if k in sol_t else None) for k in capi.SOL_FIELDS})
    settings = capi.settings_struct(F32_SETTINGS if dtype == "f32" else NMPC_SETTINGS)
    settings.f64_rescue = int(rescue)  # 0: off
    settings.f32_iters = int(f32_iters)  # 0: off
    if mode:
        settings.mode = capi.MODES[mode]
        desc += (f"; settings.mode = {mode}: HPIPM's iterative refinement of the corrector step "
                 "(the mode of the reference's own test, test/ocp_qp_ipm_solver.cpp:243)")
    ext = torch.cuda.ExternalStream(h.stream(), device=device)
    for _ in range(warmup):
        h.solve_device(batch, settings, data, sol)
    h.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(ext)
    for _ in range(steps):
        h.solve_device(batch, settings, data, sol)
    ev1.record(ext)
    h.synchronize()
    t_wall = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / steps
    status = sol_t["status"].cpu().numpy()
    iters = sol_t["iter"].cpu().numpy()
    elem = 4 if dtype == "f32" else 8
    bytes_qp = alg_bytes_per_qp(N, constraints=constraints, elem=elem)
    it = float(iters.mean())
    traffic = pmc_traffic(name, batch)
    mixed = None
    if f32_iters:
        desc += (f"; settings.f32_iters = {f32_iters}: the first {f32_iters} IPM iterations in fp32 "
                 "on a narrowed copy of the data, then fp64 from that iterate to the fp64 tolerances "
                 "(iter counts the fp64 iterations)")
        u_mix, x_mix = sol_t["u"].clone(), sol_t["x"].clone()
        settings.f32_iters = 0
        h.solve_device(batch, settings, data, sol)
        h.synchronize()
        # per-QP max-norm distance relative to the fp64 solution's max norm; both solves stop
        # at the NMPC tolerance (1e-4), so the worst QPs differ by a tolerance-level step
        rel = lambda a, b: ((a - b).abs().amax(dim=(1, 2)) / b.abs().amax(dim=(1, 2)))
        du, dx = rel(u_mix, sol_t["u"]), rel(x_mix, sol_t["x"])
        mixed = {"u_rel_diff_vs_fp64": {"max": float(du.max()), "median": float(du.median()),
                                        "p99": float(du.quantile(0.99))},
                 "x_rel_diff_vs_fp64": {"max": float(dx.max()), "median": float(dx.median()),
                                        "p99": float(dx.quantile(0.99))},
                 "fp64_success_rate": float((sol_t["status"] == 0).float().mean())}
    if rescue:
        desc += (f"; settings.f64_rescue = {rescue}: the fp32 pass runs at most {rescue} iterations, "
                 "the QPs it leaves unsolved are solved again in fp64 (their iter is the fp64 solve's)")
    dtype_s = dtype + ("+f64 rescue" if rescue else "") + (f" (first {f32_iters} iterations f32)"
                                                          if f32_iters else "")
    out = {"description": desc, "dtype": dtype_s, "batch": batch, "N": N, "steps": steps,
           "value": batch * steps / t_wall, "unit": "QP solves/s", "kernel_ms": kernel_ms,
           "success_rate": float((status == 0).mean()), "iters_mean": it,
           "iters_max": int(iters.max()),
           # the QP data must be streamed from HBM once per IPM iteration (it does not fit
           # on-chip): algorithmic bytes x iterations taken, against the 8 TB/s peak
           "hbm_alg_bytes_per_iter_frac": bytes_qp * it * batch / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
           "hbm_traffic_per_solve": traffic,
           "hbm_actual_tbs": None if traffic is None else traffic / (kernel_ms * 1e-3) / 1e12}
    if mixed is not None:
        out["mixed_precision"] = mixed
        # iterations of two precisions; the PMC traffic on file is the fp64 solve's
        out["hbm_alg_bytes_per_iter_frac"] = None
        out["hbm_traffic_per_solve"] = out["hbm_actual_tbs"] = None
    log(f"[secondary] {name}: kernel {kernel_ms:.2f} ms, {out['value']:.4g} QP/s, "
        f"success {out['success_rate']:.3f}, iters {it:.2f}")
    del h
    torch.cuda.empty_cache()
    return out


def ipm_small_batch(pkg, capi, device, seed, N=20, reps=20, with_cpu=True):
    """Small-batch IPM latency: box-u (config 3's QP) at batch 1 / 16 / 256 and the friction
    cone (config 5's QP, fp64) at batch 1, the NMPC settings, device buffers, one C-ABI call per
    solve, wall time per call (median).  Up to 512 QPs these run on the one-launch latency IPM
    (ipm_latency.hip); beside batch 1 box-u, the oracle's solve of the same QP on one host core.
    Batch 1 also with hpipm-cpp's default square-root Riccati (ric_alg 1, Speed and Balance: the
    `_ric1` cases) and the reference test's Balance with the classical Riccati (`_balance`)."""
    import torch
    ric1 = dict(NMPC_SETTINGS, ric_alg=1)
    cases = [("", "box_u", (1, 16, 256), NMPC_SETTINGS), ("", "cone", (1,), NMPC_SETTINGS),
             ("_balance", "box_u", (1,), dict(NMPC_SETTINGS, mode="Balance")),
             ("_ric1", "box_u", (1,), ric1), ("_ric1", "cone", (1,), ric1),
             ("_ric1_balance", "box_u", (1,), dict(ric1, mode="Balance"))]
    out = {"what": "wall ms per srbd_qp_solve_f64 call (launch + solve + sync), device buffers, "
                   "NMPC settings unless the case says otherwise; ipm_latency.hip up to 512 QPs",
           "N": N, "cases": {}}
    for tag, cons, batches, settings in cases:
        st = capi.settings_struct(settings)
        for b in batches:
            qp, x0 = pkg.srbd_model.generate_batch(b, N=N, seed=seed + 17, constraints=cons)
            h = capi.Handle(N, 12, 12, qp.ng, qp.has_box_u, qp.has_box_x, capacity=b,
                            device=device.index or 0)
            _, stt, data, sol = capi.device_buffers(qp, x0, str(device))
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps + 2):
                t0 = time.perf_counter()
                h.solve_device(b, st, data, sol)
                h.synchronize()
                ts.append(time.perf_counter() - t0)
            it = stt["iter"].cpu().numpy()
            out["cases"][f"{cons}_batch{b}{tag}"] = {
                "median_ms": float(np.median(ts[2:])) * 1e3, "min_ms": float(np.min(ts[2:])) * 1e3,
                "iters_mean": float(it.mean()), "success_rate": float((stt["status"].cpu().numpy() == 0).mean())}
            if with_cpu and cons == "box_u" and b == 1 and not tag:
                sys.path.insert(0, str(REPO / "oracle"))
                import oracle  # test infrastructure: CPU baseline leg only
                ts = []
                for _ in range(5):
                    t0 = time.perf_counter()
                    oracle.solve(qp, settings_dict(st), x0=x0, riccati=False)
                    ts.append(time.perf_counter() - t0)
                out["cpu_box_u_batch1"] = {"median_ms": float(np.median(ts)) * 1e3, "cores": 1, "kind": "port",
                                           "sample": "the same QP, oracle/ocp_qp_oracle.c through ctypes"}
            h.close()
    c = out["cases"]
    log("[secondary] ipm small batch: " + ", ".join(f"{k} {v['median_ms']:.3f} ms" for k, v in c.items()))
    torch.cuda.empty_cache()
    return out


def full_outputs_line(pkg, capi, device, seed, batch=65536, N=20, steps=5, warmup=1):
    """The headline workload with everything hpipm-cpp's solve() returns
    (ocp_qp_ipm_solver.cpp:337-403): x, u, pi plus the Riccati matrices P, p, K, k of
    every stage and the KKT residual norms / objective (stat row 0 too), i.e. the
    solve kernel writing P, p, K, k beside its records and the residual kernel's
    extra pass over the QP data.  Same timing as the main line (HIP events on the
    handle's stream)."""
    import torch
    h = capi.Handle(N, 12, 12, 0, False, False, capacity=batch, device=device.index or 0)
    dt, _, _, _ = device_shard(pkg, h, N, "none", batch, 0, seed, device)
    f = dict(dtype=torch.float64, device=device)
    s = {"x": torch.zeros(batch, N + 1, 12, **f), "u": torch.zeros(batch, N, 12, **f),
         "pi": torch.zeros(batch, N + 1, 12, **f),
         "P": torch.zeros(batch, N + 1, 12, 12, **f), "p": torch.zeros(batch, N + 1, 12, **f),
         "K": torch.zeros(batch, N, 12, 12, **f), "k": torch.zeros(batch, N, 12, **f),
         "status": torch.zeros(batch, dtype=torch.int32, device=device),
         "iter": torch.zeros(batch, dtype=torch.int32, device=device),
         "res": torch.zeros(batch, 4, **f), "obj": torch.zeros(batch, **f)}
    data = capi.Data(**{k: (None if dt.get(k) is None else dt[k].data_ptr()) for k in capi.DATA_FIELDS})
    sol = capi.Solution(**{k: (s[k].data_ptr() if k in s else None) for k in capi.SOL_FIELDS})
    st = capi.settings_struct(NMPC_SETTINGS)
    ext = torch.cuda.ExternalStream(h.stream(), device=device)
    for _ in range(warmup):
        h.solve_device(batch, st, data, sol)
    h.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(ext)
    for _ in range(steps):
        h.solve_device(batch, st, data, sol)
    ev1.record(ext)
    h.synchronize()
    t_wall = time.perf_counter() - t0
    ms = ev0.elapsed_time(ev1) / steps
    out_b = 8 * ((N + 1) * (144 + 12) + N * (144 + 12) + 4 + 1)  # P, p, K, k, res, obj
    res = s["res"].cpu().numpy()
    line = {"description": "unconstr_n20 with the whole hpipm-cpp output set: x, u, pi, P, p, K, k, "
                           "res (4 norms), obj; solve kernel + residual kernel",
            "batch": batch, "N": N, "steps": steps, "value": batch * steps / t_wall, "unit": "QP solves/s",
            "kernel_ms": ms, "success_rate": float((s["status"] == 0).float().mean()),
            "bytes_per_qp": {"algorithmic_x_u_pi": alg_bytes_per_qp(N), "extra_outputs": out_b,
                             "residual_pass_reads": alg_bytes_per_qp(N) - 8 * ((N + 1) * 12 + N * 12 + (N + 1) * 12)},
            "max_res_stat": float(res[:, 0].max()), "max_res_eq": float(res[:, 1].max())}
    log(f"[secondary] full outputs: kernel {ms:.2f} ms, {line['value']:.4g} QP/s")
    del h, dt, s
    torch.cuda.empty_cache()
    return line


def nmpc_config1(pkg, capi, device, seed, batch=65536, N=20, sqp_max_loop=15, reps=3,
                 with_cpu=True):
    """BASELINE config 1, batched: the reference's NMPC step (the SQP loop of
    NMPCSolver::controlLoop, NMPC_solver.cpp:362-372: linearise -> QP -> filter line
    search until converged, at most sqp_max_loop = 15) for `batch` robots, each from
    the reference's cold start (x_nmpc = 0, u_nmpc = 100, alpha_ = 1,
    NMPC_solver.cpp:56-64) with its own initial state x0 (the reference's x0 plus a
    seeded perturbation), on the device through srbd_qp_srbd_nmpc_f64.  Beside it,
    the same loop for the reference's own single robot on one host core (numpy
    model + C oracle QP + numpy line search: a port, the reference prints this as
    'Average NMPC solution time')."""
    import torch
    p = pkg.srbd_model.SrbdParams()
    _, _, dx0 = pkg.srbd_model.sample_trajectories(batch, N, seed + 7, p)
    x0_ref = np.zeros(12)
    x0_ref[8] = 1.0  # setupReference (NMPC_solver.cpp:343)
    x0 = torch.from_numpy(x0_ref + dx0).to(device)
    xs0 = torch.zeros(batch, N + 1, 12, dtype=torch.float64, device=device)
    us0 = torch.full((batch, N, 12), 100.0, dtype=torch.float64, device=device)
    h = capi.Handle(N, 12, 12, 0, False, False, capacity=batch, device=device.index or 0)
    times, it, cv = [], None, None
    for r in range(reps + 1):  # the first call allocates the scratch and warms up
        xs, us = xs0.clone(), us0.clone()
        al = torch.ones(batch, dtype=torch.float64, device=device)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        it, cv = capi.srbd_nmpc(h, xs, us, x0, al, "none", NMPC_SETTINGS, sqp_max_loop)
        torch.cuda.synchronize()
        if r:
            times.append(time.perf_counter() - t0)
    t = min(times)
    itn = it.cpu().numpy()
    out = {"what": "NMPCSolver::controlLoop SQP loop (config 1) per robot, batched on the device: "
                   "srbd_qp_srbd_nmpc_f64 (linearise + unconstrained QP + filter line search per "
                   "SQP iteration, until converged or 15 iterations)",
           "batch": batch, "N": N, "ms": t * 1e3, "nmpc_steps_per_s": batch / t,
           "sqp_iters_mean": float(itn.mean()), "sqp_iters_max": int(itn.max()),
           "converged_frac": float(cv.float().mean().item())}
    if with_cpu:
        sys.path.insert(0, str(REPO / "oracle"))
        import oracle  # test infrastructure: CPU baseline leg only
        import nmpc_linesearch as LS
        xs1, us1 = np.zeros((N + 1, 12)), np.full((N, 12), 100.0)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            _, _, _, n_it, ok = LS.sqp_loop(pkg.srbd_model, oracle, p, xs1, us1, x0_ref, 1.0,
                                            NMPC_SETTINGS, sqp_max_loop)
            ts.append(time.perf_counter() - t0)
        out["cpu_chain"] = {"ms_per_nmpc_step": min(ts) * 1e3, "sqp_iters": n_it, "converged": bool(ok),
                            "cores": 1, "kind": "port",
                            "sample": "the reference's own robot and start, 1 host core"}
    log(f"[secondary] nmpc config 1: {batch} robots in {t * 1e3:.1f} ms "
        f"({out['sqp_iters_mean']:.2f} SQP iterations mean, {out['converged_frac']:.3f} converged)")
    del h
    torch.cuda.empty_cache()
    return out


def host_path(capi, h, dt, batch, N, settings, dtype, max_batch=16384, reps=2):
    """srbd_qp_solve_host_*: the caller hands over pageable host buffers (the
    hpipm-cpp shim's situation, ocp_qp_ipm_solver.cpp:181-414); the library
    stages them H2D, solves and copies x, u, pi, status, iter back.  Timed on
    min(batch, max_batch) QPs after one warm call."""
    import torch
    nb = min(batch, max_batch)
    host = {k: (None if v is None else np.ascontiguousarray(v[:nb].cpu().numpy())) for k, v in dt.items()}
    npt = np.float32 if dtype == "f32" else np.float64
    out = {"x": np.zeros((nb, N + 1, 12), npt), "u": np.zeros((nb, N, 12), npt),
           "pi": np.zeros((nb, N + 1, 12), npt), "status": np.zeros(nb, np.int32),
           "iter": np.zeros(nb, np.int32)}
    DataT, SolT = (capi.Data32, capi.Solution32) if dtype == "f32" else (capi.Data, capi.Solution)
    data = DataT(**{k: (None if host.get(k) is None else host[k].ctypes.data) for k in capi.DATA_FIELDS})
    sol = SolT(**{k: (out[k].ctypes.data if k in out else None) for k in capi.SOL_FIELDS})
    h.solve_host(nb, settings, data, sol)
    t = time.perf_counter()
    for _ in range(reps):
        h.solve_host(nb, settings, data, sol)
    ms = (time.perf_counter() - t) / reps * 1e3
    nbytes = sum(v.nbytes for v in host.values() if v is not None) + sum(v.nbytes for v in out.values())
    # the reference's own call pattern: ONE QP per solve() (NMPC_solver.cpp:319), host buffers
    lat = []
    for _ in range(51):
        t1 = time.perf_counter()
        h.solve_host(1, settings, data, sol)
        lat.append(time.perf_counter() - t1)
    return {"what": "srbd_qp_solve_host: pageable host buffers -> H2D -> solve -> D2H (PCIe-inclusive)",
            "batch": nb, "ms_per_call": ms, "qps_per_s": nb / (ms * 1e-3),
            "host_bytes_moved": nbytes, "status_ok": float((out["status"] == 0).mean()),
            "latency_batch1_ms": float(np.median(lat[1:])) * 1e3}


def call_pattern(pkg, seed, N=20, reps=20, oracle_reps=400):
    """The reference caller's own pattern (NMPC_solver.cpp:316-330, 362-372): per SQP
    iteration a fresh hpipm::OcpQpIpmSolver is constructed, solves ONE SRBD QP from
    host Eigen-layout buffers and is destroyed, 15 times per NMPC step.  Timed by the
    compiled C++ program build/call_pattern_bench through libhpipm-cpp.so (handles come
    from the shim's pool, the host staging is pinned), beside the C oracle solving the
    same QP on one host core."""
    import subprocess
    import tempfile
    exe = REPO / "build" / "call_pattern_bench"
    if not exe.exists():
        return {"error": f"{exe} not built"}
    qp, x0 = pkg.srbd_model.generate_batch(1, N=N, seed=seed)
    p = qp.packed()
    vals = [np.array([float(N)])]
    for k in range(N):
        for name in ("A", "B", "b", "Q", "S", "R", "q", "r"):
            vals.append(p[name][0].reshape(N + (1 if name in ("Q", "q") else 0), -1)[k])
    vals += [p["Q"][0].reshape(N + 1, -1)[N], p["q"][0].reshape(N + 1, -1)[N], x0[0]]
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(np.concatenate(vals).astype("<f8").tobytes())
        path = f.name
    try:
        r = subprocess.run([str(exe), path, str(reps)], capture_output=True, text=True, timeout=300)
    finally:
        os.unlink(path)
    if r.returncode != 0:
        return {"error": (r.stdout + r.stderr)[-2000:]}
    out = json.loads(r.stdout.strip().splitlines()[-1])
    sys.path.insert(0, str(REPO / "oracle"))
    import oracle  # test infrastructure: CPU baseline leg only
    oracle.solve_batch_threaded(qp, NMPC_SETTINGS, x0, 1)
    ts = []
    for _ in range(oracle_reps):
        _, d = oracle.solve_batch_threaded(qp, NMPC_SETTINGS, x0, 1)
        ts.append(d)
    out["what"] = ("NMPC_solver.cpp:316-330 call pattern through hpipm-cpp: construct OcpQpIpmSolver, "
                   "solve one SRBD QP (N=20) from host buffers, destroy; 15 per NMPC step")
    out["oracle_1_core_us"] = {"median": float(np.median(ts)) * 1e6, "min": float(np.min(ts)) * 1e6,
                               "kind": "port", "cores": 1}
    # the fixed-size CPU port (oracle/fast_unconstr.c) on the same QP, one core
    oracle.fast_unconstr_batch(qp, x0, 1)
    ts = [oracle.fast_unconstr_batch(qp, x0, 1)[1] for _ in range(oracle_reps)]
    out["cpu_port_1_core_us"] = {"median": float(np.median(ts)) * 1e6, "min": float(np.min(ts)) * 1e6,
                                 "kind": "port", "cores": 1, "src": "oracle/fast_unconstr.c"}
    return out


def sqp_pipeline(pkg, h, N, constraints, batch, xs, us, x0, device, settings, iters=3):
    """One SQP iteration of NMPCSolver::controlLoop (NMPC_solver.cpp:362-372) for the
    whole batch on the device: srbd_qp_srbd_linearize_f64 -> solve ->
    srbd_qp_srbd_linesearch_f64, timed with HIP events on the handle's stream."""
    import torch
    capi = pkg.capi
    up = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
    xs_t, us_t, x0_t = up(xs), up(us), up(x0)
    alpha = torch.ones(batch, dtype=torch.float64, device=device)
    f64 = dict(dtype=torch.float64, device=device)
    sol = {"x": torch.zeros(batch, N + 1, 12, **f64), "u": torch.zeros(batch, N, 12, **f64),
           "pi": torch.zeros(batch, N + 1, 12, **f64)}
    S = capi.Solution(**{k: (sol[k].data_ptr() if k in sol else None) for k in capi.SOL_FIELDS})
    t, data = capi.srbd_linearize(h, xs_t, us_t, constraints)
    dx0 = torch.empty_like(x0_t)
    merit = torch.empty(batch, 3, **f64)
    conv = torch.empty(batch, dtype=torch.int32, device=device)
    ext = torch.cuda.ExternalStream(h.stream(), device=device)
    lp, mp = capi.default_linesearch(), capi.default_model_params()
    ptr = lambda x: capi.C.c_void_p(x.data_ptr())
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    tot = [0.0, 0.0, 0.0]
    h.synchronize()
    for it in range(iters + 1):  # iteration 0 warms up (lazy torch / HIP init on the stream)
        ev[0].record(ext)
        capi.srbd_linearize(h, xs_t, us_t, constraints, out=t)
        ev[1].record(ext)
        with torch.cuda.stream(ext):
            torch.sub(x0_t, xs_t[:, 0], out=dx0)  # x0 - x_nmpc(:,0) (NMPC_solver.cpp:320)
        data.x0 = dx0.data_ptr()
        h.solve_device(batch, settings, data, S)
        ev[2].record(ext)
        capi.check(capi.lib().srbd_qp_srbd_linesearch_f64(
            h.ptr, batch, capi.C.byref(mp), capi.C.byref(lp), ptr(xs_t), ptr(us_t), ptr(sol["x"]),
            ptr(sol["u"]), ptr(alpha), ptr(merit), ptr(conv), None), "linesearch")
        ev[3].record(ext)
        h.synchronize()
        if it > 0:
            for j in range(3):
                tot[j] += ev[j].elapsed_time(ev[j + 1])
    lin, solve, ls = (x / iters for x in tot)
    return {"what": "SQP iteration of NMPC_solver.cpp:362-372 on device: linearise + QP solve + "
                    "filter line search, whole batch, inputs/outputs resident",
            "iterations_timed": iters, "ms_linearize": lin, "ms_qp_solve": solve,
            "ms_line_search": ls, "ms_per_sqp_iteration": lin + solve + ls,
            "sqp_iterations_per_s": batch / ((lin + solve + ls) * 1e-3),
            "converged_after": float(conv.float().mean().item())}


def roofline(constraints, achieved_gbs, traffic, kernel_ms, bytes_qp, flops_qp, batch, iters,
             dtype="f64"):
    """HBM roofline of the solve.  Unconstrained: one streaming sweep,
    achieved = algorithmic bytes per launch / kernel time.  IPM: the QP data does not
    fit on-chip, so every iteration re-streams it; achieved = algorithmic bytes x
    iterations taken / kernel time, against the same 8 TB/s peak (no MFMA is used:
    the 12 x 12 blocks run on the FP vector pipe)."""
    if constraints == "none":
        prof, prof_ns = pmc_profile("unconstr_n20" if batch == 65536 else "", batch)
        ceil = unconstr_ceiling(bytes_qp, batch)
        return {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
                # what bounds frac for this algorithm: the two-sweep Riccati must
                # move the algorithmic bytes + its stage records (written, read back) + the A, B, b
                # the forward sweep reads again; at the guide's achievable rate that caps frac
                "ceiling": ceil["ceiling"], "frac_of_ceiling": (achieved_gbs / HBM_PEAK_GBS) / ceil["ceiling"],
                "ceiling_derivation": ceil,
                "traffic_profile": prof, "profile_kernel_avg_ms": None if prof_ns is None else prof_ns * 1e-6,
                # template argument = square-root Riccati (ric_alg; NMPC_solver.cpp:81 sets 0)
                "kernel": "riccati_unconstr_kernel<%s>" % ("true" if NMPC_SETTINGS["ric_alg"] else "false"),
                "kernel_avg_ms": kernel_ms,
                "alg_bytes_per_qp": bytes_qp}
    it = max(float(np.mean(iters)), 1.0)
    gbs = achieved_gbs * it
    peak = FP32_PEAK_TFS if dtype == "f32" else FP64_PEAK_TFS
    tf = flops_qp * 1.4 * it * batch / (kernel_ms * 1e-3) / 1e12
    return {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": gbs / HBM_PEAK_GBS, "traffic": traffic,
            "kernel": "ipm_phase_kernel<*> (init, RB+F1, B2+F2, out; whole solve)",
            "kernel_avg_ms": kernel_ms, "alg_bytes_per_qp_iter": bytes_qp, "mean_iters": it,
            "fp_vector_frac": tf / peak}


HBM_ACHIEVABLE_GBS = 6300.0  # MI355X_MICROARCH.md: "8 TB/s peak (spec); ~6.3 TB/s achievable"


def unconstr_ceiling(bytes_qp, batch, N=20, nx=12, nu=12):
    """The roofline fraction the two-sweep Riccati can reach.  Per QP it moves
    the algorithmic bytes (inputs once, x / u / pi once) plus, per stage, its record
    ([K | k], P packed, p: csrc/kernels.h kWsStage = 246 doubles) written by the backward
    sweep and read back by the forward sweep, plus the A, B, b the forward sweep reads again
    (x+ = A x + B u + b).  At the achievable HBM rate the fraction of the 8 TB/s peak that
    counts as algorithmic is then bytes_qp / min_traffic x achievable / peak."""
    rec = N * 246 * 8 * 2
    fwd = N * (nx * nx + nx * nu + nx) * 8
    min_traffic = bytes_qp + rec + fwd
    return {"alg_bytes_per_qp": bytes_qp, "record_round_trip_per_qp": rec, "forward_reread_per_qp": fwd,
            "min_traffic_per_qp": min_traffic, "achievable_gbs": HBM_ACHIEVABLE_GBS,
            "ceiling": bytes_qp / min_traffic * HBM_ACHIEVABLE_GBS / HBM_PEAK_GBS}


def settings_dict(s):
    return {k: getattr(s, k) for k, _ in s._fields_}


def cpu_baseline(pkg, qp, x0, settings, budget_s):
    """A CPU port on the host cores over a bounded sample of the same workload: for
    unconstrained 12 x 12 QPs the fixed-size vectorised port (oracle/fast_unconstr.c,
    x, u, pi only, as the GPU line), otherwise the generic C oracle (same algorithm,
    scalar C, -O3, x86-64-v3)."""
    sys.path.insert(0, str(REPO / "oracle"))
    import oracle  # test infrastructure, used here only as the CPU baseline
    fast = qp.ng == 0 and qp.nx == 12 and qp.nu == 12 and not _has_bounds(qp)
    if fast:
        run = lambda b, x, t: oracle.fast_unconstr_batch(b, x, t, settings.get("reg_prim", 1e-12))
        src = "oracle/fast_unconstr.c: fixed 12 x 12 port, AVX2 + FMA"
    else:
        run = lambda b, x, t: oracle.solve_batch_threaded(b, settings, x, t)
        src = "oracle/ocp_qp_oracle.c"
    # the GPU box's CPU share is OMP_NUM_THREADS (16 per GPU there); nproc shows
    # the whole machine
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or avail
    threads = max(1, min(threads, avail, 64))
    # calibrate on a slice big enough that thread start-up does not dominate,
    # then repeat the slice until the budget is spent
    cal = qp.subset(slice(0, min(qp.batch, 64 * threads)))
    _, dt = run(cal, x0[:cal.batch], threads)
    rate = cal.batch / max(dt, 1e-9)
    n = int(min(qp.batch, max(cal.batch, rate * budget_s / 4)))
    sample = qp.subset(slice(0, n))
    t, reps = 0.0, 0
    while t < budget_s:
        _, d = run(sample, x0[:n], threads)
        t += d
        reps += 1
    return {"value": n * reps / t, "unit": "QP solves/s", "cores": threads, "kind": "port",
            "sample": f"{n} QPs x {reps} reps of the same workload ({t:.1f} s, {threads} threads, {src})"}


def _has_bounds(qp):
    return any(getattr(qp, k) is not None for k in ("lbu", "ubu", "lbx", "ubx"))


def pmc_profile(workload, batch):
    """(profile summary file, its kernel's average ns) behind pmc_traffic, if any."""
    f = REPO / "profiles" / "pmc_traffic.json"
    try:
        e = json.loads(f.read_text()).get(workload)
        if e and int(e.get("batch", -1)) == batch:
            return e.get("profile"), e.get("avg_ns")
    except Exception:
        pass
    return None, None


def pmc_traffic(workload, batch):
    """HBM bytes per launch (unconstrained: the one kernel; IPM: one whole solve)
    from the committed rocprofv3 PMC summary, if any."""
    f = REPO / "profiles" / "pmc_traffic.json"
    if not f.exists():
        return None
    try:
        d = json.loads(f.read_text())
        e = d.get(workload)
        if e and int(e.get("batch", -1)) == batch:
            # IPM workloads: the whole solve (every phase launch of it) is the unit
            if WORKLOADS[workload][1] != "none" and e.get("per_solve"):
                return e["per_solve"].get("hbm_bytes")
            return e.get("hbm_bytes_per_launch")
    except Exception:
        return None
    return None


if __name__ == "__main__":
    main()
