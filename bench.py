#!/usr/bin/env python3
"""Benchmark: Hessian-rows/sec of the gradient/Hessian inner loop on MI355X.

Workload (BASELINE.json configs[1]/[2]): Bose-Hubbard chain
L=5, Npart=5, d=4 (p=5), maxBondDim=80, cutoff 1e-8, J=1, tstep=0.01, T=2.0
(N_t=201), GRAPE controls u_i ~ U(2,10) (seed 20261015), psi_init/psi_target
= ground states at U=2.5/50 (exact diagonalisation; synthetic controls).

One "step" = one full getHessian(u, new_control=true)
(src/OptimalControl.cpp:341-372) per rank: psi_t and xi_t trajectories, divT,
overlapFactor, xiHlist and all N_t-2 = 199 Hessian rows, plus the gradient
assembly.  Multi-GPU (one process per GPU):
  --mode weak   (default) every rank evaluates the Hessian of its own control
                vector (independent units, fixed work per GPU, no data-path
                collective): value scales with N.
  --mode strong one control vector; its rows are dealt zig-zag over the ranks
                (each rank recomputes the 400-step precompute) and the N_t x N_t
                partial Hessians are summed onto rank 0 with one RCCL reduce.
                At config 1 one GPU already runs all 199 rows concurrently, so
                the critical path (~200 steps) does not shrink with N.

value = Hessian rows completed per second (whole job).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CFG = dict(L=5, p=5, npart=5, J=1.0, tstep=0.01, T=2.0, maxm=80, cutoff=1e-8, U_init=2.5, U_target=50.0,
           seed=20261015)
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_PEAK_TFS = 78.6       # MI355X FP64 vector/matrix spec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=8)
    ap.add_argument("--mode", choices=["weak", "strong"], default="weak")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(backend="nccl")
    dev = torch.device("cuda", local)

    from optimalcontrolmps_amd import ed
    from optimalcontrolmps_amd.native import MPS, Engine
    from optimalcontrolmps_amd.sharding import zigzag_rows

    L, p, Q, J, dt = CFG["L"], CFG["p"], CFG["npart"], CFG["J"], CFG["tstep"]
    Nt = int(round(CFG["T"] / dt)) + 1
    ini = MPS(L, p, Q, *ed.mps_from_full(ed.ground_state_full(L, p, Q, J, CFG["U_init"])[0], L, p, Q))
    tgt = MPS(L, p, Q, *ed.mps_from_full(ed.ground_state_full(L, p, Q, J, CFG["U_target"])[0], L, p, Q))
    strong = args.mode == "strong"
    # weak: rank r evaluates its own control vector (seed + r); strong: one shared vector
    u = np.random.default_rng(CFG["seed"] + (0 if strong else rank)).uniform(2.0, 10.0, Nt)
    rows = zigzag_rows(Nt - 2, rank, world) if strong else list(range(1, Nt - 1))

    eng = Engine(L, p, Q, J, dt, CFG["cutoff"], CFG["maxm"], device=local)
    eng.set_states(tgt, ini)
    Hdev = torch.zeros((Nt, Nt), dtype=torch.float64, device=dev)

    def one_step():
        # fused getHessian: psi/xi chains, xiHlist and this rank's rows in one
        # pipelined launch (rows start as their psi_i appears), then divT, F
        # and the batched <xiH_j|psiH> overlaps (ocg_hessian)
        H, divT, F = eng.hessian(u, rows)
        g = dt * (divT * F * 1j).real            # calcFidelityGrad (gamma = 0)
        if world > 1 and strong:
            Hdev.copy_(torch.from_numpy(H))
            dist.reduce(Hdev, dst=0)             # RCCL sum of disjoint row entries
        return g, H

    for _ in range(args.warmup):
        one_step()
    eng.reset_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    rows_total = (Nt - 2) * args.steps * (1 if strong else world)
    value = rows_total / elapsed
    st_rows = eng.stats(5)       # k_pipeline: trajectories + row re-propagation (dominant)
    st_ovl = eng.stats(6)        # k_row_overlaps
    st_traj = eng.stats(0)
    row_steps = (Nt - 2) * (Nt - 3) // 2
    sweep_steps = args.steps * (2 * (Nt - 1) * world + row_steps * (1 if strong else world))
    result = None
    if rank == 0:
        launch_ms = st_rows["ms"] / max(1, st_rows["launches"])
        bytes_per_launch = st_rows["alg_bytes"] / max(1, st_rows["launches"])
        flops_per_launch = st_rows["alg_flops"] / max(1, st_rows["launches"])
        achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9 if launch_ms > 0 else 0.0
        result = {
            "metric": "Hessian-rows/sec (getHessian incl. psi/xi/divT/xiH precompute), N=5 d=4 chi=80 T=2.0",
            "value": value,
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": args.mode,
            "vs_baseline": None,
            "dtype": "c128/f64",
            "data": "synthetic GRAPE controls U(2,10) seed 20261015; ED ground states U=2.5 -> 50",
            "config": {"workload": "getHessian(u, new_control=true), config 1 (L=5 Npart=5 d=4 maxBondDim=80 "
                                   "tstep=0.01 T=2.0 GRAPE, N_t=201, 199 rows)",
                       "rows_per_step": (Nt - 2) * (1 if strong else world),
                       "parallelism": (f"one control, rows sharded zig-zag over {world} GPU(s) + RCCL reduce" if strong
                                       else f"{world} GPU(s), one full getHessian (own control vector) per GPU")},
            "sweep_steps_per_sec": sweep_steps / elapsed,
            "kernels": {
                "pipeline": {"avg_ms": launch_ms, "launches": st_rows["launches"]},
                "row_overlaps": {"avg_ms": st_ovl["ms"] / max(1, st_ovl["launches"]), "launches": st_ovl["launches"]},
                "divT_F_overlaps_ms": eng.stats(1)["ms"] / max(1, args.steps),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "k_pipeline",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": measured_traffic("k_pipeline"),
                "alg_bytes_per_launch": bytes_per_launch,
                "fp64_achieved_tflops": flops_per_launch / (launch_ms * 1e-3) / 1e12 if launch_ms > 0 else 0.0,
                "fp64_peak_tflops": FP64_PEAK_TFS,
            },
        }
        if world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(ini, tgt, u, args.cpu_threads)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def measured_traffic(kernel, tag="r01"):
    """HBM bytes per dispatch of `kernel` from the committed rocprofv3 PMC passes
    of this same command (profiles/<tag>_summary.json, written by
    tools/prof_summary.py; FETCH_SIZE doubled per the gfx950 calibration)."""
    try:
        with open(os.path.join(ROOT, "profiles", f"{tag}_summary.json")) as f:
            return json.load(f)["pmc_per_dispatch"][kernel]["hbm_bytes"]
    except (OSError, KeyError, ValueError):
        return None


def cpu_baseline(ini, tgt, u, threads):
    """The CPU restatement (oracle/, 'port' — ITensor cannot be built here) timed
    on host cores: full getHessian with a row worker pool like
    calcHessian_parallel (src/OptimalControl.cpp:281-338)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    L, p, Q, J, dt = CFG["L"], CFG["p"], CFG["npart"], CFG["J"], CFG["tstep"]
    threads = max(1, min(threads, os.cpu_count() or 1))
    st = O.Stepper(L, p, Q, J, dt, CFG["cutoff"], CFG["maxm"])
    oc = O.OC(st, O.MPS(L, p, Q, tgt.dims, tgt.data), O.MPS(L, p, Q, ini.dims, ini.data), len(u), 0.0)
    reps, total = 0, 0.0
    while total < 10.0 and reps < 8:
        total += oc.time_hessian(u, threads)
        reps += 1
    Nt = len(u)
    return {"value": reps * (Nt - 2) / total, "unit": "rows/s", "cores": threads, "kind": "port",
            "sample": f"{reps} full getHessian calls (config 1, 199 rows each) on the C++ CPU restatement "
                      f"(oracle/, not ITensor), {threads} row-worker threads, {total:.1f} s"}


if __name__ == "__main__":
    main()
