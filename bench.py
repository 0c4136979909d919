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

Other workloads (--workload; one JSON line each, not the driver's default):
  gradient   config 2: getAnalyticGradient with BFGS=true (psi and xi chains
             concurrently, divT, F; src/OptimalControl.cpp:204-249) at config 1,
             value = gradients/s.
  c4grad     config 4 chain (L=20 Npart=20 d=6 chi=256 tstep=0.005): one
             getAnalyticGradient over the full horizon T=4 (N_t=801) from the
             saturated warm state, value = gradients/s (+ sweep-steps/s).
  c4rows     config 4 chain: getHessian fidelity part over a T slice
             (--c4-nt time points, default 33: all N_t-2 rows), value = rows/s.
The roofline block names the limiter honestly: config 1 is latency-bound (one
chain's 200 dependent steps on one CU, state in LDS), so `frac` is reported
against HBM for the contract but the measured HBM bytes (rocprofv3 PMC,
profiles/) sit next to the model bytes.
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
FP64_MFMA_MEASURED_TFS = 48.7   # v_mfma_f64_16x16x4f64 issue rate measured on the box (tools/mfma_f64_peak.hip)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one process per GPU); without an outer launcher bench.py spawns them itself")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="largest CPU-baseline thread count (0: all available)")
    ap.add_argument("--mode", choices=["weak", "strong"], default=None,
                    help="weak: every rank its own getHessian; strong: one getHessian's rows over the ranks "
                         "(default: weak for config 1, strong for c4rows / c5rows)")
    ap.add_argument("--group-m", type=int, default=40, help="GROUP basis size of the c4rows workload (0: GRAPE)")
    ap.add_argument("--workload", choices=["hessian", "gradient", "c4grad", "c5grad", "c4rows", "c5rows"], default="hessian")
    ap.add_argument("--c4-nt", type=int, default=33)
    ap.add_argument("--c5-nt", type=int, default=17)
    ap.add_argument("--c5-warm", type=int, default=230)
    ap.add_argument("--last-rows", type=int, default=0,
                    help="c4rows / c5rows: only the last R interior rows of H (R >= 1; with --c4-nt 801 / --c5-nt "
                         "1001 the full horizon, where config 5 selects the trajectory checkpointing by itself)")
    ap.add_argument("--row-stride", type=int, default=1,
                    help="c4rows / c5rows: every S-th interior row only (rows 1, 1 + S, ...): a sample of a full "
                         "horizon whose rows span every length; the whole getHessian is priced from it")
    ap.add_argument("--state-cache", default="",
                    help="c4/c5 workloads: npz of psi_init and psi_target, loaded when it exists, else written after "
                         "they are prepared (so a profiled command holds only getHessian launches)")
    ap.add_argument("--prepare-only", action="store_true",
                    help="c4/c5 workloads: prepare the states (and write --state-cache), then exit")
    ap.add_argument("--controls", type=int, default=1,
                    help="K control vectors per GPU evaluated concurrently (K contexts, one host thread and "
                         "stream each: IPOPT trial points / multi-start); value = rows of all K per second")
    ap.add_argument("--multi", type=int, default=1,
                    help="K control vectors per GPU in one ocg_hessian_multi call (one pipeline launch for all K); "
                         "value = rows of all K per second")
    ap.add_argument("--profile-tag", default="r06")
    ap.add_argument("--profiled", action="store_true",
                    help="run only the warm-up and timed getHessian calls (no single-chain probe, no config-2 "
                         "block, no config-4 / config-5 slice blocks, no CPU baseline): the command rocprofv3 "
                         "profiles, so every dispatch of a kernel belongs to the population the roofline divides by")
    ap.add_argument("--no-slices", action="store_true",
                    help="config 1 at N=1: skip the config-4 / config-5 slice blocks (child processes run before "
                         "the config-1 line)")
    ap.add_argument("--c4-cpu-nt", type=int, default=5,
                    help="time points of the measured oracle getHessian in the c4rows CPU baseline (0: skip)")
    ap.add_argument("--multi-info", action="store_true",
                    help="after the timed region also time 8 Hessians / 64 gradients per call (ocg_*_multi; "
                         "their k_pipeline launches would enter a rocprofv3 summary of the command)")
    return ap.parse_args(argv)


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_entry(rank, world, port, argv, target):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.exit(target(argv) or 0)


def spawn_ranks(world, argv, target=None):
    """`bench.py --gpus N` without an outer launcher: N rank processes started
    with the spawn method while this process has not touched the GPU (it never
    does: no HIP call, no exec), each with the RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* environment torch.distributed.run would give it.  When a rank fails
    the others are terminated (a peer left waiting in a collective would hang);
    returns the first non-zero exit code, 0 when every rank succeeded."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    port = free_port()
    procs = [ctx.Process(target=_rank_entry, args=(r, world, port, list(argv), target or run_argv))
             for r in range(world)]
    for pr in procs:
        pr.start()
    rc = 0
    while any(pr.is_alive() for pr in procs):
        for pr in procs:
            pr.join(timeout=0.2)
            if pr.exitcode not in (None, 0) and rc == 0:
                rc = pr.exitcode
        if rc:
            for pr in procs:
                if pr.is_alive():
                    pr.terminate()
            for pr in procs:
                pr.join(timeout=30)
            break
    for pr in procs:
        if pr.exitcode not in (None, 0) and rc == 0:
            rc = pr.exitcode
    return rc if rc >= 0 else 128 - rc


def init_dist(args):
    """rank / world / local rank from the launcher's environment; the number of
    ranks must be --gpus.  Returns (rank, world, local, dist or None, backend)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but {world} rank(s) were launched")
    # OCG_BENCH_BACKEND=gloo (dry runs of the multi-rank path with several ranks
    # per GPU): ranks map onto the visible devices round-robin, collectives on
    # host tensors.  Default: nccl (= RCCL over xGMI), one rank per GPU.
    backend = os.environ.get("OCG_BENCH_BACKEND", "nccl")
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    return rank, world, local, dist, backend


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args.gpus, argv)
    blocks = None
    if (args.workload == "hessian" and args.gpus == 1 and int(os.environ.get("WORLD_SIZE", "1")) == 1
            and not args.profiled and not args.no_slices and args.multi == 1 and args.controls == 1):
        # before this process touches the GPU: the children start from a process
        # that never made a HIP call (no exec of a GPU process, no fork of one)
        blocks = slice_blocks(args)
    return run(args, blocks)


def run_argv(argv):
    return run(parse_args(argv))


SLICE_TIMEOUT_S = 420


def slice_blocks(args):
    """Configs 4 and 5 (BASELINE configs[3], configs[4]) in the default N=1 line:
    each runs as `bench.py --workload c4rows|c5rows` in a fresh child interpreter
    (its own HIP context; nothing of this process is inherited but the
    environment), one after the other and before the config-1 measurement, so
    no GPU work overlaps a timed region.  A failing or hung child leaves an
    `error` field in its block and the headline line intact.  Harness model:
    main/TestRuntimes.cpp:55-71 (getAnalyticGradient, then getHessian, each
    timed)."""
    import subprocess
    me = os.path.abspath(__file__)
    common = ["--gpus", "1", "--profile-tag", args.profile_tag, "--cpu-threads", str(args.cpu_threads)]
    if args.no_cpu_baseline:
        common.append("--no-cpu-baseline")
    jobs = [("config4_slice", ["--workload", "c4rows", "--c4-nt", "33", "--steps", "2", "--warmup", "1",
                               "--c4-cpu-nt", str(args.c4_cpu_nt)]),
            ("config5_slice", ["--workload", "c5rows", "--c5-nt", "17", "--steps", "1", "--warmup", "1"]),
            # config 4 at its stated horizon (N_t = 801, GROUP M = 40): every 25th row (32 rows of every
            # length, 13,136 of 318,801 row-steps) and the whole precompute, measured; the full
            # getHessian priced from it (366 s whole, r04/r05: too long for this command)
            ("config4_horizon_sample", ["--workload", "c4rows", "--c4-nt", "801", "--row-stride", "25", "--steps",
                                        "1", "--warmup", "0", "--c4-cpu-nt", str(args.c4_cpu_nt)])]
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    out = {}
    for name, extra in jobs:
        t0 = time.perf_counter()
        print(f"[bench] {name}: child bench.py {' '.join(extra)}", file=sys.stderr, flush=True)
        try:
            cp = subprocess.run([sys.executable, "-u", me] + extra + common, stdout=subprocess.PIPE, stderr=None,
                                text=True, timeout=SLICE_TIMEOUT_S, env=env, cwd=ROOT)
            lines = [ln for ln in cp.stdout.splitlines() if ln.startswith("{")]
            if cp.returncode != 0 or not lines:
                out[name] = {"error": f"child exited {cp.returncode}", "stdout_tail": cp.stdout[-2000:]}
            else:
                out[name] = json.loads(lines[-1])
        except subprocess.TimeoutExpired:
            out[name] = {"error": f"child timed out after {SLICE_TIMEOUT_S} s"}
        except (OSError, ValueError) as e:
            out[name] = {"error": f"{type(e).__name__}: {e}"}
        out[name]["child_wall_s"] = time.perf_counter() - t0
        print(f"[bench] {name}: {out[name]['child_wall_s']:.0f} s", file=sys.stderr, flush=True)
    return out


def run(args, blocks=None):
    if args.workload in ("c4grad", "c5grad", "c4rows", "c5rows"):
        return bench_c4(args)

    import torch
    rank, world, local, dist, backend = init_dist(args)
    dev = torch.device("cuda", local)
    cdev = dev if backend == "nccl" else torch.device("cpu")

    from optimalcontrolmps_amd import ed
    from optimalcontrolmps_amd.native import MPS, Engine
    from optimalcontrolmps_amd.sharding import zigzag_rows

    L, p, Q, J, dt = CFG["L"], CFG["p"], CFG["npart"], CFG["J"], CFG["tstep"]
    Nt = int(round(CFG["T"] / dt)) + 1
    ini = MPS(L, p, Q, *ed.mps_from_full(ed.ground_state_full(L, p, Q, J, CFG["U_init"])[0], L, p, Q))
    tgt = MPS(L, p, Q, *ed.mps_from_full(ed.ground_state_full(L, p, Q, J, CFG["U_target"])[0], L, p, Q))
    strong = args.mode == "strong"
    args.mode = args.mode or "weak"
    # weak: rank r evaluates its own control vector (seed + r); strong: one shared vector
    u = np.random.default_rng(CFG["seed"] + (0 if strong else rank)).uniform(2.0, 10.0, Nt)
    rows = zigzag_rows(Nt - 2, rank, world) if strong else list(range(1, Nt - 1))

    eng = Engine(L, p, Q, J, dt, CFG["cutoff"], CFG["maxm"], device=local)
    eng.set_states(tgt, ini)
    KM = max(1, args.multi)
    U_multi = np.stack([u] + [np.random.default_rng(CFG["seed"] + 1000 * k + rank).uniform(2.0, 10.0, Nt)
                              for k in range(1, KM)])
    K = max(1, args.controls)
    extra = []  # controls 2..K of this GPU: own context + stream, own control vector
    for k in range(1, K):
        e2 = Engine(L, p, Q, J, dt, CFG["cutoff"], CFG["maxm"], device=local)
        e2.set_states(tgt, ini)
        extra.append((e2, np.random.default_rng(CFG["seed"] + 1000 * k + rank).uniform(2.0, 10.0, Nt)))
    Hdev = torch.zeros((Nt, Nt), dtype=torch.float64, device=cdev)

    if args.workload == "gradient":
        return bench_gradient(args, eng, u, Nt, dt, world, rank, dist, cdev, U_multi)

    pool = None
    if extra:
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(len(extra))   # ctypes releases the GIL inside ocg_hessian

    def one_step():
        # fused getHessian: psi/xi chains, xiHlist and this rank's rows in one
        # pipelined launch (rows start as their psi_i appears), then divT, F
        # and the batched <xiH_j|psiH> overlaps (ocg_hessian)
        futs = [pool.submit(e2.hessian, u2, rows) for e2, u2 in extra] if extra else []
        if KM > 1:   # all KM controls in one pipeline launch (ocg_hessian_multi)
            Hm, dm, Fm = eng.hessian_multi(U_multi, rows)
            H, divT, F = Hm[0], dm[0], Fm[0]
        else:
            H, divT, F = eng.hessian(u, rows)
        for f in futs:
            f.result()
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
        tt = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    K = K * KM   # control vectors per GPU per step (contexts x controls per launch)
    rows_total = (Nt - 2) * args.steps * (1 if strong else world) * K
    value = rows_total / elapsed
    st_rows = eng.stats(5)       # k_pipeline: trajectories + row re-propagation (dominant)
    st_ovl = eng.stats(6)        # k_row_overlaps
    st_div = eng.stats(1)        # divT / F overlaps
    t_tr = None
    if not args.profiled:        # a profiled command holds only the timed population
        t_tr = time.perf_counter()
        eng.propagate(u, 3)      # one bare psi || xi trajectory (outside the timed region): single-chain step rate
        t_tr = time.perf_counter() - t_tr
    # throughput with several control vectors per call (IPOPT trial points, FD probes,
    # multi-start), outside the timed region: reported beside `value`, never as it
    multi_info = None
    if args.multi_info and K * KM == 1 and not strong:
        Um = np.random.default_rng(CFG["seed"] + 77 + rank).uniform(2.0, 10.0, (8, Nt))
        eng.hessian_multi(Um[:2], rows)              # warm the multi path's buffers
        torch.cuda.synchronize()
        t_m = time.perf_counter()
        eng.hessian_multi(Um, rows)
        t_m = time.perf_counter() - t_m
        Ug = np.random.default_rng(CFG["seed"] + 78 + rank).uniform(2.0, 10.0, (64, Nt))
        eng.gradient_multi(Ug[:2])
        t_g = time.perf_counter()
        eng.gradient_multi(Ug)
        t_g = time.perf_counter() - t_g
        multi_info = {"hessian_rows_per_sec_8_controls": 8 * len(rows) / t_m,
                      "gradients_per_sec_64_controls": 64 / t_g,
                      "note": "ocg_hessian_multi / ocg_gradient_multi, one launch for all controls, per GPU"}
    row_steps = (Nt - 2) * (Nt - 3) // 2
    sweep_steps = args.steps * K * (2 * (Nt - 1) * world + row_steps * (1 if strong else world))
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
                                   "tstep=0.01 T=2.0 GRAPE, N_t=201, 199 rows)"
                                   + (f", {K} concurrent control vectors per GPU"
                                      + (f" ({KM} per pipeline launch)" if KM > 1 else "") if K > 1 else ""),
                       "rows_per_step": (Nt - 2) * (1 if strong else world) * K,
                       "parallelism": (f"one control, rows sharded zig-zag over {world} GPU(s) + RCCL reduce" if strong
                                       else f"{world} GPU(s), one full getHessian (own control vector) per GPU")},
            "sweep_steps_per_sec": sweep_steps / elapsed,
            "kernels": {
                "pipeline": {"avg_ms": launch_ms, "launches": st_rows["launches"]},
                "row_overlaps": {"avg_ms": st_ovl["ms"] / max(1, st_ovl["launches"]), "launches": st_ovl["launches"]},
                "divT_F_overlaps_ms": st_div["ms"] / max(1, args.steps),
            },
            "single_chain_steps_per_sec": (Nt - 1) / t_tr if t_tr else None,
            "multi_control": multi_info,
            "roofline": roofline_block("k_pipeline", launch_ms, bytes_per_launch, flops_per_launch,
                                       args.profile_tag,
                                       limiter="issue latency: one chain's N_t-1 dependent steps on one CU "
                                               "(state in LDS); HBM and FP64 are both <1% busy", bound="latency"),
        }
        result["env"] = run_env()
        # config 2 (BASELINE configs[1]) after the timed region, as main/TestRuntimes.cpp:55-63
        # times getAnalyticGradient before getHessian
        if not args.profiled:
            result["config2_gradient"] = config2_gradient(eng, u, Nt, dt, args.profile_tag,
                                                          cpu=(world == 1 and not args.no_cpu_baseline),
                                                          ini=ini, tgt=tgt)
        if world == 1 and not args.no_cpu_baseline and not args.profiled:
            result["cpu_baseline"] = cpu_baseline(ini, tgt, u, args.cpu_threads)
        if blocks:   # configs 4 and 5, measured in child processes before this line's timed region
            result.update(blocks)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def run_env():
    """the run-time settings a line's numbers depend on, read back from this
    process's environment (GPU_MAX_HW_QUEUES: hardware queues per process, HIP's
    default 4 when unset; the GPU box exports 4)"""
    keys = ("GPU_MAX_HW_QUEUES", "OMP_NUM_THREADS", "OCG_HBM_PRIO", "OCG_HBM_PIPE", "OCG_HBM_COOP",
            "HIP_VISIBLE_DEVICES")
    env = {k: os.environ.get(k) for k in keys}
    env["native_lib"] = native_lib_record()
    return env


def native_lib_record():
    """which HIP library this process loaded: bench.py never compiles; it loads the
    in-tree liboptimalcontrolmps_amd.so that __graft_entry__.build() (or
    native.build_native()) compiled before the tree was shipped.  `stale` is
    true when a csrc/ source or include/ocmps.h is newer than the library."""
    import hashlib
    from optimalcontrolmps_amd import native
    path = native.LIB_PATH
    if not os.path.exists(path):
        return {"path": None}
    with open(path, "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()[:16]
    mt = os.path.getmtime(path)
    newest = max(os.path.getmtime(x) for x in native.sources())
    return {"path": os.path.relpath(path, ROOT), "sha16": sha,
            "mtime_utc": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(mt)),
            "compiled_by_this_process": False, "stale": bool(newest > mt)}


def st_traj_ms_per_step(eng, Nt):
    """ms per step of one chain: the bare two-chain trajectory (ocg_propagate(u, 3))
    timed once outside the measured region (the pipeline's critical path)."""
    st = eng.stats(0)
    if st["launches"] == 0:
        return 0.0
    return st["ms"] / st["launches"] / (Nt - 1)


def roofline_block(kernel, launch_ms, bytes_per_launch, flops_per_launch, tag, limiter, bound="hbm"):
    """Roofline of the dominant kernel.  achieved = algorithmic bytes (SURVEY.md
    §8d model) / HIP-event launch time, priced against the
    HBM peak; `bound` names what really limits the kernel ("latency": dependent
    instruction chains, neither HBM nor the MFMA pipes).  traffic = HBM bytes per
    dispatch measured by rocprofv3 PMC over THIS workload's command
    (profiles/<tag>_summary.json, tag = round + workload + N_t; FETCH_SIZE
    doubled per the gfx950 calibration), null when no such profile exists."""
    achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9 if launch_ms > 0 else 0.0
    traffic = measured_traffic(kernel, tag)
    meas = traffic / (launch_ms * 1e-3) / 1e9 if (traffic and launch_ms > 0) else None
    tf = flops_per_launch / (launch_ms * 1e-3) / 1e12 if launch_ms > 0 else 0.0
    return {
        "bound": bound,
        "limiter": limiter,
        "kernel": kernel,
        "achieved": achieved,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS,
        "traffic": traffic,
        "measured_hbm_gbs": meas,
        "measured_frac": (meas / HBM_PEAK_GBS) if meas is not None else None,
        "alg_bytes_per_launch": bytes_per_launch,
        "avg_launch_ms": launch_ms,
        "fp64_achieved_tflops": tf,
        "fp64_peak_tflops": FP64_PEAK_TFS,
        "fp64_frac": tf / FP64_PEAK_TFS,
        "fp64_mfma_measured_peak_tflops": FP64_MFMA_MEASURED_TFS,
    }


def config2_gradient(eng, u, Nt, dt, tag, cpu, ini, tgt, reps=20):
    """Config 2: getAnalyticGradient(u, new_control=true) with BFGS=true at config 1
    (calcFidelityGrad's BFGS branch, src/OptimalControl.cpp:204-249: psi_t and xi_t
    propagated, here concurrently in one launch of two chains, then the divT
    overlaps and F; ocg_propagate(u, 3) + ocg_div_t + ocg_overlap_factor), timed
    over `reps` gradients.  Roofline of k_trajectory (its launches in a profile of
    this command are all such psi || xi pairs: the single-chain probe above is the
    same call).  cpu: the oracle's BFGS gradient on one host thread (the reference
    runs this branch sequentially), median of 5."""
    import torch

    def one():
        eng.propagate(u, 3)
        divT = eng.div_t()
        F = eng.overlap_factor()
        return dt * (divT * F * 1j).real

    g = one()
    eng.reset_stats()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g = one()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    st, sov = eng.stats(0), eng.stats(1)
    launch_ms = st["ms"] / max(1, st["launches"])
    out = {"metric": "getAnalyticGradient/sec (BFGS=true: psi || xi + divT + F), N=5 d=4 chi=80 T=2.0",
           "value": reps / el, "unit": "gradients/s", "ms_per_gradient": 1e3 * el / reps, "gradients": reps,
           "sweep_steps_per_sec": reps * 2 * (Nt - 1) / el,
           "single_chain_steps_per_sec": 1e3 * (Nt - 1) / max(launch_ms, 1e-9),
           "kernels": {"trajectory_ms": launch_ms, "divT_F_ms": sov["ms"] / reps},
           "roofline": roofline_block("k_trajectory", launch_ms, st["alg_bytes"] / max(1, st["launches"]),
                                      st["alg_flops"] / max(1, st["launches"]), tag,
                                      limiter="issue latency: 200 dependent steps per chain, one CU per chain",
                                      bound="latency")}
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_ffi as O
        L, p, Q, J = CFG["L"], CFG["p"], CFG["npart"], CFG["J"]
        stp = O.Stepper(L, p, Q, J, dt, CFG["cutoff"], CFG["maxm"])
        oc = O.OC(stp, O.MPS(L, p, Q, tgt.dims, tgt.data), O.MPS(L, p, Q, ini.dims, ini.data), Nt, 0.0)
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            gc = oc.gradient(u, bfgs=True)
            ts.append(time.perf_counter() - t0)
        out["cpu_baseline"] = {"value": 1.0 / float(np.median(ts)), "unit": "gradients/s", "cores": 1, "kind": "port",
                               "sample": "5 BFGS gradients (config 1, N_t=201) on the C++ CPU restatement (oracle/, "
                                         "not ITensor), one thread, median"}
        out["max_abs_diff_vs_cpu"] = float(np.max(np.abs(gc - g)))
    return out


def bench_gradient(args, eng, u, Nt, dt, world, rank, dist, cdev, U_multi):
    """config 2: getAnalyticGradient(u) with BFGS=true at config 1 — psi_t and xi_t
    propagated concurrently in one launch (calcFidelityGrad's BFGS branch,
    src/OptimalControl.cpp:217-229, propagates xi independently of psi), then the
    batched divT overlaps and F (ocg_propagate(u, 3) + ocg_div_t + ocg_overlap_factor)."""
    import torch

    KM = len(U_multi)

    def one():
        if KM > 1:   # K control vectors: one trajectory launch of 2K chains + batched divT / F
            divT, F = eng.gradient_multi(U_multi)
            return dt * (divT * F[:, None] * 1j).real
        eng.propagate(u, 3)
        divT = eng.div_t()
        F = eng.overlap_factor()
        return dt * (divT * F * 1j).real

    for _ in range(args.warmup):
        one()
    eng.reset_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    st_traj, st_ov = eng.stats(0), eng.stats(1)
    if rank == 0:
        launch_ms = st_traj["ms"] / max(1, st_traj["launches"])
        res = {
            "metric": "getAnalyticGradient/sec (BFGS=true: psi || xi + divT), N=5 d=4 chi=80 T=2.0",
            "value": args.steps * world * KM / elapsed, "unit": "gradients/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "c128/f64",
            "data": "synthetic GRAPE controls U(2,10) seed 20261015; ED ground states U=2.5 -> 50",
            "config": {"workload": "config 2: getAnalyticGradient(u, new_control=true), BFGS=true, N_t=201"
                                   + (f", {KM} control vectors per call (ocg_gradient_multi)" if KM > 1 else "")},
            "sweep_steps_per_sec": args.steps * world * KM * 2 * (Nt - 1) / elapsed,
            "single_chain_steps_per_sec": 1e3 * (Nt - 1) / max(launch_ms, 1e-9),
            "kernels": {"trajectory_ms": launch_ms, "divT_F_ms": st_ov["ms"] / max(1, args.steps)},
            "roofline": roofline_block("k_trajectory", launch_ms, st_traj["alg_bytes"] / max(1, st_traj["launches"]),
                                       st_traj["alg_flops"] / max(1, st_traj["launches"]), args.profile_tag + "grad",
                                       limiter="issue latency: 200 dependent steps per chain, one CU per chain",
                                       bound="latency"),
        }
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


C4 = dict(L=20, p=7, npart=20, J=1.0, tstep=0.005, T=4.0, maxm=256, cutoff=1e-8, seed=20261016)
C5 = dict(L=50, p=9, npart=50, J=1.0, tstep=0.01, T=10.0, maxm=512, cutoff=1e-8, seed=20261017)


def bench_c4(args):
    """Config 4's chain (BASELINE configs[3]: L=20 Npart=20 d=6 chi=256 tstep=0.005
    T=4, GROUP M=40, 8 GPUs) and config 5's (configs[4]: L=50 Npart=50 d=8
    chi=512 tstep=0.01, 1/2/4/8 GPUs) on the HBM-resident engine.

    c4rows: one getHessian per step over a T slice of --c4-nt time points
      (default 33: 31 rows): GROUP M=40 (chopped-sine basis over the slice, u0 =
      the adiabatic seed 2 -> 10, coefficients c ~ U(-2,2), a new draw per step
      so every step is a fresh getHessian(c, new_control=true)): convertControl
      on the host, the rows of H_u dealt zig-zag over the ranks (each rank
      recomputes psi, xi, divT, xiH), one RCCL reduce onto rank 0, the
      regularisation Hessian (gamma 1e-6) and H_c = V H_u V^T on rank 0's device
      (ocg_convert_hessian).  psi_init = the saturated warm state
      (tests/golden/c4_warm256.npz: |1..1> evolved 400 steps at U=2.5, bonds
      256), psi_target = psi_init evolved 2 more steps at U=6 (config 4's |1..1>
      target has ~1e-10 overlap, which leaves every derivative at rounding
      level; cost is independent of the target).
    c5rows: the same over --c5-nt time points of config 5's chain, GRAPE
      controls U(2,10), psi_init = the Mott state |1..1> evolved --c5-warm steps
      at U=2.5 on each rank's device (untimed; the bonds saturate at 512 after
      ~220 steps).
    c4grad / c5grad: one getAnalyticGradient over the full horizon (config 4:
      N_t=801, config 5: N_t=1001) per rank (the gradient's time recursion does
      not shard: replicas).
    --last-rows R: the rows N_t-1-R .. N_t-2 only (the cheapest rows of a full
      horizon: each needs psi_i, xi_i and xiH_i of the whole trajectory).

    --mode strong (default for c4rows/c5rows): one Hessian's rows over all
    ranks; --mode weak: every rank a whole Hessian of its own control."""
    import torch
    from optimalcontrolmps_amd.control_basis import adiabatic_seed, build_chopped_sine_basis
    from optimalcontrolmps_amd.distributed import sharded_hessian, torch_reduce
    from optimalcontrolmps_amd.native import MPS, Engine
    rank, world, local, dist, backend = init_dist(args)
    cdev = torch.device("cuda", local) if backend == "nccl" else torch.device("cpu")
    c5 = args.workload in ("c5rows", "c5grad")
    grad = args.workload in ("c4grad", "c5grad")
    strong = (args.mode or ("weak" if grad else "strong")) == "strong" and not grad
    c = C5 if c5 else C4
    L, p, Q, dt = c["L"], c["p"], c["npart"], c["tstep"]
    eng = Engine(L, p, Q, c["J"], dt, c["cutoff"], c["maxm"], device=local, engine="hbm")
    # the state cache is keyed to what produced it; a file of another workload or
    # preparation is ignored (and overwritten), never loaded silently
    cache = args.state_cache
    if cache and not cache.endswith(".npz"):
        cache += ".npz"   # np.savez would append it
    key = np.array([f"{args.workload[:2]} L={L} p={p} Q={Q} maxm={c['maxm']} dt={dt} "
                    f"warm={args.c5_warm if c5 else 'c4_warm256'}"])
    if cache and world > 1:
        dist.barrier()    # rank 0 may still be writing it
    warm_s, cached = 0.0, False
    if cache and os.path.exists(cache):   # prepared by an earlier (unprofiled) process
        z = np.load(cache, allow_pickle=False)
        if "key" in z.files and str(z["key"][0]) == str(key[0]):
            ini = MPS(L, p, Q, z["ini_dims"], z["ini_data"])
            tgt = MPS(L, p, Q, z["tgt_dims"], z["tgt_data"])
            cached = True
        else:
            print(f"[bench] state cache {cache} belongs to another preparation; preparing anew", file=sys.stderr)
    if not cached:
        if c5:
            from optimalcontrolmps_amd.states import product_state, warm_state
            t0 = time.perf_counter()
            ini = warm_state(eng, product_state(L, p, Q), 2.5, args.c5_warm, chunk=10)
            warm_s = time.perf_counter() - t0
        else:
            z = np.load(os.path.join(ROOT, "tests", "golden", "c4_warm256.npz"), allow_pickle=False)
            ini = MPS(L, p, Q, z["dims"], z["data"])
        tgt = eng.steps(ini, np.full(3, 6.0), True)
        if cache and rank == 0:   # written whole, then renamed: a reader never sees a partial file
            tmp = cache[:-4] + f".tmp{os.getpid()}.npz"
            np.savez(tmp, key=key, ini_dims=ini.dims, ini_data=ini.data, tgt_dims=tgt.dims, tgt_data=tgt.data)
            os.replace(tmp, cache)
    if args.prepare_only:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return 0
    eng.set_states(tgt, ini)
    Nt = int(round(c["T"] / dt)) + 1 if grad else (args.c5_nt if c5 else args.c4_nt)
    M = 0 if (grad or c5) else args.group_m
    gamma = 1e-6 if M else 0.0
    basis = build_chopped_sine_basis(adiabatic_seed(2.0, 10.0, Nt), dt, (Nt - 1) * dt, M) if M else None
    nsteps_all = args.warmup + args.steps
    seed = c["seed"] + (0 if strong else 7919 * rank)

    def control(s):   # a fresh control vector per step (every getHessian has new_control = true)
        rng = np.random.default_rng(seed + 1000 * s)
        if basis is not None:
            return basis.convert_control(rng.uniform(-2.0, 2.0, M))
        return rng.uniform(2.0, 10.0, Nt)
    KM = max(1, args.multi)
    reduce = torch_reduce(dist, cdev, Nt) if (world > 1 and strong) else None
    project = (lambda Hu: eng.convert_hessian(Hu, basis.V)) if basis is not None else None

    R = args.last_rows if (args.last_rows and not grad) else Nt - 2
    first = Nt - 1 - R   # the first row of the computed set
    stride = max(1, args.row_stride)
    sel = [r for r in range(first, Nt - 1) if (r - 1) % stride == 0]   # the computed rows
    R = len(sel)

    def rows_of(uu, rows):
        return eng.hessian(uu, [r for r in rows if r >= first and (r - 1) % stride == 0])

    def one(s):
        if grad:
            if KM > 1:   # K controls: one batch of 2K chains + batched divT / F
                Um = np.stack([control(s * KM + k) for k in range(KM)])
                divT, F = eng.gradient_multi(Um)
                return dt * (divT * F[:, None] * 1j).real
            u = control(s)
            divT, F = eng.gradient(u)   # ocg_gradient: stored trajectories, or psi || xi meeting in the middle
            return dt * (divT * F * 1j).real
        u = control(s)   # GROUP: convertControl (src/ControlBasis.cpp:49-67), host
        H, divT, F, _ = sharded_hessian(rows_of, u, rank if strong else 0,
                                        world if strong else 1, reduce, gamma=gamma, tstep=dt, project=project)
        return H

    import threading
    done = threading.Event()

    def heartbeat():   # long slices (full N_t): a line a minute on stderr while the device works
        t_hb = time.perf_counter()
        while not done.wait(60.0):
            print(f"[bench] {args.workload} N_t={Nt}: {time.perf_counter() - t_hb:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    for s in range(args.warmup):
        one(s)
    eng.reset_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.warmup, nsteps_all):
        one(s)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    done.set()
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    gm = eng.stats(7)   # k_gemm: the MFMA-FP64 contraction kernel
    # one bare psi chain (ocg_propagate(u, 1)) outside the timed region: the single-chain step rate
    t_sc = None
    paths = eng.path_stats()
    if not args.profiled and not (grad and c5) and not paths["ckpt_runs"]:
        # a profiled command holds only the timed population; config 5's full-horizon trajectories
        # do not fit the device (the gradient meets in the middle, the getHessian checkpoints)
        t_sc = time.perf_counter()
        eng.propagate(control(nsteps_all), 1)
        t_sc = time.perf_counter() - t_sc
    steps_traj = 2 * (Nt - 1) * (KM if grad else 1)
    row_steps = sum(Nt - 2 - r for r in sel)   # row i steps from i to N_t-2
    reps = 1 if strong else world   # independent Hessians / gradients per step
    sweep = args.steps * (steps_traj * (world if (strong or grad) else reps) + (0 if grad else row_steps * reps))
    gemm_ms = gm["ms"] / max(1, gm["launches"])
    if rank == 0:
        tag = f"{args.profile_tag}{'c5' if c5 else 'c4'}{'g' if grad else ''}n{Nt}"
        par = (f"one getHessian per step, rows zig-zag over {world} GPU(s), RCCL reduce to rank 0" if strong
               else f"{world} GPU(s), one {'gradient' if grad else 'getHessian'} (own control) per GPU")
        res = {
            "metric": ("getAnalyticGradient/sec (psi || xi + divT)" if grad else "Hessian-rows/sec (getHessian)")
                      + (", config 5 chain L=50 Npart=50 d=8 chi=512 tstep=0.01" if c5 else
                         ", config 4 chain L=20 Npart=20 d=6 chi=256 tstep=0.005"),
            "value": (args.steps * KM * world if grad else args.steps * R * reps) / elapsed,
            "unit": "gradients/s" if grad else "rows/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True, "scaling": "strong" if strong else "weak", "vs_baseline": None,
            "dtype": "c128/f64",
            "data": ((f"synthetic GROUP coefficients U(-2,2) (M={M}, chopped sine, u0 adiabatic 2->10), "
                      if M else "synthetic GRAPE controls U(2,10), ") + f"seed {c['seed']}, a fresh draw per step; "
                     + "psi_init = " + (f"|1..1> evolved {args.c5_warm} steps at U=2.5 on the device (untimed"
                                        + (", loaded from the state cache" if cached else f", {warm_s:.0f} s")
                                        + f"; max bond {int(ini.bond_dims().max())})" if c5 else
                                        "saturated chi=256 warm state (|1..1> evolved 400 steps at U=2.5)")
                     + "; psi_target = psi_init evolved 2 steps at U=6 (SURVEY's |1..1> target has ~1e-10 overlap "
                       "with psi_t, which leaves every derivative at rounding level)"),
            "config": {"workload": (f"config {5 if c5 else 4} chain, getAnalyticGradient over N_t={Nt} "
                                    f"(T={c['T']:g})" if grad else
                                    f"config {5 if c5 else 4} chain, getHessian"
                                    + (f" GROUP M={M} (convertControl, regularisation gamma={gamma}, "
                                       f"convertHessian on the device)" if M else " GRAPE")
                                    + (f" over the full horizon N_t={Nt}, every {stride}-th row: {R} rows "
                                       f"({row_steps} of {(Nt - 2) * (Nt - 3) // 2} row-steps)" if stride > 1 else
                                       f" over the full horizon N_t={Nt}, the last {R} rows ({row_steps} row-steps)"
                                       if R < Nt - 2 else
                                       f" over a T slice N_t={Nt} ({Nt - 2} rows, {row_steps} row-steps)")),
                       "engine": "HBM-resident (hbm.hip)", "parallelism": par},
            "sweep_steps_per_sec": sweep / elapsed,
            "single_chain_steps_per_sec": (Nt - 1) / t_sc if t_sc else None,
            "mfma_gemm": {"kernel": "k_gemm (v_mfma_f64_16x16x4f64)", "launches_per_step": gm["launches"] / args.steps,
                          "avg_launch_ms": gemm_ms, "share_of_time": gm["ms"] / (1e3 * elapsed),
                          "achieved_tflops": gm["alg_flops"] / max(gm["ms"], 1e-9) / 1e9,
                          "achieved_gbs": gm["alg_bytes"] / max(gm["ms"], 1e-9) / 1e6},
            # the committed profile's per-dispatch traffic is this region's only when the profiled
            # command ran --profiled on cached states (no single-chain launches: warm-up, target,
            # probe); otherwise the line carries no traffic
            "roofline": roofline_block("hbm::k_gemm", gemm_ms, gm["alg_bytes"] / max(1, gm["launches"]),
                                       gm["alg_flops"] / max(1, gm["launches"]), tag,
                                       bound="latency",
                                       limiter="the per-sector Hermitian eigensolver (k_heev_*) sets the step time; "
                                               "k_gemm launches are small (tasks of m, n ~ 16-60) and latency-bound"),
        }
        if not grad:
            res["hessian_path"] = {"pipelined": paths["pipe_runs"], "pipeline_fallbacks": paths["pipe_fallbacks"],
                                   "checkpointed": paths["ckpt_runs"],
                                   "checkpoint_segment": paths["ckpt_k"] or None}
        if stride > 1 and not grad:
            # the sample's parts (hbm timers: kind 3 = the row batches of the two-phase path). The
            # rows of a sample run in smaller lockstep batches than the whole Hessian's (32 rows vs
            # 799 joining over the horizon), so their row-step rate is a lower bound of the whole
            # run's; the whole getHessian is not priced from it (measured whole: 345.9 s, r06)
            rows_ms = eng.stats(3)["ms"] / args.steps
            res["horizon_sample"] = {
                "rows": R, "of_rows": Nt - 2, "row_steps": row_steps, "of_row_steps": (Nt - 2) * (Nt - 3) // 2,
                "precompute_ms": 1e3 * elapsed / args.steps - rows_ms, "rows_ms": rows_ms,
                "row_steps_per_s": row_steps / max(rows_ms * 1e-3, 1e-9),
                "whole_getHessian_measured_s": 345.9,
                "whole_source": "profiles/r06_bench_c4full.json (round 6 code: one GPU, the two-phase path; "
                                "rounds 4-5: 359-366 s, profiles/r04_bench_c4full_prio.json)"}
        res["env"] = run_env()
        if world == 1 and not args.no_cpu_baseline and not grad and not args.profiled:
            res["cpu_baseline"] = (cpu_baseline_c5(ini, Nt, args.cpu_threads) if c5 else
                                   cpu_baseline_c4(ini, tgt, Nt, args.cpu_threads, args.c4_cpu_nt))
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def measured_traffic(kernel, tag="r01"):
    """HBM bytes per dispatch of `kernel` from the committed rocprofv3 PMC passes
    of this same command (profiles/<tag>_summary.json, written by
    tools/prof_summary.py; FETCH_SIZE doubled per the gfx950 calibration);
    None when there is no such profile (tag None)."""
    if tag is None:
        return None
    try:
        with open(os.path.join(ROOT, "profiles", f"{tag}_summary.json")) as f:
            return json.load(f)["pmc_per_dispatch"][kernel]["hbm_bytes"]
    except (OSError, KeyError, ValueError):
        return None


def cpu_baseline_c4(ini, tgt, Nt, threads, cpu_nt=5):
    """Config 4 on the CPU restatement (oracle/, 'port', not ITensor), with the
    oracle's Householder + QL block eigensolver (ORC_HEEV=ql: LAPACK zheev's
    algorithm, as ITensor's diagHermitian; the default cyclic Jacobi takes ~14x
    longer) on the same chain (psi_init, psi_target of the slice):
      measured: one full getHessian at N_t = cpu_nt (default 5: 3 rows) on the
        granted host threads — psi || xi on two threads, xiH and the rows over
        the threads (src/OptimalControl.cpp:281-338), every thread budget also
        splitting the U(1) sectors inside each step (bit-identical results) —
        beside the GPU's getHessian of the same controls (same command, HIP),
        with the two Hessians compared;
      priced: the slice's own N_t from one measured chi = 256 step on one
        thread (psi || xi serial, xiH (one dH application ~ 3 steps, measured at
        8 threads: 17.9 s vs 6.0 s) and the rows' (N_t-2)(N_t-3)/2 steps over the
        threads; overlaps not priced, so the estimate favours the CPU).
    `value` is the measured rate (rows/s of the short N_t = cpu_nt getHessian,
    whose rows average (cpu_nt - 3)/2 steps: it flatters the CPU next to the
    slice's rows)."""
    os.environ["ORC_HEEV"] = "ql"   # read at the oracle's first decomposition in this process
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    c = C4
    L, p, Q = c["L"], c["p"], c["npart"]
    st = O.Stepper(L, p, Q, c["J"], c["tstep"], c["cutoff"], c["maxm"])
    psi0 = O.MPS(L, p, Q, ini.dims, ini.data)
    O.set_sector_threads(1)
    t0 = time.perf_counter()
    st.step(psi0, 2.5, 3.0, True)
    t_step = time.perf_counter() - t0
    avail = cpu_threads_available()
    th = max(1, min(threads, avail)) if threads else avail
    rows = Nt - 2
    row_steps = rows * (rows - 1) // 2
    est = t_step * ((Nt - 1) + 3.0 * Nt / th + (row_steps + 3.0 * rows) / th)
    out = {"unit": "rows/s", "cores": th, "kind": "port", "host_threads_available": avail, "nproc": os.cpu_count(),
           "priced_slice": {"value": rows / est, "unit": "rows/s", "estimated": True, "N_t": Nt, "threads": th,
                            "measured_step_s_1thread": t_step,
                            "sample": f"one chi=256 step of this chain on one thread ({t_step:.1f} s); the N_t={Nt} "
                                      f"getHessian priced from it at {th} threads (psi || xi serial, dH = 3 steps, "
                                      f"xiH and rows over the threads, overlaps not priced)"}}
    if cpu_nt and cpu_nt >= 4:
        u = np.random.default_rng(C4["seed"] + 99).uniform(2.0, 10.0, cpu_nt)
        oc = O.OC(st, O.MPS(L, p, Q, tgt.dims, tgt.data), psi0, cpu_nt, 0.0)
        oc.set_nested(True)
        Hc = np.zeros((cpu_nt, cpu_nt))
        t_h = oc.time_hessian(u, th, Hc)
        out.update(value=(cpu_nt - 2) / t_h, measured_s=t_h, estimated=False,
                   sample=f"one full getHessian at N_t={cpu_nt} ({cpu_nt - 2} rows) of this chain (psi_init, "
                          f"psi_target of the slice, GRAPE controls U(2,10)) on the C++ CPU restatement (oracle/, not "
                          f"ITensor; Householder + QL), {th} threads: psi || xi, xiH and rows over the threads, each "
                          f"thread budget also splitting the U(1) sectors inside a step; {t_h:.1f} s")
        out["gpu_same_sample"] = gpu_same_sample(u, tgt, ini, C4, Hc)
    else:
        out.update(value=out["priced_slice"]["value"], estimated=True, sample=out["priced_slice"]["sample"])
    return out


def gpu_same_sample(u, tgt, ini, c, Hc):
    """the GPU's getHessian of the CPU sample's controls on the same chain (a
    fresh HBM-engine context, one untimed warm-up call): rows/s and the largest
    Hessian difference from the CPU restatement's, relative to max|H|"""
    from optimalcontrolmps_amd.native import Engine
    e = Engine(c["L"], c["p"], c["npart"], c["J"], c["tstep"], c["cutoff"], c["maxm"], engine="hbm")
    e.set_states(tgt, ini)
    e.hessian(u)
    t0 = time.perf_counter()
    H, _, _ = e.hessian(u)
    t = time.perf_counter() - t0
    e.close()
    return {"value": (len(u) - 2) / t, "unit": "rows/s", "s": t,
            "max_abs_diff_rel_to_max_H": float(np.abs(H - Hc).max() / max(np.abs(Hc).max(), 1e-300))}


def step_cost_model(dims, L, p, Q):
    """flop model of one BH_tDMRG step from the bond dims (flat (L+1)(Q+1)):
    per gate and middle-bond sector q, Theta (8 R C m), Gram (8 n^2 N),
    Householder + QL eigenproblem with vectors (~20 n^3) and the factors
    (8 m R C), R / C the sector's row / column counts, n = min(R, C), N = max,
    m = the sector's kept dim; the gauge moves scale the same way per gate"""
    d = np.asarray(dims).reshape(L + 1, Q + 1)
    tot = 0.0
    for b in range(1, L):   # gate on sites (b, b+1): bonds b-1, b, b+1
        for q in range(Q + 1):
            R = sum(d[b - 1, q - n] for n in range(p) if 0 <= q - n <= Q)
            C = sum(d[b + 1, q + n] for n in range(p) if q + n <= Q)
            if R == 0 or C == 0:
                continue
            n, N, m = min(R, C), max(R, C), d[b, q]
            tot += 16.0 * R * C * m + 8.0 * n * n * N + 20.0 * n ** 3
    return tot


def cpu_baseline_c5(ini, Nt, threads):
    """Config 5 (L = 50, p = 9, chi = 512) on the CPU restatement, priced: one
    chi = 512 step is measured on one thread on the 12-site chain of
    tests/golden/c5_w512.npz (config 5's p and tstep, middle bonds saturated at
    512 by the oracle itself; one L = 50 step would take minutes), scaled to the
    L = 50 state by the flop model of both chains' bond dims (step_cost_model),
    and the slice's getHessian is priced from that like config 4's (psi || xi
    serial, dH = 3 steps, xiH and rows over the granted threads; overlaps not
    priced)."""
    os.environ["ORC_HEEV"] = "ql"
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    c = C5
    z = np.load(os.path.join(ROOT, "tests", "golden", "c5_w512.npz"), allow_pickle=False)
    Lx = 12
    st = O.Stepper(Lx, c["p"], Lx, c["J"], c["tstep"], c["cutoff"], c["maxm"])
    psi = O.MPS(Lx, c["p"], Lx, z["dims"], z["data"])
    O.set_sector_threads(1)
    t0 = time.perf_counter()
    st.step(psi, 2.5, 3.0, True)
    t12 = time.perf_counter() - t0
    ratio = step_cost_model(ini.dims, c["L"], c["p"], c["npart"]) / step_cost_model(z["dims"], Lx, c["p"], Lx)
    t50 = t12 * ratio
    avail = cpu_threads_available()
    th = max(1, min(threads, avail)) if threads else avail
    rows = Nt - 2
    row_steps = rows * (rows - 1) // 2
    est = t50 * ((Nt - 1) + 3.0 * Nt / th + (row_steps + 3.0 * rows) / th)
    return {"value": rows / est, "unit": "rows/s", "cores": th, "kind": "port", "estimated": True,
            "measured_fixture_pair": c5_fixture_pair(),
            "measured_step_s_L12_1thread": t12, "model_ratio_L50_over_L12": ratio, "priced_step_s_L50": t50,
            "host_threads_available": avail, "nproc": os.cpu_count(),
            "sample": f"one chi=512 step of the 12-site config-5 chain (tests/golden/c5_w512.npz) on the C++ CPU "
                      f"restatement (oracle/, not ITensor; Householder + QL) on one thread, {t12:.1f} s, scaled "
                      f"x{ratio:.1f} to the L=50 state by a flop model of the bond dims; the N_t={Nt} getHessian "
                      f"priced from it at {th} threads (psi || xi serial, dH = 3 steps, xiH and rows over the threads, "
                      f"overlaps not priced, so the estimate favours the CPU)"}


def c5_fixture_pair():
    """A MEASURED chi = 512 getHessian on both sides, the same sample: the 12-site
    config-5 chain of tests/golden/c5_w512h9.npz (psi_init = the saturated state,
    psi_target = it stepped three times by the oracle, both at chi = 512, N_t = 9
    GRAPE controls).  CPU: the oracle's getHessian that made the fixture
    (make_c5w512_fixture.py hess9: wall seconds and threads stored in the file;
    timed in the build container, 8 cores, not on this box: 30 min of CPU).  GPU:
    the same getHessian on this box's MI355X now (HBM engine, pipelined), with
    max|dH| / max|H| against the oracle's."""
    from optimalcontrolmps_amd.native import MPS, Engine
    gd = os.path.join(ROOT, "tests", "golden")
    f9 = os.path.join(gd, "c5_w512h9.npz")
    if not os.path.exists(f9):
        return None
    c = C5
    zs = np.load(os.path.join(gd, "c5_w512.npz"), allow_pickle=False)
    z = np.load(f9, allow_pickle=False)
    Lx, nt = 12, len(z["u"])
    ini = MPS(Lx, c["p"], Lx, zs["dims"], zs["data"])
    tgt = MPS(Lx, c["p"], Lx, z["tdims"], z["tdata"])
    eng = Engine(Lx, c["p"], Lx, c["J"], c["tstep"], c["cutoff"], c["maxm"], engine="hbm")
    eng.set_states(tgt, ini)
    eng.hessian(z["u"])  # warm-up (allocations)
    t0 = time.perf_counter()
    H, _, _ = eng.hessian(z["u"])
    tg = time.perf_counter() - t0
    eng.close()
    rows = nt - 2
    cpu_s = float(z["secs"][0])
    return {"sample": f"L=12 p=9 chi=512 chain, N_t={nt} getHessian ({rows} rows), tests/golden/c5_w512h9.npz",
            "cpu_oracle_s": cpu_s, "cpu_threads": int(z["threads"][0]), "cpu_where": "build container (8 cores)",
            "cpu_rows_per_s": rows / cpu_s, "gpu_s": tg, "gpu_rows_per_s": rows / tg,
            "max_dH_rel": float(np.abs(H - z["H"]).max() / np.abs(z["H"]).max())}


def cpu_threads_available():
    """host threads this process may use: the affinity mask, capped by
    OMP_NUM_THREADS when set (the GPU box exports its CPU share, 16 per GPU)"""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(ini, tgt, u, threads):
    """The CPU restatement (oracle/, 'port' — ITensor cannot be built here) timed
    on host cores like main/TestRuntimes.cpp:25-229: one full getHessian per
    thread count 1, 2, 4, 8, ... up to the threads available (row worker pool of
    calcHessian_parallel, src/OptimalControl.cpp:281-338, psi || xi on two
    threads); value = the best rate, cores = the threads it used."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    L, p, Q, J, dt = CFG["L"], CFG["p"], CFG["npart"], CFG["J"], CFG["tstep"]
    avail = cpu_threads_available()
    cap = max(1, min(threads, avail)) if threads else avail
    counts = sorted({t for t in (1, 2, 4, 8, 16, 32) if t <= cap} | {cap})
    st = O.Stepper(L, p, Q, J, dt, CFG["cutoff"], CFG["maxm"])
    oc = O.OC(st, O.MPS(L, p, Q, tgt.dims, tgt.data), O.MPS(L, p, Q, ini.dims, ini.data), len(u), 0.0)
    Nt = len(u)
    sweep, samples, total = {}, {}, 0.0
    for t in counts:
        ts = []   # up to 3 getHessians per thread count, fewer once 8 s are spent on it; the median
        while len(ts) < 3 and (not ts or sum(ts) < 8.0):
            ts.append(oc.time_hessian(u, t))
        total += sum(ts)
        samples[str(t)] = len(ts)
        sweep[str(t)] = (Nt - 2) / float(np.median(ts))
    best = max(counts, key=lambda t: sweep[str(t)])
    return {"value": sweep[str(best)], "unit": "rows/s", "cores": best, "kind": "port",
            "threads_sweep_rows_per_sec": sweep, "samples_per_point": samples, "host_threads_available": avail, "nproc": os.cpu_count(),
            "sample": f"full getHessians (config 1, {Nt - 2} rows) at thread counts {counts}, the median of up to 3 "
                      f"per count, on the C++ CPU restatement (oracle/, not ITensor; main/TestRuntimes.cpp's thread "
                      f"sweep), {total:.1f} s"}


if __name__ == "__main__":
    sys.exit(main())
