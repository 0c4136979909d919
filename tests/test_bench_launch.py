"""bench.py's own rank launcher (`bench.py --gpus N` without torchrun): N spawned
processes with the torch.distributed.run environment, the rank count checked
against --gpus, a failing rank ending the job instead of hanging its peers.
Runs the launcher's real code path with gloo on CPU; on the GPU box the ranks
run bench.run instead of the small functions below."""
import os
import time

import pytest

import bench


def _gloo_rank(argv):
    """a rank: bench's own argument parsing + rank-count check, one gloo all-reduce;
    `--out DIR` (test only) is where it reports"""
    import torch
    import torch.distributed as dist
    i = argv.index("--out")
    out, argv = argv[i + 1], argv[:i] + argv[i + 2:]
    args = bench.parse_args(argv)
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    assert world == args.gpus
    assert os.environ["MASTER_ADDR"] == "127.0.0.1"
    dist.init_process_group("gloo")
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t)
    assert t.item() == world * (world + 1) / 2
    with open(os.path.join(out, f"rank{rank}"), "w") as f:
        f.write(f"{world}")
    dist.barrier()
    dist.destroy_process_group()
    return 0


def _failing_rank(argv):
    import torch.distributed as dist
    dist.init_process_group("gloo")
    if int(os.environ["RANK"]) == 1:
        raise SystemExit(3)
    dist.barrier()     # rank 0 would wait here forever without the launcher's watchdog
    return 0


@pytest.mark.parametrize("world", [2, 3])
def test_spawn_ranks_gloo(tmp_path, world):
    rc = bench.spawn_ranks(world, ["--gpus", str(world), "--out", str(tmp_path)], target=_gloo_rank)
    assert rc == 0
    assert sorted(os.listdir(tmp_path)) == [f"rank{r}" for r in range(world)]
    assert all(open(tmp_path / f).read() == str(world) for f in os.listdir(tmp_path))


def test_failing_rank_ends_the_job():
    t0 = time.perf_counter()
    rc = bench.spawn_ranks(2, ["--gpus", "2"], target=_failing_rank)
    assert rc == 3
    assert time.perf_counter() - t0 < 60


def test_rank_count_must_match_gpus(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "1")
    with pytest.raises(SystemExit, match="--gpus 2 but 1 rank"):
        bench.init_dist(bench.parse_args(["--gpus", "2"]))


def test_main_spawns_without_launcher(monkeypatch):
    """main() hands --gpus N > 1 to the launcher when no WORLD_SIZE is set, and
    runs in-process under an outer launcher"""
    calls = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "spawn_ranks", lambda n, argv: calls.append(("spawn", n)) or 0)
    monkeypatch.setattr(bench, "run", lambda args, blocks=None: calls.append(("run", args.gpus, blocks)) or 0)
    monkeypatch.setattr(bench, "slice_blocks", lambda args: {"config4_slice": {}, "config5_slice": {}})
    assert bench.main(["--gpus", "4"]) == 0
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert bench.main(["--gpus", "4"]) == 0
    assert bench.main(["--gpus", "1"]) == 0
    monkeypatch.delenv("WORLD_SIZE")
    assert bench.main(["--gpus", "1"]) == 0                    # N=1 default: the slice blocks first
    assert bench.main(["--gpus", "1", "--no-slices"]) == 0
    assert bench.main(["--gpus", "1", "--profiled"]) == 0
    assert calls == [("spawn", 4), ("run", 4, None), ("run", 1, None),
                     ("run", 1, {"config4_slice": {}, "config5_slice": {}}), ("run", 1, None), ("run", 1, None)]


def test_slice_blocks_children(monkeypatch):
    """the config-4 / config-5 / config-4 horizon blocks run as fresh `bench.py --workload ...`
    interpreters without the rank environment; a failing child leaves an
    `error` field and the other block intact"""
    import subprocess
    seen = []

    def fake_run(cmd, **kw):
        seen.append((cmd, kw["env"]))
        if "c4rows" in cmd:
            return subprocess.CompletedProcess(cmd, 0, stdout='[x] noise\n{"metric": "c4", "value": 1.0}\n')
        return subprocess.CompletedProcess(cmd, 1, stdout="Traceback ...\n")
    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setenv("RANK", "0")
    out = bench.slice_blocks(bench.parse_args(["--gpus", "1"]))
    assert out["config4_slice"]["value"] == 1.0 and "error" not in out["config4_slice"]
    assert "error" in out["config5_slice"] and "child_wall_s" in out["config5_slice"]
    assert out["config4_horizon_sample"]["value"] == 1.0
    assert [c[0][3:5] for c in seen] == [["--workload", "c4rows"], ["--workload", "c5rows"], ["--workload", "c4rows"]]
    assert "--row-stride" in seen[2][0] and "801" in seen[2][0]
    assert all("RANK" not in env for _, env in seen)
