"""bench.py's side-probe orchestration on a world-2 gloo group (CPU): a probe that fails on every
rank is reported and the next probe still runs; a probe that fails on one rank only is reported on
every rank and every later probe is skipped with the reason (its collectives may be unmatched);
a probe stuck past its deadline has its communicators aborted (the stuck collective returns), is
reported, and every later probe is skipped; wall times are recorded; the top-level DP scaling quantity is formed from the C3 probe's own local /
DP timings."""

import json
import os
import sys
from pathlib import Path

import torch
import torch.multiprocessing as mp

from test_finetune_loop_cpu import free_port

ROOT = Path(__file__).resolve().parents[1]


def _main(rank, world, port, out):
    sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]
    os.environ.update(OMP_NUM_THREADS="1")
    import torch.distributed as dist

    import bench

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    ctrl = dist.new_group(backend="gloo")
    r = bench.ProbeRunner(rank, "cpu", ctrl)

    def everywhere():
        raise RuntimeError(f"out of memory on rank {rank}")

    def flaky():
        if rank == 1:
            raise RuntimeError("out of memory on rank 1")
        return {"value": 1}

    def collective():
        t = torch.ones(1)
        dist.all_reduce(t)
        return {"sum": float(t)}

    census = r.run("communicators", lambda: bench.communicator_census(world, ctrl, "cpu", prl_comm=False))
    res = {"census": census, "everywhere": r.run("everywhere", everywhere), "after_all": r.run("after_all", collective),
           "flaky": r.run("flaky", flaky), "after": r.run("after", collective), "wall": r.wall}
    Path(out, f"r{rank}.json").write_text(json.dumps(res))
    dist.destroy_process_group()


def test_probe_failures_shared_and_partial_failure_skips_later_probes(tmp_path):
    mp.spawn(_main, args=(2, free_port(), str(tmp_path)), nprocs=2, join=True)
    r0, r1 = (json.loads((tmp_path / f"r{r}.json").read_text()) for r in range(2))
    for r in (r0, r1):
        assert "out of memory" in r["everywhere"]["error"]
        assert r["after_all"]["sum"] == 2.0  # a failure on every rank: the next probe still runs
        assert set(r["wall"]) == {"communicators", "everywhere", "after_all", "flaky", "after"}
        assert r["after_all"]["wall_s"] >= 0
        # the N > 1 line's communicator census: every group at the intended size
        c = r["census"]
        assert {k for k in c if not k.endswith("_s") and k != "host_rss_gib_after"} == {"dp", "ctrl"}, c
        for k in ("dp", "ctrl"):
            assert c[k]["reported"] == c[k]["participants"] == c[k]["intended"] == 2 and c[k]["ok"]
        assert "flaky" in r["after"]["skipped"]  # a failure on one rank: later probes are skipped
    assert "error" in r1["flaky"] and "out of memory" in r1["flaky"]["error"]
    assert r0["flaky"]["error_on_another_rank"] is True and r0["flaky"]["value"] == 1


def test_dp_scaling_from_the_c3_probe():
    sys.path[:0] = [str(ROOT)]
    import bench

    c3 = {"tokens_per_s": 7000.0 * 8 * 0.9, "local_tokens_per_s_per_gpu": 7000.0,
          "extrapolated": {"allreduce_share": 0.002, "tokens_per_s_per_gpu": 7100.0}}
    s = bench.dp_scaling(8, c3, {"dp_efficiency": 0.97})
    assert s["c3_efficiency"] == 0.9 and s["c3_speedup_vs_one_replica"] == 7.2
    assert s["c3_extrapolated_efficiency"] == 0.998 and s["c3_extrapolated_tokens_per_s"] == 56800.0
    assert s["trainer_step_1.5b_efficiency"] == 0.97
    assert bench.dp_scaling(8, {"error": "x"}, None) is None


def _stuck(rank, world, port, out):
    sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]
    os.environ.update(OMP_NUM_THREADS="1")
    import threading

    import torch.distributed as dist

    import bench

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    ctrl = dist.new_group(backend="gloo")
    r = bench.ProbeRunner(rank, "cpu", ctrl, deadline_s=2.0)
    released = threading.Event()
    aborted = []

    def abort():  # stands in for RCCL's abort: the stuck collective returns with an error
        aborted.append(True)
        released.set()

    r._abort_rccl = abort

    def hung():
        if not released.wait(60):
            return {"value": "never released"}
        raise RuntimeError("collective aborted")

    res = {"quick": r.run("quick", lambda: {"value": 1}), "hung": r.run("hung", hung),
           "after": r.run("after", lambda: {"value": 2}), "aborted": len(aborted), "wall": r.wall}
    Path(out, f"r{rank}.json").write_text(json.dumps(res))
    dist.destroy_process_group()


def test_probe_past_its_deadline_aborts_and_skips_the_rest(tmp_path):
    mp.spawn(_stuck, args=(2, free_port(), str(tmp_path)), nprocs=2, join=True)
    for rank in range(2):
        r = json.loads((tmp_path / f"r{rank}.json").read_text())
        assert r["quick"]["value"] == 1  # the timer of a probe that finished in time never fires
        assert "collective aborted" in r["hung"]["error"] and r["hung"]["deadline_s"] == 2.0
        assert 2.0 <= r["wall"]["hung"] < 30
        assert r["aborted"] >= 1
        assert "passed its deadline" in r["after"]["skipped"]
