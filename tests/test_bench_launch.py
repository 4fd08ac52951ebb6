"""`bench.py --gpus N` without a launcher: the launch plan (one fresh process per GPU, rendezvous on 127.0.0.1) and the
parent's handling of rank exits.  CPU only: the ranks here are tiny stand-in scripts, not the bench."""
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_single_rank_needs_no_children():
    assert bench.launch_plan(1, {}, 1, "nccl") is None
    # a launcher (torchrun) already made this process one rank of N
    assert bench.launch_plan(4, {"WORLD_SIZE": "4"}, 8, "nccl") is None


def test_plan_gives_every_rank_its_identity():
    plans = bench.launch_plan(8, {"PATH": "/bin"}, 8, "nccl")
    assert len(plans) == 8
    assert [p["RANK"] for p in plans] == [str(r) for r in range(8)]
    assert [p["LOCAL_RANK"] for p in plans] == [str(r) for r in range(8)]
    assert {p["WORLD_SIZE"] for p in plans} == {"8"}
    assert {p["MASTER_ADDR"] for p in plans} == {"127.0.0.1"}
    assert len({p["MASTER_PORT"] for p in plans}) == 1
    assert {p["HSA_ENABLE_IPC_MODE_LEGACY"] for p in plans} == {"0"}
    assert all(p["PATH"] == "/bin" for p in plans)


def test_rccl_needs_one_device_per_rank():
    with pytest.raises(ValueError, match="needs 8 visible GPUs"):
        bench.launch_plan(8, {}, 1, "nccl")
    # the gloo rehearsal may share devices (device = local rank modulo the visible devices)
    assert len(bench.launch_plan(2, {}, 1, "gloo")) == 2
    with pytest.raises(ValueError):
        bench.launch_plan(2, {}, 0, "gloo")
    with pytest.raises(ValueError):
        bench.launch_plan(0, {}, 8, "nccl")


def test_launcher_world_must_match_gpus():
    with pytest.raises(ValueError, match="WORLD_SIZE=2"):
        bench.launch_plan(4, {"WORLD_SIZE": "2"}, 8, "nccl")


def _stub(tmp_path, body):
    p = tmp_path / "rank.py"
    p.write_text(textwrap.dedent(body))
    return str(p)


def test_spawn_passes_rank0_stdout_and_waits_for_all(tmp_path, capfd):
    script = _stub(tmp_path, """
        import json, os
        if os.environ["RANK"] == "0":
            print(json.dumps({"world": int(os.environ["WORLD_SIZE"])}))
        else:
            print("rank", os.environ["RANK"])  # goes to stderr via the parent
    """)
    plans = bench.launch_plan(3, dict(os.environ, YAVO_X="1"), 3, "nccl")
    assert bench.spawn_ranks(plans, [], script=script) == 0
    out, err = capfd.readouterr()
    assert out.strip() == '{"world": 3}'
    assert "rank 1" in err and "rank 2" in err


def test_spawn_reports_a_failed_rank_and_stops_the_rest(tmp_path):
    script = _stub(tmp_path, """
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(3)
        time.sleep(60)  # would hang without the parent's stop
    """)
    plans = bench.launch_plan(3, dict(os.environ), 3, "nccl")
    assert bench.spawn_ranks(plans, [], script=script) == 3


def test_bench_cli_refuses_too_few_devices():
    # this container has no GPU: `--gpus 2` over RCCL must fail loudly, not run one rank
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.pop("YAVO_BENCH_BACKEND", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2
    assert "visible GPUs" in r.stderr
    assert r.stdout == ""


def test_exchange_summary_reports_hidden_and_exposed_gathers():
    """The bench's shared_map.collective_timing block (FrameShard.collective_stats over HIP events): mean / max gather
    time, placement time, and the fraction of exchanges whose gather ended before the run it overlapped."""
    from ya_vo_amd.sharding import exchange_summary
    assert exchange_summary([], [], []) is None
    s = exchange_summary([0.2, 0.4, 0.3, 0.1], [0.01, 0.02, 0.01, 0.01], [1.5, -0.2, 0.0, 2.0])
    assert s["exchanges"] == 4
    assert s["allgather_ms_mean"] == 0.25 and s["allgather_ms_max"] == 0.4
    assert s["hidden_fraction"] == 0.75 and s["min_slack_ms"] == -0.2


def test_bench_reports_world_size_and_collective_timing():
    """The bench line carries world_size_seen and the collective timing beside the shared map,
    and the configs[2] sequence leg is on by default."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert '"world_size_seen": dist.get_world_size() if dist.is_initialized() else 1' in src
    assert '"collective_timing": coll_stats' in src
    sys_argv = sys.argv
    try:
        sys.argv = ["bench.py"]
        a = bench.parse()
    finally:
        sys.argv = sys_argv
    assert a.sequence_frames == 1000 and a.sequence_cpu == 1  # timed over 1000, the first 200 checked
