"""CPU: `bench.py --gpus N` means N ranks (BASELINE north_star: throughput at
1, 2, 4 and 8 GPUs).  Without a launcher, --gpus N > 1 starts N ranks itself (torch.distributed.run
as a child process, 127.0.0.1); under a launcher, a WORLD_SIZE that differs from --gpus is refused;
a mode that runs on one GPU refuses --gpus > 1; over RCCL, fewer visible GPUs than --gpus is
refused.  The launch path is exercised with --launch-check (the ranks join a gloo group and count
themselves with an all-reduce; no GPU work), so it runs here."""
import json
import os
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                          text=True, timeout=timeout, cwd=ROOT)


def _json(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out  # rank 0 prints ONE line
    return json.loads(lines[0])


def test_gpus_2_without_launcher_starts_two_ranks():
    r = _run(["--gpus", "2", "--dist-backend", "gloo", "--dist-impl", "python", "--launch-check"])
    assert r.returncode == 0, r.stderr[-3000:]
    j = _json(r.stdout)
    assert j["launch_check"] and j["n_gpus"] == 2 and j["ranks_counted"] == 2 and j["gpus_arg"] == 2


def test_gpus_1_is_one_rank():
    r = _run(["--gpus", "1", "--launch-check"])
    assert r.returncode == 0, r.stderr[-3000:]
    j = _json(r.stdout)
    assert j["n_gpus"] == 1 and j["ranks_counted"] == 1


def test_mismatched_world_size_refused():
    r = _run(["--gpus", "2", "--launch-check"], env_extra={"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=3" in r.stderr and "--gpus 2" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    # a launcher's WORLD_SIZE with the default --gpus 1 is a mismatch too
    r = _run(["--launch-check"], env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2


def test_single_gpu_modes_refuse_more_gpus():
    for mode in ("train", "views", "loop"):
        r = _run(["--gpus", "2", "--mode", mode])
        assert r.returncode == 2 and "runs on one GPU" in r.stderr, (mode, r.stderr[-2000:])


def test_rccl_needs_n_devices():
    # no GPU in this container: --gpus 2 over RCCL must refuse, not run one rank
    r = _run(["--gpus", "2"])
    assert r.returncode == 2 and "visible GPUs" in r.stderr, r.stderr[-2000:]


def test_bad_gpu_count_refused():
    assert _run(["--gpus", "0", "--launch-check"]).returncode == 2


def test_store_exchange_counts_the_ranks_that_joined(tmp_path):
    """bench.py --dist-backend gloo --dist-impl cpp runs the C++ gsr::ShardStep over
    ext.store_exchange on the launcher's c10d store; its comm_world, which the
    bench line reports next to n_gpus, is the store's own count of the ranks that joined the
    exchange -- checked here with two real ranks (gloo, no device: the join needs none)."""
    script = tmp_path / "se.py"
    script.write_text(
        "import importlib, json, sys\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "import torch.distributed as dist\n"
        "native = importlib.import_module('3d_gaussian_splatting_amd.native')\n"
        "dist.init_process_group('gloo')\n"
        "r, w = dist.get_rank(), dist.get_world_size()\n"
        "ext = native.load_torch_ext()\n"
        "a = ext.store_exchange(dist.distributed_c10d._get_default_store(), r, w)\n"
        "b = ext.store_exchange(dist.distributed_c10d._get_default_store(), r, w)\n"
        "print(json.dumps({'rank': r, 'name': a.name, 'world': a.world, 'comm_world': a.comm_world,\n"
        "                  'second': b.comm_world, 'capturable': a.capturable}), flush=True)\n"
        "dist.destroy_process_group()\n")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    import socket
    with socket.socket() as sk:  # a free port (a fixed one can still be held by an earlier run)
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr=127.0.0.1", f"--master-port={port}", str(script)], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    rows = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert sorted(x["rank"] for x in rows) == [0, 1]
    for x in rows:
        assert x["name"] == "store" and x["world"] == 2 and x["comm_world"] == 2 and x["second"] == 2
        assert x["capturable"] is False
