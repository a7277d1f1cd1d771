"""bench.py's multi-GPU launch contract on CPU (gloo): `--gpus N` either runs
under torchrun with WORLD_SIZE == N or starts the N ranks itself, and a
mismatch fails loudly. --cpu-table-only runs the N > 1 control path of C5
(each rank inserts only its partition's rules of the 1M-rule set,
all-reduce, partition build, all-gather) without a GPU."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _line(out):
    lines = [x for x in out.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def _env():
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    return e


def test_torchrun_two_ranks_c5_table():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=2", "--master-addr", "127.0.0.1", "--master-port",
           str(_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--cpu-table-only", "--rules", "1048576"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300,
                       env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _line(r.stdout)
    assert line["n_gpus"] == 2
    c5 = line["C5_table"]
    assert c5["rules"] == 1 << 20 and c5["image_equals_single_build"] is True
    assert 0.45 * (1 << 20) < c5["rules_inserted_rank0"] < 0.55 * (1 << 20)
    assert c5["bytes"] == 2 * c5["part_bytes"]


def test_gpus_flag_starts_the_ranks():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus",
                        "2", "--cpu-table-only", "--c5-rules", "100000"],
                       capture_output=True, text=True, timeout=300, env=_env(),
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _line(r.stdout)
    assert line["n_gpus"] == 2
    assert line["C5_table"]["image_equals_single_build"] is True


def test_world_size_mismatch_fails():
    e = _env()
    e.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus",
                        "4", "--cpu-table-only"], capture_output=True, text=True,
                       timeout=120, env=e, cwd=ROOT)
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr
