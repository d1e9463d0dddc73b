"""bench.py runs one process per GPU under torchrun: a collective (comm.sum /
comm.max / comm.barrier) reached by rank 0 alone hangs or kills the N > 1 job
(round 2 found one in the rank-0 report). Static check, no GPU needed."""
import ast
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rank_only(test):
    src = ast.unparse(test)
    return "rank == 0" in src or "rank==0" in src


def test_no_collective_inside_rank0_blocks():
    tree = ast.parse(open(os.path.join(ROOT, "bench.py")).read())
    bad = []
    for node in ast.walk(tree):
        if isinstance(node, ast.If) and _rank_only(node.test):
            for sub in ast.walk(ast.Module(body=node.body, type_ignores=[])):
                if (isinstance(sub, ast.Call) and isinstance(sub.func, ast.Attribute)
                        and isinstance(sub.func.value, ast.Name) and sub.func.value.id == "comm"):
                    bad.append(f"bench.py:{sub.lineno} comm.{sub.func.attr} inside a rank-0 block")
    assert not bad, "\n".join(bad)


_PROBE = r'''
import json, os, sys
sys.path.insert(0, sys.argv[1])
import bench
c = bench.Comm(int(os.environ["WORLD_SIZE"]))
x = c.sum(1.0)
c.barrier()
if int(os.environ["RANK"]) == 0:
    print(json.dumps({"sum": x}))
'''


def test_two_rank_stdout_is_one_json_line(tmp_path):
    """Under torchrun with gloo, stdout must carry rank 0's JSON line and nothing
    else (gloo announces its connections on stdout unless bench.Comm redirects it)."""
    import json
    import subprocess
    import sys
    probe = tmp_path / "probe.py"
    probe.write_text(_PROBE)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29534", str(probe), ROOT],
                       capture_output=True, text=True, timeout=240, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    assert json.loads(lines[0]) == {"sum": 2.0}


def test_gpus_flag_spawns_ranks_without_launcher(tmp_path):
    """`bench.py --gpus 2` with no torchrun around it must run two ranks, not
    silently measure one GPU (round-3 review): the parent spawns the ranks before
    any GPU call, they meet at the gloo barrier, rank 0 prints n_gpus 2."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=240, cwd=str(tmp_path), env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["ranks_at_barrier"] == 2


def test_gpus_flag_disagreeing_with_launcher_fails(tmp_path):
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="3", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, cwd=str(tmp_path), env=env)
    assert r.returncode != 0 and "disagree" in r.stderr
