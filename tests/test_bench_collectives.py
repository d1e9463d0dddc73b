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
