"""world_size-2 gloo run of bench.py's Comm (barrier, max over ranks, sum):
the multi-GPU path shards reads with no data-path collective; only timing and
counter reductions cross ranks."""
import os
import socket
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_comm_world2_gloo(tmp_path):
    script = tmp_path / "w.py"
    script.write_text(textwrap.dedent(f"""
        import os, sys
        sys.path.insert(0, {ROOT!r})
        from bench import Comm
        rank = int(os.environ["RANK"])
        c = Comm(int(os.environ["WORLD_SIZE"]))
        c.barrier()
        m = c.max(1.5 + rank)
        s = c.sum(10 * (rank + 1))
        print(f"R{{rank}} {{m}} {{s}}", flush=True)
    """))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE="2")
    procs = [subprocess.Popen([sys.executable, str(script)], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = [p.communicate(timeout=120) for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    lines = sorted(l for o in outs for l in o[0].splitlines() if l.startswith("R"))
    assert lines == ["R0 2.5 30.0", "R1 2.5 30.0"]


def test_rank_shards_are_disjoint_and_deterministic():
    sys.path.insert(0, ROOT)
    from tools.synth import Dataset
    a0 = Dataset("tiny", seed=42, n_pb=5, pb_index_base=0)
    a1 = Dataset("tiny", seed=42, n_pb=5, pb_index_base=5)
    b = Dataset("tiny", seed=42, n_pb=10, pb_index_base=0)
    assert a0.sr_seqs() == a1.sr_seqs() == b.sr_seqs()  # replicated index input
    assert a0.pb_seqs() + a1.pb_seqs() == b.pb_seqs()    # rank shards tile the global read set
    assert [n.decode() for n in a1.pb_names()] == [str(i) for i in range(5, 10)]
